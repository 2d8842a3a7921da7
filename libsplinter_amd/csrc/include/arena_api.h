/*
 * arena_api.h — C launch API of the gfx950 arena kernels (libsplinter_hip.so).
 *
 * All pointers are device pointers; `stream` is a hipStream_t (NULL = the
 * default stream).  Key batches are NUL-padded records of `kstride` bytes
 * (16, 32, 48 or 64); value batches are `vstride`-byte records (multiple of
 * 16) with explicit lengths.  Per-op status: 0 ok, -11 EAGAIN, -2 ENOENT,
 * -28 ENOSPC, -90 EMSGSIZE, -71 EPROTOTYPE, -22 EINVAL; unset returns the old
 * length (>= 0) on success.  Returns a hipError_t (0 = launched).
 */
#ifndef SPLINTER_ARENA_API_H
#define SPLINTER_ARENA_API_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spl_arena {
  void    *base;      /* device address of the format-v4 header */
  uint32_t slots;
  uint32_t max_val;
  uint32_t stride;    /* 128 or 3200 */
  uint32_t flags;     /* bit0: event bus armed (maintain dirty mask) */
  uint64_t notify;    /* device address of the host-mapped event-bus notify word (0 = none) */
} spl_arena_t;

#ifndef __HIP_PLATFORM_AMD__
typedef void *hipStream_t;
#endif

/* meta ops for spl_arena_meta */
#define SPL_META_SET_LABEL      0
#define SPL_META_UNSET_LABEL    1
#define SPL_META_BUMP           2
#define SPL_META_GET_EPOCH      3
#define SPL_META_WATCH_REG      4
#define SPL_META_WATCH_UNREG    5
#define SPL_META_PULSE          6
#define SPL_META_SET_SYSTEM     7
#define SPL_META_RETRAIN        8
#define SPL_META_SET_TYPE       9
#define SPL_META_SET_CTIME     10
#define SPL_META_SET_ATIME     11
#define SPL_META_FIND          12

/* scan modes for spl_arena_scan */
#define SPL_SCAN_LIST      0
#define SPL_SCAN_LABELS    1
#define SPL_SCAN_EMBEDDED  2
#define SPL_SCAN_OCCUPIED  3
#define SPL_SCAN_ODD       4   /* watchdog: slots whose epoch is odd (writer active / crashed) */

int spl_arena_init_slots(spl_arena_t a, hipStream_t stream);
int spl_arena_set(spl_arena_t a, const char *keys, int kstride, const uint8_t *vals, int vstride,
                  const uint32_t *lens, long n, int32_t *status, int max_retry, uint64_t *stats,
                  hipStream_t stream);
int spl_arena_get(spl_arena_t a, const char *keys, int kstride, uint8_t *out, int ostride,
                  uint32_t *out_lens, long n, int32_t *status, int max_retry, uint64_t *stats,
                  hipStream_t stream);
/* Segmented variants: the batch is n/seg_cap segments of seg_cap rows of which only the first
 * seg_counts[s] are live (routed C1 buffers); dead rows get status EINVAL and are not counted. */
int spl_arena_set_seg(spl_arena_t a, const char *keys, int kstride, const uint8_t *vals, int vstride,
                      const uint32_t *lens, long n, int32_t *status, int max_retry, uint64_t *stats,
                      const int32_t *seg_counts, long seg_cap, hipStream_t stream);
int spl_arena_get_seg(spl_arena_t a, const char *keys, int kstride, uint8_t *out, int ostride,
                      uint32_t *out_lens, long n, int32_t *status, int max_retry, uint64_t *stats,
                      const int32_t *seg_counts, long seg_cap, hipStream_t stream);
int spl_arena_unset(spl_arena_t a, const char *keys, int kstride, long n, int32_t *status, int max_retry,
                    hipStream_t stream);
int spl_arena_intop(spl_arena_t a, const char *keys, int kstride, const int *ops, const uint64_t *masks,
                    long n, int32_t *status, uint64_t *results, int max_retry, hipStream_t stream);
int spl_arena_meta(spl_arena_t a, const char *keys, int kstride, int op, const uint64_t *args, long n,
                   int32_t *status, uint64_t *out, hipStream_t stream);
int spl_arena_embed_set(spl_arena_t a, const char *keys, int kstride, const float *vecs, long n,
                        int32_t *status, hipStream_t stream);
int spl_arena_embed_get(spl_arena_t a, const char *keys, int kstride, float *vecs, long n, int32_t *status,
                        hipStream_t stream);
int spl_arena_scan(spl_arena_t a, int mode, uint64_t mask, uint32_t *out_idx, uint64_t *out_epoch,
                   uint32_t cap, uint32_t *counter, hipStream_t stream);
/* the same over slots [first, last) (chunked host scans with bounded scratch) */
int spl_arena_scan_range(spl_arena_t a, int mode, uint64_t mask, uint32_t first, uint32_t last, uint32_t *out_idx,
                         uint64_t *out_epoch, uint32_t cap, uint32_t *counter, hipStream_t stream);
int spl_arena_purge(spl_arena_t a, hipStream_t stream);
int spl_arena_gather_slots(spl_arena_t a, const uint32_t *idx, long n, uint8_t *out_core, hipStream_t stream);
int spl_hash_keys(const char *keys, int kstride, long n, uint64_t *out, hipStream_t stream);
int spl_format_keys(char *out, int kstride, const uint64_t *ids, uint64_t first, long n, const char *prefix_dev,
                    int plen, int width, hipStream_t stream);
int spl_format_values(uint8_t *out, int vstride, uint32_t *lens, const uint64_t *ids, uint64_t first, long n,
                      uint32_t ver, uint32_t len, hipStream_t stream);

/* C1 routing (route_kernels.hip): pack a batch into world x cap per-destination rows
 * (shard = (fnv1a >> 40) % world); counts[world] is zeroed by the launcher and receives the
 * rows per destination (may exceed cap: ops beyond cap get pos = -1).  vals/lout/vout NULL for
 * key-only requests.  Gather: status[i] = pos[i] < 0 ? EAGAIN : rstatus[pos[i]], and likewise
 * lengths and min(rstride, ostride) value bytes. */
int spl_route_pack(const char *keys, int kstride, const uint8_t *vals, int vstride, int vwidth,
                   const uint32_t *lens, long n, int world, long cap, int32_t *counts, int64_t *pos,
                   char *kout, uint32_t *lout, uint8_t *vout, hipStream_t stream);
int spl_route_gather(const int64_t *pos, long n, const int32_t *rstatus, const uint32_t *rlens,
                     const uint8_t *rvals, int rstride, int32_t *status, uint32_t *out_lens, uint8_t *out,
                     int ostride, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
