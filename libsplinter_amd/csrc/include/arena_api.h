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
int spl_arena_purge(spl_arena_t a, hipStream_t stream);
int spl_arena_gather_slots(spl_arena_t a, const uint32_t *idx, long n, uint8_t *out_core, hipStream_t stream);
int spl_hash_keys(const char *keys, int kstride, long n, uint64_t *out, hipStream_t stream);
int spl_format_keys(char *out, int kstride, const uint64_t *ids, uint64_t first, long n, const char *prefix_dev,
                    int plen, int width, hipStream_t stream);
int spl_format_values(uint8_t *out, int vstride, uint32_t *lens, const uint64_t *ids, uint64_t first, long n,
                      uint32_t ver, uint32_t len, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
