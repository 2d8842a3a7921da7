/*
 * arena_api.h — C launch API of the gfx950 arena kernels (libsplinter_hip.so).
 *
 * All pointers are device pointers; `stream` is a hipStream_t (NULL = the
 * default stream).  Key batches are NUL-padded records of `kstride` bytes
 * (16, 32, 48 or 64); value batches are `vstride`-byte records (multiple of
 * 16) with explicit lengths.  Per-op status: 0 ok, -11 EAGAIN, -2 ENOENT,
 * -28 ENOSPC, -90 EMSGSIZE, -91 EPROTOTYPE, -22 EINVAL; unset returns the old
 * length (>= 0) on success.  Returns a hipError_t (0 = launched).
 */
#ifndef SPLINTER_ARENA_API_H
#define SPLINTER_ARENA_API_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spl_arena {
  void    *base;      /* device address of the format-v4 header */
  uint32_t slots;
  uint32_t max_val;
  uint32_t stride;    /* 128 or 3200 */
  uint32_t flags;     /* SPL_ARENA_* */
  uint64_t notify;    /* device address of the host-mapped event-bus notify word (0 = none) */
} spl_arena_t;

#define SPL_ARENA_EVENTBUS 1u  /* event bus armed (maintain the dirty mask) */
#define SPL_ARENA_SIDE     2u  /* the allocation carries the side region (splinter_layout.hpp) */
#define SPL_ARENA_VEC16    4u  /* ... with the bf16 vector copy + squared norms (embedding stores) */

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
/* maintenance passes (arena_maint.hip): probe-chain statistics into a zeroed device ProbeStats
 * (splinter_layout.hpp / spl_probe_stats); the tombstone rebuild (EXCLUSIVE access; counters:
 * device u64[4] {moved, reclaimed, clusters, skipped}, zeroed); the bf16 vector copy rebuilt from
 * the fp32 vectors (SPL_ARENA_VEC16 arenas) */
int spl_arena_probe_stats(spl_arena_t a, void *out, hipStream_t stream);
int spl_arena_rehash(spl_arena_t a, void *counters, hipStream_t stream);
/* open (begin 1) / close (0) an online maintenance pass (side header MaintRec::seq odd while open);
 * ok: device u64, 1 when the open won (no other pass was running) */
int spl_arena_maint_mark(spl_arena_t a, int begin, int pid, uint64_t t0_ns, void *ok, hipStream_t stream);
int spl_arena_vec16_rebuild(spl_arena_t a, hipStream_t stream);
/* full rebuild (exclusive): collect the live slot indices (device u32[slots], count: device u64
 * zeroed), then move them out to tmp (n * spl_arena_rebuild_rec bytes), clear the slot array and
 * re-insert every entry (fail: device u64 zeroed, entries left without a slot: 0 when n <= slots) */
uint32_t spl_arena_rebuild_rec(spl_arena_t a);
int spl_arena_rebuild_collect(spl_arena_t a, uint32_t *idx, void *count, hipStream_t stream);
int spl_arena_rebuild_move(spl_arena_t a, const uint32_t *idx, uint64_t n, void *tmp, void *fail, hipStream_t stream);
int spl_arena_gather_slots(spl_arena_t a, const uint32_t *idx, long n, uint8_t *out_core, hipStream_t stream);
int spl_hash_keys(const char *keys, int kstride, long n, uint64_t *out, hipStream_t stream);
int spl_format_keys(char *out, int kstride, const uint64_t *ids, uint64_t first, long n, const char *prefix_dev,
                    int plen, int width, hipStream_t stream);
int spl_format_values(uint8_t *out, int vstride, uint32_t *lens, const uint64_t *ids, uint64_t first, long n,
                      uint32_t ver, uint32_t len, hipStream_t stream);

/* In-place rows: row i of the launch is client op idx[i] and only the first *count rows are live
 * (the own-shard ops of a routed step run on the client's arrays). */
int spl_arena_set_idx(spl_arena_t a, const char *keys, int kstride, const uint8_t *vals, int vstride,
                      const uint32_t *lens, const int32_t *idx, const int32_t *count, long n, int32_t *status,
                      int max_retry, uint64_t *stats, hipStream_t stream);
int spl_arena_get_idx(spl_arena_t a, const char *keys, int kstride, uint8_t *out, int ostride, uint32_t *out_lens,
                      const int32_t *idx, const int32_t *count, long n, int32_t *status, int max_retry,
                      uint64_t *stats, hipStream_t stream);

/* ---- routed exchange (route_kernels.hip; parallel/xroute.py) ------------------------------------
 * Pack one kind of a client batch straight into the owners' request blocks: shard =
 * ((fnv1a >> 40) & 0xFFFFFF) % world; blk[d] = base of the block for owner d (device table),
 * rows at blk[d] + off_k / off_l / off_v (key, u32 len, vw value bytes; vw = 0: keys only).
 * counts[world] is zeroed here and receives every destination's rows (own included); own ops are
 * listed in lidx (client indices); pos[i] = d*cap + j (remote), -2 (own), -1 (block full).
 * Direct responses (off_p > 0): every remote row also carries its client index, an int32 at
 * blk[d] + off_p + 4j, so the owner writes the op's result straight into the requester's client
 * arrays; an op whose block is full gets EAGAIN in full_status (and len 0 in full_lens) here. */
int spl_xr_pack(const char *keys, int ks, const uint8_t *vals, int vstride, const uint32_t *lens, long n, int world,
                int rank, long cap, const uint64_t *blk, long off_k, long off_l, long off_v, int vw, int32_t *counts,
                int32_t *lidx, int32_t *pos, long off_p, int32_t *full_status, uint32_t *full_lens,
                hipStream_t stream);
/* Responses into client order: remote ops read status / len / value row j of blk[d]; full ops get
 * EAGAIN; own ops are left as the in-place kernels wrote them. */
int spl_xr_gather(const int32_t *pos, long n, long cap, const uint64_t *blk, long off_s, long off_l, long off_v,
                  int vw, int32_t *status, uint32_t *out_lens, uint8_t *out, int ostride, hipStream_t stream);
/* Device-side ordering of a step without a collective: post this rank's step sequence (dir 0 with
 * its pack counts [2][world], dir 1 without) into every peer window's flag area (flag_blk: device
 * table of the world flag-area addresses), or wait (one workgroup, bounded by timeout_ms; *err = 1
 * on expiry) until every peer's post has reached this rank's own area. */
int spl_xr_post(const uint64_t *flag_blk, int world, int rank, int par, int dir, uint64_t seq, const int32_t *counts,
                hipStream_t stream);
int spl_xr_wait(const void *own_flags, int world, int rank, int par, int dir, uint64_t seq, uint64_t timeout_ms,
                uint32_t *err, hipStream_t stream);
long spl_xr_flag_bytes(void);

#define SPL_XR_MAX_WORLD 64
/* One routed step's owner side for spl_kvs_step_xr (all pointers device, except the tables). */
typedef struct spl_xr_step {
  int world, rank;
  long cap_s, cap_g;            /* rows per request block: sets, gets */
  int ks, vw;                   /* key record bytes; value prefix bytes per routed row */
  /* the client batch (own ops run in place on these) */
  const char *skeys; const uint8_t *svals; int svstride; const uint32_t *slens; int32_t *sstatus; long n_set;
  const char *gkeys; uint8_t *gout; int gostride; uint32_t *glens; int32_t *gstatus; long n_get;
  const int32_t *lidx_set, *lidx_get;  /* own client indices (NULL: world 1, the batch row for row) */
  const int32_t *own_counts;           /* [world][2]: this rank's pack counts per destination (set, get);
                                          the own entry [rank] is the own rows */
  const int32_t *rcounts;              /* [world][2]: rows received from each source (set, get) */
  uint64_t req[SPL_XR_MAX_WORLD];      /* request block of source s (this rank's window) */
  uint64_t resp[SPL_XR_MAX_WORLD];     /* where this rank's responses to source s go */
  long off_sk, off_sl, off_sv, off_gk; /* request block layout */
  long off_ss, off_gs, off_gl, off_gv; /* response block layout */
  /* direct responses (> 0): the request block's client-index columns; resp[s] is then source s's
   * client output area (its status / lens / value rows at off_ss.. in client order, value rows vw
   * bytes apart) and each result is written at its op's client index; <= 0: response blocks */
  long off_sp, off_gp;
} spl_xr_step_t;

/* Exchange windows: device memory a peer process maps (VMM dmabuf chunks, abstract socket `name`). */
void *spl_xw_create(int device, size_t bytes, const char *name);
void *spl_xw_attach(const char *name, int device);
void *spl_xw_base(void *w);
size_t spl_xw_bytes(void *w);
void spl_xw_destroy(void *w);
int spl_xw_peer(int device, int peer);

/* Client-stream groups (arena_kernels.hip): one native call issues a KV step's slices on
 * `writers` + `readers` concurrent streams. */
void *spl_kvs_create(int writers, int readers);
void spl_kvs_destroy(void *h);
/* 0: one launch per client stream slice; 1 / 2 (default, SPL_KVS_FUSED): every slice in one fused grid */
int spl_kvs_set_fused(void *h, int mode);
// fused-grid scheduling of this context: 0 fixed lane streams + workgroup barrier per round, 1 chunk claims,
// 2 fixed lane streams + wave-vote exit (the SPL_KVS_SCHED default); -1: back to SPL_KVS_SCHED
int spl_kvs_set_sched(void *h, int sched);
int spl_kvs_step(void *h, spl_arena_t a, hipStream_t origin, const char *skeys, int kstride, const uint8_t *svals,
                 int vstride, const uint32_t *slens, long n_set, int32_t *sstatus, const char *gkeys, uint8_t *gout,
                 int ostride, uint32_t *glens, long n_get, int32_t *gstatus, int max_retry, uint64_t *stats);
int spl_kvs_step_xr(void *h, spl_arena_t a, hipStream_t origin, const spl_xr_step_t *x, int max_retry,
                    uint64_t *stats);

#ifdef __cplusplus
}
#endif
#endif
