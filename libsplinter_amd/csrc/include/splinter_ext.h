/*
 * splinter_ext.h — libsplinter_amd extensions to the reference C ABI.
 *
 *  - handle API: several open stores per process (the reference allows one);
 *    every splinter_xxx(args) has a twin spl_xxx(spl_store *s, args);
 *  - explicit create flags (embedding stride, persistence) and unlink;
 *  - backend introspection (shm / file / hbm) and raw region access used by
 *    the GPU checkpoint path and the bulk loaders.
 */
#ifndef SPLINTER_EXT_H
#define SPLINTER_EXT_H
#include "splinter.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spl_store spl_store;

#define SPL_CREATE_EMBEDDINGS     1u
#define SPL_CREATE_PERSISTENT     2u
#define SPL_CREATE_NO_EMBEDDINGS  4u

spl_store  *spl_store_create(const char *name, size_t slots, size_t max_val, unsigned flags, int *err);
spl_store  *spl_store_open(const char *name, int *err);
void        spl_store_close(spl_store *s);
int         spl_store_use(spl_store *s);          /* make `s` the splinter_* current store */
spl_store  *spl_store_current(void);
const char *spl_store_backend(spl_store *s);
int         spl_store_geometry(spl_store *s, uint32_t *slots, uint32_t *max_val, uint32_t *stride);
void       *spl_store_base(spl_store *s);         /* mapped region (host backends), else NULL */
size_t      spl_store_bytes(spl_store *s);
int         spl_store_sync(spl_store *s, int async);  /* msync a file-backed store (0 = MS_SYNC) */
long        spl_list_copy(char *buf, size_t cap);     /* current store's keys, NUL-separated; -(need) if short */
int         spl_unlink(const char *name);         /* remove shm object / file / hbm descriptor */
const char *spl_version(void);
const char *spl_build(void);

/* handle twins of the reference API */
int   spl_set_mop(spl_store *s, unsigned int mode);
int   spl_get_mop(spl_store *s);
void  spl_purge(spl_store *s);
int   spl_get_header_snapshot(spl_store *s, splinter_header_snapshot_t *snap);
int   spl_set(spl_store *s, const char *key, const void *val, size_t len);
int   spl_unset(spl_store *s, const char *key);
int   spl_get(spl_store *s, const char *key, void *buf, size_t buf_sz, size_t *out_sz);
int   spl_list(spl_store *s, char **out_keys, size_t max_keys, size_t *out_count);
int   spl_poll(spl_store *s, const char *key, uint64_t timeout_ms);
int   spl_get_slot_snapshot(spl_store *s, const char *key, splinter_slot_snapshot_t *snap);
int   spl_append(spl_store *s, const char *key, const void *data, size_t len, size_t *new_len);
const void *spl_get_raw_ptr(spl_store *s, const char *key, size_t *out_sz, uint64_t *out_epoch);
uint64_t spl_get_epoch(spl_store *s, const char *key);
int   spl_set_as_system(spl_store *s, const char *key);
int   spl_set_embedding(spl_store *s, const char *key, const float *vec);
int   spl_get_embedding(spl_store *s, const char *key, float *out);
int   spl_set_named_type(spl_store *s, const char *key, uint16_t mask);
int   spl_set_slot_time(spl_store *s, const char *key, unsigned short mode, uint64_t epoch, size_t offset);
int   spl_integer_op(spl_store *s, const char *key, splinter_integer_op_t op, const void *mask);
int   spl_bump_slot(spl_store *s, const char *key);
int   spl_retrain_slot(spl_store *s, const char *key);
int   spl_set_label(spl_store *s, const char *key, uint64_t mask);
int   spl_unset_label(spl_store *s, const char *key, uint64_t mask);
int   spl_watch_register(spl_store *s, const char *key, uint8_t group);
int   spl_watch_unregister(spl_store *s, const char *key, uint8_t group);
int   spl_watch_label_register(spl_store *s, uint64_t mask, uint8_t group);
int   spl_pulse_keygroup(spl_store *s, const char *key);
uint64_t spl_get_signal_count(spl_store *s, uint8_t group);
int   spl_signal_add(spl_store *s, uint8_t group, uint64_t delta);  /* counter += delta (sharded sync) */
void  spl_enumerate_matches(spl_store *s, uint64_t mask,
                            void (*cb)(const char *key, uint64_t epoch, void *data), void *ud);
int   spl_event_bus_init(spl_store *s);
int   spl_event_bus_open(spl_store *s);
void  spl_event_bus_get_dirty(spl_store *s, uint64_t *out, size_t words);
int   spl_shard_claim_ex(spl_store *s, uint32_t id, uint32_t pid, uint8_t intent, uint8_t prio,
                         uint64_t dur, uint64_t at);
int   spl_shard_claim(spl_store *s, uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur);
int   spl_shard_rebid(spl_store *s, uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur);
int   spl_shard_release(spl_store *s, uint32_t id);
uint32_t spl_shard_election(spl_store *s, uint8_t *out_intent);
int   spl_shard_table_snapshot(spl_store *s, struct splinter_shard_bid_snapshot *out, size_t max);
int   spl_madvise(spl_store *s, uint32_t id, void *addr, size_t len, int advice, uint64_t timeout);
int   spl_client_set_tandem(spl_store *s, const char *base, const void **vals, const size_t *lens, uint8_t orders);
void  spl_client_unset_tandem(spl_store *s, const char *base, uint8_t orders);

/* HBM stores and node stores of HBM shards (libsplinter_hip.so): the CLI `search` scoring on the device.  Scores every candidate
 * slot (bloom `mask`, or every key with a value) against `query` [768] fp32, filters with min_sim /
 * max_dist (> 0 = on), ranks by similarity desc then distance asc, and fills up to `cap` hits.
 * Returns the number of candidates (may exceed cap); emb == 0: a candidate without a vector. */
typedef struct spl_search_hit {
  char key[64];
  float sim, dist;
  uint64_t epoch, bloom;
  uint32_t len;
  uint8_t type, emb, pad[2];
} spl_search_hit;
long  spl_hbm_search(spl_store *s, const float *query, uint64_t mask, float min_sim, float max_dist, long cap,
                     spl_search_hit *out);

/* Batched top-k of many queries [nq][768] fp32 (host) over an HBM store, or over every shard of a node
 * store of HBM shards (merged per query): the MFMA candidate passes (on the bf16 vector copy of the
 * arena's side region) with an exact fp32 re-score, so the ranking is the exact brute force's
 * (similarity desc, distance asc; reference splinter_cli_cmd_search.c:374-416).  k <= 32; min_sim,
 * max_dist filters (-2 / 3.4e38 = off); mask: bloom labels a slot must carry (0 = any).  out[nq * k]:
 * query q's hits at out[q * k ...], unused entries with an empty key and emb = 0.  Returns nq. */
long  spl_search_batch(spl_store *s, const float *queries, int nq, int k, float min_sim, float max_dist,
                       uint64_t mask, spl_search_hit *out);

/* Probe-chain health of an HBM store (summed over a node store's shards): one device pass over the
 * slots.  disp_*: probe length of a hit per live key; miss_*: probe length of a miss averaged over
 * every home position (a miss walks to the next never-used slot); hist[b]: live keys with probe
 * length 1, 2, 3-4, 5-8, ..., > 1024.  rebuilds / reclaimed / moved: spl_hbm_rehash history. */
typedef struct spl_probe_stats {
  uint64_t live, tombstones, virgin, busy;
  uint64_t disp_sum, disp_max, miss_sum, miss_max;
  uint64_t hist[12];
  uint64_t rebuilds, reclaimed, moved, pad;
} spl_probe_stats;
int   spl_hbm_probe_stats(spl_store *s, spl_probe_stats *out);
/* Tombstone maintenance: every live key moves into the first tombstone on its own probe path and
 * the tombstones left at the end of each cluster become never-used slots again, so misses stop at
 * the cluster's new end.  ONLINE: safe beside batch and per-call ops of every process -- each move
 * holds both slots' seqlocks, and while the pass runs "absent" outcomes (get miss, insert of a new
 * key, unset / update of a missing key) report EAGAIN instead (the key may be mid-move); hits and
 * updates of present keys proceed.  flags SPL_REHASH_FULL: the full rebuild instead (copy out,
 * clear, re-insert: no tombstones left at all), EXCLUSIVE -- the caller guarantees that no op of
 * any process runs on the store; -1/EBUSY when this store's ring cannot be held, -1/ENOMEM (the
 * scratch size on stderr) when its scratch cannot be allocated.  -1/EBUSY also when another
 * process's pass is running.  out (optional): {keys moved, tombstones reclaimed, clusters,
 * clusters with more than 512 tombstones}. */
#define SPL_REHASH_FULL 1u
int   spl_hbm_rehash_ex(spl_store *s, unsigned flags, uint64_t *out);
int   spl_hbm_rehash(spl_store *s, uint64_t *out);  /* = spl_hbm_rehash_ex(s, 0, out) */
/* The maintenance seq of an hbm: store (odd while a pass runs; +2 per pass): a host that enumerates
 * reads it before and after, and enumerates again when it changed. */
int   spl_hbm_maint_seq(spl_store *s, uint64_t *seq);

/* Checkpoint / restore of any store: a host store writes its v4 image (tmp + rename), an hbm: store
 * streams its device image, a node store writes every serving shard to PATH.s<i>.  Restore loads an
 * image into an open store of the same geometry (hbm: / host; exclusive -- a restarting rank
 * restores its shard before it joins).  0, or -1 with errno. */
int   spl_store_checkpoint(spl_store *s, const char *path);
int   spl_store_restore(spl_store *s, const char *path);

/* Node stores ("node:NAME", node_store.hpp): one store over a node's per-GPU arenas, key-sharded
 * by ((fnv1a(key) >> 40) & 0xFFFFFF) % nshards.  splinter_create("node:NAME", slots, max_val)
 * creates every shard from one process (SPLINTER_NODE_SHARDS, SPLINTER_NODE_BACKEND=hbm|shm);
 * or each rank creates its shard store (spl_node_shard_name) and joins it, and any process then
 * opens "node:NAME".  backend: 0 host shm shards, 1 HBM shards; stride 128 or 3200. */
int   spl_node_join(const char *name, int shard, int nshards, unsigned backend, size_t slots_per_shard,
                    size_t max_val, unsigned stride);
/* flags SPL_NODE_OWNED: the shard is served only while the joining process lives (HBM shards
 * always: spl_node_join sets it for them); otherwise a host shard outlives its rank like any shm
 * store.  A shard that joins again (a restarted rank) is re-opened by every open node store. */
#define SPL_NODE_OWNED 1u
int   spl_node_join_ex(const char *name, int shard, int nshards, unsigned backend, size_t slots_per_shard,
                       size_t max_val, unsigned stride, unsigned flags);
int   spl_node_leave(const char *name, int shard);
int   spl_node_shard_name(const char *name, int shard, unsigned backend, char *out, size_t cap);
int   spl_node_nshards(spl_store *s);           /* -1 if s is not a node store */
/* Degraded mode of a joined node: 0 shard i serves, 1 its rank's process is gone (ops on its keys
 * return -1/EAGAIN, batch rows -EAGAIN, until the rank's restarted process re-joins), -1 no shard. */
int   spl_node_shard_state(spl_store *s, int shard);
spl_store *spl_node_shard(spl_store *s, int i);
int   spl_node_shard_of(const char *key, int nshards);
int   spl_hbm_device_count(void);               /* libsplinter_hip.so */
/* per-call ring of an hbm: store in this process: 0 its own worker, 1 this process hosts the
 * store's ring server (the owner), 2 it submits to the owner's server; -1 not an hbm: store */
int   spl_hbm_ring_mode(spl_store *s);          /* libsplinter_hip.so */
/* hold (on != 0) / release every per-call ring worker this process runs: no worker is resident
 * while held (per-call ops wait and are served after the release); for a process about to run a
 * heavy GPU job beside the store's clients (a resident worker costs it time-slices).  Nestable. */
void  spl_ring_hold(int on);                    /* libsplinter_hip.so */
/* the same for ONE store's ring from any process that has it open (e.g. a daemon whose store's
 * ring server lives in another process): its worker exits and stays off until released */
int   spl_hbm_ring_hold(spl_store *s, int on);  /* libsplinter_hip.so */

/* Host-array batches (batch_host.cpp): n fixed-stride NUL-padded key records (kstride <= 64), value
 * rows of vstride / ostride bytes, per-op status 0 or -errno (EAGAIN -11, ENOENT -2, ENOSPC -28,
 * EMSGSIZE -90, EPROTOTYPE -91, EINVAL -22, ESTALE -116).  Return: ops that succeeded (-2 on bad
 * arguments).  hbm: stores run the batch through the device kernels (staged in chunks; arrays from
 * spl_batch_alloc move by DMA without a staging copy); node: stores hash-partition the batch and
 * run every shard's part concurrently on its own GPU; host stores loop over the per-call API on
 * `threads` threads.  retries: EAGAIN retries per op (seqlock contention). */
long  spl_set_batch(spl_store *s, const char *keys, int kstride, const uint8_t *vals, int vstride,
                    const uint32_t *lens, long n, int32_t *status, int retries, int threads);
long  spl_get_batch(spl_store *s, const char *keys, int kstride, uint8_t *out, int ostride, uint32_t *out_lens,
                    long n, int32_t *status, int retries, int threads);
long  spl_intop_batch(spl_store *s, const char *keys, int kstride, const int *ops, const uint64_t *masks, long n,
                      int32_t *status, int threads);
/* the same, with each op's resulting u64 value in results[i] */
long  spl_intop_batch_ex(spl_store *s, const char *keys, int kstride, const int *ops, const uint64_t *masks, long n,
                         int32_t *status, uint64_t *results, int threads);
/* vecs [n][768] fp32; expect_epochs (optional): skip (-ESTALE) keys whose epoch moved (daemon write-back) */
long  spl_set_embedding_batch(spl_store *s, const char *keys, int kstride, const float *vecs, long n,
                              const uint64_t *expect_epochs, int32_t *status, int threads);
void *spl_batch_alloc(size_t bytes);   /* pinned when the HBM backend is present; 64-B aligned */
void  spl_batch_free(void *p);

/* bulk helpers (host backends): key -> slot index, -1 if absent */
long  spl_find_slot(spl_store *s, const char *key);
uint64_t spl_hash_key(const char *key);

#ifdef __cplusplus
}
#endif
#endif
