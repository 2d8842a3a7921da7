/*
 * splinter.h — public C ABI of libsplinter_amd.
 *
 * This is a from-scratch implementation of the splinterhq/libsplinter v1.2.0
 * API surface (reference: /root/reference/splinter.h:29-1213).  Function names,
 * argument lists, return conventions and the on-memory format v4 byte layout
 * are kept identical so that existing clients (TS/Rust/Lua/ctypes bindings,
 * splinterctl scripts, reference-built stores in /dev/shm) interoperate.
 *
 * Differences from the reference, all deliberate and documented in
 * docs/DIVERGENCES.md:
 *   - one library serves both 128-B (plain) and 3200-B (embedding) slot strides;
 *     the stride is recorded at create time in the unused `alignment` header
 *     word and re-derived from the region size on open (the reference records
 *     nothing and silently mis-maps);
 *   - store names select a backend: "name" → POSIX shm, a path containing '/'
 *     (or the persistent build) → regular file, "hbm:name" → HBM arena on the
 *     GPU (libsplinter_hip.so, loaded on demand);
 *   - `set` claims an empty slot by CAS on `hash` (no duplicate keys under
 *     racing writers); BIGUINT promotion converts in place (no val_brk alias).
 *
 * Return convention (unchanged): 0 ok, -1 recoverable (errno), -2 caller error.
 */
#ifndef SPLINTER_H
#define SPLINTER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#define SPL_ALIGNAS(n) alignas(n)
extern "C" {
#else
#include <stdalign.h>
#define SPL_ALIGNAS(n) _Alignas(n)
#endif

/* ---- format constants (format v4) -------------------------------------- */
#define SPLINTER_MAGIC      0x534C4E54u   /* "SLNT" */
#define SPLINTER_VER        4
#define SPLINTER_KEY_MAX    64
#define NS_PER_MS           1000000ULL
#ifndef SPLINTER_NO_EMBEDDINGS
#ifndef SPLINTER_EMBEDDINGS
#define SPLINTER_EMBEDDINGS 1
#endif
#endif
#define SPLINTER_EMBED_DIM  768
#define SPLINTER_MAX_GROUPS 64
#define SPLINTER_MAX_SHARDS 32
#define SPLINTER_MAX_SLOTS  1024
#define SPLINTER_EVENT_BUS_MASK_WORDS (SPLINTER_MAX_SLOTS / 64)

/* store (core) flags */
#define SPL_SYS_AUTO_SCRUB     (1u << 0)
#define SPL_SYS_HYBRID_SCRUB   (1u << 1)
#define SPL_SYS_RESERVED_2     (1u << 2)
#define SPL_SYS_RESERVED_3     (1u << 3)
#define SPL_SUSR1              (1u << 4)
#define SPL_SUSR2              (1u << 5)
#define SPL_SUSR3              (1u << 6)
#define SPL_SUSR4              (1u << 7)

/* slot named types */
#define SPL_SLOT_TYPE_VOID     (1u << 0)
#define SPL_SLOT_TYPE_BIGINT   (1u << 1)
#define SPL_SLOT_TYPE_BIGUINT  (1u << 2)
#define SPL_SLOT_TYPE_JSON     (1u << 3)
#define SPL_SLOT_TYPE_BINARY   (1u << 4)
#define SPL_SLOT_TYPE_IMGDATA  (1u << 5)
#define SPL_SLOT_TYPE_AUDIO    (1u << 6)
#define SPL_SLOT_TYPE_VARTEXT  (1u << 7)
#define SPL_SLOT_DEFAULT_TYPE  SPL_SLOT_TYPE_VOID

/* per-slot user flags */
#define SPL_FUSR1 (1u << 0)
#define SPL_FUSR2 (1u << 1)
#define SPL_FUSR3 (1u << 2)
#define SPL_FUSR4 (1u << 3)
#define SPL_FUSR5 (1u << 4)
#define SPL_FUSR6 (1u << 5)
#define SPL_FUSR7 (1u << 6)
#define SPL_FUSR8 (1u << 7)

#define SPL_TIME_CTIME 0
#define SPL_TIME_ATIME 1

/* tandem-key order separator: "car", "car.1", "car.2" … */
#define SPL_ORDER_ACCESSOR "."

typedef enum {
    SPL_INTENT_NONE       = 0,
    SPL_INTENT_WILLNEED   = 1,
    SPL_INTENT_SEQUENTIAL = 2,
    SPL_INTENT_RANDOM     = 3,
    SPL_INTENT_DONTNEED   = 4
} splinter_intent_t;

typedef enum {
    SPL_OP_AND,
    SPL_OP_OR,
    SPL_OP_XOR,
    SPL_OP_NOT,
    SPL_OP_INC,
    SPL_OP_DEC
} splinter_integer_op_t;

/* ---- shared-memory layout ------------------------------------------------
 * All multi-byte fields are accessed with atomic builtins by the library; they
 * are declared as plain integers so the header is valid C, C++ and HIP.      */

struct splinter_signal_node {
    SPL_ALIGNAS(64) uint64_t counter;
};

struct splinter_event_bus {
    uint64_t dirty_mask[SPLINTER_EVENT_BUS_MASK_WORDS];
    int32_t  owner_fd;
    int32_t  owner_pid;
};

struct splinter_shard_bid {
    uint32_t shard_id;      /* 0 = free record */
    uint32_t pid;
    uint8_t  intent;
    uint8_t  priority;
    uint8_t  _pad[2];
    uint64_t duration_tsc;
    uint64_t claimed_at;
};

struct splinter_header {
    uint32_t magic;
    uint32_t version;
    uint32_t slots;
    uint32_t max_val_sz;
    uint64_t epoch;                 /* global write counter */
    uint8_t  core_flags;
    uint8_t  user_flags;
    uint32_t val_brk;
    uint32_t val_sz;                /* low 32 bits of the region size */
    uint32_t alignment;             /* libsplinter_amd: slot stride (128/3200) */
    uint64_t parse_failures;
    uint64_t last_failure_epoch;
    uint8_t  bloom_watches[64];     /* label bit -> signal group, 0xFF = none */
    SPL_ALIGNAS(64) struct splinter_signal_node signal_groups[SPLINTER_MAX_GROUPS];
    SPL_ALIGNAS(64) struct splinter_event_bus event_bus;
    SPL_ALIGNAS(64) struct splinter_shard_bid shard_bids[SPLINTER_MAX_SHARDS];
};

/* The fixed 128-byte slot core.  Stores created with embeddings append
 * float[SPLINTER_EMBED_DIM] directly after `key` (slot stride 3200 B).    */
struct splinter_slot {
    SPL_ALIGNAS(64) uint64_t hash;  /* FNV-1a of key, 0 = empty */
    uint64_t epoch;                 /* seqlock: odd = writer active */
    uint32_t val_off;
    uint32_t val_len;
    uint8_t  type_flag;
    uint8_t  user_flag;
    uint64_t watcher_mask;
    uint64_t ctime;
    uint64_t atime;
    uint64_t bloom;
    char     key[SPLINTER_KEY_MAX];
};

typedef struct splinter_header_snapshot {
    uint32_t magic;
    uint32_t version;
    uint32_t slots;
    uint32_t max_val_sz;
    uint64_t epoch;
    uint8_t  core_flags;
    uint8_t  user_flags;
    uint64_t parse_failures;
    uint64_t last_failure_epoch;
} splinter_header_snapshot_t;

typedef struct splinter_slot_snapshot {
    uint64_t hash;
    uint64_t epoch;
    uint32_t val_off;
    uint32_t val_len;
    uint8_t  type_flag;
    uint8_t  user_flag;
    uint64_t ctime;
    uint64_t atime;
    uint64_t bloom;
    char     key[SPLINTER_KEY_MAX];
#ifdef SPLINTER_EMBEDDINGS
    float    embedding[SPLINTER_EMBED_DIM];
#endif
} splinter_slot_snapshot_t;

struct splinter_shard_bid_snapshot {
    uint32_t shard_id;
    uint32_t pid;
    uint8_t  intent;
    uint8_t  priority;
    uint64_t duration_tsc;
    uint64_t claimed_at;
    int      expired;
    int      sovereign;
};

/* ---- lifecycle ----------------------------------------------------------- */
int   splinter_create(const char *name_or_path, size_t slots, size_t max_value_sz);
int   splinter_open(const char *name_or_path);
void *splinter_open_numa(const char *name, int target_node);
int   splinter_open_or_create(const char *name_or_path, size_t slots, size_t max_value_sz);
int   splinter_create_or_open(const char *name_or_path, size_t slots, size_t max_value_sz);
void  splinter_close(void);

/* ---- store-wide ---------------------------------------------------------- */
int   splinter_set_mop(unsigned int mode);
int   splinter_get_mop(void);
void  splinter_purge(void);
int   splinter_get_header_snapshot(splinter_header_snapshot_t *snapshot);

/* ---- key/value ----------------------------------------------------------- */
int   splinter_set(const char *key, const void *val, size_t len);
int   splinter_unset(const char *key);
int   splinter_get(const char *key, void *buf, size_t buf_sz, size_t *out_sz);
int   splinter_list(char **out_keys, size_t max_keys, size_t *out_count);
int   splinter_poll(const char *key, uint64_t timeout_ms);
int   splinter_get_slot_snapshot(const char *key, splinter_slot_snapshot_t *snapshot);
int   splinter_append(const char *key, const void *data, size_t data_len, size_t *new_len);
const void *splinter_get_raw_ptr(const char *key, size_t *out_sz, uint64_t *out_epoch);
uint64_t splinter_get_epoch(const char *key);
int   splinter_set_as_system(const char *key);

/* ---- embeddings ---------------------------------------------------------- */
int   splinter_set_embedding(const char *key, const float *embedding);
int   splinter_get_embedding(const char *key, float *embedding_out);

/* ---- flags --------------------------------------------------------------- */
void     splinter_config_set(struct splinter_header *hdr, uint8_t mask);
void     splinter_config_clear(struct splinter_header *hdr, uint8_t mask);
int      splinter_config_test(struct splinter_header *hdr, uint8_t mask);
uint8_t  splinter_config_snapshot(struct splinter_header *hdr);
void     splinter_slot_usr_set(struct splinter_slot *slot, uint16_t mask);
void     splinter_slot_usr_clear(struct splinter_slot *slot, uint16_t mask);
int      splinter_slot_usr_test(struct splinter_slot *slot, uint16_t mask);
uint16_t splinter_slot_usr_snapshot(struct splinter_slot *slot);

/* ---- typing, time, integers ---------------------------------------------- */
int   splinter_set_named_type(const char *key, uint16_t mask);
int   splinter_set_slot_time(const char *key, unsigned short mode, uint64_t epoch, size_t offset);
int   splinter_integer_op(const char *key, splinter_integer_op_t op, const void *mask);

/* Monotonic tick source used for shard windows and ctime backfill. */
uint64_t splinter_now_ticks(void);
#ifndef SPLINTER_NO_INLINE_NOW
static inline uint64_t splinter_now(void) { return splinter_now_ticks(); }
#endif

/* ---- epochs, labels, tandem ---------------------------------------------- */
int   splinter_bump_slot(const char *key);
int   splinter_retrain_slot(const char *key);
int   splinter_set_label(const char *key, uint64_t mask);
int   splinter_unset_label(const char *key, uint64_t mask);
int   splinter_client_set_tandem(const char *base_key, const void **vals,
                                 const size_t *lens, uint8_t orders);
void  splinter_client_unset_tandem(const char *base_key, uint8_t orders);

/* ---- signals ------------------------------------------------------------- */
int      splinter_watch_register(const char *key, uint8_t group_id);
int      splinter_watch_unregister(const char *key, uint8_t group_id);
int      splinter_watch_label_register(uint64_t bloom_mask, uint8_t group_id);
void     splinter_pulse_watchers(struct splinter_slot *slot);
int      splinter_pulse_keygroup(const char *key);
uint64_t splinter_get_signal_count(uint8_t group_id);
void     splinter_enumerate_matches(uint64_t mask,
                                    void (*callback)(const char *key, uint64_t epoch, void *data),
                                    void *user_data);

/* ---- event bus ----------------------------------------------------------- */
int   splinter_event_bus_init(void);
int   splinter_event_bus_open(void);
int   splinter_event_bus_wait(int fd, uint64_t timeout_ms);
void  splinter_event_bus_close(int fd);
void  splinter_event_bus_get_dirty(uint64_t *out, size_t words);

/* ---- logic shard election / cooperative madvise -------------------------- */
int      splinter_shard_claim(uint32_t shard_id, uint8_t intent, uint8_t priority, uint64_t duration_tsc);
int      splinter_shard_claim_ex(uint32_t shard_id, uint32_t pid, uint8_t intent,
                                 uint8_t priority, uint64_t duration_tsc, uint64_t claimed_at);
int      splinter_shard_rebid(uint32_t shard_id, uint8_t intent, uint8_t priority, uint64_t duration_tsc);
int      splinter_shard_release(uint32_t shard_id);
uint32_t splinter_shard_election(uint8_t *out_intent);
int      splinter_shard_is_sovereign(uint32_t shard_id);
int      splinter_shard_table_snapshot(struct splinter_shard_bid_snapshot *out, size_t max);
int      splinter_madvise(uint32_t shard_id, void *addr, size_t len, int advice, uint64_t timeout_ticks);

#ifdef __cplusplus
}
#endif
#endif /* SPLINTER_H */
