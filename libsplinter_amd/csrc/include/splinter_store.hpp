// splinter_store.hpp — backend-neutral store interface.
//
// The reference keeps one process-global store (reference splinter.c:47-57).
// libsplinter_amd keeps that C API (splinter_*) as a thin shim over a "current
// store" pointer, but every operation is implemented on a StoreBase object so
// that one process can hold several stores (Python bindings, sharded arenas,
// tests) and so that the HBM backend (libsplinter_hip.so, loaded on demand)
// plugs in behind the same calls.  Only POD types cross this interface, so the
// g++-built host library and the hipcc-built HBM backend share it safely.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cerrno>
#include "splinter.h"
#include "splinter_layout.hpp"

namespace spl {

enum CreateFlags : unsigned {
  kCreateEmbeddings = 1u << 0,  // 3200-B slots with float[768]
  kCreatePersistent = 1u << 1,  // regular file instead of POSIX shm
  kCreateNoEmbeddings = 1u << 2,
};
// HBM factory flags: device ordinal + 1 in bits 16..23 (0 = the caller's current device)
constexpr unsigned kCreateDeviceShift = 16;

class StoreBase {
 public:
  virtual ~StoreBase() {}
  virtual const char* backend() const = 0;
  virtual Geometry geometry() const = 0;
  // host-visible header (host backend: the mapped header; hbm: nullptr)
  virtual splinter_header* header_ptr() = 0;

  // store-wide
  virtual int set_mop(unsigned mode) = 0;
  virtual int get_mop() = 0;
  virtual void purge() = 0;
  virtual int header_snapshot(splinter_header_snapshot_t* out) = 0;
  virtual uint8_t config_get() = 0;
  virtual void config_or(uint8_t mask) = 0;
  virtual void config_and(uint8_t mask) = 0;

  // key/value
  virtual int set(const char* key, const void* val, size_t len) = 0;
  virtual int unset(const char* key) = 0;
  virtual int get(const char* key, void* buf, size_t buf_sz, size_t* out_sz) = 0;
  virtual int list(char** out_keys, size_t max_keys, size_t* out_count) = 0;
  virtual int poll(const char* key, uint64_t timeout_ms) = 0;
  virtual int slot_snapshot(const char* key, splinter_slot_snapshot_t* out) = 0;
  virtual int append(const char* key, const void* data, size_t len, size_t* new_len) = 0;
  virtual const void* raw_ptr(const char* key, size_t* out_sz, uint64_t* out_epoch) = 0;
  virtual uint64_t epoch_of(const char* key) = 0;
  virtual int set_as_system(const char* key) = 0;

  // embeddings
  virtual int set_embedding(const char* key, const float* vec) = 0;
  virtual int get_embedding(const char* key, float* out) = 0;

  // typing / time / integers
  virtual int set_named_type(const char* key, uint16_t mask) = 0;
  virtual int set_slot_time(const char* key, unsigned short mode, uint64_t epoch, size_t offset) = 0;
  virtual int integer_op(const char* key, splinter_integer_op_t op, const void* mask) = 0;

  // epochs / labels
  virtual int bump(const char* key) = 0;
  virtual int retrain(const char* key) = 0;
  virtual int set_label(const char* key, uint64_t mask) = 0;
  virtual int unset_label(const char* key, uint64_t mask) = 0;

  // signals
  virtual int watch_register(const char* key, uint8_t group) = 0;
  virtual int watch_unregister(const char* key, uint8_t group) = 0;
  virtual int watch_label_register(uint64_t bloom_mask, uint8_t group) = 0;
  virtual int pulse_keygroup(const char* key) = 0;
  virtual void pulse_slot(splinter_slot* slot) = 0;
  virtual uint64_t signal_count(uint8_t group) = 0;
  // atomic counter += delta (node-wide signal propagation of a sharded arena, parallel/signals.py)
  virtual int signal_add(uint8_t group, uint64_t delta) = 0;
  virtual void enumerate(uint64_t mask, void (*cb)(const char*, uint64_t, void*), void* ud) = 0;

  // event bus
  virtual int event_bus_init() = 0;
  // make an existing eventfd (dup'd) this store's bus: the shards of a node store share the node's
  // one eventfd, so every writer on any shard signals the same counter
  virtual int event_bus_adopt(int fd) { (void)fd; errno = ENOTSUP; return -1; }
  virtual int event_bus_open() = 0;
  virtual void event_bus_dirty(uint64_t* out, size_t words) = 0;

  // logic shards
  virtual int shard_claim_ex(uint32_t id, uint32_t pid, uint8_t intent, uint8_t prio,
                             uint64_t dur, uint64_t at) = 0;
  virtual int shard_rebid(uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur) = 0;
  virtual int shard_release(uint32_t id) = 0;
  virtual uint32_t shard_election(uint8_t* out_intent) = 0;
  virtual int shard_table(splinter_shard_bid_snapshot* out, size_t max) = 0;
  virtual int madvise(uint32_t id, void* addr, size_t len, int advice, uint64_t timeout) = 0;

  // Batched host-array ops (splinter_ext.h spl_*_batch; fixed-stride NUL-padded key records, value
  // rows of vstride bytes, per-op status 0 / -errno).  A backend with a native batch path (HBM:
  // staged through the device kernels; node: hash-partitioned over the shards concurrently)
  // returns the number of ops that succeeded; kNoBatch makes the caller loop over the per-call API.
  static constexpr long kNoBatch = -(1L << 62);
  virtual long set_batch(const char*, int, const uint8_t*, int, const uint32_t*, long, int32_t*, int) {
    return kNoBatch;
  }
  virtual long get_batch(const char*, int, uint8_t*, int, uint32_t*, long, int32_t*, int) { return kNoBatch; }
  virtual long intop_batch(const char*, int, const int*, const uint64_t*, long, int32_t*, uint64_t*) {
    return kNoBatch;
  }
  virtual long set_embedding_batch(const char*, int, const float*, long, int32_t*) { return kNoBatch; }
};

// The per-call loops behind spl_*_batch (batch_host.cpp), for backends without a native path and
// for the host shards of a node store.
long generic_set_batch(StoreBase* s, const char* keys, int kstride, const uint8_t* vals, int vstride,
                       const uint32_t* lens, long n, int32_t* status, int retries, int threads);
long generic_get_batch(StoreBase* s, const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens,
                       long n, int32_t* status, int retries, int threads);
long generic_intop_batch(StoreBase* s, const char* keys, int kstride, const int* ops, const uint64_t* masks, long n,
                         int32_t* status, uint64_t* results, int threads);
long generic_set_embedding_batch(StoreBase* s, const char* keys, int kstride, const float* vecs, long n,
                                 const uint64_t* expect_epochs, int32_t* status, int threads);

// Factory entry point exported by libsplinter_hip.so for "hbm:" stores.
typedef StoreBase* (*HbmFactory)(const char* name, size_t slots, size_t max_val,
                                 unsigned flags, int create, int* err);

}  // namespace spl
