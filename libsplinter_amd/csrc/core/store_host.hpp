// store_host.hpp — host (mmap) backend declaration.
#pragma once
#include <cstddef>
#include <cstdint>
#include <sys/types.h>
#include "splinter_store.hpp"

namespace spl {

uint64_t now_ticks();

// SPLINTER_DEFAULT_UMASK (octal) applied around the creation of a store's shared objects
// (reference splinter.c:131-146); pop restores the process umask.
mode_t env_umask_push();
void env_umask_pop(mode_t prev);

// The HBM backend's factory (libsplinter_hip.so, loaded on first use); nullptr if unavailable.
HbmFactory load_hbm_factory();

// Canonical key: first 63 bytes, NUL padded to 64; hash = FNV-1a of those bytes.
struct KeyRef {
  char buf[kKeyMax];
  size_t len;
  uint64_t hash;
  explicit KeyRef(const char* k);
};

// Shard-table operations on a host-visible header (used by both backends).
int shard_claim_on(splinter_header* H, uint32_t id, uint32_t pid, uint8_t intent, uint8_t prio, uint64_t dur, uint64_t at);
int shard_rebid_on(splinter_header* H, uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur);
int shard_release_on(splinter_header* H, uint32_t id);
bool shard_present_on(splinter_header* H, uint32_t id);
uint32_t shard_election_on(splinter_header* H, uint8_t* out_intent);
int shard_table_on(splinter_header* H, splinter_shard_bid_snapshot* out, size_t max);

class HostStore final : public StoreBase {
 public:
  static HostStore* create(const char* name, bool file_backed, size_t slots, size_t max_val, bool embeddings, int* err);
  static HostStore* open(const char* name, bool file_backed, int* err);
  ~HostStore() override;

  const char* backend() const override { return file_backed_ ? "file" : "shm"; }
  Geometry geometry() const override { return geo_; }
  splinter_header* header_ptr() override { return H_; }
  uint8_t* base() const { return base_; }
  size_t total_bytes() const { return total_; }

  int set_mop(unsigned mode) override;
  int get_mop() override;
  void purge() override;
  int header_snapshot(splinter_header_snapshot_t* out) override;
  uint8_t config_get() override;
  void config_or(uint8_t mask) override;
  void config_and(uint8_t mask) override;

  int set(const char* key, const void* val, size_t len) override;
  int unset(const char* key) override;
  int get(const char* key, void* buf, size_t buf_sz, size_t* out_sz) override;
  int list(char** out_keys, size_t max_keys, size_t* out_count) override;
  int poll(const char* key, uint64_t timeout_ms) override;
  int slot_snapshot(const char* key, splinter_slot_snapshot_t* out) override;
  int append(const char* key, const void* data, size_t len, size_t* new_len) override;
  const void* raw_ptr(const char* key, size_t* out_sz, uint64_t* out_epoch) override;
  uint64_t epoch_of(const char* key) override;
  int set_as_system(const char* key) override;

  int set_embedding(const char* key, const float* vec) override;
  int get_embedding(const char* key, float* out) override;

  int set_named_type(const char* key, uint16_t mask) override;
  int set_slot_time(const char* key, unsigned short mode, uint64_t epoch, size_t offset) override;
  int integer_op(const char* key, splinter_integer_op_t op, const void* mask) override;

  int bump(const char* key) override;
  int retrain(const char* key) override;
  int set_label(const char* key, uint64_t mask) override;
  int unset_label(const char* key, uint64_t mask) override;

  int watch_register(const char* key, uint8_t group) override;
  int watch_unregister(const char* key, uint8_t group) override;
  int watch_label_register(uint64_t bloom_mask, uint8_t group) override;
  int pulse_keygroup(const char* key) override;
  void pulse_slot(splinter_slot* slot) override;
  uint64_t signal_count(uint8_t group) override;
  int signal_add(uint8_t group, uint64_t delta) override;
  void enumerate(uint64_t mask, void (*cb)(const char*, uint64_t, void*), void* ud) override;

  int event_bus_init() override;
  int event_bus_adopt(int fd) override;
  int event_bus_install(int fd);
  int event_bus_open() override;
  void event_bus_dirty(uint64_t* out, size_t words) override;

  int shard_claim_ex(uint32_t id, uint32_t pid, uint8_t intent, uint8_t prio, uint64_t dur, uint64_t at) override;
  int shard_rebid(uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur) override;
  int shard_release(uint32_t id) override;
  uint32_t shard_election(uint8_t* out_intent) override;
  int shard_table(splinter_shard_bid_snapshot* out, size_t max) override;
  int madvise(uint32_t id, void* addr, size_t len, int advice, uint64_t timeout) override;

  // index-level helpers (used by bulk tools and the HBM checkpoint path)
  splinter_slot* slot(size_t i) const { return (splinter_slot*)(base_ + kHeaderBytes + i * geo_.stride); }
  uint8_t* value(size_t i) const { return base_ + geo_.values_offset() + i * (size_t)geo_.max_val; }
  float* embedding(size_t i) const { return (float*)((uint8_t*)slot(i) + kOffEmbed); }
  long find(const KeyRef& k) const;

 private:
  HostStore() = default;
  void init_fresh();
  bool key_eq(const splinter_slot* s, const KeyRef& k) const;
  void notify(size_t idx);
  void bump_global(uint64_t n);
  bool scrub_on() const;
  bool hybrid_on() const;
  int write_locked(size_t idx, const KeyRef& k, const void* val, size_t len, bool fresh);

  uint8_t* base_ = nullptr;
  size_t total_ = 0;
  Geometry geo_;
  splinter_header* H_ = nullptr;
  bool file_backed_ = false;
  int event_fd_ = -1;
};

}  // namespace spl
