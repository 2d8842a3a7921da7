// node_store.hpp — one store spanning the GPUs of a node ("node:NAME").
//
// The reference has one store per host that every process maps (reference splinter.c:235-248);
// its only scale-out idea is disjoint key lanes (splinter_chi_sao.c:400-418).  A node store keeps
// the per-process API of that single store while its key space is hash-sharded over one arena per
// GPU: shard(key) = ((fnv1a(key) >> 40) & 0xFFFFFF) % nshards, the same function as the batched
// RCCL path (parallel/sharded.py shard_of, hip/route_kernels.hip shard_of_hash), so stores created
// by the bench's ranks and keys routed by the collectives land where a C-ABI client looks for them.
//
//   per-call key ops      -> the owning shard (its command ring on its GPU)
//   set_mop / config bits -> every shard (replicated on write)
//   watch_label_register  -> every shard (C6)
//   signal counts         -> sum over shards (C2: a pulse on any GPU is seen by every watcher)
//   list / enumerate      -> concatenation over shards (C5)
//   event bus             -> one eventfd fed by every shard's
//   logic-shard bids      -> the node descriptor's control header (one election per node)
//
// Shards are HBM arenas "hbm:NAME.s<i>" (one per device) or, for CPU rehearsals, host stores
// "shm:NAME.s<i>".  A node descriptor (POSIX shm "NAME.node") records the geometry and which
// shards exist: one process can create the whole node (splinter_create("node:NAME")), or every
// rank creates its own shard and joins it (spl_node_join), and any process then opens "node:NAME".
#pragma once
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "store_host.hpp"

namespace spl {

constexpr uint32_t kNodeMagic = 0x45444f4e;  // "NODE"
constexpr int kNodeMaxShards = 64;
// a shard whose memory lives and dies with its rank's process (HBM shards always; host shards when
// the rank joins with SPL_NODE_OWNED): it is down while that process is gone
constexpr uint32_t kShardOwned = 1u;

struct NodeDesc {
  uint32_t magic;
  uint32_t version;
  uint32_t nshards;
  uint32_t backend;          // 0 host shm shards, 1 HBM shards
  uint32_t slots_per_shard;
  uint32_t max_val;
  uint32_t stride;
  uint32_t pad0;
  uint64_t ready_mask;       // shard i exists (created and joined)
  int32_t creator_pid;       // single-process creation: the owner of every shard; 0 for joined ranks
  int32_t event_pid;         // node event bus: owner pid and fd of the forwarded eventfd
  int32_t event_fd;
  int32_t pad1;
  // rank ownership of joined shards (spl_node_join): the owning process and how many times the
  // shard has joined -- a rank restarted from its checkpoint re-joins with gen + 1, and every open
  // node store then re-opens that shard (NodeStore::refresh)
  int32_t shard_pid[kNodeMaxShards];
  uint32_t shard_gen[kNodeMaxShards];
  uint32_t shard_flags[kNodeMaxShards];  // kShardOwned: served only while shard_pid lives
  alignas(64) splinter_header control;  // node-level logic-shard bid table (shard_bids only)
};

inline int node_shard_of(uint64_t hash, int nshards) {
  return (int)(((hash >> 40) & 0xFFFFFFull) % (uint64_t)nshards);
}

class NodeStore final : public StoreBase {
 public:
  static NodeStore* create(const std::string& name, size_t slots, size_t max_val, bool emb, int* err);
  static NodeStore* open(const std::string& name, int* err);
  ~NodeStore() override;

  int nshards() const { return (int)shards_.size(); }
  StoreBase* shard(int i) const { return (i >= 0 && i < nshards()) ? __atomic_load_n(&shards_[i], __ATOMIC_ACQUIRE) : nullptr; }
  StoreBase* route(const char* key);
  // Degraded mode (joined nodes): a shard whose owning rank process is gone answers every op with
  // EAGAIN (DownShard) while the other shards keep serving; when the rank's restarted process
  // re-joins (shard_gen moved) the shard is re-opened.  Checked at most every kRefreshNs per store.
  void refresh(bool force = false);
  // 0 serving, 1 down (owner gone), -1 no such shard
  int shard_state(int i);

  const char* backend() const override { return "node"; }
  Geometry geometry() const override;
  splinter_header* header_ptr() override { return &desc_->control; }

  int set_mop(unsigned mode) override;
  int get_mop() override { return first_up()->get_mop(); }
  void purge() override { for (auto* s : shards_) s->purge(); }
  int header_snapshot(splinter_header_snapshot_t* out) override;
  uint8_t config_get() override { return first_up()->config_get(); }
  void config_or(uint8_t m) override { for (auto* s : shards_) s->config_or(m); }
  void config_and(uint8_t m) override { for (auto* s : shards_) s->config_and(m); }

  int set(const char* k, const void* v, size_t n) override { return k ? route(k)->set(k, v, n) : -2; }
  int unset(const char* k) override { return k ? route(k)->unset(k) : -2; }
  int get(const char* k, void* b, size_t n, size_t* o) override { return k ? route(k)->get(k, b, n, o) : -2; }
  int list(char** out_keys, size_t max_keys, size_t* out_count) override;
  int poll(const char* k, uint64_t ms) override { return k ? route(k)->poll(k, ms) : -2; }
  int slot_snapshot(const char* k, splinter_slot_snapshot_t* o) override { return k ? route(k)->slot_snapshot(k, o) : -2; }
  int append(const char* k, const void* d, size_t n, size_t* nl) override { return k ? route(k)->append(k, d, n, nl) : -2; }
  const void* raw_ptr(const char* k, size_t* sz, uint64_t* ep) override { return k ? route(k)->raw_ptr(k, sz, ep) : nullptr; }
  uint64_t epoch_of(const char* k) override { return k ? route(k)->epoch_of(k) : 0; }
  int set_as_system(const char* k) override { return k ? route(k)->set_as_system(k) : -2; }

  int set_embedding(const char* k, const float* v) override { return k ? route(k)->set_embedding(k, v) : -2; }
  int get_embedding(const char* k, float* o) override { return k ? route(k)->get_embedding(k, o) : -2; }

  int set_named_type(const char* k, uint16_t m) override { return k ? route(k)->set_named_type(k, m) : -2; }
  int set_slot_time(const char* k, unsigned short mode, uint64_t e, size_t off) override {
    return k ? route(k)->set_slot_time(k, mode, e, off) : -2;
  }
  int integer_op(const char* k, splinter_integer_op_t op, const void* m) override {
    return k ? route(k)->integer_op(k, op, m) : -2;
  }

  int bump(const char* k) override { return k ? route(k)->bump(k) : -2; }
  int retrain(const char* k) override { return k ? route(k)->retrain(k) : -2; }
  int set_label(const char* k, uint64_t m) override { return k ? route(k)->set_label(k, m) : -2; }
  int unset_label(const char* k, uint64_t m) override { return k ? route(k)->unset_label(k, m) : -2; }

  int watch_register(const char* k, uint8_t g) override { return k ? route(k)->watch_register(k, g) : -2; }
  int watch_unregister(const char* k, uint8_t g) override { return k ? route(k)->watch_unregister(k, g) : -2; }
  int watch_label_register(uint64_t mask, uint8_t g) override;
  int pulse_keygroup(const char* k) override { return k ? route(k)->pulse_keygroup(k) : -2; }
  void pulse_slot(splinter_slot*) override {}
  uint64_t signal_count(uint8_t g) override;
  int signal_add(uint8_t g, uint64_t delta) override { return first_up()->signal_add(g, delta); }
  void enumerate(uint64_t mask, void (*cb)(const char*, uint64_t, void*), void* ud) override {
    for (auto* s : shards_) s->enumerate(mask, cb, ud);
  }

  int event_bus_init() override;
  int event_bus_open() override;
  void event_bus_dirty(uint64_t* out, size_t words) override;

  int shard_claim_ex(uint32_t id, uint32_t pid, uint8_t intent, uint8_t prio, uint64_t dur, uint64_t at) override {
    return shard_claim_on(&desc_->control, id, pid, intent, prio, dur, at);
  }
  int shard_rebid(uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur) override {
    return shard_rebid_on(&desc_->control, id, intent, prio, dur);
  }
  int shard_release(uint32_t id) override { return shard_release_on(&desc_->control, id); }
  uint32_t shard_election(uint8_t* out_intent) override { return shard_election_on(&desc_->control, out_intent); }
  int shard_table(splinter_shard_bid_snapshot* out, size_t max) override {
    return shard_table_on(&desc_->control, out, max);
  }
  int madvise(uint32_t id, void* addr, size_t len, int advice, uint64_t timeout) override;

  // host-array batches: hash-partitioned over the shards, every shard's part run concurrently
  // (HBM shards: each on its own GPU through its device batch path)
  long set_batch(const char* keys, int kstride, const uint8_t* vals, int vstride, const uint32_t* lens, long n,
                 int32_t* status, int retries) override;
  long get_batch(const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens, long n,
                 int32_t* status, int retries) override;
  long intop_batch(const char* keys, int kstride, const int* ops, const uint64_t* masks, long n, int32_t* status,
                   uint64_t* results) override;
  long set_embedding_batch(const char* keys, int kstride, const float* vecs, long n, int32_t* status) override;

 private:
  NodeStore() = default;
  struct Plan;  // node_store.cpp: a batch's shard partition
  template <class Prep, class Exec>
  long pipeline(long n, long per, Prep&& prep, Exec&& exec);  // node_store.cpp: chunked batches
  long chunk_for(long n) const;
  uint8_t* scratch(size_t bytes);
  std::mutex scratch_mu_;
  std::vector<long> plan_pos_[2];      // Plan storage per pipeline half (grown, never shrunk or
  std::vector<int32_t> plan_dest_[2];  // zeroed again: no page faults on later batches)
  uint8_t* scratch_ = nullptr;
  size_t scratch_bytes_ = 0;
  bool scratch_pinned_ = false;

  StoreBase* at(int i) const { return __atomic_load_n(&shards_[(size_t)i], __ATOMIC_ACQUIRE); }
  // node-wide reads (mop, config, the node signal counter) from the first serving shard
  StoreBase* first_up() const {
    for (int i = 0; i < nshards(); ++i)
      if (at(i) != down_) return at(i);
    return at(0);
  }

  std::string name_;
  NodeDesc* desc_ = nullptr;
  bool owner_ = false;  // created the descriptor and every shard
  std::vector<StoreBase*> shards_;   // routing table (entries swapped atomically by refresh)
  std::vector<StoreBase*> real_;     // the opened shard stores (a down shard keeps its handle here)
  std::vector<uint32_t> gen_;        // shard_gen of each opened handle
  std::vector<StoreBase*> retired_;  // handles replaced by a re-open (another thread may still hold one)
  StoreBase* down_ = nullptr;        // the EAGAIN stand-in of down shards
  std::mutex refresh_mu_;
  std::atomic<uint64_t> next_refresh_ns_{0};
  int event_fd_ = -1;
};

// shard store name of shard i of node NAME, with its backend prefix ("hbm:" / "shm:")
std::string node_shard_name(const std::string& node, int i, uint32_t backend);

}  // namespace spl
