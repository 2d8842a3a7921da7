// hbm_store.hip — the HBM backend: a format-v4 arena resident in MI355X HBM.
//
// Data plane (header counters, slots, values, vectors) lives in device memory
// and is mutated only by the kernels of arena_kernels.hip (owner computes).
// Control plane lives in a POSIX shm descriptor "<name>.hbm":
//   - geometry, device ordinal, owner pid and a hipIpcMemHandle_t, so any
//     process on the node can hipIpcOpenMemHandle() the same arena zero-copy;
//   - a host-resident splinter_header mirror carrying the shard bid table and
//     the event-bus owner (host atomics; shard election is host logic).
// The per-call StoreBase API goes through the command ring of cmd_ring.hpp (a resident one-wave
// device worker serving pinned host records: a few µs per call, many host threads batched into
// one wave round); bulk work goes through the batch launchers (arena_api.h) directly.
#include <hip/hip_runtime.h>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <algorithm>
#include <cfloat>
#include <functional>
#include <cmath>
#include <atomic>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <poll.h>
#include <string>
#include <thread>
#include <sys/eventfd.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <vector>

#include "arena_api.h"
#include "cmd_ring.hpp"
#include "search_api.h"
#include "vmm_share.hpp"
#include "splinter_ext.h"
#include "splinter_store.hpp"
#include "store_host.hpp"

namespace spl {

namespace {

constexpr uint32_t kDescMagic = 0x48424d41;  // "HBMA"
constexpr size_t kAlignOffset = 64;          // base % 128 == 64 -> every 128-B slot is line aligned

struct HbmDescriptor {
  uint32_t magic;
  uint32_t version;
  uint32_t slots, max_val, stride, device;
  uint64_t total_bytes;
  uint64_t base_offset;
  int32_t owner_pid;
  int32_t pad;
  hipIpcMemHandle_t handle;              // mode 0: one hipMalloc allocation, hipIpc
  uint32_t mode;                         // 0 hipIpc, 1 VMM chunks (vmm_share.hpp)
  uint32_t nchunks;
  uint64_t chunk_bytes;
  uint32_t side_flags;                   // SPL_ARENA_SIDE | SPL_ARENA_VEC16: the allocation's side region
  uint32_t pad2;
  char sock[96];                         // mode 1: abstract socket serving the chunk fds
  alignas(64) splinter_header control;  // host control plane (shard bids, event bus owner)
  alignas(64) uint32_t notify;          // event-bus doorbell: set by kernels / per-call writers,
                                        // cleared by the owner's proxy thread
};

#define HIPCHECK(x)                                                             \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "libsplinter_hip: %s failed: %s\n", #x, hipGetErrorString(e_)); \
      return -1;                                                                \
    }                                                                           \
  } while (0)

// The calling thread's current device switched to a store's device for the scope (a process may
// hold arenas on several GPUs: a node store).
struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev >= 0 && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int neg_to_errno(int32_t st) {
  switch (st) {
    case -11: return EAGAIN;
    case -2: return ENOENT;
    case -28: return ENOSPC;
    case -90: return EMSGSIZE;
    case -91: return EPROTOTYPE;
    default: return EINVAL;
  }
}

}  // namespace

// Candidate thresholds shared by the shards of one node search (spl_search_batch on node:): per
// 256-query block every participating shard posts the k largest sampled tile maxima of each query
// (k_search_thr's topv: k real slots of ITS arena at or above each value) and continues with the
// threshold of their union -- the k-th largest over all shards' samples minus the bf16 margin, a
// lower bound of every query's k-th best similarity over the whole node, as tight as one store
// sampling the same slots -- so the shards' candidate and re-score work stays what one store of
// all the slots would do instead of growing with the shard count.  A shard with nothing to post
// (exact kernel, distance-bounded batch) posts nothing and takes the result; a shard that stops
// early (error) leaves, so nobody waits for it.
struct SearchSync {
  std::mutex mu;
  std::condition_variable cv;
  int active = 0, arrived = 0;
  uint64_t gen = 0;
  std::vector<std::vector<float>> posts;
  std::vector<float> result;
  int m = 0, k = 0;
  float delta2 = 0.f, floor_v = 0.f;
  explicit SearchSync(int n) : active(n) {}
  void release() {
    result.assign((size_t)m, floor_v);
    std::vector<float> u;
    for (int i = 0; i < m; ++i) {
      u.clear();
      for (auto& p : posts)
        for (int j = 0; j < k; ++j) {
          const float v = p[(size_t)i * k + j];
          if (v > -FLT_MAX) u.push_back(v);
        }
      if ((int)u.size() >= k) {
        std::nth_element(u.begin(), u.begin() + (k - 1), u.end(), std::greater<float>());
        result[(size_t)i] = std::max(u[(size_t)(k - 1)] - delta2, floor_v);
      }
    }
    posts.clear();
    arrived = 0;
    ++gen;
    cv.notify_all();
  }
  // topv: [mq][kq] or nullptr; thr: [mq] out
  void merge(const float* topv, int mq, int kq, float d2, float fl, float* thr) {
    std::unique_lock<std::mutex> l(mu);
    m = mq, k = kq, delta2 = d2, floor_v = fl;
    if (topv) posts.emplace_back(topv, topv + (size_t)mq * kq);
    ++arrived;
    const uint64_t g = gen;
    if (arrived >= active) release();
    else cv.wait(l, [&] { return gen != g; });
    for (int i = 0; i < mq && i < (int)result.size(); ++i) thr[i] = result[(size_t)i];
  }
  void leave() {
    std::lock_guard<std::mutex> l(mu);
    --active;
    if (arrived > 0 && arrived >= active) release();
  }
};

class HbmStore final : public StoreBase {
 public:
  static HbmStore* create(const char* name, size_t slots, size_t max_val, bool emb, int* err);
  static HbmStore* open(const char* name, int* err);
  ~HbmStore() override;

  const char* backend() const override { return "hbm"; }
  Geometry geometry() const override { return geo_; }
  splinter_header* header_ptr() override { return &desc_->control; }
  spl_arena_t arena() const {
    spl_arena_t a;
    a.base = dbase_;
    a.slots = geo_.slots;
    a.max_val = geo_.max_val;
    a.stride = geo_.stride;
    a.flags = (event_fd_ >= 0 ? SPL_ARENA_EVENTBUS : 0u) | side_flags_;
    a.notify = (uint64_t)(uintptr_t)d_notify_;
    return a;
  }
  hipStream_t stream() const { return stream_; }
  uint32_t ring_launches() const { return ring_ ? ring_->launches() : 0; }
  int ring_mode() const { return ring_ ? ring_->mode() : -1; }
  int ring_hold(bool on) { return ring_ ? ring_->hold(on) : (errno = ENOSYS, -1); }
  bool attach() { return ensure_mapped(); }

  int set_mop(unsigned mode) override {
    switch (mode) {
      case 0: return hdr_bits(offsetof(splinter_header, core_flags), 2, (uint8_t)~(SPL_SYS_AUTO_SCRUB | SPL_SYS_HYBRID_SCRUB));
      case 1: return hdr_bits(offsetof(splinter_header, core_flags), 1, SPL_SYS_AUTO_SCRUB | SPL_SYS_HYBRID_SCRUB);
      case 2: return hdr_bits(offsetof(splinter_header, core_flags), 1, SPL_SYS_AUTO_SCRUB);
      default: errno = EOPNOTSUPP; return -1;
    }
  }
  int get_mop() override {
    uint8_t f = config_get();
    if (f & SPL_SYS_HYBRID_SCRUB) return 1;
    if (f & SPL_SYS_AUTO_SCRUB) return 2;
    return 0;
  }
  void purge() override {
    if (!ensure_mapped()) return;
    DevGuard dg(device_);
    std::lock_guard<std::mutex> lk(mu_);
    spl_arena_purge(arena(), stream_);
    (void)hipStreamSynchronize(stream_);
  }
  int header_snapshot(splinter_header_snapshot_t* o) override {
    if (!o) return -2;
    splinter_header h;
    if (get_field(0, &h, 64) != 0) return -1;
    o->magic = h.magic; o->version = h.version; o->slots = h.slots; o->max_val_sz = h.max_val_sz;
    o->epoch = h.epoch; o->core_flags = h.core_flags; o->user_flags = h.user_flags;
    o->parse_failures = h.parse_failures; o->last_failure_epoch = h.last_failure_epoch;
    return 0;
  }
  uint8_t config_get() override {
    uint8_t f = 0;
    get_field(offsetof(splinter_header, core_flags), &f, 1);
    return f;
  }
  void config_or(uint8_t m) override { hdr_bits(offsetof(splinter_header, core_flags), 1, m); }
  void config_and(uint8_t m) override { hdr_bits(offsetof(splinter_header, core_flags), 2, m); }

  // ------------------------------------------------ per-call ops (command ring) --
  int set(const char* key, const void* val, size_t len) override {
    if (!key) return -2;
    if (len == 0 || len > geo_.max_val) { errno = len ? EMSGSIZE : EINVAL; return -1; }
    if (!val) return -2;
    RingResult r;
    if (ring(kRingSet, 0, key, val, (uint32_t)len, 0, nullptr, 0, &r) != 0) return -1;
    if (r.status == 0) notify_host();
    return st_ret(r.status);
  }
  int unset(const char* key) override {
    if (!key) return -2;
    RingResult r;
    if (ring(kRingUnset, 0, key, nullptr, 0, 0, nullptr, 0, &r) != 0) return -1;
    if (r.status >= 0) {
      notify_host();
      return r.status;
    }
    errno = neg_to_errno(r.status);
    return -1;
  }
  int get(const char* key, void* buf, size_t buf_sz, size_t* out_sz) override {
    if (!key) return -2;
    thread_local std::vector<uint8_t> tmp;
    RingResult r;
    const bool direct = buf && buf_sz >= geo_.max_val;  // the whole value fits: copy straight out
    if (!direct) tmp.resize(geo_.max_val + 16);
    const uint32_t cap = direct ? (uint32_t)std::min<size_t>(buf_sz, geo_.max_val) : (uint32_t)tmp.size();
    if (ring(kRingGet, 0, key, nullptr, 0, 0, direct ? buf : tmp.data(), cap, &r) != 0) return -1;
    if (r.status != 0) { errno = neg_to_errno(r.status); return -1; }
    if (out_sz) *out_sz = r.out_len;
    if (buf && !direct) {
      if (buf_sz < r.out_len) { errno = EMSGSIZE; return -1; }
      std::memcpy(buf, tmp.data(), r.out_len);
    }
    return 0;
  }
  int list(char** out, size_t max, size_t* cnt) override {
    if (!out || !cnt) return -2;
    std::vector<uint32_t> idx;
    std::vector<uint64_t> ep;
    scan(SPL_SCAN_LIST, 0, idx, ep, max);
    fetch_cores(idx);
    size_t c = 0;
    for (size_t i = 0; i < idx.size() && c < max; ++i) out[c++] = (char*)(list_cache_.data() + i * 128 + kOffKey);
    *cnt = c;
    return 0;
  }
  int poll(const char* key, uint64_t timeout_ms) override {
    uint64_t start = epoch_of(key);
    if (start == 0) return -1;
    if (start & 1) { errno = EAGAIN; return -1; }
    timespec t0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (;;) {
      uint64_t cur = epoch_of(key);
      if (!(cur & 1) && cur != start) return 0;
      timespec t;
      clock_gettime(CLOCK_MONOTONIC, &t);
      uint64_t el = (uint64_t)(t.tv_sec - t0.tv_sec) * 1000 + (uint64_t)((t.tv_nsec - t0.tv_nsec) / 1000000);
      if (el >= timeout_ms) { errno = ETIMEDOUT; return -1; }
      usleep(1000);
    }
  }
  int slot_snapshot(const char* key, splinter_slot_snapshot_t* o) override {
    if (!key || !o) return -2;
    uint8_t c[128];
    RingResult r;
    if (ring(kRingSnapshot, 0, key, nullptr, 0, 0, c, sizeof c, &r) != 0) return -1;
    if (r.status != 0) { errno = neg_to_errno(r.status); return -1; }
    std::memcpy(&o->hash, c + kOffHash, 8);
    std::memcpy(&o->epoch, c + kOffEpoch, 8);
    std::memcpy(&o->val_off, c + kOffValOff, 4);
    std::memcpy(&o->val_len, c + kOffValLen, 4);
    o->type_flag = c[kOffType];
    o->user_flag = c[kOffUser];
    std::memcpy(&o->ctime, c + kOffCtime, 8);
    std::memcpy(&o->atime, c + kOffAtime, 8);
    std::memcpy(&o->bloom, c + kOffBloom, 8);
    std::memcpy(o->key, c + kOffKey, kKeyMax);
#ifdef SPLINTER_EMBEDDINGS
    if (geo_.embeddings()) get_embedding(key, o->embedding);
    else std::memset(o->embedding, 0, kEmbedBytes);
#endif
    return 0;
  }
  int append(const char* key, const void* data, size_t len, size_t* new_len) override {
    // atomic on the device: the slot is held (odd epoch) across the tail copy (append_op)
    if (!key || !data || len == 0) return -2;
    if (len > geo_.max_val) { errno = EMSGSIZE; return -1; }
    RingResult r;
    if (ring(kRingAppend, 0, key, data, (uint32_t)len, 0, nullptr, 0, &r) != 0) return -1;
    if (r.status != 0) { errno = neg_to_errno(r.status); return -1; }
    if (new_len) *new_len = (size_t)r.result;
    notify_host();
    return 0;
  }
  const void* raw_ptr(const char* key, size_t* out_sz, uint64_t* out_epoch) override {
    // Zero-copy, as the reference (splinter.c:747-762): a host pointer into the value region
    // through the CPU mapping of the arena's dmabuf chunks (VmmArena::host_map, PCIe BAR), with the
    // slot's epoch and length from one ring snapshot; the caller re-checks the epoch.
    if (uint8_t* hb = ensure_mapped() ? host_base() : nullptr) {
      uint8_t c[128];
      RingResult r;
      if (ring(kRingSnapshot, 0, key, nullptr, 0, 0, c, sizeof c, &r) != 0) return nullptr;
      if (r.status != 0) { errno = neg_to_errno(r.status); return nullptr; }
      uint64_t e;
      uint32_t len;
      std::memcpy(&e, c + kOffEpoch, 8);
      std::memcpy(&len, c + kOffValLen, 4);
      if (out_sz) *out_sz = len;
      if (out_epoch) *out_epoch = e;
      return hb + kHeaderBytes + geo_.slots_bytes() + r.result * (size_t)geo_.max_val;
    }
    // no host mapping (hipMalloc / IPC arena, or the driver refused the mmap): a seqlock-consistent
    // host snapshot (thread-local, valid until this thread's next raw_ptr call) with the epoch it
    // was read at (docs/DIVERGENCES.md)
    thread_local std::vector<uint8_t> snap;
    snap.resize(geo_.max_val + 1);
    for (int t = 0; t < 64; ++t) {
      const uint64_t e = epoch_of(key);
      if (e == 0) return nullptr;
      size_t n = 0;
      if (e & 1) { usleep(10); continue; }
      if (get(key, snap.data(), geo_.max_val, &n) != 0) {
        if (errno == EAGAIN) continue;
        return nullptr;
      }
      if (epoch_of(key) != e) continue;
      snap[n] = 0;
      if (out_sz) *out_sz = n;
      if (out_epoch) *out_epoch = e;
      return snap.data();
    }
    errno = EAGAIN;
    return nullptr;
  }
  uint64_t epoch_of(const char* key) override {
    uint64_t out = 0;
    int32_t st = meta(key, SPL_META_GET_EPOCH, 0, &out);
    return st == 0 ? out : 0;
  }
  int set_as_system(const char* key) override { return meta_ret(meta(key, SPL_META_SET_SYSTEM, 0, nullptr)); }

  int set_embedding(const char* key, const float* vec) override {
    if (!key || !vec) return -2;
    if (!geo_.embeddings()) { errno = ENOTSUP; return -1; }
    RingResult r;
    if (ring(kRingEmbedSet, 0, key, vec, (uint32_t)kEmbedBytes, 0, nullptr, 0, &r) != 0) return -1;
    if (r.status == 0) notify_host();
    return st_ret(r.status);
  }
  int get_embedding(const char* key, float* out) override {
    if (!key || !out) return -2;
    if (!geo_.embeddings()) { errno = ENOTSUP; return -1; }
    RingResult r;
    if (ring(kRingEmbedGet, 0, key, nullptr, 0, 0, out, (uint32_t)kEmbedBytes, &r) != 0) return -1;
    return st_ret(r.status);
  }

  int set_named_type(const char* key, uint16_t mask) override {
    // BIGUINT promotion (ASCII digits -> u64) runs on the device under the slot seqlock
    return meta_ret(meta(key, SPL_META_SET_TYPE, mask, nullptr));
  }
  int set_slot_time(const char* key, unsigned short mode, uint64_t epoch, size_t offset) override {
    if (mode != SPL_TIME_CTIME && mode != SPL_TIME_ATIME) { errno = ENOTSUP; return -2; }
    return meta_ret(meta(key, mode == SPL_TIME_CTIME ? SPL_META_SET_CTIME : SPL_META_SET_ATIME, epoch - offset, nullptr));
  }
  int integer_op(const char* key, splinter_integer_op_t op, const void* mask) override {
    if (!key) return -2;
    uint64_t m = 0;
    if (mask) std::memcpy(&m, mask, 8);
    RingResult r;
    if (ring(kRingIntop, (uint32_t)op, key, nullptr, 0, m, nullptr, 0, &r) != 0) return -1;
    if (r.status == 0) notify_host();
    return st_ret(r.status);
  }

  int bump(const char* key) override { return meta_ret(meta(key, SPL_META_BUMP, 0, nullptr)); }
  int retrain(const char* key) override { return meta_ret(meta(key, SPL_META_RETRAIN, 0, nullptr)); }
  int set_label(const char* key, uint64_t m) override { return meta_ret(meta(key, SPL_META_SET_LABEL, m, nullptr)); }
  int unset_label(const char* key, uint64_t m) override { return meta_ret(meta(key, SPL_META_UNSET_LABEL, m, nullptr)); }

  int watch_register(const char* key, uint8_t g) override {
    if (g >= SPLINTER_MAX_GROUPS) { errno = EINVAL; return -2; }
    return meta_ret(meta(key, SPL_META_WATCH_REG, g, nullptr));
  }
  int watch_unregister(const char* key, uint8_t g) override {
    if (g >= SPLINTER_MAX_GROUPS) return -2;
    return meta_ret(meta(key, SPL_META_WATCH_UNREG, g, nullptr));
  }
  int watch_label_register(uint64_t mask, uint8_t g) override {
    if (g >= SPLINTER_MAX_GROUPS) return -2;
    uint8_t w[64];
    if (get_field(offsetof(splinter_header, bloom_watches), w, 64) != 0) return -1;
    for (uint64_t m = mask; m; m &= m - 1) w[__builtin_ctzll(m)] = g;
    return put_field(offsetof(splinter_header, bloom_watches), w, 64);
  }
  int pulse_keygroup(const char* key) override { return meta_ret(meta(key, SPL_META_PULSE, 0, nullptr)); }
  void pulse_slot(splinter_slot*) override {}  // slots are not host mapped
  uint64_t signal_count(uint8_t g) override {
    if (g >= SPLINTER_MAX_GROUPS) return 0;
    uint64_t v = 0;
    get_field(offsetof(splinter_header, signal_groups) + 64 * (size_t)g, &v, 8);
    return v;
  }
  int signal_add(uint8_t g, uint64_t delta) override {
    if (g >= SPLINTER_MAX_GROUPS) return -2;
    return put_field(offsetof(splinter_header, signal_groups) + 64 * (size_t)g, &delta, 8, 3);
  }
  void enumerate(uint64_t mask, void (*cb)(const char*, uint64_t, void*), void* ud) override {
    if (!cb) return;
    std::vector<uint32_t> idx;
    std::vector<uint64_t> ep;
    scan(SPL_SCAN_LABELS, mask, idx, ep, SIZE_MAX);
    fetch_cores(idx);
    for (size_t i = 0; i < idx.size(); ++i) cb((const char*)(list_cache_.data() + i * 128 + kOffKey), ep[i], ud);
  }

  // ------------------------------------------------------------- event bus --
  // The owner's eventfd is written by a host proxy thread whenever the notify word of the
  // shared descriptor is set: by this process's per-call mutations, by the batch kernels of ANY
  // process attached to the arena (system-scope store from the kernel epilogue, arena_dev.hpp
  // notify_host), and by per-call mutations of other processes.  Device kernels also maintain
  // the dirty mask once the device header records an owner (mirrored here).
  int event_bus_init() override { return event_bus_install(eventfd(0, EFD_CLOEXEC)); }
  int event_bus_adopt(int fd) override { return event_bus_install(fcntl(fd, F_DUPFD_CLOEXEC, 0)); }
  int event_bus_install(int fd) {
    if (fd < 0) return -1;
    stop_proxy();
    if (event_fd_ >= 0) close(event_fd_);
    event_fd_ = fd;
    __atomic_store_n(&desc_->control.event_bus.owner_fd, fd, __ATOMIC_RELEASE);
    __atomic_store_n(&desc_->control.event_bus.owner_pid, (int32_t)getpid(), __ATOMIC_RELEASE);
    const int32_t own[2] = {fd, (int32_t)getpid()};
    put_field(offsetof(splinter_header, event_bus) + offsetof(splinter_event_bus, owner_fd), own, 8);
    proxy_stop_.store(false);
    proxy_ = std::thread([this] { proxy_loop(); });
    return 0;
  }
  int event_bus_open() override {
    const int32_t fd = __atomic_load_n(&desc_->control.event_bus.owner_fd, __ATOMIC_ACQUIRE);
    const int32_t pid = __atomic_load_n(&desc_->control.event_bus.owner_pid, __ATOMIC_ACQUIRE);
    if (fd < 0 || pid <= 0) { errno = ENODEV; return -1; }
    if ((pid_t)pid == getpid()) return dup(fd);
#if defined(SYS_pidfd_open) && defined(SYS_pidfd_getfd)
    int pfd = (int)syscall(SYS_pidfd_open, (pid_t)pid, 0);
    if (pfd < 0) return -1;
    int r = (int)syscall(SYS_pidfd_getfd, pfd, fd, 0);
    close(pfd);
    return r;
#else
    errno = ENOSYS;
    return -1;
#endif
  }
  void event_bus_dirty(uint64_t* out, size_t words) override {
    if (!out) return;
    const size_t n = words < SPLINTER_EVENT_BUS_MASK_WORDS ? words : SPLINTER_EVENT_BUS_MASK_WORDS;
    get_field(offsetof(splinter_header, event_bus), out, n * 8);
  }

  int shard_claim_ex(uint32_t id, uint32_t pid, uint8_t it, uint8_t pr, uint64_t dur, uint64_t at) override {
    return shard_claim_on(&desc_->control, id, pid, it, pr, dur, at);
  }
  int shard_rebid(uint32_t id, uint8_t it, uint8_t pr, uint64_t dur) override {
    return shard_rebid_on(&desc_->control, id, it, pr, dur);
  }
  int shard_release(uint32_t id) override { return shard_release_on(&desc_->control, id); }
  uint32_t shard_election(uint8_t* out_intent) override { return shard_election_on(&desc_->control, out_intent); }
  int shard_table(splinter_shard_bid_snapshot* out, size_t max) override { return shard_table_on(&desc_->control, out, max); }
  int madvise(uint32_t id, void* addr, size_t len, int advice, uint64_t timeout) override {
    // Election as on the host backend; the advice maps to a residency hint on
    // the HBM range (coarse-grained hipMalloc memory: a documented no-op).
    (void)addr; (void)len; (void)advice;
    if (id == 0 || !shard_present_on(&desc_->control, id)) { errno = EINVAL; return -2; }
    const uint64_t deadline = now_ticks() + timeout;
    for (;;) {
      if (shard_election_on(&desc_->control, nullptr) == id) return 0;
      if (timeout == 0) { errno = EAGAIN; return -1; }
      if (timeout != UINT64_MAX && now_ticks() >= deadline) { errno = ETIMEDOUT; return -1; }
      usleep(5000);
    }
  }

  // ---------------------------------------------------- bulk / helpers --
  int checkpoint(const char* path);
  long search_all(const float* q, uint64_t mask, float min_sim, float max_dist, long cap, spl_search_hit* out);
  long search_batch(const float* q, int nq, int k, float min_sim, float max_dist, uint64_t mask, spl_search_hit* out,
                   int sample_div = 1, SearchSync* sync = nullptr);
  int device() const { return device_; }
  struct SearchScratch;
  SearchScratch* ss_ = nullptr;
  int restore_from(const char* path);
  int probe_stats(ProbeStats* out);
  int rehash(uint64_t out[4], unsigned flags = 0);
  int maint_seq(uint64_t* seq);

  // ------------------------------------------------------ host-array batches --
  long set_batch(const char* keys, int kstride, const uint8_t* vals, int vstride, const uint32_t* lens, long n,
                 int32_t* status, int retries) override;
  long get_batch(const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens, long n,
                 int32_t* status, int retries) override;
  long intop_batch(const char* keys, int kstride, const int* ops, const uint64_t* masks, long n, int32_t* status,
                   uint64_t* results) override;
  long set_embedding_batch(const char* keys, int kstride, const float* vecs, long n, int32_t* status) override;

 private:
  HbmStore() = default;
  // Batch staging (batch_run): two chunk slots, each its own stream, device buffer and pinned
  // host buffer, so chunk c+1's host-to-device copy overlaps chunk c's kernel and copy-back.
  struct Stage {
    hipStream_t s = nullptr;
    uint8_t* d = nullptr;
    size_t dbytes = 0;
    uint8_t* h = nullptr;
    size_t hbytes = 0;
    std::vector<std::pair<std::pair<uint8_t*, const uint8_t*>, size_t>> out;  // pageable copy-outs after sync
  };
  Stage stg_[2];
  std::mutex batch_mu_;
  // One array of a batch: caller pointer, caller row stride, device row stride, input / output.
  struct Col {
    const void* user;
    long ustride;  // caller bytes per op
    long dstride;  // device bytes per op (16-B rows for key / value records)
    bool in, out;
    bool pinned;
  };
  template <class K>
  long batch_run(long n, Col* cols, int ncols, K&& kernel);
  int setup_buffers();
  int ring(uint32_t op, uint32_t sub, const char* key, const void* in, uint32_t in_len, uint64_t arg, void* out,
           uint32_t out_cap, RingResult* r) {
    char k[64];
    uint32_t klen = 0;
    uint64_t khash = 0;
    if (key) {
      KeyRef kr(key);
      std::memcpy(k, kr.buf, 64);
      klen = (uint32_t)kr.len;
      khash = kr.hash;
    } else {
      std::memset(k, 0, 64);
    }
    if (!ring_ || !ring_->ready()) { errno = ENOSYS; return -1; }
    // a client of the owner's ring server needs no device mapping of the arena; its own worker does
    if (ring_->needs_arena() && !ensure_mapped()) return -1;
    const int rc = ring_->call(arena(), op, sub, k, klen, khash, in, in_len, arg, out, out_cap, r);
    // the owner went away between the check above and the call: the call falls over to a private
    // worker, which needs this process's own mapping of the arena -- map it and call once more
    if (rc != 0 && errno == EAGAIN && ring_->needs_arena()) {
      if (!ensure_mapped()) return -1;
      return ring_->call(arena(), op, sub, k, klen, khash, in, in_len, arg, out, out_cap, r);
    }
    return rc;
  }
  static int st_ret(int32_t st) {
    if (st == 0) return 0;
    errno = neg_to_errno(st);
    return -1;
  }
  static int meta_ret(int32_t st) { return st_ret(st); }
  int32_t meta(const char* key, int op, uint64_t arg, uint64_t* out) {
    if (!key) return -22;
    RingResult r;
    if (ring(kRingMeta, (uint32_t)op, key, nullptr, 0, arg, nullptr, 0, &r) != 0) return -5;
    if (out) *out = r.result;
    const bool mut = op == SPL_META_SET_LABEL || op == SPL_META_UNSET_LABEL || op == SPL_META_RETRAIN ||
                     op == SPL_META_SET_TYPE;
    if (r.status == 0 && mut) notify_host();
    return r.status;
  }
  // header bytes through the ring: READ / WRITE (sub 0 store, 1 atomic OR, 2 atomic AND)
  int get_field(size_t off, void* dst, size_t n) {
    RingResult r;
    if (ring(kRingRead, 0, nullptr, nullptr, (uint32_t)n, off, dst, (uint32_t)n, &r) != 0) return -1;
    return r.status == 0 ? 0 : -1;
  }
  int put_field(size_t off, const void* src, size_t n, uint32_t how = 0) {
    RingResult r;
    if (ring(kRingWrite, how, nullptr, src, (uint32_t)n, off, nullptr, 0, &r) != 0) return -1;
    return r.status == 0 ? 0 : -1;
  }
  int hdr_bits(size_t off, uint32_t how, uint8_t m) { return put_field(off, &m, 1, how); }

  // Slot-range scans into persistent, grow-only scratch (kScanChunk slots per launch), results
  // appended on the host; stops once `limit` matches are collected.
  static constexpr uint32_t kScanChunk = 1u << 22;
  void scan(int mode, uint64_t mask, std::vector<uint32_t>& idx, std::vector<uint64_t>& ep, size_t limit) {
    idx.clear();
    ep.clear();
    if (!ensure_mapped()) return;
    DevGuard dg(device_);
    std::lock_guard<std::mutex> lk(mu_);
    if (ensure_scan_scratch() != 0) return;
    std::vector<uint32_t> hi;
    std::vector<uint64_t> he;
    for (uint64_t b = 0; b < geo_.slots && idx.size() < limit; b += kScanChunk) {
      const uint32_t e = (uint32_t)std::min<uint64_t>(geo_.slots, b + kScanChunk);
      (void)hipMemsetAsync(d_scan_cnt_, 0, 4, stream_);
      spl_arena_scan_range(arena(), mode, mask, (uint32_t)b, e, d_scan_idx_, d_scan_ep_, kScanChunk, d_scan_cnt_,
                           stream_);
      uint32_t n = 0;
      (void)hipMemcpyAsync(h_u32_, d_scan_cnt_, 4, hipMemcpyDeviceToHost, stream_);
      (void)hipStreamSynchronize(stream_);
      std::memcpy(&n, h_u32_, 4);
      if (n > kScanChunk) n = kScanChunk;
      if (!n) continue;
      hi.resize(n);
      he.resize(n);
      (void)hipMemcpyAsync(hi.data(), d_scan_idx_, (size_t)n * 4, hipMemcpyDeviceToHost, stream_);
      (void)hipMemcpyAsync(he.data(), d_scan_ep_, (size_t)n * 8, hipMemcpyDeviceToHost, stream_);
      (void)hipStreamSynchronize(stream_);
      // the scan compacts in arrival order: restore slot order inside the chunk
      std::vector<uint32_t> ord(n);
      for (uint32_t i = 0; i < n; ++i) ord[i] = i;
      std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return hi[x] < hi[y]; });
      for (uint32_t i = 0; i < n && idx.size() < limit; ++i) {
        idx.push_back(hi[ord[i]]);
        ep.push_back(he[ord[i]]);
      }
    }
  }
  int ensure_scan_scratch() {
    if (d_scan_idx_) return 0;
    if (hipMalloc((void**)&d_scan_idx_, (size_t)kScanChunk * 4) != hipSuccess) return -1;
    if (hipMalloc((void**)&d_scan_ep_, (size_t)kScanChunk * 8) != hipSuccess) return -1;
    if (hipMalloc((void**)&d_scan_cnt_, 64) != hipSuccess) return -1;
    return 0;
  }
  void fetch_cores(const std::vector<uint32_t>& idx) {
    list_cache_.assign(idx.size() * 128, 0);
    if (!ensure_mapped()) return;
    DevGuard dg(device_);
    std::lock_guard<std::mutex> lk(mu_);
    if (idx.empty() || ensure_scan_scratch() != 0) return;
    // reuse the scan scratch: kScanChunk indices (4 B) + kScanChunk/16 cores (128 B) per round
    const size_t per = kScanChunk / 16;
    uint8_t* d_out = (uint8_t*)d_scan_ep_;
    for (size_t b = 0; b < idx.size(); b += per) {
      const size_t n = std::min(per, idx.size() - b);
      (void)hipMemcpyAsync(d_scan_idx_, idx.data() + b, n * 4, hipMemcpyHostToDevice, stream_);
      spl_arena_gather_slots(arena(), d_scan_idx_, (long)n, d_out, stream_);
      (void)hipMemcpyAsync(list_cache_.data() + b * 128, d_out, n * 128, hipMemcpyDeviceToHost, stream_);
      (void)hipStreamSynchronize(stream_);
    }
  }
  // Per-call mutation -> event bus: write the eventfd directly when this process owns it, else
  // raise the shared notify word for the owner's proxy.
  void notify_host() {
    if (event_fd_ >= 0) {
      uint64_t one = 1;
      ssize_t w = write(event_fd_, &one, 8);
      (void)w;
    } else if (__atomic_load_n(&desc_->control.event_bus.owner_pid, __ATOMIC_ACQUIRE) > 0) {
      __atomic_store_n(&desc_->notify, 1u, __ATOMIC_RELEASE);
    }
  }
  void proxy_loop() {
    const int us = getenv("SPLINTER_BUS_POLL_US") ? atoi(getenv("SPLINTER_BUS_POLL_US")) : 100;
    while (!proxy_stop_.load(std::memory_order_acquire)) {
      if (__atomic_load_n(&desc_->notify, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(&desc_->notify, 0u, __ATOMIC_RELEASE);
        uint64_t one = 1;
        ssize_t w = write(event_fd_, &one, 8);
        (void)w;
        continue;
      }
      usleep(us > 0 ? us : 100);
    }
  }
  void stop_proxy() {
    if (proxy_.joinable()) {
      proxy_stop_.store(true, std::memory_order_release);
      proxy_.join();
    }
  }

  std::string name_;
  Geometry geo_;
  int device_ = 0;
  bool owner_ = false;
  void* raw_ = nullptr;    // hipMalloc / IPC base, or the VMM range
  VmmArena vmm_;           // mode 1 (vmm_share.hpp)
  // host view of the arena base (dbase_) through the dmabuf mapping, nullptr without one
  uint8_t* host_base() {
    if (!vmm_mode_ || getenv_flag_off("SPLINTER_HBM_HOST_MAP")) return nullptr;
    uint8_t* h = (uint8_t*)vmm_.host_map();
    return h ? h + ((uint8_t*)dbase_ - (uint8_t*)raw_) : nullptr;
  }
  static bool getenv_flag_off(const char* n) {
    const char* e = getenv(n);
    return e && !strcmp(e, "0");
  }
  bool vmm_mode_ = false;
  uint32_t side_flags_ = 0;  // SPL_ARENA_SIDE / SPL_ARENA_VEC16 of the allocation (descriptor)
  void* dbase_ = nullptr;  // raw_ + kAlignOffset (null until mapped: an opener attaches lazily)
  // Lazy attach: an opener whose per-call ops go to the owner's ring server maps the arena into its
  // own GPU address space only on the first op that needs it (batches, scans, search, raw pointers,
  // checkpoints, a private ring).  A CLI call on a 100M-key node store then maps nothing.
  std::vector<int> pend_fds_;
  size_t pend_chunk_ = 0;
  uint64_t pend_off_ = 0;
  std::mutex map_mu_;
  bool ensure_mapped() {
    if (__atomic_load_n(&dbase_, __ATOMIC_ACQUIRE)) return true;
    std::lock_guard<std::mutex> lk(map_mu_);
    if (dbase_) return true;
    if (pend_fds_.empty()) { errno = EIO; return false; }
    RingQuiesce quiet;  // VMM map calls may wait for the device: no resident worker of this process
    DevGuard dg(device_);
    std::vector<int> fds;
    fds.swap(pend_fds_);
    if (vmm_.import(device_, fds, pend_chunk_) != 0) { errno = EACCES; return false; }
    vmm_mode_ = true;
    raw_ = vmm_.base();
    __atomic_store_n(&dbase_, (void*)((uint8_t*)raw_ + pend_off_), __ATOMIC_RELEASE);
    return true;
  }
  HbmDescriptor* desc_ = nullptr;
  bool desc_registered_ = false;
  uint32_t* d_notify_ = nullptr;  // device address of desc_->notify (hipHostRegister)
  hipStream_t stream_ = nullptr;
  std::mutex mu_;
  int event_fd_ = -1;
  std::thread proxy_;
  std::atomic<bool> proxy_stop_{false};
  size_t vstride_ = 0;
  std::unique_ptr<CmdRing> ring_;
  uint8_t* h_u32_ = nullptr;
  uint32_t* d_scan_idx_ = nullptr;
  uint64_t* d_scan_ep_ = nullptr;
  uint32_t* d_scan_cnt_ = nullptr;
  std::vector<uint8_t> list_cache_;

  friend StoreBase* hbm_factory_impl(const char*, size_t, size_t, unsigned, int, int*);
};

// One non-blocking control stream per device, shared by every store of the process (init, scans,
// purge, checkpoint): each stream the process touches can claim a hardware queue, and past ~5
// queues the GPU's queue scheduler time-slices them -- the encoder then ran 15 % slower in the
// mixed bench (profiles/r2_hw_queues.md).
static hipStream_t control_stream(int device) {
  static std::mutex mu;
  static hipStream_t s[64] = {};
  std::lock_guard<std::mutex> lk(mu);
  if (device < 0 || device >= 64) device = 0;
  if (!s[device]) (void)hipStreamCreateWithFlags(&s[device], hipStreamNonBlocking);
  return s[device];
}

// Search scratch of a store (grown, kept across calls: no allocation per call).
struct HbmStore::SearchScratch {
  float* q = nullptr;        // [256][768] fp32 queries
  void* res = nullptr;       // [256][32] CandRec
  void* scr = nullptr;       // exact kernel's lists
  uint16_t* qf = nullptr;    // [256][768] bf16 fragment operand
  float* thr = nullptr;      // [256]
  float* bmax = nullptr;     // [sample tiles][256] (also the overflow flags)
  size_t bmax_bytes = 0;
  uint32_t* cnt = nullptr;   // [256][grid]
  uint32_t* cand = nullptr;  // [256][grid][capb]
  void* cores = nullptr;     // [256][32][128] slot cores of the results
  hipEvent_t ev = nullptr;   // stream_ -> search stream ordering
  // pinned host staging (queries up, results / cores / overflow flags down): pageable copies go
  // through the runtime's staging buffer, which the shards of a node search would share
  uint8_t* hp = nullptr;
  float* hq() const { return (float*)hp; }
  void* hres() const { return hp + kHq; }
  uint8_t* hcores() const { return hp + kHq + kHres; }
  uint32_t* hover() const { return (uint32_t*)(hp + kHq + kHres + kHcores); }
  static constexpr size_t kHq = 256 * (size_t)kEmbedBytes, kHres = 256 * 32 * 16, kHcores = 256 * 32 * 128,
                          kHover = 256 * 4, kHbytes = kHq + kHres + kHcores + kHover;
};

int HbmStore::setup_buffers() {
  stream_ = control_stream(device_);
  if (!stream_) return -1;
  vstride_ = ((size_t)geo_.max_val + 15) & ~(size_t)15;
  if (vstride_ < 128) vstride_ = 128;
  HIPCHECK(hipHostMalloc((void**)&h_u32_, 64));
  if (getenv("SPLINTER_HBM_NO_RING")) return 0;  // diagnosis only: batch kernels, no per-call API
  // the shared descriptor page(s) become device-visible: kernels of every attached process
  // store the event-bus notify word there
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  const size_t span = (sizeof(HbmDescriptor) + pg - 1) / pg * pg;
  if (hipHostRegister(desc_, span, hipHostRegisterMapped) == hipSuccess) {
    desc_registered_ = true;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, &desc_->notify, 0) == hipSuccess) d_notify_ = (uint32_t*)dp;
  }
  // Per-call ring: the owner hosts the store's ring server, other processes submit to it
  // (cmd_ring.hpp RingSegHdr); SPLINTER_RING_SHARED=0, or no live server, gives a process its own
  // worker as before
  const uint32_t ps = (uint32_t)std::max<size_t>(vstride_, kEmbedBytes);
  const char* sh = getenv("SPLINTER_RING_SHARED");
  const bool shared = !(sh && !strcmp(sh, "0")) && vmm_mode_;
  const std::string seg = name_ + ".ring";
  ring_ = std::make_unique<CmdRing>();
  if (shared && owner_) {
    if (ring_->init_server(device_, ps, seg, "/dev/shm/" + name_ + ".hbm", arena()) == 0) return 0;
    ring_ = std::make_unique<CmdRing>();
  } else if (shared && ring_->init_client(seg, device_, ps) == 0) {
    return 0;
  }
  return ring_->init(device_, ps);
}

static HbmDescriptor* map_descriptor(const std::string& name, bool create, int* err) {
  const std::string dn = name + ".hbm";
  // created under SPLINTER_DEFAULT_UMASK like a host store (reference splinter.c:131-146): the
  // descriptor's mode is also what the owner's chunk-fd server admits peers by (vmm_share.hpp)
  mode_t prev = create ? env_umask_push() : (mode_t)-1;
  int fd = create ? shm_open(dn.c_str(), O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0666)
                  : shm_open(dn.c_str(), O_RDWR | O_CLOEXEC, 0666);
  if (create) env_umask_pop(prev);
  if (fd < 0) { *err = errno; return nullptr; }
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  const size_t span = (sizeof(HbmDescriptor) + pg - 1) / pg * pg;
  if (create && ftruncate(fd, (off_t)span) != 0) { *err = errno; close(fd); return nullptr; }
  void* p = mmap(nullptr, span, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) { *err = errno; return nullptr; }
  return (HbmDescriptor*)p;
}

HbmStore* HbmStore::create(const char* name, size_t slots, size_t max_val, bool emb, int* err) {
  *err = 0;
  if (slots == 0 || max_val == 0 || slots > UINT32_MAX || max_val > UINT32_MAX) { *err = ENOTSUP; return nullptr; }
  auto* s = new HbmStore();
  s->name_ = name;
  s->geo_.slots = (uint32_t)slots;
  s->geo_.max_val = (uint32_t)max_val;
  s->geo_.stride = emb ? (uint32_t)kSlotEmbedBytes : (uint32_t)kSlotCoreBytes;
  s->owner_ = true;
  (void)hipGetDevice(&s->device_);
  const size_t total = s->geo_.total_bytes();
  // the side region after the values (splinter_layout.hpp): probe statistics, and for an embedding
  // store the bf16 vector copy the batched search streams (SPLINTER_HBM_VEC16=0: none)
  const char* v16e = getenv("SPLINTER_HBM_VEC16");
  const bool vec16 = emb && !(v16e && !strcmp(v16e, "0"));
  const size_t side_off = side_offset(s->geo_.slots, s->geo_.stride, s->geo_.max_val);
  const size_t alloc = side_off + side_bytes(s->geo_.slots, vec16) + 256;
  s->side_flags_ = SPL_ARENA_SIDE | (vec16 ? SPL_ARENA_VEC16 : 0u);
  // VMM chunks (attachable by other processes at any size), else one hipMalloc allocation
  const char* ve = getenv("SPLINTER_HBM_VMM");
  const size_t chunk_mb = getenv("SPLINTER_HBM_CHUNK_MB") ? (size_t)atol(getenv("SPLINTER_HBM_CHUNK_MB")) : 1024;
  if (!(ve && !strcmp(ve, "0")) && s->vmm_.create(s->device_, alloc, (chunk_mb ? chunk_mb : 1024) << 20) == 0) {
    s->vmm_mode_ = true;
    s->raw_ = s->vmm_.base();
  } else if (hipMalloc(&s->raw_, alloc) != hipSuccess) {
    *err = ENOMEM;
    delete s;
    return nullptr;
  }
  s->dbase_ = (uint8_t*)s->raw_ + kAlignOffset;
  s->desc_ = map_descriptor(name, true, err);
  if (!s->desc_ || s->setup_buffers() != 0) { if (!*err) *err = EIO; delete s; return nullptr; }
  // header image built on the host, then the slot array initialised on device
  splinter_header h;
  std::memset(&h, 0, sizeof h);
  h.magic = kMagic;
  h.version = kVersion;
  h.slots = s->geo_.slots;
  h.max_val_sz = s->geo_.max_val;
  h.val_sz = (uint32_t)total;
  h.alignment = s->geo_.stride;
  h.epoch = 1;
  h.core_flags = SPL_SYS_AUTO_SCRUB | SPL_SYS_HYBRID_SCRUB;
  std::memset(h.bloom_watches, 0xFF, 64);
  h.event_bus.owner_fd = -1;
  (void)hipMemcpy(s->dbase_, &h, sizeof h, hipMemcpyHostToDevice);
  (void)hipMemsetAsync((uint8_t*)s->dbase_ + kHeaderBytes + s->geo_.slots_bytes(), 0, s->geo_.values_bytes(), s->stream_);
  if (s->geo_.embeddings())
    (void)hipMemsetAsync((uint8_t*)s->dbase_ + kHeaderBytes, 0, s->geo_.slots_bytes(), s->stream_);
  // side header and squared norms zeroed (no vector yet); the bf16 rows are only read where a norm is set
  (void)hipMemsetAsync((uint8_t*)s->dbase_ + side_off, 0,
                       vec16 ? side_vec16_offset(s->geo_.slots) : kSideHdrBytes, s->stream_);
  spl_arena_init_slots(s->arena(), s->stream_);
  (void)hipStreamSynchronize(s->stream_);
  HbmDescriptor* d = s->desc_;
  std::memcpy(&d->control, &h, sizeof h);
  d->slots = s->geo_.slots;
  d->max_val = s->geo_.max_val;
  d->stride = s->geo_.stride;
  d->device = (uint32_t)s->device_;
  d->total_bytes = total;
  d->base_offset = kAlignOffset;
  d->owner_pid = (int32_t)getpid();
  std::memset(&d->handle, 0, sizeof d->handle);
  d->mode = s->vmm_mode_ ? 1u : 0u;
  d->side_flags = s->side_flags_;
  if (s->vmm_mode_) {
    d->nchunks = (uint32_t)s->vmm_.chunks();
    d->chunk_bytes = s->vmm_.chunk();
    snprintf(d->sock, sizeof d->sock, "splinter-hbm-%d-%s", (int)getpid(), name);
    if (s->vmm_.serve(d->sock, "/dev/shm/" + std::string(name) + ".hbm") != 0)
      d->sock[0] = 0;  // not attachable; this process still works
  } else if (hipIpcGetMemHandle(&d->handle, s->raw_) != hipSuccess) {
    std::memset(&d->handle, 0, sizeof d->handle);
  }
  d->version = 3;
  __atomic_store_n(&d->magic, kDescMagic, __ATOMIC_RELEASE);
  return s;
}

HbmStore* HbmStore::open(const char* name, int* err) {
  *err = 0;
  HbmDescriptor* d = map_descriptor(name, false, err);
  if (!d) return nullptr;
  if (__atomic_load_n(&d->magic, __ATOMIC_ACQUIRE) != kDescMagic) {
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
    munmap(d, (sizeof(HbmDescriptor) + pg - 1) / pg * pg);
    *err = EINVAL;
    return nullptr;
  }
  auto* s = new HbmStore();
  s->name_ = name;
  s->desc_ = d;
  s->geo_.slots = d->slots;
  s->geo_.max_val = d->max_val;
  s->geo_.stride = d->stride;
  s->device_ = (int)d->device;
  s->side_flags_ = d->side_flags & (SPL_ARENA_SIDE | SPL_ARENA_VEC16);
  DevGuard dg(s->device_);
  if (d->version >= 3 && d->mode == 1) {
    std::vector<int> fds;
    size_t chunk = 0;
    if (!d->sock[0] || VmmArena::fetch(d->sock, &fds, &chunk) != 0 || fds.size() != d->nchunks) {
      for (int f : fds) close(f);
      *err = EACCES;
      delete s;
      return nullptr;
    }
    s->vmm_mode_ = true;
    s->pend_fds_ = std::move(fds);
    s->pend_chunk_ = chunk;
    s->pend_off_ = d->base_offset;
    if (s->setup_buffers() != 0) { *err = EIO; delete s; return nullptr; }
    // attach now unless the owner's ring server serves this process (SPLINTER_HBM_LAZY_ATTACH=0: always now)
    const char* lz = getenv("SPLINTER_HBM_LAZY_ATTACH");
    if ((s->ring_mode() != 2 || (lz && !strcmp(lz, "0"))) && !s->ensure_mapped()) {
      *err = EACCES;
      delete s;
      return nullptr;
    }
    return s;
  }
  if (hipIpcOpenMemHandle(&s->raw_, d->handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
    *err = EACCES;
    s->raw_ = nullptr;
    delete s;
    return nullptr;
  }
  s->dbase_ = (uint8_t*)s->raw_ + d->base_offset;
  if (s->setup_buffers() != 0) { *err = EIO; delete s; return nullptr; }
  return s;
}

HbmStore::~HbmStore() {
  // a ring server's supervisor takes the quiesce gate shared to relaunch the worker: stop it before
  // this teardown takes the gate exclusive (it would otherwise wait on the gate while ~CmdRing joins
  // it).  Clients that want a worker meanwhile keep polling until the segment closes, then fail over.
  if (ring_) ring_->stop_supervisor();
  RingQuiesce quiet;  // hipFree & co. may wait for the device: no resident worker of this process
  DevGuard dg(device_);
  for (auto& st : stg_) {
    if (st.s) {
      (void)hipStreamSynchronize(st.s);
      (void)hipStreamDestroy(st.s);
    }
    if (st.d) (void)hipFree(st.d);
    if (st.h) (void)hipHostFree(st.h);
  }
  stop_proxy();
  if (event_fd_ >= 0) {
    if (desc_ && __atomic_load_n(&desc_->control.event_bus.owner_pid, __ATOMIC_ACQUIRE) == (int32_t)getpid()) {
      __atomic_store_n(&desc_->control.event_bus.owner_fd, -1, __ATOMIC_RELEASE);
      __atomic_store_n(&desc_->control.event_bus.owner_pid, 0, __ATOMIC_RELEASE);
      // the device header's copy too, through the ring (still up: it goes below)
      const int32_t own[2] = {-1, 0};
      put_field(offsetof(splinter_header, event_bus) + offsetof(splinter_event_bus, owner_fd), own, 8);
    }
    close(event_fd_);
  }
  ring_.reset();  // the worker (and a ring server's supervisor) reads the arena: gone before it
  if (stream_) (void)hipStreamSynchronize(stream_);
  if (h_u32_) (void)hipHostFree(h_u32_);
  if (ss_) {
    for (void* p : {(void*)ss_->q, ss_->res, ss_->scr, (void*)ss_->qf, (void*)ss_->thr, (void*)ss_->bmax,
                    (void*)ss_->cnt, (void*)ss_->cand, ss_->cores})
      if (p) (void)hipFree(p);
    if (ss_->ev) (void)hipEventDestroy(ss_->ev);
    if (ss_->hp) (void)hipHostFree(ss_->hp);
    delete ss_;
    ss_ = nullptr;
  }
  if (d_scan_idx_) (void)hipFree(d_scan_idx_);
  if (d_scan_ep_) (void)hipFree(d_scan_ep_);
  if (d_scan_cnt_) (void)hipFree(d_scan_cnt_);
  for (int f : pend_fds_) close(f);
  if (raw_) {
    if (vmm_mode_) vmm_.release();
    else if (owner_) (void)hipFree(raw_);
    else (void)hipIpcCloseMemHandle(raw_);
  }
  if (desc_) {
    if (desc_registered_) (void)hipHostUnregister(desc_);
    if (owner_) __atomic_store_n(&desc_->magic, 0u, __ATOMIC_RELEASE);
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
    munmap(desc_, (sizeof(HbmDescriptor) + pg - 1) / pg * pg);
    if (owner_) shm_unlink((name_ + ".hbm").c_str());
  }
}

// CLI search (reference splinter_cli_cmd_search.c:339-416) on the device: one fused scoring pass
// over every slot (spl_arena_score_all), then the candidates ranked by similarity desc, distance
// asc on the host, and the slot metadata of the best `cap` gathered.  Returns the number of
// candidates (may exceed cap), -1 on error.
long HbmStore::search_all(const float* q, uint64_t mask, float min_sim, float max_dist, long cap,
                          spl_search_hit* out) {
  if (!geo_.embeddings()) { errno = ENOTSUP; return -1; }
  if (!ensure_mapped()) return -1;
  DevGuard dg(device_);
  std::vector<float> sd((size_t)geo_.slots * 2);
  {
    std::lock_guard<std::mutex> lk(mu_);
    float* d_q = nullptr;
    void* d_out = nullptr;
    if (hipMallocAsync((void**)&d_q, kEmbedBytes, stream_) != hipSuccess) return -1;
    if (hipMallocAsync(&d_out, (size_t)geo_.slots * 8, stream_) != hipSuccess) {
      (void)hipFreeAsync(d_q, stream_);
      return -1;
    }
    (void)hipMemcpyAsync(d_q, q, kEmbedBytes, hipMemcpyHostToDevice, stream_);
    int rc = spl_arena_score_all(arena(), d_q, min_sim, max_dist, mask, d_out, stream_);
    if (rc == 0) (void)hipMemcpyAsync(sd.data(), d_out, sd.size() * 4, hipMemcpyDeviceToHost, stream_);
    (void)hipFreeAsync(d_q, stream_);
    (void)hipFreeAsync(d_out, stream_);
    (void)hipStreamSynchronize(stream_);
    if (rc != 0) return -1;
  }
  struct C {
    float sim, dist;
    uint32_t idx;
  };
  std::vector<C> c;
  for (uint32_t i = 0; i < geo_.slots; ++i)
    if (!std::isnan(sd[2 * (size_t)i])) c.push_back(C{sd[2 * (size_t)i], sd[2 * (size_t)i + 1], i});
  const long total = (long)c.size();
  auto better = [](const C& a, const C& b) {
    if (a.sim != b.sim) return a.sim > b.sim;
    const float da = a.dist < 0 ? 0.f : a.dist, db = b.dist < 0 ? 0.f : b.dist;  // un-embedded: 0, 0
    if (da != db) return da < db;
    return a.idx < b.idx;
  };
  const size_t keep = (size_t)std::max<long>(0, std::min<long>(cap, total));
  if (keep < c.size()) std::partial_sort(c.begin(), c.begin() + keep, c.end(), better);
  else std::sort(c.begin(), c.end(), better);
  c.resize(keep);
  std::vector<uint32_t> idx(keep);
  for (size_t i = 0; i < keep; ++i) idx[i] = c[i].idx;
  fetch_cores(idx);
  for (size_t i = 0; i < keep; ++i) {
    const uint8_t* core = list_cache_.data() + i * 128;
    spl_search_hit& h = out[i];
    std::memset(&h, 0, sizeof h);
    std::memcpy(h.key, core + kOffKey, 64);
    h.key[63] = 0;
    h.emb = c[i].dist >= 0.f;
    h.sim = h.emb ? c[i].sim : 0.f;
    h.dist = h.emb ? c[i].dist : 0.f;
    std::memcpy(&h.epoch, core + kOffEpoch, 8);
    std::memcpy(&h.bloom, core + kOffBloom, 8);
    std::memcpy(&h.len, core + kOffValLen, 4);
    h.type = core[kOffType];
  }
  return total;
}

// Batched top-k search of many queries (the C form of ops/search.py VectorSearch.search_batch, on the
// MFMA passes of search_kernels.hip): per block of 256 queries a bf16 pass over a slot sample gives a
// per-query candidate threshold (k-th largest per-tile maximum - 2 delta), a bf16 pass over the
// whole arena (the side region's bf16 copy where the arena has one) emits the candidates above it,
// and an fp32 re-score with the exact kernel's arithmetic ranks them; a query whose candidate
// segment overflowed anywhere is redone with the exact kernel.  Results: out[q * k + j], ranked by
// similarity desc, distance asc (reference splinter_cli_cmd_search.c:374-416); unused entries have
// an empty key and emb = 0.  Returns nq, or -1.
namespace {
constexpr int kMmaQ = 256, kMmaTile = 256, kMmaGrid = 256, kCapb = 64, kExactQ = 16, kExactGrid = 512;
constexpr float kDelta = 0.0078125f + 1.52587890625e-05f + 4e-4f;  // 2^-7 + 2^-16 + 4e-4 (ops/search.py DELTA)
struct CandRec {
  float sim, dist;
  uint32_t idx, pad;
};
}  // namespace


// Searches of shards that share a device run on their own streams (slot > 0: node fan-out), so
// they overlap; slot 0 is the device's control stream (a lone store adds no hardware queue).
static hipStream_t search_stream(int device, int slot) {
  if (slot <= 0) return control_stream(device);
  static std::mutex mu;
  static hipStream_t s[64][4] = {};
  std::lock_guard<std::mutex> lk(mu);
  if (device < 0 || device >= 64) device = 0;
  slot = (slot - 1) & 3;
  if (!s[device][slot]) (void)hipStreamCreateWithFlags(&s[device][slot], hipStreamNonBlocking);
  return s[device][slot];
}
thread_local int g_search_slot = 0;

long HbmStore::search_batch(const float* q, int nq, int k, float min_sim, float max_dist, uint64_t mask,
                            spl_search_hit* out, int sample_div, SearchSync* sync) {
  if (!geo_.embeddings()) { errno = ENOTSUP; return -1; }
  if (nq <= 0 || k <= 0 || k > 32 || !q || !out) { errno = EINVAL; return -1; }
  if (!ensure_mapped()) return -1;
  DevGuard dg(device_);
  std::unique_lock<std::mutex> lk(mu_);
  const spl_arena_t a = arena();
  const long slots = geo_.slots;
  hipStream_t ss = search_stream(device_, g_search_slot);
  std::vector<CandRec> res((size_t)nq * k);
  std::vector<uint8_t> cores((size_t)nq * k * 128);
  const bool bounded = max_dist < 3.0e38f;
  const bool mma = nq >= 32 && slots >= kMmaTile;
  // the threshold sample: a node's shards split one store's sample between them
  const int div = sample_div > 1 ? sample_div : 1;
  long sample = std::min<long>(slots, std::max<long>((long)kMmaTile * 4096 / div, slots / 16));
  sample = std::max<long>(kMmaTile, sample / kMmaTile * kMmaTile);
  // scratch (kept across calls; the stream-ordered allocations happen once per store)
  if (!ss_) ss_ = new SearchScratch();
  SearchScratch& S = *ss_;
  const int lists = spl_search_lists(kExactGrid);
  bool ok = true;
  if (!S.q) {
    ok = hipMallocAsync((void**)&S.q, (size_t)kMmaQ * kEmbedBytes, ss) == hipSuccess &&
         hipMallocAsync(&S.res, (size_t)kMmaQ * 32 * sizeof(CandRec), ss) == hipSuccess &&
         hipMallocAsync(&S.scr, (size_t)lists * kExactQ * 32 * sizeof(CandRec), ss) == hipSuccess &&
         hipMallocAsync((void**)&S.qf, (size_t)kMmaQ * kEmbedDim * 2, ss) == hipSuccess &&
         hipMallocAsync((void**)&S.thr, (size_t)kMmaQ * 4, ss) == hipSuccess &&
         hipMallocAsync((void**)&S.cnt, (size_t)kMmaQ * kMmaGrid * 4, ss) == hipSuccess &&
         hipMallocAsync((void**)&S.cand, (size_t)kMmaQ * kMmaGrid * kCapb * 4, ss) == hipSuccess &&
         hipMallocAsync(&S.cores, (size_t)kMmaQ * 32 * 128, ss) == hipSuccess &&
         hipEventCreateWithFlags(&S.ev, hipEventDisableTiming) == hipSuccess &&
         hipHostMalloc((void**)&S.hp, SearchScratch::kHbytes) == hipSuccess;
    if (!ok) (void)hipGetLastError();
  }
  const size_t bmax_need = (size_t)std::max<long>(sample / kMmaTile, 1) * kMmaQ * 4;
  if (ok && S.bmax_bytes < bmax_need) {
    if (S.bmax) (void)hipFreeAsync(S.bmax, ss);
    S.bmax = nullptr;
    ok = hipMallocAsync((void**)&S.bmax, bmax_need, ss) == hipSuccess;
    S.bmax_bytes = ok ? bmax_need : 0;
  }
  // everything written to the arena through this store's stream is visible to the search stream
  ok = ok && hipEventRecord(S.ev, stream_) == hipSuccess && hipStreamWaitEvent(ss, S.ev, 0) == hipSuccess;
  static_assert(sizeof(CandRec) == 16, "pinned result staging assumes 16-B records");
  auto exact = [&](const float* hq, int n, CandRec* dst, uint8_t* cdst) -> bool {  // nq <= kExactQ per launch
    for (int b = 0; b < n; b += kExactQ) {
      const int m = std::min(kExactQ, n - b);
      std::memcpy(S.hq(), hq + (size_t)b * kEmbedDim, (size_t)m * kEmbedBytes);
      if (hipMemcpyAsync(S.q, S.hq(), (size_t)m * kEmbedBytes, hipMemcpyHostToDevice, ss) != hipSuccess ||
          spl_search(a, S.q, m, k, min_sim, max_dist, mask, kExactGrid, S.scr, S.res, ss) != 0 ||
          spl_search_cores(a, S.res, m * k, S.cores, ss) != 0 ||
          hipMemcpyAsync(S.hres(), S.res, (size_t)m * k * sizeof(CandRec), hipMemcpyDeviceToHost, ss) != hipSuccess ||
          hipMemcpyAsync(S.hcores(), S.cores, (size_t)m * k * 128, hipMemcpyDeviceToHost, ss) != hipSuccess ||
          hipStreamSynchronize(ss) != hipSuccess)
        return false;
      std::memcpy(dst + (size_t)b * k, S.hres(), (size_t)m * k * sizeof(CandRec));
      std::memcpy(cdst + (size_t)b * k * 128, S.hcores(), (size_t)m * k * 128);
    }
    return true;
  };
  std::vector<uint32_t> over;
  std::vector<float> thr_h, redo;
  // a distance bound with no effective similarity floor makes every live slot a candidate (every
  // query would overflow its segments and be redone alone): those batches go to the exact kernel
  // directly, kExactQ queries per arena scan
  const bool exact_only = !mma || (bounded && min_sim <= -1.f);
  for (int b = 0; ok && b < nq; b += kMmaQ) {  // (a shard that fails leaves the node's threshold merge)
    const int n = std::min(kMmaQ, nq - b);
    const float* hq = q + (size_t)b * kEmbedDim;
    const float floor_v = min_sim - kDelta;
    if (exact_only) {
      if (sync) {  // a shard on the exact kernel still takes part in the block's threshold merge
        thr_h.assign((size_t)n, floor_v);
        sync->merge(nullptr, n, k, 2 * kDelta, floor_v, thr_h.data());
      }
      ok = exact(hq, n, res.data() + (size_t)b * k, cores.data() + (size_t)b * k * 128);
      continue;
    }
    // queries up once (fp32); the bf16 fragment operand is built on the device (spl_search_qprep)
    std::memcpy(S.hq(), hq, (size_t)n * kEmbedBytes);
    ok = hipMemcpyAsync(S.q, S.hq(), (size_t)n * kEmbedBytes, hipMemcpyHostToDevice, ss) == hipSuccess &&
         spl_search_qprep(S.q, n, S.qf, ss) == 0;
    if (ok && !bounded) {
      // node search: the k largest sampled maxima per query come back (staged in S.cnt, which the
      // candidate pass clears afterwards) for the shards' union threshold
      float* topv_d = sync ? (float*)S.cnt : nullptr;
      ok = spl_search_mma_pass(a, S.qf, n, 0, sample, mask, 0, nullptr, S.bmax, nullptr, nullptr, 0, kMmaGrid, ss) ==
               0 &&
           spl_search_thr_topk(S.bmax, (int)(sample / kMmaTile), n, k, 2 * kDelta, floor_v, S.thr, topv_d, ss) == 0;
      if (sync) {
        float* tv = (float*)S.hres();  // pinned staging, free until the results come back
        const bool got = ok && hipMemcpyAsync(tv, topv_d, (size_t)n * k * 4, hipMemcpyDeviceToHost, ss) == hipSuccess &&
                         hipStreamSynchronize(ss) == hipSuccess;
        float* th = (float*)S.hover();
        sync->merge(got ? tv : nullptr, n, k, 2 * kDelta, floor_v, th);
        ok = got && hipMemcpyAsync(S.thr, th, (size_t)n * 4, hipMemcpyHostToDevice, ss) == hipSuccess;
      }
    } else {
      thr_h.assign((size_t)n, floor_v);
      if (sync) sync->merge(nullptr, n, k, 2 * kDelta, floor_v, thr_h.data());
      ok = ok && hipMemcpyAsync(S.thr, thr_h.data(), (size_t)n * 4, hipMemcpyHostToDevice, ss) == hipSuccess;
    }
    // (the overflow flags reuse S.bmax: the threshold is built by then)
    ok = ok && hipMemsetAsync(S.cnt, 0, (size_t)n * kMmaGrid * 4, ss) == hipSuccess &&
         spl_search_mma_pass(a, S.qf, n, 0, slots, mask, 1, S.thr, nullptr, S.cnt, S.cand, kCapb, kMmaGrid, ss) == 0 &&
         spl_search_rescore(a, S.q, n, k, min_sim, max_dist, mask, S.cnt, S.cand, kMmaGrid, kCapb, S.res, ss) == 0 &&
         spl_search_overflow(S.cnt, n, kMmaGrid, kCapb, (uint32_t*)S.bmax, ss) == 0 &&
         spl_search_cores(a, S.res, n * k, S.cores, ss) == 0;
    over.resize((size_t)n);
    ok = ok &&
         hipMemcpyAsync(S.hres(), S.res, (size_t)n * k * sizeof(CandRec), hipMemcpyDeviceToHost, ss) == hipSuccess &&
         hipMemcpyAsync(S.hcores(), S.cores, (size_t)n * k * 128, hipMemcpyDeviceToHost, ss) == hipSuccess &&
         hipMemcpyAsync(S.hover(), S.bmax, (size_t)n * 4, hipMemcpyDeviceToHost, ss) == hipSuccess &&
         hipStreamSynchronize(ss) == hipSuccess;
    if (ok) {
      std::memcpy(res.data() + (size_t)b * k, S.hres(), (size_t)n * k * sizeof(CandRec));
      std::memcpy(cores.data() + (size_t)b * k * 128, S.hcores(), (size_t)n * k * 128);
      std::memcpy(over.data(), S.hover(), (size_t)n * 4);
    }
    // overflowed queries: the exact kernel, kExactQ of them per launch
    std::vector<int> oi;
    for (int i = 0; ok && i < n; ++i)
      if (over[(size_t)i]) oi.push_back(i);
    if (ok && !oi.empty()) {
      redo.resize(oi.size() * kEmbedDim);
      for (size_t j = 0; j < oi.size(); ++j)
        std::memcpy(&redo[j * kEmbedDim], hq + (size_t)oi[j] * kEmbedDim, kEmbedBytes);
      std::vector<CandRec> rr(oi.size() * (size_t)k);
      std::vector<uint8_t> rc(oi.size() * (size_t)k * 128);
      ok = exact(redo.data(), (int)oi.size(), rr.data(), rc.data());
      for (size_t j = 0; ok && j < oi.size(); ++j) {
        std::memcpy(&res[(size_t)(b + oi[j]) * k], &rr[j * k], (size_t)k * sizeof(CandRec));
        std::memcpy(&cores[(size_t)(b + oi[j]) * k * 128], &rc[j * k * 128], (size_t)k * 128);
      }
    }
  }
  lk.unlock();
  if (!ok) { errno = EIO; return -1; }
  for (size_t i = 0; i < res.size(); ++i) {
    spl_search_hit& h = out[i];
    std::memset(&h, 0, sizeof h);
    if (res[i].idx == 0xffffffffu) {
      h.sim = -3.4e38f;
      continue;
    }
    const uint8_t* core = cores.data() + i * 128;
    std::memcpy(h.key, core + kOffKey, 64);
    h.key[63] = 0;
    h.emb = 1;
    h.sim = res[i].sim;
    h.dist = res[i].dist;
    std::memcpy(&h.epoch, core + kOffEpoch, 8);
    std::memcpy(&h.bloom, core + kOffBloom, 8);
    std::memcpy(&h.len, core + kOffValLen, 4);
    h.type = core[kOffType];
  }
  return nq;
}

// Checkpoint: stream the device image into a v4 store file (byte-identical
// layout, so the host backend — or the reference library — can open it).
int HbmStore::checkpoint(const char* path) {
  if (!ensure_mapped()) return -1;
  DevGuard dg(device_);
  int fd = ::open(path, O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
  if (fd < 0) return -1;
  const size_t total = geo_.total_bytes();
  const size_t chunk = 64ull << 20;
  uint8_t* pin = nullptr;
  if (hipHostMalloc((void**)&pin, chunk) != hipSuccess) { close(fd); return -1; }
  (void)hipStreamSynchronize(stream_);
  int rc = 0;
  for (size_t off = 0; off < total && rc == 0; off += chunk) {
    const size_t n = total - off < chunk ? total - off : chunk;
    if (hipMemcpy(pin, (uint8_t*)dbase_ + off, n, hipMemcpyDeviceToHost) != hipSuccess) { rc = -1; break; }
    if (off == 0) {  // the control plane (shard bids, event bus) is host-side
      auto* h = (splinter_header*)pin;
      std::memcpy(h->shard_bids, desc_->control.shard_bids, sizeof h->shard_bids);
      h->event_bus.owner_fd = -1;
      h->event_bus.owner_pid = 0;
    }
    if (pwrite(fd, pin, n, (off_t)off) != (ssize_t)n) rc = -1;
  }
  (void)hipHostFree(pin);
  if (rc == 0) rc = fsync(fd);
  close(fd);
  return rc;
}

int HbmStore::restore_from(const char* path) {
  if (!ensure_mapped()) return -1;
  DevGuard dg(device_);
  int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  struct stat sb;
  if (fstat(fd, &sb) != 0 || (size_t)sb.st_size != geo_.total_bytes()) { close(fd); errno = EINVAL; return -1; }
  const size_t total = geo_.total_bytes();
  const size_t chunk = 64ull << 20;
  uint8_t* pin = nullptr;
  if (hipHostMalloc((void**)&pin, chunk) != hipSuccess) { close(fd); return -1; }
  int rc = 0;
  for (size_t off = 0; off < total && rc == 0; off += chunk) {
    const size_t n = total - off < chunk ? total - off : chunk;
    if (pread(fd, pin, n, (off_t)off) != (ssize_t)n) { rc = -1; break; }
    if (off == 0) {
      auto* h = (splinter_header*)pin;
      if (h->magic != kMagic || h->version != kVersion || h->slots != geo_.slots || h->max_val_sz != geo_.max_val) {
        rc = -1;
        errno = EINVAL;
        break;
      }
      std::memcpy(desc_->control.shard_bids, h->shard_bids, sizeof h->shard_bids);
    }
    if (hipMemcpy((uint8_t*)dbase_ + off, pin, n, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
  }
  (void)hipHostFree(pin);
  close(fd);
  // the side region is not in the file: the bf16 vector copy is rebuilt from the restored vectors
  if (rc == 0 && (side_flags_ & SPL_ARENA_VEC16)) {
    std::lock_guard<std::mutex> lk(mu_);
    if (spl_arena_vec16_rebuild(arena(), stream_) != 0 || hipStreamSynchronize(stream_) != hipSuccess) rc = -1;
  }
  return rc;
}

// Probe-chain statistics (arena_maint.hip k_probe_stats) into *out (host).
int HbmStore::probe_stats(ProbeStats* out) {
  if (!ensure_mapped()) return -1;
  DevGuard dg(device_);
  std::lock_guard<std::mutex> lk(mu_);
  ProbeStats* d = nullptr;
  if (hipMallocAsync((void**)&d, sizeof(ProbeStats), stream_) != hipSuccess) return -1;
  (void)hipMemsetAsync(d, 0, sizeof(ProbeStats), stream_);
  int rc = spl_arena_probe_stats(arena(), d, stream_);
  if (rc == 0) (void)hipMemcpyAsync(out, d, sizeof(ProbeStats), hipMemcpyDeviceToHost, stream_);
  (void)hipFreeAsync(d, stream_);
  if (hipStreamSynchronize(stream_) != hipSuccess) rc = -1;
  if (rc == 0 && (side_flags_ & SPL_ARENA_SIDE)) {  // the maintenance counters live in the side header
    ProbeStats side;
    if (hipMemcpy(&side, (uint8_t*)dbase_ + side_offset(geo_.slots, geo_.stride, geo_.max_val), sizeof side,
                  hipMemcpyDeviceToHost) == hipSuccess) {
      out->rebuilds = side.rebuilds;
      out->reclaimed = side.reclaimed;
      out->moved = side.moved;
    }
  }
  return rc == 0 ? 0 : -1;
}

// Tombstone maintenance (arena_maint.hip).  Default: the ONLINE cluster compaction -- keys move
// under both slots' seqlocks while every process keeps running batch and per-call ops; the pass is
// bracketed by the side header's maintenance seq (odd while it runs: "absent" outcomes and
// inserts report EAGAIN meanwhile).  SPL_REHASH_FULL: the full rebuild (copy out, clear, re-insert)
// -- EXCLUSIVE, the caller guarantees that no op of any process runs on the arena; refused with
// EBUSY when this store's ring worker cannot be held, with ENOMEM (and the scratch size on stderr)
// when the scratch cannot be allocated.  out: {moved, reclaimed, clusters, clusters past the
// per-wave tombstone cap}.
// Online maintenance passes run on a low-priority stream of their own: background work, on a
// hardware queue apart from the normal-priority queues of the store's kernels and its clients, so a
// pass's kernels interleave with live traffic at kernel boundaries instead of waiting in one queue
// behind it (or it behind them).
static hipStream_t maint_stream(int device) {
  static std::mutex mu;
  static hipStream_t s[64] = {};
  std::lock_guard<std::mutex> lk(mu);
  if (device < 0 || device >= 64) device = 0;
  if (!s[device]) {
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (hipStreamCreateWithPriority(&s[device], hipStreamNonBlocking, least) != hipSuccess) s[device] = nullptr;
  }
  return s[device];
}

int HbmStore::rehash(uint64_t out[4], unsigned flags) {
  if (!ensure_mapped()) return -1;
  if (!(side_flags_ & SPL_ARENA_SIDE)) { errno = ENOTSUP; return -1; }
  DevGuard dg(device_);
  out[0] = out[1] = out[2] = out[3] = 0;
  ProbeStats ps;
  if (probe_stats(&ps) != 0) return -1;
  uint8_t* const side = (uint8_t*)dbase_ + side_offset(geo_.slots, geo_.stride, geo_.max_val);
  const spl_arena_t a = arena();
  // a pass left open by a process that died (seq odd, its pid gone) is closed first
  {
    MaintRec mr;
    if (hipMemcpy(&mr, side + kSideMaintOff, sizeof mr, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (mr.seq & 1) {
      const bool alive = mr.pid > 0 && (::kill((pid_t)mr.pid, 0) == 0 || errno == EPERM);
      if (alive) { errno = EBUSY; return -1; }
      std::lock_guard<std::mutex> lk(mu_);
      uint64_t* d = nullptr;
      if (hipMallocAsync((void**)&d, 8, stream_) != hipSuccess) return -1;
      const int rc = spl_arena_maint_mark(a, 0, 0, 0, d, stream_);
      (void)hipFreeAsync(d, stream_);
      if (rc != 0 || hipStreamSynchronize(stream_) != hipSuccess) return -1;
      fprintf(stderr, "[splinter] closed a maintenance pass left open by pid %d\n", mr.pid);
    }
  }
  int rc = 0;
  if (flags & SPL_REHASH_FULL) {
    const bool need_hold = ring_ && ring_->ready();
    const bool held = need_hold && ring_->hold(true) == 0;
    if (need_hold && !held) { errno = EBUSY; return -1; }
    {
      RingQuiesce quiet;  // hipMalloc / hipFree may wait for the device: no resident worker of this process
      std::lock_guard<std::mutex> lk(mu_);
      uint32_t* d_idx = nullptr;
      uint64_t* d_cnt = nullptr;
      void* d_tmp = nullptr;
      uint64_t hc[2] = {0, 0};
      size_t scratch = 0;
      bool alloc_ok = hipMalloc((void**)&d_idx, (size_t)geo_.slots * 4) == hipSuccess &&
                      hipMalloc((void**)&d_cnt, 16) == hipSuccess && hipMemsetAsync(d_cnt, 0, 16, stream_) == hipSuccess &&
                      spl_arena_rebuild_collect(a, d_idx, d_cnt, stream_) == 0 &&
                      hipMemcpyAsync(hc, d_cnt, 8, hipMemcpyDeviceToHost, stream_) == hipSuccess &&
                      hipStreamSynchronize(stream_) == hipSuccess;
      if (alloc_ok) {
        scratch = (size_t)hc[0] * spl_arena_rebuild_rec(a) + 16;
        alloc_ok = hipMalloc(&d_tmp, scratch) == hipSuccess;
      }
      if (!alloc_ok) {
        (void)hipGetLastError();
        size_t fr = 0, tot = 0;
        (void)hipMemGetInfo(&fr, &tot);
        fprintf(stderr, "[splinter] rehash --full: cannot allocate %zu B of scratch (%lu live entries x %u B; %zu B free "
                "on the device); the arena is unchanged -- run the online rehash instead\n",
                scratch ? scratch : (size_t)geo_.slots * 4, (unsigned long)hc[0], spl_arena_rebuild_rec(a), fr);
        errno = ENOMEM;
        rc = -1;
      } else {
        // from here on the arena is rewritten: a failure is an error
        if (spl_arena_rebuild_move(a, d_idx, hc[0], d_tmp, d_cnt + 1, stream_) != 0 ||
            hipMemcpyAsync(hc + 1, d_cnt + 1, 8, hipMemcpyDeviceToHost, stream_) != hipSuccess ||
            hipStreamSynchronize(stream_) != hipSuccess || hc[1] != 0)
          rc = -1;
        out[0] = hc[0];
        out[1] = ps.tombstones;
        out[3] = hc[1];
      }
      if (d_tmp) (void)hipFree(d_tmp);
      if (d_cnt) (void)hipFree(d_cnt);
      if (d_idx) (void)hipFree(d_idx);
    }
    if (held) ring_->hold(false);
  } else {
    std::lock_guard<std::mutex> lk(mu_);
    uint64_t* d = nullptr;
    // d[0..4]: the pass counters (moved, reclaimed, clusters, skipped, largest displacement);
    // d[6] / d[7]: the open / close results
    const hipStream_t ms = maint_stream(device_) ? maint_stream(device_) : stream_;
    {  // this process's earlier work on the store's stream comes first
      hipEvent_t ev = nullptr;
      if (ms != stream_ && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
        (void)hipEventRecord(ev, stream_);
        (void)hipStreamWaitEvent(ms, ev, 0);
        (void)hipEventDestroy(ev);
      }
    }
    if (hipMallocAsync((void**)&d, 64, ms) != hipSuccess) return -1;
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    const uint64_t t0 = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
    uint64_t won = 0;
    (void)hipMemsetAsync(d, 0, 64, ms);
    rc = spl_arena_maint_mark(a, 1, (int)getpid(), t0, d + 6, ms);
    if (rc == 0) rc = hipMemcpyAsync(&won, d + 6, 8, hipMemcpyDeviceToHost, ms) == hipSuccess ? 0 : -1;
    if (rc == 0) rc = hipStreamSynchronize(ms) == hipSuccess ? 0 : -1;
    if (rc == 0 && !won) {
      errno = EBUSY;  // another process's pass is running
      rc = -1;
    } else if (rc == 0) {
      rc = spl_arena_rehash(a, d, ms);
      // the pass is closed whatever the walk returned: an open seq would turn every miss into EAGAIN
      if (spl_arena_maint_mark(a, 0, 0, 0, d + 7, ms) != 0) rc = -1;
      if (rc == 0) (void)hipMemcpyAsync(out, d, 32, hipMemcpyDeviceToHost, ms);
      if (hipStreamSynchronize(ms) != hipSuccess) rc = -1;
    }
    (void)hipFreeAsync(d, ms);
    (void)hipStreamSynchronize(ms);
  }
  if (rc == 0) {
    std::lock_guard<std::mutex> lk(mu_);
    ProbeStats sd;
    if (hipMemcpy(&sd, side, sizeof sd, hipMemcpyDeviceToHost) == hipSuccess) {
      sd.rebuilds += 1;
      sd.moved += out[0];
      sd.reclaimed += out[1];
      (void)hipMemcpy(side, &sd, sizeof sd, hipMemcpyHostToDevice);
    }
  }
  return rc == 0 ? 0 : -1;
}

// The maintenance seq of the arena (odd while a pass runs), for hosts that enumerate and want to
// know whether a pass overlapped them.
int HbmStore::maint_seq(uint64_t* seq) {
  if (!ensure_mapped() || !(side_flags_ & SPL_ARENA_SIDE)) return -1;
  DevGuard dg(device_);
  const uint8_t* side = (const uint8_t*)dbase_ + side_offset(geo_.slots, geo_.stride, geo_.max_val);
  return hipMemcpy(seq, side + kSideMaintOff, 8, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

StoreBase* hbm_factory_impl(const char* name, size_t slots, size_t max_val, unsigned flags, int create, int* err) {
  RingQuiesce quiet;  // no resident ring worker of this process while the new store is set up
  if (create) {
    const int dev = (int)((flags >> kCreateDeviceShift) & 0xFF) - 1;  // -1: the current device
    DevGuard dg(dev);
    return HbmStore::create(name, slots, max_val, (flags & kCreateEmbeddings) != 0, err);
  }
  return HbmStore::open(name, err);
}

}  // namespace spl

namespace spl {

namespace {

bool host_pinned(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

inline long al256(long x) { return (x + 255) & ~255L; }
inline long r16(long x) { return (x + 15) & ~15L; }

long count_ok(const int32_t* st, long n) {
  long ok = 0;
  for (long i = 0; i < n; ++i) ok += st[i] == 0;
  return ok;
}

}  // namespace

// Run a batch of n ops in chunks: per chunk, every input column goes to the device (a 2-D DMA from
// the caller's array when it is pinned, else through the slot's pinned buffer), `kernel(m, dev
// column pointers, stream)` runs, and every output column comes back the same way.  Key and value
// records are widened to 16-B device rows (the 2-D copies re-stride them; pad bytes are zeroed).
template <class K>
long HbmStore::batch_run(long n, Col* cols, int ncols, K&& kernel) {
  DevGuard dg(device_);
  std::lock_guard<std::mutex> lk(batch_mu_);
  long per = 0, hper = 0;
  for (int c = 0; c < ncols; ++c) {
    cols[c].pinned = host_pinned(cols[c].user);
    per += cols[c].dstride;
    if (!cols[c].pinned) hper += cols[c].ustride;
  }
  static const long budget = (long)(getenv("SPLINTER_BATCH_CHUNK_MB") ? atol(getenv("SPLINTER_BATCH_CHUNK_MB"))
                                                                      : 96) << 20;
  const long chunk = std::max(1L, std::min(n, budget / std::max(per, 1L)));
  const size_t dneed = (size_t)(chunk * per + 256L * ncols), hneed = (size_t)(chunk * hper + 256L * ncols);
  for (auto& st : stg_) {
    if (!st.s && hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking) != hipSuccess) return -1;
    if (st.dbytes < dneed) {
      if (st.d) (void)hipFree(st.d);
      st.d = nullptr;
      st.dbytes = 0;
      if (hipMalloc((void**)&st.d, dneed) != hipSuccess) return -1;
      st.dbytes = dneed;
    }
    if (hper > 0 && st.hbytes < hneed) {
      if (st.h) (void)hipHostFree(st.h);
      st.h = nullptr;
      st.hbytes = 0;
      if (hipHostMalloc((void**)&st.h, hneed, hipHostMallocPortable) != hipSuccess) return -1;
      st.hbytes = hneed;
    }
  }
  auto drain = [&](Stage& st) -> int {
    if (hipStreamSynchronize(st.s) != hipSuccess) return -1;
    for (auto& o : st.out) std::memcpy(o.first.first, o.first.second, o.second);
    st.out.clear();
    return 0;
  };
  int rc = 0;
  for (long b = 0, ci = 0; b < n && rc == 0; b += chunk, ++ci) {
    Stage& st = stg_[ci & 1];
    if (drain(st) != 0) { rc = -1; break; }
    const long m = std::min(chunk, n - b);
    void* dptr[8];
    uint8_t* dp = st.d;
    uint8_t* hp = st.h;
    for (int c = 0; c < ncols; ++c) {
      Col& col = cols[c];
      dptr[c] = dp;
      uint8_t* user = (uint8_t*)col.user + b * col.ustride;
      const long w = std::min(col.ustride, col.dstride);
      if (col.in) {
        if (col.dstride != col.ustride) (void)hipMemsetAsync(dp, 0, (size_t)(m * col.dstride), st.s);
        const uint8_t* src = user;
        if (!col.pinned) {
          std::memcpy(hp, user, (size_t)(m * col.ustride));
          src = hp;
        }
        const hipError_t e = col.dstride == col.ustride
                                 ? hipMemcpyAsync(dp, src, (size_t)(m * col.ustride), hipMemcpyHostToDevice, st.s)
                                 : hipMemcpy2DAsync(dp, (size_t)col.dstride, src, (size_t)col.ustride, (size_t)w,
                                                    (size_t)m, hipMemcpyHostToDevice, st.s);
        if (e != hipSuccess) { rc = -1; break; }
      }
      if (!col.pinned) hp += al256(m * col.ustride);
      dp += al256(m * col.dstride);
    }
    if (rc) break;
    if (kernel(m, dptr, st.s) != 0) { rc = -1; break; }
    hp = st.h;
    for (int c = 0; c < ncols; ++c) {
      Col& col = cols[c];
      uint8_t* user = (uint8_t*)col.user + b * col.ustride;
      const long w = std::min(col.ustride, col.dstride);
      if (col.out) {
        uint8_t* dst = col.pinned ? user : hp;
        const hipError_t e = col.dstride == col.ustride
                                 ? hipMemcpyAsync(dst, dptr[c], (size_t)(m * col.ustride), hipMemcpyDeviceToHost, st.s)
                                 : hipMemcpy2DAsync(dst, (size_t)col.ustride, dptr[c], (size_t)col.dstride, (size_t)w,
                                                    (size_t)m, hipMemcpyDeviceToHost, st.s);
        if (e != hipSuccess) { rc = -1; break; }
        if (!col.pinned) st.out.push_back({{user, hp}, (size_t)(m * col.ustride)});
      }
      if (!col.pinned) hp += al256(m * col.ustride);
    }
  }
  for (auto& st : stg_)
    if (st.s && drain(st) != 0) rc = -1;
  return rc;
}

long HbmStore::set_batch(const char* keys, int kstride, const uint8_t* vals, int vstride, const uint32_t* lens,
                         long n, int32_t* status, int retries) {
  std::vector<int32_t> tmp;
  if (!status) { tmp.resize((size_t)n); status = tmp.data(); }
  Col cols[4] = {{keys, kstride, r16(kstride), true, false, false},
                 {vals, vstride, r16(vstride), true, false, false},
                 {lens, 4, 4, true, false, false},
                 {status, 4, 4, false, true, false}};
  const int ks = (int)r16(kstride), vs = (int)r16(vstride);
  if (!ensure_mapped()) return -1;
  const spl_arena_t a = arena();
  if (batch_run(n, cols, 4, [&](long m, void** d, hipStream_t st) {
        return spl_arena_set(a, (const char*)d[0], ks, (const uint8_t*)d[1], vs, (const uint32_t*)d[2], m,
                             (int32_t*)d[3], retries, nullptr, st);
      }) != 0)
    return -1;
  return count_ok(status, n);
}

long HbmStore::get_batch(const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens, long n,
                         int32_t* status, int retries) {
  std::vector<int32_t> tst;
  std::vector<uint32_t> tln;
  if (!status) { tst.resize((size_t)n); status = tst.data(); }
  if (!out_lens) { tln.resize((size_t)n); out_lens = tln.data(); }
  const int ks = (int)r16(kstride);
  const long os = out ? r16(ostride) : 0;
  Col cols[4] = {{keys, kstride, ks, true, false, false},
                 {status, 4, 4, false, true, false},
                 {out_lens, 4, 4, false, true, false},
                 {out, ostride, os, false, true, false}};
  if (!ensure_mapped()) return -1;
  const spl_arena_t a = arena();
  if (batch_run(n, cols, out ? 4 : 3, [&](long m, void** d, hipStream_t st) {
        return spl_arena_get(a, (const char*)d[0], ks, out ? (uint8_t*)d[3] : nullptr, out ? (int)os : 16,
                             (uint32_t*)d[2], m, (int32_t*)d[1], retries, nullptr, st);
      }) != 0)
    return -1;
  long ok = 0;
  for (long i = 0; i < n; ++i) {
    // a row narrower than the value: EMSGSIZE, as the per-call get into a short buffer
    if (status[i] == 0 && out && out_lens[i] > (uint32_t)ostride) {
      status[i] = -EMSGSIZE;
      out_lens[i] = 0;
    }
    ok += status[i] == 0;
  }
  return ok;
}

long HbmStore::intop_batch(const char* keys, int kstride, const int* ops, const uint64_t* masks, long n,
                           int32_t* status, uint64_t* results) {
  std::vector<int32_t> tst;
  std::vector<uint64_t> tm;
  if (!status) { tst.resize((size_t)n); status = tst.data(); }
  if (!masks) { tm.assign((size_t)n, 0); masks = tm.data(); }
  const int ks = (int)r16(kstride);
  Col cols[5] = {{keys, kstride, ks, true, false, false},
                 {ops, 4, 4, true, false, false},
                 {masks, 8, 8, true, false, false},
                 {status, 4, 4, false, true, false},
                 {results, 8, 8, false, true, false}};
  if (!ensure_mapped()) return -1;
  const spl_arena_t a = arena();
  if (batch_run(n, cols, results ? 5 : 4, [&](long m, void** d, hipStream_t st) {
        return spl_arena_intop(a, (const char*)d[0], ks, (const int*)d[1], (const uint64_t*)d[2], m, (int32_t*)d[3],
                               results ? (uint64_t*)d[4] : nullptr, 64, st);
      }) != 0)
    return -1;
  return count_ok(status, n);
}

long HbmStore::set_embedding_batch(const char* keys, int kstride, const float* vecs, long n, int32_t* status) {
  if (geo_.stride != kSlotEmbedBytes) {
    for (long i = 0; status && i < n; ++i) status[i] = -ENOTSUP;
    return 0;
  }
  std::vector<int32_t> tst;
  if (!status) { tst.resize((size_t)n); status = tst.data(); }
  const int ks = (int)r16(kstride);
  Col cols[3] = {{keys, kstride, ks, true, false, false},
                 {vecs, (long)kEmbedBytes, (long)kEmbedBytes, true, false, false},
                 {status, 4, 4, false, true, false}};
  if (!ensure_mapped()) return -1;
  const spl_arena_t a = arena();
  if (batch_run(n, cols, 3, [&](long m, void** d, hipStream_t st) {
        return spl_arena_embed_set(a, (const char*)d[0], ks, (const float*)d[1], m, (int32_t*)d[2], st);
      }) != 0)
    return -1;
  return count_ok(status, n);
}

}  // namespace spl

extern "C" {

spl::StoreBase* spl_hbm_factory(const char* name, size_t slots, size_t max_val, unsigned flags, int create, int* err) {
  return spl::hbm_factory_impl(name, slots, max_val, flags, create, err);
}

// Arena descriptor of an open HBM store (for the batch launchers).
int spl_hbm_arena(spl_store* h, spl_arena_t* out) {
  auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h);
  if (!s || !out) return -2;
  if (!s->attach()) return -5;  // an opener maps the arena on first device use
  *out = s->arena();
  return 0;
}

// Worker launches of the store's command ring so far (a relaunch follows every idle period).
uint32_t spl_hbm_ring_launches(spl_store* h) {
  auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h);
  return s ? s->ring_launches() : 0;
}

// Hold (on != 0) / release every per-call ring worker of this process (cmd_ring.hpp ring_hold):
// a process about to run a heavy GPU job keeps its resident workers off the GPU meanwhile.
void spl_ring_hold(int on) { spl::ring_hold(on != 0); }

// Store-level hold, from any process that has the store open (the owner's ring server, a client
// of it, or a private ring): the store's worker exits and stays off the GPU until every hold is
// released; the store's per-call ops wait meanwhile.  For a process that runs a heavy GPU job
// while another process hosts the store's ring.  0 / -1 (errno).
int spl_hbm_ring_hold(spl_store* h, int on) {
  auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h);
  if (!s) { errno = EINVAL; return -1; }
  return s->ring_hold(on != 0);
}

// 0: the store's calls run on this process's own ring worker; 1: this process hosts the store's
// ring server; 2: it submits to the owner's ring server (cmd_ring.hpp); -1: not an HBM store
int spl_hbm_ring_mode(spl_store* h) {
  auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h);
  return s ? s->ring_mode() : -1;
}

// Pinned, device-mapped host memory for batch arrays (splinter_ext.h spl_batch_alloc).
void* spl_hbm_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}
void spl_hbm_host_free(void* p) { (void)hipHostFree(p); }

int spl_hbm_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

// CLI search on an HBM store, or on a node store of HBM shards: every shard scores its own slots
// on its GPU, the per-shard best `cap` are merged by (similarity desc, distance asc) on the host --
// the in-process form of the C4 top-k merge (parallel/sharded.py search_topk)
long spl_hbm_search(spl_store* h, const float* query, uint64_t mask, float min_sim, float max_dist, long cap,
                    spl_search_hit* out) {
  if (!h || !query || (cap > 0 && !out)) return -2;
  if (auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h)) return s->search_all(query, mask, min_sim, max_dist, cap, out);
  const int n = spl_node_nshards(h);
  if (n < 1) return -2;
  std::vector<spl_search_hit> all;
  long total = 0;
  for (int i = 0; i < n; ++i) {
    auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)spl_node_shard(h, i));
    if (!s) return -2;
    std::vector<spl_search_hit> part((size_t)std::max<long>(cap, 0));
    const long c = s->search_all(query, mask, min_sim, max_dist, cap, part.data());
    if (c < 0) return -1;
    total += c;
    part.resize((size_t)std::min<long>(c, cap));
    all.insert(all.end(), part.begin(), part.end());
  }
  auto better = [](const spl_search_hit& a, const spl_search_hit& b) {
    const float sa = a.emb ? a.sim : 0.f, sb = b.emb ? b.sim : 0.f;
    if (sa != sb) return sa > sb;
    if (a.dist != b.dist) return a.dist < b.dist;
    return strncmp(a.key, b.key, 64) < 0;
  };
  std::sort(all.begin(), all.end(), better);
  const size_t keep = (size_t)std::min<long>((long)all.size(), std::max<long>(cap, 0));
  for (size_t i = 0; i < keep; ++i) out[i] = all[i];
  return total;
}

// Batched top-k search (HbmStore::search_batch) of an HBM store, or of a node store of HBM shards:
// every shard answers every query on its GPU, all shards concurrently, and the per-shard top-k
// lists are merged per query (similarity desc, distance asc) -- the in-process C4 merge.
// out[nq * k]; returns nq or < 0.
long spl_search_batch(spl_store* h, const float* queries, int nq, int k, float min_sim, float max_dist,
                      uint64_t mask, spl_search_hit* out) {
  if (!h || !queries || !out || nq <= 0 || k <= 0 || k > 32) return -2;
  if (auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h))
    return s->search_batch(queries, nq, k, min_sim, max_dist, mask, out);
  const int n = spl_node_nshards(h);
  if (n < 1) return -2;
  // every shard answers every query at once: one host thread per shard, each driving its own
  // store's stream on its own GPU (was one shard after another, each with its own synchronise)
  std::vector<std::vector<spl_search_hit>> part((size_t)n, std::vector<spl_search_hit>((size_t)nq * k));
  std::vector<long> rc((size_t)n, -1);
  {
    std::vector<std::thread> th;
    th.reserve((size_t)n);
    // shards on one device search on streams of their own (spl::search_stream), and split the
    // threshold sample of one store between them
    std::vector<int> slot((size_t)n, 0);
    for (int i = 0; i < n; ++i) {
      auto* si = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)spl_node_shard(h, i));
      for (int j = 0; si && j < i; ++j) {
        auto* sj = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)spl_node_shard(h, j));
        if (sj && sj->device() == si->device()) ++slot[(size_t)i];
      }
    }
    spl::SearchSync sync(n);
    for (int i = 0; i < n; ++i)
      th.emplace_back([&, i] {
        spl::g_search_slot = slot[(size_t)i];
        auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)spl_node_shard(h, i));
        rc[(size_t)i] =
            s ? s->search_batch(queries, nq, k, min_sim, max_dist, mask, part[(size_t)i].data(), n, &sync) : -1;
        sync.leave();
      });
    for (auto& t : th) t.join();
  }
  std::vector<std::vector<spl_search_hit>> all((size_t)nq);
  for (int i = 0; i < n; ++i) {
    if (rc[(size_t)i] != nq) return -1;
    for (int qi = 0; qi < nq; ++qi)
      for (int j = 0; j < k; ++j)
        if (part[(size_t)i][(size_t)qi * k + j].emb) all[qi].push_back(part[(size_t)i][(size_t)qi * k + j]);
  }
  auto better = [](const spl_search_hit& a, const spl_search_hit& b) {
    if (a.sim != b.sim) return a.sim > b.sim;
    if (a.dist != b.dist) return a.dist < b.dist;
    return strncmp(a.key, b.key, 64) < 0;
  };
  for (int qi = 0; qi < nq; ++qi) {
    std::sort(all[qi].begin(), all[qi].end(), better);
    for (int j = 0; j < k; ++j) {
      spl_search_hit& o = out[(size_t)qi * k + j];
      if ((size_t)j < all[qi].size()) {
        o = all[qi][j];
      } else {
        std::memset(&o, 0, sizeof o);
        o.sim = -3.4e38f;
      }
    }
  }
  return nq;
}

// Probe-chain statistics of an HBM store, or summed over the shards of a node store (maxima taken)
int spl_hbm_probe_stats(spl_store* h, spl_probe_stats* out) {
  static_assert(sizeof(spl_probe_stats) == sizeof(spl::ProbeStats), "ABI struct = ProbeStats");
  if (!h || !out) return -2;
  if (auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h)) return s->probe_stats((spl::ProbeStats*)out);
  const int n = spl_node_nshards(h);
  if (n < 1) return -2;
  std::memset(out, 0, sizeof *out);
  uint64_t* o = (uint64_t*)out;
  for (int i = 0; i < n; ++i) {
    auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)spl_node_shard(h, i));
    spl::ProbeStats p;
    if (!s || s->probe_stats(&p) != 0) return -1;
    const uint64_t* v = (const uint64_t*)&p;
    for (size_t f = 0; f < sizeof p / 8; ++f) {
      const bool is_max = f == offsetof(spl::ProbeStats, disp_max) / 8 || f == offsetof(spl::ProbeStats, miss_max) / 8;
      o[f] = is_max ? std::max(o[f], v[f]) : o[f] + v[f];
    }
  }
  return 0;
}

// Tombstone maintenance of an HBM store / every shard of a node store (see HbmStore::rehash:
// online compaction by default, SPL_REHASH_FULL the exclusive full rebuild).  out (optional):
// {moved, reclaimed, clusters, skipped}, summed.
int spl_hbm_rehash_ex(spl_store* h, unsigned flags, uint64_t* out) {
  uint64_t tmp[4] = {0, 0, 0, 0};
  if (!h) return -2;
  if (auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h)) {
    const int rc = s->rehash(tmp, flags);
    if (out) std::memcpy(out, tmp, sizeof tmp);
    return rc;
  }
  const int n = spl_node_nshards(h);
  if (n < 1) return -2;
  uint64_t sum[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)spl_node_shard(h, i));
    if (!s || s->rehash(tmp, flags) != 0) return -1;
    for (int k = 0; k < 4; ++k) sum[k] += tmp[k];
  }
  if (out) std::memcpy(out, sum, sizeof sum);
  return 0;
}
int spl_hbm_rehash(spl_store* h, uint64_t* out) { return spl_hbm_rehash_ex(h, 0, out); }

int spl_hbm_maint_seq(spl_store* h, uint64_t* seq) {
  auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h);
  return s && seq ? s->maint_seq(seq) : -2;
}

// checkpoint / restore of an HBM store, or of every shard of a node store (PATH.s<i>)
int spl_hbm_checkpoint(spl_store* h, const char* path) {
  if (auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h)) return s->checkpoint(path);
  const int n = path ? spl_node_nshards(h) : -1;
  if (n < 1) return -2;
  for (int i = 0; i < n; ++i) {
    auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)spl_node_shard(h, i));
    if (!s || s->checkpoint((std::string(path) + ".s" + std::to_string(i)).c_str()) != 0) return -1;
  }
  return 0;
}

int spl_hbm_restore(spl_store* h, const char* path) {
  if (auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)h)) return s->restore_from(path);
  const int n = path ? spl_node_nshards(h) : -1;
  if (n < 1) return -2;
  for (int i = 0; i < n; ++i) {
    auto* s = dynamic_cast<spl::HbmStore*>((spl::StoreBase*)spl_node_shard(h, i));
    if (!s || s->restore_from((std::string(path) + ".s" + std::to_string(i)).c_str()) != 0) return -1;
  }
  return 0;
}

}  // extern "C"
