// node_store.cpp — "node:NAME": one store over the per-GPU arenas of a node (node_store.hpp).
#include "node_store.hpp"

#include <cerrno>
#include <memory>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/eventfd.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <emmintrin.h>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <thread>
#include <vector>

#include "splinter_ext.h"

namespace spl {

void* hbm_symbol(const char* sym);  // capi.cpp: dlsym in the HBM backend (loaded on demand)

namespace {

size_t desc_span() {
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  return (sizeof(NodeDesc) + pg - 1) / pg * pg;
}

// create: O_EXCL (fails with EEXIST if the node exists); *fresh tells which happened for join
NodeDesc* map_desc(const std::string& name, bool create, bool excl, bool* fresh, int* err) {
  const std::string dn = name + ".node";
  int fd = -1;
  if (fresh) *fresh = false;
  if (create) {
    mode_t prev = env_umask_push();
    fd = shm_open(dn.c_str(), O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0666);
    env_umask_pop(prev);
    if (fd >= 0 && fresh) *fresh = true;
    if (fd >= 0 && ftruncate(fd, (off_t)desc_span()) != 0) {
      *err = errno;
      close(fd);
      shm_unlink(dn.c_str());
      return nullptr;
    }
    if (fd < 0 && (excl || errno != EEXIST)) { *err = errno; return nullptr; }
  }
  if (fd < 0) {
    fd = shm_open(dn.c_str(), O_RDWR | O_CLOEXEC, 0666);
    if (fd < 0) { *err = errno; return nullptr; }
    // a rank that lost the O_EXCL race may see the winner's object before its ftruncate: wait (up
    // to 5 s) until the descriptor is full size, so the first read of d->magic cannot SIGBUS
    struct stat st;
    for (int i = 0;; ++i) {
      if (fstat(fd, &st) != 0) { *err = errno; close(fd); return nullptr; }
      if ((size_t)st.st_size >= desc_span()) break;
      if (i >= 5000) { *err = ETIMEDOUT; close(fd); return nullptr; }
      usleep(1000);
    }
  }
  void* p = mmap(nullptr, desc_span(), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) { *err = errno; return nullptr; }
  return (NodeDesc*)p;
}

void unmap_desc(NodeDesc* d) { if (d) munmap(d, desc_span()); }

bool wait_magic(NodeDesc* d, int ms) {
  for (int i = 0; i < ms; ++i) {
    if (__atomic_load_n(&d->magic, __ATOMIC_ACQUIRE) == kNodeMagic) return true;
    usleep(1000);
  }
  return __atomic_load_n(&d->magic, __ATOMIC_ACQUIRE) == kNodeMagic;
}

// posix_madvise over [a, a+l) widened to page boundaries (the reference aligns the same way,
// splinter.c:1329-1377); errno-style return as posix_madvise
int forward_advice(void* a, size_t l, int advice) {
  const long pg = sysconf(_SC_PAGESIZE);
  if (pg > 0) {
    const uintptr_t x = (uintptr_t)a, al = x & ~((uintptr_t)pg - 1);
    l += (size_t)(x - al);
    a = (void*)al;
  }
  const int rc = posix_madvise(a, l, advice);
  if (rc != 0) errno = rc;
  return rc;
}

int hbm_devices() {
  auto f = (int (*)())hbm_symbol("spl_hbm_device_count");
  return f ? f() : 0;
}

uint32_t default_backend() {
  const char* e = getenv("SPLINTER_NODE_BACKEND");
  if (e && *e) return strcmp(e, "shm") == 0 ? 0u : 1u;
  return hbm_devices() > 0 ? 1u : 0u;
}

StoreBase* make_shard(const std::string& node, int i, uint32_t backend, bool create, size_t slots, size_t max_val,
                      bool emb, int device, int* err) {
  const std::string full = node_shard_name(node, i, backend);
  const std::string bare = full.substr(4);  // without the "hbm:" / "shm:" prefix
  if (backend == 1) {
    HbmFactory f = load_hbm_factory();
    if (!f) { *err = ENOSYS; return nullptr; }
    unsigned flags = emb ? kCreateEmbeddings : kCreateNoEmbeddings;
    if (device >= 0) flags |= (unsigned)(device + 1) << kCreateDeviceShift;
    return f(bare.c_str(), slots, max_val, flags, create ? 1 : 0, err);
  }
  return create ? (StoreBase*)HostStore::create(bare.c_str(), false, slots, max_val, emb, err)
                : (StoreBase*)HostStore::open(bare.c_str(), false, err);
}

// The stand-in of a shard whose owning rank process is gone: every op answers EAGAIN (the
// reference's recoverable status, splinter.h:400-412) -- the key's shard is not served until its
// rank's restarted process re-joins -- and the other shards of the node keep serving.
class DownShard final : public StoreBase {
 public:
  explicit DownShard(Geometry g) : g_(g) {}
  static int again() { errno = EAGAIN; return -1; }
  const char* backend() const override { return "down"; }
  Geometry geometry() const override { return g_; }
  splinter_header* header_ptr() override { return nullptr; }
  int set_mop(unsigned) override { return again(); }
  int get_mop() override { return again(); }
  void purge() override {}
  int header_snapshot(splinter_header_snapshot_t*) override { return again(); }
  uint8_t config_get() override { return 0; }
  void config_or(uint8_t) override {}
  void config_and(uint8_t) override {}
  int set(const char*, const void*, size_t) override { return again(); }
  int unset(const char*) override { return again(); }
  int get(const char*, void*, size_t, size_t*) override { return again(); }
  int list(char**, size_t, size_t* n) override { if (n) *n = 0; return 0; }
  int poll(const char*, uint64_t) override { return again(); }
  int slot_snapshot(const char*, splinter_slot_snapshot_t*) override { return again(); }
  int append(const char*, const void*, size_t, size_t*) override { return again(); }
  const void* raw_ptr(const char*, size_t*, uint64_t*) override { errno = EAGAIN; return nullptr; }
  uint64_t epoch_of(const char*) override { errno = EAGAIN; return 0; }
  int set_as_system(const char*) override { return again(); }
  int set_embedding(const char*, const float*) override { return again(); }
  int get_embedding(const char*, float*) override { return again(); }
  int set_named_type(const char*, uint16_t) override { return again(); }
  int set_slot_time(const char*, unsigned short, uint64_t, size_t) override { return again(); }
  int integer_op(const char*, splinter_integer_op_t, const void*) override { return again(); }
  int bump(const char*) override { return again(); }
  int retrain(const char*) override { return again(); }
  int set_label(const char*, uint64_t) override { return again(); }
  int unset_label(const char*, uint64_t) override { return again(); }
  int watch_register(const char*, uint8_t) override { return again(); }
  int watch_unregister(const char*, uint8_t) override { return again(); }
  int watch_label_register(uint64_t, uint8_t) override { return again(); }
  int pulse_keygroup(const char*) override { return again(); }
  void pulse_slot(splinter_slot*) override {}
  uint64_t signal_count(uint8_t) override { return 0; }
  int signal_add(uint8_t, uint64_t) override { return again(); }
  void enumerate(uint64_t, void (*)(const char*, uint64_t, void*), void*) override {}
  int event_bus_init() override { return again(); }
  int event_bus_open() override { return again(); }
  void event_bus_dirty(uint64_t* out, size_t words) override { for (size_t i = 0; i < words; ++i) out[i] = 0; }
  int shard_claim_ex(uint32_t, uint32_t, uint8_t, uint8_t, uint64_t, uint64_t) override { return again(); }
  int shard_rebid(uint32_t, uint8_t, uint8_t, uint64_t) override { return again(); }
  int shard_release(uint32_t) override { return again(); }
  uint32_t shard_election(uint8_t*) override { return 0; }
  int shard_table(splinter_shard_bid_snapshot*, size_t) override { return 0; }
  int madvise(uint32_t, void*, size_t, int, uint64_t) override { return again(); }
  static long fill(int32_t* st, long n) {
    if (st)
      for (long i = 0; i < n; ++i) st[i] = -EAGAIN;
    return 0;
  }
  long set_batch(const char*, int, const uint8_t*, int, const uint32_t*, long n, int32_t* st, int) override {
    return fill(st, n);
  }
  long get_batch(const char*, int, uint8_t*, int, uint32_t* ol, long n, int32_t* st, int) override {
    if (ol)
      for (long i = 0; i < n; ++i) ol[i] = 0;
    return fill(st, n);
  }
  long intop_batch(const char*, int, const int*, const uint64_t*, long n, int32_t* st, uint64_t*) override {
    return fill(st, n);
  }
  long set_embedding_batch(const char*, int, const float*, long n, int32_t* st) override { return fill(st, n); }

 private:
  Geometry g_;
};

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

bool pid_gone(int32_t pid) { return pid > 0 && kill((pid_t)pid, 0) != 0 && errno == ESRCH; }

}  // namespace

std::string node_shard_name(const std::string& node, int i, uint32_t backend) {
  return std::string(backend == 1 ? "hbm:" : "shm:") + node + ".s" + std::to_string(i);
}

StoreBase* NodeStore::route(const char* key) {
  refresh();
  return at(node_shard_of(KeyRef(key).hash, (int)shards_.size()));
}

// Degraded mode: see node_store.hpp.  Joined nodes only (a node created whole by one process owns
// every shard itself: shard_pid 0).
void NodeStore::refresh(bool force) {
  constexpr uint64_t kRefreshNs = 20 * 1000 * 1000;
  const uint64_t now = mono_ns();
  if (!force && now < next_refresh_ns_.load(std::memory_order_relaxed)) return;
  std::lock_guard<std::mutex> lk(refresh_mu_);
  next_refresh_ns_.store(now + kRefreshNs, std::memory_order_relaxed);
  for (int i = 0; i < nshards(); ++i) {
    const int32_t pid = __atomic_load_n(&desc_->shard_pid[i], __ATOMIC_ACQUIRE);
    const uint32_t g = __atomic_load_n(&desc_->shard_gen[i], __ATOMIC_ACQUIRE);
    const bool ready = (__atomic_load_n(&desc_->ready_mask, __ATOMIC_ACQUIRE) >> i) & 1ull;
    StoreBase* want = real_[(size_t)i];
    const bool owned = __atomic_load_n(&desc_->shard_flags[i], __ATOMIC_ACQUIRE) & kShardOwned;
    if (g != gen_[(size_t)i] && ready && !(owned && pid_gone(pid))) {
      // the shard re-joined (its rank restarted): open the new shard store
      int err = 0;
      StoreBase* sh = make_shard(name_, i, desc_->backend, false, 0, 0, false, -1, &err);
      const Geometry geo = sh ? sh->geometry() : Geometry{};
      if (sh && geo.slots == desc_->slots_per_shard && geo.max_val == desc_->max_val && geo.stride == desc_->stride) {
        retired_.push_back(real_[(size_t)i]);
        real_[(size_t)i] = sh;
        gen_[(size_t)i] = g;
        want = sh;
      } else {
        delete sh;
        want = down_;
      }
    } else if (g != gen_[(size_t)i] || !ready || (owned && pid_gone(pid))) {
      want = down_;
    }
    __atomic_store_n(&shards_[(size_t)i], want, __ATOMIC_RELEASE);
  }
}

int NodeStore::shard_state(int i) {
  if (i < 0 || i >= nshards()) return -1;
  refresh(true);
  return at(i) == down_ ? 1 : 0;
}

Geometry NodeStore::geometry() const {
  Geometry g;
  g.slots = desc_->slots_per_shard * desc_->nshards;
  g.max_val = desc_->max_val;
  g.stride = desc_->stride;
  return g;
}

NodeStore* NodeStore::create(const std::string& name, size_t slots, size_t max_val, bool emb, int* err) {
  *err = 0;
  if (slots == 0 || max_val == 0 || max_val > UINT32_MAX) { *err = ENOTSUP; return nullptr; }
  const uint32_t backend = default_backend();
  const int ndev = backend == 1 ? hbm_devices() : 0;
  if (backend == 1 && ndev <= 0) { *err = ENODEV; return nullptr; }
  int n = backend == 1 ? ndev : 8;
  if (const char* e = getenv("SPLINTER_NODE_SHARDS")) n = atoi(e);
  if (n < 1 || n > kNodeMaxShards) { *err = EINVAL; return nullptr; }
  const size_t per = (slots + n - 1) / n;
  if (per > UINT32_MAX || per * n > UINT32_MAX) { *err = ENOTSUP; return nullptr; }
  bool fresh = false;
  NodeDesc* d = map_desc(name, true, true, &fresh, err);
  if (!d) return nullptr;
  auto* s = new NodeStore();
  s->name_ = name;
  s->desc_ = d;
  s->owner_ = true;
  std::memset((void*)d, 0, sizeof(NodeDesc));
  d->nshards = (uint32_t)n;
  d->backend = backend;
  d->slots_per_shard = (uint32_t)per;
  d->max_val = (uint32_t)max_val;
  d->stride = emb ? (uint32_t)kSlotEmbedBytes : (uint32_t)kSlotCoreBytes;
  d->creator_pid = (int32_t)getpid();
  d->event_fd = -1;
  for (int i = 0; i < n; ++i) {
    StoreBase* sh = make_shard(name, i, backend, true, per, max_val, emb, backend == 1 ? i % ndev : -1, err);
    if (!sh) {
      // roll back whatever backend: the shards made so far and the descriptor, so the name is free
      // again (host shards would otherwise outlive the failed create and collide with the next one)
      const int e = *err;
      s->owner_ = false;
      for (auto* x : s->shards_) delete x;
      s->shards_.clear();
      s->real_.clear();
      for (int j = 0; j < i; ++j) spl_unlink(node_shard_name(name, j, backend).c_str());
      delete s;
      shm_unlink((name + ".node").c_str());
      *err = e;
      return nullptr;
    }
    s->shards_.push_back(sh);
    s->real_.push_back(sh);
    s->gen_.push_back(0);
    d->ready_mask |= 1ull << i;
  }
  s->down_ = new DownShard(s->shards_[0]->geometry());
  d->version = 1;
  __atomic_store_n(&d->magic, kNodeMagic, __ATOMIC_RELEASE);
  return s;
}

NodeStore* NodeStore::open(const std::string& name, int* err) {
  *err = 0;
  NodeDesc* d = map_desc(name, false, false, nullptr, err);
  if (!d) return nullptr;
  if (!wait_magic(d, 0)) { unmap_desc(d); *err = EINVAL; return nullptr; }
  const int n = (int)d->nshards;
  const uint64_t all = n >= 64 ? ~0ull : ((1ull << n) - 1);
  if (n < 1 || n > kNodeMaxShards || (__atomic_load_n(&d->ready_mask, __ATOMIC_ACQUIRE) & all) != all) {
    unmap_desc(d);
    *err = EAGAIN;  // a joined node whose ranks have not all attached their shard yet
    return nullptr;
  }
  auto* s = new NodeStore();
  s->name_ = name;
  s->desc_ = d;
  for (int i = 0; i < n; ++i) {
    StoreBase* sh = make_shard(name, i, d->backend, false, 0, 0, false, -1, err);
    if (!sh) {
      delete s;
      return nullptr;
    }
    const Geometry g = sh->geometry();
    if (g.slots != d->slots_per_shard || g.max_val != d->max_val || g.stride != d->stride) {
      delete sh;
      delete s;
      *err = EINVAL;
      return nullptr;
    }
    s->shards_.push_back(sh);
    s->real_.push_back(sh);
    s->gen_.push_back(__atomic_load_n(&d->shard_gen[i], __ATOMIC_ACQUIRE));
  }
  s->down_ = new DownShard(s->shards_[0]->geometry());
  s->refresh(true);
  return s;
}

NodeStore::~NodeStore() {
  if (scratch_) {
    using Free = void (*)(void*);
    static Free pf = (Free)hbm_symbol("spl_hbm_host_free");
    if (scratch_pinned_ && pf) pf(scratch_);
    else free(scratch_);
  }
  if (event_fd_ >= 0) {
    if (desc_ && __atomic_load_n(&desc_->event_pid, __ATOMIC_ACQUIRE) == (int32_t)getpid()) {
      __atomic_store_n(&desc_->event_fd, -1, __ATOMIC_RELEASE);
      __atomic_store_n(&desc_->event_pid, 0, __ATOMIC_RELEASE);
    }
    close(event_fd_);
  }
  for (auto* sh : real_) delete sh;
  for (auto* sh : retired_) delete sh;
  delete down_;
  if (desc_) {
    // an HBM node lives as long as its creator (the arenas are its allocations); a host-shard node
    // persists like any shm store until spl_unlink("node:NAME")
    const bool drop = owner_ && desc_->backend == 1;
    if (drop) __atomic_store_n(&desc_->magic, 0u, __ATOMIC_RELEASE);
    unmap_desc(desc_);
    if (drop) shm_unlink((name_ + ".node").c_str());
  }
}

int NodeStore::set_mop(unsigned mode) {
  int rc = 0;
  for (auto* s : shards_) {
    const int r = s->set_mop(mode);
    if (r != 0) rc = r;
  }
  return rc;
}

int NodeStore::header_snapshot(splinter_header_snapshot_t* out) {
  if (!out) return -2;
  refresh();
  StoreBase* f = first_up();
  if (f->header_snapshot(out) != 0) return -1;
  uint64_t epoch = 0;
  for (int i = 0; i < nshards(); ++i) {  // a down shard's writes are not counted until it re-joins
    splinter_header_snapshot_t h;
    if (at(i) == down_) continue;
    if (at(i)->header_snapshot(&h) != 0) return -1;
    epoch += h.epoch;
  }
  out->epoch = epoch;  // every write bumps its shard's global epoch: the sum is the node's
  out->slots = geometry().slots;
  return 0;
}

int NodeStore::list(char** out_keys, size_t max_keys, size_t* out_count) {
  if (!out_keys || !out_count) return -2;
  size_t c = 0;
  for (auto* s : shards_) {
    if (c >= max_keys) break;
    size_t n = 0;
    if (s->list(out_keys + c, max_keys - c, &n) != 0) return -1;
    c += n;
  }
  *out_count = c;
  return 0;
}

int NodeStore::watch_label_register(uint64_t mask, uint8_t g) {
  int rc = 0;
  for (auto* s : shards_) {
    const int r = s->watch_label_register(mask, g);
    if (r != 0) rc = r;
  }
  return rc;
}

uint64_t NodeStore::signal_count(uint8_t g) {
  uint64_t v = 0;
  for (auto* s : shards_) v += s->signal_count(g);
  return v;
}

void NodeStore::event_bus_dirty(uint64_t* out, size_t words) {
  if (!out) return;
  const size_t n = words < SPLINTER_EVENT_BUS_MASK_WORDS ? words : SPLINTER_EVENT_BUS_MASK_WORDS;
  std::memset(out, 0, n * 8);
  uint64_t tmp[SPLINTER_EVENT_BUS_MASK_WORDS];
  for (auto* s : shards_) {
    s->event_bus_dirty(tmp, n);
    for (size_t i = 0; i < n; ++i) out[i] |= tmp[i];
  }
}

// One node eventfd shared by every shard: each shard adopts (a dup of) it as its own bus, so a
// writer on any shard -- this process, another process through the shard header's owner fd, or a
// shard's device-notify proxy -- increments the one counter, and a single read drains every
// pending wakeup (as the reference's one eventfd, splinter.c event bus).
int NodeStore::event_bus_init() {
  const int fd = eventfd(0, EFD_CLOEXEC);
  if (fd < 0) return -1;
  for (auto* s : shards_) {
    if (s->event_bus_adopt(fd) != 0) {
      close(fd);
      return -1;
    }
  }
  if (event_fd_ >= 0) close(event_fd_);
  event_fd_ = fd;
  __atomic_store_n(&desc_->event_fd, fd, __ATOMIC_RELEASE);
  __atomic_store_n(&desc_->event_pid, (int32_t)getpid(), __ATOMIC_RELEASE);
  return 0;
}

int NodeStore::event_bus_open() {
  const int32_t fd = __atomic_load_n(&desc_->event_fd, __ATOMIC_ACQUIRE);
  const int32_t pid = __atomic_load_n(&desc_->event_pid, __ATOMIC_ACQUIRE);
  if (fd < 0 || pid <= 0) { errno = ENODEV; return -1; }
  if ((pid_t)pid == getpid()) return dup(fd);
#if defined(SYS_pidfd_open) && defined(SYS_pidfd_getfd)
  const int pfd = (int)syscall(SYS_pidfd_open, (pid_t)pid, 0);
  if (pfd < 0) return -1;
  const int r = (int)syscall(SYS_pidfd_getfd, pfd, fd, 0);
  close(pfd);
  return r;
#else
  errno = ENOSYS;
  return -1;
#endif
}

int NodeStore::madvise(uint32_t id, void* addr, size_t len, int advice, uint64_t timeout) {
  // one election per node (the node descriptor's bid table); the winner's advice is forwarded to
  // every shard's residency hint (HBM: a documented no-op, host shards: posix_madvise)
  if (id == 0 || !shard_present_on(&desc_->control, id)) { errno = EINVAL; return -2; }
  const uint64_t deadline = now_ticks() + timeout;
  for (;;) {
    if (shard_election_on(&desc_->control, nullptr) == id) break;
    if (timeout == 0) { errno = EAGAIN; return -1; }
    if (timeout != UINT64_MAX && now_ticks() >= deadline) { errno = ETIMEDOUT; return -1; }
    usleep(5000);
  }
  // forward the winner's advice: host shards get posix_madvise over their mapping (the whole arena
  // when addr is NULL; an address inside one shard's mapping goes to that shard), HBM shards take
  // their backend's documented residency no-op
  int rc = 0;
  for (auto* s : shards_) {
    void* a = addr;
    size_t l = len;
    if (auto* hs = dynamic_cast<HostStore*>(s)) {
      uint8_t* b = hs->base();
      const size_t span = hs->total_bytes();
      if (addr) {
        if ((uint8_t*)addr < b || (uint8_t*)addr >= b + span) continue;
        if ((uint8_t*)addr + len > b + span) l = (size_t)(b + span - (uint8_t*)addr);
      } else {
        a = b;
        l = span;
      }
      if (forward_advice(a, l, advice) != 0) rc = -1;
    }
  }
  return rc;
}

// ------------------------------------------------------------------ batches --
// A batch is counting-sorted by owning shard into one scratch buffer (pinned when the HBM backend
// is present, so HBM shards DMA straight from it), every shard's contiguous part runs on its own
// thread (HBM shards: HbmStore::*_batch on that shard's GPU, all GPUs at once), and the outputs go
// back into client order.  Two passes over the CLIENT order on batch_threads() pool threads: hash +
// per-part shard histogram, then placement with the input rows copied as each op is placed (the
// sort is stable per part, so each part reads its rows sequentially and writes one sequential
// stream per shard: no random row reads -- 66.7 M ops/s with per-row gathers by permutation, 4 HBM
// shards on one GPU, profiles/r4f).
namespace {
// SPLINTER_NODE_BATCH_THREADS (default min(16, hardware threads)): host threads that partition and
// copy a node batch (4 HBM shards on one GPU, 2M-op batches: 93 M ops/s before the pool, 105 M at
// 8 threads, 122 M at 16 -- profiles/r4ae)
int batch_threads() {
  static const int t = [] {
    const char* e = getenv("SPLINTER_NODE_BATCH_THREADS");
    const int hw = (int)std::thread::hardware_concurrency();
    const int v = e && *e ? atoi(e) : std::min(16, hw > 0 ? hw : 8);
    return v < 1 ? 1 : v > 64 ? 64 : v;
  }();
  return t;
}

// Fork-join pool of batch_threads() - 1 sleeping workers (the caller is part 0): the partition and
// the copies of every chunk run on it without creating threads.  One job at a time; a second
// concurrent caller (the pipeline's output copies beside the next chunk's partition) gets false
// and runs on threads of its own.  Re-created in a forked child; never destroyed (its workers
// sleep through process exit).
class BatchPool {
 public:
  explicit BatchPool(int n) : n_(n) {
    for (int i = 1; i < n; ++i) std::thread([this, i] { loop(i); }).detach();
  }
  bool run(const std::function<void(int)>& f) {
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
    return true;
  }

 private:
  void loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        f = job_;
      }
      (*f)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  const int n_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int pending_ = 0;
  uint64_t gen_ = 0;
};

BatchPool& batch_pool() {
  static std::mutex m;
  static BatchPool* p = nullptr;
  static pid_t pid = 0;
  std::lock_guard<std::mutex> lk(m);
  if (!p || pid != getpid()) {
    p = new BatchPool(batch_threads());
    pid = getpid();
  }
  return *p;
}

// parts a range of n ops is split into (the partition's per-part histograms follow the same split)
inline int par_parts(long n) { return n < 65536 ? 1 : batch_threads(); }

template <class F>
void par_range(long n, F&& f) {
  const int t = par_parts(n);
  if (t <= 1) { f(0L, n, 0); return; }
  const std::function<void(int)> job = [&](int i) { f(n * i / t, n * (i + 1) / t, i); };
  if (batch_pool().run(job)) return;
  std::vector<std::thread> th;
  for (int i = 0; i < t; ++i) th.emplace_back(job, i);
  for (auto& x : th) x.join();
}

// one row of w bytes (the common widths as fixed-size copies)
inline void copy_row(uint8_t* d, const uint8_t* s, long w) {
  switch (w) {
    case 4: std::memcpy(d, s, 4); break;
    case 8: std::memcpy(d, s, 8); break;
    case 16: std::memcpy(d, s, 16); break;
    case 32: std::memcpy(d, s, 32); break;
    default: std::memcpy(d, s, (size_t)w);
  }
}

// length of key record r (NUL-padded, kstride bytes), capped at cut: one 16-byte compare when the
// record is at least 16 bytes wide
inline int key_len(const char* r, int kstride, int cut) {
  if (kstride < 16) return (int)strnlen(r, (size_t)cut);
  const __m128i v = _mm_loadu_si128((const __m128i*)r);
  const unsigned z = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(v, _mm_setzero_si128()));
  if (z) return std::min(__builtin_ctz(z), cut);
  return cut <= 16 ? cut : 16 + (int)strnlen(r + 16, (size_t)(cut - 16));
}

// dest[i] = owning shard of key record i for i in [b, e), counted into cnt[shard].  FNV-1a is a
// serial multiply chain per key, so runs of 4 equal-length keys (the common case: fixed-format
// keys) are hashed side by side, 4 independent chains; == fnv1a_n(rec, strnlen(rec, cut)).
void shard_keys(const char* keys, int kstride, int cut, long b, long e, int nsh, int32_t* dest, long* cnt) {
  long i = b;
  for (; i + 4 <= e; i += 4) {
    const unsigned char* r0 = (const unsigned char*)keys + i * kstride;
    const unsigned char *r1 = r0 + kstride, *r2 = r1 + kstride, *r3 = r2 + kstride;
    const int l = key_len((const char*)r0, kstride, cut);
    uint64_t h[4];
    if (key_len((const char*)r1, kstride, cut) == l && key_len((const char*)r2, kstride, cut) == l &&
        key_len((const char*)r3, kstride, cut) == l) {
      uint64_t x0 = kFnvOffset, x1 = kFnvOffset, x2 = kFnvOffset, x3 = kFnvOffset;
      for (int p = 0; p < l; ++p) {
        x0 = (x0 ^ r0[p]) * kFnvPrime;
        x1 = (x1 ^ r1[p]) * kFnvPrime;
        x2 = (x2 ^ r2[p]) * kFnvPrime;
        x3 = (x3 ^ r3[p]) * kFnvPrime;
      }
      h[0] = x0; h[1] = x1; h[2] = x2; h[3] = x3;
    } else {
      for (int k = 0; k < 4; ++k) {
        const char* r = keys + (i + k) * kstride;
        h[k] = fnv1a_n(r, (size_t)key_len(r, kstride, cut));
      }
    }
    for (int k = 0; k < 4; ++k) {
      const int d = node_shard_of(h[k], nsh);
      dest[i + k] = d;
      ++cnt[d];
    }
  }
  for (; i < e; ++i) {
    const char* rec = keys + i * kstride;
    const int d = node_shard_of(fnv1a_n(rec, (size_t)key_len(rec, kstride, cut)), nsh);
    dest[i] = d;
    ++cnt[d];
  }
}

}  // namespace

// SPLINTER_NODE_BATCH_TRACE=1: per batch, ms in plan / gather / shards / scatter on stderr
struct BatchTrace {
  bool on;
  const char* what;
  long n;
  std::chrono::steady_clock::time_point t0, t;
  double ms[4] = {0, 0, 0, 0};
  BatchTrace(const char* w, long n_) : what(w), n(n_) {
    static const bool env = getenv("SPLINTER_NODE_BATCH_TRACE") && atoi(getenv("SPLINTER_NODE_BATCH_TRACE")) != 0;
    on = env;
    if (on) t0 = t = std::chrono::steady_clock::now();
  }
  void mark(int i) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    ms[i] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  }
  ~BatchTrace() {
    if (on)
      fprintf(stderr, "{\"node_batch\": \"%s\", \"n\": %ld, \"plan_ms\": %.2f, \"gather_ms\": %.2f, \"shards_ms\": %.2f, "
              "\"scatter_ms\": %.2f}\n", what, n, ms[0], ms[1], ms[2], ms[3]);
  }
};

struct NodeStore::Plan {
  long n;
  long* pos;      // pos[i]: sorted position of client op i
  int32_t* dest;  // dest[i]: owning shard of client op i
  std::vector<long> off;   // shard j's ops are sorted positions [off[j], off[j+1])
  std::vector<long> base;  // [part][shard]: next sorted position of that part's ops of the shard
  int nsh;
  // slot: which of the store's two Plan buffers (pipeline halves) holds pos / dest
  Plan(NodeStore& st, int slot, const char* keys, int kstride, long n_, int nsh_)
      : n(n_), off((size_t)nsh_ + 1, 0), nsh(nsh_) {
    auto& pv = st.plan_pos_[slot];
    auto& dv = st.plan_dest_[slot];
    if ((long)pv.size() < n) pv.resize((size_t)n);
    if ((long)dv.size() < n) dv.resize((size_t)n);
    pos = pv.data();
    dest = dv.data();
    const int cut = kstride < 64 ? kstride : 63;
    const int T = par_parts(n);
    std::vector<long> cnt((size_t)T * nsh, 0);
    par_range(n, [&](long b, long e, int t) { shard_keys(keys, kstride, cut, b, e, nsh, dest, cnt.data() + (size_t)t * nsh); });
    // stable placement: part t's ops of shard j follow those of parts < t
    base.resize((size_t)T * nsh);
    long run = 0;
    for (int j = 0; j < nsh; ++j) {
      off[(size_t)j] = run;
      for (int t = 0; t < T; ++t) {
        base[(size_t)t * nsh + j] = run;
        run += cnt[(size_t)t * nsh + j];
      }
    }
    off[(size_t)nsh] = run;
  }
  // the placement pass: pos[] filled in client order, put(i, q) copies op i's input rows to sorted
  // position q as it goes (each part reads its rows sequentially and writes one stream per shard)
  template <class F>
  void place(F&& put) {
    par_range(n, [&](long b, long e, int t) {
      long* p = base.data() + (size_t)t * nsh;
      for (long i = b; i < e; ++i) {
        const long q = p[dest[i]]++;
        pos[i] = q;
        put(i, q);
      }
    });
  }
  // sorted scratch column -> client column
  void scatter(void* dst, const uint8_t* src, long w) const {
    par_range(n, [&](long b, long e, int) {
      for (long i = b; i < e; ++i) copy_row((uint8_t*)dst + i * w, src + pos[i] * w, w);
    });
  }
  template <class F>
  void each_shard(F&& f) const {
    std::vector<std::thread> th;
    for (int j = 0; j < nsh; ++j)
      if (off[(size_t)j + 1] > off[(size_t)j]) th.emplace_back([&, j] { f(j, off[(size_t)j], off[(size_t)j + 1] - off[(size_t)j]); });
    for (auto& x : th) x.join();
  }
};

uint8_t* NodeStore::scratch(size_t bytes) {
  if (scratch_bytes_ >= bytes) return scratch_;
  using Alloc = void* (*)(size_t);
  using Free = void (*)(void*);
  static Alloc pa = (Alloc)hbm_symbol("spl_hbm_host_alloc");
  static Free pf = (Free)hbm_symbol("spl_hbm_host_free");
  if (scratch_) {
    if (scratch_pinned_ && pf) pf(scratch_);
    else free(scratch_);
  }
  scratch_ = nullptr;
  scratch_bytes_ = 0;
  scratch_pinned_ = false;
  if (desc_->backend == 1 && pa) {
    scratch_ = (uint8_t*)pa(bytes);
    scratch_pinned_ = scratch_ != nullptr;
  }
  if (!scratch_) scratch_ = (uint8_t*)aligned_alloc(64, (bytes + 63) / 64 * 64);
  if (scratch_) scratch_bytes_ = bytes;
  return scratch_;
}

namespace {
inline long a64(long x) { return (x + 63) & ~63L; }
}

namespace {
// SPLINTER_NODE_BATCH_CHUNK: ops per pipeline chunk of a node batch (default 524288)
long node_chunk_ops() {
  const char* e = getenv("SPLINTER_NODE_BATCH_CHUNK");
  const long v = e ? atol(e) : 0;
  return v > 0 ? v : 524288L;
}
}  // namespace

// HBM shards wait on their GPUs while the host prepares the next chunk; host shards would only
// compete with it for CPUs, so their batches run as one chunk
long NodeStore::chunk_for(long n) const {
  const char* e = getenv("SPLINTER_NODE_BATCH_PIPELINE");  // 1 / 0: force on / off (tests)
  const bool on = e && *e ? atoi(e) != 0 : desc_->backend == 1;
  return std::min(n, on ? node_chunk_ops() : n);
}

// Chunked two-stage pipeline: prep(c0, m, S) partitions and copies chunk [c0, c0+m) into scratch
// half S (host threads), exec(plan, c0, m, S) runs every shard on it and copies the outputs back
// (shard threads wait on their GPUs); chunk c+1 is prepared while chunk c executes.
template <class Prep, class Exec>
long NodeStore::pipeline(long n, long per, Prep&& prep, Exec&& exec) {
  const long C = chunk_for(n);
  const long nch = (n + C - 1) / C;
  uint8_t* S0 = scratch((size_t)(per * (nch > 1 ? 2 : 1)));
  if (!S0) return -1;
  long ok = 0;
  bool fail = false;
  std::unique_ptr<Plan> cur = prep(0L, C, S0, 0);
  for (long c = 0; c < nch; ++c) {
    const long c0 = c * C, m = std::min(C, n - c0);
    uint8_t* S = S0 + (c & 1) * per;
    long r = 0;
    std::unique_ptr<Plan> next;
    if (c + 1 < nch) {
      std::thread th([&] { r = exec(*cur, c0, m, S); });
      next = prep(c0 + C, std::min(C, n - c0 - C), S0 + ((c + 1) & 1) * per, (int)((c + 1) & 1));
      th.join();
    } else {
      r = exec(*cur, c0, m, S);
    }
    if (r < 0) fail = true;
    else ok += r;
    cur = std::move(next);
  }
  return fail ? -1 : ok;
}

long NodeStore::set_batch(const char* keys, int kstride, const uint8_t* vals, int vstride, const uint32_t* lens,
                          long n, int32_t* status, int retries) {
  const int nsh = nshards();
  BatchTrace tr("set", n);
  const long C = chunk_for(n);
  const long ob = 0, vb = a64(C * kstride), lb = vb + a64(C * (long)vstride), sb = lb + a64(C * 4), per = sb + a64(C * 4);
  std::lock_guard<std::mutex> lk(scratch_mu_);
  auto prep = [&](long c0, long m, uint8_t* S, int slot) {
    const char* k = keys + c0 * kstride;
    const uint8_t* v = vals + c0 * (long)vstride;
    const uint32_t* l = lens + c0;
    auto pl = std::make_unique<Plan>(*this, slot, k, kstride, m, nsh);
    tr.mark(0);
    uint8_t* sk = S + ob;
    uint8_t* sv = S + vb;
    uint32_t* sl = (uint32_t*)(S + lb);
    pl->place([&](long i, long q) {
      copy_row(sk + q * kstride, (const uint8_t*)k + i * kstride, kstride);
      copy_row(sv + q * (long)vstride, v + i * (long)vstride, vstride);
      sl[q] = l[i];
    });
    tr.mark(1);
    return pl;
  };
  auto exec = [&](const Plan& pl, long c0, long, uint8_t* S) -> long {
    std::atomic<bool> fail{false};
    std::atomic<long> ok{0};
    pl.each_shard([&](int j, long o, long m) {
      StoreBase* sh = at(j);
      const char* k = (const char*)S + ob + o * kstride;
      const uint8_t* v = S + vb + o * (long)vstride;
      const uint32_t* l = (const uint32_t*)(S + lb) + o;
      int32_t* st = (int32_t*)(S + sb) + o;
      long r = sh->set_batch(k, kstride, v, vstride, l, m, st, retries);
      if (r == kNoBatch) r = generic_set_batch(sh, k, kstride, v, vstride, l, m, st, retries, 4);
      if (r < 0) fail = true;
      else ok += r;
    });
    if (fail) return -1;
    if (status) pl.scatter(status + c0, S + sb, 4);
    return ok.load();
  };
  const long r = pipeline(n, per, prep, exec);
  tr.mark(2);
  return r;
}

long NodeStore::get_batch(const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens, long n,
                          int32_t* status, int retries) {
  const int nsh = nshards();
  BatchTrace tr("get", n);
  const long C = chunk_for(n);
  const long ob = 0, sb = a64(C * kstride), lb = sb + a64(C * 4), vb = lb + a64(C * 4);
  const long per = vb + (out ? a64(C * (long)ostride) : 0);
  std::lock_guard<std::mutex> lk(scratch_mu_);
  auto prep = [&](long c0, long m, uint8_t* S, int slot) {
    const char* k = keys + c0 * kstride;
    auto pl = std::make_unique<Plan>(*this, slot, k, kstride, m, nsh);
    tr.mark(0);
    uint8_t* sk = S + ob;
    pl->place([&](long i, long q) { copy_row(sk + q * kstride, (const uint8_t*)k + i * kstride, kstride); });
    tr.mark(1);
    return pl;
  };
  auto exec = [&](const Plan& pl, long c0, long, uint8_t* S) -> long {
    std::atomic<bool> fail{false};
    std::atomic<long> ok{0};
    pl.each_shard([&](int j, long o, long m) {
      StoreBase* sh = at(j);
      const char* k = (const char*)S + ob + o * kstride;
      uint8_t* v = out ? S + vb + o * (long)ostride : nullptr;
      uint32_t* l = (uint32_t*)(S + lb) + o;
      int32_t* st = (int32_t*)(S + sb) + o;
      long r = sh->get_batch(k, kstride, v, ostride, l, m, st, retries);
      if (r == kNoBatch) r = generic_get_batch(sh, k, kstride, v, ostride, l, m, st, retries, 4);
      if (r < 0) fail = true;
      else ok += r;
    });
    if (fail) return -1;
    if (status) pl.scatter(status + c0, S + sb, 4);
    if (out_lens) pl.scatter(out_lens + c0, S + lb, 4);
    if (out) pl.scatter(out + c0 * (long)ostride, S + vb, ostride);
    return ok.load();
  };
  const long r = pipeline(n, per, prep, exec);
  tr.mark(2);
  return r;
}

long NodeStore::intop_batch(const char* keys, int kstride, const int* ops, const uint64_t* masks, long n,
                            int32_t* status, uint64_t* results) {
  const int nsh = nshards();
  BatchTrace tr("intop", n);
  std::lock_guard<std::mutex> lk(scratch_mu_);
  Plan pl(*this, 0, keys, kstride, n, nsh);
  tr.mark(0);
  const long kb = 0, pb = a64(n * kstride), mb = pb + a64(n * 4), sb = mb + a64(n * 8), rb = sb + a64(n * 4);
  uint8_t* S = scratch((size_t)(rb + a64(n * 8)));
  if (!S) return -1;
  uint8_t* sk = S + kb;
  int* sp = (int*)(S + pb);
  uint64_t* sm = (uint64_t*)(S + mb);
  pl.place([&](long i, long q) {
    copy_row(sk + q * kstride, (const uint8_t*)keys + i * kstride, kstride);
    sp[q] = ops[i];
    sm[q] = masks ? masks[i] : 0;
  });
  tr.mark(1);
  std::atomic<bool> fail{false};
  std::atomic<long> ok{0};
  pl.each_shard([&](int j, long o, long m) {
    StoreBase* sh = at(j);
    const char* k = (const char*)S + kb + o * kstride;
    const int* op = (const int*)(S + pb) + o;
    const uint64_t* mk = (const uint64_t*)(S + mb) + o;
    int32_t* st = (int32_t*)(S + sb) + o;
    uint64_t* rs = results ? (uint64_t*)(S + rb) + o : nullptr;
    long r = sh->intop_batch(k, kstride, op, mk, m, st, rs);
    if (r == kNoBatch) r = generic_intop_batch(sh, k, kstride, op, mk, m, st, rs, 4);
    if (r < 0) fail = true;
    else ok += r;
  });
  tr.mark(2);
  if (fail) return -1;
  if (status) pl.scatter(status, S + sb, 4);
  if (results) pl.scatter(results, S + rb, 8);
  tr.mark(3);
  return ok.load();
}

long NodeStore::set_embedding_batch(const char* keys, int kstride, const float* vecs, long n, int32_t* status) {
  const int nsh = nshards();
  BatchTrace tr("set_embedding", n);
  std::lock_guard<std::mutex> lk(scratch_mu_);
  Plan pl(*this, 0, keys, kstride, n, nsh);
  tr.mark(0);
  const long kb = 0, vb = a64(n * kstride), sb = vb + n * (long)kEmbedBytes;
  uint8_t* S = scratch((size_t)(sb + a64(n * 4)));
  if (!S) return -1;
  uint8_t* sk = S + kb;
  uint8_t* sv = S + vb;
  pl.place([&](long i, long q) {
    copy_row(sk + q * kstride, (const uint8_t*)keys + i * kstride, kstride);
    std::memcpy(sv + q * (long)kEmbedBytes, (const uint8_t*)vecs + i * (long)kEmbedBytes, kEmbedBytes);
  });
  tr.mark(1);
  std::atomic<bool> fail{false};
  std::atomic<long> ok{0};
  pl.each_shard([&](int j, long o, long m) {
    StoreBase* sh = at(j);
    const char* k = (const char*)S + kb + o * kstride;
    const float* v = (const float*)(S + vb + o * (long)kEmbedBytes);
    int32_t* st = (int32_t*)(S + sb) + o;
    long r = sh->set_embedding_batch(k, kstride, v, m, st);
    if (r == kNoBatch) r = generic_set_embedding_batch(sh, k, kstride, v, m, nullptr, st, 4);
    if (r < 0) fail = true;
    else ok += r;
  });
  tr.mark(2);
  if (fail) return -1;
  if (status) pl.scatter(status, S + sb, 4);
  tr.mark(3);
  return ok.load();
}

}  // namespace spl

using spl::NodeDesc;
using spl::NodeStore;

extern "C" {

// A rank's shard joins node NAME (the shard store itself -- node_shard_name(NAME, shard, backend)
// -- is created by the caller first).  The first rank creates the node descriptor; every rank must
// pass the same geometry.  0 on success, -1 with errno.
int spl_node_join_ex(const char* name, int shard, int nshards, unsigned backend, size_t slots_per_shard,
                     size_t max_val, unsigned stride, unsigned flags);
int spl_node_join(const char* name, int shard, int nshards, unsigned backend, size_t slots_per_shard, size_t max_val,
                  unsigned stride) {
  return spl_node_join_ex(name, shard, nshards, backend, slots_per_shard, max_val, stride, backend == 1 ? 1u : 0u);
}

// flags SPL_NODE_OWNED (1): the shard is served only while this process lives (HBM shards always are:
// spl_node_join sets it for them); a host shard joined without it outlives its rank like any shm store
int spl_node_join_ex(const char* name, int shard, int nshards, unsigned backend, size_t slots_per_shard,
                     size_t max_val, unsigned stride, unsigned flags) {
  if (!name || shard < 0 || nshards < 1 || nshards > spl::kNodeMaxShards || shard >= nshards || backend > 1 ||
      slots_per_shard == 0 || slots_per_shard > UINT32_MAX || max_val == 0 || max_val > UINT32_MAX ||
      (stride != spl::kSlotCoreBytes && stride != spl::kSlotEmbedBytes)) {
    errno = EINVAL;
    return -1;
  }
  int err = 0;
  bool fresh = false;
  NodeDesc* d = spl::map_desc(name, true, false, &fresh, &err);
  if (!d) { errno = err; return -1; }
  if (fresh) {
    d->nshards = (uint32_t)nshards;
    d->backend = backend;
    d->slots_per_shard = (uint32_t)slots_per_shard;
    d->max_val = (uint32_t)max_val;
    d->stride = stride;
    d->event_fd = -1;
    d->version = 1;
    __atomic_store_n(&d->magic, spl::kNodeMagic, __ATOMIC_RELEASE);
  } else if (!spl::wait_magic(d, 5000)) {
    spl::unmap_desc(d);
    errno = ETIMEDOUT;
    return -1;
  }
  if (d->nshards != (uint32_t)nshards || d->backend != backend || d->slots_per_shard != slots_per_shard ||
      d->max_val != max_val || d->stride != stride) {
    spl::unmap_desc(d);
    errno = EINVAL;
    return -1;
  }
  // ownership: this process serves the shard from now on; a re-join (a restarted rank) moves the
  // generation, so open node stores re-open the shard (NodeStore::refresh)
  __atomic_store_n(&d->shard_flags[shard], (flags | (backend == 1 ? 1u : 0u)) & spl::kShardOwned, __ATOMIC_RELEASE);
  __atomic_store_n(&d->shard_pid[shard], (int32_t)getpid(), __ATOMIC_RELEASE);
  __atomic_fetch_add(&d->shard_gen[shard], 1u, __ATOMIC_ACQ_REL);
  __atomic_fetch_or(&d->ready_mask, 1ull << shard, __ATOMIC_ACQ_REL);
  spl::unmap_desc(d);
  return 0;
}

// The shard leaves; the last one out removes the node descriptor.
int spl_node_leave(const char* name, int shard) {
  if (!name || shard < 0 || shard >= spl::kNodeMaxShards) { errno = EINVAL; return -1; }
  int err = 0;
  NodeDesc* d = spl::map_desc(name, false, false, nullptr, &err);
  if (!d) { errno = err; return -1; }
  const uint64_t left = __atomic_and_fetch(&d->ready_mask, ~(1ull << shard), __ATOMIC_ACQ_REL);
  spl::unmap_desc(d);
  if (left == 0) shm_unlink((std::string(name) + ".node").c_str());
  return 0;
}

// shard store name (with backend prefix) of shard i of a node; length written, -1 if cap too small
int spl_node_shard_name(const char* name, int shard, unsigned backend, char* out, size_t cap) {
  if (!name || !out) return -1;
  const std::string s = spl::node_shard_name(name, shard, backend);
  if (s.size() + 1 > cap) return -1;
  std::memcpy(out, s.c_str(), s.size() + 1);
  return (int)s.size();
}

// shards of an open node store (-1 if `h` is not one) and their handles
int spl_node_nshards(spl_store* h) {
  auto* n = dynamic_cast<NodeStore*>((spl::StoreBase*)h);
  return n ? n->nshards() : -1;
}
spl_store* spl_node_shard(spl_store* h, int i) {
  auto* n = dynamic_cast<NodeStore*>((spl::StoreBase*)h);
  return n ? (spl_store*)n->shard(i) : nullptr;
}
// Checkpoint / restore of any store (the unit a restarted rank recovers from): a host store writes
// its mapped v4 image to `path` (tmp + rename), an hbm: store streams its device image
// (spl_hbm_checkpoint), a node store checkpoints every serving shard to PATH.s<i>.  Restore loads
// such an image into an OPEN store of the same geometry -- exclusive: no other process may use the
// store meanwhile (a restarting rank restores before it joins).  0 on success, -1 with errno.
static int host_checkpoint(spl::HostStore* hs, const char* path) {
  const std::string tmp = std::string(path) + ".tmp";
  const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) return -1;
  const uint8_t* p = hs->base();
  size_t left = hs->total_bytes();
  while (left) {
    const ssize_t w = ::write(fd, p, left);
    if (w <= 0) {
      const int e = errno;
      ::close(fd);
      ::unlink(tmp.c_str());
      errno = e;
      return -1;
    }
    p += w;
    left -= (size_t)w;
  }
  if (::fsync(fd) != 0 || ::close(fd) != 0 || ::rename(tmp.c_str(), path) != 0) return -1;
  return 0;
}

static int host_restore(spl::HostStore* hs, const char* path) {
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size != hs->total_bytes()) {
    ::close(fd);
    errno = EINVAL;  // another geometry
    return -1;
  }
  std::vector<uint8_t> img(hs->total_bytes());
  size_t got = 0;
  while (got < img.size()) {
    const ssize_t r = ::read(fd, img.data() + got, img.size() - got);
    if (r <= 0) {
      ::close(fd);
      errno = EIO;
      return -1;
    }
    got += (size_t)r;
  }
  ::close(fd);
  const auto* H = (const splinter_header*)img.data();
  const spl::Geometry g = hs->geometry();
  if (H->magic != spl::kMagic || H->version != spl::kVersion || H->slots != g.slots || H->max_val_sz != g.max_val) {
    errno = EINVAL;
    return -1;
  }
  std::memcpy(hs->base(), img.data(), img.size());
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  return 0;
}

int spl_store_checkpoint(spl_store* h, const char* path) {
  auto* b = (spl::StoreBase*)h;
  if (!b || !path) { errno = EINVAL; return -1; }
  if (auto* hs = dynamic_cast<spl::HostStore*>(b)) return host_checkpoint(hs, path);
  if (auto* n = dynamic_cast<NodeStore*>(b)) {
    for (int i = 0; i < n->nshards(); ++i) {
      if (n->shard_state(i) != 0) continue;  // a down shard keeps its last checkpoint
      const std::string p = std::string(path) + ".s" + std::to_string(i);
      if (spl_store_checkpoint((spl_store*)n->shard(i), p.c_str()) != 0) return -1;
    }
    return 0;
  }
  using Fn = int (*)(spl_store*, const char*);
  static Fn f = (Fn)spl::hbm_symbol("spl_hbm_checkpoint");
  if (!f) { errno = ENOSYS; return -1; }
  return f(h, path);
}

int spl_store_restore(spl_store* h, const char* path) {
  auto* b = (spl::StoreBase*)h;
  if (!b || !path) { errno = EINVAL; return -1; }
  if (auto* hs = dynamic_cast<spl::HostStore*>(b)) return host_restore(hs, path);
  if (dynamic_cast<NodeStore*>(b)) { errno = ENOTSUP; return -1; }  // per shard, by the shard's rank
  using Fn = int (*)(spl_store*, const char*);
  static Fn f = (Fn)spl::hbm_symbol("spl_hbm_restore");
  if (!f) { errno = ENOSYS; return -1; }
  return f(h, path);
}

// state of shard i of an open node store: 0 serving, 1 down (its rank's process is gone; ops on its
// keys return EAGAIN until the rank re-joins), -1 not a node store / no such shard
int spl_node_shard_state(spl_store* h, int i) {
  auto* n = dynamic_cast<NodeStore*>((spl::StoreBase*)h);
  return n ? n->shard_state(i) : -1;
}

// owning shard of a key under an n-way node (== parallel/sharded.py shard_of)
int spl_node_shard_of(const char* key, int nshards) {
  if (!key || nshards < 1) return -1;
  return spl::node_shard_of(spl::KeyRef(key).hash, nshards);
}

}  // extern "C"
