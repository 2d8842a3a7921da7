// store_host.cpp — the host (mmap) backend of libsplinter_amd.
//
// Serves POSIX shm objects ("name") and regular files (paths / "file:") with
// the exact format-v4 layout, so reference-built processes and ours can share
// one mapping.  Semantics follow the reference API contract
// (/root/reference/splinter.c) with the race fixes listed in
// docs/DIVERGENCES.md:
//   * probe chains end at a virgin slot (hash 0 && epoch 0) instead of scanning
//     all N slots on every miss (reference splinter.c:437-463);
//   * inserts claim by epoch CAS and then re-validate the chain, so two racing
//     writers of one key cannot create duplicates (reference splinter.c:377-384);
//   * reads compare the key inside the seqlock window (no ABA across
//     unset/re-insert);
//   * unset never passes through epoch 0 (a transient "virgin" would end probe
//     chains early); the final epoch is still 2 as in the reference.
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fcntl.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "store_host.hpp"

namespace spl {

// ---------------------------------------------------------------- atomics --
template <class T> static inline T ld(const T* p, int mo = __ATOMIC_ACQUIRE) { return __atomic_load_n(p, mo); }
template <class T> static inline void st(T* p, T v, int mo = __ATOMIC_RELEASE) { __atomic_store_n(p, v, mo); }
static inline bool cas64(uint64_t* p, uint64_t expect, uint64_t want) {
  return __atomic_compare_exchange_n(p, &expect, want, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
}
static inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#elif defined(__aarch64__)
  __asm__ __volatile__("yield");
#endif
}
static inline void fence_acq() { __atomic_thread_fence(__ATOMIC_ACQUIRE); }
static inline void fence_rel() { __atomic_thread_fence(__ATOMIC_RELEASE); }

// Payload copies under the seqlock are racy BY DESIGN (a reader may copy while a
// writer writes; the epoch re-check discards such reads).  TSAN builds route them
// through an uninstrumented volatile copy so the race detector reports only races
// outside the protocol (SURVEY §5 race detection); normal builds use memcpy.
#if defined(__SANITIZE_THREAD__)
__attribute__((no_sanitize_thread, noinline)) static void seq_copy(void* dst, const void* src, size_t n) {
  volatile unsigned char* d = (volatile unsigned char*)dst;
  const volatile unsigned char* s = (const volatile unsigned char*)src;
  for (size_t i = 0; i < n; ++i) d[i] = s[i];
}
#else
static inline void seq_copy(void* dst, const void* src, size_t n) { std::memcpy(dst, src, n); }
#endif

uint64_t now_ticks() {
#if defined(__x86_64__) || defined(__i386__)
  uint32_t lo, hi;
  __asm__ __volatile__("rdtsc" : "=a"(lo), "=d"(hi));
  return ((uint64_t)hi << 32) | lo;
#elif defined(__aarch64__)
  uint64_t v;
  __asm__ __volatile__("mrs %0, cntvct_el0" : "=r"(v));
  return v;
#else
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC_RAW, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
#endif
}

KeyRef::KeyRef(const char* k) {
  std::memset(buf, 0, sizeof(buf));
  len = 0;
  if (k) {
    while (len < kKeyMax - 1 && k[len]) { buf[len] = k[len]; ++len; }
  }
  hash = fnv1a_n(buf, len);
}

// ------------------------------------------------------------ lifecycle --
mode_t env_umask_push() {
  const char* env = getenv("SPLINTER_DEFAULT_UMASK");
  if (!env || !*env) return (mode_t)-1;
  char* end = nullptr;
  errno = 0;
  long v = strtol(env, &end, 8);
  if (errno || end == env || *end || v < 0 || v > 0777) return (mode_t)-1;
  return umask((mode_t)v);
}
void env_umask_pop(mode_t prev) { if (prev != (mode_t)-1) umask(prev); }

HostStore::~HostStore() {
  if (event_fd_ >= 0) close(event_fd_);
  if (base_) munmap(base_, total_);
}

HostStore* HostStore::create(const char* name, bool file_backed, size_t slots, size_t max_val,
                             bool embeddings, int* err) {
  *err = 0;
  if (slots == 0 || max_val == 0 || slots > UINT32_MAX || max_val > UINT32_MAX) {
    *err = ENOTSUP;
    return nullptr;
  }
  Geometry g;
  g.slots = (uint32_t)slots;
  g.max_val = (uint32_t)max_val;
  g.stride = embeddings ? (uint32_t)kSlotEmbedBytes : (uint32_t)kSlotCoreBytes;
  const size_t total = g.total_bytes();

  mode_t prev = env_umask_push();
  int fd = file_backed ? ::open(name, O_RDWR | O_CREAT | O_EXCL | O_NOFOLLOW | O_CLOEXEC, 0666)
                       : shm_open(name, O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0666);
  env_umask_pop(prev);
  if (fd < 0) { *err = errno; return nullptr; }
  if (ftruncate(fd, (off_t)total) != 0) {
    *err = errno;
    close(fd);
    return nullptr;
  }
  void* base = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base == MAP_FAILED) { *err = errno; return nullptr; }

  auto* s = new HostStore();
  s->base_ = (uint8_t*)base;
  s->total_ = total;
  s->geo_ = g;
  s->file_backed_ = file_backed;
  s->H_ = (splinter_header*)base;
  s->init_fresh();
  return s;
}

void HostStore::init_fresh() {
  // A fresh ftruncate()d region is zero-filled: only non-zero defaults need
  // writing.  Slot val_off keeps the reference's (u32) i*max_val value for
  // interop; this library always addresses values by slot index (64-bit).
  splinter_header* h = H_;
  h->magic = kMagic;
  h->version = kVersion;
  h->slots = geo_.slots;
  h->max_val_sz = geo_.max_val;
  h->val_sz = (uint32_t)total_;
  h->alignment = geo_.stride;
  st(&h->epoch, (uint64_t)1, __ATOMIC_RELAXED);
  st(&h->core_flags, (uint8_t)(SPL_SYS_AUTO_SCRUB | SPL_SYS_HYBRID_SCRUB), __ATOMIC_RELAXED);
  std::memset(h->bloom_watches, 0xFF, sizeof(h->bloom_watches));
  h->event_bus.owner_fd = -1;
  h->event_bus.owner_pid = 0;
  for (uint32_t i = 0; i < geo_.slots; ++i) {
    splinter_slot* s = slot(i);
    s->type_flag = SPL_SLOT_DEFAULT_TYPE;
    s->val_off = (uint32_t)((size_t)i * geo_.max_val);
  }
  fence_rel();
}

HostStore* HostStore::open(const char* name, bool file_backed, int* err) {
  *err = 0;
  int fd = file_backed ? ::open(name, O_RDWR | O_CLOEXEC) : shm_open(name, O_RDWR | O_CLOEXEC, 0666);
  if (fd < 0) { *err = errno; return nullptr; }
  struct stat sb;
  if (fstat(fd, &sb) != 0 || (size_t)sb.st_size < kHeaderBytes) {
    *err = EINVAL;
    close(fd);
    return nullptr;
  }
  const size_t total = (size_t)sb.st_size;
  void* base = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base == MAP_FAILED) { *err = errno; return nullptr; }
  auto* h = (splinter_header*)base;
  Geometry g;
  g.slots = h->slots;
  g.max_val = h->max_val_sz;
  g.stride = infer_stride(g.slots, g.max_val, total);
  if (h->magic != kMagic || h->version != kVersion || g.stride == 0) {
    munmap(base, total);
    *err = EINVAL;
    return nullptr;
  }
  auto* s = new HostStore();
  s->base_ = (uint8_t*)base;
  s->total_ = total;
  s->geo_ = g;
  s->file_backed_ = file_backed;
  s->H_ = h;
  return s;
}

// -------------------------------------------------------------- helpers --
bool HostStore::key_eq(const splinter_slot* s, const KeyRef& k) const {
  return std::strncmp(s->key, k.buf, kKeyMax) == 0;
}

long HostStore::find(const KeyRef& k) const {
  const uint32_t n = geo_.slots;
  size_t idx = (size_t)(k.hash % n);
  for (uint32_t i = 0; i < n; ++i) {
    splinter_slot* s = slot(idx);
    uint64_t sh = ld(&s->hash);
    if (sh == k.hash && key_eq(s, k)) return (long)idx;
    if (sh == 0 && ld(&s->epoch, __ATOMIC_RELAXED) == 0) return -1;  // virgin: chain ends
    if (++idx == n) idx = 0;
  }
  return -1;
}

void HostStore::notify(size_t idx) {
  if (event_fd_ < 0) return;
  const size_t m = idx % kDirtyBits;
  __atomic_fetch_or(&H_->event_bus.dirty_mask[m / 64], 1ull << (m % 64), __ATOMIC_RELEASE);
  uint64_t one = 1;
  ssize_t w = write(event_fd_, &one, sizeof(one));
  (void)w;
}

void HostStore::pulse_slot(splinter_slot* s) {
  const uint64_t wm = ld(&s->watcher_mask);
  for (uint64_t m = wm; m; m &= m - 1) {
    int g = __builtin_ctzll(m);
    __atomic_fetch_add(&H_->signal_groups[g].counter, 1, __ATOMIC_RELEASE);
  }
  const uint64_t bl = ld(&s->bloom, __ATOMIC_RELAXED);
  for (uint64_t m = bl; m; m &= m - 1) {
    int b = __builtin_ctzll(m);
    uint8_t g = ld(&H_->bloom_watches[b]);
    if (g < SPLINTER_MAX_GROUPS) __atomic_fetch_add(&H_->signal_groups[g].counter, 1, __ATOMIC_RELEASE);
  }
}

void HostStore::bump_global(uint64_t n) { __atomic_fetch_add(&H_->epoch, n, __ATOMIC_RELAXED); }

bool HostStore::scrub_on() const { return (ld(&H_->core_flags, __ATOMIC_RELAXED) & SPL_SYS_AUTO_SCRUB) != 0; }
bool HostStore::hybrid_on() const { return (ld(&H_->core_flags, __ATOMIC_RELAXED) & SPL_SYS_HYBRID_SCRUB) != 0; }

// ---------------------------------------------------------- store-wide --
int HostStore::set_mop(unsigned mode) {
  switch (mode) {
    case 0: __atomic_fetch_and(&H_->core_flags, (uint8_t)~(SPL_SYS_AUTO_SCRUB | SPL_SYS_HYBRID_SCRUB), __ATOMIC_ACQ_REL); return 0;
    case 1: __atomic_fetch_or(&H_->core_flags, (uint8_t)(SPL_SYS_AUTO_SCRUB | SPL_SYS_HYBRID_SCRUB), __ATOMIC_ACQ_REL); return 0;
    // Reference quirk kept: mode 2 sets AUTO without clearing HYBRID.
    case 2: __atomic_fetch_or(&H_->core_flags, (uint8_t)SPL_SYS_AUTO_SCRUB, __ATOMIC_ACQ_REL); return 0;
    default: errno = EOPNOTSUPP; return -1;
  }
}

int HostStore::get_mop() {
  uint8_t f = ld(&H_->core_flags);
  if (f & SPL_SYS_HYBRID_SCRUB) return 1;
  if (f & SPL_SYS_AUTO_SCRUB) return 2;
  return 0;
}

void HostStore::purge() {
  for (uint32_t i = 0; i < geo_.slots; ++i) {
    splinter_slot* s = slot(i);
    uint64_t e = ld(&s->epoch);
    if (e & 1) continue;
    const uint64_t sh = ld(&s->hash);
    if (sh == 0 && e == 0) continue;  // virgin slots are already zero; keep them virgin
    if (!cas64(&s->epoch, e, e + 1)) continue;
    const uint32_t len = ld(&s->val_len, __ATOMIC_RELAXED);
    uint8_t* dst = value(i);
    if (ld(&s->hash) == 0) std::memset(dst, 0, geo_.max_val);
    else if (len < geo_.max_val) std::memset(dst + len, 0, geo_.max_val - len);
    __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
  }
}

int HostStore::header_snapshot(splinter_header_snapshot_t* o) {
  if (!o) return -2;
  o->magic = H_->magic;
  o->version = H_->version;
  o->slots = H_->slots;
  o->max_val_sz = H_->max_val_sz;
  o->core_flags = ld(&H_->core_flags);
  o->user_flags = ld(&H_->user_flags);
  o->epoch = ld(&H_->epoch);
  o->parse_failures = ld(&H_->parse_failures, __ATOMIC_RELAXED);
  o->last_failure_epoch = ld(&H_->last_failure_epoch, __ATOMIC_RELAXED);
  return 0;
}

uint8_t HostStore::config_get() { return ld(&H_->core_flags); }
void HostStore::config_or(uint8_t m) { __atomic_fetch_or(&H_->core_flags, m, __ATOMIC_ACQ_REL); }
void HostStore::config_and(uint8_t m) { __atomic_fetch_and(&H_->core_flags, m, __ATOMIC_ACQ_REL); }

// ------------------------------------------------------------ key/value --
int HostStore::write_locked(size_t idx, const KeyRef& k, const void* val, size_t len, bool fresh) {
  splinter_slot* s = slot(idx);
  uint8_t* dst = value(idx);
  if (scrub_on()) {
    size_t n = geo_.max_val;
    if (hybrid_on()) {
      n = (len + 63) & ~(size_t)63;
      if (n > geo_.max_val) n = geo_.max_val;
    }
    std::memset(dst, 0, n);
  }
  seq_copy(dst, val, len);
  st(&s->val_len, (uint32_t)len);
  if (fresh) {
    if (geo_.embeddings()) std::memset(embedding(idx), 0, kEmbedBytes);
    seq_copy(s->key, k.buf, kKeyMax);  // NUL-padded canonical key
  }
  fence_rel();
  st(&s->hash, k.hash);
  __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
  pulse_slot(s);
  bump_global(1);
  notify(idx);
  return 0;
}

int HostStore::set(const char* key, const void* val, size_t len) {
  if (!key) return -2;
  if (len == 0 || len > geo_.max_val) { errno = len ? EMSGSIZE : EINVAL; return -1; }
  if (!val) return -2;
  const KeyRef k(key);
  const uint32_t n = geo_.slots;
  const size_t home = (size_t)(k.hash % n);

  // Pass 1: locate the key or the first reusable slot on its chain.
  long free_idx = -1;
  uint64_t free_epoch = 0;
  size_t idx = home;
  for (uint32_t i = 0; i < n; ++i) {
    splinter_slot* s = slot(idx);
    // epoch BEFORE hash: a writer stores the hash and then bumps the epoch, so an even
    // epoch read first guarantees the hash read after it is at least that new
    const uint64_t e = ld(&s->epoch);
    const uint64_t sh = ld(&s->hash);
    if (sh == k.hash && key_eq(s, k)) {
      // update in place
      if (e & 1) { errno = EAGAIN; return -1; }
      if (!cas64(&s->epoch, e, e + 1)) { errno = EAGAIN; return -1; }
      if (ld(&s->hash) != k.hash || !key_eq(s, k)) {  // lost a race with unset
        __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
        errno = EAGAIN;
        return -1;
      }
      return write_locked(idx, k, val, len, false);
    }
    if ((e & 1) && sh == k.hash) { errno = EAGAIN; return -1; }  // our key is being rewritten
    if (sh == 0 && !(e & 1)) {  // reusable slot (odd = another writer's claim: skip it)
      if (free_idx < 0) { free_idx = (long)idx; free_epoch = e; }
      if (e == 0) break;  // virgin: end of chain
    }
    if (++idx == n) idx = 0;
  }
  if (free_idx < 0) { errno = ENOSPC; return -1; }

  // Claim the free slot, then re-validate the chain while holding it.
  splinter_slot* fs = slot((size_t)free_idx);
  if (!cas64(&fs->epoch, free_epoch, free_epoch + 1)) { errno = EAGAIN; return -1; }
  if (ld(&fs->hash) != 0) {
    __atomic_fetch_add(&fs->epoch, 1, __ATOMIC_RELEASE);
    errno = EAGAIN;
    return -1;
  }
  // Re-validate the chain while holding the claim.  The claim CAS is a full barrier,
  // so of two racing inserters at least one sees the other's claim here (Dekker);
  // "the earlier claimant on the chain wins" alone is NOT enough: the earlier one may
  // miss the later one's claim's resolution order (see docs/DIVERGENCES.md), so:
  //   * the key published anywhere on the chain, or a claim in flight EARLIER on the
  //     chain (possibly our key)             -> back off (EAGAIN);
  //   * a claim in flight LATER on the chain -> wait for it to resolve (it never waits
  //     for us: it either sees our earlier claim and backs off, or publishes its key,
  //     which we then see and back off from), then re-check that slot.
  idx = home;
  bool before = true;
  for (uint32_t i = 0; i < n; ++i) {
    if ((long)idx == free_idx) {
      before = false;
    } else {
      splinter_slot* s = slot(idx);
      uint64_t e = ld(&s->epoch);
      uint64_t sh = ld(&s->hash);
      if (!before && (e & 1) && (sh == 0 || sh == k.hash)) {
        for (uint32_t spin = 0; spin < (1u << 20) && ld(&s->epoch) == e; ++spin) cpu_relax();
        e = ld(&s->epoch);
        sh = ld(&s->hash);
      }
      const bool mine = sh == k.hash && key_eq(s, k);
      if (mine || ((e & 1) && (sh == 0 || sh == k.hash))) {
        __atomic_fetch_add(&fs->epoch, 1, __ATOMIC_RELEASE);
        errno = EAGAIN;
        return -1;
      }
      if (sh == 0 && e == 0) break;
    }
    if (++idx == n) idx = 0;
  }
  return write_locked((size_t)free_idx, k, val, len, true);
}

int HostStore::unset(const char* key) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  uint64_t e = ld(&s->epoch);
  if (e & 1) { errno = EAGAIN; return -1; }
  if (!cas64(&s->epoch, e, e + 1)) { errno = EAGAIN; return -1; }
  if (ld(&s->hash) != k.hash || !key_eq(s, k)) {
    __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
    return -1;
  }
  const int old_len = (int)ld(&s->val_len);
  st(&s->hash, (uint64_t)0);
  if (scrub_on()) {
    std::memset(value((size_t)i), 0, geo_.max_val);
    std::memset(s->key, 0, kKeyMax);
  } else {
    s->key[0] = '\0';
  }
  st(&s->type_flag, (uint8_t)SPL_SLOT_DEFAULT_TYPE);
  st(&s->val_len, (uint32_t)0);
  if (geo_.embeddings()) std::memset(embedding((size_t)i), 0, kEmbedBytes);
  st(&s->ctime, (uint64_t)0);
  st(&s->atime, (uint64_t)0);
  st(&s->user_flag, (uint8_t)0);
  st(&s->watcher_mask, (uint64_t)0);
  st(&s->bloom, (uint64_t)0);
  fence_rel();
  st(&s->epoch, (uint64_t)2);  // reference contract: unset rewinds the epoch to 2
  return old_len;
}

int HostStore::get(const char* key, void* buf, size_t buf_sz, size_t* out_sz) {
  if (!key) return -2;
  const KeyRef k(key);
  const uint32_t n = geo_.slots;
  size_t idx = (size_t)(k.hash % n);
  for (uint32_t i = 0; i < n; ++i) {
    splinter_slot* s = slot(idx);
    const uint64_t sh = ld(&s->hash);
    if (sh == k.hash) {
      const uint64_t e1 = ld(&s->epoch);
      if (key_eq(s, k)) {
        if (e1 & 1) { errno = EAGAIN; return -1; }
        const size_t len = ld(&s->val_len);
        if (out_sz) *out_sz = len;
        if (buf) {
          if (buf_sz < len) { errno = EMSGSIZE; return -1; }
          seq_copy(buf, value(idx), len);
        }
        fence_acq();
        const uint64_t e2 = ld(&s->epoch);
        if (e1 == e2 && ld(&s->hash, __ATOMIC_RELAXED) == k.hash) return 0;
        errno = EAGAIN;
        return -1;
      }
    } else if (sh == 0 && ld(&s->epoch, __ATOMIC_RELAXED) == 0) {
      break;
    }
    if (++idx == n) idx = 0;
  }
  errno = ENOENT;
  return -1;
}

int HostStore::list(char** out, size_t max, size_t* cnt) {
  if (!out || !cnt) return -2;
  size_t c = 0;
  for (uint32_t i = 0; i < geo_.slots && c < max; ++i) {
    splinter_slot* s = slot(i);
    if (ld(&s->hash) && ld(&s->val_len) > 0) out[c++] = s->key;
  }
  *cnt = c;
  return 0;
}

int HostStore::poll(const char* key, uint64_t timeout_ms) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  const uint64_t start = ld(&s->epoch);
  if (start & 1) { errno = EAGAIN; return -1; }
  timespec dl;
  clock_gettime(CLOCK_MONOTONIC, &dl);
  dl.tv_sec += (time_t)(timeout_ms / 1000);
  dl.tv_nsec += (long)(timeout_ms % 1000) * 1000000L;
  if (dl.tv_nsec >= 1000000000L) { dl.tv_nsec -= 1000000000L; dl.tv_sec++; }
  const timespec nap = {0, 10 * 1000000L};
  for (;;) {
    const uint64_t cur = ld(&s->epoch);
    if (!(cur & 1) && cur != start) return 0;
    timespec now;
    clock_gettime(CLOCK_MONOTONIC, &now);
    if (!(cur & 1) && (now.tv_sec > dl.tv_sec || (now.tv_sec == dl.tv_sec && now.tv_nsec >= dl.tv_nsec))) {
      errno = ETIMEDOUT;
      return -1;
    }
    nanosleep(&nap, nullptr);
  }
}

int HostStore::slot_snapshot(const char* key, splinter_slot_snapshot_t* o) {
  if (!key || !o) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  for (int attempt = 0;; ++attempt) {
    const uint64_t e1 = ld(&s->epoch);
    if (e1 & 1) {
      if (attempt > 1000000) { errno = EAGAIN; return -1; }
      continue;
    }
    o->hash = ld(&s->hash);
    o->epoch = e1;
    o->val_off = s->val_off;
    o->val_len = ld(&s->val_len, __ATOMIC_RELAXED);
    o->type_flag = ld(&s->type_flag);
    o->user_flag = ld(&s->user_flag);
    o->ctime = ld(&s->ctime);
    o->atime = ld(&s->atime);
    o->bloom = ld(&s->bloom);
    seq_copy(o->key, s->key, kKeyMax);
#ifdef SPLINTER_EMBEDDINGS
    if (geo_.embeddings()) seq_copy(o->embedding, embedding((size_t)i), kEmbedBytes);
    else std::memset(o->embedding, 0, kEmbedBytes);
#endif
    fence_acq();
    if (ld(&s->epoch) == e1) return 0;
  }
}

int HostStore::append(const char* key, const void* data, size_t len, size_t* new_len) {
  if (!key || !data || len == 0) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  uint64_t e = ld(&s->epoch);
  if ((e & 1) || !cas64(&s->epoch, e, e + 1)) { errno = EAGAIN; return -1; }
  const size_t cur = ld(&s->val_len, __ATOMIC_RELAXED);
  if (cur + len > geo_.max_val) {
    __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
    errno = EMSGSIZE;
    return -1;
  }
  seq_copy(value((size_t)i) + cur, data, len);
  st(&s->val_len, (uint32_t)(cur + len));
  if (new_len) *new_len = cur + len;
  __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
  pulse_slot(s);
  bump_global(1);
  notify((size_t)i);
  return 0;
}

const void* HostStore::raw_ptr(const char* key, size_t* out_sz, uint64_t* out_epoch) {
  if (!key) return nullptr;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return nullptr;
  splinter_slot* s = slot((size_t)i);
  if (out_epoch) *out_epoch = ld(&s->epoch);
  if (out_sz) *out_sz = ld(&s->val_len, __ATOMIC_RELAXED);
  return value((size_t)i);
}

uint64_t HostStore::epoch_of(const char* key) {
  if (!key) return 0;
  const KeyRef k(key);
  long i = find(k);
  return i < 0 ? 0 : ld(&slot((size_t)i)->epoch);
}

int HostStore::set_as_system(const char* key) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  st(&s->type_flag, (uint8_t)SPL_SLOT_TYPE_BINARY);
  st(&s->val_len, geo_.max_val);
  return 0;
}

// ----------------------------------------------------------- embeddings --
int HostStore::set_embedding(const char* key, const float* vec) {
  if (!key || !vec) return -2;
  if (!geo_.embeddings()) { errno = ENOTSUP; return -1; }
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  uint64_t e = ld(&s->epoch, __ATOMIC_RELAXED);
  if ((e & 1) || !cas64(&s->epoch, e, e + 1)) { errno = EAGAIN; return -1; }
  seq_copy(embedding((size_t)i), vec, kEmbedBytes);
  fence_rel();
  __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
  bump_global(1);
  notify((size_t)i);
  return 0;
}

int HostStore::get_embedding(const char* key, float* out) {
  if (!key || !out) return -2;
  if (!geo_.embeddings()) { errno = ENOTSUP; return -1; }
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  const uint64_t e1 = ld(&s->epoch);
  if (e1 & 1) { errno = EAGAIN; return -1; }
  seq_copy(out, embedding((size_t)i), kEmbedBytes);
  fence_acq();
  if (ld(&s->epoch) == e1) return 0;
  errno = EAGAIN;
  return -1;
}

// ----------------------------------------------------- typing/time/int --
int HostStore::set_named_type(const char* key, uint16_t mask) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  uint64_t e = ld(&s->epoch, __ATOMIC_RELAXED);
  if ((e & 1) || !cas64(&s->epoch, e, e + 1)) { errno = EAGAIN; return -1; }
  const uint32_t cur = ld(&s->val_len);
  if ((mask & SPL_SLOT_TYPE_BIGUINT) && cur < 8) {
    // Promote to a u64 in place (the reference bump-allocates from val_brk,
    // which starts at 0 and aliases slot 0's value: SURVEY §2.2).
    uint8_t* v = value((size_t)i);
    uint64_t x = 0;
    if (cur > 0 && v[0] >= '0' && v[0] <= '9') {
      char tmp[16] = {0};
      std::memcpy(tmp, v, cur < 15 ? cur : 15);
      x = strtoull(tmp, nullptr, 0);
    } else {
      std::memcpy(&x, v, cur);
    }
    if (geo_.max_val < 8) {
      __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
      errno = ENOMEM;
      return -1;
    }
    std::memcpy(v, &x, 8);
    st(&s->val_len, (uint32_t)8, __ATOMIC_RELAXED);
  }
  st(&s->type_flag, (uint8_t)mask);
  __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
  bump_global(1);
  notify((size_t)i);
  return 0;
}

int HostStore::set_slot_time(const char* key, unsigned short mode, uint64_t epoch, size_t offset) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  if (ld(&s->epoch) & 1) { errno = EAGAIN; return -1; }
  if (mode == SPL_TIME_CTIME) { st(&s->ctime, epoch - offset); return 0; }
  if (mode == SPL_TIME_ATIME) { st(&s->atime, epoch - offset); return 0; }
  errno = ENOTSUP;
  return -2;
}

int HostStore::integer_op(const char* key, splinter_integer_op_t op, const void* mask) {
  if (!key) return -2;
  uint64_t m = 0;
  if (mask) std::memcpy(&m, mask, 8);
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  if (!(ld(&s->type_flag, __ATOMIC_RELAXED) & SPL_SLOT_TYPE_BIGUINT)) { errno = EPROTOTYPE; return -1; }
  uint64_t e = ld(&s->epoch, __ATOMIC_RELAXED);
  if ((e & 1) || !cas64(&s->epoch, e, e + 1)) { errno = EAGAIN; return -1; }
  uint64_t* v = (uint64_t*)value((size_t)i);
  uint64_t x;
  std::memcpy(&x, v, 8);
  switch (op) {
    case SPL_OP_AND: x &= m; break;
    case SPL_OP_OR: x |= m; break;
    case SPL_OP_XOR: x ^= m; break;
    case SPL_OP_NOT: x = ~x; break;
    case SPL_OP_INC: x += m; break;
    case SPL_OP_DEC: x -= m; break;
    default:
      __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
      errno = EINVAL;
      return -2;
  }
  std::memcpy(v, &x, 8);
  __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
  bump_global(1);
  notify((size_t)i);
  return 0;
}

// --------------------------------------------------------- epochs/labels --
int HostStore::bump(const char* key) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  uint64_t e = ld(&s->epoch, __ATOMIC_RELAXED);
  if ((e & 1) || !cas64(&s->epoch, e, e + 1)) return -1;
  fence_rel();
  pulse_slot(s);
  __atomic_fetch_add(&s->epoch, 1, __ATOMIC_RELEASE);
  return 0;
}

int HostStore::retrain(const char* key) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  splinter_slot* s = slot((size_t)i);
  st(&s->epoch, (uint64_t)3);
  fence_rel();
  if (geo_.embeddings()) std::memset(embedding((size_t)i), 0, kEmbedBytes);
  fence_rel();
  st(&s->epoch, (uint64_t)4);
  bump_global(1);
  pulse_slot(s);
  notify((size_t)i);
  return 0;
}

int HostStore::set_label(const char* key, uint64_t mask) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  __atomic_fetch_or(&slot((size_t)i)->bloom, mask, __ATOMIC_RELEASE);
  bump_global(1);
  notify((size_t)i);
  return 0;
}

int HostStore::unset_label(const char* key, uint64_t mask) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  __atomic_fetch_and(&slot((size_t)i)->bloom, ~mask, __ATOMIC_RELEASE);
  bump_global(1);
  notify((size_t)i);
  return 0;
}

// --------------------------------------------------------------- signals --
int HostStore::watch_register(const char* key, uint8_t g) {
  if (!key) return -2;
  if (g >= SPLINTER_MAX_GROUPS) { errno = EINVAL; return -2; }
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  __atomic_fetch_or(&slot((size_t)i)->watcher_mask, 1ull << g, __ATOMIC_RELEASE);
  return 0;
}

int HostStore::watch_unregister(const char* key, uint8_t g) {
  if (!key || g >= SPLINTER_MAX_GROUPS) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  __atomic_fetch_and(&slot((size_t)i)->watcher_mask, ~(1ull << g), __ATOMIC_RELEASE);
  return 0;
}

int HostStore::watch_label_register(uint64_t mask, uint8_t g) {
  if (g >= SPLINTER_MAX_GROUPS) return -2;
  for (uint64_t m = mask; m; m &= m - 1) st(&H_->bloom_watches[__builtin_ctzll(m)], g);
  return 0;
}

int HostStore::pulse_keygroup(const char* key) {
  if (!key) return -2;
  const KeyRef k(key);
  long i = find(k);
  if (i < 0) return -1;
  pulse_slot(slot((size_t)i));
  return 0;
}

uint64_t HostStore::signal_count(uint8_t g) {
  if (g >= SPLINTER_MAX_GROUPS) return 0;
  return ld(&H_->signal_groups[g].counter);
}

int HostStore::signal_add(uint8_t g, uint64_t delta) {
  if (g >= SPLINTER_MAX_GROUPS) return -2;
  __atomic_fetch_add(&H_->signal_groups[g].counter, delta, __ATOMIC_RELEASE);
  return 0;
}

void HostStore::enumerate(uint64_t mask, void (*cb)(const char*, uint64_t, void*), void* ud) {
  if (!cb) return;
  for (uint32_t i = 0; i < geo_.slots; ++i) {
    splinter_slot* s = slot(i);
    if (ld(&s->hash) != 0 && (ld(&s->bloom) & mask) == mask) cb(s->key, ld(&s->epoch, __ATOMIC_RELAXED), ud);
  }
}

// ------------------------------------------------------------- event bus --
int HostStore::event_bus_init() { return event_bus_install(eventfd(0, EFD_CLOEXEC)); }

int HostStore::event_bus_adopt(int fd) { return event_bus_install(fcntl(fd, F_DUPFD_CLOEXEC, 0)); }

int HostStore::event_bus_install(int fd) {
  if (fd < 0) return -1;
  if (event_fd_ >= 0) close(event_fd_);
  event_fd_ = fd;
  st(&H_->event_bus.owner_fd, (int32_t)fd);
  st(&H_->event_bus.owner_pid, (int32_t)getpid());
  return 0;
}

int HostStore::event_bus_open() {
  const int32_t fd = ld(&H_->event_bus.owner_fd);
  const int32_t pid = ld(&H_->event_bus.owner_pid);
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

void HostStore::event_bus_dirty(uint64_t* out, size_t words) {
  if (!out) return;
  const size_t n = words < SPLINTER_EVENT_BUS_MASK_WORDS ? words : SPLINTER_EVENT_BUS_MASK_WORDS;
  for (size_t i = 0; i < n; ++i) out[i] = ld(&H_->event_bus.dirty_mask[i]);
}

// ------------------------------------------------------------ shards --
int HostStore::shard_claim_ex(uint32_t id, uint32_t pid, uint8_t intent, uint8_t prio, uint64_t dur, uint64_t at) {
  return shard_claim_on(H_, id, pid, intent, prio, dur, at);
}
int HostStore::shard_rebid(uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur) {
  return shard_rebid_on(H_, id, intent, prio, dur);
}
int HostStore::shard_release(uint32_t id) { return shard_release_on(H_, id); }
uint32_t HostStore::shard_election(uint8_t* out_intent) { return shard_election_on(H_, out_intent); }
int HostStore::shard_table(splinter_shard_bid_snapshot* out, size_t max) { return shard_table_on(H_, out, max); }

int HostStore::madvise(uint32_t id, void* addr, size_t len, int advice, uint64_t timeout) {
  if (id == 0) { errno = EINVAL; return -2; }
  if (!shard_present_on(H_, id)) { errno = EINVAL; return -2; }
  if (!addr) {
    addr = base_ + geo_.values_offset();
    len = geo_.values_bytes();
  }
  const long pg = sysconf(_SC_PAGESIZE);
  if (pg > 0) {
    uintptr_t a = (uintptr_t)addr, al = a & ~((uintptr_t)pg - 1);
    len += (size_t)(a - al);
    addr = (void*)al;
  }
  const bool bounded = timeout != UINT64_MAX;
  const uint64_t deadline = now_ticks() + timeout;
  int bus = event_bus_open();
  for (;;) {
    if (shard_election_on(H_, nullptr) == id) {
      int rc = posix_madvise(addr, len, advice);
      if (bus >= 0) close(bus);
      if (rc == 0) return 0;
      errno = rc;
      return -1;
    }
    if (timeout == 0) {
      if (bus >= 0) close(bus);
      errno = EAGAIN;
      return -1;
    }
    if (bounded && now_ticks() >= deadline) {
      if (bus >= 0) close(bus);
      errno = ETIMEDOUT;
      return -1;
    }
    if (bus >= 0) {
      pollfd p = {bus, POLLIN, 0};
      if (::poll(&p, 1, 5) > 0) { uint64_t v; ssize_t r = read(bus, &v, 8); (void)r; }
    } else {
      const timespec nap = {0, 5 * 1000000L};
      nanosleep(&nap, nullptr);
    }
  }
}

// ---------------------------------------------- shard table (shared) ----
// These work on any host-visible header (host backend, or a host mirror).
static bool bid_expired(const splinter_shard_bid* b, uint64_t now) {
  const uint64_t at = ld(&b->claimed_at), dur = ld(&b->duration_tsc);
  return (now - at) >= dur;  // half-open window; duration 0 = instantly expired
}

static void bid_fill(splinter_shard_bid* b, uint32_t pid, uint8_t intent, uint8_t prio, uint64_t dur, uint64_t at) {
  st(&b->pid, pid);
  st(&b->intent, intent);
  st(&b->priority, prio);
  st(&b->duration_tsc, dur);
  st(&b->claimed_at, at);
}

int shard_claim_on(splinter_header* H, uint32_t id, uint32_t pid, uint8_t intent, uint8_t prio, uint64_t dur, uint64_t at) {
  if (!H || id == 0) return -2;
  for (auto& b : H->shard_bids)
    if (ld(&b.shard_id) == id) { bid_fill(&b, pid, intent, prio, dur, at); return 0; }
  for (auto& b : H->shard_bids) {
    uint32_t zero = 0;
    if (__atomic_compare_exchange_n(&b.shard_id, &zero, id, false, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED)) {
      bid_fill(&b, pid, intent, prio, dur, at);
      return 0;
    }
  }
  errno = ENOSPC;
  return -1;
}

int shard_rebid_on(splinter_header* H, uint32_t id, uint8_t intent, uint8_t prio, uint64_t dur) {
  if (!H || id == 0) return -2;
  for (auto& b : H->shard_bids) {
    if (ld(&b.shard_id) == id) {
      st(&b.intent, intent);
      st(&b.priority, prio);
      st(&b.duration_tsc, dur);
      st(&b.claimed_at, now_ticks());
      return 0;
    }
  }
  return -1;
}

int shard_release_on(splinter_header* H, uint32_t id) {
  if (!H || id == 0) return -2;
  for (auto& b : H->shard_bids) {
    if (ld(&b.shard_id) == id) {
      bid_fill(&b, 0, SPL_INTENT_NONE, 0, 0, 0);
      st(&b.shard_id, (uint32_t)0);
      return 0;
    }
  }
  return -1;
}

bool shard_present_on(splinter_header* H, uint32_t id) {
  for (auto& b : H->shard_bids)
    if (ld(&b.shard_id) == id) return true;
  return false;
}

uint32_t shard_election_on(splinter_header* H, uint8_t* out_intent) {
  if (out_intent) *out_intent = SPL_INTENT_NONE;
  if (!H) return 0;
  const uint64_t now = now_ticks();
  bool protective = false;
  for (auto& b : H->shard_bids) {
    if (ld(&b.shard_id) == 0 || bid_expired(&b, now)) continue;
    const uint8_t it = ld(&b.intent);
    if (it == SPL_INTENT_WILLNEED || it == SPL_INTENT_SEQUENTIAL) { protective = true; break; }
  }
  bool have = false;
  uint32_t best = 0, best_pid = 0;
  uint8_t best_int = SPL_INTENT_NONE, best_prio = 0;
  uint64_t best_at = 0;
  for (auto& b : H->shard_bids) {
    const uint32_t id = ld(&b.shard_id);
    if (id == 0 || bid_expired(&b, now)) continue;
    const uint8_t it = ld(&b.intent), pr = ld(&b.priority);
    const uint64_t at = ld(&b.claimed_at);
    const uint32_t pd = ld(&b.pid);
    if (it == SPL_INTENT_DONTNEED && protective) continue;  // soft bumper
    bool wins;
    if (!have) wins = true;
    else if (pr != best_prio) wins = pr > best_prio;
    else if (at != best_at) wins = at < best_at;
    else wins = pd < best_pid;
    if (wins) { have = true; best = id; best_int = it; best_prio = pr; best_at = at; best_pid = pd; }
  }
  if (out_intent) *out_intent = have ? best_int : (uint8_t)SPL_INTENT_NONE;
  return have ? best : 0;
}

int shard_table_on(splinter_header* H, splinter_shard_bid_snapshot* out, size_t max) {
  if (!H || !out) return -2;
  const uint64_t now = now_ticks();
  const uint32_t sov = shard_election_on(H, nullptr);
  const size_t n = max < SPLINTER_MAX_SHARDS ? max : SPLINTER_MAX_SHARDS;
  for (size_t i = 0; i < n; ++i) {
    splinter_shard_bid* b = &H->shard_bids[i];
    const uint32_t id = ld(&b->shard_id);
    out[i].shard_id = id;
    out[i].pid = ld(&b->pid);
    out[i].intent = ld(&b->intent);
    out[i].priority = ld(&b->priority);
    out[i].duration_tsc = ld(&b->duration_tsc);
    out[i].claimed_at = ld(&b->claimed_at);
    out[i].expired = id ? (int)bid_expired(b, now) : 1;
    out[i].sovereign = (id && id == sov) ? 1 : 0;
  }
  return (int)n;
}

}  // namespace spl
