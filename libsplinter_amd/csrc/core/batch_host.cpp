// batch_host.cpp — the public host-array batch ABI (splinter_ext.h spl_*_batch) over any StoreBase.
//
// The reference's API is one call per op (reference splinter.c:365-464); its benchmarks loop over
// it from threads (splinter_stress.c:64-101).  These entry points take whole arrays of fixed-stride
// records -- the same layout as the device batch API (arena_api.h) -- so a C / Rust / TS / Lua
// client reaches a backend's throughput path with one call:
//   - hbm: stores stage the arrays through the device kernels (hbm_store.hip HbmStore::*_batch),
//   - node: stores hash-partition the batch and run every shard's part concurrently
//     (node_store.cpp NodeStore::*_batch),
//   - host (shm / file) stores, and any backend without a native path, loop over the per-call API
//     on `threads` host threads (generic_*_batch below).
// spl_batch_alloc gives pinned host memory when the HBM backend is present: batches in it move by
// DMA without a staging copy.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <sched.h>
#include <time.h>
#include <thread>
#include <vector>

#include "splinter_ext.h"
#include "splinter_store.hpp"

using spl::StoreBase;

namespace spl {
void* hbm_symbol(const char* sym);  // capi.cpp: dlsym in the HBM backend (loaded on demand)
}

namespace {

template <class F>
void parallel_for(long n, int threads, F&& f) {
  if (threads <= 1 || n < 1024) {
    for (long i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<long> next{0};
  auto work = [&] {
    for (;;) {
      const long b = next.fetch_add(256);
      if (b >= n) break;
      const long e = std::min(n, b + 256);
      for (long i = b; i < e; ++i) f(i);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
}

inline void key_of(const char* rec, int kstride, char* out) {
  const int n = kstride < 64 ? kstride : 63;
  std::memcpy(out, rec, (size_t)n);
  out[n] = 0;
}

// EAGAIN = the slot's writer is mid-write; past a few immediate retries let it run (a preempted
// writer on an oversubscribed host would otherwise exhaust the retries while it sleeps)
inline void backoff(int t) {
  if (t < 4) return;
  if (t < 16) {
    sched_yield();
    return;
  }
  // still held: the holder is likely preempted (more runnable threads than CPUs) -- sleep so it runs
  const long us = 20L * (t - 15) < 1000 ? 20L * (t - 15) : 1000;
  const timespec ts{0, us * 1000};
  nanosleep(&ts, nullptr);
}

inline int32_t code_of(int rc) {
  if (rc == 0) return 0;
  const int e = errno;
  return e ? -e : -2;
}

bool bad_args(StoreBase* s, const char* keys, int kstride, long n) {
  return !s || n < 0 || (n > 0 && (!keys || kstride <= 0 || kstride > 64));
}

}  // namespace

namespace spl {

long generic_set_batch(StoreBase* s, const char* keys, int kstride, const uint8_t* vals, int vstride,
                       const uint32_t* lens, long n, int32_t* status, int retries, int threads) {
  std::atomic<long> ok{0};
  parallel_for(n, threads, [&](long i) {
    char k[64];
    key_of(keys + i * kstride, kstride, k);
    int rc = -1;
    for (int t = 0; t <= retries; ++t) {
      errno = 0;
      rc = s->set(k, vals + i * (long)vstride, lens[i]);
      if (rc == 0 || errno != EAGAIN) break;
      backoff(t);
    }
    if (status) status[i] = code_of(rc);
    if (rc == 0) ok.fetch_add(1, std::memory_order_relaxed);
  });
  return ok.load();
}

long generic_get_batch(StoreBase* s, const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens,
                       long n, int32_t* status, int retries, int threads) {
  std::atomic<long> ok{0};
  parallel_for(n, threads, [&](long i) {
    char k[64];
    key_of(keys + i * kstride, kstride, k);
    size_t len = 0;
    int rc = -1;
    for (int t = 0; t <= retries; ++t) {
      errno = 0;
      rc = s->get(k, out ? out + i * (long)ostride : nullptr, (size_t)ostride, &len);
      if (rc == 0 || errno != EAGAIN) break;
      backoff(t);
    }
    if (out_lens) out_lens[i] = rc == 0 ? (uint32_t)len : 0;
    if (status) status[i] = rc == 0 ? 0 : (errno == ENOENT || errno == 0 ? -2 : -errno);
    if (rc == 0) ok.fetch_add(1, std::memory_order_relaxed);
  });
  return ok.load();
}

long generic_intop_batch(StoreBase* s, const char* keys, int kstride, const int* ops, const uint64_t* masks, long n,
                         int32_t* status, uint64_t* results, int threads) {
  std::atomic<long> ok{0};
  parallel_for(n, threads, [&](long i) {
    char k[64];
    key_of(keys + i * kstride, kstride, k);
    uint64_t m = masks ? masks[i] : 0;
    int rc = -1;
    for (int t = 0; t < 64; ++t) {
      errno = 0;
      rc = s->integer_op(k, (splinter_integer_op_t)ops[i], &m);
      if (rc == 0 || errno != EAGAIN) break;
      backoff(t);
    }
    if (status) status[i] = code_of(rc);
    if (results) {
      uint64_t v = 0;
      size_t got = 0;
      if (rc == 0 && s->get(k, &v, sizeof v, &got) == 0) results[i] = v;
      else results[i] = 0;
    }
    if (rc == 0) ok.fetch_add(1, std::memory_order_relaxed);
  });
  return ok.load();
}

// Vectors [n, 768] fp32 -> slots.  expect_epochs (optional) implements the daemon's stale-race
// check (reference splinference.cpp:282-286): the write is skipped (status -ESTALE) when the
// key's epoch moved since its text was read.
long generic_set_embedding_batch(StoreBase* s, const char* keys, int kstride, const float* vecs, long n,
                                 const uint64_t* expect_epochs, int32_t* status, int threads) {
  std::atomic<long> ok{0};
  parallel_for(n, threads, [&](long i) {
    char k[64];
    key_of(keys + i * kstride, kstride, k);
    if (expect_epochs && s->epoch_of(k) != expect_epochs[i]) {
      if (status) status[i] = -ESTALE;
      return;
    }
    int rc = -1;
    for (int t = 0; t < 64; ++t) {
      errno = 0;
      rc = s->set_embedding(k, vecs + i * (long)spl::kEmbedDim);
      if (rc == 0 || errno != EAGAIN) break;
      backoff(t);
    }
    int32_t st = code_of(rc);
    // post-write check: exactly our +2 landed, nobody rewrote the text meanwhile
    if (rc == 0 && expect_epochs && s->epoch_of(k) != expect_epochs[i] + 2) st = -ESTALE;
    if (status) status[i] = st;
    if (st == 0) ok.fetch_add(1, std::memory_order_relaxed);
  });
  return ok.load();
}

}  // namespace spl

extern "C" {

long spl_set_batch(spl_store* h, const char* keys, int kstride, const uint8_t* vals, int vstride,
                   const uint32_t* lens, long n, int32_t* status, int retries, int threads) {
  auto* s = (StoreBase*)h;
  if (bad_args(s, keys, kstride, n) || (n > 0 && (!vals || !lens || vstride <= 0))) return -2;
  if (n == 0) return 0;
  const long r = s->set_batch(keys, kstride, vals, vstride, lens, n, status, retries);
  if (r != StoreBase::kNoBatch) return r;
  return spl::generic_set_batch(s, keys, kstride, vals, vstride, lens, n, status, retries, threads);
}

long spl_get_batch(spl_store* h, const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens,
                   long n, int32_t* status, int retries, int threads) {
  auto* s = (StoreBase*)h;
  if (bad_args(s, keys, kstride, n) || (out && ostride <= 0)) return -2;
  if (n == 0) return 0;
  const long r = s->get_batch(keys, kstride, out, ostride, out_lens, n, status, retries);
  if (r != StoreBase::kNoBatch) return r;
  return spl::generic_get_batch(s, keys, kstride, out, ostride, out_lens, n, status, retries, threads);
}

long spl_intop_batch(spl_store* h, const char* keys, int kstride, const int* ops, const uint64_t* masks, long n,
                     int32_t* status, int threads) {
  return spl_intop_batch_ex(h, keys, kstride, ops, masks, n, status, nullptr, threads);
}

long spl_intop_batch_ex(spl_store* h, const char* keys, int kstride, const int* ops, const uint64_t* masks, long n,
                        int32_t* status, uint64_t* results, int threads) {
  auto* s = (StoreBase*)h;
  if (bad_args(s, keys, kstride, n) || (n > 0 && !ops)) return -2;
  if (n == 0) return 0;
  const long r = s->intop_batch(keys, kstride, ops, masks, n, status, results);
  if (r != StoreBase::kNoBatch) return r;
  return spl::generic_intop_batch(s, keys, kstride, ops, masks, n, status, results, threads);
}

long spl_set_embedding_batch(spl_store* h, const char* keys, int kstride, const float* vecs, long n,
                             const uint64_t* expect_epochs, int32_t* status, int threads) {
  auto* s = (StoreBase*)h;
  if (bad_args(s, keys, kstride, n) || (n > 0 && !vecs)) return -2;
  if (n == 0) return 0;
  if (!expect_epochs) {  // the epoch-checked daemon write-back stays per op
    const long r = s->set_embedding_batch(keys, kstride, vecs, n, status);
    if (r != StoreBase::kNoBatch) return r;
  }
  return spl::generic_set_embedding_batch(s, keys, kstride, vecs, n, expect_epochs, status, threads);
}

// Batch arrays: pinned (page-locked, device-mapped) host memory when the HBM backend is loadable,
// so hbm: / node: batches move by DMA straight from / to them; plain aligned memory otherwise.
// A 64-B header in front of the returned pointer records which allocator to return it to.
namespace {
constexpr uint64_t kBatchMagicPinned = 0x53504c5042415431ull, kBatchMagicPlain = 0x53504c5042415430ull;
}
void* spl_batch_alloc(size_t bytes) {
  using Alloc = void* (*)(size_t);
  static Alloc pinned = (Alloc)spl::hbm_symbol("spl_hbm_host_alloc");
  void* raw = pinned ? pinned(bytes + 64) : nullptr;
  uint64_t magic = kBatchMagicPinned;
  if (!raw) {
    raw = aligned_alloc(64, (bytes + 64 + 63) / 64 * 64);
    magic = kBatchMagicPlain;
  }
  if (!raw) return nullptr;
  *(uint64_t*)raw = magic;
  return (uint8_t*)raw + 64;
}

void spl_batch_free(void* p) {
  if (!p) return;
  void* raw = (uint8_t*)p - 64;
  if (*(uint64_t*)raw == kBatchMagicPinned) {
    using Free = void (*)(void*);
    static Free f = (Free)spl::hbm_symbol("spl_hbm_host_free");
    if (f) f(raw);
  } else {
    free(raw);
  }
}

}  // extern "C"
