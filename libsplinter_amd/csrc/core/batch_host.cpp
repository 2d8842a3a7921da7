// batch_host.cpp — batched host-side entry points over any StoreBase.
// Used by the CPU plumbing benchmark (BASELINE config #1), the embedding
// daemon (bulk vector write-back) and the sharded-arena CPU tests.  Keys and
// values use the same fixed-stride record layout as the GPU batch API
// (arena_api.h), so one client batch can target either backend.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <thread>
#include <vector>

#include "splinter_ext.h"
#include "splinter_store.hpp"

using spl::StoreBase;

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

inline int32_t code_of(int rc) {
  if (rc == 0) return 0;
  const int e = errno;
  return e ? -e : -2;
}

}  // namespace

extern "C" {

long spl_set_batch(spl_store* h, const char* keys, int kstride, const uint8_t* vals, int vstride,
                   const uint32_t* lens, long n, int32_t* status, int retries, int threads) {
  auto* s = (StoreBase*)h;
  if (!s) return -2;
  std::atomic<long> ok{0};
  parallel_for(n, threads, [&](long i) {
    char k[64];
    key_of(keys + i * kstride, kstride, k);
    int rc = -1;
    for (int t = 0; t <= retries; ++t) {
      errno = 0;
      rc = s->set(k, vals + i * (long)vstride, lens[i]);
      if (rc == 0 || errno != EAGAIN) break;
    }
    if (status) status[i] = code_of(rc);
    if (rc == 0) ok.fetch_add(1, std::memory_order_relaxed);
  });
  return ok.load();
}

long spl_get_batch(spl_store* h, const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens,
                   long n, int32_t* status, int retries, int threads) {
  auto* s = (StoreBase*)h;
  if (!s) return -2;
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
    }
    if (out_lens) out_lens[i] = rc == 0 ? (uint32_t)len : 0;
    if (status) status[i] = rc == 0 ? 0 : (errno == ENOENT || errno == 0 ? -2 : -errno);
    if (rc == 0) ok.fetch_add(1, std::memory_order_relaxed);
  });
  return ok.load();
}

long spl_intop_batch(spl_store* h, const char* keys, int kstride, const int* ops, const uint64_t* masks, long n,
                     int32_t* status, int threads) {
  auto* s = (StoreBase*)h;
  if (!s) return -2;
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
    }
    if (status) status[i] = code_of(rc);
    if (rc == 0) ok.fetch_add(1, std::memory_order_relaxed);
  });
  return ok.load();
}

// Vectors [n, 768] fp32 -> slots.  expect_epochs (optional) implements the
// daemon's stale-race check (reference splinference.cpp:282-286): the write is
// skipped (status -EAGAIN... reported as -116 ESTALE) when the key's epoch
// moved since its text was read.
long spl_set_embedding_batch(spl_store* h, const char* keys, int kstride, const float* vecs, long n,
                             const uint64_t* expect_epochs, int32_t* status, int threads) {
  auto* s = (StoreBase*)h;
  if (!s) return -2;
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
    }
    int32_t st = code_of(rc);
    // post-write check: exactly our +2 landed, nobody rewrote the text meanwhile
    if (rc == 0 && expect_epochs && s->epoch_of(k) != expect_epochs[i] + 2) st = -ESTALE;
    if (status) status[i] = st;
    if (st == 0) ok.fetch_add(1, std::memory_order_relaxed);
  });
  return ok.load();
}

}  // extern "C"
