// splinter_hostapi_bench — per-call C API throughput and latency (the reference's own metric:
// splinter_set / splinter_get calls from host threads, reference splinter_stress.c:64-188) on
// any store, including "hbm:NAME" stores served by the device command ring (cmd_ring.hpp).
//
//   splinter_hostapi_bench [--store NAME] [--threads T] [--seconds S] [--keys K]
//                          [--value-len L] [--set-frac F] [--append-check N] [--batch B]
//
// --batch B: the host-array batch ABI instead (splinter_ext.h spl_set_batch / spl_get_batch): K keys
// prepopulated in batches, then for S seconds alternating set and get batches of B random keys from
// arrays allocated with spl_batch_alloc (pinned: hbm: / node: stores DMA them); every op counts.
// Afterwards every get of the last batch must have returned its key's value.
//
// Threads run a set/get mix over K prepopulated keys for S seconds; every call is timed.  One
// JSON line: ops/s (every completed call, EAGAIN included, as splinter_stress counts), successful
// ops/s, p50/p90/p99 latency (µs) per op type.  --append-check N: afterwards every thread appends
// N tagged records to ONE key concurrently; the final value must hold exactly T*N records with
// each thread's sequence in order (no lost or torn appends).  Exit status != 0 on any failure.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <sched.h>
#include <unistd.h>

#include "splinter_ext.h"

namespace {

struct Args {
  std::string store;
  int threads = 8;
  double seconds = 2.0;
  int keys = 65536;
  int value_len = 150;
  double set_frac = 0.5;
  int append_check = 0;
  long batch = 0;
};

double pct(std::vector<float>& v, double p) {
  if (v.empty()) return 0.0;
  const size_t k = std::min(v.size() - 1, (size_t)(p * (double)(v.size() - 1)));
  std::nth_element(v.begin(), v.begin() + (long)k, v.end());
  return v[k];
}

std::string key_of(int i) {
  char b[32];
  snprintf(b, sizeof b, "hk%08d", i);
  return b;
}

// value of key i: "val:<i>|" then filler up to len bytes
void fill_value(uint8_t* row, long i, int len) {
  char head[32];
  const int h = snprintf(head, sizeof head, "val:%ld|", i);
  for (int q = 0; q < len; ++q) row[q] = q < h ? (uint8_t)head[q] : (uint8_t)('a' + (i + q) % 26);
}

int batch_main(const Args& a) {
  using clk = std::chrono::steady_clock;
  const int ks = 16, vs = (a.value_len + 15) / 16 * 16;
  const long B = a.batch, K = a.keys;
  int err = 0;
  spl_store* st = spl_store_create(a.store.c_str(), (size_t)K * 2 + 1024, 256, SPL_CREATE_NO_EMBEDDINGS, &err);
  if (!st) {
    fprintf(stderr, "create %s failed: %s\n", a.store.c_str(), strerror(err));
    return 1;
  }
  auto* keys = (char*)spl_batch_alloc((size_t)B * ks * 2);
  auto* vals = (uint8_t*)spl_batch_alloc((size_t)B * vs);
  auto* lens = (uint32_t*)spl_batch_alloc((size_t)B * 4);
  auto* stat = (int32_t*)spl_batch_alloc((size_t)B * 4);
  auto* out = (uint8_t*)spl_batch_alloc((size_t)B * vs);
  auto* olen = (uint32_t*)spl_batch_alloc((size_t)B * 4);
  std::vector<long> gid((size_t)B);
  if (!keys || !vals || !lens || !stat || !out || !olen) { fprintf(stderr, "batch alloc failed\n"); return 1; }
  auto key_row = [&](char* row, long i) {
    memset(row, 0, ks);
    snprintf(row, ks, "bk%010ld", i);
  };
  // prepopulate every key (values of length value_len)
  long bad = 0;
  for (long b = 0; b < K; b += B) {
    const long m = std::min(B, K - b);
    for (long j = 0; j < m; ++j) {
      key_row(keys + j * ks, b + j);
      fill_value(vals + j * vs, b + j, a.value_len);
      lens[j] = (uint32_t)a.value_len;
    }
    const long ok = spl_set_batch(st, keys, ks, vals, vs, lens, m, stat, 64, a.threads);
    bad += m - ok;
  }
  if (bad) { fprintf(stderr, "prepopulate: %ld failures\n", bad); return 1; }
  // one set batch and one get batch of random keys, reused every round (the set rewrites values
  // with the same content, so every get stays checkable)
  char* gkeys = keys + B * ks;
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (long j = 0; j < B; ++j) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    const long i = (long)(x % (uint64_t)K);
    key_row(keys + j * ks, i);
    fill_value(vals + j * vs, i, a.value_len);
    lens[j] = (uint32_t)a.value_len;
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    gid[(size_t)j] = (long)(x % (uint64_t)K);
    key_row(gkeys + j * ks, gid[(size_t)j]);
  }
  long ops = 0, okc = 0, rounds = 0;
  const auto t0 = clk::now();
  double el = 0;
  do {
    okc += spl_set_batch(st, keys, ks, vals, vs, lens, B, stat, 64, a.threads);
    okc += spl_get_batch(st, gkeys, ks, out, vs, olen, B, stat, 64, a.threads);
    ops += 2 * B;
    ++rounds;
    el = std::chrono::duration<double>(clk::now() - t0).count();
  } while (el < a.seconds);
  // the last get batch: every value intact
  long wrong = 0;
  for (long j = 0; j < B; ++j) {
    uint8_t want[4096];
    fill_value(want, gid[(size_t)j], a.value_len);
    if (stat[j] != 0 || olen[j] != (uint32_t)a.value_len || memcmp(out + j * vs, want, (size_t)a.value_len) != 0)
      ++wrong;
  }
  printf("{\"store\": \"%s\", \"backend\": \"%s\", \"batch\": %ld, \"rounds\": %ld, \"seconds\": %.3f, "
         "\"ops_per_s\": %.1f, \"successful_ops_per_s\": %.1f, \"keys\": %ld, \"value_len\": %d, "
         "\"get_check_failures\": %ld}\n",
         a.store.c_str(), spl_store_backend(st), B, rounds, el, (double)ops / el, (double)okc / el, K, a.value_len,
         wrong);
  spl_batch_free(keys); spl_batch_free(vals); spl_batch_free(lens); spl_batch_free(stat); spl_batch_free(out);
  spl_batch_free(olen);
  spl_store_close(st);
  spl_unlink(a.store.c_str());
  return wrong ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  a.store = "hbm:hostapi" + std::to_string(getpid());
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto nxt = [&]() -> const char* { return i + 1 < argc ? argv[++i] : ""; };
    if (s == "--store") a.store = nxt();
    else if (s == "--threads") a.threads = atoi(nxt());
    else if (s == "--seconds") a.seconds = atof(nxt());
    else if (s == "--keys") a.keys = atoi(nxt());
    else if (s == "--value-len") a.value_len = atoi(nxt());
    else if (s == "--set-frac") a.set_frac = atof(nxt());
    else if (s == "--append-check") a.append_check = atoi(nxt());
    else if (s == "--batch") a.batch = atol(nxt());
    else { fprintf(stderr, "unknown option %s\n", s.c_str()); return 2; }
  }
  if (a.batch > 0) return batch_main(a);
  const size_t max_val = 4096;
  if (splinter_create(a.store.c_str(), (size_t)a.keys * 2 + 1024, max_val) != 0) {
    fprintf(stderr, "create %s failed: %s\n", a.store.c_str(), strerror(errno));
    return 1;
  }
  std::string val(a.value_len, 'v');
  // prepopulate in parallel (the same per-call path)
  {
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int t = 0; t < a.threads; ++t)
      th.emplace_back([&, t] {
        for (int i = t; i < a.keys; i += a.threads) {
          std::string k = key_of(i);
          for (int r = 0; r < 100000; ++r) {  // EAGAIN = a racing claim: back off and retry
            if (splinter_set(k.c_str(), val.data(), val.size()) == 0) break;
            if (errno != EAGAIN || r == 99999) { fprintf(stderr, "set %s: %s\n", k.c_str(), strerror(errno)); ++bad; break; }
            sched_yield();
          }
        }
      });
    for (auto& x : th) x.join();
    if (bad) { fprintf(stderr, "prepopulate: %d failures\n", bad.load()); return 1; }
  }
  using clk = std::chrono::steady_clock;
  std::atomic<bool> go{false}, stop{false};
  std::vector<std::vector<float>> lat_set(a.threads), lat_get(a.threads);
  std::vector<uint64_t> ok(a.threads, 0), again(a.threads, 0), fail(a.threads, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < a.threads; ++t)
    th.emplace_back([&, t] {
      uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1);
      std::vector<char> buf(max_val);
      lat_set[t].reserve(1 << 20);
      lat_get[t].reserve(1 << 20);
      while (!go.load(std::memory_order_acquire)) {}
      while (!stop.load(std::memory_order_relaxed)) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const std::string k = key_of((int)(x % (uint64_t)a.keys));
        const bool is_set = (double)((x >> 20) & 0xffff) / 65536.0 < a.set_frac;
        const auto t0 = clk::now();
        int rc;
        size_t n = 0;
        if (is_set) rc = splinter_set(k.c_str(), val.data(), val.size());
        else rc = splinter_get(k.c_str(), buf.data(), buf.size(), &n);
        const float us = std::chrono::duration<float, std::micro>(clk::now() - t0).count();
        (is_set ? lat_set[t] : lat_get[t]).push_back(us);
        if (rc == 0 && (is_set || n == val.size())) ++ok[t];
        else if (errno == EAGAIN) ++again[t];
        else ++fail[t];
      }
    });
  const auto t0 = clk::now();
  go.store(true, std::memory_order_release);
  std::this_thread::sleep_for(std::chrono::duration<double>(a.seconds));
  stop.store(true);
  for (auto& x : th) x.join();
  const double el = std::chrono::duration<double>(clk::now() - t0).count();
  std::vector<float> ls, lg, la;
  uint64_t tok = 0, tag = 0, tf = 0;
  for (int t = 0; t < a.threads; ++t) {
    ls.insert(ls.end(), lat_set[t].begin(), lat_set[t].end());
    lg.insert(lg.end(), lat_get[t].begin(), lat_get[t].end());
    tok += ok[t]; tag += again[t]; tf += fail[t];
  }
  la = ls;
  la.insert(la.end(), lg.begin(), lg.end());
  const uint64_t calls = la.size();
  int rc = tf ? 1 : 0;

  // concurrent append check
  int app_ok = -1;
  if (a.append_check > 0) {
    const char* ak = "__append_check";
    splinter_set(ak, "|", 1);
    std::vector<std::thread> at;
    std::atomic<int> afail{0};
    for (int t = 0; t < a.threads; ++t)
      at.emplace_back([&, t] {
        for (int s = 0; s < a.append_check; ++s) {
          char rec[32];
          const int n = snprintf(rec, sizeof rec, "%02d:%03d|", t, s);
          size_t nl = 0;
          int r = -1;
          for (int tries = 0; tries < 100000; ++tries) {
            r = splinter_append(ak, rec, (size_t)n, &nl);
            if (r == 0 || errno != EAGAIN) break;
            sched_yield();
          }
          if (r != 0) ++afail;
        }
      });
    for (auto& x : at) x.join();
    std::vector<char> out(max_val + 1, 0);
    size_t n = 0;
    app_ok = 0;
    if (afail == 0 && splinter_get(ak, out.data(), max_val, &n) == 0) {
      const size_t rec = 7;  // "tt:sss|"
      std::vector<int> next(a.threads, 0);
      bool good = n == 1 + rec * (size_t)a.threads * (size_t)a.append_check && out[0] == '|';
      for (size_t p = 1; good && p + rec <= n; p += rec) {
        int t = -1, s = -1;
        if (sscanf(out.data() + p, "%2d:%3d|", &t, &s) != 2 || t < 0 || t >= a.threads || s != next[t]) good = false;
        else ++next[t];
      }
      app_ok = good ? 1 : 0;
    }
    if (app_ok != 1) {
      fprintf(stderr, "append check failed (len %zu, %d call failures)\n", n, afail.load());
      rc = 1;
    }
  }
  printf("{\"store\": \"%s\", \"threads\": %d, \"seconds\": %.3f, \"calls\": %llu, \"ops_per_s\": %.1f, "
         "\"successful_ops_per_s\": %.1f, \"eagain\": %llu, \"failures\": %llu, "
         "\"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f, \"set_p50_us\": %.2f, \"set_p99_us\": %.2f, "
         "\"get_p50_us\": %.2f, \"get_p99_us\": %.2f, \"value_len\": %d, \"set_frac\": %.2f, \"append_check\": %d}\n",
         a.store.c_str(), a.threads, el, (unsigned long long)calls, (double)calls / el, (double)tok / el,
         (unsigned long long)tag, (unsigned long long)tf, pct(la, 0.5), pct(la, 0.9), pct(la, 0.99), pct(ls, 0.5),
         pct(ls, 0.99), pct(lg, 0.5), pct(lg, 0.99), a.value_len, a.set_frac, app_ok);
  splinter_close();
  spl_unlink(a.store.c_str());
  return rc;
}
