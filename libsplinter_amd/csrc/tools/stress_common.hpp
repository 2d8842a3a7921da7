// Shared engine of splinter_stress (MRSW) and splinter_chi_sao (MRMW).
//
// Behaviour follows the reference benches (/root/reference/splinter_stress.c:64-195,
// splinter_chi_sao.c:80-140 and 400-418): writers rewrite "ver:N|nonce:T|[w:I|]data:" +
// fill('A'+N%26) payloads over a hot key set, readers spin-get random keys and
// retry EAGAIN without backoff, ops/s = (gets + sets) / elapsed with every get
// attempt counted.  Differences (documented in docs/DIVERGENCES.md):
//   * counters are thread-local and summed at the end (the reference's shared
//     atomic_int counters serialise every thread on one cache line and overflow
//     past 2^31 on fast runs);
//   * the integrity check verifies the whole payload (fill byte matches the
//     version, writer id matches the key's lane), not just the "ver:" prefix;
//   * --incr N adds integer_op(INC) workers on BIGUINT counter keys (BASELINE
//     config #1 "set/get/incr loop"), with an exact final-count check;
//   * --store accepts hbm:NAME as well as shm names and file paths.
#pragma once
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "splinter_ext.h"

namespace stress {

struct Config {
  std::string store;
  int slots = 50000;
  int max_value = 4096;
  int threads = 32;
  int writers = 1;
  int incr = 0;
  int duration_ms = 60000;
  int keys = 20000;
  int writer_us = 0;
  bool scrub = false, quiet = false, keep = false, lanes = false;
};

struct Counters {
  uint64_t gets = 0, sets = 0, get_ok = 0, set_ok = 0, get_fail = 0, set_fail = 0, integrity = 0, retries = 0,
           get_miss = 0, get_oversize = 0, set_full = 0, set_too_big = 0, incrs = 0;
  void add(const Counters& o) {
    gets += o.gets; sets += o.sets; get_ok += o.get_ok; set_ok += o.set_ok; get_fail += o.get_fail;
    set_fail += o.set_fail; integrity += o.integrity; retries += o.retries; get_miss += o.get_miss;
    get_oversize += o.get_oversize; set_full += o.set_full; set_too_big += o.set_too_big; incrs += o.incrs;
  }
};

inline long now_ms() {
  return (long)std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// "ver:%u|nonce:%lu|[w:%d|]data:" + fill; returns false on malformed or torn data.
inline bool check_payload(const char* v, size_t len, int lane_writer) {
  if (len < 5 || memcmp(v, "ver:", 4) != 0) return false;
  size_t i = 4;
  unsigned ver = 0;
  if (v[i] < '0' || v[i] > '9') return false;
  while (i < len && v[i] >= '0' && v[i] <= '9') ver = ver * 10 + (unsigned)(v[i++] - '0');
  if (i >= len || v[i] != '|') return false;
  const char* d = (const char*)memmem(v + i, len - i, "data:", 5);
  if (!d) return false;
  if (lane_writer >= 0) {
    const char* w = (const char*)memmem(v + i, (size_t)(d - (v + i)), "|w:", 3);
    if (w && atoi(w + 3) != lane_writer) return false;
  }
  size_t off = (size_t)(d - v) + 5;
  if (ver <= 1 && len - off == 4 && !memcmp(v + off, "SEED", 4)) return true;
  const char fill = (char)('A' + ver % 26);
  for (size_t j = off; j < len; ++j)
    if (v[j] != fill) return false;
  return true;
}

inline int run(Config cfg, const char* title, const char* regime) {
  if (cfg.threads < 2) cfg.threads = 2;
  if (cfg.writers < 1) cfg.writers = 1;
  if (cfg.writers >= cfg.threads) cfg.threads = cfg.writers + 1;
  if (cfg.store.empty()) cfg.store = std::string(cfg.lanes ? "mrmw_test_" : "mrsw_test_") + std::to_string(getpid());
  if (splinter_create_or_open(cfg.store.c_str(), (size_t)cfg.slots, (size_t)cfg.max_value) != 0) {
    perror("splinter_create_or_open");
    return 1;
  }
  splinter_set_mop(cfg.scrub ? 1 : 0);
  std::vector<std::string> keys((size_t)cfg.keys);
  for (int i = 0; i < cfg.keys; ++i) {
    char b[32];
    snprintf(b, sizeof b, "k%08d", i);
    keys[(size_t)i] = b;
  }
  printf("===== %s STRESS TEST PLAN =====\n", title);
  printf("Store    : %s\nThreads  : %d\nWriters  : %d\nIncr     : %d\nDuration : %d ms\nSlots    : %d\nH-Scrub  : %s\n"
         "Hot Keys : %d\nW/Backoff: %d us\nMax Val  : %d bytes\nBackend  : %s\n",
         cfg.store.c_str(), cfg.threads, cfg.writers, cfg.incr, cfg.duration_ms, cfg.slots, cfg.scrub ? "Yes" : "No",
         cfg.keys, cfg.writer_us, cfg.max_value, spl_store_backend(spl_store_current()));
  printf("Pre-populating store with indexed backfill (%d keys) ...\n", cfg.keys);
  for (int i = 0; i < cfg.keys; ++i) {
    char v[128];
    int n = snprintf(v, sizeof v, "ver:%u|nonce:%lu|data:SEED", 1u, (unsigned long)now_ms());
    if (splinter_set(keys[(size_t)i].c_str(), v, (size_t)n) != 0) {
      fprintf(stderr, "prepopulate failed at %d: %s\n", i, strerror(errno));
      return 1;
    }
  }
  const int n_incr_keys = 8;
  for (int c = 0; c < (cfg.incr ? n_incr_keys : 0); ++c) {
    std::string k = "ctr" + std::to_string(c);
    uint64_t z = 0;
    splinter_set(k.c_str(), &z, 8);
    splinter_set_named_type(k.c_str(), SPL_SLOT_TYPE_BIGUINT);
  }
  spl_store* st = spl_store_current();
  std::atomic<int> running{1};
  const int readers = cfg.threads - cfg.writers - cfg.incr;
  std::vector<Counters> ctr((size_t)cfg.threads);
  std::vector<std::thread> th;
  auto lane_of = [&](int w, int* start, int* len) {
    const int base = cfg.keys / cfg.writers, rem = cfg.keys % cfg.writers;
    *start = w * base;
    *len = base + (w == cfg.writers - 1 ? rem : 0);
  };
  printf("Creating threadpool ...\n -> Writers - (%d), Incr - (%d), Readers - (%d)\n", cfg.writers, cfg.incr,
         readers > 0 ? readers : 0);
  long start = now_ms();
  for (int w = 0; w < cfg.writers; ++w) {
    th.emplace_back([&, w] {
      spl_store_use(st);
      Counters& c = ctr[(size_t)w];
      std::vector<char> buf((size_t)cfg.max_value);
      int ls = 0, ll = cfg.keys;
      if (cfg.lanes) lane_of(w, &ls, &ll);
      size_t payload = (size_t)cfg.max_value / 2;
      if (payload < 64) payload = 64;
      unsigned ver = 2;
      do {
        for (int i = ls; i < ls + ll && running.load(std::memory_order_relaxed); ++i) {
          int n = cfg.lanes ? snprintf(buf.data(), buf.size(), "ver:%u|nonce:%lu|w:%d|data:", ver,
                                       (unsigned long)now_ms(), w)
                            : snprintf(buf.data(), buf.size(), "ver:%u|nonce:%lu|data:", ver, (unsigned long)now_ms());
          if (n <= 0 || n >= cfg.max_value) { ++c.set_too_big; ++c.set_fail; continue; }
          size_t remain = (size_t)cfg.max_value - (size_t)n - 1, fill = payload < remain ? payload : remain;
          memset(buf.data() + n, 'A' + (int)(ver % 26), fill);
          int rc = splinter_set(keys[(size_t)i].c_str(), buf.data(), (size_t)n + fill);
          ++c.sets;
          if (rc == 0) ++c.set_ok;
          else { ++c.set_fail; ++c.set_full; }
          if (cfg.writer_us > 0) usleep((useconds_t)cfg.writer_us);
        }
        ++ver;
      } while (running.load(std::memory_order_relaxed));
    });
  }
  for (int k = 0; k < cfg.incr; ++k) {
    th.emplace_back([&, k] {
      spl_store_use(st);
      Counters& c = ctr[(size_t)(cfg.writers + k)];
      std::string key = "ctr" + std::to_string(k % n_incr_keys);
      uint64_t one = 1;
      while (running.load(std::memory_order_relaxed)) {
        for (int r = 0; r < 64; ++r) {
          one = 1;
          if (splinter_integer_op(key.c_str(), SPL_OP_INC, &one) == 0) ++c.incrs;
          else ++c.set_fail;
        }
      }
    });
  }
  for (int r = 0; r < readers; ++r) {
    th.emplace_back([&, r] {
      spl_store_use(st);
      Counters& c = ctr[(size_t)(cfg.writers + cfg.incr + r)];
      std::vector<char> buf((size_t)cfg.max_value + 1);
      uint64_t rng = 0x9E3779B97F4A7C15ull ^ ((uint64_t)r * 0xBF58476D1CE4E5B9ull) ^ (uint64_t)getpid();
      while (running.load(std::memory_order_relaxed)) {
        for (int t = 0; t < 256; ++t) {
          rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
          const int idx = (int)(rng % (uint64_t)cfg.keys);
          for (;;) {
            if (!running.load(std::memory_order_relaxed)) break;
            size_t got = 0;
            int rc = splinter_get(keys[(size_t)idx].c_str(), buf.data(), (size_t)cfg.max_value, &got);
            ++c.gets;
            if (rc == 0) {
              ++c.get_ok;
              int lw = -1;
              if (cfg.lanes) {
                const int base = cfg.keys / cfg.writers;
                lw = base ? idx / base : 0;
                if (lw >= cfg.writers) lw = cfg.writers - 1;
              }
              if (!check_payload(buf.data(), got, lw)) ++c.integrity;
              break;
            }
            if (errno == EAGAIN) { ++c.retries; continue; }
            ++c.get_fail;
            if (errno == ENOENT) ++c.get_miss;
            else if (errno == EMSGSIZE) ++c.get_oversize;
            break;
          }
        }
      }
    });
  }
  printf("Test is now running ...\n");
  int seq = 0;
  while (now_ms() - start < cfg.duration_ms) {
    usleep(10000);
    if (!cfg.quiet && ++seq % 15 == 0) { fputc('.', stdout); fflush(stdout); }
  }
  running.store(0);
  for (auto& t : th) t.join();
  const long elapsed = now_ms() - start;
  Counters tot;
  for (auto& c : ctr) tot.add(c);
  uint64_t incr_seen = 0;
  for (int c = 0; c < (cfg.incr ? n_incr_keys : 0); ++c) {
    std::string k = "ctr" + std::to_string(c);
    uint64_t v = 0;
    size_t got = 0;
    if (splinter_get(k.c_str(), &v, 8, &got) == 0) incr_seen += v;
  }
  splinter_close();
  if (!cfg.keep) spl_unlink(cfg.store.c_str());
  const double sec = elapsed / 1000.0, ops = (double)(tot.gets + tot.sets + tot.incrs) / sec;
  printf("\n\n===== %s STRESS RESULTS =====\n", title);
  printf("Threads            : %d (%s)\n", cfg.threads, regime);
  printf("Duration           : %ld ms\n", elapsed);
  printf("Hot keys           : %d\n", cfg.keys);
  printf("Writer Backoff     : %d us\n", cfg.writer_us);
  printf("Total ops          : %llu (gets=%llu, sets=%llu, incrs=%llu)\n",
         (unsigned long long)(tot.gets + tot.sets + tot.incrs), (unsigned long long)tot.gets,
         (unsigned long long)tot.sets, (unsigned long long)tot.incrs);
  printf("Throughput         : %.0f ops/sec\n", ops);
  printf("Successful ops/sec : %.0f\n", (double)(tot.get_ok + tot.set_ok + tot.incrs) / sec);
  printf("Hybrid Scrub       : %s\n", cfg.scrub ? "Yes" : "No");
  printf("Get                : ok=%llu fail=%llu (miss=%llu, oversize=%llu)\n", (unsigned long long)tot.get_ok,
         (unsigned long long)tot.get_fail, (unsigned long long)tot.get_miss, (unsigned long long)tot.get_oversize);
  printf("Set                : ok=%llu fail=%llu (full=%llu, too_big=%llu)\n", (unsigned long long)tot.set_ok,
         (unsigned long long)tot.set_fail, (unsigned long long)tot.set_full, (unsigned long long)tot.set_too_big);
  if (cfg.incr)
    printf("Incr               : %llu applied, %llu observed %s\n", (unsigned long long)tot.incrs,
           (unsigned long long)incr_seen, incr_seen == tot.incrs ? "(exact)" : "(MISMATCH)");
  printf("Integrity failures : %llu\n", (unsigned long long)tot.integrity);
  printf("Retries (EAGAIN)   : %llu (%.2f%% of gets, %.2f per successful get)\n\n", (unsigned long long)tot.retries,
         tot.gets ? 100.0 * (double)tot.retries / (double)tot.gets : 0.0,
         tot.get_ok ? (double)tot.retries / (double)tot.get_ok : 0.0);
  printf("{\"bench\":\"%s\",\"ops_per_s\":%.0f,\"gets\":%llu,\"sets\":%llu,\"incrs\":%llu,\"retries\":%llu,"
         "\"integrity_failures\":%llu,\"incr_exact\":%s,\"elapsed_ms\":%ld}\n",
         title, ops, (unsigned long long)tot.gets, (unsigned long long)tot.sets, (unsigned long long)tot.incrs,
         (unsigned long long)tot.retries, (unsigned long long)tot.integrity,
         (!cfg.incr || incr_seen == tot.incrs) ? "true" : "false", elapsed);
  return (tot.integrity || (cfg.incr && incr_seen != tot.incrs)) ? 3 : 0;
}

inline bool parse_common(Config& c, int argc, char** argv, int& i) {
  auto nxt = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
  const char* a = argv[i];
  const char* v = nullptr;
  if (!strcmp(a, "--threads") && (v = nxt())) c.threads = atoi(v);
  else if (!strcmp(a, "--writers") && (v = nxt())) c.writers = atoi(v);
  else if (!strcmp(a, "--incr") && (v = nxt())) c.incr = atoi(v);
  else if (!strcmp(a, "--duration-ms") && (v = nxt())) c.duration_ms = atoi(v);
  else if (!strcmp(a, "--keys") && (v = nxt())) c.keys = atoi(v);
  else if (!strcmp(a, "--store") && (v = nxt())) c.store = v;
  else if (!strcmp(a, "--slots") && (v = nxt())) c.slots = atoi(v);
  else if (!strcmp(a, "--max-value") && (v = nxt())) c.max_value = atoi(v);
  else if (!strcmp(a, "--writer-us") && (v = nxt())) c.writer_us = atoi(v);
  else if (!strcmp(a, "--quiet")) c.quiet = true;
  else if (!strcmp(a, "--keep-test-store")) c.keep = true;
  else if (!strcmp(a, "--scrub")) c.scrub = true;
  else return false;
  return true;
}

inline void usage(const char* prog) {
  fprintf(stderr,
          "\nUsage: %s [arguments]\nWhere arguments are:\n\t  [--threads N] [--writers W] [--incr I] "
          "[--duration-ms D] [--keys K]\n\t  [--slots S] [--max-value B] [--writer-us U]\n"
          "\t  [--quiet] [--keep-test-store] [--scrub] [--store NAME|PATH|hbm:NAME]\n",
          prog);
}

}  // namespace stress
