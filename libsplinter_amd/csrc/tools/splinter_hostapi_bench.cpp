// splinter_hostapi_bench — per-call C API throughput and latency (the reference's own metric:
// splinter_set / splinter_get calls from host threads, reference splinter_stress.c:64-188) on
// any store, including "hbm:NAME" stores served by the device command ring (cmd_ring.hpp).
//
//   splinter_hostapi_bench [--store NAME] [--threads T] [--seconds S] [--keys K]
//                          [--value-len L] [--set-frac F] [--append-check N] [--batch B]
//                          [--procs P]
//
// --procs P: P processes issue the calls (T threads each) against the one store: the parent
// creates it (and, on hbm:, hosts its ring server), P-1 children -- spawned before the parent
// touches the GPU, released through a pipe once the keys are in -- open it and submit to the same
// server.  ops/s is the sum over processes; p50_us etc. are the parent's, procs_p50_us lists all.
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
#include <dlfcn.h>
#include <sched.h>
#include <spawn.h>
#include <sys/resource.h>
#include <sys/wait.h>
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
  int procs = 1;
  bool attach = false;  // child of --procs: open the parent's store
  int go_fd = -1;       // child: read one byte before starting
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

// 0 own ring worker, 1 ring server host, 2 client of the owner's server (hbm: stores), -1 otherwise
int ring_mode() {
  using Mode = int (*)(spl_store*);
  auto f = (Mode)dlsym(RTLD_DEFAULT, "spl_hbm_ring_mode");
  return f && spl_store_current() ? f(spl_store_current()) : -1;
}

struct RunStats {
  double el = 0;
  uint64_t calls = 0, ok = 0, again = 0, fail = 0;
  double p50 = 0, p90 = 0, p99 = 0, sp50 = 0, sp99 = 0, gp50 = 0, gp99 = 0;
  // process CPU over the timed window (every thread, the runtime's included): user / system
  // seconds and context switches -- tells a CPU-bound caller population from a GPU-bound one
  double usr = 0, sys = 0;
  long vcsw = 0, ivcsw = 0;
};

inline double tv_s(const timeval& t) { return (double)t.tv_sec + 1e-6 * (double)t.tv_usec; }

// T threads, set/get mix over K keys for S seconds, every call timed
RunStats run_calls(const Args& a, size_t max_val, const std::string& val) {
  using clk = std::chrono::steady_clock;
  std::atomic<bool> go{false}, stop{false};
  std::vector<std::vector<float>> lat_set(a.threads), lat_get(a.threads);
  std::vector<uint64_t> ok(a.threads, 0), again(a.threads, 0), fail(a.threads, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < a.threads; ++t)
    th.emplace_back([&, t] {
      uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1) + 0x5851F42D4C957F2Dull * (uint64_t)getpid();
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
  rusage ru0{}, ru1{};
  getrusage(RUSAGE_SELF, &ru0);
  const auto t0 = clk::now();
  go.store(true, std::memory_order_release);
  std::this_thread::sleep_for(std::chrono::duration<double>(a.seconds));
  stop.store(true);
  for (auto& x : th) x.join();
  RunStats r;
  r.el = std::chrono::duration<double>(clk::now() - t0).count();
  getrusage(RUSAGE_SELF, &ru1);
  r.usr = tv_s(ru1.ru_utime) - tv_s(ru0.ru_utime);
  r.sys = tv_s(ru1.ru_stime) - tv_s(ru0.ru_stime);
  r.vcsw = ru1.ru_nvcsw - ru0.ru_nvcsw;
  r.ivcsw = ru1.ru_nivcsw - ru0.ru_nivcsw;
  std::vector<float> ls, lg, la;
  for (int t = 0; t < a.threads; ++t) {
    ls.insert(ls.end(), lat_set[t].begin(), lat_set[t].end());
    lg.insert(lg.end(), lat_get[t].begin(), lat_get[t].end());
    r.ok += ok[t]; r.again += again[t]; r.fail += fail[t];
  }
  la = ls;
  la.insert(la.end(), lg.begin(), lg.end());
  r.calls = la.size();
  r.p50 = pct(la, 0.5); r.p90 = pct(la, 0.9); r.p99 = pct(la, 0.99);
  r.sp50 = pct(ls, 0.5); r.sp99 = pct(ls, 0.99); r.gp50 = pct(lg, 0.5); r.gp99 = pct(lg, 0.99);
  return r;
}

// child of --procs: wait for the parent's go byte, open its store, run, report one line
int attach_main(const Args& a) {
  char b = 0;
  if (a.go_fd >= 0) {
    if (read(a.go_fd, &b, 1) != 1 || b != 'g') return 3;  // the parent gave up
    close(a.go_fd);
  }
  if (splinter_open(a.store.c_str()) != 0) {
    fprintf(stderr, "open %s failed: %s\n", a.store.c_str(), strerror(errno));
    return 1;
  }
  const RunStats r = run_calls(a, 4096, std::string(a.value_len, 'v'));
  printf("%llu %llu %llu %.6f %.3f %d\n", (unsigned long long)r.calls, (unsigned long long)r.ok,
         (unsigned long long)r.fail, r.el, r.p50, ring_mode());
  fflush(stdout);
  splinter_close();
  return r.fail ? 1 : 0;
}

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
    else if (s == "--procs") a.procs = atoi(nxt());
    else if (s == "--attach") a.attach = true;
    else if (s == "--go-fd") a.go_fd = atoi(nxt());
    else { fprintf(stderr, "unknown option %s\n", s.c_str()); return 2; }
  }
  if (a.batch > 0) return batch_main(a);
  if (a.attach) return attach_main(a);
  // --procs: children first, before this process touches the GPU (no fork of an initialised runtime)
  struct Child {
    pid_t pid;
    int out;
  };
  std::vector<Child> kids;
  int go[2] = {-1, -1};
  if (a.procs > 1) {
    if (pipe(go) != 0) return 1;
    char self[4096];
    const ssize_t n = readlink("/proc/self/exe", self, sizeof self - 1);
    if (n <= 0) return 1;
    self[n] = 0;
    for (int c = 1; c < a.procs; ++c) {
      int out[2];
      if (pipe(out) != 0) return 1;
      posix_spawn_file_actions_t fa;
      posix_spawn_file_actions_init(&fa);
      posix_spawn_file_actions_adddup2(&fa, out[1], 1);
      posix_spawn_file_actions_addclose(&fa, out[0]);
      posix_spawn_file_actions_addclose(&fa, go[1]);
      const std::string th = std::to_string(a.threads), sec = std::to_string(a.seconds),
                        ks = std::to_string(a.keys), vl = std::to_string(a.value_len),
                        sf = std::to_string(a.set_frac), gf = std::to_string(go[0]);
      const char* av[] = {self, "--attach", "--store", a.store.c_str(), "--threads", th.c_str(), "--seconds",
                          sec.c_str(), "--keys", ks.c_str(), "--value-len", vl.c_str(), "--set-frac", sf.c_str(),
                          "--go-fd", gf.c_str(), nullptr};
      pid_t pid = 0;
      const int rc = posix_spawn(&pid, self, &fa, nullptr, (char* const*)av, environ);
      posix_spawn_file_actions_destroy(&fa);
      close(out[1]);
      if (rc != 0) { fprintf(stderr, "spawn failed: %s\n", strerror(rc)); return 1; }
      kids.push_back({pid, out[0]});
    }
    close(go[0]);
  }
  auto release_kids = [&](char b) {
    if (go[1] < 0) return;
    for (size_t i = 0; i < kids.size(); ++i) (void)!write(go[1], &b, 1);
    close(go[1]);
    go[1] = -1;
  };
  const size_t max_val = 4096;
  if (splinter_create(a.store.c_str(), (size_t)a.keys * 2 + 1024, max_val) != 0) {
    fprintf(stderr, "create %s failed: %s\n", a.store.c_str(), strerror(errno));
    release_kids('x');
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
    if (bad) { fprintf(stderr, "prepopulate: %d failures\n", bad.load()); release_kids('x'); return 1; }
  }
  release_kids('g');
  const RunStats st = run_calls(a, max_val, val);
  const double el = st.el;
  uint64_t calls = st.calls, tok = st.ok, tag = st.again, tf = st.fail;
  double total_rate = (double)st.calls / st.el, ok_rate = (double)st.ok / st.el;
  std::string p50s = std::to_string(st.p50);
  int kid_fail = 0;
  for (auto& k : kids) {
    char line[256] = {0};
    size_t got = 0;
    ssize_t r;
    while (got < sizeof line - 1 && (r = read(k.out, line + got, sizeof line - 1 - got)) > 0) got += (size_t)r;
    close(k.out);
    int wst = 0;
    (void)waitpid(k.pid, &wst, 0);
    unsigned long long c = 0, o = 0, f = 0;
    double kel = 0, kp50 = 0;
    if (sscanf(line, "%llu %llu %llu %lf %lf", &c, &o, &f, &kel, &kp50) < 5 || kel <= 0 ||
        !WIFEXITED(wst) || WEXITSTATUS(wst) != 0) {
      ++kid_fail;
      continue;
    }
    calls += c; tok += o; tf += f;
    total_rate += (double)c / kel;
    ok_rate += (double)o / kel;
    p50s += ", " + std::to_string(kp50);
  }
  int rc = tf || kid_fail ? 1 : 0;
  if (kid_fail) fprintf(stderr, "%d child process(es) failed\n", kid_fail);

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
  printf("{\"store\": \"%s\", \"threads\": %d, \"procs\": %d, \"seconds\": %.3f, \"calls\": %llu, \"ops_per_s\": %.1f, "
         "\"successful_ops_per_s\": %.1f, \"eagain\": %llu, \"failures\": %llu, "
         "\"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f, \"set_p50_us\": %.2f, \"set_p99_us\": %.2f, "
         "\"get_p50_us\": %.2f, \"get_p99_us\": %.2f, \"procs_p50_us\": [%s], \"ring_mode\": %d, \"value_len\": %d, "
         "\"set_frac\": %.2f, \"append_check\": %d, \"cpu_usr_s\": %.3f, \"cpu_sys_s\": %.3f, "
         "\"cpu_us_per_call\": %.2f, \"vcsw_per_call\": %.2f, \"ivcsw_per_call\": %.2f}\n",
         a.store.c_str(), a.threads, a.procs, el, (unsigned long long)calls, total_rate, ok_rate,
         (unsigned long long)tag, (unsigned long long)tf, st.p50, st.p90, st.p99, st.sp50, st.sp99, st.gp50, st.gp99,
         p50s.c_str(), ring_mode(), a.value_len, a.set_frac, app_ok, st.usr, st.sys,
         st.calls ? 1e6 * (st.usr + st.sys) / (double)st.calls : 0.0,
         st.calls ? (double)st.vcsw / (double)st.calls : 0.0, st.calls ? (double)st.ivcsw / (double)st.calls : 0.0);
  splinter_close();
  spl_unlink(a.store.c_str());
  return rc;
}
