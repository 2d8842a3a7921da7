// cpwait_probe.hip — what would a per-call worker woken by a command-processor wait cost, against
// the resident polling worker the ring uses today (csrc/hip/cmd_ring.hpp)?
//
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/cpwait_probe scripts/probes/cpwait_probe.hip
//   ./cpwait_probe            (one JSON line per measurement)
//
// 1. interference: a compute job (ALU-bound grid over every CU, events on its own stream) timed
//    alone, beside an idle RESIDENT poller of 32 one-wave workgroups (the ring worker's shape:
//    system-scope doorbell loads + s_sleep), and beside a stream parked in hipStreamWaitValue32
//    with the serving kernel queued behind it (no wave resident);
// 2. latency: one "call" = host store of a sequence number -> the serving kernel runs (either
//    the resident poller sees it, or the command processor releases the wait and dispatches the
//    queued kernel) -> it stores the number back into pinned host memory -> the host sees it;
// 3. queue sharing: with GPU_MAX_HW_QUEUES streams created, does a job on a stream that shares
//    the parked stream's hardware queue wait for the doorbell?  (bounded: the host rings the
//    doorbell after 2 s, so the parked wait always drains).
// Every kernel has an exit every wave reaches (stop flag or s_memrealtime bound).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void k_busy(float* out, int iters) {
  float a = (float)threadIdx.x * 1e-3f, b = 1.0000001f, c = 0.999999f;
  for (int i = 0; i < iters; ++i) {
    a = fmaf(a, b, 1e-7f);
    c = fmaf(c, b, -1e-7f);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + c;
}

__device__ inline uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// resident poller: lane 0 of every wave polls the doorbell; group 0 answers each new number.
// Exits on *stop or after max_ticks of the 100 MHz realtime clock.
__global__ void k_poller(const uint32_t* door, uint32_t* done, const uint32_t* stop, uint64_t max_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t seen = 0;
  while (true) {
    const uint32_t d = ld_sys(door);
    if (d != seen) {
      seen = d;
      if (blockIdx.x == 0 && threadIdx.x == 0) st_sys(done, d);
    }
    if (ld_sys(stop) != 0u) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
}

// the CP-released server: answers the number it was queued for
__global__ void k_serve(uint32_t* done, uint32_t v) {
  if (threadIdx.x == 0) st_sys(done, v);
}

static double time_busy(hipStream_t s, float* out, int blocks, int iters, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, s, out, iters);  // warm
  CK(hipStreamSynchronize(s));
  std::vector<float> ms;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, s));
    hipLaunchKernelGGL(k_busy, dim3(blocks), dim3(256), 0, s, out, iters);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float m = 0;
    CK(hipEventElapsedTime(&m, a, b));
    ms.push_back(m);
  }
  std::sort(ms.begin(), ms.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms[ms.size() / 2];
}

int main() {
  using clk = std::chrono::steady_clock;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 8, iters = 200000, reps = 21;
  float* out = nullptr;
  CK(hipMalloc(&out, sizeof(float) * blocks * 256));
  uint32_t* hw = nullptr;  // pinned host words: door, done, stop
  CK(hipHostMalloc((void**)&hw, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  volatile uint32_t* door = hw;
  volatile uint32_t* done = hw + 16;
  volatile uint32_t* stop = hw + 32;
  *door = 0; *done = 0; *stop = 0;
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  const uint64_t max_ticks = 100000000ull * 20;  // 20 s

  // 1. interference
  const double alone = time_busy(sa, out, blocks, iters, reps);
  *stop = 0;
  hipLaunchKernelGGL(k_poller, dim3(32), dim3(64), 0, sb, (const uint32_t*)door, (uint32_t*)done,
                     (const uint32_t*)stop, max_ticks);
  const double resident = time_busy(sa, out, blocks, iters, reps);
  // 2a. latency through the resident poller
  std::vector<double> lat_res;
  bool lost = false;
  // a call not answered within 1 s ends the probe (the kernels still drain: stop / doorbell)
  auto wait_done = [&](uint32_t i, clk::time_point t0) {
    while (*done != i)
      if (std::chrono::duration<double>(clk::now() - t0).count() > 1.0) return false;
    return true;
  };
  for (uint32_t i = 1; i <= 2000 && !lost; ++i) {
    const auto t0 = clk::now();
    *door = i;
    if (!wait_done(i, t0)) { lost = true; break; }
    lat_res.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  *stop = 1;
  CK(hipStreamSynchronize(sb));
  *stop = 0;
  // parked CP wait: the doorbell is far ahead of what the host writes during the busy runs
  *door = 0; *done = 0;
  CK(hipStreamWaitValue32(sb, (void*)door, 1u, hipStreamWaitValueGte, 0xffffffffu));
  hipLaunchKernelGGL(k_serve, dim3(1), dim3(64), 0, sb, (uint32_t*)done, 1u);
  const double parked = time_busy(sa, out, blocks, iters, reps);
  *door = 1;
  CK(hipStreamSynchronize(sb));
  // 2b. latency through CP-released kernels: keep `ahead` (wait, serve) pairs queued
  std::vector<double> lat_cp;
  *door = 0; *done = 0;
  const uint32_t calls = 2000, ahead = 32;
  uint32_t queued = 0;
  auto enqueue = [&](uint32_t v) {
    CK(hipStreamWaitValue32(sb, (void*)door, v, hipStreamWaitValueGte, 0xffffffffu));
    hipLaunchKernelGGL(k_serve, dim3(1), dim3(64), 0, sb, (uint32_t*)done, v);
  };
  for (; queued < ahead; ++queued) enqueue(queued + 1);
  for (uint32_t i = 1; i <= calls && !lost; ++i) {
    const auto t0 = clk::now();
    *door = i;
    if (!wait_done(i, t0)) { lost = true; break; }
    lat_cp.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    if (queued < calls) enqueue(++queued);
  }
  *door = 0xfffffff0u;  // releases every wait still queued
  CK(hipStreamSynchronize(sb));
  if (lost || lat_res.empty() || lat_cp.empty()) {
    fprintf(stderr, "a call was not answered within 1 s\n");
    return 1;
  }
  auto pct = [](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (double)(v.size() - 1))];
  };
  printf("{\"probe\": \"interference\", \"busy_ms_alone\": %.3f, \"busy_ms_resident_poller\": %.3f, "
         "\"busy_ms_parked_cp_wait\": %.3f, \"resident_cost_pct\": %.1f, \"parked_cost_pct\": %.1f}\n",
         alone, resident, parked, 100.0 * (resident / alone - 1.0), 100.0 * (parked / alone - 1.0));
  printf("{\"probe\": \"latency\", \"resident_p50_us\": %.2f, \"resident_p99_us\": %.2f, \"cp_wait_p50_us\": %.2f, "
         "\"cp_wait_p99_us\": %.2f}\n",
         pct(lat_res, 0.5), pct(lat_res, 0.99), pct(lat_cp, 0.5), pct(lat_cp, 0.99));
  fflush(stdout);

  // 4. interference under LIVE calls: one client thread issues calls back to back while the busy
  // job is timed -- served by the resident poller, or by CP-released one-shot kernels
  auto live = [&](bool cp) {
    *door = 0; *done = 0; *stop = 0;
    std::atomic<bool> quit{false};
    std::atomic<uint64_t> ncalls{0};
    uint32_t q = 0;
    if (!cp)
      hipLaunchKernelGGL(k_poller, dim3(32), dim3(64), 0, sb, (const uint32_t*)door, (uint32_t*)done,
                         (const uint32_t*)stop, max_ticks);
    else
      for (; q < ahead; ++q) enqueue(q + 1);
    std::thread client([&] {
      for (uint32_t i = 1; !quit.load(std::memory_order_relaxed); ++i) {
        const auto t0 = clk::now();
        *door = i;
        if (!wait_done(i, t0)) { lost = true; return; }
        ncalls.fetch_add(1, std::memory_order_relaxed);
        if (cp) enqueue(++q);
      }
    });
    const auto t0 = clk::now();
    const double ms = time_busy(sa, out, blocks, iters, reps);
    const double secs = std::chrono::duration<double>(clk::now() - t0).count();
    quit = true;
    client.join();
    if (cp) *door = 0xfffffff0u;
    else *stop = 1;
    CK(hipStreamSynchronize(sb));
    *stop = 0;
    printf("{\"probe\": \"live_calls\", \"server\": \"%s\", \"busy_ms\": %.3f, \"cost_pct\": %.1f, "
           "\"calls_per_s\": %.0f}\n", cp ? "cp_wait_one_shot" : "resident_poller", ms,
           100.0 * (ms / alone - 1.0), (double)ncalls.load() / secs);
    fflush(stdout);
  };
  live(false);
  live(true);
  if (lost) { fprintf(stderr, "a live call was not answered within 1 s\n"); return 1; }

  // 5. queue sharing with the parked stream at HIGH priority and every other stream normal
  {
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t sh;
    CK(hipStreamCreateWithPriority(&sh, hipStreamNonBlocking, hi));
    std::vector<hipStream_t> sn(8);
    for (auto& s2 : sn) CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    int blocked = 0;
    for (size_t j = 0; j < sn.size(); ++j) {
      *door = 0; *done = 0;
      CK(hipStreamWaitValue32(sh, (void*)door, 1u, hipStreamWaitValueGte, 0xffffffffu));
      hipLaunchKernelGGL(k_serve, dim3(1), dim3(64), 0, sh, (uint32_t*)done, 1u);
      hipEvent_t ev;
      CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      const auto t0 = clk::now();
      hipLaunchKernelGGL(k_busy, dim3(cus), dim3(64), 0, sn[j], out, 100);
      CK(hipEventRecord(ev, sn[j]));
      bool finished = false;
      while (std::chrono::duration<double>(clk::now() - t0).count() < 1.0)
        if (hipEventQuery(ev) == hipSuccess) { finished = true; break; }
      *door = 1;
      CK(hipStreamSynchronize(sh));
      CK(hipEventSynchronize(ev));
      CK(hipEventDestroy(ev));
      blocked += finished ? 0 : 1;
    }
    printf("{\"probe\": \"queue_sharing_high_priority_park\", \"normal_streams\": %zu, \"blocked\": %d}\n",
           sn.size(), blocked);
    fflush(stdout);
    for (auto& s2 : sn) CK(hipStreamDestroy(s2));
    CK(hipStreamDestroy(sh));
  }

  // 3. queue sharing: park a wait on the first of nq streams, time a job on each of the others
  const char* e = getenv("GPU_MAX_HW_QUEUES");
  const int hwq = e ? atoi(e) : 4;
  const int nq = 2 * hwq;
  std::vector<hipStream_t> ss(nq);
  for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int j = 1; j < nq; ++j) {
    *door = 0; *done = 0;
    CK(hipStreamWaitValue32(ss[0], (void*)door, 1u, hipStreamWaitValueGte, 0xffffffffu));
    hipLaunchKernelGGL(k_serve, dim3(1), dim3(64), 0, ss[0], (uint32_t*)done, 1u);
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const auto t0 = clk::now();
    hipLaunchKernelGGL(k_busy, dim3(cus), dim3(64), 0, ss[j], out, 100);
    CK(hipEventRecord(ev, ss[j]));
    bool finished = false;
    while (std::chrono::duration<double>(clk::now() - t0).count() < 2.0)
      if (hipEventQuery(ev) == hipSuccess) { finished = true; break; }
    const double waited_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    *door = 1;  // always release the parked wait
    CK(hipStreamSynchronize(ss[0]));
    CK(hipEventSynchronize(ev));
    CK(hipEventDestroy(ev));
    printf("{\"probe\": \"queue_sharing\", \"hw_queues\": %d, \"parked_stream\": 0, \"job_stream\": %d, "
           "\"job_blocked_by_parked_wait\": %s, \"job_ms\": %.3f}\n",
           hwq, j, finished ? "false" : "true", waited_ms);
    fflush(stdout);
  }
  for (auto& s : ss) CK(hipStreamDestroy(s));
  CK(hipStreamDestroy(sa));
  CK(hipStreamDestroy(sb));
  CK(hipHostFree(hw));
  CK(hipFree(out));
  return 0;
}
