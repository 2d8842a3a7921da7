// kv_streams.hip — native submission of a KV step issued by many concurrent client streams.
//
// BASELINE config #2 runs 32 concurrent writer streams (plus readers).  Issuing their batches
// from Python costs ~30-60 µs of host time per launch (stream context switch, event record /
// wait, output allocation, ctypes), so 64 streams made the step host-bound: the GPU trace showed
// the last streams' kernels starting ~1 ms into a ~5 ms KV phase with idle queues before them
// (profiles/r2_bench_ws32_kernel_stats.csv).  Here the fan-out is one native call: each client
// stream waits on the origin stream's start event, runs its slice of the step's set (writers) or
// get (readers) batch through the regular batch launchers, and records its done event, which the
// origin stream then waits on.  Streams keep their identity and independence: every slice is
// its own launch on its own stream (the HIP runtime maps them onto GPU_MAX_HW_QUEUES hardware
// queues per priority: writers at normal priority, readers at high).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "arena_api.h"

namespace {

struct KvStreams {
  int nw = 0, nr = 0;
  std::vector<hipStream_t> s;  // nw writers, then nr readers
  std::vector<hipEvent_t> done;
  hipEvent_t start = nullptr;
};

}  // namespace

extern "C" {

void* spl_kvs_create(int writers, int readers) {
  if (writers < 1 || readers < 1 || writers + readers > 256) return nullptr;
  auto* k = new KvStreams();
  k->nw = writers;
  k->nr = readers;
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  for (int i = 0; i < writers + readers; ++i) {
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    if (hipStreamCreateWithPriority(&st, hipStreamNonBlocking, i < writers ? 0 : hi) != hipSuccess ||
        hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      delete k;
      return nullptr;
    }
    k->s.push_back(st);
    k->done.push_back(ev);
  }
  (void)hipEventCreateWithFlags(&k->start, hipEventDisableTiming);
  return k;
}

void spl_kvs_destroy(void* h) {
  auto* k = (KvStreams*)h;
  if (!k) return;
  for (auto st : k->s) {
    (void)hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
  }
  for (auto ev : k->done) (void)hipEventDestroy(ev);
  if (k->start) (void)hipEventDestroy(k->start);
  delete k;
}

// One step: writers split [0, n_set) of the set batch evenly, readers split [0, n_get) of the get
// batch; the origin stream continues after every slice.  Row-major batches (keys kstride B per
// row, values / outputs vstride / ostride B per row), per-op status and lengths.
int spl_kvs_step(void* h, spl_arena_t a, hipStream_t origin, const char* skeys, int kstride, const uint8_t* svals,
                 int vstride, const uint32_t* slens, long n_set, int32_t* sstatus, const char* gkeys, uint8_t* gout,
                 int ostride, uint32_t* glens, long n_get, int32_t* gstatus, int max_retry, uint64_t* stats) {
  auto* k = (KvStreams*)h;
  if (!k) return (int)hipErrorInvalidValue;
  hipError_t e = hipEventRecord(k->start, origin);
  if (e != hipSuccess) return (int)e;
  const int nw = n_set > 0 ? k->nw : 0, nr = n_get > 0 ? k->nr : 0;
  for (int w = 0; w < nw; ++w) {
    const long b = n_set * w / nw, end = n_set * (w + 1) / nw;
    if (end <= b) continue;
    hipStream_t st = k->s[w];
    (void)hipStreamWaitEvent(st, k->start, 0);
    int rc = spl_arena_set(a, skeys + b * (long)kstride, kstride, svals + b * (long)vstride, vstride, slens + b,
                           end - b, sstatus ? sstatus + b : nullptr, max_retry, stats, st);
    if (rc) return rc;
    (void)hipEventRecord(k->done[w], st);
    (void)hipStreamWaitEvent(origin, k->done[w], 0);
  }
  for (int r = 0; r < nr; ++r) {
    const long b = n_get * r / nr, end = n_get * (r + 1) / nr;
    if (end <= b) continue;
    hipStream_t st = k->s[k->nw + r];
    (void)hipStreamWaitEvent(st, k->start, 0);
    int rc = spl_arena_get(a, gkeys + b * (long)kstride, kstride, gout ? gout + b * (long)ostride : nullptr, ostride,
                           glens ? glens + b : nullptr, end - b, gstatus ? gstatus + b : nullptr, max_retry, stats, st);
    if (rc) return rc;
    (void)hipEventRecord(k->done[k->nw + r], st);
    (void)hipStreamWaitEvent(origin, k->done[k->nw + r], 0);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
