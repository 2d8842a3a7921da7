// Probe: can a GPU worker poll a doorbell and read a request the HOST wrote into DEVICE memory
// (through the PCIe BAR), with no stale L2 lines, and how long does a host-write -> device-seen ->
// host-completion round trip take?  Two device-memory kinds: fine-grained (hipExtMallocWithFlags
// hipDeviceMallocFinegrained, host-dereferenceable) and a VMM chunk mmap'ed through its dmabuf.
// The kernel first reads every line (so a stale copy would sit in L2), then serves N requests:
// poll doorbell (system-scope load) until it changes, read the 256-B record, write its checksum and
// the sequence number to host memory.  Every wait is bounded by a wall-clock timeout.
//
// hipcc --offload-arch=gfx950 -O2 dev/debug/vram_doorbell_probe.hip -o /tmp/vram_probe && /tmp/vram_probe
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <algorithm>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../libsplinter_amd/csrc/hip/vmm_share.hpp"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint32_t ld32s(const void* p) {
  return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st32s(void* p, uint32_t v) {
  __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// lane 0 serves; door: device memory; rec: 64 u32 of device memory; out: host {seq, sum} pairs
__global__ void k_serve(const uint32_t* door, const uint32_t* rec, uint32_t* hout, int n, uint64_t timeout_ticks) {
  if (threadIdx.x != 0) return;
  // warm the lines into L2 / L1 with plain loads: a later stale hit would show up as a wrong sum
  uint32_t warm = door[0];
  for (int i = 0; i < 64; ++i) warm += rec[i];
  hout[2 * n + 2] = warm;
  uint32_t seen = 0;
  for (int k = 0; k < n; ++k) {
    const uint64_t t0 = wall_clock64();
    uint32_t d;
    while ((d = ld32s(door)) == seen) {
      if (wall_clock64() - t0 > timeout_ticks) { st32s(&hout[2 * n], 0xdead); return; }
      __builtin_amdgcn_s_sleep(1);
    }
    uint32_t sum = 0;
    for (int i = 0; i < 64; ++i) sum += ld32s(rec + i);
    st32s(&hout[2 * k + 1], sum);
    __builtin_amdgcn_s_waitcnt(0);
    st32s(&hout[2 * k], d);
    seen = d;
  }
  st32s(&hout[2 * n], 0x600d);
}

static int run(const char* kind, uint32_t* hdoor, uint32_t* hrec, const uint32_t* ddoor, const uint32_t* drec,
               uint32_t* hout, int n, int khz) {
  memset(hout, 0, sizeof(uint32_t) * (2 * n + 4));
  *(volatile uint32_t*)hdoor = 0;
  for (int i = 0; i < 64; ++i) ((volatile uint32_t*)hrec)[i] = 7;
  _mm_sfence();
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(k_serve, dim3(1), dim3(64), 0, s, ddoor, drec, hout, n, (uint64_t)khz * 2000);  // 2 s
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  std::vector<double> lat;
  int bad = 0;
  uint32_t tmp[64];
  for (int k = 0; k < n; ++k) {
    const uint32_t seq = (uint32_t)k + 1;
    uint32_t want = 0;
    for (int i = 0; i < 64; ++i) { tmp[i] = seq * 131u + (uint32_t)i; want += tmp[i]; }
    const auto t0 = std::chrono::steady_clock::now();
    memcpy(hrec, tmp, sizeof tmp);
    _mm_sfence();
    *(volatile uint32_t*)hdoor = seq;
    _mm_sfence();
    bool ok = false;
    while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(3)) {
      if (__atomic_load_n(&hout[2 * k], __ATOMIC_ACQUIRE) == seq) { ok = true; break; }
      if (__atomic_load_n(&hout[2 * n], __ATOMIC_ACQUIRE) == 0xdead) break;
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (!ok) { printf("{\"kind\": \"%s\", \"error\": \"request %d not served\"}\n", kind, k); bad = n; break; }
    if (hout[2 * k + 1] != want) ++bad;
    lat.push_back(us);
  }
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  std::sort(lat.begin(), lat.end());
  const double p50 = lat.empty() ? 0 : lat[lat.size() / 2], p99 = lat.empty() ? 0 : lat[lat.size() * 99 / 100];
  printf("{\"kind\": \"%s\", \"requests\": %d, \"wrong_payload\": %d, \"roundtrip_p50_us\": %.2f, \"p99_us\": %.2f}\n",
         kind, (int)lat.size(), bad, p50, p99);
  return bad ? 2 : 0;
}

int main() {
  const int n = 2000;
  int khz = 100000;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  uint32_t* hout = nullptr;
  CK(hipHostMalloc((void**)&hout, sizeof(uint32_t) * (2 * n + 4), hipHostMallocCoherent | hipHostMallocMapped));
  int rc = 0;
  // (a) host memory (the current ring's transport), the reference point
  {
    uint32_t* h = nullptr;
    CK(hipHostMalloc((void**)&h, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    rc |= run("host_coherent", h, h + 64, h, h + 64, hout, n, khz);
    CK(hipHostFree(h));
  }
  // (b) fine-grained device memory, dereferenced by the host
  {
    uint32_t* d = nullptr;
    if (hipExtMallocWithFlags((void**)&d, 2u << 20, hipDeviceMallocFinegrained) == hipSuccess) {
      hipPointerAttribute_t at{};
      (void)hipPointerGetAttributes(&at, d);
      printf("{\"kind\": \"fine_grained\", \"host_ptr\": %s}\n", at.hostPointer ? "true" : "false");
      if (at.hostPointer) rc |= run("fine_grained_device", (uint32_t*)at.hostPointer, (uint32_t*)at.hostPointer + 64, d,
                                    d + 64, hout, n, khz);
      CK(hipFree(d));
    } else {
      printf("{\"kind\": \"fine_grained\", \"error\": \"alloc\"}\n");
    }
  }
  // (c) a VMM chunk (coarse-grained device memory) through its dmabuf CPU mapping
  {
    spl::VmmArena v;
    if (v.create(0, 2u << 20, 2u << 20) == 0 && v.host_map()) {
      uint32_t* h = (uint32_t*)v.host_map();
      uint32_t* d = (uint32_t*)v.base();
      rc |= run("vmm_dmabuf", h, h + 64, d, d + 64, hout, n, khz);
    } else {
      printf("{\"kind\": \"vmm_dmabuf\", \"error\": \"map\"}\n");
    }
  }
  CK(hipHostFree(hout));
  return rc;
}
