// Probe: can the host map an HBM allocation zero-copy through its dmabuf file descriptor?
// (hipMemCreate chunk -> hipMemExportToShareableHandle(fd) -> mmap(fd) on the CPU)
// Prints one JSON line; exit 0 either way unless HIP itself fails.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <unistd.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("{\"hip_error\": \"%s\", \"at\": \"%s\"}\n", hipGetErrorString(e_), #x); return 1; } } while (0)

int main() {
  const size_t bytes = 64ull << 20;
  hipMemAllocationProp p = {};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  hipMemGenericAllocationHandle_t h;
  CK(hipMemCreate(&h, bytes, &p, 0));
  void* d = nullptr;
  CK(hipMemAddressReserve(&d, bytes, 0, nullptr, 0));
  CK(hipMemMap(d, bytes, 0, h, 0));
  hipMemAccessDesc a = {};
  a.location = p.location;
  a.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(d, bytes, &a, 1));
  CK(hipMemset(d, 0x5A, bytes));
  const uint64_t magic = 0x53504C494E544552ull;
  CK(hipMemcpy(d, &magic, 8, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  int fd = -1;
  CK(hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
  void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    printf("{\"mmap\": \"failed\", \"errno\": %d, \"err\": \"%s\"}\n", errno, strerror(errno));
    return 0;
  }
  volatile uint64_t* hv = (volatile uint64_t*)m;
  const uint64_t r0 = hv[0], r1 = hv[1], rlast = hv[bytes / 8 - 1];
  // latency of dependent 8-B host reads through the mapping
  auto t0 = std::chrono::steady_clock::now();
  uint64_t acc = 0;
  const int n = 2000;
  for (int i = 0; i < n; ++i) acc += hv[(size_t)(i * 4099) % (bytes / 8)];
  auto t1 = std::chrono::steady_clock::now();
  // host write, device sees it
  hv[2] = 0x1122334455667788ull;
  __sync_synchronize();
  uint64_t back = 0;
  CK(hipMemcpy(&back, (char*)d + 16, 8, hipMemcpyDeviceToHost));
  printf("{\"mmap\": \"ok\", \"magic_ok\": %s, \"fill_ok\": %s, \"host_read_ns\": %.1f, \"host_write_seen_by_device\": %s, \"acc\": %llu}\n",
         r0 == magic ? "true" : "false", (r1 == 0x5A5A5A5A5A5A5A5Aull && rlast == 0x5A5A5A5A5A5A5A5Aull) ? "true" : "false",
         std::chrono::duration<double, std::nano>(t1 - t0).count() / n, back == 0x1122334455667788ull ? "true" : "false",
         (unsigned long long)acc);
  munmap(m, bytes);
  close(fd);
  CK(hipMemUnmap(d, bytes));
  CK(hipMemAddressFree(d, bytes));
  CK(hipMemRelease(h));
  return 0;
}
