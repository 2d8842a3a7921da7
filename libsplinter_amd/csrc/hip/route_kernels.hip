// route_kernels.hip — device side of the C1 routing collective (SURVEY §2.10 C1,
// parallel/sharded.py RoutedKV): pack a client batch into fixed-capacity
// per-destination segments, and gather routed responses back into client order.
//
// Why fixed capacity: an all-to-all with EQUAL splits needs no host-side count
// exchange, so a routed set/get step has no host synchronisation at all and
// the RCCL transfers overlap compute queued on other streams.  The receiver
// learns the live rows of each segment from a device-side count all-to-all
// and the owner kernels skip dead rows (Seg in arena_kernels.hip).  A
// destination segment that overflows `cap` returns EAGAIN for the excess ops
// (the reference's contention status, splinter.h:398-412): the caller retries.
//
// Pack layout (rank r, destination d, row j < cap): row index d*cap + j of
//   kout [world*cap, kstride]  key record
//   lout [world*cap]           value length          (sets only)
//   vout [world*cap, vwidth]   value prefix (16-B)   (sets only)
// pos[i] = d*cap + j for client op i, or -1 when its segment was full.
//
// Work split: 256-thread blocks, 4 items per thread per round (1024 ops), a
// block-local LDS histogram gives each op its rank inside (block, dest), ONE
// global atomic per destination per round reserves the block's range, and the
// value rows are copied wave-cooperatively (64 lanes stream consecutive 16-B
// chunks of consecutive rows: coalesced reads and writes).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "arena_dev.hpp"
#include "arena_api.h"

using namespace spl;
using namespace spl::dev;

namespace {

constexpr int kRB = 256;         // threads per block
constexpr int kRU = 4;           // items per thread per round
constexpr int kMaxWorld = 256;   // destinations supported by the LDS histogram

__device__ __forceinline__ int shard_of_hash(uint64_t h, int world) {
  return (int)(((h >> 40) & 0xFFFFFFull) % (uint64_t)world);  // == parallel/sharded.py shard_of
}

// Copy `C` 16-B chunks of each of the wave's 64 rows: row r (lane r's item)
// goes from src + r*sstride to dst + dpos(r)*dstride; rows with dpos < 0 or
// beyond n are skipped.  Lanes walk the flattened (row, chunk) space.
__device__ __forceinline__ void wave_copy_rows(const uint8_t* src_base, long sstride, uint8_t* dst, long dstride,
                                               long my_dpos, int C, int lane, int nvalid) {
  const int total = 64 * C;
  for (int c = lane; c < total; c += 64) {
    const int row = c / C, chunk = c - row * C;
    const long dp = __shfl(my_dpos, row);
    if (row < nvalid && dp >= 0)
      *(uint4*)(dst + dp * dstride + chunk * 16) = *(const uint4*)(src_base + row * sstride + chunk * 16);
  }
}

__global__ __launch_bounds__(kRB) void k_route_pack(const char* keys, int kstride, const uint8_t* vals, int vstride,
                                                    int vwidth, const uint32_t* lens, long n, int world, long cap,
                                                    int32_t* counts, int64_t* pos, char* kout, uint32_t* lout,
                                                    uint8_t* vout) {
  __shared__ int s_cnt[kMaxWorld];
  __shared__ int s_base[kMaxWorld];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long per_round = (long)kRB * kRU;
  for (int d = tid; d < world; d += kRB) s_cnt[d] = 0;
  __syncthreads();
  for (long base = blockIdx.x * per_round; base < n; base += (long)gridDim.x * per_round) {
    Key k[kRU];
    int dst[kRU], rk[kRU];
#pragma unroll
    for (int j = 0; j < kRU; ++j) {
      const long i = base + (long)j * kRB + tid;
      dst[j] = -1;
      if (i < n) {
        load_key(k[j], keys + i * (long)kstride, kstride);
        dst[j] = shard_of_hash(k[j].hash, world);
        rk[j] = atomicAdd(&s_cnt[dst[j]], 1);
      }
    }
    __syncthreads();
    for (int d = tid; d < world; d += kRB) {
      const int c = s_cnt[d];
      s_base[d] = c ? atomicAdd(&counts[d], c) : 0;
      s_cnt[d] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRU; ++j) {
      const long i = base + (long)j * kRB + tid;
      long p = -1;
      if (dst[j] >= 0) {
        const long slot = (long)s_base[dst[j]] + rk[j];
        if (slot < cap) p = (long)dst[j] * cap + slot;
        pos[i] = p;
      }
      if (p >= 0) {
        uint4* kr = (uint4*)(kout + p * (long)kstride);
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c * 16 < kstride) kr[c] = make_uint4(k[j].w[4 * c], k[j].w[4 * c + 1], k[j].w[4 * c + 2], k[j].w[4 * c + 3]);
        if (lout) lout[p] = lens[i];
      }
      if (vout) {
        const long w0 = base + (long)j * kRB + wave * 64;  // first item of this wave's row group
        const long left = n - w0;
        if (left > 0)
          wave_copy_rows(vals + w0 * (long)vstride, vstride, vout, vwidth, p, vwidth / 16, lane,
                         left < 64 ? (int)left : 64);
      }
    }
  }
}

__global__ __launch_bounds__(kRB) void k_route_gather(const int64_t* pos, long n, const int32_t* rstatus,
                                                      const uint32_t* rlens, const uint8_t* rvals, int rstride,
                                                      int32_t* status, uint32_t* out_lens, uint8_t* out, int ostride,
                                                      int copy_bytes) {
  const int lane = threadIdx.x & 63;
  const long wstep = (long)gridDim.x * kRB;
  for (long w0 = blockIdx.x * (long)kRB + (threadIdx.x & ~63); w0 < n; w0 += wstep) {
    const long i = w0 + lane;
    long p = -1;
    if (i < n) {
      p = pos[i];
      if (status) status[i] = p < 0 ? kAgain : rstatus[p];
      if (out_lens) out_lens[i] = p < 0 ? 0u : rlens[p];
    }
    if (out) {
      // source rows are read at rstride, written at ostride; client row i gets the routed row p
      const int C = copy_bytes / 16;
      const long left = n - w0;
      const int nvalid = left < 64 ? (int)left : 64;
      for (int c = lane; c < 64 * C; c += 64) {
        const int row = c / C, chunk = c - row * C;
        const long sp = __shfl(p, row);
        if (row < nvalid && sp >= 0)
          *(uint4*)(out + (w0 + row) * (long)ostride + chunk * 16) =
              *(const uint4*)(rvals + sp * (long)rstride + chunk * 16);
      }
    }
  }
}

inline int route_grid(long n, long per_block) {
  long g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > 256 * 8) g = 256 * 8;
  return (int)g;
}

}  // namespace

extern "C" {

int spl_route_pack(const char* keys, int kstride, const uint8_t* vals, int vstride, int vwidth, const uint32_t* lens,
                   long n, int world, long cap, int32_t* counts, int64_t* pos, char* kout, uint32_t* lout,
                   uint8_t* vout, hipStream_t s) {
  if (world < 1 || world > kMaxWorld || cap < 0) return (int)hipErrorInvalidValue;
  if ((kstride & 15) || kstride <= 0 || kstride > 64) return (int)hipErrorInvalidValue;
  if (vout && (!vals || !lens || !lout || (vstride & 15) || (vwidth & 15) || vwidth <= 0 || vwidth > vstride))
    return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(counts, 0, sizeof(int32_t) * (size_t)world, s);
  if (e != hipSuccess) return (int)e;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_route_pack, dim3(route_grid(n, (long)kRB * kRU)), dim3(kRB), 0, s, keys, kstride, vals,
                     vstride, vwidth, lens, n, world, cap, counts, pos, kout, lout, vout);
  return (int)hipGetLastError();
}

int spl_route_gather(const int64_t* pos, long n, const int32_t* rstatus, const uint32_t* rlens, const uint8_t* rvals,
                     int rstride, int32_t* status, uint32_t* out_lens, uint8_t* out, int ostride, hipStream_t s) {
  if (n <= 0) return 0;
  const int copy = rstride < ostride ? rstride : ostride;
  if (out && (!rvals || (rstride & 15) || (ostride & 15) || copy <= 0)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_route_gather, dim3(route_grid(n, kRB)), dim3(kRB), 0, s, pos, n, rstatus, rlens, rvals,
                     rstride, status, out_lens, out, ostride, copy);
  return (int)hipGetLastError();
}

}  // extern "C"
