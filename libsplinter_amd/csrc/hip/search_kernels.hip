// search_kernels.hip — fused brute-force vector search over an HBM arena
// (K7/K8 of SURVEY §2.10).
//
// Reference semantics (/root/reference/splinter_cli_cmd_search.c:43-72,
// :374-416): for every embedded slot compute cosine similarity and euclidean
// distance to the query, drop candidates below min-sim / above max-dist,
// order by similarity descending then distance ascending, keep `limit`.
// The reference does this with scalar loops and qsort on one CPU thread.
//
// Pass 1 streams the slot array once for a whole batch of queries: one wave
// scores 4 slots per iteration (64 lanes x 12 dims per 3072-B vector, twelve
// coalesced 1-KiB loads in flight per wave), queries live in LDS, the dot
// products and the slot norm come out of the same registers, and each wave
// keeps a running top-K per query in LDS (insertions are rare once warm).
// Pass 2 merges the per-wave lists per query.  Memory-bound: ~3.1 KB/slot.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

#include "arena_dev.hpp"
#include "search_api.h"

namespace {

constexpr int kD = 768;
constexpr int kWaves = 4;
constexpr int kMaxQ = 16;  // queries per launch (the host splits larger batches)
constexpr int kMaxK = 32;
constexpr int kUnroll = 4;  // slots per wave iteration

struct Cand {
  float sim;
  float dist;
  uint32_t idx;
  uint32_t pad;
};

__device__ __forceinline__ bool better(float sa, float da, uint32_t ia, float sb, float db, uint32_t ib) {
  if (sa != sb) return sa > sb;
  if (da != db) return da < db;
  return ia < ib;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// insert c into the sorted list L[0..n) of capacity K; returns the new count
__device__ __forceinline__ int insert(Cand* L, int n, int K, const Cand& c) {
  if (n == K && !better(c.sim, c.dist, c.idx, L[K - 1].sim, L[K - 1].dist, L[K - 1].idx)) return n;
  int p = n < K ? n : K - 1;
  while (p > 0 && better(c.sim, c.dist, c.idx, L[p - 1].sim, L[p - 1].dist, L[p - 1].idx)) {
    L[p] = L[p - 1];
    --p;
  }
  L[p] = c;
  return n < K ? n + 1 : n;
}

__global__ __launch_bounds__(256) void k_score_topk(spl_arena_t aa, const float* __restrict__ queries, int nq, int K,
                                                    float min_sim, float max_dist, uint64_t mask, Cand* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float Qs[kMaxQ * kD];
  __shared__ float qn[kMaxQ];
  __shared__ Cand top[kWaves][kMaxQ][kMaxK];
  __shared__ int cnt[kWaves][kMaxQ];
  using namespace spl;
  using namespace spl::dev;
  const Arena a{(uint8_t*)aa.base, aa.slots, aa.max_val, aa.stride, aa.flags};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < nq * kD; i += 256) Qs[i] = queries[i];
  if (tid < kMaxQ * kWaves) cnt[tid / kMaxQ][tid % kMaxQ] = 0;
  __syncthreads();
  if (tid < nq) {
    float s = 0.f;
    for (int d = 0; d < kD; ++d) s += Qs[tid * kD + d] * Qs[tid * kD + d];
    qn[tid] = s;
  }
  __syncthreads();

  const long gw = (long)blockIdx.x * kWaves + wave, nw = (long)gridDim.x * kWaves;
  for (long base = gw * kUnroll; base < (long)a.slots; base += nw * kUnroll) {
    float4 e[kUnroll][3];
    bool live[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const long i = base + u;
      live[u] = false;
      if (i < (long)a.slots) {
        const uint8_t* s = a.slot((size_t)i);
        const uint64_t h = *(const uint64_t*)(s + kOffHash);
        live[u] = h != 0 && (!mask || (*(const uint64_t*)(s + kOffBloom) & mask) == mask);
      }
      if (live[u]) {
        const float4* v4 = (const float4*)(a.slot((size_t)i) + kOffEmbed);
#pragma unroll
        for (int c = 0; c < 3; ++c) e[u][c] = v4[lane + 64 * c];
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (!live[u]) continue;  // wave-uniform
      float en = 0.f;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        en += e[u][c].x * e[u][c].x + e[u][c].y * e[u][c].y + e[u][c].z * e[u][c].z + e[u][c].w * e[u][c].w;
      en = wave_sum(en);
      if (en < 1e-12f) continue;  // zero vector: not embedded (reference splinference.cpp:129-133)
      const float enr = sqrtf(en);
      for (int q = 0; q < nq; ++q) {
        const float4* q4 = (const float4*)(Qs + q * kD);
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float4 qq = q4[lane + 64 * c];
          dot += e[u][c].x * qq.x + e[u][c].y * qq.y + e[u][c].z * qq.z + e[u][c].w * qq.w;
        }
        dot = wave_sum(dot);
        const float sim = dot / (enr * sqrtf(qn[q]) + 1e-30f);
        const float dist = sqrtf(fmaxf(en + qn[q] - 2.f * dot, 0.f));
        if (sim < min_sim || dist > max_dist) continue;
        if (lane == 0) cnt[wave][q] = insert(top[wave][q], cnt[wave][q], K, Cand{sim, dist, (uint32_t)(base + u), 0});
      }
    }
  }
  __syncthreads();
  for (int q = 0; q < nq; ++q) {
    Cand* dst = out + (((long)blockIdx.x * kWaves + wave) * nq + q) * K;
    const int n = cnt[wave][q];
    for (int j = lane; j < K; j += 64)
      dst[j] = j < n ? top[wave][q][j] : Cand{-FLT_MAX, FLT_MAX, 0xffffffffu, 0};
  }
}

// Merge: one block per query.  Each thread folds a strided subset of the
// per-wave lists into its own sorted list (LDS), then the 256 sorted lists
// are merged pairwise in a tree (log2 256 = 8 rounds).
__global__ __launch_bounds__(256) void k_merge(const Cand* __restrict__ cand, long lists, int nq, int K,
                                               Cand* __restrict__ result) {
  __shared__ Cand L[256][kMaxK];
  __shared__ int n[256];
  const int q = blockIdx.x, tid = threadIdx.x;
  int c = 0;
  for (long l = tid; l < lists; l += 256) {
    const Cand* src = cand + (l * nq + q) * K;
    for (int j = 0; j < K; ++j) {
      const Cand x = src[j];
      if (x.idx == 0xffffffffu) break;
      // source lists are sorted: once one entry misses a full list, the rest will too
      if (c == K && !better(x.sim, x.dist, x.idx, L[tid][K - 1].sim, L[tid][K - 1].dist, L[tid][K - 1].idx)) break;
      c = insert(L[tid], c, K, x);
    }
  }
  n[tid] = c;
  __syncthreads();
  for (int step = 1; step < 256; step <<= 1) {
    if ((tid % (2 * step)) == 0) {
      Cand tmp[kMaxK];
      const int o = tid + step;
      int i = 0, j = 0, m = 0;
      while (m < K && (i < n[tid] || j < n[o])) {
        bool takeA = j >= n[o] || (i < n[tid] && better(L[tid][i].sim, L[tid][i].dist, L[tid][i].idx, L[o][j].sim,
                                                         L[o][j].dist, L[o][j].idx));
        tmp[m++] = takeA ? L[tid][i++] : L[o][j++];
      }
      for (int t = 0; t < m; ++t) L[tid][t] = tmp[t];
      n[tid] = m;
    }
    __syncthreads();
  }
  for (int j = tid; j < K; j += 256)
    result[(long)q * K + j] = j < n[0] ? L[0][j] : Cand{-FLT_MAX, FLT_MAX, 0xffffffffu, 0};
}

}  // namespace

extern "C" {

int spl_search_lists(int grid) { return grid * kWaves; }

// queries [nq, 768] fp32 (nq <= 16), K <= 32.  `scratch` must hold
// grid * 4 * nq * K candidates (16 B each); result [nq, K] candidates
// {float sim, float dist, uint32 slot, uint32 pad}; empty entries have slot 0xffffffff.
int spl_search(spl_arena_t a, const float* queries, int nq, int K, float min_sim, float max_dist, uint64_t mask,
               int grid, void* scratch, void* result, hipStream_t s) {
  if (nq <= 0 || nq > kMaxQ || K <= 0 || K > kMaxK || a.stride != 3200) return (int)hipErrorInvalidValue;
  if (grid <= 0) grid = 512;
  hipLaunchKernelGGL(k_score_topk, dim3(grid), dim3(256), 0, s, a, queries, nq, K, min_sim, max_dist, mask,
                     (Cand*)scratch);
  hipLaunchKernelGGL(k_merge, dim3(nq), dim3(256), 0, s, (const Cand*)scratch, (long)grid * kWaves, nq, K,
                     (Cand*)result);
  return (int)hipGetLastError();
}

}  // extern "C"
