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
  const Arena a = spl::dev::from_api(aa);
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


// ===========================================================================
// Batched search on the matrix cores (config #5 of BASELINE: hundreds of
// queries against a 10^7..10^8-slot arena).  Brute force is the GEMM
// S[slots, queries] = E[slots, 768] . Q[queries, 768]^T whose A operand lives
// in the arena as fp32 at a 3200-B slot stride; with hundreds of queries per
// pass the fp32 FMA path above is compute-bound, so:
//
//   pass A (bmax): score a sample of the slots in bf16 on MFMA and keep the
//                  per-tile max per query; the k-th largest tile max T is (up
//                  to the bf16 error bound delta) a lower bound of the k-th
//                  best similarity;
//   pass B (cand): score every slot in bf16 on MFMA and emit the slots whose
//                  approximate cosine is >= T - 2*delta;
//   rescore:       re-score the candidates in fp32 with exactly the
//                  arithmetic of k_score_topk and keep the top-K.
// |cos_bf16 - cos| <= 2u + O(D u_f32) with u = 2^-8 (both operands rounded
// once, Cauchy-Schwarz), so no true top-K slot is dropped and the result is
// the fp32 brute force.  Queries whose candidate list overflows are redone
// by the host with k_score_topk.
//
// Geometry (sized for the two bandwidth limits that matter, HBM for the
// arena and L2->CU for the query fragments): 256 threads = 4 waves, one wave
// per SIMD; a tile is 256 slots x 256 queries, wave w owns queries
// [64w, 64w+64) against all 256 slots (16 x 4 tiles of
// v_mfma_f32_16x16x32_bf16 = 256 accumulators, held in AGPRs), so the query
// fragments cost 1.5 KB of L2 reads per slot, half the 3 KB of HBM reads.
// The arena streams through a 4-deep LDS ring of fp32 K-chunks (256 rows x
// 32 dims = 32 KB each) filled by buffer LDS-DMA three chunks ahead (96 KB in
// flight per CU, no staging registers); waves read their A fragments in fp32
// (two ds_read_b128, 16-B units XOR-swizzled by ((row>>1)&3)<<1:
// conflict-free) and convert to bf16 in registers.  One barrier per K-chunk;
// the DMA for chunk n+3 reuses the buffer chunk n-1 left.
// ===========================================================================
namespace mf {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kTile = 256;                // slots per tile
constexpr int kThreads = 256;             // 4 waves, one per SIMD
constexpr int kQ = 256;                   // queries per launch (64 per wave)
constexpr int kNJ = 4;                    // 16-query column tiles per wave
constexpr int kSteps = kD / 32;           // 24 K-chunks of 32 dims per tile
constexpr int kChunk = kTile * 128;       // 32 KB of fp32 per chunk
constexpr int kRing = 4;                  // LDS ring depth (chunks)
constexpr int kAhead = kRing - 1;         // DMA lead (chunks)
constexpr int kDist = 3;                  // query-fragment lead (chunks), = kAhead: see SPL_STEP_SYNC
constexpr int kDma = kChunk / 1024 / 4;   // DMA wave-instructions per wave per chunk (8)
constexpr int kRsrcWord3 = 0x00020000;    // gfx9 raw buffer
static_assert(kThreads == kQ, "one LDS candidate counter per thread");
static_assert(kSteps % kRing == 0 && kSteps % (kDist + 1) == 0 && kDist == kAhead, "static ring slots across tiles");

struct Smem {
  char ring[kRing * kChunk];  // 128 KB
  __attribute__((aligned(16))) float inv[kTile];
  __attribute__((aligned(16))) int live[kTile];
  uint32_t ncand[kQ];  // candidates of this block per query (LDS atomics: no vmcnt drain)
};

__device__ __forceinline__ long tile_start(long t, long slot_end) {
  const long s = t * kTile;
  return s + kTile <= slot_end ? s : slot_end - kTile;  // last tile shifted back: every load in bounds
}

__device__ __forceinline__ rsrc_t tile_rsrc(const spl::dev::Arena& a, long t, long slot_end) {
  return __builtin_amdgcn_make_buffer_rsrc(a.slot((size_t)tile_start(t, slot_end)), 0, kTile * 3200, kRsrcWord3);
}

// swizzle of the 16-B units of a 128-B row (unit bit 0 ^= row bit 2, unit bit 2 ^= row bit 1):
// every gfx950 ds_read_b128 lane group of the fragment reads (16 lanes, rows fr = 0..15 of one or
// two logical units) hits 16 distinct bank slots.  ((row >> 1) & 3) << 1, right for 8-lane phases,
// left the 16-lane groups 2-way conflicted (48.7 % LDS conflict rate, profiles/r4au); the pass time
// did not move with it (20.2 vs 19.9-20.0 ms, profiles/r4av): the LDS is not what bounds it.
__device__ __forceinline__ int swz(int row) { return ((row >> 2) & 1) | (((row >> 1) & 1) << 2); }

__device__ __forceinline__ bf16x8 load_qfrag(rsrc_t r, int voff, int qtile, int step) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, (qtile * kSteps + step) * 1024, 0));
}

// In-order vmcnt accounting.  Every K-step issues, in this order, the query
// fragments for 3 steps ahead (4 loads), the metadata at step 0 of a tile (2),
// and the DMA of the chunk 3 ahead (8).  Fragments go FIRST and as far ahead
// as the DMA, so waiting for a step's fragments never waits for a younger DMA
// (vmcnt is in-order).  At the top of step s the ops younger than chunk s's
// DMA (the last op of step s-3) are the two following steps: 24, or 26 when
// one of them was a step 0; the first tile's prologue (fragments 0..2, then
// DMA 0..2) gives lower bounds 16 at s = 0 and 22 at s = 1.  Wait + barrier
// carry a memory clobber: no LDS read moves above them, no DMA below.
#define SPL_STEP_SYNC(N) asm volatile("s_waitcnt vmcnt(" #N ")\n\ts_barrier" ::: "memory")
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int MODE>  // MODE 0 = per-tile max per query, 1 = emit candidates
__global__ __launch_bounds__(kThreads, 1) void k_search_mma(spl_arena_t aa, const void* __restrict__ qf, int nq,
                                                           long slot_begin, long slot_end, uint64_t mask,
                                                           const float* __restrict__ thr_in, float* __restrict__ bmax,
                                                           uint32_t* __restrict__ cnt, uint32_t* __restrict__ cand,
                                                           int capb) {
  __shared__ __attribute__((aligned(16))) Smem sm;
  const spl::dev::Arena a = spl::dev::from_api(aa);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const long tile_base = slot_begin / kTile;  // slot_begin tile aligned, slot_end - slot_begin >= kTile
  const long tile_end = (slot_end + kTile - 1) / kTile, G = gridDim.x;
  const long t0 = tile_base + blockIdx.x;
  if (t0 >= tile_end) return;  // block-uniform
  if (MODE == 1) sm.ncand[threadIdx.x] = 0;  // kThreads == kQ

  const rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(qf), 0, kQ * kD * 2, kRsrcWord3);
  const int qvoff = lane * 16, qtile0 = wave * kNJ;
  // DMA geometry: wave-instruction k of a chunk fills rows 64w+8k .. +8,
  // lane l -> row +(l>>3), physical unit l&7 <- logical unit (l&7)^swz(row)
  int dvoff[kDma];
#pragma unroll
  for (int k = 0; k < kDma; ++k) {
    const int row = wave * 64 + k * 8 + (lane >> 3);
    dvoff[k] = row * 3200 + (((lane & 7) ^ swz(row)) << 4);
  }
  // fragment read: row 16i+fr, logical units 2fq, 2fq+1 (swz(16i+fr) == swz(fr))
  const int rd0 = fr * 128 + (((2 * fq) ^ swz(fr)) << 4), rd1 = fr * 128 + (((2 * fq + 1) ^ swz(fr)) << 4);
  // ds_read immediates are 16-bit: ring slots 0,1 address off `lo`, slots 2,3
  // off `hi` (= lo + 64 KB, opaque so the compiler keeps 4 base VGPRs instead
  // of materialising 32 out-of-range offsets)
  int lo0 = rd0, lo1 = rd1, hi0 = rd0 + 2 * kChunk, hi1 = rd1 + 2 * kChunk;
  asm volatile("" : "+v"(hi0), "+v"(hi1));

  float thr[kNJ];
#pragma unroll
  for (int j = 0; j < kNJ; ++j) {
    const int q = (qtile0 + j) * 16 + fr;
    thr[j] = (MODE == 1 && q < nq) ? thr_in[q] : FLT_MAX;
  }

  // DMA of chunk c of the tile behind `er` into ring buffer `slot`
  auto issue = [&](rsrc_t er, int c, int slot) {
    char* dst = sm.ring + slot * kChunk + wave * 64 * 128;
#pragma unroll
    for (int k = 0; k < kDma; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(er, (lds_void*)(dst + k * 1024), 16, dvoff[k],
                                               (int)spl::kOffEmbed + c * 128, 0, 0);
  };
  const long last = tile_end - 1;

  // prologue: query fragments of steps 0..2, then the DMA of chunks 0..2 of the first tile
  bf16x8 b[kDist + 1][kNJ];
#pragma unroll
  for (int s = 0; s < kDist; ++s)
#pragma unroll
    for (int j = 0; j < kNJ; ++j) b[s][j] = load_qfrag(qr, qvoff, qtile0 + j, s);
  {
    const rsrc_t er = tile_rsrc(a, t0, slot_end);
    for (int c = 0; c < kAhead; ++c) issue(er, c, c);
  }

  for (long t = t0; t < tile_end; t += G) {
    const long start = tile_start(t, slot_end);
    // the stream runs one tile ahead at the end of a tile (the last tile re-reads itself: in bounds, unused)
    const rsrc_t er_cur = tile_rsrc(a, t, slot_end);
    const rsrc_t er_next = tile_rsrc(a, t + G < tile_end ? t + G : last, slot_end);
    uint64_t h = 0, bl = 0;
    f32x4 acc[16][kNJ];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < kNJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ss[4] = {0.f, 0.f, 0.f, 0.f};  // squared norms of this wave's rows 16*(4w+k)+fr, this lane's dims

#pragma clang loop unroll(full)
    for (int s = 0; s < kSteps; ++s) {
      // chunk s landed (this wave's DMA) and, after the barrier, every wave's
      // DMA landed and every wave is done with chunk s-1's ring buffer
      if (s == 0)
        SPL_STEP_SYNC(16);
      else if (s == 1)
        SPL_STEP_SYNC(22);
      else if (s == 2)
        SPL_STEP_SYNC(26);
      else
        SPL_STEP_SYNC(24);
      // query fragments are periodic in the step: the ring runs across tiles
#pragma unroll
      for (int j = 0; j < kNJ; ++j)
        b[(s + kDist) % (kDist + 1)][j] = load_qfrag(qr, qvoff, qtile0 + j, (s + kDist) % kSteps);
      if (s == 0) {  // metadata of this wave's 64 rows, one per lane
        const uint8_t* sp = a.slot((size_t)(start + wave * 64 + lane));
        h = __builtin_nontemporal_load((const uint64_t*)(sp + spl::kOffHash));
        bl = __builtin_nontemporal_load((const uint64_t*)(sp + spl::kOffBloom));
      }
      issue(s + kAhead < kSteps ? er_cur : er_next, (s + kAhead) % kSteps, (s + kAhead) % kRing);
      const int slot = s % kRing;
      const char* ch0 = sm.ring + (slot < 2 ? lo0 : hi0) + (slot & 1) * kChunk;
      const char* ch1 = sm.ring + (slot < 2 ? lo1 : hi1) + (slot & 1) * kChunk;
#pragma unroll
      for (int i0 = 0; i0 < 16; i0 += 4) {  // 4 row tiles at a time: bounded fragment registers
        f32x4 lo[4], hi[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          lo[u] = *(const f32x4*)(ch0 + (i0 + u) * 2048);
          hi[u] = *(const f32x4*)(ch1 + (i0 + u) * 2048);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = i0 + u;
          if ((i >> 2) == wave) {  // this wave's rows: norms from the same registers (wave-uniform)
            ss[u] += lo[u].x * lo[u].x + lo[u].y * lo[u].y + lo[u].z * lo[u].z + lo[u].w * lo[u].w +
                     hi[u].x * hi[u].x + hi[u].y * hi[u].y + hi[u].z * hi[u].z + hi[u].w * hi[u].w;
          }
          const bf16x8 af = {(__bf16)lo[u].x, (__bf16)lo[u].y, (__bf16)lo[u].z, (__bf16)lo[u].w,
                             (__bf16)hi[u].x, (__bf16)hi[u].y, (__bf16)hi[u].z, (__bf16)hi[u].w};
#pragma unroll
          for (int j = 0; j < kNJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b[s % (kDist + 1)][j], acc[i][j], 0, 0, 0);
        }
      }
    }
    // norms + liveness of this wave's 64 rows: lane r -> row 64w + r = 16(4w + fq) + fr
    {
      float sel = fq == 0 ? ss[0] : fq == 1 ? ss[1] : fq == 2 ? ss[2] : ss[3];
      // the four fq lanes of a row hold disjoint dims: sum them
      float tot[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v = ss[k];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        tot[k] = v;
      }
      sel = fq == 0 ? tot[0] : fq == 1 ? tot[1] : fq == 2 ? tot[2] : tot[3];
      constexpr float kMinNorm2 = MODE == 0 ? 2e-12f : 0.f;  // MODE 0 counts surely-live slots only
      const int row = wave * 64 + lane;
      sm.live[row] = h != 0 && (!mask || (bl & mask) == mask) && sel > kMinNorm2 && start + row >= t * kTile;
      sm.inv[row] = sel > 0.f ? rsqrtf(sel) : 0.f;
    }
    // the live / inv stores must have landed before another wave reads them: a raw s_barrier does
    // not wait for this wave's LDS stores
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    {
      const f32x4* invp = (const f32x4*)(sm.inv + fq * 4);  // rows 16i + 4fq + r, r = 0..3
      const int4* livp = (const int4*)(sm.live + fq * 4);
      float best[kNJ];
#pragma unroll
      for (int j = 0; j < kNJ; ++j) best[j] = -FLT_MAX;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const f32x4 iv = invp[i * 4];
        const int4 lv = livp[i * 4];
        const int lvr[4] = {lv.x, lv.y, lv.z, lv.w};
#pragma unroll
        for (int j = 0; j < kNJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float sim = acc[i][j][r] * iv[r];
            if (MODE == 0) {
              if (lvr[r]) best[j] = fmaxf(best[j], sim);
            } else if (sim >= thr[j] && lvr[r]) {
              // block-private segment [q][block][capb]: the slot index comes
              // from an LDS counter, the global write needs no return value
              const int q = (qtile0 + j) * 16 + fr;
              const uint32_t p = atomicAdd(&sm.ncand[q], 1u);
              if (p < (uint32_t)capb) cand[((long)q * gridDim.x + blockIdx.x) * capb + p] = (uint32_t)(start + i * 16 + fq * 4 + r);
            }
          }
      }
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < kNJ; ++j) {
          const int q = (qtile0 + j) * 16 + fr;
          float bj = fmaxf(best[j], __shfl_xor(best[j], 16, 64));
          bj = fmaxf(bj, __shfl_xor(bj, 32, 64));
          if (fq == 0 && q < nq) bmax[(t - tile_base) * nq + q] = bj;
        }
      }
    }
  }
  if (MODE == 1) {
    raw_barrier();
    const int q = threadIdx.x;
    if (q < nq) cnt[(long)q * gridDim.x + blockIdx.x] = sm.ncand[q];
  }
  wait_vm0();  // drain the trailing DMAs (next-tile prefetch of the last tile) before the LDS goes away
}

}  // namespace mf

// ---------------------------------------------------------------------------
// The same pass on the side region's bf16 copy (SPL_ARENA_VEC16 arenas, splinter_layout.hpp): every
// slot's vector as 1536 contiguous bytes (half the fp32 row, no 3200-B stride) and its squared norm
// precomputed by the writer.  The operands are the values the fp32 pass converts in registers
// (v_cvt_pk_bf16_f32 = round to nearest even, as the writers store them) and the norm is the fp32
// one, so the candidate bound and the result are the fp32 pass's.  K-chunks of 32 dims = 64 B per row:
// a 16 KB chunk per 256-row tile, 4 LDS-DMA wave-instructions per wave, the A fragments read straight
// as bf16 (one ds_read_b128 each).  Rows are 64 B, so a ds_read_b128 lane group (16 lanes) would hit
// the same 4 banks for rows r and r + 4: the 16-B unit u of row r is stored at u ^ f((r >> 2) & 3)
// with f = {0, 2, 3, 1}, which gives every gfx950 b128 lane group 16 distinct 4-bank groups (checked
// by hand over the four groups); the XOR goes on the global source address (glds writes lane-linearly).
namespace mf16 {
using mf::bf16x8;
using mf::f32x4;
using mf::rsrc_t;
using mf::lds_void;
constexpr int kTile = mf::kTile, kQ = mf::kQ, kNJ = mf::kNJ, kSteps = mf::kSteps;
constexpr int kWaves = 8, kThreads = kWaves * 64;  // two waves per SIMD
constexpr int kChunk = kTile * 64;        // 16 KB of bf16 slot rows per K-chunk
constexpr int kQChunk = kQ * 64;          // 16 KB of bf16 query fragments per K-chunk
constexpr int kRing = mf::kRing, kAhead = mf::kAhead;
constexpr int kRows = kTile / kWaves;     // slot rows a wave stages (DMA, metadata): 32
constexpr int kBlk = 8;                   // 16-row blocks per wave: one slot half
constexpr int kRsrcWord3 = mf::kRsrcWord3;
struct Smem {
  char ring[kRing][kChunk];   // 64 KB
  char qring[kRing][kQChunk]; // 64 KB
  __attribute__((aligned(16))) float inv[kTile];
  __attribute__((aligned(16))) int live[kTile];
  uint32_t ncand[kQ];
  float pmax[kQ];             // MODE 0: the upper slot half's per-query maxima
};
// 16-B unit swizzle of the 64-B row pieces: physical unit = logical unit ^ rsw(row & 15).  gfx950
// services a ds_read_b128 in the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, and the same
// +32 (MI355X_MICROARCH.md, LDS); with the fragment read (lane -> row lane & 15, unit lane >> 4)
// this one flip of unit bit 1 for rows 8-15 puts every group on 16 distinct 16-B bank slots (found
// by exhaustive search).  The former {0,2,3,1}[(row >> 2) & 3], right for contiguous 16-lane
// groups, cost 8 extra LDS cycles per read: a 56 % conflict rate (profiles/r5/search8/pmc_search.md).
__device__ __forceinline__ int rsw(int r) { return ((r >> 3) & 1) << 1; }

__device__ __forceinline__ rsrc_t tile_rsrc16(const spl::dev::Arena& a, long t, long slot_end) {
  return __builtin_amdgcn_make_buffer_rsrc(a.vec16((size_t)mf::tile_start(t, slot_end)), 0, kTile * 1536, kRsrcWord3);
}

// Two waves per SIMD: wave w owns the 64 queries of group w & 3 against slot half w >> 2 (8 x 4
// accumulator tiles, 128 registers), so one wave's matrix work runs while its partner waits on the
// DMA / barrier (with one wave per SIMD the two were serialised: without its MFMAs that pass took
// 8.4 of its 13.5 ms, profiles/r5/search_probes).  The query fragments of a K-chunk (16 KB) arrive
// by LDS-DMA beside the slot rows, so no wave stages them in registers three chunks ahead.
// In-order vmcnt: a wave issues per step (the metadata, 3 loads, at step 0, then) the DMA of chunk
// s + 3, 2 query + 2 row pieces; younger than chunk s's DMA at the top of step s: 8, or 11 when one
// of the two steps after its issue was a step 0 (s = 1, 2).
template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void k_search_mma16(spl_arena_t aa, const void* __restrict__ qf, int nq,
                                                             long slot_begin, long slot_end, uint64_t mask,
                                                             const float* __restrict__ thr_in, float* __restrict__ bmax,
                                                             uint32_t* __restrict__ cnt, uint32_t* __restrict__ cand,
                                                             int capb) {
  __shared__ __attribute__((aligned(16))) Smem sm;
  const spl::dev::Arena a = spl::dev::from_api(aa);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int qg = wave & 3, sh = wave >> 2;
  const long tile_base = slot_begin / kTile;
  const long tile_end = (slot_end + kTile - 1) / kTile, G = gridDim.x;
  const long t0 = tile_base + blockIdx.x;
  if (t0 >= tile_end) return;  // block-uniform
  if (MODE == 1 && tid < kQ) sm.ncand[tid] = 0;

  const rsrc_t qr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(qf), 0, kQ * kD * 2, kRsrcWord3);
  const int qtile0 = qg * kNJ;
  // row DMA: wave-instruction k of a chunk fills rows 32w + 16k .. +16 (1 KB), lane l -> row +(l >> 2),
  // physical unit l & 3 <- logical unit (l & 3) ^ rsw(row & 15); query DMA: instruction k brings the
  // 1-KB fragment block of 16-query tile 2w + k for the chunk's step (lane-linear, as read)
  int dvoff[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = wave * kRows + k * 16 + (lane >> 2);
    dvoff[k] = row * 1536 + (((lane & 3) ^ rsw(row & 15)) << 4);
  }
  const float* nrm2 = a.nrm2();
  // fragment read: row 16i + fr of this wave's slot half, logical unit fq
  const int rdo = fr * 64 + ((fq ^ rsw(fr)) << 4) + sh * kBlk * 1024;

  float thr[kNJ];
#pragma unroll
  for (int j = 0; j < kNJ; ++j) {
    const int q = (qtile0 + j) * 16 + fr;
    thr[j] = (MODE == 1 && q < nq) ? thr_in[q] : FLT_MAX;
  }
  auto issue = [&](rsrc_t er, int c, int slot) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (lds_void*)(sm.qring[slot] + (2 * wave + k) * 1024), 16, lane * 16,
                                               ((2 * wave + k) * kSteps + c) * 1024, 0, 0);
    char* dst = sm.ring[slot] + wave * kRows * 64;
#pragma unroll
    for (int k = 0; k < 2; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(er, (lds_void*)(dst + k * 1024), 16, dvoff[k], c * 64, 0, 0);
  };
  const long last = tile_end - 1;
  {
    const rsrc_t er = tile_rsrc16(a, t0, slot_end);
    for (int c = 0; c < kAhead; ++c) issue(er, c, c);
  }

  for (long t = t0; t < tile_end; t += G) {
    const long start = mf::tile_start(t, slot_end);
    const rsrc_t er_cur = tile_rsrc16(a, t, slot_end);
    const rsrc_t er_next = tile_rsrc16(a, t + G < tile_end ? t + G : last, slot_end);
    uint64_t h = 0, bl = 0;
    float n2 = 0.f;
    f32x4 acc[kBlk][kNJ];
#pragma unroll
    for (int i = 0; i < kBlk; ++i)
#pragma unroll
      for (int j = 0; j < kNJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma clang loop unroll(full)
    for (int s = 0; s < kSteps; ++s) {
      if (s == 1 || s == 2)
        SPL_STEP_SYNC(11);
      else
        SPL_STEP_SYNC(8);
      if (s == 0) {  // metadata of this wave's 32 rows (lanes 32-63 repeat 0-31)
        const long row = start + wave * kRows + (lane & (kRows - 1));
        const uint8_t* sp = a.slot((size_t)row);
        h = __builtin_nontemporal_load((const uint64_t*)(sp + spl::kOffHash));
        bl = __builtin_nontemporal_load((const uint64_t*)(sp + spl::kOffBloom));
        n2 = __builtin_nontemporal_load(nrm2 + row);
      }
      const char* qs = sm.qring[s % kRing] + lane * 16;
      bf16x8 bq[kNJ];
#pragma unroll
      for (int j = 0; j < kNJ; ++j) bq[j] = *(const bf16x8*)(qs + (qtile0 + j) * 1024);
      const char* ch = sm.ring[s % kRing] + rdo;
#pragma unroll
      for (int i0 = 0; i0 < kBlk; i0 += 4) {
        bf16x8 af[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) af[u] = *(const bf16x8*)(ch + (i0 + u) * 1024);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < kNJ; ++j)
            acc[i0 + u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u], bq[j], acc[i0 + u][j], 0, 0, 0);
        // the next chunk's DMA after the first MFMA group: its issue overlaps matrix work (11.92 vs
        // 12.15 ms per pass issued before the group; s_setprio around the groups: neutral)
        if (i0 == 0) issue(s + kAhead < kSteps ? er_cur : er_next, (s + kAhead) % kSteps, (s + kAhead) % kRing);
      }
    }
    {
      constexpr float kMinNorm2 = MODE == 0 ? 2e-12f : 0.f;  // MODE 0 counts surely-live slots only
      const int row = wave * kRows + lane;
      if (lane < kRows) {
        sm.live[row] = h != 0 && (!mask || (bl & mask) == mask) && n2 > kMinNorm2 && start + row >= t * kTile;
        sm.inv[row] = n2 > 0.f ? rsqrtf(n2) : 0.f;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    {
      const f32x4* invp = (const f32x4*)(sm.inv + fq * 4 + sh * kBlk * 16);
      const int4* livp = (const int4*)(sm.live + fq * 4 + sh * kBlk * 16);
      float best[kNJ];
#pragma unroll
      for (int j = 0; j < kNJ; ++j) best[j] = -FLT_MAX;
#pragma unroll
      for (int i = 0; i < kBlk; ++i) {
        const f32x4 iv = invp[i * 4];
        const int4 lv = livp[i * 4];
        const int lvr[4] = {lv.x, lv.y, lv.z, lv.w};
#pragma unroll
        for (int j = 0; j < kNJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float sim = acc[i][j][r] * iv[r];
            if (MODE == 0) {
              if (lvr[r]) best[j] = fmaxf(best[j], sim);
            } else if (sim >= thr[j] && lvr[r]) {
              const int q = (qtile0 + j) * 16 + fr;
              const uint32_t p = atomicAdd(&sm.ncand[q], 1u);
              if (p < (uint32_t)capb)
                cand[((long)q * gridDim.x + blockIdx.x) * capb + p] = (uint32_t)(start + (sh * kBlk + i) * 16 + fq * 4 + r);
            }
          }
      }
      if (MODE == 0) {  // per query: max over the lane quads, then the two slot halves meet in LDS
        float bj[kNJ];
#pragma unroll
        for (int j = 0; j < kNJ; ++j) {
          bj[j] = fmaxf(best[j], __shfl_xor(best[j], 16, 64));
          bj[j] = fmaxf(bj[j], __shfl_xor(bj[j], 32, 64));
        }
        if (sh == 1 && fq == 0)
#pragma unroll
          for (int j = 0; j < kNJ; ++j) sm.pmax[(qtile0 + j) * 16 + fr] = bj[j];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (sh == 0 && fq == 0)
#pragma unroll
          for (int j = 0; j < kNJ; ++j) {
            const int q = (qtile0 + j) * 16 + fr;
            if (q < nq) bmax[(t - tile_base) * nq + q] = fmaxf(bj[j], sm.pmax[q]);
          }
      }
    }
  }
  if (MODE == 1) {
    mf::raw_barrier();
    const int q = threadIdx.x;
    if (q < nq && q < kQ) cnt[(long)q * gridDim.x + blockIdx.x] = sm.ncand[q];
  }
  mf::wait_vm0();
}
}  // namespace mf16

namespace mf {
// fp32 re-score of the candidates of one query (block) and top-K selection;
// same arithmetic as k_score_topk so the ranking is identical.  Candidates
// come in block-private segments cand[q][b][0 .. min(cnt[q][b], capb)).
// 16 waves per query block (4 per SIMD): the re-score is a gather of 3-KB rows bound by loads in flight
constexpr int kRsWaves = 16;
__global__ __launch_bounds__(kRsWaves * 64) void k_rescore(spl_arena_t aa, const float* __restrict__ queries, int K,
                                                 float min_sim, float max_dist, uint64_t mask,
                                                 const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ cand,
                                                 int nblk, int capb, Cand* __restrict__ result) {
  __shared__ __attribute__((aligned(16))) float Qs[kD];
  __shared__ float qn_s;
  __shared__ Cand top[kRsWaves][kMaxK];
  __shared__ int tc[kRsWaves];
  const spl::dev::Arena a = spl::dev::from_api(aa);
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < kD; i += kRsWaves * 64) Qs[i] = queries[(long)q * kD + i];
  if (tid < kRsWaves) tc[tid] = 0;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int d = 0; d < kD; ++d) s += Qs[d] * Qs[d];
    qn_s = s;
  }
  __syncthreads();
  const float qn = qn_s;
  int c = 0;
  // kRU candidates of a wave in flight at once (their slot headers and 3-KB rows loaded together):
  // one candidate at a time left each wave on a chain of dependent loads per row
  constexpr int kRU = 4;
  const float4* q4 = (const float4*)Qs;
  for (int b = wave; b < nblk; b += kRsWaves) {
    const int n = min(cnt[(long)q * nblk + b], (uint32_t)capb);
    const uint32_t* seg = cand + ((long)q * nblk + b) * capb;
    for (int t = 0; t < n; t += kRU) {
      uint32_t idx[kRU];
      uint64_t h[kRU], bl[kRU];
      float4 e[kRU][3];
#pragma unroll
      for (int u = 0; u < kRU; ++u) idx[u] = seg[t + u < n ? t + u : t];
#pragma unroll
      for (int u = 0; u < kRU; ++u) {
        const uint8_t* s = a.slot(idx[u]);
        h[u] = *(const uint64_t*)(s + spl::kOffHash);
        bl[u] = mask ? *(const uint64_t*)(s + spl::kOffBloom) : 0;
        const float4* v4 = (const float4*)(s + spl::kOffEmbed);
#pragma unroll
        for (int k = 0; k < 3; ++k) e[u][k] = v4[lane + 64 * k];
      }
#pragma unroll
      for (int u = 0; u < kRU; ++u) {
        if (t + u >= n || h[u] == 0 || (mask && (bl[u] & mask) != mask)) continue;  // wave-uniform
        float en = 0.f, dot = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float4 qq = q4[lane + 64 * k];
          en += e[u][k].x * e[u][k].x + e[u][k].y * e[u][k].y + e[u][k].z * e[u][k].z + e[u][k].w * e[u][k].w;
          dot += e[u][k].x * qq.x + e[u][k].y * qq.y + e[u][k].z * qq.z + e[u][k].w * qq.w;
        }
        en = wave_sum(en);
        if (en < 1e-12f) continue;
        dot = wave_sum(dot);
        const float enr = sqrtf(en);
        const float sim = dot / (enr * sqrtf(qn) + 1e-30f);
        const float dist = sqrtf(fmaxf(en + qn - 2.f * dot, 0.f));
        if (sim < min_sim || dist > max_dist) continue;
        if (lane == 0) c = insert(top[wave], c, K, Cand{sim, dist, idx[u], 0});
      }
    }
  }
  if (lane == 0) tc[wave] = c;
  __syncthreads();
  if (tid == 0) {
    Cand L[kMaxK];
    int m = 0;
    for (int w = 0; w < kRsWaves; ++w)
      for (int j = 0; j < tc[w]; ++j) m = insert(L, m, K, top[w][j]);
    for (int j = 0; j < K; ++j) result[(long)q * K + j] = j < m ? L[j] : Cand{-FLT_MAX, FLT_MAX, 0xffffffffu, 0};
  }
}
}  // namespace mf

// Candidate threshold per query for the batched search (ops/search.py search_batch, spl_search_batch):
// thr[q] = max(k-th largest of bmax[0..T)[q] - 2 delta, floor); fewer than k tiles: floor.  One block
// per query: every thread keeps the k largest of its strided share, then k rounds of a block max
// (the winner drops its head).
// topv (optional): the k largest themselves, [nq][k] descending (-FLT_MAX past the tiles), for a
// node search that merges the shards' samples (HbmStore::search_batch, SearchSync).
__global__ __launch_bounds__(256) void k_search_thr(const float* __restrict__ bmax, int T, int nq, int k, float delta2,
                                                    float floor_v, float* __restrict__ thr, float* __restrict__ topv) {
  __shared__ float wv[4];
  __shared__ int wi[4];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float top[kMaxK];
  int n = 0;
  for (int t = tid; t < T; t += 256) {
    const float v = bmax[(long)t * nq + q];
    if (n == k && v <= top[k - 1]) continue;
    int p = n < k ? n : k - 1;
    while (p > 0 && top[p - 1] < v) { top[p] = top[p - 1]; --p; }
    top[p] = v;
    n = n < k ? n + 1 : n;
  }
  int head = 0;
  float kth = -FLT_MAX;
  for (int r = 0; r < k; ++r) {
    float v = head < n ? top[head] : -FLT_MAX;
    int who = tid;
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int oi = __shfl_xor(who, o, 64);
      if (ov > v || (ov == v && oi < who)) { v = ov; who = oi; }
    }
    if (lane == 0) { wv[wave] = v; wi[wave] = who; }
    __syncthreads();
    float bv = wv[0];
    int bi = wi[0];
    for (int w = 1; w < 4; ++w)
      if (wv[w] > bv || (wv[w] == bv && wi[w] < bi)) { bv = wv[w]; bi = wi[w]; }
    __syncthreads();
    if (bi == tid) ++head;
    kth = bv;
    if (topv && tid == 0) topv[(long)q * k + r] = bv;
  }
  if (tid == 0) thr[q] = (T < k || kth == -FLT_MAX) ? floor_v : fmaxf(kth - delta2, floor_v);
}

// CLI `search` over an HBM store (reference splinter_cli_cmd_search.c:339-416): every candidate
// slot -- live (hash != 0) and either carrying every bloom bit of `mask`, or, without a mask,
// holding a value (the reference's splinter_list) -- gets {sim, dist}: cosine and euclidean
// distance against the query for an embedded slot, {0, -1} for a candidate without a vector
// (listed with null scores when no score filter is set), {NaN, NaN} for a non-candidate or one a
// filter rejects (min_sim / max_dist > 0, as the reference treats 0 = off).  One wave per slot:
// the 3072-B vector arrives as 64 lanes x 3 x 16 B.
__global__ __launch_bounds__(256) void k_score_all(spl_arena_t aa, const float* __restrict__ query, float min_sim,
                                                   float max_dist, uint64_t mask, float2* __restrict__ out) {
  using namespace spl;
  using namespace spl::dev;
  const Arena a = from_api(aa);
  const int lane = threadIdx.x & 63;
  const float4* q4 = (const float4*)query;
  float4 q[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) q[c] = q4[lane + 64 * c];
  float qn = 0.f;
#pragma unroll
  for (int c = 0; c < 3; ++c) qn += q[c].x * q[c].x + q[c].y * q[c].y + q[c].z * q[c].z + q[c].w * q[c].w;
  qn = wave_sum(qn);
  const long nwv = ((long)gridDim.x * blockDim.x) >> 6;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < (long)a.slots; i += nwv) {
    const uint8_t* s = a.slot((size_t)i);
    const uint64_t h = ald64(s + kOffHash);
    bool cand = h != 0;
    if (cand) cand = mask ? (ald64(s + kOffBloom) & mask) == mask : ald32(s + kOffValLen) > 0;
    float2 r = make_float2(__builtin_nanf(""), __builtin_nanf(""));
    if (cand) {  // wave-uniform
      const float4* v4 = (const float4*)(s + kOffEmbed);
      float en = 0.f, dot = 0.f;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float4 e = v4[lane + 64 * c];
        en += e.x * e.x + e.y * e.y + e.z * e.z + e.w * e.w;
        dot += e.x * q[c].x + e.y * q[c].y + e.z * q[c].z + e.w * q[c].w;
      }
      en = wave_sum(en);
      dot = wave_sum(dot);
      if (en > 1e-12f && qn > 1e-12f) {
        const float sim = dot / (sqrtf(en) * sqrtf(qn));
        const float dist = sqrtf(fmaxf(en + qn - 2.f * dot, 0.f));
        if (!((min_sim > 0.f && sim < min_sim) || (max_dist > 0.f && dist > max_dist))) r = make_float2(sim, dist);
      } else if (!(min_sim > 0.f || max_dist > 0.f)) {
        r = make_float2(0.f, -1.f);
      }
    }
    if (lane == 0) out[i] = r;
  }
}

}  // namespace

// ---------------------------------------------------------- query prep --
// The batched search's query operand on the device (was a host loop per 256-query block): one
// workgroup per query slot of the 256-query block -- L2 norm (fp32 sum of squares over the wave
// reduction), normalised, rounded to bf16, stored in the candidate pass's fragment order
// [16 q-tiles][24 steps][4 kq][16 r][8]: dims [32 step + 8 kq, +8) of query 16 tile + r.  Query
// slots >= n are zero.
__global__ __launch_bounds__(256) void k_search_qprep(const float* __restrict__ q, int n, uint16_t* __restrict__ qf) {
  const int qi = blockIdx.x, t = threadIdx.x;
  __shared__ float red[4];
  float v[3] = {0.f, 0.f, 0.f};
  if (qi < n) {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = q[(long)qi * 768 + t + 256 * c];
  }
  float ss = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((t & 63) == 0) red[t >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float inv = tot > 1e-30f ? rsqrtf(tot) : 0.f;
  const int tile = qi >> 4, r = qi & 15;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int d = t + 256 * c;
    const int st = d >> 5, kq = (d >> 3) & 3, e = d & 7;
    qf[((((long)tile * 24 + st) * 4 + kq) * 16 + r) * 8 + e] = __builtin_bit_cast(uint16_t, (__bf16)(v[c] * inv));
  }
}

// slot cores (128 B) of a result list, gathered on the device so the hits leave with their keys
// in the same copy: res[n] Cand -> out[n][128] (zeros for an empty entry).  8 lanes per entry.
__global__ __launch_bounds__(256) void k_search_cores(spl_arena_t aa, const Cand* __restrict__ res, int n,
                                                      uint4* __restrict__ out) {
  const int i = blockIdx.x * 32 + (threadIdx.x >> 3), c = threadIdx.x & 7;
  if (i >= n) return;
  const uint32_t idx = res[i].idx;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (idx < aa.slots) {
    const uint8_t* s = (const uint8_t*)aa.base + spl::kHeaderBytes + (size_t)idx * aa.stride + 16 * c;
    const uint64_t a = __hip_atomic_load((const uint64_t*)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t b = __hip_atomic_load((const uint64_t*)(s + 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
  }
  out[(size_t)i * 8 + c] = v;
}

// over[q] = 1 when query q's candidate segment overflowed in any block (cnt[q][g] > capb)
__global__ __launch_bounds__(256) void k_search_over(const uint32_t* __restrict__ cnt, int nblk, int capb,
                                                     uint32_t* __restrict__ over) {
  const int qi = blockIdx.x;
  bool o = false;
  for (int g = threadIdx.x; g < nblk; g += 256) o |= cnt[(long)qi * nblk + g] > (uint32_t)capb;
  o = __syncthreads_or(o);
  if (threadIdx.x == 0) over[qi] = o ? 1u : 0u;
}

extern "C" {

int spl_arena_score_all(spl_arena_t a, const float* query, float min_sim, float max_dist, uint64_t mask, void* out,
                        hipStream_t s) {
  if (a.stride != 3200) return (int)hipErrorInvalidValue;
  long g = ((long)a.slots + 3) / 4;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(k_score_all, dim3((unsigned)g), dim3(256), 0, s, a, query, min_sim, max_dist, mask, (float2*)out);
  return (int)hipGetLastError();
}


int spl_search_lists(int grid) { return grid * kWaves; }

int spl_search_qprep(const float* queries, int nq, void* qfrag, hipStream_t s) {
  if (nq <= 0 || nq > mf::kQ || !queries || !qfrag) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_search_qprep, dim3(mf::kQ), dim3(256), 0, s, queries, nq, (uint16_t*)qfrag);
  return (int)hipGetLastError();
}

int spl_search_cores(spl_arena_t a, const void* result, int n, void* out_cores, hipStream_t s) {
  if (n <= 0 || !result || !out_cores) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_search_cores, dim3((unsigned)((n + 31) / 32)), dim3(256), 0, s, a, (const Cand*)result, n,
                     (uint4*)out_cores);
  return (int)hipGetLastError();
}

int spl_search_overflow(const uint32_t* cnt, int nq, int nblk, int capb, uint32_t* over, hipStream_t s) {
  if (nq <= 0 || nblk <= 0 || !cnt || !over) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_search_over, dim3(nq), dim3(256), 0, s, cnt, nblk, capb, over);
  return (int)hipGetLastError();
}

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

int spl_search_mma_queries() { return mf::kQ; }
int spl_search_mma_tile() { return mf::kTile; }

int spl_search_mma_pass(spl_arena_t a, const void* qfrag, int nq, long slot_begin, long slot_end, uint64_t mask,
                        int mode, const float* thr, float* bmax, uint32_t* cnt, uint32_t* cand, int capb, int grid,
                        hipStream_t s) {
  if (a.stride != 3200 || nq <= 0 || nq > mf::kQ || slot_begin < 0 || slot_begin % mf::kTile ||
      slot_end > (long)a.slots || slot_end - slot_begin < mf::kTile || (mode != 0 && mode != 1) || grid <= 0 ||
      (mode == 1 && (!thr || !cnt || !cand || capb <= 0)) || (mode == 0 && !bmax))
    return (int)hipErrorInvalidValue;
  const long tiles = (slot_end - slot_begin + mf::kTile - 1) / mf::kTile;
  // the bf16 copy when the arena carries one (SPLINTER_SEARCH_VEC16=0: the fp32 rows)
  static const bool v16_ok = [] {
    const char* e = getenv("SPLINTER_SEARCH_VEC16");
    return !(e && e[0] == '0');
  }();
  if ((a.flags & SPL_ARENA_VEC16) && v16_ok) {
    const int g = mode == 0 ? (int)(grid < tiles ? grid : tiles) : grid;
    if (mode == 0)
      hipLaunchKernelGGL(mf16::k_search_mma16<0>, dim3(g), dim3(mf16::kThreads), 0, s, a, qfrag, nq, slot_begin,
                         slot_end, mask, thr, bmax, cnt, cand, capb);
    else
      hipLaunchKernelGGL(mf16::k_search_mma16<1>, dim3(g), dim3(mf16::kThreads), 0, s, a, qfrag, nq, slot_begin,
                         slot_end, mask, thr, bmax, cnt, cand, capb);
    return (int)hipGetLastError();
  }
  if (mode == 0) {
    const int g = (int)(grid < tiles ? grid : tiles);
    hipLaunchKernelGGL(mf::k_search_mma<0>, dim3(g), dim3(mf::kThreads), 0, s, a, qfrag, nq, slot_begin, slot_end,
                       mask, thr, bmax, cnt, cand, capb);
  } else {
    // every one of the `grid` segments per query must be written: no clamping to the tile count
    // (blocks without a tile store a zero count)
    hipLaunchKernelGGL(mf::k_search_mma<1>, dim3(grid), dim3(mf::kThreads), 0, s, a, qfrag, nq, slot_begin, slot_end,
                       mask, thr, bmax, cnt, cand, capb);
  }
  return (int)hipGetLastError();
}

int spl_search_thr(const float* bmax, int tiles, int nq, int K, float delta2, float floor_v, float* thr,
                   hipStream_t s) {
  return spl_search_thr_topk(bmax, tiles, nq, K, delta2, floor_v, thr, nullptr, s);
}

int spl_search_thr_topk(const float* bmax, int tiles, int nq, int K, float delta2, float floor_v, float* thr,
                        float* topv, hipStream_t s) {
  if (nq <= 0 || K <= 0 || K > kMaxK || tiles < 0 || !thr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_search_thr, dim3(nq), dim3(256), 0, s, bmax, tiles, nq, K, delta2, floor_v, thr, topv);
  return (int)hipGetLastError();
}

int spl_search_rescore(spl_arena_t a, const float* queries, int nq, int K, float min_sim, float max_dist,
                       uint64_t mask, const uint32_t* cnt, const uint32_t* cand, int nblk, int capb, void* result,
                       hipStream_t s) {
  if (a.stride != 3200 || nq <= 0 || K <= 0 || K > kMaxK || nblk <= 0 || capb <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mf::k_rescore, dim3(nq), dim3(mf::kRsWaves * 64), 0, s, a, queries, K, min_sim, max_dist, mask, cnt, cand,
                     nblk, capb, (Cand*)result);
  return (int)hipGetLastError();
}

}  // extern "C"
