// gemm_bf16.hip — MFMA bf16 GEMM with fused epilogues for the Nomic-BERT
// encoder (kernels K12/K13/K15/K16 of SURVEY §2.10).
//
//   C[M, N] = A[M, K] . W[N, K]^T      (A activations, W = GGUF weight rows)
//
// Geometry (gfx950): 256 threads = 4 waves in a 2x2 arrangement, block tile
// 128x128, BK = 64; each wave owns a 64x64 sub-tile = 4x4 tiles of
// v_mfma_f32_16x16x32_bf16 with fp32 accumulators.  Both operands are
// K-contiguous, so every MFMA fragment is one 16-B ds_read_b128.
// Staging: global_load_lds_dwordx4 (LDS-DMA) into a double-buffered LDS
// image; the image is lane-linear, so the XOR swizzle (chunk ^= row & 7,
// conflict-free for the ds_read_b128 lane groups) is applied to the GLOBAL
// source address and to the LDS read address (guide rule 21).
// Block -> tile mapping is XCD-aware (bijective remap, guide §5 T1): the tiles
// that share A rows run on one XCD and reuse its L2.
// Epilogue: accumulators go through LDS in fp32, then each thread owns
// 16-B output chunks, so every fused epilogue (residual add, SwiGLU, RoPE)
// works on whole rows with vector loads/stores.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>

#include "glds_asm.hpp"
#include "nomic_api.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kThreads = 256;
constexpr int kTileBytes = BM * BK * 2;            // 16 KB per operand tile
constexpr int kEpiStride = BN + 4;                 // fp32 epilogue row stride (floats)
constexpr int kLdsBytes = (BM * kEpiStride * 4 > 4 * kTileBytes) ? BM * kEpiStride * 4 : 4 * kTileBytes;

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
// fp32 -> bf16, round-to-nearest-even, on the hardware converter (v_cvt_pk_bf16_f32: one
// instruction per PAIR via pk2, instead of a 5-op integer rounding sequence per value)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// Stage one BMxBK tile of a K-contiguous matrix (row stride ld elements)
// starting at (row0, k0) into the lane-linear LDS image at `dst`.
template <bool AS = false>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ src, long ld, long row0, int k0,
                                           char* dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = wave * 4 + i;          // 8-row block of this wave instruction
    const int r = blk * 8 + (lane >> 3);   // row in tile
    const int pc = lane & 7;               // physical 16-B chunk in the 128-B row
    const int c = pc ^ (r & 7);            // logical chunk stored there
    const uint16_t* g = src + (row0 + r) * ld + k0 + c * 8;
    if constexpr (AS)
      spl::glds16_asm(g, dst + blk * 1024);  // counted LDS waits (glds_asm.hpp)
    else
      __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)(dst + blk * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 lds_frag(const char* tile, int r, int c) {
  return *(const bf16x8*)(tile + r * 128 + ((c ^ (r & 7)) << 4));
}

__device__ __forceinline__ void remap_tile(int bid, int nb, int nt, int gn, int& mt, int& ntile) {
  // bijective XCD remap: blocks b and b+8 share an XCD; give each XCD a
  // contiguous range of the linear tile order.  The linear order is
  // band-major: bands of `gn` n-tiles, m-major inside a band, so the ~32
  // tiles an XCD runs at once cover (32/gn) A row-blocks x gn W column-blocks
  // and both fit its 4 MB L2 (gn = nt: plain row-major).
  const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_band = (nb / nt) * gn;
  const int band = wg / per_band, rem = wg - band * per_band;
  mt = rem / gn;
  ntile = band * gn + (rem - mt * gn);
}

struct EpiArgs {
  uint16_t* out;
  long ldo;
  const uint16_t* res;   // residual [M, N] (mode 1)
  long ldr;
  const float* rope;     // [max_pos, 32] x {cos, sin} interleaved (mode 3)
  const int32_t* pos;    // [M] position of each row (mode 3)
  int rope_cols;         // columns (from 0) that get RoPE (q|k = 1536)
  long M;
  int gn;                // n-tiles per band of the tile order (remap_tile)
  // LayerNorm fold (nomic_api.h NOMIC_EPI_*_FOLD / RES_*STATS)
  const float2* pin;     // [M][np] (mean, M2) 128-column partials of the rows of A (fold) or of
  int np;                //   res (RES_LN_STATS), as a stats-mode producer wrote them
  float eps;
  const float* c1;       // [N] W' 1       (fold)
  const float* c2;       // [N] W b        (fold)
  const uint16_t* lng;   // [N] LN gamma / beta of res (RES_LN_STATS)
  const uint16_t* lnb;
  float2* part;          // [M][N/128] (mean, M2) of out's rows per 128 columns (RES_*STATS)
};

constexpr bool is_fold(int m) { return m == NOMIC_EPI_ROPE_FOLD || m == NOMIC_EPI_SWIGLU_FOLD; }
constexpr bool is_stats(int m) { return m == NOMIC_EPI_RES_STATS || m == NOMIC_EPI_RES_LN_STATS; }
constexpr bool is_rope(int m) { return m == NOMIC_EPI_ROPE || m == NOMIC_EPI_ROPE_FOLD; }
constexpr bool is_swiglu(int m) { return m == NOMIC_EPI_SWIGLU || m == NOMIC_EPI_SWIGLU_FOLD; }
constexpr bool is_rowstore(int m) { return m == NOMIC_EPI_STORE || m == NOMIC_EPI_RESIDUAL || is_stats(m); }
constexpr bool needs_rowstats(int m) { return is_fold(m) || m == NOMIC_EPI_RES_LN_STATS; }

// LN fold of one GEMM output: rstd (acc - mean c1[n]) + c2[n]  (== LN(a) . w for the unfolded w)
__device__ __forceinline__ float fold(float acc, float2 st, float c1, float c2) {
  return st.y * (acc - st.x * c1) + c2;
}

// sum over the 16 lanes of a row group (lanes 16k .. 16k+15) on the DPP crossbar (no LDS
// traffic, unlike ds_bpermute): quad_perm [1,0,3,2] and [2,3,0,1] give every lane its quad's sum,
// row_half_mirror (lane i <-> 7-i) the 8-lane sum, row_mirror (i <-> 15-i) the 16-lane sum
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float sum16(float v) {
  v = dpp_add<0xB1>(v);
  v = dpp_add<0x4E>(v);
  v = dpp_add<0x141>(v);
  return dpp_add<0x140>(v);
}

__device__ __forceinline__ void load8f(const float* p, float (&o)[8]) {  // p: 32-B aligned
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// up * silu(g) with a hardware reciprocal and exp2 (v_rcp_f32 + v_exp_f32: no IEEE division
// sequence in the epilogue; ~1 ulp, far below the bf16 output rounding)
__device__ __forceinline__ float swiglu(float up, float g) {
  return up * g * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-g * 1.4426950408889634f));
}

template <int MODE, bool AS = false>
__global__ __launch_bounds__(kThreads, 2) void k_gemm_nt(const uint16_t* __restrict__ A, long lda,
                                                         const uint16_t* __restrict__ W, long ldw, int K,
                                                         int mtiles, int ntiles, EpiArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int mt, nt;
  remap_tile(blockIdx.x, mtiles * ntiles, ntiles, ep.gn, mt, nt);
  const long m0 = (long)mt * BM, n0 = (long)nt * BN;
  const int wm = wave >> 1, wn = wave & 1;


  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  // LN modes: the epilogue's per-column vectors are fixed per thread (its column group does not
  // change with the row iteration), so they are loaded here, ahead of the main loop, and the
  // block's 128 row statistics are combined from the producer's partials into LDS behind the
  // main loop (one float2 per row, past the staging / epilogue image: same __shared__ array)
  float cv1[8], cv2[8], cv3[8], cv4[8];
  uint4 lg = {}, lb = {};
  float2 pr[8];
  float2* S = (float2*)(smem + kLdsBytes);
  if constexpr (needs_rowstats(MODE)) {
    const long m = m0 + (tid & 127);
    const long mr = m < ep.M ? m : ep.M - 1;
    if (tid < 128) {
#pragma unroll
      for (int i = 0; i < 8; ++i) pr[i] = i < ep.np ? ep.pin[mr * ep.np + i] : make_float2(0.f, 0.f);
    }
  }
  if constexpr (is_rope(MODE) && is_fold(MODE)) {
    const int head = (tid >> 2) & 1, d0 = (tid & 3) * 8;
    const int pc = d0 < 16 ? d0 : d0 + 16;
    const float* c1 = ep.c1 + n0 + head * 64 + pc;
    const float* c2 = ep.c2 + n0 + head * 64 + pc;
    load8f(c1, cv1); load8f(c2, cv2); load8f(c1 + 16, cv3); load8f(c2 + 16, cv4);
  } else if constexpr (is_swiglu(MODE) && is_fold(MODE)) {
    const int c8 = (tid & 7) * 8, uc = 32 * (c8 >> 4) + (c8 & 15);
    load8f(ep.c1 + n0 + uc, cv1); load8f(ep.c2 + n0 + uc, cv2);
    load8f(ep.c1 + n0 + uc + 16, cv3); load8f(ep.c2 + n0 + uc + 16, cv4);
  } else if constexpr (MODE == NOMIC_EPI_RES_LN_STATS) {
    const int c8 = (tid & 15) * 8;
    lg = *(const uint4*)(ep.lng + n0 + c8);
    lb = *(const uint4*)(ep.lnb + n0 + c8);
  }
  // LDS: [A0 | B0 | A1 | B1], 16 KB each
  stage_tile<AS>(A, lda, m0, 0, smem, wave, lane);
  stage_tile<AS>(W, ldw, n0, 0, smem + kTileBytes, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (needs_rowstats(MODE)) {
    if (tid < 128) {  // Chan's combination of equal-size partials (as k_row_stats)
      float mean = 0.f, m2 = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) mean += pr[i].x;  // absent partials are zero
      mean /= (float)ep.np;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = pr[i].x - mean;
        if (i < ep.np) m2 += pr[i].y + (float)BN * d * d;
      }
      S[tid] = make_float2(mean, rsqrtf(m2 / ((float)BN * (float)ep.np) + ep.eps));
    }
  }
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      char* nb = smem + (cur ^ 1) * 2 * kTileBytes;
      stage_tile<AS>(A, lda, m0, (kt + 1) * BK, nb, wave, lane);
      stage_tile<AS>(W, ldw, n0, (kt + 1) * BK, nb + kTileBytes, wave, lane);
    }
    const char* ta = smem + cur * 2 * kTileBytes;
    const char* tb = ta + kTileBytes;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_frag(ta, wm * 64 + i * 16 + fr, kk * 4 + fq);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = lds_frag(tb, wn * 64 + j * 16 + fr, kk * 4 + fq);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS (fp32) -> 16-B output chunks --------
  float* E = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        E[(wm * 64 + i * 16 + fq * 4 + r) * kEpiStride + wn * 64 + j * 16 + fr] = acc[i][j][r];
  __syncthreads();

  if constexpr (is_rowstore(MODE)) {
#pragma unroll
    for (int it = 0; it < (BM * BN / 8) / kThreads; ++it) {
      const int q = tid + it * kThreads;
      const int row = q >> 4, c8 = (q & 15) * 8;  // 16 consecutive lanes share a row
      const long gm = m0 + row;
      const bool ok = gm < ep.M;
      if (!is_stats(MODE) && !ok) continue;      // stats modes keep every lane for the shuffles
      const float4 v0 = *(const float4*)&E[row * kEpiStride + c8];
      const float4 v1 = *(const float4*)&E[row * kEpiStride + c8 + 4];
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      if constexpr (MODE != NOMIC_EPI_STORE) {
        const long gr = ok ? gm : ep.M - 1;
        const uint4 rr = *(const uint4*)(ep.res + gr * ep.ldr + n0 + c8);
        const uint32_t rw[4] = {rr.x, rr.y, rr.z, rr.w};
        float r[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          r[2 * e] = bf2f((uint16_t)(rw[e] & 0xffff));
          r[2 * e + 1] = bf2f((uint16_t)(rw[e] >> 16));
        }
        if constexpr (MODE == NOMIC_EPI_RES_LN_STATS) {
          const float2 st = S[row];
          const uint32_t gw[4] = {lg.x, lg.y, lg.z, lg.w}, bw[4] = {lb.x, lb.y, lb.z, lb.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t g2 = gw[e >> 1], b2 = bw[e >> 1];
            const float gf = bf2f((uint16_t)(e & 1 ? g2 >> 16 : g2 & 0xffff));
            const float bf = bf2f((uint16_t)(e & 1 ? b2 >> 16 : b2 & 0xffff));
            r[e] = (r[e] - st.x) * st.y * gf + bf;
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
      uint4 o;
      o.x = pk2(v[0], v[1]);
      o.y = pk2(v[2], v[3]);
      o.z = pk2(v[4], v[5]);
      o.w = pk2(v[6], v[7]);
      if (ok) *(uint4*)(ep.out + gm * ep.ldo + n0 + c8) = o;
      if constexpr (is_stats(MODE)) {
        // statistics of the stored (bf16-rounded) values: the consumer folds against exactly them
        const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
        float vr[8], sm = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          vr[e] = bf2f((uint16_t)(e & 1 ? ow[e >> 1] >> 16 : ow[e >> 1] & 0xffff));
          sm += vr[e];
        }
        const float mean = sum16(sm) * (1.f / BN);
        float m2 = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) m2 += (vr[e] - mean) * (vr[e] - mean);
        m2 = sum16(m2);
        if (ok && (lane & 15) == 0) ep.part[gm * ntiles + nt] = make_float2(mean, m2);
      }
    }
  } else if constexpr (is_swiglu(MODE)) {
    // block columns: [up16 | gate16] x 4 (pack_upgate) of output columns nt*64 + 0..63
#pragma unroll
    for (int it = 0; it < (BM * 64 / 8) / kThreads; ++it) {
      const int q = tid + it * kThreads;
      const int row = q >> 3, c8 = (q & 7) * 8;
      const long gm = m0 + row;
      if (gm >= ep.M) continue;
      const int uc = 32 * (c8 >> 4) + (c8 & 15);
      float o[8];
      float2 st;
      if constexpr (is_fold(MODE)) st = S[row];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float up = E[row * kEpiStride + uc + e];
        float g = E[row * kEpiStride + uc + 16 + e];
        if constexpr (is_fold(MODE)) {
          up = fold(up, st, cv1[e], cv2[e]);
          g = fold(g, st, cv3[e], cv4[e]);
        }
        o[e] = swiglu(up, g);
      }
      uint4 w;
      w.x = pk2(o[0], o[1]);
      w.y = pk2(o[2], o[3]);
      w.z = pk2(o[4], o[5]);
      w.w = pk2(o[6], o[7]);
      *(uint4*)(ep.out + gm * ep.ldo + (long)nt * 64 + c8) = w;
    }
  } else if constexpr (is_rope(MODE)) {
    // two 64-wide heads per block; NEOX rotation pairs (d, d + 32)
#pragma unroll
    for (int it = 0; it < (BM * 2 * 4) / kThreads; ++it) {
      const int q = tid + it * kThreads;
      const int row = q >> 3, head = (q >> 2) & 1, d0 = (q & 3) * 8;
      const long gm = m0 + row;
      if (gm >= ep.M) continue;
      const int cb = head * 64;
      const long gcol = n0 + cb;
      const int pc = d0 < 16 ? d0 : d0 + 16;  // pack_qkv: [d0-15 | d32-47 | d16-31 | d48-63]
      float x1[8], x2[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        x1[e] = E[row * kEpiStride + cb + pc + e];
        x2[e] = E[row * kEpiStride + cb + pc + 16 + e];
      }
      if constexpr (is_fold(MODE)) {
        const float2 st = S[row];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          x1[e] = fold(x1[e], st, cv1[e], cv2[e]);
          x2[e] = fold(x2[e], st, cv3[e], cv4[e]);
        }
      }
      if (gcol < ep.rope_cols) {
        const float* cs = ep.rope + (long)ep.pos[gm] * 64 + d0 * 2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float c = cs[2 * e], s = cs[2 * e + 1];
          const float a = x1[e], b = x2[e];
          x1[e] = a * c - b * s;
          x2[e] = b * c + a * s;
        }
      }
      uint4 w1, w2;
      w1.x = pk2(x1[0], x1[1]);
      w1.y = pk2(x1[2], x1[3]);
      w1.z = pk2(x1[4], x1[5]);
      w1.w = pk2(x1[6], x1[7]);
      w2.x = pk2(x2[0], x2[1]);
      w2.y = pk2(x2[2], x2[3]);
      w2.z = pk2(x2[4], x2[5]);
      w2.w = pk2(x2[6], x2[7]);
      *(uint4*)(ep.out + gm * ep.ldo + gcol + d0) = w1;
      *(uint4*)(ep.out + gm * ep.ldo + gcol + d0 + 32) = w2;
    }
  } else if constexpr (MODE == NOMIC_EPI_F32) {
    float* outf = (float*)ep.out;
#pragma unroll
    for (int it = 0; it < (BM * BN / 4) / kThreads; ++it) {
      const int q = tid + it * kThreads;
      const int row = q >> 5, c4 = (q & 31) * 4;
      const long gm = m0 + row;
      if (gm >= ep.M) continue;
      *(float4*)(outf + gm * ep.ldo + n0 + c4) = *(const float4*)&E[row * kEpiStride + c4];
    }
  }
}

// ===========================================================================
// 256x256 tile, 8 waves (2M x 4N), 4 phases per K-tile, LDS-DMA prefetch kept
// in flight ACROSS barriers (counted vmcnt, raw s_barrier): the structure of
// the guide's 8-phase template (cdna_hip_programming.md §5 "The 256² 8-phase
// template"), with this kernel's own phase/stage schedule:
//
//   LDS = 2 buffers x [A0 | A1 | B0 | B1] half-tiles (128 rows x BK=64 bf16,
//   16 KB each; XOR-swizzled on the global source address).  Wave (wr, wn)
//   owns rows {qm*128 + wr*64 + 0..63} and cols {qn*128 + wn*32 + 0..31} for
//   quadrants qm, qn in {0,1}, so quadrant (qm, qn) reads only half-tiles
//   A<qm>, B<qn>.  Per K-tile t (buffer t&1):
//     phase 1: read A0,B0 -> MFMA (0,0); stage A1(t+1)
//     phase 2: read B1    -> MFMA (0,1); stage A0(t+2)
//     phase 3: read A1    -> MFMA (1,0); stage B0(t+2)
//     phase 4:               MFMA (1,1); stage B1(t+2)
//   Every half-tile is staged >= 1 phase after its previous contents were
//   read (WAR, separated by a barrier) and read >= 6 phases after it was
//   staged (RAW: the reading phase first waits vmcnt(#glds issued after it),
//   then the barrier).  Up to 6 half-tiles (12 DMA per lane) stay in flight.
// Epilogue: two 128-row halves through one fp32 LDS image (128 x 260).
// ===========================================================================
constexpr int kThreads2 = 512;
constexpr int kHalfBytes = 128 * BK * 2;           // 16 KB
constexpr int kBufBytes = 4 * kHalfBytes;          // 64 KB
constexpr int kEpi2Stride = 256 + 4;
constexpr int kLds2Bytes = (128 * kEpi2Stride * 4 > 2 * kBufBytes) ? 128 * kEpi2Stride * 4 : 2 * kBufBytes;

__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {  // wave-uniform: scalar branch to an immediate count
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint4 pack8(const float* v) {
  uint4 o;
  o.x = pk2(v[0], v[1]);
  o.y = pk2(v[2], v[3]);
  o.z = pk2(v[4], v[5]);
  o.w = pk2(v[6], v[7]);
  return o;
}

// ILV > 0: each phase's two LDS-DMA instructions are issued between its MFMA groups (before the
// groups u = ILV and ILV + 4 of the 8 (kk, i) groups of 2 MFMAs) instead of all before the first
// MFMA -- a DMA instruction's ~100-cycle issue cost then overlaps the other wave's MFMAs on the
// SIMD instead of holding both waves off the matrix core right after the barrier (the finding of
// gemm_rln.hip's ILV variants).  The issue ORDER of the DMAs is unchanged, so the counted vmcnt
// waits and the WAR/RAW distances of the phase schedule hold as they are.
// EPI 1 (SWIGLU only): the SwiGLU is applied in registers -- with pack_upgate's [up16 | gate16]
// column blocks, a lane's accumulators acc[..][j = 0] and acc[..][j = 1] are the up and gate values of
// the same output -- and the bf16 results are paired across lanes (lane ^ 1, one DPP move) into
// 4-B LDS writes of a 256 x 128 bf16 image, read back as 16-B row chunks: 32 ds_write_b32 per lane
// instead of 128 fp32 ones, one barrier pair instead of two.
// PP 1: ping-pong main loop (the guide's staggered 8-wave schedule, cdna_hip_programming.md §5 "The 256²
// 8-phase template"): every phase is a LOAD section (its fragment ds_reads, one half-tile of LDS-DMA,
// lgkmcnt(0)) and an MFMA section, each closed by a barrier, and waves 4-7 start one barrier behind
// waves 0-3, so on every SIMD one wave's 16 MFMAs run beside its partner's loads.  Counted vmcnt(6)
// once per K-tile (phase 4) retires the next K-tile; a half-tile is restaged one phase after its last
// read, which is safe because each load section drains its reads before its closing barrier.
template <int MODE, int ILV = 0, int EPI = 0, int PP = 0>
__global__ __launch_bounds__(kThreads2, 1) void k_gemm256(const uint16_t* __restrict__ A, long lda,
                                                          const uint16_t* __restrict__ W, long ldw, int K,
                                                          int mtiles, int ntiles, EpiArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wn = wave & 3;
  int mt, nt;
  remap_tile(blockIdx.x, mtiles * ntiles, ntiles, ep.gn, mt, nt);
  const long m0 = (long)mt * 256, n0 = (long)nt * 256;

  // per-lane DMA source offsets (elements): half h, instruction i -> 8-row block (i*8 + wave)
  const int srow = lane >> 3, schunk = ((lane & 7) ^ srow) * 8;
  uint32_t offA[2][2], offB[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = h * 128 + (i * 8 + wave) * 8 + srow;
      const long gr = (m0 + r < ep.M) ? m0 + r : ep.M - 1;  // clamp: tail rows re-read row M-1, never stored
      offA[h][i] = (uint32_t)(gr * lda + schunk);
      offB[h][i] = (uint32_t)((n0 + r) * ldw + schunk);
    }
  auto stage_one = [&](int which, int t, int buf, int i) {  // which: 0 A0, 1 A1, 2 B0, 3 B1
    const uint16_t* base = (which < 2 ? A : W) + (long)t * BK;
    char* dst = smem + buf * kBufBytes + which * kHalfBytes;
    const uint32_t off = which == 0 ? offA[0][i] : which == 1 ? offA[1][i] : which == 2 ? offB[0][i] : offB[1][i];
    if constexpr (PP == 2)
      spl::glds16_asm(base + off, dst + (i * 8 + wave) * 1024);  // counted LDS waits (glds_asm.hpp)
    else
      __builtin_amdgcn_global_load_lds((gbl_void*)(base + off), (lds_void*)(dst + (i * 8 + wave) * 1024), 16, 0, 0);
  };
  auto stage = [&](int which, int t, int buf) {
    stage_one(which, t, buf, 0);
    stage_one(which, t, buf, 1);
  };

  // fragment read addressing: row-in-half R = base16 + (lane&15), chunk kk*4 + (lane>>4), swizzled by R&7 = lane&7
  const int frow = (lane & 15) * 128;
  const int fsw0 = ((0 * 4 + (lane >> 4)) ^ (lane & 7)) << 4;
  const int fsw1 = ((1 * 4 + (lane >> 4)) ^ (lane & 7)) << 4;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  // prologue, in the steady-state issue order: A0 B0 B1 A1 (t=0), A0 B0 B1 (t=1)
  stage(0, 0, 0); stage(2, 0, 0); stage(3, 0, 0); stage(1, 0, 0);
  if (nk > 1) { stage(0, 1, 1); stage(2, 1, 1); stage(3, 1, 1); }

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  // one quadrant's 16 MFMAs (kk, i, j), with the phase's stage issued before them (ILV 0) or
  // between the (kk, i) groups u = ILV and ILV + 4 (ILV > 0)
  auto mma_phase = [&](f32x4 (&ac)[4][2], bf16x8 (&bf)[2][2], int which, int st, int sbuf, bool go) {
    if (ILV == 0 && go) stage(which, st, sbuf);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (ILV > 0) {
          if (go && kk * 4 + i == ILV) stage_one(which, st, sbuf, 0);
          if (go && kk * 4 + i == ILV + 4) stage_one(which, st, sbuf, 1);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
          ac[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], ac[i][j], 0, 0, 0);
        if constexpr (ILV > 0) __builtin_amdgcn_sched_barrier(0);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  if constexpr (PP == 1) {
    auto lgk0 = [] {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = [] {
      __builtin_amdgcn_sched_barrier(0);
      raw_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    auto mma_q = [&](f32x4 (&ac)[4][2], bf16x8 (&bf)[2][2]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            ac[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], ac[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    wait_vm(nk > 1 ? 6 : 0);  // K-tile 0 landed (K-tile 1's three half-tiles may still fly)
    bar();
    if (wr == 1) bar();  // the stagger
    auto pp_kt = [&](int t, auto n1c, auto n2c) {
      constexpr bool n1 = decltype(n1c)::value, n2 = decltype(n2c)::value;
      const int buf = t & 1;
      const char* hA0 = smem + buf * kBufBytes;
      const char* hA1 = hA0 + kHalfBytes;
      const char* hB0 = hA0 + 2 * kHalfBytes;
      const char* hB1 = hA0 + 3 * kHalfBytes;
      // phase 1: quadrant (0,0) -- read A0, B0; stage A1(t+1)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        b0[j][0] = *(const bf16x8*)(hB0 + (wn * 32 + j * 16) * 128 + frow + fsw0);
        b0[j][1] = *(const bf16x8*)(hB0 + (wn * 32 + j * 16) * 128 + frow + fsw1);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i][0] = *(const bf16x8*)(hA0 + (wr * 64 + i * 16) * 128 + frow + fsw0);
        af[i][1] = *(const bf16x8*)(hA0 + (wr * 64 + i * 16) * 128 + frow + fsw1);
      }
      if (n1) stage(1, t + 1, buf ^ 1);
      lgk0();
      bar();
      mma_q(acc[0][0], b0);
      bar();
      // phase 2: quadrant (0,1) -- read B1; stage A0(t+2)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        b1[j][0] = *(const bf16x8*)(hB1 + (wn * 32 + j * 16) * 128 + frow + fsw0);
        b1[j][1] = *(const bf16x8*)(hB1 + (wn * 32 + j * 16) * 128 + frow + fsw1);
      }
      if (n2) stage(0, t + 2, buf);
      lgk0();
      bar();
      mma_q(acc[0][1], b1);
      bar();
      // phase 3: quadrant (1,0) -- read A1; stage B0(t+2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i][0] = *(const bf16x8*)(hA1 + (wr * 64 + i * 16) * 128 + frow + fsw0);
        af[i][1] = *(const bf16x8*)(hA1 + (wr * 64 + i * 16) * 128 + frow + fsw1);
      }
      if (n2) stage(2, t + 2, buf);
      lgk0();
      bar();
      mma_q(acc[1][0], b0);
      bar();
      // phase 4: quadrant (1,1) from registers; stage B1(t+2); retire K-tile t+1 (all but the 3 newest
      // half-tiles, which belong to K-tile t+2)
      if (n2) stage(3, t + 2, buf);
      wait_vm(n2 ? 6 : 0);
      bar();
      mma_q(acc[1][1], b1);
      bar();
    };
    // peeled: the steady-state K-tiles carry no staging branches (the counted waits and DMA issue are
    // straight-line code the compiler can schedule around)
    int t = 0;
    for (; t + 2 < nk; ++t) pp_kt(t, std::true_type{}, std::true_type{});
    if (t + 1 < nk) pp_kt(t++, std::true_type{}, std::false_type{});
    if (t < nk) pp_kt(t, std::false_type{}, std::false_type{});
    if (wr == 0) bar();  // equal barrier counts for both groups before the epilogue
  } else if constexpr (PP == 2) {
  // the lockstep loop below, peeled (no staging branches), with its fragment reads issued in the order
  // the MFMAs consume them (k-step 0's B and A fragments first) and pinned there, so the first MFMAs wait
  // only for their own operands (counted lgkmcnt) instead of the whole phase's reads
  auto rd = [](bf16x8& dst, const char* p) {
    dst = *(const bf16x8*)p;
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mm = [&](f32x4 (&ac)[4][2], bf16x8 (&bf)[2][2], int kk) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        ac[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], ac[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto ls_kt = [&](int t, auto n1c, auto n2c) {
    constexpr bool n1 = decltype(n1c)::value, n2 = decltype(n2c)::value;
    const int buf = t & 1;
    const char* hA0 = smem + buf * kBufBytes;
    const char* hA1 = hA0 + kHalfBytes;
    const char* hB0 = hA0 + 2 * kHalfBytes;
    const char* hB1 = hA0 + 3 * kHalfBytes;
    const char* pb0 = hB0 + (wn * 32) * 128 + frow;
    const char* pb1 = hB1 + (wn * 32) * 128 + frow;
    const char* pa0 = hA0 + (wr * 64) * 128 + frow;
    const char* pa1 = hA1 + (wr * 64) * 128 + frow;
    // ---- phase 1: quadrant (0,0)
    wait_vm(n1 ? 10 : 4);
    raw_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int fs = kk ? fsw1 : fsw0;
      rd(b0[0][kk], pb0 + fs);
      rd(b0[1][kk], pb0 + 16 * 128 + fs);
#pragma unroll
      for (int i = 0; i < 4; ++i) rd(af[i][kk], pa0 + i * 16 * 128 + fs);
    }
    if constexpr (n1) stage(1, t + 1, buf ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mm(acc[0][0], b0, 0);
    mm(acc[0][0], b0, 1);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 2: quadrant (0,1)
    wait_vm(n1 ? 10 : 2);
    raw_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int fs = kk ? fsw1 : fsw0;
      rd(b1[0][kk], pb1 + fs);
      rd(b1[1][kk], pb1 + 16 * 128 + fs);
    }
    if constexpr (n2) stage(0, t + 2, buf);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mm(acc[0][1], b1, 0);
    mm(acc[0][1], b1, 1);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 3: quadrant (1,0)
    wait_vm(n2 ? 10 : (n1 ? 8 : 0));
    raw_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int fs = kk ? fsw1 : fsw0;
#pragma unroll
      for (int i = 0; i < 4; ++i) rd(af[i][kk], pa1 + i * 16 * 128 + fs);
    }
    if constexpr (n2) stage(2, t + 2, buf);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mm(acc[1][0], b0, 0);
    mm(acc[1][0], b0, 1);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 4: quadrant (1,1), registers only (B1's last read was phase 2: a barrier ago)
    if constexpr (n2) stage(3, t + 2, buf);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mm(acc[1][1], b1, 0);
    mm(acc[1][1], b1, 1);
    __builtin_amdgcn_s_setprio(0);
  };
  int t = 0;
  for (; t + 2 < nk; ++t) ls_kt(t, std::true_type{}, std::true_type{});
  if (t + 1 < nk) ls_kt(t++, std::true_type{}, std::false_type{});
  if (t < nk) ls_kt(t, std::false_type{}, std::false_type{});
  } else
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const char* hA0 = smem + buf * kBufBytes;
    const char* hA1 = hA0 + kHalfBytes;
    const char* hB0 = hA0 + 2 * kHalfBytes;
    const char* hB1 = hA0 + 3 * kHalfBytes;
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    // ---- phase 1: quadrant (0,0)
    wait_vm(n1 ? 10 : 4);
    raw_barrier();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b0[j][0] = *(const bf16x8*)(hB0 + (wn * 32 + j * 16) * 128 + frow + fsw0);
      b0[j][1] = *(const bf16x8*)(hB0 + (wn * 32 + j * 16) * 128 + frow + fsw1);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *(const bf16x8*)(hA0 + (wr * 64 + i * 16) * 128 + frow + fsw0);
      af[i][1] = *(const bf16x8*)(hA0 + (wr * 64 + i * 16) * 128 + frow + fsw1);
    }
    mma_phase(acc[0][0], b0, 1, t + 1, buf ^ 1, n1);
    // ---- phase 2: quadrant (0,1)
    wait_vm(n1 ? 10 : 2);
    raw_barrier();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b1[j][0] = *(const bf16x8*)(hB1 + (wn * 32 + j * 16) * 128 + frow + fsw0);
      b1[j][1] = *(const bf16x8*)(hB1 + (wn * 32 + j * 16) * 128 + frow + fsw1);
    }
    mma_phase(acc[0][1], b1, 0, t + 2, buf, n2);
    // ---- phase 3: quadrant (1,0)
    wait_vm(n2 ? 10 : (n1 ? 8 : 0));
    raw_barrier();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *(const bf16x8*)(hA1 + (wr * 64 + i * 16) * 128 + frow + fsw0);
      af[i][1] = *(const bf16x8*)(hA1 + (wr * 64 + i * 16) * 128 + frow + fsw1);
    }
    mma_phase(acc[1][0], b0, 2, t + 2, buf, n2);
    // ---- phase 4: quadrant (1,1), registers only (B1's last read was phase 2: a barrier ago)
    mma_phase(acc[1][1], b1, 3, t + 2, buf, n2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if constexpr (MODE == NOMIC_EPI_SWIGLU && EPI == 1) {
    constexpr int kS = 128 + 8;  // bf16 row stride of the image (272 B: conflict-free 4-B writes)
    uint16_t* E16 = (uint16_t*)smem;
    const int fq = lane >> 4, fr = lane & 15;
    const bool odd = fr & 1;
    __syncthreads();  // every wave is done reading the last K-tile's operands
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint32_t b[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) b[r] = f2bf(swiglu(acc[qm][qn][i][0][r], acc[qm][qn][i][1][r]));
          // even lanes write rows r = 0, 1 at columns (fr, fr + 1), odd lanes rows 2, 3 at (fr - 1, fr)
          const uint32_t send = odd ? (b[0] | b[1] << 16) : (b[2] | b[3] << 16);
          const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xf, 0xf, false);
          const uint32_t w0 = odd ? ((recv & 0xffffu) | b[2] << 16) : (b[0] | recv << 16);
          const uint32_t w1 = odd ? ((recv >> 16) | b[3] << 16) : (b[1] | (recv & 0xffff0000u));
          const int row = qm * 128 + wr * 64 + i * 16 + fq * 4 + (odd ? 2 : 0);
          const int col = (qn * 4 + wn) * 16 + (fr & ~1);
          *(uint32_t*)(E16 + row * kS + col) = w0;
          *(uint32_t*)(E16 + (row + 1) * kS + col) = w1;
        }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < (256 * 16) / kThreads2; ++it) {
      const int q = tid + it * kThreads2;
      const int row = q >> 4, c = q & 15;
      const long gm = m0 + row;
      if (gm >= ep.M) continue;
      *(uint4*)(ep.out + gm * ep.ldo + (long)nt * 128 + c * 8) = *(const uint4*)(E16 + row * kS + c * 8);
    }
    return;
  }

  // ---- epilogue: two 128-row halves through the fp32 LDS image ------------
  float* E = (float*)smem;
  const int fq = lane >> 4, fr = lane & 15;
#pragma unroll
  for (int qm = 0; qm < 2; ++qm) {
    __syncthreads();
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            E[(wr * 64 + i * 16 + fq * 4 + r) * kEpi2Stride + qn * 128 + wn * 32 + j * 16 + fr] = acc[qm][qn][i][j][r];
    __syncthreads();
    const long mh = m0 + qm * 128;
    if constexpr (MODE == NOMIC_EPI_STORE || MODE == NOMIC_EPI_RESIDUAL) {
#pragma unroll
      for (int it = 0; it < (128 * 256 / 8) / kThreads2; ++it) {
        const int q = tid + it * kThreads2;
        const int row = q >> 5, c8 = (q & 31) * 8;
        const long gm = mh + row;
        if (gm >= ep.M) continue;
        const float4 v0 = *(const float4*)&E[row * kEpi2Stride + c8];
        const float4 v1 = *(const float4*)&E[row * kEpi2Stride + c8 + 4];
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        if constexpr (MODE == NOMIC_EPI_RESIDUAL) {
          const uint4 rr = *(const uint4*)(ep.res + gm * ep.ldr + n0 + c8);
          const uint32_t rw[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += bf2f((uint16_t)(rw[e] & 0xffff));
            v[2 * e + 1] += bf2f((uint16_t)(rw[e] >> 16));
          }
        }
        *(uint4*)(ep.out + gm * ep.ldo + n0 + c8) = pack8(v);
      }
    } else if constexpr (MODE == NOMIC_EPI_SWIGLU) {
      // block columns [up16 | gate16] x 8 (pack_upgate) -> output columns nt*128 + 0..127
#pragma unroll
      for (int it = 0; it < (128 * 128 / 8) / kThreads2; ++it) {
        const int q = tid + it * kThreads2;
        const int row = q >> 4, oc = (q & 15) * 8;
        const long gm = mh + row;
        if (gm >= ep.M) continue;
        const int uc = 32 * (oc >> 4) + (oc & 15);
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float up = E[row * kEpi2Stride + uc + e];
          const float g = E[row * kEpi2Stride + uc + 16 + e];
          o[e] = swiglu(up, g);
        }
        *(uint4*)(ep.out + gm * ep.ldo + (long)nt * 128 + oc) = pack8(o);
      }
    } else if constexpr (MODE == NOMIC_EPI_ROPE) {
      // four 64-wide heads per block; NEOX rotation pairs (d, d + 32)
#pragma unroll
      for (int it = 0; it < (128 * 4 * 4) / kThreads2; ++it) {
        const int q = tid + it * kThreads2;
        const int row = q >> 4, head = (q >> 2) & 3, d0 = (q & 3) * 8;
        const long gm = mh + row;
        if (gm >= ep.M) continue;
        const int cb = head * 64;
        const long gcol = n0 + cb;
        const int pc = d0 < 16 ? d0 : d0 + 16;  // pack_qkv layout
        float x1[8], x2[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          x1[e] = E[row * kEpi2Stride + cb + pc + e];
          x2[e] = E[row * kEpi2Stride + cb + pc + 16 + e];
        }
        if (gcol < ep.rope_cols) {
          const float* cs = ep.rope + (long)ep.pos[gm] * 64 + d0 * 2;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float c = cs[2 * e], s = cs[2 * e + 1];
            const float a = x1[e], b = x2[e];
            x1[e] = a * c - b * s;
            x2[e] = b * c + a * s;
          }
        }
        *(uint4*)(ep.out + gm * ep.ldo + gcol + d0) = pack8(x1);
        *(uint4*)(ep.out + gm * ep.ldo + gcol + d0 + 32) = pack8(x2);
      }
    } else if constexpr (MODE == NOMIC_EPI_F32) {
      float* outf = (float*)ep.out;
#pragma unroll
      for (int it = 0; it < (128 * 256 / 4) / kThreads2; ++it) {
        const int q = tid + it * kThreads2;
        const int row = q >> 6, c4 = (q & 63) * 4;
        const long gm = mh + row;
        if (gm >= ep.M) continue;
        *(float4*)(outf + gm * ep.ldo + n0 + c4) = *(const float4*)&E[row * kEpi2Stride + c4];
      }
    }
  }
}

}  // namespace

namespace {

int g_num_cus = 256;  // MI355X: 256 CUs in 8 XCDs; refreshed from the device on first use

template <typename F>
void allow_lds(F* f, int bytes) {
  (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// Kernel choice (NOMIC_GEMM): 0 = auto, 128 = the 128^2 kernel, 256 = the 256^2 kernel.  The
// persistent / stream-K 256^2 kernel (512-515), the DMA-interleave (ILV), ping-pong (PP), asm-DMA
// 128^2 (AS128), register-SwiGLU-epilogue and persistent register-epilogue (300, gemm_pt.hip, round
// 5) knobs measured slower or equal and are gone; their A/B history is in profiles/r1_gemm_*.jsonl
// .. r3_gemm_*, r5/gemm_pt_ab_r5c.jsonl.
int g_variant = -1;
int gemm_variant() {
  if (g_variant < 0) {
    const char* e = getenv("NOMIC_GEMM");
    const int v = e ? atoi(e) : 0;
    g_variant = v == 128 || v == 256 ? v : 0;
  }
  return g_variant;
}

// band width of the tile order: the largest divisor of ntiles <= cap (NOMIC_GEMM_GN overrides;
// 0 = row-major)
int band_width(int ntiles, int cap) {
  static const int env = [] {
    const char* v = getenv("NOMIC_GEMM_GN");
    return v && *v ? atoi(v) : -1;
  }();
  if (env == 0) return ntiles;
  if (env > 0) cap = env;
  for (int g = cap < ntiles ? cap : ntiles; g > 1; --g)
    if (ntiles % g == 0) return g;
  return 1;
}

template <int MODE>
int launch(const uint16_t* A, long lda, const uint16_t* W, long ldw, long M, int N, int K, EpiArgs ep,
           hipStream_t s) {
  if (K % BK || N % BN || M <= 0) return (int)hipErrorInvalidValue;
  const long mpad = (M + 255) / 256 * 256;
  const bool fits = N % 256 == 0 && mpad * lda < (1L << 31) && (long)N * ldw < (1L << 31);
  const int var = gemm_variant();
  // the 256^2 kernel runs 1 block/CU with a serial prologue / epilogue per tile: it wins once there
  // are several waves of tiles.  From 1024 tiles: the qkv projection at 32768 tokens (1152 tiles)
  // measured 137.4 us on it against 144.5 us on the 128^2 kernel (round-3 trace); the SwiGLU GEMM
  // has 3072.  The statistics epilogues exist in the 128^2 kernel only.
  constexpr bool k256_ok = MODE <= NOMIC_EPI_F32;
  const long tiles256 = fits ? (mpad / 256) * (N / 256) : 0;
  static const long min_tiles = [] {  // NOMIC_GEMM256_MIN_TILES (A/B knob)
    const char* e = getenv("NOMIC_GEMM256_MIN_TILES");
    return e && atol(e) > 0 ? atol(e) : 1024L;
  }();
  if (k256_ok && fits && (var == 256 || (var == 0 && tiles256 >= min_tiles))) {
    static bool attr = [] {
      allow_lds(k_gemm256<MODE, 0, 0, 2>, kLds2Bytes);
      return true;
    }();
    (void)attr;
    const int mtiles = (int)(mpad / 256), ntiles = N / 256;
    ep.gn = band_width(ntiles, 4);
    if constexpr (k256_ok)
      hipLaunchKernelGGL((k_gemm256<MODE, 0, 0, 2>), dim3(mtiles * ntiles), dim3(kThreads2), kLds2Bytes, s, A, lda, W,
                         ldw, K, mtiles, ntiles, ep);
    return (int)hipGetLastError();
  }
  const int mtiles = (int)((M + BM - 1) / BM), ntiles = N / BN;
  ep.gn = band_width(ntiles, 8);
  constexpr int lds = kLdsBytes + (needs_rowstats(MODE) ? BM * 8 : 0);
  hipLaunchKernelGGL(k_gemm_nt<MODE>, dim3(mtiles * ntiles), dim3(kThreads), lds, s, A, lda, W, ldw, K, mtiles, ntiles,
                     ep);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int nomic_gemm_set_variant(int variant) {
  const int prev = gemm_variant();
  g_variant = variant == 128 || variant == 256 ? variant : 0;
  return prev;
}

extern "C" int nomic_gemm_ln(int mode, const void* A, long lda, const void* W, long ldw, long M, int N, int K,
                             void* out, long ldo, const void* res, long ldr, const float* rope, const int32_t* pos,
                             int rope_cols, const float* part_in, int nparts, float eps, const float* c1,
                             const float* c2, const void* ln_g, const void* ln_b, float* part, hipStream_t s) {
  EpiArgs ep{(uint16_t*)out, ldo, (const uint16_t*)res, ldr, rope, pos, rope_cols, M, 1, (const float2*)part_in,
             nparts, eps, c1, c2, (const uint16_t*)ln_g, (const uint16_t*)ln_b, (float2*)part};
  // operands each mode reads must be there (a fold / stats launch without them would fault)
  if ((needs_rowstats(mode) && (!part_in || nparts < 1 || nparts > 8)) || (is_fold(mode) && (!c1 || !c2)) ||
      (is_stats(mode) && (!part || !res || N % BN)) || (mode == NOMIC_EPI_RES_LN_STATS && (!ln_g || !ln_b)) ||
      (mode == NOMIC_EPI_RESIDUAL && !res) || (is_rope(mode) && (!rope || !pos)))
    return (int)hipErrorInvalidValue;
  const auto* a = (const uint16_t*)A;
  const auto* w = (const uint16_t*)W;
  switch (mode) {
    case NOMIC_EPI_STORE: return launch<NOMIC_EPI_STORE>(a, lda, w, ldw, M, N, K, ep, s);
    case NOMIC_EPI_RESIDUAL: return launch<NOMIC_EPI_RESIDUAL>(a, lda, w, ldw, M, N, K, ep, s);
    case NOMIC_EPI_SWIGLU: return launch<NOMIC_EPI_SWIGLU>(a, lda, w, ldw, M, N, K, ep, s);
    case NOMIC_EPI_ROPE: return launch<NOMIC_EPI_ROPE>(a, lda, w, ldw, M, N, K, ep, s);
    case NOMIC_EPI_F32: return launch<NOMIC_EPI_F32>(a, lda, w, ldw, M, N, K, ep, s);
    case NOMIC_EPI_ROPE_FOLD: return launch<NOMIC_EPI_ROPE_FOLD>(a, lda, w, ldw, M, N, K, ep, s);
    case NOMIC_EPI_SWIGLU_FOLD: return launch<NOMIC_EPI_SWIGLU_FOLD>(a, lda, w, ldw, M, N, K, ep, s);
    case NOMIC_EPI_RES_STATS: return launch<NOMIC_EPI_RES_STATS>(a, lda, w, ldw, M, N, K, ep, s);
    case NOMIC_EPI_RES_LN_STATS: return launch<NOMIC_EPI_RES_LN_STATS>(a, lda, w, ldw, M, N, K, ep, s);
    default: return (int)hipErrorInvalidValue;
  }
}

extern "C" int nomic_gemm(int mode, const void* A, long lda, const void* W, long ldw, long M, int N, int K, void* out,
                          long ldo, const void* res, long ldr, const float* rope, const int32_t* pos, int rope_cols,
                          hipStream_t s) {
  if (mode > NOMIC_EPI_F32) return (int)hipErrorInvalidValue;  // the LN modes go through nomic_gemm_ln
  return nomic_gemm_ln(mode, A, lda, W, ldw, M, N, K, out, ldo, res, ldr, rope, pos, rope_cols, nullptr, 0, 0.f,
                       nullptr, nullptr, nullptr, nullptr, nullptr, s);
}

namespace {
// one thread per row: Chan's combination of equal-size (128-column) partials
__global__ void k_row_stats(const float2* __restrict__ part, int np, long M, float eps, float2* __restrict__ st) {
  const long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const float2* p = part + m * np;
  float mean = 0.f;
  for (int i = 0; i < np; ++i) mean += p[i].x;
  mean /= (float)np;
  float m2 = 0.f;
  for (int i = 0; i < np; ++i) {
    const float d = p[i].x - mean;
    m2 += p[i].y + (float)BN * d * d;
  }
  const float var = m2 / ((float)BN * (float)np);
  st[m] = make_float2(mean, rsqrtf(var + eps));
}
}  // namespace

extern "C" int nomic_row_stats(const float* part, int nparts, long M, float eps, float* st, hipStream_t s) {
  if (nparts <= 0 || M <= 0 || !part || !st) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_row_stats, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, (const float2*)part, nparts, M,
                     eps, (float2*)st);
  return (int)hipGetLastError();
}
