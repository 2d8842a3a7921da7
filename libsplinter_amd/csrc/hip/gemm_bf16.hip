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
  // stream-K hand-off of split tiles (k_gemm_p<.., SK>): slot s = fp32 partial of the tile shared by
  // blocks (in remapped order) s and s+1, published with flag[s] = gen
  float4* skws;
  uint32_t* skflag;
  uint32_t skgen;
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

// ===========================================================================
// Persistent 256x256 kernel with a REGISTER epilogue (variant 512, "p").
//
// One block per CU walks its tiles (blockIdx, +grid, ...; each through the
// same XCD/L2-band remap as the launch-per-tile kernels) as ONE stream of
// K-steps: the LDS-DMA stages of the next tile's first K-steps are issued
// during the current tile's last phases, so a tile change costs no pipeline
// refill.  The MFMA operands are swapped (W fragment as the A operand), so a
// lane's accumulator holds C[m][n .. n+3] (four consecutive output columns of
// one row) and the epilogue stores 8-B (16-B for fp32) chunks straight from
// registers: no LDS round trip, no barrier, and the LDS buffers can keep the
// next tile's stages in flight.  The epilogue's global ops are younger than
// those stages, so the counted vmcnt waits of the next phases stay correct
// (vmcnt retires in issue order: MI355X_MICROARCH.md, s_waitcnt).
//
// Epilogue layouts need pairs in one lane: SWIGLU weights are packed
// [up16 | gate16] per 16 outputs (models/nomic.py pack_upgate) and the QKV
// rows of each 64-wide head as [d0-15 | d32-47 | d16-31 | d48-63]
// (pack_qkv), so x1 = acc[..][j=0] and x2 = acc[..][j=1] of the same lane.
// ===========================================================================
__device__ __forceinline__ uint2 pack4(const float* v) {
  return make_uint2(pk2(v[0], v[1]), pk2(v[2], v[3]));
}

// AS: LDS-DMA from inline asm (glds_asm.hpp: counted lgkmcnt before the MFMA groups)
template <int MODE, bool PERSIST, bool SK = false, int ILV = 0, bool AS = false>
__global__ __launch_bounds__(kThreads2, 1) void k_gemm_p(const uint16_t* __restrict__ A, long lda,
                                                         const uint16_t* __restrict__ W, long ldw, int K,
                                                         int mtiles, int ntiles, EpiArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wn = wave & 3;
  const int nb = mtiles * ntiles, G = gridDim.x;
  const int nk = K / BK;  // >= 2 (launcher): a lookahead of two K-steps spans at most one tile change
  // Stream-K (SK) for tile counts that do not divide over the G blocks: nb = q*G + r with G = p*r.
  // Every block runs q whole tiles (ids v, v+G, ...) and then 1/p of one of the r remaining
  // tiles (k-range part*nk/p ..), so all blocks carry the same q*nk + nk/p K-steps and none idles
  // through a last partial wave of tiles.  v is the block's position in XCD order (blocks b, b+8,
  // ... run on one XCD), so the p parts of a split tile run on one XCD.  The parts end their
  // blocks' streams together: parts 1..p-1 store their fp32 partials, part 0 adds them and runs
  // the epilogue -- all after the K loop, with nothing else live.
  int my_tiles, total, k_first = 0, v = 0, q = 0, parts = 1;
  if constexpr (SK) {
    const int b = (int)blockIdx.x, x = b & 7, qq = G >> 3, rr = G & 7;
    v = (x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq) + (b >> 3);
    q = nb / G;
    parts = G / (nb - q * G);
    k_first = (v % parts) * (nk / parts);
    my_tiles = q + 1;
    total = q * nk + nk / parts;
  } else {
    my_tiles = PERSIST ? (nb - (int)blockIdx.x + G - 1) / G : 1;
    total = my_tiles * nk;
  }
  if (my_tiles <= 0) return;

  const int srow = lane >> 3, schunk = ((lane & 7) ^ srow) * 8;
  // per-lane DMA source offsets (elements, 32-bit as in k_gemm256) of the current tile (C) and the
  // next one (X): half h, instruction i -> row h*128 + (i*8 + wave)*8 + srow
  uint32_t offAc[2][2], offBc[2][2], offAx[2][2], offBx[2][2];
  long m0c = 0, n0c = 0;
  auto tile_offsets = [&](int ti, uint32_t (&oa)[2][2], uint32_t (&ob)[2][2], long& m0, long& n0) {
    int mt, nt;
    if constexpr (SK) {
      const int id = ti < q ? ti * G + v : q * G + v / parts;
      mt = id / ntiles;
      nt = id - mt * ntiles;
    } else {
      remap_tile((int)blockIdx.x + ti * G, nb, ntiles, ep.gn, mt, nt);
    }
    m0 = (long)mt * 256;
    n0 = (long)nt * 256;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = h * 128 + (i * 8 + wave) * 8 + srow;
        const long gr = (m0 + r < ep.M) ? m0 + r : ep.M - 1;  // clamp: tail rows re-read row M-1, never stored
        oa[h][i] = (uint32_t)(gr * lda + schunk);
        ob[h][i] = (uint32_t)((n0 + r) * ldw + schunk);
      }
  };
  tile_offsets(0, offAc, offBc, m0c, n0c);
  long m0x = m0c, n0x = n0c;
  if (my_tiles > 1) tile_offsets(1, offAx, offBx, m0x, n0x);
  else {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) { offAx[h][i] = offAc[h][i]; offBx[h][i] = offBc[h][i]; }
  }
  int ti = 0, kt = 0;

  // stage half-tile `which` (0 A0, 1 A1, 2 B0, 3 B1) of stream step g into buffer buf
  auto stage_one = [&](int which, int g, int buf, int i) {
    const bool nx = g >= (ti + 1) * nk;
    const int tl = ti + (nx ? 1 : 0);
    const int k0 = (g - tl * nk + (SK && tl == q ? k_first : 0)) * BK;
    const uint16_t* base = (which < 2 ? A : W) + k0;
    char* dst = smem + buf * kBufBytes + which * kHalfBytes;
    const int h = which & 1;
    const uint32_t off = which < 2 ? (nx ? offAx[h][i] : offAc[h][i]) : (nx ? offBx[h][i] : offBc[h][i]);
    if constexpr (AS)
      spl::glds16_asm(base + off, dst + (i * 8 + wave) * 1024);
    else
      __builtin_amdgcn_global_load_lds((gbl_void*)(base + off), (lds_void*)(dst + (i * 8 + wave) * 1024), 16, 0, 0);
  };
  auto stage = [&](int which, int g, int buf) {
    stage_one(which, g, buf, 0);
    stage_one(which, g, buf, 1);
  };

  const int frow = (lane & 15) * 128;
  const int fsw0 = ((0 * 4 + (lane >> 4)) ^ (lane & 7)) << 4;
  const int fsw1 = ((1 * 4 + (lane >> 4)) ^ (lane & 7)) << 4;
  const int fq = lane >> 4, fr = lane & 15;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue, in the steady-state issue order: A0 B0 B1 A1 (t=0), A0 B0 B1 (t=1)
  stage(0, 0, 0); stage(2, 0, 0); stage(3, 0, 0); stage(1, 0, 0);
  if (total > 1) { stage(0, 1, 1); stage(2, 1, 1); stage(3, 1, 1); }

  auto epilogue = [&]() {
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long m = m0c + qm * 128 + wr * 64 + i * 16 + fr;
        if (m < ep.M) {
#pragma unroll
          for (int qn = 0; qn < 2; ++qn) {
            const long nb0 = n0c + qn * 128 + wn * 32;  // this wave's 32-column group
            if constexpr (MODE == NOMIC_EPI_STORE || MODE == NOMIC_EPI_RESIDUAL) {
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const long n = nb0 + j * 16 + fq * 4;
                float v[4] = {acc[qm][qn][i][j][0], acc[qm][qn][i][j][1], acc[qm][qn][i][j][2],
                              acc[qm][qn][i][j][3]};
                if constexpr (MODE == NOMIC_EPI_RESIDUAL) {
                  const uint2 rr = *(const uint2*)(ep.res + m * ep.ldr + n);
                  v[0] += bf2f((uint16_t)(rr.x & 0xffff));
                  v[1] += bf2f((uint16_t)(rr.x >> 16));
                  v[2] += bf2f((uint16_t)(rr.y & 0xffff));
                  v[3] += bf2f((uint16_t)(rr.y >> 16));
                }
                *(uint2*)(ep.out + m * ep.ldo + n) = pack4(v);
              }
            } else if constexpr (MODE == NOMIC_EPI_F32) {
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const long n = nb0 + j * 16 + fq * 4;
                *(float4*)((float*)ep.out + m * ep.ldo + n) =
                    make_float4(acc[qm][qn][i][j][0], acc[qm][qn][i][j][1], acc[qm][qn][i][j][2],
                                acc[qm][qn][i][j][3]);
              }
            } else if constexpr (MODE == NOMIC_EPI_SWIGLU) {
              float o[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) o[e] = swiglu(acc[qm][qn][i][0][e], acc[qm][qn][i][1][e]);
              *(uint2*)(ep.out + m * ep.ldo + nb0 / 2 + fq * 4) = pack4(o);
            } else if constexpr (MODE == NOMIC_EPI_ROPE) {
              const long head0 = nb0 & ~63L;
              const int d = (int)(nb0 & 32) / 2 + fq * 4;  // packed half 0: d 0-15, half 1: d 16-31
              float x1[4], x2[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                x1[e] = acc[qm][qn][i][0][e];
                x2[e] = acc[qm][qn][i][1][e];
              }
              if (head0 < ep.rope_cols) {
                const float* cs = ep.rope + (long)ep.pos[m] * 64 + d * 2;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float c = cs[2 * e], s = cs[2 * e + 1];
                  const float a = x1[e], b = x2[e];
                  x1[e] = a * c - b * s;
                  x2[e] = b * c + a * s;
                }
              }
              *(uint2*)(ep.out + m * ep.ldo + head0 + d) = pack4(x1);
              *(uint2*)(ep.out + m * ep.ldo + head0 + 32 + d) = pack4(x2);
            }
          }
        }
      }
  };

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  int relax = 0;
  // as k_gemm256's: one quadrant's 16 MFMAs with the phase's stage before (ILV 0) or between them;
  // swapped operands (W fragment as the A operand)
  auto mma_phase = [&](f32x4 (&ac)[4][2], bf16x8 (&bf)[2][2], int which, int sg, int sbuf, bool go) {
    if (ILV == 0 && go) stage(which, sg, sbuf);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (ILV > 0) {
          if (go && kk * 4 + i == ILV) stage_one(which, sg, sbuf, 0);
          if (go && kk * 4 + i == ILV + 4) stage_one(which, sg, sbuf, 1);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
          ac[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][kk], af[i][kk], ac[i][j], 0, 0, 0);
        if constexpr (ILV > 0) __builtin_amdgcn_sched_barrier(0);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  for (int g = 0; g < total; ++g) {
    const int buf = g & 1;
    const char* hA0 = smem + buf * kBufBytes;
    const char* hA1 = hA0 + kHalfBytes;
    const char* hB0 = hA0 + 2 * kHalfBytes;
    const char* hB1 = hA0 + 3 * kHalfBytes;
    const bool n1 = g + 1 < total, n2 = g + 2 < total;
    // ---- phase 1: quadrant (0,0)
    // relax: the register epilogue's global stores of the previous tile (S per wave, younger
    // than the stages these two phases wait for) may stay in flight: vmcnt retires in issue order,
    // so the counts grow by S instead of draining the stores before the new tile's first MFMAs
    wait_vm((n1 ? 10 : 4) + relax);
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
    mma_phase(acc[0][0], b0, 1, g + 1, buf ^ 1, n1);
    // ---- phase 2: quadrant (0,1)
    wait_vm((n1 ? 10 : 2) + relax);
    relax = 0;
    raw_barrier();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b1[j][0] = *(const bf16x8*)(hB1 + (wn * 32 + j * 16) * 128 + frow + fsw0);
      b1[j][1] = *(const bf16x8*)(hB1 + (wn * 32 + j * 16) * 128 + frow + fsw1);
    }
    mma_phase(acc[0][1], b1, 0, g + 2, buf, n2);
    // ---- phase 3: quadrant (1,0)
    wait_vm(n2 ? 10 : (n1 ? 8 : 0));
    raw_barrier();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *(const bf16x8*)(hA1 + (wr * 64 + i * 16) * 128 + frow + fsw0);
      af[i][1] = *(const bf16x8*)(hA1 + (wr * 64 + i * 16) * 128 + frow + fsw1);
    }
    mma_phase(acc[1][0], b0, 2, g + 2, buf, n2);
    // ---- phase 4: quadrant (1,1), registers only (B1's last read was phase 2: a barrier ago)
    mma_phase(acc[1][1], b1, 3, g + 2, buf, n2);

    if (++kt < nk) continue;
    // ---- tile done: register epilogue (lane: rows m, 4 consecutive columns per fragment) --------
    epilogue();
    // a full tile's SwiGLU epilogue issued exactly 16 store instructions per wave (2 x 4 x 2)
    if constexpr (MODE == NOMIC_EPI_SWIGLU && !SK) relax = (m0c + 256 <= ep.M && n2) ? 16 : 0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    kt = 0;
    ++ti;
    m0c = m0x;
    n0c = n0x;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) { offAc[h][i] = offAx[h][i]; offBc[h][i] = offBx[h][i]; }
    if (ti + 1 < my_tiles) tile_offsets(ti + 1, offAx, offBx, m0x, n0x);
  }
  if constexpr (SK) {
    // the split tile: parts 1..p-1 hand over, part 0 collects and writes
    const int part = v % parts;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (part != 0) {
      // a thread's 32 float4 are contiguous: one address + immediate offsets
      float4* ws = ep.skws + (size_t)v * (256 * 256 / 4) + tid * 32;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const f32x4 c = acc[a][b][i][j];
              ws[((a * 2 + b) * 4 + i) * 2 + j] = make_float4(c[0], c[1], c[2], c[3]);
            }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {  // agent-scope release, then the flag (cdna guide §6 Guideline 16)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(ep.skflag + v, ep.skgen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (tid == 0) {
      for (int o = 1; o < parts; ++o)
        while (__hip_atomic_load(ep.skflag + v + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ep.skgen)
          __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int o = 1; o < parts; ++o) {
      const float4* ws = ep.skws + (size_t)(v + o) * (256 * 256 / 4) + tid * 32;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const float4 pp = ws[((a * 2 + b) * 4 + i) * 2 + j];
              acc[a][b][i][j] += f32x4{pp.x, pp.y, pp.z, pp.w};
            }
    }
    epilogue();
  }
}

int g_num_cus = 256;  // MI355X: 256 CUs in 8 XCDs; refreshed from the device on first use

// DMA interleave of the 256^2 kernels (k_gemm256 / k_gemm_p ILV): NOMIC_GEMM_ILV 0, 1 or 2
int g_ilv = -1;
int gemm_ilv() {
  if (g_ilv < 0) {
    const char* e = getenv("NOMIC_GEMM_ILV");
    g_ilv = e && *e ? atoi(e) : 0;
    if (g_ilv < 0 || g_ilv > 2) g_ilv = 0;
  }
  return g_ilv;
}

template <typename F>
void allow_lds(F* f, int bytes) {
  (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// register SwiGLU epilogue of the launch-per-tile 256^2 kernel (k_gemm256 EPI 1): NOMIC_SWIGLU_REG 1 / 0
int g_swiglu_reg = -1;
bool swiglu_reg_epi() {
  if (g_swiglu_reg < 0) {
    const char* e = getenv("NOMIC_SWIGLU_REG");
    g_swiglu_reg = e && *e ? (atoi(e) != 0) : 0;
  }
  return g_swiglu_reg != 0;
}

// main loop of the launch-per-tile 256^2 kernel (NOMIC_GEMM_PP): 2 = peeled lockstep with asm LDS-DMA
// (default), 1 = staggered ping-pong, 0 = the round-2 lockstep loop
int g_pp = -1;
int gemm_pp() {
  if (g_pp < 0) {
    const char* e = getenv("NOMIC_GEMM_PP");
    // default 2 (peeled lockstep loop, asm LDS-DMA): SwiGLU 296.5 -> 285.2 us, embed 9.35 -> 9.20 ms
    // (profiles/r3_gemm_asm_dma.md)
    g_pp = e && *e ? atoi(e) : 2;
    if (g_pp < 0 || g_pp > 2) g_pp = 2;
  }
  return g_pp;
}

// asm LDS-DMA in the 128^2 kernel (k_gemm_nt AS): NOMIC_GEMM_AS128 1 / 0
int g_as128 = -1;
int gemm_as128() {
  if (g_as128 < 0) {
    const char* e = getenv("NOMIC_GEMM_AS128");
    g_as128 = e && *e ? (atoi(e) != 0) : 0;
  }
  return g_as128;
}

int g_variant = -1;
int gemm_variant() {
  if (g_variant < 0) {
    const char* e = getenv("NOMIC_GEMM");
    g_variant = e ? atoi(e) : 0;  // 0 = auto
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

// stream-K hand-off buffers, one set per stream (two streams' GEMMs in flight at once must not
// share slots): cus slots of one 256x256 fp32 tile + flags; flags are compared with a per-launch
// generation, so they are never reset
struct SkWorkspace {
  float4* ws = nullptr;
  uint32_t* flag = nullptr;
  uint32_t gen = 0;
};
SkWorkspace* sk_workspace(hipStream_t s, int cus) {
  static std::mutex mu;
  static std::map<hipStream_t, SkWorkspace> table;
  std::lock_guard<std::mutex> g(mu);
  auto it = table.find(s);
  if (it != table.end()) return &it->second;
  SkWorkspace w;
  if (hipMalloc((void**)&w.ws, (size_t)cus * 256 * 256 * sizeof(float)) != hipSuccess) return nullptr;
  if (hipMalloc((void**)&w.flag, (size_t)cus * sizeof(uint32_t)) != hipSuccess ||
      hipMemset(w.flag, 0, (size_t)cus * sizeof(uint32_t)) != hipSuccess) {
    (void)hipFree(w.ws);
    return nullptr;
  }
  return &(table[s] = w);
}

template <int MODE>
int launch(const uint16_t* A, long lda, const uint16_t* W, long ldw, long M, int N, int K, EpiArgs ep,
           hipStream_t s) {
  if (K % BK || N % BN || M <= 0) return (int)hipErrorInvalidValue;
  const long mpad = (M + 255) / 256 * 256;
  // the 256^2 kernel runs 1 block/CU with a serial prologue/epilogue per tile: it wins only when
  // there are several waves of tiles (measured, profiles/r1_gemm_ab.jsonl); small grids use 128^2
  const bool fits = N % 256 == 0 && mpad * lda < (1L << 31) && (long)N * ldw < (1L << 31);
  const int var = gemm_variant();
  // auto: the persistent register-epilogue kernel when there are several waves of 256^2 tiles
  // (measured per shape: profiles/r1_gemm_persistent_ab.jsonl); fewer tiles: the 128^2 kernel
  const bool many = (mpad / 256) * (N / 256) >= 2048;
  // the statistics epilogue exists in the 128^2 kernel only (its 16-lane row groups); the 256^2
  // launch-per-tile kernel has the plain epilogues only
  constexpr bool p_ok = MODE <= NOMIC_EPI_F32;
  constexpr bool k256_ok = MODE <= NOMIC_EPI_F32;
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && n > 0)
      g_num_cus = n;
    return g_num_cus;
  }();
  const int nk = K / BK;
  const long tiles256 = fits ? (mpad / 256) * (N / 256) : 0;
  // stream-K persistent kernel when the 256^2 tiles do not divide evenly over the CUs (T = 32768:
  // N = 768 -> 384 tiles = 256 + 128, N = 2304 -> 1152 = 4 x 256 + 128): the r leftover tiles are
  // cut into p = cus / r K-ranges, one per block
  const long rem = tiles256 % cus;
  const long sk_parts = rem ? cus / rem : 0;
  const bool sk_ok = p_ok && fits && nk >= 2 && rem != 0 && cus % rem == 0 && sk_parts <= 8 && nk % sk_parts == 0;
  if (sk_ok && var == 514) {
    if constexpr (p_ok) {
      static bool attr_sk = [] {
        (void)hipFuncSetAttribute((const void*)k_gemm_p<MODE, true, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kBufBytes);
        return true;
      }();
      (void)attr_sk;
      SkWorkspace* w = sk_workspace(s, cus);
      if (!w) return (int)hipErrorOutOfMemory;
      ep.skws = w->ws;
      ep.skflag = w->flag;
      ep.skgen = ++w->gen;
      hipLaunchKernelGGL((k_gemm_p<MODE, true, true>), dim3(cus), dim3(kThreads2), 2 * kBufBytes, s, A, lda, W, ldw, K,
                         (int)(mpad / 256), N / 256, ep);
    }
    return (int)hipGetLastError();
  }
  // auto no longer takes the persistent kernel: on the encoder's SwiGLU shape (3072 tiles) the
  // launch-per-tile k_gemm256 measured 1064 TFLOP/s against 1015 (1046 with ILV 2) for k_gemm_p
  // (profiles/r3_gemm_ilv_ab.jsonl); NOMIC_GEMM=512 keeps it selectable
  if (p_ok && fits && K >= 2 * BK && (var == 512 || var == 513 || var == 515)) {
    static bool attr_p = [] {
      allow_lds(k_gemm_p<MODE, true, false, 0, true>, 2 * kBufBytes);
      allow_lds(k_gemm_p<MODE, true>, 2 * kBufBytes);
      allow_lds(k_gemm_p<MODE, true, false, 1>, 2 * kBufBytes);
      allow_lds(k_gemm_p<MODE, true, false, 2>, 2 * kBufBytes);
      allow_lds(k_gemm_p<MODE, false>, 2 * kBufBytes);
      return true;
    }();
    (void)attr_p;
    const int mtiles = (int)(mpad / 256), ntiles = N / 256;
    ep.gn = band_width(ntiles, 4);
    const int tiles = mtiles * ntiles;
    if constexpr (p_ok) {
      const dim3 g(tiles < cus ? tiles : cus), b(kThreads2);
      if (var == 513)
        hipLaunchKernelGGL((k_gemm_p<MODE, false>), dim3(tiles), b, 2 * kBufBytes, s, A, lda, W, ldw, K, mtiles, ntiles,
                           ep);
      else if (var == 515)  // persistent, asm LDS-DMA
        hipLaunchKernelGGL((k_gemm_p<MODE, true, false, 0, true>), g, b, 2 * kBufBytes, s, A, lda, W, ldw, K, mtiles,
                           ntiles, ep);
      else if (gemm_ilv() == 1)
        hipLaunchKernelGGL((k_gemm_p<MODE, true, false, 1>), g, b, 2 * kBufBytes, s, A, lda, W, ldw, K, mtiles, ntiles,
                           ep);
      else if (gemm_ilv() == 2)
        hipLaunchKernelGGL((k_gemm_p<MODE, true, false, 2>), g, b, 2 * kBufBytes, s, A, lda, W, ldw, K, mtiles, ntiles,
                           ep);
      else
        hipLaunchKernelGGL((k_gemm_p<MODE, true>), g, b, 2 * kBufBytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
    }
    return (int)hipGetLastError();
  }
  if (k256_ok && fits && (var == 256 || (var == 0 && (mpad / 256) * (N / 256) >= 2048))) {
    static bool attr = [] {
      allow_lds(k_gemm256<MODE>, kLds2Bytes);
      allow_lds(k_gemm256<MODE, 1>, kLds2Bytes);
      allow_lds(k_gemm256<MODE, 2>, kLds2Bytes);
      allow_lds(k_gemm256<MODE, 0, 0, 1>, kLds2Bytes);
      allow_lds(k_gemm256<MODE, 0, 0, 2>, kLds2Bytes);
      if constexpr (MODE == NOMIC_EPI_SWIGLU) {
        allow_lds(k_gemm256<MODE, 0, 1>, kLds2Bytes);
        allow_lds(k_gemm256<MODE, 0, 1, 1>, kLds2Bytes);
        allow_lds(k_gemm256<MODE, 0, 1, 2>, kLds2Bytes);
      }
      return true;
    }();
    (void)attr;
    const int mtiles = (int)(mpad / 256), ntiles = N / 256;
    ep.gn = band_width(ntiles, 4);
    if constexpr (k256_ok) {
      const dim3 g(mtiles * ntiles), b(kThreads2);
      if (gemm_pp() == 1 && gemm_ilv() == 0 && MODE == NOMIC_EPI_SWIGLU && swiglu_reg_epi())
        hipLaunchKernelGGL((k_gemm256<MODE, 0, 1, 1>), g, b, kLds2Bytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
      else if (gemm_pp() == 1 && gemm_ilv() == 0)
        hipLaunchKernelGGL((k_gemm256<MODE, 0, 0, 1>), g, b, kLds2Bytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
      else if (gemm_pp() == 2 && gemm_ilv() == 0 && MODE == NOMIC_EPI_SWIGLU && swiglu_reg_epi())
        hipLaunchKernelGGL((k_gemm256<MODE, 0, 1, 2>), g, b, kLds2Bytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
      else if (gemm_pp() == 2 && gemm_ilv() == 0)
        hipLaunchKernelGGL((k_gemm256<MODE, 0, 0, 2>), g, b, kLds2Bytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
      else if (MODE == NOMIC_EPI_SWIGLU && gemm_ilv() == 0 && swiglu_reg_epi())
        hipLaunchKernelGGL((k_gemm256<MODE, 0, 1>), g, b, kLds2Bytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
      else if (gemm_ilv() == 1)
        hipLaunchKernelGGL((k_gemm256<MODE, 1>), g, b, kLds2Bytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
      else if (gemm_ilv() == 2)
        hipLaunchKernelGGL((k_gemm256<MODE, 2>), g, b, kLds2Bytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
      else
        hipLaunchKernelGGL((k_gemm256<MODE>), g, b, kLds2Bytes, s, A, lda, W, ldw, K, mtiles, ntiles, ep);
    }
    return (int)hipGetLastError();
  }
  const int mtiles = (int)((M + BM - 1) / BM), ntiles = N / BN;
  ep.gn = band_width(ntiles, 8);
  constexpr int lds = kLdsBytes + (needs_rowstats(MODE) ? BM * 8 : 0);
  if (gemm_as128())
    hipLaunchKernelGGL((k_gemm_nt<MODE, true>), dim3(mtiles * ntiles), dim3(kThreads), lds, s, A, lda, W, ldw, K,
                       mtiles, ntiles, ep);
  else
    hipLaunchKernelGGL(k_gemm_nt<MODE>, dim3(mtiles * ntiles), dim3(kThreads), lds, s, A, lda, W, ldw, K, mtiles,
                       ntiles, ep);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int nomic_gemm_set_variant(int variant) {
  const int prev = gemm_variant();
  g_variant = variant;
  return prev;
}

// A/B knob: ping-pong main loop of the 256^2 kernel (1) or the 4-phase lockstep loop (0); returns the previous one
extern "C" int nomic_gemm_set_pp(int on) {
  const int prev = gemm_pp();
  g_pp = on < 0 || on > 2 ? 2 : on;
  return prev;
}

// A/B knob: asm LDS-DMA in the 128^2 kernel (1) or the builtin (0); returns the previous setting
extern "C" int nomic_gemm_set_as128(int on) {
  const int prev = gemm_as128();
  g_as128 = on ? 1 : 0;
  return prev;
}

// A/B knob: register SwiGLU epilogue of the 256^2 kernel (1) or the fp32 LDS image (0); returns the previous one
extern "C" int nomic_gemm_set_swiglu_reg(int on) {
  const int prev = swiglu_reg_epi() ? 1 : 0;
  g_swiglu_reg = on ? 1 : 0;
  return prev;
}

// A/B knob: DMA interleave of the 256^2 kernels (0, 1, 2); returns the previous setting
extern "C" int nomic_gemm_set_ilv(int ilv) {
  const int prev = gemm_ilv();
  g_ilv = ilv < 0 || ilv > 2 ? 0 : ilv;
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
