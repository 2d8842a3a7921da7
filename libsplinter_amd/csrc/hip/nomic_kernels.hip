// nomic_kernels.hip — the non-GEMM kernels of the Nomic-BERT encoder on
// gfx950 (K11, K14, K17 of SURVEY §2.10) plus GGUF dequantisation.
//
//   nomic_embed_ln   token gather + token-type row + LayerNorm       (K11)
//   nomic_layernorm  post-LN after each residual GEMM                (K15/K16 tail)
//   nomic_attention  varlen non-causal flash attention, head dim 64  (K14)
//   nomic_mean_pool  per-sequence mean -> fp32, optionally written
//                    straight into arena slots under the seqlock     (K17 + K9)
//   nomic_dequant    GGUF F32/F16/BF16/Q8_0/Q4_0/Q4_1/Q4_K/Q6_K -> bf16
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstdint>

#include "arena_dev.hpp"
#include "nomic_api.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int D = 768;

__device__ __forceinline__ float bf2f(uint32_t h16) { return __uint_as_float(h16 << 16); }
// fp32 -> bf16 (RNE) on the hardware converter: v_cvt_pk_bf16_f32, one instruction per pair (pk2)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ void unpack8(uint4 v, float* f) {
  f[0] = bf2f(v.x & 0xffff); f[1] = bf2f(v.x >> 16);
  f[2] = bf2f(v.y & 0xffff); f[3] = bf2f(v.y >> 16);
  f[4] = bf2f(v.z & 0xffff); f[5] = bf2f(v.z >> 16);
  f[6] = bf2f(v.w & 0xffff); f[7] = bf2f(v.w >> 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pk2(f[0], f[1]), pk2(f[2], f[3]),
                    pk2(f[4], f[5]), pk2(f[6], f[7]));
}

// ------------------------------------------------------------ LayerNorm --
// 32 lanes per row (half a wave), 24 elements = 3 x 16-B per lane; two-pass
// statistics from registers.  256-thread blocks = 8 rows.
template <bool EMBED>
__global__ __launch_bounds__(256) void k_ln(const uint16_t* __restrict__ x, const int32_t* __restrict__ ids, long T,
                                            const uint16_t* __restrict__ tok, const uint16_t* __restrict__ type_row,
                                            const uint16_t* __restrict__ g, const uint16_t* __restrict__ b, float eps,
                                            uint16_t* __restrict__ out) {
  const long row = blockIdx.x * 8L + (threadIdx.x >> 5);
  const int l = threadIdx.x & 31;
  if (row >= T) return;
  const uint16_t* src = EMBED ? tok + (long)ids[row] * D : x + row * D;
  float v[24];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = (c * 32 + l) * 8;
    unpack8(*(const uint4*)(src + col), v + 8 * c);
    if (EMBED) {
      float t[8];
      unpack8(*(const uint4*)(type_row + col), t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[8 * c + e] += t[e];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 24; ++e) s += v[e];
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
  const float mean = s * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 24; ++e) { const float d = v[e] - mean; q += d * d; }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) q += __shfl_xor(q, o, 32);
  const float rstd = rsqrtf(q * (1.f / D) + eps);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = (c * 32 + l) * 8;
    float gg[8], bb[8], o8[8];
    unpack8(*(const uint4*)(g + col), gg);
    unpack8(*(const uint4*)(b + col), bb);
#pragma unroll
    for (int e = 0; e < 8; ++e) o8[e] = (v[8 * c + e] - mean) * rstd * gg[e] + bb[e];
    *(uint4*)(out + row * D + col) = pack8(o8);
  }
}

// ------------------------------------------------------------ attention --
// One workgroup = 64 query rows of one (sequence, head); 4 waves x 16 rows.
// Per 64-key tile: S = Q K^T (8 x mfma 16x16x32), online softmax in fp32
// (exp2 with the scale folded in), P -> LDS (bf16) -> A operand, O += P V
// with V staged transposed in LDS so the B fragment is one 16-B read.
constexpr int AQ = 64, AK = 64, HD = 64;

// ---------------------------------------------------------- attention v2 --
// One workgroup = 128 query rows of one (sequence, head); 4 waves x 32 rows
// (two 16-row q-blocks per wave).  "Swapped" products keep every per-query
// quantity lane-local (guide §3 accumulator-as-operand, T10, T12):
//   S^T = K Q^T   : mfma_16x16x32(A = K rows [key][d], B = Q rows) -> lane
//                   holds keys 4g+r of each 16-key block for ONE query
//                   (col = lane & 15), so the row max / sum is 15 in-lane
//                   ops + 2 cross-group shuffles;
//   O^T += V^T P^T: the fp32 S^T accumulators, rounded to bf16, ARE the B
//                   operand (element j <-> key 4g+j / 16+4g+(j-4) of each
//                   32-key step); the matching V^T A operand comes from a
//                   row-major V image via two ds_read_b64_tr_b16 (hardware
//                   transpose) with a chunk swizzle that keeps each
//                   32-lane half's 8 rows x 32 B on distinct banks.
// K/V tiles (64 keys) are register-staged one tile ahead: global loads for
// tile t+1 issue before tile t's math, the LDS write lands after it (T14),
// one barrier per tile, double-buffered LDS (32 KB).
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ int ksw(int key, int c) { return c ^ (key & 7); }
__device__ __forceinline__ int vsw(int key, int c) { return c ^ (((key >> 1) & 3) << 1); }

// W = minimum waves per SIMD the register allocation must allow (0: unconstrained, 236 VGPRs ->
// 2 waves/SIMD; 3: 168 VGPRs, 3 waves/SIMD, 12 waves per CU to hide the softmax/LDS latency)
// XR: 1-D grid of nqb*heads blocks through the bijective XCD remap (guide §5 T1), so the q-blocks
// of one (sequence, head) -- which all stream the same K/V -- run on ONE XCD and share its L2
// (with the 2-D grid consecutive q-blocks are dealt round-robin to 4 different XCDs and every
// K/V tile is fetched from the fabric once per q-block).
// Cross-lane reductions over the 4 lane groups g = lane >> 4 (a value of query column li sits in
// lanes li, li+16, li+32, li+48): v_permlane16_swap / v_permlane32_swap (gfx950 VALU half-row
// exchanges) instead of two ds_bpermute round trips through the LDS pipe per reduction.  With
// vdst = src = x the swap returns the partner's value in one of its two results and x in the other.
__device__ __forceinline__ float xg_max(float x) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
__device__ __forceinline__ float xg_sum(float x) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
typedef float f32x2 __attribute__((ext_vector_type(2)));

// OPT: permlane reductions, packed (v_pk_fma/v_pk_add) score scaling and row sums, and K/V
// source pointers advanced per tile instead of recomputed with 64-bit multiplies.
// CAUSAL: query row i of a sequence sees keys 0..i (the completion daemon's prefill, K18); key
// tiles past the block's last row are skipped, the diagonal tiles masked per score.  kv_heads <
// heads: grouped-query attention, q head h reads kv head h / (heads / kv_heads); the qkv rows are
// [q (heads) | k (kv_heads) | v (kv_heads)] x HD.
// LATE: the next tile's K/V global loads are issued after this tile's S^T = K Q^T MFMAs instead of
// before them (the split async stage of cdna_hip_programming.md T14: the loads' issue no longer sits
// between the barrier and the first MFMA, and their registers are live for half the tile).
template <int W, bool XR = false, bool OPT = false, bool CAUSAL = false, int KT = 64, int QW = 4, bool LATE = false>
__global__ __launch_bounds__(64 * QW) __attribute__((amdgpu_waves_per_eu(W > 0 ? W : 1))) void k_attn2(
    const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out,
                                               const int32_t* __restrict__ cu, const int32_t* __restrict__ qblocks,
                                               int heads, float scale_log2, int kv_heads) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][KT * 128];  // [buf][K | V][key * 128 B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  int qbi = blockIdx.x, head = blockIdx.y;
  if constexpr (XR) {
    const int nwg = gridDim.x, orig = blockIdx.x, q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int nqb = nwg / heads;
    head = lid / nqb;
    qbi = lid - head * nqb;
  }
  const int seq = qblocks[2 * qbi], qstart = qblocks[2 * qbi + 1];
  const long s0 = cu[seq], len = cu[seq + 1] - s0;
  const long ld = (long)(heads + 2 * kv_heads) * HD;
  const int kvhead = head / (heads / kv_heads);
  const uint16_t* Qg = qkv + head * HD;
  const uint16_t* Kg = qkv + (long)heads * HD + kvhead * HD;
  const uint16_t* Vg = qkv + (long)(heads + kv_heads) * HD + kvhead * HD;

  // Q^T B-fragments: query row qstart + wave*32 + qb*16 + li, d = kk*32 + 8g .. +7
  bf16x8 qf[2][2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const long qrow = qstart + wave * 32 + qb * 16 + li;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      qf[qb][kk] = qrow < len ? *(const bf16x8*)(Qg + (s0 + qrow) * ld + kk * 32 + g * 8) : bf16x8{};
  }
  f32x4 o[4][2];  // O^T[d = db*16 + 4g + r][q = qb*16 + li]
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) o[db][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-1e30f, -1e30f}, l[2] = {0.f, 0.f};

  // QW waves: the block covers 32 * QW query rows; NT threads stage a K/V tile in NL rounds of
  // NT / 8 keys (8 16-B chunks per 128-B key row)
  constexpr int NT = 64 * QW, NL = KT * 8 / NT, KS = KT == 128 ? 7 : 6;  // KS = log2 KT
  static_assert(KT == 64 || KT == 128, "key tile");
  static_assert(QW == 4 || QW == 8, "waves per block");
  uint4 rk[NL], rv[NL];
  // OPT: per-lane K/V source pointers of tile 0, advanced by KT rows per tile
  // (lane load `it` sits NT / 8 keys after load 0: a wave-uniform offset, so one pointer pair per lane)
  const uint16_t* kp = Kg + (s0 + (tid >> 3)) * ld + (tid & 7) * 8;
  const uint16_t* vp = Vg + (s0 + (tid >> 3)) * ld + (tid & 7) * 8;
  const long tstride = KT * ld;
  auto gload = [&](long k0) {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int c = tid + it * NT, key = c >> 3, ch = c & 7;
      if (k0 + key < len) {
        if constexpr (OPT) {
          const long off = (k0 >> KS) * tstride + it * (NT / 8) * ld;
          rk[it] = *(const uint4*)(kp + off);
          rv[it] = *(const uint4*)(vp + off);
        } else {
          rk[it] = *(const uint4*)(Kg + (s0 + k0 + key) * ld + ch * 8);
          rv[it] = *(const uint4*)(Vg + (s0 + k0 + key) * ld + ch * 8);
        }
      } else {
        rk[it] = make_uint4(0, 0, 0, 0);
        rv[it] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lwrite = [&](int buf) {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int c = tid + it * NT, key = c >> 3, ch = c & 7;
      *(uint4*)(lds[buf][0] + key * 128 + (ksw(key, ch) << 4)) = rk[it];
      *(uint4*)(lds[buf][1] + key * 128 + (vsw(key, ch) << 4)) = rv[it];
    }
  };

  int ntiles = (int)((len + KT - 1) / KT);
  if constexpr (CAUSAL) ntiles = min(ntiles, (int)((qstart + 32 * QW + KT - 1) / KT));
  gload(0);
  lwrite(0);
  __syncthreads();
  const int tq = li >> 2, tp = li & 3;  // tr-read: this lane addresses row tq, columns 4*tp..4*tp+3
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const long k0 = (long)t * KT;
    if (!LATE && t + 1 < ntiles) gload(k0 + KT);
    const char* Ks = lds[buf][0];
    const char* Vs = lds[buf][1];
    // ---- S^T = K Q^T
    f32x4 s[KT / 16][2];
#pragma unroll
    for (int kb = 0; kb < KT / 16; ++kb) {
      const int row = kb * 16 + li;
      bf16x8 kf[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) kf[kk] = *(const bf16x8*)(Ks + row * 128 + (ksw(row, kk * 4 + g) << 4));
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        s[kb][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          s[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kk], qf[qb][kk], s[kb][qb], 0, 0, 0);
      }
    }
    if (LATE && t + 1 < ntiles) gload(k0 + KT);
    // ---- online softmax, one query per lane column.  Max on the raw scores (scale > 0), one
    // FMA per score into the exp2 domain, raw v_exp_f32 (no denormal fix-up: p underflows to 0),
    // key mask only on the sequence's partial last tile, and the deferred rescale of T13
    // (cdna_hip_programming.md §5.5): the running max moves only when some query's tile max
    // exceeds it by more than kThr, so P <= 2^kThr and the O/l rescale is skipped on most tiles
    // (decided before this tile's P V, after the previous tile's: the textbook order).
    constexpr float kThr = 8.f;
    const bool full = k0 + KT <= len;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      if constexpr (CAUSAL) {
        if (k0 + KT - 1 > qstart) {  // a diagonal tile: keys after the query are masked
          const long qrow = qstart + wave * 32 + qb * 16 + li;
#pragma unroll
          for (int kb = 0; kb < KT / 16; ++kb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (k0 + kb * 16 + 4 * g + r > qrow) s[kb][qb][r] = -1e30f;
        }
      }
      if (!full) {
#pragma unroll
        for (int kb = 0; kb < KT / 16; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (k0 + kb * 16 + 4 * g + r >= len) s[kb][qb][r] = -1e30f;
      }
      float mx = -1e30f;
#pragma unroll
      for (int kb = 0; kb < KT / 16; ++kb) mx = fmaxf(fmaxf(mx, fmaxf(s[kb][qb][0], s[kb][qb][1])), fmaxf(s[kb][qb][2], s[kb][qb][3]));
      if constexpr (OPT) {
        mx = xg_max(mx);
      } else {
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      }
      const float mxs = mx * scale_log2;
      if (!__all(mxs - m[qb] <= kThr)) {  // wave-uniform: rescale O and l once to the new max
        const float mn = fmaxf(m[qb], mxs);
        const float alpha = __builtin_amdgcn_exp2f(m[qb] - mn);
        m[qb] = mn;
        l[qb] *= alpha;
#pragma unroll
        for (int db = 0; db < 4; ++db) o[db][qb] *= alpha;
      }
      const float nm = -m[qb];
      float ps = 0.f;
      if constexpr (OPT) {
        const f32x2 sc2 = {scale_log2, scale_log2}, nm2 = {nm, nm};
        f32x2 acc2 = {0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < KT / 16; ++kb)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            f32x2 x = {s[kb][qb][2 * h], s[kb][qb][2 * h + 1]};
            x = x * sc2 + nm2;  // v_pk_fma_f32
            x.x = __builtin_amdgcn_exp2f(x.x);
            x.y = __builtin_amdgcn_exp2f(x.y);
            s[kb][qb][2 * h] = x.x;
            s[kb][qb][2 * h + 1] = x.y;
            acc2 += x;  // v_pk_add_f32
          }
        ps = xg_sum(acc2.x + acc2.y);
      } else {
#pragma unroll
        for (int kb = 0; kb < KT / 16; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[kb][qb][r], scale_log2, nm));
            s[kb][qb][r] = p;
            ps += p;
          }
        ps += __shfl_xor(ps, 16, 64);
        ps += __shfl_xor(ps, 32, 64);
      }
      l[qb] += ps;
    }
    // ---- O^T += V^T P^T, two 32-key steps
#pragma unroll
    for (int st = 0; st < KT / 32; ++st) {
      bf16x8 pf[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[qb][j] = (__bf16)s[2 * st][qb][j];
          pf[qb][4 + j] = (__bf16)s[2 * st + 1][qb][j];
        }
      const int row1 = st * 32 + 4 * g + tq, row2 = row1 + 16;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int ch = db * 2 + (tp >> 1);
        const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_v4i16*)(Vs + row1 * 128 + (vsw(row1, ch) << 4) + 8 * (tp & 1)));
        const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_v4i16*)(Vs + row2 * 128 + (vsw(row2, ch) << 4) + 8 * (tp & 1)));
        const v8i16 ab = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
        const bf16x8 vf = __builtin_bit_cast(bf16x8, ab);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qb], o[db][qb], 0, 0, 0);
      }
    }
    if (t + 1 < ntiles) lwrite(buf ^ 1);
    __syncthreads();
  }
  // ---- normalise, store 4 consecutive d per lane
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const long q = qstart + wave * 32 + qb * 16 + li;
    if (q >= len) continue;
    const float inv = 1.f / l[qb];
    uint16_t* dst = out + (s0 + q) * (long)heads * HD + head * HD + 4 * g;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      uint2 w;
      w.x = pk2(o[db][qb][0] * inv, o[db][qb][1] * inv);
      w.y = pk2(o[db][qb][2] * inv, o[db][qb][3] * inv);
      *(uint2*)(dst + db * 16) = w;
    }
  }
}

// ------------------------------------------------- attention, 32x32 MFMA form --
// k_attn3: the encoder's varlen attention (hd 64, non-causal) on v_mfma_f32_32x32x16_bf16.  One
// 256-thread workgroup = 128 query rows of one (sequence, head), 4 waves x 32 rows; per 64-key tile:
//   S^T = K Q^T   two 32-key blocks x four 16-d steps = 8 MFMAs.  With the 32x32 C layout a lane
//                 holds, for its query q = lane & 31, the keys crow(r, hi) = (r&3) + 8(r>>2) + 4hi of
//                 each block (hi = lane >> 5): 32 scores, so the row max / sum are 31 in-lane ops
//                 and ONE permlane32 swap (the 16x16 form needs two swaps per 16-row block);
//   O^T += V^T P^T the MFMA's k index is mapped to keys in the order the lane already holds them:
//                 k-slot j of half hi <-> key 16s + (j&3) + 8(j>>2) + 4hi, so the bf16 P fragment
//                 of step s is the lane's own s[8s .. 8s+7] (no permute), and the matching V^T
//                 fragment is two ds_read_b64_tr_b16 of 4 consecutive key rows (4hi and 8+4hi).
// LDS images (64 keys x 128 B, double-buffered, register-staged one tile ahead as in k_attn2):
//   K chunks XOR (key >> 1) & 7: each 16-lane b128 group (16 distinct rows, one chunk) covers all
//   16 bank quads; V chunks XOR ((key >> 1) & 1) << 2: the four rows a 32-lane transposing read
//   touches land on four different 64-B quarters of the bank space.
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int k3sw(int key, int c) { return c ^ ((key >> 1) & 7); }
__device__ __forceinline__ int v3sw(int key, int c) { return c ^ (((key >> 1) & 1) << 2); }

// PF2: K/V global loads issued two tiles ahead (two register stages) instead of one, so a tile's
// loads have two tiles' compute to land before their LDS write.
// (Measured in round 6 and not kept: the next tile's K/V loads issued after the QK^T MFMAs, and
// s_setprio 1 over the MFMA runs -- alone and together within +-1.5 % of this form in isolation and
// 0.1 % in the encoder, profiles/r6/README.md.  Also measured then and not kept: the two S^T chains
// interleaved with four-way partial max / sum chains (neutral), and no row max after the first tile
// with an overflow-guarded exact path (-2 % in isolation, neutral in the encoder), attn_forms2_ab; and
// W = 4, four waves per SIMD at <= 128 VGPRs with 13 spilled: 105 vs 84 us per layer.)
template <bool PF2 = false, int W = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void k_attn3(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ out,
                                               const int32_t* __restrict__ cu, const int32_t* __restrict__ qblocks,
                                               int heads, float scale_log2) {
  constexpr int KT = 64, NT = 256, NL = KT * 8 / NT;
  __shared__ __attribute__((aligned(16))) char lds[2][2][KT * 128];  // [buf][K | V][key * 128 B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hi = lane >> 5, q32 = lane & 31, li = lane & 15, tq = li >> 2, tp = li & 3;
  // bijective XCD remap (the q-blocks of one (sequence, head) share an XCD's L2)
  const int nwg = gridDim.x, orig = blockIdx.x, q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int nqb = nwg / heads, head = lid / nqb, qbi = lid - head * nqb;
  const int seq = qblocks[2 * qbi], qstart = qblocks[2 * qbi + 1];
  const long s0 = cu[seq], len = cu[seq + 1] - s0;
  const long ld = 3L * heads * HD;
  const uint16_t* Qg = qkv + head * HD;
  const uint16_t* Kg = qkv + (long)heads * HD + head * HD;
  const uint16_t* Vg = qkv + 2L * heads * HD + head * HD;

  const long qrow = qstart + wave * 32 + q32;
  bf16x8 qf[4];  // B operand: Q[q][16 ks + 8 hi .. +7]
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    qf[ks] = qrow < len ? *(const bf16x8*)(Qg + (s0 + qrow) * ld + ks * 16 + hi * 8) : bf16x8{};
  f32x16 o[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m = -1e30f, l = 0.f;

  constexpr int NS = PF2 ? 2 : 1;  // register stages
  uint4 rk[NS][NL], rv[NS][NL];
  auto gload = [&](int stg, long k0) {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int c = tid + it * NT, key = c >> 3, ch = c & 7;
      if (k0 + key < len) {
        rk[stg][it] = *(const uint4*)(Kg + (s0 + k0 + key) * ld + ch * 8);
        rv[stg][it] = *(const uint4*)(Vg + (s0 + k0 + key) * ld + ch * 8);
      } else {
        rk[stg][it] = make_uint4(0, 0, 0, 0);
        rv[stg][it] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lwrite = [&](int stg, int buf) {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int c = tid + it * NT, key = c >> 3, ch = c & 7;
      *(uint4*)(lds[buf][0] + key * 128 + (k3sw(key, ch) << 4)) = rk[stg][it];
      *(uint4*)(lds[buf][1] + key * 128 + (v3sw(key, ch) << 4)) = rv[stg][it];
    }
  };

  const int ntiles = (int)((len + KT - 1) / KT);
  gload(0, 0);
  lwrite(0, 0);
  if (PF2 && ntiles > 1) gload(1 % NS, KT);  // tile 1 rides one stage ahead of the loop's loads
  __syncthreads();
  auto tile = [&](int t, const int sl, const int snext) {
    const int buf = t & 1;
    const long k0 = (long)t * KT;
    // sl: the stage this tile's loads go to; snext: the stage holding tile t+1 (PF2: t's
    // stage parity is a compile-time constant of each unrolled call, so the register stages
    // are never indexed at run time)
    if (PF2) {
      if (t + 2 < ntiles) gload(sl, k0 + 2 * KT);
    } else if (t + 1 < ntiles) {
      gload(0, k0 + KT);
    }
    const char* Ks = lds[buf][0];
    const char* Vs = lds[buf][1];
    // ---- S^T = K Q^T: A = K rows (key kb*32 + q32, d 16 ks + 8 hi), B = Q^T
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
      const int row = kb * 32 + q32;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 kf = *(const bf16x8*)(Ks + row * 128 + (k3sw(row, 2 * ks + hi) << 4));
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[kb], 0, 0, 0);
      }
    }

    // ---- online softmax of query q32 over the tile's 64 keys (32 here, 32 in lane ^ 32)
    if (k0 + KT > len) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (k0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi >= len) s[kb][r] = -1e30f;
    }
    float mx = fmaxf(s[0][0], s[1][0]);
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));
    {
      auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
    }
    constexpr float kThr = 8.f;
    const float mxs = mx * scale_log2;
    if (!__all(mxs - m <= kThr)) {  // wave-uniform deferred rescale (as k_attn2)
      const float mn = fmaxf(m, mxs);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int db = 0; db < 2; ++db) o[db] *= alpha;
    }
    const float nm = -m;
    float ps = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[kb][r], scale_log2, nm));
        s[kb][r] = p;
        ps += p;
      }
    {
      auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(ps), __float_as_uint(ps), false, false);
      ps = __uint_as_float(q[0]) + __uint_as_float(q[1]);
    }
    l += ps;
    // ---- O^T += V^T P^T, four 16-key steps
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (__bf16)s[kb][8 * st + j];
        const int rowA = kb * 32 + 16 * st + 4 * hi + tq, rowB = rowA + 8;
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const int col = 32 * db + 16 * ((lane >> 4) & 1) + 4 * tp;
          const int ch = col >> 3, off = (col & 7) * 2;
          const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4i16*)(Vs + rowA * 128 + (v3sw(rowA, ch) << 4) + off));
          const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4i16*)(Vs + rowB * 128 + (v3sw(rowB, ch) << 4) + off));
          const bf16x8 vf = __builtin_bit_cast(bf16x8, (v8i16)__builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[db], 0, 0, 0);
        }
      }
    if (t + 1 < ntiles) lwrite(snext, buf ^ 1);
    __syncthreads();
  };
  if constexpr (PF2) {
    for (int t = 0; t < ntiles; t += 2) {
      tile(t, 0, 1);
      if (t + 1 < ntiles) tile(t + 1, 1, 0);
    }
  } else {
    for (int t = 0; t < ntiles; ++t) tile(t, 0, 0);
  }
  // ---- normalise; lane holds d = 32 db + 8 g + 4 hi + 0..3 (g = r >> 2) of query q32
  if (qrow < len) {
    const float inv = 1.f / l;
    uint16_t* dst = out + (s0 + qrow) * (long)heads * HD + head * HD;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 w;
        w.x = pk2(o[db][4 * g] * inv, o[db][4 * g + 1] * inv);
        w.y = pk2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv);
        *(uint2*)(dst + 32 * db + 8 * g + 4 * hi) = w;
      }
  }
}

// ------------------------------------------------------------ mean pool --
// One block per document of 16 waves (a document's rows in flight across 16 waves x 4 unrolled
// rows: with 4 waves the 64 blocks of a 64-document batch waited on one row load at a time, 45 us)
constexpr int kPoolWaves = 16, kPoolThreads = 64 * kPoolWaves;
__global__ __launch_bounds__(kPoolThreads) void k_pool(const uint16_t* __restrict__ x, const int32_t* __restrict__ cu,
                                              float* __restrict__ pooled, int normalize, spl_arena_t aa,
                                              const int64_t* __restrict__ slots, const uint64_t* __restrict__ hashes,
                                              int32_t* __restrict__ status) {
  __shared__ float part[kPoolWaves][D];
  __shared__ float vec[D];
  __shared__ float red[kPoolWaves];
  __shared__ int lock_ok;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long t0 = cu[b], t1 = cu[b + 1];
  float acc[12];
#pragma unroll
  for (int e = 0; e < 12; ++e) acc[e] = 0.f;
  // lane covers columns [lane*8, +8) and [512 + lane*4, +4)
#pragma unroll 4
  for (long t = t0 + wave; t < t1; t += kPoolWaves) {
    const uint16_t* row = x + t * D;
    float f[8];
    unpack8(*(const uint4*)(row + lane * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += f[e];
    const uint2 h = *(const uint2*)(row + 512 + lane * 4);
    acc[8] += bf2f(h.x & 0xffff); acc[9] += bf2f(h.x >> 16);
    acc[10] += bf2f(h.y & 0xffff); acc[11] += bf2f(h.y >> 16);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[wave][lane * 8 + e] = acc[e];
#pragma unroll
  for (int e = 0; e < 4; ++e) part[wave][512 + lane * 4 + e] = acc[8 + e];
  __syncthreads();
  const float inv = t1 > t0 ? 1.f / (float)(t1 - t0) : 0.f;
  float ss = 0.f;
  for (int c = tid; c < D; c += kPoolThreads) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < kPoolWaves; ++w) v += part[w][c];
    v *= inv;
    vec[c] = v;
    ss += v * v;
  }
  if (normalize) {
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
    if (lane == 0) red[wave] = ss;
  }
  __syncthreads();
  float rs = 0.f;
  if (normalize)
#pragma unroll
    for (int w = 0; w < kPoolWaves; ++w) rs += red[w];
  const float scale = normalize ? rsqrtf(fmaxf(rs, 1e-24f)) : 1.f;
  if (pooled)
    for (int c = tid; c < D; c += kPoolThreads) pooled[(long)b * D + c] = vec[c] * scale;
  if (!slots) return;
  // fused write-back into the arena slot (seqlock), reference set_embedding
  // semantics (/root/reference/splinter.c:567-588): CAS even->odd, copy, +1.
  using namespace spl;
  using namespace spl::dev;
  Arena a = spl::dev::from_api(aa);
  const int64_t si = slots[b];
  if (tid == 0) {
    int ok = 0;
    if (si >= 0 && a.stride == kSlotEmbedBytes) {
      uint8_t* s = a.slot((size_t)si);
      const uint64_t e = slot_epoch(s);
      if (!(e & 1) && acas64(epoch_ptr(s), e, e + 1)) {
        if (slot_hash(s) == hashes[b]) ok = 1;
        else { aadd64(epoch_ptr(s), 1); ok = -2; }
      } else {
        ok = -11;
      }
    } else {
      ok = -2;
    }
    lock_ok = ok;
  }
  __syncthreads();
  if (lock_ok == 1) {
    float* dst = (float*)(a.slot((size_t)si) + kOffEmbed);
    for (int c = tid; c < D; c += kPoolThreads) dst[c] = vec[c] * scale;
    if (a.has_vec16() && wave == 0) {  // the bf16 copy + squared norm (wave 0, the wave layout of write_vec16_wave)
      float4 v[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float* p = vec + 4 * (lane + 64 * c);
        v[c] = make_float4(p[0] * scale, p[1] * scale, p[2] * scale, p[3] * scale);
      }
      write_vec16_wave(a, (size_t)si, v, lane);
    }
    release();
    __syncthreads();
    if (tid == 0) {
      aadd64(epoch_ptr(a.slot((size_t)si)), 1);
      aadd64(&a.hdr()->epoch, 1);
      mark_dirty(a, (size_t)si);
      notify_host(a);
    }
  }
  if (tid == 0 && status) status[b] = lock_ok == 1 ? 0 : lock_ok;
}

// ------------------------------------------------------------ dequant ----
__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

// one thread per 32-element block (legacy quants) / per 32 elements of a k-quant superblock
__global__ void k_dequant(int type, const uint8_t* __restrict__ src, long nblk, uint16_t* __restrict__ dst) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nblk; i += (long)gridDim.x * blockDim.x) {
    float y[32];
    if (type == 8) {  // Q8_0: f16 d, int8 q[32]
      const uint8_t* p = src + i * 34;
      const float d = h2f(*(const uint16_t*)p);
#pragma unroll
      for (int e = 0; e < 32; ++e) y[e] = d * (float)(int8_t)p[2 + e];
    } else if (type == 2) {  // Q4_0: f16 d, 16 B nibbles (low -> 0..15, high -> 16..31)
      const uint8_t* p = src + i * 18;
      const float d = h2f(*(const uint16_t*)p);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        y[e] = d * (float)((int)(p[2 + e] & 15) - 8);
        y[e + 16] = d * (float)((int)(p[2 + e] >> 4) - 8);
      }
    } else if (type == 3) {  // Q4_1: f16 d, f16 m, nibbles
      const uint8_t* p = src + i * 20;
      const float d = h2f(*(const uint16_t*)p), mn = h2f(*(const uint16_t*)(p + 2));
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        y[e] = d * (float)(p[4 + e] & 15) + mn;
        y[e + 16] = d * (float)(p[4 + e] >> 4) + mn;
      }
    } else if (type == 12) {  // Q4_K: 256-element superblocks of 144 B, 8 sub-blocks of 32
      const long sb = i >> 3;
      const int j = (int)(i & 7);
      const uint8_t* p = src + sb * 144;
      const float d = h2f(*(const uint16_t*)p), dmin = h2f(*(const uint16_t*)(p + 2));
      const uint8_t* sc = p + 4;
      int s, mq;
      if (j < 4) { s = sc[j] & 63; mq = sc[j + 4] & 63; }
      else { s = (sc[j + 4] & 15) | ((sc[j - 4] >> 6) << 4); mq = (sc[j + 4] >> 4) | ((sc[j] >> 6) << 4); }
      const uint8_t* q = p + 16 + (j >> 1) * 32;
      const float dl = d * (float)s, ml = dmin * (float)mq;
#pragma unroll
      for (int e = 0; e < 32; ++e) y[e] = dl * (float)((j & 1) ? (q[e] >> 4) : (q[e] & 15)) - ml;
    } else if (type == 14) {  // Q6_K: 210-B superblocks: ql[128] qh[64] scales[16] d
      const long sb = i >> 3;
      const int j = (int)(i & 7);  // 32-element group: half = j/4, quarter = j%4
      const uint8_t* p = src + sb * 210;
      const uint8_t* ql = p + (j >> 2) * 64;
      const uint8_t* qh = p + 128 + (j >> 2) * 32;
      const int8_t* scl = (const int8_t*)(p + 192) + (j >> 2) * 8;
      const float d = h2f(*(const uint16_t*)(p + 208));
      const int qd = j & 3;
#pragma unroll
      for (int e = 0; e < 32; ++e) {
        const int byte = ql[e + 32 * (qd & 1)];
        const int low = (qd >= 2) ? (byte >> 4) : (byte & 15);
        const int hi = (qh[e] >> (2 * qd)) & 3;
        const int q = (low | (hi << 4)) - 32;
        y[e] = d * (float)scl[(e >> 4) + 2 * qd] * (float)q;
      }
    } else {
      for (int e = 0; e < 32; ++e) y[e] = 0.f;
    }
    uint4* o = (uint4*)(dst + i * 32);
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = pack8(y + 8 * c);
  }
}

// plain formats: one thread per 8 elements
__global__ void k_convert(int type, const uint8_t* __restrict__ src, long n8, uint16_t* __restrict__ dst) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float y[8];
    if (type == 0) {  // F32
      const float4 a = ((const float4*)src)[2 * i], b = ((const float4*)src)[2 * i + 1];
      y[0] = a.x; y[1] = a.y; y[2] = a.z; y[3] = a.w; y[4] = b.x; y[5] = b.y; y[6] = b.z; y[7] = b.w;
    } else if (type == 1) {  // F16
      const uint4 v = ((const uint4*)src)[i];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) { y[2 * e] = h2f((uint16_t)(w[e] & 0xffff)); y[2 * e + 1] = h2f((uint16_t)(w[e] >> 16)); }
    } else {  // BF16 (30)
      ((uint4*)dst)[i] = ((const uint4*)src)[i];
      continue;
    }
    ((uint4*)dst)[i] = pack8(y);
  }
}

inline int grid_of(long n, int per) {
  long g = (n + per - 1) / per;
  return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace

extern "C" {

int nomic_embed_ln(const int32_t* ids, long T, const void* tok, const void* type_row, const void* gamma,
                   const void* beta, float eps, void* out, hipStream_t s) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(k_ln<true>, dim3((unsigned)((T + 7) / 8)), dim3(256), 0, s, nullptr, ids, T,
                     (const uint16_t*)tok, (const uint16_t*)type_row, (const uint16_t*)gamma, (const uint16_t*)beta,
                     eps, (uint16_t*)out);
  return (int)hipGetLastError();
}

int nomic_layernorm(const void* x, long T, const void* gamma, const void* beta, float eps, void* out, hipStream_t s) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(k_ln<false>, dim3((unsigned)((T + 7) / 8)), dim3(256), 0, s, (const uint16_t*)x, nullptr, T,
                     nullptr, nullptr, (const uint16_t*)gamma, (const uint16_t*)beta, eps, (uint16_t*)out);
  return (int)hipGetLastError();
}

// Two selectable forms (NOMIC_ATTN): 13 = k_attn3 (32x32x16 MFMA, default: 634 vs 514 TFLOP/s for
// 6, profiles/r3_attn_k_attn3_ab.jsonl) and 6 = k_attn2 (16x16x32 MFMA, permlane reductions, packed
// score math), the fallback.  Measured and removed in round 4: K/V staged by LDS-DMA into a 3-deep
// ring (505 vs 596 TFLOP/s, profiles/r4k/attn_bench.out).  The other A/B forms of rounds 1-3 are gone; their measurements stay in
// profiles/r1_attn_* .. r3_attn_*.
static int attn_norm(int v) { return v == 6 ? 6 : 13; }
static int g_attn_variant = [] {
  const char* e = getenv("NOMIC_ATTN");
  return attn_norm(e && *e ? atoi(e) : 13);
}();

int nomic_attention_set_variant(int v) {
  const int prev = g_attn_variant;
  g_attn_variant = attn_norm(v);
  return prev;
}

int nomic_attention(const void* qkv, void* out, const int32_t* cu, const int32_t* qblocks, int nqb, int heads,
                    float scale, hipStream_t s) {
  if (nqb <= 0) return 0;
  if (heads * HD * 3 % 8) return (int)hipErrorInvalidValue;
  const float scale_log2 = scale * 1.4426950408889634f;
  if (g_attn_variant == 6)
    hipLaunchKernelGGL((k_attn2<0, true, true>), dim3(nqb * heads), dim3(256), 0, s, (const uint16_t*)qkv,
                       (uint16_t*)out, cu, qblocks, heads, scale_log2, heads);
  else
    hipLaunchKernelGGL(k_attn3<false>, dim3(nqb * heads), dim3(256), 0, s, (const uint16_t*)qkv, (uint16_t*)out, cu,
                       qblocks, heads, scale_log2);
  return (int)hipGetLastError();
}

// causal (prefill) attention of the completion daemon's decoder: qkv rows [q (heads) | k | v
// (kv_heads each)] x 64, out [T, heads * 64]; 128-row q-blocks as nomic_attention
int dec_attn_prefill(const void* qkv, void* out, const int32_t* cu, const int32_t* qblocks, int nqb, int heads,
                     int kv_heads, float scale, hipStream_t s) {
  if (nqb <= 0) return 0;
  if (kv_heads <= 0 || heads % kv_heads || (heads + 2 * kv_heads) * HD % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((k_attn2<0, true, true, true>), dim3(nqb * heads), dim3(256), 0, s, (const uint16_t*)qkv,
                     (uint16_t*)out, cu, qblocks, heads, scale * 1.4426950408889634f, kv_heads);
  return (int)hipGetLastError();
}

int nomic_mean_pool(const void* x, const int32_t* cu, int B, float* pooled, int normalize, spl_arena_t arena,
                    const int64_t* slots, const uint64_t* hashes, int32_t* status, hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_pool, dim3(B), dim3(kPoolThreads), 0, s, (const uint16_t*)x, cu, pooled, normalize, arena, slots,
                     hashes, status);
  return (int)hipGetLastError();
}

int nomic_dequant(int type, const void* src, long n, void* dst, hipStream_t s) {
  if (n <= 0) return 0;
  if (type == 0 || type == 1 || type == 30) {
    if (n % 8) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_convert, dim3(grid_of(n / 8, 256)), dim3(256), 0, s, type, (const uint8_t*)src, n / 8,
                       (uint16_t*)dst);
  } else {
    if (n % 32 || ((type == 12 || type == 14) && n % 256)) return (int)hipErrorInvalidValue;  // K-quants: 256
    if (type != 2 && type != 3 && type != 8 && type != 12 && type != 14) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_dequant, dim3(grid_of(n / 32, 256)), dim3(256), 0, s, type, (const uint8_t*)src, n / 32,
                       (uint16_t*)dst);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
