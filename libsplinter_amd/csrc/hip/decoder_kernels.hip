// decoder_kernels.hip — the non-GEMM elementwise kernels of the completion
// daemon's llama-architecture decoder (K18 of SURVEY §2.10; reference
// splainference.cpp:272-330 runs these inside llama_decode).
//
//   dec_rmsnorm   y = x * rsqrt(mean(x^2) + eps) * w      bf16 in/out, fp32 w
//   dec_rope      llama "normal" RoPE (adjacent pairs) applied IN PLACE to the
//                 q and k column ranges of the fused QKV GEMM output
//   dec_attn_decode  single-token GQA attention over the KV cache (split-L over
//                 16 waves, online softmax, LDS merge) — the per-token decode path
//
//   dec_gemv      M = 1 projections of the decode step (optionally with the RMSNorm of x
//                 fused in): weight rows streamed once with 16-B loads, 4 rows per wave in flight
//   dec_embed_tok / dec_rope_kv / dec_sample
//                 the rest of a decode step, driven by a device-resident state {pos, token,
//                 step} so a whole step (all layers + sampling) can be captured once in a HIP
//                 graph and replayed per token with no host arguments changing
//
// Both are HBM-bound row kernels: one 64-lane wave per row, 16-B (8 x bf16)
// vector accesses, statistics reduced with __shfl_xor over the full wavefront.
// The prefill projections run on the MFMA GEMM (gemm_bf16.hip).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>

namespace {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint32_t h16) { return __uint_as_float(h16 << 16); }
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
  return make_uint4(pk2(f[0], f[1]), pk2(f[2], f[3]), pk2(f[4], f[5]), pk2(f[6], f[7]));
}

// One wave per row, 4 rows per 256-thread block.  Rows of up to 64 x 8 x 4 =
// 2048 elements stay in registers (single HBM read); wider rows re-read their
// remaining chunks in the second pass (the row is cache-resident by then).
constexpr int kRegChunks = 4;

__global__ __launch_bounds__(256) void k_rmsnorm(const uint16_t* __restrict__ x, long ldx, const float* __restrict__ w,
                                                 long T, int d, float eps, uint16_t* __restrict__ out, long ldo) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const int nch = d >> 3;
  const uint16_t* src = x + row * ldx;
  float v[kRegChunks][8];
  float ss = 0.f;
#pragma unroll
  for (int r = 0; r < kRegChunks; ++r) {
    const int c = lane + r * 64;
    if (c < nch) {
      unpack8(*(const uint4*)(src + c * 8), v[r]);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[r][e] * v[r][e];
    }
  }
  for (int c = lane + kRegChunks * 64; c < nch; c += 64) {
    float t[8];
    unpack8(*(const uint4*)(src + c * 8), t);
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += t[e] * t[e];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float rs = rsqrtf(ss / (float)d + eps);
  uint16_t* dst = out + row * ldo;
#pragma unroll
  for (int r = 0; r < kRegChunks; ++r) {
    const int c = lane + r * 64;
    if (c < nch) {
      const float4 w0 = *(const float4*)(w + c * 8), w1 = *(const float4*)(w + c * 8 + 4);
      const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = v[r][e] * rs * ww[e];
      *(uint4*)(dst + c * 8) = pack8(o);
    }
  }
  for (int c = lane + kRegChunks * 64; c < nch; c += 64) {
    float t[8], o[8];
    unpack8(*(const uint4*)(src + c * 8), t);
    const float4 w0 = *(const float4*)(w + c * 8), w1 = *(const float4*)(w + c * 8 + 4);
    const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = t[e] * rs * ww[e];
    *(uint4*)(dst + c * 8) = pack8(o);
  }
}

// In-place RoPE over columns [0, ncols) of each row (q heads then k heads, each hd wide):
// pair (2i, 2i+1) of a head rotates by angle pos * base^(-2i/hd), read from the fp32
// cos/sin tables [n_ctx, hd/2].  One thread per 8 elements (4 pairs).
__global__ __launch_bounds__(256) void k_rope(uint16_t* __restrict__ qkv, long ld, long T, int ncols, int hd,
                                              int pos0, const float* __restrict__ cs, const float* __restrict__ sn) {
  const int per_row = ncols >> 3;
  const long total = T * per_row;
  const int half = hd >> 1;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long row = q / per_row;
    const int col = (int)(q - row * per_row) * 8;
    const int i0 = (col % hd) >> 1;  // first pair index inside the head
    const long p = pos0 + row;
    uint16_t* ptr = qkv + row * ld + col;
    float f[8], o[8];
    unpack8(*(const uint4*)ptr, f);
    const float4 c4 = *(const float4*)(cs + p * half + i0), s4 = *(const float4*)(sn + p * half + i0);
    const float c[4] = {c4.x, c4.y, c4.z, c4.w}, s[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = f[2 * e], b = f[2 * e + 1];
      o[2 * e] = a * c[e] - b * s[e];
      o[2 * e + 1] = a * s[e] + b * c[e];
    }
    *(uint4*)ptr = pack8(o);
  }
}

// Single-token decode attention over the KV cache (GQA): one 1024-thread workgroup per
// query head h (kv head h / (H/KVH)); its 16 waves take interleaved 64-key chunks (a decode
// step launches only H workgroups, so the split-L width lives inside the workgroup).  Inside a
// chunk each lane scores one key (16-B loads along its cache row against the LDS-resident,
// pre-scaled q), the wave keeps an online softmax (max/sum via __shfl_xor), and the V rows
// are accumulated with p broadcast by __shfl, each lane owning DPL = hd/64 contiguous
// output dims.  The 16 partial (m, l, acc) states merge in LDS.  K/V are [L, ldkv] rows
// (ldkv = KVH*hd elements) starting at the kv head's column.
constexpr int kDecWaves = 16;

template <int DPL>
__global__ __launch_bounds__(kDecWaves * 64) void k_attn_decode(const uint16_t* __restrict__ q, const uint16_t* __restrict__ K,
                                                     const uint16_t* __restrict__ V, long ldkv, int L, int grp,
                                                     int hd, float scale, uint16_t* __restrict__ out,
                                                     const int32_t* __restrict__ st) {
  if (st) L = st[0] + 1;  // graph-captured decode step: the cache length lives on the device
  const int h = blockIdx.x;
  const int kvh = h / grp;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __shared__ float qs[256];
  __shared__ float wm[kDecWaves], wl[kDecWaves];
  __shared__ float wacc[kDecWaves][256];
  for (int d = threadIdx.x; d < hd; d += kDecWaves * 64) qs[d] = bf2f(q[(long)h * hd + d]) * scale;
  __syncthreads();
  const uint16_t* Kb = K + (long)kvh * hd;
  const uint16_t* Vb = V + (long)kvh * hd + lane * DPL;
  float m = -INFINITY, l = 0.f, acc[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) acc[i] = 0.f;
  for (int base = wave * 64; base < L; base += kDecWaves * 64) {
    const int j = base + lane;
    float s = -INFINITY;
    if (j < L) {
      const uint16_t* kr = Kb + (long)j * ldkv;
      // hd == 64 * DPL: the key row in batches of 8 16-B loads issued before their FMAs (a
      // runtime-bound loop issued them one latency at a time: 28 us per step at 32 heads); one batch
      // in flight keeps the 1024-thread block inside its 128 VGPRs
      float dot = 0.f;
#pragma unroll 1
      for (int cb = 0; cb < DPL; ++cb) {
        uint4 kv[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) kv[c] = *(const uint4*)(kr + cb * 64 + c * 8);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float f[8];
          unpack8(kv[c], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) dot += f[e] * qs[cb * 64 + c * 8 + e];
        }
      }
      s = dot;
    }
    float cm = s;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cm = fmaxf(cm, __shfl_xor(cm, o, 64));
    const float mn = fmaxf(m, cm);  // finite: lane 0 of every visited chunk holds a key
    const float corr = __expf(m - mn);
    const float p = j < L ? __expf(s - mn) : 0.f;
    float ps = p;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ps += __shfl_xor(ps, o, 64);
    l = l * corr + ps;
#pragma unroll
    for (int i = 0; i < DPL; ++i) acc[i] *= corr;
    const int nv = min(64, L - base);
#pragma unroll 8
    for (int t = 0; t < nv; ++t) {
      const float pt = __shfl(p, t, 64);
      const uint16_t* vr = Vb + (long)(base + t) * ldkv;
#pragma unroll
      for (int i = 0; i < DPL; ++i) acc[i] += pt * bf2f(vr[i]);
    }
    m = mn;
  }
  if (lane == 0) { wm[wave] = m; wl[wave] = l; }
#pragma unroll
  for (int i = 0; i < DPL; ++i) wacc[wave][lane * DPL + i] = acc[i];
  __syncthreads();
  float M = wm[0];
#pragma unroll
  for (int w = 1; w < kDecWaves; ++w) M = fmaxf(M, wm[w]);
  float c[kDecWaves], den = 0.f;
#pragma unroll
  for (int w = 0; w < kDecWaves; ++w) { c[w] = __expf(wm[w] - M); den += wl[w] * c[w]; }
  const float inv = 1.f / den;
  for (int d = threadIdx.x; d < hd; d += kDecWaves * 64) {
    float o = 0.f;
#pragma unroll
    for (int w = 0; w < kDecWaves; ++w) o += wacc[w][d] * c[w];
    o *= inv;
    out[(long)h * hd + d] = __builtin_bit_cast(uint16_t, (__bf16)o);
  }
}


// Split-L decode attention (flash-decoding) for long caches: grid (H, S), workgroup (h, j) of 4 waves
// scores keys [j c, (j + 1) c) with c = ceil(L / S) rounded up to 64 and writes its unnormalised
// partial (m, l, acc[hd]) to ws; k_attn_combine merges the S partials of a head.  One workgroup per
// head streams the whole cache through one CU (164 GB/s at L = 8192, profiles/r2_decode_q4.md).
// k_attn_decode_g: decode attention for caches of at most kSmallL keys (the single-workgroup regime).
// One workgroup per KV head serves its G query heads, so every K / V row is read once for the group
// instead of once per head, and no phase walks the keys one at a time:
//   scores  hd/8 lanes per key row (16-B pieces), U rows per lane in flight, G dot products per piece,
//           reduced across the row's lanes with xor shuffles -> LDS sc[g][key] (q pre-scaled)
//   softmax one wave per head: max, exp, sum over the keys in LDS
//   P V     the same row pieces of V, U rows in flight, fp32 accumulators per (head, 8 dims), then a
//           reduction over the 256/(hd/8) key groups through LDS.
// The single-workgroup kernel below it walks each wave's 64 keys serially in P V (a shuffle and a
// 4-B load per key): 28 us per layer at a 300-key cache, llama-7B heads (profiles/r3_decode_splits_short_ctx.jsonl);
// this kernel 11.5 us, q4 decode 0.715 -> 0.577 ms/token (profiles/r3_decode_attn_small_ab.jsonl).  A 16-wave form
// (one load round per phase, shuffle + LDS reduction) measured slower: 14.1 us (r3_decode_attn_small_wide_ab.jsonl).
// Its split form runs the flash-decoding splits of longer caches: 3000-token prompt 0.840 -> 0.672 ms/token at 4 bits
// (profiles/r3_decode_attn_grouped_split_ab.jsonl).
constexpr int kSmallL = 512;
// SPLIT: the same kernel as one split of the flash-decoding form -- workgroup (kvh, j) takes keys
// [j * chunk, (j + 1) * chunk) (chunk <= kSmallL, the k_attn_decode_split geometry) and writes each head's
// partial (max, sum, unnormalised P V) to ws for k_attn_combine.
template <int D, int G, bool SPLIT = false>
__global__ __launch_bounds__(256) void k_attn_decode_g(const uint16_t* __restrict__ q, const uint16_t* __restrict__ K,
                                                       const uint16_t* __restrict__ V, long ldkv, int L, float scale,
                                                       uint16_t* __restrict__ out, const int32_t* __restrict__ st,
                                                       float* __restrict__ ws = nullptr) {
  constexpr int hd = 64 * D, TPK = hd / 8, KP = 256 / TPK, U = 8;
  static_assert(64 % TPK == 0, "a key row's lanes must sit in one wave");
  if (st) L = st[0] + 1;
  int k0 = 0, k1 = L < kSmallL ? L : kSmallL;  // one workgroup: the host picks it only for capacities <= kSmallL
  if constexpr (SPLIT) {
    const int S = gridDim.y, chunk = ((L + S - 1) / S + 63) / 64 * 64;
    k0 = blockIdx.y * chunk;
    k1 = min(L, k0 + min(chunk, kSmallL));  // the host guarantees chunk <= kSmallL
  }
  const int n = k1 > k0 ? k1 - k0 : 0;
  const int kvh = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int sub = tid % TPK, kg = tid / TPK;
  __shared__ float sc[G][kSmallL];
  __shared__ float red[KP][G][hd];
  __shared__ float lsum[G], lmax[G];
  float qv[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float f[8];
    unpack8(*(const uint4*)(q + (long)(kvh * G + g) * hd + sub * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[g][e] = f[e] * scale;
  }
  const uint16_t* Kb = K + (long)kvh * hd + sub * 8 + (long)k0 * ldkv;
  const uint16_t* Vb = V + (long)kvh * hd + sub * 8 + (long)k0 * ldkv;
  // ---- scores
  for (int j0 = 0; j0 < n; j0 += KP * U) {
    uint4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * KP + kg;
      r[u] = j < n ? *(const uint4*)(Kb + (long)j * ldkv) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * KP + kg;
      float f[8], d[G];
      unpack8(r[u], f);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        d[g] = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d[g] = fmaf(f[e], qv[g][e], d[g]);
#pragma unroll
        for (int o = TPK / 2; o >= 1; o >>= 1) d[g] += __shfl_xor(d[g], o, 64);
      }
      if (sub == 0 && j < n) {
#pragma unroll
        for (int g = 0; g < G; ++g) sc[g][j] = d[g];
      }
    }
  }
  __syncthreads();
  // ---- softmax, one wave per head
  for (int g = wave; g < G; g += 4) {
    float mx = -INFINITY;
    for (int j = lane; j < n; j += 64) mx = fmaxf(mx, sc[g][j]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float sum = 0.f;
    for (int j = lane; j < n; j += 64) {
      const float p = __expf(sc[g][j] - mx);
      sc[g][j] = p;
      sum += p;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) {
      lsum[g] = sum;
      lmax[g] = mx;
    }
  }
  __syncthreads();
  // ---- P V
  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[g][e] = 0.f;
  for (int j0 = 0; j0 < n; j0 += KP * U) {
    uint4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * KP + kg;
      r[u] = j < n ? *(const uint4*)(Vb + (long)j * ldkv) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * KP + kg;
      if (j < n) {
        float f[8];
        unpack8(r[u], f);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float p = sc[g][j];
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[g][e] = fmaf(p, f[e], acc[g][e]);
        }
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[kg][g][sub * 8 + e] = acc[g][e];
  __syncthreads();
  if constexpr (SPLIT) {
    // ws[head][split][hd + 2] = (max, sum, unnormalised P V): the k_attn_decode_split layout; an empty split
    // leaves max = -inf, sum 0 (k_attn_combine gives it weight 0)
    const int S = gridDim.y;
    for (int idx = tid; idx < G * (hd + 2); idx += 256) {
      const int g = idx / (hd + 2), c = idx - g * (hd + 2);
      float v;
      if (c == 0) v = n ? lmax[g] : -INFINITY;
      else if (c == 1) v = n ? lsum[g] : 0.f;
      else {
        v = 0.f;
#pragma unroll 8
        for (int k = 0; k < KP; ++k) v += red[k][g][c - 2];
      }
      ws[((long)(kvh * G + g) * S + blockIdx.y) * (hd + 2) + c] = v;
    }
  } else {
    for (int idx = tid; idx < G * hd; idx += 256) {
      const int g = idx / hd, d = idx - g * hd;
      float o = 0.f;
#pragma unroll 8
      for (int k = 0; k < KP; ++k) o += red[k][g][d];
      out[(long)(kvh * G + g) * hd + d] = __builtin_bit_cast(uint16_t, (__bf16)(o / lsum[g]));
    }
  }
}

constexpr int kSplitWaves = 4;
constexpr int kMaxSplits = 32;

template <int DPL, int G>
__global__ __launch_bounds__(kSplitWaves * 64) void k_attn_decode_split(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V, long ldkv, int L,
    int grp, float scale, float* __restrict__ ws, const int32_t* __restrict__ st) {
  // G query heads of one kv group per workgroup (grouped-query attention): every key and value row
  // is loaded once for all G heads instead of once per head
  constexpr int hd = 64 * DPL;
  if (st) L = st[0] + 1;
  const int h0 = blockIdx.x * G, S = gridDim.y, j = blockIdx.y;
  const int kvh = h0 / grp;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int chunk = ((L + S - 1) / S + 63) / 64 * 64;
  const int k0 = j * chunk, k1 = min(L, k0 + chunk);
  __shared__ float qs[G][hd];
  __shared__ float wm[kSplitWaves][G], wl[kSplitWaves][G];
  __shared__ float wacc[kSplitWaves][G][hd];
  for (int d = threadIdx.x; d < G * hd; d += kSplitWaves * 64) qs[d / hd][d % hd] = bf2f(q[(long)h0 * hd + d]) * scale;
  __syncthreads();
  const uint16_t* Kb = K + (long)kvh * hd;
  const uint16_t* Vb = V + (long)kvh * hd + lane * DPL;
  float m[G], l[G], acc[G][DPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int i = 0; i < DPL; ++i) acc[g][i] = 0.f;
  }
  for (int base = k0 + wave * 64; base < k1; base += kSplitWaves * 64) {
    const int jj = base + lane;
    float sc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) sc[g] = -INFINITY;
    if (jj < k1) {
      const uint16_t* kr = Kb + (long)jj * ldkv;
      float dot[G];
#pragma unroll
      for (int g = 0; g < G; ++g) dot[g] = 0.f;
#pragma unroll 1
      for (int cb = 0; cb < DPL; ++cb) {
        uint4 kv[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) kv[c] = *(const uint4*)(kr + cb * 64 + c * 8);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float f[8];
          unpack8(kv[c], f);
#pragma unroll
          for (int g = 0; g < G; ++g)
#pragma unroll
            for (int e = 0; e < 8; ++e) dot[g] += f[e] * qs[g][cb * 64 + c * 8 + e];
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) sc[g] = dot[g];
    }
    float p[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float cm = sc[g];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) cm = fmaxf(cm, __shfl_xor(cm, o, 64));
      const float mn = fmaxf(m[g], cm);
      const float corr = __expf(m[g] - mn);
      p[g] = jj < k1 ? __expf(sc[g] - mn) : 0.f;
      float ps = p[g];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ps += __shfl_xor(ps, o, 64);
      l[g] = l[g] * corr + ps;
#pragma unroll
      for (int i = 0; i < DPL; ++i) acc[g][i] *= corr;
      m[g] = mn;
    }
    const int nv = min(64, k1 - base);
#pragma unroll 4
    for (int t = 0; t < nv; ++t) {
      const uint16_t* vr = Vb + (long)(base + t) * ldkv;
      float vv[DPL];
#pragma unroll
      for (int i = 0; i < DPL; ++i) vv[i] = bf2f(vr[i]);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float pt = __shfl(p[g], t, 64);
#pragma unroll
        for (int i = 0; i < DPL; ++i) acc[g][i] += pt * vv[i];
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (lane == 0) { wm[wave][g] = m[g]; wl[wave][g] = l[g]; }
#pragma unroll
    for (int i = 0; i < DPL; ++i) wacc[wave][g][lane * DPL + i] = acc[g][i];
  }
  __syncthreads();
  for (int g = 0; g < G; ++g) {
    float M = wm[0][g];
#pragma unroll
    for (int w = 1; w < kSplitWaves; ++w) M = fmaxf(M, wm[w][g]);
    float* o = ws + ((long)(h0 + g) * S + j) * (hd + 2);
    float c[kSplitWaves], den = 0.f;
#pragma unroll
    for (int w = 0; w < kSplitWaves; ++w) {
      c[w] = wm[w][g] == -INFINITY ? 0.f : __expf(wm[w][g] - M);  // an empty wave (or split) adds nothing
      den += wl[w][g] * c[w];
    }
    for (int d = threadIdx.x; d < hd; d += kSplitWaves * 64) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < kSplitWaves; ++w) a += wacc[w][g][d] * c[w];
      o[2 + d] = a;
    }
    if (threadIdx.x == 0) { o[0] = M; o[1] = den; }
  }
}

// out[h] = sum_j acc_j e^(m_j - M) / sum_j l_j e^(m_j - M) over the S partials of head h
__global__ void k_attn_combine(const float* __restrict__ ws, int S, int hd, uint16_t* __restrict__ out) {
  const int h = blockIdx.x;
  const float* p = ws + (long)h * S * (hd + 2);
  float M = -INFINITY;
  for (int j = 0; j < S; ++j) M = fmaxf(M, p[(long)j * (hd + 2)]);
  float den = 0.f, a = 0.f;
  const int d = threadIdx.x;
  for (int j = 0; j < S; ++j) {
    const float* pj = p + (long)j * (hd + 2);
    const float c = pj[0] == -INFINITY ? 0.f : __expf(pj[0] - M);
    den += pj[1] * c;
    if (d < hd) a += pj[2 + d] * c;
  }
  if (d < hd) out[(long)h * hd + d] = __builtin_bit_cast(uint16_t, (__bf16)(a / den));
}

// ------------------------------------------------------------------ decode step --
// Device state of a generation (int32): [0] pos = tokens already in the KV cache, [1] token = the
// token the next step consumes (the last sampled one), [2] step = sampler draws so far.
enum { ST_POS = 0, ST_TOK = 1, ST_STEP = 2 };

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// y[n] = x . W[n, :] for one token.  x (bf16 [K], optionally RMS-normalised in LDS first: the
// dec_rmsnorm + GEMV pair of a layer in one launch) is staged in LDS; each wave owns 4 weight rows
// and streams them with 16-B loads, 4 independent accumulators in flight.  MODE 0: bf16 out,
// 1: + residual (bf16, may alias out: each element is read and written by the same lane),
// 2: SwiGLU over pack_upgate rows (out[o] = up * silu(gate), o -> rows 32(o/16) + o%16 and +16),
// 4: fp32 out (logits).
constexpr int kGemvRows = 4;
constexpr int kGemvMaxK = 16384;

template <int MODE, bool RMS>
__global__ __launch_bounds__(256) void k_gemv(const uint16_t* __restrict__ x, const float* __restrict__ rw, float eps,
                                              const uint16_t* __restrict__ W, int K, int nout,
                                              const uint16_t* res, void* out) {
  __shared__ __attribute__((aligned(16))) uint16_t xs[kGemvMaxK];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nch = K >> 3;
  // this wave's outputs and their weight rows; the first chunk of every row is requested BEFORE x
  // is staged, so its HBM latency overlaps the staging and the barriers (as k_gemv_q4)
  constexpr int outs = MODE == 2 ? kGemvRows / 2 : kGemvRows;
  const int o0 = (blockIdx.x * 4 + wave) * outs;
  const bool active = o0 < nout;
  long rows[kGemvRows];
#pragma unroll
  for (int r = 0; r < kGemvRows; ++r) {
    int o = o0 + (MODE == 2 ? r / 2 : r);
    if (o >= nout) o = nout - 1;  // tail: recompute the last output, never stored twice
    rows[r] = MODE == 2 ? (long)(32 * (o / 16) + (o % 16) + (r & 1) * 16) : (long)o;
  }
  uint4 wv[kGemvRows];
  if (active && lane < nch) {
#pragma unroll
    for (int r = 0; r < kGemvRows; ++r) wv[r] = *(const uint4*)(W + rows[r] * K + lane * 8);
  }
  float ss = 0.f;
  for (int c = tid; c < nch; c += 256) {
    const uint4 v = *(const uint4*)(x + c * 8);
    *(uint4*)(xs + c * 8) = v;
    if constexpr (RMS) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += f[e] * f[e];
    }
  }
  if constexpr (RMS) {
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    const float rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)K + eps);
    for (int c = tid; c < nch; c += 256) {  // each thread rewrites the chunks it staged
      float f[8];
      unpack8(*(const uint4*)(xs + c * 8), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = f[e] * rs * rw[c * 8 + e];
      *(uint4*)(xs + c * 8) = pack8(f);
    }
  }
  __syncthreads();
  if (!active) return;
  float acc[kGemvRows] = {};
  for (int c = lane; c < nch; c += 64) {
    uint4 cw[kGemvRows];
#pragma unroll
    for (int r = 0; r < kGemvRows; ++r) cw[r] = wv[r];
    if (c + 64 < nch) {  // one chunk of look-ahead per row
#pragma unroll
      for (int r = 0; r < kGemvRows; ++r) wv[r] = *(const uint4*)(W + rows[r] * K + (c + 64) * 8);
    }
    float xf[8];
    unpack8(*(const uint4*)(xs + c * 8), xf);
#pragma unroll
    for (int r = 0; r < kGemvRows; ++r) {
      float wf[8];
      unpack8(cw[r], wf);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[r] += wf[e] * xf[e];
    }
  }
#pragma unroll
  for (int r = 0; r < kGemvRows; ++r) acc[r] = wave_sum(acc[r]);
  if (lane < outs) {
    const int o = o0 + lane;
    if (o < nout) {
      float a0 = acc[0], a1 = acc[1];
#pragma unroll
      for (int r = 0; r < kGemvRows; ++r)
        if ((MODE == 2 ? r / 2 : r) == lane) {
          if (MODE == 2) { if (r & 1) a1 = acc[r]; else a0 = acc[r]; }
          else a0 = acc[r];
        }
      if constexpr (MODE == 4) {
        ((float*)out)[o] = a0;
      } else {
        float y = a0;
        if constexpr (MODE == 1) y += bf2f(res[o]);
        if constexpr (MODE == 2) y = a0 * a1 / (1.f + __expf(-a1));
        ((uint16_t*)out)[o] = __builtin_bit_cast(uint16_t, (__bf16)y);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 4-bit weights (Q4G32): W [N, K] resident in HBM at 0.625 B per weight instead of 2.
//   q  : uint8 [N, K/2]  -- k = 2j in the low nibble of byte j, k = 2j + 1 in the high nibble
//   sm : uint32 [N, K/32] -- per 32-k group, bf16 pair (d low, m high): w = d * q + m
// The decode step is weight-bandwidth bound (every weight read once per token), so the GEMV reads
// 3.2x fewer bytes than the bf16 one.  GGUF Q4_0 / Q4_1 / Q4_K blocks are all affine 4-bit grids
// over 32-weight (sub)blocks, which is the layout this format keeps (reference: llama.cpp reads
// its Q4 weights directly in llama_decode, splainference.cpp:272-330).
// ---------------------------------------------------------------------------
constexpr int kQ4Group = 32;

// nibble pairs -> floats: for one dword of 8 nibbles (k = 0..7), lo bytes hold k = 0,2,4,6 and hi
// bytes k = 1,3,5,7; each byte converts with a single v_cvt_f32_ubyteN
__device__ __forceinline__ float q4dot8(uint32_t w, const float* x) {
  const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
  float s = (float)(lo & 0xff) * x[0];
  s = fmaf((float)(hi & 0xff), x[1], s);
  s = fmaf((float)((lo >> 8) & 0xff), x[2], s);
  s = fmaf((float)((hi >> 8) & 0xff), x[3], s);
  s = fmaf((float)((lo >> 16) & 0xff), x[4], s);
  s = fmaf((float)((hi >> 16) & 0xff), x[5], s);
  s = fmaf((float)(lo >> 24), x[6], s);
  return fmaf((float)(hi >> 24), x[7], s);
}

// y[n] = x . W[n, :] with W in Q4G32.  Structure of k_gemv: x (optionally RMS-normalised) staged
// in LDS as fp32 together with its 32-group sums (the m term: sum_k (d q_k + m) x_k =
// d sum_k q_k x_k + m sum_k x_k); each wave owns R (4 or 8) weight rows, each lane one 32-k group per row
// and iteration (one 16-B load of nibbles + one scale word per row).
constexpr int kGemvQ4MaxK = 16384;
constexpr int kQ4Rec = kQ4Group + 4;  // LDS floats per group record

// 8-bit bytes -> floats, one v_cvt_f32_ubyteN each (Q8G32: k = 4j .. 4j+3 in dword j)
__device__ __forceinline__ float q8dot4(uint32_t w, const float* x) {
  float s = (float)(w & 0xff) * x[0];
  s = fmaf((float)((w >> 8) & 0xff), x[1], s);
  s = fmaf((float)((w >> 16) & 0xff), x[2], s);
  return fmaf((float)(w >> 24), x[3], s);
}

// BITS 4: Q4G32 nibbles (16 B per group); BITS 8: Q8G32 bytes (32 B per group, the same (d, m)
// words: w = d * u + m with u in 0..255) -- the >4-bit GGUF tensors (Q6_K / Q5_x / Q8_0 / F16) of a
// mostly-4-bit file keep >= 6 bits instead of being re-gridded to 4
template <int MODE, bool RMS, int R = kGemvRows, int BITS = 4>
__global__ __launch_bounds__(256) void k_gemv_q4(const uint16_t* __restrict__ x, const float* __restrict__ rw,
                                                 float eps, const uint8_t* __restrict__ Wq,
                                                 const uint32_t* __restrict__ Wsm, int K, int nout,
                                                 const uint16_t* res, void* out) {
  // dynamic LDS, fp32, one 36-float record per 32-k group: x[32], the group sum, 3 pad.  The
  // 144-B record stride keeps the main loop's per-lane ds_read_b128 of consecutive groups
  // conflict-free (16-lane phases start on 16 distinct 4-bank quads).
  extern __shared__ __attribute__((aligned(16))) float xs[];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nch = K >> 3, ng = K / kQ4Group;
  // this wave's weight rows, and its first group's weights requested BEFORE x is staged: the HBM
  // latency of the first loads overlaps the staging and its barriers
  constexpr int outs = MODE == 2 ? R / 2 : R;
  const int o0 = (blockIdx.x * 4 + wave) * outs;
  const bool active = o0 < nout;
  long rows[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int o = o0 + (MODE == 2 ? r / 2 : r);
    if (o >= nout) o = nout - 1;  // tail: recompute the last output, never stored twice
    rows[r] = MODE == 2 ? (long)(32 * (o / 16) + (o % 16) + (r & 1) * 16) : (long)o;
  }
  constexpr int GV = BITS / 4;  // 16-B loads per group and row
  const long qrow = (long)K * BITS / 8;
  uint4 wq[R][GV];
  uint32_t sm[R];
  if (active && lane < ng) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int v = 0; v < GV; ++v) wq[r][v] = *(const uint4*)(Wq + rows[r] * qrow + lane * 16 * GV + v * 16);
      sm[r] = Wsm[rows[r] * ng + lane];
    }
  }
  float ss = 0.f;
  for (int c = tid; c < nch; c += 256) {
    float f[8];
    unpack8(*(const uint4*)(x + c * 8), f);
    float* px = xs + (c >> 2) * kQ4Rec + (c & 3) * 8;
    *(float4*)px = make_float4(f[0], f[1], f[2], f[3]);
    *(float4*)(px + 4) = make_float4(f[4], f[5], f[6], f[7]);
    if constexpr (RMS) {
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += f[e] * f[e];
    }
  }
  float rs = 1.f;
  if constexpr (RMS) {
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)K + eps);
  }
  // each thread revisits the chunks it staged: RMS scaling (x * rs * w rounded to bf16, as the bf16
  // path feeds its GEMV) and the 32-group sums over the 4 consecutive lanes holding a group's chunks
  // (nch % 4 == 0 and the stride 256 keep a group's 4 lanes active together)
  for (int c = tid; c < nch; c += 256) {
    float* px = xs + (c >> 2) * kQ4Rec + (c & 3) * 8;
    float4 a = *(const float4*)px, b = *(const float4*)(px + 4);
    if constexpr (RMS) {
      const float4 wa = *(const float4*)(rw + c * 8), wb = *(const float4*)(rw + c * 8 + 4);
      a = make_float4((float)(__bf16)(a.x * rs * wa.x), (float)(__bf16)(a.y * rs * wa.y),
                      (float)(__bf16)(a.z * rs * wa.z), (float)(__bf16)(a.w * rs * wa.w));
      b = make_float4((float)(__bf16)(b.x * rs * wb.x), (float)(__bf16)(b.y * rs * wb.y),
                      (float)(__bf16)(b.z * rs * wb.z), (float)(__bf16)(b.w * rs * wb.w));
      *(float4*)px = a;
      *(float4*)(px + 4) = b;
    }
    float s = ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if ((c & 3) == 0) xs[(c >> 2) * kQ4Rec + kQ4Group] = s;
  }
  __syncthreads();
  if (!active) return;
  float acc[R] = {};
  for (int g = lane; g < ng; g += 64) {
    // the group's weights are in registers; request the next group's before the math (one group
    // of look-ahead per lane: 2 x 4 x 20 B in flight)
    uint4 cq[R][GV];
    uint32_t csm[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int v = 0; v < GV; ++v) cq[r][v] = wq[r][v];
      csm[r] = sm[r];
    }
    if (g + 64 < ng) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int v = 0; v < GV; ++v) wq[r][v] = *(const uint4*)(Wq + rows[r] * qrow + (g + 64) * 16 * GV + v * 16);
        sm[r] = Wsm[rows[r] * ng + g + 64];
      }
    }
    float xg[kQ4Group];
#pragma unroll
    for (int e = 0; e < kQ4Group; e += 4) *(float4*)(xg + e) = *(const float4*)(xs + g * kQ4Rec + e);
    const float gs = xs[g * kQ4Rec + kQ4Group];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float dot;
      if constexpr (BITS == 4) {
        dot = q4dot8(cq[r][0].x, xg);
        dot += q4dot8(cq[r][0].y, xg + 8);
        dot += q4dot8(cq[r][0].z, xg + 16);
        dot += q4dot8(cq[r][0].w, xg + 24);
      } else {
        dot = q8dot4(cq[r][0].x, xg);
        dot += q8dot4(cq[r][0].y, xg + 4);
        dot += q8dot4(cq[r][0].z, xg + 8);
        dot += q8dot4(cq[r][0].w, xg + 12);
        dot += q8dot4(cq[r][GV - 1].x, xg + 16);
        dot += q8dot4(cq[r][GV - 1].y, xg + 20);
        dot += q8dot4(cq[r][GV - 1].z, xg + 24);
        dot += q8dot4(cq[r][GV - 1].w, xg + 28);
      }
      acc[r] = fmaf(bf2f(csm[r] & 0xffff), dot, fmaf(bf2f(csm[r] >> 16), gs, acc[r]));
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (lane < outs) {
    const int o = o0 + lane;
    if (o < nout) {
      float a0 = acc[0], a1 = acc[1];
#pragma unroll
      for (int r = 0; r < R; ++r)
        if ((MODE == 2 ? r / 2 : r) == lane) {
          if (MODE == 2) { if (r & 1) a1 = acc[r]; else a0 = acc[r]; }
          else a0 = acc[r];
        }
      if constexpr (MODE == 4) {
        ((float*)out)[o] = a0;
      } else {
        float y = a0;
        if constexpr (MODE == 1) y += bf2f(res[o]);
        if constexpr (MODE == 2) y = a0 * a1 / (1.f + __expf(-a1));
        ((uint16_t*)out)[o] = __builtin_bit_cast(uint16_t, (__bf16)y);
      }
    }
  }
}

// bf16 W [N, K] -> Q4G32 (one thread per 32-weight group): affine min/max grid, d and m rounded
// to bf16 first and the nibbles chosen against the rounded pair
__global__ void k_q4_quant(const uint16_t* __restrict__ W, long groups, int ng, uint8_t* __restrict__ Wq,
                           uint32_t* __restrict__ Wsm) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= groups) return;
  float v[kQ4Group];
  const uint4* src = (const uint4*)(W + i * kQ4Group);
#pragma unroll
  for (int c = 0; c < 4; ++c) unpack8(src[c], v + c * 8);
  float lo = v[0], hi = v[0];
#pragma unroll
  for (int e = 1; e < kQ4Group; ++e) { lo = fminf(lo, v[e]); hi = fmaxf(hi, v[e]); }
  const float m = (float)(__bf16)lo;
  float d = (float)(__bf16)((hi - m) / 15.f);
  if (!(d > 0.f)) d = 0.f;
  const float inv = d > 0.f ? 1.f / d : 0.f;
  uint32_t packed[4] = {0, 0, 0, 0};
#pragma unroll
  for (int e = 0; e < kQ4Group; ++e) {
    int q = (int)rintf((v[e] - m) * inv);
    q = q < 0 ? 0 : (q > 15 ? 15 : q);
    packed[e >> 3] |= (uint32_t)q << (4 * (e & 7));
  }
  *(uint4*)(Wq + i * 16) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
  Wsm[i] = pk2(d, m);
  (void)ng;
}

// Q4G32 -> bf16 W [N, K] (prefill: the MFMA GEMM consumes one dequantised matrix at a time)
__global__ void k_q4_dequant(const uint8_t* __restrict__ Wq, const uint32_t* __restrict__ Wsm, long groups,
                             uint16_t* __restrict__ W) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= groups) return;
  const uint4 q = *(const uint4*)(Wq + i * 16);
  const uint32_t sm = Wsm[i];
  const float d = bf2f(sm & 0xffff), m = bf2f(sm >> 16);
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
  uint4* dst = (uint4*)(W + i * kQ4Group);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fmaf(d, (float)((qw[c] >> (4 * e)) & 15u), m);
    dst[c] = pack8(f);
  }
}

__device__ __forceinline__ float bf16_floor(float x) {
  uint32_t u = __float_as_uint(x) & 0xFFFF0000u;
  if (__uint_as_float(u) > x) u += 0x10000u;  // negative: truncation went toward zero, one ulp down
  return __uint_as_float(u);
}
__device__ __forceinline__ float bf16_ceil(float x) {
  uint32_t u = __float_as_uint(x) & 0xFFFF0000u;
  if (__uint_as_float(u) < x) u += 0x10000u;  // positive: one ulp up
  return __uint_as_float(u);
}

// bf16 W [N, K] <-> Q8G32 (one thread per 32-weight group): affine 255-step grid over the group's
// [min, max], (d, m) rounded to bf16 outward first and the bytes chosen against the rounded pair
__global__ void k_q8_quant(const uint16_t* __restrict__ W, long groups, uint8_t* __restrict__ Wq,
                           uint32_t* __restrict__ Wsm) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= groups) return;
  float v[kQ4Group];
  const uint4* src = (const uint4*)(W + i * kQ4Group);
#pragma unroll
  for (int c = 0; c < 4; ++c) unpack8(src[c], v + c * 8);
  float lo = v[0], hi = v[0];
#pragma unroll
  for (int e = 1; e < kQ4Group; ++e) { lo = fminf(lo, v[e]); hi = fmaxf(hi, v[e]); }
  // m rounded DOWN and d UP to bf16, so the 255-step grid still spans [lo, hi]: at 8 bits a
  // round-to-nearest m would move the grid by up to |m| 2^-9, most of a step
  const float m = bf16_floor(lo);
  float d = bf16_ceil((hi - m) / 255.f);
  if (!(d > 0.f)) d = 0.f;
  const float inv = d > 0.f ? 1.f / d : 0.f;
  uint32_t packed[8] = {};
#pragma unroll
  for (int e = 0; e < kQ4Group; ++e) {
    int q = (int)rintf((v[e] - m) * inv);
    q = q < 0 ? 0 : (q > 255 ? 255 : q);
    packed[e >> 2] |= (uint32_t)q << (8 * (e & 3));
  }
  *(uint4*)(Wq + i * 32) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
  *(uint4*)(Wq + i * 32 + 16) = make_uint4(packed[4], packed[5], packed[6], packed[7]);
  Wsm[i] = pk2(d, m);
}

__global__ void k_q8_dequant(const uint8_t* __restrict__ Wq, const uint32_t* __restrict__ Wsm, long groups,
                             uint16_t* __restrict__ W) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= groups) return;
  const uint4 a = *(const uint4*)(Wq + i * 32), b = *(const uint4*)(Wq + i * 32 + 16);
  const uint32_t sm = Wsm[i];
  const float d = bf2f(sm & 0xffff), m = bf2f(sm >> 16);
  const uint32_t qw[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint4* dst = (uint4*)(W + i * kQ4Group);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fmaf(d, (float)((qw[2 * c + (e >> 2)] >> (8 * (e & 3))) & 255u), m);
    dst[c] = pack8(f);
  }
}

// x = emb[state.token]
__global__ void k_embed_tok(const uint16_t* __restrict__ emb, int d, const int32_t* __restrict__ st,
                            uint16_t* __restrict__ x) {
  const long t = st[ST_TOK];
  for (int c = threadIdx.x; c < d / 8; c += blockDim.x) *(uint4*)(x + c * 8) = *(const uint4*)(emb + t * d + c * 8);
}

// RoPE of the step's q (in place) and k at position state.pos, and the k / v rows appended to the
// layer's KV cache (row pos of [n_ctx, ldkv]).  One thread per rotation pair / per 8 v elements.
__global__ void k_rope_kv(uint16_t* __restrict__ qkv, int H, int KVH, int hd, const float* __restrict__ cs,
                          const float* __restrict__ sn, const int32_t* __restrict__ st, uint16_t* __restrict__ kc,
                          uint16_t* __restrict__ vc, long ldkv) {
  const long p = st[ST_POS];
  const int half = hd >> 1;
  const int npairs = (H + KVH) * half;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npairs + KVH * hd; i += gridDim.x * blockDim.x) {
    if (i < npairs) {
      const int head = i / half, j = i - head * half;
      uint16_t* ptr = qkv + (long)head * hd + 2 * j;
      const float a = bf2f(ptr[0]), b = bf2f(ptr[1]);
      const float c = cs[p * half + j], s = sn[p * half + j];
      const uint16_t y0 = __builtin_bit_cast(uint16_t, (__bf16)(a * c - b * s));
      const uint16_t y1 = __builtin_bit_cast(uint16_t, (__bf16)(a * s + b * c));
      if (head < H) {
        ptr[0] = y0;
        ptr[1] = y1;
      } else {
        uint16_t* kr = kc + p * ldkv + (long)(head - H) * hd + 2 * j;
        kr[0] = y0;
        kr[1] = y1;
      }
    } else {
      const int e = i - npairs;
      vc[p * ldkv + e] = qkv[(long)(H + KVH) * hd + e];
    }
  }
}

// counter-based uniform in [0, 1): splitmix64 of (seed, draw index)
__device__ __forceinline__ double uniform01(uint64_t seed, uint64_t n) {
  uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// top-p -> temperature -> categorical draw on the device (the reference's llama sampler chain,
// splainference.cpp:272-279): the nucleus is the smallest set of the most probable tokens whose
// probability reaches top_p, found as a logit threshold by bisection (no sort); the kept logits are
// divided by temp and one token is drawn by an inclusive scan in index order.  One 1024-thread
// workgroup; logits stay in L2 between the passes.  Writes state.token (and pos += inc_pos,
// step += 1) and the token to `host_tok` (pinned, may be null).
constexpr int kSampThreads = 1024;

__device__ float block_reduce(float v, float* sh, bool is_max) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = is_max ? wave_max(v) : wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float r = sh[0];
  for (int w = 1; w < kSampThreads / 64; ++w) r = is_max ? fmaxf(r, sh[w]) : r + sh[w];
  return r;
}

__global__ __launch_bounds__(kSampThreads) void k_sample(const float* __restrict__ logits, int V,
                                                         const uint8_t* __restrict__ mask, float top_p, float temp,
                                                         uint64_t seed, int32_t* __restrict__ st, int inc_pos,
                                                         int32_t* host_tok) {
  __shared__ float sh[kSampThreads / 64];
  __shared__ float scan[kSampThreads];
  const int tid = threadIdx.x;
  auto lg = [&](int i) { return (mask && !mask[i]) ? -INFINITY : logits[i]; };
  float m = -INFINITY;
#pragma unroll 8  // 8 logit loads in flight per thread (a rolled loop waits one L2 latency per element)
  for (int i = tid; i < V; i += kSampThreads) m = fmaxf(m, lg(i));
  const float M = block_reduce(m, sh, true);
  float z = 0.f;
#pragma unroll 8  // 8 logit loads in flight per thread (a rolled loop waits one L2 latency per element)
  for (int i = tid; i < V; i += kSampThreads) z += __expf(lg(i) - M);
  const float Z = block_reduce(z, sh, false);
  // nucleus threshold t: the largest logit cut whose kept mass reaches top_p.  Found by two
  // levels of a 1024-bin mass histogram over the current interval [lo, hi) (LDS float atomics),
  // each level keeping the bin where the suffix mass crosses top_p * Z: 2 passes over the logits
  // to a resolution of 40 / 2^20 (a few float ulps of a logit), instead of one pass per bisection
  // step (24 passes: 163 us per token for a 32000-token vocabulary).
  __shared__ float hist[kSampThreads];
  // 8 copies of every bin, picked by lane & 7: flat logits (a random-init model: every logit in
  // one or two bins) put a wave's 64 same-address LDS atomics into one 64-way conflict; the copies
  // cut it to 8-way (83 -> ? us per token at V = 32000, profiles/r2_decode_q4.md)
  __shared__ float hist8[kSampThreads * 8];
  __shared__ int jstar;
  float lo = M - 40.f;  // mass below M - 40 is < V e^-40
  if (top_p < 1.f) {
    const float target = top_p * Z;
    float w = 40.f / kSampThreads * (1.f + 1e-6f);  // bin width: the top bin holds l == M
    float above = 0.f;                              // mass at or above the interval's upper end
    for (int level = 0; level < 2; ++level) {
#pragma unroll
      for (int c = 0; c < 8; ++c) hist8[c * kSampThreads + tid] = 0.f;
      if (tid == 0) jstar = 0;
      __syncthreads();
      const float inv_w = 1.f / w, hi = lo + w * kSampThreads;
#pragma unroll 8  // 8 logit loads in flight per thread (a rolled loop waits one L2 latency per element)
      for (int i = tid; i < V; i += kSampThreads) {
        const float l = lg(i);
        if (l >= lo && l < hi) {
          const int bin = min(kSampThreads - 1, (int)((l - lo) * inv_w));
          atomicAdd(&hist8[bin * 8 + (tid & 7)], __expf(l - M));
        }
      }
      __syncthreads();
      {
        float h = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) h += hist8[tid * 8 + c];
        hist[tid] = h;
      }
      __syncthreads();
      for (int off = 1; off < kSampThreads; off <<= 1) {  // suffix sums: S[j] = mass(l >= lo + j w)
        const float v = tid + off < kSampThreads ? hist[tid + off] : 0.f;
        __syncthreads();
        hist[tid] += v;
        __syncthreads();
      }
      if (hist[tid] + above >= target) atomicMax(&jstar, tid);  // S is non-increasing: the last bin
      __syncthreads();
      const int j = jstar;
      above += j + 1 < kSampThreads ? hist[j + 1] : 0.f;
      lo += j * w;
      w *= 1.f / kSampThreads;
      __syncthreads();
    }
  } else {
    lo = -INFINITY;
  }
  const float cut = lo;
  const float it = 1.f / fmaxf(temp, 1e-6f);
  // contiguous chunk per thread for the ordered scan
  const int chunk = (V + kSampThreads - 1) / kSampThreads;
  const int b = tid * chunk, e = min(V, b + chunk);
  float part = 0.f;
#pragma unroll 8  // 8 logit loads in flight per thread (a rolled loop waits one L2 latency per element)
  for (int i = b; i < e; ++i) {
    const float l = lg(i);
    if (l >= cut) part += __expf((l - M) * it);
  }
  scan[tid] = part;
  __syncthreads();
  for (int off = 1; off < kSampThreads; off <<= 1) {  // Hillis-Steele inclusive scan
    const float v = tid >= off ? scan[tid - off] : 0.f;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  const float total = scan[kSampThreads - 1];
  const float u = (float)(uniform01(seed, (uint64_t)st[ST_STEP]) * total);
  const float before = tid ? scan[tid - 1] : 0.f;
  __shared__ int pick;
  if (tid == 0) pick = -1;
  __syncthreads();
  if (u >= before && u < scan[tid] && part > 0.f) {
    float run = before;
    int sel = -1;
#pragma unroll 8  // 8 logit loads in flight per thread (a rolled loop waits one L2 latency per element)
    for (int i = b; i < e; ++i) {
      const float l = lg(i);
      if (l < cut) continue;
      sel = i;
      run += __expf((l - M) * it);
      if (u < run) break;
    }
    pick = sel;
  }
  __syncthreads();
  if (tid == 0) {
    int t = pick;
    if (t < 0) {  // u landed on a rounding gap at the very top: take the most probable token
      for (int i = 0; i < V; ++i)
        if (lg(i) == M) { t = i; break; }
    }
    st[ST_TOK] = t;
    st[ST_POS] += inc_pos;
    st[ST_STEP] += 1;
    if (host_tok) __hip_atomic_store(host_tok, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The same sampler with the vocabulary held in registers (V <= 1024 * R): every pass reads the
// thread's R logits from VGPRs instead of re-reading the logit vector (the global-memory form
// above costs ~2.5 ns per logit per call: 82 us at V = 32000).  Thread t owns tokens t + 1024 k;
// the categorical draw walks the threads' masses in that fixed order, which is a different but
// equally valid order of the same distribution.
template <int R>
__global__ __launch_bounds__(kSampThreads) void k_sample_reg(const float* __restrict__ logits, int V,
                                                             const uint8_t* __restrict__ mask, float top_p,
                                                             float temp, uint64_t seed, int32_t* __restrict__ st,
                                                             int inc_pos, int32_t* host_tok) {
  __shared__ float sh[kSampThreads / 64];
  __shared__ float scan[kSampThreads];
  __shared__ float hist[kSampThreads];
  __shared__ float hist8[kSampThreads * 8];
  __shared__ int jstar, pick;
  const int tid = threadIdx.x;
  float v[R];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = tid + k * kSampThreads;
    v[k] = (i < V && !(mask && !mask[i])) ? logits[i] : -INFINITY;
    m = fmaxf(m, v[k]);
  }
  const float M = block_reduce(m, sh, true);
  float z = 0.f;
#pragma unroll
  for (int k = 0; k < R; ++k) z += __expf(v[k] - M);
  const float Z = block_reduce(z, sh, false);
  float lo = M - 40.f;  // nucleus cut: two levels of the replicated 1024-bin histogram (k_sample)
  if (top_p < 1.f) {
    const float target = top_p * Z;
    float w = 40.f / kSampThreads * (1.f + 1e-6f);
    float above = 0.f;
    for (int level = 0; level < 2; ++level) {
#pragma unroll
      for (int c = 0; c < 8; ++c) hist8[c * kSampThreads + tid] = 0.f;
      if (tid == 0) jstar = 0;
      __syncthreads();
      const float inv_w = 1.f / w, hi = lo + w * kSampThreads;
#pragma unroll
      for (int k = 0; k < R; ++k)
        if (v[k] >= lo && v[k] < hi)
          atomicAdd(&hist8[min(kSampThreads - 1, (int)((v[k] - lo) * inv_w)) * 8 + (tid & 7)], __expf(v[k] - M));
      __syncthreads();
      float h = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) h += hist8[tid * 8 + c];
      hist[tid] = h;
      __syncthreads();
      for (int off = 1; off < kSampThreads; off <<= 1) {
        const float x = tid + off < kSampThreads ? hist[tid + off] : 0.f;
        __syncthreads();
        hist[tid] += x;
        __syncthreads();
      }
      if (hist[tid] + above >= target) atomicMax(&jstar, tid);
      __syncthreads();
      const int j = jstar;
      above += j + 1 < kSampThreads ? hist[j + 1] : 0.f;
      lo += j * w;
      w *= 1.f / kSampThreads;
      __syncthreads();
    }
  } else {
    lo = -INFINITY;
  }
  const float cut = lo;
  const float it = 1.f / fmaxf(temp, 1e-6f);
  float part = 0.f;
#pragma unroll
  for (int k = 0; k < R; ++k)
    if (v[k] >= cut) part += __expf((v[k] - M) * it);
  scan[tid] = part;
  if (tid == 0) pick = 0x7fffffff;
  __syncthreads();
  for (int off = 1; off < kSampThreads; off <<= 1) {
    const float x = tid >= off ? scan[tid - off] : 0.f;
    __syncthreads();
    scan[tid] += x;
    __syncthreads();
  }
  const float total = scan[kSampThreads - 1];
  const float u = (float)(uniform01(seed, (uint64_t)st[ST_STEP]) * total);
  const float before = tid ? scan[tid - 1] : 0.f;
  if (u >= before && u < scan[tid] && part > 0.f) {
    float run = before;
    int sel = -1;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (sel < 0 && v[k] >= cut) {
        run += __expf((v[k] - M) * it);
        if (u < run) sel = tid + k * kSampThreads;
      }
    }
    if (sel < 0)  // rounding at the thread's upper edge: its last kept token
#pragma unroll
      for (int k = 0; k < R; ++k)
        if (v[k] >= cut) sel = tid + k * kSampThreads;
    atomicMin(&pick, sel);
  }
  __syncthreads();
  if (pick == 0x7fffffff) {  // u landed on a rounding gap at the very top: the most probable token
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (v[k] == M) atomicMin(&pick, tid + k * kSampThreads);
    __syncthreads();
  }
  if (tid == 0) {
    const int t = pick;
    st[ST_TOK] = t;
    st[ST_POS] += inc_pos;
    st[ST_STEP] += 1;
    if (host_tok) __hip_atomic_store(host_tok, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ------------------------------------------------------------------ multi-block sampler --
// The same sampler spread over kSbBlocks workgroups (one contiguous vocabulary slice each), as a
// chain of small kernels: a single workgroup is bound by one CU (61 us at V 32000, 255-275 us at
// V 128256).  Workspace layout (floats, caller-owned so the chain can be graph-captured):
constexpr int kSbBlocks = 64, kSbThreads = 256, kSbBins = 1024;
enum {
  SB_BMAX = 0,                          // [64] block max
  SB_BIDX = SB_BMAX + kSbBlocks,        // [64] first index of the block max (as int bits)
  SB_BZ = SB_BIDX + kSbBlocks,          // [64] block mass sum exp(l - M)
  SB_BPART = SB_BZ + kSbBlocks,         // [64] block kept mass (tempered)
  SB_SCAL = SB_BPART + kSbBlocks,       // [8]  M, Z, lo, w, above, cut
  SB_HIST = SB_SCAL + 8,                // [64][1024] per-block histograms
  SB_FLOATS = SB_HIST + kSbBlocks * kSbBins
};

__device__ __forceinline__ float sb_logit(const float* logits, const uint8_t* mask, int i) {
  return (mask && !mask[i]) ? -INFINITY : logits[i];
}

template <int NT>
__device__ float sb_reduce(float v, bool is_max) {
  __shared__ float sh[NT / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = is_max ? wave_max(v) : wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float r = sh[0];
  for (int w = 1; w < NT / 64; ++w) r = is_max ? fmaxf(r, sh[w]) : r + sh[w];
  return r;
}

// A: block max and its first index
__global__ __launch_bounds__(kSbThreads) void k_sb_max(const float* __restrict__ logits, int V,
                                                       const uint8_t* __restrict__ mask, float* __restrict__ ws) {
  const int chunk = (V + kSbBlocks - 1) / kSbBlocks, b0 = blockIdx.x * chunk, b1 = min(V, b0 + chunk);
  float m = -INFINITY;
  int mi = 0x7fffffff;
#pragma unroll 8
  for (int i = b0 + (int)threadIdx.x; i < b1; i += kSbThreads) {
    const float l = sb_logit(logits, mask, i);
    if (l > m) { m = l; mi = i; }
  }
  const float M = sb_reduce<kSbThreads>(m, true);
  __shared__ int first;
  if (threadIdx.x == 0) first = 0x7fffffff;
  __syncthreads();
  if (m == M) atomicMin(&first, mi);
  __syncthreads();
  if (threadIdx.x == 0) {
    ws[SB_BMAX + blockIdx.x] = M;
    ws[SB_BIDX + blockIdx.x] = __int_as_float(first);
  }
}

// B / D: block mass (level 0) and the mass histogram of [lo, lo + 1024 w) (replicated bins, k_sample)
template <int LEVEL>
__global__ __launch_bounds__(kSbThreads) void k_sb_hist(const float* __restrict__ logits, int V,
                                                        const uint8_t* __restrict__ mask, float* __restrict__ ws) {
  __shared__ float h8[kSbBins * 8];
  const int tid = threadIdx.x;
  float M, lo, w;
  if (LEVEL == 0) {
    float m = -INFINITY;
    for (int b = 0; b < kSbBlocks; ++b) m = fmaxf(m, ws[SB_BMAX + b]);
    M = m;
    lo = M - 40.f;
    w = 40.f / kSbBins * (1.f + 1e-6f);
  } else {
    M = ws[SB_SCAL + 0];
    lo = ws[SB_SCAL + 2];
    w = ws[SB_SCAL + 3];
  }
  for (int i = tid; i < kSbBins * 8; i += kSbThreads) h8[i] = 0.f;
  __syncthreads();
  const float inv_w = 1.f / w, hi = lo + w * kSbBins;
  const int chunk = (V + kSbBlocks - 1) / kSbBlocks, b0 = blockIdx.x * chunk, b1 = min(V, b0 + chunk);
  float z = 0.f;
#pragma unroll 8
  for (int i = b0 + tid; i < b1; i += kSbThreads) {
    const float l = sb_logit(logits, mask, i);
    const float e = __expf(l - M);
    if (LEVEL == 0) z += e;
    if (l >= lo && l < hi) atomicAdd(&h8[min(kSbBins - 1, (int)((l - lo) * inv_w)) * 8 + (tid & 7)], e);
  }
  if (LEVEL == 0) {
    z = sb_reduce<kSbThreads>(z, false);
    if (tid == 0) ws[SB_BZ + blockIdx.x] = z;
  }
  __syncthreads();
  float* out = ws + SB_HIST + (long)blockIdx.x * kSbBins;
  for (int t = tid; t < kSbBins; t += kSbThreads) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) v += h8[t * 8 + c];
    out[t] = v;
  }
}

// C / E: one workgroup of 1024 threads sums the block histograms, finds the bin where the suffix
// mass crosses top_p Z and narrows [lo, lo + 1024 w) to it (level 1: the cut)
template <int LEVEL>
__global__ __launch_bounds__(kSbBins) void k_sb_select(float top_p, float* __restrict__ ws) {
  __shared__ float hs[kSbBins];
  __shared__ int jstar;
  const int tid = threadIdx.x;
  float M, Z, lo, w, above;
  if (LEVEL == 0) {
    float m = -INFINITY;
    for (int b = 0; b < kSbBlocks; ++b) m = fmaxf(m, ws[SB_BMAX + b]);
    M = m;
    Z = 0.f;
    for (int b = 0; b < kSbBlocks; ++b) Z += ws[SB_BZ + b];
    lo = M - 40.f;
    w = 40.f / kSbBins * (1.f + 1e-6f);
    above = 0.f;
  } else {
    M = ws[SB_SCAL + 0]; Z = ws[SB_SCAL + 1]; lo = ws[SB_SCAL + 2]; w = ws[SB_SCAL + 3]; above = ws[SB_SCAL + 4];
  }
  float h = 0.f;
  for (int b = 0; b < kSbBlocks; ++b) h += ws[SB_HIST + (long)b * kSbBins + tid];
  hs[tid] = h;
  if (tid == 0) jstar = 0;
  __syncthreads();
  for (int off = 1; off < kSbBins; off <<= 1) {  // suffix sums
    const float x = tid + off < kSbBins ? hs[tid + off] : 0.f;
    __syncthreads();
    hs[tid] += x;
    __syncthreads();
  }
  if (hs[tid] + above >= top_p * Z) atomicMax(&jstar, tid);
  __syncthreads();
  if (tid == 0) {
    const int j = jstar;
    ws[SB_SCAL + 0] = M;
    ws[SB_SCAL + 1] = Z;
    ws[SB_SCAL + 4] = above + (j + 1 < kSbBins ? hs[j + 1] : 0.f);
    ws[SB_SCAL + 2] = lo + j * w;
    ws[SB_SCAL + 3] = w * (1.f / kSbBins);
    ws[SB_SCAL + 5] = lo + j * w;  // the cut after the last level
  }
}

// F: kept (tempered) mass per block; with top_p >= 1 the cut is -inf and M comes from the maxima
__global__ __launch_bounds__(kSbThreads) void k_sb_part(const float* __restrict__ logits, int V,
                                                        const uint8_t* __restrict__ mask, float temp, int nucleus,
                                                        float* __restrict__ ws) {
  float M, cut;
  if (nucleus) {
    M = ws[SB_SCAL + 0];
    cut = ws[SB_SCAL + 5];
  } else {
    float m = -INFINITY;
    for (int b = 0; b < kSbBlocks; ++b) m = fmaxf(m, ws[SB_BMAX + b]);
    M = m;
    cut = -INFINITY;
    if (blockIdx.x == 0 && threadIdx.x == 0) { ws[SB_SCAL + 0] = M; ws[SB_SCAL + 5] = cut; }
  }
  const float it = 1.f / fmaxf(temp, 1e-6f);
  const int chunk = (V + kSbBlocks - 1) / kSbBlocks, b0 = blockIdx.x * chunk, b1 = min(V, b0 + chunk);
  float part = 0.f;
#pragma unroll 8
  for (int i = b0 + (int)threadIdx.x; i < b1; i += kSbThreads) {
    const float l = sb_logit(logits, mask, i);
    if (l >= cut) part += __expf((l - M) * it);
  }
  part = sb_reduce<kSbThreads>(part, false);
  if (threadIdx.x == 0) ws[SB_BPART + blockIdx.x] = part;
}

// G: the draw -- the block whose prefix range holds u, then inside its slice (thread t owns the
// contiguous elements [t c, t c + c)) the token; state update as k_sample
__global__ __launch_bounds__(kSbBins) void k_sb_draw(const float* __restrict__ logits, int V,
                                                     const uint8_t* __restrict__ mask, float temp, uint64_t seed,
                                                     const float* __restrict__ ws, int32_t* __restrict__ st,
                                                     int inc_pos, int32_t* host_tok) {
  __shared__ float scan[kSbBins];
  __shared__ int pick;
  __shared__ float base_u;
  __shared__ int blk;
  const int tid = threadIdx.x;
  const float M = ws[SB_SCAL + 0], cut = ws[SB_SCAL + 5];
  const float it = 1.f / fmaxf(temp, 1e-6f);
  if (tid == 0) {
    double total = 0.0;
    for (int b = 0; b < kSbBlocks; ++b) total += ws[SB_BPART + b];
    const double u = uniform01(seed, (uint64_t)st[ST_STEP]) * total;
    double run = 0.0;
    int bb = -1;
    for (int b = 0; b < kSbBlocks; ++b) {
      const double p = ws[SB_BPART + b];
      if (p > 0.0) {
        if (u < run + p) { bb = b; break; }
        bb = b;  // rounding at the very end: the last block with mass
      }
      run += p;
    }
    if (bb >= 0 && u >= run + ws[SB_BPART + bb]) run -= ws[SB_BPART + bb];
    blk = bb;
    base_u = (float)(u - run);
    pick = 0x7fffffff;
  }
  __syncthreads();
  const int chunk = (V + kSbBlocks - 1) / kSbBlocks;
  if (blk >= 0) {
    const int b0 = blk * chunk, b1 = min(V, b0 + chunk);
    const int per = (b1 - b0 + kSbBins - 1) / kSbBins;
    const int t0 = b0 + tid * per, t1 = min(b1, t0 + per);
    float part = 0.f;
    for (int i = t0; i < t1; ++i) {
      const float l = sb_logit(logits, mask, i);
      if (l >= cut) part += __expf((l - M) * it);
    }
    scan[tid] = part;
    __syncthreads();
    for (int off = 1; off < kSbBins; off <<= 1) {
      const float x = tid >= off ? scan[tid - off] : 0.f;
      __syncthreads();
      scan[tid] += x;
      __syncthreads();
    }
    const float u = base_u, before = tid ? scan[tid - 1] : 0.f;
    if (part > 0.f && u >= before && (u < scan[tid] || tid == kSbBins - 1 || scan[tid] >= scan[kSbBins - 1])) {
      float run = before;
      int sel = -1;
      for (int i = t0; i < t1; ++i) {
        const float l = sb_logit(logits, mask, i);
        if (l < cut) continue;
        sel = i;
        run += __expf((l - M) * it);
        if (u < run) break;
      }
      if (sel >= 0) atomicMin(&pick, sel);
    }
    __syncthreads();
  }
  if (tid == 0) {
    int t = pick;
    if (t == 0x7fffffff) {  // rounding gap: the most probable token (first block holding the max)
      for (int b = 0; b < kSbBlocks; ++b)
        if (ws[SB_BMAX + b] == M) { t = __float_as_int(ws[SB_BIDX + b]); break; }
    }
    st[ST_TOK] = t;
    st[ST_POS] += inc_pos;
    st[ST_STEP] += 1;
    if (host_tok) __hip_atomic_store(host_tok, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ------------------------------------------------------- prefill attention over the KV cache --
// Causal grouped-query attention of a prompt chunk of n tokens at absolute positions pos0 ..
// pos0+n-1 against the KV cache rows 0 .. pos0+n-1 (the chunk's own k/v already appended): the
// first prompt (pos0 = 0) and every continuation (a new turn over a live cache) alike, for head
// dims 64 and 128 (llama 1B-class and 7B-class).  One 256-thread workgroup = 128 query rows of
// one q head, 4 waves x 2 16-row q-blocks; per 64-key tile (LDS double buffer, register-staged
// one tile ahead):
//   S^T = K Q^T    mfma_f32_16x16x32_bf16 with the K rows as the A operand, so one query's
//                  scores sit in one lane column and the softmax statistics reduce in-lane plus
//                  two permlane swaps;
//   O^T += V^T P^T the rounded probabilities are the B operand as they lie; V^T fragments come
//                  from the row-major V tile through ds_read_b64_tr_b16.
// The K tile's 16-B chunks are XOR-swizzled by the key (mod HD/8 chunks) so a 16-lane group's
// b128 reads of 16 key rows cover all 64 banks; V chunks swap bits 1..2 by key pair for the
// transposing reads.  Grid: nqb * heads blocks through the bijective XCD remap, so the q-blocks
// of one head (which stream the same K/V) share one XCD's L2.
typedef __bf16 pa_bf16x8 __attribute__((ext_vector_type(8)));
typedef float pa_f32x4 __attribute__((ext_vector_type(4)));
typedef float pa_f32x2 __attribute__((ext_vector_type(2)));
typedef short pa_v4i16 __attribute__((ext_vector_type(4)));
typedef short pa_v8i16 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) pa_v4i16 pa_lds_v4i16;

__device__ __forceinline__ float pa_xg_max(float x) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
__device__ __forceinline__ float pa_xg_sum(float x) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

template <int HD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_prefill_attn(const uint16_t* __restrict__ qg, long ldq,
                                                      const uint16_t* __restrict__ kc,
                                                      const uint16_t* __restrict__ vc, long ldkv, int n, int pos0,
                                                      int heads, int kv_heads, float scale_log2,
                                                      uint16_t* __restrict__ out, long ldo) {
  constexpr int KT = HD == 128 ? 32 : 64, RB = HD * 2, NCH = HD / 8, NKK = HD / 32, NDB = HD / 16, NL = KT * NCH / 256;
  __shared__ __attribute__((aligned(16))) char lds[2][2][KT * RB];  // [buf][K | V][key * RB]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const int nwg = gridDim.x, orig = blockIdx.x, q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int nqb = nwg / heads, head = lid / nqb, qstart = (lid - head * nqb) * 128;
  const int kvhead = head / (heads / kv_heads);
  const long lenk = (long)pos0 + n;
  auto ksw = [](int key, int c) { return c ^ (key & (NCH - 1)); };
  auto vsw = [](int key, int c) { return c ^ (((key >> 1) & 3) << 1); };

  pa_bf16x8 qf[2][NKK];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qrow = qstart + wave * 32 + qb * 16 + li;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk)
      qf[qb][kk] = qrow < n ? *(const pa_bf16x8*)(qg + (long)qrow * ldq + head * HD + kk * 32 + g * 8) : pa_bf16x8{};
  }
  pa_f32x4 o[NDB][2];
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) o[db][qb] = pa_f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-1e30f, -1e30f}, l[2] = {0.f, 0.f};

  uint4 rk[NL], rv[NL];
  const uint16_t* kp = kc + (long)kvhead * HD;
  const uint16_t* vp = vc + (long)kvhead * HD;
  auto gload = [&](long k0) {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int c = tid + it * 256, key = c / NCH, ch = c % NCH;
      if (k0 + key < lenk) {
        rk[it] = *(const uint4*)(kp + (k0 + key) * ldkv + ch * 8);
        rv[it] = *(const uint4*)(vp + (k0 + key) * ldkv + ch * 8);
      } else {
        rk[it] = make_uint4(0, 0, 0, 0);
        rv[it] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lwrite = [&](int buf) {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int c = tid + it * 256, key = c / NCH, ch = c % NCH;
      *(uint4*)(lds[buf][0] + key * RB + (ksw(key, ch) << 4)) = rk[it];
      *(uint4*)(lds[buf][1] + key * RB + (vsw(key, ch) << 4)) = rv[it];
    }
  };

  // causal: the block's last query (absolute pos0 + qstart + 127) bounds the key tiles
  const int ntiles = (int)min((lenk + KT - 1) / KT, ((long)pos0 + qstart + 128 + KT - 1) / KT);
  gload(0);
  lwrite(0);
  __syncthreads();
  const int tq = li >> 2, tp = li & 3;
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const long k0 = (long)t * KT;
    if (t + 1 < ntiles) gload(k0 + KT);
    const char* Ks = lds[buf][0];
    const char* Vs = lds[buf][1];
    pa_f32x4 s[KT / 16][2];
#pragma unroll
    for (int kb = 0; kb < KT / 16; ++kb) {
      const int row = kb * 16 + li;
      pa_bf16x8 kf[NKK];
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) kf[kk] = *(const pa_bf16x8*)(Ks + row * RB + (ksw(row, kk * 4 + g) << 4));
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        s[kb][qb] = pa_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk)
          s[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kk], qf[qb][kk], s[kb][qb], 0, 0, 0);
      }
    }
    // online softmax with the deferred rescale (max moves only past a 2^8 margin); keys after a
    // query's absolute position are masked on the diagonal tiles, which also covers the keys
    // past the cache length for every stored row
    constexpr float kThr = 8.f;
    const bool diag = k0 + KT - 1 > (long)pos0 + qstart + wave * 32;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      if (diag) {
        const long qabs = (long)pos0 + qstart + wave * 32 + qb * 16 + li;
#pragma unroll
        for (int kb = 0; kb < KT / 16; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (k0 + kb * 16 + 4 * g + r > qabs) s[kb][qb][r] = -1e30f;
      }
      float mx = -1e30f;
#pragma unroll
      for (int kb = 0; kb < KT / 16; ++kb)
        mx = fmaxf(fmaxf(mx, fmaxf(s[kb][qb][0], s[kb][qb][1])), fmaxf(s[kb][qb][2], s[kb][qb][3]));
      const float mxs = pa_xg_max(mx) * scale_log2;
      if (!__all(mxs - m[qb] <= kThr)) {
        const float mn = fmaxf(m[qb], mxs);
        const float alpha = __builtin_amdgcn_exp2f(m[qb] - mn);
        m[qb] = mn;
        l[qb] *= alpha;
#pragma unroll
        for (int db = 0; db < NDB; ++db) o[db][qb] *= alpha;
      }
      const pa_f32x2 sc2 = {scale_log2, scale_log2}, nm2 = {-m[qb], -m[qb]};
      pa_f32x2 acc2 = {0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < KT / 16; ++kb)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          pa_f32x2 x = {s[kb][qb][2 * h], s[kb][qb][2 * h + 1]};
          x = x * sc2 + nm2;
          x.x = __builtin_amdgcn_exp2f(x.x);
          x.y = __builtin_amdgcn_exp2f(x.y);
          s[kb][qb][2 * h] = x.x;
          s[kb][qb][2 * h + 1] = x.y;
          acc2 += x;
        }
      l[qb] += pa_xg_sum(acc2.x + acc2.y);
    }
#pragma unroll
    for (int st = 0; st < KT / 32; ++st) {
      pa_bf16x8 pf[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[qb][j] = (__bf16)s[2 * st][qb][j];
          pf[qb][4 + j] = (__bf16)s[2 * st + 1][qb][j];
        }
      const int row1 = st * 32 + 4 * g + tq, row2 = row1 + 16;
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        const int ch = db * 2 + (tp >> 1);
        const pa_v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (pa_lds_v4i16*)(Vs + row1 * RB + (vsw(row1, ch) << 4) + 8 * (tp & 1)));
        const pa_v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (pa_lds_v4i16*)(Vs + row2 * RB + (vsw(row2, ch) << 4) + 8 * (tp & 1)));
        const pa_bf16x8 vf = __builtin_bit_cast(pa_bf16x8, (pa_v8i16)__builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
          o[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qb], o[db][qb], 0, 0, 0);
      }
    }
    if (t + 1 < ntiles) lwrite(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qrow = qstart + wave * 32 + qb * 16 + li;
    if (qrow >= n) continue;
    const float inv = 1.f / l[qb];
    uint16_t* dst = out + (long)qrow * ldo + head * HD + 4 * g;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      uint2 w;
      w.x = pk2(o[db][qb][0] * inv, o[db][qb][1] * inv);
      w.y = pk2(o[db][qb][2] * inv, o[db][qb][3] * inv);
      *(uint2*)(dst + db * 16) = w;
    }
  }
}

}  // namespace

extern "C" {

// Causal prefill attention over the KV cache (k_prefill_attn): q rows [n, ldq] (H heads x hd,
// RoPE applied), k / v cache rows [pos0 + n, ldkv] (KVH heads x hd; rows pos0 .. pos0+n-1 are
// this chunk's), out rows [n, ldo].  hd 64 or 128; rows and bases 16-B aligned.
int dec_attn_prefill_kv(const void* q, long ldq, const void* k, const void* v, long ldkv, int n, int pos0, int H,
                        int KVH, int hd, float scale, void* out, long ldo, hipStream_t s) {
  if (n <= 0) return 0;
  if (pos0 < 0 || H <= 0 || KVH <= 0 || H % KVH || (hd != 64 && hd != 128) || ldq % 8 || ldkv % 8 || ldo % 8 ||
      ldq < (long)H * hd || ldkv < (long)KVH * hd || ldo < (long)H * hd ||
      ((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)out) & 15)
    return (int)hipErrorInvalidValue;
  const int nqb = (n + 127) / 128;
  const float sl2 = scale * 1.4426950408889634f;
  if (hd == 64)
    hipLaunchKernelGGL(k_prefill_attn<64>, dim3(nqb * H), dim3(256), 0, s, (const uint16_t*)q, ldq,
                       (const uint16_t*)k, (const uint16_t*)v, ldkv, n, pos0, H, KVH, sl2, (uint16_t*)out, ldo);
  else
    hipLaunchKernelGGL(k_prefill_attn<128>, dim3(nqb * H), dim3(256), 0, s, (const uint16_t*)q, ldq,
                       (const uint16_t*)k, (const uint16_t*)v, ldkv, n, pos0, H, KVH, sl2, (uint16_t*)out, ldo);
  return (int)hipGetLastError();
}

// q: bf16 [H*hd] (one token, RoPE applied); k/v: bf16 cache rows [L, ldkv] (ldkv = KVH*hd);
// out: bf16 [H*hd].  hd in {64, 128, 192, 256}, H % KVH == 0, L >= 1, 16-B aligned rows.
int dec_attn_decode_st(const void* q, const void* k, const void* v, long ldkv, int L, int H, int KVH, int hd,
                       float scale, void* out, const int32_t* st, hipStream_t s);
int dec_attn_decode(const void* q, const void* k, const void* v, long ldkv, int L, int H, int KVH, int hd,
                    float scale, void* out, hipStream_t s) {
  return dec_attn_decode_st(q, k, v, ldkv, L, H, KVH, hd, scale, out, nullptr, s);
}

// as dec_attn_decode; with st != null the cache length is st[0] + 1 (L is ignored)
// split-L workspace, one per stream (the decode step's layers run in order on one stream): H <= 128
// heads x kMaxSplits partials of hd + 2 floats, allocated on first use (outside graph capture: the
// decode engine runs one step eagerly before capturing)
static float* split_workspace(hipStream_t s) {
  static std::mutex mu;
  static std::map<hipStream_t, float*> table;
  std::lock_guard<std::mutex> g(mu);
  auto it = table.find(s);
  if (it != table.end()) return it->second;
  float* w = nullptr;
  if (hipMalloc((void**)&w, (size_t)128 * kMaxSplits * (256 + 2) * sizeof(float)) != hipSuccess) return nullptr;
  return table[s] = w;
}

// splits for a cache of (up to) L keys: the single-workgroup kernel up to 512 keys, then one split per
// 256 keys, at most kMaxSplits (sweep over 4..32 splits at H 32 / KVH 8 / hd 128:
// profiles/r2_decode_splits.jsonl)
static int decode_splits(int L) {
  static const int env = [] {
    const char* e = getenv("SPL_DEC_SPLITS");
    return e && *e ? atoi(e) : -1;
  }();
  if (env >= 1) return env < kMaxSplits ? env : kMaxSplits;
  if (L <= 512) return 1;
  const int sp = (L + 255) / 256;
  return sp > kMaxSplits ? kMaxSplits : sp;
}

int dec_attn_decode_ws(const void* q, const void* k, const void* v, long ldkv, int L, int H, int KVH, int hd,
                       float scale, void* out, const int32_t* st, float* ws, hipStream_t s);
int dec_attn_decode_st(const void* q, const void* k, const void* v, long ldkv, int L, int H, int KVH, int hd,
                       float scale, void* out, const int32_t* st, hipStream_t s) {
  return dec_attn_decode_ws(q, k, v, ldkv, L, H, KVH, hd, scale, out, st, nullptr, s);
}

// dec_attn_decode_st with a caller-owned split workspace ws (H * 32 * (hd + 2) floats; null: a
// per-stream one allocated on first use -- a graph-captured step must pass its own, since nothing
// may be allocated during capture)
int dec_attn_decode_ws(const void* q, const void* k, const void* v, long ldkv, int L, int H, int KVH, int hd,
                       float scale, void* out, const int32_t* st, float* ws, hipStream_t s) {
  // with st, L is the cache CAPACITY (sizes the split count; the length itself is read on the device)
  if (L <= 0 || H <= 0 || KVH <= 0 || H % KVH || hd <= 0 || hd % 64 || hd > 256 || ldkv % 8 ||
      ldkv < (long)KVH * hd || ((uintptr_t)k | (uintptr_t)v) % 16)
    return (int)hipErrorInvalidValue;
  const int grp = H / KVH;
  const int S = decode_splits(L);
  // SPL_DEC_SMALL: caches of at most kSmallL keys on the grouped three-phase kernel, and the splits of longer
  // ones on its split form (chunks of at most kSmallL keys); 0 = the per-head / per-group walking kernels
  static const int small = [] {
    const char* e = getenv("SPL_DEC_SMALL");
    return e && *e ? atoi(e) : 1;
  }();
  const bool grouped = small && (hd == 64 || hd == 128 || hd == 256) && (grp == 1 || grp == 2 || grp == 4 || grp == 8);
  if (S > 1 && H <= 128) {
    if (!ws) ws = split_workspace(s);
    if (!ws) return (int)hipErrorOutOfMemory;
    if (grouped && ((L + S - 1) / S + 63) / 64 * 64 <= kSmallL) {
      const uint16_t *qq = (const uint16_t*)q, *kk = (const uint16_t*)k, *vv = (const uint16_t*)v;
      const dim3 gg((unsigned)KVH, (unsigned)S), bb(256);
#define GSPLIT(D_, G_) hipLaunchKernelGGL((k_attn_decode_g<D_, G_, true>), gg, bb, 0, s, qq, kk, vv, ldkv, L, scale, \
                                          (uint16_t*)nullptr, st, ws)
#define GSPLIT_G(D_) switch (grp) { case 1: GSPLIT(D_, 1); break; case 2: GSPLIT(D_, 2); break; \
                                    case 4: GSPLIT(D_, 4); break; default: GSPLIT(D_, 8); break; }
      switch (hd) {
        case 64: GSPLIT_G(1); break;
        case 128: GSPLIT_G(2); break;
        default: GSPLIT_G(4); break;
      }
#undef GSPLIT_G
#undef GSPLIT
      hipLaunchKernelGGL(k_attn_combine, dim3((unsigned)H), dim3(256), 0, s, ws, S, hd, (uint16_t*)out);
      return (int)hipGetLastError();
    }
    // heads per workgroup: the whole kv group when it is 2, 4 or 8 heads (shared K/V rows), else 1
    const int G = (grp == 2 || grp == 4 || grp == 8) ? grp : 1;
    const dim3 gs((unsigned)(H / G), (unsigned)S), bs(kSplitWaves * 64);
    const uint16_t *qq = (const uint16_t*)q, *kk = (const uint16_t*)k, *vv = (const uint16_t*)v;
#define SPLIT(D_, G_) hipLaunchKernelGGL((k_attn_decode_split<D_, G_>), gs, bs, 0, s, qq, kk, vv, ldkv, L, grp, scale, ws, st)
#define SPLIT_G(D_) switch (G) { case 2: SPLIT(D_, 2); break; case 4: SPLIT(D_, 4); break; \
                                 case 8: SPLIT(D_, 8); break; default: SPLIT(D_, 1); break; }
    switch (hd / 64) {
      case 1: SPLIT_G(1); break;
      case 2: SPLIT_G(2); break;
      case 3: SPLIT_G(3); break;
      default: SPLIT_G(4); break;
    }
#undef SPLIT_G
#undef SPLIT
    hipLaunchKernelGGL(k_attn_combine, dim3((unsigned)H), dim3(256), 0, s, ws, S, hd, (uint16_t*)out);
    return (int)hipGetLastError();
  }
  const uint16_t *qq = (const uint16_t*)q, *kk = (const uint16_t*)k, *vv = (const uint16_t*)v;
  uint16_t* oo = (uint16_t*)out;
  if (grouped && L <= kSmallL) {
    const dim3 gg((unsigned)KVH), bb(256);
#define SMALL(D_, G_) hipLaunchKernelGGL((k_attn_decode_g<D_, G_>), gg, bb, 0, s, qq, kk, vv, ldkv, L, scale, oo, st, \
                                         (float*)nullptr)
#define SMALL_G(D_) switch (grp) { case 1: SMALL(D_, 1); break; case 2: SMALL(D_, 2); break; \
                                   case 4: SMALL(D_, 4); break; default: SMALL(D_, 8); break; }
    switch (hd) {
      case 64: SMALL_G(1); break;
      case 128: SMALL_G(2); break;
      default: SMALL_G(4); break;
    }
#undef SMALL_G
#undef SMALL
    return (int)hipGetLastError();
  }
  const dim3 g((unsigned)H), b(kDecWaves * 64);
  switch (hd / 64) {
    case 1: hipLaunchKernelGGL(k_attn_decode<1>, g, b, 0, s, qq, kk, vv, ldkv, L, grp, hd, scale, oo, st); break;
    case 2: hipLaunchKernelGGL(k_attn_decode<2>, g, b, 0, s, qq, kk, vv, ldkv, L, grp, hd, scale, oo, st); break;
    case 3: hipLaunchKernelGGL(k_attn_decode<3>, g, b, 0, s, qq, kk, vv, ldkv, L, grp, hd, scale, oo, st); break;
    default: hipLaunchKernelGGL(k_attn_decode<4>, g, b, 0, s, qq, kk, vv, ldkv, L, grp, hd, scale, oo, st); break;
  }
  return (int)hipGetLastError();
}

// x/out: bf16 rows (strides in elements), w: fp32 [d]; d % 8 == 0, 16-B aligned rows.
int dec_rmsnorm(const void* x, long ldx, const float* w, long T, int d, float eps, void* out, long ldo,
                hipStream_t s) {
  if (T <= 0) return 0;
  if (d <= 0 || d % 8 || ldx % 8 || ldo % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rmsnorm, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s, (const uint16_t*)x, ldx, w, T, d, eps,
                     (uint16_t*)out, ldo);
  return (int)hipGetLastError();
}

// qkv: bf16 [T, ld]; columns [0, ncols) hold q|k heads of width hd; row t has position pos0 + t;
// cos/sin: fp32 [n_ctx, hd/2] (the caller guarantees pos0 + T <= n_ctx).
int dec_rope(void* qkv, long ld, long T, int ncols, int hd, int pos0, const float* cos_tab, const float* sin_tab,
             hipStream_t s) {
  if (T <= 0) return 0;
  if (hd % 8 || ncols % hd || ld % 8 || pos0 < 0) return (int)hipErrorInvalidValue;
  const long work = T * (ncols / 8);
  long g = (work + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(k_rope, dim3((unsigned)g), dim3(256), 0, s, (uint16_t*)qkv, ld, T, ncols, hd, pos0, cos_tab,
                     sin_tab);
  return (int)hipGetLastError();
}

// y = x . W^T for one token (see k_gemv).  mode 0 store, 1 residual, 2 SwiGLU (N = packed rows,
// out has N / 2), 4 fp32; rms_w != null: x is RMS-normalised with rms_w / eps first.
// K % 8 == 0, K <= 16384, 16-B aligned W / x.
int dec_gemv(int mode, const void* x, const float* rms_w, float eps, const void* W, int N, int K, const void* res,
             void* out, hipStream_t s) {
  if (K <= 0 || K % 8 || K > kGemvMaxK || N <= 0 || (mode == 2 && N % 32) || (mode == 1 && !res) ||
      ((uintptr_t)W | (uintptr_t)x) % 16)
    return (int)hipErrorInvalidValue;
  const int nout = mode == 2 ? N / 2 : N;
  const int per_block = 4 * (mode == 2 ? kGemvRows / 2 : kGemvRows);
  const dim3 g((unsigned)((nout + per_block - 1) / per_block)), b(256);
  const uint16_t *xx = (const uint16_t*)x, *ww = (const uint16_t*)W, *rr = (const uint16_t*)res;
#define GEMV(M_, R_) hipLaunchKernelGGL((k_gemv<M_, R_>), g, b, 0, s, xx, rms_w, eps, ww, K, nout, rr, out)
  const bool rms = rms_w != nullptr;
  switch (mode) {
    case 0: if (rms) GEMV(0, true); else GEMV(0, false); break;
    case 1: if (rms) GEMV(1, true); else GEMV(1, false); break;
    case 2: if (rms) GEMV(2, true); else GEMV(2, false); break;
    case 4: if (rms) GEMV(4, true); else GEMV(4, false); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef GEMV
  return (int)hipGetLastError();
}

// dec_gemv over Q4G32 weights (k_gemv_q4): Wq [N, K/2] nibbles, Wsm [N, K/32] bf16 (d, m) pairs.
// K % 32 == 0, K <= 16384, 16-B aligned x / Wq, 4-B aligned Wsm.
}  // extern "C"

template <int BITS>
static int gemv_qn(int mode, const void* x, const float* rms_w, float eps, const void* Wq, const void* Wsm, int N,
                   int K, const void* res, void* out, hipStream_t s) {
  if (K <= 0 || K % kQ4Group || K > kGemvQ4MaxK || N <= 0 || (mode == 2 && N % 32) || (mode == 1 && !res) ||
      ((uintptr_t)Wq | (uintptr_t)x) % 16 || (uintptr_t)Wsm % 4 || (rms_w && (uintptr_t)rms_w % 16))
    return (int)hipErrorInvalidValue;
  // rows per wave: 4, or 8 with SPL_Q4_ROWS=8 (A/B knob: more bytes in flight per wave, half the blocks)
  static const int R = [] {
    const char* e = getenv("SPL_Q4_ROWS");
    return e && atoi(e) == 8 ? 8 : 4;
  }();
  const int nout = mode == 2 ? N / 2 : N;
  const int per_block = 4 * (mode == 2 ? R / 2 : R);
  const dim3 g((unsigned)((nout + per_block - 1) / per_block)), b(256);
  const size_t lds = (size_t)(K / kQ4Group) * kQ4Rec * sizeof(float);
  const uint16_t *xx = (const uint16_t*)x, *rr = (const uint16_t*)res;
  const uint8_t* wq = (const uint8_t*)Wq;
  const uint32_t* wsm = (const uint32_t*)Wsm;
#define GEMV(M_, R_)                                                                                           \
  do {                                                                                                         \
    if (R == 8) hipLaunchKernelGGL((k_gemv_q4<M_, R_, 8, BITS>), g, b, lds, s, xx, rms_w, eps, wq, wsm, K, nout, rr, out); \
    else hipLaunchKernelGGL((k_gemv_q4<M_, R_, 4, BITS>), g, b, lds, s, xx, rms_w, eps, wq, wsm, K, nout, rr, out);      \
  } while (0)
  const bool rms = rms_w != nullptr;
  switch (mode) {
    case 0: if (rms) GEMV(0, true); else GEMV(0, false); break;
    case 1: if (rms) GEMV(1, true); else GEMV(1, false); break;
    case 2: if (rms) GEMV(2, true); else GEMV(2, false); break;
    case 4: if (rms) GEMV(4, true); else GEMV(4, false); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef GEMV
  return (int)hipGetLastError();
}

extern "C" {

int dec_gemv_q4(int mode, const void* x, const float* rms_w, float eps, const void* Wq, const void* Wsm, int N,
                int K, const void* res, void* out, hipStream_t s) {
  return gemv_qn<4>(mode, x, rms_w, eps, Wq, Wsm, N, K, res, out, s);
}

// dec_gemv over Q8G32 weights: Wq [N, K] bytes, Wsm [N, K/32] bf16 (d, m) pairs, w = d u + m
int dec_gemv_q8(int mode, const void* x, const float* rms_w, float eps, const void* Wq, const void* Wsm, int N,
                int K, const void* res, void* out, hipStream_t s) {
  return gemv_qn<8>(mode, x, rms_w, eps, Wq, Wsm, N, K, res, out, s);
}

// bf16 W [N, K] (row-major, contiguous) <-> Q8G32 planes
int dec_q8_quantize(const void* W, long N, int K, void* Wq, void* Wsm, hipStream_t s) {
  if (N <= 0 || K <= 0 || K % kQ4Group || ((uintptr_t)W | (uintptr_t)Wq) % 16 || (uintptr_t)Wsm % 4)
    return (int)hipErrorInvalidValue;
  const long groups = N * (K / kQ4Group);
  hipLaunchKernelGGL(k_q8_quant, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, (const uint16_t*)W, groups,
                     (uint8_t*)Wq, (uint32_t*)Wsm);
  return (int)hipGetLastError();
}

int dec_q8_dequant(const void* Wq, const void* Wsm, long N, int K, void* W, hipStream_t s) {
  if (N <= 0 || K <= 0 || K % kQ4Group || ((uintptr_t)W | (uintptr_t)Wq) % 16 || (uintptr_t)Wsm % 4)
    return (int)hipErrorInvalidValue;
  const long groups = N * (K / kQ4Group);
  hipLaunchKernelGGL(k_q8_dequant, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, (const uint8_t*)Wq,
                     (const uint32_t*)Wsm, groups, (uint16_t*)W);
  return (int)hipGetLastError();
}

// bf16 W [N, K] (row-major, contiguous) <-> Q4G32 planes
int dec_q4_quantize(const void* W, long N, int K, void* Wq, void* Wsm, hipStream_t s) {
  if (N <= 0 || K <= 0 || K % kQ4Group || ((uintptr_t)W | (uintptr_t)Wq) % 16 || (uintptr_t)Wsm % 4)
    return (int)hipErrorInvalidValue;
  const long groups = N * (K / kQ4Group);
  hipLaunchKernelGGL(k_q4_quant, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, (const uint16_t*)W, groups,
                     K / kQ4Group, (uint8_t*)Wq, (uint32_t*)Wsm);
  return (int)hipGetLastError();
}

int dec_q4_dequant(const void* Wq, const void* Wsm, long N, int K, void* W, hipStream_t s) {
  if (N <= 0 || K <= 0 || K % kQ4Group || ((uintptr_t)W | (uintptr_t)Wq) % 16 || (uintptr_t)Wsm % 4)
    return (int)hipErrorInvalidValue;
  const long groups = N * (K / kQ4Group);
  hipLaunchKernelGGL(k_q4_dequant, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, (const uint8_t*)Wq,
                     (const uint32_t*)Wsm, groups, (uint16_t*)W);
  return (int)hipGetLastError();
}

int dec_embed_tok(const void* emb, int d, const int32_t* st, void* x, hipStream_t s) {
  if (d % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_embed_tok, dim3(1), dim3(256), 0, s, (const uint16_t*)emb, d, st, (uint16_t*)x);
  return (int)hipGetLastError();
}

// qkv: bf16 [(H + 2 KVH) hd] of the step's token; kc / vc: the layer's cache [n_ctx, ldkv]
int dec_rope_kv(void* qkv, int H, int KVH, int hd, const float* cos_tab, const float* sin_tab, const int32_t* st,
                void* kc, void* vc, long ldkv, hipStream_t s) {
  if (hd % 2 || H <= 0 || KVH <= 0 || ldkv < (long)KVH * hd) return (int)hipErrorInvalidValue;
  const int work = (H + KVH) * hd / 2 + KVH * hd;
  hipLaunchKernelGGL(k_rope_kv, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, (uint16_t*)qkv, H, KVH, hd,
                     cos_tab, sin_tab, st, (uint16_t*)kc, (uint16_t*)vc, ldkv);
  return (int)hipGetLastError();
}

// floats of the workspace dec_sample_ws needs
long dec_sample_ws_floats() { return SB_FLOATS; }

// dec_sample with a caller-owned workspace (dec_sample_ws_floats() floats): vocabularies past 4096
// tokens run the multi-block chain (k_sb_*), smaller ones the single-workgroup register sampler
int dec_sample_ws(const float* logits, int V, const uint8_t* mask, float top_p, float temp, uint64_t seed,
                  int32_t* st, int inc_pos, int32_t* host_tok, float* ws, hipStream_t s) {
  if (V <= 0 || !ws) return (int)hipErrorInvalidValue;
  if (V <= 4096) {
    hipLaunchKernelGGL(k_sample_reg<4>, dim3(1), dim3(kSampThreads), 0, s, logits, V, mask, top_p, temp, seed, st,
                       inc_pos, host_tok);
    return (int)hipGetLastError();
  }
  const dim3 g(kSbBlocks), b(kSbThreads);
  hipLaunchKernelGGL(k_sb_max, g, b, 0, s, logits, V, mask, ws);
  const int nucleus = top_p < 1.f;
  if (nucleus) {
    hipLaunchKernelGGL(k_sb_hist<0>, g, b, 0, s, logits, V, mask, ws);
    hipLaunchKernelGGL(k_sb_select<0>, dim3(1), dim3(kSbBins), 0, s, top_p, ws);
    hipLaunchKernelGGL(k_sb_hist<1>, g, b, 0, s, logits, V, mask, ws);
    hipLaunchKernelGGL(k_sb_select<1>, dim3(1), dim3(kSbBins), 0, s, top_p, ws);
  }
  hipLaunchKernelGGL(k_sb_part, g, b, 0, s, logits, V, mask, temp, nucleus, ws);
  hipLaunchKernelGGL(k_sb_draw, dim3(1), dim3(kSbBins), 0, s, logits, V, mask, temp, seed, ws, st, inc_pos, host_tok);
  return (int)hipGetLastError();
}

int dec_sample(const float* logits, int V, const uint8_t* mask, float top_p, float temp, uint64_t seed, int32_t* st,
               int inc_pos, int32_t* host_tok, hipStream_t s) {
  if (V <= 0) return (int)hipErrorInvalidValue;
  if (V <= kSampThreads * 32)  // registers hold the vocabulary (llama-2 / mistral: 32000)
    hipLaunchKernelGGL(k_sample_reg<32>, dim3(1), dim3(kSampThreads), 0, s, logits, V, mask, top_p, temp, seed, st,
                       inc_pos, host_tok);
  else
    hipLaunchKernelGGL(k_sample, dim3(1), dim3(kSampThreads), 0, s, logits, V, mask, top_p, temp, seed, st, inc_pos,
                       host_tok);
  return (int)hipGetLastError();
}

}  // extern "C"
