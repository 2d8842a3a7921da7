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
// Both are HBM-bound row kernels: one 64-lane wave per row, 16-B (8 x bf16)
// vector accesses, statistics reduced with __shfl_xor over the full wavefront.
// The projections run on the MFMA GEMM (gemm_bf16.hip).
#include <hip/hip_runtime.h>
#include <cstdint>

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
                                                     int hd, float scale, uint16_t* __restrict__ out) {
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
      float dot = 0.f;
      for (int c = 0; c < hd; c += 8) {
        float f[8];
        unpack8(*(const uint4*)(kr + c), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) dot += f[e] * qs[c + e];
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

}  // namespace

extern "C" {

// q: bf16 [H*hd] (one token, RoPE applied); k/v: bf16 cache rows [L, ldkv] (ldkv = KVH*hd);
// out: bf16 [H*hd].  hd in {64, 128, 192, 256}, H % KVH == 0, L >= 1, 16-B aligned rows.
int dec_attn_decode(const void* q, const void* k, const void* v, long ldkv, int L, int H, int KVH, int hd,
                    float scale, void* out, hipStream_t s) {
  if (L <= 0 || H <= 0 || KVH <= 0 || H % KVH || hd <= 0 || hd % 64 || hd > 256 || ldkv % 8 ||
      ldkv < (long)KVH * hd || ((uintptr_t)k | (uintptr_t)v) % 16)
    return (int)hipErrorInvalidValue;
  const int grp = H / KVH;
  const dim3 g((unsigned)H), b(kDecWaves * 64);
  const uint16_t *qq = (const uint16_t*)q, *kk = (const uint16_t*)k, *vv = (const uint16_t*)v;
  uint16_t* oo = (uint16_t*)out;
  switch (hd / 64) {
    case 1: hipLaunchKernelGGL(k_attn_decode<1>, g, b, 0, s, qq, kk, vv, ldkv, L, grp, hd, scale, oo); break;
    case 2: hipLaunchKernelGGL(k_attn_decode<2>, g, b, 0, s, qq, kk, vv, ldkv, L, grp, hd, scale, oo); break;
    case 3: hipLaunchKernelGGL(k_attn_decode<3>, g, b, 0, s, qq, kk, vv, ldkv, L, grp, hd, scale, oo); break;
    default: hipLaunchKernelGGL(k_attn_decode<4>, g, b, 0, s, qq, kk, vv, ldkv, L, grp, hd, scale, oo); break;
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

}  // extern "C"
