// gemm_rln.hip — residual projection + post-LayerNorm in one kernel (K15 / K16-down of SURVEY
// §2.10): the o-proj and FFN-down GEMMs of the Nomic-BERT encoder, whose output width is the model
// width (N = 768), so ONE workgroup owns whole output rows and finishes the LayerNorm in registers:
//
//   out[m, :] = LN( A[m, :] . W^T + res[m, :] ) * gamma + beta        (out may alias res)
//
// This replaces the reference daemon's llama.cpp decode of these layers
// (/root/reference/splinference.cpp:236-251) and the round-2 pairing of a library GEMM with a
// separate LayerNorm pass (one extra read + write of the [M, 768] activations per projection).
//
// Geometry (gfx950, 256 CUs): workgroup tile 128 rows x 768 columns, 512 threads = 8 waves as
// 2 (rows) x 4 (columns); each wave owns 64 rows x 192 columns = 4 x 12 tiles of
// v_mfma_f32_16x16x32_bf16 (192 fp32 accumulators per lane).  At M = 32768 tokens the grid is
// exactly 256 workgroups: one per CU, no tail wave.  The MFMA operands are swapped (the W fragment
// is the A operand), so a lane's accumulator holds four CONSECUTIVE output columns of one row:
// residual loads, LayerNorm and the bf16 stores work on 8-byte row pieces straight from registers.
//
// K loop: BK = 32 (one MFMA k-step), two LDS buffers of [A 128 x 32 | W 768 x 32] bf16 (56 KB
// each), filled by global_load_lds_dwordx4 (LDS-DMA; 7 wave-instructions per wave per stage) one
// stage ahead of the MFMAs, counted vmcnt + raw s_barrier (no vmcnt(0) drain in the loop).  The
// LDS image has 64-byte rows; the 16-byte chunk c of row r is stored at chunk c ^ ((r >> 1) & 3),
// which makes every ds_read_b128 lane group (16 lanes) hit 16 distinct bank slots (brute-forced
// over the gfx950 b128 lane groups); glds writes lane-linearly, so the XOR is applied to the
// global source address and to the read address (guide rule 21).
//
// Epilogue: v = acc + res (fp32), row sums over the wave's 48 values per row, then across the 4
// lanes that share the row (xor 16 / 32) and the 4 column waves (LDS), two passes (mean, then
// centred variance), then (v - mean) * rstd * gamma + beta -> bf16.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>

#include "glds_asm.hpp"
#include "nomic_api.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int kBM = 128;          // rows per workgroup
constexpr int kN = 768;           // output width (= model width)
constexpr int kBK = 32;           // K per stage
constexpr int kWN = kN / 4;       // columns per wave (192)
constexpr int kNT = kWN / 16;     // 16-wide n-tiles per wave (12)
constexpr int kThreads = 512;
constexpr int kRowBytes = kBK * 2;                   // 64
constexpr int kABytes = kBM * kRowBytes;             // 8 KB per A stage
constexpr int kWBytes = kN * kRowBytes;              // 48 KB per W stage
constexpr int kGldsW = kWBytes / 1024 / 8;           // W wave-instructions per wave per stage (6)
// epilogue staging: half a tile (64 rows x 768 bf16, rows padded to 1552 B) + two [4][64] fp32
// reduction arrays
constexpr int kHalfRows = 64;
constexpr int kOutRowBytes = kN * 2;                  // 1536
constexpr int kRowPitch = kOutRowBytes + 16;          // 1552: 16 rows of one column -> 16 bank groups
constexpr int kHalfBytes = kHalfRows * kRowPitch;     // 97 KB
constexpr int kEpiLds = kHalfBytes + 2 * 4 * kHalfRows * 4;

// K pipelines (template PIPE): LDS rings of NW W-stages and NA A-stages, one barrier per stage.
// Iteration t, after its barrier, issues the stages W(t + NW - 1) and A(t + NA - 1) (the one with
// the shorter lead first) into ring slots last read in iteration t-1, then computes stage t.
//   PIPE 1: NW 2, NA 4 (128 KB): A -- streamed from HBM, read once -- three stages ahead
//   PIPE 2: NW 3, NA 2 (160 KB): W -- L2-resident, re-read by every workgroup -- two stages ahead
//   PIPE 3: NW 2, NA 2 (112 KB): both one stage ahead
template <int PIPE> struct Pipe;
template <> struct Pipe<1> { static constexpr int NW = 2, NA = 4; };
template <> struct Pipe<2> { static constexpr int NW = 3, NA = 2; };
template <> struct Pipe<3> { static constexpr int NW = 2, NA = 2; };
//   PIPE 4: NW 2, NA 6 (144 KB): A five stages ahead
template <> struct Pipe<4> { static constexpr int NW = 2, NA = 6; };
template <int PIPE>
constexpr int lds_bytes() {
  return Pipe<PIPE>::NW * kWBytes + Pipe<PIPE>::NA * kABytes > kEpiLds
             ? Pipe<PIPE>::NW * kWBytes + Pipe<PIPE>::NA * kABytes
             : kEpiLds;
}

__device__ __forceinline__ float bf2f(uint32_t h16) { return __uint_as_float(h16 << 16); }
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {  // wave-uniform: a scalar branch to an immediate count
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// physical 16-B chunk of logical chunk c in 64-B row r
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 3); }

// WM: waves along M.  2: 8 waves (2 x 4), 64 rows x 192 columns each (192 accumulators, two
// waves per SIMD).  1: 4 waves (1 x 4), 128 rows x 192 columns each (384 accumulators in the
// AGPR half of a 512-register wave, one wave per SIMD, 8 A fragments per stage: a third less
// LDS read traffic per MFMA and half the waves at each barrier).
// ILV > 0: the loads an iteration issues are spread over its MFMA groups (ILV LDS-DMA
// instructions ahead of each group of 8 MFMAs, in issue order) instead of all issued after the
// barrier, where they held both waves of a SIMD off the matrix core for the ~100-cycle issue cost
// of each DMA instruction.  ILV 0: all after the barrier.
// EPI 0: residual added in the epilogue (8-B loads); 1: LDS-staged epilogue; 2: the residual is
// the first K step -- one MFMA per tile against an identity operand (acc = I . R, exact: 1.0 x a
// bf16 value) with R fragments loaded in the prologue beside the first stages, so the epilogue
// reads nothing.  3 (K = 768, the o-proj): the residual is added during the K loop -- stage t
// loads the lane's residual pieces of two of its 48 (m-tile, n-tile) accumulator tiles, stage t + 1
// adds them -- so the epilogue only normalises and stores: the residual's 50 MB at M = 32768 no
// longer arrive while every workgroup sits in its epilogue (o-proj 62.6 -> 56.3 us; the down
// projection, K = 3072, gains nothing from it: 146.3 vs 147.1 us, profiles/r4aq).  PF: W fragment pairs read PF pairs
// ahead of their MFMAs.
// AS: the K-loop's LDS-DMAs issued from inline asm (glds_asm.hpp: counted lgkmcnt before the MFMAs)
// ROT: block b walks the K steps starting at step b mod nk (the sum is order-free up to fp32 rounding), so
// the 256 blocks that start together fetch different W stages instead of all hitting the same L2 lines
template <int PIPE, int EPI, int WM, int ILV = 0, int PF = 1, bool AS = false, bool ROT = false>
__global__ __launch_bounds__(256 * WM, 1) void k_gemm_rln(const uint16_t* __restrict__ A, long lda,
                                                          const uint16_t* __restrict__ W, long ldw, int K, long M,
                                                          const uint16_t* res, long ldr,
                                                          const uint16_t* __restrict__ gamma,
                                                          const uint16_t* __restrict__ beta, float eps,
                                                          uint16_t* out, long ldo) {
  constexpr int NW = Pipe<PIPE>::NW, NA = Pipe<PIPE>::NA;
  constexpr int LW = NW - 1, LA = NA - 1;              // stages of lead
  constexpr int kABase = NW * kWBytes;                 // LDS: [W ring | A ring]
  constexpr int kWaves = 4 * WM, kNThreads = 64 * kWaves;
  constexpr int RW = kBM / WM, MT = RW / 16;           // rows and m-tiles per wave
  constexpr int GA = 8 / kWaves, GW = 48 / kWaves;     // LDS-DMA wave-instructions per wave per stage
  static_assert(EPI == 0 || WM == 2, "the LDS-staged epilogue splits the tile by wave rows");
  static_assert(EPI != 3 || MT * kNT == 48, "EPI 3 spreads 48 accumulator tiles over 24 stages");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = WM == 2 ? wave >> 2 : 0, wn = wave & 3;
  // W is read by every block and A rows by one block only: no reuse for an XCD remap to exploit
  const long m0 = (long)blockIdx.x * kBM;

  // ---- per-lane LDS-DMA sources: a wave-instruction covers 16 rows x 64 B, lane -> (row, chunk)
  const int drow = lane >> 2, dpc = lane & 3;
  uint32_t offA[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int r = (wave + kWaves * i) * 16 + drow;
    const long gr = (m0 + r < M) ? m0 + r : M - 1;       // tail rows re-read row M-1, never stored
    offA[i] = (uint32_t)(gr * lda + swz(r, dpc) * 8);
  }
  uint32_t offW[GW];
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int r = (wave + kWaves * i) * 16 + drow;
    offW[i] = (uint32_t)(r * ldw + swz(r, dpc) * 8);
  }
  const int nk = K / kBK;
  // ring slot of stage t: t % NW (W), t % NA (A) -- stages enter each ring in order
  const int rot = ROT ? (int)(blockIdx.x % (unsigned)nk) : 0;
  auto kcol = [&](int t) -> long {  // global K offset of stage t
    if constexpr (ROT) {
      const int k = t + rot;
      return (long)(k < nk ? k : k - nk) * kBK;
    }
    return (long)t * kBK;
  };
  auto glds_w = [&](int t, int i) {
    if constexpr (AS)
      spl::glds16_asm(W + kcol(t) + offW[i], smem + (t % NW) * kWBytes + (wave + kWaves * i) * 1024);
    else
      __builtin_amdgcn_global_load_lds((gbl_void*)(W + kcol(t) + offW[i]),
                                       (lds_void*)(smem + (t % NW) * kWBytes + (wave + kWaves * i) * 1024), 16, 0, 0);
  };
  auto glds_a = [&](int t, int i) {
    if constexpr (AS)
      spl::glds16_asm(A + kcol(t) + offA[i], smem + kABase + (t % NA) * kABytes + (wave + kWaves * i) * 1024);
    else
      __builtin_amdgcn_global_load_lds((gbl_void*)(A + kcol(t) + offA[i]),
                                       (lds_void*)(smem + kABase + (t % NA) * kABytes + (wave + kWaves * i) * 1024),
                                       16, 0, 0);
  };
  // op u (0 .. GW+GA-1) of the loads iteration s issues: stage W(s + LW) and A(s + LA), the one
  // with the shorter lead first (younger() counts on that order)
  constexpr int kOps = GW + GA;
  auto issue_op = [&](int s, int u) {
    const int tw = s + LW, ta = s + LA;
    if (LW <= LA) {
      if (u < GW) { if (tw >= 0 && tw < nk) glds_w(tw, u); }
      else if (ta >= 0 && ta < nk) glds_a(ta, u - GW);
    } else {
      if (u < GA) { if (ta >= 0 && ta < nk) glds_a(ta, u); }
      else if (tw >= 0 && tw < nk) glds_w(tw, u - GA);
    }
  };
  auto issue = [&](int s) {
#pragma unroll
    for (int u = 0; u < kOps; ++u) issue_op(s, u);
  };
  // ops issued after the later of W(t) / A(t): they may stay in flight at the top of iteration t
  auto younger = [&](int t) -> int {
    if (LW < LA) return t + LA - 1 < nk ? GA : 0;           // A(t + LA - 1), issued after W(t)
    if (LW > LA) return t + LW - 1 < nk ? GW : 0;           // W(t + LW - 1), issued after A(t)
    return 0;
  };

  // fragment read: row = base16 + (lane & 15), logical chunk lane >> 4
  const int fl = (lane & 15) * kRowBytes + (swz(lane & 15, lane >> 4) << 4);
  const int aoff = kABase + (wr * RW) * kRowBytes + fl;
  const int woff = (wn * kWN) * kRowBytes + fl;

  f32x4 acc[MT][kNT];
  constexpr int L = LW > LA ? LW : LA;
  if constexpr (EPI == 2) {
    // residual fragments (B operand of a 16x16x32 MFMA: lane l holds k = 8 (l >> 4) .. +7 of column
    // l & 15): lanes 0-31 load res[m][n0 + 8 (l >> 4) .. +8] (16 B), lanes 32-63 (k 16-31) zero;
    // identity A operand: row n = l & 15 has its 1 at k = n
    bf16x8 rf[MT][kNT];
    const int rl = lane & 15;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const long m = m0 + wr * RW + i * 16 + rl;
      const uint16_t* rp = res + (m < M ? m : M - 1) * ldr + wn * kWN + 8 * ((lane >> 4) & 1);
#pragma unroll
      for (int j = 0; j < kNT; ++j) {
        if (lane < 32) rf[i][j] = *(const bf16x8*)(rp + j * 16);
        else rf[i][j] = bf16x8{};
      }
    }
    for (int s = -L; s < 0; ++s) issue(s);
    bf16x8 eye = bf16x8{};
    if (lane < 32 && (rl >> 3) == (lane >> 4)) eye[rl & 7] = (__bf16)1.0f;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < kNT; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(eye, rf[i][j], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  } else {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < kNT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = -L; s < 0; ++s) issue(s);
  }
  // EPI 3: residual pieces of accumulator tile u = (u / kNT, u % kNT), two tiles per stage
  const long rmb = m0 + wr * RW + (lane & 15);
  const int rcq = (lane >> 4) * 4;
  uint2 rq[2] = {make_uint2(0, 0), make_uint2(0, 0)};
  auto res_load = [&](int u, uint2& d) {
    const int i = u / kNT, j = u % kNT;
    const long m = rmb + 16 * i < M ? rmb + 16 * i : M - 1;
    d = *(const uint2*)(res + m * ldr + wn * kWN + j * 16 + rcq);
  };
  auto res_add = [&](int u, const uint2& rr) {
    const int i = u / kNT, j = u % kNT;
    acc[i][j][0] += bf2f(rr.x & 0xffff);
    acc[i][j][1] += bf2f(rr.x >> 16);
    acc[i][j][2] += bf2f(rr.y & 0xffff);
    acc[i][j][3] += bf2f(rr.y >> 16);
  };
  for (int t = 0; t < nk; ++t) {
    wait_vm(younger(t));
    raw_barrier();  // stage t visible to every wave; every wave is done with stage t-1's slots
    if (EPI == 3 && t < 24) {
      // loaded one stage ahead of their add, issued before this stage's DMAs (older than them: the
      // counted waits above stay exact); a chain of uniform branches keeps the tile indices static
#pragma unroll
      for (int k = 0; k < 24; ++k) {
        if (t == k) {
          if (k > 0) {
            res_add(2 * (k - 1), rq[0]);
            res_add(2 * (k - 1) + 1, rq[1]);
          }
          res_load(2 * k, rq[0]);
          res_load(2 * k + 1, rq[1]);
        }
      }
    }
    if (ILV == 0) issue(t);
    const char* bw = smem + (t % NW) * kWBytes;
    const char* ba = smem + (t % NA) * kABytes;
    // A fragments for the whole stage, W fragments two n-tiles at a time with the next pair's reads
    // issued ahead of the current pair's MFMAs (sched_barrier pins the pairs: hoisting all 12 W
    // reads would need 48 more registers than the 256 two waves per SIMD allow)
    bf16x8 af[MT], w0, w1, x0, x1, y0, y1;
#pragma unroll
    for (int i = 0; i < MT; ++i) af[i] = *(const bf16x8*)(ba + aoff + i * 16 * kRowBytes);
    w0 = *(const bf16x8*)(bw + woff);
    w1 = *(const bf16x8*)(bw + woff + 16 * kRowBytes);
    if (PF == 2) {
      x0 = *(const bf16x8*)(bw + woff + 2 * 16 * kRowBytes);
      x1 = *(const bf16x8*)(bw + woff + 3 * 16 * kRowBytes);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int jp = 0; jp < kNT / 2; ++jp) {
      if (ILV > 0) {
#pragma unroll
        for (int u = jp * ILV; u < (jp + 1) * ILV; ++u)
          if (u < kOps) issue_op(t, u);
      }
      if (jp + PF < kNT / 2) {
        bf16x8& d0 = PF == 2 ? y0 : x0;
        bf16x8& d1 = PF == 2 ? y1 : x1;
        d0 = *(const bf16x8*)(bw + woff + (2 * (jp + PF)) * 16 * kRowBytes);
        d1 = *(const bf16x8*)(bw + woff + (2 * (jp + PF) + 1) * 16 * kRowBytes);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        acc[i][2 * jp] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, af[i], acc[i][2 * jp], 0, 0, 0);
        acc[i][2 * jp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, af[i], acc[i][2 * jp + 1], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      w0 = x0;
      w1 = x1;
      if (PF == 2) {
        x0 = y0;
        x1 = y1;
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (ILV > 0) {
#pragma unroll
      for (int u = (kNT / 2) * ILV; u < kOps; ++u) issue_op(t, u);
    }
  }
  if constexpr (EPI == 3) {  // the last pair (loaded at stage 23)
    res_add(46, rq[0]);
    res_add(47, rq[1]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  raw_barrier();  // every wave is done with the rings: the LDS is the epilogue's

  // ---- epilogue -------------------------------------------------------------------------
  // lane: rows m_i = m0 + wr*64 + i*16 + (lane & 15); columns n_j = wn*192 + j*16 + (lane>>4)*4 + 0..3
  const int rl = lane & 15, cq = (lane >> 4) * 4;
  if constexpr (EPI != 1) {
    // direct: residual loads (EPI 0; EPI 2 has it in the accumulators) and 8-B stores from registers
    float* red = (float*)smem;  // [4 column waves][128 rows]
    const long mb = m0 + wr * RW + rl;  // row of m-tile i: mb + 16 i
    float s[MT] = {};
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
      const int n = wn * kWN + j * 16 + cq;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if constexpr (EPI == 0) {
          const long m = mb + 16 * i < M ? mb + 16 * i : M - 1;
          const uint2 rr = *(const uint2*)(res + m * ldr + n);
          acc[i][j][0] += bf2f(rr.x & 0xffff);
          acc[i][j][1] += bf2f(rr.x >> 16);
          acc[i][j][2] += bf2f(rr.y & 0xffff);
          acc[i][j][3] += bf2f(rr.y >> 16);
        }
        (void)n;
        s[i] += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
      }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      s[i] += __shfl_xor(s[i], 16);
      s[i] += __shfl_xor(s[i], 32);
    }
    if (lane < 16) {
#pragma unroll
      for (int i = 0; i < MT; ++i) red[wn * kBM + wr * RW + i * 16 + rl] = s[i];
    }
    __syncthreads();
    float mean[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int r = wr * RW + i * 16 + rl;
      mean[i] = (red[r] + red[kBM + r] + red[2 * kBM + r] + red[3 * kBM + r]) * (1.f / kN);
      s[i] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < kNT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = acc[i][j][e] - mean[i];
          s[i] += d * d;
        }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      s[i] += __shfl_xor(s[i], 16);
      s[i] += __shfl_xor(s[i], 32);
    }
    __syncthreads();  // every wave has read the row sums
    if (lane < 16) {
#pragma unroll
      for (int i = 0; i < MT; ++i) red[wn * kBM + wr * RW + i * 16 + rl] = s[i];
    }
    __syncthreads();
    float rstd[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int r = wr * RW + i * 16 + rl;
      const float var = (red[r] + red[kBM + r] + red[2 * kBM + r] + red[3 * kBM + r]) * (1.f / kN);
      rstd[i] = rsqrtf(var + eps);
    }
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
      const int n = wn * kWN + j * 16 + cq;
      const uint2 gg = *(const uint2*)(gamma + n), bb = *(const uint2*)(beta + n);
      const float g[4] = {bf2f(gg.x & 0xffff), bf2f(gg.x >> 16), bf2f(gg.y & 0xffff), bf2f(gg.y >> 16)};
      const float be[4] = {bf2f(bb.x & 0xffff), bf2f(bb.x >> 16), bf2f(bb.y & 0xffff), bf2f(bb.y >> 16)};
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const long m = mb + 16 * i;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (acc[i][j][e] - mean[i]) * rstd[i] * g[e] + be[e];
        if (m < M) *(uint2*)(out + m * ldo + n) = make_uint2(pk2(o[0], o[1]), pk2(o[2], o[3]));
      }
    }
  } else {
    // LDS-staged, one 64-row half at a time: the residual half-tile comes in by LDS-DMA with every
    // request in flight at once (whole rows in 16-B pieces), the waves that own the half add it and
    // normalise in registers, write bf16 back in place, and all 512 threads store whole rows with
    // 16-B stores.  Rows are padded to 1552 B, so the 16 lanes that read one column of 16 rows hit 16
    // different bank groups and every (m-tile, n-tile) element of a lane sits at a fixed offset
    // from one base address.  A padded row cannot take a 1-KB DMA piece across its end: each row is
    // one 64-lane piece (bytes 0-1023) and one 32-lane piece (1024-1535).
    char* R = smem;
    float* red1 = (float*)(smem + kHalfBytes);
    float* red2 = red1 + 4 * kHalfRows;
    const int ebase = rl * kRowPitch + (wn * kWN + cq) * 2;  // + i*16 rows + j*16 columns
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      const long mh = m0 + h * kHalfRows;
#pragma unroll 1
      for (int u = 0; u < kHalfRows / 8; ++u) {
        const int row = wave * 8 + u;
        const long gr = mh + row < M ? mh + row : M - 1;
        const uint16_t* src = res + gr * ldr + lane * 8;
        __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(R + row * kRowPitch), 16, 0, 0);
        if (lane < 32)
          __builtin_amdgcn_global_load_lds((gbl_void*)(src + 512), (lds_void*)(R + row * kRowPitch + 1024), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const bool mine = wr == h;
      float mean[4], rstd[4];
      if (mine) {
        float sm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < kNT; ++j) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint2 rr = *(const uint2*)(R + ebase + i * 16 * kRowPitch + j * 32);
            acc[i][j][0] += bf2f(rr.x & 0xffff);
            acc[i][j][1] += bf2f(rr.x >> 16);
            acc[i][j][2] += bf2f(rr.y & 0xffff);
            acc[i][j][3] += bf2f(rr.y >> 16);
            sm[i] += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sm[i] += __shfl_xor(sm[i], 16);
          sm[i] += __shfl_xor(sm[i], 32);
          if (lane < 16) red1[wn * kHalfRows + i * 16 + rl] = sm[i];
        }
      }
      __syncthreads();
      if (mine) {
        float sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = i * 16 + rl;
          mean[i] = (red1[r] + red1[kHalfRows + r] + red1[2 * kHalfRows + r] + red1[3 * kHalfRows + r]) * (1.f / kN);
        }
#pragma unroll
        for (int j = 0; j < kNT; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float d = acc[i][j][e] - mean[i];
              sq[i] += d * d;
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sq[i] += __shfl_xor(sq[i], 16);
          sq[i] += __shfl_xor(sq[i], 32);
          if (lane < 16) red2[wn * kHalfRows + i * 16 + rl] = sq[i];
        }
      }
      __syncthreads();
      if (mine) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = i * 16 + rl;
          const float var = (red2[r] + red2[kHalfRows + r] + red2[2 * kHalfRows + r] + red2[3 * kHalfRows + r]) *
                            (1.f / kN);
          rstd[i] = rsqrtf(var + eps);
        }
#pragma unroll
        for (int j = 0; j < kNT; ++j) {
          const int n = wn * kWN + j * 16 + cq;
          const uint2 gg = *(const uint2*)(gamma + n), bb = *(const uint2*)(beta + n);
          const float g[4] = {bf2f(gg.x & 0xffff), bf2f(gg.x >> 16), bf2f(gg.y & 0xffff), bf2f(gg.y >> 16)};
          const float be[4] = {bf2f(bb.x & 0xffff), bf2f(bb.x >> 16), bf2f(bb.y & 0xffff), bf2f(bb.y >> 16)};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (acc[i][j][e] - mean[i]) * rstd[i] * g[e] + be[e];
            *(uint2*)(R + ebase + i * 16 * kRowPitch + j * 32) = make_uint2(pk2(o[0], o[1]), pk2(o[2], o[3]));
          }
        }
      }
      __syncthreads();
      // the normalised half -> global, whole rows in 16-B pieces
#pragma unroll 2
      for (int u = 0; u < kHalfRows * 96 / kThreads; ++u) {
        const int L = u * kThreads + tid;
        const int row = L / 96, pc = L - row * 96;
        const uint4 v = *(const uint4*)(R + row * kRowPitch + pc * 16);
        if (mh + row < M) *(uint4*)(out + (mh + row) * ldo + pc * 8) = v;
      }
      __syncthreads();  // R is refilled by the next half
    }
  }
}

// Two selectable forms (NOMIC_RLN): 222 (default) = PIPE 2 (3 W stages, 2 A stages), DMA
// interleave 2, residual added in the epilogue; 232 = the same with the residual added during the
// K loop at K = 768 (EPI 3): 10 % faster on the o-proj with a cold residual (profiles/r4aq), but in
// the encoder the residual was just written by the previous layer and is warm, and the mixed step
// measured 12.452 (222) vs 12.500 ms (232) over three alternating runs each (profiles/r4ax).  The
// other A/B forms of round 3 are gone; their measurements stay in profiles/r3_rln_*.
int g_rln_variant = -1;
int rln_pick(int v) { return v == 232 ? 232 : 222; }
int rln_variant() {
  if (g_rln_variant < 0) {
    const char* e = getenv("NOMIC_RLN");
    g_rln_variant = rln_pick(e && *e ? atoi(e) : 222);
  }
  return g_rln_variant;
}

template <int PIPE, int EPI, int WM = 2, int ILV = 0, int PF = 1, bool AS = false, bool ROT = false>
void launch_rln(unsigned blocks, hipStream_t s, const uint16_t* A, long lda, const uint16_t* W, long ldw, int K, long M,
                const uint16_t* res, long ldr, const uint16_t* gamma, const uint16_t* beta, float eps, uint16_t* out,
                long ldo) {
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_gemm_rln<PIPE, EPI, WM, ILV, PF, AS, ROT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds_bytes<PIPE>());
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL((k_gemm_rln<PIPE, EPI, WM, ILV, PF, AS, ROT>), dim3(blocks), dim3(256 * WM), lds_bytes<PIPE>(), s, A, lda, W, ldw, K,
                     M, res, ldr, gamma, beta, eps, out, ldo);
}

}  // namespace

extern "C" int nomic_gemm_res_ln(const void* A, long lda, const void* W, long ldw, long M, int N, int K,
                                 const void* res, long ldr, const void* gamma, const void* beta, float eps, void* out,
                                 long ldo, hipStream_t s) {
  // shapes the kernel and its grid assume: row-complete 768-wide tiles, whole K stages, 16-B
  // aligned rows, 32-bit DMA offsets
  if (N != kN || K < kBK || K % kBK || M <= 0 || !A || !W || !res || !gamma || !beta || !out)
    return (int)hipErrorInvalidValue;
  if (lda % 8 || ldw % 8 || ldr % 4 || ldo % 4 || lda < K || ldw < K || ldr < N || ldo < N)
    return (int)hipErrorInvalidValue;
  if ((M - 1) * lda + K >= (1L << 32) || (long)kN * ldw >= (1L << 32)) return (int)hipErrorInvalidValue;
  static_assert(lds_bytes<2>() <= 160 * 1024, "LDS budget");
  const unsigned blocks = (unsigned)((M + kBM - 1) / kBM);
  const auto* a = (const uint16_t*)A;
  const auto* w = (const uint16_t*)W;
  const auto* r = (const uint16_t*)res;
  const auto* g = (const uint16_t*)gamma;
  const auto* b = (const uint16_t*)beta;
  auto* o = (uint16_t*)out;
  if (rln_variant() == 232 && K / kBK >= 24 && K <= 768) launch_rln<2, 3, 2, 2>(blocks, s, a, lda, w, ldw, K, M, r, ldr, g, b, eps, o, ldo);
  else launch_rln<2, 0, 2, 2>(blocks, s, a, lda, w, ldw, K, M, r, ldr, g, b, eps, o, ldo);
  return (int)hipGetLastError();
}

extern "C" int nomic_gemm_res_ln_set_variant(int variant) {
  const int prev = rln_variant();
  g_rln_variant = rln_pick(variant);
  return prev;
}
