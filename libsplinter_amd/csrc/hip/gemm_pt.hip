// gemm_pt.hip — persistent 256x256 MFMA GEMM with a register epilogue, for the encoder's
// projections whose K is short (K = 768: the qkv and up|gate GEMMs of Nomic-BERT, SURVEY §2.10
// K12/K13/K16).  Same math as k_gemm256 (gemm_bf16.hip):
//
//   C[M, N] = A[M, K] . W[N, K]^T      with a fused STORE / SWIGLU / ROPE epilogue
//
// Why a second kernel: at K = 768 a 256x256 tile is only 12 K-steps, and the launch-per-tile kernel
// spends a third of each tile outside its K loop -- the first two K-tiles' loads arrive before any
// MFMA can run (prologue), and the epilogue is an LDS round trip with two block barriers and a store
// tail with every wave waiting (profiles/r4k: 24.9 us per tile wave against ~11 us of MFMA work).
// Here each workgroup (one per CU) walks a strided list of tiles as ONE continuous K-step stream:
//   * the LDS-DMA prefetch runs two K-steps ahead ACROSS tile boundaries -- the next tile's first
//     K-tiles are in flight while the current tile finishes -- so no tile after the first waits
//     for its operands;
//   * the MFMA operands are swapped (the W fragment is the A operand), so a lane's accumulator holds
//     four CONSECUTIVE output columns of one row, and the epilogue (SwiGLU / RoPE / plain) works on
//     registers and stores 8-B row pieces with buffer stores: no LDS image, no barrier.  The stores
//     are left in flight (counted in the next tile's vmcnt waits) while the next tile's MFMAs start.
//     Buffer stores are range-checked by the hardware (num_records = M rows), so tail rows need no
//     branch and every wave issues exactly the same number of store instructions -- which the
//     counted waits rely on.
//   * RoPE computes its angle from the token position (staged per tile into LDS by one LDS-DMA per
//     wave of the first half) and the rotary frequency of the lane's head dims, read once from row 1
//     of the caller's table (theta_d = atan2(sin, cos) of position 1): the same linear NEOX RoPE the
//     table holds, without table loads in the epilogue (a plain load there would force a vmcnt(0)
//     that drains the next tile's prefetch).
//
// K loop: the phase schedule of k_gemm256's lockstep form (8 waves as 2 (M) x 4 (N), 4 phases per
// K-tile, quadrant (qm, qn) per phase, LDS = 2 buffers x [A0 | A1 | B0 | B1] half-tiles of 128 rows
// x 64 bf16, XOR-swizzled on the global source address; LDS-DMA from inline asm; counted vmcnt +
// raw s_barrier).  The counted waits gain the tile boundary's extra in-flight operations: after an
// epilogue its S stores sit between K-tile kt0's and kt1's DMAs, and (RoPE) the position DMA after
// kt0's phase-1 reads -- each wait up to kt1's phase 2 allows them (derivation above kt_step).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

#include "glds_asm.hpp"
#include "nomic_api.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int BK = 64;
constexpr int kThreads = 512;
constexpr int kHalfBytes = 128 * BK * 2;           // 16 KB
constexpr int kBufBytes = 4 * kHalfBytes;          // 64 KB
constexpr int kPosBytes = 512 * 4;                 // one tile's token positions (two copies)
constexpr int kLdsBytes = 2 * kBufBytes + 2 * kPosBytes;
constexpr int kRsrcWord3 = 0x00020000;             // gfx9 raw buffer

struct PtArgs {
  uint16_t* out;
  long ldo;
  const float* rope;     // [max_pos][32] x (cos, sin): row 1 gives theta_d
  const int32_t* pos;    // [M] position of each row
  int rope_cols;
  long M;
  int gn;
};

__device__ __forceinline__ uint32_t pk2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float swiglu(float up, float g) {
  return up * g * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-g * 1.4426950408889634f));
}

#define SPL_VM(n) \
  case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
// wave-uniform count -> immediate (scalar branch)
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    SPL_VM(1) SPL_VM(2) SPL_VM(3) SPL_VM(4) SPL_VM(5) SPL_VM(6) SPL_VM(7) SPL_VM(8) SPL_VM(9) SPL_VM(10)
    SPL_VM(11) SPL_VM(12) SPL_VM(13) SPL_VM(14) SPL_VM(15) SPL_VM(16) SPL_VM(17) SPL_VM(18) SPL_VM(19)
    SPL_VM(20) SPL_VM(21) SPL_VM(22) SPL_VM(23) SPL_VM(24) SPL_VM(25) SPL_VM(26) SPL_VM(27) SPL_VM(28)
    SPL_VM(29) SPL_VM(30) SPL_VM(31) SPL_VM(32) SPL_VM(33) SPL_VM(34) SPL_VM(35) SPL_VM(36) SPL_VM(37)
    SPL_VM(38) SPL_VM(39) SPL_VM(40) SPL_VM(41) SPL_VM(42) SPL_VM(43) SPL_VM(44) SPL_VM(45) SPL_VM(46)
    SPL_VM(47) SPL_VM(48)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
#undef SPL_VM
template <int N>
__device__ __forceinline__ void vm_wait_c() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one 4-B-per-lane LDS-DMA (global_load_lds_dword) from inline asm, like spl::glds16_asm: hidden from
// hipcc's wait insertion, ordered by this kernel's own counted vmcnt waits
__device__ __forceinline__ void glds4_asm(const void* gsrc, const void* lds_dst) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  uint32_t save;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(save)
               : "v"(gsrc), "s"(l)
               : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void remap_tile(int bid, int nb, int nt, int gn, int& mt, int& ntile) {
  // bijective XCD remap (as gemm_bf16.hip): blocks b and b+8 share an XCD; each XCD walks a
  // contiguous range of the band-major tile order
  const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_band = (nb / nt) * gn;
  const int band = wg / per_band, rem = wg - band * per_band;
  mt = rem / gn;
  ntile = band * gn + (rem - mt * gn);
}

// store instructions each wave's epilogue issues (exact: the counted waits of the next tile rely on it)
template <int MODE> constexpr int stores_per_tile() { return MODE == NOMIC_EPI_SWIGLU ? 16 : 32; }

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void k_gemm_pt(const uint16_t* __restrict__ A, long lda,
                                                         const uint16_t* __restrict__ W, long ldw, int K,
                                                         int mtiles, int ntiles, PtArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int S = stores_per_tile<MODE>();
  constexpr bool kRope = MODE == NOMIC_EPI_ROPE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wn = wave & 3;
  const int nk = K / BK;
  const int total = mtiles * ntiles;
  const int G = gridDim.x;
  const int mine = (total - (int)blockIdx.x + G - 1) / G;  // >= 1 (grid <= tiles)
  const long M = ep.M;

  // per-lane DMA geometry (k_gemm256): half h, instruction i -> row h*128 + (i*8 + wave)*8 + srow
  const int srow = lane >> 3, schunk = ((lane & 7) ^ srow) * 8;
  uint32_t offB[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) offB[h][i] = (uint32_t)((h * 128 + (i * 8 + wave) * 8 + srow) * ldw + schunk);

  struct Tile {
    const uint16_t* a;   // A + m0 * lda (wave-uniform)
    const uint16_t* w;   // W + n0 * ldw
    uint32_t offA[2][2]; // lane offsets, rows clamped to M - 1 (tail rows re-read, never stored)
    long m0, n0;
    int nt;
  };
  auto tile_of = [&](int it, Tile& t) {
    int mt, ntl;
    remap_tile((int)blockIdx.x + it * G, total, ntiles, ep.gn, mt, ntl);
    t.m0 = (long)mt * 256;
    t.n0 = (long)ntl * 256;
    t.nt = ntl;
    t.a = A + t.m0 * lda;
    t.w = W + t.n0 * ldw;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const long r = h * 128 + (i * 8 + wave) * 8 + srow;
        const long gr = (t.m0 + r < M) ? r : M - 1 - t.m0;
        t.offA[h][i] = (uint32_t)(gr * lda + schunk);
      }
  };
  auto stage = [&](const Tile& t, int which, int kt, int buf) {  // which: 0 A0, 1 A1, 2 B0, 3 B1
    const uint16_t* base = (which < 2 ? t.a : t.w) + (long)kt * BK;
    char* dst = smem + buf * kBufBytes + which * kHalfBytes;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t off = which == 0 ? t.offA[0][i] : which == 1 ? t.offA[1][i] : which == 2 ? offB[0][i] : offB[1][i];
      spl::glds16_asm(base + off, dst + (i * 8 + wave) * 1024);
    }
  };

  // RoPE: rotary frequency of the lane's four head dims d = (wn & 1) * 16 + (lane >> 4) * 4 + r, in
  // revolutions per position, from the table's position-1 row (waited for here, before any DMA)
  float rev[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (kRope) {
    const int d0 = (wn & 1) * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float c = ep.rope[64 + 2 * (d0 + r)], s = ep.rope[64 + 2 * (d0 + r) + 1];
      rev[r] = atan2f(s, c) * 0.15915494309189535f;
    }
    asm volatile("" ::"v"(rev[0]), "v"(rev[1]), "v"(rev[2]), "v"(rev[3]));
  }
  const rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
      ep.out, 0, (int)(M * ep.ldo * 2 < 0x7fffffffL ? M * ep.ldo * 2 : 0x7fffffffL), kRsrcWord3);
  int32_t* posl = (int32_t*)(smem + 2 * kBufBytes);

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
  bf16x8 af[4][2], b0[2][2], b1[2][2];

  Tile tc, tn;
  tile_of(0, tc);
  tn = tc;
  if (mine > 1) tile_of(1, tn);
  // prologue, in the steady-state issue order: A0 B0 B1 A1 (kt 0), A0 B0 B1 (kt 1) -- nk >= 4
  stage(tc, 0, 0, 0); stage(tc, 2, 0, 0); stage(tc, 3, 0, 0); stage(tc, 1, 0, 0);
  stage(tc, 0, 1, 1); stage(tc, 2, 1, 1); stage(tc, 3, 1, 1);

  auto rd = [](bf16x8& dst, const char* p) {
    dst = *(const bf16x8*)p;
    __builtin_amdgcn_sched_barrier(0);
  };
  // operands swapped: D rows = W rows (output columns), D cols = A rows (tokens)
  auto mm = [&](f32x4 (&ac)[4][2], bf16x8 (&bf)[2][2], int kk) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        ac[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][kk], af[i][kk], ac[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // extra operations in flight at the counted waits of a tile's first two K-tiles (xs: the previous
  // tile's S epilogue stores, issued after kt0/kt1's DMAs were; xp: this tile's position DMA, issued
  // after kt0's phase-1 wait).  Target of each wait and what is younger than it:
  //   kt0 P1  A0/B0(t)   B1(t) A1(t) A0/B0/B1(t+1)                 + stores            -> 10 + xs
  //   kt0 P2  B1(t)      A1(t) A0/B0/B1(t+1) A1(t+1)               + stores + pos      -> 10 + xs + xp
  //   kt0 P3  A1(t)      A0/B0/B1(t+1) A1(t+1) A0(t+2)             + stores + pos      -> 10 + xs + xp
  //   kt1 P1  A0/B0(t+1) B1(t+1) A1(t+1) A0/B0/B1(t+2)             + stores + pos      -> 10 + xs + xp
  //   kt1 P2  B1(t+1)    A1(t+1) A0/B0/B1(t+2) A1(t+2)             + stores + pos      -> 10 + xs + xp
  //   kt1 P3  A1(t+1)    A0/B0/B1(t+2) A1(t+2) A0(t+3)             (stores, pos older) -> 10
  // counted wait for base count B plus the tile boundary's extra in-flight operations `ext` (one of
  // 0, XP, S, S + XP): one compare per possible value, then ONE s_waitcnt with an immediate
  constexpr int XP = kRope ? 1 : 0;
  auto wait_ext = [](auto bc, int ext) {
    constexpr int B = decltype(bc)::value;
    if (ext == 0) vm_wait_c<B>();
    else if (ext == S + XP) vm_wait_c<B + S + XP>();
    else if (ext == S) vm_wait_c<B + S>();
    else vm_wait_c<B + XP>();
  };
  using I10 = std::integral_constant<int, 10>;
  using I8 = std::integral_constant<int, 8>;
  using I4 = std::integral_constant<int, 4>;
  using I2 = std::integral_constant<int, 2>;
  using I0 = std::integral_constant<int, 0>;
  auto kt_step = [&](const Tile& t, int kt, int buf, bool n1, bool n2, int e1, int e2, int e3, const Tile& tnx,
                     int ppar) {
    const char* hA0 = smem + buf * kBufBytes;
    const char* hA1 = hA0 + kHalfBytes;
    const char* hB0 = hA0 + 2 * kHalfBytes;
    const char* hB1 = hA0 + 3 * kHalfBytes;
    const char* pb0 = hB0 + (wn * 32) * 128 + frow;
    const char* pb1 = hB1 + (wn * 32) * 128 + frow;
    const char* pa0 = hA0 + (wr * 64) * 128 + frow;
    const char* pa1 = hA1 + (wr * 64) * 128 + frow;
    // staging targets: step +1 (A1) and step +2 (A0, B0, B1), in this tile or the next
    const bool in1 = kt + 1 < nk, in2 = kt + 2 < nk;
    const Tile& t1 = in1 ? t : tnx;
    const Tile& t2 = in2 ? t : tnx;
    const int k1 = in1 ? kt + 1 : kt + 1 - nk, k2 = in2 ? kt + 2 : kt + 2 - nk;
    // ---- phase 1: quadrant (0,0)
    if (n1) wait_ext(I10{}, e1);
    else wait_ext(I4{}, e1);
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
    if (kRope && kt == 0) {
      // this tile's token positions -> LDS (the tile's parity buffer): every wave one DMA of 64 rows,
      // waves 4-7 a second copy of waves 0-3's rows, so every wave's wait counts are the same
      const long m = t.m0 + (wave & 3) * 64 + lane;
      glds4_asm(ep.pos + (m < M ? m : M - 1), posl + ppar * 512 + wave * 64);
    }
    if (n1) stage(t1, 1, k1, buf ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mm(acc[0][0], b0, 0);
    mm(acc[0][0], b0, 1);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 2: quadrant (0,1)
    if (n1) wait_ext(I10{}, e2);
    else wait_ext(I2{}, e2);
    raw_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int fs = kk ? fsw1 : fsw0;
      rd(b1[0][kk], pb1 + fs);
      rd(b1[1][kk], pb1 + 16 * 128 + fs);
    }
    if (n2) stage(t2, 0, k2, buf);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mm(acc[0][1], b1, 0);
    mm(acc[0][1], b1, 1);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 3: quadrant (1,0)
    if (n2) wait_ext(I10{}, e3);
    else if (n1) wait_ext(I8{}, e3);
    else wait_ext(I0{}, e3);
    raw_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int fs = kk ? fsw1 : fsw0;
#pragma unroll
      for (int i = 0; i < 4; ++i) rd(af[i][kk], pa1 + i * 16 * 128 + fs);
    }
    if (n2) stage(t2, 2, k2, buf);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mm(acc[1][0], b0, 0);
    mm(acc[1][0], b0, 1);
    __builtin_amdgcn_s_setprio(0);
    // ---- phase 4: quadrant (1,1), registers only
    if (n2) stage(t2, 3, k2, buf);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mm(acc[1][1], b1, 0);
    mm(acc[1][1], b1, 1);
    __builtin_amdgcn_s_setprio(0);
  };

  const long steps = (long)mine * nk;
  for (int it = 0; it < mine; ++it) {
    const int xs = it > 0 ? S : 0;
    for (int kt = 0; kt < nk; ++kt) {
      const long st = (long)it * nk + kt;
      const bool n1 = st + 1 < steps, n2 = st + 2 < steps;
      const int e1 = kt == 0 ? xs : kt == 1 ? xs + XP : 0;
      const int e2 = kt <= 1 ? xs + XP : 0;
      const int e3 = kt == 0 ? xs + XP : 0;
      kt_step(tc, kt, (int)(st & 1), n1, n2, e1, e2, e3, tn, it & 1);
    }

    // ---- epilogue from registers: 8-B row pieces, buffer stores left in flight ----------------
    const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rloc = qm * 128 + wr * 64 + i * 16 + fr;
        const uint32_t rowoff = (uint32_t)((tc.m0 + rloc) * ep.ldo) * 2u;
        if constexpr (MODE == NOMIC_EPI_SWIGLU) {
#pragma unroll
          for (int qn = 0; qn < 2; ++qn) {
            const f32x4 u = acc[qm][qn][i][0], g = acc[qm][qn][i][1];
            const i32x2 v = {(int)pk2(swiglu(u[0], g[0]), swiglu(u[1], g[1])),
                             (int)pk2(swiglu(u[2], g[2]), swiglu(u[3], g[3]))};
            const uint32_t col = (uint32_t)(tc.nt * 128 + qn * 64 + wn * 16 + fq * 4);
            __builtin_amdgcn_raw_buffer_store_b64(v, orsrc, rowoff + col * 2u, 0, 0);
          }
        } else if constexpr (kRope) {
          const float p = (float)posl[(it & 1) * 512 + rloc];
#pragma unroll
          for (int qn = 0; qn < 2; ++qn) {
            const long hb = tc.n0 + qn * 128 + (wn >> 1) * 64;  // head's first column
            const int d = (wn & 1) * 16 + fq * 4;
            f32x4 x1 = acc[qm][qn][i][0], x2 = acc[qm][qn][i][1];
            if (hb < ep.rope_cols) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float ph = __builtin_amdgcn_fractf(p * rev[r]);
                const float c = __builtin_amdgcn_cosf(ph), sn = __builtin_amdgcn_sinf(ph);
                const float a = x1[r], b = x2[r];
                x1[r] = a * c - b * sn;
                x2[r] = b * c + a * sn;
              }
            }
            const i32x2 v1 = {(int)pk2(x1[0], x1[1]), (int)pk2(x1[2], x1[3])};
            const i32x2 v2 = {(int)pk2(x2[0], x2[1]), (int)pk2(x2[2], x2[3])};
            __builtin_amdgcn_raw_buffer_store_b64(v1, orsrc, rowoff + (uint32_t)(hb + d) * 2u, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64(v2, orsrc, rowoff + (uint32_t)(hb + d + 32) * 2u, 0, 0);
          }
        } else {
#pragma unroll
          for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const f32x4 x = acc[qm][qn][i][j];
              const i32x2 v = {(int)pk2(x[0], x[1]), (int)pk2(x[2], x[3])};
              const uint32_t col = (uint32_t)(tc.n0 + qn * 128 + wn * 32 + j * 16 + fq * 4);
              __builtin_amdgcn_raw_buffer_store_b64(v, orsrc, rowoff + col * 2u, 0, 0);
            }
        }
      }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (it + 1 < mine) {
      tc = tn;
      if (it + 2 < mine) tile_of(it + 2, tn);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename F>
void allow_lds(F* f, int bytes) {
  (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

int g_cus = 0;

}  // namespace

// Internal entry (gemm_bf16.hip's launcher): -1 when the shape is not one this kernel takes (the
// caller then uses k_gemm256 / k_gemm_nt), else the HIP status of the launch.
int spl_gemm_pt(int mode, const uint16_t* A, long lda, const uint16_t* W, long ldw, long M, int N, int K,
                uint16_t* out, long ldo, const float* rope, const int32_t* pos, int rope_cols, int gn_cap,
                hipStream_t s) {
  if (mode != NOMIC_EPI_STORE && mode != NOMIC_EPI_SWIGLU && mode != NOMIC_EPI_ROPE) return -1;
  if (K % BK || K / BK < 4 || N % 256 || M <= 0) return -1;
  const long mpad = (M + 255) / 256 * 256;
  if (mpad * lda >= (1L << 31) || (long)N * ldw >= (1L << 31) || M * ldo * 2 >= 0x7fffffffL) return -1;
  if (lda % 8 || ldw % 8 || ldo % 4) return -1;
  if (mode == NOMIC_EPI_ROPE && (!rope || !pos)) return -1;
  if (!g_cus) {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    g_cus = n > 0 ? n : 256;
  }
  const int mtiles = (int)(mpad / 256), ntiles = N / 256, total = mtiles * ntiles;
  int grid = total <= g_cus ? total : (g_cus / 8) * 8;
  int gn = 1;
  for (int g = gn_cap < ntiles ? gn_cap : ntiles; g > 1; --g)
    if (ntiles % g == 0) { gn = g; break; }
  PtArgs ep{out, ldo, rope, pos, rope_cols, M, gn};
  switch (mode) {
    case NOMIC_EPI_STORE: {
      static bool a = (allow_lds(k_gemm_pt<NOMIC_EPI_STORE>, kLdsBytes), true);
      (void)a;
      hipLaunchKernelGGL(k_gemm_pt<NOMIC_EPI_STORE>, dim3(grid), dim3(kThreads), kLdsBytes, s, A, lda, W, ldw, K,
                         mtiles, ntiles, ep);
      break;
    }
    case NOMIC_EPI_SWIGLU: {
      static bool a = (allow_lds(k_gemm_pt<NOMIC_EPI_SWIGLU>, kLdsBytes), true);
      (void)a;
      hipLaunchKernelGGL(k_gemm_pt<NOMIC_EPI_SWIGLU>, dim3(grid), dim3(kThreads), kLdsBytes, s, A, lda, W, ldw, K,
                         mtiles, ntiles, ep);
      break;
    }
    default: {
      static bool a = (allow_lds(k_gemm_pt<NOMIC_EPI_ROPE>, kLdsBytes), true);
      (void)a;
      hipLaunchKernelGGL(k_gemm_pt<NOMIC_EPI_ROPE>, dim3(grid), dim3(kThreads), kLdsBytes, s, A, lda, W, ldw, K,
                         mtiles, ntiles, ep);
      break;
    }
  }
  return (int)hipGetLastError();
}
