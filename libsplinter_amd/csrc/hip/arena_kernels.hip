// arena_kernels.hip — batched format-v4 arena kernels for gfx950 (K1-K6, K9
// of SURVEY §2.10) and their C launchers.
//
// Every launcher takes device pointers and a hipStream_t, so the same entry
// points serve the C++ HBM store (single ops, n = 1), the Python bindings
// (torch tensors' data_ptr on torch's current stream) and the benchmarks.
// Work distribution: 256-thread blocks, grid-stride loop capped at
// 8 blocks/CU x 256 CUs, one op per thread.  Global-epoch increments and
// retry statistics are reduced per block (one atomic per block instead of one
// per op: a single contended word saturates near 88 M atomics/s on MI355X).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "arena_dev.hpp"
#include "arena_api.h"

using namespace spl;
using namespace spl::dev;

namespace {

constexpr int kBlock = 256;
constexpr int kMaxGrid = 256 * 8;

// Segmented batch (routed C1 buffers, parallel/sharded.py): the batch is `n / cap` segments of
// `cap` rows, one per source rank, of which only the first counts[seg] rows are live.  Dead rows
// are skipped (status EINVAL, not counted in the stats).  counts == nullptr: every row is live.
// idx != nullptr (in-place rows, the own-shard ops of a routed step, parallel/xroute.py): row i is
// client op idx[i], and every array the launch takes (keys, values, lens, status, outputs) is a
// client-order array indexed by that op; dead rows are skipped without any write.
struct Seg {
  const int32_t* counts;
  long cap;
  long base = 0;  // row of this launch's element 0 in the segmented buffer (a stream's slice of it)
  const int32_t* idx = nullptr;
  __device__ __forceinline__ bool live(long i) const {
    if (!counts) return true;
    const long j = i + base, s = j / cap;
    return j - s * cap < (long)counts[s];
  }
  __device__ __forceinline__ long row(long i) const { return idx ? (long)idx[i] : i; }
};

inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

inline int grid_for(long n) {
  long g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return (int)(g > kMaxGrid ? kMaxGrid : g);
}
inline int grid_for_b(long n, int b) {  // same resident-thread cap as grid_for, any block size
  long g = (n + b - 1) / b;
  const long cap = (long)kMaxGrid * kBlock / b;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

__device__ __forceinline__ Arena to_dev(const spl_arena_t& a) { return from_api(a); }

// Block-wide sum of a per-thread counter; thread 0 returns the total.
__device__ __forceinline__ uint64_t block_sum(uint64_t v) {
  __shared__ uint64_t part[kBlock / 64];
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) part[wid] = v;
  __syncthreads();
  uint64_t t = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < kBlock / 64; ++w) t += part[w];
  __syncthreads();
  return t;
}

// Per-lane counters of one launch, 32-bit (a lane sees at most its share of the batch times the retry
// bound), widened in flush_stats: 5 registers instead of 10 in the round loops
struct Stats {
  uint32_t attempts = 0, ok = 0, again = 0, miss = 0;
};

__device__ __forceinline__ void flush_stats(const Arena& a, Stats st, uint64_t* stats, uint32_t mutations) {
  const uint64_t at = block_sum(st.attempts);
  const uint64_t ok = block_sum(st.ok);
  const uint64_t ag = block_sum(st.again);
  const uint64_t ms = block_sum(st.miss);
  const uint64_t mu = block_sum(mutations);
  if (threadIdx.x == 0) {
    if (stats) {
      if (at) aadd64(stats + 0, at);
      if (ok) aadd64(stats + 1, ok);
      if (ag) aadd64(stats + 2, ag);
      if (ms) aadd64(stats + 3, ms);
    }
    if (mu) {
      aadd64(&a.hdr()->epoch, mu);
      notify_host(a);
    }
  }
}

// Lanes of one wave retry in lockstep (s_sleep is per wave); progress between
// racing inserters comes from the claim-order rule in set_op, not from timing.
__device__ __forceinline__ void backoff(int attempt) {
  if (attempt < 4) __builtin_amdgcn_s_sleep(1);
  else __builtin_amdgcn_s_sleep(8);
}

// ------------------------------------------------------------- init -----
__global__ void k_init_slots(spl_arena_t aa) {
  const Arena a = to_dev(aa);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < a.slots; i += (size_t)gridDim.x * blockDim.x) {
    uint8_t* s = a.slot(i);
    // zero the 128-B core, then set val_off / type
    for (int c = 0; c < 8; ++c) *(uint4*)(s + 16 * c) = make_uint4(0, 0, 0, 0);
    *(uint32_t*)(s + kOffValOff) = (uint32_t)(i * (size_t)a.max_val);
    *(s + kOffType) = SPL_SLOT_DEFAULT_TYPE;
  }
}

// ------------------------------------------------ cooperative row copy ---
// A wave's round copies up to U*64 value rows (150-B values = 10 x 16 B).  Copied lane-by-op,
// every 16-B wave instruction touches 64 different rows (64 lines); copied here cooperatively,
// 16 lanes take the 16 chunks of one 256-B row and an instruction covers 4 rows (8 lines), with
// 4 instructions' loads in flight.  Entries come from a wave-private LDS table:
// p = {src lo, src hi, dst lo, dst hi}, l = {len (bytes of the value), wend (chunks to write;
// chunks in [ceil(len/16), wend) are zero-filled: mop scrubbing)}.  l.y == 0: no row.
// rowb: bytes of a destination row (value regions are max_val long; a last chunk past it is
// stored bytewise so it cannot spill into the next row); 0xFFFFFFFF: no limit.
// MO: store flavour of the destination rows (st16<MO>); LD1: source rows read with 16-B `sc1` loads
// (L1-bypassing, so a reader needs no L1-invalidating acquire before them).
template <int NE, int MO = 0, bool LD1 = false, int kUnr = 4>
__device__ __forceinline__ void coop_copy(const uint4* __restrict__ ep, const uint2* __restrict__ el, int lane,
                                          int groups, uint32_t rowb) {
  const int q = lane >> 4, cl = lane & 15;
  // kUnr x 4 rows in flight per wave (kUnr 4: 16 rows; the round-1 note: 8 cost 80 VGPRs at 1 wave/SIMD)
  for (int e0 = 0; e0 < NE; e0 += 4 * kUnr) {
    uint4 P[kUnr];
    uint2 L[kUnr];
#pragma unroll
    for (int u = 0; u < kUnr; ++u) {
      P[u] = ep[e0 + 4 * u + q];
      L[u] = el[e0 + 4 * u + q];
    }
    for (int g = 0; g < groups; ++g) {
      const uint32_t c = (uint32_t)(g * 16 + cl);
      uint4 d[kUnr];
      if constexpr (LD1) {
        u32x4c_t t[kUnr];
#pragma unroll
        for (int u = 0; u < kUnr; ++u) {
          const uint32_t n16 = (L[u].x + 15) >> 4;
          const uint4* src = (const uint4*)(((uint64_t)P[u].y << 32) | P[u].x);
          t[u] = u32x4c_t{0u, 0u, 0u, 0u};
          if (c < n16) t[u] = ld16c(src + c);
        }
        static_assert(kUnr % 4 == 0, "each wait ties four loads");
#pragma unroll
        for (int u = 0; u < kUnr; u += 4)
          asm volatile("s_waitcnt vmcnt(0)" : "+v"(t[u]), "+v"(t[u + 1]), "+v"(t[u + 2]), "+v"(t[u + 3])::"memory");
#pragma unroll
        for (int u = 0; u < kUnr; ++u) d[u] = make_uint4(t[u].x, t[u].y, t[u].z, t[u].w);
      } else {
#pragma unroll
        for (int u = 0; u < kUnr; ++u) {
          const uint32_t n16 = (L[u].x + 15) >> 4;
          const uint4* src = (const uint4*)(((uint64_t)P[u].y << 32) | P[u].x);
          d[u] = make_uint4(0, 0, 0, 0);
          if (c < n16) d[u] = src[c];
        }
      }
#pragma unroll
      for (int u = 0; u < kUnr; ++u) {
        if (c >= L[u].y) continue;
        const uint32_t n16 = (L[u].x + 15) >> 4;
        uint4 v = d[u];
        if (c == n16 - 1 && (L[u].x & 15)) {
          const int r = (int)(L[u].x & 15);
          v.x &= keep_mask(r); v.y &= keep_mask(r - 4); v.z &= keep_mask(r - 8); v.w &= keep_mask(r - 12);
        }
        uint4* dst = (uint4*)(((uint64_t)P[u].w << 32) | P[u].z);
        if (c * 16 + 16 > rowb) store_partial((uint8_t*)(dst + c), v, rowb - c * 16);
        else st16<MO>(dst + c, v);
      }
    }
  }
}

// The same copy with the source rows staged through LDS by LDS-DMA (global_load_lds_dwordx4: a
// wave instruction moves 4 rows x 16 chunks into 1 KB of LDS without passing through VGPRs), so NB x 4
// rows are in flight per wave instead of 16 while the registers the round body needs stay free; the
// stores read the chunks back from LDS (ds_read_b128 of the lane's own 16 B) and go out as in
// coop_copy.  One 256-B group per row (max_val <= 256); `stage`: the wave's NB KB of LDS.
// LD1: the DMA carries `sc1` (L1-bypassing, as ld16c).
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base, bool sc1) {
  uint32_t save;
  if (sc1)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(save)
                 : "v"(gsrc), "s"(lds_base)
                 : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(save)
                 : "v"(gsrc), "s"(lds_base)
                 : "memory");
}

// NR > 0: NR more row instructions per batch go through registers beside the NB staged ones
// (4 (NB + NR) rows in flight).
template <int NE, int MO = 0, bool LD1 = false, int NB = 6, int NR = 0>
__device__ __forceinline__ void coop_copy_dma(const uint4* __restrict__ ep, const uint2* __restrict__ el, int lane,
                                              uint32_t rowb, uint4* stage) {
  const int q = lane >> 4, cl = lane & 15;
  const uint32_t sbase =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)stage);
  constexpr int NT = NB + NR;
  auto put = [&](int e, uint4 v, uint32_t c) {  // chunk c of entry e's row: masked, to its destination
    const uint2 L = el[e];
    if (c >= L.y) return;
    const uint32_t n16 = (L.x + 15) >> 4;
    if (c >= n16) v = make_uint4(0, 0, 0, 0);
    if (c == n16 - 1 && (L.x & 15)) {
      const int r = (int)(L.x & 15);
      v.x &= keep_mask(r); v.y &= keep_mask(r - 4); v.z &= keep_mask(r - 8); v.w &= keep_mask(r - 12);
    }
    const uint4 P = ep[e];
    uint4* dst = (uint4*)(((uint64_t)P.w << 32) | P.z);
    if (c * 16 + 16 > rowb) store_partial((uint8_t*)(dst + c), v, rowb - c * 16);
    else st16<MO>(dst + c, v);
  };
  for (int e0 = 0; e0 < NE; e0 += 4 * NT) {
    // issue: row e0 + 4u + q, chunk cl of every instruction u; u < NB into stage[u KB + lane 16 B]
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = e0 + 4 * u + q;
      if (e >= NE) break;
      const uint4 P = ep[e];
      const uint32_t n16 = (el[e].x + 15) >> 4;
      const uint4* src = (const uint4*)(((uint64_t)P.y << 32) | P.x);
      if ((uint32_t)cl < n16) dma16(src + cl, sbase + u * 1024, LD1);
    }
    u32x4c_t t[NR > 0 ? NR : 1];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int e = e0 + 4 * (NB + u) + q;
      t[u] = u32x4c_t{0u, 0u, 0u, 0u};
      if (e < NE) {
        const uint4 P = ep[e];
        const uint32_t n16 = (el[e].x + 15) >> 4;
        const uint4* src = (const uint4*)(((uint64_t)P.y << 32) | P.x);
        if ((uint32_t)cl < n16) t[u] = LD1 ? ld16c(src + cl) : __builtin_bit_cast(u32x4c_t, src[cl]);
      }
    }
    // this wave's DMAs and register loads have landed
    if constexpr (NR == 4)
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3])::"memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = e0 + 4 * u + q;
      if (e >= NE) break;
      put(e, stage[u * 64 + lane], (uint32_t)cl);
    }
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int e = e0 + 4 * (NB + u) + q;
      if (e < NE) put(e, make_uint4(t[u].x, t[u].y, t[u].z, t[u].w), (uint32_t)cl);
    }
    // the next batch's DMAs overwrite the stage: every ds_read of this one has returned
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// ------------------------------------------------ carried-retry rounds -----
// The batched set / get kernels (K2 / K3 of SURVEY §2.10).  U ops per lane per round: U claims
// (or lookups) in flight, then the round's value rows move through the cooperative copy.  An op
// that meets a contended slot (EAGAIN) is NOT retried inline: it stays in its lane's slot and is
// retried in the lane's next round while the lane's other slots take new ops, so a round of other
// work is the natural backoff.  Attempts per op are bounded by 1 + max_retry; the round loop is
// block-uniform (barriers).  Lane sequence: op c of a lane is first + (c / U) * stride + c % U.
// WT: the value rows and slot metadata go out as write-through `sc1` 16-B stores and each wave
// publishes its own ops after its vmcnt(0) drain -- recipe R1 of cdna_hip_programming.md
// Guideline 16 -- so a round needs neither the workgroup barrier pair nor the XCD-serialised L2
// write-back of a release (default; SPLINTER_ARENA_COOP=1: plain rows + one release per round).
template <int U, int B, bool WT>
__global__ __launch_bounds__(B) void k_set_carry(spl_arena_t aa, const char* keys, int kstride, const uint8_t* vals,
                                                 int vstride, const uint32_t* lens, long n, int32_t* status,
                                                 int max_retry, uint64_t* stats, Seg seg) {
  __shared__ uint4 cp_p[B / 64][U * 64];
  __shared__ uint2 cp_l[B / 64][U * 64];
  const Arena a = to_dev(aa);
  bool hybrid;
  const bool scrub = scrub_flags(a, hybrid);
  Stats st;
  uint32_t muts = 0;
  const long stride = (long)gridDim.x * blockDim.x * U;
  const long first = (long)blockIdx.x * blockDim.x * U + (long)threadIdx.x * U;
  long cursor = 0;
  bool more = true;
  Key k[U];
  Claim c[U];
  uint32_t len[U];
  long op[U];
  int tries[U];
  uint64_t ms = maint_begin(a);  // maintenance seq, re-read after every round's drain (arena_dev.hpp)
#pragma unroll
  for (int j = 0; j < U; ++j) op[j] = -1;
  for (;;) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      while (op[j] < 0 && more) {  // refill: next live op of this lane's sequence
        const long i = first + (cursor / U) * stride + (cursor % U);
        ++cursor;
        if (i >= n) { more = false; break; }
        if (!seg.live(i)) {
          if (status && !seg.idx) status[i] = kInval;
          continue;
        }
        const long r = seg.row(i);
        op[j] = r;
        tries[j] = 0;
        load_key(k[j], keys + r * (long)kstride, kstride);
        len[j] = lens[r];
      }
    }
    bool busy = false;
#pragma unroll
    for (int j = 0; j < U; ++j) busy |= op[j] >= 0;
    if (!__syncthreads_or(busy)) break;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      c[j] = Claim{-1, false, kInval};
      if (op[j] >= 0) {
        ++st.attempts;
        ++tries[j];
        if (len[j] == 0 || len[j] > a.max_val || len[j] > (uint32_t)vstride) c[j].rc = kMsgSize;
        else c[j] = claim_set(a, k[j], ms);
      }
    }
    // value rows through the cooperative copy (wave-private table), metadata per lane
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool go = op[j] >= 0 && c[j].rc == kOk;
      const uint64_t sp = go ? (uint64_t)(vals + op[j] * (long)vstride) : 0;
      const uint64_t dp = go ? (uint64_t)a.value((size_t)c[j].idx) : 0;
      cp_p[w][j * 64 + lane] = make_uint4((uint32_t)sp, (uint32_t)(sp >> 32), (uint32_t)dp, (uint32_t)(dp >> 32));
      cp_l[w][j * 64 + lane] = make_uint2(go ? len[j] : 0u, go ? set_chunks(a, len[j], scrub, hybrid) : 0u);
    }
    __builtin_amdgcn_wave_barrier();
    coop_copy<U * 64, WT ? 3 : 0>(cp_p[w], cp_l[w], lane, (int)((a.max_val + 255) >> 8), a.max_val);
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (op[j] >= 0 && c[j].rc == kOk) write_meta<WT ? 3 : 0>(a, c[j], len[j]);
    {
      u32x2c_t mw = ld8c(maint_addr(a));
      vm_wait1(mw);  // = drain(): the round's stores and this load
      ms = u64of(mw);
    }
    if constexpr (!WT) {
      __syncthreads();
      if (threadIdx.x == 0) release();
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (op[j] < 0) continue;
      const int32_t rc = c[j].rc;
      if (rc == kAgain) {
        ++st.again;
        if (tries[j] <= max_retry) continue;  // carried into the next round
      }
      if (rc == kOk) {
        finish_set(a, c[j]);
        ++st.ok;
        ++muts;
        pulse_masks(a, c[j].wm, c[j].bl);
        mark_dirty(a, (size_t)c[j].idx);
      }
      if (status) status[op[j]] = rc;
      op[j] = -1;
    }
  }
  flush_stats(a, st, stats, muts);
}

// FAST: no workgroup acquire.  Every load of slot words and value bytes is an `sc1` load,
// which bypasses the (possibly stale) L1 and is served by the XCD's L2.  That is enough because every
// writer of these bytes (k_set_carry WT, the ring's set) stores them write-through (`sc1`) and drains
// vmcnt before publishing, so no dirty copy lingers in the writer XCD's L2, and an `sc1` load on another
// XCD then returns the written bytes -- the "sc1 stores + sc1 loads" hand-off of the MI355X guide
// (measured, not an architectural guarantee; pinned by tests/test_arena_gpu.py
// test_acquire_free_get_cross_xcd_hot_keys; SPLINTER_ARENA_COOP_GET=1 is the acquire fallback).
// Ops that store with plain (write-back) stores must release before a reader may rely on this (see
// the ring's serve()).  The key is re-checked in the same round trip as the closing (hash, epoch)
// load instead of a separate one before the copy: a key change between the probe and the value
// loads moves the epoch or, for an unset that rewinds it, clears the hash.
template <int U, int B, bool FAST>
__global__ __launch_bounds__(B) void k_get_carry(spl_arena_t aa, const char* keys, int kstride, uint8_t* out,
                                                 int ostride, uint32_t* out_lens, long n, int32_t* status,
                                                 int max_retry, uint64_t* stats, Seg seg) {
  __shared__ uint4 cp_p[B / 64][U * 64];
  __shared__ uint2 cp_l[B / 64][U * 64];
  const Arena a = to_dev(aa);
  Stats st;
  const long stride = (long)gridDim.x * blockDim.x * U;
  const long first = (long)blockIdx.x * blockDim.x * U + (long)threadIdx.x * U;
  long cursor = 0;
  bool more = true;
  Key k[U];
  long op[U], sidx[U];
  uint64_t e1[U];
  int32_t rc[U];
  uint32_t len[U];
  int tries[U];
  uint64_t ms = maint_begin(a);  // maintenance seq, re-read after every round's copies
#pragma unroll
  for (int j = 0; j < U; ++j) op[j] = -1;
  for (;;) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      while (op[j] < 0 && more) {
        const long i = first + (cursor / U) * stride + (cursor % U);
        ++cursor;
        if (i >= n) { more = false; break; }
        if (!seg.live(i)) {
          if (!seg.idx) {
            if (out_lens) out_lens[i] = 0;
            if (status) status[i] = kInval;
          }
          continue;
        }
        const long r = seg.row(i);
        op[j] = r;
        tries[j] = 0;
        load_key(k[j], keys + r * (long)kstride, kstride);
      }
    }
    bool busy = false;
#pragma unroll
    for (int j = 0; j < U; ++j) busy |= op[j] >= 0;
    if (!__syncthreads_or(busy)) break;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      rc[j] = kInval;
      if (op[j] >= 0) {
        ++st.attempts;
        ++tries[j];
        len[j] = 0;
        sidx[j] = locate_peek(a, k[j], &e1[j], &len[j], ms);
        rc[j] = sidx[j] >= 0 ? kOk : sidx[j] == kMaintMiss ? kAgain : kNoEnt;
      }
    }
    if constexpr (FAST) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (op[j] < 0 || rc[j] != kOk) continue;
        if ((e1[j] & 1) || len[j] > a.max_val) rc[j] = kAgain;
        else if (out && len[j] > (uint32_t)ostride) rc[j] = kMsgSize;
      }
    } else {
      drain();
      __syncthreads();
      if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __syncthreads();
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (op[j] < 0 || rc[j] != kOk) continue;
        const uint8_t* s = a.slot((size_t)sidx[j]);
        if ((e1[j] & 1) || len[j] > a.max_val) { rc[j] = kAgain; continue; }
        KeyProbe<16> kp;
        kp.issue(s, k[j]);
        kp.wait();
        if (out && len[j] > (uint32_t)ostride) { rc[j] = kMsgSize; continue; }
        if (!kp.eq(k[j])) rc[j] = kAgain;
      }
    }
    {
      // value rows of this round's matched ops through the cooperative copy (see coop_copy)
      const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const bool go = out && op[j] >= 0 && rc[j] == kOk;
        const uint64_t sp = go ? (uint64_t)a.value((size_t)sidx[j]) : 0;
        const uint64_t dp = go ? (uint64_t)(out + op[j] * (long)ostride) : 0;
        const uint32_t n16 = (len[j] + 15) >> 4;
        cp_p[w][j * 64 + lane] = make_uint4((uint32_t)sp, (uint32_t)(sp >> 32), (uint32_t)dp, (uint32_t)(dp >> 32));
        cp_l[w][j * 64 + lane] = make_uint2(go ? n16 * 16 : 0u, go ? n16 : 0u);
      }
      __builtin_amdgcn_wave_barrier();
      coop_copy<U * 64, 0, FAST>(cp_p[w], cp_l[w], lane, (int)((a.max_val + 255) >> 8), 0xFFFFFFFFu);
    }
    {
      u32x2c_t mw = ld8c(maint_addr(a));
      vm_wait1(mw);  // = drain()
      ms = u64of(mw);
    }
    if constexpr (FAST) {
      // closing round trip: (hash, epoch) and the key words of every op of the lane together
      u32x4c_t he[U];
      KeyProbe<16> kp[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const bool live = op[j] >= 0 && rc[j] == kOk;
        const uint8_t* s = a.slot(live ? (size_t)sidx[j] : 0);
        he[j] = ld16c(s + kOffHash);
        kp[j].issue(s, k[j]);
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        vm_wait(he[j]);
        kp[j].wait();
      }
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (op[j] >= 0 && rc[j] == kOk && (hi64(he[j]) != e1[j] || lo64(he[j]) != k[j].hash || !kp[j].eq(k[j])))
          rc[j] = kAgain;
    } else {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (op[j] < 0 || rc[j] != kOk) continue;
        u32x4c_t he = ld16c(a.slot((size_t)sidx[j]) + kOffHash);  // hash + epoch: one request
        vm_wait(he);
        if (hi64(he) != e1[j] || lo64(he) != k[j].hash) rc[j] = kAgain;
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (op[j] < 0) continue;
      const int32_t r = rc[j];
      if (r == kAgain) {
        ++st.again;
        if (tries[j] <= max_retry) continue;
      }
      if (r == kOk) ++st.ok;
      else if (r == kNoEnt) ++st.miss;
      if (out_lens) out_lens[op[j]] = r == kOk ? len[j] : 0;
      if (status) status[op[j]] = r;
      op[j] = -1;
    }
  }
  flush_stats(a, st, stats, 0);
}

// ------------------------------------------------------- fused set + get -----
// One grid for a whole KV step (spl_kvs_step / spl_kvs_step_xr in fused mode): the step's row
// segments -- the client streams' slices of the set and the get batch, or a routed step's own rows
// (through lidx) and every peer's request block -- are consumed by one launch instead of one
// dispatch per slice.  With 32 + 32 client streams the per-slice dispatches are capped by the
// hardware queues (about 2 set and 2 get dispatches resident at a time, profiles/r3_pmc_kv.md), and
// the step is latency bound (79 % of set wave cycles wait on memory); here every CU holds waves of
// both kinds at once.  The op space is the concatenation of the segments' LIVE rows (a request
// block's count is read on the device); lane sequence as the carried-retry kernels (op c of a lane:
// first + (c / U) * stride + c % U): a round's U slots may hold sets and gets side by side, their
// probes / claims in flight together; the value rows of the two kinds go through two
// cooperative-copy passes (sets: write-through rows into the arena, as k_set_carry WT; gets: sc1
// reads of arena rows, as k_get_carry FAST), then sets publish and gets re-validate.
constexpr int kFusedSegs = 32;  // segments per fused launch (sets + gets; a routed step: 2 x world)

struct FSeg {
  const char* keys;       // row r's key record at keys + row(r) * ks
  uint8_t* vals;          // set: input value rows; get: output rows (null: no value output)
  uint32_t* lens;         // set: input lengths; get: output lengths (nullable)
  int32_t* status;        // per-row status (nullable)
  const int32_t* idx;     // row map (own rows of a routed step), null: identity
  const int32_t* count;   // live rows, read on the device (request blocks), null: n
  long n;                 // rows (upper bound when count is set)
  int vstride;            // value row bytes
  int set;                // 1 set, 0 get
  const int32_t* oidx;    // outputs (status, get lens / values) at row oidx[r] instead of the input
                          // row: a routed step's direct responses into the requester's client arrays
};
static_assert(sizeof(FSeg) == 72, "segment record");

struct FSegs {
  FSeg s[kFusedSegs];
  int n;
  int ks;
};

// A lane's U op slots in the fused / server round loops.  OI: segments may map outputs elsewhere
// (FSeg::oidx, the routed step's direct responses); without it the output row is the input row and
// costs no register.
template <int U, int KW, bool OI = false>
struct OpSlots {
  KeyT<KW> k[U];
  long row[U];
  int32_t orow[OI ? U : 1];
  int seg[U];  // -1: slot empty
  uint32_t len[U];
  int tries[U];
  bool set[U];
};
template <int U, int KW, bool OI>
__device__ __forceinline__ long out_row(const OpSlots<U, KW, OI>& o, int j) {
  if constexpr (OI) return (long)o.orow[j];
  else return o.row[j];
}

// Put row r of segment q (sg[q]) into the empty slot j.
template <int U, int KW, bool OI>
__device__ __forceinline__ void fill_slot(OpSlots<U, KW, OI>& o, int j, const FSeg& f, int q, long r, int ks) {
  o.seg[j] = q;
  o.row[j] = f.idx ? (long)f.idx[r] : r;
  if constexpr (OI) o.orow[j] = f.oidx ? f.oidx[r] : (int32_t)o.row[j];
  o.set[j] = f.set != 0;
  o.tries[j] = 0;
  load_key(o.k[j], f.keys + o.row[j] * (long)ks, ks);
  o.len[j] = o.set[j] ? f.lens[o.row[j]] : 0u;
}

// One round over a lane's U slots: probes / claims of every occupied slot, the two cooperative row
// copies (cp*0: set rows, cp*1: get rows; a wave-private LDS table each), set publication, get
// re-validation, completion.  An op that met EAGAIN stays in its slot for the next round while
// tries <= max_retry.  Called by every lane of the wave (the row copies are wave-cooperative).
// ms: the arena's maintenance seq as read (and waited for) before this round's probes; re-read in
// the round's closing round trip for the next round (arena_dev.hpp, online maintenance).
// flags: kKvSkipLen (an update that keeps its length leaves val_len alone).  (Measured and removed in
// round 6: a get's home-slot value row requested by LDS-DMA beside its probe, 4.45-4.47 vs 4.84-4.88 G
// ops/s KV-only: the extra requests cost more than the row copy's L2 hit saves, profiles/r6/README.md.)
constexpr int kKvSkipLen = 1;
// kKvCopyDma: the round's row copies stage their source rows through LDS by LDS-DMA (coop_copy_dma)
constexpr int kKvCopyDma = 4;
// (SPL_KVS_COPY_DMA=1, default: KV-only 5.15-5.29 vs 4.92-4.99 G ops/s; 16 more rows per batch through
// registers beside the staged 24 measured the same, 5.21-5.30: profiles/r6/README.md)
constexpr int kKvStageKB = 6;  // LDS-DMA stage per wave (KB): 24 rows in flight
// kKvPadOut (SPL_KVS_PAD_OUT, default 1): a get's output row is written through the next 64-B boundary
// inside its stride (zeros past the value), so the row's last line is a whole-line write, not a partial
// one (a read-modify-write below the HBM3E ECC granule): KV-only 5.35-5.47 vs 5.15-5.24 G ops/s, mixed
// step 12.06-12.10 vs 12.30 ms (profiles/r6/README.md)
constexpr int kKvPadOut = 8;
template <int U, int KW, bool OI = false>
__device__ __forceinline__ void kv_round(const Arena& a, const FSeg* sg, OpSlots<U, KW, OI>& o, bool scrub, bool hybrid,
                                         int max_retry, Stats& st, uint32_t& muts, uint4* cpp0, uint2* cpl0,
                                         uint4* cpp1, uint2* cpl1, int lane, int flags, uint64_t& ms,
                                         uint4* stage = nullptr) {
  const bool skip_len = flags & kKvSkipLen;
  Claim c[U];
  long sidx[U];
  uint64_t e1[U];
  int32_t rc[U];
  // probes / claims of every slot of the round
#pragma unroll
  for (int j = 0; j < U; ++j) {
    rc[j] = kInval;
    c[j] = Claim{-1, false, kInval};
    if (o.seg[j] < 0) continue;
    ++st.attempts;
    ++o.tries[j];
    const int vs = sg[o.seg[j]].vstride;
    if (o.set[j]) {
      if (o.len[j] == 0 || o.len[j] > a.max_val || o.len[j] > (uint32_t)vs) c[j].rc = kMsgSize;
      else c[j] = claim_set(a, o.k[j], ms);
      rc[j] = c[j].rc;
    } else {
      uint32_t L = 0;
      sidx[j] = locate_peek(a, o.k[j], &e1[j], &L, ms);
      o.len[j] = L;
      rc[j] = sidx[j] >= 0 ? kOk : sidx[j] == kMaintMiss ? kAgain : kNoEnt;
      if (rc[j] == kOk && ((e1[j] & 1) || L > a.max_val)) rc[j] = kAgain;
      else if (rc[j] == kOk && sg[o.seg[j]].vals && L > (uint32_t)vs) rc[j] = kMsgSize;
    }
  }
  // an update that keeps its length leaves val_len alone (SPL_KVS_SKIP_LEN, default 1: KV-only 4.94-4.96
  // vs 4.85-4.89 G ops/s, profiles/r5/kv_skip_len.md): the held claim
  // makes the slot's val_len stable, and a 4-B write is a partial-line write (read-modify-write
  // below the 64-B ECC granule of HBM3E); the loads are issued here and consumed after the row copies
  uint32_t oldlen[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    oldlen[j] = 0xFFFFFFFFu;
    if (skip_len && o.seg[j] >= 0 && o.set[j] && rc[j] == kOk && !c[j].fresh)
      oldlen[j] = ald32(a.slot((size_t)c[j].idx) + kOffValLen);
  }
  // value rows: table 0 = sets (client row -> arena, write-through), table 1 = gets (arena -> client)
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const FSeg* f = o.seg[j] >= 0 ? &sg[o.seg[j]] : nullptr;
    const bool gs = f && o.set[j] && rc[j] == kOk;
    const bool gg = f && f->vals && !o.set[j] && rc[j] == kOk;
    const uint64_t ss = gs ? (uint64_t)(f->vals + o.row[j] * (long)f->vstride) : 0;
    const uint64_t sd = gs ? (uint64_t)a.value((size_t)c[j].idx) : 0;
    cpp0[j * 64 + lane] = make_uint4((uint32_t)ss, (uint32_t)(ss >> 32), (uint32_t)sd, (uint32_t)(sd >> 32));
    cpl0[j * 64 + lane] = make_uint2(gs ? o.len[j] : 0u, gs ? set_chunks(a, o.len[j], scrub, hybrid) : 0u);
    const uint64_t gsrc = gg ? (uint64_t)a.value((size_t)sidx[j]) : 0;
    const uint64_t gdst = gg ? (uint64_t)(f->vals + out_row(o, j) * (long)f->vstride) : 0;
    const uint32_t n16 = (o.len[j] + 15) >> 4;
    cpp1[j * 64 + lane] = make_uint4((uint32_t)gsrc, (uint32_t)(gsrc >> 32), (uint32_t)gdst, (uint32_t)(gdst >> 32));
    // kKvPadOut: the output row is written to the next 64-B boundary (zeros past the value, inside the
    // row's stride), so its last line is a whole-line write instead of a partial one
    uint32_t wend = n16;
    if ((flags & kKvPadOut) && gg) {
      const uint32_t pad = (n16 + 3u) & ~3u, cap = (uint32_t)f->vstride >> 4;
      wend = pad < cap ? pad : (cap > n16 ? cap : n16);
    }
    cpl1[j * 64 + lane] = make_uint2(gg ? n16 * 16 : 0u, gg ? wend : 0u);
  }
  __builtin_amdgcn_wave_barrier();
#ifndef SPL_KV_COPY_UNR
#define SPL_KV_COPY_UNR 4
#endif
#ifndef SPL_KV_DIAG_NO_COPY
  if ((flags & kKvCopyDma) && stage && a.max_val <= 256) {
    coop_copy_dma<U * 64, 3, false, kKvStageKB>(cpp0, cpl0, lane, a.max_val, stage);
    coop_copy_dma<U * 64, 0, true, kKvStageKB>(cpp1, cpl1, lane, 0xFFFFFFFFu, stage);
  } else {
    coop_copy<U * 64, 3, false, SPL_KV_COPY_UNR>(cpp0, cpl0, lane, (int)((a.max_val + 255) >> 8), a.max_val);
    coop_copy<U * 64, 0, true, SPL_KV_COPY_UNR>(cpp1, cpl1, lane, (int)((a.max_val + 255) >> 8), 0xFFFFFFFFu);
  }
#endif
#pragma unroll
  for (int j = 0; j < U; ++j)
    if (o.seg[j] >= 0 && o.set[j] && rc[j] == kOk && oldlen[j] != o.len[j]) write_meta<3>(a, c[j], o.len[j]);
  drain();
  // gets: closing round trip, (hash, epoch) and the key words together
  {
    u32x4c_t he[U];
    KeyProbe<KW> kp[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool live = o.seg[j] >= 0 && !o.set[j] && rc[j] == kOk;
      const uint8_t* s = a.slot(live ? (size_t)sidx[j] : 0);
      he[j] = ld16c(s + kOffHash);
      kp[j].issue(s, o.k[j]);
    }
    u32x2c_t mw = ld8c(maint_addr(a));  // the next round's maintenance seq, in the same round trip
#pragma unroll
    for (int j = 0; j < U; ++j) {
      vm_wait(he[j]);
      kp[j].wait();
    }
    vm_wait1(mw);
    ms = u64of(mw);
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (o.seg[j] >= 0 && !o.set[j] && rc[j] == kOk &&
          (hi64(he[j]) != e1[j] || lo64(he[j]) != o.k[j].hash || !kp[j].eq(o.k[j])))
        rc[j] = kAgain;
  }
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if (o.seg[j] < 0) continue;
    const int32_t r = rc[j];
    if (r == kAgain) {
      ++st.again;
      if (o.tries[j] <= max_retry) continue;  // carried into the next round
    }
    const FSeg& f = sg[o.seg[j]];
    if (o.set[j]) {
      if (r == kOk) {
        finish_set(a, c[j]);
        ++st.ok;
        ++muts;
        pulse_masks(a, c[j].wm, c[j].bl);
        mark_dirty(a, (size_t)c[j].idx);
      }
    } else {
      if (r == kOk) ++st.ok;
      else if (r == kNoEnt) ++st.miss;
      if (f.lens) f.lens[out_row(o, j)] = r == kOk ? o.len[j] : 0;
    }
    if (f.status) f.status[out_row(o, j)] = r;
    o.seg[j] = -1;
  }
}

// SCHED, how a workgroup's lanes get their rows and when its round loop ends:
//   0 kSchedBarrier: fixed lane streams (lane i of the grid: rows i, i + stride, ...), the loop's exit
//     test a workgroup barrier each round (the round-5 form);
//   1 kSchedChunks: workgroups claim chunks of rows from a launch-wide counter (shrinking toward the
//     end), so they finish together.  The counter word is [tag (24 bits) | rows claimed (40)]: a launch
//     owns a word of its context's ring (KvStreams::claim_slot) under its own tag, and the first claim
//     that finds another tag there installs this launch's with one CAS, every claim then one atomic add;
//   2 kSchedWaves (default): fixed lane streams, the exit test a wave vote, so the four waves of a
//     group never wait for each other.
// Per-wave chunk claims were measured too and lost (the claim round trip stalls the whole wave;
// profiles/r6/README.md).
constexpr int kSchedBarrier = 0, kSchedChunks = 1, kSchedWaves = 2;
template <int U, int B, int KW = 16, int OCC = 1, bool OI = false, int SCHED = kSchedBarrier>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(OCC))) void k_kv_fused(spl_arena_t aa, FSegs tab,
                                                                                         int max_retry, uint64_t* stats,
                                                                                         int skip_len,
                                                                                         unsigned long long* claim,
                                                                                         uint32_t tag, long chunk,
                                                                                         int chunk_div) {
  __shared__ uint4 cp_p[2][B / 64][U * 64];
  __shared__ uint2 cp_l[2][B / 64][U * 64];
  __shared__ uint4 cp_stage[B / 64][kKvStageKB * 64];  // kKvCopyDma: the waves' LDS-DMA stages
  __shared__ FSeg sg[kFusedSegs];
  __shared__ long sstart[kFusedSegs + 1];
  __shared__ long sh_c, sh_cs;  // kSchedChunks: the claimed chunk's first row and size
  const int nseg = tab.n, ks = tab.ks;
  if ((int)threadIdx.x < nseg) {
    FSeg f = tab.s[threadIdx.x];
    if (f.count) {
      const long c = (long)*f.count;
      f.n = c < 0 ? 0 : (c < f.n ? c : f.n);
    }
    sg[threadIdx.x] = f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long run = 0;
    for (int q = 0; q < nseg; ++q) {
      sstart[q] = run;
      run += sg[q].n;
    }
    sstart[nseg] = run;
  }
  __syncthreads();
  const Arena a = to_dev(aa);
  bool hybrid;
  const bool scrub = scrub_flags(a, hybrid);
  Stats st;
  uint32_t muts = 0;
  const long n = sstart[nseg];
  const long stride = (long)gridDim.x * blockDim.x * U;
  const long first = (long)blockIdx.x * blockDim.x * U + (long)threadIdx.x * U;
  long cursor = 0;
  bool more = true;
  OpSlots<U, KW, OI> o;
#pragma unroll
  for (int j = 0; j < U; ++j) o.seg[j] = -1;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint64_t ms = maint_begin(a);
  int32_t row = 0, end = 0;  // kSchedChunks: the lane's next row of the group's chunk, the chunk's end (< 2^31)
  int part = 0;
  for (;;) {
    if constexpr (SCHED == kSchedChunks) {
      if (more && !__syncthreads_or(row < end)) {  // no lane has rows of the chunk left: claim the next
        if (threadIdx.x == 0) {
          const long left = n - (end > 0 ? end : 0);
          long c = left / ((long)chunk_div * gridDim.x);
          c = c < chunk ? c : chunk;
          c = c > (long)B * U ? c : (long)B * U;
          // the word still carries an older launch's tag: install ours with a zero count (one CAS of the
          // launch wins, the others fail once); then every claim is one atomic add
          unsigned long long cur = __hip_atomic_load(claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((cur >> 40) != tag)
            __hip_atomic_compare_exchange_strong(claim, &cur, (unsigned long long)tag << 40, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sh_c = (long)(atomicAdd(claim, (unsigned long long)c) & ((1ull << 40) - 1));
          sh_cs = c;
        }
        __syncthreads();
        const long c0 = sh_c, cs = sh_cs;
        if (c0 >= n) {
          more = false;
        } else {
          row = (int32_t)(c0 + (long)threadIdx.x * U);
          end = (int32_t)(c0 + cs < n ? c0 + cs : n);
          part = 0;
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (o.seg[j] < 0 && row < end) {
          int q = 0;
          while (q + 1 < nseg && sstart[q + 1] <= row) ++q;
          fill_slot(o, j, sg[q], q, row - sstart[q], ks);
          if (++part == U) {
            part = 0;
            row += B * U - (U - 1);
          } else {
            ++row;
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (o.seg[j] < 0 && more) {
          const long i = first + (cursor / U) * stride + (cursor % U);
          ++cursor;
          if (i >= n) {
            more = false;
          } else {
            int q = 0;
            while (q + 1 < nseg && sstart[q + 1] <= i) ++q;
            fill_slot(o, j, sg[q], q, i - sstart[q], ks);
          }
        }
      }
    }
    bool busy = false;
#pragma unroll
    for (int j = 0; j < U; ++j) busy |= o.seg[j] >= 0;
    if (!(SCHED == kSchedWaves ? __any(busy) : __syncthreads_or(busy))) {
      if (SCHED == kSchedChunks && more) continue;  // (uniform: every lane's chunk rows are used up) the next claim
      break;
    }
    kv_round<U, KW, OI>(a, sg, o, scrub, hybrid, max_retry, st, muts, cp_p[0][w], cp_l[0][w], cp_p[1][w], cp_l[1][w], lane,
                    skip_len, ms, cp_stage[w]);
  }
  flush_stats(a, st, stats, muts);
}

// ------------------------------------------------------ stream-posted server --
// Asynchronous submission of a KV step (spl_kvs_set_fused mode 3): every client stream posts its
// slice with a stream-ordered doorbell write (hipStreamWriteValue64 of the step's sequence number
// into AsyncCtl::door[slot]) once its own preceding work is done, and ONE resident grid on the
// server stream consumes the slices as they are posted: a workgroup claims a chunk of rows of a
// posted slice (atomic on AsyncCtl::next[slot]), runs the fused round loop over it, and claims the
// next, so slices start independently, in the order their streams reach the post, and no slice
// waits for the others.  Slice boundaries are multiples of kAsyncAlign rows, so two slices never
// share a cache line of the keys / values / outputs.  The grid ends when every slice is exhausted,
// or -- a post that never comes -- after wait_ticks of s_memrealtime (100 MHz) without finding any
// work, with AsyncCtl::err set (spl_kvs_async_error); every wave reaches one of the two exits.
constexpr int kAsyncSegs = 64;     // client streams per server step (writers + readers)
constexpr long kAsyncAlign = 128;  // slice boundary granularity (rows)

struct AsyncCtl {
  uint64_t door[kAsyncSegs];                 // last step sequence posted by each client stream
  unsigned long long next[2][kAsyncSegs];    // rows of each slice claimed so far, banked by the step's
                                             // parity: a server zeroes the other bank for the next step
  uint32_t err;                              // a post did not arrive within the wait limit
  uint32_t pad[15];
};

__host__ __device__ inline long async_bound(long n, int i, int parts) {  // first row of slice i of n rows
  if (i <= 0) return 0;
  if (i >= parts) return n;
  const long b = (n * i / parts + kAsyncAlign - 1) / kAsyncAlign * kAsyncAlign;
  return b < n ? b : n;
}

// WV: inside a chunk each wave runs its rows' rounds on its own (the loop's exit a wave vote) and the
// waves meet only at the next claim, as the fused grid's kSchedWaves form
template <int U, int B, int KW = 16, int OCC = 1, bool WV = false>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(OCC))) void k_kv_server(
    spl_arena_t aa, FSeg sset, FSeg sget, int nw, int nr, int ks, AsyncCtl* ctl, uint64_t seq, long chunk,
    uint64_t wait_ticks, int spread, int max_retry, uint64_t* stats, int skip_len) {
  __shared__ uint4 cp_p[2][B / 64][U * 64];
  __shared__ uint2 cp_l[2][B / 64][U * 64];
  __shared__ uint4 cp_stage[B / 64][kKvStageKB * 64];  // kKvCopyDma: the waves' LDS-DMA stages
  __shared__ FSeg sg[2];  // 0: the set batch, 1: the get batch
  __shared__ long sh_b, sh_e;
  __shared__ int sh_kind, sh_state, sh_scan;
  __shared__ uint64_t sh_exhausted, sh_posted, sh_idle;  // thread 0's scan state (LDS: no registers)
  __shared__ unsigned long long sh_st[5];  // attempts, ok, again, miss, mutations of the chunks run
  __shared__ long sh_tb[kAsyncSegs], sh_te[kAsyncSegs];  // timeout: rows of unposted slices this group took
  const int nseg = nw + nr;
  if (threadIdx.x < 5) sh_st[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    sg[0] = sset;
    sg[1] = sget;
    sh_exhausted = 0;
    sh_posted = 0;
    // first slice looked at: spread over the slices (1) or in post-slot order, writers first (0);
    // 2 (diagnosis only): every slice taken as posted
    sh_scan = spread ? (int)(blockIdx.x % (unsigned)nseg) : 0;
    sh_idle = __builtin_amdgcn_s_memrealtime();
  }
  const Arena a = to_dev(aa);
  bool hybrid;
  const bool scrub = scrub_flags(a, hybrid);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long long* next = ctl->next[seq & 1];
  if (blockIdx.x == 0 && threadIdx.x < kAsyncSegs)  // the next step's bank (its last user has ended)
    __hip_atomic_store(&ctl->next[(seq + 1) & 1][threadIdx.x], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // A lane's op slots live across chunks: an op that met EAGAIN is carried into the next chunk's
  // rounds (as in the fused grid) instead of holding the workgroup in extra, mostly empty rounds at
  // the end of every chunk
  OpSlots<U, KW> o;
#pragma unroll
  for (int j = 0; j < U; ++j) o.seg[j] = -1;
  Stats st;
  uint32_t muts = 0;
  uint64_t ms = maint_begin(a);
  for (;;) {
    __syncthreads();  // the previous chunk's readers of sh_* are done
    if (w == 0) {
      // wave 0 claims: lane i looks at slice i (its post and how far it is claimed) in one round
      // trip for all slices, then the first available slice at or after the last one served (a
      // workgroup stays on a slice while it lasts) gets the atomic claim.  The lane index is
      // laundered per claim: values derived from it are recomputed here (once per chunk) instead of
      // being hoisted out of the loop and held -- spilled -- across the round body
      int lane = threadIdx.x & 63;
      asm volatile("" : "+v"(lane));
      const uint64_t all = nseg >= 64 ? ~0ull : ((1ull << nseg) - 1);
      uint64_t exhausted = sh_exhausted, posted = sh_posted;
      const int scan = sh_scan;
      bool p = false, av = false;
      long b = 0, e = 0;
      if (lane < nseg && !((exhausted >> lane) & 1)) {
        const bool isset = lane < nw;
        const int parts = isset ? nw : nr, pi = isset ? lane : lane - nw;
        const long n = sg[isset ? 0 : 1].n;
        b = async_bound(n, pi, parts);
        e = async_bound(n, pi + 1, parts);
        // slot i is always rung by client stream i, in that stream's order, so door >= seq: this
        // step's post has happened (an empty slice needs none)
        p = b >= e || spread >= 2 || ((posted >> lane) & 1) ||
            __hip_atomic_load(&ctl->door[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= seq;
        if (p && b < e) {
          const long nx = (long)__hip_atomic_load(&next[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          av = b + nx < e;  // next only grows: "not available" is final
        }
      }
      posted |= __ballot(p);
      exhausted |= __ballot(p && !av);
      uint64_t avm = __ballot(av);
      int state = 0, pick = scan;
      long cb = 0, ce = 0;
      while (avm) {
        const uint64_t up = avm & (~0ull << scan);
        const int i = __builtin_ctzll(up ? up : avm);
        long c = 0;
        if (lane == i) c = (long)atomicAdd(&next[i], (unsigned long long)chunk);
        c = __shfl(c, i);
        const long bi = __shfl(b, i), ei = __shfl(e, i);
        if (bi + c < ei) {
          cb = bi + c;
          ce = cb + chunk < ei ? cb + chunk : ei;
          pick = i;
          state = 1;
          break;
        }
        avm &= ~(1ull << i);
        exhausted |= 1ull << i;
      }
      int timed = 0;
      if (lane == 0) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (state == 1) {
          sh_idle = now;
          sh_kind = pick < nw ? 0 : 1;
          sh_b = cb;
          sh_e = ce;
          // the slice's keys / values were written by the client stream's work before its post:
          // an agent acquire after the poll, before any wave of the group reads them (this CU's L1
          // may hold lines of the previous step's rows), MI355X guide "Valid forms", consumer side
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (exhausted == all) {
          state = 2;
        } else if (now - sh_idle > wait_ticks) {
          __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          state = 2;
          timed = 1;
        }
        sh_exhausted = exhausted;
        sh_posted = posted;
        sh_scan = pick;
        sh_state = state;
      }
      // a post that never came: every row of an unposted slice that no group has claimed is taken
      // (one claim of the whole remainder) and reported EAGAIN, so no status is left stale
      timed = __shfl(timed, 0, 64);
      long tb = 0, te = 0;
      if (timed && lane < nseg && !((exhausted >> lane) & 1) && !((posted >> lane) & 1) && b < e) {
        const long c = (long)atomicAdd(&next[lane], (unsigned long long)(e - b));
        if (b + c < e) {
          tb = b + c;
          te = e;
        }
      }
      if (lane < kAsyncSegs) {
        sh_tb[lane] = tb;
        sh_te[lane] = te;
      }
    }
    __syncthreads();
    const int state = sh_state;
    if (state == 2) {
      for (int i = 0; i < nseg; ++i) {
        const FSeg& f = sg[i < nw ? 0 : 1];
        for (long r = sh_tb[i] + (long)threadIdx.x; r < sh_te[i]; r += B) {
          if (f.status) f.status[r] = kAgain;
          if (!f.set && f.lens) f.lens[r] = 0;
        }
      }
      break;
    }
    bool carried = false;
#pragma unroll
    for (int j = 0; j < U; ++j) carried |= o.seg[j] >= 0;
    carried = __syncthreads_or(carried);
    if (state == 0) {
      // nothing claimable yet: carried ops still progress
      if (carried)
        kv_round<U, KW>(a, sg, o, scrub, hybrid, max_retry, st, muts, cp_p[0][w], cp_l[0][w], cp_p[1][w], cp_l[1][w],
                        lane, skip_len, ms, cp_stage[w]);
      else
        __builtin_amdgcn_s_sleep(32);
      continue;
    }
    const int q = sh_kind;
    const long end = sh_e;
    long row = sh_b + (long)threadIdx.x * U;  // the lane's next row: U consecutive rows per B * U
    int part = 0;
    for (;;) {
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (o.seg[j] < 0 && row < end) {
          fill_slot(o, j, sg[q], q, row, ks);
          if (++part == U) {
            part = 0;
            row += (long)B * U - (U - 1);
          } else {
            ++row;
          }
        }
      }
      bool busy = false;
#pragma unroll
      for (int j = 0; j < U; ++j) busy |= o.seg[j] >= 0;
      // once no lane has rows of this chunk left the group claims the next one; the ops still in
      // slots (the chunk's last fills, carried retries) ride along into its rounds
      const bool more = row < end;
      if (!(WV ? __any(more && busy) : __syncthreads_or(more && busy))) break;
      kv_round<U, KW>(a, sg, o, scrub, hybrid, max_retry, st, muts, cp_p[0][w], cp_l[0][w], cp_p[1][w], cp_l[1][w],
                      lane, skip_len, ms, cp_stage[w]);
    }
  }
  // the last chunk's ops and any carried retries
  for (;;) {
    bool busy = false;
#pragma unroll
    for (int j = 0; j < U; ++j) busy |= o.seg[j] >= 0;
    if (!(WV ? __any(busy) : __syncthreads_or(busy))) break;
    kv_round<U, KW>(a, sg, o, scrub, hybrid, max_retry, st, muts, cp_p[0][w], cp_l[0][w], cp_p[1][w], cp_l[1][w], lane,
                    skip_len, ms, cp_stage[w]);
  }
  __syncthreads();  // (WV: every wave's drain is done before the group's totals are read)
  {
    const uint64_t v[5] = {st.attempts, st.ok, st.again, st.miss, muts};
#pragma unroll
    for (int c = 0; c < 5; ++c)
      if (v[c]) __hip_atomic_fetch_add(&sh_st[c], (unsigned long long)v[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (stats)
      for (int c = 0; c < 4; ++c)
        if (sh_st[c]) aadd64(stats + c, sh_st[c]);
    if (sh_st[4]) {
      aadd64(&a.hdr()->epoch, sh_st[4]);
      notify_host(a);
    }
  }
}

// CUs a stream's kernels may occupy: the popcount of its CU mask (the whole device for an unmasked
// stream; a runtime query, no device round trip)
int stream_cus(hipStream_t s) {
  int dev = 0, n = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  uint32_t m[16] = {};
  if (s != nullptr && hipExtStreamGetCUMask(s, 16, m) == hipSuccess) {
    int c = 0;
    for (uint32_t w : m) c += __builtin_popcount(w);
    if (c > 0 && c < n) n = c;
  } else {
    (void)hipGetLastError();
  }
  return n;
}

// Launch the fused grid over `tab` (rows: an upper bound of the live rows); mode 2 with 16-B keys
// holds them in 4 words at 3 workgroups per CU, otherwise 16 words at 2
int launch_fused(spl_arena_t a, const FSegs& tab, long rows, int mode, int max_retry, uint64_t* stats,
                 hipStream_t s, unsigned long long* claim = nullptr, uint32_t tag = 0, int sched_set = -1) {
  if (rows <= 0) return 0;
  // (measured and removed: 4 workgroups per CU at <= 128 VGPRs, 34 spilled: 4.43 vs 4.84 G ops/s,
  // profiles/r4k/kv_fused3.out)
  const bool kw4 = mode >= 2 && tab.ks == 16;
  static const int wpc_env = env_int("SPL_KVS_FUSED_WG_PER_CU", 0);
  const int wpc = wpc_env > 0 ? wpc_env : kw4 ? 3 : 2;
  const long need = (rows + 2 * 256 - 1) / (2 * 256);
  // the grid is resident (every workgroup walks its lane stream to the end): sized to the CUs the
  // launch stream may use, so a CU-masked stream (hipExtStreamCreateWithCUMask) gets no second wave
  const long cap = (long)stream_cus(s) * wpc;
  const dim3 g((unsigned)(need < cap ? need : cap));
  // SPL_KVS_SKIP_LEN (A/B knob): kv_round flags
  static const int skip_len = (env_int("SPL_KVS_SKIP_LEN", 1) ? kKvSkipLen : 0) |
                              (env_int("SPL_KVS_COPY_DMA", 1) ? kKvCopyDma : 0) |
                              (env_int("SPL_KVS_PAD_OUT", 1) ? kKvPadOut : 0);
  // segments with an output map (direct routed responses) take the OI form of the grid
  bool oi = false;
  for (int q = 0; q < tab.n; ++q) oi |= tab.s[q].oidx != nullptr;
  // SPL_KVS_SCHED (kSched*, above): 2 = fixed lane streams with the wave-vote exit (default), 1 = workgroup
  // chunk claims (SPL_KVS_CHUNK rows at most, shrinking to (rows left) / (SPL_KVS_CHUNK_DIV x groups)),
  // 0 = fixed lane streams with the per-round workgroup barrier.  KV-only 4.97-4.99 / 4.97-5.00 /
  // 4.74-4.84 G ops/s (profiles/r6/kv_dyn_chunks.jsonl)
  static const int sched_env = env_int("SPL_KVS_SCHED", kSchedWaves);
  const int sched = sched_set >= 0 ? sched_set : sched_env;  // spl_kvs_set_sched, else the environment
  static const long dchunk = std::max(512, env_int("SPL_KVS_CHUNK", 4096));
  static const int ddiv = std::max(1, env_int("SPL_KVS_CHUNK_DIV", 2));
  if (kw4 && sched == kSchedChunks && claim && rows < (1L << 31) - (1L << 20)) {
    if (oi)
      hipLaunchKernelGGL((k_kv_fused<2, 256, 4, 3, true, kSchedChunks>), g, dim3(256), 0, s, a, tab, max_retry, stats,
                         skip_len, claim, tag, dchunk, ddiv);
    else
      hipLaunchKernelGGL((k_kv_fused<2, 256, 4, 3, false, kSchedChunks>), g, dim3(256), 0, s, a, tab, max_retry,
                         stats, skip_len, claim, tag, dchunk, ddiv);
  } else if (kw4 && sched == kSchedWaves) {
    if (oi)
      hipLaunchKernelGGL((k_kv_fused<2, 256, 4, 3, true, kSchedWaves>), g, dim3(256), 0, s, a, tab, max_retry, stats,
                         skip_len, nullptr, 0u, 0L, 1);
    else
      hipLaunchKernelGGL((k_kv_fused<2, 256, 4, 3, false, kSchedWaves>), g, dim3(256), 0, s, a, tab, max_retry,
                         stats, skip_len, nullptr, 0u, 0L, 1);
  } else if (kw4 && oi)
    hipLaunchKernelGGL((k_kv_fused<2, 256, 4, 3, true>), g, dim3(256), 0, s, a, tab, max_retry, stats, skip_len,
                       nullptr, 0u, 0L, 1);
  else if (kw4)
    hipLaunchKernelGGL((k_kv_fused<2, 256, 4, 3>), g, dim3(256), 0, s, a, tab, max_retry, stats, skip_len, nullptr,
                       0u, 0L, 1);
  else if (oi && sched == kSchedWaves)
    hipLaunchKernelGGL((k_kv_fused<2, 256, 16, 1, true, kSchedWaves>), g, dim3(256), 0, s, a, tab, max_retry, stats,
                       skip_len, nullptr, 0u, 0L, 1);
  else if (oi)
    hipLaunchKernelGGL((k_kv_fused<2, 256, 16, 1, true>), g, dim3(256), 0, s, a, tab, max_retry, stats, skip_len,
                       nullptr, 0u, 0L, 1);
  else if (sched == kSchedWaves)
    hipLaunchKernelGGL((k_kv_fused<2, 256, 16, 1, false, kSchedWaves>), g, dim3(256), 0, s, a, tab, max_retry, stats,
                       skip_len, nullptr, 0u, 0L, 1);
  else
    hipLaunchKernelGGL((k_kv_fused<2, 256>), g, dim3(256), 0, s, a, tab, max_retry, stats, skip_len, nullptr, 0u, 0L, 1);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------- unset ----
__global__ __launch_bounds__(kBlock) void k_unset(spl_arena_t aa, const char* keys, int kstride, long n,
                                                  int32_t* status, int max_retry) {
  const Arena a = to_dev(aa);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    Key k;
    load_key(k, keys + i * (long)kstride, kstride);
    long idx = -1;
    int32_t rc = kAgain;
    for (int t = 0; t <= max_retry; ++t) {
      rc = unset_op(a, k, &idx);
      if (rc != kAgain) break;
      backoff(t);
    }
    if (status) status[i] = rc;
  }
}

// ------------------------------------------------------------- integer --
__global__ __launch_bounds__(kBlock) void k_intop(spl_arena_t aa, const char* keys, int kstride, const int* ops,
                                                  const uint64_t* masks, long n, int32_t* status, uint64_t* results,
                                                  int max_retry) {
  const Arena a = to_dev(aa);
  uint32_t muts = 0;
  Stats st;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    Key k;
    load_key(k, keys + i * (long)kstride, kstride);
    long idx = -1;
    uint64_t r = 0;
    int32_t rc = kAgain;
    for (int t = 0; t <= max_retry; ++t) {
      rc = integer_op(a, k, ops[i], masks ? masks[i] : 0, &r, &idx);
      if (rc != kAgain) break;
      backoff(t);
    }
    if (rc == kOk) { ++muts; mark_dirty(a, (size_t)idx); }
    if (results) results[i] = r;
    if (status) status[i] = rc;
  }
  flush_stats(a, st, nullptr, muts);
}

// ------------------------------------------------- keyed metadata ops ----
// op: 0 set_label, 1 unset_label, 2 bump, 3 get_epoch, 4 watch_register,
//     5 watch_unregister, 6 pulse_keygroup, 7 set_as_system, 8 retrain,
//     9 set_named_type (arg = mask; no BIGUINT promotion: see host path),
//     10 set ctime, 11 set atime, 12 find (out = slot index)
__global__ __launch_bounds__(kBlock) void k_meta(spl_arena_t aa, const char* keys, int kstride, int op,
                                                 const uint64_t* args, long n, int32_t* status, uint64_t* out) {
  const Arena a = to_dev(aa);
  uint32_t muts = 0;
  Stats st;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    Key k;
    load_key(k, keys + i * (long)kstride, kstride);
    const uint64_t arg = args ? args[i] : 0;
    uint64_t o = 0;
    bool mut = false;
    const int32_t rc = meta_op(a, k, op, arg, &o, &mut);
    if (mut) ++muts;
    if (out) out[i] = o;
    if (status) status[i] = rc;
  }
  flush_stats(a, st, nullptr, muts);
}

// ------------------------------------------------------ embeddings ------
// One wave per key: the 3072-B vector moves as 64 lanes x 3 x 16 B.
__global__ __launch_bounds__(kBlock) void k_embed_set(spl_arena_t aa, const char* keys, int kstride,
                                                      const float* vecs, long n, int32_t* status) {
  const Arena a = to_dev(aa);
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  uint32_t muts = 0;
  Stats st;
  for (long i = wave; i < n; i += nwaves) {
    Key k;
    load_key(k, keys + i * (long)kstride, kstride);
    long idx = find(a, k);
    int32_t rc = kOk;
    uint8_t* s = idx >= 0 ? a.slot((size_t)idx) : nullptr;
    if (idx < 0) rc = miss_rc(idx);
    else if (a.stride != kSlotEmbedBytes) rc = kInval;
    bool locked = false;
    if (rc == kOk && lane == 0) {
      const uint64_t e = slot_epoch(s);
      locked = !(e & 1) && acas64(epoch_ptr(s), e, e + 1);
    }
    locked = __shfl(locked, 0, 64);
    if (rc == kOk && !locked) rc = kAgain;
    if (rc == kOk) {
      const uint4* src = (const uint4*)(vecs + i * (long)kEmbedDim);
      uint4* dst = (uint4*)(s + kOffEmbed);
      float4 v[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const uint4 x = src[lane + 64 * c];
        dst[lane + 64 * c] = x;
        v[c] = __builtin_bit_cast(float4, x);
      }
      write_vec16_wave(a, (size_t)idx, v, lane);
      release();
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
        aadd64(epoch_ptr(s), 1);
        mark_dirty(a, (size_t)idx);
      }
      ++muts;
    }
    if (status && lane == 0) status[i] = rc;
  }
  if (lane != 0) muts = 0;
  flush_stats(a, st, nullptr, muts);
}

__global__ __launch_bounds__(kBlock) void k_embed_get(spl_arena_t aa, const char* keys, int kstride, float* vecs,
                                                      long n, int32_t* status) {
  const Arena a = to_dev(aa);
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long i = wave; i < n; i += nwaves) {
    Key k;
    load_key(k, keys + i * (long)kstride, kstride);
    long idx = find(a, k);
    int32_t rc = kOk;
    if (idx < 0) rc = miss_rc(idx);
    else if (a.stride != kSlotEmbedBytes) rc = kInval;
    if (rc == kOk) {
      const uint8_t* s = a.slot((size_t)idx);
      const uint64_t e1 = ald64_acq(s + kOffEpoch);
      if (e1 & 1) {
        rc = kAgain;
      } else {
        const uint4* src = (const uint4*)(s + kOffEmbed);
        uint4* dst = (uint4*)(vecs + i * (long)kEmbedDim);
#pragma unroll
        for (int c = 0; c < 3; ++c) dst[lane + 64 * c] = src[lane + 64 * c];
        drain();
        if (slot_epoch(s) != e1) rc = kAgain;
      }
    }
    if (status && lane == 0) status[i] = rc;
  }
}

// ------------------------------------------------------------- scans ----
// mode 0: list (hash != 0 && val_len > 0); mode 1: enumerate ((bloom&mask)==mask)
// mode 2: embedded (hash != 0 and vector not all-zero)  mode 3: occupied (hash != 0)
// Compacts matching slot indices with one atomic per wave (ballot + mbcnt).
__global__ __launch_bounds__(kBlock) void k_scan(spl_arena_t aa, int mode, uint64_t mask, uint32_t* out_idx,
                                                 uint64_t* out_epoch, uint32_t cap, uint32_t* counter,
                                                 uint32_t first, uint32_t last) {
  const Arena a = to_dev(aa);
  const int lane = threadIdx.x & 63;
  const size_t end = last < a.slots ? last : a.slots;
  for (size_t base = first + blockIdx.x * (size_t)blockDim.x; base < end; base += (size_t)gridDim.x * blockDim.x) {
    const size_t i = base + threadIdx.x;  // base is block-uniform: every lane reaches the ballot
    bool hit = false;
    uint64_t ep = 0;
    if (i < end) {
      const uint8_t* s = a.slot(i);
      const uint64_t h = slot_hash(s);
      if (mode == 4) {  // watchdog: writer-active (odd) epochs, claimed-but-unpublished slots included
        ep = slot_epoch(s);
        hit = (ep & 1) != 0;
      } else if (h != 0) {
        ep = slot_epoch(s);
        if (mode == 0) hit = ald32((const uint32_t*)(s + kOffValLen)) > 0;
        else if (mode == 1) hit = (ald64((const uint64_t*)(s + kOffBloom)) & mask) == mask;
        else if (mode == 3) hit = true;
        else if (a.stride == kSlotEmbedBytes) {
          const uint32_t* v = (const uint32_t*)(s + kOffEmbed);
          for (int d = 0; d < (int)kEmbedDim && !hit; ++d) hit = (v[d] & 0x7fffffffu) != 0;
        }
      }
    }
    const uint64_t bal = __ballot(hit);
    if (bal) {
      uint32_t basepos = 0;
      if (lane == 0) basepos = atomicAdd(counter, (uint32_t)__popcll(bal));
      basepos = __shfl(basepos, 0, 64);
      if (hit) {
        const uint32_t pos = basepos + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        if (pos < cap) {
          out_idx[pos] = (uint32_t)i;
          if (out_epoch) out_epoch[pos] = ep;
        }
      }
    }
  }
}

__global__ void k_purge(spl_arena_t aa) {
  const Arena a = to_dev(aa);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < a.slots; i += (size_t)gridDim.x * blockDim.x) {
    uint8_t* s = a.slot(i);
    const uint64_t e = slot_epoch(s);
    if (e & 1) continue;
    const uint64_t h = slot_hash(s);
    if (h == 0 && e == 0) continue;
    if (!acas64(epoch_ptr(s), e, e + 1)) continue;
    const uint32_t len = h == 0 ? 0 : ald32((const uint32_t*)(s + kOffValLen));
    uint8_t* v = a.value(i);
    uint32_t c = len;
    for (; c < a.max_val && (c & 15); ++c) v[c] = 0;
    for (; c + 16 <= a.max_val; c += 16) *(uint4*)(v + c) = make_uint4(0, 0, 0, 0);
    for (; c < a.max_val; ++c) v[c] = 0;
    release();
    aadd64(epoch_ptr(s), 1);
  }
}

// Gather slot metadata + keys for a list of slot indices (host list/snapshot).
__global__ void k_gather_slots(spl_arena_t aa, const uint32_t* idx, long n, uint8_t* out_core) {
  const Arena a = to_dev(aa);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint8_t* s = a.slot(idx[i]);
    for (int c = 0; c < 16; ++c) *(uint64_t*)(out_core + i * 128 + 8 * c) = ald64(s + 8 * c);
  }
}

// FNV-1a of canonical key records (shard routing, C1 of SURVEY §2.10).
__global__ void k_hash_keys(const char* keys, int kstride, long n, uint64_t* out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    Key k;
    load_key(k, keys + i * (long)kstride, kstride);
    out[i] = k.hash;
  }
}

// Bench/tool helper: key i of a batch = printf("%s%0*llu", prefix, width, ids[i])
// written NUL-padded into kstride-byte records.  Not on any timed path.
__global__ void k_format_keys(char* out, int kstride, const uint64_t* ids, uint64_t first, long n, const char* prefix,
                              int plen, int width) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    char* r = out + i * (long)kstride;
    uint64_t v = ids ? ids[i] : first + (uint64_t)i;
    int p = 0;
    for (; p < plen && p < kstride - 1; ++p) r[p] = prefix[p];
    char digits[24];
    int nd = 0;
    do { digits[nd++] = (char)('0' + v % 10); v /= 10; } while (v && nd < 20);
    while (nd < width && nd < 20) digits[nd++] = '0';
    for (int d = nd - 1; d >= 0 && p < kstride - 1; --d) r[p++] = digits[d];
    for (; p < kstride; ++p) r[p] = 0;
  }
}

// Bench helper: value i = "ver:<ver>|id:<id>|data:" + fill bytes to `len`.
__global__ void k_format_values(uint8_t* out, int vstride, uint32_t* lens, const uint64_t* ids, uint64_t first,
                                long n, uint32_t ver, uint32_t len) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint8_t* r = out + i * (long)vstride;
    const uint64_t id = ids ? ids[i] : first + (uint64_t)i;
    char tmp[64];
    int p = 0;
    const char* a = "ver:";
    for (int q = 0; a[q]; ++q) tmp[p++] = a[q];
    char d[24];
    int nd = 0;
    uint32_t v = ver;
    do { d[nd++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (nd) tmp[p++] = d[--nd];
    const char* b = "|id:";
    for (int q = 0; b[q]; ++q) tmp[p++] = b[q];
    uint64_t w = id;
    do { d[nd++] = (char)('0' + w % 10); w /= 10; } while (w);
    while (nd) tmp[p++] = d[--nd];
    const char* c = "|data:";
    for (int q = 0; c[q]; ++q) tmp[p++] = c[q];
    uint32_t L = len < (uint32_t)vstride ? len : (uint32_t)vstride;
    for (uint32_t q = 0; q < L; ++q) r[q] = q < (uint32_t)p ? (uint8_t)tmp[q] : (uint8_t)('A' + ver % 26);
    for (uint32_t q = L; q < (uint32_t)vstride; ++q) r[q] = 0;
    if (lens) lens[i] = L;
  }
}

}  // namespace

// ====================================================== C launchers ======
extern "C" {

int spl_arena_init_slots(spl_arena_t a, hipStream_t s) {
  hipLaunchKernelGGL(k_init_slots, dim3(grid_for(a.slots)), dim3(kBlock), 0, s, a);
  return (int)hipGetLastError();
}

}  // extern "C"

namespace {

// Batched set / get launches (every public entry point and the stream fan-outs go through these).
// Two forms each, chosen once per process: SPLINTER_ARENA_COOP (sets) / SPLINTER_ARENA_COOP_GET
// (gets) = 2 (default: write-through rows, acquire-free sc1 reads) or 1 (plain rows + one release
// per round / one agent acquire per round).  The measured-and-rejected forms (single-op, non-carried
// rounds, 512-thread blocks, U = 1/4/8, batched claims, pipelined copies) are gone; their A/B
// history is in profiles/r1_* .. r3_*.
constexpr int kU = 2, kB = 256;

int launch_set(const spl_arena_t& a, const char* keys, int kstride, const uint8_t* vals, int vstride,
               const uint32_t* lens, long n, int32_t* status, int max_retry, uint64_t* stats, const Seg& seg,
               hipStream_t s) {
  if (n <= 0) return 0;
  if ((kstride & 15) || kstride > 64 || (vstride & 15)) return (int)hipErrorInvalidValue;
  if (seg.counts && seg.cap <= 0) return (int)hipErrorInvalidValue;
  static const int coop = env_int("SPLINTER_ARENA_COOP", 2);
  const dim3 g(grid_for_b((n + kU - 1) / kU, kB));
  if (coop == 1)
    hipLaunchKernelGGL((k_set_carry<kU, kB, false>), g, dim3(kB), 0, s, a, keys, kstride, vals, vstride, lens, n,
                       status, max_retry, stats, seg);
  else
    hipLaunchKernelGGL((k_set_carry<kU, kB, true>), g, dim3(kB), 0, s, a, keys, kstride, vals, vstride, lens, n,
                       status, max_retry, stats, seg);
  return (int)hipGetLastError();
}

int launch_get(const spl_arena_t& a, const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens,
               long n, int32_t* status, int max_retry, uint64_t* stats, const Seg& seg, hipStream_t s) {
  if (n <= 0) return 0;
  if ((kstride & 15) || kstride > 64 || (ostride & 15)) return (int)hipErrorInvalidValue;
  if (seg.counts && seg.cap <= 0) return (int)hipErrorInvalidValue;
  static const int coop = env_int("SPLINTER_ARENA_COOP_GET", 2);
  const dim3 g(grid_for_b((n + kU - 1) / kU, kB));
  if (coop == 1)
    hipLaunchKernelGGL((k_get_carry<kU, kB, false>), g, dim3(kB), 0, s, a, keys, kstride, out, ostride, out_lens, n,
                       status, max_retry, stats, seg);
  else
    hipLaunchKernelGGL((k_get_carry<kU, kB, true>), g, dim3(kB), 0, s, a, keys, kstride, out, ostride, out_lens, n,
                       status, max_retry, stats, seg);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int spl_arena_set(spl_arena_t a, const char* keys, int kstride, const uint8_t* vals, int vstride, const uint32_t* lens,
                  long n, int32_t* status, int max_retry, uint64_t* stats, hipStream_t s) {
  return launch_set(a, keys, kstride, vals, vstride, lens, n, status, max_retry, stats, Seg{nullptr, 1}, s);
}

int spl_arena_set_seg(spl_arena_t a, const char* keys, int kstride, const uint8_t* vals, int vstride,
                      const uint32_t* lens, long n, int32_t* status, int max_retry, uint64_t* stats,
                      const int32_t* seg_counts, long seg_cap, hipStream_t s) {
  if (seg_counts && (seg_cap <= 0 || n % seg_cap)) return (int)hipErrorInvalidValue;
  return launch_set(a, keys, kstride, vals, vstride, lens, n, status, max_retry, stats,
                    Seg{seg_counts, seg_cap > 0 ? seg_cap : 1}, s);
}

int spl_arena_get(spl_arena_t a, const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens, long n,
                  int32_t* status, int max_retry, uint64_t* stats, hipStream_t s) {
  return launch_get(a, keys, kstride, out, ostride, out_lens, n, status, max_retry, stats, Seg{nullptr, 1}, s);
}

int spl_arena_get_seg(spl_arena_t a, const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens,
                      long n, int32_t* status, int max_retry, uint64_t* stats, const int32_t* seg_counts,
                      long seg_cap, hipStream_t s) {
  if (seg_counts && (seg_cap <= 0 || n % seg_cap)) return (int)hipErrorInvalidValue;
  return launch_get(a, keys, kstride, out, ostride, out_lens, n, status, max_retry, stats,
                    Seg{seg_counts, seg_cap > 0 ? seg_cap : 1}, s);
}

// In-place rows (idx: client op indices; live rows: the first *count of them): the own-shard ops of
// a routed step run on the client's own arrays (parallel/xroute.py).
int spl_arena_set_idx(spl_arena_t a, const char* keys, int kstride, const uint8_t* vals, int vstride,
                      const uint32_t* lens, const int32_t* idx, const int32_t* count, long n, int32_t* status,
                      int max_retry, uint64_t* stats, hipStream_t s) {
  if (!idx || !count) return (int)hipErrorInvalidValue;
  return launch_set(a, keys, kstride, vals, vstride, lens, n, status, max_retry, stats, Seg{count, n > 0 ? n : 1, 0, idx},
                    s);
}

int spl_arena_get_idx(spl_arena_t a, const char* keys, int kstride, uint8_t* out, int ostride, uint32_t* out_lens,
                      const int32_t* idx, const int32_t* count, long n, int32_t* status, int max_retry,
                      uint64_t* stats, hipStream_t s) {
  if (!idx || !count) return (int)hipErrorInvalidValue;
  return launch_get(a, keys, kstride, out, ostride, out_lens, n, status, max_retry, stats,
                    Seg{count, n > 0 ? n : 1, 0, idx}, s);
}

int spl_arena_unset(spl_arena_t a, const char* keys, int kstride, long n, int32_t* status, int max_retry,
                    hipStream_t s) {
  if (n <= 0) return 0;
  if ((kstride & 15) || kstride > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_unset, dim3(grid_for(n)), dim3(kBlock), 0, s, a, keys, kstride, n, status, max_retry);
  return (int)hipGetLastError();
}

int spl_arena_intop(spl_arena_t a, const char* keys, int kstride, const int* ops, const uint64_t* masks, long n,
                    int32_t* status, uint64_t* results, int max_retry, hipStream_t s) {
  if (n <= 0) return 0;
  if ((kstride & 15) || kstride > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_intop, dim3(grid_for(n)), dim3(kBlock), 0, s, a, keys, kstride, ops, masks, n, status, results,
                     max_retry);
  return (int)hipGetLastError();
}

int spl_arena_meta(spl_arena_t a, const char* keys, int kstride, int op, const uint64_t* args, long n, int32_t* status,
                   uint64_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  if ((kstride & 15) || kstride > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_meta, dim3(grid_for(n)), dim3(kBlock), 0, s, a, keys, kstride, op, args, n, status, out);
  return (int)hipGetLastError();
}

int spl_arena_embed_set(spl_arena_t a, const char* keys, int kstride, const float* vecs, long n, int32_t* status,
                        hipStream_t s) {
  if (n <= 0) return 0;
  if ((kstride & 15) || kstride > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_embed_set, dim3(grid_for(n * 64)), dim3(kBlock), 0, s, a, keys, kstride, vecs, n, status);
  return (int)hipGetLastError();
}

int spl_arena_embed_get(spl_arena_t a, const char* keys, int kstride, float* vecs, long n, int32_t* status,
                        hipStream_t s) {
  if (n <= 0) return 0;
  if ((kstride & 15) || kstride > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_embed_get, dim3(grid_for(n * 64)), dim3(kBlock), 0, s, a, keys, kstride, vecs, n, status);
  return (int)hipGetLastError();
}

int spl_arena_scan(spl_arena_t a, int mode, uint64_t mask, uint32_t* out_idx, uint64_t* out_epoch, uint32_t cap,
                   uint32_t* counter, hipStream_t s) {
  return spl_arena_scan_range(a, mode, mask, 0, a.slots, out_idx, out_epoch, cap, counter, s);
}

int spl_arena_scan_range(spl_arena_t a, int mode, uint64_t mask, uint32_t first, uint32_t last, uint32_t* out_idx,
                         uint64_t* out_epoch, uint32_t cap, uint32_t* counter, hipStream_t s) {
  if (last > a.slots) last = a.slots;
  if (first >= last) return 0;
  hipLaunchKernelGGL(k_scan, dim3(grid_for(last - first)), dim3(kBlock), 0, s, a, mode, mask, out_idx, out_epoch, cap,
                     counter, first, last);
  return (int)hipGetLastError();
}

int spl_arena_purge(spl_arena_t a, hipStream_t s) {
  hipLaunchKernelGGL(k_purge, dim3(grid_for(a.slots)), dim3(kBlock), 0, s, a);
  return (int)hipGetLastError();
}

int spl_arena_gather_slots(spl_arena_t a, const uint32_t* idx, long n, uint8_t* out_core, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_gather_slots, dim3(grid_for(n)), dim3(kBlock), 0, s, a, idx, n, out_core);
  return (int)hipGetLastError();
}

int spl_hash_keys(const char* keys, int kstride, long n, uint64_t* out, hipStream_t s) {
  if (n <= 0) return 0;
  if ((kstride & 15) || kstride > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_hash_keys, dim3(grid_for(n)), dim3(kBlock), 0, s, keys, kstride, n, out);
  return (int)hipGetLastError();
}

int spl_format_keys(char* out, int kstride, const uint64_t* ids, uint64_t first, long n, const char* prefix_dev,
                    int plen, int width, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_format_keys, dim3(grid_for(n)), dim3(kBlock), 0, s, out, kstride, ids, first, n, prefix_dev,
                     plen, width);
  return (int)hipGetLastError();
}

int spl_format_values(uint8_t* out, int vstride, uint32_t* lens, const uint64_t* ids, uint64_t first, long n,
                      uint32_t ver, uint32_t len, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_format_values, dim3(grid_for(n)), dim3(kBlock), 0, s, out, vstride, lens, ids, first, n, ver,
                     len);
  return (int)hipGetLastError();
}

}  // extern "C"

// ======================================================= kv streams ======
// Native submission of a KV step issued by many concurrent client streams (formerly
// kv_streams.hip; kept in this translation unit: with the fan-out and the command ring in two
// further HIP objects the post-KV encoder kernels ran 15 % slower, profiles/r2_lib_layout_ab.md).
//
// BASELINE config #2 runs 32 concurrent writer streams (plus readers).  Issuing their batches
// from Python costs ~30-60 µs of host time per launch (stream context switch, event record /
// wait, output allocation, ctypes), so 64 streams made the step host-bound: the GPU trace showed
// the last streams' kernels starting ~1 ms into a ~5 ms KV phase with idle queues before them.
// Here the fan-out is one native call: each client stream waits on the origin stream's start
// event, runs its slice of the step's set (writers) or get (readers) batch through the regular
// batch launchers, and records its done event, which the origin stream then waits on.  Streams
// keep their identity and independence: every slice is its own launch on its own stream (the HIP
// runtime maps them onto GPU_MAX_HW_QUEUES hardware queues per priority: writers at normal
// priority, readers at high).
#include <vector>

namespace {

struct KvStreams {
  int nw = 0, nr = 0;
  int fused = 2;  // spl_kvs_set_fused
  std::vector<hipStream_t> s;  // nw writers, then nr readers
  std::vector<hipEvent_t> done;
  hipEvent_t start = nullptr;
  // mode 3 (stream-posted server): the last server grid's end event, the device control block
  hipEvent_t srv_done = nullptr;
  AsyncCtl* ctl = nullptr;
  uint64_t seq = 0;
  // kSchedChunks: the fused grids' chunk counters, one word per launch from a ring of kClaimRing words
  // (a word is reused kClaimRing launches later, long after its launch has ended), tagged per launch
  static constexpr int kClaimRing = 1024;
  unsigned long long* claim = nullptr;
  uint32_t launches = 0;
  int sched = -1;  // spl_kvs_set_sched (kSched*); -1: SPL_KVS_SCHED
  unsigned long long* claim_slot(uint32_t* tag) {
    if (!claim) {
      if (hipMalloc((void**)&claim, kClaimRing * sizeof *claim) != hipSuccess ||
          hipMemset(claim, 0, kClaimRing * sizeof *claim) != hipSuccess) {
        (void)hipGetLastError();
        if (claim) (void)hipFree(claim);
        claim = nullptr;
        return nullptr;
      }
    }
    uint32_t id = __atomic_add_fetch(&launches, 1u, __ATOMIC_RELAXED) & 0xFFFFFFu;
    if (id == 0) id = __atomic_add_fetch(&launches, 1u, __ATOMIC_RELAXED) & 0xFFFFFFu;  // 0: a zeroed word's tag
    *tag = id;
    return claim + (*tag % kClaimRing);
  }
};

// The server grid of one step (mode 3), launched on the origin stream after every client stream's
// post has been enqueued (a post queued behind the server dispatch on a shared hardware queue would
// otherwise wait for the server's end).  A client stream posts once ITS preceding work is done; the
// rows themselves are ordered by the origin stream (the server runs behind the origin's work), so
// the posts gate each slice on its stream's readiness without a cross-stream event per step (the
// event chain origin -> server stream -> origin cost ~300 us per step: profiles/r5/kv_async.md).
int kvs_step_async(KvStreams* k, spl_arena_t a, hipStream_t origin, const FSeg& sset, const FSeg& sget, int ks,
                   int max_retry, uint64_t* stats) {
  const int nw = k->nw, nr = k->nr;  // slot i <-> client stream i, every step
  if (sset.n + sget.n <= 0) return 0;
  if (nw + nr > kAsyncSegs || ks != 16) return (int)hipErrorInvalidValue;
  if (!k->ctl) {
    if (hipMalloc(&k->ctl, sizeof(AsyncCtl)) != hipSuccess) return (int)hipErrorOutOfMemory;
    if (hipMemset(k->ctl, 0, sizeof(AsyncCtl)) != hipSuccess) return (int)hipErrorUnknown;
    if (hipEventCreateWithFlags(&k->srv_done, hipEventDisableTiming) != hipSuccess) return (int)hipErrorUnknown;
  }
  const uint64_t seq = ++k->seq;
  hipError_t e;
  // the posts: each client stream with rows in this step rings its slot once its own preceding work
  // is done
  for (int i = 0; i < nw + nr; ++i) {
    const bool isset = i < nw;
    const long n = isset ? sset.n : sget.n;
    const int parts = isset ? nw : nr, pi = isset ? i : i - nw;
    if (async_bound(n, pi, parts) >= async_bound(n, pi + 1, parts)) continue;
    e = hipStreamWriteValue64(k->s[i], &k->ctl->door[i], seq, 0);
    if (e != hipSuccess) return (int)e;
  }
  static const int wpc_env = env_int("SPL_KVS_FUSED_WG_PER_CU", 0);
  const int wpc = wpc_env > 0 ? wpc_env : 3;
  const long rows = sset.n + sget.n;
  const long need = (rows + 2 * 256 - 1) / (2 * 256);
  const long cap = (long)stream_cus(origin) * wpc;  // resident grid: the CUs the origin stream may use
  static const long chunk = [] {  // rows per claim: 4 rounds of a 256-thread workgroup at 2 ops per lane
    const int c = env_int("SPL_KVS_ASYNC_CHUNK", 2048);
    return (long)(c >= 512 ? c : 512);
  }();
  static const uint64_t wait_ticks = (uint64_t)env_int("SPL_KVS_ASYNC_WAIT_MS", 2000) * 100000ull;  // 100 MHz
  static const int spread = env_int("SPL_KVS_ASYNC_SPREAD", 1);
  static const int wv = env_int("SPL_KVS_ASYNC_WV", 1);
  const dim3 grid((unsigned)(need < cap ? need : cap));
  const int flags = (env_int("SPL_KVS_SKIP_LEN", 1) ? kKvSkipLen : 0) | (env_int("SPL_KVS_COPY_DMA", 1) ? kKvCopyDma : 0) |
                    (env_int("SPL_KVS_PAD_OUT", 1) ? kKvPadOut : 0);
  if (wv)
    hipLaunchKernelGGL((k_kv_server<2, 256, 4, 3, true>), grid, dim3(256), 0, origin, a, sset, sget, nw, nr, ks, k->ctl,
                       seq, chunk, wait_ticks, spread, max_retry, stats, flags);
  else
    hipLaunchKernelGGL((k_kv_server<2, 256, 4, 3>), grid, dim3(256), 0, origin, a, sset, sget, nw, nr, ks, k->ctl, seq,
                       chunk, wait_ticks, spread, max_retry, stats, flags);
  e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  (void)hipEventRecord(k->srv_done, origin);
  return 0;
}

}  // namespace

extern "C" {

void* spl_kvs_create(int writers, int readers) {
  if (writers < 1 || readers < 1 || writers + readers > 256) return nullptr;
  auto* k = new KvStreams();
  k->nw = writers;
  k->nr = readers;
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  // SPL_KVS_SPREAD=1 (A/B knob): every other writer at the low priority level, so the writer slices
  // spread over two hardware-queue pools instead of one (profiles/r2_kvs_order.md)
  // (2: readers also alternate between the high and the normal pool)
  static const int spread = [] {
    const char* e = getenv("SPL_KVS_SPREAD");
    return e && *e ? atoi(e) : 0;
  }();
  // SPL_KVS_PRIO=1 (A/B knob): writers on the high-priority pool and readers on the normal one (sets are the
  // slower half of a step; by default the readers win dispatch arbitration)
  static const int swap = [] {
    const char* e = getenv("SPL_KVS_PRIO");
    return e && *e ? atoi(e) : 0;
  }();
  for (int i = 0; i < writers + readers; ++i) {
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    int prio = i < writers ? ((spread >= 1 && (i & 1)) ? lo : 0) : ((spread >= 2 && (i & 1)) ? 0 : hi);
    if (swap == 1) prio = i < writers ? hi : 0;
    if (hipStreamCreateWithPriority(&st, hipStreamNonBlocking, prio) != hipSuccess ||
        hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      delete k;
      return nullptr;
    }
    k->s.push_back(st);
    k->done.push_back(ev);
  }
  (void)hipEventCreateWithFlags(&k->start, hipEventDisableTiming);
  k->fused = env_int("SPL_KVS_FUSED", 2);
  if (k->fused == 1) k->fused = 2;  // (1, the fused grid with 16-word keys, was an A/B form of 2)
  return k;
}

// 0: one launch per client stream's slice on that stream (the literal W-writer-stream form); 2: one
// fused grid (k_kv_fused; 1 is taken as 2); 3: the client streams post their slices to a resident
// server grid (k_kv_server)
int spl_kvs_set_fused(void* h, int mode) {
  auto* k = (KvStreams*)h;
  if (!k || mode < 0 || mode > 3) return (int)hipErrorInvalidValue;
  k->fused = mode == 1 ? 2 : mode;
  return 0;
}

// The fused grid's scheduling for this context (kSchedBarrier 0, kSchedChunks 1, kSchedWaves 2; -1:
// SPL_KVS_SCHED)
int spl_kvs_set_sched(void* h, int sched) {
  auto* k = (KvStreams*)h;
  if (!k || sched < -1 || sched > kSchedWaves) return (int)hipErrorInvalidValue;
  k->sched = sched;
  return 0;
}

// Mode 3: 1 when a server grid gave up waiting for a post (its step's unposted slices were not
// run), and clears the flag; waits for the last step's server first.  0: none, <0: no server yet.
int spl_kvs_async_error(void* h) {
  auto* k = (KvStreams*)h;
  if (!k || !k->ctl) return -1;
  (void)hipEventSynchronize(k->srv_done);
  uint32_t err = 0;
  if (hipMemcpy(&err, &k->ctl->err, sizeof err, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (err) (void)hipMemset(&k->ctl->err, 0, sizeof err);
  return err ? 1 : 0;
}

void spl_kvs_destroy(void* h) {
  auto* k = (KvStreams*)h;
  if (!k) return;
  for (auto st : k->s) {
    (void)hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
  }
  for (auto ev : k->done) (void)hipEventDestroy(ev);
  if (k->start) (void)hipEventDestroy(k->start);
  if (k->srv_done) (void)hipEventDestroy(k->srv_done);
  if (k->ctl) (void)hipFree(k->ctl);
  if (k->claim) (void)hipFree(k->claim);
  delete k;
}

// One step: writers split [0, n_set) of the set batch evenly, readers split [0, n_get) of the get
// batch; the origin stream continues after every slice.  Row-major batches (keys kstride B per
// row, values / outputs vstride / ostride B per row), per-op status and lengths.
int spl_kvs_step(void* h, spl_arena_t a, hipStream_t origin, const char* skeys, int kstride, const uint8_t* svals,
                 int vstride, const uint32_t* slens, long n_set, int32_t* sstatus, const char* gkeys, uint8_t* gout,
                 int ostride, uint32_t* glens, long n_get, int32_t* gstatus, int max_retry, uint64_t* stats) {
  auto* k = (KvStreams*)h;
  if (!k) return (int)hipErrorInvalidValue;
  // fused (default): every stream's slice consumed by ONE grid on the origin stream (k_kv_fused):
  // 100M keys, 32 + 32 streams, 3.96 G ops/s per-slice dispatches (0) -> 4.15 G (1, 16-word keys)
  // -> 4.85 G (2, 16-B keys in 4 words at 3 workgroups per CU), gpurun_out/r4d bench_kv_fused*.out
  const int fused = k->fused;
  if (fused == 3 && n_set + n_get > 0 && kstride == 16 && k->nw + k->nr <= kAsyncSegs) {
    if ((vstride & 15) || (ostride & 15)) return (int)hipErrorInvalidValue;
    const FSeg sset{skeys, (uint8_t*)svals, (uint32_t*)slens, sstatus, nullptr, nullptr, n_set, vstride, 1};
    const FSeg sget{gkeys, gout, glens, gstatus, nullptr, nullptr, n_get, ostride, 0};
    return kvs_step_async(k, a, origin, sset, sget, kstride, max_retry, stats);
  }
  if (fused && n_set + n_get > 0) {
    if ((kstride & 15) || kstride > 64 || (vstride & 15) || (ostride & 15)) return (int)hipErrorInvalidValue;
    FSegs tab{};
    tab.ks = kstride;
    if (n_set > 0)
      tab.s[tab.n++] = FSeg{skeys, (uint8_t*)svals, (uint32_t*)slens, sstatus, nullptr, nullptr, n_set, vstride, 1};
    if (n_get > 0) tab.s[tab.n++] = FSeg{gkeys, gout, glens, gstatus, nullptr, nullptr, n_get, ostride, 0};
    uint32_t tag = 0;
    unsigned long long* cw = k->claim_slot(&tag);
    return launch_fused(a, tab, n_set + n_get, fused, max_retry, stats, origin, cw, tag, k->sched);
  }
  hipError_t e = hipEventRecord(k->start, origin);
  if (e != hipSuccess) return (int)e;
  const int nw = n_set > 0 ? k->nw : 0, nr = n_get > 0 ? k->nr : 0;
  for (int w = 0; w < nw; ++w) {
    const long b = n_set * w / nw, end = n_set * (w + 1) / nw;
    if (end <= b) continue;
    hipStream_t st = k->s[w];
    (void)hipStreamWaitEvent(st, k->start, 0);
    int rc = spl_arena_set(a, skeys + b * (long)kstride, kstride, svals + b * (long)vstride, vstride, slens + b,
                           end - b, sstatus ? sstatus + b : nullptr, max_retry, stats, st);
    if (rc) return rc;
    (void)hipEventRecord(k->done[w], st);
    (void)hipStreamWaitEvent(origin, k->done[w], 0);
  }
  for (int r = 0; r < nr; ++r) {
    const long b = n_get * r / nr, end = n_get * (r + 1) / nr;
    if (end <= b) continue;
    hipStream_t st = k->s[k->nw + r];
    (void)hipStreamWaitEvent(st, k->start, 0);
    int rc = spl_arena_get(a, gkeys + b * (long)kstride, kstride, gout ? gout + b * (long)ostride : nullptr, ostride,
                           glens ? glens + b : nullptr, end - b, gstatus ? gstatus + b : nullptr, max_retry, stats, st);
    if (rc) return rc;
    (void)hipEventRecord(k->done[k->nw + r], st);
    (void)hipStreamWaitEvent(origin, k->done[k->nw + r], 0);
  }
  return (int)hipGetLastError();
}

// The owner side of a routed step (parallel/xroute.py, route_kernels.hip) on the same writer /
// reader streams as a local step.  The set rows are the concatenation of one segment per source
// rank -- the own segment (the client's own ops, in place through lidx, or the whole client batch
// when lidx is null: world 1) and every peer's request block -- and each writer stream takes an
// equal slice of that row space, one launch per segment it touches; gets likewise on the readers.
// A peer segment's results go straight to x->resp[s]: the requester's response block (peer
// transport: that rank's window, mapped here; RCCL transport: this rank's send staging block).
int spl_kvs_step_xr(void* h, spl_arena_t a, hipStream_t origin, const spl_xr_step_t* x, int max_retry,
                    uint64_t* stats) {
  auto* k = (KvStreams*)h;
  if (!k || !x || x->world < 1 || x->world > SPL_XR_MAX_WORLD || x->rank < 0 || x->rank >= x->world ||
      (x->world > 1 && (!x->lidx_set || !x->lidx_get || !x->own_counts || !x->rcounts)))
    return (int)hipErrorInvalidValue;
  const int W = x->world, r = x->rank;
  if (k->fused && 2 * W <= kFusedSegs && !(x->ks & 15) && x->ks <= 64 && !(x->svstride & 15) &&
      !(x->gostride & 15) && !(x->vw & 15)) {
    // one fused grid over every segment: own rows (in place) and each peer's request block
    FSegs tab{};
    tab.ks = x->ks;
    long rows = 0;
    for (int kind = 0; kind < 2; ++kind) {
      const bool set = kind == 0;
      const long n_own = set ? x->n_set : x->n_get;
      const long cap = set ? x->cap_s : x->cap_g;
      const int32_t* lidx = set ? x->lidx_set : x->lidx_get;
      if (n_own <= 0 && W == 1) continue;
      for (int sg = 0; sg < W; ++sg) {
        FSeg f;
        if (sg == r) {
          f = set ? FSeg{x->skeys, (uint8_t*)x->svals, (uint32_t*)x->slens, x->sstatus, lidx, nullptr, 0, x->svstride, 1}
                  : FSeg{x->gkeys, x->gout, x->glens, x->gstatus, lidx, nullptr, 0, x->gostride, 0};
          f.count = lidx ? x->own_counts + r * 2 + kind : nullptr;
          f.n = lidx ? cap : n_own;
        } else {
          uint8_t* q = (uint8_t*)x->req[sg];
          uint8_t* p = (uint8_t*)x->resp[sg];
          f = set ? FSeg{(const char*)(q + x->off_sk), q + x->off_sv, (uint32_t*)(q + x->off_sl),
                         (int32_t*)(p + x->off_ss), nullptr, x->rcounts + sg * 2 + kind, cap, x->vw, 1}
                  : FSeg{(const char*)(q + x->off_gk), p + x->off_gv, (uint32_t*)(p + x->off_gl),
                         (int32_t*)(p + x->off_gs), nullptr, x->rcounts + sg * 2 + kind, cap, x->vw, 0};
          // direct responses: results at the op's client index in source sg's client arrays
          const long op = set ? x->off_sp : x->off_gp;
          if (op > 0) f.oidx = (const int32_t*)(q + op);
        }
        tab.s[tab.n++] = f;
        rows += f.n;
      }
    }
    uint32_t tag = 0;
    unsigned long long* cw = k->claim_slot(&tag);
    return launch_fused(a, tab, rows, k->fused, max_retry, stats, origin, cw, tag, k->sched);
  }
  if (W > 1 && (x->off_sp > 0 || x->off_gp > 0)) return (int)hipErrorInvalidValue;  // direct: the fused grid only
  hipError_t e = hipEventRecord(k->start, origin);
  if (e != hipSuccess) return (int)e;
  for (int kind = 0; kind < 2; ++kind) {
    const bool set = kind == 0;
    const long n_own = set ? x->n_set : x->n_get;
    const long cap = set ? x->cap_s : x->cap_g;
    const bool ident = (set ? x->lidx_set : x->lidx_get) == nullptr;
    if (n_own <= 0 && W == 1) continue;
    // segment lengths: own = n (identity) or cap (lidx rows, the first own_counts[kind] live)
    long len[SPL_XR_MAX_WORLD], start[SPL_XR_MAX_WORLD + 1];
    start[0] = 0;
    for (int sg = 0; sg < W; ++sg) {
      len[sg] = sg == r ? (ident ? n_own : cap) : cap;
      start[sg + 1] = start[sg] + len[sg];
    }
    const long total = start[W];
    if (total <= 0) continue;
    const int ns = set ? k->nw : k->nr;
    for (int w = 0; w < ns; ++w) {
      const long lo = total * w / ns, hi = total * (w + 1) / ns;
      if (hi <= lo) continue;
      hipStream_t st = k->s[set ? w : k->nw + w];
      (void)hipStreamWaitEvent(st, k->start, 0);
      for (int sg = 0; sg < W; ++sg) {
        const long b0 = lo > start[sg] ? lo - start[sg] : 0;
        const long b1 = (hi < start[sg + 1] ? hi : start[sg + 1]) - start[sg];
        if (b1 <= b0) continue;
        const long m = b1 - b0;
        int rc;
        if (sg == r && ident) {  // world 1: the client batch itself, row for row
          rc = set ? launch_set(a, x->skeys + b0 * (long)x->ks, x->ks, x->svals + b0 * (long)x->svstride,
                                x->svstride, x->slens + b0, m, x->sstatus + b0, max_retry, stats, Seg{nullptr, 1}, st)
                   : launch_get(a, x->gkeys + b0 * (long)x->ks, x->ks, x->gout + b0 * (long)x->gostride, x->gostride,
                                x->glens + b0, m, x->gstatus + b0, max_retry, stats, Seg{nullptr, 1}, st);
        } else if (sg == r) {  // own ops in place: rows are lidx entries into the client arrays
          const Seg seg{x->own_counts + r * 2 + kind, cap, b0, (set ? x->lidx_set : x->lidx_get) + b0};
          rc = set ? launch_set(a, x->skeys, x->ks, x->svals, x->svstride, x->slens, m, x->sstatus, max_retry, stats,
                                seg, st)
                   : launch_get(a, x->gkeys, x->ks, x->gout, x->gostride, x->glens, m, x->gstatus, max_retry, stats,
                                seg, st);
        } else {  // peer sg's request block -> its response block
          const uint8_t* q = (const uint8_t*)x->req[sg];
          uint8_t* p = (uint8_t*)x->resp[sg];
          const Seg seg{x->rcounts + sg * 2 + kind, cap, b0};
          rc = set ? launch_set(a, (const char*)(q + x->off_sk) + b0 * (long)x->ks, x->ks,
                                q + x->off_sv + b0 * (long)x->vw, x->vw, (const uint32_t*)(q + x->off_sl) + b0, m,
                                (int32_t*)(p + x->off_ss) + b0, max_retry, stats, seg, st)
                   : launch_get(a, (const char*)(q + x->off_gk) + b0 * (long)x->ks, x->ks,
                                p + x->off_gv + b0 * (long)x->vw, x->vw, (uint32_t*)(p + x->off_gl) + b0, m,
                                (int32_t*)(p + x->off_gs) + b0, max_retry, stats, seg, st);
        }
        if (rc) return rc;
      }
      const int ev = set ? w : k->nw + w;
      (void)hipEventRecord(k->done[ev], st);
      (void)hipStreamWaitEvent(origin, k->done[ev], 0);
    }
  }
  return (int)hipGetLastError();
}

}  // extern "C"
