// arena_maint.hip — maintenance passes over an HBM arena: probe-chain statistics, the tombstone
// rebuild (rehash), and the rebuild of the bf16 vector copy of the side region.
//
// Chains and tombstones.  Lookups probe linearly from the key's home slot (hash % slots) and stop
// at a never-used ("virgin": hash 0, epoch 0) slot (arena_dev.hpp locate / claim_set).  An unset
// leaves a tombstone (hash 0, epoch 2: the reference contract, /root/reference/splinter.c:302-318
// and the unset path), which inserts reuse but lookups walk past, so under insert / unset churn the
// clusters between virgin slots only grow and a miss walks the whole cluster (the reference scans
// every slot on a miss, splinter.c:437-463).  SURVEY §7.3.2.
//
//   k_probe_stats   exact chain health of the arena in one pass: live / tombstone / virgin / busy
//                   counts, the probe length of a hit for every live key (histogram, sum, max) and
//                   the probe length of a miss averaged over all home positions (each virgin slot
//                   walks back over the cluster that ends at it: a cluster of L slots contributes
//                   (L+1)(L+2)/2 over its L+1 home positions).
//   k_rehash        cluster compaction, one wave per cluster START inside its slot range: walking the
//                   cluster, every live key moves into the first tombstone on its own probe path
//                   (between its home and its slot: still reachable, now earlier), its old slot
//                   becomes the next tombstone; the tombstones left at the end of the cluster become
//                   virgin slots, which splits the cluster.  Keys, values, vectors, the bf16 copy and
//                   the slot metadata move together; a slot's value row stays its own (val_off is
//                   per position).  EXCLUSIVE: no other op may run on the arena meanwhile (the store
//                   takes its ring hold and its stream; batch clients must be stopped).
//   k_vec16_rebuild the side region's bf16 copy + squared norms from the fp32 vectors (after a
//                   restore, or for an arena whose copy is missing).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <algorithm>

#include "arena_api.h"
#include "arena_dev.hpp"

namespace {
using namespace spl;
using namespace spl::dev;

__device__ __forceinline__ int bucket_of(uint64_t len) {
  if (len <= 1) return 0;
  const int b = 64 - __builtin_clzll(len - 1);  // ceil(log2(len))
  return b < kProbeBuckets - 1 ? b : kProbeBuckets - 1;
}

__device__ __forceinline__ uint64_t cyc(uint64_t a, uint64_t b, uint64_t n) { return a >= b ? a - b : a + n - b; }

constexpr int kStatThreads = 256;

__global__ __launch_bounds__(kStatThreads) void k_probe_stats(spl_arena_t aa, ProbeStats* __restrict__ out) {
  const Arena a = from_api(aa);
  __shared__ unsigned long long sh[8 + kProbeBuckets];
  for (int i = threadIdx.x; i < 8 + kProbeBuckets; i += kStatThreads) sh[i] = 0;
  __syncthreads();
  uint64_t live = 0, tomb = 0, virg = 0, busy = 0, dsum = 0, dmax = 0, msum = 0, mmax = 0;
  uint64_t hist[kProbeBuckets] = {};
  const uint64_t n = a.slots;
  for (uint64_t i = blockIdx.x * (uint64_t)kStatThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kStatThreads) {
    const uint8_t* s = a.slot(i);
    const uint64_t h = ald64(s + kOffHash), e = ald64(s + kOffEpoch);
    if (e & 1) {
      ++busy;
    } else if (h != 0) {
      ++live;
      const uint64_t d = cyc(i, h % n, n) + 1;
      dsum += d;
      dmax = d > dmax ? d : dmax;
      ++hist[bucket_of(d)];
    } else if (e != 0) {
      ++tomb;
    } else {
      ++virg;
      // the cluster that ends here: walk back to the previous virgin slot
      uint64_t L = 0, j = i;
      while (L < n - 1) {
        j = j == 0 ? n - 1 : j - 1;
        const uint8_t* t = a.slot(j);
        if (ald64(t + kOffHash) == 0 && ald64(t + kOffEpoch) == 0) break;
        ++L;
      }
      msum += (L + 1) * (L + 2) / 2;
      mmax = L + 1 > mmax ? L + 1 : mmax;
    }
  }
  atomicAdd(&sh[0], (unsigned long long)live);
  atomicAdd(&sh[1], (unsigned long long)tomb);
  atomicAdd(&sh[2], (unsigned long long)virg);
  atomicAdd(&sh[3], (unsigned long long)busy);
  atomicAdd(&sh[4], (unsigned long long)dsum);
  atomicMax(&sh[5], (unsigned long long)dmax);
  atomicAdd(&sh[6], (unsigned long long)msum);
  atomicMax(&sh[7], (unsigned long long)mmax);
#pragma unroll
  for (int b = 0; b < kProbeBuckets; ++b)
    if (hist[b]) atomicAdd(&sh[8 + b], (unsigned long long)hist[b]);
  __syncthreads();
  if (threadIdx.x < 8 + kProbeBuckets) {
    unsigned long long* o = (unsigned long long*)out;
    const int f = threadIdx.x;
    // ProbeStats: live, tombstones, virgin, busy, disp_sum, disp_max, miss_sum, miss_max, hist[]
    if (f == 5 || f == 7) atomicMax(o + f, sh[f]);
    else if (sh[f]) atomicAdd(o + f, sh[f]);
  }
}

// ---------------------------------------------------------------- rehash --
constexpr int kRhWaves = 4;        // waves per block, each its own slot range
constexpr int kRhHoles = 1024;     // tombstones a wave keeps track of per cluster (a power of two; more: the oldest dropped)

struct RhCounters {
  unsigned long long moved, reclaimed, clusters, skipped;
};

// move slot j's entry into tombstone slot q (whole wave; exclusive access)
__device__ void move_entry(const Arena& a, uint64_t q, uint64_t j, int lane) {
  uint8_t* d = a.slot(q);
  uint8_t* s = a.slot(j);
  // core: 16-B chunks 0..7 except the val_off word (bytes 16..19 stay the destination's own)
  if (lane < 8) {
    uint4 v = *(const uint4*)(s + 16 * lane);
    if (lane == 1) v.x = *(const uint32_t*)(d + kOffValOff);
    *(uint4*)(d + 16 * lane) = v;
  }
  // value row
  const uint32_t n16 = a.max_val / 16;
  for (uint32_t c = lane; c < n16; c += 64) ((uint4*)a.value(q))[c] = ((const uint4*)a.value(j))[c];
  for (uint32_t b = n16 * 16 + lane; b < a.max_val; b += 64) a.value(q)[b] = a.value(j)[b];
  if (a.stride == kSlotEmbedBytes) {
    for (uint32_t c = lane; c < kEmbedBytes / 16; c += 64) ((uint4*)(d + kOffEmbed))[c] = ((const uint4*)(s + kOffEmbed))[c];
    if (a.has_vec16()) {
      for (uint32_t c = lane; c < kVec16Bytes / 16; c += 64) ((uint4*)a.vec16(q))[c] = ((const uint4*)a.vec16(j))[c];
      if (lane == 0) a.nrm2()[q] = a.nrm2()[j];
    }
  }
  __builtin_amdgcn_wave_barrier();
  // the source becomes a tombstone (as unset leaves it): hash 0, key / metadata cleared, epoch 2
  if (lane < 8 && lane != 1) *(uint4*)(s + 16 * lane) = make_uint4(0, 0, 0, 0);
  if (lane == 1) {
    uint4 v = *(const uint4*)(s + 16);
    *(uint4*)(s + 16) = make_uint4(v.x, 0, SPL_SLOT_DEFAULT_TYPE, 0);
  }
  if (lane == 0) {
    *(uint64_t*)(s + kOffEpoch) = 2;
    if (a.has_vec16()) a.nrm2()[j] = 0.f;
  }
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64 * kRhWaves) void k_rehash(spl_arena_t aa, uint64_t range, RhCounters* __restrict__ cnt) {
  const Arena a = from_api(aa);
  __shared__ uint32_t holes_all[kRhWaves][kRhHoles];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t* holes = holes_all[wave];
  const uint64_t n = a.slots;
  const uint64_t w = blockIdx.x * (uint64_t)kRhWaves + wave;
  const uint64_t r0 = w * range;
  if (r0 >= n) return;
  const uint64_t r1 = r0 + range < n ? r0 + range : n;
  unsigned long long moved = 0, reclaimed = 0, clusters = 0, skipped = 0;
  auto is_virgin = [&](uint64_t i) {
    const uint8_t* s = a.slot(i);
    return ald64(s + kOffHash) == 0 && ald64(s + kOffEpoch) == 0;
  };
  for (uint64_t base = r0; base < r1; base += 64) {
    // cluster starts in this chunk: a non-virgin slot after a virgin one
    const uint64_t i = base + lane;
    bool start = false;
    if (i < r1) start = !is_virgin(i) && is_virgin(i == 0 ? n - 1 : i - 1);
    uint64_t m = __ballot(start);
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      const uint64_t cs = base + l;  // cluster start
      ++clusters;
      // holes: tombstone positions in cluster order, a ring of kRhHoles (h0 = oldest); when it is full
      // the oldest hole is dropped (left a tombstone): later keys rarely have homes that far back
      int nh = 0, h0 = 0;
      bool overflow = false;
      auto H = [&](int t) -> uint32_t& { return holes[(h0 + t) & (kRhHoles - 1)]; };
      int64_t rl_used = -1;          // cluster-relative position of the last slot holding an entry
      uint64_t pos = cs, steps = 0;
      while (steps < n) {
        const uint8_t* s = a.slot(pos);
        // one value for the whole wave (exclusive access: nothing changes under the pass)
        const uint64_t hv = ald64(s + kOffHash);
        const uint64_t h = __builtin_amdgcn_readfirstlane((uint32_t)hv) |
                           ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(hv >> 32)) << 32);
        const uint64_t e = ald64(s + kOffEpoch);
        const bool odd = __builtin_amdgcn_readfirstlane((uint32_t)(e & 1)) != 0;
        const bool zero_e = __builtin_amdgcn_readfirstlane((uint32_t)(e != 0)) == 0;
        const int64_t rp = (int64_t)cyc(pos, cs, n);
        if (h == 0 && zero_e) break;  // cluster end
        if (h == 0 && !odd) {
          if (nh == kRhHoles) {  // full: drop the oldest
            h0 = (h0 + 1) & (kRhHoles - 1);
            --nh;
            overflow = true;
          }
          __builtin_amdgcn_wave_barrier();
          if (lane == 0) H(nh) = (uint32_t)pos;
          __builtin_amdgcn_wave_barrier();
          ++nh;
        } else if (!odd && nh > 0) {
          // live key: the first hole on its own probe path (rel(home) <= rel(hole) < rel(pos))
          const uint64_t rh = cyc(h % n, cs, n);
          int k = -1;
          for (int t0 = 0; t0 < nh && k < 0; t0 += 64) {
            const int t = t0 + lane;
            const uint64_t rq = t < nh ? cyc(H(t), cs, n) : 0;
            const bool ok = t < nh && rq >= rh && (int64_t)rq < rp;
            const uint64_t bm = __ballot(ok);
            if (bm) k = t0 + __builtin_ctzll(bm);
          }
          if (k >= 0) {
            const uint64_t q = H(k);
            move_entry(a, q, pos, lane);
            ++moved;
            // drop hole k (order kept); the vacated slot is the newest hole
            for (int t = k; t < nh - 1; ++t) {
              const uint32_t v = H(t + 1);
              __builtin_amdgcn_wave_barrier();
              if (lane == 0) H(t) = v;
              __builtin_amdgcn_wave_barrier();
            }
            if (lane == 0) H(nh - 1) = (uint32_t)pos;
            __builtin_amdgcn_wave_barrier();
            const int64_t rq = (int64_t)cyc(q, cs, n);
            rl_used = rq > rl_used ? rq : rl_used;
          } else {
            rl_used = rp;
          }
        } else {
          rl_used = rp;  // live without a hole before it, or busy (a writer in flight: never moved)
        }
        pos = pos + 1 == n ? 0 : pos + 1;
        ++steps;
      }
      // trailing tombstones (after the last slot holding an entry) become virgin: the cluster ends earlier
      __builtin_amdgcn_wave_barrier();
      for (int t = nh - 1; t >= 0; --t) {
        const uint64_t q = H(t);
        if ((int64_t)cyc(q, cs, n) <= rl_used) break;
        if (lane == 0) *(uint64_t*)(a.slot(q) + kOffEpoch) = 0;
        ++reclaimed;
      }
      if (overflow) ++skipped;
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (lane == 0) {
    atomicAdd(&cnt->moved, moved);
    atomicAdd(&cnt->reclaimed, reclaimed);
    atomicAdd(&cnt->clusters, clusters);
    atomicAdd(&cnt->skipped, skipped);
  }
}

// ------------------------------------------------------------ full rebuild --
// For an arena whose clusters have merged (few never-used slots left, e.g. high load under churn)
// the in-place compaction degenerates into one wave walking the whole table; instead every live
// entry is copied out, the slot array cleared, and the entries re-inserted in parallel (each at the
// first free slot from its home: no tombstones at all afterwards).  Temporary memory: one record of
// stride + max_val (+ the bf16 copy and norm) bytes per live entry.  Exclusive, as k_rehash.
struct RbGeom {
  uint32_t rec;      // bytes per record (16-B multiple)
  uint32_t off_val;  // value row in the record
  uint32_t off_v16;  // bf16 vector (vec16 arenas)
  uint32_t off_n2;   // squared norm
};
__device__ __forceinline__ void copy16(uint8_t* d, const uint8_t* s, uint32_t bytes, int lane) {
  const uint32_t n16 = bytes / 16;
  for (uint32_t c = lane; c < n16; c += 64) ((uint4*)d)[c] = ((const uint4*)s)[c];
  for (uint32_t b = n16 * 16 + lane; b < bytes; b += 64) d[b] = s[b];
}

__global__ __launch_bounds__(256) void k_rb_collect(spl_arena_t aa, uint32_t* __restrict__ idx,
                                                    unsigned long long* __restrict__ count) {
  const Arena a = from_api(aa);
  const int lane = threadIdx.x & 63;
  for (uint64_t base = blockIdx.x * 256ull; base < a.slots; base += gridDim.x * 256ull) {
    const uint64_t i = base + threadIdx.x;
    const bool live = i < a.slots && ald64(a.slot(i) + kOffHash) != 0;
    const uint64_t bm = __ballot(live);
    if (!bm) continue;
    unsigned long long b0 = 0;
    if (lane == 0) b0 = atomicAdd(count, (unsigned long long)__popcll(bm));
    b0 = __shfl(b0, 0, 64);
    if (live) idx[b0 + __popcll(bm & ((1ull << lane) - 1))] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(256) void k_rb_gather(spl_arena_t aa, const uint32_t* __restrict__ idx, uint64_t n,
                                                   uint8_t* __restrict__ tmp, RbGeom g) {
  const Arena a = from_api(aa);
  const int lane = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < n; w += nw) {
    const uint64_t i = idx[w];
    uint8_t* r = tmp + w * g.rec;
    copy16(r, a.slot(i), a.stride, lane);  // core (+ fp32 vector)
    copy16(r + g.off_val, a.value(i), a.max_val, lane);
    if (a.has_vec16()) {
      copy16(r + g.off_v16, (const uint8_t*)a.vec16(i), kVec16Bytes, lane);
      if (lane == 0) *(float*)(r + g.off_n2) = a.nrm2()[i];
    }
  }
}

__global__ __launch_bounds__(256) void k_rb_insert(spl_arena_t aa, const uint8_t* __restrict__ tmp, uint64_t n,
                                                   RbGeom g, unsigned long long* __restrict__ fail) {
  const Arena a = from_api(aa);
  const int lane = threadIdx.x & 63;
  const uint64_t ns = a.slots;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < n; w += nw) {
    const uint8_t* r = tmp + w * g.rec;
    const uint64_t h = *(const uint64_t*)r, ep = *(const uint64_t*)(r + kOffEpoch);
    const uint64_t home = h % ns;
    // lane-parallel probe: 64 consecutive slots per round, the first virgin claimed by CAS 0 -> 1
    int64_t tgt = -1;
    for (uint64_t base = 0; base < ns && tgt < 0; base += 64) {
      const uint64_t p = (home + base + lane) % ns;
      const uint8_t* s = a.slot(p);
      bool v = base + lane < ns && ald64(s + kOffHash) == 0 && ald64(s + kOffEpoch) == 0;
      uint64_t bm = __ballot(v);
      while (bm && tgt < 0) {
        const int l = __builtin_ctzll(bm);
        bm &= bm - 1;
        bool got = false;
        if (lane == l) got = acas64((void*)(a.slot(p) + kOffEpoch), 0, 1);
        const uint64_t g2 = __ballot(got);
        if (g2) tgt = (int64_t)((home + base + l) % ns);
      }
    }
    if (tgt < 0) {
      if (lane == 0) atomicAdd(fail, 1ull);
      continue;
    }
    uint8_t* d = a.slot((uint64_t)tgt);
    // record -> slot: bytes 16.. of the core (val_off stays the slot's own), vector, value, copy; then
    // the key's hash and finally its epoch (a reader never sees the hash before the key bytes)
    const uint32_t voff = *(const uint32_t*)(d + kOffValOff);
    copy16(d + 16, r + 16, a.stride - 16, lane);
    copy16(a.value((uint64_t)tgt), r + g.off_val, a.max_val, lane);
    if (a.has_vec16()) {
      copy16((uint8_t*)a.vec16((uint64_t)tgt), r + g.off_v16, kVec16Bytes, lane);
      if (lane == 0) a.nrm2()[tgt] = *(const float*)(r + g.off_n2);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      *(uint32_t*)(d + kOffValOff) = voff;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      ast64(d + kOffHash, h);
      ast64(d + kOffEpoch, ep < 2 ? 2 : ep);
    }
  }
}

// one wave per slot: bf16 copy + squared norm from the fp32 vector (0 for an empty slot)
__global__ __launch_bounds__(256) void k_vec16_rebuild(spl_arena_t aa) {
  const Arena a = from_api(aa);
  const int lane = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < a.slots; i += nw) {
    const uint8_t* s = a.slot(i);
    if (ald64(s + kOffHash) == 0) {
      if (lane == 0) a.nrm2()[i] = 0.f;
      continue;
    }
    const float4* src = (const float4*)(s + kOffEmbed);
    float4 v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = src[lane + 64 * c];
    write_vec16_wave(a, i, v, lane);
  }
}

}  // namespace

extern "C" {

// Probe-chain statistics into `out` (device ProbeStats, zeroed by the caller).
int spl_arena_probe_stats(spl_arena_t a, void* out, hipStream_t s) {
  if (!a.base || !out) return (int)hipErrorInvalidValue;
  long g = ((long)a.slots + kStatThreads - 1) / kStatThreads;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(k_probe_stats, dim3((unsigned)g), dim3(kStatThreads), 0, s, a, (ProbeStats*)out);
  return (int)hipGetLastError();
}

// Cluster compaction (EXCLUSIVE access).  `counters`: device u64[4] {moved, reclaimed, clusters,
// skipped (clusters with more than kRhHoles tombstones, compacted only up to there)}, zeroed by
// the caller.
int spl_arena_rehash(spl_arena_t a, void* counters, hipStream_t s) {
  if (!a.base || !counters) return (int)hipErrorInvalidValue;
  // ranges of 1024 slots: a cluster is handled by the wave whose range holds its start
  const uint64_t range = 1024;
  const uint64_t waves = ((uint64_t)a.slots + range - 1) / range;
  const uint64_t blocks = (waves + kRhWaves - 1) / kRhWaves;
  hipLaunchKernelGGL(k_rehash, dim3((unsigned)blocks), dim3(64 * kRhWaves), 0, s, a, range, (RhCounters*)counters);
  return (int)hipGetLastError();
}

// Full rebuild (see k_rb_*): live entries -> tmp, slot array cleared, entries re-inserted.
// scratch_idx: device u32[slots]; tmp: device, slots_live * rec bytes (spl_arena_rebuild_rec);
// count: device u64 (zeroed); fail: device u64 (zeroed, entries that found no free slot: 0).
uint32_t spl_arena_rebuild_rec(spl_arena_t a) {
  uint32_t rec = a.stride + ((a.max_val + 15) & ~15u);
  if (a.flags & SPL_ARENA_VEC16) rec += (uint32_t)kVec16Bytes + 16;
  return rec;
}
int spl_arena_rebuild_collect(spl_arena_t a, uint32_t* idx, void* count, hipStream_t s) {
  long g = ((long)a.slots + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(k_rb_collect, dim3((unsigned)(g < 1 ? 1 : g)), dim3(256), 0, s, a, idx, (unsigned long long*)count);
  return (int)hipGetLastError();
}
int spl_arena_rebuild_move(spl_arena_t a, const uint32_t* idx, uint64_t n, void* tmp, void* fail, hipStream_t s) {
  RbGeom g;
  g.off_val = a.stride;
  g.off_v16 = a.stride + ((a.max_val + 15) & ~15u);
  g.off_n2 = g.off_v16 + (uint32_t)kVec16Bytes;
  g.rec = spl_arena_rebuild_rec(a);
  const unsigned blocks = (unsigned)std::min<uint64_t>((n + 3) / 4 + 1, 16384);
  hipLaunchKernelGGL(k_rb_gather, dim3(blocks), dim3(256), 0, s, a, idx, n, (uint8_t*)tmp, g);
  // the slot array and the value rows to zero, then val_off / default type (spl_arena_init_slots);
  // the squared norms to zero (no vector until re-inserted)
  const size_t slot_bytes = (size_t)a.slots * a.stride, val_bytes = (size_t)a.slots * a.max_val;
  (void)hipMemsetAsync((uint8_t*)a.base + spl::kHeaderBytes, 0, slot_bytes + val_bytes, s);
  if (a.flags & SPL_ARENA_VEC16)
    (void)hipMemsetAsync((uint8_t*)a.base + side_offset(a.slots, a.stride, a.max_val) + side_nrm2_offset(), 0,
                         (size_t)a.slots * 4, s);
  if (spl_arena_init_slots(a, s) != 0) return (int)hipGetLastError();
  hipLaunchKernelGGL(k_rb_insert, dim3(blocks), dim3(256), 0, s, a, (const uint8_t*)tmp, n, g,
                     (unsigned long long*)fail);
  return (int)hipGetLastError();
}

int spl_arena_vec16_rebuild(spl_arena_t a, hipStream_t s) {
  if (!a.base || !(a.flags & SPL_ARENA_VEC16) || a.stride != 3200) return (int)hipErrorInvalidValue;
  long g = ((long)a.slots + 3) / 4;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(k_vec16_rebuild, dim3((unsigned)g), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

}  // extern "C"
