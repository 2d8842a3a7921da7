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
//   k_rehash        cluster compaction beside live traffic, one wave per 1024-slot range: walking it,
//                   every live key moves into the first tombstone on its own probe path (between its
//                   home and its slot: still reachable, now earlier) under both slots' seqlocks, its
//                   old slot becomes the next tombstone; the tombstones left at the end of a cluster
//                   become virgin slots, which splits the cluster.  Keys, values, vectors, the bf16
//                   copy and the slot metadata move together; a slot's value row stays its own
//                   (val_off is per position).  ONLINE: see "rehash" below for the protocol.
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
// ONLINE: runs beside live batch / per-call ops of any process (arena_dev.hpp, "online
// maintenance").  The host opens the pass (k_maint_mark: MaintRec::seq odd), runs k_rehash, and
// closes it (seq even).  While seq is odd no probe reports "absent" and no insert is decided
// (EAGAIN instead), so the set of slots holding entries only shrinks or moves toward the homes;
// every move holds both slots' seqlocks:
//   1. CAS the destination tombstone's epoch eq -> eq+1 (fails if anything reused it),
//   2. CAS the source's epoch ej -> ej+1 (fails if a writer holds it or it changed),
//   3. copy slot bytes 16.. (val_off stays the destination's own), value row, fp32 vector, bf16
//      copy and norm with write-through stores, release, publish the hash, epoch eq+2,
//   4. clear the source as unset does (hash 0 first), release, epoch ej+2 -- forward, never
//      rewound, so a writer that read ej before the move cannot claim the tombstone by ABA.
// A reader that reaches the destination first finds the entry (or an odd epoch: EAGAIN); one that
// passed the destination before step 3 and reaches the source after step 4 has overlapped the
// pass and turns its miss into EAGAIN.  Each wave walks its own 1024-slot range from its start
// (the middle of a cluster included: a key whose home lies before the range start may move into
// any hole of the range before its slot), then continues past the range to the cluster's end (at
// most kRhTail slots).  Tombstones become virgin in a second kernel, k_reclaim, once every move
// is done.
constexpr int kRhWaves = 4;        // waves per block, each its own slot range
constexpr int kRhHoles = 512;      // tombstones a wave keeps track of per cluster (a power of two; more: the oldest dropped)
constexpr uint64_t kRhRange = 1024, kRhTail = 8192;

struct RhCounters {
  unsigned long long moved, reclaimed, clusters, skipped;
  unsigned long long dmax;  // largest displacement (slots past the home) of any keyed slot the walk saw
};

__device__ __forceinline__ void copy16(uint8_t* d, const uint8_t* s, uint32_t bytes, int lane) {
  const uint32_t n16 = bytes / 16;
  for (uint32_t c = lane; c < n16; c += 64) ((uint4*)d)[c] = ((const uint4*)s)[c];
  for (uint32_t b = n16 * 16 + lane; b < bytes; b += 64) d[b] = s[b];
}
__device__ __forceinline__ void copy16_wt(uint8_t* d, const uint8_t* s, uint32_t bytes, int lane) {
  const uint32_t n16 = bytes / 16;
  for (uint32_t c = lane; c < n16; c += 64) st16_wt((uint4*)d + c, ((const uint4*)s)[c]);
  for (uint32_t b = n16 * 16 + lane; b < bytes; b += 64) d[b] = s[b];
}

// Move the entry at slot j (observed hash h, even epoch ej) into tombstone q (observed epoch eq),
// holding both seqlocks (whole wave).  Returns 1 moved; -1 the hole was taken (drop it);
// -2 the source changed (the hole stays, now at epoch eq + 2).
__device__ int move_online(const Arena& a, uint64_t q, uint64_t eq, uint64_t j, uint64_t h, uint64_t ej, int lane) {
  uint8_t* d = a.slot(q);
  uint8_t* s = a.slot(j);
  int st = 0;
  if (lane == 0) {
    if (!acas64(epoch_ptr(d), eq, eq + 1)) {
      st = -1;
    } else if (slot_hash(d) != 0) {  // (an even epoch with a hash is a live entry: not ours to take)
      ast64(epoch_ptr(d), eq);
      st = -1;
    } else if (!acas64(epoch_ptr(s), ej, ej + 1)) {
      ast64(epoch_ptr(d), eq + 2);
      st = -2;
    } else if (slot_hash(s) != h) {  // unset rewound the epoch to the value we read: a tombstone now
      ast64(epoch_ptr(s), ej + 2);
      ast64(epoch_ptr(d), eq + 2);
      st = -2;
    } else {
      st = 1;
    }
  }
  st = __shfl(st, 0, 64);
  if (st != 1) return st;
  // both held: bytes 16..127 of the core (lane 1's first word: the destination's own val_off)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the source's bytes as their last writer left them
  if (lane >= 1 && lane < 8) {
    uint4 v = *(const uint4*)(s + 16 * lane);
    if (lane == 1) v.x = ald32(d + kOffValOff);
    st16_wt(d + 16 * lane, v);
  }
  if (a.max_val & 15) copy16(a.value(q), a.value(j), a.max_val, lane);  // rows not 16-B aligned: plain (released below)
  else copy16_wt(a.value(q), a.value(j), a.max_val, lane);
  if (a.stride == kSlotEmbedBytes) {
    copy16_wt(d + kOffEmbed, s + kOffEmbed, (uint32_t)kEmbedBytes, lane);
    if (a.has_vec16()) {
      copy16_wt((uint8_t*)a.vec16(q), (const uint8_t*)a.vec16(j), (uint32_t)kVec16Bytes, lane);
      if (lane == 0) a.nrm2()[q] = a.nrm2()[j];
    }
  }
  release();  // every lane's stores have left (the write-through ones and the plain tails)
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    ast64(d + kOffHash, h);
    drain();
    ast64(epoch_ptr(d), eq + 2);  // the entry lives at q now
    // the source becomes a tombstone as unset leaves it: hash 0 first
    ast64(s + kOffHash, 0);
    drain();
  }
  __builtin_amdgcn_wave_barrier();
  if (lane >= 1 && lane < 8) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (lane == 1) v = make_uint4(ald32(s + kOffValOff), 0, SPL_SLOT_DEFAULT_TYPE, 0);
    st16_wt(s + 16 * lane, v);
  }
  if (lane == 0 && a.has_vec16()) a.nrm2()[j] = 0.f;
  release();
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) ast64(epoch_ptr(s), ej + 2);
  __builtin_amdgcn_wave_barrier();
  return 1;
}

__device__ __forceinline__ void uni_he(const Arena& a, uint64_t pos, uint64_t& h, uint64_t& e) {
  u32x4c_t v = ld16c(a.slot(pos) + kOffHash);  // hash + epoch in one request (every lane: one line)
  vm_wait(v);
  h = (uint64_t)__builtin_amdgcn_readfirstlane(v.x) | ((uint64_t)__builtin_amdgcn_readfirstlane(v.y) << 32);
  e = (uint64_t)__builtin_amdgcn_readfirstlane(v.z) | ((uint64_t)__builtin_amdgcn_readfirstlane(v.w) << 32);
}

__global__ __launch_bounds__(64 * kRhWaves) void k_rehash(spl_arena_t aa, RhCounters* __restrict__ cnt) {
  const Arena a = from_api(aa);
  __shared__ uint32_t hpos_all[kRhWaves][kRhHoles];
  __shared__ uint64_t hep_all[kRhWaves][kRhHoles];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t* hpos = hpos_all[wave];
  uint64_t* hep = hep_all[wave];
  const uint64_t n = a.slots;
  const uint64_t w = blockIdx.x * (uint64_t)kRhWaves + wave;
  const uint64_t r0 = w * kRhRange;
  if (r0 >= n) return;
  const uint64_t r1 = r0 + kRhRange < n ? r0 + kRhRange : n;
  const uint64_t limit = (r1 - r0) + kRhTail < n ? (r1 - r0) + kRhTail : n;  // slots walked at most
  unsigned long long moved = 0, clusters = 0, skipped = 0, dmax = 0;
  // holes: tombstones in walk order, a ring of kRhHoles (h0 = oldest); when full the oldest is dropped
  int nh = 0, h0 = 0;
  bool overflow = false;
  auto at = [&](int t) { return (h0 + t) & (kRhHoles - 1); };
  uint64_t cs = r0;          // origin of the current cluster piece
  bool in_cluster = false;
  auto set_hole = [&](int t, uint32_t p, uint64_t e) {
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) { hpos[at(t)] = p; hep[at(t)] = e; }
    __builtin_amdgcn_wave_barrier();
  };
  auto drop_hole = [&](int k) {  // order kept
    for (int t = k; t < nh - 1; ++t) {
      const uint32_t p = hpos[at(t + 1)];
      const uint64_t e = hep[at(t + 1)];
      set_hole(t, p, e);
    }
    --nh;
  };
  for (uint64_t step = 0, pos = r0; step < limit; ++step) {
    uint64_t h, e;
    uni_he(a, pos, h, e);
    const bool odd = e & 1;
    if (h != 0) {
      const uint64_t dsp = cyc(pos, h % n, n);
      dmax = dsp > dmax ? dsp : dmax;
    }
    if (h == 0 && e == 0) {  // virgin: the cluster piece ends here (holes before it serve no later key)
      if (in_cluster && overflow) ++skipped;
      nh = 0;
      h0 = 0;
      overflow = false;
      in_cluster = false;
      if (step + 1 >= r1 - r0) break;  // past the own range: done
      pos = pos + 1 == n ? 0 : pos + 1;
      cs = pos;
      continue;
    }
    if (!in_cluster) {
      in_cluster = true;
      ++clusters;
    }
    const int64_t rp = (int64_t)cyc(pos, cs, n);
    if (h == 0 && !odd) {
      if (nh == kRhHoles) {
        h0 = (h0 + 1) & (kRhHoles - 1);
        --nh;
        overflow = true;
      }
      set_hole(nh, (uint32_t)pos, e);
      ++nh;
    } else if (!odd && nh > 0) {
      // live key: the first hole on its own probe path (between its home and its slot)
      const uint64_t home = h % n;
      const uint64_t rh = cyc(pos, home, n) >= cyc(pos, cs, n) ? 0 : cyc(home, cs, n);
      int k = -1;
      for (int t0 = 0; t0 < nh && k < 0; t0 += 64) {
        const int t = t0 + lane;
        const uint64_t rq = t < nh ? cyc(hpos[at(t)], cs, n) : 0;
        const bool ok = t < nh && rq >= rh && (int64_t)rq < rp;
        const uint64_t bm = __ballot(ok);
        if (bm) k = t0 + __builtin_ctzll(bm);
      }
      if (k >= 0) {
        const uint64_t q = hpos[at(k)], eq = hep[at(k)];
        const int st = move_online(a, q, eq, pos, h, e, lane);
        if (st == 1) {
          ++moved;
          drop_hole(k);
          set_hole(nh, (uint32_t)pos, e + 2);  // the vacated slot is the newest hole
          ++nh;
        } else {
          if (st == -1) drop_hole(k);
          else set_hole(k, (uint32_t)q, eq + 2);
        }
      }
    }  // else: live without a hole before it, or busy (a writer in flight: never moved)
    pos = pos + 1 == n ? 0 : pos + 1;
  }
  if (lane == 0) {
    atomicAdd(&cnt->moved, moved);
    atomicAdd(&cnt->clusters, clusters);
    atomicAdd(&cnt->skipped, skipped);
    atomicMax(&cnt->dmax, dmax);
  }
}

// Phase 2 of the pass, after every move (a kernel boundary): tombstones no probe chain needs become
// virgin slots again, which ends the chains there.  A tombstone at t is needed iff some entry at a
// later slot p has its home at or before t (its probe from home to p walks over t); entries are
// at most dmax slots from their homes (phase 1 saw every keyed slot, in-flight inserts of before
// the pass included: their hash is published before their seq check, and no insert is decided
// after the pass opened), so a wave decides its 1024-slot range from the slots up to dmax past it:
// a backward sweep keeps the minimum home position of the entries after each slot (64 slots per
// step, suffix minimum across the wave), and a tombstone whose every later entry starts after it
// is reclaimed by a CAS from the epoch just read (a slot that changed meanwhile keeps its state).
// A claim whose hash is not visible counts as reaching back over its whole window.
constexpr uint64_t kReclaimMaxD = 1u << 20;  // beyond this displacement the sweep would walk too far: skipped
__global__ __launch_bounds__(256) void k_reclaim(spl_arena_t aa, const RhCounters* __restrict__ rc_in,
                                                 RhCounters* __restrict__ cnt) {
  const Arena a = from_api(aa);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t n = a.slots;
  const uint64_t r0 = (blockIdx.x * 4ull + wave) * kRhRange;
  if (r0 >= n) return;
  const uint64_t D = rc_in->dmax;
  if (D > kReclaimMaxD) return;
  const int64_t len = (int64_t)(kRhRange < n - r0 ? kRhRange : n - r0);
  const int64_t span = (int64_t)((uint64_t)len + D < n ? (uint64_t)len + D : n);
  const int64_t kNone = INT64_MAX;
  int64_t carry = kNone;  // minimum home position (range-relative) of the entries past this chunk
  unsigned long long rec = 0;
  for (int64_t xc = (span - 1) / 64 * 64; xc >= 0; xc -= 64) {
    const int64_t x = xc + lane;
    int64_t hr = kNone;
    bool tomb = false;
    uint64_t eobs = 0, p = 0;
    if (x < span) {
      p = (r0 + (uint64_t)x) % n;
      u32x4c_t v = ld16c(a.slot(p) + kOffHash);
      vm_wait(v);
      const uint64_t h = lo64(v), e = hi64(v);
      if (h != 0) hr = x - (int64_t)cyc(p, h % n, n);
      else if (e & 1) hr = x - (int64_t)D - 1;
      else if (e != 0) { tomb = true; eobs = e; }
    }
    int64_t m = hr;  // inclusive suffix minimum over the chunk's lanes
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t o = __shfl_down(m, off, 64);
      if (lane + off < 64) m = o < m ? o : m;
    }
    int64_t ex = __shfl_down(m, 1, 64);  // entries strictly after x
    if (lane == 63) ex = kNone;
    ex = carry < ex ? carry : ex;
    if (tomb && x < len && ex > x && acas64(epoch_ptr(a.slot(p)), eobs, 0)) ++rec;
    const int64_t cm = __shfl(m, 0, 64);
    carry = cm < carry ? cm : carry;
  }
  for (int o = 32; o > 0; o >>= 1) rec += __shfl_xor(rec, o, 64);
  if (lane == 0 && rec) atomicAdd(&cnt->reclaimed, rec);
}

// open (begin = 1) or close (0) a maintenance pass: MaintRec::seq odd while it runs.  Opening is a
// CAS from an even seq (ok[0] = 1 when this call opened it); closing adds one.  The fence after
// the store orders it before every later access of the stream's next kernel (k_rehash).
__global__ void k_maint_mark(spl_arena_t aa, int begin, int pid, uint64_t t0, unsigned long long* ok) {
  const Arena a = from_api(aa);
  if (threadIdx.x != 0 || !a.has_side()) return;
  MaintRec* m = (MaintRec*)(a.side() + kSideMaintOff);
  if (begin) {
    const uint64_t s0 = ald64(&m->seq);
    const bool won = !(s0 & 1) && acas64(&m->seq, s0, s0 + 1);
    if (won) {
      ast32(&m->pid, (uint32_t)pid);
      ast64(&m->t0_ns, t0);
    }
    *ok = won ? 1ull : 0ull;
  } else {
    aadd64(&m->seq, 1);
    aadd64(&m->passes, 1);
    ast32(&m->pid, 0u);
    *ok = 1ull;
  }
  release();
}

// ------------------------------------------------------------ full rebuild --
// For an arena whose clusters have merged (few never-used slots left, e.g. high load under churn)
// the in-place compaction only moves keys within ranges; instead every live entry is copied out,
// the slot array cleared, and the entries re-inserted in parallel (each at the first free slot
// from its home: no tombstones at all afterwards).  Temporary memory: one record of stride +
// max_val (+ the bf16 copy and norm) bytes per live entry.  EXCLUSIVE (unlike k_rehash): no other
// op of any process may run on the arena meanwhile (spl_hbm_rehash_ex SPL_REHASH_FULL).
struct RbGeom {
  uint32_t rec;      // bytes per record (16-B multiple)
  uint32_t off_val;  // value row in the record
  uint32_t off_v16;  // bf16 vector (vec16 arenas)
  uint32_t off_n2;   // squared norm
};

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

// Cluster compaction, ONLINE (k_rehash, then k_reclaim; the caller opens and closes the pass with
// spl_arena_maint_mark).  `counters`: device u64[5] {moved, reclaimed, clusters, skipped (clusters
// with more than kRhHoles tombstones, compacted only up to there), largest displacement}, zeroed by
// the caller.
int spl_arena_rehash(spl_arena_t a, void* counters, hipStream_t s) {
  if (!a.base || !counters || !(a.flags & SPL_ARENA_SIDE)) return (int)hipErrorInvalidValue;
  const uint64_t waves = ((uint64_t)a.slots + kRhRange - 1) / kRhRange;
  const uint64_t blocks = (waves + kRhWaves - 1) / kRhWaves;
  hipLaunchKernelGGL(k_rehash, dim3((unsigned)blocks), dim3(64 * kRhWaves), 0, s, a, (RhCounters*)counters);
  hipLaunchKernelGGL(k_reclaim, dim3((unsigned)blocks), dim3(256), 0, s, a, (const RhCounters*)counters,
                     (RhCounters*)counters);
  return (int)hipGetLastError();
}

// Open (begin 1) / close (0) a maintenance pass; `ok`: device u64, 1 when the open won.
int spl_arena_maint_mark(spl_arena_t a, int begin, int pid, uint64_t t0_ns, void* ok, hipStream_t s) {
  if (!a.base || !ok || !(a.flags & SPL_ARENA_SIDE)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_maint_mark, dim3(1), dim3(64), 0, s, a, begin, pid, t0_ns, (unsigned long long*)ok);
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
