// arena_dev.hpp — device-side format-v4 arena operations for gfx950.
//
// Owner-computes design: every mutation of an HBM arena
// runs on the GPU that holds it, so the seqlock CAS / fetch_add are
// agent-scope atomics on device memory.  Visibility across workgroups and
// XCDs follows the CDNA4 rules (MI355X_MICROARCH.md, "Workgroup dispatch, XCD
// placement & inter-workgroup visibility"):
//   * probe words (hash, epoch, key, val_len) are read with agent-scope
//     relaxed atomic loads (global_load ... sc1: L1-bypassing, never stale);
//   * a writer stores the payload with plain 16-B stores, then ONE agent
//     release fence (buffer_wbl2 sc1) + explicit s_waitcnt vmcnt(0) — the
//     guide's ROCm 7.2 hazard fix — before publishing hash and epoch;
//   * a reader takes the epoch with an agent ACQUIRE load (buffer_inv sc1 on
//     this CU's L1), so its plain 16-B value loads cannot hit stale L1 lines;
//     s_waitcnt vmcnt(0) then orders the value loads before the closing epoch
//     load.
//
// Seqlock per slot (same protocol as the host backend, store_host.cpp):
//   writer : CAS epoch even->odd, write payload, release, publish hash,
//            epoch += 1;  unset rewinds the epoch to 2, retrain to 4.
//   reader : e1 = epoch (acquire); odd -> EAGAIN; key + value; e2 = epoch;
//            e1 != e2 -> EAGAIN.
// Probe chains end at a virgin slot (hash 0 && epoch 0).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "splinter_layout.hpp"
#include "arena_api.h"

namespace spl {
namespace dev {

enum : int32_t {
  kOk = 0,
  kAgain = -11,    // -EAGAIN
  kNoEnt = -2,     // -ENOENT
  kNoSpc = -28,    // -ENOSPC
  kMsgSize = -90,  // -EMSGSIZE
  kProto = -91,    // -EPROTOTYPE (Linux errno 91)
  kInval = -22,
};

struct Arena {
  uint8_t* base;
  uint32_t slots;
  uint32_t max_val;
  uint32_t stride;
  uint32_t flags;  // bit0: event bus armed (maintain the dirty mask)
  uint64_t notify = 0;  // device address of the host-mapped notify word (event-bus proxy), 0 = none
  __device__ __forceinline__ splinter_header* hdr() const { return (splinter_header*)base; }
  __device__ __forceinline__ uint8_t* slot(size_t i) const { return base + kHeaderBytes + i * (size_t)stride; }
  __device__ __forceinline__ uint8_t* value(size_t i) const {
    return base + kHeaderBytes + (size_t)slots * stride + i * (size_t)max_val;
  }
  // side region (splinter_layout.hpp): present when the allocation was made with it
  __device__ __forceinline__ bool has_side() const { return flags & SPL_ARENA_SIDE; }
  __device__ __forceinline__ bool has_vec16() const { return flags & SPL_ARENA_VEC16; }
  __device__ __forceinline__ uint8_t* side() const { return base + side_offset(slots, stride, max_val); }
  __device__ __forceinline__ float* nrm2() const { return (float*)(side() + side_nrm2_offset()); }
  __device__ __forceinline__ uint16_t* vec16(size_t i) const {
    return (uint16_t*)(side() + side_vec16_offset(slots)) + i * kEmbedDim;
  }
};

// ---------------------------------------------------- bf16 vector copy ------
// Vector of one slot, distributed over a wave as the embedding kernels hold it (lane l: float4
// chunks l, l + 64, l + 128 of the 768 dims) -> the side region's bf16 copy (three 8-B stores per
// lane, coalesced) and squared norm (wave sum; lane 0 stores it).  Called while the caller holds
// the slot's seqlock, before its release fence: the copy is published with the fp32 vector.
__device__ __forceinline__ void write_vec16_wave(const Arena& a, size_t idx, const float4 (&v)[3], int lane) {
  if (!a.has_vec16()) return;
  uint2* d = (uint2*)a.vec16(idx);
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
    const bf2_t lo = {(__bf16)v[c].x, (__bf16)v[c].y}, hi = {(__bf16)v[c].z, (__bf16)v[c].w};
    d[lane + 64 * c] = make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
    ss += v[c].x * v[c].x + v[c].y * v[c].y + v[c].z * v[c].z + v[c].w * v[c].w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if (lane == 0) a.nrm2()[idx] = ss;
}
// one thread's form (the ring worker, single lanes): the whole vector from `src` (768 floats)
__device__ __forceinline__ void write_vec16_one(const Arena& a, size_t idx, const float* src) {
  if (!a.has_vec16()) return;
  uint2* d = (uint2*)a.vec16(idx);
  float ss = 0.f;
  for (uint32_t c = 0; c < kEmbedDim / 4; ++c) {
    const float4 x = ((const float4*)src)[c];
    typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
    const bf2_t lo = {(__bf16)x.x, (__bf16)x.y}, hi = {(__bf16)x.z, (__bf16)x.w};
    d[c] = make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
    ss += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
  }
  a.nrm2()[idx] = ss;
}
// the slot holds no vector (fresh insert, unset, retrain): its norm 0 marks the copy dead
__device__ __forceinline__ void clear_vec16(const Arena& a, size_t idx) {
  if (a.has_vec16()) a.nrm2()[idx] = 0.f;
}

// ------------------------------------------------------------- atomics --
__device__ __forceinline__ uint64_t ald64(const void* p) {
  return __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ald64_acq(const void* p) {
  return __hip_atomic_load((const uint64_t*)p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ald32(const void* p) {
  return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint8_t ald8(const void* p) {
  return __hip_atomic_load((const uint8_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast64(void* p, uint64_t v) {
  __hip_atomic_store((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast32(void* p, uint32_t v) {
  __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast8(void* p, uint8_t v) {
  __hip_atomic_store((uint8_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool acas64(void* p, uint64_t expect, uint64_t want) {
  return __hip_atomic_compare_exchange_strong((uint64_t*)p, &expect, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t aadd64(void* p, uint64_t v) {
  return __hip_atomic_fetch_add((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void aor64(void* p, uint64_t v) {
  __hip_atomic_fetch_or((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void aand64(void* p, uint64_t v) {
  __hip_atomic_fetch_and((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait for every outstanding vector-memory op of this wave (loads AND stores).
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Agent release: write back this XCD's L2, then wait (explicit wait: the
// ROCm 7.2 compiler may drop the fence's own wait, MI355X guide hazard note).
__device__ __forceinline__ void release() {
  drain();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  drain();
}

// Kernel-side view of a launch descriptor.  The event bus counts as armed when the launching
// process says so (flags bit 0) OR the device header records an owner (any process on the node
// may have called splinter_event_bus_init on this arena: hbm_store.hip mirrors owner_pid into
// the device header), so batch kernels of every attached process maintain the dirty mask.
__device__ __forceinline__ Arena from_api(const spl_arena_t& aa) {
  Arena d;
  d.base = (uint8_t*)aa.base;
  d.slots = aa.slots;
  d.max_val = aa.max_val;
  d.stride = aa.stride;
  d.notify = aa.notify;
#ifdef SPL_NO_BUS_PROBE
  d.flags = aa.flags;
#else
  const uint32_t owner = __hip_atomic_load((const uint32_t*)&((splinter_header*)aa.base)->event_bus.owner_pid,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  d.flags = aa.flags | (owner != 0 ? 1u : 0u);
#endif
  return d;
}

// Wake the host event-bus proxy: one system-scope (vector) store of 1 into the host-mapped
// notify word, after this lane's dirty-mask updates have drained.  Idempotent, so any number of
// blocks / kernels / processes may store it; the proxy clears it before it signals the eventfd.
__device__ __forceinline__ void notify_host(const Arena& a) {
  if (!(a.flags & 1u) || !a.notify) return;
  drain();
  __hip_atomic_store((uint32_t*)a.notify, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------- keys ----
// A key arrives as a NUL-padded record of `kstride` bytes (16/32/48/64).
// Canonical form: first 63 bytes, NUL padded to 64, FNV-1a over its length.
// KW = key words held in registers: a batch whose records are <= 4*KW bytes
// (kstride 16 -> KW 4) keeps only those words live, the rest are the constant
// 0 (word(i) below), which frees 12 VGPRs per key for occupancy in the
// latency-bound batch kernels (U keys per lane).
template <int KW = 16>
struct KeyT {
  static_assert(KW == 4 || KW == 8 || KW == 16, "key words");
  uint32_t w[KW];  // canonical key words (registers: every index is static)
  uint32_t len;
  uint64_t hash;
  __device__ __forceinline__ uint32_t word(int i) const { return i < KW ? w[i < KW ? i : 0] : 0u; }
  __device__ __forceinline__ uint64_t qword(int q) const { return ((uint64_t)word(2 * q + 1) << 32) | word(2 * q); }
};
using Key = KeyT<16>;

// Canonicalise key words already in k.w (the first kstride bytes of a record): length, FNV-1a,
// and every byte at or past the terminating NUL (or byte 63) zeroed.
template <int KW>
__device__ __forceinline__ void canon_key(KeyT<KW>& k, int kstride) {
  uint64_t h = kFnvOffset;
  uint32_t len = 0;
  bool live = true;
#pragma unroll
  for (int wi = 0; wi < KW; ++wi) {
    if (wi * 4 < kstride) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t ch = (k.w[wi] >> (8 * b)) & 0xffu;
        live = live && ch != 0 && (wi * 4 + b) < 63;
        if (live) { h = (h ^ ch) * kFnvPrime; ++len; }
      }
    }
  }
#pragma unroll
  for (int wi = 0; wi < KW; ++wi) {  // zero every byte at or past len
    const int keep = (int)len - 4 * wi;
    const uint32_t m = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u);
    k.w[wi] &= m;
  }
  k.len = len;
  k.hash = h;
}

template <int KW>
__device__ __forceinline__ void load_key(KeyT<KW>& k, const char* rec, int kstride) {
  const uint4* r = (const uint4*)rec;
#pragma unroll
  for (int c = 0; c < KW / 4; ++c) {
    uint4 v = (c * 16 < kstride) ? r[c] : make_uint4(0, 0, 0, 0);
    k.w[4 * c + 0] = v.x; k.w[4 * c + 1] = v.y; k.w[4 * c + 2] = v.z; k.w[4 * c + 3] = v.w;
  }
  canon_key(k, kstride);
}

// Compare the stored key with ours through sc1 loads, 8 bytes at a time, up
// to and including our terminating NUL (stored keys are NUL padded).
template <int KW>
__device__ __forceinline__ bool key_eq(const uint8_t* slot, const KeyT<KW>& k) {
  const uint8_t* sk = slot + kOffKey;
  const uint32_t nq = (k.len >> 3) + 1;  // 8-byte words holding the key + NUL
  bool eq = true;
  // a KW-word key is at most 4*KW bytes long: its NUL lies within q-word KW/2
  constexpr int kMaxQ = KW / 2 + 1 < 8 ? KW / 2 + 1 : 8;
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) {
    if ((uint32_t)q < nq) {
      const uint64_t v = ald64(sk + 8 * q);
      eq = eq && v == k.qword(q);
    }
  }
  return eq;
}

template <int KW>
__device__ __forceinline__ void store_key(uint8_t* slot, const KeyT<KW>& k) {
  uint4* d = (uint4*)(slot + kOffKey);
#pragma unroll
  for (int c = 0; c < 4; ++c) d[c] = make_uint4(k.word(4 * c), k.word(4 * c + 1), k.word(4 * c + 2), k.word(4 * c + 3));
}

// ---------------------------------------------------- 16-B coherent probes --
// global_load_dwordx4 ... sc1: L1-bypassing and L2-served exactly like the relaxed agent-scope
// 8-B atomic loads above (MI355X_MICROARCH.md, agent-scope forms), but ONE request per 16 B: a
// probe of (hash, epoch) + key takes 2 requests instead of 4-5 (8-B sc1 accesses run at roughly
// the same request rate, so half the bytes each).  hipcc does not track inline-asm loads in its
// own waits: a result is valid only after vm_wait() on it, which ties the registers.
typedef unsigned int u32x4c_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4c_t ld16c(const void* p) {
  u32x4c_t r;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ void vm_wait(u32x4c_t& a) { asm volatile("s_waitcnt vmcnt(0)" : "+v"(a)::"memory"); }
__device__ __forceinline__ void vm_wait(u32x4c_t& a, u32x4c_t& b) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b)::"memory");
}
__device__ __forceinline__ void vm_wait(u32x4c_t& a, u32x4c_t& b, u32x4c_t& c) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b), "+v"(c)::"memory");
}
typedef unsigned int u32x2c_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2c_t ld8c(const void* p) {
  u32x2c_t r;
  asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ void vm_wait2(u32x2c_t& a, u32x2c_t& b) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b)::"memory");
}
__device__ __forceinline__ uint64_t lo64(const u32x4c_t& v) { return ((uint64_t)v.y << 32) | v.x; }
__device__ __forceinline__ uint64_t u64of(const u32x2c_t& v) { return ((uint64_t)v.y << 32) | v.x; }
__device__ __forceinline__ void vm_wait1(u32x2c_t& a) { asm volatile("s_waitcnt vmcnt(0)" : "+v"(a)::"memory"); }
__device__ __forceinline__ uint64_t hi64(const u32x4c_t& v) { return ((uint64_t)v.w << 32) | v.z; }

// Stored-key probe in 16-B chunks: chunk 0 always, the rest only where our key + NUL reaches
// (a KW-word key is at most 4*KW bytes: chunk KW/4 can still hold its NUL).
template <int KW>
struct KeyProbe {
  static constexpr int kMaxC = KW / 4 + 1 < 4 ? KW / 4 + 1 : 4;
  u32x4c_t c[kMaxC];
  __device__ __forceinline__ void issue(const uint8_t* slot, const KeyT<KW>& k) {
    const int nch = ((int)k.len >> 4) + 1;
    c[0] = ld16c(slot + kOffKey);
#pragma unroll
    for (int i = 1; i < kMaxC; ++i) {
      c[i] = u32x4c_t{0u, 0u, 0u, 0u};
      if (i < nch) c[i] = ld16c(slot + kOffKey + 16 * i);
    }
  }
  __device__ __forceinline__ void wait() {
#pragma unroll
    for (int i = 0; i < kMaxC; ++i) vm_wait(c[i]);
  }
  __device__ __forceinline__ bool eq(const KeyT<KW>& k) const {
    const int nch = ((int)k.len >> 4) + 1;
    bool e = true;
#pragma unroll
    for (int i = 0; i < kMaxC; ++i)
      if (i < nch)
        e = e && c[i].x == k.word(4 * i) && c[i].y == k.word(4 * i + 1) && c[i].z == k.word(4 * i + 2) &&
            c[i].w == k.word(4 * i + 3);
    return e;
  }
};

__device__ __forceinline__ uint64_t slot_hash(const uint8_t* s) { return ald64(s + kOffHash); }
__device__ __forceinline__ uint64_t slot_epoch(const uint8_t* s) { return ald64(s + kOffEpoch); }
__device__ __forceinline__ uint64_t* epoch_ptr(uint8_t* s) { return (uint64_t*)(s + kOffEpoch); }

// ------------------------------------------------------ online maintenance --
// The maintenance pass (arena_maint.hip k_rehash) moves live entries toward their home slots
// while batch and per-call ops keep running: each move holds BOTH slots' seqlocks (destination
// tombstone and source claimed by epoch CAS), publishes the entry at the destination, then
// releases the source as a tombstone.  A hit is covered by the slot's own seqlock.  An "absent"
// outcome is not: a probe can pass the destination before the entry lands there and reach the
// source after it was cleared.  So the side header's MaintRec::seq is odd while a pass runs, and
// an absent outcome (get miss, insert decision, unset / update of a missing key) is trusted only
// when seq was even before the probe's loads and is unchanged after them; otherwise the op
// reports EAGAIN (retry).  Reference contract: a miss only after the whole chain was scanned
// (/root/reference/splinter.c:431-464), purge beside live ops (splinter.c:302-318).
constexpr long kMaintMiss = -2;  // probe result: absent, but a maintenance pass overlapped it
__device__ __forceinline__ uint64_t* maint_ptr(const Arena& a) { return (uint64_t*)(a.side() + kSideMaintOff); }
// seq before a probe: acquire-ordered, no later load of the probe can be performed before it
__device__ __forceinline__ uint64_t maint_begin(const Arena& a) {
  return a.has_side() ? __hip_atomic_load(maint_ptr(a), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) : 0;
}
// after a probe that found nothing: every load of the probe has returned (the fence waits
// vmcnt(0)) before seq is read again
__device__ __forceinline__ bool maint_quiet(const Arena& a, uint64_t s0) {
  if (!a.has_side()) return true;
  if (s0 & 1) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return ald64(maint_ptr(a)) == s0;
}
// the same check with seq already re-read by the caller after its probe loads returned
__device__ __forceinline__ bool maint_same(uint64_t s0, uint64_t s1) { return !(s0 & 1) && s0 == s1; }
// seq word load issued without a wait (batched into a round trip the caller waits for anyway)
__device__ __forceinline__ const void* maint_addr(const Arena& a) {
  // no side region: the header's (magic, version) word, constant and even
  return a.has_side() ? (const void*)maint_ptr(a) : (const void*)a.base;
}

// Locate `k`; returns the slot index, -1 (absent) or kMaintMiss.  Pure lookup (no seqlock).
template <int KW>
__device__ __forceinline__ long find(const Arena& a, const KeyT<KW>& k) {
  const uint64_t s0 = maint_begin(a);
  size_t idx = (size_t)(k.hash % a.slots);
  for (uint32_t i = 0; i < a.slots; ++i) {
    const uint8_t* s = a.slot(idx);
    const uint64_t sh = slot_hash(s);
    if (sh == k.hash && key_eq(s, k)) return (long)idx;
    if (sh == 0 && slot_epoch(s) == 0) break;
    if (++idx == a.slots) idx = 0;
  }
  return maint_quiet(a, s0) ? -1 : kMaintMiss;
}
// status of a failed find
__device__ __forceinline__ int32_t miss_rc(long i) { return i == kMaintMiss ? kAgain : kNoEnt; }

// ------------------------------------------------------------- signals --
__device__ __forceinline__ void pulse(const Arena& a, const uint8_t* s) {
  splinter_header* H = a.hdr();
  const uint64_t wm = ald64(s + kOffWatch);
  for (uint64_t m = wm; m; m &= m - 1) aadd64(&H->signal_groups[__builtin_ctzll(m)].counter, 1);
  const uint64_t bl = ald64(s + kOffBloom);
  for (uint64_t m = bl; m; m &= m - 1) {
    const uint8_t g = ald8(&H->bloom_watches[__builtin_ctzll(m)]);
    if (g < SPLINTER_MAX_GROUPS) aadd64(&H->signal_groups[g].counter, 1);
  }
}

// pulse with masks already in registers (Claim::wm / bl): no extra round trip at the end of a set
__device__ __forceinline__ void pulse_masks(const Arena& a, uint64_t wm, uint64_t bl) {
  splinter_header* H = a.hdr();
  for (uint64_t m = wm; m; m &= m - 1) aadd64(&H->signal_groups[__builtin_ctzll(m)].counter, 1);
  for (uint64_t m = bl; m; m &= m - 1) {
    const uint8_t g = ald8(&H->bloom_watches[__builtin_ctzll(m)]);
    if (g < SPLINTER_MAX_GROUPS) aadd64(&H->signal_groups[g].counter, 1);
  }
}

__device__ __forceinline__ void mark_dirty(const Arena& a, size_t idx) {
  if (!(a.flags & 1u)) return;
  const size_t m = idx % kDirtyBits;
  aor64(&a.hdr()->event_bus.dirty_mask[m / 64], 1ull << (m % 64));
}

// ------------------------------------------------------------- writes --
__device__ __forceinline__ bool scrub_flags(const Arena& a, bool& hybrid) {
  const uint8_t f = ald8(&a.hdr()->core_flags);
  hybrid = (f & SPL_SYS_HYBRID_SCRUB) != 0;
  return (f & SPL_SYS_AUTO_SCRUB) != 0;
}

__device__ __forceinline__ uint32_t keep_mask(int keep) {
  return keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u);
}

// Copy a value into slot idx's value region in 16-B chunks.  The tail of the
// last chunk is zeroed; with scrubbing the region is zeroed to the 64-B
// boundary (hybrid) or to max_val (full) — the reference's mop modes
// (reference splinter.c:393-401).  Source records are 16-B aligned.
// Memory-ordering discipline of the payload (template parameter MO):
//   0  plain 16-B payload accesses + agent release (writer) / acquire (reader)
//   1  sc1 (L1-bypassing, write-through) 8-B atomic payload accesses, no fences
//   2  unordered (measurement only: NOT a valid seqlock)
//   3  write-through: 16-B `global_store_dwordx4 ... sc1` payload stores (no L2 dirty lines),
//      published by every writing wave's vmcnt(0) drain + the atomic epoch increment, with no
//      L2 write-back fence (cdna_hip_programming.md Guideline 16, recipe R1); readers unchanged
//      (agent acquire + plain loads)
// Write-through 16-B store.  hipcc does not count asm stores in its waits: callers drain()
// before publishing; `s_nop 1` keeps the data registers live until the store has read them.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_wt(void* p, uint4 v) {
  const u32x4_t d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
}

template <int MO>
__device__ __forceinline__ void st16(void* p, uint4 v) {
  if constexpr (MO == 3) {
    st16_wt(p, v);
  } else if constexpr (MO == 1) {
    ast64(p, ((uint64_t)v.y << 32) | v.x);
    ast64((uint8_t*)p + 8, ((uint64_t)v.w << 32) | v.z);
  } else {
    *(uint4*)p = v;
  }
}
template <int MO>
__device__ __forceinline__ uint4 ld16(const void* p) {
  if constexpr (MO == 1) {
    const uint64_t a = ald64(p), b = ald64((const uint8_t*)p + 8);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
  } else {
    return *(const uint4*)p;
  }
}

// Store the first nb (< 16) bytes of v: the last chunk of a value row whose length (max_val)
// is not a multiple of 16 must not spill into the next row.
__device__ __forceinline__ void store_partial(uint8_t* d, uint4 v, uint32_t nb) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (uint32_t b = 0; b < nb; ++b) d[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
}

template <int MO>
__device__ __forceinline__ void write_value(const Arena& a, size_t idx, const uint8_t* src, uint32_t len, bool scrub,
                                            bool hybrid) {
  uint4* dst = (uint4*)a.value(idx);
  const uint4* s4 = (const uint4*)src;
  const uint32_t n16 = (len + 15) >> 4;
  // 8 source loads in flight per batch (one memory round trip per 128 B instead of one per
  // 16 B); the loads are unconditional (clamped into the record) so hipcc does not branch and
  // wait around each one
  for (uint32_t b = 0; b < n16; b += 8) {
    uint4 t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) t[q] = s4[min(b + (uint32_t)q, n16 - 1)];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint32_t c = b + (uint32_t)q;
      if (c >= n16) break;
      if (c == n16 - 1 && (len & 15)) {
        const int r = (int)(len & 15);
        t[q].x &= keep_mask(r); t[q].y &= keep_mask(r - 4); t[q].z &= keep_mask(r - 8); t[q].w &= keep_mask(r - 12);
      }
      if (c * 16 + 16 > a.max_val) store_partial((uint8_t*)(dst + c), t[q], a.max_val - c * 16);
      else st16<MO>(dst + c, t[q]);
    }
  }
  uint32_t done = n16 << 4;
  if (scrub) {
    uint32_t end = hybrid ? ((len + 63u) & ~63u) : a.max_val;
    if (end > a.max_val) end = a.max_val;
    for (; done + 16 <= end; done += 16) st16<MO>(dst + (done >> 4), make_uint4(0, 0, 0, 0));
  }
}

// ------------------------------------------------------------ SET ------
// A set is split into three phases so that a batch kernel can lock several
// slots per lane, write all their payloads, and pay ONE agent release fence
// for all of them (a release fence writes back the XCD's L2 and is
// serialised per XCD at ~1.7 us, which otherwise caps sets near 0.3 G/s).
//   claim_set   locate the key (update) or claim a free slot (insert); on
//               success the slot's epoch is odd and owned by this lane
//   write_set   payload with plain 16-B stores
//   release()   once, by the caller, covering every write_set of the wave
//   finish_set  epoch += 1 (the hash is already in place)
// Inserts publish key + hash EARLY (right after the claim, with an
// "insert in flight" marker val_len = kInsertMark) so that racing inserters
// of one key see each other: the claim that sits earlier on the probe chain
// wins, the later one backs off with EAGAIN.  Readers that meet a slot with
// their hash and an odd epoch report EAGAIN, as for any in-flight write.
constexpr uint32_t kInsertMark = 0xFFFFFFFFu;

struct Claim {
  long idx;       // slot index (valid when rc == kOk)
  bool fresh;     // true: insert into a free slot
  int32_t rc;
  uint64_t wm = 0, bl = 0;  // watcher mask / bloom labels read while holding the slot (pulse_masks)
  uint64_t ep = 0;          // the held (odd) epoch
};

__device__ __forceinline__ void clear_claim(const Arena& a, long idx) {
  uint8_t* s = a.slot((size_t)idx);
  ast64(s + kOffHash, 0);
  ast32(s + kOffValLen, 0);
  drain();
  aadd64(epoch_ptr(s), 1);
}

// s0: the maintenance seq read before this probe (maint_begin, or a value the caller waited for
// before issuing the probe's loads); an insert is decided only when no pass overlapped the probe.
template <int KW>
__device__ Claim claim_set(const Arena& a, const KeyT<KW>& k, uint64_t s0) {
  const size_t home = (size_t)(k.hash % a.slots);
  long free_idx = -1;
  uint64_t free_ep = 0;
  size_t idx = home;
  for (uint32_t i = 0; i < a.slots; ++i) {
    uint8_t* s = a.slot(idx);
    // hash, epoch and key in ONE round trip of 16-B coherent loads (the key compare is speculative)
    u32x4c_t he = ld16c(s + kOffHash);
#ifndef SPL_SET_RECHECK
    // ... and the watcher mask / labels the set will pulse (same 128-B slot line)
    u32x4c_t wc0 = ld16c(s + kOffWatch), ab0 = ld16c(s + kOffAtime);
#endif
    KeyProbe<KW> kp;
    kp.issue(s, k);
    vm_wait(he);
#ifndef SPL_SET_RECHECK
    vm_wait(wc0, ab0);
#endif
    kp.wait();
    const uint64_t sh = lo64(he), e = hi64(he);
    const bool keq = kp.eq(k);
    if (sh == k.hash && keq) {  // update in place
      if ((e & 1) || !acas64(epoch_ptr(s), e, e + 1)) return Claim{-1, false, kAgain};
#ifndef SPL_SET_RECHECK
      // No re-check round trip after the claim: hash and epoch came from ONE 16-B load, every
      // change of the slot's hash or key happens under a claim that moves the epoch, so a CAS
      // that still finds the epoch read with hash == k.hash proves the slot held this key for the
      // whole window (a key compare against stale bytes can only fail, which sends the op down the
      // insert path, whose re-validation finds the slot).  Watcher mask and labels change by
      // atomics outside the seqlock (reference splinter.c:968-1003), so the probe-time values
      // are as current as a re-read would be.  SPL_SET_RECHECK restores the round trip.
      return Claim{(long)idx, false, kOk, lo64(wc0), hi64(ab0), e + 1};
#endif
      // re-check after the claim: hash + key together, with the watcher mask and labels the
      // set will pulse (same 128-B slot line, same round trip)
      u32x4c_t h2 = ld16c(s + kOffHash), wc = ld16c(s + kOffWatch), ab = ld16c(s + kOffAtime);
      kp.issue(s, k);
      vm_wait(h2, wc, ab);
      kp.wait();
      const uint64_t sh2 = lo64(h2), wm = lo64(wc), bl = hi64(ab);
      const bool keq2 = kp.eq(k);
      if (sh2 != k.hash || !keq2) {  // raced with unset / reuse
        aadd64(epoch_ptr(s), 1);
        return Claim{-1, false, kAgain};
      }
      return Claim{(long)idx, false, kOk, wm, bl, e + 1};
    }
    if (sh == 0 && !(e & 1)) {  // reusable (odd = someone's claim in flight: skip)
      if (free_idx < 0) { free_idx = (long)idx; free_ep = e; }
      if (e == 0) break;        // virgin slot ends the chain
    }
    if (++idx == a.slots) idx = 0;
  }
  if (free_idx < 0) return Claim{-1, false, kNoSpc};
  uint8_t* fs = a.slot((size_t)free_idx);
  if (!acas64(epoch_ptr(fs), free_ep, free_ep + 1)) return Claim{-1, false, kAgain};
  if (slot_hash(fs) != 0) { aadd64(epoch_ptr(fs), 1); return Claim{-1, false, kAgain}; }
  // early publication: marker, key, then hash (each visible before the next)
  ast32(fs + kOffValLen, kInsertMark);
#pragma unroll
  for (int q = 0; q < 8; ++q) ast64(fs + kOffKey + 8 * q, k.qword(q));
  drain();
  ast64(fs + kOffHash, k.hash);
  drain();
  // the insert is decided on "absent": not while a maintenance pass may be moving our key (the
  // claim and its publication have drained, so this read is performed after them and after the
  // probe -- a pass that starts later sees our claim as a busy slot and never moves across it)
  if (!maint_same(s0, ald64(maint_addr(a)))) {
    clear_claim(a, free_idx);
    return Claim{-1, false, kAgain};
  }
  // Re-validate the chain while holding the claim (the claim CAS + publish drains make
  // our claim visible before these reads, so of two racing inserters at least one sees
  // the other).  "Earlier claimant wins" alone is unsafe: the later inserter may not see
  // the earlier claim while the earlier one sees (and ignores) the later claim -> two
  // copies (found by the TSAN runs of the same protocol on the host store).  So:
  //   * our key published, or a claim in flight EARLIER on the chain  -> back off;
  //   * a claim in flight LATER on the chain that may be our key -> wait (bounded) for
  //     it to resolve -- it never waits for us -- then judge the slot again; back off if
  //     it is still in flight.
  // Epoch is read BEFORE hash + key (publishers store the hash, then bump the epoch).
  idx = home;
  bool before = true;
  for (uint32_t i = 0; i < a.slots; ++i) {
    if ((long)idx == free_idx) {
      before = false;
    } else {
      uint8_t* s = a.slot(idx);
      uint64_t e = slot_epoch(s);
      drain();
      uint64_t sh = slot_hash(s);
      bool keq = key_eq(s, k);
      const bool maybe_ours = sh == 0 || (sh == k.hash && keq);
      if (!before && (e & 1) && maybe_ours) {
        for (int t = 0; t < 64 && slot_epoch(s) == e; ++t) __builtin_amdgcn_s_sleep(8);
        e = slot_epoch(s);
        drain();
        sh = slot_hash(s);
        keq = key_eq(s, k);
      }
      const bool ours = sh == k.hash && keq;
      if (ours || ((e & 1) && sh == 0)) {
        clear_claim(a, free_idx);
        return Claim{-1, false, kAgain};
      }
      if (sh == 0 && e == 0) break;
    }
    if (++idx == a.slots) idx = 0;
  }
  return Claim{free_idx, true, kOk, 0, 0, free_ep + 1};
}

// Slot metadata part of a set (everything but the value bytes): fresh-slot defaults and val_len.
template <int MO = 0>
__device__ __forceinline__ void write_meta(const Arena& a, const Claim& c, uint32_t len) {
  uint8_t* s = a.slot((size_t)c.idx);
  if (c.fresh) {
    // fresh slot: metadata bytes 24..63 to defaults (type VOID), clear a stale vector
    st16<MO>(s + 32, make_uint4(0, 0, 0, 0));  // watcher_mask, ctime
    st16<MO>(s + 48, make_uint4(0, 0, 0, 0));  // atime, bloom
    ast8(s + kOffType, (uint8_t)SPL_SLOT_DEFAULT_TYPE);
    ast8(s + kOffUser, 0);
    if (a.stride == kSlotEmbedBytes) {
      uint4* ev = (uint4*)(s + kOffEmbed);
      for (uint32_t q = 0; q < kEmbedBytes / 16; ++q) st16<MO>(ev + q, make_uint4(0, 0, 0, 0));
      clear_vec16(a, (size_t)c.idx);
    }
  }
  ast32(s + kOffValLen, len);
}

// 16-B chunks of a value region a set writes: the value, then (with scrubbing) zeros to the
// 64-B boundary (hybrid) or to max_val (full) -- the chunk count write_value covers.
__device__ __forceinline__ uint32_t set_chunks(const Arena& a, uint32_t len, bool scrub, bool hybrid) {
  const uint32_t n16 = (len + 15) >> 4;
  if (!scrub) return n16;
  uint32_t end = hybrid ? ((len + 63u) & ~63u) : a.max_val;
  if (end > a.max_val) end = a.max_val;
  return (end >> 4) > n16 ? (end >> 4) : n16;
}

template <int MO = 0>
__device__ __forceinline__ void write_set(const Arena& a, const Claim& c, const uint8_t* val, uint32_t len,
                                          bool scrub, bool hybrid) {
  uint8_t* s = a.slot((size_t)c.idx);
  write_value<MO>(a, (size_t)c.idx, val, len, scrub, hybrid);
  if (c.fresh) {
    // fresh slot: metadata bytes 24..63 to defaults (type VOID), clear a stale vector
    st16<MO>(s + 32, make_uint4(0, 0, 0, 0));  // watcher_mask, ctime
    st16<MO>(s + 48, make_uint4(0, 0, 0, 0));  // atime, bloom
    ast8(s + kOffType, (uint8_t)SPL_SLOT_DEFAULT_TYPE);
    ast8(s + kOffUser, 0);
    if (a.stride == kSlotEmbedBytes) {
      uint4* ev = (uint4*)(s + kOffEmbed);
      for (uint32_t q = 0; q < kEmbedBytes / 16; ++q) st16<MO>(ev + q, make_uint4(0, 0, 0, 0));
      clear_vec16(a, (size_t)c.idx);
    }
  }
  ast32(s + kOffValLen, len);
}

// (A plain store of the held epoch + 1 instead of the atomic add measured neutral in round 6, KV-only
// 4.86-4.94 vs 4.92-4.93 G ops/s; a lane-batched claim of U ops, claim_many, was pruned in round 4.)
__device__ __forceinline__ void finish_set(const Arena& a, const Claim& c) { aadd64(epoch_ptr(a.slot((size_t)c.idx)), 1); }
// Single-op SET (insert or update) with its own release.
template <int MO = 0, int KW>
__device__ int32_t set_op(const Arena& a, const KeyT<KW>& k, const uint8_t* val, uint32_t len, long* out_idx) {
  if (len == 0 || len > a.max_val) return kMsgSize;
  bool hybrid;
  const bool scrub = scrub_flags(a, hybrid);
  const Claim c = claim_set(a, k, maint_begin(a));
  if (c.rc != kOk) return c.rc;
  write_set<MO>(a, c, val, len, scrub, hybrid);
  if constexpr (MO == 0) release();
  else if constexpr (MO == 1) drain();
  finish_set(a, c);
  *out_idx = c.idx;
  return kOk;
}

// GET: seqlock read into out (may be null: size query).
template <int MO = 0, int KW>
__device__ int32_t get_op(const Arena& a, const KeyT<KW>& k, uint8_t* out, uint32_t out_cap, uint32_t* out_len) {
  const uint64_t s0 = maint_begin(a);
  size_t idx = (size_t)(k.hash % a.slots);
  for (uint32_t i = 0; i < a.slots; ++i) {
    const uint8_t* s = a.slot(idx);
    const uint64_t sh = slot_hash(s);
    if (sh == k.hash) {
      const uint64_t e1 = MO == 0 ? ald64_acq(s + kOffEpoch) : ald64(s + kOffEpoch);
      if (key_eq(s, k)) {
        if (e1 & 1) return kAgain;
        const uint32_t len = ald32(s + kOffValLen);
        *out_len = len;
        if (out) {
          if (len > out_cap) return kMsgSize;
          const uint4* src = (const uint4*)a.value(idx);
          uint4* dst = (uint4*)out;
          const uint32_t n16 = (len + 15) >> 4;
          for (uint32_t c = 0; c < n16; ++c) dst[c] = ld16<MO>(src + c);
        }
        if constexpr (MO != 2) drain();
        const uint64_t e2 = slot_epoch(s);
        return (e2 == e1 && slot_hash(s) == k.hash) ? kOk : kAgain;
      }
    } else if (sh == 0 && slot_epoch(s) == 0) {
      break;
    }
    if (++idx == a.slots) idx = 0;
  }
  return maint_quiet(a, s0) ? kNoEnt : kAgain;
}

// One-round-trip probe for batched gets: hash, epoch, length and the key
// words of each probed slot are loaded together; returns the slot index with
// its epoch / length as observed, or -1 for a miss.  The caller validates the
// whole read afterwards (key words again with the data, epoch unchanged).
// s0: the maintenance seq read (and waited for) before this probe; a miss is -1 only when no pass
// overlapped the probe, else kMaintMiss.
template <int KW>
__device__ __forceinline__ long locate_peek(const Arena& a, const KeyT<KW>& k, uint64_t* e1, uint32_t* len,
                                            uint64_t s0) {
  size_t idx = (size_t)(k.hash % a.slots);
  for (uint32_t i = 0; i < a.slots; ++i) {
    const uint8_t* s = a.slot(idx);
    u32x4c_t he = ld16c(s + kOffHash), vl = ld16c(s + kOffValOff);
    KeyProbe<KW> kp;
    kp.issue(s, k);
    vm_wait(he, vl);
    kp.wait();
    const uint64_t sh = lo64(he), e = hi64(he);
    const uint32_t L = vl.y;  // val_len at offset 20
    const bool keq = kp.eq(k);
    if (sh == k.hash && keq) {
      *e1 = e;
      *len = L;
      return (long)idx;
    }
    if (sh == 0 && e == 0) break;
    if (++idx == a.slots) idx = 0;
  }
  return maint_quiet(a, s0) ? -1 : kMaintMiss;
}

// Copy n16 16-B chunks with 8 loads in flight per batch (see write_value).
__device__ __forceinline__ void copy_chunks(uint4* dst, const uint4* src, uint32_t n16, uint32_t src_chunks) {
  for (uint32_t b = 0; b < n16; b += 8) {
    uint4 t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) t[q] = src[min(b + (uint32_t)q, src_chunks - 1)];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (b + (uint32_t)q < n16) dst[b + q] = t[q];
  }
}

// Batched GET, phase helpers (see k_get_rounds): locate without the seqlock,
// then one acquire for all of a lane's ops, then copy, then validate.
// Returns the slot index holding k (possibly mid-write), or -1 for a miss.
template <int KW>
__device__ __forceinline__ long locate(const Arena& a, const KeyT<KW>& k) {
  const uint64_t s0 = maint_begin(a);
  size_t idx = (size_t)(k.hash % a.slots);
  for (uint32_t i = 0; i < a.slots; ++i) {
    const uint8_t* s = a.slot(idx);
    const uint64_t sh = slot_hash(s);
    if (sh == k.hash) {
      if (key_eq(s, k)) return (long)idx;
    } else if (sh == 0 && slot_epoch(s) == 0) {
      break;
    }
    if (++idx == a.slots) idx = 0;
  }
  return maint_quiet(a, s0) ? -1 : kMaintMiss;
}

// UNSET: returns the old length (>= 0) or a negative status.
template <int KW>
__device__ int32_t unset_op(const Arena& a, const KeyT<KW>& k, long* out_idx) {
  const long i = find(a, k);
  if (i < 0) return miss_rc(i);
  uint8_t* s = a.slot((size_t)i);
  const uint64_t e = slot_epoch(s);
  if ((e & 1) || !acas64(epoch_ptr(s), e, e + 1)) return kAgain;
  if (slot_hash(s) != k.hash || !key_eq(s, k)) { aadd64(epoch_ptr(s), 1); return kNoEnt; }
  const uint32_t old = ald32(s + kOffValLen);
  bool hybrid;
  const bool scrub = scrub_flags(a, hybrid);
  ast64(s + kOffHash, 0);
  uint4* key4 = (uint4*)(s + kOffKey);
  if (scrub) {
    uint4* v = (uint4*)a.value((size_t)i);
    for (uint32_t c = 0; c < a.max_val / 16; ++c) v[c] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int c = 0; c < 4; ++c) key4[c] = make_uint4(0, 0, 0, 0);
  } else {
    key4[0] = make_uint4(0, 0, 0, 0);
  }
  // bytes 16..63: val_off kept, val_len 0, type VOID, user 0, watcher/ctime/atime/bloom 0
  const uint32_t voff = ald32(s + kOffValOff);
  *(uint4*)(s + 16) = make_uint4(voff, 0, SPL_SLOT_DEFAULT_TYPE, 0);
  *(uint4*)(s + 32) = make_uint4(0, 0, 0, 0);
  *(uint4*)(s + 48) = make_uint4(0, 0, 0, 0);
  if (a.stride == kSlotEmbedBytes) {
    uint4* ev = (uint4*)(s + kOffEmbed);
    for (uint32_t c = 0; c < kEmbedBytes / 16; ++c) ev[c] = make_uint4(0, 0, 0, 0);
    clear_vec16(a, (size_t)i);
  }
  release();
  ast64(epoch_ptr(s), 2);  // reference contract: unset rewinds the epoch to 2
  *out_idx = i;
  return (int32_t)old;
}

// In-place u64 integer op under the seqlock.
template <int KW>
__device__ int32_t integer_op(const Arena& a, const KeyT<KW>& k, int op, uint64_t m, uint64_t* result, long* out_idx) {
  const long i = find(a, k);
  if (i < 0) return miss_rc(i);
  uint8_t* s = a.slot((size_t)i);
  if (!(ald8(s + kOffType) & SPL_SLOT_TYPE_BIGUINT)) return kProto;
  const uint64_t e = slot_epoch(s);
  if ((e & 1) || !acas64(epoch_ptr(s), e, e + 1)) return kAgain;
  uint8_t* v = a.value((size_t)i);
  // the slot is held (odd epoch): plain accesses, and byte-safe -- a value row starts at
  // i * max_val, which is 8-B aligned only when max_val is.  The previous holder may have run on
  // another CU / XCD: acquire before reading (no stale L1 line) and release before publishing (the
  // new value leaves this XCD's L2), else concurrent increments of one key lose updates
  // (tests/test_batch_api.py: 400 increments over 40 keys in one batch).
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  uint64_t x;
  __builtin_memcpy(&x, v, 8);
  switch (op) {
    case SPL_OP_AND: x &= m; break;
    case SPL_OP_OR: x |= m; break;
    case SPL_OP_XOR: x ^= m; break;
    case SPL_OP_NOT: x = ~x; break;
    case SPL_OP_INC: x += m; break;
    case SPL_OP_DEC: x -= m; break;
    default: break;
  }
  __builtin_memcpy(v, &x, 8);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  drain();
  aadd64(epoch_ptr(s), 1);
  if (result) *result = x;
  *out_idx = i;
  return kOk;
}

// APPEND under the slot seqlock (reference splinter.c:1062-1108): claim e -> e+1, bound check,
// copy the new bytes at the current tail, publish val_len, release, e+1.  The tail is not 16-B
// aligned in general, so the copy is bytewise (appends are small, streaming text).  `src` is a
// device pointer; the caller pulses / marks dirty on success.
template <int KW>
__device__ int32_t append_op(const Arena& a, const KeyT<KW>& k, const uint8_t* src, uint32_t len,
                             uint32_t* new_len, long* out_idx) {
  if (len == 0) return kInval;
  const long i = find(a, k);
  if (i < 0) return miss_rc(i);
  uint8_t* s = a.slot((size_t)i);
  const uint64_t e = slot_epoch(s);
  if ((e & 1) || !acas64(epoch_ptr(s), e, e + 1)) return kAgain;
  if (slot_hash(s) != k.hash || !key_eq(s, k)) { aadd64(epoch_ptr(s), 1); return kNoEnt; }
  const uint32_t cur = ald32(s + kOffValLen);
  if ((uint64_t)cur + len > a.max_val) { aadd64(epoch_ptr(s), 1); return kMsgSize; }
  uint8_t* v = a.value((size_t)i) + cur;
  for (uint32_t b = 0; b < len; ++b) v[b] = src[b];
  release();
  ast32(s + kOffValLen, cur + len);
  drain();
  aadd64(epoch_ptr(s), 1);
  *new_len = cur + len;
  *out_idx = i;
  return kOk;
}

// strtoull(s, 0, 0) of an ASCII value (at most 15 bytes, as the reference parses it):
// 0x / 0X prefix = hex, a leading 0 = octal, else decimal; stops at the first invalid digit.
__device__ __forceinline__ uint64_t parse_u64(const uint8_t* p, uint32_t n) {
  uint32_t i = 0;
  uint64_t base = 10, x = 0;
  if (n >= 2 && p[0] == '0' && (p[1] == 'x' || p[1] == 'X')) { base = 16; i = 2; }
  else if (n >= 1 && p[0] == '0') { base = 8; i = 1; }
  for (; i < n; ++i) {
    const uint8_t c = p[i];
    uint64_t d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
    else break;
    if (d >= base) break;
    x = x * base + d;
  }
  return x;
}

// set_named_type under the seqlock, with the BIGUINT promotion done in place on the device
// (reference splinter.c:637-680 parses a short ASCII value with strtoull, or takes its raw
// bytes, into a u64; its bump allocation from val_brk aliases slot 0's value, so the u64 is
// written into the slot's own value row instead -- docs/DIVERGENCES.md).
template <int KW>
__device__ int32_t named_type_op(const Arena& a, const KeyT<KW>& k, uint8_t mask, long* out_idx) {
  const long i = find(a, k);
  if (i < 0) return miss_rc(i);
  uint8_t* s = a.slot((size_t)i);
  const uint64_t e = slot_epoch(s);
  if ((e & 1) || !acas64(epoch_ptr(s), e, e + 1)) return kAgain;
  if (slot_hash(s) != k.hash || !key_eq(s, k)) { aadd64(epoch_ptr(s), 1); return kNoEnt; }
  const uint32_t cur = ald32(s + kOffValLen);
  if ((mask & SPL_SLOT_TYPE_BIGUINT) && cur < 8 && a.max_val >= 8) {
    uint8_t* v = a.value((size_t)i);
    uint8_t tmp[16];
    for (uint32_t b = 0; b < 16; ++b) tmp[b] = b < cur ? v[b] : 0;
    uint64_t x = 0;
    if (cur > 0 && tmp[0] >= '0' && tmp[0] <= '9') x = parse_u64(tmp, cur < 15 ? cur : 15);
    else for (uint32_t b = 0; b < cur; ++b) x |= (uint64_t)tmp[b] << (8 * b);
    __builtin_memcpy(v, &x, 8);
    release();
    ast32(s + kOffValLen, 8);
  }
  ast8(s + kOffType, mask);
  drain();
  aadd64(epoch_ptr(s), 1);
  *out_idx = i;
  return kOk;
}

// Keyed metadata ops (spl_arena_meta, the command ring):
// op: 0 set_label, 1 unset_label, 2 bump, 3 get_epoch, 4 watch_register,
//     5 watch_unregister, 6 pulse_keygroup, 7 set_as_system, 8 retrain,
//     9 set_named_type (arg = mask, BIGUINT promotion on the device), 10 set ctime,
//     11 set atime, 12 find (out = slot index)
// *mut: the op changed the slot (global epoch +1; dirty mask already marked here).
template <int KW>
__device__ int32_t meta_apply(const Arena& a, const KeyT<KW>& k, int op, uint64_t arg, uint64_t* out, bool* mut,
                              long idx);
template <int KW>
__device__ int32_t meta_op(const Arena& a, const KeyT<KW>& k, int op, uint64_t arg, uint64_t* out, bool* mut) {
  *mut = false;
  *out = 0;
  if (op == 9) {
    long idx = -1;
    const int32_t rc = named_type_op(a, k, (uint8_t)arg, &idx);
    if (rc == kOk) { *mut = true; mark_dirty(a, (size_t)idx); }
    return rc;
  }
  // ops that change a slot WITHOUT claiming its seqlock (labels, watchers, system / times, the
  // reference's unconditional retrain stores) could land on an entry a maintenance pass is copying
  // and be lost with its old slot: they run only outside a pass, and report EAGAIN when a pass
  // overlapped them (each is idempotent: the retry re-applies it where the entry now lives)
  const bool unlocked = op == 0 || op == 1 || op == 4 || op == 5 || op == 7 || op == 8 || op == 10 || op == 11;
  const uint64_t s0 = maint_begin(a);
  if (unlocked && (s0 & 1)) return kAgain;
  const long idx = find(a, k);
  if (idx < 0) return miss_rc(idx);
  const int32_t rc = meta_apply(a, k, op, arg, out, mut, idx);
  if (unlocked && rc == kOk && !maint_quiet(a, s0)) return kAgain;
  return rc;
}

template <int KW>
__device__ int32_t meta_apply(const Arena& a, const KeyT<KW>& k, int op, uint64_t arg, uint64_t* out, bool* mut,
                              long idx) {
  (void)k;
  uint8_t* s = a.slot((size_t)idx);
  switch (op) {
    case 0: aor64((uint64_t*)(s + kOffBloom), arg); *mut = true; mark_dirty(a, idx); return kOk;
    case 1: aand64((uint64_t*)(s + kOffBloom), ~arg); *mut = true; mark_dirty(a, idx); return kOk;
    case 2: {
      const uint64_t e = slot_epoch(s);
      if ((e & 1) || !acas64(epoch_ptr(s), e, e + 1)) return kAgain;
      pulse(a, s);
      drain();
      aadd64(epoch_ptr(s), 1);
      return kOk;
    }
    case 3: *out = slot_epoch(s); return kOk;
    case 4: aor64((uint64_t*)(s + kOffWatch), 1ull << (arg & 63)); return kOk;
    case 5: aand64((uint64_t*)(s + kOffWatch), ~(1ull << (arg & 63))); return kOk;
    case 6: pulse(a, s); return kOk;
    case 7:
      ast8(s + kOffType, (uint8_t)SPL_SLOT_TYPE_BINARY);
      ast32((uint32_t*)(s + kOffValLen), a.max_val);
      return kOk;
    case 8:
      ast64(epoch_ptr(s), 3);
      drain();
      if (a.stride == kSlotEmbedBytes) {
        for (uint32_t c = 0; c < kEmbedBytes / 16; ++c) ((uint4*)(s + kOffEmbed))[c] = make_uint4(0, 0, 0, 0);
        clear_vec16(a, (size_t)idx);
      }
      release();
      ast64(epoch_ptr(s), 4);
      *mut = true;
      pulse(a, s);
      mark_dirty(a, idx);
      return kOk;
    case 10: ast64((uint64_t*)(s + kOffCtime), arg); return kOk;
    case 11: ast64((uint64_t*)(s + kOffAtime), arg); return kOk;
    case 12: *out = (uint64_t)idx; return kOk;
    default: return kInval;
  }
}

}  // namespace dev
}  // namespace spl
