// cmd_ring.hip — the per-call command ring of an HBM store (protocol: cmd_ring.hpp).
//
// Device side: k_ring_worker, ONE wave; lane i serves ring entry i.  Every word the host wrote is
// read with system-scope loads (global_load ... sc0 sc1: no L1/L2 line of the pinned host page can
// be stale across a reuse of the entry) and every word the host reads is written with
// system-scope stores, drained before the DONE doorbell store, so neither side needs a fence over
// the whole cache.  The arena itself is touched only through the seqlock ops of arena_dev.hpp,
// exactly as the batch kernels touch it (set_op / get_op / unset_op / append_op / integer_op /
// meta_op), so single calls and batches interleave under the same protocol.
#include <hip/hip_runtime.h>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>
#include <sched.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <set>
#include <vector>
#include <shared_mutex>

#include "arena_dev.hpp"
#include "cmd_ring.hpp"
#include "store_host.hpp"

namespace spl {
namespace {
// Quiesce gate (RingQuiesce, cmd_ring.hpp).  Per-call ops hold it shared for their whole call;
// store set-up holds it exclusive and first stops every live worker of the process: HIP calls made
// while setting up a store (VMM maps, host registration, device memsets) may wait for the device's
// queues, and a resident worker kept alive by another thread's traffic never drains.
std::shared_mutex g_gate;
std::mutex g_reg_mu;
std::set<CmdRing*> g_rings;
thread_local bool t_exclusive = false;
std::atomic<int> g_hold{0};  // spl_ring_hold: no worker of this process runs while > 0
}  // namespace

// A process's resident ring workers cost a heavy GPU job of the same process dearly while they are
// resident (profiles/r4x: the encoder +84 % beside an idle resident worker: the queue scheduler
// time-slices the worker's queue against the job's).  A process about to run such a job can hold
// its rings: every worker stops, none relaunches until the hold is released, and per-call ops --
// its own and its clients' -- wait meanwhile (they are served once the hold ends).
void ring_hold(bool on) {
  if (on) {
    if (g_hold.fetch_add(1) == 0) {
      std::lock_guard<std::mutex> lk(g_reg_mu);
      for (CmdRing* r : g_rings) r->stop();
    }
    return;
  }
  if (g_hold.fetch_sub(1) != 1) return;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (CmdRing* r : g_rings) r->resume();
}

RingQuiesce::RingQuiesce() {
  if (t_exclusive) return;
  g_gate.lock();
  t_exclusive = held_ = true;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (CmdRing* r : g_rings) r->stop();
}
RingQuiesce::~RingQuiesce() {
  if (!held_) return;
  t_exclusive = false;
  g_gate.unlock();
}
}  // namespace spl

namespace spl {

namespace {

using namespace spl::dev;

typedef unsigned int u32x4s_t __attribute__((ext_vector_type(4)));

// 16-B system-scope load / store (hipcc does not track inline-asm memory ops: ld16s results are
// valid after sys_wait(); st16s callers drain() before anything that publishes the bytes).
__device__ __forceinline__ u32x4s_t ld16s(const void* p) {
  u32x4s_t r;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ void sys_wait(u32x4s_t& a) { asm volatile("s_waitcnt vmcnt(0)" : "+v"(a)::"memory"); }
__device__ __forceinline__ void st16s(void* p, u32x4s_t v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t ld32s(const void* p) {
  return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld64s(const void* p) {
  return __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st32s(void* p, uint32_t v) {
  __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st64s(void* p, uint64_t v) {
  __hip_atomic_store((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// doorbell reads kept in flight by the worker's idle loop (inline asm: hipcc does not count them,
// each is retired by an explicit wait that ties its register)
constexpr int kPollGap = 16;  // s_sleep units (64 clocks) between the first reads: ~0.4 us
__device__ __forceinline__ uint32_t ld32s_issue(const void* p) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off sc0 sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ void wait_oldest_of4(uint32_t& r) { asm volatile("s_waitcnt vmcnt(3)" : "+v"(r)::"memory"); }
__device__ __forceinline__ void drain_polls(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
}

// host payload -> device scratch, chunks [from, n16) (8 loads in flight)
__device__ void pull(uint4* dst, const uint8_t* src, uint32_t from, uint32_t n16) {
  for (uint32_t b = from; b < n16; b += 8) {
    u32x4s_t t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) t[q] = ld16s(src + 16 * (size_t)min(b + (uint32_t)q, n16 - 1));
#pragma unroll
    for (int q = 0; q < 8; ++q) sys_wait(t[q]);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (b + (uint32_t)q < n16) dst[b + q] = make_uint4(t[q].x, t[q].y, t[q].z, t[q].w);
  }
}

// arena value row -> host payload with agent-coherent loads (sc1: never a stale L1 line, so a get
// needs no acquire fence), 8 in flight, system-scope stores
__device__ void push_c(uint8_t* dst, const uint4* src, uint32_t n16) {
  for (uint32_t b = 0; b < n16; b += 8) {
    u32x4c_t t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) t[q] = ld16c(src + min(b + (uint32_t)q, n16 - 1));
#pragma unroll
    for (int q = 0; q < 8; ++q) vm_wait(t[q]);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (b + (uint32_t)q < n16) st16s(dst + 16 * (size_t)(b + q), u32x4s_t{t[q].x, t[q].y, t[q].z, t[q].w});
  }
}

// device bytes -> host payload, n16 chunks: 8 loads in flight, system-scope stores
__device__ void push(uint8_t* dst, const uint4* src, uint32_t n16) {
  for (uint32_t b = 0; b < n16; b += 8) {
    uint4 t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) t[q] = src[min(b + (uint32_t)q, n16 - 1)];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (b + (uint32_t)q < n16) st16s(dst + 16 * (size_t)(b + q), u32x4s_t{t[q].x, t[q].y, t[q].z, t[q].w});
  }
}

// The event-bus wakeup of a per-call mutation is raised by the calling host thread once the call
// returns (HbmStore::notify_host: the eventfd directly in the owner, the shared notify word
// elsewhere), so the worker does not raise the device notify too: that second, proxied signal
// would land up to a proxy period later and wake a waiter that has already drained the first.
__device__ __forceinline__ void count_mutation(const Arena& a, long idx) {
  aadd64(&a.hdr()->epoch, 1);
  if (idx >= 0) mark_dirty(a, (size_t)idx);
}

#ifdef SPL_RING_STAMPS
__device__ uint64_t g_ts[kRingEntries][5];  // this call's op checkpoints (serving lane only)
// per-entry sums (device memory, read back by ~CmdRing): doorbell seen -> record loaded -> op done
// -> completion drained, call count; set / get op segments; shader-clock and wall ticks
__device__ uint64_t g_stamp[kRingEntries][4];
__device__ uint64_t g_opstamp[kRingEntries][10];
__device__ uint64_t g_clk[kRingEntries][2];
__device__ int g_ent[64 * kRingGroups];     // entry of the serving lane
#define RING_TS(i) (g_ts[g_ent[blockIdx.x * 64 + threadIdx.x]][i] = wall_clock64())
#else
#define RING_TS(i) ((void)0)
#endif

constexpr uint32_t kSpec = 16;  // payload chunks fetched speculatively with the record (256 B)

// A value of at most kSpec chunks arrives in registers with the record (serve's speculative
// payload loads): it is written from there, with no staging row in device memory.
struct Spec {
  u32x4s_t c[kSpec];
};

// SET for one lane: claim, payload with write-through (sc1) stores, drain, publish -- no L2
// write-back fence on this latency path (MO 3 of arena_dev.hpp; readers are unchanged).  A value
// row that is not a multiple of 16 B ends in bytewise plain stores: those take the release path.
// reg: the value is in sp (len <= kSpec * 16, max_val a multiple of 16); else in the staged row.
// ms: the arena's maintenance seq, loaded with the request record (waited before the probe).
__device__ __forceinline__ int32_t ring_set(const Arena& a, const Key& k, const uint8_t* pay, const Spec& sp,
                                            bool reg, uint32_t len, bool scrub, bool hybrid, uint64_t ms) {
  if (len == 0 || len > a.max_val) return kMsgSize;
  RING_TS(1);
  const Claim c = claim_set(a, k, ms);
  RING_TS(2);
  if (c.rc != kOk) return c.rc;
  if (reg) {
    uint4* dst = (uint4*)a.value((size_t)c.idx);
    const uint32_t n16 = (len + 15) >> 4;
#pragma unroll
    for (uint32_t q = 0; q < kSpec; ++q) {
      if (q < n16) {
        uint4 t = make_uint4(sp.c[q].x, sp.c[q].y, sp.c[q].z, sp.c[q].w);
        if (q == n16 - 1 && (len & 15)) {
          const int r = (int)(len & 15);
          t.x &= keep_mask(r); t.y &= keep_mask(r - 4); t.z &= keep_mask(r - 8); t.w &= keep_mask(r - 12);
        }
        st16_wt(dst + q, t);
      }
    }
    if (scrub) {  // the mop of write_value: zeros to the 64-B boundary (hybrid) or to max_val
      uint32_t end = hybrid ? ((len + 63u) & ~63u) : a.max_val;
      if (end > a.max_val) end = a.max_val;
      for (uint32_t done = n16 << 4; done + 16 <= end; done += 16) st16_wt(dst + (done >> 4), make_uint4(0, 0, 0, 0));
    }
    write_meta<3>(a, c, len);
    drain();
  } else if (a.max_val & 15) {
    write_set<0>(a, c, pay, len, scrub, hybrid);
    release();
  } else {
    write_set<3>(a, c, pay, len, scrub, hybrid);
    drain();
  }
  RING_TS(3);
  finish_set(a, c);
  pulse_masks(a, c.wm, c.bl);
  count_mutation(a, c.idx);
  RING_TS(4);
  return kOk;
}

// GET for one lane straight into the host payload: one-round-trip probe, acquire, copy
// (arena -> host, system-scope stores), then the seqlock re-check; on EAGAIN the host ignores
// the bytes it may have received.
__device__ __forceinline__ int32_t ring_get(const Arena& a, const Key& k, uint8_t* hp, uint32_t cap, uint32_t* out_len,
                                            uint64_t ms) {
  uint64_t e1 = 0;
  uint32_t L = 0;
  RING_TS(1);
  const long idx = locate_peek(a, k, &e1, &L, ms);
  RING_TS(2);
  if (idx < 0) return miss_rc(idx);
  if ((e1 & 1) || L == kInsertMark) return kAgain;
  const uint8_t* s = a.slot((size_t)idx);
  // no acquire fence: the value row is read with agent-coherent loads (push_c), as the batched
  // acquire-free get (arena_kernels.hip k_get_carry FAST).  An agent-scope acquire costs a cache
  // invalidate per call, and beside a running encoder it is the encoder's cache that goes
  RING_TS(3);
  *out_len = L;
  if (L > cap) return kMsgSize;
#ifdef SPL_RING_GET_REGS
  if (L <= kSpec * 16) {
    // (measured variant: profiles/r2_hostapi_ring_v3.md -- 1 µs lower single-thread get latency,
    // 20 % fewer ops/s at 16-24 host threads than the copy below, so not the default)
    // value into registers, THEN the (hash, epoch) re-check in one 16-B load, then the host
    // stores: the re-check waits on no host-bound store and the value costs one round trip
    const uint32_t n16 = (L + 15) >> 4;
    const uint4* src = (const uint4*)a.value((size_t)idx);
    u32x4c_t v[kSpec];
#pragma unroll
    for (uint32_t q = 0; q < kSpec; ++q) v[q] = q < n16 ? ld16c(src + q) : u32x4c_t{0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t q = 0; q < kSpec; ++q) vm_wait(v[q]);
    u32x4c_t re = ld16c(s + kOffHash);
    vm_wait(re);
    const bool ok = lo64(re) == k.hash && hi64(re) == e1;
    RING_TS(4);
    if (!ok) return kAgain;
#pragma unroll
    for (uint32_t q = 0; q < kSpec; ++q)
      if (q < n16) st16s(hp + 16 * q, u32x4s_t{v[q].x, v[q].y, v[q].z, v[q].w});
    return kOk;
  }
#endif
  // the value loads complete before their bytes are stored (data dependency) and the epoch
  // re-check is issued after those stores, so the seqlock order holds without draining the
  // host-bound stores here: the one drain before the DONE doorbell covers them
  if (L) push_c(hp, (const uint4*)a.value((size_t)idx), (L + 15) >> 4);
  const bool ok = slot_epoch(s) == e1 && slot_hash(s) == k.hash;
  RING_TS(4);
  return ok ? kOk : kAgain;
}

__device__ int32_t serve_plain(const Arena& a, const Key& k, uint32_t op, uint32_t sub, uint32_t len, uint32_t cap,
                               uint64_t arg, uint8_t* hp, uint8_t* pay, uint32_t* out_len, uint64_t* result);

// one op of one lane; scratch = this entry's device staging row (payload)
// c / hin: the request record and input payload (host memory, or device memory the host writes
// through the BAR in the VRAM mode); hp: the output payload (host memory)
__device__ int32_t serve(const spl_arena_t& aa, const RingCmd* c, const uint8_t* hin, uint8_t* hp, uint8_t* pay,
                         uint32_t* out_len, uint64_t* result, uint64_t* t_loaded) {
  // the two header words every op needs (event-bus owner, mop flags) are loaded first, so their
  // device round trip overlaps the record's host round trip below
  const splinter_header* H = (const splinter_header*)aa.base;
  const uint32_t owner = __hip_atomic_load(&H->event_bus.owner_pid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint8_t cflags = ald8(&H->core_flags);
  // the maintenance seq (arena_dev.hpp, online maintenance) rides along: waited with the record,
  // so it is read before any probe load of the op
  const uint8_t* mp = (aa.flags & SPL_ARENA_SIDE)
                          ? (const uint8_t*)aa.base + side_offset(aa.slots, aa.stride, aa.max_val) + kSideMaintOff
                          : (const uint8_t*)aa.base;
  u32x2c_t mw = ld8c(mp);
  // ONE round of system-scope loads: record header (32 B + key length), key (64 B) and the
  // first kSpec payload chunks (speculative: the length is in the header)
  u32x4s_t h0 = ld16s(c), h1 = ld16s((const uint8_t*)c + 16), h3 = ld16s((const uint8_t*)c + 48);
  u32x4s_t kk[4];
  Spec sp;
#pragma unroll
  for (int q = 0; q < 4; ++q) kk[q] = ld16s(c->key + 16 * q);
#pragma unroll
  for (uint32_t q = 0; q < kSpec; ++q) sp.c[q] = ld16s(hin + 16 * q);
  sys_wait(h0);
  sys_wait(h1);
  sys_wait(h3);
#pragma unroll
  for (int q = 0; q < 4; ++q) sys_wait(kk[q]);
#pragma unroll
  for (uint32_t q = 0; q < kSpec; ++q) sys_wait(sp.c[q]);
  vm_wait1(mw);
  const uint64_t ms = u64of(mw);
  const uint32_t op = h0.x, sub = h0.y, len = h0.z, cap = h0.w;
#ifdef SPL_RING_STAMPS
  *t_loaded = wall_clock64();
  g_ts[g_ent[blockIdx.x * 64 + threadIdx.x]][0] = *t_loaded;
#else
  (void)t_loaded;
#endif
  const uint64_t arg = ((uint64_t)h1.y << 32) | h1.x;
  Arena a;
  a.base = (uint8_t*)aa.base;
  a.slots = aa.slots;
  a.max_val = aa.max_val;
  a.stride = aa.stride;
  a.notify = aa.notify;
  a.flags = aa.flags | (owner != 0 ? 1u : 0u);  // from_api(), with the owner word loaded above
  const bool scrub = (cflags & SPL_SYS_AUTO_SCRUB) != 0, hybrid = (cflags & SPL_SYS_HYBRID_SCRUB) != 0;
  const bool has_in = op == kRingSet || op == kRingAppend || op == kRingEmbedSet || op == kRingWrite;
#ifdef SPL_RING_SET_STAGED
  const bool reg = false;
#else
  const bool reg = op == kRingSet && len <= kSpec * 16 && (a.max_val & 15) == 0;
#endif
  if (has_in && !reg) {
    const uint32_t n16 = (len + 15) >> 4;
#pragma unroll
    for (uint32_t q = 0; q < kSpec; ++q)
      if (q < n16) ((uint4*)pay)[q] = make_uint4(sp.c[q].x, sp.c[q].y, sp.c[q].z, sp.c[q].w);
    if (n16 > kSpec) pull((uint4*)pay, hin, kSpec, n16);
    drain();  // the staged payload is in place before any op reads it
  }
  // the key is canonical with its hash computed by the host (KeyRef)
  Key k;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    k.w[4 * q] = kk[q].x; k.w[4 * q + 1] = kk[q].y; k.w[4 * q + 2] = kk[q].z; k.w[4 * q + 3] = kk[q].w;
  }
  k.len = h3.x < 63u ? h3.x : 63u;
  k.hash = ((uint64_t)h1.w << 32) | h1.z;
  *out_len = 0;
  *result = 0;
  // set (write-through stores + drain) and get (acquire load of the epoch) carry their own
  // cross-XCD ordering (the same write-through discipline as the batched kernels, arena_kernels.hip
  // k_get_carry FAST); every other op reads and writes the slot with plain accesses: plain loads may
  // hit lines this CU's L1 holds from before another XCD's write (acquire first: L1 invalidate), and
  // plain stores leave dirty lines in this XCD's L2 that a reader on another XCD would not see
  // (release after: L2 write-back), both at agent scope
  if (op == kRingSet) return ring_set(a, k, pay, sp, reg, len, scrub, hybrid, ms);
  if (op == kRingGet) return ring_get(a, k, hp, cap, out_len, ms);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int32_t rc = serve_plain(a, k, op, sub, len, cap, arg, hp, pay, out_len, result);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  return rc;
}

__device__ int32_t serve_plain(const Arena& a, const Key& k, uint32_t op, uint32_t sub, uint32_t len, uint32_t cap,
                               uint64_t arg, uint8_t* hp, uint8_t* pay, uint32_t* out_len, uint64_t* result) {
  long idx = -1;
  switch (op) {
    case kRingUnset:
      return unset_op(a, k, &idx);
    case kRingAppend: {
      uint32_t nl = 0;
      const int32_t rc = append_op(a, k, pay, len, &nl, &idx);
      if (rc == kOk) {
        *result = nl;
        pulse(a, a.slot((size_t)idx));
        count_mutation(a, idx);
      }
      return rc;
    }
    case kRingIntop: {
      uint64_t r = 0;
      const int32_t rc = integer_op(a, k, (int)sub, arg, &r, &idx);
      if (rc == kOk) {
        *result = r;
        count_mutation(a, idx);
      }
      return rc;
    }
    case kRingMeta: {
      bool mut = false;
      uint64_t o = 0;
      const int32_t rc = meta_op(a, k, (int)sub, arg, &o, &mut);
      *result = o;
      if (mut) count_mutation(a, -1);
      return rc;
    }
    case kRingEmbedSet: {
      if (a.stride != kSlotEmbedBytes) return kInval;
      idx = find(a, k);
      if (idx < 0) return miss_rc(idx);
      uint8_t* s = a.slot((size_t)idx);
      const uint64_t e = slot_epoch(s);
      if ((e & 1) || !acas64(epoch_ptr(s), e, e + 1)) return kAgain;
      if (slot_hash(s) != k.hash || !key_eq(s, k)) { aadd64(epoch_ptr(s), 1); return kNoEnt; }
      uint4* dst = (uint4*)(s + kOffEmbed);
      for (uint32_t q = 0; q < kEmbedBytes / 16; ++q) st16_wt(dst + q, ((const uint4*)pay)[q]);
      write_vec16_one(a, (size_t)idx, (const float*)pay);
      drain();
      aadd64(epoch_ptr(s), 1);
      count_mutation(a, idx);
      return kOk;
    }
    case kRingEmbedGet: {
      if (a.stride != kSlotEmbedBytes) return kInval;
      idx = find(a, k);
      if (idx < 0) return miss_rc(idx);
      const uint8_t* s = a.slot((size_t)idx);
      const uint64_t e1 = ald64_acq(s + kOffEpoch);
      if (e1 & 1) return kAgain;
      push(hp, (const uint4*)(s + kOffEmbed), kEmbedBytes / 16);
      drain();
      if (slot_epoch(s) != e1) return kAgain;
      *out_len = kEmbedBytes;
      return kOk;
    }
    case kRingSnapshot: {
      idx = find(a, k);
      if (idx < 0) return miss_rc(idx);
      const uint8_t* s = a.slot((size_t)idx);
      for (int q = 0; q < 16; ++q) st64s(hp + 8 * q, ald64(s + 8 * q));
      *out_len = 128;
      *result = (uint64_t)idx;
      return kOk;
    }
    case kRingRead: {  // header / arena bytes; 8-B sc1 loads when aligned, else bytewise
      if (len > cap) return kMsgSize;
      if (((arg | len) & 7) == 0) {
        for (uint32_t q = 0; q < len / 8; ++q) st64s(hp + 8 * q, ald64(a.base + arg + 8 * q));
      } else {
        for (uint32_t q = 0; q < len; ++q) pay[q] = ald8(a.base + arg + q);
        drain();
        push(hp, (const uint4*)pay, (len + 15) >> 4);
      }
      *out_len = len;
      return kOk;
    }
    case kRingWrite: {  // sub 0: store the bytes; sub 1 / 2: atomic OR / AND of ONE byte (config
                        // flags); sub 3: atomic add of a u64 (signal counters)
      if (sub == 3) {
        if (len != 8 || (arg & 7)) return kInval;
        uint64_t d;
        __builtin_memcpy(&d, pay, 8);
        aadd64(a.base + arg, d);
        return kOk;
      }
      if (sub == 1 || sub == 2) {
        if (len != 1) return kInval;
        const uintptr_t wa = (uintptr_t)(a.base + arg);
        uint32_t* w = (uint32_t*)(wa & ~(uintptr_t)3);
        const uint32_t sh = 8u * (uint32_t)(wa & 3);
        const uint32_t m = pay[0];
        if (sub == 1) __hip_atomic_fetch_or(w, m << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_and(w, ~((~m & 0xffu) << sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return kOk;
      }
      if (((arg | len) & 7) == 0) {
        for (uint32_t q = 0; q < len / 8; ++q) {
          uint64_t v;
          __builtin_memcpy(&v, pay + 8 * q, 8);
          ast64(a.base + arg + 8 * q, v);
        }
      } else {
        for (uint32_t q = 0; q < len; ++q) ast8(a.base + arg + q, pay[q]);
      }
      drain();
      return kOk;
    }
    default:
      return kInval;
  }
}

// Workgroup g serves entries g*per + lane (lanes 0..per-1, per = kRingEntries / groups).
// ctrl (device): [0] u64 wall clock of the last served call (any group), [8] u32 dying,
// [12] u32 live waves (set to gridDim.x by the launcher).
// VR (VRAM requests): records, input payloads and doorbells live in device memory that the host
// writes through the PCIe BAR (posted writes), so the worker polls and loads them locally instead
// of over PCIe; a doorbell is the entry's call sequence number (host-written only, never reset: a
// call is new when it differs from the lane's last served number, kept in `served` across
// relaunches), and the completion -- status words, output payload, DONE = the same number -- goes
// to host memory as in the host mode.
template <bool VR>
__global__ __launch_bounds__(64) void k_ring_worker(spl_arena_t aa, RingCmd* cmds, RingCmd* hcmds, RingShared* sh,
                                                    const uint32_t* vdoor, const uint8_t* payload_in,
                                                    uint8_t* payload, uint32_t pstride, uint8_t* scratch,
                                                    uint8_t* ctrl, uint32_t* served, RingDone* vdone,
                                                    uint64_t idle_ticks, int per) {
  const int lane = threadIdx.x, g = blockIdx.x;
  const bool mine = lane < per;
  const int e = g * per + (mine ? lane : 0);
#ifdef SPL_RING_STAMPS
  g_ent[g * 64 + lane] = e;
#endif
  uint64_t last = wall_clock64();
  uint32_t idle = 0, busy_rounds = 0;
  const uint32_t* door = VR ? &vdoor[e] : &sh->state[e];
  uint32_t seen = VR && mine ? served[e] : 0u, bell = 0u;
  for (;;) {
#ifndef SPL_RING_POLL4
    bool ready;
    if constexpr (VR) {
      bell = mine ? ld32s(door) : 0u;
      ready = mine && bell != seen;
    } else {
      ready = mine && ld32s(door) == kRingReady;
    }
#else
    // (measured variant, slower: profiles/r2_hostapi_ring_v3.md) 4 doorbell reads in flight,
    // issued ~1/4 of a host round trip apart, so a doorbell is seen one round trip + a fraction
    // after the host rings it instead of 1.5 round trips on average -- but the reads still in
    // flight must land before the op starts, which costs more than the earlier detection saves.
    // vmcnt retires loads in issue order, so vmcnt(3) waits for exactly the oldest read.
    uint32_t p0 = ld32s_issue(door);
    __builtin_amdgcn_s_sleep(kPollGap);
    uint32_t p1 = ld32s_issue(door);
    __builtin_amdgcn_s_sleep(kPollGap);
    uint32_t p2 = ld32s_issue(door);
    __builtin_amdgcn_s_sleep(kPollGap);
    uint32_t p3 = ld32s_issue(door);
    bool ready = false;
    for (int round = 0; round < 8; ++round) {
      wait_oldest_of4(p0);
      if (__ballot(mine && p0 == kRingReady)) { ready = mine && p0 == kRingReady; break; }
      p0 = ld32s_issue(door);
      wait_oldest_of4(p1);
      if (__ballot(mine && p1 == kRingReady)) { ready = mine && p1 == kRingReady; break; }
      p1 = ld32s_issue(door);
      wait_oldest_of4(p2);
      if (__ballot(mine && p2 == kRingReady)) { ready = mine && p2 == kRingReady; break; }
      p2 = ld32s_issue(door);
      wait_oldest_of4(p3);
      if (__ballot(mine && p3 == kRingReady)) { ready = mine && p3 == kRingReady; break; }
      p3 = ld32s_issue(door);
    }
    drain_polls(p0, p1, p2, p3);  // the reads still in flight land before anything else
#endif
    if (__ballot(ready) == 0) {  // wave-uniform
      // the stop flag, the shared activity clock and the idle timeout are checked every 32nd
      // poll (every pipelined round of polls) only
#ifndef SPL_RING_POLL4
      if ((++idle & 31) != 0) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
#endif
      if ((ld32s(&sh->stop) | ld32s(&sh->hold)) != 0) break;
      u32x4c_t cl = ld16c(ctrl);
      vm_wait(cl);
      if (cl.z != 0) break;  // another group timed out: leave together
      const uint64_t now = wall_clock64(), ga = lo64(cl);
      if (now - (ga > last ? ga : last) > idle_ticks) {
        if (lane == 0) ast32(ctrl + 8, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    // a wave that never goes idle (every round has a call) still sees stop / dying every 64th round
    if ((++busy_rounds & 63) == 0) {
      if ((ld32s(&sh->stop) | ld32s(&sh->hold)) != 0) break;
      u32x4c_t cl = ld16c(ctrl);
      vm_wait(cl);
      if (cl.z != 0) break;
    }
    last = wall_clock64();
#ifdef SPL_RING_STAMPS
    const uint64_t mt0 = __builtin_amdgcn_s_memtime();
#endif
    idle = 0;
    if (lane == 0) ast64(ctrl, last);
    if (ready) {
      RingCmd* c = cmds + e;
      uint32_t out_len = 0;
      uint64_t result = 0, t_loaded = 0;
      const int32_t st = serve(aa, c, (VR ? payload_in : payload) + (size_t)e * pstride, payload + (size_t)e * pstride,
                               scratch + (size_t)e * pstride, &out_len, &result, &t_loaded);
#ifdef SPL_RING_STAMPS
      const uint64_t t_op = wall_clock64();
#endif
      // status, out_len and result share one 16-B chunk of the record: one system-scope store,
      // one drain (it also covers a get's payload stores) before the DONE doorbell
      if constexpr (VR) {
        // out_len only for ops that returned bytes (the host zeroed it); the drain orders the
        // payload and the op's own writes before the completion chunk, which is ONE store
        if (out_len) st32s(&hcmds[e].out_len, out_len);
        drain();
      } else {
        st16s(&c->status, u32x4s_t{(uint32_t)st, out_len, (uint32_t)result, (uint32_t)(result >> 32)});
        drain();
      }
#ifdef SPL_RING_STAMPS
      const uint64_t t_done = wall_clock64();
      const uint64_t mt1 = __builtin_amdgcn_s_memtime();
      const uint32_t sop = ld32s(&c->op);
#endif
      if constexpr (VR) {
        seen = bell;
        served[e] = bell;  // read by the next launch only (kernel boundary)
        st16s(&vdone[e], u32x4s_t{bell, (uint32_t)st, (uint32_t)result, (uint32_t)(result >> 32)});
      } else {
        st32s(&sh->state[e], kRingDone);
      }
#ifdef SPL_RING_STAMPS
      // accumulated AFTER the completion, in device memory (plain loads / stores: one lane owns an
      // entry at a time), so the stamps do not lengthen the call they measure; ~CmdRing reads them
      g_clk[e][0] += mt1 - mt0;
      g_clk[e][1] += t_done - last;
      g_stamp[e][0] += t_loaded - last;
      g_stamp[e][1] += t_op - t_loaded;
      g_stamp[e][2] += t_done - t_op;
      g_stamp[e][3] += 1;
      if (st == 0 && (sop == kRingSet || sop == kRingGet)) {
        uint64_t* q = g_opstamp[e] + (sop == kRingSet ? 0 : 5);
        for (int i = 0; i < 4; ++i) q[i] += g_ts[e][i + 1] - g_ts[e][i];
        q[4] += 1;
      }
#endif
    }
  }
  drain();
  if (lane == 0 &&
      __hip_atomic_fetch_add((uint32_t*)(ctrl + 12), 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u)
    st32s(&sh->alive, 0u);  // the last wave out
}

inline int env_int(const char* n, int d) {
  const char* e = getenv(n);
  return e ? atoi(e) : d;
}

// CPUs this process may actually run on at once: its affinity mask, capped by a cgroup-v2 CPU
// quota (cpu.max "quota period"; the GPU boxes grant a share of the machine this way, so the
// affinity mask alone overstates it).  SPLINTER_RING_CPUS overrides.
int effective_cpus() {
  if (const char* e = getenv("SPLINTER_RING_CPUS")) return atoi(e) > 0 ? atoi(e) : 1;
  cpu_set_t set;
  int n = sched_getaffinity(0, sizeof set, &set) == 0 ? CPU_COUNT(&set) : 0;
  if (n <= 0) n = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long period = 0;
    if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
      const long quota = atol(q);
      const int cap = (int)((quota + period - 1) / period);
      if (cap > 0 && cap < n) n = cap;
    }
    fclose(f);
  }
  return n > 0 ? n : 1;
}

}  // namespace

void CmdRing::read_env() {
  pid_ = (int32_t)getpid();
  spread_ = env_int("SPLINTER_RING_SPREAD", 1) != 0;
  yield_after_us_ = (uint64_t)env_int("SPLINTER_RING_SPIN_US", 20);
  cpus_ = effective_cpus();
  sleep_ns_ = env_int("SPLINTER_RING_SLEEP_NS", 5000);  // 32 threads: 1.73 vs 1.41 M ops/s at 2000 (profiles/r3_hostapi_vram_single_store.jsonl)
  // oversubscribed waiters sleep at once, first for ~6 us (a good part of a 32-thread call's ~15 us):
  // 32 threads 1.60 -> 1.85 M ops/s with 8 us (profiles/r3_hostapi_oversub_wait_ab.jsonl), 1.84 -> 1.99 M
  // for 8 -> 6 us (means of 3 alternating rounds, profiles/r3_hostapi_sweep_s2.jsonl)
  first_sleep_ns_ = env_int("SPLINTER_RING_FIRST_SLEEP_NS", 6000);
  oversub_spin_us_ = (uint64_t)env_int("SPLINTER_RING_OVERSUB_SPIN_US", 0);
  adaptive_ = env_int("SPLINTER_RING_ADAPTIVE_SLEEP", 1) != 0;
  // SPLINTER_RING_GROUPS: worker waves (4..32, a power of two; entries per wave = 256 / groups: a
  // wave's 64 lanes serve at most 64 entries, so fewer than 4 waves would leave entries unserved and
  // their calls would time out).  Each resident worker wave (233 VGPRs) keeps the encoder's
  // 2-wave-per-SIMD GEMM workgroups off its CU
  int g = env_int("SPLINTER_RING_GROUPS", kDefaultRingGroups);
  int p2 = kRingMinGroups;
  while (p2 * 2 <= g && p2 < kRingGroups) p2 *= 2;
  groups_ = p2;
  static_assert(kRingEntries / kRingMinGroups <= 64, "one lane per entry");
}

// Host-side buffers of a private ring: pinned, coherent, device-mapped (host view == device view).
int CmdRing::alloc_host(size_t) {
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
  if (hipHostMalloc((void**)&shared_, sizeof(RingShared), fl) != hipSuccess) return -1;
  if (hipHostMalloc((void**)&cmds_, sizeof(RingCmd) * kRingEntries, fl) != hipSuccess) return -1;
  if (hipHostMalloc((void**)&payload_, (size_t)pstride_ * kRingEntries, fl) != hipSuccess) return -1;
  std::memset(shared_, 0, sizeof(RingShared));
  std::memset(cmds_, 0, sizeof(RingCmd) * kRingEntries);
  d_shared_ = shared_;
  d_cmds_ = cmds_;
  d_payload_ = payload_;
  ent_ = own_.ent;
  ticket_ = &own_.ticket;
  return 0;
}

int CmdRing::init(int device, uint32_t pstride) {
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_rings.insert(this);
  }
  device_ = device;
  pstride_ = (pstride + 15) & ~15u;
  if (pstride_ < kEmbedBytes) pstride_ = kEmbedBytes;
  read_env();
  if (alloc_host(0) != 0) return -1;
  if (hipMalloc((void**)&scratch_, (size_t)pstride_ * kRingEntries) != hipSuccess) return -1;
  if (hipMalloc((void**)&ctrl_, 64) != hipSuccess) return -1;
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
  clock_khz_ = khz > 0 ? khz : 100000;
  idle_ticks_ = (uint64_t)khz * (uint64_t)env_int("SPLINTER_RING_IDLE_US", 5000) / 1000u;
#ifndef SPL_RING_POLL4
  // default on: 1 thread p50 9.1 -> 7.3 us, 16 threads 1.18 -> 1.50 M ops/s (profiles/r3_hostapi_vram_ab.jsonl);
  // SPLINTER_RING_VRAM=0, or a failed VMM / BAR mapping, keeps everything in host memory
  if (env_int("SPLINTER_RING_VRAM", 1) != 0 && init_vram() != 0) vr_ = false;
#endif
  if (vr_) {
    if (hipHostMalloc((void**)&vdone_, sizeof(RingDone) * kRingEntries, hipHostMallocCoherent | hipHostMallocMapped) !=
        hipSuccess)
      return -1;
    std::memset(vdone_, 0, sizeof(RingDone) * kRingEntries);
    d_vdone_ = vdone_;
  }
  return 0;
}

namespace {
// segment layout: header | RingShared | RingCmd[entries] | RingDone[entries] | payload
struct SegLayout {
  size_t shared, cmds, done, pay, total;
  explicit SegLayout(uint32_t pstride) {
    auto up = [](size_t v, size_t a) { return (v + a - 1) / a * a; };
    shared = up(sizeof(RingSegHdr), 4096);
    cmds = up(shared + sizeof(RingShared), 4096);
    done = up(cmds + sizeof(RingCmd) * kRingEntries, 4096);
    pay = up(done + sizeof(RingDone) * kRingEntries, 4096);
    total = up(pay + (size_t)pstride * kRingEntries, 4096);
  }
};

long futex_op(uint32_t* w, int op, uint32_t v, const timespec* ts) {
  return syscall(SYS_futex, w, op, v, ts, nullptr, 0);
}
}  // namespace

int CmdRing::init_server(int device, uint32_t pstride, const std::string& seg, const std::string& perm_path,
                         const spl_arena_t& a) {
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_rings.insert(this);
  }
  mode_ = kServer;  // (a partial set-up is torn down as a server's)
  device_ = device;
  pstride_ = (pstride + 15) & ~15u;
  if (pstride_ < kEmbedBytes) pstride_ = kEmbedBytes;
  read_env();
  arena_ = a;
  if (hipMalloc((void**)&scratch_, (size_t)pstride_ * kRingEntries) != hipSuccess) return -1;
  if (hipMalloc((void**)&ctrl_, 64) != hipSuccess) return -1;
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
  clock_khz_ = khz > 0 ? khz : 100000;
  // 5 ms as a private worker: a device-wide synchronize in the owner (torch.cuda.synchronize)
  // waits for the resident worker until it idles out (profiles/r4r/sync_probe: 1000 ms at a 1 s
  // timeout), which cost the embedding daemon's loop 15x at 1 s (profiles/r4q/bench.out)
  idle_ticks_ = (uint64_t)khz * (uint64_t)env_int("SPLINTER_RING_IDLE_US", 5000) / 1000u;
  if (init_vram() != 0) return -1;
  // the segment: created under the store's umask like its descriptor, and fresh: a stale one of a
  // crashed owner of the same name is unlinked first (never truncated: its clients may still map it)
  const SegLayout L(pstride_);
  (void)shm_unlink(seg.c_str());
  mode_t prev = env_umask_push();
  const int fd = shm_open(seg.c_str(), O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0666);
  env_umask_pop(prev);
  if (fd < 0) return -1;
  if (ftruncate(fd, (off_t)L.total) != 0) { close(fd); shm_unlink(seg.c_str()); return -1; }
  void* p = mmap(nullptr, L.total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) { shm_unlink(seg.c_str()); return -1; }
  seg_ = (RingSegHdr*)p;
  seg_bytes_ = L.total;
  seg_name_ = seg;
  // (hipExtHostRegisterUncached measured no better: profiles/r4h t32_rf*, p4t8_rf*)
  if (hipHostRegister(p, L.total, hipHostRegisterMapped) != hipSuccess) return -1;
  seg_registered_ = true;
  uint8_t* dp = nullptr;
  if (hipHostGetDevicePointer((void**)&dp, p, 0) != hipSuccess) return -1;
  uint8_t* hp = (uint8_t*)p;
  shared_ = (RingShared*)(hp + L.shared);
  d_shared_ = (RingShared*)(dp + L.shared);
  cmds_ = (RingCmd*)(hp + L.cmds);
  d_cmds_ = (RingCmd*)(dp + L.cmds);
  vdone_ = (RingDone*)(hp + L.done);
  d_vdone_ = (RingDone*)(dp + L.done);
  payload_ = hp + L.pay;
  d_payload_ = dp + L.pay;
  ent_ = seg_->ent;
  ticket_ = &seg_->ticket;
  waiters_ = &seg_->waiters;
  // the request chunk's descriptors, for clients' BAR mappings
  char sock[96];
  snprintf(sock, sizeof sock, "splinter-ring-%d-%s", (int)getpid(), seg.c_str() + (seg[0] == '/'));
  if (vram_.serve(sock, perm_path) != 0) return -1;
  std::memcpy(seg_->sock, sock, sizeof sock);
  seg_->pstride = pstride_;
  seg_->entries = kRingEntries;
  seg_->groups = (uint32_t)groups_;
  seg_->version = 1;
  seg_->owner_pid = pid_;
  sup_ = std::thread([this] { supervise(); });
  __atomic_store_n(&seg_->magic, kRingSegMagic, __ATOMIC_RELEASE);
  return 0;
}

// The owner's supervisor: sleeps on the `want` futex; a client that found the worker gone bumps
// it, and the worker is relaunched here (only the owner's HIP runtime holds the arena mapping the
// worker runs on).  The 20 ms timeout only re-checks the stop flag.
void CmdRing::supervise() {
  uint32_t seen = __atomic_load_n(&seg_->want, __ATOMIC_ACQUIRE);
  while (!sup_stop_.load(std::memory_order_acquire)) {
    const timespec ts{0, 20 * 1000 * 1000};
    (void)futex_op(&seg_->want, FUTEX_WAIT, seen, &ts);
    const uint32_t w = __atomic_load_n(&seg_->want, __ATOMIC_ACQUIRE);
    if (w == seen || sup_stop_.load(std::memory_order_acquire)) continue;
    seen = w;
    // not while this process sets up or tears down a store (it holds the gate exclusive); poll for the
    // gate instead of blocking on it, so a teardown that joins this thread never waits on a supervisor
    // that waits on the teardown's gate
    std::shared_lock<std::shared_mutex> gate(g_gate, std::defer_lock);
    while (!gate.try_lock()) {
      if (sup_stop_.load(std::memory_order_acquire)) break;
      usleep(200);
    }
    if (!gate.owns_lock()) continue;
    if (!__atomic_load_n(&shared_->alive, __ATOMIC_ACQUIRE)) launch(arena_);
  }
}

int CmdRing::init_client(const std::string& seg, int device, uint32_t pstride) {
  const int fd = shm_open(seg.c_str(), O_RDWR | O_CLOEXEC, 0666);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(RingSegHdr)) { close(fd); return -1; }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return -1;
  seg_ = (RingSegHdr*)p;
  seg_bytes_ = (size_t)st.st_size;
  auto fail = [this]() {
    if (cmap_) munmap(cmap_, cmap_bytes_);
    cmap_ = nullptr;
    munmap(seg_, seg_bytes_);
    seg_ = nullptr;
    return -1;
  };
  if (__atomic_load_n(&seg_->magic, __ATOMIC_ACQUIRE) != kRingSegMagic || seg_->entries != (uint32_t)kRingEntries)
    return fail();
  const SegLayout L(seg_->pstride);
  if (L.total > seg_bytes_ || seg_->pstride < ((pstride + 15) & ~15u) || server_gone()) return fail();
  pstride_ = seg_->pstride;
  std::vector<int> fds;
  size_t chunk = 0;
  char sock[97] = {0};
  std::memcpy(sock, seg_->sock, 96);
  if (VmmArena::fetch(sock, &fds, &chunk) != 0 || fds.empty()) return fail();
  const size_t total = chunk * fds.size();
  void* r = mmap(nullptr, total, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  bool ok = r != MAP_FAILED;
  for (size_t i = 0; ok && i < fds.size(); ++i)
    ok = mmap((uint8_t*)r + i * chunk, chunk, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fds[i], 0) != MAP_FAILED;
  for (int f : fds) close(f);
  if (!ok) {
    if (r != MAP_FAILED) munmap(r, total);
    return fail();
  }
  cmap_ = r;
  cmap_bytes_ = total;
  const size_t door_b = 4096, cmd_b = sizeof(RingCmd) * kRingEntries;
  uint8_t* h = (uint8_t*)r;
  v_door_h_ = (uint32_t*)h;
  v_cmds_h_ = (RingCmd*)(h + door_b);
  v_pay_h_ = h + door_b + cmd_b;
  uint8_t* hp = (uint8_t*)p;
  shared_ = (RingShared*)(hp + L.shared);
  cmds_ = (RingCmd*)(hp + L.cmds);
  vdone_ = (RingDone*)(hp + L.done);
  payload_ = hp + L.pay;
  ent_ = seg_->ent;
  ticket_ = &seg_->ticket;
  waiters_ = &seg_->waiters;
  device_ = device;
  read_env();
  if (seg_->groups >= (uint32_t)kRingMinGroups && seg_->groups <= (uint32_t)kRingGroups) groups_ = (int)seg_->groups;
  vr_ = true;
  mode_ = kClient;
  return 0;
}

void CmdRing::stop_supervisor() {
  if (mode_ != kServer) return;
  sup_stop_.store(true, std::memory_order_release);
  if (sup_.joinable()) {
    want_worker();
    sup_.join();
  }
}

bool CmdRing::server_gone() const {
  if (__atomic_load_n(&seg_->magic, __ATOMIC_ACQUIRE) != kRingSegMagic) return true;
  const int32_t o = seg_->owner_pid;
  return o <= 0 || (kill(o, 0) != 0 && errno == ESRCH);
}

void CmdRing::want_worker() {
  __atomic_fetch_add(&seg_->want, 1u, __ATOMIC_RELEASE);
  (void)futex_op(&seg_->want, FUTEX_WAKE, 1, nullptr);
}

// The request side in device memory: one VMM chunk (2 MiB granules) exported as a dmabuf and
// mapped on the CPU through the PCIe BAR (VmmArena::host_map, profiles/r2_hbm_host_map.md):
// [doorbells 4 KiB | records 32 KiB | input payloads kRingEntries x pstride].
int CmdRing::init_vram() {
  const size_t door_b = 4096, cmd_b = sizeof(RingCmd) * kRingEntries, pay_b = (size_t)pstride_ * kRingEntries;
  if (vram_.create(device_, door_b + cmd_b + pay_b, 2u << 20) != 0) return -1;
  uint8_t* h = (uint8_t*)vram_.host_map();
  if (!h) return -1;
  uint8_t* d = (uint8_t*)vram_.base();
  if (hipMalloc((void**)&served_, sizeof(uint32_t) * kRingEntries) != hipSuccess) return -1;
  // the clears go on a private non-blocking stream and only that stream is waited for: a device-wide
  // synchronize (or a null-stream memset) would also wait for every other store's resident ring
  // worker and for unrelated kernels, so opening a second store beside live traffic could block
  hipStream_t z = nullptr;
  if (hipStreamCreateWithFlags(&z, hipStreamNonBlocking) != hipSuccess) return -1;
  const bool ok = hipMemsetAsync(d, 0, door_b + cmd_b, z) == hipSuccess &&
                  hipMemsetAsync(served_, 0, sizeof(uint32_t) * kRingEntries, z) == hipSuccess &&
                  hipStreamSynchronize(z) == hipSuccess;
  (void)hipStreamDestroy(z);
  if (!ok) return -1;
  v_door_h_ = (uint32_t*)h;
  v_cmds_h_ = (RingCmd*)(h + door_b);
  v_pay_h_ = h + door_b + cmd_b;
  v_door_d_ = (uint32_t*)d;
  v_cmds_d_ = (RingCmd*)(d + door_b);
  v_pay_d_ = d + door_b + cmd_b;
  vr_ = true;
  return 0;
}

void CmdRing::launch(const spl_arena_t& a) {
  std::lock_guard<std::mutex> lk(launch_mu_);
  if (mode_ == kPrivate) arena_ = a;  // (for resume)
  if (!a.base) return;  // no arena mapped in this process (a lazily attached client): nothing to serve
  // held (this process, or the store by any process): the waiters retry later
  if (__atomic_load_n(&shared_->hold, __ATOMIC_ACQUIRE)) reap_holds();
  if (g_hold.load(std::memory_order_acquire) > 0 || __atomic_load_n(&shared_->hold, __ATOMIC_ACQUIRE)) return;
  if (__atomic_load_n(&shared_->alive, __ATOMIC_ACQUIRE)) return;
  __atomic_store_n(&shared_->alive, 1u, __ATOMIC_RELEASE);
  __atomic_fetch_add(seg_ ? &seg_->launches : &shared_->launches, 1u, __ATOMIC_RELAXED);
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != device_) (void)hipSetDevice(device_);
  if (!stream_) {  // created on first use: a store that never takes a per-call op claims no queue
    // normal priority (SPLINTER_RING_PRIORITY=1: high): a resident worker on a high-priority queue
    // cost a concurrent encoder +84 %, on a normal one +30 % (profiles/r4y); a CU-masked queue
    // measured worse (profiles/r4h interf_cus*)
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    (void)hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, env_int("SPLINTER_RING_PRIORITY", 0) ? hi : 0);
  }
  // stream order: the previous worker (if still draining) has exited before ctrl is reset
  const uint32_t init[4] = {0u, 0u, 0u, (uint32_t)groups_};
  (void)hipMemcpyAsync(ctrl_, init, sizeof init, hipMemcpyHostToDevice, stream_);
  if (vr_)
    hipLaunchKernelGGL(k_ring_worker<true>, dim3(groups_), dim3(64), 0, stream_, a, v_cmds_d_, d_cmds_, d_shared_,
                       v_door_d_, v_pay_d_, d_payload_, pstride_, scratch_, ctrl_, served_, d_vdone_, idle_ticks_,
                       kRingEntries / groups_);
  else
    hipLaunchKernelGGL(k_ring_worker<false>, dim3(groups_), dim3(64), 0, stream_, a, d_cmds_, d_cmds_, d_shared_,
                       (const uint32_t*)nullptr, (const uint8_t*)nullptr, d_payload_, pstride_, scratch_, ctrl_,
                       (uint32_t*)nullptr, (RingDone*)nullptr, idle_ticks_, kRingEntries / groups_);
  if (cur != device_) (void)hipSetDevice(cur);
}

int CmdRing::call(const spl_arena_t& a, uint32_t op, uint32_t sub, const char key64[64], uint32_t klen,
                  uint64_t khash, const void* in, uint32_t in_len, uint64_t arg, void* out, uint32_t out_cap,
                  RingResult* r) {
  if (mode_ == kClient && (gone_.load(std::memory_order_acquire) || server_gone())) {
    // the owner closed the store or died: this process serves itself from now on (the arena it
    // imported stays valid in VMM mode)
    gone_.store(true, std::memory_order_release);
    // the private worker runs on THIS process's mapping of the arena: a client that attached lazily
    // and has not mapped it yet gets EAGAIN (HbmStore::ring maps it and calls again), never a worker
    // launched on a null arena
    if (!a.base) { errno = EAGAIN; return -1; }
    std::unique_lock<std::mutex> lk(priv_mu_);
    if (!priv_) {
      RingQuiesce quiet;  // ring set-up makes HIP calls: as for a store set-up
      auto p = std::make_unique<CmdRing>();
      if (p->init(device_, pstride_) != 0) { errno = EIO; return -1; }
      priv_ = std::move(p);
    }
    CmdRing* pr = priv_.get();
    lk.unlock();
    return pr->call(a, op, sub, key64, klen, khash, in, in_len, arg, out, out_cap, r);
  }
  return call_private(a, op, sub, key64, klen, khash, in, in_len, arg, out, out_cap, r);
}

#ifdef SPL_RING_STAMPS
// Host half of the per-call latency breakdown (stamps build): per call, CLOCK_MONOTONIC ns from
// entry to owning a ring entry, to the record + payload + doorbell written through the BAR, to the
// completion observed, to the return; the wait's time inside nanosleep (CPU released) and its
// sleeps.  Summed per thread, folded into the process totals when the thread exits, printed by
// ~CmdRing beside the worker's device-side segments.
struct HostStampSums {
  std::atomic<uint64_t> n{0}, own{0}, post{0}, wait{0}, slept{0}, sleeps{0}, fin{0};
};
static HostStampSums g_hstamps;
struct HostStampLocal {
  uint64_t n = 0, own = 0, post = 0, wait = 0, slept = 0, sleeps = 0, fin = 0;
  void flush() {
    g_hstamps.n += n, g_hstamps.own += own, g_hstamps.post += post, g_hstamps.wait += wait;
    g_hstamps.slept += slept, g_hstamps.sleeps += sleeps, g_hstamps.fin += fin;
    n = own = post = wait = slept = sleeps = fin = 0;
  }
  ~HostStampLocal() { flush(); }
};
static thread_local HostStampLocal t_hstamps;
static inline uint64_t mono_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}
#define HOST_TS(v) const uint64_t v = mono_ns()
#else
#define HOST_TS(v) ((void)0)
#endif

int CmdRing::call_private(const spl_arena_t& a, uint32_t op, uint32_t sub, const char key64[64], uint32_t klen,
                          uint64_t khash, const void* in, uint32_t in_len, uint64_t arg, void* out, uint32_t out_cap,
                          RingResult* r) {
  if (in_len > pstride_) { errno = EMSGSIZE; return -1; }
  HOST_TS(hs0);
  std::shared_lock<std::shared_mutex> gate(g_gate, std::defer_lock);
  if (!t_exclusive) gate.lock();  // (a store set-up on this thread already holds it exclusive)
  // own an entry: start at a rotating ticket, CAS the busy flag (in the shared segment for a ring
  // server: every process's callers draw from one ticket).  Consecutive tickets map to different
  // groups (entry = (t % groups) * per_group + t / groups), so concurrent callers land on
  // different worker waves -- which run in parallel -- instead of sharing one wave whose lanes
  // would serve them with divergent ops
  const bool spread = spread_;
  const uint32_t G = (uint32_t)groups_, per = (uint32_t)(kRingEntries / groups_);
  auto entry_of = [spread, G, per](uint32_t t) {
    t %= kRingEntries;
    return spread ? (t % G) * per + t / G : t;
  };
  auto finished = [this](uint32_t e) {
    return vr_ ? __atomic_load_n(&vdone_[e].seq, __ATOMIC_ACQUIRE) == __atomic_load_n(&ent_[e].seq, __ATOMIC_ACQUIRE)
               : __atomic_load_n(&shared_->state[e], __ATOMIC_ACQUIRE) == (uint32_t)kRingDone;
  };
  uint32_t t = __atomic_fetch_add(ticket_, 1u, __ATOMIC_RELAXED);
  uint32_t e = entry_of(t);
  timespec t0;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  auto elapsed_us = [&t0]() {
    timespec n;
    clock_gettime(CLOCK_MONOTONIC, &n);
    return (uint64_t)(n.tv_sec - t0.tv_sec) * 1000000u + (uint64_t)((n.tv_nsec - t0.tv_nsec) / 1000);
  };
  for (uint32_t spins = 0;; ++spins) {
    const uint32_t me = (uint32_t)pid_;
    uint32_t z = 0;
    if (__atomic_compare_exchange_n(&ent_[e].busy, &z, me, true, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) break;
    // an entry a timed-out caller abandoned is reclaimed once the worker has finished it
    z = kRingAbandoned;
    if (finished(e) && __atomic_compare_exchange_n(&ent_[e].busy, &z, me, false, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) {
      if (!vr_) __atomic_store_n(&shared_->state[e], (uint32_t)kRingFree, __ATOMIC_RELEASE);
      break;
    }
    if ((spins & 63) == 63) {
      // an entry held by a process that died is abandoned (its call is reclaimed once finished); the
      // CAS only succeeds on the exact dead pid it read, so a live owner is never abandoned
      const uint32_t h = __atomic_load_n(&ent_[e].busy, __ATOMIC_RELAXED);
      z = h;
      if (mode_ != kPrivate && h != 0 && h != kRingAbandoned && h != me && kill((pid_t)h, 0) != 0 && errno == ESRCH)
        (void)__atomic_compare_exchange_n(&ent_[e].busy, &z, kRingAbandoned, false, __ATOMIC_RELAXED,
                                          __ATOMIC_RELAXED);
      _mm_pause();
      if (elapsed_us() > 30000000u) {  // every entry held for 30 s: the GPU stopped serving
        errno = EBUSY;
        return -1;
      }
      sched_yield();
    }
    e = entry_of(++t);
  }
  HOST_TS(hs1);
  RingCmd* c = cmds_ + e;
  uint32_t done_word = kRingDone;
  if (vr_) {
    // the record is assembled locally and copied to the device-memory record with wide stores
    // (the BAR mapping is write-combining): payload, record, sfence, then the doorbell
    RingCmd rc{};
    rc.op = op;
    rc.sub = sub;
    rc.len = in_len;
    rc.cap = out_cap ? (out_cap < pstride_ ? out_cap : pstride_) : pstride_;
    rc.arg = arg;
    rc.khash = khash;
    rc.klen = klen;
    if (key64) std::memcpy(rc.key, key64, 64);
    if (in && in_len) std::memcpy(v_pay_h_ + (size_t)e * pstride_, in, in_len);
    std::memcpy((void*)(v_cmds_h_ + e), &rc, sizeof rc);
    c->out_len = 0;  // written by the worker only when the op returns bytes
    uint32_t seq = ent_[e].seq + 1;
    if (seq == 0) seq = 1;  // 0 is the initial "served" value
    __atomic_store_n(&ent_[e].seq, seq, __ATOMIC_RELEASE);
    done_word = seq;
    _mm_sfence();
    *(volatile uint32_t*)(v_door_h_ + e) = seq;
    _mm_sfence();
  } else {
    c->op = op;
    c->sub = sub;
    c->len = in_len;
    c->cap = out_cap ? (out_cap < pstride_ ? out_cap : pstride_) : pstride_;
    c->arg = arg;
    c->khash = khash;
    c->klen = klen;
    if (key64) std::memcpy(c->key, key64, 64);
    if (in && in_len) std::memcpy(payload_ + (size_t)e * pstride_, in, in_len);
    __atomic_store_n(&shared_->state[e], (uint32_t)kRingReady, __ATOMIC_RELEASE);
  }
  auto ensure_worker = [&]() {
    if (__atomic_load_n(&shared_->alive, __ATOMIC_ACQUIRE)) return;
    if (mode_ == kClient) want_worker();
    else launch(mode_ == kServer ? arena_ : a);
  };
  ensure_worker();
  HOST_TS(hs2);
#ifdef SPL_RING_STAMPS
  uint64_t hslept = 0, hsleeps = 0;
#endif
  clock_gettime(CLOCK_MONOTONIC, &t0);
  // Wait for completion: spin (a call is served in ~10 us), then give the CPU away between polls.
  // With more waiting callers than CPUs the process may run on (cgroup quota included), spinning
  // burns the quota every waiter shares -- the scheduler then throttles the whole process, the
  // 16 -> 32 thread collapse of profiles/r2_hostapi_ring_v3.md -- so while more callers wait than
  // there are CPUs every waiter sleeps ~2 us between polls (1 us timer slack): the calls stay in
  // flight on the GPU without holding a CPU each.  A ring server's waiters are counted over every
  // process that submits to it (the segment's counter: the processes share the same CPUs; a client
  // that dies mid-call leaves its count behind, which only makes waiters sleep-poll sooner).
  __atomic_fetch_add(waiters_, 1, __ATOMIC_RELAXED);
  struct Leave {
    int32_t* w;
    ~Leave() { __atomic_fetch_sub(w, 1, __ATOMIC_RELAXED); }
  } leave{waiters_};
  bool slept = false;
  for (uint64_t spins = 1;; ++spins) {
    if (vr_ ? __atomic_load_n(&vdone_[e].seq, __ATOMIC_ACQUIRE) == done_word
            : __atomic_load_n(&shared_->state[e], __ATOMIC_ACQUIRE) == done_word)
      break;
    _mm_pause();
    if ((spins & 31) == 0) {
      const uint64_t us = elapsed_us();
      // re-decided every poll round: once more callers wait than there are CPUs, EVERY waiter
      // (also those that started spinning before the others arrived) sleep-polls
      const bool oversub = __atomic_load_n(waiters_, __ATOMIC_RELAXED) > cpus_;
      if (us > (oversub ? oversub_spin_us_ : yield_after_us_) || (oversub && oversub_spin_us_ == 0)) {
        if (oversub) {
          static thread_local bool slack = false;
          if (!slack) {
            (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
            slack = true;
          }
          // the first sleep covers most of a call's expected latency under this load (EWMA of
          // recent oversubscribed calls): one or two wakeups per call instead of one per ~5 us
          long first = first_sleep_ns_;
          if (adaptive_) {
            const long est = ewma_ns_.load(std::memory_order_relaxed) * 5 / 8;
            if (est > first) first = est < 100000 ? est : 100000;
          }
          const timespec ts{0, slept ? sleep_ns_ : first};
          slept = true;
#ifdef SPL_RING_STAMPS
          const uint64_t z0 = mono_ns();
          nanosleep(&ts, nullptr);
          hslept += mono_ns() - z0;
          ++hsleeps;
#else
          nanosleep(&ts, nullptr);
#endif
        } else {
          sched_yield();
        }
      }
      if ((spins & 1023) == 0) {
        ensure_worker();  // the worker idled out meanwhile
        const bool dead = mode_ == kClient && server_gone();
        if (dead || us > 30000000u) {  // the GPU stopped serving: abandon the entry (reclaimed once done)
          __atomic_store_n(&ent_[e].busy, kRingAbandoned, __ATOMIC_RELEASE);
          if (dead) gone_.store(true, std::memory_order_release);
          errno = dead ? EIO : ETIMEDOUT;
          return -1;
        }
      }
    }
  }
  HOST_TS(hs3);
  if (slept && adaptive_) {  // latency of an oversubscribed call, for the next first sleeps
    const long ns = (long)elapsed_us() * 1000;
    const long o = ewma_ns_.load(std::memory_order_relaxed);
    ewma_ns_.store(o + (ns - o) / 8, std::memory_order_relaxed);
  }
  if (vr_) {
    r->status = vdone_[e].status;
    r->result = vdone_[e].result;
    r->out_len = __atomic_load_n(&c->out_len, __ATOMIC_ACQUIRE);
  } else {
    uint64_t sl;
    std::memcpy(&sl, &c->status, 8);
    r->status = (int32_t)(uint32_t)sl;
    r->out_len = (uint32_t)(sl >> 32);
    r->result = c->result;
  }
  if (out && out_cap && r->out_len && r->status >= 0)
    std::memcpy(out, payload_ + (size_t)e * pstride_, r->out_len < out_cap ? r->out_len : out_cap);
  if (!vr_) __atomic_store_n(&shared_->state[e], (uint32_t)kRingFree, __ATOMIC_RELEASE);
  __atomic_store_n(&ent_[e].busy, 0u, __ATOMIC_RELEASE);
#ifdef SPL_RING_STAMPS
  {
    HostStampLocal& h = t_hstamps;
    const uint64_t hs4 = mono_ns();
    ++h.n, h.own += hs1 - hs0, h.post += hs2 - hs1, h.wait += hs3 - hs2, h.fin += hs4 - hs3;
    h.slept += hslept, h.sleeps += hsleeps;
    if ((h.n & 1023) == 0) h.flush();
  }
#endif
  return 0;
}

int CmdRing::hold(bool on) {
  if (!shared_) { errno = ENOSYS; return -1; }
  if (mode_ == kClient && gone_.load(std::memory_order_acquire) && priv_) return priv_->hold(on);
  RingShared::HoldSlot* hs = shared_->holds;
  if (on) {
    const int slot = hold_slot(true);
    if (slot < 0) { errno = EBUSY; return -1; }  // kRingHoldSlots processes hold the store already
    __atomic_fetch_add(&hs[slot].count, 1u, __ATOMIC_ACQ_REL);
    __atomic_fetch_add(&shared_->hold, 1u, __ATOMIC_ACQ_REL);
    // the worker sees the flag within a poll round; wait until its last wave is out
    timespec t0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    while (__atomic_load_n(&shared_->alive, __ATOMIC_ACQUIRE)) {
      timespec n;
      clock_gettime(CLOCK_MONOTONIC, &n);
      if ((n.tv_sec - t0.tv_sec) * 1000000000L + (n.tv_nsec - t0.tv_nsec) > 10000000000L) {
        hold(false);  // the hold was not granted: take it back (a caller that sees -1 never releases it)
        errno = ETIMEDOUT;
        return -1;
      }
      sched_yield();
    }
    return 0;
  }
  const int slot = hold_slot(false);
  if (slot < 0) { errno = EINVAL; return -1; }  // this process holds nothing
  uint32_t c = __atomic_load_n(&hs[slot].count, __ATOMIC_ACQUIRE);
  do {
    if (c == 0) { errno = EINVAL; return -1; }
  } while (!__atomic_compare_exchange_n(&hs[slot].count, &c, c - 1, true, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE));
  if (__atomic_sub_fetch(&shared_->hold, 1u, __ATOMIC_ACQ_REL) != 0) return 0;
  if (__atomic_load_n(waiters_, __ATOMIC_RELAXED) > 0) {  // calls are waiting: a worker again
    if (mode_ == kClient) want_worker();
    else if (arena_.base) launch(arena_);
  }
  return 0;
}

// This process's hold slot: the one carrying its pid, or (claim) a free one -- after taking back the
// slots of holders that died when none is free.  A slot stays with its process until the process
// dies (clearing it on release would race a second thread of the same process that found it).
int CmdRing::hold_slot(bool claim) {
  RingShared::HoldSlot* hs = shared_->holds;
  for (int i = 0; i < kRingHoldSlots; ++i)
    if (__atomic_load_n(&hs[i].pid, __ATOMIC_ACQUIRE) == pid_) return i;
  if (!claim) return -1;
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = 0; i < kRingHoldSlots; ++i) {
      int32_t z = 0;
      if (__atomic_compare_exchange_n(&hs[i].pid, &z, pid_, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) return i;
      if (z == pid_) return i;  // another thread of this process claimed it meanwhile
    }
    reap_holds();
  }
  return -1;
}

// A holder that died (crash, kill) leaves its count in shared_->hold and would keep every worker of
// the store down for good: its slot's count is taken back (exchanged to 0 first, so two reapers never
// both subtract it) and the slot freed.
void CmdRing::reap_holds() {
  RingShared::HoldSlot* hs = shared_->holds;
  for (int i = 0; i < kRingHoldSlots; ++i) {
    const int32_t p = __atomic_load_n(&hs[i].pid, __ATOMIC_ACQUIRE);
    if (p <= 0 || p == pid_ || !(kill(p, 0) != 0 && errno == ESRCH)) continue;
    const uint32_t c = __atomic_exchange_n(&hs[i].count, 0u, __ATOMIC_ACQ_REL);
    if (c) __atomic_fetch_sub(&shared_->hold, c, __ATOMIC_ACQ_REL);
    int32_t exp = p;
    (void)__atomic_compare_exchange_n(&hs[i].pid, &exp, 0, false, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED);
  }
}

// after a hold: relaunch the worker if calls are waiting for it
void CmdRing::resume() {
  if (!shared_ || mode_ == kClient || !arena_.base) return;
  if (__atomic_load_n(waiters_, __ATOMIC_RELAXED) > 0) launch(arena_);
}

void CmdRing::stop() {
  if (!shared_ || mode_ == kClient) {  // a client's only worker is its private fallback's
    if (priv_) priv_->stop();
    return;
  }
  __atomic_store_n(&shared_->stop, 1u, __ATOMIC_RELEASE);
  if (stream_) (void)hipStreamSynchronize(stream_);
  __atomic_store_n(&shared_->stop, 0u, __ATOMIC_RELEASE);
}

CmdRing::~CmdRing() {
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_rings.erase(this);
  }
  priv_.reset();
  if (mode_ == kClient) {
    if (cmap_) munmap(cmap_, cmap_bytes_);
    if (seg_) munmap(seg_, seg_bytes_);
    return;
  }
  if (mode_ == kServer) {
    // clients see the segment close first (their calls then fail over to private rings), then
    // the supervisor and the worker stop
    if (seg_) __atomic_store_n(&seg_->magic, 0u, __ATOMIC_RELEASE);
    stop_supervisor();
  }
  stop();
#ifdef SPL_RING_STAMPS
  if (shared_) {
    static uint64_t hst[kRingEntries][4], hop[kRingEntries][10], hck[kRingEntries][2];
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device_);
    const bool got = hipDeviceSynchronize() == hipSuccess &&
                     hipMemcpyFromSymbol(hst, HIP_SYMBOL(g_stamp), sizeof hst) == hipSuccess &&
                     hipMemcpyFromSymbol(hop, HIP_SYMBOL(g_opstamp), sizeof hop) == hipSuccess &&
                     hipMemcpyFromSymbol(hck, HIP_SYMBOL(g_clk), sizeof hck) == hipSuccess;
    (void)hipSetDevice(cur);
    uint64_t sum[4] = {0, 0, 0, 0};
    for (int e = 0; got && e < kRingEntries; ++e)
      for (int q = 0; q < 4; ++q) sum[q] += hst[e][q];
    if (sum[3]) {
      const double us = 1000.0 / clock_khz_ / (double)sum[3];
      fprintf(stderr,
              "{\"ring_stamps\": %llu, \"seen_to_loaded_us\": %.3f, \"loaded_to_op_done_us\": %.3f, "
              "\"op_done_to_drained_us\": %.3f}\n",
              (unsigned long long)sum[3], sum[0] * us, sum[1] * us, sum[2] * us);
    }
    uint64_t ck[2] = {0, 0};
    for (int e = 0; got && e < kRingEntries; ++e) ck[0] += hck[e][0], ck[1] += hck[e][1];
    if (ck[1]) fprintf(stderr, "{\"shader_clock_mhz\": %.1f}\n", (double)ck[0] / ((double)ck[1] / (clock_khz_ * 1e3)) / 1e6);
    uint64_t o[10] = {};
    for (int e = 0; got && e < kRingEntries; ++e)
      for (int q = 0; q < 10; ++q) o[q] += hop[e][q];
    for (int k = 0; k < 2; ++k) {
      const uint64_t* v = o + 5 * k;
      if (!v[4]) continue;
      const double us = 1000.0 / clock_khz_ / (double)v[4];
      fprintf(stderr, "{\"op\": \"%s\", \"n\": %llu, \"seg_us\": [%.3f, %.3f, %.3f, %.3f]}\n", k ? "get" : "set",
              (unsigned long long)v[4], v[0] * us, v[1] * us, v[2] * us, v[3] * us);
    }
  }
  t_hstamps.flush();
  if (const uint64_t n = g_hstamps.n.load()) {
    const double k = 1e-3 / (double)n;  // ns sums -> us per call
    fprintf(stderr,
            "{\"host_stamps\": %llu, \"own_entry_us\": %.3f, \"post_record_doorbell_us\": %.3f, "
            "\"doorbell_to_completion_seen_us\": %.3f, \"of_it_asleep_us\": %.3f, \"sleeps_per_call\": %.3f, "
            "\"completion_to_return_us\": %.3f}\n",
            (unsigned long long)n, g_hstamps.own.load() * k, g_hstamps.post.load() * k, g_hstamps.wait.load() * k,
            g_hstamps.slept.load() * k, (double)g_hstamps.sleeps.load() / (double)n, g_hstamps.fin.load() * k);
  }
#endif
  if (stream_) (void)hipStreamDestroy(stream_);
  if (served_) (void)hipFree(served_);
  if (ctrl_) (void)hipFree(ctrl_);
  if (scratch_) (void)hipFree(scratch_);
  if (mode_ == kServer) {
    vram_.release();
    if (seg_) {
      if (seg_registered_) (void)hipHostUnregister(seg_);
      munmap(seg_, seg_bytes_);
      shm_unlink(seg_name_.c_str());
    }
    return;
  }
  if (vdone_) (void)hipHostFree(vdone_);
  if (payload_) (void)hipHostFree(payload_);
  if (cmds_) (void)hipHostFree(cmds_);
  if (shared_) (void)hipHostFree(shared_);
}

}  // namespace spl
