// cmd_ring.hpp — per-call API of an HBM store through a host-mapped command ring.
//
// The reference's splinter_set/get are in-process calls of a few hundred ns on a CPU mapping
// (reference splinter.c:365-464).  On the HBM backend every mutation runs on the GPU that owns
// the arena (owner computes), so a per-call op must reach a device thread.
// A kernel launch + copies + stream sync per call costs tens of µs; instead each process keeps
//   * a ring of kEntries command records in pinned, host-coherent memory (one per lane),
//   * a contiguous doorbell array state[kEntries],
//   * ONE resident worker kernel (k_ring_worker) of `groups` one-wave workgroups on a
//     normal-priority stream (SPLINTER_RING_GROUPS, default 32); lane i of group g serves entry
//     g*per+i (per = kRingEntries / groups) and each group polls its doorbells in one coalesced
//     read, so concurrent host threads' calls run in parallel waves.  A resident worker costs a
//     concurrent GPU job of the same process queue time-slices (+29 % for the encoder on a
//     normal-priority queue, +84 % on a high-priority one, whatever the wave count: profiles/r4y),
//     hence ring_hold() for processes that run such a job.  (One kernel, not one per group: streams share
//     GPU_MAX_HW_QUEUES hardware queues, and a group queued behind another group's resident
//     kernel would wait out that kernel's idle timeout.)
// Ring server: the process that created the store (its owner) runs the store's ONE worker and
// keeps the host side of the ring in a shared segment (RingSegHdr below); every other process that
// opens the store submits its calls to that worker instead of launching its own, so a GPU carries
// one polling worker per store, not one per client process, and the callers of every process share
// the same wave rounds.  SPLINTER_RING_SHARED=0 (or a store without VMM chunks) keeps a worker
// per process.
// Host callers take entries in ticket order spread over the groups (consecutive calls land on
// different waves, so up to kRingGroups concurrent callers are served in parallel waves, not
// as divergent lanes of one wave): 1 thread p50 11.7 us, 16 threads 1.02 M ops/s at p50 14.9 us
// (profiles/r2_hostapi_ring_v2.jsonl).  Ops other than set / get touch slots with plain
// accesses, so the worker brackets them with agent-scope acquire / release: the next call may
// run on another XCD.
// The worker exits after SPLINTER_RING_IDLE_US without any call (default 5000 µs; the activity
// clock is shared by the groups through device memory, and the first group to time out tells
// the others to exit, so no group outlives the rest) or on stop: a process that stops issuing
// per-call ops holds no CU and hipDeviceSynchronize returns.  The next call relaunches it (a waiter
// that sees the worker gone relaunches it itself, so a call can never be stranded between the
// worker's last poll and its exit).
//
// Entry protocol (host thread <-> worker lane), all on the shared doorbell word:
//   FREE --host: fill record + payload, store-release READY--> READY
//   READY --lane: system-scope loads of the record, run the op, write results with system-scope
//            stores, drain, system-scope store DONE--> DONE
//   DONE --host: read results, store FREE--> FREE
// Host threads own an entry through a host-only busy flag (CAS), never through the doorbell.
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "arena_api.h"
#include "vmm_share.hpp"

namespace spl {

enum RingOp : uint32_t {
  kRingSet = 1,
  kRingGet = 2,
  kRingUnset = 3,
  kRingAppend = 4,
  kRingIntop = 5,      // sub = splinter_integer_op_t, arg = mask
  kRingMeta = 6,       // sub = SPL_META_* (arena_api.h), arg
  kRingEmbedSet = 7,   // payload = 768 f32
  kRingEmbedGet = 8,
  kRingRead = 9,       // arg = arena byte offset, len bytes (8-B aligned) -> payload
  kRingWrite = 10,     // payload -> arena byte offset arg (8-B aligned), agent release
  kRingSnapshot = 11,  // slot core (128 B) of the key's slot + its index in result
};

enum RingState : uint32_t { kRingFree = 0, kRingReady = 1, kRingDone = 2 };

struct alignas(128) RingCmd {
  uint32_t op, sub, len, cap;  // cap: payload capacity for outputs
  uint64_t arg;
  uint64_t khash;              // FNV-1a of the canonical key (host-computed: no hashing on the device)
  int32_t status;              // device status (0 / -EAGAIN / -ENOENT / ...; unset: old length)
  uint32_t out_len;            // status, out_len, result: one 16-B chunk (one device store)
  uint64_t result;
  uint32_t klen;               // canonical key length (<= 63)
  uint32_t pad[3];
  char key[64];                // canonical key record (NUL padded past klen)
};
static_assert(sizeof(RingCmd) == 128, "ring record");
static_assert(offsetof(RingCmd, status) % 16 == 0 && offsetof(RingCmd, result) == offsetof(RingCmd, status) + 8,
              "the completion words must form one 16-B chunk");

constexpr int kRingGroups = 32;                     // most one-wave workers (SPLINTER_RING_GROUPS)
constexpr int kDefaultRingGroups = 32;              // default worker waves (32 vs 8: 1.29-1.32 vs 1.05-1.09 M ops/s at
                                                    // 64 host threads, no fall-off from 32 threads; profiles/r4ab)
constexpr int kRingEntries = 256;                   // entries (per wave: kRingEntries / groups)
constexpr int kRingMinGroups = kRingEntries / 64;   // a wave's 64 lanes serve at most 64 entries
constexpr int kRingHoldSlots = 16;                  // processes that may hold a store's ring at once

struct RingShared {
  uint32_t state[kRingEntries];  // doorbells (one 32-B read per group)
  uint32_t alive;                // the worker is running or queued (cleared by its last wave)
  uint32_t stop;                 // ask the worker to exit
  uint32_t launches;             // host statistic
  uint32_t hold;                 // store-level holds (CmdRing::hold, any attached process): no worker
  uint32_t pad[12];
  // who holds `hold`: one slot per holding process (pid, its count), so the count a holder that died
  // left behind is taken back (CmdRing::reap_holds) instead of stopping the store's worker for good
  struct HoldSlot {
    int32_t pid;
    uint32_t count;
  } holds[kRingHoldSlots];
};

// VRAM mode completion, one 16-B chunk per entry in host memory, written by ONE device store (the
// NVMe completion-entry pattern): the call's sequence number with its status and result, so an op
// without output bytes completes with a single PCIe write and no drain of it
struct alignas(64) RingDone {  // one cache line per entry: a completion never disturbs another entry's poller
  uint32_t seq;
  int32_t status;
  uint64_t result;
  uint8_t pad[48];
};

// Host-side ownership of one entry (own cache line: callers on different entries share no line).
// `busy` is the owner's pid (0 free, kRingAbandoned abandoned -- reclaimed once its call is done):
// ownership and the owner's identity are ONE word, taken by one CAS, so a live owner can never be
// mistaken for a dead one between taking the entry and recording who took it.
constexpr uint32_t kRingAbandoned = 0xffffffffu;
struct alignas(64) RingEntryCtl {
  uint32_t busy;    // 0 free, pid of the holding process, or kRingAbandoned
  uint32_t seq;     // last sequence number issued
  uint32_t pad[14];
};

struct RingResult {
  int32_t status = 0;
  uint32_t out_len = 0;
  uint64_t result = 0;
};

// Scope guard held while a store of this process is set up or torn down (hbm_store.hip): waits
// for in-flight per-call ops, stops every live ring worker of the process and keeps new calls out
// until the scope ends (they then relaunch their worker).  Re-entrant on one thread.
class RingQuiesce {
 public:
  RingQuiesce();
  ~RingQuiesce();
  RingQuiesce(const RingQuiesce&) = delete;
  RingQuiesce& operator=(const RingQuiesce&) = delete;

 private:
  bool held_ = false;
};

// Shared ring segment of a store's ring SERVER: POSIX shm "<store>.ring", created by the store's
// owner (the process that created the arena) and mapped by every process that opens the store.
// It holds the host-side half of the ring -- entry ownership, sequence numbers, completion chunks,
// output payloads, the worker's control words -- registered with the owner's HIP runtime so its one
// resident worker writes completions straight into it; the request side (records, input payloads,
// doorbells) is the owner's VRAM chunk, which every client maps through the PCIe BAR (dmabuf fds
// from the owner's socket, `sock`).  A client process runs no worker kernel at all: it rings the
// doorbell and, when the worker has idled out, bumps `want` (a futex) for the owner's supervisor
// thread to relaunch it.  So a GPU carries one polling worker per store however many processes
// issue per-call ops, and concurrent callers of every process are served in the same wave rounds.
struct RingSegHdr {
  uint32_t magic, version, pstride, entries;
  int32_t owner_pid;
  uint32_t want;     // futex word: bumped by a client that found the worker gone
  uint32_t ticket;   // entry tickets of every process
  uint32_t launches;
  uint32_t groups;   // worker waves (the server's SPLINTER_RING_GROUPS)
  uint32_t pad0[3];
  char sock[96];     // abstract socket serving the request chunk's dmabuf fds
  alignas(64) int32_t waiters;  // callers of every process waiting on a completion right now
  RingEntryCtl ent[kRingEntries];
};
constexpr uint32_t kRingSegMagic = 0x52494e47;  // "RING"

// Hold every ring worker of this process (stopped, no relaunch) until the matching release;
// nestable.  Per-call ops wait meanwhile.  spl_ring_hold (arena_api.h) is the C entry point.
void ring_hold(bool on);

class CmdRing {
 public:
  // Private ring of this process (its own worker).  device: ordinal of the arena's GPU; pstride:
  // payload bytes per entry (>= max value, vector)
  int init(int device, uint32_t pstride);
  // Ring server of a store this process owns: the private ring's worker, with its host side in the
  // shared segment `seg` (shm name) so other processes can submit to it.  `perm_path`: file whose
  // mode admits peers to the request chunk (the store's descriptor).  Needs the VRAM request mode.
  int init_server(int device, uint32_t pstride, const std::string& seg, const std::string& perm_path,
                  const spl_arena_t& a);
  // Client of another process's (or this process's) ring server; no HIP call.  -1: no live server.
  int init_client(const std::string& seg, int device, uint32_t pstride);
  ~CmdRing();
  bool ready() const { return shared_ != nullptr; }
  bool shared_mode() const { return mode_ != kPrivate; }
  int mode() const { return (int)mode_; }  // 0 private, 1 ring server, 2 client of a server
  // whether call() will run this process's own worker on the arena passed to it (a client of a
  // live server passes nothing to the device)
  bool needs_arena() const { return mode_ != kClient || gone_.load(std::memory_order_acquire) || server_gone(); }
  // Blocking call: stage key / input, ring the doorbell, wait for DONE.  `in` may be null;
  // `out` (may be null) receives min(out_len, out_cap) payload bytes.  Returns 0 when the op ran
  // (its own status in r.status), -1 on a ring failure (errno set; e.g. ETIMEDOUT).
  // key64 must be canonical (KeyRef: NUL padded past klen) with its FNV-1a hash in khash.
  int call(const spl_arena_t& a, uint32_t op, uint32_t sub, const char key64[64], uint32_t klen, uint64_t khash,
           const void* in, uint32_t in_len, uint64_t arg, void* out, uint32_t out_cap, RingResult* r);
  void stop();
  void resume();  // after ring_hold(false): relaunch if calls wait
  // Store-level hold from any process attached to the store's ring (server, client or private):
  // the worker exits and is not relaunched until every hold is released.  0, or -1 (ETIMEDOUT) if
  // the worker did not exit within 10 s.
  int hold(bool on);
  uint32_t launches() const { return seg_ ? seg_->launches : shared_ ? shared_->launches : 0; }
  // ring server: stop and join the supervisor thread (the store's teardown does this BEFORE it
  // takes the quiesce gate, which the supervisor takes shared to relaunch a worker)
  void stop_supervisor();

 private:
  enum Mode { kPrivate, kServer, kClient };
  void launch(const spl_arena_t& a);
  void want_worker();        // client: ask the owner's supervisor for a worker
  bool server_gone() const;  // client: the owner closed the store or died
  void supervise();          // server: relaunch the worker when a client asks
  void reap_holds();         // take back the hold counts of holder processes that died
  int hold_slot(bool claim); // this process's slot in shared_->holds (-1: none / table full)
  int call_private(const spl_arena_t& a, uint32_t op, uint32_t sub, const char key64[64], uint32_t klen,
                   uint64_t khash, const void* in, uint32_t in_len, uint64_t arg, void* out, uint32_t out_cap,
                   RingResult* r);
  int alloc_host(size_t seg_bytes);
  Mode mode_ = kPrivate;
  // host side: host / device views (the same pointer in the private ring's pinned allocations)
  RingShared* shared_ = nullptr;  // worker control words (alive, stop)
  RingShared* d_shared_ = nullptr;
  RingCmd* cmds_ = nullptr;       // completion words (out_len) / the whole records (host mode)
  RingCmd* d_cmds_ = nullptr;
  uint8_t* payload_ = nullptr;    // output payloads, kRingEntries x pstride_
  uint8_t* d_payload_ = nullptr;
  RingDone* vdone_ = nullptr;     // VRAM mode completion chunks
  RingDone* d_vdone_ = nullptr;
  RingEntryCtl* ent_ = nullptr;   // entry ownership (own_ or the segment)
  uint32_t* ticket_ = nullptr;
  struct Own {
    RingEntryCtl ent[kRingEntries] = {};
    alignas(64) uint32_t ticket = 0;
  } own_;
  uint8_t* scratch_ = nullptr;    // device, kRingEntries x pstride_ (+64 key)
  uint32_t pstride_ = 0;
  int device_ = 0;
  int32_t pid_ = 0;
  uint64_t idle_ticks_ = 0;
  int clock_khz_ = 100000;
  bool spread_ = true;            // SPLINTER_RING_SPREAD: consecutive calls on different waves
  int groups_ = kDefaultRingGroups;  // worker waves
  uint64_t yield_after_us_ = 20;  // SPLINTER_RING_SPIN_US: spin this long, then yield between polls
  int cpus_ = 1;                  // CPUs the process may run on (affinity, cgroup quota)
  // VRAM request mode (SPLINTER_RING_VRAM=1): records, input payloads and sequence-number doorbells
  // in device memory written by the host through the BAR mapping of a VMM chunk; completions stay
  // in host memory (k_ring_worker<true>)
  bool vr_ = false;
  VmmArena vram_;
  RingCmd* v_cmds_h_ = nullptr;   // host (BAR) view
  uint32_t* v_door_h_ = nullptr;
  uint8_t* v_pay_h_ = nullptr;
  RingCmd* v_cmds_d_ = nullptr;   // device view
  uint32_t* v_door_d_ = nullptr;
  uint8_t* v_pay_d_ = nullptr;
  uint32_t* served_ = nullptr;    // device: last sequence number served per entry
  int init_vram();
  // shared segment (server / client)
  RingSegHdr* seg_ = nullptr;
  size_t seg_bytes_ = 0;
  std::string seg_name_;
  bool seg_registered_ = false;
  void* cmap_ = nullptr;          // client: BAR mapping of the owner's request chunk
  size_t cmap_bytes_ = 0;
  std::thread sup_;               // server: supervisor
  std::atomic<bool> sup_stop_{false};
  spl_arena_t arena_{};           // server: the arena its worker serves
  std::atomic<bool> gone_{false}; // client: the server went away; calls use priv_
  std::unique_ptr<CmdRing> priv_;
  std::mutex priv_mu_;
  int32_t waiters_own_ = 0;       // host threads of this process waiting on a completion right now
  int32_t* waiters_ = &waiters_own_;  // ... or of every process of a ring server (segment)
  long sleep_ns_ = 5000;          // SPLINTER_RING_SLEEP_NS: sleep between polls while oversubscribed
  long first_sleep_ns_ = 6000;    // SPLINTER_RING_FIRST_SLEEP_NS: the first of those sleeps (a call's bulk)
  uint64_t oversub_spin_us_ = 0;  // SPLINTER_RING_OVERSUB_SPIN_US: spin this long first while oversubscribed
  bool adaptive_ = true;          // SPLINTER_RING_ADAPTIVE_SLEEP: first sleep from the latency EWMA
  std::atomic<long> ewma_ns_{0};  // latency of recent oversubscribed calls
  uint8_t* ctrl_ = nullptr;       // device: {u64 last activity, u32 dying, u32 live waves}
  hipStream_t stream_ = nullptr;
  std::mutex launch_mu_;
  void read_env();
};

}  // namespace spl
