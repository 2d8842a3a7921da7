// route_kernels.hip — device side of the routed exchange (SURVEY §2.10 C1, §2.13;
// parallel/xroute.py): pack a client batch straight into the owners' request blocks, gather the
// owners' responses back into client order, and the exchange windows those blocks live in.
//
// One exchange per direction per step.  Every (requester r, owner o) pair has ONE request block
// in o's window -- [set keys | set lens | set value prefixes | get keys], `cap` rows per kind --
// and ONE response block in r's window -- [set status | get status | get lens | get values].
// The pack kernel writes each remote op's record directly into its owner's block: on the peer
// transport that block is the owner's own window mapped into this process (VMM dmabuf import,
// xGMI stores from the pack kernel: no copy kernel and no collective moves the bytes); on the
// RCCL transport it is this rank's send staging block for o, moved by ONE all-to-all.  Ops whose
// owner is this rank never enter the exchange: the pack kernel only lists their client indices
// (`lidx`) and the owner kernels run them in place on the client arrays (arena_kernels.hip Seg.idx).
// The per-destination counts are the only thing a collective must carry (they double as the
// step's cross-rank ordering point).
//
// Fixed capacity per block: an op whose block is full returns EAGAIN (the reference's retry
// status, splinter.h:398-412); route_capacity() makes that < 1e-15 per block for hashed keys.
//
// pos[i] (int32): d * cap + j for a remote op in row j of owner d's block, kPosOwn for an own
// op (its results are written in place), kPosFull for an op that found its block full.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

#include "arena_dev.hpp"
#include "arena_api.h"
#include "vmm_share.hpp"

using namespace spl;
using namespace spl::dev;

namespace {

constexpr int kRB = 256;         // threads per block
constexpr int kRU = 4;           // items per thread per round
constexpr int kMaxWorld = 64;    // destinations of the LDS histogram (== kNodeMaxShards)
constexpr int32_t kPosOwn = -2, kPosFull = -1;

__device__ __forceinline__ int shard_of_hash(uint64_t h, int world) {
  return (int)(((h >> 40) & 0xFFFFFFull) % (uint64_t)world);  // == parallel/sharded.py shard_of
}

// One routed kind of a pack: where its rows go inside a destination block.
struct XKind {
  long off_k, off_l, off_v;  // byte offsets of keys / lens / value rows in a block (off_l, off_v: sets)
  int vw;                    // value bytes per row (16-B multiple; 0: no values)
  long off_p;                // direct responses: the client-index column (<= 0: none)
};

__global__ __launch_bounds__(kRB) void k_xpack(const char* keys, int ks, const uint8_t* vals, int vstride,
                                               const uint32_t* lens, long n, int world, int rank, long cap,
                                               const uint64_t* blk, XKind kd, int32_t* counts, int32_t* lidx,
                                               int32_t* pos, int32_t* full_status, uint32_t* full_lens) {
  __shared__ int s_cnt[kMaxWorld];
  __shared__ int s_base[kMaxWorld];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long per_round = (long)kRB * kRU;
  for (int d = tid; d < world; d += kRB) s_cnt[d] = 0;
  __syncthreads();
  for (long base = blockIdx.x * per_round; base < n; base += (long)gridDim.x * per_round) {
    Key k[kRU];
    int dst[kRU], rk[kRU];
#pragma unroll
    for (int j = 0; j < kRU; ++j) {
      const long i = base + (long)j * kRB + tid;
      dst[j] = -1;
      if (i < n) {
        load_key(k[j], keys + i * (long)ks, ks);
        dst[j] = shard_of_hash(k[j].hash, world);
        rk[j] = atomicAdd(&s_cnt[dst[j]], 1);
      }
    }
    __syncthreads();
    for (int d = tid; d < world; d += kRB) {
      const int c = s_cnt[d];
      s_base[d] = c ? atomicAdd(&counts[d], c) : 0;
      s_cnt[d] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRU; ++j) {
      const long i = base + (long)j * kRB + tid;
      long row = -1;  // row in the destination block (remote ops only)
      uint8_t* b = nullptr;
      if (dst[j] >= 0) {
        const long slot = (long)s_base[dst[j]] + rk[j];
        int32_t p = kPosFull;
        if (slot < cap) {
          if (dst[j] == rank) {
            lidx[slot] = (int32_t)i;
            p = kPosOwn;
          } else {
            p = (int32_t)(dst[j] * cap + slot);
            row = slot;
            b = (uint8_t*)blk[dst[j]];
          }
        }
        pos[i] = p;
        if (p == kPosFull && full_status) {  // direct responses: no gather will mark it
          full_status[i] = kAgain;
          if (full_lens) full_lens[i] = 0u;
        }
      }
      if (row >= 0) {
        uint4* kr = (uint4*)(b + kd.off_k + row * (long)ks);
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c * 16 < ks) kr[c] = make_uint4(k[j].w[4 * c], k[j].w[4 * c + 1], k[j].w[4 * c + 2], k[j].w[4 * c + 3]);
        if (kd.vw) *(uint32_t*)(b + kd.off_l + row * 4) = lens[i];
        if (kd.off_p > 0) *(int32_t*)(b + kd.off_p + row * 4) = (int32_t)i;
      }
      if (kd.vw) {
        // value prefixes, wave-cooperatively: the wave's 64 rows of this item index, lanes walk the
        // flattened (row, 16-B chunk) space so reads and writes of consecutive lanes are contiguous
        const long w0 = base + (long)j * kRB + wave * 64;
        const long left = n - w0;
        const uint64_t my_dst = row >= 0 ? (uint64_t)(b + kd.off_v + row * (long)kd.vw) : 0ull;
        if (left > 0) {
          const int C = kd.vw / 16, nvalid = left < 64 ? (int)left : 64;
          for (int c = lane; c < 64 * C; c += 64) {
            const int r = c / C, ch = c - r * C;
            const uint64_t dp = __shfl(my_dst, r);
            if (r < nvalid && dp)
              *(uint4*)(dp + ch * 16) = *(const uint4*)(vals + (w0 + r) * (long)vstride + ch * 16);
          }
        }
      }
    }
  }
}

// Responses back into client order.  blk[d]: the response block owner d filled (in this rank's
// window, or its receive area); off_s / off_l / off_v: status, lens, value rows inside it.
__global__ __launch_bounds__(kRB) void k_xgather(const int32_t* pos, long n, long cap, const uint64_t* blk, long off_s,
                                                 long off_l, long off_v, int vw, int32_t* status, uint32_t* out_lens,
                                                 uint8_t* out, int ostride, int copy_bytes) {
  const int lane = threadIdx.x & 63;
  const long wstep = (long)gridDim.x * kRB;
  for (long w0 = blockIdx.x * (long)kRB + (threadIdx.x & ~63); w0 < n; w0 += wstep) {
    const long i = w0 + lane;
    uint64_t src = 0;
    if (i < n) {
      const int32_t p = pos[i];
      if (p == kPosFull) {
        status[i] = kAgain;
        if (out_lens) out_lens[i] = 0u;
      } else if (p >= 0) {
        const long d = p / cap, j = p - d * cap;
        const uint8_t* b = (const uint8_t*)blk[d];
        const int32_t st = *(const int32_t*)(b + off_s + j * 4);
        status[i] = st;
        if (out_lens) out_lens[i] = st == kOk ? *(const uint32_t*)(b + off_l + j * 4) : 0u;
        if (out && st == kOk) src = (uint64_t)(b + off_v + j * (long)vw);
      }
    }
    if (out) {
      const int C = copy_bytes / 16;
      const long left = n - w0;
      const int nvalid = left < 64 ? (int)left : 64;
      for (int c = lane; c < 64 * C; c += 64) {
        const int r = c / C, ch = c - r * C;
        const uint64_t sp = __shfl(src, r);
        if (r < nvalid && sp) *(uint4*)(out + (w0 + r) * (long)ostride + ch * 16) = *(const uint4*)(sp + ch * 16);
      }
    }
  }
}

inline int route_grid(long n, long per_block) {
  long g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > 256 * 8) g = 256 * 8;
  return (int)g;
}

// ------------------------------------------------------- device-side step ordering --
// The flag area at the end of every window (parallel/xroute.py XGeom.off_flag) orders a step
// without a collective (SPLINTER_XR_SYNC=flags): a requester posts -- after its pack kernel, stream
// order -- its per-kind row counts and then flag[parity][0][its rank] = seq into every owner's
// window; an owner's one-workgroup wait kernel polls its own flags until every peer's seq has
// arrived, and the owner grid behind it reads the counts.  Responses likewise (dir 1, no counts).
// Every flag slot has one writer (its source rank) whose posts are stream-ordered, so "flag >= seq"
// means "this step's post has landed".  Waits are bounded (s_memrealtime, 100 MHz): a post that never
// comes sets *err and the wait kernel ends, so no grid is left spinning.
constexpr int kXfFlagBytes = 2 * 2 * kMaxWorld * 8;  // [parity][dir][source] uint64
// counts follow: [parity][source][kind] int32

__global__ void k_xr_post(const uint64_t* flag_blk, int world, int rank, int par, int dir, uint64_t seq,
                          const int32_t* counts) {
  const int d = (int)threadIdx.x;
  if (d >= world || d == rank) return;
  uint8_t* f = (uint8_t*)flag_blk[d];
  if (counts) {  // counts[kind * world + d]: this rank's rows for owner d
    int32_t* c = (int32_t*)(f + kXfFlagBytes) + (par * kMaxWorld + rank) * 2;
    __hip_atomic_store(c, counts[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(c + 1, counts[world + d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  uint64_t* fl = (uint64_t*)f + (par * 2 + dir) * kMaxWorld + rank;
  __hip_atomic_store(fl, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_xr_wait(const uint8_t* own, int world, int rank, int par, int dir, uint64_t seq, uint64_t ticks,
                          uint32_t* err) {
  const int src = (int)threadIdx.x;
  if (src >= world || src == rank) return;
  const uint64_t* fl = (const uint64_t*)own + (par * 2 + dir) * kMaxWorld + src;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(fl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

}  // namespace

extern "C" {

// Device-side ordering of a routed step (see k_xr_post): post into every peer's flag area
// (flag_blk: device table of the `world` windows' flag-area addresses; counts: the pack counts
// [2][world] for dir 0, null for dir 1), or wait for every peer's post in this rank's own area.
int spl_xr_post(const uint64_t* flag_blk, int world, int rank, int par, int dir, uint64_t seq, const int32_t* counts,
                hipStream_t s) {
  if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world || (par & ~1) || (dir & ~1))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_xr_post, dim3(1), dim3(kMaxWorld), 0, s, flag_blk, world, rank, par, dir, seq, counts);
  return (int)hipGetLastError();
}

int spl_xr_wait(const void* own_flags, int world, int rank, int par, int dir, uint64_t seq, uint64_t timeout_ms,
                uint32_t* err, hipStream_t s) {
  if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world || (par & ~1) || (dir & ~1) || !err)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_xr_wait, dim3(1), dim3(kMaxWorld), 0, s, (const uint8_t*)own_flags, world, rank, par, dir, seq,
                     timeout_ms * 100000ull, err);
  return (int)hipGetLastError();
}

// Bytes of the flag area (flags + counts) a window reserves for the device-side ordering.
long spl_xr_flag_bytes(void) { return kXfFlagBytes + 2L * kMaxWorld * 2 * 4; }

// Pack one batch kind (sets: vals/lens/vw given; gets: vals = lens = null, vw = 0).  counts[world]
// is zeroed here and accumulates every destination's rows, the own destination included (its rows
// are lidx entries).  blk: device table of `world` block base pointers (the own entry is unused).
int spl_xr_pack(const char* keys, int ks, const uint8_t* vals, int vstride, const uint32_t* lens, long n, int world,
                int rank, long cap, const uint64_t* blk, long off_k, long off_l, long off_v, int vw, int32_t* counts,
                int32_t* lidx, int32_t* pos, long off_p, int32_t* full_status, uint32_t* full_lens, hipStream_t s) {
  if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world || cap < 0) return (int)hipErrorInvalidValue;
  if ((ks & 15) || ks <= 0 || ks > 64 || (off_k & 15)) return (int)hipErrorInvalidValue;
  if (vw && (!vals || !lens || (vstride & 15) || (vw & 15) || vw > vstride || (off_v & 15) || (off_l & 3)))
    return (int)hipErrorInvalidValue;
  if (cap * (long)world > INT32_MAX || n > INT32_MAX || (off_p > 0 && (off_p & 3))) return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(counts, 0, sizeof(int32_t) * (size_t)world, s);
  if (e != hipSuccess) return (int)e;
  if (n <= 0) return 0;
  const XKind kd{off_k, off_l, off_v, vw, off_p};
  hipLaunchKernelGGL(k_xpack, dim3(route_grid(n, (long)kRB * kRU)), dim3(kRB), 0, s, keys, ks, vals, vstride, lens, n,
                     world, rank, cap, blk, kd, counts, lidx, pos, off_p > 0 ? full_status : nullptr,
                     off_p > 0 ? full_lens : nullptr);
  return (int)hipGetLastError();
}

// Gather one batch kind's responses (gets: out / out_lens given; sets: status only).
int spl_xr_gather(const int32_t* pos, long n, long cap, const uint64_t* blk, long off_s, long off_l, long off_v, int vw,
                  int32_t* status, uint32_t* out_lens, uint8_t* out, int ostride, hipStream_t s) {
  if (n <= 0) return 0;
  const int copy = out ? (vw < ostride ? vw : ostride) : 0;
  if (out && ((vw & 15) || (ostride & 15) || copy <= 0 || (off_v & 15) || !out_lens)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_xgather, dim3(route_grid(n, kRB)), dim3(kRB), 0, s, pos, n, cap, blk, off_s, off_l, off_v, vw,
                     status, out_lens, out, ostride, copy);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- exchange windows --
// A rank's window is device memory other ranks of the node map into their own address space: HIP
// virtual-memory chunks exported as dmabuf descriptors (vmm_share.hpp, the same machinery as the
// shareable HBM arenas), handed to peers over an abstract UNIX socket named after the window.  An
// attached window is the peer's memory mapped for THIS process's device: on another GPU the
// mapping is an xGMI peer mapping, so this device's kernels store into it directly.

void* spl_xw_create(int device, size_t bytes, const char* name) {
  if (!name || !bytes || hipSetDevice(device) != hipSuccess) return nullptr;
  auto* w = new VmmArena();
  if (w->create(device, bytes, (size_t)256 << 20) != 0 || w->serve(name) != 0) {
    delete w;
    return nullptr;
  }
  return w;
}

void* spl_xw_attach(const char* name, int device) {
  if (!name || hipSetDevice(device) != hipSuccess) return nullptr;
  std::vector<int> fds;
  size_t chunk = 0;
  if (VmmArena::fetch(name, &fds, &chunk) != 0) return nullptr;
  auto* w = new VmmArena();
  if (w->import(device, fds, chunk) != 0) {
    delete w;
    return nullptr;
  }
  return w;
}

void* spl_xw_base(void* h) { return h ? ((VmmArena*)h)->base() : nullptr; }
size_t spl_xw_bytes(void* h) { return h ? ((VmmArena*)h)->chunk() * ((VmmArena*)h)->chunks() : 0; }

void spl_xw_destroy(void* h) { delete (VmmArena*)h; }

// Direct access from `device` to memory on `peer` (xGMI): 0 when usable (already enabled counts),
// else the HIP error.  Same device: 0.
int spl_xw_peer(int device, int peer) {
  if (device == peer) return 0;
  int can = 0;
  hipError_t e = hipDeviceCanAccessPeer(&can, device, peer);
  if (e != hipSuccess) return (int)e;
  if (!can) return (int)hipErrorPeerAccessUnsupported;
  if ((e = hipSetDevice(device)) != hipSuccess) return (int)e;
  e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return 0;
  }
  return (int)e;
}

}  // extern "C"
