// splinter_layout.hpp — format-v4 geometry shared by the host library, the
// HBM arena kernels and the tools.  Usable from host C++ and HIP device code.
//
// Byte layout (reference: /root/reference/splinter.h:126-255):
//   [header 5440 B][slots x stride][values: slots x max_val_sz]
//   stride = 128 (plain) or 3200 (128-B core + float[768] embedding).
#pragma once
#include <cstddef>
#include <cstdint>
#include "splinter.h"

#if defined(__HIPCC__) || defined(__HIP_DEVICE_COMPILE__)
#define SPL_HD __host__ __device__ __forceinline__
#else
#define SPL_HD inline
#endif

namespace spl {

constexpr uint32_t kMagic = SPLINTER_MAGIC;
constexpr uint32_t kVersion = SPLINTER_VER;
constexpr size_t kHeaderBytes = 5440;
constexpr size_t kSlotCoreBytes = 128;
constexpr size_t kEmbedDim = SPLINTER_EMBED_DIM;
constexpr size_t kEmbedBytes = kEmbedDim * sizeof(float);
constexpr size_t kSlotEmbedBytes = kSlotCoreBytes + kEmbedBytes;  // 3200
constexpr size_t kKeyMax = SPLINTER_KEY_MAX;
constexpr uint64_t kFnvOffset = 14695981039346656037ULL;
constexpr uint64_t kFnvPrime = 1099511628211ULL;
constexpr uint32_t kDirtyBits = SPLINTER_EVENT_BUS_MASK_WORDS * 64;

// slot core field offsets (bytes)
constexpr size_t kOffHash = 0, kOffEpoch = 8, kOffValOff = 16, kOffValLen = 20,
                 kOffType = 24, kOffUser = 25, kOffWatch = 32, kOffCtime = 40,
                 kOffAtime = 48, kOffBloom = 56, kOffKey = 64, kOffEmbed = 128;

// Side region of an HBM arena (not part of the v4 file format: runtime data of one allocation,
// never checkpointed, rebuilt on restore).  It follows the value area at a 4-KiB boundary:
//   [0, 4 KiB)            ArenaSide: probe-chain statistics written by the maintenance passes
//   nrm2 [slots] float    embedding stores only: squared norm of each slot's vector (0 = none)
//   vec16 [slots][768]    embedding stores only: the vector in bf16 (round to nearest even), the
//                         operand the batched search's candidate pass streams (half the bytes of
//                         the fp32 rows, contiguous); written under the slot's seqlock with the
//                         fp32 vector by every embedding writer
constexpr size_t kSideAlign = 4096;
constexpr size_t kSideHdrBytes = 4096;
constexpr size_t kVec16Bytes = kEmbedDim * 2;
SPL_HD size_t side_align_up(size_t v) { return (v + kSideAlign - 1) / kSideAlign * kSideAlign; }
// offset of the side region from the header, for a geometry
SPL_HD size_t side_offset(size_t slots, size_t stride, size_t max_val) {
  return side_align_up(kHeaderBytes + slots * stride + slots * max_val);
}
SPL_HD size_t side_nrm2_offset() { return kSideHdrBytes; }
SPL_HD size_t side_vec16_offset(size_t slots) { return kSideHdrBytes + side_align_up(slots * 4); }
SPL_HD size_t side_bytes(size_t slots, bool vec16) {
  return vec16 ? side_vec16_offset(slots) + slots * kVec16Bytes : kSideHdrBytes;
}

// probe-chain statistics (ArenaSide, and spl_hbm_probe_stats): a pass over the slot array
constexpr int kProbeBuckets = 12;  // probe lengths 1, 2, 3-4, 5-8, ..., 513-1024, > 1024
struct ProbeStats {
  uint64_t live;          // slots holding a key
  uint64_t tombstones;    // hash 0, even epoch != 0 (unset / reclaimed): lookups walk past them
  uint64_t virgin;        // hash 0, epoch 0: a chain ends here
  uint64_t busy;          // odd epoch (a writer in flight)
  uint64_t disp_sum;      // sum of (probe length of a hit) over live keys
  uint64_t disp_max;
  uint64_t miss_sum;      // sum over home positions of the probe length of a miss (to the next virgin)
  uint64_t miss_max;
  uint64_t hist[kProbeBuckets];  // live keys by probe length of a hit
  uint64_t rebuilds;      // spl_hbm_rehash passes run on this arena
  uint64_t reclaimed;     // tombstones turned back into virgin slots (purge / rehash)
  uint64_t moved;         // keys moved toward their home slot (rehash)
  uint64_t pad[1];
};
static_assert(sizeof(ProbeStats) % 16 == 0, "16-B rows");

// Online maintenance record, at kSideMaintOff of the side header (its own 128-B line, past the
// ProbeStats block the host rewrites): `seq` is odd while a maintenance pass moves entries
// (arena_maint.hip k_rehash), `pid` / `t0_ns` name the process that opened the pass, so a pass
// whose process died can be closed by the next one (HbmStore::rehash).  Device probes read `seq`
// around every "absent" outcome (arena_dev.hpp maint_quiet).
constexpr size_t kSideMaintOff = 256;
struct MaintRec {
  uint64_t seq;
  int32_t pid;
  uint32_t pad;
  uint64_t t0_ns;
  uint64_t passes;  // passes completed
};
static_assert(kSideMaintOff >= sizeof(ProbeStats) && kSideMaintOff % 128 == 0, "maint record line");

static_assert(sizeof(splinter_header) == kHeaderBytes, "v4 header must be 5440 B");
static_assert(alignof(splinter_header) == 64, "header alignment");
static_assert(sizeof(splinter_slot) == kSlotCoreBytes, "slot core must be 128 B");
static_assert(alignof(splinter_slot) == 64, "slot alignment");
static_assert(offsetof(splinter_header, epoch) == 16, "layout");
static_assert(offsetof(splinter_header, core_flags) == 24, "layout");
static_assert(offsetof(splinter_header, val_brk) == 28, "layout");
static_assert(offsetof(splinter_header, alignment) == 36, "layout");
static_assert(offsetof(splinter_header, bloom_watches) == 56, "layout");
static_assert(offsetof(splinter_header, signal_groups) == 128, "layout");
static_assert(offsetof(splinter_header, event_bus) == 4224, "layout");
static_assert(offsetof(splinter_header, shard_bids) == 4416, "layout");
static_assert(sizeof(splinter_shard_bid) == 32, "bid record is 32 B");
static_assert(offsetof(splinter_slot, epoch) == kOffEpoch, "layout");
static_assert(offsetof(splinter_slot, val_len) == kOffValLen, "layout");
static_assert(offsetof(splinter_slot, watcher_mask) == kOffWatch, "layout");
static_assert(offsetof(splinter_slot, bloom) == kOffBloom, "layout");
static_assert(offsetof(splinter_slot, key) == kOffKey, "layout");
static_assert(sizeof(splinter_header_snapshot_t) == 48, "snapshot ABI");
#ifdef SPLINTER_EMBEDDINGS
static_assert(sizeof(splinter_slot_snapshot_t) == 3192, "slot snapshot ABI");
#endif

SPL_HD uint64_t fnv1a(const char* s) {
  uint64_t h = kFnvOffset;
  while (*s) { h ^= (unsigned char)*s++; h *= kFnvPrime; }
  return h;
}

SPL_HD uint64_t fnv1a_n(const char* s, size_t n) {
  uint64_t h = kFnvOffset;
  for (size_t i = 0; i < n && s[i]; ++i) { h ^= (unsigned char)s[i]; h *= kFnvPrime; }
  return h;
}

struct Geometry {
  uint32_t slots = 0;
  uint32_t max_val = 0;
  uint32_t stride = kSlotCoreBytes;   // 128 or 3200
  SPL_HD bool embeddings() const { return stride == kSlotEmbedBytes; }
  SPL_HD size_t slots_bytes() const { return (size_t)slots * stride; }
  SPL_HD size_t values_bytes() const { return (size_t)slots * max_val; }
  SPL_HD size_t total_bytes() const { return kHeaderBytes + slots_bytes() + values_bytes(); }
  SPL_HD size_t slot_offset(size_t i) const { return kHeaderBytes + i * stride; }
  SPL_HD size_t values_offset() const { return kHeaderBytes + slots_bytes(); }
};

// Infer the slot stride of an existing region from its byte size.  Returns 0
// when neither stride reproduces `total` exactly.
SPL_HD uint32_t infer_stride(uint32_t slots, uint32_t max_val, size_t total) {
  if (slots == 0) return 0;
  const size_t core = kHeaderBytes + (size_t)slots * max_val;
  if (total == core + (size_t)slots * kSlotCoreBytes) return (uint32_t)kSlotCoreBytes;
  if (total == core + (size_t)slots * kSlotEmbedBytes) return (uint32_t)kSlotEmbedBytes;
  return 0;
}

}  // namespace spl
