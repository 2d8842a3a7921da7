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
