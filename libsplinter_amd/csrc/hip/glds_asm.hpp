// glds_asm.hpp — one 16-B-per-lane LDS-DMA (global_load_lds_dwordx4) issued from inline asm.
//
// Why not __builtin_amdgcn_global_load_lds: with builtin LDS-DMAs inside a K loop, hipcc's wait
// insertion stops counting LDS reads and puts `s_waitcnt lgkmcnt(0)` in front of every MFMA group that
// consumes fragment reads (checked in the .s of k_gemm256 and k_gemm_rln), so each phase's MFMAs wait
// for ALL of its ds_reads instead of the first few.  Hidden in asm, the DMA leaves the compiler's
// LDS-read accounting alone (counted lgkmcnt(N) again).  The kernels already order these DMAs with their
// own counted `s_waitcnt vmcnt` + barriers, exactly as for the builtin.  M0 (the DMA's LDS base) is saved
// and restored around the issue, so no compiler-owned M0 value is lost; `s_nop 0` covers the
// M0-write -> LDS-DMA hazard (the wait state hipcc itself inserts there).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace spl {
__device__ __forceinline__ void glds16_asm(const void* gsrc, const void* lds_dst) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  uint32_t save;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(save)
               : "v"(gsrc), "s"(l)
               : "memory");
}
}  // namespace spl
