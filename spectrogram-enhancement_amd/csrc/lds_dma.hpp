// lds_dma.hpp — LDS-DMA (global_load_lds) issued so the compiler leaves its completion to
// the kernel (conv_rows.hip, decoder_tail.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace specenh {

// one 16-byte LDS-DMA per lane: LDS destination = wave-uniform dst + 16 x lane. Issued as
// inline asm: with __builtin_amdgcn_global_load_lds the compiler knows the load writes LDS
// and puts s_waitcnt vmcnt(0) before the next LDS access — every step then waited for the
// DMA it had just issued (the whole HBM latency), defeating the ring. The kernel counts
// these loads itself (its vmcnt waits and barriers are volatile asm with a memory clobber,
// and the DMA, also volatile, is not moved across them); an op the compiler does not know
// about only makes the compiler's own vmcnt waits stricter. No "memory" clobber on the DMA
// itself: with one, the waitcnt pass again put vmcnt(0) before the next LDS access.
// s_nop 0: the wait state between an M0 write and an LDS-DMA.
__device__ __forceinline__ void lds_dma16(const void* src, void* dst) {
  const unsigned m0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)dst;
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(m0)
               : "m0");
}

}  // namespace specenh
