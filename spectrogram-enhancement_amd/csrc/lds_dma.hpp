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

// The same DMA from a wave-uniform base address (SGPR pair) + a 32-bit per-lane byte offset
// (the global instruction's saddr form): no 64-bit per-lane address register to keep live
// across a loop (enc2_rows_kernel spilled one, and the spill reload's vmcnt(0) then waited for
// every DMA in flight each step).
__device__ __forceinline__ void lds_dma16_s(const void* sbase, unsigned voff, void* dst) {
  const unsigned m0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)dst;
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :
               : "v"(voff), "s"(sbase), "s"(m0)
               : "m0");
}

// one 8-byte global store per lane as exactly ONE vector-memory instruction, so a kernel that
// keeps a ledger of its own vector-memory ops (vmcnt counts stores as well as loads on gfx9)
// knows how many were issued after a given DMA
__device__ __forceinline__ void gstore8(void* dst, uint2 v) {
  asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(dst), "v"(v) : "memory");
}

// The launch-resident fragments (weights, biases) loaded before a step loop have landed:
// s_waitcnt vmcnt(0) as the builtin, which the compiler's wait insertion sees. Without it the
// compiler puts its wait for those loads at their first use INSIDE the loop, where it runs
// every step and drains every LDS-DMA and store in flight (vmcnt counts both on gfx9).
__device__ __forceinline__ void resident_loads_landed() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// s_waitcnt vmcnt(n) for a wave-uniform run-time n: wait until at most n of this wave's
// vector-memory ops are outstanding (n > 15 waits as for 15: stricter, never laxer)
__device__ __forceinline__ void wait_vmcnt(int n) {
  // (readfirstlane: the count is wave-uniform, but the compiler cannot always prove it and
  // then compiled the switch into a ladder of VALU compares)
  switch (__builtin_amdgcn_readfirstlane(n)) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}

// wait_vmcnt with the loop's steady-state count as a compile-time fast path: n >= STEADY waits
// with vmcnt(STEADY) (stricter for n > STEADY, never laxer) in two scalar instructions instead
// of the switch's compare ladder
template <int STEADY>
__device__ __forceinline__ void wait_vmcnt_ss(int n) {
  static_assert(STEADY >= 0 && STEADY <= 15, "vmcnt is 4 bits on gfx9");
  if (__builtin_amdgcn_readfirstlane(n) >= STEADY)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(STEADY) : "memory");
  else
    wait_vmcnt(n);
}

}  // namespace specenh
