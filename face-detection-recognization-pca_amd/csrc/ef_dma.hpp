// LDS-DMA helpers (global_load_lds) shared by the streaming kernels.
#pragma once

#include <hip/hip_runtime.h>

namespace ef {

// LDS-DMA (global_load_lds) in inline asm: hipcc would otherwise treat the pending DMA
// as an aliasing LDS write and put s_waitcnt vmcnt(0) before every ds_read, serialising the
// prefetch of tile t+1 with the MFMAs of tile t.  M0 (the wave-uniform LDS destination) is
// written and restored inside the statement; completion is waited for explicitly with
// s_waitcnt vmcnt(0) before the barrier that publishes the tile.
__device__ __forceinline__ unsigned lds_addr(const void* p) {  // wave-uniform by construction
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)p);
}
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
// SGPR-base forms: global address = sbase (wave-uniform, 64-bit) + voff (per lane, 32-bit
// byte offset) — no per-lane 64-bit address arithmetic.
__device__ __forceinline__ unsigned long long uniform_ptr(const void* p) {
  const unsigned long long v = (unsigned long long)(size_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ void glds16s(unsigned voff, unsigned long long sbase, unsigned lds) {
  sbase = uniform_ptr((const void*)sbase);  // pin to SGPRs (hipcc may otherwise spill it to a VGPR)
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(sbase) : "memory");
}
__device__ __forceinline__ void glds4s(unsigned voff, unsigned long long sbase, unsigned lds) {
  sbase = uniform_ptr((const void*)sbase);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, %3\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds), "s"(sbase) : "memory");
}
// Two half-wave DMAs from one address register: lanes 0-31 land at m0a + 16*lane, lanes
// 32-63 at m0b + 16*lane — i.e. two rows placed anywhere in LDS (padded row strides),
// each half written by its own exec-masked instruction.  EXEC and M0 are restored.
__device__ __forceinline__ void glds16s_halves(unsigned voff, unsigned long long sbase, unsigned m0a, unsigned m0b) {
  sbase = uniform_ptr((const void*)sbase);
  unsigned long long sexec;
  unsigned keep;
  asm volatile(
      "s_mov_b64 %0, exec\n\ts_mov_b32 %1, m0\n\t"
      "s_mov_b32 exec_hi, 0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
      "s_mov_b64 exec, %0\n\ts_mov_b32 exec_lo, 0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
      "s_mov_b64 exec, %0\n\ts_mov_b32 m0, %1"
      : "=&s"(sexec), "=&s"(keep)
      : "v"(voff), "s"(m0a), "s"(m0b), "s"(sbase)
      : "memory");
}
__device__ __forceinline__ void glds16_halves(const void* gsrc, unsigned m0a, unsigned m0b) {
  unsigned long long sexec;
  unsigned keep;
  asm volatile(
      "s_mov_b64 %0, exec\n\ts_mov_b32 %1, m0\n\t"
      "s_mov_b32 exec_hi, 0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\t"
      "s_mov_b64 exec, %0\n\ts_mov_b32 exec_lo, 0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\t"
      "s_mov_b64 exec, %0\n\ts_mov_b32 m0, %1"
      : "=&s"(sexec), "=&s"(keep)
      : "v"(gsrc), "s"(m0a), "s"(m0b)
      : "memory");
}
__device__ __forceinline__ void dma_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace ef
