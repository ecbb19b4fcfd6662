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
__device__ __forceinline__ void dma_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace ef
