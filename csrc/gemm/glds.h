// LDS-DMA helper shared by the GEMM kernels.
#pragma once
#include "common/hip_common.h"

namespace fan {

// 16 bytes per lane global -> LDS (global_load_lds_dwordx4), LDS destination = wave-uniform base + lane*16.
// Issued from inline asm so hipcc does not track it: otherwise its waitcnt pass conservatively inserts
// s_waitcnt vmcnt(0) in front of LDS fragment reads (observed in front of ds_read_b64_tr_b16), draining the
// prefetch every K-tile. Completion is counted by hand with s_waitcnt vmcnt(N) + a raw s_barrier.
// M0 is set inside the same statement and not restored (cdna_hip_programming.md §5.7's clobbering form; the compiler
// emits no M0 access of its own in these kernels: see glds16_s in gemm_bf16_kernel.h).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_addr) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

}  // namespace fan
