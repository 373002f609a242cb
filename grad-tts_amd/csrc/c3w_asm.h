// Inline-asm memory and wait helpers shared by the wide-tile 3x3 convolutions (conv3w.hip, conv3w_a8.hip).
#pragma once
#include "common.h"

namespace gt {

typedef unsigned u32x4c_t __attribute__((ext_vector_type(4)));

template <int N>
GT_DEV void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }
// counted wait that names the registers of an asm load (they are written when it retires)
template <int N>
GT_DEV void vm_wait_dep(u32x4c_t& x) { asm volatile("s_waitcnt vmcnt(%1)" : "+v"(x) : "n"(N) : "memory"); }
template <int N>
GT_DEV void vm_wait_dep2(u32x4c_t& x, u32x4c_t& y) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(x), "+v"(y) : "n"(N) : "memory");
}
// LDS DMA (1 KiB per wave instruction) hidden from hipcc's waitcnt bookkeeping: hipcc models its builtin twin as an LDS
// access too and then waits lgkmcnt(0) in front of the fragment reads that follow it. M0 is written and restored in the
// same statement (guide §5.7). Scalar base + one per-lane 32-bit offset register (the saddr form) for every DMA of the
// kernel, where a 64-bit per-lane address per slot used to be held: 2-4 fewer VGPRs, no spill in the 256-wide GN form.
GT_DEV void asm_dma16(const void* sbase, unsigned voff, unsigned lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_addr) : "memory");
}
GT_DEV void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }
// raw buffer load hidden from hipcc's waitcnt bookkeeping (the s_nop covers an SGPR operand written just before)
GT_DEV void asm_buffer_load(u32x4c_t& dst, int voff, __amdgpu_buffer_rsrc_t rs, int soff) {
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(dst) : "v"(voff), "s"(rs), "s"(soff) : "memory");
}
// two consecutive 16-B pieces (bytes [voff, voff + 32)): two loads, both counted by vmcnt
GT_DEV void asm_buffer_load2(u32x4c_t& d0, u32x4c_t& d1, int voff, __amdgpu_buffer_rsrc_t rs, int soff) {
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %2, %3, %4 offen\n\tbuffer_load_dwordx4 %1, %2, %3, %4 offen offset:16"
               : "=&v"(d0), "=&v"(d1) : "v"(voff), "s"(rs), "s"(soff) : "memory");
}

}  // namespace gt
