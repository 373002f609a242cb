// Diagnostic s_memtime phase stamps of the hot conv loops (conv3w.hip, conv3w_a8.hip, conv64.hip), read by
// tools/diag_c3w_stamps.py and tools/diag_c64_stamps.py. Only a diagnostic build stamps (-DGT_C3W_STAMP=1,
// -DGT_C3W8_STAMP=1, -DGT_C64_STAMP=1, each for one instantiation): in the product build a kernel's Stamps<false> has
// no state and every call below is an empty inline function, so the kernels carry one-line calls and no stamp code
// (the product listings are unchanged by them).
#pragma once
#include "common.h"

namespace gt {

// 8 counters per wave: what each counter means is the kernel's (its comment at GT_STAMP_BUFFER); flush() stores them
// from lanes 0..7 with vector stores into dst[(slot * nwave + wave) * 8 + counter]. `live`: a run-time condition on top
// of the compile-time one (conv64 stamps only its F = 80 launches).
template <bool ON>
struct Stamps {
  GT_DEV explicit Stamps(bool = true) {}
  GT_DEV unsigned long long now() const { return 0ull; }
  template <class... X>
  GT_DEV unsigned long long now_after(const X&...) const { return 0ull; }
  GT_DEV void add(int, unsigned long long) {}
  GT_DEV void set(int, unsigned long long) {}
  GT_DEV void flush(unsigned long long*, int, int, int, int) const {}
};

template <class X>
GT_DEV void retired(const X& x) { asm volatile("" ::"v"(x)); }   // x's value exists past this point

template <>
struct Stamps<true> {
  bool on;
  unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  GT_DEV explicit Stamps(bool live = true) : on(live) {}
  GT_DEV unsigned long long now() const { return on ? __builtin_amdgcn_s_memtime() : 0ull; }
  // a stamp taken once the values x exist (else it would read the issue time of the instructions producing them)
  template <class... X>
  GT_DEV unsigned long long now_after(const X&... x) const {
    (retired(x), ...);
    return now();
  }
  GT_DEV void add(int i, unsigned long long d) { st[i] += d; }
  GT_DEV void set(int i, unsigned long long v) { st[i] = v; }
  GT_DEV void flush(unsigned long long* dst, int slot, int nwave, int wave, int lane) const {
    if (!on) return;
    unsigned long long v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v = lane == i ? st[i] : v;
    if (lane < 8) dst[(slot * nwave + wave) * 8 + lane] = v;
  }
};

}  // namespace gt

// The stamp buffer [workgroup slot 0..511][wave 0..NWAVE-1][counter 0..7] of one kernel and its host accessor
// (extern "C" int ACCESSOR(unsigned long long* out, long n)); a kernel defines it under its diagnostic switch.
#define GT_STAMP_BUFFER(SYM, ACCESSOR, NWAVE)                                                                 \
  __device__ unsigned long long SYM[512 * (NWAVE) * 8];                                                       \
  extern "C" int ACCESSOR(unsigned long long* out, long n) {                                                  \
    if (n > 512 * (NWAVE) * 8) n = 512 * (NWAVE) * 8;                                                         \
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(SYM), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1; \
  }
