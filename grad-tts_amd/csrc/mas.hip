// Monotonic Alignment Search on gfx950 -- bit-exact replacement of model/monotonic_align/core.pyx.
//
// Reference (core.pyx:9-35, generated C core.c:2653-2940), per utterance:
//   forward  for y < t_y, x in [max(0, t_x+y-t_y), min(t_x, y+1)):
//              v_cur  = (x == y) ? NEG : V[x, y-1];  v_prev = (x == 0) ? (y == 0 ? 0 : NEG) : V[x-1, y-1]
//              V[x, y] = ((v_prev > v_cur) ? v_prev : v_cur) + V[x, y]          (one fp32 max + one fp32 add)
//   backtrack idx = t_x-1; for y = t_y-1..0: P[idx, y] = 1;
//              if idx != 0 && (idx == y || V[idx, y-1] < V[idx-1, y-1]) idx -= 1
// Column y depends only on column y-1, so the DP runs column-parallel: ONE wave per utterance, lane L
// owns rows x = L*XPL .. L*XPL+XPL-1 in registers; the only cross-lane traffic per column is the
// neighbour's last row (one shuffle). The backtrack needs only the comparison V[x,y-1] < V[x-1,y-1] that
// the forward already evaluates for in-band cells, so the forward stores one "step down" bit per cell
// (in LDS, XPL bits per lane per column) instead of the fp32 DP table. Both steps use exactly the
// reference's fp32 operations in the same order -> bit-identical paths.
// The {0,1} path tensor is then written by a separate full-bandwidth kernel from the per-column row
// index (t_y ints per utterance).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "gradtts.h"

namespace {

// MODE bits (A/B via GT_MAS_MODE; default 53 = 1|4|16|32, measured 1.9x (b=32, 200x800) and 2.2x (ragged
// training batch) faster than MODE 0, the first version, on the same box; bench_mas.py):
//   1  the neighbour row arrives by DPP wave_shr:1 (a VALU op) instead of ds_bpermute
//   2  deeper register prefetch of the value columns (measured slower; kept for A/B only)
//   4  windowed backtrack: 64 columns per LDS round trip instead of one dependent LDS read per column
//  16  lean row update: every row updated unconditionally, one compare serves the max and the step bit
//  32  16-byte value loads (4 columns of a row per load instruction)
template <int XPL, int YCAP, int MODE>
__global__ __launch_bounds__(64) void mas_dp_kernel(const float* __restrict__ values, const int32_t* t_xs,
                                                    const int32_t* t_ys, int tx_max, int ty_max, float neg,
                                                    int32_t* __restrict__ pidx) {
  constexpr int kYB = (MODE & 32) ? (XPL >= 8 ? 4 : 8) : (MODE & 2) ? (XPL >= 16 ? 4 : (XPL >= 8 ? 8 : 16))
                           : (XPL >= 16 ? 2 : (XPL >= 8 ? 4 : 8));   // value columns prefetched per block
  __shared__ uint16_t bits[YCAP][64];
  const int b = blockIdx.x, L = threadIdx.x;
  int tx = t_xs[b], ty = t_ys[b];
  tx = tx > tx_max ? tx_max : tx;
  ty = ty > ty_max ? ty_max : ty;
  int32_t* P = pidx + (long)b * ty_max;
  if (tx <= 0 || ty <= 0) {
    for (int y = L; y < ty_max; y += 64) P[y] = -1;
    return;
  }
  const float* V0 = values + (long)b * tx_max * ty_max;
  float V[XPL];
  float cur[XPL][kYB], nxt[XPL][kYB];
#pragma unroll
  for (int i = 0; i < XPL; ++i) V[i] = 0.f;

  // Unconditional loads at clamped indices (rows >= tx_max read the last row, columns >= ty the last
  // column): those values never enter the band, so no per-load branch is needed; 32-bit offsets from the
  // utterance's (uniform) grid base.
  uint32_t roff[XPL];
#pragma unroll
  for (int i = 0; i < XPL; ++i) {
    const int x = L * XPL + i;
    roff[i] = (uint32_t)((x < tx_max ? x : tx_max - 1) * ty_max) * 4u;   // bytes
  }
  auto load_block = [&](float (&dst)[XPL][kYB], int y0) {
    if constexpr ((MODE & 32) != 0) {
      // 16-byte loads of 4 consecutive columns per row (rows are only 4-byte aligned: global loads need dword
      // alignment only). The last block of a grid falls back to clamped dword loads (uniform branch), so no
      // load reaches past the row end.
      if (y0 + kYB <= ty_max) {
        typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
#pragma unroll
        for (int q = 0; q < kYB / 4; ++q)
#pragma unroll
          for (int i = 0; i < XPL; ++i) {
            const f4u v = __builtin_nontemporal_load((const f4u*)((const char*)V0 + (roff[i] + (uint32_t)(y0 + 4 * q) * 4u)));
            dst[i][4 * q] = v.x; dst[i][4 * q + 1] = v.y; dst[i][4 * q + 2] = v.z; dst[i][4 * q + 3] = v.w;
          }
        return;
      }
    }
#pragma unroll
    for (int k = 0; k < kYB; ++k) {
      const uint32_t y4 = (uint32_t)(y0 + k < ty ? y0 + k : ty - 1) * 4u;
#pragma unroll
      for (int i = 0; i < XPL; ++i)
        dst[i][k] = __builtin_nontemporal_load((const float*)((const char*)V0 + (roff[i] + y4)));
    }
  };
  load_block(cur, 0);
  for (int y0 = 0; y0 < ty; y0 += kYB) {
    if (y0 + kYB < ty) load_block(nxt, y0 + kYB);
#pragma unroll
    for (int k = 0; k < kYB; ++k) {
      const int y = y0 + k;
      if (y < ty) {   // wave-uniform
        // V[L*XPL-1, y-1] from lane L-1 (lane 0's value is never used: its x = 0 row takes the constant)
        const float left = (MODE & 1) ? __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(V[XPL - 1]), 0x138,
                                                                             0xf, 0xf, false))
                                : __shfl_up(V[XPL - 1], 1);
        uint32_t w = 0;
        if constexpr ((MODE & 16) != 0) {
          // Lean update. Cells in the band (lo <= x < min(tx, y+1), lo = tx + y - ty) read only in-band cells
          // of column y-1 (or the NEG / 0 constants), and the backtrack visits only in-band cells, so every
          // row is updated unconditionally: out-of-band rows hold values nothing reads. For x != y, x != 0
          // the backtrack's compare V[x,y-1] < V[x-1,y-1] is the max's own v_prev > v_cur, so one compare
          // serves both; x == y forces the step (and takes NEG as v_cur), x == 0 never steps.
          const int dy = y - L * XPL;   // x == y  <=>  i == dy
#pragma unroll
          for (int i = XPL - 1; i >= 0; --i) {
            const bool diag = dy == i;
            const float v_cur = diag ? neg : V[i];
            float v_prev = (i > 0) ? V[i - 1] : left;
            if (i == 0) v_prev = (L == 0) ? (y == 0 ? 0.f : neg) : v_prev;
            const bool gt = v_prev > v_cur;
            V[i] = (gt ? v_prev : v_cur) + cur[i][k];
            const bool down = (i > 0 || L != 0) && (diag || gt);
            w |= (down ? 1u : 0u) << i;
          }
          bits[y][L] = (uint16_t)w;
          continue;
        }
        const int lo = tx + y - ty;                     // band: lo <= x < min(tx, y+1)
        const int hi = min(tx, y + 1);
#pragma unroll
        for (int i = XPL - 1; i >= 0; --i) {
          const int x = L * XPL + i;
          const float vc_real = V[i];
          const float vp_real = (i > 0) ? V[i - 1] : left;
          const float v_cur = (x == y) ? neg : vc_real;
          const float v_prev = (x == 0) ? (y == 0 ? 0.f : neg) : vp_real;
          const float mx = (v_prev > v_cur) ? v_prev : v_cur;
          const bool in_band = (x >= lo) && (x < hi);
          const float val = cur[i][k];
          V[i] = in_band ? (mx + val) : val;
          const bool down = in_band && (x != 0) && ((x == y) || (vc_real < vp_real));
          w |= (down ? 1u : 0u) << i;
        }
        bits[y][L] = (uint16_t)w;
      }
    }
#pragma unroll
    for (int i = 0; i < XPL; ++i)
#pragma unroll
      for (int k = 0; k < kYB; ++k) cur[i][k] = nxt[i][k];
  }
  __syncthreads();
  if constexpr ((MODE & 4) != 0) {
    // Windowed backtrack. Within 64 steps idx falls by at most 63, so for the chunk of columns yc, yc-1, ...,
    // yc-63 every row visited lies in [idx0-63, idx0]. Lane l gathers the "step down" bits of column yc-l for
    // exactly those rows into a 64-bit window (parallel LDS reads); the serial walk then reads lane l's
    // window with v_readlane (scalar registers, no memory latency) and records the falls as a 64-bit mask, from
    // which every lane recovers its own idx (mbcnt), so the chunk's 64 path entries are one coalesced store.
    int idx = tx - 1;
    for (int yc = ty - 1; yc >= 0; yc -= 64) {
      const int rb = idx - 63;   // window row 0
      const int y = yc - L;
      uint64_t win = 0;
      if (y >= 0) {
        const int w1 = idx / XPL;
        for (int lw = (rb > 0 ? rb : 0) / XPL; lw <= w1; ++lw) {
          const uint64_t w = bits[y][lw];
          const int rel = lw * XPL - rb;
          win |= rel >= 0 ? (w << rel) : (w >> (-rel));
        }
      }
      const uint32_t lo = (uint32_t)win, hi = (uint32_t)(win >> 32);
      const int n = yc + 1 < 64 ? yc + 1 : 64;
      const int idx0 = idx;
      uint64_t D = 0;   // bit l: idx fell at step l
#pragma unroll
      for (int l = 0; l < 64; ++l) {
        if (l < n) {
          const uint64_t sw = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(hi, l) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane(lo, l);   // (readlane returns int)
          const uint64_t d = (sw >> (idx - rb)) & 1u;
          D |= d << l;
          idx -= (int)d;
        }
      }
      // lane L's entry = idx0 - (falls before step L) = idx0 - popcount(D below lane L)
      if (y >= 0) P[y] = idx0 - (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(D >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)D, 0u));
    }
  } else if (L == 0) {
    int idx = tx - 1;
    for (int y = ty - 1; y >= 0; --y) {
      P[y] = idx;
      const uint32_t w = bits[y][idx / XPL];
      if ((w >> (idx % XPL)) & 1u) idx -= 1;
    }
  }
  for (int y = ty + L; y < ty_max; y += 64) P[y] = -1;
}

// Serial fallback for utterances beyond the register/LDS budget (t_x > 1024 or t_y > 1024): the
// reference loop verbatim on a scratch copy of `values`, one thread per utterance.
__global__ void mas_serial_kernel(const float* values, float* scratch, const int32_t* t_xs, const int32_t* t_ys,
                                  int b_total, int tx_max, int ty_max, float neg, int32_t* pidx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= b_total) return;
  const long base = (long)b * tx_max * ty_max;
  float* V = scratch + base;
  for (long i = 0; i < (long)tx_max * ty_max; ++i) V[i] = values[base + i];
  int tx = min(t_xs[b], tx_max), ty = min(t_ys[b], ty_max);
  int32_t* P = pidx + (long)b * ty_max;
  for (int y = 0; y < ty_max; ++y) P[y] = -1;
  if (tx <= 0 || ty <= 0) return;
  for (int y = 0; y < ty; ++y) {
    const int lo = max(0, tx + y - ty), hi = min(tx, y + 1);
    for (int x = lo; x < hi; ++x) {
      const float v_cur = (x == y) ? neg : V[(long)x * ty_max + y - 1];
      const float v_prev = (x == 0) ? (y == 0 ? 0.f : neg) : V[(long)(x - 1) * ty_max + y - 1];
      const float mx = (v_prev > v_cur) ? v_prev : v_cur;
      V[(long)x * ty_max + y] = mx + V[(long)x * ty_max + y];
    }
  }
  int idx = tx - 1;
  for (int y = ty - 1; y >= 0; --y) {
    P[y] = idx;
    if (idx != 0 && (idx == y || (y > 0 && V[(long)idx * ty_max + y - 1] < V[(long)(idx - 1) * ty_max + y - 1]))) idx -= 1;
  }
}

// paths[b][x][y] = (pidx[b][y] == x): every element written once, coalesced along y.
__global__ __launch_bounds__(256) void mas_fill_kernel(const int32_t* __restrict__ pidx, int tx_max, int ty_max,
                                                       int32_t* __restrict__ paths) {
  const int b = blockIdx.y;
  const long row = (long)blockIdx.x;   // x
  const int x = (int)row;
  const int32_t* P = pidx + (long)b * ty_max;
  int32_t* out = paths + ((long)b * tx_max + x) * ty_max;
  for (int y = threadIdx.x; y < ty_max; y += 256) out[y] = (P[y] == x) ? 1 : 0;
}

int mas_mode() {
  static const int v = [] {
    const char* e = getenv("GT_MAS_MODE");
    return e ? atoi(e) : 53;
  }();
  return v;
}

// ty_max % 4 == 0: 16-byte stores, 4 columns per thread (rows are then 16-byte aligned)
__global__ __launch_bounds__(256) void mas_fill4_kernel(const int32_t* __restrict__ pidx, int tx_max, int ty_max,
                                                        int32_t* __restrict__ paths) {
  const int b = blockIdx.y, x = blockIdx.x;
  const int4* P = reinterpret_cast<const int4*>(pidx + (long)b * ty_max);
  int4* out = reinterpret_cast<int4*>(paths + ((long)b * tx_max + x) * ty_max);
  for (int q = threadIdx.x; q < ty_max / 4; q += 256) {
    const int4 p = P[q];
    out[q] = make_int4(p.x == x, p.y == x, p.z == x, p.w == x);
  }
}

template <int XPL, int MODE>
void launch_dp_v(int ycap, const float* values, const int32_t* t_xs, const int32_t* t_ys, int b, int tx_max,
                 int ty_max, float neg, int32_t* pidx, hipStream_t s) {
  if (ycap <= 256) hipLaunchKernelGGL((mas_dp_kernel<XPL, 256, MODE>), dim3(b), dim3(64), 0, s, values, t_xs, t_ys, tx_max, ty_max, neg, pidx);
  else hipLaunchKernelGGL((mas_dp_kernel<XPL, 1024, MODE>), dim3(b), dim3(64), 0, s, values, t_xs, t_ys, tx_max, ty_max, neg, pidx);
}

template <int XPL>
hipError_t launch_dp(int ycap, const float* values, const int32_t* t_xs, const int32_t* t_ys, int b, int tx_max,
                     int ty_max, float neg, int32_t* pidx, hipStream_t s) {
  switch (mas_mode()) {
    case 0: launch_dp_v<XPL, 0>(ycap, values, t_xs, t_ys, b, tx_max, ty_max, neg, pidx, s); break;
    case 21: launch_dp_v<XPL, 21>(ycap, values, t_xs, t_ys, b, tx_max, ty_max, neg, pidx, s); break;
    default: launch_dp_v<XPL, 53>(ycap, values, t_xs, t_ys, b, tx_max, ty_max, neg, pidx, s); break;
  }
  return hipGetLastError();
}

}  // namespace

extern "C" {

// Workspace = [<=15 B alignment slack][pidx: b x ty_max int32, 16-B aligned (the 16-byte fill reads it as int4)]
// [fp32 scratch for the serial path]; any caller alignment works.
size_t gt_maximum_path_workspace_bytes(int64_t b, int64_t tx_max, int64_t ty_max) {
  if (b <= 0 || tx_max <= 0 || ty_max <= 0) return 0;
  size_t n = 16 + (((size_t)b * ty_max * 4 + 255) & ~size_t(255));
  if (tx_max > 1024 || ty_max > 1024) n += (size_t)b * tx_max * ty_max * 4;
  return n;
}

int gt_maximum_path(int32_t* paths, const float* values, const int32_t* t_xs, const int32_t* t_ys, int64_t b,
                    int64_t tx_max, int64_t ty_max, float max_neg_val, void* workspace, size_t workspace_bytes,
                    void* stream) {
  if (b == 0) return GT_OK;
  if (!paths || !values || !t_xs || !t_ys || b < 0 || tx_max <= 0 || ty_max <= 0) return GT_ERR_ARG;
  if (b > 65535 || tx_max > (1 << 20) || ty_max > (1 << 20)) return GT_ERR_UNSUPPORTED;
  if (!workspace || workspace_bytes < gt_maximum_path_workspace_bytes(b, tx_max, ty_max)) return GT_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  int32_t* pidx = (int32_t*)(((uintptr_t)workspace + 15) & ~(uintptr_t)15);
  const int B = (int)b, TX = (int)tx_max, TY = (int)ty_max;
  hipError_t e;
  if (TX > 1024 || TY > 1024) {
    float* scratch = (float*)((uint8_t*)pidx + (((size_t)b * ty_max * 4 + 255) & ~size_t(255)));
    hipLaunchKernelGGL(mas_serial_kernel, dim3((B + 63) / 64), dim3(64), 0, s, values, scratch, t_xs, t_ys, B, TX, TY,
                       max_neg_val, pidx);
    e = hipGetLastError();
  } else {
    const int xpl = (TX + 63) / 64;
    if (xpl <= 1) e = launch_dp<1>(TY, values, t_xs, t_ys, B, TX, TY, max_neg_val, pidx, s);
    else if (xpl <= 2) e = launch_dp<2>(TY, values, t_xs, t_ys, B, TX, TY, max_neg_val, pidx, s);
    else if (xpl <= 4) e = launch_dp<4>(TY, values, t_xs, t_ys, B, TX, TY, max_neg_val, pidx, s);
    else if (xpl <= 8) e = launch_dp<8>(TY, values, t_xs, t_ys, B, TX, TY, max_neg_val, pidx, s);
    else e = launch_dp<16>(TY, values, t_xs, t_ys, B, TX, TY, max_neg_val, pidx, s);
  }
  if (e != hipSuccess) return GT_ERR_HIP;
  if (TY % 4 == 0 && ((uintptr_t)paths & 15) == 0) hipLaunchKernelGGL(mas_fill4_kernel, dim3(TX, B), dim3(256), 0, s, pidx, TX, TY, paths);
  else hipLaunchKernelGGL(mas_fill_kernel, dim3(TX, B), dim3(256), 0, s, pidx, TX, TY, paths);
  return hipGetLastError() == hipSuccess ? GT_OK : GT_ERR_HIP;
}

}  // extern "C"
