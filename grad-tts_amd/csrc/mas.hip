// Monotonic Alignment Search on gfx950 -- bit-exact replacement of model/monotonic_align/core.pyx.
//
// Reference (core.pyx:9-35, generated C core.c:2653-2940), per utterance:
//   forward  for y < t_y, x in [max(0, t_x+y-t_y), min(t_x, y+1)):
//              v_cur  = (x == y) ? NEG : V[x, y-1];  v_prev = (x == 0) ? (y == 0 ? 0 : NEG) : V[x-1, y-1]
//              V[x, y] = ((v_prev > v_cur) ? v_prev : v_cur) + V[x, y]          (one fp32 max + one fp32 add)
//   backtrack idx = t_x-1; for y = t_y-1..0: P[idx, y] = 1;
//              if idx != 0 && (idx == y || V[idx, y-1] < V[idx-1, y-1]) idx -= 1
// Column y depends only on column y-1, so the DP runs column-parallel. One workgroup per utterance, NW waves
// (one per SIMD up to 4, two per SIMD at 8), wave w owning rows [w*64*XPL, (w+1)*64*XPL), lane L rows
// w*64*XPL + L*XPL + i in registers. Inside a wave the neighbour row arrives by a DPP wave_shr:1; across waves the
// schedule is skewed: the columns go in blocks of 32 and wave w runs block j in step j + w, one workgroup barrier
// per step, so the row above a wave's first row (the previous wave's last row, 32 columns of it) was written to LDS
// one step earlier. The backtrack needs only the comparison V[x,y-1] < V[x-1,y-1], which the forward's max already
// evaluates (for x != y, x != 0 it IS v_prev > v_cur), so the forward keeps one "step down" bit per cell -- shifted
// into a per-row register word, one LDS word per row and 32-column block -- instead of the fp32 DP table; row 0
// clears it, and the backtrack adds the diagonal's forced step. Both steps use exactly the reference's fp32 operations in the same order
// -> bit-identical paths. Cells outside the band are updated too (unconditionally): in-band cells read only in-band
// cells of the previous column (or the NEG / 0 constants), and the backtrack visits only in-band cells.
// The value columns stream through a ring of register blocks, several 32-column blocks ahead of the column being
// computed (one wave per utterance with a single block ahead had left the DP waiting on HBM latency), by temporal
// loads (nontemporal ones, each 16 B of a different 128-B line per lane, re-fetched every line eight times), and the
// {0,1} path tensor is written by a separate full-bandwidth kernel from the per-column row index.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "gradtts.h"

#define GT_MAS_DEV __device__ __forceinline__

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMasCols = 32;             // columns per block (= bits per LDS word)
constexpr int kMasMaxBlk = 1024 / kMasCols;
constexpr int kMasMaxRows = 1024;
constexpr int kMasMaxWaves = 8;

// value blocks held in registers per lane (the block being computed + RING-1 in flight)
template <int XPL> struct MasRing { static constexpr int n = XPL == 1 ? 4 : 2; };

// Value loads: 16-byte buffer loads, 8 per row and 32-column block. Rows at or past t_x, and blocks past the
// utterance's last, carry an offset outside the buffer (num_records = the utterance's grid), so the range check
// returns zeros without touching memory; a grid row's last block reads past the row end into the next row (columns
// >= t_y_max: computed, never read) or out of the buffer (zeros). Every wave issues exactly the same loads in every
// step, outside any branch, so hipcc's vmcnt bookkeeping sees the ring exactly and waits for a block only when its
// first value is used (loads inside the compute branch, with an idle path beside it, had merged into vmcnt(0) waits
// that drained the ring).
GT_MAS_DEV void mas_ld(f32x4& dst, __amdgpu_buffer_rsrc_t rs, uint32_t voff) {
  dst = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
}

// One 32-column block of one wave. DIAG: the block meets the diagonal x == y inside this wave's rows, where v_cur is
// NEG (the diagonal's forced step is added by the backtrack).
template <int XPL, int RING, bool DIAG>
GT_MAS_DEV void mas_block(float (&V)[XPL], f32x4 (&val)[XPL][kMasCols / 4], const f32x4* bsrc, float& carry,
                          f32x4* bdst, bool lane63, uint32_t (&wb)[XPL], int r0, int y0, float neg) {
  int kd[XPL];   // column (within the block) of this lane's diagonal cell, per row
#pragma unroll
  for (int i = 0; i < XPL; ++i) kd[i] = r0 + i - y0;
  // the row above this wave's first row (the previous wave's last row, or NEG for wave 0: x == 0 has v_prev = NEG for
  // y > 0), 4 columns per LDS read, one read ahead; `old` = its column y-1
  f32x4 ch = bsrc[0], chn = bsrc[1], bo4;
  float old = carry;
#pragma unroll
  for (int k = 0; k < kMasCols; ++k) {
    // V[r0-1, y-1] from lane L-1; lane 0 takes `old` (bound_ctrl off: an invalid source lane keeps the old value)
    const float left = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(V[XPL - 1]),
                                                                  0x138, 0xf, 0xf, false));
#pragma unroll
    for (int i = XPL - 1; i >= 0; --i) {
      const float v_prev = i > 0 ? V[i - 1] : left;
      float v_cur = V[i];
      if constexpr (DIAG) v_cur = kd[i] == k ? neg : v_cur;
      const bool gt = v_prev > v_cur;
      V[i] = (gt ? v_prev : v_cur) + val[i][k >> 2][k & 3];
      wb[i] = wb[i] + wb[i] + (gt ? 1u : 0u);   // bit (31 - k) <-> column y0 + k
      asm volatile("" : "+v"(wb[i]));   // fold the bit in now: hipcc otherwise keeps 32 compare masks alive in SGPRs
    }
    bo4[k % 4] = V[XPL - 1];
    old = ch[k % 4];
    if (k % 4 == 3) {
      if (lane63) bdst[k / 4] = bo4;   // this wave's last row, for the next wave (the last wave's goes unread)
      ch = chn;
      if (k / 4 + 2 < kMasCols / 4) chn = bsrc[k / 4 + 2];
    }
  }
  carry = old;
}

// One backtrack column: SCC = bit f of the column's word (step down from row idx0 - f); D |= BIT if so; f += SCC.
template <uint32_t BIT>
GT_MAS_DEV void mas_walk_step(uint32_t& f, uint32_t& D, uint32_t cw) {
  uint32_t t;
  asm volatile("s_bitcmp1_b32 %3, %0\n\ts_cselect_b32 %2, %4, 0\n\ts_addc_u32 %0, %0, 0\n\ts_or_b32 %1, %1, %2"
               : "+s"(f), "+s"(D), "=&s"(t) : "s"(cw), "n"(BIT) : "scc");
}

// Columns K and K-1 (one ballot), then the pair below, down to column 0.
template <int K>
GT_MAS_DEV void mas_walk(uint32_t& f, uint32_t& D, uint32_t word) {
  if constexpr (K > 0) {
    const uint64_t cw = __builtin_amdgcn_ballot_w64(((word >> (31 - K)) & 1u) != 0u);
    mas_walk_step<(1u << K)>(f, D, (uint32_t)cw);
    mas_walk_step<(1u << (K - 1))>(f, D, (uint32_t)(cw >> 32));
    mas_walk<K - 2>(f, D, word);
  }
}

template <int XPL>
__global__ __launch_bounds__(kMasMaxWaves * 64) void mas_dp_kernel(const float* __restrict__ values,
                                                                  const int32_t* t_xs, const int32_t* t_ys,
                                                                  int tx_max, int ty_max, float neg,
                                                                  int32_t* __restrict__ pidx) {
  constexpr int RING = MasRing<XPL>::n;
  constexpr int RW = 64 * XPL;                                  // rows per wave
  __shared__ uint32_t bits[kMasMaxBlk * kMasMaxRows];           // [block][row]: step-down bits, bit 31-k = column 32j+k
  __shared__ __attribute__((aligned(16))) float bnd[kMasMaxWaves][2][kMasCols];   // wave w's last row, by block parity
  __shared__ f32x4 bneg[kMasCols / 4];   // wave 0's "row above": x == 0 has v_prev = NEG for y > 0
  const int nw = blockDim.x >> 6, RP = nw * RW;
  // w through readfirstlane: hipcc then knows it is wave-uniform, and the per-wave conditions (active, diagonal block,
  // boundary writer) become scalar branches, not exec-masked both-sides code
  const int b = blockIdx.x, L = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tx = t_xs[b], ty = t_ys[b];
  tx = tx > tx_max ? tx_max : tx;
  ty = ty > ty_max ? ty_max : ty;
  int32_t* P = pidx + (long)b * ty_max;
  for (int y = (ty > 0 ? ty : 0) + (int)threadIdx.x; y < ty_max; y += blockDim.x) P[y] = -1;
  if (tx <= 0 || ty <= 0) return;   // uniform over the workgroup: no barrier has run
  if (threadIdx.x < kMasCols / 4) bneg[threadIdx.x] = f32x4{neg, neg, neg, neg};   // read by wave 0 only
  const float* V0 = values + (long)b * tx_max * ty_max;
  const int nblk = (ty + kMasCols - 1) / kMasCols;
  const int r0 = w * RW + L * XPL;

  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)V0, (short)0, (int)((uint32_t)tx_max * ty_max * 4u), 0x00020000);
  constexpr uint32_t kOut = 0x80000000u;   // an offset past any grid (at most 1024 x 1024 x 4 B)
  uint32_t roff[XPL];
#pragma unroll
  for (int i = 0; i < XPL; ++i) roff[i] = r0 + i < tx ? (uint32_t)((r0 + i) * ty_max) * 4u : kOut;
  auto boff = [&](int j) { return j < nblk ? (uint32_t)(j * kMasCols) * 4u : kOut; };
  f32x4 vb[RING][XPL][kMasCols / 4];
#pragma unroll
  for (int s = 0; s < RING - 1; ++s)
#pragma unroll
    for (int q = 0; q < kMasCols / 4; ++q)
#pragma unroll
      for (int i = 0; i < XPL; ++i) mas_ld(vb[s][i][q], rs, roff[i] + boff(s) + 16u * q);
  float V[XPL];
#pragma unroll
  for (int i = 0; i < XPL; ++i) V[i] = 0.f;
  float carry = 0.f;   // row above, column 32j - 1 (column -1: the reference's y == 0 constant 0 for row 0)
  for (int i = 0; i < w; ++i) __syncthreads();   // skew: wave w starts block 0 in step w
  for (int j0 = 0; j0 < nblk; j0 += RING) {
#pragma unroll
    for (int s = 0; s < RING; ++s) {
      const int j = j0 + s;
      // the next ring block's loads, in one burst outside every branch (issued inside the column loop, the register
      // allocator reused the slot's registers around them and hipcc's vmcnt waits drained the ring)
#pragma unroll
      for (int q = 0; q < kMasCols / 4; ++q)
#pragma unroll
        for (int i = 0; i < XPL; ++i) mas_ld(vb[(s + RING - 1) % RING][i][q], rs, roff[i] + boff(j + RING - 1) + 16u * q);
      if (j < nblk) {   // workgroup-uniform
        if (w * RW < tx) {   // wave-uniform: a wave whose rows all lie past t_x only keeps the barrier count
          uint32_t wb[XPL];
#pragma unroll
          for (int i = 0; i < XPL; ++i) wb[i] = 0u;
          const int y0 = j * kMasCols;
          f32x4* bdst = (f32x4*)bnd[w][j & 1];
          const f32x4* bsrc = w > 0 ? (const f32x4*)bnd[w - 1][j & 1] : bneg;
          if (y0 < w * RW + RW && y0 + kMasCols > w * RW)
            mas_block<XPL, RING, true>(V, vb[s], bsrc, carry, bdst, L == 63, wb, r0, y0, neg);
          else
            mas_block<XPL, RING, false>(V, vb[s], bsrc, carry, bdst, L == 63, wb, r0, y0, neg);
#pragma unroll
          for (int i = 0; i < XPL; ++i) bits[j * RP + r0 + i] = r0 + i == 0 ? 0u : wb[i];   // row 0 never steps
        }
        __syncthreads();
      }
    }
  }
  for (int i = w; i < nw - 1; ++i) __syncthreads();
  if (w != 0) return;

  // Backtrack, 32 columns per LDS round trip. Within a block idx falls by at most 31, so lane l < 32 holds the bits
  // of row idx0 - l, and lane 32 + l the same word shifted by one column: one ballot gives column k's bits over those
  // rows (low half) and column k-1's (high half). The walk is scalar: per column, SCC = bit f of the column word,
  // f += SCC, and the fall recorded in D (s_bitcmp1 / s_cselect / s_addc / s_or).
  int idx = tx - 1;
  for (int j = nblk - 1; j >= 0; --j) {
    const int y0 = j * kMasCols;
    const int ncol = ty - y0 < kMasCols ? ty - y0 : kMasCols;   // uniform
    const int row = idx - (L & 31);
    uint32_t word = row >= 0 ? bits[j * RP + row] : 0u;
    if (row > 0 && row >= y0 && row < y0 + kMasCols) word |= 1u << (31 - (row - y0));   // x == y: the step is forced
    if (ncol < kMasCols) word &= ~((1u << (kMasCols - ncol)) - 1u);   // columns >= t_y: no step
    word = L < 32 ? word : word >> 1;
    uint32_t f = 0, D = 0;   // falls so far; bit k: idx fell at column y0 + k
    mas_walk<kMasCols - 1>(f, D, word);
    // column y0 + L: idx before its step = idx0 - (falls at columns > L)
    if (L < ncol) P[y0 + L] = idx - (int)__builtin_popcountll((uint64_t)D >> (L + 1));
    idx -= (int)f;
  }
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

template <int XPL>
hipError_t launch_dp(int nw, const float* values, const int32_t* t_xs, const int32_t* t_ys, int b, int tx_max,
                     int ty_max, float neg, int32_t* pidx, hipStream_t s) {
  hipLaunchKernelGGL(mas_dp_kernel<XPL>, dim3(b), dim3(64 * nw), 0, s, values, t_xs, t_ys, tx_max, ty_max, neg, pidx);
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
    // one wave per 64 rows up to 512 rows, then two rows per lane (8 waves, 1024 rows)
    if (TX <= 64 * kMasMaxWaves) e = launch_dp<1>((TX + 63) / 64, values, t_xs, t_ys, B, TX, TY, max_neg_val, pidx, s);
    else e = launch_dp<2>((TX + 127) / 128, values, t_xs, t_ys, B, TX, TY, max_neg_val, pidx, s);
  }
  if (e != hipSuccess) return GT_ERR_HIP;
  if (TY % 4 == 0 && ((uintptr_t)paths & 15) == 0) hipLaunchKernelGGL(mas_fill4_kernel, dim3(TX, B), dim3(256), 0, s, pidx, TX, TY, paths);
  else hipLaunchKernelGGL(mas_fill_kernel, dim3(TX, B), dim3(256), 0, s, pidx, TX, TY, paths);
  return hipGetLastError() == hipSuccess ? GT_OK : GT_ERR_HIP;
}

}  // extern "C"
