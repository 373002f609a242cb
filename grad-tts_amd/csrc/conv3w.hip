// Wide-tile 3x3 convolution (stride 1, pad 1) for the 128- and 256-channel U-Net levels, bf16 (gfx950).
//
// Covers Block.block[0] (model/diffusion.py:52) at U-Net levels 1-2 with Cin % 32 == 0 -- the convs that carry half
// of a U-Net evaluation's FLOPs. conv_kernel (conv.hip) runs them as 128-wide, 4-wave tiles, two workgroups per CU,
// three barriers per 16-channel chunk: the structure that tops out near 900-1100 TFLOP/s on CDNA4 (every chunk waits
// on its own weight DMA), with the GroupNorm operand transform recomputed by both 128-channel tiles of a 256-output
// conv and by the 7/5 halo rows. This kernel is the one-workgroup-per-CU, deep-pipelined form:
//
//   * 8 waves (512 threads), ONE workgroup per CU. The workgroup owns ALL output channels of its spatial tile (BN = Cout:
//     256, 128 or 64), so every input element of the tile is loaded and (IN_GN) GroupNorm + Mish + time-bias transformed
//     exactly once per tile; halo rows add (TR + 2) / TR (1.2x at 10 rows, 1.1x at 20).
//   * Tile = TR mel rows x 32 frames. Wave (wn, wm) computes CB x 32 output channels x RB = 5 rows: 2 RB x 2 CB blocks of
//     16 positions x 16 channels on v_mfma_f32_16x16x32_bf16 (weights as A, positions as B), accumulated in place by
//     inline asm (mfma16). The 16x16x32 shape holds a higher clock than 32x32x16 under this load (profiles/r05/
//     mfma_shape_bench.txt).
//   * K loop = phases: one phase = one tap x 32 input channels (one 16x16x32 k-step). A weight slot (BN rows x 32 channels,
//     BN x 64 B) is staged by LDS DMA (global_load_lds, 1 KiB per wave instruction) into a ring of S slots, D = S - 1
//     phases ahead; the counted `s_waitcnt vmcnt` at the top of phase k retires DMA(k+1), so each slot is visible one
//     phase before it is read and the first fragments of phase k+1 are read during phase k (no MFMA bubble at the
//     barrier). One barrier per phase.
//   * The input patch ((TR + 2) x 34 positions x 32 channels) is double-buffered per 32-channel chunk: the next chunk's
//     items are loaded into registers at phase 0 (raw buffer loads: padding / masked frames read past the end of the
//     tensor, zeros), transformed and written one item per phase during phases 2..7, behind the MFMAs.
//   * LDS layouts are PLANAR: 8-channel planes of 16-B entries, [plane][position] for the patch and [plane][channel] for
//     a weight slot, so a fragment (32 consecutive positions / channels of one plane) is a contiguous 512 B: conflict-free
//     ds_read_b128 at any tap shift, and every fragment address is one per-lane base plus a compile-time offset. The patch
//     plane stride is 2 mod 16 entries, so the item writes (4 planes of one position per lane quad) are conflict-free too.
//     The weight image in HBM is pre-packed in exactly the slot layout (decoder.cpp pack_conv3w): a slot is one straight
//     DMA.
// Epilogue: bias, GroupNorm partial sums of the output (one slot per tile, fixed-order reduction), 16-B bf16 stores, from
// the accumulators through v_permlane16_swap.
#include "common.h"
#include "kernels.h"
#include "wimage.h"
#include "c3w_asm.h"
#include "stamps.h"

namespace gt {

#ifndef GT_C3W_STAMP
#define GT_C3W_STAMP 0   // diagnostic builds only: s_memtime stamps of the phase waits (gt_diag_conv3w_stamps)
#endif
#ifndef GT_C3W_STAMP_BN
#define GT_C3W_STAMP_BN 256
#endif
#ifndef GT_C3W_STAMP_IN
#define GT_C3W_STAMP_IN 2
#endif

namespace c3w {
constexpr int NTHR = 512, NW = 8, RB = 5, TT = 32, PCOL = TT + 2;
constexpr int S256 = 5;   // weight ring slots of the 256-wide tiles
constexpr int PF = 2;     // fragment prefetch distance in MFMA steps (the B ring of PF + 1 must divide a chunk's 90 steps)

template <int BN, int CB>
struct Cfg {
  static constexpr int WN = BN / (32 * CB);        // waves along output channels
  static constexpr int WM = NW / WN;               // waves along mel rows
  static constexpr int TR = WM * RB;               // tile rows
  static constexpr int PR = TR + 2;                // patch rows
  static constexpr int PP = PR * PCOL;             // patch positions
  static constexpr int PPAD = (PP + 15) & ~15;     // plane stride in 16-B entries, == 0 mod 16 (see the fragments)
  static constexpr int PLANE = PPAD * 16;
  static constexpr int PBUF = 4 * PLANE;           // one 32-channel patch buffer
  static constexpr int SLOT = BN * 64;             // one weight slot: BN channels x 32 input channels
  static constexpr int PIECES = SLOT / 1024;       // DMA pieces per slot
  static constexpr int PWMAX = (PIECES + NW - 1) / NW;
  static constexpr int PWLO = PIECES / NW;         // pieces of waves >= PIECES % NW
  static constexpr int S = BN == 256 ? S256 : (CB == 2 ? 6 : 8);   // weight ring slots (LDS budget below)
  static constexpr int D = S - 1;                  // DMA issue distance in phases
  static constexpr int ITEMS = PP * 4;             // 16-B patch items per chunk
  static constexpr int NPT = (ITEMS + NTHR - 1) / NTHR;
  static constexpr int NCB = 2 * CB;               // 16-channel blocks per wave
  static constexpr int NS = 2 * RB;                // MFMA steps per phase (16-position blocks: row block x half)
  // phases between an item's load and its transform (item j: loaded at phase j, transformed at phase j + XD <= 7)
  static constexpr int XD = (8 - NPT) < 2 ? (8 - NPT) : 2;
  // phase of item j's transform (TP) and of its load (LP): XD phases apart, consecutive items in consecutive phases;
  // NPT <= 4 (SPREAD): transforms every other phase (1, 3, 5, 7), each load two phases ahead, so the VALU of the
  // operand transform is spread over the chunk instead of filling phases XD .. XD + NPT - 1
  static constexpr bool SPREAD = NPT <= 4;
  static constexpr int TP(int j) { return SPREAD ? 1 + 2 * j : j + XD; }
  static constexpr int LP(int j) { return SPREAD ? (TP(j) >= 2 ? TP(j) - 2 : 0) : j; }
  static constexpr int jl(int t) {   // item loaded at phase t, or -1
    for (int j = 0; j < NPT; ++j) if (LP(j) == t) return j;
    return -1;
  }
  static constexpr int jt(int t) {   // item transformed at phase t, or -1
    for (int j = 0; j < NPT; ++j) if (TP(j) == t) return j;
    return -1;
  }
  static constexpr int OFF_W = 2 * PBUF;
  static constexpr int OFF_F = OFF_W + S * SLOT;   // float area
  // floats: s_sc, s_sh, s_tb [256] each, s_bias [256], s_wsc [256], s_sub [NW][CB][4][2], s_mean, s_rstd [8]
  static constexpr int NF = 5 * 256 + NW * CB * 8 + 16;
  static constexpr int SMEM = OFF_F + NF * 4;
  static_assert(WN * WM == NW && WN >= 1, "wave grid");
  static_assert(PIECES * 1024 == SLOT, "whole DMA pieces");
  static_assert(D >= 2 && D <= 8, "DMA distance");
  static_assert(NPT <= 6, "items transformed in phases 2..7");
  static_assert(SMEM <= 160 * 1024, "LDS budget: one workgroup per CU");
  static_assert(PBUF >= 272 * 8, "s_red aliases patch buffer 1");
};
}  // namespace c3w

// stamps.h counters: cycles in the DMA wait, the phase barrier, the item waits, the item transforms + writes, the whole
// chunk loop, phases, prologue, epilogue (the last launch of the stamped instantiation wins)
#if GT_C3W_STAMP
GT_STAMP_BUFFER(gt_c3w_stamps, gt_diag_conv3w_stamps, 8)
#define GT_C3W_STAMP_DST gt_c3w_stamps
#else
#define GT_C3W_STAMP_DST nullptr
#endif

// v_mfma_f32_16x16x32_bf16 accumulating in place. hipcc does not tie the builtin's destination to its C operand (a third
// of the builtin MFMAs of this loop wrote a fresh register set, the accumulators rotated through the register file and
// the kernel spilled); the asm form keeps every accumulator in its registers. hipcc pads no hazards inside asm: the
// accumulators are written by these MFMAs only, their A / B operands come from LDS reads (waited for by the compiler:
// register inputs of the statement) and are overwritten no earlier than one MFMA group later, and the epilogue
// (mfma_drain) waits out the last MFMAs before any other instruction reads an accumulator.
GT_DEV void mfma16(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}

// IN: IN_MASK (x * mask), IN_GN ((Mish(GN(h)) + tb) * mask), IN_PLAIN. OUT: OUT_STATS.
template <int IN, int BN, int CB>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void conv3w_kernel(ConvParams p) {
  typedef c3w::Cfg<BN, CB> C;
  using c3w::NTHR; using c3w::RB; using c3w::PCOL;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];   // ONE LDS object
  float* const s_sc = reinterpret_cast<float*>(smem + C::OFF_F);
  float* const s_sh = s_sc + 256;
  float* const s_tb = s_sh + 256;
  float* const s_bias = s_tb + 256;
  float* const s_wsc = s_bias + 256;   // fp8-weight images (GT_BF16_W8): per-output-channel weight scale
  float* const s_sub = s_wsc + 256;
  float* const s_mean = s_sub + c3w::NW * CB * 8;
  float* const s_rstd = s_mean + 8;
  double* const s_red = reinterpret_cast<double*>(smem + C::PBUF);   // patch buffer 1 is free until chunk 0, phase 2

  const int F = p.Fout, T = p.Tout;
  const int n_ft = F / C::TR, n_tt = (T + 31) / 32;
  const int nsp = p.B * n_ft * n_tt;
  // XCD-aware order (as conv_kernel): XCD x walks the contiguous tile range [x Q, x Q + Q)
  int bid = (blockIdx.x & 7) * ((nsp + 7) >> 3) + (blockIdx.x >> 3);
  if (bid >= nsp) return;   // grid padding: the whole workgroup, before any barrier
  const int tt = bid % n_tt; bid /= n_tt;
  const int ft = bid % n_ft;
  const int b = bid / n_ft;
  const int f0 = ft * C::TR, t0 = tt * 32;

  constexpr bool STAMP = GT_C3W_STAMP && BN == GT_C3W_STAMP_BN && IN == GT_C3W_STAMP_IN;
  Stamps<STAMP> ps;
  const unsigned long long t_entry = ps.now();
  // v_mfma_f32_16x16x32_bf16 lanes: r = row of A (output channel) / column of B (position) in a 16 x 16 block, g = the
  // 8-channel plane (k group) of both operands
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wv % C::WN, wm = wv / C::WN;
  // patch items: a wave's 64 consecutive items are 16 consecutive positions x 4 planes, lanes 16q .. 16q + 15 on plane q
  // (8 contiguous lanes store 128 contiguous bytes of one plane: conflict-free at any plane stride)
  const int q16 = g;                             // this thread's 8-channel plane inside a chunk (fixed)
  auto item_pos = [&](int j) { return (((tid + NTHR * j) >> 6) << 4) | r; };

  // ---- prologue loads: GroupNorm slots (IN_GN), per-channel coefficients, bias, masks
  GnLoad gl;
  if (IN == IN_GN) gl = gn_load(p.gn_part, p.gn_nparts, b);
  float c_g = 0.f, c_b = 0.f, c_t = 0.f;
  if (IN == IN_GN && tid < p.Cin) {
    c_g = p.gn_gamma[tid]; c_b = p.gn_beta[tid]; c_t = tb_at(p.tb, p.stepp)[(long)b * p.tb_bstride + tid];
  }
  const float c_bias = tid < BN ? p.bias[tid] : 0.f;
  // fp8 weights (the image holds their e4m3 values, exact in bf16): out = acc * scale + bias, as conv_kernel's W8
  const bool w8 = p.wscale != nullptr;
  const float c_wsc = (w8 && tid < BN) ? p.wscale[tid] : 1.f;

  const int npos = p.B * F * T;
  int pidx[C::NPT];
  float pm[C::NPT];
  bool frac = false;
#pragma unroll
  for (int j = 0; j < C::NPT; ++j) {
    const int pp = item_pos(j);
    const int pr = pp / PCOL, pc = pp - pr * PCOL;
    const int fi = f0 - 1 + pr, ti = t0 - 1 + pc;
    const bool ok = pp < C::PP && fi >= 0 && fi < F && ti >= 0 && ti < T;
    const float m = ok ? mask_at(p.mask, p.T0, b, ti, p.lvl_in) : 0.f;
    int qi = ok ? (b * F + fi) * T + ti : npos;
    if (IN == IN_MASK && m == 0.f) qi = npos;   // x * 0: the range-checked load returns zeros
    if (IN != IN_PLAIN) frac |= (m != 0.f && m != 1.f);
    pidx[j] = qi;
    pm[j] = (IN == IN_PLAIN) ? (ok ? 1.f : 0.f) : m;
  }
  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.in0, (short)0, npos * p.C0 * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.in1 ? p.in1 : p.in0), (short)0, npos * (p.in1 ? p.C1 : p.C0) * 2, 0x00020000);
  const int nchunk = p.Cin / 32;
  const int K = nchunk * 9;

  // The next chunk's patch items are loaded by inline-asm buffer loads: hipcc would otherwise wait for them with a
  // conservative vmcnt(0) (draining the weight DMAs in flight). Item j is loaded at phase j and transformed at phase
  // j + XD, behind that phase's MFMAs, after a counted wait naming its registers (guide §5.7 form (ii)): at most XD + 1
  // items are in registers at once.
  u32x4c_t preg[C::NPT];
  auto load_items = [&](int c, auto JLO, auto JHI) {   // items [JLO, JHI) of chunk c
    const int c0 = c * 32;
    const bool first = c0 < p.C0;
    const int pb = (first ? p.C0 : p.C1) * 2;
    const int so = __builtin_amdgcn_readfirstlane((first ? c0 : c0 - p.C0) * 2);
    const __amdgpu_buffer_rsrc_t rs = first ? rs0 : rs1;
#pragma unroll
    for (int j = decltype(JLO)::value; j < decltype(JHI)::value && j < C::NPT; ++j) {
      const int vo = pidx[j] * pb + q16 * 16;
      asm_buffer_load(preg[j], vo, rs, so);
    }
  };
  auto load_patch = [&](int c) {   // every item (prologue: hipcc-visible loads are fine there)
    const int c0 = c * 32;
    if (c0 < p.C0) {
      const int pb = p.C0 * 2;
#pragma unroll
      for (int j = 0; j < C::NPT; ++j)
        preg[j] = __builtin_amdgcn_raw_buffer_load_b128(rs0, pidx[j] * pb + q16 * 16, c0 * 2, 0);
    } else {
      const int pb = p.C1 * 2;
#pragma unroll
      for (int j = 0; j < C::NPT; ++j)
        preg[j] = __builtin_amdgcn_raw_buffer_load_b128(rs1, pidx[j] * pb + q16 * 16, (c0 - p.C0) * 2, 0);
    }
  };
  // transform item j of chunk c and write it to patch buffer `buf`. IN_GN: (Mish(GN(h)) + tb) * m in base 2 (common.h
  // gn_mish_tb_l2), 4 channels at a time with their coefficients read from LDS right before (fewer registers live
  // across the MFMA stream than one coefficient set per chunk)
  auto put_item = [&](int j, int c, int buf) {
    const int pp = item_pos(j);
    if (pp >= C::PP) return;
    u32x4c_t v4 = preg[j];
    if (IN == IN_GN) {
      float v[8];
      item_to_f(make_uint4(v4[0], v4[1], v4[2], v4[3]), v, bf16());
      const int ch = c * 32 + q16 * 8;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const f32x4 sc = *reinterpret_cast<const f32x4*>(s_sc + ch + 4 * u);
        const f32x4 sh = *reinterpret_cast<const f32x4*>(s_sh + ch + 4 * u);
        const f32x4 tb = *reinterpret_cast<const f32x4*>(s_tb + ch + 4 * u);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[4 * u + k] = gn_mish_tb_l2(v[4 * u + k], sc[k], sh[k], tb[k]);
      }
      if (frac) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= pm[j];
      }
      const uint4 o = f_to_item(v, bf16());
      const bool z = !frac && pm[j] == 0.f;
      v4 = u32x4c_t{z ? 0u : o.x, z ? 0u : o.y, z ? 0u : o.z, z ? 0u : o.w};
    } else if (IN == IN_MASK) {
      if (frac) {
        float v[8];
        item_to_f(make_uint4(v4[0], v4[1], v4[2], v4[3]), v, bf16());
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= pm[j];
        const uint4 o = f_to_item(v, bf16());
        v4 = u32x4c_t{o.x, o.y, o.z, o.w};
      }
    }
    *reinterpret_cast<u32x4c_t*>(smem + buf * C::PBUF + q16 * C::PLANE + pp * 16) = v4;
  };

  // weight DMA: slot of phase k = image bytes [k SLOT, (k+1) SLOT) (decoder.cpp pack_conv3w). Every wave issues PW
  // pieces per slot (BN = 64: 4 pieces; waves 4..7 repeat waves 0..3's, same bytes to the same LDS), so the counted
  // waits below are the same in every wave.
  constexpr int PW = C::PIECES >= c3w::NW ? C::PIECES / c3w::NW : 1;
  static_assert(C::PIECES % c3w::NW == 0 || c3w::NW % C::PIECES == 0, "pieces split evenly");
  const char* const wimg = reinterpret_cast<const char*>(p.w);
  const unsigned lds_base = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(smem));
  const unsigned dma_voff = lane * 16;
  auto dma = [&](int k, int slot) {
    const char* src = wimg + (long)k * C::SLOT;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int piece = C::PIECES >= c3w::NW ? wv + c3w::NW * i : wv % C::PIECES;
      asm_dma16(src + piece * 1024, dma_voff, lds_base + C::OFF_W + slot * C::SLOT + piece * 1024);
    }
  };
  // items of the next chunk loaded at phases in [lo, hi] (item j at phase LP(j))
  constexpr auto n_lp = [](int lo, int hi) {
    int n = 0;
    for (int j = 0; j < C::NPT; ++j) n += (C::LP(j) >= lo && C::LP(j) <= hi) ? 1 : 0;
    return n;
  };
  // top of phase (t = tap, MORE: chunk c+1 exists): retire DMA(k+1). Younger VMEM ops of this wave: the DMAs of phases
  // k+2 .. k+D-1 that exist and the next chunk's items loaded at phases t+1-D .. t-1 of this chunk (issued after the
  // DMA of their phase).
  constexpr int NPRE = c3w::PF + C::NCB;   // LDS reads of the next phase: its first PF steps' B and its A (top_wait)
  auto top_wait = [&](auto Tc, auto MOREc) {
    constexpr int t = decltype(Tc)::value;
    constexpr bool MORE = decltype(MOREc)::value;
    // DMAs issued after DMA(k+1) before the top of phase k: up to DMA(k-1+D), or DMA(K-1) in the last chunk
    constexpr int ndma0 = MORE ? C::D - 2 : ((8 - t - 1) < (C::D - 2) ? (8 - t - 1) : (C::D - 2));
    constexpr int ndma = ndma0 > 0 ? ndma0 : 0;
    // items loaded in phases k + 1 - D .. k - 1 (each issued after the DMA of its phase)
    constexpr int npl = MORE ? n_lp(t + 1 - C::D, t - 1) : 0;
    const unsigned long long a = ps.now();
    vm_wait<ndma * PW + npl>();
    const unsigned long long b = ps.now();
    // LDS: every access of this wave but its last NPRE (the next phase's first fragments, read at the end of the
    // previous phase; they need no barrier, so their latency stays hidden) has completed -- the reads of the slot the
    // DMA below overwrites and the item writes of the next chunk's patch included (LDS ops complete in order)
    if (GT_C3W_STAMP) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(%0)\n\ts_barrier" :: "n"(NPRE) : "memory");
    ps.add(0, b - a); ps.add(1, ps.now() - b); ps.add(5, 1);
  };
  // before transforming item j at phase TP(j): younger VMEM ops are the items loaded at phases LP(j)+1 .. TP(j) and the
  // DMAs of those phases (each phase issues its DMA, then its item load, then this wait)
  auto item_wait = [&](auto Jc) {
    constexpr int j = decltype(Jc)::value;
    constexpr int n = n_lp(C::LP(j) + 1, C::TP(j)) + (C::TP(j) - C::LP(j)) * PW;
    const unsigned long long a = ps.now();
    vm_wait_dep<n>(preg[j]);
    ps.add(2, ps.now() - a);
  };

  // ---- fragments (v_mfma_f32_16x16x32_bf16: one 32-channel phase = one k of 32). A (weights): slot + plane g x BN +
  // channel; B (patch): buffer + plane g + position. Each is 16 consecutive 16-B entries per plane: with plane strides
  // == 0 mod 16 entries the four lane groups of a ds_read_b128 cover the 64 banks once.
  const int a_lane = C::OFF_W + (g * BN + wn * 32 * CB + r) * 16;
  const int b_lane = g * C::PLANE + (wm * RB * PCOL + r) * 16;
  auto rd_a = [&](int slot, int cb) {
    return *reinterpret_cast<const bf16x8*>(smem + a_lane + slot * C::SLOT + cb * 16 * 16);
  };
  auto rd_b = [&](int buf, int t, int pb) {   // 16-position block pb = row block pb / 2, frames 16 (pb % 2) ..
    const int dr = t / 3, dc = t % 3;
    return *reinterpret_cast<const bf16x8*>(smem + b_lane + buf * C::PBUF + ((pb / 2 + dr) * PCOL + (pb % 2) * 16 + dc) * 16);
  };

  f32x4 acc[C::NS][C::NCB];   // [16-position block][16-channel block]
#pragma unroll
  for (int i = 0; i < C::NS; ++i)
#pragma unroll
    for (int j = 0; j < C::NCB; ++j) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[i][j][k] = 0.f;
      asm volatile("" : "+v"(acc[i][j]));   // the zeros are written here, ahead of the wait states below
    }
  asm volatile("s_nop 4" ::: "memory");   // VALU write -> MFMA C-operand read (mfma16 pads nothing)

  // ---- prologue: chunk 0 patch loads, then the first D weight slots, then the GroupNorm reduction
  load_patch(0);
#pragma unroll
  for (int k = 0; k < C::D; ++k)
    if (k < K) dma(k, k);
  if (IN == IN_GN) {
    gn_finish(gl, p.gn_part, p.gn_nparts, b, p.gn_count, s_mean, s_rstd, s_red);
    if (tid < p.Cin) {
      const int gi = tid / (p.Cin >> 3);
      const float sc = c_g * s_rstd[gi];
      s_sc[tid] = sc * kLog2e; s_sh[tid] = (c_b - s_mean[gi] * sc) * kLog2e; s_tb[tid] = c_t;
    }
  }
  if (tid < BN) { s_bias[tid] = c_bias; s_wsc[tid] = c_wsc; }
  lds_barrier();
#pragma unroll
  for (int j = 0; j < C::NPT; ++j) put_item(j, 0, 0);
  // DMA(0), DMA(1) landed (younger: DMA(2 .. D-1)); chunk 0's patch written
  vm_wait<(C::D - 2) * PW>();
  lds_barrier();

  // MFMA steps i (16-position block i) of a phase, NCB MFMAs each; B fragments are read PF steps ahead (a ring of PF + 1
  // by the chunk-global step index, a chunk being 90 steps), across phase boundaries too: phase k+1's slot and patch are
  // visible from the top of phase k. The NCB A fragments of a phase are read after the previous phase's last MFMAs
  // (into the same registers), so they land during the phase barrier.
  constexpr int PF = c3w::PF, NB = PF + 1;
  static_assert(9 * C::NS % NB == 0 && PF <= C::NS, "B ring index chunk-periodic");
  bf16x8 fa[C::NCB], fb[NB];
#pragma unroll
  for (int cb = 0; cb < C::NCB; ++cb) fa[cb] = rd_a(0, cb);
#pragma unroll
  for (int n = 0; n < PF; ++n) fb[n] = rd_b(0, 0, n);

  int slot = 0;   // weight slot of the current phase (k mod S)
  // MFMA steps of the item transforms: waves 0-3 at XS0, waves 4-7 at XS1
  constexpr int XS0 = 1, XS1 = C::NS - 3;
  // One chunk: 9 phases. MORE: a chunk c+1 exists (its patch is loaded and written during this chunk).
  auto chunk = [&](int c, auto MOREc) {
    constexpr bool MORE = decltype(MOREc)::value;
    const int cur = c & 1, nxt = cur ^ 1;
    const int k0 = c * 9;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int k = k0 + t;
      // (a) DMA(k+1) landed for every wave, every read of phase k-1 done
      switch (t) {   // compile-time t for the wait immediates
        case 0: top_wait(std::integral_constant<int, 0>{}, MOREc); break;
        case 1: top_wait(std::integral_constant<int, 1>{}, MOREc); break;
        case 2: top_wait(std::integral_constant<int, 2>{}, MOREc); break;
        case 3: top_wait(std::integral_constant<int, 3>{}, MOREc); break;
        case 4: top_wait(std::integral_constant<int, 4>{}, MOREc); break;
        case 5: top_wait(std::integral_constant<int, 5>{}, MOREc); break;
        case 6: top_wait(std::integral_constant<int, 6>{}, MOREc); break;
        case 7: top_wait(std::integral_constant<int, 7>{}, MOREc); break;
        default: top_wait(std::integral_constant<int, 8>{}, MOREc); break;
      }
      int nslot = slot + 1;
      nslot = nslot == C::S ? 0 : nslot;
      // (b) DMA of phase k + D into the slot phase k - 1 used
      if (MORE || t + C::D < 9) {
        int ds = slot + C::D;
        ds = ds >= C::S ? ds - C::S : ds;
        dma(k + C::D, ds);
      }
      // (c) the next chunk's patch item of this phase (item t), and the counted wait for item t - XD's registers
      // (loaded XD phases ago; younger: items t-XD+1 .. t and the DMAs of XD phases -- the same count in both wave
      // halves). Unconditional in every wave: an asm load whose wait a wave skipped would land in a reused register.
      if (MORE) {
        if (C::jl(t) >= 0) {
          switch (C::jl(t)) {
            case 0: load_items(c + 1, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}); break;
            case 1: load_items(c + 1, std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{}); break;
            case 2: load_items(c + 1, std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{}); break;
            case 3: load_items(c + 1, std::integral_constant<int, 3>{}, std::integral_constant<int, 4>{}); break;
            case 4: load_items(c + 1, std::integral_constant<int, 4>{}, std::integral_constant<int, 5>{}); break;
            default: load_items(c + 1, std::integral_constant<int, 5>{}, std::integral_constant<int, 6>{}); break;
          }
        }
        if (C::jt(t) >= 0) {
          switch (C::jt(t)) {
            case 0: item_wait(std::integral_constant<int, 0>{}); break;
            case 1: if constexpr (C::NPT > 1) item_wait(std::integral_constant<int, 1>{}); break;
            case 2: if constexpr (C::NPT > 2) item_wait(std::integral_constant<int, 2>{}); break;
            case 3: if constexpr (C::NPT > 3) item_wait(std::integral_constant<int, 3>{}); break;
            case 4: if constexpr (C::NPT > 4) item_wait(std::integral_constant<int, 4>{}); break;
            default: if constexpr (C::NPT > 5) item_wait(std::integral_constant<int, 5>{}); break;
          }
        }
      }
      // (d) MFMAs of phase k
#pragma unroll
      for (int i = 0; i < C::NS; ++i) {
        const int gi = t * C::NS + i;         // chunk-global step (90 per chunk: the B ring index is chunk-periodic)
        const int n = i + PF;                 // step whose B fragment is read now
        int nrd = 0;
        if (n < C::NS) {
          fb[(gi + PF) % NB] = rd_b(cur, t, n);
          nrd = 1;
        } else if (MORE || t < 8) {           // phase k+1's steps 0 .. PF-1
          fb[(gi + PF) % NB] = t < 8 ? rd_b(cur, t + 1, n - C::NS) : rd_b(nxt, 0, n - C::NS);
          nrd = 1;
        }
#pragma unroll
        for (int cb = 0; cb < C::NCB; ++cb) mfma16(acc[i][cb], fa[cb], fb[gi % NB]);
        if (i == C::NS - 1 && (MORE || t < 8)) {   // phase k+1's A fragments, after this phase's last use
#pragma unroll
          for (int cb = 0; cb < C::NCB; ++cb) fa[cb] = rd_a(nslot, cb);
        }
        // (e) one patch item of chunk c+1 per phase, phases 2 .. 1 + NPT, behind this phase's MFMAs
        // Staggered between the two waves of a SIMD (waves w and w + 4 share one; MI355X_MICROARCH.md, two waves per
        // SIMD, item 9): waves 0-3 at step XS0, waves 4-7 at step XS1, so one wave's transform VALU runs beside its
        // partner's MFMAs instead of both leaving the matrix pipe idle at the same step.
        if (MORE && (i == XS0 || i == XS1) && C::jt(t) >= 0) {
          if ((i == XS0 && wv < c3w::NW / 2) || (i == XS1 && wv >= c3w::NW / 2)) {
            const unsigned long long a = ps.now();
            put_item(C::jt(t), c + 1, nxt);
            asm volatile("" ::: "memory");   // the item's LDS write stays ahead of the phase-end fragment reads (NPRE)
            ps.add(3, ps.now() - a);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      slot = nslot;
    }
  };
  int c = 0;
  const unsigned long long t_loop = ps.now();
  for (; c + 1 < nchunk; ++c) chunk(c, std::true_type{});
  chunk(c, std::false_type{});
  const unsigned long long t_loop_end = ps.now();
  ps.set(4, t_loop_end - t_loop); ps.set(6, t_loop - t_entry);

  // ---- epilogue: bias, GroupNorm partial sums, 16-B stores. Lane (r, g) of 16 x 16 block (i, cb) holds channels
  // cb*16 + 4g + 0..3 of position r of block i; one v_permlane16_swap per register of the block pair (2rb, 2rb+1) (the
  // two 16-frame halves of row block rb) leaves lane (r, g) with channels cb*16 + 8 (g >> 1) + 0..7 of position
  // 16 (g & 1) + r: one 16-B item and one GroupNorm 8-channel subgroup per lane and pair.
  mfma_drain();
#pragma unroll
  for (int i = 0; i < C::NS; ++i)
#pragma unroll
    for (int j = 0; j < C::NCB; ++j) asm volatile("" : "+v"(acc[i][j]));   // every read of acc stays after the drain
  float gs[C::NCB], gq[C::NCB];
#pragma unroll
  for (int cb = 0; cb < C::NCB; ++cb) { gs[cb] = gq[cb] = 0.f; }
  bf16* out = reinterpret_cast<bf16*>(p.out);
  const int tcol = t0 + (g & 1) * 16 + r;
  const bool valid = tcol < T;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int frow = f0 + wm * RB + rb;
    const long ob = (((long)b * F + frow) * T + tcol) * BN;
#pragma unroll
    for (int cb = 0; cb < C::NCB; ++cb) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * rb][cb][q]),
                                                         __float_as_uint(acc[2 * rb + 1][cb][q]), false, false);
        v[q] = __uint_as_float(sw[0]);
        v[4 + q] = __uint_as_float(sw[1]);
      }
      const int cl = wn * 32 * CB + cb * 16 + 8 * (g >> 1);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(s_bias + cl);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(s_bias + cl + 4);
      float o[8];
      if (w8) {   // wave-uniform
        const f32x4 s0 = *reinterpret_cast<const f32x4*>(s_wsc + cl);
        const f32x4 s1 = *reinterpret_cast<const f32x4*>(s_wsc + cl + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) { o[k] = v[k] * s0[k] + b0[k]; o[4 + k] = v[4 + k] * s1[k] + b1[k]; }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) { o[k] = v[k] + b0[k]; o[4 + k] = v[4 + k] + b1[k]; }
      }
      if (valid) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          gs[cb] += o[k]; gq[cb] += o[k] * o[k];
          asm volatile("" : "+v"(gs[cb]), "+v"(gq[cb]));   // scalar chains (conv.hip, packed-FP32 hazard)
        }
        *reinterpret_cast<uint4*>(out + ob + cl) = f_to_item(o, bf16());
      }
    }
  }
#pragma unroll
  for (int cb = 0; cb < C::NCB; ++cb) {   // over the 32 lanes of each lane half (the subgroup 8 (g >> 1) of block cb)
    const float sm = half_sum32(gs[cb]), sq = half_sum32(gq[cb]);
    if ((lane & 31) == 0) {
      s_sub[((wv * C::NCB + cb) * 2 + (g >> 1)) * 2 + 0] = sm;
      s_sub[((wv * C::NCB + cb) * 2 + (g >> 1)) * 2 + 1] = sq;
    }
  }
  lds_barrier();
  if (tid < 8) {   // per GroupNorm group, over waves and 8-channel sub-groups in a fixed order: one slot per tile
    const int gshift = __builtin_ctz(BN >> 3);
    float S = 0.f, Q = 0.f;
#pragma unroll
    for (int w = 0; w < c3w::NW; ++w)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int g8 = 0; g8 < 4; ++g8) {
          const int co = (w % C::WN) * 32 * CB + cb * 32 + g8 * 8;
          if ((co >> gshift) == tid) {
            S += s_sub[((w * CB + cb) * 4 + g8) * 2 + 0];
            Q += s_sub[((w * CB + cb) * 4 + g8) * 2 + 1];
          }
        }
    const int nparts = n_ft * n_tt;
    float* dst = p.out_part + ((long)b * nparts + ft * n_tt + tt) * 16 + tid * 2;
    dst[0] = S;
    dst[1] = Q;
  }
  ps.set(7, ps.now() - t_loop_end);
  ps.flush(GT_C3W_STAMP_DST, blockIdx.x & 511, 8, wv, lane);
}

// (BN, CB) of a conv on an F-row grid with Cout outputs, or 0 if conv3w does not cover it (shared with conv3w_a8.hip)
int conv3w_cfg(int Cout, int F) {
  if (Cout == 256 && F % 10 == 0) return 1;    // <256, 2>: 10-row tiles (level 2)
  if (Cout == 128 && F % 20 == 0 && F >= 40) return 2;   // <128, 2>: 20-row tiles (level 1)
  if (Cout == 128 && F % 10 == 0) return 3;    // <128, 1>: 10-row tiles (level 2)
  if (Cout == 64 && F % 20 == 0 && F >= 40) return 4;    // <64, 1>: 20-row tiles (level 1)
  return 0;
}
static int c3w_rows(int cfg) { return (cfg == 1 || cfg == 3) ? 10 : 20; }

// shapes and input modes either form (bf16 operands / fp8 operands) covers
static bool c3w_shape_ok(const ConvParams& p, InMode im) {
  if (im != IN_MASK && im != IN_GN && im != IN_PLAIN) return false;
  if (p.small || p.w_bstride || p.Fin != p.Fout || p.Tin != p.Tout) return false;
  if (p.Cin % 32 || p.C0 % 32 || (p.in1 && p.C1 % 32) || p.Cin_pad != p.Cin || p.Cin != p.C0 + (p.in1 ? p.C1 : 0)) return false;
  if (im == IN_GN && p.Cin > 256) return false;
  if (!conv3w_cfg(p.Cout, p.Fout)) return false;
  return (long)p.B * p.Fin * p.Tin * (p.C0 > p.C1 ? p.C0 : p.C1) * 2 < (1L << 31);
}

bool conv3w_eligible(const ConvParams& p, InMode im) { return !p.a8 && c3w_shape_ok(p, im); }
bool conv3w_a8_eligible(const ConvParams& p, InMode im) { return p.a8 && p.wscale && c3w_shape_ok(p, im); }

int conv3w_nparts(int F, int T, int Cout) {
  const int cfg = conv3w_cfg(Cout, F);
  return cfg ? (F / c3w_rows(cfg)) * ((T + 31) / 32) : 0;
}

template <int IN, int BN, int CB>
static hipError_t launch_c3w_t(const ConvParams& p, hipStream_t s) {
  typedef c3w::Cfg<BN, CB> C;
  if (p.Fout % C::TR || p.Cout != BN) return hipErrorInvalidValue;
  const long nsp = (long)p.B * (p.Fout / C::TR) * ((p.Tout + 31) / 32);
  hipLaunchKernelGGL((conv3w_kernel<IN, BN, CB>), dim3((unsigned)(8 * ((nsp + 7) / 8))), dim3(512), 0, s, p);
  return hipGetLastError();
}
template <int BN, int CB>
static hipError_t launch_c3w_in(InMode im, const ConvParams& p, hipStream_t s) {
  if (im == IN_MASK) return launch_c3w_t<IN_MASK, BN, CB>(p, s);
  if (im == IN_GN) return launch_c3w_t<IN_GN, BN, CB>(p, s);
  if (im == IN_PLAIN) return launch_c3w_t<IN_PLAIN, BN, CB>(p, s);
  return hipErrorNotSupported;
}

hipError_t launch_conv3w(InMode im, const ConvParams& p, hipStream_t s) {
  if (!conv3w_eligible(p, im)) return hipErrorInvalidValue;
  switch (conv3w_cfg(p.Cout, p.Fout)) {
    case 1: return launch_c3w_in<256, 2>(im, p, s);
    case 2: return launch_c3w_in<128, 2>(im, p, s);
    case 3: return launch_c3w_in<128, 1>(im, p, s);
    case 4: return launch_c3w_in<64, 1>(im, p, s);
  }
  return hipErrorNotSupported;
}


}  // namespace gt
