// Wide-tile 3x3 convolution with fp8 operands (GT_FP8's throughput plan), gfx950.
//
// The fp8-operand twin of conv3w (conv3w.hip): same convs (Block.block[0], model/diffusion.py:52, at U-Net levels 1-2
// with Cin % 32 == 0), same tiles (one 8-wave workgroup per CU owning all BN = Cout output channels of TR mel rows x 32
// frames), same GroupNorm partial slots -- but the operands are e4m3 and the matrix op is v_mfma_scale_f32_32x32x64_f8f6f4,
// as conv_kernel's A8 form (conv.hip), which it replaces for these shapes. Quantization is conv_kernel's exactly: one
// E8M0 scale per (position, 32-channel block), 2^k with k the least exponent keeping max|x| / 2^k <= 448, the weights
// e4m3 per output channel with their fp32 scale applied in the epilogue. Taps go in pairs (0,1) (2,3) (4,5) (6,7) (8,-):
// one K = 64 MFMA covers two taps x 32 channels; the ninth pair's second half has zero weights and re-reads tap 8.
//
//   * K loop = phases: one phase = one tap pair x 32 input channels, 5 phases per 32-channel chunk. Wave (wn, wm) runs
//     RB = 5 row blocks x CB column blocks of 32 x 32 per phase. A weight slot (BN rows x 2 taps x 32 channels = BN x 64 B)
//     is DMA'd (global_load_lds) into a ring of S = 6 slots, D = 5 phases ahead, one counted vmcnt wait + one barrier
//     per phase (conv3w's pipeline).
//   * The patch is double-buffered per chunk and PLANAR: 2 planes (channels 0-15 / 16-31 of the chunk) of 16-B e4m3
//     entries per position, plus one scale byte per position. A wave's 64 consecutive items are 32 consecutive positions
//     x 2 planes (lane 32h + r: position r, plane h): the two lanes of a position are 32 apart, their |x| maxima meet
//     through one v_permlane32_swap, and 8 contiguous lanes write 128 contiguous bytes of one plane.
//   * Items of the next chunk are transformed behind the MFMAs: the mask / plain forms one whole item per wave at one
//     step (the wave halves staggered, as conv3w), the GroupNorm form a quarter of the item (4 channels) after each of
//     steps 0-3 in every wave, quantized and written at step 3 -- its transform outlasts one wave's phase of MFMAs.
//   * Fragments: lane (r, h) of the patch operand holds plane h of tap t's position (bytes 0-15) and of tap t''s (16-31),
//     with the scale byte of tap t's position (h = 0) or tap t''s (h = 1) -- the operand semantics conv.hip probes; the
//     weight operand the same planes of slot rows. Each is a contiguous 512 B per 32 lanes: conflict-free ds_read_b128.
// Epilogue: acc * weight scale + bias, GroupNorm partial sums of the output (one slot per tile, fixed-order reduction),
// 16-B bf16 stores after v_permlane32_swap (conv3w's 32x32 form).
#include "common.h"
#include "kernels.h"
#include "c3w_asm.h"
#include "stamps.h"

namespace gt {

namespace c3w8 {
constexpr int NTHR = 512, NW = 8, RB = 5, PCOL = 34;
constexpr int NPH = 5;            // phases per 32-channel chunk (tap pairs)
constexpr int S = 6, D = S - 1;   // weight ring slots, DMA distance (D <= NPH: DMA(k + D) exists iff chunk c+1 does or t + D < NPH)
// B fragment prefetch distance in steps (ring of RB by step: chunk-periodic), and phases from an item's load to its
// transform (2 / 2 spilled 5-230 registers: the 160 accumulators leave about 90). Two steps ahead only where it fits and
// paid: the 256-wide mask / plain forms (level-2 mask conv 53.2 -> 52.2 us, same box; the 64/128-wide CB = 1 forms did
// not move, the GroupNorm forms' split transform needs steps 0-3 before the first prefetch read)
constexpr int LAT = 1;
template <int IN, int BN, int CB>
constexpr int pf() { return IN != IN_GN && BN == 256 ? 2 : 1; }

template <int BN, int CB>
struct Cfg {
  static constexpr int WN = BN / (32 * CB);        // waves along output channels
  static constexpr int WM = NW / WN;               // waves along mel rows
  static constexpr int TR = WM * RB;               // tile rows
  static constexpr int PR = TR + 2;                // patch rows
  static constexpr int PP = PR * PCOL;             // patch positions
  static constexpr int PPAD = (PP + 16) & ~15;      // > PP: the scale byte at PP is read (pair 4, below)
  static constexpr int PLANE = PPAD * 16;          // 16 e4m3 channels per entry
  static constexpr int PBUF = 2 * PLANE;           // one 32-channel patch buffer
  static constexpr int SLOT = BN * 64;             // one weight slot: BN rows x 2 taps x 32 channels
  static constexpr int PIECES = SLOT / 1024;
  static constexpr int ITEMS = PP * 2;             // 16-channel items per chunk
  static constexpr int NPT = (ITEMS + NTHR - 1) / NTHR;
  // item j of the next chunk: loaded at phase LP(j), transformed and written at phase TP(j) <= NPH - 2 (the last phase
  // reads the next chunk's first fragments after its top barrier: every item write must precede that barrier)
  static constexpr int TP(int j) { return j + (NPH - 1 - NPT); }
  static constexpr int LP(int j) { return TP(j) >= LAT ? TP(j) - LAT : 0; }
  static constexpr int OFF_S = 2 * PBUF;                      // scale bytes [2][PPAD]
  static constexpr int OFF_W = OFF_S + ((2 * PPAD + 15) & ~15);
  static constexpr int OFF_I = OFF_W + S * SLOT;              // per-thread item words: input index, mask [NPT][NTHR] each
  static constexpr int OFF_F = OFF_I + 2 * NPT * NTHR * 4;     // float area
  // floats: s_sc, s_sh, s_tb [256] each, s_bias [256], s_wsc [256], s_sub [NW][CB][4][2], s_mean, s_rstd [8]
  static constexpr int NF = 5 * 256 + NW * CB * 8 + 16;
  static constexpr int SMEM = OFF_F + NF * 4;
  static_assert(WN * WM == NW && WN >= 1, "wave grid");
  static_assert(PIECES * 1024 == SLOT, "whole DMA pieces");
  static_assert(NPT >= 1 && NPT <= 3 && TP(0) >= 1, "items transformed in phases 1..3");
  static_assert(NTHR / 64 * 32 * NPT >= PP, "item map covers the patch");
  static_assert(SMEM <= 160 * 1024, "LDS budget: one workgroup per CU");
  static_assert(PBUF >= 272 * 8, "s_red aliases patch buffer 1");
};

template <int I, int N, class F>
GT_DEV void sfor(F&& f) {   // f(integral_constant<I>) ... f(integral_constant<N - 1>)
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}
}  // namespace c3w8

#ifndef GT_C3W8_STAMP
#define GT_C3W8_STAMP 0   // diagnostic builds only: s_memtime stamps of the phase waits (gt_diag_conv3w_a8_stamps)
#endif
#ifndef GT_C3W8_STAMP_BN
#define GT_C3W8_STAMP_BN 256
#endif
#ifndef GT_C3W8_STAMP_IN
#define GT_C3W8_STAMP_IN 2
#endif
#ifndef GT_C3W8_STAMP_CB
#define GT_C3W8_STAMP_CB 2
#endif
// stamps.h counters: cycles in the DMA wait, the phase barrier, the item waits, the item transforms + writes, the whole
// chunk loop, phases, prologue, epilogue (the last launch of the stamped instantiation wins)
#if GT_C3W8_STAMP
GT_STAMP_BUFFER(gt_c3w8_stamps, gt_diag_conv3w_a8_stamps, 8)
#define GT_C3W8_STAMP_DST gt_c3w8_stamps
#else
#define GT_C3W8_STAMP_DST nullptr
#endif

typedef int v8i_t __attribute__((ext_vector_type(8)));
struct FragP8 { v8i_t v; int s; };

// v_mfma_scale_f32_32x32x64_f8f6f4 accumulating in place (weights A with E8M0 scale sa, patch B with scale sb; e4m3 both).
// As conv3w's mfma16: the asm form keeps each accumulator in its registers; the operands come from LDS reads waited for
// by the compiler, and mfma_drain waits out the last MFMAs before the epilogue reads an accumulator. The 160 accumulator
// registers stay VGPRs: with two waves per SIMD the unified 512-entry file gives a wave 256 registers in all, and hipcc
// splits them 128 / 128 as soon as AGPRs are used (measured: 300-450 spilled); in VGPRs only the item words' move to
// LDS (s_pidx / s_pm) and one-item-at-a-time transforms were needed.
GT_DEV void mfma8s(f32x16& c, const v8i_t& a, const v8i_t& b, int sa, int sb) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0]"
               : "+v"(c) : "v"(a), "v"(b), "v"(sa), "v"(sb));
}

// IN: IN_MASK (x * mask), IN_GN ((Mish(GN(h)) + tb) * mask), IN_PLAIN. OUT: OUT_STATS.
template <int IN, int BN, int CB>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void conv3w_a8_kernel(ConvParams p) {
  typedef c3w8::Cfg<BN, CB> C;
  using c3w8::NTHR; using c3w8::RB; using c3w8::PCOL; using c3w8::NPH; using c3w8::D; using c3w8::S;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];   // ONE LDS object
  float* const s_sc = reinterpret_cast<float*>(smem + C::OFF_F);
  float* const s_sh = s_sc + 256;
  float* const s_tb = s_sh + 256;
  float* const s_bias = s_tb + 256;
  float* const s_wsc = s_bias + 256;
  float* const s_sub = s_wsc + 256;
  float* const s_mean = s_sub + c3w8::NW * CB * 8;
  float* const s_rstd = s_mean + 8;
  unsigned char* const s_psc = reinterpret_cast<unsigned char*>(smem + C::OFF_S);
  double* const s_red = reinterpret_cast<double*>(smem + C::PBUF);   // patch buffer 1 is free until chunk 0's items
  // item input index and mask, per thread: read back where used instead of held in registers across the loop (the
  // 160 accumulator registers leave none to spare)
  int* const s_pidx = reinterpret_cast<int*>(smem + C::OFF_I);
  float* const s_pm = reinterpret_cast<float*>(smem + C::OFF_I + C::NPT * NTHR * 4);

  const int F = p.Fout, T = p.Tout;
  const int n_ft = F / C::TR, n_tt = (T + 31) / 32;
  const int nsp = p.B * n_ft * n_tt;
  int bid = (blockIdx.x & 7) * ((nsp + 7) >> 3) + (blockIdx.x >> 3);   // XCD-aware order (conv3w)
  if (bid >= nsp) return;   // grid padding: the whole workgroup, before any barrier
  const int tt = bid % n_tt; bid /= n_tt;
  const int ft = bid % n_ft;
  const int b = bid / n_ft;
  const int f0 = ft * C::TR, t0 = tt * 32;
  constexpr bool STAMP = GT_C3W8_STAMP && BN == GT_C3W8_STAMP_BN && IN == GT_C3W8_STAMP_IN && CB == GT_C3W8_STAMP_CB;
  Stamps<STAMP> ps;
  const unsigned long long t_entry = ps.now();

  // v_mfma_*_32x32x64 lanes: r = row of A (output channel) / column of B (position), h = the 16-channel plane
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wv % C::WN, wm = wv / C::WN;
  auto item_pos = [&](int j) { return (((tid + NTHR * j) >> 6) << 5) | r; };
  const int item_wbase = h * C::PLANE + item_pos(0) * 16;

  // ---- prologue loads: GroupNorm slots (IN_GN), per-channel coefficients, bias, weight scale, masks
  GnLoad gl;
  if (IN == IN_GN) gl = gn_load(p.gn_part, p.gn_nparts, b);
  float c_g = 0.f, c_b = 0.f, c_t = 0.f;
  if (IN == IN_GN && tid < p.Cin) {
    c_g = p.gn_gamma[tid]; c_b = p.gn_beta[tid]; c_t = tb_at(p.tb, p.stepp)[(long)b * p.tb_bstride + tid];
  }
  const float c_bias = tid < BN ? p.bias[tid] : 0.f;
  const float c_wsc = tid < BN ? p.wscale[tid] : 1.f;

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
    s_pidx[j * NTHR + tid] = qi;
    s_pm[j * NTHR + tid] = pm[j];
  }
  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.in0, (short)0, npos * p.C0 * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.in1 ? p.in1 : p.in0), (short)0, npos * (p.in1 ? p.C1 : p.C0) * 2, 0x00020000);
  const int nchunk = p.Cin / 32;
  const int K = nchunk * NPH;

  // item j = 16 bf16 channels (two 16-B loads) of one position; the next chunk's by inline asm (counted waits)
  u32x4c_t preg[C::NPT][2];
  auto load_item = [&](int c, int j) {
    const int c0 = c * 32;
    const bool first = c0 < p.C0;
    const int pb = (first ? p.C0 : p.C1) * 2;
    const int so = __builtin_amdgcn_readfirstlane((first ? c0 : c0 - p.C0) * 2);
    asm_buffer_load2(preg[j][0], preg[j][1], s_pidx[j * NTHR + tid] * pb + h * 32, first ? rs0 : rs1, so);
  };
  auto load_patch = [&](int c) {   // every item (prologue: hipcc-visible loads)
    const int c0 = c * 32;
    const bool first = c0 < p.C0;
    const int pb = (first ? p.C0 : p.C1) * 2;
    const int so = (first ? c0 : c0 - p.C0) * 2;
#pragma unroll
    for (int j = 0; j < C::NPT; ++j) {
      preg[j][0] = __builtin_amdgcn_raw_buffer_load_b128(first ? rs0 : rs1, pidx[j] * pb + h * 32, so, 0);
      preg[j][1] = __builtin_amdgcn_raw_buffer_load_b128(first ? rs0 : rs1, pidx[j] * pb + h * 32 + 16, so, 0);
    }
  };
  // transform item j of chunk c, quantize (conv.hip store_item_a8's arithmetic) and write it with its scale byte
  // GroupNorm + Mish + time bias of channels 4p .. 4p+3 of item j (chunk c) into v[4p ..]
  auto gn_part = [&](int j, int c, int p, float* v) {
    const unsigned w0 = preg[j][p >> 1][2 * (p & 1)], w1 = preg[j][p >> 1][2 * (p & 1) + 1];
    const float x[4] = {__uint_as_float(w0 << 16), __uint_as_float(w0 & 0xffff0000u),
                        __uint_as_float(w1 << 16), __uint_as_float(w1 & 0xffff0000u)};
    const int ch = c * 32 + h * 16 + 4 * p;
    const f32x4 sc = *reinterpret_cast<const f32x4*>(s_sc + ch);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(s_sh + ch);
    const f32x4 tb = *reinterpret_cast<const f32x4*>(s_tb + ch);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[4 * p + k] = gn_mish_tb_l2(x[k], sc[k], sh[k], tb[k]);
  };
  // quantize item j's 16 transformed channels (conv.hip store_item_a8's arithmetic) and write them with the scale byte
  auto finish_item = [&](int j, int buf, float* v) {
    if ((IN == IN_GN || IN == IN_MASK) && frac) {
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] *= s_pm[j * NTHR + tid];
    }
    float am = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) am = fmaxf(am, fabsf(v[k]));
    {   // the other plane of this position: lane ^ 32
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(am), __float_as_uint(am), false, false);
      am = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    const unsigned ab = __float_as_uint(am);
    int e = (int)(ab >> 23) - 8 + ((ab & 0x7fffffu) > 0x600000u ? 1 : 0);   // max|x| <= 1.75 * 2^(8 + k)
    e = ab == 0u ? 127 : (e < 1 ? 1 : e);
    const float scl = __uint_as_float((unsigned)e << 23);
    // IN_GN, masks in {0, 1}: a masked position's bytes are zeroed after the conversion (conv_kernel's rule)
    const bool zero = IN == IN_GN && !frac && s_pm[j * NTHR + tid] == 0.f;
    typedef short v2s __attribute__((ext_vector_type(2)));
    u32x4c_t q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v2s o = {0, 0};
      o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, v[4 * i], v[4 * i + 1], scl, false);
      o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, v[4 * i + 2], v[4 * i + 3], scl, true);
      q[i] = zero ? 0u : __builtin_bit_cast(unsigned, o);
    }
    // item j's position = item 0's + 256 j: one base register, compile-time offsets
    if (item_pos(j) < C::PP) {
      *reinterpret_cast<u32x4c_t*>(smem + buf * C::PBUF + item_wbase + j * 256 * 16) = q;
      if (h == 0) s_psc[buf * C::PPAD + (item_wbase >> 4) + j * 256] = (unsigned char)e;   // h = 0: wbase = 16 pos
    }
  };
  // the whole item at once (prologue; the mask / plain forms in the loop)
  auto put_item = [&](int j, int c, int buf) {
    float v[16];
    if (IN == IN_GN) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        gn_part(j, c, p, v);
        asm volatile("" ::: "memory");   // one coefficient group in registers at a time (register budget)
      }
    } else {
      item_to_f(make_uint4(preg[j][0][0], preg[j][0][1], preg[j][0][2], preg[j][0][3]), v, bf16());
      item_to_f(make_uint4(preg[j][1][0], preg[j][1][1], preg[j][1][2], preg[j][1][3]), v + 8, bf16());
    }
    finish_item(j, buf, v);
  };

  // weight DMA: slot of phase k = image bytes [k SLOT, (k+1) SLOT) (decoder.cpp pack_conv3w_a8); every wave issues PW
  // pieces per slot (BN = 64: waves 4..7 repeat waves 0..3's), so the counted waits are the same in every wave
  constexpr int PW = C::PIECES >= c3w8::NW ? C::PIECES / c3w8::NW : 1;
  static_assert(C::PIECES % c3w8::NW == 0 || c3w8::NW % C::PIECES == 0, "pieces split evenly");
  const char* const wimg = reinterpret_cast<const char*>(p.w);
  const unsigned lds_base = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(smem));
  const unsigned dma_voff = lane * 16;
  auto dma = [&](int k, int slot) {
    const char* src = wimg + (long)k * C::SLOT;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int piece = C::PIECES >= c3w8::NW ? wv + c3w8::NW * i : wv % C::PIECES;
      asm_dma16(src + piece * 1024, dma_voff, lds_base + C::OFF_W + slot * C::SLOT + piece * 1024);
    }
  };
  constexpr auto n_lp = [](int lo, int hi) {   // items loaded at phases [lo, hi]
    int n = 0;
    for (int j = 0; j < C::NPT; ++j) n += (C::LP(j) >= lo && C::LP(j) <= hi) ? 1 : 0;
    return n;
  };
  // VMEM ops a wave issues after item j's loads, up to its wait at the top of phase TP(j): the DMAs of phases
  // LP(j)+1 .. TP(j) and the items loaded after j up to that phase (each phase: DMA, item loads, wait); PW ops per DMA,
  // 2 per item
  constexpr auto n_after = [](int j) {
    int n = (C::TP(j) - C::LP(j)) * PW;
    for (int i = j + 1; i < C::NPT; ++i)
      if (C::LP(i) <= C::TP(j)) n += 2;
    return n;
  };
  // LDS reads of the next phase issued before its barrier: its first PF steps' B (2 x b128 + 1 byte each) and its A
  // (pair 4's second tap is its first again: one b128 fewer, rd_b)
  constexpr int PF = c3w8::pf<IN, BN, CB>();
  static_assert(PF >= 1 && PF < RB, "prefetch distance");
  constexpr auto npre = [](int pr) { return PF * (pr == 4 ? 2 : 3) + 2 * CB; };

  // ---- fragments. A (weights): plane q = 2u + h of the slot, row; B (patch): plane h, position; scale byte of tap t
  // (h = 0) or t' (h = 1): t' - t = +1 column, except pair 1 (tap 3 opens the next row) and pair 4 (t' = t = 8)
  const int a_lane = C::OFF_W + (h * BN + wn * 32 * CB + r) * 16;
  const int pos_lane = wm * RB * PCOL + r;
  const int b_lane = h * C::PLANE + pos_lane * 16;
  const int sd1 = h, sd2 = h ? PCOL - 2 : 0;
  auto tap_off = [](int t) { t = t > 8 ? 8 : t; return (t / 3) * PCOL + t % 3; };
  auto rd_a = [&](int slot, int cb) {
    const char* base = smem + a_lane + slot * C::SLOT + cb * 32 * 16;
    const u32x4c_t lo = *reinterpret_cast<const u32x4c_t*>(base);
    const u32x4c_t hi = *reinterpret_cast<const u32x4c_t*>(base + 2 * BN * 16);
    return v8i_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  auto rd_b = [&](int buf, int pr, int rb) {   // tap pair pr, row block rb
    const char* base = smem + b_lane + buf * C::PBUF + rb * PCOL * 16;
    const u32x4c_t lo = *reinterpret_cast<const u32x4c_t*>(base + tap_off(2 * pr) * 16);
    const u32x4c_t hi = pr == 4 ? lo : *reinterpret_cast<const u32x4c_t*>(base + tap_off(2 * pr + 1) * 16);
    FragP8 f;
    f.v = v8i_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    // pair 4's second tap is the zero-weight slot 9: any valid scale serves its lanes h = 1, so they take tap 8's
    // position + 1 as pairs 0, 2, 3 do (at most position PP, a pad byte set to 127 in the prologue)
    const int sd = pr == 1 ? sd2 : sd1;
    f.s = s_psc[buf * C::PPAD + pos_lane + sd + rb * PCOL + tap_off(2 * pr)];
    return f;
  };

  // ---- prologue: chunk 0 patch loads, the first D weight slots, the GroupNorm reduction
  load_patch(0);
#pragma unroll
  for (int k = 0; k < D; ++k)
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
  if (tid < 2 * (C::PPAD - C::PP)) s_psc[(tid & 1) * C::PPAD + C::PP + (tid >> 1)] = 127;   // pad scale bytes: 2^0
  lds_barrier();
#pragma unroll
  for (int j = 0; j < C::NPT; ++j) put_item(j, 0, 0);
  vm_wait<(D - 2) * PW>();   // DMA(0), DMA(1) landed (younger: DMA(2 .. D-1); K >= NPH >= D)
  lds_barrier();

  f32x16 acc[RB][CB];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) {
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;
      asm volatile("" : "+v"(acc[i][j]));   // zeros written here, after the prologue, ahead of the wait states below
    }
  int scale_one = 127;   // the weight operand's E8M0 1.0 (its per-channel fp32 scale is applied in the epilogue)
  asm volatile("" : "+v"(scale_one));
  asm volatile("s_nop 7" ::: "memory");   // VALU writes -> MFMA operand reads (mfma8s pads nothing)

  v8i_t fa[CB];
  FragP8 fb[RB];   // B ring by step index (a phase is RB steps, so step i of every phase uses entry i)
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) fa[cb] = rd_a(0, cb);
#pragma unroll
  for (int n = 0; n < PF; ++n) fb[n] = rd_b(0, 0, n);

  int slot = 0;
  // steps of the item transforms: waves 0-3 / 4-7 (conv3w's stagger); both before step RB - PF, whose B read is the first
  // of the NPRE reads the next barrier may leave in flight (the item write must be older)
  constexpr int XS0 = 0, XS1 = RB - PF - 1;
  // GroupNorm form: the item transform spread over MFMA steps 0-3 (measured against the staggered whole-item form:
  // 0.4-1.6 % faster per GN launch, 12 fewer VGPRs)
  constexpr bool SPLIT = IN == IN_GN;
  static_assert(!SPLIT || 3 <= RB - PF - 1, "the split transform's write precedes the next phase's prefetch reads");
  float vit[16];   // SPLIT: the item's transformed channels between its steps
  auto chunk = [&](int c, auto MOREc) {
    constexpr bool MORE = decltype(MOREc)::value;
    const int cur = c & 1, nxt = cur ^ 1;
    const int k0 = c * NPH;
    c3w8::sfor<0, NPH>([&](auto Tc) {
      constexpr int t = decltype(Tc)::value;
      const int k = k0 + t;
      {   // (a) DMA(k+1) landed, every LDS access of phase k-1 but the NPRE prefetch reads done, one barrier
        constexpr int ndma0 = MORE ? D - 2 : ((NPH - t - 2) < (D - 2) ? (NPH - t - 2) : (D - 2));
        constexpr int ndma = ndma0 > 0 ? ndma0 : 0;
        constexpr int npl = MORE ? 2 * n_lp(t + 1 - D, t - 1) : 0;
        const unsigned long long s0 = ps.now();
        vm_wait<ndma * PW + npl>();
        const unsigned long long s1 = ps.now();
        asm volatile("s_waitcnt lgkmcnt(%0)\n\ts_barrier" :: "n"(npre(t)) : "memory");
        ps.add(0, s1 - s0); ps.add(1, ps.now() - s1); ps.add(5, 1);
      }
      int nslot = slot + 1;
      nslot = nslot == S ? 0 : nslot;
      if (MORE || t + D < NPH) {   // (b) DMA of phase k + D into the slot phase k - 1 used
        int ds = slot + D;
        ds = ds >= S ? ds - S : ds;
        dma(k + D, ds);
      }
      if constexpr (MORE) {   // (c) the next chunk's item loads of this phase, and the wait for this phase's item:
        // unconditional in every wave (an asm load whose wait a wave skipped would land in a reused register)
        c3w8::sfor<0, C::NPT>([&](auto Jc) {
          constexpr int j = decltype(Jc)::value;
          if constexpr (C::LP(j) == t) load_item(c + 1, j);
        });
        c3w8::sfor<0, C::NPT>([&](auto Jc) {
          constexpr int j = decltype(Jc)::value;
          if constexpr (C::TP(j) == t) {
            const unsigned long long s0 = ps.now();
            vm_wait_dep2<n_after(j)>(preg[j][0], preg[j][1]);
            ps.add(2, ps.now() - s0);
          }
        });
      }
      // (d) MFMAs of phase k: step i = row block i, CB MFMAs; B read PF steps ahead (into phase k+1 for the last PF)
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int n = i + PF;
        if (n < RB) fb[n] = rd_b(cur, t, n);
        else if (MORE || t < NPH - 1) fb[n - RB] = t < NPH - 1 ? rd_b(cur, t + 1, n - RB) : rd_b(nxt, 0, n - RB);
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) mfma8s(acc[i][cb], fa[cb], fb[i].v, scale_one, fb[i].s);
        if (i == RB - 1 && (MORE || t < NPH - 1)) {   // phase k+1's A fragments, after this phase's last use
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) fa[cb] = rd_a(nslot, cb);
        }
        // (e) this phase's item of chunk c+1 (waited for at the phase top), behind the MFMAs. Mask / plain forms: the
        // whole item at one step, staggered between the wave halves (conv3w's stagger). GroupNorm form (SPLIT): its
        // transform outlasts a phase's MFMAs of one wave, so every wave runs a quarter of it (4 channels) after each of
        // steps 0-3 and quantizes + writes at step 3, between MFMAs instead of in one block
        if constexpr (MORE) {
          if constexpr (SPLIT) {
            if (i < 4) {
              c3w8::sfor<0, C::NPT>([&](auto Jc) {
                constexpr int j = decltype(Jc)::value;
                if constexpr (C::TP(j) == t) {
                  const unsigned long long s0 = ps.now();
                  gn_part(j, c + 1, i, vit);
                  if (i == 3) finish_item(j, nxt, vit);
                  asm volatile("" ::: "memory");
                  ps.add(3, ps.now() - s0);
                }
              });
            }
          } else if ((i == XS0 && wv < c3w8::NW / 2) || (i == XS1 && wv >= c3w8::NW / 2)) {
            c3w8::sfor<0, C::NPT>([&](auto Jc) {
              constexpr int j = decltype(Jc)::value;
              if constexpr (C::TP(j) == t) {
                const unsigned long long s0 = ps.now();
                put_item(j, c + 1, nxt);
                asm volatile("" ::: "memory");
                ps.add(3, ps.now() - s0);
              }
            });
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      slot = nslot;
    });
  };
  int c = 0;
  const unsigned long long t_loop = ps.now();
  for (; c + 1 < nchunk; ++c) chunk(c, std::true_type{});
  chunk(c, std::false_type{});
  const unsigned long long t_loop_end = ps.now();

  // ---- epilogue: lane (r, h) of block (rb, cb) holds channels cb*32 + {0-3, 8-11, 16-19, 24-27} + 4h of position r;
  // v_permlane32_swap leaves it 8 consecutive channels per 16-channel half
  mfma_drain();
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) asm volatile("" : "+v"(acc[i][j]));   // every read of acc stays after the drain
  float gs[CB][2], gq[CB][2];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) { gs[cb][0] = gs[cb][1] = gq[cb][0] = gq[cb][1] = 0.f; }
  bf16* out = reinterpret_cast<bf16*>(p.out);
  const int tcol = t0 + r;
  const bool valid = tcol < T;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int frow = f0 + wm * RB + rb;
    const long ob = (((long)b * F + frow) * T + tcol) * BN;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = acc[rb][cb][q];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[8 * pr + q]),
                                                           __float_as_uint(v[8 * pr + 4 + q]), false, false);
          v[8 * pr + q] = __uint_as_float(sw[0]);
          v[8 * pr + 4 + q] = __uint_as_float(sw[1]);
        }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int cl = wn * 32 * CB + cb * 32 + pr * 16 + 8 * h;
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(s_bias + cl);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(s_bias + cl + 4);
        const f32x4 s0 = *reinterpret_cast<const f32x4*>(s_wsc + cl);
        const f32x4 s1 = *reinterpret_cast<const f32x4*>(s_wsc + cl + 4);
        float o[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) { o[k] = v[8 * pr + k] * s0[k] + b0[k]; o[4 + k] = v[8 * pr + 4 + k] * s1[k] + b1[k]; }
        if (valid) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            gs[cb][pr] += o[k]; gq[cb][pr] += o[k] * o[k];
            asm volatile("" : "+v"(gs[cb][pr]), "+v"(gq[cb][pr]));   // scalar chains (conv.hip, packed-FP32 hazard)
          }
          *reinterpret_cast<uint4*>(out + ob + cl) = f_to_item(o, bf16());
        }
      }
    }
  }
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const float sm = half_sum32(gs[cb][pr]), sq = half_sum32(gq[cb][pr]);
      if (r == 0) {
        s_sub[((wv * CB + cb) * 4 + pr * 2 + h) * 2 + 0] = sm;
        s_sub[((wv * CB + cb) * 4 + pr * 2 + h) * 2 + 1] = sq;
      }
    }
  lds_barrier();
  if (tid < 8) {   // per GroupNorm group, over waves and 8-channel sub-groups in a fixed order: one slot per tile
    const int gshift = __builtin_ctz(BN >> 3);
    float Ssum = 0.f, Qsum = 0.f;
#pragma unroll
    for (int w = 0; w < c3w8::NW; ++w)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int g8 = 0; g8 < 4; ++g8) {
          const int co = (w % C::WN) * 32 * CB + cb * 32 + g8 * 8;
          if ((co >> gshift) == tid) {
            Ssum += s_sub[((w * CB + cb) * 4 + g8) * 2 + 0];
            Qsum += s_sub[((w * CB + cb) * 4 + g8) * 2 + 1];
          }
        }
    const int nparts = n_ft * n_tt;
    float* dst = p.out_part + ((long)b * nparts + ft * n_tt + tt) * 16 + tid * 2;
    dst[0] = Ssum;
    dst[1] = Qsum;
  }
  ps.set(4, t_loop_end - t_loop); ps.set(6, t_loop - t_entry); ps.set(7, ps.now() - t_loop_end);
  ps.flush(GT_C3W8_STAMP_DST, blockIdx.x & 511, 8, wv, lane);
}

template <int IN, int BN, int CB>
static hipError_t launch_c3w8_t(const ConvParams& p, hipStream_t s) {
  typedef c3w8::Cfg<BN, CB> C;
  if (p.Fout % C::TR || p.Cout != BN) return hipErrorInvalidValue;
  const long nsp = (long)p.B * (p.Fout / C::TR) * ((p.Tout + 31) / 32);
  hipLaunchKernelGGL((conv3w_a8_kernel<IN, BN, CB>), dim3((unsigned)(8 * ((nsp + 7) / 8))), dim3(512), 0, s, p);
  return hipGetLastError();
}
template <int BN, int CB>
static hipError_t launch_c3w8_in(InMode im, const ConvParams& p, hipStream_t s) {
  if (im == IN_MASK) return launch_c3w8_t<IN_MASK, BN, CB>(p, s);
  if (im == IN_GN) return launch_c3w8_t<IN_GN, BN, CB>(p, s);
  if (im == IN_PLAIN) return launch_c3w8_t<IN_PLAIN, BN, CB>(p, s);
  return hipErrorNotSupported;
}

hipError_t launch_conv3w_a8(InMode im, const ConvParams& p, hipStream_t s) {
  if (!conv3w_a8_eligible(p, im)) return hipErrorInvalidValue;
  switch (conv3w_cfg(p.Cout, p.Fout)) {
    case 1: return launch_c3w8_in<256, 2>(im, p, s);
    case 2: return launch_c3w8_in<128, 2>(im, p, s);
    case 3: return launch_c3w8_in<128, 1>(im, p, s);
    case 4: return launch_c3w8_in<64, 1>(im, p, s);
  }
  return hipErrorNotSupported;
}


}  // namespace gt
