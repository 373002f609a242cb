// Persistent, register-resident-weight 3x3 convolution for the 64-channel U-Net levels (bf16).
//
// Covers Block.block[0] (model/diffusion.py:52) whenever Cin = Cout = 64: the second conv of the level-0
// ResnetBlocks, the final block (level 0) and the 64-channel up-path blocks at level 1 -- convs that are
// HBM- and MFMA-balanced (≈40 µs each at B = 32, T = 512) but that conv_kernel runs 3-5x slower: each of its
// 5120 short-lived tiles restages the 78 KB weight image from L2 (≈400 MB of L2->LDS traffic per launch) and
// pays its prologue/epilogue for only 4 K-chunks.
//
// Structure (4-wave workgroups, two per CU; one workgroup = one SEGMENT: L consecutive 4-row x 32-frame tiles
// walking down the mel axis of one utterance's 32-frame column):
//   * weights stay RESIDENT for the whole launch: wave w owns output channels 32*(w&1) .. +31 and holds their
//     4 chunks x 8 (IN_GN: 7) taps of A fragments in VGPRs, the other taps in LDS, loaded once from a
//     fragment-ordered image (decoder.cpp pack_conv64) -- no weight traffic after the prologue;
//   * wave w computes mel rows 2(w>>1) and 2(w>>1)+1 of each tile, one row per pass: one 32x32 accumulator,
//     36 MFMAs (v_mfma_f32_32x32x16_bf16, weights as A, patch positions as B -> C = channel x position);
//   * the input lives in a RING of 10 patch rows (34 positions x 64 channels, 144-B rows: conflict-free
//     fragment reads): tile k reads rows 4k .. 4k+5; while its MFMAs run, the same waves store the 4 new rows of
//     tile k+1 (from registers, one 16-B item per K-chunk, with the producer's GroupNorm apply + Mish + time
//     bias + mask for IN_GN, or x * mask) and issue the raw buffer loads of tile k+2's rows (padding reads
//     past the end of the tensor and returns zeros). Every input row is staged once per segment: 1.06x the
//     compulsory reads (2 halo columns) instead of the 1.59x of independent 4 x 32 tiles. One LDS barrier per
//     tile; the two workgroups of a CU drift out of phase, so one's staging VALU overlaps the other's MFMAs;
//   * epilogue from the accumulators: one v_permlane32_swap per register pair leaves each lane with 8
//     consecutive output channels (= one GroupNorm group) of one position -> bias, 16-B stores and the
//     GroupNorm partial sums (DPP row sums + one v_permlane16_swap), no LDS transposition.
// GroupNorm partial slots: ONE per segment (conv64_nparts: 16 per utterance at level 0, T = 512, instead of
// 160 for conv_kernel's tiles), accumulated per lane tile by tile in a fixed order and reduced once at the end --
// the consumers' per-workgroup slot reduction shrinks accordingly. The segment length depends only on the grid
// height, so results are deterministic and batch-invariant.
#include "common.h"
#include "kernels.h"
#include "wimage.h"
#include "stamps.h"

namespace gt {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

#ifndef GT_C64_STAMP
#define GT_C64_STAMP 0  // diagnostic builds only: s_memtime stamps (gt_diag_conv64_stamps), instantiation GT_C64_STAMP_IN, F = 80
#endif
#ifndef GT_C64_STAMP_IN
#define GT_C64_STAMP_IN 1
#endif

namespace c64 {
constexpr int TF = 4, TT = 32, PC = TT + 2;               // tile: 4 mel rows x 32 frames; patch rows of 34 positions
constexpr int POSB = 144;                                 // 128 B of channels + 16 B pad (conflict-free fragments)
constexpr int ROWB = PC * POSB;                           // 4896 B per patch row
constexpr int RING = 10;                                  // patch rows resident: 6 of the current tile + 4 of the next
constexpr int NTHR = 256, NW = 4;
constexpr int NEW_ITEMS = 4 * PC * 8;                     // 16-B items of the 4 new rows per tile: 1088
constexpr int PPT = (NEW_ITEMS + NTHR - 1) / NTHR;        // 5 (the 5th only for threads < 64)
constexpr int COLD_ITEMS = 6 * PC * 8;                    // first tile of a segment: all 6 rows
constexpr int CPT = (COLD_ITEMS + NTHR - 1) / NTHR;       // 7
constexpr int NCH = 4;                                    // 16-channel chunks
constexpr int WLDS_MAX = 3;                               // taps whose weights live in LDS (the rest in registers)
constexpr int WTAP_B = 2 * NCH * 64 * 16;                 // one tap's fragments of both channel halves: 8 KB
constexpr int SMEM = RING * ROWB + WLDS_MAX * WTAP_B + (2 * 4 * 64 + 64 + 64 + NW * 8 + 16) * 4 + 272 * 8;
// taps in registers: 8 (128 VGPRs); 7 for the GroupNorm-input variant, whose operand transform needs the room; 6 for
// IN_RB0 (the ResnetBlock-output transform plus each in-flight item's input channels)
constexpr int wreg_of(int in) { return in == IN_RB0 ? 6 : (in == IN_GN || in == IN_X0) ? 7 : 8; }
static_assert(9 - wreg_of(IN_RB0) <= WLDS_MAX && 9 - wreg_of(IN_GN) <= WLDS_MAX, "LDS weight taps");
// IN_X0: the U-Net input {mu, x_t} * m as bf16 pairs (one dword per position) in a window ring of XR rows x XC frames
// (t0 - 2 .. t0 + 33: the 34 patch columns and their 3x3 neighbourhood)
constexpr int XC = 36, XR = 12, XBYTES = XR * XC * 4;
constexpr int smem_of(int in) { return in == IN_X0 ? SMEM + XBYTES : SMEM; }
static_assert(SMEM <= 80 * 1024 && SMEM + XBYTES <= 80 * 1024, "LDS budget: two workgroups per CU");

// The U-Net input conv (Block(2, 64).block[0], diffusion.py:52, 181: 3x3 over {mu, x_t} * m) for 32 positions x 32 output
// channels as two v_mfma_f32_32x32x16_bf16 over K = taps x 2 channels: lane half h of k-step 0 holds taps (h, 0..2) and
// (2, h), k-step 1 tap (2, 2) in half 0 (decoder.cpp pack_x0 orders the A fragments a0, a1 the same way). Lane (r, h)
// supplies the B column of its position: window rows r1 (its row - 1 + h) and r2 (its row + 1), window column c = its
// frame - (t0 - 2) - 1. Accumulates onto acc (the bias, in accumulator layout): register q = channel acc_row(q, h).
GT_DEV f32x16 x0_mfma(const uint32_t* sX, int r1, int r2, int c, int h, const bf16x8& a0, const bf16x8& a1, f32x16 acc) {
  const uint32_t* p1 = sX + r1 * XC + c;
  const uint32_t* p2 = sX + r2 * XC + c;
  const u32x4_t b0 = {p1[0], p1[1], p1[2], p2[h]};
  const uint32_t t8 = p2[2];
  const u32x4_t b1 = {h ? 0u : t8, 0u, 0u, 0u};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, __builtin_bit_cast(bf16x8, b0), acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, __builtin_bit_cast(bf16x8, b1), acc, 0, 0, 0);
}
// x0 = bf16({mu, x_t} * m) of one position (the unfused input conv's operand rounding), 0 outside the grid
GT_DEV uint32_t x0_pair(float mu, float xt, float m) { return pack_bf16x2(mu * m, xt * m); }
}  // namespace c64

// IN: IN_MASK / IN_GN / IN_PLAIN / IN_RB0. Masks from sequence_mask are 0/1: x * m is then a select, decided per item
// on the device (a fractional mask value takes a multiply in a branch that 0/1 masks never enter).
// IN_RB0 (downs.0.1's block1, diffusion.py:70-79, 192): the operand x * m with x = the first ResnetBlock's output
// r0 = Mish(GN(h2)) * m + res_conv(in * m) (in = {mu, x_t, spk}, 2-3 channels) formed per staged item from h2, in the
// same fp32 operations as gn_mish_kernel<RES = 1> (misc.hip, the pass it replaces), so r0 -- which this kernel also
// writes once per position for the residual of downs.0.1 (attn_kv) -- is bit-identical to that pass's output.
// One workgroup = one segment: L consecutive 4 x 32 tiles down the mel axis of one utterance's 32-frame column.
// Two workgroups share a CU (one wave of each per SIMD) and drift out of phase, so one's staging/epilogue VALU
// work overlaps the other's MFMAs.
// W8: fp8 weights (GT_BF16_W8 / GT_FP8) -- the image holds the e4m3 values (exact in bf16) and p.wscale the
// per-output-channel scale: the accumulator starts at bias / scale and the epilogue multiplies by the scale.
// stamps.h counters (4 waves): prologue, loop, barrier wait, pass MFMA streams, pass epilogues, tiles, segment end, unused
#if GT_C64_STAMP
GT_STAMP_BUFFER(gt_c64_stamps, gt_diag_conv64_stamps, 4)
#define GT_C64_STAMP_DST gt_c64_stamps
#else
#define GT_C64_STAMP_DST nullptr
#endif

template <int IN, bool W8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv64_kernel(ConvParams p, int L) {
  using namespace c64;
  __shared__ __attribute__((aligned(16))) char smem[smem_of(IN)];   // one LDS object
  char* const sR = smem;                                     // ring of RING patch rows
  constexpr int WREG = wreg_of(IN);
  char* const sWL = smem + RING * ROWB;                      // [tap - WREG][cb][chunk][lane] LDS-resident A fragments
  float* const s_coef = reinterpret_cast<float*>(smem + RING * ROWB + WLDS_MAX * WTAP_B);   // [scale, shift, tb, x0 bias][64]
  float* const s_wsc = s_coef + 2 * 4 * 64;                  // W8: per-output-channel weight scales
  float* const s_bias = s_wsc + 64;                         // the conv bias in accumulator layout, per (cb, h)
  float* const s_sub = s_bias + 64;                         // [wave][(pr, h) group][sum, sq]
  float* const s_mean = s_sub + NW * 8;
  float* const s_rstd = s_mean + 8;
  double* const s_red = reinterpret_cast<double*>(s_rstd + 8);
  uint32_t* const sX = reinterpret_cast<uint32_t*>(smem + SMEM);   // IN_X0: the {mu, x_t} window ring

  Stamps<GT_C64_STAMP && IN == GT_C64_STAMP_IN && !W8> stp(p.Fout == 80);
  const unsigned long long t_entry = stp.now();
  const int tid = threadIdx.x & 255, lane = tid & 63, r = lane & 31, h = lane >> 5;   // (range known: 256 threads)
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: ring-row addressing stays scalar
  const int cb = wv & 1, rp = wv >> 1;   // output channels cb*32.., mel rows 2 rp, 2 rp + 1 of the tile
  const int F = p.Fout, T = p.Tout;
  const int n_ft = F / TF, n_tt = (T + TT - 1) / TT;
  const int kseg = n_ft / L;                                 // segments per column
  const int seg = blockIdx.x;
  const int col = seg / kseg, part = seg - col * kseg;
  const int b = col / n_tt, tt = col - b * n_tt;
  const int ft0 = part * L;

  // ---- weights -> registers: A fragment (ch, tap) = output channel cb*32 + r, input channels 16 ch + 8h .. +7,
  // from the fragment-ordered image (decoder.cpp pack_conv64): one contiguous 1 KiB per wave instruction
  // (taps 0..WREG-1 in VGPRs; the others from LDS, 4 extra ds_read_b128 per tap and pass, leaving registers for the
  // staging)
  bf16x8 wf[NCH][WREG];
  {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(p.w) + cb * NCH * 9 * 64 + lane;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
      for (int tap = 0; tap < WREG; ++tap) wf[ch][tap] = src[(ch * 9 + tap) * 64];
      if (wv < 2)
#pragma unroll
        for (int tap = WREG; tap < 9; ++tap)
          reinterpret_cast<bf16x8*>(sWL + (tap - WREG) * WTAP_B)[(cb * NCH + ch) * 64 + lane] = src[(ch * 9 + tap) * 64];
    }
  }
  const char* const wlp = sWL + (cb * NCH * 64 + lane) * 16;
  bf16x8 xa0, xa1;   // IN_X0: the input conv's A fragments of this wave's channel half (k-steps 0, 1)
  if (IN == IN_X0) {
    xa0 = reinterpret_cast<const bf16x8*>(p.x0w)[(cb * 2 + 0) * 64 + lane];
    xa1 = reinterpret_cast<const bf16x8*>(p.x0w)[(cb * 2 + 1) * 64 + lane];
  }
  // the conv bias in accumulator layout: register q of lane (r, h) is channel cb*32 + acc_row(q, h). Held in registers
  // across the loop, except for IN_RB0 and IN_X0, which need them for their operand transforms: there it is re-read
  // from LDS (s_bias[(cb * 2 + h) * 16 + q]) at the start of every pass
  f32x16 bias_reg;
  if (IN == IN_RB0 || IN == IN_X0) {
    if (tid < 64) {
      const int c = (tid >> 5) * 32 + acc_row(tid & 15, (tid >> 4) & 1);
      s_bias[tid] = W8 ? p.bias[c] / p.wscale[c] : p.bias[c];
    }
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = cb * 32 + acc_row(q, h);
      bias_reg[q] = W8 ? p.bias[c] / p.wscale[c] : p.bias[c];
    }
  }
  if (W8 && tid < 64) s_wsc[tid] = p.wscale[tid];   // read by the epilogues, after the first tile's barrier

  // ---- staging. Item (row i, column c, 8-channel group sub) of patch row i: input frame t0 - 1 + c, mel row
  // given by the caller; out-of-range positions read past the end of the tensor (zeros).
  const int sub = tid & 7;
  const int npos = p.B * F * T;
  const int t0 = tt * TT;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.in0, (short)0, npos * 128, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, npos * 128, 0x00020000);
  // IN_RB0: the U-Net input channels of an item's position (fp32 [B][F][T]; spk per mel row), 0 when out of range
  // (raw buffer loads at 32-bit offsets: out-of-range positions read past the end, zeros)
  const __amdgpu_buffer_rsrc_t rs_mu =
      __builtin_amdgcn_make_buffer_rsrc((void*)((IN == IN_RB0 || IN == IN_X0) ? p.mu : nullptr), (short)0, npos * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_xt =
      __builtin_amdgcn_make_buffer_rsrc((void*)((IN == IN_RB0 || IN == IN_X0) ? p.xt : nullptr), (short)0, npos * 4, 0x00020000);
  auto load_in = [&](int frow, int ti, float* xi) {
    const bool ok = frow >= 0 && frow < F && ti >= 0 && ti < T;
    const int q = ok ? ((b * F + frow) * T + ti) * 4 : npos * 4;
    xi[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_mu, q, 0, 0));   // (the builtin returns the bits)
    xi[1] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_xt, q, 0, 0));
    xi[2] = 0.f;   // (spk: per mel row, read from LDS by the transform: s_coef + 384)
  };
  // IN_RB0: r0 is stored by the segment that owns the position (interior columns 1..32, rows of its tiles)
  const __amdgpu_buffer_rsrc_t rs_rb =
      __builtin_amdgcn_make_buffer_rsrc(IN == IN_RB0 ? p.rb_out : p.out, (short)0, npos * 128, 0x00020000);
  auto rb_dst = [&](int frow, int c) {   // byte offset of the item's r0, or past the end (dropped)
    const int ti = t0 - 1 + c;
    const bool own = c >= 1 && c <= TT && ti < T && frow >= ft0 * TF && frow < (ft0 + L) * TF && frow < F;
    return own ? ((b * F + frow) * T + ti) * 128 + sub * 16 : npos * 128;
  };
  auto load_item = [&](int it, int frow, u32x4_t& v, float& m, float* xi) {
    const int c = (it >> 3) % PC;
    const int ti = t0 - 1 + c;
    const bool ok = frow >= 0 && frow < F && ti >= 0 && ti < T;
    const int q = ok ? (b * F + frow) * T + ti : npos;
    v = __builtin_amdgcn_raw_buffer_load_b128(rs, q * 128 + sub * 16, 0, 0);
    if (IN != IN_PLAIN) {   // unconditional load at a clamped frame, then select (no branch around the load)
      const float mv = mask_at(p.mask, p.T0, b, ti < 0 ? 0 : (ti < T ? ti : T - 1), p.lvl_in);
      m = ok ? mv : 0.f;
    }
    if (IN == IN_RB0) load_in(frow, ti, xi);
  };
  const bool spk3 = IN == IN_RB0 && p.cin_input == 3;   // IN_RB0: n_spks > 1 (a third U-Net input channel)
  // (Mish(GN(h)) * m + tb) * m of the 8 channels of group g (diffusion.py:57-58, 76) as a bf16 item: a select for the
  // 0/1 masks of sequence_mask; a fractional mask value (C-ABI callers: the boundary rejects them) takes the multiply in
  // a branch 0/1 masks never enter, so the result is conv_kernel IN_GN's (Mish(GN(h)) + tb) * m on every path
  auto gn_tb_item = [&](float* v, float m, int g) __attribute__((always_inline)) {
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {   // 4 channels at a time: fewer coefficient registers live
      const float* cf = s_coef + g * 8 + hq * 4;
      const f32x4 sc = *reinterpret_cast<const f32x4*>(cf);
      const f32x4 sh = *reinterpret_cast<const f32x4*>(cf + 64);
      const f32x4 tb = *reinterpret_cast<const f32x4*>(cf + 128);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[4 * hq + k] = gn_mish_tb_l2(v[4 * hq + k], sc[k], sh[k], tb[k]);
    }
    if (__builtin_expect(m != 0.f && m != 1.f, 0)) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= m;
    }
    const uint4 o = f_to_item(v, bf16());
    return m != 0.f ? u32x4_t{o.x, o.y, o.z, o.w} : u32x4_t{0u, 0u, 0u, 0u};
  };
  // g: the item's 8-channel group (the thread's `sub`)
  auto put_item_at = [&](int lds_off, u32x4_t v4, float m, float xi0, float xi1, int frow, int rbo, int g)
      __attribute__((always_inline)) {
    if (IN == IN_MASK) {
      if (__builtin_expect(m != 0.f && m != 1.f, 0)) {   // x * m, fractional mask value
        float v[8];
        item_to_f(make_uint4(v4[0], v4[1], v4[2], v4[3]), v, bf16());
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= m;
        const uint4 o = f_to_item(v, bf16());
        v4 = u32x4_t{o.x, o.y, o.z, o.w};
      } else {
        v4 = m == 0.f ? u32x4_t{0u, 0u, 0u, 0u} : v4;
      }
    } else if (IN == IN_GN) {   // (Mish(GN(h)) * m + tb) * m, m in {0,1}  (diffusion.py:57-58, 76)
      float v[8];
      item_to_f(make_uint4(v4[0], v4[1], v4[2], v4[3]), v, bf16());
      v4 = gn_tb_item(v, m, g);
    } else if (IN == IN_RB0) {   // r0 = Mish(GN(h2)) * m + res_conv(in * m), as gn_mish_kernel<RES = 1>
      float v[8];
      item_to_f(make_uint4(v4[0], v4[1], v4[2], v4[3]), v, bf16());
      const float x0 = xi0 * m, x1 = xi1 * m;
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) {
        const float* cf = s_coef + g * 8 + hq * 4;
        float r[4];
        {
          const f32x4 w0 = *reinterpret_cast<const f32x4*>(cf + 128);
          const f32x4 w1 = *reinterpret_cast<const f32x4*>(cf + 192);
          const f32x4 rbv = *reinterpret_cast<const f32x4*>(cf + 320);
#pragma unroll
          for (int k = 0; k < 4; ++k) r[k] = fmaf(w1[k], x1, fmaf(w0[k], x0, rbv[k]));
        }
        if (spk3) {   // (wave-uniform) the third input channel: spk of this mel row, outermost as in the pass
          const float x2 = ((frow >= 0 && frow < F) ? s_coef[384 + frow] : 0.f) * m;
          const f32x4 w2 = *reinterpret_cast<const f32x4*>(cf + 256);
#pragma unroll
          for (int k = 0; k < 4; ++k) r[k] = fmaf(w2[k], x2, r[k]);
        }
        const f32x4 sc = *reinterpret_cast<const f32x4*>(cf);
        const f32x4 sh = *reinterpret_cast<const f32x4*>(cf + 64);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[4 * hq + k] = gn_mish_add<bf16>(v[4 * hq + k], sc[k], sh[k], r[k], m);
      }
      const uint4 o = f_to_item(v, bf16());
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{o.x, o.y, o.z, o.w}, rs_rb, rbo, 0, 0);   // r0 (unmasked)
      if (__builtin_expect(m != 0.f && m != 1.f, 0)) {   // r0 * m, fractional mask value: the unfused pass's
        float rv[8];                                     // IN_MASK operand (bf16(r0) * m, rounded to bf16)
        item_to_f(o, rv, bf16());
#pragma unroll
        for (int k = 0; k < 8; ++k) rv[k] *= m;
        const uint4 om = f_to_item(rv, bf16());
        v4 = u32x4_t{om.x, om.y, om.z, om.w};
      } else {
        v4 = m != 0.f ? u32x4_t{o.x, o.y, o.z, o.w} : u32x4_t{0u, 0u, 0u, 0u};   // r0 * m
      }
    }
    *reinterpret_cast<u32x4_t*>(sR + lds_off) = v4;
  };
  auto put_item = [&](int it, int slot, u32x4_t v4, float m, const float* xi, int frow) __attribute__((always_inline)) {
    const int c = (it >> 3) % PC;
    put_item_at(slot * ROWB + c * POSB + sub * 16, v4, m, xi[0], xi[1], frow, IN == IN_RB0 ? rb_dst(frow, c) : 0, sub);
  };

  // GroupNorm scale/shift (and time bias) of the input channels of utterance b (IN_GN): once per segment
  if (IN == IN_RB0) {   // GroupNorm affine of h2 (gn_affine, as gn_mish_kernel) and the res_conv weights, bias
    static_assert(NTHR >= 256, "gn_load / gn_finish use 256 threads");
    const GnLoad gl = gn_load(p.gn_part, p.gn_nparts, b, tid);
    gn_finish(gl, p.gn_part, p.gn_nparts, b, p.gn_count, s_mean, s_rstd, s_red, tid);
    if (tid < 64) {
      float sc, sh;
      gn_affine(s_mean, s_rstd, 64, tid, p.gn_gamma, p.gn_beta, sc, sh);
      gn_res_coef<bf16>(sc, sh);   // (base 2: gn_mish_add, as rbout_input)
      s_coef[tid] = sc; s_coef[64 + tid] = sh;
#pragma unroll
      for (int j = 0; j < 3; ++j) s_coef[128 + 64 * j + tid] = j < p.cin_input ? p.rb_w[tid * p.cin_input + j] : 0.f;
      s_coef[320 + tid] = p.rb_b[tid];
    }
    for (int f = tid; f < F; f += NTHR) s_coef[384 + f] = p.cin_input == 3 ? p.spk_s[(long)b * F + f] : 0.f;
    lds_barrier();
  }
  if (IN == IN_GN || IN == IN_X0) {
    const float c_g = tid < 64 ? p.gn_gamma[tid] : 0.f, c_b = tid < 64 ? p.gn_beta[tid] : 0.f;
    if (IN == IN_X0 && tid < 64) {   // the input conv's bias in accumulator layout, per (cb, h): the C operand of x0_mfma
      const int c = (tid >> 5) * 32 + acc_row(tid & 15, (tid >> 4) & 1);
      s_coef[192 + tid] = p.x0s ? p.x0b[c] / p.x0s[c] : p.x0b[c];
    }
    static_assert(NTHR >= 256, "gn_load / gn_finish use 256 threads");
    const GnLoad gl = gn_load(p.gn_part, p.gn_nparts, b, tid);
    const float tbv = tid < 64 ? tb_at(p.tb, p.stepp)[(long)b * p.tb_bstride + tid] : 0.f;
    gn_finish(gl, p.gn_part, p.gn_nparts, b, p.gn_count, s_mean, s_rstd, s_red, tid);
    if (tid < 64) {
      const float sc = c_g * s_rstd[tid >> 3];   // the affine in base 2 (common.h gn_mish_tb_l2)
      // (IN_X0 with fp8 weights: the accumulators hold h1 / scale, so the scale joins the GroupNorm multiplier)
      const float xs = (IN == IN_X0 && p.x0s) ? p.x0s[tid] : 1.f;
      s_coef[tid] = sc * kLog2e * xs; s_coef[64 + tid] = (c_b - s_mean[tid >> 3] * sc) * kLog2e; s_coef[128 + tid] = tbv;
    }
    lds_barrier();
  }

  // ---- prologue: tile 0's 6 patch rows (mel rows 4 ft0 - 1 .. 4 ft0 + 4) into ring slots 0..5
  if (IN != IN_X0) {
    u32x4_t cv[CPT];
    float cm[CPT], cx[IN == IN_RB0 ? CPT : 1][3];
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int it = tid + NTHR * j;
      load_item(it < COLD_ITEMS ? it : 0, ft0 * TF - 1 + (it < COLD_ITEMS ? it / (PC * 8) : 0), cv[j], cm[j],
                cx[IN == IN_RB0 ? j : 0]);
    }
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int it = tid + NTHR * j;
      if (CPT * NTHR == COLD_ITEMS || it < COLD_ITEMS)
        put_item(it, it / (PC * 8), cv[j], cm[j], cx[IN == IN_RB0 ? j : 0], ft0 * TF - 1 + it / (PC * 8));
    }
  }
  // The next tiles' new rows (tile k: mel rows 4 (ft0+k) + 1 .. + 4). A thread's item j of every tile has the same
  // row-in-tile, frame and 8-channel group, so its frame's mask and column offsets are fixed for the whole segment:
  // computed once here, so the loop issues only the raw buffer loads (no mask loads, no index division) and the
  // compiler's vmcnt waits count only loads and stores. A masked (IN_MASK) or out-of-range item reads past the end
  // of the tensor (zeros from the range check, no traffic).
  const int oob = npos * 128;
  int nrow[PPT], ncol[IN == IN_RB0 ? 1 : PPT], ngo[PPT], nti[IN == IN_RB0 ? PPT : 1];
  float nm[PPT];
#pragma unroll
  for (int j = 0; j < (IN == IN_X0 ? 0 : PPT); ++j) {
    const int it = tid + NTHR * j;
    const bool have = PPT * NTHR == NEW_ITEMS || it < NEW_ITEMS;
    const int c = (it >> 3) % PC, ti = t0 - 1 + c;
    const bool ok = have && ti >= 0 && ti < T;
    const float mv = mask_at(p.mask, p.T0, b, ti < 0 ? 0 : (ti < T ? ti : T - 1), p.lvl_in);
    nm[j] = (IN != IN_PLAIN && ok) ? mv : (IN == IN_PLAIN && ok ? 1.f : 0.f);
    nrow[j] = it / (PC * 8);
    if (IN == IN_RB0) nti[j] = c;   // (IN_RB0: the column, for the r0 store; its LDS offset formed per use)
    else ncol[j] = c * POSB + sub * 16;
    ngo[j] = (ok && !(IN == IN_MASK && nm[j] == 0.f)) ? ti * 128 + sub * 16 : -1;
  }
  u32x4_t preg[PPT];
  float pin[IN == IN_RB0 ? PPT : 1][3];   // IN_RB0: mu, x_t of each in-flight item's position ([2] unused)
  auto issue_new = [&](int j, int k) __attribute__((always_inline)) {   // item j of tile k's new rows (past the mel axis: zeros)
    const int frow = (ft0 + k) * TF + 1 + nrow[j];
    const int off = (ngo[j] >= 0 && frow < F) ? (b * F + frow) * T * 128 + ngo[j] : oob;
    preg[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    if (IN == IN_RB0) load_in(frow, t0 - 1 + nti[j], pin[j]);   // (nti: IN_RB0 only)
  };
  auto put_new = [&](int j, int k) __attribute__((always_inline)) {   // item j of tile k's new rows -> ring slots 4k + 2 + i
    if (PPT * NTHR == NEW_ITEMS || tid + NTHR * j < NEW_ITEMS) {
      int slot = (4 * k + 2) % RING + nrow[j];
      slot = slot >= RING ? slot - RING : slot;
      const int frow = (ft0 + k) * TF + 1 + nrow[j];
      const bool inrow = frow < F;   // the zero padding row below the mel axis (IN_GN: no transform)
      const float* xi = pin[IN == IN_RB0 ? j : 0];
      const int col_off = IN == IN_RB0 ? nti[j] * POSB + sub * 16 : ncol[j];
      put_item_at(slot * ROWB + col_off, preg[j], inrow ? nm[j] : 0.f, xi[0], xi[1], frow,
                  IN == IN_RB0 ? rb_dst(frow, nti[j]) : 0, sub);
    }
  };
  // IN_X0: h1 of patch row i_rel (mel row 4 ft0 - 1 + i_rel, ring slot i_rel % RING) at column c for this wave's 32
  // channels, from the window (x0 frame row fr in window row (fr - (4 ft0 - 2)) % XR), GroupNorm + Mish + time-bias
  // transformed straight from the fp32 accumulators (h1 is never stored, so it is never rounded to bf16: the
  // statistics and the values they normalise are the same fp32 numbers). `valid`: lanes that store.
  auto h1_block = [&](int i_rel, int c, float mc, bool valid) __attribute__((always_inline)) {
    const f32x16 bias = *reinterpret_cast<const f32x16*>(s_coef + 192 + (cb * 2 + h) * 16);
    const f32x16 acc = x0_mfma(sX, (i_rel + h) % XR, (i_rel + 2) % XR, c, h, xa0, xa1, bias);
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = acc[q];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)   // lane h: channels cb*32 + 16 pr + 8h + 0..7 (as the epilogue)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[8 * pr + q]), __float_as_uint(v[8 * pr + 4 + q]),
                                                         false, false);
        v[8 * pr + q] = __uint_as_float(sw[0]);
        v[8 * pr + 4 + q] = __uint_as_float(sw[1]);
      }
    const int frow = 4 * ft0 - 1 + i_rel;
    const float m = (frow >= 0 && frow < F) ? mc : 0.f;
    const int base = (i_rel % RING) * ROWB + c * POSB;
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int g = cb * 4 + 2 * pr + h;
      const u32x4_t item = gn_tb_item(v + 8 * pr, m, g);
      if (valid) *reinterpret_cast<u32x4_t*>(sR + base + g * 16) = item;
    }
  };
  // IN_X0 masks of this lane's columns: interior (c = r + 1, frame t0 + r) and halo (c = 0 / 33: frames t0 - 1, t0 + 32)
  float m_int = 0.f, m_halo = 0.f;
  // IN_X0 window loads: thread tid < 144 owns window column xc of new row xr (4 rows per tile), frame t0 - 2 + xc
  const int xr = tid / XC, xc = tid - xr * XC, xt_ = t0 - 2 + xc;
  float x_mk = 0.f, x_mu = 0.f, x_xt = 0.f;
  auto x0_issue = [&](int fr) {   // x0 frame row fr of this thread's column (zeros outside the grid)
    const bool ok = fr >= 0 && fr < F && xt_ >= 0 && xt_ < T;
    const int q = ok ? ((b * F + fr) * T + xt_) * 4 : npos * 4;
    x_mu = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_mu, q, 0, 0));
    x_xt = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_xt, q, 0, 0));
  };
  if (IN == IN_X0) {
    {
      const int t = t0 + r;
      m_int = t < T ? mask_at(p.mask, p.T0, b, t, p.lvl_in) : 0.f;
      const int th = (r & 1) ? t0 + TT : t0 - 1;
      m_halo = (th >= 0 && th < T) ? mask_at(p.mask, p.T0, b, th, p.lvl_in) : 0.f;
      x_mk = (xt_ >= 0 && xt_ < T) ? mask_at(p.mask, p.T0, b, xt_, p.lvl_in) : 0.f;
    }
    // window rows 0..11 = x0 frame rows 4 ft0 - 2 .. 4 ft0 + 9 (tile 0's rows and tile 1's new rows)
    float a[2], c2[2], mk[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int it = tid + NTHR * j;
      const int wr = it / XC, wc = it - wr * XC, fr = 4 * ft0 - 2 + wr, t = t0 - 2 + wc;
      const bool ok = it < XR * XC && fr >= 0 && fr < F && t >= 0 && t < T;
      const int q = ok ? ((b * F + fr) * T + t) * 4 : npos * 4;
      a[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_mu, q, 0, 0));
      c2[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_xt, q, 0, 0));
      mk[j] = (t >= 0 && t < T) ? mask_at(p.mask, p.T0, b, t < T ? t : T - 1, p.lvl_in) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int it = tid + NTHR * j;
      if (it < XR * XC) sX[it] = x0_pair(a[j], c2[j], mk[j]);
    }
    lds_barrier();
    // tile 0's 6 rows: interior rows rp, rp + 2, rp + 4 per wave; the 12 halo positions (row r >> 1) by the rp = 0 waves
#pragma unroll
    for (int i = 0; i < 3; ++i) h1_block(rp + 2 * i, r + 1, m_int, true);
    if (rp == 0) h1_block(r < 12 ? r >> 1 : 5, (r & 1) * (TT + 1), m_halo, r < 12);
    if (tid < 4 * XC) x0_issue(4 * ft0 + 10 + xr);   // tile 2's new window rows, stored at the end of tile 0
  } else {
#pragma unroll
    for (int j = 0; j < PPT; ++j) issue_new(j, 1);
  }
  lds_barrier();

  // per-lane GroupNorm partials of the whole segment (group cb*4 + pr*2 + h), accumulated tile by tile, pass by
  // pass in a fixed order; reduced across lanes and waves once, at the end
  float gs[2] = {0.f, 0.f}, gq[2] = {0.f, 0.f};
  const unsigned long long t_loop = stp.now();
  // The two workgroups sharing a CU start together, and the arbiter favours the older one's waves: the second-dispatched
  // (upper half of the grid) used to run the last ~20 % of its segment alone. Its waves take priority 1 for the first
  // two thirds of their tiles (measured: level-0 GN conv 112.7 -> 109.4 us, same box; switching at 1/4, 1/3, 1/2 of
  // the tiles or never back: less).
  const bool young = (int)blockIdx.x >= (int)(gridDim.x / 2);
  if (young) __builtin_amdgcn_s_setprio(1);
  for (int k = 0; k < L; ++k) {
    if (young && k == (2 * L) / 3) __builtin_amdgcn_s_setprio(0);
    const int ft = ft0 + k;
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
      const int lrow = 2 * rp + ps;
      // this pass's three patch rows (tap rows dr = 0, 1, 2) in the ring
      const int sbase = 4 * k + lrow;
      const char* rowp0 = sR + ((sbase + 0) % RING) * ROWB + r * POSB + h * 16;
      const char* rowp1 = sR + ((sbase + 1) % RING) * ROWB + r * POSB + h * 16;
      const char* rowp2 = sR + ((sbase + 2) % RING) * ROWB + r * POSB + h * 16;
      f32x16 acc;
      const unsigned long long t_pass = stp.now();
      // 36 MFMAs (4 chunks x 9 taps), fragment reads software-pipelined PF steps ahead (issued in the natural
      // order the compiler waited on each read right before its MFMA); behind each chunk's MFMAs one staging item of
      // tile k+1's new rows is stored and reloaded for tile k+2 (items spread over the 8 chunk slots of two passes)
      auto xread = [&](int st) {
        const int ch = st / 9, tap = st % 9, dr = tap / 3, dc = tap - 3 * dr;
        const char* rp_ = dr == 0 ? rowp0 : (dr == 1 ? rowp1 : rowp2);
        return *reinterpret_cast<const bf16x8*>(rp_ + dc * POSB + ch * 32);
      };
      auto wread = [&](int st) {
        const int ch = st / 9, tap = st % 9;
        return tap < WREG ? wf[ch][tap < WREG ? tap : 0]
                          : *reinterpret_cast<const bf16x8*>(wlp + (tap - WREG) * WTAP_B + ch * 1024);
      };
      constexpr int PF = 2, NB = PF + 1, NST = NCH * 9;   // (3, 4, 6 steps ahead: unchanged or spilling)
      // the first MFMA of the pass accumulates onto the conv bias (the C operand: no epilogue adds)
      const f32x16 bias_acc = (IN == IN_RB0 || IN == IN_X0) ? *reinterpret_cast<const f32x16*>(s_bias + (cb * 2 + h) * 16) : bias_reg;
      bf16x8 xb[NB], wb[NB];
#pragma unroll
      for (int st = 0; st < PF; ++st) { xb[st] = xread(st); wb[st] = wread(st); }
#pragma unroll
      for (int st = 0; st < NST; ++st) {
        if (st + PF < NST) { xb[(st + PF) % NB] = xread(st + PF); wb[(st + PF) % NB] = wread(st + PF); }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wb[st % NB], xb[st % NB], st == 0 ? bias_acc : acc, 0, 0, 0);
        if (st + PF < NST) {   // pin: the reads of step st + PF ahead of step st's MFMA
          if ((st + PF) % 9 < WREG) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          else __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        if (st % 9 == 8) {
          const int j = ps * NCH + st / 9;
          if (IN == IN_X0) {   // tile k+1's new rows (rel 4k + 6 ..): interior rows 2 rp, 2 rp + 1; halo every other tile
            if (j == 1) h1_block(4 * k + 6 + 2 * rp, r + 1, m_int, true);
            if (j == 3 && (k & 1) == rp) h1_block(4 * k + 6 + (r < 8 ? r >> 1 : 3), (r & 1) * (TT + 1), m_halo, r < 8);
            if (j == 5) h1_block(4 * k + 7 + 2 * rp, r + 1, m_int, true);
            if (j == 7 && tid < 4 * XC) {   // tile k+2's window rows (rel 4k + 12 + xr), then tile k+3's loads
              sX[((4 * k + xr) % XR) * XC + xc] = x0_pair(x_mu, x_xt, x_mk);
              x0_issue(4 * (ft0 + k) + 14 + xr);
            }
          } else if (j < PPT) {
            put_new(j, k + 1);
            issue_new(j, k + 2);
          }
        }
      }

      // ---- epilogue of this pass. Lane (j = r, h) holds channels cb*32 + {0-3, 8-11, 16-19, 24-27} + 4h of
      // position j (registers 0-3, 4-7, 8-11, 12-15); swapping registers 4-7 <-> 0-3 and 12-15 <-> 8-11 across
      // the half-waves leaves lane h with channels cb*32 + 8h + 0..7 (regs 0-7) and cb*32 + 16 + 8h + 0..7.
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = acc[q];
      const unsigned long long t_epi = stp.now_after(v[15]);   // the MFMA stream retired
      stp.add(3, t_epi - t_pass);
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[8 * pr + q]), __float_as_uint(v[8 * pr + 4 + q]),
                                                           false, false);
          v[8 * pr + q] = __uint_as_float(sw[0]);
          v[8 * pr + 4 + q] = __uint_as_float(sw[1]);
        }
      const int t = t0 + r;
      const bool valid = t < T;
      const int obyte = valid ? (((b * F + ft * TF + lrow) * T + t) * 64) * 2 : oob;   // past the end: dropped
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int c0 = cb * 32 + pr * 16 + 8 * h;   // first of this lane's 8 channels
        float o[8], ws[8];
        if (W8) {
          *reinterpret_cast<f32x4*>(ws) = *reinterpret_cast<const f32x4*>(s_wsc + c0);
          *reinterpret_cast<f32x4*>(ws + 4) = *reinterpret_cast<const f32x4*>(s_wsc + c0 + 4);
        }
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[e] = W8 ? v[8 * pr + e] * ws[e] : v[8 * pr + e];
          s += o[e];
          q += o[e] * o[e];
          asm volatile("" : "+v"(s), "+v"(q));   // scalar chains: see conv.hip (packed-FP32 op_sel hazard)
        }
        const uint4 ov = f_to_item(o, bf16());
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{ov.x, ov.y, ov.z, ov.w}, rs_out, obyte + c0 * 2, 0, 0);
        gs[pr] += valid ? s : 0.f;
        gq[pr] += valid ? q : 0.f;
      }
      stp.add(4, stp.now_after(gs[1], gq[1]) - t_epi);
    }
    const unsigned long long t_bar = stp.now();
    lds_barrier();   // tile k+1's rows complete
    stp.add(2, stp.now() - t_bar); stp.add(5, 1);
  }
  const unsigned long long t_loop_end = stp.now();
  // segment done: this wave's groups over its positions, then the 2 waves of each channel half -> one slot
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    const float s = half_sum32(gs[pr]), q = half_sum32(gq[pr]);
    if (r == 0) {
      s_sub[wv * 8 + (pr * 2 + h) * 2 + 0] = s;
      s_sub[wv * 8 + (pr * 2 + h) * 2 + 1] = q;
    }
  }
  lds_barrier();
  if (tid < 8) {   // fixed-order sum over the 2 waves of the group's channel half
    const int g = tid, gcb = g >> 2, e = (g & 3) * 2;
    float S = 0.f, Q = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < 2; ++w2) {
      const float* q = s_sub + (w2 * 2 + gcb) * 8 + e;
      S += q[0];
      Q += q[1];
    }
    float* dst = p.out_part + ((long)b * (n_tt * kseg) + tt * kseg + part) * 16 + g * 2;
    dst[0] = S;
    dst[1] = Q;
  }
  stp.set(0, t_loop - t_entry); stp.set(1, t_loop_end - t_loop); stp.set(6, stp.now() - t_loop_end);
  stp.flush(GT_C64_STAMP_DST, seg & 511, 4, wv, lane);
}

// GroupNorm statistics of the U-Net input conv's output h1 (block1 of downs.0.0, diffusion.py:52-58, 181), which the
// consumer conv64<IN_X0> recomputes instead of reading: one workgroup per utterance x 32-frame column x 20 mel rows,
// the {mu, x_t} * m window (22 x 36) in LDS, h1 per 32 positions x 32 channels by c64::x0_mfma (the same instructions
// on the same operands as the consumer, so the statistics are those of the values it transforms), fp32 sums of h1 and
// h1^2 per 8-channel group over the valid positions in a fixed order, one partial slot per workgroup (common.h
// layout). Optionally stores bf16(h1) (p.out: the "pre1" probe of the unfused path's storage point).
#ifndef GT_X0_RG
#define GT_X0_RG 20
#endif
namespace x0s {
constexpr int RG = GT_X0_RG, WR = RG + 2;   // mel rows per workgroup; window rows
}
__global__ __launch_bounds__(256) void x0_stats_kernel(ConvParams p) {
  using namespace c64;
  __shared__ __attribute__((aligned(16))) uint32_t sX[x0s::WR * XC];
  __shared__ __attribute__((aligned(16))) float s_xb[64], s_xs[64];   // bias (/ scale), scale: accumulator layout
  __shared__ float s_sub[4 * 16];   // [wave][group g][h][sum, sq]
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), cb = wv & 1, rsel = wv >> 1;
  const int F = p.Fout, T = p.Tout, n_tt = (T + 31) / 32, nrg = F / x0s::RG;
  int wg = blockIdx.x;
  const int rg = wg % nrg; wg /= nrg;
  const int tt = wg % n_tt, b = wg / n_tt;
  const int fr0 = rg * x0s::RG, t0 = tt * 32;
  const int npos = p.B * F * T;
  const __amdgpu_buffer_rsrc_t rs_mu = __builtin_amdgcn_make_buffer_rsrc((void*)p.mu, (short)0, npos * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_xt = __builtin_amdgcn_make_buffer_rsrc((void*)p.xt, (short)0, npos * 4, 0x00020000);
  constexpr int NWIN = x0s::WR * XC, NJ = (NWIN + 255) / 256;
  float a[NJ], c2[NJ], mk[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {   // window row w = x0 frame row fr0 - 1 + w, column = frame t0 - 2 + column
    const int it = tid + 256 * j;
    const int wr = it / XC, wc = it - wr * XC, fr = fr0 - 1 + wr, t = t0 - 2 + wc;
    const bool ok = it < NWIN && fr >= 0 && fr < F && t >= 0 && t < T;
    const int q = ok ? ((b * F + fr) * T + t) * 4 : npos * 4;
    a[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_mu, q, 0, 0));
    c2[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_xt, q, 0, 0));
    mk[j] = (t >= 0 && t < T) ? mask_at(p.mask, p.T0, b, t, p.lvl_in) : 0.f;
  }
  if (tid < 64) {
    const int c = (tid >> 5) * 32 + acc_row(tid & 15, (tid >> 4) & 1);
    s_xs[tid] = p.x0s ? p.x0s[c] : 1.f;
    s_xb[tid] = p.x0s ? p.x0b[c] / p.x0s[c] : p.x0b[c];
  }
  const bf16x8 xa0 = reinterpret_cast<const bf16x8*>(p.x0w)[(cb * 2 + 0) * 64 + lane];
  const bf16x8 xa1 = reinterpret_cast<const bf16x8*>(p.x0w)[(cb * 2 + 1) * 64 + lane];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int it = tid + 256 * j;
    if (it < NWIN) sX[it] = x0_pair(a[j], c2[j], mk[j]);
  }
  lds_barrier();
  const f32x16 bias = *reinterpret_cast<const f32x16*>(s_xb + (cb * 2 + h) * 16);
  const int t = t0 + r;
  const bool valid = t < T, full = t0 + 32 <= T;
  float gs[4] = {0.f, 0.f, 0.f, 0.f}, gq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 5
  for (int ii = 0; ii < x0s::RG / 2; ++ii) {   // output row fr0 + i (window rows i + h, i + 2), interior column r + 1
    const int i = rsel + 2 * ii;
    f32x16 acc = x0_mfma(sX, i + h, i + 2, r + 1, h, xa0, xa1, bias);
    if (p.x0s) {   // (uniform) fp8 weights: h1 = accumulator * scale
      const f32x16 xs = *reinterpret_cast<const f32x16*>(s_xs + (cb * 2 + h) * 16);
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] *= xs[q];
    }
    if (full) {   // (wave-uniform) every position of the column valid: straight into the running sums
#pragma unroll
      for (int g = 0; g < 4; ++g)   // register q = channel cb*32 + acc_row(q, h): group cb*4 + (q >> 2)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = acc[4 * g + e];
          gs[g] += v;
          gq[g] = __builtin_fmaf(v, v, gq[g]);
          asm volatile("" : "+v"(gs[g]), "+v"(gq[g]));   // scalar chains (conv.hip: packed-FP32 op_sel hazard)
        }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float s = 0.f, q2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = acc[4 * g + e];
          s += v;
          q2 = __builtin_fmaf(v, v, q2);
          asm volatile("" : "+v"(s), "+v"(q2));
        }
        gs[g] += valid ? s : 0.f;
        gq[g] += valid ? q2 : 0.f;
      }
    }
    if (p.out) {   // diagnostics: bf16(h1), 8 consecutive channels per lane after the half-wave swap
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = acc[q];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[8 * pr + q]), __float_as_uint(v[8 * pr + 4 + q]),
                                                           false, false);
          v[8 * pr + q] = __uint_as_float(sw[0]);
          v[8 * pr + 4 + q] = __uint_as_float(sw[1]);
        }
      if (valid) {
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const uint4 o = f_to_item(v + 8 * pr, bf16());
          *reinterpret_cast<uint4*>(reinterpret_cast<char*>(p.out) + (((long)(b * F + fr0 + i) * T + t) * 64 +
                                                                      cb * 32 + 16 * pr + 8 * h) * 2) = o;
        }
      }
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float s = half_sum32(gs[g]), q2 = half_sum32(gq[g]);
    if (r == 0) {
      s_sub[wv * 16 + (g * 2 + h) * 2 + 0] = s;
      s_sub[wv * 16 + (g * 2 + h) * 2 + 1] = q2;
    }
  }
  lds_barrier();
  if (tid < 8) {   // group G = cb*4 + g: fixed-order sum over the two waves of channel half cb and both lane halves
    const int gcb = tid >> 2, g = tid & 3;
    float S = 0.f, Q = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < 2; ++w2)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const float* q = s_sub + (w2 * 2 + gcb) * 16 + (g * 2 + hh) * 2;
        S += q[0];
        Q += q[1];
      }
    float* dst = p.out_part + ((long)b * (n_tt * nrg) + tt * nrg + rg) * 16 + tid * 2;
    dst[0] = S;
    dst[1] = Q;
  }
}

int x0_stats_nparts(int F, int T) { return ((T + 31) / 32) * (F / x0s::RG); }

bool x0_eligible(const ConvParams& p) {
  return p.cin_input == 2 && p.Cout == 64 && p.Fout == p.Fin && p.Tout == p.Tin && p.Fout % x0s::RG == 0 && p.mu &&
         p.xt && p.x0w && p.x0b && p.mask && (long)p.B * p.Fout * p.Tout * 128 < (1L << 31);
}

hipError_t launch_x0_stats(const ConvParams& p, hipStream_t s) {
  if (!x0_eligible(p) || !p.out_part) return hipErrorInvalidValue;
  const long nwg = (long)p.B * ((p.Tout + 31) / 32) * (p.Fout / x0s::RG);
  hipLaunchKernelGGL(x0_stats_kernel, dim3((unsigned)nwg), dim3(256), 0, s, p);
  return hipGetLastError();
}

static int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

bool conv64_eligible(const ConvParams& p) {
  return p.Cin == 64 && p.Cout == 64 && p.Cin_pad == 64 && p.C0 == 64 && p.in1 == nullptr && p.Fin == p.Fout &&
         p.Tin == p.Tout && p.Fout % 4 == 0 && p.w_bstride == 0 &&
         (long)p.B * p.Fout * p.Tout * 128 < (1L << 31);
}

// Segment length: a function of the grid height only (never of B), so the GroupNorm partial slots -- one per
// segment -- and with them every rounding are the same in any batch or GPU shard. 80 rows: the whole column (20
// tiles; 512 workgroups at B = 32, T = 512); 40 rows: half a column (5 tiles), which keeps two workgroups per CU
// at level 1.
// The small-batch plan (decoder.cpp) walks one tile per segment: at B = 1 the throughput plan launches 16
// workgroups at level 0.
static int conv64_seg(int F, int small) {
  const int n_ft = F / 4;
  if (small) return 1;
  return (n_ft >= 20 || n_ft % 2) ? n_ft : n_ft / 2;
}

int conv64_nparts(int F, int T, int small) { return ((T + 31) / 32) * ((F / 4) / conv64_seg(F, small)); }

hipError_t launch_conv64(InMode im, const ConvParams& p, hipStream_t s) {
  if (!conv64_eligible(p)) return hipErrorInvalidValue;
  const int L = conv64_seg(p.Fout, p.small);
  const long nseg = (long)p.B * ((p.Tout + 31) / 32) * (p.Fout / 4 / L);
  const unsigned grid = (unsigned)nseg;
  const dim3 block(256);
  const bool rb_ok = p.rb_out && p.rb_w && p.rb_b && p.mu && p.xt && p.cin_input >= 2 && p.cin_input <= 3 &&
                     (p.cin_input == 2 || p.spk_s);
  if (im == IN_X0) {   // (p.wscale: block2's fp8 weights; p.x0s: the input conv's)
    if (!x0_eligible(p) || !p.gn_part) return hipErrorInvalidValue;
    if (p.wscale) hipLaunchKernelGGL((conv64_kernel<IN_X0, true>), dim3(grid), block, 0, s, p, L);
    else hipLaunchKernelGGL((conv64_kernel<IN_X0, false>), dim3(grid), block, 0, s, p, L);
    return hipGetLastError();
  }
  if (p.wscale) {   // fp8 weights (the conv64-layout image of their e4m3 values)
    if (im == IN_RB0) {
      if (!rb_ok) return hipErrorInvalidValue;
      hipLaunchKernelGGL((conv64_kernel<IN_RB0, true>), dim3(grid), block, 0, s, p, L);
    } else if (im == IN_MASK) hipLaunchKernelGGL((conv64_kernel<IN_MASK, true>), dim3(grid), block, 0, s, p, L);
    else if (im == IN_GN) hipLaunchKernelGGL((conv64_kernel<IN_GN, true>), dim3(grid), block, 0, s, p, L);
    else if (im == IN_PLAIN) hipLaunchKernelGGL((conv64_kernel<IN_PLAIN, true>), dim3(grid), block, 0, s, p, L);
    else return hipErrorNotSupported;
  } else {
    if (im == IN_RB0) {
      if (!rb_ok) return hipErrorInvalidValue;
      hipLaunchKernelGGL((conv64_kernel<IN_RB0, false>), dim3(grid), block, 0, s, p, L);
      return hipGetLastError();
    }
    if (im == IN_MASK) hipLaunchKernelGGL((conv64_kernel<IN_MASK, false>), dim3(grid), block, 0, s, p, L);
    else if (im == IN_GN) hipLaunchKernelGGL((conv64_kernel<IN_GN, false>), dim3(grid), block, 0, s, p, L);
    else if (im == IN_PLAIN) hipLaunchKernelGGL((conv64_kernel<IN_PLAIN, false>), dim3(grid), block, 0, s, p, L);
    else return hipErrorNotSupported;
  }
  return hipGetLastError();
}


}  // namespace gt
