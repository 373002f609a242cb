// Attention output + Downsample as one pass (bf16), U-Net level 0 (C = 64).
//
// Reference (model/diffusion.py:186-191, 30-36, 103-110): at the first two U-Net levels
//     y = x + g * to_out(attn(x))                      Residual(Rezero(LinearAttention))
//     hiddens.append(y); x = downsample(y * mask)      Conv2d(C, C, 3, stride 2, padding 1)
// hiddens[0] is never popped (the up path has two levels; it pops the level-2 and level-1 entries), so the 168 MB
// (B = 32, T = 512) level-0 attention output is only ever read by the downsample. (The level-1 one is also the skip
// connection of ups.1: that level keeps the two launches -- a fused form that also stored y measured 236 us against
// 101 us, one 87 KB workgroup per CU.) With the attention folded into one per-utterance 1x1 (attn.hip:
// y = x + M_b x + g b_out) both convolutions fit one kernel:
//
//   stage 1  a workgroup's input patch (5 mel rows x 65 frames: the stride-2 3x3 window of 2 output rows x 32 output
//            frames) -> y = (M_b x + g b_out) + x on MFMA (M_b as A, positions as B; the residual x is the B fragment
//            itself), masked, rounded to bf16 into LDS;
//   stage 2  the 3x3 stride-2 conv of the LDS patch (weights as A from a fragment-ordered image, L2-resident) + bias.
//
// Same operations in the same order as conv_kernel CONV1/OUT_RESID followed by conv_kernel CONV3_S2/IN_MASK (1x1 over
// k-steps in order; the residual added after the bias; y rounded to bf16; x * m as a select for {0,1} masks; the 3x3
// over 16-channel chunks outer, taps inner; bias after), so the outputs are bit-identical to the two-kernel path
// (tests/test_attn_down_gpu.py) while the HBM traffic drops from read x + write y + read y + write out to read x (1.27x:
// the 5 x 65 patch of a 2 x 32 output tile) + write out.
//
// LDS patch: C/8 planes (8 channels each) x 5 rows x 69 entries of 16 B, the 65 columns deinterleaved by parity (even
// columns at entries 0..32, odd ones from entry 36 or 37: ad::odd_entry): a stride-2 tap then reads 32 CONSECUTIVE
// entries (conflict-free ds_read_b128), and the stage-1 item writes (even and odd columns alternating) land 16 banks
// apart.
#include "common.h"
#include "kernels.h"
#include "wimage.h"

namespace gt {

namespace ad {
constexpr int PROWS = 5, PCOLS = 65, NPOS = PROWS * PCOLS;   // input patch of one 2 x 32 output tile
constexpr int NPB = (NPOS + 31) / 32;                        // 11 position blocks of 32
// Odd columns of patch row r start at entry odd(r) = 36 + (r & 1). A group of 8 consecutive positions stored by one
// ds_write_b128 lane group is 4 even and 4 odd columns; their two 16-bank ranges are disjoint when the odd entries
// start 4 (mod 8) entries after the even ones -- odd(r) = 36 when the group starts at an even column, 37 when it starts
// at an odd one, which in a 65-column patch enumerated row by row happens exactly in the odd rows (a single offset
// of 36 left every odd-row group with a 2-way conflict: 0.77 conflict cycles per LDS instruction).
constexpr int RS = 69;                                       // row stride (entries): odd entries reach 37 + 31 = 68
GT_DEV int odd_entry(int prow) { return 36 + (prow & 1); }
constexpr int PLANE = PROWS * RS;                            // 345 entries
template <int C> constexpr int smem_bytes() { return (C / 8) * PLANE * 16; }   // 44,160 B (C = 64)
}  // namespace ad

typedef unsigned u32x4a_t __attribute__((ext_vector_type(4)));

// 4 waves (the attention output itself is not needed at level 0).
// W8: fp8 weights (p.wsc): the stage-2 epilogue is conv_kernel W8's acc * scale + bias (a template parameter: a run-time
// test in the epilogue cost attn_up 82 -> 119 us)
template <int C, bool W8>
__global__ __launch_bounds__(4 * C) __attribute__((amdgpu_waves_per_eu(3))) void attn_down_kernel(AttnDownParams p) {
  using namespace ad;
  constexpr int NCB = C / 32;   // 32-channel blocks
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<C>()];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = p.F, T = p.T, Fo = F / 2, To = T / 2;
  const int n_tt = (To + 31) / 32, n_ft = Fo / 2;
  int bid = blockIdx.x;
  const int tt = bid % n_tt; bid /= n_tt;
  const int ft = bid % n_ft;
  const int b = bid / n_ft;
  const int fo0 = 2 * ft, to0 = 32 * tt;
  const int fi0 = 2 * fo0 - 1, ti0 = 2 * to0 - 1;   // patch origin in the input grid

  const int npos_all = p.B * F * T;
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, npos_all * C * 2, 0x00020000);
  const int oob = npos_all * C * 2;
  const WImg W1 = conv_wimg(1, 1, C, C);
  const char* mimg = reinterpret_cast<const char*>(p.mw) + (long)b * p.mw_bstride;

  // position pb*32 + r of the patch: its x fragments (k-steps 0 .. C/16-1; out-of-range positions read zeros), mask,
  // LDS entry
  auto xfrags = [&](int pb, u32x4a_t* xf, float& m, int& ent) __attribute__((always_inline)) {
    const int pos = pb * 32 + r;
    const int prow = pos / PCOLS, pcol = pos - prow * PCOLS;
    const int fi = fi0 + prow, ti = ti0 + pcol;
    const bool inside = pos < NPOS && fi >= 0 && fi < F && ti >= 0 && ti < T;
    const int off = inside ? ((b * F + fi) * T + ti) * (C * 2) + h * 16 : oob;
#pragma unroll
    for (int ks = 0; ks < C / 16; ++ks) xf[ks] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off + ks * 32, 0, 0);
    m = inside ? mask_at(p.mask, p.T0, b, ti, p.lvl) : 0.f;
    ent = pos < NPOS ? prow * RS + ((pcol & 1) ? odd_entry(prow) : 0) + (pcol >> 1) : -1;
  };
  // the epilogue of one 32 x 32 stage-1 block (channels cb*32.., positions of one block): the accumulator (M_b x), the
  // bias g b_out, the residual (this lane's own x fragments of k-steps 2cb, 2cb+1) -> bf16 y -> LDS (masked)
  auto y_block = [&](const f32x16& acc, int cb, const float (*gbc)[8], const u32x4a_t* xf, float m, int ent)
      __attribute__((always_inline)) {
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
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      float e[8], o[8];
      const u32x4a_t xr = xf[2 * cb + pr];   // (cb compile-time at every call: no dynamic register indexing)
      item_to_f(make_uint4(xr[0], xr[1], xr[2], xr[3]), e, bf16());
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = v[8 * pr + k] + gbc[pr][k];   // conv_kernel OUT_RESID: bias, then the residual
        o[k] += e[k];
      }
      const uint4 ov = f_to_item(o, bf16());
      const int c0 = cb * 32 + pr * 16 + 8 * h;
      // y * mask as the downsample's IN_MASK select ({0,1} masks; a fractional mask multiplies the bf16 value)
      u32x4a_t y;
      if (m == 1.f) {
        y = u32x4a_t{ov.x, ov.y, ov.z, ov.w};
      } else if (m == 0.f) {
        y = u32x4a_t{0u, 0u, 0u, 0u};
      } else {
        float t[8];
        item_to_f(ov, t, bf16());
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] *= m;
        const uint4 tv = f_to_item(t, bf16());
        y = u32x4a_t{tv.x, tv.y, tv.z, tv.w};
      }
      if (ent >= 0) *reinterpret_cast<u32x4a_t*>(smem + ((c0 >> 3) * PLANE + ent) * 16) = y;   // plane = c0 / 8
    }
  };

  // ---- stage 1, 4 waves: wave w takes position blocks w, w+4, w+8 (< 11) and both 32-channel halves (the x fragments
  // are shared by the two halves); every x fragment of the wave in flight at once (one HBM round trip)
  bf16x8 ma[2][4];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      ma[cb][ks] = *reinterpret_cast<const bf16x8*>(mimg + conv_wimg_off(W1, cb * 32 + r, 0, 16 * ks + 8 * h, 2));
  float gb[2][2][8];   // g b_out of this lane's channels after the swap: cb*32 + 16 pr + 8h + 0..7
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int k = 0; k < 8; ++k) gb[cb][pr][k] = p.gb[cb * 32 + pr * 16 + 8 * h + k];
  constexpr int NPW = (NPB + 3) / 4;
  u32x4a_t xf[NPW][4];
  float m[NPW];
  int ent[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) xfrags(wv + 4 * i < NPB ? wv + 4 * i : NPB, xf[i], m[i], ent[i]);
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    if (wv + 4 * i >= NPB) break;   // wave-uniform
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      f32x16 acc;
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[k] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 xb;
        __builtin_memcpy(&xb, &xf[i][ks], 16);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ma[cb][ks], xb, acc, 0, 0, 0);
      }
      y_block(acc, cb, gb[cb], xf[i], m[i], ent[i]);
    }
  }

  // ---- stage 2: 3x3 stride-2 conv of the patch. Wave w: output channels cb*32.. (cb = w % NCB) of output row
  // orow = w / NCB, 32 output frames; k-steps (16-channel chunk ch, tap) in conv_kernel's order (chunk outer, tap inner).
  const int cb = wv % NCB, orow = wv / NCB;
  const bf16x8* wsrc = reinterpret_cast<const bf16x8*>(p.wds) + cb * (C / 16) * 9 * 64 + lane;   // pack_frag3x3 order
  auto aread = [&](int st) { return wsrc[st * 64]; };   // st = ch * 9 + tap
  auto bread = [&](int st) {
    const int ch = st / 9, tap = st % 9, dr = tap / 3, dc = tap - 3 * dr;
    const int prow = 2 * orow + dr;
    const int ent = prow * RS + (dc == 1 ? odd_entry(prow) : (dc >> 1)) + r;
    return *reinterpret_cast<const bf16x8*>(smem + ((2 * ch + h) * PLANE + ent) * 16);
  };
  // weight fragments (L2) PFA steps ahead, patch fragments (LDS) PFB steps ahead
  constexpr int PFA = 10, NBA = PFA + 1, PFB = 3, NBB = PFB + 1, NST = 9 * C / 16;
  bf16x8 af[NBA], bf[NBB];
#pragma unroll
  for (int st = 0; st < PFA; ++st) af[st] = aread(st);
  lds_barrier();
#pragma unroll
  for (int st = 0; st < PFB; ++st) bf[st] = bread(st);
  f32x16 acc;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;
#pragma unroll
  for (int st = 0; st < NST; ++st) {
    if (st + PFA < NST) af[(st + PFA) % NBA] = aread(st + PFA);
    if (st + PFB < NST) bf[(st + PFB) % NBB] = bread(st + PFB);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[st % NBA], bf[st % NBB], acc, 0, 0, 0);
  }
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
  const int to = to0 + r;
  if (to < To) {
    bf16* out = reinterpret_cast<bf16*>(p.out) + (((long)b * Fo + fo0 + orow) * To + to) * C;
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int c0 = cb * 32 + pr * 16 + 8 * h;
      float o[8];
      if (W8) {   // fp8 weights (their e4m3 values in the image): conv_kernel W8's epilogue, acc * scale + bias
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = v[8 * pr + k] * p.wsc[c0 + k] + p.bds[c0 + k];
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = v[8 * pr + k] + p.bds[c0 + k];
      }
      *reinterpret_cast<uint4*>(out + c0) = f_to_item(o, bf16());
    }
  }
}

bool attn_down_eligible(const AttnDownParams& p) {
  return p.C == 64 && p.F % 4 == 0 && p.T % 2 == 0 && (long)p.B * p.F * p.T * p.C * 2 < (1L << 31);
}

hipError_t launch_attn_down(const AttnDownParams& p, hipStream_t s) {
  if (!attn_down_eligible(p)) return hipErrorInvalidValue;
  const long grid = (long)p.B * (p.F / 4) * ((p.T / 2 + 31) / 32);
  if (p.wsc) hipLaunchKernelGGL((attn_down_kernel<64, true>), dim3((unsigned)grid), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((attn_down_kernel<64, false>), dim3((unsigned)grid), dim3(256), 0, s, p);
  return hipGetLastError();
}

// ---- attention output + Upsample (ConvTranspose2d(64, 64, 4, 2, 1)) as one pass: ups.1 (diffusion.py:201-205), whose
// attention output (level 1, 64 channels) feeds only the upsample. Stage 1 as above on a coarse patch of 6 rows x 34
// frames (the 4 x 32 coarse positions of the tile plus a one-position halo); stage 2 the four sub-pixel 2x2 convs of
// conv_kernel CONVT4 (out[2J + pf][2K + pt] from coarse rows J + pf - a, columns K + pt - b, taps (a, b)), wave w taking
// parity w, in conv_kernel's order (16-channel chunk outer, tap inner): bit-identical to the two launches.
namespace au {
constexpr int PROWS = 6, PCOLS = 34, NPOS = PROWS * PCOLS, NPB = (NPOS + 31) / 32;   // 204 positions, 7 blocks
constexpr int PLANE = NPOS;                                                          // entries per 8-channel plane
constexpr int SMEM = 8 * PLANE * 16;                                                 // 26,112 B
}  // namespace au

template <bool W8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_up_kernel(AttnUpParams p) {
  using namespace au;
  constexpr int C = 64;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int F = p.F, T = p.T;                     // coarse grid
  const int n_tt = (T + 31) / 32, n_ft = F / 4;
  int bid = blockIdx.x;
  const int tt = bid % n_tt; bid /= n_tt;
  const int ft = bid % n_ft;
  const int b = bid / n_ft;
  const int J0 = 4 * ft, K0 = 32 * tt;
  const int fi0 = J0 - 1, ti0 = K0 - 1;           // patch origin (coarse)
  const int npos_all = p.B * F * T;
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, npos_all * C * 2, 0x00020000);
  const int oob = npos_all * C * 2;

  // ---- stage 1: y = (M_b x + g b_out) + x, masked, into LDS. Wave w: position blocks w, w + 4 (< 7), both halves.
  {
    const WImg W1 = conv_wimg(1, 1, C, C);
    const char* mimg = reinterpret_cast<const char*>(p.mw) + (long)b * p.mw_bstride;
    bf16x8 ma[2][4];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        ma[cb][ks] = *reinterpret_cast<const bf16x8*>(mimg + conv_wimg_off(W1, cb * 32 + r, 0, 16 * ks + 8 * h, 2));
    u32x4a_t xf[2][4];
    float m[2];
    int ent[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pos = (wv + 4 * i) * 32 + r;
      const int prow = pos / PCOLS, pcol = pos - prow * PCOLS;
      const int fi = fi0 + prow, ti = ti0 + pcol;
      const bool inside = pos < NPOS && fi >= 0 && fi < F && ti >= 0 && ti < T;
      const int off = inside ? ((b * F + fi) * T + ti) * (C * 2) + h * 16 : oob;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) xf[i][ks] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off + ks * 32, 0, 0);
      m[i] = inside ? mask_at(p.mask, p.T0, b, ti, p.lvl) : 0.f;
      ent[i] = pos < NPOS ? pos : -1;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (wv + 4 * i >= NPB) break;   // wave-uniform
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        f32x16 acc;
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[k] = 0.f;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          bf16x8 xb;
          __builtin_memcpy(&xb, &xf[i][ks], 16);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ma[cb][ks], xb, acc, 0, 0, 0);
        }
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = acc[q];
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
          const int c0 = cb * 32 + pr * 16 + 8 * h;
          float e[8], o[8];
          const u32x4a_t xr = xf[i][2 * cb + pr];
          item_to_f(make_uint4(xr[0], xr[1], xr[2], xr[3]), e, bf16());
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            o[k] = v[8 * pr + k] + p.gb[c0 + k];   // conv_kernel OUT_RESID: bias, then the residual
            o[k] += e[k];
          }
          const uint4 ov = f_to_item(o, bf16());
          u32x4a_t y;   // y * mask: conv_kernel CONVT4 IN_MASK's select ({0,1} masks), multiply otherwise
          if (m[i] == 1.f) {
            y = u32x4a_t{ov.x, ov.y, ov.z, ov.w};
          } else if (m[i] == 0.f) {
            y = u32x4a_t{0u, 0u, 0u, 0u};
          } else {
            float t[8];
            item_to_f(ov, t, bf16());
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] *= m[i];
            const uint4 tv = f_to_item(t, bf16());
            y = u32x4a_t{tv.x, tv.y, tv.z, tv.w};
          }
          if (ent[i] >= 0) *reinterpret_cast<u32x4a_t*>(smem + ((c0 >> 3) * PLANE + ent[i]) * 16) = y;
        }
      }
    }
  }

  // ---- stage 2: wave w = sub-pixel parity (pf, pt) = (w >> 1, w & 1); for each 32-channel half cb and coarse row j of
  // the tile: 16 k-steps (chunk ch of 16 channels, tap (a, b) = (t >> 1, t & 1)) -> fine row 2 (J0 + j) + pf, fine
  // columns 2 (K0 + r) + pt. Weights: the parity's fragment image (pack_fragT), A operand, 16 fragments per half.
  const int pf = wv >> 1, pt = wv & 1;
  const int Ff = 2 * F, Tf = 2 * T;
  const bf16x8* wsrc = reinterpret_cast<const bf16x8*>(p.wup) + wv * 2 * 16 * 64 + lane;   // [par][cb][ch][tap][lane]
  // (weight fragments requested before stage 1 or during the first half's MFMAs measured slower: the extra registers
  // cost the third wave per SIMD, 82 -> 88-91 us)
  lds_barrier();
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    bf16x8 wa[16];
#pragma unroll
    for (int st = 0; st < 16; ++st) wa[st] = wsrc[(cb * 16 + st) * 64];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      auto bread = [&](int st) {
        const int ch = st >> 2, tap = st & 3, a = tap >> 1, bb = tap & 1;
        const int ent = (j + 1 + pf - a) * PCOLS + (r + 1 + pt - bb);
        return *reinterpret_cast<const bf16x8*>(smem + ((2 * ch + h) * PLANE + ent) * 16);
      };
      constexpr int PFB = 3, NBB = PFB + 1;
      bf16x8 bf[NBB];
#pragma unroll
      for (int st = 0; st < PFB; ++st) bf[st] = bread(st);
      f32x16 acc;
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[k] = 0.f;
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        if (st + PFB < 16) bf[(st + PFB) % NBB] = bread(st + PFB);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[st], bf[st % NBB], acc, 0, 0, 0);
      }
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = acc[q];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[8 * pr + q]),
                                                           __float_as_uint(v[8 * pr + 4 + q]), false, false);
          v[8 * pr + q] = __uint_as_float(sw[0]);
          v[8 * pr + 4 + q] = __uint_as_float(sw[1]);
        }
      const int frow = 2 * (J0 + j) + pf, fcol = 2 * (K0 + r) + pt;
      if (K0 + r < T) {
        bf16* out = reinterpret_cast<bf16*>(p.out) + (((long)b * Ff + frow) * Tf + fcol) * C;
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const int c0 = cb * 32 + pr * 16 + 8 * h;
          float o[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = W8 ? v[8 * pr + k] * p.wsc[c0 + k] + p.bup[c0 + k] : v[8 * pr + k] + p.bup[c0 + k];
          *reinterpret_cast<uint4*>(out + c0) = f_to_item(o, bf16());
        }
      }
    }
  }
}

bool attn_up_eligible(const AttnUpParams& p) {
  return p.C == 64 && p.F % 4 == 0 && (long)p.B * 4 * p.F * p.T * 128 < (1L << 31);
}

hipError_t launch_attn_up(const AttnUpParams& p, hipStream_t s) {
  if (!attn_up_eligible(p)) return hipErrorInvalidValue;
  const long grid = (long)p.B * (p.F / 4) * ((p.T + 31) / 32);
  if (p.wsc) hipLaunchKernelGGL(attn_up_kernel<true>, dim3((unsigned)grid), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(attn_up_kernel<false>, dim3((unsigned)grid), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace gt
