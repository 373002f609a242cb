// Implicit-GEMM convolutions of the Grad-TTS score U-Net on CDNA4 MFMA.
//
// One kernel template covers every convolution of GradLogPEstimator2d (model/diffusion.py:49-216):
//   CONV3    3x3 stride 1 pad 1   -- Block.block[0]            (diffusion.py:52)
//   CONV3_S2 3x3 stride 2 pad 1   -- Downsample                (diffusion.py:33)
//   CONV1    1x1                  -- ResnetBlock.res_conv (:70) and the folded LinearAttention output
//   CONVT4   ConvTranspose 4x4 s2 -- Upsample (diffusion.py:24) as four 2x2 sub-pixel convolutions
//
// GEMM view: M = output positions of a tile (4 mel rows x TT frames), N = NT output channels (64 or
// 128), K = taps x input channels, walked in chunks of 16 channels (one MFMA k-step) per position.
//   waves: NT=64  -> 4 waves along M (1 mel row each);  NT=128 -> 2 x 2 waves (2 mel rows x 64 ch each)
//   each wave holds RBW x 2 fp32 32x32 accumulators (v_mfma_f32_32x32x16_bf16 / 32x32x2_f32).
//   occupancy: 3 workgroups per CU for NT=64 (42 KB LDS), 2 for NT=128.
// Per chunk:
//   * weight slab: one contiguous global_load_lds DMA of the pre-packed image (wimage.h) -- no VGPRs;
//   * input patch: raw buffer loads at precomputed 32-bit offsets, prefetched into registers while the
//     previous chunk's MFMAs run. Padding and masked frames (mask 0) point past the end of the tensor,
//     so the range check returns zeros: no address arithmetic or selects per chunk. IN_GN transforms
//     in registers (the producer's GroupNorm apply + Mish + mask + time bias, diffusion.py:57-58,76);
//     rows are padded to an odd number of 16-B slots in LDS (conflict-free fragments);
//   * 9 (or 4, 1) taps of MFMA.
// Epilogue: each 32x32 accumulator block is transposed through the wave's own LDS scratch so every lane
// owns 8 consecutive output channels of one position: 16-B vector stores, vector loads of the
// ResnetBlock pre-activation (OUT_RBOUT) or the attention residual (OUT_RESID), and GroupNorm partial
// sums (padded frames included, as torch's group_norm does) written to this workgroup's slot.
#include "common.h"
#include "kernels.h"
#include "wimage.h"

namespace gt {

constexpr int TF1_DBW = 101;   // tile-height code: 1-row tiles with double-buffered weight slabs (ConvCfg::SMALLDB)

template <class A, int KIND, int IN, int OUT, int NT, int W8, int TF_>
struct ConvCfg {
  static constexpr bool CONVT = KIND == CONVT4;
  static constexpr int KS = (KIND == CONV1) ? 1 : 3;
  static constexpr int S = (KIND == CONV3_S2) ? 2 : 1;
  static constexpr int TF = TF_ == TF1_DBW ? 1 : TF_;
  static constexpr int TT = (KIND == CONV3_S2) ? 32 : 64;
  static constexpr int RBT = TT / 32;
  static constexpr int WN = NT / 64;
  static constexpr int WM = 4 / WN;
  static constexpr int RBW = TF * RBT / WM;   // 32-position row blocks per wave: wave wm owns blocks wm*RBW ..
  static constexpr int NTAP = CONVT ? 4 : KS * KS;
  static constexpr int PAD = (KIND == CONV1) ? 0 : 1;
  static constexpr int PR = (TF - 1) * S + KS;
  static constexpr int PC = (TT - 1) * S + KS;
  // stride 2: the patch columns of a row are stored deinterleaved by parity (even columns at 0 .. ODDC-1, odd ones from
  // ODDC), so a tap's 32 lanes (columns 2r + dc) read 32 CONSECUTIVE positions: with 48-B positions a stride of two
  // (96 B = 6 slots) put lanes 8 apart on the same banks (2-way conflicts); consecutive ones (3 slots) never do
  static constexpr bool DEINT = KIND == CONV3_S2;
  static constexpr int ODDC = (PC + 1) / 2;
  static constexpr __host__ __device__ int pcol(int pc) { return DEINT ? ((pc & 1) ? ODDC + (pc >> 1) : (pc >> 1)) : pc; }
  // W8 == 2 (A8): fp8 operands on v_mfma_scale_f32_32x32x64_f8f6f4 -- 32-channel chunks of e4m3 activations
  // (32 B per position in LDS + an E8M0 scale byte in the pad) and the conv_wimga8 weight image
  static constexpr bool A8 = W8 == 2;
  static constexpr int CKB = A8 ? 32 : conv_ckb(sizeof(A) == 2, KIND == CONV1 ? 1 : 9, IN == IN_INPUT ? 3 : 64);
  static constexpr int SUBS = A8 ? 4 : CKB / 16;   // LDS items per position (A8: 8 e4m3 channels = 8 B per item)
  static constexpr int POSB = CKB + 16;   // an odd number of 16-B slots per position: conflict-free fragment reads
  // weight slab: bf16/fp32 image (wimage.h: half A = taps [0, NA), half B = the rest) or the fp8 image
  // (conv8_wrow, W8: e4m3 weights, bf16 operands; conv_wimga8, A8)
  static constexpr int ABF = sizeof(A) == 2 ? 1 : 0;
  // (A8: NA counts the 32-B tap slots of half A)
  static constexpr int NA = A8 ? CONVA8_SLOTS_A : W8 ? NTAP : conv_na(ABF, NTAP);
  static constexpr int WROW = A8 ? CONVA8_WROWA : W8 ? conv8_wrow(NTAP) : conv_wrow(NA, CKB);   // half A rows (all taps if unsplit)
  static constexpr int WROWB = A8 ? CONVA8_WROWB : conv_wrow(NTAP - NA, CKB);
  static constexpr int HA = A8 ? round4k(NT * CONVA8_WROWA) : W8 ? conv8_wbytes(NT, NTAP) : conv_habytes(ABF, NT, NTAP, CKB);
  static constexpr int WBYTES = A8 ? HA + round4k(NT * CONVA8_WROWB) : W8 ? HA : HA + conv_hbbytes(ABF, NT, NTAP, CKB);
  static constexpr int WPIECES_ALL = WBYTES / 1024;        // 1 KiB DMA pieces per chunk
  static constexpr int WPIECES = (WPIECES_ALL + 3) / 4;    // per wave (the last round may be partial)
  // Split pipeline (bf16, multi-tap, operand from an activation): the two halves of chunk c+1 are staged while
  // the other half of chunk c is in the MFMAs. Every wave issues exactly PA / PB DMA pieces per half and PPT
  // patch loads per chunk, so counted vmcnt waits retire exactly the right ones.
  // Small-batch plan, 1-row 128-wide 3x3 tiles when the grid has at most one workgroup per CU (TF_ = TF1_DBW, launch_c3):
  // the whole next weight slab is staged into a second buffer during the current chunk (DBW) instead of the split
  // half-slab pipeline, whose half-A DMA has only half a chunk of MFMAs to land behind. Same MFMA order, so the same
  // bits; twice the weight LDS, so one workgroup per CU (slower once the grid exceeds the CUs: B = 4 measured -11 %)
  static constexpr bool SMALLDB = TF_ == TF1_DBW;
  static constexpr bool SPLIT = ((!W8 && NA < NTAP && IN != IN_INPUT) || A8) && !SMALLDB;
  // 1x1 convs: two weight slabs, chunk c+1's DMA in flight during chunk c's MFMAs (a 1x1 chunk is one tap, too
  // short to hide a weight round trip behind; the slab is 4-8 KB)
  static constexpr bool DBW = (!SPLIT && KIND == CONV1) || SMALLDB;
  // Split-K (small-batch plan, 128-wide 3x3 tiles, bf16 activations): p.ksplit workgroups per output tile each run a contiguous
  // range of input-channel chunks and leave their fp32 accumulators in p.sk_part; the last to finish (a counter per
  // tile, which it re-arms) adds the partials in split order -- a fixed order, so the result does not depend on which
  // finished last -- and runs the epilogue. A single utterance's level-2 convs otherwise occupy 80 of the 256 CUs, each
  // streaming 590 KB of weights through LDS.
  static constexpr bool SK = KIND == CONV3 && OUT == OUT_STATS && NT == 128 && (TF_ == TF1_DBW || TF_ == 1) &&
                             IN != IN_INPUT && sizeof(A) == 2;   // (bf16, fp8-weight and fp8-operand tiles)
  static constexpr int PA = HA / 4096, PB = (WBYTES - HA) / 4096;
  static constexpr int CK = A8 ? 32 : CKB / (int)sizeof(A);   // input channels per chunk
  static constexpr int ICH = 16 / (int)sizeof(A);            // channels per item (one 16-B global load)
  static constexpr int KSTEP_B = 16 * (int)sizeof(A);
  static constexpr int KSTEPS = CKB / KSTEP_B;
  // Patch items (16 B: sub-group `sub` of SUBS of a position). A ds_write_b128 serves lanes in groups of 8 with banks
  // (a/4) mod 32 (8 slots of 16 B), while the conflict-free fragment reads need a position stride of an odd number of
  // slots (P = POSB / 16): in position-major order (lanes 4i..4i+3 = one position, as A8 keeps for its DPP scale
  // exchange) a group's two positions p, p + 1 share a bank. IMAP permutes the positions only, keeping each quad of
  // lanes on one position (SUBS = 4: its 64 contiguous bytes, what the load coalesces) or two (SUBS = 2), so that a
  // group's slots cover all 8 banks: SUBS = 4 (P = 5) pairs positions p and p + 4 in a group, SUBS = 2 (P = 3) takes
  // positions {0, 2, 4, 6} or {1, 3, 5, 7} of a block of 8. Stride 2: positions in LDS (deinterleaved) order.
  static constexpr bool IMAP = !A8 && (SUBS == 4 || SUBS == 2);
  static constexpr int NPOS = PR * PC;
  static constexpr int PITEMS = IMAP ? 8 * SUBS * ((NPOS + 7) / 8) : NPOS * SUBS;
  static __host__ __device__ constexpr int ipos(int it) {
    return !IMAP ? it / SUBS
                 : 8 * (it / (8 * SUBS)) + (SUBS == 4 ? (((it >> 2) & 7) >> 1) + 4 * ((it >> 2) & 1)
                                                      : 2 * ((it & 7) >> 1) + ((it >> 3) & 1));
  }
  static __host__ __device__ constexpr int isub(int it) { return it % SUBS; }
  static __host__ __device__ constexpr int gcol(int lc) { return DEINT ? (lc < ODDC ? 2 * lc : 2 * (lc - ODDC) + 1) : lc; }
  static constexpr int PPT = (PITEMS + 255) / 256;
  static constexpr int A_BYTES = PR * PC * POSB;
  static constexpr int WBUF = DBW ? 2 * WBYTES : WBYTES;   // weight slab(s) in LDS
  static constexpr int SMEM0 = A_BYTES + WBUF + (3 * 256 + 128 + 64 + 16 + 128) * 4;
  // Workgroups per CU are capped by LDS where more resident tiles measured slower (cache/write
  // contention, not latency hiding, bounds them): CAP = 0 leaves occupancy to registers and LDS.
  // (measured, tools/ab_variants.sh: 64-wide 1x1 and sub-pixel convs 3, stride-2 64-wide 2; the fp8-weight
  // 3x3 tiles need fewer registers than the bf16 ones and would otherwise run 4 per CU)
  static constexpr int CAP = NT != 64 ? 0 : KIND == CONVT4 ? 3 : KIND == CONV1 ? 3 : KIND == CONV3_S2 ? 2 : (W8 ? 3 : 0);
  static constexpr int SMEM = (CAP && SMEM0 <= 160 * 1024 / (CAP + 1)) ? 160 * 1024 / (CAP + 1) + 512 : SMEM0;
  static_assert(KSTEPS >= 1, "chunk smaller than one MFMA k-step");
  static_assert(TF * RBT % WM == 0, "row blocks split evenly over the waves");
  static_assert(256 % (IMAP ? 8 * SUBS : SUBS) == 0, "per-thread channel group must be fixed");
  static_assert(WBYTES % 1024 == 0, "whole DMA pieces");
  static_assert(!DBW || WPIECES_ALL % 4 == 0, "counted waits: every wave issues WPIECES weight pieces");
  static_assert(!SPLIT || (HA % 4096 == 0 && (WBYTES - HA) % 4096 == 0 && PB + PPT <= 63), "wave-even halves");
  static_assert(!W8 || (sizeof(A) == 2 && KIND != CONV1), "fp8 weights: bf16 operands, 3x3 / 2x2 convs");
  static_assert(!A8 || (KIND == CONV3 && IN != IN_INPUT), "fp8 operands: stride-1 3x3 convs over activations");
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// fp8 weight fragment (W8): 8 consecutive e4m3 input-channel weights of one output channel -> bf16x8
// (exact: every e4m3 value is a bf16 value; the per-channel scale is applied to the accumulator)
GT_DEV bf16x8 w8_frag(const char* src) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const uint2 q = *reinterpret_cast<const uint2*>(src);
  const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(q.x, 1.0f, false);
  const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(q.x, 1.0f, true);
  const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(q.y, 1.0f, false);
  const bf16x2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(q.y, 1.0f, true);
  return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

template <class A, int KIND, int IN, int OUT, int NT, int W8, int TF_>
// 64-wide tiles: 3 workgroups per CU (42 KB LDS, <= 168 registers); 128-wide: 2
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NT == 64 && W8 != 2 ? 3 : 2))) void conv_kernel(ConvParams p) {
  typedef ConvCfg<A, KIND, IN, OUT, NT, W8, TF_> C;
  typedef typename Mma<A>::frag frag;
  constexpr bool CONVT = C::CONVT;

  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];   // ONE LDS object (see guide §5 trap a)
  char* sA = smem;
  char* const sW = smem + C::A_BYTES;
  float* s_sc = reinterpret_cast<float*>(smem + C::A_BYTES + C::WBUF);
  float* s_sh = s_sc + 256;
  float* s_tb = s_sh + 256;
  float* s_bias = s_tb + 256;    // bias of this tile's NT output channels
  float* s_sub = s_bias + 128;   // [4 waves][2 col blocks][4 x 8-channel groups][2] GroupNorm sub-partials
  float* s_mean = s_sub + 64;
  float* s_rstd = s_mean + 8;
  float* s_wsc = s_rstd + 8;     // W8: per-output-channel weight scale of this tile

  const int Fg = CONVT ? p.Fin : p.Fout;
  const int Tg = CONVT ? p.Tin : p.Tout;
  const int n_ft = Fg / C::TF, n_tt = (Tg + C::TT - 1) / C::TT;
  // 1-D grid, XCD-aware (launch_t): workgroup ids go round robin over the 8 XCDs, so the ny output-channel tiles (x 4
  // sub-pixel parities for CONVT4) of one spatial tile -- which all read the same input patch -- get ids 8 apart: the
  // same XCD, dispatched together, the patch fetched into that XCD's L2 once instead of once per tile.
  const int ksplit = C::SK && p.ksplit > 1 ? p.ksplit : 1;
  const int ny = p.Cout / NT, nyz = ny * (CONVT ? 4 : ksplit);
  // XCD x walks the contiguous spatial range [x S, x S + S) in order (S = ceil(nsp / 8)), so the tiles one XCD runs
  // together are vertical neighbours whose halo rows its L2 already holds (round 2: -19 % fetched bytes per U-Net
  // evaluation against the 3-D grid, +0.9 % against an interleaved 1-D order)
  const int nsp = p.B * n_ft * n_tt, lin = blockIdx.x, j = lin >> 3, yz = j % nyz;
  int bid = (lin & 7) * ((nsp + 7) >> 3) + j / nyz;
  const int ntile = yz % ny;
  const int par = CONVT ? yz / ny : 0;
  const int split = C::SK ? yz / ny : 0;
  if (bid >= nsp) return;   // grid padding: the whole workgroup, before any barrier
  const int sp_id = bid;    // spatial tile (split-K: the counter / partial slot is per (spatial tile, ntile))
  const int tt = bid % n_tt; bid /= n_tt;
  const int ft = bid % n_ft;
  const int b = bid / n_ft;
  const int f0 = ft * C::TF, t0 = tt * C::TT;
  const int cout0 = ntile * NT;
  const int pf = par >> 1, pt = par & 1;

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar) wave index
  const int wm = wv % C::WM, wn = wv / C::WM;
  const int fi0 = f0 * C::S - C::PAD, ti0 = t0 * C::S - C::PAD;
  const int sub = C::isub(tid);           // this thread's fixed 16-B channel group inside a chunk

  // ---- prologue, ordered so that its global round trips overlap: GroupNorm slot loads, the per-channel
  // coefficients and the mask are issued together; the first patch prefetch goes out before the fp64
  // GroupNorm reduction (which needs barriers) runs.
  double* s_red = reinterpret_cast<double*>(sA);   // the patch area is free until the first chunk
  GnLoad gl;
  if (IN == IN_GN) gl = gn_load(p.gn_part, p.gn_nparts, b);
  if (OUT == OUT_RBOUT) gl = gn_load(p.pre_part, p.pre_nparts, b);
  float c_g = 0.f, c_b = 0.f, c_t = 0.f;            // gamma, beta, time bias of channel tid
  if (IN == IN_GN && tid < p.Cin) {
    c_g = p.gn_gamma[tid]; c_b = p.gn_beta[tid]; c_t = tb_at(p.tb, p.stepp)[(long)b * p.tb_bstride + tid];
  }
  if (OUT == OUT_RBOUT && tid < NT) { c_g = p.pre_gamma[cout0 + tid]; c_b = p.pre_beta[cout0 + tid]; }
  const float c_bias = tid < NT ? p.bias[cout0 + tid] : 0.f;
  const float c_wsc = (W8 && tid < NT) ? p.wscale[cout0 + tid] : 1.f;

  // per-thread patch items, computed once: input position (npos = out of range) and mask
  constexpr int ES = (int)sizeof(A);
  const int npos = p.B * p.Fin * p.Tin;
  int pidx[C::PPT];
  float pm[C::PPT];
  bool frac = false;     // a mask value other than 0/1 among this thread's items (sequence_mask gives 0/1)
#pragma unroll
  for (int j = 0; j < C::PPT; ++j) {
    const int it = tid + 256 * j;
    const int pos = C::ipos(it);   // LDS position
    const int pr = pos / C::PC, pc = C::gcol(pos - pr * C::PC);
    const int fi = fi0 + pr, ti = ti0 + pc;
    const bool ok = pos < C::NPOS && fi >= 0 && fi < p.Fin && ti >= 0 && ti < p.Tin;
    const float m = ok ? mask_at(p.mask, p.T0, b, ti, p.lvl_in) : 0.f;
    int q = ok ? ((b * p.Fin + fi) * p.Tin + ti) : npos;
    if (IN == IN_MASK) {
      if (m == 0.f) q = npos;              // x * 0: the range-checked load returns zeros
    }
    if (IN == IN_MASK || IN == IN_GN) frac |= (m != 0.f && m != 1.f);
    pidx[j] = q;
    pm[j] = m;
  }

  // raw buffer descriptors over the (one or two) input tensors: an offset past the end reads 0
  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.in0, (short)0, npos * p.C0 * ES, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.in1 ? p.in1 : p.in0), (short)0, npos * (p.in1 ? p.C1 : p.C0) * ES, 0x00020000);
  // byte offset of item j = pidx[j] * pos_bytes + sub * 16, formed per load (one VALU op; no offset registers)
  // split-K: this workgroup's input-channel chunks [c_lo, c_lo + nchunk) of nchunk_all
  const int nchunk_all = p.Cin_pad / C::CK;
  const int c_lo = split * nchunk_all / ksplit;
  const int nchunk = (split + 1) * nchunk_all / ksplit - c_lo;
  const int cb0 = c_lo * C::CK;   // first input channel; load_patch / store_patch / issue_patch take offsets from it
  int pos_bytes = (IN != IN_INPUT && p.C1 != 0 && cb0 >= p.C0 ? p.C1 : p.C0) * ES;
  auto set_offsets = [&](int Cs) { pos_bytes = Cs * ES; };
  auto voff = [&](int j) { return pidx[j] * pos_bytes + sub * 16; };

  u32x4 preg[C::PPT];
  auto load_patch = [&](int c0) {
    c0 += cb0;
    if (IN == IN_INPUT) {   // channels {mu, x_t, spk} (diffusion.py:181/184) -- single chunk
#pragma unroll
      for (int j = 0; j < C::PPT; ++j) {
        u32x4 u = {0u, 0u, 0u, 0u};
        if (pidx[j] < npos && sub == 0) {
          u[0] = __float_as_uint(p.mu[pidx[j]]);
          u[1] = __float_as_uint(p.xt[pidx[j]]);
          if (p.cin_input == 3) u[2] = __float_as_uint(p.spk_s[(long)b * p.Fin + (pidx[j] / p.Tin) % p.Fin]);
        }
        preg[j] = u;
      }
    } else if (c0 < p.C0) {
#pragma unroll
      for (int j = 0; j < C::PPT; ++j) preg[j] = __builtin_amdgcn_raw_buffer_load_b128(rs0, voff(j), c0 * ES, 0);
    } else {
#pragma unroll
      for (int j = 0; j < C::PPT; ++j)
        preg[j] = __builtin_amdgcn_raw_buffer_load_b128(rs1, voff(j), (c0 - p.C0) * ES, 0);
    }
  };
  // A8: one item = 8 channels of a position -> 8 e4m3 bytes, with one E8M0 scale per (position, 32-channel chunk): the
  // four items of a position sit in lanes 4i..4i+3 (sub = tid & 3), whose |x| maxima meet through two DPP quad swaps.
  // Scale 2^k with k the least exponent that keeps max|x| / 2^k <= 448 (e4m3's largest finite); an all-zero block
  // (padding, masked frames) gets 2^0. The conversion divides by the scale (v_cvt_scalef32_pk_fp8_f32, probed).
  auto store_item_a8 = [&](int it, const float* v, bool zero) {
    float am = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) am = fmaxf(am, fabsf(v[k]));
    am = fmaxf(am, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(am), 0xB1, 0xf, 0xf, false)));   // lane ^ 1
    am = fmaxf(am, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(am), 0x4E, 0xf, 0xf, false)));   // lane ^ 2
    const unsigned ab = __float_as_uint(am);
    int e = (int)(ab >> 23) - 8 + ((ab & 0x7fffffu) > 0x600000u ? 1 : 0);   // max|x| <= 1.75 * 2^(8 + k)
    e = ab == 0u ? 127 : (e < 1 ? 1 : e);
    const float sc = __uint_as_float((unsigned)e << 23);
    typedef short v2s __attribute__((ext_vector_type(2)));
    unsigned q[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      v2s o = {0, 0};
      o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, v[4 * i], v[4 * i + 1], sc, false);
      o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, v[4 * i + 2], v[4 * i + 3], sc, true);
      q[i] = zero ? 0u : __builtin_bit_cast(unsigned, o);
    }
    if (it < C::PITEMS) {
      char* dst = sA + (it / C::SUBS) * C::POSB;
      *reinterpret_cast<uint2*>(dst + sub * 8) = make_uint2(q[0], q[1]);
      if (sub == 0) dst[32] = (char)e;
    }
  };
  auto store_patch = [&](int c0) {
    c0 += cb0;
    float sc[C::ICH], sh[C::ICH], tb[C::ICH];
    if (IN == IN_GN) {
#pragma unroll
      for (int k = 0; k < C::ICH; ++k) {
        const int c = c0 + sub * C::ICH + k;
        sc[k] = s_sc[c]; sh[k] = s_sh[c]; tb[k] = s_tb[c];
      }
    }
    if constexpr (C::A8) {   // every lane takes part (the scale exchange is a DPP swap)
#pragma unroll
      for (int j = 0; j < C::PPT; ++j) {
        float v[8];
        item_to_f(make_uint4(preg[j][0], preg[j][1], preg[j][2], preg[j][3]), v, A());
        if (IN == IN_GN) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = gn_mish_tb_l2(v[k], sc[k], sh[k], tb[k]);
        }
        if ((IN == IN_GN || IN == IN_MASK) && frac) {
          const float m = pm[j];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] *= m;
        }
        // IN_GN, masks in {0, 1}: a masked position's bytes are zeroed after the conversion (its scale byte is then
        // immaterial); IN_MASK's masked positions already loaded as zeros
        store_item_a8(tid + 256 * j, v, IN == IN_GN && !frac && pm[j] == 0.f);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < C::PPT; ++j) {
      const int it = tid + 256 * j;
      if (C::ipos(it) < C::NPOS) {
        char* dst = sA + C::ipos(it) * C::POSB + sub * 16;
        const u32x4 u = preg[j];
        if (IN == IN_PLAIN || (IN == IN_MASK && !frac)) {   // zeros already came from the range check
          *reinterpret_cast<u32x4*>(dst) = u;
          continue;
        }
        const float m = pm[j];
        float v[C::ICH];
        const uint4 w = make_uint4(u[0], u[1], u[2], u[3]);
        if (IN == IN_INPUT) {
          const float f3[3] = {__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z)};
#pragma unroll
          for (int k = 0; k < C::ICH; ++k) v[k] = (k < 3 ? f3[k < 3 ? k : 0] : 0.f) * m;
        } else {
          item_to_f(w, v, A());
          if (IN == IN_GN && sizeof(A) == 2) {   // (Mish(GN(h)) + tb) * m: m in {0, 1} selects the packed item
#pragma unroll
            for (int k = 0; k < C::ICH; ++k) v[k] = gn_mish_tb_l2(v[k], sc[k], sh[k], tb[k]);
            if (frac) {
#pragma unroll
              for (int k = 0; k < C::ICH; ++k) v[k] *= m;
            }
            const uint4 o = f_to_item(v, A());
            const bool z = !frac && m == 0.f;
            *reinterpret_cast<u32x4*>(dst) = u32x4{z ? 0u : o.x, z ? 0u : o.y, z ? 0u : o.z, z ? 0u : o.w};
            continue;
          } else if (IN == IN_GN) {
#pragma unroll
            for (int k = 0; k < C::ICH; ++k)   // (Mish(GN(h)) * m + tb) * m, m in {0,1}
              v[k] = (mish_act<A>(v[k] * sc[k] + sh[k]) + tb[k]) * m;
          } else {                             // IN_MASK, a fractional mask among this thread's items
#pragma unroll
            for (int k = 0; k < C::ICH; ++k) v[k] *= m;
          }
        }
        const uint4 o = f_to_item(v, A());
        *reinterpret_cast<u32x4*>(dst) = u32x4{o.x, o.y, o.z, o.w};
      }
    }
  };

  f32x16 acc[C::RBW][2];
#pragma unroll
  for (int i = 0; i < C::RBW; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;

  const char* wimg = reinterpret_cast<const char*>(p.w) + (long)b * p.w_bstride;
  wimg += ((long)(par * ny + ntile) * nchunk_all + c_lo) * C::WBYTES;

  auto dma_weights_to = [&](int ch, char* dst) {   // contiguous slab, 1 KiB per wave instruction, compile-time count
    const char* src = wimg + (long)ch * C::WBYTES + lane * 16;
#pragma unroll
    for (int k = 0; k < C::WPIECES; ++k) {
      const int i = wv + 4 * k;
      if (C::WPIECES_ALL % 4 != 0 && i >= C::WPIECES_ALL) break;   // wave-uniform
      __builtin_amdgcn_global_load_lds((const void*)(src + i * 1024),
                                       (__attribute__((address_space(3))) void*)(dst + i * 1024), 16, 0, 0);
    }
  };
  auto dma_weights = [&](int ch) { dma_weights_to(ch, sW); };
  const char* wcur = sW;   // weight slab the MFMAs read (DBW: alternates between the two buffers)
  // Workgroup barrier for the chunk loop without the memory-model fence of __syncthreads() (which waits
  // for every LDS-DMA in flight); what must be visible is made explicit: own LDS stores (lgkmcnt) and
  // this chunk's weight DMA (vmcnt below).
  auto cta_sync = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  load_patch(0);                                      // in flight during the GroupNorm reduction
  if (IN == IN_GN || OUT == OUT_RBOUT) {
    if (IN == IN_GN) gn_finish(gl, p.gn_part, p.gn_nparts, b, p.gn_count, s_mean, s_rstd, s_red);
    else gn_finish(gl, p.pre_part, p.pre_nparts, b, p.pre_count, s_mean, s_rstd, s_red);
    // per-channel GroupNorm scale/shift (and time bias) of the INPUT (IN_GN) / OUTPUT (OUT_RBOUT) channels
    if (IN == IN_GN && tid < p.Cin) {   // bf16 / fp8 operands: the affine in base 2 (gn_mish_tb_l2)
      const int g = tid / (p.Cin >> 3);
      const float sc = c_g * s_rstd[g];
      const float l2 = sizeof(A) == 2 ? kLog2e : 1.f;
      s_sc[tid] = sc * l2; s_sh[tid] = (c_b - s_mean[g] * sc) * l2; s_tb[tid] = c_t;
    }
    if (OUT == OUT_RBOUT && tid < NT) {
      const int g = (cout0 + tid) / (p.Cout >> 3);
      float sc = c_g * s_rstd[g], sh = c_b - s_mean[g] * sc;
      gn_res_coef<A>(sc, sh);   // bf16: base 2 (gn_mish_add)
      s_sc[tid] = sc; s_sh[tid] = sh;
    }
  }
  if (tid < NT) s_bias[tid] = c_bias;                 // all visible after the first chunk barrier
  if (W8 && tid < NT) s_wsc[tid] = c_wsc;

  // MFMAs of taps [t0, t1) of the staged chunk (t0, t1 compile-time at every call site). Software-pipelined
  // over the flattened (tap, row block) steps: the fragments of step i+1 (and the next tap's weight fragments)
  // are read from LDS before step i's two MFMAs, so the LDS latency hides behind them (issued in the natural
  // order, the compiler waited lgkmcnt(0) in front of every MFMA pair).
  // Row block rb of wave wm is block rb * WM + wm (mel row rb * WM / RBT + wm / RBT, 32-frame block wm % RBT):
  // a fragment's LDS address is one per-lane base plus a compile-time offset per (tap, rb), which the ds_read
  // offset field absorbs (no address register per fragment).
  static_assert(C::WM % C::RBT == 0, "row blocks interleave over the waves");
  // ConvTranspose2d(k4, s2, p1): out[2j+p] takes in[j] (k=1) & in[j-1] (k=3) for p=0, in[j+1] (k=0) & in[j]
  // (k=2) for p=1; with the patch origin at (j0-1, j0'-1) tap (a, b) reads patch row 1 + pf - a, column
  // 1 + pt - b. The parity part goes into the base.
  const int a_base = ((wm / C::RBT) * C::S * C::PC + ((wm % C::RBT) * 32 + r) * (C::DEINT ? 1 : C::S) +
                      (CONVT ? (1 + pf) * C::PC + 1 + pt : 0)) * C::POSB + h * (C::KSTEP_B / 2);
  auto load_a = [&](int tap, int rb, int ks) {
    const int dr = CONVT ? -(tap >> 1) : tap / C::KS;
    const int dc = CONVT ? -(tap & 1) : tap % C::KS;
    const int dci = C::DEINT ? (dc == 1 ? C::ODDC : dc >> 1) : dc;   // (stride 2: column 2r + dc, deinterleaved)
    const int off = ((rb * (C::WM / C::RBT) * C::S + dr) * C::PC + dci) * C::POSB + ks * C::KSTEP_B;
    return Mma<A>::load(sA + a_base + off);
  };
  auto load_b = [&](int tap, int cb, int ks) {
    const int koff = ks * C::KSTEP_B + h * (C::KSTEP_B / 2);
    const int row = wn * 64 + cb * 32 + r;
    if constexpr (W8)   // 8-byte units swizzled per row (wimage.h conv8_swz; row base is a multiple of 32)
      return w8_frag(wcur + row * C::WROW + ((2 * tap + h) ^ conv8_swz(C::NTAP, r)) * 8);
    else if (tap < C::NA)
      return Mma<A>::load(wcur + row * C::WROW + tap * C::CKB + koff);
    else
      return Mma<A>::load(wcur + C::HA + row * C::WROWB + (tap - C::NA) * C::CKB + koff);
  };
  auto mma_taps = [&](int t0, int t1) {
    constexpr int RB = C::RBW, KS = C::KSTEPS;
    frag fa[2], fb[2][2];
    fa[0] = load_a(t0, 0, 0);
    fb[0][0] = load_b(t0, 0, 0);
    fb[0][1] = load_b(t0, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, W8 ? 1 : 3, 0);   // LDS reads of the first step
#pragma unroll
    for (int i = 0; i < C::NTAP * KS * RB; ++i) {
      const int u = i / RB, rb = i % RB;          // u = tap-kstep unit
      const int tap = t0 + u / KS, ks = u % KS;
      if (tap >= t1) break;
      const int n = i + 1, un = n / RB, rbn = n % RB;
      const int tapn = t0 + un / KS, ksn = un % KS;
      if (tapn < t1) {
        if (rbn == 0) {                             // next unit: its weight fragments first
          fb[un & 1][0] = load_b(tapn, 0, ksn);
          fb[un & 1][1] = load_b(tapn, 1, ksn);
        }
        fa[n & 1] = load_a(tapn, rbn, ksn);
      }
      // weights as the A operand, positions as B: the accumulator is channel x position (epilogue below)
      Mma<A>::mma(fb[u & 1][0], fa[i & 1], acc[rb][0]);
      Mma<A>::mma(fb[u & 1][1], fa[i & 1], acc[rb][1]);
      // pin the order: step i+1's LDS reads, then step i's MFMAs (the compiler otherwise groups a tap's reads
      // ahead of its MFMAs behind one lgkmcnt(0))
      if constexpr (sizeof(A) == 2 && !W8) {
        if (tapn < t1 && rbn == 0) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        if (tapn < t1 && rbn != 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
    }
  };
  // A8 MFMAs of the staged chunk: K = 64 per v_mfma_scale_f32_32x32x64_f8f6f4 = two taps x 32 channels. Lane (., h) of
  // both operands holds channels 16h..16h+15 of tap t in bytes 0..15 and of tap t' in bytes 16..31, so the patch
  // operand's scale block 0 (bytes 0..15 of both lane halves) is tap t's 32 channels of one position and block 1 tap
  // t''s: lane (c, 0) supplies the E8M0 scale of column c's tap-t position, lane (c, 1) that of its tap-t' position
  // (the probed operand semantics, tools/micro/mfma_scale_probe.hip). Taps go in pairs (0,1) (2,3) (4,5) (6,7) (8,9):
  // slot 9 of the weight image is zero and its patch half re-reads tap 8's position.
  typedef int v8i_t __attribute__((ext_vector_type(8)));
  struct FragP { v8i_t v; int s; };
  int scale_one = 127;                  // weight operand: E8M0 1.0 (its per-channel fp32 scale is applied in the epilogue)
  if constexpr (C::A8) asm volatile("" : "+v"(scale_one));   // held in a VGPR, as the scale operands are read per lane
  const int a8_base = ((wm / C::RBT) * C::PC + (wm % C::RBT) * 32 + r) * C::POSB;   // (stride 1, not transposed)
  // scale byte of lane h = 1: tap t + 1 = the next column, except pair (2, 3) (tap 3 opens the next row) and pair 4
  const int a8_sc1 = a8_base + 32 + (h ? C::POSB : 0), a8_sc2 = a8_base + 32 + (h ? (C::PC - 2) * C::POSB : 0),
            a8_sc4 = a8_base + 32;
  auto a8_off = [&](int tap, int rb) {
    tap = tap > 8 ? 8 : tap;
    return ((rb * (C::WM / C::RBT) + tap / 3) * C::PC + tap % 3) * C::POSB;
  };
  auto load_pa8 = [&](int pr, int rb) {
    const char* base = sA + a8_base + h * 16;
    const u32x4 lo = *reinterpret_cast<const u32x4*>(base + a8_off(2 * pr, rb));
    const u32x4 hi = *reinterpret_cast<const u32x4*>(base + a8_off(2 * pr + 1, rb));
    FragP f;
    f.v = v8i_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    const int sb = pr == 1 ? a8_sc2 : pr == 4 ? a8_sc4 : a8_sc1;
    f.s = *reinterpret_cast<const unsigned char*>(sA + sb + a8_off(2 * pr, rb));
    return f;
  };
  auto load_wa8 = [&](int pr, int cb) {   // pairs 0-2 in half A, 3-4 in half B
    const int row = wn * 64 + cb * 32 + r;
    const char* base = pr < 3 ? wcur + row * C::WROW + h * 16 + pr * 64
                              : wcur + C::HA + row * C::WROWB + h * 16 + (pr - 3) * 64;
    const u32x4 lo = *reinterpret_cast<const u32x4*>(base);
    const u32x4 hi = *reinterpret_cast<const u32x4*>(base + 32);
    return v8i_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  auto mma_a8 = [&](auto P0, auto P1) {   // pairs [P0, P1): compile-time (std::integral_constant), so every index folds
    constexpr int RB = C::RBW, p0 = decltype(P0)::value, NP = decltype(P1)::value - p0;
    // weight fragments double-buffered (the next pair's read one step ahead) when the registers allow; 128-wide tiles
    // (4 row blocks, 128 accumulator VGPRs) read them after the pair's last MFMAs instead
    constexpr bool WDB = RB < 4;
    FragP fa[2];
    v8i_t fb[WDB ? 2 : 1][2];
    fa[0] = load_pa8(p0, 0);
    fb[0][0] = load_wa8(p0, 0);
    fb[0][1] = load_wa8(p0, 1);
    __builtin_amdgcn_sched_group_barrier(0x100, 7, 0);   // LDS reads of the first step
#pragma unroll
    for (int i = 0; i < NP * RB; ++i) {
      const int u = i / RB, rb = i % RB;
      const int n = i + 1, un = n / RB, rbn = n % RB;
      const int wb = WDB ? (u & 1) : 0;
      if (un < NP) {                                    // step i+1's fragments ahead of step i's MFMAs
        if (WDB && rbn == 0) {
          fb[un & 1][0] = load_wa8(p0 + un, 0);
          fb[un & 1][1] = load_wa8(p0 + un, 1);
        }
        fa[n & 1] = load_pa8(p0 + un, rbn);
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        acc[rb][cb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fb[wb][cb], fa[i & 1].v, acc[rb][cb], 0, 0, 0,
                                                                      scale_one, 0, fa[i & 1].s);
      // pin the order (the scheduler otherwise hoists every fragment read of the call ahead of the MFMAs)
      if constexpr (WDB) {
        if (un < NP && rbn == 0) __builtin_amdgcn_sched_group_barrier(0x100, 7, 0);
        if (un < NP && rbn != 0) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      } else {
        if (un < NP) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if (un < NP && rbn == 0) {                      // the pair's last MFMAs issued: its weights are free
          fb[0][0] = load_wa8(p0 + un, 0);
          fb[0][1] = load_wa8(p0 + un, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        }
      }
    }
    // Keep this call's MFMAs ahead of the barrier that follows it: MFMAs touch no memory, so the compiler otherwise
    // sinks the half-A MFMAs below the next barrier and the half-B DMA, next to half B's -- every fragment of the
    // chunk live at once (256 VGPRs, 200-490 spilled).
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) asm volatile("" : "+v"(acc[rb][cb]));
  };
  // patch loads of chunk k (channels k*CK..): switch to the second tensor's offsets at the concat boundary
  auto issue_patch = [&](int k) {
    const int ck0 = k * C::CK;
    if (IN != IN_INPUT && p.C1 != 0 && p.C1 != p.C0 && cb0 + ck0 == p.C0) set_offsets(p.C1);
    load_patch(ck0);
  };

  if constexpr (C::SPLIT) {
    // Per chunk ch (3 barriers): [A(ch) landed] taps of half A | [B(ch) landed, A free] stage A(ch+1), taps of
    // half B | [B and patch free] patch ch+1 -> LDS, stage B(ch+1), patch loads of ch+2. VMEM issue order per
    // wave: A(ch+1), B(ch+1), patch(ch+2) -- the counted waits below retire exactly the needed group (in-order
    // vmcnt; the compiler's own waits cover the patch registers).
    auto dma_half = [&](int ch, int half) {
      const char* src = wimg + (long)ch * C::WBYTES + (half ? C::HA : 0) + lane * 16;
      char* dst = sW + (half ? C::HA : 0);
#pragma unroll
      for (int k = 0; k < (half ? C::PB : C::PA); ++k) {
        const int i = wv + 4 * k;
        __builtin_amdgcn_global_load_lds((const void*)(src + i * 1024),
                                         (__attribute__((address_space(3))) void*)(dst + i * 1024), 16, 0, 0);
      }
    };
    lds_barrier();                                     // s_sc / s_sh / s_tb / s_bias visible; s_red (sA) free
    dma_half(0, 0);
    store_patch(0);
    dma_half(0, 1);
    if (nchunk > 1) issue_patch(1);
    for (int ch = 0; ch < nchunk; ++ch) {
      const bool more = ch + 1 < nchunk;             // patch(ch+1) loads are in flight
      if (more) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::PB + C::PPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::PB) : "memory");
      cta_sync();                                      // A(ch) landed for every wave; patch(ch) stores visible
      if constexpr (C::A8) mma_a8(std::integral_constant<int, 0>{}, std::integral_constant<int, 3>{});
      else mma_taps(0, C::NA);
      if (more) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::PPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      cta_sync();                                      // B(ch) landed; every wave is done with half A
      if (more) dma_half(ch + 1, 0);
      if constexpr (C::A8) mma_a8(std::integral_constant<int, 3>{}, std::integral_constant<int, 5>{});
      else mma_taps(C::NA, C::NTAP);
      if (more) {
        cta_sync();                                    // half B and the patch are free
        store_patch((ch + 1) * C::CK);
        dma_half(ch + 1, 1);
        if (ch + 2 < nchunk) issue_patch(ch + 2);
      }
    }
  } else if constexpr (C::DBW) {
    // Per chunk ch: [MFMAs of ch-1 done] patch ch -> LDS (its registers, loaded one chunk ahead, arrive after
    // weight slab ch, which was issued before them: in-order vmcnt), weight DMA of ch+1 into the other buffer,
    // counted wait leaving only that DMA in flight | [patch and slab ch visible] patch loads of ch+1, MFMAs.
    char* const sW1 = sW + C::WBYTES;
    dma_weights(0);
    for (int ch = 0; ch < nchunk; ++ch) {
      cta_sync();
      store_patch(ch * C::CK);
      if (ch + 1 < nchunk) {
        dma_weights_to(ch + 1, (ch & 1) ? sW : sW1);
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::WPIECES) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      cta_sync();
      if (ch + 1 < nchunk) issue_patch(ch + 1);
      wcur = (ch & 1) ? sW1 : sW;
      mma_taps(0, C::NTAP);
    }
  } else {
    for (int ch = 0; ch < nchunk; ++ch) {
      const int c0 = ch * C::CK;
      cta_sync();                                        // previous chunk's fragments are consumed
      dma_weights(ch);                                   // issued first: its latency overlaps the patch store
      store_patch(c0);
      // The weight DMA must have landed before any wave reads sW; the compiler does not track
      // global_load_lds reliably (it was missing in the 1x1/128-wide instantiation: an intermittent,
      // load-dependent race), so the wait is explicit.
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      cta_sync();
      if (ch + 1 < nchunk) issue_patch(ch + 1);        // in flight during this chunk's MFMAs
      mma_taps(0, C::NTAP);
    }
  }

  if constexpr (C::SK) {
    if (ksplit > 1) {   // split-K: publish this split's accumulators; the tile's last workgroup reduces and goes on
      // The partials and the counter are accessed as agent-scope relaxed atomics (stores / loads at the device
      // coherence point, past the XCDs' non-coherent L2s; vector memory instructions) and ordered by waiting for the
      // stores' completion before the counter increment: a __threadfence() here (L2 write-back + invalidate per
      // workgroup) measured slower than not splitting at all. That lowering (sc1 on the partial stores and loads, the
      // drain and barrier before the increment) is pinned by a CPU audit of the listing: tools/sk_order_audit.py,
      // tests/test_asm_audit.py.
      constexpr int PW = C::RBW * 2 * 16 * 256;   // floats per (tile, split), [rb][cb][k][thread]
      const long slot = (long)sp_id * ny + ntile;
      float* mine = p.sk_part + (slot * ksplit + split) * PW;
#pragma unroll
      for (int rb = 0; rb < C::RBW; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int k = 0; k < 16; ++k)
            __hip_atomic_store(mine + ((rb * 2 + cb) * 16 + k) * 256 + tid, acc[rb][cb][k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's partial stores completed
      __syncthreads();                                    // ... and every other wave's
      int* s_flag = reinterpret_cast<int*>(s_mean);       // (s_mean / s_rstd are prologue-only)
      if (tid == 0) s_flag[0] = __hip_atomic_fetch_add(p.sk_cnt + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if (s_flag[0] != ksplit - 1) return;                // workgroup-uniform: another split finishes the tile
      const float* base = p.sk_part + slot * ksplit * PW;
#pragma unroll
      for (int rb = 0; rb < C::RBW; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          f32x16 sum = acc[rb][cb];
          for (int sp = 0; sp < ksplit; ++sp) {           // fixed order: split 0 + split 1 + ...
            f32x16 v = acc[rb][cb];
            if (sp != split) {
#pragma unroll
              for (int k = 0; k < 16; ++k)
                v[k] = __hip_atomic_load(base + sp * PW + ((rb * 2 + cb) * 16 + k) * 256 + tid, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            }
            if (sp == 0) {
              sum = v;
            } else {
#pragma unroll
              for (int k = 0; k < 16; ++k) sum[k] += v[k];
            }
          }
          acc[rb][cb] = sum;
        }
      if (tid == 0) __hip_atomic_store(p.sk_cnt + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-armed
    }
  }

  // ---- epilogue straight from the accumulators. Lane (r, h) of block (rb, cb) holds channels
  // cb*32 + {0-3, 8-11, 16-19, 24-27} + 4h of position r; one v_permlane32_swap per register pair leaves it
  // with channels cb*32 + 16 pr + 8h + 0..7 (pr = 0, 1) of position r: bias, the ResnetBlock-output /
  // residual fusion, 16-B stores and the GroupNorm partial sums (one 8-channel group per lane) with no LDS
  // round trip. Stores never wait, but vmcnt is one in-order counter: a load waited on after a store waits for
  // that store too, so the residual / pre-activation inputs are loaded ahead of the stores.
  float gs[2][2] = {{0.f, 0.f}, {0.f, 0.f}}, gq[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  A* out = reinterpret_cast<A*>(p.out);
  long obase[C::RBW];
  float om[C::RBW];
#pragma unroll
  for (int rb = 0; rb < C::RBW; ++rb) {
    const int blk = rb * C::WM + wm, lrow = blk / C::RBT, tblk = blk % C::RBT;   // as load_a
    const int tc = t0 + tblk * 32 + r;
    const int frow = f0 + lrow;
    const int fo = CONVT ? 2 * frow + pf : frow;
    const int to = CONVT ? 2 * tc + pt : tc;
    const bool valid = tc < Tg;
    obase[rb] = valid ? (((long)b * p.Fout + fo) * p.Tout + to) * p.Cout + cout0 : -1;
    om[rb] = (OUT == OUT_RBOUT && valid) ? mask_at(p.mask, p.T0, b, to, p.lvl_out) : 0.f;
  }
  constexpr bool EIN = OUT == OUT_RBOUT || OUT == OUT_RESID;
  constexpr int EIPI = (int)sizeof(A) / 2;                         // 16-B items per 8 channels
  constexpr bool EALL = EIN && C::RBW * 2 * 2 * EIPI <= 16;        // all up front (<= 64 VGPRs)
  // otherwise (128-wide tiles) row block rb+1's inputs are loaded before row block rb's stores
  constexpr int NE = EIN ? (EALL ? C::RBW : 2) * 2 * 2 * EIPI : 1;
  uint4 ein[NE];
  const A* esrc = reinterpret_cast<const A*>(OUT == OUT_RBOUT ? p.pre : p.in0);
  auto load_ein = [&](int rb, int slot) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int q = 0; q < EIPI; ++q) {
          const long ob = obase[rb];
          const int cl = wn * 64 + cb * 32 + pr * 16 + 8 * h + 4 * q;
          ein[((slot * 2 + cb) * 2 + pr) * EIPI + q] =
              ob >= 0 ? *reinterpret_cast<const uint4*>(esrc + ob + cl) : make_uint4(0, 0, 0, 0);
        }
  };
  if (EALL) {
#pragma unroll
    for (int rb = 0; rb < C::RBW; ++rb) load_ein(rb, rb);
  } else if (EIN) {
    load_ein(0, 0);
  }
#pragma unroll
  for (int rb = 0; rb < C::RBW; ++rb) {
    if (EIN && !EALL && rb + 1 < C::RBW) load_ein(rb + 1, (rb + 1) & 1);
    const long ob = obase[rb];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = acc[rb][cb][q];
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
        const int cl = wn * 64 + cb * 32 + pr * 16 + 8 * h;   // tile-local first channel of this lane
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(s_bias + cl);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(s_bias + cl + 4);
        float o[8];
        if (W8) {
          const f32x4 s0 = *reinterpret_cast<const f32x4*>(s_wsc + cl);
          const f32x4 s1 = *reinterpret_cast<const f32x4*>(s_wsc + cl + 4);
#pragma unroll
          for (int k = 0; k < 4; ++k) { o[k] = v[8 * pr + k] * s0[k] + b0[k]; o[4 + k] = v[8 * pr + 4 + k] * s1[k] + b1[k]; }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) { o[k] = v[8 * pr + k] + b0[k]; o[4 + k] = v[8 * pr + 4 + k] + b1[k]; }
        }
        if (ob >= 0) {
          if (OUT == OUT_STATS) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              gs[cb][pr] += o[k]; gq[cb][pr] += o[k] * o[k];
              // Keep the two running sums scalar. With packed FP32 enabled the compiler pairs these chains into
              // v_pk_add/v_pk_fma_f32 whose op_sel_hi makes the high lane read the LOW dword of an operand that the
              // previous VALU instruction just wrote; on gfx950 that read can return the stale value (no wait state
              // is inserted): GroupNorm sum-of-squares partials then varied run to run.
              asm volatile("" : "+v"(gs[cb][pr]), "+v"(gq[cb][pr]));
            }
          } else if (EIN) {
            const int ei = (((EALL ? rb : (rb & 1)) * 2 + cb) * 2 + pr) * EIPI;
            float e[8];
            item_to_f(ein[ei], e, A());
            if (EIPI == 2) item_to_f(ein[ei + (EIPI - 1)], e + 4, A());
            if (OUT == OUT_RBOUT) {
              // ResnetBlock output: Mish(GN(h2)) * mask + res_conv(x * mask)   (diffusion.py:57-58, 77-78)
              const float m = om[rb];
#pragma unroll
              for (int k = 0; k < 8; ++k) o[k] = gn_mish_add<A>(e[k], s_sc[cl + k], s_sh[cl + k], o[k], m);
            } else {                                   // Residual: fn(x) + x   (diffusion.py:108)
#pragma unroll
              for (int k = 0; k < 8; ++k) o[k] += e[k];
            }
          }
          if (sizeof(A) == 2) {
            *reinterpret_cast<uint4*>(out + ob + cl) = f_to_item(o, A());
          } else {
            *reinterpret_cast<uint4*>(out + ob + cl) = f_to_item(o, A());
            *reinterpret_cast<uint4*>(out + ob + cl + 4) = f_to_item(o + 4, A());
          }
        }
      }
    }
  }
  if (OUT == OUT_STATS) {
    // per 8-channel group (cb, pr, h): sum over the half-wave's 32 positions, then over waves and groups
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const float s = half_sum32(gs[cb][pr]), q = half_sum32(gq[cb][pr]);
        if (r == 0) {
          s_sub[((wv * 2 + cb) * 4 + pr * 2 + h) * 2 + 0] = s;
          s_sub[((wv * 2 + cb) * 4 + pr * 2 + h) * 2 + 1] = q;
        }
      }
    __syncthreads();
    // ... then per GroupNorm group over waves / sub-groups in a fixed order, one slot per workgroup
    if (tid < 8) {
      const int gshift = __builtin_ctz(p.Cout >> 3);   // group size Cout/8 is a power of two (host check)
      float S = 0.f, Q = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
          for (int g8 = 0; g8 < 4; ++g8) {
            const int co = cout0 + (w / C::WM) * 64 + cb * 32 + g8 * 8;
            if ((co >> gshift) == tid) {
              S += s_sub[((w * 2 + cb) * 4 + g8) * 2 + 0];
              Q += s_sub[((w * 2 + cb) * 4 + g8) * 2 + 1];
            }
          }
      const int nparts = n_ft * n_tt * ny;
      const int slot = (ft * n_tt + tt) * ny + ntile;
      float* dst = p.out_part + ((long)b * nparts + slot) * 16 + tid * 2;
      dst[0] = S;
      dst[1] = Q;
    }
  }
}

template <class A, int KIND, int IN, int OUT, int NT, int W8 = 0, int TF_ = 4>
static hipError_t launch_t(const ConvParams& p, hipStream_t s);

// 3x3 launch with the tile height conv_tf picks (5 rows only exists for 128-wide tiles; the small-batch plan's
// 1-row (128-wide) / 2-row (64-wide) tiles for bf16 activations, with bf16 or fp8 weights)
template <class A, int IN, int NT, int W8>
static hipError_t launch_c3(const ConvParams& p, hipStream_t s) {
  if constexpr (sizeof(A) == 2) {
    if constexpr (NT == 128 && !W8 && IN != IN_INPUT)
      if (p.small && (long)p.B * p.Fout * ((p.Tout + 63) / 64) * (p.Cout / 128) * (p.ksplit > 1 ? p.ksplit : 1) <= 256)
        return launch_t<A, CONV3, IN, OUT_STATS, NT, W8, TF1_DBW>(p, s);
    if (p.small) return launch_t<A, CONV3, IN, OUT_STATS, NT, W8, NT == 128 ? 1 : 2>(p, s);
  }
  if constexpr (NT == 128 && IN != IN_INPUT && W8 != 2)   // (A8: 4-row tiles)
    if (conv_tf(CONV3, IN, NT, p.Cout, p.Fout) == 5) return launch_t<A, CONV3, IN, OUT_STATS, NT, W8, 5>(p, s);
  return launch_t<A, CONV3, IN, OUT_STATS, NT, W8, 4>(p, s);
}
template <class A, int NT, int W8>
static hipError_t launch_ct(const ConvParams& p, hipStream_t s) {   // Upsample (f = fine grid rows, as conv_tf takes)
  if constexpr (NT == 128)
    if (conv_tf(CONVT4, IN_MASK, NT, p.Cout, p.Fout) == 5) return launch_t<A, CONVT4, IN_MASK, OUT_PLAIN, NT, W8, 5>(p, s);
  return launch_t<A, CONVT4, IN_MASK, OUT_PLAIN, NT, W8>(p, s);
}
template <class A, int IN, int OUT, int NT>
static hipError_t launch_c1(const ConvParams& p, hipStream_t s) {
  if constexpr (sizeof(A) == 2)
    if (p.small) return launch_t<A, CONV1, IN, OUT, NT, 0, NT == 128 ? 1 : 2>(p, s);
  if constexpr (NT == 128 && IN != IN_INPUT)
    if (conv_tf(CONV1, IN, NT, p.Cout, p.Fout) == 5) return launch_t<A, CONV1, IN, OUT, NT, 0, 5>(p, s);
  return launch_t<A, CONV1, IN, OUT, NT>(p, s);
}

template <class A, int KIND, int IN, int OUT, int NT, int W8, int TF_>
static hipError_t launch_t(const ConvParams& p, hipStream_t s) {
  typedef ConvCfg<A, KIND, IN, OUT, NT, W8, TF_> C;
  const int Fg = (KIND == CONVT4) ? p.Fin : p.Fout;
  const int Tg = (KIND == CONVT4) ? p.Tin : p.Tout;
  if (Fg % C::TF != 0 || p.Cout % NT != 0 || p.Cin_pad % C::CK != 0) return hipErrorInvalidValue;
  if (OUT == OUT_STATS && ((p.Cout >> 3) & ((p.Cout >> 3) - 1)) != 0) return hipErrorInvalidValue;  // group size 2^k
  if ((long)p.B * p.Fin * p.Tin * (p.C0 > p.C1 ? p.C0 : p.C1) * (long)sizeof(A) >= (1L << 31))
    return hipErrorInvalidValue;   // raw buffer ranges are 32-bit
  const long nsp = (long)p.B * (Fg / C::TF) * ((Tg + C::TT - 1) / C::TT);   // spatial tiles
  const unsigned ks = C::SK && p.ksplit > 1 ? (unsigned)p.ksplit : 1u;
  if (ks > 1 && (ks > (unsigned)(p.Cin_pad / C::CK) || !p.sk_part || !p.sk_cnt)) return hipErrorInvalidValue;
  const unsigned nyz = (unsigned)(p.Cout / NT) * (KIND == CONVT4 ? 4u : ks);
  const dim3 grid((unsigned)(8 * nyz * ((nsp + 7) / 8)));
  if (W8 && !p.wscale) return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_kernel<A, KIND, IN, OUT, NT, W8, TF_>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

template <class A, int NT>
static hipError_t dispatch(ConvKind kind, InMode im, OutMode om, const ConvParams& p, hipStream_t s) {
  // Instantiated combinations (the U-Net uses exactly these):
  if (kind == CONV3 && im == IN_INPUT && om == OUT_STATS) return launch_c3<A, IN_INPUT, NT, 0>(p, s);
  if (kind == CONV3 && im == IN_MASK && om == OUT_STATS) return launch_c3<A, IN_MASK, NT, 0>(p, s);
  if (kind == CONV3 && im == IN_GN && om == OUT_STATS) return launch_c3<A, IN_GN, NT, 0>(p, s);
  if (kind == CONV3 && im == IN_PLAIN && om == OUT_STATS) return launch_c3<A, IN_PLAIN, NT, 0>(p, s);
  if (kind == CONV1 && im == IN_INPUT && om == OUT_RBOUT) return launch_c1<A, IN_INPUT, OUT_RBOUT, NT>(p, s);
  if (kind == CONV1 && im == IN_MASK && om == OUT_RBOUT) return launch_c1<A, IN_MASK, OUT_RBOUT, NT>(p, s);
  if (kind == CONV1 && im == IN_PLAIN && om == OUT_RESID) return launch_c1<A, IN_PLAIN, OUT_RESID, NT>(p, s);
  if (kind == CONV3_S2 && im == IN_MASK && om == OUT_PLAIN) return launch_t<A, CONV3_S2, IN_MASK, OUT_PLAIN, NT>(p, s);
  if (kind == CONVT4 && im == IN_MASK && om == OUT_PLAIN) return launch_ct<A, NT, 0>(p, s);
  return hipErrorNotSupported;
}

// fp8-weight instantiations (GT_BF16_W8): the 3x3, stride-2 and transposed convs
template <int NT>
static hipError_t dispatch_w8(ConvKind kind, InMode im, OutMode om, const ConvParams& p, hipStream_t s) {
  if (kind == CONV3 && om == OUT_STATS) {
    if (im == IN_INPUT) return launch_c3<bf16, IN_INPUT, NT, 1>(p, s);
    if (im == IN_MASK) return launch_c3<bf16, IN_MASK, NT, 1>(p, s);
    if (im == IN_GN) return launch_c3<bf16, IN_GN, NT, 1>(p, s);
    if (im == IN_PLAIN) return launch_c3<bf16, IN_PLAIN, NT, 1>(p, s);
  }
  if (kind == CONV3_S2 && im == IN_MASK && om == OUT_PLAIN) return launch_t<bf16, CONV3_S2, IN_MASK, OUT_PLAIN, NT, 1>(p, s);
  if (kind == CONVT4 && im == IN_MASK && om == OUT_PLAIN) return launch_ct<bf16, NT, 1>(p, s);
  return hipErrorNotSupported;
}
// fp8-operand instantiations (GT_FP8, conv_wimga8 images): the stride-1 3x3 convs over activations
template <int NT>
static hipError_t dispatch_a8(ConvKind kind, InMode im, OutMode om, const ConvParams& p, hipStream_t s) {
  if (kind == CONV3 && om == OUT_STATS) {
    if (im == IN_MASK) return launch_c3<bf16, IN_MASK, NT, 2>(p, s);
    if (im == IN_GN) return launch_c3<bf16, IN_GN, NT, 2>(p, s);
    if (im == IN_PLAIN) return launch_c3<bf16, IN_PLAIN, NT, 2>(p, s);
  }
  return hipErrorNotSupported;
}

int conv_small_ksplit(int F, int T, int Cout, int Cin_pad, int target, int a8) {
  if (Cout % 128 != 0 || target <= 0) return 1;
  const long tiles = (long)F * ((T + 63) / 64) * (Cout / 128);   // 1-row 64-frame tiles of one utterance
  const int nchunk = Cin_pad / (a8 ? 32 : conv_ckb(1, 9, Cin_pad) / 2);   // input chunks (ConvCfg::CK of these tiles)
  long ks = target / tiles;
  ks = std::min<long>(ks, std::min(4, nchunk / 2));              // at least two chunks per split
  return ks > 1 ? (int)ks : 1;
}

int conv_gn_nparts(int act_bf16, InMode im, int F, int T, int Cout, int small, int a8) {   // CONV3: TF rows x 64 frames x NT
  const int nt = conv_nt(act_bf16, Cout);
  const int tf = (a8 && !small) ? 4 : conv_tf(CONV3, im, nt, Cout, F, small);   // launch_c3: A8 never takes 5-row tiles
  return (F / tf) * ((T + 63) / 64) * (Cout / nt);
}

hipError_t launch_conv(int act_bf16, ConvKind kind, InMode im, OutMode om, const ConvParams& p, hipStream_t s) {
  if (p.small && !act_bf16) return hipErrorNotSupported;   // small-batch plan: bf16 weights and activations only
  if (p.wscale) {   // fp8 weight image
    if (!act_bf16) return hipErrorNotSupported;
    if (p.a8) return conv_nt(1, p.Cout) == 128 ? dispatch_a8<128>(kind, im, om, p, s) : dispatch_a8<64>(kind, im, om, p, s);
    return conv_nt(1, p.Cout) == 128 ? dispatch_w8<128>(kind, im, om, p, s) : dispatch_w8<64>(kind, im, om, p, s);
  }
  if (!act_bf16) return dispatch<float, 64>(kind, im, om, p, s);
  return conv_nt(1, p.Cout) == 128 ? dispatch<bf16, 128>(kind, im, om, p, s) : dispatch<bf16, 64>(kind, im, om, p, s);
}

}  // namespace gt
