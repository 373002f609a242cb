// 1x1 convolutions of the throughput plan, streamed: ResnetBlock.res_conv with the block output formed in the epilogue
// (diffusion.py:70, 77-78: Mish(GN(h2)) * m + res_conv(x * m)) and the folded LinearAttention output with its residual
// (diffusion.py:108: x + M_b x + g b_out, decoder.cpp attention_out).
//
// These are HBM-bound (K = 64..512 input channels per position, 2 * Cin * Cout FLOP against (Cin + 2 Cout) * 2 bytes),
// and conv_kernel ran them latency-bound: its patch came through registers one 32-channel chunk ahead, two barriers a
// chunk, and the epilogue's pre-activation / residual loads were issued only after the last chunk (r06 PMC: waves
// waiting 54-57 % of their cycles, 2.6-4.4 TB/s). Here:
//   * the patch goes global -> LDS by buffer_load ... lds (no VGPRs, no store pass) into a ring of three stages, two
//     chunks ahead of the MFMAs, one barrier per chunk. A stage keeps conv_kernel's LDS layout (80-B positions:
//     conflict-free fragment reads); the DMA writes lane-linear 16-B slots, so the lane that owns a pad slot loads from
//     an offset past the buffer (zeros, no memory traffic), as do masked positions (m = 0) and frames past T;
//   * the weight fragments (L2-resident image, wimage.h, shared by every tile) load straight into registers two chunks
//     ahead; the epilogue's second operand (h2 pre-activation / residual) is loaded at kernel start;
//   * 2-row x 64-frame tiles (128 positions), up to 3 workgroups per CU (37 KB of LDS, <= 168 VGPRs).
// The MFMA sequence of every accumulator is conv_kernel's (32x32x16 bf16, weights as A, 16-channel k-steps in
// ascending channel order), so the output is bit-identical to it for 0/1 masks (tests/test_conv1s_gpu.py). A fractional
// mask (C-ABI callers) multiplies the fp32 accumulator instead of the bf16 operand: res_conv(x m) = m W x + b per
// position (a 1x1 conv is linear per position).
#include "common.h"
#include "kernels.h"
#include "wimage.h"

namespace gt {
namespace c1s {
constexpr int TF = 2, TT = 64, NPOS = TF * TT;     // tile: 2 mel rows x 64 frames
constexpr int CK = 32, POSB = 80;                   // 32 input channels (64 B) per chunk; 80-B position stride in LDS
constexpr int SLOTS = NPOS * (POSB / 16);           // 640 16-B slots (4 data + 1 pad per position)
constexpr int DPW = 3;                              // patch DMA wave instructions per wave and chunk (12 x 64 >= 640)
constexpr int STAGE = 4 * DPW * 64 * 16;            // 12 KiB per stage (slots past 640: scratch, never read)
constexpr int NSTAGE = 3;
constexpr int SMEM = NSTAGE * STAGE + (128 * 3 + 16) * 4;
static_assert(SLOTS <= 4 * DPW * 64, "patch slots fit the DMA instructions");
static_assert(272 * 8 <= STAGE, "the GroupNorm reduction scratch fits one stage");
}  // namespace c1s

template <int IN, int OUT, int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void conv1s_kernel(ConvParams p) {
  using namespace c1s;
  constexpr int WN = NT / 64, WM = 4 / WN, RBT = TT / 32, RBW = TF * RBT / WM;
  constexpr int WROW = conv_wrow(1, 64);                        // 80-B weight rows (wimage.h, 1x1 bf16 image)
  constexpr int WBYTES = conv_habytes(1, NT, 1, 64);            // one chunk of one NT-channel tile
  static_assert(WM % RBT == 0 && RBW >= 1, "row blocks interleave over the waves");

  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  float* s_sc = reinterpret_cast<float*>(smem + NSTAGE * STAGE);
  float* s_sh = s_sc + 128;
  float* s_bias = s_sh + 128;
  float* s_mean = s_bias + 128;
  float* s_rstd = s_mean + 8;

  const int n_ft = p.Fout / TF, n_tt = (p.Tout + TT - 1) / TT;
  const int ny = p.Cout / NT;
  // XCD-aware 1-D grid (as conv_kernel): the ny channel tiles of a spatial tile get ids 8 apart (one XCD, one L2)
  const int nsp = p.B * n_ft * n_tt, lin = blockIdx.x, j8 = lin >> 3;
  const int ntile = j8 % ny;
  int bid = (lin & 7) * ((nsp + 7) >> 3) + j8 / ny;
  if (bid >= nsp) return;   // grid padding: the whole workgroup, before any barrier
  const int tt = bid % n_tt; bid /= n_tt;
  const int ft = bid % n_ft;
  const int b = bid / n_ft;
  const int f0 = ft * TF, t0 = tt * TT, cout0 = ntile * NT;

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv % WM, wn = wv / WM;

  // ---- epilogue operand (h2 pre-activation / residual) of this lane's positions, loaded first
  const int npos = p.B * p.Fin * p.Tin;
  long obase[RBW];
  float om[RBW];
#pragma unroll
  for (int rb = 0; rb < RBW; ++rb) {
    const int blk = rb * WM + wm, lrow = blk / RBT, tblk = blk % RBT;
    const int tc = t0 + tblk * 32 + r;
    const bool valid = tc < p.Tout;
    obase[rb] = valid ? (((long)b * p.Fout + f0 + lrow) * p.Tout + tc) * p.Cout + cout0 : -1;
    om[rb] = (IN == IN_MASK && valid) ? mask_at(p.mask, p.T0, b, tc, p.lvl_out) : 0.f;
  }
  GnLoad gl;
  if (OUT == OUT_RBOUT) gl = gn_load(p.pre_part, p.pre_nparts, b);
  const bf16* esrc = reinterpret_cast<const bf16*>(OUT == OUT_RBOUT ? p.pre : p.in0);
  uint4 ein[RBW][2][2];
#pragma unroll
  for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int cl = wn * 64 + cb * 32 + pr * 16 + 8 * h;
        ein[rb][cb][pr] = obase[rb] >= 0 ? *reinterpret_cast<const uint4*>(esrc + obase[rb] + cl) : make_uint4(0, 0, 0, 0);
      }
  float c_g = 0.f, c_b = 0.f;
  if (OUT == OUT_RBOUT && tid < NT) { c_g = p.pre_gamma[cout0 + tid]; c_b = p.pre_beta[cout0 + tid]; }
  const float c_bias = tid < NT ? p.bias[cout0 + tid] : 0.f;

  // ---- patch slots of this thread: wave instruction i = wv + 4 k covers slots 64 i .. 64 i + 63 (lane-linear)
  int sq[DPW];          // input position, npos (zeros: masked / past T) or -1 (pad / scratch slot)
  int ssub[DPW];
#pragma unroll
  for (int k = 0; k < DPW; ++k) {
    const int s = 64 * (wv + 4 * k) + lane;
    const int pos = s / 5, sub = s - 5 * pos;
    int q = -1;
    if (pos < NPOS && sub < 4) {
      const int fi = f0 + pos / TT, ti = t0 + pos % TT;
      q = npos;
      if (ti < p.Tin) {
        q = (b * p.Fin + fi) * p.Tin + ti;
        if (IN == IN_MASK && mask_at(p.mask, p.T0, b, ti, p.lvl_in) == 0.f) q = npos;   // x * 0
      }
    }
    sq[k] = q;
    ssub[k] = sub;
  }
  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.in0, (short)0, npos * p.C0 * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.in1 ? p.in1 : p.in0), (short)0, npos * (p.in1 ? p.C1 : p.C0) * 2, 0x00020000);
  const int nchunk = p.Cin_pad / CK;
  // Every chunk issues the same VMEM ops (DPW patch DMAs, then 4 weight loads), chunks past the end included (offsets
  // past the buffers: zeros, no memory traffic): the counted waits below and the compiler's own waits for the weight
  // registers then see one issue pattern on every path (with a conditional tail the compiler's loop-carried count fell
  // to the shortest path and it drained everything in front of the MFMAs).
  auto dma_patch = [&](int ch) {   // chunk ch -> stage ch % 3
    const int c0 = ch * CK;
    const bool live = ch < nchunk;
    const bool second = live && p.in1 && c0 >= p.C0;
    const int pb = (second ? p.C1 : p.C0) * 2, soff = live ? (second ? c0 - p.C0 : c0) * 2 : 0;
    char* stage = smem + (ch % NSTAGE) * STAGE;
#pragma unroll
    for (int k = 0; k < DPW; ++k) {
      const unsigned vo = (sq[k] < 0 || !live) ? 0x80000000u : (unsigned)(sq[k] * pb + ssub[k] * 16);
      auto* dst = (__attribute__((address_space(3))) void*)(stage + (wv + 4 * k) * 1024);
      if (second) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs1, dst, 16, vo, soff, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rs0, dst, 16, vo, soff, 0, 0);
    }
  };
  // weight fragments of chunk ch: rows wn*64 + cb*32 + r, k-step ks, lane half h (the A operand)
  // (raw buffer over this tile's image: chunks past the end read zeros)
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(reinterpret_cast<const char*>(p.w) + (long)b * p.w_bstride + (long)ntile * nchunk * WBYTES), (short)0,
      nchunk * WBYTES, 0x00020000);
  const int wl = (wn * 64 + r) * WROW + h * 16;
  auto load_w = [&](int ch, bf16x8 (&w)[2][2]) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        w[cb][ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsw, wl + ch * WBYTES,
                                                                                      cb * 32 * WROW + ks * 32, 0));
  };

  f32x16 acc[RBW][2];
#pragma unroll
  for (int i = 0; i < RBW; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;

  bf16x8 wA[2][2], wB[2][2];
  dma_patch(0);
  load_w(0, wA);
  dma_patch(1);
  load_w(1, wB);

  // GroupNorm of h2 (OUT_RBOUT): scratch in stage 2, which no DMA writes before the first chunk's barrier
  if (OUT == OUT_RBOUT) {
    gn_finish(gl, p.pre_part, p.pre_nparts, b, p.pre_count, s_mean, s_rstd,
              reinterpret_cast<double*>(smem + 2 * STAGE));
    if (tid < NT) {
      const int g = (cout0 + tid) / (p.Cout >> 3);
      float sc = c_g * s_rstd[g], sh = c_b - s_mean[g] * sc;
      gn_res_coef<bf16>(sc, sh);   // base 2 (gn_mish_add)
      s_sc[tid] = sc; s_sh[tid] = sh;
    }
  }
  if (tid < NT) s_bias[tid] = c_bias;   // visible after the first chunk barrier

  const int a_base = ((wm / RBT) * TT + (wm % RBT) * 32 + r) * POSB + h * 16;
  // VMEM issue order per wave: patch(0) w(0) patch(1) w(1) | chunk k: patch(k+2), MFMAs, w(k+2). At the top of chunk k
  // the ops younger than patch(k) are w(k), patch(k+1), w(k+1).
  auto chunk = [&](int ch, bf16x8 (&w)[2][2]) {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 + DPW + 4) : "memory");
    lds_barrier();   // patch(ch) landed for every wave; every wave is done with stage (ch + 2) % 3 = (ch - 1) % 3
    dma_patch(ch + 2);
    const char* st = smem + (ch % NSTAGE) * STAGE + a_base;
    bf16x8 fa[2];
    fa[0] = *reinterpret_cast<const bf16x8*>(st);
#pragma unroll
    for (int i = 0; i < 2 * RBW; ++i) {   // (ks, rb) in conv_kernel's order: k-step outer, row block inner
      const int ks = i / RBW, rb = i % RBW;
      if (i + 1 < 2 * RBW) {
        const int ksn = (i + 1) / RBW, rbn = (i + 1) % RBW;
        fa[(i + 1) & 1] = *reinterpret_cast<const bf16x8*>(st + rbn * (WM / RBT) * TT * POSB + ksn * 32);
      }
      acc[rb][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0][ks], fa[i & 1], acc[rb][0], 0, 0, 0);
      acc[rb][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1][ks], fa[i & 1], acc[rb][1], 0, 0, 0);
    }
    load_w(ch + 2, w);
  };
  for (int ch = 0; ch < nchunk; ch += 2) {   // (nchunk even: conv1s_eligible)
    chunk(ch, wA);
    chunk(ch + 1, wB);
  }
  // the tail's zero DMAs write LDS: drained before the workgroup can end (its LDS is then reallocated)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue straight from the accumulators (conv_kernel's: one v_permlane32_swap per register pair leaves lane
  // (r, h) channels cb*32 + 16 pr + 8h + 0..7 of position r)
  bf16* out = reinterpret_cast<bf16*>(p.out);
#pragma unroll
  for (int rb = 0; rb < RBW; ++rb) {
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
        const int cl = wn * 64 + cb * 32 + pr * 16 + 8 * h;
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(s_bias + cl);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(s_bias + cl + 4);
        float o[8], e[8];
        // IN_MASK: m W x + b (m in {0, 1}: exactly conv_kernel's W (x m) + b; see the header for fractional masks)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[k] = IN == IN_MASK ? fmaf(v[8 * pr + k], om[rb], b0[k]) : v[8 * pr + k] + b0[k];
          o[4 + k] = IN == IN_MASK ? fmaf(v[8 * pr + 4 + k], om[rb], b1[k]) : v[8 * pr + 4 + k] + b1[k];
        }
        item_to_f(ein[rb][cb][pr], e, bf16());
        if (OUT == OUT_RBOUT) {
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = gn_mish_add<bf16>(e[k], s_sc[cl + k], s_sh[cl + k], o[k], om[rb]);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += e[k];
        }
        if (ob >= 0) *reinterpret_cast<uint4*>(out + ob + cl) = f_to_item(o, bf16());
      }
    }
  }
}

bool conv1s_eligible(InMode im, OutMode om, const ConvParams& p) {
  const bool mode = (im == IN_MASK && om == OUT_RBOUT && p.pre && p.pre_part) || (im == IN_PLAIN && om == OUT_RESID && !p.in1);
  const int cin = p.in1 ? p.C0 + p.C1 : p.C0;
  return mode && !p.small && !p.wscale && !p.a8 && p.Fin == p.Fout && p.Tin == p.Tout && p.Fout % c1s::TF == 0 &&
         (p.Cout == 64 || p.Cout % 128 == 0) && p.Cout <= 512 && p.Cin_pad == cin && cin % c1s::CK == 0 &&
         p.C0 % c1s::CK == 0 && cin % (2 * c1s::CK) == 0 && (im != IN_PLAIN || p.Cin == p.Cout) &&
         (long)p.B * p.Fin * p.Tin * (p.C0 > p.C1 ? p.C0 : p.C1) * 2 < (1L << 31);
}

hipError_t launch_conv1s(InMode im, OutMode om, const ConvParams& p, hipStream_t s) {
  if (!conv1s_eligible(im, om, p)) return hipErrorInvalidValue;
  const int nt = conv_nt(1, p.Cout);
  const long nsp = (long)p.B * (p.Fout / c1s::TF) * ((p.Tout + c1s::TT - 1) / c1s::TT);
  const dim3 grid((unsigned)(8 * (p.Cout / nt) * ((nsp + 7) / 8)));
  if (im == IN_MASK) {
    if (nt == 128) hipLaunchKernelGGL((conv1s_kernel<IN_MASK, OUT_RBOUT, 128>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv1s_kernel<IN_MASK, OUT_RBOUT, 64>), grid, dim3(256), 0, s, p);
  } else {
    if (nt == 128) hipLaunchKernelGGL((conv1s_kernel<IN_PLAIN, OUT_RESID, 128>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv1s_kernel<IN_PLAIN, OUT_RESID, 64>), grid, dim3(256), 0, s, p);
  }
  return hipGetLastError();
}

}  // namespace gt
