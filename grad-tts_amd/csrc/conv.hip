// Implicit-GEMM convolutions of the Grad-TTS score U-Net on CDNA4 MFMA.
//
// One kernel template covers every convolution of GradLogPEstimator2d (model/diffusion.py:49-216):
//   CONV3    3x3 stride 1 pad 1   -- Block.block[0]            (diffusion.py:52)
//   CONV3_S2 3x3 stride 2 pad 1   -- Downsample                (diffusion.py:33)
//   CONV1    1x1                  -- ResnetBlock.res_conv (:70) and the folded LinearAttention output
//   CONVT4   ConvTranspose 4x4 s2 -- Upsample (diffusion.py:24) as four 2x2 sub-pixel convolutions
// GEMM view: M = output frames of a tile (4 mel rows x 32*RB frames), N = 64 output channels,
// K = taps x input channels. Four waves, wave w owns mel row f0+w; each wave holds RB x 2 32x32 fp32
// accumulators. Per input-channel chunk (64 B per position = 32 bf16 / 16 fp32 channels) the
// workgroup stages the input patch (with the producer's GroupNorm-apply + Mish + mask + time-bias
// fused into the load: "IN_GN") and the weight slab into LDS, then runs the tap x k-step MFMA loop.
// LDS rows are padded to 80 B per position / NTAP*64+16 B per output channel so the 16-B fragment
// reads of a 16-lane group hit 16 distinct bank slots.
// Epilogues: +bias, GroupNorm partial sums (fp64 atomics, all grid positions incl. padded frames),
// ResnetBlock output (Mish(GN(h2))*mask + res), attention residual.
#include "common.h"
#include "kernels.h"

namespace gt {

template <class A, int KIND, int IN, int OUT, int RB>
__global__ __launch_bounds__(256) void conv_kernel(ConvParams p) {
  constexpr bool CONVT = KIND == CONVT4;
  constexpr int KS = (KIND == CONV1) ? 1 : 3;
  constexpr int S = (KIND == CONV3_S2) ? 2 : 1;
  constexpr int TF = 4, TT = 32 * RB;
  constexpr int NTAP = CONVT ? 4 : KS * KS;
  constexpr int PAD = (KIND == CONV1) ? 0 : 1;
  constexpr int PR = (TF - 1) * S + KS;
  constexpr int PC = (TT - 1) * S + KS;
  constexpr int POSB = 80;
  constexpr int WROW = NTAP * 64 + 16;
  constexpr int CK = 64 / (int)sizeof(A);
  constexpr int ICH = 16 / (int)sizeof(A);
  constexpr int KSTEP_B = 16 * (int)sizeof(A);
  constexpr int KSTEPS = 64 / KSTEP_B;
  typedef typename Mma<A>::frag frag;

  __shared__ __attribute__((aligned(16))) char smem[PR * PC * POSB + 64 * WROW];
  __shared__ float s_sc[256], s_sh[256], s_tb[256];   // IN_GN: per input channel; OUT_RBOUT: per tile cout
  char* sA = smem;
  char* sW = smem + PR * PC * POSB;

  const int Fg = CONVT ? p.Fin : p.Fout;
  const int Tg = CONVT ? p.Tin : p.Tout;
  const int n_ft = Fg / TF, n_tt = (Tg + TT - 1) / TT;
  int bid = blockIdx.x;
  const int tt = bid % n_tt; bid /= n_tt;
  const int ft = bid % n_ft;
  const int b = bid / n_ft;
  const int f0 = ft * TF, t0 = tt * TT;
  const int cout0 = blockIdx.y * 64;
  const int par = blockIdx.z, pf = par >> 1, pt = par & 1;

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  const int fi0 = f0 * S - PAD, ti0 = t0 * S - PAD;

  if (IN == IN_GN) {
    for (int c = tid; c < p.Cin; c += 256) {
      float sc, sh;
      gn_scale_shift(p.gn_stats, b, p.Cin, c, p.gn_count, p.gn_gamma, p.gn_beta, sc, sh);
      s_sc[c] = sc; s_sh[c] = sh; s_tb[c] = p.tb[(long)b * p.tb_bstride + c];
    }
  }
  if (OUT == OUT_RBOUT) {
    if (tid < 64) {
      float sc, sh;
      gn_scale_shift(p.pre_stats, b, p.Cout, cout0 + tid, p.pre_count, p.pre_gamma, p.pre_beta, sc, sh);
      s_sc[tid] = sc; s_sh[tid] = sh;
    }
  }

  f32x16 acc[RB][2];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;

  const A* wbase = reinterpret_cast<const A*>(p.w) + (long)b * p.w_bstride +
                   (CONVT ? (long)par * p.Cout * NTAP * p.Cin_pad : 0L);
  const int nchunk = p.Cin_pad / CK;

  for (int ch = 0; ch < nchunk; ++ch) {
    const int c0 = ch * CK;
    __syncthreads();
    // ---- stage the input patch (transform fused into the load)
    for (int it = tid; it < PR * PC * 4; it += 256) {
      const int sub = it & 3, pos = it >> 2;
      const int pr = pos / PC, pc = pos - pr * PC;
      const int fi = fi0 + pr, ti = ti0 + pc;
      float v[ICH];
#pragma unroll
      for (int k = 0; k < ICH; ++k) v[k] = 0.f;
      if (fi >= 0 && fi < p.Fin && ti >= 0 && ti < p.Tin) {
        const int c = c0 + sub * ICH;
        const float m = mask_at(p.mask, p.T0, b, ti, p.lvl_in);
        if (IN == IN_INPUT) {
          const long o = ((long)b * p.Fin + fi) * p.Tin + ti;
#pragma unroll
          for (int k = 0; k < ICH; ++k) {
            const int cc = c + k;
            float x = 0.f;
            if (cc == 0) x = p.mu[o];
            else if (cc == 1) x = p.xt[o];
            else if (cc == 2 && p.cin_input == 3) x = p.spk_s[(long)b * p.Fin + fi];
            v[k] = x * m;
          }
        } else {
          const A* src; int cs, Cs;
          if (c < p.C0) { src = reinterpret_cast<const A*>(p.in0); cs = c; Cs = p.C0; }
          else { src = reinterpret_cast<const A*>(p.in1); cs = c - p.C0; Cs = p.C1; }
          const uint4 u = *reinterpret_cast<const uint4*>(src + (((long)b * p.Fin + fi) * p.Tin + ti) * Cs + cs);
          item_to_f(u, v, A());
          if (IN == IN_GN) {
#pragma unroll
            for (int k = 0; k < ICH; ++k) {
              const float y = v[k] * s_sc[c + k] + s_sh[c + k];
              float z = mishf(y) * m;          // Block: Mish(GN(.)) * mask            (diffusion.py:57-58)
              z = (z + s_tb[c + k]) * m;       // h += mlp(t) ; block2 conv input h*mask (diffusion.py:76,57)
              v[k] = z;
            }
          } else if (IN == IN_MASK) {
#pragma unroll
            for (int k = 0; k < ICH; ++k) v[k] *= m;
          }
        }
      }
      *reinterpret_cast<uint4*>(sA + pos * POSB + sub * 16) = f_to_item(v, A());
    }
    // ---- stage the weight slab [64 cout][NTAP][chunk]
    for (int it = tid; it < 64 * NTAP * 4; it += 256) {
      const int sub = it & 3, rowi = it >> 2;
      const int n = rowi / NTAP, tap = rowi - n * NTAP;
      const uint4 u = *reinterpret_cast<const uint4*>(wbase + ((long)(cout0 + n) * NTAP + tap) * p.Cin_pad + c0 + sub * ICH);
      *reinterpret_cast<uint4*>(sW + n * WROW + tap * 64 + sub * 16) = u;
    }
    __syncthreads();
    // ---- MFMA main loop
#pragma unroll
    for (int tap = 0; tap < NTAP; ++tap) {
      int dr, dc;
      if (CONVT) {
        // ConvTranspose2d(k4, s2, p1): out[2j+p] takes in[j] (k=1) & in[j-1] (k=3) for p=0,
        // in[j+1] (k=0) & in[j] (k=2) for p=1.  Patch origin is (j0-1, j0'-1).
        const int a = tap >> 1, bb = tap & 1;
        dr = 1 + (pf ? (a ? 0 : 1) : (a ? -1 : 0));
        dc = 1 + (pt ? (bb ? 0 : 1) : (bb ? -1 : 0));
      } else {
        dr = tap / KS;
        dc = tap - dr * KS;
      }
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        frag af[RB], bfr[2];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const int prow = wv * S + dr;
          const int pcol = (rb * 32 + r) * S + dc;
          af[rb] = Mma<A>::load(sA + (prow * PC + pcol) * POSB + ks * KSTEP_B + h * (KSTEP_B / 2));
        }
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          bfr[cb] = Mma<A>::load(sW + (cb * 32 + r) * WROW + tap * 64 + ks * KSTEP_B + h * (KSTEP_B / 2));
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) Mma<A>::mma(af[rb], bfr[cb], acc[rb][cb]);
      }
    }
  }

  // ---- epilogue
  A* out = reinterpret_cast<A*>(p.out);
  const int frow = f0 + wv;
  float gs[2] = {0.f, 0.f}, gq[2] = {0.f, 0.f};
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int co = cout0 + cb * 32 + r;
    const float bias = p.bias[co];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int tc = t0 + rb * 32 + acc_row(j, h);
        if (tc < Tg) {
          const int fo = CONVT ? 2 * frow + pf : frow;
          const int to = CONVT ? 2 * tc + pt : tc;
          const long o = (((long)b * p.Fout + fo) * p.Tout + to) * p.Cout + co;
          float v = acc[rb][cb][j] + bias;
          if (OUT == OUT_STATS) {
            gs[cb] += v;
            gq[cb] += v * v;
          } else if (OUT == OUT_RBOUT) {
            // ResnetBlock output: Block2 result + res_conv(x*mask)   (diffusion.py:77-78)
            const float m = mask_at(p.mask, p.T0, b, to, p.lvl_out);
            const float pre = Act<A>::to_f(reinterpret_cast<const A*>(p.pre)[o]);
            v = mishf(pre * s_sc[cb * 32 + r] + s_sh[cb * 32 + r]) * m + v;
          } else if (OUT == OUT_RESID) {
            v = v + Act<A>::to_f(reinterpret_cast<const A*>(p.in0)[o]);   // Residual (diffusion.py:108)
          }
          out[o] = Act<A>::from_f(v);
        }
      }
    }
  }
  if (OUT == OUT_STATS) {
    const int gsz = p.Cout / 8;   // channels per GroupNorm group: 8, 16 or 32
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      float s = gs[cb], q = gq[cb];
      for (int off = 1; off < gsz && off < 32; off <<= 1) {
        s += __shfl_xor(s, off);
        q += __shfl_xor(q, off);
      }
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 32);
      const int co = cout0 + cb * 32 + r;
      if (h == 0 && (r % gsz) == 0) {
        const int g = co / gsz;
        atomicAdd(p.out_stats + (b * 8 + g) * 2 + 0, (double)s);
        atomicAdd(p.out_stats + (b * 8 + g) * 2 + 1, (double)q);
      }
    }
  }
}

template <class A, int KIND, int IN, int OUT>
static hipError_t launch_t(const ConvParams& p, hipStream_t s) {
  constexpr int RB = (KIND == CONV3_S2) ? 1 : 2;
  constexpr int TT = 32 * RB;
  const int Fg = (KIND == CONVT4) ? p.Fin : p.Fout;
  const int Tg = (KIND == CONVT4) ? p.Tin : p.Tout;
  if (Fg % 4 != 0 || p.Cout % 64 != 0) return hipErrorInvalidValue;
  dim3 grid((unsigned)(p.B * (Fg / 4) * ((Tg + TT - 1) / TT)), (unsigned)(p.Cout / 64), KIND == CONVT4 ? 4u : 1u);
  hipLaunchKernelGGL((conv_kernel<A, KIND, IN, OUT, RB>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

template <class A>
static hipError_t dispatch(ConvKind kind, InMode im, OutMode om, const ConvParams& p, hipStream_t s) {
  // Instantiated combinations (the U-Net uses exactly these):
  if (kind == CONV3 && im == IN_INPUT && om == OUT_STATS) return launch_t<A, CONV3, IN_INPUT, OUT_STATS>(p, s);
  if (kind == CONV3 && im == IN_MASK && om == OUT_STATS) return launch_t<A, CONV3, IN_MASK, OUT_STATS>(p, s);
  if (kind == CONV3 && im == IN_GN && om == OUT_STATS) return launch_t<A, CONV3, IN_GN, OUT_STATS>(p, s);
  if (kind == CONV1 && im == IN_INPUT && om == OUT_RBOUT) return launch_t<A, CONV1, IN_INPUT, OUT_RBOUT>(p, s);
  if (kind == CONV1 && im == IN_MASK && om == OUT_RBOUT) return launch_t<A, CONV1, IN_MASK, OUT_RBOUT>(p, s);
  if (kind == CONV1 && im == IN_PLAIN && om == OUT_RESID) return launch_t<A, CONV1, IN_PLAIN, OUT_RESID>(p, s);
  if (kind == CONV3_S2 && im == IN_MASK && om == OUT_PLAIN) return launch_t<A, CONV3_S2, IN_MASK, OUT_PLAIN>(p, s);
  if (kind == CONVT4 && im == IN_MASK && om == OUT_PLAIN) return launch_t<A, CONVT4, IN_MASK, OUT_PLAIN>(p, s);
  return hipErrorNotSupported;
}

hipError_t launch_conv(int act_bf16, ConvKind kind, InMode im, OutMode om, const ConvParams& p, hipStream_t s) {
  return act_bf16 ? dispatch<bf16>(kind, im, om, p, s) : dispatch<float>(kind, im, om, p, s);
}

}  // namespace gt
