// Backward of the score U-Net for the training step (model/diffusion.py:16-216 through
// Diffusion.loss_t :274-281), fp32, channels-last activations [B][F_l][T_l][C] as in the forward.
//
// Generic building blocks on fp32 MFMA (v_mfma_f32_32x32x2_f32; every conv of the U-Net is one of three gather
// relations u -> v = u*S - PAD + k):
//   mconv_kernel    out[u][a] (+)= sum_{k,c} W(a, c, k) in[v(u, k)][c] (* mask)   3x3 / 4x4 convs; with flipped taps
//                   and transposed weight strides also the stride-1 dgrad, and the transposed relation (the dgrad of
//                   the stride-2 Downsample conv, ConvTranspose2d itself) as a stride-1 conv over the dilated input
//   mconv1_kernel   the 1x1 convs and their dgrads
//   mwgrad_kernel   dW(a, b, k) = sum_u P[u][a] Q[v(u, k)][b]                      every weight gradient (split over
//                   positions, fixed-order reduction by mwgrad_reduce_kernel)
// plus GroupNorm/Mish (Block) backward, per-channel / per-utterance sums, the LinearAttention algebra, the small
// MLPs and the loss. Weights are read in the reference layouts (Conv2d [out][in][kh][kw], ConvTranspose2d
// [in][out][kh][kw]) through element strides. Deterministic: every reduction runs in a fixed order.
// Measured against torch eager on the same MI355X and the per-kernel breakdown: DESIGN.md §9.
#include <algorithm>
#include <cstdlib>

#include "bwd.h"
#include "common.h"

namespace gt {

// tanh(softplus(x)) = n / (n + 2) with n = e (e + 2), e = exp(x): one exponential per element (softplus threshold
// 20 as torch: x > 20 -> mish = x, mish' = 1)
GT_DEV float mish_grad(float x) {   // d/dx x tanh(softplus(x)) = th + x (1 - th^2) sigmoid(x)
  if (x > 20.f) return 1.f;
  const float e = __expf(x), n = e * (e + 2.f);
  const float th = n * __builtin_amdgcn_rcpf(n + 2.f), sg = e * __builtin_amdgcn_rcpf(1.f + e);   // v_rcp_f32
  return th + x * (1.f - th * th) * sg;
}
GT_DEV float mish_f(float x) {
  if (x > 20.f) return x;
  const float e = __expf(x), n = e * (e + 2.f);
  return x * (n * __builtin_amdgcn_rcpf(n + 2.f));
}

GT_DEV void split_range(long n, int S, int s, long* lo, long* hi) {
  const long per = (n + S - 1) / S;
  *lo = (long)s * per;
  *hi = *lo + per < n ? *lo + per : n;
}

// ---------------------------------------------------------------- mconv: the gconv relation on fp32 MFMA
// Implicit GEMM on v_mfma_f32_32x32x2_f32 (exact fp32 fma chains): M = 64 output positions of one row, N = 64 output
// channels, K = input channels x taps in chunks of MC_KC channels staged in LDS (input patch [row][col][c], weights
// [c][tap][a]); wave w owns the 32 x 32 block (positions (w & 1) * 32, channels (w >> 1) * 32).
// Tile: RH output rows x TW frames (RH TW <= 256 positions, flattened q = row TW + col) x 64 output channels; wave w
// owns positions q in [64 w, 64 w + 64) (2 x 2 blocks of 32 x 32 with the channel halves). The input patch
// ((RH - 1) SE + KS rows x (TW - 1) SE + KS columns) and the weight chunk are staged once per 8-channel chunk and
// shared by the whole tile; the next chunk's global loads are in flight during the current chunk's MFMAs. The tile
// shape is picked per launch to fit the level's mel rows x frames (4 x 64, 8 x 32, 5 x 48: level 1 / 2 frame
// counts like 86 / 43 waste 12-19 % instead of 49 % on 64-frame tiles).
template <int KS, int SE, int RH, int TW>
__global__ __launch_bounds__(256) void mconv_kernel(GConvParams p) {
  constexpr int MC_KC = 8, NCL = 32;   // input channels per staged chunk, staging column lanes per pass
  constexpr int KK = KS * KS, PC = (TW - 1) * SE + KS, PR = (RH - 1) * SE + KS, NCOL = (PC + NCL - 1) / NCL;
  constexpr int NW = 64 * MC_KC * KK, NWJ = (NW + 255) / 256;
  __shared__ float s_in[PR][PC][MC_KC + 1];
  __shared__ float s_w[MC_KC][KK][65];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int n_tt = (p.To + TW - 1) / TW, n_fr = (p.Fo + RH - 1) / RH;
  int bid = blockIdx.x;
  const int tt = bid % n_tt; bid /= n_tt;
  const int fo0 = (bid % n_fr) * RH;
  const int b = bid / n_fr;
  const int to0 = tt * TW, a0 = blockIdx.y * 64;
  // transposed relation (ConvTranspose2d, strided-conv dgrad): a stride-1 conv over the S-dilated input with the
  // taps flipped and padding KS - 1 - PAD
  const bool dil = p.transposed != 0;
  const int pad = dil ? KS - 1 - p.PAD : p.PAD;
  const bool flip = dil ? !p.flip : p.flip != 0;
  const bool a_fast = p.wsa < p.wsc;   // stage weights along their contiguous axis
  const int ic = tid % MC_KC, iq = tid / MC_KC;   // input staging: channel, column lane (NCL columns per pass)
  float rin[PR][NCOL], rw[NWJ], rm[NCOL];
  auto load = [&](int c0) {   // next chunk into registers (in flight during the MFMAs of the current one)
    const int ci = c0 + ic;
#pragma unroll
    for (int row = 0; row < PR; ++row) {
      const int fd = fo0 * SE - pad + row;
#pragma unroll
      for (int q = 0; q < NCOL; ++q) {
        const int col = iq + NCL * q;
        const int td = to0 * SE - pad + col;
        float v = 0.f;
        bool ok = col < PC && fd >= 0 && td >= 0 && ci < p.Cin;
        int fi = fd, ti = td;
        if (dil) { ok = ok && fd % p.S == 0 && td % p.S == 0; fi = fd / p.S; ti = td / p.S; }
        if (ok && fi < p.Fi && ti < p.Ti) v = p.in[(((long)b * p.Fi + fi) * p.Ti + ti) * p.Cin + ci];
        rin[row][q] = v;
        if (row == 0) {   // the mask depends on the column only; multiplied in when staged
          const int tc = dil ? td / p.S : td;
          rm[q] = (p.mask && tc >= 0 && tc < p.Ti) ? mask_at(p.mask, p.T0, b, tc, p.lvl_in) : 1.f;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NWJ; ++j) {
      const int i = tid + 256 * j;
      float v = 0.f;
      if (i < NW) {
        const int k = i % KK, rest = i / KK;
        const int a = a_fast ? rest % 64 : rest / MC_KC, c = a_fast ? rest / 64 : rest % MC_KC;
        const int kk = flip ? KK - 1 - k : k;
        if (a0 + a < p.Cout && c0 + c < p.Cin) v = p.w[(long)(a0 + a) * p.wsa + (long)(c0 + c) * p.wsc + kk];
      }
      rw[j] = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int row = 0; row < PR; ++row)
#pragma unroll
      for (int q = 0; q < NCOL; ++q)
        if (iq + NCL * q < PC) s_in[row][iq + NCL * q][ic] = rin[row][q] * rm[q];
#pragma unroll
    for (int j = 0; j < NWJ; ++j) {
      const int i = tid + 256 * j;
      if (i < NW) {
        const int k = i % KK, rest = i / KK;
        const int a = a_fast ? rest % 64 : rest / MC_KC, c = a_fast ? rest / 64 : rest % MC_KC;
        s_w[c][k][a] = rw[j];
      }
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[x][y][j] = 0.f;
  // this lane's A-operand positions (one per 32-position block)
  int prow[2], pcol[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int q = 64 * wv + 32 * x + r;
    prow[x] = q / TW < RH ? (q / TW) * SE : 0;   // positions past RH rows read row 0; their outputs are dropped
    pcol[x] = (q % TW) * SE;
  }
  load(0);
  for (int c0 = 0; c0 < p.Cin; c0 += MC_KC) {
    __syncthreads();
    store();
    __syncthreads();
    if (c0 + MC_KC < p.Cin) load(c0 + MC_KC);
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      const int kh = k / KS, kw = k % KS;
#pragma unroll
      for (int cp = 0; cp < MC_KC / 2; ++cp) {
        const int c = 2 * cp + hh;
        const float x0 = s_in[prow[0] + kh][pcol[0] + kw][c], x1 = s_in[prow[1] + kh][pcol[1] + kw][c];
        const float w0 = s_w[c][k][r], w1 = s_w[c][k][32 + r];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, w0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, w1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, w0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, w1, acc[1][1], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int a = a0 + 32 * y + r;
    if (a >= p.Cout) continue;
    const float bias = p.bias ? p.bias[a] : 0.f;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int q = 64 * wv + 32 * x + acc_row(j, hh);
        const int fo = fo0 + q / TW, to = to0 + q % TW;
        if (q / TW >= RH || fo >= p.Fo || to >= p.To) continue;
        const float om = p.out_mask ? mask_at(p.out_mask, p.T0, b, to, p.lvl_out) : 1.f;
        const long o = (((long)b * p.Fo + fo) * p.To + to) * p.out_cs + p.out_c0 + a;
        const float v = (acc[x][y][j] + bias) * om;
        p.out[o] = p.accumulate ? p.out[o] + v : v;
      }
  }
}

// wpk[a][k][c] = W(a, c, flip ? KK - 1 - k : k): the weights of one gconv launch with the input channel contiguous,
// so mconv_pk_kernel stages a chunk of KC channels of every (a, k) row as float4 runs
__global__ void gconv_wpack_kernel(const float* w, long wsa, long wsc, int KK, int flip, int Cout, int Cin, float* wpk) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)Cout * KK * Cin) return;
  const int c = (int)(i % Cin);
  const long rk = i / Cin;
  const int k = (int)(rk % KK), a = (int)(rk / KK);
  wpk[i] = w[(long)a * wsa + (long)c * wsc + (flip ? KK - 1 - k : k)];
}

// Many repacks in one launch (the training step's ~95 conv launches): descriptors in the kernel arguments, a
// workgroup finds its descriptor by the running element counts
constexpr int kPackBatch = 32;
struct PackBatch {
  GconvPack d[kPackBatch];
  long start[kPackBatch + 1];
  int n;
};
__global__ void gconv_wpack_batch_kernel(PackBatch pb) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= pb.start[pb.n]) return;
  int j = 0;
  while (j + 1 < pb.n && pb.start[j + 1] <= i) ++j;
  const GconvPack& d = pb.d[j];
  const long e = i - pb.start[j];
  const int c = (int)(e % d.Cin);
  const long rk = e / d.Cin;
  const int k = (int)(rk % d.KK), a = (int)(rk / d.KK);
  d.dst[e] = d.w[(long)a * d.wsa + (long)c * d.wsc + (d.flip ? d.KK - 1 - k : k)];
}

hipError_t launch_gconv_wpack_batch(const GconvPack* packs, int n, hipStream_t s) {
  for (int b0 = 0; b0 < n; b0 += kPackBatch) {
    PackBatch pb{};
    pb.n = std::min(kPackBatch, n - b0);
    pb.start[0] = 0;
    for (int j = 0; j < pb.n; ++j) {
      pb.d[j] = packs[b0 + j];
      pb.start[j + 1] = pb.start[j] + (long)pb.d[j].Cout * pb.d[j].KK * pb.d[j].Cin;
    }
    hipLaunchKernelGGL(gconv_wpack_batch_kernel, dim3((unsigned)((pb.start[pb.n] + 255) / 256)), dim3(256), 0, s, pb);
  }
  return hipGetLastError();
}

// The stride-1 relations (3x3 convs and their dgrads; with the S = 2 dilated input, the Downsample dgrad and
// ConvTranspose2d) with packed weights: same tile and wave ownership as mconv_kernel (RH x TW positions x 64 output
// channels, each wave 64 positions x 64 channels as 2 x 2 blocks of 32 x 32), but KC-channel chunks staged as float4
// (input [row][col][c] and weights [a][k][c], LDS rows of KC + 4 floats), the next chunk fetched into registers
// during the MFMAs (mask applied when the registers are written to LDS), and operands read as float4: channels
// 8g + 4h .. + 3 for lane half h feed four v_mfma_f32_32x32x2_f32 (element e = K index h of channel 8g + 4h + e on
// both operands), so one read of each of the four operands feeds 16 MFMAs.
// NY = 32-channel blocks per wave (tile of 32 NY output channels): NY = 1 doubles the workgroups of the small
// levels (level 2 has 64 position tiles per batch of 16) and fits three workgroups per CU.
template <int KS, int RH, int TW, int KC, int NY>
__global__ __launch_bounds__(256, NY == 1 ? 3 : 2) void mconv_pk_kernel(GConvParams p) {
  constexpr int KK = KS * KS, PC = TW - 1 + KS, PR = RH - 1 + KS, LD = KC + 4, G4 = KC / 4;
  constexpr int G4S = G4 == 8 ? 3 : G4 == 4 ? 2 : 1;   // log2(G4)
  // output-channel row stride of the weights: an odd number of 16-byte groups, so the 16 lanes of a float4 read
  // (16 output channels) hit distinct bank groups (KS = 4, KC = 8: 16 x 12 floats would put all of them on one)
  constexpr int WAS = ((KK * LD / 4) & 1) ? KK * LD : KK * LD + 4;
  constexpr int CT = 32 * NY, NPOS = PR * PC, NIN = (NPOS * G4 + 255) / 256, NWT = (CT * KK * G4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float s_in[NPOS * LD];
  __shared__ __attribute__((aligned(16))) float s_w[CT * WAS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int n_tt = (p.To + TW - 1) / TW, n_fr = (p.Fo + RH - 1) / RH;
  int bid = blockIdx.x;
  const int tt = bid % n_tt; bid /= n_tt;
  const int fo0 = (bid % n_fr) * RH;
  const int b = bid / n_fr;
  const int to0 = tt * TW, a0 = blockIdx.y * CT;
  const bool dil = p.transposed != 0;   // the S = 2 dilated input: odd coordinates are zeros
  const int pad = dil ? KS - 1 - p.PAD : p.PAD;
  const int nw = CT * KK * G4, wrows = KK * (p.Cout - a0);
  float4 rin[NIN], rw[NWT];
  float rm[NIN];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int n = 0; n < NIN; ++n) {
      const int i = tid + 256 * n, rc = i >> G4S, g = i & (G4 - 1);
      const int row = rc / PC, col = rc - row * PC;
      int fi = fo0 - pad + row, ti = to0 - pad + col;
      bool ok = rc < NPOS && fi >= 0 && ti >= 0 && c0 + 4 * g < p.Cin;
      if (dil) { ok = ok && !(fi & 1) && !(ti & 1); fi >>= 1; ti >>= 1; }
      rin[n] = make_float4(0.f, 0.f, 0.f, 0.f);
      rm[n] = 1.f;
      if (ok && fi < p.Fi && ti < p.Ti) {
        rin[n] = *reinterpret_cast<const float4*>(p.in + (((long)b * p.Fi + fi) * p.Ti + ti) * p.Cin + c0 + 4 * g);
        if (p.mask) rm[n] = mask_at(p.mask, p.T0, b, ti, p.lvl_in);
      }
    }
#pragma unroll
    for (int n = 0; n < NWT; ++n) {
      const int i = tid + 256 * n, ok = i >> G4S, g = i & (G4 - 1);
      rw[n] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < nw && ok < wrows && c0 + 4 * g < p.Cin)
        rw[n] = *reinterpret_cast<const float4*>(p.wpk + ((long)a0 * KK + ok) * p.Cin + c0 + 4 * g);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int n = 0; n < NIN; ++n) {
      const int i = tid + 256 * n, rc = i >> G4S, g = i & (G4 - 1);
      if (rc < NPOS) {
        float4 v = rin[n];
        v.x *= rm[n]; v.y *= rm[n]; v.z *= rm[n]; v.w *= rm[n];
        *reinterpret_cast<float4*>(s_in + rc * LD + 4 * g) = v;
      }
    }
#pragma unroll
    for (int n = 0; n < NWT; ++n) {
      const int i = tid + 256 * n;
      if (i < nw) {
        const int ak = i >> G4S, a = ak / KK;
        *reinterpret_cast<float4*>(s_w + a * WAS + (ak - a * KK) * LD + 4 * (i & (G4 - 1))) = rw[n];
      }
    }
  };
  f32x16 acc[2][NY];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < NY; ++y)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[x][y][j] = 0.f;
  const float* pa[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int q = 64 * wv + 32 * x + r;
    const int prow = q / TW < RH ? q / TW : 0;   // positions past RH rows read row 0; their outputs are dropped
    pa[x] = s_in + (prow * PC + q % TW) * LD + 4 * hh;
  }
  const float* pw = s_w + r * WAS + 4 * hh;   // output channel r; + 32 WAS for the second block
  fetch(0);
  store();
  __syncthreads();
  for (int c0 = 0; c0 < p.Cin; c0 += KC) {
    const bool more = c0 + KC < p.Cin;
    if (more) fetch(c0 + KC);
    // (tap, 8-channel group) steps, software-pipelined: the operands of step s + 1 are read before the 16 MFMAs of
    // step s are issued
    constexpr int NST = KK * (KC / 8);
    auto rd = [&](int st, float4* o) {
      const int k = st / (KC / 8), g = st % (KC / 8);
      const int off = ((k / KS) * PC + k % KS) * LD + 8 * g;
      o[0] = *reinterpret_cast<const float4*>(pa[0] + off);
      o[1] = *reinterpret_cast<const float4*>(pa[1] + off);
      o[2] = *reinterpret_cast<const float4*>(pw + k * LD + 8 * g);
      if (NY == 2) o[3] = *reinterpret_cast<const float4*>(pw + 32 * WAS + k * LD + 8 * g);
    };
    float4 opd[2][4];
    rd(0, opd[0]);
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      if (st + 1 < NST) rd(st + 1, opd[(st + 1) & 1]);
      const float4 x0 = opd[st & 1][0], x1 = opd[st & 1][1], w0 = opd[st & 1][2], w1 = opd[st & 1][3];
#define MC4_STEP(E)                                                                                    \
  acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.E, w0.E, acc[0][0], 0, 0, 0);                  \
  if (NY == 2) acc[0][NY - 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.E, w1.E, acc[0][NY - 1], 0, 0, 0); \
  acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.E, w0.E, acc[1][0], 0, 0, 0);                  \
  if (NY == 2) acc[1][NY - 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.E, w1.E, acc[1][NY - 1], 0, 0, 0);
      MC4_STEP(x) MC4_STEP(y) MC4_STEP(z) MC4_STEP(w)
#undef MC4_STEP
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
#pragma unroll
  for (int y = 0; y < NY; ++y) {
    const int a = a0 + 32 * y + r;
    if (a >= p.Cout) continue;
    const float bias = p.bias ? p.bias[a] : 0.f;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int q = 64 * wv + 32 * x + acc_row(j, hh);
        const int fo = fo0 + q / TW, to = to0 + q % TW;
        if (q / TW >= RH || fo >= p.Fo || to >= p.To) continue;
        const float om = p.out_mask ? mask_at(p.out_mask, p.T0, b, to, p.lvl_out) : 1.f;
        const long o = (((long)b * p.Fo + fo) * p.To + to) * p.out_cs + p.out_c0 + a;
        const float v = (acc[x][y][j] + bias) * om;
        p.out[o] = p.accumulate ? p.out[o] + v : v;
      }
  }
}

// 1x1 convs (qkv / to_out / res_conv / final_conv and their dgrads): one row of 64 positions x 64 channels per
// workgroup, 32-channel chunks (128-byte input rows), waves 2 x 2 over (positions, channels)
__global__ __launch_bounds__(256) void mconv1_kernel(GConvParams p) {
  constexpr int KC = 32;
  __shared__ float s_in[64][KC + 1];
  __shared__ float s_w[KC][65];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int n_tt = (p.To + 63) / 64;
  int bid = blockIdx.x;
  const int tt = bid % n_tt; bid /= n_tt;
  const int fo = bid % p.Fo;
  const int b = bid / p.Fo;
  const int to0 = tt * 64, a0 = blockIdx.y * 64;
  const int pb = (wv & 1) * 32, cb = (wv >> 1) * 32;
  const bool a_fast = p.wsa < p.wsc;
  float rin[8], rw[8], rm[8];
  auto load = [&](int c0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {   // input: 32 channels x 64 positions (mask multiplied in when staged)
      const int i = tid + 256 * j, c = i & 31, pp = i >> 5;
      const int ti = to0 + pp, ci = c0 + c;
      float v = 0.f, m = 1.f;
      if (ti < p.Ti && ci < p.Cin) {
        v = p.in[(((long)b * p.Fi + fo) * p.Ti + ti) * p.Cin + ci];
        if (p.mask) m = mask_at(p.mask, p.T0, b, ti, p.lvl_in);
      }
      rin[j] = v;
      rm[j] = m;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {   // weights: 64 a x 32 c
      const int i = tid + 256 * j;
      const int a = a_fast ? (i & 63) : (i >> 5), c = a_fast ? (i >> 6) : (i & 31);
      rw[j] = (a0 + a < p.Cout && c0 + c < p.Cin) ? p.w[(long)(a0 + a) * p.wsa + (long)(c0 + c) * p.wsc] : 0.f;
    }
  };
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  load(0);
  for (int c0 = 0; c0 < p.Cin; c0 += KC) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = tid + 256 * j;
      s_in[i >> 5][i & 31] = rin[j] * rm[j];
      const int a = a_fast ? (i & 63) : (i >> 5), c = a_fast ? (i >> 6) : (i & 31);
      s_w[c][a] = rw[j];
    }
    __syncthreads();
    if (c0 + KC < p.Cin) load(c0 + KC);
#pragma unroll
    for (int cp = 0; cp < KC / 2; ++cp)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(s_in[pb + r][2 * cp + hh], s_w[2 * cp + hh][cb + r], acc, 0, 0, 0);
  }
  const int a = a0 + cb + r;
  if (a >= p.Cout) return;
  const float bias = p.bias ? p.bias[a] : 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int to = to0 + pb + acc_row(j, hh);
    if (to >= p.To) continue;
    const float om = p.out_mask ? mask_at(p.out_mask, p.T0, b, to, p.lvl_out) : 1.f;
    const long o = (((long)b * p.Fo + fo) * p.To + to) * p.out_cs + p.out_c0 + a;
    const float v = (acc[j] + bias) * om;
    p.out[o] = p.accumulate ? p.out[o] + v : v;
  }
}

// ---------------------------------------------------------------- mwgrad: weight gradients on fp32 MFMA
// dW(a, b, k) = sum_u P[u][a] Q[v(u, k)][b] as a GEMM with M = 64 a, N = 64 b, K = positions: each workgroup walks
// its share of 32-position row segments, staging P [32][64] and the KS-row patch of Q the segment's taps touch (the
// next segment's loads in flight during the current MFMAs); wave w owns the 32 x 32 (a, b) block
// ((w & 1) * 32, (w >> 1) * 32) for the KG taps of its group. LDS row strides put the two half-waves' rows 32 banks
// apart. part[split][k][a][b] -> mwgrad_reduce_kernel (splits in order).
template <int KS, int S, int SEG>
__global__ __launch_bounds__(256) void mwgrad_kernel(WGradParams p, int splits, float* part) {
  constexpr int KG = KS == 4 ? 8 : KS * KS, NR = KG / KS;                    // taps / patch rows of a group
  constexpr int NCOL = (SEG - 1) * S + KS, QS = S == 1 ? 96 : 80, PS = 96;   // patch columns, LDS row strides
  constexpr int NQ = (NCOL + 3) / 4, NPJ = SEG / 4;                          // staging per lane: Q columns, P rows
  __shared__ float s_p[SEG * PS];
  __shared__ float s_q[NR * NCOL * QS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int sc = tid & 63, sl = tid >> 6;   // staging: channel, row lane
  const int a0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
  const int split = blockIdx.z % splits, k0 = (blockIdx.z / splits) * KG;
  const int kh0 = k0 / KS;
  const int n_tt = (p.Tu + SEG - 1) / SEG;
  const long nseg = (long)p.B * p.Fu * n_tt;
  const long per = (nseg + splits - 1) / splits;
  const long s_lo = split * per, s_hi = s_lo + per < nseg ? s_lo + per : nseg;
  const int ab = (wv & 1) * 32, bb = (wv >> 1) * 32;
  f32x16 acc[KG];
#pragma unroll
  for (int g = 0; g < KG; ++g)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[g][j] = 0.f;
  float rp[NPJ], rq[NR][NQ], pm[NPJ], qm[NQ];   // masks kept apart: multiplied in when staged, so the loads stay
                                                //   in flight during the MFMAs
  auto load = [&](long sg) {
    const int tt = (int)(sg % n_tt);
    const int fu = (int)((sg / n_tt) % p.Fu);
    const int b = (int)(sg / ((long)n_tt * p.Fu));
    const int t0 = tt * SEG;
#pragma unroll
    for (int j = 0; j < NPJ; ++j) {
      const int u = sl + 4 * j;
      float v = 0.f, m = 1.f;
      if (t0 + u < p.Tu && a0 + sc < p.A) {
        v = p.P[(((long)b * p.Fu + fu) * p.Tu + t0 + u) * p.A + a0 + sc];
        if (p.pmask) m = mask_at(p.pmask, p.T0, b, t0 + u, p.lvl_p);
      }
      rp[j] = v;
      pm[j] = m;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int col = sl + 4 * q, tv = t0 * S - p.PAD + col;
      qm[q] = (p.qmask && col < NCOL && tv >= 0 && tv < p.Tv) ? mask_at(p.qmask, p.T0, b, tv, p.lvl_q) : 1.f;
    }
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int fv = fu * S - p.PAD + kh0 + rr;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int col = sl + 4 * q, tv = t0 * S - p.PAD + col;
        float v = 0.f;
        if (col < NCOL && fv >= 0 && fv < p.Fv && tv >= 0 && tv < p.Tv && b0 + sc < p.Bc)
          v = p.Q[(((long)b * p.Fv + fv) * p.Tv + tv) * p.Bc + b0 + sc];
        rq[rr][q] = v;
      }
    }
  };
  if (s_lo < s_hi) load(s_lo);
  for (long sg = s_lo; sg < s_hi; ++sg) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NPJ; ++j) s_p[(sl + 4 * j) * PS + sc] = rp[j] * pm[j];
#pragma unroll
    for (int rr = 0; rr < NR; ++rr)
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        if (sl + 4 * q < NCOL) s_q[(rr * NCOL + sl + 4 * q) * QS + sc] = rq[rr][q] * qm[q];
    __syncthreads();
    if (sg + 1 < s_hi) load(sg + 1);
#pragma unroll 2
    for (int up = 0; up < SEG / 2; ++up) {   // one P read feeds the KG taps: independent accumulator chains
      const int u = 2 * up + hh;
      const float pa = s_p[u * PS + ab + r];
#pragma unroll
      for (int g = 0; g < KG; ++g) {
        const int kh = g / KS, kw = g % KS;
        acc[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(pa, s_q[(kh * NCOL + u * S + kw) * QS + bb + r], acc[g], 0, 0, 0);
      }
    }
  }
  const int bc = b0 + bb + r;
  constexpr int KKt = KS * KS;
#pragma unroll
  for (int g = 0; g < KG; ++g) {
    const int k = k0 + g;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int a = a0 + ab + acc_row(j, hh);
      if (a < p.A && bc < p.Bc) part[(((long)split * KKt + k) * p.A + a) * p.Bc + bc] = acc[g][j];
    }
  }
}

__global__ void mwgrad_reduce_kernel(const float* part, int splits, int A, int Bc, int KK, long sa, long sb, float* dw,
                                     int accumulate) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long n = (long)KK * A * Bc;
  if (i >= n) return;
  float s = 0.f;
#pragma unroll 8
  for (int q = 0; q < splits; ++q) s += part[(long)q * n + i];
  const int bc = (int)(i % Bc), a = (int)((i / Bc) % A), k = (int)(i / ((long)A * Bc));
  float* d = dw + a * sa + bc * sb + k;
  *d = accumulate ? *d + s : s;
}

// 3x3 stride-1 weight gradient with the positions contiguous in LDS: P^T [a][u] and the 3-row Q^T patch [b][kh][col]
// staged from float4 loads along the channels (transposed on the LDS write; masks multiplied in there, so the next
// segment's loads stay in flight during the MFMAs). Per 8 positions u0: one float4 of P^T (positions u0 + 4h .. + 3)
// feeds the nine taps; tap (kh, kw) reads Q^T at column u0 + 4h + kw (16-, 4- or 8-byte aligned for kw = 0, 1, 2),
// four v_mfma_f32_32x32x2_f32 each (element e = K index h of position u0 + 4h + e on both operands). Same tile, split
// and partial layout as mwgrad_kernel; LDS row strides of an odd number of 16-byte groups.
template <int SEG>
__global__ __launch_bounds__(256, 2) void mwgrad_pk_kernel(WGradParams p, int splits, float* part) {
  constexpr int NCOL = SEG + 2, PST = SEG + 4, QW = SEG + 4, QBS = 3 * QW;
  static_assert(((PST / 4) & 1) && ((QBS / 4) & 1) && SEG % 16 == 0, "LDS strides");
  constexpr int NPF = SEG * 16 / 256, NQF = (3 * NCOL * 16 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float s_p[64 * PST];
  __shared__ __attribute__((aligned(16))) float s_q[64 * QBS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int a0 = blockIdx.x * 64, b0 = blockIdx.y * 64, split = blockIdx.z;
  const int n_tt = (p.Tu + SEG - 1) / SEG, nseg = p.B * p.Fu * n_tt;
  const int per = (nseg + splits - 1) / splits;
  const int s_lo = split * per, s_hi = s_lo + per < nseg ? s_lo + per : nseg;
  const int ab = (wv & 1) * 32, bb = (wv >> 1) * 32;
  f32x16 acc[9];
#pragma unroll
  for (int g = 0; g < 9; ++g)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[g][j] = 0.f;
  float4 rp[NPF], rq[NQF];
  float pm[NPF], qm[NQF];
  auto fetch = [&](int sg) {
    const int tt = sg % n_tt, fu = (sg / n_tt) % p.Fu, b = sg / (n_tt * p.Fu), t0 = tt * SEG;
#pragma unroll
    for (int n = 0; n < NPF; ++n) {
      const int i = tid + 256 * n, u = i >> 4, a4 = i & 15, t = t0 + u;
      const bool ok = t < p.Tu && a0 + 4 * a4 < p.A;
      rp[n] = ok ? *reinterpret_cast<const float4*>(p.P + (((long)b * p.Fu + fu) * p.Tu + t) * p.A + a0 + 4 * a4)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
      pm[n] = (ok && p.pmask) ? mask_at(p.pmask, p.T0, b, t, p.lvl_p) : 1.f;
    }
#pragma unroll
    for (int n = 0; n < NQF; ++n) {
      const int i = tid + 256 * n, rc = i >> 4, b4 = i & 15, row = rc / NCOL, col = rc - row * NCOL;
      const int fv = fu - p.PAD + row, tv = t0 - p.PAD + col;
      const bool ok = rc < 3 * NCOL && fv >= 0 && fv < p.Fv && tv >= 0 && tv < p.Tv && b0 + 4 * b4 < p.Bc;
      rq[n] = ok ? *reinterpret_cast<const float4*>(p.Q + (((long)b * p.Fv + fv) * p.Tv + tv) * p.Bc + b0 + 4 * b4)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
      qm[n] = (ok && p.qmask) ? mask_at(p.qmask, p.T0, b, tv, p.lvl_q) : 1.f;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int n = 0; n < NPF; ++n) {
      const int i = tid + 256 * n, u = i >> 4, a4 = i & 15;
      float* d = s_p + 4 * a4 * PST + u;
      d[0] = rp[n].x * pm[n]; d[PST] = rp[n].y * pm[n]; d[2 * PST] = rp[n].z * pm[n]; d[3 * PST] = rp[n].w * pm[n];
    }
#pragma unroll
    for (int n = 0; n < NQF; ++n) {
      const int i = tid + 256 * n, rc = i >> 4, b4 = i & 15, row = rc / NCOL, col = rc - row * NCOL;
      if (rc < 3 * NCOL) {
        float* d = s_q + 4 * b4 * QBS + row * QW + col;
        d[0] = rq[n].x * qm[n]; d[QBS] = rq[n].y * qm[n]; d[2 * QBS] = rq[n].z * qm[n]; d[3 * QBS] = rq[n].w * qm[n];
      }
    }
  };
  const float* pp = s_p + (ab + r) * PST + 4 * hh;
  const float* pq = s_q + (bb + r) * QBS + 4 * hh;
  if (s_lo < s_hi) fetch(s_lo);
  for (int sg = s_lo; sg < s_hi; ++sg) {
    __syncthreads();
    store();
    __syncthreads();
    if (sg + 1 < s_hi) fetch(sg + 1);
#pragma unroll
    for (int u0 = 0; u0 < SEG; u0 += 8) {
      const float4 a = *reinterpret_cast<const float4*>(pp + u0);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const float* q = pq + kh * QW + u0;
        const float4 q0 = *reinterpret_cast<const float4*>(q);
        const float4 q1 = make_float4(q[1], q[2], q[3], q[4]);
        const float2 q2a = *reinterpret_cast<const float2*>(q + 2), q2b = *reinterpret_cast<const float2*>(q + 4);
        const float4 q2 = make_float4(q2a.x, q2a.y, q2b.x, q2b.y);
#define WG3_STEP(E)                                                                          \
  acc[3 * kh] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.E, q0.E, acc[3 * kh], 0, 0, 0);         \
  acc[3 * kh + 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.E, q1.E, acc[3 * kh + 1], 0, 0, 0); \
  acc[3 * kh + 2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.E, q2.E, acc[3 * kh + 2], 0, 0, 0);
        WG3_STEP(x) WG3_STEP(y) WG3_STEP(z) WG3_STEP(w)   // three independent accumulator chains interleaved
#undef WG3_STEP
      }
    }
  }
  const int bc = b0 + bb + r;
#pragma unroll
  for (int g = 0; g < 9; ++g)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int a = a0 + ab + acc_row(j, hh);
      if (a < p.A && bc < p.Bc) part[(((long)split * 9 + g) * p.A + a) * p.Bc + bc] = acc[g][j];
    }
}

// 1x1 weight gradient dW(a, b) = sum_u P[u][a] Q[u][b] with the positions flattened over (utterance, row, frame)
// (a 1x1 conv has no spatial neighbourhood): 64-position segments, P^T [a][u] and Q^T [b][u] in LDS (transposed at
// the LDS write from float4 loads along the channels, masks applied there, next segment in flight during the MFMAs);
// waves 2 x 2 over (a, b), one float4 of each operand feeds four v_mfma_f32_32x32x2_f32. Partials as mwgrad_kernel.
constexpr int kW1Seg = 64;
__global__ __launch_bounds__(256) void mwgrad1_pk_kernel(WGradParams p, int splits, float* part) {
  constexpr int SEG = kW1Seg, ST = SEG + 4, NF = SEG * 16 / 256;
  static_assert((ST / 4) & 1, "LDS stride");
  __shared__ __attribute__((aligned(16))) float s_p[64 * ST];
  __shared__ __attribute__((aligned(16))) float s_q[64 * ST];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int a0 = blockIdx.x * 64, b0 = blockIdx.y * 64, split = blockIdx.z;
  const int FT = p.Fu * p.Tu;
  const long npos = (long)p.B * FT;
  const long nseg = (npos + SEG - 1) / SEG;
  const long per = (nseg + splits - 1) / splits;
  const long s_lo = split * per, s_hi = s_lo + per < nseg ? s_lo + per : nseg;
  const int ab = (wv & 1) * 32, bb = (wv >> 1) * 32;
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  float4 rp[NF], rq[NF];
  float pm[NF], qm[NF];
  auto fetch = [&](long sg) {
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      const int i = tid + 256 * n, c4 = i & 15;
      const long u = sg * SEG + (i >> 4);
      const bool in = u < npos;
      const int b = in ? (int)(u / FT) : 0, t = in ? (int)(u % p.Tu) : 0;
      const bool okp = in && a0 + 4 * c4 < p.A, okq = in && b0 + 4 * c4 < p.Bc;
      rp[n] = okp ? *reinterpret_cast<const float4*>(p.P + u * p.A + a0 + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      rq[n] = okq ? *reinterpret_cast<const float4*>(p.Q + u * p.Bc + b0 + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      pm[n] = (in && p.pmask) ? mask_at(p.pmask, p.T0, b, t, p.lvl_p) : 1.f;
      qm[n] = (in && p.qmask) ? mask_at(p.qmask, p.T0, b, t, p.lvl_q) : 1.f;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      const int i = tid + 256 * n, u = i >> 4, c4 = i & 15;
      float* dp = s_p + 4 * c4 * ST + u;
      float* dq = s_q + 4 * c4 * ST + u;
      dp[0] = rp[n].x * pm[n]; dp[ST] = rp[n].y * pm[n]; dp[2 * ST] = rp[n].z * pm[n]; dp[3 * ST] = rp[n].w * pm[n];
      dq[0] = rq[n].x * qm[n]; dq[ST] = rq[n].y * qm[n]; dq[2 * ST] = rq[n].z * qm[n]; dq[3 * ST] = rq[n].w * qm[n];
    }
  };
  const float* pp = s_p + (ab + r) * ST + 4 * hh;
  const float* pq = s_q + (bb + r) * ST + 4 * hh;
  if (s_lo < s_hi) fetch(s_lo);
  for (long sg = s_lo; sg < s_hi; ++sg) {
    __syncthreads();
    store();
    __syncthreads();
    if (sg + 1 < s_hi) fetch(sg + 1);
#pragma unroll
    for (int u0 = 0; u0 < SEG; u0 += 8) {
      const float4 a = *reinterpret_cast<const float4*>(pp + u0);
      const float4 q = *reinterpret_cast<const float4*>(pq + u0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, q.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, q.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, q.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, q.w, acc, 0, 0, 0);
    }
  }
  const int bc = b0 + bb + r;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int a = a0 + ab + acc_row(j, hh);
    if (a < p.A && bc < p.Bc) part[((long)split * p.A + a) * p.Bc + bc] = acc[j];
  }
}

// 48-position segments where they cut the padded frames (a level-2 row of 43 frames: 48 instead of 64)
static int mwgrad_seg(const WGradParams& p) {
  return (p.KS == 3 && p.S == 1 && (p.Tu + 47) / 48 * 48 < (p.Tu + 31) / 32 * 32) ? 48 : 32;
}

int mwgrad_splits(const WGradParams& p) {
  const int groups = p.KS == 4 ? 2 : 1;
  const long tiles = (long)((p.A + 63) / 64) * ((p.Bc + 63) / 64) * groups;
  const int seg = mwgrad_seg(p);
  const long nseg = (long)p.B * p.Fu * ((p.Tu + seg - 1) / seg);
  long s = std::max<long>(1, 512 / tiles);
  s = std::min<long>(s, nseg);
  s = std::min<long>(s, kWPartCap / ((long)p.KS * p.KS * p.A * p.Bc));
  return (int)std::max<long>(1, s);
}

hipError_t launch_mwgrad(const WGradParams& p, float* part, float* dw, long sa, long sb, int accumulate, hipStream_t strm) {
  const int cfg = p.KS * 10 + p.S;
  if (!(cfg == 11 || cfg == 31 || cfg == 32 || cfg == 42)) return hipErrorInvalidValue;
  const int splits = mwgrad_splits(p);
  const int groups = p.KS == 4 ? 2 : 1;
  const dim3 grid((p.A + 63) / 64, (p.Bc + 63) / 64, splits * groups);
  const bool aligned = p.A % 4 == 0 && p.Bc % 4 == 0 && ((uintptr_t)p.P & 15) == 0 && ((uintptr_t)p.Q & 15) == 0;
  const bool pk = cfg == 31 && aligned;
  if (cfg == 11 && aligned && p.PAD == 0 && p.Fu == p.Fv && p.Tu == p.Tv) {   // 1x1: flattened positions
    const long tiles = (long)((p.A + 63) / 64) * ((p.Bc + 63) / 64);
    const long nseg = ((long)p.B * p.Fu * p.Tu + kW1Seg - 1) / kW1Seg;
    long sp = std::max<long>(1, 1024 / tiles);
    sp = std::min<long>(sp, nseg);
    sp = std::min<long>(sp, kWPartCap / ((long)p.A * p.Bc));
    const int s1 = (int)std::max<long>(1, sp);
    hipLaunchKernelGGL(mwgrad1_pk_kernel, dim3((p.A + 63) / 64, (p.Bc + 63) / 64, s1), dim3(256), 0, strm, p, s1, part);
    const long n = (long)p.A * p.Bc;
    hipLaunchKernelGGL(mwgrad_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, strm, part, s1, p.A,
                       p.Bc, 1, sa, sb, dw, accumulate);
    return hipGetLastError();
  }
  // (48-position segments for the 43-frame rows would need more registers than two waves per SIMD leave)
  if (pk) hipLaunchKernelGGL((mwgrad_pk_kernel<32>), grid, dim3(256), 0, strm, p, splits, part);
  else if (cfg == 11) hipLaunchKernelGGL((mwgrad_kernel<1, 1, 32>), grid, dim3(256), 0, strm, p, splits, part);
  else if (cfg == 31 && mwgrad_seg(p) == 48)
    hipLaunchKernelGGL((mwgrad_kernel<3, 1, 48>), grid, dim3(256), 0, strm, p, splits, part);
  else if (cfg == 31) hipLaunchKernelGGL((mwgrad_kernel<3, 1, 32>), grid, dim3(256), 0, strm, p, splits, part);
  else if (cfg == 32) hipLaunchKernelGGL((mwgrad_kernel<3, 2, 32>), grid, dim3(256), 0, strm, p, splits, part);
  else hipLaunchKernelGGL((mwgrad_kernel<4, 2, 32>), grid, dim3(256), 0, strm, p, splits, part);
  const long n = (long)p.KS * p.KS * p.A * p.Bc;
  hipLaunchKernelGGL(mwgrad_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, strm, part, splits, p.A,
                     p.Bc, p.KS * p.KS, sa, sb, dw, accumulate);
  return hipGetLastError();
}

// ---------------------------------------------------------------- per-utterance channel sums
// out[b][c] (+)= sum over the utterance's positions of x[b][pos][c] (optionally x * y), one workgroup per (b, 256
// channels); positions summed per thread in ascending order
__global__ __launch_bounds__(256) void bsum_kernel(const float* x, const float* y, int npos, int C, float* out,
                                                   int accumulate) {
  const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  const float* xb = x + (long)b * npos * C + c;
  const float* yb = y ? y + (long)b * npos * C + c : nullptr;
  float s = 0.f;
  for (int i = 0; i < npos; ++i) s += yb ? xb[(long)i * C] * yb[(long)i * C] : xb[(long)i * C];
  float* o = out + (long)b * C + c;
  *o = accumulate ? *o + s : s;
}

// out[c] (+)= sum_b in[b][c]
__global__ void colsum_kernel(const float* in, int B, int C, float* out, int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += in[(long)b * C + c];
  out[c] = accumulate ? out[c] + s : s;
}

// GroupNorm statistics in two levels: fp64 (sum, sum of squares) per (b, group, split), then the splits in order
__global__ __launch_bounds__(256) void gn_partial_kernel(const float* h, int npos, int C, double* part) {
  __shared__ double s[2][256];
  const int b = blockIdx.x, g = blockIdx.y, sp = blockIdx.z, S = gridDim.z, tid = threadIdx.x;
  const int cg = C / 8;
  long lo, hi;
  split_range((long)npos * cg, S, sp, &lo, &hi);
  const float* hb = h + (long)b * npos * C + g * cg;
  double s1 = 0.0, s2 = 0.0;
  for (long i = lo + tid; i < hi; i += 256) {
    const double v = hb[(i / cg) * C + i % cg];
    s1 += v; s2 += v * v;
  }
  s[0][tid] = s1; s[1][tid] = s2;
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, q = 0.0;
    for (int i = 0; i < 256; ++i) { a += s[0][i]; q += s[1][i]; }
    part[(((long)b * 8 + g) * S + sp) * 2] = a;
    part[(((long)b * 8 + g) * S + sp) * 2 + 1] = q;
  }
}
__global__ void gn_final_kernel(const double* part, int S, int nbg, double n, float* stats) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // b * 8 + g
  if (i >= nbg) return;
  double a = 0.0, q = 0.0;
  for (int sp = 0; sp < S; ++sp) { a += part[((long)i * S + sp) * 2]; q += part[((long)i * S + sp) * 2 + 1]; }
  const double mean = a / n;
  double var = q / n - mean * mean;
  var = var > 0.0 ? var : 0.0;
  stats[i * 2] = (float)mean;
  stats[i * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
}
int gn_splits(long npos) { return (int)std::max<long>(1, std::min<long>(32, npos / 512)); }
hipError_t launch_gn_stats_split(const float* h, int B, int npos, int C, double* part, float* stats, hipStream_t strm) {
  const int S = gn_splits(npos);
  hipLaunchKernelGGL(gn_partial_kernel, dim3(B, 8, S), dim3(256), 0, strm, h, npos, C, part);
  hipLaunchKernelGGL(gn_final_kernel, dim3((B * 8 + 255) / 256), dim3(256), 0, strm, part, S, B * 8,
                     (double)npos * (C / 8), stats);
  return hipGetLastError();
}

// ---------------------------------------------------------------- GroupNorm statistics of a forward tensor
// mean / rstd per (b, group) straight from the tensor (fp64 sums, fixed order): [B][8][2]
__global__ __launch_bounds__(256) void gn_stats_kernel(const float* h, int npos, int C, float* stats) {
  __shared__ double s[2][256];
  const int b = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
  const int cg = C / 8;
  const float* hb = h + (long)b * npos * C + g * cg;
  double s1 = 0.0, s2 = 0.0;
  for (long i = tid; i < (long)npos * cg; i += 256) {
    const double v = hb[(i / cg) * C + i % cg];
    s1 += v; s2 += v * v;
  }
  s[0][tid] = s1; s[1][tid] = s2;
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, q = 0.0;
    for (int i = 0; i < 256; ++i) { a += s[0][i]; q += s[1][i]; }
    const double n = (double)npos * cg, mean = a / n;
    double var = q / n - mean * mean;
    var = var > 0.0 ? var : 0.0;
    stats[(b * 8 + g) * 2] = (float)mean;
    stats[(b * 8 + g) * 2 + 1] = (float)(1.0 / sqrt(var + 1e-5));
  }
}

// ---------------------------------------------------------------- Block backward (Mish(GN(h)) * m)
// dn = dA * m * mish'(n), n = xhat * gamma + beta; per (b, group): S1 = sum dn gamma, S2 = sum dn gamma xhat;
// per (b, channel): dgamma = sum dn xhat, dbeta = sum dn. One workgroup per (b, group); fixed order.
__global__ __launch_bounds__(256) void block_bwd_reduce_kernel(BlockBwdParams p) {
  __shared__ double s[2][256];
  const int b = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
  const int cg = p.C / 8;
  const float mean = p.stats[(b * 8 + g) * 2], rstd = p.stats[(b * 8 + g) * 2 + 1];
  double s1 = 0.0, s2 = 0.0;
  for (long i = tid; i < (long)p.npos * cg; i += 256) {
    const long pos = i / cg;
    const int c = g * cg + (int)(i % cg);
    const long o = ((long)b * p.npos + pos) * p.C + c;
    const float xh = (p.h[o] - mean) * rstd;
    const float n = xh * p.gamma[c] + p.beta[c];
    const float m = mask_at(p.mask, p.T0, b, (int)(pos % p.T), p.lvl);
    const float dn = p.dA[o] * m * mish_grad(n);
    s1 += (double)(dn * p.gamma[c]);
    s2 += (double)(dn * p.gamma[c] * xh);
  }
  s[0][tid] = s1; s[1][tid] = s2;
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, q = 0.0;
    for (int i = 0; i < 256; ++i) { a += s[0][i]; q += s[1][i]; }
    p.gsum[(b * 8 + g) * 2] = (float)a;
    p.gsum[(b * 8 + g) * 2 + 1] = (float)q;
  }
  // per-channel dgamma / dbeta of this utterance: thread c' of the group's channels
  for (int cc = tid; cc < cg; cc += 256) {
    const int c = g * cg + cc;
    float dgm = 0.f, dbt = 0.f;
    for (long pos = 0; pos < p.npos; ++pos) {
      const long o = ((long)b * p.npos + pos) * p.C + c;
      const float xh = (p.h[o] - mean) * rstd;
      const float n = xh * p.gamma[c] + p.beta[c];
      const float m = mask_at(p.mask, p.T0, b, (int)(pos % p.T), p.lvl);
      const float dn = p.dA[o] * m * mish_grad(n);
      dgm += dn * xh;
      dbt += dn;
    }
    p.dgb[((long)b * p.C + c) * 2] = dgm;
    p.dgb[((long)b * p.C + c) * 2 + 1] = dbt;
  }
}

// dh = rstd (dn gamma - S1 / N - xhat S2 / N)
__global__ __launch_bounds__(256) void block_bwd_apply_kernel(BlockBwdParams p) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long n = (long)p.B * p.npos * p.C;
  if (i >= n) return;
  const int c = (int)(i % p.C);
  const long pos = (i / p.C) % p.npos;
  const int b = (int)(i / ((long)p.npos * p.C));
  const int g = c / (p.C / 8);
  const float mean = p.stats[(b * 8 + g) * 2], rstd = p.stats[(b * 8 + g) * 2 + 1];
  const float N = (float)((double)p.npos * (p.C / 8));
  const float xh = (p.h[i] - mean) * rstd;
  const float nn = xh * p.gamma[c] + p.beta[c];
  const float m = mask_at(p.mask, p.T0, b, (int)(pos % p.T), p.lvl);
  const float dn = p.dA[i] * m * mish_grad(nn);
  const float S1 = p.gsum[(b * 8 + g) * 2], S2 = p.gsum[(b * 8 + g) * 2 + 1];
  p.dh[i] = rstd * (dn * p.gamma[c] - S1 / N - xh * S2 / N);
}

// Block forward output from the saved pre-activation: a = Mish(GN(h)) * m (+ tb) * m2 (recompute for the tape)
__global__ __launch_bounds__(256) void block_fwd_kernel(BlockBwdParams p, const float* tb, float* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long n = (long)p.B * p.npos * p.C;
  if (i >= n) return;
  const int c = (int)(i % p.C);
  const long pos = (i / p.C) % p.npos;
  const int b = (int)(i / ((long)p.npos * p.C));
  const int g = c / (p.C / 8);
  const float mean = p.stats[(b * 8 + g) * 2], rstd = p.stats[(b * 8 + g) * 2 + 1];
  const float m = mask_at(p.mask, p.T0, b, (int)(pos % p.T), p.lvl);
  float v = mish_f((p.h[i] - mean) * rstd * p.gamma[c] + p.beta[c]) * m;
  if (tb) v = v + tb[(long)b * p.C + c];
  out[i] = v;
}

// ---------------------------------------------------------------- elementwise helpers on [B][F][T][C]
// y = alpha * x * (mask ? m : 1) (+ y if accumulate); channels [c0, c0 + C) of a tensor with cs channels
__global__ void ew_kernel(EwParams p) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long n = (long)p.B * p.F * p.T * p.C;
  if (i >= n) return;
  const int c = (int)(i % p.C);
  const long pos = i / p.C;
  const int t = (int)(pos % p.T);
  const int b = (int)(pos / ((long)p.F * p.T));
  const float alpha = p.alphap ? *p.alphap : p.alpha, alpha2 = p.alpha2p ? *p.alpha2p : p.alpha2;
  float v = alpha * p.x[pos * p.xcs + p.xc0 + c];
  if (p.mask) v *= mask_at(p.mask, p.T0, b, t, p.lvl);
  if (p.x2) v += alpha2 * p.x2[pos * p.C + c];
  float* o = p.y + pos * p.ycs + p.yc0 + c;
  *o = p.accumulate ? *o + v : v;
}

// ---------------------------------------------------------------- LinearAttention pieces (4 heads x 32)
// softmax statistics of k over the positions: per (b, row) max and sum of exp; k rows at channel offset 128 of qkv
__global__ __launch_bounds__(256) void attn_kstats_kernel(const float* qkv, int npos, float* st) {
  __shared__ float s_m[256];
  __shared__ double s_l[256];
  const int b = blockIdx.x, r = blockIdx.y, tid = threadIdx.x;
  const float* kb = qkv + (long)b * npos * 384 + 128 + r;
  float m = -__builtin_huge_valf();
  for (long i = tid; i < npos; i += 256) m = fmaxf(m, kb[i * 384]);
  s_m[tid] = m;
  __syncthreads();
  if (tid == 0) { float M = s_m[0]; for (int i = 1; i < 256; ++i) M = fmaxf(M, s_m[i]); s_m[0] = M; }
  __syncthreads();
  const float M = s_m[0];
  double l = 0.0;
  for (long i = tid; i < npos; i += 256) l += (double)expf(kb[i * 384] - M);
  s_l[tid] = l;
  __syncthreads();
  if (tid == 0) {
    double L = 0.0;
    for (int i = 0; i < 256; ++i) L += s_l[i];
    st[((long)b * 128 + r) * 2] = M;
    st[((long)b * 128 + r) * 2 + 1] = (float)L;
  }
}

// in place: k rows of qkv -> softmax(k) over the positions
__global__ void attn_ksoftmax_kernel(float* qkv, int B, int npos, const float* st) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * npos * 128) return;
  const int r = (int)(i % 128);
  const long pos = i / 128;
  const int b = (int)(pos / npos);
  float* k = qkv + pos * 384 + 128 + r;
  *k = expf(*k - st[((long)b * 128 + r) * 2]) / st[((long)b * 128 + r) * 2 + 1];
}

// R[b][h][d][e] = sum_pos X1[b][pos][x1o + 32h + d] X2[b][pos][x2o + 32h + e]   (grid (B, 4), 1024 threads)
__global__ __launch_bounds__(1024) void attn_outer_kernel(const float* X1, int cs1, int x1o, const float* X2, int cs2,
                                                          int x2o, int npos, float* R) {
  const int b = blockIdx.x, h = blockIdx.y, d = threadIdx.x >> 5, e = threadIdx.x & 31;
  const float* p1 = X1 + (long)b * npos * cs1 + x1o + 32 * h + d;
  const float* p2 = X2 + (long)b * npos * cs2 + x2o + 32 * h + e;
  float s = 0.f;
  for (long i = 0; i < npos; ++i) s = fmaf(p1[i * cs1], p2[i * cs2], s);
  R[(((long)b * 4 + h) * 32 + d) * 32 + e] = s;
}

// Y[b][pos][yo + 32h + j] (+)= sum_i M'[i][j] X[b][pos][xo + 32h + i], M' = M[b][h] (trans = 0: M[i][j]; 1: M[j][i])
__global__ void attn_headmm_kernel(const float* M, int trans, const float* X, int csx, int xo, int B, int npos,
                                   float* Y, int csy, int yo, int accumulate) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * npos * 128) return;
  const int hj = (int)(i % 128), h = hj >> 5, j = hj & 31;
  const long pos = i / 128;
  const int b = (int)(pos / npos);
  const float* m = M + ((long)b * 4 + h) * 1024;
  const float* x = X + pos * csx + xo + 32 * h;
  float s = 0.f;
  for (int ii = 0; ii < 32; ++ii) s = fmaf(trans ? m[j * 32 + ii] : m[ii * 32 + j], x[ii], s);
  float* y = Y + pos * csy + yo + hj;
  *y = accumulate ? *y + s : s;
}

// softmax backward of the k rows: dk = ks (dks - sum_pos ks dks), in place on the dk rows of dqkv (which hold dks)
__global__ void attn_ksoftmax_bwd_kernel(const float* qkv_s, float* dqkv, int B, int npos, const float* S) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * npos * 128) return;
  const int r = (int)(i % 128);
  const long pos = i / 128;
  const int b = (int)(pos / npos);
  const float ks = qkv_s[pos * 384 + 128 + r];
  float* d = dqkv + pos * 384 + 128 + r;
  *d = ks * (*d - S[(long)b * 128 + r]);
}

// sum over positions (per b) of a[pos][ao + r] * c[pos][co + r], r < 128: S[b][r]
__global__ void attn_rowdot_kernel(const float* a, int csa, int ao, const float* c, int csc, int co, int npos, float* S) {
  const int b = blockIdx.x, r = threadIdx.x;
  float s = 0.f;
  for (long i = 0; i < npos; ++i) s = fmaf(a[((long)b * npos + i) * csa + ao + r], c[((long)b * npos + i) * csc + co + r], s);
  S[(long)b * 128 + r] = s;
}

// scalar dot (fp64 sum, fixed order): out[0] (+)= sum_i x[i] y[i]
__global__ __launch_bounds__(256) void dot_kernel(const float* x, const float* y, long n, float* out, int accumulate) {
  __shared__ double s[256];
  double a = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) a += (double)x[i] * (double)y[i];
  s[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 256; ++i) t += s[i];
    out[0] = accumulate ? out[0] + (float)t : (float)t;
  }
}

// ---------------------------------------------------------------- small dense layers ([B] rows)
// Y[b][o] = act(sum_i W[o][i] X[b][i] + bias[o]); act 0: none, 1: Mish
__global__ void linear_fwd_kernel(const float* X, int I, const float* W, const float* bias, int O, int act, float* Y) {
  const int b = blockIdx.x;
  for (int o = threadIdx.x; o < O; o += blockDim.x) {
    float s = bias ? bias[o] : 0.f;
    for (int i = 0; i < I; ++i) s += W[(long)o * I + i] * X[(long)b * I + i];
    Y[(long)b * O + o] = act == 1 ? mish_f(s) : s;
  }
}
// dW[o][i] (+)= sum_b dY[b][o] X[b][i]; db[o] (+)= sum_b dY[b][o]  (grid O rows)
__global__ void linear_wgrad_kernel(const float* dY, const float* X, int B, int I, int O, float* dW, float* db) {
  const int o = blockIdx.x;
  for (int i = threadIdx.x; i < I; i += blockDim.x) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dY[(long)b * O + o] * X[(long)b * I + i];
    dW[(long)o * I + i] += s;
  }
  if (threadIdx.x == 0 && db) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dY[(long)b * O + o];
    db[o] += s;
  }
}
// dX[b][i] (+)= (sum_o W[o][i] dY[b][o]) * (pre ? mish'(pre[b][i]) : 1)
__global__ __launch_bounds__(256) void linear_dgrad_kernel(const float* dY, const float* W, int I, int O,
                                                           const float* pre, float* dX, int accumulate) {
  // four partial sums over o (o = q mod 4) per input i, added in a fixed order
  __shared__ float red[4][64];
  const int b = blockIdx.x, il = threadIdx.x & 63, q = threadIdx.x >> 6;
  for (int i0 = 0; i0 < I; i0 += 64) {
    const int i = i0 + il;
    float s = 0.f;
    if (i < I)
#pragma unroll 4
      for (int o = q; o < O; o += 4) s += W[(long)o * I + i] * dY[(long)b * O + o];
    red[q][il] = s;
    __syncthreads();
    if (q == 0 && i < I) {
      float t = ((red[0][il] + red[1][il]) + red[2][il]) + red[3][il];
      if (pre) t *= mish_grad(pre[(long)b * I + i]);
      dX[(long)b * I + i] = accumulate ? dX[(long)b * I + i] + t : t;
    }
    __syncthreads();
  }
}
// SinusoidalPosEmb (diffusion.py:113-125) of t[b] -> [B][64]
__global__ void posemb_kernel(const float* t, float scale, const float* freqs, float* out) {
  const int b = blockIdx.x, j = threadIdx.x;
  const float arg = (scale * t[b]) * freqs[j & 31];
  out[b * 64 + j] = j < 32 ? sinf(arg) : cosf(arg);
}

// ---------------------------------------------------------------- loss / input layer / final layer
// dL/ds = 2 (s sigma_b + z m) sigma_b / N, times mask (the score is (out * mask)); sigma_b = sqrt(1 - e^-cum)
__global__ void loss_bwd_kernel(const float* score, const float* z, const float* mask, const float* t, const float* tot,
                                int B, int T, float bmin, float half_delta, float* ds) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * 80 * T) return;
  const int b = (int)(i / (80L * T)), tt = (int)(i % T);
  const float tv = t[b];
  const float cum = bmin * tv + half_delta * (tv * tv);
  const float sg = sqrtf(1.f - expf(-cum));
  const float m = mask[(long)b * T + tt];
  const float N = tot[1] * 80.f;
  ds[i] = 2.f * (score[i] * sg + z[i] * m) * sg / N * m;
}
// channels-last U-Net input [B][80][T][cin] = (mu, x_t, spk_mlp(spk) repeated over T)
__global__ void input_pack_kernel(const float* mu, const float* xt, const float* s, int B, int T, int cin, float* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * 80 * T) return;
  const int b = (int)(i / (80L * T)), f = (int)((i / T) % 80);
  out[i * cin] = mu[i];
  out[i * cin + 1] = xt[i];
  if (cin == 3) out[i * cin + 2] = s[(long)b * 80 + f];
}

bool gconv_pack_desc(const GConvParams& p, GconvPack* out) {
  if (gconv_wpk_floats(p) <= 0 || !p.wpk) return false;
  out->w = p.w; out->dst = p.wpk; out->wsa = p.wsa; out->wsc = p.wsc; out->KK = p.KS * p.KS;
  out->flip = (p.transposed ? !p.flip : p.flip != 0) ? 1 : 0;
  out->Cout = p.Cout; out->Cin = p.Cin;
  return true;
}

long gconv_wpk_floats(const GConvParams& p) {
  // the stride-1 relations (S = 2 only through the dilated input of the transposed relation), whole float4 runs
  const bool ok = (p.KS == 1 || p.KS == 3 || p.KS == 4) && (p.transposed ? p.S == 2 : p.S == 1) && p.Cin % 4 == 0 &&
                  (p.KS == 4 ? p.transposed : true) && (p.KS == 1 ? !p.transposed : true);
  return ok ? (long)p.Cout * p.KS * p.KS * p.Cin : 0;
}

hipError_t launch_gconv(const GConvParams& p, hipStream_t s) {
  if (p.KS > 4 || p.S > 2) return hipErrorInvalidValue;
  auto mgrid = [&](int rh, int tw) {
    return dim3((unsigned)((long)p.B * ((p.Fo + rh - 1) / rh) * ((p.To + tw - 1) / tw)), (unsigned)((p.Cout + 63) / 64));
  };
  auto slots = [&](int rh, int tw) { return (long)((p.Fo + rh - 1) / rh) * ((p.To + tw - 1) / tw); };
  const int se = p.transposed ? 1 : p.S, cfg = p.KS * 10 + se;
  if (gconv_wpk_floats(p) > 0 && p.wpk && ((uintptr_t)p.in & 15) == 0 && ((uintptr_t)p.wpk & 15) == 0) {
    GconvPack pk;
    if (!p.wpk_ready && gconv_pack_desc(p, &pk)) {
      const long n = (long)pk.Cout * pk.KK * pk.Cin;
      hipLaunchKernelGGL(gconv_wpack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pk.w, pk.wsa, pk.wsc,
                         pk.KK, pk.flip, pk.Cout, pk.Cin, pk.dst);
    }
    // 32-channel tiles when 64-channel tiles would leave the CUs less than two workgroups each
    auto ny1 = [&](int rh, int tw) { return (long)p.B * slots(rh, tw) * ((p.Cout + 63) / 64) < 384; };
    auto g2 = [&](int rh, int tw, int ct) {
      return dim3((unsigned)((long)p.B * slots(rh, tw)), (unsigned)((p.Cout + ct - 1) / ct));
    };
#define MPK_LAUNCH(KS_, RH_, TW_, KC_)                                                                            \
  do {                                                                                                        \
    if (ny1(RH_, TW_)) hipLaunchKernelGGL((mconv_pk_kernel<KS_, RH_, TW_, KC_, 1>), g2(RH_, TW_, 32), dim3(256), 0, s, p); \
    else hipLaunchKernelGGL((mconv_pk_kernel<KS_, RH_, TW_, KC_, 2>), g2(RH_, TW_, 64), dim3(256), 0, s, p);           \
  } while (0)
    const long s4 = slots(4, 64), s8 = slots(8, 32), s5 = slots(5, 48);
    const int shape = (s4 <= s8 && s4 <= s5) ? 4 : (s8 <= s5) ? 8 : 5;
    if (p.KS == 4) MPK_LAUNCH(4, 4, 64, 8);
    else if (p.KS == 1) {   // 1x1: 32-channel chunks
      if (shape == 4) MPK_LAUNCH(1, 4, 64, 32);
      else if (shape == 8) MPK_LAUNCH(1, 8, 32, 32);
      else MPK_LAUNCH(1, 5, 48, 32);
    } else {
      if (shape == 4) MPK_LAUNCH(3, 4, 64, 16);
      else if (shape == 8) MPK_LAUNCH(3, 8, 32, 16);
      else MPK_LAUNCH(3, 5, 48, 16);
    }
#undef MPK_LAUNCH
    return hipGetLastError();
  }
  if (cfg == 11) {
    hipLaunchKernelGGL(mconv1_kernel, dim3((unsigned)((long)p.B * p.Fo * ((p.To + 63) / 64)),
                                           (unsigned)((p.Cout + 63) / 64)), dim3(256), 0, s, p);
  } else if (cfg == 31) {   // the 3x3 stride-1 convs: tile shape with the fewest 256-position tiles
    const long s4 = slots(4, 64), s8 = slots(8, 32), s5 = slots(5, 48);
    if (s4 <= s8 && s4 <= s5) hipLaunchKernelGGL((mconv_kernel<3, 1, 4, 64>), mgrid(4, 64), dim3(256), 0, s, p);
    else if (s8 <= s5) hipLaunchKernelGGL((mconv_kernel<3, 1, 8, 32>), mgrid(8, 32), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((mconv_kernel<3, 1, 5, 48>), mgrid(5, 48), dim3(256), 0, s, p);
  }
  else if (cfg == 32) hipLaunchKernelGGL((mconv_kernel<3, 2, 4, 64>), mgrid(4, 64), dim3(256), 0, s, p);
  else if (cfg == 41) hipLaunchKernelGGL((mconv_kernel<4, 1, 4, 64>), mgrid(4, 64), dim3(256), 0, s, p);
  else if (cfg == 42) hipLaunchKernelGGL((mconv_kernel<4, 2, 4, 64>), mgrid(4, 64), dim3(256), 0, s, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// dX[b][i] = dY[b][i] * mish'(pre[b][i])   (grid B, block >= n)
__global__ void mish_bwd_kernel(const float* dY, const float* pre, int n, float* dX) {
  const int b = blockIdx.x, i = threadIdx.x;
  if (i < n) dX[(long)b * n + i] = dY[(long)b * n + i] * mish_grad(pre[(long)b * n + i]);
}
// dmu = dx_in[.., 0] + dx_in[.., 1] (1 - e) m: mu enters the U-Net directly and through x_t (diffusion.py:247, 251)
__global__ void dmu_kernel(const float* dxin, int cin, const float* t, const float* mask, int B, int T, float bmin,
                           float half_delta, float* dmu) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * 80 * T) return;
  const int b = (int)(i / (80L * T)), tt = (int)(i % T);
  const float tv = t[b];
  const float cum = __fadd_rn(__fmul_rn(bmin, tv), __fmul_rn(half_delta, __fmul_rn(tv, tv)));
  const float e = expf(-0.5f * cum);
  dmu[i] = dxin[i * cin] + dxin[i * cin + 1] * (1.f - e) * mask[(long)b * T + tt];
}
// ds[b][f] = sum_t dx_in[b][f][t][2]   (the speaker channel is spk_mlp(spk) repeated over T, diffusion.py:183-184)
__global__ void spk_chan_sum_kernel(const float* dxin, int cin, int T, float* ds) {
  const int b = blockIdx.x, f = threadIdx.x;
  if (f >= 80) return;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += dxin[(((long)b * 80 + f) * T + t) * cin + 2];
  ds[b * 80 + f] = s;
}
// out[0] = sum of the mask (fp64, fixed order)
__global__ void mask_sum_kernel(const float* mask, long n, float* out) {
  __shared__ double s[256];
  double a = 0.0;
  for (long i = threadIdx.x; i < n; i += 256) a += mask[i];
  s[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 256; ++i) t += s[i];
    out[0] = (float)t;
  }
}

// ---------------------------------------------------------------- split reductions over the positions
// Every position sum below runs in two fixed-order levels: S splits of each utterance's positions (pos_splits), then
// the splits in order (sum_splits_kernel). Deterministic, and the grid fills the chip at every level.
int pos_splits(long npos) { return (int)std::max<long>(1, std::min<long>(128, npos / 128)); }


// out[g][j] (+)= sum_q part[g][q][j]: 16 outputs x 16 split lanes per workgroup; lane l sums q = l, l + 16, ...
// ascending, then the 16 lane sums are added in lane order (fixed order: deterministic)
__global__ __launch_bounds__(256) void sum_splits_kernel(const float* part, int G, int S, long n, float* out,
                                                         int accumulate) {
  __shared__ float red[16][17];
  const int jl = threadIdx.x & 15, ql = threadIdx.x >> 4;
  const long nj = (n + 15) / 16;
  const long g = blockIdx.x / nj, j = (blockIdx.x % nj) * 16 + jl;
  float s = 0.f;
  if (j < n) {
    const float* pg = part + g * S * n + j;
#pragma unroll 4
    for (int q = ql; q < S; q += 16) s += pg[(long)q * n];
  }
  red[ql][jl] = s;
  __syncthreads();
  if (ql == 0 && j < n) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < 16; ++l) t += red[l][jl];
    const long i = g * n + j;
    out[i] = accumulate ? out[i] + t : t;
  }
}

// part[b][s][c] = sum over split s of utterance b's positions of x[b][pos][c] (* y): grid (C/64, S, B), 64 channels
// x 4 position lanes per workgroup (each wave reads 64 consecutive channels of one position)
__global__ __launch_bounds__(256) void chan_partial_kernel(const float* x, int xcs, int xo, const float* y, int ycs,
                                                           int yo, int npos, int C, float* part) {
  __shared__ float s_r[4][64];
  const int tid = threadIdx.x, cl = tid & 63, pl = tid >> 6;
  const int c = blockIdx.x * 64 + cl, s = blockIdx.y, b = blockIdx.z, S = gridDim.y;
  long lo, hi;
  split_range(npos, S, s, &lo, &hi);
  float acc = 0.f;
  if (c < C) {
    const float* xb = x + (long)b * npos * xcs + xo + c;
    const float* yb = y ? y + (long)b * npos * ycs + yo + c : nullptr;
    for (long i = lo + pl; i < hi; i += 4) acc += yb ? xb[i * xcs] * yb[i * ycs] : xb[i * xcs];
  }
  s_r[pl][cl] = acc;
  __syncthreads();
  if (pl == 0 && c < C) part[((long)b * S + s) * C + c] = ((s_r[0][cl] + s_r[1][cl]) + s_r[2][cl]) + s_r[3][cl];
}

// Block backward sums: part[b][s][c] = (sum dn xhat, sum dn) over split s (dn = dA m mish'(n), as block_bwd_apply)
__global__ __launch_bounds__(256) void block_bwd_partial_kernel(BlockBwdParams p, float* part) {
  __shared__ float s_r[2][4][64];
  const int tid = threadIdx.x, cl = tid & 63, pl = tid >> 6;
  const int c = blockIdx.x * 64 + cl, s = blockIdx.y, b = blockIdx.z, S = gridDim.y;
  long lo, hi;
  split_range(p.npos, S, s, &lo, &hi);
  float a1 = 0.f, a2 = 0.f;
  if (c < p.C) {
    const int g = c / (p.C / 8);
    const float mean = p.stats[(b * 8 + g) * 2], rstd = p.stats[(b * 8 + g) * 2 + 1];
    const float gm = p.gamma[c], bt = p.beta[c];
    for (long pos = lo + pl; pos < hi; pos += 4) {
      const long o = ((long)b * p.npos + pos) * p.C + c;
      const float xh = (p.h[o] - mean) * rstd;
      const float m = mask_at(p.mask, p.T0, b, (int)(pos % p.T), p.lvl);
      const float dn = p.dA[o] * m * mish_grad(xh * gm + bt);
      a1 += dn * xh;
      a2 += dn;
    }
  }
  s_r[0][pl][cl] = a1;
  s_r[1][pl][cl] = a2;
  __syncthreads();
  if (pl == 0 && c < p.C) {
    float* o = part + (((long)b * S + s) * p.C + c) * 2;
    o[0] = ((s_r[0][0][cl] + s_r[0][1][cl]) + s_r[0][2][cl]) + s_r[0][3][cl];
    o[1] = ((s_r[1][0][cl] + s_r[1][1][cl]) + s_r[1][2][cl]) + s_r[1][3][cl];
  }
}

// per utterance (one workgroup, C <= 256): dgb[b][c] = splits summed in order (fp64); gsum[b][g] = (S1, S2) with
// S1 = sum_c gamma_c sum dn = sum dn gamma, S2 = sum_c gamma_c sum dn xhat
__global__ __launch_bounds__(256) void block_bwd_final_kernel(BlockBwdParams p, const float* part, int S) {
  __shared__ double s_g[2][256];
  const int b = blockIdx.x, c = threadIdx.x;
  if (c < p.C) {
    double d1 = 0.0, d2 = 0.0;
    for (int q = 0; q < S; ++q) {
      const float* o = part + (((long)b * S + q) * p.C + c) * 2;
      d1 += (double)o[0];
      d2 += (double)o[1];
    }
    p.dgb[((long)b * p.C + c) * 2] = (float)d1;
    p.dgb[((long)b * p.C + c) * 2 + 1] = (float)d2;
    s_g[0][c] = (double)p.gamma[c] * d2;
    s_g[1][c] = (double)p.gamma[c] * d1;
  }
  __syncthreads();
  if (c < 8) {
    const int cg = p.C / 8;
    double S1 = 0.0, S2 = 0.0;
    for (int i = 0; i < cg; ++i) { S1 += s_g[0][c * cg + i]; S2 += s_g[1][c * cg + i]; }
    p.gsum[(b * 8 + c) * 2] = (float)S1;
    p.gsum[(b * 8 + c) * 2 + 1] = (float)S2;
  }
}

// dot product: 256 workgroups of fp64 partials, then one thread in order
__global__ __launch_bounds__(256) void dot_partial_kernel(const float* x, const float* y, long n, double* part) {
  __shared__ double s[256];
  long lo, hi;
  split_range(n, gridDim.x, blockIdx.x, &lo, &hi);
  double a = 0.0;
  for (long i = lo + threadIdx.x; i < hi; i += 256) a += (double)x[i] * (double)y[i];
  s[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 256; ++i) t += s[i];
    part[blockIdx.x] = t;
  }
}
__global__ void dot_final_kernel(const double* part, int nblk, float* out, int accumulate) {
  if (threadIdx.x != 0) return;
  double t = 0.0;
  for (int i = 0; i < nblk; ++i) t += part[i];
  out[0] = accumulate ? out[0] + (float)t : (float)t;
}

// attn_outer over a split of the positions: part[s][b][h][d][e]   (grid (B, 4, S), 1024 threads)
__global__ __launch_bounds__(1024) void attn_outer_split_kernel(const float* X1, int cs1, int x1o, const float* X2,
                                                                int cs2, int x2o, int npos, float* part) {
  const int b = blockIdx.x, h = blockIdx.y, s = blockIdx.z, B = gridDim.x, d = threadIdx.x >> 5, e = threadIdx.x & 31;
  long lo, hi;
  split_range(npos, gridDim.z, s, &lo, &hi);
  const float* p1 = X1 + (long)b * npos * cs1 + x1o + 32 * h + d;
  const float* p2 = X2 + (long)b * npos * cs2 + x2o + 32 * h + e;
  float acc = 0.f;
  for (long i = lo; i < hi; ++i) acc = fmaf(p1[i * cs1], p2[i * cs2], acc);
  part[((((long)s * B + b) * 4 + h) * 32 + d) * 32 + e] = acc;
}

// attn_rowdot over a split: part[s][b][r]   (grid (B, S), 128 threads)
__global__ void attn_rowdot_split_kernel(const float* a, int csa, int ao, const float* c, int csc, int co, int npos,
                                         float* part) {
  const int b = blockIdx.x, s = blockIdx.y, B = gridDim.x, r = threadIdx.x;
  long lo, hi;
  split_range(npos, gridDim.y, s, &lo, &hi);
  float acc = 0.f;
  for (long i = lo; i < hi; ++i)
    acc = fmaf(a[((long)b * npos + i) * csa + ao + r], c[((long)b * npos + i) * csc + co + r], acc);
  part[((long)s * B + b) * 128 + r] = acc;
}

// Y[b][pos][yo + 32h + j] (+)= sum_i M'[i][j] X[b][pos][xo + 32h + i] on fp32 MFMA: 64 positions x 4 heads per
// workgroup (wave = head), X slice and M staged in LDS
__global__ __launch_bounds__(256) void attn_headmm_mfma_kernel(const float* M, int trans, const float* X, int csx, int xo,
                                                               int npos, float* Y, int csy, int yo, int accumulate) {
  __shared__ float s_x[64][129];
  __shared__ float s_m[4][32][33];
  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int p0 = blockIdx.x * 64, b = blockIdx.y;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int i = tid + 256 * j, pp = i >> 7, ch = i & 127;
    s_x[pp][ch] = p0 + pp < npos ? X[((long)b * npos + p0 + pp) * csx + xo + ch] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int i = tid + 256 * j, hd = i >> 10, ii = (i >> 5) & 31, jj = i & 31;
    s_m[hd][ii][jj] = M[(long)b * 4096 + i];
  }
  __syncthreads();
#pragma unroll
  for (int pbk = 0; pbk < 2; ++pbk) {
    f32x16 acc;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int i = 2 * ks + hh;
      const float bv = trans ? s_m[h][r][i] : s_m[h][i][r];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(s_x[pbk * 32 + r][32 * h + i], bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int pos = p0 + pbk * 32 + acc_row(j, hh);
      if (pos >= npos) continue;
      float* y = Y + ((long)b * npos + pos) * csy + yo + 32 * h + r;
      *y = accumulate ? *y + acc[j] : acc[j];
    }
  }
}

// R_part[s][b][h][d][e] = sum over split s of X1[pos][x1o + 32h + d] X2[pos][x2o + 32h + e] on fp32 MFMA
// (grid (S, B), wave = head, 32-position segments staged in LDS)
__global__ __launch_bounds__(256) void attn_outer_mfma_kernel(const float* X1, int cs1, int x1o, const float* X2, int cs2,
                                                              int x2o, int npos, float* part) {
  __shared__ float s1[32][129], s2[32][129];
  const int tid = threadIdx.x, lane = tid & 63, h = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int sp = blockIdx.x, b = blockIdx.y, S = gridDim.x, B = gridDim.y;
  long lo, hi;
  split_range(npos, S, sp, &lo, &hi);
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (long p0 = lo; p0 < hi; p0 += 32) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int i = tid + 256 * j, pp = i >> 7, ch = i & 127;
      const bool ok = p0 + pp < hi;
      s1[pp][ch] = ok ? X1[((long)b * npos + p0 + pp) * cs1 + x1o + ch] : 0.f;
      s2[pp][ch] = ok ? X2[((long)b * npos + p0 + pp) * cs2 + x2o + ch] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int pp = 2 * ks + hh;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(s1[pp][32 * h + r], s2[pp][32 * h + r], acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < 16; ++j)
    part[((((long)sp * B + b) * 4 + h) * 32 + acc_row(j, hh)) * 32 + r] = acc[j];
}

hipError_t launch_attn_headmm_mfma(const float* M, int trans, const float* X, int csx, int xo, int B, int npos, float* Y,
                                   int csy, int yo, int accumulate, hipStream_t strm) {
  hipLaunchKernelGGL(attn_headmm_mfma_kernel, dim3((npos + 63) / 64, B), dim3(256), 0, strm, M, trans, X, csx, xo, npos, Y,
                     csy, yo, accumulate);
  return hipGetLastError();
}

static hipError_t sum_splits(const float* part, int G, int S, long n, float* out, int accumulate, hipStream_t strm) {
  hipLaunchKernelGGL(sum_splits_kernel, dim3((unsigned)((long)G * ((n + 15) / 16))), dim3(256), 0, strm, part, G, S, n,
                     out, accumulate);
  return hipGetLastError();
}

hipError_t launch_chan_sums(const float* x, const float* y, int B, int npos, int C, float* part, float* out, int per_b,
                            int accumulate, hipStream_t strm) {
  return launch_chan_sums_strided(x, C, 0, y, C, 0, B, npos, C, part, out, per_b, accumulate, strm);
}
hipError_t launch_chan_sums_strided(const float* x, int xcs, int xo, const float* y, int ycs, int yo, int B, int npos,
                                    int C, float* part, float* out, int per_b, int accumulate, hipStream_t strm) {
  const int S = pos_splits(npos);
  hipLaunchKernelGGL(chan_partial_kernel, dim3((C + 63) / 64, S, B), dim3(256), 0, strm, x, xcs, xo, y, ycs, yo, npos, C,
                     part);
  return per_b ? sum_splits(part, B, S, C, out, accumulate, strm) : sum_splits(part, 1, B * S, C, out, accumulate, strm);
}

hipError_t launch_block_bwd_sums(const BlockBwdParams& p, float* part, hipStream_t strm) {
  if (p.C > 256) return hipErrorInvalidValue;
  const int S = pos_splits(p.npos);
  hipLaunchKernelGGL(block_bwd_partial_kernel, dim3((p.C + 63) / 64, S, p.B), dim3(256), 0, strm, p, part);
  hipLaunchKernelGGL(block_bwd_final_kernel, dim3(p.B), dim3(256), 0, strm, p, part, S);
  return hipGetLastError();
}

hipError_t launch_dot_sum(const float* x, const float* y, long n, double* part, float* out, int accumulate,
                          hipStream_t strm) {
  hipLaunchKernelGGL(dot_partial_kernel, dim3(kDotBlocks), dim3(256), 0, strm, x, y, n, part);
  hipLaunchKernelGGL(dot_final_kernel, dim3(1), dim3(64), 0, strm, part, kDotBlocks, out, accumulate);
  return hipGetLastError();
}

hipError_t launch_attn_outer_split(const float* X1, int cs1, int x1o, const float* X2, int cs2, int x2o, int B, int npos,
                                   float* part, float* R, hipStream_t strm) {
  const int S = pos_splits(npos);
  hipLaunchKernelGGL(attn_outer_mfma_kernel, dim3(S, B), dim3(256), 0, strm, X1, cs1, x1o, X2, cs2, x2o, npos, part);
  return sum_splits(part, 1, S, (long)B * 4096, R, 0, strm);
}

hipError_t launch_attn_rowdot_split(const float* a, int csa, int ao, const float* c, int csc, int co, int B, int npos,
                                    float* part, float* S_out, hipStream_t strm) {
  return launch_chan_sums_strided(a, csa, ao, c, csc, co, B, npos, 128, part, S_out, 1, 0, strm);
}

// ---- launchers
hipError_t launch_bsum(dim3 grid, dim3 block, hipStream_t strm, const float* x, const float* y, int npos, int C, float* out, int accumulate) {
  hipLaunchKernelGGL(bsum_kernel, grid, block, 0, strm, x, y, npos, C, out, accumulate);
  return hipGetLastError();
}
hipError_t launch_colsum(dim3 grid, dim3 block, hipStream_t strm, const float* in, int B, int C, float* out, int accumulate) {
  hipLaunchKernelGGL(colsum_kernel, grid, block, 0, strm, in, B, C, out, accumulate);
  return hipGetLastError();
}
hipError_t launch_gn_stats(dim3 grid, dim3 block, hipStream_t strm, const float* h, int npos, int C, float* stats) {
  hipLaunchKernelGGL(gn_stats_kernel, grid, block, 0, strm, h, npos, C, stats);
  return hipGetLastError();
}
hipError_t launch_block_bwd_reduce(dim3 grid, dim3 block, hipStream_t strm, BlockBwdParams p) {
  hipLaunchKernelGGL(block_bwd_reduce_kernel, grid, block, 0, strm, p);
  return hipGetLastError();
}
hipError_t launch_block_bwd_apply(dim3 grid, dim3 block, hipStream_t strm, BlockBwdParams p) {
  hipLaunchKernelGGL(block_bwd_apply_kernel, grid, block, 0, strm, p);
  return hipGetLastError();
}
hipError_t launch_block_fwd(dim3 grid, dim3 block, hipStream_t strm, BlockBwdParams p, const float* tb, float* out) {
  hipLaunchKernelGGL(block_fwd_kernel, grid, block, 0, strm, p, tb, out);
  return hipGetLastError();
}
hipError_t launch_ew(dim3 grid, dim3 block, hipStream_t strm, EwParams p) {
  hipLaunchKernelGGL(ew_kernel, grid, block, 0, strm, p);
  return hipGetLastError();
}
hipError_t launch_attn_kstats(dim3 grid, dim3 block, hipStream_t strm, const float* qkv, int npos, float* st) {
  hipLaunchKernelGGL(attn_kstats_kernel, grid, block, 0, strm, qkv, npos, st);
  return hipGetLastError();
}
hipError_t launch_attn_ksoftmax(dim3 grid, dim3 block, hipStream_t strm, float* qkv, int B, int npos, const float* st) {
  hipLaunchKernelGGL(attn_ksoftmax_kernel, grid, block, 0, strm, qkv, B, npos, st);
  return hipGetLastError();
}
hipError_t launch_attn_outer(dim3 grid, dim3 block, hipStream_t strm, const float* X1, int cs1, int x1o, const float* X2, int cs2, int x2o, int npos, float* R) {
  hipLaunchKernelGGL(attn_outer_kernel, grid, block, 0, strm, X1, cs1, x1o, X2, cs2, x2o, npos, R);
  return hipGetLastError();
}
hipError_t launch_attn_headmm(dim3 grid, dim3 block, hipStream_t strm, const float* M, int trans, const float* X, int csx, int xo, int B, int npos, float* Y, int csy, int yo, int accumulate) {
  hipLaunchKernelGGL(attn_headmm_kernel, grid, block, 0, strm, M, trans, X, csx, xo, B, npos, Y, csy, yo, accumulate);
  return hipGetLastError();
}
hipError_t launch_attn_ksoftmax_bwd(dim3 grid, dim3 block, hipStream_t strm, const float* qkv_s, float* dqkv, int B, int npos, const float* S) {
  hipLaunchKernelGGL(attn_ksoftmax_bwd_kernel, grid, block, 0, strm, qkv_s, dqkv, B, npos, S);
  return hipGetLastError();
}
hipError_t launch_attn_rowdot(dim3 grid, dim3 block, hipStream_t strm, const float* a, int csa, int ao, const float* c, int csc, int co, int npos, float* S) {
  hipLaunchKernelGGL(attn_rowdot_kernel, grid, block, 0, strm, a, csa, ao, c, csc, co, npos, S);
  return hipGetLastError();
}
hipError_t launch_dot(dim3 grid, dim3 block, hipStream_t strm, const float* x, const float* y, long n, float* out, int accumulate) {
  hipLaunchKernelGGL(dot_kernel, grid, block, 0, strm, x, y, n, out, accumulate);
  return hipGetLastError();
}
hipError_t launch_linear_fwd(dim3 grid, dim3 block, hipStream_t strm, const float* X, int I, const float* W, const float* bias, int O, int act, float* Y) {
  hipLaunchKernelGGL(linear_fwd_kernel, grid, block, 0, strm, X, I, W, bias, O, act, Y);
  return hipGetLastError();
}
hipError_t launch_linear_wgrad(dim3 grid, dim3 block, hipStream_t strm, const float* dY, const float* X, int B, int I, int O, float* dW, float* db) {
  hipLaunchKernelGGL(linear_wgrad_kernel, grid, block, 0, strm, dY, X, B, I, O, dW, db);
  return hipGetLastError();
}
hipError_t launch_linear_dgrad(dim3 grid, dim3 block, hipStream_t strm, const float* dY, const float* W, int I, int O, const float* pre, float* dX, int accumulate) {
  (void)block;   // 256 threads: 64 inputs x 4 partial sums
  hipLaunchKernelGGL(linear_dgrad_kernel, grid, dim3(256), 0, strm, dY, W, I, O, pre, dX, accumulate);
  return hipGetLastError();
}
hipError_t launch_posemb(dim3 grid, dim3 block, hipStream_t strm, const float* t, float scale, const float* freqs, float* out) {
  hipLaunchKernelGGL(posemb_kernel, grid, block, 0, strm, t, scale, freqs, out);
  return hipGetLastError();
}
hipError_t launch_loss_bwd(dim3 grid, dim3 block, hipStream_t strm, const float* score, const float* z, const float* mask, const float* t, const float* tot, int B, int T, float bmin, float half_delta, float* ds) {
  hipLaunchKernelGGL(loss_bwd_kernel, grid, block, 0, strm, score, z, mask, t, tot, B, T, bmin, half_delta, ds);
  return hipGetLastError();
}
hipError_t launch_input_pack(dim3 grid, dim3 block, hipStream_t strm, const float* mu, const float* xt, const float* s, int B, int T, int cin, float* out) {
  hipLaunchKernelGGL(input_pack_kernel, grid, block, 0, strm, mu, xt, s, B, T, cin, out);
  return hipGetLastError();
}

hipError_t launch_mish_bwd(dim3 grid, dim3 block, hipStream_t strm, const float* dY, const float* pre, int n, float* dX) {
  hipLaunchKernelGGL(mish_bwd_kernel, grid, block, 0, strm, dY, pre, n, dX);
  return hipGetLastError();
}
hipError_t launch_dmu(dim3 grid, dim3 block, hipStream_t strm, const float* dxin, int cin, const float* t,
                      const float* mask, int B, int T, float bmin, float half_delta, float* dmu) {
  hipLaunchKernelGGL(dmu_kernel, grid, block, 0, strm, dxin, cin, t, mask, B, T, bmin, half_delta, dmu);
  return hipGetLastError();
}
hipError_t launch_spk_chan_sum(dim3 grid, dim3 block, hipStream_t strm, const float* dxin, int cin, int T, float* ds) {
  hipLaunchKernelGGL(spk_chan_sum_kernel, grid, block, 0, strm, dxin, cin, T, ds);
  return hipGetLastError();
}
hipError_t launch_mask_sum(dim3 grid, dim3 block, hipStream_t strm, const float* mask, long n, float* out) {
  hipLaunchKernelGGL(mask_sum_kernel, grid, block, 0, strm, mask, n, out);
  return hipGetLastError();
}

}  // namespace gt
