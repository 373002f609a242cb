// Text encoder of GradTTS (model/text_encoder.py:285-335) and the front-end of GradTTS.forward
// (model/tts.py:86-101, utils.py:6-39) for gfx950. fp32 (the reference's inference precision), activations
// channels-last [B][T][C]:
//
//   c1d_kernel      every Conv1d (prenet k5, FFN k3, duration predictor k3, the 1x1 q/k/v/o and projections) as an
//                   implicit GEMM on v_mfma_f32_32x32x2_f32: 64 frames x 64 output channels per workgroup, 16-channel
//                   chunks of the input (+ K - 1 halo frames) and of the weights in LDS; the epilogue adds the bias,
//                   ReLU, the residual and the mask, and writes channels-last or channel-major (mu_x, logw)
//   te_ln_kernel    LayerNorm over channels (+ residual, + ReLU, * mask), one wave per frame
//   te_attn_kernel  relative-position attention: 16 query frames per workgroup, 64-frame key/value tiles in LDS,
//                   online softmax; the relative key logits and value terms (|j - i| <= window) from LDS copies
//                   of emb_rel_k / emb_rel_v; masked_fill(-1e4) semantics kept (padded rows average all keys)
//   te_durations / te_expand   durations, y_lengths, generate_path and mu_y = attn^T mu_x as a gather
#include <math.h>

#include "common.h"
#include "textenc.h"

namespace gt {

GT_DEV float wave_sum(float x) {   // butterfly over the 64 lanes (every lane gets the total)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

constexpr int C1_KMAX = 11, C1_SPAN = 80;   // taps, (K - 1) |dilation| (HiFi-GAN V3: (7 - 1) x 12 = 72)
C1dParams c1d_defaults() {
  C1dParams p{};
  p.tap_step = 1;
  p.dil = 1;
  p.out_stride = 1;
  return p;
}

// LDS sized per kernel-size class: KM taps at most, KC input channels per chunk, patch rows 64 + SP (short kernels
// take 32-channel chunks: a 3-tap conv has too few MFMAs per chunk to hide two barriers on 16)
template <int KM, int KC, int SP>
__global__ __launch_bounds__(256) void c1d_kernel(C1dParams p) {
  constexpr int C1_KC = KC;
  __shared__ float s_in[64 + SP][C1_KC + 1];
  __shared__ float s_w[C1_KC][KM][65];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int n_qt = (p.Q + 63) / 64;
  const int qt = blockIdx.x % n_qt, b = blockIdx.x / n_qt;
  const int q0 = qt * 64, a0 = blockIdx.y * 64;
  const int pb = (wv & 1) * 32, cb = (wv >> 1) * 32;
  const int K = p.K, span = (K - 1) * p.dil;
  const int lo = span < 0 ? span : 0, NP = 64 + (span < 0 ? -span : span);
  const int start = q0 - p.pad + lo;   // input frame of patch row 0
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (int c0 = 0; c0 < p.Cin; c0 += C1_KC) {
    __syncthreads();
    for (int i = tid; i < NP * C1_KC; i += 256) {
      const int c = i & (C1_KC - 1), pp = i / C1_KC;
      const int t = start + pp, ci = c0 + c;
      float v = 0.f;
      if (t >= 0 && t < p.T && ci < p.Cin) {
        v = p.in_chan_major ? p.in[((long)b * p.Cin + ci) * p.T + t] : p.in[((long)b * p.T + t) * p.in_cs + ci];
        if (p.in_act && v < 0.f) v *= p.in_slope;
        if (p.in_mask) v *= p.in_mask[(long)b * p.T + t];
      }
      s_in[pp][c] = v;
    }
    for (int i = tid; i < 64 * C1_KC * K; i += 256) {
      const int k = i % K, rest = i / K, c = rest % C1_KC, a = rest / C1_KC;
      s_w[c][k][a] = (a0 + a < p.Cout && c0 + c < p.Cin)
                         ? p.w[(long)(a0 + a) * p.wso + (long)(c0 + c) * p.wsc + p.tap0 + k * p.tap_step] : 0.f;
    }
    __syncthreads();
    for (int k = 0; k < K; ++k) {
      const int row = pb + r + k * p.dil - lo;
#pragma unroll
      for (int cp = 0; cp < C1_KC / 2; ++cp) {
        const int c = 2 * cp + hh;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(s_in[row][c], s_w[c][k][cb + r], acc, 0, 0, 0);
      }
    }
  }
  const int o = a0 + cb + r;
  if (o >= p.Cout) return;
  const float bias = p.bias ? p.bias[o] : 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int q = q0 + pb + acc_row(j, hh);
    if (q >= p.Q) continue;
    const int t = q * p.out_stride + p.out_off;
    if (t < 0 || t >= p.Tout) continue;
    float v = acc[j] + bias;
    if (p.relu) v = fmaxf(v, 0.f);
    v *= drop_scale(p.drop, ((uint64_t)b * p.Tout + t) * p.Cout + o);
    if (p.res) v = p.res[((long)b * p.Tout + t) * p.res_cs + o] + v;
    const long oi = p.chan_major ? ((long)b * p.Cout + o) * p.Tout + t : ((long)b * p.Tout + t) * p.out_cs + p.out_c0 + o;
    if (p.accumulate) v = p.out[oi] + v;
    if (p.div != 0.f) v = v / p.div;
    if (p.out_tanh) v = tanhf(v);
    if (p.out_mask) v *= p.out_mask[(long)b * p.Tout + t];
    p.out[oi] = v;
  }
}

// Packed fp32 variant for channels-last inputs (the HiFi-GAN generator's convs, hifi-gan/models.py:13-128): weights
// pre-packed [Cout][K][Cin] so a chunk of KC input channels is one float4 run per (o, k) row, staged without index
// divisions; the next chunk is fetched into registers while the MFMAs run on the current one (one LDS buffer, two
// barriers per chunk); the leaky ReLU / mask are applied when the registers are written to LDS. Tile: CT output
// channels x FT frames, each wave 32 channels x NB 32-frame blocks; operands read as float4 (channels 8g + 4h ..
// + 3 for lane half h) and fed to four v_mfma_f32_32x32x2_f32 (element e = K index h of channel 8g + 4h + e on
// both operands), one B read shared by the NB frame blocks.
template <int KM, int KC, int SP, int CT, int NB>
__global__ __launch_bounds__(256, 2) void c1d_pk_kernel(C1dParams p) {
  constexpr int WC = CT / 32, WF = 4 / WC, FT = WF * 32 * NB, LD = KC + 4, G4 = KC / 4;
  constexpr int G4S = G4 == 4 ? 2 : 3;   // log2(G4)
  constexpr int NIN = ((FT + SP) * G4 + 255) / 256, NW = (KM * CT * G4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float s_in[(FT + SP) * LD];
  __shared__ __attribute__((aligned(16))) float s_w[KM * CT * LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int n_qt = (p.Q + FT - 1) / FT;
  const int qt = blockIdx.x % n_qt, b = blockIdx.x / n_qt;
  const int q0 = qt * FT, a0 = blockIdx.y * CT;
  const int pb = (wv % WF) * 32 * NB, cb = (wv / WF) * 32;
  const int K = p.K, span = (K - 1) * p.dil;
  const int lo = span < 0 ? span : 0, NP = FT + (span < 0 ? -span : span);
  const int start = q0 - p.pad + lo;
  const int nw = K * CT * G4, wrows = K * (p.Cout - a0);   // packed (o, k) rows valid: o < Cout - a0
  float4 rin[NIN], rw[NW];
  float rm[NIN];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int n = 0; n < NIN; ++n) {
      const int i = tid + 256 * n, pp = i >> G4S, g = i & (G4 - 1), t = start + pp;
      rin[n] = make_float4(0.f, 0.f, 0.f, 0.f);
      rm[n] = 1.f;
      if (pp < NP && t >= 0 && t < p.T && c0 + 4 * g < p.Cin) {
        rin[n] = *reinterpret_cast<const float4*>(p.in + ((long)b * p.T + t) * p.in_cs + c0 + 4 * g);
        if (p.in_mask) rm[n] = p.in_mask[(long)b * p.T + t];
      }
    }
#pragma unroll
    for (int n = 0; n < NW; ++n) {
      const int i = tid + 256 * n, ok = i >> G4S, g = i & (G4 - 1);
      rw[n] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < nw && ok < wrows && c0 + 4 * g < p.Cin)
        rw[n] = *reinterpret_cast<const float4*>(p.wpk + ((long)a0 * K + ok) * p.Cin + c0 + 4 * g);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int n = 0; n < NIN; ++n) {
      const int i = tid + 256 * n, pp = i >> G4S, g = i & (G4 - 1);
      if (pp < NP) {
        float4 v = rin[n];
        if (p.in_act) {
          v.x = v.x < 0.f ? v.x * p.in_slope : v.x;
          v.y = v.y < 0.f ? v.y * p.in_slope : v.y;
          v.z = v.z < 0.f ? v.z * p.in_slope : v.z;
          v.w = v.w < 0.f ? v.w * p.in_slope : v.w;
        }
        v.x *= rm[n]; v.y *= rm[n]; v.z *= rm[n]; v.w *= rm[n];
        *reinterpret_cast<float4*>(s_in + pp * LD + 4 * g) = v;
      }
    }
#pragma unroll
    for (int n = 0; n < NW; ++n) {
      const int i = tid + 256 * n;
      if (i < nw) *reinterpret_cast<float4*>(s_w + (i >> G4S) * LD + 4 * (i & (G4 - 1))) = rw[n];
    }
  };
  f32x16 acc[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[m][j] = 0.f;
  fetch(0);
  store();
  __syncthreads();
  for (int c0 = 0; c0 < p.Cin; c0 += KC) {
    const bool more = c0 + KC < p.Cin;
    if (more) fetch(c0 + KC);
    const float* pw = s_w + (cb + r) * K * LD + 4 * hh;
    const float* pa = s_in + (pb + r - lo) * LD + 4 * hh;
    for (int k = 0; k < K; ++k) {
      const float* pak = pa + k * p.dil * LD;
      const float* pwk = pw + k * LD;
#pragma unroll
      for (int g = 0; g < KC / 8; ++g) {
        const float4 w = *reinterpret_cast<const float4*>(pwk + 8 * g);
        float4 a[NB];
#pragma unroll
        for (int m = 0; m < NB; ++m) a[m] = *reinterpret_cast<const float4*>(pak + m * 32 * LD + 8 * g);
#pragma unroll
        for (int m = 0; m < NB; ++m) {
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].x, w.x, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].y, w.y, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].z, w.z, acc[m], 0, 0, 0);
          acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m].w, w.w, acc[m], 0, 0, 0);
        }
      }
    }
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
  const int o = a0 + cb + r;
  if (o >= p.Cout) return;
  const float bias = p.bias ? p.bias[o] : 0.f;
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int q = q0 + pb + 32 * m + acc_row(j, hh);
      if (q >= p.Q) continue;
      const int t = q * p.out_stride + p.out_off;
      if (t < 0 || t >= p.Tout) continue;
      float v = acc[m][j] + bias;
      if (p.relu) v = fmaxf(v, 0.f);
      v *= drop_scale(p.drop, ((uint64_t)b * p.Tout + t) * p.Cout + o);
      if (p.res) v = p.res[((long)b * p.Tout + t) * p.res_cs + o] + v;
      const long oi = p.chan_major ? ((long)b * p.Cout + o) * p.Tout + t : ((long)b * p.Tout + t) * p.out_cs + p.out_c0 + o;
      if (p.accumulate) v = p.out[oi] + v;
      if (p.div != 0.f) v = v / p.div;
      if (p.out_tanh) v = tanhf(v);
      if (p.out_mask) v *= p.out_mask[(long)b * p.Tout + t];
      p.out[oi] = v;
    }
}

// bf16 variant (HiFi-GAN throughput mode): operands rounded to bf16 when staged, fp32 accumulation on
// v_mfma_f32_32x32x16_bf16; 32-channel chunks = two 16-deep MFMA steps per tap; same tile, epilogue and semantics
template <int KM, int SP>
__global__ __launch_bounds__(256) void c1d_bf16_kernel(C1dParams p) {
  constexpr int KC = 32, LD = KC + 8;   // row of 40 bf16 = 80 bytes: 16-byte aligned fragments
  __shared__ __attribute__((aligned(16))) bf16 s_in[64 + SP][LD];
  __shared__ __attribute__((aligned(16))) bf16 s_w[KM][64][LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int n_qt = (p.Q + 63) / 64;
  const int qt = blockIdx.x % n_qt, b = blockIdx.x / n_qt;
  const int q0 = qt * 64, a0 = blockIdx.y * 64;
  const int pb = (wv & 1) * 32, cb = (wv >> 1) * 32;
  const int K = p.K, span = (K - 1) * p.dil;
  const int lo = span < 0 ? span : 0, NP = 64 + (span < 0 ? -span : span);
  const int start = q0 - p.pad + lo;
  f32x16 acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (int c0 = 0; c0 < p.Cin; c0 += KC) {
    __syncthreads();
    for (int i = tid; i < NP * 4; i += 256) {   // 8-channel groups of the input patch
      const int g = i & 3, pp = i >> 2;
      const int t = start + pp, cg = c0 + 8 * g;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      if (t >= 0 && t < p.T && cg < p.Cin) {
        const float m = p.in_mask ? p.in_mask[(long)b * p.T + t] : 1.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = p.in_chan_major ? p.in[((long)b * p.Cin + cg + e) * p.T + t] : p.in[((long)b * p.T + t) * p.in_cs + cg + e];
          if (p.in_act && x < 0.f) x *= p.in_slope;
          v[e] = x * m;
        }
      }
      *reinterpret_cast<uint4*>(&s_in[pp][8 * g]) = f_to_item(v, bf16());
    }
    for (int i = tid; i < 64 * K * 4; i += 256) {   // weights [o][k][c]: 16-byte groups of 8 input channels
      const int g = i & 3, rest = i >> 2, k = rest % K, o = rest / K;
      uint4 w = make_uint4(0, 0, 0, 0);
      if (a0 + o < p.Cout && c0 + 8 * g < p.Cin)
        w = *reinterpret_cast<const uint4*>(p.wbf + ((long)(a0 + o) * K + k) * p.Cin + c0 + 8 * g);
      *reinterpret_cast<uint4*>(&s_w[k][o][8 * g]) = w;
    }
    __syncthreads();
    for (int k = 0; k < K; ++k) {
      const int row = pb + r + k * p.dil - lo;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(&s_in[row][16 * ks + 8 * hh]);
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(&s_w[k][cb + r][16 * ks + 8 * hh]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
      }
    }
  }
  const int o = a0 + cb + r;
  if (o >= p.Cout) return;
  const float bias = p.bias ? p.bias[o] : 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int q = q0 + pb + acc_row(j, hh);
    if (q >= p.Q) continue;
    const int t = q * p.out_stride + p.out_off;
    if (t < 0 || t >= p.Tout) continue;
    float v = acc[j] + bias;
    if (p.relu) v = fmaxf(v, 0.f);
    v *= drop_scale(p.drop, ((uint64_t)b * p.Tout + t) * p.Cout + o);
    if (p.res) v = p.res[((long)b * p.Tout + t) * p.res_cs + o] + v;
    const long oi = p.chan_major ? ((long)b * p.Cout + o) * p.Tout + t : ((long)b * p.Tout + t) * p.out_cs + p.out_c0 + o;
    if (p.accumulate) v = p.out[oi] + v;
    if (p.div != 0.f) v = v / p.div;
    if (p.out_tanh) v = tanhf(v);
    if (p.out_mask) v *= p.out_mask[(long)b * p.Tout + t];
    p.out[oi] = v;
  }
}

hipError_t launch_c1d(const C1dParams& p, hipStream_t s) {
  const int span = (p.K - 1) * (p.dil < 0 ? -p.dil : p.dil);
  if (p.K < 1 || p.K > C1_KMAX || span > C1_SPAN || p.Q <= 0) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(p.B * ((p.Q + 63) / 64)), (unsigned)((p.Cout + 63) / 64));
  if (p.bf16) {
    if (!p.wbf || p.Cin % 8) return hipErrorInvalidValue;
    if (p.K <= 3 && span <= 10) hipLaunchKernelGGL((c1d_bf16_kernel<3, 10>), grid, dim3(256), 0, s, p);
    else if (p.K <= 7 && span <= 30) hipLaunchKernelGGL((c1d_bf16_kernel<7, 30>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((c1d_bf16_kernel<C1_KMAX, C1_SPAN>), grid, dim3(256), 0, s, p);
    return hipGetLastError();
  }
  if (p.wpk && !p.in_chan_major && p.Cin % 4 == 0 && p.in_cs % 4 == 0 && ((uintptr_t)p.in & 15) == 0 &&
      ((uintptr_t)p.wpk & 15) == 0) {
    // output-channel tile 32 for narrow convs (HiFi-GAN's last stage, conv_post); 64 frames per wave, or 32 when the
    // 64-frame grid leaves most of the last round of workgroups (2 per CU) empty
    const bool narrow = p.Cout <= 32;
    const int ft2 = narrow ? 256 : 128, ct = narrow ? 32 : 64;
    const long n2 = (long)p.B * ((p.Q + ft2 - 1) / ft2) * ((p.Cout + ct - 1) / ct);
    const long n1 = (long)p.B * ((p.Q + ft2 / 2 - 1) / (ft2 / 2)) * ((p.Cout + ct - 1) / ct);
    auto fill = [](long n) { const long slots = 512; return (double)n / (double)(((n + slots - 1) / slots) * slots); };
    const int nb = fill(n1) > fill(n2) + 0.2 ? 1 : 2;
    const dim3 g((unsigned)(p.B * ((p.Q + (nb == 2 ? ft2 : ft2 / 2) - 1) / (nb == 2 ? ft2 : ft2 / 2))),
                 (unsigned)((p.Cout + ct - 1) / ct));
#define C1D_PK_LAUNCH(KM, KC, SP)                                                                               \
  do {                                                                                                      \
    if (narrow) {                                                                                           \
      if (nb == 2) hipLaunchKernelGGL((c1d_pk_kernel<KM, KC, SP, 32, 2>), g, dim3(256), 0, s, p);           \
      else hipLaunchKernelGGL((c1d_pk_kernel<KM, KC, SP, 32, 1>), g, dim3(256), 0, s, p);                   \
    } else {                                                                                                \
      if (nb == 2) hipLaunchKernelGGL((c1d_pk_kernel<KM, KC, SP, 64, 2>), g, dim3(256), 0, s, p);           \
      else hipLaunchKernelGGL((c1d_pk_kernel<KM, KC, SP, 64, 1>), g, dim3(256), 0, s, p);                   \
    }                                                                                                       \
  } while (0)
    if (p.K <= 3 && span <= 10) C1D_PK_LAUNCH(3, 32, 10);
    else if (p.K <= 7 && span <= 30) C1D_PK_LAUNCH(7, 16, 30);
    else if (span <= 50) C1D_PK_LAUNCH(11, 16, 50);
    else C1D_PK_LAUNCH(11, 16, C1_SPAN);
#undef C1D_PK_LAUNCH
    return hipGetLastError();
  }
  if (p.K <= 3 && span <= 10) hipLaunchKernelGGL((c1d_kernel<3, 32, 10>), grid, dim3(256), 0, s, p);
  else if (p.K <= 7 && span <= 30) hipLaunchKernelGGL((c1d_kernel<7, 16, 30>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((c1d_kernel<C1_KMAX, 16, C1_SPAN>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------- LayerNorm
__global__ __launch_bounds__(256) void te_ln_kernel(const float* x, int x_cs, const float* res, int res_cs,
                                                    const float* gamma, const float* beta, long npos, int C, float eps,
                                                    int relu_after, const float* mask, float* out, int out_cs,
                                                    Drop drop) {
  const long pos = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (pos >= npos) return;
  float v[4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = lane + 64 * k;
    v[k] = 0.f;
    if (c < C) {
      v[k] = x[pos * x_cs + c];
      if (res) v[k] = v[k] + res[pos * res_cs + c];
      s += v[k];
    }
  }
  s = wave_sum(s);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (lane + 64 * k < C) q += (v[k] - mean) * (v[k] - mean);
  q = wave_sum(q);
  const float rs = rsqrtf(q / (float)C + eps);
  const float m = mask ? mask[pos] : 1.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = lane + 64 * k;
    if (c >= C) continue;
    float y = (v[k] - mean) * rs * gamma[c] + beta[c];
    if (relu_after) y = fmaxf(y, 0.f);
    y *= drop_scale(drop, (uint64_t)pos * C + c);
    out[pos * out_cs + c] = y * m;
  }
}

hipError_t launch_te_ln(const float* x, int x_cs, const float* res, int res_cs, const float* gamma, const float* beta,
                        long npos, int C, float eps, int relu_after, const float* mask, float* out, int out_cs,
                        hipStream_t s, Drop drop) {
  if (C > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(te_ln_kernel, dim3((unsigned)((npos + 3) / 4)), dim3(256), 0, s, x, x_cs, res, res_cs, gamma, beta,
                     npos, C, eps, relu_after, mask, out, out_cs, drop);
  return hipGetLastError();
}

// ---------------------------------------------------------------- embedding + x_mask (text_encoder.py:322-324)
__global__ void te_embed_kernel(const int64_t* tokens, const int64_t* lengths, const float* emb, int n_vocab, int B,
                                int T, int C, float scale, float* x, float* x_mask) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * T * C) return;
  const long pos = i / C;
  const int c = (int)(i % C);
  const int b = (int)(pos / T), t = (int)(pos % T);
  const int64_t tok = tokens[pos];
  x[i] = (tok >= 0 && tok < n_vocab) ? emb[tok * C + c] * scale : __builtin_nanf("");   // out of range: NaN, no read
  if (c == 0) x_mask[pos] = t < lengths[b] ? 1.f : 0.f;
}

hipError_t launch_te_embed(const int64_t* tokens, const int64_t* lengths, const float* emb, int n_vocab, int B, int T,
                           int C, float scale, float* x, float* x_mask, hipStream_t s) {
  const long n = (long)B * T * C;
  hipLaunchKernelGGL(te_embed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tokens, lengths, emb, n_vocab,
                     B, T, C, scale, x, x_mask);
  return hipGetLastError();
}

// ---------------------------------------------------------------- attention
constexpr int TA_Q = 16, TA_KT = 64, TA_D = 96, TA_WMAX = 17;
__global__ __launch_bounds__(256) void te_attn_kernel(const float* qkv, const float* x_mask, const float* erk,
                                                      const float* erv, int T, int C, int W, float* out) {
  __shared__ float s_q[TA_Q][TA_D + 1], s_k[TA_KT][TA_D + 1], s_v[TA_KT][TA_D];
  __shared__ float s_ek[TA_WMAX][TA_D + 1], s_ev[TA_WMAX][TA_D];
  __shared__ float s_s[TA_Q][TA_KT + 1], s_win[TA_Q][TA_WMAX];
  const int tid = threadIdx.x, i0 = blockIdx.x * TA_Q, h = blockIdx.y, b = blockIdx.z;
  const int row = tid >> 4, g = tid & 15;   // query row of this thread; 6 output dims / 4 keys per thread
  const int i = i0 + row, nw = 2 * W + 1, C3 = 3 * C;
  const float* base = qkv + (long)b * T * C3;
  const float sq = sqrtf((float)TA_D);
  for (int e = tid; e < TA_Q * TA_D; e += 256) {
    const int rr = e / TA_D, d = e % TA_D;
    s_q[rr][d] = i0 + rr < T ? base[(long)(i0 + rr) * C3 + h * TA_D + d] : 0.f;
  }
  for (int e = tid; e < nw * TA_D; e += 256) {
    s_ek[e / TA_D][e % TA_D] = erk[e];
    s_ev[e / TA_D][e % TA_D] = erv[e];
  }
  for (int e = tid; e < TA_Q * TA_WMAX; e += 256) s_win[e / TA_WMAX][e % TA_WMAX] = -INFINITY;
  const float xi = i < T ? x_mask[(long)b * T + i] : 0.f;
  float m = -INFINITY, l = 0.f, o[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < T; j0 += TA_KT) {
    __syncthreads();
    for (int e = tid; e < TA_KT * TA_D; e += 256) {
      const int jj = e / TA_D, d = e % TA_D;
      const bool ok = j0 + jj < T;
      s_k[jj][d] = ok ? base[(long)(j0 + jj) * C3 + C + h * TA_D + d] : 0.f;
      s_v[jj][d] = ok ? base[(long)(j0 + jj) * C3 + 2 * C + h * TA_D + d] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int jj = g * 4 + e, j = j0 + jj;
      float sc = -INFINITY;   // frames past T are not keys
      if (j < T) {
        float dot = 0.f;
        for (int d = 0; d < TA_D; ++d) dot = fmaf(s_q[row][d], s_k[jj][d], dot);
        sc = dot / sq;
        const int rel = j - i;
        if (rel >= -W && rel <= W) {
          float dr = 0.f;
          for (int d = 0; d < TA_D; ++d) dr = fmaf(s_q[row][d], s_ek[rel + W][d], dr);
          sc = sc + dr / sq;
        }
        if (!(xi != 0.f && x_mask[(long)b * T + j] != 0.f)) sc = -1e4f;   // masked_fill(mask == 0, -1e4)
        if (rel >= -W && rel <= W) s_win[row][rel + W] = sc;
      }
      s_s[row][jj] = sc;
    }
    __syncthreads();
    float mt = m;
    for (int jj = 0; jj < TA_KT; ++jj) mt = fmaxf(mt, s_s[row][jj]);
    const float corr = __expf(m - mt);   // m = -inf on the first tile: corr = 0, l = o = 0 anyway
    float lt = 0.f, ot[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int jj = 0; jj < TA_KT; ++jj) {
      const float pj = __expf(s_s[row][jj] - mt);
      lt += pj;
#pragma unroll
      for (int dd = 0; dd < 6; ++dd) ot[dd] = fmaf(pj, s_v[jj][g * 6 + dd], ot[dd]);
    }
    l = l * corr + lt;
#pragma unroll
    for (int dd = 0; dd < 6; ++dd) o[dd] = o[dd] * corr + ot[dd];
    m = mt;
  }
  if (i >= T) return;
  const float il = 1.f / l;
#pragma unroll
  for (int dd = 0; dd < 6; ++dd) o[dd] *= il;
  for (int w = 0; w < nw; ++w) {
    const float sw = s_win[row][w];
    if (sw == -INFINITY) continue;
    const float pw = __expf(sw - m) * il;
#pragma unroll
    for (int dd = 0; dd < 6; ++dd) o[dd] = fmaf(pw, s_ev[w][g * 6 + dd], o[dd]);
  }
#pragma unroll
  for (int dd = 0; dd < 6; ++dd) out[((long)b * T + i) * C + h * TA_D + g * 6 + dd] = o[dd];
}

hipError_t launch_te_attn(const float* qkv, const float* x_mask, const float* erk, const float* erv, int B, int T, int C,
                          int H, int W, float* out, hipStream_t s) {
  if (C != H * TA_D || 2 * W + 1 > TA_WMAX) return hipErrorInvalidValue;
  // erk / erv: [2W + 1][96] per layer (heads share them, text_encoder.py:119-124)
  hipLaunchKernelGGL(te_attn_kernel, dim3((unsigned)((T + TA_Q - 1) / TA_Q), H, B), dim3(256), 0, s, qkv, x_mask, erk, erv,
                     T, C, W, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------- durations, generate_path, mu_y
// per utterance, in frame order: w = exp(logw) m; w_ceil = ceil(w) * length_scale; cum = cumsum(w_ceil);
// y_length = max(1, (long) sum(w_ceil))   (tts.py:86-89, utils.py:29)
__global__ void te_durations_kernel(const float* logw, const float* x_mask, int B, int Tx, float ls, float* w_ceil,
                                    float* cum, int64_t* y_lengths) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  float c = 0.f;
  for (int t = 0; t < Tx; ++t) {
    const long i = (long)b * Tx + t;
    const float w = expf(logw[i]) * x_mask[i];   // accurate exp: ceil() flips on a 1-ulp difference
    const float wc = ceilf(w) * ls;
    w_ceil[i] = wc;
    c += wc;
    cum[i] = c;
  }
  y_lengths[b] = (int64_t)fmaxf(c, 1.f);
}

// per output frame j: the token i* with cum[i*-1] <= j < cum[i*] (generate_path's one nonzero in column j), if
// x_mask[i*] y_mask[j]; mu_y[:, j] = mu_x[:, i*] (the matmul with a 0/1 column is exact), y_mask, attn
__global__ void te_expand_kernel(const float* mu_x, const float* cum, const float* x_mask, const int64_t* y_lengths,
                                 int B, int Tx, int Ty, int F, float* mu_y, float* y_mask, float* attn) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)B * Ty) return;
  const int b = (int)(e / Ty), j = (int)(e % Ty);
  const float* cb = cum + (long)b * Tx;
  const float jf = (float)j;
  int lo = 0, hi = Tx;   // first i with jf < cum[i]
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (jf < cb[mid]) hi = mid; else lo = mid + 1;
  }
  const float ym = j < y_lengths[b] ? 1.f : 0.f;
  y_mask[e] = ym;
  const bool on = lo < Tx && ym != 0.f && x_mask[(long)b * Tx + lo] != 0.f;
  for (int f = 0; f < F; ++f) mu_y[((long)b * F + f) * Ty + j] = on ? mu_x[((long)b * F + f) * Tx + lo] : 0.f;
  if (attn)
    for (int t = 0; t < Tx; ++t) attn[((long)b * Tx + t) * Ty + j] = (on && t == lo) ? 1.f : 0.f;
}

// mu_y[b][f][j] = sum_i attn[b][i][j] mu_x[b][f][i]  (tts.py:233-234, with the MAS path of get_score_model); a 0/1
// monotonic path has at most one nonzero per column, so the sum is that single product (exact)
__global__ __launch_bounds__(256) void te_path_gather_kernel(const float* attn, const float* mu_x, int Tx, int Ty, int F,
                                                             float* mu_y) {
  const int b = blockIdx.y, j = blockIdx.x * 64 + (threadIdx.x & 63), fg = threadIdx.x >> 6;
  if (j >= Ty) return;
  const int f0 = fg * ((F + 3) / 4), f1 = min(F, f0 + (F + 3) / 4);
  float acc[32];
#pragma unroll
  for (int f = 0; f < 32; ++f) acc[f] = 0.f;
  for (int i = 0; i < Tx; ++i) {
    const float a = attn[((long)b * Tx + i) * Ty + j];
    if (a == 0.f) continue;
#pragma unroll
    for (int f = 0; f < 32; ++f)
      if (f0 + f < f1) acc[f] += a * mu_x[((long)b * F + f0 + f) * Tx + i];
  }
#pragma unroll
  for (int f = 0; f < 32; ++f)
    if (f0 + f < f1) mu_y[((long)b * F + f0 + f) * Ty + j] = acc[f];
}

hipError_t launch_te_path_gather(const float* attn, const float* mu_x, int B, int Tx, int Ty, int F, float* mu_y,
                                 hipStream_t s) {
  if ((F + 3) / 4 > 32) return hipErrorInvalidValue;
  hipLaunchKernelGGL(te_path_gather_kernel, dim3((unsigned)((Ty + 63) / 64), B), dim3(256), 0, s, attn, mu_x, Tx, Ty, F,
                     mu_y);
  return hipGetLastError();
}

hipError_t launch_te_durations(const float* logw, const float* x_mask, int B, int Tx, float length_scale, float* w_ceil,
                               float* cum, int64_t* y_lengths, hipStream_t s) {
  hipLaunchKernelGGL(te_durations_kernel, dim3((B + 63) / 64), dim3(64), 0, s, logw, x_mask, B, Tx, length_scale, w_ceil,
                     cum, y_lengths);
  return hipGetLastError();
}

hipError_t launch_te_expand(const float* mu_x, const float* cum, const float* x_mask, const int64_t* y_lengths, int B,
                            int Tx, int Ty, int F, float* mu_y, float* y_mask, float* attn, hipStream_t s) {
  const long n = (long)B * Ty;
  hipLaunchKernelGGL(te_expand_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, mu_x, cum, x_mask, y_lengths, B,
                     Tx, Ty, F, mu_y, y_mask, attn);
  return hipGetLastError();
}

}  // namespace gt
