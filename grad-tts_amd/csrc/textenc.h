// Text encoder kernels (textenc.hip): parameter blocks and launchers. fp32, channels-last [B][T][C].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gt {

// Dropout of the training pass (torch.nn.Dropout(p) in train mode): element idx of site `site` is kept iff
// u(seed, site, idx) >= thr, u = the top 24 bits of splitmix64's finaliser over seed + site K1 + idx K2 (our own
// counter-based generator, restated by oracle/text_encoder.py:dropout_keep), and kept elements are scaled by
// 1 / (1 - p). thr = 0: no dropout (p = 0 or eval mode).
struct Drop {
  uint64_t seed;
  uint32_t site, thr;
  float scale;
};
__device__ __forceinline__ float drop_scale(const Drop& d, uint64_t idx) {
  if (d.thr == 0) return 1.f;
  uint64_t x = d.seed + (uint64_t)d.site * 0x9E3779B97F4A7C15ull + idx * 0xD1B54A32D192ED03ull;
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 40) >= d.thr ? d.scale : 0.f;
}
inline Drop make_drop(uint64_t seed, uint32_t site, float p) {
  Drop d{seed, site, 0u, 1.f};
  if (p > 0.f) {
    d.thr = (uint32_t)(p * 16777216.0 + 0.5);
    if (d.thr == 0) d.thr = 1;
    d.scale = (float)(1.0 / (1.0 - (double)p));
  }
  return d;
}

// conv1d on fp32 MFMA, general enough for the text encoder and the HiFi-GAN generator:
//   out[row(q)][o] = epi( sum_{j < K, c} W(o, c, j) act(in[q + j dil - pad][c]) ),  row(q) = q out_stride + out_off
// W(o, c, j) = w[o wso + c wsc + tap0 + j tap_step] (Conv1d [Cout][Cin][K]: wso = Cin K, wsc = K, tap0 = 0,
// tap_step = 1; one phase r of ConvTranspose1d [Cin][Cout][k]: wso = k, wsc = Cout k, tap0 = r, tap_step = u,
// dil = -1). act = identity or leaky ReLU(in_slope) (* in_mask). epi: + bias, ReLU, + res, out (+)= ..., / div,
// tanh, * out_mask.
struct C1dParams {
  const float* in; int in_cs;          // input [B][Tin][in_cs] channels [0, Cin) (in_chan_major: [B][Cin][Tin])
  int in_chan_major;
  const float* in_mask;                // multiply the input by mask[b][t] (null: no mask)
  int in_act; float in_slope;          // 1: leaky ReLU with in_slope
  const float* w; const float* bias;
  long wso, wsc; int tap0, tap_step;
  int B, T, Cin, Cout, K, pad, dil;    // T = input frames; q runs over [0, Q)
  int Q, Tout, out_stride, out_off;    // output frames Tout; rows outside [0, Tout) are skipped
  float* out; int out_cs, out_c0;      // channels-last output, or channel-major [B][Cout][Tout] if chan_major
  int chan_major, relu;
  const float* res; int res_cs;        // out = res + conv (after bias / ReLU)
  int accumulate;                      // out = out + (...)
  float div;                           // 0: none; else out = (...) / div
  int out_tanh;
  const float* out_mask;
  const uint16_t* wbf;                 // bf16 mode: weights [Cout][K][Cin] bf16 (Cin % 8 == 0); operands rounded to
  int bf16;                            // bf16 at staging, fp32 accumulation (v_mfma_f32_32x32x16_bf16)
  const float* wpk;                    // fp32 weights packed [Cout][K][Cin] (Cin % 4 == 0): with a channels-last input
                                       // (in_cs % 4 == 0) the packed kernel runs (float4 staging, register prefetch)
  Drop drop;                           // training dropout after the ReLU (element index (b Tout + t) Cout + o)
};
// Conv1d defaults (wso = Cin K, wsc = K, tap_step = 1, dil = 1, Q = Tout = T, out_stride = 1)
C1dParams c1d_defaults();
hipError_t launch_c1d(const C1dParams& p, hipStream_t s);

// LayerNorm over channels (text_encoder.py:11-29): out = LN(x (+ res)) * gamma + beta, then ReLU, then dropout,
// then * mask
hipError_t launch_te_ln(const float* x, int x_cs, const float* res, int res_cs, const float* gamma, const float* beta,
                        long npos, int C, float eps, int relu_after, const float* mask, float* out, int out_cs,
                        hipStream_t s, Drop drop = Drop{0, 0, 0, 1.f});

// tokens outside [0, n_vocab) embed as NaN (the reference raises an index error) instead of reading out of range
hipError_t launch_te_embed(const int64_t* tokens, const int64_t* lengths, const float* emb, int n_vocab, int B, int T,
                           int C, float scale, float* x, float* x_mask, hipStream_t s);

// relative-position multi-head self-attention core (text_encoder.py:145-174), head dim 96, window <= 8:
// qkv [B][T][3C] (q | k | v), out [B][T][C]
hipError_t launch_te_attn(const float* qkv, const float* x_mask, const float* erk, const float* erv, int B, int T, int C,
                          int H, int W, float* out, hipStream_t s);

// GradTTS.forward front-end (tts.py:86-101)
hipError_t launch_te_durations(const float* logw, const float* x_mask, int B, int Tx, float length_scale, float* w_ceil,
                               float* cum, int64_t* y_lengths, hipStream_t s);
hipError_t launch_te_expand(const float* mu_x, const float* cum, const float* x_mask, const int64_t* y_lengths, int B,
                            int Tx, int Ty, int F, float* mu_y, float* y_mask, float* attn, hipStream_t s);

// mu_y = attn^T mu_x for a 0/1 alignment attn [B][Tx][Ty] (GradTTS.get_score_model, tts.py:233-234)
hipError_t launch_te_path_gather(const float* attn, const float* mu_x, int B, int Tx, int Ty, int F, float* mu_y,
                                 hipStream_t s);

}  // namespace gt
