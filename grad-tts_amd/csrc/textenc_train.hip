// Training pass of GradTTS's text encoder and the encoder-side losses of GradTTS.compute_loss (gfx950, fp32):
//
//   tt_attn_p_kernel      relative-position attention probabilities (text_encoder.py:145-165) with the training
//                         dropout of p_attn (:166); writes P (softmax) and Pd (dropped) for the backward
//   tt_attn_pv_kernel     output = Pd v + relative-value term (:167-172)
//   tt_attn_ds_kernel     backward of the attention core: dPd -> dP (dropout) -> dS (softmax, masked_fill)
//   tt_attn_dqkv_kernel   dq (keys + relative keys), dk, dv from dS / Pd
//   tt_attn_drel_kernel   gradients of emb_rel_k / emb_rel_v (shared by the heads), per-utterance partials
//   tt_ln_bwd_kernel      LayerNorm backward (:11-29) with the ReLU / dropout / mask factors around it and
//                         per-workgroup partial dgamma / dbeta
//   tt_wgrad_kernel       Conv1d weight gradient dW[o][c][k] = sum_t dout[t][o] x[t + k - pad][c] as a GEMM over
//                         positions on v_mfma_f32_32x32x2_f32 (64 x 64 tiles, all taps per staged chunk), position
//                         splits reduced in a fixed order
//   tt_colsum_kernel      bias gradients (channel sums over positions), split + fixed-order reduction
//   tt_emb_bwd_kernel     embedding gradient (:322), per vocabulary row in position order (no atomics)
//   tt_ew_kernel          elementwise gradient factors (mask, dropout, ReLU) and the channel-major -> channels-last
//                         transpose of dmu_x / dlogw
//   tt_path_scatter_kernel  backward of mu_y = attn^T mu_x (tts.py:184-185)
//   tt_aux_loss_kernel    dur_loss (tts.py:155-156, utils.py:42-44) and prior_loss (tts.py:191-192) with their unit
//                         gradients, one workgroup, fixed summation order
// Every reduction has a fixed order: two calls give bit-identical gradients.
#include <math.h>

#include <algorithm>

#include "common.h"
#include "textenc.h"
#include "textenc_train.h"

namespace gt {

constexpr int TT_D = 96, TT_WMAX = 17;

GT_DEV float tt_wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
GT_DEV float tt_wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}
// 256-thread block reductions (every thread gets the result; waves combined in order)
GT_DEV float tt_block_sum(float x, float* red) {
  x = tt_wave_sum(x);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = x;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}
GT_DEV float tt_block_max(float x, float* red) {
  x = tt_wave_max(x);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = x;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

GT_DEV float dot96(const float* s, const float* g) {   // s in LDS, g 16-byte aligned global row
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float d = 0.f;
#pragma unroll 4
  for (int k = 0; k < TT_D / 4; ++k) {
    const float4 v = g4[k];
    d = fmaf(s[4 * k], v.x, d);
    d = fmaf(s[4 * k + 1], v.y, d);
    d = fmaf(s[4 * k + 2], v.z, d);
    d = fmaf(s[4 * k + 3], v.w, d);
  }
  return d;
}

// ---------------------------------------------------------------- attention, forward (training)
// one workgroup per (query i, head h, utterance b); the score row lives in LDS (T <= TT_TMAX)
__global__ __launch_bounds__(256) void tt_attn_p_kernel(const float* qkv, const float* x_mask, const float* erk, int T,
                                                        int C, int W, Drop drop, float* P, float* Pd, float* PdT) {
  __shared__ float s_q[TT_D], s_ek[TT_WMAX * TT_D], s_row[TT_TMAX], s_red[4];
  const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z, H = gridDim.y, tid = threadIdx.x, nw = 2 * W + 1;
  const long C3 = 3L * C;
  const float* base = qkv + (long)b * T * C3;
  for (int e = tid; e < TT_D; e += 256) s_q[e] = base[(long)i * C3 + h * TT_D + e];
  for (int e = tid; e < nw * TT_D; e += 256) s_ek[e] = erk[e];
  __syncthreads();
  const float sq = sqrtf((float)TT_D);
  const bool qi = x_mask[(long)b * T + i] != 0.f;
  float mx = -INFINITY;
  for (int j = tid; j < T; j += 256) {
    float sc = dot96(s_q, base + (long)j * C3 + C + h * TT_D) / sq;
    const int rel = j - i;
    if (rel >= -W && rel <= W) {
      float dr = 0.f;
      for (int d = 0; d < TT_D; ++d) dr = fmaf(s_q[d], s_ek[(rel + W) * TT_D + d], dr);
      sc = sc + dr / sq;
    }
    if (!(qi && x_mask[(long)b * T + j] != 0.f)) sc = -1e4f;   // masked_fill(mask == 0, -1e4)
    s_row[j] = sc;
    mx = fmaxf(mx, sc);
  }
  mx = tt_block_max(mx, s_red);
  float l = 0.f;
  for (int j = tid; j < T; j += 256) {
    const float e = expf(s_row[j] - mx);
    s_row[j] = e;
    l += e;
  }
  l = tt_block_sum(l, s_red);
  const long row = (((long)b * H + h) * T + i) * T;
  for (int j = tid; j < T; j += 256) {
    const float p = s_row[j] / l;
    P[row + j] = p;
    const float pd = p * drop_scale(drop, (uint64_t)(row + j));
    Pd[row + j] = pd;
    PdT[(((long)b * H + h) * T + j) * T + i] = pd;   // transposed copy: the backward's dv reads rows of it
  }
}

// out[b][i][h 96 + d] = sum_j Pd[i][j] v[j][h 96 + d] + sum_{|r| <= W} Pd[i][i + r] erv[r + W][d]
__global__ __launch_bounds__(256) void tt_attn_pv_kernel(const float* qkv, const float* Pd, const float* erv, int T,
                                                         int C, int H, int W, float* out) {
  const int i = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  if (tid >= C) return;
  const int h = tid / TT_D, d = tid % TT_D;
  const long C3 = 3L * C;
  const float* prow = Pd + (((long)b * H + h) * T + i) * T;
  const float* vb = qkv + (long)b * T * C3 + 2 * C + tid;
  float o = 0.f;
#pragma unroll 8
  for (int j = 0; j < T; ++j) o = fmaf(prow[j], vb[(long)j * C3], o);
  for (int r = -W; r <= W; ++r) {
    const int j = i + r;
    if (j >= 0 && j < T) o = fmaf(prow[j], erv[(r + W) * TT_D + d], o);
  }
  out[((long)b * T + i) * C + tid] = o;
}

// ---------------------------------------------------------------- attention, backward
// dPd[j] = g_i . v_j + [|j - i| <= W] g_i . erv[j - i + W]; dP = dPd * drop; dS = P (dP - sum_j P dP), 0 where masked
__global__ __launch_bounds__(256) void tt_attn_ds_kernel(const float* qkv, const float* P, const float* datt,
                                                         const float* x_mask, const float* erv, int T, int C, int W,
                                                         Drop drop, float* dS, float* dST) {
  __shared__ float s_g[TT_D], s_ev[TT_WMAX * TT_D], s_dp[TT_TMAX], s_red[4];
  const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z, H = gridDim.y, tid = threadIdx.x, nw = 2 * W + 1;
  const long C3 = 3L * C;
  const float* base = qkv + (long)b * T * C3;
  for (int e = tid; e < TT_D; e += 256) s_g[e] = datt[((long)b * T + i) * C + h * TT_D + e];
  for (int e = tid; e < nw * TT_D; e += 256) s_ev[e] = erv[e];
  __syncthreads();
  const long row = (((long)b * H + h) * T + i) * T;
  float acc = 0.f;
  for (int j = tid; j < T; j += 256) {
    float dpd = dot96(s_g, base + (long)j * C3 + 2 * C + h * TT_D);
    const int rel = j - i;
    if (rel >= -W && rel <= W) {
      float dr = 0.f;
      for (int d = 0; d < TT_D; ++d) dr = fmaf(s_g[d], s_ev[(rel + W) * TT_D + d], dr);
      dpd += dr;
    }
    const float dp = dpd * drop_scale(drop, (uint64_t)(row + j));
    s_dp[j] = dp;
    acc = fmaf(P[row + j], dp, acc);
  }
  acc = tt_block_sum(acc, s_red);
  const bool qi = x_mask[(long)b * T + i] != 0.f;
  for (int j = tid; j < T; j += 256) {
    float ds = P[row + j] * (s_dp[j] - acc);
    if (!(qi && x_mask[(long)b * T + j] != 0.f)) ds = 0.f;
    dS[row + j] = ds;
    dST[(((long)b * H + h) * T + j) * T + i] = ds;   // transposed copy: dk reads rows of it
  }
}

// position i of utterance b, thread = (h, d): dq_i = (sum_j dS[i][j] k_j + sum_r dS[i][i + r] erk[r]) / sqrt(96),
// dk_i = sum_j dS[j][i] q_j / sqrt(96), dv_i = sum_j Pd[j][i] g_j   -> dqkv [B][T][3C] (q | k | v)
__global__ __launch_bounds__(256) void tt_attn_dqkv_kernel(const float* qkv, const float* PdT, const float* dS,
                                                           const float* dST, const float* datt, const float* erk, int T,
                                                           int C, int H, int W, float* dqkv) {
  const int i = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  if (tid >= C) return;
  const int h = tid / TT_D, d = tid % TT_D;
  const long C3 = 3L * C, hb = ((long)b * H + h) * T * T;
  const float* q = qkv + (long)b * T * C3 + tid;
  const float* g = datt + (long)b * T * C + tid;
  float dq = 0.f, dk = 0.f, dv = 0.f;
  const float* ds_r = dS + hb + (long)i * T;    // row i of dS
  const float* dst_r = dST + hb + (long)i * T;  // column i of dS
  const float* pdt_r = PdT + hb + (long)i * T;  // column i of Pd
#pragma unroll 4
  for (int j = 0; j < T; ++j) {
    dq = fmaf(ds_r[j], q[(long)j * C3 + C], dq);
    dk = fmaf(dst_r[j], q[(long)j * C3], dk);
    dv = fmaf(pdt_r[j], g[(long)j * C], dv);
  }
  for (int r = -W; r <= W; ++r) {
    const int j = i + r;
    if (j >= 0 && j < T) dq = fmaf(dS[hb + (long)i * T + j], erk[(r + W) * TT_D + d], dq);
  }
  const float sq = sqrtf((float)TT_D);
  float* o = dqkv + ((long)b * T + i) * C3 + tid;
  o[0] = dq / sq;
  o[C] = dk / sq;
  o[2 * C] = dv;
}

// per utterance b (grid z), offset r (grid x) and tensor (grid y: 0 = emb_rel_k, 1 = emb_rel_v):
// part[b][y][r][d] = sum_{h, i} dS[h][i][i + r] q[i][h 96 + d] / sqrt(96)   |   Pd[h][i][i + r] g[i][h 96 + d]
__global__ __launch_bounds__(128) void tt_attn_drel_kernel(const float* qkv, const float* Pd, const float* dS,
                                                           const float* datt, int T, int C, int H, int W, float* part) {
  const int r = (int)blockIdx.x - W, which = blockIdx.y, b = blockIdx.z, d = threadIdx.x, nw = 2 * W + 1;
  if (d >= TT_D) return;
  const long C3 = 3L * C;
  const float* M = which ? Pd : dS;
  float acc = 0.f;
  for (int h = 0; h < H; ++h) {
    const long hb = ((long)b * H + h) * T * T;
    const float* v = which ? datt + (long)b * T * C + h * TT_D + d : qkv + (long)b * T * C3 + h * TT_D + d;
    const long vs = which ? C : C3;
    const int i0 = r < 0 ? -r : 0, i1 = r > 0 ? T - r : T;   // rows whose column i + r exists
    const float* md = M + hb + (long)i0 * T + i0 + r;        // the r-th diagonal, stride T + 1
#pragma unroll 8
    for (int i = i0; i < i1; ++i) acc = fmaf(md[(long)(i - i0) * (T + 1)], v[(long)i * vs], acc);
  }
  if (!which) acc = acc / sqrtf((float)TT_D);
  part[(((long)b * 2 + which) * nw + (r + W)) * TT_D + d] = acc;
}

// ---------------------------------------------------------------- LayerNorm backward
constexpr int TT_LN_NPB = 32;   // positions per workgroup (8 per wave)
__global__ __launch_bounds__(256) void tt_ln_bwd_kernel(LnBwdParams p) {
  __shared__ float s_part[4][2][256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, C = p.C;
  const long p0 = (long)blockIdx.x * TT_LN_NPB, p1 = min(p.npos, p0 + TT_LN_NPB);
  float ga[4] = {0.f, 0.f, 0.f, 0.f}, ba[4] = {0.f, 0.f, 0.f, 0.f};
  for (long pos = p0 + wv; pos < p1; pos += 4) {
    float v[4], g[4], xh[4];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = lane + 64 * k;
      v[k] = 0.f;
      if (c < C) {
        v[k] = p.x[pos * p.x_cs + c];
        if (p.res) v[k] = v[k] + p.res[pos * p.res_cs + c];
        s += v[k];
      }
    }
    s = tt_wave_sum(s);
    const float mean = s / (float)C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (lane + 64 * k < C) q += (v[k] - mean) * (v[k] - mean);
    q = tt_wave_sum(q);
    const float rs = rsqrtf(q / (float)C + p.eps);
    const float dm = p.dy_mask ? p.dy_mask[pos] : 1.f;
    float m1 = 0.f, m2 = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = lane + 64 * k;
      g[k] = 0.f;
      xh[k] = 0.f;
      if (c >= C) continue;
      xh[k] = (v[k] - mean) * rs;
      float gy = p.dy[pos * p.dy_cs + c] * dm * drop_scale(p.drop, (uint64_t)pos * C + c);
      if (p.relu_ref && !(p.relu_ref[pos * C + c] > 0.f)) gy = 0.f;
      ga[k] = fmaf(gy, xh[k], ga[k]);
      ba[k] += gy;
      g[k] = gy * p.gamma[c];
      m1 += g[k];
      m2 = fmaf(g[k], xh[k], m2);
    }
    m1 = tt_wave_sum(m1) / (float)C;
    m2 = tt_wave_sum(m2) / (float)C;
    const float xm = p.dx_mask ? p.dx_mask[pos] : 1.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = lane + 64 * k;
      if (c >= C) continue;
      float dx = rs * (g[k] - m1 - xh[k] * m2);
      if (p.post_relu && !(v[k] > 0.f)) dx = 0.f;
      dx *= xm;
      float* o = p.dx + pos * p.dx_cs + c;
      *o = p.dx_accumulate ? *o + dx : dx;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    s_part[wv][0][lane + 64 * k] = ga[k];
    s_part[wv][1][lane + 64 * k] = ba[k];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * C; e += 256) {
    const int w2 = e / C, c = e % C;
    p.part[(long)blockIdx.x * 2 * C + e] =
        ((s_part[0][w2][c] + s_part[1][w2][c]) + s_part[2][w2][c]) + s_part[3][w2][c];
  }
}

// ---------------------------------------------------------------- conv1d weight gradient
template <int KM>
__global__ __launch_bounds__(256) void tt_wgrad_kernel(WgradParams p) {
  __shared__ float s_d[32][65];
  __shared__ float s_x[32 + KM - 1][65];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int o0 = blockIdx.x * 64, c0 = blockIdx.y * 64, split = blockIdx.z;
  const int wo = (wv & 1) * 32, wc = (wv >> 1) * 32, K = p.K;
  const int nct = (p.T + 31) / 32, nch = p.B * nct;
  const int ch0 = (int)((long)split * nch / p.nsplit), ch1 = (int)((long)(split + 1) * nch / p.nsplit);
  f32x16 acc[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[k][j] = 0.f;
  for (int ch = ch0; ch < ch1; ++ch) {
    const int b = ch / nct, t0 = (ch % nct) * 32;
    __syncthreads();
    for (int e = tid; e < 32 * 64; e += 256) {
      const int pp = e >> 6, oo = e & 63, t = t0 + pp;
      s_d[pp][oo] = (t < p.T && o0 + oo < p.Cout) ? p.dout[((long)b * p.T + t) * p.d_cs + o0 + oo] : 0.f;
    }
    for (int e = tid; e < (32 + K - 1) * 64; e += 256) {
      const int pp = e >> 6, cc = e & 63, t = t0 + pp - p.pad;
      float v = 0.f;
      if (t >= 0 && t < p.T && c0 + cc < p.Cin) {
        v = p.x[((long)b * p.T + t) * p.x_cs + c0 + cc];
        if (p.x_mask) v *= p.x_mask[(long)b * p.T + t];
      }
      s_x[pp][cc] = v;
    }
    __syncthreads();
#pragma unroll 4
    for (int s = 0; s < 16; ++s) {
      const int kp = 2 * s + hh;
      const float a = s_d[kp][wo + r];
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k < K) acc[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, s_x[kp + k][wc + r], acc[k], 0, 0, 0);
    }
  }
  const int c = c0 + wc + r;
  if (c >= p.Cin) return;
  float* out = p.out + (long)split * p.Cout * p.Cin * K;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k >= K) break;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int o = o0 + wo + acc_row(j, hh);
      if (o < p.Cout) out[((long)o * p.Cin + c) * K + k] = acc[k][j];
    }
  }
}

// out[c] = sum_pos x[pos][c]: one workgroup per 64 channels, 16 position lanes (strided), combined in lane order
__global__ __launch_bounds__(1024) void tt_colsum_kernel(const float* x, int x_cs, long npos, int C, float* out) {
  __shared__ float s_p[16][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6, c = blockIdx.x * 64 + cl;
  float acc = 0.f;
  if (c < C)
#pragma unroll 4
    for (long pos = g; pos < npos; pos += 16) acc += x[pos * x_cs + c];
  s_p[g][cl] = acc;
  __syncthreads();
  if (g == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += s_p[k][cl];
    out[c] = t;
  }
}

// out[i] = sum_s part[s n + i] in split order
__global__ void tt_sum_splits_kernel(const float* part, int nsplit, long n, float* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float a = 0.f;
  for (int s = 0; s < nsplit; ++s) a += part[(long)s * n + i];
  out[i] = a;
}

// ---------------------------------------------------------------- embedding, elementwise
// part[s][v][c] = scale * sum over split s's positions (in order) with token v of dx0[pos][c]
__global__ __launch_bounds__(256) void tt_emb_bwd_kernel(const int64_t* tokens, long npos, const float* dx0, int C,
                                                         float scale, int nv, float* part) {
  const int v = blockIdx.x, sp = blockIdx.y, ns = gridDim.y, c = threadIdx.x;
  if (c >= C) return;
  const long a = (long)sp * npos / ns, z = (long)(sp + 1) * npos / ns;
  float acc = 0.f;
  for (long pos = a; pos < z; ++pos)
    if (tokens[pos] == v) acc += dx0[pos * C + c];
  part[((long)sp * nv + v) * C + c] = acc * scale;
}

__global__ void tt_ew_kernel(EwParams p) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= p.npos * p.C) return;
  const long pos = e / p.C;
  const int c = (int)(e % p.C);
  float v;
  if (!p.src) {
    v = 0.f;
  } else if (p.src_chan_major) {
    const long b = pos / p.T, t = pos % p.T;
    v = p.src[(b * p.C + c) * p.T + t];
  } else {
    v = p.src[pos * p.src_cs + c];
  }
  if (p.mask) v *= p.mask[pos];
  v *= drop_scale(p.drop, (uint64_t)pos * p.C + c);
  if (p.relu_ref && !(p.relu_ref[pos * p.relu_cs + c] > 0.f)) v = 0.f;
  p.dst[pos * p.dst_cs + c] = v;
}

__global__ void tt_copy_words_kernel(uint32_t* dst, const uint32_t* src, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// ---------------------------------------------------------------- GradTTS.compute_loss glue
// dmu_x[b][f][i] = sum_j attn[b][i][j] dmu_y[b][f][j]   (backward of tts.py:184-185's matmul)
__global__ __launch_bounds__(128) void tt_path_scatter_kernel(const float* attn, const float* dmu_y, int Tx, int Ty,
                                                              int F, float* dmu_x) {
  const int i = blockIdx.x, b = blockIdx.y, f = threadIdx.x;
  if (f >= F) return;
  const float* a = attn + ((long)b * Tx + i) * Ty;
  const float* g = dmu_y + ((long)b * F + f) * Ty;
  float acc = 0.f;
  for (int j = 0; j < Ty; ++j) {
    const float w = a[j];
    if (w != 0.f) acc = fmaf(w, g[j], acc);
  }
  dmu_x[((long)b * F + f) * Tx + i] = acc;
}

// dur_loss (tts.py:155-156, utils.py:42-44) and prior_loss (tts.py:191-192) in four fixed-order passes:
//   tt_dur_kernel        per (b, i): d = logw - log(1e-8 + sum_j attn) x_mask -> dlogw_unit (unscaled), block
//                        partial of d^2 (fp64)
//   tt_prior_kernel      block partials of 0.5 ((y - mu_y)^2 + log 2 pi) y_mask and of y_mask (fp64)
//   tt_aux_final_kernel  out[0] = dur_loss, out[1] = prior_loss, out[2] = 2 / sum x_lengths,
//                        out[3] = 1 / (sum y_mask F)
//   tt_aux_grad_kernel   dlogw_unit *= out[2]; dmu_unit = -(y - mu_y) y_mask out[3]
constexpr int TT_PRIOR_BLOCKS = 256;
GT_DEV double tt_block_sum_d(double x, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}
// one wave per (b, i) row of attn (coalesced; the 0/1 sum is exact in any order), 4 rows per workgroup
__global__ __launch_bounds__(256) void tt_dur_kernel(const float* logw, const float* attn, const float* x_mask,
                                                     long n, int Ta, float* dlogw_unit, double* part) {
  __shared__ double s_sq[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 4 + wv;
  double sq = 0.0;
  if (e < n) {
    const float* a = attn + e * Ta;
    float dur = 0.f;
    for (int j = lane; j < Ta; j += 64) dur += a[j];
    dur = tt_wave_sum(dur);
    const float df = logw[e] - logf(1e-8f + dur) * x_mask[e];
    if (lane == 0) dlogw_unit[e] = df;
    sq = (double)df * df;
  }
  if (lane == 0) s_sq[wv] = sq;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((s_sq[0] + s_sq[1]) + s_sq[2]) + s_sq[3];
}
__global__ __launch_bounds__(256) void tt_prior_kernel(const float* y, const float* mu_y, const float* y_mask, int B,
                                                       int F, int Ty, double* part) {
  __shared__ double s_red[4];
  const long n = (long)B * F * Ty, a = (long)blockIdx.x * n / gridDim.x, z = (long)(blockIdx.x + 1) * n / gridDim.x;
  const long nm = (long)B * Ty, am = (long)blockIdx.x * nm / gridDim.x, zm = (long)(blockIdx.x + 1) * nm / gridDim.x;
  const float l2pi = 1.8378770664093453f;   // log(2 pi)
  double ps = 0.0, ms = 0.0;
  for (long e = a + threadIdx.x; e < z; e += 256) {
    const long b = e / ((long)F * Ty), t = e % Ty;
    const float d = y[e] - mu_y[e];
    ps += (double)(0.5f * (d * d + l2pi) * y_mask[b * Ty + t]);
  }
  for (long e = am + threadIdx.x; e < zm; e += 256) ms += (double)y_mask[e];
  ps = tt_block_sum_d(ps, s_red);
  ms = tt_block_sum_d(ms, s_red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ps;
    part[2 * blockIdx.x + 1] = ms;
  }
}
__global__ __launch_bounds__(256) void tt_aux_final_kernel(const double* dpart, int nd, const double* ppart, int np,
                                                           const int64_t* x_lengths, int B, int F, float* out) {
  __shared__ double s_red[4];
  const int tid = threadIdx.x;
  double ds = 0.0, ps = 0.0, ms = 0.0, ls = 0.0;   // per thread strided, then a fixed-order block reduction
  for (int i = tid; i < nd; i += 256) ds += dpart[i];
  for (int i = tid; i < np; i += 256) { ps += ppart[2 * i]; ms += ppart[2 * i + 1]; }
  for (int b = tid; b < B; b += 256) ls += (double)x_lengths[b];
  ds = tt_block_sum_d(ds, s_red);
  ps = tt_block_sum_d(ps, s_red);
  ms = tt_block_sum_d(ms, s_red);
  ls = tt_block_sum_d(ls, s_red);
  if (tid != 0) return;
  const double pden = ms * F;
  out[0] = (float)(ds / ls);
  out[1] = (float)(ps / pden);
  out[2] = (float)(2.0 / ls);
  out[3] = (float)(1.0 / pden);
}
__global__ void tt_aux_grad_kernel(const float* y, const float* mu_y, const float* y_mask, int B, int F, int Ty, long nx,
                                   const float* out, float* dlogw_unit, float* dmu_unit) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e < nx) dlogw_unit[e] = dlogw_unit[e] * out[2];
  if (e < (long)B * F * Ty) {
    const long b = e / ((long)F * Ty), t = e % Ty;
    dmu_unit[e] = -(y[e] - mu_y[e]) * y_mask[b * Ty + t] * out[3];
  }
}

// ---------------------------------------------------------------- device-side weight repack
// pk[(o K + k) Ci + c] = W[o][c][k] and pkt[(c K + K - 1 - k) O + o] = W[o][c][k] for every conv weight of the table
// (the layouts textenc.cpp's upload() builds on the host), after a device-side parameter update
__global__ void tt_repack_kernel(const float* raw, const RepackEntry* tab, float* pk) {
  const RepackEntry t = tab[blockIdx.y];
  const long n = (long)t.O * t.Ci * t.K;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int k = (int)(i % t.K);
    const long oc = i / t.K;
    const int c = (int)(oc % t.Ci), o = (int)(oc / t.Ci);
    const float v = raw[t.raw_off + i];
    pk[t.pk_off + ((long)o * t.K + k) * t.Ci + c] = v;
    pk[t.pkt_off + ((long)c * t.K + (t.K - 1 - k)) * t.O + o] = v;
  }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_tt_attn_fwd(const float* qkv, const float* x_mask, const float* erk, const float* erv, int B, int T,
                              int C, int H, int W, Drop drop, float* P, float* Pd, float* PdT, float* out,
                              hipStream_t s) {
  if (C != H * TT_D || 2 * W + 1 > TT_WMAX || T > TT_TMAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tt_attn_p_kernel, dim3(T, H, B), dim3(256), 0, s, qkv, x_mask, erk, T, C, W, drop, P, Pd, PdT);
  hipLaunchKernelGGL(tt_attn_pv_kernel, dim3(T, B), dim3(256), 0, s, qkv, Pd, erv, T, C, H, W, out);
  return hipGetLastError();
}

hipError_t launch_tt_attn_bwd(const float* qkv, const float* P, const float* Pd, const float* PdT, const float* datt,
                              const float* x_mask, const float* erk, const float* erv, int B, int T, int C, int H,
                              int W, Drop drop, float* dS, float* dST, float* dqkv, float* drel_part, float* derk_derv,
                              hipStream_t s) {
  if (C != H * TT_D || 2 * W + 1 > TT_WMAX || T > TT_TMAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tt_attn_ds_kernel, dim3(T, H, B), dim3(256), 0, s, qkv, P, datt, x_mask, erv, T, C, W, drop, dS,
                     dST);
  hipLaunchKernelGGL(tt_attn_dqkv_kernel, dim3(T, B), dim3(256), 0, s, qkv, PdT, dS, dST, datt, erk, T, C, H, W, dqkv);
  const int nw = 2 * W + 1;
  hipLaunchKernelGGL(tt_attn_drel_kernel, dim3(nw, 2, B), dim3(128), 0, s, qkv, Pd, dS, datt, T, C, H, W, drel_part);
  // derk_derv = [emb_rel_k grad (nw x 96) | emb_rel_v grad (nw x 96)] summed over utterances in order
  const long n = 2L * nw * TT_D;
  hipLaunchKernelGGL(tt_sum_splits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, drel_part, B, n,
                     derk_derv);
  return hipGetLastError();
}

long tt_ln_bwd_blocks(long npos) { return (npos + TT_LN_NPB - 1) / TT_LN_NPB; }

hipError_t launch_tt_ln_bwd(const LnBwdParams& p, float* dgamma_dbeta, hipStream_t s) {
  if (p.C > 256 || p.npos <= 0) return hipErrorInvalidValue;
  const long nb = tt_ln_bwd_blocks(p.npos);
  hipLaunchKernelGGL(tt_ln_bwd_kernel, dim3((unsigned)nb), dim3(256), 0, s, p);
  const long n = 2L * p.C;
  hipLaunchKernelGGL(tt_sum_splits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p.part, (int)nb, n,
                     dgamma_dbeta);
  return hipGetLastError();
}

int tt_wgrad_splits(const WgradParams& p) {
  const long tiles = (long)((p.Cout + 63) / 64) * ((p.Cin + 63) / 64);
  const long nch = (long)p.B * ((p.T + 31) / 32);
  long ns = (512 + tiles - 1) / tiles;
  ns = std::min(ns, std::max(1L, nch / 2));
  return (int)std::max(1L, ns);
}

hipError_t launch_tt_wgrad(WgradParams p, float* dW, float* partial, long partial_floats, hipStream_t s) {
  if (p.K < 1 || p.K > 5) return hipErrorInvalidValue;
  p.nsplit = tt_wgrad_splits(p);
  const long n = (long)p.Cout * p.Cin * p.K;
  if (p.nsplit > 1 && (long)p.nsplit * n > partial_floats) p.nsplit = (int)std::max(1L, partial_floats / n);
  p.out = p.nsplit > 1 ? partial : dW;
  const dim3 grid((unsigned)((p.Cout + 63) / 64), (unsigned)((p.Cin + 63) / 64), (unsigned)p.nsplit);
  if (p.K == 1) hipLaunchKernelGGL((tt_wgrad_kernel<1>), grid, dim3(256), 0, s, p);
  else if (p.K <= 3) hipLaunchKernelGGL((tt_wgrad_kernel<3>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((tt_wgrad_kernel<5>), grid, dim3(256), 0, s, p);
  if (p.nsplit > 1)
    hipLaunchKernelGGL(tt_sum_splits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, partial, p.nsplit, n,
                       dW);
  return hipGetLastError();
}

hipError_t launch_tt_colsum(const float* x, int x_cs, long npos, int C, float* part, long part_floats, float* out,
                            hipStream_t s) {
  (void)part; (void)part_floats;
  hipLaunchKernelGGL(tt_colsum_kernel, dim3((unsigned)((C + 63) / 64)), dim3(1024), 0, s, x, x_cs, npos, C, out);
  return hipGetLastError();
}

hipError_t launch_tt_emb_bwd(const int64_t* tokens, long npos, const float* dx0, int n_vocab, int C, float scale,
                             float* demb, float* part, long part_floats, hipStream_t s) {
  if (C > 256) return hipErrorInvalidValue;
  const long n = (long)n_vocab * C;
  const int ns = (int)std::max(1L, std::min(std::min(32L, (npos + 127) / 128), part_floats / n));
  if (ns == 1) {   // one position split (short inputs, or a vocabulary whose n_vocab x C exceeds the partials): straight
                   // into demb, as launch_tt_wgrad does -- never more than part_floats into the partials
    hipLaunchKernelGGL(tt_emb_bwd_kernel, dim3(n_vocab, 1), dim3(256), 0, s, tokens, npos, dx0, C, scale, n_vocab, demb);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(tt_emb_bwd_kernel, dim3(n_vocab, ns), dim3(256), 0, s, tokens, npos, dx0, C, scale, n_vocab, part);
  hipLaunchKernelGGL(tt_sum_splits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, ns, n, demb);
  return hipGetLastError();
}

hipError_t launch_tt_ew(const EwParams& p, hipStream_t s) {
  const long n = p.npos * p.C;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(tt_ew_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_tt_copy_words(uint32_t* dst, const uint32_t* src, long n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(tt_copy_words_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}

hipError_t launch_tt_repack(const float* raw, const RepackEntry* tab, int n_entries, float* pk, hipStream_t s) {
  if (n_entries <= 0) return hipSuccess;
  hipLaunchKernelGGL(tt_repack_kernel, dim3(64, n_entries), dim3(256), 0, s, raw, tab, pk);
  return hipGetLastError();
}

hipError_t launch_tt_path_scatter(const float* attn, const float* dmu_y, int B, int Tx, int Ty, int F, float* dmu_x,
                                  hipStream_t s) {
  if (F > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tt_path_scatter_kernel, dim3(Tx, B), dim3(128), 0, s, attn, dmu_y, Tx, Ty, F, dmu_x);
  return hipGetLastError();
}

hipError_t launch_tt_aux_loss(const float* logw, const float* attn, const float* x_mask, const int64_t* x_lengths,
                              const float* y, const float* mu_y, const float* y_mask, int B, int Tx, int Ta, int Ty,
                              int F, float* out, float* dlogw_unit, float* dmu_unit, double* scratch, hipStream_t s) {
  const long nx = (long)B * Tx, ny = (long)B * F * Ty;
  const int nd = (int)((nx + 3) / 4);   // tt_dur_kernel: 4 rows per workgroup
  double* dpart = scratch;
  double* ppart = scratch + nd;
  hipLaunchKernelGGL(tt_dur_kernel, dim3(nd), dim3(256), 0, s, logw, attn, x_mask, nx, Ta, dlogw_unit, dpart);
  hipLaunchKernelGGL(tt_prior_kernel, dim3(TT_PRIOR_BLOCKS), dim3(256), 0, s, y, mu_y, y_mask, B, F, Ty, ppart);
  hipLaunchKernelGGL(tt_aux_final_kernel, dim3(1), dim3(256), 0, s, dpart, nd, ppart, TT_PRIOR_BLOCKS, x_lengths, B, F,
                     out);
  const long ng = std::max(nx, ny);
  hipLaunchKernelGGL(tt_aux_grad_kernel, dim3((unsigned)((ng + 255) / 256)), dim3(256), 0, s, y, mu_y, y_mask, B, F, Ty,
                     nx, out, dlogw_unit, dmu_unit);
  return hipGetLastError();
}

long tt_aux_loss_scratch_doubles(long B, long Tx) { return (B * Tx + 3) / 4 + 2 * TT_PRIOR_BLOCKS; }

}  // namespace gt
