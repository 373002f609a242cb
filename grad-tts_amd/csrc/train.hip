// Training-path forward of the decoder and the alignment step of GradTTS.compute_loss (gfx950).
//
//   log_prior_kernel       the log-prior GradTTS.compute_loss aligns with MAS (model/tts.py:143-149): three
//                          fp32 contractions over the 80 mel channels plus a constant, masked with
//                          x_mask (x) y_mask (tts.py:141, the `value * mask` of monotonic_align/__init__.py:13)
//   mask_len_kernel        t_x / t_y of maximum_path (__init__.py:20-21) from the two sequence masks
//   fwd_diffusion_kernel   Diffusion.forward_diffusion (model/diffusion.py:244-252) with the noise passed in
//   loss_partial_kernel /  Diffusion.loss_t's reduction (diffusion.py:279-280): sum((s * sqrt(1 - e^-cum) + z)^2)
//   loss_final_kernel      / (sum(mask) * n_feats), two fixed-order levels (deterministic)
//
// Layouts are the reference's: mu_x [B][F][Tx], y / x0 / mu / z [B][F][T], masks [B][T] (0/1), output
// log-prior [B][Tx][Ty] fp32. Bound: HBM (every kernel streams its operands once; the log-prior contraction is
// 2*F FLOP per output against 4 B written).
#include <algorithm>

#include "common.h"
#include "gradtts.h"
#include "train.h"

namespace gt {

// 64 x 64 (x, t) output tile per 256-thread workgroup; mu_x / y columns of the tile staged in LDS over all F
// channels (F <= 128); thread (tx, ty) computes a 4 x 4 register tile. Per output, in the reference's order of
// terms: ((y_square - y_mu_double) + mu_square) + const, each sum over f ascending in fp32.
constexpr int LP_T = 64, LP_FMAX = 128;
__global__ __launch_bounds__(256) void log_prior_kernel(const float* __restrict__ mu_x, const float* __restrict__ y,
                                                        const float* __restrict__ x_mask, const float* __restrict__ y_mask,
                                                        int F, int Tx, int Ty, float cst, float* __restrict__ out) {
  __shared__ float s_mu[LP_FMAX][LP_T + 1], s_y[LP_FMAX][LP_T + 1];
  const int b = blockIdx.z, x0 = blockIdx.y * LP_T, t0 = blockIdx.x * LP_T, tid = threadIdx.x;
  const float* mub = mu_x + (long)b * F * Tx;
  const float* yb = y + (long)b * F * Ty;
  for (int i = tid; i < F * LP_T; i += 256) {
    const int f = i / LP_T, c = i % LP_T;
    s_mu[f][c] = x0 + c < Tx ? mub[(long)f * Tx + x0 + c] : 0.f;
    s_y[f][c] = t0 + c < Ty ? yb[(long)f * Ty + t0 + c] : 0.f;
  }
  __syncthreads();
  const int tx = tid / 16, ty = tid % 16;   // rows x0 + tx + 16 i, columns t0 + ty + 16 j
  float ymu[4][4] = {}, ysq[4] = {}, musq[4] = {};
  for (int f = 0; f < F; ++f) {
    float m[4], v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { m[i] = s_mu[f][tx + 16 * i]; v[i] = s_y[f][ty + 16 * i]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      musq[i] = __fadd_rn(musq[i], __fmul_rn(-0.5f, __fmul_rn(m[i], m[i])));   // sum(factor * mu^2)  (:147)
      ysq[i] = __fadd_rn(ysq[i], __fmul_rn(-0.5f, __fmul_rn(v[i], v[i])));     // factor^T @ y^2     (:145)
#pragma unroll
      for (int j = 0; j < 4; ++j) ymu[i][j] = __fadd_rn(ymu[i][j], __fmul_rn(-m[i], v[j]));   // (2 factor mu)^T @ y (:146)
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int x = x0 + tx + 16 * i;
    if (x >= Tx) continue;
    const float xm = x_mask ? x_mask[(long)b * Tx + x] : 1.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = t0 + ty + 16 * j;
      if (t >= Ty) continue;
      float lp = __fadd_rn(__fadd_rn(__fsub_rn(ysq[j], ymu[i][j]), musq[i]), cst);   // (:148)
      if (x_mask) lp = lp * (xm * y_mask[(long)b * Ty + t]);
      out[((long)b * Tx + x) * Ty + t] = lp;
    }
  }
}

// t_x = sum_x x_mask[b, x], t_y = sum_t y_mask[b, t] (fp32 sums truncated to int32, as numpy's astype does)
__global__ __launch_bounds__(64) void mask_len_kernel(const float* x_mask, const float* y_mask, int Tx, int Ty,
                                                      int32_t* t_xs, int32_t* t_ys) {
  const int b = blockIdx.x, lane = threadIdx.x;
  float sx = 0.f, sy = 0.f;
  for (int i = lane; i < Tx; i += 64) sx += x_mask[(long)b * Tx + i];
  for (int i = lane; i < Ty; i += 64) sy += y_mask[(long)b * Ty + i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { sx += __shfl_xor(sx, o); sy += __shfl_xor(sy, o); }
  if (lane == 0) { t_xs[b] = (int32_t)sx; t_ys[b] = (int32_t)sy; }
}

// cum_noise = beta_min t + (0.5 (beta_max - beta_min)) t^2 in fp32 (get_noise, diffusion.py:219-224)
GT_DEV float cum_noise(float t, float bmin, float half_delta) {
  return __fadd_rn(__fmul_rn(bmin, t), __fmul_rn(half_delta, __fmul_rn(t, t)));
}

__global__ __launch_bounds__(256) void fwd_diffusion_kernel(FwdDiffParams p) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long n = (long)p.B * p.F * p.T;
  if (i >= n) return;
  const int b = (int)(i / ((long)p.F * p.T)), t = (int)(i % p.T);
  const float cum = cum_noise(p.t[b], p.beta_min, p.half_delta);
  const float e = expf(__fmul_rn(-0.5f, cum));
  const float mean = __fadd_rn(__fmul_rn(p.x0[i], e), __fmul_rn(p.mu[i], __fsub_rn(1.f, e)));   // (:247)
  const float var = __fsub_rn(1.f, expf(-cum));                                                  // (:248)
  const float m = p.mask[(long)b * p.T + t];
  p.xt[i] = __fmul_rn(__fadd_rn(mean, __fmul_rn(p.z[i], sqrtf(var))), m);                      // (:251-252)
  if (p.zm) p.zm[i] = __fmul_rn(p.z[i], m);
}

// per block of 256 x 8 elements: sum of (s sqrt(1 - e^-cum) + z m)^2 (fixed order: thread items ascending, then a
// fixed butterfly over the wave, then the 4 waves in order); mask sums likewise
__global__ __launch_bounds__(256) void loss_partial_kernel(LossParams p) {
  __shared__ float s_w[2][4];
  const int tid = threadIdx.x;
  const long n = (long)p.B * p.F * p.T;
  float acc = 0.f;
  for (int k = 0; k < 8; ++k) {
    const long i = ((long)blockIdx.x * 8 + k) * 256 + tid;
    if (i < n) {
      const int b = (int)(i / ((long)p.F * p.T)), t = (int)(i % p.T);
      const float cum = cum_noise(p.t[b], p.beta_min, p.half_delta);
      const float ne = __fmul_rn(p.score[i], sqrtf(__fsub_rn(1.f, expf(-cum))));   // (:278)
      const float d = __fadd_rn(ne, __fmul_rn(p.z[i], p.mask[(long)b * p.T + t]));
      acc = __fadd_rn(acc, __fmul_rn(d, d));
    }
  }
  float ms = 0.f;   // mask elements of this block's share of [B][T]
  const long nm = (long)p.B * p.T;
  for (long i = (long)blockIdx.x * 256 + tid; i < nm; i += (long)gridDim.x * 256) ms = __fadd_rn(ms, p.mask[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { acc += __shfl_xor(acc, o); ms += __shfl_xor(ms, o); }
  if ((tid & 63) == 0) { s_w[0][tid >> 6] = acc; s_w[1][tid >> 6] = ms; }
  __syncthreads();
  if (tid == 0) {
    p.part[2 * blockIdx.x] = ((s_w[0][0] + s_w[0][1]) + s_w[0][2]) + s_w[0][3];
    p.part[2 * blockIdx.x + 1] = ((s_w[1][0] + s_w[1][1]) + s_w[1][2]) + s_w[1][3];
  }
}

__global__ __launch_bounds__(256) void loss_final_kernel(const float* part, int nblk, int F, float* loss) {
  __shared__ double s[2][256];
  const int tid = threadIdx.x;
  double a = 0.0, m = 0.0;
  for (int i = tid; i < nblk; i += 256) { a += (double)part[2 * i]; m += (double)part[2 * i + 1]; }
  s[0][tid] = a; s[1][tid] = m;
  __syncthreads();
  if (tid == 0) {
    double A = 0.0, M = 0.0;
    for (int i = 0; i < 256; ++i) { A += s[0][i]; M += s[1][i]; }
    loss[0] = (float)(A / (M * (double)F));   // (:280)
  }
}

// ---------------------------------------------------------------- likelihood (n_best/likelihood, §8 f3)
// Probability-flow drift of SPEECHSDE and its Hutchinson divergence (likelihood.py:27-38, 61-68;
// sde_lib.py:278-282, reverse :93-100): with x1 = x m, beta = beta_0 + t (beta_1 - beta_0), g2 = sqrt(beta)^2,
//   drift = (0.5 beta (mu - x1) - g2 s(x1) 0.5) m
//   div   = sum eps . d(sum drift . eps)/dx = sum eps m (-0.5 beta m eps - 0.5 g2 u),  u = J_s(x1)^T (m eps)
GT_DEV float lik_beta(float t, float bmin, float delta) { return __fadd_rn(bmin, __fmul_rn(t, delta)); }

__global__ void lik_prep_kernel(const float* x, const float* mask, const float* eps, int B, int T, float* xm, float* v) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * 80 * T) return;
  const float m = mask[(i / (80L * T)) * T + i % T];
  xm[i] = __fmul_rn(x[i], m);
  v[i] = __fmul_rn(eps[i], m);
}

// grid (nblk, B): drift per element; part[b][blk] = this block's sum of eps m (-0.5 beta m eps - 0.5 g2 u)
__global__ __launch_bounds__(256) void lik_partial_kernel(LikParams p) {
  __shared__ float s_w[4];
  const int b = blockIdx.y, tid = threadIdx.x;
  const long n = 80L * p.T, base = (long)b * n;
  const float tb = p.t[b];
  const float beta = lik_beta(tb, p.beta_min, p.delta);
  const float sq = sqrtf(beta), g2 = __fmul_rn(sq, sq), hb = __fmul_rn(0.5f, beta);
  float acc = 0.f;
  for (int k = 0; k < 4; ++k) {
    const long j = ((long)blockIdx.x * 4 + k) * 256 + tid;
    if (j >= n) continue;
    const long i = base + j;
    const float m = p.mask[(long)b * p.T + j % p.T];
    const float x1 = p.xm[i], e = p.eps[i];
    const float d = __fsub_rn(__fmul_rn(hb, __fsub_rn(p.mu[i], x1)), __fmul_rn(__fmul_rn(g2, p.score[i]), 0.5f));
    p.drift[i] = __fmul_rn(d, m);
    const float gr = __fmul_rn(m, __fsub_rn(__fmul_rn(-hb, __fmul_rn(m, e)), __fmul_rn(__fmul_rn(0.5f, g2), p.u[i])));
    acc = __fadd_rn(acc, __fmul_rn(gr, e));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((tid & 63) == 0) s_w[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) p.part[(long)b * gridDim.x + blockIdx.x] = ((s_w[0] + s_w[1]) + s_w[2]) + s_w[3];
}

__global__ void lik_final_kernel(const float* part, int nblk, int B, float* div) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  double a = 0.0;
  for (int i = 0; i < nblk; ++i) a += (double)part[(long)b * nblk + i];
  div[b] = (float)a;
}

int lik_blocks(int T) { return (int)((80L * T + 1023) / 1024); }

hipError_t launch_lik_prep(const float* x, const float* mask, const float* eps, int B, int T, float* xm, float* v,
                           hipStream_t s) {
  const long n = (long)B * 80 * T;
  hipLaunchKernelGGL(lik_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, mask, eps, B, T, xm, v);
  return hipGetLastError();
}

hipError_t launch_lik_drift_div(const LikParams& p, float* div, hipStream_t s) {
  const int nblk = lik_blocks(p.T);
  hipLaunchKernelGGL(lik_partial_kernel, dim3(nblk, p.B), dim3(256), 0, s, p);
  hipLaunchKernelGGL(lik_final_kernel, dim3((p.B + 63) / 64), dim3(64), 0, s, p.part, nblk, p.B, div);
  return hipGetLastError();
}

// Euler integration state (likelihood.py:99-107): fp64 as the reference's numpy state, cast to fp32 per evaluation
__global__ void lik_init_kernel(const float* data, const float* mask, int B, int T, double* y, double* logp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < B) logp[i] = 0.0;
  if (i >= (long)B * 80 * T) return;
  y[i] = (double)__fmul_rn(data[i], mask[(i / (80L * T)) * T + i % T]);
}
__global__ void lik_cast_kernel(const double* y, long n, float* x, float* tbuf, int B, float tval) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < B) tbuf[i] = tval;
  if (i < n) x[i] = (float)y[i];
}
__global__ void lik_step_kernel(double* y, const float* drift, long n, double h, double* logp, const float* div, int B) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = y[i] + (double)drift[i] * h;
  if (i < B) logp[i] = logp[i] + (double)div[i] * h;
}
__global__ void lik_out_kernel(const double* y, long n, const double* logp, int B, float* z, float* dlogp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) z[i] = (float)y[i];
  if (i < B) dlogp[i] = (float)logp[i];
}

static dim3 lik_grid(long n, int B) { return dim3((unsigned)((std::max<long>(n, B) + 255) / 256)); }
hipError_t launch_lik_init(const float* data, const float* mask, int B, int T, double* y, double* logp, hipStream_t s) {
  hipLaunchKernelGGL(lik_init_kernel, lik_grid((long)B * 80 * T, B), dim3(256), 0, s, data, mask, B, T, y, logp);
  return hipGetLastError();
}
hipError_t launch_lik_cast(const double* y, long n, float* x, float* tbuf, int B, float tval, hipStream_t s) {
  hipLaunchKernelGGL(lik_cast_kernel, lik_grid(n, B), dim3(256), 0, s, y, n, x, tbuf, B, tval);
  return hipGetLastError();
}
hipError_t launch_lik_step(double* y, const float* drift, long n, double h, double* logp, const float* div, int B,
                           hipStream_t s) {
  hipLaunchKernelGGL(lik_step_kernel, lik_grid(n, B), dim3(256), 0, s, y, drift, n, h, logp, div, B);
  return hipGetLastError();
}
hipError_t launch_lik_out(const double* y, long n, const double* logp, int B, float* z, float* dlogp, hipStream_t s) {
  hipLaunchKernelGGL(lik_out_kernel, lik_grid(n, B), dim3(256), 0, s, y, n, logp, B, z, dlogp);
  return hipGetLastError();
}

hipError_t launch_log_prior(const float* mu_x, const float* y, const float* x_mask, const float* y_mask, int B, int F,
                            int Tx, int Ty, float cst, float* out, hipStream_t s) {
  if (F > LP_FMAX) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((Ty + LP_T - 1) / LP_T), (unsigned)((Tx + LP_T - 1) / LP_T), (unsigned)B);
  hipLaunchKernelGGL(log_prior_kernel, grid, dim3(256), 0, s, mu_x, y, x_mask, y_mask, F, Tx, Ty, cst, out);
  return hipGetLastError();
}

hipError_t launch_mask_len(const float* x_mask, const float* y_mask, int B, int Tx, int Ty, int32_t* t_xs, int32_t* t_ys,
                           hipStream_t s) {
  hipLaunchKernelGGL(mask_len_kernel, dim3(B), dim3(64), 0, s, x_mask, y_mask, Tx, Ty, t_xs, t_ys);
  return hipGetLastError();
}

hipError_t launch_fwd_diffusion(const FwdDiffParams& p, hipStream_t s) {
  const long n = (long)p.B * p.F * p.T;
  hipLaunchKernelGGL(fwd_diffusion_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

int loss_blocks(long n) { return (int)((n + 256 * 8 - 1) / (256 * 8)); }

hipError_t launch_loss(const LossParams& p, float* loss, hipStream_t s) {
  const int nblk = loss_blocks((long)p.B * p.F * p.T);
  hipLaunchKernelGGL(loss_partial_kernel, dim3(nblk), dim3(256), 0, s, p);
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, s, p.part, nblk, p.F, loss);
  return hipGetLastError();
}

}  // namespace gt
