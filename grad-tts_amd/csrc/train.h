// Training-path forward kernels (train.hip): parameter blocks and launchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gt {

struct FwdDiffParams {
  const float* x0; const float* mu; const float* z; const float* mask; const float* t;   // [B][F][T], mask [B][T], t [B]
  int B, F, T;
  float beta_min, half_delta;        // half_delta = fp32(0.5 * (beta_max - beta_min)) as torch rounds the scalar
  float* xt; float* zm;              // outputs: x_t * mask, z * mask (zm may be null)
};
struct LossParams {
  const float* score; const float* z; const float* mask; const float* t;
  int B, F, T;
  float beta_min, half_delta;
  float* part;                       // 2 floats per partial block (loss_blocks)
};

// likelihood drift / divergence (train.hip)
struct LikParams {
  const float* xm; const float* mu; const float* mask; const float* eps; const float* score; const float* u;
  const float* t; int B, T;
  float beta_min, delta;             // delta = fp32(beta_max - beta_min)
  float* drift; float* part;         // part: B * lik_blocks(T) floats
};
int lik_blocks(int T);
hipError_t launch_lik_prep(const float* x, const float* mask, const float* eps, int B, int T, float* xm, float* v,
                           hipStream_t s);
hipError_t launch_lik_drift_div(const LikParams& p, float* div, hipStream_t s);
hipError_t launch_lik_init(const float* data, const float* mask, int B, int T, double* y, double* logp, hipStream_t s);
hipError_t launch_lik_cast(const double* y, long n, float* x, float* tbuf, int B, float tval, hipStream_t s);
hipError_t launch_lik_step(double* y, const float* drift, long n, double h, double* logp, const float* div, int B,
                           hipStream_t s);
hipError_t launch_lik_out(const double* y, long n, const double* logp, int B, float* z, float* dlogp, hipStream_t s);

hipError_t launch_log_prior(const float* mu_x, const float* y, const float* x_mask, const float* y_mask, int B, int F,
                            int Tx, int Ty, float cst, float* out, hipStream_t s);
hipError_t launch_mask_len(const float* x_mask, const float* y_mask, int B, int Tx, int Ty, int32_t* t_xs,
                           int32_t* t_ys, hipStream_t s);
hipError_t launch_fwd_diffusion(const FwdDiffParams& p, hipStream_t s);
int loss_blocks(long n);
hipError_t launch_loss(const LossParams& p, float* loss, hipStream_t s);

}  // namespace gt
