// Small fused kernels of the Grad-TTS decoder step (gfx950).
//   final_kernel          final_block GN-apply + Mish + mask, final_conv 1x1 (64->1), mask, and either
//                         the score output (GradLogPEstimator2d.forward, diffusion.py:212-216) or the
//                         Euler update of Diffusion.reverse_diffusion (diffusion.py:264-267) in place.
//   gn_mish_kernel        ResnetBlock output with identity residual: Mish(GN(h2))*m + x*m (diffusion.py:77-79),
//                         with the first block's res_conv over the 2-3 U-Net input channels (mu, x_t, spk:
//                         diffusion.py:70, 78, 181-184) as 2-3 FMAs per element, or block2's input
//                         (Mish(GN(h1))*m + t_emb)*m applied once in place (wide levels)
//   temb_kernel           SinusoidalPosEmb -> time MLP -> every ResnetBlock's Mish+Linear time bias
//                         (diffusion.py:113-125, 143-144, 64-65, 76); one row per Euler step.
//   spk_mlp_kernel        spk_mlp (diffusion.py:139-141, 175-176)
//   mask_copy_kernel      x_T = z * mask (diffusion.py:257)
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace gt {

template <class A>
__global__ __launch_bounds__(256) void final_kernel(FinalParams p) {
  __shared__ float s_sc[64], s_sh[64], s_w[64], s_mean[8], s_rstd[8];
  __shared__ double s_red[272];
  const int b = blockIdx.y, tid = threadIdx.x;
  constexpr int ICH = Act<A>::kItemCh;
  const int npos = 80 * p.T;
  // this thread's position: pre-activation, mask, x_t and mu loads go out before the GroupNorm reduction
  const int idx = blockIdx.x * 256 + tid;                    // position within [80][T]
  const bool live = idx < npos;
  const long o = (long)b * npos + idx;
  uint4 u[64 / ICH];
  float m = 0.f, x = 0.f, mu = 0.f;
  if (live) {
    const A* pre = reinterpret_cast<const A*>(p.pre) + o * 64;
#pragma unroll
    for (int it = 0; it < 64 / ICH; ++it) u[it] = reinterpret_cast<const uint4*>(pre)[it];
    m = p.mask[(long)b * p.T + idx % p.T];
    if (p.euler) { x = p.xt[o]; mu = p.mu[o]; }
  }
  gn_reduce(p.part, p.nparts, b, p.count, s_mean, s_rstd, s_red);
  constexpr bool L2 = sizeof(A) == 2;   // bf16: the base-2 Mish of gn_mish_tb_l2 with the final_conv weight folded in
  if (tid < 64) {
    float sc, sh;
    gn_affine(s_mean, s_rstd, 64, tid, p.gamma, p.beta, sc, sh);
    s_sc[tid] = L2 ? sc * kLog2e : sc; s_sh[tid] = L2 ? sh * kLog2e : sh; s_w[tid] = L2 ? p.wf[tid] * kLn2 : p.wf[tid];
  }
  __syncthreads();
  {
    if (!live) return;
    // final_conv(y * m) with y = Mish(GN(h)) * m (final_block, Block: * mask): the mask is constant over the channels,
    // so acc = sum_c w_c Mish(GN(h))_c and the output is (acc m^2 + b) m (diffusion.py:215-216)
    float acc = 0.f;
#pragma unroll
    for (int it = 0; it < 64 / ICH; ++it) {
      float v[ICH];
      item_to_f(u[it], v, A());
#pragma unroll
      for (int k = 0; k < ICH; ++k) {
        const int c = it * ICH + k;
        if (L2) {   // w Mish(y) = (w ln2) yl (1 - 2 / ((1 + 2^yl)^2 + 1)), yl = log2(e) y
          const float yl = __builtin_fmaf(v[k], s_sc[c], s_sh[c]);
          const float t = __builtin_amdgcn_exp2f(yl) + 1.f;
          const float g = __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(__builtin_fmaf(t, t, 1.f)), 1.f);
          acc = __builtin_fmaf(yl * s_w[c], g, acc);
        } else {
          acc += s_w[c] * mish_act<A>(v[k] * s_sc[c] + s_sh[c]);
        }
      }
    }
    const float s = (acc * (m * m) + p.bf[0]) * m;             // (output * mask).squeeze(1)
    if (!p.euler) {
      p.out[o] = s;
    } else {
      float dxt = 0.5f * ((mu - x) - s);
      dxt = dxt * (p.betas ? p.betas[*p.stepp] : p.beta_t);
      dxt = dxt * p.hstep;
      p.xt[o] = (x - dxt) * m;
    }
  }
}

// 8 x 16-B items per thread; the block stride (256 items) is a multiple of C, so every thread keeps one
// channel group (and its GroupNorm scale/shift) for all of its items.
// ResnetBlock output, out = Mish(GN(pre))*m + x*m (diffusion.py:57-58, 77-79).
constexpr int RB_IPT = 8;   // items per thread (4 / 16 measured no faster, round 3)
// RES = 1: the residual is res_conv(x*m) over the U-Net input channels (p.mu, p.xt, p.spk_s; level 0) instead of x*m
template <class A, int RES = 0>
__global__ __launch_bounds__(256) void gn_mish_kernel(RbOutParams p) {
  __shared__ float s_mean[8], s_rstd[8];
  __shared__ double s_red[272];
  const int b = blockIdx.y, tid = threadIdx.x;
  constexpr int ICH = Act<A>::kItemCh;
  const int total = p.F * p.T * p.C;                       // elements of one utterance
  const int e0 = (blockIdx.x * RB_IPT * 256 + tid) * ICH;
  const int c0 = e0 % p.C;
  const long ub = (long)b * total;
  const A* pre = reinterpret_cast<const A*>(p.pre) + ub;
  const A* xin = reinterpret_cast<const A*>(RES ? p.pre : p.x) + ub;
  A* out = reinterpret_cast<A*>(p.out) + ub;
  // Data and mask loads go out first; the GroupNorm reduction (its own loads + LDS barriers) overlaps them.
  // Item i is position pos0 + i * pstep (C divides the 256-item block stride): frame index by increments.
  const int pstep = 256 * ICH / p.C;
  int t = (e0 / p.C) % p.T;
  uint4 vp[RB_IPT], vx[RB_IPT];
  float mk[RB_IPT], xr[RES ? RB_IPT : 1][3];
#pragma unroll
  for (int i = 0; i < RB_IPT; ++i) {
    const int e = e0 + i * 256 * ICH;
    if (e < total) {
      vp[i] = *reinterpret_cast<const uint4*>(pre + e);
      if (!RES) vx[i] = *reinterpret_cast<const uint4*>(xin + e);
      mk[i] = mask_at(p.mask, p.T0, b, t, p.lvl);
      if (RES) {   // input channels of this position ([B][F][T] fp32 sampler state; spk projected per mel row)
        const int f = e / p.C / p.T;
        const long q = ((long)b * p.F + f) * p.T + t;
        xr[i][0] = p.mu[q];
        xr[i][1] = p.xt[q];
        xr[i][2] = p.cin == 3 ? p.spk_s[(long)b * p.F + f] : 0.f;
      }
    }
    t += pstep;
    while (t >= p.T) t -= p.T;
  }
  float rw[RES ? ICH : 1][3], rbias[RES ? ICH : 1];
  if (RES) {
#pragma unroll
    for (int k = 0; k < ICH; ++k) {
      rbias[k] = p.rb[c0 + k];
#pragma unroll
      for (int j = 0; j < 3; ++j) rw[k][j] = j < p.cin ? p.rw[(c0 + k) * p.cin + j] : 0.f;
    }
  }
  gn_reduce(p.part, p.nparts, b, p.count, s_mean, s_rstd, s_red);
  float sc[ICH], sh[ICH];
#pragma unroll
  for (int k = 0; k < ICH; ++k) {
    gn_affine(s_mean, s_rstd, p.C, c0 + k, p.gamma, p.beta, sc[k], sh[k]);
    gn_res_coef<A>(sc[k], sh[k]);   // (the base-2 forms gn_mish_res / gn_mish_add, as attn_kv / conv64 IN_RB0)
  }
#pragma unroll
  for (int i = 0; i < RB_IPT; ++i) {
    const int e = e0 + i * 256 * ICH;
    if (e < total) {
      const float m = mk[i];
      float v[ICH];
      item_to_f(vp[i], v, A());
      if (RES) {   // res_conv(x * m): bias + W (x m), fp32
        const float x0 = xr[i][0] * m, x1 = xr[i][1] * m, x2 = xr[i][2] * m;
#pragma unroll
        for (int k = 0; k < ICH; ++k) {
          const float r = fmaf(rw[k][2], x2, fmaf(rw[k][1], x1, fmaf(rw[k][0], x0, rbias[k])));
          v[k] = gn_mish_add<A>(v[k], sc[k], sh[k], r, m);
        }
      } else {
        float x[ICH];
        item_to_f(vx[i], x, A());
#pragma unroll
        for (int k = 0; k < ICH; ++k) v[k] = gn_mish_res<A>(v[k], sc[k], sh[k], x[k], m);
      }
      *reinterpret_cast<uint4*>(out + e) = f_to_item(v, A());
    }
  }
}

__global__ __launch_bounds__(256) void temb_kernel(TembParams p) {
  __shared__ float s_emb[64], s_h[256], s_t[64];
  const int row = blockIdx.x, tid = threadIdx.x;
  float t;
  if (p.tvals) {
    t = p.tvals[row];
  } else {   // t = 1 - (i + 0.5) h in double, rounded once to fp32 (diffusion.py:259-260); no contraction
    t = (float)__dsub_rn(1.0, __dmul_rn((double)row + 0.5, 1.0 / (double)p.n_steps));
    // noise_t = beta_min + (beta_max - beta_min) * t with the two fp32 roundings of the reference (:262-263)
    if (p.betas && tid == 0) p.betas[row] = __fadd_rn(p.beta_min, __fmul_rn(p.beta_delta, t));
  }
  if (tid < 64) {
    const int k = tid & 31;
    const float arg = (p.pe_scale * t) * p.freqs[k];       // scale * x * emb (diffusion.py:122)
    s_emb[tid] = tid < 32 ? sinf(arg) : cosf(arg);
  }
  __syncthreads();
  {   // mlp.0 (64 -> 256) + Mish
    float s = p.b0[tid];
    for (int k = 0; k < 64; ++k) s += p.w0[tid * 64 + k] * s_emb[k];
    s_h[tid] = mishf(s);
  }
  __syncthreads();
  if (tid < 64) {   // mlp.2 (256 -> 64), then the Mish that opens every ResnetBlock.mlp
    float s = p.b2[tid];
    for (int k = 0; k < 256; ++k) s += p.w2[tid * 256 + k] * s_h[k];
    s_t[tid] = mishf(s);
  }
  __syncthreads();
  for (int j = tid; j < p.nr; j += 256) {
    float s = p.br[j];
    for (int k = 0; k < 64; ++k) s += p.wr[(long)j * 64 + k] * s_t[k];
    p.tb[(long)row * p.nr + j] = s;
  }
}

__global__ __launch_bounds__(256) void spk_mlp_kernel(const float* spk, const float* w0, const float* b0, const float* w2,
                                                     const float* b2, float* s_out) {
  __shared__ float s_x[64], s_h[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid < 64) s_x[tid] = spk[b * 64 + tid];
  __syncthreads();
  float s = b0[tid];
  for (int k = 0; k < 64; ++k) s += w0[tid * 64 + k] * s_x[k];
  s_h[tid] = mishf(s);
  __syncthreads();
  if (tid < 80) {
    float o = b2[tid];
    for (int k = 0; k < 256; ++k) o += w2[tid * 256 + k] * s_h[k];
    s_out[b * 80 + tid] = o;
  }
}

__global__ void mask_copy_kernel(const float* z, const float* mask, int F, int T, long n, float* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long b = i / ((long)F * T);
  const int t = (int)(i % T);
  out[i] = z[i] * mask[b * T + t];
}

template <class A>
__global__ void to_nchw_kernel(const A* src, int F, int T, int C, long n, float* dst) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // index into dst [B][C][F][T]
  if (i >= n) return;
  const int t = (int)(i % T);
  const int f = (int)((i / T) % F);
  const int c = (int)((i / ((long)T * F)) % C);
  const long b = i / ((long)T * F * C);
  dst[i] = Act<A>::to_f(src[((b * F + f) * T + t) * C + c]);
}

hipError_t launch_to_nchw(int act_bf16, const void* src, int B, int F, int T, int C, float* dst, hipStream_t s) {
  const long n = (long)B * C * F * T;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (act_bf16) hipLaunchKernelGGL(to_nchw_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)src, F, T, C, n, dst);
  else hipLaunchKernelGGL(to_nchw_kernel<float>, grid, dim3(256), 0, s, (const float*)src, F, T, C, n, dst);
  return hipGetLastError();
}

hipError_t launch_final(int act_bf16, const FinalParams& p, hipStream_t s) {
  dim3 grid((unsigned)((80L * p.T + 255) / 256), (unsigned)p.B);
  if (act_bf16) hipLaunchKernelGGL(final_kernel<bf16>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(final_kernel<float>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_rbout_identity(int act_bf16, const RbOutParams& p, hipStream_t s) {
  const int ich = act_bf16 ? 8 : 4;
  const long total = (long)p.F * p.T * p.C;
  if ((256 * ich) % p.C != 0 || total >= (1L << 31)) return hipErrorInvalidValue;
  const long items = total / ich;
  dim3 grid((unsigned)((items + 256 * RB_IPT - 1) / (256 * RB_IPT)), (unsigned)p.B);
  if (act_bf16) hipLaunchKernelGGL((gn_mish_kernel<bf16>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((gn_mish_kernel<float>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_rbout_input(int act_bf16, const RbOutParams& p, hipStream_t s) {
  const int ich = act_bf16 ? 8 : 4;
  const long total = (long)p.F * p.T * p.C;
  if ((256 * ich) % p.C != 0 || total >= (1L << 31) || p.cin < 2 || p.cin > 3 || p.lvl != 0) return hipErrorInvalidValue;
  const long items = total / ich;
  dim3 grid((unsigned)((items + 256 * RB_IPT - 1) / (256 * RB_IPT)), (unsigned)p.B);
  if (act_bf16) hipLaunchKernelGGL((gn_mish_kernel<bf16, 1>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((gn_mish_kernel<float, 1>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_temb(const TembParams& p, hipStream_t s) {
  hipLaunchKernelGGL(temb_kernel, dim3(p.rows), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_spk_mlp(const float* spk, int B, const float* w0, const float* b0, const float* w2, const float* b2,
                          float* s_out, hipStream_t s) {
  hipLaunchKernelGGL(spk_mlp_kernel, dim3(B), dim3(256), 0, s, spk, w0, b0, w2, b2, s_out);
  return hipGetLastError();
}

// device step index of the sampler (kernels.h tb_at): one lane stores it (a kernel node in every kind of capture)
__global__ void set_step_kernel(int* stepp, int v) {
  if (threadIdx.x == 0) stepp[0] = v;
}
hipError_t launch_set_step(int* stepp, int v, hipStream_t s) {
  hipLaunchKernelGGL(set_step_kernel, dim3(1), dim3(64), 0, s, stepp, v);
  return hipGetLastError();
}

// fill / copy of fp32 buffers as kernel launches: a kernel node in any capture. Memset and memcpy nodes are avoided:
// a HIP graph's memset node wrote garbage from its second launch on when the graph was launched on a stream other
// than its capture stream -- which torch.cuda.graph's replay does (tools/memset_capture_probe.py).
__global__ void fill_f32_kernel(float* p, long n, float v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = v;
}
__global__ void copy_f32_kernel(float* dst, const float* src, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = src[i];
}
static unsigned grid_for(long n) { return (unsigned)std::max<long>(1, std::min<long>((n + 255) / 256, 8192)); }
hipError_t launch_fill_f32(float* p, long n, float v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, n, v);
  return hipGetLastError();
}
hipError_t launch_copy_f32(float* dst, const float* src, long n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(copy_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}

hipError_t launch_mask_copy(const float* z, const float* mask, int B, int F, int T, float* out, hipStream_t s) {
  const long n = (long)B * F * T;
  hipLaunchKernelGGL(mask_copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, z, mask, F, T, n, out);
  return hipGetLastError();
}

}  // namespace gt
