// LinearAttention (model/diffusion.py:82-100) + Rezero/Residual (:39-46, 103-110), restructured.
//
// Reference: qkv = W_qkv x; k = softmax_n(k); ctx_h = k_h v_h^T (32x32 per head); out = ctx^T q;
//            y = x + g * (W_out out + b_out).
// Everything after the softmax statistics is linear in x, so per batch item
//            y = x + M_b x + g b_out,   M_b = g * W_out * blockdiag_h(ctx_h^T) * W_q    (C x C)
// The pass over the activation therefore costs one k/v projection (kernel attn_kv) plus one C x C
// 1x1 convolution (conv_kernel CONV1/OUT_RESID with per-batch weights), instead of materialising
// q, k, v (6x the activation at level 0).
//
// attn_kv: workgroup = 4 waves = 4 heads, tile of `tile_pos` positions processed as 64-position
// sub-blocks. Per sub-block each wave computes k_h, v_h (64 x 32 each) with MFMA, then updates an
// online softmax (running max m, running sum l, 32x32 context) where the context update
// ctx += P^T V uses the two fp32 accumulator tiles directly as MFMA operands (both are indexed by
// position along their rows, so no LDS transpose is needed). Tiles write {m, l, ctx} partials.
// attn_merge: rescale+sum the partials -> normalised ctx, then G_h = ctx_h^T W_q,h  (fp32).
// attn_mbuild: M_b = g * W_out G  written in the activation dtype as the per-batch 1x1 weight.
#include "common.h"
#include "kernels.h"
#include "wimage.h"

namespace gt {

template <class A, bool RES>
__global__ __launch_bounds__(256) void attn_kv_kernel(AttnKVParams p) {
  constexpr int CK = 64 / (int)sizeof(A);
  constexpr int ICH = 16 / (int)sizeof(A);
  constexpr int KSTEP_B = 16 * (int)sizeof(A);
  constexpr int XROW_MAX = 256 + 16;   // resident layout only used when Cpad*sizeof(A) <= 256 B
  constexpr int SX_BYTES = RES ? 64 * XROW_MAX : 64 * 80;
  constexpr int SW_BYTES = RES ? 256 * XROW_MAX : 256 * 80;
  typedef typename Mma<A>::frag frag;
  __shared__ __attribute__((aligned(16))) char sX[SX_BYTES];
  __shared__ __attribute__((aligned(16))) char sW[SW_BYTES];

  const int b = blockIdx.x / p.ntile, tile = blockIdx.x % p.ntile;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  const int row_b = RES ? p.Cpad * (int)sizeof(A) + 16 : 80;   // LDS row stride (odd # of 16-B slots)
  const A* x = reinterpret_cast<const A*>(p.x) + (long)b * p.n * p.C;
  const A* wkv = reinterpret_cast<const A*>(p.wkv);
  const int itemsPerRow = RES ? p.Cpad / ICH : 4;

  if (RES) {   // whole [256][Cpad] k/v projection resident in LDS
    for (int it = tid; it < 256 * itemsPerRow; it += 256) {
      const int row = it / itemsPerRow, sub = it - row * itemsPerRow;
      *reinterpret_cast<uint4*>(sW + row * row_b + sub * 16) =
          *reinterpret_cast<const uint4*>(wkv + (long)row * p.Cpad + sub * ICH);
    }
  }

  const float NEG_INF = -__builtin_huge_valf();
  float m_run = NEG_INF, l_run = 0.f;
  f32x16 ctx;
#pragma unroll
  for (int k = 0; k < 16; ++k) ctx[k] = 0.f;

  const int tbeg = tile * p.tile_pos;
  const int tend = min(p.n, tbeg + p.tile_pos);
  for (int pos0 = tbeg; pos0 < tend; pos0 += 64) {
    f32x16 ak[2], av[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) { ak[i][k] = 0.f; av[i][k] = 0.f; }

    const int nch = RES ? 1 : p.Cpad / CK;
    for (int ch = 0; ch < nch; ++ch) {
      __syncthreads();
      const int c0 = ch * CK;
      for (int it = tid; it < 64 * itemsPerRow; it += 256) {
        const int row = it / itemsPerRow, sub = it - row * itemsPerRow;
        const int pos = pos0 + row;
        uint4 u = make_uint4(0, 0, 0, 0);
        if (pos < tend) u = *reinterpret_cast<const uint4*>(x + (long)pos * p.C + c0 + sub * ICH);
        *reinterpret_cast<uint4*>(sX + row * row_b + sub * 16) = u;
      }
      if (!RES) {
        for (int it = tid; it < 256 * 4; it += 256) {
          const int row = it >> 2, sub = it & 3;
          *reinterpret_cast<uint4*>(sW + row * 80 + sub * 16) =
              *reinterpret_cast<const uint4*>(wkv + (long)row * p.Cpad + c0 + sub * ICH);
        }
      }
      __syncthreads();
      const int nks = RES ? p.Cpad / 16 : CK / 16;
      for (int ks = 0; ks < nks; ++ks) {
        const int off = ks * KSTEP_B + h * (KSTEP_B / 2);
        const frag bk = Mma<A>::load(sW + (wv * 32 + r) * row_b + off);
        const frag bv = Mma<A>::load(sW + (128 + wv * 32 + r) * row_b + off);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const frag a = Mma<A>::load(sX + (rb * 32 + r) * row_b + off);
          Mma<A>::mma(a, bk, ak[rb]);
          Mma<A>::mma(a, bv, av[rb]);
        }
      }
    }

    // ---- online softmax over positions (k.softmax(dim=-1), diffusion.py:95) for column d = r
    float mloc = NEG_INF;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (pos0 + rb * 32 + acc_row(j, h) < tend) mloc = fmaxf(mloc, ak[rb][j]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = (m_run == NEG_INF) ? 0.f : __expf(m_run - m_new);
    float lsum = 0.f;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const bool valid = pos0 + rb * 32 + acc_row(j, h) < tend;
        const float e = valid ? __expf(ak[rb][j] - m_new) : 0.f;
        ak[rb][j] = e;
        lsum += e;
      }
    lsum += __shfl_xor(lsum, 32);
    l_run = l_run * alpha + lsum;
    // ctx rows are d = acc_row(j, h); the factor for row d lives in lane d
#pragma unroll
    for (int j = 0; j < 16; ++j) ctx[j] *= __shfl(alpha, acc_row(j, h));
    // ---- ctx[d][e] += sum_pos P[pos][d] V[pos][e]   (einsum 'bhdn,bhen->bhde', diffusion.py:96)
    if constexpr (sizeof(A) == 2) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 pa, pv;
#pragma unroll
          for (int i = 0; i < 8; ++i) { pa[i] = (bf16)ak[rb][8 * s + i]; pv[i] = (bf16)av[rb][8 * s + i]; }
          ctx = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, pv, ctx, 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int j = 0; j < 16; ++j) ctx = __builtin_amdgcn_mfma_f32_32x32x2f32(ak[rb][j], av[rb][j], ctx, 0, 0, 0);
    }
    m_run = m_new;
  }

  float* part = p.part + (((long)b * p.ntile + tile) * 4 + wv) * 1088;
  if (h == 0) { part[r] = m_run; part[32 + r] = l_run; }
#pragma unroll
  for (int j = 0; j < 16; ++j) part[64 + acc_row(j, h) * 32 + r] = ctx[j];
}

// grid (B, 4 heads): merge tile partials, normalise, G[b][32h+e][ci] = sum_d ctx[d][e] Wq[32h+d][ci]
__global__ __launch_bounds__(256) void attn_merge_kernel(const float* part, int ntile, int C, const float* wq, float* G) {
  __shared__ float s_ctx[32][33];
  const int b = blockIdx.x, hd = blockIdx.y, tid = threadIdx.x;
  const int d = tid >> 3, e0 = (tid & 7) * 4;
  const float* base = part + ((long)b * ntile * 4 + hd) * 1088;
  const long tstride = 4 * 1088;
  float M = -__builtin_huge_valf();
  for (int t = 0; t < ntile; ++t) M = fmaxf(M, base[t * tstride + d]);
  float L = 0.f, c[4] = {0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < ntile; ++t) {
    const float* pt = base + t * tstride;
    const float w = __expf(pt[d] - M);
    L += w * pt[32 + d];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] += w * pt[64 + d * 32 + e0 + k];
  }
  const float inv = 1.f / L;
#pragma unroll
  for (int k = 0; k < 4; ++k) s_ctx[d][e0 + k] = c[k] * inv;
  __syncthreads();
  float* Gb = G + (long)b * 128 * C;
  for (int idx = tid; idx < 32 * C; idx += 256) {
    const int e = idx / C, ci = idx - e * C;
    float s = 0.f;
#pragma unroll 8
    for (int dd = 0; dd < 32; ++dd) s += s_ctx[dd][e] * wq[(long)(hd * 32 + dd) * C + ci];
    Gb[(long)(hd * 32 + e) * C + ci] = s;
  }
}

// grid (B, C/16): M_b[co][ci] = g * sum_r Wout[co][r] G[b][r][ci], written straight into the packed
// 1x1 weight image (wimage.h) that conv_kernel DMAs into LDS.
template <class A>
__global__ __launch_bounds__(256) void attn_mbuild_kernel(const float* G, const float* wout, const float* g, int C,
                                                          char* Mw, WImg W) {
  __shared__ float s_w[16][129];
  const int b = blockIdx.x, co0 = blockIdx.y * 16, tid = threadIdx.x;
  for (int i = tid; i < 16 * 128; i += 256) s_w[i >> 7][i & 127] = wout[(long)(co0 + (i >> 7)) * 128 + (i & 127)];
  __syncthreads();
  const float gg = g[0];
  const float* Gb = G + (long)b * 128 * C;
  char* img = Mw + (long)b * W.total;
  const int row = tid >> 4;   // 16 rows x 16 column lanes
  for (int ci = tid & 15; ci < C; ci += 16) {
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < 128; ++k) s += s_w[row][k] * Gb[(long)k * C + ci];
    *reinterpret_cast<A*>(img + conv_wimg_off(W, co0 + row, 0, ci, (int)sizeof(A))) = Act<A>::from_f(gg * s);
  }
}

hipError_t launch_attn_kv(int act_bf16, const AttnKVParams& p, hipStream_t s) {
  const dim3 grid((unsigned)(p.B * p.ntile));
  if (act_bf16) {
    if (p.Cpad * 2 <= 256) hipLaunchKernelGGL((attn_kv_kernel<bf16, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((attn_kv_kernel<bf16, false>), grid, dim3(256), 0, s, p);
  } else {
    if (p.Cpad * 4 <= 256) hipLaunchKernelGGL((attn_kv_kernel<float, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((attn_kv_kernel<float, false>), grid, dim3(256), 0, s, p);
  }
  return hipGetLastError();
}

hipError_t launch_attn_merge(const float* part, int B, int ntile, int C, const float* wq, float* G, hipStream_t s) {
  hipLaunchKernelGGL(attn_merge_kernel, dim3(B, 4), dim3(256), 0, s, part, ntile, C, wq, G);
  return hipGetLastError();
}

hipError_t launch_attn_mbuild(int act_bf16, const float* G, const float* wout, const float* g, int B, int C, void* Mw,
                              hipStream_t s) {
  const WImg W = conv_wimg(act_bf16, 1, C, C);
  if (act_bf16)
    hipLaunchKernelGGL(attn_mbuild_kernel<bf16>, dim3(B, C / 16), dim3(256), 0, s, G, wout, g, C, (char*)Mw, W);
  else
    hipLaunchKernelGGL(attn_mbuild_kernel<float>, dim3(B, C / 16), dim3(256), 0, s, G, wout, g, C, (char*)Mw, W);
  return hipGetLastError();
}

}  // namespace gt
