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
// attn_merge: rescale+sum the partials -> normalised ctx -> A_b = g W_out blockdiag(ctx^T)   (fp32, C x 128)
// attn_fold:  M_b = A_b W_q on fp32 MFMA, written as the per-batch 1x1 weight image.
#include "common.h"
#include "kernels.h"
#include "wimage.h"

namespace gt {

// bytes per position of a bf16 chunk of the chunked attn_kv (128: 64 channels, half the barriers of 64 B; measured
// 48.8 -> 42.2 us at C = 256, 82.4 -> 72.4 us at C = 128)
constexpr int kKvCkb = 128;
// positions per sub-block of the chunked (C > 64) bf16 attn_kv (128 spills at 256 VGPRs)
constexpr int kKvSb = 64;

// RB: the input is formed from the ResnetBlock's block2 pre-activation and its residual in the operand load
// (AttnKVParams::rb_pre); the formed rows also go to rb_out. Same expression and GroupNorm reduction as
// gn_mish_kernel, so the stored activation is bit-identical to the separate pass it replaces.
// SB: positions per sub-block (64 or 128; the chunked path stages every k/v weight slice once per sub-block, so 128 halves
// that traffic and the barriers per position)
template <class A, int CPR, bool RB, int SB = 64>   // CPR > 0: all CPR input channels resident in LDS; 0: chunked (large C)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_kv_kernel(AttnKVParams p) {
  constexpr int NRB = SB / 32;                                  // 32-position row blocks per sub-block
  constexpr bool RES = CPR > 0;
  constexpr int CKB = (sizeof(A) == 2 && !RES) ? kKvCkb : 64;   // bytes of a position's channel chunk
  constexpr int CK = CKB / (int)sizeof(A);
  constexpr int ICH = 16 / (int)sizeof(A);
  constexpr int KSTEP_B = 16 * (int)sizeof(A);
  constexpr int ROWB = RES ? CPR * (int)sizeof(A) + 16 : CKB + 16;   // LDS row stride: odd number of 16-B slots
  constexpr int IPR = RES ? CPR / ICH : CKB / 16;                    // 16-B items per staged row
  constexpr int WPT = RES ? 1 : CKB / 16;                            // weight-slice items per thread (256 rows)
  constexpr int XIT = SB * IPR / 256;                           // x items per thread per sub-block
  static_assert(SB * IPR % 256 == 0, "x staging must split evenly");
  typedef typename Mma<A>::frag frag;
  __shared__ __attribute__((aligned(16))) char smem[(SB + 256) * ROWB];
  char* sX = smem;
  char* sW = smem + SB * ROWB;

  const int b = blockIdx.x / p.ntile, tile = blockIdx.x % p.ntile;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  const A* x = reinterpret_cast<const A*>(p.x) + (long)b * p.n * p.C;
  const A* wkv = reinterpret_cast<const A*>(p.wkv);
  const A* pre = RB ? reinterpret_cast<const A*>(p.rb_pre) + (long)b * p.n * p.C : nullptr;
  A* rb_out = RB ? reinterpret_cast<A*>(p.rb_out) + (long)b * p.n * p.C : nullptr;
  // GroupNorm coefficients of channel c at c + c / 8: the operand loads read 8 consecutive channels at 8 different
  // 8-channel groups per half-wave (ds_read2_b32, banks (a/4) mod 32), which unskewed put groups g and g + 4 on one bank
  __shared__ float s_sc[RB ? 288 : 1], s_sh[RB ? 288 : 1], s_mean[8], s_rstd[8];
  auto cix = [](int c) { return c + (c >> 3); };
  __shared__ double s_red[RB ? 272 : 1];
  GnLoad gl;
  if (RB) gl = gn_load(p.rb_part, p.rb_nparts, b);   // slot loads in flight with the weight / first x loads

  if (RES) {   // whole [256][C] k/v projection resident in LDS
    for (int it = tid; it < 256 * IPR; it += 256) {
      const int row = it / IPR, sub = it - row * IPR;
      *reinterpret_cast<uint4*>(sW + row * ROWB + sub * 16) =
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
  uint4 xr[XIT], xq[RB ? XIT : 1];   // RB: xr = block2 pre-activation, xq = residual input
  float mk[RB ? XIT : 1];
  // raw buffer access over this utterance's rows (byte offsets < 2^31: launch_attn_kv checks n * C): a position past the
  // tile's end takes an offset outside the buffer, so its loads return zeros and its rb_out stores are dropped
  const unsigned nbytes = (unsigned)(p.n * p.C * (int)sizeof(A));
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_pre = __builtin_amdgcn_make_buffer_rsrc((void*)(RB ? pre : x), (short)0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_rb = __builtin_amdgcn_make_buffer_rsrc((void*)(RB ? rb_out : x), (short)0, nbytes, 0x00020000);
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  auto ld16 = [](__amdgpu_buffer_rsrc_t rs, int off) {
    const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };
  auto xoff = [&](int pos, int c) { return pos < tend ? (pos * p.C + c) * (int)sizeof(A) : (int)0x80000000; };
  auto load_x = [&](int pos0, int c0) {
#pragma unroll
    for (int j = 0; j < XIT; ++j) {
      const int it = tid + 256 * j, row = it / IPR, sub = it - row * IPR;
      const int pos = pos0 + row;
      const int off = xoff(pos, c0 + sub * ICH);
      if (RB) {
        xr[j] = ld16(rs_pre, off);
        xq[j] = ld16(rs_x, off);
        // the mask depends on the position only: once per sub-block (chunk 0), kept for its other chunks
        if (c0 == 0) mk[j] = pos < tend ? mask_at(p.mask, p.T0, b, pos % p.T, p.lvl) : 0.f;
      } else {
        xr[j] = ld16(rs_x, off);
      }
    }
  };
  auto store_x = [&](int pos0, int c0) {
#pragma unroll
    for (int j = 0; j < XIT; ++j) {
      const int it = tid + 256 * j, row = it / IPR, sub = it - row * IPR;
      uint4 u = xr[j];
      if (RB) {   // x_in = (Mish(GN(pre)) + x) * m, as gn_mish_kernel<A, false>; positions past the tile: zeros, dropped
        const int pos = pos0 + row, c = c0 + sub * ICH;
        float v[ICH], xv[ICH];
        item_to_f(xr[j], v, A());
        item_to_f(xq[j], xv, A());
        const float m = mk[j];
#pragma unroll
        for (int k = 0; k < ICH; ++k) v[k] = gn_mish_res<A>(v[k], s_sc[cix(c) + k], s_sh[cix(c) + k], xv[k], m);
        u = f_to_item(v, A());
        const u32x4_t o = {u.x, u.y, u.z, u.w};
        __builtin_amdgcn_raw_buffer_store_b128(o, rs_rb, xoff(pos, c), 0, 0);
      }
      *reinterpret_cast<uint4*>(sX + row * ROWB + sub * 16) = u;
    }
  };
  // chunked path: the next chunk's x (and pre / mask) rows are loaded into registers while the current chunk is in
  // the MFMAs (a load issued right before its LDS store left one HBM round trip exposed per 32-channel chunk)
  load_x(tbeg, 0);
  if (RB) {
    gn_finish(gl, p.rb_part, p.rb_nparts, b, p.rb_count, s_mean, s_rstd, s_red);
    for (int c = tid; c < p.C; c += 256) {
      gn_affine(s_mean, s_rstd, p.C, c, p.rb_gamma, p.rb_beta, s_sc[cix(c)], s_sh[cix(c)]);
      gn_res_coef<A>(s_sc[cix(c)], s_sh[cix(c)]);
    }
  }
  // chunked path: the next k/v weight slice (item i of thread tid: row tid / IPR + (256 / IPR) i, 16 B at
  // (tid % IPR) * 16) is loaded into registers during the current chunk (level 1: 94.5 -> 82.4 us)
  static_assert(WPT == 4 || WPT == 8 || RES, "weight-slice prefetch holds 4 or 8 items");
  uint4 w0, w1, w2, w3, w4, w5, w6, w7;   // named: an array here lands in scratch
  bool wpf_ok = false;
  const A* wrow = wkv + (long)(tid / IPR) * p.Cpad + (tid % IPR) * ICH;
  const long wstep = (long)(256 / IPR) * p.Cpad;
#define KV_W_(I_, CH_) (*reinterpret_cast<const uint4*>(wrow + (I_) * wstep + (CH_) * CK))
#define KV_LOAD_W(CH_)                                                                    \
  do {                                                                                       \
    if constexpr (!RES) {                                                                    \
      w0 = KV_W_(0, CH_); w1 = KV_W_(1, CH_); w2 = KV_W_(2, CH_); w3 = KV_W_(3, CH_); \
      if constexpr (WPT == 8) {                                                              \
        w4 = KV_W_(4, CH_); w5 = KV_W_(5, CH_); w6 = KV_W_(6, CH_); w7 = KV_W_(7, CH_); \
      }                                                                                      \
    }                                                                                        \
  } while (0)
  // Two workgroups per CU in one round (level 0: 16 tiles per utterance): the second-dispatched one takes wave priority
  // 1 for the first two thirds of its sub-blocks, as conv64 does (level-0 form 133.6 -> 127.2 us, same box)
  const bool young = (int)blockIdx.x >= (int)(gridDim.x / 2);
  if (young) __builtin_amdgcn_s_setprio(1);
  const int pos_lo = tbeg + (2 * (tend - tbeg)) / 3;
  for (int pos0 = tbeg; pos0 < tend; pos0 += SB) {
    if (young && pos0 >= pos_lo && pos0 < pos_lo + SB) __builtin_amdgcn_s_setprio(0);
    f32x16 ak[NRB], av[NRB];
#pragma unroll
    for (int i = 0; i < NRB; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) { ak[i][k] = 0.f; av[i][k] = 0.f; }

    const int nch = RES ? 1 : p.Cpad / CK;
    for (int ch = 0; ch < nch; ++ch) {
      lds_barrier();                                   // every wave is done with the previous chunk's fragments
      store_x(pos0, ch * CK);
      if (!RES) {                                      // the k/v weight slice: L2-resident, loaded straight into LDS
        if (!wpf_ok) KV_LOAD_W(ch);                    // (prefetched into registers during the previous chunk)
        char* wd = sW + (tid / IPR) * ROWB + (tid % IPR) * 16;
        constexpr int WS = (256 / IPR) * ROWB;
        *reinterpret_cast<uint4*>(wd) = w0;
        *reinterpret_cast<uint4*>(wd + WS) = w1;
        *reinterpret_cast<uint4*>(wd + 2 * WS) = w2;
        *reinterpret_cast<uint4*>(wd + 3 * WS) = w3;
        if constexpr (WPT == 8) {
          *reinterpret_cast<uint4*>(wd + 4 * WS) = w4;
          *reinterpret_cast<uint4*>(wd + 5 * WS) = w5;
          *reinterpret_cast<uint4*>(wd + 6 * WS) = w6;
          *reinterpret_cast<uint4*>(wd + 7 * WS) = w7;
        }
      }
      lds_barrier();
      if (RES) {
        if (pos0 + SB < tend) load_x(pos0 + SB, 0);   // next sub-block in flight during the MFMAs
      } else if (ch + 1 < nch) {
        load_x(pos0, (ch + 1) * CK);
      } else if (pos0 + SB < tend) {
        load_x(pos0 + SB, 0);
      }
      if (!RES) {   // the next chunk's weight slice (chunk 0 again after the last: the next sub-block)
        KV_LOAD_W(ch + 1 < nch ? ch + 1 : 0);
        wpf_ok = true;
      }
      const int nks = RES ? CPR / 16 : CK / 16;
      for (int ks = 0; ks < nks; ++ks) {
        const int off = ks * KSTEP_B + h * (KSTEP_B / 2);
        const frag bk = Mma<A>::load(sW + (wv * 32 + r) * ROWB + off);
        const frag bv = Mma<A>::load(sW + (128 + wv * 32 + r) * ROWB + off);
#pragma unroll
        for (int rb = 0; rb < NRB; ++rb) {
          const frag a = Mma<A>::load(sX + (rb * 32 + r) * ROWB + off);
          Mma<A>::mma(a, bk, ak[rb]);
          Mma<A>::mma(a, bv, av[rb]);
        }
      }
    }

  // ---- online softmax over positions (k.softmax(dim=-1), diffusion.py:95) for column d = r
    const bool full = pos0 + SB <= tend;             // wave-uniform: no per-element validity test
    float mloc = NEG_INF;
    if (full) {
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int j = 0; j < 16; ++j) mloc = fmaxf(mloc, ak[rb][j]);
    } else {
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (pos0 + rb * 32 + acc_row(j, h) < tend) mloc = fmaxf(mloc, ak[rb][j]);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32));
    // exp(a - m) as exp2(fma(a, log2 e, -mL)) with mL = fl(m log2 e): one FMA + v_exp_f32 per element. The running
    // statistic is mL itself (rounding is monotonic, so max and argmax are unchanged), and every rescale below and
    // in attn_merge is exp2 of a difference of these rounded values: the factors cancel exactly across blocks.
    constexpr float L2E = 1.44269504088896341f;
    const float mL = fmaxf(m_run, mloc * L2E);
    const float m_new = mL;
    float lsum = 0.f;
    if (full) {
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(ak[rb][j], L2E, -mL));
          ak[rb][j] = e;
          lsum += e;
        }
    } else {
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const bool valid = pos0 + rb * 32 + acc_row(j, h) < tend;
          const float e = valid ? __builtin_amdgcn_exp2f(__builtin_fmaf(ak[rb][j], L2E, -mL)) : 0.f;
          ak[rb][j] = e;
          lsum += e;
        }
    }
    lsum += __shfl_xor(lsum, 32);
    // rescale the running sum/context only where the running max moved (rare after the first blocks)
    if (__any(m_new != m_run)) {
      const float alpha = (m_run == NEG_INF) ? 0.f : __builtin_amdgcn_exp2f(m_run - m_new);
      l_run *= alpha;
      // ctx rows are d = acc_row(j, h); the factor for row d lives in lane d
#pragma unroll
      for (int j = 0; j < 16; ++j) ctx[j] *= __shfl(alpha, acc_row(j, h));
    }
    l_run += lsum;
    // ---- ctx[d][e] += sum_pos P[pos][d] V[pos][e]   (einsum 'bhdn,bhen->bhde', diffusion.py:96)
    if constexpr (sizeof(A) == 2) {
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          typedef float f32x8_t __attribute__((ext_vector_type(8)));
          f32x8_t fa, fv;
#pragma unroll
          for (int i = 0; i < 8; ++i) { fa[i] = ak[rb][8 * s + i]; fv[i] = av[rb][8 * s + i]; }
          const bf16x8 pa = __builtin_convertvector(fa, bf16x8), pv = __builtin_convertvector(fv, bf16x8);   // 4 packed converts each
          ctx = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, pv, ctx, 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int j = 0; j < 16; ++j) ctx = __builtin_amdgcn_mfma_f32_32x32x2f32(ak[rb][j], av[rb][j], ctx, 0, 0, 0);
    }
    m_run = m_new;
  }

  float* part = p.part + (((long)b * p.ntile + tile) * 4 + wv) * 1088;
  if (h == 0) { part[r] = m_run; part[32 + r] = l_run; }   // m_run = fl(max k * log2 e)
#pragma unroll
  for (int j = 0; j < 16; ++j) part[64 + acc_row(j, h) * 32 + r] = ctx[j];
}
#undef KV_LOAD_W
#undef KV_W_

// grid (B, 4 heads, 32 / DR): merge the tiles' online-softmax partials, normalise, and fold the head's part of
// the output projection (m_t, M: running maxima in log2 units, as attn_kv keeps them):
//   ctx_h[d][e]  = sum_t 2^(m_t[d] - M[d]) ctx_t[d][e] / sum_t 2^(m_t[d] - M[d]) l_t[d]
//   A[co][32h+d] = g * sum_e Wout[co][32h+e] ctx_h[d][e]     (einsum 'bhde,bhdn->bhen' + to_out + Rezero)
// Rows d are independent, so a workgroup owns DR of them: DR = 32 (throughput plan) merges in NG = 4 tile groups;
// DR = 4 (small-batch plan: few utterances, up to 256 tiles each) spreads a head over 8 workgroups and merges in
// NG = 32 groups of a few tiles each (the serial chain of dependent loads is what a B = 1 merge waits on).
template <int DR>
__global__ __launch_bounds__(1024) void attn_merge_kernel(const float* part, int ntile, const float* wout, const float* g,
                                                          int C, float* Aout) {
  constexpr int NG = 1024 / (DR * 8);   // tile groups
  __shared__ float s_ctx[DR][33];
  __shared__ float s_w[256][33];
  __shared__ float s_gc[NG][DR][33];   // per tile group: unnormalised context, running max, running sum
  __shared__ float s_gm[NG][DR], s_gl[NG][DR];
  const int b = blockIdx.x, hd = blockIdx.y, d0 = blockIdx.z * DR, tid = threadIdx.x;
  const int grp = tid / (DR * 8), lt = tid % (DR * 8);
  const int dl = lt >> 3, d = d0 + dl, e0 = (lt & 7) * 4;
  // tile group grp merges tiles [t0, t1) online (running max), in tile order
  const int per = (ntile + NG - 1) / NG, t0 = grp * per, t1 = min(ntile, t0 + per);
  const float* base = part + ((long)b * ntile * 4 + hd) * 1088;
  const long tstride = 4 * 1088;
  float M = -__builtin_huge_valf(), L = 0.f, c[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int t = t0; t < t1; ++t) {
    const float* pt = base + t * tstride;
    const float mt = pt[d], lt_ = pt[32 + d];
    const f32x4 v = *reinterpret_cast<const f32x4*>(pt + 64 + d * 32 + e0);
    if (mt > M) {                                      // rescale what was merged so far (m in log2 units)
      const float r = __builtin_amdgcn_exp2f(M - mt);
      L *= r;
#pragma unroll
      for (int k = 0; k < 4; ++k) c[k] *= r;
      M = mt;
    }
    const float w = __builtin_amdgcn_exp2f(mt - M);
    L += w * lt_;
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] += w * v[k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) s_gc[grp][dl][e0 + k] = c[k];
  if ((lt & 7) == 0) { s_gm[grp][dl] = M; s_gl[grp][dl] = L; }
  for (int i = tid; i < C * 8; i += 1024) {            // Wout[:, 32h : 32h+32] -> LDS (float4 loads)
    const int co = i >> 3, e4 = (i & 7) * 4;
    const f32x4 w = *reinterpret_cast<const f32x4*>(wout + (long)co * 128 + hd * 32 + e4);
#pragma unroll
    for (int k = 0; k < 4; ++k) s_w[co][e4 + k] = w[k];
  }
  __syncthreads();
  if (grp == 0) {                                      // combine the groups in a fixed order
    float Mt = -__builtin_huge_valf();
#pragma unroll
    for (int q = 0; q < NG; ++q) Mt = fmaxf(Mt, s_gm[q][dl]);
    float Lt = 0.f, ct[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int q = 0; q < NG; ++q) {
      if (s_gl[q][dl] == 0.f) continue;                // empty group (ntile < NG)
      const float r = __builtin_amdgcn_exp2f(s_gm[q][dl] - Mt);
      Lt += r * s_gl[q][dl];
#pragma unroll
      for (int k = 0; k < 4; ++k) ct[k] += r * s_gc[q][dl][e0 + k];
    }
    const float inv = 1.f / Lt;
#pragma unroll
    for (int k = 0; k < 4; ++k) s_ctx[dl][e0 + k] = ct[k] * inv;
  }
  __syncthreads();
  const float gg = g[0];
  for (int idx = tid; idx < C * DR; idx += 1024) {     // (co, d), d fastest: s_w broadcast, s_ctx stride 33
    const int co = idx / DR, dd = idx % DR;
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) acc += s_w[co][e] * s_ctx[dd][e];
    Aout[((long)b * C + co) * 128 + hd * 32 + d0 + dd] = gg * acc;
  }
}

// grid (B, C/64, C/64): M_b = A_b Wq  (C x 128 times 128 x C) with exact-fp32 MFMA (v_mfma_f32_32x32x2_f32),
// 4 waves x one 32x32 block each, written straight into the packed 1x1 weight image (wimage.h). Both operands are staged
// row-major from [row][128] fp32 (A_b rows co, W_q^T rows ci: the decoder packs W_q transposed), each row's 128 k
// split by parity into two halves of 64 (row stride 132 floats): lane (r, h) of the MFMA then reads k + 2t + h,
// t = 0..3, as one ds_read_b128 (16 lanes of a read group on 16 distinct 4-bank slots), and the float4 global loads
// store as two ds_write_b64 of 16 consecutive lanes on 32 consecutive words: no bank conflicts either way (a 129-float
// transposing stage had 2.67 conflict cycles per LDS instruction).
template <class A>
__global__ __launch_bounds__(256) void attn_fold_kernel(const float* Ain, const float* wqt, int C, char* Mw, WImg W) {
  constexpr int RS = 132;
  __shared__ __attribute__((aligned(16))) float s_a[64 * RS];   // A rows co0..co0+63
  __shared__ __attribute__((aligned(16))) float s_q[64 * RS];   // W_q^T rows ci0..ci0+63
  const int b = blockIdx.x, co0 = blockIdx.y * 64, ci0 = blockIdx.z * 64, tid = threadIdx.x;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  auto stage = [&](float* dst, const float* src) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = tid + 256 * j, rr = i >> 5, k4 = (i & 31) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(src + (long)rr * 128 + k4);
      *reinterpret_cast<f32x2*>(dst + rr * RS + k4 / 2) = f32x2{v.x, v.z};        // even k
      *reinterpret_cast<f32x2*>(dst + rr * RS + 64 + k4 / 2) = f32x2{v.y, v.w};   // odd k
    }
  };
  stage(s_a, Ain + ((long)b * C + co0) * 128);
  stage(s_q, wqt + (long)ci0 * 128);
  __syncthreads();
  const int lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  const int bm = (wv >> 1) * 32, bn = (wv & 1) * 32;
  const float* pa = s_a + (bm + r) * RS + h * 64;
  const float* pq = s_q + (bn + r) * RS + h * 64;
  f32x16 acc;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;
#pragma unroll 4
  for (int k = 0; k < 128; k += 8) {   // A[i = lane&31][k + 2t + h], B[k + 2t + h][j = lane&31]
    const f32x4 a4 = *reinterpret_cast<const f32x4*>(pa + k / 2);
    const f32x4 q4 = *reinterpret_cast<const f32x4*>(pq + k / 2);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[t], q4[t], acc, 0, 0, 0);
  }
  char* img = Mw + (long)b * W.total;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int co = co0 + bm + acc_row(j, h), ci = ci0 + bn + r;
    *reinterpret_cast<A*>(img + conv_wimg_off(W, co, 0, ci, (int)sizeof(A))) = Act<A>::from_f(acc[j]);
  }
}

hipError_t launch_attn_kv(int act_bf16, const AttnKVParams& p, hipStream_t s) {
  const dim3 grid((unsigned)(p.B * p.ntile));
  if (p.rb_pre && (p.C > 256 || p.C != p.Cpad)) return hipErrorInvalidValue;   // s_sc / s_sh hold 256 channels
  if ((long)p.n * p.C * (act_bf16 ? 2 : 4) >= (1L << 31)) return hipErrorInvalidValue;   // 32-bit buffer offsets
  if (p.Cpad > 64 && p.Cpad % (act_bf16 ? kKvCkb / 2 : 16) != 0) return hipErrorInvalidValue;   // whole chunks
  // resident k/v weights only for C = 64; wider inputs stream 64-channel chunks (bf16; 3 workgroups/CU,
  // measured faster at C = 128 than the 87 KB resident variant at 1 workgroup/CU)
#define KV_LAUNCH(A_, CPR_, SB_)                                                                          \
  do {                                                                                                \
    if (p.rb_pre) hipLaunchKernelGGL((attn_kv_kernel<A_, CPR_, true, SB_>), grid, dim3(256), 0, s, p);  \
    else hipLaunchKernelGGL((attn_kv_kernel<A_, CPR_, false, SB_>), grid, dim3(256), 0, s, p);          \
  } while (0)
  if (act_bf16) {
    if (p.Cpad <= 64) KV_LAUNCH(bf16, 64, 64); else KV_LAUNCH(bf16, 0, kKvSb);
  } else {
    if (p.Cpad <= 64) KV_LAUNCH(float, 64, 64); else KV_LAUNCH(float, 0, 64);
  }
#undef KV_LAUNCH
  return hipGetLastError();
}

hipError_t launch_attn_merge(const float* part, int B, int ntile, const float* wout, const float* g, int C, float* Aout,
                             int dr, hipStream_t s) {
  if (C > 256 || C % 4 != 0) return hipErrorInvalidValue;    // s_w holds at most 256 output rows
  if (dr == 32) hipLaunchKernelGGL(attn_merge_kernel<32>, dim3(B, 4, 1), dim3(1024), 0, s, part, ntile, wout, g, C, Aout);
  else if (dr == 4) hipLaunchKernelGGL(attn_merge_kernel<4>, dim3(B, 4, 8), dim3(1024), 0, s, part, ntile, wout, g, C, Aout);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_attn_fold(int act_bf16, const float* Ain, const float* wqt, int B, int C, void* Mw, hipStream_t s) {
  if (C % 64 != 0) return hipErrorInvalidValue;
  const WImg W = conv_wimg(act_bf16, 1, C, C);
  const dim3 grid(B, C / 64, C / 64);
  if (act_bf16) hipLaunchKernelGGL(attn_fold_kernel<bf16>, grid, dim3(256), 0, s, Ain, wqt, C, (char*)Mw, W);
  else hipLaunchKernelGGL(attn_fold_kernel<float>, grid, dim3(256), 0, s, Ain, wqt, C, (char*)Mw, W);
  return hipGetLastError();
}

}  // namespace gt
