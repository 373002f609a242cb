// Shared device helpers for the gfx950 (CDNA4) Grad-TTS decoder kernels.
//
// Activation storage type `A` is either float (fp32 parity path) or __bf16 (throughput path).
// Every 3x3 / 1x1 / transposed convolution of the score U-Net is an implicit GEMM on MFMA:
//   bf16 : v_mfma_f32_32x32x16_bf16   (one instruction per 16-channel k-step)
//   fp32 : v_mfma_f32_32x32x2_f32     (exact f32, eight instructions per 16-channel k-step)
// Both flavours read their operand fragments as "8 contiguous channels at byte offset 8*h*sizeof(A)"
// (h = lane >> 5); for fp32 the 16-channel step is split so that the k index of sub-step s, half h is
// channel 8h+s on BOTH operands (the k order inside a step is free as long as A and B agree).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define GT_DEV __device__ __forceinline__

// ---------------------------------------------------------------- numerics
// Mish (model/diffusion.py:16-18) = x * tanh(softplus(x)); torch softplus returns x for x > 20.
// tanh(log1p(e^x)) = n / (n + 2) with n = e^x (e^x + 2): one exp + one divide.
// For x > 20 the clamp keeps e finite and n/(n+2) rounds to 1, i.e. Mish(x) = x as torch's threshold gives.
GT_DEV float mishf(float x) {
  const float e = __expf(fminf(x, 20.f));
  const float n = e * (e + 2.f);
  return x * (n * __builtin_amdgcn_rcpf(n + 2.f));   // v_rcp_f32 (1 ulp): __fdividef lowered to the IEEE divide
}
// Mish for a bf16 activation path: tanh(softplus(x)) = 1 - 2 / ((e^x + 1)^2 + 1) -> one exp2, one rcp, four
// FMA-class ops (the gn_mish_tb_l2 form below, without its folded affine). e^x = inf gives x (torch's threshold); absolute error <= |x| 2^-23
// (cancellation for x << 0), far below the bf16 rounding of the result. fp32 paths keep mishf.
template <class A> GT_DEV float mish_act(float x) { return mishf(x); }
template <> GT_DEV float mish_act<bf16>(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 1.44269504088896341f);
  const float t = e + 1.f;
  return x * __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(__builtin_fmaf(t, t, 1.f)), 1.f);
}

// Block-conv operand transform of the bf16 / fp8 paths, Mish(GN(h)) + tb (diffusion.py:57-58, 76), in base 2: with the
// GroupNorm affine's coefficients pre-scaled by log2(e), yl = log2(e) y = fma(h, sc, sh), and
//   Mish(y) = y (1 - 2 / ((1 + e^y)^2 + 1)) = yl (ln2 - 2 ln2 / ((1 + 2^yl)^2 + 1)),
// so the whole transform is fma(yl, fma(-2 ln2, rcp((1 + 2^yl)^2 + 1), ln2), tb): five FMA-class ops, one exp2 and
// one rcp (the mish_act<bf16> form plus the separate affine, time-bias add and log2(e) scaling took eight).
// 2^yl = inf gives yl ln2 = y (torch's softplus threshold); 2^yl = 0 gives tb.
constexpr float kLog2e = 1.44269504088896341f, kLn2 = 0.69314718055994531f;
GT_DEV float gn_mish_tb_l2(float h, float sc_l2, float sh_l2, float tb) {
  const float yl = __builtin_fmaf(h, sc_l2, sh_l2);
  const float t = __builtin_amdgcn_exp2f(yl) + 1.f;
  const float r = __builtin_amdgcn_rcpf(__builtin_fmaf(t, t, 1.f));
  return __builtin_fmaf(yl, __builtin_fmaf(-2.f * kLn2, r, kLn2), tb);
}

// ResnetBlock output with identity residual (diffusion.py:57-58, 77-79), Mish(GN(h)) * m + x * m = (Mish(GN(h)) + x) * m.
// The bf16 paths take the base-2 form of gn_mish_tb_l2 with the residual as its addend (GroupNorm coefficients
// pre-scaled by log2 e, gn_res_coef): 5 FMA-class ops, exp2, rcp and the mask multiply per element, where the mish_act
// form took 9 and the two transcendentals. fp32 keeps the reference formula.
template <class A> GT_DEV void gn_res_coef(float&, float&) {}
template <> GT_DEV void gn_res_coef<bf16>(float& sc, float& sh) { sc *= kLog2e; sh *= kLog2e; }
template <class A> GT_DEV float gn_mish_res(float h, float sc, float sh, float x, float m) {
  return mish_act<A>(h * sc + sh) * m + x * m;
}
template <> GT_DEV float gn_mish_res<bf16>(float h, float sc_l2, float sh_l2, float x, float m) {
  return gn_mish_tb_l2(h, sc_l2, sh_l2, x) * m;
}
// ResnetBlock output with a res_conv residual r (unmasked: res_conv(x * m)), Mish(GN(h)) * m + r (diffusion.py:78);
// bf16: the base-2 Mish (coefficients from gn_res_coef), then one FMA
template <class A> GT_DEV float gn_mish_add(float h, float sc, float sh, float r, float m) {
  return mish_act<A>(h * sc + sh) * m + r;
}
template <> GT_DEV float gn_mish_add<bf16>(float h, float sc_l2, float sh_l2, float r, float m) {
  return __builtin_fmaf(gn_mish_tb_l2(h, sc_l2, sh_l2, 0.f), m, r);
}

// ---------------------------------------------------------------- storage
template <class A> struct Act;
template <> struct Act<float> {
  static constexpr int kItemCh = 4;  // channels per 16-byte item
  GT_DEV static float to_f(float v) { return v; }
  GT_DEV static float from_f(float v) { return v; }
};
template <> struct Act<bf16> {
  static constexpr int kItemCh = 8;
  GT_DEV static float to_f(bf16 v) { return (float)v; }
  GT_DEV static bf16 from_f(float v) { return (bf16)v; }
};

// 16-byte item <-> float[kItemCh]
GT_DEV void item_to_f(const uint4& u, float* f, float) {
  f[0] = __uint_as_float(u.x); f[1] = __uint_as_float(u.y); f[2] = __uint_as_float(u.z); f[3] = __uint_as_float(u.w);
}
GT_DEV uint4 f_to_item(const float* f, float) {
  return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
}
GT_DEV void item_to_f(const uint4& u, float* f, bf16) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
// one v_cvt_pk_bf16_f32 (round to nearest even) for the pair; two scalar (bf16) casts cost four instructions
// (two half-empty converts, a shift and an or) -- a quarter of the VALU work of some operand transforms
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
GT_DEV uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}
GT_DEV uint4 f_to_item(const float* f, bf16) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
}

// ---------------------------------------------------------------- MFMA traits
template <class A> struct Mma;
template <> struct Mma<bf16> {
  typedef bf16x8 frag;
  GT_DEV static frag load(const char* p) { return *reinterpret_cast<const frag*>(p); }
  GT_DEV static void mma(const frag& a, const frag& b, f32x16& c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  struct frag { f32x4 lo, hi; };
  GT_DEV static frag load(const char* p) {
    frag f;
    f.lo = *reinterpret_cast<const f32x4*>(p);
    f.hi = *reinterpret_cast<const f32x4*>(p + 16);
    return f;
  }
  GT_DEV static void mma(const frag& a, const frag& b, f32x16& c) {
#pragma unroll
    for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.lo[s], b.lo[s], c, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.hi[s], b.hi[s], c, 0, 0, 0);
  }
};

// Row (within a 32x32 accumulator block) held by register j of lane half h (CDNA4 C/D map:
// col = lane & 31, row = (j & 3) + 8 * (j >> 2) + 4 * h).
GT_DEV int acc_row(int j, int h) { return (j & 3) + 8 * (j >> 2) + 4 * h; }

// ---------------------------------------------------------------- cross-lane sums
// Sum of x over the 16-lane row (every lane, fixed order): DPP row rotations by 1, 2, 4, 8
GT_DEV float row_sum16(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xf, 0xf, false));
  return x;
}
// Sum over the 32 lanes of this half-wave, valid in lanes 0 and 32: row sums, then rows 1/3 brought down to
// rows 0/2 by v_permlane16_swap
GT_DEV float half_sum32(float x) {
  const float s = row_sum16(x);
  const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return s + __uint_as_float(sw[1]);
}

// ---------------------------------------------------------------- GroupNorm statistics
// GroupNorm (model/diffusion.py:53, 8 groups, eps 1e-5) normalises over (C/8) x F x T -- every grid
// position, padded frames included. The producing conv writes, per workgroup, the fp32 sum and sum of
// squares of each of the 8 groups it touches into its own slot
//     part[(b * nparts + slot) * 16 + g * 2 + {0,1}]      (plain stores, no atomics, no memset)
// and every consumer reduces the slots of its utterance in a fixed order in fp64: deterministic,
// and independent of how many utterances share the launch.
// Reduction in two halves so callers can overlap other loads with the slot loads:
//   GnLoad gl = gn_load(part, nparts, b);     issues this thread's slot loads (threads 0..255)
//   gn_finish(gl, ...);                        fp64 sums in a fixed order -> s_mean / s_rstd (LDS)
// Thread t reads value k = t & 15 of slots t>>4, t>>4 + 16, ... (GN_Q at once, coalesced 64-B rows); the
// 256 fp64 partials are then summed per value by 16 threads in slot-group order. The order depends only
// on nparts: deterministic and independent of the launch. Call with all threads of the block (>= 256).
// Workgroup barrier that orders LDS only (no memory-model fence: outstanding global loads, e.g. a
// prefetch, stay in flight).
GT_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

constexpr int GN_Q = 24;   // slot loads per thread issued up front: 16 thread groups x 24 = 384 slots per utterance
struct GnLoad {
  float v[GN_Q];
};
// t: the calling thread's index among the 256 that take part (default threadIdx.x; a 512-thread workgroup running two
// independent 256-thread halves passes threadIdx.x & 255 -- both halves then call gn_finish, whose barriers they share)
GT_DEV GnLoad gn_load(const float* part, int nparts, int b, int t = -1) {
  GnLoad g;
  if (t < 0) t = threadIdx.x;
  const int k = t & 15, grp = t >> 4;
  const float* pb = part + (long)b * nparts * 16 + k;
#pragma unroll
  for (int q = 0; q < GN_Q; ++q) {
    const int i = grp + 16 * q;
    g.v[q] = (t < 256 && i < nparts) ? pb[(long)i * 16] : 0.f;
  }
  return g;
}
// s_red: LDS scratch of >= 272 doubles
GT_DEV void gn_finish(const GnLoad& g, const float* part, int nparts, int b, long count, float* s_mean, float* s_rstd,
                      double* s_red, int t = -1) {
  if (t < 0) t = threadIdx.x;
  const int k = t & 15, grp = t >> 4;
  if (t < 256) {
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < GN_Q; ++q) acc += (double)g.v[q];
    // slots past the first 16 * GN_Q (long utterances): 8 loads in flight per round, same ascending order
    for (int i0 = grp + 16 * GN_Q; i0 < nparts; i0 += 16 * 8) {
      float w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 16 * u;
        w[u] = i < nparts ? part[((long)b * nparts + i) * 16 + k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (double)w[u];
    }
    s_red[t] = acc;
  }
  lds_barrier();
  if (t < 16) {
    double a = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) a += s_red[q * 16 + t];
    s_red[256 + t] = a;
  }
  lds_barrier();
  if (t < 8) {
    const double mean = s_red[256 + 2 * t] / (double)count;
    double var = s_red[256 + 2 * t + 1] / (double)count - mean * mean;
    var = var > 0.0 ? var : 0.0;
    s_mean[t] = (float)mean;
    s_rstd[t] = (float)(1.0 / sqrt(var + 1e-5));
  }
  lds_barrier();
}
GT_DEV void gn_reduce(const float* part, int nparts, int b, long count, float* s_mean, float* s_rstd, double* s_red) {
  const GnLoad g = gn_load(part, nparts, b);
  gn_finish(g, part, nparts, b, count, s_mean, s_rstd, s_red);
}

// per-channel affine of the normalisation: y = x * scale + shift
GT_DEV void gn_affine(const float* s_mean, const float* s_rstd, int C, int c, const float* gamma, const float* beta,
                      float& scale, float& shift) {
  const int g = c / (C / 8);
  scale = gamma[c] * s_rstd[g];
  shift = beta[c] - s_mean[g] * scale;
}

GT_DEV float mask_at(const float* mask, int T0, int b, int t, int lvl) { return mask[(long)b * T0 + ((long)t << lvl)]; }
