// 1x1 convolutions of the throughput plan, streamed: ResnetBlock.res_conv with the block output formed in the epilogue
// (diffusion.py:70, 77-78: Mish(GN(h2)) * m + res_conv(x * m)) and the folded LinearAttention output with its residual
// (diffusion.py:108: x + M_b x + g b_out, decoder.cpp attention_out).
//
// These are HBM-bound: K = 64..512 input channels per position, 2 Cin Cout FLOP against (Cin + 2 Cout) * 2 bytes (the
// ridge point of bf16 MFMA against HBM is ~310 FLOP/B). conv_kernel ran them as 3x3-style tiles, walking K in 32-channel
// chunks: per chunk it read 64 B of every position of its tile (half a cache line, the other half a chunk later, by
// then often evicted), re-read the residual in the epilogue, and kept one chunk in flight (r06 PMC: waves waiting
// 54-57 % of their cycles, 2.6-4.4 TB/s). Here the roles are swapped to match the data:
//   * weights resident in VGPRs: wave w of a workgroup owns 32 output channels (NT = 64 / 128: 2 / 4 waves per
//     position block) and holds all Cin / 16 of its MFMA A fragments for the workgroup's lifetime (Cin / 4 VGPRs);
//   * positions streamed: a stage is 32 (NT = 128) or 64 (NT = 64) consecutive positions of one utterance with ALL
//     their input channels -- one contiguous run of HBM -- plus, for the ResnetBlock output, the h2 pre-activation of
//     the tile's output channels. It goes global -> LDS by global_load_lds (no VGPRs), 16-B slots with one pad slot per
//     position row (odd 16-B stride: conflict-free fragment reads); a ring of 3-8 stages filling the LDS, all but one
//     in flight, one barrier per stage;
//   * the residual of the attention output is the staged input itself (Cin == Cout): read once;
//   * persistent: B x (Cout / NT) x P workgroups fill the CUs once; workgroup (b, part) streams a contiguous range of
//     utterance b's positions (the attention's M_b and the GroupNorm of h2 are per utterance), its channel tiles on one
//     XCD (neighbouring ids) so the second reads the stage from L2.
// Every per-accumulator MFMA sequence is conv_kernel's (32x32x16 bf16, weights as A, 16-channel k-steps ascending over
// all of Cin), and so is the epilogue arithmetic: bit-identical for 0/1 masks (tests/test_conv1s_gpu.py). Input
// positions are loaded unmasked; the epilogue takes m W x + b for IN_MASK with the m = 0 case selected (W 0 + b = b, as
// conv_kernel's zero-loaded operand gives), so a fractional mask (C-ABI callers) scales the fp32 accumulator.
#include "common.h"
#include "kernels.h"
#include "wimage.h"

#include <cstdlib>

namespace gt {
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
namespace c1s {
#ifndef GT_C1S_AUX
#define GT_C1S_AUX 0   // cache policy of the stage DMAs (experiment builds: 2 = nt)
#endif
constexpr int TMAX = 1024;   // frames per row at the conv's level (the mask row kept in LDS)
template <int OUT, int NT, int CIN>
struct Cfg {
  static constexpr int WCO = NT / 32;                 // waves along output channels
  static constexpr int WP = 4 / WCO;                  // 32-position blocks per stage
  static constexpr int PB = 32 * WP;                  // positions per stage
  static constexpr int SP = CIN / 8 + 1;              // 16-B slots per staged input position (odd)
  static constexpr int SPP = OUT == OUT_RBOUT ? NT / 8 + 1 : 0;   // ... per staged h2 position
  static constexpr int SLOTS = PB * (SP + SPP);
  static constexpr int DPW = (SLOTS + 255) / 256;     // global_load_lds wave instructions per wave and stage
  static constexpr int STAGE = DPW * 4 * 1024;
  static constexpr int EXTRA = TMAX * 4 + NT * 3 * 4 + 64;
  // The ring fills the LDS: two workgroups per CU when that leaves >= 3 stages each (same-box A/B: two workgroups with
  // three stages beat one with seven), else one with up to 8.
  static constexpr int S2 = (80 * 1024 - EXTRA) / STAGE;
#ifndef GT_C1S_STORE_AUX
#define GT_C1S_STORE_AUX 0   // cache policy of the output stores (experiment builds: 2 = nt)
#endif
#ifndef GT_C1S_NOSTORE
#define GT_C1S_NOSTORE 0
#endif
#ifndef GT_C1S_ONE_WG
#define GT_C1S_ONE_WG 0   // experiment builds: 1 = one workgroup per CU with the deepest ring everywhere
#endif
  static constexpr int WGCU = S2 >= 3 && !GT_C1S_ONE_WG ? 2 : 1;   // workgroups per CU
  static constexpr int S1 = (160 * 1024 - EXTRA) / STAGE;
  static constexpr int NSTAGE = WGCU == 2 ? (S2 > 8 ? 8 : S2) : (S1 > 8 ? 8 : S1);
  static constexpr int SMEM = NSTAGE * STAGE + EXTRA;
  static_assert(NSTAGE >= 3 && STAGE >= 272 * 8, "a ring of >= 3 stages; GroupNorm scratch fits the last one");
  static_assert((NSTAGE - 2) * DPW <= 63, "the counted wait fits vmcnt");
};
}  // namespace c1s

// byte offset of a __shared__ address in the workgroup's LDS (the operand of ds_read)
__device__ __forceinline__ unsigned lds_off(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p);
}

template <int IN, int OUT, int NT, int CIN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(c1s::Cfg<OUT, NT, CIN>::WGCU))) void conv1s_kernel(ConvParams p, int P) {
  using namespace c1s;
  typedef Cfg<OUT, NT, CIN> C;
  constexpr int NSTAGE = C::NSTAGE;
  constexpr int WROW = conv_wrow(1, 64);                        // 80-B weight rows (wimage.h, 1x1 bf16 image)
  constexpr int WBYTES = conv_habytes(1, NT, 1, 64);            // one 32-channel chunk of one NT-channel tile
  constexpr int KS = CIN / 16;

  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  float* s_mask = reinterpret_cast<float*>(smem + NSTAGE * C::STAGE);
  float* s_sc = s_mask + TMAX;
  float* s_sh = s_sc + NT;
  float* s_bias = s_sh + NT;
  float* s_mean = s_bias + NT;
  float* s_rstd = s_mean + 8;

  // ---- persistent item: (utterance b, part, channel tile); the ny tiles of one (b, part) on one XCD
  const int ny = p.Cout / NT, G = p.B * ny * P, per = (G + 7) >> 3;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= G) return;   // grid padding: the whole workgroup, before any barrier
  const int ntile = L % ny, part = (L / ny) % P, b = L / (ny * P);
  const int n = p.Fout * p.Tout;                                 // positions of one utterance
  const int nb = (n + C::PB - 1) / C::PB;
  const int blk0 = (int)((long)part * nb / P), nst = (int)((long)(part + 1) * nb / P) - blk0;
  const long g0 = (long)b * n + (long)blk0 * C::PB;             // first position of this workgroup
  const long glast = (long)b * n + n - 1;

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wv % C::WCO, wp = wv / C::WCO;
  const int cout0 = ntile * NT;

  // ---- weights: this wave's 32 output channels x all Cin as MFMA A fragments (conv_kernel's image, wimage.h)
  bf16x8 wf[KS];
  {
    const char* wimg = reinterpret_cast<const char*>(p.w) + (long)b * p.w_bstride + (long)ntile * (CIN / 32) * WBYTES +
                       (wc * 32 + r) * WROW + h * 16;
#pragma unroll
    for (int k = 0; k < KS; ++k) wf[k] = *reinterpret_cast<const bf16x8*>(wimg + (long)(k >> 1) * WBYTES + (k & 1) * 32);
  }
  GnLoad gl;
  if (OUT == OUT_RBOUT) gl = gn_load(p.pre_part, p.pre_nparts, b);
  float c_g = 0.f, c_b = 0.f;
  if (OUT == OUT_RBOUT && tid < NT) { c_g = p.pre_gamma[cout0 + tid]; c_b = p.pre_beta[cout0 + tid]; }
  const float c_bias = tid < NT ? p.bias[cout0 + tid] : 0.f;
  constexpr int MQ = TMAX / 256;
  float mrow[MQ];
  if (IN == IN_MASK) {
#pragma unroll
    for (int q = 0; q < MQ; ++q) {
      const int t = tid + 256 * q;
      mrow[q] = t < p.Tout ? mask_at(p.mask, p.T0, b, t, p.lvl_out) : 0.f;
    }
  }

  // ---- stage slots of this thread (wave instruction i = wv + 4 j covers slots 64 i .. 64 i + 63, lane-linear):
  // source tensor (0 in0, 1 in1, 2 h2), position within the stage, byte offset within the position's row
  const char* base[3] = {reinterpret_cast<const char*>(p.in0), reinterpret_cast<const char*>(p.in1 ? p.in1 : p.in0),
                         reinterpret_cast<const char*>(OUT == OUT_RBOUT ? p.pre : p.in0) + cout0 * 2};
  const int rowb[3] = {p.C0 * 2, (p.in1 ? p.C1 : p.C0) * 2, p.Cout * 2};
  // per slot: its source address in this workgroup's first stage, the row stride of its tensor, and how far (in
  // positions) it may advance before passing the utterance's last position (later stages clamp there)
  const char* sp[C::DPW];
  int srow[C::DPW], slim[C::DPW];
#pragma unroll
  for (int j = 0; j < C::DPW; ++j) {
    const int s = 64 * (wv + 4 * j) + lane;
    int code = 0, pos = 0, off = 0;   // pad and scratch slots: a valid address (data never read)
    if (s < C::PB * C::SP) {
      pos = s / C::SP;
      const int ch = (s - pos * C::SP) * 8;
      if (ch < CIN) {
        code = ch < p.C0 ? 0 : 1;
        off = (ch < p.C0 ? ch : ch - p.C0) * 2;
      }
    } else if (OUT == OUT_RBOUT && s < C::SLOTS) {
      const int s2 = s - C::PB * C::SP;
      pos = s2 / C::SPP;
      const int ch = (s2 - pos * C::SPP) * 8;
      code = 2;
      off = ch < NT ? ch * 2 : 0;
    }
    const long lim = glast - g0 - pos;                        // >= 0 unless the first stage already passes the end
    const long g = lim < 0 ? glast : g0 + pos;
    srow[j] = code == 0 ? rowb[0] : code == 1 ? rowb[1] : rowb[2];
    sp[j] = (code == 0 ? base[0] : code == 1 ? base[1] : base[2]) + g * srow[j] + off;
    slim[j] = lim < 0 ? 0 : (int)lim;
  }
  // Stage k of this workgroup -> LDS stage k % NSTAGE. Stages past the end load clamped addresses (valid, never used): every
  // stage issues the same DPW DMAs, so the counted wait below holds on every path.
  auto dma_stage = [&](int k) {
    char* st = smem + (k % NSTAGE) * C::STAGE;
#pragma unroll
    for (int j = 0; j < C::DPW; ++j) {
      const int d = k * C::PB < slim[j] ? k * C::PB : slim[j];
      const char* src = sp[j] + (long)d * srow[j];
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(st + (wv + 4 * j) * 1024),
                                       16, 0, GT_C1S_AUX);
    }
  };
  // Output: raw buffer stores, lanes past the utterance at an offset past the buffer (dropped; no branch around them).
  const __amdgpu_buffer_rsrc_t rso =
      __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, (int)((long)p.B * n * p.Cout * 2), 0x00020000);
  auto store2 = [&](const u32x4* v, const unsigned* off) {
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
#if GT_C1S_NOSTORE   // timing-only experiment build: outputs dropped (wrong results)
      __builtin_amdgcn_raw_buffer_store_b128(v[pr], rso, 0x80000000u, 0, 0);
#else
      __builtin_amdgcn_raw_buffer_store_b128(v[pr], rso, off[pr], 0, GT_C1S_STORE_AUX);
#endif
    }
  };
#pragma unroll
  for (int k = 0; k < NSTAGE - 1; ++k) dma_stage(k);

  if (IN == IN_MASK) {
#pragma unroll
    for (int q = 0; q < MQ; ++q) s_mask[tid + 256 * q] = mrow[q];
  }
  // GroupNorm of h2 (OUT_RBOUT): scratch in the last stage, which no DMA writes before the first stage's barrier
  if (OUT == OUT_RBOUT) {
    gn_finish(gl, p.pre_part, p.pre_nparts, b, p.pre_count, s_mean, s_rstd,
              reinterpret_cast<double*>(smem + (NSTAGE - 1) * C::STAGE));
    if (tid < NT) {
      const int g = (cout0 + tid) / (p.Cout >> 3);
      float sc = c_g * s_rstd[g], sh = c_b - s_mean[g] * sc;
      gn_res_coef<bf16>(sc, sh);   // base 2 (gn_mish_add)
      s_sc[tid] = sc; s_sh[tid] = sh;
    }
  }
  if (tid < NT) s_bias[tid] = c_bias;
  lds_barrier();
  // this lane's 16 output channels' bias (and h2 GroupNorm coefficients) in registers for the workgroup's life
  float rbias[2][8], rsc[2][8], rsh[2][8];
#pragma unroll
  for (int pr = 0; pr < 2; ++pr)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int cl = wc * 32 + pr * 16 + 8 * h + q;
      rbias[pr][q] = s_bias[cl];
      rsc[pr][q] = OUT == OUT_RBOUT ? s_sc[cl] : 0.f;
      rsh[pr][q] = OUT == OUT_RBOUT ? s_sh[cl] : 0.f;
    }

  const int prow = wp * 32 + r;                 // this lane's position within a stage
  for (int k = 0; k < nst; ++k) {
    // Stage k's DMAs are retired by counting only the DMAs issued after them (stages k+1 .. k+NSTAGE-2). The epilogue
    // stores are younger vector-memory ops too, but a store may complete before an older load, so counting on it being
    // outstanding would not be safe (measured: wrong results); a pending store just makes this wait stricter.
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"((NSTAGE - 2) * C::DPW) : "memory");
    lds_barrier();   // stage k landed for every wave; every wave is done with stage (k - 1) % NSTAGE
    const char* st = smem + (k % NSTAGE) * C::STAGE;
    // The epilogue's LDS operands (h2 / residual, mask) are read by inline asm: the compiler cannot tell a plain LDS read
    // of the stage from the pending DMAs' destinations and would drain vmcnt (both stages in flight) in front of it.
    // Stage k's slots are complete (the wait + barrier above). The asm's own lgkmcnt(0) makes its outputs valid when it
    // ends: the compiler treats asm outputs as written at once and may copy them on (with the wait outside, a copy taken
    // before the data landed gave rare wrong elements under load).
    const long gp = g0 + (long)k * C::PB + prow;
    uint4 eu[2];
    float m = 1.f;
    {
      const unsigned sbase = lds_off(st);
      unsigned a[2];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int cl = wc * 32 + pr * 16 + 8 * h;
        a[pr] = sbase + (OUT == OUT_RBOUT ? (C::PB * C::SP + prow * C::SPP) * 16 + cl * 2
                                          : prow * C::SP * 16 + (cout0 + cl) * 2);
      }
      if (IN == IN_MASK) {
        const unsigned am = lds_off(s_mask) + 4u * (unsigned)((gp - (long)b * n) % p.Tout);
        asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b32 %2, %5\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(eu[0]), "=&v"(eu[1]), "=&v"(m) : "v"(a[0]), "v"(a[1]), "v"(am));
      } else {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(eu[0]), "=&v"(eu[1]) : "v"(a[0]), "v"(a[1]));
      }
    }
    dma_stage(k + NSTAGE - 1);
    const char* pa = st + prow * C::SP * 16 + h * 16;
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    bf16x8 fa[2];
    fa[0] = *reinterpret_cast<const bf16x8*>(pa);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {   // one chain, k-steps ascending: conv_kernel's order
      if (ks + 1 < KS) fa[(ks + 1) & 1] = *reinterpret_cast<const bf16x8*>(pa + (ks + 1) * 32);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], fa[ks & 1], acc, 0, 0, 0);
    }
    // ---- epilogue (conv_kernel's: one v_permlane32_swap per register pair leaves lane (r, h) channels
    // wc*32 + 16 pr + 8h + 0..7 of position prow)
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = acc[q];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[8 * pr + q]), __float_as_uint(v[8 * pr + 4 + q]),
                                                         false, false);
        v[8 * pr + q] = __uint_as_float(sw[0]);
        v[8 * pr + 4 + q] = __uint_as_float(sw[1]);
      }
    u32x4 ov[2];
    unsigned oo[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int cl = wc * 32 + pr * 16 + 8 * h;   // channel within the tile
      const float* b0 = rbias[pr];
      const float* b1 = rbias[pr] + 4;
      float o[8], e[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (IN == IN_MASK) {   // m W x + b; m = 0 selects b (conv_kernel: W 0 + b)
          o[q] = m == 0.f ? b0[q] : fmaf(v[8 * pr + q], m, b0[q]);
          o[4 + q] = m == 0.f ? b1[q] : fmaf(v[8 * pr + 4 + q], m, b1[q]);
        } else {
          o[q] = v[8 * pr + q] + b0[q];
          o[4 + q] = v[8 * pr + 4 + q] + b1[q];
        }
      }
      item_to_f(eu[pr], e, bf16());
      if (OUT == OUT_RBOUT) {
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = gn_mish_add<bf16>(e[q], rsc[pr][q], rsh[pr][q], o[q], m);
      } else {   // residual: the staged input (Cin == Cout)
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] += e[q];
      }
      const uint4 w = f_to_item(o, bf16());
      ov[pr] = u32x4{w.x, w.y, w.z, w.w};
      oo[pr] = gp <= glast ? (unsigned)((gp * p.Cout + cout0 + cl) * 2) : 0x80000000u;
    }
    store2(ov, oo);
  }
  // the tail's DMAs write LDS: drained before the workgroup can end (its LDS is then reallocated)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

namespace {
template <int IN, int OUT, int NT, int CIN>
hipError_t launch1(const ConvParams& p, hipStream_t s) {
  typedef c1s::Cfg<OUT, NT, CIN> C;
  const int ny = p.Cout / NT, n = p.Fout * p.Tout, nb = (n + C::PB - 1) / C::PB;
  int P = (256 * C::WGCU) / (p.B * ny);
  // GT_CONV1S_PARTS (tests): workgroups per (utterance, channel tile), so small batches run many stages per workgroup
  if (const char* e = getenv("GT_CONV1S_PARTS")) P = atoi(e);
  P = P < 1 ? 1 : P > nb ? nb : P;
  const long G = (long)p.B * ny * P;
  hipLaunchKernelGGL((conv1s_kernel<IN, OUT, NT, CIN>), dim3((unsigned)(8 * ((G + 7) / 8))), dim3(256), 0, s, p, P);
  return hipGetLastError();
}
}  // namespace

bool conv1s_eligible(InMode im, OutMode om, const ConvParams& p) {
  const int cin = p.in1 ? p.C0 + p.C1 : p.C0;
  const int nt = conv_nt(1, p.Cout);
  const bool mode = (im == IN_MASK && om == OUT_RBOUT && p.pre && p.pre_part) ||
                    (im == IN_PLAIN && om == OUT_RESID && !p.in1 && cin == p.Cout && (cin == 64 ? nt == 64 : nt == 128));
  return mode && !p.wscale && !p.a8 && p.Fin == p.Fout && p.Tin == p.Tout && p.Tout <= c1s::TMAX &&
         (cin == 64 || cin == 128 || cin == 256 || (cin == 512 && nt == 128)) && p.Cin_pad == cin && p.C0 % 8 == 0 &&
         (p.Cout == 64 || p.Cout % 128 == 0) && p.Cout <= 512 && p.B >= 1 && (long)p.Fout * p.Tout >= 1 &&
         (long)p.B * p.Fout * p.Tout * p.Cout * 2 < (1L << 31);   // (the output's raw buffer range is 32-bit)
}

hipError_t launch_conv1s(InMode im, OutMode om, const ConvParams& p, hipStream_t s) {
  if (!conv1s_eligible(im, om, p)) return hipErrorInvalidValue;
  const int cin = p.in1 ? p.C0 + p.C1 : p.C0;
  const bool n128 = conv_nt(1, p.Cout) == 128;
  if (im == IN_PLAIN) {
    if (cin == 64) return launch1<IN_PLAIN, OUT_RESID, 64, 64>(p, s);
    if (cin == 128) return launch1<IN_PLAIN, OUT_RESID, 128, 128>(p, s);
    if (cin == 256) return launch1<IN_PLAIN, OUT_RESID, 128, 256>(p, s);
    return launch1<IN_PLAIN, OUT_RESID, 128, 512>(p, s);
  }
  if (n128) {
    if (cin == 64) return launch1<IN_MASK, OUT_RBOUT, 128, 64>(p, s);
    if (cin == 128) return launch1<IN_MASK, OUT_RBOUT, 128, 128>(p, s);
    if (cin == 256) return launch1<IN_MASK, OUT_RBOUT, 128, 256>(p, s);
    return launch1<IN_MASK, OUT_RBOUT, 128, 512>(p, s);
  }
  if (cin == 64) return launch1<IN_MASK, OUT_RBOUT, 64, 64>(p, s);
  if (cin == 128) return launch1<IN_MASK, OUT_RBOUT, 64, 128>(p, s);
  return launch1<IN_MASK, OUT_RBOUT, 64, 256>(p, s);
}

}  // namespace gt
