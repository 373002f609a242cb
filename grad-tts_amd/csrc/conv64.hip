// Persistent, register-resident-weight 3x3 convolution for the 64-channel U-Net levels (bf16).
//
// Covers Block.block[0] (model/diffusion.py:52) whenever Cin = Cout = 64: the second conv of the level-0
// ResnetBlocks, the final block (level 0) and the 64-channel up-path blocks at level 1 -- convs that are
// HBM- and MFMA-balanced (≈40 µs each at B = 32, T = 512) but that conv_kernel runs 3-5x slower: each of its
// 5120 short-lived tiles restages the 78 KB weight image from L2 (≈400 MB of L2->LDS traffic per launch) and
// pays its prologue/epilogue for only 4 K-chunks.
//
// Structure (one workgroup of 8 waves per CU, grid = CU count, each workgroup a contiguous run of tiles):
//   * weights live in REGISTERS for the whole launch: wave w owns output channels 32*(w&1) .. +31 and holds
//     their 4 chunks x 9 taps of A fragments (144 VGPRs), loaded once from a fragment-ordered image;
//   * wave w computes mel row (w>>1) of a 4-row x 32-frame sub-tile: one 32x32 accumulator, 36 MFMAs
//     (v_mfma_f32_32x32x16_bf16, weights as A, patch positions as B -> C = channel x position);
//   * the 6 x 34-position input patch (64 channels, 144-B rows: conflict-free fragment reads) is
//     DOUBLE-BUFFERED in LDS: while the MFMAs read sub-tile u from one buffer, the same waves store sub-tile
//     u+1 into the other (from registers, with the producer's GroupNorm apply + Mish + time bias + mask
//     for IN_GN, or x * mask) and issue the raw buffer loads of sub-tile u+2 (padding and past-the-end
//     reads return zeros). One LDS barrier per sub-tile, no weight traffic after the prologue;
//   * epilogue from the accumulators: one v_permlane32_swap per register pair leaves each lane with 8
//     consecutive output channels (= one GroupNorm group) of one position -> bias, 16-B stores and the
//     GroupNorm partial sums (DPP row sums + one v_permlane16_swap), no LDS transposition.
// Tiles of conv_kernel (4 rows x 64 frames) are processed as two 32-frame sub-tiles, so the GroupNorm partial
// slots are exactly conv_kernel's (conv_gn_nparts): producers and consumers are unchanged, and every slot is
// summed in a fixed order (deterministic, batch-invariant).
#include "common.h"
#include "kernels.h"
#include "wimage.h"

namespace gt {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

namespace c64 {
constexpr int TF = 4, TS = 32, PR = TF + 2, PC = TS + 2, NPOS = PR * PC;   // 6 x 34 patch positions
constexpr int POSB = 144;                                                   // 128 B of channels + 16 B pad
constexpr int NTHR = 512, NW = 8;
constexpr int PITEMS = NPOS * 8;                                            // 16-B items: 1632
constexpr int PPT = (PITEMS + NTHR - 1) / NTHR;                             // 4 per thread
constexpr int NCH = 4;                                                      // 16-channel chunks
constexpr int PATCH_B = NPOS * POSB;                                        // 29376
constexpr int SMEM = 2 * PATCH_B + (2 * 4 * 64 + 64 + 2 * NW * 8 + 16) * 4 + 272 * 8;
constexpr int SPH = 4;   // stamps per sub-tile (diagnostics)
static_assert(PATCH_B % 16 == 0, "aligned buffers");
static_assert(SMEM <= 64 * 1024, "LDS budget");
}  // namespace c64

#ifdef GT_C64_STAMPS
// Diagnostic timeline (tools/stamps64.py): s_memtime at phase boundaries of waves 0 and 7 of every workgroup,
// last launch of conv64_kernel<GT_C64_STAMPS> on an 80-row grid.
constexpr int S64_WG = 256, S64_TILES = 48, S64_PH = c64::SPH;
__device__ unsigned long long g_s64[S64_WG * 2 * (2 + S64_TILES * S64_PH)];
#define ST64(k)                                                                                           \
  do {                                                                                                    \
    if (st_on && (lane == 0) && (wv == 0 || wv == 7))                                                    \
      g_s64[(blockIdx.x * 2 + (wv == 7)) * (2 + S64_TILES * S64_PH) + (k)] = __builtin_readcyclecounter(); \
  } while (0)
#else
#define ST64(k) do {} while (0)
#endif

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

// Mish(y) + tb for the bf16 operand path: tanh(softplus(y)) = 1 - 2 / ((e^y + 1)^2 + 1), so
// Mish(y) + tb = y * (1 - 2 r) + tb with r = 1 / ((e^y + 1)^2 + 1): one v_exp_f32, one v_rcp_f32, five FMA-class
// ops. e^y = inf for large y gives r = 0, i.e. y + tb (torch's softplus threshold). Absolute error
// <= |y| * 2^-23 (cancellation in 1 - 2r for y << 0), far below the bf16 rounding of the result.
GT_DEV float mish_tb(float y, float tb) {
  const float e = __builtin_amdgcn_exp2f(y * 1.44269504088896341f);
  const float t = e + 1.f;
  const float r = __builtin_amdgcn_rcpf(__builtin_fmaf(t, t, 1.f));
  return __builtin_fmaf(y, __builtin_fmaf(-2.f, r, 1.f), tb);
}

// IN: IN_MASK / IN_GN / IN_PLAIN; FRAC (IN_MASK only): the mask may hold values other than 0 and 1
template <int IN, bool FRAC>
__global__ __launch_bounds__(512) void conv64_kernel(ConvParams p) {
  using namespace c64;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];   // one LDS object
  char* const sP = smem;                                     // 2 patch buffers
  float* const s_coef = reinterpret_cast<float*>(smem + 2 * PATCH_B);   // [b & 1][scale, shift, tb, unused][64]
  float* const s_bias = s_coef + 2 * 4 * 64;
  float* const s_sub = s_bias + 64;                          // [slot & 1][wave][(pr, h) group][sum, sq]
  float* const s_mean = s_sub + 2 * NW * 8;
  float* const s_rstd = s_mean + 8;
  double* const s_red = reinterpret_cast<double*>(s_rstd + 8);

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, h = lane >> 5;
  const int cb = wv & 1, lrow = wv >> 1;
  const int F = p.Fout, T = p.Tout;
  const int n_ft = F / TF, n_tt = (T + 63) / 64, per_b = n_ft * n_tt;
  const long nslots = (long)p.B * per_b;
  const int s_beg = (int)(nslots * blockIdx.x / gridDim.x), s_end = (int)(nslots * (blockIdx.x + 1) / gridDim.x);
  if (s_beg >= s_end) return;   // whole workgroup (uniform)
  const int u0 = 2 * s_beg, u_end = 2 * s_end;   // sub-tile u = 2 * slot + half
#ifdef GT_C64_STAMPS
  const bool st_on = IN == GT_C64_STAMPS && F == 80 && blockIdx.x < S64_WG && u_end - u0 <= S64_TILES;
#endif
  ST64(0);

  // ---- weights -> registers: A fragment (ch, tap) = output channel cb*32 + r, input channels 16 ch + 8h .. +7,
  // from the fragment-ordered image (decoder.cpp pack_conv64): one contiguous 1 KiB per wave instruction
  bf16x8 wf[NCH][9];
  {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(p.w) + cb * NCH * 9 * 64 + lane;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) wf[ch][tap] = src[(ch * 9 + tap) * 64];
  }
  if (tid < 64) s_bias[tid] = p.bias[tid];
  float c_g = 0.f, c_b = 0.f;
  if (IN == IN_GN && tid < 64) { c_g = p.gn_gamma[tid]; c_b = p.gn_beta[tid]; }

  // ---- patch items: thread tid owns items tid + 512 j (position it/8, 8-channel group it%8 = tid%8)
  const int sub = tid & 7;
  const int npos = p.B * F * T;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.in0, (short)0, npos * 128, 0x00020000);
  u32x4_t preg[PPT];
  float pm[PPT];
  auto coords = [&](int u, int& b, int& ft, int& tt, int& t0) {
    const int slot = u >> 1;
    b = slot / per_b;
    const int rem = slot - b * per_b;
    ft = rem / n_tt;
    tt = rem - ft * n_tt;
    t0 = tt * 64 + (u & 1) * TS;
  };
  // Item j of a sub-tile: issue its load (u past the range: clamped to the last sub-tile, a harmless reload)
  // and store it (transformed per IN) into a patch buffer. One item per K-chunk of the MFMA loop keeps the
  // live transform temporaries to one item.
  struct Sub { int b, fi0, ti0; };
  auto sub_of = [&](int u) {
    u = u < u_end ? u : u_end - 1;
    int b, ft, tt, t0;
    coords(u, b, ft, tt, t0);
    return Sub{b, ft * TF - 1, t0 - 1};
  };
  auto issue_item = [&](int j, const Sub& sb) {
    const int it = tid + NTHR * j;
    const int pos = it >> 3, pr = pos / PC, pc = pos - pr * PC;
    const int fi = sb.fi0 + pr, ti = sb.ti0 + pc;
    const bool ok = it < PITEMS && fi >= 0 && fi < F && ti >= 0 && ti < T;
    const int q = ok ? (sb.b * F + fi) * T + ti : npos;
    preg[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, q * 128 + sub * 16, 0, 0);
    if (IN != IN_PLAIN) {   // unconditional load at a clamped frame, then select (no branch around the load)
      const float mv = mask_at(p.mask, p.T0, sb.b, ti < 0 ? 0 : (ti < T ? ti : T - 1), p.lvl_in);
      pm[j] = ok ? mv : 0.f;
    }
  };
  auto store_item = [&](int j, const Sub& sb, int buf) {
    const int it = tid + NTHR * j;
    u32x4_t v4 = preg[j];
    if (IN == IN_MASK && !FRAC) {
      v4 = pm[j] == 0.f ? u32x4_t{0u, 0u, 0u, 0u} : v4;
    } else if (IN != IN_PLAIN) {
      const float m = pm[j];
      float v[8];
      item_to_f(make_uint4(v4[0], v4[1], v4[2], v4[3]), v, bf16());
      if (IN == IN_GN) {   // (Mish(GN(h)) * m + tb) * m, m in {0,1}  (diffusion.py:57-58, 76)
        const float* cf = s_coef + (sb.b & 1) * 256 + sub * 8;
        const f32x4 sc0 = *reinterpret_cast<const f32x4*>(cf), sc1 = *reinterpret_cast<const f32x4*>(cf + 4);
        const f32x4 sh0 = *reinterpret_cast<const f32x4*>(cf + 64), sh1 = *reinterpret_cast<const f32x4*>(cf + 68);
        const f32x4 tb0 = *reinterpret_cast<const f32x4*>(cf + 128), tb1 = *reinterpret_cast<const f32x4*>(cf + 132);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = mish_tb(v[k] * sc0[k] + sh0[k], tb0[k]);
          v[4 + k] = mish_tb(v[4 + k] * sc1[k] + sh1[k], tb1[k]);
        }
        const uint4 o = f_to_item(v, bf16());
        v4 = m != 0.f ? u32x4_t{o.x, o.y, o.z, o.w} : u32x4_t{0u, 0u, 0u, 0u};
      } else {             // x * m, fractional mask
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= m;
        const uint4 o = f_to_item(v, bf16());
        v4 = u32x4_t{o.x, o.y, o.z, o.w};
      }
    }
    if (PITEMS % NTHR == 0 || it < PITEMS) *reinterpret_cast<u32x4_t*>(sP + buf * PATCH_B + (it >> 3) * POSB + sub * 16) = v4;
  };
  // GroupNorm scale/shift (and time bias) of the input channels for utterance b into set b & 1 (IN_GN)
  auto gn_coefs = [&](int b) {
    const GnLoad gl = gn_load(p.gn_part, p.gn_nparts, b);
    const float tbv = tid < 64 ? p.tb[(long)b * p.tb_bstride + tid] : 0.f;
    gn_finish(gl, p.gn_part, p.gn_nparts, b, p.gn_count, s_mean, s_rstd, s_red);
    if (tid < 64) {
      float* cf = s_coef + (b & 1) * 256;
      const float sc = c_g * s_rstd[tid >> 3];
      cf[tid] = sc; cf[64 + tid] = c_b - s_mean[tid >> 3] * sc; cf[128 + tid] = tbv;
    }
    lds_barrier();
  };

  // ---- prologue: sub-tile u0 into buffer 0, loads of u0 + 1 in flight
  {
    const Sub s0 = sub_of(u0), s1 = sub_of(u0 + 1);
#pragma unroll
    for (int j = 0; j < PPT; ++j) issue_item(j, s0);
    if (IN == IN_GN) gn_coefs(s_beg / per_b);
#pragma unroll
    for (int j = 0; j < PPT; ++j) store_item(j, s0, 0);
#pragma unroll
    for (int j = 0; j < PPT; ++j) issue_item(j, s1);
  }
  lds_barrier();
  ST64(1);

  float gs[2] = {0.f, 0.f}, gq[2] = {0.f, 0.f};   // per-lane GroupNorm partials of the current slot
  for (int u = u0; u < u_end; ++u) {
    const int buf = (u - u0) & 1;
    int b, ft, tt, t0;
    coords(u, b, ft, tt, t0);
    ST64(2 + (u - u0) * SPH + 0);

    f32x16 acc;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = 0.f;
    const char* pa = sP + buf * PATCH_B + (lrow * PC + r) * POSB + h * 16;
    const Sub s1 = sub_of(u + 1), s2 = sub_of(u + 2);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dr = tap / 3, dc = tap - 3 * dr;
        const bf16x8 x = *reinterpret_cast<const bf16x8*>(pa + (dr * PC + dc) * POSB + ch * 32);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ch][tap], x, acc, 0, 0, 0);
      }
      // behind this chunk's MFMAs: stage item ch of sub-tile u+1 into the other buffer, then load it for u+2
      static_assert(PPT == NCH, "one patch item per K-chunk");
      store_item(ch, s1, buf ^ 1);
      issue_item(ch, s2);
    }
    ST64(2 + (u - u0) * SPH + 1);

    // ---- epilogue. Lane (j = r, h) holds channels cb*32 + {0-3, 8-11, 16-19, 24-27} + 4h of position j
    // (registers 0-3, 4-7, 8-11, 12-15); swapping registers 4-7 <-> 0-3 and 12-15 <-> 8-11 across the
    // half-waves leaves lane h with channels cb*32 + 8h + 0..7 (regs 0-7) and cb*32 + 16 + 8h + 0..7 (8-15).
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = acc[k];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[8 * pr + k]), __float_as_uint(v[8 * pr + 4 + k]),
                                                         false, false);
        v[8 * pr + k] = __uint_as_float(sw[0]);
        v[8 * pr + 4 + k] = __uint_as_float(sw[1]);
      }
    const int t = t0 + r;
    const bool valid = t < T;
    bf16* const outp = reinterpret_cast<bf16*>(p.out) + (((long)b * F + ft * TF + lrow) * T + t) * 64;
    const int slot = u >> 1, half = u & 1;
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int c0 = cb * 32 + pr * 16 + 8 * h;   // first of this lane's 8 channels
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(s_bias + c0);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(s_bias + c0 + 4);
      float o[8];
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = v[8 * pr + k] + (k < 4 ? b0[k] : b1[k - 4]);
        s += o[k];
        q += o[k] * o[k];
      }
      if (valid) *reinterpret_cast<uint4*>(outp + c0) = f_to_item(o, bf16());
      // per-lane GroupNorm partials of the slot: half 0, then half 0 + half 1 (fixed order)
      gs[pr] = (half ? gs[pr] : 0.f) + (valid ? s : 0.f);
      gq[pr] = (half ? gq[pr] : 0.f) + (valid ? q : 0.f);
    }
    if (half) {   // slot complete in this wave: group cb*4 + pr*2 + h, summed over its 64 positions
      float* const sub_w = s_sub + (slot & 1) * NW * 8 + wv * 8;
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const float s = half_sum32(gs[pr]), q = half_sum32(gq[pr]);
        if (r == 0) {
          sub_w[(pr * 2 + h) * 2 + 0] = s;
          sub_w[(pr * 2 + h) * 2 + 1] = q;
        }
      }
    }
    ST64(2 + (u - u0) * SPH + 2);
    // coefficients for sub-tile u+2 (staged during the next iteration) when it starts a new utterance
    if (IN == IN_GN && u + 2 < u_end) {
      const int b2 = ((u + 2) >> 1) / per_b;
      if (b2 != ((u + 1) >> 1) / per_b) gn_coefs(b2);   // workgroup-uniform
    }
    lds_barrier();   // buffer u+1 complete, buffer u free, sub-partials visible
    if (half == 1 && tid < 8) {   // slot complete: fixed-order sum over the 4 waves of the group's cb
      const int g = tid, gcb = g >> 2, e = (g & 3) * 2;
      float S = 0.f, Q = 0.f;
#pragma unroll
      for (int lr = 0; lr < 4; ++lr) {
        const float* q = s_sub + (slot & 1) * NW * 8 + (lr * 2 + gcb) * 8 + e;
        S += q[0];
        Q += q[1];
      }
      float* dst = p.out_part + ((long)b * per_b + ft * n_tt + tt) * 16 + g * 2;
      dst[0] = S;
      dst[1] = Q;
    }
    ST64(2 + (u - u0) * SPH + 3);
  }
}

#ifdef GT_C64_STAMPS
extern "C" int gt_debug_read_c64_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_s64), sizeof(g_s64)) == hipSuccess ? 0 : -1;
}
#endif

static int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

bool conv64_eligible(const ConvParams& p) {
  return p.Cin == 64 && p.Cout == 64 && p.Cin_pad == 64 && p.C0 == 64 && p.in1 == nullptr && p.Fin == p.Fout &&
         p.Tin == p.Tout && p.Fout % 4 == 0 && p.wscale == nullptr && p.w_bstride == 0 &&
         (long)p.B * p.Fout * p.Tout * 128 < (1L << 31);
}

hipError_t launch_conv64(InMode im, bool mask01, const ConvParams& p, hipStream_t s) {
  if (!conv64_eligible(p)) return hipErrorInvalidValue;
  const long nslots = (long)p.B * (p.Fout / 4) * ((p.Tout + 63) / 64);
  const unsigned grid = (unsigned)(nslots < cu_count() ? nslots : cu_count());
  if (im == IN_MASK && mask01) hipLaunchKernelGGL((conv64_kernel<IN_MASK, false>), dim3(grid), dim3(512), 0, s, p);
  else if (im == IN_MASK) hipLaunchKernelGGL((conv64_kernel<IN_MASK, true>), dim3(grid), dim3(512), 0, s, p);
  else if (im == IN_GN) hipLaunchKernelGGL((conv64_kernel<IN_GN, false>), dim3(grid), dim3(512), 0, s, p);
  else if (im == IN_PLAIN) hipLaunchKernelGGL((conv64_kernel<IN_PLAIN, false>), dim3(grid), dim3(512), 0, s, p);
  else return hipErrorNotSupported;
  return hipGetLastError();
}

}  // namespace gt
