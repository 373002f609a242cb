// 3x3 stride-1 convolution of the score U-Net (Block.block[0], model/diffusion.py:52) on bf16 MFMA with an
// all-LDS-DMA staging pipeline -- the throughput path for every 3x3 conv whose input needs no transform
// (plain activations, or x*mask with a 0/1 mask, or block2's input after gn_apply).
//
// GEMM view as in conv.hip: M = 4 mel rows x TT frames of one utterance, N = NT output channels, K = 9 taps
// x Cin in 16-channel stages. 8 waves (one workgroup per CU, 2 waves per SIMD): WN = NT/64 column groups x
// WM row groups; each wave owns RBW 32-position blocks x 64 channels (v_mfma_f32_32x32x16_bf16).
//
// Stage s (channels 16s .. 16s+15) lives in LDS as two images, both written by LDS-DMA only:
//   patch   : two half-planes (channels 0-7 / 8-15), each [6 rows x (TT+2) cols] x 16 B, filled with
//             buffer_load_dwordx4 ... lds at per-lane byte offsets computed once per workgroup. Padding
//             positions and masked frames (mask 0) get an offset past the end of the tensor: the buffer
//             range check returns zeros, which is exactly the conv's zero padding and x*mask.
//   weights : the packed v4 image (decoder.cpp pack_conv4): [half][tap][NT] x 16 B, global_load_lds.
// Consecutive lanes of an MFMA fragment read consecutive 16-B units of one half-plane, so every
// ds_read_b128 lane group covers 16 distinct bank slots (conflict-free without padding, which lane-linear
// DMA could not express).
// Pipeline: NS-stage ring; stage s+NS-1 is issued right after the barrier that ends stage s-1's reads;
// one raw barrier per stage (s_waitcnt lgkmcnt(0); s_barrier -- __syncthreads() would drain every
// LDS-DMA in flight), each wave waits with a counted vmcnt for its own pieces of stage s only.
// Epilogue: as conv.hip (per-wave LDS transposition, bias, GroupNorm partial sums to this tile's slot).
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "wimage.h"

namespace gt {

template <int NT, int TT, int NW, int NS>
struct C4 {
  static constexpr int TF = 4, PR = TF + 2, PC = TT + 2, NPOS = PR * PC;
  static constexpr int PPP = (NPOS + 63) / 64;              // patch pieces (1 KiB) per half-plane
  static constexpr int PLANE_B = PPP * 1024;
  static constexpr int PATCH_B = 2 * PLANE_B;
  static constexpr int WPLANE_B = conv4_wplane_bytes(NT);
  static constexpr int W_B = 2 * WPLANE_B;                    // NT*9*32: a whole number of KiB
  static constexpr int PIECES = 2 * PPP + W_B / 1024;
  static constexpr int STAGE_B = PATCH_B + W_B;
  static constexpr int MAXPW = (PIECES + NW - 1) / NW;        // pieces per wave (upper bound)
  static constexpr int WN = NT / 64, WM = NW / WN;
  static constexpr int RBT = TT / 32, NBLK = TF * RBT, RBW = NBLK / WM;
  static constexpr int EPI_ROW = 36, EPI_B = NW * 32 * EPI_ROW * 4;
  static constexpr int RING_B = NS * STAGE_B > EPI_B ? NS * STAGE_B : EPI_B;
  static constexpr int SMEM = RING_B + (NT + NW * 16 + 16) * 4;
  static_assert(W_B % 1024 == 0, "weight slab is whole pieces");
  static_assert(NBLK % WM == 0, "blocks per wave");
  static_assert(SMEM <= 160 * 1024, "LDS budget");
};

// buffer_load_dwordx4 ... lds behind a device-only function: with a runtime voffset written directly in
// the kernel body, hipcc (ROCm 7.2) silently drops the kernel's host launch stub (link error).
GT_DEV void buf_lds16(__amdgpu_buffer_rsrc_t rs, char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

GT_DEV void vm_wait(int n) {   // s_waitcnt vmcnt(n) for a wave-uniform runtime n (immediate operand)
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;   // conservative
  }
}

template <int NT, int TT, int NW, int NS>
__global__ __launch_bounds__(512) void conv4_kernel(ConvParams p) {   // blockDim = 64 * NW <= 512
  typedef C4<NT, TT, NW, NS> C;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];   // ONE LDS object (guide §5, trap 4a)
  char* ring = smem;
  float* s_bias = reinterpret_cast<float*>(smem + C::RING_B);
  float* s_sub = s_bias + NT;                                    // [NW][2 cb][4 g8][2]

  const int Fg = p.Fout, Tg = p.Tout;
  const int n_ft = Fg / C::TF, n_tt = (Tg + TT - 1) / TT;
  int bid = blockIdx.x;
  const int tt = bid % n_tt; bid /= n_tt;
  const int ft = bid % n_ft;
  const int b = bid / n_ft;
  const int f0 = ft * C::TF, t0 = tt * TT;
  const int ntile = blockIdx.y, cout0 = ntile * NT;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  // wave index as a provably wave-uniform (SGPR) value: piece loops and the counted waits stay scalar
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv % C::WM, wn = wv / C::WM;

  if (tid < NT) s_bias[tid] = p.bias[cout0 + tid];

  // ---- this wave's DMA pieces: k = wv + NW*j (k < 2*PPP: patch half-plane k/PPP; else weights)
  const int npos = p.B * p.Fin * p.Tin;
  const int cnt = (C::PIECES - wv + NW - 1) / NW;                // pieces per stage of this wave
  int pidx[C::MAXPW];
#pragma unroll
  for (int j = 0; j < C::MAXPW; ++j) {
    const int k = wv + NW * j;
    int q = -1;
    if (k < 2 * C::PPP) {
      const int pos = (k % C::PPP) * 64 + lane;
      const int pr = pos / C::PC, pc = pos - pr * C::PC;
      const int fi = f0 - 1 + pr, ti = t0 - 1 + pc;
      bool ok = pos < C::NPOS && fi >= 0 && fi < p.Fin && ti >= 0 && ti < p.Tin;
      if (ok && p.mask_in) ok = mask_at(p.mask, p.T0, b, ti, p.lvl_in) != 0.f;   // 0/1 mask (host-checked)
      q = ok ? (b * p.Fin + fi) * p.Tin + ti : -1;
    }
    pidx[j] = q;
  }
  int poff[C::MAXPW];
  auto set_offsets = [&](int Cs) {
#pragma unroll
    for (int j = 0; j < C::MAXPW; ++j) {
      const int k = wv + NW * j;
      poff[j] = pidx[j] >= 0 ? pidx[j] * (Cs * 2) + (k / C::PPP) * 16 : 0x7ff00000;
    }
  };
  set_offsets(p.C0);
  __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.in0, (short)0, npos * p.C0 * 2, 0x00020000);
  __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.in1 ? p.in1 : p.in0), (short)0, npos * (p.in1 ? p.C1 : p.C0) * 2, 0x00020000);
  const int nchunk = p.Cin / 16;
  const char* wimg = reinterpret_cast<const char*>(p.w) + (long)ntile * nchunk * C::W_B + lane * 16;

#define CONV4_DMA(ST, BUF)                                                                                    \
  do {                                                                                                        \
    char* base_ = ring + (BUF) * C::STAGE_B;                                                                  \
    const int c0_ = (ST) * 16;                                                                                \
    const bool second_ = c0_ >= p.C0;                                                                         \
    const int soff_ = (second_ ? c0_ - p.C0 : c0_) * 2;                                                       \
    _Pragma("unroll") for (int j = 0; j < C::MAXPW; ++j) {                                                    \
      const int k = wv + NW * j;                                                                              \
      if (k >= C::PIECES) break;                                                                              \
      if (k < 2 * C::PPP) {                                                                                   \
        buf_lds16(second_ ? rs1 : rs0, base_ + k * 1024, poff[j], soff_);                                     \
      } else {                                                                                                \
        __builtin_amdgcn_global_load_lds((const void*)(wimg + (long)(ST) * C::W_B + (k - 2 * C::PPP) * 1024), \
                                         (__attribute__((address_space(3))) void*)(base_ + k * 1024), 16, 0, 0); \
      }                                                                                                       \
    }                                                                                                         \
  } while (0)
  auto lds_sync = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  f32x16 acc[C::RBW][2];
#pragma unroll
  for (int i = 0; i < C::RBW; ++i)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][c][k] = 0.f;

  const bool switch_src = p.C1 != 0 && p.C1 != p.C0;
  int issued = 0;
  for (; issued < NS - 1 && issued < nchunk; ++issued) {
    if (switch_src && issued * 16 == p.C0) set_offsets(p.C1);
    CONV4_DMA(issued, issued % NS);
  }
  for (int st = 0; st < nchunk; ++st) {
    const int after = (issued - 1) - st;                          // stages issued after st (in flight)
    vm_wait(after * cnt);                                         // this wave's pieces of stage st landed
    lds_sync();                                                   // everyone's landed; stage st-1 reads done
    if (issued < nchunk) {                                        // into the buffer stage st-1 used
      if (switch_src && issued * 16 == p.C0) set_offsets(p.C1);
      CONV4_DMA(issued, issued % NS);
      ++issued;
    }
    const char* pa = ring + (st % NS) * C::STAGE_B;
    const char* pw = pa + C::PATCH_B;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dr = tap / 3, dc = tap - 3 * dr;
      bf16x8 bfr[2], af[C::RBW];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
        bfr[cb] = *reinterpret_cast<const bf16x8*>(pw + h * C::WPLANE_B + (tap * NT + wn * 64 + cb * 32 + r) * 16);
#pragma unroll
      for (int rb = 0; rb < C::RBW; ++rb) {
        const int bi = wm * C::RBW + rb, lrow = bi / C::RBT, tblk = bi % C::RBT;
        af[rb] = *reinterpret_cast<const bf16x8*>(pa + h * C::PLANE_B + ((lrow + dr) * C::PC + tblk * 32 + r + dc) * 16);
      }
#pragma unroll
      for (int rb = 0; rb < C::RBW; ++rb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[rb], bfr[cb], acc[rb][cb], 0, 0, 0);
    }
  }

  // ---- epilogue: transpose each 32x32 block through the wave's own LDS scratch (lane = position, 8
  // channels), bias, 16-B stores, GroupNorm partial sums. No global loads: stores never wait.
  lds_sync();                                                     // the ring is free
  auto wave_sync = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  float* scr = reinterpret_cast<float*>(ring) + wv * 32 * C::EPI_ROW;
  const int g8 = lane & 3;
  float gs[2] = {0.f, 0.f}, gq[2] = {0.f, 0.f};
  bf16* out = reinterpret_cast<bf16*>(p.out);
#pragma unroll
  for (int rb = 0; rb < C::RBW; ++rb) {
    const int bi = wm * C::RBW + rb, lrow = bi / C::RBT, tblk = bi % C::RBT;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
      for (int j = 0; j < 16; ++j) scr[acc_row(j, h) * C::EPI_ROW + r] = acc[rb][cb][j];
      wave_sync();
      const int cl = wn * 64 + cb * 32 + g8 * 8;
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(s_bias + cl);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(s_bias + cl + 4);
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int pos = (lane >> 2) + 16 * half;
        const int tc = t0 + tblk * 32 + pos;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(scr + pos * C::EPI_ROW + g8 * 8);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(scr + pos * C::EPI_ROW + g8 * 8 + 4);
        float v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) { v[k] = lo[k] + b0[k]; v[4 + k] = hi[k] + b1[k]; }
        if (tc < Tg) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { gs[cb] += v[k]; gq[cb] += v[k] * v[k]; }
          const long o = (((long)b * p.Fout + f0 + lrow) * p.Tout + tc) * p.Cout + cout0 + cl;
          *reinterpret_cast<uint4*>(out + o) = f_to_item(v, bf16());
        }
      }
      wave_sync();
    }
  }
  auto ror4 = [](float x) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xf, 0xf, false)); };
  auto ror8 = [](float x) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xf, 0xf, false)); };
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {   // over the wave's positions: 16 lanes with equal lane&3
    float s = gs[cb], q = gq[cb];
    s += ror4(s); q += ror4(q);
    s += ror8(s); q += ror8(q);
    s += __shfl_xor(s, 16); q += __shfl_xor(q, 16);
    s += __shfl_xor(s, 32); q += __shfl_xor(q, 32);
    if (lane < 4) {
      s_sub[((wv * 2 + cb) * 4 + lane) * 2 + 0] = s;
      s_sub[((wv * 2 + cb) * 4 + lane) * 2 + 1] = q;
    }
  }
  lds_sync();
  if (tid < 8) {   // per GroupNorm group, fixed order over waves / blocks / 8-channel groups
    const int gshift = __builtin_ctz(p.Cout >> 3);
    float S = 0.f, Q = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = cout0 + (w / C::WM) * 64 + cb * 32 + g * 8;
          if ((co >> gshift) == tid) {
            S += s_sub[((w * 2 + cb) * 4 + g) * 2 + 0];
            Q += s_sub[((w * 2 + cb) * 4 + g) * 2 + 1];
          }
        }
    const int nparts = n_ft * n_tt * gridDim.y;
    const int slot = (ft * n_tt + tt) * gridDim.y + ntile;
    float* dst = p.out_part + ((long)b * nparts + slot) * 16 + tid * 2;
    dst[0] = S;
    dst[1] = Q;
  }
}

// ---- host side ----
Conv4Cfg conv4_pick(int Cout) {
  // GT_CONV4_CFG = "nt,tt,nw,ns" forces one configuration for every layer (tuning runs); the weight
  // images are packed with the same choice (decoder.cpp pack_conv4).
  static const char* forced = getenv("GT_CONV4_CFG");
  Conv4Cfg c;
  if (forced && sscanf(forced, "%d,%d,%d,%d", &c.nt, &c.tt, &c.nw, &c.ns) == 4) {
    if (c.nt > Cout) c.nt = 64;
    return c;
  }
  if (Cout >= 128) { c.nt = 128; c.tt = 64; c.ns = 2; }
  else { c.nt = 64; c.tt = 128; c.ns = 3; }
  c.nw = 8;
  return c;
}

int conv4_nparts(int F, int T, int Cout, Conv4Cfg c) { return (F / 4) * ((T + c.tt - 1) / c.tt) * (Cout / c.nt); }

template <int NT, int TT, int NW, int NS>
static hipError_t launch4(const ConvParams& p, hipStream_t s) {
  typedef C4<NT, TT, NW, NS> C;
  dim3 grid((unsigned)(p.B * (p.Fout / C::TF) * ((p.Tout + TT - 1) / TT)), (unsigned)(p.Cout / NT));
  hipLaunchKernelGGL((conv4_kernel<NT, TT, NW, NS>), grid, dim3(NW * 64), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_conv4(const ConvParams& p, Conv4Cfg c, hipStream_t s) {
  if (p.Fout != p.Fin || p.Tout != p.Tin || p.Fout % 4 != 0 || p.Cout % c.nt != 0 || p.Cin % 16 != 0 ||
      p.C0 % 16 != 0 || p.C1 % 16 != 0 || (p.Cout >> 3) & ((p.Cout >> 3) - 1))
    return hipErrorInvalidValue;
  if ((long)p.B * p.Fin * p.Tin * (p.C0 > p.C1 ? p.C0 : p.C1) * 2 >= (1L << 31)) return hipErrorInvalidValue;
#define CFG(NT_, TT_, NW_, NS_) \
  if (c.nt == NT_ && c.tt == TT_ && c.nw == NW_ && c.ns == NS_) return launch4<NT_, TT_, NW_, NS_>(p, s);
  CFG(64, 128, 8, 3) CFG(64, 64, 8, 3) CFG(128, 64, 8, 2) CFG(128, 128, 8, 2) CFG(64, 64, 4, 2) CFG(64, 128, 4, 2)
#undef CFG
  return hipErrorNotSupported;
}

#undef CONV4_DMA

}  // namespace gt
