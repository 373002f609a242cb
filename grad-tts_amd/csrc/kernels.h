// Kernel parameter blocks + host launchers for the Grad-TTS decoder (gfx950).
// Tensor layout in HBM ("frame rows of channel vectors"): an activation at U-Net level l is
// [B][F_l][T_l][C] (channels contiguous), F_l = 80 >> l, T_l = T >> l. The sampler state
// (x_t, mu, z, output) keeps the reference layout [B][80][T] in fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gt {

// IN_RB0 (conv64 only): the input is the first ResnetBlock's output formed in the operand load (ConvParams::rb_*)
// IN_X0 (conv64 only): the input is the first ResnetBlock's block1 output h1, recomputed from {mu, x_t} on the MFMA in the
// operand load (ConvParams::x0w / x0b) and GroupNorm-transformed as IN_GN; its statistics come from launch_x0_stats
enum InMode { IN_INPUT = 0, IN_MASK = 1, IN_GN = 2, IN_PLAIN = 3, IN_RB0 = 4, IN_X0 = 5 };
enum OutMode { OUT_STATS = 0, OUT_PLAIN = 1, OUT_RBOUT = 2, OUT_RESID = 3 };
enum ConvKind { CONV3 = 0, CONV3_S2 = 1, CONV1 = 2, CONVT4 = 3 };

// Time-bias table: one row of kTbRow floats (the 12 ResnetBlocks' mlp(t_emb) slices) per Euler step.
// Step-dependent values are addressed through a device step index (`stepp`, may be null = 0): a captured
// HIP graph of S sampler steps bakes row offsets 0..S-1 into its kernels and is replayed with the index
// advanced between replays (decoder.cpp, graph segments).
constexpr int kTbRow = 1792;
__device__ __forceinline__ const float* tb_at(const float* tb, const int* stepp) {
  return stepp ? tb + (long)(*stepp) * kTbRow : tb;
}

struct ConvParams {
  int B, Fin, Tin, Fout, Tout;   // CONVT4: (Fin,Tin) coarse input grid, (Fout,Tout) = 2x fine grid
  int Cin, Cout, Cin_pad;
  int T0;                        // level-0 frame count (mask row length)
  const float* mask;             // [B][T0]
  int lvl_in, lvl_out;           // mask pyramid level of input / output grid (mask[..., ::2] per level)
  // ---- input
  const void* in0; const void* in1; int C0, C1;      // channels-last sources, concatenated on C
  const float* mu; const float* xt; const float* spk_s; int cin_input;   // IN_INPUT (level 0)
  const float* gn_part; int gn_nparts; const float* gn_gamma; const float* gn_beta; long gn_count;  // IN_GN, IN_RB0
  // IN_RB0 (conv64): in0 is the first ResnetBlock's block2 pre-activation h2 and gn_* its GroupNorm; the operand is
  // its output r0 = Mish(GN(h2))*m + res_conv(x*m) over the U-Net input channels (mu, xt, spk_s; cin_input of them)
  // with rb_w [64][cin] fp32 and rb_b [64]; r0 itself is also written to rb_out ([B][F][T][64] bf16, each position once)
  const float* rb_w; const float* rb_b; void* rb_out;
  // IN_X0 (conv64) and launch_x0_stats: the U-Net input conv (2 channels -> 64) as MFMA A fragments (decoder.cpp pack_x0)
  // and its bias; x0s non-null: the fragments hold e4m3 weight values and x0s the per-output-channel scale
  // (the fp8-weight modes: h1 = (bias / scale + sum) * scale)
  const void* x0w; const float* x0b; const float* x0s;
  const float* tb; long tb_bstride;                   // IN_GN: time bias [.., Cin]; row b*tb_bstride
  const int* stepp;                                   // IN_GN: device step index (tb_at), or null
  // ---- weights
  const void* w; long w_bstride;                      // packed weight image (wimage.h); per-batch stride in BYTES
  const float* wscale;                                // non-null: fp8 e4m3 image (conv_wimg8), per-Cout scale
  int a8;                                             // with wscale: fp8 operands too (conv_wimga8 image, CONV3)
  const float* bias;                                  // [Cout]
  // ---- output
  void* out; float* out_part;                         // OUT_STATS: GroupNorm partials of the output (common.h)
  const void* pre; const float* pre_part; int pre_nparts; const float* pre_gamma; const float* pre_beta; long pre_count;  // OUT_RBOUT
  int small;                     // small-batch tile plan (wimage.h conv_tf; conv64 one-tile segments)
  // split-K of the small plan's 128-wide bf16 3x3 tiles (conv.hip ConvCfg::SK; ignored elsewhere): ksplit <= 1 off;
  // sk_part: fp32 partials [spatial tile][Cout/128][ksplit][8192]; sk_cnt: one zeroed counter per (spatial tile,
  // Cout/128), left zeroed by every launch (the last workgroup of a tile re-arms it)
  int ksplit; float* sk_part; int* sk_cnt;
};
// split count of the small plan's 128-wide 3x3 convs: a function of the utterance's grid and the input chunks only
// (never of the batch, so a small-plan decode stays batch-invariant); 1 = no split
int conv_small_ksplit(int F, int T, int Cout, int Cin_pad, int target, int a8);

hipError_t launch_conv(int act_bf16, ConvKind kind, InMode im, OutMode om, const ConvParams& p, hipStream_t s);
// bf16 1x1 convs of the throughput plan (res_conv + ResnetBlock output: IN_MASK/OUT_RBOUT; attention output + residual:
// IN_PLAIN/OUT_RESID) streamed through an LDS-DMA ring (conv1s.hip); same results as launch_conv for 0/1 masks
bool conv1s_eligible(InMode im, OutMode om, const ConvParams& p);
hipError_t launch_conv1s(InMode im, OutMode om, const ConvParams& p, hipStream_t s);
// number of GroupNorm partial slots per utterance written by a CONV3/OUT_STATS launch on an F x T grid
int conv_gn_nparts(int act_bf16, InMode im, int F, int T, int Cout, int small, int a8 = 0);

struct AttnKVParams {
  const void* x; int B, n, C, Cpad;   // x: [B][n][C] (n = F*T)
  const void* wkv;                    // [256][Cpad]: rows 0..127 = k (head*32+d), 128..255 = v
  int tile_pos, ntile;                // positions per workgroup (multiple of 64), tiles per batch item
  float* part;                        // [B][ntile][4][1088] = {m[32], l[32], ctx[32][32]}
  // rb_pre != null: the attention input is the preceding ResnetBlock's output with identity residual, formed in the
  // operand load, x_in = Mish(GN(rb_pre))*m + x*m (diffusion.py:57-58, 77-79), and written to rb_out for the attention
  // output conv (replaces the separate ResnetBlock-output pass).
  const void* rb_pre; const float* rb_part; int rb_nparts; const float* rb_gamma; const float* rb_beta; long rb_count;
  void* rb_out; const float* mask; int T, T0, lvl;
};
hipError_t launch_attn_kv(int act_bf16, const AttnKVParams& p, hipStream_t s);

// attention output (y = x + M_b x + g b_out, per-utterance 1x1) + Downsample (3x3 stride 2) in one pass, bf16
// (attn_down.hip): level 0 (C = 64; y is never written: hiddens[0] is never read by the up path, diffusion.py:186-201)
struct AttnDownParams {
  const void* x; int B, F, T, C;   // attention input [B][F][T][C] (level-0 grid)
  int T0; const float* mask; int lvl;
  const void* mw; long mw_bstride;  // per-utterance 1x1 weight image M_b (wimage.h conv_wimg(1, 1, C, C)), stride in BYTES
  const float* gb;                  // g * b_out [C]
  const void* wds;                  // downsample weight in fragment order (decoder.cpp pack_frag3x3)
  const float* bds;                 // downsample bias [C]
  const float* wsc;                 // fp8 weights: per-output-channel scale of the e4m3 values in wds (else null)
  void* out;                        // [B][F/2][T/2][C]
};
bool attn_down_eligible(const AttnDownParams& p);
hipError_t launch_attn_down(const AttnDownParams& p, hipStream_t s);

// ups.1's attention output (never read but by the upsample) + Upsample (ConvTranspose 4x4 stride 2) in one pass, bf16,
// C = 64 (attn_down.hip): level-1 input, level-0 output
struct AttnUpParams {
  const void* x; int B, F, T, C;   // attention input [B][F][T][C] (coarse grid)
  int T0; const float* mask; int lvl;
  const void* mw; long mw_bstride;  // per-utterance 1x1 weight image M_b
  const float* gb;                  // g * b_out [C]
  const void* wup;                  // upsample weight, four parities in fragment order (decoder.cpp pack_fragT)
  const float* bup;                 // upsample bias [C]
  const float* wsc;                 // fp8 weights: per-output-channel scale of the e4m3 values in wup (else null)
  void* out;                        // [B][2F][2T][C]
};
bool attn_up_eligible(const AttnUpParams& p);
hipError_t launch_attn_up(const AttnUpParams& p, hipStream_t s);
// dr: rows d per workgroup, 32 (4 tile groups) or 4 (32 tile groups, 8 workgroups per head: small batches)
hipError_t launch_attn_merge(const float* part, int B, int ntile, const float* wout, const float* g, int C, float* Aout,
                             int dr, hipStream_t s);
hipError_t launch_attn_fold(int act_bf16, const float* Ain, const float* wqt, int B, int C, void* Mw, hipStream_t s);   // wqt: W_q^T [C][128]

struct FinalParams {
  const void* pre; const float* part; int nparts; const float* gamma; const float* beta; long count;
  const float* wf; const float* bf;   // final_conv [64], [1]
  const float* mask; int B, T;
  int euler;                          // 0: out = score s; 1: Euler update of xt in place
  float* out; const float* mu; float* xt; float beta_t; float hstep;
  const float* betas; const int* stepp;   // non-null: beta_t = betas[*stepp] (graph segments)
};
hipError_t launch_final(int act_bf16, const FinalParams& p, hipStream_t s);

struct RbOutParams {
  const void* pre; const float* part; int nparts; const float* gamma; const float* beta; long count;
  const void* x; void* out; const float* mask; int B, F, T, C, T0, lvl;
  // rbout_input only: res_conv over the U-Net input channels {mu, x_t, spk} (level 0): fp32 weight [C][cin], bias
  const float* mu; const float* xt; const float* spk_s; int cin;
  const float* rw; const float* rb;
};
hipError_t launch_rbout_identity(int act_bf16, const RbOutParams& p, hipStream_t s);
// the first ResnetBlock's output: Mish(GN(h2))*m + res_conv(x*m) with x = {mu, x_t (, spk)} (2-3 channels, level 0):
// an elementwise pass (the 1x1 conv over 2-3 input channels is 2-3 FMAs per output element)
hipError_t launch_rbout_input(int act_bf16, const RbOutParams& p, hipStream_t s);

struct TembParams {
  int rows; const float* tvals;   // tvals == nullptr: row i is Euler step i of n_steps (t computed on device)
  int n_steps; float pe_scale; const float* freqs;   // freqs [32]
  const float* w0; const float* b0; const float* w2; const float* b2;   // mlp.0 [256][64], mlp.2 [64][256]
  const float* wr; const float* br; int nr;           // stacked ResnetBlock mlp.1: [nr][64], [nr]
  float* tb;                                          // [rows][nr]
  float* betas; float beta_min, beta_delta;           // non-null: betas[row] = beta(t_row) (diffusion.py:262-263)
};
hipError_t launch_temb(const TembParams& p, hipStream_t s);
hipError_t launch_spk_mlp(const float* spk, int B, const float* w0, const float* b0, const float* w2,
                          const float* b2, float* s_out, hipStream_t s);
hipError_t launch_set_step(int* stepp, int v, hipStream_t s);
hipError_t launch_fill_f32(float* p, long n, float v, hipStream_t s);            // (kernel nodes in captures, misc.hip)
hipError_t launch_copy_f32(float* dst, const float* src, long n, hipStream_t s);
hipError_t launch_mask_copy(const float* z, const float* mask, int B, int F, int T, float* out, hipStream_t s);
// debug probe: channels-last activation [B][F][T][C] (act dtype) -> fp32 NCHW [B][C][F][T]
hipError_t launch_to_nchw(int act_bf16, const void* src, int B, int F, int T, int C, float* dst, hipStream_t s);

// weight-resident 3x3 conv for Cin = Cout = 64, bf16 (conv64.hip); GroupNorm partial slots: one per 4 x 32 tile
// (conv64_nparts). conv64_eligible: shape/layout preconditions (no concat, no fp8 image).
int conv64_nparts(int F, int T, int small);
bool conv64_eligible(const ConvParams& p);
hipError_t launch_conv64(InMode im, const ConvParams& p, hipStream_t s);
// The U-Net input conv's GroupNorm statistics without its output (conv64.hip): h1 = conv3x3({mu, x_t} * m) + b over
// every position, recomputed on the MFMA exactly as conv64<IN_X0> recomputes it, summed per 8-channel group into
// x0_stats_nparts slots per utterance (p.out_part); p.out non-null also stores bf16(h1) ([B][F][T][64], diagnostics).
// Preconditions (x0_eligible): 2 input channels, 64 outputs, F % 20 == 0.
int x0_stats_nparts(int F, int T);
bool x0_eligible(const ConvParams& p);
hipError_t launch_x0_stats(const ConvParams& p, hipStream_t s);

// wide-tile 3x3 conv for the 64/128/256-output convs of levels 1-2, bf16, throughput plan (conv3w.hip): one 8-wave
// workgroup per CU owns all output channels of a tile; weight image decoder.cpp pack_conv3w (key ".w3w"). GroupNorm
// partial slots: one per tile (conv3w_nparts, 0 if the shape is not covered). GT_CONV3W=0 disables it.
bool conv3w_eligible(const ConvParams& p, InMode im);
int conv3w_nparts(int F, int T, int Cout);
hipError_t launch_conv3w(InMode im, const ConvParams& p, hipStream_t s);
int conv3w_cfg(int Cout, int F);
// fp8-operand form (conv3w_a8.hip; GT_FP8's throughput plan): the same tiles and partial slots as conv3w, the conv's
// .w3a image (decoder.cpp pack_conv3w_a8) and its per-output-channel weight scale (p.wscale)
bool conv3w_a8_eligible(const ConvParams& p, InMode im);
hipError_t launch_conv3w_a8(InMode im, const ConvParams& p, hipStream_t s);

}  // namespace gt
