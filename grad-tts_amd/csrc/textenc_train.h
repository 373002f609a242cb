// Training pass of the text encoder and GradTTS.compute_loss glue (textenc_train.hip): parameter blocks and launchers.
// fp32, activations channels-last [B][T][C] as in textenc.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "textenc.h"

namespace gt {

constexpr int TT_TMAX = 4096;   // longest token sequence of the training attention (one LDS score row)

// attention forward with explicit probabilities: P = softmax(masked scores) [B][H][T][T], Pd = dropout(P) and its
// transpose PdT, out
hipError_t launch_tt_attn_fwd(const float* qkv, const float* x_mask, const float* erk, const float* erv, int B, int T,
                              int C, int H, int W, Drop drop, float* P, float* Pd, float* PdT, float* out,
                              hipStream_t s);
// attention backward: datt [B][T][C] -> dqkv [B][T][3C], d emb_rel_k | d emb_rel_v (2 (2W+1) 96 floats);
// dS [B][H][T][T] and drel_part [B][2][2W+1][96] are scratch
hipError_t launch_tt_attn_bwd(const float* qkv, const float* P, const float* Pd, const float* PdT, const float* datt,
                              const float* x_mask, const float* erk, const float* erv, int B, int T, int C, int H,
                              int W, Drop drop, float* dS, float* dST, float* dqkv, float* drel_part, float* derk_derv,
                              hipStream_t s);

// LayerNorm backward. LN input = x (+ res); dy_eff = dy * dy_mask * drop * [relu_ref > 0]; dx = LN'(dy_eff)
// * [LN input > 0 if post_relu] * dx_mask, written or accumulated; dgamma | dbeta (2C floats) via per-workgroup
// partials part [tt_ln_bwd_blocks(npos)][2C]
struct LnBwdParams {
  const float* x; int x_cs;
  const float* res; int res_cs;
  const float* gamma; int C; float eps; long npos;
  const float* dy; int dy_cs;
  const float* dy_mask;
  Drop drop;
  const float* relu_ref;   // [npos][C]
  int post_relu;
  const float* dx_mask;
  float* dx; int dx_cs, dx_accumulate;
  float* part;
};
long tt_ln_bwd_blocks(long npos);
hipError_t launch_tt_ln_bwd(const LnBwdParams& p, float* dgamma_dbeta, hipStream_t s);

// Conv1d weight gradient dW[o][c][k] = sum_{b,t} dout[b][t][o] (x m)[b][t + k - pad][c], K <= 5, into dW
// ([Cout][Cin][K], the reference layout); position splits go through `partial` (nsplit x Cout Cin K floats at most
// partial_floats) and a fixed-order reduction
struct WgradParams {
  const float* dout; int d_cs;
  const float* x; int x_cs;
  const float* x_mask;
  int B, T, Cin, Cout, K, pad;
  int nsplit;
  float* out;
};
int tt_wgrad_splits(const WgradParams& p);
hipError_t launch_tt_wgrad(WgradParams p, float* dW, float* partial, long partial_floats, hipStream_t s);
// out[c] = sum_pos x[pos][c] (split partials in part, at most part_floats)
hipError_t launch_tt_colsum(const float* x, int x_cs, long npos, int C, float* part, long part_floats, float* out,
                            hipStream_t s);
hipError_t launch_tt_emb_bwd(const int64_t* tokens, long npos, const float* dx0, int n_vocab, int C, float scale,
                             float* demb, float* part, long part_floats, hipStream_t s);

// dst[pos][c] = src(pos, c) (0 if src is NULL) * mask[pos] * drop(pos C + c) * [relu_ref[pos][c] > 0]; src channels-last or
// channel-major [B][C][T]
struct EwParams {
  float* dst; int dst_cs;
  const float* src; int src_cs, src_chan_major;
  long npos; int T, C;
  const float* mask;
  Drop drop;
  const float* relu_ref; int relu_cs;
};
hipError_t launch_tt_ew(const EwParams& p, hipStream_t s);
hipError_t launch_tt_copy_words(uint32_t* dst, const uint32_t* src, long n, hipStream_t s);

// device-side repack of the conv weights (after gt_text_encoder_set_params_device)
struct RepackEntry {
  long raw_off, pk_off, pkt_off;
  int O, Ci, K;
};
hipError_t launch_tt_repack(const float* raw, const RepackEntry* tab, int n_entries, float* pk, hipStream_t s);

// GradTTS.compute_loss glue
hipError_t launch_tt_path_scatter(const float* attn, const float* dmu_y, int B, int Tx, int Ty, int F, float* dmu_x,
                                  hipStream_t s);
// losses: out[0] dur_loss, out[1] prior_loss, out[2..3] gradient scales (out holds 4 floats)
hipError_t launch_tt_aux_loss(const float* logw, const float* attn, const float* x_mask, const int64_t* x_lengths,
                              const float* y, const float* mu_y, const float* y_mask, int B, int Tx, int Ta, int Ty,
                              int F, float* out, float* dlogw_unit, float* dmu_unit, double* scratch, hipStream_t s);
// fp64 scratch of launch_tt_aux_loss (block partials)
long tt_aux_loss_scratch_doubles(long B, long Tx);

}  // namespace gt
