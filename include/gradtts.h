/*
 * gradtts.h -- C ABI of the MI355X-native Grad-TTS reverse-diffusion decoder and monotonic alignment.
 *
 * Library: grad-tts_amd/gradtts_amd/libgradtts.so (hipcc, gfx950). Plain pointers and sizes only.
 * Device pointers (all tensors passed to compute calls) must be HIP device memory; `stream` is a
 * hipStream_t (NULL = default stream). Every compute call is stream-ordered and asynchronous.
 * Return value: GT_OK or an error code; gt_last_error() gives a thread-local message.
 *
 * Reference interfaces replaced (Mattias421/Grad-TTS, files under model/):
 *   gt_decoder_create        <- Diffusion.__init__ / GradLogPEstimator2d.__init__   diffusion.py:228-242, 128-172
 *   gt_decoder_set_param     <- nn.Module.load_state_dict on the estimator           (keys: diffusion.py:128-172,
 *                               saved by train.py:174-175, loaded by inference.py:66)
 *   gt_estimator_forward     <- GradLogPEstimator2d.forward(x, mask, mu, t, spk)     diffusion.py:174-216
 *   gt_reverse_diffusion     <- Diffusion.forward / reverse_diffusion(z, mask, mu, n_timesteps, stoc, spk)
 *                                                                                     diffusion.py:254-272
 *   gt_maximum_path          <- monotonic_align.core.maximum_path_c(paths, values, t_xs, t_ys, max_neg_val)
 *                                                                                     monotonic_align/core.pyx:38-45
 */
#ifndef GRADTTS_H
#define GRADTTS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  GT_OK = 0,
  GT_ERR_ARG = 1,          /* bad shape / pointer / value */
  GT_ERR_HIP = 2,          /* a HIP runtime call failed */
  GT_ERR_PARAM = 3,        /* unknown parameter name, wrong numel, or a parameter was never set */
  GT_ERR_UNSUPPORTED = 4,  /* configuration outside what the kernels implement */
  GT_ERR_WORKSPACE = 5     /* workspace smaller than the *_workspace_bytes() query */
};

/* Compute dtype of the U-Net activations / MFMA operands (accumulation is always fp32;
 * the sampler state x_t, mu, z and outputs are always fp32).
 * GT_BF16_W8: bf16 activations with fp8 (OCP e4m3) weights for every 3x3 conv, Downsample and
 * Upsample (ConvTranspose) -- 90 % of the U-Net's parameters -- quantized per output channel by
 * gt_quantize_e4m3 when the weights are packed; 1x1, attention and linear weights stay bf16 / fp32
 * (BASELINE.json config 5).
 * GT_FP8: as GT_BF16_W8, and the stride-1 3x3 convs over activations (every Block conv but the U-Net input's) run
 * on the block-scaled fp8 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4): their inputs are quantized to e4m3 in the
 * conv's operand load with one power-of-two (E8M0) scale per position and 32-channel block. */
enum { GT_F32 = 0, GT_BF16 = 1, GT_BF16_W8 = 2, GT_FP8 = 3 };

typedef struct gt_decoder gt_decoder;

const char* gt_version(void);
const char* gt_last_error(void);

/* Diffusion(n_feats, dim, n_spks, spk_emb_dim, beta_min, beta_max, pe_scale).
 * Supported: n_feats == 80, dim == 64, spk_emb_dim == 64 (the reference configurations, params.py). */
int gt_decoder_create(int n_feats, int dim, int n_spks, int spk_emb_dim, float beta_min, float beta_max,
                      float pe_scale, gt_decoder** out);
void gt_decoder_destroy(gt_decoder* dec);
/* Change beta_min / beta_max (Diffusion.beta_min/beta_max; SPEECHSDE.beta_0/beta_1, sde_lib.py:258-262) of an
 * existing decoder: the noise schedule is read at each call, so weights stay packed; captured sampler graphs
 * are dropped when the values change. */
int gt_decoder_set_betas(gt_decoder* dec, float beta_min, float beta_max);

/* Parameter inventory = GradLogPEstimator2d.state_dict() keys in registration order (no "estimator." prefix). */
int gt_decoder_num_params(const gt_decoder* dec);
const char* gt_decoder_param_name(const gt_decoder* dec, int i);
int64_t gt_decoder_param_numel(const gt_decoder* dec, int i);
/* Copy one parameter (host fp32, contiguous, reference shape) into the decoder. Packing to device
 * layouts happens lazily at the next compute call (synchronously, outside any stream capture). */
int gt_decoder_set_param(gt_decoder* dec, const char* name, const float* host_data, int64_t numel);
/* Device-side parameter update (a training loop's optimizer step, no host round trip): params = every parameter in
 * inventory order, fp32 contiguous on the device (gt_decoder_grad_numel floats, the gradient buffer's layout),
 * copied on `stream` into the fp32 block the training / VJP / likelihood calls read. Inference weight images are
 * re-packed from it lazily (one device -> host read) at the next inference call. Every parameter must have been set
 * once with gt_decoder_set_param. */
int gt_decoder_set_params_device(gt_decoder* dec, const float* params, int64_t numel, void* stream);

/* Number of times the weights were packed into device layouts so far (one per compute dtype in use after
 * each parameter change; the reference re-reads weights on every call, this library packs them once). */
int64_t gt_decoder_pack_count(const gt_decoder* dec);

/* Workspace (device bytes) needed by a compute call with this batch B, padded frame count T and
 * step count (0 for gt_estimator_forward). Any alignment: the call aligns the base itself. */
size_t gt_decoder_workspace_bytes(const gt_decoder* dec, int dtype, int64_t B, int64_t T, int32_t n_timesteps);

/* One score evaluation: out[B,80,T] = s_theta(x, mask, mu, t, spk).
 * x, mu, out: [B,80,T] fp32; mask: [B,1,T] fp32 (0/1); t: [B] fp32; spk: [B,64] fp32 or NULL.
 * T must be a multiple of 4 (fix_len_compatibility, model/utils.py:13-17).
 * Masks are sequence_mask outputs, 0 or 1: the kernels compute the reference's x * m * m as x * m, exact only then.
 * The C ABI does not scan the mask (device memory, the caller's stream); the Python / torch.ops boundary rejects any
 * other value (gradtts_amd.diffusion, csrc/torch_ops.cpp). A fractional mask here gives a consistent result on every
 * kernel path, but not the reference's. */
int gt_estimator_forward(gt_decoder* dec, int dtype, const float* x, const float* mask, const float* mu,
                         const float* t, const float* spk, int64_t B, int64_t T, float* out, void* workspace,
                         size_t workspace_bytes, void* stream);

/* Full sampler: out[B,80,T] = x_0 after n_timesteps deterministic Euler steps from x_T = z*mask
 * (reverse_diffusion ignores `stoc` in the reference; so does this). */
int gt_reverse_diffusion(gt_decoder* dec, int dtype, const float* z, const float* mask, const float* mu,
                         const float* spk, int64_t B, int64_t T, int32_t n_timesteps, float* out, void* workspace,
                         size_t workspace_bytes, void* stream);

/* HIP-graph replay of the sampler (default off -- measured no faster, the sampler is GPU-bound at every batch
 * size; environment GT_GRAPHS=1 turns it on at creation).
 * gt_reverse_diffusion captures its Euler steps once per (shape, dtype, tensor and workspace addresses) into
 * graphs of up to 100 steps (50-step segments plus a remainder beyond that; a device-side step index selects
 * each step's time-bias row and beta(t)) and replays them on the caller's stream. Captures are skipped while
 * profiling is on or when the caller's stream is itself being captured (the launches then join the caller's
 * graph). Results are bit-identical with and without graphs. gt_decoder_graph_captures counts captures. */
int gt_decoder_set_graphs(gt_decoder* dec, int on);
int64_t gt_decoder_graph_captures(const gt_decoder* dec);
/* Small-batch tile plan: GT_BF16 and GT_BF16_W8 calls on at most max_b utterances (env GT_SMALL_B at creation)
 * use 1-/2-row conv tiles and (GT_BF16) one-tile conv64 segments, so a single utterance fills the GPU (latency). Default 4. Each plan
 * is batch-invariant on its own; across plans results agree to fp32 rounding of the GroupNorm sums. 0 disables;
 * max_b > 16 is rejected (GT_ERR_ARG: the workspace holds the small plan's attention partials up to 16 utterances). */
int gt_decoder_set_small_batch(gt_decoder* dec, int64_t max_b);
/* Wide-tile 3x3 convs (default on; env GT_CONV3W=0 at creation turns them off): GT_BF16 / GT_BF16_W8 throughput-plan
 * calls run the level-1/2 Block convs (model/diffusion.py:52; Cout 64/128/256, Cin % 32 == 0) as one 8-wave workgroup per
 * CU that owns every output channel of a 10- or 20-row x 32-frame tile (csrc/conv3w.hip); GT_FP8 calls run the same
 * convs on their fp8-operand twin (csrc/conv3w_a8.hip, same quantization as the conv_kernel A8 tiles; env
 * GT_CONV3W_A8=0 keeps fp8 on conv_kernel). Off: the 128-wide conv_kernel tiles. The forms agree to fp32 accumulation
 * order (different K order and GroupNorm partition). */
int gt_decoder_set_wide_conv(gt_decoder* dec, int on);

/* Batches of any size: a compute call runs the batch in chunks of at most
 * floor((2^31 - 1) / (80 * T * 64 * element_size)) utterances (the kernels' 32-bit buffer ranges), each a
 * complete evaluation in the same workspace, which gt_decoder_workspace_bytes sizes for one chunk. Results do
 * not depend on the chunking (per-utterance GroupNorm / attention statistics). */

/* Diagnostics: run gt_estimator_forward and additionally copy the activation produced by `stage`
 * (a module path of the reference, e.g. "downs.0.1", "downs.1.2", "mid_block1", "ups.0.3", with
 * ".pre1"/".pre2" for a ResnetBlock's pre-GroupNorm conv outputs, or "final_block.pre") to
 * probe_out as fp32 [B, C, F_l, T_l]. Used by the parity tests to localise a mismatch. */
int gt_estimator_probe(gt_decoder* dec, int dtype, const float* x, const float* mask, const float* mu,
                       const float* t, const float* spk, int64_t B, int64_t T, const char* stage, float* probe_out,
                       float* out, void* workspace, size_t workspace_bytes, void* stream);

/* Profiling: when enabled, every kernel launch of subsequent compute calls is bracketed by HIP events
 * on the caller's stream. gt_decoder_profile_read synchronises on them and writes a JSON array
 * aggregated per kernel: [{"kernel": name, "launches": n, "ms": total, "flop": algorithmic FLOPs,
 * "bytes": compulsory HBM bytes}, ...] (FLOPs as the reference counts them). */
int gt_decoder_profile_enable(gt_decoder* dec, int on);
int gt_decoder_profile_read(gt_decoder* dec, char* json_buf, size_t capacity);
/* Restrict profiling to launches whose "<kernel>@<shape>" name starts with `prefix` (NULL or "" = all).
 * Each event pair costs a few microseconds of stream time, so bench.py times its steps with events on
 * one kernel instantiation only. */
int gt_decoder_profile_filter(gt_decoder* dec, const char* prefix);

/* fp8 weight quantization used by GT_BF16_W8 (host, no GPU): for each of `rows` output channels o,
 * scale[o] = max_i |w[o*row_stride + i*col_stride]| / 448 (1 for an all-zero row) and
 * q[same index] = e4m3(w / scale[o]) (fp32 division, round to nearest even, saturating at 448; the
 * rounding of torch.Tensor.to(torch.float8_e4m3fn)). gt_f32_to_e4m3 converts one value. */
uint8_t gt_f32_to_e4m3(float x);
int gt_quantize_e4m3(const float* w, int64_t rows, int64_t cols, int64_t row_stride, int64_t col_stride, uint8_t* q,
                     float* scale);

/* ---- Training path, forward values ----
 * Diffusion.forward_diffusion (model/diffusion.py:244-252) with the noise passed in: xt = (x0 e + mu (1 - e) +
 * z sqrt(1 - e^2)) * mask, zm = z * mask, e = exp(-cum_noise(t) / 2). All [B,80,T] fp32, mask [B,1,T], t [B].
 * zm may be NULL. No workspace. */
int gt_forward_diffusion(gt_decoder* dec, const float* x0, const float* mask, const float* mu, const float* t,
                         const float* z, int64_t B, int64_t T, float* xt, float* zm, void* stream);
/* Diffusion.loss_t (diffusion.py:274-281) forward value with the noise passed in: loss[0] (device fp32) =
 * sum((s_theta(xt) sqrt(1 - e^-cum) + z mask)^2) / (sum(mask) * 80), xt = the forward-diffused input (out,
 * [B,80,T]). Deterministic (fixed-order reductions). Forward value only: the parameter gradients are
 * gt_diffusion_loss_grad's, below. */
size_t gt_diffusion_loss_workspace_bytes(const gt_decoder* dec, int dtype, int64_t B, int64_t T);
int gt_diffusion_loss_t(gt_decoder* dec, int dtype, const float* x0, const float* mask, const float* mu,
                        const float* t, const float* z, const float* spk, int64_t B, int64_t T, float* loss,
                        float* xt, void* workspace, size_t workspace_bytes, void* stream);
/* Training step (fp32): loss_t forward with a tape and the backward of the U-Net. loss[0], xt as
 * gt_diffusion_loss_t; grads: fp32 [gt_decoder_grad_numel] = d loss / d every estimator parameter, concatenated in
 * state_dict inventory order (gt_decoder_param_name) in the reference layouts; dmu [B,80,T] = d loss / d mu
 * (NULL: not written; mu enters the U-Net and x_t, diffusion.py:247/181); dspk [B,64] = d loss / d spk (n_spks > 1,
 * NULL: not written). Deterministic. workspace: gt_train_workspace_bytes (the tape). */
size_t gt_train_workspace_bytes(gt_decoder* dec, int64_t B, int64_t T);
int64_t gt_decoder_grad_numel(gt_decoder* dec);
int gt_diffusion_loss_grad(gt_decoder* dec, const float* x0, const float* mask, const float* mu, const float* t,
                           const float* z, const float* spk, int64_t B, int64_t T, float* loss, float* xt, float* grads,
                           float* dmu, float* dspk, void* workspace, size_t workspace_bytes, void* stream);

/* Estimator VJP (fp32), the building block of the likelihood's Hutchinson divergence (SURVEY §8 f3;
 * n_best/likelihood/likelihood.py:27-38 takes it with torch.autograd.grad): score [B,80,T] = the estimator
 * output on (x, mask, mu, t, spk) (NULL: not written); vjp_x [B,80,T] = (d score / d x)^T v.
 * workspace: gt_estimator_vjp_workspace_bytes. */
size_t gt_estimator_vjp_workspace_bytes(gt_decoder* dec, int64_t B, int64_t T);
int gt_estimator_vjp(gt_decoder* dec, const float* x, const float* mask, const float* mu, const float* t,
                     const float* spk, const float* v, int64_t B, int64_t T, float* score, float* vjp_x,
                     void* workspace, size_t workspace_bytes, void* stream);

/* Likelihood of a mel under SPEECHSDE's probability-flow ODE (n_best/likelihood/likelihood.py:41-133,
 * sde_lib.py:256-297), fp32 evaluations:
 * gt_likelihood_drift_div: one ODE evaluation = likelihood_fn's ode_func (likelihood.py:92-97): drift [B,80,T]
 *   = drift_fn(x, t) (:61-65) and div [B] = the Hutchinson divergence of drift_fn with probe eps (:27-38, 67-68).
 * gt_likelihood_euler: the euler > 0 branch (:99-115) on the device: state in fp64 as the reference's numpy
 *   state, t_i = (i + 0.5) / n_steps, from data * mask; returns z [B,80,T] and delta_logp [B] (fp32).
 * workspace (both): gt_likelihood_workspace_bytes. */
size_t gt_likelihood_workspace_bytes(gt_decoder* dec, int64_t B, int64_t T);
int gt_likelihood_drift_div(gt_decoder* dec, const float* x, const float* mask, const float* mu, const float* t,
                            const float* spk, const float* eps, int64_t B, int64_t T, float* drift, float* div,
                            void* workspace, size_t workspace_bytes, void* stream);
int gt_likelihood_euler(gt_decoder* dec, const float* data, const float* mask, const float* mu, const float* spk,
                        const float* eps, int64_t B, int64_t T, int32_t n_steps, float* z, float* delta_logp,
                        void* workspace, size_t workspace_bytes, void* stream);

/* Text encoder of GradTTS (model/text_encoder.py:285-335; speaker-agnostic as GradTTS builds it, tts.py:49-51) and
 * the front-end of GradTTS.forward (tts.py:84-101). fp32. Parameters by the reference TextEncoder's state_dict
 * names (host data, uploaded on the next forward after a change). gt_text_encoder_forward = TextEncoder.forward:
 * tokens / x_lengths int64 [B,Tx] / [B]; outputs mu_x [B,n_feats,Tx], logw [B,1,Tx], x_mask [B,1,Tx].
 * gt_durations: w_ceil = ceil(exp(logw) x_mask) * length_scale, cum = cumsum(w_ceil), y_lengths =
 * max(1, (long) sum w_ceil) (tts.py:86-89). gt_expand: y_mask, generate_path's alignment (attn [B,Tx,Ty] fp32, NULL:
 * not written) and mu_y = attn^T mu_x [B,n_feats,Ty] (tts.py:93-99, utils.py:26-39); Ty = fix_len_compatibility(max
 * y_lengths) is the caller's (it needs y_lengths on the host, as the reference's int(y_lengths.max()) does). */
typedef struct gt_text_encoder gt_text_encoder;
int gt_text_encoder_create(int n_vocab, int n_feats, int n_channels, int filter_channels, int filter_channels_dp,
                           int n_heads, int n_layers, int kernel_size, int window_size, gt_text_encoder** out);
void gt_text_encoder_destroy(gt_text_encoder* enc);
int gt_text_encoder_num_params(gt_text_encoder* enc);
const char* gt_text_encoder_param_name(gt_text_encoder* enc, int i);
int64_t gt_text_encoder_param_numel(gt_text_encoder* enc, int i);
int gt_text_encoder_set_param(gt_text_encoder* enc, const char* name, const float* data, int64_t numel);
size_t gt_text_encoder_workspace_bytes(gt_text_encoder* enc, int64_t B, int64_t Tx);
int gt_text_encoder_forward(gt_text_encoder* enc, const int64_t* tokens, const int64_t* x_lengths, int64_t B,
                            int64_t Tx, float* mu_x, float* logw, float* x_mask, void* workspace,
                            size_t workspace_bytes, void* stream);
int gt_durations(const float* logw, const float* x_mask, int64_t B, int64_t Tx, float length_scale, float* w_ceil,
                 float* cum, int64_t* y_lengths, void* stream);
int gt_expand(const float* mu_x, const float* cum, const float* x_mask, const int64_t* y_lengths, int64_t B,
              int64_t Tx, int64_t Ty, int32_t n_feats, float* mu_y, float* y_mask, float* attn, void* stream);
/* mu_y [B,n_feats,Ty] = attn^T mu_x for a 0/1 alignment attn [B,Tx,Ty] (GradTTS.get_score_model, tts.py:233-234) */
int gt_path_gather(const float* attn, const float* mu_x, int64_t B, int64_t Tx, int64_t Ty, int32_t n_feats,
                   float* mu_y, void* stream);

/* Text-encoder training pass of GradTTS.compute_loss (model/tts.py:136: TextEncoder.forward in train mode,
 * text_encoder.py:321-335) and its backward. gt_text_encoder_forward_train = gt_text_encoder_forward plus the
 * training dropouts (p_dropout: attention probabilities, attention / FFN outputs, FFN hidden, duration predictor;
 * p_dropout_prenet: ConvReluNorm's 0.5; 0 = eval semantics) drawn from `seed` by the library's counter-based
 * generator, and a tape of the activations in `workspace` (gt_text_encoder_train_workspace_bytes). Tx <= 4096.
 * gt_text_encoder_backward: given dmu_x [B,n_feats,Tx] and dlogw [B,1,Tx] (either may be NULL = zero), writes the
 * gradient of every encoder parameter into grads (gt_text_encoder_grad_numel floats, state_dict inventory order,
 * reference layouts); the duration predictor sees a detached input (text_encoder.py:332), so dlogw reaches only its
 * parameters. Takes the tape (workspace), B, Tx and dropout arguments of the forward_train call it differentiates
 * (no state in the handle: several taped forwards may precede their backwards, e.g. gradient accumulation); the
 * parameters must be unchanged in between. */
size_t gt_text_encoder_train_workspace_bytes(gt_text_encoder* enc, int64_t B, int64_t Tx);
/* Device-side parameter update (a training loop's optimizer step, no host round trip): params = every parameter in
 * inventory order, fp32 contiguous on the device (the gradient buffer's layout), copied and repacked on `stream`.
 * Every parameter must have been set once with gt_text_encoder_set_param; a later host-side set_param first reads
 * the device values back. */
int gt_text_encoder_set_params_device(gt_text_encoder* enc, const float* params, int64_t numel, void* stream);
int64_t gt_text_encoder_grad_numel(gt_text_encoder* enc);
int gt_text_encoder_forward_train(gt_text_encoder* enc, const int64_t* tokens, const int64_t* x_lengths, int64_t B,
                                  int64_t Tx, float p_dropout, float p_dropout_prenet, uint64_t seed, float* mu_x,
                                  float* logw, float* x_mask, void* workspace, size_t workspace_bytes, void* stream);
int gt_text_encoder_backward(gt_text_encoder* enc, const float* dmu_x, const float* dlogw, int64_t B, int64_t Tx,
                             float p_dropout, float p_dropout_prenet, uint64_t seed, float* grads, void* workspace,
                             size_t workspace_bytes, void* stream);
/* dmu_x [B,n_feats,Tx] = attn dmu_y: the backward of mu_y = attn^T mu_x (tts.py:184-185), attn [B,Tx,Ty] 0/1 */
int gt_path_scatter(const float* attn, const float* dmu_y, int64_t B, int64_t Tx, int64_t Ty, int32_t n_feats,
                    float* dmu_x, void* stream);
/* dur_loss (tts.py:155-156 with utils.py:42-44 duration_loss over logw [B,1,Tx] and the MAS attn [B,Tx,Ty]) and
 * prior_loss (tts.py:191-192 over y, mu_y [B,n_feats,Ty'] and y_mask [B,1,Ty']) in one call: losses (4 floats,
 * device): [0] = dur_loss, [1] = prior_loss, [2..3] internal scales; dlogw_unit = d dur_loss / d logw, dmu_y_unit =
 * d prior_loss / d mu_y. Fixed summation order (fp64 block partials). */
size_t gt_tts_aux_losses_workspace_bytes(int64_t B, int64_t Tx);
int gt_tts_aux_losses(const float* logw, const float* attn, const float* x_mask, const int64_t* x_lengths, int64_t B,
                      int64_t Tx, int64_t Ty_attn, const float* y, const float* mu_y, const float* y_mask, int64_t Ty,
                      int32_t n_feats, float* losses, float* dlogw_unit, float* dmu_y_unit, void* workspace,
                      size_t workspace_bytes, void* stream);

/* HiFi-GAN generator (hifi-gan/models.py:77-128, ResBlock1 :13-48 / ResBlock2 :53-74; the vocoder of
 * inference.py:73-97). fp32. Parameters by the reference Generator's state_dict names (bias, weight_g, weight_v per
 * conv); weight norm baked on upload as remove_weight_norm() does. gt_vocoder_forward: mel [B,n_mels,T] -> audio
 * [B,1,T*hop], hop = prod(upsample_rates). Implemented: upsampling kernel = 2 x rate (V1 / V2 / V3), resblock kernels
 * <= 11 with (k - 1) dilation <= 80.
 * gt_vocoder_create: ResBlock1 with 3 dilations per resblock (h.resblock == '1'); resblock_dilations [n_kernels][3].
 * gt_vocoder_create2: resblock = 1 or 2 (h.resblock), n_dil dilations per resblock, resblock_dilations
 * [n_kernels][n_dil] (HiFi-GAN V3: resblock 2, 2 dilations). */
typedef struct gt_vocoder gt_vocoder;
int gt_vocoder_create(int n_mels, int upsample_initial_channel, int n_up, const int* upsample_rates,
                      const int* upsample_kernel_sizes, int n_kernels, const int* resblock_kernel_sizes,
                      const int* resblock_dilations, gt_vocoder** out);
int gt_vocoder_create2(int n_mels, int upsample_initial_channel, int n_up, const int* upsample_rates,
                       const int* upsample_kernel_sizes, int n_kernels, const int* resblock_kernel_sizes, int resblock,
                       int n_dil, const int* resblock_dilations, gt_vocoder** out);
void gt_vocoder_destroy(gt_vocoder* voc);
int gt_vocoder_num_params(gt_vocoder* voc);
const char* gt_vocoder_param_name(gt_vocoder* voc, int i);
int64_t gt_vocoder_param_numel(gt_vocoder* voc, int i);
int gt_vocoder_set_param(gt_vocoder* voc, const char* name, const float* data, int64_t numel);
int64_t gt_vocoder_hop(gt_vocoder* voc);
/* 0: fp32 (default, the parity path); 1: bf16 operands with fp32 accumulation (throughput mode) */
int gt_vocoder_set_compute_dtype(gt_vocoder* voc, int dtype);
size_t gt_vocoder_workspace_bytes(gt_vocoder* voc, int64_t B, int64_t T);
int gt_vocoder_forward(gt_vocoder* voc, const float* mel, int64_t B, int64_t T, float* audio, void* workspace,
                       size_t workspace_bytes, void* stream);

/* The alignment step of GradTTS.compute_loss (model/tts.py:141-152) in one call: the log-prior of mu_x
 * [B,n_feats,Tx] against y [B,n_feats,Ty] (three fp32 contractions + const, tts.py:143-149), masked with
 * x_mask [B,Tx] (x) y_mask [B,Ty], then maximum_path on device (t_x, t_y from the masks). paths: [B,Tx,Ty]
 * int32 (0/1); log_prior: optional [B,Tx,Ty] fp32 copy of the masked log-prior (NULL: kept in the workspace).
 * n_feats <= 128. */
size_t gt_alignment_workspace_bytes(int64_t B, int64_t Tx, int64_t Ty);
int gt_log_prior_maximum_path(const float* mu_x, const float* y, const float* x_mask, const float* y_mask, int64_t B,
                              int64_t n_feats, int64_t Tx, int64_t Ty, int32_t* paths, float* log_prior,
                              void* workspace, size_t workspace_bytes, void* stream);

/* Monotonic alignment search.  values: [b, tx_max, ty_max] fp32 (already multiplied by the mask,
 * as maximum_path does before calling the Cython core); t_xs, t_ys: [b] int32 (device);
 * paths: [b, tx_max, ty_max] int32 output, fully written (0/1). `values` is not modified
 * (the reference mutates only its private numpy copy). Requires t_x <= t_y per item (t_x > t_y
 * makes the reference read out of bounds, core.pyx:34). workspace: device memory of
 * gt_maximum_path_workspace_bytes() bytes, any alignment. */
size_t gt_maximum_path_workspace_bytes(int64_t b, int64_t tx_max, int64_t ty_max);
int gt_maximum_path(int32_t* paths, const float* values, const int32_t* t_xs, const int32_t* t_ys, int64_t b,
                    int64_t tx_max, int64_t ty_max, float max_neg_val, void* workspace, size_t workspace_bytes,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GRADTTS_H */
