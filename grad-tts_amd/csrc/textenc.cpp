// Host side of the text encoder (model/text_encoder.py:285-335) and the GradTTS.forward front-end
// (model/tts.py:84-101): parameter registry (state_dict names of the reference TextEncoder), one fp32 device block,
// and the launch sequence of textenc.hip in the reference's order of operations.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "decoder_internal.h"
#include "gradtts.h"
#include "kernels.h"
#include "textenc.h"
#include "textenc_train.h"

using namespace gt;

struct gt_text_encoder {
  int n_vocab, n_feats, C, Fc, Fdp, H, L, K, W;
  std::vector<std::pair<std::string, std::vector<int64_t>>> inv;
  std::map<std::string, int> index;
  std::vector<std::vector<float>> host;
  std::vector<bool> set;
  std::vector<int64_t> off;
  int64_t numel = 0;
  float* dev = nullptr;
  bool dirty = true;
  // conv weights repacked [Cout][K][Cin] (16-byte aligned) for c1d_pk_kernel
  std::map<std::string, int64_t> pkoff;
  float* devpk = nullptr;
  int64_t pk_numel = 0;
  // the same weights flipped and transposed, [Cin][K][Cout] with W^T(c, j, o) = W(o, c, K - 1 - j): the input
  // gradient of a conv as a packed conv over its output gradient (training backward)
  std::map<std::string, int64_t> pktoff;
  // device-side parameter updates: the repack table (device) and the host copies' staleness
  RepackEntry* devtab = nullptr;
  int ntab = 0;
  bool host_stale = false;
  hipEvent_t dev_done = nullptr;   // recorded on the caller's stream by set_params_device (refresh_host waits on it)
  // parameter generation: bumped by every host or device parameter change; forward_train records it per tape (keyed by
  // the workspace base) and backward refuses a tape taken under other parameters. The 256 most recently written
  // tapes are tracked (kMaxTapes): past that the OLDEST by insertion order is dropped, so a backward on a tape that is
  // older than the last 256 forward_train calls of this encoder reports "no forward_train tape".
  uint64_t gen = 0;
  uint64_t tape_seq = 0;
  std::map<const void*, std::pair<uint64_t, uint64_t>> tape_gen;   // base -> (parameter generation, insertion number)
};

namespace {

int64_t prod(const std::vector<int64_t>& d) { int64_t n = 1; for (auto v : d) n *= v; return n; }

void build_inventory(gt_text_encoder* e) {
  auto add = [&](const std::string& k, std::vector<int64_t> d) { e->inv.push_back({k, d}); };
  const int64_t C = e->C, kc = e->C / e->H, nw = 2 * e->W + 1;
  add("emb.weight", {e->n_vocab, C});
  for (int i = 0; i < 3; ++i) { add("prenet.conv_layers." + std::to_string(i) + ".weight", {C, C, 5});
                                add("prenet.conv_layers." + std::to_string(i) + ".bias", {C}); }
  for (int i = 0; i < 3; ++i) { add("prenet.norm_layers." + std::to_string(i) + ".gamma", {C});
                                add("prenet.norm_layers." + std::to_string(i) + ".beta", {C}); }
  add("prenet.proj.weight", {C, C, 1}); add("prenet.proj.bias", {C});
  for (int l = 0; l < e->L; ++l) {
    const std::string p = "encoder.attn_layers." + std::to_string(l) + ".";
    add(p + "emb_rel_k", {1, nw, kc}); add(p + "emb_rel_v", {1, nw, kc});
    for (const char* n : {"conv_q", "conv_k", "conv_v", "conv_o"}) { add(p + n + ".weight", {C, C, 1}); add(p + n + ".bias", {C}); }
  }
  for (int l = 0; l < e->L; ++l) { add("encoder.norm_layers_1." + std::to_string(l) + ".gamma", {C});
                                    add("encoder.norm_layers_1." + std::to_string(l) + ".beta", {C}); }
  for (int l = 0; l < e->L; ++l) {
    const std::string p = "encoder.ffn_layers." + std::to_string(l) + ".";
    add(p + "conv_1.weight", {e->Fc, C, e->K}); add(p + "conv_1.bias", {e->Fc});
    add(p + "conv_2.weight", {C, e->Fc, e->K}); add(p + "conv_2.bias", {C});
  }
  for (int l = 0; l < e->L; ++l) { add("encoder.norm_layers_2." + std::to_string(l) + ".gamma", {C});
                                    add("encoder.norm_layers_2." + std::to_string(l) + ".beta", {C}); }
  add("proj_m.weight", {e->n_feats, C, 1}); add("proj_m.bias", {e->n_feats});
  add("proj_w.conv_1.weight", {e->Fdp, C, e->K}); add("proj_w.conv_1.bias", {e->Fdp});
  add("proj_w.norm_1.gamma", {e->Fdp}); add("proj_w.norm_1.beta", {e->Fdp});
  add("proj_w.conv_2.weight", {e->Fdp, e->Fdp, e->K}); add("proj_w.conv_2.bias", {e->Fdp});
  add("proj_w.norm_2.gamma", {e->Fdp}); add("proj_w.norm_2.beta", {e->Fdp});
  add("proj_w.proj.weight", {1, e->Fdp, 1}); add("proj_w.proj.bias", {1});
  for (size_t i = 0; i < e->inv.size(); ++i) {
    e->index[e->inv[i].first] = (int)i;
    e->off.push_back(e->numel);
    e->numel += prod(e->inv[i].second);
  }
  e->host.resize(e->inv.size());
  e->set.assign(e->inv.size(), false);
}

int upload(gt_text_encoder* e) {
  for (size_t i = 0; i < e->inv.size(); ++i)
    if (!e->set[i]) return gt_internal_fail(GT_ERR_PARAM, "text encoder parameter never set: " + e->inv[i].first);
  if (!e->dirty) return GT_OK;
  std::vector<float> h((size_t)e->numel);
  for (size_t i = 0; i < e->inv.size(); ++i) memcpy(h.data() + e->off[i], e->host[i].data(), e->host[i].size() * 4);
  if (!e->dev && hipMalloc(&e->dev, h.size() * 4) != hipSuccess) return gt_internal_fail(GT_ERR_HIP, "hipMalloc failed");
  if (hipMemcpy(e->dev, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, "hipMemcpy failed");
  std::vector<float> hp;
  e->pkoff.clear();
  e->pktoff.clear();
  for (size_t i = 0; i < e->inv.size(); ++i) {
    const auto& d = e->inv[i].second;
    if (d.size() != 3 || e->inv[i].first.find(".weight") == std::string::npos) continue;
    e->pkoff[e->inv[i].first] = (int64_t)hp.size();
    const float* w = e->host[i].data();
    for (int64_t o = 0; o < d[0]; ++o)
      for (int64_t k = 0; k < d[2]; ++k)
        for (int64_t c = 0; c < d[1]; ++c) hp.push_back(w[(o * d[1] + c) * d[2] + k]);
    while (hp.size() % 4) hp.push_back(0.f);   // 16-byte aligned starts
    e->pktoff[e->inv[i].first] = (int64_t)hp.size();
    for (int64_t c = 0; c < d[1]; ++c)
      for (int64_t j = 0; j < d[2]; ++j)
        for (int64_t o = 0; o < d[0]; ++o) hp.push_back(w[(o * d[1] + c) * d[2] + (d[2] - 1 - j)]);
    while (hp.size() % 4) hp.push_back(0.f);
  }
  std::vector<RepackEntry> tab;
  for (size_t i = 0; i < e->inv.size(); ++i) {
    const auto it = e->pkoff.find(e->inv[i].first);
    if (it == e->pkoff.end()) continue;
    const auto& d = e->inv[i].second;
    tab.push_back(RepackEntry{(long)e->off[i], (long)it->second, (long)e->pktoff.at(e->inv[i].first), (int)d[0],
                              (int)d[1], (int)d[2]});
  }
  if (!e->devtab) {
    if (hipMalloc(&e->devtab, tab.size() * sizeof(RepackEntry)) != hipSuccess) return gt_internal_fail(GT_ERR_HIP, "hipMalloc failed");
    if (hipMemcpy(e->devtab, tab.data(), tab.size() * sizeof(RepackEntry), hipMemcpyHostToDevice) != hipSuccess)
      return gt_internal_fail(GT_ERR_HIP, "hipMemcpy failed");
    e->ntab = (int)tab.size();
  }
  if (e->devpk && (int64_t)hp.size() != e->pk_numel) { (void)hipFree(e->devpk); e->devpk = nullptr; }
  if (!e->devpk && !hp.empty() && hipMalloc(&e->devpk, hp.size() * 4) != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, "hipMalloc failed");
  e->pk_numel = (int64_t)hp.size();
  if (!hp.empty() && hipMemcpy(e->devpk, hp.data(), hp.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, "hipMemcpy failed");
  e->dirty = false;
  return GT_OK;
}

struct Ws {   // workspace layout (floats), 256-byte aligned pieces
  size_t x0, xa, xb, x1, hid, qkv, att, d1, d2, total;
};
Ws ws_layout(const gt_text_encoder* e, int64_t B, int64_t T) {
  Ws w{};
  size_t off = 0;
  auto put = [&](size_t floats) { const size_t o = off; off += (floats * 4 + 255) & ~size_t(255); return o; };
  const size_t n = (size_t)B * T;
  w.x0 = put(n * e->C); w.xa = put(n * e->C); w.xb = put(n * e->C); w.x1 = put(n * e->C);
  w.hid = put(n * e->Fc); w.qkv = put(n * 3 * e->C); w.att = put(n * e->C);
  w.d1 = put(n * e->Fdp); w.d2 = put(n * e->Fdp);
  w.total = off + 256;
  return w;
}

}  // namespace

extern "C" {

int gt_text_encoder_create(int n_vocab, int n_feats, int n_channels, int filter_channels, int filter_channels_dp,
                           int n_heads, int n_layers, int kernel_size, int window_size, gt_text_encoder** out) {
  if (!out) return gt_internal_fail(GT_ERR_ARG, "null out");
  *out = nullptr;
  if (n_channels != n_heads * 96 || n_channels > 256 || filter_channels_dp > 256 || kernel_size > 5 ||
      window_size > 8 || n_vocab <= 0 || n_layers <= 0)
    return gt_internal_fail(GT_ERR_UNSUPPORTED, "text encoder kernels implement 96-dim heads, <= 256 channels in "
                                                "LayerNorms, kernel <= 5, window <= 8");
  gt_text_encoder* e = new gt_text_encoder();
  e->n_vocab = n_vocab; e->n_feats = n_feats; e->C = n_channels; e->Fc = filter_channels; e->Fdp = filter_channels_dp;
  e->H = n_heads; e->L = n_layers; e->K = kernel_size; e->W = window_size;
  build_inventory(e);
  *out = e;
  return GT_OK;
}

void gt_text_encoder_destroy(gt_text_encoder* e) {
  if (!e) return;
  if (e->devtab) (void)hipFree(e->devtab);
  if (e->dev) (void)hipFree(e->dev);
  if (e->devpk) (void)hipFree(e->devpk);
  if (e->dev_done) (void)hipEventDestroy(e->dev_done);
  delete e;
}

int gt_text_encoder_num_params(gt_text_encoder* e) { return e ? (int)e->inv.size() : -1; }
const char* gt_text_encoder_param_name(gt_text_encoder* e, int i) {
  return (e && i >= 0 && i < (int)e->inv.size()) ? e->inv[i].first.c_str() : nullptr;
}
int64_t gt_text_encoder_param_numel(gt_text_encoder* e, int i) {
  return (e && i >= 0 && i < (int)e->inv.size()) ? prod(e->inv[i].second) : -1;
}

// host copies <- the device block after gt_text_encoder_set_params_device (only when a host-side change needs them)
static int refresh_host(gt_text_encoder* e) {
  if (!e->host_stale) return GT_OK;
  // the update's own completion event, not its stream: the caller may have destroyed the stream since
  if (e->dev_done && hipEventSynchronize(e->dev_done) != hipSuccess) return gt_internal_fail(GT_ERR_HIP, "hipEventSynchronize failed");
  std::vector<float> h((size_t)e->numel);
  if (hipMemcpy(h.data(), e->dev, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, "hipMemcpy failed");
  for (size_t i = 0; i < e->inv.size(); ++i) memcpy(e->host[i].data(), h.data() + e->off[i], e->host[i].size() * 4);
  e->host_stale = false;
  return GT_OK;
}

int gt_text_encoder_set_param(gt_text_encoder* e, const char* name, const float* data, int64_t numel) {
  if (!e || !name || !data) return gt_internal_fail(GT_ERR_ARG, "null argument");
  if (int rc = refresh_host(e)) return rc;
  auto it = e->index.find(name);
  if (it == e->index.end()) return gt_internal_fail(GT_ERR_PARAM, std::string("unknown parameter: ") + name);
  if (numel != prod(e->inv[it->second].second)) return gt_internal_fail(GT_ERR_PARAM, std::string("numel mismatch for ") + name);
  e->host[it->second].assign(data, data + numel);
  e->set[it->second] = true;
  e->dirty = true;
  e->gen += 1;
  return GT_OK;
}

int gt_text_encoder_set_params_device(gt_text_encoder* e, const float* params, int64_t numel, void* stream) {
  if (!e || !params) return gt_internal_fail(GT_ERR_ARG, "null argument");
  if (int rc = upload(e)) return rc;   // device blocks exist (every parameter was set once from the host)
  if (numel != e->numel) return gt_internal_fail(GT_ERR_ARG, "numel != gt_text_encoder_grad_numel");
  hipStream_t s = (hipStream_t)stream;
  hipError_t err = launch_copy_f32(e->dev, params, (long)numel, s);
  if (err == hipSuccess) err = launch_tt_repack(e->dev, e->devtab, e->ntab, e->devpk, s);
  if (err != hipSuccess) return gt_internal_fail(GT_ERR_HIP, std::string("parameter update: ") + hipGetErrorString(err));
  if (!e->dev_done && hipEventCreateWithFlags(&e->dev_done, hipEventDisableTiming) != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, "hipEventCreate failed");
  if (hipEventRecord(e->dev_done, s) != hipSuccess) return gt_internal_fail(GT_ERR_HIP, "hipEventRecord failed");
  e->host_stale = true;
  e->gen += 1;
  return GT_OK;
}

size_t gt_text_encoder_workspace_bytes(gt_text_encoder* e, int64_t B, int64_t T) {
  if (!e || B <= 0 || T <= 0) return 0;
  return ws_layout(e, B, T).total;
}

int gt_text_encoder_forward(gt_text_encoder* e, const int64_t* tokens, const int64_t* x_lengths, int64_t B, int64_t T,
                            float* mu_x, float* logw, float* x_mask, void* workspace, size_t workspace_bytes,
                            void* stream) {
  if (!e || !tokens || !x_lengths || !mu_x || !logw || !x_mask || !workspace) return gt_internal_fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || T <= 0) return gt_internal_fail(GT_ERR_ARG, "bad B / T");
  const Ws w = ws_layout(e, B, T);
  if (workspace_bytes < w.total) return gt_internal_fail(GT_ERR_WORKSPACE, "workspace too small");
  int rc = upload(e);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  float* base = (float*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  auto buf = [&](size_t o) { return (float*)((char*)base + o * 1); };
  float* x0 = buf(w.x0); float* xa = buf(w.xa); float* xb = buf(w.xb); float* x1 = buf(w.x1);
  float* hid = buf(w.hid); float* qkv = buf(w.qkv); float* att = buf(w.att); float* d1 = buf(w.d1); float* d2 = buf(w.d2);
  auto P = [&](const std::string& k) { return e->dev + e->off[e->index.at(k)]; };
  // weights in the [Cout][K][Cin] layout of c1d_pk_kernel (channels-last inputs)
  auto PK = [&](const std::string& k) {
    const auto it = e->pkoff.find(k);
    return it != e->pkoff.end() ? e->devpk + it->second : P(k);
  };
  hipError_t err = hipSuccess;
  auto chk = [&](hipError_t x) { if (err == hipSuccess) err = x; };
  const int C = e->C, Bi = (int)B, Ti = (int)T;
  const long npos = (long)B * T;
  auto conv = [&](const float* in, int cin, int in_cs, const float* in_mask, const std::string& key, int cout, int k,
                  float* out, int out_cs, int out_c0, int relu, const float* res, const float* out_mask, int chan_major) {
    C1dParams p = c1d_defaults();
    p.in = in; p.in_cs = in_cs; p.in_mask = in_mask; p.w = P(key + ".weight"); p.bias = P(key + ".bias");
    p.wpk = PK(key + ".weight");
    p.B = Bi; p.T = Ti; p.Q = Ti; p.Tout = Ti; p.Cin = cin; p.Cout = cout; p.K = k; p.pad = k / 2;
    p.wso = (long)cin * k; p.wsc = k;
    p.out = out; p.out_cs = out_cs; p.out_c0 = out_c0; p.chan_major = chan_major; p.relu = relu;
    p.res = res; p.res_cs = C; p.out_mask = out_mask;
    chk(launch_c1d(p, s));
  };
  auto ln = [&](const float* x, const float* res, const std::string& key, int c, int relu, const float* mask, float* out) {
    chk(launch_te_ln(x, c, res, c, P(key + ".gamma"), P(key + ".beta"), npos, c, 1e-4f, relu, mask, out, c, s));
  };
  // embedding * sqrt(C), x_mask (text_encoder.py:322-324)
  chk(launch_te_embed(tokens, x_lengths, P("emb.weight"), e->n_vocab, Bi, Ti, C, (float)std::sqrt((double)C), x0, x_mask, s));
  // prenet: ConvReluNorm (:57-64)
  const float* h = x0;
  float* bufs[2] = {xa, xb};
  for (int i = 0; i < 3; ++i) {
    conv(h, C, C, x_mask, "prenet.conv_layers." + std::to_string(i), C, 5, att, C, 0, 0, nullptr, nullptr, 0);
    ln(att, nullptr, "prenet.norm_layers." + std::to_string(i), C, 1, nullptr, bufs[i & 1]);
    h = bufs[i & 1];
  }
  float* x = x1;
  conv(h, C, C, nullptr, "prenet.proj", C, 1, x, C, 0, 0, x0, x_mask, 0);   // (x_org + proj(x)) * x_mask
  // encoder layers (:271-282); x is masked on entry to every layer
  for (int l = 0; l < e->L; ++l) {
    const std::string a = "encoder.attn_layers." + std::to_string(l) + ".";
    conv(x, C, C, nullptr, a + "conv_q", C, 1, qkv, 3 * C, 0, 0, nullptr, nullptr, 0);
    conv(x, C, C, nullptr, a + "conv_k", C, 1, qkv, 3 * C, C, 0, nullptr, nullptr, 0);
    conv(x, C, C, nullptr, a + "conv_v", C, 1, qkv, 3 * C, 2 * C, 0, nullptr, nullptr, 0);
    chk(launch_te_attn(qkv, x_mask, P(a + "emb_rel_k"), P(a + "emb_rel_v"), Bi, Ti, C, e->H, e->W, att, s));
    conv(att, C, C, nullptr, a + "conv_o", C, 1, xa, C, 0, 0, nullptr, nullptr, 0);
    ln(x, xa, "encoder.norm_layers_1." + std::to_string(l), C, 0, nullptr, xb);          // x = LN(x + y)
    const std::string f = "encoder.ffn_layers." + std::to_string(l) + ".";
    conv(xb, C, C, x_mask, f + "conv_1", e->Fc, e->K, hid, e->Fc, 0, 1, nullptr, nullptr, 0);
    C1dParams p = c1d_defaults();
    p.in = hid; p.in_cs = e->Fc; p.in_mask = x_mask; p.w = P(f + "conv_2.weight"); p.bias = P(f + "conv_2.bias");
    p.wpk = PK(f + "conv_2.weight");
    p.B = Bi; p.T = Ti; p.Q = Ti; p.Tout = Ti; p.Cin = e->Fc; p.Cout = C; p.K = e->K; p.pad = e->K / 2;
    p.wso = (long)e->Fc * e->K; p.wsc = e->K;
    p.out = xa; p.out_cs = C; p.out_mask = x_mask;
    chk(launch_c1d(p, s));
    ln(xb, xa, "encoder.norm_layers_2." + std::to_string(l), C, 0, x_mask, x);         // LN(x + y), * mask
  }
  // mu = proj_m(x) * x_mask -> [B][n_feats][T]
  conv(x, C, C, nullptr, "proj_m", e->n_feats, 1, mu_x, 0, 0, 0, nullptr, x_mask, 1);
  // duration predictor (:83-93)
  conv(x, C, C, x_mask, "proj_w.conv_1", e->Fdp, e->K, d1, e->Fdp, 0, 1, nullptr, nullptr, 0);
  ln(d1, nullptr, "proj_w.norm_1", e->Fdp, 0, nullptr, d2);
  {
    C1dParams p = c1d_defaults();
    p.in = d2; p.in_cs = e->Fdp; p.in_mask = x_mask; p.w = P("proj_w.conv_2.weight"); p.bias = P("proj_w.conv_2.bias");
    p.wpk = PK("proj_w.conv_2.weight");
    p.B = Bi; p.T = Ti; p.Q = Ti; p.Tout = Ti; p.Cin = e->Fdp; p.Cout = e->Fdp; p.K = e->K; p.pad = e->K / 2;
    p.wso = (long)e->Fdp * e->K; p.wsc = e->K;
    p.out = d1; p.out_cs = e->Fdp; p.relu = 1;
    chk(launch_c1d(p, s));
  }
  ln(d1, nullptr, "proj_w.norm_2", e->Fdp, 0, nullptr, d2);
  {
    C1dParams p = c1d_defaults();
    p.in = d2; p.in_cs = e->Fdp; p.in_mask = x_mask; p.w = P("proj_w.proj.weight"); p.bias = P("proj_w.proj.bias");
    p.wpk = PK("proj_w.proj.weight");
    p.B = Bi; p.T = Ti; p.Q = Ti; p.Tout = Ti; p.Cin = e->Fdp; p.Cout = 1; p.K = 1; p.pad = 0;
    p.wso = e->Fdp; p.wsc = 1;
    p.out = logw; p.chan_major = 1; p.out_mask = x_mask;
    chk(launch_c1d(p, s));
  }
  if (err != hipSuccess) return gt_internal_fail(GT_ERR_HIP, std::string("text encoder launch failed: ") + hipGetErrorString(err));
  return GT_OK;
}

int gt_durations(const float* logw, const float* x_mask, int64_t B, int64_t Tx, float length_scale, float* w_ceil,
                 float* cum, int64_t* y_lengths, void* stream) {
  if (!logw || !x_mask || !w_ceil || !cum || !y_lengths || B <= 0 || Tx <= 0) return gt_internal_fail(GT_ERR_ARG, "bad argument");
  const hipError_t e = launch_te_durations(logw, x_mask, (int)B, (int)Tx, length_scale, w_ceil, cum, y_lengths,
                                           (hipStream_t)stream);
  return e == hipSuccess ? GT_OK : gt_internal_fail(GT_ERR_HIP, hipGetErrorString(e));
}

int gt_expand(const float* mu_x, const float* cum, const float* x_mask, const int64_t* y_lengths, int64_t B, int64_t Tx,
              int64_t Ty, int32_t n_feats, float* mu_y, float* y_mask, float* attn, void* stream) {
  if (!mu_x || !cum || !x_mask || !y_lengths || !mu_y || !y_mask || B <= 0 || Tx <= 0 || Ty <= 0)
    return gt_internal_fail(GT_ERR_ARG, "bad argument");
  const hipError_t e = launch_te_expand(mu_x, cum, x_mask, y_lengths, (int)B, (int)Tx, (int)Ty, n_feats, mu_y, y_mask,
                                        attn, (hipStream_t)stream);
  return e == hipSuccess ? GT_OK : gt_internal_fail(GT_ERR_HIP, hipGetErrorString(e));
}

int gt_path_gather(const float* attn, const float* mu_x, int64_t B, int64_t Tx, int64_t Ty, int32_t n_feats, float* mu_y,
                   void* stream) {
  if (!attn || !mu_x || !mu_y || B <= 0 || Tx <= 0 || Ty <= 0) return gt_internal_fail(GT_ERR_ARG, "bad argument");
  const hipError_t e = launch_te_path_gather(attn, mu_x, (int)B, (int)Tx, (int)Ty, n_feats, mu_y, (hipStream_t)stream);
  return e == hipSuccess ? GT_OK : gt_internal_fail(GT_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"

// ================================================================ training pass (GradTTS.compute_loss's encoder)
namespace {

// tape + backward scratch (floats unless noted), 256-byte aligned pieces
struct TrWs {
  size_t tokens, mask, x0, pre_c[3], pre_h[3], x1, d1c, d1d, d2c, d2d;
  std::vector<size_t> qkv, P, Pd, PdT, att, y1, xmid, hd, y2, xout;
  size_t g1, g2, datt, dy, dh, dqkv, ds, dsT, drel, wpart, cpart, lpart, dmu;
  long wpart_floats, cpart_floats;
  size_t total;
  std::map<size_t, size_t> bytes;   // piece offset -> its size: tape pointers are checked against it (tape_ptr)
};

TrWs tr_layout(const gt_text_encoder* e, int64_t B, int64_t T) {
  TrWs w{};
  size_t off = 0;
  auto put = [&](size_t floats) {
    const size_t o = off;
    off += (floats * 4 + 255) & ~size_t(255);
    w.bytes[o] = floats * 4;
    return o;
  };
  const size_t n = (size_t)B * T, C = e->C, Fc = e->Fc, Fd = e->Fdp, att = (size_t)B * e->H * T * T;
  w.tokens = put(2 * n);
  w.mask = put(n);
  w.x0 = put(n * C);
  for (int i = 0; i < 3; ++i) { w.pre_c[i] = put(n * C); w.pre_h[i] = put(n * C); }
  w.x1 = put(n * C);
  for (int l = 0; l < e->L; ++l) {
    w.qkv.push_back(put(n * 3 * C)); w.P.push_back(put(att)); w.Pd.push_back(put(att)); w.PdT.push_back(put(att));
    w.att.push_back(put(n * C)); w.y1.push_back(put(n * C)); w.xmid.push_back(put(n * C));
    w.hd.push_back(put(n * Fc)); w.y2.push_back(put(n * C)); w.xout.push_back(put(n * C));
  }
  w.d1c = put(n * Fd); w.d1d = put(n * Fd); w.d2c = put(n * Fd); w.d2d = put(n * Fd);
  const size_t wide = std::max({C, Fc, Fd, (size_t)e->n_feats});
  w.g1 = put(n * C); w.g2 = put(n * C); w.datt = put(n * C);
  w.dy = put(n * wide); w.dh = put(n * wide); w.dqkv = put(n * 3 * C); w.ds = put(att); w.dsT = put(att);
  w.drel = put((size_t)B * 2 * (2 * e->W + 1) * 96);
  w.wpart_floats = 8L << 20;
  w.wpart = put((size_t)w.wpart_floats);
  w.cpart_floats = 64L * (long)wide;
  w.cpart = put((size_t)w.cpart_floats);
  w.lpart = put((size_t)tt_ln_bwd_blocks((long)n) * 2 * 256);
  w.dmu = put(n * wide);
  w.total = off + 256;
  return w;
}

// pointer to the tape piece at byte offset o: a host-side guard against offset misuse. An offset that is not a piece
// start, or a piece reaching past the workspace, flags the call (it then fails with GT_ERR_WORKSPACE) and yields the
// workspace base, so the launch that uses it stays inside the caller's allocation instead of faulting the GPU.
float* tape_ptr(const TrWs& w, char* base, size_t o, size_t ws_usable, bool& bad) {
  const auto it = w.bytes.find(o);
  if (it == w.bytes.end() || o + it->second > ws_usable) { bad = true; return (float*)base; }
  return (float*)(base + o);
}

}  // namespace

extern "C" {

size_t gt_text_encoder_train_workspace_bytes(gt_text_encoder* e, int64_t B, int64_t T) {
  if (!e || B <= 0 || T <= 0 || T > TT_TMAX) return 0;
  return tr_layout(e, B, T).total;
}

int64_t gt_text_encoder_grad_numel(gt_text_encoder* e) { return e ? e->numel : -1; }

int gt_text_encoder_forward_train(gt_text_encoder* e, const int64_t* tokens, const int64_t* x_lengths, int64_t B,
                                  int64_t T, float p_dropout, float p_dropout_prenet, uint64_t seed, float* mu_x,
                                  float* logw, float* x_mask, void* workspace, size_t workspace_bytes, void* stream) {
  if (!e || !tokens || !x_lengths || !mu_x || !logw || !x_mask || !workspace) return gt_internal_fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || T <= 0) return gt_internal_fail(GT_ERR_ARG, "bad B / T");
  if (T > TT_TMAX) return gt_internal_fail(GT_ERR_UNSUPPORTED, "training attention supports Tx <= 4096");
  if (!(p_dropout >= 0.f && p_dropout < 1.f && p_dropout_prenet >= 0.f && p_dropout_prenet < 1.f))
    return gt_internal_fail(GT_ERR_ARG, "dropout probabilities must lie in [0, 1)");
  const TrWs w = tr_layout(e, B, T);
  if (workspace_bytes < w.total) return gt_internal_fail(GT_ERR_WORKSPACE, "workspace too small");
  int rc = upload(e);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  char* base = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  const size_t usable = workspace_bytes - (size_t)(base - (char*)workspace);
  bool bad_ptr = false;
  auto F = [&](size_t o) { return tape_ptr(w, base, o, usable, bad_ptr); };   // o: byte offset (tr_layout)
  auto P = [&](const std::string& k) { return e->dev + e->off[e->index.at(k)]; };
  auto PK = [&](const std::string& k) {
    const auto it = e->pkoff.find(k);
    return it != e->pkoff.end() ? e->devpk + it->second : P(k);
  };
  hipError_t err = hipSuccess;
  auto chk = [&](hipError_t x) { if (err == hipSuccess) err = x; };
  const int C = e->C, Bi = (int)B, Ti = (int)T;
  const long npos = (long)B * T;
  float* mask = F(w.mask);
  auto conv = [&](const float* in, int cin, const float* in_mask, const std::string& key, int cout, int k, float* out,
                  int out_cs, int out_c0, int relu, const float* res, const float* out_mask, int chan_major, Drop drop) {
    C1dParams p = c1d_defaults();
    p.in = in; p.in_cs = cin; p.in_mask = in_mask; p.w = P(key + ".weight"); p.bias = P(key + ".bias");
    p.wpk = PK(key + ".weight");
    p.B = Bi; p.T = Ti; p.Q = Ti; p.Tout = Ti; p.Cin = cin; p.Cout = cout; p.K = k; p.pad = k / 2;
    p.wso = (long)cin * k; p.wsc = k;
    p.out = out; p.out_cs = out_cs; p.out_c0 = out_c0; p.chan_major = chan_major; p.relu = relu;
    p.res = res; p.res_cs = C; p.out_mask = out_mask; p.drop = drop;
    chk(launch_c1d(p, s));
  };
  auto ln = [&](const float* x, const float* res, const std::string& key, int c, int relu, const float* m, float* out,
                Drop drop) {
    chk(launch_te_ln(x, c, res, c, P(key + ".gamma"), P(key + ".beta"), npos, c, 1e-4f, relu, m, out, c, s, drop));
  };
  const Drop none = make_drop(0, 0, 0.f);
  // tokens into the tape (the embedding gradient needs them), embedding * sqrt(C), x_mask (text_encoder.py:322-324)
  chk(launch_tt_copy_words((uint32_t*)F(w.tokens), (const uint32_t*)tokens, 2 * npos, s));
  chk(launch_te_embed(tokens, x_lengths, P("emb.weight"), e->n_vocab, Bi, Ti, C, (float)std::sqrt((double)C), F(w.x0),
                      mask, s));
  // prenet: ConvReluNorm (:57-64), relu_drop = ReLU + Dropout(p_dropout_prenet)
  const float* h = F(w.x0);
  for (int i = 0; i < 3; ++i) {
    const std::string k = std::to_string(i);
    conv(h, C, mask, "prenet.conv_layers." + k, C, 5, F(w.pre_c[i]), C, 0, 0, nullptr, nullptr, 0, none);
    ln(F(w.pre_c[i]), nullptr, "prenet.norm_layers." + k, C, 1, nullptr, F(w.pre_h[i]),
       make_drop(seed, 1 + i, p_dropout_prenet));
    h = F(w.pre_h[i]);
  }
  conv(h, C, nullptr, "prenet.proj", C, 1, F(w.x1), C, 0, 0, F(w.x0), mask, 0, none);
  const float* x = F(w.x1);
  for (int l = 0; l < e->L; ++l) {
    const std::string a = "encoder.attn_layers." + std::to_string(l) + ".";
    const std::string f = "encoder.ffn_layers." + std::to_string(l) + ".";
    const uint32_t site = 16 + 8 * l;
    float* qkv = F(w.qkv[l]);
    conv(x, C, nullptr, a + "conv_q", C, 1, qkv, 3 * C, 0, 0, nullptr, nullptr, 0, none);
    conv(x, C, nullptr, a + "conv_k", C, 1, qkv, 3 * C, C, 0, nullptr, nullptr, 0, none);
    conv(x, C, nullptr, a + "conv_v", C, 1, qkv, 3 * C, 2 * C, 0, nullptr, nullptr, 0, none);
    chk(launch_tt_attn_fwd(qkv, mask, P(a + "emb_rel_k"), P(a + "emb_rel_v"), Bi, Ti, C, e->H, e->W,
                           make_drop(seed, site, p_dropout), F(w.P[l]), F(w.Pd[l]), F(w.PdT[l]), F(w.att[l]), s));
    conv(F(w.att[l]), C, nullptr, a + "conv_o", C, 1, F(w.y1[l]), C, 0, 0, nullptr, nullptr, 0,
         make_drop(seed, site + 1, p_dropout));                                                      // y = drop(attn)
    ln(x, F(w.y1[l]), "encoder.norm_layers_1." + std::to_string(l), C, 0, nullptr, F(w.xmid[l]), none);
    conv(F(w.xmid[l]), C, mask, f + "conv_1", e->Fc, e->K, F(w.hd[l]), e->Fc, 0, 1, nullptr, nullptr, 0,
         make_drop(seed, site + 2, p_dropout));                                                      // drop(relu(conv_1))
    {
      C1dParams p = c1d_defaults();
      p.in = F(w.hd[l]); p.in_cs = e->Fc; p.in_mask = mask; p.w = P(f + "conv_2.weight"); p.bias = P(f + "conv_2.bias");
      p.wpk = PK(f + "conv_2.weight");
      p.B = Bi; p.T = Ti; p.Q = Ti; p.Tout = Ti; p.Cin = e->Fc; p.Cout = C; p.K = e->K; p.pad = e->K / 2;
      p.wso = (long)e->Fc * e->K; p.wsc = e->K;
      p.out = F(w.y2[l]); p.out_cs = C; p.out_mask = mask; p.drop = make_drop(seed, site + 3, p_dropout);
      chk(launch_c1d(p, s));
    }
    ln(F(w.xmid[l]), F(w.y2[l]), "encoder.norm_layers_2." + std::to_string(l), C, 0, mask, F(w.xout[l]), none);
    x = F(w.xout[l]);
  }
  conv(x, C, nullptr, "proj_m", e->n_feats, 1, mu_x, 0, 0, 0, nullptr, mask, 1, none);
  // duration predictor on the detached x (:332, :83-93)
  conv(x, C, mask, "proj_w.conv_1", e->Fdp, e->K, F(w.d1c), e->Fdp, 0, 1, nullptr, nullptr, 0, none);
  ln(F(w.d1c), nullptr, "proj_w.norm_1", e->Fdp, 0, nullptr, F(w.d1d), make_drop(seed, 8, p_dropout));
  conv(F(w.d1d), e->Fdp, mask, "proj_w.conv_2", e->Fdp, e->K, F(w.d2c), e->Fdp, 0, 1, nullptr, nullptr, 0, none);
  ln(F(w.d2c), nullptr, "proj_w.norm_2", e->Fdp, 0, nullptr, F(w.d2d), make_drop(seed, 9, p_dropout));
  conv(F(w.d2d), e->Fdp, mask, "proj_w.proj", 1, 1, logw, 0, 0, 0, nullptr, mask, 1, none);
  {
    EwParams c{};
    c.dst = x_mask; c.dst_cs = 1; c.src = mask; c.src_cs = 1; c.npos = npos; c.T = Ti; c.C = 1; c.drop = none;
    chk(launch_tt_ew(c, s));
  }
  if (err != hipSuccess) return gt_internal_fail(GT_ERR_HIP, std::string("text encoder training forward: ") + hipGetErrorString(err));
  if (bad_ptr) return gt_internal_fail(GT_ERR_WORKSPACE, "text encoder training forward: tape offset outside the layout");
  constexpr size_t kMaxTapes = 256;
  if (e->tape_gen.size() >= kMaxTapes && !e->tape_gen.count(base)) {
    auto oldest = e->tape_gen.begin();
    for (auto it = e->tape_gen.begin(); it != e->tape_gen.end(); ++it)
      if (it->second.second < oldest->second.second) oldest = it;
    e->tape_gen.erase(oldest);
  }
  e->tape_gen[base] = {e->gen, e->tape_seq++};
  return GT_OK;
}

int gt_text_encoder_backward(gt_text_encoder* e, const float* dmu_x, const float* dlogw, int64_t B, int64_t T,
                             float p_dropout, float p_dropout_prenet, uint64_t seed, float* grads, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (!e || !grads || !workspace) return gt_internal_fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || T <= 0 || T > TT_TMAX) return gt_internal_fail(GT_ERR_ARG, "bad B / T");
  const TrWs w = tr_layout(e, B, T);
  if (workspace_bytes < w.total) return gt_internal_fail(GT_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  char* base = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  {
    const auto it = e->tape_gen.find(base);
    if (it == e->tape_gen.end()) return gt_internal_fail(GT_ERR_ARG, "backward: no forward_train tape in this workspace");
    if (e->dirty || it->second.first != e->gen)
      return gt_internal_fail(GT_ERR_PARAM, "parameters changed between forward_train and backward");
  }
  const size_t usable = workspace_bytes - (size_t)(base - (char*)workspace);
  bool bad_ptr = false;
  auto F = [&](size_t o) { return tape_ptr(w, base, o, usable, bad_ptr); };   // o: byte offset (tr_layout)
  auto P = [&](const std::string& k) { return e->dev + e->off[e->index.at(k)]; };
  auto G = [&](const std::string& k) { return grads + e->off[e->index.at(k)]; };
  hipError_t err = hipSuccess;
  auto chk = [&](hipError_t x) { if (err == hipSuccess) err = x; };
  const int C = e->C, Bi = (int)B, Ti = (int)T, K = e->K, Fc = e->Fc, Fd = e->Fdp, NF = e->n_feats;
  const long npos = (long)B * T;
  const float pd = p_dropout, ppre = p_dropout_prenet;
  const float* mask = F(w.mask);
  const Drop none = make_drop(0, 0, 0.f);
  float *G1 = F(w.g1), *G2 = F(w.g2), *DATT = F(w.datt), *DY = F(w.dy), *DH = F(w.dh), *DQKV = F(w.dqkv);
  // dW / db of conv `key` (Cout x Cin x k) from dout [npos][d_cs] and its input x [npos][x_cs] (* xm)
  auto wgrad = [&](const float* dout, int d_cs, const float* xin, int x_cs, const float* xm, const std::string& key,
                   int cout, int cin, int k) {
    WgradParams p{};
    p.dout = dout; p.d_cs = d_cs; p.x = xin; p.x_cs = x_cs; p.x_mask = xm;
    p.B = Bi; p.T = Ti; p.Cin = cin; p.Cout = cout; p.K = k; p.pad = k / 2;
    chk(launch_tt_wgrad(p, G(key + ".weight"), F(w.wpart), w.wpart_floats, s));
    chk(launch_tt_colsum(dout, d_cs, npos, cout, F(w.cpart), w.cpart_floats, G(key + ".bias"), s));
  };
  // dx [npos][out_cs] (=|+=) conv^T(dout) (* m): the input gradient of conv `key` as a conv over dout with the taps
  // flipped and the weight strides swapped (W'(c, o, j) = W(o, c, k - 1 - j), padding k - 1 - k / 2)
  auto dgrad = [&](const float* dout, int d_cs, const std::string& key, int cout, int cin, int k, float* dx,
                   int out_cs, int accumulate, const float* m) {
    C1dParams p = c1d_defaults();
    p.in = dout; p.in_cs = d_cs; p.w = P(key + ".weight"); p.bias = nullptr;
    p.wpk = e->devpk + e->pktoff.at(key + ".weight");   // packed path when the channel counts allow it
    p.B = Bi; p.T = Ti; p.Q = Ti; p.Tout = Ti; p.Cin = cout; p.Cout = cin; p.K = k; p.pad = k - 1 - k / 2;
    p.wso = k; p.wsc = (long)cin * k; p.tap0 = k - 1; p.tap_step = -1;
    p.out = dx; p.out_cs = out_cs; p.accumulate = accumulate; p.out_mask = m;
    chk(launch_c1d(p, s));
  };
  auto lnb = [&](const float* x, const float* res, const std::string& key, int c, const float* dy, Drop drop,
                 const float* relu_ref, int post_relu, float* dx, int accumulate, const float* dx_mask) {
    LnBwdParams p{};
    p.x = x; p.x_cs = c; p.res = res; p.res_cs = c; p.gamma = P(key + ".gamma"); p.C = c; p.eps = 1e-4f; p.npos = npos;
    p.dy = dy; p.dy_cs = c; p.drop = drop; p.relu_ref = relu_ref; p.post_relu = post_relu; p.dx_mask = dx_mask;
    p.dx = dx; p.dx_cs = c; p.dx_accumulate = accumulate; p.part = F(w.lpart);
    chk(launch_tt_ln_bwd(p, G(key + ".gamma"), s));   // gamma | beta are adjacent in the inventory
  };
  auto ew = [&](float* dst, int dst_cs, const float* src, int src_cs, int chan_major, int c, const float* m, Drop drop,
                const float* relu_ref, int relu_cs) {
    EwParams p{};
    p.dst = dst; p.dst_cs = dst_cs; p.src = src; p.src_cs = src_cs; p.src_chan_major = chan_major; p.npos = npos;
    p.T = Ti; p.C = c; p.mask = m; p.drop = drop; p.relu_ref = relu_ref; p.relu_cs = relu_cs;
    chk(launch_tt_ew(p, s));
  };
  const float* xf = F(w.xout[e->L - 1]);
  // ---- duration predictor (its input is detached: the gradient stops at proj_w.conv_1's parameters)
  float* DLW = F(w.dmu);
  ew(DLW, 1, dlogw, 1, 0, 1, mask, none, nullptr, 0);   // NULL upstream gradient: zeros
  wgrad(DLW, 1, F(w.d2d), Fd, mask, "proj_w.proj", 1, Fd, 1);
  dgrad(DLW, 1, "proj_w.proj", 1, Fd, 1, DH, Fd, 0, mask);
  lnb(F(w.d2c), nullptr, "proj_w.norm_2", Fd, DH, make_drop(seed, 9, pd), nullptr, 1, DY, 0, nullptr);
  wgrad(DY, Fd, F(w.d1d), Fd, mask, "proj_w.conv_2", Fd, Fd, K);
  dgrad(DY, Fd, "proj_w.conv_2", Fd, Fd, K, DH, Fd, 0, mask);
  lnb(F(w.d1c), nullptr, "proj_w.norm_1", Fd, DH, make_drop(seed, 8, pd), nullptr, 1, DY, 0, nullptr);
  wgrad(DY, Fd, xf, C, mask, "proj_w.conv_1", Fd, C, K);
  // ---- mu_x = proj_m(x) * x_mask, x = x * x_mask (:281, :330)
  float* DMU = F(w.dmu);
  ew(DMU, NF, dmu_x, NF, 1, NF, mask, none, nullptr, 0);
  wgrad(DMU, NF, xf, C, nullptr, "proj_m", NF, C, 1);
  dgrad(DMU, NF, "proj_m", NF, C, 1, G1, C, 0, mask);
  // ---- encoder layers, last to first; G1 = dL/d(layer output), masked
  for (int l = e->L - 1; l >= 0; --l) {
    const std::string a = "encoder.attn_layers." + std::to_string(l) + ".";
    const std::string f = "encoder.ffn_layers." + std::to_string(l) + ".";
    const uint32_t site = 16 + 8 * l;
    const float* xin = l ? F(w.xout[l - 1]) : F(w.x1);
    // x_out = LN2(x_mid + drop(FFN(x_mid)))
    lnb(F(w.xmid[l]), F(w.y2[l]), "encoder.norm_layers_2." + std::to_string(l), C, G1, none, nullptr, 0, G2, 0,
        nullptr);
    ew(DY, C, G2, C, 0, C, mask, make_drop(seed, site + 3, pd), nullptr, 0);
    wgrad(DY, C, F(w.hd[l]), Fc, mask, f + "conv_2", C, Fc, K);
    dgrad(DY, C, f + "conv_2", C, Fc, K, DH, Fc, 0, nullptr);
    ew(DH, Fc, DH, Fc, 0, Fc, mask, make_drop(seed, site + 2, pd), F(w.hd[l]), Fc);
    wgrad(DH, Fc, F(w.xmid[l]), C, mask, f + "conv_1", Fc, C, K);
    dgrad(DH, Fc, f + "conv_1", Fc, C, K, G2, C, 1, mask);
    // x_mid = LN1(x_in + drop(attn(x_in)))
    lnb(xin, F(w.y1[l]), "encoder.norm_layers_1." + std::to_string(l), C, G2, none, nullptr, 0, G1, 0, nullptr);
    ew(DY, C, G1, C, 0, C, nullptr, make_drop(seed, site + 1, pd), nullptr, 0);
    wgrad(DY, C, F(w.att[l]), C, nullptr, a + "conv_o", C, C, 1);
    dgrad(DY, C, a + "conv_o", C, C, 1, DATT, C, 0, nullptr);
    chk(launch_tt_attn_bwd(F(w.qkv[l]), F(w.P[l]), F(w.Pd[l]), F(w.PdT[l]), DATT, mask, P(a + "emb_rel_k"),
                           P(a + "emb_rel_v"), Bi, Ti, C, e->H, e->W, make_drop(seed, site, pd), F(w.ds), F(w.dsT), DQKV,
                           F(w.drel), G(a + "emb_rel_k"), s));
    const char* qkvn[3] = {"conv_q", "conv_k", "conv_v"};
    for (int j = 0; j < 3; ++j) {
      wgrad(DQKV + j * C, 3 * C, xin, C, nullptr, a + qkvn[j], C, C, 1);
      dgrad(DQKV + j * C, 3 * C, a + qkvn[j], C, C, 1, G1, C, 1, mask);   // x_in = x * x_mask (:274)
    }
  }
  // ---- prenet: x1 = (x0 + proj(h2)) * x_mask; G1 = dL/dx1 (masked) is also dL/dx0's residual part
  wgrad(G1, C, F(w.pre_h[2]), C, nullptr, "prenet.proj", C, C, 1);
  dgrad(G1, C, "prenet.proj", C, C, 1, DH, C, 0, nullptr);
  for (int i = 2; i >= 0; --i) {
    const std::string k = std::to_string(i);
    lnb(F(w.pre_c[i]), nullptr, "prenet.norm_layers." + k, C, DH, make_drop(seed, 1 + i, ppre), F(w.pre_h[i]), 0, DY,
        0, nullptr);
    const float* xin = i ? F(w.pre_h[i - 1]) : F(w.x0);
    wgrad(DY, C, xin, C, mask, "prenet.conv_layers." + k, C, C, 5);
    if (i) dgrad(DY, C, "prenet.conv_layers." + k, C, C, 5, DH, C, 0, mask);
    else dgrad(DY, C, "prenet.conv_layers." + k, C, C, 5, G1, C, 1, mask);
  }
  chk(launch_tt_emb_bwd((const int64_t*)F(w.tokens), npos, G1, e->n_vocab, C, (float)std::sqrt((double)C),
                        G("emb.weight"), F(w.wpart), w.wpart_floats, s));
  if (err != hipSuccess) return gt_internal_fail(GT_ERR_HIP, std::string("text encoder backward: ") + hipGetErrorString(err));
  if (bad_ptr) return gt_internal_fail(GT_ERR_WORKSPACE, "text encoder backward: tape offset outside the layout");
  return GT_OK;
}

int gt_path_scatter(const float* attn, const float* dmu_y, int64_t B, int64_t Tx, int64_t Ty, int32_t n_feats,
                    float* dmu_x, void* stream) {
  if (!attn || !dmu_y || !dmu_x || B <= 0 || Tx <= 0 || Ty <= 0 || n_feats <= 0 || n_feats > 128)
    return gt_internal_fail(GT_ERR_ARG, "bad argument");
  const hipError_t e = launch_tt_path_scatter(attn, dmu_y, (int)B, (int)Tx, (int)Ty, n_feats, dmu_x, (hipStream_t)stream);
  return e == hipSuccess ? GT_OK : gt_internal_fail(GT_ERR_HIP, hipGetErrorString(e));
}

size_t gt_tts_aux_losses_workspace_bytes(int64_t B, int64_t Tx) {
  return B > 0 && Tx > 0 ? (size_t)tt_aux_loss_scratch_doubles(B, Tx) * 8 + 8 : 0;
}

int gt_tts_aux_losses(const float* logw, const float* attn, const float* x_mask, const int64_t* x_lengths, int64_t B,
                      int64_t Tx, int64_t Ty_attn, const float* y, const float* mu_y, const float* y_mask, int64_t Ty,
                      int32_t n_feats, float* losses, float* dlogw_unit, float* dmu_y_unit, void* workspace,
                      size_t workspace_bytes, void* stream) {
  if (!logw || !attn || !x_mask || !x_lengths || !y || !mu_y || !y_mask || !losses || !dlogw_unit || !dmu_y_unit ||
      !workspace || B <= 0 || Tx <= 0 || Ty_attn <= 0 || Ty <= 0 || n_feats <= 0)
    return gt_internal_fail(GT_ERR_ARG, "bad argument");
  if (workspace_bytes < gt_tts_aux_losses_workspace_bytes(B, Tx)) return gt_internal_fail(GT_ERR_WORKSPACE, "workspace too small");
  double* scratch = (double*)(((uintptr_t)workspace + 7) & ~(uintptr_t)7);
  const hipError_t e = launch_tt_aux_loss(logw, attn, x_mask, x_lengths, y, mu_y, y_mask, (int)B, (int)Tx, (int)Ty_attn,
                                          (int)Ty, n_feats, losses, dlogw_unit, dmu_y_unit, scratch, (hipStream_t)stream);
  return e == hipSuccess ? GT_OK : gt_internal_fail(GT_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
