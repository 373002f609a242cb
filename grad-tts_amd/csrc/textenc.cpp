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
#include "textenc.h"

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
  for (size_t i = 0; i < e->inv.size(); ++i) {
    const auto& d = e->inv[i].second;
    if (d.size() != 3 || e->inv[i].first.find(".weight") == std::string::npos) continue;
    e->pkoff[e->inv[i].first] = (int64_t)hp.size();
    const float* w = e->host[i].data();
    for (int64_t o = 0; o < d[0]; ++o)
      for (int64_t k = 0; k < d[2]; ++k)
        for (int64_t c = 0; c < d[1]; ++c) hp.push_back(w[(o * d[1] + c) * d[2] + k]);
    while (hp.size() % 4) hp.push_back(0.f);   // 16-byte aligned starts
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
  if (e->dev) (void)hipFree(e->dev);
  if (e->devpk) (void)hipFree(e->devpk);
  delete e;
}

int gt_text_encoder_num_params(gt_text_encoder* e) { return e ? (int)e->inv.size() : -1; }
const char* gt_text_encoder_param_name(gt_text_encoder* e, int i) {
  return (e && i >= 0 && i < (int)e->inv.size()) ? e->inv[i].first.c_str() : nullptr;
}
int64_t gt_text_encoder_param_numel(gt_text_encoder* e, int i) {
  return (e && i >= 0 && i < (int)e->inv.size()) ? prod(e->inv[i].second) : -1;
}

int gt_text_encoder_set_param(gt_text_encoder* e, const char* name, const float* data, int64_t numel) {
  if (!e || !name || !data) return gt_internal_fail(GT_ERR_ARG, "null argument");
  auto it = e->index.find(name);
  if (it == e->index.end()) return gt_internal_fail(GT_ERR_PARAM, std::string("unknown parameter: ") + name);
  if (numel != prod(e->inv[it->second].second)) return gt_internal_fail(GT_ERR_PARAM, std::string("numel mismatch for ") + name);
  e->host[it->second].assign(data, data + numel);
  e->set[it->second] = true;
  e->dirty = true;
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
