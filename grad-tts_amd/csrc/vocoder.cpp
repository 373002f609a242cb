// HiFi-GAN generator (hifi-gan/models.py:77-128, ResBlock1 :13-48, ResBlock2 :53-74) on the MI355X: the vocoder that turns the
// decoder's mel into audio (inference.py:97). fp32; activations channels-last [B][T][C]; every conv is the fp32-MFMA
// c1d kernel (textenc.hip) with the leaky ReLU folded into its operand staging and the residual / resblock
// average / tanh into its epilogue:
//   conv_pre                 k7 on the channel-major mel
//   ups[i] (ConvTranspose1d)  u phases, each a 2-tap conv over the input (taps r and r + u of the kernel, input
//                             frames q and q - 1) writing output frames q u + r - P: no zero-stuffed input
//   resblocks                 per stage num_kernels resblocks (ResBlock1: per dilation leaky -> dilated conv -> leaky ->
//                             conv -> + x; ResBlock2: per dilation leaky -> dilated conv -> + x); the last conv of each
//                             adds the residual and accumulates into the stage sum (the last resblock divides by
//                             num_kernels: x = xs / num_kernels)
//   conv_post                 leaky ReLU (0.01) staged, k7, tanh in the epilogue
// Weight norm (weight_g, weight_v) is baked on upload as remove_weight_norm() does (inference.py:76).
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

struct gt_vocoder {
  int n_mels, c0, n_up, nk;
  int rb_type = 1;                       // h.resblock: 1 (ResBlock1) or 2 (ResBlock2)
  std::vector<int> rates, kernels, rb_k;
  std::vector<std::vector<int>> rb_d;
  std::vector<std::pair<std::string, std::vector<int64_t>>> inv;
  std::map<std::string, int> index;
  std::vector<std::vector<float>> host;
  std::vector<bool> set;
  std::map<std::string, int64_t> woff;   // effective (weight-normed) weight / bias offsets in dev
  float* dev = nullptr;
  int64_t dev_numel = 0;
  bool dirty = true;
  int bf16 = 0;                          // compute dtype: 0 fp32, 1 bf16 operands (fp32 accumulation)
  std::map<std::string, int64_t> bfoff;  // bf16 weights [o][k][c] (ups: [phase][o][2][c]) in devbf
  uint16_t* devbf = nullptr;
  int64_t devbf_numel = 0;
  float* devpk = nullptr;                // fp32 weights in the same [o][k][c] layout (c1d_pk_kernel), offsets = bfoff
  int64_t devpk_numel = 0;
};

namespace {

int64_t prod(const std::vector<int64_t>& d) { int64_t n = 1; for (auto v : d) n *= v; return n; }

uint16_t to_bf16(float f) {   // round to nearest even (finite weights)
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

void add_wn(gt_vocoder* v, const std::string& k, std::vector<int64_t> w, int64_t bias_n) {
  v->inv.push_back({k + ".bias", {bias_n}});
  v->inv.push_back({k + ".weight_g", {w[0], 1, 1}});
  v->inv.push_back({k + ".weight_v", w});
}

int upload(gt_vocoder* v) {
  for (size_t i = 0; i < v->inv.size(); ++i)
    if (!v->set[i]) return gt_internal_fail(GT_ERR_PARAM, "vocoder parameter never set: " + v->inv[i].first);
  if (!v->dirty) return GT_OK;
  std::vector<float> h;
  v->woff.clear();
  for (size_t i = 0; i < v->inv.size(); i += 3) {   // (bias, weight_g, weight_v) per conv
    const std::string key = v->inv[i].first.substr(0, v->inv[i].first.size() - 5);
    const std::vector<float>& b = v->host[i];
    const std::vector<float>& g = v->host[i + 1];
    const std::vector<float>& vv = v->host[i + 2];
    const int64_t d0 = v->inv[i + 2].second[0], rest = prod(v->inv[i + 2].second) / d0;
    v->woff[key + ".weight"] = (int64_t)h.size();
    for (int64_t a = 0; a < d0; ++a) {   // w = v * (g / ||v||), norm over all dims but 0 (torch._weight_norm, dim 0)
      double n2 = 0.0;
      for (int64_t j = 0; j < rest; ++j) n2 += (double)vv[a * rest + j] * vv[a * rest + j];
      const double sc = (double)g[a] / std::sqrt(n2);
      for (int64_t j = 0; j < rest; ++j) h.push_back((float)((double)vv[a * rest + j] * sc));
    }
    v->woff[key + ".bias"] = (int64_t)h.size();
    h.insert(h.end(), b.begin(), b.end());
  }
  // bf16 and fp32 copies of the effective weights in the operand layout of c1d_bf16_kernel / c1d_pk_kernel
  std::vector<uint16_t> hb;
  std::vector<float> hp;
  v->bfoff.clear();
  for (size_t i = 0; i < v->inv.size(); i += 3) {
    const std::string key = v->inv[i].first.substr(0, v->inv[i].first.size() - 5);
    const std::vector<int64_t>& d = v->inv[i + 2].second;
    const float* w = h.data() + v->woff[key + ".weight"];
    v->bfoff[key] = (int64_t)hp.size();
    if (key.rfind("ups.", 0) == 0) {   // ConvTranspose1d [Cin][Cout][k], k = 2u: per phase r, [o][j][c] = w[c][o][r + u j]
      const int64_t ci = d[0], co = d[1], kk = d[2], u = kk / 2;
      for (int64_t r = 0; r < u; ++r)
        for (int64_t o = 0; o < co; ++o)
          for (int64_t j = 0; j < 2; ++j)
            for (int64_t c = 0; c < ci; ++c) hp.push_back(w[(c * co + o) * kk + r + u * j]);
    } else {                             // Conv1d [Cout][Cin][k] -> [o][k][c]
      const int64_t co = d[0], ci = d[1], kk = d[2];
      for (int64_t o = 0; o < co; ++o)
        for (int64_t k = 0; k < kk; ++k)
          for (int64_t c = 0; c < ci; ++c) hp.push_back(w[(o * ci + c) * kk + k]);
    }
    while (hp.size() % 8) hp.push_back(0.f);   // 16-byte aligned bf16 starts (32-byte fp32)
  }
  hb.reserve(hp.size());
  for (float x : hp) hb.push_back(to_bf16(x));
  if (v->devpk && (int64_t)hp.size() != v->devpk_numel) { (void)hipFree(v->devpk); v->devpk = nullptr; }
  if (!v->devpk && hipMalloc(&v->devpk, hp.size() * 4) != hipSuccess) return gt_internal_fail(GT_ERR_HIP, "hipMalloc failed");
  v->devpk_numel = (int64_t)hp.size();
  if (hipMemcpy(v->devpk, hp.data(), hp.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, "hipMemcpy failed");
  if (v->devbf && (int64_t)hb.size() != v->devbf_numel) { (void)hipFree(v->devbf); v->devbf = nullptr; }
  if (!v->devbf && hipMalloc(&v->devbf, hb.size() * 2) != hipSuccess) return gt_internal_fail(GT_ERR_HIP, "hipMalloc failed");
  v->devbf_numel = (int64_t)hb.size();
  if (hipMemcpy(v->devbf, hb.data(), hb.size() * 2, hipMemcpyHostToDevice) != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, "hipMemcpy failed");
  if (v->dev && (int64_t)h.size() != v->dev_numel) { (void)hipFree(v->dev); v->dev = nullptr; }
  if (!v->dev && hipMalloc(&v->dev, h.size() * 4) != hipSuccess) return gt_internal_fail(GT_ERR_HIP, "hipMalloc failed");
  v->dev_numel = (int64_t)h.size();
  if (hipMemcpy(v->dev, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, "hipMemcpy failed");
  v->dirty = false;
  return GT_OK;
}

int64_t max_buf(const gt_vocoder* v, int64_t T) {   // largest [T_stage][C_stage] of the generator
  int64_t t = T, c = v->c0, m = t * c;
  for (int i = 0; i < v->n_up; ++i) { t *= v->rates[i]; c /= 2; m = std::max(m, t * c); }
  return m;
}

}  // namespace

extern "C" {

int gt_vocoder_create2(int n_mels, int upsample_initial_channel, int n_up, const int* upsample_rates,
                       const int* upsample_kernel_sizes, int n_kernels, const int* resblock_kernel_sizes, int resblock,
                       int n_dil, const int* resblock_dilations, gt_vocoder** out) {
  if (!out || !upsample_rates || !upsample_kernel_sizes || !resblock_kernel_sizes || !resblock_dilations)
    return gt_internal_fail(GT_ERR_ARG, "null argument");
  *out = nullptr;
  if (n_up <= 0 || n_kernels <= 0 || n_dil <= 0 || upsample_initial_channel >> n_up <= 0)
    return gt_internal_fail(GT_ERR_ARG, "bad configuration");
  if (resblock != 1 && resblock != 2) return gt_internal_fail(GT_ERR_ARG, "resblock must be 1 or 2 (h.resblock)");
  for (int i = 0; i < n_up; ++i)
    if (upsample_kernel_sizes[i] != 2 * upsample_rates[i])
      return gt_internal_fail(GT_ERR_UNSUPPORTED, "upsampling implemented for kernel = 2 x rate (HiFi-GAN V1/V2/V3)");
  for (int j = 0; j < n_kernels; ++j)
    for (int m = 0; m < n_dil; ++m)
      if ((resblock_kernel_sizes[j] - 1) * resblock_dilations[j * n_dil + m] > 80 || resblock_kernel_sizes[j] > 11 ||
          resblock_dilations[j * n_dil + m] < 1)
        return gt_internal_fail(GT_ERR_UNSUPPORTED, "resblock kernel <= 11 and 1 <= dilation, (k - 1) dilation <= 80");
  gt_vocoder* v = new gt_vocoder();
  v->n_mels = n_mels; v->c0 = upsample_initial_channel; v->n_up = n_up; v->nk = n_kernels; v->rb_type = resblock;
  v->rates.assign(upsample_rates, upsample_rates + n_up);
  v->kernels.assign(upsample_kernel_sizes, upsample_kernel_sizes + n_up);
  v->rb_k.assign(resblock_kernel_sizes, resblock_kernel_sizes + n_kernels);
  for (int j = 0; j < n_kernels; ++j)
    v->rb_d.push_back(std::vector<int>(resblock_dilations + j * n_dil, resblock_dilations + (j + 1) * n_dil));
  add_wn(v, "conv_pre", {v->c0, n_mels, 7}, v->c0);
  for (int i = 0; i < n_up; ++i)
    add_wn(v, "ups." + std::to_string(i), {v->c0 >> i, v->c0 >> (i + 1), v->kernels[i]}, v->c0 >> (i + 1));
  int n = 0;
  for (int i = 0; i < n_up; ++i) {   // registration order of the reference modules (weight_norm: bias, g, v)
    const int64_t ch = v->c0 >> (i + 1);
    for (int j = 0; j < n_kernels; ++j, ++n) {
      const std::string rk = "resblocks." + std::to_string(n) + ".";
      if (resblock == 1) {
        for (const char* part : {"convs1", "convs2"})
          for (int m = 0; m < n_dil; ++m) add_wn(v, rk + part + "." + std::to_string(m), {ch, ch, v->rb_k[j]}, ch);
      } else {
        for (int m = 0; m < n_dil; ++m) add_wn(v, rk + "convs." + std::to_string(m), {ch, ch, v->rb_k[j]}, ch);
      }
    }
  }
  add_wn(v, "conv_post", {1, v->c0 >> n_up, 7}, 1);
  for (size_t i = 0; i < v->inv.size(); ++i) v->index[v->inv[i].first] = (int)i;
  v->host.resize(v->inv.size());
  v->set.assign(v->inv.size(), false);
  *out = v;
  return GT_OK;
}

int gt_vocoder_create(int n_mels, int upsample_initial_channel, int n_up, const int* upsample_rates,
                      const int* upsample_kernel_sizes, int n_kernels, const int* resblock_kernel_sizes,
                      const int* resblock_dilations, gt_vocoder** out) {
  return gt_vocoder_create2(n_mels, upsample_initial_channel, n_up, upsample_rates, upsample_kernel_sizes, n_kernels,
                            resblock_kernel_sizes, 1, 3, resblock_dilations, out);
}

void gt_vocoder_destroy(gt_vocoder* v) {
  if (!v) return;
  if (v->dev) (void)hipFree(v->dev);
  if (v->devbf) (void)hipFree(v->devbf);
  if (v->devpk) (void)hipFree(v->devpk);
  delete v;
}

int gt_vocoder_num_params(gt_vocoder* v) { return v ? (int)v->inv.size() : -1; }
const char* gt_vocoder_param_name(gt_vocoder* v, int i) {
  return (v && i >= 0 && i < (int)v->inv.size()) ? v->inv[i].first.c_str() : nullptr;
}
int64_t gt_vocoder_param_numel(gt_vocoder* v, int i) {
  return (v && i >= 0 && i < (int)v->inv.size()) ? prod(v->inv[i].second) : -1;
}
int gt_vocoder_set_param(gt_vocoder* v, const char* name, const float* data, int64_t numel) {
  if (!v || !name || !data) return gt_internal_fail(GT_ERR_ARG, "null argument");
  auto it = v->index.find(name);
  if (it == v->index.end()) return gt_internal_fail(GT_ERR_PARAM, std::string("unknown parameter: ") + name);
  if (numel != prod(v->inv[it->second].second)) return gt_internal_fail(GT_ERR_PARAM, std::string("numel mismatch for ") + name);
  v->host[it->second].assign(data, data + numel);
  v->set[it->second] = true;
  v->dirty = true;
  return GT_OK;
}

int gt_vocoder_set_compute_dtype(gt_vocoder* v, int dtype) {
  if (!v || (dtype != 0 && dtype != 1)) return gt_internal_fail(GT_ERR_ARG, "dtype must be 0 (fp32) or 1 (bf16)");
  v->bf16 = dtype;
  return GT_OK;
}

int64_t gt_vocoder_hop(gt_vocoder* v) {
  if (!v) return -1;
  int64_t h = 1;
  for (int r : v->rates) h *= r;
  return h;
}

size_t gt_vocoder_workspace_bytes(gt_vocoder* v, int64_t B, int64_t T) {
  if (!v || B <= 0 || T <= 0) return 0;
  const size_t n = (size_t)B * max_buf(v, T);
  return 4 * (((n * 4 + 255) & ~size_t(255))) + 256;
}

int gt_vocoder_forward(gt_vocoder* v, const float* mel, int64_t B, int64_t T, float* audio, void* workspace,
                       size_t workspace_bytes, void* stream) {
  if (!v || !mel || !audio || !workspace || B <= 0 || T <= 0) return gt_internal_fail(GT_ERR_ARG, "bad argument");
  if (workspace_bytes < gt_vocoder_workspace_bytes(v, B, T)) return gt_internal_fail(GT_ERR_WORKSPACE, "workspace too small");
  int rc = upload(v);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const size_t nb = (((size_t)B * max_buf(v, T) * 4 + 255) & ~size_t(255));
  char* base = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  float* buf[4] = {(float*)base, (float*)(base + nb), (float*)(base + 2 * nb), (float*)(base + 3 * nb)};
  auto W = [&](const std::string& k) { return v->dev + v->woff.at(k + ".weight"); };
  auto Bs = [&](const std::string& k) { return v->dev + v->woff.at(k + ".bias"); };
  hipError_t err = hipSuccess;
  auto chk = [&](hipError_t x) { if (err == hipSuccess) err = x; };
  const int Bi = (int)B;
  auto launch = [&](C1dParams& p, const std::string& key, int phase) {   // fp32 or bf16 operands per the handle
    const int64_t off = v->bfoff.at(key) + (int64_t)phase * p.Cout * p.K * p.Cin;
    if (v->bf16) {
      p.bf16 = 1;
      p.wbf = v->devbf + off;
    } else {
      p.wpk = v->devpk + off;
    }
    chk(launch_c1d(p, s));
  };
  // conv_pre: channel-major mel [B][n_mels][T] -> [B][T][c0]
  float* x = buf[0];
  {
    C1dParams p = c1d_defaults();
    p.in = mel; p.in_chan_major = 1; p.w = W("conv_pre"); p.bias = Bs("conv_pre");
    p.wso = (long)v->n_mels * 7; p.wsc = 7;
    p.B = Bi; p.T = (int)T; p.Q = (int)T; p.Tout = (int)T; p.Cin = v->n_mels; p.Cout = v->c0; p.K = 7; p.pad = 3;
    p.out = x; p.out_cs = v->c0;
    launch(p, "conv_pre", 0);
  }
  int Tin = (int)T, cin = v->c0, n = 0;
  for (int i = 0; i < v->n_up; ++i) {
    const int u = v->rates[i], k = v->kernels[i], P = (k - u) / 2, cout = cin / 2, Tout = Tin * u;
    const std::string key = "ups." + std::to_string(i);
    float* xu = buf[1];
    for (int r = 0; r < u; ++r) {   // phase r: out[q u + r - P] = W[:, :, r] x[q] + W[:, :, r + u] x[q - 1]
      C1dParams p = c1d_defaults();
      p.in = x; p.in_cs = cin; p.in_act = 1; p.in_slope = 0.1f;
      p.w = W(key); p.bias = Bs(key); p.wso = k; p.wsc = (long)cout * k; p.tap0 = r; p.tap_step = u;
      p.B = Bi; p.T = Tin; p.Cin = cin; p.Cout = cout; p.K = 2; p.pad = 0; p.dil = -1;
      p.Q = Tin + 1; p.Tout = Tout; p.out_stride = u; p.out_off = r - P;
      p.out = xu; p.out_cs = cout;
      launch(p, key, r);
    }
    float* cur = buf[2];
    float* t1 = buf[3];
    float* xs = buf[0];   // the stage input x is dead after the upsampling
    for (int j = 0; j < v->nk; ++j, ++n) {
      const int kk = v->rb_k[j], nd = (int)v->rb_d[j].size();
      const float* y = xu;
      if (v->rb_type == 2) {   // ResBlock2 (models.py:68-72): y = conv_m(leaky_relu(y, 0.1)) + y per dilation
        for (int m = 0; m < nd; ++m) {
          const int d = v->rb_d[j][m];
          const std::string c = "resblocks." + std::to_string(n) + ".convs." + std::to_string(m);
          C1dParams q = c1d_defaults();
          q.in = y; q.in_cs = cout; q.in_act = 1; q.in_slope = 0.1f;
          q.w = W(c); q.bias = Bs(c); q.wso = (long)cout * kk; q.wsc = kk;
          q.B = Bi; q.T = Tout; q.Q = Tout; q.Tout = Tout; q.Cin = cout; q.Cout = cout; q.K = kk; q.dil = d;
          q.pad = (kk * d - d) / 2; q.res = y; q.res_cs = cout; q.out_cs = cout;
          if (m < nd - 1) {
            q.out = (y == cur) ? t1 : cur;   // ping-pong: a dilated conv never writes the tensor it reads
          } else {
            q.out = xs; q.accumulate = j > 0;
            if (j == v->nk - 1) q.div = (float)v->nk;
          }
          launch(q, c, 0);
          y = q.out;
        }
        continue;
      }
      for (int m = 0; m < nd; ++m) {
        const int d = v->rb_d[j][m];
        const std::string c1 = "resblocks." + std::to_string(n) + ".convs1." + std::to_string(m);
        const std::string c2 = "resblocks." + std::to_string(n) + ".convs2." + std::to_string(m);
        C1dParams p = c1d_defaults();   // xt = c1(leaky_relu(y, 0.1))
        p.in = y; p.in_cs = cout; p.in_act = 1; p.in_slope = 0.1f;
        p.w = W(c1); p.bias = Bs(c1); p.wso = (long)cout * kk; p.wsc = kk;
        p.B = Bi; p.T = Tout; p.Q = Tout; p.Tout = Tout; p.Cin = cout; p.Cout = cout; p.K = kk; p.dil = d;
        p.pad = (kk * d - d) / 2; p.out = t1; p.out_cs = cout;
        launch(p, c1, 0);
        C1dParams q = c1d_defaults();   // y = c2(leaky_relu(xt, 0.1)) + y
        q.in = t1; q.in_cs = cout; q.in_act = 1; q.in_slope = 0.1f;
        q.w = W(c2); q.bias = Bs(c2); q.wso = (long)cout * kk; q.wsc = kk;
        q.B = Bi; q.T = Tout; q.Q = Tout; q.Tout = Tout; q.Cin = cout; q.Cout = cout; q.K = kk; q.pad = (kk - 1) / 2;
        q.res = y; q.res_cs = cout; q.out_cs = cout;
        if (m < nd - 1) {
          q.out = cur;
        } else {   // last conv of the resblock: xs (+)= y; the stage's last divides by num_kernels
          q.out = xs; q.accumulate = j > 0;
          if (j == v->nk - 1) q.div = (float)v->nk;
        }
        launch(q, c2, 0);
        y = cur;
      }
    }
    x = xs;   // = buf[0] again: every stage reads buf[0], upsamples into buf[1], sums its resblocks into buf[0]
    Tin = Tout; cin = cout;
  }
  {
    C1dParams p = c1d_defaults();   // tanh(conv_post(leaky_relu(x, 0.01)))
    p.in = x; p.in_cs = cin; p.in_act = 1; p.in_slope = 0.01f;
    p.w = W("conv_post"); p.bias = Bs("conv_post"); p.wso = (long)cin * 7; p.wsc = 7;
    p.B = Bi; p.T = Tin; p.Q = Tin; p.Tout = Tin; p.Cin = cin; p.Cout = 1; p.K = 7; p.pad = 3;
    p.out = audio; p.out_cs = 1; p.out_tanh = 1;
    launch(p, "conv_post", 0);
  }
  if (err != hipSuccess) return gt_internal_fail(GT_ERR_HIP, std::string("vocoder launch failed: ") + hipGetErrorString(err));
  return GT_OK;
}

}  // extern "C"
