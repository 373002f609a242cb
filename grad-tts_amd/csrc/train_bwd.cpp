// Training step of the decoder: Diffusion.loss_t forward with a tape, then the backward of
// the score U-Net to every parameter of GradLogPEstimator2d and to mu (model/diffusion.py:16-216, 244-281).
//
// fp32 throughout, channels-last activations; forward and backward are built from the fp32-MFMA kernels of bwd.hip
// (v_mfma_f32_32x32x2_f32 gather-relation convs, weight gradients, attention products), launched in the
// order of oracle/decoder.py's estimator and its reverse.
// Every intermediate the backward needs is kept in the workspace (the tape); a measuring pass of the same code
// sizes the workspace (gt_train_workspace_bytes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bwd.h"
#include "decoder_internal.h"
#include "gradtts.h"
#include "kernels.h"
#include "train.h"

using namespace gt;

namespace {

using Regions = std::vector<std::pair<uintptr_t, size_t>>;

struct Arena {   // bump allocator over the workspace; measure-only when base == nullptr
  uint8_t* base = nullptr;
  size_t off = 0;
  Regions* rec = nullptr;   // extent checking (GT_TRAIN_DEBUG=2): every buffer handed out
  float* take(size_t floats) {
    const size_t o = off;
    off = (off + floats * 4 + 255) & ~size_t(255);
    if (base && rec) rec->push_back({(uintptr_t)(base + o), floats * 4});
    return base ? reinterpret_cast<float*>(base + o) : nullptr;
  }
};

struct Lvl { int F, T; };

struct Trainer {
  gt_decoder* d;
  int B, T, n_spks, cin;
  float bmin, bmax, pe_scale, half_delta;
  hipStream_t s;
  Arena A;
  bool run;                 // false: measure the workspace only
  hipError_t err = hipSuccess;
  const float* mask;        // [B][T]
  float* grads;             // flat [numel] in inventory order
  std::vector<float*> dtb;  // per ResnetBlock: [B][C] gradient of its time bias

  int err_line = 0;
  std::string err_cur;
  bool debug = false;       // GT_TRAIN_DEBUG=1: synchronise after every launch and name the failing call site
  // GT_TRAIN_DEBUG=2 (dry): no launches; every helper checks on the host that the extents its kernel will touch lie
  // inside one buffer (arena allocation, caller buffer or the parameter block) and names the first that does not
  bool dry = false;
  Regions regions;
  std::string bad;
  bool live() const { return run && !dry; }
  bool pgrads = true;       // false (estimator VJP): no parameter-gradient work, only the input cotangents
  std::vector<GconvPack>* packs = nullptr;   // dry pass: every conv's weight repack (same arena, same addresses)
  bool packed_ahead = false;                 // live pass: the repacks ran before the forward
  void need(const void* p, long elems, const char* what, int line) {
    if (!dry || !bad.empty() || elems <= 0) return;
    const uintptr_t a = (uintptr_t)p, e = a + (uintptr_t)elems * 4;
    for (auto& r : regions)
      if (a >= r.first && e <= r.first + r.second) return;
    bad = std::string(what) + " out of range at train_bwd.cpp:" + std::to_string(line) + " (" + cur + ", " +
          std::to_string(elems) + " elements)";
  }
  void chk(hipError_t e, int line = __builtin_LINE()) {
    if (debug && e == hipSuccess && run) e = hipStreamSynchronize(s);
    if (err == hipSuccess && e != hipSuccess) { err = e; err_line = line; err_cur = cur; }
  }
  Lvl L(int l) const { return {80 >> l, T >> l}; }
  const float* P(const std::string& k) { return gt_internal_param(d, k); }
  float* G(const std::string& k) { return grads + gt_internal_param_offset(d, k); }
  static dim3 g1(long n) { return dim3((unsigned)((n + 255) / 256)); }

  // ------------------------------------------------------------ generic ops
  void gconv(const float* in, int Ci, int l_in, bool in_mask, const float* w, long wsa, long wsc, int KS, int S, int PAD,
             int flip, const float* bias, float* out, int Co, int l_out, bool out_mask, int out_cs, int out_c0, int acc,
             bool transposed = false, int line = __builtin_LINE()) {
    GConvParams p{};
    p.Cin = Ci; p.Cout = Co; p.KS = KS; p.S = S; p.transposed = transposed;
    const long nwpk = gconv_wpk_floats(p);   // repacked weights of this launch (taken in the measuring pass too)
    float* wpk = nwpk > 0 ? A.take((size_t)nwpk) : nullptr;
    if (!run) return;
    {
      const Lvl I = L(l_in), O = L(l_out);
      need(in, (long)B * I.F * I.T * Ci, "gconv in", line);
      need(out, ((long)B * O.F * O.T - 1) * out_cs + out_c0 + Co, "gconv out", line);
      need(w, (long)(Co - 1) * wsa + (long)(Ci - 1) * wsc + KS * KS, "gconv weight", line);
      if (bias) need(bias, Co, "gconv bias", line);
    }
    if (wpk) need(wpk, nwpk, "gconv packed weights", line);
    p.wpk = wpk;
    p.B = B; p.Fi = L(l_in).F; p.Ti = L(l_in).T; p.Cin = Ci; p.Fo = L(l_out).F; p.To = L(l_out).T; p.Cout = Co;
    p.KS = KS; p.S = S; p.PAD = PAD; p.transposed = transposed; p.flip = flip;
    p.in = in; p.w = w; p.wsa = wsa; p.wsc = wsc; p.bias = bias;
    p.mask = in_mask ? mask : nullptr; p.T0 = T; p.lvl_in = l_in;
    p.out_mask = out_mask ? mask : nullptr; p.lvl_out = l_out;
    p.out = out; p.out_cs = out_cs; p.out_c0 = out_c0; p.accumulate = acc;
    if (dry) {   // the dry pass collects the weight repacks; the live pass does them up front in a few launches
      GconvPack pk;
      if (packs && gconv_pack_desc(p, &pk)) packs->push_back(pk);
      return;
    }
    p.wpk_ready = packed_ahead ? 1 : 0;
    chk(launch_gconv(p, s), line);
  }
  // dW(a, b, k) (+)= sum_u P[u][a] Q[v(u,k)][b]; written at dw + a*sa + b*sb + k
  void wgrad(const float* Pt, int Ad, int l_u, bool pmask, const float* Qt, int Bd, int l_v, bool qmask, int KS, int S,
             int PAD, float* dw, long sa, long sb, int acc, int line = __builtin_LINE()) {
    const long nU = (long)B * L(l_u).F * L(l_u).T;
    float* part = wpart;
    if (!run) return;
    need(Pt, nU * Ad, "wgrad P", line);
    need(Qt, (long)B * L(l_v).F * L(l_v).T * Bd, "wgrad Q", line);
    if (!pgrads) return;
    need(dw, (long)(Ad - 1) * sa + (long)(Bd - 1) * sb + KS * KS, "wgrad dW", line);
    if (dry) return;
    WGradParams p{};
    p.B = B; p.Fu = L(l_u).F; p.Tu = L(l_u).T; p.A = Ad; p.Fv = L(l_v).F; p.Tv = L(l_v).T; p.Bc = Bd;
    p.KS = KS; p.S = S; p.PAD = PAD; p.P = Pt; p.pmask = pmask ? mask : nullptr; p.lvl_p = l_u;
    p.Q = Qt; p.qmask = qmask ? mask : nullptr; p.lvl_q = l_v; p.T0 = T;
    chk(launch_mwgrad(p, part, dw, sa, sb, acc, s), line);
  }
  // out[c] (+)= sum_{b, pos} x   (bias gradients): per-utterance sums, then over the batch in order
  void chansum(const float* x, int l, int C, float* out, int acc, int line = __builtin_LINE()) {
    const int npos = L(l).F * L(l).T;
    float* part = A.take((size_t)B * pos_splits(npos) * C);
    if (!run) return;
    need(x, (long)B * npos * C, "chansum x", line);
    if (!pgrads) return;
    need(out, C, "chansum out", line);
    if (dry) return;
    chk(launch_chan_sums(x, nullptr, B, npos, C, part, out, 0, acc, s), line);
  }
  // alphap / alpha2p: device scalars (a parameter in the fp32 block) in place of alpha / alpha2
  const float* ew_alphap = nullptr;
  const float* ew_alpha2p = nullptr;
  void ew(const float* x, int xcs, int xc0, float alpha, const float* x2, float alpha2, int l, int C, bool m, float* y,
          int ycs, int yc0, int acc, int line = __builtin_LINE()) {
    if (!run) return;
    {
      const long np = (long)B * L(l).F * L(l).T;
      need(x, (np - 1) * xcs + xc0 + C, "ew x", line);
      if (x2) need(x2, np * C, "ew x2", line);
      need(y, (np - 1) * ycs + yc0 + C, "ew y", line);
    }
    if (dry) return;
    EwParams p{};
    p.B = B; p.F = L(l).F; p.T = L(l).T; p.C = C; p.x = x; p.xcs = xcs; p.xc0 = xc0; p.alpha = alpha;
    p.x2 = x2; p.alpha2 = alpha2; p.mask = m ? mask : nullptr; p.T0 = T; p.lvl = l; p.y = y; p.ycs = ycs; p.yc0 = yc0;
    p.accumulate = acc;
    p.alphap = ew_alphap; p.alpha2p = ew_alpha2p;
    chk(launch_ew(g1((long)B * L(l).F * L(l).T * C), dim3(256), s, p), line);
  }
  BlockBwdParams bp(int l, int C, const float* h, const float* st, const std::string& gn) {
    BlockBwdParams p{};
    p.B = B; p.npos = L(l).F * L(l).T; p.T = L(l).T; p.C = C; p.h = h; p.stats = st;
    p.gamma = P(gn + ".weight"); p.beta = P(gn + ".bias"); p.mask = mask; p.T0 = T; p.lvl = l;
    return p;
  }
  float* gn_stats(const float* h, int l, int C) {
    float* st = A.take((size_t)B * 16);
    const int npos = L(l).F * L(l).T;
    double* part = reinterpret_cast<double*>(A.take((size_t)B * 8 * gn_splits(npos) * 4));
    if (live()) chk(launch_gn_stats_split(h, B, npos, C, part, st, s));
    return st;
  }
  float* block_fwd(int l, int C, const float* h, const float* st, const std::string& gn, const float* tb) {
    float* out = A.take((size_t)B * L(l).F * L(l).T * C);
    if (live()) chk(launch_block_fwd(g1((long)B * L(l).F * L(l).T * C), dim3(256), s, bp(l, C, h, st, gn), tb, out));
    return out;
  }
  // Block backward: dA -> dh, and the GroupNorm affine gradients
  float* block_bwd(int l, int C, const float* dAv, const float* h, const float* st, const std::string& gn,
                   int line = __builtin_LINE()) {
    float* gsum = A.take((size_t)B * 16);
    float* dgb = A.take((size_t)B * C * 2);
    float* dh = A.take((size_t)B * L(l).F * L(l).T * C);
    float* tw = A.take((size_t)B * C);
    float* tb2 = A.take((size_t)B * C);
    float* part = A.take((size_t)B * pos_splits((long)L(l).F * L(l).T) * C * 2);
    if (!run) return dh;
    {
      const long n = (long)B * L(l).F * L(l).T * C;
      need(dAv, n, "block_bwd dA", line);
      need(h, n, "block_bwd h", line);
      need(st, (long)B * 16, "block_bwd stats", line);
      need(P(gn + ".weight"), C, "block_bwd gamma", line);
      if (pgrads) {
        need(G(gn + ".weight"), C, "block_bwd dgamma", line);
        need(G(gn + ".bias"), C, "block_bwd dbeta", line);
      }
    }
    if (dry) return dh;
    BlockBwdParams p = bp(l, C, h, st, gn);
    p.dA = dAv; p.gsum = gsum; p.dgb = dgb; p.dh = dh;
    chk(launch_block_bwd_sums(p, part, s), line);
    chk(launch_block_bwd_apply(g1((long)B * p.npos * C), dim3(256), s, p), line);
    if (pgrads) chk(launch_colsum_strided(gn, dgb, C, tw, tb2), line);   // dgamma, dbeta = sums over the batch
    return dh;
  }
  // dgb [B][C][2] -> G(gn.weight)[c] += sum_b dgb[b][c][0]; G(gn.bias)[c] += sum_b dgb[b][c][1]
  hipError_t launch_colsum_strided(const std::string& gn, const float* dgb, int C, float* tw, float* tb2) {
    EwParams p{};
    p.alpha = 1.f; p.T0 = 1; p.accumulate = 0; p.x = dgb;
    // the two planes of [B][C][2] viewed as [B*C] positions of 2 channels
    p.B = 1; p.F = 1; p.T = B * C; p.C = 1; p.xcs = 2; p.xc0 = 0; p.y = tw; p.ycs = 1; p.yc0 = 0;
    hipError_t e = launch_ew(g1((long)B * C), dim3(256), s, p);
    if (e != hipSuccess) return e;
    p.xc0 = 1; p.y = tb2;
    e = launch_ew(g1((long)B * C), dim3(256), s, p);
    if (e != hipSuccess) return e;
    e = launch_colsum(dim3((C + 255) / 256), dim3(256), s, tw, B, C, G(gn + ".weight"), 1);
    if (e != hipSuccess) return e;
    return launch_colsum(dim3((C + 255) / 256), dim3(256), s, tb2, B, C, G(gn + ".bias"), 1);
  }

  // ------------------------------------------------------------ tape
  struct RB {   // ResnetBlock
    std::string k; int l, C0, C1, C; const float* x0; const float* x1;
    float *h1, *st1, *u, *h2, *st2, *out; const float* tb; int r;
  };
  struct AT {   // Residual(Rezero(LinearAttention))
    std::string k; int l, C; const float* x; float *qkv, *ctx, *o, *z, *y;
  };
  std::vector<RB> rbs;
  std::vector<AT> ats;
  float *temb_s, *temb_pre0, *temb_h, *temb, *temb_m;   // posemb, mlp.0 pre, Mish, mlp.2 out, Mish(t_emb)
  std::vector<float*> tbs;                              // per ResnetBlock: mlp(t_emb) [B][C]
  float *spk_pre, *spk_h, *spk_s;                       // spk_mlp
  float* xin;                                           // [B][80][T][cin]
  float *hf, *stf, *af, *score;

  static constexpr const char* kRes[12] = {"downs.0.0.", "downs.0.1.", "downs.1.0.", "downs.1.1.", "downs.2.0.",
                                            "downs.2.1.", "mid_block1.", "mid_block2.", "ups.0.0.", "ups.0.1.",
                                            "ups.1.0.", "ups.1.1."};

  // ResnetBlock forward (diffusion.py:61-79 / oracle resnet_block)
  float* resnet_fwd(const std::string& k, int r, int l, const float* x0, int C0, const float* x1, int C1, int C) {
    cur = k + " fwd";
    RB b{k, l, C0, C1, C, x0, x1};
    const int Ci = C0 + C1;
    const long n = (long)B * L(l).F * L(l).T * C;
    b.h1 = A.take(n);
    const float* w1 = P(k + "block1.block.0.weight");
    gconv(x0, C0, l, true, w1, (long)Ci * 9, 9, 3, 1, 1, 0, P(k + "block1.block.0.bias"), b.h1, C, l, false, C, 0, 0);
    if (C1 > 0) gconv(x1, C1, l, true, w1 + C0 * 9, (long)Ci * 9, 9, 3, 1, 1, 0, nullptr, b.h1, C, l, false, C, 0, 1);
    b.st1 = gn_stats(b.h1, l, C);
    b.tb = tbs[r]; b.r = r;
    b.u = block_fwd(l, C, b.h1, b.st1, k + "block1.block.1", b.tb);   // Mish(GN(h1)) m + tb
    b.h2 = A.take(n);
    gconv(b.u, C, l, true, P(k + "block2.block.0.weight"), (long)C * 9, 9, 3, 1, 1, 0, P(k + "block2.block.0.bias"),
          b.h2, C, l, false, C, 0, 0);
    b.st2 = gn_stats(b.h2, l, C);
    b.out = block_fwd(l, C, b.h2, b.st2, k + "block2.block.1", nullptr);
    if (gt_internal_has_param(d, k + "res_conv.weight")) {
      const float* wr = P(k + "res_conv.weight");
      gconv(x0, C0, l, true, wr, Ci, 1, 1, 1, 0, 0, P(k + "res_conv.bias"), b.out, C, l, false, C, 0, 1);
      if (C1 > 0) gconv(x1, C1, l, true, wr + C0, Ci, 1, 1, 1, 0, 0, nullptr, b.out, C, l, false, C, 0, 1);
    } else {
      ew(x0, C, 0, 1.f, nullptr, 0.f, l, C, true, b.out, C, 0, 1);
    }
    rbs.push_back(b);
    return b.out;
  }

  // LinearAttention forward (diffusion.py:82-110 / oracle linear_attention)
  float* attn_fwd(const std::string& k, int l, const float* x, int C) {
    cur = k + " fwd";
    AT a{k, l, C, x};
    const long np = (long)L(l).F * L(l).T;
    a.qkv = A.take((size_t)B * np * 384);
    gconv(x, C, l, false, P(k + "fn.fn.to_qkv.weight"), C, 1, 1, 1, 0, 0, nullptr, a.qkv, 384, l, false, 384, 0, 0);
    float* st = A.take((size_t)B * 256);
    a.ctx = A.take((size_t)B * 4096);
    a.o = A.take((size_t)B * np * 128);
    a.z = A.take((size_t)B * np * C);
    a.y = A.take((size_t)B * np * C);
    float* opart = A.take((size_t)pos_splits(np) * B * 4096);
    if (live()) {
      chk(launch_attn_kstats(dim3(B, 128), dim3(256), s, a.qkv, (int)np, st));
      chk(launch_attn_ksoftmax(g1((long)B * np * 128), dim3(256), s, a.qkv, B, (int)np, st));
      chk(launch_attn_outer_split(a.qkv, 384, 128, a.qkv, 384, 256, B, (int)np, opart, a.ctx, s));
      chk(launch_attn_headmm_mfma(a.ctx, 0, a.qkv, 384, 0, B, (int)np, a.o, 128, 0, 0, s));
    }
    gconv(a.o, 128, l, false, P(k + "fn.fn.to_out.weight"), 128, 1, 1, 1, 0, 0, P(k + "fn.fn.to_out.bias"), a.z, C, l,
          false, C, 0, 0);
    ew_alpha2p = P(k + "fn.g");   // Rezero g read on the device (the block may have been updated there)
    ew(x, C, 0, 1.f, a.z, 0.f, l, C, false, a.y, C, 0, 0);
    ew_alpha2p = nullptr;
    ats.push_back(a);
    return a.y;
  }

  // ------------------------------------------------------------ forward (oracle estimator order)
  float* wpart = nullptr;   // weight-gradient partials, one buffer reused by every wgrad (stream-ordered)
  void forward(const float* mu, const float* xt, const float* spk, const float* t) {
    wpart = A.take((size_t)kWPartCap);
    // time embedding (diffusion.py:113-125, 143-144, 177-178) and every ResnetBlock's mlp (64-65, 76)
    temb_s = A.take((size_t)B * 64); temb_pre0 = A.take((size_t)B * 256); temb_h = A.take((size_t)B * 256);
    temb = A.take((size_t)B * 64); temb_m = A.take((size_t)B * 64);
    if (live()) {
      chk(launch_posemb(dim3(B), dim3(64), s, t, pe_scale, gt_internal_freqs(d), temb_s));
      chk(launch_linear_fwd(dim3(B), dim3(256), s, temb_s, 64, P("mlp.0.weight"), P("mlp.0.bias"), 256, 0, temb_pre0));
      chk(launch_linear_fwd(dim3(B), dim3(256), s, temb_s, 64, P("mlp.0.weight"), P("mlp.0.bias"), 256, 1, temb_h));
      chk(launch_linear_fwd(dim3(B), dim3(64), s, temb_h, 256, P("mlp.2.weight"), P("mlp.2.bias"), 64, 0, temb));
      chk(launch_linear_fwd(dim3(B), dim3(64), s, temb_h, 256, P("mlp.2.weight"), P("mlp.2.bias"), 64, 1, temb_m));
    }
    const int Cs[12] = {64, 64, 128, 128, 256, 256, 256, 256, 128, 128, 64, 64};
    for (int r = 0; r < 12; ++r) {
      float* tb = A.take((size_t)B * Cs[r]);
      if (live()) chk(launch_linear_fwd(dim3(B), dim3(256), s, temb_m, 64, P(std::string(kRes[r]) + "mlp.1.weight"),
                                     P(std::string(kRes[r]) + "mlp.1.bias"), Cs[r], 0, tb));
      tbs.push_back(tb);
      dtb.push_back(A.take((size_t)B * Cs[r]));
    }
    // speaker conditioning (diffusion.py:139-141, 175-176) -> third input channel
    spk_pre = spk_h = spk_s = nullptr;
    if (n_spks > 1) {
      spk_pre = A.take((size_t)B * 256); spk_h = A.take((size_t)B * 256); spk_s = A.take((size_t)B * 80);
      if (live()) {
        chk(launch_linear_fwd(dim3(B), dim3(256), s, spk, 64, P("spk_mlp.0.weight"), P("spk_mlp.0.bias"), 256, 0, spk_pre));
        chk(launch_linear_fwd(dim3(B), dim3(256), s, spk, 64, P("spk_mlp.0.weight"), P("spk_mlp.0.bias"), 256, 1, spk_h));
        chk(launch_linear_fwd(dim3(B), dim3(128), s, spk_h, 256, P("spk_mlp.2.weight"), P("spk_mlp.2.bias"), 80, 0, spk_s));
      }
    }
    xin = A.take((size_t)B * 80 * T * cin);
    if (live()) chk(launch_input_pack(g1((long)B * 80 * T), dim3(256), s, mu, xt, spk_s, B, T, cin, xin));
    // down path
    float* h = resnet_fwd("downs.0.0.", 0, 0, xin, cin, nullptr, 0, 64);
    h = resnet_fwd("downs.0.1.", 1, 0, h, 64, nullptr, 0, 64);
    h = attn_fwd("downs.0.2.", 0, h, 64);
    float* d0 = A.take((size_t)B * L(1).F * L(1).T * 64);
    gconv(h, 64, 0, true, P("downs.0.3.conv.weight"), 64 * 9, 9, 3, 2, 1, 0, P("downs.0.3.conv.bias"), d0, 64, 1,
          false, 64, 0, 0);
    h = resnet_fwd("downs.1.0.", 2, 1, d0, 64, nullptr, 0, 128);
    h = resnet_fwd("downs.1.1.", 3, 1, h, 128, nullptr, 0, 128);
    float* hid1 = attn_fwd("downs.1.2.", 1, h, 128);
    float* d1 = A.take((size_t)B * L(2).F * L(2).T * 128);
    gconv(hid1, 128, 1, true, P("downs.1.3.conv.weight"), 128 * 9, 9, 3, 2, 1, 0, P("downs.1.3.conv.bias"), d1, 128, 2,
          false, 128, 0, 0);
    h = resnet_fwd("downs.2.0.", 4, 2, d1, 128, nullptr, 0, 256);
    h = resnet_fwd("downs.2.1.", 5, 2, h, 256, nullptr, 0, 256);
    float* hid2 = attn_fwd("downs.2.2.", 2, h, 256);
    // mid (input: Identity(hidden2 * mask), the mask applied by mid_block1's own input masking)
    h = resnet_fwd("mid_block1.", 6, 2, hid2, 256, nullptr, 0, 256);
    h = attn_fwd("mid_attn.", 2, h, 256);
    h = resnet_fwd("mid_block2.", 7, 2, h, 256, nullptr, 0, 256);
    // up path
    h = resnet_fwd("ups.0.0.", 8, 2, h, 256, hid2, 256, 128);
    h = resnet_fwd("ups.0.1.", 9, 2, h, 128, nullptr, 0, 128);
    h = attn_fwd("ups.0.2.", 2, h, 128);
    float* u0 = A.take((size_t)B * L(1).F * L(1).T * 128);
    gconv(h, 128, 2, true, P("ups.0.3.conv.weight"), 16, 128 * 16, 4, 2, 1, 0, P("ups.0.3.conv.bias"), u0, 128, 1,
          false, 128, 0, 0, true);
    h = resnet_fwd("ups.1.0.", 10, 1, u0, 128, hid1, 128, 64);
    h = resnet_fwd("ups.1.1.", 11, 1, h, 64, nullptr, 0, 64);
    h = attn_fwd("ups.1.2.", 1, h, 64);
    float* u1 = A.take((size_t)B * 80 * T * 64);
    gconv(h, 64, 1, true, P("ups.1.3.conv.weight"), 16, 64 * 16, 4, 2, 1, 0, P("ups.1.3.conv.bias"), u1, 64, 0, false,
          64, 0, 0, true);
    up1 = u1;
    // final block + final conv (diffusion.py:212-216)
    hf = A.take((size_t)B * 80 * T * 64);
    gconv(u1, 64, 0, true, P("final_block.block.0.weight"), 64 * 9, 9, 3, 1, 1, 0, P("final_block.block.0.bias"), hf,
          64, 0, false, 64, 0, 0);
    stf = gn_stats(hf, 0, 64);
    af = block_fwd(0, 64, hf, stf, "final_block.block.1", nullptr);
    score = A.take((size_t)B * 80 * T);
    gconv(af, 64, 0, true, P("final_conv.weight"), 64, 1, 1, 1, 0, 0, P("final_conv.bias"), score, 1, 0, true, 1, 0, 0);
    down0 = d0; down1 = d1; hidden1 = hid1; hidden2 = hid2; up0 = u0;
  }
  float *down0, *down1, *hidden1, *hidden2, *up0, *up1;

  // ------------------------------------------------------------ backward
  // ResnetBlock backward; dx0 / dx1 receive (accumulate) the input gradients
  void resnet_bwd(const RB& b, const float* dout, float* dx0, float* dx1) {
    const std::string& k = b.k;
    cur = k + " bwd";
    const int l = b.l, C = b.C, Ci = b.C0 + b.C1;
    // residual branch
    if (gt_internal_has_param(d, k + "res_conv.weight")) {
      const float* wr = P(k + "res_conv.weight");
      float* gw = G(k + "res_conv.weight");
      wgrad(dout, C, l, false, b.x0, b.C0, l, true, 1, 1, 0, gw, Ci, 1, 1);
      if (b.C1 > 0) wgrad(dout, C, l, false, b.x1, b.C1, l, true, 1, 1, 0, gw + b.C0, Ci, 1, 1);
      chansum(dout, l, C, G(k + "res_conv.bias"), 1);
      gconv(dout, C, l, false, wr, 1, Ci, 1, 1, 0, 0, nullptr, dx0, b.C0, l, true, b.C0, 0, 1);
      if (b.C1 > 0) gconv(dout, C, l, false, wr + b.C0, 1, Ci, 1, 1, 0, 0, nullptr, dx1, b.C1, l, true, b.C1, 0, 1);
    } else {
      ew(dout, C, 0, 1.f, nullptr, 0.f, l, C, true, dx0, C, 0, 1);
    }
    // block2
    float* dh2 = block_bwd(l, C, dout, b.h2, b.st2, k + "block2.block.1");
    wgrad(dh2, C, l, false, b.u, C, l, true, 3, 1, 1, G(k + "block2.block.0.weight"), (long)C * 9, 9, 1);
    chansum(dh2, l, C, G(k + "block2.block.0.bias"), 1);
    float* du = A.take((size_t)B * L(l).F * L(l).T * C);
    gconv(dh2, C, l, false, P(k + "block2.block.0.weight"), 9, (long)C * 9, 3, 1, 1, 1, nullptr, du, C, l, true, C, 0, 0);
    {
      const int npos = L(l).F * L(l).T;
      float* part = A.take((size_t)B * pos_splits(npos) * C);
      if (live() && pgrads) chk(launch_chan_sums(du, nullptr, B, npos, C, part, dtb[b.r], 1, 0, s));
    }
    // block1
    float* dh1 = block_bwd(l, C, du, b.h1, b.st1, k + "block1.block.1");
    const float* w1 = P(k + "block1.block.0.weight");
    float* gw1 = G(k + "block1.block.0.weight");
    wgrad(dh1, C, l, false, b.x0, b.C0, l, true, 3, 1, 1, gw1, (long)Ci * 9, 9, 1);
    if (b.C1 > 0) wgrad(dh1, C, l, false, b.x1, b.C1, l, true, 3, 1, 1, gw1 + b.C0 * 9, (long)Ci * 9, 9, 1);
    chansum(dh1, l, C, G(k + "block1.block.0.bias"), 1);
    gconv(dh1, C, l, false, w1, 9, (long)Ci * 9, 3, 1, 1, 1, nullptr, dx0, b.C0, l, true, b.C0, 0, 1);
    if (b.C1 > 0) gconv(dh1, C, l, false, w1 + b.C0 * 9, 9, (long)Ci * 9, 3, 1, 1, 1, nullptr, dx1, b.C1, l, true, b.C1, 0, 1);
  }

  // LinearAttention backward; dx (accumulate) receives the input gradient
  void attn_bwd(const AT& a, const float* dy, float* dx) {
    const std::string& k = a.k;
    cur = k + " bwd";
    const int l = a.l, C = a.C;
    const long np = (long)L(l).F * L(l).T, n = (long)B * np;
    ew(dy, C, 0, 1.f, nullptr, 0.f, l, C, false, dx, C, 0, 1);                 // residual
    double* dpart = reinterpret_cast<double*>(A.take(2 * kDotBlocks));
    if (live() && pgrads) chk(launch_dot_sum(dy, a.z, n * C, dpart, G(k + "fn.g"), 1, s));   // d g = sum dy . z
    float* dz = A.take((size_t)n * C);
    ew_alphap = P(k + "fn.g");
    ew(dy, C, 0, 0.f, nullptr, 0.f, l, C, false, dz, C, 0, 0);
    ew_alphap = nullptr;
    wgrad(dz, C, l, false, a.o, 128, l, false, 1, 1, 0, G(k + "fn.fn.to_out.weight"), 128, 1, 1);
    chansum(dz, l, C, G(k + "fn.fn.to_out.bias"), 1);
    float* dO = A.take((size_t)n * 128);
    gconv(dz, C, l, false, P(k + "fn.fn.to_out.weight"), 1, 128, 1, 1, 0, 0, nullptr, dO, 128, l, false, 128, 0, 0);
    float* dctx = A.take((size_t)B * 4096);
    float* dqkv = A.take((size_t)n * 384);
    float* S = A.take((size_t)B * 128);
    float* opart = A.take((size_t)pos_splits(np) * B * 4096);
    float* rpart = A.take((size_t)B * pos_splits(np) * 128);
    if (live()) {
      chk(launch_attn_outer_split(a.qkv, 384, 0, dO, 128, 0, B, (int)np, opart, dctx, s));      // q do^T
      chk(launch_attn_headmm_mfma(a.ctx, 1, dO, 128, 0, B, (int)np, dqkv, 384, 0, 0, s));     // dq
      chk(launch_attn_headmm_mfma(dctx, 1, a.qkv, 384, 256, B, (int)np, dqkv, 384, 128, 0, s));  // dks
      chk(launch_attn_headmm_mfma(dctx, 0, a.qkv, 384, 128, B, (int)np, dqkv, 384, 256, 0, s));  // dv
      chk(launch_attn_rowdot_split(a.qkv, 384, 128, dqkv, 384, 128, B, (int)np, rpart, S, s));
      chk(launch_attn_ksoftmax_bwd(g1(n * 128), dim3(256), s, a.qkv, dqkv, B, (int)np, S));
    }
    wgrad(dqkv, 384, l, false, a.x, C, l, false, 1, 1, 0, G(k + "fn.fn.to_qkv.weight"), C, 1, 1);
    gconv(dqkv, 384, l, false, P(k + "fn.fn.to_qkv.weight"), 1, C, 1, 1, 0, 0, nullptr, dx, C, l, false, C, 0, 1);
  }

  void backward(const float* z, const float* t, const float* xt_e, float* dmu, float* dspk) {
    const long n0 = (long)B * 80 * T;
    // dL/dscore (diffusion.py:278-280)
    float* ds = A.take(n0);
    if (live()) chk(launch_loss_bwd(g1(n0), dim3(256), s, score, z, mask, t, lossp, B, T, bmin, half_delta, ds));
    (void)xt_e;
    backward_core(ds, t, dmu, dspk);
  }
  float* dxin = nullptr;   // d / d(U-Net input channels (mu, x_t[, s])), [B][80][T][cin]
  // backward from ds = d/d(pre-mask estimator output) (the output mask already applied)
  void backward_core(const float* ds, const float* t, float* dmu, float* dspk) {
    const long n0 = (long)B * 80 * T;
    // final conv (1x1, 64 -> 1) on af * m, output * m
    wgrad(ds, 1, 0, false, af, 64, 0, true, 1, 1, 0, G("final_conv.weight"), 64, 1, 1);
    chansum(ds, 0, 1, G("final_conv.bias"), 1);
    float* daf = A.take(n0 * 64);
    gconv(ds, 1, 0, false, P("final_conv.weight"), 1, 64, 1, 1, 0, 0, nullptr, daf, 64, 0, true, 64, 0, 0);
    float* dhf = block_bwd(0, 64, daf, hf, stf, "final_block.block.1");
    wgrad(dhf, 64, 0, false, up1, 64, 0, true, 3, 1, 1, G("final_block.block.0.weight"), 64 * 9, 9, 1);
    chansum(dhf, 0, 64, G("final_block.block.0.bias"), 1);
    float* dup1 = A.take(n0 * 64);
    gconv(dhf, 64, 0, false, P("final_block.block.0.weight"), 9, 64 * 9, 3, 1, 1, 1, nullptr, dup1, 64, 0, true, 64, 0, 0);
    // ups.1.3: ConvTranspose 64 -> 64, level 1 -> 0, on x * m1
    const AT& a_u1 = ats[5];
    wgrad(a_u1.y, 64, 1, true, dup1, 64, 0, false, 4, 2, 1, G("ups.1.3.conv.weight"), 64 * 16, 16, 1);
    chansum(dup1, 0, 64, G("ups.1.3.conv.bias"), 1);
    const long n1 = (long)B * L(1).F * L(1).T, n2 = (long)B * L(2).F * L(2).T;
    float* dy_u1 = A.take(n1 * 64);
    gconv(dup1, 64, 0, false, P("ups.1.3.conv.weight"), 64 * 16, 16, 4, 2, 1, 0, nullptr, dy_u1, 64, 1, true, 64, 0, 0);
    float* dx = A.take(n1 * 64);
    zero(dx, n1 * 64);
    attn_bwd(a_u1, dy_u1, dx);                                           // ups.1.2
    float* dx2 = A.take(n1 * 64);
    zero(dx2, n1 * 64);
    resnet_bwd(rbs[11], dx, dx2, nullptr);                               // ups.1.1
    float* dup0 = A.take(n1 * 128);
    float* dhid1 = A.take(n1 * 128);
    zero(dup0, n1 * 128); zero(dhid1, n1 * 128);
    resnet_bwd(rbs[10], dx2, dup0, dhid1);                               // ups.1.0 (concat up0 | hidden1)
    // ups.0.3: ConvTranspose 128 -> 128, level 2 -> 1
    const AT& a_u0 = ats[4];
    wgrad(a_u0.y, 128, 2, true, dup0, 128, 1, false, 4, 2, 1, G("ups.0.3.conv.weight"), 128 * 16, 16, 1);
    chansum(dup0, 1, 128, G("ups.0.3.conv.bias"), 1);
    float* dy_u0 = A.take(n2 * 128);
    gconv(dup0, 128, 1, false, P("ups.0.3.conv.weight"), 128 * 16, 16, 4, 2, 1, 0, nullptr, dy_u0, 128, 2, true, 128, 0, 0);
    float* dx3 = A.take(n2 * 128);
    zero(dx3, n2 * 128);
    attn_bwd(a_u0, dy_u0, dx3);                                          // ups.0.2
    float* dx4 = A.take(n2 * 128);
    zero(dx4, n2 * 128);
    resnet_bwd(rbs[9], dx3, dx4, nullptr);                               // ups.0.1
    float* dmid = A.take(n2 * 256);
    float* dhid2 = A.take(n2 * 256);
    zero(dmid, n2 * 256); zero(dhid2, n2 * 256);
    resnet_bwd(rbs[8], dx4, dmid, dhid2);                                // ups.0.0 (concat mid | hidden2)
    float* dx5 = A.take(n2 * 256);
    zero(dx5, n2 * 256);
    resnet_bwd(rbs[7], dmid, dx5, nullptr);                              // mid_block2
    float* dx6 = A.take(n2 * 256);
    zero(dx6, n2 * 256);
    attn_bwd(ats[3], dx5, dx6);                                          // mid_attn
    resnet_bwd(rbs[6], dx6, dhid2, nullptr);                             // mid_block1 (input hidden2, masked in it)
    float* dx7 = A.take(n2 * 256);
    zero(dx7, n2 * 256);
    attn_bwd(ats[2], dhid2, dx7);                                        // downs.2.2
    float* dx8 = A.take(n2 * 256);
    zero(dx8, n2 * 256);
    resnet_bwd(rbs[5], dx7, dx8, nullptr);                               // downs.2.1
    float* dd1 = A.take(n2 * 128);
    zero(dd1, n2 * 128);
    resnet_bwd(rbs[4], dx8, dd1, nullptr);                               // downs.2.0
    // downs.1.3: conv 3x3 stride 2 on hidden1 * m1 (level 1 -> 2)
    wgrad(dd1, 128, 2, false, hidden1, 128, 1, true, 3, 2, 1, G("downs.1.3.conv.weight"), 128 * 9, 9, 1);
    chansum(dd1, 2, 128, G("downs.1.3.conv.bias"), 1);
    gconv(dd1, 128, 2, false, P("downs.1.3.conv.weight"), 9, 128 * 9, 3, 2, 1, 0, nullptr, dhid1, 128, 1, true, 128, 0,
          1, true);
    float* dx9 = A.take(n1 * 128);
    zero(dx9, n1 * 128);
    attn_bwd(ats[1], dhid1, dx9);                                        // downs.1.2
    float* dx10 = A.take(n1 * 128);
    zero(dx10, n1 * 128);
    resnet_bwd(rbs[3], dx9, dx10, nullptr);                              // downs.1.1
    float* dd0 = A.take(n1 * 64);
    zero(dd0, n1 * 64);
    resnet_bwd(rbs[2], dx10, dd0, nullptr);                              // downs.1.0
    // downs.0.3: conv 3x3 stride 2 on y0 * m0 (level 0 -> 1)
    const AT& a_d0 = ats[0];
    wgrad(dd0, 64, 1, false, a_d0.y, 64, 0, true, 3, 2, 1, G("downs.0.3.conv.weight"), 64 * 9, 9, 1);
    chansum(dd0, 1, 64, G("downs.0.3.conv.bias"), 1);
    float* dy0 = A.take(n0 * 64);
    gconv(dd0, 64, 1, false, P("downs.0.3.conv.weight"), 9, 64 * 9, 3, 2, 1, 0, nullptr, dy0, 64, 0, true, 64, 0, 0, true);
    float* dx11 = A.take(n0 * 64);
    zero(dx11, n0 * 64);
    attn_bwd(a_d0, dy0, dx11);                                           // downs.0.2
    float* dx12 = A.take(n0 * 64);
    zero(dx12, n0 * 64);
    resnet_bwd(rbs[1], dx11, dx12, nullptr);                             // downs.0.1
    dxin = A.take(n0 * cin);
    zero(dxin, n0 * cin);
    resnet_bwd(rbs[0], dx12, dxin, nullptr);                             // downs.0.0 (input channels mu, x_t[, s])
    // time MLPs: dtb_r -> mlp.1 of every block, d Mish(t_emb) -> mlp.2 -> Mish -> mlp.0
    const int Cs[12] = {64, 64, 128, 128, 256, 256, 256, 256, 128, 128, 64, 64};
    float* dtm = A.take((size_t)B * 64);
    float* dte = A.take((size_t)B * 64);
    float* dh0 = A.take((size_t)B * 256);
    if (live() && pgrads) {
      for (int r = 0; r < 12; ++r) {
        const std::string kr = std::string(kRes[r]) + "mlp.1.";
        chk(launch_linear_wgrad(dim3(Cs[r]), dim3(64), s, dtb[r], temb_m, B, 64, Cs[r], G(kr + "weight"), G(kr + "bias")));
        chk(launch_linear_dgrad(dim3(B), dim3(64), s, dtb[r], P(kr + "weight"), 64, Cs[r], nullptr, dtm, r > 0));
      }
      chk(launch_mish_bwd(dim3(B), dim3(64), s, dtm, temb, 64, dte));
      chk(launch_linear_wgrad(dim3(64), dim3(256), s, dte, temb_h, B, 256, 64, G("mlp.2.weight"), G("mlp.2.bias")));
      chk(launch_linear_dgrad(dim3(B), dim3(256), s, dte, P("mlp.2.weight"), 256, 64, temb_pre0, dh0, 0));
      chk(launch_linear_wgrad(dim3(256), dim3(64), s, dh0, temb_s, B, 64, 256, G("mlp.0.weight"), G("mlp.0.bias")));
    }
    // inputs: dmu = dxin[..0] + dxin[..1] (1 - e) m (x_t = x0 e + mu (1 - e) + ..., masked); speaker channel
    if (live() && dmu) chk(launch_dmu(g1(n0), dim3(256), s, dxin, cin, t, mask, B, T, bmin, half_delta, dmu));
    if (n_spks > 1) {
      float* dsv = A.take((size_t)B * 80);
      float* dsh = A.take((size_t)B * 256);
      if (live() && pgrads) {
        chk(launch_spk_chan_sum(dim3(B), dim3(128), s, dxin, cin, T, dsv));
        chk(launch_linear_wgrad(dim3(80), dim3(256), s, dsv, spk_h, B, 256, 80, G("spk_mlp.2.weight"), G("spk_mlp.2.bias")));
        chk(launch_linear_dgrad(dim3(B), dim3(256), s, dsv, P("spk_mlp.2.weight"), 256, 80, spk_pre, dsh, 0));
        chk(launch_linear_wgrad(dim3(256), dim3(64), s, dsh, spkin, B, 64, 256, G("spk_mlp.0.weight"), G("spk_mlp.0.bias")));
        if (dspk) chk(launch_linear_dgrad(dim3(B), dim3(64), s, dsh, P("spk_mlp.0.weight"), 64, 256, nullptr, dspk, 0));
      }
    }
  }
  std::string cur;                // the ResnetBlock / attention being processed (error messages)
  const float* lossp = nullptr;   // device [2]: loss, sum(mask)
  const float* spkin = nullptr;
  void zero(float* p, long n, int line = __builtin_LINE()) {
    if (run) need(p, n, "zero", line);
    if (live()) chk(launch_fill_f32(p, n, 0.f, s), line);
  }
};

}  // namespace

extern "C" {

size_t gt_train_workspace_bytes(gt_decoder* d, int64_t B, int64_t T) {
  if (!d || B <= 0 || T <= 0 || gt_internal_layout(d) != GT_OK) return 0;
  Trainer tr;
  tr.d = d; tr.B = (int)B; tr.T = (int)T; tr.run = false; tr.s = nullptr;
  float bmax;
  gt_internal_consts(d, &tr.n_spks, &tr.bmin, &bmax, &tr.pe_scale);
  tr.cin = tr.n_spks > 1 ? 3 : 2;
  tr.A.take((size_t)B * 80 * T);       // zm, loss partials, loss (as train_pass takes them)
  tr.A.take((size_t)B * 80 * T * 2);
  tr.A.take(2);
  tr.forward(nullptr, nullptr, nullptr, nullptr);
  tr.backward(nullptr, nullptr, nullptr, nullptr, nullptr);
  return tr.A.off + 4096;
}

}  // extern "C"

// One pass of the training step. dry: no launches; every helper checks on the host that the extents its kernels will
// touch lie inside one buffer (arena allocation, caller buffer, parameter block) -- run before every live pass, so a
// host-side indexing error fails loudly instead of faulting the GPU.
static int train_pass(gt_decoder* d, const float* x0, const float* mask, const float* mu, const float* t,
                      const float* z, const float* spk, int64_t B, int64_t T, float* loss, float* xt, float* grads,
                      float* dmu, float* dspk, void* workspace, size_t workspace_bytes, hipStream_t stream, bool dry,
                      bool debug, std::vector<GconvPack>* packs) {
  Trainer tr;
  tr.d = d; tr.B = (int)B; tr.T = (int)T; tr.run = true; tr.s = stream;
  float bmax;
  gt_internal_consts(d, &tr.n_spks, &tr.bmin, &bmax, &tr.pe_scale);
  tr.half_delta = (float)(0.5 * ((double)bmax - (double)tr.bmin));
  tr.cin = tr.n_spks > 1 ? 3 : 2;
  tr.mask = mask; tr.grads = grads; tr.spkin = spk;
  tr.debug = debug;
  tr.dry = dry;
  if (dry) {
    const size_t n0b = (size_t)B * 80 * T * 4;
    tr.regions = {{(uintptr_t)x0, n0b}, {(uintptr_t)mu, n0b}, {(uintptr_t)z, n0b}, {(uintptr_t)xt, n0b},
                  {(uintptr_t)mask, (size_t)B * T * 4}, {(uintptr_t)t, (size_t)B * 4},
                  {(uintptr_t)grads, (size_t)gt_internal_numel(d) * 4},
                  {(uintptr_t)gt_internal_param(d, "mlp.0.weight") - (uintptr_t)gt_internal_param_offset(d, "mlp.0.weight") * 4,
                   (size_t)(gt_internal_numel(d) + 32) * 4}};
    if (dmu) tr.regions.push_back({(uintptr_t)dmu, n0b});
    if (spk) tr.regions.push_back({(uintptr_t)spk, (size_t)B * 64 * 4});
    if (dspk) tr.regions.push_back({(uintptr_t)dspk, (size_t)B * 64 * 4});
    tr.A.rec = &tr.regions;
  }
  tr.A.base = (uint8_t*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  if (dry) {
    tr.packs = packs;
  } else if (packs && !packs->empty()) {
    tr.chk(launch_gconv_wpack_batch(packs->data(), (int)packs->size(), tr.s));
    tr.packed_ahead = true;
  }
  const long n0 = (long)B * 80 * T;
  float* zm = tr.A.take((size_t)n0);
  float* lpart = tr.A.take((size_t)n0 * 2);   // loss partials (generous)
  float* lossv = tr.A.take(2);
  if (!dry) tr.chk(launch_fill_f32(grads, gt_internal_numel(d), 0.f, tr.s));
  // forward diffusion (diffusion.py:275), then the taped U-Net forward on x_t
  FwdDiffParams fp;
  fp.x0 = x0; fp.mu = mu; fp.z = z; fp.mask = mask; fp.t = t; fp.B = (int)B; fp.F = 80; fp.T = (int)T;
  fp.beta_min = tr.bmin; fp.half_delta = tr.half_delta; fp.xt = xt; fp.zm = zm;
  if (!dry) tr.chk(launch_fwd_diffusion(fp, tr.s));
  tr.forward(mu, xt, spk, t);
  // loss value and sum(mask) (for the gradient's normaliser)
  LossParams lp;
  lp.score = tr.score; lp.z = z; lp.mask = mask; lp.t = t; lp.B = (int)B; lp.F = 80; lp.T = (int)T;
  lp.beta_min = tr.bmin; lp.half_delta = tr.half_delta; lp.part = lpart;
  if (!dry) {
    tr.chk(launch_loss(lp, lossv, tr.s));
    tr.chk(launch_mask_sum(dim3(1), dim3(256), tr.s, mask, n0 / 80, lossv + 1));
  }
  tr.lossp = lossv;
  tr.backward(z, t, xt, dmu, dspk);
  if (dry) {
    if (!tr.bad.empty()) return gt_internal_fail(GT_ERR_WORKSPACE, "training step extent check: " + tr.bad);
    if (tr.A.off + 255 > workspace_bytes)
      return gt_internal_fail(GT_ERR_WORKSPACE, "training step extent check: arena " + std::to_string(tr.A.off) +
                                                   " B past the workspace " + std::to_string(workspace_bytes) + " B");
    return GT_OK;
  }
  tr.chk(launch_copy_f32(loss, lossv, 1, tr.s));
  if (tr.err != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, std::string("HIP launch failed: ") + hipGetErrorString(tr.err) +
                                            " (train_bwd.cpp:" + std::to_string(tr.err_line) + ", block " + tr.err_cur + ")");
  return GT_OK;
}

extern "C" {

int gt_diffusion_loss_grad(gt_decoder* d, const float* x0, const float* mask, const float* mu, const float* t,
                           const float* z, const float* spk, int64_t B, int64_t T, float* loss, float* xt, float* grads,
                           float* dmu, float* dspk, void* workspace, size_t workspace_bytes, void* stream) {
  if (!d || !x0 || !mask || !mu || !t || !z || !loss || !xt || !grads || !workspace)
    return gt_internal_fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || T <= 0 || T % 4 != 0) return gt_internal_fail(GT_ERR_ARG, "bad B / T");
  // GT_TRAIN_DEBUG=1: synchronise after every launch and name the failing call site; =2: the host extent check
  // only (nothing touches the device: runs without a GPU, tests/test_train_cpu.py)
  const char* dbg = getenv("GT_TRAIN_DEBUG");
  const bool dry_only = dbg && dbg[0] == '2';
  int rc = dry_only ? gt_internal_layout(d) : gt_internal_prepare_raw(d);
  if (rc) return rc;
  if (workspace_bytes < gt_train_workspace_bytes(d, B, T)) return gt_internal_fail(GT_ERR_WORKSPACE, "workspace too small");
  int n_spks; float bmin, bmax, pe;
  gt_internal_consts(d, &n_spks, &bmin, &bmax, &pe);
  if (n_spks > 1 && !spk) return gt_internal_fail(GT_ERR_ARG, "n_spks > 1 needs spk");
  std::vector<GconvPack> packs;
  rc = train_pass(d, x0, mask, mu, t, z, spk, B, T, loss, xt, grads, dmu, dspk, workspace, workspace_bytes,
                  (hipStream_t)stream, true, false, &packs);
  if (rc || dry_only) return rc;
  return train_pass(d, x0, mask, mu, t, z, spk, B, T, loss, xt, grads, dmu, dspk, workspace, workspace_bytes,
                    (hipStream_t)stream, false, dbg && dbg[0] == '1', &packs);
}

int64_t gt_decoder_grad_numel(gt_decoder* d) {
  if (!d || gt_internal_layout(d) != GT_OK) return -1;
  return gt_internal_numel(d);
}

}  // extern "C"

// ---------------------------------------------------------------- estimator VJP and likelihood (§8 f3)
static size_t al256(size_t n) { return (n + 255) & ~size_t(255); }

// score = estimator(x, mask, mu, t, spk); vjp = (d score / d x)^T v. The training tape and backward without the
// parameter-gradient work (Trainer::pgrads = false), started from the output cotangent v (times the output mask).
static int vjp_pass(gt_decoder* d, const float* x, const float* mask, const float* mu, const float* t, const float* spk,
                    const float* v, int64_t B, int64_t T, float* score, float* vjp, void* workspace,
                    size_t workspace_bytes, hipStream_t stream, bool dry, bool debug) {
  Trainer tr;
  tr.d = d; tr.B = (int)B; tr.T = (int)T; tr.run = true; tr.s = stream;
  float bmax;
  gt_internal_consts(d, &tr.n_spks, &tr.bmin, &bmax, &tr.pe_scale);
  tr.half_delta = (float)(0.5 * ((double)bmax - (double)tr.bmin));
  tr.cin = tr.n_spks > 1 ? 3 : 2;
  tr.mask = mask; tr.grads = nullptr; tr.spkin = spk; tr.pgrads = false;
  tr.debug = debug; tr.dry = dry;
  const long n0 = (long)B * 80 * T;
  if (dry) {
    const size_t n0b = (size_t)n0 * 4;
    tr.regions = {{(uintptr_t)x, n0b}, {(uintptr_t)mu, n0b}, {(uintptr_t)v, n0b}, {(uintptr_t)vjp, n0b},
                  {(uintptr_t)mask, (size_t)B * T * 4}, {(uintptr_t)t, (size_t)B * 4},
                  {(uintptr_t)gt_internal_param(d, "mlp.0.weight") - (uintptr_t)gt_internal_param_offset(d, "mlp.0.weight") * 4,
                   (size_t)(gt_internal_numel(d) + 32) * 4}};
    if (score) tr.regions.push_back({(uintptr_t)score, n0b});
    if (spk) tr.regions.push_back({(uintptr_t)spk, (size_t)B * 64 * 4});
    tr.A.rec = &tr.regions;
  }
  tr.A.base = (uint8_t*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  float* ds = tr.A.take((size_t)n0);   // the same leading takes as train_pass (one workspace size for both)
  tr.A.take((size_t)n0 * 2);
  tr.A.take(2);
  tr.forward(mu, x, spk, t);
  tr.cur = "vjp cotangent";
  tr.ew(v, 1, 0, 1.f, nullptr, 0.f, 0, 1, true, ds, 1, 0, 0);   // d/d(pre-mask output) = v m
  tr.backward_core(ds, t, nullptr, nullptr);
  tr.cur = "vjp input channel";
  tr.ew(tr.dxin, tr.cin, 1, 1.f, nullptr, 0.f, 0, 1, false, vjp, 1, 0, 0);   // channel 1 of the U-Net input = x
  if (dry) {
    if (!tr.bad.empty()) return gt_internal_fail(GT_ERR_WORKSPACE, "estimator VJP extent check: " + tr.bad);
    if (tr.A.off + 255 > workspace_bytes)
      return gt_internal_fail(GT_ERR_WORKSPACE, "estimator VJP extent check: arena past the workspace");
    return GT_OK;
  }
  if (score) tr.chk(launch_copy_f32(score, tr.score, n0, tr.s));
  if (tr.err != hipSuccess)
    return gt_internal_fail(GT_ERR_HIP, std::string("HIP launch failed: ") + hipGetErrorString(tr.err) +
                                            " (train_bwd.cpp:" + std::to_string(tr.err_line) + ", " + tr.err_cur + ")");
  return GT_OK;
}

namespace {
struct LikWs { size_t xm, vv, u, score, part, y, logp, x32, tbuf, drift, div, total; };
LikWs lik_ws(gt_decoder* d, int64_t B, int64_t T) {
  const size_t n0 = (size_t)B * 80 * T;
  LikWs w{};
  size_t off = al256(gt_train_workspace_bytes(d, B, T));
  auto put = [&](size_t bytes) { const size_t o = off; off = al256(off + bytes); return o; };
  w.xm = put(n0 * 4); w.vv = put(n0 * 4); w.u = put(n0 * 4); w.score = put(n0 * 4);
  w.part = put((size_t)B * lik_blocks((int)T) * 4);
  w.y = put(n0 * 8); w.logp = put((size_t)B * 8); w.x32 = put(n0 * 4); w.tbuf = put((size_t)B * 4);
  w.drift = put(n0 * 4); w.div = put((size_t)B * 4);
  w.total = off + 256;
  return w;
}
}  // namespace

// drift and divergence of one probability-flow evaluation; base = 256-aligned workspace laid out by lik_ws
static int drift_div_pass(gt_decoder* d, const float* x, const float* mask, const float* mu, const float* t,
                          const float* spk, const float* eps, int64_t B, int64_t T, float* drift, float* div,
                          uint8_t* base, const LikWs& w, hipStream_t stream, bool dry, bool debug) {
  float* xm = (float*)(base + w.xm);
  float* vv = (float*)(base + w.vv);
  float* u = (float*)(base + w.u);
  float* sc = (float*)(base + w.score);
  if (!dry) {
    const hipError_t e = launch_lik_prep(x, mask, eps, (int)B, (int)T, xm, vv, stream);
    if (e != hipSuccess) return gt_internal_fail(GT_ERR_HIP, std::string("lik_prep: ") + hipGetErrorString(e));
  }
  int rc = vjp_pass(d, xm, mask, mu, t, spk, vv, B, T, sc, u, base, w.xm, stream, dry, debug);
  if (rc || dry) return rc;
  int n_spks; float bmin, bmax, pe;
  gt_internal_consts(d, &n_spks, &bmin, &bmax, &pe);
  LikParams lp;
  lp.xm = xm; lp.mu = mu; lp.mask = mask; lp.eps = eps; lp.score = sc; lp.u = u; lp.t = t;
  lp.B = (int)B; lp.T = (int)T; lp.beta_min = bmin; lp.delta = (float)((double)bmax - (double)bmin);
  lp.drift = drift; lp.part = (float*)(base + w.part);
  const hipError_t e = launch_lik_drift_div(lp, div, stream);
  if (e != hipSuccess) return gt_internal_fail(GT_ERR_HIP, std::string("lik_drift_div: ") + hipGetErrorString(e));
  return GT_OK;
}

extern "C" {

size_t gt_estimator_vjp_workspace_bytes(gt_decoder* d, int64_t B, int64_t T) { return gt_train_workspace_bytes(d, B, T); }

int gt_estimator_vjp(gt_decoder* d, const float* x, const float* mask, const float* mu, const float* t, const float* spk,
                     const float* v, int64_t B, int64_t T, float* score, float* vjp_x, void* workspace,
                     size_t workspace_bytes, void* stream) {
  if (!d || !x || !mask || !mu || !t || !v || !vjp_x || !workspace) return gt_internal_fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || T <= 0 || T % 4 != 0) return gt_internal_fail(GT_ERR_ARG, "bad B / T");
  const char* dbg = getenv("GT_TRAIN_DEBUG");
  const bool dry_only = dbg && dbg[0] == '2';
  int rc = dry_only ? gt_internal_layout(d) : gt_internal_prepare_raw(d);
  if (rc) return rc;
  if (workspace_bytes < gt_train_workspace_bytes(d, B, T)) return gt_internal_fail(GT_ERR_WORKSPACE, "workspace too small");
  int n_spks; float bmin, bmax, pe;
  gt_internal_consts(d, &n_spks, &bmin, &bmax, &pe);
  if (n_spks > 1 && !spk) return gt_internal_fail(GT_ERR_ARG, "n_spks > 1 needs spk");
  rc = vjp_pass(d, x, mask, mu, t, spk, v, B, T, score, vjp_x, workspace, workspace_bytes, (hipStream_t)stream, true, false);
  if (rc || dry_only) return rc;
  return vjp_pass(d, x, mask, mu, t, spk, v, B, T, score, vjp_x, workspace, workspace_bytes, (hipStream_t)stream, false,
                  dbg && dbg[0] == '1');
}

size_t gt_likelihood_workspace_bytes(gt_decoder* d, int64_t B, int64_t T) {
  if (!d || B <= 0 || T <= 0 || gt_internal_layout(d) != GT_OK) return 0;
  return lik_ws(d, B, T).total;
}

static int lik_common(gt_decoder* d, const float* mask, const float* mu, const float* spk, const float* eps, int64_t B,
                      int64_t T, size_t workspace_bytes, bool* dry_only, bool* debug) {
  if (!d || !mask || !mu || !eps) return gt_internal_fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || T <= 0 || T % 4 != 0) return gt_internal_fail(GT_ERR_ARG, "bad B / T");
  const char* dbg = getenv("GT_TRAIN_DEBUG");
  *dry_only = dbg && dbg[0] == '2';
  *debug = dbg && dbg[0] == '1';
  int rc = *dry_only ? gt_internal_layout(d) : gt_internal_prepare_raw(d);
  if (rc) return rc;
  if (workspace_bytes < lik_ws(d, B, T).total) return gt_internal_fail(GT_ERR_WORKSPACE, "workspace too small");
  int n_spks; float bmin, bmax, pe;
  gt_internal_consts(d, &n_spks, &bmin, &bmax, &pe);
  if (n_spks > 1 && !spk) return gt_internal_fail(GT_ERR_ARG, "n_spks > 1 needs spk");
  return GT_OK;
}

int gt_likelihood_drift_div(gt_decoder* d, const float* x, const float* mask, const float* mu, const float* t,
                            const float* spk, const float* eps, int64_t B, int64_t T, float* drift, float* div,
                            void* workspace, size_t workspace_bytes, void* stream) {
  if (!x || !t || !drift || !div || !workspace) return gt_internal_fail(GT_ERR_ARG, "null argument");
  bool dry_only, debug;
  int rc = lik_common(d, mask, mu, spk, eps, B, T, workspace_bytes, &dry_only, &debug);
  if (rc) return rc;
  const LikWs w = lik_ws(d, B, T);
  uint8_t* base = (uint8_t*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  rc = drift_div_pass(d, x, mask, mu, t, spk, eps, B, T, drift, div, base, w, (hipStream_t)stream, true, false);
  if (rc || dry_only) return rc;
  return drift_div_pass(d, x, mask, mu, t, spk, eps, B, T, drift, div, base, w, (hipStream_t)stream, false, debug);
}

int gt_likelihood_euler(gt_decoder* d, const float* data, const float* mask, const float* mu, const float* spk,
                        const float* eps, int64_t B, int64_t T, int32_t n_steps, float* z, float* delta_logp,
                        void* workspace, size_t workspace_bytes, void* stream) {
  if (!data || !z || !delta_logp || !workspace || n_steps <= 0) return gt_internal_fail(GT_ERR_ARG, "null argument");
  bool dry_only, debug;
  int rc = lik_common(d, mask, mu, spk, eps, B, T, workspace_bytes, &dry_only, &debug);
  if (rc) return rc;
  const LikWs w = lik_ws(d, B, T);
  uint8_t* base = (uint8_t*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  double* y = (double*)(base + w.y);
  double* logp = (double*)(base + w.logp);
  float* x32 = (float*)(base + w.x32);
  float* tbuf = (float*)(base + w.tbuf);
  float* drift = (float*)(base + w.drift);
  float* div = (float*)(base + w.div);
  rc = drift_div_pass(d, x32, mask, mu, tbuf, spk, eps, B, T, drift, div, base, w, (hipStream_t)stream, true, false);
  if (rc || dry_only) return rc;
  hipStream_t s = (hipStream_t)stream;
  const long n0 = (long)B * 80 * T;
  const double h = 1.0 / n_steps;
  hipError_t e = launch_lik_init(data, mask, (int)B, (int)T, y, logp, s);
  for (int i = 0; i < n_steps && e == hipSuccess; ++i) {
    e = launch_lik_cast(y, n0, x32, tbuf, (int)B, (float)((i + 0.5) * h), s);   // t = (i + 0.5) h (likelihood.py:104)
    if (e != hipSuccess) break;
    rc = drift_div_pass(d, x32, mask, mu, tbuf, spk, eps, B, T, drift, div, base, w, s, false, debug);
    if (rc) return rc;
    e = launch_lik_step(y, drift, n0, h, logp, div, (int)B, s);
  }
  if (e == hipSuccess) e = launch_lik_out(y, n0, logp, (int)B, z, delta_logp, s);
  if (e != hipSuccess) return gt_internal_fail(GT_ERR_HIP, std::string("likelihood Euler: ") + hipGetErrorString(e));
  return GT_OK;
}

}  // extern "C"
