// Host side of the C ABI (include/gradtts.h): parameter registry, one-time weight packing into the
// kernels' device layouts, workspace layout and the launch sequence of one U-Net evaluation.
//
// Launch sequence of GradLogPEstimator2d.forward (model/diffusion.py:174-216), per Euler step:
//   down level l (l = 0,1,2):  ResnetBlock x2 -> LinearAttention -> Downsample (l < 2)
//   mid:                       ResnetBlock -> LinearAttention -> ResnetBlock
//   up level l (l = 2,1):      concat skip (read in place) -> ResnetBlock x2 -> LinearAttention -> Upsample
//   final_block conv + fused {GN, Mish, final_conv, Euler update}
// ResnetBlock = conv3(+GN sums) -> conv3 with GN/Mish/time-bias fused in its load (+GN sums)
//             -> res_conv 1x1 with the block output fused in its epilogue (or an elementwise kernel)
// LinearAttention = attn_kv (k/v GEMM + online softmax + context) -> merge -> M_b build -> 1x1 apply
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "gradtts.h"
#include "decoder_internal.h"
#include "kernels.h"
#include "train.h"
#include "wimage.h"

using namespace gt;

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct Shape { std::string name; std::vector<int64_t> dims; int64_t numel() const { int64_t n = 1; for (auto d : dims) n *= d; return n; } };

void add_resnet(std::vector<Shape>& v, const std::string& p, int din, int dout, int dim) {
  v.push_back({p + "mlp.1.weight", {dout, dim}});
  v.push_back({p + "mlp.1.bias", {dout}});
  v.push_back({p + "block1.block.0.weight", {dout, din, 3, 3}});
  v.push_back({p + "block1.block.0.bias", {dout}});
  v.push_back({p + "block1.block.1.weight", {dout}});
  v.push_back({p + "block1.block.1.bias", {dout}});
  v.push_back({p + "block2.block.0.weight", {dout, dout, 3, 3}});
  v.push_back({p + "block2.block.0.bias", {dout}});
  v.push_back({p + "block2.block.1.weight", {dout}});
  v.push_back({p + "block2.block.1.bias", {dout}});
  if (din != dout) {
    v.push_back({p + "res_conv.weight", {dout, din, 1, 1}});
    v.push_back({p + "res_conv.bias", {dout}});
  }
}
void add_attn(std::vector<Shape>& v, const std::string& p, int c) {
  v.push_back({p + "fn.g", {1}});
  v.push_back({p + "fn.fn.to_qkv.weight", {384, c, 1, 1}});
  v.push_back({p + "fn.fn.to_out.weight", {c, 128, 1, 1}});
  v.push_back({p + "fn.fn.to_out.bias", {c}});
}

// GradLogPEstimator2d.state_dict() inventory, registration order (diffusion.py:128-172).
std::vector<Shape> inventory(int dim, int n_spks, int spk_emb_dim, int n_feats) {
  std::vector<Shape> v;
  if (n_spks > 1 || n_spks == -1) {
    v.push_back({"spk_mlp.0.weight", {spk_emb_dim * 4, spk_emb_dim}});
    v.push_back({"spk_mlp.0.bias", {spk_emb_dim * 4}});
    v.push_back({"spk_mlp.2.weight", {n_feats, spk_emb_dim * 4}});
    v.push_back({"spk_mlp.2.bias", {n_feats}});
  }
  v.push_back({"mlp.0.weight", {dim * 4, dim}});
  v.push_back({"mlp.0.bias", {dim * 4}});
  v.push_back({"mlp.2.weight", {dim, dim * 4}});
  v.push_back({"mlp.2.bias", {dim}});
  const int dims[4] = {2 + (n_spks > 1 ? 1 : 0), dim, dim * 2, dim * 4};
  for (int i = 0; i < 3; ++i) {
    const std::string p = "downs." + std::to_string(i) + ".";
    add_resnet(v, p + "0.", dims[i], dims[i + 1], dim);
    add_resnet(v, p + "1.", dims[i + 1], dims[i + 1], dim);
    add_attn(v, p + "2.", dims[i + 1]);
    if (i < 2) {
      v.push_back({p + "3.conv.weight", {dims[i + 1], dims[i + 1], 3, 3}});
      v.push_back({p + "3.conv.bias", {dims[i + 1]}});
    }
  }
  for (int i = 0; i < 2; ++i) {   // reversed(in_out[1:]) = (128,256), (64,128)
    const int din = dims[2 - i], dout = dims[3 - i];
    const std::string p = "ups." + std::to_string(i) + ".";
    add_resnet(v, p + "0.", dout * 2, din, dim);
    add_resnet(v, p + "1.", din, din, dim);
    add_attn(v, p + "2.", din);
    v.push_back({p + "3.conv.weight", {din, din, 4, 4}});
    v.push_back({p + "3.conv.bias", {din}});
  }
  add_resnet(v, "mid_block1.", dims[3], dims[3], dim);
  add_attn(v, "mid_attn.", dims[3]);
  add_resnet(v, "mid_block2.", dims[3], dims[3], dim);
  v.push_back({"final_block.block.0.weight", {dim, dim, 3, 3}});
  v.push_back({"final_block.block.0.bias", {dim}});
  v.push_back({"final_block.block.1.weight", {dim}});
  v.push_back({"final_block.block.1.bias", {dim}});
  v.push_back({"final_conv.weight", {1, dim, 1, 1}});
  v.push_back({"final_conv.bias", {1}});
  return v;
}

// ResnetBlocks in execution order; their time-bias slices are stacked into one [rows][1792] table.
const char* kResnets[12] = {"downs.0.0.", "downs.0.1.", "downs.1.0.", "downs.1.1.", "downs.2.0.", "downs.2.1.",
                            "mid_block1.", "mid_block2.", "ups.0.0.", "ups.0.1.", "ups.1.0.", "ups.1.1."};

bool ends_with(const std::string& s, const char* suf) {
  const size_t n = strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}
bool starts_with(const std::string& s, const char* pre) { return s.compare(0, strlen(pre), pre) == 0; }

uint16_t f2bf(float f) {   // round to nearest even (finite inputs)
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct Blob {   // host staging of one packed device arena
  std::vector<uint8_t> bytes;
  std::map<std::string, size_t> off;
  size_t put(const std::string& key, const void* src, size_t n) {
    size_t o = (bytes.size() + 255) & ~size_t(255);
    bytes.resize(o + n);
    memcpy(bytes.data() + o, src, n);
    off[key] = o;
    return o;
  }
};

// largest call batch on the small-batch tile plan (small_plan). Measured (50-step decodes, T = 512, one box):
// B = 1 47.3 vs 78.9 ms, B = 2 50.7 vs 80.6, B = 4 61.0 vs 82.7, B = 8 94.9 vs 94.3, B = 16 152.9 vs 116.3
constexpr int64_t kSmallB = 4;
// the largest small_b accepted (gt_decoder_set_small_batch, GT_SMALL_B): chunks of more utterances never take the
// small-batch plan, so the workspace holds its 256 attention tiles per utterance only up to this batch size
constexpr int64_t kSmallBMax = 16;
// small-batch plan attention tiles per utterance and merge rows per workgroup. Measured (B = 1, T = 512, N = 50, one
// box): 64 tiles + one merge workgroup per head 43.9 ms per decode, + 8 merge workgroups 42.9, 128 tiles 42.3, 256 42.0
constexpr int kSmallTiles = 256;
constexpr int kMergeDrSmall = 4;
// small-batch plan split-K target: workgroups per utterance the 128-wide 3x3 convs aim for (conv_small_ksplit; 0 off).
// Measured in round 4 (T = 512, N = 50, one box, ms per decode, off / 256): B = 1 42.4 / 37.8, B = 2 45.7 / 42.6, B = 4
// 57.2 / 59.4; targets 384 and 512 38.4 at B = 1 (level-1 tiles split too: two workgroup rounds)
constexpr int kSkTarget = 256;

}  // namespace

struct gt_decoder {
  int n_feats, dim, n_spks, spk_emb_dim;
  float beta_min, beta_max, pe_scale;
  std::vector<Shape> inv;
  std::map<std::string, int> index;
  std::vector<std::vector<float>> host;
  std::vector<bool> set;
  // one packed device arena per compute dtype code (GT_F32, GT_BF16, GT_BF16_W8, GT_FP8)
  static constexpr int kCodes = 4;
  bool dirty[kCodes] = {true, true, true, true};
  void* arena[kCodes] = {nullptr, nullptr, nullptr, nullptr};
  std::map<std::string, void*> dp[kCodes];
  std::map<std::string, int> cinpad[kCodes];
  float freqs[32];
  int64_t packs = 0;          // weight packings performed (checkpoint tests: exactly one per parameter change)
  // profiling (diagnostics / bench roofline): HIP events around every launch
  bool prof = false;
  std::string prof_prefix;   // non-empty: only launches whose "<kernel>@<shape>" name starts with it
  struct Rec { std::string kernel; double flop, bytes; hipEvent_t e0, e1; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  size_t pool_used = 0;
  // captured sampler segments (gt_reverse_diffusion): HIP graphs of S Euler steps, keyed by everything the
  // captured kernels bake in (shapes, dtype, tensor / workspace / weight-arena addresses)
  // off by default: same-box A/B (tools/ab_graph.sh) measured no gain at B = 32 and a 7 % loss at B = 4 (every
  // batch size is GPU-bound; graph replay adds inter-node gaps); GT_GRAPHS=1 or gt_decoder_set_graphs enables
  bool graphs = false;
  hipStream_t cap_stream = nullptr;
  struct Graph { std::vector<uintptr_t> key; hipGraphExec_t exec; };
  std::vector<Graph> gcache;   // most recently used last
  int64_t captures = 0;
  int64_t max_chunk = 0;       // > 0: cap on utterances per internal batch chunk (GT_MAX_CHUNK, tests)
  // bf16 calls on at most small_b utterances run the small-batch tile plan (small_plan below);
  // GT_SMALL_B at creation or gt_decoder_set_small_batch
  int64_t small_b = kSmallB;
  // bf16 throughput-plan 3x3 convs at levels 1-2 on conv3w (one 8-wave workgroup per CU owning all output channels of
  // a tile); GT_CONV3W=0 at creation or gt_decoder_set_wide_conv(dec, 0) runs them on conv_kernel
  bool wide = true;
  // fp8-operand convs (GT_FP8) of the same shapes on conv3w_a8 (conv3w_a8.hip) instead of conv_kernel's A8 form, when
  // `wide` too; GT_CONV3W_A8=0 disables it (A/B)
  bool wide_a8 = true;
  // level-0 attention output + Downsample as one pass (attn_down_kernel); GT_ATTN_DS=0 at creation: two launches
  bool attn_ds = true;
  // the first ResnetBlock's output formed by the next block's conv (conv64 IN_RB0) instead of its own pass
  // (rbout_input); GT_RB0_FUSE=0 at creation: the pass
  bool rb0_fuse = true;
  // the 64 -> 64 3x3 convs on conv64 (persistent weight-resident, conv64.hip) for bf16 / fp8-weight calls; GT_CONV64=0
  // at creation: conv_kernel (A/B, and the fractional-mask path agreement test)
  bool conv64 = true;
  // the U-Net input conv (downs.0.0's block1, 2 -> 64 channels) recomputed inside the next conv (conv64 IN_X0) from
  // {mu, x_t}, with a statistics-only pass for its GroupNorm, instead of written and read back (bf16 compute dtype,
  // single speaker); GT_X0_FUSE=0 at creation: the input conv
  bool x0_fuse = true;
  // the throughput plan's bf16 1x1 convs (res_conv + block output, attention output + residual) on conv1s (LDS-DMA
  // ring, conv1s.hip); GT_CONV1S=0 at creation: conv_kernel
  bool conv1s = true;
  // ups.1's attention output + Upsample as one pass (attn_up_kernel); GT_ATTN_US=0 at creation: two launches
  bool attn_us = true;
  // small-batch plan attention: tiles per utterance (GT_ATTN_TILES_SMALL) and the merge's rows per workgroup
  // (GT_MERGE_DR_SMALL: 4 spreads a head's merge over 8 workgroups; 32 is the throughput plan's single workgroup)
  int small_tiles = kSmallTiles;
  int merge_dr_small = kMergeDrSmall;
  int sk_target = kSkTarget;   // GT_SK_TARGET (0: no split-K)
  // training path: every parameter in fp32, reference layout, contiguous in inventory order (the layout of the
  // flat gradient buffer too), plus the SinusoidalPosEmb frequencies at the end
  bool raw_dirty = true;
  // gt_decoder_set_params_device wrote the fp32 block on the device: the host copies (and every weight image
  // packed from them) are stale until refresh_host() reads the block back
  bool host_stale = false;
  hipEvent_t dev_done = nullptr;   // recorded on the caller's stream by set_params_device (refresh_host waits on it)
  float* raw = nullptr;
  std::vector<int64_t> raw_off;
  int64_t raw_numel = 0;
  void drop_graphs() {
    for (auto& g : gcache) (void)hipGraphExecDestroy(g.exec);
    gcache.clear();
  }
  hipEvent_t ev() {
    if (pool_used == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    return pool[pool_used++];
  }
};

namespace {

int ck_of(int dt) { return dt ? 32 : 16; }
size_t esize(int dt) { return dt ? 2 : 4; }


// pack [Cout][Cin][KH][KW] (or ConvTranspose [Cin][Cout][4][4], as 4 parity images) into the
// conv_kernel weight image (wimage.h) in the compute dtype
void pack_conv(Blob& blob, gt_decoder* d, int dt, int code, const std::string& key, const std::vector<float>& w,
               const std::vector<int64_t>& shp, bool convT) {
  int cin, cout, ntap, npar;
  if (!convT) {
    cout = (int)shp[0]; cin = (int)shp[1]; ntap = (int)(shp[2] * shp[3]); npar = 1;
  } else {
    cin = (int)shp[0]; cout = (int)shp[1]; ntap = 4; npar = 4;
  }
  const WImg W = conv_wimg(dt, ntap, cin, cout);
  const int es = (int)esize(dt);
  std::vector<uint8_t> img((size_t)npar * W.total, 0);
  auto put = [&](int par, int co, int tap, int ci, float v) {
    uint8_t* q = img.data() + (size_t)par * W.total + conv_wimg_off(W, co, tap, ci, es);
    if (dt) { const uint16_t hb = f2bf(v); memcpy(q, &hb, 2); }
    else memcpy(q, &v, 4);
  };
  if (!convT) {
    for (int co = 0; co < cout; ++co)
      for (int ci = 0; ci < cin; ++ci)
        for (int t = 0; t < ntap; ++t) put(0, co, t, ci, w[((size_t)co * cin + ci) * ntap + t]);
  } else {
    // parity p = 2*pf + pt, tap = 2*a + b; kernel index K(parity, a): p=0 -> {1, 3}, p=1 -> {0, 2}
    const int K[2][2] = {{1, 3}, {0, 2}};
    for (int par = 0; par < 4; ++par) {
      const int pf = par >> 1, pt = par & 1;
      for (int co = 0; co < cout; ++co)
        for (int tap = 0; tap < 4; ++tap) {
          const int kh = K[pf][tap >> 1], kw = K[pt][tap & 1];
          for (int ci = 0; ci < cin; ++ci) put(par, co, tap, ci, w[(((size_t)ci * cout + co) * 4 + kh) * 4 + kw]);
        }
    }
  }
  blob.put(key, img.data(), img.size());
  d->cinpad[code][key] = W.nchunk * W.ck;
}

}  // namespace

// e4m3fn (OCP FP8: bias 7, no infinities, 0x7f = NaN, max 448) of a finite float, round to nearest even,
// saturating at 448 -- the rounding of torch's float8_e4m3fn conversion for in-range values.
extern "C" uint8_t gt_f32_to_e4m3(float x) {
  const uint8_t sgn = std::signbit(x) ? 0x80 : 0;
  const double a = std::fabs((double)x);
  if (a != a) return 0x7f;
  if (a < 0.015625) return sgn | (uint8_t)std::nearbyint(a * 512.0);   // subnormals (2^-9 steps); 8 = 2^-6
  int e;
  const double m = std::frexp(a, &e);            // a = m * 2^e, m in [0.5, 1)
  int E = e - 1;
  int q = (int)std::nearbyint((2.0 * m - 1.0) * 8.0);
  if (q == 8) { q = 0; ++E; }
  if (E > 8 || (E == 8 && q == 7)) return sgn | 0x7e;
  return sgn | (uint8_t)(((E + 7) << 3) | q);
}

// Per-output-channel e4m3 quantization (GT_BF16_W8): scale[o] = max|w[o,:]| / 448 (1 if the row is zero),
// q = e4m3(w / scale[o]) in fp32 arithmetic; row o of `rows` is `cols` values at stride `col_stride`
// starting at o * row_stride.
extern "C" int gt_quantize_e4m3(const float* w, int64_t rows, int64_t cols, int64_t row_stride, int64_t col_stride,
                                uint8_t* q, float* scale) {
  if (!w || !q || !scale || rows < 0 || cols < 0) return GT_ERR_ARG;
  for (int64_t o = 0; o < rows; ++o) {
    float amax = 0.f;
    for (int64_t i = 0; i < cols; ++i) amax = std::max(amax, std::fabs(w[o * row_stride + i * col_stride]));
    const float sc = amax > 0.f ? amax / 448.0f : 1.0f;
    scale[o] = sc;
    for (int64_t i = 0; i < cols; ++i) q[o * row_stride + i * col_stride] = gt_f32_to_e4m3(w[o * row_stride + i * col_stride] / sc);
  }
  return GT_OK;
}

namespace {

// fp8 image (wimage.h conv_wimg8) of a 3x3 [Cout][Cin][3][3] or ConvTranspose [Cin][Cout][4][4] weight,
// quantized per output channel; the scales go to key + ".s"
void pack_conv8(Blob& blob, gt_decoder* d, int code, const std::string& key, const std::vector<float>& w,
                const std::vector<int64_t>& shp, bool convT) {
  int cin, cout, ntap, npar;
  if (!convT) {
    cout = (int)shp[0]; cin = (int)shp[1]; ntap = (int)(shp[2] * shp[3]); npar = 1;
  } else {
    cin = (int)shp[0]; cout = (int)shp[1]; ntap = 4; npar = 4;
  }
  const int kk = convT ? 16 : ntap;   // kernel taps per (co, ci)
  std::vector<uint8_t> q(w.size());
  std::vector<float> sc(cout);
  if (!convT) gt_quantize_e4m3(w.data(), cout, (int64_t)cin * kk, (int64_t)cin * kk, 1, q.data(), sc.data());
  else {   // output channel co: elements ci*cout*16 + co*16 + k
    for (int co = 0; co < cout; ++co) {
      std::vector<float> row((size_t)cin * 16);
      for (int ci = 0; ci < cin; ++ci)
        for (int k = 0; k < 16; ++k) row[(size_t)ci * 16 + k] = w[((size_t)ci * cout + co) * 16 + k];
      std::vector<uint8_t> qr(row.size());
      gt_quantize_e4m3(row.data(), 1, (int64_t)row.size(), 0, 1, qr.data(), &sc[co]);
      for (int ci = 0; ci < cin; ++ci)
        for (int k = 0; k < 16; ++k) q[((size_t)ci * cout + co) * 16 + k] = qr[(size_t)ci * 16 + k];
    }
  }
  const WImg W = conv_wimg8(ntap, cin, cout);
  std::vector<uint8_t> img((size_t)npar * W.total, 0);
  if (!convT) {
    for (int co = 0; co < cout; ++co)
      for (int ci = 0; ci < cin; ++ci)
        for (int t = 0; t < ntap; ++t) img[conv_wimg8_off(W, co, t, ci)] = q[((size_t)co * cin + ci) * ntap + t];
  } else {
    const int K[2][2] = {{1, 3}, {0, 2}};   // as pack_conv
    for (int par = 0; par < 4; ++par) {
      const int pf = par >> 1, pt = par & 1;
      for (int co = 0; co < cout; ++co)
        for (int tap = 0; tap < 4; ++tap) {
          const int kh = K[pf][tap >> 1], kw = K[pt][tap & 1];
          for (int ci = 0; ci < cin; ++ci)
            img[(size_t)par * W.total + conv_wimg8_off(W, co, tap, ci)] = q[(((size_t)ci * cout + co) * 4 + kh) * 4 + kw];
        }
    }
  }
  blob.put(key, img.data(), img.size());
  blob.put(key + ".s", sc.data(), sc.size() * 4);
  d->cinpad[code][key] = W.nchunk * W.ck;
}

// fp8-operand image (wimage.h conv_wimga8, GT_FP8) of a 3x3 [Cout][Cin][3][3] weight, quantized per output channel as
// pack_conv8 does; scales to key + ".s", and key + ".a8" marks the image kind for the launch (Run::setw)
void pack_conva8(Blob& blob, gt_decoder* d, int code, const std::string& key, const std::vector<float>& w,
                 const std::vector<int64_t>& shp) {
  const int cout = (int)shp[0], cin = (int)shp[1];
  std::vector<uint8_t> q(w.size());
  std::vector<float> sc(cout);
  gt_quantize_e4m3(w.data(), cout, (int64_t)cin * 9, (int64_t)cin * 9, 1, q.data(), sc.data());
  const WImg W = conv_wimga8(cin, cout);
  std::vector<uint8_t> img((size_t)W.total, 0);   // tap slot 9 and the row pads stay zero
  for (int co = 0; co < cout; ++co)
    for (int ci = 0; ci < cin; ++ci)
      for (int t = 0; t < 9; ++t) img[conv_wimga8_off(W, co, t, ci)] = q[((size_t)co * cin + ci) * 9 + t];
  blob.put(key, img.data(), img.size());
  blob.put(key + ".s", sc.data(), sc.size() * 4);
  const int one = 1;
  blob.put(key + ".a8", &one, sizeof(one));
  d->cinpad[code][key] = W.nchunk * W.ck;
}

// pack a 64->64 3x3 [Cout][Cin][3][3] weight in conv64's register-fragment order (conv64.hip), bf16:
// [cb 2][chunk 4][tap 9][lane 64][8 ci]: lane (r, h) = output channel cb*32 + r, input channels 16 chunk + 8h .. +7
// The U-Net input conv [64][2][3][3] as the A fragments of conv64.hip c64::x0_mfma: [cb][k-step][lane][8] bf16, lane (r, h)
// = output channel cb*32 + r; element j of k-step 0 is channel j & 1 of tap (h, j >> 1) for j < 6 and of tap (2, h) for
// j = 6, 7; k-step 1 holds tap (2, 2) in elements 0, 1 of half 0, zeros elsewhere
void pack_x0(Blob& blob, const std::string& key, const std::vector<float>& w) {
  std::vector<uint16_t> img(2 * 2 * 64 * 8, 0);
  for (int cb = 0; cb < 2; ++cb)
    for (int ks = 0; ks < 2; ++ks)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int r = lane & 31, h = lane >> 5, co = cb * 32 + r, ch = j & 1, t = j >> 1;
          int dr = -1, dc = -1;
          if (ks == 0) { dr = t < 3 ? h : 2; dc = t < 3 ? t : h; }
          else if (h == 0 && t == 0) { dr = 2; dc = 2; }
          if (dr < 0) continue;
          img[((cb * 2 + ks) * 64 + lane) * 8 + j] = f2bf(w[((co * 2 + ch) * 3 + dr) * 3 + dc]);
        }
  blob.put(key, img.data(), img.size() * 2);
}

void pack_conv64(Blob& blob, const std::string& key, const std::vector<float>& w) {
  std::vector<uint16_t> img((size_t)2 * 4 * 9 * 64 * 8);
  size_t i = 0;
  for (int cb = 0; cb < 2; ++cb)
    for (int ch = 0; ch < 4; ++ch)
      for (int tap = 0; tap < 9; ++tap)
        for (int lane = 0; lane < 64; ++lane)
          for (int k = 0; k < 8; ++k) {
            const int co = cb * 32 + (lane & 31), ci = ch * 16 + (lane >> 5) * 8 + k;
            img[i++] = f2bf(w[((size_t)co * 64 + ci) * 9 + tap]);
          }
  blob.put(key, img.data(), img.size() * 2);
}

// pack a 3x3 [Cout][Cin][3][3] weight as MFMA A fragments (attn_down.hip's stride-2 stage), bf16:
// [cb Cout/32][chunk Cin/16][tap 9][lane 64][8 ci]: lane (r, h) = output channel 32 cb + r, input channels 16 chunk + 8h ..
// (for 64 -> 64 the same bytes as pack_conv64)
void pack_frag3x3(Blob& blob, const std::string& key, const std::vector<float>& w, int cout, int cin) {
  std::vector<uint16_t> img((size_t)cout * cin * 9);
  size_t i = 0;
  for (int cb = 0; cb < cout / 32; ++cb)
    for (int ch = 0; ch < cin / 16; ++ch)
      for (int tap = 0; tap < 9; ++tap)
        for (int lane = 0; lane < 64; ++lane)
          for (int k = 0; k < 8; ++k) {
            const int co = cb * 32 + (lane & 31), ci = ch * 16 + (lane >> 5) * 8 + k;
            img[i++] = f2bf(w[((size_t)co * cin + ci) * 9 + tap]);
          }
  blob.put(key, img.data(), img.size() * 2);
}

// pack a ConvTranspose2d [Cin][Cout][4][4] weight (stride 2, padding 1) as MFMA A fragments of its four sub-pixel 2x2
// convs (attn_up_kernel), bf16: [parity 2 pf + pt][cb Cout/32][chunk Cin/16][tap 2a + b][lane 64][8 ci], kernel index
// kh = K[pf][a], kw = K[pt][b] with K = {{1, 3}, {0, 2}} (as pack_conv's transposed images)
void pack_fragT(Blob& blob, const std::string& key, const std::vector<float>& w, int cin, int cout) {
  const int K[2][2] = {{1, 3}, {0, 2}};
  std::vector<uint16_t> img((size_t)4 * cout * cin * 4);
  size_t i = 0;
  for (int par = 0; par < 4; ++par)
    for (int cb = 0; cb < cout / 32; ++cb)
      for (int ch = 0; ch < cin / 16; ++ch)
        for (int tap = 0; tap < 4; ++tap)
          for (int lane = 0; lane < 64; ++lane)
            for (int k = 0; k < 8; ++k) {
              const int co = cb * 32 + (lane & 31), ci = ch * 16 + (lane >> 5) * 8 + k;
              const int kh = K[par >> 1][tap >> 1], kw = K[par & 1][tap & 1];
              img[i++] = f2bf(w[(((size_t)ci * cout + co) * 4 + kh) * 4 + kw]);
            }
  blob.put(key, img.data(), img.size() * 2);
}

// pack a 3x3 [Cout][Cin][3][3] weight (Cin % 32 == 0) in conv3w's slot order (conv3w.hip), bf16: one slot per
// (32-channel chunk c, tap t) in phase order k = 9 c + t, each [plane q 0..3][co][8 channels 32 c + 8 q ..] -- the LDS
// image of a weight slot, so staging one is a straight DMA
void pack_conv3w(Blob& blob, const std::string& key, const std::vector<float>& w, int cout, int cin) {
  std::vector<uint16_t> img((size_t)(cin / 32) * 9 * cout * 32);
  size_t i = 0;
  for (int c = 0; c < cin / 32; ++c)
    for (int t = 0; t < 9; ++t)
      for (int q = 0; q < 4; ++q)
        for (int co = 0; co < cout; ++co)
          for (int e = 0; e < 8; ++e) img[i++] = f2bf(w[((size_t)co * cin + 32 * c + 8 * q + e) * 9 + t]);
  blob.put(key, img.data(), img.size() * 2);
}

// pack a 3x3 [Cout][Cin][3][3] weight (Cin % 32 == 0) for conv3w_a8 (conv3w_a8.hip): e4m3 codes quantized per output
// channel exactly as pack_conva8 (its ".s" scale serves both), one slot per (32-channel chunk c, tap pair u) in phase
// order k = 5 c + u, each [plane q = 2 v + h][co][16 channels 32 c + 16 h ..] of tap 2 u + v (tap 9: zero) -- the LDS
// image of a weight slot
void pack_conv3w_a8(Blob& blob, const std::string& key, const std::vector<float>& w, int cout, int cin) {
  std::vector<uint8_t> q(w.size());
  std::vector<float> sc(cout);
  gt_quantize_e4m3(w.data(), cout, (int64_t)cin * 9, (int64_t)cin * 9, 1, q.data(), sc.data());
  std::vector<uint8_t> img((size_t)(cin / 32) * 5 * cout * 64, 0);
  size_t i = 0;
  for (int c = 0; c < cin / 32; ++c)
    for (int u = 0; u < 5; ++u)
      for (int pl = 0; pl < 4; ++pl) {
        const int t = 2 * u + (pl >> 1), hh = pl & 1;
        for (int co = 0; co < cout; ++co)
          for (int e = 0; e < 16; ++e, ++i)
            if (t < 9) img[i] = q[((size_t)co * cin + 32 * c + 16 * hh + e) * 9 + t];
      }
  blob.put(key, img.data(), img.size());
}

// e4m3 values (codes decoded, without the scale) of a [rows][...] weight quantized per row as gt_quantize_e4m3 does:
// exact in bf16, for the conv64 image of an fp8-weight conv (the scale is applied in conv64's epilogue)
std::vector<float> e4m3_values(const std::vector<float>& w, int rows) {
  const int64_t cols = (int64_t)w.size() / rows;
  std::vector<uint8_t> q(w.size());
  std::vector<float> sc(rows);
  gt_quantize_e4m3(w.data(), rows, cols, cols, 1, q.data(), sc.data());
  std::vector<float> v(w.size());
  for (size_t i = 0; i < q.size(); ++i) {
    const int s = q[i] >> 7, e = (q[i] >> 3) & 15, m = q[i] & 7;
    const float a = e ? std::ldexp(1.f + m / 8.f, e - 7) : std::ldexp(m / 8.f, -6);
    v[i] = s ? -a : a;
  }
  return v;
}

// the same for a ConvTranspose2d [Cin][Cout][4][4] weight, quantized per output channel (dim 1) as pack_conv8's
// transposed path does; returned in the weight's own layout
std::vector<float> e4m3_values_t(const std::vector<float>& w, int cin, int cout) {
  std::vector<float> rows((size_t)cout * cin * 16), v(w.size());
  for (int co = 0; co < cout; ++co)
    for (int ci = 0; ci < cin; ++ci)
      for (int k = 0; k < 16; ++k) rows[((size_t)co * cin + ci) * 16 + k] = w[((size_t)ci * cout + co) * 16 + k];
  const std::vector<float> q = e4m3_values(rows, cout);
  for (int co = 0; co < cout; ++co)
    for (int ci = 0; ci < cin; ++ci)
      for (int k = 0; k < 16; ++k) v[((size_t)ci * cout + co) * 16 + k] = q[((size_t)co * cin + ci) * 16 + k];
  return v;
}

// a 3x3 [Cout][Cin][3][3] weight conv3w covers (Cin % 32 == 0, Cout 64 / 128 / 256; not the 64 -> 64 convs of conv64)
static bool conv3w_shape(const std::vector<int64_t>& shp) {
  return shp.size() == 4 && shp[2] == 3 && shp[3] == 3 && shp[1] % 32 == 0 && (shp[0] == 64 || shp[0] == 128 || shp[0] == 256) &&
         !(shp[0] == 64 && shp[1] == 64);
}

int prepare(gt_decoder* d, int code) {
  if (!d->dirty[code]) return GT_OK;
  if (int rc = gt_internal_refresh_host(d)) return rc;
  const int dt = code ? 1 : 0;          // activation dtype: fp32 / bf16
  const bool w8 = code == GT_BF16_W8 || code == GT_FP8;   // fp8 images for the 3x3 / stride-2 / transposed convs
  const bool a8 = code == GT_FP8;   // ... fp8 operands too for the 3x3 convs over activations (Cin >= 32)
  for (size_t i = 0; i < d->inv.size(); ++i)
    if (!d->set[i]) return fail(GT_ERR_PARAM, "parameter never set: " + d->inv[i].name);
  Blob blob;
  auto H = [&](const std::string& k) -> const std::vector<float>& { return d->host[d->index.at(k)]; };
  for (size_t i = 0; i < d->inv.size(); ++i) {
    const std::string& k = d->inv[i].name;
    const auto& shp = d->inv[i].dims;
    const auto& w = d->host[i];
    const bool c64 = dt && ends_with(k, ".block.0.weight") && shp[0] == 64 && shp[1] == 64 && shp[2] == 3 && shp[3] == 3;
    if (w8 && c64) {   // 64 -> 64 (level 0): conv64 with the e4m3 values (fp8 modes alike: bf16 operands there)
      pack_conv8(blob, d, code, k, w, shp, false);
      pack_conv64(blob, k + ".w64", e4m3_values(w, 64));
    } else if (a8 && ends_with(k, ".block.0.weight") && shp[1] >= 32) {
      pack_conva8(blob, d, code, k, w, shp);
      if (conv3w_shape(shp)) pack_conv3w_a8(blob, k + ".w3a", w, (int)shp[0], (int)shp[1]);   // conv3w_a8
    } else if (w8 && (ends_with(k, ".block.0.weight") || (starts_with(k, "downs.") && ends_with(k, ".3.conv.weight")))) {
      pack_conv8(blob, d, code, k, w, shp, false);
      if (ends_with(k, ".block.0.weight") && shp[0] == 64 && shp[1] == 2 && shp[2] == 3 && shp[3] == 3)
        pack_x0(blob, k + ".x0", e4m3_values(w, 64));   // the input conv recomputed by conv64 IN_X0: e4m3 values
      if (code == GT_BF16_W8 && ends_with(k, ".block.0.weight") && conv3w_shape(shp))   // conv3w: the e4m3 values
        pack_conv3w(blob, k + ".w3w", e4m3_values(w, (int)shp[0]), (int)shp[0], (int)shp[1]);
      if (starts_with(k, "downs.") && ends_with(k, ".3.conv.weight") && shp[0] == 64 && shp[1] == 64)
        pack_frag3x3(blob, k + ".wfr", e4m3_values(w, 64), 64, 64);   // attn_down_kernel: the e4m3 values
    } else if (w8 && starts_with(k, "ups.") && ends_with(k, ".3.conv.weight")) {
      pack_conv8(blob, d, code, k, w, shp, true);
      if (shp[0] == 64 && shp[1] == 64) pack_fragT(blob, k + ".wfr", e4m3_values_t(w, 64, 64), 64, 64);   // attn_up_kernel
    } else if (ends_with(k, ".block.0.weight") || (starts_with(k, "downs.") && ends_with(k, ".3.conv.weight")) ||
        ends_with(k, "res_conv.weight")) {
      pack_conv(blob, d, dt, code, k, w, shp, false);
      if (c64) pack_conv64(blob, k + ".w64", w);
      if (code == GT_BF16 && ends_with(k, ".block.0.weight") && !c64 && conv3w_shape(shp))
        pack_conv3w(blob, k + ".w3w", w, (int)shp[0], (int)shp[1]);
      if (code == GT_BF16 && starts_with(k, "downs.") && ends_with(k, ".3.conv.weight") && shp[0] == shp[1] &&
          (shp[0] == 64 || shp[0] == 128))
        pack_frag3x3(blob, k + ".wfr", w, (int)shp[0], (int)shp[1]);   // the Downsample of attn_down_kernel
      if (ends_with(k, "res_conv.weight") && shp[1] <= 3) blob.put(k + ".f32", w.data(), w.size() * 4);   // rbout_input
      if (code == GT_BF16 && ends_with(k, ".block.0.weight") && shp[0] == 64 && shp[1] == 2 && shp[2] == 3 && shp[3] == 3)
        pack_x0(blob, k + ".x0", w);   // the input conv recomputed by conv64 IN_X0 / x0_stats
    } else if (starts_with(k, "ups.") && ends_with(k, ".3.conv.weight")) {
      pack_conv(blob, d, dt, code, k, w, shp, true);
      if (code == GT_BF16 && shp[0] == 64 && shp[1] == 64)
        pack_fragT(blob, k + ".wfr", w, (int)shp[0], (int)shp[1]);   // the Upsample of attn_up_kernel
    } else if (ends_with(k, "to_qkv.weight")) {
      const int C = (int)shp[1];
      std::vector<float> qT((size_t)C * 128);   // W_q^T [C][128] for attn_fold (row-major staging like A_b)
      for (int j = 0; j < 128; ++j)
        for (int c = 0; c < C; ++c) qT[(size_t)c * 128 + j] = w[(size_t)j * C + c];
      blob.put(k + ".qT", qT.data(), qT.size() * 4);
      std::vector<float> kv(w.begin() + 128 * C, w.end());   // [256][C], Cpad == C (multiple of 32)
      if (dt) {
        std::vector<uint16_t> hb(kv.size());
        for (size_t j = 0; j < kv.size(); ++j) hb[j] = f2bf(kv[j]);
        blob.put(k, hb.data(), hb.size() * 2);
      } else {
        blob.put(k, kv.data(), kv.size() * 4);
      }
    } else {
      blob.put(k, w.data(), w.size() * 4);
      if (ends_with(k, "to_out.bias")) {   // Rezero: g * (W_out o + b_out) -> fold g into the bias
        const std::string gk = k.substr(0, k.size() - strlen("fn.to_out.bias")) + "g";
        const float g = H(gk)[0];
        std::vector<float> gb(w.size());
        for (size_t j = 0; j < w.size(); ++j) gb[j] = g * w[j];
        blob.put(k + ".g", gb.data(), gb.size() * 4);
      }
    }
  }
  {   // stacked ResnetBlock time MLPs
    std::vector<float> wr, br;
    for (const char* rk : kResnets) {
      const auto& W = H(std::string(rk) + "mlp.1.weight");
      const auto& Bv = H(std::string(rk) + "mlp.1.bias");
      wr.insert(wr.end(), W.begin(), W.end());
      br.insert(br.end(), Bv.begin(), Bv.end());
    }
    blob.put("tb.w", wr.data(), wr.size() * 4);
    blob.put("tb.b", br.data(), br.size() * 4);
  }
  blob.put("freqs", d->freqs, sizeof(d->freqs));
  if (d->arena[code]) { (void)hipFree(d->arena[code]); d->arena[code] = nullptr; }
  if (hipMalloc(&d->arena[code], blob.bytes.size()) != hipSuccess) return fail(GT_ERR_HIP, "hipMalloc(weights) failed");
  if (hipMemcpy(d->arena[code], blob.bytes.data(), blob.bytes.size(), hipMemcpyHostToDevice) != hipSuccess)
    return fail(GT_ERR_HIP, "hipMemcpy(weights) failed");
  d->dp[code].clear();
  for (auto& kv : blob.off) d->dp[code][kv.first] = (uint8_t*)d->arena[code] + kv.second;
  d->dirty[code] = false;
  d->packs += 1;
  d->drop_graphs();   // captured graphs point into the old arena
  return GT_OK;
}

// ---------------------------------------------------------------- workspace
struct Layout {
  size_t act[3][5];        // per level: 4-5 activation buffers
  size_t stats, part, G, Mw, tb, spk, betas, step, total;
  size_t skcnt, skpart; long skcnt_n, skpart_n;   // small plan split-K: counters, fp32 partials (0: not allocated)
  int pmax;
  int tile_pos[3], ntile[3];
};

// Attention tile size depends only on the positions per utterance and the tile plan (never on B), so an utterance gets
// the same online-softmax partition -- hence bit-identical arithmetic -- whatever batch or GPU shard it
// is decoded in (sharded runs must match the single-GPU run).
// `target` tiles per utterance: the throughput plan takes 16 for utterances of 8192+ positions and 32 below (fewer
// online-softmax partials to merge, longer streams per workgroup: same-box +1.0-1.3 %), the small-batch plan 256
// (kSmallTiles) so that one utterance still spreads over the GPU; the workspace is sized for the larger of the two.
void attn_tiles(int64_t n, int target, int& tile_pos, int& ntile) {
  int64_t tp = (n + target - 1) / target;
  tp = (tp + 63) / 64 * 64;
  if (tp < 64) tp = 64;
  tile_pos = (int)tp;
  ntile = (int)((n + tp - 1) / tp);
}

// Largest number of GroupNorm partial slots one utterance's producer writes, over every level, output width,
// operand mode and both tile plans (conv_kernel tiles and conv64 segments). Each stats slot holds this many, so no
// producer spills into the next slot whatever plan a call takes (the small plan's 2-row 64-wide level-0 tiles write
// 40*ceil(T/64) partials, more than conv64's 20*ceil(T/32) when T % 64 is 1..32). Run::conv3_stats checks it again
// per launch.
int max_gn_parts(int dt, int64_t T) {
  int m = 0;
  for (int l = 0; l < 3; ++l)
    for (int small = 0; small < 2; ++small) {
      if (small && !dt) continue;
      m = std::max(m, conv64_nparts(80 >> l, (int)(T >> l), small));
      m = std::max(m, x0_stats_nparts(80 >> l, (int)(T >> l)));
      for (int cout : {64, 128, 256}) m = std::max(m, conv3w_nparts(80 >> l, (int)(T >> l), cout));
      for (int cout : {64, 128, 256})
        for (int im : {IN_INPUT, IN_MASK, IN_GN, IN_PLAIN})
          for (int a8 = 0; a8 <= dt; ++a8)   // fp8-operand convs (GT_FP8) tile differently
            m = std::max(m, conv_gn_nparts(dt, (InMode)im, 80 >> l, (int)(T >> l), cout, small, a8));
    }
  return m;
}

Layout layout(int dt, int64_t B, int64_t T, int32_t N, int small_tiles, int small, int sk_target) {
  Layout L{};
  size_t o = 0;
  auto take = [&](size_t bytes) { size_t r = o; o = (o + bytes + 255) & ~size_t(255); return r; };
  const int C[3] = {64, 128, 256};
  for (int l = 0; l < 3; ++l) {
    const size_t n = (size_t)B * (80 >> l) * (T >> l) * C[l] * esize(dt);
    for (int i = 0; i < 5; ++i) L.act[l][i] = take(n);
  }
  L.pmax = max_gn_parts(dt, T);   // GroupNorm partial slots per utterance: the largest producer grid of either tile plan
  L.stats = take((size_t)25 * B * L.pmax * 16 * sizeof(float));
  int maxtile = 0;
  for (int l = 0; l < 3; ++l) {
    attn_tiles((int64_t)(80 >> l) * (T >> l), small_tiles, L.tile_pos[l], L.ntile[l]);   // small-batch plan
    if (B <= kSmallBMax) maxtile = std::max(maxtile, L.ntile[l]);   // (larger chunks never run it)
    int tp, nt;
    attn_tiles((int64_t)(80 >> l) * (T >> l), 32, tp, nt);   // the throughput plan takes at most 32
    maxtile = std::max(maxtile, nt);
  }
  L.part = take((size_t)B * maxtile * 4 * 1088 * 4);
  L.G = take((size_t)B * 128 * 256 * 4);
  L.Mw = take((size_t)B * conv_wimg(dt, 1, 256, 256).total);
  L.tb = take((size_t)std::max<int64_t>(B, N) * 1792 * 4);
  L.spk = take((size_t)B * 80 * 4);
  L.betas = take((size_t)std::max<int32_t>(N, 1) * 4);
  L.step = take(4);
  if (small && dt && sk_target > 0) {
    // 128-wide 3x3 tiles of levels 1-2 (at most 2 x 128 output channels): one counter per tile; conv_small_ksplit
    // splits an utterance's tiles only while tiles x splits <= sk_target (and at most 4 ways), so its fp32 partials
    // (8192 floats per split tile) need B x min(sk_target, 4 x tiles) slabs, not 4 x every tile (Run::conv3_stats
    // checks each launch against both sizes)
    const long tiles = 40L * (((T >> 1) + 63) / 64) * 2;
    L.skcnt_n = (long)B * tiles;
    L.skpart_n = (long)B * std::min<long>(sk_target, 4 * tiles) * 8192;
    L.skcnt = take((size_t)L.skcnt_n * 4);
    L.skpart = take((size_t)L.skpart_n * 4);
  }
  L.total = o;
  return L;
}

// ---------------------------------------------------------------- one U-Net evaluation
struct Run {
  gt_decoder* d;
  int dt;       // activation dtype: 0 fp32, 1 bf16
  int wi;       // compute dtype code (GT_F32 / GT_BF16 / GT_BF16_W8 / GT_FP8) = packed arena index
  int B, T;
  hipStream_t s;
  uint8_t* ws;
  Layout L;
  const float* mask; const float* mu; const float* xt; const float* spk_s;
  const float* tb; long tb_bstride;
  const int* stepp = nullptr;     // device step index of graph segments (kernels.h tb_at); null = 0
  const float* betas = nullptr;   // per-step beta(t) table (sampler), indexed by *stepp
  int small = 0;                  // small-batch tile plan (small_plan)
  int stat_slot = 0;
  hipError_t err = hipSuccess;
  const char* probe = nullptr;   // diagnostics: copy the activation named `probe` to probe_out (NCHW fp32)
  float* probe_out = nullptr;
  bool probed = false;

  template <class Fn>
  void timed(const std::string& kernel, double flop, double bytes, Fn&& fn) {
    if (!d->prof || (!d->prof_prefix.empty() && kernel.compare(0, d->prof_prefix.size(), d->prof_prefix) != 0)) {
      chk(fn());
      return;
    }
    hipEvent_t e0 = d->ev(), e1 = d->ev();
    if (e0) chk(hipEventRecord(e0, s));
    chk(fn());
    if (e1) chk(hipEventRecord(e1, s));
    if (e0 && e1) d->recs.push_back({kernel, flop, bytes, e0, e1});
  }

  // conv launch with its algorithmic FLOPs (the reference's conv MACs x 2) and compulsory HBM bytes
  void conv(ConvKind kind, InMode im, OutMode om, const ConvParams& p) {
    const double es = (double)esize(dt);
    const double pin = (double)p.B * p.Fin * p.Tin, pout = (double)p.B * p.Fout * p.Tout;
    const int taps = kind == CONV1 ? 1 : 9;
    double flop = kind == CONVT4 ? 2.0 * p.Cin * p.Cout * 16 * pin : 2.0 * p.Cin * p.Cout * taps * pout;
    double bytes = (im == IN_INPUT ? pin * p.Cin * 4.0 : pin * p.Cin * es) + pout * p.Cout * es +
                   (double)p.Cout * (kind == CONVT4 ? 16 : taps) * p.Cin_pad * (p.wscale ? 1.0 : es) * (p.w_bstride ? p.B : 1);
    if (om == OUT_RBOUT || om == OUT_RESID) bytes += pout * p.Cout * es;
    // "<instantiation as rocprof names it>@<shape>": bench.py aggregates per instantiation
    const int nt = dt ? conv_nt(1, p.Cout) : 64;
    if (kind == CONV1 && dt && d->conv1s && conv1s_eligible(im, om, p)) {
      const std::string name = "conv1s_kernel<" + std::to_string((int)im) + "," + std::to_string((int)om) + "," +
                               std::to_string(nt) + ">@" + std::to_string(p.Cin) + "x" + std::to_string(p.Cout) + "x" +
                               std::to_string(p.Fout);
      timed(name, flop, bytes, [&] { return launch_conv1s(im, om, p, s); });
      return;
    }
    const int tf = (dt && !(p.a8 && !p.small)) ? conv_tf(kind, im, nt, p.Cout, p.Fout, p.small) : 4;
    const std::string name = std::string("conv_kernel<") + (dt ? "bf16" : "float") + "," + std::to_string((int)kind) +
                             "," + std::to_string((int)im) + "," + std::to_string((int)om) + "," + std::to_string(nt) +
                             (p.a8 ? ",a8" : p.wscale ? ",w8" : "") + (tf != 4 ? ",tf" + std::to_string(tf) : "") + ">@" + std::to_string(p.Cin) + "x" + std::to_string(p.Cout) + "x" + std::to_string(p.Fout);
    timed(name, flop, bytes, [&] { return launch_conv(dt, kind, im, om, p, s); });
  }

  // 3x3 stride-1 conv with GroupNorm partial sums of the output; returns the number of partial slots per
  // utterance it wrote. bf16-operand 64 -> 64 convs (bf16 or fp8 weights; GT_FP8 too) take conv64 (weight-resident),
  // everything else conv_kernel.
  int conv3_stats(InMode im, ConvParams p, const std::string& wkey) {
    if (pend0.on) {   // the first ResnetBlock's output is pending: formed here if this conv reads it, else by its pass
      if (im == IN_MASK && p.in0 == pend0.out && !p.in1 && dt && conv64_eligible(p) && d->dp[wi].count(wkey + ".w64")) {
        p.w = W(wkey + ".w64");   // (fp8 weights: their e4m3 values, p.wscale the per-channel scale; bf16 operands)
        p.a8 = 0;
        p.in0 = pend0.pre;
        p.gn_part = pend0.part; p.gn_nparts = pend0.nparts; p.gn_gamma = pend0.gamma; p.gn_beta = pend0.beta;
        p.gn_count = pend0.count;
        p.cin_input = pend0.cin; p.rb_w = pend0.rw; p.rb_b = pend0.rb; p.rb_out = pend0.out;
        const double pos = (double)p.B * p.Fout * p.Tout;
        const int np = conv64_nparts(p.Fout, p.Tout, p.small);
        if (np > L.pmax) { chk(hipErrorInvalidValue); return np; }
        pend0.on = false;
        timed(std::string("conv64_kernel<4") + (p.wscale ? ",w8" : "") + ">@64x64x" + std::to_string(p.Fout), 2.0 * 64 * 64 * 9 * pos + 2.0 * pend0.cin * 64 * pos,
              pos * (3 * 128.0 + 8.0) + 64.0 * 9 * 64 * 2, [&] { return launch_conv64(IN_RB0, p, s); });
        tap(pend0.name, pend0.lvl, pend0.out, 64);   // r0 is in place from here on
        return np;
      }
      flush_rb0();
    }
    if (dt && d->conv64 && (im == IN_MASK || im == IN_GN || im == IN_PLAIN) && conv64_eligible(p) &&
        d->dp[wi].count(wkey + ".w64")) {
      p.w = W(wkey + ".w64");   // (fp8 weights: their e4m3 values; p.wscale stays the per-channel scale)
      p.a8 = 0;
      const double pos = (double)p.B * p.Fout * p.Tout;
      const int np = conv64_nparts(p.Fout, p.Tout, p.small);
      if (np > L.pmax) { chk(hipErrorInvalidValue); return np; }   // would spill into the next stats slot
      timed(std::string("conv64_kernel<") + std::to_string((int)im) + (p.wscale ? ",w8" : "") + ">@64x64x" +
                std::to_string(p.Fout),
            2.0 * 64 * 64 * 9 * pos, pos * 128 * 2.0 + 64.0 * 9 * 64 * 2, [&] { return launch_conv64(im, p, s); });
      return np;
    }
    if (dt && (wi == GT_BF16 || wi == GT_BF16_W8) && d->wide && conv3w_eligible(p, im) && d->dp[wi].count(wkey + ".w3w")) {
      p.w = W(wkey + ".w3w");
      const int np = conv3w_nparts(p.Fout, p.Tout, p.Cout);
      if (np <= 0 || np > L.pmax) { chk(hipErrorInvalidValue); return np; }
      const double pos = (double)p.B * p.Fout * p.Tout;
      const int cb = (p.Cout == 256 || (p.Cout == 128 && p.Fout % 20 == 0 && p.Fout >= 40)) ? 2 : 1;
      timed(std::string("conv3w_kernel<") + std::to_string((int)im) + "," + std::to_string(p.Cout) + "," +
                std::to_string(cb) + (p.wscale ? ",w8" : "") + ">@" + std::to_string(p.Cin) + "x" + std::to_string(p.Cout) +
                "x" + std::to_string(p.Fout),
            2.0 * p.Cin * p.Cout * 9 * pos, pos * (p.Cin + p.Cout) * 2.0 + 9.0 * p.Cin * p.Cout * 2,
            [&] { return launch_conv3w(im, p, s); });
      return np;
    }
    if (dt && wi == GT_FP8 && d->wide && d->wide_a8 && conv3w_a8_eligible(p, im) && d->dp[wi].count(wkey + ".w3a")) {
      p.w = W(wkey + ".w3a");   // (p.wscale: the per-channel scale of the e4m3 codes, shared with conv_kernel's image)
      const int np = conv3w_nparts(p.Fout, p.Tout, p.Cout);
      if (np <= 0 || np > L.pmax) { chk(hipErrorInvalidValue); return np; }
      const double pos = (double)p.B * p.Fout * p.Tout;
      const int cb = (p.Cout == 256 || (p.Cout == 128 && p.Fout % 20 == 0 && p.Fout >= 40)) ? 2 : 1;
      timed(std::string("conv3w_a8_kernel<") + std::to_string((int)im) + "," + std::to_string(p.Cout) + "," +
                std::to_string(cb) + ">@" + std::to_string(p.Cin) + "x" + std::to_string(p.Cout) + "x" + std::to_string(p.Fout),
            2.0 * p.Cin * p.Cout * 9 * pos, pos * (p.Cin + p.Cout) * 2.0 + 9.0 * p.Cin * p.Cout,
            [&] { return launch_conv3w_a8(im, p, s); });
      return np;
    }
    const int np = conv_gn_nparts(dt, im, p.Fout, p.Tout, p.Cout, p.small, p.a8);
    if (np > L.pmax) { chk(hipErrorInvalidValue); return np; }
    if (small && dt && p.Cout % 128 == 0 && im != IN_INPUT && L.skcnt_n) {   // split-K (conv.hip ConvCfg::SK)
      p.ksplit = conv_small_ksplit(p.Fout, p.Tout, p.Cout, p.Cin_pad, d->sk_target, p.a8);
      const long tiles = (long)p.B * p.Fout * ((p.Tout + 63) / 64) * (p.Cout / 128);
      if (p.ksplit > 1 && (tiles > L.skcnt_n || tiles * p.ksplit * 8192 > L.skpart_n)) { chk(hipErrorInvalidValue); return np; }
      p.sk_part = (float*)(ws + L.skpart); p.sk_cnt = (int*)(ws + L.skcnt);
    }
    conv(CONV3, im, OUT_STATS, p);
    return np;
  }

  // diagnostics: "gnpart.<k>" copies GroupNorm partial slot k (B x pmax x 16 floats) after the launch that
  // produced it
  void tap_part(int k) {
    if (probe && !probed && std::string(probe) == "gnpart." + std::to_string(k)) {
      chk(hipMemcpyAsync(probe_out, ws + L.stats + (size_t)k * B * L.pmax * 16 * sizeof(float),
                         (size_t)B * L.pmax * 16 * sizeof(float), hipMemcpyDeviceToDevice, s));
      probed = true;
    }
  }

  void tap(const std::string& name, int lvl, const void* buf, int C) {
    if (probe && !probed && name == probe) {
      chk(launch_to_nchw(dt, buf, B, Fl(lvl), Tl(lvl), C, probe_out, s));
      probed = true;
    }
  }

  // downs.0.0 on the fused input-conv path (conv64 IN_X0 + x0_stats): bf16 weights and activations, two input channels
  bool x0_fused(const std::string& k, int lvl, int cin, int Cout) {
    if (!(d->x0_fuse && dt && (wi == GT_BF16 || wi == GT_BF16_W8 || wi == GT_FP8) && d->conv64 && cin == 2 && Cout == 64 && Fl(lvl) % 20 == 0 &&
          d->dp[wi].count(k + "block1.block.0.weight.x0") && d->dp[wi].count(k + "block2.block.0.weight.w64")))
      return false;
    ConvParams p = base(lvl, lvl);
    p.Cin = p.C0 = p.Cin_pad = Cout; p.Cout = Cout; p.cin_input = cin; p.mu = mu; p.xt = xt;
    p.x0w = W(k + "block1.block.0.weight.x0"); p.x0b = Fp(k + "block1.block.0.bias");
    return x0_eligible(p) && conv64_eligible(p);
  }
  const float* x0_scale(const std::string& k) {   // the input conv's fp8 scale (fp8-weight modes), else null
    const auto it = d->dp[wi].find(k + "block1.block.0.weight.s");
    return it != d->dp[wi].end() ? (const float*)it->second : nullptr;
  }
  void* W(const std::string& k) { return d->dp[wi].at(k); }
  const float* Fp(const std::string& k) { return (const float*)d->dp[wi].at(k); }
  // weight image of a conv: its fp8 scales too when the image is fp8 (GT_BF16_W8, GT_FP8), and the fp8-operand flag
  void setw(ConvParams& p, const std::string& k) {
    p.w = W(k);
    const auto it = d->dp[wi].find(k + ".s");
    p.wscale = it != d->dp[wi].end() ? (const float*)it->second : nullptr;
    p.a8 = d->dp[wi].count(k + ".a8") ? 1 : 0;
  }
  void* act(int l, int i) { return ws + L.act[l][i]; }
  float* stats() { return (float*)(ws + L.stats) + (size_t)(stat_slot++) * B * L.pmax * 16; }
  int Fl(int l) const { return 80 >> l; }
  int Tl(int l) const { return T >> l; }
  void chk(hipError_t e) { if (err == hipSuccess && e != hipSuccess) err = e; }

  ConvParams base(int lvl_in, int lvl_out) {
    ConvParams p;
    memset(&p, 0, sizeof(p));
    p.B = B; p.T0 = T; p.mask = mask; p.stepp = stepp;
    p.Fin = Fl(lvl_in); p.Tin = Tl(lvl_in); p.Fout = Fl(lvl_out); p.Tout = Tl(lvl_out);
    p.lvl_in = lvl_in; p.lvl_out = lvl_out;
    p.small = small;
    return p;
  }

  // ResnetBlock (diffusion.py:61-79). `in1` != null: channel concat (up path). in0 == null: U-Net input.
  // Identity-residual ResnetBlock output held back for the attention that consumes it (attn_kv forms it in its
  // operand load and writes it to `out`): see resnet(..., defer) and attention().
  struct PendingRb {
    bool on = false;
    std::string name;
    const void* pre; const float* part; int nparts; const float* gamma; const float* beta; long count;
    const void* x; void* out;
  } pend;
  // The first ResnetBlock's output r0 = Mish(GN(h2))*m + res_conv(x*m) held back for downs.0.1's block1 conv, which
  // forms it in its operand load and writes it (conv64 IN_RB0, conv3_stats); any other next step runs its pass first
  // (flush_rb0: rbout_input_kernel).
  struct PendingRb0 {
    bool on = false;
    std::string name;
    const void* pre; const float* part; int nparts; const float* gamma; const float* beta; long count;
    void* out; const float* rw; const float* rb; int cin, lvl, C;
  } pend0;
  void flush_rb0() {
    if (!pend0.on) return;
    pend0.on = false;
    const int lvl = pend0.lvl;
    RbOutParams p{};
    p.pre = pend0.pre; p.part = pend0.part; p.nparts = pend0.nparts; p.gamma = pend0.gamma; p.beta = pend0.beta;
    p.count = pend0.count; p.out = pend0.out; p.mask = mask; p.B = B; p.F = Fl(lvl); p.T = Tl(lvl); p.C = pend0.C;
    p.T0 = T; p.lvl = lvl; p.mu = mu; p.xt = xt; p.spk_s = spk_s; p.cin = pend0.cin; p.rw = pend0.rw; p.rb = pend0.rb;
    const double by = (2.0 * pend0.C * esize(dt) + 8.0) * B * Fl(lvl) * Tl(lvl);
    timed(std::string("rbout_input_kernel<") + (dt ? "bf16>" : "float>") + "@" + std::to_string(pend0.C) + "x" +
              std::to_string(Fl(lvl)), 2.0 * pend0.cin * pend0.C * B * Fl(lvl) * Tl(lvl), by,
          [&] { return launch_rbout_input(dt, p, s); });
    tap(pend0.name, lvl, pend0.out, pend0.C);
  }

  void resnet(const std::string& k, int lvl, const void* in0, int C0, const void* in1, int C1, int Cout, void* out,
              int tb_off, bool defer = false) {
    const bool input = (in0 == nullptr);
    const int cin = input ? (d->n_spks > 1 ? 3 : 2) : C0 + C1;
    void* pre1 = act(lvl, 3);
    void* pre2 = act(lvl, 4);
    float* st1 = stats();
    float* st2 = stats();
    int np1 = 0, np2 = 0;                         // GroupNorm partial slots written by block1 / block2
    const long count = (long)(Cout / 8) * Fl(lvl) * Tl(lvl);
    if (input && x0_fused(k, lvl, cin, Cout)) {
      // block1's output h1 is never written: its GroupNorm statistics come from a statistics-only recompute (x0_stats)
      // and block2's conv recomputes h1 itself in its operand load (conv64 IN_X0) -- the same MFMA instructions on the
      // same operands, so the statistics are those of the values it transforms
      ConvParams p = base(lvl, lvl);
      p.Cin = cin; p.Cout = Cout; p.cin_input = cin; p.mu = mu; p.xt = xt;
      p.x0w = W(k + "block1.block.0.weight.x0"); p.x0b = Fp(k + "block1.block.0.bias"); p.x0s = x0_scale(k);
      p.out_part = st1;
      p.out = (probe && std::string(probe) == k + "pre1") ? pre1 : nullptr;   // diagnostics: bf16(h1)
      np1 = x0_stats_nparts(Fl(lvl), Tl(lvl));
      if (np1 > L.pmax) { chk(hipErrorInvalidValue); return; }
      const double pos = (double)B * Fl(lvl) * Tl(lvl);
      timed("x0_stats_kernel@2x64x" + std::to_string(Fl(lvl)), 2.0 * cin * Cout * 9 * pos, pos * (2 * 4.0 + 4.0),
            [&] { return launch_x0_stats(p, s); });
      tap(k + "pre1", lvl, pre1, Cout);
      tap_part(stat_slot - 2);
      ConvParams q = base(lvl, lvl);
      q.Cin = Cout; q.Cout = Cout; q.Cin_pad = 64; q.C0 = Cout; q.in0 = nullptr;
      q.cin_input = cin; q.mu = mu; q.xt = xt; q.x0w = p.x0w; q.x0b = p.x0b; q.x0s = p.x0s;
      q.gn_part = st1; q.gn_nparts = np1; q.gn_gamma = Fp(k + "block1.block.1.weight"); q.gn_beta = Fp(k + "block1.block.1.bias");
      q.gn_count = count; q.tb = tb + tb_off; q.tb_bstride = tb_bstride;
      setw(q, k + "block2.block.0.weight"); q.bias = Fp(k + "block2.block.0.bias");
      q.w = W(k + "block2.block.0.weight.w64");
      q.out = pre2; q.out_part = st2;
      np2 = conv64_nparts(q.Fout, q.Tout, q.small);
      if (np2 > L.pmax) { chk(hipErrorInvalidValue); return; }
      timed(std::string("conv64_kernel<5") + (q.wscale ? ",w8" : "") + ">@64x64x" + std::to_string(Fl(lvl)), 2.0 * 64 * 64 * 9 * pos + 2.0 * cin * Cout * 9 * pos,
            pos * (2 * 4.0 + 4.0 + 128.0) + 64.0 * 9 * 64 * 2, [&] { return launch_conv64(IN_X0, q, s); });
      tap(k + "pre2", lvl, pre2, Cout);
      tap_part(stat_slot - 1);
    } else {
    {   // block1 conv on x*mask
      ConvParams p = base(lvl, lvl);
      p.Cin = cin; p.Cout = Cout; p.Cin_pad = d->cinpad[wi].at(k + "block1.block.0.weight");
      p.in0 = in0; p.C0 = C0; p.in1 = in1; p.C1 = C1;
      p.mu = mu; p.xt = xt; p.spk_s = spk_s; p.cin_input = cin;
      setw(p, k + "block1.block.0.weight"); p.bias = Fp(k + "block1.block.0.bias");
      p.out = pre1; p.out_part = st1;
      if (input) {
        np1 = conv_gn_nparts(dt, IN_INPUT, Fl(lvl), Tl(lvl), Cout, small);
        if (np1 > L.pmax) { chk(hipErrorInvalidValue); return; }
        conv(CONV3, IN_INPUT, OUT_STATS, p);
      } else {
        np1 = conv3_stats(IN_MASK, p, k + "block1.block.0.weight");
      }
      tap(k + "pre1", lvl, pre1, Cout);
      tap_part(stat_slot - 2);
    }
    {   // block2 conv on (Mish(GN(h1))*m + tb)*m: the transform in the conv's operand load (IN_GN). (Round 1 ran it as a
        // separate in-place pass at 256 channels; since round 2 the operand-load form is faster everywhere.)
      ConvParams p = base(lvl, lvl);
      p.Cin = Cout; p.Cout = Cout; p.Cin_pad = d->cinpad[wi].at(k + "block2.block.0.weight");
      p.in0 = pre1; p.C0 = Cout;
      p.gn_part = st1; p.gn_nparts = np1; p.gn_gamma = Fp(k + "block1.block.1.weight"); p.gn_beta = Fp(k + "block1.block.1.bias");
      p.gn_count = count; p.tb = tb + tb_off; p.tb_bstride = tb_bstride;
      setw(p, k + "block2.block.0.weight"); p.bias = Fp(k + "block2.block.0.bias");
      p.out = pre2; p.out_part = st2;
      np2 = conv3_stats(IN_GN, p, k + "block2.block.0.weight");
      tap(k + "pre2", lvl, pre2, Cout);
      tap_part(stat_slot - 1);
    }
    }
    if (d->index.count(k + "res_conv.weight") && input) {
      // the first block (2-3 input channels): Mish(GN(h2))*m + res_conv(x*m), formed by the next block's conv
      // (conv64 IN_RB0) on the bf16 path, else as an elementwise pass (flush_rb0; a 1x1 conv_kernel over 2-3 channels
      // measured slower: 100.4 vs 86.3 us, round 3)
      pend0.on = true; pend0.name = k.substr(0, k.size() - 1);
      pend0.pre = pre2; pend0.part = st2; pend0.nparts = np2; pend0.gamma = Fp(k + "block2.block.1.weight");
      pend0.beta = Fp(k + "block2.block.1.bias"); pend0.count = count; pend0.out = out;
      pend0.rw = Fp(k + "res_conv.weight.f32"); pend0.rb = Fp(k + "res_conv.bias"); pend0.cin = cin; pend0.lvl = lvl;
      pend0.C = Cout;
      if (!(dt && d->rb0_fuse && d->conv64 && Cout == 64)) flush_rb0();
      return;
    } else if (d->index.count(k + "res_conv.weight")) {   // Mish(GN(h2))*m + res_conv(x*m)
      ConvParams p = base(lvl, lvl);
      p.Cin = cin; p.Cout = Cout; p.Cin_pad = d->cinpad[wi].at(k + "res_conv.weight");
      p.in0 = in0; p.C0 = C0; p.in1 = in1; p.C1 = C1;
      p.mu = mu; p.xt = xt; p.spk_s = spk_s; p.cin_input = cin;
      p.w = W(k + "res_conv.weight"); p.bias = Fp(k + "res_conv.bias");
      p.pre = pre2; p.pre_part = st2; p.pre_nparts = np2; p.pre_gamma = Fp(k + "block2.block.1.weight");
      p.pre_beta = Fp(k + "block2.block.1.bias"); p.pre_count = count;
      p.out = out;
      conv(CONV1, input ? IN_INPUT : IN_MASK, OUT_RBOUT, p);
    } else if (defer) {                            // Mish(GN(h2))*m + x*m, formed by the next attn_kv
      pend.on = true; pend.name = k.substr(0, k.size() - 1);
      pend.pre = pre2; pend.part = st2; pend.nparts = np2; pend.gamma = Fp(k + "block2.block.1.weight");
      pend.beta = Fp(k + "block2.block.1.bias"); pend.count = count; pend.x = in0; pend.out = out;
      return;
    } else {                                       // Mish(GN(h2))*m + x*m
      RbOutParams p{};
      p.pre = pre2; p.part = st2; p.nparts = np2; p.gamma = Fp(k + "block2.block.1.weight"); p.beta = Fp(k + "block2.block.1.bias");
      p.count = count; p.x = in0; p.out = out; p.mask = mask; p.B = B; p.F = Fl(lvl); p.T = Tl(lvl); p.C = Cout;
      p.T0 = T; p.lvl = lvl;
      const double by = 3.0 * B * Fl(lvl) * Tl(lvl) * Cout * esize(dt);
      timed(std::string("rbout_identity_kernel<") + (dt ? "bf16>" : "float>") + "@" + std::to_string(Cout) + "x" +
                std::to_string(Fl(lvl)), 0.0, by,
            [&] { return launch_rbout_identity(dt, p, s); });
    }
    tap(k.substr(0, k.size() - 1), lvl, out, Cout);
  }

  // Residual(Rezero(LinearAttention)) (diffusion.py:82-110)
  void attention(const std::string& k, int lvl, const void* in, int C, void* out) {
    attention_fold(k, lvl, in, C);
    attention_out(k, lvl, in, C, out);
  }

  // level 0: the attention output and the Downsample after it as one pass (attn_down.hip; the attention output is
  // never materialised). false (nothing launched) when not applicable: another dtype, the fused form disabled
  // (GT_ATTN_DS=0), or a probe of the attention output itself.
  bool attention_down(const std::string& ka, const std::string& kd, int lvl, const void* in, int C, void* out) {
    if (!(dt && d->attn_ds && lvl == 0 && d->dp[wi].count(kd + "conv.weight.wfr"))) return false;
    if (probe && std::string(probe) == ka.substr(0, ka.size() - 1)) return false;
    AttnDownParams a{};
    a.x = in; a.B = B; a.F = Fl(lvl); a.T = Tl(lvl); a.C = C; a.T0 = T; a.mask = mask; a.lvl = lvl;
    a.mw = ws + L.Mw; a.mw_bstride = conv_wimg(dt, 1, C, C).total; a.gb = Fp(ka + "fn.fn.to_out.bias.g");
    a.wds = W(kd + "conv.weight.wfr"); a.bds = Fp(kd + "conv.bias"); a.out = out;
    a.wsc = d->dp[wi].count(kd + "conv.weight.s") ? Fp(kd + "conv.weight.s") : nullptr;   // fp8 weights
    if (!attn_down_eligible(a)) return false;
    attention_fold(ka, lvl, in, C);
    const double pin = (double)B * a.F * a.T, pout = pin / 4;
    timed(std::string("attn_down_kernel<bf16") + (a.wsc ? ",w8" : "") + ">@" + std::to_string(C) + "x" + std::to_string(Fl(lvl)),
          2.0 * C * C * pin + 2.0 * C * C * 9 * pout, (pin + pout) * C * 2.0, [&] { return launch_attn_down(a, s); });
    tap(kd.substr(0, kd.size() - 1), lvl + 1, out, C);
    return true;
  }

  // attn_kv + merge/fold: M_b for every utterance in the workspace (the ResnetBlock output before it formed on the way)
  // ups.1: the attention output and the Upsample after it as one pass (attn_up.hip); false (nothing launched) when not
  // applicable: another dtype, disabled (GT_ATTN_US=0), or a probe of the attention output
  bool attention_up(const std::string& ka, const std::string& ku, int lvl, const void* in, int C, void* out) {
    if (!(dt && d->attn_us && d->dp[wi].count(ku + "conv.weight.wfr"))) return false;
    if (probe && std::string(probe) == ka.substr(0, ka.size() - 1)) return false;
    AttnUpParams a{};
    a.x = in; a.B = B; a.F = Fl(lvl); a.T = Tl(lvl); a.C = C; a.T0 = T; a.mask = mask; a.lvl = lvl;
    a.mw = ws + L.Mw; a.mw_bstride = conv_wimg(dt, 1, C, C).total; a.gb = Fp(ka + "fn.fn.to_out.bias.g");
    a.wup = W(ku + "conv.weight.wfr"); a.bup = Fp(ku + "conv.bias"); a.out = out;
    a.wsc = d->dp[wi].count(ku + "conv.weight.s") ? Fp(ku + "conv.weight.s") : nullptr;   // fp8 weights
    if (!attn_up_eligible(a)) return false;
    attention_fold(ka, lvl, in, C);
    const double pin = (double)B * a.F * a.T, pout = pin * 4;
    timed(std::string("attn_up_kernel<bf16") + (a.wsc ? ",w8" : "") + ">@" + std::to_string(C) + "x" + std::to_string(Fl(lvl)),
          2.0 * C * C * pin + 2.0 * C * C * 16 * pin, (pin + pout) * C * 2.0, [&] { return launch_attn_up(a, s); });
    tap(ku.substr(0, ku.size() - 1), lvl - 1, out, C);
    return true;
  }

  void attention_fold(const std::string& k, int lvl, const void* in, int C) {
    flush_rb0();   // (defensive: only downs.0.1's block1 conv ever consumes the pending first-block output)
    float* part = (float*)(ws + L.part);
    float* G = (float*)(ws + L.G);
    void* Mw = ws + L.Mw;
    AttnKVParams a;
    a.x = in; a.B = B; a.n = Fl(lvl) * Tl(lvl); a.C = C; a.Cpad = C;
    a.wkv = W(k + "fn.fn.to_qkv.weight");
    a.part = part;
    if (small) {
      a.tile_pos = L.tile_pos[lvl]; a.ntile = L.ntile[lvl];
    } else {
      attn_tiles(a.n, a.n >= 8192 ? 16 : 32, a.tile_pos, a.ntile);   // never more tiles than the workspace holds
    }
    a.rb_pre = nullptr;
    const bool rb = pend.on;
    if (rb) {   // the preceding ResnetBlock's output is formed here and written to `in`
      if (pend.out != in) { chk(hipErrorInvalidValue); return; }
      a.x = pend.x; a.rb_pre = pend.pre; a.rb_part = pend.part; a.rb_nparts = pend.nparts; a.rb_gamma = pend.gamma;
      a.rb_beta = pend.beta; a.rb_count = pend.count; a.rb_out = pend.out; a.mask = mask; a.T = Tl(lvl); a.T0 = T;
      a.lvl = lvl;
      pend.on = false;
    }
    const double npos = (double)B * a.n;
    // reference FLOPs of the attention block: qkv 1x1 (2*C*384) + two einsums (2 * 2*4*32*32) + to_out (2*128*C)
    // label = the template instantiation (launch_attn_kv: all C channels resident in LDS for C <= 64, else chunked)
    timed(std::string("attn_kv_kernel<") + (dt ? "bf16" : "float") + (C <= 64 ? ",res" : ",chunk") + (rb ? ",rb>" : ">") +
              "@" + std::to_string(C) +
              "x" + std::to_string(Fl(lvl)), npos * (2.0 * C * 256 + 2.0 * 4 * 32 * 32),
          npos * C * esize(dt) * (rb ? 3.0 : 1.0), [&] { return launch_attn_kv(dt, a, s); });
    if (rb) tap(pend.name, lvl, in, C);
    timed("attn_merge_kernel@" + std::to_string(C), 0.0, 0.0, [&] {
      return launch_attn_merge(part, B, a.ntile, Fp(k + "fn.fn.to_out.weight"), Fp(k + "fn.g"), C, G,
                               small ? d->merge_dr_small : 32, s);
    });
    timed(std::string("attn_fold_kernel<") + (dt ? "bf16>" : "float>") + "@" + std::to_string(C), 2.0 * B * C * 128.0 * C, 0.0,
          [&] { return launch_attn_fold(dt, G, Fp(k + "fn.fn.to_qkv.weight.qT"), B, C, Mw, s); });
  }

  void attention_out(const std::string& k, int lvl, const void* in, int C, void* out) {   // y = x + M_b x + g b_out
    void* Mw = ws + L.Mw;
    ConvParams p = base(lvl, lvl);
    p.Cin = C; p.Cout = C; p.Cin_pad = C;
    p.in0 = in; p.C0 = C;
    p.w = Mw; p.w_bstride = conv_wimg(dt, 1, C, C).total; p.bias = Fp(k + "fn.fn.to_out.bias.g");
    p.out = out;
    conv(CONV1, IN_PLAIN, OUT_RESID, p);
    tap(k.substr(0, k.size() - 1), lvl, out, C);
  }

  void downsample(const std::string& k, int lvl, const void* in, int C, void* out) {   // diffusion.py:30-36
    ConvParams p = base(lvl, lvl + 1);
    p.Cin = C; p.Cout = C; p.Cin_pad = d->cinpad[wi].at(k + "conv.weight");
    p.in0 = in; p.C0 = C;
    setw(p, k + "conv.weight"); p.bias = Fp(k + "conv.bias"); p.out = out;
    conv(CONV3_S2, IN_MASK, OUT_PLAIN, p);
    tap(k.substr(0, k.size() - 1), lvl + 1, out, C);
  }

  void upsample(const std::string& k, int lvl, const void* in, int C, void* out) {     // diffusion.py:21-27
    ConvParams p = base(lvl, lvl - 1);
    p.Cin = C; p.Cout = C; p.Cin_pad = d->cinpad[wi].at(k + "conv.weight");
    p.in0 = in; p.C0 = C;
    setw(p, k + "conv.weight"); p.bias = Fp(k + "conv.bias"); p.out = out;
    conv(CONVT4, IN_MASK, OUT_PLAIN, p);
    tap(k.substr(0, k.size() - 1), lvl - 1, out, C);
  }

  // GradLogPEstimator2d.forward body; final stage either writes the score or does the Euler update.
  void unet(int euler, float* out, float* xt_inout, float beta_t, float hstep) {
    stat_slot = 0;
    int tb_off = 0;
    auto next_tb = [&](int c) { int o = tb_off; tb_off += c; return o; };
    // down 0 (80 x T, 64 ch)
    resnet("downs.0.0.", 0, nullptr, 0, nullptr, 0, 64, act(0, 0), next_tb(64));
    resnet("downs.0.1.", 0, act(0, 0), 64, nullptr, 0, 64, act(0, 1), next_tb(64), true);
    if (!attention_down("downs.0.2.", "downs.0.3.", 0, act(0, 1), 64, act(1, 0))) {
      attention("downs.0.2.", 0, act(0, 1), 64, act(0, 0));
      downsample("downs.0.3.", 0, act(0, 0), 64, act(1, 0));
    }
    // down 1 (40 x T/2, 128 ch); hidden 1 -> act(1,2)
    resnet("downs.1.0.", 1, act(1, 0), 64, nullptr, 0, 128, act(1, 1), next_tb(128));
    resnet("downs.1.1.", 1, act(1, 1), 128, nullptr, 0, 128, act(1, 0), next_tb(128), true);
    attention("downs.1.2.", 1, act(1, 0), 128, act(1, 2));
    downsample("downs.1.3.", 1, act(1, 2), 128, act(2, 0));
    // down 2 (20 x T/4, 256 ch); hidden 2 -> act(2,2); Identity(x*mask) is absorbed by the next block's mask
    resnet("downs.2.0.", 2, act(2, 0), 128, nullptr, 0, 256, act(2, 1), next_tb(256));
    resnet("downs.2.1.", 2, act(2, 1), 256, nullptr, 0, 256, act(2, 0), next_tb(256), true);
    attention("downs.2.2.", 2, act(2, 0), 256, act(2, 2));
    // mid
    resnet("mid_block1.", 2, act(2, 2), 256, nullptr, 0, 256, act(2, 0), next_tb(256), true);
    attention("mid_attn.", 2, act(2, 0), 256, act(2, 1));
    resnet("mid_block2.", 2, act(2, 1), 256, nullptr, 0, 256, act(2, 0), next_tb(256));
    // up 0 at level 2: cat(x, hidden2) -> 128 ch, then ConvTranspose to level 1
    resnet("ups.0.0.", 2, act(2, 0), 256, act(2, 2), 256, 128, act(2, 1), next_tb(128));
    resnet("ups.0.1.", 2, act(2, 1), 128, nullptr, 0, 128, act(2, 0), next_tb(128), true);
    attention("ups.0.2.", 2, act(2, 0), 128, act(2, 1));
    upsample("ups.0.3.", 2, act(2, 1), 128, act(1, 0));
    // up 1 at level 1: cat(x, hidden1) -> 64 ch, then ConvTranspose to level 0
    resnet("ups.1.0.", 1, act(1, 0), 128, act(1, 2), 128, 64, act(1, 1), next_tb(64));
    resnet("ups.1.1.", 1, act(1, 1), 64, nullptr, 0, 64, act(1, 0), next_tb(64), true);
    if (!attention_up("ups.1.2.", "ups.1.3.", 1, act(1, 0), 64, act(0, 0))) {
      attention("ups.1.2.", 1, act(1, 0), 64, act(1, 1));
      upsample("ups.1.3.", 1, act(1, 1), 64, act(0, 0));
    }
    // final_block conv (+GN sums), then the fused GN/Mish/final_conv/(Euler) kernel
    float* st = stats();
    int fnp = 0;
    {
      ConvParams p = base(0, 0);
      p.Cin = 64; p.Cout = 64; p.Cin_pad = d->cinpad[wi].at("final_block.block.0.weight");
      p.in0 = act(0, 0); p.C0 = 64;
      setw(p, "final_block.block.0.weight"); p.bias = Fp("final_block.block.0.bias");
      p.out = act(0, 3); p.out_part = st;
      fnp = conv3_stats(IN_MASK, p, "final_block.block.0.weight");
      tap("final_block.pre", 0, act(0, 3), 64);
    }
    FinalParams f;
    f.pre = act(0, 3); f.part = st; f.nparts = fnp; f.gamma = Fp("final_block.block.1.weight"); f.beta = Fp("final_block.block.1.bias");
    f.count = (long)8 * 80 * T; f.wf = Fp("final_conv.weight"); f.bf = Fp("final_conv.bias");
    f.mask = mask; f.B = B; f.T = T; f.euler = euler; f.out = out; f.mu = mu; f.xt = xt_inout;
    f.beta_t = beta_t; f.hstep = hstep; f.betas = betas; f.stepp = stepp;
    timed(std::string("final_kernel<") + (dt ? "bf16>" : "float>"), 2.0 * 64 * B * 80 * T,
          (double)B * 80 * T * (64 * esize(dt) + 16), [&] { return launch_final(dt, f, s); });
  }
};

// Small-batch tile plan: bf16-activation calls (bf16 or fp8 weights) on at most d->small_b utterances take 1-row (128-wide)
// and 2-row (64-wide) conv tiles and one-tile conv64 segments -- at B = 1 the throughput tiles fill 16-40 of the 256
// CUs at levels 1-2 and 16 at level 0. Every utterance's arithmetic is the same within a plan (batch-invariant
// for any B on either side of the threshold); the two plans partition the GroupNorm partial sums differently, so
// results across plans agree to fp32 rounding of those sums (GPU test: plan agreement within the bf16 gate).
int small_plan(const gt_decoder* d, int dtype, int64_t nb) {
  return ((dtype == GT_BF16 || dtype == GT_BF16_W8 || dtype == GT_FP8) && nb <= d->small_b) ? 1 : 0;
}

uint8_t* align_ws(void* ws) { return (uint8_t*)(((uintptr_t)ws + 255) & ~(uintptr_t)255); }

// Utterances per internal batch chunk. The conv kernels address an activation tensor through a raw buffer
// descriptor with a 32-bit byte range, so one launch covers at most 2^31 bytes of its largest input (the
// level-0 64-channel activation, B x 80 x T x 64 elements). Larger batches run as consecutive chunks; the
// arithmetic is batch-invariant (GroupNorm slots and attention tiles are per utterance), so chunked results
// are bit-identical to one launch over the whole batch.
int64_t chunk_b(const gt_decoder* d, int dt, int64_t B, int64_t T) {
  const int64_t per_utt = 80 * T * 64 * (int64_t)esize(dt);
  int64_t cap = std::max<int64_t>(1, ((int64_t(1) << 31) - 1) / per_utt);
  if (d && d->max_chunk > 0) cap = std::min(cap, d->max_chunk);   // GT_MAX_CHUNK at creation (tests)
  return std::min(B, cap);
}

int check_common(gt_decoder* d, int dtype, int64_t B, int64_t T, void* ws, size_t ws_bytes, int32_t N) {
  if (!d) return fail(GT_ERR_ARG, "null decoder");
  if (dtype != GT_F32 && dtype != GT_BF16 && dtype != GT_BF16_W8 && dtype != GT_FP8)
    return fail(GT_ERR_ARG, "dtype must be GT_F32, GT_BF16, GT_BF16_W8 or GT_FP8");
  if (B <= 0 || T <= 0) return fail(GT_ERR_ARG, "B and T must be positive");
  if (T % 4 != 0) return fail(GT_ERR_ARG, "T must be a multiple of 4 (fix_len_compatibility)");
  if (B > 65535 || T > (1 << 20)) return fail(GT_ERR_UNSUPPORTED, "B or T too large");
  if (!ws) return fail(GT_ERR_ARG, "null workspace");
  if (80 * T * 64 * (int64_t)esize(dtype ? 1 : 0) >= (int64_t(1) << 31))
    return fail(GT_ERR_UNSUPPORTED, "T too large for one utterance per launch");
  if (ws_bytes < gt_decoder_workspace_bytes(d, dtype, B, T, N)) return fail(GT_ERR_WORKSPACE, "workspace too small");
  return GT_OK;
}

}  // namespace

extern "C" {

const char* gt_version(void) { return "gradtts-mi355x 0.1 (gfx950)"; }
const char* gt_last_error(void) { return g_err.c_str(); }

int gt_decoder_create(int n_feats, int dim, int n_spks, int spk_emb_dim, float beta_min, float beta_max,
                      float pe_scale, gt_decoder** out) {
  if (!out) return fail(GT_ERR_ARG, "null out");
  *out = nullptr;
  if (n_feats != 80 || dim != 64 || spk_emb_dim != 64)
    return fail(GT_ERR_UNSUPPORTED, "kernels implement n_feats=80, dim=64, spk_emb_dim=64");
  if (!(n_spks == 1 || n_spks == -1 || n_spks > 1)) return fail(GT_ERR_ARG, "n_spks must be 1, -1 or > 1");
  gt_decoder* d = new gt_decoder();
  d->n_feats = n_feats; d->dim = dim; d->n_spks = n_spks; d->spk_emb_dim = spk_emb_dim;
  d->beta_min = beta_min; d->beta_max = beta_max; d->pe_scale = pe_scale;
  d->inv = inventory(dim, n_spks, spk_emb_dim, n_feats);
  for (size_t i = 0; i < d->inv.size(); ++i) d->index[d->inv[i].name] = (int)i;
  d->host.resize(d->inv.size());
  d->set.assign(d->inv.size(), false);
  // SinusoidalPosEmb frequencies, as torch computes them: exp(float(k) * float(-ln(1e4)/31)) in fp32
  const float negc = (float)(-std::log(10000.0) / 31.0);
  for (int k = 0; k < 32; ++k) d->freqs[k] = expf((float)k * negc);
  if (const char* e = getenv("GT_GRAPHS")) d->graphs = atoi(e) != 0;
  if (const char* e = getenv("GT_MAX_CHUNK")) d->max_chunk = atoll(e);
  if (const char* e = getenv("GT_SMALL_B")) d->small_b = std::max<int64_t>(0, std::min<int64_t>(kSmallBMax, atoll(e)));
  if (const char* e = getenv("GT_CONV3W")) d->wide = atoi(e) != 0;
  if (const char* e = getenv("GT_CONV3W_A8")) d->wide_a8 = atoi(e) != 0;
  if (const char* e = getenv("GT_ATTN_DS")) d->attn_ds = atoi(e) != 0;
  if (const char* e = getenv("GT_ATTN_US")) d->attn_us = atoi(e) != 0;
  if (const char* e = getenv("GT_RB0_FUSE")) d->rb0_fuse = atoi(e) != 0;
  if (const char* e = getenv("GT_CONV64")) d->conv64 = atoi(e) != 0;
  if (const char* e = getenv("GT_X0_FUSE")) d->x0_fuse = atoi(e) != 0;
  if (const char* e = getenv("GT_CONV1S")) d->conv1s = atoi(e) != 0;
  if (const char* e = getenv("GT_ATTN_TILES_SMALL")) d->small_tiles = std::max(1, std::min(256, atoi(e)));
  if (const char* e = getenv("GT_MERGE_DR_SMALL")) d->merge_dr_small = atoi(e) == 32 ? 32 : 4;
  if (const char* e = getenv("GT_SK_TARGET")) d->sk_target = std::max(0, atoi(e));
  *out = d;
  return GT_OK;
}

void gt_decoder_destroy(gt_decoder* d) {
  if (!d) return;
  d->drop_graphs();
  if (d->cap_stream) (void)hipStreamDestroy(d->cap_stream);
  if (d->raw) (void)hipFree(d->raw);
  for (auto e : d->pool) (void)hipEventDestroy(e);
  if (d->dev_done) (void)hipEventDestroy(d->dev_done);
  for (int i = 0; i < gt_decoder::kCodes; ++i)
    if (d->arena[i]) (void)hipFree(d->arena[i]);
  delete d;
}

int gt_decoder_profile_enable(gt_decoder* d, int on) {
  if (!d) return fail(GT_ERR_ARG, "null decoder");
  d->prof = on != 0;
  return GT_OK;
}

int gt_decoder_profile_filter(gt_decoder* d, const char* prefix) {
  if (!d) return fail(GT_ERR_ARG, "null decoder");
  d->prof_prefix = prefix ? prefix : "";
  return GT_OK;
}

int gt_decoder_profile_read(gt_decoder* d, char* buf, size_t cap) {
  if (!d || !buf || cap == 0) return fail(GT_ERR_ARG, "null argument");
  struct Agg { long n = 0; double ms = 0, flop = 0, bytes = 0; };
  std::map<std::string, Agg> agg;
  for (auto& r : d->recs) {
    if (hipEventSynchronize(r.e1) != hipSuccess) return fail(GT_ERR_HIP, "hipEventSynchronize failed");
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.e0, r.e1) != hipSuccess) return fail(GT_ERR_HIP, "hipEventElapsedTime failed");
    Agg& a = agg[r.kernel];
    a.n += 1; a.ms += ms; a.flop += r.flop; a.bytes += r.bytes;
  }
  std::string js = "[";
  for (auto& kv : agg) {
    char line[512];
    snprintf(line, sizeof(line), "%s{\"kernel\": \"%s\", \"launches\": %ld, \"ms\": %.6f, \"flop\": %.6e, \"bytes\": %.6e}",
             js.size() > 1 ? ", " : "", kv.first.c_str(), kv.second.n, kv.second.ms, kv.second.flop, kv.second.bytes);
    js += line;
  }
  js += "]";
  d->recs.clear();
  d->pool_used = 0;
  if (js.size() + 1 > cap) return fail(GT_ERR_ARG, "buffer too small");
  memcpy(buf, js.c_str(), js.size() + 1);
  return GT_OK;
}

int64_t gt_decoder_pack_count(const gt_decoder* d) { return d ? d->packs : -1; }

int gt_decoder_num_params(const gt_decoder* d) { return d ? (int)d->inv.size() : 0; }
const char* gt_decoder_param_name(const gt_decoder* d, int i) {
  return (d && i >= 0 && i < (int)d->inv.size()) ? d->inv[i].name.c_str() : nullptr;
}
int64_t gt_decoder_param_numel(const gt_decoder* d, int i) {
  return (d && i >= 0 && i < (int)d->inv.size()) ? d->inv[i].numel() : -1;
}

int gt_decoder_set_param(gt_decoder* d, const char* name, const float* data, int64_t numel) {
  if (!d || !name || !data) return fail(GT_ERR_ARG, "null argument");
  if (int rc = gt_internal_refresh_host(d)) return rc;   // the other parameters' current values first
  auto it = d->index.find(name);
  if (it == d->index.end()) return fail(GT_ERR_PARAM, std::string("unknown parameter: ") + name);
  const Shape& sh = d->inv[it->second];
  if (numel != sh.numel()) return fail(GT_ERR_PARAM, std::string("numel mismatch for ") + name);
  d->host[it->second].assign(data, data + numel);
  d->set[it->second] = true;
  for (bool& x : d->dirty) x = true;
  d->raw_dirty = true;
  return GT_OK;
}

// The workspace may have any alignment: compute calls align its base up to 256 bytes (the slack is in the size).
// Sized for one batch chunk (chunk_b): batches past the 32-bit buffer range run chunk by chunk in it.
size_t gt_decoder_workspace_bytes(const gt_decoder* d, int dtype, int64_t B, int64_t T, int32_t n_timesteps) {
  (void)d;
  if (B <= 0 || T <= 0) return 0;
  const int dt = dtype ? 1 : 0;
  return layout(dt, chunk_b(d, dt, B, T), T, n_timesteps, d->small_tiles, small_plan(d, dtype, B), d->sk_target).total + 256;
}

static int estimator_impl(gt_decoder* d, int dtype, const float* x, const float* mask, const float* mu,
                          const float* t, const float* spk, int64_t B, int64_t T, float* out, void* workspace,
                          size_t workspace_bytes, void* stream, const char* probe, float* probe_out) {
  int rc = check_common(d, dtype, B, T, workspace, workspace_bytes, 0);
  if (rc) return rc;
  if (!x || !mask || !mu || !t || !out) return fail(GT_ERR_ARG, "null tensor");
  if (d->n_spks > 1 && !spk) return fail(GT_ERR_ARG, "n_spks > 1 needs spk [B,64]");
  if ((rc = prepare(d, dtype))) return rc;
  const int64_t Bc = chunk_b(d, dtype ? 1 : 0, B, T);
  if (probe && Bc < B) return fail(GT_ERR_UNSUPPORTED, "probes need the batch in one chunk");
  bool probed = false;
  for (int64_t b0 = 0; b0 < B; b0 += Bc) {   // batch chunks (chunk_b), each a complete evaluation
    const int64_t nb = std::min(Bc, B - b0);
    const size_t fo = (size_t)b0 * 80 * T;
    Run R;
    R.d = d; R.dt = dtype ? 1 : 0; R.wi = dtype; R.B = (int)nb; R.T = (int)T; R.small = small_plan(d, dtype, B); R.s = (hipStream_t)stream;
    R.ws = align_ws(workspace);
    R.L = layout(R.dt, nb, T, 0, d->small_tiles, R.small, d->sk_target);
    // split-K counters start at zero (every launch leaves them zeroed); a kernel node, not a memset, in captures
    if (R.L.skcnt_n) R.chk(launch_fill_f32((float*)(R.ws + R.L.skcnt), R.L.skcnt_n, 0.f, R.s));
    R.mask = mask + (size_t)b0 * T; R.mu = mu + fo; R.xt = x + fo; R.spk_s = nullptr;
    R.probe = probe; R.probe_out = probe_out;
    float* tbuf = (float*)(R.ws + R.L.tb);
    TembParams tp;
    tp.rows = (int)nb; tp.tvals = t + b0; tp.n_steps = 0; tp.pe_scale = d->pe_scale; tp.freqs = R.Fp("freqs");
    tp.w0 = R.Fp("mlp.0.weight"); tp.b0 = R.Fp("mlp.0.bias"); tp.w2 = R.Fp("mlp.2.weight"); tp.b2 = R.Fp("mlp.2.bias");
    tp.wr = R.Fp("tb.w"); tp.br = R.Fp("tb.b"); tp.nr = 1792; tp.tb = tbuf;
    tp.betas = nullptr; tp.beta_min = 0.f; tp.beta_delta = 0.f;
    R.chk(launch_temb(tp, R.s));
    if (d->n_spks > 1) {
      float* sbuf = (float*)(R.ws + R.L.spk);
      R.chk(launch_spk_mlp(spk + (size_t)b0 * 64, (int)nb, R.Fp("spk_mlp.0.weight"), R.Fp("spk_mlp.0.bias"),
                           R.Fp("spk_mlp.2.weight"), R.Fp("spk_mlp.2.bias"), sbuf, R.s));
      R.spk_s = sbuf;
    }
    R.tb = tbuf; R.tb_bstride = 1792;
    R.unet(0, out + fo, nullptr, 0.f, 0.f);
    if (R.err != hipSuccess) return fail(GT_ERR_HIP, std::string("HIP launch failed: ") + hipGetErrorString(R.err));
    probed = probed || R.probed;
  }
  if (probe && !probed) return fail(GT_ERR_ARG, std::string("unknown probe stage: ") + probe);
  return GT_OK;
}

int gt_estimator_forward(gt_decoder* d, int dtype, const float* x, const float* mask, const float* mu, const float* t,
                         const float* spk, int64_t B, int64_t T, float* out, void* workspace, size_t workspace_bytes,
                         void* stream) {
  return estimator_impl(d, dtype, x, mask, mu, t, spk, B, T, out, workspace, workspace_bytes, stream, nullptr, nullptr);
}

}  // extern "C"

// ---------------------------------------------------------------- internal accessors (train_bwd.cpp, C++ linkage)
int gt_internal_layout(gt_decoder* d) {   // offsets of the raw block (the inventory's, fixed per decoder)
  if (d->raw_off.size() == d->inv.size()) return GT_OK;
  d->raw_off.clear();
  int64_t n = 0;
  for (auto& s : d->inv) { d->raw_off.push_back(n); n += s.numel(); }
  d->raw_numel = n;
  return GT_OK;
}
int gt_internal_prepare_raw(gt_decoder* d) {
  for (size_t i = 0; i < d->inv.size(); ++i)
    if (!d->set[i]) return fail(GT_ERR_PARAM, "parameter never set: " + d->inv[i].name);
  if (!d->raw_dirty) return GT_OK;
  gt_internal_layout(d);
  const int64_t n = d->raw_numel;
  std::vector<float> h((size_t)n + 32);
  for (size_t i = 0; i < d->inv.size(); ++i) memcpy(h.data() + d->raw_off[i], d->host[i].data(), d->host[i].size() * 4);
  memcpy(h.data() + n, d->freqs, sizeof(d->freqs));
  if (d->raw) { (void)hipFree(d->raw); d->raw = nullptr; }
  if (hipMalloc(&d->raw, h.size() * 4) != hipSuccess) return fail(GT_ERR_HIP, "hipMalloc(raw params) failed");
  if (hipMemcpy(d->raw, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return fail(GT_ERR_HIP, "hipMemcpy(raw params) failed");
  d->raw_dirty = false;
  return GT_OK;
}
const float* gt_internal_param(gt_decoder* d, const std::string& name) {
  auto it = d->index.find(name);
  return it == d->index.end() ? nullptr : d->raw + d->raw_off[it->second];
}
int64_t gt_internal_param_offset(gt_decoder* d, const std::string& name) {
  auto it = d->index.find(name);
  return it == d->index.end() ? -1 : d->raw_off[it->second];
}
bool gt_internal_has_param(gt_decoder* d, const std::string& name) { return d->index.count(name) != 0; }
float gt_internal_host_scalar(gt_decoder* d, const std::string& name) {
  (void)gt_internal_refresh_host(d);
  return d->host[d->index.at(name)][0];
}

// host copies <- the device fp32 block after gt_decoder_set_params_device (synchronous; only when an inference
// image, a host scalar or a host-side parameter change needs them)
int gt_internal_refresh_host(gt_decoder* d) {
  if (!d->host_stale) return GT_OK;
  // the update's own completion event, not its stream: the caller may have destroyed the stream since
  if (d->dev_done && hipEventSynchronize(d->dev_done) != hipSuccess) return fail(GT_ERR_HIP, "hipEventSynchronize failed");
  std::vector<float> h((size_t)d->raw_numel);
  if (hipMemcpy(h.data(), d->raw, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(GT_ERR_HIP, "hipMemcpy(raw params -> host) failed");
  for (size_t i = 0; i < d->inv.size(); ++i)
    memcpy(d->host[i].data(), h.data() + d->raw_off[i], d->host[i].size() * 4);
  d->host_stale = false;
  return GT_OK;
}

int gt_decoder_set_params_device(gt_decoder* d, const float* params, int64_t numel, void* stream) {
  if (!d || !params) return fail(GT_ERR_ARG, "null argument");
  if (int rc = gt_internal_prepare_raw(d)) return rc;   // the block exists (parameters were set once from the host)
  if (numel != d->raw_numel) return fail(GT_ERR_ARG, "numel != gt_decoder_grad_numel");
  const hipError_t e = launch_copy_f32(d->raw, params, (long)numel, (hipStream_t)stream);
  if (e != hipSuccess) return fail(GT_ERR_HIP, std::string("parameter copy: ") + hipGetErrorString(e));
  if (!d->dev_done && hipEventCreateWithFlags(&d->dev_done, hipEventDisableTiming) != hipSuccess)
    return fail(GT_ERR_HIP, "hipEventCreate failed");
  if (hipEventRecord(d->dev_done, (hipStream_t)stream) != hipSuccess) return fail(GT_ERR_HIP, "hipEventRecord failed");
  for (bool& x : d->dirty) x = true;
  d->host_stale = true;
  return GT_OK;
}
const float* gt_internal_freqs(gt_decoder* d) { return d->raw + d->raw_numel; }
int64_t gt_internal_numel(gt_decoder* d) { return d->raw_numel; }
void gt_internal_consts(gt_decoder* d, int* n_spks, float* bmin, float* bmax, float* pe_scale) {
  *n_spks = d->n_spks; *bmin = d->beta_min; *bmax = d->beta_max; *pe_scale = d->pe_scale;
}
int gt_internal_fail(int code, const std::string& msg) { return fail(code, msg); }

extern "C" {

// ---------------------------------------------------------------- training path (forward values)
static size_t align256(size_t n) { return (n + 255) & ~size_t(255); }

int gt_forward_diffusion(gt_decoder* d, const float* x0, const float* mask, const float* mu, const float* t,
                         const float* z, int64_t B, int64_t T, float* xt, float* zm, void* stream) {
  if (!d || !x0 || !mask || !mu || !t || !z || !xt) return fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || T <= 0 || B * 80 * T >= (int64_t(1) << 31)) return fail(GT_ERR_ARG, "bad B / T");
  FwdDiffParams p;
  p.x0 = x0; p.mu = mu; p.z = z; p.mask = mask; p.t = t; p.B = (int)B; p.F = 80; p.T = (int)T;
  p.beta_min = d->beta_min;
  p.half_delta = (float)(0.5 * ((double)d->beta_max - (double)d->beta_min));
  p.xt = xt; p.zm = zm;
  if (launch_fwd_diffusion(p, (hipStream_t)stream) != hipSuccess) return fail(GT_ERR_HIP, "forward_diffusion launch failed");
  return GT_OK;
}

size_t gt_diffusion_loss_workspace_bytes(const gt_decoder* d, int dtype, int64_t B, int64_t T) {
  if (B <= 0 || T <= 0) return 0;
  const size_t n = (size_t)B * 80 * T * 4;
  return align256(gt_decoder_workspace_bytes(d, dtype, B, T, 0)) + 2 * align256(n) +
         align256((size_t)loss_blocks((long)B * 80 * T) * 8) + 256;
}

int gt_diffusion_loss_t(gt_decoder* d, int dtype, const float* x0, const float* mask, const float* mu, const float* t,
                        const float* z, const float* spk, int64_t B, int64_t T, float* loss, float* xt, void* workspace,
                        size_t workspace_bytes, void* stream) {
  if (!d || !loss || !xt || !workspace) return fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || T <= 0 || B * 80 * T >= (int64_t(1) << 31)) return fail(GT_ERR_ARG, "bad B / T");
  if (workspace_bytes < gt_diffusion_loss_workspace_bytes(d, dtype, B, T)) return fail(GT_ERR_WORKSPACE, "workspace too small");
  uint8_t* ws = align_ws(workspace);
  const size_t est_bytes = align256(gt_decoder_workspace_bytes(d, dtype, B, T, 0));
  const size_t n = (size_t)B * 80 * T * 4;
  float* zm = (float*)(ws + est_bytes);
  float* score = (float*)(ws + est_bytes + align256(n));
  float* part = (float*)(ws + est_bytes + 2 * align256(n));
  const hipStream_t s = (hipStream_t)stream;
  int rc = gt_forward_diffusion(d, x0, mask, mu, t, z, B, T, xt, zm, stream);   // diffusion.py:275
  if (rc) return rc;
  rc = estimator_impl(d, dtype, xt, mask, mu, t, spk, B, T, score, ws, est_bytes, stream, nullptr, nullptr);  // :277
  if (rc) return rc;
  LossParams lp;
  lp.score = score; lp.z = z; lp.mask = mask; lp.t = t; lp.B = (int)B; lp.F = 80; lp.T = (int)T;
  lp.beta_min = d->beta_min;
  lp.half_delta = (float)(0.5 * ((double)d->beta_max - (double)d->beta_min));
  lp.part = part;
  if (launch_loss(lp, loss, s) != hipSuccess) return fail(GT_ERR_HIP, "loss launch failed");   // :278-280
  return GT_OK;
}

size_t gt_alignment_workspace_bytes(int64_t B, int64_t Tx, int64_t Ty) {
  if (B <= 0 || Tx <= 0 || Ty <= 0) return 0;
  return align256((size_t)B * Tx * Ty * 4) + align256((size_t)B * 8) + gt_maximum_path_workspace_bytes(B, Tx, Ty) + 256;
}

int gt_log_prior_maximum_path(const float* mu_x, const float* y, const float* x_mask, const float* y_mask, int64_t B,
                              int64_t n_feats, int64_t Tx, int64_t Ty, int32_t* paths, float* log_prior,
                              void* workspace, size_t workspace_bytes, void* stream) {
  if (!mu_x || !y || !x_mask || !y_mask || !paths || !workspace) return fail(GT_ERR_ARG, "null argument");
  if (B <= 0 || Tx <= 0 || Ty <= 0 || n_feats <= 0) return fail(GT_ERR_ARG, "bad shape");
  if (n_feats > 128) return fail(GT_ERR_UNSUPPORTED, "n_feats > 128");
  if (B > 65535 || B * Tx * Ty >= (int64_t(1) << 31)) return fail(GT_ERR_UNSUPPORTED, "alignment grid too large");
  if (workspace_bytes < gt_alignment_workspace_bytes(B, Tx, Ty)) return fail(GT_ERR_WORKSPACE, "workspace too small");
  uint8_t* ws = align_ws(workspace);
  const size_t nlp = align256((size_t)B * Tx * Ty * 4);
  float* lp = log_prior ? log_prior : (float*)ws;
  int32_t* lens = (int32_t*)(ws + nlp);
  void* mas_ws = ws + nlp + align256((size_t)B * 8);
  const size_t mas_bytes = workspace_bytes - (size_t)((uint8_t*)mas_ws - (uint8_t*)workspace);
  const hipStream_t s = (hipStream_t)stream;
  const float cst = (float)(-0.5 * std::log(2.0 * M_PI) * (double)n_feats);   // tts.py:143 (Python float -> fp32 add)
  if (launch_log_prior(mu_x, y, x_mask, y_mask, (int)B, (int)n_feats, (int)Tx, (int)Ty, cst, lp, s) != hipSuccess ||
      launch_mask_len(x_mask, y_mask, (int)B, (int)Tx, (int)Ty, lens, lens + B, s) != hipSuccess)
    return fail(GT_ERR_HIP, "log-prior launch failed");
  const int rc = gt_maximum_path(paths, lp, lens, lens + B, B, Tx, Ty, -1e9f, mas_ws, mas_bytes, stream);
  if (rc) return fail(rc, "maximum_path failed");
  return GT_OK;
}

int gt_estimator_probe(gt_decoder* d, int dtype, const float* x, const float* mask, const float* mu, const float* t,
                       const float* spk, int64_t B, int64_t T, const char* stage, float* probe_out, float* out,
                       void* workspace, size_t workspace_bytes, void* stream) {
  if (!stage || !probe_out) return fail(GT_ERR_ARG, "null stage / probe_out");
  return estimator_impl(d, dtype, x, mask, mu, t, spk, B, T, out, workspace, workspace_bytes, stream, stage, probe_out);
}

// Replay (capturing first if needed) the HIP graph of S Euler steps for this key on `stream`.
static int run_segment_graph(gt_decoder* d, Run& R, const std::vector<uintptr_t>& key, int S, float* xt, float hf,
                             hipStream_t stream, hipGraphExec_t* out_exec) {
  for (size_t i = 0; i < d->gcache.size(); ++i)
    if (d->gcache[i].key == key) {
      gt_decoder::Graph g = d->gcache[i];
      d->gcache.erase(d->gcache.begin() + i);
      d->gcache.push_back(g);
      *out_exec = g.exec;
      return GT_OK;
    }
  if (!d->cap_stream && hipStreamCreateWithFlags(&d->cap_stream, hipStreamNonBlocking) != hipSuccess)
    return fail(GT_ERR_HIP, "hipStreamCreate(capture) failed");
  if (hipStreamBeginCapture(d->cap_stream, hipStreamCaptureModeRelaxed) != hipSuccess)
    return fail(GT_ERR_HIP, "hipStreamBeginCapture failed");
  R.s = d->cap_stream;
  const float* tb0 = R.tb;
  const float* be0 = R.betas;
  for (int j = 0; j < S && R.err == hipSuccess; ++j) {   // step j of the segment reads row (*stepp + j)
    R.tb = tb0 + (size_t)j * kTbRow;
    R.betas = be0 + j;
    R.unet(1, nullptr, xt, 0.f, hf);
  }
  R.tb = tb0; R.betas = be0; R.s = stream;
  hipGraph_t g = nullptr;
  const hipError_t ec = hipStreamEndCapture(d->cap_stream, &g);
  if (R.err != hipSuccess || ec != hipSuccess || !g) {
    if (g) (void)hipGraphDestroy(g);
    return fail(GT_ERR_HIP, std::string("graph capture failed: ") + hipGetErrorString(R.err != hipSuccess ? R.err : ec));
  }
  hipGraphExec_t ex = nullptr;
  const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (ei != hipSuccess) return fail(GT_ERR_HIP, std::string("hipGraphInstantiate failed: ") + hipGetErrorString(ei));
  if (d->gcache.size() >= 8) {
    (void)hipGraphExecDestroy(d->gcache.front().exec);
    d->gcache.erase(d->gcache.begin());
  }
  d->gcache.push_back({key, ex});
  d->captures += 1;
  *out_exec = ex;
  return GT_OK;
}

int gt_reverse_diffusion(gt_decoder* d, int dtype, const float* z, const float* mask, const float* mu, const float* spk,
                         int64_t B, int64_t T, int32_t n_timesteps, float* out, void* workspace, size_t workspace_bytes,
                         void* stream) {
  int rc = check_common(d, dtype, B, T, workspace, workspace_bytes, n_timesteps);
  if (rc) return rc;
  if (!z || !mask || !mu || !out) return fail(GT_ERR_ARG, "null tensor");
  if (n_timesteps < 0) return fail(GT_ERR_ARG, "n_timesteps must be >= 0");
  if (d->n_spks > 1 && !spk) return fail(GT_ERR_ARG, "n_spks > 1 needs spk [B,64]");
  if ((rc = prepare(d, dtype))) return rc;
  const hipStream_t st = (hipStream_t)stream;
  // Graph segments unless profiling (events per launch) or the caller's stream is itself being captured
  // (then the launches below simply become part of the caller's graph).
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return fail(GT_ERR_HIP, "hipStreamIsCapturing failed");
  const bool use_graph = d->graphs && !d->prof && cs == hipStreamCaptureStatusNone;
  const int64_t Bc = chunk_b(d, dtype ? 1 : 0, B, T);
  for (int64_t b0 = 0; b0 < B; b0 += Bc) {   // batch chunks (chunk_b): independent utterances
    const int64_t nb = std::min(Bc, B - b0);
    const size_t fo = (size_t)b0 * 80 * T;
    Run R;
    R.d = d; R.dt = dtype ? 1 : 0; R.wi = dtype; R.B = (int)nb; R.T = (int)T; R.small = small_plan(d, dtype, B); R.s = st;
    R.ws = align_ws(workspace);
    R.L = layout(R.dt, nb, T, n_timesteps, d->small_tiles, R.small, d->sk_target);
    if (R.L.skcnt_n) R.chk(launch_fill_f32((float*)(R.ws + R.L.skcnt), R.L.skcnt_n, 0.f, R.s));
    R.mask = mask + (size_t)b0 * T; R.mu = mu + fo; R.xt = out + fo; R.spk_s = nullptr;
    float* xt = out + fo;
    R.chk(launch_mask_copy(z + fo, R.mask, (int)nb, 80, (int)T, xt, R.s));   // xt = z * mask  (diffusion.py:257)
    if (n_timesteps > 0) {
      float* tbuf = (float*)(R.ws + R.L.tb);
      float* betas = (float*)(R.ws + R.L.betas);
      int* stepp = (int*)(R.ws + R.L.step);
      // time biases and beta(t) of every step (t_i = 1 - (i + 0.5)/N, diffusion.py:259-263), on device
      TembParams tp;
      tp.rows = n_timesteps; tp.tvals = nullptr; tp.n_steps = n_timesteps; tp.pe_scale = d->pe_scale;
      tp.freqs = R.Fp("freqs");
      tp.w0 = R.Fp("mlp.0.weight"); tp.b0 = R.Fp("mlp.0.bias"); tp.w2 = R.Fp("mlp.2.weight"); tp.b2 = R.Fp("mlp.2.bias");
      tp.wr = R.Fp("tb.w"); tp.br = R.Fp("tb.b"); tp.nr = kTbRow; tp.tb = tbuf;
      tp.betas = betas; tp.beta_min = d->beta_min;
      tp.beta_delta = (float)((double)d->beta_max - (double)d->beta_min);
      R.chk(launch_temb(tp, R.s));
      if (d->n_spks > 1) {
        float* sbuf = (float*)(R.ws + R.L.spk);
        R.chk(launch_spk_mlp(spk + (size_t)b0 * 64, (int)nb, R.Fp("spk_mlp.0.weight"), R.Fp("spk_mlp.0.bias"),
                             R.Fp("spk_mlp.2.weight"), R.Fp("spk_mlp.2.bias"), sbuf, R.s));
        R.spk_s = sbuf;
      }
      const float hf = (float)(1.0 / (double)n_timesteps);
      R.tb_bstride = 0; R.stepp = stepp;
      R.tb = tbuf; R.betas = betas;
      if (!use_graph) {
        // a kernel, not hipMemsetD32Async: captured into a caller's graph (torch.cuda.graph), a memset node misbehaves
        // from its second replay on (tools/memset_capture_probe.py)
        R.chk(launch_set_step(stepp, 0, R.s));
        for (int i = 0; i < n_timesteps && R.err == hipSuccess; ++i) {
          R.tb = tbuf + (size_t)i * kTbRow;
          R.betas = betas + i;
          R.unet(1, nullptr, xt, 0.f, hf);
        }
      } else if (R.err == hipSuccess) {
        // segments of S steps (the whole loop up to 100 steps); a graph's kernels read rows *stepp + j
        const int S = n_timesteps <= 100 ? n_timesteps : 50;
        const int q = n_timesteps / S, rem = n_timesteps % S;
        auto key = [&](int steps) {
          return std::vector<uintptr_t>{(uintptr_t)dtype, (uintptr_t)nb, (uintptr_t)R.small, (uintptr_t)T, (uintptr_t)steps,
                                        (uintptr_t)n_timesteps, (uintptr_t)R.ws, (uintptr_t)xt, (uintptr_t)R.mask,
                                        (uintptr_t)R.mu, (uintptr_t)d->arena[dtype]};
        };
        hipGraphExec_t seg = nullptr, tail = nullptr;
        if ((rc = run_segment_graph(d, R, key(S), S, xt, hf, st, &seg))) return rc;
        if (rem && (rc = run_segment_graph(d, R, key(rem), rem, xt, hf, st, &tail))) return rc;
        for (int k = 0; k <= q && R.err == hipSuccess; ++k) {
          if (k == q && !rem) break;
          R.chk(launch_set_step(stepp, k * S, st));
          R.chk(hipGraphLaunch(k < q ? seg : tail, st));
        }
      }
    }
    if (R.err != hipSuccess) return fail(GT_ERR_HIP, std::string("HIP launch failed: ") + hipGetErrorString(R.err));
  }
  return GT_OK;
}

int gt_decoder_set_graphs(gt_decoder* d, int on) {
  if (!d) return fail(GT_ERR_ARG, "null decoder");
  d->graphs = on != 0;
  if (!d->graphs) d->drop_graphs();
  return GT_OK;
}

int64_t gt_decoder_graph_captures(const gt_decoder* d) { return d ? d->captures : -1; }

int gt_decoder_set_betas(gt_decoder* d, float beta_min, float beta_max) {
  if (!d) return fail(GT_ERR_ARG, "null decoder");
  if (d->beta_min != beta_min || d->beta_max != beta_max) {
    d->beta_min = beta_min; d->beta_max = beta_max;
    d->drop_graphs();   // captured sampler graphs hold the old beta table
  }
  return GT_OK;
}

int gt_decoder_set_wide_conv(gt_decoder* d, int on) {
  if (!d) return fail(GT_ERR_ARG, "null decoder");
  d->wide = on != 0;
  d->drop_graphs();
  return GT_OK;
}

int gt_decoder_set_small_batch(gt_decoder* d, int64_t max_b) {
  if (!d) return fail(GT_ERR_ARG, "null decoder");
  if (max_b < 0 || max_b > kSmallBMax) return fail(GT_ERR_ARG, "max_b must be in [0, 16]");
  d->small_b = max_b;
  d->drop_graphs();
  return GT_OK;
}

}  // extern "C"
