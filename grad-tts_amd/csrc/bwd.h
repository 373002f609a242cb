// U-Net backward building blocks (bwd.hip): parameter blocks and launchers. fp32, channels-last [B][F][T][C].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gt {

// gather relation v = u*S - PAD + k over a KS x KS kernel (k = kh*KS + kw)
struct GConvParams {
  int B, Fi, Ti, Cin, Fo, To, Cout;   // in grid (Fi, Ti, Cin) -> out grid (Fo, To, Cout)
  int KS, S, PAD;
  int transposed;                     // 0: out[u] = sum W in[v(u,k)] (gconv);  1: out[v] = sum W in[u] (tconv)
  int flip;                           // gconv: tap k reads weight KK-1-k (stride-1 dgrad)
  const float* in; const float* w; long wsa, wsc;   // weight element (a = out channel, c = in channel, k) at a*wsa + c*wsc + k
  const float* bias;
  const float* mask; int T0, lvl_in;  // non-null: multiply the input by the level mask
  const float* out_mask; int lvl_out; // non-null: multiply the output by the level mask
  float* out; int out_cs, out_c0;     // output channel stride / first channel (writes into a wider tensor)
  int accumulate;
  float* wpk;                         // scratch of Cout * KS^2 * Cin floats (gconv_wpk_floats): the 3x3 / 4x4
                                      // stride-1 relations repack the weights there and run the float4-staged kernel
  int wpk_ready;                      // 1: wpk already holds the repacked weights (launch_gconv_wpack_batch)
};
// scratch the packed-weight path of launch_gconv needs (0: the relation runs without it)
long gconv_wpk_floats(const GConvParams& p);
// one weight repack of a launch_gconv (wpk[a][k][c] = W(a, c, flip' ? KK - 1 - k : k)), batched
struct GconvPack {
  const float* w; float* dst; long wsa, wsc; int KK, flip, Cout, Cin;
};
// the repacks a launch_gconv of p would do itself (p.wpk set, packed path eligible); false: none
bool gconv_pack_desc(const GConvParams& p, GconvPack* out);
hipError_t launch_gconv_wpack_batch(const GconvPack* packs, int n, hipStream_t s);
// dW(a, b, k) = sum_u P[u][a] Q[v(u,k)][b]; U grid (Fu, Tu), V grid (Fv, Tv)
struct WGradParams {
  int B, Fu, Tu, A, Fv, Tv, Bc, KS, S, PAD;
  const float* P; const float* pmask; int lvl_p;
  const float* Q; const float* qmask; int lvl_q;
  int T0;
  float* part;
};
struct BlockBwdParams {
  int B, npos, T, C;                  // npos = F * T of the level; T = frames of the level
  const float* dA; const float* h; const float* stats; const float* gamma; const float* beta;
  const float* mask; int T0, lvl;
  float* gsum; float* dgb; float* dh;
};
struct EwParams {
  int B, F, T, C;
  const float* x; int xcs, xc0; float alpha;
  const float* x2; float alpha2;      // optional second term (same channel count, dense)
  const float* mask; int T0, lvl;
  float* y; int ycs, yc0; int accumulate;
  const float* alphap; const float* alpha2p;   // device scalars: alpha / alpha2 read from memory when non-null
};

hipError_t launch_gconv(const GConvParams& p, hipStream_t s);
// launchers of the single kernels (grid / block chosen by the caller)
hipError_t launch_mish_bwd(dim3 grid, dim3 block, hipStream_t strm, const float* dY, const float* pre, int n, float* dX);
hipError_t launch_dmu(dim3 grid, dim3 block, hipStream_t strm, const float* dxin, int cin, const float* t,
                      const float* mask, int B, int T, float bmin, float half_delta, float* dmu);
hipError_t launch_spk_chan_sum(dim3 grid, dim3 block, hipStream_t strm, const float* dxin, int cin, int T, float* ds);
hipError_t launch_mask_sum(dim3 grid, dim3 block, hipStream_t strm, const float* mask, long n, float* out);
hipError_t launch_bsum(dim3 grid, dim3 block, hipStream_t strm, const float* x, const float* y, int npos, int C, float* out, int accumulate);
hipError_t launch_colsum(dim3 grid, dim3 block, hipStream_t strm, const float* in, int B, int C, float* out, int accumulate);
hipError_t launch_gn_stats(dim3 grid, dim3 block, hipStream_t strm, const float* h, int npos, int C, float* stats);
hipError_t launch_block_bwd_reduce(dim3 grid, dim3 block, hipStream_t strm, BlockBwdParams p);
hipError_t launch_block_bwd_apply(dim3 grid, dim3 block, hipStream_t strm, BlockBwdParams p);
hipError_t launch_block_fwd(dim3 grid, dim3 block, hipStream_t strm, BlockBwdParams p, const float* tb, float* out);
hipError_t launch_ew(dim3 grid, dim3 block, hipStream_t strm, EwParams p);
hipError_t launch_attn_kstats(dim3 grid, dim3 block, hipStream_t strm, const float* qkv, int npos, float* st);
hipError_t launch_attn_ksoftmax(dim3 grid, dim3 block, hipStream_t strm, float* qkv, int B, int npos, const float* st);
hipError_t launch_attn_outer(dim3 grid, dim3 block, hipStream_t strm, const float* X1, int cs1, int x1o, const float* X2, int cs2, int x2o, int npos, float* R);
hipError_t launch_attn_headmm(dim3 grid, dim3 block, hipStream_t strm, const float* M, int trans, const float* X, int csx, int xo, int B, int npos, float* Y, int csy, int yo, int accumulate);
hipError_t launch_attn_ksoftmax_bwd(dim3 grid, dim3 block, hipStream_t strm, const float* qkv_s, float* dqkv, int B, int npos, const float* S);
hipError_t launch_attn_rowdot(dim3 grid, dim3 block, hipStream_t strm, const float* a, int csa, int ao, const float* c, int csc, int co, int npos, float* S);
hipError_t launch_dot(dim3 grid, dim3 block, hipStream_t strm, const float* x, const float* y, long n, float* out, int accumulate);
hipError_t launch_linear_fwd(dim3 grid, dim3 block, hipStream_t strm, const float* X, int I, const float* W, const float* bias, int O, int act, float* Y);
hipError_t launch_linear_wgrad(dim3 grid, dim3 block, hipStream_t strm, const float* dY, const float* X, int B, int I, int O, float* dW, float* db);
hipError_t launch_linear_dgrad(dim3 grid, dim3 block, hipStream_t strm, const float* dY, const float* W, int I, int O, const float* pre, float* dX, int accumulate);
hipError_t launch_posemb(dim3 grid, dim3 block, hipStream_t strm, const float* t, float scale, const float* freqs, float* out);
hipError_t launch_loss_bwd(dim3 grid, dim3 block, hipStream_t strm, const float* score, const float* z, const float* mask, const float* t, const float* tot, int B, int T, float bmin, float half_delta, float* ds);
hipError_t launch_input_pack(dim3 grid, dim3 block, hipStream_t strm, const float* mu, const float* xt, const float* s, int B, int T, int cin, float* out);

// split position reductions (fixed order; part sizes from pos_splits)
constexpr int kDotBlocks = 256;
int pos_splits(long npos);
// part: B * pos_splits(npos) * C floats; out[b][c] (per_b) or out[c]
hipError_t launch_chan_sums(const float* x, const float* y, int B, int npos, int C, float* part, float* out, int per_b,
                            int accumulate, hipStream_t strm);
hipError_t launch_chan_sums_strided(const float* x, int xcs, int xo, const float* y, int ycs, int yo, int B, int npos,
                                    int C, float* part, float* out, int per_b, int accumulate, hipStream_t strm);
// GroupNorm (mean, rstd) per (b, group) [B][8][2]; part: B * 8 * gn_splits(npos) * 2 doubles
int gn_splits(long npos);
hipError_t launch_gn_stats_split(const float* h, int B, int npos, int C, double* part, float* stats, hipStream_t strm);
hipError_t launch_attn_headmm_mfma(const float* M, int trans, const float* X, int csx, int xo, int B, int npos, float* Y,
                                   int csy, int yo, int accumulate, hipStream_t strm);
// part: B * pos_splits(npos) * C * 2 floats; writes p.dgb [B][C][2] and p.gsum [B][8][2]
hipError_t launch_block_bwd_sums(const BlockBwdParams& p, float* part, hipStream_t strm);
// part: kDotBlocks doubles
hipError_t launch_dot_sum(const float* x, const float* y, long n, double* part, float* out, int accumulate,
                          hipStream_t strm);
// part: pos_splits(npos) * B * 4096 floats
hipError_t launch_attn_outer_split(const float* X1, int cs1, int x1o, const float* X2, int cs2, int x2o, int B, int npos,
                                   float* part, float* R, hipStream_t strm);
// part: B * pos_splits(npos) * 128 floats
hipError_t launch_attn_rowdot_split(const float* a, int csa, int ao, const float* c, int csc, int co, int B, int npos,
                                    float* part, float* S_out, hipStream_t strm);

// fp32-MFMA weight gradient: part holds mwgrad_splits(p) * KS^2 * A * Bc floats (<= kWPartCap, one shared buffer)
constexpr long kWPartCap = 40L << 20;   // 160 MB: 32 splits of the 256 x 256 x 9 level-2 gradients
int mwgrad_splits(const WGradParams& p);
hipError_t launch_mwgrad(const WGradParams& p, float* part, float* dw, long sa, long sb, int accumulate, hipStream_t strm);

}  // namespace gt
