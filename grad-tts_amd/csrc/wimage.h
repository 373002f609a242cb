// Packed weight image of one convolution, shared by the host packer (decoder.cpp), the attention
// matrix builder (attn.hip) and conv_kernel (conv.hip).
//
// The image is laid out in exactly the order conv_kernel keeps the weight slab in LDS, so staging a
// K-chunk is a straight, fully coalesced global->LDS DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction) with no register round trip:
//   image[n_tile][chunk] = WBYTES bytes = half A, then half B (bf16 images with more than one tap):
//   half A          = NT rows x WROWA bytes, taps [0, NA): NA x CKB bytes + 16 B pad, zero padded to 4 KiB
//   half B          = NT rows x WROWB bytes, taps [NA, NTAP): (NTAP - NA) x CKB + 16 B pad, padded to 4 KiB
// (fp32 and 1x1 images: one half with every tap). The 16-byte row pad makes the row stride an odd number of
// 16-B LDS slots, so the 16 lanes of a ds_read_b128 group (16 different output channels) hit 16 different
// slots. The two halves are staged separately: conv_kernel computes the taps of one half while the other
// half of the next chunk lands (wave-even 1 KiB DMA pieces: each half is a multiple of 4 KiB).
#pragma once

namespace gt {

// output channels per workgroup: 128 for bf16 layers with >= 128 output channels, else 64
inline __host__ __device__ constexpr int conv_nt(int act_bf16, int cout) { return (act_bf16 && cout >= 128) ? 128 : 64; }
// 3x3 tiles with 256+ output channels (two 128-wide channel tiles) and no operand transform cover 5 mel rows
// (320 positions): every level's row count (80 >> l) divides by 5, and at B = 32 the level-2 grid becomes one
// whole round of 2 workgroups per CU (512 tiles instead of 640). The GroupNorm-input variant keeps 4 rows (the
// extra accumulators spill there), as do 128-output convs (256 tiles would leave half the slots empty).
// Also on 5-row tiles (round-2 same-box A/Bs):
//  * 128-output convs without an operand transform on the 40-row level-1 grid (1024 tiles at B = 32 instead of 1280;
//    97.5 -> 95.0 us and 65.4 -> 62.3 us for the two level-1 block1 convs);
//  * the level-1 GroupNorm-input conv (128 -> 128, 40 rows) with the in-register GroupNorm transform: two whole rounds
//    of 512 slots instead of 1280 tiles; fits 247 VGPRs with the interleaved row blocks (+0.7-0.9 % end to end);
//  * 128-wide 1x1 convs where that removes a partial round of workgroups (2 per CU): level 2 with 256 output channels
//    (640 -> 512 tiles at B = 32) and level 1 (1280 -> 1024);
//  * the 128-channel Upsample (level 2 -> 1, 20 coarse rows): 1280 -> 1024 workgroups at B = 32.
// (conv3w, conv3w.hip, now runs most of these 3x3 convs on the bf16 throughput plan; conv_kernel keeps the rest.)
// mel rows per 3x3 / 1x1 tile (kind/im: ConvKind/InMode values, nt: channel tile, cout: output channels, f: grid
// rows, small: the small-batch plan). Small batches (decoder.cpp small_plan) take one-row tiles for 128-wide and
// two-row tiles for 64-wide convs (64 positions per wave pair: 4-5x the workgroups of the throughput tiles, which at
// B = 1 fill 16-40 of the 256 CUs).
inline __host__ __device__ constexpr int conv_tf(int kind, int im, int nt, int cout, int f, int small = 0) {
  return (small && (kind == 0 /*CONV3*/ || kind == 2 /*CONV1*/)) ? (nt == 128 ? 1 : 2)
         : (kind == 2 /*CONV1*/ && nt == 128 && (cout >= 256 || f == 40)) ? 5
         : (kind == 3 /*CONVT4*/ && nt == 128 && f == 40) ? 5
         : (kind == 0 /*CONV3*/ && nt == 128 && (cout >= 256 || (cout == 128 && f == 40))) ? 5 : 4;
}
// bytes of one position's channel chunk in LDS: 16 channels = one MFMA k-step (32 B bf16, 64 B fp32). bf16 1x1 convs
// over activations (cin > 16) take 64 bytes (32 channels = two k-steps): a 1x1 chunk is one tap, so a 16-channel chunk
// left one barrier + weight/patch round trip per 10 MFMAs per wave (64-channel chunks measured slower: registers).
inline __host__ __device__ constexpr int conv_ckb(int act_bf16, int ntap = 9, int cin = 0) {
  return act_bf16 ? ((ntap == 1 && cin > 16) ? 64 : 32) : 64;
}
inline __host__ __device__ constexpr int conv_wrow(int ntap, int ckb) { return ntap * ckb + 16; }
inline __host__ __device__ constexpr int round4k(int b) { return ((b + 4095) / 4096) * 4096; }
// taps in half A: split images (bf16, more than one tap) put the first ceil(NTAP/2) taps there
inline __host__ __device__ constexpr int conv_na(int act_bf16, int ntap) { return (act_bf16 && ntap > 1) ? (ntap + 1) / 2 : ntap; }
inline __host__ __device__ constexpr int conv_habytes(int act_bf16, int nt, int ntap, int ckb) {
  return round4k(nt * conv_wrow(conv_na(act_bf16, ntap), ckb));
}
inline __host__ __device__ constexpr int conv_hbbytes(int act_bf16, int nt, int ntap, int ckb) {
  return conv_na(act_bf16, ntap) == ntap ? 0 : round4k(nt * conv_wrow(ntap - conv_na(act_bf16, ntap), ckb));
}

struct WImg {
  int nt, ckb, ck, ntap, na, wrowa, wrowb, habytes, wbytes, nchunk, nntile;
  long total;   // bytes of the whole image
};

inline __host__ __device__ WImg conv_wimg(int act_bf16, int ntap, int cin, int cout) {
  WImg w;
  w.nt = conv_nt(act_bf16, cout);
  w.ckb = conv_ckb(act_bf16, ntap, cin);
  w.ck = w.ckb / (act_bf16 ? 2 : 4);
  w.ntap = ntap;
  w.na = conv_na(act_bf16, ntap);
  w.wrowa = conv_wrow(w.na, w.ckb);
  w.wrowb = conv_wrow(ntap - w.na, w.ckb);
  w.habytes = conv_habytes(act_bf16, w.nt, ntap, w.ckb);
  w.wbytes = w.habytes + conv_hbbytes(act_bf16, w.nt, ntap, w.ckb);
  w.nchunk = (cin + w.ck - 1) / w.ck;
  w.nntile = (cout + w.nt - 1) / w.nt;
  w.total = (long)w.nntile * w.nchunk * w.wbytes;
  return w;
}

// byte offset of weight (co, tap, ci) inside the image (element size esz)
inline __host__ __device__ long conv_wimg_off(const WImg& w, int co, int tap, int ci, int esz) {
  const int tile = co / w.nt, n = co - tile * w.nt;
  const int ch = ci / w.ck, k = ci - ch * w.ck;
  const long base = ((long)tile * w.nchunk + ch) * w.wbytes + (long)k * esz;
  if (tap < w.na) return base + (long)n * w.wrowa + (long)tap * w.ckb;
  return base + w.habytes + (long)n * w.wrowb + (long)(tap - w.na) * w.ckb;
}

// ---- fp8 weight image (GT_BF16_W8: e4m3 weights, bf16 activations) for the 3x3 / strided / transposed
// convs. Same tiling as above with 1-byte weights and no row pad: row n = NTAP taps x 16 B (16 input
// channels) = 2*NTAP 8-byte units u = (tap, channels 8h..8h+7), stored at u ^ conv8_swz(NTAP, n).
// The B fragment is a ds_read_b64: 32 lanes (32 rows, one unit each) per bank group, which must fall on
// 32 different 8-byte bank units of the 256-B bank row. 3x3 (144-B rows): rows r and r+16 coincide, so
// rows with bit 4 set swap the two halves of a tap (u ^ 1); 2x2 (64-B rows): rows r, r+4, ..., r+28
// coincide, so u ^ ((r >> 2) & 7). The slab is a whole number of 1 KiB DMA pieces (9 / 18 for 3x3,
// 4 / 8 for the 2x2 sub-pixel convs).
inline __host__ __device__ constexpr int conv8_swz(int ntap, int n) { return ntap == 4 ? (n >> 2) & 7 : (n >> 4) & 1; }
inline __host__ __device__ constexpr int conv8_wrow(int ntap) { return ntap * 16; }
inline __host__ __device__ constexpr int conv8_wbytes(int nt, int ntap) { return ((nt * conv8_wrow(ntap) + 1023) / 1024) * 1024; }

inline __host__ __device__ WImg conv_wimg8(int ntap, int cin, int cout) {
  WImg w;
  w.nt = conv_nt(1, cout);
  w.ckb = 16;
  w.ck = 16;
  w.ntap = ntap;
  w.na = ntap;
  w.wrowa = conv8_wrow(ntap);
  w.wrowb = 0;
  w.wbytes = w.habytes = conv8_wbytes(w.nt, ntap);
  w.nchunk = (cin + w.ck - 1) / w.ck;
  w.nntile = (cout + w.nt - 1) / w.nt;
  w.total = (long)w.nntile * w.nchunk * w.wbytes;
  return w;
}

inline __host__ __device__ long conv_wimg8_off(const WImg& w, int co, int tap, int ci) {
  const int tile = co / w.nt, n = co - tile * w.nt;
  const int ch = ci / 16, k = ci & 15;
  const int unit = (2 * tap + (k >> 3)) ^ conv8_swz(w.ntap, n);
  return ((long)tile * w.nchunk + ch) * w.wbytes + (long)n * w.wrowa + unit * 8 + (k & 7);
}

// ---- fp8 weight image for fp8 ACTIVATIONS too (GT_FP8: v_mfma_scale_f32_32x32x64_f8f6f4) of the stride-1 3x3 convs
// over activations. Chunks of 32 input channels (one E8M0 scale block of the operand); 10 tap slots of 32 B (channels
// 0..31 of the chunk; slot 9 is zero: the K = 64 MFMA takes the taps in pairs (0,1) (2,3) (4,5) (6,7) (8,9)), split
// like the bf16 images into half A = slots 0..5 (pairs 0-2) and half B = slots 6..9 (pairs 3-4), each row padded by
// 16 B to an odd number of 16-B slots (208 / 144 B: conflict-free ds_read_b128 fragments) and each half to whole
// 4 KiB (wave-even DMA pieces): conv_kernel stages one half of chunk c+1 while the other half of chunk c is in the
// MFMAs. NT = 128: 28 + 20 KiB, NT = 64: 16 + 12 KiB.
constexpr int CONVA8_SLOTS_A = 6, CONVA8_WROWA = CONVA8_SLOTS_A * 32 + 16, CONVA8_WROWB = (10 - CONVA8_SLOTS_A) * 32 + 16;
inline __host__ __device__ WImg conv_wimga8(int cin, int cout) {
  WImg w;
  w.nt = conv_nt(1, cout);
  w.ckb = 32;
  w.ck = 32;
  w.ntap = 9;
  w.na = CONVA8_SLOTS_A;
  w.wrowa = CONVA8_WROWA;
  w.wrowb = CONVA8_WROWB;
  w.habytes = round4k(w.nt * CONVA8_WROWA);
  w.wbytes = w.habytes + round4k(w.nt * CONVA8_WROWB);
  w.nchunk = (cin + w.ck - 1) / w.ck;
  w.nntile = (cout + w.nt - 1) / w.nt;
  w.total = (long)w.nntile * w.nchunk * w.wbytes;
  return w;
}
inline __host__ __device__ long conv_wimga8_off(const WImg& w, int co, int tap, int ci) {
  const int tile = co / w.nt, n = co - tile * w.nt;
  const long base = ((long)tile * w.nchunk + ci / 32) * w.wbytes + (ci & 31);
  if (tap < w.na) return base + (long)n * w.wrowa + tap * 32;
  return base + w.habytes + (long)n * w.wrowb + (tap - w.na) * 32;
}

}  // namespace gt
