// Probe of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3, E8M0 block scales) on gfx950: operand lane maps and the
// scale granularity, checked against a host reference with exact data (small integers and powers of two, so every
// product and sum is exact in fp32). Measured on MI355X (this probe and mfma_scale_map.hip):
//   * A lane (r, h) byte j and B lane (c, h) byte j meet in the same K: the K correspondence is the identity;
//   * the scale operand (E8M0, byte 0) of lane (r, h) scales bytes [16 h', 16 h' + 16) ... of BOTH lane halves: it
//     covers the bytes j with j / 16 == h of lanes (r, 0) and (r, 1) -- NOT the 32 bytes lane (r, h) holds. With
//     K = 32 h + j the scaled blocks are {k : (k / 16) & 1 == h} (case "ref block = (k/16)&1" below);
//   * D: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)  (the bf16 32x32 map).
// So a 32-channel scale block b of a position is laid out as lane h = 0 bytes [16 b, 16 b + 16) + lane h = 1 bytes
// [16 b, 16 b + 16) (csrc/conv8.hip).
// Build: hipcc --offload-arch=gfx950 -O2 -o mfma_scale_probe tools/micro/mfma_scale_probe.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void probe(const unsigned char* a, const unsigned char* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  v8i A, B;
  memcpy(&A, a + l * 32, 32);
  memcpy(&B, b + l * 32, 32);
  v16f c = {};
  const int scale_a = sa[l], scale_b = sb[l];   // E8M0 in byte 0, from memory (never a compile-time constant)
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 0, 0, 0, scale_a, 0, scale_b);
  for (int q = 0; q < 16; ++q) d[l * 16 + q] = c[q];
}

static unsigned char to_e4m3(float v) {   // exact for the values used (|v| small integer or power of two)
  if (v == 0.f) return 0;
  const unsigned s = v < 0 ? 0x80 : 0;
  float a = std::fabs(v);
  int e = (int)std::floor(std::log2(a));
  float m = a / std::ldexp(1.f, e) - 1.f;   // [0, 1)
  int mi = (int)std::lround(m * 8);
  if (mi == 8) { mi = 0; ++e; }
  return (unsigned char)(s | ((e + 7) << 3) | mi);
}

static int run_case(const char* name, bool vary_a, bool vary_b, bool swap_ref, int kmap = 0);
int main() {
  int bad = 0;
  bad += run_case("unit scales", false, false, false);
  bad += run_case("A scales vary", true, false, false);
  bad += run_case("B scales vary", false, true, false);
  bad += run_case("both vary", true, true, false);
  bad += run_case("both vary, reference with swapped roles", true, true, true);
  bad += run_case("A vary, ref block = 1 - k/32", true, false, false, 1);
  bad += run_case("A vary, ref block = (k/8)&1", true, false, false, 2);
  bad += run_case("A vary, ref block = (k/16)&1", true, false, false, 3);
  bad += run_case("A vary, ref block = (k/4)&1", true, false, false, 4);
  return 0;
}
static int run_case(const char* name, bool vary_a, bool vary_b, bool swap_ref, int kmap) {
  float A[32][64], B[64][32];
  int ea[32][2], eb[32][2];   // E8M0 exponents (bias 127) per (row, k-half), (col, k-half)
  srand(7);
  for (int i = 0; i < 32; ++i)
    for (int k = 0; k < 64; ++k) A[i][k] = (float)(rand() % 9 - 4);
  for (int k = 0; k < 64; ++k)
    for (int j = 0; j < 32; ++j) B[k][j] = (float)(rand() % 7 - 3);
  for (int i = 0; i < 32; ++i)
    for (int h = 0; h < 2; ++h) {
      ea[i][h] = vary_a ? 127 + rand() % 3 - 1 : 127;
      eb[i][h] = vary_b ? 127 + rand() % 3 - 1 : 127;
    }
  std::vector<unsigned char> ha(64 * 32), hb(64 * 32);
  std::vector<int> hsa(64), hsb(64);
  for (int l = 0; l < 64; ++l) {
    const int r = l & 31, h = l >> 5;
    for (int j = 0; j < 32; ++j) {
      ha[l * 32 + j] = to_e4m3(A[r][32 * h + j]);
      hb[l * 32 + j] = to_e4m3(B[32 * h + j][r]);
    }
    hsa[l] = ea[r][h];
    hsb[l] = eb[r][h];
  }
  unsigned char *da, *db; int *dsa, *dsb; float* dd;
  hipMalloc(&da, 2048); hipMalloc(&db, 2048); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dd, 64 * 16 * 4);
  hipMemcpy(da, ha.data(), 2048, hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), 2048, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa.data(), 256, hipMemcpyHostToDevice);
  hipMemcpy(dsb, hsb.data(), 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
  std::vector<float> hd(64 * 16);
  if (hipMemcpy(hd.data(), dd, hd.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
  int bad = 0;
  double maxerr = 0;
  for (int l = 0; l < 64; ++l)
    for (int q = 0; q < 16; ++q) {
      const int col = l & 31, row = (q & 3) + 8 * (q >> 2) + 4 * (l >> 5);
      double ref = 0;
      for (int k = 0; k < 64; ++k) {
        const int kb = kmap == 0 ? k / 32 : kmap == 1 ? 1 - k / 32 : kmap == 2 ? (k / 8) & 1 : kmap == 3 ? (k / 16) & 1 : (k / 4) & 1;
        if (kmap) { ref += std::ldexp((double)A[row][k], ea[row][kb] - 127) * std::ldexp((double)B[k][col], eb[col][kb] - 127); continue; }
        ref += swap_ref ? std::ldexp((double)A[row][k], eb[row][k / 32] - 127) * std::ldexp((double)B[k][col], ea[col][k / 32] - 127)
                        : std::ldexp((double)A[row][k], ea[row][k / 32] - 127) * std::ldexp((double)B[k][col], eb[col][k / 32] - 127);
      }
      const double e = std::fabs(ref - hd[l * 16 + q]);
      maxerr = e > maxerr ? e : maxerr;
      if (e > 1e-3) bad++;
    }
  printf("%-45s: %4d mismatches of 1024, max |err| %g\n", name, bad, maxerr);
  return bad;
}
