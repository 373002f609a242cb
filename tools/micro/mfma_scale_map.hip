// Discovery of the K correspondence between A and B fragment bytes of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3, unit
// scales): A = one-hot at fragment position (h, j) in every lane of half h; B byte (h', j') = a distinct value v(h', j').
// D (every element) = v of the B position that multiplies A's one-hot K.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
__global__ void probe(const unsigned char* b, const int* one, float* d) {
  const int l = threadIdx.x, h = l >> 5;
  v8i B;
  memcpy(&B, b + l * 32, 32);
  const int s = one[0];   // 127 from memory
  for (int pa = 0; pa < 64; ++pa) {
    unsigned char a[32] = {};
    if ((pa >> 5) == h) a[pa & 31] = 0x38;   // 1.0 in e4m3
    v8i A;
    memcpy(&A, a, 32);
    v16f c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 0, 0, 0, s, 0, s);
    d[pa * 64 + l] = c[0];
  }
}
static unsigned char e4m3(float v) {
  const unsigned s = v < 0 ? 0x80 : 0; float a = std::fabs(v); int e = (int)std::floor(std::log2(a));
  int mi = (int)std::lround((a / std::ldexp(1.f, e) - 1.f) * 8); if (mi == 8) { mi = 0; ++e; }
  return (unsigned char)(s | ((e + 7) << 3) | mi);
}
int main() {
  std::vector<float> vals;
  for (int i = 1; i <= 16; ++i) vals.push_back(i);
  for (int i = 18; i <= 32; i += 2) vals.push_back(i);
  for (int i = 36; i <= 64; i += 4) vals.push_back(i);
  const int nv = (int)vals.size();   // 32 positive values; negatives for the second half
  std::vector<unsigned char> hb(64 * 32);
  float vb[64];
  for (int p = 0; p < 64; ++p) vb[p] = p < nv ? vals[p] : -vals[p - nv];
  for (int l = 0; l < 64; ++l) for (int j = 0; j < 32; ++j) hb[l * 32 + j] = e4m3(vb[(l >> 5) * 32 + j]);
  unsigned char* db; int* done; float* dd; int one = 127;
  hipMalloc(&db, 2048); hipMalloc(&done, 4); hipMalloc(&dd, 64 * 64 * 4);
  hipMemcpy(db, hb.data(), 2048, hipMemcpyHostToDevice); hipMemcpy(done, &one, 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, db, done, dd);
  std::vector<float> hd(64 * 64);
  hipMemcpy(hd.data(), dd, hd.size() * 4, hipMemcpyDeviceToHost);
  int ident = 0;
  for (int pa = 0; pa < 64; ++pa) {
    const float v = hd[pa * 64];   // lane 0, reg 0
    int pb = -1;
    for (int p = 0; p < 64; ++p) if (vb[p] == v) pb = p;
    bool uniform = true;
    for (int l = 0; l < 64; ++l) uniform &= hd[pa * 64 + l] == v;
    printf("A(h%d,j%2d) -> B(h%d,j%2d)%s%s", pa >> 5, pa & 31, pb >> 5, pb & 31, uniform ? "" : " [not uniform]", (pa % 4 == 3) ? "\n" : "   ");
    ident += pb == pa;
  }
  printf("identity positions: %d of 64\n", ident);
  return 0;
}
