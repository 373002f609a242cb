// Which A elements does the scale operand of lane L scale? A = all ones, B = ones; scale_a = 127 everywhere except
// lane L (128 = x2): D[row][col] - 64 reveals the scaled (row, k) set through D's row.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
__global__ void probe(const int* base, float* d) {
  const int l = threadIdx.x;
  v8i A, B;
  for (int i = 0; i < 8; ++i) { A[i] = 0x38383838; B[i] = 0x38383838; }   // all 1.0
  for (int L = 0; L < 64; ++L) {
    const int sa = (l == L) ? base[0] + 1 : base[0];
    v16f c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 0, 0, 0, sa, 0, base[0]);
    for (int q = 0; q < 16; ++q) d[(L * 64 + l) * 16 + q] = c[q];
  }
}
int main() {
  int* db; float* dd; int one = 127;
  hipMalloc(&db, 4); hipMalloc(&dd, 64 * 64 * 16 * 4);
  hipMemcpy(db, &one, 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, db, dd);
  std::vector<float> hd(64 * 64 * 16);
  hipMemcpy(hd.data(), dd, hd.size() * 4, hipMemcpyDeviceToHost);
  for (int L = 0; L < 64; L += 7) {
    // rows whose D exceeds 64 (the scaled K-block adds 32 more per row)
    printf("scale_a of lane %2d raises D rows:", L);
    for (int row = 0; row < 32; ++row) {
      const int l = 4 * 0 + (row & 4 ? 32 : 0), q = (row & 3) + 4 * (row >> 3);   // col 0 element of that row
      const float v = hd[(L * 64 + (row & 4 ? 32 : 0)) * 16 + q];
      if (v != 64.f) printf(" %d(%g)", row, v);
    }
    printf("\n");
  }
  return 0;
}
