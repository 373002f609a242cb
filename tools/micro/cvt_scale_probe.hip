// Semantics of gfx950 v_cvt_scalef32_pk_fp8_{f32,bf16}: is the fp32 scale operand divided out or multiplied in?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short v2s __attribute__((ext_vector_type(2)));
__global__ void k(const float* in, const float* sc, unsigned* out) {
  const int i = threadIdx.x;   // i: scale index
  v2s o = {0, 0};
  o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, in[0], in[1], sc[i], false);
  const bf16x2 b = {(__bf16)in[0], (__bf16)in[1]};
  o = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o, b, sc[i], true);
  out[i] = __builtin_bit_cast(unsigned, o);
}
static float e4m3(unsigned char c) {
  const int s = c >> 7, e = (c >> 3) & 15, m = c & 7;
  const float v = e ? (1 + m / 8.f) * __builtin_ldexpf(1.f, e - 7) : m / 8.f * __builtin_ldexpf(1.f, -6);
  return s ? -v : v;
}
int main() {
  float hin[2] = {8.f, 3.f}, hsc[3] = {1.f, 2.f, 0.5f};
  float *din, *dsc; unsigned* dout; unsigned hout[3];
  hipMalloc(&din, 8); hipMalloc(&dsc, 12); hipMalloc(&dout, 12);
  hipMemcpy(din, hin, 8, hipMemcpyHostToDevice); hipMemcpy(dsc, hsc, 12, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(3), 0, 0, din, dsc, dout);
  hipMemcpy(hout, dout, 12, hipMemcpyDeviceToHost);
  for (int i = 0; i < 3; ++i)
    printf("scale %g: f32 path (8, 3) -> (%g, %g); bf16 path -> (%g, %g)\n", hsc[i], e4m3(hout[i] & 255),
           e4m3((hout[i] >> 8) & 255), e4m3((hout[i] >> 16) & 255), e4m3(hout[i] >> 24));
  return 0;
}
