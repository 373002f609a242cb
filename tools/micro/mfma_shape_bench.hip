// Microbenchmark: the conv3w<256> phase loop (8 waves, one 512-thread workgroup per CU, 2 waves per SIMD, one
// s_barrier per phase, every operand re-read from LDS by ds_read_b128) with the same wave tile (64 channels x 160
// positions, 160 fp32 accumulator registers) on
//   SHAPE 0: v_mfma_f32_32x32x16_bf16 (20 per wave per phase: 2 k-steps x 5 row blocks x 2 channel blocks)
//   SHAPE 1: v_mfma_f32_16x16x32_bf16 (40 per wave per phase: 10 position blocks x 4 channel blocks)
// Same LDS bytes per phase (4 A + 10 B fragments of 1 KiB per wave), same MFMA cycles; random bf16 data. Prints
// TFLOP/s and the in-kernel clock (s_memtime / s_memrealtime x 100 MHz) of each shape.
// hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_shape_bench.hip -o /tmp/msb && /tmp/msb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NPH = 1024;           // phases per launch
constexpr int PLB = 416;            // patch plane stride (entries of 16 B), multiple of 16
constexpr int SMEM = 4 * 256 * 16 + 4 * PLB * 16;   // weight slot (4 planes x 256 ch) + patch (4 planes)

template <int SHAPE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void loop(const uint4* src, float* out,
                                                                                   unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < SMEM / 16; i += 512) reinterpret_cast<uint4*>(smem)[i] = src[(blockIdx.x * 977 + i) & 65535];
  __syncthreads();
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), wn = wv & 3, wm = wv >> 2;
  const char* sa = smem;
  const char* sb = smem + 4 * 256 * 16;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float res = 0.f;
  if constexpr (SHAPE == 0) {
    const int r = lane & 31, h = lane >> 5;
    f32x16 acc[5][2];
    for (int i = 0; i < 5; ++i) for (int j = 0; j < 2; ++j) for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;
    for (int ph = 0; ph < NPH; ++ph) {
      const int dr = (ph % 9) / 3, dc = ph % 3;
      bf16x8 fa[2][2], fb[2][5];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          fa[s][cb] = *reinterpret_cast<const bf16x8*>(sa + ((2 * s + h) * 256 + wn * 64 + cb * 32 + r) * 16);
#pragma unroll
        for (int rb = 0; rb < 5; ++rb)
          fb[s][rb] = *reinterpret_cast<const bf16x8*>(sb + ((2 * s + h) * PLB + (wm * 5 + rb + dr) * 34 + r + dc) * 16);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int rb = 0; rb < 5; ++rb)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][cb], fb[s][rb], acc[rb][cb], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    for (int i = 0; i < 5; ++i) for (int j = 0; j < 2; ++j) for (int k = 0; k < 16; ++k) res += acc[i][j][k];
  } else {
    const int r = lane & 15, g = lane >> 4;
    f32x4 acc[10][4];
    for (int i = 0; i < 10; ++i) for (int j = 0; j < 4; ++j) for (int k = 0; k < 4; ++k) acc[i][j][k] = 0.f;
    for (int ph = 0; ph < NPH; ++ph) {
      const int dr = (ph % 9) / 3, dc = ph % 3;
      bf16x8 fa[4], fb[10];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) fa[cb] = *reinterpret_cast<const bf16x8*>(sa + (g * 256 + wn * 64 + cb * 16 + r) * 16);
#pragma unroll
      for (int p = 0; p < 10; ++p)
        fb[p] = *reinterpret_cast<const bf16x8*>(sb + (g * PLB + (wm * 5 + p / 2 + dr) * 34 + (p & 1) * 16 + r + dc) * 16);
#pragma unroll
      for (int p = 0; p < 10; ++p)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[p][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cb], fb[p], acc[p][cb], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    for (int i = 0; i < 10; ++i) for (int j = 0; j < 4; ++j) for (int k = 0; k < 4; ++k) res += acc[i][j][k];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 512 + tid] = res;
  if (tid == 0) {   // vector stores only
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int SHAPE>
static void run(const uint4* d_src, float* d_out, unsigned long long* d_clk, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(loop<SHAPE>, dim3(256), dim3(512), 0, 0, d_src, d_out, d_clk);
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(loop<SHAPE>, dim3(256), dim3(512), 0, 0, d_src, d_out, d_clk);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  std::vector<unsigned long long> c(512);
  hipMemcpy(c.data(), d_clk, 512 * 8, hipMemcpyDeviceToHost);
  double ghz = 0;
  for (int i = 0; i < 256; ++i) ghz += (double)c[2 * i] / (double)c[2 * i + 1] * 0.1;
  ghz /= 256;
  const double flop = 256.0 * 8 * NPH * 20 * 32768.0 * reps;
  printf("shape %s: %.1f us per launch, %.1f TFLOP/s, in-kernel clock %.2f GHz, cycles/phase %.0f\n",
         SHAPE == 0 ? "32x32x16" : "16x16x32", ms * 1e3 / reps, flop / (ms * 1e-3) / 1e12, ghz,
         (double)c[0] / NPH);
}

int main() {
  std::vector<uint4> h(65536);
  srand(1);
  for (auto& v : h) {   // random bf16 in [-1, 1)
    unsigned w[4];
    for (int k = 0; k < 4; ++k) {
      unsigned lo = 0x3c00 | (rand() & 0x7f) | ((rand() & 1) << 15), hi = 0x3c00 | (rand() & 0x7f) | ((rand() & 1) << 15);
      w[k] = (lo & 0xffff) | (hi << 16);
    }
    v = make_uint4(w[0], w[1], w[2], w[3]);
  }
  uint4* d_src; float* d_out; unsigned long long* d_clk;
  hipMalloc(&d_src, 65536 * 16); hipMalloc(&d_out, 256 * 512 * 4); hipMalloc(&d_clk, 512 * 8);
  hipMemcpy(d_src, h.data(), 65536 * 16, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(d_src, d_out, d_clk, 200);
    run<1>(d_src, d_out, d_clk, 200);
  }
  return 0;
}
