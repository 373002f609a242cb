// Microbenchmark: in-place elementwise pass over a level-0 activation ([32][80][512][64] bf16, 168 MB):
//   copy      load 16 B, store 16 B (same grid/IPT as gn_mish_kernel)
//   mish      + the GroupNorm-apply Mish transform (no GN reduction)
//   ipt/grid  variants of items per thread.
// hipcc --offload-arch=gfx950 -O3 tools/micro/ew_bench.hip -o /tmp/ew && /tmp/ew
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16;
__device__ __forceinline__ float mishf(float x) {
  const float e = __expf(fminf(x, 20.f));
  const float n = e * (e + 2.f);
  return x * __fdividef(n, n + 2.f);
}
__device__ __forceinline__ void unpack(uint4 u, float* v) {
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
  for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
}
__device__ __forceinline__ uint4 pack(const float* v) {
  unsigned w[4];
  for (int i = 0; i < 4; ++i) {
    bf16 a = (bf16)v[2 * i], b = (bf16)v[2 * i + 1];
    w[i] = (unsigned)__builtin_bit_cast(unsigned short, a) | ((unsigned)__builtin_bit_cast(unsigned short, b) << 16);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}
template <int IPT, int MODE>
__global__ __launch_bounds__(256) void ew(uint4* p, long n_items, const float* sc, const float* sh) {
  const long base = (long)blockIdx.x * IPT * 256 + threadIdx.x;
  uint4 v[IPT];
#pragma unroll
  for (int i = 0; i < IPT; ++i) { long it = base + i * 256; if (it < n_items) v[i] = p[it]; }
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < IPT; ++i) { long it = base + i * 256; if (it < n_items) p[it] = v[i]; }
    return;
  }
  const int c0 = (threadIdx.x * 8) & 63;
  float s[8], h[8];
  for (int k = 0; k < 8; ++k) { s[k] = sc[c0 + k]; h[k] = sh[c0 + k]; }
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    long it = base + i * 256;
    if (it < n_items) {
      float f[8];
      unpack(v[i], f);
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = mishf(f[k] * s[k] + h[k]);
      p[it] = pack(f);
    }
  }
}
// grid-stride persistent variant with a 2-deep register pipeline
template <int IPT>
__global__ __launch_bounds__(256) void ew_pipe(uint4* p, long n_items, const float* sc, const float* sh, int nblk) {
  const int c0 = (threadIdx.x * 8) & 63;
  float s[8], h[8];
  for (int k = 0; k < 8; ++k) { s[k] = sc[c0 + k]; h[k] = sh[c0 + k]; }
  uint4 v[IPT], w[IPT];
  long blk = blockIdx.x;
  auto load = [&](uint4* dst, long b) {
#pragma unroll
    for (int i = 0; i < IPT; ++i) { long it = (b * IPT + i) * 256 + threadIdx.x; if (b < nblk && it < n_items) dst[i] = p[it]; }
  };
  load(v, blk);
  for (; blk < nblk; blk += gridDim.x) {
    load(w, blk + gridDim.x);
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
      long it = (blk * IPT + i) * 256 + threadIdx.x;
      if (it < n_items) {
        float f[8];
        unpack(v[i], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = mishf(f[k] * s[k] + h[k]);
        p[it] = pack(f);
      }
    }
#pragma unroll
    for (int i = 0; i < IPT; ++i) v[i] = w[i];
  }
}
int main() {
  const long n_elem = 32L * 80 * 512 * 64, n_items = n_elem / 8;
  uint4* p; float *sc, *sh;
  hipMalloc(&p, n_items * 16); hipMalloc(&sc, 256); hipMalloc(&sh, 256);
  hipMemset(p, 0, n_items * 16); hipMemset(sc, 0, 256); hipMemset(sh, 0, 256);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(a);
    for (int i = 0; i < 20; ++i) launch();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ms /= 20;
    printf("%-28s %8.1f us  %6.2f TB/s (read+write)\n", name, ms * 1e3, 2.0 * n_items * 16 / (ms * 1e-3) / 1e12);
  };
#define G(IPT) dim3((unsigned)((n_items + IPT * 256 - 1) / (IPT * 256)))
  run("copy ipt4", [&] { ew<4, 0><<<G(4), 256>>>(p, n_items, sc, sh); });
  run("copy ipt8", [&] { ew<8, 0><<<G(8), 256>>>(p, n_items, sc, sh); });
  run("copy ipt16", [&] { ew<16, 0><<<G(16), 256>>>(p, n_items, sc, sh); });
  run("mish ipt2", [&] { ew<2, 1><<<G(2), 256>>>(p, n_items, sc, sh); });
  run("mish ipt4", [&] { ew<4, 1><<<G(4), 256>>>(p, n_items, sc, sh); });
  run("mish ipt8", [&] { ew<8, 1><<<G(8), 256>>>(p, n_items, sc, sh); });
  run("mish ipt16", [&] { ew<16, 1><<<G(16), 256>>>(p, n_items, sc, sh); });
  for (int g : {1024, 2048, 4096}) {
    const int nblk4 = (int)((n_items + 1023) / 1024);
    char nm[64]; snprintf(nm, 64, "pipe ipt4 grid %d", g);
    run(nm, [&] { ew_pipe<4><<<g, 256>>>(p, n_items, sc, sh, nblk4); });
    const int nblk2 = (int)((n_items + 511) / 512);
    snprintf(nm, 64, "pipe ipt2 grid %d", g);
    run(nm, [&] { ew_pipe<2><<<g, 256>>>(p, n_items, sc, sh, nblk2); });
  }
  return 0;
}
