// Times the library's GroupNorm/Mish elementwise kernels (misc.hip, compiled in) at the bench's level
// shapes, standalone: hipcc --offload-arch=gfx950 -O3 -x hip -I include -I grad-tts_amd/csrc
//   tools/micro/gn_bench.cpp -o /tmp/gnb [-DGT_... variant flags]
#include "../../grad-tts_amd/csrc/misc.hip"

#include <cstdio>
#include <vector>

using namespace gt;

int main() {
  const int B = 32, T0 = 512;
  struct L { int lvl, C; } levels[3] = {{0, 64}, {1, 128}, {2, 256}};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (auto lv : levels) {
    const int F = 80 >> lv.lvl, T = T0 >> lv.lvl, C = lv.C;
    const long n = (long)B * F * T * C;
    void *pre, *x, *out;
    float *part, *gamma, *beta, *mask, *tb;
    const int nparts = (F / 4) * ((T + 63) / 64) * (C / (C >= 128 ? 128 : 64));
    (void)hipMalloc(&pre, n * 2); (void)hipMalloc(&x, n * 2); (void)hipMalloc(&out, n * 2);
    (void)hipMalloc(&part, (size_t)B * nparts * 16 * 4);
    (void)hipMalloc(&gamma, C * 4); (void)hipMalloc(&beta, C * 4); (void)hipMalloc(&mask, B * T0 * 4);
    (void)hipMalloc(&tb, C * 4);
    (void)hipMemset(pre, 0, n * 2); (void)hipMemset(x, 0, n * 2);
    std::vector<float> hp((size_t)B * nparts * 16, 1.f), hm((size_t)B * T0, 1.f);
    (void)hipMemcpy(part, hp.data(), hp.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(mask, hm.data(), hm.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemset(gamma, 0, C * 4); (void)hipMemset(beta, 0, C * 4); (void)hipMemset(tb, 0, C * 4);
    RbOutParams p{};
    p.pre = pre; p.part = part; p.nparts = nparts; p.gamma = gamma; p.beta = beta; p.count = (long)(C / 8) * F * T;
    p.x = x; p.out = out; p.mask = mask; p.B = B; p.F = F; p.T = T; p.C = C; p.T0 = T0; p.lvl = lv.lvl;
    p.tb = tb; p.tb_bstride = 0;
    for (int mode = 0; mode < 2; ++mode) {
      RbOutParams q = p;
      if (mode == 1) q.out = pre;   // gn_apply is in place
      auto launch = [&] { return mode ? launch_gn_apply(1, q, 0) : launch_rbout_identity(1, q, 0); };
      for (int i = 0; i < 3; ++i) (void)launch();
      (void)hipEventRecord(a);
      for (int i = 0; i < 20; ++i) (void)launch();
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      ms /= 20;
      const double bytes = (mode ? 2.0 : 3.0) * n * 2;
      printf("%-14s C=%3d F=%2d: %7.1f us  %5.2f TB/s\n", mode ? "gn_apply" : "rbout_identity", C, F, ms * 1e3,
             bytes / (ms * 1e-3) / 1e12);
    }
    (void)hipFree(pre); (void)hipFree(x); (void)hipFree(out); (void)hipFree(part);
    (void)hipFree(gamma); (void)hipFree(beta); (void)hipFree(mask); (void)hipFree(tb);
  }
  return 0;
}
