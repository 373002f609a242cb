// PyTorch custom-op registration of the C ABI (include/gradtts.h): torch.ops.gradtts.*
//
//   gradtts::reverse_diffusion(int decoder, int dtype, Tensor z, Tensor mask, Tensor mu, int n_timesteps,
//                              Tensor? spk) -> Tensor          Diffusion.reverse_diffusion, model/diffusion.py:254-268
//   gradtts::estimator(int decoder, int dtype, Tensor x, Tensor mask, Tensor mu, Tensor t, Tensor? spk) -> Tensor
//                                                             GradLogPEstimator2d.forward, model/diffusion.py:174-216
//   gradtts::maximum_path(Tensor value, Tensor mask) -> Tensor monotonic_align.maximum_path, __init__.py:8-23
//   gradtts::bind(str library_path) -> ()                     resolve the C ABI (once per process)
//
// `decoder` is the gt_decoder* of the module that owns the weights (gradtts_amd.diffusion keeps it and syncs the
// parameters before the call); `dtype` is GT_F32 / GT_BF16 / GT_BF16_W8. The HIP (dispatch key CUDA) kernels
// run on the current HIP stream with workspace from PyTorch's caching allocator on that stream; the Meta kernels
// give shapes and dtypes to torch.compile's fake tensors. Errors raise (TORCH_CHECK) with gt_last_error().
// The C ABI is looked up with dlsym in the library libgradtts.so that the Python package loaded (the same path,
// so the same instance: no second copy of the decoder state and no link-time dependency).
#include <dlfcn.h>

#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "gradtts.h"

namespace {

struct Api {
  decltype(&gt_last_error) last_error = nullptr;
  decltype(&gt_decoder_workspace_bytes) ws_bytes = nullptr;
  decltype(&gt_reverse_diffusion) reverse = nullptr;
  decltype(&gt_estimator_forward) estimator = nullptr;
  decltype(&gt_maximum_path_workspace_bytes) mas_ws = nullptr;
  decltype(&gt_maximum_path) mas = nullptr;
};
Api g_api;

const Api& api() {
  TORCH_CHECK(g_api.reverse != nullptr, "gradtts ops: call torch.ops.gradtts.bind(<path of libgradtts.so>) first");
  return g_api;
}

void bind(c10::string_view path) {
  void* h = dlopen(std::string(path).c_str(), RTLD_NOW | RTLD_GLOBAL);
  TORCH_CHECK(h != nullptr, "gradtts ops: dlopen failed: ", dlerror());
  Api a;
  auto sym = [&](const char* n) {
    void* p = dlsym(h, n);
    TORCH_CHECK(p != nullptr, "gradtts ops: missing symbol ", n);
    return p;
  };
  a.last_error = reinterpret_cast<decltype(a.last_error)>(sym("gt_last_error"));
  a.ws_bytes = reinterpret_cast<decltype(a.ws_bytes)>(sym("gt_decoder_workspace_bytes"));
  a.reverse = reinterpret_cast<decltype(a.reverse)>(sym("gt_reverse_diffusion"));
  a.estimator = reinterpret_cast<decltype(a.estimator)>(sym("gt_estimator_forward"));
  a.mas_ws = reinterpret_cast<decltype(a.mas_ws)>(sym("gt_maximum_path_workspace_bytes"));
  a.mas = reinterpret_cast<decltype(a.mas)>(sym("gt_maximum_path"));
  g_api = a;
}

void check_decoder_io(const at::Tensor& x, const at::Tensor& mask, const at::Tensor& mu, const char* xname) {
  TORCH_CHECK(x.dim() == 3 && x.size(1) == 80, "gradtts: ", xname, " must be [B, 80, T], got ", x.sizes());
  TORCH_CHECK(mu.sizes() == x.sizes(), "gradtts: mu must match ", xname, " ", x.sizes(), ", got ", mu.sizes());
  TORCH_CHECK(mask.dim() == 3 && mask.size(0) == x.size(0) && mask.size(1) == 1 && mask.size(2) == x.size(2),
              "gradtts: mask must be [B, 1, T], got ", mask.sizes());
  TORCH_CHECK(x.size(2) % 4 == 0, "gradtts: T must be a multiple of 4 (fix_len_compatibility, model/utils.py:13-17)");
  TORCH_CHECK(x.is_floating_point() && mu.is_floating_point() && mask.is_floating_point(),
              "gradtts: floating-point inputs expected");
}

at::Tensor f32c(const at::Tensor& t, const at::Device& dev) { return t.to(dev, at::kFloat).contiguous(); }

hipStream_t stream_of(const at::Device& dev) { return c10::hip::getCurrentHIPStream(dev.index()).stream(); }

// Masks are 0/1 (sequence_mask, model/utils.py:6-10; the reference's callers never build others). The decoder's fused
// kernels rely on it: the reference masks some operands twice (Block: (Mish(GN(h))*m + tb)*m, diffusion.py:56-58,
// 74-77), which the library computes as one multiply -- exact for 0/1 masks, 40-60 % off for fractional ones. A
// fractional mask is therefore rejected here instead of decoded wrongly. The check reads one flag back (a host
// sync); inside a HIP-graph capture, where no host read is allowed, it is skipped (the captured call was checked when
// its inputs were made, or is the caller's contract).
void check_binary_mask(const at::Tensor& m32, hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return;
  const bool bad = (m32.ne(0) & m32.ne(1)).any().item<bool>();
  TORCH_CHECK(!bad, "gradtts: mask values must be 0 or 1 (sequence_mask); fractional masks are not supported by the "
              "fused decoder (the reference's double masking x*m*m is computed as x*m)");
}

at::Tensor reverse_diffusion_hip(int64_t decoder, int64_t dtype, const at::Tensor& z, const at::Tensor& mask,
                                 const at::Tensor& mu, int64_t n_timesteps, const std::optional<at::Tensor>& spk) {
  check_decoder_io(z, mask, mu, "z");
  TORCH_CHECK(n_timesteps >= 0 && n_timesteps < (int64_t(1) << 31), "gradtts: bad n_timesteps ", n_timesteps);
  const at::Device dev = z.device();
  c10::DeviceGuard guard(dev);
  const int64_t B = z.size(0), T = z.size(2);
  at::Tensor z32 = f32c(z, dev), m32 = f32c(mask, dev), mu32 = f32c(mu, dev);
  at::Tensor s32;
  if (spk.has_value()) s32 = f32c(*spk, dev);
  at::Tensor out = at::empty({B, 80, T}, z32.options());
  if (B == 0) return out.to(z.scalar_type());
  check_binary_mask(m32, stream_of(dev));
  auto* d = reinterpret_cast<gt_decoder*>(decoder);
  const Api& A = api();
  const size_t nb = A.ws_bytes(d, (int)dtype, B, T, (int32_t)n_timesteps);
  at::Tensor ws = at::empty({(int64_t)nb}, z32.options().dtype(at::kByte));
  const int rc = A.reverse(d, (int)dtype, z32.data_ptr<float>(), m32.data_ptr<float>(), mu32.data_ptr<float>(),
                           s32.defined() ? s32.data_ptr<float>() : nullptr, B, T, (int32_t)n_timesteps,
                           out.data_ptr<float>(), ws.data_ptr(), nb, stream_of(dev));
  TORCH_CHECK(rc == GT_OK, "gt_reverse_diffusion failed (code ", rc, "): ", A.last_error());
  return out.to(z.scalar_type());
}

at::Tensor estimator_hip(int64_t decoder, int64_t dtype, const at::Tensor& x, const at::Tensor& mask,
                         const at::Tensor& mu, const at::Tensor& t, const std::optional<at::Tensor>& spk) {
  check_decoder_io(x, mask, mu, "x");
  const at::Device dev = x.device();
  c10::DeviceGuard guard(dev);
  const int64_t B = x.size(0), T = x.size(2);
  TORCH_CHECK(t.numel() == B || t.numel() == 1, "gradtts: t must have B or 1 elements, got ", t.numel());
  at::Tensor x32 = f32c(x, dev), m32 = f32c(mask, dev), mu32 = f32c(mu, dev);
  at::Tensor t32 = f32c(t.reshape({-1}).expand({B}), dev);
  at::Tensor s32;
  if (spk.has_value()) s32 = f32c(*spk, dev);
  at::Tensor out = at::empty({B, 80, T}, x32.options());
  if (B == 0) return out.to(x.scalar_type());
  check_binary_mask(m32, stream_of(dev));
  auto* d = reinterpret_cast<gt_decoder*>(decoder);
  const Api& A = api();
  const size_t nb = A.ws_bytes(d, (int)dtype, B, T, 0);
  at::Tensor ws = at::empty({(int64_t)nb}, x32.options().dtype(at::kByte));
  const int rc = A.estimator(d, (int)dtype, x32.data_ptr<float>(), m32.data_ptr<float>(), mu32.data_ptr<float>(),
                             t32.data_ptr<float>(), s32.defined() ? s32.data_ptr<float>() : nullptr, B, T,
                             out.data_ptr<float>(), ws.data_ptr(), nb, stream_of(dev));
  TORCH_CHECK(rc == GT_OK, "gt_estimator_forward failed (code ", rc, "): ", A.last_error());
  return out.to(x.scalar_type());
}

// maximum_path (monotonic_align/__init__.py:8-23): value * mask in fp32, t_x = mask.sum(1)[:, 0],
// t_y = mask.sum(2)[:, 0], the DP on device; the path comes back as value.dtype.
at::Tensor maximum_path_hip(const at::Tensor& value, const at::Tensor& mask) {
  TORCH_CHECK(value.dim() == 3 && mask.sizes() == value.sizes(), "gradtts: value and mask must both be [b, t_x, t_y]");
  const at::Device dev = value.device();
  c10::DeviceGuard guard(dev);
  at::Tensor v = (value * mask.to(dev)).to(at::kFloat).contiguous();
  at::Tensor m = mask.to(dev);
  at::Tensor t_x = m.sum(1).select(1, 0).to(at::kInt).contiguous();
  at::Tensor t_y = m.sum(2).select(1, 0).to(at::kInt).contiguous();
  at::Tensor path = at::empty(v.sizes(), v.options().dtype(at::kInt));
  if (v.numel() > 0) {
    const Api& A = api();
    const int64_t b = v.size(0), tx = v.size(1), ty = v.size(2);
    const size_t nb = A.mas_ws(b, tx, ty);
    at::Tensor ws = at::empty({(int64_t)std::max<size_t>(nb, 1)}, v.options().dtype(at::kByte));
    const int rc = A.mas(path.data_ptr<int32_t>(), v.data_ptr<float>(), t_x.data_ptr<int32_t>(),
                         t_y.data_ptr<int32_t>(), b, tx, ty, -1e9f, ws.data_ptr(), (size_t)ws.numel(), stream_of(dev));
    TORCH_CHECK(rc == GT_OK, "gt_maximum_path failed (code ", rc, "): ", A.last_error());
  }
  return path.to(value.scalar_type());
}

// ---- Meta kernels (shapes / dtypes only)
at::Tensor reverse_diffusion_meta(int64_t, int64_t, const at::Tensor& z, const at::Tensor& mask, const at::Tensor& mu,
                                  int64_t, const std::optional<at::Tensor>&) {
  check_decoder_io(z, mask, mu, "z");
  return at::empty_like(z);
}
at::Tensor estimator_meta(int64_t, int64_t, const at::Tensor& x, const at::Tensor& mask, const at::Tensor& mu,
                          const at::Tensor&, const std::optional<at::Tensor>&) {
  check_decoder_io(x, mask, mu, "x");
  return at::empty_like(x);
}
at::Tensor maximum_path_meta(const at::Tensor& value, const at::Tensor& mask) {
  TORCH_CHECK(value.dim() == 3 && mask.sizes() == value.sizes(), "gradtts: value and mask must both be [b, t_x, t_y]");
  return at::empty_like(value);
}

}  // namespace

TORCH_LIBRARY(gradtts, m) {
  m.def("bind(str library_path) -> ()", &bind);
  m.def("reverse_diffusion(int decoder, int dtype, Tensor z, Tensor mask, Tensor mu, int n_timesteps, Tensor? spk) -> Tensor");
  m.def("estimator(int decoder, int dtype, Tensor x, Tensor mask, Tensor mu, Tensor t, Tensor? spk) -> Tensor");
  m.def("maximum_path(Tensor value, Tensor mask) -> Tensor");
}

TORCH_LIBRARY_IMPL(gradtts, CUDA, m) {
  m.impl("reverse_diffusion", &reverse_diffusion_hip);
  m.impl("estimator", &estimator_hip);
  m.impl("maximum_path", &maximum_path_hip);
}

TORCH_LIBRARY_IMPL(gradtts, Meta, m) {
  m.impl("reverse_diffusion", &reverse_diffusion_meta);
  m.impl("estimator", &estimator_meta);
  m.impl("maximum_path", &maximum_path_meta);
}
