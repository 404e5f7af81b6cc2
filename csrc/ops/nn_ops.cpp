// Torch op layer for the non-spectral FourCastNet helpers: patchify / un-patchify.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

namespace amd_dft {
void launch_patch_remap(const void* src, void* dst, int64_t B, int C, int h, int w, bool to_tokens, void* stream);

namespace {

// x [B, C, h*p, w*p] -> [B*h*w, C*p*p]
at::Tensor patchify_cpu(const at::Tensor& x, int64_t p) {
  const int64_t B = x.size(0), C = x.size(1), h = x.size(2) / p, w = x.size(3) / p;
  return x.reshape({B, C, h, p, w, p}).permute({0, 2, 4, 1, 3, 5}).reshape({B * h * w, C * p * p}).contiguous();
}

// t [B, h, w, C*p*p] (feature order (c, py, px)) -> [B, C, h*p, w*p]
at::Tensor unpatchify_cpu(const at::Tensor& t, int64_t C, int64_t h, int64_t w, int64_t p) {
  const int64_t B = t.numel() / (h * w * C * p * p);
  return t.reshape({B, h, w, C, p, p}).permute({0, 3, 1, 4, 2, 5}).reshape({B, C, h * p, w * p}).contiguous();
}

bool vec_ok(const at::Tensor& x, int64_t p) {
  return x.scalar_type() == at::kBFloat16 && p == 8 && x.is_contiguous() &&
         reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0;
}

at::Tensor patchify_cuda(const at::Tensor& x_, int64_t p) {
  TORCH_CHECK(x_.dim() == 4 && x_.size(2) % p == 0 && x_.size(3) % p == 0, "patchify: x must be [B, C, h*p, w*p]");
  const c10::DeviceGuard guard(x_.device());
  at::Tensor x = x_.contiguous();
  if (!vec_ok(x, p)) return patchify_cpu(x, p);
  const int64_t B = x.size(0), C = x.size(1), h = x.size(2) / p, w = x.size(3) / p;
  at::Tensor out = at::empty({B * h * w, C * p * p}, x.options());
  launch_patch_remap(x.data_ptr(), out.data_ptr(), B, static_cast<int>(C), static_cast<int>(h), static_cast<int>(w), true,
                     c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return out;
}

at::Tensor unpatchify_cuda(const at::Tensor& t_, int64_t C, int64_t h, int64_t w, int64_t p) {
  TORCH_CHECK(t_.numel() % (h * w * C * p * p) == 0, "unpatchify: size mismatch");
  const c10::DeviceGuard guard(t_.device());
  at::Tensor t = t_.contiguous();
  if (!vec_ok(t, p)) return unpatchify_cpu(t, C, h, w, p);
  const int64_t B = t.numel() / (h * w * C * p * p);
  at::Tensor out = at::empty({B, C, h * p, w * p}, t.options());
  launch_patch_remap(t.data_ptr(), out.data_ptr(), B, static_cast<int>(C), static_cast<int>(h), static_cast<int>(w), false,
                     c10::hip::getCurrentHIPStream(t.device().index()).stream());
  return out;
}

at::Tensor patchify_meta(const at::Tensor& x, int64_t p) {
  const int64_t B = x.size(0), C = x.size(1), h = x.size(2) / p, w = x.size(3) / p;
  return at::empty({B * h * w, C * p * p}, x.options());
}
at::Tensor unpatchify_meta(const at::Tensor& t, int64_t C, int64_t h, int64_t w, int64_t p) {
  return at::empty({t.numel() / (h * w * C * p * p), C, h * p, w * p}, t.options());
}

}  // namespace
}  // namespace amd_dft

TORCH_LIBRARY_FRAGMENT(amd_dft, m) {
  m.def("patchify(Tensor x, int p) -> Tensor");
  m.def("unpatchify(Tensor t, int C, int h, int w, int p) -> Tensor");
}
TORCH_LIBRARY_IMPL(amd_dft, CUDA, m) {
  m.impl("patchify", &amd_dft::patchify_cuda);
  m.impl("unpatchify", &amd_dft::unpatchify_cuda);
}
TORCH_LIBRARY_IMPL(amd_dft, CPU, m) {
  m.impl("patchify", &amd_dft::patchify_cpu);
  m.impl("unpatchify", &amd_dft::unpatchify_cpu);
}
TORCH_LIBRARY_IMPL(amd_dft, Meta, m) {
  m.impl("patchify", &amd_dft::patchify_meta);
  m.impl("unpatchify", &amd_dft::unpatchify_meta);
}
