// Torch op layer for the non-spectral FourCastNet pieces: patchify / un-patchify and the
// fused-epilogue linear layer.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <algorithm>

#include "trace.h"
#include "../nn/gemm.h"
#include "../spectral/spectral.h"
#include "checks.h"

namespace amd_dft {
void launch_patch_remap(const void* src, void* dst, int64_t B, int C, int h, int w, bool to_tokens, void* stream,
                        int elem_bytes);

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
  return (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) && p == 8 && x.is_contiguous() &&
         reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0;
}

at::Tensor patchify_cuda(const at::Tensor& x_, int64_t p) {
  TORCH_CHECK(x_.dim() == 4 && x_.size(2) % p == 0 && x_.size(3) % p == 0, "patchify: x must be [B, C, h*p, w*p]");
  const c10::DeviceGuard guard(x_.device());
  at::Tensor x = x_.contiguous();
  if (!vec_ok(x, p)) {
    fallback_note("patchify", "needs bf16 / fp32, p == 8, 16-byte aligned");
    return patchify_cpu(x, p);
  }
  const int64_t B = x.size(0), C = x.size(1), h = x.size(2) / p, w = x.size(3) / p;
  at::Tensor out = at::empty({B * h * w, C * p * p}, x.options());
  launch_patch_remap(x.data_ptr(), out.data_ptr(), B, static_cast<int>(C), static_cast<int>(h), static_cast<int>(w), true,
                     c10::hip::getCurrentHIPStream(x.device().index()).stream(), static_cast<int>(x.element_size()));
  return out;
}

at::Tensor unpatchify_cuda(const at::Tensor& t_, int64_t C, int64_t h, int64_t w, int64_t p) {
  TORCH_CHECK(t_.numel() % (h * w * C * p * p) == 0, "unpatchify: size mismatch");
  const c10::DeviceGuard guard(t_.device());
  at::Tensor t = t_.contiguous();
  if (!vec_ok(t, p)) {
    fallback_note("unpatchify", "needs bf16 / fp32, p == 8, 16-byte aligned");
    return unpatchify_cpu(t, C, h, w, p);
  }
  const int64_t B = t.numel() / (h * w * C * p * p);
  at::Tensor out = at::empty({B, C, h * p, w * p}, t.options());
  launch_patch_remap(t.data_ptr(), out.data_ptr(), B, static_cast<int>(C), static_cast<int>(h), static_cast<int>(w), false,
                     c10::hip::getCurrentHIPStream(t.device().index()).stream(), static_cast<int>(t.element_size()));
  return out;
}

at::Tensor patchify_meta(const at::Tensor& x, int64_t p) {
  const int64_t B = x.size(0), C = x.size(1), h = x.size(2) / p, w = x.size(3) / p;
  return at::empty({B * h * w, C * p * p}, x.options());
}
at::Tensor unpatchify_meta(const at::Tensor& t, int64_t C, int64_t h, int64_t w, int64_t p) {
  return at::empty({t.numel() / (h * w * C * p * p), C, h * p, w * p}, t.options());
}


// ------------------------------------------------------------------ fused-epilogue linear
// y = act(x @ w^T + bias) (+ residual); x [..., K] bf16, w [N, K] bf16, y [..., N] bf16.
// act: 0 none, 1 GELU (erf).  CUDA: the hand-written MFMA GEMM (csrc/nn/gemm.hip) when
// N % 64 == 0 and K % 64 == 0 (a ragged last 256-feature panel is masked in the kernel), otherwise
// hipBLASLt through at::linear (counted: fallback_counts / MI_DFT_STRICT).
// act 3: the bf16 paths' erf GELU, x sigmoid(x q(x^2)) (csrc/nn/gelu.h: gelu_erf_fit), same constants
at::Tensor gelu_erf_fit_ref(const at::Tensor& y) {
  const at::Tensor x2 = at::clamp_max(y * y, 64.0);
  const at::Tensor z = y * (x2 * (x2 * 0.0010148165747523308 + -0.10677912831306458) + -2.3011176586151123);
  return y / (at::exp2(z) + 1.0);
}

at::Tensor apply_act_ref(const at::Tensor& y, int64_t act) {
  if (act == 1) return at::gelu(y);
  if (act == 2) return at::gelu(y, "tanh");
  if (act == 3) return gelu_erf_fit_ref(y);
  return y;
}

at::Tensor linear_ref(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t act,
                      const c10::optional<at::Tensor>& residual) {
  at::Tensor y = at::linear(x.to(at::kFloat), w.to(at::kFloat),
                            bias.has_value() && bias->defined() ? c10::optional<at::Tensor>(bias->to(at::kFloat))
                                                                : c10::nullopt);
  y = apply_act_ref(y, act);
  if (residual.has_value() && residual->defined()) y = y + residual->to(at::kFloat);
  return y.to(x.scalar_type());
}

at::Tensor linear_cpu(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t act,
                      const c10::optional<at::Tensor>& residual) {
  TORCH_CHECK(act >= 0 && act <= 3, "amd_dft.linear: act must be 0 (none), 1 (gelu), 2 (gelu, tanh form) or 3 (gelu, bf16 erf fit)");
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == w.size(0), "amd_dft.linear: bias must have N entries");
  return linear_ref(x, w, bias, act, residual);
}

at::Tensor linear_cuda(const at::Tensor& x_, const at::Tensor& w_, const c10::optional<at::Tensor>& bias,
                       int64_t act, const c10::optional<at::Tensor>& residual) {
  const c10::DeviceGuard guard(x_.device());
  TORCH_CHECK(act >= 0 && act <= 3, "amd_dft.linear: act must be 0 (none), 1 (gelu), 2 (gelu, tanh form) or 3 (gelu, bf16 erf fit)");
  TORCH_CHECK(w_.dim() == 2 && x_.size(-1) == w_.size(1), "amd_dft.linear: x [..., K], w [N, K]");
  const int64_t K = w_.size(1), N = w_.size(0), M = x_.numel() / std::max<int64_t>(K, 1);
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == N, "amd_dft.linear: bias must have N entries");
  if (x_.scalar_type() != at::kBFloat16 || w_.scalar_type() != at::kBFloat16 || !gemm_supported(M, N, K))
  {
    fallback_note("linear", "needs bf16 operands, N % 64 == 0, K % 64 == 0 (fp32: use linear3)");
    return linear_ref(x_, w_, bias, act, residual);
  }
  at::Tensor x = x_.contiguous(), w = w_.contiguous();
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = N;
  at::Tensor y = at::empty(os, x.options());
  at::Tensor b, r;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->numel() == M * N, "amd_dft.linear: residual must have the output's shape");
    r = residual->to(at::kBFloat16).contiguous();
  }
  GemmLaunch p;
  p.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  p.w = reinterpret_cast<const uint16_t*>(w.data_ptr());
  p.bias = b.defined() ? b.data_ptr<float>() : nullptr;
  p.residual = r.defined() ? r.data_ptr() : nullptr;
  p.y = y.data_ptr();
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.act = static_cast<int>(act);
  launch_gemm(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return y;
}

// ------------------------------------------------------------------ LayerNorm folded into a GEMM
// linear_ln: y = act(LN(x) W^T + b) computed from the RAW rows x (no normalised copy):
//   w = W * gamma (per k, as used by the GEMM), c1[n] = sum_k w[n, k], bias = W beta + b,
//   stats[m] = (mean_m, rstd_m) of x  ->  y = act(rstd_m * (x w^T - mean_m c1) + bias).
// c1 must be summed from the same (bf16-rounded) w the GEMM reads: x w^T - mean c1 is then
// (x - mean) w exactly, with no cancellation beyond fp32 accumulation.
void check_linear_ln(const at::Tensor& x, const at::Tensor& w, const at::Tensor& c1, const c10::optional<at::Tensor>& bias,
                     const at::Tensor& stats, int64_t act) {
  TORCH_CHECK(act >= 0 && act <= 3, "amd_dft.linear_ln: act must be 0 (none), 1 (gelu), 2 (gelu, tanh form) or 3 (gelu, bf16 erf fit)");
  TORCH_CHECK(w.dim() == 2 && x.size(-1) == w.size(1), "amd_dft.linear_ln: x [..., K], w [N, K]");
  const int64_t K = w.size(1), N = w.size(0), M = x.numel() / std::max<int64_t>(K, 1);
  TORCH_CHECK(c1.numel() == N, "amd_dft.linear_ln: c1 must have N entries");
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == N, "amd_dft.linear_ln: bias must have N entries");
  TORCH_CHECK(stats.numel() == 2 * M && stats.size(-1) == 2, "amd_dft.linear_ln: stats must be [M, 2] (mean, rstd)");
}

at::Tensor linear_ln_ref(const at::Tensor& x, const at::Tensor& w, const at::Tensor& c1, const c10::optional<at::Tensor>& bias,
                         const at::Tensor& stats, int64_t act) {
  const int64_t K = w.size(1);
  at::Tensor xf = x.to(at::kFloat).reshape({-1, K});
  at::Tensor st = stats.to(at::kFloat).reshape({-1, 2});
  at::Tensor t = at::matmul(xf, w.to(at::kFloat).t());
  at::Tensor y = st.select(1, 1).unsqueeze(1) * (t - st.select(1, 0).unsqueeze(1) * c1.to(at::kFloat).reshape({1, -1}));
  if (bias.has_value() && bias->defined()) y = y + bias->to(at::kFloat).reshape({1, -1});
  y = apply_act_ref(y, act);
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = w.size(0);
  return y.reshape(os).to(x.scalar_type());
}

at::Tensor linear_ln_cpu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& c1, const c10::optional<at::Tensor>& bias,
                         const at::Tensor& stats, int64_t act) {
  check_linear_ln(x, w, c1, bias, stats, act);
  return linear_ln_ref(x, w, c1, bias, stats, act);
}

at::Tensor linear_ln_cuda(const at::Tensor& x_, const at::Tensor& w_, const at::Tensor& c1_,
                          const c10::optional<at::Tensor>& bias, const at::Tensor& stats_, int64_t act) {
  const c10::DeviceGuard guard(x_.device());
  check_linear_ln(x_, w_, c1_, bias, stats_, act);
  const int64_t K = w_.size(1), N = w_.size(0), M = x_.numel() / std::max<int64_t>(K, 1);
  if (x_.scalar_type() != at::kBFloat16 || w_.scalar_type() != at::kBFloat16 || !gemm_supported(M, N, K)) {
    fallback_note("linear_ln", "needs bf16 operands, N % 64 == 0, K % 64 == 0");
    return linear_ln_ref(x_, w_, c1_, bias, stats_, act);
  }
  at::Tensor x = x_.contiguous(), w = w_.contiguous();
  at::Tensor c1 = c1_.to(at::kFloat).contiguous(), stats = stats_.to(at::kFloat).contiguous();
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = N;
  at::Tensor y = at::empty(os, x.options());
  at::Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  GemmLaunch p;
  p.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  p.w = reinterpret_cast<const uint16_t*>(w.data_ptr());
  p.bias = b.defined() ? b.data_ptr<float>() : nullptr;
  p.y = y.data_ptr();
  p.ln_stats = stats.data_ptr<float>();
  p.ln_c1 = c1.data_ptr<float>();
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.act = static_cast<int>(act);
  launch_gemm(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return y;
}

at::Tensor linear_ln_meta(const at::Tensor& x, const at::Tensor& w, const at::Tensor&, const c10::optional<at::Tensor>&,
                          const at::Tensor&, int64_t) {
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = w.size(0);
  return at::empty(os, x.options());
}

// ------------------------------------------------------------------ patch embedding / head
// patch_linear: tokens = patchify(x) @ w^T + bias + pos[token % (h*w)]  ([B*h*w, N] bf16)
// linear_unpatch: image = unpatchify(t @ w^T + bias)                     ([B, C, h*p, w*p])
// CUDA with p == 8 and bf16: one MFMA GEMM each, the (un)patchify folded into its operand
// gather / output scatter (csrc/nn/gemm.hip MODE 1 / 2).  The reference conv / linear +
// permute path is the CPU implementation.
at::Tensor patch_linear_cpu(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                            const c10::optional<at::Tensor>& pos, int64_t p) {
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == w.size(0), "patch_linear: bias must have N entries");
  at::Tensor t = patchify_cpu(x, p);
  at::Tensor y = linear_ref(t, w, bias, 0, c10::nullopt).to(at::kFloat);
  if (pos.has_value() && pos->defined()) {
    const int64_t hw = (x.size(2) / p) * (x.size(3) / p);
    y = (y.reshape({-1, hw, w.size(0)}) + pos->to(at::kFloat).reshape({1, hw, w.size(0)})).reshape({-1, w.size(0)});
  }
  return y.to(x.scalar_type()).contiguous();
}

at::Tensor patch_linear_cuda(const at::Tensor& x_, const at::Tensor& w_, const c10::optional<at::Tensor>& bias,
                             const c10::optional<at::Tensor>& pos, int64_t p) {
  const c10::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.dim() == 4 && x_.size(2) % p == 0 && x_.size(3) % p == 0, "patch_linear: x must be [B, C, h*p, w*p]");
  TORCH_CHECK(w_.dim() == 2 && w_.size(1) == x_.size(1) * p * p, "patch_linear: w must be [N, C*p*p]");
  const int64_t B = x_.size(0), C = x_.size(1), h = x_.size(2) / p, w = x_.size(3) / p, N = w_.size(0);
  const int64_t M = B * h * w, K = C * p * p;
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == N, "patch_linear: bias must have N entries");
  const bool native = p == 8 && x_.scalar_type() == at::kBFloat16 && w_.scalar_type() == at::kBFloat16 &&
                      gemm_supported(M, N, K) && x_.numel() < (int64_t(1) << 31);
  if (!native) {  // ATen ops on the device tensors
    fallback_note("patch_linear", "needs bf16, p == 8, N % 64 == 0 (fp32: use patch_linear3)");
    return patch_linear_cpu(x_, w_, bias, pos, p);
  }
  at::Tensor x = x_.contiguous(), wc = w_.contiguous();
  at::Tensor y = at::empty({M, N}, x.options());
  at::Tensor b, r;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->numel() == h * w * N, "patch_linear: pos must be [h*w, N]");
    r = pos->to(at::kBFloat16).contiguous();
  }
  GemmLaunch g;
  g.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  g.w = reinterpret_cast<const uint16_t*>(wc.data_ptr());
  g.bias = b.defined() ? b.data_ptr<float>() : nullptr;
  g.residual = r.defined() ? r.data_ptr() : nullptr;
  g.res_rows = static_cast<int>(h * w);
  g.y = y.data_ptr();
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.K = static_cast<int>(K);
  g.gC = static_cast<int>(C);
  g.gh = static_cast<int>(h);
  g.gw = static_cast<int>(w);
  launch_gemm(g, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return y;
}

at::Tensor patch_linear_meta(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>&,
                             const c10::optional<at::Tensor>&, int64_t p) {
  return at::empty({x.size(0) * (x.size(2) / p) * (x.size(3) / p), w.size(0)}, x.options());
}

at::Tensor linear_unpatch_cpu(const at::Tensor& t, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                              int64_t C, int64_t h, int64_t wd, int64_t p) {
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == w.size(0), "linear_unpatch: bias must have N entries");
  return unpatchify_cpu(linear_ref(t, w, bias, 0, c10::nullopt), C, h, wd, p);
}

at::Tensor linear_unpatch_cuda(const at::Tensor& t_, const at::Tensor& w_, const c10::optional<at::Tensor>& bias,
                               int64_t C, int64_t h, int64_t wd, int64_t p) {
  const c10::DeviceGuard guard(t_.device());
  TORCH_CHECK(w_.dim() == 2 && t_.size(-1) == w_.size(1) && w_.size(0) == C * p * p,
              "linear_unpatch: t [..., K], w [C*p*p, K] in (c, py, px) feature order");
  const int64_t K = w_.size(1), N = w_.size(0), M = t_.numel() / std::max<int64_t>(K, 1);
  TORCH_CHECK(M % (h * wd) == 0, "linear_unpatch: token count must be a multiple of h*w");
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == N, "linear_unpatch: bias must have N entries");
  const bool native = p == 8 && t_.scalar_type() == at::kBFloat16 && w_.scalar_type() == at::kBFloat16 &&
                      gemm_supported(M, N, K) && M * N < (int64_t(1) << 31);
  if (!native) {
    fallback_note("linear_unpatch", "needs bf16, p == 8, N % 64 == 0 (fp32: use linear_unpatch3)");
    return linear_unpatch_cpu(t_, w_, bias, C, h, wd, p);
  }
  at::Tensor t = t_.contiguous(), wc = w_.contiguous();
  const int64_t B = M / (h * wd);
  at::Tensor y = at::empty({B, C, h * p, wd * p}, t.options());
  at::Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  // N % 256 != 0 (C % 4 != 0): token-major GEMM with a ragged last panel, then the remap kernel
  const bool ragged = N % 256 != 0;
  at::Tensor yt = ragged ? at::empty({M, N}, t.options()) : at::Tensor();
  GemmLaunch g;
  g.x = reinterpret_cast<const uint16_t*>(t.data_ptr());
  g.w = reinterpret_cast<const uint16_t*>(wc.data_ptr());
  g.bias = b.defined() ? b.data_ptr<float>() : nullptr;
  g.y = ragged ? yt.data_ptr() : y.data_ptr();
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.K = static_cast<int>(K);
  if (!ragged) {
    g.sC = static_cast<int>(C);
    g.sh = static_cast<int>(h);
    g.sw = static_cast<int>(wd);
  }
  auto stream = c10::hip::getCurrentHIPStream(t.device().index()).stream();
  launch_gemm(g, stream);
  if (ragged)
    launch_patch_remap(yt.data_ptr(), y.data_ptr(), B, static_cast<int>(C), static_cast<int>(h), static_cast<int>(wd),
                       false, stream, 2);
  return y;
}

at::Tensor linear_unpatch_meta(const at::Tensor& t, const at::Tensor& w, const c10::optional<at::Tensor>&, int64_t C,
                               int64_t h, int64_t wd, int64_t p) {
  return at::empty({t.numel() / w.size(1) / (h * wd), C, h * p, wd * p}, t.options());
}

at::Tensor linear_meta(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>&, int64_t,
                       const c10::optional<at::Tensor>&) {
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = w.size(0);
  return at::empty(os, x.options());
}

// ------------------------------------------------------------------ bf16x3 (fp32-class) GEMMs
// An fp32 operand is carried as a bf16 pair a = hi + lo (hi = bf16(a), lo = bf16(a - hi)):
// split_bf16 packs rows as [..., 2K] k32-interleaved (every 32 columns [hi(32) | lo(32)],
// rows=true) or planes [2, ...] (rows=false).
// linear3 / patch_linear3 / linear_unpatch3 take split operands and run the 3-product GEMM
// (csrc/nn/gemm.hip SPLIT mode) with fp32 accumulation and fp32 (or split-pair) outputs.
// k32-interleaved split rows: every 32 columns c.. stored as [hi(32) | lo(32)]
at::Tensor unsplit_rows(const at::Tensor& xs) {
  const int64_t K2 = xs.size(-1);
  TORCH_CHECK(K2 % 64 == 0, "amd_dft: split rows must have a last dim that is a multiple of 64");
  std::vector<int64_t> s(xs.sizes().begin(), xs.sizes().end() - 1);
  std::vector<int64_t> v = s;
  v.insert(v.end(), {K2 / 64, 2, 32});
  s.push_back(K2 / 2);
  return xs.to(at::kFloat).reshape(v).sum(-2).reshape(s);
}

at::Tensor split_ref(const at::Tensor& x, bool rows) {
  at::Tensor xf = x.to(at::kFloat);
  at::Tensor hi = xf.to(at::kBFloat16);
  at::Tensor lo = (xf - hi.to(at::kFloat)).to(at::kBFloat16);
  if (!rows) return at::stack({hi, lo}, 0).contiguous();
  const int64_t K = x.size(-1);
  TORCH_CHECK(K % 32 == 0, "amd_dft.split_bf16: rows need a last dim that is a multiple of 32");
  std::vector<int64_t> v(x.sizes().begin(), x.sizes().end() - 1), o = v;
  v.insert(v.end(), {K / 32, 32});
  o.push_back(2 * K);
  return at::cat({hi.reshape(v), lo.reshape(v)}, -1).reshape(o).contiguous();
}

at::Tensor split_bf16_cpu(const at::Tensor& x, bool rows) { return split_ref(x, rows); }

at::Tensor split_bf16_cuda(const at::Tensor& x_, bool rows) {
  const c10::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.scalar_type() == at::kFloat, "amd_dft.split_bf16: x must be float32");
  TORCH_CHECK(x_.dim() >= 1, "amd_dft.split_bf16: x must have at least one dim");
  at::Tensor x = x_.contiguous();
  const int64_t cols = x.size(-1);
  TORCH_CHECK(x.numel() % 8 == 0 && (!rows || cols % 32 == 0),
              "amd_dft.split_bf16: needs multiples of 8 elements (rows: a last dim that is a multiple of 32)");
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  if (rows) os.back() = 2 * cols;
  else os.insert(os.begin(), 2);
  at::Tensor y = at::empty(os, x.options().dtype(at::kBFloat16));
  launch_split_bf16(x.data_ptr<float>(), reinterpret_cast<uint16_t*>(y.data_ptr()), x.numel(), static_cast<int>(cols),
                    rows, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return y;
}

at::Tensor split_bf16_meta(const at::Tensor& x, bool rows) {
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  if (rows) os.back() = 2 * os.back();
  else os.insert(os.begin(), 2);
  return at::empty(os, x.options().dtype(at::kBFloat16));
}

void check_split_linear(const at::Tensor& xs, const at::Tensor& ws, const c10::optional<at::Tensor>& bias,
                        const char* op) {
  TORCH_CHECK(xs.scalar_type() == at::kBFloat16 && ws.scalar_type() == at::kBFloat16, "amd_dft.", op,
              ": split operands must be bfloat16 pairs");
  TORCH_CHECK(ws.dim() == 2 && ws.size(1) % 2 == 0, "amd_dft.", op, ": ws must be [N, 2K] = [hi | lo]");
  TORCH_CHECK(!bias.has_value() || !bias->defined() || bias->numel() == ws.size(0), "amd_dft.", op,
              ": bias must have N entries");
}

at::Tensor linear3_cpu(const at::Tensor& xs, const at::Tensor& ws, const c10::optional<at::Tensor>& bias, int64_t act,
                       const c10::optional<at::Tensor>& residual, bool split_out) {
  check_split_linear(xs, ws, bias, "linear3");
  TORCH_CHECK(xs.size(-1) == ws.size(1), "amd_dft.linear3: xs [..., 2K], ws [N, 2K]");
  TORCH_CHECK(act == 0 || act == 1, "amd_dft.linear3: act must be 0 (none) or 1 (gelu)");
  at::Tensor y = at::linear(unsplit_rows(xs), unsplit_rows(ws),
                            bias.has_value() && bias->defined() ? c10::optional<at::Tensor>(bias->to(at::kFloat))
                                                                : c10::nullopt);
  if (act == 1) y = at::gelu(y);
  if (residual.has_value() && residual->defined()) y = y + residual->to(at::kFloat).reshape(y.sizes());
  return split_out ? split_ref(y, true) : y.contiguous();
}

at::Tensor linear3_cuda(const at::Tensor& xs_, const at::Tensor& ws_, const c10::optional<at::Tensor>& bias,
                        int64_t act, const c10::optional<at::Tensor>& residual, bool split_out) {
  const c10::DeviceGuard guard(xs_.device());
  check_split_linear(xs_, ws_, bias, "linear3");
  TORCH_CHECK(act == 0 || act == 1, "amd_dft.linear3: act must be 0 (none) or 1 (gelu)");
  TORCH_CHECK(xs_.size(-1) == ws_.size(1), "amd_dft.linear3: xs [..., 2K], ws [N, 2K]");
  const int64_t K = ws_.size(1) / 2, N = ws_.size(0), M = xs_.numel() / std::max<int64_t>(2 * K, 1);
  TORCH_CHECK(gemm_supported(M, N, K), "amd_dft.linear3: the bf16x3 GEMM needs N % 64 == 0 and K % 64 == 0 (got N=",
              N, ", K=", K, ")");
  TORCH_CHECK(!(split_out && residual.has_value() && residual->defined() &&
                (act != 0 || (bias.has_value() && bias->defined()))),
              "amd_dft.linear3: a split-pair output takes a residual only without activation and bias");
  at::Tensor xs = xs_.contiguous(), ws = ws_.contiguous();
  std::vector<int64_t> os(xs.sizes().begin(), xs.sizes().end());
  os.back() = split_out ? 2 * N : N;
  at::Tensor y = at::empty(os, xs.options().dtype(split_out ? at::kBFloat16 : at::kFloat));
  at::Tensor b, r;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->numel() == M * N, "amd_dft.linear3: residual must have the output's shape");
    r = residual->to(at::kFloat).contiguous();
  }
  GemmLaunch p;
  p.x = reinterpret_cast<const uint16_t*>(xs.data_ptr());
  p.w = reinterpret_cast<const uint16_t*>(ws.data_ptr());
  p.bias = b.defined() ? b.data_ptr<float>() : nullptr;
  p.residual = r.defined() ? r.data_ptr() : nullptr;
  p.y = y.data_ptr();
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.act = static_cast<int>(act);
  p.split = 1;
  p.out = split_out ? 2 : 1;
  if (M > 0) launch_gemm(p, c10::hip::getCurrentHIPStream(xs.device().index()).stream());
  return y;
}

// fc2 of the fp32 FourCastNet block: y = xs ws^T + residual (bf16x3, fp32 out) and, from the same
// epilogue, the next LayerNorm's partial statistics of y + pre: part [M, N/64, 2] = per 64-feature
// chunk (mean, M2); ln_stats_merge turns them into (mean, rstd) without another pass over y
std::tuple<at::Tensor, at::Tensor> linear3_stats_cpu(const at::Tensor& xs, const at::Tensor& ws, const at::Tensor& residual,
                                                     const c10::optional<at::Tensor>& pre) {
  at::Tensor y = linear3_cpu(xs, ws, c10::nullopt, 0, residual, false);
  const int64_t N = ws.size(0);
  TORCH_CHECK(N % 64 == 0, "amd_dft.linear3_stats: N must be a multiple of 64");
  at::Tensor w = y.reshape({-1, N});
  if (pre.has_value() && pre->defined()) w = w + pre->to(at::kFloat).reshape({1, N});
  w = w.reshape({w.size(0), N / 64, 64});
  at::Tensor mean = w.mean(2);
  at::Tensor m2 = (w - mean.unsqueeze(2)).pow(2).sum(2);
  return {y, at::stack({mean, m2}, 2).contiguous()};
}

std::tuple<at::Tensor, at::Tensor> linear3_stats_cuda(const at::Tensor& xs_, const at::Tensor& ws_, const at::Tensor& residual,
                                                      const c10::optional<at::Tensor>& pre_) {
  const c10::DeviceGuard guard(xs_.device());
  check_split_linear(xs_, ws_, c10::nullopt, "linear3_stats");
  TORCH_CHECK(xs_.size(-1) == ws_.size(1), "amd_dft.linear3_stats: xs [..., 2K], ws [N, 2K]");
  const int64_t K = ws_.size(1) / 2, N = ws_.size(0), M = xs_.numel() / std::max<int64_t>(2 * K, 1);
  TORCH_CHECK(gemm_supported(M, N, K), "amd_dft.linear3_stats: the bf16x3 GEMM needs N % 64 == 0 and K % 64 == 0");
  TORCH_CHECK(residual.numel() == M * N, "amd_dft.linear3_stats: residual must have the output's shape");
  at::Tensor xs = xs_.contiguous(), ws = ws_.contiguous(), r = residual.to(at::kFloat).contiguous();
  // the kernel always reads pre (zeros when absent): an optional load behind a branch made the compiler
  // wait for it -- and for every store before it -- right where it was issued
  at::Tensor pre;
  if (pre_.has_value() && pre_->defined()) {
    pre = pre_->to(at::kFloat).contiguous();
    TORCH_CHECK(pre.numel() == N, "amd_dft.linear3_stats: pre must have N entries");
  } else {
    pre = at::zeros({N}, xs.options().dtype(at::kFloat));
  }
  std::vector<int64_t> os(xs.sizes().begin(), xs.sizes().end());
  os.back() = N;
  at::Tensor y = at::empty(os, xs.options().dtype(at::kFloat));
  at::Tensor part = at::empty({M, N / 64, 2}, xs.options().dtype(at::kFloat));
  GemmLaunch p;
  p.x = reinterpret_cast<const uint16_t*>(xs.data_ptr());
  p.w = reinterpret_cast<const uint16_t*>(ws.data_ptr());
  p.residual = r.data_ptr();
  p.y = y.data_ptr();
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.split = 1;
  p.out = 1;
  p.stats_part = part.data_ptr<float>();
  p.stats_pre = pre.data_ptr<float>();
  if (M > 0) launch_gemm(p, c10::hip::getCurrentHIPStream(xs.device().index()).stream());
  return {y, part};
}

// fc2 of the fp32 block with the residual stream carried as c2r_ln_add_split's split pairs (no fp32 copy of it):
// residual = m + (hi + lo), rpairs [M, 2N] bf16 k32-interleaved pairs of x - m, rstats [M, 2] with m = rstats[:, 0]
// (the block's LN1 statistics, which centred those pairs).  2^-18 of |x - m| off the fp32 residual.
// rlo2 (optional): the split's third term bf16(x - m - (hi + lo)) [M, N] (c2r_ln_add_split out_mode 2): the
// residual then matches the fp32 stream to ~2^-27 of |x - m| (fp32 rounding: 2^-24 of |x|)
at::Tensor pairs_residual_cpu(const at::Tensor& rpairs, const at::Tensor& rstats, int64_t N,
                              const c10::optional<at::Tensor>& rlo2) {
  at::Tensor pr = rpairs.to(at::kFloat).reshape({-1, N / 32, 2, 32});
  at::Tensor z = (pr.select(2, 0) + pr.select(2, 1)).reshape({-1, N});
  if (rlo2.has_value() && rlo2->defined()) z = z + rlo2->to(at::kFloat).reshape({-1, N});
  return z + rstats.to(at::kFloat).reshape({-1, 2}).select(1, 0).unsqueeze(1);
}

void check_pairs_residual(const at::Tensor& rpairs, const at::Tensor& rstats, int64_t M, int64_t N) {
  TORCH_CHECK(rpairs.scalar_type() == at::kBFloat16 && rpairs.numel() == M * 2 * N,
              "amd_dft.linear3_stats_pr: rpairs must be [M, 2N] bf16 split pairs");
  TORCH_CHECK(rstats.numel() == M * 2, "amd_dft.linear3_stats_pr: rstats must be [M, 2] (shift, rstd)");
  TORCH_CHECK(N % 32 == 0, "amd_dft.linear3_stats_pr: N must be a multiple of 32");
}

std::tuple<at::Tensor, at::Tensor> linear3_stats_pr_cpu(const at::Tensor& xs, const at::Tensor& ws, const at::Tensor& rpairs,
                                                        const at::Tensor& rstats, const c10::optional<at::Tensor>& pre,
                                                        const c10::optional<at::Tensor>& rlo2) {
  const int64_t N = ws.size(0), M = xs.numel() / std::max<int64_t>(xs.size(-1), 1);
  check_pairs_residual(rpairs, rstats, M, N);
  return linear3_stats_cpu(xs, ws, pairs_residual_cpu(rpairs, rstats, N, rlo2), pre);
}

std::tuple<at::Tensor, at::Tensor> linear3_stats_pr_cuda(const at::Tensor& xs_, const at::Tensor& ws_, const at::Tensor& rpairs_,
                                                         const at::Tensor& rstats_, const c10::optional<at::Tensor>& pre_,
                                                         const c10::optional<at::Tensor>& rlo2_) {
  const c10::DeviceGuard guard(xs_.device());
  check_split_linear(xs_, ws_, c10::nullopt, "linear3_stats_pr");
  TORCH_CHECK(xs_.size(-1) == ws_.size(1), "amd_dft.linear3_stats_pr: xs [..., 2K], ws [N, 2K]");
  const int64_t K = ws_.size(1) / 2, N = ws_.size(0), M = xs_.numel() / std::max<int64_t>(2 * K, 1);
  TORCH_CHECK(gemm_supported(M, N, K), "amd_dft.linear3_stats_pr: the bf16x3 GEMM needs N % 64 == 0 and K % 64 == 0");
  check_pairs_residual(rpairs_, rstats_, M, N);
  at::Tensor xs = xs_.contiguous(), ws = ws_.contiguous(), rp = rpairs_.contiguous(), rs = rstats_.to(at::kFloat).contiguous();
  at::Tensor pre;
  if (pre_.has_value() && pre_->defined()) {
    pre = pre_->to(at::kFloat).contiguous();
    TORCH_CHECK(pre.numel() == N, "amd_dft.linear3_stats_pr: pre must have N entries");
  } else {
    pre = at::zeros({N}, xs.options().dtype(at::kFloat));
  }
  std::vector<int64_t> os(xs.sizes().begin(), xs.sizes().end());
  os.back() = N;
  at::Tensor y = at::empty(os, xs.options().dtype(at::kFloat));
  at::Tensor part = at::empty({M, N / 64, 2}, xs.options().dtype(at::kFloat));
  GemmLaunch p;
  p.x = reinterpret_cast<const uint16_t*>(xs.data_ptr());
  p.w = reinterpret_cast<const uint16_t*>(ws.data_ptr());
  at::Tensor rl;
  if (rlo2_.has_value() && rlo2_->defined()) {
    TORCH_CHECK(rlo2_->scalar_type() == at::kBFloat16 && rlo2_->numel() == M * N,
                "amd_dft.linear3_stats_pr: rlo2 must be [M, N] bf16");
    rl = rlo2_->contiguous();
  }
  p.residual = rp.data_ptr();
  p.res_mean = rs.data_ptr<float>();
  p.res_lo2 = rl.defined() ? reinterpret_cast<const uint16_t*>(rl.data_ptr()) : nullptr;
  p.y = y.data_ptr();
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.split = 1;
  p.out = 1;
  p.stats_part = part.data_ptr<float>();
  p.stats_pre = pre.data_ptr<float>();
  if (M > 0) launch_gemm(p, c10::hip::getCurrentHIPStream(xs.device().index()).stream());
  return {y, part};
}

std::tuple<at::Tensor, at::Tensor> linear3_stats_pr_meta(const at::Tensor& xs, const at::Tensor& ws, const at::Tensor&,
                                                         const at::Tensor&, const c10::optional<at::Tensor>&,
                                                         const c10::optional<at::Tensor>&) {
  std::vector<int64_t> os(xs.sizes().begin(), xs.sizes().end());
  os.back() = ws.size(0);
  const int64_t M = xs.numel() / std::max<int64_t>(xs.size(-1), 1);
  return {at::empty(os, xs.options().dtype(at::kFloat)), at::empty({M, ws.size(0) / 64, 2}, xs.options().dtype(at::kFloat))};
}

std::tuple<at::Tensor, at::Tensor> linear3_stats_meta(const at::Tensor& xs, const at::Tensor& ws, const at::Tensor&,
                                                      const c10::optional<at::Tensor>&) {
  std::vector<int64_t> os(xs.sizes().begin(), xs.sizes().end());
  os.back() = ws.size(0);
  const int64_t M = xs.numel() / std::max<int64_t>(xs.size(-1), 1);
  return {at::empty(os, xs.options().dtype(at::kFloat)), at::empty({M, ws.size(0) / 64, 2}, xs.options().dtype(at::kFloat))};
}

// fc2 of the bf16 FourCastNet block: y = x w^T + residual (bf16) and, from the same epilogue, the
// next LayerNorm's partial statistics of y + pre -- taken on the stored (bf16-rounded) y, so they
// describe exactly the tensor that LayerNorm reads: part [M, N/64, 2] = per 64-feature chunk
// (mean, M2), merged by ln_stats_merge (replaces an ln_stats pass over y)
std::tuple<at::Tensor, at::Tensor> chunk_partials(const at::Tensor& y, const c10::optional<at::Tensor>& pre, int64_t N) {
  at::Tensor w = y.to(at::kFloat).reshape({-1, N});
  if (pre.has_value() && pre->defined()) w = w + pre->to(at::kFloat).reshape({1, N});
  w = w.reshape({w.size(0), N / 64, 64});
  at::Tensor mean = w.mean(2);
  at::Tensor m2 = (w - mean.unsqueeze(2)).pow(2).sum(2);
  return {y, at::stack({mean, m2}, 2).contiguous()};
}

std::tuple<at::Tensor, at::Tensor> linear_stats_cpu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& residual,
                                                    const c10::optional<at::Tensor>& pre) {
  TORCH_CHECK(w.dim() == 2 && x.size(-1) == w.size(1), "amd_dft.linear_stats: x [..., K], w [N, K]");
  const int64_t N = w.size(0);
  TORCH_CHECK(N % 64 == 0, "amd_dft.linear_stats: N must be a multiple of 64");
  TORCH_CHECK(!pre.has_value() || !pre->defined() || pre->numel() == N, "amd_dft.linear_stats: pre must have N entries");
  return chunk_partials(linear_ref(x, w, c10::nullopt, 0, residual), pre, N);
}

std::tuple<at::Tensor, at::Tensor> linear_stats_cuda(const at::Tensor& x_, const at::Tensor& w_, const at::Tensor& residual,
                                                     const c10::optional<at::Tensor>& pre_) {
  const c10::DeviceGuard guard(x_.device());
  TORCH_CHECK(w_.dim() == 2 && x_.size(-1) == w_.size(1), "amd_dft.linear_stats: x [..., K], w [N, K]");
  const int64_t K = w_.size(1), N = w_.size(0), M = x_.numel() / std::max<int64_t>(K, 1);
  TORCH_CHECK(N % 64 == 0, "amd_dft.linear_stats: N must be a multiple of 64");
  TORCH_CHECK(residual.numel() == M * N, "amd_dft.linear_stats: residual must have the output's shape");
  TORCH_CHECK(!pre_.has_value() || !pre_->defined() || pre_->numel() == N, "amd_dft.linear_stats: pre must have N entries");
  if (x_.scalar_type() != at::kBFloat16 || w_.scalar_type() != at::kBFloat16 || !gemm_supported(M, N, K)) {
    fallback_note("linear_stats", "needs bf16 operands, N % 64 == 0, K % 64 == 0");
    return chunk_partials(linear_ref(x_, w_, c10::nullopt, 0, residual), pre_, N);
  }
  at::Tensor x = x_.contiguous(), w = w_.contiguous(), r = residual.to(at::kBFloat16).contiguous();
  // the kernel always reads pre (zeros when absent): see linear3_stats
  at::Tensor pre = pre_.has_value() && pre_->defined() ? pre_->to(at::kFloat).contiguous()
                                                       : at::zeros({N}, x.options().dtype(at::kFloat));
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = N;
  at::Tensor y = at::empty(os, x.options());
  at::Tensor part = at::empty({M, N / 64, 2}, x.options().dtype(at::kFloat));
  GemmLaunch p;
  p.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  p.w = reinterpret_cast<const uint16_t*>(w.data_ptr());
  p.residual = r.data_ptr();
  p.y = y.data_ptr();
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.stats_part = part.data_ptr<float>();
  p.stats_pre = pre.data_ptr<float>();
  if (M > 0) launch_gemm(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return {y, part};
}

std::tuple<at::Tensor, at::Tensor> linear_stats_meta(const at::Tensor& x, const at::Tensor& w, const at::Tensor&,
                                                     const c10::optional<at::Tensor>&) {
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = w.size(0);
  const int64_t M = x.numel() / std::max<int64_t>(x.size(-1), 1);
  return {at::empty(os, x.options()), at::empty({M, w.size(0) / 64, 2}, x.options().dtype(at::kFloat))};
}

// fc1 of the fp32 FourCastNet block: y = split(act(LN(x) W^T + b)) from the split pairs of the RAW
// residual stream x (the AFNO C2R epilogue writes them, c2r_ln_add_split), the LayerNorm folded into
// the bf16x3 GEMM's epilogue exactly as linear_ln does for bf16: ws = split(W * gamma),
// c1[n] = sum_k (hi + lo)(ws)[n, k] (from the split pairs the GEMM reads), bias = W beta + b,
// stats [M, 2] = (mean, rstd) of x.  Output: split-pair rows (the next GEMM's operand).
void check_linear3_ln(const at::Tensor& xs, const at::Tensor& ws, const at::Tensor& c1, const c10::optional<at::Tensor>& bias,
                      const at::Tensor& stats, int64_t act) {
  check_split_linear(xs, ws, bias, "linear3_ln");
  TORCH_CHECK(act == 0 || act == 1, "amd_dft.linear3_ln: act must be 0 (none) or 1 (gelu)");
  TORCH_CHECK(xs.size(-1) == ws.size(1), "amd_dft.linear3_ln: xs [..., 2K], ws [N, 2K]");
  const int64_t N = ws.size(0), M = xs.numel() / std::max<int64_t>(ws.size(1), 1);
  TORCH_CHECK(c1.numel() == N, "amd_dft.linear3_ln: c1 must have N entries");
  TORCH_CHECK(stats.numel() == 2 * M && stats.size(-1) == 2, "amd_dft.linear3_ln: stats must be [M, 2] (mean, rstd)");
}

at::Tensor linear3_ln_cpu(const at::Tensor& xs, const at::Tensor& ws, const at::Tensor& c1, const c10::optional<at::Tensor>& bias,
                          const at::Tensor& stats, int64_t act) {
  check_linear3_ln(xs, ws, c1, bias, stats, act);
  at::Tensor y = linear_ln_ref(unsplit_rows(xs), unsplit_rows(ws), c1, bias, stats, act);
  return split_ref(y, true);
}

at::Tensor linear3_ln_cuda(const at::Tensor& xs_, const at::Tensor& ws_, const at::Tensor& c1_,
                           const c10::optional<at::Tensor>& bias, const at::Tensor& stats_, int64_t act) {
  const c10::DeviceGuard guard(xs_.device());
  check_linear3_ln(xs_, ws_, c1_, bias, stats_, act);
  const int64_t K = ws_.size(1) / 2, N = ws_.size(0), M = xs_.numel() / std::max<int64_t>(2 * K, 1);
  TORCH_CHECK(gemm_supported(M, N, K), "amd_dft.linear3_ln: the bf16x3 GEMM needs N % 64 == 0 and K % 64 == 0 (got N=",
              N, ", K=", K, ")");
  at::Tensor xs = xs_.contiguous(), ws = ws_.contiguous();
  at::Tensor c1 = c1_.to(at::kFloat).contiguous(), stats = stats_.to(at::kFloat).contiguous();
  std::vector<int64_t> os(xs.sizes().begin(), xs.sizes().end());
  os.back() = 2 * N;
  at::Tensor y = at::empty(os, xs.options());
  at::Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  GemmLaunch p;
  p.x = reinterpret_cast<const uint16_t*>(xs.data_ptr());
  p.w = reinterpret_cast<const uint16_t*>(ws.data_ptr());
  p.bias = b.defined() ? b.data_ptr<float>() : nullptr;
  p.y = y.data_ptr();
  p.ln_stats = stats.data_ptr<float>();
  p.ln_c1 = c1.data_ptr<float>();
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.act = static_cast<int>(act);
  p.split = 1;
  p.out = 2;
  if (M > 0) launch_gemm(p, c10::hip::getCurrentHIPStream(xs.device().index()).stream());
  return y;
}

at::Tensor linear3_ln_meta(const at::Tensor& xs, const at::Tensor& ws, const at::Tensor&, const c10::optional<at::Tensor>&,
                           const at::Tensor&, int64_t) {
  std::vector<int64_t> os(xs.sizes().begin(), xs.sizes().end());
  os.back() = 2 * ws.size(0);
  return at::empty(os, xs.options());
}

at::Tensor linear3_meta(const at::Tensor& xs, const at::Tensor& ws, const c10::optional<at::Tensor>&, int64_t,
                        const c10::optional<at::Tensor>&, bool split_out) {
  std::vector<int64_t> os(xs.sizes().begin(), xs.sizes().end());
  os.back() = split_out ? 2 * ws.size(0) : ws.size(0);
  return at::empty(os, xs.options().dtype(split_out ? at::kBFloat16 : at::kFloat));
}

// xs = split planes [2, B, C, h*p, w*p] of the fp32 image; ws [N, 2*C*p*p]; fp32 tokens [B*h*w, N]
// patch_linear3 takes the image either as bf16 split planes [2, B, C, H, W] or as the raw fp32 image
// [B, C, H, W] (split here first).  Round 5 measured folding that split into the GEMM's fragment reads
// (the raw fp32 gathered into LDS, split per read): the embed GEMM went from 2.32 to 4.69 ms, more
// than the 0.90 ms split pass it removed (profiles/patch_embed_raw_f32_r5.txt), so the pass stays.
bool raw_f32_image(const at::Tensor& xs) { return xs.dim() == 4 && xs.scalar_type() == at::kFloat; }

at::Tensor patch_linear3_cpu(const at::Tensor& xs, const at::Tensor& ws, const c10::optional<at::Tensor>& bias,
                             const c10::optional<at::Tensor>& pos, int64_t p) {
  const bool raw = raw_f32_image(xs);
  check_split_linear(raw ? ws : xs, ws, bias, "patch_linear3");
  TORCH_CHECK(raw || (xs.dim() == 5 && xs.size(0) == 2),
              "amd_dft.patch_linear3: xs must be split planes [2, B, C, H, W] or the fp32 image [B, C, H, W]");
  // the split pair of the raw image is exactly what the GEMM multiplies (hi + lo of each value)
  at::Tensor planes = raw ? split_ref(xs, false) : xs;
  at::Tensor x = planes.select(0, 0).to(at::kFloat) + planes.select(0, 1).to(at::kFloat);
  at::Tensor t = patchify_cpu(x, p);
  at::Tensor y = at::linear(t, unsplit_rows(ws),
                            bias.has_value() && bias->defined() ? c10::optional<at::Tensor>(bias->to(at::kFloat))
                                                                : c10::nullopt);
  if (pos.has_value() && pos->defined()) {
    const int64_t hw = (x.size(2) / p) * (x.size(3) / p);
    y = (y.reshape({-1, hw, ws.size(0)}) + pos->to(at::kFloat).reshape({1, hw, ws.size(0)})).reshape({-1, ws.size(0)});
  }
  return y.contiguous();
}

at::Tensor patch_linear3_cuda(const at::Tensor& xs_, const at::Tensor& ws_, const c10::optional<at::Tensor>& bias,
                              const c10::optional<at::Tensor>& pos, int64_t p) {
  const c10::DeviceGuard guard(xs_.device());
  const bool raw = raw_f32_image(xs_);
  check_split_linear(raw ? ws_ : xs_, ws_, bias, "patch_linear3");
  const int o = raw ? 0 : 1;  // leading plane dim of the split form
  TORCH_CHECK((raw || (xs_.dim() == 5 && xs_.size(0) == 2)) && xs_.size(2 + o) % p == 0 && xs_.size(3 + o) % p == 0,
              "amd_dft.patch_linear3: xs must be split planes [2, B, C, h*p, w*p] or the fp32 image [B, C, h*p, w*p]");
  const int64_t B = xs_.size(o), C = xs_.size(1 + o), h = xs_.size(2 + o) / p, w = xs_.size(3 + o) / p, N = ws_.size(0);
  const int64_t M = B * h * w, K = C * p * p;
  TORCH_CHECK(p == 8 && ws_.size(1) == 2 * K && gemm_supported(M, N, K) && xs_.numel() < (int64_t(1) << 31),
              "amd_dft.patch_linear3: needs p == 8, ws [N, 2*C*64], N % 64 == 0 and < 2^31 image elements");
  at::Tensor xs = raw ? split_bf16_cuda(xs_, false) : xs_.contiguous(), ws = ws_.contiguous();
  at::Tensor y = at::empty({M, N}, xs.options().dtype(at::kFloat));
  at::Tensor b, r;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->numel() == h * w * N, "amd_dft.patch_linear3: pos must be [h*w, N]");
    r = pos->to(at::kFloat).contiguous();
  }
  GemmLaunch g;
  g.x = reinterpret_cast<const uint16_t*>(xs.data_ptr());
  g.w = reinterpret_cast<const uint16_t*>(ws.data_ptr());
  g.bias = b.defined() ? b.data_ptr<float>() : nullptr;
  g.residual = r.defined() ? r.data_ptr() : nullptr;
  g.res_rows = static_cast<int>(h * w);
  g.y = y.data_ptr();
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.K = static_cast<int>(K);
  g.gC = static_cast<int>(C);
  g.gh = static_cast<int>(h);
  g.gw = static_cast<int>(w);
  g.split = 1;
  g.out = 1;
  g.x_lo = xs.numel() / 2;
  launch_gemm(g, c10::hip::getCurrentHIPStream(xs.device().index()).stream());
  return y;
}

at::Tensor patch_linear3_meta(const at::Tensor& xs, const at::Tensor& ws, const c10::optional<at::Tensor>&,
                              const c10::optional<at::Tensor>&, int64_t p) {
  const int o = raw_f32_image(xs) ? 0 : 1;
  return at::empty({xs.size(o) * (xs.size(2 + o) / p) * (xs.size(3 + o) / p), ws.size(0)}, xs.options().dtype(at::kFloat));
}

at::Tensor linear_unpatch3_cpu(const at::Tensor& ts, const at::Tensor& ws, const c10::optional<at::Tensor>& bias,
                               int64_t C, int64_t h, int64_t wd, int64_t p) {
  check_split_linear(ts, ws, bias, "linear_unpatch3");
  at::Tensor y = at::linear(unsplit_rows(ts), unsplit_rows(ws),
                            bias.has_value() && bias->defined() ? c10::optional<at::Tensor>(bias->to(at::kFloat))
                                                                : c10::nullopt);
  return unpatchify_cpu(y, C, h, wd, p);
}

at::Tensor linear_unpatch3_cuda(const at::Tensor& ts_, const at::Tensor& ws_, const c10::optional<at::Tensor>& bias,
                                int64_t C, int64_t h, int64_t wd, int64_t p) {
  const c10::DeviceGuard guard(ts_.device());
  check_split_linear(ts_, ws_, bias, "linear_unpatch3");
  const int64_t K = ws_.size(1) / 2, N = ws_.size(0), M = ts_.numel() / std::max<int64_t>(2 * K, 1);
  TORCH_CHECK(ts_.size(-1) == 2 * K && N == C * p * p && p == 8 && M % (h * wd) == 0 && gemm_supported(M, N, K),
              "amd_dft.linear_unpatch3: ts [..., 2K], ws [C*64, 2K] in (c, py, px) order, p == 8");
  at::Tensor ts = ts_.contiguous(), ws = ws_.contiguous();
  const int64_t B = M / (h * wd);
  at::Tensor y = at::empty({B, C, h * p, wd * p}, ts.options().dtype(at::kFloat));
  at::Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(at::kFloat).contiguous();
  const bool ragged = N % 256 != 0;  // see linear_unpatch_cuda
  at::Tensor yt = ragged ? at::empty({M, N}, ts.options().dtype(at::kFloat)) : at::Tensor();
  GemmLaunch g;
  g.x = reinterpret_cast<const uint16_t*>(ts.data_ptr());
  g.w = reinterpret_cast<const uint16_t*>(ws.data_ptr());
  g.bias = b.defined() ? b.data_ptr<float>() : nullptr;
  g.y = ragged ? yt.data_ptr() : y.data_ptr();
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.K = static_cast<int>(K);
  if (!ragged) {
    g.sC = static_cast<int>(C);
    g.sh = static_cast<int>(h);
    g.sw = static_cast<int>(wd);
  }
  g.split = 1;
  g.out = 1;
  auto stream = c10::hip::getCurrentHIPStream(ts.device().index()).stream();
  launch_gemm(g, stream);
  if (ragged)
    launch_patch_remap(yt.data_ptr(), y.data_ptr(), B, static_cast<int>(C), static_cast<int>(h), static_cast<int>(wd),
                       false, stream, 4);
  return y;
}

at::Tensor linear_unpatch3_meta(const at::Tensor& ts, const at::Tensor& ws, const c10::optional<at::Tensor>&, int64_t C,
                                int64_t h, int64_t wd, int64_t p) {
  return at::empty({ts.numel() / ws.size(1) / (h * wd), C, h * p, wd * p}, ts.options().dtype(at::kFloat));
}

}  // namespace
}  // namespace amd_dft

TORCH_LIBRARY_FRAGMENT(amd_dft, m) {
  m.def("patchify(Tensor x, int p) -> Tensor");
  m.def("unpatchify(Tensor t, int C, int h, int w, int p) -> Tensor");
  m.def("linear(Tensor x, Tensor w, Tensor? bias=None, int act=0, Tensor? residual=None) -> Tensor");
  m.def("linear_ln(Tensor x, Tensor w, Tensor c1, Tensor? bias, Tensor stats, int act=0) -> Tensor");
  m.def("patch_linear(Tensor x, Tensor w, Tensor? bias=None, Tensor? pos=None, int p=8) -> Tensor");
  m.def("linear_unpatch(Tensor t, Tensor w, Tensor? bias, int C, int h, int w, int p=8) -> Tensor");
  m.def("split_bf16(Tensor x, bool rows=True) -> Tensor");
  m.def("linear3(Tensor xs, Tensor ws, Tensor? bias=None, int act=0, Tensor? residual=None, bool split_out=False) -> Tensor");
  m.def("linear3_stats(Tensor xs, Tensor ws, Tensor residual, Tensor? pre=None) -> (Tensor, Tensor)");
  m.def("linear3_stats_pr(Tensor xs, Tensor ws, Tensor rpairs, Tensor rstats, Tensor? pre=None, Tensor? rlo2=None) -> "
        "(Tensor, Tensor)");
  m.def("linear_stats(Tensor x, Tensor w, Tensor residual, Tensor? pre=None) -> (Tensor, Tensor)");
  m.def("linear3_ln(Tensor xs, Tensor ws, Tensor c1, Tensor? bias, Tensor stats, int act=0) -> Tensor");
  m.def("patch_linear3(Tensor xs, Tensor ws, Tensor? bias=None, Tensor? pos=None, int p=8) -> Tensor");
  m.def("linear_unpatch3(Tensor ts, Tensor ws, Tensor? bias, int C, int h, int w, int p=8) -> Tensor");
}
TORCH_LIBRARY_IMPL(amd_dft, CUDA, m) {
  m.impl("patchify", AMD_DFT_TRACED("amd_dft::patchify", amd_dft::patchify_cuda));
  m.impl("unpatchify", AMD_DFT_TRACED("amd_dft::unpatchify", amd_dft::unpatchify_cuda));
  m.impl("linear", AMD_DFT_TRACED("amd_dft::linear", amd_dft::linear_cuda));
  m.impl("linear_ln", AMD_DFT_TRACED("amd_dft::linear_ln", amd_dft::linear_ln_cuda));
  m.impl("patch_linear", AMD_DFT_TRACED("amd_dft::patch_linear", amd_dft::patch_linear_cuda));
  m.impl("linear_unpatch", AMD_DFT_TRACED("amd_dft::linear_unpatch", amd_dft::linear_unpatch_cuda));
  m.impl("split_bf16", AMD_DFT_TRACED("amd_dft::split_bf16", amd_dft::split_bf16_cuda));
  m.impl("linear3", AMD_DFT_TRACED("amd_dft::linear3", amd_dft::linear3_cuda));
  m.impl("linear3_stats", AMD_DFT_TRACED("amd_dft::linear3_stats", amd_dft::linear3_stats_cuda));
  m.impl("linear3_stats_pr", AMD_DFT_TRACED("amd_dft::linear3_stats_pr", amd_dft::linear3_stats_pr_cuda));
  m.impl("linear_stats", AMD_DFT_TRACED("amd_dft::linear_stats", amd_dft::linear_stats_cuda));
  m.impl("linear3_ln", AMD_DFT_TRACED("amd_dft::linear3_ln", amd_dft::linear3_ln_cuda));
  m.impl("patch_linear3", AMD_DFT_TRACED("amd_dft::patch_linear3", amd_dft::patch_linear3_cuda));
  m.impl("linear_unpatch3", AMD_DFT_TRACED("amd_dft::linear_unpatch3", amd_dft::linear_unpatch3_cuda));
}
TORCH_LIBRARY_IMPL(amd_dft, CPU, m) {
  m.impl("patchify", AMD_DFT_TRACED("amd_dft::patchify", amd_dft::patchify_cpu));
  m.impl("unpatchify", AMD_DFT_TRACED("amd_dft::unpatchify", amd_dft::unpatchify_cpu));
  m.impl("linear", AMD_DFT_TRACED("amd_dft::linear", amd_dft::linear_cpu));
  m.impl("linear_ln", AMD_DFT_TRACED("amd_dft::linear_ln", amd_dft::linear_ln_cpu));
  m.impl("patch_linear", AMD_DFT_TRACED("amd_dft::patch_linear", amd_dft::patch_linear_cpu));
  m.impl("linear_unpatch", AMD_DFT_TRACED("amd_dft::linear_unpatch", amd_dft::linear_unpatch_cpu));
  m.impl("split_bf16", AMD_DFT_TRACED("amd_dft::split_bf16", amd_dft::split_bf16_cpu));
  m.impl("linear3", AMD_DFT_TRACED("amd_dft::linear3", amd_dft::linear3_cpu));
  m.impl("linear3_stats", AMD_DFT_TRACED("amd_dft::linear3_stats", amd_dft::linear3_stats_cpu));
  m.impl("linear3_stats_pr", AMD_DFT_TRACED("amd_dft::linear3_stats_pr", amd_dft::linear3_stats_pr_cpu));
  m.impl("linear_stats", AMD_DFT_TRACED("amd_dft::linear_stats", amd_dft::linear_stats_cpu));
  m.impl("linear3_ln", AMD_DFT_TRACED("amd_dft::linear3_ln", amd_dft::linear3_ln_cpu));
  m.impl("patch_linear3", AMD_DFT_TRACED("amd_dft::patch_linear3", amd_dft::patch_linear3_cpu));
  m.impl("linear_unpatch3", AMD_DFT_TRACED("amd_dft::linear_unpatch3", amd_dft::linear_unpatch3_cpu));
}
TORCH_LIBRARY_IMPL(amd_dft, Meta, m) {
  m.impl("patchify", &amd_dft::patchify_meta);
  m.impl("unpatchify", &amd_dft::unpatchify_meta);
  m.impl("linear", &amd_dft::linear_meta);
  m.impl("linear_ln", &amd_dft::linear_ln_meta);
  m.impl("patch_linear", &amd_dft::patch_linear_meta);
  m.impl("linear_unpatch", &amd_dft::linear_unpatch_meta);
  m.impl("split_bf16", &amd_dft::split_bf16_meta);
  m.impl("linear3", &amd_dft::linear3_meta);
  m.impl("linear3_stats", &amd_dft::linear3_stats_meta);
  m.impl("linear3_stats_pr", &amd_dft::linear3_stats_pr_meta);
  m.impl("linear_stats", &amd_dft::linear_stats_meta);
  m.impl("linear3_ln", &amd_dft::linear3_ln_meta);
  m.impl("patch_linear3", &amd_dft::patch_linear3_meta);
  m.impl("linear_unpatch3", &amd_dft::linear_unpatch3_meta);
}
