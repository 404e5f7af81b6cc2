// Torch op layer for the fused spectral-layer kernels (FourCastNet AFNO, FNO) and the
// fused LayerNorm.  CPU implementations are plain ATen math (reference semantics); the
// CUDA (HIP) implementations launch the hand-written gfx950 kernels.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <ATen/core/dispatch/Dispatcher.h>
#include <torch/library.h>

#include "trace.h"
#include "../spectral/dft_gemm.h"
#include "../spectral/spectral.h"
#include "checks.h"
#include "plan_cache.h"

namespace amd_dft {
namespace {

// ------------------------------------------------------------------ AFNO spectral filter
// xw [B, H, KM, C, 2] fp32 (W-direction half spectrum), w1t/w2t [NB, 2BS, 2BS] bf16 ([n][k]),
// b1/b2 [NB, 2BS] fp32.  Returns [B, H, KM, C, 2] fp32:
//   IFFT_H( softshrink( ReLU(FFT_H(x) W1' + b1') W2' + b2' ) )   (FFTs unnormalised)
void check_afno(const at::Tensor& xw, const at::Tensor& w1t, const at::Tensor& w2t, const at::Tensor& b1,
                const at::Tensor& b2) {
  TORCH_CHECK(xw.dim() == 5 && xw.size(4) == 2 &&
                  (xw.scalar_type() == at::kFloat || xw.scalar_type() == at::kBFloat16),
              "afno_spectral: x must be [B, H, KM, C, 2] float32 or bfloat16");
  TORCH_CHECK(w1t.dim() == 3, "afno_spectral: bad weight shapes");
  const int64_t NB = w1t.size(0), K = w1t.size(1);
  TORCH_CHECK((w1t.size(2) == K || w1t.size(2) == 2 * K) && w2t.sizes() == w1t.sizes(),
              "afno_spectral: weights must be [NB, 2BS, 2BS] (bf16) or split [NB, 2BS, 2*2BS] (bf16x3, fp32 path)");
  TORCH_CHECK(NB * K == 2 * xw.size(3), "afno_spectral: NB * 2 * block_size must equal 2 * C");
  TORCH_CHECK(b1.sizes() == at::IntArrayRef({NB, K}) && b2.sizes() == b1.sizes(), "afno_spectral: bad bias shapes");
}

at::Tensor afno_spectral_cpu(const at::Tensor& xw, const at::Tensor& w1t, const at::Tensor& w2t, const at::Tensor& b1,
                             const at::Tensor& b2, double lam) {
  check_afno(xw, w1t, w2t, b1, b2);
  const int64_t B = xw.size(0), H = xw.size(1), KM = xw.size(2), C = xw.size(3);
  const int64_t NB = w1t.size(0), BS = C / NB;
  at::Tensor X = at::fft_fft(at::view_as_complex(xw.to(at::kFloat).contiguous()), std::nullopt, 1, "backward");
  at::Tensor Xr = at::view_as_real(X).reshape({B, H, KM, NB, BS, 2});
  at::Tensor A = at::cat({Xr.select(-1, 0), Xr.select(-1, 1)}, -1);  // [..., NB, 2BS]
  auto unsplit = [&](const at::Tensor& w) {  // k32-interleaved split rows -> fp32
    if (w.size(2) == w.size(1)) return w.to(at::kFloat);
    const int64_t k = w.size(1);
    return w.to(at::kFloat).reshape({w.size(0), w.size(1), k / 32, 2, 32}).sum(3).reshape({w.size(0), w.size(1), k});
  };
  at::Tensor W1 = unsplit(w1t).transpose(1, 2);                      // [NB, k, n]
  at::Tensor W2 = unsplit(w2t).transpose(1, 2);
  at::Tensor H1 = at::relu(at::einsum("...bk,bkn->...bn", {A, W1}) + b1);
  at::Tensor O = at::einsum("...bk,bkn->...bn", {H1, W2}) + b2;
  O = at::softshrink(O, lam);
  at::Tensor Oc = at::complex(O.narrow(-1, 0, BS), O.narrow(-1, BS, BS)).reshape({B, H, KM, C});
  at::Tensor Y = at::fft_ifft(Oc, std::nullopt, 1, "forward");
  return at::view_as_real(Y).to(xw.scalar_type()).contiguous();
}

at::Tensor afno_spectral_cuda(const at::Tensor& xw_, const at::Tensor& w1t_, const at::Tensor& w2t_, const at::Tensor& b1_,
                              const at::Tensor& b2_, double lam) {
  check_afno(xw_, w1t_, w2t_, b1_, b2_);
  const c10::DeviceGuard guard(xw_.device());
  at::Tensor xw = xw_.contiguous();
  at::Tensor w1t = w1t_.to(at::kBFloat16).contiguous(), w2t = w2t_.to(at::kBFloat16).contiguous();
  at::Tensor b1 = b1_.to(at::kFloat).contiguous(), b2 = b2_.to(at::kFloat).contiguous();
  const int64_t B = xw.size(0), H = xw.size(1), KM = xw.size(2), C = xw.size(3), NB = w1t.size(0);
  TORCH_CHECK(afno_spectral_supported(static_cast<int>(H), static_cast<int>(C / NB)),
              "afno_spectral: no fused instance for H = ", H, ", block size ", C / NB,
              " (afno_spectral_shapes() lists them; use the generic path)");
  const bool x3 = w1t.size(2) == 2 * w1t.size(1);
  TORCH_CHECK(!x3 || xw.scalar_type() == at::kFloat, "afno_spectral: split (bf16x3) weights go with a float32 spectrum");
  at::Tensor y = at::empty_like(xw);
  if (xw.numel() == 0) return y;
  auto dp = get_plan(H, xw.device());
  AfnoLaunch p;
  p.x3 = x3 ? 1 : 0;
  p.x = xw.data_ptr();
  p.y = y.data_ptr();
  p.bf16_in = p.bf16_out = xw.scalar_type() == at::kBFloat16;
  p.w1t = reinterpret_cast<const uint16_t*>(w1t.data_ptr());
  p.w2t = reinterpret_cast<const uint16_t*>(w2t.data_ptr());
  p.b1 = b1.data_ptr<float>();
  p.b2 = b2.data_ptr<float>();
  p.tw = dp->tw.data_ptr();
  TORCH_CHECK(dp->plan.radices.size() == 2, "afno_spectral: H = ", H, " is not a two-pass plan");
  p.r0 = dp->plan.radices[0];
  p.r1 = dp->plan.radices[1];
  p.B = static_cast<int>(B);
  p.H = static_cast<int>(H);
  p.KM = static_cast<int>(KM);
  p.C = static_cast<int>(C);
  p.NB = static_cast<int>(NB);
  p.lambda = static_cast<float>(lam);
  launch_afno_spectral(p, c10::hip::getCurrentHIPStream(xw.device().index()).stream());
  return checked(y, "afno_spectral");
}

std::vector<int64_t> afno_spectral_shape_list() {  // flattened (H, block size) pairs
  std::vector<int64_t> v;
  for (const auto& hb : afno_spectral_shapes()) {
    v.push_back(hb.first);
    v.push_back(hb.second);
  }
  return v;
}

bool afno_spectral_ok(int64_t H, int64_t block_size) {
  return afno_spectral_supported(static_cast<int>(H), static_cast<int>(block_size));
}

// ------------------------------------------------------------------ FNO mode mixing
// x [B, Cin, M, 2] fp32, w [Cin, Cout, M, 2] fp32 -> y [B, Cout, M, 2] fp32
at::Tensor fno_mix_cpu(const at::Tensor& x, const at::Tensor& w, int64_t /*path*/) {
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 2 && w.dim() == 4 && w.size(3) == 2 && w.size(0) == x.size(1) &&
                  w.size(2) == x.size(2),
              "fno_mix: x [B, Cin, M, 2], w [Cin, Cout, M, 2]");
  at::Tensor xc = at::view_as_complex(x.to(at::kFloat).contiguous());
  at::Tensor wc = at::view_as_complex(w.to(at::kFloat).contiguous());
  return at::view_as_real(at::einsum("bim,iom->bom", {xc, wc})).contiguous();
}

bool fno_mix_fits(int64_t B, int64_t Cin, int64_t Cout) {
  const int64_t K = 2 * Cin, N = 2 * Cout, Kp = (K + 3) & ~3, Bp = (B + 15) & ~15, Np = (N + 15) & ~15;
  return 4 * 8 * (Bp * Kp + Kp * Np + Bp * Np) <= 160 * 1024;
}

// path: 0 = auto (scalar split-K stream for B <= 8, the MFMA kernel above), 2 = the MFMA kernel at any B
at::Tensor fno_mix_cuda(const at::Tensor& x_, const at::Tensor& w_, int64_t path) {
  const c10::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.dim() == 4 && x_.size(3) == 2 && w_.dim() == 4 && w_.size(3) == 2 && w_.size(0) == x_.size(1) &&
                  w_.size(2) == x_.size(2),
              "fno_mix: x [B, Cin, M, 2], w [Cin, Cout, M, 2]");
  const int64_t B = x_.size(0), Cin = x_.size(1), M = x_.size(2), Cout = w_.size(1);
  if (!fno_mix_fits(B, Cin, Cout)) {  // ATen on the device tensors
    fallback_note("fno_mix", "operand tiles exceed the 160 KB LDS");
    return fno_mix_cpu(x_, w_, path);
  }
  at::Tensor x = x_.to(at::kFloat).contiguous(), w = w_.to(at::kFloat).contiguous();
  at::Tensor y = at::empty({B, Cout, M, 2}, x.options());
  FnoMixLaunch p;
  p.x = x.data_ptr<float>();
  p.w = w.data_ptr<float>();
  p.y = y.data_ptr<float>();
  p.B = static_cast<int>(B);
  p.Cin = static_cast<int>(Cin);
  p.Cout = static_cast<int>(Cout);
  p.M = static_cast<int>(M);
  p.mfma = path == 2 ? 1 : 0;
  launch_fno_mix(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return checked(y, "fno_mix");
}

at::Tensor fno_mix_meta(const at::Tensor& x, const at::Tensor& w, int64_t) {
  return at::empty({x.size(0), w.size(1), x.size(2), 2}, x.options().dtype(at::kFloat));
}

// ------------------------------------------------------------------ FNO pointwise epilogue
// y = act(spec + conv1x1(x, w) + bias); x [B, Cin, *S], spec [B, Cout, *S] (or None), w [Cout, Cin(,1,1)]
at::Tensor fno_pointwise_cpu(const c10::optional<at::Tensor>& spec, const at::Tensor& x, const at::Tensor& w,
                             const c10::optional<at::Tensor>& bias, bool gelu) {
  TORCH_CHECK(x.dim() >= 2, "fno_pointwise: x [B, Cin, ...]");
  const int64_t B = x.size(0), Cin = x.size(1);
  at::Tensor w2 = w.reshape({w.size(0), -1}).to(at::kFloat);
  TORCH_CHECK(w2.size(1) == Cin, "fno_pointwise: weight must be [Cout, Cin]");
  at::Tensor xf = x.to(at::kFloat).reshape({B, Cin, -1});
  at::Tensor y = at::einsum("oi,bip->bop", {w2, xf});
  if (bias.has_value() && bias->defined()) y = y + bias->to(at::kFloat).reshape({1, -1, 1});
  if (spec.has_value() && spec->defined()) y = y + spec->to(at::kFloat).reshape({B, w2.size(0), -1});
  if (gelu) y = at::gelu(y);
  std::vector<int64_t> shape = x.sizes().vec();
  shape[1] = w2.size(0);
  return y.reshape(shape).to(x.scalar_type());
}

at::Tensor fno_pointwise_cuda(const c10::optional<at::Tensor>& spec_, const at::Tensor& x_, const at::Tensor& w,
                              const c10::optional<at::Tensor>& bias, bool gelu) {
  const c10::DeviceGuard guard(x_.device());
  TORCH_CHECK(x_.dim() >= 2, "fno_pointwise: x [B, Cin, ...]");
  TORCH_CHECK(x_.scalar_type() == at::kFloat || x_.scalar_type() == at::kBFloat16,
              "fno_pointwise: x must be float32 or bfloat16");
  const int64_t B = x_.size(0), Cin = x_.size(1);
  const int64_t P = x_.numel() / std::max<int64_t>(B * Cin, 1);
  at::Tensor w2 = w.reshape({w.size(0), -1}).to(at::kFloat).contiguous();
  TORCH_CHECK(w2.size(1) == Cin, "fno_pointwise: weight must be [Cout, Cin]");
  const int64_t Cout = w2.size(0);
  TORCH_CHECK(fno_pointwise_supported(static_cast<int>(Cin)), "fno_pointwise: unsupported channel count ", Cin,
              " (kernel instances: 4, 8, 16, 20, 32, 64, 128)");
  TORCH_CHECK(P < (int64_t(1) << 31) / 4 && B <= 65535, "fno_pointwise: tensor too large");
  at::Tensor x = x_.contiguous();
  at::Tensor spec;
  if (spec_.has_value() && spec_->defined()) {
    TORCH_CHECK(spec_->numel() == B * Cout * P, "fno_pointwise: spec must be [B, Cout, ...] like the output");
    spec = spec_->to(x.scalar_type()).contiguous();
  }
  at::Tensor bf;
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  std::vector<int64_t> shape = x.sizes().vec();
  shape[1] = Cout;
  at::Tensor y = at::empty(shape, x.options());
  FnoPointwiseLaunch p;
  p.spec = spec.defined() ? spec.data_ptr() : nullptr;
  p.x = x.data_ptr();
  p.w = w2.data_ptr<float>();
  p.bias = bf.defined() ? bf.data_ptr<float>() : nullptr;
  p.y = y.data_ptr();
  p.B = static_cast<int>(B);
  p.Cin = static_cast<int>(Cin);
  p.Cout = static_cast<int>(Cout);
  p.P = static_cast<int>(P);
  p.bf16 = x.scalar_type() == at::kBFloat16;
  p.gelu = gelu;
  launch_fno_pointwise(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return checked(y, "fno_pointwise");
}

at::Tensor fno_pointwise_meta(const c10::optional<at::Tensor>& spec, const at::Tensor& x, const at::Tensor& w,
                              const c10::optional<at::Tensor>& bias, bool gelu) {
  std::vector<int64_t> shape = x.sizes().vec();
  shape[1] = w.size(0);
  return at::empty(shape, x.options());
}

// ------------------------------------------------------------------ FNO layer tail (C2R-W + pointwise)
// yw [B, Cout, H, m, 2] fp32 (inverse-H-transformed kept modes, carrying the 1/(H W) scale),
// x [B, Cin, H, W] -> y [B, Cout, H, W] = act(irfft_W(yw) + conv1x1(x, wc) + bias), dtype of x.
void check_fno_c2r(const at::Tensor& yw, const at::Tensor& x, const at::Tensor& wc) {
  TORCH_CHECK(x.dim() == 4 && yw.dim() == 5 && yw.size(4) == 2, "fno_c2r_pw: yw [B, Cout, H, m, 2], x [B, Cin, H, W]");
  TORCH_CHECK(yw.size(0) == x.size(0) && yw.size(2) == x.size(2), "fno_c2r_pw: batch / H mismatch");
  TORCH_CHECK(wc.numel() == yw.size(1) * x.size(1), "fno_c2r_pw: wc must be [Cout, Cin]");
  TORCH_CHECK(2 * (yw.size(3) - 1) <= x.size(3), "fno_c2r_pw: more modes than the half spectrum");
}

at::Tensor fno_c2r_pw_cpu(const at::Tensor& yw, const at::Tensor& x, const at::Tensor& wc,
                          const c10::optional<at::Tensor>& bias, bool gelu) {
  check_fno_c2r(yw, x, wc);
  const int64_t W = x.size(3), m = yw.size(3);
  at::Tensor full = at::zeros({yw.size(0), yw.size(1), yw.size(2), W / 2 + 1}, yw.options().dtype(at::kComplexDouble));
  full.narrow(3, 0, m).copy_(at::view_as_complex(yw.to(at::kDouble).contiguous()));
  at::Tensor spec = at::fft_irfft(full, W, 3, "forward").to(at::kFloat);
  return fno_pointwise_cpu(spec, x, wc.reshape({yw.size(1), x.size(1)}), bias, gelu);
}

at::Tensor fno_c2r_pw_cuda(const at::Tensor& yw_, const at::Tensor& x_, const at::Tensor& wc_,
                           const c10::optional<at::Tensor>& bias, bool gelu) {
  const c10::DeviceGuard guard(x_.device());
  check_fno_c2r(yw_, x_, wc_);
  TORCH_CHECK(x_.scalar_type() == at::kFloat || x_.scalar_type() == at::kBFloat16,
              "fno_c2r_pw: x must be float32 or bfloat16");
  const int64_t B = x_.size(0), Cin = x_.size(1), H = x_.size(2), W = x_.size(3), Cout = yw_.size(1),
                m = yw_.size(3);
  if (!fno_c2r_pw_supported(static_cast<int>(Cin), static_cast<int>(Cout), static_cast<int>(m),
                            static_cast<int>(W), x_.scalar_type() == at::kBFloat16)) {
    // shapes outside the fused kernel: C2R on the FFT kernels + the pointwise kernel
    static auto c2r = c10::Dispatcher::singleton()
                          .findSchemaOrThrow("amd_dft::c2r", "")
                          .typed<at::Tensor(const at::Tensor&, at::IntArrayRef, at::IntArrayRef, double,
                                            at::IntArrayRef, std::optional<at::ScalarType>)>();
    const std::vector<int64_t> dim{3}, out_size{W};
    at::Tensor spec = c2r.call(yw_.to(at::kFloat).contiguous(), dim, out_size, 1.0, {}, x_.scalar_type());
    return fno_pointwise_cuda(spec, x_, wc_.reshape({Cout, Cin}), bias, gelu);
  }
  TORCH_CHECK(B * Cin * H * W < (int64_t(1) << 31) && B * Cout * H * W < (int64_t(1) << 31),
              "fno_c2r_pw: tensor too large");
  at::Tensor x = x_.contiguous();
  at::Tensor yw = yw_.to(at::kFloat).contiguous();
  // the tail kernel reads 4 modes per 16-byte load: a view at an odd float2 offset gets its own copy
  if (reinterpret_cast<uintptr_t>(yw.data_ptr()) % 16 != 0) yw = yw.clone();
  at::Tensor wc = wc_.to(at::kFloat).reshape({Cout, Cin}).contiguous();
  at::Tensor bf;
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  at::Tensor y = at::empty({B, Cout, H, W}, x.options());
  auto tabs = get_dft_gemm_tables(x.scalar_type() == at::kBFloat16 ? DftTable::C2R_BF16 : DftTable::C2R_F32,
                                  static_cast<int>(W), static_cast<int>(m), x.device());
  FnoC2RPwLaunch p;
  p.yw = yw.data_ptr();
  p.x = x.data_ptr();
  p.wc = wc.data_ptr<float>();
  p.bias = bf.defined() ? bf.data_ptr<float>() : nullptr;
  p.y = y.data_ptr();
  p.g0 = tabs.first.data_ptr();
  p.rot = tabs.second.data_ptr();
  p.B = static_cast<int>(B);
  p.Cin = static_cast<int>(Cin);
  p.Cout = static_cast<int>(Cout);
  p.H = static_cast<int>(H);
  p.W = static_cast<int>(W);
  p.m = static_cast<int>(m);
  p.bf16 = x.scalar_type() == at::kBFloat16;
  p.gelu = gelu;
  launch_fno_c2r_pw(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return checked(y, "fno_c2r_pw");
}

at::Tensor fno_c2r_pw_meta(const at::Tensor& yw, const at::Tensor& x, const at::Tensor& wc,
                           const c10::optional<at::Tensor>&, bool) {
  return at::empty({x.size(0), yw.size(1), x.size(2), x.size(3)}, x.options());
}

// ------------------------------------------------------------------ SpectralConv2d tail (C2R-W only)
// yw [B, Cout, H, m, 2] fp32 (inverse-H-transformed kept modes, carrying the 1/(H W) scale) ->
// y [B, Cout, H, W] = irfft_W(yw) in out_dtype (float32 default, or bfloat16): the fno_c2r_pw kernel
// without its pointwise branch (no x read, no 1x1 conv, no activation) -- the classic FNO
// SpectralConv2d ends here (BASELINE config 3: rfft2 -> complex mul -> irfft2).
at::ScalarType fno_c2r_dtype(const at::Tensor& yw, int64_t W, const std::optional<at::ScalarType>& out_dtype) {
  TORCH_CHECK(yw.dim() == 5 && yw.size(4) == 2, "fno_c2r: yw must be [B, Cout, H, m, 2]");
  TORCH_CHECK(W >= 1 && 2 * (yw.size(3) - 1) <= W, "fno_c2r: more modes than the half spectrum of W");
  const at::ScalarType dt = out_dtype.has_value() ? *out_dtype : at::kFloat;
  TORCH_CHECK(dt == at::kFloat || dt == at::kBFloat16, "fno_c2r: out_dtype must be float32 or bfloat16");
  return dt;
}

at::Tensor fno_c2r_cpu(const at::Tensor& yw, int64_t W, std::optional<at::ScalarType> out_dtype) {
  const at::ScalarType dt = fno_c2r_dtype(yw, W, out_dtype);
  const int64_t m = yw.size(3);
  at::Tensor full = at::zeros({yw.size(0), yw.size(1), yw.size(2), W / 2 + 1}, yw.options().dtype(at::kComplexDouble));
  full.narrow(3, 0, m).copy_(at::view_as_complex(yw.to(at::kDouble).contiguous()));
  return at::fft_irfft(full, W, 3, "forward").to(dt);
}

at::Tensor fno_c2r_cuda(const at::Tensor& yw_, int64_t W, std::optional<at::ScalarType> out_dtype) {
  const c10::DeviceGuard guard(yw_.device());
  const at::ScalarType dt = fno_c2r_dtype(yw_, W, out_dtype);
  const int64_t B = yw_.size(0), Cout = yw_.size(1), H = yw_.size(2), m = yw_.size(3);
  if (!fno_c2r_pw_supported(1, static_cast<int>(Cout), static_cast<int>(m), static_cast<int>(W), dt == at::kBFloat16) ||
      B * Cout * H * W >= (int64_t(1) << 31)) {
    // shapes outside the fused kernel: C2R on the FFT kernels
    static auto c2r = c10::Dispatcher::singleton()
                          .findSchemaOrThrow("amd_dft::c2r", "")
                          .typed<at::Tensor(const at::Tensor&, at::IntArrayRef, at::IntArrayRef, double,
                                            at::IntArrayRef, std::optional<at::ScalarType>)>();
    const std::vector<int64_t> dim{3}, out_size{W};
    return c2r.call(yw_.to(at::kFloat).contiguous(), dim, out_size, 1.0, {}, dt);
  }
  at::Tensor yw = yw_.to(at::kFloat).contiguous();
  // the tail kernel reads 4 modes per 16-byte load: a view at an odd float2 offset gets its own copy
  if (reinterpret_cast<uintptr_t>(yw.data_ptr()) % 16 != 0) yw = yw.clone();
  at::Tensor y = at::empty({B, Cout, H, W}, yw.options().dtype(dt));
  auto tabs = get_dft_gemm_tables(dt == at::kBFloat16 ? DftTable::C2R_BF16 : DftTable::C2R_F32, static_cast<int>(W),
                                  static_cast<int>(m), yw.device());
  FnoC2RPwLaunch p;
  p.yw = yw.data_ptr();
  p.x = nullptr;  // spectral path only
  p.wc = nullptr;
  p.bias = nullptr;
  p.y = y.data_ptr();
  p.g0 = tabs.first.data_ptr();
  p.rot = tabs.second.data_ptr();
  p.B = static_cast<int>(B);
  p.Cin = 0;
  p.Cout = static_cast<int>(Cout);
  p.H = static_cast<int>(H);
  p.W = static_cast<int>(W);
  p.m = static_cast<int>(m);
  p.bf16 = dt == at::kBFloat16;
  p.gelu = 0;
  launch_fno_c2r_pw(p, c10::hip::getCurrentHIPStream(yw.device().index()).stream());
  return checked(y, "fno_c2r");
}

at::Tensor fno_c2r_meta(const at::Tensor& yw, int64_t W, std::optional<at::ScalarType> out_dtype) {
  return at::empty({yw.size(0), yw.size(1), yw.size(2), W}, yw.options().dtype(out_dtype.has_value() ? *out_dtype : at::kFloat));
}

// ------------------------------------------------------------------ LayerNorm (+ residual)
std::tuple<at::Tensor, at::Tensor> layer_norm_cpu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                                  double eps, const std::optional<at::Tensor>& residual) {
  at::Tensor xs = residual.has_value() ? (x.to(at::kFloat) + residual->to(at::kFloat)).to(x.scalar_type()) : x;
  at::Tensor y = at::layer_norm(xs.to(at::kFloat), {x.size(-1)}, w.to(at::kFloat), b.to(at::kFloat), eps);
  return {y.to(x.scalar_type()), xs};
}

std::tuple<at::Tensor, at::Tensor> layer_norm_cuda(const at::Tensor& x_, const at::Tensor& w_, const at::Tensor& b_,
                                                   double eps, const std::optional<at::Tensor>& residual) {
  const c10::DeviceGuard guard(x_.device());
  if (x_.scalar_type() == at::kFloat && !residual.has_value() && x_.size(-1) % 4 == 0 && x_.size(-1) <= 2048) {
    at::Tensor x = x_.contiguous();
    at::Tensor w = w_.to(at::kFloat).contiguous(), b = b_.to(at::kFloat).contiguous();
    at::Tensor y = at::empty_like(x);
    LayerNormLaunch p;
    p.x = x.data_ptr();
    p.y = y.data_ptr();
    p.gamma = w.data_ptr();
    p.beta = b.data_ptr();
    p.residual = nullptr;
    p.resid_out = nullptr;
    p.cols = static_cast<int>(x.size(-1));
    p.rows = x.numel() / p.cols;
    p.eps = static_cast<float>(eps);
    p.bf16 = 0;
    if (p.rows > 0) launch_layernorm(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
    return {y, x};
  }
  if (x_.scalar_type() != at::kBFloat16 || x_.size(-1) % 8 != 0 || x_.size(-1) > 2048) {
    fallback_note("layer_norm", "dtype/shape outside the LayerNorm kernels");
    return layer_norm_cpu(x_, w_, b_, eps, residual);  // ATen ops on the device tensors
  }
  at::Tensor x = x_.contiguous();
  at::Tensor w = w_.to(at::kBFloat16).contiguous(), b = b_.to(at::kBFloat16).contiguous();
  at::Tensor y = at::empty_like(x);
  at::Tensor xs = x;
  LayerNormLaunch p;
  p.x = x.data_ptr();
  p.y = y.data_ptr();
  p.gamma = w.data_ptr();
  p.beta = b.data_ptr();
  p.residual = nullptr;
  p.resid_out = nullptr;
  at::Tensor r;
  if (residual.has_value()) {
    r = residual->to(at::kBFloat16).contiguous();
    TORCH_CHECK(r.sizes() == x.sizes(), "layer_norm: residual shape mismatch");
    xs = at::empty_like(x);
    p.residual = r.data_ptr();
    p.resid_out = xs.data_ptr();
  }
  p.cols = static_cast<int>(x.size(-1));
  p.rows = x.numel() / p.cols;
  p.eps = static_cast<float>(eps);
  p.bf16 = 1;
  if (p.rows > 0) launch_layernorm(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return {y, xs};
}

std::tuple<at::Tensor, at::Tensor> layer_norm_meta(const at::Tensor& x, const at::Tensor&, const at::Tensor&, double,
                                                   const std::optional<at::Tensor>&) {
  return {at::empty_like(x), at::empty_like(x)};
}

// ------------------------------------------------------------------ fp32 LayerNorm -> bf16 split pairs
// y = [..., 2C] = [hi | lo] of LN(x + pre): the A operand of the bf16x3 fc1 GEMM (fp32 path)
at::Tensor layer_norm_split_cpu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, double eps,
                                const std::optional<at::Tensor>& pre) {
  at::Tensor xf = x.to(at::kFloat);
  if (pre.has_value()) xf = xf + pre->to(at::kFloat);
  at::Tensor y = at::layer_norm(xf, {x.size(-1)}, w.to(at::kFloat), b.to(at::kFloat), eps);
  at::Tensor hi = y.to(at::kBFloat16);
  at::Tensor lo = (y - hi.to(at::kFloat)).to(at::kBFloat16);
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 32 == 0, "amd_dft.layer_norm_split: C must be a multiple of 32");
  std::vector<int64_t> v(x.sizes().begin(), x.sizes().end() - 1), o = v;
  v.insert(v.end(), {C / 32, 32});
  o.push_back(2 * C);
  return at::cat({hi.reshape(v), lo.reshape(v)}, -1).reshape(o).contiguous();  // k32-interleaved
}

at::Tensor layer_norm_split_cuda(const at::Tensor& x_, const at::Tensor& w_, const at::Tensor& b_, double eps,
                                 const std::optional<at::Tensor>& pre_) {
  const c10::DeviceGuard guard(x_.device());
  const int64_t C = x_.size(-1);
  TORCH_CHECK(x_.scalar_type() == at::kFloat && C % 32 == 0 && C <= 2048,
              "amd_dft.layer_norm_split: x must be float32 with C % 32 == 0 and C <= 2048");
  TORCH_CHECK(w_.numel() == C && b_.numel() == C && (!pre_.has_value() || pre_->numel() == C),
              "amd_dft.layer_norm_split: weight/bias/pre must have C entries");
  at::Tensor x = x_.contiguous();
  at::Tensor w = w_.to(at::kFloat).contiguous(), b = b_.to(at::kFloat).contiguous(), pre;
  if (pre_.has_value()) pre = pre_->to(at::kFloat).contiguous();
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = 2 * C;
  at::Tensor y = at::empty(os, x.options().dtype(at::kBFloat16));
  LayerNormLaunch p;
  p.x = x.data_ptr();
  p.y = y.data_ptr();
  p.gamma = w.data_ptr();
  p.beta = b.data_ptr();
  p.residual = nullptr;
  p.resid_out = nullptr;
  p.cols = static_cast<int>(C);
  p.rows = x.numel() / C;
  p.eps = static_cast<float>(eps);
  p.bf16 = 0;
  p.split_out = 1;
  p.pre = pre.defined() ? pre.data_ptr<float>() : nullptr;
  if (p.rows > 0) launch_layernorm(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return y;
}

at::Tensor layer_norm_split_meta(const at::Tensor& x, const at::Tensor&, const at::Tensor&, double,
                                 const std::optional<at::Tensor>&) {
  std::vector<int64_t> os(x.sizes().begin(), x.sizes().end());
  os.back() = 2 * os.back();
  return at::empty(os, x.options().dtype(at::kBFloat16));
}

// ------------------------------------------------------------------ LayerNorm statistics only
// (mean, rstd) per row of x' = x + pre: the AFNO W-transforms apply LN(x') on load.
at::Tensor ln_stats_cpu(const at::Tensor& x, const std::optional<at::Tensor>& pre, double eps) {
  at::Tensor xp = x.to(at::kFloat);
  if (pre.has_value()) xp = xp + pre->to(at::kFloat);
  xp = xp.reshape({-1, x.size(-1)});
  auto vm = at::var_mean(xp, {1}, /*correction=*/0, /*keepdim=*/false);
  return at::stack({std::get<1>(vm), at::rsqrt(std::get<0>(vm) + eps)}, 1).contiguous();
}

at::Tensor ln_stats_cuda(const at::Tensor& x_, const std::optional<at::Tensor>& pre_, double eps) {
  const c10::DeviceGuard guard(x_.device());
  const int64_t C = x_.size(-1);
  const bool f32 = x_.scalar_type() == at::kFloat && C % 4 == 0 && C <= 2048;
  if (!f32 && (x_.scalar_type() != at::kBFloat16 || C % 8 != 0 || C > 2048)) {
    fallback_note("ln_stats", "dtype/shape outside the LayerNorm kernels");
    return ln_stats_cpu(x_, pre_, eps);
  }
  at::Tensor x = x_.contiguous();
  at::Tensor pre;
  if (pre_.has_value()) {
    pre = pre_->to(at::kFloat).contiguous();
    TORCH_CHECK(pre.numel() == C, "amd_dft.ln_stats: pre must have one entry per channel");
  }
  const int64_t rows = x.numel() / C;
  at::Tensor st = at::empty({rows, 2}, x.options().dtype(at::kFloat));
  LnStatsLaunch p;
  p.x = x.data_ptr();
  p.pre = pre_.has_value() ? pre.data_ptr<float>() : nullptr;
  p.stats = st.data_ptr<float>();
  p.rows = rows;
  p.cols = static_cast<int>(C);
  p.eps = static_cast<float>(eps);
  p.f32 = f32 ? 1 : 0;
  if (rows > 0) launch_ln_stats(p, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  return checked(st, "ln_stats");
}

at::Tensor ln_stats_meta(const at::Tensor& x, const std::optional<at::Tensor>&, double) {
  return at::empty({x.numel() / std::max<int64_t>(x.size(-1), 1), 2}, x.options().dtype(at::kFloat));
}

// (mean, rstd) per row from [rows, nc, 2] per-64-chunk (mean, M2) partials (linear3_stats);
// shift [rows, 2] (optional): its column 0 is subtracted from the mean (statistics of an operand
// centred on that offset, e.g. c2r_ln_add_split's pairs)
static void check_merge_shift(const at::Tensor& part, const std::optional<at::Tensor>& shift) {
  TORCH_CHECK(part.dim() == 3 && part.size(2) == 2, "amd_dft.ln_stats_merge: part must be [rows, chunks, 2]");
  if (shift) {
    TORCH_CHECK(shift->numel() == part.size(0) * 2 && shift->size(-1) == 2 && shift->device() == part.device(),
                "amd_dft.ln_stats_merge: shift must hold [rows, 2] on the device of part");
  }
}

at::Tensor ln_stats_merge_cpu(const at::Tensor& part, double eps, const std::optional<at::Tensor>& shift) {
  check_merge_shift(part, shift);
  at::Tensor p = part.to(at::kFloat);
  at::Tensor m = p.select(2, 0), q = p.select(2, 1);
  at::Tensor mean = m.mean(1);
  at::Tensor m2 = q.sum(1) + 64.0 * (m - mean.unsqueeze(1)).pow(2).sum(1);
  if (shift) mean = mean - shift->reshape({-1, 2}).select(1, 0).to(at::kFloat);
  return at::stack({mean, at::rsqrt(m2 / (64.0 * p.size(1)) + eps)}, 1).contiguous();
}

at::Tensor ln_stats_merge_cuda(const at::Tensor& part_, double eps, const std::optional<at::Tensor>& shift_) {
  const c10::DeviceGuard guard(part_.device());
  check_merge_shift(part_, shift_);
  TORCH_CHECK(part_.scalar_type() == at::kFloat, "amd_dft.ln_stats_merge: part must be fp32 [rows, chunks, 2]");
  at::Tensor part = part_.contiguous();
  at::Tensor shift = shift_ ? shift_->to(at::kFloat).contiguous() : at::Tensor();
  at::Tensor st = at::empty({part.size(0), 2}, part.options());
  launch_ln_stats_merge(part.data_ptr<float>(), st.data_ptr<float>(), part.size(0), static_cast<int>(part.size(1)), 64,
                        static_cast<float>(eps), c10::hip::getCurrentHIPStream(part.device().index()).stream(),
                        shift.defined() ? shift.data_ptr<float>() : nullptr);
  return checked(st, "ln_stats_merge");
}

at::Tensor ln_stats_merge_meta(const at::Tensor& part, double, const std::optional<at::Tensor>&) {
  return at::empty({part.size(0), 2}, part.options());
}

at::Tensor afno_spectral_meta(const at::Tensor& xw, const at::Tensor&, const at::Tensor&, const at::Tensor&,
                              const at::Tensor&, double) {
  return at::empty_like(xw);
}

}  // namespace
}  // namespace amd_dft

TORCH_LIBRARY_FRAGMENT(amd_dft, m) {
  m.def("afno_spectral(Tensor x, Tensor w1t, Tensor w2t, Tensor b1, Tensor b2, float lam) -> Tensor");
  m.def("afno_spectral_supported(int H, int block_size) -> bool", &amd_dft::afno_spectral_ok);
  m.def("afno_spectral_shapes() -> int[]", &amd_dft::afno_spectral_shape_list);
  m.def("layer_norm(Tensor x, Tensor weight, Tensor bias, float eps, Tensor? residual=None) -> (Tensor, Tensor)");
  m.def("ln_stats(Tensor x, Tensor? pre=None, float eps=1e-6) -> Tensor");
  m.def("ln_stats_merge(Tensor part, float eps=1e-6, Tensor? shift=None) -> Tensor");
  m.def("layer_norm_split(Tensor x, Tensor weight, Tensor bias, float eps, Tensor? pre=None) -> Tensor");
  m.def("fno_mix(Tensor x, Tensor w, int path=0) -> Tensor");
  m.def("fno_pointwise(Tensor? spec, Tensor x, Tensor w, Tensor? bias=None, bool gelu=True) -> Tensor");
  m.def("fno_c2r_pw(Tensor yw, Tensor x, Tensor wc, Tensor? bias=None, bool gelu=True) -> Tensor");
  m.def("fno_c2r(Tensor yw, int W, ScalarType? out_dtype=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(amd_dft, CUDA, m) {
  m.impl("afno_spectral", AMD_DFT_TRACED("amd_dft::afno_spectral", amd_dft::afno_spectral_cuda));
  m.impl("layer_norm", AMD_DFT_TRACED("amd_dft::layer_norm", amd_dft::layer_norm_cuda));
  m.impl("ln_stats", AMD_DFT_TRACED("amd_dft::ln_stats", amd_dft::ln_stats_cuda));
  m.impl("ln_stats_merge", AMD_DFT_TRACED("amd_dft::ln_stats_merge", amd_dft::ln_stats_merge_cuda));
  m.impl("layer_norm_split", AMD_DFT_TRACED("amd_dft::layer_norm_split", amd_dft::layer_norm_split_cuda));
  m.impl("fno_mix", AMD_DFT_TRACED("amd_dft::fno_mix", amd_dft::fno_mix_cuda));
  m.impl("fno_pointwise", AMD_DFT_TRACED("amd_dft::fno_pointwise", amd_dft::fno_pointwise_cuda));
  m.impl("fno_c2r_pw", AMD_DFT_TRACED("amd_dft::fno_c2r_pw", amd_dft::fno_c2r_pw_cuda));
  m.impl("fno_c2r", AMD_DFT_TRACED("amd_dft::fno_c2r", amd_dft::fno_c2r_cuda));
}

TORCH_LIBRARY_IMPL(amd_dft, CPU, m) {
  m.impl("afno_spectral", AMD_DFT_TRACED("amd_dft::afno_spectral", amd_dft::afno_spectral_cpu));
  m.impl("layer_norm", AMD_DFT_TRACED("amd_dft::layer_norm", amd_dft::layer_norm_cpu));
  m.impl("ln_stats", AMD_DFT_TRACED("amd_dft::ln_stats", amd_dft::ln_stats_cpu));
  m.impl("ln_stats_merge", AMD_DFT_TRACED("amd_dft::ln_stats_merge", amd_dft::ln_stats_merge_cpu));
  m.impl("layer_norm_split", AMD_DFT_TRACED("amd_dft::layer_norm_split", amd_dft::layer_norm_split_cpu));
  m.impl("fno_mix", AMD_DFT_TRACED("amd_dft::fno_mix", amd_dft::fno_mix_cpu));
  m.impl("fno_pointwise", AMD_DFT_TRACED("amd_dft::fno_pointwise", amd_dft::fno_pointwise_cpu));
  m.impl("fno_c2r_pw", AMD_DFT_TRACED("amd_dft::fno_c2r_pw", amd_dft::fno_c2r_pw_cpu));
  m.impl("fno_c2r", AMD_DFT_TRACED("amd_dft::fno_c2r", amd_dft::fno_c2r_cpu));
}

TORCH_LIBRARY_IMPL(amd_dft, Meta, m) {
  m.impl("afno_spectral", &amd_dft::afno_spectral_meta);
  m.impl("layer_norm", &amd_dft::layer_norm_meta);
  m.impl("ln_stats", &amd_dft::ln_stats_meta);
  m.impl("ln_stats_merge", &amd_dft::ln_stats_merge_meta);
  m.impl("layer_norm_split", &amd_dft::layer_norm_split_meta);
  m.impl("fno_mix", &amd_dft::fno_mix_meta);
  m.impl("fno_pointwise", &amd_dft::fno_pointwise_meta);
  m.impl("fno_c2r_pw", &amd_dft::fno_c2r_pw_meta);
  m.impl("fno_c2r", &amd_dft::fno_c2r_meta);
}
