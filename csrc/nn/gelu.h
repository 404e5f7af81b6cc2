// erf-GELU for the hand GEMM epilogues (exact-erf form, as torch.nn.functional.gelu's default).
//
// Abramowitz & Stegun 7.1.26, |erf error| <= 1.5e-7, rearranged for the VALU: with h = x / 2,
//   x Phi(x) = h (1 + sign(x) erf(|x| / sqrt2)) = h + |h| - |h| P(t) e^{-x^2/2}
//            = max(x, 0) - |x| (P(t) / 2) e^{-x^2/2},   t = 1 / (1 + p |x| / sqrt2)
// (the 1/2 and 1/sqrt2 folded into the constants): 12 VALU + rcp + exp2 per value, against 14 + 2
// transcendental-rate ops for the textbook 0.5 x (1 + erf) form.  |x| is clamped to 1e30 so
// that x = +-inf gives inf / 0 instead of inf * 0.
#pragma once

namespace amd_dft {

__device__ __forceinline__ float gelu_erf(float x) {
  const float ax = fminf(fabsf(x), 1e30f);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, ax, 1.f));
  float p = fmaf(0.5f * 1.061405429f, t, 0.5f * -1.453152027f);
  p = fmaf(p, t, 0.5f * 1.421413741f);
  p = fmaf(p, t, 0.5f * -0.284496736f);
  p = fmaf(p, t, 0.5f * 0.254829592f);
  p *= t;
  const float ex = __builtin_amdgcn_exp2f(x * x * (-0.5f * 1.4426950408889634f));
  return fmaf(-ax * p, ex, fmaxf(x, 0.f));
}

}  // namespace amd_dft

namespace amd_dft {

// The same erf-GELU on two values with packed fp32 VALU (v_pk_fma_f32 / v_pk_mul_f32: one issue
// slot for both values; rcp / exp2 / min / max stay per value).  Bit-identical to gelu_erf (same
// operations in the same order, one rounding each).  For epilogues only: beside MFMAs packed
// f32 VALU is an anti-lever (MI355X_MICROARCH.md, cycle constants), in an epilogue it halves the
// polynomial's issue cost.
typedef float gelu_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ gelu_f2 gelu_erf2(gelu_f2 x) {
  const gelu_f2 ax = {fminf(fabsf(x.x), 1e30f), fminf(fabsf(x.y), 1e30f)};
  const gelu_f2 d = __builtin_elementwise_fma(gelu_f2(0.3275911f * 0.70710678118654752f), ax, gelu_f2(1.f));
  const gelu_f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  gelu_f2 p = __builtin_elementwise_fma(gelu_f2(0.5f * 1.061405429f), t, gelu_f2(0.5f * -1.453152027f));
  p = __builtin_elementwise_fma(p, t, gelu_f2(0.5f * 1.421413741f));
  p = __builtin_elementwise_fma(p, t, gelu_f2(0.5f * -0.284496736f));
  p = __builtin_elementwise_fma(p, t, gelu_f2(0.5f * 0.254829592f));
  p *= t;
  const gelu_f2 e = (x * x) * gelu_f2(-0.5f * 1.4426950408889634f);
  const gelu_f2 ex = {__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
  const gelu_f2 m = {fmaxf(x.x, 0.f), fmaxf(x.y, 0.f)};
  return __builtin_elementwise_fma(-ax * p, ex, m);
}

}  // namespace amd_dft

namespace amd_dft {

// GELU in the tanh form (torch.nn.functional.gelu(approximate="tanh")), two values per packed op:
//   x Phi(x) ~= x / (1 + 2^(x (c1 + c2 x^2))),  c1 = -2 sqrt(2/pi) log2(e), c2 = 0.044715 c1
// |error vs the erf form| < 5e-4 absolute (3.4e-4 at |x| ~ 2): below half a bf16 ulp for |y| >= 0.25.
// 5 packed VALU + 2 exp2 + 2 rcp per pair (the erf form: 11 + 4 min/max/abs + the same 4 transcendentals).
__device__ __forceinline__ gelu_f2 gelu_tanh2(gelu_f2 x) {
  constexpr float c1 = -1.5957691216057308f * 1.4426950408889634f;
  constexpr float c2 = c1 * 0.044715f;
  const gelu_f2 z = x * __builtin_elementwise_fma(gelu_f2(c2), x * x, gelu_f2(c1));
  const gelu_f2 d = gelu_f2{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} + gelu_f2(1.f);
  return x * gelu_f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

}  // namespace amd_dft

namespace amd_dft {

// erf-GELU for bf16 outputs: x Phi(x) ~= x sigmoid(x q(x^2)), q a quadratic in x^2 (x^2 clamped at 64,
// where Phi is 1 to fp32 precision) fitted minimax on [-10, 10]:
//   |error vs the exact erf form| <= 2.6e-5 absolute (fp32 evaluation; the tanh form: 4.7e-4),
// i.e. 1/40 of half a bf16 ulp at |y| = 0.25 -- FourCastNet's nn.GELU at the resolution of a bf16
// output, for one packed FMA and two min more than the tanh form (the A&S erf: 11 packed + 4 + the
// same transcendentals).  Used where the bf16 models' GELU is configured as "erf".
//   x sigmoid(x q) = x / (1 + 2^(x k(x^2))),  k = -q log2(e)
constexpr float kGeluFitK0 = -2.3011176586151123f;
constexpr float kGeluFitK1 = -0.10677912831306458f;
constexpr float kGeluFitK2 = 0.0010148165747523308f;

__device__ __forceinline__ float gelu_erf_fit(float x) {
  const float x2 = fminf(x * x, 64.f);
  const float z = x * fmaf(x2, fmaf(x2, kGeluFitK2, kGeluFitK1), kGeluFitK0);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));
}

__device__ __forceinline__ gelu_f2 gelu_erf_fit2(gelu_f2 x) {
  const gelu_f2 xx = x * x;
  const gelu_f2 x2 = {fminf(xx.x, 64.f), fminf(xx.y, 64.f)};
  const gelu_f2 q = __builtin_elementwise_fma(x2, __builtin_elementwise_fma(x2, gelu_f2(kGeluFitK2), gelu_f2(kGeluFitK1)),
                                              gelu_f2(kGeluFitK0));
  const gelu_f2 z = x * q;
  const gelu_f2 d = gelu_f2{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} + gelu_f2(1.f);
  return x * gelu_f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

}  // namespace amd_dft
