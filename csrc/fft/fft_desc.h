// Pass descriptor shared between the host planner and the HIP FFT kernels.
//
// A "pass" is one LDS-resident, batched, mixed-radix Stockham transform of
// length L along one tensor axis.  Every multi-dimensional R2C / C2R / C2C
// transform in this library is a chain of such passes (innermost axis first
// for the forward direction, outermost first for the inverse).  This replaces
// the reference's single cufftXtMakePlanMany/cufftXtExec call
// (/root/reference/src/dft_plugins/dft_plugins.cpp:171-176, :192-195) and the
// separate cublasScalEx normalisation (:457-468), which is fused into the
// store of the last pass here.
//
// All strides are in *scalar* units of the tensor they index (a complex
// element occupies two consecutive scalars, re then im).
#pragma once

#include <cstdint>

namespace amd_dft {

constexpr int kMaxPasses = 16;

enum class Kind : int32_t {
  C2C = 0,  // complex -> complex
  R2C = 1,  // real -> half spectrum (two real signals packed per complex FFT)
  C2R = 2,  // half spectrum -> real (two real signals produced per complex FFT)
};

enum class DType : int32_t { F32 = 0, BF16 = 1 };

// Division by a runtime-invariant divisor via multiply-high (valid for n < 2^31).
struct FastDiv {
  uint32_t d = 1, m = 1, s = 0;
  FastDiv() = default;
  explicit FastDiv(uint32_t div) : d(div) {
    s = 0;
    while ((uint64_t(1) << s) < d) ++s;
    m = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1);
  }
};

struct PassDesc {
  const void* in = nullptr;
  void* out = nullptr;
  const void* tw = nullptr;  // device float2 table: per-pass twiddles + generic radix roots
  const void* add1 = nullptr;  // C2R epilogue addends (same layout and dtype as out), or null
  const void* add2 = nullptr;
  // LayerNorm fused into the IO of a channel-last transform (AFNO W-direction passes over
  // [B, H, W, C]: outer o = (b, h), inner = channel, token = o * L + n).  R2C: the input is
  // normalised on load, LN(x + pre).  C2R: add1 = x (stored residual stream) and the epilogue
  // adds x' + LN(x'), x' = x + pre.  Fixed (specialised) kernels only.
  const float* ln_stats = nullptr;  // [O * L] x (mean, rstd) of x' per token
  const float* ln_gamma = nullptr;  // [I] fp32
  const float* ln_beta = nullptr;   // [I] fp32
  const float* ln_pre = nullptr;    // [I] fp32 or null
  // FNO mode mixing fused into the first-pass gather of a pruned C2C (fixed column kernels,
  // fp32): the transform input is never stored; element (outer o = b * mix_cout + oc, signal c,
  // stored mode s) is  sum_i in[b][i][s][c] * mix_w[i][oc][s][c]  (complex), where `in` is the
  // [B, mix_cin, S, I] mode tensor and mix_w the [mix_cin, mix_cout, S, I] weights (the per-outer
  // stride So_in is that of one [S, I] channel slice).
  const float* mix_w = nullptr;
  int32_t mix_cin = 0, mix_cout = 0;

  int32_t L = 1;       // transform length
  int32_t npass = 0;   // number of Stockham passes (0 when L == 1)
  int32_t radix[kMaxPasses] = {};
  int32_t ns[kMaxPasses] = {};       // product of the radices of the previous passes
  int32_t twoff[kMaxPasses] = {};    // offset of this pass' twiddles in the table
  int32_t rootoff[kMaxPasses] = {};  // offset of R-th roots of unity (generic radices only)
  FastDiv ns_div[kMaxPasses];        // j % ns[p]
  FastDiv L_div;                     // position loops over L
  FastDiv out_div;                   // store loop over the stored output count
  int32_t tw_count = 0;              // number of float2 entries in the table

  int32_t T = 1;      // complex FFTs per workgroup (power of two)
  int32_t logT = 0;
  int32_t nthreads = 256;
  int32_t tiles_per_outer = 1;

  int64_t O = 1, So_in = 0, So_out = 0;   // outer batch
  int64_t I = 1, Si_in = 0, Si_out = 0;   // inner (logical) signals
  int64_t Sn_in = 1, Sn_out = 1;          // element stride along the transformed axis

  // Pruning.  Input: only positions [0,in_lo) u [L-in_hi,L) are non-zero and they are
  // stored compactly (in_lo+in_hi entries).  Output: only [0,out_lo) u [L-out_hi,L) are
  // stored, compactly.  R2C: out_lo <= L/2+1, out_hi == 0.  C2R: in_lo <= L/2+1, in_hi == 0.
  int32_t in_lo = 1, in_hi = 0, out_lo = 1, out_hi = 0;

  float scale = 1.0f;
  int32_t inverse = 0;   // 1: e^{+2 pi i nk/L}
  int32_t vec_in = 0;    // R2C: the two paired real inputs are adjacent + aligned (one vector load)
  int32_t vec_out = 0;   // R2C: the two paired complex outputs adjacent + aligned; C2R: real outputs adjacent

  Kind kind = Kind::C2C;
  DType tin = DType::F32, tout = DType::F32;
};

// Host-side launcher implemented in fft_kernels.hip.  `stream` is a hipStream_t.
void launch_fft_pass(const PassDesc& d, void* stream);
// Dynamic LDS bytes the pass kernel needs.
int64_t pass_lds_bytes(const PassDesc& d);
// Largest LDS a single workgroup may use on gfx950 (160 KiB).
constexpr int64_t kMaxLdsBytes = 160 * 1024;

}  // namespace amd_dft
