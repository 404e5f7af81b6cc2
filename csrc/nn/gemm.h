// Host interface of the fused-epilogue bf16 GEMM (csrc/nn/gemm.hip).
#pragma once

#include <cstdint>

namespace amd_dft {

struct GemmLaunch {
  const uint16_t* x = nullptr;       // [M, K] bf16 (activations)
  const uint16_t* w = nullptr;       // [N, K] bf16 (weight, F.linear layout)
  const float* bias = nullptr;       // [N] fp32 or nullptr
  const void* residual = nullptr;    // [M, N] bf16 (fp32 when out == 1) or nullptr (added after the activation)
  void* y = nullptr;                 // [M, N] bf16 / fp32 (out == 1) / [M, 2N] split pair (out == 2)
  const float* ln_stats = nullptr;     // [M, 2] (mean, rstd) fp32 or nullptr: LayerNorm fold (see gemm.hip)
  const float* ln_c1 = nullptr;        // [N] fp32: sum_k W'[n, k] (required with ln_stats)
  int M = 0, N = 0, K = 0;
  int act = 0;               // 0 none, 1 GELU (erf)
  // bf16x3 mode (fp32-class accuracy): x rows are [hi(K) | lo(K)] (row stride 2K; the
  // gathered image instead has its lo plane x_lo elements after the hi plane), w rows [hi | lo]
  int split = 0;
  int out = 0;               // 0 bf16, 1 fp32, 2 split pair [hi(N) | lo(N)] (split mode only)
  int64_t x_lo = 0;
  // Patch-embedding gather (x is an image [B, gC, gh*8, gw*8]; token t = (b, i, j) reads its
  // 8x8 patch of every channel, feature order (c, py, px): one 16-byte chunk per (c, py)).
  int gC = 0, gh = 0, gw = 0;
  int res_rows = 0;          // > 0: residual row = token % res_rows (broadcast over the batch)
  // Un-patchify scatter (y is an image [B, sC, sh*8, sw*8]; feature order (c, py, px)).
  int sC = 0, sh = 0, sw = 0;
  int direct_epi = 0;        // gemm.hip MODE 0: 1 = store straight from the MFMA layout (A/B only)
  float* stats_part = nullptr;       // + residual output (fp32 split mode or bf16): [M, N/64, 2] (mean, M2) per 64-feature chunk
  const float* stats_pre = nullptr;  // [N] added to the output before the statistics (required with stats_part)
  // split-pair residual (fp32 fc2 with statistics only): residual = [M, 2N] bf16x3 pairs of x - m (k32-interleaved)
  // and res_mean = [M, 2] whose .x is the per-token shift m
  const float* res_mean = nullptr;
  const uint16_t* res_lo2 = nullptr;  // optional with res_mean: [M, N] bf16 third split term of x - m
  int ntiles = 0;            // set by launch_gemm: > 0 = persistent grid (gemm.hip PERSIST), tiles in turn
#ifdef AMD_DFT_GEMM_STAMPS
  long long* stamps = nullptr;  // diagnostic build only (bench/gemm_stamps.hip): per-block phase clocks
#endif
};
bool gemm_supported(int64_t M, int64_t N, int64_t K);
void launch_gemm(const GemmLaunch& p, void* stream);

}  // namespace amd_dft
