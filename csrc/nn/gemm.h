// Host interface of the fused-epilogue bf16 GEMM (csrc/nn/gemm.hip).
#pragma once

#include <cstdint>

namespace amd_dft {

struct GemmLaunch {
  const uint16_t* x;         // [M, K] bf16 (activations)
  const uint16_t* w;         // [N, K] bf16 (weight, F.linear layout)
  const float* bias;         // [N] fp32 or nullptr
  const uint16_t* residual;  // [M, N] bf16 or nullptr (added after the activation)
  uint16_t* y;               // [M, N] bf16
  int M, N, K;
  int act = 0;               // 0 none, 1 GELU (erf)
};
bool gemm_supported(int64_t M, int64_t N, int64_t K);
void launch_gemm(const GemmLaunch& p, void* stream);

}  // namespace amd_dft
