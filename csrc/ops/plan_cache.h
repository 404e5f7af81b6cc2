// Per-device cache of FFT plans (radix factorisation + device twiddle table).
#pragma once

#include <ATen/ATen.h>

#include <memory>

#include "../fft/fft_plan.h"

namespace amd_dft {

struct DevPlan {
  Plan1D plan;
  at::Tensor tw;  // device float32 [2*tw_count]
};

// Returns the cached plan for length L on `dev` (created on first use; creation is refused
// while the current stream is capturing a hipGraph).
std::shared_ptr<DevPlan> get_plan(int64_t L, const at::Device& dev);
size_t plan_cache_entries();
size_t plan_cache_pinned();  // plans looked up during a hipGraph capture (never evicted)

// Fragment-ordered twiddle tables of the DFT-as-GEMM kernels, (fragments, phases) on `dev`.
enum class DftTable { R2C = 0, C2R_F32 = 1, C2R_BF16 = 2 };
std::pair<at::Tensor, at::Tensor> get_dft_gemm_tables(DftTable kind, int W, int m, const at::Device& dev);
void plan_cache_reset();

}  // namespace amd_dft
