// Compile-time specialised Stockham configurations (host-visible table).
//
// For the hot transform lengths (FourCastNet / FNO grids and powers of two) the radix
// sequence, threads per FFT (TP) and FFTs per workgroup (T) are template parameters of
// fft_fixed_kernel (fft_fixed.hip): every loop is unrolled, strides along the transform are
// constants, the first pass reads global memory straight into registers and the last pass
// writes global memory straight from registers (C2C / C2R), so only NPASS-1 LDS round
// trips remain.  The generic runtime-radix kernel (fft_kernels.hip) covers everything else.
#pragma once

#include <cstdint>
#include <vector>

#include "fft_desc.h"

namespace amd_dft {

struct FixedCfg {
  int32_t L;
  bool cols;      // true: signals interleaved along the fast global dim (lane = signal)
  int32_t TP;     // threads per FFT
  int32_t T;      // FFTs per workgroup
  int32_t npass;
  int32_t radix[4];
};

// All compiled configurations (order = preference for the same (L, cols)).
const std::vector<FixedCfg>& fixed_configs();
// Radix order used for L by the fixed kernels (empty if L has no fixed config).
std::vector<int32_t> fixed_radices(int32_t L);
// Launch the best fixed configuration for d; returns false when none applies.
bool launch_fft_fixed(const PassDesc& d, void* stream);


}  // namespace amd_dft
