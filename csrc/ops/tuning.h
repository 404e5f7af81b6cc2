// A/B and tuning switches of the kernel selection (FFT tile / radix / kernel-family choices, GEMM
// epilogue and persistent-grid variants, LayerNorm split kernel).  Each selects between correct
// implementations; the shipped library never reads them (untested product
// surface).  A tuning build reads them from the environment:
//   MI_DFT_HIPCC_EXTRA=-DAMD_DFT_TUNING=1 python -m tensorrt_dft_plugins_amd._build --out build/tuning
// and the benches under bench/ that sweep them load it through MI_DFT_LIB.
// Product switches (MI_DFT_CHECK_FINITE, MI_DFT_STRICT, MI_DFT_TRACE, MI_DFT_PLAN_CACHE_SIZE) are
// read with std::getenv where they are used.
#pragma once

#include <cstdlib>

#ifndef AMD_DFT_TUNING
#define AMD_DFT_TUNING 0
#endif

namespace amd_dft {

inline const char* tuning_env(const char* name) {
#if AMD_DFT_TUNING
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

constexpr bool tuning_build() { return AMD_DFT_TUNING != 0; }

}  // namespace amd_dft
