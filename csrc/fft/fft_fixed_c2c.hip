// C2C instantiations of the specialised Stockham kernels (see fft_fixed_impl.h).
#include "fft_fixed_impl.h"

namespace amd_dft {
namespace fixed_detail {

#define AMD_DFT_LAUNCHER(L_, COLS_, TP_, T_, ...) &launch_one<Kind::C2C, COLS_, TP_, T_, FL<__VA_ARGS__>>,

LaunchFn c2c_launcher(int idx) {
  static const LaunchFn table[] = {AMD_DFT_FIXED_CONFIGS(AMD_DFT_LAUNCHER)};
  return table[idx];
}

}  // namespace fixed_detail
}  // namespace amd_dft
