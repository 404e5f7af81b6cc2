// Device-side bounds checks for debug builds (GPU ASan / XNACK are not
// available on MI355X here).  Build with MI_DFT_DEVICE_CHECKS=1 (tensorrt_dft_plugins_amd/_build.py
// adds -DAMD_DFT_DEVICE_CHECKS): a failed check prints the kernel, the condition and the
// workgroup, then that workgroup returns before the access it guards -- no trap, so a bad
// launch geometry is reported without faulting the device.  Release builds compile the
// checks away.
#pragma once

#include <hip/hip_runtime.h>

#ifdef AMD_DFT_DEVICE_CHECKS
#define AMD_DFT_DEV_CHECK(cond, kernel)                                                              \
  do {                                                                                           \
    if (!(cond)) {                                                                               \
      if (threadIdx.x == 0)                                                                      \
        printf("amd_dft device check failed in %s: %s (block %u)\n", kernel, #cond, blockIdx.x); \
      return;                                                                                    \
    }                                                                                            \
  } while (0)
#else
#define AMD_DFT_DEV_CHECK(cond, kernel) \
  do {                                  \
  } while (0)
#endif
