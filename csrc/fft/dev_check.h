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
// LDS access check for vectorised (ds_read/write_b128) staging: prints when a byte offset is not
// aligned to the access width or the access ends past the workgroup's LDS size (no return: it
// sits inside inline helpers)
#define AMD_DFT_DEV_LDS(off, width, limit, what)                                                    \
  do {                                                                                            \
    const long long o_ = static_cast<long long>(off);                                             \
    if ((o_ % (width)) != 0 || o_ < 0 || o_ + (width) > static_cast<long long>(limit))            \
      printf("amd_dft LDS check failed in %s: offset %lld width %d limit %lld (block %u thread %u)\n", what, o_, \
             static_cast<int>(width), static_cast<long long>(limit), blockIdx.x, threadIdx.x);    \
  } while (0)
#else
#define AMD_DFT_DEV_CHECK(cond, kernel) \
  do {                                  \
  } while (0)
#define AMD_DFT_DEV_LDS(off, width, limit, what) \
  do {                                           \
  } while (0)
#endif
