// Host-side FFT planning (no torch dependency).
//
// Replaces the reference's per-configure cufftXtMakePlanMany
// (/root/reference/src/dft_plugins/dft_plugins.cpp:154-177): a plan here is a radix
// factorisation plus an fp64-accurate twiddle table for one transform length; the
// geometry of each pass (batch folding, strides, tiling) is derived per call, which is
// how leading dims are folded into the batch (splitSignalDims, dft_plugins.cpp:249-266).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "fft_desc.h"

namespace amd_dft {

struct Plan1D {
  int32_t L = 1;
  std::vector<int32_t> radices;  // pass order
  std::vector<int32_t> ns, twoff, rootoff;
  int32_t tw_count = 0;
  std::vector<float> tw_host;    // 2 * tw_count floats (re, im)
};

// Radices with register-resident butterflies (radix.h).
bool radix_is_specialised(int r);
// Factorise L into Stockham passes (fewest passes, then cheapest butterflies).
std::vector<int32_t> factorize(int32_t L);
Plan1D make_plan_1d(int32_t L);
std::string describe(const Plan1D& p);

// Copy factorisation / twiddle offsets of `p` into `d` (tw pointer is set by the caller).
void apply_plan(PassDesc& d, const Plan1D& p);

// Geometry of a transform along `axis` of a contiguous tensor.  Logical shapes exclude the
// trailing re/im dim of complex tensors; in/out shapes differ only along `axis`.
void set_axis_geometry(PassDesc& d, const std::vector<int64_t>& in_shape,
                       const std::vector<int64_t>& out_shape, int axis, bool in_complex,
                       bool out_complex);

// Choose T (FFTs per workgroup) and the workgroup size; returns false if even T=1 does not
// fit in LDS.
bool choose_tiling(PassDesc& d);

// Set the vector-IO flags once pointers are known (element size in bytes).
void finalize_vec_flags(PassDesc& d, int in_esize, int out_esize);

// Longest transform a single LDS-resident pass supports.
int64_t max_lds_length();

}  // namespace amd_dft
