// Patchify / un-patchify for FourCastNet's 8x8 patch embedding and head (bf16; fp32 moves two
// 16-byte chunks per patch row).
//
// patchify:   x [B, C, h*p, w*p]  ->  tokens [B*h*w, C*p*p]   (feature order (c, py, px))
// unpatchify: t [B, h, w, C, p, p] -> x [B, C, h*p, w*p]
// With p*sizeof(bf16) == 16 bytes every 16-byte chunk (one patch row of one channel) maps to a
// 16-byte chunk: one dwordx4 load and one dwordx4 store per lane.  A 256-thread workgroup owns
// (b, c, patch-row i, 32 consecutive patches j): its 8 x 32 chunks are 8 image rows x 512
// contiguous bytes on one side and 32 tokens x one full 128-byte line on the other, so both
// sides are line-complete within one workgroup (no cross-XCD re-fetch of shared lines) and all
// index math is 32-bit with no divisions (the first version decomposed a 64-bit linear index
// with 64-bit div/mod: ~90 VALU per 16-byte chunk and 3.6x read over-fetch, see
// profiles/).  The head weight is permuted once on the host so that its GEMM emits the
// (c, py, px) order the un-patchify kernel consumes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace amd_dft {
namespace {

constexpr int kP = 8;   // patch size of the vector path (8 bf16 = 16 B)
constexpr int kJ = 32;  // patches per workgroup

template <bool TO_TOKENS, int CPR>  // CPR: 16-byte chunks per patch row (1: bf16, 2: fp32)
__global__ void __launch_bounds__(256) patch_remap_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          int C, int h, int w) {
  // grid: x = ceil(w / kJ), y = h, z = B * C
  const int jj = threadIdx.x & (kJ - 1);
  const int py = threadIdx.x / kJ;  // 0..7
  const int j = blockIdx.x * kJ + jj;
  if (j >= w) return;
  const int i = blockIdx.y;
  const int bc = blockIdx.z;
  const int b = bc / C, c = bc - b * C;
  // image chunk: ((b*C + c) * (h*p) + i*p + py) * w + j
  const int64_t img = ((static_cast<int64_t>(bc) * h * kP + i * kP + py) * w + j) * CPR;
  // token chunk: ((b*h + i) * w + j) * (C*p) + c*p + py
  const int64_t tok = (((static_cast<int64_t>(b) * h + i) * w + j) * (C * kP) + c * kP + py) * CPR;
  uint4 v[CPR];
#pragma unroll
  for (int q = 0; q < CPR; ++q) v[q] = TO_TOKENS ? src[img + q] : src[tok + q];
#pragma unroll
  for (int q = 0; q < CPR; ++q) {
    if constexpr (TO_TOKENS) dst[tok + q] = v[q];
    else dst[img + q] = v[q];
  }
}

}  // namespace

void launch_patch_remap(const void* src, void* dst, int64_t B, int C, int h, int w, bool to_tokens, void* stream,
                        int elem_bytes) {
  if (B * C == 0 || h == 0 || w == 0) return;
  if (B * C > 65535 || h > 65535) throw std::runtime_error("amd_dft: patch_remap grid too large");
  if (elem_bytes != 2 && elem_bytes != 4) throw std::runtime_error("amd_dft: patch_remap: bf16 or fp32 only");
  const dim3 grid((w + kJ - 1) / kJ, h, static_cast<uint32_t>(B * C));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint4* s = static_cast<const uint4*>(src);
  uint4* d = static_cast<uint4*>(dst);
  if (elem_bytes == 2) {
    if (to_tokens) hipLaunchKernelGGL((patch_remap_kernel<true, 1>), grid, dim3(256), 0, st, s, d, C, h, w);
    else hipLaunchKernelGGL((patch_remap_kernel<false, 1>), grid, dim3(256), 0, st, s, d, C, h, w);
  } else {
    if (to_tokens) hipLaunchKernelGGL((patch_remap_kernel<true, 2>), grid, dim3(256), 0, st, s, d, C, h, w);
    else hipLaunchKernelGGL((patch_remap_kernel<false, 2>), grid, dim3(256), 0, st, s, d, C, h, w);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: patch_remap launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
