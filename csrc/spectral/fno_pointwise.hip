// FNO layer epilogue (SURVEY §2.5 K4 companion): the pointwise half of an FNO layer,
//   y[b, o, p] = act( spec[b, o, p] + sum_i w[o, i] * x[b, i, p] + bias[o] ),
// i.e. the 1x1 convolution ("W" path), the add of the spectral path's inverse FFT, the bias and
// the GELU in ONE pass over HBM (channel-first [B, C, H*W] tensors, bf16 or fp32 I/O, fp32 math).
// Unfused this is conv2d + add + gelu = three kernels and ~3x the bytes.
//
// Each lane owns VP consecutive pixels and keeps all CIN input channels of them in registers
// (VP*CIN VGPRs); the weights are wave-uniform, so w[o][i] / bias[o] come in through scalar
// loads and feed v_fma as SGPR operands.  Loads are VP-wide vectors (8 B bf16 / 16 B fp32).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "spectral.h"

namespace amd_dft {
namespace {

constexpr int kNT = 256;

template <bool BF, int VP>
struct Vec;
template <>
struct Vec<true, 4> {
  __device__ static void load(const void* p, float (&v)[4]) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16);
    v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16);
    v[3] = __uint_as_float(u.y & 0xffff0000u);
  }
  __device__ static uint32_t pk(float a, float b) {
    return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(a))) |
           (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(b))) << 16);
  }
  __device__ static void store(void* p, const float (&v)[4]) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
  }
};
template <>
struct Vec<false, 4> {
  __device__ static void load(const void* p, float (&v)[4]) {
    const float4 f = *reinterpret_cast<const float4*>(p);
    v[0] = f.x;
    v[1] = f.y;
    v[2] = f.z;
    v[3] = f.w;
  }
  __device__ static void store(void* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <>
struct Vec<true, 1> {
  __device__ static void load(const void* p, float (&v)[1]) {
    v[0] = __uint_as_float(static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(p)) << 16);
  }
  __device__ static void store(void* p, const float (&v)[1]) {
    *reinterpret_cast<uint16_t*>(p) = __builtin_bit_cast(uint16_t, static_cast<__bf16>(v[0]));
  }
};
template <>
struct Vec<false, 1> {
  __device__ static void load(const void* p, float (&v)[1]) { v[0] = *reinterpret_cast<const float*>(p); }
  __device__ static void store(void* p, const float (&v)[1]) { *reinterpret_cast<float*>(p) = v[0]; }
};

__device__ __forceinline__ float gelu_erf(float v) { return 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); }

template <int CIN, int VP, bool BF, bool GELU, bool HAS_SPEC>
__global__ void __launch_bounds__(kNT) fno_pointwise_kernel(const void* __restrict__ spec, const void* __restrict__ x,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            void* __restrict__ y, int Cout, int P) {
  constexpr int ES = BF ? 2 : 4;
  const int p0 = (blockIdx.x * kNT + threadIdx.x) * VP;
  if (p0 >= P) return;
  const int64_t b = blockIdx.y;
  const char* xb = static_cast<const char*>(x) + (b * CIN * P + p0) * ES;
  float xv[CIN][VP];
#pragma unroll
  for (int i = 0; i < CIN; ++i) Vec<BF, VP>::load(xb + static_cast<int64_t>(i) * P * ES, xv[i]);
  const char* sb = static_cast<const char*>(spec) + (b * Cout * P + p0) * ES;
  char* yb = static_cast<char*>(y) + (b * Cout * P + p0) * ES;
  for (int o = 0; o < Cout; ++o) {
    float acc[VP];
    if constexpr (HAS_SPEC) {
      Vec<BF, VP>::load(sb + static_cast<int64_t>(o) * P * ES, acc);
    } else {
#pragma unroll
      for (int v = 0; v < VP; ++v) acc[v] = 0.f;
    }
    const float bo = bias ? bias[o] : 0.f;
#pragma unroll
    for (int v = 0; v < VP; ++v) acc[v] += bo;
#pragma unroll
    for (int i = 0; i < CIN; ++i) {
      const float wi = w[o * CIN + i];
#pragma unroll
      for (int v = 0; v < VP; ++v) acc[v] = fmaf(wi, xv[i][v], acc[v]);
    }
    if constexpr (GELU) {
#pragma unroll
      for (int v = 0; v < VP; ++v) acc[v] = gelu_erf(acc[v]);
    }
    Vec<BF, VP>::store(yb + static_cast<int64_t>(o) * P * ES, acc);
  }
}

template <int CIN, int VP, bool BF>
void launch_cin(const FnoPointwiseLaunch& p, hipStream_t st) {
  const dim3 grid((p.P / VP + kNT - 1) / kNT, p.B);
#define L_(G, S)                                                                                             \
  hipLaunchKernelGGL((fno_pointwise_kernel<CIN, VP, BF, G, S>), grid, dim3(kNT), 0, st, p.spec, p.x, p.w, p.bias, \
                     p.y, p.Cout, p.P)
  if (p.gelu) {
    if (p.spec) L_(true, true);
    else L_(true, false);
  } else {
    if (p.spec) L_(false, true);
    else L_(false, false);
  }
#undef L_
}

template <int CIN>
void launch_vp(const FnoPointwiseLaunch& p, hipStream_t st) {
  // VP * CIN input values live in VGPRs; vector IO needs every row start 4-element aligned
  const uintptr_t al = 4 * (p.bf16 ? 2 : 4) - 1;
  const bool aligned = !((reinterpret_cast<uintptr_t>(p.x) | reinterpret_cast<uintptr_t>(p.y) |
                          reinterpret_cast<uintptr_t>(p.spec)) & al);
  const bool vec = p.P % 4 == 0 && CIN <= 32 && aligned;
  if (p.bf16) {
    if (vec) launch_cin<CIN, 4, true>(p, st);
    else launch_cin<CIN, 1, true>(p, st);
  } else {
    if (vec) launch_cin<CIN, 4, false>(p, st);
    else launch_cin<CIN, 1, false>(p, st);
  }
}

}  // namespace

bool fno_pointwise_supported(int cin) { return cin == 4 || cin == 8 || cin == 16 || cin == 20 || cin == 32 || cin == 64 || cin == 128; }

void launch_fno_pointwise(const FnoPointwiseLaunch& p, void* stream) {
  if (p.B == 0 || p.P == 0 || p.Cout == 0) return;
  if (p.B > 65535) throw std::runtime_error("amd_dft: fno_pointwise: batch > 65535");
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (p.Cin) {
    case 4: launch_vp<4>(p, st); break;
    case 8: launch_vp<8>(p, st); break;
    case 16: launch_vp<16>(p, st); break;
    case 20: launch_vp<20>(p, st); break;
    case 32: launch_vp<32>(p, st); break;
    case 64: launch_vp<64>(p, st); break;
    case 128: launch_vp<128>(p, st); break;
    default: throw std::runtime_error("amd_dft: fno_pointwise: unsupported Cin " + std::to_string(p.Cin));
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: fno_pointwise launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
