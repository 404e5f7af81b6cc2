// Row LayerNorm (FourCastNet LN1/LN2 over 768 channels), one wave per row.
//
// bf16 or fp32 I/O, fp32 statistics (two-pass over registers: mean, then centred variance),
// 16-byte vector loads/stores (Guideline 13), wave-level shuffle reductions (64 lanes).
// Optional fused residual: x_out = x + residual is written and normalised in the same pass
// (saves a separate elementwise kernel and one read of x).
#include <hip/hip_runtime.h>

#include <atomic>

#include <cstdlib>

#include <stdexcept>
#include <string>

#include "spectral.h"
#include "../ops/tuning.h"

namespace amd_dft {
namespace {

constexpr int kWaves = 4;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void unpack8(uint4 u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint32_t bfpack(float a, float b) {
  return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(a))) |
         (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(b))) << 16);
}

// NCH = 16-byte chunks (8 bf16) per lane, cols <= 64 * 8 * NCH
template <int NCH, bool RES>
__global__ void __launch_bounds__(64 * kWaves) ln_bf16_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                              const uint16_t* __restrict__ g, const uint16_t* __restrict__ b,
                                                              const uint16_t* __restrict__ res, uint16_t* __restrict__ xo,
                                                              int64_t rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nchunk = cols >> 3;
  const uint16_t* xr = x + row * cols;
  float v[NCH][8];
  bool ok[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = lane + 64 * c;
    ok[c] = ch < nchunk;
    const int chc = ok[c] ? ch : 0;
    unpack8(*reinterpret_cast<const uint4*>(xr + chc * 8), v[c]);
    if constexpr (RES) {
      float r[8];
      unpack8(*reinterpret_cast<const uint4*>(res + row * cols + chc * 8), r);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] += r[i];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) s += ok[c] ? v[c][i] : 0.f;
  const float mean = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = v[c][i] - mean;
      q += ok[c] ? d * d : 0.f;
    }
  const float rstd = rsqrtf(wave_sum(q) / cols + eps);
  float gg[NCH][8], bb[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int chc = ok[c] ? lane + 64 * c : 0;
    unpack8(*reinterpret_cast<const uint4*>(g + chc * 8), gg[c]);
    unpack8(*reinterpret_cast<const uint4*>(b + chc * 8), bb[c]);
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (!ok[c]) continue;
    const int ch = lane + 64 * c;
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mean) * rstd * gg[c][i] + bb[c][i];
    *reinterpret_cast<uint4*>(y + row * cols + ch * 8) =
        make_uint4(bfpack(o[0], o[1]), bfpack(o[2], o[3]), bfpack(o[4], o[5]), bfpack(o[6], o[7]));
    if constexpr (RES) {
      *reinterpret_cast<uint4*>(xo + row * cols + ch * 8) = make_uint4(
          bfpack(v[c][0], v[c][1]), bfpack(v[c][2], v[c][3]), bfpack(v[c][4], v[c][5]), bfpack(v[c][6], v[c][7]));
    }
  }
}

template <int NCH>
void launch_bf16(const LayerNormLaunch& p, hipStream_t st) {
  const dim3 grid(static_cast<uint32_t>((p.rows + kWaves - 1) / kWaves));
  const auto* x = static_cast<const uint16_t*>(p.x);
  auto* y = static_cast<uint16_t*>(p.y);
  const auto* g = static_cast<const uint16_t*>(p.gamma);
  const auto* b = static_cast<const uint16_t*>(p.beta);
  if (p.residual)
    hipLaunchKernelGGL((ln_bf16_kernel<NCH, true>), grid, dim3(64 * kWaves), 0, st, x, y, g, b,
                       static_cast<const uint16_t*>(p.residual), static_cast<uint16_t*>(p.resid_out), p.rows, p.cols,
                       p.eps);
  else
    hipLaunchKernelGGL((ln_bf16_kernel<NCH, false>), grid, dim3(64 * kWaves), 0, st, x, y, g, b, nullptr, nullptr,
                       p.rows, p.cols, p.eps);
}

// Statistics only: (mean, rstd) of x' = x + pre per row, fp32 [rows, 2].  The normalised
// row is never written: the consumers (AFNO W-transforms) apply LN(x') on load.
template <int NCH, bool PRE>
__global__ void __launch_bounds__(64 * kWaves) ln_stats_kernel(const uint16_t* __restrict__ x,
                                                               const float* __restrict__ pre, float2* __restrict__ st,
                                                               int64_t rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nchunk = cols >> 3;
  const uint16_t* xr = x + row * cols;
  float v[NCH][8];
  bool ok[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = lane + 64 * c;
    ok[c] = ch < nchunk;
    const int chc = ok[c] ? ch : 0;
    unpack8(*reinterpret_cast<const uint4*>(xr + chc * 8), v[c]);
    if constexpr (PRE) {
      const float4 p0 = *reinterpret_cast<const float4*>(pre + chc * 8);
      const float4 p1 = *reinterpret_cast<const float4*>(pre + chc * 8 + 4);
      v[c][0] += p0.x; v[c][1] += p0.y; v[c][2] += p0.z; v[c][3] += p0.w;
      v[c][4] += p1.x; v[c][5] += p1.y; v[c][6] += p1.z; v[c][7] += p1.w;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) s += ok[c] ? v[c][i] : 0.f;
  const float mean = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = v[c][i] - mean;
      q += ok[c] ? d * d : 0.f;
    }
  const float rstd = rsqrtf(wave_sum(q) / cols + eps);
  if (lane == 0) st[row] = make_float2(mean, rstd);
}

// Two rows per wave for rows of 96 chunks (768 channels): 192 chunks = exactly 3 per lane, all
// loads of both rows in flight at once (the one-row-per-wave kernel leaves half the lanes
// idle on its second chunk and waits on one row's latency per wave).
template <bool PRE>
__global__ void __launch_bounds__(64 * kWaves) ln_stats_768_kernel(const uint16_t* __restrict__ x,
                                                                   const float* __restrict__ pre,
                                                                   float2* __restrict__ st, int64_t rows, float eps) {
  constexpr int kCPR = 96;  // chunks per row
  const int lane = threadIdx.x & 63;
  const int64_t row0 = (static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6)) * 2;
  if (row0 >= rows) return;
  const bool two = row0 + 1 < rows;
  float v[3][8];
  int rsel[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int c = lane + 64 * i;  // chunk in the two-row span
    const int r = c >= kCPR ? 1 : 0;
    rsel[i] = r;
    const int ch = c - r * kCPR;
    const int64_t row = (r == 1 && !two) ? row0 : row0 + r;
    unpack8(*reinterpret_cast<const uint4*>(x + row * (kCPR * 8) + ch * 8), v[i]);
    if constexpr (PRE) {
      const float4 p0 = *reinterpret_cast<const float4*>(pre + ch * 8);
      const float4 p1 = *reinterpret_cast<const float4*>(pre + ch * 8 + 4);
      v[i][0] += p0.x; v[i][1] += p0.y; v[i][2] += p0.z; v[i][3] += p0.w;
      v[i][4] += p1.x; v[i][5] += p1.y; v[i][6] += p1.z; v[i][7] += p1.w;
    }
  }
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += v[i][k];
    if (rsel[i]) s1 += t;
    else s0 += t;
  }
  const float m0 = wave_sum(s0) * (1.f / 768.f), m1 = wave_sum(s1) * (1.f / 768.f);
  float q0 = 0.f, q1 = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float m = rsel[i] ? m1 : m0;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = v[i][k] - m;
      t += d * d;
    }
    if (rsel[i]) q1 += t;
    else q0 += t;
  }
  const float r0 = rsqrtf(wave_sum(q0) * (1.f / 768.f) + eps), r1 = rsqrtf(wave_sum(q1) * (1.f / 768.f) + eps);
  if (lane == 0) {
    st[row0] = make_float2(m0, r0);
    if (two) st[row0 + 1] = make_float2(m1, r1);
  }
}

template <int NCH>
void launch_stats_n(const LnStatsLaunch& p, hipStream_t st) {
  const dim3 grid(static_cast<uint32_t>((p.rows + kWaves - 1) / kWaves));
  const auto* x = static_cast<const uint16_t*>(p.x);
  auto* o = reinterpret_cast<float2*>(p.stats);
  if (p.pre)
    hipLaunchKernelGGL((ln_stats_kernel<NCH, true>), grid, dim3(64 * kWaves), 0, st, x, p.pre, o, p.rows, p.cols, p.eps);
  else
    hipLaunchKernelGGL((ln_stats_kernel<NCH, false>), grid, dim3(64 * kWaves), 0, st, x, nullptr, o, p.rows, p.cols,
                       p.eps);
}

// ---- fp32 rows (the fp32 FourCastNet path): one wave per row, 16-byte loads, NCH float4
// chunks per lane.  STATS: write (mean, rstd) only.  Otherwise y = LN(x + pre) either as fp32
// or (SPLIT) as a bf16 pair row [hi(cols) | lo(cols)], the operand of the bf16x3 GEMM.
__device__ __forceinline__ uint32_t bfpack_lo(float a, float b, uint32_t hi) {
  const float ha = __uint_as_float(hi << 16), hb = __uint_as_float(hi & 0xffff0000u);
  return bfpack(a - ha, b - hb);
}

template <int NCH, bool STATS, bool SPLIT, bool PRE>
__global__ void __launch_bounds__(64 * kWaves) ln_f32_kernel(const float* __restrict__ x, const float* __restrict__ pre,
                                                             const float* __restrict__ g, const float* __restrict__ b,
                                                             void* __restrict__ y, float2* __restrict__ st,
                                                             int64_t rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nchunk = cols >> 2;
  const float* xr = x + row * cols;
  float v[NCH][4];
  bool ok[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = lane + 64 * c;
    ok[c] = ch < nchunk;
    const int chc = ok[c] ? ch : 0;
    const float4 q = *reinterpret_cast<const float4*>(xr + chc * 4);
    v[c][0] = q.x; v[c][1] = q.y; v[c][2] = q.z; v[c][3] = q.w;
    if constexpr (PRE) {
      const float4 pp = *reinterpret_cast<const float4*>(pre + chc * 4);
      v[c][0] += pp.x; v[c][1] += pp.y; v[c][2] += pp.z; v[c][3] += pp.w;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) s += ok[c] ? v[c][i] : 0.f;
  const float mean = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = v[c][i] - mean;
      q += ok[c] ? d * d : 0.f;
    }
  const float rstd = rsqrtf(wave_sum(q) / cols + eps);
  if constexpr (STATS) {
    if (lane == 0) st[row] = make_float2(mean, rstd);
    return;
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (!ok[c]) continue;
    const int ch = lane + 64 * c;
    const float4 g4 = *reinterpret_cast<const float4*>(g + ch * 4);
    const float4 b4 = *reinterpret_cast<const float4*>(b + ch * 4);
    float o[4];
    o[0] = (v[c][0] - mean) * rstd * g4.x + b4.x;
    o[1] = (v[c][1] - mean) * rstd * g4.y + b4.y;
    o[2] = (v[c][2] - mean) * rstd * g4.z + b4.z;
    o[3] = (v[c][3] - mean) * rstd * g4.w + b4.w;
    if constexpr (SPLIT) {  // k32-interleaved pair row: column c -> (c / 32) * 64 + part * 32 + c % 32
      const int c = ch * 4;
      uint16_t* yr = static_cast<uint16_t*>(y) + row * (2 * cols) + (c >> 5) * 64 + (c & 31);
      const uint32_t h0 = bfpack(o[0], o[1]), h1 = bfpack(o[2], o[3]);
      *reinterpret_cast<uint2*>(yr) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(yr + 32) = make_uint2(bfpack_lo(o[0], o[1], h0), bfpack_lo(o[2], o[3], h1));
    } else {
      *reinterpret_cast<float4*>(static_cast<float*>(y) + row * cols + ch * 4) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

// LayerNorm with the split-pair output, for rows of cols % 256 == 0: the k32-interleaved pair
// row (4 cols bytes) is written as NK full 1-KB wave stores (lane l of store k writes bytes
// [1024 k + 16 l, +16): chunk 8k + l / 8, part (l / 4) & 1, 8 columns (l & 3) * 8) instead of
// 8-byte half-line pieces; lanes l and l ^ 4 normalise the same 8 columns (their loads hit the
// same L1 lines) and store the hi resp. lo half.
template <int NK, bool PRE>
__global__ void __launch_bounds__(64 * kWaves) ln_split_kernel(const float* __restrict__ x, const float* __restrict__ pre,
                                                               const float* __restrict__ g, const float* __restrict__ b,
                                                               uint16_t* __restrict__ y, int64_t rows, float eps) {
  constexpr int cols = NK * 256;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * cols;
  const int cbase = (lane >> 3) * 32 + (lane & 3) * 8;
  float v[NK][8];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = k * 256 + cbase;
    const float4 a = *reinterpret_cast<const float4*>(xr + c0);
    const float4 c = *reinterpret_cast<const float4*>(xr + c0 + 4);
    v[k][0] = a.x; v[k][1] = a.y; v[k][2] = a.z; v[k][3] = a.w;
    v[k][4] = c.x; v[k][5] = c.y; v[k][6] = c.z; v[k][7] = c.w;
    if constexpr (PRE) {
      const float4 pa = *reinterpret_cast<const float4*>(pre + c0);
      const float4 pc = *reinterpret_cast<const float4*>(pre + c0 + 4);
      v[k][0] += pa.x; v[k][1] += pa.y; v[k][2] += pa.z; v[k][3] += pa.w;
      v[k][4] += pc.x; v[k][5] += pc.y; v[k][6] += pc.z; v[k][7] += pc.w;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[k][i];
  const float mean = wave_sum(s) * (0.5f / cols);  // every column is held by two lanes
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = v[k][i] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(wave_sum(q) * (0.5f / cols) + eps);
  const bool lo_half = (lane >> 2) & 1;
  uint16_t* yr = y + row * (2 * cols) + lane * 8;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = k * 256 + cbase;
    const float4 ga = *reinterpret_cast<const float4*>(g + c0), gc = *reinterpret_cast<const float4*>(g + c0 + 4);
    const float4 ba = *reinterpret_cast<const float4*>(b + c0), bc = *reinterpret_cast<const float4*>(b + c0 + 4);
    const float gg[8] = {ga.x, ga.y, ga.z, ga.w, gc.x, gc.y, gc.z, gc.w};
    const float bb[8] = {ba.x, ba.y, ba.z, ba.w, bc.x, bc.y, bc.z, bc.w};
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mean) * rstd * gg[i] + bb[i];
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t h = bfpack(o[2 * i], o[2 * i + 1]);
      w[i] = lo_half ? bfpack_lo(o[2 * i], o[2 * i + 1], h) : h;
    }
    *reinterpret_cast<uint4*>(yr + k * 512) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Same output as ln_split_kernel, but every lane loads 4 UNIQUE columns per 1-KB row slice
// (no duplicated loads across lane pairs: half the vector-memory requests) and the pair row is
// assembled in LDS (3 KB per wave) before the full 1-KB wave stores.
template <int NK, bool PRE>
__global__ void __launch_bounds__(64 * kWaves) ln_split_lds_kernel(const float* __restrict__ x, const float* __restrict__ pre,
                                                                   const float* __restrict__ g, const float* __restrict__ b,
                                                                   uint16_t* __restrict__ y, int64_t rows, float eps) {
  constexpr int cols = NK * 256;
  __shared__ __attribute__((aligned(16))) uint16_t stage[kWaves][2 * cols];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + w;
  if (row >= rows) return;  // no workgroup barrier below: each wave owns its LDS row
  const float* xr = x + row * cols;
  float v[NK][4];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = k * 256 + 4 * lane;
    const float4 a = *reinterpret_cast<const float4*>(xr + c0);
    v[k][0] = a.x; v[k][1] = a.y; v[k][2] = a.z; v[k][3] = a.w;
    if constexpr (PRE) {
      const float4 pa = *reinterpret_cast<const float4*>(pre + c0);
      v[k][0] += pa.x; v[k][1] += pa.y; v[k][2] += pa.z; v[k][3] += pa.w;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) s += v[k][i];
  const float mean = wave_sum(s) * (1.f / cols);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = v[k][i] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / cols) + eps);
  uint16_t* st = stage[w];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c0 = k * 256 + 4 * lane;
    const float4 g4 = *reinterpret_cast<const float4*>(g + c0);
    const float4 b4 = *reinterpret_cast<const float4*>(b + c0);
    const float o0 = (v[k][0] - mean) * rstd * g4.x + b4.x, o1 = (v[k][1] - mean) * rstd * g4.y + b4.y;
    const float o2 = (v[k][2] - mean) * rstd * g4.z + b4.z, o3 = (v[k][3] - mean) * rstd * g4.w + b4.w;
    const uint32_t h0 = bfpack(o0, o1), h1 = bfpack(o2, o3);
    uint16_t* e = st + (c0 >> 5) * 64 + (c0 & 31);  // k32-interleaved: hi at +0, lo at +32
    *reinterpret_cast<uint2*>(e) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(e + 32) = make_uint2(bfpack_lo(o0, o1, h0), bfpack_lo(o2, o3, h1));
  }
  uint16_t* yr = y + row * (2 * cols);
#pragma unroll
  for (int k = 0; k < NK; ++k)
    *reinterpret_cast<uint4*>(yr + k * 512 + lane * 8) = *reinterpret_cast<const uint4*>(st + k * 512 + lane * 8);
}

template <bool STATS, bool SPLIT>
void launch_f32(const float* x, const float* pre, const float* g, const float* b, void* y, float2* st, int64_t rows,
                int cols, float eps, hipStream_t s) {
  const dim3 grid(static_cast<uint32_t>((rows + kWaves - 1) / kWaves)), blk(64 * kWaves);
  const int nch = (cols / 4 + 63) / 64;
#define AMD_DFT_LNF(N)                                                                                       \
  if (pre) hipLaunchKernelGGL((ln_f32_kernel<N, STATS, SPLIT, true>), grid, blk, 0, s, x, pre, g, b, y, st, rows, cols, eps); \
  else hipLaunchKernelGGL((ln_f32_kernel<N, STATS, SPLIT, false>), grid, blk, 0, s, x, pre, g, b, y, st, rows, cols, eps);
  if (nch <= 1) { AMD_DFT_LNF(1) }
  else if (nch == 2) { AMD_DFT_LNF(2) }
  else if (nch == 3) { AMD_DFT_LNF(3) }
  else if (nch <= 4) { AMD_DFT_LNF(4) }
  else { AMD_DFT_LNF(8) }
#undef AMD_DFT_LNF
}

// ---- fp32 -> bf16 split pairs (hi = bf16(x), lo = bf16(x - hi)), 8 elements per thread.
// ROWS: row-major [rows, cols] -> [rows, 2 cols] k32-interleaved pair rows (every 32 columns
// stored as [hi(32) | lo(32)], the bf16x3 GEMM operand layout); else planes [2, n] (hi, lo).
template <bool ROWS>
__global__ void __launch_bounds__(256) split_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                         int64_t n, int cols) {
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 8;
  if (i >= n) return;
  const float4 a = *reinterpret_cast<const float4*>(x + i);
  const float4 c = *reinterpret_cast<const float4*>(x + i + 4);
  const uint32_t h0 = bfpack(a.x, a.y), h1 = bfpack(a.z, a.w), h2 = bfpack(c.x, c.y), h3 = bfpack(c.z, c.w);
  const uint4 hi = make_uint4(h0, h1, h2, h3);
  const uint4 lo = make_uint4(bfpack_lo(a.x, a.y, h0), bfpack_lo(a.z, a.w, h1), bfpack_lo(c.x, c.y, h2),
                              bfpack_lo(c.z, c.w, h3));
  if constexpr (ROWS) {  // k32-interleaved pair rows (8 elements never straddle a 32-chunk)
    const int64_t r = i / cols, col = i - r * cols;
    uint16_t* yr = y + r * 2 * cols + (col >> 5) * 64 + (col & 31);
    *reinterpret_cast<uint4*>(yr) = hi;
    *reinterpret_cast<uint4*>(yr + 32) = lo;
  } else {
    *reinterpret_cast<uint4*>(y + i) = hi;
    *reinterpret_cast<uint4*>(y + n + i) = lo;
  }
}

}  // namespace

// (mean, rstd) per row from per-chunk partials (mean_c, M2_c) of equal chunk width W (Chan et al.:
// mean = avg mean_c, M2 = sum M2_c + W sum (mean_c - mean)^2): the statistics the fp32 fc2 GEMM
// epilogue leaves for the next block's LayerNorm (csrc/nn/gemm.hip, STATS)
// 256 rows per workgroup: the block's partials ([256][nc] float2, contiguous) are staged in LDS
// with coalesced 16-byte loads, then every thread merges its own row (Chan: M2 = sum M2_c +
// width * sum (mean_c - mean)^2).  shift (or nullptr): [rows] float2 whose .x is subtracted from the
// mean -- the statistics of a split-pair operand that was written relative to that offset
// (c2r_ln_add_split centres its pairs on the input stream's mean, see afno_wfft.hip)
constexpr int kMergeMaxNc = 64;  // dynamic LDS 2 KB per chunk: <= 128 KB
__global__ void __launch_bounds__(256) ln_stats_merge_kernel(const float2* __restrict__ part, float2* __restrict__ st,
                                                             const float2* __restrict__ shift, int64_t rows, int nc,
                                                             float width, float eps) {
  extern __shared__ float4 tile[];  // [256 rows][nc] float2
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * 256;
  const int nrow = static_cast<int>(rows - r0 < 256 ? rows - r0 : 256);
  const int n4 = nrow * nc / 2;  // nc is even (checked on the host)
  const float4* src = reinterpret_cast<const float4*>(part + r0 * nc);
  // 8 loads in flight per thread before the first store (clamped, unconditional): the plain copy
  // loop waited one memory round trip per iteration (6 for 12 chunks)
  for (int b = 0; b < n4; b += 256 * 8) {
    float4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = src[min(b + 256 * q + static_cast<int>(threadIdx.x), n4 - 1)];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = b + 256 * q + static_cast<int>(threadIdx.x);
      if (i < n4) tile[i] = v[q];
    }
  }
  __syncthreads();
  if (static_cast<int>(threadIdx.x) >= nrow) return;
  const float2* pp = reinterpret_cast<const float2*>(tile) + threadIdx.x * nc;
  float s = 0.f;
  for (int c = 0; c < nc; ++c) s += pp[c].x;
  const float mean = s / static_cast<float>(nc);
  float m2 = 0.f;
  for (int c = 0; c < nc; ++c) {
    const float2 q = pp[c];
    const float d = q.x - mean;
    m2 += fmaf(width * d, d, q.y);
  }
  const float sh = shift ? shift[r0 + threadIdx.x].x : 0.f;
  st[r0 + threadIdx.x] = make_float2(mean - sh, rsqrtf(m2 / (width * static_cast<float>(nc)) + eps));
}

void launch_ln_stats_merge(const float* part, float* stats, int64_t rows, int nc, int width, float eps, void* stream,
                           const float* shift) {
  if (rows <= 0) return;
  if (nc <= 0 || nc % 2 || nc > kMergeMaxNc || width <= 0)
    throw std::runtime_error("amd_dft: ln_stats_merge: needs an even chunk count <= 64");
  const dim3 grid(static_cast<uint32_t>((rows + 255) / 256));
  const int lds = 256 * nc * 8;
  if (lds > 64 * 1024) {  // above the default dynamic-LDS limit (per device, like the GEMM's)
    static std::atomic<uint64_t> attr_done{0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) throw std::runtime_error("amd_dft: ln_stats_merge: bad device");
    if (!(attr_done.load(std::memory_order_acquire) & (uint64_t(1) << dev))) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(ln_stats_merge_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 256 * kMergeMaxNc * 8);
      if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: ln_stats_merge attr: ") + hipGetErrorString(e));
      attr_done.fetch_or(uint64_t(1) << dev, std::memory_order_acq_rel);
    }
  }
  hipLaunchKernelGGL(ln_stats_merge_kernel, grid, dim3(256), lds, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const float2*>(part), reinterpret_cast<float2*>(stats),
                     reinterpret_cast<const float2*>(shift), rows, nc,
                     static_cast<float>(width), eps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: ln_stats_merge launch: ") + hipGetErrorString(e));
}

void launch_ln_stats(const LnStatsLaunch& p, void* stream) {
  if (p.f32) {
    if (p.cols % 4 != 0 || p.cols > 64 * 4 * 8) throw std::runtime_error("amd_dft: ln_stats: fp32 rows need cols % 4 == 0, <= 2048");
    launch_f32<true, false>(static_cast<const float*>(p.x), p.pre, nullptr, nullptr, nullptr,
                            reinterpret_cast<float2*>(p.stats), p.rows, p.cols, p.eps, static_cast<hipStream_t>(stream));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: ln_stats launch: ") + hipGetErrorString(e));
    return;
  }
  if (p.cols % 8 != 0 || p.cols > 64 * 8 * 4)
    throw std::runtime_error("amd_dft: ln_stats kernel supports bf16 rows with cols % 8 == 0 and cols <= 2048");
  if (p.rows > static_cast<int64_t>(0x7fffffff) * kWaves) throw std::runtime_error("amd_dft: ln_stats: too many rows");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nch = (p.cols / 8 + 63) / 64;
  if (p.cols == 768) {
    const dim3 grid(static_cast<uint32_t>((p.rows + 2 * kWaves - 1) / (2 * kWaves)));
    const auto* x = static_cast<const uint16_t*>(p.x);
    auto* o = reinterpret_cast<float2*>(p.stats);
    if (p.pre)
      hipLaunchKernelGGL((ln_stats_768_kernel<true>), grid, dim3(64 * kWaves), 0, st, x, p.pre, o, p.rows, p.eps);
    else
      hipLaunchKernelGGL((ln_stats_768_kernel<false>), grid, dim3(64 * kWaves), 0, st, x, nullptr, o, p.rows, p.eps);
  } else if (nch <= 1) launch_stats_n<1>(p, st);
  else if (nch == 2) launch_stats_n<2>(p, st);
  else launch_stats_n<4>(p, st);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: ln_stats launch: ") + hipGetErrorString(e));
}

void launch_layernorm(const LayerNormLaunch& p, void* stream) {
  if (!p.bf16) {
    if (p.residual || p.cols % 4 != 0 || p.cols > 64 * 4 * 8)
      throw std::runtime_error("amd_dft: layernorm: fp32 rows need cols % 4 == 0, <= 2048, no residual");
    if (p.split_out && p.cols % 32 != 0) throw std::runtime_error("amd_dft: layernorm: split output needs cols % 32 == 0");
    const auto* x = static_cast<const float*>(p.x);
    const auto* g = static_cast<const float*>(p.gamma);
    const auto* b = static_cast<const float*>(p.beta);
    if (p.split_out && p.cols == 768 && p.rows <= static_cast<int64_t>(0x7fffffff) * kWaves) {
      const dim3 grid(static_cast<uint32_t>((p.rows + kWaves - 1) / kWaves)), blk(64 * kWaves);
      auto* y = static_cast<uint16_t*>(p.y);
      hipStream_t s = static_cast<hipStream_t>(stream);
      static const bool dup = [] {  // MI_DFT_LN_SPLIT=dup: the duplicated-load kernel (A/B only)
        const char* e = tuning_env("MI_DFT_LN_SPLIT");
        return e && std::string(e) == "dup";
      }();
      if (dup) {
        if (p.pre) hipLaunchKernelGGL((ln_split_kernel<3, true>), grid, blk, 0, s, x, p.pre, g, b, y, p.rows, p.eps);
        else hipLaunchKernelGGL((ln_split_kernel<3, false>), grid, blk, 0, s, x, nullptr, g, b, y, p.rows, p.eps);
      } else {
        if (p.pre) hipLaunchKernelGGL((ln_split_lds_kernel<3, true>), grid, blk, 0, s, x, p.pre, g, b, y, p.rows, p.eps);
        else hipLaunchKernelGGL((ln_split_lds_kernel<3, false>), grid, blk, 0, s, x, nullptr, g, b, y, p.rows, p.eps);
      }
    } else if (p.split_out) {
      launch_f32<false, true>(x, p.pre, g, b, p.y, nullptr, p.rows, p.cols, p.eps, static_cast<hipStream_t>(stream));
    }
    else launch_f32<false, false>(x, p.pre, g, b, p.y, nullptr, p.rows, p.cols, p.eps, static_cast<hipStream_t>(stream));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: layernorm launch: ") + hipGetErrorString(e));
    return;
  }
  if (!p.bf16 || p.cols % 8 != 0 || p.cols > 64 * 8 * 4)
    throw std::runtime_error("amd_dft: layernorm kernel supports bf16 rows with cols % 8 == 0 and cols <= 2048");
  if (p.rows > static_cast<int64_t>(0x7fffffff) * kWaves) throw std::runtime_error("amd_dft: layernorm: too many rows");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int nch = (p.cols / 8 + 63) / 64;
  if (nch <= 1) launch_bf16<1>(p, st);
  else if (nch == 2) launch_bf16<2>(p, st);
  else launch_bf16<4>(p, st);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: layernorm launch: ") + hipGetErrorString(e));
}

void launch_split_bf16(const float* x, uint16_t* y, int64_t n, int cols, bool rows, void* stream) {
  if (n % 8 != 0 || (rows && cols % 32 != 0))
    throw std::runtime_error("amd_dft: split_bf16: needs 8-element multiples (rows: cols % 32 == 0)");
  if (n == 0) return;
  const dim3 grid(static_cast<uint32_t>((n / 8 + 255) / 256));
  if (rows) hipLaunchKernelGGL(split_bf16_kernel<true>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), x, y, n, cols);
  else hipLaunchKernelGGL(split_bf16_kernel<false>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), x, y, n, cols);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: split_bf16 launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
