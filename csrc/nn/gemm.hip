// bf16 GEMM with fused epilogue for the FourCastNet MLP / embed / head layers:
//   Y[m, n] = act( sum_k X[m, k] * W[n, k] + bias[n] ) (+ R[m, n])        (F.linear layout)
// X [M, K] and W [N, K] are both K-contiguous; Y [M, N] bf16; fp32 accumulation.
//
// MI355X design:
//  * computed as Y^T = W . X^T so that an MFMA accumulator holds 4 CONSECUTIVE output features of
//    one token (C/D row = feature): the epilogue adds a 4-wide bias vector, applies the
//    activation and writes 8 contiguous bytes per lane (16 lanes = one 32-byte row run);
//  * 256 (features) x 256 (tokens) x 64 (k) block tile, 8 waves as 2 x 4, 128 x 64 per wave on
//    v_mfma_f32_16x16x32_bf16 (8 x 4 accumulator tiles = 128 fp32 per lane);
//  * both operand tiles staged HBM -> LDS by global_load_lds_dwordx4 (no VGPR round trip),
//    double-buffered (2 x 64 KB); LDS rows are 128 B with the 16-byte chunk index XOR-swizzled
//    by (row & 7): the DMA writes lane-linear, so the swizzle is applied to the SOURCE address
//    and undone on the ds_read_b128 fragment reads (conflict-free 8-row groups);
//  * blockIdx -> tile remap keeps consecutive tiles (same token panel, different feature
//    panels) on one XCD so the token panel is served from that XCD's L2.
// Status (profiles/gemm_vs_hipblaslt_r1k.txt, pmc_gemm_r1k.txt): correct, bank-conflict free,
// 0.73-0.82x of hipBLASLt on the FourCastNet MLP shapes (MFMA busy ~34 %, ~40 % of wave time
// waiting on the one-K-tile-deep DMA prefetch).  The models keep hipBLASLt for their plain
// GEMMs until this kernel gets the ping-pong (staggered wave-group) schedule.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "gemm.h"

namespace amd_dft {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kBF = 256;  // features per block (MFMA M)
constexpr int kBT = 256;  // tokens per block (MFMA N)
constexpr int kBK = 64;
constexpr int kThreads = 512;

__device__ __forceinline__ float gelu_erf(float v) {
  const float z = fabsf(v) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = fmaf(-p, __builtin_amdgcn_exp2f(-1.4426950408889634f * z * z), 1.f);
  return 0.5f * v * (1.f + copysignf(e, v));
}

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 v;
  v[0] = static_cast<__bf16>(a);
  v[1] = static_cast<__bf16>(b);
  return __builtin_bit_cast(uint32_t, v);
}

// Pipeline: K-tiles of 64 in two LDS buffers (2 x 64 KB), one K-tile of global_load_lds in
// flight while the current one is computed; fragment reads run one MFMA k-step ahead in a
// second register set, so the barrier that publishes the next K-tile sits between the two
// k-steps' MFMA bursts instead of in front of an idle LDS read.
constexpr int kTileBytes = kBF * kBK * 2;  // one operand, one K-tile: 32 KB

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 7)); }

// one operand tile: rows [r0, r0 + 256) clamped to rmax, k-block kb (64 wide)
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ src, int64_t ld, int r0, int rmax, int kb,
                                           char* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rb = (wave * 4 + i) * 8;  // 8 rows x 128 B per wave-instruction (1 KB, lane-linear)
    const int row = rb + (lane >> 3), pos = lane & 7;
    const int chunk = pos ^ (row & 7);  // source swizzle = inverse of the read swizzle
    const int grow = min(r0 + row, rmax);
    const uint16_t* g = src + static_cast<int64_t>(grow) * ld + kb * kBK + chunk * 8;
    __builtin_amdgcn_global_load_lds(static_cast<const void*>(g), (lds_void*)(lds_tile + rb * 128), 16, 0, 0);
  }
}

// Fragments of one phase: A = 4 of the wave's 8 feature tiles (half `ah`) at k-step `ks`,
// B = the wave's 4 token tiles at k-step `ks` (loaded on ah == 0, reused on ah == 1).
__device__ __forceinline__ void read_a(bf16x8 (&a)[4], const char* buf, int ks, int ah, int wf, int r16, int kq) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    a[i] = *reinterpret_cast<const bf16x8*>(buf + swz(wf * 128 + (ah * 4 + i) * 16 + r16, ks * 4 + kq));
}
__device__ __forceinline__ void read_b(bf16x8 (&bq)[4], const char* buf, int ks, int wt, int r16, int kq) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    bq[j] = *reinterpret_cast<const bf16x8*>(buf + kTileBytes + swz(wt * 64 + j * 16 + r16, ks * 4 + kq));
}

template <int AH>
__device__ __forceinline__ void mfma_phase(f32x4 (&acc)[8][4], const bf16x8 (&a)[4], const bf16x8 (&bq)[4]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[AH * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bq[j], acc[AH * 4 + i][j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

template <int ACT, bool BIAS, bool RES>
__global__ void __launch_bounds__(kThreads) gemm_bf16_kernel(const uint16_t* __restrict__ X,
                                                             const uint16_t* __restrict__ Wt,
                                                             const float* __restrict__ bias,
                                                             const uint16_t* __restrict__ R,
                                                             uint16_t* __restrict__ Y, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [2][W tile | X tile]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wf = wave >> 2, wt = wave & 3;  // 2 (features) x 4 (tokens)
  // ---- XCD-aware tile order (bijective for any grid size)
  const int tiles_f = N / kBF;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = b % 8;
  const int lid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
  const int tt = lid / tiles_f, ft = lid - tt * tiles_f;  // token panel outer, feature panels inner
  const int f0 = ft * kBF, t0 = tt * kBT;
  const int KT = K / kBK;
  const int r16 = lane & 15, kq = lane >> 4;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int kt) {
    char* buf = smem + (kt & 1) * 2 * kTileBytes;
    stage_tile(Wt, K, f0, N - 1, kt, buf, wave, lane);
    stage_tile(X, K, t0, M - 1, kt, buf + kTileBytes, wave, lane);
  };
  stage(0);
  if (KT > 1) {
    stage(1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 landed, tile 1 may fly
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  // phases per K-tile: (ks, ah) = (0,0) (0,1) (1,0) (1,1); fragments are read one phase ahead
  bf16x8 a0[4], a1[4], b0[4], b1[4];
  read_a(a0, smem, 0, 0, wf, r16, kq);
  read_b(b0, smem, 0, wt, r16, kq);

  for (int kt = 0; kt < KT; ++kt) {
    const char* cur = smem + (kt & 1) * 2 * kTileBytes;
    read_a(a1, cur, 0, 1, wf, r16, kq);
    mfma_phase<0>(acc, a0, b0);
    read_a(a0, cur, 1, 0, wf, r16, kq);
    read_b(b1, cur, 1, wt, r16, kq);
    mfma_phase<1>(acc, a1, b0);
    read_a(a1, cur, 1, 1, wf, r16, kq);
    mfma_phase<0>(acc, a0, b1);
    // publish tile kt+1 (this wave's only outstanding DMA) after every read of tile kt retired
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < KT) stage(kt + 2);  // into the buffer every wave just finished reading
    if (kt + 1 < KT) {
      const char* nxt = smem + ((kt + 1) & 1) * 2 * kTileBytes;
      read_a(a0, nxt, 0, 0, wf, r16, kq);
      read_b(b0, nxt, 0, wt, r16, kq);
    }
    mfma_phase<1>(acc, a1, b1);
  }

  // ---- epilogue: lane holds features f..f+3 of token t for each (i, j) tile
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int f = f0 + wf * 128 + i * 16 + 4 * kq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (BIAS) {
      const float4 b4 = *reinterpret_cast<const float4*>(bias + f);
      bv[0] = b4.x;
      bv[1] = b4.y;
      bv[2] = b4.z;
      bv[3] = b4.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = t0 + wt * 64 + j * 16 + r16;
      if (t >= M) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[i][j][e] + bv[e];
        if constexpr (ACT == 1) v[e] = gelu_erf(v[e]);
      }
      const int64_t off = static_cast<int64_t>(t) * N + f;
      if constexpr (RES) {
        const uint2 rr = *reinterpret_cast<const uint2*>(R + off);
        v[0] += __uint_as_float(rr.x << 16);
        v[1] += __uint_as_float(rr.x & 0xffff0000u);
        v[2] += __uint_as_float(rr.y << 16);
        v[3] += __uint_as_float(rr.y & 0xffff0000u);
      }
      *reinterpret_cast<uint2*>(Y + off) = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
    }
  }
}

template <int ACT, bool BIAS>
void launch_res(const GemmLaunch& p, hipStream_t st, dim3 grid, size_t lds) {
  if (p.residual)
    hipLaunchKernelGGL((gemm_bf16_kernel<ACT, BIAS, true>), grid, dim3(kThreads), lds, st, p.x, p.w, p.bias,
                       p.residual, p.y, p.M, p.N, p.K);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<ACT, BIAS, false>), grid, dim3(kThreads), lds, st, p.x, p.w, p.bias,
                       p.residual, p.y, p.M, p.N, p.K);
}

template <int ACT, bool BIAS>
void set_attr() {
  for (bool res : {false, true}) {
    const void* f = res ? reinterpret_cast<const void*>(gemm_bf16_kernel<ACT, BIAS, true>)
                        : reinterpret_cast<const void*>(gemm_bf16_kernel<ACT, BIAS, false>);
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kTileBytes);
    if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: gemm attr: ") + hipGetErrorString(e));
  }
}

}  // namespace

bool gemm_supported(int64_t M, int64_t N, int64_t K) {
  return M >= 1 && N % kBF == 0 && K % kBK == 0 && K >= kBK && M * K < (int64_t(1) << 31) &&
         M * N < (int64_t(1) << 31) && N * K < (int64_t(1) << 31);
}

void launch_gemm(const GemmLaunch& p, void* stream) {
  if (!gemm_supported(p.M, p.N, p.K)) throw std::runtime_error("amd_dft: gemm: needs N % 256 == 0, K % 64 == 0");
  static bool attr_done = false;
  if (!attr_done) {
    set_attr<0, false>();
    set_attr<0, true>();
    set_attr<1, false>();
    set_attr<1, true>();
    attr_done = true;
  }
  const int64_t nwg = ((p.M + kBT - 1) / kBT) * (p.N / kBF);
  const dim3 grid(static_cast<uint32_t>(nwg));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t lds = 4 * kTileBytes;
  const bool bias = p.bias != nullptr;
  if (p.act == 1) {
    if (bias) launch_res<1, true>(p, st, grid, lds);
    else launch_res<1, false>(p, st, grid, lds);
  } else {
    if (bias) launch_res<0, true>(p, st, grid, lds);
    else launch_res<0, false>(p, st, grid, lds);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: gemm launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
