// Four-wave 256x256x64 MFMA GEMM for the FourCastNet MLP (plain token-major operands):
//   Y[m, n] = act( sum_k X[m, k] * W[n, k] + bias[n] ) (+ R[m, n]),   bf16 or bf16x3 (SPLIT)
//
// Design (gfx950), compared with the 8-wave ping-pong kernel in gemm.hip:
//  * 4 waves, one per SIMD, each owning a 128 (features) x 128 (tokens) quadrant: 8 x 8
//    v_mfma_f32_16x16x32_bf16 accumulators = 256 fp32 per lane, held in the accumulator file
//    (AGPRs) -- 16 ds_read_b128 fragments feed 64 MFMAs per k-step, 1.5x fewer LDS reads per
//    MFMA than 128 x 64 per wave, and a wave never waits for a partner wave's cluster;
//  * one raw s_barrier per 64-deep K-tile; the fragments of the next k-step are read while the
//    current k-step's 64 MFMAs run (register double buffer), and the LDS-DMA
//    (global_load_lds_dwordx4, XOR-swizzled source addresses, lane-linear LDS image) of K-tile
//    t+2 is issued right after the barrier that frees its buffer, so each stage has a full
//    K-tile of MFMA time to land;
//  * Y^T = W . X^T, so a lane's accumulator holds 4 consecutive features of one token: the
//    epilogue adds a float4 bias and stores 8 / 16 contiguous bytes;
//  * XCD-aware bijective blockIdx -> tile remap (token panel outer, feature panels inner).
// Same SPLIT ("bf16x3") convention as gemm.hip: rows [hi(K) | lo(K)], 3 K-segments.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "../fft/dev_check.h"
#include "gelu.h"
#include "gemm.h"

namespace amd_dft {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kBF = 256;                // features per tile
constexpr int kBT = 256;                // tokens per tile
constexpr int kBK = 64;                 // K per stage
constexpr int kThreads = 256;
constexpr int kOpBytes = 256 * 128;     // one operand tile: 256 rows x 128 B
constexpr int kStage = 2 * kOpBytes;    // W tile + X tile (64 KB)
constexpr int kLds = 2 * kStage;        // double buffer (128 KB)
constexpr int kDmaPerWave = 16;         // global_load_lds_dwordx4 per wave per stage

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 7)); }

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 v;
  v[0] = static_cast<__bf16>(a);
  v[1] = static_cast<__bf16>(b);
  return __builtin_bit_cast(uint32_t, v);
}

// Per-lane DMA source offsets of a tile (computed once): wave-instruction q (0..15) moves
// operand q >> 3 (0 = W, 1 = X), rows ((q & 7) * 4 + wave) * 8 + lane / 8, 16-byte chunk
// (lane & 7) ^ (row & 7) (source swizzle = inverse of the read swizzle; row & 7 = lane / 8).
// Offsets are 32-bit from the tile's row-0 pointer (uniform, 64-bit); X rows past M are
// clamped to the last row (their outputs are never stored).
struct DmaLane {
  int wo;       // W: row offset + chunk (q adds (q & 7) * 32 rows, uniform)
  int xo[8];    // X: clamped row offset + chunk per q & 7
};

__device__ __forceinline__ DmaLane dma_lane(const GemmLaunch& p, int64_t ld, int t0, int wave, int lane) {
  DmaLane d;
  const int rsub = lane >> 3;
  const int chunk8 = ((lane & 7) ^ rsub) * 8;
  d.wo = (wave * 8 + rsub) * static_cast<int>(ld) + chunk8;
  const int last = p.M - 1 - t0;
#pragma unroll
  for (int q = 0; q < 8; ++q) d.xo[q] = min(q * 32 + wave * 8 + rsub, last) * static_cast<int>(ld) + chunk8;
  return d;
}

// DMA K-tile kt (of the 3K loop in SPLIT mode) of both operands into stage `st`
template <bool SPLIT>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ wt, const uint16_t* __restrict__ xt, int64_t K,
                                           int64_t ld, const DmaLane& d, int kt, char* st, int wave) {
  int64_t wcol = 0, xcol = 0;
  if constexpr (SPLIT) {
    const int KT0 = static_cast<int>(K / kBK);
    const int seg = kt >= 2 * KT0 ? 2 : (kt >= KT0 ? 1 : 0);
    kt -= seg * KT0;
    wcol = seg == 2 ? K : 0;
    xcol = seg == 1 ? K : 0;
  }
  const uint16_t* wk = wt + wcol + kt * kBK;
  const uint16_t* xk = xt + xcol + kt * kBK;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int rb = (q * 4 + wave) * 8;
    __builtin_amdgcn_global_load_lds(static_cast<const void*>(wk + (d.wo + q * 32 * static_cast<int>(ld))),
                                     (lds_void*)(st + rb * 128), 16, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int rb = (q * 4 + wave) * 8;
    __builtin_amdgcn_global_load_lds(static_cast<const void*>(xk + d.xo[q]), (lds_void*)(st + kOpBytes + rb * 128), 16,
                                     0, 0);
  }
}

// fragments of k-step s (0/1) of the stage: A = 8 feature row-groups, B = 8 token row-groups
__device__ __forceinline__ void read_frags(bf16x8 (&a)[8], bf16x8 (&b)[8], const char* st, int wr, int wc, int r16,
                                           int kq, int s) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = *reinterpret_cast<const bf16x8*>(st + swz(wr * 128 + i * 16 + r16, s * 4 + kq));
#pragma unroll
  for (int j = 0; j < 8; ++j)
    b[j] = *reinterpret_cast<const bf16x8*>(st + kOpBytes + swz(wc * 128 + j * 16 + r16, s * 4 + kq));
}

__device__ __forceinline__ void mfma_block(f32x4 (&acc)[8][8], const bf16x8 (&a)[8], const bf16x8 (&b)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// interleave hints: NDS fragment reads and NVM LDS-DMA instructions spread over the 64 MFMAs
// of a k-step (one wave per SIMD: the wave issues them in the MFMAs' shadow)
template <int NDS, int NVM>
__device__ __forceinline__ void interleave_hint() {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if constexpr (NVM > 0) __builtin_amdgcn_sched_group_barrier(0x020, NVM / 16, 0);  // VMEM read (LDS DMA)
    if constexpr (NDS > 0) __builtin_amdgcn_sched_group_barrier(0x100, NDS / 16, 0);  // DS read
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                // MFMA
  }
}

// One 64-deep K-tile t: k-step 0 from (a0, b0) while the k-step-1 fragments are read, the
// barrier that publishes stage t+1 and frees stage t, then k-step 1 from (a1, b1) while
// K-tile t+2 is DMA'd into the freed stage (DMA) and the k-step-0 fragments of t+1 are read
// (NEXT).  Branch-free body: the loop is peeled into <DMA, NEXT> = <1,1>* <0,1> <0,0>.
template <bool DMA, bool NEXT, bool SPLIT>
__device__ __forceinline__ void ktile(f32x4 (&acc)[8][8], bf16x8 (&a0)[8], bf16x8 (&b0)[8], bf16x8 (&a1)[8],
                                      bf16x8 (&b1)[8], char* cur, char* nxt, int t, const uint16_t* wt,
                                      const uint16_t* xt, int64_t K, int64_t ld, const DmaLane& dl, int wave, int wr,
                                      int wc, int r16, int kq) {
  read_frags(a1, b1, cur, wr, wc, r16, kq, 1);
  mfma_block(acc, a0, b0);
  interleave_hint<16, 0>();
  // stage t+1 landed (its DMA is the only one in flight) and every wave is done with stage t
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  barrier();
  if constexpr (DMA) stage_tile<SPLIT>(wt, xt, K, ld, dl, t + 2, cur, wave);
  if constexpr (NEXT) read_frags(a0, b0, nxt, wr, wc, r16, kq, 0);
  mfma_block(acc, a1, b1);
  interleave_hint<NEXT ? 16 : 0, DMA ? 16 : 0>();
}

template <int ACT, bool BIAS, bool RES, bool SPLIT, int OUT>
__global__ void __launch_bounds__(kThreads, 1) gemm4w_kernel(GemmLaunch p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = p.M, N = p.N, K = p.K;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  // ---- XCD-aware tile order (bijective for any grid size)
  const int tiles_f = N / kBF;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tt = lid / tiles_f, ft = lid - tt * tiles_f;
  const int f0 = ft * kBF, t0 = tt * kBT;
  const int KT = (SPLIT ? 3 : 1) * (K / kBK);
  AMD_DFT_DEV_CHECK(f0 + kBF <= N && t0 < M && (K / kBK) * kBK == K && KT > 0, "gemm4w_kernel");
  const int r16 = lane & 15, kq = lane >> 4;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[8], a1[8], b1[8];

  // ---- prologue: stages 0 and 1 in flight, wait for stage 0, fragments of k-step 0
  const int64_t ld = SPLIT ? 2 * static_cast<int64_t>(K) : K;
  const uint16_t* wt = p.w + static_cast<int64_t>(f0) * ld;
  const uint16_t* xt = p.x + static_cast<int64_t>(t0) * ld;
  const DmaLane dl = dma_lane(p, ld, t0, wave, lane);
  stage_tile<SPLIT>(wt, xt, K, ld, dl, 0, smem, wave);
  if (KT > 1) {
    stage_tile<SPLIT>(wt, xt, K, ld, dl, 1, smem + kStage, wave);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  read_frags(a0, b0, smem, wr, wc, r16, kq, 0);

  int t = 0;
  for (; t + 2 < KT; ++t)
    ktile<true, true, SPLIT>(acc, a0, b0, a1, b1, smem + (t & 1) * kStage, smem + ((t + 1) & 1) * kStage, t, wt, xt, K,
                             ld, dl, wave, wr, wc, r16, kq);
  if (t + 1 < KT) {
    ktile<false, true, SPLIT>(acc, a0, b0, a1, b1, smem + (t & 1) * kStage, smem + ((t + 1) & 1) * kStage, t, wt, xt,
                              K, ld, dl, wave, wr, wc, r16, kq);
    ++t;
  }
  ktile<false, false, SPLIT>(acc, a0, b0, a1, b1, smem + (t & 1) * kStage, smem + ((t + 1) & 1) * kStage, t, wt, xt, K,
                             ld, dl, wave, wr, wc, r16, kq);

  // ---- epilogue: lane holds features f..f+3 of token t for each (i, j) tile
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int f = f0 + wr * 128 + i * 16 + 4 * kq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (BIAS) {
      const float4 b4 = *reinterpret_cast<const float4*>(p.bias + f);
      bv[0] = b4.x;
      bv[1] = b4.y;
      bv[2] = b4.z;
      bv[3] = b4.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = t0 + wc * 128 + j * 16 + r16;
      if (t >= M) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[i][j][e] + bv[e];
        if constexpr (ACT == 1) v[e] = gelu_erf(v[e]);
      }
      const int64_t off = static_cast<int64_t>(t) * N + f;
      if constexpr (RES) {
        if constexpr (OUT == 1) {
          const float4 rr = *reinterpret_cast<const float4*>(static_cast<const float*>(p.residual) + off);
          v[0] += rr.x;
          v[1] += rr.y;
          v[2] += rr.z;
          v[3] += rr.w;
        } else {
          const uint2 rr = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p.residual) + off);
          v[0] += __uint_as_float(rr.x << 16);
          v[1] += __uint_as_float(rr.x & 0xffff0000u);
          v[2] += __uint_as_float(rr.y << 16);
          v[3] += __uint_as_float(rr.y & 0xffff0000u);
        }
      }
      if constexpr (OUT == 1) {
        *reinterpret_cast<float4*>(static_cast<float*>(p.y) + off) = make_float4(v[0], v[1], v[2], v[3]);
      } else if constexpr (OUT == 2) {
        float lo[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) lo[e] = v[e] - static_cast<float>(static_cast<__bf16>(v[e]));
        uint16_t* yr = static_cast<uint16_t*>(p.y) + static_cast<int64_t>(t) * (2 * N) + f;
        *reinterpret_cast<uint2*>(yr) = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
        *reinterpret_cast<uint2*>(yr + N) = make_uint2(pk_bf16(lo[0], lo[1]), pk_bf16(lo[2], lo[3]));
      } else {
        *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p.y) + off) = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
      }
    }
  }
}

template <int ACT, bool BIAS, bool RES, bool SPLIT, int OUT>
void launch4(const GemmLaunch& p, hipStream_t st, dim3 grid) {
  auto kern = gemm4w_kernel<ACT, BIAS, RES, SPLIT, OUT>;
  static bool attr_done = false;
  if (!attr_done) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: gemm4w attr: ") + hipGetErrorString(e));
    attr_done = true;
  }
  hipLaunchKernelGGL(kern, grid, dim3(kThreads), kLds, st, p);
}

template <int ACT, bool BIAS>
void dispatch_out(const GemmLaunch& p, hipStream_t st, dim3 grid) {
  const bool res = p.residual != nullptr;
  if (!p.split) {
    if (res) launch4<ACT, BIAS, true, false, 0>(p, st, grid);
    else launch4<ACT, BIAS, false, false, 0>(p, st, grid);
  } else if (p.out == 2) {
    launch4<ACT, BIAS, false, true, 2>(p, st, grid);
  } else if (res) {
    launch4<ACT, BIAS, true, true, 1>(p, st, grid);
  } else {
    launch4<ACT, BIAS, false, true, 1>(p, st, grid);
  }
}

}  // namespace

bool gemm4w_applicable(const GemmLaunch& p) {
  // bf16 operands only (the split rows use gemm.hip's k32-interleaved layout)
  return p.split == 0 && p.gC == 0 && p.sC == 0 && p.ln_stats == nullptr && p.N % kBF == 0 && p.K % kBK == 0 &&
         p.K >= kBK && p.M >= 1;
}

void launch_gemm4w(const GemmLaunch& p, void* stream) {
  if (!gemm4w_applicable(p)) throw std::runtime_error("amd_dft: gemm4w: unsupported GEMM configuration");
  const int64_t nwg = ((static_cast<int64_t>(p.M) + kBT - 1) / kBT) * (p.N / kBF);
  const dim3 grid(static_cast<uint32_t>(nwg));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool bias = p.bias != nullptr;
  if (p.act == 1) {
    if (bias) dispatch_out<1, true>(p, st, grid);
    else dispatch_out<1, false>(p, st, grid);
  } else {
    if (bias) dispatch_out<0, true>(p, st, grid);
    else dispatch_out<0, false>(p, st, grid);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: gemm4w launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
