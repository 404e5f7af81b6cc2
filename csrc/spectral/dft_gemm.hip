// Pruned real DFTs along the innermost axis as MFMA GEMMs (FNO path).
//
// When only the first m <= 64 of the W/2+1 half-spectrum modes are kept (FNO keeps 16-32 of
// 721), a Stockham FFT computes ~20x more outputs than are used and is bound by its LDS passes.
// A truncated DFT is a tall-skinny GEMM  X[r, n] = sum_k x[r, k] e^{-2 pi i n k / W}  that the
// matrix cores finish far below the HBM time of reading x once.  The twiddle operand would
// have to be re-read for every row tile (W x 2m complex, 368 KB for 1440 x 32 -- more L2
// traffic than x itself), so it is factored instead:
//   k = KB*s + k',   e^{-2 pi i n k/W} = e^{-2 pi i n KB s/W} * e^{-2 pi i n k'/W}
// The KB x 16G block B0[k'][n] (bf16 hi/lo split, so the twiddles are exact to ~2^-17) lives
// in registers for the whole kernel; each KB-block of x contributes  ph_s[n] * (x_s . B0)  with
// one complex scale of the MFMA accumulator per block and mode.
//
//   x:   [R, W] bf16 or fp32 rows (contiguous)     out: [R, m] complex fp32 (re, im)
//   A fragment (16x32 bf16): lane l holds x[row0 + (l&15)][k0 + 8(l>>4) + j], j < 8 -- one
//   16-byte load per lane straight from HBM (no LDS); fp32 input is split hi + lo on the fly.
// A workgroup (NW = 2..4 waves) owns 16 rows; the waves take interleaved KB-blocks (split-K) and
// are summed through LDS, so a 20x720-row FNO input still launches 900 workgroups.  NW is picked
// per launch so the whole grid is resident at once when possible: 900 4-wave workgroups at 3
// waves/SIMD are 1.17 rounds of 768 (the second round costs a full workgroup latency), 900
// 3-wave workgroups fit in one round of 1024 at 4/3 of the per-wave work.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "dft_gemm.h"

namespace amd_dft {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kNKS = kDftGemmKB / 32;  // 32-deep MFMA k-steps per block

#ifndef DFTW_B0_LDS
#define DFTW_B0_LDS 1  // twiddle block staged once per workgroup in LDS (0: every wave loads it from L2)
#endif

__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = static_cast<__bf16>(v[j]);
    hi[j] = h;
    lo[j] = static_cast<__bf16>(v[j] - static_cast<float>(h));
  }
}

template <bool BF, int G, int NW>
// waves_per_eu pins the register budget (3 waves up to 32 modes): without it the scheduler
// trades the batched prefetch for occupancy it cannot reach anyway (LDS, grid size).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(G <= 2 ? 3 : 5 - G, G <= 2 ? 3 : 5 - G)))
dftw_r2c_kernel(const void* __restrict__ x, float2* __restrict__ out,
                                                       const bf16x8* __restrict__ b0, const float2* __restrict__ ph,
                                                       int R, int W, int m, float scale, int nblk) {
  __shared__ f32x4 red[NW - 1][G][2][64];
  // block phases in LDS: read once per block and mode right before use, so an L2 round trip
  // there would sit on every block's critical path
  // (launch_dftw_r2c guarantees nblk * 16 G <= kDftwPhMax)
  __shared__ float2 phs[kDftwPhMax];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int row0 = blockIdx.x * 16;
  const int rowA = min(row0 + (lane & 15), R - 1);
  const int kq = 8 * (lane >> 4);
  // twiddle block, fragment order [kk][g][re/im][hi/lo][lane]
  constexpr int NB0 = kNKS * G * 4 * 64;
  bf16x8 bfr[kNKS][G][2][2];
#if DFTW_B0_LDS
  // copied once per workgroup through LDS: read by every wave straight from global, the same 16 KB
  // (G = 2) was fetched ~2700 times at kernel start (44 MB of L2 reads next to the 41.5 MB input)
  __shared__ bf16x8 b0s[NB0];
  constexpr int NBT = (NB0 + 64 * NW - 1) / (64 * NW);
  bf16x8 b0v[NBT];
#pragma unroll
  for (int q = 0; q < NBT; ++q) b0v[q] = b0[min(static_cast<int>(threadIdx.x) + 64 * NW * q, NB0 - 1)];
#else
#pragma unroll
  for (int kk = 0; kk < kNKS; ++kk)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int h = 0; h < 2; ++h) bfr[kk][g][c][h] = b0[(((kk * G + g) * 2 + c) * 2 + h) * 64 + lane];
#endif
  f32x4 are[G], aim[G];
#pragma unroll
  for (int g = 0; g < G; ++g) are[g] = aim[g] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A operand: one 16-byte (bf16) / two 16-byte (fp32) loads per lane and k-step.
  using Raw = u32x4;  // 8 bf16 / 4 fp32 (native vector: HIP's uint4/float4 structs copy badly)
  constexpr int NR = BF ? 1 : 2;
  const char* xrow = static_cast<const char*>(x) + static_cast<int64_t>(rowA) * W * (BF ? 2 : 4);
  // Loads are unconditional (clamped address); samples past W are zeroed where they are
  // consumed -- a select right after the load would make the compiler wait for it there and
  // serialise the prefetch batch.
  auto load = [&](int s, Raw (&r)[kNKS][NR]) {
#pragma unroll
    for (int kk = 0; kk < kNKS; ++kk) {
      const int k0 = s * kDftGemmKB + 32 * kk + kq;
      const bool ok = k0 < W;  // W % 8 == 0: a lane's 8 samples are all in or all out
      const Raw* p = reinterpret_cast<const Raw*>(xrow + static_cast<int64_t>(ok ? k0 : 0) * (BF ? 2 : 4));
#pragma unroll
      for (int t = 0; t < NR; ++t) r[kk][t] = p[t];
    }
  };
  // Batches of PF blocks per wave are loaded before any is consumed (4-6 KB per wave in
  // flight at 3 waves per SIMD).  Every block of a batch is consumed unconditionally (blocks
  // past nblk are clamped loads with zeroed data): a conditional consumer lets the compiler
  // sink each load down to its use, which serialises the batch into one round trip per block.
  // PF divides the per-wave block count of the 1440-wide FNO rows (8 at NW = 3, 6 at NW = 4).
#ifndef DFTW_PF_BF3
#define DFTW_PF_BF3 4  // bf16 blocks per batch at NW = 3 (8 = a wave's whole share of a 1440 row in one batch)
#endif
  constexpr int PF = G >= 4 ? 2 : BF ? (NW == 3 ? DFTW_PF_BF3 : 6) : 3;
  // The first batch is requested before the phase table is copied and the workgroup synchronises,
  // so the table's and the samples' global round trips overlap instead of following each other.
  Raw buf[PF][kNKS][NR];
#pragma unroll
  for (int j = 0; j < PF; ++j) load(min(wv + NW * j, nblk - 1), buf[j]);
  // the phase table: every entry's load issued before the first store (clamped, unconditional) --
  // a copy loop waits one L2 round trip per iteration (up to 4 for a 1440-wide row) behind the batch
  const int nph = nblk * 16 * G;
  constexpr int NPH = (kDftwPhMax + 64 * NW - 1) / (64 * NW);
  float2 phv[NPH];
#pragma unroll
  for (int q = 0; q < NPH; ++q) phv[q] = ph[min(static_cast<int>(threadIdx.x) + 64 * NW * q, nph - 1)];
#pragma unroll
  for (int q = 0; q < NPH; ++q) {
    const int t = static_cast<int>(threadIdx.x) + 64 * NW * q;
    if (t < nph) phs[t] = phv[q];
  }
#if DFTW_B0_LDS
#pragma unroll
  for (int q = 0; q < NBT; ++q) {
    const int t = static_cast<int>(threadIdx.x) + 64 * NW * q;
    if (t < NB0) b0s[t] = b0v[q];
  }
#endif
  __syncthreads();
#if DFTW_B0_LDS
#pragma unroll
  for (int kk = 0; kk < kNKS; ++kk)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int h = 0; h < 2; ++h) bfr[kk][g][c][h] = b0s[(((kk * G + g) * 2 + c) * 2 + h) * 64 + lane];
#endif
  for (int s0 = wv; s0 < nblk; s0 += NW * PF) {
    if (s0 != wv) {
#pragma unroll
      for (int j = 0; j < PF; ++j) load(min(s0 + NW * j, nblk - 1), buf[j]);
    }
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const bool live = s0 + NW * j < nblk;
      const int s = live ? s0 + NW * j : nblk - 1;
      f32x4 tr[G], ti[G];
#pragma unroll
      for (int g = 0; g < G; ++g) tr[g] = ti[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < kNKS; ++kk) {
        const bool ok = live && s * kDftGemmKB + 32 * kk + kq < W;
        if (!ok)
#pragma unroll
          for (int t = 0; t < NR; ++t) buf[j][kk][t] = Raw{};
        if constexpr (BF) {
          const bf16x8 a = __builtin_bit_cast(bf16x8, buf[j][kk][0]);
#pragma unroll
          for (int g = 0; g < G; ++g) {
            tr[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[kk][g][0][0], tr[g], 0, 0, 0);
            tr[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[kk][g][0][1], tr[g], 0, 0, 0);
            ti[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[kk][g][1][0], ti[g], 0, 0, 0);
            ti[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[kk][g][1][1], ti[g], 0, 0, 0);
          }
        } else {
          const f32x4 f0 = __builtin_bit_cast(f32x4, buf[j][kk][0]), f1 = __builtin_bit_cast(f32x4, buf[j][kk][NR - 1]);
          const float v[8] = {f0[0], f0[1], f0[2], f0[3], f1[0], f1[1], f1[2], f1[3]};
          bf16x8 ah, al;
          split8(v, ah, al);
#pragma unroll
          for (int g = 0; g < G; ++g) {
            tr[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bfr[kk][g][0][0], tr[g], 0, 0, 0);
            tr[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bfr[kk][g][0][1], tr[g], 0, 0, 0);
            tr[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bfr[kk][g][0][0], tr[g], 0, 0, 0);
            ti[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bfr[kk][g][1][0], ti[g], 0, 0, 0);
            ti[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bfr[kk][g][1][1], ti[g], 0, 0, 0);
            ti[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bfr[kk][g][1][0], ti[g], 0, 0, 0);
          }
        }
      }
      // block phase e^{-2 pi i n KB s / W}: one complex scale per accumulator column (mode n)
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float2 p = phs[s * 16 * G + 16 * g + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          are[g][i] = fmaf(p.x, tr[g][i], fmaf(-p.y, ti[g][i], are[g][i]));
          aim[g][i] = fmaf(p.x, ti[g][i], fmaf(p.y, tr[g][i], aim[g][i]));
        }
      }
    }
  }
  // split-K reduction of the NW waves
  if (wv > 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      red[wv - 1][g][0][lane] = are[g];
      red[wv - 1][g][1][lane] = aim[g];
    }
  }
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int w = 0; w < NW - 1; ++w)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      are[g] += red[w][g][0][lane];
      aim[g] += red[w][g][1][lane];
    }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int n = 16 * g + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + 4 * (lane >> 4) + i;
      if (row < R && n < m)
        out[static_cast<int64_t>(row) * m + n] = make_float2(are[g][i] * scale, aim[g][i] * scale);
    }
  }
}

// resident workgroups of one instance on the current device (occupancy x CUs), cached per device
template <bool BF, int G, int NW>
int64_t resident_wgs() {
  static int64_t cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] == 0) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const auto kern = reinterpret_cast<const void*>(&dftw_r2c_kernel<BF, G, NW>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * NW, 0) != hipSuccess || per_cu <= 0)
      per_cu = 1;
    cache[dev] = static_cast<int64_t>(cus) * per_cu;
  }
  return cache[dev];
}

template <bool BF, int G>
void launch_nw(const DftwR2CLaunch& p, hipStream_t st) {
  const int64_t groups = (p.R + 15) / 16;
  const int nblk = (p.W + kDftGemmKB - 1) / kDftGemmKB;
  // cost ~ rounds of workgroups x blocks per wave; ties go to more waves (more loads in flight)
  const int64_t r4 = resident_wgs<BF, G, 4>(), r3 = resident_wgs<BF, G, 3>();
  const int64_t c4 = (groups + r4 - 1) / r4 * ((nblk + 3) / 4), c3 = (groups + r3 - 1) / r3 * ((nblk + 2) / 3);
  const int nw = c3 < c4 ? 3 : 4;
  const dim3 grid(static_cast<uint32_t>(groups));
  const bf16x8* b0 = static_cast<const bf16x8*>(p.b0);
  float2* out = static_cast<float2*>(p.out);
  const float2* ph = static_cast<const float2*>(p.phase);
#define L_(NW_)                                                                                                  \
  hipLaunchKernelGGL((dftw_r2c_kernel<BF, G, NW_>), grid, dim3(64 * NW_), 0, st, p.x, out, b0, ph, p.R, p.W, p.m, \
                     p.scale, nblk)
  if (nw == 3) L_(3);
  else L_(4);
#undef L_
}

template <bool BF>
void launch_g(const DftwR2CLaunch& p, hipStream_t st) {
  switch ((p.m + 15) / 16) {
    case 1: launch_nw<BF, 1>(p, st); break;
    case 2: launch_nw<BF, 2>(p, st); break;
    case 3: launch_nw<BF, 3>(p, st); break;
    case 4: launch_nw<BF, 4>(p, st); break;
    default: throw std::runtime_error("amd_dft: dftw_r2c: m must be in [1, 64]");
  }
}

}  // namespace

bool dftw_r2c_supported(int W, int m) {
  if (m < 1 || m > 64 || W % 8 != 0 || W < 8) return false;
  return static_cast<int64_t>((W + kDftGemmKB - 1) / kDftGemmKB) * 16 * ((m + 15) / 16) <= kDftwPhMax;
}

void launch_dftw_r2c(const DftwR2CLaunch& p, void* stream) {
  if (p.R == 0) return;
  if (!dftw_r2c_supported(p.W, p.m))
    throw std::runtime_error("amd_dft: dftw_r2c needs 1 <= m <= 64, W % 8 == 0 and W <= 8192 (m = 64)");
  if (static_cast<int64_t>(p.R) * p.W >= (int64_t(1) << 31))
    throw std::runtime_error("amd_dft: dftw_r2c: tensor too large for 32-bit row offsets");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (p.bf16) launch_g<true>(p, st);
  else launch_g<false>(p, st);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: dftw_r2c launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
