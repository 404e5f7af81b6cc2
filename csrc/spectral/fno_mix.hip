// FNO spectral mode mixing on MFMA (K4 in SURVEY §2.5):
//   y[b, o, m] = sum_i x[b, i, m] * w[i, o, m]        (complex, per retained mode m)
// as a batch of small real-block GEMMs  [Xr | Xi] (B x 2Cin) . [[Wr, Wi], [-Wi, Wr]] (2Cin x 2Cout)
// on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation: the same numerics as an
// fp32 einsum).  A workgroup owns MT consecutive modes: x, w and y tiles are moved between HBM
// and LDS in 8*MT-byte contiguous runs per (b, i) / (i, o) / (b, o), and each wave runs the
// GEMMs of its modes straight out of LDS.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "spectral.h"

namespace amd_dft {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMT = 8;     // modes per workgroup
constexpr int kNT = 256;   // threads (4 waves)

__global__ void __launch_bounds__(kNT) fno_mix_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                      float* __restrict__ y, int B, int Cin, int Cout, int M) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = 2 * Cin, N = 2 * Cout;
  const int Kp = (K + 3) & ~3;             // k padded to the MFMA k-step
  const int Bp = (B + 15) & ~15, Np = (N + 15) & ~15;
  float* Xs = smem;                        // [kMT][Bp][Kp]
  float* Ws = Xs + kMT * Bp * Kp;          // [kMT][Kp][Np]
  float* Ys = Ws + kMT * Kp * Np;          // [kMT][Bp][Np]
  const int m0 = blockIdx.x * kMT;
  const int tid = threadIdx.x;
  // ---- zero-fill the padded tiles, then load (coalesced along the mode index)
  for (int i = tid; i < kMT * Bp * Kp; i += kNT) Xs[i] = 0.f;
  for (int i = tid; i < kMT * Kp * Np; i += kNT) Ws[i] = 0.f;
  __syncthreads();
  // x[b][i][m][2]: one thread per (b, i, mt, part)
  for (int idx = tid; idx < B * Cin * kMT * 2; idx += kNT) {
    const int part = idx & 1;
    const int mt = (idx >> 1) % kMT;
    const int bi = (idx >> 1) / kMT;
    const int i = bi % Cin, b = bi / Cin;
    const int m = m0 + mt;
    const float v = m < M ? x[(static_cast<int64_t>(bi) * M + m) * 2 + part] : 0.f;
    Xs[(mt * Bp + b) * Kp + part * Cin + i] = v;
  }
  // w[i][o][m][2] -> real block [[wr, wi], [-wi, wr]]
  for (int idx = tid; idx < Cin * Cout * kMT * 2; idx += kNT) {
    const int part = idx & 1;
    const int mt = (idx >> 1) % kMT;
    const int io = (idx >> 1) / kMT;
    const int o = io % Cout, i = io / Cout;
    const int m = m0 + mt;
    const float v = m < M ? w[(static_cast<int64_t>(io) * M + m) * 2 + part] : 0.f;
    float* Wm = Ws + mt * Kp * Np;
    if (part == 0) {
      Wm[i * Np + o] = v;                    // Wr
      Wm[(Cin + i) * Np + Cout + o] = v;     // Wr
    } else {
      Wm[i * Np + Cout + o] = v;             // Wi
      Wm[(Cin + i) * Np + o] = -v;           // -Wi
    }
  }
  __syncthreads();
  // ---- per-mode GEMMs on MFMA: wave wv handles modes wv, wv + 4, ...
  const int lane = tid & 63, wv = tid >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
  for (int mt = wv; mt < kMT; mt += kNT / 64) {
    const float* Xm = Xs + mt * Bp * Kp;
    const float* Wm = Ws + mt * Kp * Np;
    float* Ym = Ys + mt * Bp * Np;
    for (int mi = 0; mi < Bp / 16; ++mi)
      for (int ni = 0; ni < Np / 16; ++ni) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < Kp / 4; ++ks) {
          const float a = Xm[(mi * 16 + r16) * Kp + ks * 4 + kq];
          const float bv = Wm[(ks * 4 + kq) * Np + ni * 16 + r16];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) Ym[(mi * 16 + kq * 4 + i) * Np + ni * 16 + r16] = acc[i];
      }
  }
  __syncthreads();
  // ---- store y[b][o][m][2]
  for (int idx = tid; idx < B * Cout * kMT * 2; idx += kNT) {
    const int part = idx & 1;
    const int mt = (idx >> 1) % kMT;
    const int bo = (idx >> 1) / kMT;
    const int o = bo % Cout, b = bo / Cout;
    const int m = m0 + mt;
    if (m < M) y[(static_cast<int64_t>(bo) * M + m) * 2 + part] = Ys[(mt * Bp + b) * Np + part * Cout + o];
  }
}

// Small batch (B <= 8): the MFMA M dimension (batch) would be >= 50% padding and the op is
// a pure stream over the per-mode weights (Cin*Cout*M complex, 6.5 MB for 20x20x2048).  A
// workgroup owns 64 consecutive (o, m) outputs (coalesced along m); its 4 waves split the Cin
// sum (split-K, reduced through LDS) so a 20x2048-mode layer runs 2560 waves instead of 640 --
// with one wave per SIMD the per-thread chain of Cin dependent loads was the whole kernel time.
template <int NB>
__global__ void __launch_bounds__(256) fno_mix_small_kernel(const float2* __restrict__ x, const float2* __restrict__ w,
                                                            float2* __restrict__ y, int B, int Cin, int Cout, int M) {
  __shared__ float2 red[3][NB][64];
  const int lane = threadIdx.x & 63, s = threadIdx.x >> 6;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  const bool live = t < static_cast<int64_t>(Cout) * M;
  const int o = live ? static_cast<int>(t / M) : 0;
  const int mm = live ? static_cast<int>(t - static_cast<int64_t>(o) * M) : 0;
  float2 acc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = make_float2(0.f, 0.f);
  const int i0 = s * Cin / 4, i1 = (s + 1) * Cin / 4;
  if (live) {
#pragma unroll 8
    for (int i = i0; i < i1; ++i) {
      const float2 wv = w[(static_cast<int64_t>(i) * Cout + o) * M + mm];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if (b < B) {
          const float2 xv = x[(static_cast<int64_t>(b) * Cin + i) * M + mm];
          acc[b].x = fmaf(xv.x, wv.x, fmaf(-xv.y, wv.y, acc[b].x));
          acc[b].y = fmaf(xv.x, wv.y, fmaf(xv.y, wv.x, acc[b].y));
        }
      }
    }
  }
  if (s > 0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) red[s - 1][b][lane] = acc[b];
  }
  __syncthreads();
  if (s != 0 || !live) return;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b < B) {
      float2 v = acc[b];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        v.x += red[r][b][lane].x;
        v.y += red[r][b][lane].y;
      }
      y[(static_cast<int64_t>(b) * Cout + o) * M + mm] = v;
    }
  }
}

}  // namespace

void launch_fno_mix(const FnoMixLaunch& p, void* stream) {
  if (p.B <= 0 || p.M <= 0) return;
  if (p.B <= 8 && !p.mfma) {
    const int64_t n = static_cast<int64_t>(p.Cout) * p.M;
    const dim3 grid(static_cast<uint32_t>((n + 63) / 64));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const float2* xx = reinterpret_cast<const float2*>(p.x);
    const float2* ww = reinterpret_cast<const float2*>(p.w);
    float2* yy = reinterpret_cast<float2*>(p.y);
    if (p.B <= 1) hipLaunchKernelGGL(fno_mix_small_kernel<1>, grid, dim3(256), 0, st, xx, ww, yy, p.B, p.Cin, p.Cout, p.M);
    else if (p.B <= 2) hipLaunchKernelGGL(fno_mix_small_kernel<2>, grid, dim3(256), 0, st, xx, ww, yy, p.B, p.Cin, p.Cout, p.M);
    else if (p.B <= 4) hipLaunchKernelGGL(fno_mix_small_kernel<4>, grid, dim3(256), 0, st, xx, ww, yy, p.B, p.Cin, p.Cout, p.M);
    else hipLaunchKernelGGL(fno_mix_small_kernel<8>, grid, dim3(256), 0, st, xx, ww, yy, p.B, p.Cin, p.Cout, p.M);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: fno_mix launch: ") + hipGetErrorString(e));
    return;
  }
  const int K = 2 * p.Cin, N = 2 * p.Cout;
  const int Kp = (K + 3) & ~3, Bp = (p.B + 15) & ~15, Np = (N + 15) & ~15;
  const size_t lds = sizeof(float) * kMT * (static_cast<size_t>(Bp) * Kp + static_cast<size_t>(Kp) * Np +
                                            static_cast<size_t>(Bp) * Np);
  if (lds > 160 * 1024)
    throw std::runtime_error("amd_dft: fno_mix: batch/channels too large for the LDS tile (B*2Cin, 2Cin*2Cout)");
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fno_mix_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: fno_mix attr: ") + hipGetErrorString(e));
  }
  const dim3 grid((p.M + kMT - 1) / kMT);
  hipLaunchKernelGGL(fno_mix_kernel, grid, dim3(kNT), lds, static_cast<hipStream_t>(stream), p.x, p.w, p.y, p.B, p.Cin,
                     p.Cout, p.M);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: fno_mix launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
