// Host interfaces of the DFT-as-GEMM kernels (pruned real transforms along the innermost axis)
// and their twiddle tables (built on the host in fp64, uploaded once, cached by the op layer).
#pragma once

#include <cstdint>
#include <vector>

namespace amd_dft {

constexpr int kDftGemmKB = 64;     // samples per phase block of the forward kernel
// output pixels per phase block of the inverse kernel (bf16 / fp32 I/O)
constexpr int kFnoChunkBF = 128;
constexpr int kFnoChunkF32 = 64;
// per-block phase / per-chunk rotation tables are LDS-resident (float2 entries)
constexpr int kDftwPhMax = 2048;
constexpr int kFnoRotMax = 2048;

// ---- forward: out[r, n] = scale * sum_k x[r, k] e^{-2 pi i n k / W},  n < m <= 64
struct DftwR2CLaunch {
  const void* x;      // [R, W] bf16 / fp32
  void* out;          // [R, m] complex fp32
  const void* b0;     // twiddle-block fragments (dftw_r2c_tables)
  const void* phase;  // [ceil(W/KB)][16G] float2
  int R, W, m;
  float scale = 1.f;
  int bf16 = 0;
};
// b0: uint16 bf16 bits, [kk][g][re/im][hi/lo][64 lanes][8];  phase: float (re, im) pairs
void dftw_r2c_tables(int W, int m, std::vector<uint16_t>& b0, std::vector<float>& phase);
// 1 <= m <= 64, W % 8 == 0 and the phase table (ceil(W/KB) x 16 ceil(m/16)) fits in LDS
bool dftw_r2c_supported(int W, int m);
void launch_dftw_r2c(const DftwR2CLaunch& p, void* stream);

// ---- FNO layer tail: inverse real DFT along W of the kept modes, fused with the pointwise path
//   y[b,o,h,w] = act( sum_{k<m} s_k Re(Y[b,o,h,k] e^{2 pi i k w / W}) + sum_i Wc[o,i] x[b,i,h,w] + bias[o] )
// (s_0 = 1, s_k = 2: the Hermitian half-spectrum C2R of torch.fft.irfft, Im Y[.,0] ignored)
struct FnoC2RPwLaunch {
  const void* yw;     // [B, Cout, H, m] complex fp32 (already carries the inverse-FFT scale)
  const void* x;      // [B, Cin, H, W] bf16 / fp32
  const float* wc;    // [Cout, Cin] fp32
  const float* bias;  // [Cout] or nullptr
  void* y;            // [B, Cout, H, W] (dtype of x)
  const void* g0;     // inverse twiddle-block fragments (fno_c2r_tables)
  const void* rot;    // [ceil(W/CHUNK)][16KS] float2
  int B, Cin, Cout, H, W, m;
  int bf16 = 0, gelu = 1;
};
// g0: uint16 bf16 bits, [ks][pt][hi/lo][64 lanes][8] (pt < chunk/16);  rot: [ceil(W/chunk)][16KS] (cos, sin)
void fno_c2r_tables(int W, int m, int chunk, std::vector<uint16_t>& g0, std::vector<float>& rot);
// Cin, Cout <= 32, m <= 64, W % 8 == 0 and the rotation table fits in LDS (W <= 4096 bf16 / 2048 fp32 at m = 64)
bool fno_c2r_pw_supported(int cin, int cout, int m, int W, bool bf16);
void launch_fno_c2r_pw(const FnoC2RPwLaunch& p, void* stream);

}  // namespace amd_dft
