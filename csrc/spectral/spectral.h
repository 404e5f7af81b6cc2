// Host interfaces of the fused spectral-layer kernels (no torch dependency).
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

namespace amd_dft {

// ---- AFNO: fused FFT_H -> block-diagonal complex MLP (MFMA) -> softshrink -> IFFT_H
struct AfnoLaunch {
  const void* x;        // [B, H, KM, C, 2] fp32/bf16 (W-direction half spectrum, KM kept modes)
  void* y;              // same shape (fp32/bf16)
  int bf16_in = 0, bf16_out = 0;
  int x3 = 0;           // fp32 bf16x3 variant: fp32 in/out, weights [NB][2*BS][hi 2*BS | lo 2*BS]
  const uint16_t* w1t;  // [NB][2*BS][2*BS] bf16, real-block weight transposed ([n][k])
  const uint16_t* w2t;
  const float* b1;      // [NB][2*BS] = [b_re | b_im]
  const float* b2;
  const void* tw;       // FFT plan twiddles for length H
  int r0 = 0, r1 = 0;   // the plan's radix order (must match the instance's two passes)
  int B, H, KM, C, NB;
  float lambda;
};
bool afno_spectral_supported(int H, int block_size);
std::vector<std::pair<int, int>> afno_spectral_shapes();  // instantiated (H, block size) pairs
int64_t afno_spectral_lds_bytes(int H, int block_size, bool x3);
void launch_afno_spectral(const AfnoLaunch& p, void* stream);

// ---- FNO: per-mode complex channel mixing out[b,o,m] = sum_i x[b,i,m] * w[i,o,m]
struct FnoMixLaunch {
  const float* x;   // [B, Cin, M, 2] fp32 (M = kept modes, flattened)
  const float* w;   // [Cin, Cout, M, 2] fp32
  float* y;         // [B, Cout, M, 2] fp32
  int B, Cin, Cout, M;
  int mfma = 0;     // 1: the batched MFMA kernel even for B <= 8 (weights read once per mode tile)
};
void launch_fno_mix(const FnoMixLaunch& p, void* stream);

// ---- FNO pointwise epilogue: y[b,o,p] = act(spec[b,o,p] + sum_i w[o,i] x[b,i,p] + bias[o])
struct FnoPointwiseLaunch {
  const void* spec;    // [B, Cout, P] (same dtype as x) or nullptr
  const void* x;       // [B, Cin, P]
  const float* w;      // [Cout, Cin] fp32
  const float* bias;   // [Cout] fp32 or nullptr
  void* y;             // [B, Cout, P]
  int B, Cin, Cout, P;
  int bf16 = 0, gelu = 1;
};
bool fno_pointwise_supported(int cin);
void launch_fno_pointwise(const FnoPointwiseLaunch& p, void* stream);

// ---- LayerNorm over the last dim (bf16/fp32 I/O, fp32 statistics)
struct LayerNormLaunch {
  const void* x;
  void* y;
  const void* gamma;
  const void* beta;
  const void* residual;  // optional: y = LN(x) ; x_out = x + residual written to resid_out
  void* resid_out;
  int64_t rows;
  int cols;
  float eps;
  int bf16;  // 1: bf16 tensors, 0: fp32 (gamma/beta fp32)
  int split_out = 0;           // fp32 only: y = [rows, 2 cols] bf16 pair rows [hi | lo]
  const float* pre = nullptr;  // fp32 only: per-channel addend applied before the statistics
};
void launch_layernorm(const LayerNormLaunch& p, void* stream);

// ---- AFNO W-direction transforms with LayerNorm fused into the IO (afno_wfft.hip)
struct AfnoWLaunch {
  const void* x = nullptr;        // [O, L, C] bf16 (fp32 if f32) stored residual stream
  const float* stats = nullptr;   // [O, L, 2] (mean, rstd) of x + pre
  const float* gamma = nullptr;   // [C] fp32
  const float* beta = nullptr;    // [C] fp32
  const float* pre = nullptr;     // [C] fp32 or nullptr
  const void* spec = nullptr;     // C2R input [O, KM, C, 2] bf16
  void* out = nullptr;            // R2C: [O, KM, C, 2] bf16; C2R: [O, L, C] bf16
  int O = 0, L = 0, C = 0, KM = 0;
  float scale = 1.f;
  int f32 = 0;                    // fp32 residual stream, spectrum and output
  // C2R, fp32 only: also the output's bf16x3 split-pair rows [O*L, 2C] (k32-interleaved, the
  // next GEMM's operand) and its per-64-channel LayerNorm partials [O*L, C/64] (mean, M2)
  uint16_t* pairs = nullptr;
  float* part = nullptr;
  // C2R SPLIT, optional: [O*L, C] bf16 third term of the split, bf16(out - m - (hi + lo)): with the pairs it
  // carries out to ~2^-27 of |out - m| (below fp32 rounding), so the fp32 copy (out) can be skipped
  uint16_t* lo2 = nullptr;
};
bool afno_w_supported(int L, int C, int KM);
void launch_afno_w_r2c_ln(const AfnoWLaunch& p, void* stream);
void launch_afno_w_c2r_ln(const AfnoWLaunch& p, void* stream);

// ---- LayerNorm statistics only: stats[r] = (mean, rstd) of x[r, :] + pre (bf16 rows)
struct LnStatsLaunch {
  const void* x;       // [rows, cols] bf16
  const float* pre;    // [cols] fp32 or nullptr
  float* stats;        // [rows, 2] fp32
  int64_t rows;
  int cols;
  float eps;
  int f32 = 0;         // x is fp32
};
void launch_ln_stats(const LnStatsLaunch& p, void* stream);
// [rows, nc, 2] per-chunk (mean, M2) partials of chunk width `width` -> [rows, 2] (mean, rstd)
void launch_ln_stats_merge(const float* part, float* stats, int64_t rows, int nc, int width, float eps, void* stream,
                           const float* shift = nullptr);

// ---- fp32 -> bf16 (hi, lo) split pairs for the bf16x3 GEMM: rows -> [rows, 2 cols] [hi | lo],
// else planes [2, n]
void launch_split_bf16(const float* x, uint16_t* y, int64_t n, int cols, bool rows, void* stream);

}  // namespace amd_dft
