// Host-side (fp64) twiddle tables for the DFT-as-GEMM kernels, laid out in MFMA fragment order
// so each lane fetches its operand with one 16-byte load.  Angles are reduced exactly in
// integers ((n*k) mod W) before the trig call, so large n*k lose no precision.
#include <cmath>
#include <cstring>

#include "dft_gemm.h"

namespace amd_dft {
namespace {

uint16_t bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return static_cast<uint16_t>(u >> 16);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}
float bf16_to_f(uint16_t h) {
  const uint32_t u = static_cast<uint32_t>(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
void split(double v, uint16_t& hi, uint16_t& lo) {
  hi = bf16_rne(static_cast<float>(v));
  lo = bf16_rne(static_cast<float>(v - static_cast<double>(bf16_to_f(hi))));
}
double angle(int64_t nk, int W) {
  const int64_t r = ((nk % W) + W) % W;
  return 2.0 * M_PI * static_cast<double>(r) / static_cast<double>(W);
}

}  // namespace

void dftw_r2c_tables(int W, int m, std::vector<uint16_t>& b0, std::vector<float>& phase) {
  const int G = (m + 15) / 16;
  const int NKS = kDftGemmKB / 32;
  b0.assign(static_cast<size_t>(NKS) * G * 2 * 2 * 64 * 8, 0);
  for (int kk = 0; kk < NKS; ++kk)
    for (int g = 0; g < G; ++g)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * kk + 8 * (lane >> 4) + j;
          const int n = 16 * g + (lane & 15);
          const double th = angle(static_cast<int64_t>(n) * k, W);
          const double v[2] = {std::cos(th), -std::sin(th)};
          for (int c = 0; c < 2; ++c) {
            uint16_t hi, lo;
            split(v[c], hi, lo);
            const size_t base = ((static_cast<size_t>((kk * G + g) * 2 + c) * 2) * 64 + lane) * 8 + j;
            b0[base] = hi;
            b0[base + 64 * 8] = lo;
          }
        }
  const int nblk = (W + kDftGemmKB - 1) / kDftGemmKB;
  phase.assign(static_cast<size_t>(nblk) * 16 * G * 2, 0.f);
  for (int s = 0; s < nblk; ++s)
    for (int n = 0; n < 16 * G; ++n) {
      const double th = angle(static_cast<int64_t>(n) * kDftGemmKB * s, W);
      phase[(static_cast<size_t>(s) * 16 * G + n) * 2] = static_cast<float>(std::cos(th));
      phase[(static_cast<size_t>(s) * 16 * G + n) * 2 + 1] = static_cast<float>(-std::sin(th));
    }
}

void fno_c2r_tables(int W, int m, int chunk, std::vector<uint16_t>& g0, std::vector<float>& rot) {
  const int KS = (m + 15) / 16;  // 16 complex modes (32 k-entries) per MFMA k-step
  const int PT = chunk / 16;
  g0.assign(static_cast<size_t>(KS) * PT * 2 * 64 * 8, 0);
  for (int ks = 0; ks < KS; ++ks)
    for (int pt = 0; pt < PT; ++pt)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          // A[m = px][k'] with k' = 2*mode + (re/im); lane holds k' = 32ks + 8(lane>>4) + j, px = 16pt + (lane&15)
          const int kp = 32 * ks + 8 * (lane >> 4) + j;
          const int mode = kp >> 1, c = kp & 1;
          const int px = 16 * pt + (lane & 15);
          double v = 0.0;
          if (mode < m) {
            const double s = (mode == 0 || 2 * mode == W) ? 1.0 : 2.0;
            const double th = angle(static_cast<int64_t>(mode) * px, W);
            v = c == 0 ? s * std::cos(th) : -s * std::sin(th);
          }
          uint16_t hi, lo;
          split(v, hi, lo);
          const size_t base = ((static_cast<size_t>(ks * PT + pt) * 2) * 64 + lane) * 8 + j;
          g0[base] = hi;
          g0[base + 64 * 8] = lo;
        }
  const int nch = (W + chunk - 1) / chunk;
  rot.assign(static_cast<size_t>(nch) * 16 * KS * 2, 0.f);
  for (int c = 0; c < nch; ++c)
    for (int k = 0; k < 16 * KS; ++k) {
      const double th = angle(static_cast<int64_t>(k) * chunk * c, W);
      rot[(static_cast<size_t>(c) * 16 * KS + k) * 2] = static_cast<float>(std::cos(th));
      rot[(static_cast<size_t>(c) * 16 * KS + k) * 2 + 1] = static_cast<float>(std::sin(th));
    }
}

}  // namespace amd_dft
