// Phase timeline of the rfft2 720x1440 fixed-kernel passes (diagnostic, standalone):
// compiles fft_fixed_impl.h with AMD_DFT_FFT_STAMPS, launches the row R2C (TP=144) and the
// column C2C (TP=90, T=4, XCD order) kernels on zero data with a dummy twiddle table (timing
// only; results are not checked), and prints per-phase shader-clock durations over blocks
// (median / p90 / max) plus the dispatch skew (s_memrealtime, 100 MHz) of block starts / ends.
//
//   hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -DAMD_DFT_FFT_STAMPS \
//         -Icsrc bench/fft_stamps.hip -o /tmp/fft_stamps && /tmp/fft_stamps
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fft/fft_fixed_impl.h"

using namespace amd_dft;
using namespace amd_dft::fixed_detail;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

namespace {

void report(const char* name, const std::vector<long long>& st, int nb, int nphase) {
  auto q = [](std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v[std::min<size_t>(v.size() - 1, static_cast<size_t>(p * v.size()))];
  };
  std::printf("%s (%d blocks)\n", name, nb);
  // shader-clock phases: start(1) -> pass0(3) -> pass1(4) -> ... -> end(2)
  std::vector<int> order = {1};
  for (int p = 0; p < nphase; ++p) order.push_back(3 + p);
  order.push_back(2);
  for (size_t i = 1; i < order.size(); ++i) {
    std::vector<double> d;
    for (int b = 0; b < nb; ++b) d.push_back(static_cast<double>(st[b * 16 + order[i]] - st[b * 16 + order[i - 1]]));
    const char* lbl = i == 1 ? "load+pass0" : (i + 1 == order.size() ? "post/store" : "pass");
    std::printf("  %-11s %zu: cycles median %7.0f  p90 %7.0f  max %7.0f\n", lbl, i, q(d, 0.5), q(d, 0.9), q(d, 1.0));
  }
  std::vector<double> tot, s0, s1;
  long long r0 = st[0];
  for (int b = 0; b < nb; ++b) r0 = std::min(r0, st[b * 16 + 0]);
  for (int b = 0; b < nb; ++b) {
    tot.push_back(static_cast<double>(st[b * 16 + 2] - st[b * 16 + 1]));
    s0.push_back((st[b * 16 + 0] - r0) * 10.0);  // ns (100 MHz)
    s1.push_back((st[b * 16 + 8] - r0) * 10.0);
  }
  std::printf("  block total cycles median %7.0f max %7.0f | start skew ns: p50 %6.0f p90 %6.0f max %6.0f | "
              "end ns: p50 %6.0f max %6.0f\n",
              q(tot, 0.5), q(tot, 1.0), q(s0, 0.5), q(s0, 0.9), q(s0, 1.0), q(s1, 0.5), q(s1, 1.0));
}

}  // namespace

int main() {
  constexpr int H = 720, W = 1440, KW = W / 2 + 1;
  float* x;
  float2 *y, *z, *tw;
  long long* stamps;
  CK(hipMalloc(&x, sizeof(float) * H * W));
  CK(hipMalloc(&y, sizeof(float2) * H * KW));
  CK(hipMalloc(&z, sizeof(float2) * H * KW));
  CK(hipMalloc(&tw, sizeof(float2) * 8192));
  CK(hipMalloc(&stamps, sizeof(long long) * 16 * 4096));
  CK(hipMemset(x, 0, sizeof(float) * H * W));
  CK(hipMemset(y, 0, sizeof(float2) * H * KW));
  CK(hipMemset(tw, 0, sizeof(float2) * 8192));
  std::vector<long long> st(16 * 4096);

  FixedArgs a;
  std::memset(&a, 0, sizeof(a));
  a.tw = tw;
  a.scale = 1.f;
  a.stamps = stamps;
  // rows: 720 real rows of 1440 -> 360 paired complex FFTs, 721 modes per row
  {
    FixedArgs r = a;
    r.in = x;
    r.out = y;
    r.I = H;
    r.Si_in = W;
    r.Sn_in = 1;
    r.Si_out = 2 * KW;
    r.Sn_out = 2;
    r.out_lo = KW;
    r.in_lo = W;
    r.tiles_per_outer = H / 2;
    using Fr = FL<10, 12, 12>;
    for (int it = 0; it < 20; ++it)
      hipLaunchKernelGGL((fft_fixed_kernel<Kind::R2C, false, 144, 1, Fr, false, false, false, 0, false>), dim3(H / 2),
                         dim3(144), 0, 0, r);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), stamps, sizeof(long long) * 16 * (H / 2), hipMemcpyDeviceToHost));
    report("row R2C 1440 TP=144", st, H / 2, 3);
  }
  // columns: 721 complex columns of 720, 4 per block, XCD-aware order
  for (int xcd = 0; xcd < 2; ++xcd) {
    FixedArgs c = a;
    c.in = y;
    c.out = z;
    c.I = KW;
    c.Si_in = 2;
    c.Sn_in = 2 * KW;
    c.Si_out = 2;
    c.Sn_out = 2 * KW;
    c.in_lo = H;
    c.out_lo = H;
    c.tiles_per_outer = (KW + 3) / 4;
    c.xcd_nb = xcd ? c.tiles_per_outer : 0;
    using Fc = FL<8, 9, 10>;
    for (int it = 0; it < 20; ++it)
      hipLaunchKernelGGL((fft_fixed_kernel<Kind::C2C, true, 90, 4, Fc, false, false, false, 0, false>),
                         dim3(c.tiles_per_outer), dim3(360), 0, 0, c);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), stamps, sizeof(long long) * 16 * c.tiles_per_outer, hipMemcpyDeviceToHost));
    report(xcd ? "col C2C 720 TP=90 T=4 xcd" : "col C2C 720 TP=90 T=4", st, c.tiles_per_outer, 3);
  }
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(z));
  CK(hipFree(tw));
  CK(hipFree(stamps));
  return 0;
}
