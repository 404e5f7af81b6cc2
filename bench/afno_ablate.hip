// Timing ablations of the fused AFNO H-filter at FourCastNet's shape [32, 90, 46, 768]
// (standalone: includes the kernel source; zero data, timing only).  Build one binary per
// AFNO_ABLATE value (0 = full, 1 = no FFT butterflies, 2 = no GEMM MFMAs, 3 = neither):
//   hipcc -O1 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -Icsrc -DAFNO_ABLATE=1 \
//         bench/afno_ablate.hip -o /tmp/afno_ablate1
#include "spectral/afno_spectral.hip"

#include <cstdio>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

int main() {
  using namespace amd_dft;
  const int B = 32, H = 90, KM = 46, C = 768, NB = 8, BS = 96;
  const size_t n = static_cast<size_t>(B) * H * KM * C * 2;
  void *x, *y, *w1, *w2, *b1, *b2, *tw;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&w1, NB * 2 * BS * 4 * BS * 2));
  CK(hipMalloc(&w2, NB * 2 * BS * 4 * BS * 2));
  CK(hipMalloc(&b1, NB * 2 * BS * 4));
  CK(hipMalloc(&b2, NB * 2 * BS * 4));
  CK(hipMalloc(&tw, 4096 * 8));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMemset(w1, 0, NB * 2 * BS * 4 * BS * 2));
  CK(hipMemset(w2, 0, NB * 2 * BS * 4 * BS * 2));
  CK(hipMemset(b1, 0, NB * 2 * BS * 4));
  CK(hipMemset(b2, 0, NB * 2 * BS * 4));
  CK(hipMemset(tw, 0, 4096 * 8));
  for (int x3 = 0; x3 < 2; ++x3) {
    AfnoLaunch p;
    p.x = x;
    p.y = y;
    p.bf16_in = p.bf16_out = x3 ? 0 : 1;
    p.x3 = x3;
    p.w1t = static_cast<const uint16_t*>(w1);
    p.w2t = static_cast<const uint16_t*>(w2);
    p.b1 = static_cast<const float*>(b1);
    p.b2 = static_cast<const float*>(b2);
    p.tw = tw;
    p.r0 = 9;
    p.r1 = 10;
    p.B = B;
    p.H = H;
    p.KM = KM;
    p.C = C;
    p.NB = NB;
    p.lambda = 0.01f;
    for (int i = 0; i < 5; ++i) launch_afno_spectral(p, nullptr);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, nullptr));
    for (int i = 0; i < 20; ++i) launch_afno_spectral(p, nullptr);
    CK(hipEventRecord(e1, nullptr));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("AFNO_ABLATE=%d %s: %.1f us\n", AFNO_ABLATE, x3 ? "x3  " : "bf16", ms * 1000.f / 20);
  }
  return 0;
}
