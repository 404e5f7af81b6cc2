// Phase timeline of the fused bf16x3 AFNO H-filter (afno_spectral_x3_kernel) at FourCastNet's
// shape [32, 90, 46, 768], block size 96 (diagnostic, standalone): includes the kernel source with
// AFNO_STAMPS and prints the shader cycles of every phase (median / p90 over workgroups) and the
// workgroup start rounds (s_memrealtime, 100 MHz), on random data.
//
//   hipcc -O3 -mllvm -amdgpu-load-store-vectorizer=0 --offload-arch=gfx950 -munsafe-fp-atomics \
//         -fno-slp-vectorize -DAFNO_STAMPS -Icsrc bench/afno_stamps.hip -o /tmp/afno_stamps
#include "spectral/afno_spectral.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void fill_f32(float* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 256LL * gridDim.x) {
    uint32_t h = static_cast<uint32_t>(i) * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = (static_cast<float>(h & 0xffff) / 65536.f - 0.5f) * scale;
  }
}
__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 256LL * gridDim.x) {
    uint32_t h = static_cast<uint32_t>(i) * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = static_cast<uint16_t>(__float_as_uint((static_cast<float>(h & 0xffff) / 65536.f - 0.5f) * 0.1f) >> 16);
  }
}

static long long pct(std::vector<long long> v, double q) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, static_cast<size_t>(q * v.size()))];
}

int main() {
  using namespace amd_dft;
  const int B = 32, H = 90, KM = 46, C = 768, NB = 8, BS = 96;
  const int64_t n = static_cast<int64_t>(B) * H * KM * C * 2;
  const int64_t nw = static_cast<int64_t>(NB) * 2 * BS * 4 * BS;
  float *x, *y, *b1, *b2, *tw;
  uint16_t *w1, *w2;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&w1, nw * 2));
  CK(hipMalloc(&w2, nw * 2));
  CK(hipMalloc(&b1, NB * 2 * BS * 4));
  CK(hipMalloc(&b2, NB * 2 * BS * 4));
  CK(hipMalloc(&tw, 4096 * 8));
  fill_f32<<<1024, 256>>>(x, n, 1, 2.f);
  fill_bf16<<<1024, 256>>>(w1, nw, 2);
  fill_bf16<<<1024, 256>>>(w2, nw, 3);
  fill_f32<<<8, 256>>>(b1, NB * 2 * BS, 4, 0.1f);
  fill_f32<<<8, 256>>>(b2, NB * 2 * BS, 5, 0.1f);
  fill_f32<<<32, 256>>>(tw, 4096 * 2, 6, 2.f);
  const int64_t nblocks = static_cast<int64_t>(B) * KM * NB;
  long long* st;
  CK(hipMalloc(&st, nblocks * 16 * 8));
  CK(hipMemset(st, 0, nblocks * 16 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_afno_stamps), &st, sizeof(st)));
  AfnoLaunch p;
  p.x = x;
  p.y = y;
  p.bf16_in = p.bf16_out = 0;
  p.x3 = 1;
  p.w1t = w1;
  p.w2t = w2;
  p.b1 = b1;
  p.b2 = b2;
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
  launch_afno_spectral(p, nullptr);
  CK(hipEventRecord(e1, nullptr));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> h(nblocks * 16);
  CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  const char* names[] = {"", "", "pass0 (global load, DFT, LDS store)", "pass1 LDS gather", "pass1 DFT + split A",
                         "GEMM1 (x3)", "epilogue1 (ReLU, split)", "GEMM2 (x3)", "epilogue2 (softshrink)",
                         "ifft pass0 gather", "ifft pass0 DFT + LDS store", "", "ifft pass1 + global store"};
  long long tot = 0;
  std::vector<long long> wall;
  for (int64_t b = 0; b < nblocks; ++b) wall.push_back(h[b * 16 + 12] - h[b * 16 + 1]);
  std::printf("afno_spectral_x3 [32,90,46,768] bs96: %.1f us, %lld workgroups, workgroup cycles median %lld p90 %lld\n",
              ms * 1000.f, static_cast<long long>(nblocks), pct(wall, 0.5), pct(wall, 0.9));
  const int order[] = {2, 3, 4, 5, 6, 7, 8, 9, 10, 12};
  int prev = 1;
  for (int s : order) {
    std::vector<long long> d;
    for (int64_t b = 0; b < nblocks; ++b) d.push_back(h[b * 16 + s] - h[b * 16 + prev]);
    const long long m = pct(d, 0.5);
    tot += m;
    std::printf("  %-40s median %7lld p90 %7lld\n", names[s], m, pct(d, 0.9));
    prev = s;
  }
  std::vector<long long> starts;
  for (int64_t b = 0; b < nblocks; ++b) starts.push_back(h[b * 16 + 0]);
  std::sort(starts.begin(), starts.end());
  std::printf("  sum of medians %lld; starts (us) of workgroups #0, 512, 1024, 2048, last: %.1f %.1f %.1f %.1f %.1f\n", tot,
              0.0, (starts[512] - starts[0]) / 100.0, (starts[1024] - starts[0]) / 100.0,
              (starts[2048] - starts[0]) / 100.0, (starts.back() - starts[0]) / 100.0);
  return 0;
}
