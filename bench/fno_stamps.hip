// Phase clocks of the fused FNO layer tail (fno_c2r_pw_kernel) at BASELINE config 3 (20 channels,
// 720x1440, modes 32): per wave, the s_memtime cycles spent in setup, spectrum reloads, x staging +
// rotation, MFMAs and the epilogue, summed over its units (median / p90 over waves), bf16 and fp32,
// random operands and tables (timing only).
//
//   hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -DFNO_STAMPS -Icsrc \
//         bench/fno_stamps.hip -o /tmp/fno_stamps && /tmp/fno_stamps
#include "spectral/fno_c2r_pw.hip"

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

__global__ void fill_u16(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 256LL * gridDim.x) {
    uint32_t h = static_cast<uint32_t>(i) * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = static_cast<uint16_t>(__float_as_uint((static_cast<float>(h & 0xffff) / 65536.f - 0.5f)) >> 16);
  }
}
__global__ void fill_f32(float* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 256LL * gridDim.x) {
    uint32_t h = static_cast<uint32_t>(i) * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = (static_cast<float>(h & 0xffff) / 65536.f - 0.5f) * scale;
  }
}

static long long pct(std::vector<long long> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, static_cast<size_t>(q * v.size()))];
}

int main() {
  using namespace amd_dft;
  const int B = 1, C = 20, H = 720, W = 1440, m = 32;
  const int64_t nx = static_cast<int64_t>(B) * C * H * W;
  for (int bf = 1; bf >= 0; --bf) {
    const int es = bf ? 2 : 4;
    void *x, *y;
    float *yw, *wc, *bias, *rot;
    uint16_t* g0;
    CK(hipMalloc(&x, nx * es));
    CK(hipMalloc(&y, nx * es));
    CK(hipMalloc(&yw, static_cast<int64_t>(B) * C * H * m * 8));
    CK(hipMalloc(&wc, C * C * 4));
    CK(hipMalloc(&bias, C * 4));
    CK(hipMalloc(&g0, 1 << 20));
    CK(hipMalloc(&rot, kFnoRotMax * 8));
    if (bf) fill_u16<<<1024, 256>>>(static_cast<uint16_t*>(x), nx, 1);
    else fill_f32<<<1024, 256>>>(static_cast<float*>(x), nx, 1, 1.f);
    fill_f32<<<256, 256>>>(yw, static_cast<int64_t>(B) * C * H * m * 2, 2, 0.1f);
    fill_f32<<<1, 256>>>(wc, C * C, 3, 0.2f);
    fill_f32<<<1, 256>>>(bias, C, 4, 0.1f);
    fill_u16<<<64, 256>>>(g0, (1 << 20) / 2, 5);
    fill_f32<<<16, 256>>>(rot, kFnoRotMax * 2, 6, 2.f);
    long long* st;
    const int64_t slots = 8LL * 4 * 4096;
    CK(hipMalloc(&st, slots * 8));
    CK(hipMemset(st, 0, slots * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_fno_stamps), &st, sizeof(st)));
    for (int pw = 1; pw >= 0; --pw) {  // the FNO layer tail, then the SpectralConv2d tail (fno_c2r: no x)
    FnoC2RPwLaunch p;
    p.yw = yw;
    p.x = pw ? x : nullptr;
    p.wc = wc;
    p.bias = bias;
    p.y = y;
    p.g0 = g0;
    p.rot = rot;
    p.B = B;
    p.Cin = pw ? C : 0;
    p.Cout = C;
    p.H = H;
    p.W = W;
    p.m = m;
    p.bf16 = bf;
    p.gelu = pw;
    for (int i = 0; i < 5; ++i) launch_fno_c2r_pw(p, nullptr);
    CK(hipDeviceSynchronize());
    CK(hipMemset(st, 0, slots * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, nullptr));
    launch_fno_c2r_pw(p, nullptr);
    CK(hipEventRecord(e1, nullptr));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> h(slots);
    CK(hipMemcpy(h.data(), st, slots * 8, hipMemcpyDeviceToHost));
    std::vector<long long> ph[6], tot, starts;
    for (int64_t wv = 0; wv < slots / 8; ++wv) {
      const long long* r = &h[wv * 8];
      if (r[5] == 0) continue;
      long long t = 0;
      for (int i = 0; i < 6; ++i) ph[i].push_back(r[i]);
      for (int i = 0; i < 5; ++i) t += r[i];
      tot.push_back(t);
      starts.push_back(r[6]);
    }
    std::sort(starts.begin(), starts.end());
    std::printf("%s %s [1,20,720,1440] m32: %.1f us (one call), %zu waves, units/wave median %lld\n",
                pw ? "fno_c2r_pw" : "fno_c2r (no x)", bf ? "bf16" : "fp32", ms * 1000.f, tot.size(), pct(ph[5], 0.5));
    const char* names[] = {"setup (tables, weights, zero)", "spectrum reload (row change)", "x staging + rotate/split",
                           "MFMA", "epilogue (act + stores)"};
    for (int i = 0; i < 5; ++i) std::printf("  %-32s median %7lld p90 %7lld\n", names[i], pct(ph[i], 0.5), pct(ph[i], 0.9));
    std::printf("  wave total                       median %7lld p90 %7lld; wave start spread p90 %.2f us\n", pct(tot, 0.5),
                pct(tot, 0.9), starts.empty() ? 0.0 : (pct(starts, 0.9) - starts[0]) / 100.0);
    CK(hipMemset(st, 0, slots * 8));
    }
    CK(hipFree(x));
    CK(hipFree(y));
    CK(hipFree(yw));
    CK(hipFree(wc));
    CK(hipFree(bias));
    CK(hipFree(g0));
    CK(hipFree(rot));
    CK(hipFree(st));
  }
  return 0;
}
