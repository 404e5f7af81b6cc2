// Phase timeline of the bf16x3 MLP GEMMs at FourCastNet's shapes (diagnostic, standalone):
// includes csrc/nn/gemm.hip with AMD_DFT_GEMM_STAMPS and prints, per workgroup, the shader
// cycles of prologue / main loop / epilogue (median, p90, max) and how the workgroup start
// times cluster into rounds (s_memrealtime, 100 MHz), on random-ish operands.
//
//   hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -DAMD_DFT_GEMM_STAMPS \
//         -Icsrc bench/gemm_stamps.hip -o /tmp/gemm_stamps && /tmp/gemm_stamps
//   (-DGEMM_ABLATE=4: the epilogue computes everything but skips its stores; 1: no main-loop DMA, 2: no
//   main-loop fragment reads -- timing-only, profiles/gemm_mainloop_ablation_r3.txt)
#include "nn/gemm.hip"

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

__global__ void fill_stats(float* st, int64_t rows) {  // (mean, rstd) = (0.1, 1)
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < rows; i += 256LL * gridDim.x) {
    st[2 * i] = 0.1f;
    st[2 * i + 1] = 1.f;
  }
}

__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 256LL * gridDim.x) {
    uint32_t h = static_cast<uint32_t>(i) * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    const float v = (static_cast<float>(h & 0xffff) / 65536.f - 0.5f) * 0.1f;
    p[i] = static_cast<uint16_t>(__float_as_uint(v) >> 16);
  }
}

static double q(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[std::min<size_t>(v.size() - 1, static_cast<size_t>(p * v.size()))];
}

static void run(const char* name, amd_dft::GemmLaunch p, long long* dst) {
  using namespace amd_dft;
  const int64_t nwg = ((p.M + 255) / 256) * (p.N / 256);
  for (int i = 0; i < 3; ++i) launch_gemm(p, nullptr);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, nullptr));
  launch_gemm(p, nullptr);
  CK(hipEventRecord(e1, nullptr));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> st(nwg * 8);
  CK(hipMemcpy(st.data(), dst, sizeof(long long) * nwg * 8, hipMemcpyDeviceToHost));
  std::vector<double> pro, loop, epi, tot, start, dur;
  long long r0 = st[0];
  for (int64_t b = 0; b < nwg; ++b) r0 = std::min(r0, st[b * 8]);
  for (int64_t b = 0; b < nwg; ++b) {
    const long long* s = &st[b * 8];
    pro.push_back(static_cast<double>(s[2] - s[1]));
    loop.push_back(static_cast<double>(s[3] - s[2]));
    epi.push_back(static_cast<double>(s[4] - s[3]));
    tot.push_back(static_cast<double>(s[4] - s[1]));
    start.push_back((s[0] - r0) * 0.01);  // us
    dur.push_back((s[5] - s[0]) * 0.01);
  }
  const double clk = q(tot, 0.5) / (q(dur, 0.5) * 1e3);  // GHz
  std::printf("%s: %.1f us, %lld workgroups, clock ~%.2f GHz\n", name, ms * 1e3, static_cast<long long>(nwg), clk);
  std::printf("  prologue  cycles median %8.0f p90 %8.0f max %8.0f\n", q(pro, .5), q(pro, .9), q(pro, 1.));
  std::printf("  main loop cycles median %8.0f p90 %8.0f max %8.0f\n", q(loop, .5), q(loop, .9), q(loop, 1.));
  std::printf("  epilogue  cycles median %8.0f p90 %8.0f max %8.0f\n", q(epi, .5), q(epi, .9), q(epi, 1.));
  std::printf("  workgroup wall us median %7.2f p90 %7.2f max %7.2f\n", q(dur, .5), q(dur, .9), q(dur, 1.));
  // start-time histogram: how synchronized are the rounds?
  std::vector<double> s2 = start;
  std::sort(s2.begin(), s2.end());
  std::printf("  starts (us) of workgroups #0, 256, 512, 768, 1024, 2048, last: %.1f %.1f %.1f %.1f %.1f %.1f %.1f\n", s2[0],
              s2[std::min<size_t>(256, s2.size() - 1)], s2[std::min<size_t>(512, s2.size() - 1)],
              s2[std::min<size_t>(768, s2.size() - 1)], s2[std::min<size_t>(1024, s2.size() - 1)],
              s2[std::min<size_t>(2048, s2.size() - 1)], s2.back());
  // spread of starts within the second round (workgroups 256..511 by start order)
  if (s2.size() > 512) std::printf("  round-2 start spread: %.2f us\n", s2[511] - s2[256]);
}

int main() {
  using namespace amd_dft;
  const int M = 32 * 16200, C = 768, Hd = 3072;
  uint16_t *x, *w1, *w2, *h;
  float *b1, *res;
  long long* stamps;
  CK(hipMalloc(&x, sizeof(uint16_t) * M * 2 * C));
  CK(hipMalloc(&w1, sizeof(uint16_t) * Hd * 2 * C));
  CK(hipMalloc(&w2, sizeof(uint16_t) * C * 2 * Hd));
  CK(hipMalloc(&h, sizeof(uint16_t) * static_cast<size_t>(M) * 2 * Hd));
  CK(hipMalloc(&b1, sizeof(float) * Hd));
  CK(hipMalloc(&res, sizeof(float) * static_cast<size_t>(M) * C));
  CK(hipMalloc(&stamps, sizeof(long long) * 8 * 40000));
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, x, static_cast<int64_t>(M) * 2 * C, 1u);
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w1, static_cast<int64_t>(Hd) * 2 * C, 2u);
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w2, static_cast<int64_t>(C) * 2 * Hd, 3u);
  CK(hipMemset(b1, 0, sizeof(float) * Hd));
  CK(hipMemset(res, 0, sizeof(float) * static_cast<size_t>(M) * C));
  CK(hipDeviceSynchronize());
  GemmLaunch f1;
  f1.x = x;
  f1.w = w1;
  f1.bias = b1;
  f1.y = h;
  f1.M = M;
  f1.N = Hd;
  f1.K = C;
  f1.act = 1;
  f1.split = 1;
  f1.out = 2;
  f1.stamps = stamps;
  run("fc1 x3 + GELU (split out)", f1, stamps);
  GemmLaunch f2;
  f2.x = h;
  f2.w = w2;
  f2.residual = res;
  f2.y = res;
  f2.M = M;
  f2.N = C;
  f2.K = Hd;
  f2.split = 1;
  f2.out = 1;
  f2.stamps = stamps;
  run("fc2 x3 (+fp32 residual)", f2, stamps);
  // the fp32 block's forms: LayerNorm folded into fc1 (ln_stats / c1), fc2 + the next LN's partial statistics
  float *lnst = nullptr, *c1 = nullptr, *part = nullptr;
  CK(hipMalloc(&lnst, sizeof(float) * 2 * static_cast<size_t>(M)));
  CK(hipMalloc(&c1, sizeof(float) * Hd));
  CK(hipMalloc(&part, sizeof(float) * 2 * static_cast<size_t>(M) * (C / 64)));
  hipLaunchKernelGGL(fill_stats, dim3(1024), dim3(256), 0, 0, lnst, static_cast<int64_t>(M));
  CK(hipMemset(c1, 0, sizeof(float) * Hd));
  GemmLaunch f1l = f1;
  f1l.ln_stats = lnst;
  f1l.ln_c1 = c1;
  run("fc1 x3 + LN fold + GELU (split out)", f1l, stamps);
  GemmLaunch f2s = f2;
  f2s.stats_part = part;
  f2s.stats_pre = c1;  // zeros (the op layer passes zeros when there is no per-channel pre)
  run("fc2 x3 (+fp32 residual, LN partials)", f2s, stamps);
  // bf16 operands (the bf16 model's MLP): x rows [M, K], hidden [M, 4C] bf16, bf16 residual
  GemmLaunch g1;
  g1.x = x;
  g1.w = w1;
  g1.bias = b1;
  g1.y = h;
  g1.M = M;
  g1.N = Hd;
  g1.K = C;
  g1.act = 1;
  g1.stamps = stamps;
  run("fc1 bf16 + GELU", g1, stamps);
  GemmLaunch g1f = g1;  // the bf16 model's fc1: LayerNorm folded, fitted erf GELU (act 3)
  g1f.act = 3;
  g1f.ln_stats = lnst;
  g1f.ln_c1 = c1;
  run("fc1 bf16 + LN fold + GELU (erf fit)", g1f, stamps);
  GemmLaunch g1p = g1;  // plain: no bias, no activation (the hipBLASLt comparison shape)
  g1p.act = 0;
  g1p.bias = nullptr;
  run("fc1 bf16 plain", g1p, stamps);
  GemmLaunch g2;
  g2.x = h;
  g2.w = w2;
  g2.residual = x;
  g2.y = x;
  g2.M = M;
  g2.N = C;
  g2.K = Hd;
  g2.stamps = stamps;
  run("fc2 bf16 (+bf16 residual)", g2, stamps);
  return 0;
}
