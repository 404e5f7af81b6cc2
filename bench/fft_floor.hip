// Memory-path floors for the rfft2 720x1440 fp32 kernels (standalone, no torch):
// each probe is captured 50x into one hipGraph and timed per launch, so the numbers are
// directly comparable with bench/bench_fft.py's graph medians.
//
//   empty          one 64-thread workgroup doing nothing (launch-to-launch gap floor)
//   copy16         4.15 MB float4 copy, 256-thread workgroups (the "4 MB copy" bound)
//   row_io         the R2C row kernel's access pattern without the FFT: 360 workgroups x
//                  144 threads, rows 2c / 2c+1 read as 4-byte scalars (10 per row per thread),
//                  721 complex outputs per row written as 8-byte stores
//   row_io_v       same rows, 8 x 16-byte loads per thread (192 threads per pair of rows)
//   col_io T xcd   the column pass's pattern: T adjacent columns x 720 rows of complex
//                  (8-byte) elements per workgroup, in and out, XCD-aware tile order on/off
//   pair           copy16 followed by a dependent copy16 (two kernels per iteration)
//
// Build + run:  hipcc -O3 --offload-arch=gfx950 bench/fft_floor.hip -o /tmp/fft_floor && /tmp/fft_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

constexpr int H = 720, W = 1440, KW = W / 2 + 1;

__global__ void k_empty() {}

__global__ void k_copy16(const float4* __restrict__ a, float4* __restrict__ b, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}

// R2C row access pattern: workgroup c owns rows 2c, 2c+1
__global__ void __launch_bounds__(144) k_row_io(const float* __restrict__ x, float2* __restrict__ y) {
  const int c = blockIdx.x, t = threadIdx.x;
  const float* r0 = x + static_cast<size_t>(2 * c) * W;
  const float* r1 = r0 + W;
  float a[10], b[10];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    a[r] = r0[t + 144 * r];
    b[r] = r1[t + 144 * r];
  }
  float2* o0 = y + static_cast<size_t>(2 * c) * KW;
  float2* o1 = o0 + KW;
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    const int k = t + 144 * r;
    o0[k] = make_float2(a[2 * r], a[2 * r + 1]);
    o1[k] = make_float2(b[2 * r], b[2 * r + 1]);
  }
  if (t == 0) {
    o0[720] = make_float2(a[0], 0.f);
    o1[720] = make_float2(b[0], 0.f);
  }
}

// same rows, 16-byte loads: 1440 floats = 360 float4 per row, 2 rows = 720 float4 / 192 thr
__global__ void __launch_bounds__(192) k_row_io_v(const float* __restrict__ x, float2* __restrict__ y) {
  const int c = blockIdx.x, t = threadIdx.x;
  const float4* r0 = reinterpret_cast<const float4*>(x + static_cast<size_t>(2 * c) * W);
  float4 v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = t + 192 * r;
    v[r] = i < 720 ? r0[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float2* o = y + static_cast<size_t>(2 * c) * KW;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = t + 192 * r;
    if (i < 720) {
      const int row = i / 360, k = 2 * (i % 360);
      o[row * KW + k] = make_float2(v[r].x, v[r].y);
      o[row * KW + k + 1] = make_float2(v[r].z, v[r].w);
    }
  }
}

__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int per = nb >> 3, rem = nb & 7, xcd = b & 7, k = b >> 3;
  return (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + k;
}

// column access pattern: T columns x 720 rows per workgroup, TP = 90 threads per column
template <int T>
__global__ void __launch_bounds__(90 * T) k_col_io(const float2* __restrict__ x, float2* __restrict__ y, int xcd) {
  const int nb = gridDim.x;
  const int b = xcd ? xcd_block(blockIdx.x, nb) : static_cast<int>(blockIdx.x);
  const int t = threadIdx.x % T, tp = threadIdx.x / T;
  const int col = b * T + t;
  const int cc = col < KW ? col : KW - 1;
  float2 v[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = x[static_cast<size_t>(tp + 90 * r) * KW + cc];
#pragma unroll
  for (int r = 0; r < 8; ++r)
    if (col < KW) y[static_cast<size_t>(tp + 90 * r) * KW + col] = make_float2(v[r].y, v[r].x);
}

struct Probe {
  const char* name;
  std::function<void(hipStream_t)> launch;
};

float time_graph(const Probe& p, hipStream_t s, int iters) {
  for (int i = 0; i < 3; ++i) p.launch(s);
  CK(hipStreamSynchronize(s));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < iters; ++i) p.launch(s);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 7; ++rep) {
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms * 1000.f / iters);
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return best;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t nreal = static_cast<size_t>(H) * W, ncplx = static_cast<size_t>(H) * KW;
  float *x;
  float2 *y, *z;
  CK(hipMalloc(&x, nreal * 4));
  CK(hipMalloc(&y, ncplx * 8 + 64));
  CK(hipMalloc(&z, ncplx * 8 + 64));
  CK(hipMemset(x, 0, nreal * 4));
  CK(hipMemset(y, 0, ncplx * 8));
  const int n16 = static_cast<int>(ncplx * 8 / 16);
  std::vector<Probe> probes = {
      {"empty", [&](hipStream_t st) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st); }},
      {"copy16", [&](hipStream_t st) {
         hipLaunchKernelGGL(k_copy16, dim3((n16 + 255) / 256), dim3(256), 0, st, reinterpret_cast<const float4*>(y),
                            reinterpret_cast<float4*>(z), n16);
       }},
      {"pair(copy16,copy16)", [&](hipStream_t st) {
         hipLaunchKernelGGL(k_copy16, dim3((n16 + 255) / 256), dim3(256), 0, st, reinterpret_cast<const float4*>(y),
                            reinterpret_cast<float4*>(z), n16);
         hipLaunchKernelGGL(k_copy16, dim3((n16 + 255) / 256), dim3(256), 0, st, reinterpret_cast<const float4*>(z),
                            reinterpret_cast<float4*>(y), n16);
       }},
      {"row_io", [&](hipStream_t st) { hipLaunchKernelGGL(k_row_io, dim3(H / 2), dim3(144), 0, st, x, y); }},
      {"row_io_v", [&](hipStream_t st) { hipLaunchKernelGGL(k_row_io_v, dim3(H / 2), dim3(192), 0, st, x, y); }},
      {"col_io T=2 xcd=0", [&](hipStream_t st) { hipLaunchKernelGGL(k_col_io<2>, dim3((KW + 1) / 2), dim3(180), 0, st, y, z, 0); }},
      {"col_io T=2 xcd=1", [&](hipStream_t st) { hipLaunchKernelGGL(k_col_io<2>, dim3((KW + 1) / 2), dim3(180), 0, st, y, z, 1); }},
      {"col_io T=4 xcd=0", [&](hipStream_t st) { hipLaunchKernelGGL(k_col_io<4>, dim3((KW + 3) / 4), dim3(360), 0, st, y, z, 0); }},
      {"col_io T=4 xcd=1", [&](hipStream_t st) { hipLaunchKernelGGL(k_col_io<4>, dim3((KW + 3) / 4), dim3(360), 0, st, y, z, 1); }},
      {"col_io T=8 xcd=1", [&](hipStream_t st) { hipLaunchKernelGGL(k_col_io<8>, dim3((KW + 7) / 8), dim3(720), 0, st, y, z, 1); }},
      {"row_io+col_io4x", [&](hipStream_t st) {
         hipLaunchKernelGGL(k_row_io, dim3(H / 2), dim3(144), 0, st, x, y);
         hipLaunchKernelGGL(k_col_io<4>, dim3((KW + 3) / 4), dim3(360), 0, st, y, z, 1);
       }},
  };
  for (int round = 0; round < 2; ++round)
    for (const auto& p : probes) std::printf("%-24s %7.2f us\n", p.name, time_graph(p, s, 50));
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(z));
  return 0;
}
