// Minimal-kernel attempt at the AFNO -O3 trigger (profiles/afno_o3_bisect_r3.txt): a VGPR pair loaded from LDS by
// ds_read_b64 (fully waited), then read by `v_pk_mul_f32 vD, vA, vB op_sel:[0,1]` (high half of src1 broadcast),
// with co-resident workgroups keeping the CU's LDS and VALU busy.  Every lane checks its products against the
// unpacked fp32 products of the same registers and counts mismatches.
//   hipcc -O3 --offload-arch=gfx950 scripts/diag/opsel_lds_repro.hip -o opsel_lds_repro && ./opsel_lds_repro
// Modes: 0 = table in LDS (ds_read_b64), 1 = the same table from global memory (global_load_dwordx2),
//        2 = LDS, but the pair read by ds_read2_b32.  Args: mode, dynamic LDS bytes, workgroups, iterations, seq
// (1 = the full packed complex multiply of the failing builds: two op_sel:[0,1] products, then the two packed FMAs).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

typedef float f2v __attribute__((ext_vector_type(2)));

template <int MODE, bool SEQ>
__global__ void __launch_bounds__(256) repro(const float2* __restrict__ gtab, unsigned* __restrict__ bad, int lds_bytes,
                                             int iters) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int ntab = 81;
  float2* tab = reinterpret_cast<float2*>(smem + lds_bytes - ntab * 8);  // the table at the top, like the AFNO twl
  if (tid < ntab) tab[tid] = gtab[tid];
  // busy data below the table: every thread writes and later re-reads its own 16-byte slots
  float4* busy = reinterpret_cast<float4*>(smem);
  const int nbusy = (lds_bytes - ntab * 8) / 16;
  for (int i = tid; i < nbusy; i += 256) busy[i] = make_float4(i, -i, 0.5f * i, 1.f);
  __syncthreads();
  unsigned mism = 0;
  f2v a = {1.0f + 0.001f * tid, -2.0f + 0.003f * tid};
  f2v b = {0.5f - 0.002f * tid, 1.5f + 0.001f * tid};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const int idx = r * 9 + (tid + it) % 9;
      f2v t;
      if constexpr (MODE == 1) {
        t = __builtin_bit_cast(f2v, gtab[idx]);
      } else {
        typedef __attribute__((address_space(3))) const float2 lds_f2;
        const unsigned addr = static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_f2*)(tab + idx)));
        if constexpr (MODE == 2)
          asm volatile("ds_read2_b32 %0, %1 offset1:1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(addr) : "memory");
        else
          asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(addr) : "memory");
      }
      f2v p;
      if constexpr (SEQ) {
        // the AFNO twiddle multiply exactly as the failing builds issue it: two op_sel:[0,1] products, then the two
        // packed FMAs that consume them (3 and 3 instructions later, no wait states in between)
        f2v q1, q2, re, im;
        asm volatile(
            "v_pk_mul_f32 %0, %4, %6 op_sel:[0,1]\n\t"
            "v_pk_mul_f32 %1, %5, %6 op_sel:[0,1]\n\t"
            "v_pk_mul_f32 %2, %5, %6 op_sel:[0,1]\n\t"
            "v_pk_fma_f32 %3, %5, %6, %0 op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[0,0,1]\n\t"
            "v_pk_fma_f32 %2, %4, %6, %1 op_sel_hi:[1,0,1]"
            : "=&v"(q1), "=&v"(q2), "=&v"(im), "=&v"(re)
            : "v"(b), "v"(a), "v"(t));
        (void)q2;
        const float r0 = fmaf(a.x, t.x, -(b.x * t.y)), r1 = fmaf(a.y, t.x, -(b.y * t.y));
        const float i0 = fmaf(b.x, t.x, a.x * t.y), i1 = fmaf(b.y, t.x, a.y * t.y);
        mism += (re.x != r0 || re.y != r1 || im.x != i0 || im.y != i1) ? 1u : 0u;
        p = re;
        b = f2v{b.x + 1e-6f * im.x, b.y - 1e-6f * im.y};
      } else {
        asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1]" : "=v"(p) : "v"(a), "v"(t));
        const float e0 = a.x * t.y, e1 = a.y * t.y;  // unpacked reference of the same registers
        mism += (p.x != e0 || p.y != e1) ? 1u : 0u;
      }
      a = f2v{a.x + 1e-6f * p.x, a.y - 1e-6f * p.y};
    }
    // LDS traffic between the rounds (as the FFT passes between two twiddle uses)
    const int i = (tid * 7 + it) % nbusy;
    float4 v = busy[i];
    v.w += 1.f;
    busy[i] = v;
  }
  if (mism) atomicAdd(bad, mism);
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int lds = argc > 2 ? std::atoi(argv[2]) : 77448;
  const int nwg = argc > 3 ? std::atoi(argv[3]) : 2944;
  const int iters = argc > 4 ? std::atoi(argv[4]) : 200;
  std::vector<float2> h(81);
  for (int i = 0; i < 81; ++i) h[i] = make_float2(0.5f + 0.01f * i, -0.25f + 0.02f * i);
  float2* gt;
  unsigned* bad;
  CK(hipMalloc(&gt, 81 * sizeof(float2)));
  CK(hipMalloc(&bad, sizeof(unsigned)));
  CK(hipMemcpy(gt, h.data(), 81 * sizeof(float2), hipMemcpyHostToDevice));
  CK(hipMemset(bad, 0, sizeof(unsigned)));
  const bool seq = argc > 5 && std::atoi(argv[5]) != 0;
  auto k = seq ? (mode == 1 ? repro<1, true> : (mode == 2 ? repro<2, true> : repro<0, true>))
               : (mode == 1 ? repro<1, false> : (mode == 2 ? repro<2, false> : repro<0, false>));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(k, dim3(nwg), dim3(256), lds, 0, gt, bad, lds, iters);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  unsigned nb = 0;
  CK(hipMemcpy(&nb, bad, sizeof(unsigned), hipMemcpyDeviceToHost));
  const double total = 5.0 * nwg * 256.0 * iters * 9.0;
  std::printf("mode %d seq %d lds %d wgs %d iters %d: mismatches %u of %.0f packed products\n", mode, seq ? 1 : 0, lds, nwg, iters, nb, total);
  return 0;
}
