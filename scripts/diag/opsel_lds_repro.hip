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

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// CO: 512-thread workgroups whose waves 0-3 run a dependent MFMA chain for the whole kernel while waves 4-7 (one per
// SIMD beside an MFMA wave) run the packed-multiply check -- the co-execution the AFNO kernels see when a co-resident
// workgroup is in its GEMM phase
template <int MODE, bool SEQ, bool CO, int FORM = 0>
__global__ void __launch_bounds__(512) repro(const float2* __restrict__ gtab, unsigned* __restrict__ bad, int lds_bytes,
                                             int iters) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int ct = CO ? tid - 256 : tid;  // checker thread index
  const int ntab = 81;
  float2* tab = reinterpret_cast<float2*>(smem + lds_bytes - ntab * 8);  // the table at the top, like the AFNO twl
  if (tid < ntab) tab[tid] = gtab[tid];
  // busy data below the table: every thread writes and later re-reads its own 16-byte slots
  float4* busy = reinterpret_cast<float4*>(smem);
  const int nbusy = (lds_bytes - ntab * 8) / 16;
  for (int i = tid; i < nbusy; i += 256) busy[i] = make_float4(i, -i, 0.5f * i, 1.f);
  __syncthreads();
  if constexpr (CO) {
    if (tid < 256) {  // MFMA waves
      bf16x8 x, y;
      for (int j = 0; j < 8; ++j) {
        x[j] = static_cast<__bf16>(0.001f * (tid + j));
        y[j] = static_cast<__bf16>(0.002f * (tid - j));
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int it = 0; it < iters * 24; ++it) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y, x, acc, 0, 0, 0);
      }
      if (acc[0] == 12345.f) atomicAdd(bad, 1u << 30);  // keep the chain live
      return;
    }
  }
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
      if constexpr (FORM != 0) {
        // single packed product next to the MFMA waves, in one of four forms (expected a * t.y for both lanes):
        //  1: v_pk_mul op_sel:[0,1]            (src1 high half -> both lanes; the failing AFNO form)
        //  2: v_pk_mul op_sel_hi:[1,0] on (t.y, t.y) copied by v_mov   (the shipped AFNO form)
        //  3: v_pk_mul op_sel:[1,0] op_sel_hi:[1,1] with the operands swapped (src0 high half -> both lanes)
        //  4: v_pk_fma op_sel:[0,1,0] with a zero addend   (src1 high half, FMA instead of MUL)
        if constexpr (FORM == 1) {
          asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1]" : "=v"(p) : "v"(a), "v"(t));
        } else if constexpr (FORM == 2) {
          f2v ty;
          asm volatile("v_mov_b32 %0, %1" : "=v"(ty.x) : "v"(t.y));
          ty.y = 0.f;
          asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(p) : "v"(a), "v"(ty));
        } else if constexpr (FORM == 3) {
          asm volatile("v_pk_mul_f32 %0, %2, %1 op_sel:[1,0]" : "=v"(p) : "v"(a), "v"(t));
        } else {
          const f2v z = {0.f, 0.f};
          asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0]" : "=v"(p) : "v"(a), "v"(t), "v"(z));
        }
        mism += (p.x != a.x * t.y || p.y != a.y * t.y) ? 1u : 0u;
      } else if constexpr (SEQ) {
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
  const int seqa = argc > 5 ? std::atoi(argv[5]) : 0;  // 0: single product, 1: full sequence, 2: + MFMA co-runner waves
  const bool seq = seqa != 0;
  // seq 11..14: MFMA co-runner waves + single product in form 1..4 (global-loaded table)
  auto k = seqa == 11 ? repro<1, false, true, 1> : seqa == 12 ? repro<1, false, true, 2>
         : seqa == 13 ? repro<1, false, true, 3> : seqa == 14 ? repro<1, false, true, 4>
         : seqa == 2 ? (mode == 1 ? repro<1, true, true> : (mode == 2 ? repro<2, true, true> : repro<0, true, true>))
           : seq ? (mode == 1 ? repro<1, true, false> : (mode == 2 ? repro<2, true, false> : repro<0, true, false>))
                 : (mode == 1 ? repro<1, false, false> : (mode == 2 ? repro<2, false, false> : repro<0, false, false>));
  const int nthr = seqa >= 2 ? 512 : 256;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(k, dim3(nwg), dim3(nthr), lds, 0, gt, bad, lds, iters);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  unsigned nb = 0;
  CK(hipMemcpy(&nb, bad, sizeof(unsigned), hipMemcpyDeviceToHost));
  const double total = 5.0 * nwg * 256.0 * iters * 9.0;
  std::printf("mode %d seq %d lds %d wgs %d iters %d: mismatches %u of %.0f packed products\n", mode, seq ? 1 : 0, lds, nwg, iters, nb, total);
  return 0;
}
