// Fused AFNO spectral filter along H (FourCastNet AFNO2D, K5 in SURVEY §2.5).
//
// History (profiles/afno_o1_fix_r2.txt, profiles/afno_o3_bisect_r3.txt): with the AMDGPU load/store
// vectorizer on, both kernels of this file used to return slightly wrong values (bf16x3 rel-L2 ~6e-3
// instead of 6.2e-6), differently from launch to launch, only when two or more workgroups shared a
// CU; rounds 2-3 built the file with the vectorizer off.
// Root cause (round 3): a packed-FP32 misbehaviour observed on this toolchain and pool (ROCm 7.2.0,
// AMD clang 22 / LLVM from /opt/rocm/lib/llvm, gfx950 MI355X boxes), not a race in this source.
// Whether it is a hardware erratum or a hazard the compiler's hazard recognizer should pad (wait
// states between MFMA co-runners and op_sel'd packed-FP32 reads) is not established -- only that
// the form below fails there and the avoided form does not.  With the vectorizer
// on, the pass-1 twiddle multiply was issued as `v_pk_mul_f32 vD, vA, vB op_sel:[0,1]` -- the high
// half of the twiddle pair broadcast through src1's op_sel.  Packed-FP32 ops that select src1's high
// half through op_sel (v_pk_mul_f32 and v_pk_fma_f32 alike) return wrong products while another wave
// on the same SIMD executes MFMAs: scripts/diag/opsel_lds_repro.hip, a minimal kernel whose waves 0-3
// run an MFMA chain while waves 4-7 check packed products against unpacked ones, sees 7.7 % of the
// products wrong (0 without the MFMA waves; 0 with op_sel on src0, or with the operand first copied
// to its own register).  Here the MFMA co-runner was the co-resident workgroup's GEMM phase -- hence
// 'only when two or more workgroups share a CU'.  The vectorizer-off bisection builds agree (the
// single change 'twiddle consumed through op_sel:[0,1]' fails with either LDS load form, after a full
// s_waitcnt plus 16 wait states; unpacked FMAs on the same loaded values are exact).
// Fix, at the source: radix.h's c_mul(cpair, float2) routes the twiddle's imaginary part through its
// own register, so no kernel issues the form (0 of 893 kernels); with it the vectorizer-on build is
// exact and deterministic at every grid of the race screen and 4 % faster for bf16x3 (754 vs 786 us
// at [32, 90, 46, 768]), so this file builds with the default flags again.  Guards:
// tests/test_codegen.py (CPU tier) fails if any kernel of the built library issues the form
// (scripts/diag/scan_so.py) and checks this file with the vectorizer on; the determinism screen
// (tests/test_determinism_gpu.py) runs every kernel family at co-resident grids.
//
// One workgroup owns one (batch b, W-mode kw, channel block k) tile: X[h][c], h < H,
// c < BS (block size), complex, produced by the W-direction R2C pass.  In one launch it runs
//   FFT_H (two-pass Stockham [R0, R1] = the plan order of H, register first pass)  ->
//   O1 = ReLU([Xr|Xi] . W1' + b1')  (bf16 MFMA 16x16x32, fp32 accumulate)  ->
//   O2 = O1 . W2' + b2'  -> softshrink(lambda)  ->
//   IFFT_H (register last pass, stored straight to global)
// where W' = [[W0, W1], [-W1, W0]] is the real 2BS x 2BS form of the complex BS x BS block
// weight (pre-packed transposed, [n][k], so a lane's B fragment is 16 contiguous bytes).
// Everything between the global load and the global store stays in LDS (fp16 FFT staging
// aliased with the bf16 GEMM tile: 38 KB at H = 90, BS = 96, 3 workgroups / CU) and in
// registers; the reference FourCastNet path is ~10 separate kernels with 4 spectrum round
// trips through HBM.
//
// Instances (AFNO_SHAPES below): H in {45 = 9x5, 64 = 16x4, 90 = 9x10} (FourCastNet at patch
// 16 / square 512-pixel grids / patch 8) x block size in {48, 64, 96, 128} (48: embed 384 at 8
// blocks).  The GEMMs are [16 MT x 2BS] = A . W' with MT = ceil(H / 16) row tiles (rows >= H are
// padding whose outputs are discarded) and 2BS / 16 column tiles over the 4 waves (BS = 48: 6 tiles,
// the fourth wave's slots repeat the last tile and store nothing).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../fft/dev_check.h"
#include "../fft/radix.h"
#include "spectral.h"

namespace amd_dft {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kNT = 256;  // threads
#ifndef AFNO_BPF
#define AFNO_BPF 2  // k-steps of B-fragment prefetch in the block-MLP GEMMs
#endif
#ifndef AFNO_BPF3
#define AFNO_BPF3 2  // k-steps of B-fragment prefetch in the bf16x3 block-MLP GEMMs
#endif
#ifdef AFNO_STAMPS
// phase clocks (bench/afno_stamps.hip): thread 0 of each workgroup records s_memtime after every
// phase barrier of the bf16x3 kernel (slot 0 / 11: s_memrealtime at entry / exit, 12: s_memtime at exit; 16 per workgroup)
__device__ long long* g_afno_stamps;
#define AFNO_STAMP(slot, v) \
  do { if (threadIdx.x == 0) g_afno_stamps[static_cast<int64_t>(blockIdx.x) * 16 + (slot)] = static_cast<long long>(v); } while (0)
#else
#define AFNO_STAMP(slot, v) do { } while (0)
#endif

// Compile-time geometry of one instance: H = L = R0 x R1, block size BS.
template <int L_, int R0_, int R1_, int BS_>
struct AfnoShape {
  static constexpr int L = L_, R0 = R0_, R1 = R1_, BS = BS_;
  static constexpr int NP = BS / 2;       // channel pairs per row
  static constexpr int K = 2 * BS;        // real-block GEMM K = N
  static constexpr int APitch = K + 8;    // bf16 elements per A row (+16 B: ds_read_b128 spread)
  static constexpr int MT = (L + 15) / 16;  // GEMM row tiles (rows >= L are padding)
  static constexpr int NCT = BS / 8;      // 16-wide column tiles of the 2BS-wide GEMM output
  static constexpr int NTW = (NCT + 3) / 4;  // column tiles per wave (4 waves)
  static constexpr bool CT_EXACT = NCT % 4 == 0;  // BS % 32 == 0: every wave owns NTW real tiles
  // column tile of (wave w, slot nj); BS % 32 != 0 (e.g. 48): the last wave's extra slots repeat the
  // last tile (their MFMAs are discarded, their stores skipped: ct_live)
  __device__ static constexpr int ct(int w, int nj) { return CT_EXACT ? NTW * w + nj : min(NTW * w + nj, NCT - 1); }
  __device__ static constexpr bool ct_live(int w, int nj) { return CT_EXACT || NTW * w + nj < NCT; }
  static constexpr int KS = BS / 16;      // 32-deep k-steps
  static constexpr int OCC = BS <= 96 ? 3 : 2;  // workgroups per SIMD the bf16 register budget targets
  // dynamic LDS: the FFT staging / GEMM A tile(s) (bf16 kernel: fp16 staging | one bf16 plane;
  // x3: fp32 staging | hi + lo planes), then the pass-1 twiddles (TWN float2, copied from the plan
  // table at kernel start: an LDS read instead of an L2 round trip after each pass-1 barrier)
  static constexpr int TWN = (R1 - 1) * R0;
  // row pitch (complex elements) of the GEMM-2 output staging X: the epilogue writes 4 consecutive
  // values (two channels' re, im) of one row per lane, 16 lanes on 16 rows, so the pitch is padded
  // off a multiple of the bank row (fp16 rows shift by 2 banks, fp32 rows by 4: conflict-free)
  static constexpr int XP = BS + 2;
  static constexpr int64_t cmax(int64_t a, int64_t b) { return a > b ? a : b; }
  static constexpr int64_t MAIN16 = cmax(cmax(L * BS * 4, L * XP * 4), 32 * MT * APitch);
  static constexpr int64_t MAIN32 = cmax(cmax(2 * L * BS * 4, 2 * L * XP * 4), 64 * MT * APitch);
  static constexpr int64_t LDS16 = MAIN16 + TWN * 8, LDS32 = MAIN32 + TWN * 8;
  static constexpr int64_t LDS16X2 = 2 * MAIN16 + TWN * 8;  // two-tile bf16 kernel: one region per tile
  // the two-tile kernel where two of its workgroups share a CU and its 2 MT x NTW accumulators fit
  // beside the FFT registers without spilling (BS <= 96)
  static constexpr bool TPW2 = BS <= 96 && 2 * LDS16X2 <= 160 * 1024;
  static_assert(MAIN16 % 16 == 0, "tile regions 16-byte aligned");
  static_assert(R0 * R1 == L && BS % 16 == 0 && L <= 128, "AFNO instance geometry");
};

__device__ __forceinline__ uint16_t f2bf16(float f) { return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f)); }

// FFT staging in LDS as fp16 complex (half the bytes of fp32: 3 workgroups per CU instead of
// 2).  fp16 keeps 11 significant bits (the GEMM operands downstream are bf16, 8 bits); the
// spectra of the AFNO filter stay orders of magnitude inside fp16 range.
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
// two adjacent channels' complex values (fp16 LDS staging)
__device__ __forceinline__ void st_hp(h2_t* p, int i, const cpair& v) {
  *reinterpret_cast<h4_t*>(p + i) = h4_t{static_cast<_Float16>(v.re[0]), static_cast<_Float16>(v.im[0]),
                                        static_cast<_Float16>(v.re[1]), static_cast<_Float16>(v.im[1])};
}
__device__ __forceinline__ cpair ld_hp(const h2_t* p, int i) {
  const h4_t h = *reinterpret_cast<const h4_t*>(p + i);
  return cpair{f2v{static_cast<float>(h[0]), static_cast<float>(h[2])}, f2v{static_cast<float>(h[1]), static_cast<float>(h[3])}};
}
// two adjacent channels' complex values in global memory (off in scalars)
template <bool BF>
__device__ __forceinline__ void ldc2(const void* p, int off, float2& a, float2& b) {
  if constexpr (BF) {
    const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + off);
    a = make_float2(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u));
    b = make_float2(__uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  } else {
    const float4 f = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + off);
    a = make_float2(f.x, f.y);
    b = make_float2(f.z, f.w);
  }
}
template <bool BF>
__device__ __forceinline__ void stc2(void* p, int off, float2 a, float2 b) {
  if constexpr (BF) {
    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p) + off) =
        make_uint2(static_cast<uint32_t>(f2bf16(a.x)) | (static_cast<uint32_t>(f2bf16(a.y)) << 16),
                   static_cast<uint32_t>(f2bf16(b.x)) | (static_cast<uint32_t>(f2bf16(b.y)) << 16));
  } else {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + off) = make_float4(a.x, a.y, b.x, b.y);
  }
}

// Stockham pass over BS interleaved signals in LDS (layout [n][BS]) with register staging:
// gather -> barrier -> twiddle/DFT -> scatter.  A work item is one butterfly of a PAIR of
// adjacent channels (8-byte global / LDS accesses, twiddles shared by the pair), held as a
// cpair (radix.h) so every butterfly op is one packed fp32 instruction for both channels.
template <int R, int L, int NP>
struct HPass {
  static constexpr int LR = L / R;
  static constexpr int NB = LR * NP;
  static constexpr int Q = (NB + kNT - 1) / kNT;
};

template <int R, int L, int NP, int Ns, int Q>
__device__ __forceinline__ void h_twiddle_dft(cpair (&v)[Q][R], const float2* __restrict__ tw) {
  using P = HPass<R, L, NP>;
  static_assert(P::Q == Q, "pass geometry");
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int b = threadIdx.x + q * kNT;
    if (P::NB % kNT == 0 || b < P::NB) {
      const int j = b / NP;
      if constexpr (Ns > 1) {
        const int k = j % Ns;
#pragma unroll
        for (int r = 1; r < R; ++r) v[q][r] = c_mul(v[q][r], tw[(r - 1) * Ns + k]);
      }
      Dft<R>::run(v[q]);
    }
    __builtin_amdgcn_sched_barrier(0);  // one item at a time: bounds the live registers
  }
}

struct AfnoArgs {
  const void* x;        // [B, H, KM, C, 2] fp32 or bf16
  void* y;              // [B, H, KM, C, 2] fp32 or bf16
  const uint16_t* w1t;  // [NB][2BS][2BS] bf16, [n][k]  (x3: [NB][2BS][2 * 2BS] split rows)
  const uint16_t* w2t;
  const float* b1;      // [NB][2BS]
  const float* b2;
  const float2* tw;     // plan twiddles for length H ([R0, R1] order)
  int KM, C, NB, H;
  float lambda;
};

// GEMM [16 MT x 2BS] = A (LDS bf16, pitch APitch) x Bt^T (global bf16 [n][k]); wave w owns
// column tiles NTW w .. NTW w + NTW - 1 for all MT row tiles.
// TR: MFMA operands swapped (transposed accumulator: a lane holds 4 consecutive columns of one row)
// AFNO_X3_T: GEMM 1 of both kernels runs transposed, so its epilogue writes 8-byte pieces
#ifndef AFNO_X3_T
#define AFNO_X3_T 1
#endif
// PERM: output column n' of the tile computes weight row (n' & 1) BS + (n' >> 1), i.e. the
// columns come out as interleaved (re, im) pairs of each channel (GEMM 2: with TR a lane then holds
// two channels' complex values of one row, one 8 / 16-byte LDS write)
template <class S, bool PERM>
__device__ __forceinline__ int brow(int n) { return PERM ? (n & 1) * S::BS + (n >> 1) : n; }

// B (weight) fragments of a GEMM's first D k-steps.  The weights do not depend on the tile, so
// (AFNO_BEARLY16 / AFNO_BEARLY3) GEMM 1's are requested right after the tile's input loads and GEMM 2's right after
// GEMM 1: their L2 round trips overlap the FFT passes / epilogue 1 instead of opening each GEMM
// (the barriers between are LDS-only for loads: __syncthreads waits on no outstanding global load).
// bit 0: GEMM 1's fragments early, bit 1: GEMM 2's; per kernel (bf16 / bf16x3).  Measured
// (profiles/afno_bearly_r5.txt): bf16x3 both -1.3 %, bf16 GEMM 2 early +3 % (168 VGPRs at 3 workgroups
// per CU), so the bf16 kernel keeps the in-GEMM prefetch
#ifndef AFNO_BEARLY16
#define AFNO_BEARLY16 0
#endif
#ifndef AFNO_BEARLY3
#define AFNO_BEARLY3 3
#endif
template <class S>
struct BFrags {
  static constexpr int D = AFNO_BPF < S::KS ? AFNO_BPF : S::KS - 1, NQ = D + 1;
  bf16x8 q[NQ][S::NTW];
};
template <class S, bool PERM>
__device__ __forceinline__ void b_prefetch(BFrags<S>& f, const uint16_t* __restrict__ Bt) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int s2 = 0; s2 < BFrags<S>::D; ++s2)
#pragma unroll
    for (int nj = 0; nj < S::NTW; ++nj)
      f.q[s2][nj] = *reinterpret_cast<const bf16x8*>(Bt + brow<S, PERM>(S::ct(w, nj) * 16 + r16) * S::K + s2 * 32 + kq * 8);
}

// TPW > 1 (two-tile kernel): row tiles mi of TPW (b, kw) tiles, tile mi / MT's A in its own LDS region
// (RSE bf16 elements apart); every weight fragment then feeds TPW x MT row tiles
template <class S, bool EARLY, bool TR = false, bool PERM = false, int TPW = 1>
__device__ __forceinline__ void gemm_tile(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                                          f32x4 (&acc)[TPW * S::MT][S::NTW], BFrags<S>& f) {
  constexpr int RSE = static_cast<int>(S::MAIN16 / 2);
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int mi = 0; mi < TPW * S::MT; ++mi)
#pragma unroll
    for (int nj = 0; nj < S::NTW; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
  // B fragments stream from L2 AFNO_BPF k-steps ahead (a full preload would need 24 KS VGPRs); the
  // first D are in f (b_prefetch)
  constexpr int D = BFrags<S>::D, NQ = BFrags<S>::NQ;
  auto& bq = f.q;
  if constexpr (!EARLY) b_prefetch<S, PERM>(f, Bt);
#pragma unroll
  for (int ks = 0; ks < S::KS; ++ks) {
    if (ks + D < S::KS) {
#pragma unroll
      for (int nj = 0; nj < S::NTW; ++nj)
        bq[(ks + D) % NQ][nj] =
            *reinterpret_cast<const bf16x8*>(Bt + brow<S, PERM>(S::ct(w, nj) * 16 + r16) * S::K + (ks + D) * 32 + kq * 8);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of its use (see gemm_tile_x3)
    bf16x8 afr[TPW * S::MT];
#pragma unroll
    for (int mi = 0; mi < TPW * S::MT; ++mi)
      afr[mi] = *reinterpret_cast<const bf16x8*>(A + (mi / S::MT) * RSE + ((mi % S::MT) * 16 + r16) * S::APitch + ks * 32 + kq * 8);
#pragma unroll
    for (int mi = 0; mi < TPW * S::MT; ++mi)
#pragma unroll
      for (int nj = 0; nj < S::NTW; ++nj) {
        if constexpr (TR) acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ks % NQ][nj], afr[mi], acc[mi][nj], 0, 0, 0);
        else acc[mi][nj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[mi], bq[ks % NQ][nj], acc[mi][nj], 0, 0, 0);
      }
  }
}

template <class S, bool BFI, bool BFO>
__global__ void __launch_bounds__(kNT, S::OCC) afno_spectral_kernel(const AfnoArgs a) {
  constexpr int L = S::L, R0 = S::R0, R1 = S::R1, BS = S::BS, NP = S::NP, K = S::K, AP = S::APitch;
  extern __shared__ __attribute__((aligned(16))) h2_t lds[];  // [L][BS] complex fp16
  uint16_t* A = reinterpret_cast<uint16_t*>(lds);             // aliases lds: [16 MT][APitch] bf16
  float2* twl = reinterpret_cast<float2*>(reinterpret_cast<char*>(lds) + S::MAIN16);
  const int tid = threadIdx.x;
  for (int i = tid; i < S::TWN; i += kNT) twl[i] = a.tw[i];  // visible after the pass-0 barrier
  const int blk = blockIdx.x % a.NB;
  const int bk = blockIdx.x / a.NB;  // b * KM + kw
  const int kw = bk % a.KM;
  const int b = bk / a.KM;
  AMD_DFT_DEV_CHECK((blk + 1) * BS <= a.C && kw < a.KM && L == a.H, "afno_spectral_kernel");
  const int row_stride = a.KM * a.C * 2;  // scalars between consecutive h (host-checked: 32-bit offsets)
  const int64_t base = ((static_cast<int64_t>(b) * L * a.KM + kw) * a.C + blk * BS) * 2;
  const void* xin = static_cast<const char*>(a.x) + base * (BFI ? 2 : 4);
  void* yout = static_cast<char*>(a.y) + base * (BFO ? 2 : 4);
  using P0 = HPass<R0, L, NP>;
  using P1 = HPass<R1, L, NP>;

  const uint16_t* w1t = a.w1t + static_cast<int64_t>(blk) * K * K;
  const uint16_t* w2t = a.w2t + static_cast<int64_t>(blk) * K * K;
  BFrags<S> pre1, pre2;  // the GEMMs' first k-steps of weight fragments
  // ---------------- forward FFT_H: pass 0 straight from global
  {
    cpair v[P0::Q][R0];
#pragma unroll
    for (int q = 0; q < P0::Q; ++q) {
      const int bb = tid + q * kNT;
      const bool ok = P0::NB % kNT == 0 || bb < P0::NB;
      const int bc = ok ? bb : 0;
      const int tp = bc % NP, j = bc / NP;
#pragma unroll
      for (int r = 0; r < R0; ++r) {
        float2 c0, c1;
        ldc2<BFI>(xin, (j + r * P0::LR) * row_stride + 4 * tp, c0, c1);
        v[q][r] = make_cpair(c0, c1);
      }
    }
    if constexpr ((AFNO_BEARLY16 & 1) != 0) b_prefetch<S, false>(pre1, w1t);  // behind the tile loads: pass 0 waits for those only
    h_twiddle_dft<R0, L, NP, 1, P0::Q>(v, nullptr);  // first pass: no twiddles
#pragma unroll
    for (int q = 0; q < P0::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P0::NB % kNT == 0 || bb < P0::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R0; ++r) st_hp(lds, (j * R0 + r) * BS + 2 * tp, v[q][r]);
      }
    }
  }
  __syncthreads();
  // ---------------- pass 1: LDS -> registers -> A (bf16, [h][re 0..BS-1 | im BS..2BS-1])
  {
    cpair v[P1::Q][R1];
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) v[q][r] = ld_hp(lds, (j + r * P1::LR) * BS + 2 * tp);
      }
    }
    __syncthreads();
    h_twiddle_dft<R1, L, NP, R0, P1::Q>(v, twl);
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;  // last pass: outputs at n = j + r * R0
#pragma unroll
        for (int r = 0; r < R1; ++r) {
          const int n = j + r * R0;
          uint32_t* row = reinterpret_cast<uint32_t*>(A + n * AP);
          row[tp] = static_cast<uint32_t>(f2bf16(v[q][r].re[0])) | (static_cast<uint32_t>(f2bf16(v[q][r].re[1])) << 16);
          row[NP + tp] = static_cast<uint32_t>(f2bf16(v[q][r].im[0])) | (static_cast<uint32_t>(f2bf16(v[q][r].im[1])) << 16);
        }
      }
    }
  }
  // rows L..16 MT - 1 of A (GEMM M padding) are never written: their outputs are discarded
  __syncthreads();
  // ---------------- GEMM1 + bias + ReLU -> H1 (bf16, in place of A)
  const int lane = tid & 63, w = tid >> 6;
  const float* b1 = a.b1 + blk * K;
  const float* b2 = a.b2 + blk * K;
  f32x4 acc[S::MT][S::NTW];
  gemm_tile<S, (AFNO_BEARLY16 & 1) != 0, AFNO_X3_T>(A, w1t, acc, pre1);
  if constexpr ((AFNO_BEARLY16 & 2) != 0) b_prefetch<S, true>(pre2, w2t);  // overlaps epilogue 1
  __syncthreads();
#pragma unroll
  for (int nj = 0; nj < S::NTW; ++nj) {
    if (!S::ct_live(w, nj)) continue;  // wave-uniform (BS % 32 != 0 only)
    if constexpr (AFNO_X3_T) {  // lane: columns n0 .. n0 + 3 of row m -> one 8-byte write
      const int n0 = (S::NTW * w + nj) * 16 + 4 * (lane >> 4);
      const float4 bias = *reinterpret_cast<const float4*>(b1 + n0);
#pragma unroll
      for (int mi = 0; mi < S::MT; ++mi) {
        const int m = mi * 16 + (lane & 15);
        *reinterpret_cast<uint2*>(A + m * AP + n0) =
            make_uint2(static_cast<uint32_t>(f2bf16(fmaxf(acc[mi][nj][0] + bias.x, 0.f))) |
                           (static_cast<uint32_t>(f2bf16(fmaxf(acc[mi][nj][1] + bias.y, 0.f))) << 16),
                       static_cast<uint32_t>(f2bf16(fmaxf(acc[mi][nj][2] + bias.z, 0.f))) |
                           (static_cast<uint32_t>(f2bf16(fmaxf(acc[mi][nj][3] + bias.w, 0.f))) << 16));
      }
    } else {
      const int n = (S::NTW * w + nj) * 16 + (lane & 15);
      const float bias = b1[n];
#pragma unroll
      for (int mi = 0; mi < S::MT; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mi * 16 + 4 * (lane >> 4) + i;
          A[m * AP + n] = f2bf16(fmaxf(acc[mi][nj][i] + bias, 0.f));
        }
    }
  }
  __syncthreads();
  // ---------------- GEMM2 + bias + softshrink -> X (fp16 complex, conjugated for the inverse):
  // transposed tile with (re, im)-interleaved columns, so a lane holds channels c0, c0 + 1 of one
  // row and writes them as one 8-byte piece (row pitch XP)
  gemm_tile<S, (AFNO_BEARLY16 & 2) != 0, true, true>(A, w2t, acc, pre2);
  __syncthreads();
  const float lam = a.lambda;
#pragma unroll
  for (int nj = 0; nj < S::NTW; ++nj) {
    if (!S::ct_live(w, nj)) continue;  // wave-uniform (BS % 32 != 0 only)
    const int c0 = ((S::NTW * w + nj) * 16 + 4 * (lane >> 4)) >> 1;
    const float2 bre = *reinterpret_cast<const float2*>(b2 + c0), bim = *reinterpret_cast<const float2*>(b2 + BS + c0);
#pragma unroll
    for (int mi = 0; mi < S::MT; ++mi) {
      const int m = mi * 16 + (lane & 15);
      if (m < L) {
        const float v0 = acc[mi][nj][0] + bre.x, v1 = acc[mi][nj][1] + bim.x;
        const float v2 = acc[mi][nj][2] + bre.y, v3 = acc[mi][nj][3] + bim.y;
        // softshrink; conj(Z) for the forward-FFT-as-inverse trick
        *reinterpret_cast<h4_t*>(lds + m * S::XP + c0) =
            h4_t{static_cast<_Float16>(v0 - __builtin_amdgcn_fmed3f(v0, -lam, lam)),
                 static_cast<_Float16>(__builtin_amdgcn_fmed3f(v1, -lam, lam) - v1),
                 static_cast<_Float16>(v2 - __builtin_amdgcn_fmed3f(v2, -lam, lam)),
                 static_cast<_Float16>(__builtin_amdgcn_fmed3f(v3, -lam, lam) - v3)};
      }
    }
  }
  __syncthreads();
  // ---------------- inverse FFT_H (conj trick): pass 0 LDS (pitch XP) -> LDS (pitch BS)
  {
    cpair v[P0::Q][R0];
#pragma unroll
    for (int q = 0; q < P0::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P0::NB % kNT == 0 || bb < P0::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R0; ++r) v[q][r] = ld_hp(lds, (j + r * P0::LR) * S::XP + 2 * tp);
      }
    }
    __syncthreads();
    h_twiddle_dft<R0, L, NP, 1, P0::Q>(v, nullptr);  // first pass: no twiddles
#pragma unroll
    for (int q = 0; q < P0::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P0::NB % kNT == 0 || bb < P0::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R0; ++r) st_hp(lds, (j * R0 + r) * BS + 2 * tp, v[q][r]);
      }
    }
  }
  __syncthreads();
  // ---------------- pass 1: LDS -> registers -> global (conj back)
  {
    cpair v[P1::Q][R1];
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) v[q][r] = ld_hp(lds, (j + r * P1::LR) * BS + 2 * tp);
      }
    }
    h_twiddle_dft<R1, L, NP, R0, P1::Q>(v, twl);
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) {
          const int n = j + r * R0;
          stc2<BFO>(yout, n * row_stride + 4 * tp, make_float2(v[q][r].re[0], -v[q][r].im[0]),
                    make_float2(v[q][r].re[1], -v[q][r].im[1]));
        }
      }
    }
  }
}

// ------------------------------------------------------------------ two tiles per workgroup (bf16)
// The same stages for two (b, kw) tiles of one channel block: each tile has its own LDS region
// (staging / A / X, MAIN16 bytes), the FFT passes run both tiles between the same barriers, and the two
// GEMMs see 2 MT row tiles -- every weight fragment loaded from L2 feeds twice the MFMAs.  LDS 2 x 38.4 KB
// at H = 90, BS = 96: 2 workgroups (4 tiles) per CU instead of 3 single-tile ones; -2 % at [32, 90, 46, 768]
// (profiles/afno_two_tile_r5.txt).
#ifndef AFNO_TPW16
#define AFNO_TPW16 2  // (b, kw) tiles per workgroup of the bf16 kernel: 1 or 2
#endif
template <class S, bool BFI, bool BFO>
__global__ void __launch_bounds__(kNT, 2) afno_spectral2_kernel(const AfnoArgs a) {
  static_assert(AFNO_X3_T, "the two-tile kernel has only the transposed GEMM-1 epilogue");
  constexpr int L = S::L, R0 = S::R0, R1 = S::R1, BS = S::BS, NP = S::NP, K = S::K, AP = S::APitch;
  constexpr int64_t RB = S::MAIN16;  // bytes per tile region
  extern __shared__ __attribute__((aligned(16))) h2_t lds[];
  auto reg = [&](int t) { return reinterpret_cast<h2_t*>(reinterpret_cast<char*>(lds) + t * RB); };
  auto areg = [&](int t) { return reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(lds) + t * RB); };
  float2* twl = reinterpret_cast<float2*>(reinterpret_cast<char*>(lds) + 2 * RB);
  const int tid = threadIdx.x;
  for (int i = tid; i < S::TWN; i += kNT) twl[i] = a.tw[i];  // visible after the pass-0 barrier
  const int blk = blockIdx.x % a.NB;
  const int pair = blockIdx.x / a.NB;  // tiles bk = 2 pair, 2 pair + 1 (host: B KM even)
  const int row_stride = a.KM * a.C * 2;
  const void* xin[2];
  void* yout[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int bk = 2 * pair + t, kw = bk % a.KM, b = bk / a.KM;
    AMD_DFT_DEV_CHECK((blk + 1) * BS <= a.C && kw < a.KM && L == a.H, "afno_spectral2_kernel");
    const int64_t base = ((static_cast<int64_t>(b) * L * a.KM + kw) * a.C + blk * BS) * 2;
    xin[t] = static_cast<const char*>(a.x) + base * (BFI ? 2 : 4);
    yout[t] = static_cast<char*>(a.y) + base * (BFO ? 2 : 4);
  }
  using P0 = HPass<R0, L, NP>;
  using P1 = HPass<R1, L, NP>;
  const uint16_t* w1t = a.w1t + static_cast<int64_t>(blk) * K * K;
  const uint16_t* w2t = a.w2t + static_cast<int64_t>(blk) * K * K;
  BFrags<S> pre1, pre2;
  // ---------------- forward FFT_H: pass 0 straight from global, both tiles' loads first
  {
    cpair v[2][P0::Q][R0];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < P0::Q; ++q) {
        const int bb = tid + q * kNT;
        const bool ok = P0::NB % kNT == 0 || bb < P0::NB;
        const int bc = ok ? bb : 0;
        const int tp = bc % NP, j = bc / NP;
#pragma unroll
        for (int r = 0; r < R0; ++r) {
          float2 c0, c1;
          ldc2<BFI>(xin[t], (j + r * P0::LR) * row_stride + 4 * tp, c0, c1);
          v[t][q][r] = make_cpair(c0, c1);
        }
      }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      h_twiddle_dft<R0, L, NP, 1, P0::Q>(v[t], nullptr);
#pragma unroll
      for (int q = 0; q < P0::Q; ++q) {
        const int bb = tid + q * kNT;
        if (P0::NB % kNT == 0 || bb < P0::NB) {
          const int tp = bb % NP, j = bb / NP;
#pragma unroll
          for (int r = 0; r < R0; ++r) st_hp(reg(t), (j * R0 + r) * BS + 2 * tp, v[t][q][r]);
        }
      }
    }
  }
  __syncthreads();
  // ---------------- pass 1: LDS -> registers -> A_t (bf16, [h][re | im])
  {
    cpair v[2][P1::Q][R1];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < P1::Q; ++q) {
        const int bb = tid + q * kNT;
        if (P1::NB % kNT == 0 || bb < P1::NB) {
          const int tp = bb % NP, j = bb / NP;
#pragma unroll
          for (int r = 0; r < R1; ++r) v[t][q][r] = ld_hp(reg(t), (j + r * P1::LR) * BS + 2 * tp);
        }
      }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      h_twiddle_dft<R1, L, NP, R0, P1::Q>(v[t], twl);
#pragma unroll
      for (int q = 0; q < P1::Q; ++q) {
        const int bb = tid + q * kNT;
        if (P1::NB % kNT == 0 || bb < P1::NB) {
          const int tp = bb % NP, j = bb / NP;
#pragma unroll
          for (int r = 0; r < R1; ++r) {
            const int n = j + r * R0;
            uint32_t* row = reinterpret_cast<uint32_t*>(areg(t) + n * AP);
            row[tp] = static_cast<uint32_t>(f2bf16(v[t][q][r].re[0])) | (static_cast<uint32_t>(f2bf16(v[t][q][r].re[1])) << 16);
            row[NP + tp] = static_cast<uint32_t>(f2bf16(v[t][q][r].im[0])) | (static_cast<uint32_t>(f2bf16(v[t][q][r].im[1])) << 16);
          }
        }
      }
    }
  }
  __syncthreads();
  // ---------------- GEMM1 + bias + ReLU -> H1 (in place of A_t)
  const int lane = tid & 63, w = tid >> 6;
  const float* b1 = a.b1 + blk * K;
  const float* b2 = a.b2 + blk * K;
  f32x4 acc[2 * S::MT][S::NTW];
  gemm_tile<S, false, AFNO_X3_T, false, 2>(areg(0), w1t, acc, pre1);
  __syncthreads();
#pragma unroll
  for (int nj = 0; nj < S::NTW; ++nj) {
    if (!S::ct_live(w, nj)) continue;
    const int n0 = (S::NTW * w + nj) * 16 + 4 * (lane >> 4);
    const float4 bias = *reinterpret_cast<const float4*>(b1 + n0);
#pragma unroll
    for (int mi = 0; mi < 2 * S::MT; ++mi) {
      const int m = (mi % S::MT) * 16 + (lane & 15);
      *reinterpret_cast<uint2*>(areg(mi / S::MT) + m * AP + n0) =
          make_uint2(static_cast<uint32_t>(f2bf16(fmaxf(acc[mi][nj][0] + bias.x, 0.f))) |
                         (static_cast<uint32_t>(f2bf16(fmaxf(acc[mi][nj][1] + bias.y, 0.f))) << 16),
                     static_cast<uint32_t>(f2bf16(fmaxf(acc[mi][nj][2] + bias.z, 0.f))) |
                         (static_cast<uint32_t>(f2bf16(fmaxf(acc[mi][nj][3] + bias.w, 0.f))) << 16));
    }
  }
  __syncthreads();
  // ---------------- GEMM2 + bias + softshrink -> X_t (fp16, pitch XP, conjugated)
  gemm_tile<S, false, true, true, 2>(areg(0), w2t, acc, pre2);
  __syncthreads();
  const float lam = a.lambda;
#pragma unroll
  for (int nj = 0; nj < S::NTW; ++nj) {
    if (!S::ct_live(w, nj)) continue;
    const int c0 = ((S::NTW * w + nj) * 16 + 4 * (lane >> 4)) >> 1;
    const float2 bre = *reinterpret_cast<const float2*>(b2 + c0), bim = *reinterpret_cast<const float2*>(b2 + BS + c0);
#pragma unroll
    for (int mi = 0; mi < 2 * S::MT; ++mi) {
      const int m = (mi % S::MT) * 16 + (lane & 15);
      if (m < L) {
        const float v0 = acc[mi][nj][0] + bre.x, v1 = acc[mi][nj][1] + bim.x;
        const float v2 = acc[mi][nj][2] + bre.y, v3 = acc[mi][nj][3] + bim.y;
        *reinterpret_cast<h4_t*>(reg(mi / S::MT) + m * S::XP + c0) =
            h4_t{static_cast<_Float16>(v0 - __builtin_amdgcn_fmed3f(v0, -lam, lam)),
                 static_cast<_Float16>(__builtin_amdgcn_fmed3f(v1, -lam, lam) - v1),
                 static_cast<_Float16>(v2 - __builtin_amdgcn_fmed3f(v2, -lam, lam)),
                 static_cast<_Float16>(__builtin_amdgcn_fmed3f(v3, -lam, lam) - v3)};
      }
    }
  }
  __syncthreads();
  // ---------------- inverse FFT_H: pass 0 LDS (pitch XP) -> LDS (pitch BS), both tiles
  {
    cpair v[2][P0::Q][R0];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < P0::Q; ++q) {
        const int bb = tid + q * kNT;
        if (P0::NB % kNT == 0 || bb < P0::NB) {
          const int tp = bb % NP, j = bb / NP;
#pragma unroll
          for (int r = 0; r < R0; ++r) v[t][q][r] = ld_hp(reg(t), (j + r * P0::LR) * S::XP + 2 * tp);
        }
      }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      h_twiddle_dft<R0, L, NP, 1, P0::Q>(v[t], nullptr);
#pragma unroll
      for (int q = 0; q < P0::Q; ++q) {
        const int bb = tid + q * kNT;
        if (P0::NB % kNT == 0 || bb < P0::NB) {
          const int tp = bb % NP, j = bb / NP;
#pragma unroll
          for (int r = 0; r < R0; ++r) st_hp(reg(t), (j * R0 + r) * BS + 2 * tp, v[t][q][r]);
        }
      }
    }
  }
  __syncthreads();
  // ---------------- pass 1: LDS -> registers -> global (conj back), one tile at a time
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    cpair v[P1::Q][R1];
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) v[q][r] = ld_hp(reg(t), (j + r * P1::LR) * BS + 2 * tp);
      }
    }
    h_twiddle_dft<R1, L, NP, R0, P1::Q>(v, twl);
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) {
          const int n = j + r * R0;
          stc2<BFO>(yout[t], n * row_stride + 4 * tp, make_float2(v[q][r].re[0], -v[q][r].im[0]),
                    make_float2(v[q][r].re[1], -v[q][r].im[1]));
        }
      }
    }
  }
}

// ================================================================== fp32 variant (bf16x3)
// Same structure for the fp32 FourCastNet path: fp32 spectrum in/out, fp32 LDS staging of the
// H-FFT, and the two block-MLP GEMMs as 3-product split GEMMs -- an fp32 operand is the bf16
// pair hi + lo and A.B = Ah.Bh + Al.Bh + Ah.Bl with fp32 accumulation (relative error ~5e-6,
// the exact-f32 MFMA would cost 16x the bf16 rate, this 3x).  The A operand is split into two
// bf16 planes [16 MT][APitch] (hi, lo) when it is written to LDS; the weights arrive pre-split
// as k32-interleaved rows [NB][2BS n][2 * 2BS k].  76.8 KB of LDS at H = 90, BS = 96: 2
// workgroups per CU.
// LIMIT: the workgroup's dynamic LDS bytes; MI_DFT_DEVICE_CHECKS builds check every 16-byte
// staging access against it and its alignment (the accesses the -O3 vectorizer turns into
// ds_read_b128 / ds_write_b128)
template <int64_t LIMIT>
__device__ __forceinline__ void st_fp(float2* p, int i, const cpair& v) {
  AMD_DFT_DEV_LDS(static_cast<int64_t>(i) * 8, 16, LIMIT, "afno st_fp");
  *reinterpret_cast<float4*>(p + i) = make_float4(v.re[0], v.im[0], v.re[1], v.im[1]);
}
template <int64_t LIMIT>
__device__ __forceinline__ cpair ld_fp(const float2* p, int i) {
  AMD_DFT_DEV_LDS(static_cast<int64_t>(i) * 8, 16, LIMIT, "afno ld_fp");
  const float4 q = *reinterpret_cast<const float4*>(p + i);
  return cpair{f2v{q.x, q.z}, f2v{q.y, q.w}};
}
__device__ __forceinline__ void put_split(uint16_t* Ahi, uint16_t* Alo, int idx, float v) {
  const uint16_t h = f2bf16(v);
  Ahi[idx] = h;
  Alo[idx] = f2bf16(v - __uint_as_float(static_cast<uint32_t>(h) << 16));
}
__device__ __forceinline__ void put_split2(uint16_t* Ahi, uint16_t* Alo, int idx2, float a, float b) {
  const uint16_t ha = f2bf16(a), hb = f2bf16(b);
  reinterpret_cast<uint32_t*>(Ahi)[idx2] = static_cast<uint32_t>(ha) | (static_cast<uint32_t>(hb) << 16);
  reinterpret_cast<uint32_t*>(Alo)[idx2] =
      static_cast<uint32_t>(f2bf16(a - __uint_as_float(static_cast<uint32_t>(ha) << 16))) |
      (static_cast<uint32_t>(f2bf16(b - __uint_as_float(static_cast<uint32_t>(hb) << 16))) << 16);
}

// four consecutive values (8-byte aligned idx) as bf16 hi / lo pieces
__device__ __forceinline__ void put_split4(uint16_t* Ahi, uint16_t* Alo, int idx, float a, float b, float c, float d) {
  const uint16_t ha = f2bf16(a), hb = f2bf16(b), hc = f2bf16(c), hd = f2bf16(d);
  const auto up = [](uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); };
  *reinterpret_cast<uint2*>(Ahi + idx) = make_uint2(static_cast<uint32_t>(ha) | (static_cast<uint32_t>(hb) << 16),
                                                    static_cast<uint32_t>(hc) | (static_cast<uint32_t>(hd) << 16));
  *reinterpret_cast<uint2*>(Alo + idx) =
      make_uint2(static_cast<uint32_t>(f2bf16(a - up(ha))) | (static_cast<uint32_t>(f2bf16(b - up(hb))) << 16),
                 static_cast<uint32_t>(f2bf16(c - up(hc))) | (static_cast<uint32_t>(f2bf16(d - up(hd))) << 16));
}

// [16 MT x 2BS] = (Ah + Al) x (Bh + Bl)^T without Al.Bl; wave w owns column tiles NTW w ..
// TR: the same products with the MFMA operands swapped, so the accumulator tile is the transpose:
// a lane holds 4 CONSECUTIVE output columns n of one row m (instead of 4 rows of one column) --
// the epilogue then writes 8-byte bf16x4 pieces instead of single bf16 values.
// B (weight) fragments stream from L2 AFNO_BPF3 k-steps ahead: with one k-step of lookahead the L2
// latency is exposed every k-step (a timing-only build that reused the first k-step's fragments ran
// 164 us faster, round 2).  The first D k-steps are requested early (b_prefetch_x3, AFNO_BEARLY3).
template <class S>
struct BFragsX3 {
  static constexpr int D0 = S::NTW >= 4 ? 1 : AFNO_BPF3;  // 4 column tiles per wave: no registers for 2
  static constexpr int D = D0 < S::KS ? D0 : S::KS - 1, NQ = D + 1;
  bf16x8 h[NQ][S::NTW], l[NQ][S::NTW];
};
template <class S, bool PERM>
__device__ __forceinline__ void b_prefetch_x3(BFragsX3<S>& f, const uint16_t* __restrict__ Bt) {
  constexpr int K2 = 2 * S::K;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int s2 = 0; s2 < BFragsX3<S>::D; ++s2)
#pragma unroll
    for (int nj = 0; nj < S::NTW; ++nj) {
      const uint16_t* row = Bt + brow<S, PERM>(S::ct(w, nj) * 16 + r16) * K2 + s2 * 64 + kq * 8;
      f.h[s2][nj] = *reinterpret_cast<const bf16x8*>(row);
      f.l[s2][nj] = *reinterpret_cast<const bf16x8*>(row + 32);
    }
}

template <class S, bool EARLY, bool TR = false, bool PERM = false>
__device__ __forceinline__ void gemm_tile_x3(const uint16_t* __restrict__ Ah, const uint16_t* __restrict__ Al,
                                             const uint16_t* __restrict__ Bt, f32x4 (&acc)[S::MT][S::NTW],
                                             BFragsX3<S>& f) {
  constexpr int K2 = 2 * S::K;  // split weight row: k32-interleaved [hi(32) | lo(32)] chunks
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int mi = 0; mi < S::MT; ++mi)
#pragma unroll
    for (int nj = 0; nj < S::NTW; ++nj) acc[mi][nj] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int D = BFragsX3<S>::D, NQ = BFragsX3<S>::NQ;
  auto& bh = f.h;
  auto& bl = f.l;
  if constexpr (!EARLY) b_prefetch_x3<S, PERM>(f, Bt);
#pragma unroll
  for (int ks = 0; ks < S::KS; ++ks) {
    if (ks + D < S::KS) {
#pragma unroll
      for (int nj = 0; nj < S::NTW; ++nj) {
        const uint16_t* row = Bt + brow<S, PERM>(S::ct(w, nj) * 16 + r16) * K2 + (ks + D) * 64 + kq * 8;
        bh[(ks + D) % NQ][nj] = *reinterpret_cast<const bf16x8*>(row);
        bl[(ks + D) % NQ][nj] = *reinterpret_cast<const bf16x8*>(row + 32);
      }
    }
    // keep the prefetch where it is written: the scheduler otherwise sinks these loads next to
    // their MFMAs (lower register pressure) and every k-step waits for an L2 round trip
    __builtin_amdgcn_sched_barrier(0);
    // row tiles in groups of MG, the three products outermost within a group: consecutive MFMAs
    // write different accumulators (MG x NTW apart) instead of chaining three on one accumulator
    constexpr int MG = S::MT % 3 == 0 ? 3 : (S::MT % 2 == 0 ? 2 : 1);
#pragma unroll
    for (int m0 = 0; m0 < S::MT; m0 += MG) {
      bf16x8 ah[MG], al[MG];
#pragma unroll
      for (int g = 0; g < MG; ++g) {
        ah[g] = *reinterpret_cast<const bf16x8*>(Ah + ((m0 + g) * 16 + r16) * S::APitch + ks * 32 + kq * 8);
        al[g] = *reinterpret_cast<const bf16x8*>(Al + ((m0 + g) * 16 + r16) * S::APitch + ks * 32 + kq * 8);
      }
#pragma unroll
      for (int pr = 0; pr < 3; ++pr)
#pragma unroll
        for (int g = 0; g < MG; ++g)
#pragma unroll
          for (int nj = 0; nj < S::NTW; ++nj) {
            const bf16x8 av = pr == 0 ? al[g] : ah[g];
            const bf16x8 bv = pr == 1 ? bl[ks % NQ][nj] : bh[ks % NQ][nj];
            f32x4& c = acc[m0 + g][nj];
            if constexpr (TR) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv, av, c, 0, 0, 0);
            else c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
          }
    }
  }
}

template <class S>
__global__ void __launch_bounds__(kNT, 2) afno_spectral_x3_kernel(const AfnoArgs a) {
  AFNO_STAMP(0, __builtin_amdgcn_s_memrealtime());
  AFNO_STAMP(1, __builtin_amdgcn_s_memtime());
  constexpr int L = S::L, R0 = S::R0, R1 = S::R1, BS = S::BS, NP = S::NP, K = S::K, AP = S::APitch;
  constexpr int plane = 16 * S::MT * AP;                         // bf16 elements per A plane
  constexpr int64_t LDSB = S::MAIN32;  // the staging / A-plane area (twiddles follow it)
  static_assert(S::MAIN32 >= 2LL * L * S::XP * 4 && S::MAIN32 >= 4LL * plane, "x3 LDS layout");
  extern __shared__ __attribute__((aligned(16))) float2 ldsf[];  // [L][BS] complex fp32
  uint16_t* Ah = reinterpret_cast<uint16_t*>(ldsf);              // aliases: [16 MT][APitch] bf16 hi
  uint16_t* Al = Ah + plane;                                     //          [16 MT][APitch] bf16 lo
  float2* twl = reinterpret_cast<float2*>(reinterpret_cast<char*>(ldsf) + S::MAIN32);
  const int tid = threadIdx.x;
  for (int i = tid; i < S::TWN; i += kNT) twl[i] = a.tw[i];  // visible after the pass-0 barrier
  const int blk = blockIdx.x % a.NB;
  const int bk = blockIdx.x / a.NB;
  const int kw = bk % a.KM;
  const int b = bk / a.KM;
  AMD_DFT_DEV_CHECK((blk + 1) * BS <= a.C && kw < a.KM && L == a.H, "afno_spectral_x3_kernel");
  const int row_stride = a.KM * a.C * 2;
  const int64_t base = ((static_cast<int64_t>(b) * L * a.KM + kw) * a.C + blk * BS) * 2;
  const float* xin = static_cast<const float*>(a.x) + base;
  float* yout = static_cast<float*>(a.y) + base;
  using P0 = HPass<R0, L, NP>;
  using P1 = HPass<R1, L, NP>;
  const uint16_t* w1t = a.w1t + static_cast<int64_t>(blk) * K * 2 * K;
  const uint16_t* w2t = a.w2t + static_cast<int64_t>(blk) * K * 2 * K;
  BFragsX3<S> pre1, pre2;  // the GEMMs' first k-steps of weight fragments
  // ---------------- forward FFT_H: pass 0 straight from global
  {
    cpair v[P0::Q][R0];
#pragma unroll
    for (int q = 0; q < P0::Q; ++q) {
      const int bb = tid + q * kNT;
      const bool ok = P0::NB % kNT == 0 || bb < P0::NB;
      const int bc = ok ? bb : 0;
      const int tp = bc % NP, j = bc / NP;
#pragma unroll
      for (int r = 0; r < R0; ++r) {
        float2 c0, c1;
        ldc2<false>(xin, (j + r * P0::LR) * row_stride + 4 * tp, c0, c1);
        v[q][r] = make_cpair(c0, c1);
      }
    }
    if constexpr ((AFNO_BEARLY3 & 1) != 0) b_prefetch_x3<S, false>(pre1, w1t);  // behind the tile loads: pass 0 waits for those only
    h_twiddle_dft<R0, L, NP, 1, P0::Q>(v, nullptr);  // first pass: no twiddles
#pragma unroll
    for (int q = 0; q < P0::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P0::NB % kNT == 0 || bb < P0::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R0; ++r) st_fp<LDSB>(ldsf, (j * R0 + r) * BS + 2 * tp, v[q][r]);
      }
    }
  }
  __syncthreads();
  AFNO_STAMP(2, __builtin_amdgcn_s_memtime());
  // ---------------- pass 1: LDS -> registers -> A planes ([h][re 0..BS-1 | im BS..2BS-1], hi / lo)
  {
    cpair v[P1::Q][R1];
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) v[q][r] = ld_fp<LDSB>(ldsf, (j + r * P1::LR) * BS + 2 * tp);
      }
    }
    __syncthreads();
    AFNO_STAMP(3, __builtin_amdgcn_s_memtime());
    h_twiddle_dft<R1, L, NP, R0, P1::Q>(v, twl);
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) {
          const int n = j + r * R0;
          put_split2(Ah, Al, (n * AP) / 2 + tp, v[q][r].re[0], v[q][r].re[1]);
          put_split2(Ah, Al, (n * AP) / 2 + NP + tp, v[q][r].im[0], v[q][r].im[1]);
        }
      }
    }
  }
  // rows L..16 MT - 1 of A (GEMM M padding) are never written: their outputs are discarded
  __syncthreads();
  AFNO_STAMP(4, __builtin_amdgcn_s_memtime());
  const int lane = tid & 63, w = tid >> 6;
  const float* b1 = a.b1 + blk * K;
  const float* b2 = a.b2 + blk * K;
  f32x4 acc[S::MT][S::NTW];
  gemm_tile_x3<S, (AFNO_BEARLY3 & 1) != 0, AFNO_X3_T>(Ah, Al, w1t, acc, pre1);
  if constexpr ((AFNO_BEARLY3 & 2) != 0) b_prefetch_x3<S, true>(pre2, w2t);  // overlaps epilogue 1
  __syncthreads();
  AFNO_STAMP(5, __builtin_amdgcn_s_memtime());
#pragma unroll
  for (int nj = 0; nj < S::NTW; ++nj) {
    if (!S::ct_live(w, nj)) continue;  // wave-uniform (BS % 32 != 0 only)
    if constexpr (AFNO_X3_T) {  // lane: columns n0 .. n0 + 3 of row m -> one 8-byte piece per plane
      const int n0 = (S::NTW * w + nj) * 16 + 4 * (lane >> 4);
      const float4 bias = *reinterpret_cast<const float4*>(b1 + n0);
#pragma unroll
      for (int mi = 0; mi < S::MT; ++mi) {
        const int m = mi * 16 + (lane & 15);
        put_split4(Ah, Al, m * AP + n0, fmaxf(acc[mi][nj][0] + bias.x, 0.f), fmaxf(acc[mi][nj][1] + bias.y, 0.f),
                   fmaxf(acc[mi][nj][2] + bias.z, 0.f), fmaxf(acc[mi][nj][3] + bias.w, 0.f));
      }
    } else {
      const int n = (S::NTW * w + nj) * 16 + (lane & 15);
      const float bias = b1[n];
#pragma unroll
      for (int mi = 0; mi < S::MT; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = mi * 16 + 4 * (lane >> 4) + i;
          put_split(Ah, Al, m * AP + n, fmaxf(acc[mi][nj][i] + bias, 0.f));
        }
    }
  }
  __syncthreads();
  AFNO_STAMP(6, __builtin_amdgcn_s_memtime());
  // transposed tile, (re, im)-interleaved columns: one 16-byte write of two channels per lane and row
  gemm_tile_x3<S, (AFNO_BEARLY3 & 2) != 0, true, true>(Ah, Al, w2t, acc, pre2);
  __syncthreads();
  AFNO_STAMP(7, __builtin_amdgcn_s_memtime());
  const float lam = a.lambda;
#pragma unroll
  for (int nj = 0; nj < S::NTW; ++nj) {
    if (!S::ct_live(w, nj)) continue;  // wave-uniform (BS % 32 != 0 only)
    const int c0 = ((S::NTW * w + nj) * 16 + 4 * (lane >> 4)) >> 1;
    const float2 bre = *reinterpret_cast<const float2*>(b2 + c0), bim = *reinterpret_cast<const float2*>(b2 + BS + c0);
#pragma unroll
    for (int mi = 0; mi < S::MT; ++mi) {
      const int m = mi * 16 + (lane & 15);
      if (m < L) {
        const float v0 = acc[mi][nj][0] + bre.x, v1 = acc[mi][nj][1] + bim.x;
        const float v2 = acc[mi][nj][2] + bre.y, v3 = acc[mi][nj][3] + bim.y;
        // softshrink; conj(Z) for the forward-FFT-as-inverse trick
        AMD_DFT_DEV_LDS(static_cast<int64_t>(m * S::XP + c0) * 8, 16, LDSB, "afno x3 epilogue 2");
        *reinterpret_cast<float4*>(ldsf + m * S::XP + c0) =
            make_float4(v0 - __builtin_amdgcn_fmed3f(v0, -lam, lam), __builtin_amdgcn_fmed3f(v1, -lam, lam) - v1,
                        v2 - __builtin_amdgcn_fmed3f(v2, -lam, lam), __builtin_amdgcn_fmed3f(v3, -lam, lam) - v3);
      }
    }
  }
  __syncthreads();
  AFNO_STAMP(8, __builtin_amdgcn_s_memtime());
  // ---------------- inverse FFT_H (conj trick): pass 0 LDS (pitch XP) -> LDS (pitch BS)
  {
    cpair v[P0::Q][R0];
#pragma unroll
    for (int q = 0; q < P0::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P0::NB % kNT == 0 || bb < P0::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R0; ++r) v[q][r] = ld_fp<LDSB>(ldsf, (j + r * P0::LR) * S::XP + 2 * tp);
      }
    }
    __syncthreads();
    AFNO_STAMP(9, __builtin_amdgcn_s_memtime());
    h_twiddle_dft<R0, L, NP, 1, P0::Q>(v, nullptr);  // first pass: no twiddles
#pragma unroll
    for (int q = 0; q < P0::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P0::NB % kNT == 0 || bb < P0::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R0; ++r) st_fp<LDSB>(ldsf, (j * R0 + r) * BS + 2 * tp, v[q][r]);
      }
    }
  }
  __syncthreads();
  AFNO_STAMP(10, __builtin_amdgcn_s_memtime());
  // ---------------- pass 1: LDS -> registers -> global (conj back)
  {
    cpair v[P1::Q][R1];
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) v[q][r] = ld_fp<LDSB>(ldsf, (j + r * P1::LR) * BS + 2 * tp);
      }
    }
    h_twiddle_dft<R1, L, NP, R0, P1::Q>(v, twl);
#pragma unroll
    for (int q = 0; q < P1::Q; ++q) {
      const int bb = tid + q * kNT;
      if (P1::NB % kNT == 0 || bb < P1::NB) {
        const int tp = bb % NP, j = bb / NP;
#pragma unroll
        for (int r = 0; r < R1; ++r) {
          const int n = j + r * R0;
          stc2<false>(yout, n * row_stride + 4 * tp, make_float2(v[q][r].re[0], -v[q][r].im[0]),
                      make_float2(v[q][r].re[1], -v[q][r].im[1]));
        }
      }
    }
  }
  AFNO_STAMP(12, __builtin_amdgcn_s_memtime());
  AFNO_STAMP(11, __builtin_amdgcn_s_memrealtime());
}

// ------------------------------------------------------------------ instance table
// (H, R0, R1, block size): (R0, R1) must be the FFT plan's radix order for H (plan_info),
// because the kernel reads the plan's twiddle table; launch_afno_spectral checks it.
#define AFNO_SHAPES(X) \
  X(90, 9, 10, 96)     \
  X(90, 9, 10, 64)     \
  X(90, 9, 10, 128)    \
  X(90, 9, 10, 48)     \
  X(45, 9, 5, 96)      \
  X(45, 9, 5, 64)      \
  X(45, 9, 5, 128)     \
  X(45, 9, 5, 48)      \
  X(64, 16, 4, 64)     \
  X(64, 16, 4, 96)     \
  X(64, 16, 4, 128)    \
  X(64, 16, 4, 48)

using KernFn = void (*)(AfnoArgs);
struct AfnoInstance {
  int H, R0, R1, BS;
  int64_t lds_bf16, lds_x3, lds_bf16x2;  // dynamic LDS bytes of the bf16, bf16x3 and two-tile bf16 kernels
  KernFn bf16[2][2];                     // [bf16_in][bf16_out]
  KernFn x3;
  KernFn bf16x2[2][2];                   // two (b, kw) tiles per workgroup
};

template <class S>
AfnoInstance make_instance() {
  AfnoInstance r{S::L, S::R0, S::R1, S::BS, S::LDS16, S::LDS32, S::LDS16X2,
                 {{afno_spectral_kernel<S, false, false>, afno_spectral_kernel<S, false, true>},
                  {afno_spectral_kernel<S, true, false>, afno_spectral_kernel<S, true, true>}},
                 afno_spectral_x3_kernel<S>,
                 {{nullptr, nullptr}, {nullptr, nullptr}}};
  if constexpr (S::TPW2) {
    r.bf16x2[0][0] = afno_spectral2_kernel<S, false, false>;
    r.bf16x2[0][1] = afno_spectral2_kernel<S, false, true>;
    r.bf16x2[1][0] = afno_spectral2_kernel<S, true, false>;
    r.bf16x2[1][1] = afno_spectral2_kernel<S, true, true>;
  }
  return r;
}

#define AFNO_INSTANCE(H, R0, R1, BS) make_instance<AfnoShape<H, R0, R1, BS>>(),
const std::vector<AfnoInstance>& instances() {
  static const std::vector<AfnoInstance> v = {AFNO_SHAPES(AFNO_INSTANCE)};
  return v;
}

const AfnoInstance* find_instance(int H, int bs) {
  for (const auto& i : instances())
    if (i.H == H && i.BS == bs) return &i;
  return nullptr;
}

void launch_kernel(KernFn kern, int64_t lds, int64_t nblocks, const AfnoArgs& a, void* stream) {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     static_cast<int>(lds));
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: afno_spectral attr: ") + hipGetErrorString(e));
  hipLaunchKernelGGL(kern, dim3(static_cast<uint32_t>(nblocks)), dim3(kNT), static_cast<size_t>(lds),
                     static_cast<hipStream_t>(stream), a);
  e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: afno_spectral launch: ") + hipGetErrorString(e));
}

}  // namespace

bool afno_spectral_supported(int H, int block_size) { return find_instance(H, block_size) != nullptr; }

std::vector<std::pair<int, int>> afno_spectral_shapes() {
  std::vector<std::pair<int, int>> v;
  for (const auto& i : instances()) v.emplace_back(i.H, i.BS);
  return v;
}

int64_t afno_spectral_lds_bytes(int H, int block_size, bool x3) {
  const AfnoInstance* in = find_instance(H, block_size);
  return in ? (x3 ? in->lds_x3 : in->lds_bf16) : 0;
}

void launch_afno_spectral(const AfnoLaunch& p, void* stream) {
  if (p.NB <= 0 || p.C % p.NB) throw std::runtime_error("amd_dft: afno_spectral: C must be a multiple of NB");
  const AfnoInstance* in = find_instance(p.H, p.C / p.NB);
  if (!in) throw std::runtime_error("amd_dft: afno_spectral: unsupported shape");
  if (p.r0 != in->R0 || p.r1 != in->R1)
    throw std::runtime_error("amd_dft: afno_spectral: twiddle table radix order does not match the kernel");
  if (static_cast<int64_t>(p.H) * p.KM * p.C * 2 >= (int64_t(1) << 31))
    throw std::runtime_error("amd_dft: afno_spectral: per-batch spectrum exceeds 32-bit offsets");
  AfnoArgs a;
  a.x = p.x;
  a.y = p.y;
  a.w1t = p.w1t;
  a.w2t = p.w2t;
  a.b1 = p.b1;
  a.b2 = p.b2;
  a.tw = static_cast<const float2*>(p.tw);
  a.KM = p.KM;
  a.C = p.C;
  a.NB = p.NB;
  a.H = p.H;
  a.lambda = p.lambda;
  const int64_t nblocks = static_cast<int64_t>(p.B) * p.KM * p.NB;
  if (nblocks <= 0) return;
  if (p.x3) {
    if (p.bf16_in || p.bf16_out) throw std::runtime_error("amd_dft: afno_spectral: the bf16x3 variant is fp32 in/out");
    launch_kernel(in->x3, in->lds_x3, nblocks, a, stream);
    return;
  }
  if (AFNO_TPW16 == 2 && in->bf16x2[0][0] != nullptr && (static_cast<int64_t>(p.B) * p.KM) % 2 == 0) {
    launch_kernel(in->bf16x2[p.bf16_in ? 1 : 0][p.bf16_out ? 1 : 0], in->lds_bf16x2, nblocks / 2, a, stream);
    return;
  }
  launch_kernel(in->bf16[p.bf16_in ? 1 : 0][p.bf16_out ? 1 : 0], in->lds_bf16, nblocks, a, stream);
}

}  // namespace amd_dft
