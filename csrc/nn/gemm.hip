// bf16 GEMM with fused epilogue for the FourCastNet MLP / embed / head layers:
//   Y[m, n] = act( sum_k X[m, k] * W[n, k] + bias[n] ) (+ R[m, n])        (F.linear layout)
// X [M, K] and W [N, K] are both K-contiguous; Y [M, N] bf16; fp32 accumulation.
// Optional LayerNorm fold (p.ln_stats): the GEMM consumes the raw residual stream x and the
// caller passes W' = W * gamma (per k), c1[n] = sum_k W'[n,k], c2[n] = sum_k beta_k W[n,k] + bias;
// then LN(x) W^T + bias = rstd_m * (x W'^T - mean_m * c1) + c2 is applied in the epilogue.
//
// MI355X design (256 x 256 x 64 block tile, 512 threads, one workgroup per CU):
//  * computed as Y^T = W . X^T so that an MFMA accumulator holds 4 CONSECUTIVE output features of
//    one token: the epilogue adds a 4-wide bias vector and writes 8 contiguous bytes per lane;
//  * 8 waves as 2 (features, "wr") x 4 (tokens, "wc"), 128 x 64 outputs per wave on
//    v_mfma_f32_16x16x32_bf16 (8 x 4 accumulator tiles = 128 fp32 per lane);
//  * ping-pong schedule: the two wave groups (wr = 0 / 1, one wave of each per SIMD) run one
//    barrier apart, so on every SIMD one wave issues its LDS fragment reads and DMA while the
//    other one runs its MFMA cluster;
//  * each 64-deep K-tile is 2 phases (GEMM_HALF, default: one 64x64 half of the wave's output
//    per phase, 32 bf16 / 48 bf16x3 MFMAs) over 4 LDS regions of 16 KB, filled with
//    global_load_lds_dwordx4 (no VGPR round trip) one K-tile ahead: counted vmcnt, never 0 in the
//    main loop, raw s_barrier (no __syncthreads, which would drain the DMA).  The 4-phase
//    schedule (64x32 quadrants, 16 / 24 MFMAs per phase) remains for the persistent variant and
//    the gathered patch embedding (MODE 1); the 2-phase one measured 6-9 % faster on the bf16 and
//    3-5 % on the bf16x3 MLP GEMMs (profiles/gemm_half_r4.txt);
//  * region = 128 rows x 128 B with the 16-byte chunk XOR-swizzled by (row & 7): the DMA writes
//    lane-linear, so the swizzle is applied to the SOURCE address; fragment reads are
//    bank-conflict free for the ds_read_b128 lane groups;
//  * blockIdx -> tile remap keeps consecutive tiles (same token panel, different feature
//    panels) on one XCD so the token panel is served from that XCD's L2.
//
// fp32 mode (SPLIT, "bf16x3"): fp32 operands are carried as bf16 pairs a = a_hi + a_lo
// (a_hi = bf16(a), a_lo = bf16(a - a_hi); 16 significant bits) and the product is
// A_hi.B_hi + A_lo.B_hi + A_hi.B_lo with fp32 accumulation: relative error ~5e-6 per GEMM
// (fp32 FMA: ~3e-7, bf16: ~3e-3) at 3x the bf16 MFMA work, vs 16x for the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32 runs at 1/16 of the bf16 rate on gfx950).  Operand rows use the
// k32-interleaved split layout: every 32-deep k chunk is stored as [hi(32) | lo(32)]
// (physical column (k / 32) * 64 + part * 32 + k % 32, row length 2K), so a 128-byte region
// row of the pipeline below holds hi AND lo of one 32-deep K-tile: the same DMA, LDS images
// and fragment reads as the bf16 kernel (its k-step 0 / 1 fragments become the hi / lo
// fragments) feed 24 MFMAs per phase instead of 16 -- 2x the bf16 loads for 3x the MFMAs.
// Outputs: fp32 (OUT 1) or a split pair row in the same layout (OUT 2), ready to be the
// next GEMM's operand.  The LayerNorm fold works in split mode too (fc1 of the fp32 block reads
// the raw residual stream's split pairs written by the AFNO C2R epilogue; c1 is summed from the
// split weight pairs, so x W'^T - mean c1 cancels the mean exactly up to the split's 2^-17).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "../fft/dev_check.h"
#include "gelu.h"
#include "gemm.h"
#include "../ops/tuning.h"

namespace amd_dft {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kBF = 256;  // features per block (MFMA M)
constexpr int kBT = 256;  // tokens per block (MFMA N)
constexpr int kBK = 64;
constexpr int kThreads = 512;
constexpr int kRegion = 128 * 128;     // 128 rows x 128 B (64 bf16 of K)
constexpr int kStage = 4 * kRegion;    // one K-tile: 64 KB
constexpr int kLds = 2 * kStage;       // two K-tiles: 128 KB

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 v;
  v[0] = static_cast<__bf16>(a);
  v[1] = static_cast<__bf16>(b);
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 7)); }

// Regions of one K-tile stage (phase q of K-tile t reads region kReadRegion[q]):
//   R0: feature rows {0-63, 128-191}   -> A fragments, row group mi = 0 of each wave group
//   R1: token rows {64c + 0..31}       -> B fragments, ni = 0 of each token wave c
//   R2: token rows {64c + 32..63}      -> B fragments, ni = 1
//   R3: feature rows {64-127, 192-255} -> A fragments, mi = 1
template <int REG>
__device__ __forceinline__ int region_row(int r) {
  if constexpr (REG == 0) return (r >> 6) * 128 + (r & 63);
  else if constexpr (REG == 3) return (r >> 6) * 128 + 64 + (r & 63);
  else if constexpr (REG == 1) return (r >> 5) * 64 + (r & 31);
  else return (r >> 5) * 64 + 32 + (r & 31);
}

// DMA one region (2 x 1 KB per wave: 8 rows x 128 B per instruction, lane-linear in LDS).
// MODE 1 (patch embedding): the token operand is gathered straight from the image -- K-tile kt
// is channel kt and the 16-byte chunk c of a token row is patch row py = c (8 pixels), so the
// un-patchified tensor never exists.
// OPQ (persistent kernel): the lane offsets are recomputed at every call from an opaque lane id
// instead of being hoisted (held across the tile loop they spill: a few VALU ops per piece instead).
// ASM (persistent kernel, the next tile's DMA issued at the epilogue's start): the DMA as inline asm,
// invisible to the compiler's LDS-DMA hazard tracking -- which would otherwise put a vmcnt(0)
// before the epilogue's first staging write (different LDS bytes) and drain these very DMAs.  Every
// read of the regions they fill sits behind an explicit counted wait and a barrier.
#ifndef GEMM_DMA_DWORD
#define GEMM_DMA_DWORD 0  // timing-only ablation: bit R = region R's DMA moves 4 instead of 16 bytes per lane
#endif                    // (same instructions and vmcnt counts, a quarter of the bytes: power vs operand traffic)
// NPC: pieces (8-row instructions) per calling wave; wave = the caller's slot (rows 8 NPC wave ..)
template <int REG, int MODE, bool SPLIT, bool OPQ = false, bool ASM = false, int NPC = 2>
__device__ __forceinline__ void stage_region(const uint16_t* __restrict__ W, const uint16_t* __restrict__ X,
                                             int64_t K, int f0, int t0, int M, int kt, char* stage, int wave,
                                             int lane, const GemmLaunch& p, const int (&gb)[2][2]) {
  static_assert(NPC == 2 || MODE != 1, "gathered token rows: 2 pieces per wave");
  if constexpr (OPQ) asm volatile("" : "+v"(lane));
  char* dst = stage + REG * kRegion;
  // SPLIT: K-tile kt = logical k [32 kt, 32 kt + 32); its hi and lo halves are adjacent in the
  // k32-interleaved rows (row stride 2K), so the physical 64-element column block is kt * 64
  const int64_t ld = SPLIT ? 2 * K : K;
#pragma unroll
  for (int i = 0; i < NPC; ++i) {
    const int rb = (wave * NPC + i) * 8;
    const int row = rb + (lane >> 3), pos = lane & 7;
    const int chunk = pos ^ (row & 7);  // source swizzle = inverse of the read swizzle
    const int tr = region_row<REG>(row);
    const uint16_t* g;
    // operands as a wave-uniform 64-bit base + a 32-bit lane offset (the SGPR-base form of
    // global_load_lds: two fewer VGPRs per piece while the DMA issues inside an MFMA cluster)
    if constexpr (REG == 0 || REG == 3) {
      // feature rows past N (the ragged last panel of an N % 256 != 0 GEMM) read row N - 1: their
      // outputs are never stored; for full panels the clamp is a no-op
      const uint16_t* base = W + static_cast<int64_t>(f0) * ld + kt * kBK;  // uniform
      g = base + static_cast<uint32_t>(min(tr, p.N - 1 - f0) * static_cast<int>(ld) + chunk * 8);
    } else if constexpr (MODE == 1) {  // gb: this lane's token base offsets (32-bit, host-checked)
      if constexpr (SPLIT) {  // channel kt / 2, patch rows (kt & 1) * 4 + c % 4 of the hi / lo plane
        const int py = (kt & 1) * 4 + (chunk & 3);
        g = X + (chunk >= 4 ? p.x_lo : 0) + (gb[REG - 1][i] + ((kt >> 1) * (p.gh * 8) + py) * (p.gw * 8));
      } else {
        g = X + (gb[REG - 1][i] + (kt * (p.gh * 8) + chunk) * (p.gw * 8));
      }
    } else {
      const uint16_t* base = X + static_cast<int64_t>(t0) * ld + kt * kBK;  // uniform
      g = base + static_cast<uint32_t>(min(tr, M - 1 - t0) * static_cast<int>(ld) + chunk * 8);
    }
    if constexpr (ASM) {
      const uint32_t m0v = __builtin_amdgcn_readfirstlane(
          static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void*)(dst + rb * 128))));
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0v) : "memory", "m0");
    } else {
      if constexpr ((GEMM_DMA_DWORD >> REG) & 1)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(g), (lds_void*)(dst + rb * 128), 4, 0, 0);
      else
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(g), (lds_void*)(dst + rb * 128), 16, 0, 0);
    }
  }
}

// 4 A fragments (16 rows each) x 2 k-steps from region REG (rows wr*64 + i*16 + r16)
template <int REG>
__device__ __forceinline__ void read_a(bf16x8 (&a)[8], const char* stage, int wr, int r16, int kq) {
  const char* base = stage + REG * kRegion;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[s * 4 + i] = *reinterpret_cast<const bf16x8*>(base + swz(wr * 64 + i * 16 + r16, s * 4 + kq));
}
// 2 B fragments x 2 k-steps from region REG (rows wc*32 + j*16 + r16)
template <int REG>
__device__ __forceinline__ void read_b(bf16x8 (&b)[4], const char* stage, int wc, int r16, int kq) {
  const char* base = stage + REG * kRegion;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      b[s * 2 + j] = *reinterpret_cast<const bf16x8*>(base + swz(wc * 32 + j * 16 + r16, s * 4 + kq));
}

// bf16: k-steps 0 and 1.  SPLIT: fragments [0..3] / [4..7] of A and [0..1] / [2..3] of B are
// the hi / lo halves of one 32-deep K-tile: hi.hi + lo.hi + hi.lo, products outermost so
// consecutive MFMAs never chain on one accumulator
//
// DMA placement (GEMM_DMA_MID, experiment, default OFF): the phase's two global_load_lds pieces
// issued by this (MFMA) wave after the first product's MFMAs, in the issue slots an MFMA leaves
// free, instead of by the partner wave's read section.  Same pieces in the same order per wave,
// so every vmcnt count is unchanged.  Measured slower (profiles/gemm_dma_mid_r3.txt: bf16x3 fc1
// 5.99 vs 5.50-5.57 ms, fc2 5.10-5.15 vs 4.55 ms, bf16 fc2 2.20 vs 2.11 ms, ABAB on one box):
// the pieces then start half a phase later and the MFMA cluster itself stalls on their issue.
#ifndef GEMM_DMA_MID
#define GEMM_DMA_MID 0
#endif
// GEMM_HALF: the two-phase K-tile schedule of the main loop (32 / 48 MFMAs per section instead of
// 16 / 24) -- bit 0: bf16 instances, bit 1: bf16x3 (SPLIT) instances; 0 = the 4-phase schedule (A/B)
#ifndef GEMM_HALF
#define GEMM_HALF 3
#endif
// GEMM_HALF_BAL: the two-phase schedule's B-region DMA spread over wave group 1's two read sections
// (see half_batch in gemm_bf16_kernel); 0 (default) = all of it in the read-B section (the round-4 form)
#ifndef GEMM_HALF_BAL
#define GEMM_HALF_BAL 0  // 1: measured slower (profiles/gemm_dma_balance_r6.txt)
#endif
// GEMM_PRIO: wave priority in the main loop -- 2 (default): none (both waves of a SIMD at priority 0; the clusters
// stay between their barriers through barrier()'s sched_barrier fences); 0: s_setprio 1 around every MFMA cluster (the
// round 2-5 form); 1: one static s_setprio 1 for the younger wave group (waves 4-7, the VALU-arbitration loser;
// MI355X_MICROARCH.md "Two waves per SIMD" item 4).  profiles/gemm_prio_r6.txt: the x3 GEMMs 0.5-1.5 % faster without
// priorities, the fp32 step +0.25 % over six paired runs.
#ifndef GEMM_PRIO
#define GEMM_PRIO 2
#endif
template <int MI, int NI, bool SPLIT, class Mid>
__device__ __forceinline__ void mfma_quadrant(f32x4 (&acc)[8][4], const bf16x8 (&a)[8], const bf16x8 (&b)[4],
                                              Mid&& mid) {
  if (GEMM_PRIO == 0) __builtin_amdgcn_s_setprio(1);
  constexpr int NP = SPLIT ? 3 : 2;
#pragma unroll
  for (int s = 0; s < NP; ++s) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int sa = SPLIT ? (s == 1 ? 1 : 0) : s;  // SPLIT products: (hi, hi), (lo, hi), (hi, lo)
        const int sb = SPLIT ? (s == 2 ? 1 : 0) : s;
        acc[MI * 4 + i][NI * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[sa * 4 + i], b[sb * 2 + j],
                                                                                acc[MI * 4 + i][NI * 2 + j], 0, 0, 0);
      }
    if (GEMM_DMA_MID && s == 0) {
      __builtin_amdgcn_sched_barrier(0);
      mid();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (GEMM_PRIO == 0) __builtin_amdgcn_s_setprio(0);
}

// vmcnt(2n): the region issued 3 phases ago has landed, n younger regions may still fly
__device__ __forceinline__ void wait_regions(int n) {
  if (n >= 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

#ifdef AMD_DFT_GEMM_STAMPS
// slot 0 / 5: s_memrealtime at entry / exit; 1..4: s_memtime at entry, after the prologue,
// after the main loop, after the epilogue (thread 0 only, vector store)
#define GEMM_STAMP(slot, v) \
  do { if (threadIdx.x == 0) p.stamps[static_cast<int64_t>(blockIdx.x) * 8 + (slot)] = static_cast<long long>(v); } while (0)
#else
#define GEMM_STAMP(slot, v) do { } while (0)
#endif

// act(acc (LN-folded) + bias) of one accumulator tile (4 consecutive features of one token),
// as two packed pairs: every FMA / MUL / ADD issues once for two values (epilogue VALU is 60 %
// of a bf16x3 fc1 tile's epilogue).  Same operations and order as the per-value form.
template <int ACT, bool LN>
__device__ __forceinline__ void epi_act(const f32x4& a4, const float4& bias, const float4& c1, const float2& st,
                                        gelu_f2 (&v)[2]) {
  v[0] = gelu_f2{a4[0], a4[1]};
  v[1] = gelu_f2{a4[2], a4[3]};
  if constexpr (LN) {
    // rstd (acc - mean c1) + bias = rstd acc + (bias - rstd mean c1): two packed FMAs per pair
    // (st.x = -rstd * mean, st.y = rstd: the per-token operands folded once by the caller)
    v[0] = __builtin_elementwise_fma(gelu_f2(st.y), v[0],
                                     __builtin_elementwise_fma(gelu_f2(st.x), gelu_f2{c1.x, c1.y}, gelu_f2{bias.x, bias.y}));
    v[1] = __builtin_elementwise_fma(gelu_f2(st.y), v[1],
                                     __builtin_elementwise_fma(gelu_f2(st.x), gelu_f2{c1.z, c1.w}, gelu_f2{bias.z, bias.w}));
  } else {
    v[0] += gelu_f2{bias.x, bias.y};
    v[1] += gelu_f2{bias.z, bias.w};
  }
  if constexpr (ACT == 1) {
    v[0] = gelu_erf2(v[0]);
    v[1] = gelu_erf2(v[1]);
  } else if constexpr (ACT == 2) {
    v[0] = gelu_tanh2(v[0]);
    v[1] = gelu_tanh2(v[1]);
  } else if constexpr (ACT == 3) {
    v[0] = gelu_erf_fit2(v[0]);
    v[1] = gelu_erf_fit2(v[1]);
  }
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// sum over a 16-lane DPP row (every lane gets the total): quad swaps, then the 8- and 16-lane mirrors
__device__ __forceinline__ float row_sum16(float x) {
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xf, 0xf, false));  // row_half_mirror
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xf, 0xf, false));  // row_mirror
  return x;
}

// STATS (fp32 or bf16 output, LDS-staged epilogue): per token and 64-feature chunk of the output (bf16:
// the stored, rounded values) plus the per-channel p.stats_pre, the chunk's (mean, M2 = sum of squared deviations) into
// p.stats_part[t][chunk] -- the next LayerNorm's statistics without a pass over the output
// (merged per token by ln_stats_merge, Chan's formula)
//
// PERSIST (MODE 0, staged epilogue): one workgroup per CU walks the tiles vb, vb + grid, ...:
//   * the epilogue first DMAs the next tile's K-tile 0 into stage 0 (idle after the last K-tile,
//     which is odd: KT even) and R0 of its K-tile 1 into stage 1, then stages its outputs through
//     regions R1 / R2 of stage 1 only (4 KB per wave, 16-token quarters);
//   * vmcnt counts across the epilogue: it issues at least kEpiVm vector memory ops (residual
//     loads, stores, statistics) behind the prefetched regions, so the waits that let those
//     regions land allow that many younger ops in flight -- the stores drain while the next
//     tile's first MFMAs run (the epilogue's stores are unconditional, ragged tiles included);
//     the first tile's prologue waits for all of its DMAs, so the relaxed waits of phases 0-2 of
//     K-tile 0 are exact in every case;
//   * the main loop is the one-tile loop unchanged (its register budget is full: a version that
//     also streamed the next tile in under the last K-tile spilled its DMA addresses).
// It removes the per-tile workgroup turnaround (launch, prologue DMA latency, epilogue drain) of a
// grid of one tile per workgroup -- and measured 4-12 % SLOWER (profiles/gemm_persistent_r4.txt: the
// GEMMs run power-limited, the turnaround gaps were the cheap part), so it stays opt-in
// (MI_DFT_GEMM_PERSIST=1, bit-exact: tests/test_gemm_variants.py).
// NT: N % 256 != 0 -- the last feature panel is ragged (N % 64 == 0): its W rows past N are clamped in
// the DMA, its bias / c1 loads clamped, and the epilogue halves past N store nothing (wave-uniform).
template <int ACT, bool BIAS, int RES, bool LN, int MODE, bool SPLIT, int OUT, bool STATS = false, bool PERSIST = false,
          bool NT = false>
__global__ void __launch_bounds__(kThreads) gemm_bf16_kernel(GemmLaunch p) {
  static_assert(!PERSIST || MODE == 0, "persistent tiles: token-major operands and outputs only");
  static_assert(!NT || (!PERSIST && MODE != 2), "ragged feature panels: token-major, one tile per workgroup");
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [2 stages][4 regions]
  const uint16_t* __restrict__ W = p.w;
  const uint16_t* __restrict__ X = p.x;
  const int M = p.M, N = p.N, K = p.K;
  const int lane0 = threadIdx.x & 63;
  // PERSIST: the wave index as a scalar, so the DMA's LDS destinations are SGPR arithmetic instead
  // of hoisted VGPRs (which spilled)
  const int wave = PERSIST ? __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)) : static_cast<int>(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;  // 2 (features) x 4 (tokens)
  GEMM_STAMP(0, __builtin_amdgcn_s_memrealtime());
  GEMM_STAMP(1, __builtin_amdgcn_s_memtime());
  // ---- XCD-aware tile order (bijective for any tile count).  PERSIST: virtual workgroup
  // v = blockIdx + k grid (grid % 8 == 0, so v stays on blockIdx's XCD)
  const int tiles_f = NT ? (N + kBF - 1) / kBF : N / kBF;
  const int ntl = PERSIST ? p.ntiles : static_cast<int>(gridDim.x);
  auto tile_of = [&](int v, int& f0_, int& t0_) {
    const int q8 = ntl / 8, r8 = ntl % 8, xcd = v % 8;
    const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + v / 8;
    const int tt = lid / tiles_f, ft = lid - tt * tiles_f;  // token panel outer, feature panels inner
    f0_ = ft * kBF;
    t0_ = tt * kBT;
  };
  int vb = blockIdx.x, f0, t0;
  tile_of(vb, f0, t0);
  const int KT = SPLIT ? K / 32 : K / kBK;  // SPLIT: 32-deep logical K-tiles (hi | lo = 64 elements)
  AMD_DFT_DEV_CHECK((NT ? f0 < N && N % 64 == 0 : f0 + kBF <= N) && t0 < M && (SPLIT ? (K / 32) * 32 : (K / kBK) * kBK) == K && KT > 0,
                    "gemm_bf16_kernel");
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Linear phase index P = 4 t + q.  Phase P DMAs region (q+1) & 3 of K-tile tgt(P) into
  // stage tgt(P) & 1 and reads the region that phase P - 4 DMA'd.
  //   q = 0: R1(t+1)   q = 1: R2(t+1)   q = 2: R3(t+1)   q = 3: R0(t+2)
  auto tgt = [](int P) { return (P >> 2) + 1 + ((P & 3) == 3 ? 1 : 0); };
  auto issued = [&](int P) { return tgt(P) < KT ? 1 : 0; };
  // PERSIST: vector memory ops the staged epilogue issues at least (full tiles) after the next
  // tile's K-tile-0 / R0(1) DMA: per pass one store, the residual row (OUT 2: 2 loads), the statistics
  constexpr int kNitE = OUT == 1 ? 16 : 8;  // passes per half
  constexpr int kEpiVm = 2 * kNitE * ((OUT == 2 ? 2 : 1) + (RES ? (OUT == 2 ? 2 : 1) : 0) + (STATS ? 1 : 0));
  constexpr int kRelaxed = kEpiVm + 4 < 63 ? kEpiVm + 4 : 63;

  // MODE 1: per-lane token base offsets of the gathered image rows (regions 1, 2 x 2 pieces)
  int gb[2][2] = {{0, 0}, {0, 0}};
  if constexpr (MODE == 1) {
    const int hw = p.gh * p.gw, rowlen = p.gw * 8;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (wave * 2 + i) * 8 + (lane0 >> 3);
        const int tr = r == 0 ? region_row<1>(row) : region_row<2>(row);
        const int t = min(t0 + tr, M - 1);
        const int b = t / hw, rem = t - b * hw;
        const int ii = rem / p.gw, jj = rem - ii * p.gw;
        gb[r][i] = (b * p.gC * (p.gh * 8) + ii * 8) * rowlen + jj * 8;
      }
  }
  // HALF: two-phase K-tile schedule (see the main loop); wave group as a scalar for its branches
  constexpr bool HALF = ((GEMM_HALF >> (SPLIT ? 1 : 0)) & 1) && !PERSIST && MODE != 1;
  const int wrs = __builtin_amdgcn_readfirstlane(wr);
  if (GEMM_PRIO == 1 && wrs == 1) __builtin_amdgcn_s_setprio(1);  // wave-uniform (readfirstlane): a real branch
  // HALF batch(kt): R0 (each group its own feature rows) + R1 / R2 (all token rows, wave group 1 only).
  // BAL (GEMM_HALF_BAL): wave group 1 issues R2(kt) one section later, in its read-A section of K-tile
  // kt - 1 (ahead of that section's R3), instead of in the read-B section with R0 / R1: its sections
  // then carry 6 + 6 DMA pieces instead of 2 + 10, and no read section's DMA issue outlasts the partner
  // wave's MFMA cluster.  R2(kt)'s old contents (K-tile kt - 2) were last read in read-A(kt - 2) by both
  // groups; it lands before the read-B wait of K-tile kt - 1 (issued ahead of R3(kt), so that wait keeps
  // counting R3's two pieces as the only younger ones).
  constexpr bool BAL = HALF && GEMM_HALF_BAL;
  auto half_batch = [&](int kt, char* st, bool with_r2) {
    if constexpr (HALF) {
      stage_region<0, MODE, SPLIT>(W, X, K, f0, t0, M, kt, st, wave, lane0, p, gb);
      if (wrs == 1) {
        stage_region<1, MODE, SPLIT, false, false, 4>(W, X, K, f0, t0, M, kt, st, wave - 4, lane0, p, gb);
        if (with_r2) stage_region<2, MODE, SPLIT, false, false, 4>(W, X, K, f0, t0, M, kt, st, wave - 4, lane0, p, gb);
      }
    }
  };
  bf16x8 a0[8], a1[8], b0[4], b1[4];
  if constexpr (HALF) {
    // ---- prologue: batch(0), R3(0), batch(1) (BAL: batch(1) without R2(1), which read-A(0) issues)
    half_batch(0, smem, true);
    stage_region<3, MODE, SPLIT>(W, X, K, f0, t0, M, 0, smem, wave, lane0, p, gb);
    if (KT > 1) {
      half_batch(1, smem + kStage, !BAL);
      if (wrs == 1) wait_vm<BAL ? 8 : 12>();  // batch(0) landed; younger: R3(0) (2) + batch(1) (6 / 10 / 2)
      else wait_vm<4>();
    } else {
      wait_vm<2>();
    }
    barrier();
    if (wr == 1) barrier();  // stagger
  } else {
    // ---- prologue: R0(0) R1(0) R2(0) R3(0) R0(1) = phases -5..-1
    stage_region<0, MODE, SPLIT>(W, X, K, f0, t0, M, 0, smem, wave, lane0, p, gb);
    stage_region<1, MODE, SPLIT>(W, X, K, f0, t0, M, 0, smem, wave, lane0, p, gb);
    stage_region<2, MODE, SPLIT>(W, X, K, f0, t0, M, 0, smem, wave, lane0, p, gb);
    stage_region<3, MODE, SPLIT>(W, X, K, f0, t0, M, 0, smem, wave, lane0, p, gb);
    if (KT > 1) {
      stage_region<0, MODE, SPLIT>(W, X, K, f0, t0, M, 1, smem + kStage, wave, lane0, p, gb);
      if constexpr (PERSIST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K-tile 0 and R0(1) (see PERSIST)
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // R0(0), R1(0) landed
    } else {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    barrier();
    read_a<0>(a0, smem, wr, lane0 & 15, lane0 >> 4);
    if (wr == 1) barrier();  // stagger: wave group 1 runs one barrier behind group 0
  }
  if constexpr (!PERSIST) GEMM_STAMP(2, __builtin_amdgcn_s_memtime());

  for (;;) {  // PERSIST: one pass per tile (otherwise exactly one)
    // PERSIST: everything lane-derived (DMA offsets, output geometry) is re-derived per tile from
    // an opaque copy of the lane id -- hoisted out of the tile loop it would stay live through
    // the whole kernel and spill
    int lane = lane0;
    if constexpr (PERSIST) asm volatile("" : "+v"(lane));
    const int r16 = lane & 15, kq = lane >> 4;

    // ---- output geometry: lane holds features f..f+3 of token t for each (i, j) accumulator tile
    // (recomputed where used instead of held in registers across the main loop)
    auto tok = [&](int j) { return t0 + wc * 64 + j * 16 + r16; };
    auto tokc = [&](int j) { return min(tok(j), M - 1); };  // loads use clamped (valid) rows; stores check t < M
    auto out_off = [&](int i, int j) -> int64_t {
      const int f = f0 + wr * 128 + i * 16 + 4 * kq;
      const int t = tokc(j);
      if constexpr (MODE == 2) {  // un-patchify: feature f = (c, py, px), 4 consecutive px
        const int hw = p.sh * p.sw;
        const int bb = t / hw, rem = t - bb * hw;
        const int ii = rem / p.sw, jj = rem - ii * p.sw;
        return (static_cast<int64_t>(bb * p.sC + (f >> 6)) * (p.sh * 8) + ii * 8 + ((f >> 3) & 7)) * (p.sw * 8) + jj * 8 +
               (f & 7);
      } else {
        return static_cast<int64_t>(t) * N + f;
      }
    };
    auto res_off = [&](int i, int j) -> int64_t {
      const int f = f0 + wr * 128 + i * 16 + 4 * kq;
      if constexpr (MODE == 1) {
        if (p.res_rows > 0) return static_cast<int64_t>(tokc(j) % p.res_rows) * N + f;
      }
      return out_off(i, j);
    };
    typedef typename std::conditional<OUT != 0, float4, uint2>::type ResT;  // split modes: fp32 residual
    auto load_res = [&](int i, int j) -> ResT {
      if constexpr (OUT != 0) return *reinterpret_cast<const float4*>(static_cast<const float*>(p.residual) + res_off(i, j));
      else return *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p.residual) + res_off(i, j));
    };

#ifndef GEMM_STATS_ABL
#define GEMM_STATS_ABL 0  // timing-only (wrong partials): bit 0 = no per-row sweep, bit 1 = no partials store,
#endif                    // bit 2 = no write-back of the stored values into the staging slots
#ifndef GEMM_ABLATE
#define GEMM_ABLATE 0  // timing-only: bit 0 = no main-loop DMA, bit 1 = no main-loop fragment reads,
#endif                 // bit 2 = epilogue computes but skips its stores
    if constexpr (HALF) {
      // Two phases per K-tile instead of four: A(t) = feature rows mi 0 x all 4 token tiles (32 bf16 /
      // 48 bf16x3 MFMAs; reads R0, R1, R2), B(t) = mi 1 x all token tiles (reads R3, B fragments
      // kept).  Each wave alternates a read section and an MFMA section, the two wave groups one
      // barrier apart as above.  DMA: each group fills its own A rows of R0 / R3 (rows 64 wr ..), and
      // wave group 1 alone fills the B regions R1 / R2 (4 pieces per wave) -- so a region is never
      // refilled while the other group's reads of it may still be in flight:
      //   read A(t): wait R3(t) (issued at A(t-1)), DMA R3(t+1);
      //   read B(t): wait batch(t+1) = R0 (+ R1, R2) (issued at B(t-1)), DMA batch(t+2) into stage t & 1
      // (every region read by group 0 in section k was confirmed by both groups' waits in sections
      // <= k - 1; a refill of stage t & 1 starts two barriers after the last read of the old contents).
      for (int t = 0; t < KT; ++t) {
        char* cur = smem + (t & 1) * kStage;
        char* nxt = smem + ((t + 1) & 1) * kStage;
        const bool n1 = t + 1 < KT, n2 = t + 2 < KT;
        // ---- read A(t)
        if (n1) {
          if (wrs == 1) wait_vm<BAL ? 6 : 10>();  // R3(t) landed; younger: batch(t+1) (BAL: without R2(t+1))
          else wait_vm<2>();
          if (BAL && wrs == 1)  // R2(t+1) ahead of R3(t+1) (see half_batch)
            stage_region<2, MODE, SPLIT, false, false, 4>(W, X, K, f0, t0, M, t + 1, nxt, wave - 4, lane, p, gb);
          stage_region<3, MODE, SPLIT>(W, X, K, f0, t0, M, t + 1, nxt, wave, lane, p, gb);
        } else {
          wait_vm<0>();
        }
        read_a<0>(a0, cur, wr, r16, kq);
        read_b<1>(b0, cur, wc, r16, kq);
        read_b<2>(b1, cur, wc, r16, kq);
        barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        mfma_quadrant<0, 0, SPLIT>(acc, a0, b0, [] {});
        mfma_quadrant<0, 1, SPLIT>(acc, a0, b1, [] {});
        barrier();
        // ---- read B(t)
        if (n1) wait_vm<2>();  // batch(t+1) landed; younger: R3(t+1)
        if (n2) half_batch(t + 2, cur, !BAL);
        read_a<3>(a0, cur, wr, r16, kq);
        barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        mfma_quadrant<1, 0, SPLIT>(acc, a0, b0, [] {});
        mfma_quadrant<1, 1, SPLIT>(acc, a0, b1, [] {});
        barrier();
      }
    } else
    for (int t = 0; t < KT; ++t) {
      char* cur = smem + (t & 1) * kStage;
      char* nxt = smem + ((t + 1) & 1) * kStage;
      const int P = 4 * t;
      // ---- phase 0: quadrant (mi 0, ni 0)
      if (PERSIST && t == 0) wait_vm<kRelaxed>();
      else wait_regions(issued(P - 2) + issued(P - 1));
      auto dma0 = [&] {
        if (!(GEMM_ABLATE & 1) && issued(P)) stage_region<1, MODE, SPLIT, PERSIST>(W, X, K, f0, t0, M, t + 1, nxt, wave, lane, p, gb);
      };
      if (!GEMM_DMA_MID) dma0();
      if (!(GEMM_ABLATE & 2)) read_b<1>(b0, cur, wc, r16, kq);
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_quadrant<0, 0, SPLIT>(acc, a0, b0, dma0);
      barrier();
      // ---- phase 1: (0, 1)
      if (PERSIST && t == 0) wait_vm<kRelaxed>();
      else wait_regions(issued(P - 1) + issued(P));
      auto dma1 = [&] {
        if (!(GEMM_ABLATE & 1) && issued(P + 1)) stage_region<2, MODE, SPLIT, PERSIST>(W, X, K, f0, t0, M, t + 1, nxt, wave, lane, p, gb);
      };
      if (!GEMM_DMA_MID) dma1();
      if (!(GEMM_ABLATE & 2)) read_b<2>(b1, cur, wc, r16, kq);
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_quadrant<0, 1, SPLIT>(acc, a0, b1, dma1);
      barrier();
      // ---- phase 2: (1, 1)
      if (PERSIST && t == 0) wait_vm<kRelaxed>();
      else wait_regions(issued(P) + issued(P + 1));
      auto dma2 = [&] {
        if (!(GEMM_ABLATE & 1) && issued(P + 2)) stage_region<3, MODE, SPLIT, PERSIST>(W, X, K, f0, t0, M, t + 1, nxt, wave, lane, p, gb);
      };
      if (!GEMM_DMA_MID) dma2();
      if (!(GEMM_ABLATE & 2)) read_a<3>(a1, cur, wr, r16, kq);
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_quadrant<1, 1, SPLIT>(acc, a1, b1, dma2);
      barrier();
      // ---- phase 3: (1, 0); fragments A0 of K-tile t+1 are read here
      wait_regions(issued(P + 1) + issued(P + 2));
      auto dma3 = [&] {
        if (!(GEMM_ABLATE & 1) && issued(P + 3)) stage_region<0, MODE, SPLIT, PERSIST>(W, X, K, f0, t0, M, t + 2, cur, wave, lane, p, gb);
      };
      if (!GEMM_DMA_MID) dma3();
      if (!(GEMM_ABLATE & 2) && t + 1 < KT) read_a<0>(a0, nxt, wr, r16, kq);
      barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mfma_quadrant<1, 0, SPLIT>(acc, a1, b0, dma3);
      barrier();
    }
    if (wr == 0) barrier();  // re-align the two wave groups
    if constexpr (!PERSIST) GEMM_STAMP(3, __builtin_amdgcn_s_memtime());

    // ---- epilogue: lane holds features f..f+3 of token t for each (i, j) tile.
    // No load sits behind a per-element branch (hipcc would then wait for each one in turn:
    // 32 serialised round trips per wave, ~20 us per tile): bias / c1 / LN statistics are loaded
    // up front, residual rows from clamped (always valid) addresses two i-tiles at a time with
    // the next pair in flight, and only the stores are predicated on t < M.
    float4 bias4[8], c14[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int f = NT ? min(f0 + wr * 128 + i * 16 + 4 * kq, N - 4) : f0 + wr * 128 + i * 16 + 4 * kq;
      bias4[i] = BIAS ? *reinterpret_cast<const float4*>(p.bias + f) : make_float4(0.f, 0.f, 0.f, 0.f);
      c14[i] = LN ? *reinterpret_cast<const float4*>(p.ln_c1 + f) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float2 lst[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lst[j] = LN ? *reinterpret_cast<const float2*>(p.ln_stats + 2 * static_cast<int64_t>(tokc(j))) : make_float2(0.f, 1.f);
      lst[j].x = -lst[j].x * lst[j].y;  // (mean, rstd) -> (-rstd mean, rstd), epi_act's operands
    }
    if constexpr (MODE != 2) {  // token-major outputs (MODE 1 only gathers its B operand differently)
      if (PERSIST || !p.direct_epi) {
        // ---- LDS-staged epilogue (token-major outputs).  Writing straight from the MFMA layout
        // makes every store instruction touch 16 rows with 32-64 B each (partial lines; the
        // epilogue was 25 % of a bf16x3 fc1 tile and nearly all of it stores: profiles/
        // gemm_epilogue_r2.txt).  Instead each wave parks act(acc + bias) as fp32 in its own 16 KB
        // of the (now idle) stage buffers -- 64 tokens x 64 features per half, 16-byte chunks
        // XOR-swizzled by row -- and reads it back row-contiguous: 16 B per lane, whole 128-byte
        // lines per store instruction, the residual read the same coalesced way (prefetched
        // before the half is staged), then the bf16 / fp32 / split-pair conversion.
        // PERSIST: stage 0 and region R0 of stage 1 receive the next tile's K-tile 0 and R0 of its
        // K-tile 1, so each wave stages 16-token quarters in its 4 KB of regions R1 / R2 of stage 1
        // (same passes and stores, four staging rounds per half)
        // The next tile's DMAs are issued after the first staging writes (the compiler drains
        // every LDS DMA it knows of before the epilogue's first LDS write) and before any
        // epilogue load (so the compiler's own counted waits for those loads stay exact).
        barrier();  // every wave is past its last fragment read of the stage buffers
        int nf0 = 0, nt0 = 0;
        const bool has_next = PERSIST && vb + static_cast<int>(gridDim.x) < ntl;
        if constexpr (PERSIST) {
          if (has_next) tile_of(vb + static_cast<int>(gridDim.x), nf0, nt0);
        }
        auto next_dma = [&] {
          if (has_next) {
            stage_region<0, MODE, SPLIT, true, true>(W, X, K, nf0, nt0, M, 0, smem, wave, lane, p, gb);
            stage_region<1, MODE, SPLIT, true, true>(W, X, K, nf0, nt0, M, 0, smem, wave, lane, p, gb);
            stage_region<2, MODE, SPLIT, true, true>(W, X, K, nf0, nt0, M, 0, smem, wave, lane, p, gb);
            stage_region<3, MODE, SPLIT, true, true>(W, X, K, nf0, nt0, M, 0, smem, wave, lane, p, gb);
            stage_region<0, MODE, SPLIT, true, true>(W, X, K, nf0, nt0, M, 1, smem + kStage, wave, lane, p, gb);
          }
        };
        constexpr int SUB = PERSIST ? 4 : 1;  // token sub-blocks per half
        char* reg = PERSIST ? smem + kStage + kRegion + wave * (16 * 256) : smem + wave * (64 * 256);
        const int tbase = t0 + wc * 64;
        // OUT 0 / 2: a lane owns 8 consecutive features (OUT 2: writes their hi AND lo halves --
        // 16 B each into the k32-interleaved pair row), OUT 1: 4
        constexpr int LPR = OUT == 1 ? 16 : 8;    // lanes per token row
        constexpr int RPI = 64 / LPR;             // rows per pass
        constexpr int NIT = 64 / RPI;             // passes per half
        const int c = lane % LPR, rsub = lane / LPR;
        // residual per lane and pass: OUT 1 4 fp32, OUT 0 8 bf16, OUT 2 8 fp32
        struct F8 { float4 a, b; };
        // RES 2 (OUT 1): the residual as bf16x3 split pairs of x - m (k32-interleaved rows, c2r_ln_add_split's
        // pairs) plus the per-token shift m = p.res_mean[2 t]: x = m + (hi + lo), 2^-18 of |x - m| off
        // RES 3: plus the third split term p.res_lo2 [M, N] bf16 (x to ~2^-27 of |x - m|, below fp32 rounding)
        struct P4 { uint2 h, l; float m; };
        struct P6 { uint2 h, l, t; float m; };
        typedef typename std::conditional<
            OUT == 1, typename std::conditional<RES == 3, P6, typename std::conditional<RES == 2, P4, float4>::type>::type,
            typename std::conditional<OUT == 2, F8, uint4>::type>::type RT;
        static_assert(RES < 2 || (OUT == 1 && SPLIT), "split-pair residual: fp32 output of the bf16x3 GEMM");
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int fh = f0 + wr * 128 + h * 64;  // first feature of this half
          if constexpr (NT) {
            if (fh >= N) continue;  // past the ragged panel's last feature: wave-uniform, nothing to store
          }
          RT rr[RES ? NIT : 1];
          // residual rows are prefetched PD passes ahead of their use: all NIT before the half is
          // staged (OUT 0 / 1: 4 VGPRs per pass), half of them with bias / LN vectors live, 4 ahead
          // for OUT 2 (8 fp32 per pass: the whole half would hold 128 VGPRs beside the accumulators)
          // -- each of those spilled when the whole half was prefetched
          // RES 2 / 3 (5 / 7 VGPRs per pass): 4 / 2 passes ahead in the persistent form, 8 / 2 otherwise (deeper spilled)
          constexpr int PD = RES == 3 ? 2
                             : (OUT == 2 || PERSIST) ? 4
                             : RES == 2 ? NIT / 2
                                        : (BIAS || LN ? NIT / 2 : NIT);  // bias / c1 vectors hold 64 more VGPRs
          auto load_rr = [&](int it) {  // OUT 1: 4 fp32 features per lane; OUT 0: 8 bf16; OUT 2: 8 fp32
            int rt = min(tbase + it * RPI + rsub, M - 1);
            if constexpr (MODE == 1) {
              if (p.res_rows > 0) rt %= p.res_rows;  // position embedding broadcast over the batch
            }
            if constexpr (RES >= 2) {
              const int f = fh + 4 * c;  // 4 features in one 32-chunk: hi at (f / 32) 64 + f % 32, lo 32 after
              const uint16_t* rp = static_cast<const uint16_t*>(p.residual) + static_cast<int64_t>(rt) * (2 * N) +
                                   (f >> 5) * 64 + (f & 31);
              if constexpr (RES == 3)
                rr[it] = P6{*reinterpret_cast<const uint2*>(rp), *reinterpret_cast<const uint2*>(rp + 32),
                            *reinterpret_cast<const uint2*>(p.res_lo2 + static_cast<int64_t>(rt) * N + f),
                            p.res_mean[static_cast<int64_t>(rt) * 2]};
              else
                rr[it] = P4{*reinterpret_cast<const uint2*>(rp), *reinterpret_cast<const uint2*>(rp + 32),
                            p.res_mean[static_cast<int64_t>(rt) * 2]};
            } else if constexpr (OUT == 2) {
              const int64_t o = static_cast<int64_t>(rt) * N + fh + 8 * c;
              const float* rp = static_cast<const float*>(p.residual) + o;
              rr[it] = F8{*reinterpret_cast<const float4*>(rp), *reinterpret_cast<const float4*>(rp + 4)};
            } else {
              const int64_t o = static_cast<int64_t>(rt) * N + fh + (OUT == 1 ? 4 : 8) * c;
              if constexpr (OUT == 1) rr[it] = *reinterpret_cast<const float4*>(static_cast<const float*>(p.residual) + o);
              else rr[it] = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p.residual) + o);
            }
          };
          auto prefetch = [&] {
            if constexpr (RES) {
#pragma unroll
              for (int it = 0; it < PD; ++it) load_rr(it);
            }
          };
          float4 spre = make_float4(0.f, 0.f, 0.f, 0.f), spre2 = spre;  // OUT 0: the lane's 8 features
          if constexpr (STATS && !PERSIST) {  // ahead of the residual prefetch: the wait for its first row covers it
            // required (host: zeros if none)
            spre = *reinterpret_cast<const float4*>(p.stats_pre + fh + (OUT == 1 ? 4 : 8) * c);
            if constexpr (OUT == 0) spre2 = *reinterpret_cast<const float4*>(p.stats_pre + fh + 8 * c + 4);
          }
          if (!PERSIST || h > 0) prefetch();
#pragma unroll
          for (int sh = 0; sh < SUB; ++sh) {
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) {
              const int i = 4 * h + ii;
#pragma unroll
              for (int jj = 0; jj < 4 / SUB; ++jj) {
                const int j = sh * (4 / SUB) + jj;
                gelu_f2 v[2];
                epi_act<ACT, LN>(acc[i][j], bias4[i], c14[i], lst[j], v);
                const int row = jj * 16 + r16, ch = ii * 4 + kq;  // row & 15 == r16 in either layout
                *reinterpret_cast<float4*>(reg + row * 256 + ((ch ^ (row & 15)) << 4)) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
              }
            }
            if (sh == 0) {
              if constexpr (PERSIST) {
                if (h == 0) {
                  next_dma();
                  prefetch();
                }
              }
              if constexpr (STATS && PERSIST) {
                spre = *reinterpret_cast<const float4*>(p.stats_pre + fh + 4 * c);
              }
            }
#pragma unroll
            for (int it = sh * (NIT / SUB); it < (sh + 1) * (NIT / SUB); ++it) {
              if constexpr (RES && PD < NIT) {
                if (it + PD < NIT) load_rr(it + PD);
              }
              // Stores are unconditional: a token row t >= M (ragged last panel) was computed from
              // the clamped operand / residual / statistics rows of M - 1, so its values equal row
              // M - 1's bit for bit and it is stored there (a benign duplicate).  Predicated stores
              // would sit behind exec branches, and the compiler's vmcnt bookkeeping then assumes
              // they may not have issued: its waits for the residual prefetch came out as
              // vmcnt(4), i.e. waiting for the stores of two passes back to complete.
              const int row = it * RPI + rsub, t = min(tbase + row, M - 1);
              const char* rp = reg + (row - sh * (64 / SUB)) * 256;  // same row & 15 (64 / SUB is a multiple of 16)
              if constexpr (OUT == 1) {
                float4 v = *reinterpret_cast<const float4*>(rp + ((c ^ (row & 15)) << 4));
                if constexpr (RES >= 2) {
                  const auto& q = rr[it];
                  const auto bf = [](uint32_t w, bool hi) { return __uint_as_float(hi ? (w & 0xffff0000u) : (w << 16)); };
                  float r4[4] = {bf(q.h.x, false) + bf(q.l.x, false), bf(q.h.x, true) + bf(q.l.x, true),
                                 bf(q.h.y, false) + bf(q.l.y, false), bf(q.h.y, true) + bf(q.l.y, true)};
                  if constexpr (RES == 3) {
                    r4[0] += bf(q.t.x, false);
                    r4[1] += bf(q.t.x, true);
                    r4[2] += bf(q.t.y, false);
                    r4[3] += bf(q.t.y, true);
                  }
                  v.x += r4[0] + q.m;
                  v.y += r4[1] + q.m;
                  v.z += r4[2] + q.m;
                  v.w += r4[3] + q.m;
                } else if constexpr (RES) {
                  v.x += rr[it].x;
                  v.y += rr[it].y;
                  v.z += rr[it].z;
                  v.w += rr[it].w;
                }
                *reinterpret_cast<float4*>(static_cast<float*>(p.y) + static_cast<int64_t>(t) * N + fh + 4 * c) = v;
                if constexpr (STATS && !PERSIST) {
                  // v + pre back into the staging slot; the statistics are taken per row after the
                  // half's passes (one lane per token row: no cross-lane reductions)
                  *reinterpret_cast<float4*>(const_cast<char*>(rp) + ((c ^ (row & 15)) << 4)) =
                      make_float4(v.x + spre.x, v.y + spre.y, v.z + spre.z, v.w + spre.w);
                } else if constexpr (STATS) {  // the 16 lanes of this token row hold its 64 features fh .. fh + 63
                  const float w0 = v.x + spre.x, w1 = v.y + spre.y, w2 = v.z + spre.z, w3 = v.w + spre.w;
                  const float mean = row_sum16((w0 + w1) + (w2 + w3)) * (1.f / 64.f);
                  const float d0 = w0 - mean, d1 = w1 - mean, d2 = w2 - mean, d3 = w3 - mean;
                  const float m2 = row_sum16((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3));
                  if (c == 0)
                    *reinterpret_cast<float2*>(p.stats_part + (static_cast<int64_t>(t) * (N / 64) + fh / 64) * 2) =
                        make_float2(mean, m2);
                }
              } else {
                // lane = 8 features fl .. fl + 7 (staging chunks 2c, 2c + 1)
                const int fl = 8 * c;
                const float4 u0 = *reinterpret_cast<const float4*>(rp + (((fl >> 2) ^ (row & 15)) << 4));
                const float4 u1 = *reinterpret_cast<const float4*>(rp + ((((fl >> 2) + 1) ^ (row & 15)) << 4));
                float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
                if constexpr (OUT == 2 && RES) {
                  const float r8[8] = {rr[it].a.x, rr[it].a.y, rr[it].a.z, rr[it].a.w,
                                       rr[it].b.x, rr[it].b.y, rr[it].b.z, rr[it].b.w};
#pragma unroll
                  for (int k = 0; k < 8; ++k) v[k] += r8[k];
                }
                if constexpr (OUT == 0 && RES) {
                  const uint32_t rw[4] = {rr[it].x, rr[it].y, rr[it].z, rr[it].w};
#pragma unroll
                  for (int k = 0; k < 4; ++k) {
                    v[2 * k] += __uint_as_float(rw[k] << 16);
                    v[2 * k + 1] += __uint_as_float(rw[k] & 0xffff0000u);
                  }
                }
                uint4 w = make_uint4(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7]));
                if constexpr (OUT == 0) {
                  *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.y) + static_cast<int64_t>(t) * N + fh + fl) = w;
                  if constexpr (STATS && !PERSIST && !(GEMM_STATS_ABL & 4)) {
                    // the STORED (bf16-rounded) values + pre back into the two staging slots: the
                    // statistics describe exactly the tensor the next LayerNorm reads
                    // (the stored words pinned: unpacked as stored, not re-converted from v; + pre as
                    // packed adds)
                    uint32_t ws[4] = {w.x, w.y, w.z, w.w};
                    asm volatile("" : "+v"(ws[0]), "+v"(ws[1]), "+v"(ws[2]), "+v"(ws[3]));
                    const gelu_f2 pp[4] = {{spre.x, spre.y}, {spre.z, spre.w}, {spre2.x, spre2.y}, {spre2.z, spre2.w}};
                    gelu_f2 sv[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                      sv[k] = gelu_f2{__uint_as_float(ws[k] << 16), __uint_as_float(ws[k] & 0xffff0000u)} + pp[k];
                    char* rw = const_cast<char*>(rp);
                    *reinterpret_cast<float4*>(rw + (((fl >> 2) ^ (row & 15)) << 4)) = make_float4(sv[0].x, sv[0].y, sv[1].x, sv[1].y);
                    *reinterpret_cast<float4*>(rw + ((((fl >> 2) + 1) ^ (row & 15)) << 4)) =
                        make_float4(sv[2].x, sv[2].y, sv[3].x, sv[3].y);
                  }
                } else {  // split pair: hi = bf16(v), lo = bf16(v - hi), both stored by this lane
                  uint4 lw;
                  const uint32_t* wp = &w.x;
                  uint32_t* lp = &lw.x;
#pragma unroll
                  for (int k = 0; k < 4; ++k) {
                    const gelu_f2 hf = {__uint_as_float(wp[k] << 16), __uint_as_float(wp[k] & 0xffff0000u)};
                    const gelu_f2 d = gelu_f2{v[2 * k], v[2 * k + 1]} - hf;
                    lp[k] = pk_bf16(d.x, d.y);
                  }
                  const int f = fh + fl;
                  uint16_t* yr = static_cast<uint16_t*>(p.y) + static_cast<int64_t>(t) * (2 * N) + (f >> 5) * 64 + (f & 31);
                  *reinterpret_cast<uint4*>(yr) = w;
                  *reinterpret_cast<uint4*>(yr + 32) = lw;
                }
              }
            }
          }
          if constexpr (STATS && !PERSIST) {
            // lane l: token row l of this half, its 64 features (output + pre) from the staging slots
            // written above, in ONE sweep of shifted sums (shift = the row's first value, so the
            // M2 = S2 - S1^2 / 64 cancellation stays at a few std): no cross-lane reductions
            // (~45 VALU per pass as 16-lane DPP row sums: 9.6k cycles per tile, profiles/phases_r4.txt)
            const char* rl = reg + lane * 256;
            // (pairs as packed VALU: one v_pk_add / v_pk_fma per two values)
            const f32x4 q0 = *reinterpret_cast<const f32x4*>(rl + ((0 ^ (lane & 15)) << 4));
            const float sh = q0[0];
            const gelu_f2 shv = {sh, sh};
            gelu_f2 s1a = gelu_f2{q0[0], q0[1]} - shv, s1b = gelu_f2{q0[2], q0[3]} - shv;
            gelu_f2 s2a = s1a * s1a, s2b = s1b * s1b;
#pragma unroll
            for (int ch = 1; ch < ((GEMM_STATS_ABL & 1) ? 1 : 16); ++ch) {
              const f32x4 q = *reinterpret_cast<const f32x4*>(rl + ((ch ^ (lane & 15)) << 4));
              const gelu_f2 d0 = gelu_f2{q[0], q[1]} - shv, d1 = gelu_f2{q[2], q[3]} - shv;
              s1a += d0;
              s1b += d1;
              s2a = __builtin_elementwise_fma(d0, d0, s2a);
              s2b = __builtin_elementwise_fma(d1, d1, s2b);
            }
            const float t1 = (s1a.x + s1a.y) + (s1b.x + s1b.y), t2 = (s2a.x + s2a.y) + (s2b.x + s2b.y);
            const int t = min(tbase + lane, M - 1);  // rows >= M: bit-identical copies of row M - 1
            if (!(GEMM_STATS_ABL & 2) || t1 == 1234.5f)
            *reinterpret_cast<float2*>(p.stats_part + (static_cast<int64_t>(t) * (N / 64) + fh / 64) * 2) =
                make_float2(sh + t1 * (1.f / 64.f), fmaxf(t2 - t1 * t1 * (1.f / 64.f), 0.f));
          }
        }
        if constexpr (PERSIST) {
          if (!has_next) return;
          // ---- next tile: its K-tile 0 regions, R0 of its K-tile 1 and this epilogue's ops are in
          // flight.  Wait for R0 / R1 of K-tile 0' (read next: fragments A0 here, B in phase 0) --
          // younger: R2, R3, R0(1') (6) and the epilogue's >= kEpiVm ops -- and resume at phase 0
          // (relaxed waits in phases 0-2 of K-tile 0)
          wait_vm<kRelaxed + 2 < 63 ? kRelaxed + 2 : 63>();  // (ragged tiles store every pass too)
          barrier();  // every wave's pieces landed, every wave past its staging reads
          vb += gridDim.x;
          f0 = nf0;
          t0 = nt0;
          read_a<0>(a0, smem, wr, r16, kq);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (wr == 1) barrier();  // the stagger again
          continue;
        }
        GEMM_STAMP(4, __builtin_amdgcn_s_memtime());
        GEMM_STAMP(5, __builtin_amdgcn_s_memrealtime());
        return;
      }
    }
    if constexpr (MODE == 2 && !PERSIST) {  // MI_DFT_GEMM_EPI=direct: the scatter straight from the MFMA layout (A/B)
      if (!p.direct_epi) {
        // ---- un-patchify epilogue through LDS (the head GEMM).  Straight from the MFMA layout a lane
        // writes 4 pixels (8 / 16 B) of one (token, feature row) -- partial lines all over the image.
        // A half is one output channel's 64 (py, px) features: it is parked as fp32 like the
        // token-major epilogue above, then pass py has lane l write the 8 pixels px = 0..7 of token
        // tbase + l in image row (patch row) * 8 + py -- consecutive tokens of one patch row are
        // consecutive 8-pixel runs, so a store instruction covers whole lines (16 / 32 B per lane).
        // Token rows >= M (ragged last panel) hold bit-identical copies of row M - 1 and are stored
        // there (benign duplicates), so no store is predicated.  fp32 head 2468 -> 2277 us per call
        // (profiles/kernels_r4_final_fp32.txt vs session 18).
        barrier();  // every wave is past its last fragment read of the stage buffers
        char* reg = smem + wave * (64 * 256);
        const int t = min(t0 + wc * 64 + lane, M - 1);
        const int hw = p.sh * p.sw;
        const int bb = t / hw, rem = t - bb * hw;
        const int pi = rem / p.sw, pj = rem - pi * p.sw;
        const int64_t rowlen = static_cast<int64_t>(p.sw) * 8;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ch = (f0 + wr * 128 + h * 64) >> 6;  // output channel of this half
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) {
            const int i = 4 * h + ii;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              gelu_f2 v[2];
              epi_act<ACT, LN>(acc[i][j], bias4[i], c14[i], lst[j], v);
              const int row = j * 16 + r16, chk = ii * 4 + kq;
              *reinterpret_cast<float4*>(reg + row * 256 + ((chk ^ (row & 15)) << 4)) = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
            }
          }
          const char* rl = reg + lane * 256;  // this lane's token row of the staged half
          const int64_t obase = ((static_cast<int64_t>(bb) * p.sC + ch) * (p.sh * 8) + pi * 8) * rowlen + pj * 8;
#pragma unroll
          for (int py = 0; py < 8; ++py) {
            const float4 u0 = *reinterpret_cast<const float4*>(rl + (((2 * py) ^ (lane & 15)) << 4));
            const float4 u1 = *reinterpret_cast<const float4*>(rl + (((2 * py + 1) ^ (lane & 15)) << 4));
            const int64_t o = obase + py * rowlen;
            if constexpr (OUT == 1) {
              float* yp = static_cast<float*>(p.y) + o;
              *reinterpret_cast<float4*>(yp) = u0;
              *reinterpret_cast<float4*>(yp + 4) = u1;
            } else {
              *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.y) + o) =
                  make_uint4(pk_bf16(u0.x, u0.y), pk_bf16(u0.z, u0.w), pk_bf16(u1.x, u1.y), pk_bf16(u1.z, u1.w));
            }
          }
        }
        GEMM_STAMP(4, __builtin_amdgcn_s_memtime());
        GEMM_STAMP(5, __builtin_amdgcn_s_memrealtime());
        return;
      }
    }
    constexpr bool ERES = RES == 1;  // RES 2 (split-pair residual) only with the staged statistics epilogue (host-checked)
    ResT rq[ERES ? 2 : 1][2][4];  // [buffer][i of the pair][j]
    if constexpr (ERES) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) rq[0][ii][j] = load_res(ii, j);
    }
#pragma unroll
    for (int ip = 0; ip < 4; ++ip) {  // i-tile pairs (2 ip, 2 ip + 1)
      if constexpr (ERES) {
        if (ip + 1 < 4) {
#pragma unroll
          for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < 4; ++j) rq[(ip + 1) & 1][ii][j] = load_res(2 * (ip + 1) + ii, j);
        }
      }
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * ip + ii;
        const int f = f0 + wr * 128 + i * 16 + 4 * kq;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          gelu_f2 vp[2];
          epi_act<ACT, LN>(acc[i][j], bias4[i], c14[i], lst[j], vp);
          float v[4] = {vp[0].x, vp[0].y, vp[1].x, vp[1].y};
          if constexpr (ERES) {
            const ResT rr = rq[ip & 1][ii][j];
            if constexpr (OUT != 0) {  // fp32 residual (in place allowed: same lane reads, then writes)
              v[0] += rr.x;
              v[1] += rr.y;
              v[2] += rr.z;
              v[3] += rr.w;
            } else {
              v[0] += __uint_as_float(rr.x << 16);
              v[1] += __uint_as_float(rr.x & 0xffff0000u);
              v[2] += __uint_as_float(rr.y << 16);
              v[3] += __uint_as_float(rr.y & 0xffff0000u);
            }
          }
          if (tok(j) < M && !((GEMM_ABLATE & 4) && p.M > 0)) {
            if constexpr (OUT == 1) {
              *reinterpret_cast<float4*>(static_cast<float*>(p.y) + out_off(i, j)) = make_float4(v[0], v[1], v[2], v[3]);
            } else if constexpr (OUT == 2) {  // split pair row, k32-interleaved: features f..f+3 in one chunk
              const uint2 hw = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
              const gelu_f2 d0 = gelu_f2{v[0], v[1]} - gelu_f2{__uint_as_float(hw.x << 16), __uint_as_float(hw.x & 0xffff0000u)};
              const gelu_f2 d1 = gelu_f2{v[2], v[3]} - gelu_f2{__uint_as_float(hw.y << 16), __uint_as_float(hw.y & 0xffff0000u)};
              uint16_t* yr = static_cast<uint16_t*>(p.y) + static_cast<int64_t>(tok(j)) * (2 * N) + (f >> 5) * 64 + (f & 31);
              *reinterpret_cast<uint2*>(yr) = hw;
              *reinterpret_cast<uint2*>(yr + 32) = make_uint2(pk_bf16(d0.x, d0.y), pk_bf16(d1.x, d1.y));
            } else {
              *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p.y) + out_off(i, j)) =
                  make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
            }
          }
        }
      }
    }
    GEMM_STAMP(4, __builtin_amdgcn_s_memtime());
    GEMM_STAMP(5, __builtin_amdgcn_s_memrealtime());
    return;
  }  // tile loop
}

template <int ACT, bool BIAS, int RES, bool LN, int MODE, bool SPLIT, int OUT, bool STATS, bool PERSIST, bool NT>
void launch_kernel_nt(const GemmLaunch& p, hipStream_t st, dim3 grid) {
  auto kern = gemm_bf16_kernel<ACT, BIAS, RES, LN, MODE, SPLIT, OUT, STATS, PERSIST, NT>;
  // the dynamic-LDS limit is a per-device function attribute: set it once per (instance, device)
  static std::atomic<uint64_t> attr_done{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) throw std::runtime_error("amd_dft: gemm: bad device");
  if (!(attr_done.load(std::memory_order_acquire) & (uint64_t(1) << dev))) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: gemm attr: ") + hipGetErrorString(e));
    attr_done.fetch_or(uint64_t(1) << dev, std::memory_order_acq_rel);
  }
  hipLaunchKernelGGL(kern, grid, dim3(kThreads), kLds, st, p);
}

template <int ACT, bool BIAS, int RES, bool LN, int MODE, bool SPLIT, int OUT, bool STATS, bool PERSIST>
void launch_kernel(const GemmLaunch& p, hipStream_t st, dim3 grid) {
  if constexpr (!PERSIST && MODE != 2) {
    if (p.N % kBF != 0) {  // ragged last feature panel (launch_gemm: staged epilogue, one tile per workgroup)
      launch_kernel_nt<ACT, BIAS, RES, LN, MODE, SPLIT, OUT, STATS, false, true>(p, st, grid);
      return;
    }
  }
  if (p.N % kBF != 0) throw std::runtime_error("amd_dft: gemm: N % 256 != 0 needs a token-major, non-persistent GEMM");
  launch_kernel_nt<ACT, BIAS, RES, LN, MODE, SPLIT, OUT, STATS, PERSIST, false>(p, st, grid);
}

// CAN_PERSIST: the instance has a persistent variant (the fp32 block's GEMMs); p.ntiles > 0 (set by
// launch_gemm, MI_DFT_GEMM_PERSIST=1) selects it with grid = workgroups, else one tile per workgroup
template <int ACT, bool BIAS, int RES, bool LN, int MODE, bool SPLIT, int OUT, bool STATS = false, bool CAN_PERSIST = false>
void launch_one(const GemmLaunch& p, hipStream_t st, dim3 grid) {
  if constexpr (CAN_PERSIST) {
    if (p.ntiles > 0) {
      launch_kernel<ACT, BIAS, RES, LN, MODE, SPLIT, OUT, STATS, true>(p, st, grid);
      return;
    }
  }
  if (p.ntiles > 0) {  // no persistent variant of this instance: one workgroup per tile
    GemmLaunch q = p;
    q.ntiles = 0;
    launch_kernel<ACT, BIAS, RES, LN, MODE, SPLIT, OUT, STATS, false>(q, st, dim3(static_cast<uint32_t>(p.ntiles)));
    return;
  }
  launch_kernel<ACT, BIAS, RES, LN, MODE, SPLIT, OUT, STATS, false>(p, st, grid);
}

// bf16 path: every (act, bias, residual, LN) combination of the plain GEMM
// (the bf16 block's forms -- LN-folded fc1, fc2 + residual -- have persistent variants)
template <int ACT, bool BIAS, bool RES>
void launch_ln(const GemmLaunch& p, hipStream_t st, dim3 grid) {
  if constexpr (RES && ACT == 0 && !BIAS) {
    if (p.stats_part) {  // fc2 of the bf16 block: + the next LayerNorm's partial statistics (staged epilogue)
      if (p.ln_stats || p.direct_epi || !p.stats_pre)
        throw std::runtime_error("amd_dft: gemm: bf16 statistics need the staged epilogue, stats_pre and no LayerNorm fold");
      launch_one<0, false, true, false, 0, false, 0, true>(p, st, grid);
      return;
    }
  }
  if (p.stats_part) throw std::runtime_error("amd_dft: gemm: output statistics only with a residual, no activation / bias");
  if (p.ln_stats) launch_one<ACT, BIAS, RES, true, 0, false, 0, false, !RES>(p, st, grid);
  else launch_one<ACT, BIAS, RES, false, 0, false, 0, false, RES>(p, st, grid);
}

template <int ACT, bool BIAS>
void launch_res(const GemmLaunch& p, hipStream_t st, dim3 grid) {
  if (p.residual) launch_ln<ACT, BIAS, true>(p, st, grid);
  else launch_ln<ACT, BIAS, false>(p, st, grid);
}

// split (bf16x3) path: fp32 output (+ fp32 residual) or split-pair output (no residual)
template <int ACT, bool BIAS>
void launch_split(const GemmLaunch& p, hipStream_t st, dim3 grid) {
  if (p.ln_stats) {  // fc1 of the fp32 block: LayerNorm folded in (raw residual-stream pairs), split-pair output
    if (p.out != 2 || p.residual) throw std::runtime_error("amd_dft: gemm: a split LayerNorm fold writes split pairs, no residual");
    launch_one<ACT, BIAS, false, true, 0, true, 2, false, true>(p, st, grid);
    return;
  }
  if (p.out == 2) {
    if (p.residual) {  // last fp32 block: x + h W2^T straight to the head GEMM's split-pair operand
      if constexpr (ACT == 0 && !BIAS) {
        launch_one<0, false, true, false, 0, true, 2, false, true>(p, st, grid);
      } else {
        throw std::runtime_error("amd_dft: gemm: a split-pair output takes a residual only without activation and bias");
      }
      return;
    }
    launch_one<ACT, BIAS, false, false, 0, true, 2>(p, st, grid);
  } else if (p.residual && p.stats_part) {  // fc2 of the fp32 block: + next LayerNorm's partial statistics
    if (!p.stats_pre) throw std::runtime_error("amd_dft: gemm: statistics need stats_pre (zeros when there is none)");
    if constexpr (ACT == 0 && !BIAS) {
      if (p.direct_epi) throw std::runtime_error("amd_dft: gemm: statistics need the LDS-staged epilogue");
      if (p.res_mean && p.res_lo2) launch_one<ACT, BIAS, 3, false, 0, true, 1, true, true>(p, st, grid);
      else if (p.res_mean) launch_one<ACT, BIAS, 2, false, 0, true, 1, true, true>(p, st, grid);
      else launch_one<ACT, BIAS, true, false, 0, true, 1, true, true>(p, st, grid);
    } else {
      throw std::runtime_error("amd_dft: gemm: output statistics only without activation and bias");
    }
  } else if (p.residual) {
    launch_one<ACT, BIAS, true, false, 0, true, 1>(p, st, grid);
  } else {
    launch_one<ACT, BIAS, false, false, 0, true, 1>(p, st, grid);
  }
}

void throw_last(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: ") + what + ": " + hipGetErrorString(e));
}

}  // namespace

// N: whole 256-feature panels, or a ragged last panel of 64-feature halves (N % 64 == 0; token-major
// outputs); K: whole 64-deep K-tiles
bool gemm_supported(int64_t M, int64_t N, int64_t K) {
  return M >= 1 && N >= 64 && N % 64 == 0 && K % kBK == 0 && K >= kBK && M < (int64_t(1) << 31) &&
         N * K < (int64_t(1) << 31);
}
// logical K of a split (bf16x3) GEMM: 32-deep K-tiles, at least 2 (the pipeline prologue)
static bool split_k_ok(int64_t K) { return K % 32 == 0 && K >= 64; }

// MI_DFT_GEMM_EPI=direct: the token-major (MODE 0 / 1) epilogue stores straight from the MFMA layout (A/B only)
static int gemm_direct_epi() {
  static const int v = [] {
    const char* e = tuning_env("MI_DFT_GEMM_EPI");
    return (e && std::string(e) == "direct") ? 1 : 0;
  }();
  return v;
}

// MI_DFT_GEMM_PERSIST=1: the FourCastNet block GEMMs on a persistent grid (gemm_bf16_kernel PERSIST; A/B)
static int gemm_persist() {
  static const int v = [] {
    const char* e = tuning_env("MI_DFT_GEMM_PERSIST");
    return (e && std::string(e) == "1") ? 1 : 0;
  }();
  return v;
}

// persistent grid: one workgroup per CU (kLds = 128 KB), a multiple of 8 so that a workgroup's
// virtual indices stay on its XCD
static int persist_grid() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cache[dev] = cus / 8 * 8 > 0 ? cus / 8 * 8 : 8;
  }
  return cache[dev];
}

void launch_gemm(const GemmLaunch& p_, void* stream) {
  if (!gemm_supported(p_.M, p_.N, p_.K)) throw std::runtime_error("amd_dft: gemm: needs N % 64 == 0, K % 64 == 0");
  if (p_.ln_stats && !p_.ln_c1) throw std::runtime_error("amd_dft: gemm: LayerNorm fold needs c1");
  if (p_.out < 0 || p_.out > 2 || (p_.out != 0) != (p_.split != 0))
    throw std::runtime_error("amd_dft: gemm: fp32 / split-pair outputs come with split (bf16x3) operands only");
  if (p_.split && !split_k_ok(p_.K)) throw std::runtime_error("amd_dft: gemm: split mode needs K % 32 == 0, K >= 64");
  GemmLaunch p = p_;
  const bool ragged = p.N % kBF != 0;
  if (ragged && p.sC > 0) throw std::runtime_error("amd_dft: gemm: the un-patchify scatter needs N % 256 == 0");
  p.direct_epi = ragged ? 0 : gemm_direct_epi();  // the ragged panel's epilogue is the staged one
  const int64_t nwg = ((p.M + kBT - 1) / kBT) * ((p.N + kBF - 1) / kBF);
  dim3 grid(static_cast<uint32_t>(nwg));
  p.ntiles = 0;
  // persistent variant: token-major GEMMs with an even K-tile count (the next tile's K-tile 0 lands
  // in stage 0) and more tiles than workgroups; instances without one fall back to a full grid
  if (gemm_persist() && !ragged && !p.direct_epi && p.gC == 0 && p.sC == 0 && (p.split ? p.K / 32 : p.K / kBK) % 2 == 0 &&
      nwg > persist_grid()) {
    p.ntiles = static_cast<int>(nwg);
    grid = dim3(static_cast<uint32_t>(persist_grid()));
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool bias = p.bias != nullptr;
  if (p.gC > 0 || p.sC > 0) {  // patch-embedding gather / un-patchify scatter (no activation, no LN)
    if (p.act != 0 || p.ln_stats) throw std::runtime_error("amd_dft: gemm: patch modes take no activation / LN");
    if (p.split && p.out != 1) throw std::runtime_error("amd_dft: gemm: split patch modes write fp32");
    if (p.gC > 0) {
      if (p.K != p.gC * 64 || static_cast<int64_t>(p.M) % (static_cast<int64_t>(p.gh) * p.gw) != 0)
        throw std::runtime_error("amd_dft: gemm: patch gather needs K = C*64 and M = B*h*w");
      if (static_cast<int64_t>(p.M) * p.K >= (int64_t(1) << 31) || (p.split && p.x_lo + static_cast<int64_t>(p.M) * p.K >= (int64_t(1) << 31)))
        throw std::runtime_error("amd_dft: gemm: patch gather uses 32-bit offsets");
      if (p.split) {
        if (bias && p.residual) launch_one<0, true, true, false, 1, true, 1>(p, st, grid);
        else if (bias) launch_one<0, true, false, false, 1, true, 1>(p, st, grid);
        else if (p.residual) launch_one<0, false, true, false, 1, true, 1>(p, st, grid);
        else launch_one<0, false, false, false, 1, true, 1>(p, st, grid);
      } else {
        if (bias && p.residual) launch_one<0, true, true, false, 1, false, 0>(p, st, grid);
        else if (bias) launch_one<0, true, false, false, 1, false, 0>(p, st, grid);
        else if (p.residual) launch_one<0, false, true, false, 1, false, 0>(p, st, grid);
        else launch_one<0, false, false, false, 1, false, 0>(p, st, grid);
      }
    } else {
      if (p.N != p.sC * 64 || p.residual || static_cast<int64_t>(p.M) % (static_cast<int64_t>(p.sh) * p.sw) != 0)
        throw std::runtime_error("amd_dft: gemm: un-patchify scatter needs N = C*64, M = B*h*w, no residual");
      if (p.split) {
        if (bias) launch_one<0, true, false, false, 2, true, 1>(p, st, grid);
        else launch_one<0, false, false, false, 2, true, 1>(p, st, grid);
      } else {
        if (bias) launch_one<0, true, false, false, 2, false, 0>(p, st, grid);
        else launch_one<0, false, false, false, 2, false, 0>(p, st, grid);
      }
    }
    throw_last("gemm launch");
    return;
  }
  if (p.split) {
    if (p.act == 2 || p.act == 3)
      throw std::runtime_error("amd_dft: gemm: the tanh / fitted GELU forms are bf16-path options (split GEMMs: act 1)");
    if (p.act == 1) {
      if (bias) launch_split<1, true>(p, st, grid);
      else launch_split<1, false>(p, st, grid);
    } else {
      if (bias) launch_split<0, true>(p, st, grid);
      else launch_split<0, false>(p, st, grid);
    }
  } else if (p.act == 1) {
    if (bias) launch_res<1, true>(p, st, grid);
    else launch_res<1, false>(p, st, grid);
  } else if (p.act == 2) {  // tanh-form GELU (the bf16 path's option, see gelu.h)
    if (bias) launch_res<2, true>(p, st, grid);
    else launch_res<2, false>(p, st, grid);
  } else if (p.act == 3) {  // erf GELU at bf16-output resolution (gelu.h: gelu_erf_fit)
    if (bias) launch_res<3, true>(p, st, grid);
    else launch_res<3, false>(p, st, grid);
  } else {
    if (bias) launch_res<0, true>(p, st, grid);
    else launch_res<0, false>(p, st, grid);
  }
  throw_last("gemm launch");
}

}  // namespace amd_dft
