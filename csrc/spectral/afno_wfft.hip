// AFNO W-direction transforms with LayerNorm fused into their IO (FourCastNet 90 x 180 token
// grid, channel-last [B, H, W=180, C] bf16).  Two kernels per block:
//
//   afno_w_r2c_ln : X[o, k, c] = scale * sum_w LN1(x'[o, w, :])[c] e^{-2 pi i k w / 180},  k < KM
//   afno_w_c2r_ln : y[o, w, c] = scale * irfft_w(Y[o, :, c]) + x'[o, w, c] + LN1(x')[o, w, c]
//
// with x' = x + pre (pre = the previous block's fc2 bias, carried per channel), o = (b, h) and
// per-token LayerNorm statistics from ln_stats.  Same math as the generic fixed-kernel path
// (fft_fixed_impl.h, NADD = 3) but laid out for the memory system:
//  * a lane owns 4 consecutive channels = 2 packed real pairs (z = x_c + i x_{c+1}): every
//    global access is an 8- or 16-byte vector (the generic column kernel moves 4 bytes per
//    lane); 16 lanes cover 64 channels = one full 128-byte line per row;
//  * 180 = 12 x 15 Cooley-Tukey in two register passes: pass 0 (12-point DFTs over
//    n = n2 + 15 n1, one thread per n2, straight from global) and pass 1 (15-point DFTs, one
//    thread per k1) with one LDS transpose between them; the C2R output and its addends
//    stream straight from registers to global;
//  * the C2R input is the pruned half spectrum: which of the 12 pass-0 inputs can be non-zero
//    is resolved at compile time from KM (6 of 12 loads at KM = 46), the rest are constants.
//  * fp32 instantiation (F32, the fp32 FourCastNet path): fp32 residual stream and spectrum,
//    fp32 LDS staging, addends loaded to registers (the bf16 LDS image of the x tile would not
//    fit beside an fp32 staging buffer at 3 workgroups per CU).
// Reference: the AFNO filter runs rfft2/irfft2 on the whole [B, C, H, W] tensor after a
// separate LayerNorm kernel (FourCastNet AFNO2D; this repo's SURVEY.md §2.5 K5/K1e).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "../fft/dev_check.h"
#include "../fft/radix.h"
#include "spectral.h"
#include "w180_table.h"

namespace amd_dft {
namespace {

constexpr int kL = 180, kA = 12, kB = 15;  // n = kB * n1 + n2, k = k1 + kA * k2
constexpr int kPPL = 2;                     // packed pairs per lane (4 channels)
constexpr int kCh = 2 * kPPL;               // channels per lane
#ifndef AFNO_W_G
#define AFNO_W_G 16
#endif
constexpr int kG = AFNO_W_G;                // lanes per row (16: 64 channels / workgroup)
constexpr int kSlab = kCh * kG;             // 64
constexpr int kPairs = kPPL * kG;           // packed pairs per workgroup
constexpr int kPitch = kPairs + 2;          // float2 per LDS position (+16 B: spreads the k1 stride)
constexpr int kThreads = kB * kG;           // 240
#ifndef AFNO_C2R_XLDS
#define AFNO_C2R_XLDS 1  // C2R: residual tile + stats DMA'd into LDS at kernel start, fp16 FFT staging
#endif
// C2R addend image in LDS: [x tile: 180 positions x 128 B | stats: 180 x 8 B | pad], DMA'd
// (global_load_lds, no VGPRs) in 7 rounds of 3 full waves x 1 KB + the 48-lane wave x 768 B --
// the same instruction count in every wave and no branches.  Issued just BEFORE the spectrum
// loads: the compiler treats LDS DMA and plain loads as unordered and waits vmcnt(0) before
// the first use of the spectrum anyway, so both transfers share one memory round trip (the
// addends used to be a second, dependent one after pass 0).
constexpr int kXBytes = kL * 128, kSBytes = kL * 8;
constexpr int kRound = 3 * 1024 + 768, kRounds = (kXBytes + kSBytes + kRound - 1) / kRound;  // 7
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void unpack4(uint2 u, float (&f)[4]) {
  f[0] = __uint_as_float(u.x << 16);
  f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16);
  f[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ uint32_t bfpack(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 v;
  v[0] = static_cast<__bf16>(a);
  v[1] = static_cast<__bf16>(b);
  return __builtin_bit_cast(uint32_t, v);
}

struct WArgs {
  const void* x;         // [O, 180, C] bf16 / fp32 (stored residual stream)
  const float2* stats;   // [O, 180] (mean, rstd) of x'
  const float* gamma;    // [C]
  const float* beta;     // [C]
  const float* pre;      // [C] or nullptr
  const void* spec;      // C2R input [O, KM, C, 2] bf16 / fp32
  void* out;             // R2C: [O, KM, C, 2]; C2R: [O, 180, C]
  uint16_t* pairs;       // C2R, SPLIT: [O * 180, 2C] bf16 split pairs of out - mean(x) (stats .x)
  float* part;           // C2R, SPLIT / PART: [O * 180, C / 64, 2] (mean, M2) of out per 64-channel slab
  uint16_t* lo2;         // C2R, SPLIT, optional: [O * 180, C] bf16(out - mean(x) - (hi + lo))
  int C, nslab;
  float scale;
};

struct ChanParams {
  float g[kCh], b[kCh], p[kCh];
};

__device__ __forceinline__ void load_params(const WArgs& a, int c0, ChanParams& cp) {
  const float4 g4 = *reinterpret_cast<const float4*>(a.gamma + c0);
  const float4 b4 = *reinterpret_cast<const float4*>(a.beta + c0);
  const float4 p4 = a.pre ? *reinterpret_cast<const float4*>(a.pre + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
  cp.g[0] = g4.x; cp.g[1] = g4.y; cp.g[2] = g4.z; cp.g[3] = g4.w;
  cp.b[0] = b4.x; cp.b[1] = b4.y; cp.b[2] = b4.z; cp.b[3] = b4.w;
  cp.p[0] = p4.x; cp.p[1] = p4.y; cp.p[2] = p4.z; cp.p[3] = p4.w;
}

// x' (4 channels) and LN(x') of one token
__device__ __forceinline__ void ln4(const uint2 raw, const float2 st, const ChanParams& cp, float (&xp)[kCh],
                                    float (&h)[kCh]) {
  unpack4(raw, xp);
#pragma unroll
  for (int i = 0; i < kCh; ++i) {
    xp[i] += cp.p[i];
    h[i] = (xp[i] - st.x) * st.y * cp.g[i] + cp.b[i];
  }
}

// 4 consecutive channels of one token, bf16 (8 bytes) or fp32 (16 bytes); off in elements
template <bool F32>
__device__ __forceinline__ void ldx4(const void* base, int64_t off, float (&f)[4]) {
  if constexpr (F32) {
    const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(base) + off);
    f[0] = q.x; f[1] = q.y; f[2] = q.z; f[3] = q.w;
  } else {
    unpack4(*reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(base) + off), f);
  }
}
template <bool F32>
__device__ __forceinline__ void stx4(void* base, int64_t off, float a, float b, float c, float d) {
  if constexpr (F32) {
    *reinterpret_cast<float4*>(static_cast<float*>(base) + off) = make_float4(a, b, c, d);
  } else {
    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(base) + off) = make_uint2(bfpack(a, b), bfpack(c, d));
  }
}
__device__ __forceinline__ void ln4f(float (&xp)[kCh], const float2 st, const ChanParams& cp, float (&h)[kCh]) {
#pragma unroll
  for (int i = 0; i < kCh; ++i) {
    xp[i] += cp.p[i];
    h[i] = (xp[i] - st.x) * st.y * cp.g[i] + cp.b[i];
  }
}

// LDS image of one position: kPitch slots per position, a lane's 2 pairs in slots 2g, 2g+1.
// fp32 (float2 slots) or fp16 (h2_t slots: half the bytes -> twice the workgroups per CU).
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_pair(float2* l, int i, float2 a, float2 b) {
  *reinterpret_cast<float4*>(l + i) = make_float4(a.x, a.y, b.x, b.y);
}
__device__ __forceinline__ void st_pair(h2_t* l, int i, float2 a, float2 b) {
  *reinterpret_cast<h4_t*>(l + i) = h4_t{static_cast<_Float16>(a.x), static_cast<_Float16>(a.y),
                                         static_cast<_Float16>(b.x), static_cast<_Float16>(b.y)};
}
__device__ __forceinline__ void ld_pair(const float2* l, int i, float2& a, float2& b) {
  const float4 q = *reinterpret_cast<const float4*>(l + i);
  a = make_float2(q.x, q.y);
  b = make_float2(q.z, q.w);
}
__device__ __forceinline__ void ld_pair(const h2_t* l, int i, float2& a, float2& b) {
  const h4_t q = *reinterpret_cast<const h4_t*>(l + i);
  a = make_float2(static_cast<float>(q[0]), static_cast<float>(q[1]));
  b = make_float2(static_cast<float>(q[2]), static_cast<float>(q[3]));
}

// pass 0 epilogue: 12-point DFTs, twiddle W_180^{n2 k1}, store s[k1] at LDS position k1 * 15 + n2
template <class T>
__device__ __forceinline__ void pass0_store(cpair (&v)[kA], int n2, int g, T* lds) {
  Dft<kA>::run(v);
#pragma unroll
  for (int k1 = 0; k1 < kA; ++k1) {
    const cpair t = k1 == 0 ? v[0] : c_mul(v[k1], kW180[n2 * k1]);  // n2 * k1 <= 154
    st_pair(lds, (k1 * kB + n2) * kPitch + kPPL * g, cpair_lo(t), cpair_hi(t));
  }
}

// pass 1: 15-point DFTs of row k1; result u[p][k2] = X[k1 + 12 k2]
template <class T>
__device__ __forceinline__ void pass1(int k1, int g, const T* lds, cpair (&u)[kB]) {
#pragma unroll
  for (int n2 = 0; n2 < kB; ++n2) {
    float2 a, b;
    ld_pair(lds, (k1 * kB + n2) * kPitch + kPPL * g, a, b);
    u[n2] = make_cpair(a, b);
  }
  Dft<kB>::run(u);
}

template <int KM, bool F32>
__global__ void __launch_bounds__(kThreads) afno_w_r2c_ln_kernel(const WArgs a) {
  // bf16 output: fp16 staging (24.5 KB -> 6 workgroups per CU); fp32: fp32 staging (49 KB)
  using ST = typename std::conditional<F32, float2, h2_t>::type;
  __shared__ __attribute__((aligned(16))) ST lds[kL * kPitch];
  const int o = blockIdx.x / a.nslab, slab = blockIdx.x - o * a.nslab;
  AMD_DFT_DEV_CHECK((slab + 1) * kSlab <= a.C, "afno_w_kernel");
  const int g = threadIdx.x % kG, n2 = threadIdx.x / kG;
  const int c0 = slab * kSlab + kCh * g;
  const int C = a.C;
  // workgroup-uniform bases + 32-bit lane offsets (SGPR base + VGPR offset addressing)
  const int64_t xbase = static_cast<int64_t>(o) * kL * C + slab * kSlab;
  const void* xb = F32 ? static_cast<const void*>(static_cast<const float*>(a.x) + xbase)
                       : static_cast<const void*>(static_cast<const uint16_t*>(a.x) + xbase);
  const float2* st = a.stats + static_cast<int64_t>(o) * kL;
  const int lo = n2 * C + kCh * g;
  // ---- pass 0: n = n2 + 15 n1 straight from global, LayerNorm on load
  using Raw = typename std::conditional<F32, float4, uint2>::type;  // raw until use (bf16: 2 VGPRs)
  Raw raw[kA];
  float2 sv[kA];
#pragma unroll
  for (int n1 = 0; n1 < kA; ++n1) {
    raw[n1] = *(reinterpret_cast<const Raw*>(static_cast<const char*>(xb) + static_cast<int64_t>(lo + kB * n1 * C) * (F32 ? 4 : 2)));
    sv[n1] = st[n2 + kB * n1];
  }
  ChanParams cp;
  load_params(a, c0, cp);
  cpair v[kA];  // the lane's two packed channel pairs (h0 + i h1, h2 + i h3) as one cpair
#pragma unroll
  for (int n1 = 0; n1 < kA; ++n1) {
    float xr[kCh], h[kCh];
    if constexpr (F32) {
      xr[0] = raw[n1].x; xr[1] = raw[n1].y; xr[2] = raw[n1].z; xr[3] = raw[n1].w;
    } else {
      unpack4(raw[n1], xr);
    }
    ln4f(xr, sv[n1], cp, h);
    v[n1] = cpair{f2v{h[0], h[2]}, f2v{h[1], h[3]}};
  }
  pass0_store(v, n2, g, lds);
  __syncthreads();
  // ---- pass 1 (threads k1 < 12), result back to LDS in natural order k = k1 + 12 k2
  cpair u[kB];
  const int k1 = n2;
  if (k1 < kA) pass1(k1, g, lds, u);
  __syncthreads();
  if (k1 < kA) {
#pragma unroll
    for (int k2 = 0; k2 < kB; ++k2) st_pair(lds, (k1 + kA * k2) * kPitch + kPPL * g, cpair_lo(u[k2]), cpair_hi(u[k2]));
  }
  __syncthreads();
  // ---- separate the packed pairs: X_a[k] = (Z[k] + conj Z[L-k]) / 2, X_b[k] = (Z[k] - conj Z[L-k]) / 2i
  const float hs = 0.5f * a.scale;
  const int64_t obase = (static_cast<int64_t>(o) * KM * C + slab * kSlab) * 2;
  constexpr int kItems = KM * kG;
#pragma unroll
  for (int it = 0; it < (kItems + kThreads - 1) / kThreads; ++it) {
    const int item = it * kThreads + threadIdx.x;
    if (item >= kItems) break;
    const int k = item / kG, gg = item % kG;
    const int km = k == 0 ? 0 : kL - k;
    float2 Zk[2], Zm[2];
    ld_pair(lds, k * kPitch + kPPL * gg, Zk[0], Zk[1]);
    ld_pair(lds, km * kPitch + kPPL * gg, Zm[0], Zm[1]);
    float w[8];
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
      w[4 * p + 0] = (Zk[p].x + Zm[p].x) * hs;
      w[4 * p + 1] = (Zk[p].y - Zm[p].y) * hs;
      w[4 * p + 2] = (Zk[p].y + Zm[p].y) * hs;
      w[4 * p + 3] = (Zm[p].x - Zk[p].x) * hs;
    }
    const int64_t off = obase + (k * C + kCh * gg) * 2;
    if constexpr (F32) {
      float* op = static_cast<float*>(a.out) + off;
      *reinterpret_cast<float4*>(op) = make_float4(w[0], w[1], w[2], w[3]);
      *reinterpret_cast<float4*>(op + 4) = make_float4(w[4], w[5], w[6], w[7]);
    } else {
      *reinterpret_cast<uint4*>(static_cast<uint16_t*>(a.out) + off) =
          make_uint4(bfpack(w[0], w[1]), bfpack(w[2], w[3]), bfpack(w[4], w[5]), bfpack(w[6], w[7]));
    }
  }
}

// compile-time support of the pruned C2R input: 0 = never stored, 1 = always, 2 = depends on n2
template <int KM>
constexpr int c2r_load_kind(int n1) {
  bool all = true, any = false;
  for (int n = kB * n1; n < kB * n1 + kB; ++n) {
    const bool ok = n < KM || kL - n < KM;
    all = all && ok;
    any = any || ok;
  }
  return all ? 1 : (any ? 2 : 0);
}


// SPLIT (fp32 block, round 4): the epilogue also writes the next GEMM's operand -- the bf16x3 split
// pairs of y - mean(x), centred per token -- and the next LayerNorm's partial statistics of y over this workgroup's 64 channels
// (y staged in the LDS buffer, one thread per position sweeping its 64 channels).  That removes the separate
// LayerNorm -> split pass over the residual stream (one full read of it per block); LN2 is then
// folded into fc1's epilogue (linear3_ln) from per-token stats merged by ln_stats_merge.
// Register budget (workgroups per CU): the fp32 instantiation holds the 15-point DFT (60 VGPRs) and
// its 15 positions' addends (90) across the DFT; with the split / statistics epilogue that needs
// ~256 VGPRs, i.e. 2 workgroups per CU (at 3 it spilled ~400 bytes per lane).
#ifndef AFNO_C2R_SPLIT_OCC
#define AFNO_C2R_SPLIT_OCC 2
#endif
#ifndef AFNO_C2R_JIT
#define AFNO_C2R_JIT 0  // fp32: addends loaded 3 positions ahead inside the epilogue (A/B; see below)
#endif
// PART (bf16 block): the epilogue also writes the next LayerNorm's per-64-channel partials of the STORED
// (bf16-rounded) output -- the rounded values written over the lane's own slot of the residual tile in LDS,
// one thread per position sweeping its 64 channels -- so the bf16 block needs no ln_stats pass over x1 either.
template <int KM, bool F32, bool SPLIT = false, bool PART = false>
__global__ void __launch_bounds__(kThreads, SPLIT ? AFNO_C2R_SPLIT_OCC : 3) afno_w_c2r_ln_kernel(const WArgs a) {
  static_assert(!SPLIT || F32, "split-pair outputs come with the fp32 instantiation");
  static_assert(!PART || (!F32 && AFNO_C2R_XLDS), "bf16 partials: the fp16-staged bf16 instantiation");
  static_assert(KM >= 1 && 2 * KM <= kL, "pruned half spectrum");
  // bf16 (XLDS): fp16 FFT staging (24.5 KB) + the residual tile x[o, 0..179, slab] (23 KB) + its
  // LN statistics: 49.6 KB -> still 3 workgroups per CU, and the addends need no VGPRs.
  // fp32: fp32 staging (49 KB), addends loaded to registers.
  constexpr bool XLDS = AFNO_C2R_XLDS && !F32;
  using ST = typename std::conditional<XLDS, h2_t, float2>::type;
  constexpr int kStageBytes = kL * kPitch * static_cast<int>(sizeof(ST));
  constexpr int kImgBytes = XLDS ? kRounds * kRound : 0;
  __shared__ __attribute__((aligned(16))) char smem[kStageBytes + kImgBytes];
  ST* lds = reinterpret_cast<ST*>(smem);
  char* dimg = smem + kStageBytes;
  const uint2* xt = reinterpret_cast<const uint2*>(dimg);               // [pos][16 lanes x 4 ch] bf16
  const float2* stl = reinterpret_cast<const float2*>(dimg + kXBytes);  // [pos] (mean, rstd)
  const int o = blockIdx.x / a.nslab, slab = blockIdx.x - o * a.nslab;
  AMD_DFT_DEV_CHECK((slab + 1) * kSlab <= a.C, "afno_w_kernel");
  const int g = threadIdx.x % kG, n2 = threadIdx.x / kG;
  const int c0 = slab * kSlab + kCh * g;
  const int C = a.C;
  const int64_t sbase = (static_cast<int64_t>(o) * KM * C + slab * kSlab) * 2;
  const int64_t xbase = static_cast<int64_t>(o) * kL * C + slab * kSlab;
  const void* xb = F32 ? static_cast<const void*>(static_cast<const float*>(a.x) + xbase)
                       : static_cast<const void*>(static_cast<const uint16_t*>(a.x) + xbase);
  const float2* st = a.stats + static_cast<int64_t>(o) * kL;
  if constexpr (XLDS) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const char* xbc = static_cast<const char*>(xb);
    const char* stc = reinterpret_cast<const char*>(st);
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int b = r * kRound + wave * 1024 + lane * 16;  // byte of the image this lane fills
      const int bx = min(b, kXBytes - 16);
      const char* src_x = xbc + (bx >> 7) * (2 * C) + (bx & 127);
      const char* src_s = stc + min(max(b - kXBytes, 0), kSBytes - 16);
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(b < kXBytes ? src_x : src_s),
                                       (lds_void*)(dimg + r * kRound + wave * 1024), 16, 0, 0);
    }
  }
  // ---- pass 0: Hermitian assembly of the packed pair spectrum Z = X_a + i X_b, conjugated
  // (inverse transform as conj(FFT(conj Z))); only the stored modes are loaded
  struct F8 { float4 a, b; };
  using Raw = typename std::conditional<F32, F8, uint4>::type;  // raw until use (bf16: 4 VGPRs)
  Raw raw[kA];
#pragma unroll
  for (int n1 = 0; n1 < kA; ++n1) {
    if (c2r_load_kind<KM>(n1) != 0) {
      const int n = n2 + kB * n1;
      const int kk = 2 * n > kL ? kL - n : n;
      const int kc = kk < KM ? kk : 0;  // clamped: unconditional load, masked below
      const int64_t off = sbase + (kc * C + kCh * g) * 2;
      raw[n1] = *reinterpret_cast<const Raw*>(static_cast<const char*>(a.spec) + off * (F32 ? 4 : 2));
    }
  }
  cpair v[kA];
#pragma unroll
  for (int n1 = 0; n1 < kA; ++n1) {
    const int kind = c2r_load_kind<KM>(n1);
    if (kind == 0) {
      v[n1] = cpair{f2v{0.f, 0.f}, f2v{0.f, 0.f}};
      continue;
    }
    const int n = n2 + kB * n1;
    const bool upper = 2 * n > kL;
    const int kk = upper ? kL - n : n;
    const bool ok = kind == 1 || kk < KM;
    float f[8];
    if constexpr (F32) {
      f[0] = raw[n1].a.x; f[1] = raw[n1].a.y; f[2] = raw[n1].a.z; f[3] = raw[n1].a.w;
      f[4] = raw[n1].b.x; f[5] = raw[n1].b.y; f[6] = raw[n1].b.z; f[7] = raw[n1].b.w;
    } else {
      unpack4(make_uint2(raw[n1].x, raw[n1].y), *reinterpret_cast<float(*)[4]>(f));
      unpack4(make_uint2(raw[n1].z, raw[n1].w), *reinterpret_cast<float(*)[4]>(f + 4));
    }
    float2 zp[kPPL];
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
      // channel pair (c0 + 2p, c0 + 2p + 1): A = X_a[kk], B = X_b[kk] (complex)
      float2 A = make_float2(f[4 * p], f[4 * p + 1]);
      float2 B = make_float2(f[4 * p + 2], f[4 * p + 3]);
      if (kk == 0 || 2 * kk == kL) {
        A.y = 0.f;
        B.y = 0.f;
      }
      if (upper) {
        A.y = -A.y;
        B.y = -B.y;
      }
      const float2 z = make_float2(A.x - B.y, -(A.y + B.x));  // conj(A + iB)
      zp[p] = ok ? z : make_float2(0.f, 0.f);
    }
    v[n1] = make_cpair(zp[0], zp[1]);
  }
  pass0_store(v, n2, g, lds);
  if constexpr (XLDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS DMA landed before the barrier publishes it
  __syncthreads();
  const int k1 = n2;
  if (k1 >= kA) return;
  // pass-1 operands from LDS, then the residual-stream addends (their latency hides under the
  // 15-point DFTs); sched barriers keep the compiler from hoisting the 30 addend loads above
  // the LDS reads (register pressure -> occupancy)
  cpair u[kB];
#pragma unroll
  for (int n2i = 0; n2i < kB; ++n2i) {
    float2 pa, pb;
    ld_pair(lds, (k1 * kB + n2i) * kPitch + kPPL * g, pa, pb);
    u[n2i] = make_cpair(pa, pb);
  }
  __builtin_amdgcn_sched_barrier(0);
  const int lo = k1 * C + kCh * g;  // 32-bit lane offset from the workgroup-uniform base
  float xr[XLDS ? 1 : kB][kCh];
  float2 sv[XLDS ? 1 : kB];
  // register addends: all 15 positions' loads issued before the DFT (latency hidden under it), or
  // (AFNO_C2R_JIT) only the first JD, the rest JD positions ahead inside the epilogue (fewer live
  // VGPRs: the split instantiation then fits 3 workgroups per CU without spilling)
  constexpr bool JIT = AFNO_C2R_JIT && !XLDS;
  constexpr int JD = JIT ? 3 : kB;
  auto ld_add = [&](int k2) {
    ldx4<F32>(xb, lo + kA * k2 * C, xr[k2]);
    sv[k2] = st[k1 + kA * k2];
  };
  if constexpr (!XLDS) {
#pragma unroll
    for (int k2 = 0; k2 < JD; ++k2) ld_add(k2);
  }
  ChanParams cp;
  load_params(a, c0, cp);
  __builtin_amdgcn_sched_barrier(0);
  Dft<kB>::run(u);
  __builtin_amdgcn_sched_barrier(0);
  // SPLIT: the staging buffer takes the outputs for the per-position statistics below -- every
  // wave past its pass-1 reads first (the k1 >= 12 wave has exited: barriers count live waves)
  if constexpr (SPLIT) __syncthreads();
  // ---- epilogue: y = scale * conj(u) + x' + LN(x'), output n = k1 + 12 k2
  const int64_t obase = xbase;
  void* ob = F32 ? static_cast<void*>(static_cast<float*>(a.out) + obase)
                 : static_cast<void*>(static_cast<uint16_t*>(a.out) + obase);
  const float sc = a.scale;
  uint16_t* const pbase = SPLIT ? a.pairs + static_cast<int64_t>(o) * kL * (2 * C) : nullptr;
  float* const sbase_part = SPLIT || PART ? a.part + (static_cast<int64_t>(o) * kL * a.nslab + slab) * 2 : nullptr;
#pragma unroll
  for (int k2 = 0; k2 < kB; ++k2) {
    if constexpr (JIT) {
      if (k2 + JD < kB) ld_add(k2 + JD);
    }
    float xp[kCh], h[kCh];
    if constexpr (XLDS) {
      const int n = k1 + kA * k2;
      ln4(xt[n * kG + g], stl[n], cp, xp, h);
    } else {
#pragma unroll
      for (int i = 0; i < kCh; ++i) xp[i] = xr[k2][i];
      ln4f(xp, sv[k2], cp, h);
    }
    float y[kCh];
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
      y[2 * p] = u[k2].re[p] * sc + xp[2 * p] + h[2 * p];
      y[2 * p + 1] = -u[k2].im[p] * sc + xp[2 * p + 1] + h[2 * p + 1];
    }
    // SPLIT with out == nullptr: only the split pairs (the residual then travels as them, see
    // linear3_stats_pr) -- the fp32 store is the largest of this kernel's three output streams
    if (!SPLIT || a.out != nullptr) stx4<F32>(ob, lo + kA * k2 * C, y[0], y[1], y[2], y[3]);
    if constexpr (PART) {
      // the stored bf16 values (8 B) over this lane's own residual slot of the LDS image, which no other
      // thread reads: no barrier between the FFT and the epilogue (one before the sweep below)
      const int n = k1 + kA * k2;
      reinterpret_cast<uint2*>(dimg)[n * kG + g] = make_uint2(bfpack(y[0], y[1]), bfpack(y[2], y[3]));
    }
    if constexpr (SPLIT) {
      // workgroup-uniform bases (o's first token) + 32-bit lane offsets: position n = k1 + 12 k2
      // the pairs hold y - mean(x) (x's LayerNorm mean, already in sv): the split then resolves y's
      // deviation from a per-token offset to 2^-17 instead of its absolute value, so fc1's folded
      // mean cancellation keeps fp32-class accuracy when |mean| >> std (ln_stats_merge(shift=) of
      // the same stats hands fc1 mean(y) - mean(x))
      const int n = k1 + kA * k2;
      const float m0 = sv[k2].x;
      const float z0 = y[0] - m0, z1 = y[1] - m0, z2 = y[2] - m0, z3 = y[3] - m0;
      const uint32_t h01 = bfpack(z0, z1), h23 = bfpack(z2, z3);
      const uint32_t l01 = bfpack(z0 - __uint_as_float(h01 << 16), z1 - __uint_as_float(h01 & 0xffff0000u));
      const uint32_t l23 = bfpack(z2 - __uint_as_float(h23 << 16), z3 - __uint_as_float(h23 & 0xffff0000u));
      uint16_t* pr = pbase + (n * (2 * C) + (c0 >> 5) * 64 + (c0 & 31));  // k32-interleaved [hi(32) | lo(32)]
      *reinterpret_cast<uint2*>(pr) = make_uint2(h01, h23);
      *reinterpret_cast<uint2*>(pr + 32) = make_uint2(l01, l23);
      if (a.lo2 != nullptr) {  // wave-uniform: the split's third term, 16 lanes x 8 B = a 128-byte row piece
        const auto up = [](uint32_t w, bool hi) { return __uint_as_float(hi ? (w & 0xffff0000u) : (w << 16)); };
        const float r0 = z0 - (up(h01, false) + up(l01, false)), r1 = z1 - (up(h01, true) + up(l01, true));
        const float r2 = z2 - (up(h23, false) + up(l23, false)), r3 = z3 - (up(h23, true) + up(l23, true));
        *reinterpret_cast<uint2*>(a.lo2 + static_cast<int64_t>(o) * kL * C + n * C + c0) =
            make_uint2(bfpack(r0, r1), bfpack(r2, r3));
      }
      *reinterpret_cast<float4*>(lds + n * kPitch + kPPL * g) = make_float4(y[0], y[1], y[2], y[3]);
    }
    // one output position at a time: interleaving the positions' epilogues (the scheduler's
    // choice) keeps several positions' temporaries live and spills the fp32 instantiations
    if constexpr (F32) __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (SPLIT) {
    // LN2 partials of this slab: one thread per output position sweeps its 64 staged channels once,
    // as shifted sums (shift = the position's first value: M2 = S2 - S1^2 / 64 cancels only a few std)
    // -- two 16-lane DPP reductions per position and lane cost ~10x the VALU
    __syncthreads();
    const int n = threadIdx.x;
    if (n < kL) {
      const float4* row = reinterpret_cast<const float4*>(lds + n * kPitch);
      const float sh = row[0].x;
      float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
#pragma unroll
      for (int j = 0; j < kG; ++j) {
        const float4 q = row[j];
        const float d0 = q.x - sh, d1 = q.y - sh, d2 = q.z - sh, d3 = q.w - sh;
        s1.x += d0;
        s1.y += d1;
        s1.z += d2;
        s1.w += d3;
        s2.x = fmaf(d0, d0, s2.x);
        s2.y = fmaf(d1, d1, s2.y);
        s2.z = fmaf(d2, d2, s2.z);
        s2.w = fmaf(d3, d3, s2.w);
      }
      const float t1 = (s1.x + s1.y) + (s1.z + s1.w), t2 = (s2.x + s2.y) + (s2.z + s2.w);
      *reinterpret_cast<float2*>(sbase_part + n * (2 * a.nslab)) =
          make_float2(sh + t1 * (1.f / 64.f), fmaxf(t2 - t1 * t1 * (1.f / 64.f), 0.f));
    }
  }
  if constexpr (PART) {
    // one sweep of shifted sums (shift = the position's first value; M2 = S2 - S1^2 / 64 then cancels
    // only a few std): the 64 stored values are read once
    __syncthreads();
    const int n = threadIdx.x;
    if (n < kL) {
      const uint4* row = reinterpret_cast<const uint4*>(dimg + n * (kG * 8));
      const float sh = __uint_as_float(row[0].x << 16);
      float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // 8 bf16 per 16 B
        const uint4 q = row[j];
        const uint32_t u[4] = {q.x, q.y, q.z, q.w};
        float* a1 = &s1.x;
        float* a2 = &s2.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float d0 = __uint_as_float(u[k] << 16) - sh, d1 = __uint_as_float(u[k] & 0xffff0000u) - sh;
          a1[k] += d0 + d1;
          a2[k] = fmaf(d0, d0, fmaf(d1, d1, a2[k]));
        }
      }
      const float t1 = (s1.x + s1.y) + (s1.z + s1.w), t2 = (s2.x + s2.y) + (s2.z + s2.w);
      *reinterpret_cast<float2*>(sbase_part + n * (2 * a.nslab)) =
          make_float2(sh + t1 * (1.f / 64.f), fmaxf(t2 - t1 * t1 * (1.f / 64.f), 0.f));
    }
  }
}

WArgs make_args(const AfnoWLaunch& p) {
  WArgs a;
  a.x = p.x;
  a.stats = reinterpret_cast<const float2*>(p.stats);
  a.gamma = p.gamma;
  a.beta = p.beta;
  a.pre = p.pre;
  a.spec = p.spec;
  a.out = p.out;
  a.pairs = p.pairs;
  a.part = p.part;
  a.lo2 = p.lo2;
  a.C = p.C;
  a.nslab = p.C / kSlab;
  a.scale = p.scale;
  return a;
}

void check_launch(const AfnoWLaunch& p, const char* what) {
  if (!afno_w_supported(p.L, p.C, p.KM)) throw std::runtime_error(std::string("amd_dft: ") + what + ": unsupported shape");
  const int64_t nwg = static_cast<int64_t>(p.O) * (p.C / kSlab);
  if (nwg <= 0 || nwg > 0x7fffffffLL) throw std::runtime_error(std::string("amd_dft: ") + what + ": bad grid");
  if (static_cast<int64_t>(p.O) * kL * p.C >= (int64_t(1) << 40)) throw std::runtime_error("amd_dft: afno_w: too large");
}

}  // namespace

bool afno_w_supported(int L, int C, int KM) { return L == kL && C % kSlab == 0 && KM == 46; }

void launch_afno_w_r2c_ln(const AfnoWLaunch& p, void* stream) {
  check_launch(p, "afno_w_r2c_ln");
  const WArgs a = make_args(p);
  const dim3 grid(static_cast<uint32_t>(static_cast<int64_t>(p.O) * a.nslab));
  if (p.f32) hipLaunchKernelGGL((afno_w_r2c_ln_kernel<46, true>), grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
  else hipLaunchKernelGGL((afno_w_r2c_ln_kernel<46, false>), grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: afno_w_r2c_ln launch: ") + hipGetErrorString(e));
}

void launch_afno_w_c2r_ln(const AfnoWLaunch& p, void* stream) {
  check_launch(p, "afno_w_c2r_ln");
  const WArgs a = make_args(p);
  const dim3 grid(static_cast<uint32_t>(static_cast<int64_t>(p.O) * a.nslab));
  if (p.f32 ? (p.pairs != nullptr) != (p.part != nullptr) : p.pairs != nullptr)
    throw std::runtime_error("amd_dft: afno_w_c2r_ln: fp32: split pairs and partial statistics come together; bf16: partials only");
  if (p.pairs) hipLaunchKernelGGL((afno_w_c2r_ln_kernel<46, true, true>), grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
  else if (p.part) hipLaunchKernelGGL((afno_w_c2r_ln_kernel<46, false, false, true>), grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
  else if (p.f32) hipLaunchKernelGGL((afno_w_c2r_ln_kernel<46, true>), grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
  else hipLaunchKernelGGL((afno_w_c2r_ln_kernel<46, false>), grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: afno_w_c2r_ln launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
