// Kernel templates of the compile-time specialised Stockham FFT (see fft_fixed.h).
// Included by fft_fixed_k{0,1,2}.hip (one translation unit per transform kind, compiled in
// parallel) -- do not include elsewhere.
//
// Structure of one workgroup (T FFTs of length L, TP threads each):
//   pass 0      : global -> registers (coalesced: lane = butterfly index j, or signal t for
//                 column layouts), radix-R0 DFT, registers -> LDS
//   pass 1..P-2 : LDS -> registers, twiddle (prefetched one pass ahead from the plan's
//                 fp64-accurate table), DFT, registers -> LDS
//   pass P-1    : LDS -> registers, twiddle, DFT, registers -> global (C2C / C2R) -- the
//                 Stockham last pass writes n = j + r*L/R, i.e. contiguous across lanes;
//                 R2C goes through LDS once more to pair Z[k] with Z[L-k].
// Normalisation and the inverse conjugation are fused into the first load / last store.
#pragma once

#include <hip/hip_runtime.h>

// Twiddle source of passes 1..P-1:
//   0: the plan's global table (L1/L2 resident), each thread's twiddles of pass p + 1 prefetched
//      into registers while pass p runs;
//   1: the whole table staged into LDS by the workgroup at kernel start (coalesced 8-byte loads
//      issued together with pass 0's global loads), each pass reading its twiddles from LDS after
//      its barrier (no prefetch registers).
#ifndef AMD_DFT_TW_LDS
#define AMD_DFT_TW_LDS 0
#endif
// Twiddle powers: each butterfly loads only w = W^k from the table and forms
// w^2 .. w^(R-1) by a complex recurrence (one c_mul each, ~1 ulp per step) in the butterfly pass:
// R - 2 fewer table loads and prefetch registers per butterfly and pass.  rfft2 -0.16 us,
// irfft2 -0.3 us at 720x1440 (profiles/fft_twiddle_rec_r5.txt); the GPU DFT tests' eps log N
// error bounds hold.  -DAMD_DFT_TW_REC=0 restores one table load per twiddle.
#ifndef AMD_DFT_TW_REC
#define AMD_DFT_TW_REC 1
#endif

#include "fft_fixed.h"
#include "radix.h"

namespace amd_dft {
namespace fixed_detail {

struct FixedArgs {
  const void* in;
  void* out;
  const float2* tw;
  int64_t So_in, So_out;              // outer offsets (64-bit, applied once per block)
  int32_t I, Si_in, Si_out, Sn_in, Sn_out;  // per-element offsets fit 32 bits (host-checked)
  int32_t in_lo, in_hi, out_lo, out_hi, tiles_per_outer;
  int32_t xcd_nb;    // > 0: XCD-aware remap of the nb = xcd_nb blocks (see xcd_block)
  float scale;
  int32_t inverse, vec_in, vec_out, bf16_in, bf16_out;
  const void* add1;  // C2R epilogue: out = scale * irfft + add1 (+ add2); same layout/dtype as out
  const void* add2;
  int32_t pairvec;   // paired real signals adjacent in memory (channel-last) and I even
  // LayerNorm IO fusion (NADD == 3 instantiations, see PassDesc::ln_stats)
  const float* ln_stats;
  const float* ln_gamma;
  const float* ln_beta;
  const float* ln_pre;
  // NADD == 4 (C2C only): FNO mode mixing on the first-pass gather (see PassDesc::mix_w)
  const float* mix_w;
  int32_t mix_cin, mix_cout;
#ifdef AMD_DFT_FFT_STAMPS
  long long* stamps;  // diagnostic build only (bench/fft_stamps.hip): per-block phase clocks
#endif
};

#ifdef AMD_DFT_FFT_STAMPS
// slot 0: s_memrealtime at entry, 1..: s_memtime after each phase (vector store by thread 0)
#define AMD_DFT_STAMP(a, slot, v) \
  do { if (threadIdx.x == 0) (a).stamps[static_cast<int64_t>(blockIdx.x) * 16 + (slot)] = (v); } while (0)
#else
#define AMD_DFT_STAMP(a, slot, v) do { } while (0)
#endif

template <int... Rs>
struct FL {
  static constexpr int N = sizeof...(Rs);
  static constexpr int r[N] = {Rs...};
  static constexpr int L = (Rs * ... * 1);
  static constexpr int ns(int p) {
    int v = 1;
    for (int i = 0; i < p; ++i) v *= r[i];
    return v;
  }
  // offset of pass p's twiddles in the plan table (passes with ns == 1 store none)
  static constexpr int goff(int p) {
    int o = 0;
    for (int i = 0; i < p; ++i)
      if (ns(i) > 1) o += (r[i] - 1) * ns(i);
    return o;
  }
};

constexpr __host__ __device__ int lds_pad(int i) { return i + (i >> 4); }
// Row-layout padding per length: one float2 every 2^S elements (S = 0: none).  Chosen from a
// bank-conflict simulation of the Stockham read / write patterns (ds_read_b64 / ds_write_b64,
// two 32-lane groups): 1440 = (10, 12, 12) at 144 threads is conflict-free unpadded (the n/16
// pad made its writes 3x), and an unpadded index is linear in the radix step, so the compiler
// folds it into ds_read / ds_write immediate offsets (no per-element index arithmetic);
// 720 = (8, 9, 10) is best with one pad per 8.  Column layouts (position-major, T signals per
// position) use a stride of T + 1 slots per position for T >= 4: the same or fewer conflicts than
// the n/16 pad on every configured shape and, again, an index linear in the position.
template <bool COLS, int L>
constexpr __host__ __device__ int row_pad_shift() {
  return COLS ? 4 : (L == 1440 ? 0 : (L == 720 ? 3 : 4));
}
template <bool COLS, int L>
constexpr __host__ __device__ int lds_padl(int i) {
  return row_pad_shift<COLS, L>() == 0 ? i : i + (i >> row_pad_shift<COLS, L>());
}

__device__ __forceinline__ float bf_to_f(uint32_t u16) { return __uint_as_float(u16 << 16); }
__device__ __forceinline__ uint32_t f_to_bf(float f) {
  return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(f)));
}
template <bool BF>
__device__ __forceinline__ float ld_r(const void* p, int32_t off) {
  if constexpr (BF) return bf_to_f(static_cast<const uint16_t*>(p)[off]);
  else return static_cast<const float*>(p)[off];
}
template <bool BF>
__device__ __forceinline__ float2 ld_c(const void* p, int32_t off) {
  if constexpr (BF) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(static_cast<const uint16_t*>(p) + off);
    return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
  } else {
    return *reinterpret_cast<const float2*>(static_cast<const float*>(p) + off);
  }
}
template <bool BF>
__device__ __forceinline__ void st_r(void* p, int32_t off, float v) {
  if constexpr (BF) static_cast<uint16_t*>(p)[off] = static_cast<uint16_t>(f_to_bf(v));
  else static_cast<float*>(p)[off] = v;
}
// AMD_DFT_FFT_NT_STORE=1 (A/B build): complex stores non-temporal -- written through to memory / the
// Infinity Cache instead of left dirty in the XCD's L2, which a kernel boundary then writes back
#ifndef AMD_DFT_FFT_NT_STORE
#define AMD_DFT_FFT_NT_STORE 0
#endif
template <bool BF>
__device__ __forceinline__ void st_c(void* p, int32_t off, float2 v) {
  if constexpr (BF) {
    *reinterpret_cast<uint32_t*>(static_cast<uint16_t*>(p) + off) = f_to_bf(v.x) | (f_to_bf(v.y) << 16);
  } else if constexpr (AMD_DFT_FFT_NT_STORE) {
    float* q = static_cast<float*>(p) + off;
    __builtin_nontemporal_store(v.x, q);
    __builtin_nontemporal_store(v.y, q + 1);
  } else {
    *reinterpret_cast<float2*>(static_cast<float*>(p) + off) = v;
  }
}
template <bool BF>
__device__ __forceinline__ void st_c2(void* p, int32_t off, float2 a, float2 b) {
  if constexpr (BF) {
    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p) + off) =
        make_uint2(f_to_bf(a.x) | (f_to_bf(a.y) << 16), f_to_bf(b.x) | (f_to_bf(b.y) << 16));
  } else {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + off) = make_float4(a.x, a.y, b.x, b.y);
  }
}
template <bool BF>
__device__ __forceinline__ float4 ld_c2(const void* p, int32_t off) {  // two adjacent complex values
  if constexpr (BF) {
    const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + off);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
  } else {
    return *reinterpret_cast<const float4*>(static_cast<const float*>(p) + off);
  }
}
__device__ __forceinline__ float2 sel(bool ok, float2 v) { return make_float2(ok ? v.x : 0.f, ok ? v.y : 0.f); }

struct Ctx {
  FixedArgs a;
  const void* in;   // outer-offset applied
  void* out;
  const void* add1;  // outer-offset applied
  const void* add2;
  int32_t c;        // complex signal index
  int32_t cc;       // c clamped into [0, I) (C2C) -- loads are never predicated by branches
  int32_t i0c, i1c; // paired logical signals 2c, 2c+1 clamped into [0, I) (R2C / C2R)
  bool ok0, ok1;    // c < I (C2C) / 2c < I, 2c+1 < I (paired)
  int t, tp;
  float2* lds;
  float2* twl;  // AMD_DFT_TW_LDS: the plan's twiddle table staged in LDS (filled during pass 0)
  // NADD == 3 (LayerNorm IO): stats of this outer row, per-channel params of the signal pair
  const float2* st;
  float2 g, be, pre;
};

// LayerNorm of one stored channel pair at position n: x' = v + pre, LN(x') (x' returned in xp)
__device__ __forceinline__ float2 ln_pair(const Ctx& x, int n, float2 v, float2& xp) {
  const float2 s = x.st[n];  // (mean, rstd) of token (o, n)
  xp = make_float2(v.x + x.pre.x, v.y + x.pre.y);
  return make_float2((xp.x - s.x) * s.y * x.g.x + x.be.x, (xp.y - s.x) * s.y * x.g.y + x.be.y);
}

// Column layouts of the 720-point transforms at T = 4 (rfft2 / irfft2 columns, the FNO H transforms),
// A/B build -DAMD_DFT_COL_PW8=1: position n of slot t at n*T + t + COL_PW * (n / 8) -- two pad slots per
// 8 positions instead of one per position.  Bank-conflict cycles per LDS instruction 3.72 -> 1.08
// (VERDICT r5 #6), but the extra index arithmetic is not folded into ds_read / ds_write immediates:
// +29 % VALU and +18 % LDS instructions per wave, rfft2 / irfft2 +0.5 us and the FNO block +1.3 us
// (profiles/fft_lds_pad_r6.txt; the conflicts it removes were ~90 cycles of a ~10k-cycle wave).  The
// shipped default keeps the T + 1 stride.
#ifndef AMD_DFT_COL_PW8
#define AMD_DFT_COL_PW8 0  // 1: the two-pads-per-8 column layout (A/B build, measured slower)
#endif
template <bool COLS, int T, int L>
constexpr __host__ __device__ int col_pw() {
  return (AMD_DFT_COL_PW8 && COLS && L == 720 && T == 4) ? 2 : 0;
}

template <bool COLS, int T, int L>
__device__ __forceinline__ int lidx(const Ctx& x, int n) {
  constexpr int LP = lds_padl<COLS, L>(L) + 1;
  if constexpr (col_pw<COLS, T, L>() > 0) return n * T + x.t + col_pw<COLS, T, L>() * (n >> 3);
  else if constexpr (COLS && T >= 4) return n * (T + 1) + x.t;  // one pad slot per position: linear in n
  else if constexpr (COLS) return lds_pad(n * T + x.t);
  else return x.t * LP + lds_padl<COLS, L>(n);
}

// First-pass element fetch (includes the C2R Hermitian assembly and input pruning).
// Every load is unconditional from a clamped (valid) address and masked afterwards with a
// select: a branch around a load makes hipcc wait vmcnt(0) per element.
template <Kind K, int L, bool BF, bool PR, bool PV, int NADD = 0>
__device__ __forceinline__ float2 gather(const Ctx& x, int n) {
  const FixedArgs& a = x.a;
  float2 z;
  if constexpr (K == Kind::C2C) {
    if constexpr (PR && NADD == 4) {
      // mixed input: x.in = this batch's [Cin][S][I] modes, x.add1 = this output channel's
      // weights (input-channel stride Cout * So_in).  Only stored modes run the channel loop
      // (at most one or two of a thread's R elements), so the branch costs less than the loads.
      const int s = n < a.in_lo ? n : (n >= L - a.in_hi ? a.in_lo + (n - (L - a.in_hi)) : -1);
      float zr = 0.f, zi = 0.f;
      if (x.ok0 && s >= 0) {
        const int32_t off = x.cc * a.Si_in + s * a.Sn_in;
        const int32_t sx = static_cast<int32_t>(a.So_in), sw = static_cast<int32_t>(a.So_in) * a.mix_cout;
        // batches of 20 channels: all 40 loads of a batch in flight before the first FMA
        // (clamped channel index, masked product) -- one L2 round trip per batch
        constexpr int U = 20;
        for (int i0 = 0; i0 < a.mix_cin; i0 += U) {
          float2 xv[U], wv[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int i = min(i0 + u, a.mix_cin - 1);
            xv[u] = ld_c<false>(x.in, i * sx + off);
            wv[u] = ld_c<false>(x.add1, i * sw + off);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const float m = i0 + u < a.mix_cin ? 1.f : 0.f;
            zr = fmaf(m * xv[u].x, wv[u].x, fmaf(-m * xv[u].y, wv[u].y, zr));
            zi = fmaf(m * xv[u].x, wv[u].y, fmaf(m * xv[u].y, wv[u].x, zi));
          }
        }
      }
      z = make_float2(zr, zi);
    } else if constexpr (PR) {
      const int s = n < a.in_lo ? n : (n >= L - a.in_hi ? a.in_lo + (n - (L - a.in_hi)) : -1);
      const bool ok = x.ok0 && s >= 0;
      z = sel(ok, ld_c<BF>(x.in, x.cc * a.Si_in + (s < 0 ? 0 : s) * a.Sn_in));
    } else {
      z = sel(x.ok0, ld_c<BF>(x.in, x.cc * a.Si_in + n * a.Sn_in));
    }
    if (a.inverse) z.y = -z.y;
  } else if constexpr (K == Kind::R2C) {
    if constexpr (PV && NADD == 3) {  // LayerNorm on load
      float2 xp;
      z = sel(x.ok0, ln_pair(x, n, ld_c<BF>(x.in, x.i0c * a.Si_in + n * a.Sn_in), xp));
    } else if constexpr (PV) {  // the two packed real signals are adjacent: one vector load
      z = sel(x.ok0, ld_c<BF>(x.in, x.i0c * a.Si_in + n * a.Sn_in));
    } else {
      const float va = ld_r<BF>(x.in, x.i0c * a.Si_in + n * a.Sn_in);
      const float vb = ld_r<BF>(x.in, x.i1c * a.Si_in + n * a.Sn_in);
      z = make_float2(x.ok0 ? va : 0.f, x.ok1 ? vb : 0.f);
    }
  } else {
    const bool upper = 2 * n > L;
    const int kk = upper ? L - n : n;
    const bool okk = kk < a.in_lo;
    const int kc = okk ? kk : 0;
    float2 A, B;
    if constexpr (PV) {
      const float4 ab = ld_c2<BF>(x.in, x.i0c * a.Si_in + kc * a.Sn_in);
      A = sel(okk && x.ok0, make_float2(ab.x, ab.y));
      B = sel(okk && x.ok0, make_float2(ab.z, ab.w));
    } else {
      A = sel(okk && x.ok0, ld_c<BF>(x.in, x.i0c * a.Si_in + kc * a.Sn_in));
      B = sel(okk && x.ok1, ld_c<BF>(x.in, x.i1c * a.Si_in + kc * a.Sn_in));
    }
    if (kk == 0 || 2 * kk == L) { A.y = 0.f; B.y = 0.f; }
    if (upper) { A.y = -A.y; B.y = -B.y; }
    z = make_float2(A.x - B.y, A.y + B.x);
    if (a.inverse) z.y = -z.y;
  }
  return z;
}

// Last-pass element store (C2C / C2R), with output pruning, the fused scale and (C2R) the
// pre-loaded addend pair `ad` (add1 + add2 at this element, zero when NADD == 0).
template <Kind K, int L, bool BF, bool PR, bool PV>
__device__ __forceinline__ void scatter(const Ctx& x, int n, float2 v, float2 ad) {
  const FixedArgs& a = x.a;
  if constexpr (K == Kind::C2C) {
    if (a.inverse) v.y = -v.y;
    if constexpr (PR) {
      const int s = n < a.out_lo ? n : (n >= L - a.out_hi ? a.out_lo + (n - (L - a.out_hi)) : -1);
      if (x.ok0 && s >= 0) st_c<BF>(x.out, x.c * a.Si_out + s * a.Sn_out, make_float2(v.x * a.scale, v.y * a.scale));
    } else {
      if (x.ok0) st_c<BF>(x.out, x.c * a.Si_out + n * a.Sn_out, make_float2(v.x * a.scale, v.y * a.scale));
    }
  } else {
    const float va = v.x * a.scale + ad.x;
    const float vb = (a.inverse ? -v.y : v.y) * a.scale + ad.y;
    const int32_t off = x.i0c * a.Si_out + n * a.Sn_out;
    if constexpr (PV) {
      if (x.ok0) st_c<BF>(x.out, off, make_float2(va, vb));
    } else {
      if (x.ok0) st_r<BF>(x.out, off, va);
      if (x.ok1) st_r<BF>(x.out, x.i1c * a.Si_out + n * a.Sn_out, vb);
    }
  }
}

// C2R addends of one output element (both packed signals), summed.
template <int NADD, bool BF, bool PV>
__device__ __forceinline__ float2 load_addend(const Ctx& x, int n) {
  float2 r = make_float2(0.f, 0.f);
  if constexpr (NADD > 0) {
    const FixedArgs& a = x.a;
    const int32_t off = x.i0c * a.Si_out + n * a.Sn_out;
    const int32_t offb = x.i1c * a.Si_out + n * a.Sn_out;
    if constexpr (PV && NADD == 3) {  // x' + LN(x') of the stored residual stream x
      float2 xp;
      const float2 h = ln_pair(x, n, ld_c<BF>(x.add1, off), xp);
      r = make_float2(xp.x + h.x, xp.y + h.y);
    } else if constexpr (PV) {
      r = ld_c<BF>(x.add1, off);
      if constexpr (NADD == 2) {
        const float2 t = ld_c<BF>(x.add2, off);
        r.x += t.x;
        r.y += t.y;
      }
    } else {
      r = make_float2(ld_r<BF>(x.add1, off), ld_r<BF>(x.add1, offb));
      if constexpr (NADD == 2) {
        r.x += ld_r<BF>(x.add2, off);
        r.y += ld_r<BF>(x.add2, offb);
      }
    }
  }
  return r;
}

template <class F, int TP, int P>
struct PassGeom {
  static constexpr int R = F::r[P];
  static constexpr int LR = F::L / R;
  static constexpr int Q = (LR + TP - 1) / TP;
  static constexpr int Ns = F::ns(P);
  static constexpr bool EXACT = (LR % TP) == 0;
  static constexpr int TWR = R > 1 ? R - 1 : 1;
};

// Twiddles of pass P for this thread's butterflies (global table, L1/L2 resident).
template <class F, int TP, int P>
__device__ __forceinline__ void load_tw(const Ctx& x, float2 (&tw)[PassGeom<F, TP, P>::Q][PassGeom<F, TP, P>::TWR]) {
  using G = PassGeom<F, TP, P>;
  if constexpr (G::Ns > 1) {
#pragma unroll
    for (int q = 0; q < G::Q; ++q) {
      const int j = x.tp + q * TP;
      if (G::EXACT || j < G::LR) {
        const int k = j % G::Ns;
#pragma unroll
        for (int r = 1; r < (AMD_DFT_TW_REC ? 2 : G::R); ++r) {
          if constexpr (AMD_DFT_TW_LDS) tw[q][r - 1] = x.twl[F::goff(P) + (r - 1) * G::Ns + k];
          else tw[q][r - 1] = x.a.tw[F::goff(P) + (r - 1) * G::Ns + k];
        }
      }
    }
  }
}

template <Kind K, bool COLS, int TP, int T, class F, int P, bool BFI, bool BFO, bool PR, int NADD, bool PV>
struct Step {
  using G = PassGeom<F, TP, P>;
  static constexpr int NP = F::N;
  static constexpr int L = F::L;
  static constexpr bool LAST = P == NP - 1;

  __device__ __forceinline__ static void run(const Ctx& x, float2 (&tw)[G::Q][G::TWR]) {
    constexpr int R = G::R, LR = G::LR, Q = G::Q, Ns = G::Ns;
    if constexpr (AMD_DFT_TW_LDS) {  // twiddles read from LDS inside body, after its barrier
      body(x, tw);
      AMD_DFT_STAMP(x.a, 3 + P, static_cast<long long>(__builtin_amdgcn_s_memtime()));
      if constexpr (!LAST) {
        using GN = PassGeom<F, TP, P + 1>;
        float2 twn[GN::Q][GN::TWR];
        Step<K, COLS, TP, T, F, P + 1, BFI, BFO, PR, NADD, PV>::run(x, twn);
      }
      return;
    }
    // prefetch next pass' twiddles
    if constexpr (!LAST) {
      using GN = PassGeom<F, TP, P + 1>;
      float2 twn[GN::Q][GN::TWR];
      load_tw<F, TP, P + 1>(x, twn);
      body(x, tw);
      AMD_DFT_STAMP(x.a, 3 + P, static_cast<long long>(__builtin_amdgcn_s_memtime()));
      Step<K, COLS, TP, T, F, P + 1, BFI, BFO, PR, NADD, PV>::run(x, twn);
    } else {
      body(x, tw);
      AMD_DFT_STAMP(x.a, 3 + P, static_cast<long long>(__builtin_amdgcn_s_memtime()));
    }
  }

  __device__ __forceinline__ static void body(const Ctx& x, float2 (&tw)[G::Q][G::TWR]) {
    constexpr int R = G::R, LR = G::LR, Q = G::Q, Ns = G::Ns;
    float2 v[Q][R];
    // C2R epilogue addends: issued before this pass' gather so their latency hides under it
    constexpr bool ADDS = LAST && K == Kind::C2R && NADD > 0;
    float2 addv[ADDS ? Q : 1][ADDS ? R : 1];
    if constexpr (ADDS) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int jr = x.tp + q * TP;
        const int j = (G::EXACT || jr < LR) ? jr : 0;
#pragma unroll
        for (int r = 0; r < R; ++r) addv[q][r] = load_addend<NADD, BFO, PV>(x, j + r * Ns);
      }
    }
    // ---- gather
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int j = x.tp + q * TP;
      if (G::EXACT || j < LR) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if constexpr (P == 0) v[q][r] = gather<K, L, BFI, PR, PV, NADD>(x, j + r * LR);
          else v[q][r] = x.lds[lidx<COLS, T, L>(x, j + r * LR)];
        }
      }
    }
    if constexpr (AMD_DFT_TW_LDS && P == 0 && F::goff(F::N) > 0) {
      // stage the twiddle table behind pass 0's gather loads (one memory round trip for both);
      // pass 0's closing barrier publishes it to passes 1..P-1
      for (int i = static_cast<int>(threadIdx.x); i < F::goff(F::N); i += TP * T) x.twl[i] = x.a.tw[i];
    }
    if constexpr (P > 0) __syncthreads();  // all reads of the shared buffer done
    if constexpr (AMD_DFT_TW_LDS) load_tw<F, TP, P>(x, tw);  // staged table, visible since pass 0's barrier
    // ---- twiddle + butterfly
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int j = x.tp + q * TP;
      if (G::EXACT || j < LR) {
        if constexpr (Ns > 1) {
          if constexpr (AMD_DFT_TW_REC) {
            const float2 w = tw[q][0];
            float2 wr = w;
            v[q][1] = c_mul(v[q][1], w);
#pragma unroll
            for (int r = 2; r < R; ++r) {
              wr = c_mul(wr, w);
              v[q][r] = c_mul(v[q][r], wr);
            }
          } else {
#pragma unroll
            for (int r = 1; r < R; ++r) v[q][r] = c_mul(v[q][r], tw[q][r - 1]);
          }
        }
        Dft<R>::run(v[q]);
      }
    }
    // ---- scatter
    if constexpr (LAST && K != Kind::R2C) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int j = x.tp + q * TP;
        if (G::EXACT || j < LR) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if constexpr (ADDS) scatter<K, L, BFO, PR, PV>(x, j + r * Ns, v[q][r], addv[q][r]);
            else scatter<K, L, BFO, PR, PV>(x, j + r * Ns, v[q][r], make_float2(0.f, 0.f));
          }
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int j = x.tp + q * TP;
        if (G::EXACT || j < LR) {
          const int k = j % Ns;
          const int base = (j - k) * R + k;
#pragma unroll
          for (int r = 0; r < R; ++r) x.lds[lidx<COLS, T, L>(x, base + r * Ns)] = v[q][r];
        }
      }
      __syncthreads();
    }
  }
};

// Workgroups are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), each with its
// own L2.  Column tiles narrower than a 128-B line share lines with their neighbours; the remap
// gives every XCD one contiguous range of tiles so those neighbours meet in the same L2
// instead of each XCD fetching the whole line.  Bijective for any nb.
__device__ __forceinline__ int32_t xcd_block(int32_t b, int32_t nb) {
  const int32_t per = nb >> 3, rem = nb & 7, xcd = b & 7, k = b >> 3;
  return (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + k;
}

template <Kind K, bool COLS, int TP, int T, class F, bool BFI, bool BFO, bool PR, int NADD, bool PV>
__device__ __forceinline__ void fixed_tile(const FixedArgs& a, int32_t bid, int tid, bool active, float2* lds,
                                           float2* twl = nullptr) {
  constexpr int L = F::L;
  Ctx x;
  x.a = a;
  x.t = COLS ? tid % T : tid / TP;
  x.tp = COLS ? tid / T : tid % TP;
  const int32_t o = bid / a.tiles_per_outer;
  const int32_t tile = bid - o * a.tiles_per_outer;
  x.c = tile * T + x.t;
  if constexpr (K == Kind::C2C) {
    x.ok0 = x.c < a.I;
    x.cc = x.ok0 ? x.c : a.I - 1;
  } else {
    x.ok0 = 2 * x.c < a.I;
    x.ok1 = 2 * x.c + 1 < a.I;
    if constexpr (PV) {  // I even (host-checked): clamp to the last complete pair
      x.i0c = x.ok0 ? 2 * x.c : a.I - 2;
      x.i1c = x.i0c + 1;
    } else {
      x.i0c = x.ok0 ? 2 * x.c : a.I - 1;
      x.i1c = x.ok1 ? 2 * x.c + 1 : a.I - 1;
    }
  }
  if (!active) {  // spare threads of a larger fused workgroup: run the same passes on a private
    x.ok0 = false;  // LDS slot (barriers stay uniform), store nothing
    x.ok1 = false;
  }
  if constexpr (K == Kind::C2C && NADD == 4) {  // mixing gather: batch / output-channel bases
    const int32_t b = o / a.mix_cout, oc = o - b * a.mix_cout;
    x.in = static_cast<const float*>(a.in) + static_cast<int64_t>(b) * a.mix_cin * a.So_in;
    x.add1 = a.mix_w + static_cast<int64_t>(oc) * a.So_in;
  } else {
    x.in = static_cast<const char*>(a.in) + static_cast<int64_t>(o) * a.So_in * (BFI ? 2 : 4);
  }
  x.out = static_cast<char*>(a.out) + static_cast<int64_t>(o) * a.So_out * (BFO ? 2 : 4);
  if constexpr (NADD >= 1 && NADD <= 3) x.add1 = static_cast<const char*>(a.add1) + static_cast<int64_t>(o) * a.So_out * (BFO ? 2 : 4);
  if constexpr (NADD == 2) x.add2 = static_cast<const char*>(a.add2) + static_cast<int64_t>(o) * a.So_out * (BFO ? 2 : 4);
  if constexpr (NADD == 3) {
    x.st = reinterpret_cast<const float2*>(a.ln_stats) + static_cast<int64_t>(o) * L;
    const int ch = x.i0c;  // pairvec: channels ch, ch + 1
    x.g = *reinterpret_cast<const float2*>(a.ln_gamma + ch);
    x.be = *reinterpret_cast<const float2*>(a.ln_beta + ch);
    x.pre = a.ln_pre ? *reinterpret_cast<const float2*>(a.ln_pre + ch) : make_float2(0.f, 0.f);
  }
  x.lds = lds;
  x.twl = twl;
  AMD_DFT_STAMP(a, 0, static_cast<long long>(__builtin_amdgcn_s_memrealtime()));
  AMD_DFT_STAMP(a, 1, static_cast<long long>(__builtin_amdgcn_s_memtime()));
  using G0 = PassGeom<F, TP, 0>;
  float2 tw0[G0::Q][G0::TWR];
  Step<K, COLS, TP, T, F, 0, BFI, BFO, PR, NADD, PV>::run(x, tw0);
  if constexpr (K == Kind::R2C) {
    // Z (natural order) is in LDS: separate the two packed real signals' half spectra.
    constexpr int KMAX = L / 2 + 1;
    constexpr int Q2 = (KMAX + TP - 1) / TP;
    const float h = 0.5f * a.scale;
#pragma unroll
    for (int q = 0; q < Q2; ++q) {
      const int k = x.tp + q * TP;
      if (k < a.out_lo) {
        const float2 zk = lds[lidx<COLS, T, L>(x, k)];
        const float2 zm = lds[lidx<COLS, T, L>(x, k == 0 ? 0 : L - k)];
        float2 xa = make_float2((zk.x + zm.x) * h, (zk.y - zm.y) * h);
        float2 xb = make_float2((zk.y + zm.y) * h, (zm.x - zk.x) * h);
        if (a.inverse) { xa.y = -xa.y; xb.y = -xb.y; }
        const int32_t off = x.i0c * a.Si_out + k * a.Sn_out;
        if constexpr (PV) {
          if (x.ok0) st_c2<BFO>(x.out, off, xa, xb);
        } else if (a.vec_out && x.ok1) {  // paired outputs adjacent (transposed rfft2 intermediate)
          st_c2<BFO>(x.out, off, xa, xb);
        } else {
          if (x.ok0) st_c<BFO>(x.out, off, xa);
          if (x.ok1) st_c<BFO>(x.out, x.i1c * a.Si_out + k * a.Sn_out, xb);
        }
      }
    }
  }
  AMD_DFT_STAMP(a, 2, static_cast<long long>(__builtin_amdgcn_s_memtime()));
  AMD_DFT_STAMP(a, 8, static_cast<long long>(__builtin_amdgcn_s_memrealtime()));
}

// LDS image of one tile (float2 entries) for T signal slots
template <bool COLS, int T, int L>
constexpr int tile_lds(int slots = T) {
  return col_pw<COLS, T, L>() > 0 ? L * T + col_pw<COLS, T, L>() * (L / 8 + 1) + 2
         : COLS ? (T >= 4 ? L * (T + 1) + 2 : lds_pad(L * T) + 2) : slots * (lds_padl<COLS, L>(L) + 1);
}

template <Kind K, bool COLS, int TP, int T, class F, bool BFI, bool BFO, bool PR, int NADD, bool PV>
__global__ void __launch_bounds__(TP * T) fft_fixed_kernel(const FixedArgs a) {
  __shared__ __attribute__((aligned(16))) float2 lds[tile_lds<COLS, T, F::L>()];
  const int32_t bid = a.xcd_nb > 0 ? xcd_block(static_cast<int32_t>(blockIdx.x), a.xcd_nb)
                                   : static_cast<int32_t>(blockIdx.x);
  if constexpr (AMD_DFT_TW_LDS) {
    constexpr int TWN = F::goff(F::N) > 0 ? F::goff(F::N) : 1;
    __shared__ float2 twl[TWN];  // filled by pass 0 after its gather loads are issued
    fixed_tile<K, COLS, TP, T, F, BFI, BFO, PR, NADD, PV>(a, bid, static_cast<int>(threadIdx.x), true, lds, twl);
  } else {
    fixed_tile<K, COLS, TP, T, F, BFI, BFO, PR, NADD, PV>(a, bid, static_cast<int>(threadIdx.x), true, lds);
  }
}

// ------------------------------------------------------------------ config table
// The first entry of a length fixes its plan's radix order (fixed_radices; MI_DFT_FFT_RADICES picks
// another configured order for A/B runs).  1440 rows: (5, 6, 6, 8) at 288 threads -- one butterfly
// of 5..8 points per thread per pass, ~4.5 waves per transform -- beat (10, 12, 12) at 144 threads
// (10-12 points per thread, ~2.3 waves) on rfft2 720x1440: 12.27-12.32 vs 12.70-12.78 us, irfft2
// unchanged (12.14-12.23 vs 12.13-12.14); 180-thread (4, 4, 5, 9) 720-point columns lost
// (irfft2 12.36-12.42): profiles/fft_plans_r3.txt.  720 = (24, 30): two passes (one LDS round trip
// fewer) at 30 threads per transform, A/B via MI_DFT_FFT_RADICES="720:24,30" (round 4).
#define AMD_DFT_FIXED_CONFIGS(X)          \
  X(1440, false, 288, 1, 5, 6, 6, 8)      \
  X(1440, false, 144, 1, 10, 12, 12)      \
  X(720, false, 90, 2, 8, 9, 10)          \
  X(1024, false, 128, 1, 8, 8, 16)        \
  X(2048, false, 256, 1, 8, 16, 16)       \
  X(512, false, 64, 2, 8, 8, 8)           \
  X(256, false, 16, 4, 16, 16)            \
  X(720, false, 30, 2, 24, 30)            \
  X(720, true, 90, 4, 8, 9, 10)           \
  X(720, true, 90, 2, 8, 9, 10)           \
  X(720, true, 45, 8, 8, 9, 10)           \
  X(720, true, 45, 4, 8, 9, 10)           \
  X(720, true, 90, 8, 8, 9, 10)           \
  X(720, true, 45, 16, 8, 9, 10)          \
  X(720, true, 30, 4, 24, 30)             \
  X(720, true, 30, 8, 24, 30)             \
  X(90, true, 10, 16, 9, 10)              \
  X(180, true, 15, 16, 12, 15)            \
  X(180, true, 15, 32, 12, 15)

template <Kind K, bool COLS, int TP, int T, class F, bool PR, int NADD, bool PV>
void launch_dt(const FixedArgs& a, dim3 grid, hipStream_t st) {
  const dim3 blk(TP * T);
  if (a.bf16_in) {
    if (a.bf16_out) hipLaunchKernelGGL((fft_fixed_kernel<K, COLS, TP, T, F, true, true, PR, NADD, PV>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((fft_fixed_kernel<K, COLS, TP, T, F, true, false, PR, NADD, PV>), grid, blk, 0, st, a);
  } else {
    if (a.bf16_out) hipLaunchKernelGGL((fft_fixed_kernel<K, COLS, TP, T, F, false, true, PR, NADD, PV>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((fft_fixed_kernel<K, COLS, TP, T, F, false, false, PR, NADD, PV>), grid, blk, 0, st, a);
  }
}

template <Kind K, bool COLS, int TP, int T, class F>
void launch_one(const FixedArgs& a, dim3 grid, hipStream_t st) {
  // pruned C2C (FNO/AFNO mode windows) gets its own instantiation; R2C/C2R handle their
  // (cheap, Hermitian) truncation in the common path.  Column layouts (channel-last) get the
  // paired-vector variant (PV) and the C2R addend epilogue (NADD).
  const bool pr = K == Kind::C2C && (a.in_lo + a.in_hi != F::L || a.out_lo + a.out_hi != F::L);
  if constexpr (K == Kind::C2C && COLS) {
    if (a.mix_w) {  // FNO mixing gather: fp32 pruned column transforms only (host-checked)
      hipLaunchKernelGGL((fft_fixed_kernel<K, COLS, TP, T, F, false, false, true, 4, false>), grid, dim3(TP * T), 0, st, a);
      return;
    }
  }
  if constexpr (K == Kind::C2C) {
    if (pr) return launch_dt<K, COLS, TP, T, F, true, 0, false>(a, grid, st);
  }
  if constexpr (COLS && K != Kind::C2C) {
    if (a.ln_stats) {  // LayerNorm IO: bf16 channel-last pairs only (host-checked)
      if (a.bf16_in && a.bf16_out && a.pairvec)
        hipLaunchKernelGGL((fft_fixed_kernel<K, COLS, TP, T, F, true, true, false, 3, true>), grid, dim3(TP * T), 0, st, a);
      return;
    }
    if (a.pairvec) {
      if constexpr (K == Kind::C2R) {
        if (a.add2) return launch_dt<K, COLS, TP, T, F, false, 2, true>(a, grid, st);
        if (a.add1) return launch_dt<K, COLS, TP, T, F, false, 1, true>(a, grid, st);
      }
      return launch_dt<K, COLS, TP, T, F, false, 0, true>(a, grid, st);
    }
    if constexpr (K == Kind::C2R) {
      if (a.add2) return launch_dt<K, COLS, TP, T, F, false, 2, false>(a, grid, st);
      if (a.add1) return launch_dt<K, COLS, TP, T, F, false, 1, false>(a, grid, st);
    }
  }
  if constexpr (!COLS && K == Kind::C2R) {
    if (a.add2) return launch_dt<K, COLS, TP, T, F, false, 2, false>(a, grid, st);
    if (a.add1) return launch_dt<K, COLS, TP, T, F, false, 1, false>(a, grid, st);
  }
  launch_dt<K, COLS, TP, T, F, false, 0, false>(a, grid, st);
}

using LaunchFn = void (*)(const FixedArgs&, dim3, hipStream_t);
// per-kind launcher tables, index = position in AMD_DFT_FIXED_CONFIGS
LaunchFn c2c_launcher(int idx);
LaunchFn r2c_launcher(int idx);
LaunchFn c2r_launcher(int idx);

}  // namespace fixed_detail
}  // namespace amd_dft
