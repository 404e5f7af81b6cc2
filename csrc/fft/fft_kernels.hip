// LDS-resident mixed-radix Stockham FFT pass kernels for gfx950 (MI355X).
//
// One workgroup transforms T complex signals of length L that live along one tensor
// axis (any element stride), staged through LDS in an interleaved [n][t] layout so that
// both row-like (stride-1 along n) and column-like (stride-1 along the signal index)
// global accesses coalesce.  Each Stockham pass reads R values per butterfly from one
// LDS buffer, applies LDS-staged twiddles, runs a register-resident radix-R DFT
// (radix.h) and writes the other buffer (ping-pong: one barrier per pass).
//
// R2C packs two real signals into one complex FFT (z = a + i b) and separates the two
// half spectra at store time; C2R assembles z from two Hermitian half spectra at load
// time.  Normalisation is fused into the final store (the reference issues a separate
// cublasScalEx for it: /root/reference/src/dft_plugins/dft_plugins.cpp:457-468).
// Kernels never write their input (cuFFT may for C2R: SURVEY Q8).

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "fft_desc.h"
#include "fft_fixed.h"
#include "radix.h"

namespace amd_dft {

namespace {

using bf16_t = uint16_t;

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// ---------------------------------------------------------------- element IO
template <typename T> struct IO;

template <> struct IO<float> {
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static float2 ld2(const float* p) { return *reinterpret_cast<const float2*>(p); }
  __device__ __forceinline__ static float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
  __device__ __forceinline__ static void st2(float* p, float2 v) { *reinterpret_cast<float2*>(p) = v; }
  __device__ __forceinline__ static void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
};

__device__ __forceinline__ float bf2f(uint32_t u16) { return __uint_as_float(u16 << 16); }
__device__ __forceinline__ uint32_t f2bf(float f) {
  return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<__bf16>(f)));
}

template <> struct IO<bf16_t> {
  __device__ __forceinline__ static float ld(const bf16_t* p) { return bf2f(*p); }
  __device__ __forceinline__ static float2 ld2(const bf16_t* p) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
    return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
  }
  __device__ __forceinline__ static float4 ld4(const bf16_t* p) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
  __device__ __forceinline__ static void st(bf16_t* p, float v) { *p = static_cast<bf16_t>(f2bf(v)); }
  __device__ __forceinline__ static void st2(bf16_t* p, float2 v) {
    *reinterpret_cast<uint32_t*>(p) = f2bf(v.x) | (f2bf(v.y) << 16);
  }
  __device__ __forceinline__ static void st4(bf16_t* p, float4 v) {
    *reinterpret_cast<uint2*>(p) =
        make_uint2(f2bf(v.x) | (f2bf(v.y) << 16), f2bf(v.z) | (f2bf(v.w) << 16));
  }
};

// LDS index with one float2 of padding every 16 entries: breaks the stride-R write
// pattern of the first Stockham pass (16-way bank conflict -> conflict-free per
// 16-lane ds_write_b64 group).
__device__ __forceinline__ int lds_ix(int i) { return i + (i >> 4); }

// ---------------------------------------------------------------- one Stockham pass
template <int R>
__device__ __forceinline__ void stockham_pass(const float2* __restrict__ src, float2* __restrict__ dst,
                                              const float2* __restrict__ tw, int L, int logT, int Ns,
                                              const FastDiv& ns_div) {
  const int T = 1 << logT;
  const int LR = L / R;
  const int nb = LR << logT;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const int t = b & (T - 1);
    const int j = b >> logT;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = src[lds_ix(((j + r * LR) << logT) + t)];
    const int k = j - static_cast<int>(fdiv(static_cast<uint32_t>(j), ns_div)) * Ns;
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = c_mul(v[r], tw[(r - 1) * Ns + k]);
    }
    Dft<R>::run(v);
    const int base = (j - k) * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) dst[lds_ix(((base + r * Ns) << logT) + t)] = v[r];
  }
}

// Any radix (large primes): O(R^2) straight from LDS, roots of unity from the table.
__device__ void stockham_pass_generic(const float2* __restrict__ src, float2* __restrict__ dst,
                                      const float2* __restrict__ tw, const float2* __restrict__ roots,
                                      int R, int L, int logT, int Ns, const FastDiv& ns_div) {
  const int T = 1 << logT;
  const int LR = L / R;
  const int nb = LR << logT;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const int t = b & (T - 1);
    const int j = b >> logT;
    const int k = j - static_cast<int>(fdiv(static_cast<uint32_t>(j), ns_div)) * Ns;
    const int base = (j - k) * R + k;
    for (int q = 0; q < R; ++q) {
      float2 acc = make_float2(0.f, 0.f);
      int e = 0;  // (r*q) mod R
      for (int r = 0; r < R; ++r) {
        float2 a = src[lds_ix(((j + r * LR) << logT) + t)];
        if (r > 0 && Ns > 1) a = c_mul(a, tw[(r - 1) * Ns + k]);
        acc = c_add(acc, c_mul(a, roots[e]));
        e += q;
        if (e >= R) e -= R;
      }
      dst[lds_ix(((base + q * Ns) << logT) + t)] = acc;
    }
  }
}

__device__ __forceinline__ int stored_index(int n, int L, int lo, int hi) {
  if (n < lo) return n;
  if (n >= L - hi) return lo + (n - (L - hi));
  return -1;
}

// ---------------------------------------------------------------- kernel
template <Kind K, typename TI, typename TO>
__global__ void __launch_bounds__(256) fft_pass_kernel(const PassDesc d) {
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int L = d.L;
  const int logT = d.logT;
  const int T = 1 << logT;
  const int tid = threadIdx.x;
  const int nth = blockDim.x;
  const int twc = (d.tw_count + 1) & ~1;
  const int bufsz = lds_ix(L * T) + 2;
  float2* tw_s = smem;
  float2* buf0 = smem + twc;
  float2* buf1 = buf0 + ((bufsz + 1) & ~1);

  const int64_t o = blockIdx.x / d.tiles_per_outer;
  const int64_t tile = blockIdx.x - o * d.tiles_per_outer;
  const TI* __restrict__ in = static_cast<const TI*>(d.in) + o * d.So_in;
  TO* __restrict__ out = static_cast<TO*>(d.out) + o * d.So_out;
  const float2* __restrict__ twg = static_cast<const float2*>(d.tw);

  // Twiddles: 8 loads in flight per thread before the LDS writes.
  for (int base = tid; base < d.tw_count; base += 8 * nth) {
    float2 w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * nth;
      w[u] = twg[i < d.tw_count ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * nth;
      if (i < d.tw_count) tw_s[i] = w[u];
    }
  }

  // signals of this tile: complex index c = tile*T + t; logical signals for R2C/C2R are
  // (2c, 2c+1).
  const int64_t c0 = tile * T;
  const bool nfast_in = d.Sn_in < d.Si_in || d.I == 1;
  const int nload = L << logT;

  // ------------------------------------------------------------ load (+ C2R assembly)
  // LOADU independent global loads are issued per thread before any LDS write so that the
  // HBM/L2 latency is paid once per batch, not once per element.
  constexpr int LOADU = 8;
  for (int base = tid; base < nload; base += LOADU * nth) {
  float2 zb[LOADU];
  int lpos[LOADU];
#pragma unroll
  for (int u = 0; u < LOADU; ++u) {
    // Unconditional loads from clamped addresses + selects: a branch around a load makes
    // hipcc wait vmcnt(0) per element.
    const int idx_raw = base + u * nth;
    const bool in_range = idx_raw < nload;
    const int idx = in_range ? idx_raw : 0;
    int t, n;
    if (nfast_in) {
      t = static_cast<int>(fdiv(static_cast<uint32_t>(idx), d.L_div));
      n = idx - t * L;
    } else {
      t = idx & (T - 1);
      n = idx >> logT;
    }
    float2 z;
    if constexpr (K == Kind::C2C) {
      const int64_t i = c0 + t;
      const int s = stored_index(n, L, d.in_lo, d.in_hi);
      const bool ok = i < d.I && s >= 0;
      const int64_t ic = i < d.I ? i : d.I - 1;
      z = IO<TI>::ld2(in + ic * d.Si_in + (s < 0 ? 0 : s) * d.Sn_in);
      z = make_float2(ok ? z.x : 0.f, ok ? z.y : 0.f);
      if (d.inverse) z.y = -z.y;
    } else if constexpr (K == Kind::R2C) {
      const int64_t i0 = 2 * (c0 + t);
      const bool ok0 = i0 < d.I, ok1 = i0 + 1 < d.I;
      const float va = IO<TI>::ld(in + (ok0 ? i0 : d.I - 1) * d.Si_in + n * d.Sn_in);
      const float vb = IO<TI>::ld(in + (ok1 ? i0 + 1 : d.I - 1) * d.Si_in + n * d.Sn_in);
      z = make_float2(ok0 ? va : 0.f, ok1 ? vb : 0.f);
    } else {  // C2R: z = A + iB with A, B the Hermitian extensions of the two half spectra
      const int64_t i0 = 2 * (c0 + t);
      const bool ok0 = i0 < d.I, ok1 = i0 + 1 < d.I;
      const bool upper = 2 * n > L;
      const int kk = upper ? L - n : n;
      const bool okk = kk < d.in_lo;
      const int kc = okk ? kk : 0;
      float2 A = IO<TI>::ld2(in + (ok0 ? i0 : d.I - 1) * d.Si_in + kc * d.Sn_in);
      float2 B = IO<TI>::ld2(in + (ok1 ? i0 + 1 : d.I - 1) * d.Si_in + kc * d.Sn_in);
      A = make_float2(okk && ok0 ? A.x : 0.f, okk && ok0 ? A.y : 0.f);
      B = make_float2(okk && ok1 ? B.x : 0.f, okk && ok1 ? B.y : 0.f);
      if (kk == 0 || 2 * kk == L) { A.y = 0.f; B.y = 0.f; }
      if (upper) { A.y = -A.y; B.y = -B.y; }
      z = make_float2(A.x - B.y, A.y + B.x);
      if (d.inverse) z.y = -z.y;
    }
    zb[u] = z;
    lpos[u] = in_range ? lds_ix((n << logT) + t) : -1;
  }
#pragma unroll
  for (int u = 0; u < LOADU; ++u)
    if (lpos[u] >= 0) buf0[lpos[u]] = zb[u];
  }
  __syncthreads();

  // ------------------------------------------------------------ Stockham passes
  float2* src = buf0;
  float2* dst = buf1;
  for (int p = 0; p < d.npass; ++p) {
    const int R = d.radix[p];
    const int Ns = d.ns[p];
    const float2* tw = tw_s + d.twoff[p];
    switch (R) {
      case 2: stockham_pass<2>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 3: stockham_pass<3>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 4: stockham_pass<4>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 5: stockham_pass<5>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 6: stockham_pass<6>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 7: stockham_pass<7>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 8: stockham_pass<8>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 9: stockham_pass<9>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 10: stockham_pass<10>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 11: stockham_pass<11>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 12: stockham_pass<12>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 13: stockham_pass<13>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 15: stockham_pass<15>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 16: stockham_pass<16>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 24: stockham_pass<24>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      case 30: stockham_pass<30>(src, dst, tw, L, logT, Ns, d.ns_div[p]); break;
      default:
        stockham_pass_generic(src, dst, tw, tw_s + d.rootoff[p], R, L, logT, Ns, d.ns_div[p]);
        break;
    }
    __syncthreads();
    float2* tmp = src;
    src = dst;
    dst = tmp;
  }

  // ------------------------------------------------------------ store
  const float sc = d.scale;
  const bool nfast_out = d.Sn_out < d.Si_out || d.I == 1;
  if constexpr (K == Kind::C2C) {
    const int nst = d.out_lo + d.out_hi;
    const int total = nst << logT;
    for (int idx = tid; idx < total; idx += nth) {
      int t, s;
      if (nfast_out) {
        t = static_cast<int>(fdiv(static_cast<uint32_t>(idx), d.out_div));
        s = idx - t * nst;
      } else {
        t = idx & (T - 1);
        s = idx >> logT;
      }
      const int64_t i = c0 + t;
      if (i >= d.I) continue;
      const int n = s < d.out_lo ? s : L - d.out_hi + (s - d.out_lo);
      float2 v = src[lds_ix((n << logT) + t)];
      if (d.inverse) v.y = -v.y;
      IO<TO>::st2(out + i * d.Si_out + s * d.Sn_out, c_scale(v, sc));
    }
  } else if constexpr (K == Kind::R2C) {
    const int nst = d.out_lo;
    const int total = nst << logT;
    const float h = 0.5f * sc;
    for (int idx = tid; idx < total; idx += nth) {
      int t, k;
      if (nfast_out) {
        t = static_cast<int>(fdiv(static_cast<uint32_t>(idx), d.out_div));
        k = idx - t * nst;
      } else {
        t = idx & (T - 1);
        k = idx >> logT;
      }
      const int64_t i0 = 2 * (c0 + t);
      if (i0 >= d.I) continue;
      const float2 zk = src[lds_ix((k << logT) + t)];
      const int km = k == 0 ? 0 : L - k;
      const float2 zm = src[lds_ix((km << logT) + t)];
      // Xa = (Zk + conj Zm)/2 ; Xb = (Zk - conj Zm)/(2i)
      float2 xa = make_float2((zk.x + zm.x) * h, (zk.y - zm.y) * h);
      float2 xb = make_float2((zk.y + zm.y) * h, (zm.x - zk.x) * h);
      if (d.inverse) { xa.y = -xa.y; xb.y = -xb.y; }
      TO* p = out + i0 * d.Si_out + k * d.Sn_out;
      if (d.vec_out && i0 + 1 < d.I) {
        IO<TO>::st4(p, make_float4(xa.x, xa.y, xb.x, xb.y));
      } else {
        IO<TO>::st2(p, xa);
        if (i0 + 1 < d.I) IO<TO>::st2(p + d.Si_out, xb);
      }
    }
  } else {  // C2R
    const int total = L << logT;
    for (int idx = tid; idx < total; idx += nth) {
      int t, n;
      if (nfast_out) {
        t = static_cast<int>(fdiv(static_cast<uint32_t>(idx), d.L_div));
        n = idx - t * L;
      } else {
        t = idx & (T - 1);
        n = idx >> logT;
      }
      const int64_t i0 = 2 * (c0 + t);
      if (i0 >= d.I) continue;
      const float2 y = src[lds_ix((n << logT) + t)];
      float a = y.x * sc;
      float b = (d.inverse ? -y.y : y.y) * sc;
      TO* p = out + i0 * d.Si_out + n * d.Sn_out;
      const int64_t poff = (p - static_cast<TO*>(d.out));
      if (d.add1) {
        a += IO<TO>::ld(static_cast<const TO*>(d.add1) + poff);
        if (i0 + 1 < d.I) b += IO<TO>::ld(static_cast<const TO*>(d.add1) + poff + d.Si_out);
      }
      if (d.add2) {
        a += IO<TO>::ld(static_cast<const TO*>(d.add2) + poff);
        if (i0 + 1 < d.I) b += IO<TO>::ld(static_cast<const TO*>(d.add2) + poff + d.Si_out);
      }
      if (d.vec_out && i0 + 1 < d.I) {
        IO<TO>::st2(p, make_float2(a, b));
      } else {
        IO<TO>::st(p, a);
        if (i0 + 1 < d.I) IO<TO>::st(p + d.Si_out, b);
      }
    }
  }
}

template <Kind K, typename TI, typename TO>
void launch_t(const PassDesc& d, hipStream_t st) {
  const int64_t lds = pass_lds_bytes(d);
  const int64_t nblocks = d.O * d.tiles_per_outer;
  if (nblocks <= 0) return;
  if (nblocks > 0x7fffffffLL) throw std::runtime_error("amd_dft: FFT grid too large");
  auto kern = fft_pass_kernel<K, TI, TO>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: hipFuncSetAttribute: ") + hipGetErrorString(e));
  }
  hipLaunchKernelGGL(kern, dim3(static_cast<uint32_t>(nblocks)), dim3(d.nthreads), static_cast<size_t>(lds), st, d);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: FFT pass launch failed: ") + hipGetErrorString(e));
}

template <Kind K>
void launch_k(const PassDesc& d, hipStream_t st) {
  if (d.tin == DType::F32 && d.tout == DType::F32) return launch_t<K, float, float>(d, st);
  if (d.tin == DType::BF16 && d.tout == DType::F32) return launch_t<K, bf16_t, float>(d, st);
  if (d.tin == DType::F32 && d.tout == DType::BF16) return launch_t<K, float, bf16_t>(d, st);
  return launch_t<K, bf16_t, bf16_t>(d, st);
}

}  // namespace

int64_t pass_lds_bytes(const PassDesc& d) {
  const int64_t twc = (d.tw_count + 1) & ~1;
  const int64_t n = static_cast<int64_t>(d.L) << d.logT;
  const int64_t bufsz = ((n + (n >> 4) + 2) + 1) & ~1;
  return (twc + 2 * bufsz) * static_cast<int64_t>(sizeof(float2));
}

void launch_fft_pass(const PassDesc& d, void* stream) {
  if (launch_fft_fixed(d, stream)) return;
  if (d.ln_stats) throw std::runtime_error("amd_dft: LayerNorm-fused pass needs a specialised (fixed) kernel");
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (d.kind) {
    case Kind::C2C: return launch_k<Kind::C2C>(d, st);
    case Kind::R2C: return launch_k<Kind::R2C>(d, st);
    case Kind::C2R: return launch_k<Kind::C2R>(d, st);
  }
}

}  // namespace amd_dft
