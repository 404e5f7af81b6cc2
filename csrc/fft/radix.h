// Register-resident forward DFT butterflies for the Stockham passes (gfx950).
//
// Dft<R>::run(v) transforms R complex values held in registers (fully unrolled;
// every root of unity is a compile-time constant from radix_consts.h).
// Supported radices: 2,3,4,5,6,7,8,9,10,11,12,13,15,16 (composites are
// built Cooley-Tukey style from the small ones).  The inverse transform is
// obtained by conjugating input and output (conj(DFT(conj x))), so only the
// forward butterflies exist.
#pragma once

#include <hip/hip_runtime.h>

#include "radix_consts.h"

namespace amd_dft {

// One complex value as (re, im) in a register pair: every add / sub / scale is ONE packed fp32
// instruction (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32; broadcasts and the re/im swap of a
// quarter turn fold into op_sel / neg modifiers), half the VALU issue of the scalar form.  The
// FFT passes are VALU-issue bound at about one wave per SIMD (profiles/fft_xcd_r2.txt), so the
// instruction count per point is their cost.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v v2(float2 a) { return f2v{a.x, a.y}; }
__device__ __forceinline__ float2 f2(f2v a) { return make_float2(a.x, a.y); }
__device__ __forceinline__ float2 c_add(float2 a, float2 b) { return f2(v2(a) + v2(b)); }
__device__ __forceinline__ float2 c_sub(float2 a, float2 b) { return f2(v2(a) - v2(b)); }
__device__ __forceinline__ float2 c_neg(float2 a) { return f2(-v2(a)); }
__device__ __forceinline__ float2 c_mul(float2 a, float2 b) {  // (ax bx - ay by, ax by + ay bx)
  const f2v va = v2(a), vb = v2(b);
  return f2(__builtin_elementwise_fma(va.yy, f2v{-vb.y, vb.x}, va.xx * vb));
}
// a * e^{-i theta} with (c, s) = (cos theta, sin theta): (ax c + ay s, ay c - ax s)
__device__ __forceinline__ float2 c_mul_w(float2 a, float c, float s) {
  const f2v va = v2(a);
  return f2(__builtin_elementwise_fma(va.yx, f2v{s, -s}, va * f2v{c, c}));
}
__device__ __forceinline__ float2 c_mul_negi(float2 a) { return make_float2(a.y, -a.x); }  // -i*a
__device__ __forceinline__ float2 c_mul_posi(float2 a) { return make_float2(-a.y, a.x); }  //  i*a
__device__ __forceinline__ float2 c_scale(float2 a, float s) { return f2(v2(a) * f2v{s, s}); }
__device__ __forceinline__ float2 c_fmas(float s, float2 a, float2 acc) {  // acc + s * a
  return f2(__builtin_elementwise_fma(f2v{s, s}, v2(a), v2(acc)));
}

// Two complex signals that share every twiddle (e.g. two adjacent channels of a batched FFT),
// held as planes: re = (re0, re1), im = (im0, im1).  Every butterfly op is then one packed
// fp32 instruction (v_pk_add/mul/fma_f32) per plane with no re/im shuffles, and a quarter
// turn (+-i) is a free plane swap -- half the VALU issue of two scalar float2 signals.
struct cpair {
  f2v re, im;
};
__device__ __forceinline__ cpair make_cpair(float2 a, float2 b) { return cpair{f2v{a.x, b.x}, f2v{a.y, b.y}}; }
__device__ __forceinline__ float2 cpair_lo(const cpair& v) { return make_float2(v.re[0], v.im[0]); }
__device__ __forceinline__ float2 cpair_hi(const cpair& v) { return make_float2(v.re[1], v.im[1]); }
__device__ __forceinline__ cpair c_add(cpair a, cpair b) { return cpair{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cpair c_sub(cpair a, cpair b) { return cpair{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cpair c_neg(cpair a) { return cpair{-a.re, -a.im}; }
// w.y goes through its own register first: broadcast straight from the pair, the compiler takes it as the high half
// of src1 through op_sel (v_pk_mul_f32 ... op_sel:[0,1]), and on gfx950 such packed-FP32 ops return wrong products
// while another wave on the same SIMD executes MFMAs (profiles/afno_o3_bisect_r3.txt,
// scripts/diag/opsel_lds_repro.hip); from its own register the broadcast reads the low half of a pair (unaffected).
__device__ __forceinline__ cpair c_mul(cpair a, float2 w) {
  float wy;
  asm("v_mov_b32 %0, %1" : "=v"(wy) : "v"(w.y));
  return cpair{a.re * w.x - a.im * wy, a.re * wy + a.im * w.x};
}
__device__ __forceinline__ cpair c_mul_w(cpair a, float c, float s) { return cpair{a.re * c + a.im * s, a.im * c - a.re * s}; }
__device__ __forceinline__ cpair c_mul_negi(cpair a) { return cpair{a.im, -a.re}; }
__device__ __forceinline__ cpair c_mul_posi(cpair a) { return cpair{-a.im, a.re}; }
__device__ __forceinline__ cpair c_scale(cpair a, float s) { return cpair{a.re * s, a.im * s}; }
__device__ __forceinline__ cpair c_fmas(float s, cpair a, cpair acc) { return cpair{s * a.re + acc.re, s * a.im + acc.im}; }

// Multiply by w_R^m = e^{-2 pi i m / R}, exact for the quarter turns.
template <int R, class T>
__device__ __forceinline__ T c_rot(T a, int m) {
  m %= R;
  if (m == 0) return a;
  if (4 * m == R) return c_mul_negi(a);
  if (2 * m == R) return c_neg(a);
  if (4 * m == 3 * R) return c_mul_posi(a);
  return c_mul_w(a, RootTab<R>::c[m], RootTab<R>::s[m]);
}

template <int R>
struct Dft;

template <>
struct Dft<1> {
  template <class T>
  __device__ __forceinline__ static void run(T*) {}
};

template <>
struct Dft<2> {
  template <class T>
  __device__ __forceinline__ static void run(T* v) {
    const T a = v[0], b = v[1];
    v[0] = c_add(a, b);
    v[1] = c_sub(a, b);
  }
};

template <>
struct Dft<4> {
  template <class T>
  __device__ __forceinline__ static void run(T* v) {
    const T y0 = c_add(v[0], v[2]), y1 = c_sub(v[0], v[2]);
    const T y2 = c_add(v[1], v[3]), y3 = c_mul_negi(c_sub(v[1], v[3]));
    v[0] = c_add(y0, y2);
    v[2] = c_sub(y0, y2);
    v[1] = c_add(y1, y3);
    v[3] = c_sub(y1, y3);
  }
};

template <>
struct Dft<8> {
  template <class T>
  __device__ __forceinline__ static void run(T* v) {
    constexpr float r = 0.70710678118654752f;
    T e[4], o[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      e[n] = c_add(v[n], v[n + 4]);
      o[n] = c_sub(v[n], v[n + 4]);
    }
    // o[n] *= w8^n
    o[1] = c_scale(c_add(o[1], c_mul_negi(o[1])), r);  // ((x + y) r, (y - x) r)
    o[2] = c_mul_negi(o[2]);
    o[3] = c_scale(c_sub(c_mul_negi(o[3]), o[3]), r);  // ((y - x) r, -(x + y) r)
    Dft<4>::run(e);
    Dft<4>::run(o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = e[k];
      v[2 * k + 1] = o[k];
    }
  }
};

// Odd prime radix: pairwise symmetric form (R-1)^2/2 real FMAs per component.
template <int R>
struct DftOdd {
  template <class T>
  __device__ __forceinline__ static void run(T* v) {
    constexpr int H = (R - 1) / 2;
    T t[H], d[H];
#pragma unroll
    for (int m = 1; m <= H; ++m) {
      t[m - 1] = c_add(v[m], v[R - m]);
      d[m - 1] = c_sub(v[m], v[R - m]);
    }
    const T x0 = v[0];
    T sum = x0;
#pragma unroll
    for (int m = 0; m < H; ++m) sum = c_add(sum, t[m]);
#pragma unroll
    for (int q = 1; q <= H; ++q) {
      T re = c_fmas(RootTab<R>::c[q % R], t[0], x0);
      T im = c_scale(d[0], RootTab<R>::s[q % R]);
#pragma unroll
      for (int m = 2; m <= H; ++m) {
        const int idx = (m * q) % R;
        re = c_fmas(RootTab<R>::c[idx], t[m - 1], re);
        im = c_fmas(RootTab<R>::s[idx], d[m - 1], im);
      }
      // X_q = re - i*im ; X_{R-q} = re + i*im
      v[q] = c_add(re, c_mul_negi(im));
      v[R - q] = c_sub(re, c_mul_negi(im));
    }
    v[0] = sum;
  }
};

template <> struct Dft<3> : DftOdd<3> {};
template <> struct Dft<5> : DftOdd<5> {};
template <> struct Dft<7> : DftOdd<7> {};
template <> struct Dft<11> : DftOdd<11> {};
template <> struct Dft<13> : DftOdd<13> {};

// Composite A*B: n = B*n1 + n2, k = k1 + A*k2.
template <int A, int B>
struct DftComp {
  template <class T>
  __device__ __forceinline__ static void run(T* v) {
    constexpr int R = A * B;
    T y[R];
#pragma unroll
    for (int n2 = 0; n2 < B; ++n2) {
      T s[A];
#pragma unroll
      for (int n1 = 0; n1 < A; ++n1) s[n1] = v[B * n1 + n2];
      Dft<A>::run(s);
#pragma unroll
      for (int k1 = 0; k1 < A; ++k1) y[k1 * B + n2] = c_rot<R, T>(s[k1], n2 * k1);
    }
#pragma unroll
    for (int k1 = 0; k1 < A; ++k1) {
      T s[B];
#pragma unroll
      for (int n2 = 0; n2 < B; ++n2) s[n2] = y[k1 * B + n2];
      Dft<B>::run(s);
#pragma unroll
      for (int k2 = 0; k2 < B; ++k2) v[k1 + A * k2] = s[k2];
    }
  }
};

template <> struct Dft<6> : DftComp<2, 3> {};
template <> struct Dft<9> : DftComp<3, 3> {};
template <> struct Dft<10> : DftComp<2, 5> {};
template <> struct Dft<12> : DftComp<4, 3> {};
template <> struct Dft<15> : DftComp<3, 5> {};
template <> struct Dft<16> : DftComp<4, 4> {};
// fixed-kernel-only radices (two-pass 720 = 24 x 30; never picked by the generic planner's search)
template <> struct Dft<24> : DftComp<8, 3> {};
template <> struct Dft<30> : DftComp<10, 3> {};

}  // namespace amd_dft
