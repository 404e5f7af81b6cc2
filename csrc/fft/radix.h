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

__device__ __forceinline__ float2 c_add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 c_sub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 c_mul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// a * e^{-i theta} with (c, s) = (cos theta, sin theta)
__device__ __forceinline__ float2 c_mul_w(float2 a, float c, float s) {
  return make_float2(a.x * c + a.y * s, a.y * c - a.x * s);
}
__device__ __forceinline__ float2 c_mul_negi(float2 a) { return make_float2(a.y, -a.x); }  // -i*a
__device__ __forceinline__ float2 c_mul_posi(float2 a) { return make_float2(-a.y, a.x); }  //  i*a
__device__ __forceinline__ float2 c_scale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

// Multiply by w_R^m = e^{-2 pi i m / R}, exact for the quarter turns.
template <int R>
__device__ __forceinline__ float2 c_rot(float2 a, int m) {
  m %= R;
  if (m == 0) return a;
  if (4 * m == R) return c_mul_negi(a);
  if (2 * m == R) return make_float2(-a.x, -a.y);
  if (4 * m == 3 * R) return c_mul_posi(a);
  return c_mul_w(a, RootTab<R>::c[m], RootTab<R>::s[m]);
}

template <int R>
struct Dft;

template <>
struct Dft<1> {
  __device__ __forceinline__ static void run(float2*) {}
};

template <>
struct Dft<2> {
  __device__ __forceinline__ static void run(float2* v) {
    const float2 a = v[0], b = v[1];
    v[0] = c_add(a, b);
    v[1] = c_sub(a, b);
  }
};

template <>
struct Dft<4> {
  __device__ __forceinline__ static void run(float2* v) {
    const float2 y0 = c_add(v[0], v[2]), y1 = c_sub(v[0], v[2]);
    const float2 y2 = c_add(v[1], v[3]), y3 = c_mul_negi(c_sub(v[1], v[3]));
    v[0] = c_add(y0, y2);
    v[2] = c_sub(y0, y2);
    v[1] = c_add(y1, y3);
    v[3] = c_sub(y1, y3);
  }
};

template <>
struct Dft<8> {
  __device__ __forceinline__ static void run(float2* v) {
    constexpr float r = 0.70710678118654752f;
    float2 e[4], o[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      e[n] = c_add(v[n], v[n + 4]);
      o[n] = c_sub(v[n], v[n + 4]);
    }
    // o[n] *= w8^n
    o[1] = make_float2((o[1].x + o[1].y) * r, (o[1].y - o[1].x) * r);
    o[2] = c_mul_negi(o[2]);
    o[3] = make_float2((o[3].y - o[3].x) * r, -(o[3].x + o[3].y) * r);
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
  __device__ __forceinline__ static void run(float2* v) {
    constexpr int H = (R - 1) / 2;
    float2 t[H], d[H];
#pragma unroll
    for (int m = 1; m <= H; ++m) {
      t[m - 1] = c_add(v[m], v[R - m]);
      d[m - 1] = c_sub(v[m], v[R - m]);
    }
    const float2 x0 = v[0];
    float2 sum = x0;
#pragma unroll
    for (int m = 0; m < H; ++m) sum = c_add(sum, t[m]);
#pragma unroll
    for (int q = 1; q <= H; ++q) {
      float2 re = x0, im = make_float2(0.f, 0.f);
#pragma unroll
      for (int m = 1; m <= H; ++m) {
        const int idx = (m * q) % R;
        const float c = RootTab<R>::c[idx], s = RootTab<R>::s[idx];
        re.x = fmaf(c, t[m - 1].x, re.x);
        re.y = fmaf(c, t[m - 1].y, re.y);
        im.x = fmaf(s, d[m - 1].x, im.x);
        im.y = fmaf(s, d[m - 1].y, im.y);
      }
      // X_q = re - i*im ; X_{R-q} = re + i*im
      v[q] = make_float2(re.x + im.y, re.y - im.x);
      v[R - q] = make_float2(re.x - im.y, re.y + im.x);
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
  __device__ __forceinline__ static void run(float2* v) {
    constexpr int R = A * B;
    float2 y[R];
#pragma unroll
    for (int n2 = 0; n2 < B; ++n2) {
      float2 s[A];
#pragma unroll
      for (int n1 = 0; n1 < A; ++n1) s[n1] = v[B * n1 + n2];
      Dft<A>::run(s);
#pragma unroll
      for (int k1 = 0; k1 < A; ++k1) y[k1 * B + n2] = c_rot<R>(s[k1], n2 * k1);
    }
#pragma unroll
    for (int k1 = 0; k1 < A; ++k1) {
      float2 s[B];
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

}  // namespace amd_dft
