// FNO layer tail in one kernel: inverse real DFT along W of the kept modes (as an MFMA GEMM),
// + the 1x1 convolution of the layer input (MFMA), + bias, + GELU, one store of the output.
//
//   y[b,o,h,w] = act( sum_{k<m} s_k Re(Y[b,o,h,k] e^{2 pi i k w/W}) + sum_i Wc[o,i] x[b,i,h,w] + bias[o] )
//
// Replaces C2R-along-W (writes the full-resolution spectral output) + a pointwise kernel
// (reads it back): the only HBM traffic left is reading x and writing y.
//
// GEMM orientation: C[m = pixel][n = out channel] so a lane's accumulator holds 4 consecutive
// pixels of one channel (8/16-byte stores).  Per CH-pixel chunk starting at w0:
//   spec:  A = G[k'][px]  (bf16 hi/lo fragments of s_k cos / -s_k sin, identical for every chunk,
//          staged once per workgroup in LDS),  B = Y rotated by e^{2 pi i k w0/W} (fp32 in
//          registers, split hi/lo per chunk) -- the same phase factorisation as dft_gemm.hip.
//          bf16 output: G hi and Y hi only (bf16 MFMA operands, fp32 accumulation, the precision
//          of a bf16 nn.Linear); the Y lo plane would only refine an operand whose partner G is
//          already rounded to bf16 (FNO_BF_YLO=1 restores it: 8 instead of 4 spectral MFMAs per
//          pixel tile and channel tile);
//   conv:  A = x[i][px] from a per-wave LDS tile of the channel-planar input, read transposed by
//          ds_read_b64_tr_b16 (bf16; two reads give a lane its 8 channels of one pixel),
//          B = Wc^T (hi/lo split once).
// Scheduling: the (row, chunk) units of the whole tensor are split into equal contiguous ranges,
// one per wave (persistent-style), so no tail of half-empty rows; Y is reloaded on row change.
// GELU: exact-erf form (A&S 7.1.26, |err| < 1.5e-7) for fp32 output; for bf16 output the fitted
// erf form of csrc/nn/gelu.h (x sigmoid(x q(x^2)), |err| <= 2.6e-5 absolute against the exact
// erf GELU, 1/40 of half a bf16 ulp at |y| = 0.25) at about the tanh form's instruction cost.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "../nn/gelu.h"
#include "../ops/tuning.h"
#include "dft_gemm.h"

#ifndef FNO_EPI_SWAP
#define FNO_EPI_SWAP 1  // bf16 output: lane-transposed 16-byte stores (v_permlane16/32_swap), see the epilogue
#endif
#ifndef FNO_BF_YLO
#define FNO_BF_YLO 0  // bf16 output: also the G_hi * Y_lo spectral products (see the header)
#endif
#ifndef FNO_EPI_STAGED
// 1: output through a per-wave LDS tile in 64-byte row pieces; 0 (default): straight from the MFMA
// layout.  Measured slower staged (profiles/fno_epilogue_r3.txt: FNO block bf16 61.7-62.3 vs
// 59.2-59.6 us, fp32 89.5-92.5 vs 84.4 us, ABAB on one box): the block is latency-bound, and the
// staging adds an LDS round trip and a wave barrier per tile for no store-efficiency gain.
#define FNO_EPI_STAGED 0
#endif

namespace amd_dft {
namespace {

#ifdef FNO_STAMPS
// phase clocks (bench/fno_stamps.hip): per wave, s_memtime cycles summed over its units per phase
// -- [0] setup, [1] spectrum (re)load on a row change, [2] x staging + rotation/split, [3] MFMAs,
// [4] epilogue; [5] units, [6] s_memrealtime at entry; 8 per wave, written by lane 0 at exit
__device__ long long* g_fno_stamps;
#define FNO_T(slot)                                       \
  do {                                                    \
    const long long tn_ = __builtin_amdgcn_s_memtime();   \
    fno_acc[slot] += tn_ - fno_tp;                        \
    fno_tp = tn_;                                         \
  } while (0)
#else
#define FNO_T(slot) do { } while (0)
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ void split1(float v, __bf16& hi, __bf16& lo) {
  hi = static_cast<__bf16>(v);
  lo = static_cast<__bf16>(v - static_cast<float>(hi));
}

__device__ __forceinline__ float gelu_erf(float v) {
  const float z = fabsf(v) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = fmaf(-p, __builtin_amdgcn_exp2f(-1.4426950408889634f * z * z), 1.f);  // erf(|v|/sqrt2)
  return 0.5f * v * (1.f + copysignf(e, v));
}

__device__ __forceinline__ float gelu_tanh(float v) {
  // x * sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)) = x / (1 + 2^(v (c1 + c2 v^2)))
  constexpr float c1 = -1.5957691216057308f * 1.4426950408889634f;
  constexpr float c2 = c1 * 0.044715f;
  const float z = v * fmaf(c2, v * v, c1);
  return v * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));
}

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <bool BF>
struct Geo {
  static constexpr int CH = BF ? kFnoChunkBF : kFnoChunkF32;  // pixels per chunk
  static constexpr int PT = CH / 16;                           // MFMA pixel tiles per chunk
  static constexpr int XP = BF ? CH + 16 : CH + 4;             // LDS row pitch (elements) of the x tile
  static constexpr int ES = BF ? 2 : 4;
};

// two floats -> packed bf16x2 (v_cvt_pk_bf16_f32, round-to-nearest-even)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 v;
  v[0] = static_cast<__bf16>(a);
  v[1] = static_cast<__bf16>(b);
  return __builtin_bit_cast(uint32_t, v);
}
// hi = bf16(a, b); lo = bf16(a - hi.a, b - hi.b)
__device__ __forceinline__ void split_pk(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pk_bf16(a, b);
  lo = pk_bf16(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}

template <int ACT>
__device__ __forceinline__ float act(float v) {
  if constexpr (ACT == 1) return gelu_erf(v);
  if constexpr (ACT == 2) return gelu_tanh(v);
  if constexpr (ACT == 3) return gelu_erf_fit(v);
  return v;
}

#ifndef FNO_BF_ACT
#define FNO_BF_ACT 3  // bf16 output's GELU: 3 the fitted erf form (default), 2 the tanh form (A/B build: its cost)
#endif
#ifndef FNO_Y_VEC
#define FNO_Y_VEC 1  // spectrum row: 16-byte loads of 4 modes (0: one 8-byte load per mode)
#endif
#ifndef FNO_ROT_TRIM
#define FNO_ROT_TRIM 1  // setup: load only the rotation-table rows the grid uses (0: the kFnoRotMax bound)
#endif
#ifndef FNO_ACT_PACKED
#define FNO_ACT_PACKED 1  // epilogue GELU on value pairs with packed f32 VALU (csrc/nn/gelu.h); 0: per value
#endif
// the activation of two values: packed f32 FMAs / MULs issue once for both (the transcendentals stay per
// value); the fp32 form is gelu.h's A&S arrangement (same 1.5e-7 bound as gelu_erf above)
template <int ACT>
__device__ __forceinline__ float2 act2(float a, float b) {
  if constexpr (FNO_ACT_PACKED && ACT != 0) {
    gelu_f2 r;
    if constexpr (ACT == 1) r = gelu_erf2(gelu_f2{a, b});
    else if constexpr (ACT == 2) r = gelu_tanh2(gelu_f2{a, b});
    else r = gelu_erf_fit2(gelu_f2{a, b});
    return make_float2(r.x, r.y);
  } else {
    return make_float2(act<ACT>(a), act<ACT>(b));
  }
}

// row_ror:n inside 16-lane rows: lane i receives lane (i - n) mod 16 of its row
template <int N>
__device__ __forceinline__ float row_ror(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x120 + N, 0xf, 0xf, false));
}

template <bool BF>
__device__ __forceinline__ void store4(char* dst, const float (&v)[4]) {
  if constexpr (BF) *reinterpret_cast<uint2*>(dst) = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
  else *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
}

// PW = false: the spectral path alone (SpectralConv2d: y = irfft_W(Y), no x, no 1x1 conv, no activation) --
// no x staging in LDS (32 KB per workgroup instead of 69) and no x prefetch registers
template <bool BF, int KS, int CO, int ACT, bool PW = true>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, PW ? 2 : 4))) fno_c2r_pw_kernel(const float2* __restrict__ yw, const void* __restrict__ x,
                                                         const float* __restrict__ wc, const float* __restrict__ bias,
                                                         void* __restrict__ y, const bf16x8* __restrict__ g0,
                                                         const float2* __restrict__ rot, int Cin, int Cout, int H,
                                                         int W, int m, int nch, int64_t units) {
  using GG = Geo<BF>;
  constexpr int PT = GG::PT, XP = GG::XP, ES = GG::ES, CH = GG::CH;
  constexpr bool PREC3 = !BF;  // fp32 output: also the G_lo * Y_hi term (twiddles exact to ~2^-17)
  constexpr bool YLO = !BF || FNO_BF_YLO;  // the G_hi * Y_lo term
  constexpr int NG = PREC3 ? 2 : 1;
  __shared__ bf16x8 g0s[KS][PT][NG][64];
  static_assert(PW || ACT == 0, "the spectral-only tail has no activation");
  __shared__ __attribute__((aligned(16))) char xs_raw[4][PW ? 32 * XP * ES : 16];
  // chunk rotations in LDS (needed right before each chunk's MFMAs; an L2 round trip there
  // stalled every chunk)
  // (launch_fno_c2r_pw guarantees nch * 16 KS <= kFnoRotMax)
  __shared__ float2 rots[kFnoRotMax];
#if FNO_EPI_STAGED
  // per-wave output staging: [32 channel rows][PXS pixels] (64 bytes of a row), pitch + 16 B (bank
  // spread); 10 KB per workgroup, so two workgroups still share a CU
  // (m > 32: the larger twiddle table leaves no room -- straight stores)
  constexpr bool STG = KS <= 2;
  constexpr int PXS = 64 / ES, EP = 64 + 16;
  __shared__ __attribute__((aligned(16))) char es_raw[STG ? 4 : 1][STG ? 32 * EP : 16];
#endif
#ifdef FNO_STAMPS
  long long fno_acc[6] = {0, 0, 0, 0, 0, 0};
  const long long fno_rt0 = __builtin_amdgcn_s_memrealtime();
  long long fno_tp = __builtin_amdgcn_s_memtime();
#endif
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l15 = lane & 15, lq = lane >> 4;

  const int64_t nw = static_cast<int64_t>(gridDim.x) * 4;
  const int64_t gw = static_cast<int64_t>(blockIdx.x) * 4 + wv;
  const int64_t u0 = gw * units / nw, u1 = (gw + 1) * units / nw;

  char* xs = xs_raw[wv];
  lds_v4s* xs_tr = (lds_v4s*)(xs_raw[wv]);
  const int64_t plane = static_cast<int64_t>(H) * W * ES;  // bytes between channel planes
  // the sparse second channel tile (Cout in (16, 20]) is packed 4 pixel tiles per lane-row
  const bool pack = CO == 2 && Cout <= 20;
  constexpr int LPR = CH / 8;    // lanes per staged channel row (8 pixels each)
  constexpr int RPI = 64 / LPR;  // channel rows per wave instruction
  const int st_ch = lane / LPR, st_px = (lane % LPR) * 8;  // staging role of this lane
  float2 Yv[CO][KS][4];
  int cur_b = -1, cur_h = -1;  // (b, h) of the spectrum row held in Yv
  // byte offsets (not pointers: a pointer carried around the loop loses its global address
  // space and the stores become flat stores, which every later LDS wait would also drain)
  int64_t yrow[CO];  // &y[b][16 ot + l15][h][4 lq] - y  (clamped to a valid channel)
  int64_t yrowp = 0;  // same for the packed channel tile: channel 16 + (l15 & 3)
  int64_t ybase = 0;  // &y[b][0][h][0] - y (staged epilogue)
  char* const yb = static_cast<char*>(y);

  // x staging: this lane's 8-pixel pieces of channel rows st_ch + RPI*q of unit u, kept in
  // registers one unit ahead so the loads are in flight while the previous chunk computes.
  constexpr int NQ = 32 / RPI;
  using Raw = u32x4;  // 16 bytes = 8 bf16 or 4 fp32 (a native vector: HIP's uint4 struct copies went to scratch)
  constexpr int NR = BF ? 1 : 2;
  Raw xr[NQ][NR];
  // Unit u = (b * H + h) * nch + c, kept as (c, h, b) counters advanced once per unit: the
  // divisions by the runtime nch / H (64-bit: ~150 instructions each with branches) stay out of
  // the loop
  struct UPos {
    int c, h, b;
  };
  auto advance = [&](UPos& q) {
    if (++q.c == nch) {
      q.c = 0;
      if (++q.h == H) {
        q.h = 0;
        ++q.b;
      }
    }
  };
  auto load_x = [&](const UPos& q) {
    if constexpr (!PW) return;
    const int cw = q.c * CH + st_px;
    const char* src = static_cast<const char*>(x) +
                      (((static_cast<int64_t>(q.b) * Cin + st_ch) * H + q.h) * W + cw) * ES;
    // Unconditional loads (clamped address when out of range): pixels >= W only reach outputs
    // that are never stored and channels >= Cin are never staged, so no zeroing is needed --
    // a select on the loaded value here would make the compiler wait for the load right away
    // and serialise the prefetch with the chunk it is meant to overlap.
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool ok = cw < W && st_ch + RPI * q < Cin;
      const Raw* sp = reinterpret_cast<const Raw*>(ok ? src + RPI * q * plane : static_cast<const char*>(x));
#pragma unroll
      for (int t = 0; t < NR; ++t) xr[q][t] = sp[t];
    }
  };
  // the spectrum operand of one (b, h) row and its output row offsets
  auto load_row = [&](const UPos& q) {
    cur_b = q.b;
    cur_h = q.h;
    const int64_t b = q.b, h = q.h;
#pragma unroll
    for (int ot = 0; ot < CO; ++ot)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k0 = 16 * ks + 4 * lq;
        if (FNO_Y_VEC && (m & 1) == 0 && k0 + 3 < m) {
          // 4 consecutive modes as two 16-byte loads; channels >= Cout read channel Cout - 1 (their
          // MFMA output columns are never stored, and a column only feeds its own outputs)
          const int o = min(16 * ot + l15, Cout - 1);
          const float4* src = reinterpret_cast<const float4*>(yw + ((b * Cout + o) * H + h) * m + k0);
          const float4 v0 = src[0], v1 = src[1];
          Yv[ot][ks][0] = make_float2(v0.x, v0.y);
          Yv[ot][ks][1] = make_float2(v0.z, v0.w);
          Yv[ot][ks][2] = make_float2(v1.x, v1.y);
          Yv[ot][ks][3] = make_float2(v1.z, v1.w);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int o = 16 * ot + l15, k = k0 + q;
            Yv[ot][ks][q] = (o < Cout && k < m) ? yw[((b * Cout + o) * H + h) * m + k] : make_float2(0.f, 0.f);
          }
        }
      }
    const int64_t y0 = ((b * Cout * H + h) * W + 4 * lq) * ES;
    ybase = (b * Cout * H + h) * W * ES;
#pragma unroll
    for (int ot = 0; ot < CO; ++ot) yrow[ot] = y0 + min(16 * ot + l15, Cout - 1) * plane;
    yrowp = y0 + min(16 + (l15 & 3), Cout - 1) * plane;
  };
  // this wave's first x chunk and spectrum row are requested before the table setup below, so the
  // three global round trips overlap instead of following each other (the setup was ~17 % of a
  // wave's time, profiles/fno_phases_r3.txt)
  UPos cur;
  {
    const int64_t row = u0 / nch;  // once per wave
    cur.c = static_cast<int>(u0 - row * nch);
    cur.b = static_cast<int>(row / H);
    cur.h = static_cast<int>(row - static_cast<int64_t>(cur.b) * H);
  }
  if (u0 < u1) {
    load_x(cur);
    load_row(cur);
  }


  // ---- tables: every load issued before the first is consumed -- loop-carried loads waited one
  // memory latency per iteration (the setup was a third of a wave's cycles, profiles/fno_r3_fused_mix.txt);
  // addresses clamped so nothing sits behind a branch, out-of-range entries masked after the wait
  const int nrot = nch * 16 * KS;
  constexpr int NRT = kFnoRotMax / 256;                // rotation entries per thread, upper bound
  constexpr int NGT = (KS * PT * NG * 64 + 255) / 256;  // G-table fragments per thread
  float2 rv[NRT];
  bf16x8 gv[NGT];
#pragma unroll
  for (int q = 0; q < NRT; ++q)  // (wave-uniform guard: only the table's ceil(nrot / 256) rows are requested)
    if (!FNO_ROT_TRIM || 256 * q < nrot) rv[q] = rot[min(static_cast<int>(threadIdx.x) + 256 * q, nrot - 1)];
#pragma unroll
  for (int q = 0; q < NGT; ++q) {
    const int t = min(static_cast<int>(threadIdx.x) + 256 * q, KS * PT * NG * 64 - 1);
    const int ln = t & 63, r = t >> 6;
    const int hl = r % NG, f = r / NG;  // f = ks * PT + pt
    gv[q] = g0[(f * 2 + hl) * 64 + ln];
  }
  // conv B operand: Wc^T[i][o], lane holds i = 8lq + j of channel 16ot + l15
  float wcv[CO][8], bo[CO];
#pragma unroll
  for (int ot = 0; ot < CO; ++ot) {
    const int o = min(16 * ot + l15, Cout - 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) wcv[ot][j] = PW ? wc[o * Cin + min(8 * lq + j, Cin - 1)] : 0.f;
    bo[ot] = bias != nullptr ? bias[o] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < NRT; ++q) {
    const int t = static_cast<int>(threadIdx.x) + 256 * q;
    if (t < nrot) rots[t] = rv[q];
  }
#pragma unroll
  for (int q = 0; q < NGT; ++q) {
    const int t = static_cast<int>(threadIdx.x) + 256 * q;
    if (t < KS * PT * NG * 64) (&g0s[0][0][0][0])[t] = gv[q];
  }
  bf16x8 Wh[CO], Wl[CO];
#pragma unroll
  for (int ot = 0; ot < CO; ++ot) {
    const bool ok = 16 * ot + l15 < Cout;
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 8 * lq + 2 * j;
      split_pk(ok && i < Cin ? wcv[ot][2 * j] : 0.f, ok && i + 1 < Cin ? wcv[ot][2 * j + 1] : 0.f, hi[j], lo[j]);
    }
    Wh[ot] = __builtin_bit_cast(bf16x8, make_uint4(hi[0], hi[1], hi[2], hi[3]));
    Wl[ot] = __builtin_bit_cast(bf16x8, make_uint4(lo[0], lo[1], lo[2], lo[3]));
    if (!ok) bo[ot] = 0.f;
  }
  // channel rows >= Cin stay zero (their weights are zero, but 0 * stale-NaN is not); rows < Cin
  // are rewritten by every chunk before they are read
  if constexpr (PW) {
    constexpr int RW = XP * ES / 16;  // 16-byte words per channel row
    const int nz = (32 - Cin) * RW;   // per wave tile
    for (int t = threadIdx.x; t < 4 * nz; t += 256) {
      const int wq = t / nz, r = t - wq * nz;
      reinterpret_cast<uint4*>(&xs_raw[wq][0])[Cin * RW + r] = make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();

  if (u0 >= u1) return;  // no barriers below this point
  FNO_T(0);

  for (int64_t u = u0; u < u1; ++u) {
    const int c = cur.c;
    if (cur.h != cur_h || cur.b != cur_b) load_row(cur);
    UPos nxt = cur;
    advance(nxt);
    FNO_T(1);
    const int w0 = c * CH;
    // ---- x chunk (channels x pixels) into this wave's LDS tile
    wave_lds_fence();
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int ch = st_ch + RPI * q;
      if (PW && ch < Cin) {
        Raw* dst = reinterpret_cast<Raw*>(xs + (ch * XP + st_px) * ES);
#pragma unroll
        for (int t = 0; t < NR; ++t) dst[t] = xr[q][t];
      }
    }
    // ---- rotate + split the spectral operand for this chunk
    bf16x8 Bh[CO][KS], Bl[YLO ? CO : 1][YLO ? KS : 1];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint32_t hi[CO][4], lo[CO][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float2 r = rots[c * 16 * KS + 16 * ks + 4 * lq + q];
#pragma unroll
        for (int ot = 0; ot < CO; ++ot) {
          const float2 v = Yv[ot][ks][q];
          const float re = v.x * r.x - v.y * r.y, im = v.x * r.y + v.y * r.x;
          if constexpr (YLO) split_pk(re, im, hi[ot][q], lo[ot][q]);
          else hi[ot][q] = pk_bf16(re, im);
        }
      }
#pragma unroll
      for (int ot = 0; ot < CO; ++ot) {
        Bh[ot][ks] = __builtin_bit_cast(bf16x8, make_uint4(hi[ot][0], hi[ot][1], hi[ot][2], hi[ot][3]));
        if constexpr (YLO) Bl[ot][ks] = __builtin_bit_cast(bf16x8, make_uint4(lo[ot][0], lo[ot][1], lo[ot][2], lo[ot][3]));
      }
    }
    // prefetch the next unit's x (unconditionally -- the last unit re-loads itself: behind a
    // branch, the waits after the join would be merged conservatively to vmcnt(0) and drain it)
    load_x(u + 1 < u1 ? nxt : cur);
    wave_lds_fence();
    FNO_T(2);
    // ---- MFMA, 4 pixel tiles at a time: conv + spectral into bias-initialised accumulators
#pragma unroll
    for (int pg = 0; pg < PT / 4; ++pg) {
      f32x4 acc[4][CO];
#pragma unroll
      for (int p4 = 0; p4 < 4; ++p4) {
        const int pt = 4 * pg + p4;
#pragma unroll
        for (int ot = 0; ot < CO; ++ot) acc[p4][ot] = f32x4{bo[ot], bo[ot], bo[ot], bo[ot]};
        bf16x8 ax, axl;
        if constexpr (!PW) {
        } else if constexpr (BF) {
          // rows 8lq + (0..3) and 8lq + (4..7), cols 16pt..16pt+15: lane 4q'+p addresses row q', cols 4p..4p+3
          const int e0 = (8 * lq + (l15 >> 2)) * XP + 16 * pt + 4 * (l15 & 3);
          const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(xs_tr + e0 / 4);
          const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(xs_tr + (e0 + 4 * XP) / 4);
          const uint2 u0v = __builtin_bit_cast(uint2, a0), u1v = __builtin_bit_cast(uint2, a1);
          ax = __builtin_bit_cast(bf16x8, make_uint4(u0v.x, u0v.y, u1v.x, u1v.y));
        } else {
          uint32_t hi[4], lo[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float* rp = reinterpret_cast<const float*>(xs) + (8 * lq + 2 * j) * XP + 16 * pt + l15;
            split_pk(rp[0], rp[XP], hi[j], lo[j]);
          }
          ax = __builtin_bit_cast(bf16x8, make_uint4(hi[0], hi[1], hi[2], hi[3]));
          axl = __builtin_bit_cast(bf16x8, make_uint4(lo[0], lo[1], lo[2], lo[3]));
        }
#pragma unroll
        for (int ot = 0; ot < CO && PW; ++ot) {
          acc[p4][ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax, Wh[ot], acc[p4][ot], 0, 0, 0);
          if constexpr (!BF) {  // bf16 output: bf16 conv weights, as a bf16 nn.Conv2d has
            acc[p4][ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax, Wl[ot], acc[p4][ot], 0, 0, 0);
            acc[p4][ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(axl, Wh[ot], acc[p4][ot], 0, 0, 0);
          }
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 gh = g0s[ks][pt][0][lane];
#pragma unroll
          for (int ot = 0; ot < CO; ++ot) {
            acc[p4][ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh, Bh[ot][ks], acc[p4][ot], 0, 0, 0);
            if constexpr (YLO) acc[p4][ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh, Bl[ot][YLO ? ks : 0], acc[p4][ot], 0, 0, 0);
          }
          if constexpr (PREC3) {
            const bf16x8 gl = g0s[ks][pt][NG - 1][lane];
#pragma unroll
            for (int ot = 0; ot < CO; ++ot)
              acc[p4][ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gl, Bh[ot][ks], acc[p4][ot], 0, 0, 0);
          }
        }
      }
      FNO_T(3);
      // ---- epilogue: activation + store, 4 consecutive pixels of one channel per lane
      const int pxg = w0 + 64 * pg + 4 * lq;  // pixel of row i = 0 in tile p4 = 0
#if FNO_EPI_STAGED
      // Through LDS: straight from the MFMA layout every store instruction would write 16
      // channel rows x 32 B (partial lines); staged, a lane stores 16 B and 8 (bf16) / 16 (fp32)
      // lanes fill one 128 / 256-byte run of a channel row.
      if constexpr (STG) {
        char* es = es_raw[wv];
        constexpr int TPS = PXS / 16;  // pixel tiles per staging pass
#pragma unroll
        for (int hp = 0; hp < 4 / TPS; ++hp) {
          wave_lds_fence();
#pragma unroll
          for (int ot = 0; ot < CO; ++ot) {
            const int ch = 16 * ot + l15;
#pragma unroll
            for (int pp = 0; pp < TPS; ++pp) {
              const int p4 = hp * TPS + pp;
              float v[4];
#pragma unroll
              for (int i = 0; i < 4; i += 2) {
                const float2 r = act2<ACT>(acc[p4][ot][i], acc[p4][ot][i + 1]);
                v[i] = r.x;
                v[i + 1] = r.y;
              }
              if (ch < Cout) store4<BF>(es + ch * EP + (16 * pp + 4 * lq) * ES, v);
            }
          }
          wave_lds_fence();
          // 4 lanes x 16 B = one 64-byte run of a channel row; 16 rows per store instruction
          const int sub = lane >> 2, px = (lane & 3) * (16 / ES);
          const int wpx = w0 + 64 * pg + PXS * hp + px;
#pragma unroll
          for (int r0 = 0; r0 < 32; r0 += 16) {
            const int ch = r0 + sub;
            if (r0 < Cout && ch < Cout && wpx < W) {
              const uint4 q = *reinterpret_cast<const uint4*>(es + ch * EP + px * ES);
              *reinterpret_cast<uint4*>(yb + ybase + ch * plane + static_cast<int64_t>(wpx) * ES) = q;
            }
          }
        }
      }
      if constexpr (!STG)
#endif
      {
#pragma unroll
      for (int ot = 0; ot < CO; ++ot) {
        if (ot == 1 && pack) break;
        const int o = 16 * ot + l15;
        if constexpr (BF && FNO_EPI_SWAP) {
          // 4x4 transpose of the 8-byte pieces across the lanes of one channel (rows lq of the
          // wave): lane (c, lq) ends up with pixel tile lq's four 4-pixel groups, i.e. 32
          // contiguous bytes -> two 16-byte stores instead of four 8-byte ones (same bytes, half
          // the store instructions).  permlane32_swap exchanges rows {2,3} of its first operand
          // with rows {0,1} of its second; permlane16_swap rows {1,3} with {0,2}.
          uint32_t d[4][2];
#pragma unroll
          for (int p4 = 0; p4 < 4; ++p4) {
            const float2 r0 = act2<ACT>(acc[p4][ot][0], acc[p4][ot][1]), r1 = act2<ACT>(acc[p4][ot][2], acc[p4][ot][3]);
            d[p4][0] = pk_bf16(r0.x, r0.y);
            d[p4][1] = pk_bf16(r1.x, r1.y);
          }
#pragma unroll
          for (int pp = 0; pp < 2; ++pp)
#pragma unroll
            for (int w = 0; w < 2; ++w) {
              const auto r = __builtin_amdgcn_permlane32_swap(d[pp][w], d[pp + 2][w], false, false);
              d[pp][w] = r[0];
              d[pp + 2][w] = r[1];
            }
#pragma unroll
          for (int pp = 0; pp < 4; pp += 2)
#pragma unroll
            for (int w = 0; w < 2; ++w) {
              const auto r = __builtin_amdgcn_permlane16_swap(d[pp][w], d[pp + 1][w], false, false);
              d[pp][w] = r[0];
              d[pp + 1][w] = r[1];
            }
          const int px0 = w0 + 64 * pg + 16 * lq;  // this lane's 16 pixels
          char* dst = yb + yrow[ot] + static_cast<int64_t>(w0 + 64 * pg + 12 * lq) * ES;  // yrow carries +4 lq pixels
          if (o < Cout && px0 + 8 <= W) *reinterpret_cast<uint4*>(dst) = make_uint4(d[0][0], d[0][1], d[1][0], d[1][1]);
          if (o < Cout && px0 + 16 <= W) *reinterpret_cast<uint4*>(dst + 16) = make_uint4(d[2][0], d[2][1], d[3][0], d[3][1]);
        } else {
#pragma unroll
          for (int p4 = 0; p4 < 4; ++p4) {
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
              const float2 r = act2<ACT>(acc[p4][ot][i], acc[p4][ot][i + 1]);
              v[i] = r.x;
              v[i + 1] = r.y;
            }
            if (o < Cout && pxg + 16 * p4 < W) store4<BF>(yb + yrow[ot] + (w0 + 64 * pg + 16 * p4) * ES, v);
          }
        }
      }
      if (CO == 2 && pack) {
        // channel tile 1 holds <= 4 live columns: gather tiles p4 = 0..3 into lane groups l15 / 4
        const int s = l15 >> 2, cc = l15 & 3;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a0 = acc[0][CO - 1][i], a1 = row_ror<4>(acc[1][CO - 1][i]), a2 = row_ror<8>(acc[2][CO - 1][i]),
                      a3 = row_ror<12>(acc[3][CO - 1][i]);
          v[i] = s == 0 ? a0 : s == 1 ? a1 : s == 2 ? a2 : a3;
        }
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const float2 r = act2<ACT>(v[i], v[i + 1]);
          v[i] = r.x;
          v[i + 1] = r.y;
        }
        const int o = 16 + cc;
        if (o < Cout && pxg + 16 * s < W) store4<BF>(yb + yrowp + (w0 + 64 * pg + 16 * s) * ES, v);
      }
      }
      FNO_T(4);
    }
    cur = nxt;
  }
#ifdef FNO_STAMPS
  if (lane == 0) {
    long long* st = g_fno_stamps + gw * 8;
    for (int i = 0; i < 5; ++i) st[i] = fno_acc[i];
    st[5] = u1 - u0;
    st[6] = fno_rt0;
  }
#endif
}

// workgroups of one kernel instance resident on the current device (occupancy x CUs), cached
// compute units of the current device, cached
int64_t device_cus() {
  static int64_t cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cache[dev] = cus;
  }
  return cache[dev];
}

template <bool BF, int KS, int CO, bool PW>
int64_t resident_wgs() {
  static int64_t cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] == 0) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const auto kern = PW ? reinterpret_cast<const void*>(&fno_c2r_pw_kernel<BF, KS, CO, BF ? FNO_BF_ACT : 1>)
                         : reinterpret_cast<const void*>(&fno_c2r_pw_kernel<BF, KS, CO, 0, false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess || per_cu <= 0) per_cu = 1;
    cache[dev] = static_cast<int64_t>(cus) * per_cu;
  }
  return cache[dev];
}

template <bool BF, int KS, int CO>
void launch_g(const FnoC2RPwLaunch& p, hipStream_t st) {
  constexpr int CH = Geo<BF>::CH;
  const int nch = (p.W + CH - 1) / CH;
  const int64_t units = static_cast<int64_t>(p.B) * p.H * nch;
  // Persistent grid: at most as many workgroups as are resident at once (a second partial round
  // of workgroups would double the kernel time), and >= 4 chunks per wave (tuning builds:
  // MI_DFT_FNO_UPW = minimum chunks per wave, MI_DFT_FNO_WGS = workgroup cap)
  static const int upw = [] {
    const char* e = tuning_env("MI_DFT_FNO_UPW");
    return e ? std::max(1, std::atoi(e)) : 4;
  }();
  static const int64_t wgs_cap = [] {
    const char* e = tuning_env("MI_DFT_FNO_WGS");
    return e ? std::max<int64_t>(1, std::atoll(e)) : int64_t(1) << 40;
  }();
  const int64_t res = p.x ? resident_wgs<BF, KS, CO, true>() : resident_wgs<BF, KS, CO, false>();
  int64_t nwg = std::max<int64_t>(std::min<int64_t>(std::min<int64_t>((units + 4 * upw - 1) / (4 * upw), res), wgs_cap), 1);
  // a whole number of workgroups per CU: the grid is one round, so a CU holding one workgroup more than
  // the others finishes last (fno_c2r at 720 x 1440: 540 -> 512 workgroups, 45.0 -> 42.6 us SpectralConv2d;
  // profiles/fno_tail_phases_r6.txt)
  const int64_t cus = device_cus();
  if (nwg > cus) nwg = nwg / cus * cus;
  const dim3 grid(static_cast<uint32_t>(nwg));
  const float2* yw = static_cast<const float2*>(p.yw);
  const bf16x8* g0 = static_cast<const bf16x8*>(p.g0);
  const float2* rot = static_cast<const float2*>(p.rot);
#define L_(A)                                                                                                     \
  hipLaunchKernelGGL((fno_c2r_pw_kernel<BF, KS, CO, A>), grid, dim3(256), 0, st, yw, p.x, p.wc, p.bias, p.y, g0, rot, \
                     p.Cin, p.Cout, p.H, p.W, p.m, nch, units)
  if (p.x == nullptr) {  // spectral path only (p.gelu is 0: checked by launch_fno_c2r_pw)
    hipLaunchKernelGGL((fno_c2r_pw_kernel<BF, KS, CO, 0, false>), grid, dim3(256), 0, st, yw, nullptr, nullptr, p.bias,
                       p.y, g0, rot, 0, p.Cout, p.H, p.W, p.m, nch, units);
  } else if (!p.gelu) {
    L_(0);
  } else if (BF) {
    L_(FNO_BF_ACT);
  } else {
    L_(1);
  }
#undef L_
}

template <bool BF, int KS>
void launch_co(const FnoC2RPwLaunch& p, hipStream_t st) {
  if (p.Cout <= 16) launch_g<BF, KS, 1>(p, st);
  else launch_g<BF, KS, 2>(p, st);
}

template <bool BF>
void launch_ks(const FnoC2RPwLaunch& p, hipStream_t st) {
  switch ((p.m + 15) / 16) {
    case 1: launch_co<BF, 1>(p, st); break;
    case 2: launch_co<BF, 2>(p, st); break;
    case 3: launch_co<BF, 3>(p, st); break;
    default: launch_co<BF, 4>(p, st); break;
  }
}

}  // namespace

bool fno_c2r_pw_supported(int cin, int cout, int m, int W, bool bf16) {
  if (!(cin >= 1 && cin <= 32 && cout >= 1 && cout <= 32 && m >= 1 && m <= 64 && 2 * (m - 1) <= W && W % 8 == 0))
    return false;
  const int ch = bf16 ? kFnoChunkBF : kFnoChunkF32;
  return static_cast<int64_t>((W + ch - 1) / ch) * 16 * ((m + 15) / 16) <= kFnoRotMax;
}

void launch_fno_c2r_pw(const FnoC2RPwLaunch& p, void* stream) {
  if (p.B == 0 || p.H == 0) return;
  if (p.x == nullptr && p.gelu) throw std::runtime_error("amd_dft: fno_c2r: the spectral-only tail takes no activation");
  if (!fno_c2r_pw_supported(p.x == nullptr ? 1 : p.Cin, p.Cout, p.m, p.W, p.bf16 != 0))
    throw std::runtime_error("amd_dft: fno_c2r_pw: needs Cin, Cout <= 32, m <= 64, W % 8 == 0, W <= 4096 (bf16)");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (p.bf16) launch_ks<true>(p, st);
  else launch_ks<false>(p, st);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: fno_c2r_pw launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
