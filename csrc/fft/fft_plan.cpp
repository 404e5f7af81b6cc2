#include "fft_plan.h"

#include "fft_fixed.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <sstream>
#include "../ops/tuning.h"

namespace amd_dft {

namespace {

// Relative butterfly cost per point (flops-ish); passes dominate (one LDS round trip and
// one barrier each), so factorisations are ranked by pass count first.
double radix_cost(int r) {
  switch (r) {
    case 2: return 1.0;
    case 3: return 2.7;
    case 4: return 1.5;
    case 5: return 3.4;
    case 6: return 2.5;
    case 7: return 4.6;
    case 8: return 2.1;
    case 9: return 3.3;
    case 10: return 3.2;
    case 11: return 6.5;
    case 12: return 3.0;
    case 13: return 7.5;
    case 15: return 4.0;
    case 16: return 2.6;
    default: return 2.0 * r;  // generic O(R) per point
  }
}

const int kSpecialised[] = {16, 15, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2};

struct Best {
  int passes = 1 << 30;
  double cost = 1e300;
  std::vector<int32_t> f;
};

Best search(int32_t L, std::map<int32_t, Best>& memo) {
  if (L == 1) return Best{0, 0.0, {}};
  auto it = memo.find(L);
  if (it != memo.end()) return it->second;
  Best best;
  for (int r : kSpecialised) {
    if (L % r) continue;
    Best sub = search(L / r, memo);
    const int passes = sub.passes + 1;
    const double cost = sub.cost + radix_cost(r);
    if (passes < best.passes || (passes == best.passes && cost < best.cost)) {
      best.passes = passes;
      best.cost = cost;
      best.f = sub.f;
      best.f.insert(best.f.begin(), r);
    }
  }
  if (best.passes == (1 << 30)) {
    // No specialised radix divides L: peel the smallest prime factor with the generic path.
    int32_t p = 2;
    while (static_cast<int64_t>(p) * p <= L && L % p) ++p;
    if (L % p) p = L;
    Best sub = search(L / p, memo);
    best.passes = sub.passes + 1;
    best.cost = sub.cost + radix_cost(p);
    best.f = sub.f;
    best.f.push_back(p);
  }
  memo[L] = best;
  return best;
}

}  // namespace

// radices with a compile-time butterfly that only a fixed-kernel configuration's radix order
// selects (AMD_DFT_FIXED_CONFIGS): no root table in the plan, never chosen by search()
const int kFixedOnly[] = {24, 30};

bool radix_is_specialised(int r) {
  for (int s : kSpecialised)
    if (s == r) return true;
  for (int s : kFixedOnly)
    if (s == r) return true;
  return false;
}

std::vector<int32_t> factorize(int32_t L) {
  // Lengths with a compile-time specialised kernel use that kernel's radix order.
  std::vector<int32_t> fx = fixed_radices(L);
  if (!fx.empty()) return fx;
  std::map<int32_t, Best> memo;
  std::vector<int32_t> f = search(L, memo).f;
  // Large radices first: later passes then write contiguous runs (Ns grows fast).
  std::stable_sort(f.begin(), f.end(), [](int a, int b) {
    const bool sa = radix_is_specialised(a), sb = radix_is_specialised(b);
    if (sa != sb) return sa;  // generic (prime) radices last
    return a > b;
  });
  return f;
}

Plan1D make_plan_1d(int32_t L) {
  Plan1D p;
  p.L = L;
  p.radices = factorize(L);
  if (static_cast<int>(p.radices.size()) > kMaxPasses) throw std::runtime_error("amd_dft: too many FFT passes");
  int32_t ns = 1;
  int32_t off = 0;
  std::vector<double> tw;
  for (int32_t r : p.radices) {
    p.ns.push_back(ns);
    p.twoff.push_back(off);
    if (ns > 1) {
      const int64_t N = static_cast<int64_t>(ns) * r;
      for (int32_t q = 1; q < r; ++q)
        for (int32_t k = 0; k < ns; ++k) {
          const double a = -2.0 * M_PI * static_cast<double>(static_cast<int64_t>(q) * k % N) / static_cast<double>(N);
          tw.push_back(std::cos(a));
          tw.push_back(std::sin(a));
        }
      off += (r - 1) * ns;
    }
    p.rootoff.push_back(off);
    if (!radix_is_specialised(r)) {
      for (int32_t m = 0; m < r; ++m) {
        const double a = -2.0 * M_PI * static_cast<double>(m) / static_cast<double>(r);
        tw.push_back(std::cos(a));
        tw.push_back(std::sin(a));
      }
      off += r;
    }
    ns *= r;
  }
  p.tw_count = off;
  p.tw_host.assign(tw.begin(), tw.end());
  if (p.tw_host.empty()) p.tw_host = {1.0f, 0.0f};  // keep the device buffer non-empty
  return p;
}

std::string describe(const Plan1D& p) {
  std::ostringstream os;
  os << "L=" << p.L << " radices=[";
  for (size_t i = 0; i < p.radices.size(); ++i) os << (i ? "," : "") << p.radices[i];
  os << "] twiddles=" << p.tw_count;
  return os.str();
}

void apply_plan(PassDesc& d, const Plan1D& p) {
  d.L = p.L;
  d.npass = static_cast<int32_t>(p.radices.size());
  for (int i = 0; i < d.npass; ++i) {
    d.radix[i] = p.radices[i];
    d.ns[i] = p.ns[i];
    d.twoff[i] = p.twoff[i];
    d.rootoff[i] = p.rootoff[i];
    d.ns_div[i] = FastDiv(static_cast<uint32_t>(p.ns[i]));
  }
  d.tw_count = p.tw_count;
  d.L_div = FastDiv(static_cast<uint32_t>(p.L));
}

void set_axis_geometry(PassDesc& d, const std::vector<int64_t>& in_shape,
                       const std::vector<int64_t>& out_shape, int axis, bool in_complex,
                       bool out_complex) {
  int64_t outer = 1, inner = 1;
  for (int i = 0; i < axis; ++i) outer *= in_shape[i];
  for (size_t i = axis + 1; i < in_shape.size(); ++i) inner *= in_shape[i];
  const int64_t ein = in_complex ? 2 : 1, eout = out_complex ? 2 : 1;
  d.Sn_in = inner * ein;
  d.Sn_out = inner * eout;
  d.So_in = in_shape[axis] * inner * ein;
  d.So_out = out_shape[axis] * inner * eout;
  if (inner == 1) {
    // Row-like: every outer index is one signal; fold it into the inner (tiled) index.
    d.I = outer;
    d.Si_in = d.So_in;
    d.Si_out = d.So_out;
    d.O = 1;
    d.So_in = d.So_out = 0;
  } else {
    d.I = inner;
    d.Si_in = ein;
    d.Si_out = eout;
    d.O = outer;
  }
}

int64_t max_lds_length() {
  PassDesc d;
  int64_t lo = 1, hi = 1 << 16;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) / 2;
    d.L = static_cast<int32_t>(mid);
    d.tw_count = static_cast<int32_t>(mid);
    d.logT = 0;
    if (pass_lds_bytes(d) <= kMaxLdsBytes) lo = mid; else hi = mid - 1;
  }
  return lo;
}

bool choose_tiling(PassDesc& d) {
  const bool paired = d.kind != Kind::C2C;
  const int64_t nsig = paired ? (d.I + 1) / 2 : d.I;  // complex FFTs along the inner index
  const bool col_like = d.Si_in < d.Sn_in || d.Si_out < d.Sn_out;
  auto lds_of = [&](int logT) {
    PassDesc t = d;
    t.logT = logT;
    return pass_lds_bytes(t);
  };
  if (lds_of(0) > kMaxLdsBytes) return false;
  int logT = 0;
  const int64_t budget = 64 * 1024;
  while (logT < 6 && (int64_t(1) << (logT + 1)) <= std::max<int64_t>(nsig, 1) && lds_of(logT + 1) <= budget) {
    const int64_t next_wgs = d.O * ((nsig + (int64_t(2) << logT) - 1) >> (logT + 1));
    if (next_wgs >= 1024) { ++logT; continue; }
    if (col_like && logT < 3 && next_wgs >= 128) { ++logT; continue; }
    break;
  }
  // Tuning overrides (experiments only): MI_DFT_LOGT_ROW / MI_DFT_LOGT_COL force log2(T).
  if (const char* e = tuning_env(col_like ? "MI_DFT_LOGT_COL" : "MI_DFT_LOGT_ROW")) {
    const int f = std::atoi(e);
    if (f >= 0 && f <= 6 && lds_of(f) <= kMaxLdsBytes) logT = f;
  }
  d.logT = logT;
  d.T = 1 << logT;
  d.tiles_per_outer = static_cast<int32_t>((nsig + d.T - 1) / d.T);
  int64_t work = (static_cast<int64_t>(d.L) << logT) / 4;
  for (int p = 0; p < d.npass; ++p) work = std::max<int64_t>(work, (static_cast<int64_t>(d.L) << logT) / d.radix[p]);
  int64_t nt = ((work + 63) / 64) * 64;
  d.nthreads = static_cast<int32_t>(std::min<int64_t>(256, std::max<int64_t>(64, nt)));
  if (const char* e = tuning_env("MI_DFT_THREADS")) {
    const int f = std::atoi(e);
    if (f >= 64 && f <= 256 && f % 64 == 0) d.nthreads = f;
  }
  const int32_t nout = d.kind == Kind::C2C ? d.out_lo + d.out_hi : (d.kind == Kind::R2C ? d.out_lo : d.L);
  d.out_div = FastDiv(static_cast<uint32_t>(std::max(nout, 1)));
  return true;
}

void finalize_vec_flags(PassDesc& d, int in_esize, int out_esize) {
  const uintptr_t pin = reinterpret_cast<uintptr_t>(d.in);
  const uintptr_t pout = reinterpret_cast<uintptr_t>(d.out);
  d.vec_in = 0;
  d.vec_out = 0;
  if (d.kind == Kind::R2C) {
    d.vec_in = d.Si_in == 1 && d.So_in % 2 == 0 && d.Sn_in % 2 == 0 && pin % (2 * in_esize) == 0;
    d.vec_out = d.Si_out == 2 && d.So_out % 4 == 0 && d.Sn_out % 4 == 0 && pout % (4 * out_esize) == 0;
  } else if (d.kind == Kind::C2R) {
    d.vec_out = d.Si_out == 1 && d.So_out % 2 == 0 && d.Sn_out % 2 == 0 && pout % (2 * out_esize) == 0;
  }
}

}  // namespace amd_dft
