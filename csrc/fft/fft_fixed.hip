// Host side of the compile-time specialised Stockham kernels: configuration table and
// selection (kernels: fft_fixed_impl.h, instantiated in fft_fixed_{c2c,r2c,c2r}.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "fft_fixed_impl.h"
#include "../ops/tuning.h"

namespace amd_dft {
namespace fixed_detail {
namespace {

#define AMD_DFT_CFG(L_, COLS_, TP_, T_, ...) FixedCfg{L_, COLS_, TP_, T_, FL<__VA_ARGS__>::N, {__VA_ARGS__}},

const std::vector<FixedCfg>& table() {
  static const std::vector<FixedCfg> v = {AMD_DFT_FIXED_CONFIGS(AMD_DFT_CFG)};
  return v;
}

}  // namespace
}  // namespace fixed_detail

using namespace fixed_detail;

const std::vector<FixedCfg>& fixed_configs() { return table(); }

// The radix order of the first configuration of length L (the plan adopts it).
// MI_DFT_FFT_RADICES="L:r,r,...;L:..." picks another configured order for L (A/B runs; read
// when the plan of L is first built).
std::vector<int32_t> fixed_radices(int32_t L) {
  static const std::string spec = [] {
    const char* e = tuning_env("MI_DFT_FFT_RADICES");
    return std::string(e ? e : "");
  }();
  if (!spec.empty()) {
    size_t pos = 0;
    while (pos < spec.size()) {
      size_t end = spec.find(';', pos);
      if (end == std::string::npos) end = spec.size();
      const std::string item = spec.substr(pos, end - pos);
      pos = end + 1;
      const size_t colon = item.find(':');
      if (colon == std::string::npos || std::atoi(item.substr(0, colon).c_str()) != L) continue;
      std::vector<int32_t> want;
      for (size_t q = colon + 1; q < item.size();) {
        size_t c = item.find(',', q);
        if (c == std::string::npos) c = item.size();
        want.push_back(std::atoi(item.substr(q, c - q).c_str()));
        q = c + 1;
      }
      for (const auto& c : fixed_configs())
        if (c.L == L && std::vector<int32_t>(c.radix, c.radix + c.npass) == want) return want;
    }
  }
  for (const auto& c : fixed_configs())
    if (c.L == L) return std::vector<int32_t>(c.radix, c.radix + c.npass);
  return {};
}

namespace {

// Process-wide A/B knobs of the fixed kernels, read once (never per launch).  None of them can
// change a result: they pick between correct kernels / tile orders.
//   MI_DFT_FIXED=0         the generic pass kernels instead of the specialised ones
//   MI_DFT_FIXED_CFG=TP,T  force one configured (threads per signal, signals per tile) pair
//   MI_DFT_FFT_XCD=0|1     force the XCD-aware column-tile order off / on
struct FixedKnobs {
  bool enabled = true;
  int force_tp = 0, force_t = 0;
  int xcd = -1;  // -1: automatic
};
const FixedKnobs& knobs() {
  static const FixedKnobs k = [] {
    FixedKnobs r;
    if (const char* fe = tuning_env("MI_DFT_FIXED")) r.enabled = std::atoi(fe) != 0;
    if (const char* fc = tuning_env("MI_DFT_FIXED_CFG")) std::sscanf(fc, "%d,%d", &r.force_tp, &r.force_t);
    if (const char* xe = tuning_env("MI_DFT_FFT_XCD")) r.xcd = std::atoi(xe) != 0 ? 1 : 0;
    return r;
  }();
  return k;
}

// Picks the configuration for d and fills its kernel arguments; false if none applies.
bool prepare_fixed(const PassDesc& d, int& best_out, FixedArgs& a, int64_t& nblocks_out) {
  const FixedKnobs& kn = knobs();
  if (!kn.enabled) return false;
  const bool cols = d.Si_in < d.Sn_in || d.Si_out < d.Sn_out;
  const bool paired = d.kind != Kind::C2C;
  const int64_t nsig = paired ? (d.I + 1) / 2 : d.I;
  int force_tp = kn.force_tp, force_t = kn.force_t;
  const auto& cfgs = fixed_configs();
  if (force_tp) {  // the override only applies where such a configuration exists
    bool any = false;
    for (const auto& c : cfgs) any |= c.L == d.L && c.cols == cols && c.TP == force_tp && c.T == force_t;
    if (!any) force_tp = force_t = 0;
  }
  int best = -1;
  double best_score = -1e300;
  for (int i = 0; i < static_cast<int>(cfgs.size()); ++i) {
    const FixedCfg& c = cfgs[i];
    if (c.L != d.L || c.cols != cols) continue;
    if (c.npass != d.npass || !std::equal(c.radix, c.radix + c.npass, d.radix)) continue;
    if (force_tp && (c.TP != force_tp || c.T != force_t)) continue;
    const int64_t wgs = d.O * ((nsig + c.T - 1) / c.T);
    const int64_t waves = wgs * ((c.TP * c.T + 63) / 64);
    // enough waves to put >= 2 on every SIMD (1024 SIMDs), then the widest tile
    // (coalescing, fewer twiddle re-reads); otherwise the most waves.
    // Measured on the AFNO W-transforms ([32,90,180,768] bf16, bench/bench_afno_w.py): the
    // C2R with fused addends prefers 32-channel tiles, the R2C 16 (wider R2C tiles lose).
    const int t_pref = (cols && d.kind == Kind::R2C) ? 16 : 1 << 30;
    const double tw = c.T <= t_pref ? c.T : -c.T;
    // Small problems (rfft2 720x1440 column pass: 721 columns): with the XCD-aware tile order
    // (tiles sharing a 128-B line run on one XCD, see xcd_block) 4-column tiles win
    // (bench/bench_fft_cfg.py, rfft2/irfft2 us: T=4 12.85/13.2, T=2 13.1/13.8, T=8 13.7/13.9;
    // profiles/fft_xcd_r2.txt).
    const double tmid = cols ? -std::abs(c.T - 4) : tw;
    const double score = waves >= 2048 ? 1e12 + tw * 1e6 + c.TP
                         : waves >= 1000 ? 1e9 + tmid * 1e3 + c.TP
                                         : static_cast<double>(waves);
    if (score > best_score) {
      best_score = score;
      best = i;
    }
  }
  if (best < 0) return false;
  const FixedCfg& cfg = cfgs[best];
  a = FixedArgs{};
  a.in = d.in;
  a.out = d.out;
  a.tw = static_cast<const float2*>(d.tw);
  // per-element offsets must fit in int32 (else the generic 64-bit kernel runs)
  const int64_t lim = 0x7fffffffLL;
  const int64_t nin = d.kind == Kind::C2C ? d.in_lo + d.in_hi : (d.kind == Kind::C2R ? d.in_lo : d.L);
  const int64_t nout = d.kind == Kind::C2C ? d.out_lo + d.out_hi : (d.kind == Kind::R2C ? d.out_lo : d.L);
  if ((d.I + 1) * d.Si_in + nin * d.Sn_in + 4 >= lim || (d.I + 1) * d.Si_out + nout * d.Sn_out + 4 >= lim) return false;
  a.So_in = d.So_in; a.So_out = d.So_out; a.I = static_cast<int32_t>(d.I);
  a.Si_in = static_cast<int32_t>(d.Si_in); a.Si_out = static_cast<int32_t>(d.Si_out);
  a.Sn_in = static_cast<int32_t>(d.Sn_in); a.Sn_out = static_cast<int32_t>(d.Sn_out);
  a.in_lo = d.in_lo; a.in_hi = d.in_hi; a.out_lo = d.out_lo; a.out_hi = d.out_hi;
  a.tiles_per_outer = static_cast<int32_t>((nsig + cfg.T - 1) / cfg.T);
  a.scale = d.scale;
  a.inverse = d.inverse; a.vec_in = d.vec_in; a.vec_out = d.vec_out;
  a.bf16_in = d.tin == DType::BF16; a.bf16_out = d.tout == DType::BF16;
  a.add1 = d.add1;
  a.add2 = d.add2;
  a.ln_stats = d.ln_stats;
  a.ln_gamma = d.ln_gamma;
  a.ln_beta = d.ln_beta;
  a.ln_pre = d.ln_pre;
  {
    // paired-vector IO: the two real signals of a complex FFT are adjacent (and 2 scalars
    // apart on the complex side), I even, and every pair offset suitably aligned
    const int64_t rin = d.kind == Kind::R2C ? 1 : 2, rout = d.kind == Kind::C2R ? 1 : 2;
    const int esi = a.bf16_in ? 2 : 4, eso = a.bf16_out ? 2 : 4;
    const uintptr_t pin = reinterpret_cast<uintptr_t>(d.in), pout = reinterpret_cast<uintptr_t>(d.out);
    bool pv = d.kind != Kind::C2C && d.I % 2 == 0 && d.Si_in == rin && d.Si_out == rout;
    pv = pv && d.Sn_in % (2 * rin) == 0 && d.So_in % (2 * rin) == 0 && pin % (2 * rin * esi) == 0;
    pv = pv && d.Sn_out % (2 * rout) == 0 && d.So_out % (2 * rout) == 0 && pout % (2 * rout * eso) == 0;
    for (const void* ad : {d.add1, d.add2})
      pv = pv && (ad == nullptr || reinterpret_cast<uintptr_t>(ad) % (2 * rout * eso) == 0);
    a.pairvec = pv ? 1 : 0;
  }
  a.mix_w = d.mix_w;
  a.mix_cin = d.mix_cin;
  a.mix_cout = d.mix_cout;
  if (d.mix_w) {  // mixing gather: pruned fp32 C2C over a column layout (outer = batch x Cout)
    const bool ok = cfg.cols && d.kind == Kind::C2C && !a.bf16_in && !a.bf16_out && d.mix_cin > 0 && d.mix_cout > 0 &&
                    d.O % d.mix_cout == 0 && (d.in_lo + d.in_hi != d.L || d.out_lo + d.out_hi != d.L) &&
                    d.So_in * d.mix_cin * d.mix_cout < 0x7fffffffLL;
    if (!ok) return false;
  }
  if (d.ln_stats) {  // LayerNorm IO: channel-last bf16 pairs, R2C input / C2R addend only
    const bool ok = cfg.cols && d.kind != Kind::C2C && a.pairvec && a.bf16_in && a.bf16_out && d.ln_gamma &&
                    d.ln_beta && (d.kind == Kind::R2C || (d.add1 && !d.add2)) && d.I % 2 == 0;
    if (!ok) return false;
  }
  const int64_t nblocks = d.O * a.tiles_per_outer;
  if (nblocks > 0x7fffffffLL) throw std::runtime_error("amd_dft: FFT grid too large");
  {
    // XCD-aware tile order for column layouts whose tile row is narrower than a 128-B line
    // (MI_DFT_FFT_XCD=0/1 forces it off/on for A/B runs)
    const int eb = a.bf16_in ? 2 : 4;
    const int64_t row_bytes = static_cast<int64_t>(cfg.T) * 2 * eb;  // complex or paired-real elements
    bool on = cfg.cols && row_bytes < 128 && nblocks >= 16;
    if (kn.xcd >= 0) on = kn.xcd != 0;
    a.xcd_nb = on ? static_cast<int32_t>(nblocks) : 0;
  }
  best_out = best;
  nblocks_out = nblocks;
  return true;
}

}  // namespace

bool launch_fft_fixed(const PassDesc& d, void* stream) {
  int best = -1;
  FixedArgs a;
  int64_t nblocks = 0;
  if (!prepare_fixed(d, best, a, nblocks)) return false;
  if (nblocks <= 0) return true;
  LaunchFn fn = d.kind == Kind::C2C ? c2c_launcher(best) : (d.kind == Kind::R2C ? r2c_launcher(best) : c2r_launcher(best));
  fn(a, dim3(static_cast<uint32_t>(nblocks)), static_cast<hipStream_t>(stream));
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) throw std::runtime_error(std::string("amd_dft: fixed FFT launch failed: ") + hipGetErrorString(err));
  return true;
}

}  // namespace amd_dft
