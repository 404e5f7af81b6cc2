// Opt-in output validation for the device ops (the reference only
// asserts and always returns 0 from enqueue).  MI_DFT_CHECK_FINITE=1 makes every op verify
// that its output is finite and raise otherwise.  It synchronises the stream, so it is
// skipped while a hipGraph is being captured.
#pragma once

#include <ATen/ATen.h>
#include <c10/hip/HIPGraphsC10Utils.h>

#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>

namespace amd_dft {

// Both switches start from their environment variable and can be flipped at run time
// (torch.ops.amd_dft.set_finite_check / set_strict; utils.runtime.finite_checks / strict_mode).
inline bool env_flag(const char* name) {
  const char* e = std::getenv(name);
  return e && std::string(e) != "0";
}
inline std::atomic<bool>& finite_check_flag() {
  static std::atomic<bool> on{env_flag("MI_DFT_CHECK_FINITE")};
  return on;
}
inline std::atomic<bool>& strict_flag() {
  static std::atomic<bool> on{env_flag("MI_DFT_STRICT")};
  return on;
}
inline bool finite_check_enabled() { return finite_check_flag().load(std::memory_order_relaxed); }

inline const at::Tensor& checked(const at::Tensor& out, const char* op) {
  if (finite_check_enabled() && out.defined() && out.numel() > 0 &&
      c10::hip::currentStreamCaptureStatusMayInitCtx() == c10::hip::CaptureStatus::None) {
    const bool ok = at::isfinite(out).all().item<bool>();
    TORCH_CHECK(ok, "amd_dft.", op, ": output contains NaN/Inf (MI_DFT_CHECK_FINITE=1)");
  }
  return out;
}

// ---- visible fallbacks: every time a GPU op routes to ATen / a vendor
// library instead of its hand kernel it is counted per op, warned once per op, and raises
// when MI_DFT_STRICT=1 (tests and benches assert zero fallbacks on the hot paths).
struct FallbackRegistry {
  std::mutex mu;
  std::map<std::string, int64_t> counts;
  std::atomic<int64_t> total{0};
};
inline FallbackRegistry& fallback_registry() {
  static FallbackRegistry r;
  return r;
}
inline void fallback_note(const char* op, const char* why) {
  TORCH_CHECK(!strict_flag().load(std::memory_order_relaxed), "amd_dft.", op, ": no hand kernel for this call (", why, ") and MI_DFT_STRICT=1");
  auto& r = fallback_registry();
  bool first = false;
  {
    std::lock_guard<std::mutex> g(r.mu);
    first = r.counts[op]++ == 0;
  }
  r.total.fetch_add(1);
  if (first) TORCH_WARN("amd_dft.", op, ": falling back to ATen (", why, "); counted in amd_dft.fallback_counts()");
}

}  // namespace amd_dft
