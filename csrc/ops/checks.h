// Opt-in output validation for the device ops (the reference only
// asserts and always returns 0 from enqueue).  MI_DFT_CHECK_FINITE=1 makes every op verify
// that its output is finite and raise otherwise.  It synchronises the stream, so it is
// skipped while a hipGraph is being captured.
#pragma once

#include <ATen/ATen.h>
#include <c10/hip/HIPGraphsC10Utils.h>

#include <cstdlib>
#include <string>

namespace amd_dft {

inline bool finite_check_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("MI_DFT_CHECK_FINITE");
    return e && std::string(e) != "0";
  }();
  return on;
}

inline const at::Tensor& checked(const at::Tensor& out, const char* op) {
  if (finite_check_enabled() && out.defined() && out.numel() > 0 &&
      c10::hip::currentStreamCaptureStatusMayInitCtx() == c10::hip::CaptureStatus::None) {
    const bool ok = at::isfinite(out).all().item<bool>();
    TORCH_CHECK(ok, "amd_dft.", op, ": output contains NaN/Inf (MI_DFT_CHECK_FINITE=1)");
  }
  return out;
}

}  // namespace amd_dft
