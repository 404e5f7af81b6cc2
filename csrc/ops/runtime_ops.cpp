// Runtime helpers for the engine layer.
//
// wrap_device_ptr: view a raw device pointer as a tensor (no copy).  Used by
// Engine.execute_v2(bindings), the TensorRT-style entry point that takes raw device
// addresses (/root/reference/tests/test_dft.py:112-114: context.execute_v2([x_ptr, y_ptr])).
#include <ATen/ATen.h>
#include <torch/library.h>

#include "checks.h"
#include "tuning.h"

namespace amd_dft {
namespace {

at::Tensor wrap_device_ptr(int64_t ptr, at::IntArrayRef shape, at::ScalarType dtype, int64_t device_index) {
  TORCH_CHECK(ptr != 0, "amd_dft.wrap_device_ptr: null pointer");
  auto opts = at::TensorOptions().dtype(dtype).device(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device_index)));
  return at::from_blob(reinterpret_cast<void*>(ptr), shape, opts);
}

at::Tensor wrap_host_ptr(int64_t ptr, at::IntArrayRef shape, at::ScalarType dtype) {
  TORCH_CHECK(ptr != 0, "amd_dft.wrap_host_ptr: null pointer");
  return at::from_blob(reinterpret_cast<void*>(ptr), shape, at::TensorOptions().dtype(dtype));
}

// fallback_counts(): (op names, counts) of every GPU op call that ran without its hand kernel
std::tuple<std::vector<std::string>, std::vector<int64_t>> fallback_counts() {
  auto& r = fallback_registry();
  std::lock_guard<std::mutex> g(r.mu);
  std::vector<std::string> names;
  std::vector<int64_t> counts;
  for (const auto& kv : r.counts) {
    names.push_back(kv.first);
    counts.push_back(kv.second);
  }
  return {names, counts};
}

// fallback_note(op, why): the Python-level generic paths (models/afno.py afno2d_amd's baddbmm
// spectral MLP, ops/spectral.py's F.linear / hipBLASLt MLP) report into the same registry, so
// fallback_counts() and MI_DFT_STRICT cover them too
void fallback_note_op(const std::string& op, const std::string& why) { fallback_note(op.c_str(), why.c_str()); }

void fallback_reset() {
  auto& r = fallback_registry();
  std::lock_guard<std::mutex> g(r.mu);
  r.counts.clear();
  r.total.store(0);
}

// run-time switches (checks.h): return the previous setting
bool set_finite_check(bool on) { return finite_check_flag().exchange(on); }
bool set_strict(bool on) { return strict_flag().exchange(on); }
bool is_tuning_build() { return tuning_build(); }

}  // namespace
}  // namespace amd_dft

TORCH_LIBRARY_FRAGMENT(amd_dft, m) {
  m.def("wrap_device_ptr(int ptr, int[] shape, ScalarType dtype, int device_index) -> Tensor",
        &amd_dft::wrap_device_ptr);
  m.def("wrap_host_ptr(int ptr, int[] shape, ScalarType dtype) -> Tensor", &amd_dft::wrap_host_ptr);
  m.def("fallback_counts() -> (str[], int[])", &amd_dft::fallback_counts);
  m.def("fallback_reset() -> ()", &amd_dft::fallback_reset);
  m.def("fallback_note(str op, str why) -> ()", &amd_dft::fallback_note_op);
  m.def("set_finite_check(bool on) -> bool", &amd_dft::set_finite_check);
  m.def("set_strict(bool on) -> bool", &amd_dft::set_strict);
  m.def("tuning_build() -> bool", &amd_dft::is_tuning_build);
}
