// Opt-in op tracing (the reference has none and leaves timing to trtexec,
// /root/reference/README.md:61-75).  MI_DFT_TRACE=1 wraps every device op in a roctx range
// named "amd_dft::<op>", so `rocprofv3 --marker-trace --kernel-trace` lines each kernel up with
// the op (and the Python-level block ranges, tensorrt_dft_plugins_amd/utils/trace.py) that
// launched it.  The roctx library is dlopen'ed on first use (rocprofiler-sdk's, else the
// legacy libroctx64), so the op library has no link-time dependency on it; when tracing is
// off the cost is one predictable branch per op.
#pragma once

#include <dlfcn.h>

#include <cstdlib>
#include <string>
#include <utility>

namespace amd_dft {

struct RoctxApi {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
};

inline const RoctxApi& roctx_api() {
  static const RoctxApi api = [] {
    RoctxApi a;
    const char* e = std::getenv("MI_DFT_TRACE");
    if (!e || std::string(e) == "0") return a;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                            "libroctx64.so"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      a.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      a.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      if (a.push && a.pop) break;
      a = RoctxApi{};
    }
    return a;
  }();
  return api;
}

inline bool trace_enabled() { return roctx_api().push != nullptr; }

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(trace_enabled()) {
    if (on_) roctx_api().push(name);
  }
  ~TraceRange() {
    if (on_) roctx_api().pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

// Registration-time wrapper: m.impl("r2c", AMD_DFT_TRACED("amd_dft::r2c", r2c_cuda)).
template <auto F, class Sig = decltype(F)>
struct Traced;
template <auto F, class R, class... A>
struct Traced<F, R (*)(A...)> {
  static inline const char* name = "amd_dft::op";
  static R call(A... a) {
    TraceRange t(name);
    return F(std::forward<A>(a)...);
  }
};

template <auto F>
inline auto traced(const char* name) {
  Traced<F>::name = name;
  return &Traced<F>::call;
}

}  // namespace amd_dft

#define AMD_DFT_TRACED(NAME, FN) ::amd_dft::traced<&FN>(NAME)
