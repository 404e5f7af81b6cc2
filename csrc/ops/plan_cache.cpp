#include "plan_cache.h"

#include <c10/hip/HIPGraphsC10Utils.h>

#include <cstdlib>
#include <list>
#include <mutex>
#include <map>
#include <tuple>
#include <unordered_map>

#include "../spectral/dft_gemm.h"

namespace amd_dft {
namespace {

// ------------------------------------------------------------------ plan cache
class PlanCache {
 public:
  std::shared_ptr<DevPlan> get(int64_t L, const at::Device& dev) {
    const uint64_t key = (static_cast<uint64_t>(dev.index() + 1) << 40) | static_cast<uint64_t>(L);
    std::lock_guard<std::mutex> g(mu_);
    auto it = map_.find(key);
    if (it != map_.end()) {
      lru_.splice(lru_.begin(), lru_, it->second.second);
      return it->second.first;
    }
    TORCH_CHECK(c10::hip::currentStreamCaptureStatusMayInitCtx() == c10::hip::CaptureStatus::None,
                "amd_dft: FFT plan for length ", L,
                " was not created before graph capture; run the model once (warm-up) before capturing");
    auto dp = std::make_shared<DevPlan>();
    dp->plan = make_plan_1d(static_cast<int32_t>(L));
    auto host = at::from_blob(dp->plan.tw_host.data(), {static_cast<int64_t>(dp->plan.tw_host.size())},
                              at::TensorOptions().dtype(at::kFloat));
    dp->tw = host.to(dev);
    lru_.push_front(key);
    map_[key] = {dp, lru_.begin()};
    while (map_.size() > capacity()) {
      map_.erase(lru_.back());
      lru_.pop_back();
    }
    return dp;
  }
  void clear() {
    std::lock_guard<std::mutex> g(mu_);
    map_.clear();
    lru_.clear();
  }
  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return map_.size();
  }

 private:
  static size_t capacity() {
    static size_t cap = [] {
      const char* e = std::getenv("MI_DFT_PLAN_CACHE_SIZE");
      long v = e ? std::atol(e) : 256;
      return static_cast<size_t>(v > 0 ? v : 256);
    }();
    return cap;
  }
  std::mutex mu_;
  std::list<uint64_t> lru_;
  std::unordered_map<uint64_t, std::pair<std::shared_ptr<DevPlan>, std::list<uint64_t>::iterator>> map_;
};

PlanCache& plan_cache() {
  static PlanCache c;
  return c;
}

}  // namespace

std::shared_ptr<DevPlan> get_plan(int64_t L, const at::Device& dev) { return plan_cache().get(L, dev); }

std::pair<at::Tensor, at::Tensor> get_dft_gemm_tables(DftTable kind, int W, int m, const at::Device& dev) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int>, std::pair<at::Tensor, at::Tensor>> cache;
  const auto key = std::make_tuple(static_cast<int>(kind), W, m, static_cast<int>(dev.index()));
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  TORCH_CHECK(c10::hip::currentStreamCaptureStatusMayInitCtx() == c10::hip::CaptureStatus::None,
              "amd_dft: DFT-GEMM tables for length ", W, " were not created before graph capture; run the model "
              "once (warm-up) before capturing");
  std::vector<uint16_t> frag;
  std::vector<float> ph;
  if (kind == DftTable::R2C) dftw_r2c_tables(W, m, frag, ph);
  else fno_c2r_tables(W, m, kind == DftTable::C2R_BF16 ? kFnoChunkBF : kFnoChunkF32, frag, ph);
  auto f = at::from_blob(frag.data(), {static_cast<int64_t>(frag.size())}, at::TensorOptions().dtype(at::kShort))
               .to(dev);
  auto p = at::from_blob(ph.data(), {static_cast<int64_t>(ph.size())}, at::TensorOptions().dtype(at::kFloat)).to(dev);
  // Never evicted: captured graphs keep raw pointers to these tables.
  return cache[key] = {f, p};
}
size_t plan_cache_entries() { return plan_cache().size(); }
void plan_cache_reset() { plan_cache().clear(); }

}  // namespace amd_dft
