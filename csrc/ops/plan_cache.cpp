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
// LRU over (device, length), capacity MI_DFT_PLAN_CACHE_SIZE (default 256).  A plan looked up
// while the current stream is capturing a hipGraph is PINNED: the graph holds the raw
// pointer of its twiddle table, so a pinned plan is never evicted and survives
// plan_cache_clear() (eviction after capture would let the allocator hand the
// twiddles' memory to another tensor under a live graph).
class PlanCache {
 public:
  std::shared_ptr<DevPlan> get(int64_t L, const at::Device& dev) {
    const uint64_t key = (static_cast<uint64_t>(dev.index() + 1) << 40) | static_cast<uint64_t>(L);
    const bool capturing = c10::hip::currentStreamCaptureStatusMayInitCtx() != c10::hip::CaptureStatus::None;
    std::lock_guard<std::mutex> g(mu_);
    auto it = map_.find(key);
    if (it != map_.end()) {
      lru_.splice(lru_.begin(), lru_, it->second.pos);
      if (capturing) it->second.pinned = true;
      return it->second.plan;
    }
    TORCH_CHECK(!capturing, "amd_dft: FFT plan for length ", L,
                " was not created before graph capture; run the model once (warm-up) before capturing");
    auto dp = std::make_shared<DevPlan>();
    dp->plan = make_plan_1d(static_cast<int32_t>(L));
    auto host = at::from_blob(dp->plan.tw_host.data(), {static_cast<int64_t>(dp->plan.tw_host.size())},
                              at::TensorOptions().dtype(at::kFloat));
    dp->tw = host.to(dev);
    lru_.push_front(key);
    map_[key] = Entry{dp, lru_.begin(), false};
    evict_locked();
    return dp;
  }
  // drops every unpinned plan; refused while a graph is being captured
  void clear() {
    TORCH_CHECK(c10::hip::currentStreamCaptureStatusMayInitCtx() == c10::hip::CaptureStatus::None,
                "amd_dft.plan_cache_clear: not allowed during hipGraph capture");
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = lru_.begin(); it != lru_.end();) {
      auto e = map_.find(*it);
      if (e->second.pinned) {
        ++it;
      } else {
        map_.erase(e);
        it = lru_.erase(it);
      }
    }
  }
  size_t size() {
    std::lock_guard<std::mutex> g(mu_);
    return map_.size();
  }
  size_t pinned() {
    std::lock_guard<std::mutex> g(mu_);
    size_t n = 0;
    for (const auto& kv : map_) n += kv.second.pinned ? 1 : 0;
    return n;
  }

 private:
  struct Entry {
    std::shared_ptr<DevPlan> plan;
    std::list<uint64_t>::iterator pos;
    bool pinned;
  };
  void evict_locked() {
    auto it = lru_.end();
    while (map_.size() > capacity() && it != lru_.begin()) {
      --it;
      auto e = map_.find(*it);
      if (e->second.pinned) continue;  // oldest unpinned first
      map_.erase(e);
      it = lru_.erase(it);
    }
  }
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
  std::unordered_map<uint64_t, Entry> map_;
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
size_t plan_cache_pinned() { return plan_cache().pinned(); }
void plan_cache_reset() { plan_cache().clear(); }

}  // namespace amd_dft
