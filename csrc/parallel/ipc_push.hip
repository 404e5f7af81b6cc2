// One launch that copies a shard into up to 16 destination buffers at once (the direct-mesh
// all-gather of parallel/ipc_gather.py): blockIdx.y picks the destination, so the copies to the
// world-1 peers stream over their xGMI links concurrently instead of one after another (a
// hipMemcpyAsync per peer on one stream serialises them).  16-byte vector loads and stores,
// 4 per thread in flight; the source is read once per destination (L2/MALL-resident after the
// first pass).
//
// Visibility: the peer stores go over the fabric into another GPU's memory, and the consumer
// learns of them from a stream packet (flag write / interprocess event) that the command processor
// runs after this kernel.  Each workgroup therefore ends with a SYSTEM-scope release once all of
// its waves' stores have completed: every storing wave waits for its stores (vmcnt(0)), the
// workgroup synchronises, and one lane issues the release fence, which writes back anything the
// local L2 still holds for the peer lines before the kernel can be seen as complete.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "ipc_push.h"

namespace amd_dft {
namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 4;

__global__ void __launch_bounds__(kThreads) ipc_push_kernel(const uint4* __restrict__ src, IpcPushDsts d,
                                                            int64_t n16, int64_t off16) {
  uint4* dst = reinterpret_cast<uint4*>(d.ptr[blockIdx.y]) + off16;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads * kUnroll;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kThreads * kUnroll + threadIdx.x; base < n16; base += stride) {
    if (base + static_cast<int64_t>(kUnroll - 1) * kThreads < n16) {
      // whole batch in range: kUnroll independent loads in flight, then the stores (no per-element
      // guard -- with one the compiler parks the array in LDS and waits for every load in turn)
      uint4 v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) v[u] = src[base + static_cast<int64_t>(u) * kThreads];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) dst[base + static_cast<int64_t>(u) * kThreads] = v[u];
    } else {
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t i = base + static_cast<int64_t>(u) * kThreads;
        if (i < n16) dst[i] = src[i];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: peers and host
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

}  // namespace

void launch_ipc_push(const void* src, int64_t nbytes, const IpcPushDsts& d, int ndst, int64_t offset, void* stream) {
  if (ndst <= 0 || ndst > kIpcMaxDst) throw std::runtime_error("amd_dft: ipc_push: 1..16 destinations");
  if (nbytes % 16 != 0 || offset % 16 != 0 || reinterpret_cast<uintptr_t>(src) % 16 != 0)
    throw std::runtime_error("amd_dft: ipc_push: 16-byte aligned sizes, offsets and source");
  for (int i = 0; i < ndst; ++i)
    if (d.ptr[i] == nullptr || reinterpret_cast<uintptr_t>(d.ptr[i]) % 16 != 0)
      throw std::runtime_error("amd_dft: ipc_push: null or misaligned destination");
  const int64_t n16 = nbytes / 16;
  if (n16 == 0) return;
  const int64_t per = static_cast<int64_t>(kThreads) * kUnroll;
  // ~2 workgroups per CU per destination: enough bytes in flight per link
  const int64_t want = (512 + ndst - 1) / ndst;
  const uint32_t gx = static_cast<uint32_t>(std::max<int64_t>(1, std::min<int64_t>((n16 + per - 1) / per, want)));
  hipLaunchKernelGGL(ipc_push_kernel, dim3(gx, static_cast<uint32_t>(ndst)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint4*>(src), d, n16, offset / 16);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("amd_dft: ipc_push launch: ") + hipGetErrorString(e));
}

}  // namespace amd_dft
