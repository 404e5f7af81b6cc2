// Host interface of the multi-destination push kernel (ipc_push.hip).
#pragma once

#include <cstdint>

namespace amd_dft {

constexpr int kIpcMaxDst = 16;
struct IpcPushDsts {
  void* ptr[kIpcMaxDst];
};
// src (nbytes, 16-byte multiple) -> every d.ptr[i] + offset, i < ndst, on `stream`
void launch_ipc_push(const void* src, int64_t nbytes, const IpcPushDsts& d, int ndst, int64_t offset, void* stream);

}  // namespace amd_dft
