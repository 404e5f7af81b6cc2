// Runtime helpers of the direct-mesh (IPC) all-gather over xGMI (SURVEY §5.8, C-1 call site).
//
// RCCL's all_gather moves (world-1) shards through every link of a ring; on the MI355X's
// point-to-point xGMI mesh each GPU has a direct link to every peer, so a rank can instead
// write its shard straight into every peer's output buffer (world-1 concurrent peer copies,
// one per link).  These ops expose the HIP pieces that needs:
//   _ipc_alloc      hipMalloc'd buffer (an IPC handle names a whole allocation, so the gather
//                   buffers cannot come from the caching allocator's sub-blocks)
//   _ipc_mem_handle / _ipc_open_mem / _ipc_close_mem      hipIpc{Get,Open,Close}MemHandle
//   _ipc_event_*    inter-process events (hipEventInterprocess): record on the producer's
//                   stream, hipStreamWaitEvent on the consumer's
//   _ipc_write_value / _ipc_wait_value   stream-ordered flag words (hipStreamWrite/WaitValue32)
//   _ipc_can_access_peer                 hipDeviceCanAccessPeer (checked for every rank pair first)
//   _ipc_push       one kernel copying a source to N destination pointers concurrently on
//                   the current stream (peer stores over xGMI, one link per destination)
// Names start with '_' so they are never exported into ONNX graphs (raw device pointers).
// The reference has no multi-GPU path at all ("assuming single GPU",
// /root/reference/src/dft_plugins/dft_plugins.cpp:341).
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include "../parallel/ipc_push.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

namespace amd_dft {
namespace {

void hip_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "amd_dft.", what, ": ", hipGetErrorString(e));
}

at::Tensor ipc_alloc(int64_t bytes, int64_t device) {
  TORCH_CHECK(bytes > 0, "amd_dft._ipc_alloc: bytes must be positive");
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));  // restores the caller's device
  void* p = nullptr;
  hip_ok(hipMalloc(&p, static_cast<size_t>(bytes)), "_ipc_alloc(hipMalloc)");
  auto opts = at::TensorOptions().dtype(at::kByte).device(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device)));
  // freed only when the last tensor reference goes: IpcAllGather.close() drops it in its second
  // teardown phase, after a barrier that every peer reaches only once it has unmapped this
  // buffer (hipIpcCloseMemHandle) and released the events it opened -- never while mapped
  return at::from_blob(p, {bytes}, [](void* q) { (void)hipFree(q); }, opts);
}

at::Tensor ipc_mem_handle(const at::Tensor& buf) {
  TORCH_CHECK(buf.is_cuda() && buf.storage_offset() == 0, "amd_dft._ipc_mem_handle: needs the base of an _ipc_alloc buffer");
  hipIpcMemHandle_t h;
  hip_ok(hipIpcGetMemHandle(&h, buf.data_ptr()), "_ipc_mem_handle");
  at::Tensor out = at::empty({HIP_IPC_HANDLE_SIZE}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &h, HIP_IPC_HANDLE_SIZE);
  return out;
}

hipIpcMemHandle_t as_mem_handle(const at::Tensor& h) {
  TORCH_CHECK(h.numel() == HIP_IPC_HANDLE_SIZE && h.scalar_type() == at::kByte, "amd_dft: IPC handles are uint8[64]");
  hipIpcMemHandle_t m;
  std::memcpy(&m, h.contiguous().cpu().data_ptr(), HIP_IPC_HANDLE_SIZE);
  return m;
}

int64_t ipc_open_mem(const at::Tensor& handle, int64_t device) {
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  void* p = nullptr;
  hip_ok(hipIpcOpenMemHandle(&p, as_mem_handle(handle), hipIpcMemLazyEnablePeerAccess), "_ipc_open_mem");
  return reinterpret_cast<int64_t>(p);
}

void ipc_close_mem(int64_t ptr) { hip_ok(hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr)), "_ipc_close_mem"); }

int64_t ipc_event_create(int64_t device) {
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  hipEvent_t ev;
  hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventInterprocess), "_ipc_event_create");
  return reinterpret_cast<int64_t>(ev);
}

at::Tensor ipc_event_handle(int64_t ev) {
  hipIpcEventHandle_t h;
  hip_ok(hipIpcGetEventHandle(&h, reinterpret_cast<hipEvent_t>(ev)), "_ipc_event_handle");
  at::Tensor out = at::empty({HIP_IPC_HANDLE_SIZE}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &h, HIP_IPC_HANDLE_SIZE);
  return out;
}

int64_t ipc_event_open(const at::Tensor& handle, int64_t device) {
  TORCH_CHECK(handle.numel() == HIP_IPC_HANDLE_SIZE && handle.scalar_type() == at::kByte,
              "amd_dft._ipc_event_open: IPC handles are uint8[64]");
  c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
  hipIpcEventHandle_t h;
  std::memcpy(&h, handle.contiguous().cpu().data_ptr(), HIP_IPC_HANDLE_SIZE);
  hipEvent_t ev;
  hip_ok(hipIpcOpenEventHandle(&ev, h), "_ipc_event_open");
  return reinterpret_cast<int64_t>(ev);
}

void ipc_event_record(int64_t ev, int64_t device) {
  auto st = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device)).stream();
  hip_ok(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), st), "_ipc_event_record");
}

void ipc_stream_wait(int64_t ev, int64_t device) {
  auto st = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device)).stream();
  hip_ok(hipStreamWaitEvent(st, reinterpret_cast<hipEvent_t>(ev), 0), "_ipc_stream_wait");
}

void ipc_event_destroy(int64_t ev) { (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)); }

// Whether `device` can map and store into `peer`'s memory (the direct mesh's precondition: every
// push is a peer store over the xGMI link between the two GPUs).
bool ipc_can_access_peer(int64_t device, int64_t peer) {
  if (device == peer) return true;
  int ok = 0;
  hip_ok(hipDeviceCanAccessPeer(&ok, static_cast<int>(device), static_cast<int>(peer)), "_ipc_can_access_peer");
  return ok != 0;
}

// Stream-ordered 32-bit flag write / wait (the counted gather protocol: no host handshake).  The
// write runs on the command processor after everything enqueued before it on the current stream;
// the wait blocks the stream (not the host, not a CU) until *ptr >= value.  ptr: a hipMalloc'd
// flag word of this process or one mapped from a peer (hipIpcOpenMemHandle).
void ipc_write_value(int64_t ptr, int64_t value, int64_t device) {
  TORCH_CHECK(ptr != 0 && ptr % 4 == 0 && value >= 0 && value <= 0xffffffffLL, "amd_dft._ipc_write_value: bad flag");
  auto st = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device)).stream();
  hip_ok(hipStreamWriteValue32(st, reinterpret_cast<void*>(ptr), static_cast<uint32_t>(value), 0), "_ipc_write_value");
}

void ipc_wait_value(int64_t ptr, int64_t value, int64_t device) {
  TORCH_CHECK(ptr != 0 && ptr % 4 == 0 && value >= 0 && value <= 0xffffffffLL, "amd_dft._ipc_wait_value: bad flag");
  auto st = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device)).stream();
  hip_ok(hipStreamWaitValue32(st, reinterpret_cast<void*>(ptr), static_cast<uint32_t>(value), hipStreamWaitValueGte,
                              0xffffffffu),
         "_ipc_wait_value");
}

// src -> every dst_ptrs[i] + offset (bytes), stream-ordered on the current stream: one kernel,
// all destinations concurrently (csrc/parallel/ipc_push.hip); hipMemcpyAsync fallback for
// unaligned sizes
void ipc_push(const at::Tensor& src, at::IntArrayRef dst_ptrs, int64_t offset) {
  TORCH_CHECK(src.is_cuda() && src.is_contiguous(), "amd_dft._ipc_push: src must be a contiguous device tensor");
  TORCH_CHECK(!dst_ptrs.empty() && dst_ptrs.size() <= static_cast<size_t>(kIpcMaxDst), "amd_dft._ipc_push: 1..16 destinations");
  auto st = c10::hip::getCurrentHIPStream(src.device().index()).stream();
  const int64_t n = src.numel() * src.element_size();
  IpcPushDsts d{};
  for (size_t i = 0; i < dst_ptrs.size(); ++i) {
    TORCH_CHECK(dst_ptrs[i] != 0, "amd_dft._ipc_push: null destination");
    d.ptr[i] = reinterpret_cast<void*>(dst_ptrs[i]);
  }
  const bool aligned = n % 16 == 0 && offset % 16 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 &&
                       std::all_of(dst_ptrs.begin(), dst_ptrs.end(), [](int64_t p) { return p % 16 == 0; });
  if (aligned) {
    launch_ipc_push(src.data_ptr(), n, d, static_cast<int>(dst_ptrs.size()), offset, st);
    return;
  }
  for (int64_t p : dst_ptrs)
    hip_ok(hipMemcpyAsync(reinterpret_cast<char*>(p) + offset, src.data_ptr(), static_cast<size_t>(n),
                          hipMemcpyDeviceToDevice, st),
           "_ipc_push");
}

}  // namespace
}  // namespace amd_dft

TORCH_LIBRARY_FRAGMENT(amd_dft, m) {
  m.def("_ipc_alloc(int bytes, int device) -> Tensor", &amd_dft::ipc_alloc);
  m.def("_ipc_mem_handle(Tensor buf) -> Tensor", &amd_dft::ipc_mem_handle);
  m.def("_ipc_open_mem(Tensor handle, int device) -> int", &amd_dft::ipc_open_mem);
  m.def("_ipc_close_mem(int ptr) -> ()", &amd_dft::ipc_close_mem);
  m.def("_ipc_event_create(int device) -> int", &amd_dft::ipc_event_create);
  m.def("_ipc_event_handle(int ev) -> Tensor", &amd_dft::ipc_event_handle);
  m.def("_ipc_event_open(Tensor handle, int device) -> int", &amd_dft::ipc_event_open);
  m.def("_ipc_event_record(int ev, int device) -> ()", &amd_dft::ipc_event_record);
  m.def("_ipc_stream_wait(int ev, int device) -> ()", &amd_dft::ipc_stream_wait);
  m.def("_ipc_event_destroy(int ev) -> ()", &amd_dft::ipc_event_destroy);
  m.def("_ipc_can_access_peer(int device, int peer) -> bool", &amd_dft::ipc_can_access_peer);
  m.def("_ipc_write_value(int ptr, int value, int device) -> ()", &amd_dft::ipc_write_value);
  m.def("_ipc_wait_value(int ptr, int value, int device) -> ()", &amd_dft::ipc_wait_value);
  m.def("_ipc_push(Tensor src, int[] dst_ptrs, int offset) -> ()", &amd_dft::ipc_push);
}
