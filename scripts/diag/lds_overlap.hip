// Co-resident workgroups must never see each other's LDS: every WG fills its dynamic LDS with
// its own id, spins, and counts words that changed.  Usage: ./lds_overlap <lds_bytes> <nwg>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(256) fill_check(unsigned* bad, int words, int spins) {
  extern __shared__ unsigned lds[];
  const unsigned tag = 0x5a000000u | blockIdx.x;
  for (int i = threadIdx.x; i < words; i += blockDim.x) lds[i] = tag ^ i;
  __syncthreads();
  unsigned acc = 0;
  for (int s = 0; s < spins; ++s) {
    for (int i = threadIdx.x; i < words; i += blockDim.x) acc += (lds[i] != (tag ^ i)) ? 1u : 0u;
    __syncthreads();
  }
  if (acc) atomicAdd(bad, acc);
}

int main(int argc, char** argv) {
  const int bytes = argc > 1 ? atoi(argv[1]) : 38400;
  const int nwg = argc > 2 ? atoi(argv[2]) : 2048;
  unsigned* d;
  hipMalloc(&d, 4);
  hipMemset(d, 0, 4);
  hipFuncSetAttribute(reinterpret_cast<const void*>(fill_check), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  hipLaunchKernelGGL(fill_check, dim3(nwg), dim3(256), bytes, 0, d, bytes / 4, 50);
  hipError_t e = hipDeviceSynchronize();
  unsigned h = 0;
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("lds_bytes=%d nwg=%d err=%s mismatches=%u\n", bytes, nwg, hipGetErrorString(e), h);
  return 0;
}
