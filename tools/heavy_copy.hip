// A stand-in for RCCL's gather kernel on gfx950 (tools/overlap_probe.py, dev tool): 256 VGPRs per
// wave (the v255 clobber forces the allocation), 37.6 KB of LDS per 256-thread block, a few blocks
// copying a buffer -- the resource shape of ncclDevKernel_Generic, so whether it can
// run beside the persistent render grid is decided by the same CU resources.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void __launch_bounds__(256) heavy_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                         size_t n) {
  extern __shared__ uint4 stage[];
  asm volatile("" ::: "v255");
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    stage[threadIdx.x] = src[i];
    dst[i] = stage[threadIdx.x];
  }
}

extern "C" int heavy_copy(const void* src, void* dst, size_t bytes, int blocks, void* stream) {
  const size_t n = bytes / sizeof(uint4);
  hipLaunchKernelGGL(heavy_copy_kernel, dim3(blocks), dim3(256), 37632, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(src), static_cast<uint4*>(dst), n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
