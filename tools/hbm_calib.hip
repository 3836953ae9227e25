// hbm_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths the render kernel uses (dev tool; MI355X_MICROARCH.md: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Each kernel streams a 2 GiB buffer (8x the 256 MiB Infinity Cache, so every line comes
// from HBM) once, coalesced, with one access width per lane: read_b32 / read_b64 /
// read_b128 and write_b32 / write_b64 / write_b128.  Under `rocprofv3 --pmc FETCH_SIZE`
// (and a separate WRITE_SIZE pass) the counter per dispatch against the known 2 GiB gives
// the bytes-per-counted-KB factor of each width (tools/pmc_summary.py --calib).
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/hbm_calib.bin tools/hbm_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr size_t kBytes = 2ull << 30;

template <typename T>
__device__ void read_kernel(const T* __restrict__ src, size_t n, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = src[i];
    const unsigned* w = reinterpret_cast<const unsigned*>(&v);
    for (size_t k = 0; k < sizeof(T) / 4; ++k) acc ^= w[k];   // every word, so the load stays full width
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;   // practically never: keeps the loads alive
}

template <typename T>
__device__ void write_kernel(T* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v;
    unsigned* w = reinterpret_cast<unsigned*>(&v);
    for (size_t k = 0; k < sizeof(T) / 4; ++k) w[k] = (unsigned)(i + k);
    dst[i] = v;
  }
}

__global__ void read_b32(const unsigned* s, size_t n, unsigned* k) { read_kernel(s, n, k); }
__global__ void read_b64(const uint2* s, size_t n, unsigned* k) { read_kernel(s, n, k); }
__global__ void read_b128(const uint4* s, size_t n, unsigned* k) { read_kernel(s, n, k); }
__global__ void write_b32(unsigned* d, size_t n) { write_kernel(d, n); }
__global__ void write_b64(uint2* d, size_t n) { write_kernel(d, n); }
__global__ void write_b128(uint4* d, size_t n) { write_kernel(d, n); }

int main() {
  char* buf = nullptr;
  unsigned* sink = nullptr;
  CHECK(hipMalloc(&buf, kBytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(buf, 1, kBytes));
  const dim3 grid(256 * 16), block(256);
  // reads; a 2 GiB write between two reads evicts the Infinity Cache
  read_b32<<<grid, block>>>((const unsigned*)buf, kBytes / 4, sink);
  write_b32<<<grid, block>>>((unsigned*)buf, kBytes / 4);
  read_b64<<<grid, block>>>((const uint2*)buf, kBytes / 8, sink);
  write_b64<<<grid, block>>>((uint2*)buf, kBytes / 8);
  read_b128<<<grid, block>>>((const uint4*)buf, kBytes / 16, sink);
  write_b128<<<grid, block>>>((uint4*)buf, kBytes / 16);
  CHECK(hipDeviceSynchronize());
  std::printf("hbm_calib: 6 kernels, %zu bytes each\n", kBytes);
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
