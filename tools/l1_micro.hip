// L1-resident gather microbenchmark (dev tool): what a wave-level "node visit"
// costs on gfx950 as a function of loads per visit, bytes per load and how many
// distinct lines the 64 lanes touch.  Dependent pointer chase over a small
// table of 128-B records (stays in the 32 KiB L1), 16 waves per CU.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/l1_micro tools/l1_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int LOADS>
__global__ void __launch_bounds__(256) chase(const uint4* __restrict__ tab, int nrec, int iters, int group, unsigned* out,
                                             int active) {
  const int lane = threadIdx.x & 63;
  if (lane >= active) return;   // partially active waves: does the gather cost scale with lanes?
  // lanes in the same group of `group` lanes start on the same record
  unsigned idx = (unsigned)(((lane / group) * 7919u + blockIdx.x * 131u + (threadIdx.x >> 6) * 17u) % (unsigned)nrec);
  unsigned acc = 0;
  for (int it = 0; it < iters; ++it) {
    const uint4* r = tab + (size_t)idx * 8;
    unsigned s = 0, nxt = 0;
#pragma unroll
    for (int k = 0; k < LOADS; ++k) {
      const uint4 v = r[k];
      if (k == 0) nxt = v.x;
      s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    acc += s;
    idx = nxt;   // next record: a dependent chase through a permutation
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int LOADS>
float run(const uint4* d_tab, int nrec, int iters, int group, unsigned* d_out, int blocks, int active = 64) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  chase<LOADS><<<blocks, 256>>>(d_tab, nrec, 10, group, d_out, active);
  CHECK(hipEventRecord(a));
  chase<LOADS><<<blocks, 256>>>(d_tab, nrec, iters, group, d_out, active);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main() {
  int dev = 0; hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, dev));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 4;          // 16 waves / CU
  const int iters = 4000;
  const double ghz = prop.clockRate / 1e6;
  printf("CUs %d  clock %.2f GHz\n", cus, ghz);
  for (int nrec : {64, 200}) {
    std::vector<uint4> tab((size_t)nrec * 8);
    srand(1);
    std::vector<unsigned> perm(nrec);
    for (int i = 0; i < nrec; ++i) perm[i] = i;
    for (int i = nrec - 1; i > 0; --i) { int j = rand() % (i + 1); std::swap(perm[i], perm[j]); }
    for (int i = 0; i < nrec; ++i)
      for (int k = 0; k < 8; ++k) tab[(size_t)i * 8 + k] = make_uint4(k == 0 ? perm[i] : rand(), rand(), rand(), rand());
    uint4* d_tab; unsigned* d_out;
    CHECK(hipMalloc(&d_tab, tab.size() * sizeof(uint4)));
    CHECK(hipMalloc(&d_out, 4));
    CHECK(hipMemcpy(d_tab, tab.data(), tab.size() * sizeof(uint4), hipMemcpyHostToDevice));
    for (int group : {64, 16, 4, 1}) {
      float ms[4] = {run<1>(d_tab, nrec, iters, group, d_out, blocks), run<4>(d_tab, nrec, iters, group, d_out, blocks),
                     run<7>(d_tab, nrec, iters, group, d_out, blocks), run<8>(d_tab, nrec, iters, group, d_out, blocks)};
      const int L[4] = {1, 4, 7, 8};
      printf("records %3d (%5d B) lanes/line %2d:", nrec, nrec * 128, group);
      for (int i = 0; i < 4; ++i) {
        // cycles per wave-iteration per CU (16 waves share the CU)
        const double cyc = ms[i] * 1e-3 * ghz * 1e9 / ((double)iters * 16);
        printf("  %d loads: %6.1f cyc/visit/CU (%5.1f per load)", L[i], cyc, cyc / L[i]);
      }
      printf("\n");
    }
    for (int active : {64, 32, 16, 4}) {
      const float ms = run<7>(d_tab, nrec, iters, 1, d_out, blocks, active);
      const float ms2 = run<7>(d_tab, nrec, iters, 64, d_out, blocks, active);
      const double c1 = ms * 1e-3 * ghz * 1e9 / ((double)iters * 16), c2 = ms2 * 1e-3 * ghz * 1e9 / ((double)iters * 16);
      printf("records %3d active lanes %2d, 7 loads: divergent %6.1f cyc/visit/CU, coherent %6.1f\n", nrec, active, c1, c2);
    }
    CHECK(hipFree(d_tab)); CHECK(hipFree(d_out));
  }
  return 0;
}
