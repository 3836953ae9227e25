// soffset_hazard.hip — does a wide buffer access read its SGPR soffset after issue? (dev tool)
//
// Round 2 saw "stale" path-state reads only with 16-B (dwordx4) path-state accesses, never with
// 8-B ones, and only under some code layouts.  The production ISA shows the
// compiler emitting, for two adjacent path-state accesses of one lane,
//     buffer_store_dwordx4 v[a:a+3], vOFF, s[R:R+3], sX offen
//     s_movk_i32 sX, <offset of the next access>          <- overwrites the first one's soffset
//     buffer_store_dwordx4 v[b:b+3], vOFF, s[R:R+3], sX offen
// If the hardware samples sX per pass of a wide access (a 64-lane dwordx4 is several passes of
// the texture-address unit), the later lanes of the first access would use the NEW offset.
// This program issues exactly such sequences with inline asm (vector-memory instructions only)
// and checks where every lane's data landed / what every lane loaded.
//
//   case 0: store x4 ; s_mov soff ; store x4          (the pattern above)
//   case 1: store x4 ; s_nop 7 ; s_mov soff ; store x4
//   case 2: store x2 ; s_mov soff ; store x2          (the round-2 b64 layout's pattern)
//   case 3: load  x4 ; s_mov soff ; (wait)            loaded data must come from the first offset
//   case 4: load  x2 ; s_mov soff ; (wait)
//   case 5: store x4 ; s_mov soff (different SGPR) ; store x4   (control: no reuse of the SGPR)
//   case 6: case 0 behind 32 outstanding scattered dwordx4 loads (a backed-up address unit)
//   case 7: case 3 behind the same backlog
//   case 8: case 0 with the resource descriptor restored by v_readlane + s_nop 4 just before
//           (the compiler's SGPR-spill reload in front of the kernel's path-state accesses)
// usage: hipcc --offload-arch=gfx950 -O2 -o tools/soffset_hazard.bin tools/soffset_hazard.hip
//        ./tools/soffset_hazard.bin [iterations]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int kLaneBytes = 32;                 // per lane: [+0, +16) first access, [+16, +32) second
constexpr int kWaveBytes = 64 * kLaneBytes;

__device__ inline u32x4 rsrc_of(void* p, unsigned bytes) {
  const unsigned long long a = (unsigned long long)p;
  return u32x4{(unsigned)a, (unsigned)(a >> 32) & 0xffffu, bytes, 0x00020000u};
}

__global__ void hazard_kernel(unsigned* buf, unsigned bytes, int mode, int iter, unsigned* bad) {
  const unsigned lane = threadIdx.x & 63;
  const unsigned wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const unsigned voff = wave * kWaveBytes + lane * kLaneBytes;
  const u32x4 rs = rsrc_of(buf, bytes);
  unsigned* rec = buf + voff / 4;
  unsigned nbad = 0;
  for (int it = 0; it < iter; ++it) {
    const unsigned tag = (unsigned)it * 1000003u + wave * 131u + lane;
    const u32x4 d1 = {tag, tag + 1, tag + 2, tag + 3}, d2 = {~tag, ~tag - 1, ~tag - 2, ~tag - 3};
    // skip lanes in a pattern that changes per iteration (divergent exec, like the render kernel)
    const bool act = ((lane * 2654435761u + (unsigned)it * 40503u) >> 9) & 3u;
    // cases 6, 7: a backlog of 16 scattered dwordx4 loads issued in the SAME asm block just ahead
    // of the tested access (their destinations are clobbered registers; the block ends with
    // s_waitcnt vmcnt(0), so nothing of them is in flight when the compiler's code resumes)
    const unsigned bl = ((tag * 2246822519u) % (bytes / 4096u - 1u)) * 4096u;   // < bytes - 4096
    if (mode <= 2 || mode == 5 || mode == 6 || mode == 8) {
      for (int k = 0; k < 8; ++k) rec[k] = 0xdeadbeefu;   // poison (flat stores)
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (act) {
        unsigned so, so2;
        if (mode == 8) {
          // rsrc words parked in VGPR lanes and restored with v_readlane (SGPR-spill reload)
          unsigned w0 = rs.x, w1 = rs.y, w2 = rs.z, w3 = rs.w;
          // (v_readfirstlane: the first ACTIVE lane, so the words are the ones written here)
          asm volatile(
              "v_mov_b32 v250, %2\n\t"
              "v_mov_b32 v251, %3\n\t"
              "v_mov_b32 v252, %4\n\t"
              "v_mov_b32 v253, %5\n\t"
              "s_nop 7\n\t"
              "v_readfirstlane_b32 s88, v250\n\t"
              "s_mov_b32 %0, 0\n\t"
              "v_readfirstlane_b32 s89, v251\n\t"
              "v_readfirstlane_b32 s90, v252\n\t"
              "v_readfirstlane_b32 s91, v253\n\t"
              "s_nop 4\n\t"
              "buffer_store_dwordx4 %1, %6, s[88:91], %0 offen\n\t"
              "s_mov_b32 %0, 16\n\t"
              "buffer_store_dwordx4 %7, %6, s[88:91], %0 offen\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&s"(so) : "v"(d1), "s"(w0), "s"(w1), "s"(w2), "s"(w3), "v"(voff), "v"(d2)
              : "memory", "v250", "v251", "v252", "v253", "s88", "s89", "s90", "s91");
        } else if (mode == 6) {
          asm volatile(
              "buffer_load_dwordx4 v[192:195], %5, %3, 0 offen offset:0\n\t"
              "buffer_load_dwordx4 v[196:199], %5, %3, 0 offen offset:256\n\t"
              "buffer_load_dwordx4 v[200:203], %5, %3, 0 offen offset:512\n\t"
              "buffer_load_dwordx4 v[204:207], %5, %3, 0 offen offset:768\n\t"
              "buffer_load_dwordx4 v[208:211], %5, %3, 0 offen offset:1024\n\t"
              "buffer_load_dwordx4 v[212:215], %5, %3, 0 offen offset:1280\n\t"
              "buffer_load_dwordx4 v[216:219], %5, %3, 0 offen offset:1536\n\t"
              "buffer_load_dwordx4 v[220:223], %5, %3, 0 offen offset:1792\n\t"
              "buffer_load_dwordx4 v[224:227], %5, %3, 0 offen offset:2048\n\t"
              "buffer_load_dwordx4 v[228:231], %5, %3, 0 offen offset:2304\n\t"
              "buffer_load_dwordx4 v[232:235], %5, %3, 0 offen offset:2560\n\t"
              "buffer_load_dwordx4 v[236:239], %5, %3, 0 offen offset:2816\n\t"
              "buffer_load_dwordx4 v[240:243], %5, %3, 0 offen offset:3072\n\t"
              "buffer_load_dwordx4 v[244:247], %5, %3, 0 offen offset:3328\n\t"
              "buffer_load_dwordx4 v[248:251], %5, %3, 0 offen offset:3584\n\t"
              "buffer_load_dwordx4 v[252:255], %5, %3, 0 offen offset:3840\n\t"
              "s_mov_b32 %0, 0\n\t"
              "buffer_store_dwordx4 %1, %2, %3, %0 offen\n\t"
              "s_mov_b32 %0, 16\n\t"
              "buffer_store_dwordx4 %4, %2, %3, %0 offen\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&s"(so) : "v"(d1), "v"(voff), "s"(rs), "v"(d2), "v"(bl) : "memory", "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255");
        } else if (mode == 0) {
          asm volatile(
              "s_mov_b32 %0, 0\n\t"
              "buffer_store_dwordx4 %1, %2, %3, %0 offen\n\t"
              "s_mov_b32 %0, 16\n\t"
              "buffer_store_dwordx4 %4, %2, %3, %0 offen\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&s"(so) : "v"(d1), "v"(voff), "s"(rs), "v"(d2) : "memory");
        } else if (mode == 1) {
          asm volatile(
              "s_mov_b32 %0, 0\n\t"
              "buffer_store_dwordx4 %1, %2, %3, %0 offen\n\t"
              "s_nop 7\n\t"
              "s_mov_b32 %0, 16\n\t"
              "buffer_store_dwordx4 %4, %2, %3, %0 offen\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&s"(so) : "v"(d1), "v"(voff), "s"(rs), "v"(d2) : "memory");
        } else if (mode == 2) {
          const u32x2 a = {d1.x, d1.y}, b = {d2.x, d2.y};
          asm volatile(
              "s_mov_b32 %0, 0\n\t"
              "buffer_store_dwordx2 %1, %2, %3, %0 offen\n\t"
              "s_mov_b32 %0, 16\n\t"
              "buffer_store_dwordx2 %4, %2, %3, %0 offen\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&s"(so) : "v"(a), "v"(voff), "s"(rs), "v"(b) : "memory");
        } else {
          asm volatile(
              "s_mov_b32 %0, 0\n\t"
              "buffer_store_dwordx4 %2, %3, %4, %0 offen\n\t"
              "s_mov_b32 %1, 16\n\t"
              "buffer_store_dwordx4 %5, %3, %4, %1 offen\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&s"(so), "=&s"(so2) : "v"(d1), "v"(voff), "s"(rs), "v"(d2) : "memory");
        }
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned n = (mode == 2) ? 2 : 4;
        const unsigned w1[4] = {d1.x, d1.y, d1.z, d1.w}, w2[4] = {d2.x, d2.y, d2.z, d2.w};
        bool ok = true;
        for (unsigned k = 0; k < n; ++k) ok = ok && rec[k] == w1[k] && rec[4 + k] == w2[k];
        if (!ok) nbad++;
      }
      __syncthreads();
    } else {
      // loads: the record holds d1 at +0 and d2 at +16 (flat stores), the asm loads +0
      // (cases 3, 4, 7)
      rec[0] = d1.x; rec[1] = d1.y; rec[2] = d1.z; rec[3] = d1.w;
      rec[4] = d2.x; rec[5] = d2.y; rec[6] = d2.z; rec[7] = d2.w;
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (act) {
        unsigned so;
        bool ok;
        if (mode == 7) {
          u32x4 r;
          asm volatile(
              "buffer_load_dwordx4 v[192:195], %4, %3, 0 offen offset:0\n\t"
              "buffer_load_dwordx4 v[196:199], %4, %3, 0 offen offset:256\n\t"
              "buffer_load_dwordx4 v[200:203], %4, %3, 0 offen offset:512\n\t"
              "buffer_load_dwordx4 v[204:207], %4, %3, 0 offen offset:768\n\t"
              "buffer_load_dwordx4 v[208:211], %4, %3, 0 offen offset:1024\n\t"
              "buffer_load_dwordx4 v[212:215], %4, %3, 0 offen offset:1280\n\t"
              "buffer_load_dwordx4 v[216:219], %4, %3, 0 offen offset:1536\n\t"
              "buffer_load_dwordx4 v[220:223], %4, %3, 0 offen offset:1792\n\t"
              "buffer_load_dwordx4 v[224:227], %4, %3, 0 offen offset:2048\n\t"
              "buffer_load_dwordx4 v[228:231], %4, %3, 0 offen offset:2304\n\t"
              "buffer_load_dwordx4 v[232:235], %4, %3, 0 offen offset:2560\n\t"
              "buffer_load_dwordx4 v[236:239], %4, %3, 0 offen offset:2816\n\t"
              "buffer_load_dwordx4 v[240:243], %4, %3, 0 offen offset:3072\n\t"
              "buffer_load_dwordx4 v[244:247], %4, %3, 0 offen offset:3328\n\t"
              "buffer_load_dwordx4 v[248:251], %4, %3, 0 offen offset:3584\n\t"
              "buffer_load_dwordx4 v[252:255], %4, %3, 0 offen offset:3840\n\t"
              "s_mov_b32 %1, 0\n\t"
              "buffer_load_dwordx4 %0, %2, %3, %1 offen\n\t"
              "s_mov_b32 %1, 16\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&v"(r), "=&s"(so) : "v"(voff), "s"(rs), "v"(bl) : "memory", "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255");
          ok = r.x == d1.x && r.y == d1.y && r.z == d1.z && r.w == d1.w;
        } else if (mode == 3) {
          u32x4 r;
          asm volatile(
              "s_mov_b32 %1, 0\n\t"
              "buffer_load_dwordx4 %0, %2, %3, %1 offen\n\t"
              "s_mov_b32 %1, 16\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&v"(r), "=&s"(so) : "v"(voff), "s"(rs) : "memory");
          ok = r.x == d1.x && r.y == d1.y && r.z == d1.z && r.w == d1.w;
        } else {
          u32x2 r;
          asm volatile(
              "s_mov_b32 %1, 0\n\t"
              "buffer_load_dwordx2 %0, %2, %3, %1 offen\n\t"
              "s_mov_b32 %1, 16\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&v"(r), "=&s"(so) : "v"(voff), "s"(rs) : "memory");
          ok = r.x == d1.x && r.y == d1.y;
        }
        if (!ok) nbad++;
      }
      __syncthreads();
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main(int argc, char** argv) {
  const int iter = argc > 1 ? std::atoi(argv[1]) : 200;
  const int blocks = 1024, threads = 256;
  const size_t bytes = (size_t)blocks * (threads / 64) * kWaveBytes;
  unsigned *buf = nullptr, *bad = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&bad, sizeof(unsigned)) != hipSuccess) return 2;
  const char* names[] = {"store x4; s_mov soff; store x4", "store x4; s_nop 7; s_mov soff; store x4",
                         "store x2; s_mov soff; store x2", "load x4; s_mov soff",
                         "load x2; s_mov soff", "store x4; s_mov OTHER sgpr; store x4 (control)",
                         "backlog + store x4; s_mov soff; store x4", "backlog + load x4; s_mov soff",
                         "readlane rsrc; s_nop 4; store x4; s_mov; store x4"};
  for (int mode = 0; mode < 9; ++mode) {
    unsigned h = 0;
    (void)hipMemset(bad, 0, sizeof h);
    hipLaunchKernelGGL(hazard_kernel, dim3(blocks), dim3(threads), 0, nullptr, buf, (unsigned)bytes, mode, iter, bad);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("kernel failed\n"); return 3; }
    (void)hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost);
    const double checks = (double)iter * blocks * threads * 0.75;
    std::printf("case %d  %-48s wrong lane-accesses %10u of ~%.3g (%.2e)\n", mode, names[mode], h, checks,
                h / checks);
  }
  return 0;
}
