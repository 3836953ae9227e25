// rt_render.hip — the MI355X render path: one flattened, persistent CDNA4
// kernel plus the C-ABI boundary of librt_hip.so (include/rt_hip.h).
//
// Replaces the reference's device chain (mytracer_gpu.cu:119-693)
//   compute_image_device -> trace_device -> intersect_scene_device ->
//   intersectBVH_device -> intersect_triangle_device / intersectAABB_device
//   -> lighting_device (+ diffuse_device, reflection_device)
// with ONE kernel in which every lane runs a small state machine over the
// rays of its pixel (primary -> per-light shadow rays -> reflection -> ...),
// all ray kinds sharing one traversal loop:
//   * traversal: ordered, t-culled, speculative while-while over 4-wide fp32
//     nodes (128 B, conservative outward-rounded boxes) of the device hierarchy
//     (binned SAH with spatial splits by default); the top treelet is copied
//     into each block's LDS; the per-ray stack is an LDS ring (8 entries, 16 on
//     deep scenes: render_kernel<4, false, false, 16>) spilling to global
//     memory; closest-hit for primary / reflection rays, any-hit bounded by the
//     light distance for shadow rays (the reference traces full closest-hit
//     shadow rays, mytracer_gpu.cu:653-660; the shadow predicate is the same);
//     the closest hit is the smallest (t, reference slot), so any hierarchy
//     over the same records gives the same bits;
//   * triangle test and all shading in fp64 with the reference CPU
//     renderer's operation order (mymesh.cpp:186-235, mytracer.cpp:510-608),
//     compiled with fp-contract off, so hits are bit-identical to the oracle;
//   * rays live in LDS slots (fp64 origin / direction / t-limit + 3 aux words
//     holding the hit's barycentrics or the bounce normal); idle lanes are lent
//     to owners for their extra shadow rays and reflection ray (fan-out);
//   * work distribution: persistent workgroups pull 8x8 pixel tiles from 8
//     work heads on separate cache lines, one per XCD group, refilled per wave
//     with a single atomic when >= kRefill lanes are idle; several frames per
//     launch share the queue in band-major order (each head serves one row band
//     of every frame); once the queue is empty, sparse waves hand their pixels
//     to the other waves of their block (tail compaction);
//   * reflection rays are spawned only when mirror > 0 (CPU semantics,
//     mytracer.cpp:547); the reference GPU traces max_depth zero-weight
//     bounces (mytracer_gpu.cu:281-310) — same pixels, less work.
// No MFMA: the path is a traversal / latency problem.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <atomic>
#include <climits>
#include <thread>
#include <deque>
#include <chrono>

#include "../../../include/rt_hip.h"
#include "rt_layout.hpp"

#pragma clang fp contract(off)

using namespace rtk;

namespace {

#ifndef RT_BLOCK
#define RT_BLOCK 256
#endif
constexpr int kBlock = RT_BLOCK;   // threads per persistent block
constexpr int kGroups = 8;          // work heads (XCD groups)
#ifndef RT_REFILL
#define RT_REFILL 16
#endif
constexpr int kRefill = RT_REFILL;  // refill a wave when this many lanes are idle
constexpr int kCtrWords = 40;       // [8,16) stats (STATS variants), [16,40) diagnostics (31: guard)
#ifndef RT_SHORT_STACK
#define RT_SHORT_STACK 8
#endif
// Traversal stack: the top kShortStack entries live in an LDS ring (slot i & kStackMask),
// deeper entries spill to a per-lane global array.  Bounds LDS per block independently
// of tree depth, so occupancy stays VGPR-limited.
constexpr int kShortStack = RT_SHORT_STACK;
// Top treelet in LDS: the first kTopNodes 4-wide nodes (breadth-first numbering) are copied
// into each block's LDS; a node iteration whose active lanes all sit in the treelet reads
// LDS instead of the vector-L1 path.  0 disables.
// LDS per thread: kSlotDoubles fp64 slot words, task + visibility words, the stack ring
#define RT_SLOT_DOUBLES 10
#ifndef RT_TOP_NODES   // fills the CU's 160 KB at 4 blocks with the slots, ring, lights, pool
#define RT_TOP_NODES \
  ((40960 - RT_BLOCK * (RT_SLOT_DOUBLES * 8 + (2 + RT_SHORT_STACK) * 4) - RT_MAX_LIGHTS * 48 - 64) / 128)
#endif
constexpr int kTopNodes = RT_TOP_NODES > 0 ? RT_TOP_NODES : 1;
constexpr int kStackMask = kShortStack - 1;
// Tail compaction: once the work queue is empty, a wave with at most kDonateMax
// pixels in flight hands them to the other waves of its block and exits, so the last pixels
// of a launch run in fewer, fuller waves.  A handed-over lane's registers travel through the
// donor thread's LDS stack entries (free between traversals): kMigWords words (packed; the
// closest-hit distance and the hit attributes travel in the LDS slot, copied with it).
#ifndef RT_BAND_ORDER   // several frames per launch: band-major work order
#define RT_BAND_ORDER 1
#endif
#ifndef RT_DONATE_MAX
#define RT_DONATE_MAX 24
#endif
constexpr int kDonateMax = RT_DONATE_MAX;
constexpr int kMigWords = 8;
static_assert(kMigWords <= kShortStack, "migration words travel in the stack ring entries");
constexpr int kPoolBytes = 64;   // LDS: live-wave count, one 64-bit lane mask per wave of the block, exhausted heads
static_assert(8 + 8 * (RT_BLOCK / 64) + 4 <= kPoolBytes, "compaction pool does not fit");
static_assert((kShortStack & kStackMask) == 0, "RT_SHORT_STACK must be a power of two");

// Lane states.  Owners carry a pixel (CLOSEST: closest-hit ray in flight; SHADOW: a
// batch of shadow rays in flight).  Idle lanes (FETCH / DONE) may be lent to an
// owner of the same wave for one round (HSHADOW / HCLOSEST): they trace one of its
// extra shadow rays or its reflection ray, so a bounce costs one round, not 1 + lights.
enum : int { ST_FETCH = 0, ST_CLOSEST = 1, ST_SHADOW = 2, ST_DONE = 3, ST_HSHADOW = 4, ST_HCLOSEST = 5 };
constexpr uint32_t kTaskNone = 0xffffffffu;
// task word: owner lane | (light - owner's first light of the batch) << 6 | light << 11, or
// owner lane | kTaskRefl.  The helper derives its ray itself at the start of the traversal from
// the owner's slot (closest-hit ray, hit distance, hit normal in the aux words).
constexpr uint32_t kTaskRefl = 0x80000000u;
static_assert(RT_LIGHTS_LIMIT <= (1 << 20), "light index must fit the task word");
// a bounce's shadow rays go out in batches of at most 1 + kBatchExtra lights (the owner's
// own ray + one helper per extra light): the helpers' occlusion bits fit one LDS word
constexpr int kBatchExtra = 31;

// Orders LDS traffic between lanes of one wave: LDS executes a wave's operations in
// issue order, so it suffices to stop the compiler from moving memory operations
// across this point and to drain outstanding LDS operations.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Raw buffer access (gfx9 resource word 3; no format conversion).
constexpr int kBufWord3 = 0x00020000;
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double x) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, x), r, voff, soff, 0);
}


// Lane of the k-th (0-based) set bit of m (k < popcount(m)).
__device__ __forceinline__ int kth_set_bit(unsigned long long m, int k) {
  int base = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int c = __popcll(m & ((1ull << w) - 1ull));
    if (k >= c) { k -= c; m >>= w; base += w; }
  }
  return base;
}
enum : int { CS_PRIMARY = 8, CS_SHADOW, CS_REFLECT, CS_NODES, CS_TRIS, CS_HITS, CS_PIXELS };
// diagnostics (STATS variants only): wave-level loop iterations and the active
// lanes summed over them (SIMD efficiency), s_memtime cycles per phase.
enum : int {
  CD_NODE_ITERS = 16, CD_NODE_LANES, CD_LEAF_ITERS, CD_LEAF_LANES, CD_TRAV_CYCLES, CD_SHADE_CYCLES,
  CD_FETCH_CYCLES, CD_OUTER_ITERS, CD_TRAV_ROUNDS, CD_TRAV_ROUND_LANES, CD_SPILLS, CD_NODE_LINES,
  CD_LEAF_LINES, CD_BIG_LEAF_TESTS, CD_NODE_LDS_ITERS, CD_GUARD = 31,   // CD_GUARD: a wave hit the iteration guard
  CD_GNODE_UNIFORM = 32, CD_GNODE_DISTINCT, CD_LEAF_UNIFORM
};
// Watchdogs (never reached by a correct kernel): the persistent loop, and the wave-level
// iterations of one traversal round (round, node and leaf loops together).  A wave that
// trips either ends its work instead of spinning and flags the launch (CD_GUARD), which
// the host reports as an error.
constexpr unsigned kGuardIters = 1u << 24;
constexpr unsigned kTravGuard = 1u << 24;
constexpr int kTlCap = 256;   // TL variant: traversal rounds recorded per wave
constexpr int kTlWords = 8;   // ... and words per round

constexpr int kMaxFrames = RT_MAX_FRAMES;   // frames per launch
// adaptive-pass list entries: frame << 25 | local pixel id (lrow * W + x)
constexpr int kListFrameShift = 25;
constexpr uint32_t kListPixMask = (1u << kListFrameShift) - 1u;
static_assert(kMaxFrames <= (1 << (32 - kListFrameShift)), "frame index must fit a list entry");
// per-frame camera and output buffer; a launch's table follows its counters in device memory
struct FrameDesc {
  double eye[3], ll[3], xd[3], yd[3];
  void* out;
  long long pad;
};
static_assert(sizeof(FrameDesc) == 112, "FrameDesc must be 112 bytes");
// Launch control block (one H2D copy per launch): counter words, the work heads (one per 256-B
// line: device-scope atomics on one line serialise at the memory side, and a refilling wave
// waits for its atomic -- DESIGN.md §4 "work heads") and the frame table.
constexpr size_t kHeadsOff = 512;
constexpr int kHeadStride = 32;   // u64 words between two work heads
constexpr size_t kCtrBytes = kHeadsOff + kGroups * 256;
constexpr size_t kCtlBytes = kCtrBytes + kMaxFrames * sizeof(FrameDesc);
struct KParams {
  const GNode* nodes;
  const GNode4* nodes4;
  const GTri* tris;
  const uint32_t* slot2dev; // reference slot -> device record (2-wide canonical kernel)
  const TriShade* shade;
  const double* tnorm;   // [record][12]: face normal, then the 3 vertex normals (device order)
  const double* tu;
  const double* tv;
  const unsigned char* texels;
  const GMat* mats;
  unsigned long long* ctr;
  unsigned long long* heads;  // work head h at heads[h * kHeadStride]
  unsigned long long* wctr;   // per wave {primary, shadow, reflection, 0} rays (plain stores at exit)
  double* pstate;       // path state, [nslots / 64][kFields][64] fp64
  uint32_t* spill;      // [stack_words][nslots] traversal-stack entries below the LDS ring
  unsigned long long* wavelog;  // STATS: per wave {start, last refill, end, pixels} (s_memrealtime)
  unsigned long long* tl;       // TL: per wave and traversal round {start, end, lanes, iterations}
  const double* lights; // [n_lights][6] position xyz, colour rgb
  size_t nslots;
  int n_gnodes;
  int out_fmt;
  int n_top;        // 4-wide nodes cached in LDS (ids [0, n_top))
  int top_off;      // their LDS byte offset
  double root_lo[3], root_hi[3];
  int W, H;
  int n_lights, max_depth;
  double bg[3], amb[3];
  int spp_n;
  int row_begin, stripe_h, stripe_count, stripe_index;
  int rows;
  int tiles_x;
  int pad1;
  long long n_tiles;
  // list mode (adaptive pass): list entries are frame << 25 | local pixel id; work item w = one
  // sample (w % nsamp) of pixel list[w / nsamp] (a pixel's samples run on neighbouring lanes:
  // coherent rays); its trace() colour goes to sample_out[3w..3w+2] (summed in order later).
  const uint32_t* list;
  const unsigned long long* list_count;
  double* sample_out;
  int nsamp;
  int n_prims;              // analytic primitives (0 unless rt_scene_set_analytic)
  const GPrim* prims;
  // frames of this launch (rt_launch_frames): work item w belongs to frame w / (64 * frame_tiles)
  int n_frames;
  int lights_off;           // LDS byte offset of the lights copy ([n_lights][6] doubles)
  int pool_off;             // LDS byte offset of the compaction pool (kPoolBytes)
  long long frame_tiles;
  const FrameDesc* frames;  // [n_frames]
};

// ---- fp64 vector ops (course vec4 semantics on xyz) ----
struct D3 {
  double x, y, z;
};
__device__ __forceinline__ D3 d3(double x, double y, double z) { return D3{x, y, z}; }
__device__ __forceinline__ D3 add(D3 a, D3 b) { return D3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ D3 sub(D3 a, D3 b) { return D3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ D3 scl(double s, D3 a) { return D3{s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ D3 mul(D3 a, D3 b) { return D3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ D3 normalize(D3 v) {
  const double n = sqrt(dot(v, v));
  if (n > 0.0) return D3{v.x / n, v.y / n, v.z / n};
  return v;
}
__device__ __forceinline__ double stdmax(double a, double b) { return (a < b) ? b : a; }
__device__ __forceinline__ double stdmin(double a, double b) { return (b < a) ? b : a; }

// det4D_device (myutils_gpu.h:33-37) / det4D (myutils.cpp:47-51).
__device__ __forceinline__ double det3(D3 v1, D3 v2, D3 v3) {
  return v1.x * (v2.y * v3.z - v3.y * v2.z) - v2.x * (v1.y * v3.z - v3.y * v1.z) +
         v3.x * (v1.y * v2.z - v2.y * v1.z);
}

// Analytic hits in fp64, the oracle's operation order (oracle/rt_oracle.c plane_hit /
// sphere_hit, myplane.cpp:22-49); returns the hit distance or DBL_MAX.
__device__ __forceinline__ double prim_hit(const GPrim& G, D3 o, D3 d) {
  const D3 c = d3(G.c[0], G.c[1], G.c[2]);
  if (G.type == kPrimPlane) {
    const D3 n = d3(G.n[0], G.n[1], G.n[2]);
    const double cos_theta = dot(n, d);
    if (fabs(cos_theta) < 1e-9) return DBL_MAX;
    const double t = (dot(n, c) - dot(n, o)) / cos_theta;
    return t > 1e-5 ? t : DBL_MAX;
  }
  const D3 oc = sub(o, c);
  const double a = dot(d, d);
  const double b = 2.0 * dot(d, oc);
  const double cc = dot(oc, oc) - G.r * G.r;
  const double disc = b * b - 4.0 * a * cc;
  if (disc < 0.0) return DBL_MAX;
  const double sq = sqrt(disc);
  const double t1 = (-b - sq) / (2.0 * a), t2 = (-b + sq) / (2.0 * a);
  double t = DBL_MAX;
  if (t1 > 1e-5 && t1 < t) t = t1;
  if (t2 > 1e-5 && t2 < t) t = t2;
  return t;
}

__device__ __forceinline__ float next_up(float f) {
  if (f != f || f == INFINITY) return f;
  if (f == 0.0f) return __uint_as_float(1u);
  const uint32_t u = __float_as_uint(f);
  return __uint_as_float(f > 0.0f ? u + 1u : u - 1u);
}
__device__ __forceinline__ float next_down(float f) {
  if (f != f || f == -INFINITY) return f;
  if (f == 0.0f) return __uint_as_float(0x80000001u);
  const uint32_t u = __float_as_uint(f);
  return __uint_as_float(f > 0.0f ? u - 1u : u + 1u);
}
__device__ __forceinline__ float round_up_f(double x) {
  float f = (float)x;
  if ((double)f < x) f = next_up(f);
  return f;
}
__device__ __forceinline__ float round_down_f(double x) {
  float f = (float)x;
  if ((double)f > x) f = next_down(f);
  return f;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// Counts one wave-level iteration (and its active lanes) on the first active lane.
__device__ __forceinline__ void wave_tick(unsigned long long& iters, unsigned long long& lanes, int lane) {
  const unsigned long long m = __ballot(1);
  if (lane == __ffsll((long long)m) - 1) { iters++; lanes += __popcll(m); }
}

// Adds the number of distinct keys among the active lanes (wave-uniform loop) on the
// first active lane: distinct lines one load instruction touches, the L1 tag rate's unit.
__device__ __forceinline__ void wave_distinct(uint32_t key, unsigned long long& acc, int lane) {
  unsigned long long m = __ballot(1);
  const int first = __ffsll((long long)m) - 1;
  unsigned n = 0;
  while (m) {
    const uint32_t k = __shfl(key, __ffsll((long long)m) - 1);
    m &= ~__ballot(key == k);
    n++;
  }
  if (lane == first) acc += n;
}

struct TriOps {
  D3 e1, e2, p2;
  int mesh;
  uint32_t meta;
};
__device__ __forceinline__ TriOps load_tri(const GTri* tris, uint32_t i) {
  const double2* q = reinterpret_cast<const double2*>(tris + i);
  const double2 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
  TriOps T;
  T.e1 = d3(a.x, a.y, b.x);
  T.e2 = d3(b.y, c.x, c.y);
  T.p2 = d3(d.x, d.y, e.x);
  const int2 meta = *reinterpret_cast<const int2*>(&q[4].y);
  T.mesh = meta.x;
  T.meta = (uint32_t)meta.y;
  return T;
}

// Path state kept in global memory between a lane's rays, wave-interleaved
// [wave][field][64 lanes] fp64: one field access of a wave is one b64 buffer instruction over
// 512 contiguous bytes.  Only what cannot be recomputed or kept in the LDS slot is kept (the
// normal of the bounce being shaded lives in the slot's aux words, below):
//   the textured diffuse colour (HD; untextured hits re-read the material's kd);
//   the light sum across shadow batches (LACC; a bounce whose lights fit one batch restarts
//     from the recomputed ambient term);
//   the sample's colour and weight across mirror bounces (SCOL, W) and the pixel's sum
//     across samples (PCOL).
// The mirror coefficient comes from the material (the lane keeps the mesh id).  (16-B slots
// with b128 accesses were tried: no faster, and some pixels of mirror chains read stale
// path state under some code layouts -- DESIGN.md §4.)
enum : int {
  F_SCOL = 0, F_W = 3, F_PCOL = 4, F_HD = 7, F_LACC = 10, kFields = 13
};

// LDS slots ([field][thread], conflict-free): the ray (the only hand-over between the
// shading phase, which writes the next ray, and the traversal phase, which reads it) and
// three aux words, time-shared:
//   closest-hit ray in flight: the accepted hit's barycentrics alpha, beta and its mesh id,
//     written by the leaf test when it accepts a hit, so shading reads them instead of
//     re-loading the triangle record and recomputing the determinants (same operands, same
//     operations: bit-identical);
//   shadow batch in flight: the hit normal HN of the bounce being shaded.
constexpr int kSlotDoubles = RT_SLOT_DOUBLES;
struct RaySlots {
  double* o[3];
  double* d[3];
  double* tlim;
  double* a[3];
};

// Per-wave loop, two phases:
//   TRAVERSE: every busy lane loads its ray from LDS, sets up the fp32 box
//             ray and runs ordered traversal until ALL lanes of the wave are
//             done (while-while); only (best, t, shadow flag) survive.
//   SHADE:    lanes whose ray finished run the pixel's state machine from the
//             global path state and write their next ray (if any) to LDS.
// Nothing but a few ids is live across the phase boundary, which keeps the
// kernel at 4 waves/SIMD despite fp64 shading.
__device__ __forceinline__ float f4c(const float4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}
__device__ __forceinline__ uint32_t u4c(const uint4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}

#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 4   // 4 waves/SIMD = 16 waves/CU (register budget 128 VGPRs)
#endif

// RING: entries of the per-lane traversal-stack ring in LDS (8: room for the 73-node treelet;
// 16: deep hierarchies, e.g. millions of random triangles, which spill an 8-entry ring often;
// the treelet then gets what is left, 9 nodes -- rt_scene picks per scene)
template <int WIDTH, bool STATS, bool TL = false, int RING = kShortStack>
__global__ void __launch_bounds__(kBlock, RT_WAVES_PER_EU * 256 / kBlock) render_kernel(KParams P) {
  static_assert(RING >= kMigWords && (RING & (RING - 1)) == 0, "ring: a power of two holding the migration words");
  constexpr int kRingMask = RING - 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  double* lds_d = reinterpret_cast<double*>(lds_raw);
  RaySlots R;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    R.o[k] = lds_d + k * kBlock + threadIdx.x;
    R.d[k] = lds_d + (3 + k) * kBlock + threadIdx.x;
  }
  R.tlim = lds_d + 6 * kBlock + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 3; ++k) R.a[k] = lds_d + (7 + k) * kBlock + threadIdx.x;
  uint32_t* ltask = reinterpret_cast<uint32_t*>(lds_raw + kSlotDoubles * kBlock * sizeof(double));   // [kBlock]
  uint32_t* lvis = ltask + kBlock;                                                             // [kBlock]
  uint32_t* stk = lvis + kBlock + threadIdx.x;
  lvis[threadIdx.x] = 0u;
  // compaction pool: [0] waves of the block still running and not donors, [1..] per wave the
  // lanes it handed over (bits cleared as other waves adopt them)
  uint32_t* pool_live = reinterpret_cast<uint32_t*>(lds_raw + P.pool_off);
  unsigned long long* pool_mask = reinterpret_cast<unsigned long long*>(lds_raw + P.pool_off + 8);
  // heads this block found exhausted (skipped without an atomic)
  uint32_t* pool_exh = reinterpret_cast<uint32_t*>(lds_raw + P.pool_off + 8 + 8 * (kBlock / 64));
  if (threadIdx.x == 0) {
    *pool_live = kBlock / 64;
    for (int w = 0; w < kBlock / 64; ++w) pool_mask[w] = 0ull;
    *pool_exh = 0u;
  }
  // once per persistent block: the top treelet and the lights -> LDS
  if (WIDTH == 4 && P.n_top > 0) {
    float4* dst = reinterpret_cast<float4*>(lds_raw + P.top_off);
    const float4* src = reinterpret_cast<const float4*>(P.nodes4);
    for (int i = threadIdx.x; i < P.n_top * (int)(sizeof(GNode4) / sizeof(float4)); i += kBlock) dst[i] = src[i];
  }
  // lights: staged in LDS when the table fits (RT_MAX_LIGHTS), else read from global memory
  double* lds_lights = reinterpret_cast<double*>(lds_raw + P.lights_off);
  const bool lights_lds = P.n_lights <= RT_MAX_LIGHTS;
  if (lights_lds)
    for (int i = threadIdx.x; i < P.n_lights * 6; i += kBlock) lds_lights[i] = P.lights[i];
  __syncthreads();
  const int wbase = threadIdx.x & ~63;   // first thread of this wave
  uint32_t* spill = P.spill + (size_t)blockIdx.x * kBlock + threadIdx.x;

  const int lane = threadIdx.x & 63;
  const unsigned long long lane_below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  // path state, wave-interleaved [wave][field][64 lanes] (see kFields): buffer ops with the
  // lane offset in one VGPR and the field offset f*512 as an SGPR constant.
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(P.pstate, 0, (int)(P.nslots * kFields * sizeof(double)), kBufWord3);
  // (a lane handed over by tail compaction keeps its pixel's path state: pvo travels with it)
  uint32_t pvo = ((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * (uint32_t)kFields * 64u + (uint32_t)lane) * 8u;
  auto LDF = [&](int f) { return buf_ld(prs, pvo, (uint32_t)f * 512u); };
  auto STF = [&](int f, double v) { buf_st(prs, pvo, (uint32_t)f * 512u, v); };
  auto LDV = [&](int f) { return d3(LDF(f), LDF(f + 1), LDF(f + 2)); };
  auto STV = [&](int f, D3 v) { STF(f, v.x); STF(f + 1, v.y); STF(f + 2, v.z); };
  auto LD_HN = [&]() { return d3(*R.a[0], *R.a[1], *R.a[2]); };
  auto ST_HN = [&](D3 v) { *R.a[0] = v.x; *R.a[1] = v.y; *R.a[2] = v.z; };
  // colour and weight carried across mirror bounces
  auto LD_SCOL_W = [&](D3& scol, double& w) {
    scol = LDV(F_SCOL);
    w = LDF(F_W);
  };
  auto ST_SCOL_W = [&](D3 scol, double w) { STV(F_SCOL, scol); STF(F_W, w); };

  // wave-uniform work-head cursor; in list mode the work count comes from the device
  const long long n_list = P.list ? (long long)*P.list_count * P.nsamp : 0;   // work items
  const long long n_tiles = P.list ? (n_list + 63) / 64 : P.n_tiles;
  int head = blockIdx.x % kGroups;
  int heads_left = kGroups;

  // ---- per-lane state live across phases ----
  int state = ST_FETCH;
  int px = 0, lrow = 0, py = 0, sample = 0, depth = 0, light = 0, mesh = 0, frame = 0;
  long long item = 0;       // list mode: work item (pixel * nsamp + sample), may exceed 2^31
  int best = kNoHit;        // device record of the closest hit
  int best_slot = kNoHit;   // its reference slot (tie-break key)
  double thit = DBL_MAX;
  bool shadow_hit = false;
  int batch_end = 0;      // owner: lights [light, batch_end) in flight
  int refl_h = -1;        // owner: thread tracing its reflection ray this round (-1: none)
  int want = 0;           // owner: extra rays it would lend lanes for
  uint32_t htask = kTaskNone;   // helper: its task word
  unsigned c_primary = 0, c_shadow = 0, c_refl = 0, c_hits = 0;
  unsigned long long c_nodes = 0, c_tris = 0;
  unsigned long long d_node_it = 0, d_node_ln = 0, d_leaf_it = 0, d_leaf_ln = 0;
  unsigned long long d_trav = 0, d_shade = 0, d_fetch = 0, d_outer = 0, d_round_it = 0, d_round_ln = 0;
  unsigned long long d_spills = 0, d_node_lines = 0, d_leaf_lines = 0, d_big_leaf = 0, d_node_lds = 0, d_dummy = 0, d_gn_uni = 0, d_gn_dist = 0, d_leaf_uni = 0;
  unsigned long long w_start = STATS ? __builtin_amdgcn_s_memrealtime() : 0ull, w_refill = 0, w_pixels = 0;
  unsigned long long t_stamp = 0;
  // TL (round timeline, diagnostics): rounds recorded by this wave, the round's start stamp and
  // the lane's wave-level node + leaf iterations in it
  unsigned tl_n = 0;
  unsigned long long tl_t0 = 0;
  unsigned tl_it = 0, tl_leaf = 0, tl_spill = 0, tl_gnode = 0;
  unsigned long long tl_wn = 0, tl_wl = 0, tl_wr = 0, tl_dummy = 0;   // wave-level node / leaf / round iterations
  // time per wave-level iteration by kind (1 global-memory node, 2 LDS-treelet node, 3 leaf): the
  // previous iteration's stamp and kind live in ltask[wave's lanes 63, 62] (unused during TRAVERSE);
  // the first active lane of each iteration charges the time since then to the previous kind
  unsigned long long tl_gsum[4] = {0, 0, 0, 0}, tl_gcnt[4] = {0, 0, 0, 0}, tl_gap = 0;
  auto tl_wave_gap = [&](uint32_t kind) {
    const unsigned long long m = __ballot(1);
    if (lane == __ffsll((long long)m) - 1) {
      const uint32_t now = (uint32_t)__builtin_amdgcn_s_memrealtime();
      const uint32_t prev = ltask[wbase + 63], pk = ltask[wbase + 62];
      ltask[wbase + 63] = now;
      ltask[wbase + 62] = kind;
      const unsigned long long g = now - prev;
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k)
        if (pk == k) { tl_gsum[k] += g; tl_gcnt[k]++; }
      if (g > tl_gap) tl_gap = g;
    }
  };
  auto stamp = [&]() -> unsigned long long { return STATS ? __builtin_amdgcn_s_memtime() : 0ull; };

  // light j: position xyz, colour rgb (the branch is wave-uniform)
  struct Light6 { D3 pos, col; };
  // (two explicitly typed paths: a pointer chosen between LDS and global memory would make every
  // light read a flat load through the vector-memory pipeline)
  typedef __attribute__((address_space(3))) double lds_double;
  typedef __attribute__((address_space(1))) const double glb_double;
  auto light_of = [&](int j) -> Light6 {
    if (lights_lds) {
      const lds_double* L = (const lds_double*)(lds_double*)(lds_lights) + 6 * j;
      return Light6{d3(L[0], L[1], L[2]), d3(L[3], L[4], L[5])};
    }
    const glb_double* L = (const glb_double*)(P.lights) + 6 * (size_t)j;
    return Light6{d3(L[0], L[1], L[2]), d3(L[3], L[4], L[5])};
  };

  // Ray(o, d): stores origin, normalised direction and t-limit to the LDS slot.
  auto emit_ray = [&](D3 o, D3 dir, double t_limit) {
    const D3 d = normalize(dir);
    *R.o[0] = o.x; *R.o[1] = o.y; *R.o[2] = o.z;
    *R.d[0] = d.x; *R.d[1] = d.y; *R.d[2] = d.z;
    *R.tlim = t_limit;
  };

  // primary ray of the current sample (mytracer_gpu.cu:202-209; Camera::primary_ray)
  auto start_sample = [&]() {
    const int n = P.spp_n;
    const int si = sample / n, sj = sample - si * n;
    const double xo = (si) / (double)n - 0.5 + 1.0 / (2.0 * n);
    const double yo = (sj) / (double)n - 0.5 + 1.0 / (2.0 * n);
    const double X = (double)px + xo, Y = (double)py + yo;
    const FrameDesc& K = P.frames[frame];
    const D3 dir = d3(K.ll[0] + X * K.xd[0] + Y * K.yd[0] - K.eye[0],
                      K.ll[1] + X * K.xd[1] + Y * K.yd[1] - K.eye[1],
                      K.ll[2] + X * K.xd[2] + Y * K.yd[2] - K.eye[2]);
    // SCOL = 0 and W = 1 are implicit at depth 0, PCOL = 0 at sample 0 (never stored)
    depth = 0;
    c_primary++;
    emit_ray(d3(K.eye[0], K.eye[1], K.eye[2]), dir, DBL_MAX);
    state = ST_CLOSEST;
  };

  unsigned guard = 0;
  for (;;) {
    if (++guard > kGuardIters) {   // watchdog: end the wave instead of spinning, flag the launch
      if (lane == 0) atomicOr(&P.ctr[CD_GUARD], 1ull);
      break;
    }
    if (STATS) { d_outer++; t_stamp = stamp(); }
    // ---------------- refill idle lanes (one atomic per wave) ----------------
    unsigned long long m_fetch = __ballot(state == ST_FETCH);
    unsigned long long m_busy = __ballot(state == ST_CLOSEST || state == ST_SHADOW || state >= ST_HSHADOW);
    while (m_fetch && (__popcll(m_fetch) >= kRefill || m_busy == 0) && heads_left > 0) {
      const long long g0 = (n_tiles * head / kGroups) * 64;
      const long long g1 = (n_tiles * (head + 1) / kGroups) * 64;
      const int cnt = __popcll(m_fetch);
      const int leader = __ffsll((long long)m_fetch) - 1;
      if ((*pool_exh >> head) & 1u) {   // another wave of the block found it exhausted
        head = (head + 1) % kGroups;
        heads_left--;
        continue;
      }
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(&P.heads[head * kHeadStride], (unsigned long long)cnt);
      base = __shfl(base, leader);
      const long long start = g0 + (long long)base;
      if (start >= g1) {   // head exhausted: move to the next XCD group's range
        if (lane == leader) atomicOr(pool_exh, 1u << head);
        head = (head + 1) % kGroups;
        heads_left--;
        continue;
      }
      if (STATS) { w_refill = __builtin_amdgcn_s_memrealtime(); w_pixels += (unsigned long long)min((long long)cnt, g1 - start); }
      if (state == ST_FETCH) {
        const long long wk = start + __popcll(m_fetch & lane_below);
        if (wk < g1) {
          if (P.list) {   // adaptive pass: one sample of a listed pixel
            const uint32_t id = wk < n_list ? P.list[wk / P.nsamp] : 0xffffffffu;
            const uint32_t pix = id & kListPixMask;
            frame = id != 0xffffffffu ? (int)(id >> kListFrameShift) : 0;
            px = id != 0xffffffffu ? (int)(pix % (uint32_t)P.W) : P.W;
            lrow = id != 0xffffffffu ? (int)(pix / (uint32_t)P.W) : P.rows;
            item = wk;
          } else {
#if RT_BAND_ORDER
            const long long tile = wk >> 6;
            const int j = (int)(wk & 63);
            // several frames: tile row ty of every frame, then row ty + 1, so each XCD head's
            // contiguous range is a band of rows of all frames (its L2 holds one band's nodes)
            const long long row_tiles = (long long)P.n_frames * P.tiles_x;
            const long long ty = tile / row_tiles;
            const long long rem = tile - ty * row_tiles;
            frame = P.n_frames > 1 ? (int)(rem / P.tiles_x) : 0;
            const int tx = (int)(rem - (long long)frame * P.tiles_x);
#else
            long long tile = wk >> 6;
            const int j = (int)(wk & 63);
            frame = P.n_frames > 1 ? (int)(tile / P.frame_tiles) : 0;
            tile -= (long long)frame * P.frame_tiles;
            const long long ty = tile / P.tiles_x;
            const int tx = (int)(tile - ty * P.tiles_x);
#endif
            px = tx * 8 + (j & 7);
            lrow = (int)ty * 8 + (j >> 3);
          }
          if (px < P.W && lrow < P.rows) {
            py = (P.stripe_count == 1)
                     ? P.row_begin + lrow
                     : ((lrow / P.stripe_h) * P.stripe_count + P.stripe_index) * P.stripe_h + (lrow % P.stripe_h);
            sample = P.list ? (int)(item % P.nsamp) : 0;
            start_sample();
          }
        }
      }
      m_fetch = __ballot(state == ST_FETCH);
      m_busy = __ballot(state == ST_CLOSEST || state == ST_SHADOW || state >= ST_HSHADOW);
      if (__popcll(m_fetch) < kRefill && m_busy != 0) break;
    }
    if (heads_left == 0 && state == ST_FETCH) state = ST_DONE;
    const bool busy = (state == ST_CLOSEST || state == ST_SHADOW || state >= ST_HSHADOW);
    if (__ballot(busy) == 0) {
      if (__ballot(state != ST_DONE) != 0) continue;
      // every lane done: leave the block's live set.  The last live wave stays while lanes
      // handed over by donors are still pooled (it adopts them below; no traversal runs).
      bool leave = true;
      if (lane == 0) {
        uint32_t v = *pool_live;
        for (;;) {
          if (v >= 2u) {
            const uint32_t seen = atomicCAS(pool_live, v, v - 1u);
            if (seen == v) break;
            v = seen;
            continue;
          }
          bool pooled = false;
          for (int w = 0; w < kBlock / 64; ++w) pooled |= pool_mask[w] != 0ull;
          if (pooled) leave = false;
          else *pool_live = 0u;
          break;
        }
      }
      if (__shfl(leave ? 1 : 0, 0)) break;
    }

    if (STATS) { const unsigned long long t = stamp(); d_fetch += t - t_stamp; t_stamp = t; }
    if constexpr (TL) {
      tl_t0 = __builtin_amdgcn_s_memrealtime();
      tl_it = tl_leaf = tl_spill = tl_gnode = 0;
      tl_wn = tl_wl = tl_wr = 0;
      tl_gap = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) tl_gsum[k] = tl_gcnt[k] = 0;
      if (lane == 0) { ltask[wbase + 63] = (uint32_t)tl_t0; ltask[wbase + 62] = 0u; }
      wave_lds_sync();
    }
    // ================= TRAVERSE phase =================
    {
      const bool anyhit = (state == ST_SHADOW || state == ST_HSHADOW);
      // helpers read their owner's slot (its closest-hit ray and hit distance)
      const int src = (state >= ST_HSHADOW) ? wbase + (int)(htask & 63u) : (int)threadIdx.x;
      D3 ro = d3(lds_d[0 * kBlock + src], lds_d[1 * kBlock + src], lds_d[2 * kBlock + src]);
      D3 rd = d3(lds_d[3 * kBlock + src], lds_d[4 * kBlock + src], lds_d[5 * kBlock + src]);
      double tlim = lds_d[6 * kBlock + src];
      if (anyhit) {
        // a shadow ray (mytracer.cpp:589-600) for light j of the owner's bounce, derived from the
        // closest-hit ray and hit distance kept in the owner's slot: the same operations, in the
        // same order, as the emission of an explicit ray (emit_ray normalises the direction again)
        const int j = (state == ST_SHADOW) ? light : (int)((htask >> 11) & 0xFFFFFu);
        const D3 hp = add(ro, scl(tlim, rd));
        const D3 to_l = sub(light_of(j).pos, hp);
        const D3 l = normalize(to_l);
        ro = add(hp, scl(1e-4, l));
        rd = normalize(l);
        tlim = sqrt(dot(to_l, to_l));
      } else if (state == ST_HCLOSEST) {
        // the owner's reflection ray (mytracer.cpp:547-552), from its hit and its normal (the
        // owner's aux words); kept in this helper's slot, from which the owner takes it over
        const D3 hp = add(ro, scl(tlim, rd));
        const D3 hn = d3(lds_d[7 * kBlock + src], lds_d[8 * kBlock + src], lds_d[9 * kBlock + src]);
        const double s2 = 2.0 * dot(hn, rd);   // reflect(d, n) = d - 2(n.d)n, d = -view = rd
        const D3 v = sub(rd, scl(s2, hn));
        ro = add(hp, scl(1e-4, v));
        rd = normalize(v);
        tlim = DBL_MAX;
        *R.o[0] = ro.x; *R.o[1] = ro.y; *R.o[2] = ro.z;
        *R.d[0] = rd.x; *R.d[1] = rd.y; *R.d[2] = rd.z;
      }
      best = kNoHit;
      best_slot = kNoHit;
      shadow_hit = false;
      uint32_t cur = kDone;
      double t_off = 0.0;
      // analytic primitives first, in scene order (oracle/rt_oracle.c intersect_scene /
      // shadowed): a hit sets the running best with slot -1, so only a strictly closer
      // triangle replaces it; a shadow ray they block skips the BVH.
      for (int k = 0; k < P.n_prims; ++k) {
        if (!busy) break;
        const double t = prim_hit(P.prims[k], ro, rd);
        if (t < tlim) {
          if (anyhit) { shadow_hit = true; break; }
          tlim = t;
          best = kPrimHit | k;
          best_slot = -1;
        }
      }
      if (busy && P.n_gnodes > 0 && !shadow_hit) {   // conservative fp32 box ray (oracle/rt_oracle.c gray_setup)
        bool miss = false;
        const double o3[3] = {ro.x, ro.y, ro.z}, d3v[3] = {rd.x, rd.y, rd.z};
        bool inside = true;
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (!(o3[k] >= P.root_lo[k] && o3[k] <= P.root_hi[k])) inside = false;
        if (!inside) {
          double tn = -DBL_MAX, tf = DBL_MAX;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            if (d3v[k] == 0.0) {
              if (o3[k] < P.root_lo[k] || o3[k] > P.root_hi[k]) miss = true;
              continue;
            }
            double t0 = (P.root_lo[k] - o3[k]) / d3v[k];
            double t1 = (P.root_hi[k] - o3[k]) / d3v[k];
            if (t0 > t1) { const double t = t0; t0 = t1; t1 = t; }
            if (t0 > tn) tn = t0;
            if (t1 < tf) tf = t1;
          }
          if (tn > tf || tf < 0.0) miss = true;
          t_off = tn > 0.0 ? tn : 0.0;
        }
        if (miss) t_off = 0.0;
        else cur = 0;
      }
      float inv[3];
      {
        const double d3v[3] = {rd.x, rd.y, rd.z};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          float df = (float)d3v[k];
          if (fabsf(df) < 1e-20f) df = signbit(d3v[k]) ? -1e-20f : 1e-20f;
          inv[k] = 1.0f / df;
        }
      }
      const float ofx = (float)(ro.x + t_off * rd.x);
      const float ofy = (float)(ro.y + t_off * rd.y);
      const float ofz = (float)(ro.z + t_off * rd.z);
      const float ivx = inv[0], ivy = inv[1], ivz = inv[2];
      // 4-wide node: per-ray near/far plane byte offsets (lo at +0, hi at +16 of each axis
      // block) and o*inv, so a slab is one FMA: t = plane*inv - o*inv.  Conservative under
      // the delta box growth; only the 2-wide canonical kernel replicates the
      // oracle's sub-then-mul bit for bit.
      const uint32_t nxo = ivx >= 0.f ? 0u : 16u, nyo = ivy >= 0.f ? 32u : 48u, nzo = ivz >= 0.f ? 64u : 80u;
      const float oix = ofx * ivx, oiy = ofy * ivy, oiz = ofz * ivz;
      const float lo_c = round_down_f(-t_off);
      float hi_c = round_up_f(tlim - t_off);
      // logical stack [0, sp); the LDS ring holds [slo, sp), spill[] holds [0, slo)
      int sp = 0, slo = 0;
      auto push = [&](uint32_t x) {
        if (sp - slo == RING) {
          spill[(size_t)slo * P.nslots] = stk[(slo & kRingMask) * kBlock];
          slo++;
          if (STATS) d_spills++;
          if constexpr (TL) tl_spill++;
        }
        stk[(sp & kRingMask) * kBlock] = x;
        sp++;
      };
      auto pop = [&]() -> uint32_t {
        if (sp == 0) return kDone;
        --sp;
        if (sp >= slo) return stk[(sp & kRingMask) * kBlock];
        slo = sp;
        return spill[(size_t)sp * P.nslots];
      };
      const D3 c3 = d3(-rd.x, -rd.y, -rd.z);

      // Watchdog of the traversal loops that could cycle on a corrupt hierarchy (the round loop
      // and the node loops): each counts its own wave-level iterations in a counter that lives
      // only inside that loop, so it stays wave-uniform (an SGPR: the check costs SALU only).
      // A loop that runs past kTravGuard iterations abandons the ray (results void) and flags
      // the launch.  (Cost: 0.3 % for the node loop, A/B.)
      auto guard_trip = [&]() {
        if (lane == __ffsll((long long)__ballot(1)) - 1) atomicOr(&P.ctr[CD_GUARD], 1ull);
      };
      // tests the triangles of leaf `lref` in record order; true = any-hit ray occluded
      auto test_leaf = [&](uint32_t lref) -> bool {
          // 2-wide: iterate reference slots in order (the oracle's order); 4-wide: device
          // records of the (possibly refined) leaf.  Either way the hit kept is the
          // smallest (t, slot), which does not depend on the order.
          uint32_t i = lref & ~kLeaf;
          const uint32_t leaf0 = i;
          bool occluded = false;
          // a linear scan to the record flagged last of its leaf: it cannot cycle (a corrupt flag
          // would run into the end of the record buffer, a fault, not a hang), so it has no watchdog
          for (;;) {
            const uint32_t rec = (WIDTH == 2) ? P.slot2dev[i] : i;
            if constexpr (TL) {
              tl_it++; tl_leaf++; wave_tick(tl_wl, tl_dummy, lane);
              tl_wave_gap(3);
            }
            if (STATS) {
              c_tris++;
              wave_tick(d_leaf_it, d_leaf_ln, lane);
              wave_distinct((uint32_t)(((unsigned long long)i * sizeof(GTri)) >> 7), d_leaf_lines, lane);
              const uint32_t i0 = __shfl(i, __ffsll((long long)__ballot(1)) - 1);
              if (__ballot(i != i0) == 0) wave_tick(d_leaf_uni, d_dummy, lane);
            }
            const TriOps T = load_tri(P.tris, rec);
            const int slot = (int)(T.meta & kSlotMask);
            // Mesh::intersect_triangle (mymesh.cpp:190-215): the same fp64 S, Da, Db, Dt as
            // the CPU (bit-identical operands and operation order).  Division-free early
            // rejections first: they fire only where the CPU's rounded quotients certainly
            // fail the same test (margins in DESIGN.md §4), so accept decisions are unchanged.
            const D3 c4 = sub(ro, T.p2);
            const double S = det3(T.e1, T.e2, c3);
            if (fabs(S) >= 1e-10) {
              const double Da = det3(c4, T.e2, c3);
              const double Db = det3(T.e1, c4, c3);
              const double sS = S > 0.0 ? 1.0 : -1.0;
              const double aS = fabs(S);
              const double ua = Da * sS, ub = Db * sS;                       // sign-normalised numerators
              const double tiny = aS * 0x1p-1000, big = aS * (1.0 + 0x1p-48);
              const bool out = (ua < 0.0 && -ua >= tiny) || (ub < 0.0 && -ub >= tiny) || ua > big || ub > big ||
                               (Da + Db - S) * sS > 0x1p-40 * (fabs(Da) + fabs(Db) + aS);
              if (!out) {
                const double t = det3(T.e1, T.e2, c4) / S;
                const bool cand = anyhit ? (t < tlim) : (t <= tlim);
                if (t > 1e-5 && cand) {
                  const double alpha = Da / S;
                  const double beta = Db / S;
                  const double gamma = (1.0 - alpha - beta);
                  const bool inside = (0.0 <= alpha && alpha <= 1.0) && (0.0 <= beta && beta <= 1.0) &&
                                      (0.0 <= gamma && gamma <= 1.0);
                  if (inside) {
                    if (anyhit) {
                      shadow_hit = true;
                      occluded = true;
                      break;
                    }
                    if (t < tlim || slot < best_slot) {   // ties: smallest slot (mybvh.cpp:169 visit order)
                      tlim = t;
                      best = (int)rec;
                      best_slot = slot;
                      hi_c = round_up_f(tlim - t_off);
                      // hit attributes for shading (slot aux words: free while a closest-hit ray is in flight)
                      *R.a[0] = alpha;
                      *R.a[1] = beta;
                      *R.a[2] = __longlong_as_double((long long)T.mesh);
                    }
                  }
                }
              }
            }
            if (T.meta & (WIDTH == 2 ? kLastRef : kLastDev)) break;
            ++i;
          }
          if (STATS && i - leaf0 + 1 > 4) d_big_leaf += i - leaf0 + 1;
          return occluded;
      };
      uint32_t pleaf = kDone;   // 4-wide: postponed leaf

      uint32_t rounds = 0;
      while (__ballot(cur != kDone || pleaf != kDone) != 0) {
        if (++rounds > kTravGuard) {   // watchdog: abandon the round (results void, launch flagged)
          guard_trip();
          cur = kDone;
          pleaf = kDone;
          break;
        }
        if (STATS) wave_tick(d_round_it, d_round_ln, lane);
        if constexpr (TL) wave_tick(tl_wr, tl_dummy, lane);
        if constexpr (WIDTH == 2) {
        for (uint32_t it = 0; !(cur & kLeaf); ++it) {   // internal node (kDone carries the leaf bit)
          if (it > kTravGuard) { guard_trip(); cur = kDone; break; }
          if (STATS) { c_nodes++; wave_tick(d_node_it, d_node_ln, lane); wave_distinct(cur, d_node_lines, lane); }
          const float4* nq = reinterpret_cast<const float4*>(P.nodes + cur);
          const float4 bx = nq[0], by = nq[1], bz = nq[2];
          const uint2 rf = *reinterpret_cast<const uint2*>(nq + 3);
          const float ax0 = (bx.x - ofx) * ivx, ax1 = (bx.y - ofx) * ivx;
          const float ay0 = (by.x - ofy) * ivy, ay1 = (by.y - ofy) * ivy;
          const float az0 = (bz.x - ofz) * ivz, az1 = (bz.y - ofz) * ivz;
          const float bx0 = (bx.z - ofx) * ivx, bx1 = (bx.w - ofx) * ivx;
          const float by0 = (by.z - ofy) * ivy, by1 = (by.w - ofy) * ivy;
          const float bz0 = (bz.z - ofz) * ivz, bz1 = (bz.w - ofz) * ivz;
          const float tn0 = fmaxf(fmaxf(fminf(ax0, ax1), fminf(ay0, ay1)), fmaxf(fminf(az0, az1), lo_c));
          const float tf0 = fminf(fminf(fmaxf(ax0, ax1), fmaxf(ay0, ay1)), fminf(fmaxf(az0, az1), hi_c));
          const float tn1 = fmaxf(fmaxf(fminf(bx0, bx1), fminf(by0, by1)), fmaxf(fminf(bz0, bz1), lo_c));
          const float tf1 = fminf(fminf(fmaxf(bx0, bx1), fmaxf(by0, by1)), fminf(fmaxf(bz0, bz1), hi_c));
          const bool h0 = tn0 <= tf0;
          const bool h1 = (tn1 <= tf1) && (rf.y != kEmpty);
          if (h0 && h1) {
            const bool swap = tn1 < tn0;
            push(swap ? rf.x : rf.y);
            cur = swap ? rf.y : rf.x;
          } else if (h0) {
            cur = rf.x;
          } else if (h1) {
            cur = rf.y;
          } else {
            cur = pop();
          }
        }
        } else {
        for (uint32_t it = 0; !(cur & kLeaf); ++it) {   // 4-wide node: test 4 boxes, visit nearest, push the rest far-first
          if (it > kTravGuard) { guard_trip(); cur = kDone; pleaf = kDone; break; }
          if constexpr (TL) {
            tl_it++; wave_tick(tl_wn, tl_dummy, lane);
          }
          if (STATS) { c_nodes++; wave_tick(d_node_it, d_node_ln, lane); wave_distinct(cur, d_node_lines, lane); }
          float k[4];
          uint32_t v[4];
          int cnt = 0;
          float4 nx, fx, ny, fy, nz, fz;
          uint4 rf;
          // wave-uniform: every active lane's node is in the LDS treelet -> ds_read, no TD cost
          if (__ballot(cur >= (uint32_t)P.n_top) == 0) {
            if (STATS) wave_tick(d_node_lds, d_dummy, lane);
            if constexpr (TL) tl_wave_gap(2);
            const unsigned char* lb = lds_raw + P.top_off + cur * (uint32_t)sizeof(GNode4);
            nx = *reinterpret_cast<const float4*>(lb + nxo);
            fx = *reinterpret_cast<const float4*>(lb + (nxo ^ 16u));
            ny = *reinterpret_cast<const float4*>(lb + nyo);
            fy = *reinterpret_cast<const float4*>(lb + (nyo ^ 16u));
            nz = *reinterpret_cast<const float4*>(lb + nzo);
            fz = *reinterpret_cast<const float4*>(lb + (nzo ^ 16u));
            rf = *reinterpret_cast<const uint4*>(lb + 96);
          } else {
            const char* nb = reinterpret_cast<const char*>(P.nodes4) + (size_t)cur * sizeof(GNode4);
            if constexpr (TL) { tl_gnode++; tl_wave_gap(1); }
            if (STATS) {
              wave_distinct(cur, d_gn_dist, lane);
              const uint32_t c0 = __shfl(cur, __ffsll((long long)__ballot(1)) - 1);
              if (__ballot(cur != c0) == 0) wave_tick(d_gn_uni, d_dummy, lane);
            }
            nx = *reinterpret_cast<const float4*>(nb + nxo);
            fx = *reinterpret_cast<const float4*>(nb + (nxo ^ 16u));
            ny = *reinterpret_cast<const float4*>(nb + nyo);
            fy = *reinterpret_cast<const float4*>(nb + (nyo ^ 16u));
            nz = *reinterpret_cast<const float4*>(nb + nzo);
            fz = *reinterpret_cast<const float4*>(nb + (nzo ^ 16u));
            rf = *reinterpret_cast<const uint4*>(nb + 96);
          }
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float tx0 = __builtin_fmaf(f4c(nx, c), ivx, -oix), tx1 = __builtin_fmaf(f4c(fx, c), ivx, -oix);
            const float ty0 = __builtin_fmaf(f4c(ny, c), ivy, -oiy), ty1 = __builtin_fmaf(f4c(fy, c), ivy, -oiy);
            const float tz0 = __builtin_fmaf(f4c(nz, c), ivz, -oiz), tz1 = __builtin_fmaf(f4c(fz, c), ivz, -oiz);
            const float tn = fmaxf(fmaxf(tx0, ty0), fmaxf(tz0, lo_c));
            const float tf = fminf(fminf(tx1, ty1), fminf(tz1, hi_c));
            const uint32_t r = u4c(rf, c);
            const bool h = tn <= tf;   // absent children carry the empty box [+inf, -inf]
            k[c] = h ? tn : INFINITY;
            v[c] = r;
            cnt += h ? 1 : 0;
          }
#define RT_CSWAP(a, b)                                        \
  if (k[b] < k[a]) {                                          \
    const float tk = k[a]; k[a] = k[b]; k[b] = tk;            \
    const uint32_t tv = v[a]; v[a] = v[b]; v[b] = tv;         \
  }
          RT_CSWAP(0, 1) RT_CSWAP(2, 3) RT_CSWAP(0, 2) RT_CSWAP(1, 3) RT_CSWAP(1, 2)
#undef RT_CSWAP
          if (cnt == 0) {
            cur = pop();
          } else {
            if (cnt > 3) push(v[3]);
            if (cnt > 2) push(v[2]);
            if (cnt > 1) push(v[1]);
            cur = v[0];
          }
          if ((cur & kLeaf) && cur != kDone && pleaf == kDone) {   // first leaf: postpone, keep going
            pleaf = cur;
            cur = pop();
          }
          if (__ballot(pleaf == kDone && cur != kDone) == 0) break;   // every lane holds a leaf
        }
        }
        // leaves: 2-wide -- the leaf the lane stopped at; 4-wide -- the postponed leaf, then
        // any leaf the lane stopped at after it (chained), so lanes that found leaves early
        // kept traversing instead of idling (speculative while-while, Aila & Laine 2009)
        if constexpr (WIDTH == 2) {
          if (cur != kDone) {
            if (test_leaf(cur)) cur = kDone;
            else cur = pop();
          }
        } else {
          if (pleaf == kDone && cur != kDone) {   // stopped at a leaf without postponing one
            pleaf = cur;
            cur = pop();
          }
          while (pleaf != kDone) {
            if (test_leaf(pleaf)) {   // any-hit: occluded, the ray is finished
              cur = kDone;
              pleaf = kDone;
              break;
            }
            pleaf = kDone;
            if ((cur & kLeaf) && cur != kDone) {
              pleaf = cur;
              cur = pop();
            }
          }
        }
      }
      thit = tlim;
    }
    asm volatile("" ::: "memory");
    if (STATS) { const unsigned long long t = stamp(); d_trav += t - t_stamp; t_stamp = t; }
    if constexpr (TL) {   // kTlWords words per round (rt_debug_timeline)
      tl_wave_gap(0);   // charges the last iteration
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
      unsigned m = tl_it;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
      const unsigned long long w_r = wave_sum(tl_wr);
      unsigned long long gs[4], gc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) { gs[k] = wave_sum(tl_gsum[k]); gc[k] = wave_sum(tl_gcnt[k]); }
      unsigned long long gmax = tl_gap;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long x = __shfl_xor(gmax, o);
        gmax = x > gmax ? x : gmax;
      }
      const unsigned nb = (unsigned)__popcll(__ballot(busy));
      const unsigned no = (unsigned)__popcll(__ballot(state == ST_CLOSEST || state == ST_SHADOW));
      const unsigned nsh = (unsigned)__popcll(__ballot(busy && (state == ST_SHADOW || state == ST_HSHADOW)));
      if (lane == 0 && tl_n < (unsigned)kTlCap) {
        unsigned long long* r =
            P.tl + kTlWords * ((size_t)(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * kTlCap + tl_n);
        r[0] = tl_t0;
        r[1] = t1;
        r[2] = nb | (no << 8) | ((heads_left > 0 ? 1u : 0u) << 16) | ((unsigned long long)nsh << 24);
        r[3] = m | (w_r << 32);
        r[4] = gs[1] | (gc[1] << 40);
        r[5] = gs[2] | (gc[2] << 40);
        r[6] = gs[3] | (gc[3] << 40);
        r[7] = gmax | (gs[0] << 32);   // longest iteration; round setup (before the first iteration)
      }
      tl_n++;
    }

    // ---- helpers hand their result to the owner, then go idle ----
    // (a reflection helper's LDS ray slot still holds the ray its owner reads in SHADE below:
    // that lane must not adopt a handed-over pixel this iteration)
    bool refl_held = false;
    {
      const int idle_state = heads_left > 0 ? ST_FETCH : ST_DONE;
      if (state == ST_HSHADOW) {
        if (shadow_hit) atomicOr(&lvis[wbase + (int)(htask & 63u)], 1u << ((htask >> 6) & 31u));   // bit: light - batch start
        state = idle_state;
      } else if (state == ST_HCLOSEST) {
        ltask[threadIdx.x] = (uint32_t)best;
        *R.tlim = thit;
        state = idle_state;
        refl_held = true;
      }
      wave_lds_sync();
    }

    // ---- tail compaction: donate (sparse wave, queue empty) or adopt pooled lanes ----
    if (heads_left == 0) {
      const int wib = threadIdx.x >> 6;   // wave in block
      const bool owner = (state == ST_CLOSEST || state == ST_SHADOW);
      const unsigned long long O = __ballot(owner);
      if (O != 0ull && __popcll(O) <= kDonateMax && *pool_live >= 2u) {
        // registers -> this thread's LDS stack entries, then publish the lane mask
        if (owner) {
          // packed: state (3 bits) | shadow hit | frame (< 128) | sample (< 4096) | refl_h + 1 (9 bits);
          // item; depth; light; batch size | item >> 32 << 6; best (closest-hit ray) or mesh (shadow
          // batch); path-state offset; px | lrow << 16.  py is recomputed from lrow; a closest-hit
          // ray's distance goes to its slot's t-limit word (the slot is copied to the adopter)
          const unsigned long long it = (unsigned long long)item;
          const uint32_t w[kMigWords] = {
              (uint32_t)state | (shadow_hit ? 8u : 0u) | ((uint32_t)frame << 4) | ((uint32_t)sample << 11) |
                  ((uint32_t)(refl_h + 1) << 23),
              (uint32_t)it, (uint32_t)depth, (uint32_t)light,
              ((uint32_t)(batch_end - light) & 63u) | ((uint32_t)(it >> 32) << 6),
              (uint32_t)(state == ST_CLOSEST ? best : mesh), pvo, (uint32_t)px | ((uint32_t)lrow << 16)};
#pragma unroll
          for (int k = 0; k < kMigWords; ++k) stk[k * kBlock] = w[k];
          if (state == ST_CLOSEST) *R.tlim = thit;
        }
        wave_lds_sync();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's path-state stores have landed
        bool donated = false;
        if (lane == 0) {
          atomicOr(&pool_mask[wib], O);
          uint32_t v = *pool_live;   // leave the live set only if another live wave remains
          while (v >= 2u) {
            const uint32_t seen = atomicCAS(pool_live, v, v - 1u);
            if (seen == v) { donated = true; break; }
            v = seen;
          }
        }
        if (__shfl(donated ? 1 : 0, 0)) break;   // exit: the counters below keep this thread's sums
        // no other live wave: take back what nobody adopted and carry on
        unsigned long long back = 0ull;
        if (lane == 0) back = atomicAnd(&pool_mask[wib], 0ull);
        back = __shfl(back, 0);
        if (owner && !((back >> lane) & 1ull)) state = ST_DONE;   // adopted by another wave
      } else {
        // adopt pooled lanes of other waves into idle lanes
        unsigned long long I = __ballot((state == ST_FETCH || state == ST_DONE) && !refl_held);
        for (int w = 0; w < kBlock / 64 && I != 0ull; ++w) {
          if (w == wib || pool_mask[w] == 0ull) continue;
          unsigned long long got = 0ull;
          if (lane == 0) {
            unsigned long long m = pool_mask[w], pick = 0ull;
            for (int k = __popcll(I); k > 0 && m != 0ull; --k) {
              const unsigned long long b = m & (~m + 1ull);
              pick |= b;
              m &= ~b;
            }
            got = pick & atomicAnd(&pool_mask[w], ~pick);
          }
          got = __shfl(got, 0);
          const int n = __popcll(got);
          if (n == 0) continue;
          // the r-th idle lane takes the r-th adopted lane of donor wave w
          const bool idle = (I >> lane) & 1ull;
          const int r = __popcll(I & lane_below);
          const bool take = idle && r < n;
          if (take) {
            const int t = w * 64 + kth_set_bit(got, r);   // donor thread
            const uint32_t* ds = lvis + kBlock + t;        // its stack entries
            uint32_t v_[kMigWords];
#pragma unroll
            for (int k = 0; k < kMigWords; ++k) v_[k] = ds[k * kBlock];
            state = (int)(v_[0] & 7u);
            shadow_hit = (v_[0] & 8u) != 0u;
            frame = (int)((v_[0] >> 4) & 127u);
            sample = (int)((v_[0] >> 11) & 4095u);
            refl_h = (int)(v_[0] >> 23) - 1;
            item = (long long)(((unsigned long long)(v_[4] >> 6) << 32) | v_[1]);
            depth = (int)v_[2];
            light = (int)v_[3];
            batch_end = light + (int)(v_[4] & 63u);
            if (state == ST_CLOSEST) best = (int)v_[5];
            else mesh = (int)v_[5];
            pvo = v_[6];
            px = (int)(v_[7] & 0xffffu);
            lrow = (int)(v_[7] >> 16);
            py = (P.stripe_count == 1)
                     ? P.row_begin + lrow
                     : ((lrow / P.stripe_h) * P.stripe_count + P.stripe_index) * P.stripe_h + (lrow % P.stripe_h);
            lvis[threadIdx.x] = lvis[t];
#pragma unroll
            for (int k = 0; k < kSlotDoubles; ++k) lds_d[k * kBlock + threadIdx.x] = lds_d[k * kBlock + t];
            thit = *R.tlim;   // a closest-hit ray's distance (a shadow batch's owner does not read thit)
          }
          I &= ~__ballot(take);
        }
      }
      wave_lds_sync();
    }

    // ================= SHADE phase (owners) =================
    want = 0;
    if (state == ST_CLOSEST || state == ST_SHADOW) {
      D3 hp = d3(0, 0, 0), hn = d3(0, 0, 0), hview = d3(0, 0, 0);   // the hit being shaded
      bool hit_ready = (state == ST_CLOSEST), finish = false;
      D3 scol = d3(0, 0, 0);   // the sample's colour so far once the path ends (finish)
      double mirror = 0.0;
      // lighting() for one light (mytracer.cpp:579-606): Lambert + Phong term of light j
      auto contrib_of = [&](int j, D3 hp_, D3 hn_, D3 hv_, D3 hd_, const GMat& M) {
        const Light6 L6 = light_of(j);
        const D3 l = normalize(sub(L6.pos, hp_));
        const double diff = stdmax(0.0, dot(hn_, l));
        double refl = 0.0;
        if (diff > 0.0) {   // reflection(), mytracer.cpp:524-534
          const double s2 = 2.0 * dot(hn_, l);
          const D3 r = normalize(sub(scl(s2, hn_), l));
          refl = stdmax(0.0, dot(r, hv_));
        }
        // pow(+0, y > 0) = +0 exactly: skip the fp64 pow for the (frequent) zero highlight
        if (!(refl == 0.0 && M.shininess > 0.0)) refl = pow(refl, M.shininess);
        return d3(L6.col.x * (hd_.x * diff + M.ks[0] * refl), L6.col.y * (hd_.y * diff + M.ks[1] * refl),
                  L6.col.z * (hd_.z * diff + M.ks[2] * refl));
      };
      // own shadow ray for light `light`; the rest of the bounce is offered to idle lanes
      // (the ray itself is derived at the start of the next traversal from the slot's closest-hit
      // ray and distance)
      auto launch_batch = [&](double mirror_) {
        c_shadow++;
        state = ST_SHADOW;
        lvis[threadIdx.x] = 0u;
        batch_end = light + 1;
        refl_h = -1;
        // extra lights of this batch, then the reflection ray once the batch covers every light
        const int rest = P.n_lights - light - 1;
        want = min(rest, kBatchExtra) + ((rest <= kBatchExtra && mirror_ > 0.0 && depth < P.max_depth) ? 1 : 0);
      };
      if (state == ST_SHADOW) {   // batch finished: lights [light, batch_end) in order
        {   // the hit again, from the closest-hit ray and distance kept in the slot
          const D3 ro = d3(*R.o[0], *R.o[1], *R.o[2]);
          const D3 rd = d3(*R.d[0], *R.d[1], *R.d[2]);
          hp = add(ro, scl(*R.tlim, rd));
          hview = d3(-rd.x, -rd.y, -rd.z);
        }
        hn = LD_HN();
        const GMat& M = P.mats[mesh];
        const D3 hdiff = M.tex_w > 0 ? LDV(F_HD) : d3(M.kd[0], M.kd[1], M.kd[2]);
        mirror = M.mirror;
        // first batch: the ambient term (mytracer.cpp:574-576) again, else the stored sum
        D3 lacc = light == 0 ? d3(0.0 + P.amb[0] * M.ka[0], 0.0 + P.amb[1] * M.ka[1], 0.0 + P.amb[2] * M.ka[2])
                             : LDV(F_LACC);
        const uint32_t vw = lvis[threadIdx.x];
        for (int j = light; j < batch_end; ++j) {
          const bool occluded = (j == light) ? shadow_hit : (((vw >> (j - light)) & 1u) != 0u);
          // an occluded light adds colour * 0 * (finite term) = +-0, which leaves the sum (never -0)
          // unchanged: skip it (the term is finite for any material with finite shininess >= 0)
          if (!occluded) lacc = add(lacc, contrib_of(j, hp, hn, hview, hdiff, M));
        }
        light = batch_end;
        if (light < P.n_lights) {
          STV(F_LACC, lacc);
          launch_batch(mirror);
        } else {   // bounce complete (subtrace, mytracer.cpp:546-555)
          D3 s0 = d3(0, 0, 0);
          double w = 1.0;
          if (depth > 0) LD_SCOL_W(s0, w);
          scol = add(s0, scl(w, scl(1.0 - mirror, lacc)));
          if (mirror > 0.0 && depth < P.max_depth) {
            ST_SCOL_W(scol, w * mirror);
            depth++;
            if (refl_h >= 0) {   // reflection ray traced by a helper this round
              const int ht = refl_h;
#pragma unroll
              for (int k = 0; k < 3; ++k) {
                *R.o[k] = lds_d[k * kBlock + ht];
                *R.d[k] = lds_d[(3 + k) * kBlock + ht];
              }
              best = (int)ltask[ht];
              thit = lds_d[6 * kBlock + ht];
#pragma unroll
              for (int k = 0; k < 3; ++k) *R.a[k] = lds_d[(7 + k) * kBlock + ht];   // its hit attributes
              hit_ready = true;
            } else {
              const D3 d = d3(-hview.x, -hview.y, -hview.z);   // reflect(d, n) = d - 2(n.d)n
              const double s2 = 2.0 * dot(hn, d);
              const D3 v = sub(d, scl(s2, hn));
              c_refl++;
              emit_ray(add(hp, scl(1e-4, v)), v, DBL_MAX);
              state = ST_CLOSEST;
            }
          } else {
            finish = true;
          }
        }
      }
      if (hit_ready) {
        if (best == kNoHit) {   // miss: background (mytracer_gpu.cu:262, :292)
          D3 s0 = d3(0, 0, 0);
          double w = 1.0;
          if (depth > 0) LD_SCOL_W(s0, w);
          scol = add(s0, scl(w, d3(P.bg[0], P.bg[1], P.bg[2])));
          finish = true;
        } else {
          if (STATS) c_hits++;
          // hit attributes: mymesh.cpp:217-235 (texture :70-95)
          const D3 ro = d3(*R.o[0], *R.o[1], *R.o[2]);
          const D3 rd = d3(*R.d[0], *R.d[1], *R.d[2]);
          const D3 c3 = d3(-rd.x, -rd.y, -rd.z);
          hp = add(ro, scl(thit, rd));
          hview = c3;
          D3 hdiff;
          if (best & kPrimHit) {   // analytic hit (oracle/rt_oracle.c intersect_scene): no texture
            const GPrim& G = P.prims[best & (kPrimHit - 1)];
            hn = G.type == kPrimPlane ? d3(G.n[0], G.n[1], G.n[2])
                                      : d3((ro.x + thit * rd.x - G.c[0]) / G.r, (ro.y + thit * rd.y - G.c[1]) / G.r,
                                           (ro.z + thit * rd.z - G.c[2]) / G.r);
            mesh = G.mat;
            const GMat& Mp = P.mats[mesh];
            hdiff = d3(Mp.kd[0], Mp.kd[1], Mp.kd[2]);
          } else {
            // barycentrics and mesh from the leaf test that accepted the hit (slot aux words: the
            // CPU's Da / S and Db / S of mymesh.cpp:205-215 on the same operands); the normal
            // record is indexed by the hit record
            const double alpha = *R.a[0], beta = *R.a[1];
            const double gamma = (1.0 - alpha - beta);
            mesh = (int)__double_as_longlong(*R.a[2]);
            const GMat& Mt = P.mats[mesh];
            const double* nr = P.tnorm + 12 * (size_t)best;
            if (Mt.draw_mode == RT_DRAW_FLAT) {   // normals_[i] (mytracer_gpu.cu:498-500)
              const double2 q0 = *reinterpret_cast<const double2*>(nr);
              hn = d3(q0.x, q0.y, nr[2]);
            } else {   // alpha*vn0 + beta*vn1 + gamma*vn2, not renormalised (:501-505)
              const double2* nq = reinterpret_cast<const double2*>(nr + 2);   // [2, 12): _, vn0, vn1, vn2
              const double2 q1 = nq[0], q2 = nq[1], q3 = nq[2], q4 = nq[3], q5 = nq[4];
              const double n0[3] = {q1.y, q2.x, q2.y}, n1[3] = {q3.x, q3.y, q4.x}, n2[3] = {q4.y, q5.x, q5.y};
              hn = d3(alpha * n0[0] + beta * n1[0] + gamma * n2[0], alpha * n0[1] + beta * n1[1] + gamma * n2[1],
                      alpha * n0[2] + beta * n1[2] + gamma * n2[2]);
            }
            if (Mt.tex_w > 0) {
              const TriShade sh = P.shade[best];
              double u = alpha * P.tu[sh.t[0]] + beta * P.tu[sh.t[1]] + gamma * P.tu[sh.t[2]];
              double v = alpha * P.tv[sh.t[0]] + beta * P.tv[sh.t[1]] + gamma * P.tv[sh.t[2]];
              u = fmin(fmax(u, 0.0), 1.0);   // NaN -> 0, as mytracer_gpu.cu:532-533
              v = fmin(fmax(v, 0.0), 1.0);
              const unsigned TW = (unsigned)Mt.tex_w, TH = (unsigned)Mt.tex_h;
              const int tx = (int)round(u * (TW - 1));
              const int ty = (int)round((1.0 - v) * (TH - 1));
              const unsigned char* t3 = P.texels + 3 * (Mt.tex_off + (long long)ty * TW + tx);
              hdiff = d3((double)t3[0] / 255.0, (double)t3[1] / 255.0, (double)t3[2] / 255.0);
            } else {
              hdiff = d3(Mt.kd[0], Mt.kd[1], Mt.kd[2]);
            }
          }
          const GMat& M = P.mats[mesh];
          mirror = M.mirror;
          // ambient term (mytracer.cpp:574-576)
          D3 lacc = d3(0.0 + P.amb[0] * M.ka[0], 0.0 + P.amb[1] * M.ka[1], 0.0 + P.amb[2] * M.ka[2]);
          light = 0;
          if (M.shadowable && P.n_lights > 0) {   // shadow rays, mytracer.cpp:589-600
            ST_HN(hn);
            *R.tlim = thit;   // the slot keeps the closest-hit ray and its distance
            if (M.tex_w > 0) STV(F_HD, hdiff);
            launch_batch(mirror);
          } else {
            for (int j = 0; j < P.n_lights; ++j) lacc = add(lacc, contrib_of(j, hp, hn, hview, hdiff, M));
            D3 s0 = d3(0, 0, 0);
            double w = 1.0;
            if (depth > 0) LD_SCOL_W(s0, w);
            scol = add(s0, scl(w, scl(1.0 - mirror, lacc)));
            if (mirror > 0.0 && depth < P.max_depth) {
              ST_SCOL_W(scol, w * mirror);
              depth++;
              const D3 d = d3(-hview.x, -hview.y, -hview.z);
              const double s2 = 2.0 * dot(hn, d);
              const D3 v = sub(d, scl(s2, hn));
              c_refl++;
              emit_ray(add(hp, scl(1e-4, v)), v, DBL_MAX);
              state = ST_CLOSEST;
            } else {
              finish = true;
            }
          }
        }
      }
      if (finish && P.list) {   // adaptive pass: this sample's trace() colour
        const D3 c = scol;
        double* so = P.sample_out + 3 * (size_t)item;
        so[0] = c.x; so[1] = c.y; so[2] = c.z;
        state = heads_left > 0 ? ST_FETCH : ST_DONE;
      } else if (finish) {
        const D3 pcol = add(sample == 0 ? d3(0, 0, 0) : LDV(F_PCOL), scol);
        sample++;
        if (sample < P.spp_n * P.spp_n) {
          STV(F_PCOL, pcol);
          start_sample();
        } else {   // compute_image: average, clamp, store (mytracer_gpu.cu:155-159, 221-227)
          const double nn = (double)(P.spp_n * P.spp_n);
          const double r = stdmin(pcol.x / nn, 1.0), g = stdmin(pcol.y / nn, 1.0), b = stdmin(pcol.z / nn, 1.0);
          const size_t o = 3 * ((size_t)lrow * P.W + px);
          if (P.out_fmt == RT_OUT_RGB_F64) {
            double* out = reinterpret_cast<double*>(P.frames[frame].out) + o;
            out[0] = r; out[1] = g; out[2] = b;
          } else {
            float* out = reinterpret_cast<float*>(P.frames[frame].out) + o;
            out[0] = (float)r; out[1] = (float)g; out[2] = (float)b;
          }
          state = heads_left > 0 ? ST_FETCH : ST_DONE;
        }
      }
    }
    asm volatile("" ::: "memory");

    // ---- lend idle lanes to owners' extra rays (extra lights in order, then reflection) ----
    {
      const bool idle = (state == ST_FETCH || state == ST_DONE);
      const unsigned long long I = __ballot(idle);
      if (I != 0ull && __ballot(want > 0) != 0ull) {
        if (idle) ltask[threadIdx.x] = kTaskNone;
        int incl = want;   // inclusive prefix sum of want over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int v = __shfl_up(incl, o);
          if (lane >= o) incl += v;
        }
        wave_lds_sync();
        const int off = incl - want;
        const int avail = (int)__popcll(I);   // __popcll is unsigned: keep the subtraction signed
        const int got = min(want, max(0, avail - off));
        if (got > 0) {
          const int n_extra_lights = min(P.n_lights - light - 1, kBatchExtra);
          for (int t = 0; t < got; ++t) {   // task words only: each helper derives its own ray
            const int ht = wbase + kth_set_bit(I, off + t);
            uint32_t tw;
            if (t < n_extra_lights) {
              tw = (uint32_t)lane | ((uint32_t)(t + 1) << 6) | ((uint32_t)(light + 1 + t) << 11);
              c_shadow++;
            } else {   // reflection ray
              tw = (uint32_t)lane | kTaskRefl;
              c_refl++;
              refl_h = ht;
            }
            ltask[ht] = tw;
          }
          batch_end = light + 1 + min(got, n_extra_lights);
        }
        wave_lds_sync();
        if (idle) {
          htask = ltask[threadIdx.x];
          if (htask != kTaskNone) state = (htask & kTaskRefl) ? ST_HCLOSEST : ST_HSHADOW;
        }
      }
    }
    if (STATS) { const unsigned long long t = stamp(); d_shade += t - t_stamp; t_stamp = t; }
  }

  if (STATS && lane == 0) {
    unsigned long long* wl = P.wavelog + 4 * ((size_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6));
    wl[0] = w_start;
    wl[1] = w_refill;
    wl[2] = __builtin_amdgcn_s_memrealtime();
    wl[3] = w_pixels;
  }
  // ---------------- counters: one atomic per wave and counter ----------------
  const unsigned long long s0 = wave_sum(c_primary), s1 = wave_sum(c_shadow), s2 = wave_sum(c_refl);
  unsigned long long s3 = 0, s4 = 0, s5 = 0;
  if (STATS) { s3 = wave_sum(c_nodes); s4 = wave_sum(c_tris); s5 = wave_sum(c_hits); }
  if (lane == 0) {
    // plain stores to this wave's slot (summed by the host): no contended atomics at exit
    unsigned long long* wc = P.wctr + 4 * ((size_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6));
    wc[0] = s0; wc[1] = s1; wc[2] = s2; wc[3] = 0;
    if (STATS) {
      atomicAdd(&P.ctr[CS_NODES], s3);
      atomicAdd(&P.ctr[CS_TRIS], s4);
      atomicAdd(&P.ctr[CS_HITS], s5);
      atomicAdd(&P.ctr[CD_TRAV_CYCLES], d_trav);     // wave-uniform values: lane 0's copy
      atomicAdd(&P.ctr[CD_SHADE_CYCLES], d_shade);
      atomicAdd(&P.ctr[CD_FETCH_CYCLES], d_fetch);
      atomicAdd(&P.ctr[CD_OUTER_ITERS], d_outer);
    }
  }
  if (STATS) {   // per-lane partial sums of the wave-level ticks
    const unsigned long long a = wave_sum(d_node_it), b = wave_sum(d_node_ln), c = wave_sum(d_leaf_it);
    const unsigned long long d = wave_sum(d_leaf_ln), e = wave_sum(d_round_it), f = wave_sum(d_round_ln);
    const unsigned long long g = wave_sum(d_spills), h = wave_sum(d_node_lines), q = wave_sum(d_leaf_lines);
    const unsigned long long r = wave_sum(d_big_leaf), t = wave_sum(d_node_lds);
    const unsigned long long gu = wave_sum(d_gn_uni), gd = wave_sum(d_gn_dist), lu = wave_sum(d_leaf_uni);
    if (lane == 0) {
      atomicAdd(&P.ctr[CD_NODE_LDS_ITERS], t);
      atomicAdd(&P.ctr[CD_GNODE_UNIFORM], gu);
      atomicAdd(&P.ctr[CD_GNODE_DISTINCT], gd);
      atomicAdd(&P.ctr[CD_LEAF_UNIFORM], lu);
      atomicAdd(&P.ctr[CD_NODE_ITERS], a);
      atomicAdd(&P.ctr[CD_NODE_LANES], b);
      atomicAdd(&P.ctr[CD_LEAF_ITERS], c);
      atomicAdd(&P.ctr[CD_LEAF_LANES], d);
      atomicAdd(&P.ctr[CD_TRAV_ROUNDS], e);
      atomicAdd(&P.ctr[CD_TRAV_ROUND_LANES], f);
      atomicAdd(&P.ctr[CD_SPILLS], g);
      atomicAdd(&P.ctr[CD_NODE_LINES], h);
      atomicAdd(&P.ctr[CD_LEAF_LINES], q);
      atomicAdd(&P.ctr[CD_BIG_LEAF_TESTS], r);
    }
  }
}

// ---------------------------------------------------------------------------
// Adaptive supersampling, selection step (adaptive_supersampling_device,
// mytracer_gpu.cu:162-200): an interior pixel is re-rendered with subp x subp
// samples when the squared colour differences to its 4 neighbours in the
// primary image sum above the threshold.  fp64, the reference's operation
// order; one wave = one 8x8 tile, selected pixel ids are compacted with one
// atomic per wave.  Pixels not selected are copied to the output here.
__device__ __forceinline__ double nsq3(const double* a, const double* b) {
  const double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
  return dx * dx + dy * dy + dz * dz;
}

// Row geometry of a shard for the adaptive neighbour test: local (packed) rows are cut
// into segments of consecutive global rows (one per stripe, or one row range); the rows
// just outside a segment come from the halo [segment][0: row below, 1: row above].
struct ShardRows {
  int rows, W, H;
  int row_begin, stripe_h, stripe_count, stripe_index;
  __host__ __device__ int global_row(int lrow) const {
    return stripe_count == 1 ? row_begin + lrow
                             : ((lrow / stripe_h) * stripe_count + stripe_index) * stripe_h + (lrow % stripe_h);
  }
  __host__ __device__ int seg_first(int lrow) const { return stripe_count == 1 ? 0 : lrow - lrow % stripe_h; }
  __host__ __device__ int seg_last(int lrow) const {
    return stripe_count == 1 ? rows - 1 : min(seg_first(lrow) + stripe_h, rows) - 1;
  }
  __host__ __device__ int segment(int lrow) const { return stripe_count == 1 ? 0 : lrow / stripe_h; }
  __host__ __device__ int segments() const { return stripe_count == 1 ? (rows > 0) : (rows + stripe_h - 1) / stripe_h; }
};

// adaptive_supersampling_device's selection (mytracer_gpu.cu:170-200) over the shard's
// rows: normSq differences to the 4 neighbours in the reference order (x+1, y+1, x-1,
// y-1), interior pixels of the FRAME only; unselected pixels are copied to the output,
// selected ones are compacted into list as local pixel ids.  A wave takes an 8x8 tile (the
// list keeps a tile's pixels together: 64-pixel row chunks instead made the adaptive render 5 %
// slower); a block of kSelThreads walks kSelTilesPerWave tiles per wave, gathers its selection
// in LDS and appends it with ONE
// device atomic (one per wave serialised ~8 k atomics on the counter's line: 68 us per 1080p
// frame).
constexpr int kSelThreads = 1024;
#ifndef RT_SEL_TILES
#define RT_SEL_TILES 8
#endif
constexpr int kSelTilesPerWave = RT_SEL_TILES;
constexpr int kSelTilesPerBlock = (kSelThreads / 64) * kSelTilesPerWave;
__global__ void __launch_bounds__(kSelThreads) adaptive_select_kernel(const double* prim, const double* halo, void* out,
                                                                      int out_fmt, ShardRows G, double threshold,
                                                                      int tiles_x, long long n_tiles, uint32_t* list,
                                                                      unsigned long long* count, uint32_t frame_tag,
                                                                      const double* const* prims, void* const* outs) {
  if (prims) {   // several frames in one launch: frame blockIdx.y
    prim = prims[blockIdx.y];
    out = outs[blockIdx.y];
    frame_tag = (uint32_t)blockIdx.y << kListFrameShift;
  }
  __shared__ uint32_t s_list[kSelThreads * kSelTilesPerWave];
  __shared__ uint32_t s_n;
  __shared__ unsigned long long s_base;
  if (threadIdx.x == 0) s_n = 0u;
  __syncthreads();
  const int j = threadIdx.x & 63;
  const int W = G.W;
  for (int it = 0; it < kSelTilesPerWave; ++it) {
    // consecutive waves take consecutive tiles
    const long long tile = (long long)blockIdx.x * kSelTilesPerBlock + it * (kSelThreads / 64) + (threadIdx.x >> 6);
    bool sel = false;
    int x = 0, lrow = 0;
    if (tile < n_tiles) {
      const long long ty = tile / tiles_x;
      x = (int)(tile - ty * tiles_x) * 8 + (j & 7);
      lrow = (int)ty * 8 + (j >> 3);
      if (x < W && lrow < G.rows) {
        const size_t o = 3 * ((size_t)lrow * W + x);
        const double* c = prim + o;
        const int y = G.global_row(lrow);
        if (x >= 1 && y >= 1 && x < W - 1 && y < G.H - 1) {
          const int seg = G.segment(lrow);
          const double* up = lrow < G.seg_last(lrow) ? c + 3 * (size_t)W : halo + 3 * ((size_t)(2 * seg + 1) * W + x);
          const double* dn = lrow > G.seg_first(lrow) ? c - 3 * (size_t)W : halo + 3 * ((size_t)(2 * seg) * W + x);
          const double n = nsq3(c, c + 3) + nsq3(c, up) + nsq3(c, c - 3) + nsq3(c, dn);
          sel = n > threshold;
        }
        if (!sel) {
          if (out_fmt == RT_OUT_RGB_F64) {
            double* d = reinterpret_cast<double*>(out) + o;
            d[0] = c[0]; d[1] = c[1]; d[2] = c[2];
          } else {
            float* d = reinterpret_cast<float*>(out) + o;
            d[0] = (float)c[0]; d[1] = (float)c[1]; d[2] = (float)c[2];
          }
        }
      }
    }
    const unsigned long long m = __ballot(sel);
    if (m != 0ull) {
      const int leader = __ffsll((long long)m) - 1;
      uint32_t base = 0u;
      if (j == leader) base = atomicAdd(&s_n, (uint32_t)__popcll(m));   // LDS
      base = __shfl(base, leader);
      if (sel) {
        const unsigned long long below = j == 0 ? 0ull : (m & (~0ull >> (64 - j)));
        s_list[base + __popcll(below)] = frame_tag | (uint32_t)((size_t)lrow * W + x);
      }
    }
  }
  __syncthreads();
  const uint32_t n = s_n;
  if (n == 0u) return;
  if (threadIdx.x == 0) s_base = atomicAdd(count, (unsigned long long)n);
  __syncthreads();
  const unsigned long long b = s_base;
  for (uint32_t k = threadIdx.x; k < n; k += kSelThreads) list[b + k] = s_list[k];
}

// Adaptive pass, final step (mytracer_gpu.cu:202-227): sum each listed pixel's
// samples in (si, sj) order, divide by subp^2, clamp, store.
__global__ void __launch_bounds__(256) adaptive_reduce_kernel(const uint32_t* list, const unsigned long long* count,
                                                              const double* samples, int nsamp, void* out,
                                                              int out_fmt, const FrameDesc* frames) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)*count) return;
  const double* s = samples + 3 * (size_t)i * nsamp;
  double r = 0.0, g = 0.0, b = 0.0;
  for (int k = 0; k < nsamp; ++k) {
    r = r + s[3 * k];
    g = g + s[3 * k + 1];
    b = b + s[3 * k + 2];
  }
  const double nn = (double)nsamp;
  r = stdmin(r / nn, 1.0);
  g = stdmin(g / nn, 1.0);
  b = stdmin(b / nn, 1.0);
  const uint32_t id = list[i];
  const size_t o = 3 * (size_t)(id & kListPixMask);
  if (frames) out = frames[id >> kListFrameShift].out;   // several frames: the launch's frame table
  if (out_fmt == RT_OUT_RGB_F64) {
    double* d = reinterpret_cast<double*>(out) + o;
    d[0] = r; d[1] = g; d[2] = b;
  } else {
    float* d = reinterpret_cast<float*>(out) + o;
    d[0] = (float)r; d[1] = (float)g; d[2] = (float)b;
  }
}

// ===========================================================================
// host side
// ===========================================================================
thread_local std::string g_error;

int fail(int code, const std::string& msg) {
  g_error = msg;
  return code;
}

#define HIP_TRY(call)                                                                          \
  do {                                                                                         \
    const hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess)                                                                      \
      return fail(RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));              \
  } while (0)

float round_down_host(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafterf(f, -INFINITY);
  return f;
}
float round_up_host(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafterf(f, INFINITY);
  return f;
}

using KernelFn = void (*)(KParams);

struct Variant {
  KernelFn fn;
  bool stats;
};

// [0] production (4-wide), [1] 4-wide + counters, [2] canonical 2-wide counters
// (the traversal the oracle replicates: tests pin its node / triangle counts),
// [3] production + per-round timeline (RT_FLAG_TIMELINE, diagnostics), [4] production with a
// 16-entry stack ring (deep hierarchies).
const Variant kVariants[] = {
    {render_kernel<4, false>, false},
    {render_kernel<4, true>, true},
    {render_kernel<2, true>, true},
    {render_kernel<4, false, true>, false},
    {render_kernel<4, false, false, 16>, false},
};
constexpr int kNumVariants = 5;
constexpr int kRingDeep = 16;
inline int variant_ring(int v) { return v == 4 ? kRingDeep : kShortStack; }
constexpr int kMaxDepth = 4096;  // traversal stack entries (LDS ring + global spill)
// LDS per block: kSlotDoubles doubles of slot, task + visibility words and
// min(stack_words, ring) stack entries per thread.
size_t lds_bytes(int stack_words, int ring = kShortStack) {
  stack_words = std::max(stack_words, kMigWords);   // compaction hands registers over in stack entries
  return (size_t)kBlock *
         (kSlotDoubles * sizeof(double) + (2 + (size_t)std::min(stack_words, ring)) * sizeof(uint32_t));
}
// ... plus the top treelet (n_top 128-B nodes) after it
size_t lds_bytes_total(int stack_words, int n_top, int ring = kShortStack) {
  return lds_bytes(stack_words, ring) + (size_t)n_top * sizeof(GNode4) + RT_MAX_LIGHTS * 6 * sizeof(double) + kPoolBytes;
}
// treelet nodes that fit next to a ring of the given size in a block's 40 KB
int top_nodes_for(int stack_words, int ring, int n_gnodes4) {
  const long long room = 40960 - (long long)lds_bytes_total(stack_words, 0, ring);
  return (int)std::max(0LL, std::min<long long>({room / (long long)sizeof(GNode4), (long long)kTopNodes, (long long)n_gnodes4}));
}

}  // namespace

// Per-launch mutable state.  A scene owns a ring of kContexts so launches on
// different streams can run concurrently: the drain of one frame (waves finishing
// their last pixels) overlaps the next frame's work.  A context is
// reused only after its previous launch completed (stream wait on `done`).
constexpr int kContexts = 8;
struct LaunchCtx {
  unsigned long long* d_ctr = nullptr;       // [kCtrWords] work heads, stats, diagnostics, then
                                             // FrameDesc[kMaxFrames] (one H2D copy per launch)
  unsigned char* h_ctl = nullptr;            // pinned staging of the same bytes
  double* d_pstate = nullptr;                // path state, nslots x kFields fp64
  uint32_t* d_spill = nullptr;               // [stack_words][nslots] (only when stack_words > kShortStack)
  unsigned long long* d_wavelog = nullptr;   // [nslots / 64][4]
  unsigned long long* d_wctr = nullptr;      // [nslots / 64][4] per-wave ray counts
  unsigned long long* d_tl = nullptr;        // [nslots / 64][kTlCap][kTlWords], allocated by the first TL launch
  hipEvent_t ev0 = nullptr, ev1 = nullptr;   // kernel start / end (timing, reuse fence)
  long long waves = 0;                       // waves of the last launch (per-wave counter slots)
  bool used = false;
};

struct rt_scene {
  int device = 0;
  GNode* d_nodes = nullptr;
  GTri* d_tris = nullptr;
  uint32_t* d_slot2dev = nullptr;
  TriShade* d_shade = nullptr;
  double* d_tnorm = nullptr;      // [record][12] face + vertex normals
  double* d_tu = nullptr;
  double* d_tv = nullptr;
  unsigned char* d_texels = nullptr;
  GMat* d_mats = nullptr;
  int n_gnodes = 0;
  long long n_tris = 0;
  int n_meshes = 0;
  int depth = 0;
  int stack_words = 1;          // LDS stack entries per thread (>= tree depth)
  LaunchCtx ctx[kContexts];
  int next_ctx = 0;             // ring cursor
  int last_ctx = -1;            // context of the most recent launch
  size_t nslots = 0;
  double* d_lights = nullptr;   // [light_cap][6] position xyz, colour rgb
  int light_cap = 0;            // lights d_lights can hold
  std::vector<double> cached_light_data;   // the table currently in d_lights
  double delta = 0.0;
  double root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};
  long long bytes = 0;
  int n_cu = 0;
  int blocks_per_cu[kNumVariants] = {0, 0, 0, 0, 0};
  bool deep = false;            // launches use the 16-entry ring variant (deep hierarchy)
  int n_top_deep = 0;           // treelet nodes beside the 16-entry ring
  GNode4* d_nodes4 = nullptr;
  int n_gnodes4 = 0;
  int n_top = 0;                // 4-wide nodes each block caches in LDS
  std::vector<GMat> mesh_mats;  // host copy: the analytic materials are appended after these
  GPrim* d_prims = nullptr;     // analytic primitives (rt_scene_set_analytic), spheres then planes
  int n_prims = 0;
  long long table_bytes = 0;    // device bytes of d_mats + d_prims
};

namespace {

template <typename T>
int upload(T** dst, const std::vector<T>& src, long long& bytes) {
  const size_t n = std::max<size_t>(src.size(), 1);
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(dst), n * sizeof(T)));
  if (!src.empty()) HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  bytes += (long long)(n * sizeof(T));
  return RT_OK;
}

#ifndef RT_LEAF_MAX
#define RT_LEAF_MAX 1
#endif
constexpr int kLeafMax = RT_LEAF_MAX;   // device leaves hold at most this many triangles

// Binary tree the device layouts are built from: the reference tree (mybvh.cpp)
// node for node, with reference leaves of more than kLeafMax triangles refined.
struct DevTree {
  std::vector<std::array<double, 3>> lo, hi;
  std::vector<int> left, right;    // internal: children (device-tree ids)
  std::vector<int> first, count;   // count > 0: leaf of device records [first, first + count)
  void reserve(size_t n) {
    lo.reserve(n); hi.reserve(n); left.reserve(n); right.reserve(n); first.reserve(n); count.reserve(n);
  }
  void resize(size_t n) {
    lo.resize(n); hi.resize(n); left.resize(n, -1); right.resize(n, -1); first.resize(n, 0); count.resize(n, 0);
  }
  int add() {
    lo.push_back({0, 0, 0});
    hi.push_back({0, 0, 0});
    left.push_back(-1);
    right.push_back(-1);
    first.push_back(0);
    count.push_back(0);
    return (int)left.size() - 1;
  }
};

void build_device_tree(const rt_scene_soa* s, const rt_bvh_soa* b, DevTree& E, std::vector<uint32_t>& dev2slot) {
  const long long nt = s->n_vertex_idx / 3;
  E.reserve(2 * (size_t)nt);
  for (long long i = 0; i < nt; ++i) dev2slot[i] = (uint32_t)i;
  auto vtx = [&](uint32_t slot, int c) { return s->vertex_pos + 3 * (size_t)s->vertex_idx[3 * (size_t)slot + c]; };
  auto centroid = [&](uint32_t slot, int k) { return (vtx(slot, 0)[k] + vtx(slot, 1)[k] + vtx(slot, 2)[k]) / 3.0; };
  // refines device records [first, first + count) under node id (explicit work list)
  struct Job { int id, first, count; };
  std::vector<Job> jobs;
  auto refine = [&](int root, int first0, int count0) {
    jobs.push_back({root, first0, count0});
    while (!jobs.empty()) {
      const Job j = jobs.back();
      jobs.pop_back();
      std::array<double, 3> lo = {DBL_MAX, DBL_MAX, DBL_MAX}, hi = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
      std::array<double, 3> clo = lo, chi = hi;
      for (int r = j.first; r < j.first + j.count; ++r)
        for (int k = 0; k < 3; ++k) {
          for (int c = 0; c < 3; ++c) {
            lo[k] = std::min(lo[k], vtx(dev2slot[r], c)[k]);
            hi[k] = std::max(hi[k], vtx(dev2slot[r], c)[k]);
          }
          clo[k] = std::min(clo[k], centroid(dev2slot[r], k));
          chi[k] = std::max(chi[k], centroid(dev2slot[r], k));
        }
      E.lo[j.id] = lo;
      E.hi[j.id] = hi;
      if (j.count <= kLeafMax) {
        E.first[j.id] = j.first;
        E.count[j.id] = j.count;
        continue;
      }
      int axis = 0;
      for (int k = 1; k < 3; ++k)
        if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
      if (chi[axis] > clo[axis])   // median of centroids on the longest axis (else: halve in slot order)
        std::stable_sort(dev2slot.begin() + j.first, dev2slot.begin() + j.first + j.count,
                         [&](uint32_t a, uint32_t c) { return centroid(a, axis) < centroid(c, axis); });
      const int l = E.add(), r = E.add();
      E.left[j.id] = l;
      E.right[j.id] = r;
      const int half = j.count / 2;
      jobs.push_back({r, j.first + half, j.count - half});
      jobs.push_back({l, j.first, half});
    }
  };
  // reference tree, node for node (explicit stack: reference depth is unbounded)
  std::vector<std::pair<int, int>> stk;   // (reference node, device-tree id)
  stk.emplace_back(0, E.add());
  while (!stk.empty()) {
    const auto [n, id] = stk.back();
    stk.pop_back();
    for (int k = 0; k < 3; ++k) {
      E.lo[id][k] = b->bb_min[3 * (size_t)n + k];
      E.hi[id][k] = b->bb_max[3 * (size_t)n + k];
    }
    if (b->tri_count[n] == 0) {
      const int l = E.add(), r = E.add();
      E.left[id] = l;
      E.right[id] = r;
      stk.emplace_back(b->left_child[n] + 1, r);
      stk.emplace_back(b->left_child[n], l);
    } else if (b->tri_count[n] <= kLeafMax) {
      E.first[id] = b->first_tri[n];
      E.count[id] = b->tri_count[n];
    } else {
      refine(id, b->first_tri[n], b->tri_count[n]);
    }
  }
}

// Device hierarchy option "sah": a binned-SAH tree over all triangles, split down to
// kLeafMax per leaf, instead of the reference tree + refinement.  Pixels do not depend
// on it (smallest (t, slot) over a conservative superset); the canonical
// 2-wide kernel keeps walking the reference tree through slot2dev.  Parallel: the top
// splits bin on all threads, the subtrees below them are built on threads into local
// arenas and appended in job order, so the tree does not depend on the thread count.
int sah_threads() {
  const char* e = std::getenv("RT_BUILD_THREADS");
  int t = e ? std::atoi(e) : 0;
  if (t <= 0) {
    const char* o = std::getenv("OMP_NUM_THREADS");
    t = o ? std::atoi(o) : 0;
  }
  if (t <= 0) t = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(t, 64));
}

struct SahData {
  std::vector<std::array<double, 3>> lo, hi, c;   // per reference slot: bounds, centroid
};
using V3 = std::array<double, 3>;
#ifndef RT_SAH_BINS
#define RT_SAH_BINS 16   // A/B: 8/16/24 +2 %, 32 baseline, 64/128 -4 % (office); 16 -1 % on random triangles
#endif
constexpr int kSahBins = RT_SAH_BINS;   // binned SAH: bins per axis
const V3 kV3Lo = {DBL_MAX, DBL_MAX, DBL_MAX}, kV3Hi = {-DBL_MAX, -DBL_MAX, -DBL_MAX};

inline void grow3(V3& lo, V3& hi, const V3& l2, const V3& h2) {
  for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], l2[k]); hi[k] = std::max(hi[k], h2[k]); }
}
inline double half_area(const V3& lo, const V3& hi) {
  const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}

// Splits records [first, first + count) of idx (partitioned in place): fills the node box,
// returns the split position, or -1 for a leaf.  `threads` > 1 bins in parallel chunks.
long long sah_split(const SahData& D, std::vector<uint32_t>& idx, long long first, long long count, V3& lo, V3& hi,
                    int threads) {
  struct Part { V3 lo, hi, clo, chi; };
  struct Bins { V3 lo[3][kSahBins], hi[3][kSahBins]; long long n[3][kSahBins]; };
  const int T = (threads > 1 && count >= (1 << 16)) ? threads : 1;
  auto chunk = [&](int t, long long& a, long long& b) { a = first + count * t / T; b = first + count * (t + 1) / T; };
  Part parts_local[1];
  std::vector<Part> parts_vec(T > 1 ? T : 0);
  Part* parts = T > 1 ? parts_vec.data() : parts_local;
  auto run = [&](auto&& fn) {
    if (T == 1) { fn(0); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(fn, t);
    for (auto& x : th) x.join();
  };
  run([&](int t) {
    long long a, b;
    chunk(t, a, b);
    Part P{kV3Lo, kV3Hi, kV3Lo, kV3Hi};
    for (long long r = a; r < b; ++r) {
      const uint32_t q = idx[r];
      grow3(P.lo, P.hi, D.lo[q], D.hi[q]);
      grow3(P.clo, P.chi, D.c[q], D.c[q]);
    }
    parts[t] = P;
  });
  V3 clo = kV3Lo, chi = kV3Hi;
  lo = kV3Lo; hi = kV3Hi;
  for (int t = 0; t < T; ++t) { grow3(lo, hi, parts[t].lo, parts[t].hi); grow3(clo, chi, parts[t].clo, parts[t].chi); }
  if (count <= kLeafMax) return -1;
  if (count <= 4) {   // tiny node: object median on the longest centroid axis
    int axis = 0;
    for (int k = 1; k < 3; ++k)
      if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
    const long long mid = first + count / 2;
    std::nth_element(idx.begin() + first, idx.begin() + mid, idx.begin() + first + count,
                     [&](uint32_t a, uint32_t b) { return D.c[a][axis] < D.c[b][axis] || (D.c[a][axis] == D.c[b][axis] && a < b); });
    return mid;
  }
  const int nb = (int)std::min<long long>(kSahBins, count);   // bins in use
  double scale[3];
  for (int k = 0; k < 3; ++k) scale[k] = chi[k] > clo[k] ? nb / (chi[k] - clo[k]) : 0.0;
  auto bin_of = [&](uint32_t q, int k) { return std::min(nb - 1, (int)((D.c[q][k] - clo[k]) * scale[k])); };
  Bins local;
  std::vector<Bins> extra(T > 1 ? T - 1 : 0);
  auto bins_of = [&](int t) -> Bins& { return t == 0 ? local : extra[t - 1]; };
  run([&](int t) {
    Bins& B = bins_of(t);
    for (int k = 0; k < 3; ++k)
      for (int i = 0; i < nb; ++i) { B.lo[k][i] = kV3Lo; B.hi[k][i] = kV3Hi; B.n[k][i] = 0; }
    long long a, b;
    chunk(t, a, b);
    for (long long r = a; r < b; ++r) {
      const uint32_t q = idx[r];
      for (int k = 0; k < 3; ++k) {
        if (scale[k] == 0.0) continue;
        const int bi = bin_of(q, k);
        grow3(B.lo[k][bi], B.hi[k][bi], D.lo[q], D.hi[q]);
        B.n[k][bi]++;
      }
    }
  });
  for (int t = 1; t < T; ++t)
    for (int k = 0; k < 3; ++k)
      for (int i = 0; i < nb; ++i) {
        grow3(local.lo[k][i], local.hi[k][i], extra[t - 1].lo[k][i], extra[t - 1].hi[k][i]);
        local.n[k][i] += extra[t - 1].n[k][i];
      }
  const Bins& B = local;
  double best_cost = DBL_MAX;
  int best_axis = -1, best_split = 0;
  for (int k = 0; k < 3; ++k) {
    if (scale[k] == 0.0) continue;
    double right_cost[kSahBins];
    V3 rlo = kV3Lo, rhi = kV3Hi;
    long long rn = 0;
    for (int i = nb - 1; i > 0; --i) {
      grow3(rlo, rhi, B.lo[k][i], B.hi[k][i]);
      rn += B.n[k][i];
      right_cost[i] = rn ? half_area(rlo, rhi) * (double)rn : 0.0;
    }
    V3 llo = kV3Lo, lhi = kV3Hi;
    long long ln = 0;
    for (int i = 0; i < nb - 1; ++i) {
      grow3(llo, lhi, B.lo[k][i], B.hi[k][i]);
      ln += B.n[k][i];
      if (ln == 0 || ln == count) continue;
      const double cost = half_area(llo, lhi) * (double)ln + right_cost[i + 1];
      if (cost < best_cost) { best_cost = cost; best_axis = k; best_split = i + 1; }
    }
  }
  if (best_axis < 0) return first + count / 2;   // all centroids equal: halve in slot order
  return std::partition(idx.begin() + first, idx.begin() + first + count,
                        [&](uint32_t q) { return bin_of(q, best_axis) < best_split; }) - idx.begin();
}

// Builds the subtree of records [first, first + count) under node `root` of T.
void sah_subtree(const SahData& D, std::vector<uint32_t>& idx, DevTree& T, int root, long long first, long long count) {
  struct Job { int id; long long first, count; };
  std::vector<Job> jobs = {{root, first, count}};
  while (!jobs.empty()) {
    const Job j = jobs.back();
    jobs.pop_back();
    V3 lo, hi;
    const long long mid = sah_split(D, idx, j.first, j.count, lo, hi, 1);
    T.lo[j.id] = lo;
    T.hi[j.id] = hi;
    if (mid < 0) {
      T.first[j.id] = (int)j.first;
      T.count[j.id] = (int)j.count;
      continue;
    }
    const int l = T.add(), r = T.add();
    T.left[j.id] = l;
    T.right[j.id] = r;
    jobs.push_back({r, mid, j.first + j.count - mid});
    jobs.push_back({l, j.first, mid - j.first});
  }
}

void build_sah_tree(const rt_scene_soa* s, DevTree& E, std::vector<uint32_t>& dev2slot) {
  const bool timing = std::getenv("RT_UPLOAD_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto tick = [&](const char* phase) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "  sah: %-14s %8.3f s\n", phase, std::chrono::duration<double>(t - t_last).count());
    t_last = t;
  };
  const long long nt = s->n_vertex_idx / 3;
  const int threads = nt >= 200000 ? sah_threads() : 1;
  E.reserve(2 * (size_t)nt);
  SahData D;
  D.lo.resize((size_t)nt); D.hi.resize((size_t)nt); D.c.resize((size_t)nt);
  auto prep = [&](long long a, long long b) {
    for (long long i = a; i < b; ++i) {
      dev2slot[i] = (uint32_t)i;
      for (int k = 0; k < 3; ++k) {
        double lo = DBL_MAX, hi = -DBL_MAX, sum = 0.0;
        for (int c = 0; c < 3; ++c) {
          const double v = s->vertex_pos[3 * (size_t)s->vertex_idx[3 * i + c] + k];
          lo = std::min(lo, v); hi = std::max(hi, v); sum += v;
        }
        D.lo[i][k] = lo; D.hi[i][k] = hi; D.c[i][k] = sum / 3.0;
      }
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(prep, nt * t / threads, nt * (t + 1) / threads);
    for (auto& x : th) x.join();
  }
  tick("prep");
  // top levels: big jobs split with parallel binning, breadth first
  struct Job { int id; long long first, count; };
  const long long kBig = threads > 1 ? std::max<long long>(1 << 15, nt / (8LL * threads)) : LLONG_MAX;
  std::vector<Job> pending, queue = {{E.add(), 0, nt}};
  for (size_t q = 0; q < queue.size(); ++q) {
    const Job j = queue[q];
    if (j.count < kBig) { pending.push_back(j); continue; }
    V3 lo, hi;
    const long long mid = sah_split(D, dev2slot, j.first, j.count, lo, hi, threads);
    E.lo[j.id] = lo;
    E.hi[j.id] = hi;
    if (mid < 0) { E.first[j.id] = (int)j.first; E.count[j.id] = (int)j.count; continue; }
    const int l = E.add(), r = E.add();
    E.left[j.id] = l;
    E.right[j.id] = r;
    queue.push_back({l, j.first, mid - j.first});
    queue.push_back({r, mid, j.first + j.count - mid});
  }
  tick("top");
  // subtrees on threads, each into its own arena (local node 0 = the pending node)
  std::vector<DevTree> arena(pending.size());
  std::atomic<size_t> next{0};
  auto worker = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < pending.size();) {
      arena[k].add();
      sah_subtree(D, dev2slot, arena[k], 0, pending[k].first, pending[k].count);
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < std::min<int>(threads, (int)pending.size()); ++t) th.emplace_back(worker);
    if (th.empty()) worker();
    for (auto& x : th) x.join();
  }
  tick("subtrees");
  // append in job order (thread-count independent): arena k's node i > 0 -> base[k] + i
  std::vector<long long> base(pending.size());
  long long total = (long long)E.left.size();
  for (size_t k = 0; k < pending.size(); ++k) {
    base[k] = total - 1;
    total += (long long)arena[k].left.size() - 1;
  }
  E.resize((size_t)total);
  next = 0;
  auto merge = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < pending.size();) {
      DevTree& A = arena[k];
      auto map = [&](int i) { return i == 0 ? pending[k].id : (int)(base[k] + i); };
      for (size_t i = 0; i < A.left.size(); ++i) {
        const int id = map((int)i);
        E.lo[id] = A.lo[i];
        E.hi[id] = A.hi[i];
        E.first[id] = A.first[i];
        E.count[id] = A.count[i];
        E.left[id] = A.count[i] > 0 ? -1 : map(A.left[i]);
        E.right[id] = A.count[i] > 0 ? -1 : map(A.right[i]);
      }
      A = DevTree();   // free as we go
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < std::min<int>(threads, (int)pending.size()); ++t) th.emplace_back(merge);
    if (th.empty()) merge();
    for (auto& x : th) x.join();
  }
  tick("merge");
}

// Device hierarchy option "sbvh": binned SAH with spatial splits.  A node whose best
// object split leaves children that overlap may instead cut space at a bin plane: a
// triangle straddling the plane is referenced from both sides, each reference bounded
// by the part of the triangle on its side (clipped in fp64; the fp32 boxes are grown
// by delta >> the fp64 clipping error, so every point of a triangle stays inside the
// box of some leaf that references it).  Leaves index device records; a triangle may
// own several identical records, and the kernel's (t, slot) rule makes duplicates
// harmless.  Top splits bin on all threads, subtrees build on threads, and the tree does
// not depend on the thread count.  Config 4 (10 M random triangles): +65 % records, +28 %
// (1988 -> 2554 Mrays/s), build 16 s on the GPU box's 16 threads (SAH: ~3 s).  Office
// proxy: 29 % extra records, 4-wide node visits -18 %, triangle tests -53 %, +17 % (A/B);
// alpha 0 (spatial splits everywhere) -3 %, 16/64/128 spatial bins within noise.
constexpr int kSbvhBins = 32;            // spatial bins per axis
constexpr int kSbvhBinsMax = 128;        // RT_SBVH_BINS cap
constexpr double kSbvhAlpha = 1e-5;      // try spatial splits when overlap > alpha * root area
constexpr double kSbvhBudget = 0.75;     // at most this many extra references per triangle
// SAH-terminated leaves of up to 2 references (node visit = 1 triangle test): office +3.9 %
// (15707 -> 16324 Mrays/s, A/B), 4K 16 spp +4.1 %, random triangles -2 %; 3 / 4 references or
// node costs 0.3 / 2 / 4 lose 0.3-6 %
constexpr int kSbvhLeafMax = 2;

struct SRef { uint32_t slot; V3 lo, hi; };

inline bool box_valid(const V3& lo, const V3& hi) { return lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2]; }

// Bounds of the parts of triangle r.slot on either side of plane x[axis] = pos, each
// intersected with r's box.  An empty side comes back with an invalid box.
void split_ref(const rt_scene_soa* s, const SRef& r, int axis, double pos, SRef& L, SRef& R) {
  L = {r.slot, kV3Lo, kV3Hi};
  R = {r.slot, kV3Lo, kV3Hi};
  V3 v[3];
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 3; ++k) v[c][k] = s->vertex_pos[3 * (size_t)s->vertex_idx[3 * (size_t)r.slot + c] + k];
  for (int e = 0; e < 3; ++e) {
    const V3& a = v[e];
    const V3& b = v[(e + 1) % 3];
    if (a[axis] <= pos) grow3(L.lo, L.hi, a, a);
    if (a[axis] >= pos) grow3(R.lo, R.hi, a, a);
    if ((a[axis] < pos && b[axis] > pos) || (a[axis] > pos && b[axis] < pos)) {
      const double t = (pos - a[axis]) / (b[axis] - a[axis]);
      V3 p;
      for (int k = 0; k < 3; ++k) p[k] = a[k] + t * (b[k] - a[k]);
      p[axis] = pos;
      grow3(L.lo, L.hi, p, p);
      grow3(R.lo, R.hi, p, p);
    }
  }
  for (int k = 0; k < 3; ++k) {
    L.lo[k] = std::max(L.lo[k], r.lo[k]); L.hi[k] = std::min(L.hi[k], r.hi[k]);
    R.lo[k] = std::max(R.lo[k], r.lo[k]); R.hi[k] = std::min(R.hi[k], r.hi[k]);
  }
  L.hi[axis] = std::min(L.hi[axis], pos);
  R.lo[axis] = std::max(R.lo[axis], pos);
}

struct SbvhCtx {
  const rt_scene_soa* s;
  double alpha, root_area;
  int sbins;
  int leaf_max;      // SAH-terminated leaves of up to this many references (1: always split)
  double c_trav;     // node visit cost in triangle-test units (leaf termination only)
};

// Splits the references R of one node (consumed): fills the node box; returns false for a
// leaf, else the two children's references.  `budget` = extra references this subtree may
// still create; `threads` > 1 bins in parallel chunks (deterministic merge order).
bool sbvh_split(const SbvhCtx& C, std::vector<SRef>& R, int depth, long long& budget, int threads, V3& lo, V3& hi,
                std::vector<SRef>& left, std::vector<SRef>& right) {
  const long long n = (long long)R.size();
  const int T = (threads > 1 && n >= (1 << 16)) ? threads : 1;
  auto chunk = [&](int t, long long& a, long long& b) { a = n * t / T; b = n * (t + 1) / T; };
  auto run = [&](auto&& fn) {
    if (T == 1) { fn(0); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(fn, t);
    for (auto& x : th) x.join();
  };
  auto cen = [](const SRef& r, int k) { return 0.5 * (r.lo[k] + r.hi[k]); };
  struct Box4 { V3 lo, hi, clo, chi; };
  std::vector<Box4> parts(T, Box4{kV3Lo, kV3Hi, kV3Lo, kV3Hi});
  run([&](int t) {
    long long a, b;
    chunk(t, a, b);
    Box4& P = parts[t];
    for (long long i = a; i < b; ++i) {
      const SRef& r = R[i];
      grow3(P.lo, P.hi, r.lo, r.hi);
      const V3 c = {cen(r, 0), cen(r, 1), cen(r, 2)};
      grow3(P.clo, P.chi, c, c);
    }
  });
  lo = kV3Lo; hi = kV3Hi;
  V3 clo = kV3Lo, chi = kV3Hi;
  for (const Box4& P : parts) { grow3(lo, hi, P.lo, P.hi); grow3(clo, chi, P.clo, P.chi); }
  if (n <= kLeafMax) return false;
  struct Bin { V3 lo, hi; long long n, enter, exit; };
  // ---- object split: binned SAH over reference centroids ----
  const int nb = (int)std::min<long long>(kSahBins, n);
  double best_cost = DBL_MAX, obj_overlap = 0.0;
  int ob_axis = -1, ob_split = 0;
  double oscale[3];
  for (int k = 0; k < 3; ++k) oscale[k] = chi[k] > clo[k] ? nb / (chi[k] - clo[k]) : 0.0;
  auto obin = [&](const SRef& r, int k) { return std::min(nb - 1, (int)((cen(r, k) - clo[k]) * oscale[k])); };
  {
    std::vector<std::array<Bin, 3 * kSahBins>> OB(T);
    run([&](int t) {
      auto& B = OB[t];
      for (auto& b : B) b = {kV3Lo, kV3Hi, 0, 0, 0};
      long long a, e;
      chunk(t, a, e);
      for (long long i = a; i < e; ++i)
        for (int k = 0; k < 3; ++k) {
          if (oscale[k] == 0.0) continue;
          Bin& b = B[k * kSahBins + obin(R[i], k)];
          grow3(b.lo, b.hi, R[i].lo, R[i].hi);
          b.n++;
        }
    });
    for (int t = 1; t < T; ++t)
      for (int i = 0; i < 3 * kSahBins; ++i) {
        grow3(OB[0][i].lo, OB[0][i].hi, OB[t][i].lo, OB[t][i].hi);
        OB[0][i].n += OB[t][i].n;
      }
    for (int k = 0; k < 3; ++k) {
      if (oscale[k] == 0.0) continue;
      const Bin* B = &OB[0][k * kSahBins];
      V3 rlo[kSahBins], rhi[kSahBins];
      V3 alo = kV3Lo, ahi = kV3Hi;
      for (int i = nb - 1; i > 0; --i) { grow3(alo, ahi, B[i].lo, B[i].hi); rlo[i] = alo; rhi[i] = ahi; }
      V3 llo = kV3Lo, lhi = kV3Hi;
      long long ln = 0;
      for (int i = 0; i < nb - 1; ++i) {
        grow3(llo, lhi, B[i].lo, B[i].hi);
        ln += B[i].n;
        if (ln == 0 || ln == n) continue;
        const double cost = half_area(llo, lhi) * (double)ln + half_area(rlo[i + 1], rhi[i + 1]) * (double)(n - ln);
        if (cost < best_cost) {
          best_cost = cost; ob_axis = k; ob_split = i + 1;
          V3 olo, ohi;
          for (int q = 0; q < 3; ++q) { olo[q] = std::max(llo[q], rlo[i + 1][q]); ohi[q] = std::min(lhi[q], rhi[i + 1][q]); }
          obj_overlap = box_valid(olo, ohi) ? half_area(olo, ohi) : 0.0;
        }
      }
    }
  }
  // ---- spatial split: bin planes, straddling references clipped into every bin they span ----
  int sp_axis = -1;
  double sp_cost = DBL_MAX, sp_pos = 0.0;
  if (budget > 0 && depth < 48 && obj_overlap > C.alpha * C.root_area) {
    const int sb = C.sbins;
    std::vector<std::array<Bin, 3 * kSbvhBinsMax>> SB(T);
    run([&](int t) {
      auto& B = SB[t];
      for (int i = 0; i < 3 * sb; ++i) B[i] = {kV3Lo, kV3Hi, 0, 0, 0};
      long long a, e;
      chunk(t, a, e);
      for (int k = 0; k < 3; ++k) {
        const double w = (hi[k] - lo[k]) / sb;
        if (!(w > 0.0)) continue;
        Bin* Bk = &B[k * sb];
        auto sbin = [&](double x) { return std::max(0, std::min(sb - 1, (int)((x - lo[k]) / w))); };
        for (long long i = a; i < e; ++i) {
          const SRef& r = R[i];
          const int b0 = sbin(r.lo[k]), b1 = sbin(r.hi[k]);
          Bk[b0].enter++;
          Bk[b1].exit++;
          SRef cur = r;
          for (int b = b0; b < b1; ++b) {
            SRef Lp, Rp;
            split_ref(C.s, cur, k, lo[k] + w * (b + 1), Lp, Rp);
            if (box_valid(Lp.lo, Lp.hi)) grow3(Bk[b].lo, Bk[b].hi, Lp.lo, Lp.hi);
            if (!box_valid(Rp.lo, Rp.hi)) { cur.lo = kV3Lo; cur.hi = kV3Hi; break; }
            cur = Rp;
          }
          if (box_valid(cur.lo, cur.hi)) grow3(Bk[b1].lo, Bk[b1].hi, cur.lo, cur.hi);
        }
      }
    });
    for (int t = 1; t < T; ++t)
      for (int i = 0; i < 3 * sb; ++i) {
        grow3(SB[0][i].lo, SB[0][i].hi, SB[t][i].lo, SB[t][i].hi);
        SB[0][i].enter += SB[t][i].enter;
        SB[0][i].exit += SB[t][i].exit;
      }
    for (int k = 0; k < 3; ++k) {
      const double w = (hi[k] - lo[k]) / sb;
      if (!(w > 0.0)) continue;
      const Bin* B = &SB[0][k * sb];
      V3 rlo[kSbvhBinsMax], rhi[kSbvhBinsMax];
      long long rn[kSbvhBinsMax];
      V3 alo = kV3Lo, ahi = kV3Hi;
      long long an = 0;
      for (int i = sb - 1; i > 0; --i) {
        grow3(alo, ahi, B[i].lo, B[i].hi); an += B[i].exit;
        rlo[i] = alo; rhi[i] = ahi; rn[i] = an;
      }
      V3 llo = kV3Lo, lhi = kV3Hi;
      long long ln = 0;
      for (int i = 0; i < sb - 1; ++i) {
        grow3(llo, lhi, B[i].lo, B[i].hi);
        ln += B[i].enter;
        if (ln == 0 || rn[i + 1] == 0 || (ln == n && rn[i + 1] == n)) continue;
        const double cost = half_area(llo, lhi) * (double)ln + half_area(rlo[i + 1], rhi[i + 1]) * (double)rn[i + 1];
        if (cost < sp_cost) { sp_cost = cost; sp_axis = k; sp_pos = lo[k] + w * (i + 1); }
      }
    }
  }
  if (n <= C.leaf_max) {   // SAH leaf termination: testing n triangles beats one more level
    const double a = half_area(lo, hi);
    if ((double)n * a <= std::min(best_cost, sp_cost) + C.c_trav * a) return false;
  }
  left.clear();
  right.clear();
  bool done = false;
  if (sp_axis >= 0 && sp_cost < best_cost) {
    // partition with reference unsplitting (keep a straddler whole on one side when cheaper)
    const int k = sp_axis;
    V3 llo = kV3Lo, lhi = kV3Hi, rlo = kV3Lo, rhi = kV3Hi;
    std::vector<SRef> straddle;
    for (const SRef& r : R) {
      if (r.hi[k] <= sp_pos) { left.push_back(r); grow3(llo, lhi, r.lo, r.hi); }
      else if (r.lo[k] >= sp_pos) { right.push_back(r); grow3(rlo, rhi, r.lo, r.hi); }
      else straddle.push_back(r);
    }
    long long nl = (long long)left.size() + (long long)straddle.size();
    long long nr = (long long)right.size() + (long long)straddle.size();
    for (const SRef& r : straddle) {
      SRef Lp, Rp;
      split_ref(C.s, r, k, sp_pos, Lp, Rp);
      const bool lv = box_valid(Lp.lo, Lp.hi), rv = box_valid(Rp.lo, Rp.hi);
      if (!lv || !rv) {   // the triangle lies on one side after all
        const SRef& keep = lv ? Lp : Rp;
        if (lv) { left.push_back(keep); grow3(llo, lhi, keep.lo, keep.hi); nr--; }
        else { right.push_back(keep); grow3(rlo, rhi, keep.lo, keep.hi); nl--; }
        continue;
      }
      V3 slo = llo, shi = lhi, tlo = rlo, thi = rhi;
      grow3(slo, shi, Lp.lo, Lp.hi); grow3(tlo, thi, Rp.lo, Rp.hi);
      const double c_split = half_area(slo, shi) * (double)nl + half_area(tlo, thi) * (double)nr;
      V3 ulo = llo, uhi = lhi, vlo = rlo, vhi = rhi;
      grow3(ulo, uhi, r.lo, r.hi); grow3(vlo, vhi, r.lo, r.hi);
      const double c_left = half_area(ulo, uhi) * (double)nl + half_area(tlo, thi) * (double)(nr - 1);
      const double c_right = half_area(slo, shi) * (double)(nl - 1) + half_area(vlo, vhi) * (double)nr;
      if (c_split <= c_left && c_split <= c_right && budget > 0) {
        left.push_back(Lp); right.push_back(Rp);
        llo = slo; lhi = shi; rlo = tlo; rhi = thi;
        budget--;
      } else if (c_left <= c_right) {
        left.push_back(r); llo = ulo; lhi = uhi; nr--;
      } else {
        right.push_back(r); rlo = vlo; rhi = vhi; nl--;
      }
    }
    done = !left.empty() && !right.empty() && !((long long)left.size() == n && (long long)right.size() == n);
    if (!done) { left.clear(); right.clear(); }
  }
  if (!done) {
    if (ob_axis < 0) {   // all centroids equal: halve in order
      left.assign(R.begin(), R.begin() + n / 2);
      right.assign(R.begin() + n / 2, R.end());
    } else {
      for (const SRef& r : R) (obin(r, ob_axis) < ob_split ? left : right).push_back(r);
    }
  }
  std::vector<SRef>().swap(R);
  return true;
}

// Builds the subtree of references R under node `root` of T (single thread); leaves index
// `records` (local to this subtree).
void sbvh_subtree(const SbvhCtx& C, DevTree& T, int root, std::vector<SRef>&& R, int depth, long long budget,
                  std::vector<uint32_t>& records) {
  struct Job { int id; std::vector<SRef> refs; int depth; };
  std::vector<Job> jobs;
  jobs.push_back({root, std::move(R), depth});
  std::vector<SRef> left, right;
  while (!jobs.empty()) {
    Job j = std::move(jobs.back());
    jobs.pop_back();
    V3 lo, hi;
    const long long n = (long long)j.refs.size();
    const bool split = sbvh_split(C, j.refs, j.depth, budget, 1, lo, hi, left, right);
    T.lo[j.id] = lo;
    T.hi[j.id] = hi;
    if (!split) {   // a leaf leaves the references in place
      T.first[j.id] = (int)records.size();
      T.count[j.id] = (int)n;
      for (const SRef& r : j.refs) records.push_back(r.slot);
      continue;
    }
    const int l = T.add(), r = T.add();
    T.left[j.id] = l;
    T.right[j.id] = r;
    jobs.push_back({r, std::move(right), j.depth + 1});
    jobs.push_back({l, std::move(left), j.depth + 1});
    left = {};
    right = {};
  }
}

void build_sbvh_tree(const rt_scene_soa* s, DevTree& E, std::vector<uint32_t>& records) {
  const bool timing = std::getenv("RT_UPLOAD_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto tick = [&](const char* phase) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "  sbvh: %-13s %8.3f s\n", phase, std::chrono::duration<double>(t - t_last).count());
    t_last = t;
  };
  const long long nt = s->n_vertex_idx / 3;
  const int threads = nt >= 200000 ? sah_threads() : 1;
  std::vector<SRef> refs((size_t)nt);
  {
    auto prep = [&](long long a, long long b) {
      for (long long i = a; i < b; ++i) {
        SRef& r = refs[i];
        r.slot = (uint32_t)i;
        r.lo = kV3Lo; r.hi = kV3Hi;
        for (int c = 0; c < 3; ++c) {
          const double* p = s->vertex_pos + 3 * (size_t)s->vertex_idx[3 * i + c];
          const V3 q = {p[0], p[1], p[2]};
          grow3(r.lo, r.hi, q, q);
        }
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) th.emplace_back(prep, nt * t / threads, nt * (t + 1) / threads);
    prep(0, nt / threads);
    for (auto& x : th) x.join();
  }
  SbvhCtx C{s, kSbvhAlpha, 0.0, kSbvhBins, kSbvhLeafMax, 1.0};
  if (const char* e = std::getenv("RT_SBVH_LEAF")) C.leaf_max = std::max(1, std::min(8, std::atoi(e)));
  if (const char* e = std::getenv("RT_SBVH_CTRAV")) C.c_trav = std::atof(e);
  double budget_frac = kSbvhBudget;   // A/B knobs
  if (const char* e = std::getenv("RT_SBVH_ALPHA")) C.alpha = std::atof(e);
  if (const char* e = std::getenv("RT_SBVH_BUDGET")) budget_frac = std::atof(e);
  if (const char* e = std::getenv("RT_SBVH_BINS")) C.sbins = std::max(2, std::min(kSbvhBinsMax, std::atoi(e)));
  {
    V3 lo = kV3Lo, hi = kV3Hi;
    for (const SRef& r : refs) grow3(lo, hi, r.lo, r.hi);
    C.root_area = half_area(lo, hi);
  }
  long long budget = (long long)(budget_frac * (double)nt);
  E.reserve(2 * (size_t)nt);
  tick("prep");
  // top levels: big nodes split with parallel binning, breadth first; their budget is shared
  struct Job { int id; std::vector<SRef> refs; int depth; };
  // (independent of the thread count, so the tree and the budget shares are too)
  const long long kBig = nt >= 200000 ? std::max<long long>(1 << 15, nt / 64) : LLONG_MAX;
  std::vector<Job> pending;
  std::deque<Job> queue;
  queue.push_back({E.add(), std::move(refs), 0});
  std::vector<uint32_t> top_records;   // leaves created above the subtrees (tiny scenes / degenerate)
  std::vector<int> top_leaf_ids;
  while (!queue.empty()) {
    Job j = std::move(queue.front());
    queue.pop_front();
    if ((long long)j.refs.size() < kBig) { pending.push_back(std::move(j)); continue; }
    V3 lo, hi;
    std::vector<SRef> left, right;
    const long long n = (long long)j.refs.size();
    const bool split = sbvh_split(C, j.refs, j.depth, budget, threads, lo, hi, left, right);
    E.lo[j.id] = lo;
    E.hi[j.id] = hi;
    if (!split) {   // unreachable for n >= kBig > kLeafMax; kept for safety
      E.first[j.id] = -1;
      E.count[j.id] = (int)n;
      continue;
    }
    const int l = E.add(), r = E.add();
    E.left[j.id] = l;
    E.right[j.id] = r;
    queue.push_back({l, std::move(left), j.depth + 1});
    queue.push_back({r, std::move(right), j.depth + 1});
  }
  tick("top");
  // subtrees on threads, each with its own arena, records and a budget share by size
  long long pend_refs = 0;
  for (const Job& j : pending) pend_refs += (long long)j.refs.size();
  std::vector<DevTree> arena(pending.size());
  std::vector<std::vector<uint32_t>> recs(pending.size());
  std::vector<long long> share(pending.size());
  for (size_t k = 0; k < pending.size(); ++k)
    share[k] = pend_refs > 0 ? (long long)((double)budget * (double)pending[k].refs.size() / (double)pend_refs) : 0;
  std::atomic<size_t> next{0};
  auto worker = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < pending.size();) {
      arena[k].add();
      sbvh_subtree(C, arena[k], 0, std::move(pending[k].refs), pending[k].depth, share[k], recs[k]);
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < std::min<int>(threads, (int)pending.size()); ++t) th.emplace_back(worker);
    if (th.empty()) worker();
    for (auto& x : th) x.join();
  }
  tick("subtrees");
  // append in job order (thread-count independent): arena k's node i > 0 -> base[k] + i,
  // its records -> rbase[k] + local index
  std::vector<long long> base(pending.size()), rbase(pending.size());
  long long total = (long long)E.left.size(), rtotal = 0;
  for (size_t k = 0; k < pending.size(); ++k) {
    base[k] = total - 1;
    total += (long long)arena[k].left.size() - 1;
    rbase[k] = rtotal;
    rtotal += (long long)recs[k].size();
  }
  E.resize((size_t)total);
  records.assign((size_t)rtotal, 0);
  next = 0;
  auto merge = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < pending.size();) {
      DevTree& A = arena[k];
      auto map = [&](int i) { return i == 0 ? pending[k].id : (int)(base[k] + i); };
      for (size_t i = 0; i < A.left.size(); ++i) {
        const int id = map((int)i);
        E.lo[id] = A.lo[i];
        E.hi[id] = A.hi[i];
        E.first[id] = A.count[i] > 0 ? (int)(rbase[k] + A.first[i]) : 0;
        E.count[id] = A.count[i];
        E.left[id] = A.count[i] > 0 ? -1 : map(A.left[i]);
        E.right[id] = A.count[i] > 0 ? -1 : map(A.right[i]);
      }
      std::copy(recs[k].begin(), recs[k].end(), records.begin() + rbase[k]);
      A = DevTree();
      std::vector<uint32_t>().swap(recs[k]);
    }
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < std::min<int>(threads, (int)pending.size()); ++t) th.emplace_back(merge);
    if (th.empty()) merge();
    for (auto& x : th) x.join();
  }
  tick("merge");
}


int validate(const rt_scene_soa* s, const rt_bvh_soa* b) {
  if (!s || !b) return fail(RT_ERR_INVALID, "rt_scene_upload: null scene or bvh");
  if (s->n_vertex_idx % 3 != 0 || s->n_vertex_idx < 0 || s->n_vertices < 0 || s->n_meshes < 0)
    return fail(RT_ERR_INVALID, "rt_scene_upload: inconsistent counts");
  const long long nt = s->n_vertex_idx / 3;
  if (nt > (long long)kSlotMask)
    return fail(RT_ERR_UNSUPPORTED, "rt_scene_upload: more than 2^30 triangles");
  if (nt > 0 && (b->n_nodes < 1 || b->n_nodes > 2 * nt - 1))
    return fail(RT_ERR_INVALID, "rt_scene_upload: bvh node count out of range");
  for (long long i = 0; i < s->n_vertex_idx; ++i)
    if (s->vertex_idx[i] < 0 || s->vertex_idx[i] >= s->n_vertices)
      return fail(RT_ERR_INVALID, "rt_scene_upload: vertex index out of range");
  for (int m = 0; m < s->n_meshes; ++m) {
    if (s->mesh_draw_mode[m] != RT_DRAW_FLAT && s->mesh_draw_mode[m] != RT_DRAW_PHONG)
      return fail(RT_ERR_INVALID, "rt_scene_upload: invalid draw mode (mytracer_gpu.cu:507)");
    if (s->mesh_tex_width[m] > 0) {
      if (s->mesh_tex_height[m] <= 0 || s->mesh_tex_offset[m] < 0 ||
          s->mesh_tex_offset[m] + (long long)s->mesh_tex_width[m] * s->mesh_tex_height[m] > s->n_texels)
        return fail(RT_ERR_INVALID, "rt_scene_upload: texture range out of bounds");
    }
  }
  for (int v = 0; v < s->n_vertices; ++v)
    if (s->vertex_mesh_id[v] < 0 || s->vertex_mesh_id[v] >= s->n_meshes)
      return fail(RT_ERR_INVALID, "rt_scene_upload: vertex mesh id out of range");
  for (int n = 0; n < b->n_nodes; ++n) {
    if (b->tri_count[n] < 0 || b->first_tri[n] < 0 || (long long)b->first_tri[n] + b->tri_count[n] > nt)
      return fail(RT_ERR_INVALID, "rt_scene_upload: bvh leaf range out of bounds");
    if (b->tri_count[n] == 0 && (b->left_child[n] < 1 || b->left_child[n] + 1 >= b->n_nodes))
      return fail(RT_ERR_INVALID, "rt_scene_upload: bvh child index out of range");
  }
  return RT_OK;
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_error.c_str(); }

const char* rt_build_info(void) {
  return "librt_hip: gfx950 persistent flattened render kernel; variants {4-wide 8-entry stack ring, 4-wide 16-entry ring (>= 2^18 triangle records), "
         "4-wide+stats, 2-wide canonical stats, 4-wide+round timeline}; fp32 4-wide nodes (128 B) with an LDS treelet, "
         "fp64 triangles/shading, LDS ray slots + stack ring (global spill), global path state, 8 XCD work heads";
}

int rt_scene_upload(const rt_scene_soa* s, const rt_bvh_soa* b, int device, rt_scene** out) {
  return rt_scene_upload_ex(s, b, device, nullptr, out);
}

}  // extern "C"

namespace {
// Host-side device layout of a scene: built once (the expensive part: device hierarchy,
// records), then copied to any number of devices (upload_image).
struct SceneImage {
  std::vector<GNode> nodes;
  std::vector<GNode4> nodes4;
  std::vector<GTri> tris;
  std::vector<uint32_t> slot2dev;
  std::vector<TriShade> shade;
  std::vector<double> tnorm, tu, tv;
  std::vector<unsigned char> texels;
  std::vector<GMat> mats;
  long long n_tris = 0;
  int n_meshes = 0;
  int depth = 0, stack4 = 1;
  double delta = 0.0;
  double root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};
};

int build_image(const rt_scene_soa* s, const rt_bvh_soa* b, const rt_upload_options* opt, SceneImage& I) {
  int tree_kind = RT_TREE_SBVH;
  if (const char* e = std::getenv("RT_DEVICE_TREE"))   // process default override (A/B runs)
    tree_kind = std::strcmp(e, "reference") == 0 || std::strcmp(e, "median") == 0 ? RT_TREE_REFERENCE
              : std::strcmp(e, "sbvh") == 0                                         ? RT_TREE_SBVH
                                                                                    : RT_TREE_SAH;
  if (opt) tree_kind = opt->device_tree;
  if (tree_kind != RT_TREE_SAH && tree_kind != RT_TREE_REFERENCE && tree_kind != RT_TREE_SBVH)
    return fail(RT_ERR_INVALID, "rt_scene_upload: unknown device_tree");
  const bool timing = std::getenv("RT_UPLOAD_TIMING") != nullptr;   // phase times to stderr (diagnostics)
  auto t_last = std::chrono::steady_clock::now();
  auto tick = [&](const char* phase) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "rt_scene_upload: %-14s %8.3f s\n", phase, std::chrono::duration<double>(t - t_last).count());
    t_last = t;
  };
  int rc = validate(s, b);
  if (rc != RT_OK) return rc;
  tick("validate");
  const long long nt = s->n_vertex_idx / 3;

  // ---- delta: conservative growth of the fp32 boxes ----
  double M = 0.0;
  for (long long k = 0; k < 3LL * s->n_vertices; ++k) M = std::max(M, std::fabs(s->vertex_pos[k]));
  if (!(M > 0.0)) M = 1.0;
  const double delta = M * 9.5367431640625e-07;   // 2^-20

  // ---- 2-wide fp32 nodes in preorder ----
  std::vector<GNode> nodes;
  std::vector<uint32_t> last(std::max<long long>(nt, 1), 0);
  int depth = 0;
  auto set_child = [&](GNode& g, int s_, int c) {
    float* ax[3] = {g.x, g.y, g.z};
    for (int k = 0; k < 3; ++k) {
      ax[k][2 * s_] = round_down_host(b->bb_min[3 * (size_t)c + k] - delta);
      ax[k][2 * s_ + 1] = round_up_host(b->bb_max[3 * (size_t)c + k] + delta);
    }
  };
  if (nt > 0) {
    for (int n = 0; n < b->n_nodes; ++n)
      if (b->tri_count[n] > 0) last[b->first_tri[n] + b->tri_count[n] - 1] = 1;
    if (b->tri_count[0] > 0) {   // root is a leaf
      GNode g{};
      set_child(g, 0, 0);
      g.ref[0] = kLeaf | (uint32_t)b->first_tri[0];
      g.ref[1] = kEmpty;
      nodes.push_back(g);
      depth = 1;
    } else {
      std::vector<int> gidx(b->n_nodes, -1);
      std::vector<std::pair<int, int>> stk;   // (node, depth)
      std::vector<int> order;
      stk.emplace_back(0, 0);
      while (!stk.empty()) {
        const auto [n, d] = stk.back();
        stk.pop_back();
        gidx[n] = (int)order.size();
        order.push_back(n);
        depth = std::max(depth, d + 1);
        const int l = b->left_child[n], r = l + 1;
        if (b->tri_count[r] == 0) stk.emplace_back(r, d + 1);
        if (b->tri_count[l] == 0) stk.emplace_back(l, d + 1);
      }
      nodes.resize(order.size());
      for (size_t gi = 0; gi < order.size(); ++gi) {
        const int n = order[gi];
        GNode& g = nodes[gi];
        std::memset(&g, 0, sizeof g);
        for (int s_ = 0; s_ < 2; ++s_) {
          const int c = b->left_child[n] + s_;
          set_child(g, s_, c);
          g.ref[s_] = (b->tri_count[c] == 0) ? (uint32_t)gidx[c] : (kLeaf | (uint32_t)b->first_tri[c]);
        }
      }
    }
  }
  tick("nodes2");
  // ---- device binary tree: the reference tree with oversize leaves refined ----
  // Reference leaves of more than kLeafMax triangles (coplanar grids the fixed-axis
  // median split cannot separate, mybvh.cpp:95-130) get a sub-tree split on the
  // longest centroid axis; their triangles are permuted within the leaf's slot
  // range.  The closest hit is the smallest (t, slot) over a conservative superset
  // of the triangles the ray can hit, so it does not depend on the tree.
  DevTree E;
  std::vector<uint32_t> dev2slot((size_t)std::max<long long>(nt, 1));
  if (nt > 0) {
    if (tree_kind == RT_TREE_SBVH) build_sbvh_tree(s, E, dev2slot);
    else if (tree_kind == RT_TREE_SAH) build_sah_tree(s, E, dev2slot);
    else build_device_tree(s, b, E, dev2slot);
  }
  tick("device tree");
  if (timing) std::fprintf(stderr, "rt_scene_upload: %lld triangles, %zu device records, %zu tree nodes\n", nt,
                           nt > 0 ? dev2slot.size() : (size_t)0, E.left.size());
  // device records: one per triangle, or more where spatial splits duplicated references
  const long long nrec = nt > 0 ? (long long)dev2slot.size() : 0;
  if (nrec > (long long)kSlotMask) return fail(RT_ERR_UNSUPPORTED, "rt_scene_upload: more than 2^30 device records");
  std::vector<uint32_t> slot2dev((size_t)std::max<long long>(nt, 1), 0);
  for (long long g = nrec - 1; g >= 0; --g) slot2dev[dev2slot[g]] = (uint32_t)g;

  // ---- 4-wide collapse of the device tree (production layout) ----
  std::vector<GNode4> nodes4;
  int stack4 = 1;
  if (nt > 0) {
    auto area = [&](int c) {
      const double dx = E.hi[c][0] - E.lo[c][0], dy = E.hi[c][1] - E.lo[c][1], dz = E.hi[c][2] - E.lo[c][2];
      return dx * dy + dy * dz + dz * dx;
    };
    auto internal = [&](int c) { return E.count[c] == 0; };
    struct Kids { int c[4]; int n; };
    // Optional SAH-optimal collapse (RT_COLLAPSE=dp): D[n][j] = the least SAH cost of covering
    // binary subtree n with at most j child slots; a slot costs area * c_tri for a leaf and
    // area * c_node + D(children, 4) for a wide node (the 4 box tests of a visit are charged to
    // the visited node).  Children ids exceed their parent's in every builder, so one reverse
    // sweep fills the table.
    const char* ce = std::getenv("RT_COLLAPSE");
    const bool dp = ce && std::strcmp(ce, "dp") == 0;
    double c_tri = 1.0;
    if (const char* e = std::getenv("RT_COLLAPSE_CTRI")) c_tri = std::atof(e);
    std::vector<std::array<double, 5>> D;
    std::vector<std::array<int8_t, 5>> Dk;   // 0: n itself is the slot, k > 0: k slots to the left child
    std::vector<int8_t> Ik;                  // wide node n: slots given to its left child
    if (dp) {
      const size_t nn = E.left.size();
      D.assign(nn, {0, 0, 0, 0, 0});
      Dk.assign(nn, {0, 0, 0, 0, 0});
      Ik.assign(nn, 0);
      for (long long n = (long long)nn - 1; n >= 0; --n) {
        if (!internal((int)n)) {
          for (int j = 1; j <= 4; ++j) D[n][j] = area((int)n) * c_tri;
          continue;
        }
        const int l = E.left[n], r = E.right[n];
        double best = DBL_MAX;
        for (int k = 1; k <= 3; ++k)
          if (D[l][k] + D[r][4 - k] < best) { best = D[l][k] + D[r][4 - k]; Ik[n] = (int8_t)k; }
        const double self = area((int)n) + best;   // c_node = 1
        D[n][1] = self;
        for (int j = 2; j <= 4; ++j) {
          D[n][j] = self;
          for (int k = 1; k < j; ++k)
            if (D[l][k] + D[r][j - k] < D[n][j]) { D[n][j] = D[l][k] + D[r][j - k]; Dk[n][j] = (int8_t)k; }
        }
      }
    }
    auto kids_of = [&](int n) {   // open the largest internal child until 4 children
      if (dp) {
        Kids k{{-1, -1, -1, -1}, 0};
        auto expand = [&](auto&& self, int m, int j) -> void {
          if (!internal(m) || Dk[m][j] == 0) { k.c[k.n++] = m; return; }
          self(self, E.left[m], Dk[m][j]);
          self(self, E.right[m], j - Dk[m][j]);
        };
        expand(expand, E.left[n], Ik[n]);
        expand(expand, E.right[n], 4 - Ik[n]);
        return k;
      }
      Kids k{{E.left[n], E.right[n], -1, -1}, 2};
      while (k.n < 4) {
        int pick = -1;
        double best_a = -1.0;
        for (int i = 0; i < k.n; ++i)
          if (internal(k.c[i]) && area(k.c[i]) > best_a) { best_a = area(k.c[i]); pick = i; }
        if (pick < 0) break;
        const int c = k.c[pick];
        for (int i = k.n; i > pick + 1; --i) k.c[i] = k.c[i - 1];
        k.c[pick] = E.left[c];
        k.c[pick + 1] = E.right[c];
        k.n++;
      }
      return k;
    };
    auto set4 = [&](GNode4& g, int s_, int c) {
      g.lox[s_] = round_down_host(E.lo[c][0] - delta);
      g.hix[s_] = round_up_host(E.hi[c][0] + delta);
      g.loy[s_] = round_down_host(E.lo[c][1] - delta);
      g.hiy[s_] = round_up_host(E.hi[c][1] + delta);
      g.loz[s_] = round_down_host(E.lo[c][2] - delta);
      g.hiz[s_] = round_up_host(E.hi[c][2] + delta);
    };
    // an absent child gets the empty box [+inf, -inf]: every slab test misses it, so the
    // kernel needs no separate "child present" test
    auto set_empty = [&](GNode4& g, int s_) {
      g.lox[s_] = g.loy[s_] = g.loz[s_] = INFINITY;
      g.hix[s_] = g.hiy[s_] = g.hiz[s_] = -INFINITY;
      g.ref[s_] = kEmpty;
    };
    if (!internal(0)) {
      GNode4 g;
      std::memset(&g, 0, sizeof g);
      set4(g, 0, 0);
      g.ref[0] = kLeaf | (uint32_t)E.first[0];
      for (int s_ = 1; s_ < 4; ++s_) set_empty(g, s_);
      nodes4.push_back(g);
    } else {
      // Numbering: the first kTopNodes collapsed nodes in breadth-first order (the top
      // treelet each block caches in LDS), the rest in preorder so a
      // subtree stays contiguous.  Children always get larger ids than their parent.
      std::vector<int> order;                  // device-tree ids of the collapsed nodes
      std::vector<Kids> kids;
      std::vector<int> g4(E.left.size(), -1);
      auto assign = [&](int n) {
        g4[n] = (int)order.size();
        order.push_back(n);
        kids.push_back(kids_of(n));
      };
      assign(0);
      for (size_t q = 0; q < order.size() && (int)order.size() < kTopNodes; ++q) {   // breadth-first top
        const Kids k = kids[q];
        for (int i = 0; i < k.n && (int)order.size() < kTopNodes; ++i)
          if (internal(k.c[i])) assign(k.c[i]);
      }
      std::vector<int> stk;                    // preorder below the treelet
      for (int gi = (int)order.size() - 1; gi >= 0; --gi) {
        const Kids k = kids[gi];
        for (int i = k.n - 1; i >= 0; --i)
          if (internal(k.c[i]) && g4[k.c[i]] < 0) stk.push_back(k.c[i]);
        while (!stk.empty()) {
          const int n = stk.back();
          stk.pop_back();
          if (g4[n] >= 0) continue;
          assign(n);
          const Kids& kn = kids.back();
          for (int i = kn.n - 1; i >= 0; --i)
            if (internal(kn.c[i])) stk.push_back(kn.c[i]);
        }
      }
      nodes4.resize(order.size());
      std::vector<int> need(order.size(), 0);   // stack entries needed below each node
      for (int gi = (int)order.size() - 1; gi >= 0; --gi) {
        GNode4& g = nodes4[gi];
        std::memset(&g, 0, sizeof g);
        const Kids& k = kids[gi];
        int deeper = 0;
        for (int s_ = 0; s_ < 4; ++s_) {
          if (s_ < k.n) {
            const int c = k.c[s_];
            set4(g, s_, c);
            g.ref[s_] = internal(c) ? (uint32_t)g4[c] : (kLeaf | (uint32_t)E.first[c]);
            if (internal(c)) deeper = std::max(deeper, need[g4[c]]);
          } else {
            set_empty(g, s_);
          }
        }
        need[gi] = k.n - 1 + deeper;
      }
      stack4 = std::max(1, need[0]);
    }
  }

  tick("collapse4");
  if (depth > kMaxDepth || stack4 > kMaxDepth)
    return fail(RT_ERR_UNSUPPORTED, "rt_scene_upload: BVH needs more than 4096 traversal-stack entries");

  // ---- triangle records / shading data in device order ----
  std::vector<uint8_t> last_dev((size_t)std::max<long long>(nrec, 1), 0);
  for (size_t n = 0; n < E.left.size(); ++n)
    if (E.count[n] > 0) last_dev[(size_t)E.first[n] + E.count[n] - 1] = 1;
  std::vector<GTri> tris((size_t)nrec);
  std::vector<TriShade> shade((size_t)nrec);
  std::vector<double> tnorm(12 * (size_t)nrec);
  std::atomic<bool> bad_uv{false};
  auto fill = [&](long long g0, long long g1) {
  for (long long g = g0; g < g1; ++g) {
    const long long i = dev2slot[g];   // reference slot
    const int v0 = s->vertex_idx[3 * i], v1 = s->vertex_idx[3 * i + 1], v2 = s->vertex_idx[3 * i + 2];
    const double* p0 = s->vertex_pos + 3 * (size_t)v0;
    const double* p1 = s->vertex_pos + 3 * (size_t)v1;
    const double* p2 = s->vertex_pos + 3 * (size_t)v2;
    GTri& T = tris[g];
    for (int k = 0; k < 3; ++k) {
      T.e1[k] = p0[k] - p2[k];
      T.e2[k] = p1[k] - p2[k];
      T.p2[k] = p2[k];
    }
    T.mesh = s->vertex_mesh_id[v0];                 // meshId = vertexMeshId_[vi0], mytracer_gpu.cu:492
    T.meta = (uint32_t)i | (last[i] ? kLastRef : 0u) | (last_dev[g] ? kLastDev : 0u);
    TriShade& sh = shade[g];
    sh.v[0] = v0; sh.v[1] = v1; sh.v[2] = v2;
    for (int k = 0; k < 3; ++k) sh.t[k] = s->texture_idx ? s->texture_idx[3 * i + k] : -1;
    sh.pad[0] = sh.pad[1] = 0;
    if (s->mesh_tex_width[T.mesh] > 0)
      for (int k = 0; k < 3; ++k)
        if (sh.t[k] < 0 || sh.t[k] >= s->n_tex_coords)
          bad_uv = true;
    double* tn = tnorm.data() + 12 * (size_t)g;
    for (int k = 0; k < 3; ++k) {
      tn[k] = s->face_normals[3 * i + k];
      tn[3 + k] = s->vertex_normals[3 * (size_t)v0 + k];
      tn[6 + k] = s->vertex_normals[3 * (size_t)v1 + k];
      tn[9 + k] = s->vertex_normals[3 * (size_t)v2 + k];
    }
  }
  };
  {
    const int T = nrec >= 200000 ? sah_threads() : 1;
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(fill, nrec * t / T, nrec * (t + 1) / T);
    fill(0, nrec / T);
    for (auto& x : th) x.join();
  }
  if (bad_uv) return fail(RT_ERR_INVALID, "rt_scene_upload: textured mesh with invalid uv index");
  tick("records");
  std::vector<GMat> mats((size_t)s->n_meshes);
  for (int m = 0; m < s->n_meshes; ++m) {
    GMat& G = mats[m];
    std::memset(&G, 0, sizeof G);
    for (int k = 0; k < 3; ++k) {
      G.ka[k] = s->mat_ambient[3 * m + k];
      G.kd[k] = s->mat_diffuse[3 * m + k];
      G.ks[k] = s->mat_specular[3 * m + k];
    }
    G.shininess = s->mat_shininess[m];
    G.mirror = s->mat_mirror[m];
    G.shadowable = s->mat_shadowable[m];
    G.draw_mode = s->mesh_draw_mode[m];
    G.tex_w = s->mesh_tex_width[m] > 0 ? s->mesh_tex_width[m] : -1;
    G.tex_h = s->mesh_tex_height[m];
    G.tex_off = s->mesh_tex_offset[m];
  }
  I.tu.assign(s->tex_u, s->tex_u + s->n_tex_coords);
  I.tv.assign(s->tex_v, s->tex_v + s->n_tex_coords);
  I.texels.assign(s->texels, s->texels + 3 * s->n_texels);
  I.nodes = std::move(nodes);
  I.nodes4 = std::move(nodes4);
  I.tris = std::move(tris);
  I.slot2dev = std::move(slot2dev);
  I.shade = std::move(shade);
  I.tnorm = std::move(tnorm);
  I.mats = std::move(mats);
  I.n_tris = nt;
  I.n_meshes = s->n_meshes;
  I.depth = depth;
  I.stack4 = stack4;
  I.delta = delta;
  if (nt > 0)
    for (int k = 0; k < 3; ++k) {
      I.root_lo[k] = b->bb_min[k] - delta;
      I.root_hi[k] = b->bb_max[k] + delta;
    }
  tick("misc");
  return RT_OK;
}

// Copies a built scene image to `device` and allocates its launch contexts.
int upload_image(const SceneImage& I, int device, rt_scene** out) {
  HIP_TRY(hipSetDevice(device));
  {   // the adaptive passes take their list and sample buffers (up to GBs) from the device's
      // stream-ordered pool on every call: keep freed blocks in the pool instead of unmapping
      // them at each synchronisation (re-mapping them cost ~60 ms per 107-frame batch)
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
      uint64_t keep = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
  }
  auto* sc = new rt_scene();
  sc->device = device;
  long long bytes = 0;
  int rc = RT_OK;
  if (rc == RT_OK) rc = upload(&sc->d_nodes, I.nodes, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_nodes4, I.nodes4, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_tris, I.tris, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_slot2dev, I.slot2dev, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_shade, I.shade, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_tnorm, I.tnorm, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_tu, I.tu, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_tv, I.tv, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_texels, I.texels, bytes);
  if (rc == RT_OK) rc = upload(&sc->d_mats, I.mats, bytes);
  if (rc != RT_OK) {
    rt_scene_free(sc);
    return rc;
  }
  sc->n_gnodes = (int)I.nodes.size();
  sc->n_tris = I.n_tris;
  sc->n_meshes = I.n_meshes;
  sc->mesh_mats = I.mats;
  sc->table_bytes = (long long)(std::max<size_t>(I.mats.size(), 1) * sizeof(GMat));
  sc->depth = I.depth;
  sc->stack_words = std::max(std::max(1, I.depth), I.stack4);
  sc->n_gnodes4 = (int)I.nodes4.size();
  sc->n_top = RT_TOP_NODES > 0 ? std::min(kTopNodes, sc->n_gnodes4) : 0;
  if (const char* e = std::getenv("RT_LDS_TOP"))   // A/B knob: cache fewer nodes (0 = none)
    sc->n_top = std::max(0, std::min(sc->n_top, std::atoi(e)));
  // deep hierarchies (half a million device records and more: random-triangle soups of ~1 M and
  // up spill an 8-entry ring on every other ray, the office proxy on 1 in 130) render with the
  // 16-entry ring and the 9-node treelet that fits beside it (A/B)
  sc->deep = I.tris.size() >= (size_t)(1u << 18);   // device records (office 77 k prefers 8, 500 k random 16)
  if (const char* e = std::getenv("RT_RING")) sc->deep = std::atoi(e) >= 16;   // A/B knob
  sc->n_top_deep = RT_TOP_NODES > 0 ? top_nodes_for(sc->stack_words, kRingDeep, sc->n_gnodes4) : 0;
  sc->delta = I.delta;
  for (int k = 0; k < 3; ++k) {
    sc->root_lo[k] = I.root_lo[k];
    sc->root_hi[k] = I.root_hi[k];
  }
  sc->bytes = bytes;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { rt_scene_free(sc); return fail(RT_ERR_HIP, "hipGetDeviceProperties failed"); }
  sc->n_cu = prop.multiProcessorCount;
  int max_blocks = 1;
  for (int v = 0; v < kNumVariants; ++v) {
    const int ring = variant_ring(v);
    const size_t lds = lds_bytes_total(sc->stack_words, ring == kRingDeep ? sc->n_top_deep : sc->n_top, ring);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(kVariants[v].fn), kBlock, lds) !=
            hipSuccess || nb < 1)
      nb = 1;
    // the occupancy API can report one block per CU more than fits (MI355X_MICROARCH.md: at some
    // SGPR counts), which would leave a persistent grid's last blocks waiting for the first to
    // exit: bound it by the VGPR file (512 per SIMD lane, granule 8) and the CU's 160 KB of LDS
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kVariants[v].fn)) == hipSuccess && fa.numRegs > 0) {
      const int waves_per_simd = 512 / ((fa.numRegs + 7) / 8 * 8);
      nb = std::min(nb, std::max(1, waves_per_simd * 4 / (kBlock / 64)));
    }
    nb = std::min(nb, std::max(1, (int)(160 * 1024 / lds)));
    sc->blocks_per_cu[v] = nb;
    max_blocks = std::max(max_blocks, nb);
  }
  sc->nslots = (size_t)sc->n_cu * max_blocks * kBlock;
  if (hipMalloc(reinterpret_cast<void**>(&sc->d_lights), RT_MAX_LIGHTS * 6 * sizeof(double)) != hipSuccess) {
    rt_scene_free(sc);
    return fail(RT_ERR_HIP, "hipMalloc of lights failed");
  }
  sc->light_cap = RT_MAX_LIGHTS;
  sc->bytes += (long long)(RT_MAX_LIGHTS * 6 * sizeof(double));
  for (LaunchCtx& c : sc->ctx) {
    const size_t pb = sc->nslots * kFields * sizeof(double);
    const size_t wb = sc->nslots / 64 * 4 * sizeof(unsigned long long);
    const size_t sb = sc->stack_words > kShortStack ? sc->nslots * (size_t)sc->stack_words * sizeof(uint32_t) : 0;
    if (hipMalloc(reinterpret_cast<void**>(&c.d_ctr), kCtlBytes) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c.h_ctl), kCtlBytes, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c.d_pstate), pb) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c.d_wavelog), wb) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c.d_wctr), wb) != hipSuccess ||
        (sb > 0 && hipMalloc(reinterpret_cast<void**>(&c.d_spill), sb) != hipSuccess) ||
        hipMemset(c.d_ctr, 0, kCtrBytes) != hipSuccess ||
        hipEventCreate(&c.ev0) != hipSuccess || hipEventCreate(&c.ev1) != hipSuccess) {
      rt_scene_free(sc);
      return fail(RT_ERR_HIP, "allocation of launch contexts failed");
    }
    sc->bytes += (long long)(kCtlBytes + pb + 2 * wb + sb);
  }
  *out = sc;
  return RT_OK;
}
}  // namespace

extern "C" {

int rt_scene_upload_ex(const rt_scene_soa* s, const rt_bvh_soa* b, int device, const rt_upload_options* opt,
                       rt_scene** out) {
  if (!out) return fail(RT_ERR_INVALID, "rt_scene_upload: null out");
  *out = nullptr;
  SceneImage I;
  const int rc = build_image(s, b, opt, I);
  return rc != RT_OK ? rc : upload_image(I, device, out);
}

int rt_scene_upload_multi(const rt_scene_soa* s, const rt_bvh_soa* b, const int* devices, int n_devices,
                          const rt_upload_options* opt, rt_scene** outs) {
  if (!outs || !devices || n_devices < 1) return fail(RT_ERR_INVALID, "rt_scene_upload_multi: bad argument");
  for (int g = 0; g < n_devices; ++g) outs[g] = nullptr;
  SceneImage I;
  int rc = build_image(s, b, opt, I);
  if (rc != RT_OK) return rc;
  // one host thread per device: the copies and context allocations proceed in parallel
  std::vector<int> rcs(n_devices, RT_OK);
  std::vector<std::string> errs(n_devices);
  std::vector<std::thread> th;
  for (int g = 0; g < n_devices; ++g)
    th.emplace_back([&, g]() {
      rcs[g] = upload_image(I, devices[g], &outs[g]);
      if (rcs[g] != RT_OK) errs[g] = g_error;   // thread-local message of that thread
    });
  for (auto& t : th) t.join();
  for (int g = 0; g < n_devices; ++g)
    if (rcs[g] != RT_OK) {
      for (int k = 0; k < n_devices; ++k) {
        rt_scene_free(outs[k]);
        outs[k] = nullptr;
      }
      return fail(rcs[g], "rt_scene_upload_multi: device " + std::to_string(devices[g]) + ": " + errs[g]);
    }
  return RT_OK;
}

long long rt_scene_device_bytes(const rt_scene* s) { return s ? s->bytes : 0; }

int rt_rows_in_shard(const rt_render_params* p) {
  if (!p) return 0;
  const int H = p->camera.height;
  const int sc = p->stripe_count > 0 ? p->stripe_count : 1;
  const int sh = p->stripe_height > 0 ? p->stripe_height : 1;
  if (sc == 1) {
    const int rb = std::max(0, p->row_begin);
    const int re = (p->row_end <= 0 || p->row_end > H) ? H : p->row_end;
    return std::max(0, re - rb);
  }
  int rows = 0;
  for (int y = 0; y < H; ++y)
    if ((y / sh) % sc == p->stripe_index) rows++;
  return rows;
}

}  // extern "C"

namespace {
// Counter words of a finished launch, with the per-wave ray-count slots summed into
// [CS_PRIMARY, CS_REFLECT] (the kernel stores them per wave instead of adding atomically).
int read_counters(const LaunchCtx& C, unsigned long long* c) {
  HIP_TRY(hipMemcpy(c, C.d_ctr, kCtrWords * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  if (C.waves > 0) {
    std::vector<unsigned long long> w((size_t)C.waves * 4);
    HIP_TRY(hipMemcpy(w.data(), C.d_wctr, w.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < w.size(); i += 4) {
      c[CS_PRIMARY] += w[i];
      c[CS_SHADOW] += w[i + 1];
      c[CS_REFLECT] += w[i + 2];
    }
  }
  return RT_OK;
}

// One render launch; list != nullptr: adaptive pass over the pixel ids list[0 .. *count)
// (at most list_cap of them) of the full frame.
// n_frames > 1 (rt_launch_frames): params p[0..n_frames) differ only in their camera vectors,
// frame f is written to outs[f].
int launch_render(rt_scene* sc, const rt_render_params* p, int n_frames, void* const* outs, rt_stats* stats,
                  void* stream, const uint32_t* list, const unsigned long long* count, long long list_cap,
                  double* sample_out = nullptr) {
  if (!sc || !p || !outs) return fail(RT_ERR_INVALID, "rt_launch_compute_image: null argument");
  if (n_frames < 1 || n_frames > kMaxFrames) return fail(RT_ERR_INVALID, "rt_launch_frames: n_frames out of range");
  for (int f = 0; f < n_frames; ++f) {
    if (!outs[f]) return fail(RT_ERR_INVALID, "rt_launch_compute_image: null output buffer");
    if (f == 0) continue;
    rt_render_params q = p[f];   // everything but the camera vectors must match frame 0
    for (int k = 0; k < 3; ++k) {
      q.camera.eye[k] = p[0].camera.eye[k]; q.camera.lower_left[k] = p[0].camera.lower_left[k];
      q.camera.x_dir[k] = p[0].camera.x_dir[k]; q.camera.y_dir[k] = p[0].camera.y_dir[k];
    }
    if (std::memcmp(&q, &p[0], sizeof q) != 0)
      return fail(RT_ERR_INVALID, "rt_launch_frames: frames may differ only in camera position and direction");
  }
  if (p->camera.width <= 0 || p->camera.height <= 0 || p->camera.width > 65535 || p->camera.height > 65535)
    return fail(RT_ERR_INVALID, "bad image size (1..65535 per side)");
  if (p->n_lights < 0 || p->n_lights > (p->lights_ext ? RT_LIGHTS_LIMIT : RT_MAX_LIGHTS))
    return fail(RT_ERR_INVALID, "n_lights out of range (more than RT_MAX_LIGHTS lights need lights_ext)");
  if (p->spp_n < 1 || p->spp_n > 64) return fail(RT_ERR_INVALID, "spp_n must be in [1, 64]");
  if (p->max_depth < 0) return fail(RT_ERR_INVALID, "max_depth must be >= 0");
  if (p->out_format != RT_OUT_RGB_F32 && p->out_format != RT_OUT_RGB_F64) return fail(RT_ERR_INVALID, "bad out_format");
  const int scount = p->stripe_count > 0 ? p->stripe_count : 1;
  if (p->stripe_index < 0 || p->stripe_index >= scount) return fail(RT_ERR_INVALID, "stripe_index out of range");
  if (scount > 1 && (p->row_begin != 0 || (p->row_end > 0 && p->row_end != p->camera.height)))
    return fail(RT_ERR_INVALID, "row ranges cannot be combined with stripe_count > 1");
  const int rows = rt_rows_in_shard(p);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(sc->device));

  KParams P;
  std::memset(&P, 0, sizeof P);
  P.nodes = sc->d_nodes; P.nodes4 = sc->d_nodes4; P.tris = sc->d_tris; P.slot2dev = sc->d_slot2dev; P.shade = sc->d_shade; P.tnorm = sc->d_tnorm;
  P.tu = sc->d_tu; P.tv = sc->d_tv; P.texels = sc->d_texels; P.mats = sc->d_mats;
  P.prims = sc->d_prims; P.n_prims = sc->n_prims;
  LaunchCtx& C = sc->ctx[sc->next_ctx];
  const int ci = sc->next_ctx;
  P.ctr = C.d_ctr;
  P.heads = reinterpret_cast<unsigned long long*>(reinterpret_cast<unsigned char*>(C.d_ctr) + kHeadsOff);
  P.wctr = C.d_wctr;
  P.n_frames = n_frames;
  P.frames = reinterpret_cast<const FrameDesc*>(reinterpret_cast<unsigned char*>(C.d_ctr) + kCtrBytes);
  P.n_gnodes = sc->n_gnodes;
  P.out_fmt = p->out_format;
  for (int k = 0; k < 3; ++k) {
    P.root_lo[k] = sc->root_lo[k]; P.root_hi[k] = sc->root_hi[k];
    P.bg[k] = p->background[k]; P.amb[k] = p->ambience[k];
  }
  P.W = p->camera.width;
  P.H = p->camera.height;
  P.n_lights = p->n_lights;
  P.max_depth = p->max_depth;
  {  // lights live in device memory; re-uploaded (device-synchronising) only when they change
    std::vector<double> ld(6 * (size_t)p->n_lights);
    for (int i = 0; i < p->n_lights; ++i) {
      const rt_light* L = rt_params_light(p, i);
      for (int k = 0; k < 3; ++k) { ld[6 * i + k] = L->position[k]; ld[6 * i + 3 + k] = L->color[k]; }
    }
    if (ld != sc->cached_light_data) {
      HIP_TRY(hipDeviceSynchronize());   // launches in flight may still read the old table
      if (p->n_lights > sc->light_cap) {
        HIP_TRY(hipFree(sc->d_lights));
        sc->d_lights = nullptr;
        sc->bytes -= (long long)(sc->light_cap * 6 * sizeof(double));
        sc->light_cap = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&sc->d_lights), ld.size() * sizeof(double)));
        sc->light_cap = p->n_lights;
        sc->bytes += (long long)(ld.size() * sizeof(double));
      }
      if (!ld.empty()) HIP_TRY(hipMemcpy(sc->d_lights, ld.data(), ld.size() * sizeof(double), hipMemcpyHostToDevice));
      sc->cached_light_data = std::move(ld);
    }
  }
  P.lights = sc->d_lights;
  P.pstate = C.d_pstate;
  P.spill = C.d_spill;
  P.wavelog = C.d_wavelog;
  P.nslots = sc->nslots;
  P.spp_n = p->spp_n;
  P.row_begin = scount == 1 ? std::max(0, p->row_begin) : 0;
  P.stripe_h = p->stripe_height > 0 ? p->stripe_height : 1;
  P.stripe_count = scount;
  P.stripe_index = p->stripe_index;
  P.rows = rows;
  P.tiles_x = (P.W + 7) / 8;
  P.nsamp = p->spp_n * p->spp_n;
  P.frame_tiles = list ? (list_cap * P.nsamp + 63) / 64 : (long long)P.tiles_x * ((rows + 7) / 8);
  P.n_tiles = P.frame_tiles * n_frames;
  P.list = list;
  P.list_count = count;
  P.sample_out = sample_out;

  const int v = (p->flags & RT_FLAG_TRAVERSAL_STATS) ? 2
                : (p->flags & RT_FLAG_WIDE_STATS) ? 1
                : (p->flags & RT_FLAG_TIMELINE) ? 3
                : sc->deep ? 4 : 0;   // 4: the 16-entry-ring production variant
  const int ring = variant_ring(v);
  const int n_top = ring == kRingDeep ? sc->n_top_deep : sc->n_top;
  const size_t lds = lds_bytes_total(sc->stack_words, n_top, ring);
  P.n_top = n_top;
  P.top_off = (int)lds_bytes(sc->stack_words, ring);
  P.lights_off = P.top_off + n_top * (int)sizeof(GNode4);
  P.pool_off = P.lights_off + RT_MAX_LIGHTS * 6 * (int)sizeof(double);
  const long long waves_needed = (P.n_tiles * 64 + 63) / 64;
  int bpc = sc->blocks_per_cu[v];
  if (const char* e = std::getenv("RT_BLOCKS_PER_CU"))   // A/B knob: a smaller persistent grid
    bpc = std::max(1, std::min(bpc, std::atoi(e)));
  long long blocks = (long long)sc->n_cu * bpc;
  blocks = std::max<long long>(1, std::min<long long>(blocks, (waves_needed + kBlock / 64 - 1) / (kBlock / 64)));
  blocks = std::min<long long>(blocks, (long long)(sc->nslots / kBlock));
  if (const char* e = std::getenv("RT_GRID_SPARE"))   // A/B knob: leave block slots to concurrent kernels
    blocks = std::max<long long>(1, blocks - std::max(0, std::atoi(e)));

  if (C.used) {
    HIP_TRY(hipStreamWaitEvent(st, C.ev1, 0));   // previous launch on this context done (device side)
    HIP_TRY(hipEventSynchronize(C.ev1));         // ... and its staged copy consumed (host side)
  }
  // zeroed counters + frame table, one copy from the context's pinned staging
  std::memset(C.h_ctl, 0, kCtrBytes);
  FrameDesc* fd = reinterpret_cast<FrameDesc*>(C.h_ctl + kCtrBytes);
  for (int f = 0; f < n_frames; ++f) {
    std::memset(&fd[f], 0, sizeof(FrameDesc));
    for (int k = 0; k < 3; ++k) {
      fd[f].eye[k] = p[f].camera.eye[k]; fd[f].ll[k] = p[f].camera.lower_left[k];
      fd[f].xd[k] = p[f].camera.x_dir[k]; fd[f].yd[k] = p[f].camera.y_dir[k];
    }
    fd[f].out = outs[f];
  }
  HIP_TRY(hipMemcpyAsync(C.d_ctr, C.h_ctl, kCtrBytes + (size_t)n_frames * sizeof(FrameDesc), hipMemcpyHostToDevice, st));
  if (v == 3) {   // round timeline: zeroed, so unused records read as t = 0
    const size_t tb = sc->nslots / 64 * kTlCap * kTlWords * sizeof(unsigned long long);
    if (!C.d_tl) {
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&C.d_tl), tb));
      sc->bytes += (long long)tb;
    }
    HIP_TRY(hipMemsetAsync(C.d_tl, 0, tb, st));
  }
  P.tl = C.d_tl;
  HIP_TRY(hipEventRecord(C.ev0, st));
  if (rows > 0) {
    void* args[] = {&P};
    HIP_TRY(hipLaunchKernel(reinterpret_cast<const void*>(kVariants[v].fn), dim3((unsigned)blocks), dim3(kBlock),
                            args, lds, st));
  }
  HIP_TRY(hipEventRecord(C.ev1, st));
  C.used = true;
  C.waves = rows > 0 ? blocks * (kBlock / 64) : 0;
  sc->last_ctx = ci;
  sc->next_ctx = (ci + 1) % kContexts;
  if (stats) {
    HIP_TRY(hipStreamSynchronize(st));
    unsigned long long c[kCtrWords];
    const int rc = read_counters(C, c);
    if (rc != RT_OK) return rc;
    std::memset(stats, 0, sizeof *stats);
    stats->primary_rays = (long long)c[CS_PRIMARY];
    stats->shadow_rays = (long long)c[CS_SHADOW];
    stats->reflection_rays = (long long)c[CS_REFLECT];
    stats->node_visits = (long long)c[CS_NODES];
    stats->tri_tests = (long long)c[CS_TRIS];
    stats->closest_hits = (long long)c[CS_HITS];
    stats->pixels = (long long)c[CS_PIXELS];
    if (c[CD_GUARD] != 0)
      return fail(RT_ERR_HIP, "rt_launch_compute_image: persistent-loop watchdog fired (kernel bug)");
  }
  return RT_OK;
}
}  // namespace

namespace {
// stream-ordered scratch of one adaptive call, released on every return path (errors included)
struct StreamScratch {
  hipStream_t st;
  std::vector<void*> ptrs;
  template <typename T>
  hipError_t alloc(T** out, size_t bytes) {
    const hipError_t e = hipMallocAsync(reinterpret_cast<void**>(out), bytes, st);
    if (e == hipSuccess) ptrs.push_back(*out);
    return e;
  }
  ~StreamScratch() {
    for (void* x : ptrs) (void)hipFreeAsync(x, st);
  }
};

}  // namespace

extern "C" {

int rt_launch_compute_image(rt_scene* sc, const rt_render_params* p, void* d_out, rt_stats* stats, void* stream) {
  return launch_render(sc, p, 1, &d_out, stats, stream, nullptr, nullptr, 0);
}

int rt_launch_frames(rt_scene* sc, const rt_render_params* p, int n_frames, void* const* d_outs, rt_stats* stats,
                     void* stream) {
  return launch_render(sc, p, n_frames, d_outs, stats, stream, nullptr, nullptr, 0);
}

namespace {
ShardRows shard_rows_of(const rt_render_params* p) {
  ShardRows G;
  G.W = p->camera.width;
  G.H = p->camera.height;
  G.rows = rt_rows_in_shard(p);
  G.stripe_count = p->stripe_count > 0 ? p->stripe_count : 1;
  G.stripe_h = p->stripe_height > 0 ? p->stripe_height : 1;
  G.stripe_index = p->stripe_index;
  G.row_begin = G.stripe_count == 1 ? std::max(0, p->row_begin) : 0;
  return G;
}
}  // namespace

int rt_adaptive_halo_rows(const rt_render_params* p, int* rows_out, int cap) {
  if (!p) return fail(RT_ERR_INVALID, "rt_adaptive_halo_rows: null params");
  const ShardRows G = shard_rows_of(p);
  const int nseg = G.segments();
  if (rows_out && cap < 2 * nseg) return fail(RT_ERR_INVALID, "rt_adaptive_halo_rows: buffer too small");
  for (int sgi = 0; rows_out && sgi < nseg; ++sgi) {
    const int l0 = G.stripe_count == 1 ? 0 : sgi * G.stripe_h;
    const int l1 = G.seg_last(l0);
    const int below = G.global_row(l0) - 1, above = G.global_row(l1) + 1;
    rows_out[2 * sgi] = below >= 0 ? below : -1;
    rows_out[2 * sgi + 1] = above < G.H ? above : -1;
  }
  return 2 * nseg;
}

int rt_launch_adaptive_shard(rt_scene* sc, const rt_render_params* p, const double* d_primary, const double* d_halo,
                             void* d_out, int subp, double threshold, rt_stats* stats, long long* n_selected,
                             void* stream) {
  if (!sc || !p || !d_primary || !d_out) return fail(RT_ERR_INVALID, "rt_launch_adaptive: null argument");
  if (subp < 1 || subp > 64) return fail(RT_ERR_INVALID, "rt_launch_adaptive: subp must be in [1, 64]");
  const int W = p->camera.width, H = p->camera.height;
  if (W <= 0 || H <= 0) return fail(RT_ERR_INVALID, "bad image size");
  if (p->out_format != RT_OUT_RGB_F32 && p->out_format != RT_OUT_RGB_F64) return fail(RT_ERR_INVALID, "bad out_format");
  const int scount = p->stripe_count > 0 ? p->stripe_count : 1;
  if (p->stripe_index < 0 || p->stripe_index >= scount) return fail(RT_ERR_INVALID, "stripe_index out of range");
  if (scount > 1 && (p->row_begin != 0 || (p->row_end > 0 && p->row_end != H)))
    return fail(RT_ERR_INVALID, "row ranges cannot be combined with stripe_count > 1");
  const ShardRows G = shard_rows_of(p);
  if (!d_halo) {   // only a shard whose segments border nothing but the frame edge may omit the halo
    std::vector<int> hr((size_t)std::max(1, 2 * G.segments()));
    rt_adaptive_halo_rows(p, hr.data(), (int)hr.size());
    for (int i = 0; i < 2 * G.segments(); ++i)
      if (hr[(size_t)i] >= 0) return fail(RT_ERR_INVALID, "rt_launch_adaptive_shard: this shard needs halo rows");
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(sc->device));
  uint32_t* list = nullptr;
  unsigned long long* cnt = nullptr;
  double* samples = nullptr;
  // interior pixels only can be selected
  const long long cap = (long long)std::max(0, W - 2) * G.rows;
  const int nsamp = subp * subp;
  StreamScratch scratch{st, {}};
  HIP_TRY(scratch.alloc(&list, (size_t)std::max(1LL, cap) * sizeof(uint32_t)));
  HIP_TRY(scratch.alloc(&cnt, sizeof(unsigned long long)));
  HIP_TRY(scratch.alloc(&samples, (size_t)std::max(1LL, cap) * nsamp * 3 * sizeof(double)));
  HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), st));
  const int tiles_x = (W + 7) / 8;
  const long long n_tiles = (long long)tiles_x * ((G.rows + 7) / 8);
  if (n_tiles > 0) {
    hipLaunchKernelGGL(adaptive_select_kernel, dim3((unsigned)((n_tiles + kSelTilesPerBlock - 1) / kSelTilesPerBlock)),
                       dim3(kSelThreads), 0, st, d_primary,
                       d_halo, d_out, p->out_format, G, threshold, tiles_x, n_tiles, list, cnt, 0u, nullptr, nullptr);
    HIP_TRY(hipGetLastError());
  }
  rt_render_params q = *p;
  q.spp_n = subp;
  int rc = launch_render(sc, &q, 1, &d_out, stats, stream, list, cnt, cap, samples);
  if (rc == RT_OK && cap > 0) {
    hipLaunchKernelGGL(adaptive_reduce_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, st, list, cnt,
                       samples, nsamp, d_out, p->out_format, nullptr);
    HIP_TRY(hipGetLastError());
  }
  if (rc == RT_OK && n_selected) {
    unsigned long long h = 0;
    HIP_TRY(hipMemcpyAsync(&h, cnt, sizeof h, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *n_selected = (long long)h;
  }
  return rc;
}

int rt_launch_adaptive(rt_scene* sc, const rt_render_params* p, const double* d_primary, void* d_out, int subp,
                       double threshold, rt_stats* stats, long long* n_selected, void* stream) {
  if (!p) return fail(RT_ERR_INVALID, "rt_launch_adaptive: null argument");
  const int H = p->camera.height;
  if ((p->stripe_count > 1) || p->row_begin != 0 || (p->row_end > 0 && p->row_end != H))
    return fail(RT_ERR_INVALID, "rt_launch_adaptive: needs the full frame (neighbour test), no stripes/row range");
  return rt_launch_adaptive_shard(sc, p, d_primary, nullptr, d_out, subp, threshold, stats, n_selected, stream);
}

int rt_launch_adaptive_frames(rt_scene* sc, const rt_render_params* p, int n_frames, const double* const* d_primary,
                              void* const* d_out, int subp, double threshold, rt_stats* stats, long long* n_selected,
                              void* stream) {
  if (!sc || !p || !d_primary || !d_out) return fail(RT_ERR_INVALID, "rt_launch_adaptive_frames: null argument");
  if (n_frames < 1 || n_frames > kMaxFrames) return fail(RT_ERR_INVALID, "rt_launch_adaptive_frames: n_frames out of range");
  if (subp < 1 || subp > 64) return fail(RT_ERR_INVALID, "rt_launch_adaptive_frames: subp must be in [1, 64]");
  if (n_frames == 1)
    return rt_launch_adaptive(sc, p, d_primary[0], d_out[0], subp, threshold, stats, n_selected, stream);
  const int W = p->camera.width, H = p->camera.height;
  if (W <= 0 || H <= 0) return fail(RT_ERR_INVALID, "bad image size");
  if ((long long)W * H > (long long)kListPixMask) return fail(RT_ERR_INVALID, "rt_launch_adaptive_frames: frame too large");
  if (p->out_format != RT_OUT_RGB_F32 && p->out_format != RT_OUT_RGB_F64) return fail(RT_ERR_INVALID, "bad out_format");
  if ((p->stripe_count > 1) || p->row_begin != 0 || (p->row_end > 0 && p->row_end != H))
    return fail(RT_ERR_INVALID, "rt_launch_adaptive_frames: needs full frames (neighbour test), no stripes/row range");
  for (int f = 0; f < n_frames; ++f)
    if (!d_primary[f] || !d_out[f]) return fail(RT_ERR_INVALID, "rt_launch_adaptive_frames: null frame buffer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipSetDevice(sc->device));
  const ShardRows G = shard_rows_of(p);
  const long long per = (long long)std::max(0, W - 2) * G.rows;   // interior pixels only can be selected
  const long long cap = per * n_frames;
  uint32_t* list = nullptr;
  unsigned long long* cnt = nullptr;
  StreamScratch scratch{st, {}};
  HIP_TRY(scratch.alloc(&list, (size_t)std::max(1LL, cap) * sizeof(uint32_t)));
  HIP_TRY(scratch.alloc(&cnt, sizeof(unsigned long long)));
  HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), st));
  const int tiles_x = (W + 7) / 8;
  const long long n_tiles = (long long)tiles_x * ((G.rows + 7) / 8);
  // every frame's selection into one list, one launch (grid y = frame; the frame buffers'
  // pointers travel in a small device table)
  std::vector<const void*> ptrs(2 * (size_t)n_frames);
  for (int f = 0; f < n_frames; ++f) {
    ptrs[f] = d_primary[f];
    ptrs[n_frames + f] = d_out[f];
  }
  void** d_ptrs = nullptr;
  HIP_TRY(scratch.alloc(&d_ptrs, ptrs.size() * sizeof(void*)));
  HIP_TRY(hipMemcpyAsync(d_ptrs, ptrs.data(), ptrs.size() * sizeof(void*), hipMemcpyHostToDevice, st));
  if (n_tiles > 0) {
    hipLaunchKernelGGL(adaptive_select_kernel,
                       dim3((unsigned)((n_tiles + kSelTilesPerBlock - 1) / kSelTilesPerBlock), (unsigned)n_frames),
                       dim3(kSelThreads), 0, st, nullptr, nullptr, nullptr, p->out_format, G, threshold, tiles_x,
                       n_tiles, list, cnt, 0u, reinterpret_cast<const double* const*>(d_ptrs), d_ptrs + n_frames);
    HIP_TRY(hipGetLastError());
  }
  // every sample of every selected pixel of every frame in one launch: the sample buffer is sized
  // by the selection count (read back: one synchronisation per batch)
  unsigned long long n_sel = 0;
  HIP_TRY(hipMemcpyAsync(&n_sel, cnt, sizeof n_sel, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const int nsamp = subp * subp;
  double* samples = nullptr;
  HIP_TRY(scratch.alloc(&samples, (size_t)std::max(1ull, n_sel) * nsamp * 3 * sizeof(double)));
  std::vector<rt_render_params> q(p, p + n_frames);
  for (auto& x : q) x.spp_n = subp;
  int rc = launch_render(sc, q.data(), n_frames, d_out, stats, stream, list, cnt, (long long)n_sel, samples);
  if (rc == RT_OK && n_sel > 0) {   // sums in (si, sj) order into each frame's output (that launch's frame table)
    const FrameDesc* table = reinterpret_cast<const FrameDesc*>(
        reinterpret_cast<const unsigned char*>(sc->ctx[sc->last_ctx].d_ctr) + kCtrBytes);
    hipLaunchKernelGGL(adaptive_reduce_kernel, dim3((unsigned)((n_sel + 255) / 256)), dim3(256), 0, st, list, cnt,
                       samples, nsamp, nullptr, p->out_format, table);
    HIP_TRY(hipGetLastError());
  }
  if (n_selected) *n_selected = (long long)n_sel;
  return rc;
}

int rt_render_to_host(rt_scene* sc, const rt_render_params* p, void* host_out, rt_stats* stats) {
  if (!sc || !p || !host_out) return fail(RT_ERR_INVALID, "rt_render_to_host: null argument");
  HIP_TRY(hipSetDevice(sc->device));
  const int rows = rt_rows_in_shard(p);
  const size_t elem = p->out_format == RT_OUT_RGB_F64 ? sizeof(double) : sizeof(float);
  const size_t bytes = std::max<size_t>(1, (size_t)rows * p->camera.width * 3 * elem);
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, bytes));
  rt_stats local;
  int rc = rt_launch_compute_image(sc, p, d, stats ? stats : &local, nullptr);
  if (rc == RT_OK) {
    const hipError_t e = hipMemcpy(host_out, d, (size_t)rows * p->camera.width * 3 * elem, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(RT_ERR_HIP, std::string("hipMemcpy D2H: ") + hipGetErrorString(e));
  }
  (void)hipFree(d);
  return rc;
}

int rt_debug_counters(rt_scene* sc, unsigned long long* out, int n) {
  if (!sc || !out || n <= 0) return fail(RT_ERR_INVALID, "rt_debug_counters: bad argument");
  HIP_TRY(hipSetDevice(sc->device));
  HIP_TRY(hipDeviceSynchronize());
  unsigned long long c[kCtrWords];
  if (sc->last_ctx < 0) return fail(RT_ERR_INVALID, "rt_debug_counters: no launch recorded");
  const int rc = read_counters(sc->ctx[sc->last_ctx], c);
  if (rc != RT_OK) return rc;
  for (int i = 0; i < n && i < kCtrWords; ++i) out[i] = c[i];
  return std::min(n, kCtrWords);
}

int rt_debug_blocks_per_cu(rt_scene* sc, int variant) {
  if (!sc || variant < 0 || variant >= kNumVariants) return fail(RT_ERR_INVALID, "rt_debug_blocks_per_cu: bad argument");
  return sc->blocks_per_cu[variant];
}

long long rt_debug_timeline(rt_scene* sc, unsigned long long* out, long long n) {
  if (!sc || !out || n <= 0) return fail(RT_ERR_INVALID, "rt_debug_timeline: bad argument");
  HIP_TRY(hipSetDevice(sc->device));
  HIP_TRY(hipDeviceSynchronize());
  if (sc->last_ctx < 0 || !sc->ctx[sc->last_ctx].d_tl)
    return fail(RT_ERR_INVALID, "rt_debug_timeline: the last launch was not an RT_FLAG_TIMELINE launch");
  const long long words = std::min<long long>(n, (long long)(sc->nslots / 64 * kTlCap * kTlWords));
  HIP_TRY(hipMemcpy(out, sc->ctx[sc->last_ctx].d_tl, (size_t)words * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return words;
}

long long rt_debug_wave_log(rt_scene* sc, unsigned long long* out, long long n) {
  if (!sc || !out || n <= 0) return fail(RT_ERR_INVALID, "rt_debug_wave_log: bad argument");
  HIP_TRY(hipSetDevice(sc->device));
  HIP_TRY(hipDeviceSynchronize());
  const long long words = std::min<long long>(n, (long long)(sc->nslots / 64 * 4));
  if (sc->last_ctx < 0) return fail(RT_ERR_INVALID, "rt_debug_wave_log: no launch recorded");
  HIP_TRY(hipMemcpy(out, sc->ctx[sc->last_ctx].d_wavelog, (size_t)words * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost));
  return words;
}

int rt_last_kernel_ms(rt_scene* sc, float* ms) {
  if (!sc || !ms || sc->last_ctx < 0) return fail(RT_ERR_INVALID, "rt_last_kernel_ms: no launch recorded");
  const LaunchCtx& C = sc->ctx[sc->last_ctx];
  HIP_TRY(hipEventSynchronize(C.ev1));
  HIP_TRY(hipEventElapsedTime(ms, C.ev0, C.ev1));
  return RT_OK;
}

int rt_scene_set_analytic(rt_scene* sc, const rt_sphere* spheres, int n_spheres, const rt_plane* planes,
                          int n_planes) {
  if (!sc) return fail(RT_ERR_INVALID, "rt_scene_set_analytic: null scene");
  if (n_spheres < 0 || n_planes < 0 || (n_spheres > 0 && !spheres) || (n_planes > 0 && !planes))
    return fail(RT_ERR_INVALID, "rt_scene_set_analytic: bad primitive arrays");
  const long long n = (long long)n_spheres + n_planes;
  if (n > (1 << 20)) return fail(RT_ERR_INVALID, "rt_scene_set_analytic: more than 2^20 primitives");
  std::vector<GMat> mats = sc->mesh_mats;
  std::vector<GPrim> prims((size_t)n);
  auto add_mat = [&](const rt_material& m) {
    GMat G;
    std::memset(&G, 0, sizeof G);
    for (int k = 0; k < 3; ++k) {
      G.ka[k] = m.ambient[k];
      G.kd[k] = m.diffuse[k];
      G.ks[k] = m.specular[k];
    }
    G.shininess = m.shininess;
    G.mirror = m.mirror;
    G.shadowable = m.shadowable;
    G.draw_mode = RT_DRAW_FLAT;
    G.tex_w = -1;
    mats.push_back(G);
    return (int)mats.size() - 1;
  };
  for (int i = 0; i < n_spheres; ++i) {
    GPrim& G = prims[i];
    std::memset(&G, 0, sizeof G);
    for (int k = 0; k < 3; ++k) G.c[k] = spheres[i].center[k];
    G.r = spheres[i].radius;
    G.type = kPrimSphere;
    G.mat = add_mat(spheres[i].material);
  }
  for (int i = 0; i < n_planes; ++i) {
    GPrim& G = prims[(size_t)n_spheres + i];
    std::memset(&G, 0, sizeof G);
    for (int k = 0; k < 3; ++k) {
      G.c[k] = planes[i].center[k];
      G.n[k] = planes[i].normal[k];
    }
    G.type = kPrimPlane;
    G.mat = add_mat(planes[i].material);
  }
  HIP_TRY(hipSetDevice(sc->device));
  HIP_TRY(hipDeviceSynchronize());   // launches in flight read the old tables
  long long bytes = 0;
  GMat* d_mats = nullptr;
  GPrim* d_prims = nullptr;
  int rc = upload(&d_mats, mats, bytes);
  if (rc == RT_OK) rc = upload(&d_prims, prims, bytes);
  if (rc != RT_OK) {
    if (d_mats) (void)hipFree(d_mats);
    if (d_prims) (void)hipFree(d_prims);
    return rc;
  }
  if (sc->d_mats) (void)hipFree(sc->d_mats);
  if (sc->d_prims) (void)hipFree(sc->d_prims);
  sc->d_mats = d_mats;
  sc->d_prims = d_prims;
  sc->n_prims = (int)n;
  sc->bytes += bytes - sc->table_bytes;
  sc->table_bytes = bytes;
  return RT_OK;
}

void rt_scene_free(rt_scene* sc) {
  if (!sc) return;
  (void)hipSetDevice(sc->device);
  (void)hipDeviceSynchronize();   // launches may still be reading the scene
  void* ptrs[] = {sc->d_nodes, sc->d_nodes4, sc->d_tris, sc->d_shade, sc->d_tnorm, sc->d_tu,
                  sc->d_tv, sc->d_texels, sc->d_mats, sc->d_lights, sc->d_slot2dev, sc->d_prims};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  for (LaunchCtx& c : sc->ctx) {
    void* cp[] = {c.d_ctr, c.d_pstate, c.d_spill, c.d_wavelog, c.d_tl, c.d_wctr};
    for (void* q : cp)
      if (q) (void)hipFree(q);
    if (c.h_ctl) (void)hipHostFree(c.h_ctl);
    if (c.ev0) (void)hipEventDestroy(c.ev0);
    if (c.ev1) (void)hipEventDestroy(c.ev1);
  }
  delete sc;
}

}  // extern "C"
