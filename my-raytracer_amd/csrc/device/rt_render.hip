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
#include <hip/hip_ext.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <rocprim/block/block_radix_sort.hpp>

#include "../../../include/rt_hip.h"
#include "../host/device_image.hpp"
#include "rt_layout.hpp"

#pragma clang fp contract(off)

using namespace rtk;

namespace {

constexpr int kBlock = 256;        // threads per persistent block
constexpr int kGroups = 8;          // work heads (XCD groups)
#ifndef RT_REFILL
#define RT_REFILL 16
#endif
constexpr int kRefill = RT_REFILL;  // refill a wave when this many lanes are idle (8 / 32: -1.1 / -1.0 %, r06y)
constexpr int kCtrWords = 40;       // [8,16) stats (STATS variants), [16,40) diagnostics (31: guard)
// Traversal stack: the top kShortStack entries live in an LDS ring (slot i & kStackMask),
// deeper entries spill to a per-lane global array.  Bounds LDS per block independently
// of tree depth, so occupancy stays VGPR-limited.
constexpr int kShortStack = 8;
// Top treelet in LDS: the first kTopNodes 4-wide nodes (breadth-first numbering) are copied
// into each block's LDS; a node iteration whose active lanes all sit in the treelet reads
// LDS instead of the vector-L1 path.  0 disables.
// LDS per thread: kSlotDoubles fp64 slot words, task + visibility words, the stack ring
constexpr int kSlotDoubles = 10;
// fills the CU's 160 KB at 4 blocks with the slots, ring, lights, pool (73 nodes)
constexpr int kTopNodes = (40960 - kBlock * (kSlotDoubles * 8 + (2 + kShortStack) * 4) - RT_MAX_LIGHTS * 48 - 64) / 128;
constexpr int kStackMask = kShortStack - 1;
// Tail compaction: once the work queue is empty, a wave with at most kDonateMax
// pixels in flight hands them to the other waves of its block and exits, so the last pixels
// of a launch run in fewer, fuller waves.  A handed-over lane's registers travel through the
// donor thread's LDS stack entries (free between traversals): kMigWords words (packed; the
// closest-hit distance and the hit attributes travel in the LDS slot, copied with it).
#ifndef RT_DONATE_MAX
#define RT_DONATE_MAX 24
#endif
constexpr int kDonateMax = RT_DONATE_MAX;   // (0 = tail compaction off: -2.8 % batched, -1.4 % one frame;
                                            //  16 / 32 / 40: within noise, r06zr/r06zs)
constexpr int kMigWords = 8;
static_assert(kMigWords <= kShortStack, "migration words travel in the stack ring entries");
constexpr int kPoolBytes = 64;   // LDS: live-wave count, one 64-bit lane mask per wave of the block, exhausted heads
static_assert(8 + 8 * (kBlock / 64) + 4 <= kPoolBytes, "compaction pool does not fit");
static_assert((kShortStack & kStackMask) == 0, "the stack ring must be a power of two");

// Lane states.  Owners carry a pixel (CLOSEST: closest-hit ray in flight; SHADOW: a
// batch of shadow rays in flight).  Idle lanes (FETCH / DONE) may be lent to an
// owner of the same wave for one round (HSHADOW / HCLOSEST): they trace one of its
// extra shadow rays or its reflection ray, so a bounce costs one round, not 1 + lights.
// PARKED (sample groups, spp > 1): the lane's sample is finished and its colour waits in the lane's
// slot for its group's ordered sum (below); a parked lane is neither busy nor idle.
// a tile's pixels claimed in Morton order (RT_TILE_ROW_ORDER: row order): a partial refill's run of
// items, or the 2-4 pixels of a wave's sample groups, is a compact block instead of a strip of rows
// (r06t: configs 3 / 5 +0.4 %; r06u: office +0.5 %, config 4 +0.8 %)
#ifdef RT_TILE_ROW_ORDER
constexpr bool kTileMorton = false;
#else
constexpr bool kTileMorton = true;
#endif
enum : int { ST_FETCH = 0, ST_CLOSEST = 1, ST_SHADOW = 2, ST_DONE = 3, ST_PARKED = 4, ST_HSHADOW = 5, ST_HCLOSEST = 6 };
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
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
struct D2 {
  double a, b;
};
__device__ __forceinline__ D2 buf_ld2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return D2{__builtin_bit_cast(double, u32x2_t{v.x, v.y}), __builtin_bit_cast(double, u32x2_t{v.z, v.w})};
}
// (no b128 store helper: path-state stores are b64, see ST4 in render_kernel)


// Inclusive prefix sum over the wave's 64 lanes (all lanes active).  (A DPP row-shift / broadcast scan
// measured +-0.5 %: not kept.)
__device__ __forceinline__ int wave_incl_scan(int x) {
  int incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if ((int)(threadIdx.x & 63) >= o) incl += v;
  }
  return incl;
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
  CD_GNODE_UNIFORM = 32, CD_GNODE_DISTINCT, CD_LEAF_UNIFORM, CD_ANYHIT_TRIS, CD_OWN_TRIS,
  CT_ORDER_JOBS = 39   // cost-ordered launches: order / zeroing jobs claimed by blocks that finished
};
// Watchdogs (never reached by a correct kernel): the persistent loop, and the wave-level
// iterations of one traversal round (round, node and leaf loops together).  A wave that
// trips either ends its work instead of spinning and flags the launch (CD_GUARD), which
// the host reports as an error.
constexpr unsigned kGuardIters = 1u << 24;
constexpr unsigned kTravGuard = 1u << 24;
// A watchdog fired: the launch's counter word (stats launches) and the scene's host-mapped word,
// written with a vector store and released at system scope, so the host sees it after launches
// without stats too (rt_scene_status).  One lane of the wave calls it.
__device__ __forceinline__ void trip_watchdog(unsigned long long* ctr, unsigned int* host_word) {
  atomicOr(&ctr[CD_GUARD], 1ull);
  __builtin_nontemporal_store(1u, host_word);
  __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
constexpr int kTlCap = 256;   // TL variant: traversal rounds recorded per wave
constexpr int kTlWords = 8;   // ... and words per round

// Division of 32-bit n < 2^31 by a launch-invariant d >= 1 as mulhi(n, m) >> s (Granlund-Montgomery;
// m, s chosen on the host so that the quotient is exact for every n < 2^31): 2 VALU instead of
// the ~20 of a 32-bit (or the SALU/VALU mix of a 64-bit) division in the refill's tile decode.
struct DivMagic {
  uint32_t m, s;
  __host__ __device__ uint32_t div(uint32_t n) const {   // m == 0: d == 1 (m would need 33 bits)
#ifdef __HIP_DEVICE_COMPILE__
    return m ? __umulhi(n, m) >> s : n;
#else
    return m ? (uint32_t)(((unsigned long long)n * m) >> 32) >> s : n;
#endif
  }
};
inline DivMagic div_magic(uint32_t d) {
  // smallest s with m = ceil(2^(32+s) / d) < 2^32 and error e = m d - 2^(32+s) < 2^(s+1), which makes
  // floor(n m / 2^(32+s)) = floor(n / d) for all n < 2^31 (e n < 2^(32+s))
  for (uint32_t s = 0; s < 32; ++s) {
    const unsigned __int128 p = (unsigned __int128)1 << (32 + s);
    const unsigned __int128 m = (p + d - 1) / d;
    if (m >> 32) continue;
    const unsigned __int128 e = m * d - p;
    if ((e << 31) < p) return DivMagic{(uint32_t)m, s};
  }
  return DivMagic{0u, 0u};   // unreachable for d >= 1
}
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
  double* pstate;       // path state, [nslots / 64][kRegions][64 lanes][4] fp64
  uint32_t* spill;      // [stack_words][nslots] traversal-stack entries below the LDS ring
  unsigned long long* wavelog;  // STATS: per wave {start, last refill, end, pixels} (s_memrealtime)
  unsigned long long* tl;       // TL: per wave and traversal round {start, end, lanes, iterations}
  const double* lights; // [n_lights][6] position xyz, colour rgb (this launch's control block)
  unsigned int* guard_host;   // the scene's watchdog word in page-locked host memory (trip_watchdog)
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
  // sample groups (spp > 1, rt_upload_options.spp_lanes): a pixel's samples run on G = 2^group_log
  // neighbouring lanes of one wave, `chunks` x G samples in all (0: one lane per pixel, its samples in
  // sequence)
  int group_log, chunks;
  int row_begin, stripe_h, stripe_count, stripe_index;
  int rows;
  int tiles_x;
  int out_global;           // RT_FLAG_GLOBAL_ROWS: pixels go to their global row of a whole-frame buffer
  int order_dilate;         // cost-ordered launches: cost window half-width along a tile row (order_range)
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
  // tile order (RT_FLAG_COST_ORDER): work item w belongs to linear tile tile_order[w / 64] instead of
  // w / 64 (a permutation within each work head's range); tile_cost[ty * tiles_x + tx] accumulates
  // the cost of the tile position's finished samples over the launch's frames (the next order)
  const uint32_t* tile_order;
  uint32_t* tile_cost;
  int cost_time;            // tile_cost in 10-ns ticks of pixel lifetime instead of bounces
  DivMagic div_row_tiles, div_tiles_x, div_stripe_h;   // n / (frames x tiles_x), n / tiles_x, n / stripe_h
  // cost-ordered launches: blocks whose work is done (the launch's drain, when CUs idle) build the
  // order of a later launch from a complete cost map and zero the map that launch will fill
  const uint32_t* order_src;   // complete per-position cost map (an earlier launch's)
  uint32_t* next_order;        // its tile order, for the launch after this one
  uint32_t* zero_map;          // cost map to clear for the launch after this one
  long long n_pos;             // tile positions (= tiles of a one-frame launch)
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
// normalize: the same sqrt, then x / n for each component -- with ONE refined reciprocal of n for
// the three divisions.  The compiler's correctly rounded fp64 division is
//   d0 = div_scale(n), r = rcp(d0), r = fma(r, fma(-d0, r, 1), r) twice, q = d1 * r,
//   q = div_fmas(fma(-d0, q, d1), r, q), div_fixup(q, n, x)
// and div_scale / div_fixup are identities when no operand is zero, denormal or near an exponent
// limit and the quotient cannot over- or underflow: here every |component| in [2^-200, 2^200]
// (so n in [2^-200, 2^201]).  Inside that range this is the same sequence of operations on the same
// operands with the reciprocal steps done once, so the result is bit-identical to normalize;
// outside it (a zero component included) normalize runs.  n = |v| is returned too (the shadow ray's
// light distance is that same sqrt).  (Production variants only: in the diagnostic ones the extra
// live ranges spill.)
// sqrt of q >= 2^-767, finite: the compiler's fp64 sqrt expansion is "scale q up by 2^256 if below
// 2^-767, v_rsq_f64 + two Newton refinements, scale back, return q itself for +-0 / +inf"; for such
// q the scaling and the fix-up are identities, and this is the rest of it -- the same operations in
// the same order, bit-identical to sqrt(q).
__device__ __forceinline__ double sqrt_normal(double q) {
  const double y = __builtin_amdgcn_rsq(q);
  double g = q * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  double d = __builtin_fma(-g, g, q);
  h = __builtin_fma(h, r, h);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, q);
  return __builtin_fma(d, h, g);
}
// the refined reciprocal of the compiler's fp64 division x / n (see above), and one quotient with it
__device__ __forceinline__ double rcp_refined(double n) {
  double r = __builtin_amdgcn_rcp(n);
  r = __builtin_fma(r, __builtin_fma(-n, r, 1.0), r);
  return __builtin_fma(r, __builtin_fma(-n, r, 1.0), r);
}
__device__ __forceinline__ double div_by(double x, double n, double r) {
  const double q = x * r;
  return __builtin_fma(__builtin_fma(-n, q, x), r, q);
}
// |x| in [2^-300, 2^300]: quotients of two such values need neither div_scale nor div_fixup
__device__ __forceinline__ D3 normalize_rcp(D3 v, double& n) {
  // every |component| >= 2^-200 and |v|^2 <= 2^400 (so every |component| <= 2^200); NaN / inf fail
  const double q = dot(v, v);
  const bool ok = fabs(v.x) >= 0x1p-200 && fabs(v.y) >= 0x1p-200 && fabs(v.z) >= 0x1p-200 &&
                  q <= 0x1p400;
  if (!ok) {
    n = sqrt(q);
    return normalize(v);
  }
  n = sqrt_normal(q);
  const double r = rcp_refined(n);
  return D3{div_by(v.x, n, r), div_by(v.y, n, r), div_by(v.z, n, r)};
}
// Shading-only helpers for the specular term (never a ray, never a branch that switches a term on or
// off): results within a few ulp of the reference's sqrt-and-divide normalisation and libm pow --
// far inside the fp64 parity tolerance (1e-12), while everything that defines a ray (camera, shadow
// and reflection directions, the triangle test) or decides a branch keeps the reference's exact
// operations.
// normalize: v_rsq_f64 + one Newton step and three multiplies instead of a sqrt and three divisions.
__device__ __forceinline__ D3 normalize_shade(D3 v) {
  const double q = dot(v, v);
  if (!(q > 1e-200 && q < 1e200)) return normalize(v);   // zero, tiny, huge or NaN: the exact path
  const double r0 = __builtin_amdgcn_rsq(q);
  const double e = __builtin_fma(-(q * r0), r0, 1.0);   // 1 - q r0^2
  const double r = __builtin_fma(0.5 * r0, e, r0);
  return D3{v.x * r, v.y * r, v.z * r};
}
// pow for the Phong highlight: integer exponents 1 .. 256 (the usual material exponents) by binary
// powering (relative error below 2^8 ulp for x in [0, 1]), others through pow.
__device__ __forceinline__ double pow_shade(double x, double y) {
  if (y >= 1.0 && y <= 256.0 && y == __builtin_floor(y)) {
    uint32_t n = (uint32_t)y;
    double r = 1.0, b = x;
    for (;;) {
      if (n & 1u) r *= b;
      n >>= 1;
      if (n == 0u) break;
      b *= b;
    }
    return r;
  }
  return pow(x, y);
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
// wave ballot of a per-lane predicate (a ballot of a single compare is its mask; of a combined
// predicate the backend re-materialises it with a v_cndmask + v_cmp pair, so hot loops OR / AND
// the ballots of the single compares instead)
__device__ __forceinline__ unsigned long long wballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
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
  const unsigned long long m = wballot(1);
  if (lane == __ffsll((long long)m) - 1) { iters++; lanes += __popcll(m); }
}

// Adds the number of distinct keys among the active lanes (wave-uniform loop) on the
// first active lane: distinct lines one load instruction touches, the L1 tag rate's unit.
__device__ __forceinline__ void wave_distinct(uint32_t key, unsigned long long& acc, int lane) {
  unsigned long long m = wballot(1);
  const int first = __ffsll((long long)m) - 1;
  unsigned n = 0;
  while (m) {
    const uint32_t k = __shfl(key, __ffsll((long long)m) - 1);
    m &= ~wballot(key == k);
    n++;
  }
  if (lane == first) acc += n;
}

// global row of local (packed) row lrow of a striped shard: (lrow / h) * count + index stripes of h rows
__device__ __forceinline__ int stripe_row(const KParams& P, int lrow) {
  const uint32_t st = P.div_stripe_h.div((uint32_t)lrow);
  return (int)((st * (uint32_t)P.stripe_count + (uint32_t)P.stripe_index) * (uint32_t)P.stripe_h +
               ((uint32_t)lrow - st * (uint32_t)P.stripe_h));
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

// Work tiles: one wave's 64 pixels, kTileW x kTileH, 8 x 8 (the most coherent primary rays); the
// unit is also the grain of the cost order (rt_debug_tile_cost and friends).  A tile row of fp32
// RGB is a 96-B segment, which straddles the image's 64-B HBM write units: the office's 24.9 MB
// image costs 36.2 MB of HBM writes per frame.  16 x 4 tiles (192-B segments, whole units) cut that
// to 28.9 MB but cost 2.9 % batched / 3.9 % one frame, 32 x 2 cost 9 % (profiles/r05/r05g_*).
#ifndef RT_TILE_W
#define RT_TILE_W 8
#endif
constexpr int kTileW = RT_TILE_W, kTileH = 64 / RT_TILE_W;
constexpr int kTileWLog = kTileW == 8 ? 3 : kTileW == 16 ? 4 : kTileW == 32 ? 5 : -1;
constexpr int kTileHLog = 6 - kTileWLog;
static_assert(kTileWLog > 0 && kTileW * kTileH == 64, "a tile is one wave's 64 pixels (8, 16 or 32 wide)");

// Path state kept in global memory between a lane's rays: per wave kRegions regions of
// [64 lanes][4 fp64], so a lane's record of a region is ONE 32-B sector, read with two b128 and
// written with four b64 buffer accesses at the lane offset (one VGPR) plus the region's offset
// (an SGPR constant).  A lane's store dirties whole sectors: the L2 writes back 32 B per lane
// and region instead of four partly written 32-B sectors of four field-major arrays (round 2:
// 13 field-major fp64 arrays, HBM writes 56.6 MB per office frame against a 24.9 MB image;
// DESIGN.md §4 "path state").  Only what cannot be recomputed or kept in the LDS slot:
//   the sample's colour and weight across mirror bounces (R_SCOLW: SCOL xyz, W);
//   the pixel's sum across samples (R_PCOL, spp > 1);
//   the textured diffuse colour (R_HD; untextured hits re-read the material's kd);
//   the light sum across shadow batches of more than 32 lights (R_LACC; a bounce whose lights
//     fit one batch restarts from the recomputed ambient term).
// The mirror coefficient comes from the material (the lane keeps the mesh id); the normal of
// the bounce being shaded lives in the slot's aux words (below).
enum : int { R_SCOLW = 0, R_PCOL = 1, R_HD = 2, R_LACC = 3, kRegions = 4 };
constexpr uint32_t kLaneRec = 32;                 // bytes per lane and region
constexpr uint32_t kRegionBytes = 64 * kLaneRec;  // 2 KB per wave and region

// LDS slots ([field][thread], conflict-free): the ray (the only hand-over between the
// shading phase, which writes the next ray, and the traversal phase, which reads it) and
// three aux words, time-shared:
//   closest-hit ray in flight: the accepted hit's barycentrics alpha, beta and its mesh id,
//     written by the leaf test when it accepts a hit, so shading reads them instead of
//     re-loading the triangle record and recomputing the determinants (same operands, same
//     operations: bit-identical);
//   shadow batch in flight: the hit normal HN of the bounce being shaded.
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


// 4 waves/SIMD = 16 waves/CU (register budget 128 VGPRs); measurement builds may ask for 5
// (make variant V="-DRT_WAVES_PER_EU=5": 96 VGPRs, spills; 5 blocks per CU also need <= 32 KB of LDS:
// upload option lds_treelet=9)
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 4
#endif
constexpr int kWavesPerEU = RT_WAVES_PER_EU;

// RING: entries of the per-lane traversal-stack ring in LDS (8: room for the 73-node treelet;
// 16: deep hierarchies, e.g. millions of random triangles, which spill an 8-entry ring often;
// the treelet then gets what is left, 9 nodes -- rt_scene picks per scene)
// ---------------------------------------------------------------------------
// Cost-ordered work (RT_FLAG_COST_ORDER, one-frame launches): each work head's range of tiles
// [n h / 8, n (h + 1) / 8) is reordered so its expensive tiles come first, by the cost its tile
// position had in the previous ordered launch (pixel lifetimes, 10-ns ticks).  A one-frame
// launch's drain -- waves finishing the paths they started just before the queue ran dry -- is
// then made of cheap tiles (office 1080p: kernel -11 %, HISTORY.md §4; DESIGN.md §4
// "cost-ordered tiles").  The order is built inside the render kernel by its first blocks to run
// out of work, from the cost map of the launch before, so it costs no launch and no busy CU.
constexpr int kOrderItems = 16;
constexpr int kOrderDilate = 4;   // tiles (A/B: 2 / 4 / 8 along the row; 2-D windows slower, r04v)
constexpr long long kOrderMaxRange = (long long)kBlock * kOrderItems;   // tiles per head range (4096)
// Sort keys: a log-scale cost class (4 per octave from 2^8 ticks; 16 per octave: -1.5 %, 1 per
// octave: +-0, profiles/r03/r03u_ab_order_*.txt) inverted so that higher costs sort first, above the
// 12-bit local index; one radix pass over the 8 class bits (stable: equal classes keep band order).
constexpr int kOrderShift = 21;   // cost classes per octave: 2^(23 - kOrderShift)
__device__ __forceinline__ uint32_t order_class(uint32_t cost) {
  const int q = (int)(__float_as_uint((float)cost) >> kOrderShift) - ((127 + 8) << (23 - kOrderShift));
  return 255u - (uint32_t)min(255, max(0, q));
}
// dilate > 0: a tile's sort cost is the largest cost within +-dilate tiles of its tile row.  The
// order then follows the expensive regions rather than single expensive tiles, which keeps the
// costliest paths first when the camera moved since the costs were recorded (the frame two
// launches back) and keeps neighbouring tiles together (stable sort): office 1080p one frame
// -9 % (same view) / -13 % (driver-shape animation); random-triangle soups lose by it (-4 %),
// so deep hierarchies keep the exact costs (DESIGN.md §4 "cost-ordered tiles")
__device__ void order_range(const uint32_t* cost, uint32_t* order, long long n_tiles, int h, unsigned char* lds,
                            int tiles_x, int dilate) {
  using Sort = rocprim::block_radix_sort<unsigned int, kBlock, kOrderItems>;
  static_assert(sizeof(typename Sort::storage_type) <= 30720, "sort storage must fit the block's LDS (at least 30 KB)");
  auto& storage = *reinterpret_cast<typename Sort::storage_type*>(lds);
  const long long t0 = n_tiles * h / kGroups, t1 = n_tiles * (h + 1) / kGroups;
  unsigned int keys[kOrderItems];
#pragma unroll
  for (int j = 0; j < kOrderItems; ++j) {
    const long long li = (long long)threadIdx.x * kOrderItems + j;   // local index in the range
    uint32_t c = 0u;
    if (t0 + li < t1) {
      const long long t = t0 + li, row = t / tiles_x, col = t - row * tiles_x;
      const long long x0 = max(0LL, col - dilate), x1 = min((long long)tiles_x - 1, col + dilate);
      for (long long x = x0; x <= x1; ++x) c = max(c, cost[row * tiles_x + x]);
    }
    keys[j] = t0 + li < t1 ? (order_class(c) << 12) | (uint32_t)li : 0xffffffffu;   // padding last
  }
  Sort().sort(keys, storage, 12, 20);
#pragma unroll
  for (int j = 0; j < kOrderItems; ++j) {
    const long long pos = (long long)threadIdx.x * kOrderItems + j;
    if (t0 + pos < t1) order[t0 + pos] = (uint32_t)(t0 + (keys[j] & 0xfffu));
  }
}

template <int WIDTH, bool STATS, bool TL = false, int RING = kShortStack, bool GRP = false>
__global__ void __launch_bounds__(kBlock, kWavesPerEU * 256 / kBlock) render_kernel(KParams P) {
  static_assert(RING >= kMigWords && (RING & (RING - 1)) == 0, "ring: a power of two holding the migration words");
  constexpr int kRingMask = RING - 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  // LDS: [stack ring: RING rows of kBlock words][slots: kSlotDoubles x kBlock doubles][task words]
  // [visibility words][treelet][lights][pool] -- the ring at address 0 (below)
  constexpr uint32_t kRingRegion = (uint32_t)RING * kBlock * sizeof(uint32_t);
  unsigned char* const lds_s = lds_raw + kRingRegion;
  double* lds_d = reinterpret_cast<double*>(lds_s);
  RaySlots R;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    R.o[k] = lds_d + k * kBlock + threadIdx.x;
    R.d[k] = lds_d + (3 + k) * kBlock + threadIdx.x;
  }
  R.tlim = lds_d + 6 * kBlock + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 3; ++k) R.a[k] = lds_d + (7 + k) * kBlock + threadIdx.x;
  uint32_t* ltask = reinterpret_cast<uint32_t*>(lds_s + kSlotDoubles * kBlock * sizeof(double));   // [kBlock]
  uint32_t* lvis = ltask + kBlock;                                                             // [kBlock]
  uint32_t* stk = reinterpret_cast<uint32_t*>(lds_raw) + threadIdx.x;
  // the ring as plain LDS byte addresses: the render kernels have no static LDS, so the dynamic
  // block, and the ring with it, starts at LDS address 0; this lane's byte offset within a ring row
  // sits below the row stride, so a ring address is one AND-OR (push / pop below)
  const uint32_t lane_b = threadIdx.x * 4u;
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
  // bit `lane` of a wave-uniform mask (lane opaque at the use: the compiler would otherwise hold a
  // 64-bit 1 << lane in registers across the loop)
  auto lane_bit = [&](unsigned long long m) -> bool {
    int l = lane;
    asm volatile("" : "+v"(l));
    return ((m >> l) & 1ull) != 0ull;
  };
  // lanes of mask m below this lane: v_mbcnt (no 64-bit lane mask held in registers)
  auto below = [](unsigned long long m) -> int {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  };
  // sample groups (the GRP variants only: the others compile none of it): log2 G, 0 = off
  const int group_log = GRP ? P.group_log : 0;
  // sample groups: of a wave mask m, the first-lane bits of the groups whose G lanes are all set
  // (wave-uniform; G a power of two <= 64)
  auto full_groups = [&](unsigned long long m) -> unsigned long long {
    const int gl = group_log;
    for (int sh = 1; sh < (1 << gl); sh <<= 1) m &= m >> sh;
    unsigned long long first = 0ull;   // bit 0 of every group
    for (int b = 0; b < 64; b += 1 << gl) first |= 1ull << b;
    return m & first;
  };
  // path state, [wave][region][64 lanes][4 fp64] (see kRegions): b128 buffer ops with the lane
  // offset in one VGPR and the region offset as an SGPR constant.
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(P.pstate, 0, (int)(P.nslots * kRegions * kLaneRec), kBufWord3);
  // (a lane handed over by tail compaction keeps its pixel's path state: pvo travels with it)
  uint32_t pvo = (blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * (uint32_t)kRegions * kRegionBytes +
                 (uint32_t)lane * kLaneRec;
  // a region's record: (x, y) at +0, (z, w) at +16 -- one 32-B sector
  // loads: two b128; stores: four b64.  A buffer store of more than 64 bits reads its data VGPRs
  // over more than one cycle, and a VALU write of those VGPRs right after it needs one wait state
  // -- which the compiler does not insert when the store's soffset is an SGPR (as here: the
  // region offset), so a b128 store lost the high half of z whenever the scheduler put such a
  // write next to it (round 2's "stale path-state reads"; DESIGN.md §4, tools/isa_audit.py).
  // 8-byte stores have no such hazard; the four of them fill the record's 32-B sector.
  auto LD4 = [&](int r, D3& v, double& w) {
    const D2 a = buf_ld2(prs, pvo, (uint32_t)r * kRegionBytes), b = buf_ld2(prs, pvo, (uint32_t)r * kRegionBytes + 16u);
    v = d3(a.a, a.b, b.a);
    w = b.b;
  };
  auto ST4 = [&](int r, D3 v, double w) {
#ifdef RT_MEAS_NO_PSTATE   // write-attribution build (wrong colours, same control flow): no path-state stores
    return;
#endif
    const uint32_t o = (uint32_t)r * kRegionBytes;
    buf_st(prs, pvo, o, v.x); buf_st(prs, pvo, o + 8u, v.y); buf_st(prs, pvo, o + 16u, v.z); buf_st(prs, pvo, o + 24u, w);
  };
  auto LDV = [&](int r) { D3 v; double w; LD4(r, v, w); return v; };
  auto STV = [&](int r, D3 v) { ST4(r, v, 0.0); };   // the whole sector (no partial write)
  auto LD_HN = [&]() { return d3(*R.a[0], *R.a[1], *R.a[2]); };
  auto ST_HN = [&](D3 v) { *R.a[0] = v.x; *R.a[1] = v.y; *R.a[2] = v.z; };
  // colour and weight carried across mirror bounces
  auto LD_SCOL_W = [&](D3& scol, double& w) {
    LD4(R_SCOLW, scol, w);
  };
  auto ST_SCOL_W = [&](D3 scol, double w) { ST4(R_SCOLW, scol, w); };

  // wave-uniform work-head cursor; in list mode the work count comes from the device
  // work items of the list mode: one per (listed pixel, sample), or per listed pixel with sample groups
  const long long n_list = P.list ? (long long)*P.list_count * (group_log ? 1 : P.nsamp) : 0;
  const long long n_tiles = P.list ? (n_list + 63) / 64 : P.n_tiles;
  int head = blockIdx.x % kGroups;
  int heads_left = kGroups;

  // ---- per-lane state live across phases ----
  int state = ST_FETCH;
  int px = 0, lrow = 0, py = 0, sample = 0, depth = 0, light = 0, mesh = 0, frame = 0;
  long long item = 0;       // list mode: work item (pixel * nsamp + sample), may exceed 2^31
  uint32_t pix_t0 = 0;      // start of the pixel (s_memrealtime; cost maps in time mode.  A pixel handed
                            // over by tail compaction restarts it at its adoption)
  int best = kNoHit;        // device record of the closest hit
  int own_rec = -1;         // device record the bounce being shaded hit (its shadow rays start on it)
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
  unsigned long long d_any_tris = 0, d_own_tris = 0;   // any-hit triangle tests; of those, the ray's own record
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
    const unsigned long long m = wballot(1);
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

  // normalize(): one shared reciprocal in the production variants (bit-identical, normalize_rcp)
  auto nrm_n = [](D3 v, double& n) -> D3 {
    if constexpr (STATS || TL) {
      n = sqrt(dot(v, v));
      return normalize(v);
    } else {
      return normalize_rcp(v, n);
    }
  };
  auto nrm = [&](D3 v) -> D3 {
    double n;
    return nrm_n(v, n);
  };
  // Ray(o, d): stores origin, normalised direction and t-limit to the LDS slot.
  auto emit_ray = [&](D3 o, D3 dir, double t_limit) {
    const D3 d = nrm(dir);
    *R.o[0] = o.x; *R.o[1] = o.y; *R.o[2] = o.z;
    *R.d[0] = d.x; *R.d[1] = d.y; *R.d[2] = d.z;
    *R.tlim = t_limit;
  };

  // primary ray of the current sample (mytracer_gpu.cu:202-209; Camera::primary_ray)
  auto start_sample = [&]() {
    int n = P.spp_n;
    asm volatile("" : "+s"(n));   // not hoisted: the fp64 offsets below stay temporaries of this block
    double X, Y;
    if (n == 1) {   // xo = 0/1 - 0.5 + 1/2 = +0 exactly: X = px + 0 = px
      X = (double)px;
      Y = (double)py;
    } else {
      const int si = sample / n, sj = sample - si * n;
      const double xo = (si) / (double)n - 0.5 + 1.0 / (2.0 * n);
      const double yo = (sj) / (double)n - 0.5 + 1.0 / (2.0 * n);
      X = (double)px + xo;
      Y = (double)py + yo;
    }
    const FrameDesc& K = P.frames[frame];
    const D3 dir = d3(K.ll[0] + X * K.xd[0] + Y * K.yd[0] - K.eye[0],
                      K.ll[1] + X * K.xd[1] + Y * K.yd[1] - K.eye[1],
                      K.ll[2] + X * K.xd[2] + Y * K.yd[2] - K.eye[2]);
    // SCOL = 0 and W = 1 are implicit at depth 0, PCOL = 0 at sample 0 (never stored)
    depth = 0;
    c_primary++;
    if (sample == 0) pix_t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();   // the pixel's start (100 MHz)
    emit_ray(d3(K.eye[0], K.eye[1], K.eye[2]), dir, DBL_MAX);
    state = ST_CLOSEST;
  };
  // compute_image's last step for the pixel (px, lrow, frame): average the sum over the n x n
  // samples, clamp, store (mytracer_gpu.cu:155-159, 221-227)
  auto store_pixel = [&](D3 pcol) {
    int n2 = P.spp_n * P.spp_n;
    asm volatile("" : "+s"(n2));   // converted here, not hoisted into a VGPR live across the loop
    const double nn = (double)n2;
    double r, g, b;
    if ((n2 & (n2 - 1)) == 0) {
      // n2 = 2^k: x / n2 = x * 2^-k exactly (one rounding of the same exact value), no division
      const double s = __builtin_ldexp(1.0, -__builtin_ctz((unsigned)n2));
      r = stdmin(pcol.x * s, 1.0); g = stdmin(pcol.y * s, 1.0); b = stdmin(pcol.z * s, 1.0);
    } else {
      r = stdmin(pcol.x / nn, 1.0); g = stdmin(pcol.y / nn, 1.0); b = stdmin(pcol.z / nn, 1.0);
    }
    // RT_FLAG_GLOBAL_ROWS: the row's place in the whole frame (the buffer may be another GPU's,
    // mapped over xGMI: the shard's pixels land in the assembled frame as they finish)
    const int orow = P.out_global ? (P.stripe_count == 1 ? P.row_begin + lrow : stripe_row(P, lrow)) : lrow;
    const size_t o = 3 * ((size_t)orow * P.W + px);
    // nontemporal (evict-first): the frame is written once and never read here, so its lines
    // should not push the path-state lines out of L2 (office: HBM writes 50.9 -> 45.5 MB per
    // frame, time unchanged; profiles/r03/write_traffic_r03.json)
#ifdef RT_MEAS_NO_IMAGE   // write-attribution build: no image stores
    if (false)
#else
    if (P.out_fmt == RT_OUT_RGB_F64)
#endif
    {
      double* out = reinterpret_cast<double*>(P.frames[frame].out) + o;
      __builtin_nontemporal_store(r, out); __builtin_nontemporal_store(g, out + 1);
      __builtin_nontemporal_store(b, out + 2);
    } else {
#ifndef RT_MEAS_NO_IMAGE
      float* out = reinterpret_cast<float*>(P.frames[frame].out) + o;
      __builtin_nontemporal_store((float)r, out); __builtin_nontemporal_store((float)g, out + 1);
      __builtin_nontemporal_store((float)b, out + 2);
#endif
    }
  };

  unsigned guard = 0;
  for (;;) {
    if (++guard > kGuardIters) {   // watchdog: end the wave instead of spinning, flag the launch
      if (lane == 0) trip_watchdog(P.ctr, P.guard_host);
      break;
    }
    if (STATS) { d_outer++; t_stamp = stamp(); }
    // ---------------- refill idle lanes (one atomic per wave) ----------------
    unsigned long long m_fetch = wballot(state == ST_FETCH);
    unsigned long long m_busy = wballot(state == ST_CLOSEST || state == ST_SHADOW || state >= ST_HSHADOW);
    // lanes that claim a work item: every idle lane, or (sample groups) the first lane of every idle
    // group, which claims a pixel for its G lanes
    unsigned long long m_claim = group_log ? full_groups(m_fetch) : m_fetch;
    while (m_claim && (group_log || __popcll(m_fetch) >= kRefill || m_busy == 0) && heads_left > 0) {
      const long long g0 = (n_tiles * head / kGroups) * 64;
      const long long g1 = (n_tiles * (head + 1) / kGroups) * 64;
      const int cnt = __popcll(m_claim);
      const int leader = __ffsll((long long)m_claim) - 1;
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
      // this lane's item: its rank among the claiming lanes (sample groups: its group's rank)
      const int gbase = group_log ? (lane & ~((1 << group_log) - 1)) : lane;
      const bool claims = state == ST_FETCH && (!group_log || ((m_claim >> gbase) & 1ull) != 0ull);
      if (claims) {
        const long long wk = start + (group_log ? __popcll(m_claim & ((1ull << gbase) - 1ull)) : below(m_fetch));
        if (wk < g1) {
          if (P.list) {   // adaptive pass: one sample of a listed pixel
            // (the divisors made opaque here: the compiler would otherwise keep their reciprocals in
            // registers across the whole persistent loop)
            long long ns = group_log ? 1 : P.nsamp;   // sample groups: one work item per listed pixel
            uint32_t wd = (uint32_t)P.W;
            asm volatile("" : "+s"(ns), "+s"(wd));
            const uint32_t id = wk < n_list ? P.list[wk / ns] : 0xffffffffu;
            const uint32_t pix = id & kListPixMask;
            frame = id != 0xffffffffu ? (int)(id >> kListFrameShift) : 0;
            px = id != 0xffffffffu ? (int)(pix % wd) : P.W;
            lrow = id != 0xffffffffu ? (int)(pix / wd) : P.rows;
            item = wk;
          } else {
            // (tile indices < 2^31, checked at launch: 32-bit divisions by the launch's invariant
            // divisors as a multiply-high and a shift, DivMagic)
            const uint32_t tile = P.tile_order ? P.tile_order[wk >> 6] : (uint32_t)(wk >> 6);
            const int j = (int)(wk & 63);
            // several frames: tile row ty of every frame, then row ty + 1, so each XCD head's
            // contiguous range is a band of rows of all frames (its L2 holds one band's nodes)
            const uint32_t row_tiles = (uint32_t)P.n_frames * (uint32_t)P.tiles_x;
            const uint32_t ty = P.div_row_tiles.div(tile);
            const uint32_t rem = tile - ty * row_tiles;
            frame = P.n_frames > 1 ? (int)P.div_tiles_x.div(rem) : 0;
            const int tx = (int)(rem - (uint32_t)frame * (uint32_t)P.tiles_x);
            int jx = j & (kTileW - 1), jy = j >> kTileWLog;
            if (kTileMorton && kTileW == 8) {   // (kTileMorton)
              jx = (j & 1) | ((j >> 1) & 2) | ((j >> 2) & 4);
              jy = ((j >> 1) & 1) | ((j >> 2) & 2) | ((j >> 3) & 4);
            }
            px = tx * kTileW + jx;
            lrow = (int)ty * kTileH + jy;
          }
          if (px < P.W && lrow < P.rows) {
            py = (P.stripe_count == 1)
                     ? P.row_begin + lrow
                     : stripe_row(P, lrow);
            if (P.list && !group_log) {
              long long ns = P.nsamp;
              asm volatile("" : "+s"(ns));
              sample = (int)(item % ns);
            } else {
              sample = lane - gbase;   // sample groups: the lane's place in its group (chunk 0); else 0
            }
            start_sample();
          }
        }
      }
      m_fetch = wballot(state == ST_FETCH);
      m_busy = wballot(state == ST_CLOSEST || state == ST_SHADOW || state >= ST_HSHADOW);
      m_claim = group_log ? full_groups(m_fetch) : m_fetch;
      if (!group_log && __popcll(m_fetch) < kRefill && m_busy != 0) break;
    }
    if (heads_left == 0 && state == ST_FETCH) state = ST_DONE;
    const bool busy = (state == ST_CLOSEST || state == ST_SHADOW || state >= ST_HSHADOW);
    if (wballot(busy) == 0) {
      if (wballot(state != ST_DONE) != 0) continue;
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
        double nl;   // |to_l|: the light distance, the same sqrt as the normalisation's
        const D3 l = nrm_n(to_l, nl);
        ro = add(hp, scl(1e-4, l));
        rd = nrm(l);
        tlim = nl;
      } else if (state == ST_HCLOSEST) {
        // the owner's reflection ray (mytracer.cpp:547-552), from its hit and its normal (the
        // owner's aux words); kept in this helper's slot, from which the owner takes it over
        const D3 hp = add(ro, scl(tlim, rd));
        const D3 hn = d3(lds_d[7 * kBlock + src], lds_d[8 * kBlock + src], lds_d[9 * kBlock + src]);
        const double s2 = 2.0 * dot(hn, rd);   // reflect(d, n) = d - 2(n.d)n, d = -view = rd
        const D3 v = sub(rd, scl(s2, hn));
        ro = add(hp, scl(1e-4, v));
        rd = nrm(v);
        tlim = DBL_MAX;
        *R.o[0] = ro.x; *R.o[1] = ro.y; *R.o[2] = ro.z;
        *R.d[0] = rd.x; *R.d[1] = rd.y; *R.d[2] = rd.z;
      }
      // the record this any-hit ray starts on (the owner's shading hit; helpers read their owner's)
      int own = -1;
      if (anyhit) own = (state == ST_SHADOW) ? own_rec : __shfl(own_rec, (int)(htask & 63u));
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
          if constexpr (WIDTH == 4) {
            // v_rcp_f32 (1 ulp) + one Newton step: within about half an ulp of 1 / df, as the
            // correctly rounded division (11 VALU) it replaces; the box error bound of DESIGN.md
            // §4 stays far inside delta.  (The 2-wide canonical kernel keeps the oracle's division.)
            const float r0 = __builtin_amdgcn_rcpf(df);
            inv[k] = __builtin_fmaf(__builtin_fmaf(-df, r0, 1.0f), r0, r0);
          } else {
            inv[k] = 1.0f / df;
          }
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
      float pinf = INFINITY;   // opaque to the combiner: a constant med3 operand folds back to min / max
      asm volatile("" : "+s"(pinf));
      // logical stack [0, sp); the LDS ring holds [slo, sp), spill[] holds [0, slo).  Kept byte-scaled
      // by a lane's ring stride (kSW = kBlock words, in bytes): sq = sp * kSW, sqlim = (slo + RING) * kSW, so a
      // push is one compare with sqlim, one AND-OR for the ring address (the lane's byte offset sits
      // below kSW) and one add; sp / slo themselves are only formed on the spill path
      constexpr uint32_t kSW = kBlock * 4u, kRingB = (uint32_t)RING * kSW, kRingBMask = (uint32_t)kRingMask * kSW;
      uint32_t sq = 0, sqlim = kRingB;
      auto ring = [&](uint32_t q) -> __attribute__((address_space(3))) uint32_t& {
        return *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>((size_t)((q & kRingBMask) | lane_b));
      };
      auto push = [&](uint32_t x) {
        if (sq == sqlim) {   // ring full: its bottom entry goes to the spill stack
          const uint32_t qlo = sqlim - kRingB;
          spill[(size_t)(qlo / kSW) * P.nslots] = ring(qlo);
          sqlim += kSW;
          if (STATS) d_spills++;
          if constexpr (TL) tl_spill++;
        }
        ring(sq) = x;
        sq += kSW;
      };
      auto pop = [&]() -> uint32_t {
        if (sq == 0) return kDone;
        sq -= kSW;
        if (sq + kRingB >= sqlim) return ring(sq);
        sqlim = sq + kRingB;
        return spill[(size_t)(sq / kSW) * P.nslots];
      };
      const D3 c3 = d3(-rd.x, -rd.y, -rd.z);

      // Watchdog of the traversal loops that could cycle on a corrupt hierarchy (the round loop
      // and the node loops): each counts its own wave-level iterations in a counter that lives
      // only inside that loop, so it stays wave-uniform (an SGPR: the check costs SALU only).
      // A loop that runs past kTravGuard iterations abandons the ray (results void) and flags
      // the launch.  (Cost: 0.3 % for the node loop, A/B.)
      // (the ray is abandoned; a corrupt hierarchy costs each traversal that enters it one guard's
      // worth of iterations -- a per-wave exit flag measured -1.4 % on the office, r06e)
      auto guard_trip = [&]() {
        if (lane == __ffsll((long long)wballot(1)) - 1) trip_watchdog(P.ctr, P.guard_host);
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
              const uint32_t i0 = __shfl(i, __ffsll((long long)wballot(1)) - 1);
              if (wballot(i != i0) == 0) wave_tick(d_leaf_uni, d_dummy, lane);
            }
            if (STATS && anyhit) {   // (r06zg: the own record is 14 % of the office's any-hit tests; skipping
              d_any_tris++;          // it, unchecked, cost 3.7 %: DESIGN.md §11.12)
              if ((int)rec == own) d_own_tris++;
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
                const double Dt = det3(T.e1, T.e2, c4);
                // (t's division shared with alpha / beta's reciprocal: -0.9 %, more live registers)
                const double t = Dt / S;
                const bool cand = anyhit ? (t < tlim) : (t <= tlim);
                if (t > 1e-5 && cand) {
                  double alpha, beta;
                  // alpha, beta: one reciprocal of S for the two quotients where that is bit-identical:
                  // |S| >= 1e-10 here and |Da|, |Db| <= |S|(1 + 2^-48) (the early rejections), so with
                  // |Da|, |Db| >= |S| 2^-900 and |S| < 2^1000 no operand or quotient is denormal, zero or
                  // near an exponent limit
                  const double lim = aS * 0x1p-900;
                  const bool fab = !STATS && !TL && fabs(Da) >= lim && fabs(Db) >= lim && aS < 0x1p1000;
                  if (fab) {
                    const double r = rcp_refined(S);
                    alpha = div_by(Da, S, r);
                    beta = div_by(Db, S, r);
                  } else {
                    alpha = Da / S;
                    beta = Db / S;
                  }
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
      // a wave whose traversing lanes are all any-hit rays visits children without the distance
      // sort (any visit order finds the same occluded / not-occluded answer): office +3.6 %
      // batched, +2.3 % one frame; config 4 +3.2 % one frame, -1.1 % batched; testing the hit bits
      // instead of the keys (which then serve only the sorted path): office +2.1 % / +2.0 % more
      // (A/B).  The diagnostic (STATS) variants sort every wave: their node and
      // triangle counts then follow each lane's own distance order, not the mix of rays a wave holds
      const bool w_any = !STATS && wballot(!anyhit && cur != kDone) == 0;   // wave-uniform
      while ((wballot(cur != kDone) | wballot(pleaf != kDone)) != 0) {
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
          bool hb[4];   // child hit (any-hit waves test these; the keys and count then serve only the sort)
          int cnt = 0;
          float4 nx, fx, ny, fy, nz, fz;
          uint4 rf;
          // wave-uniform: every active lane's node is in the LDS treelet -> ds_read, no TD cost
          if (wballot(cur >= (uint32_t)P.n_top) == 0) {
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
            // 32-bit byte offsets from the node array's base (an SGPR pair): global_load's saddr
            // form, one 32-bit OR per plane instead of 64-bit address arithmetic (office +0.7 %,
            // config 4 +1.1 %; the node array stays below 4 GB: checked at upload)
            const char* nbase = reinterpret_cast<const char*>(P.nodes4);
            const uint32_t nbo = cur * (uint32_t)sizeof(GNode4);
#define RT_NODE_AT(off) (nbase + (uint32_t)(nbo + (off)))
            if constexpr (TL) { tl_gnode++; tl_wave_gap(1); }
            if (STATS) {
              wave_distinct(cur, d_gn_dist, lane);
              const uint32_t c0 = __shfl(cur, __ffsll((long long)wballot(1)) - 1);
              if (wballot(cur != c0) == 0) wave_tick(d_gn_uni, d_dummy, lane);
            }
            nx = *reinterpret_cast<const float4*>(RT_NODE_AT(nxo));
            fx = *reinterpret_cast<const float4*>(RT_NODE_AT(nxo ^ 16u));
            ny = *reinterpret_cast<const float4*>(RT_NODE_AT(nyo));
            fy = *reinterpret_cast<const float4*>(RT_NODE_AT(nyo ^ 16u));
            nz = *reinterpret_cast<const float4*>(RT_NODE_AT(nzo));
            fz = *reinterpret_cast<const float4*>(RT_NODE_AT(nzo ^ 16u));
            rf = *reinterpret_cast<const uint4*>(RT_NODE_AT(96u));
#undef RT_NODE_AT
          }
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float tx0 = __builtin_fmaf(f4c(nx, c), ivx, -oix), tx1 = __builtin_fmaf(f4c(fx, c), ivx, -oix);
            const float ty0 = __builtin_fmaf(f4c(ny, c), ivy, -oiy), ty1 = __builtin_fmaf(f4c(fy, c), ivy, -oiy);
            const float tz0 = __builtin_fmaf(f4c(nz, c), ivz, -oiz), tz1 = __builtin_fmaf(f4c(fz, c), ivz, -oiz);
            // the window bound enters through med3 (med3(t, lo, +inf) = max, med3(t, hi, -inf) = min;
            // no operand is ever NaN: |inv| <= 1e20, finite or empty-box planes): fminf / fmaxf of
            // the loop-carried bound made the compiler re-canonicalise it every iteration (2 VALU)
            const float tn = fmaxf(fmaxf(tx0, ty0), __builtin_amdgcn_fmed3f(tz0, lo_c, pinf));
            const float tf = fminf(fminf(tx1, ty1), __builtin_amdgcn_fmed3f(tz1, hi_c, -pinf));
            const uint32_t r = u4c(rf, c);
            const bool h = tn <= tf;   // absent children carry the empty box [+inf, -inf]
            hb[c] = h;
            k[c] = h ? tn : INFINITY;
            v[c] = r;
            cnt += h ? 1 : 0;
          }
#define RT_CSWAP(a, b)                                        \
  if (k[b] < k[a]) {                                          \
    const float tk = k[a]; k[a] = k[b]; k[b] = tk;            \
    const uint32_t tv = v[a]; v[a] = v[b]; v[b] = tv;         \
  }
          if (w_any) {   // a wave of any-hit rays: the last hit child first, the others pushed
            // (orders chosen per lane or per wave from the ray's entry distances lost 2-11 %, the
            // swaps' cost included; the fixed first-slot-first order 4 %: DESIGN.md §4)
            uint32_t nxt = kDone;
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (hb[c]) {
                if (nxt != kDone) push(nxt);
                nxt = v[c];
              }
            cur = nxt == kDone ? pop() : nxt;
          } else {
          RT_CSWAP(0, 1) RT_CSWAP(2, 3) RT_CSWAP(0, 2) RT_CSWAP(1, 3) RT_CSWAP(1, 2)
          if (cnt == 0) {
            cur = pop();
          } else {
            if (cnt > 3) push(v[3]);
            if (cnt > 2) push(v[2]);
            if (cnt > 1) push(v[1]);
            cur = v[0];
          }
          }
#undef RT_CSWAP
          if ((cur & kLeaf) && cur != kDone && pleaf == kDone) {   // first leaf: postpone, keep going
            pleaf = cur;
            cur = pop();
          }
          if ((wballot(pleaf == kDone) & wballot(cur != kDone)) == 0) break;   // every lane holds a leaf (one mask per compare)
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
      const unsigned nb = (unsigned)__popcll(wballot(busy));
      const unsigned no = (unsigned)__popcll(wballot(state == ST_CLOSEST || state == ST_SHADOW));
      const unsigned nsh = (unsigned)__popcll(wballot(busy && (state == ST_SHADOW || state == ST_HSHADOW)));
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
    // (not with sample groups: a group's lanes and their parked colours stay in their wave)
    if (heads_left == 0 && !group_log) {
      // wave in block, wave-uniform (an SGPR: derived at the use, not a VGPR held across the loop)
      const int wib = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
      const bool owner = (state == ST_CLOSEST || state == ST_SHADOW);
      const unsigned long long O = wballot(owner);
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
        if (owner && !lane_bit(back)) state = ST_DONE;   // adopted by another wave
      } else {
        // adopt pooled lanes of other waves into idle lanes
        unsigned long long I = wballot((state == ST_FETCH || state == ST_DONE) && !refl_held);
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
          const bool idle = lane_bit(I);
          const int r = below(I);
          const bool take = idle && r < n;
          if (take) {
            const int t = w * 64 + kth_set_bit(got, r);   // donor thread
            const uint32_t* ds = reinterpret_cast<const uint32_t*>(lds_raw) + t;   // its stack entries
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
                     : stripe_row(P, lrow);
            lvis[threadIdx.x] = lvis[t];
#pragma unroll
            for (int k = 0; k < kSlotDoubles; ++k) lds_d[k * kBlock + threadIdx.x] = lds_d[k * kBlock + t];
            thit = *R.tlim;   // a closest-hit ray's distance (a shadow batch's owner does not read thit)
            own_rec = -1;     // (not migrated: an adopted shadow batch tests every record)
            pix_t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
          }
          I &= ~wballot(take);
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
        const D3 l = nrm(sub(L6.pos, hp_));   // exact: it decides diff > 0 (a discontinuity)
        const double diff = stdmax(0.0, dot(hn_, l));
        double refl = 0.0;
        if (diff > 0.0) {   // reflection(), mytracer.cpp:524-534
          const double s2 = 2.0 * dot(hn_, l);
          const D3 r = normalize_shade(sub(scl(s2, hn_), l));   // feeds only max(0, r.v)^shininess: continuous
          refl = stdmax(0.0, dot(r, hv_));
        }
        // pow(+0, y > 0) = +0 exactly: skip the fp64 pow for the (frequent) zero highlight
        if (!(refl == 0.0 && M.shininess > 0.0)) refl = pow_shade(refl, M.shininess);
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
        const D3 hdiff = M.tex_w > 0 ? LDV(R_HD) : d3(M.kd[0], M.kd[1], M.kd[2]);
        mirror = M.mirror;
        // first batch: the ambient term (mytracer.cpp:574-576) again, else the stored sum
        D3 lacc = light == 0 ? d3(0.0 + P.amb[0] * M.ka[0], 0.0 + P.amb[1] * M.ka[1], 0.0 + P.amb[2] * M.ka[2])
                             : LDV(R_LACC);
        const uint32_t vw = lvis[threadIdx.x];
        for (int j = light; j < batch_end; ++j) {
          const bool occluded = (j == light) ? shadow_hit : (((vw >> (j - light)) & 1u) != 0u);
          // an occluded light adds colour * 0 * (finite term) = +-0, which leaves the sum (never -0)
          // unchanged: skip it (the term is finite for any material with finite shininess >= 0)
          if (!occluded) lacc = add(lacc, contrib_of(j, hp, hn, hview, hdiff, M));
        }
        light = batch_end;
        if (light < P.n_lights) {
          STV(R_LACC, lacc);
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
          own_rec = best;
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
            if (M.tex_w > 0) STV(R_HD, hdiff);
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
      if (finish && group_log) {
        // sample groups: the colour waits in the (now free) ray slot for the group's ordered sum
        *R.o[0] = scol.x; *R.o[1] = scol.y; *R.o[2] = scol.z;
        state = ST_PARKED;
      } else if (finish && P.list) {   // adaptive pass: this sample's trace() colour
        const D3 c = scol;
        double* so = P.sample_out + 3 * (size_t)item;
        so[0] = c.x; so[1] = c.y; so[2] = c.z;
        state = heads_left > 0 ? ST_FETCH : ST_DONE;
      } else if (finish) {
        if (P.tile_cost) {   // cost of this sample: its bounces, or in time mode the pixel's lifetime at its
                             // last sample, summed per tile position over the launch's frames
          const long long t = (long long)(lrow >> kTileHLog) * P.tiles_x + (px >> kTileWLog);   // tile position (all frames)
          uint32_t c = (uint32_t)(depth + 1);
          if (P.cost_time) {
            c = 0;
            if (sample + 1 == P.spp_n * P.spp_n)
              c = (uint32_t)__builtin_amdgcn_s_memrealtime() - pix_t0;
          }
          // one atomic per distinct tile among the lanes finishing here (a wave's lanes mostly share
          // one or two tiles; 64 atomics on one address queue at the memory side)
          unsigned long long m = wballot(1);
          while (m != 0ull) {
            const int ld = __ffsll((long long)m) - 1;
            const uint32_t tl = (uint32_t)__shfl((int)t, ld);
            const bool same = (uint32_t)t == tl;
            const unsigned long long ms = wballot(same);
            uint32_t sum = same ? c : 0u;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) sum += (uint32_t)__shfl_xor((int)sum, o);
            if (lane == ld) atomicAdd(&P.tile_cost[tl], sum);
            m &= ~ms;
          }
        }
        const D3 pcol = add(sample == 0 ? d3(0, 0, 0) : LDV(R_PCOL), scol);
        sample++;
        if (sample < P.spp_n * P.spp_n) {
          STV(R_PCOL, pcol);
          start_sample();
        } else {   // compute_image: average, clamp, store (mytracer_gpu.cu:155-159, 221-227)
          store_pixel(pcol);
          state = heads_left > 0 ? ST_FETCH : ST_DONE;
        }
      }
    }
    asm volatile("" ::: "memory");

    // ---- sample groups: a group whose G samples are all parked is summed by its first lane ----
    // in sample order (the reference's (si, sj) order, mytracer_gpu.cu:202-221: sample s = si n + sj,
    // and a group holds samples chunk * G .. chunk * G + G - 1 on its lanes in order), then the group
    // starts its next chunk, or the pixel is stored and the group fetches another
    if (group_log) {
      const unsigned long long full = full_groups(wballot(state == ST_PARKED));
      if (full != 0ull) {
        wave_lds_sync();   // the group's colours, written by its lanes in SHADE, are in LDS
        const int gl = group_log;
        const int gbase = lane & ~((1 << gl) - 1);
        const bool group_done = ((full >> gbase) & 1ull) != 0ull;
        if (group_done && lane == gbase) {
          D3 pc = sample == 0 ? d3(0, 0, 0) : LDV(R_PCOL);   // (the first lane holds sample chunk * G)
          for (int k = 0; k < (1 << gl); ++k) {
            const int t = wbase + gbase + k;
            pc = add(pc, d3(lds_d[0 * kBlock + t], lds_d[1 * kBlock + t], lds_d[2 * kBlock + t]));
          }
          if (sample + (1 << gl) < P.spp_n * P.spp_n) STV(R_PCOL, pc);   // more chunks: the running sum
          else store_pixel(pc);
        }
        wave_lds_sync();   // the first lane has read the group's slots before they take new rays
        if (group_done) {
          sample += 1 << gl;
          if (sample < P.spp_n * P.spp_n) start_sample();
          else state = heads_left > 0 ? ST_FETCH : ST_DONE;
        }
      }
    }

    // ---- lend idle lanes to owners' extra rays (extra lights in order, then reflection) ----
    {
      const bool idle = (state == ST_FETCH || state == ST_DONE);
      const unsigned long long I = wballot(idle);
      if (I != 0ull && wballot(want > 0) != 0ull) {
        if (idle) ltask[threadIdx.x] = kTaskNone;
        const int incl = wave_incl_scan(want);   // inclusive prefix sum of want over the wave
        wave_lds_sync();
        const int off = incl - want;
        const int avail = (int)__popcll(I);   // __popcll is unsigned: keep the subtraction signed
        const int got = min(want, max(0, avail - off));
        if (got > 0) {
          const int n_extra_lights = min(P.n_lights - light - 1, kBatchExtra);
          for (int t = 0; t < got; ++t) {   // task words only: each helper derives its own ray
            const int ht = wbase + kth_set_bit(I, off + t);   // (a ranked idle-lane list instead: +-0.5 %)
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
  // RT_FLAG_GLOBAL_ROWS into a peer GPU's frame: this wave's image stores are written back to
  // memory before it exits (system-scope release), so they are there when the launch ends
  // (the explicit wait: ROCm 7.2 may drop the fence's own vmcnt wait after its L2 write-back when it
  // believes the wave's counter empty, MI355X_MICROARCH.md "Compiler hazard")
  if (P.out_global) {
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
    const unsigned long long at = wave_sum(d_any_tris), ot = wave_sum(d_own_tris);
    if (lane == 0) {
      atomicAdd(&P.ctr[CD_ANYHIT_TRIS], at);
      atomicAdd(&P.ctr[CD_OWN_TRIS], ot);
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
  if (P.zero_map) {
    // the next launch's work order, built by the first blocks to finish (their CUs would idle in the
    // drain): job h < 8 sorts head range h of order_src by cost, descending (stable: equal costs keep
    // the natural band order); jobs 8..15 clear an eighth of zero_map.  The block's LDS is free now.
    // A block takes jobs until none is left, so a launch of fewer than 16 blocks (a small image)
    // still completes all of them (one job per block left the order of the last head ranges stale:
    // a non-permutation, tiles rendered twice or not at all).
    uint32_t* job = reinterpret_cast<uint32_t*>(lds_raw);
    for (;;) {
      __syncthreads();   // the previous job is done with the LDS
      if (threadIdx.x == 0) *job = (uint32_t)atomicAdd(&P.ctr[CT_ORDER_JOBS], 1ull);
      __syncthreads();
      const uint32_t j = *job;
      __syncthreads();   // every thread has read it before the sort reuses the LDS
      if (j >= 2u * kGroups) break;
      if (j < (uint32_t)kGroups) {
        if (P.order_src) order_range(P.order_src, P.next_order, P.n_pos, (int)j, lds_raw, P.tiles_x, P.order_dilate);
      } else {
        for (long long i = P.n_pos * (j - kGroups) / kGroups + threadIdx.x; i < P.n_pos * (j - kGroups + 1) / kGroups;
             i += kBlock)
          P.zero_map[i] = 0u;
      }
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
constexpr int kSelTilesPerWave = 8;
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
    const unsigned long long m = wballot(sel);
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
// outs (several frames): frame f's output buffer is outs[f] -- a table owned by the call (its
// stream-ordered scratch), not the launch context's frame table, which a later launch on another
// stream may overwrite once the render kernel has finished.
__global__ void __launch_bounds__(256) adaptive_reduce_kernel(const uint32_t* list, const unsigned long long* count,
                                                              const double* samples, int nsamp, void* out,
                                                              int out_fmt, void* const* outs) {
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
  if (outs) out = outs[id >> kListFrameShift];   // several frames
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


using KernelFn = void (*)(KParams);

struct Variant {
  KernelFn fn;
  bool stats;
};

// [0] production (4-wide), [1] 4-wide + counters, [2] canonical 2-wide counters
// (the traversal the oracle replicates: tests pin its node / triangle counts),
// [3] production + per-round timeline (RT_FLAG_TIMELINE, diagnostics), [4] production with a
// 16-entry stack ring (deep hierarchies), [5] / [6] = [0] / [4] with sample groups (spp > 1, DESIGN.md
// §11.6; separate instances, so the one-sample kernels carry none of the group code).  (A suspend/resume variant for deep scenes' several-frame
// launches, rounds 3-4, was removed in round 5: +0.2 % on config 4 against 21-30 MB per frame of
// parked-state writes)
const Variant kVariants[] = {
    {render_kernel<4, false>, false},
    {render_kernel<4, true>, true},
    {render_kernel<2, true>, true},
    {render_kernel<4, false, true>, false},
    {render_kernel<4, false, false, 16>, false},
    {render_kernel<4, false, false, kShortStack, true>, false},
    {render_kernel<4, false, false, 16, true>, false},
};
constexpr int kNumVariants = 7;
// rt_upload_options.spp_lanes = 0: sample groups for spp > 1 launches or not
constexpr bool kSppLanesDefault = true;   // config 3 +22.6 %, config 5 +19.3 % (r06d)
// default group-size cap: 8K 64 spp at G = 32 (2 pixels per wave, 2 chunks each) +3.2 % over G = 64,
// +0.7 % over G = 16; 4K 16 spp best at G = 16 = n^2 (r06o)
constexpr int kGroupLanes = 32;
constexpr int kRingDeep = 16;
inline int variant_ring(int v) { return (v == 4 || v == 6) ? kRingDeep : kShortStack; }
// LDS per block: the variant's stack ring (ring entries per thread, at address 0: the kernel's
// slot offsets are compile-time constants), kSlotDoubles doubles of slot, task + visibility words.
size_t lds_bytes(int /*stack_words*/, int ring = kShortStack) {
  return (size_t)kBlock * (kSlotDoubles * sizeof(double) + (2 + (size_t)ring) * sizeof(uint32_t));
}
// ... plus the top treelet (n_top 128-B nodes) after it
size_t lds_bytes_total(int stack_words, int n_top, int ring = kShortStack) {
  return lds_bytes(stack_words, ring) + (size_t)n_top * sizeof(GNode4) + RT_MAX_LIGHTS * 6 * sizeof(double) + kPoolBytes;
}
// treelet nodes that fit next to a ring of the given size in a block's 40 KB (kTopNodes beside the
// 8-entry ring)
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
  unsigned long long* d_ctr = nullptr;       // control block: [kCtrWords] work heads, stats, diagnostics,
                                             // then FrameDesc[n_frames], then the light table
                                             // [n_lights][6] (one H2D copy per launch)
  unsigned char* h_ctl = nullptr;            // pinned staging of the same bytes
  size_t ctl_cap = 0;                        // bytes of d_ctr / h_ctl (grown for > RT_MAX_LIGHTS lights)
  long long blocks = 0;                      // persistent grid of the last launch (rt_debug_last_grid)
  long long full_blocks = 0;                 // ... and the grid that launch shape gets on an idle device
  double* d_pstate = nullptr;                // path state, nslots x kRegions x 32 B
  uint32_t* d_spill = nullptr;               // [stack_words][nslots] (only when stack_words > kShortStack)
  unsigned long long* d_wavelog = nullptr;   // [nslots / 64][4]
  unsigned long long* d_wctr = nullptr;      // [nslots / 64][4] per-wave ray counts
  unsigned long long* d_tl = nullptr;        // [nslots / 64][kTlCap][kTlWords], allocated by the first TL launch
  hipEvent_t ev0 = nullptr, ev1 = nullptr;   // kernel start / end (timing, reuse fence)
  hipEvent_t ev_in = nullptr;                // reserve_cus: the caller's stream joined to the launch stream
  long long waves = 0;                       // waves of the last launch (per-wave counter slots)
  int variant = -1;                          // kernel variant of the last launch (3: round timeline)
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
  hipStream_t last_stream = nullptr;   // ... and its stream
  size_t nslots = 0;
  // kernel watchdog (CD_GUARD), mirrored by the kernel into page-locked host memory, so a launch
  // without stats reports it too: the next launch on the scene, rt_last_kernel_ms and
  // rt_scene_status return RT_ERR_HIP once it is set (sticky: the scene's results are void)
  unsigned int* h_guard = nullptr;   // host view
  unsigned int* d_guard = nullptr;   // the same word as the kernel addresses it
  double delta = 0.0;
  double root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};
  long long bytes = 0;
  int n_cu = 0;
  int blocks_per_cu[kNumVariants] = {};
  bool deep = false;            // launches use the 16-entry ring variant (deep hierarchy)
  bool big = false;             // >= 2^18 device records, whatever ring rt_upload_options.stack_ring forced
  int n_top_v[kNumVariants] = {};   // treelet nodes of each kernel variant (by its stack ring)
  GNode4* d_nodes4 = nullptr;
  int n_gnodes4 = 0;
  int bpc_cap = 0;              // rt_upload_options.blocks_per_cu (0: as many as fit)
  int grid_spare = 0;           // rt_upload_options.grid_spare
  std::vector<GMat> mesh_mats;  // host copy: the analytic materials are appended after these
  GPrim* d_prims = nullptr;     // analytic primitives (rt_scene_set_analytic), spheres then planes
  int n_prims = 0;
  long long table_bytes = 0;    // device bytes of d_mats + d_prims
  // per-tile-position cost maps (RT_FLAG_COST_ORDER / RT_FLAG_TILE_COST*) of one image geometry
  // (cost_n positions, cost_tiles_x wide): launch s of the sequence writes d_cost[s % 3]; an ordered
  // launch s also builds d_order[(s + 1) % 2] from d_cost[(s - 1) % 3] and clears d_cost[(s + 1) % 3]
  // in its drain, so launch s + 1 is ordered by the costs of launch s - 1
  uint32_t* d_cost[3] = {nullptr, nullptr, nullptr};
  uint32_t* d_order[2] = {nullptr, nullptr};
  long long cost_cap = 0, cost_n = 0;
  int cost_tiles_x = 0;
  long long cost_seq = 0;             // launches of the current sequence
  long long order_for = -1;           // the sequence launch d_order[order_for % 2] was built for
  long long last_order_n = 0;         // tiles of the last ordered launch (rt_debug_last_tile_order)
  int last_order_buf = 0;
  uint32_t* d_tile_order = nullptr;  // rt_debug_set_tile_order: work order of launches with that many tiles
  void* d_host_stage = nullptr;       // rt_render_to_host into pageable memory: the frame before its copy
  size_t host_stage_bytes = 0;
  long long tile_order_n = 0;
  // the last launch that read or wrote the cost / order maps (ordered or cost-debug): its stream and
  // an event recorded after it.  A map-touching launch on another stream waits for that event; an
  // implicitly ordered launch needs that stream (stream order is then the fence)
  bool maps_used = false;
  hipStream_t maps_stream = nullptr;
  hipEvent_t maps_ev = nullptr;
  double build_s = 0.0, copy_s = 0.0;   // rt_scene_upload_seconds
  // rt_upload_options.reserve_cus: launches run on internal streams whose CU mask leaves that many
  // CUs free, one per caller stream (at most kMaskedStreams; further callers share slot hash % 4)
  int reserve_cus = 0;
  int order_window = 0;   // rt_upload_options.order_window (0: by depth)
  int spp_lanes = 0;      // rt_upload_options.spp_lanes (sample groups for spp > 1)
  static constexpr int kMaskedStreams = 4;
  hipStream_t masked[kMaskedStreams] = {};
  hipStream_t masked_for[kMaskedStreams] = {};
  int n_masked = 0;
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

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_error.c_str(); }

const char* rt_build_info(void) {
  return "librt_hip: gfx950 persistent flattened render kernel; variants {4-wide 8-entry stack ring, 4-wide 16-entry ring (>= 2^18 triangle records), "
         "4-wide+stats, 2-wide canonical stats, 4-wide+round timeline, sample groups (spp > 1) on both rings}; "
         "fp32 4-wide nodes (128 B) with an LDS treelet, "
         "fp64 triangles/shading, LDS ray slots + stack ring (global spill), global path state, 8 XCD work heads";
}

int rt_scene_upload(const rt_scene_soa* s, const rt_bvh_soa* b, int device, rt_scene** out) {
  return rt_scene_upload_ex(s, b, device, nullptr, out);
}

}  // extern "C"

namespace {
// Copies a built scene image to `device` and allocates its launch contexts.
int upload_image(const SceneImage& I, const rt_upload_options& opt, int device, rt_scene** out) {
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
  if ((unsigned long long)I.nodes4.size() * sizeof(GNode4) >= (1ull << 32)) {   // 32-bit node offsets
    rt_scene_free(sc);
    return fail(RT_ERR_UNSUPPORTED, "rt_scene_upload: more than 2^25 4-wide nodes");
  }
  // deep hierarchies (half a million device records and more: random-triangle soups of ~1 M and
  // up spill an 8-entry ring on every other ray, the office proxy on 1 in 130) render with the
  // 16-entry ring and the 9-node treelet that fits beside it (A/B)
  sc->big = I.tris.size() >= (size_t)(1u << 18);   // device records (office 77 k prefers 8, 500 k random 16)
  sc->deep = sc->big;
  if (opt.stack_ring != 0) sc->deep = opt.stack_ring >= 16;   // forced ring size (the order window keeps `big`)
  for (int v = 0; v < kNumVariants; ++v) {
    int& nt = sc->n_top_v[v];
    nt = top_nodes_for(sc->stack_words, variant_ring(v), sc->n_gnodes4);
    if (opt.lds_treelet > 0) nt = std::min(nt, opt.lds_treelet);   // cache at most this many nodes
    if (opt.lds_treelet < 0) nt = 0;                                // none
  }
  sc->bpc_cap = opt.blocks_per_cu;
  sc->grid_spare = opt.grid_spare;
  sc->reserve_cus = opt.reserve_cus;   // bounded by the CU count below
  sc->order_window = opt.order_window;
  sc->spp_lanes = opt.spp_lanes;
  sc->delta = I.delta;
  for (int k = 0; k < 3; ++k) {
    sc->root_lo[k] = I.root_lo[k];
    sc->root_hi[k] = I.root_hi[k];
  }
  sc->bytes = bytes;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { rt_scene_free(sc); return fail(RT_ERR_HIP, "hipGetDeviceProperties failed"); }
  sc->n_cu = prop.multiProcessorCount;
  sc->reserve_cus = std::max(0, std::min(sc->reserve_cus, sc->n_cu - 1));
  int max_blocks = 1;
  for (int v = 0; v < kNumVariants; ++v) {
    const int ring = variant_ring(v);
    const size_t lds = lds_bytes_total(sc->stack_words, sc->n_top_v[v], ring);
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
  // the watchdog word: page-locked, mapped into the device's address space
  if (hipHostMalloc(reinterpret_cast<void**>(&sc->h_guard), 64, hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&sc->d_guard), sc->h_guard, 0) != hipSuccess) {
    rt_scene_free(sc);
    return fail(RT_ERR_HIP, "allocation of the watchdog word failed");
  }
  *reinterpret_cast<volatile unsigned int*>(sc->h_guard) = 0u;
  for (LaunchCtx& c : sc->ctx) {
    const size_t pb = sc->nslots * kRegions * kLaneRec;
    const size_t wb = sc->nslots / 64 * 4 * sizeof(unsigned long long);
    const size_t sb = sc->stack_words > kShortStack ? sc->nslots * (size_t)sc->stack_words * sizeof(uint32_t) : 0;
    c.ctl_cap = kCtlBytes + RT_MAX_LIGHTS * 6 * sizeof(double);
    if (hipMalloc(reinterpret_cast<void**>(&c.d_ctr), c.ctl_cap) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c.h_ctl), c.ctl_cap, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c.d_pstate), pb) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c.d_wavelog), wb) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c.d_wctr), wb) != hipSuccess ||
        (sb > 0 && hipMalloc(reinterpret_cast<void**>(&c.d_spill), sb) != hipSuccess) ||
        hipMemset(c.d_ctr, 0, kCtrBytes) != hipSuccess ||
        hipEventCreate(&c.ev0) != hipSuccess || hipEventCreate(&c.ev1) != hipSuccess) {
      rt_scene_free(sc);
      return fail(RT_ERR_HIP, "allocation of launch contexts failed");
    }
    sc->bytes += (long long)(c.ctl_cap + pb + 2 * wb + sb);
  }
  *out = sc;
  return RT_OK;
}
// Defaults, then the caller's fields, validated.
int resolve_options(const rt_upload_options* opt, rt_upload_options& o) {
  upload_options_defaults(&o);
  if (!opt) return RT_OK;
  o = *opt;
  // zero-initialised fields mean their defaults (a C caller's `rt_upload_options o = {0}` or
  // designated initialiser stays valid and changes nothing but the fields it names)
  rt_upload_options d;
  upload_options_defaults(&d);
  if (o.sbvh_bins == 0) o.sbvh_bins = d.sbvh_bins;
  if (o.sbvh_c_trav == 0.0) o.sbvh_c_trav = d.sbvh_c_trav;
  if (o.collapse_c_tri == 0.0) o.collapse_c_tri = d.collapse_c_tri;
  if (o.lds_treelet < -1) return fail(RT_ERR_INVALID, "rt_scene_upload: lds_treelet must be >= -1");
  if (o.reserve_cus < -1) return fail(RT_ERR_INVALID, "rt_scene_upload: reserve_cus must be >= -1");
  if (o.order_window < -1 || o.order_window > 64)
    return fail(RT_ERR_INVALID, "rt_scene_upload: order_window must be in [-1, 64]");
  if (o.spp_lanes < -1 || o.spp_lanes > 64 || (o.spp_lanes > 1 && (o.spp_lanes & (o.spp_lanes - 1)) != 0))
    return fail(RT_ERR_INVALID, "rt_scene_upload: spp_lanes must be -1, 0, 1 or a power of two <= 64");
  if (o.stack_ring != 0 && o.stack_ring != 8 && o.stack_ring != 16)
    return fail(RT_ERR_INVALID, "rt_scene_upload: stack_ring must be 0, 8 or 16");
  if (o.blocks_per_cu < 0 || o.grid_spare < 0 || o.build_threads < 0)
    return fail(RT_ERR_INVALID, "rt_scene_upload: negative blocks_per_cu / grid_spare / build_threads");
  if (o.sbvh_leaf_max < 0 || o.sbvh_leaf_max > 8 || o.sbvh_bins < 2 || o.sbvh_bins > 128 ||
      o.sbvh_alpha != o.sbvh_alpha || o.sbvh_budget != o.sbvh_budget ||   // NaN; negative = by size
       !(o.sbvh_c_trav >= 0.0) || !(o.collapse_c_tri >= 0.0))
    return fail(RT_ERR_INVALID, "rt_scene_upload: SBVH / collapse parameter out of range");
  return RT_OK;
}
}  // namespace

extern "C" {

void rt_upload_options_init(rt_upload_options* opt) {
  if (opt) upload_options_defaults(opt);
}

int rt_scene_upload_ex(const rt_scene_soa* s, const rt_bvh_soa* b, int device, const rt_upload_options* opt,
                       rt_scene** out) {
  if (!out) return fail(RT_ERR_INVALID, "rt_scene_upload: null out");
  *out = nullptr;
  rt_upload_options o;
  int rc = resolve_options(opt, o);
  if (rc != RT_OK) return rc;
  SceneImage I;
  const auto t0 = std::chrono::steady_clock::now();
  rc = build_image(s, b, o, kTopNodes, I);
  if (rc != RT_OK) return fail(rc, build_image_error());
  const auto t1 = std::chrono::steady_clock::now();
  rc = upload_image(I, o, device, out);
  if (rc == RT_OK) {
    (*out)->build_s = std::chrono::duration<double>(t1 - t0).count();
    (*out)->copy_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
  }
  return rc;
}

int rt_scene_upload_multi(const rt_scene_soa* s, const rt_bvh_soa* b, const int* devices, int n_devices,
                          const rt_upload_options* opt, rt_scene** outs) {
  if (!outs || !devices || n_devices < 1) return fail(RT_ERR_INVALID, "rt_scene_upload_multi: bad argument");
  for (int g = 0; g < n_devices; ++g) outs[g] = nullptr;
  rt_upload_options o;
  int rc = resolve_options(opt, o);
  if (rc != RT_OK) return rc;
  SceneImage I;
  const auto t0 = std::chrono::steady_clock::now();
  rc = build_image(s, b, o, kTopNodes, I);
  if (rc != RT_OK) return fail(rc, build_image_error());
  const double build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  // one host thread per device: the copies and context allocations proceed in parallel
  std::vector<int> rcs(n_devices, RT_OK);
  std::vector<std::string> errs(n_devices);
  std::vector<std::thread> th;
  for (int g = 0; g < n_devices; ++g)
    th.emplace_back([&, g]() {
      const auto t1 = std::chrono::steady_clock::now();
      rcs[g] = upload_image(I, o, devices[g], &outs[g]);
      if (rcs[g] != RT_OK) {
        errs[g] = g_error;   // thread-local message of that thread
      } else {
        outs[g]->build_s = build_s;
        outs[g]->copy_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
      }
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

int rt_scene_upload_seconds(const rt_scene* s, double* build_s, double* copy_s) {
  if (!s) return fail(RT_ERR_INVALID, "rt_scene_upload_seconds: null scene");
  if (build_s) *build_s = s->build_s;
  if (copy_s) *copy_s = s->copy_s;
  return RT_OK;
}

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

// The CU-masked stream a launch from caller stream `caller` runs on (reserve_cus > 0): the mask
// clears the first reserve_cus CU bits, so a concurrent kernel -- an RCCL gather whose waves need
// 256 VGPRs, more than any single free block slot of the persistent grid offers -- finds whole CUs
// free.  Measured with a kernel of RCCL's resource shape (git 1a5bb03:tools/cumask_probe.py,
// profiles/r04/r04e_cumask.txt): it runs beside the grid only when the first 32 bits are clear
// (one XCD's worth); 8 or 16 CUs, or 32 spread over the mask, leave it waiting for the grid's end
// (DESIGN.md §8).
int masked_stream(rt_scene* sc, hipStream_t caller, hipStream_t* out) {
  for (int i = 0; i < sc->n_masked; ++i)
    if (sc->masked_for[i] == caller) { *out = sc->masked[i]; return RT_OK; }
  if (sc->n_masked >= rt_scene::kMaskedStreams) {
    // more caller streams than masked ones: a further caller always shares the same slot (its
    // handle hashed), so its launches stay in order on one internal stream
    const uintptr_t h = reinterpret_cast<uintptr_t>(caller);
    *out = sc->masked[(size_t)((h >> 4) ^ (h >> 12)) % rt_scene::kMaskedStreams];
    return RT_OK;
  }
  std::vector<uint32_t> mask((size_t)(sc->n_cu + 31) / 32, 0u);
  for (int c = sc->reserve_cus; c < sc->n_cu; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
  hipStream_t s = nullptr;
  // cuMaskSize counts uint32 words of the mask (as hipExtStreamGetCUMask's does)
  HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  {   // read the mask back: the stream must leave exactly the first reserve_cus CUs free
    std::vector<uint32_t> got(mask.size(), 0u);
    const hipError_t e = hipExtStreamGetCUMask(s, (uint32_t)got.size(), got.data());
    if (e != hipSuccess || got != mask) {
      (void)hipStreamDestroy(s);
      return fail(RT_ERR_HIP, e != hipSuccess ? "hipExtStreamGetCUMask failed"
                                              : "reserve_cus: the CU-masked stream did not take the requested mask");
    }
  }
  sc->masked[sc->n_masked] = s;
  sc->masked_for[sc->n_masked] = caller;
  sc->n_masked++;
  *out = s;
  return RT_OK;
}

// One render launch; list != nullptr: adaptive pass over the pixel ids list[0 .. *count)
// (at most list_cap of them) of the full frame.
// n_frames > 1 (rt_launch_frames): params p[0..n_frames) differ only in their camera vectors,
// frame f is written to outs[f].
// Has the work before event e finished?  hipErrorNotReady from the query is an answer, not a
// failure; should a HIP runtime keep it as the last error, it is taken back out, so a caller's later
// error check (torch's launch checks) does not report it (ROCm 7 on the MI355X box does not keep it:
// tools/notready_probe.py, profiles/r05/r05zzh_notready.txt)
static bool event_done(hipEvent_t e) {
  const hipError_t q = hipEventQuery(e);
  if (q == hipErrorNotReady && hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();
  return q == hipSuccess;
}

// Has a launch on this scene tripped a kernel watchdog (the CHECK-and-continue the reference has,
// common/common.h:6-15, made an error)?  The kernel writes the flag into page-locked host memory
// at system scope, so this sees launches that ended without stats, whatever their stream.
const char* const kGuardMsg =
    "a launch on this scene tripped the kernel watchdog (cyclic or corrupt hierarchy, or a kernel bug): "
    "its pixels and every later result of this scene are void";
static bool guard_tripped(const rt_scene* sc) {
  return sc->h_guard && *reinterpret_cast<const volatile unsigned int*>(sc->h_guard) != 0u;
}

// Sample groups for this launch (spp > 1, n^2 a power of two, rt_upload_options.spp_lanes): a pixel's
// samples on neighbouring lanes, summed in order on chip.  The tile-cost maps record per-lane pixel
// costs and the diagnostic variants have no group instance, so those launches keep one lane per pixel.
bool use_groups(const rt_scene* sc, const rt_render_params* p) {
  const int nsamp = p->spp_n * p->spp_n;
  return nsamp > 1 && (nsamp & (nsamp - 1)) == 0 && (sc->spp_lanes > 0 || (sc->spp_lanes == 0 && kSppLanesDefault)) &&
         !(p->flags & (RT_FLAG_COST_ORDER | RT_FLAG_TRAVERSAL_STATS | RT_FLAG_WIDE_STATS | RT_FLAG_TIMELINE |
                       RT_FLAG_TILE_COST | RT_FLAG_TILE_COST_TIME));
}

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
  if (guard_tripped(sc)) return fail(RT_ERR_HIP, kGuardMsg);

  KParams P;
  std::memset(&P, 0, sizeof P);
  P.nodes = sc->d_nodes; P.nodes4 = sc->d_nodes4; P.tris = sc->d_tris; P.slot2dev = sc->d_slot2dev; P.shade = sc->d_shade; P.tnorm = sc->d_tnorm;
  P.tu = sc->d_tu; P.tv = sc->d_tv; P.texels = sc->d_texels; P.mats = sc->d_mats;
  P.prims = sc->d_prims; P.n_prims = sc->n_prims;
  LaunchCtx& C = sc->ctx[sc->next_ctx];
  const int ci = sc->next_ctx;
  // reserve_cus: everything of this launch goes to the caller's CU-masked stream, joined to the
  // caller's stream by events (in: after the caller's prior work; out: the caller waits for the end)
  const hipStream_t caller = st;
  if (sc->reserve_cus > 0) {
    hipStream_t ks = nullptr;
    const int mrc = masked_stream(sc, caller, &ks);
    if (mrc != RT_OK) return mrc;
    if (!C.ev_in) HIP_TRY(hipEventCreateWithFlags(&C.ev_in, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(C.ev_in, caller));
    HIP_TRY(hipStreamWaitEvent(ks, C.ev_in, 0));
    st = ks;
  }
  // the context's previous launch done (device side) and its staged copy consumed (host side); a
  // launch eight back has normally ended, and then no wait goes into the stream
  // (with the events below: one frame per call 0.4130 -> 0.4089 ms kernel, 0.4295 -> 0.4265 ms call; r05p)
  if (C.used && !event_done(C.ev1)) {
    HIP_TRY(hipStreamWaitEvent(st, C.ev1, 0));
    HIP_TRY(hipEventSynchronize(C.ev1));
  }
  // control block of this launch: counters, frame table, light table (grown for a larger light
  // table; the context is idle here, so its old buffers can go)
  const size_t lights_at = kCtrBytes + (size_t)n_frames * sizeof(FrameDesc);
  const size_t ctl_bytes = lights_at + (size_t)p->n_lights * 6 * sizeof(double);
  if (ctl_bytes > C.ctl_cap) {
    HIP_TRY(hipFree(C.d_ctr));
    C.d_ctr = nullptr;
    HIP_TRY(hipHostFree(C.h_ctl));
    C.h_ctl = nullptr;
    sc->bytes -= (long long)C.ctl_cap;
    C.ctl_cap = 0;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&C.d_ctr), ctl_bytes));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&C.h_ctl), ctl_bytes, hipHostMallocDefault));
    C.ctl_cap = ctl_bytes;
    sc->bytes += (long long)ctl_bytes;
  }
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
  // lights: in this launch's control block, staged with its counters and frame table (the
  // reference copies them on every call too, mytracer.cpp:105-118); no device-wide synchronisation,
  // so launches on other streams with other lights run on
  P.lights = reinterpret_cast<const double*>(reinterpret_cast<unsigned char*>(C.d_ctr) + lights_at);
  P.guard_host = sc->d_guard;
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
  P.out_global = (p->flags & RT_FLAG_GLOBAL_ROWS) ? 1 : 0;
  if (P.out_global && list) return fail(RT_ERR_INVALID, "RT_FLAG_GLOBAL_ROWS is not supported by the adaptive pass");
  P.tiles_x = (P.W + kTileW - 1) / kTileW;
  P.nsamp = p->spp_n * p->spp_n;
  // sample groups (spp > 1): a pixel's samples on G = min(n^2, 32) neighbouring lanes (use_groups);
  // in list mode (the adaptive pass) the caller chose it: no sample buffer
  const bool group = list ? sample_out == nullptr : use_groups(sc, p);
  if (group) {
    P.group_log = 0;
    // G = min(n^2, kGroupLanes), or the group-size cap spp_lanes >= 2 (chunks of G samples, the
    // running sum in the path state between them)
    const int gmax = sc->spp_lanes >= 2 ? sc->spp_lanes : kGroupLanes;
    while ((1 << (P.group_log + 1)) <= std::min(P.nsamp, gmax)) P.group_log++;
    P.chunks = P.nsamp >> P.group_log;
  }
  P.frame_tiles = list ? (list_cap * (group ? 1 : P.nsamp) + 63) / 64
                       : (long long)P.tiles_x * ((rows + kTileH - 1) / kTileH);
  // (list mode: one list holds every frame's items, list_cap counts them all)
  P.n_tiles = list ? P.frame_tiles : P.frame_tiles * n_frames;
  if (P.n_tiles >= (1LL << 31)) return fail(RT_ERR_INVALID, "rt_launch: more than 2^31 tiles in one launch");
  P.div_row_tiles = div_magic((uint32_t)P.tiles_x * (uint32_t)n_frames);
  P.div_tiles_x = div_magic((uint32_t)P.tiles_x);
  P.div_stripe_h = div_magic((uint32_t)P.stripe_h);
  P.list = list;
  P.list_count = count;
  P.sample_out = sample_out;
  if (!list && sc->d_tile_order && sc->tile_order_n == P.n_tiles) P.tile_order = sc->d_tile_order;
  // cost-ordered work (one-frame launches): ordered by the costs of the launch before the previous
  // one of the same geometry, while this launch's costs are recorded
  // (several frames per launch: natural order and no cost map -- the same tile position of every
  // frame finishing together made the cost atomics contend: +57-86 % on 20-frame launches)
  // The library default for one-frame launches (the reference's use) when they follow each other on
  // one stream: implicit, so it never adds a cross-stream dependency; explicit RT_FLAG_COST_ORDER
  // also orders launches on other streams (each then waits for the previous launch's end).
  // Diagnostics, a debug order and RT_FLAG_NATURAL_ORDER keep the natural order.
  const bool debug_order = sc->d_tile_order && sc->tile_order_n == P.n_tiles;
  // (implicit: only on the stream of the last launch that touched the maps, so stream order fences
  // it against that launch's reads and its drain's writes of the maps -- whatever ran on other
  // streams in between)
  const bool implicit_order =
      !(p->flags & (RT_FLAG_TRAVERSAL_STATS | RT_FLAG_WIDE_STATS | RT_FLAG_TIMELINE | RT_FLAG_TILE_COST |
                    RT_FLAG_TILE_COST_TIME | RT_FLAG_NATURAL_ORDER)) &&
      !debug_order && (!sc->maps_used || sc->maps_stream == st);
  const bool cost_debug = !list && (p->flags & (RT_FLAG_TILE_COST | RT_FLAG_TILE_COST_TIME));
  const bool cost_order = !list && !group && n_frames == 1 && ((p->flags & RT_FLAG_COST_ORDER) || implicit_order);
  if (cost_order || cost_debug) {
    const long long n_pos = (long long)P.tiles_x * ((rows + kTileH - 1) / kTileH);
    if (sc->cost_cap < n_pos) {
      HIP_TRY(hipDeviceSynchronize());   // launches in flight may still use the old buffers
      for (uint32_t*& q : sc->d_cost) { if (q) HIP_TRY(hipFree(q)); q = nullptr; }
      for (uint32_t*& q : sc->d_order) { if (q) HIP_TRY(hipFree(q)); q = nullptr; }
      sc->cost_cap = 0;
      for (uint32_t*& q : sc->d_cost) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&q), (size_t)n_pos * sizeof(uint32_t)));
      for (uint32_t*& q : sc->d_order) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&q), (size_t)n_pos * sizeof(uint32_t)));
      sc->cost_cap = n_pos;
      sc->cost_seq = 0;
      sc->order_for = -1;
    }
    if (sc->cost_n != n_pos || sc->cost_tiles_x != P.tiles_x) {   // another geometry: a new sequence
      sc->cost_seq = 0;
      sc->order_for = -1;   // (an order built for the old geometry is no permutation of this one)
    }
    sc->cost_n = n_pos;
    sc->cost_tiles_x = P.tiles_x;
    if (sc->maps_used && sc->maps_stream != st)   // the last map launch (another stream) is done with the maps
      HIP_TRY(hipStreamWaitEvent(st, sc->maps_ev, 0));
    // cost unit: pixel lifetime (RT_FLAG_TILE_COST_TIME, and RT_FLAG_COST_ORDER alone) or bounces
    // (RT_FLAG_TILE_COST, also with RT_FLAG_COST_ORDER)
    P.cost_time = (p->flags & RT_FLAG_TILE_COST) ? 0 : 1;
    if (!cost_order) {   // diagnostics: a fresh map, the first launch of a new sequence
      sc->cost_seq = 0;
      HIP_TRY(hipMemsetAsync(sc->d_cost[0], 0, (size_t)n_pos * sizeof(uint32_t), st));
      P.tile_cost = sc->d_cost[0];
      sc->cost_seq = 1;
      sc->order_for = -1;
    } else {
      const long long q = sc->cost_seq;
      if (q == 0)
        for (uint32_t* m : sc->d_cost) HIP_TRY(hipMemsetAsync(m, 0, (size_t)n_pos * sizeof(uint32_t), st));
      P.tile_cost = sc->d_cost[q % 3];
      if (sc->order_for == q && n_pos == P.n_tiles) {
        P.tile_order = sc->d_order[q % 2];
        sc->last_order_n = P.n_tiles;
        sc->last_order_buf = (int)(q % 2);
      }
      if ((n_pos + kGroups - 1) / kGroups <= kOrderMaxRange) {   // the drain jobs: next order, next map cleared
        P.order_src = q >= 1 ? sc->d_cost[(q + 2) % 3] : nullptr;
        P.order_dilate = sc->order_window > 0 ? sc->order_window : sc->order_window < 0 ? 0
                         : sc->big ? 0 : kOrderDilate;
        P.next_order = sc->d_order[(q + 1) % 2];
        P.zero_map = sc->d_cost[(q + 1) % 3];
        P.n_pos = n_pos;
        if (q >= 1) sc->order_for = q + 1;
      } else {
        HIP_TRY(hipMemsetAsync(sc->d_cost[(q + 1) % 3], 0, (size_t)n_pos * sizeof(uint32_t), st));
      }
      sc->cost_seq = q + 1;
    }
  }

  const int v = (p->flags & RT_FLAG_TRAVERSAL_STATS) ? 2
                : (p->flags & RT_FLAG_WIDE_STATS) ? 1
                : (p->flags & RT_FLAG_TIMELINE) ? 3
                : sc->deep ? (group ? 6 : 4)   // the 16-entry-ring production variant
                : group ? 5 : 0;
  const int ring = variant_ring(v);
  const int n_top = sc->n_top_v[v];
  const size_t lds = lds_bytes_total(sc->stack_words, n_top, ring);
  P.n_top = n_top;
  P.top_off = (int)lds_bytes(sc->stack_words, ring);
  P.lights_off = P.top_off + n_top * (int)sizeof(GNode4);
  P.pool_off = P.lights_off + RT_MAX_LIGHTS * 6 * (int)sizeof(double);
  const long long waves_needed = (P.n_tiles * 64 + 63) / 64;
  int bpc = sc->blocks_per_cu[v];
  if (sc->bpc_cap > 0) bpc = std::min(bpc, sc->bpc_cap);   // a smaller persistent grid (upload option)
  auto grid_of = [&](int bpc_) {
    long long b = (long long)(sc->n_cu - sc->reserve_cus) * bpc_;
    b = std::max<long long>(1, std::min<long long>(b, (waves_needed + kBlock / 64 - 1) / (kBlock / 64)));
    b = std::min<long long>(b, (long long)(sc->nslots / kBlock));
    if (sc->grid_spare > 0)   // leave block slots to concurrent kernels (upload option)
      b = std::max<long long>(1, b - sc->grid_spare);
    return b;
  };
  const long long full_blocks = grid_of(bpc);
  // one-frame launches in flight on several streams (a caller pipelining the reference's call
  // shape): while the previous launch, on another stream, still runs, this one takes half the
  // block slots, so two launches are co-resident and each one's drain runs beside the other's work
  // (3 in flight: 0.334 -> 0.325 ms per frame at half grids, r05zzb; multi-frame launches in
  // flight lose with half grids, r05zzc, and keep the whole grid).  Pixels and counts do not depend
  // on the grid; the grid used is recorded (rt_debug_last_grid)
  if (n_frames == 1 && sc->last_ctx >= 0 && sc->last_stream != st &&
      !event_done(sc->ctx[sc->last_ctx].ev1))
    bpc = std::max(1, bpc / 2);
  const long long blocks = grid_of(bpc);

  // zeroed counters + frame table + light table, one copy from the context's pinned staging
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
  double* ld = reinterpret_cast<double*>(C.h_ctl + lights_at);
  for (int i = 0; i < p->n_lights; ++i) {
    const rt_light* L = rt_params_light(p, i);
    for (int k = 0; k < 3; ++k) { ld[6 * i + k] = L->position[k]; ld[6 * i + 3 + k] = L->color[k]; }
  }
  HIP_TRY(hipMemcpyAsync(C.d_ctr, C.h_ctl, ctl_bytes, hipMemcpyHostToDevice, st));
  if (v == 3) {   // round timeline: zeroed, so unused records read as t = 0
    const size_t tb = sc->nslots / 64 * kTlCap * kTlWords * sizeof(unsigned long long);
    if (!C.d_tl) {
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&C.d_tl), tb));
      sc->bytes += (long long)tb;
    }
    HIP_TRY(hipMemsetAsync(C.d_tl, 0, tb, st));
  }
  P.tl = C.d_tl;
  if (rows > 0) {   // the launch's start / stop events travel with the kernel's dispatch (no marker packets)
    void* args[] = {&P};
    HIP_TRY(hipExtLaunchKernel(reinterpret_cast<const void*>(kVariants[v].fn), dim3((unsigned)blocks), dim3(kBlock),
                               args, lds, st, C.ev0, C.ev1, 0));
  } else {
    HIP_TRY(hipEventRecord(C.ev0, st));
    HIP_TRY(hipEventRecord(C.ev1, st));
  }
  if (st != caller) HIP_TRY(hipStreamWaitEvent(caller, C.ev1, 0));   // the caller's later work follows the launch
  if (cost_order || cost_debug) {   // this launch read / wrote the maps: the next map launch is fenced on it
    if (!sc->maps_ev) HIP_TRY(hipEventCreateWithFlags(&sc->maps_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(sc->maps_ev, st));
    sc->maps_used = true;
    sc->maps_stream = st;
  }
  C.used = true;
  C.variant = v;
  C.waves = rows > 0 ? blocks * (kBlock / 64) : 0;
  C.blocks = rows > 0 ? blocks : 0;
  C.full_blocks = rows > 0 ? full_blocks : 0;
  sc->last_ctx = ci;
  sc->last_stream = st;
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
    // pixels written: every pixel of the shard per frame; in list mode (adaptive pass) the
    // listed pixels, which the reduce kernel writes after this launch
    if (list) {
      unsigned long long n_list = 0;
      HIP_TRY(hipMemcpy(&n_list, count, sizeof n_list, hipMemcpyDeviceToHost));
      stats->pixels = (long long)std::min<unsigned long long>(n_list, (unsigned long long)std::max(0LL, list_cap));
    } else {
      stats->pixels = (long long)rows * p->camera.width * n_frames;
    }
    if (c[CD_GUARD] != 0 || guard_tripped(sc)) return fail(RT_ERR_HIP, kGuardMsg);
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
  rt_render_params q = *p;
  q.spp_n = subp;
  // sample groups: a selected pixel's subp^2 samples on neighbouring lanes, summed in order and stored
  // by the render kernel itself -- no sample buffer, no reduce kernel
  const bool grp = use_groups(sc, &q);
  StreamScratch scratch{st, {}};
  HIP_TRY(scratch.alloc(&list, (size_t)std::max(1LL, cap) * sizeof(uint32_t)));
  HIP_TRY(scratch.alloc(&cnt, sizeof(unsigned long long)));
  if (!grp) HIP_TRY(scratch.alloc(&samples, (size_t)std::max(1LL, cap) * nsamp * 3 * sizeof(double)));
  HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), st));
  const int tiles_x = (W + 7) / 8;
  const long long n_tiles = (long long)tiles_x * ((G.rows + 7) / 8);
  if (n_tiles > 0) {
    hipLaunchKernelGGL(adaptive_select_kernel, dim3((unsigned)((n_tiles + kSelTilesPerBlock - 1) / kSelTilesPerBlock)),
                       dim3(kSelThreads), 0, st, d_primary,
                       d_halo, d_out, p->out_format, G, threshold, tiles_x, n_tiles, list, cnt, 0u, nullptr, nullptr);
    HIP_TRY(hipGetLastError());
  }
  int rc = launch_render(sc, &q, 1, &d_out, stats, stream, list, cnt, cap, samples);
  if (rc == RT_OK && cap > 0 && !grp) {
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
  // every sample of every selected pixel of every frame in one launch.  Sample groups (use_groups):
  // the render kernel sums and stores each pixel itself, its work count read on the device -- nothing
  // to size, no host synchronisation; otherwise the sample buffer is sized by the selection count
  // (read back: one synchronisation per batch) and a reduce kernel sums it
  std::vector<rt_render_params> q(p, p + n_frames);
  for (auto& x : q) x.spp_n = subp;
  const bool grp = use_groups(sc, &q[0]);
  const int nsamp = subp * subp;
  unsigned long long n_sel = 0;
  double* samples = nullptr;
  if (!grp) {
    HIP_TRY(hipMemcpyAsync(&n_sel, cnt, sizeof n_sel, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(scratch.alloc(&samples, (size_t)std::max(1ull, n_sel) * nsamp * 3 * sizeof(double)));
  }
  int rc = launch_render(sc, q.data(), n_frames, d_out, stats, stream, list, cnt, grp ? cap : (long long)n_sel, samples);
  if (rc == RT_OK && grp && n_selected) {
    HIP_TRY(hipMemcpyAsync(&n_sel, cnt, sizeof n_sel, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  if (rc == RT_OK && !grp && n_sel > 0) {   // sums in (si, sj) order into each frame's output (this call's table)
    hipLaunchKernelGGL(adaptive_reduce_kernel, dim3((unsigned)((n_sel + 255) / 256)), dim3(256), 0, st, list, cnt,
                       samples, nsamp, nullptr, p->out_format, d_ptrs + n_frames);
    HIP_TRY(hipGetLastError());
  }
  if (n_selected) *n_selected = (long long)n_sel;
  return rc;
}

int rt_render_to_host(rt_scene* sc, const rt_render_params* p, void* host_out, rt_stats* stats) {
  if (!sc || !p || !host_out) return fail(RT_ERR_INVALID, "rt_render_to_host: null argument");
  // the host buffer holds the shard's packed rows (rt_rows_in_shard): a frame-sized layout would
  // overrun it (and the pageable path's shard-sized staging buffer)
  if (p->flags & RT_FLAG_GLOBAL_ROWS)
    return fail(RT_ERR_INVALID, "rt_render_to_host: RT_FLAG_GLOBAL_ROWS is not supported (the output is the packed shard)");
  HIP_TRY(hipSetDevice(sc->device));
  const int rows = rt_rows_in_shard(p);
  const size_t elem = p->out_format == RT_OUT_RGB_F64 ? sizeof(double) : sizeof(float);
  const size_t bytes = std::max<size_t>(1, (size_t)rows * p->camera.width * 3 * elem);
  rt_stats local;   // (the stats path synchronises and checks the watchdog word)
  // page-locked, device-mapped caller buffer (hipHostMalloc, torch pin_memory, hipHostRegister): the
  // kernel stores the frame straight into it over PCIe as pixels finish -- no staging buffer, and the
  // transfer overlaps the render (office 1080p: 1.18 -> 0.81 ms per call, DESIGN.md §5 "Host-buffer rate")
  hipPointerAttribute_t at;
  void* direct = nullptr;
  if (hipPointerGetAttributes(&at, host_out) == hipSuccess && at.type == hipMemoryTypeHost) {
    if (hipHostGetDevicePointer(&direct, host_out, 0) != hipSuccess) direct = nullptr;
  }
  (void)hipGetLastError();   // pageable memory: the queries above fail, which is not an error here
  if (direct) return rt_launch_compute_image(sc, p, direct, stats ? stats : &local, nullptr);
  // pageable: render into the scene's staging buffer (kept between calls), then one copy
  if (sc->host_stage_bytes < bytes) {
    if (sc->d_host_stage) HIP_TRY(hipFree(sc->d_host_stage));
    sc->d_host_stage = nullptr;
    sc->host_stage_bytes = 0;
    HIP_TRY(hipMalloc(&sc->d_host_stage, bytes));
    sc->host_stage_bytes = bytes;
  }
  int rc = rt_launch_compute_image(sc, p, sc->d_host_stage, stats ? stats : &local, nullptr);
  if (rc == RT_OK) {
    const hipError_t e = hipMemcpy(host_out, sc->d_host_stage, (size_t)rows * p->camera.width * 3 * elem,
                                   hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(RT_ERR_HIP, std::string("hipMemcpy D2H: ") + hipGetErrorString(e));
  }
  return rc;
}

int rt_render_adaptive_to_host(rt_scene* sc, const rt_render_params* p, int subp, double threshold, void* host_out,
                               rt_stats* st_primary, rt_stats* st_adaptive, long long* n_selected) {
  if (!sc || !p || !host_out) return fail(RT_ERR_INVALID, "rt_render_adaptive_to_host: null argument");
  if (p->flags & RT_FLAG_GLOBAL_ROWS)
    return fail(RT_ERR_INVALID, "rt_render_adaptive_to_host: RT_FLAG_GLOBAL_ROWS is not supported");
  const int W = p->camera.width, H = p->camera.height;
  if (W <= 0 || H <= 0) return fail(RT_ERR_INVALID, "bad image size");
  if (p->stripe_count > 1 || p->row_begin != 0 || (p->row_end > 0 && p->row_end != H))
    return fail(RT_ERR_INVALID, "rt_render_adaptive_to_host: needs the full frame (neighbour test), no stripes/row range");
  if (p->out_format != RT_OUT_RGB_F32 && p->out_format != RT_OUT_RGB_F64) return fail(RT_ERR_INVALID, "bad out_format");
  HIP_TRY(hipSetDevice(sc->device));
  const size_t elem = p->out_format == RT_OUT_RGB_F64 ? sizeof(double) : sizeof(float);
  const size_t bytes = (size_t)H * W * 3 * elem;
  // the primary pass in fp64 (the selection compares fp64 colours, mytracer_gpu.cu:66-81), into
  // stream-ordered scratch on the null stream
  StreamScratch scratch{nullptr, {}};
  double* prim = nullptr;
  HIP_TRY(scratch.alloc(&prim, (size_t)H * W * 3 * sizeof(double)));
  rt_render_params q = *p;
  q.out_format = RT_OUT_RGB_F64;
  int rc = rt_launch_compute_image(sc, &q, prim, st_primary, nullptr);
  if (rc != RT_OK) return rc;
  // the adaptive pass (mytracer_gpu.cu:83-109) writes every pixel of the output: straight into a
  // page-locked, device-mapped caller buffer, else into the scene's staging buffer and one copy
  hipPointerAttribute_t at;
  void* direct = nullptr;
  if (hipPointerGetAttributes(&at, host_out) == hipSuccess && at.type == hipMemoryTypeHost) {
    if (hipHostGetDevicePointer(&direct, host_out, 0) != hipSuccess) direct = nullptr;
  }
  (void)hipGetLastError();   // pageable memory: the queries above fail, which is not an error here
  if (!direct && sc->host_stage_bytes < bytes) {
    HIP_TRY(hipDeviceSynchronize());   // an earlier call's copy may still read the old buffer
    if (sc->d_host_stage) HIP_TRY(hipFree(sc->d_host_stage));
    sc->d_host_stage = nullptr;
    sc->host_stage_bytes = 0;
    HIP_TRY(hipMalloc(&sc->d_host_stage, bytes));
    sc->host_stage_bytes = bytes;
  }
  rc = rt_launch_adaptive(sc, p, prim, direct ? direct : sc->d_host_stage, subp, threshold, st_adaptive, n_selected,
                          nullptr);
  if (rc != RT_OK) return rc;
  if (!direct) {
    const hipError_t e = hipMemcpy(host_out, sc->d_host_stage, bytes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("hipMemcpy D2H: ") + hipGetErrorString(e));
  } else {
    HIP_TRY(hipStreamSynchronize(nullptr));
  }
  if (guard_tripped(sc)) return fail(RT_ERR_HIP, kGuardMsg);
  return RT_OK;
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

long long rt_debug_tile_cost(rt_scene* sc, unsigned int* out, long long n) {
  if (!sc) return fail(RT_ERR_INVALID, "rt_debug_tile_cost: null scene");
  if (sc->cost_seq < 1) return 0;
  if (hipSetDevice(sc->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return fail(RT_ERR_HIP, "rt_debug_tile_cost: synchronize failed");
  const long long m = std::min(n, sc->cost_n);
  if (out && m > 0 &&
      hipMemcpy(out, sc->d_cost[(sc->cost_seq - 1) % 3], (size_t)m * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
    return fail(RT_ERR_HIP, "rt_debug_tile_cost: copy failed");
  return sc->cost_n;
}

long long rt_debug_last_tile_order(rt_scene* sc, unsigned int* out, long long n) {
  if (!sc) return fail(RT_ERR_INVALID, "rt_debug_last_tile_order: null scene");
  if (!sc->d_order[0] || sc->last_order_n <= 0) return 0;
  if (hipSetDevice(sc->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return fail(RT_ERR_HIP, "rt_debug_last_tile_order: synchronize failed");
  const long long m = std::min(n, sc->last_order_n);
  if (out && m > 0 &&
      hipMemcpy(out, sc->d_order[sc->last_order_buf], (size_t)m * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
    return fail(RT_ERR_HIP, "rt_debug_last_tile_order: copy failed");
  return sc->last_order_n;
}

int rt_debug_set_tile_order(rt_scene* sc, const unsigned int* order, long long n) {
  if (!sc || n < 0 || (n > 0 && !order)) return fail(RT_ERR_INVALID, "rt_debug_set_tile_order: bad argument");
  if (hipSetDevice(sc->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return fail(RT_ERR_HIP, "rt_debug_set_tile_order: synchronize failed");
  {   // a permutation: every index below n exactly once (a duplicate would render a tile twice and
      // leave another unwritten)
    std::vector<bool> seen((size_t)n, false);
    for (long long i = 0; i < n; ++i) {
      if ((long long)order[i] >= n || seen[order[i]])
        return fail(RT_ERR_INVALID, "rt_debug_set_tile_order: not a permutation");
      seen[order[i]] = true;
    }
  }
  if (sc->d_tile_order) (void)hipFree(sc->d_tile_order);
  sc->d_tile_order = nullptr;
  sc->tile_order_n = 0;
  if (n == 0) return RT_OK;
  if (hipMalloc(reinterpret_cast<void**>(&sc->d_tile_order), (size_t)n * sizeof(uint32_t)) != hipSuccess ||
      hipMemcpy(sc->d_tile_order, order, (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess)
    return fail(RT_ERR_HIP, "rt_debug_set_tile_order: upload failed");
  sc->tile_order_n = n;
  return RT_OK;
}

long long rt_debug_timeline(rt_scene* sc, unsigned long long* out, long long n) {
  if (!sc || !out || n <= 0) return fail(RT_ERR_INVALID, "rt_debug_timeline: bad argument");
  HIP_TRY(hipSetDevice(sc->device));
  HIP_TRY(hipDeviceSynchronize());
  if (sc->last_ctx < 0 || !sc->ctx[sc->last_ctx].d_tl || sc->ctx[sc->last_ctx].variant != 3)
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

int rt_tile_shape(int* tile_w, int* tile_h) {
  if (!tile_w || !tile_h) return fail(RT_ERR_INVALID, "rt_tile_shape: null argument");
  *tile_w = kTileW;
  *tile_h = kTileH;
  return RT_OK;
}

int rt_ipc_get_handle(const void* d_ptr, unsigned char* handle, unsigned long long* offset) {
  if (!d_ptr || !handle || !offset) return fail(RT_ERR_INVALID, "rt_ipc_get_handle: null argument");
  static_assert(sizeof(hipIpcMemHandle_t) == RT_IPC_HANDLE_BYTES, "IPC handle size");
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  HIP_TRY(hipMemGetAddressRange(&base, &size, const_cast<void*>(d_ptr)));
  hipIpcMemHandle_t h;
  HIP_TRY(hipIpcGetMemHandle(&h, base));
  std::memcpy(handle, &h, sizeof h);
  *offset = (unsigned long long)(reinterpret_cast<const char*>(d_ptr) - reinterpret_cast<const char*>(base));
  return RT_OK;
}

int rt_ipc_open(const unsigned char* handle, unsigned long long offset, int device, int owner_device, void** d_ptr) {
  if (!handle || !d_ptr) return fail(RT_ERR_INVALID, "rt_ipc_open: null argument");
  *d_ptr = nullptr;
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof h);
  HIP_TRY(hipSetDevice(device));
  if (owner_device >= 0 && owner_device != device) {   // kernels on `device` will access the owner's memory
    int can = 0;
    HIP_TRY(hipDeviceCanAccessPeer(&can, device, owner_device));
    if (!can) return fail(RT_ERR_UNSUPPORTED, "rt_ipc_open: the device cannot access the owner device's memory");
    const hipError_t e = hipDeviceEnablePeerAccess(owner_device, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
      return fail(RT_ERR_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
    (void)hipGetLastError();   // clear an already-enabled status
  }
  void* base = nullptr;
  HIP_TRY(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess));
  *d_ptr = reinterpret_cast<char*>(base) + offset;
  return RT_OK;
}

int rt_ipc_close(void* d_ptr, unsigned long long offset) {
  if (!d_ptr) return fail(RT_ERR_INVALID, "rt_ipc_close: null pointer");
  HIP_TRY(hipIpcCloseMemHandle(reinterpret_cast<char*>(d_ptr) - offset));
  return RT_OK;
}

int rt_last_kernel_ms(rt_scene* sc, float* ms) {
  if (!sc || !ms || sc->last_ctx < 0) return fail(RT_ERR_INVALID, "rt_last_kernel_ms: no launch recorded");
  const LaunchCtx& C = sc->ctx[sc->last_ctx];
  HIP_TRY(hipEventSynchronize(C.ev1));
  HIP_TRY(hipEventElapsedTime(ms, C.ev0, C.ev1));
  if (guard_tripped(sc)) return fail(RT_ERR_HIP, kGuardMsg);
  return RT_OK;
}

int rt_scene_status(const rt_scene* sc) {
  if (!sc) return fail(RT_ERR_INVALID, "rt_scene_status: null scene");
  return guard_tripped(sc) ? fail(RT_ERR_HIP, kGuardMsg) : RT_OK;
}

int rt_debug_last_grid(rt_scene* sc, long long* blocks, long long* full_blocks) {
  if (!sc || sc->last_ctx < 0) return fail(RT_ERR_INVALID, "rt_debug_last_grid: no launch recorded");
  const LaunchCtx& C = sc->ctx[sc->last_ctx];
  if (blocks) *blocks = C.blocks;
  if (full_blocks) *full_blocks = C.full_blocks;
  return RT_OK;
}

int rt_debug_corrupt_hierarchy(rt_scene* sc) {
  if (!sc) return fail(RT_ERR_INVALID, "rt_debug_corrupt_hierarchy: null scene");
  if (sc->n_gnodes4 < 1) return fail(RT_ERR_INVALID, "rt_debug_corrupt_hierarchy: the scene has no 4-wide node");
  HIP_TRY(hipSetDevice(sc->device));
  HIP_TRY(hipDeviceSynchronize());   // launches in flight read the hierarchy
  // node 0 becomes a cycle that never grows the stack: one child, node 0 itself, whose box holds
  // every ray; the other slots empty ([+inf, -inf], kEmpty)
  GNode4 n;
  std::memset(&n, 0, sizeof n);
  for (int c = 0; c < 4; ++c) {
    const float lo = c == 0 ? -1e30f : INFINITY, hi = c == 0 ? 1e30f : -INFINITY;
    n.lox[c] = n.loy[c] = n.loz[c] = lo;
    n.hix[c] = n.hiy[c] = n.hiz[c] = hi;
    n.ref[c] = c == 0 ? 0u : kEmpty;
  }
  HIP_TRY(hipMemcpy(sc->d_nodes4, &n, sizeof n, hipMemcpyHostToDevice));
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
  void* ptrs[] = {sc->d_cost[0], sc->d_cost[1], sc->d_cost[2], sc->d_order[0], sc->d_order[1], sc->d_tile_order, sc->d_host_stage, sc->d_nodes, sc->d_nodes4, sc->d_tris, sc->d_shade, sc->d_tnorm, sc->d_tu,
                  sc->d_tv, sc->d_texels, sc->d_mats, sc->d_slot2dev, sc->d_prims};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (sc->h_guard) (void)hipHostFree(sc->h_guard);
  for (LaunchCtx& c : sc->ctx) {
    void* cp[] = {c.d_ctr, c.d_pstate, c.d_spill, c.d_wavelog, c.d_tl, c.d_wctr};
    for (void* q : cp)
      if (q) (void)hipFree(q);
    if (c.h_ctl) (void)hipHostFree(c.h_ctl);
    if (c.ev0) (void)hipEventDestroy(c.ev0);
    if (c.ev1) (void)hipEventDestroy(c.ev1);
  }
  if (sc->maps_ev) (void)hipEventDestroy(sc->maps_ev);
  for (LaunchCtx& c : sc->ctx)
    if (c.ev_in) (void)hipEventDestroy(c.ev_in);
  for (int i = 0; i < rt_scene::kMaskedStreams; ++i)
    if (sc->masked[i]) (void)hipStreamDestroy(sc->masked[i]);
  delete sc;
}

}  // extern "C"
