// device_image.cpp — host builders of the device layout (device_image.hpp).
//
// Moved out of the HIP translation unit: everything here runs on the host once per upload.
//   * build_device_tree: the reference median-split tree (mybvh.cpp:375-539) node for node, with
//     reference leaves of more than kLeafMax triangles refined (RT_TREE_REFERENCE);
//   * build_sah_tree: binned SAH over all triangles (RT_TREE_SAH);
//   * build_sbvh_tree: binned SAH with spatial splits (RT_TREE_SBVH, the default);
//   * build_image: 2-wide canonical nodes over the reference tree, the 4-wide collapse of the
//     device tree (breadth-first treelet prefix, preorder below), conservative fp32 boxes
//     (outward rounding + delta growth), fp64 triangle / shading records in device order.
// Parallel builds partition work so the result never depends on the thread count (tested).
#include "device_image.hpp"

#include <algorithm>
#include <array>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <deque>
#include <sched.h>
#include <string>
#include <thread>
#include <vector>

namespace rtk {
namespace {

thread_local std::string g_build_error;

int fail(int code, const std::string& msg) {
  g_build_error = msg;
  return code;
}

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
thread_local int g_threads = 1;   // build threads of the current build_image call (from the options)
int sah_threads() { return g_threads; }

// CPUs this process may run on: its affinity mask, capped by a cgroup v2 CPU quota (cpu.max
// "quota period"); a GPU box's job sees the whole node in hardware_concurrency() but may use
// only its share (16 CPUs per GPU there).
int usable_cpus() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long per = 0;
    if (std::fscanf(f, "%31s %lld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
      const long long quota = std::atoll(q);
      if (quota > 0) n = std::min<long long>(n, std::max(1LL, quota / per));
    }
    std::fclose(f);
  }
  return std::max(1, n);
}
thread_local bool g_verbose = false;

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
  const bool timing = g_verbose;
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
// SAH leaf termination (leaves of up to 2 references): office +3.9 %, 4K 16 spp +4.1 %; random
// triangle soups prefer single-reference leaves (config 4, 10 M: +4.8 %, profiles/r03/r03zh_ab_rt10m_tree.txt).
// 0 = by size: 1 from kSbvhLeafBySize input triangles on (the size that also selects the 16-entry ring), else 2.
constexpr int kSbvhLeafMax = 0;
constexpr long long kSbvhLeafBySize = 1ll << 18;

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

void build_sbvh_tree(const rt_scene_soa* s, const rt_upload_options& opt, DevTree& E,
                     std::vector<uint32_t>& records) {
  const bool timing = g_verbose;
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
  SbvhCtx C{s, opt.sbvh_alpha, 0.0, std::max(2, std::min(kSbvhBinsMax, opt.sbvh_bins)),
            std::max(1, std::min(8, opt.sbvh_leaf_max)), opt.sbvh_c_trav};
  const double budget_frac = opt.sbvh_budget;
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

// Options left "by size" (the defaults) resolved for a scene of nt input triangles: from
// kSbvhLeafBySize triangles on (random soups, config 4) single-reference leaves, the SAH-optimal
// collapse and spatial splits wherever they pay (alpha 0, budget 1.5): 10 M random triangles
// 4722 -> 4804 Mrays/s for the last three (profiles/r03/r03zl_ab_rt10m_tree.txt); below it the
// office's tuning (leaves of up to 2, alpha 1e-5, budget 0.75).  The SAH-optimal collapse is the
// default at every size since round 5 (office one frame -1.5 %, batched -0.9 %,
// profiles/r05/r05u_ab_tree_office.txt, r05v_ab_collapse_office.txt); RT_COLLAPSE_BY_SIZE, the
// earlier default, resolves to it as well.
static rt_upload_options options_by_size(rt_upload_options o, long long nt) {
  const bool deep = nt >= kSbvhLeafBySize;
  if (o.sbvh_leaf_max == 0) o.sbvh_leaf_max = deep ? 1 : 2;
  if (o.collapse == RT_COLLAPSE_BY_SIZE) o.collapse = RT_COLLAPSE_SAH;
  if (o.sbvh_alpha < 0.0) o.sbvh_alpha = deep ? 0.0 : kSbvhAlpha;
  if (o.sbvh_budget < 0.0) o.sbvh_budget = deep ? 1.5 : kSbvhBudget;
  return o;
}

int build_image(const rt_scene_soa* s, const rt_bvh_soa* b, const rt_upload_options& opt_in, int bfs_top,
                SceneImage& I) {
  const rt_upload_options opt = options_by_size(opt_in, s ? s->n_vertex_idx / 3 : 0);
  const int tree_kind = opt.device_tree;
  if (tree_kind != RT_TREE_SAH && tree_kind != RT_TREE_REFERENCE && tree_kind != RT_TREE_SBVH)
    return fail(RT_ERR_INVALID, "rt_scene_upload: unknown device_tree");
  if (opt.collapse != RT_COLLAPSE_GREEDY && opt.collapse != RT_COLLAPSE_SAH)
    return fail(RT_ERR_INVALID, "rt_scene_upload: unknown collapse");
  if (opt.build_threads < 0) return fail(RT_ERR_INVALID, "rt_scene_upload: build_threads < 0");
  g_threads = opt.build_threads > 0 ? std::min(opt.build_threads, 64) : std::max(1, std::min(usable_cpus(), 64));
  g_verbose = opt.verbose != 0;
  const bool timing = g_verbose;   // phase times to stderr (diagnostics)
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
    if (tree_kind == RT_TREE_SBVH) build_sbvh_tree(s, opt, E, dev2slot);
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
    // Optional SAH-optimal collapse (RT_COLLAPSE_SAH): D[n][j] = the least SAH cost of covering
    // binary subtree n with at most j child slots; a slot costs area * c_tri for a leaf and
    // area * c_node + D(children, 4) for a wide node (the 4 box tests of a visit are charged to
    // the visited node).  Children ids exceed their parent's in every builder, so one reverse
    // sweep fills the table.
    const bool dp = opt.collapse == RT_COLLAPSE_SAH;
    const double c_tri = opt.collapse_c_tri;
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
      // Numbering: the first bfs_top collapsed nodes in breadth-first order (the top
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
      for (size_t q = 0; q < order.size() && (int)order.size() < bfs_top; ++q) {   // breadth-first top
        const Kids k = kids[q];
        for (int i = 0; i < k.n && (int)order.size() < bfs_top; ++i)
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
  if (depth > kMaxStackDepth || stack4 > kMaxStackDepth)
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

const std::string& build_image_error() { return g_build_error; }

void upload_options_defaults(rt_upload_options* o) {
  std::memset(o, 0, sizeof *o);
  o->device_tree = RT_TREE_SBVH;
  o->build_threads = 0;
  o->stack_ring = 0;
  o->lds_treelet = 0;   // as many as fit
  o->collapse = RT_COLLAPSE_SAH;
  o->sbvh_leaf_max = kSbvhLeafMax;
  o->sbvh_bins = kSbvhBins;
  o->blocks_per_cu = 0;
  o->grid_spare = 0;
  o->verbose = 0;
  o->sbvh_alpha = -1.0;    // by size
  o->sbvh_budget = -1.0;   // by size
  o->sbvh_c_trav = 1.0;
  o->collapse_c_tri = 1.0;
}

}  // namespace rtk
