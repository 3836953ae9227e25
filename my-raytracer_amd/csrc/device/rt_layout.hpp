// rt_layout.hpp — device-resident scene layout of the MI355X render path.
//
// Replaces the reference's managed-memory struct Data (mydata.h:28-72) and
// BVH::BVHNodes_SoA (mybvh.h:49-55) for the traversal loop:
//
//  * GNode (64 B = half a 128-B line): one INTERNAL node of the reference's
//    median-split tree holding the boxes of its two children (the reference
//    re-reads 5 SoA arrays per pop, mytracer_gpu.cu:360-364, then 2 child
//    boxes, :397-403).  Boxes are fp32, rounded outward and grown by
//    delta = 2^-20 * max|vertex| so the fp32 slab test is conservative for
//    the fp64 ray.  Per axis one float4 {lo0, hi0, lo1, hi1}
//    so one dwordx4 load feeds both children's slab on that axis.  Nodes are
//    numbered in depth-first preorder (left child = parent + 1).
//    ref: internal child -> its GNode index; leaf child -> LEAF | first slot;
//    EMPTY marks the absent sibling of a single-leaf root.
//  * GTri (80 B): fp64 triangle record in device leaf order, holding exactly
//    the operands of the reference's Cramer test (mymesh.cpp:190-193):
//    e1 = p0 - p2, e2 = p1 - p2, p2, plus mesh id, reference slot and
//    end-of-leaf flags.
//  * Shading data is only touched once per closest hit: per-slot vertex /
//    uv indices, face normals, vertex normals, uvs, texels, materials.
#pragma once
#include <cstdint>

namespace rtk {

constexpr uint32_t kLeaf = 0x80000000u;
constexpr uint32_t kEmpty = 0x7fffffffu;
constexpr uint32_t kDone = 0xffffffffu;
constexpr int kNoHit = 0x7fffffff;
constexpr int kPrimHit = 0x40000000;   // best = kPrimHit | k: analytic primitive k (never a triangle record)

struct alignas(64) GNode {
  float x[4];   // lo0, hi0, lo1, hi1
  float y[4];
  float z[4];
  uint32_t ref[2];
  uint32_t pad[2];
};
static_assert(sizeof(GNode) == 64, "GNode must be 64 bytes");

// 4-wide node (128 B = one cache line): the same median-split tree with two
// levels of the binary tree collapsed into one node (children chosen by the
// largest box area), per axis 4 lo + 4 hi fp32 bounds, 4 child refs.  The
// production traversal uses it: half the dependent node fetches per ray.
struct alignas(128) GNode4 {
  float lox[4], hix[4];
  float loy[4], hiy[4];
  float loz[4], hiz[4];
  uint32_t ref[4];
  uint32_t pad[4];
};
static_assert(sizeof(GNode4) == 128, "GNode4 must be 128 bytes");

// GTri.meta: reference leaf slot (the tie-break key and the 2-wide iteration
// order) plus two end-of-leaf flags.  Records sit in DEVICE order: the reference
// leaf order, except that oversize reference leaves are refined into sub-leaves
// whose triangles are permuted within the leaf's slot range.
constexpr uint32_t kSlotMask = 0x3fffffffu;
constexpr uint32_t kLastRef = 0x40000000u;   // slot is the last of its reference leaf
constexpr uint32_t kLastDev = 0x80000000u;   // record is the last of its device leaf

struct alignas(16) GTri {
  double e1[3];
  double e2[3];
  double p2[3];
  int32_t mesh;
  uint32_t meta;   // slot | kLastRef | kLastDev
};
static_assert(sizeof(GTri) == 80, "GTri must be 80 bytes");

struct alignas(16) TriShade {
  int32_t v[3];    // global vertex ids (vertexIdx_)
  int32_t t[3];    // global uv ids (textureIdx_), -1 = none
  int32_t pad[2];
};
static_assert(sizeof(TriShade) == 32, "TriShade must be 32 bytes");

struct alignas(16) GMat {
  double ka[3];
  double kd[3];
  double ks[3];
  double shininess;
  double mirror;
  int32_t shadowable;
  int32_t draw_mode;
  int32_t tex_w;    // -1: none
  int32_t tex_h;
  int64_t tex_off;  // texel offset
  int64_t pad;
};
static_assert(sizeof(GMat) == 128, "GMat must be 128 bytes");

// Analytic primitive (opt-in, rt_scene_set_analytic): spheres first, then planes, each in
// scene order -- the order intersect_scene tests them (oracle/rt_oracle.c intersect_scene).
enum : int32_t { kPrimSphere = 0, kPrimPlane = 1 };
struct alignas(16) GPrim {
  double c[3];      // sphere centre / point on the plane
  double r;         // sphere radius (unused for planes)
  double n[3];      // plane unit normal (unused for spheres)
  int32_t type;     // kPrimSphere / kPrimPlane
  int32_t mat;      // index into the material table (after the meshes' materials)
};
static_assert(sizeof(GPrim) == 64, "GPrim must be 64 bytes");

}  // namespace rtk
