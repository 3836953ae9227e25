/*
 * rt_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of hvkwak/my-raytracer's CPU renderer (the
 * "reference CPU renderer" of SURVEY.md §8a/a15), used ONLY by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
 * The product path (librt_hip.so / librt_host.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned" with respect to the reference's own
 * outputs.  The reference ships no tests, fixtures or golden vectors for this
 * path and cannot be built here: every translation unit needs
 * the absent TU Dortmund course headers (utils/vec4.h, Camera.h, Ray.h, ...).
 * The restatement is instead checked against hand-derived known answers
 * (tests/golden/kat_*.json, tests/test_oracle_kat.py) and cross-checked
 * against the independently written C++ host builder and the HIP kernel.
 * Functions cite the reference file:line they follow; semantics of the
 * [ABSENT] course pieces (Camera, Ray, trace, intersect_scene, compute_image,
 * Sphere) are fixed in DESIGN.md §2.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include "../include/rt_scene.h"
#include "../include/rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_ctx or_ctx;

typedef struct or_counts {
  long long primary_rays;
  long long shadow_rays;
  long long reflection_rays;
  long long node_visits;   /* ordered mode: 2-wide fp32 nodes fetched */
  long long tri_tests;     /* triangle tests (either mode) */
  long long closest_hits;  /* closest-hit rays that hit something */
  long long pixels;
  long long box_tests;     /* reference mode: AABB tests */
} or_counts;

enum {
  OR_MODE_REFERENCE = 0,  /* recursive unordered fp64 traversal, closest-hit shadows (mybvh.cpp:147-210) */
  OR_MODE_ORDERED = 1     /* replica of the GPU algorithm: ordered, t-culled fp32 2-wide traversal, any-hit shadows */
};

/* Derives normals (mymesh.cpp:103-163) and the AoS median-split BVH
 * (mybvh.cpp:44-81, 220-362).  Returns NULL on error. */
or_ctx* or_prepare(const rt_raw_scene* scene);
void or_free(or_ctx* ctx);

/* Restated course Camera from its definition. */
void or_camera(const rt_camera_def* def, int width, int height, rt_camera* out);

/* Renders the rows selected by p (same stripe rules as rt_launch_compute_image)
 * into out (rows*width*3 doubles).  nthreads <= 0: OpenMP default. */
int or_render(or_ctx* ctx, const rt_render_params* p, int mode, int nthreads,
              double* out, or_counts* counts);

/* Renders pixels given as a list of (x, y) (for sampled CPU-baseline timing). */
int or_render_pixels(or_ctx* ctx, const rt_render_params* p, int mode, int nthreads,
                     const int* xy, long long n_pixels, double* out, or_counts* counts);

/* ---- exports for parity tests ---- */
long long or_n_triangles(const or_ctx* ctx);
int or_n_nodes(const or_ctx* ctx);
/* Tree in the reference's node numbering: bb_min/bb_max [3*n_nodes],
 * left/first/count [n_nodes]; perm [n_tris] = global triangle id (mesh
 * triangles numbered consecutively in mesh order) at each leaf slot. */
void or_export_bvh(const or_ctx* ctx, double* bb_min, double* bb_max, int* left, int* first,
                   int* count, int* perm);
/* Vertex normals of all meshes concatenated [3*total_vertices] and face
 * normals [3*total_triangles] in original mesh order. */
void or_export_normals(const or_ctx* ctx, double* vertex_normals, double* face_normals);
int or_tree_depth(const or_ctx* ctx);

/* Closest hit of one ray in the given mode (KAT tests): returns 1 on hit,
 * writes t, global triangle id (or -1 for analytic objects), point, normal. */
int or_closest_hit(or_ctx* ctx, const double o[3], const double d[3], int mode,
                   double* t, int* tri_id, double point[3], double normal[3]);

/* Single-function restatements exposed for known-answer tests. */
int or_intersect_triangle(const double p0[3], const double p1[3], const double p2[3],
                          const double o[3], const double d[3],
                          double* t, double* alpha, double* beta, double* gamma);
int or_intersect_aabb(const double o[3], const double d[3], const double bmin[3],
                      const double bmax[3]);
double or_median(double* values, int n);

#ifdef __cplusplus
}
#endif
#endif
