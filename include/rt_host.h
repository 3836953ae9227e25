/*
 * rt_host.h — C-ABI of the C++ host side (librt_host.so): scene loading and
 * generation, normals, SoA flattening and the median-split BVH build.
 *
 * Reference interfaces this side replaces:
 *   Raytracer::init_cuda(filename)           mytracer.cpp:54-60
 *     pre_read_scene / pre_read_obj           mytracer.cpp:302-350, 424-500
 *     read_scene / Mesh::read_obj             [ABSENT course framework]
 *     Mesh::compute_normals                   mymesh.cpp:103-163
 *     Raytracer::build_Data                   mytracer.cpp:166-296
 *     BVH::initSoA (+updateNodeBoundsSoA, subdivideSoA,
 *                   inplace_partitionSoA, medianSoA, median_inplace)
 *                                             mybvh.cpp:375-539, 346-362
 *   Camera(eye, center, up, fovy, w, h)       [ABSENT course framework]
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include "rt_scene.h"
#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_host_scene rt_host_scene;   /* opaque, owns all host arrays */

/* Parameters of the procedural scenes. */
typedef struct rt_gen_params {
  int width;            /* image size stored in the camera (<=0: scene default) */
  int height;
  long long n_triangles;/* random_tris: triangle count */
  unsigned long long seed;
  int max_depth;        /* <0: scene default */
  int detail;           /* office: tessellation level (<=0: default) */
} rt_gen_params;

/* Reads a .sce scene file (grammar in DESIGN.md §6) with its .obj meshes. */
int rt_host_load(const char* sce_path, rt_host_scene** out);

/* kind: "office" (office_proxy), "spheres" (spheres_proxy), "random_tris",
 * "cornell" (small test room).  params may be NULL (defaults). */
int rt_host_generate(const char* kind, const rt_gen_params* params, rt_host_scene** out);

/* Plain view of the raw scene (valid while the scene lives). */
const rt_raw_scene* rt_host_raw(const rt_host_scene* s);

/* compute_normals for every mesh, build_Data (AoS -> SoA) and BVH::initSoA.
 * Idempotent.  Returns the build time in *seconds if non-NULL. */
int rt_host_prepare(rt_host_scene* s, double* seconds);

/* rt_host_prepare with the median-split builder's thread count: 0 = the CPUs this process may
 * use (affinity mask, capped by a cgroup CPU quota; the rt_host_prepare default), else at most 64.
 * The tree and the slot permutation do not depend on it.  The library reads no environment. */
int rt_host_prepare_ex(rt_host_scene* s, int build_threads, double* seconds);

/* Valid after rt_host_prepare. */
const rt_scene_soa* rt_host_soa(const rt_host_scene* s);
const rt_bvh_soa* rt_host_bvh(const rt_host_scene* s);

/* Derived camera at an explicit resolution (<=0: the scene's). */
int rt_host_camera(const rt_host_scene* s, int width, int height, rt_camera* out);

/* Render parameters for the scene at the given resolution / spp (full frame,
 * one stripe, RT_OUT_RGB_F32). */
int rt_host_render_params(const rt_host_scene* s, int width, int height, int spp_n,
                          rt_render_params* out);

/* Writes a .sce + .obj set that rt_host_load reads back into the same scene. */
int rt_host_save(const rt_host_scene* s, const char* sce_path);

/* Writes an RGB float image (rows bottom-up as rendered, y = 0 first) as a
 * binary PPM (P6), flipped so that row y = height-1 is the top line. */
int rt_write_ppm(const char* path, const float* rgb, int width, int height);

long long rt_host_triangle_count(const rt_host_scene* s);
int rt_host_bvh_depth(const rt_host_scene* s);   /* max node depth (root = 0) */

void rt_host_free(rt_host_scene* s);
const char* rt_host_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_HOST_H */
