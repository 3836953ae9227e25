/*
 * rt_hip.h — C-ABI of the MI355X render path (librt_hip.so).
 *
 * This is the drop-in boundary that replaces the reference's device entry
 *   void launch_compute_image_device(vec4* d_pixels, vec4* d_tmpPixels,
 *        vec4* d_image, const int& width, const int& height,
 *        const Camera& camera, const vec4* d_lightsPos,
 *        const vec4* d_lightsColor, const int& nLights,
 *        const vec4& background, const vec4& ambience, const int& max_depth,
 *        const Data* data, const BVH::BVHNodes_SoA* bvhNodes);
 *   (declared mytracer_gpu.h:43-56, defined mytracer_gpu.cu:44-113)
 * together with the managed-memory scene it reads (struct Data, mydata.h:28-72;
 * BVH::BVHNodes_SoA, mybvh.h:49-55; allocated by Raytracer::build_Data,
 * mytracer.cpp:166-296, and BVH::initSoA, mybvh.cpp:375-406).
 *
 * Differences by design:
 *  - the scene is uploaded once with explicit hipMalloc/hipMemcpy into an
 *    MI355X layout (fp32 4-wide BVH nodes collapsed from the reference's
 *    binary tree, child boxes in the parent; the 2-wide form for the canonical
 *    counters; fp64 triangle records in leaf order); no managed memory;
 *  - the caller passes host SoA arrays (the reference's Data/BVHNodes_SoA
 *    content, same meaning, packed xyz instead of vec4) and owns the output;
 *  - errors are returned as status codes with the message in rt_last_error()
 *    (the reference's CHECK prints and continues, common/common.h:6-15);
 *  - rows can be restricted / interleaved so one process per GPU renders its
 *    share of the image (the reference only uses device 0, mytracer_gpu.cu:34).
 * All pointers are plain; no torch or HIP types appear in the signatures
 * (streams are passed as void*).
 * Current device: a call that takes a scene makes the scene's device current on the calling
 * thread and leaves it so (rt_scene_upload*: `device`; rt_ipc_open: `device`), as the
 * reference's single-device code assumes; a caller driving several GPUs from one thread sets
 * its own device again after a call (rt_multi.h does).
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include "rt_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_ERR_INVALID (-1)     /* bad argument / inconsistent scene */
#define RT_ERR_HIP (-2)         /* HIP runtime failure */
#define RT_ERR_UNSUPPORTED (-3) /* scene exceeds a compiled limit (e.g. BVH depth) */

/* Lights held inline in rt_render_params (and staged in LDS by the kernel).  Scenes with
 * more lights pass them through rt_render_params.lights_ext (any count up to
 * RT_LIGHTS_LIMIT); the reference shades any nLights (mytracer_gpu.cu:632).  Every launch copies
 * its light table with its control block (as the reference's copyLights per call,
 * mytracer.cpp:105-118), so lights may change from call to call, on any stream, without a
 * device synchronisation. */
#define RT_MAX_LIGHTS 16
#define RT_LIGHTS_LIMIT (1 << 20)

/* Host SoA scene: the content of struct Data (mydata.h:28-72) after
 * BVH::initSoA has permuted the per-triangle arrays into leaf order
 * (mybvh.cpp:497-503).  Vectors are packed xyz (3 doubles). */
typedef struct rt_scene_soa {
  int n_meshes;          /* tMeshCount_ */
  int n_vertices;        /* tVertexCount_ */
  int n_vertex_idx;      /* tVertexIdxCount_ = 3 * n_triangles */
  int n_tex_coords;      /* tTextCoordCount_ */
  long long n_texels;    /* tTexelCount_ */
  const int* vertex_mesh_id;     /* [n_vertices]          vertexMeshId_ */
  const double* vertex_pos;      /* [3*n_vertices]        vertexPos_ */
  const double* vertex_normals;  /* [3*n_vertices]        vertexNormals_ */
  const double* face_normals;    /* [3*n_triangles]       normals_ (leaf order) */
  const int* vertex_idx;         /* [n_vertex_idx]        vertexIdx_ (leaf order, global ids) */
  const int* texture_idx;        /* [n_vertex_idx]        textureIdx_ (leaf order, global ids) */
  const double* tex_u;           /* [n_tex_coords]        textureCoordinatesU_ */
  const double* tex_v;           /* [n_tex_coords]        textureCoordinatesV_ */
  const unsigned char* texels;   /* [3*n_texels] RGB8     meshTexels_ (vec4 in the reference) */
  const int* mesh_tex_width;     /* [n_meshes], -1 = none meshTexWidth_ */
  const int* mesh_tex_height;    /* [n_meshes]            meshTexHeight_ */
  const long long* mesh_tex_offset; /* [n_meshes]         firstMeshTex_ */
  const int* mesh_draw_mode;     /* [n_meshes]            meshDrawMode_ */
  const double* mat_ambient;     /* [3*n_meshes]          materialAmbient_ */
  const double* mat_diffuse;     /* [3*n_meshes]          materialDiffuse_ */
  const double* mat_specular;    /* [3*n_meshes]          materialSpecular_ */
  const double* mat_shininess;   /* [n_meshes]            materialShininess_ */
  const double* mat_mirror;      /* [n_meshes]            materialMirror_ */
  const int* mat_shadowable;     /* [n_meshes]            materialShadowable_ */
} rt_scene_soa;

/* The reference's BVH::BVHNodes_SoA (mybvh.h:49-55), nodes [0, n_nodes). */
typedef struct rt_bvh_soa {
  int n_nodes;                 /* nodesUsed_ */
  const double* bb_min;        /* [3*n_nodes] */
  const double* bb_max;        /* [3*n_nodes] */
  const int* left_child;       /* [n_nodes]; right child = left_child + 1 */
  const int* first_tri;        /* [n_nodes] */
  const int* tri_count;        /* [n_nodes]; 0 = internal */
} rt_bvh_soa;

/* Output formats of rt_launch_compute_image. */
enum {
  RT_OUT_RGB_F32 = 0,  /* 3 floats per pixel (production) */
  RT_OUT_RGB_F64 = 1   /* 3 doubles per pixel (parity tests) */
};

/* Flags of rt_render_params.flags. */
enum {
  RT_FLAG_TRAVERSAL_STATS = 1, /* canonical counters: 2-wide traversal (the one the oracle replicates),
                                  counts node visits / triangle tests / closest hits */
  RT_FLAG_WIDE_STATS = 2,      /* same counters on the production 4-wide traversal (diagnostics) */
  RT_FLAG_TIMELINE = 4,        /* production kernel + per-round timeline (diagnostics, rt_debug_timeline) */
  RT_FLAG_TILE_COST = 8,       /* diagnostics: per-tile cost of the launch (rt_debug_tile_cost): bounces */
  RT_FLAG_TILE_COST_TIME = 16, /* ... the same, as pixel lifetimes (10-ns ticks) */
  RT_FLAG_COST_ORDER = 32,     /* cost-ordered work for one-frame launches (the reference's use): every work head
                                  renders first the tiles that took longest (pixel lifetimes) in the launch before
                                  the previous one of the same image geometry (animation: frame i - 2's costs
                                  order frame i), and this launch's costs are kept; shortens the end-of-launch
                                  drain, pixels unchanged.  The DEFAULT for one-frame launches
                                  on the stream of the scene's last ordered launch (or the first one-frame
                                  launch); launches on another stream keep the natural order unless they set
                                  this flag, which then makes them wait for the last ordered launch.
                                  Launches of several frames and adaptive passes keep the natural order and
                                  record nothing; one-frame launches of more than 32768 tiles (rt_tile_shape) keep
                                  the natural order */
  RT_FLAG_NATURAL_ORDER = 64,  /* one-frame launch in the natural tile order, recording no costs */
  RT_FLAG_GLOBAL_ROWS = 128    /* the output buffer holds the whole frame (camera.height rows): the shard's rows
                                  are written at their global positions (row y at y * width * 3), not packed.
                                  With a peer GPU's frame buffer (rt_ipc_open) every rank writes its stripes
                                  straight into the assembled frame over xGMI; each wave's stores are released
                                  at system scope before it exits.  Not for the adaptive pass nor
                                  rt_render_to_host (RT_ERR_INVALID) */
};

/* One render call.  Rows are rendered as interleaved stripes:
 * row y is rendered iff row_begin <= y < row_end and
 * (y / stripe_height) % stripe_count == stripe_index; rendered rows are
 * packed into the output in increasing y, row-major, pixel (x, y) of local
 * row r at out[(r*width + x)*3 + c] (the reference's pixels[y*W+x],
 * mytracer_gpu.cu:158).  stripe_count == 1 renders every row in range. */
typedef struct rt_render_params {
  rt_camera camera;
  int n_lights;                          /* <= RT_MAX_LIGHTS, or <= RT_LIGHTS_LIMIT with lights_ext */
  int max_depth;                         /* reflection bounces after the primary hit */
  rt_light lights[RT_MAX_LIGHTS];        /* used when lights_ext == NULL */
  double background[3];
  double ambience[3];
  int spp_n;            /* n: n*n stratified samples per pixel (mytracer_gpu.cu:202-221); 1 = one ray through (x,y) */
  int row_begin;
  int row_end;          /* <= 0 means camera.height */
  int stripe_height;    /* >= 1 */
  int stripe_count;     /* >= 1 */
  int stripe_index;     /* [0, stripe_count) */
  int out_format;       /* RT_OUT_* */
  int flags;            /* RT_FLAG_* */
  const rt_light* lights_ext;  /* non-NULL: the n_lights lights (host memory, read during the call) */
} rt_render_params;

/* Light i of a render call (lights_ext when set, else the inline table). */
static inline const rt_light* rt_params_light(const rt_render_params* p, int i) {
  return p->lights_ext ? &p->lights_ext[i] : &p->lights[i];
}

/* Ray counters of one launch (canonical definition: DESIGN.md §5).
 * primary = pixels*spp; shadow = shading points x lights with a shadowable
 * material (mytracer.cpp:589); reflection = shading points with mirror > 0
 * below max_depth (mytracer.cpp:547).  node_visits / tri_tests / hits are
 * filled only with RT_FLAG_TRAVERSAL_STATS (canonical 2-wide walk: exact, equal to the oracle's)
 * or RT_FLAG_WIDE_STATS (the 4-wide production traversal, every wave sorting children: with
 * shadow rays these vary by ~1e-5 between runs, as the postponed-leaf timing and the fan-out of
 * shadow rays to idle lanes depend on which rays share a wave). */
typedef struct rt_stats {
  long long primary_rays;
  long long shadow_rays;
  long long reflection_rays;
  long long node_visits;      /* fp32 2-wide nodes fetched (= internal-node pops) */
  long long tri_tests;        /* triangle records tested */
  long long closest_hits;     /* closest-hit rays that hit (shading fetches) */
  long long pixels;           /* pixels written */
  long long reserved_;
} rt_stats;

typedef struct rt_scene rt_scene;   /* opaque device-resident scene */

/* Uploads the scene to HIP device `device` (hipSetDevice), converting the
 * host SoA + reference BVH into the MI355X layout.  Leaves the device current. */
int rt_scene_upload(const rt_scene_soa* soa, const rt_bvh_soa* bvh, int device, rt_scene** out);

/* Device traversal hierarchy (never changes a pixel or a ray count: the closest hit is
 * the smallest (t, reference slot) over a conservative superset of candidates, DESIGN.md
 * §4; the canonical counters always walk the reference tree given in `bvh`).
 *   RT_TREE_SBVH       binned SAH with spatial splits (straddling triangles referenced from
 *                      both sides, clipped bounds), 4-wide collapsed (default; builds ~5x
 *                      slower than RT_TREE_SAH: 16 s at 10 M triangles on 16 threads)
 *   RT_TREE_SAH        binned-SAH tree over all triangles (object splits only), 4-wide collapsed
 *   RT_TREE_REFERENCE  the reference median-split tree, oversize leaves refined */
enum { RT_TREE_SAH = 0, RT_TREE_REFERENCE = 1, RT_TREE_SBVH = 2 };
/* 4-wide collapse of the device hierarchy: open the child with the largest box, or the
 * SAH-optimal choice of up to 4 slots per node (dynamic programme; the default).
 * RT_COLLAPSE_BY_SIZE (the default before round 5: greedy below 2^18 input triangles) now
 * resolves to RT_COLLAPSE_SAH at every size. */
enum { RT_COLLAPSE_GREEDY = 0, RT_COLLAPSE_SAH = 1, RT_COLLAPSE_BY_SIZE = 2 };

/* Upload options.  The library reads nothing from the environment: its behaviour depends only
 * on these fields and the call's arguments.  Fill with rt_upload_options_init (the defaults),
 * then change fields:
 *     rt_upload_options o; rt_upload_options_init(&o); o.device_tree = RT_TREE_SAH;
 * A zero-initialised struct is valid too: zero in sbvh_bins, sbvh_c_trav, collapse_c_tri and
 * lds_treelet means their defaults; zero in device_tree / collapse / sbvh_alpha / sbvh_budget
 * selects RT_TREE_SAH / RT_COLLAPSE_GREEDY / alpha 0 / budget 0 (valid, but not the defaults).
 * None of them changes a pixel or a ray count: they pick the device hierarchy,
 * its build, and the kernel's LDS / grid layout. */
typedef struct rt_upload_options {
  int device_tree;       /* RT_TREE_* (default RT_TREE_SBVH) */
  int build_threads;     /* host threads of the builders; 0 = the CPUs this process may use (its
                            affinity mask, capped by a cgroup CPU quota), at most 64.
                            The hierarchy does not depend on it */
  int stack_ring;        /* LDS stack-ring entries of the production kernel: 0 = by size (16 from 2^18
                            device records on, else 8; default), 8 or 16 */
  int lds_treelet;       /* 4-wide nodes each block caches in LDS: 0 = as many as fit (default),
                            > 0 = at most this many, -1 = none */
  int collapse;          /* RT_COLLAPSE_* (default RT_COLLAPSE_SAH; RT_COLLAPSE_BY_SIZE resolves to it) */
  int sbvh_leaf_max;     /* SBVH: SAH-terminated leaves of up to this many references, 1..8 (1 = split
                            down to single references); 0 = by size (default): 1 from 2^18 input
                            triangles on, else 2 */
  int sbvh_bins;         /* SBVH: spatial bins per axis (default 32; 0 = default), 2..128 (64: 10 M random
                            triangles +1.7 % per frame for +64 % build time) */
  int blocks_per_cu;     /* persistent blocks per CU: 0 = as many as fit (default), else at most this many */
  int grid_spare;        /* block slots of the persistent grid left free for concurrent kernels (default 0) */
  int verbose;           /* 1: build phase times to stderr (default 0) */
  double sbvh_alpha;     /* SBVH: try spatial splits where the best object split's children overlap by
                            more than alpha x the root's surface area; < 0 = by size (default):
                            0 from 2^18 input triangles on, else 1e-5 */
  double sbvh_budget;    /* SBVH: at most this many extra references per triangle; < 0 = by size
                            (default): 1.5 from 2^18 input triangles on, else 0.75 */
  double sbvh_c_trav;    /* SBVH: node visit cost in triangle tests, for leaf termination (default 1.0;
                            0 = default) */
  double collapse_c_tri; /* RT_COLLAPSE_SAH: cost of a leaf slot per unit area (default 1.0; 0 = default) */
  int reserve_cus;       /* CUs each render launch leaves free for concurrent kernels (an RCCL gather of the
                            previous launch: its 256-VGPR waves fit no single free block slot of the
                            persistent grid): > 0 = the launches run on an internal stream
                            whose CU mask clears the first reserve_cus CUs, the grid sized to the rest
                            (32 = one XCD's worth: the smallest reservation a 256-VGPR kernel was
                            measured to run beside a stand-in of RCCL's kernel shape); 0 = none (default,
                            also in rt_multi_create: the reservation slows the render by ~12 % and
                            its gain at N > 1 is unmeasured; bench.py times both at N > 1); -1 = none */
  int order_window;      /* one-frame cost order (RT_FLAG_COST_ORDER, the default on one stream): a tile sorts by
                            the largest recorded cost within +-order_window tiles of its row; 0 = by size (4,
                            exact costs for hierarchies from 2^18 device records on, whatever stack_ring forces;
                            default), -1 = exact */
  int spp_lanes;         /* n x n > 1 samples per pixel, n^2 a power of two: 1 = a pixel's samples on
                            neighbouring lanes of one wave (groups of G = min(n^2, 32) lanes, summed in sample
                            order on chip), 2..64 (a power of two) = the same with G capped at that many
                            lanes (chunks of G samples in sequence), -1 = one lane per pixel, its samples in
                            sequence; 0 = the default,
                            groups (4K 16 spp +22.6 %, 8K 64 spp +19.3 %).  Launches with
                            other n, the diagnostic flags, tile-cost maps or RT_FLAG_COST_ORDER keep one lane
                            per pixel.  The adaptive pass follows it too (groups: no sample buffer, no
                            reduce kernel).  Pixels and ray counts are identical either way */
  int reserved_[5];
} rt_upload_options;

/* Fills *opt with the defaults listed above. */
void rt_upload_options_init(rt_upload_options* opt);

/* rt_scene_upload with options (NULL = defaults). */
int rt_scene_upload_ex(const rt_scene_soa* soa, const rt_bvh_soa* bvh, int device, const rt_upload_options* opt,
                       rt_scene** out);

/* Uploads one scene to several devices: the device layout (hierarchy, records) is built
 * once on the host and copied to devices[0..n_devices), one host thread per device.
 * outs[g] receives the scene on devices[g]; on failure every outs[g] is NULL.  The
 * multi-GPU driver (rt_multi.h) uses it. */
int rt_scene_upload_multi(const rt_scene_soa* soa, const rt_bvh_soa* bvh, const int* devices, int n_devices,
                          const rt_upload_options* opt, rt_scene** outs);

/* Device bytes held by the scene (nodes, triangles, shading data). */
long long rt_scene_device_bytes(const rt_scene* scene);

/* Host seconds of the scene's upload: build_s = the device layout built on the host (the device
 * hierarchy -- SBVH / SAH / refined reference tree --, its wide collapse, the triangle and shading
 * records; once for every device of rt_scene_upload_multi), copy_s = device allocation and the
 * H2D copies of this device.  The reference's own build (BVH::initSoA, mybvh.cpp:375-406) is the
 * caller's rt_host_prepare, timed separately.  Either pointer may be NULL. */
int rt_scene_upload_seconds(const rt_scene* scene, double* build_s, double* copy_s);

/* Opt-in analytic primitives: the spheres and planes of the
 * raw scene (rt_raw_scene.spheres / .planes), tested in fp64 before the BVH in
 * the CPU's order -- spheres, then planes, nearest strictly closer wins, then
 * triangles only if strictly closer (oracle intersect_scene; Sphere/Plane
 * intersect, myplane.cpp:22-49).  The reference GPU path traces meshes only
 * (intersect_scene_device, mytracer_gpu.cu:314-328); a scene without this call
 * matches it.  Replaces
 * any previous set; n = 0 removes them.  Synchronises the device. */
int rt_scene_set_analytic(rt_scene* scene, const rt_sphere* spheres, int n_spheres, const rt_plane* planes,
                          int n_planes);

/* Number of rows rt_launch_compute_image writes for these params. */
int rt_rows_in_shard(const rt_render_params* p);

/* Renders into the caller-owned DEVICE buffer d_out (rows x width x 3 of the
 * chosen format) on `stream` (hipStream_t, NULL = the null stream).
 * Asynchronous unless stats != NULL, in which case it synchronises the stream
 * and fills *stats.  Launches on different streams may run concurrently: the
 * scene keeps a ring of 8 launch contexts (path state, work heads, counters)
 * and a context is reused only after its previous launch completed.  Calls on
 * one scene must come from one host thread at a time.  Replaces launch_compute_image_device's primary pass
 * (mytracer_gpu.cu:66-81); the adaptive pass (:83-109) is SURVEY §8f "next". */
int rt_launch_compute_image(rt_scene* scene, const rt_render_params* p, void* d_out,
                            rt_stats* stats, void* stream);

/* Up to RT_MAX_FRAMES frames in ONE launch of the persistent kernel: frame f renders
 * p[f] into d_outs[f].  The frames share one work queue, so the tail of one frame is
 * filled with the next frame's pixels instead of idling (the per-launch drain is paid
 * once per batch).  p[f] may differ from p[0] only in camera.eye / lower_left / x_dir /
 * y_dir (an animation path); everything else must be identical.  stats (optional,
 * synchronising) sums the frames.  Results equal n_frames rt_launch_compute_image calls. */
#define RT_MAX_FRAMES 128
int rt_launch_frames(rt_scene* scene, const rt_render_params* p, int n_frames, void* const* d_outs,
                     rt_stats* stats, void* stream);

/* Adaptive supersampling pass: replaces adaptive_supersampling_device
 * (mytracer_gpu.cu:162-229, launched at :83-109 with subp = 4, threshold = 0.02).
 * d_primary: the primary pass of the SAME params rendered with
 * RT_OUT_RGB_F64 (H x W x 3 doubles, device).  Every interior pixel whose
 * squared colour differences to its 4 neighbours (x+1, y+1, x-1, y-1, in that
 * order) sum above `threshold` is re-rendered with subp x subp stratified
 * samples (averaged, clamped); all other pixels are copied from d_primary.
 * d_out (H x W x 3, p->out_format) must not alias d_primary.  Full frame only
 * (stripe_count 1, no row range).  stats (optional, synchronising) counts the
 * rays of this pass; *n_selected (optional, synchronising) = re-rendered pixels. */
int rt_launch_adaptive(rt_scene* scene, const rt_render_params* p, const double* d_primary, void* d_out, int subp,
                       double threshold, rt_stats* stats, long long* n_selected, void* stream);

/* Adaptive pass over n_frames full frames at once (animation / batched frames):
 * p[0..n_frames) differ only in their camera vectors (as rt_launch_frames), d_primary[f] is frame
 * f's fp64 primary image, d_out[f] its output.  Every frame's selection goes into one list and
 * one launch traces every sample of every selected pixel of every frame (a pixel's samples on
 * neighbouring lanes, as rt_launch_adaptive), so the per-launch drain is paid once per batch.
 * subp^2 a power of two (sample groups, rt_upload_options.spp_lanes >= 0): the render kernel sums
 * and stores each selected pixel itself and the call does not synchronise; otherwise a sample
 * buffer sized by the selection count, which the call reads back (one host synchronisation per
 * call), and a reduce kernel.  Results equal rt_launch_adaptive on each frame.  W x H < 2^25.
 * *n_selected (optional, synchronising) = pixels re-rendered over all frames. */
int rt_launch_adaptive_frames(rt_scene* scene, const rt_render_params* p, int n_frames, const double* const* d_primary,
                              void* const* d_out, int subp, double threshold, rt_stats* stats, long long* n_selected,
                              void* stream);

/* Adaptive pass over a row shard (the multi-GPU case).  p may use
 * stripes or a row range; d_primary / d_out are the shard's packed rows (as
 * rt_launch_compute_image writes them), d_primary in RT_OUT_RGB_F64.  The
 * neighbour test of a shard's first / last row in each run of consecutive rows
 * (a stripe, or the row range) needs the primary colour of the row just outside
 * it: d_halo holds those rows, [segment][2][W][3] doubles, [s][0] = the row
 * below segment s, [s][1] = the row above it, in the order rt_adaptive_halo_rows
 * lists them (rows outside the frame are never read; d_halo may be NULL when all
 * of them are).  Selection and results equal rt_launch_adaptive on the full frame
 * restricted to the shard's rows. */
int rt_launch_adaptive_shard(rt_scene* scene, const rt_render_params* p, const double* d_primary,
                             const double* d_halo, void* d_out, int subp, double threshold, rt_stats* stats,
                             long long* n_selected, void* stream);

/* Global rows the halo of rt_launch_adaptive_shard must hold: rows_out[2s] = the
 * row below segment s, rows_out[2s+1] = the row above it, -1 outside the frame.
 * Returns the entry count (2 x segments); rows_out may be NULL to query it. */
int rt_adaptive_halo_rows(const rt_render_params* p, int* rows_out, int cap);

/* The reference's whole launch_compute_image_device (mytracer_gpu.cu:44-113) in one synchronous
 * call: the primary pass (fp64, device scratch), the adaptive pass (subp, threshold: the reference
 * uses 4 and 0.02) and the copy of the final image into host_out (H x W x 3 of p->out_format; a
 * page-locked, device-mapped buffer is written directly).  Full frame only.  st_primary /
 * st_adaptive / n_selected optional.  Results equal rt_launch_compute_image (fp64) +
 * rt_launch_adaptive on device buffers. */
int rt_render_adaptive_to_host(rt_scene* scene, const rt_render_params* p, int subp, double threshold, void* host_out,
                               rt_stats* st_primary, rt_stats* st_adaptive, long long* n_selected);

/* Renders into a HOST buffer, synchronously (the reference's call pattern: Raytracer::
 * compute_image_cuda copies every frame back, mytracer.cpp:123-159).  A page-locked, device-mapped
 * buffer (hipHostMalloc, hipHostRegister, torch pin_memory) is written by the kernel directly over
 * PCIe as pixels finish; pageable memory goes through a device staging buffer kept by the scene
 * (allocated on first use, grown as needed, freed by rt_scene_free) and one copy. */
int rt_render_to_host(rt_scene* scene, const rt_render_params* p, void* host_out, rt_stats* stats);

/* Cross-process access to a device buffer, for one process per GPU (the frame-assembly mode
 * RT_FLAG_GLOBAL_ROWS: every rank writes its stripes straight into rank 0's frame buffer).
 * rt_ipc_get_handle exports the device allocation that holds d_ptr (an RT_IPC_HANDLE_BYTES-byte
 * handle, plain bytes to send to the other processes) and d_ptr's byte offset in it.  Another
 * process maps it with rt_ipc_open, with its own `device` current and the exporter's device id as
 * this process numbers it (`owner_device`, -1 = unknown: then the mapping's lazy peer access only):
 * peer access from `device` to `owner_device` is checked and enabled, and the call returns a pointer
 * to the same bytes; rt_ipc_close(ptr, offset) unmaps it.  The
 * exporting process must keep the allocation alive while it is mapped elsewhere. */
#define RT_IPC_HANDLE_BYTES 64
int rt_ipc_get_handle(const void* d_ptr, unsigned char* handle, unsigned long long* offset);
int rt_ipc_open(const unsigned char* handle, unsigned long long offset, int device, int owner_device, void** d_ptr);
int rt_ipc_close(void* d_ptr, unsigned long long offset);

/* Milliseconds of the last launch on this scene, measured with hipEvents
 * recorded around the kernel on its stream (waits for it).  Returns RT_ERR_HIP when a launch on
 * the scene tripped the kernel watchdog (rt_scene_status). */
int rt_last_kernel_ms(rt_scene* scene, float* ms);

/* RT_OK, or RT_ERR_HIP once any finished launch on this scene tripped a kernel watchdog (a
 * traversal loop that ran past its iteration bound: a cyclic or corrupt hierarchy, or a kernel
 * bug).  The kernel mirrors the flag into page-locked host memory, so launches without stats
 * report it too: from then on every launch on the scene, rt_last_kernel_ms and this call return
 * RT_ERR_HIP (sticky; the scene's results are void -- free it and upload again).  Replaces the
 * reference's CHECK-and-continue (common/common.h:6-15).  Does not synchronise. */
int rt_scene_status(const rt_scene* scene);

/* Diagnostics: raw device counter words of the last launch (synchronises the
 * device).  Words [8,16) = rt_stats order (from node_visits on: STATS flags only;
 * the ray counts [8,11) are the kernel's per-wave slots, summed here); with a STATS flag, words [16,30) =
 * node-loop iterations / active lanes, leaf-loop iterations / active lanes,
 * traverse / shade / refill cycles (s_memtime), outer iterations, traversal
 * rounds / active lanes (per wave, summed), traversal-stack entries spilled
 * from the LDS ring to global memory, distinct nodes / triangle lines per
 * wave-level node / leaf iteration (summed), triangle tests in leaves of > 4,
 * node iterations served from the LDS treelet; word 31 = watchdog flag; words
 * [32,35) = global-node iterations with one node for the whole wave, distinct
 * nodes of global-node iterations (summed), leaf iterations with one record.
 * Returns the number of words copied (at most 40). */
int rt_debug_counters(rt_scene* scene, unsigned long long* out, int n);

/* Diagnostics: per-wave timeline of the last launch with a STATS flag: words
 * [4w, 4w+4) of wave w of the persistent grid = {start, last successful work
 * fetch, end} (s_memrealtime, 100 MHz) and pixels fetched; waves that were not
 * launched keep stale words.  Synchronises the device; returns words copied. */
long long rt_debug_wave_log(rt_scene* scene, unsigned long long* out, long long n);

/* Diagnostics: persistent-grid blocks per CU of kernel variant 0 (production), 1 (4-wide
 * STATS), 2 (2-wide canonical STATS), 3 (timeline), 4 (production, 16-entry stack ring), 5 / 6
 * (0 / 4 with sample groups, spp > 1), as the launches use it. */
int rt_debug_blocks_per_cu(rt_scene* scene, int variant);

/* Diagnostics: the persistent grid (blocks) the last launch on the scene used, and the grid a
 * launch of that shape gets when the device is otherwise idle.  They differ for a one-frame launch
 * issued while the scene's previous launch, on another stream, was still running: it takes half
 * the block slots, so the two overlap (pixels and counts do not depend on it).  Either pointer may
 * be NULL. */
int rt_debug_last_grid(rt_scene* scene, long long* blocks, long long* full_blocks);

/* Test hook: replaces the scene's first 4-wide node by a cycle (its one child is itself, with a
 * box that holds every ray), so every production traversal that enters the hierarchy loops until
 * the kernel watchdog ends it.  Synchronises the device.  The scene is unusable afterwards. */
int rt_debug_corrupt_hierarchy(rt_scene* scene);

/* Diagnostics: per-round timeline of the last launch with RT_FLAG_TIMELINE: for wave w of the
 * persistent grid and its r-th traversal round (r < 256), words [8(256w + r), +8) = {round start,
 * round end} (s_memrealtime, 100 MHz ticks), busy lanes | owner lanes << 8 | (work queue not yet
 * empty) << 16 | shadow-ray lanes << 24, the most node + leaf iterations of a lane | the wave's
 * round-loop iterations << 32, then the time (ticks) | count << 40 of the wave-level iterations of
 * each kind: global-memory node, LDS-treelet node, leaf; last word: the longest wave-level iteration
 * | the round's setup time << 32.  Unused records are zero.  Synchronises the device; returns
 * words copied. */
long long rt_debug_timeline(rt_scene* scene, unsigned long long* out, long long n);

/* The render kernel's work tile: one wave's 64 pixels, *tile_w x *tile_h (8 x 8).  Tile positions
 * of the diagnostics below are ty * ceil(width / tile_w) + tx over the shard's
 * ceil(rows / tile_h) tile rows. */
int rt_tile_shape(int* tile_w, int* tile_h);

/* Diagnostics (tile-order experiments): the per-tile-position cost map of the last launch with
 * RT_FLAG_TILE_COST / RT_FLAG_TILE_COST_TIME / RT_FLAG_COST_ORDER (index ty * tiles_x + tx over the
 * shard's tiles (rt_tile_shape); per finished sample its bounces + 1, or per pixel its lifetime in 10-ns ticks;
 * summed over the launch's frames) into out[0..n); returns the number of positions, 0 if none. */
long long rt_debug_tile_cost(rt_scene* scene, unsigned int* out, long long n);
/* Diagnostics: launches with exactly n tiles take linear tile order[w / 64] for work item w (a
 * permutation; pixels do not depend on it); n = 0 clears. */
int rt_debug_set_tile_order(rt_scene* scene, const unsigned int* order, long long n);
/* Diagnostics: the tile order the last RT_FLAG_COST_ORDER launch used (order[i] = tile rendered i-th
 * within its work head's range) into out[0..n); returns its length, 0 if none. */
long long rt_debug_last_tile_order(rt_scene* scene, unsigned int* out, long long n);

void rt_scene_free(rt_scene* scene);

/* Thread-local message of the last failing call. */
const char* rt_last_error(void);

/* Build info string (kernel variants, arch) for logs. */
const char* rt_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_H */
