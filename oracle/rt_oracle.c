/*
 * rt_oracle.c — CPU ORACLE (test infrastructure only; see rt_oracle.h).
 *
 * Plain-C restatement of the reference CPU renderer of hvkwak/my-raytracer:
 *   normals            mymesh.cpp:103-163   (Mesh::compute_normals)
 *   triangle test      mymesh.cpp:176-236   (Mesh::intersect_triangle)
 *   texture lookup     mymesh.cpp:70-95     (Mesh::compute_texture)
 *   plane test         myplane.cpp:22-49    (Plane::intersect)
 *   det helpers        myutils.cpp:21-51
 *   BVH build (AoS)    mybvh.cpp:44-81, 220-362
 *   AABB test          mybvh.cpp:99-135     (BVH::intersectAABB, incl. its NaN behaviour)
 *   BVH traversal      mybvh.cpp:147-210    (recursive, unordered, strict t < best)
 *   lighting           mytracer.cpp:510-534, 568-608
 *   reflection         mytracer.cpp:546-555 (subtrace: recurse only if mirror > 0)
 *   sample pattern     mytracer_gpu.cu:202-224
 * and the [ABSENT] course pieces as fixed in DESIGN.md §2 (Camera, Ray,
 * trace, intersect_scene, compute_image, Sphere::intersect).
 *
 * PARITY UNPINNED against reference outputs (no reference tests/fixtures
 * exist and the reference cannot be compiled here without the absent course
 * headers).  Pinned instead by hand-derived known answers, tests/golden/.
 *
 * OR_MODE_ORDERED replicates the GPU traversal ALGORITHM (ordered, t-culled,
 * conservative fp32 boxes, any-hit shadow rays) so tests can pin the
 * kernel's traversal counters (algorithmic bytes).  Compile
 * with -ffp-contract=off: every fp op here must round exactly once.
 */
#include "rt_oracle.h"

#include <alloca.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* fp64 vector helpers (course vec4 ops on xyz)          */
/* ------------------------------------------------------------------ */
static inline double dot3(const double a[3], const double b[3]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static inline double norm3(const double a[3]) { return sqrt(dot3(a, a)); }
static inline void normalize3(double v[3]) {
  double n = norm3(v);
  if (n > 0.0) { v[0] = v[0] / n; v[1] = v[1] / n; v[2] = v[2] / n; }
}
static inline void sub3(const double a[3], const double b[3], double r[3]) {
  r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2];
}
static inline void cross3(const double a[3], const double b[3], double r[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
/* std::max / std::min argument semantics (NaN in the first slot survives). */
static inline double std_max(double a, double b) { return (a < b) ? b : a; }
static inline double std_min(double a, double b) { return (b < a) ? b : a; }

/* det2D / det4D, myutils.cpp:21-51 (det4D = 3x3 determinant of three columns). */
static inline double det2(double a, double b, double c, double d) { return a * d - b * c; }
static inline double det3c(const double v1[3], const double v2[3], const double v3[3]) {
  return v1[0] * det2(v2[1], v3[1], v2[2], v3[2]) - v2[0] * det2(v1[1], v3[1], v1[2], v3[2]) +
         v3[0] * det2(v1[1], v2[1], v1[2], v2[2]);
}

typedef struct { double o[3]; double d[3]; } ray_t;

/* Ray(o, d): the course Ray normalises its direction. */
static inline void make_ray(const double o[3], const double d[3], ray_t* r) {
  r->o[0] = o[0]; r->o[1] = o[1]; r->o[2] = o[2];
  r->d[0] = d[0]; r->d[1] = d[1]; r->d[2] = d[2];
  normalize3(r->d);
}

/* ------------------------------------------------------------------ */
/* context                                                            */
/* ------------------------------------------------------------------ */
typedef struct { int mesh; int tri; } tri_ref;

#define GREF_LEAF 0x80000000u
#define GREF_EMPTY 0x7fffffffu

struct or_ctx {
  const rt_raw_scene* s;
  int n_meshes;
  long long* tri_base;       /* [n_meshes] global triangle id of mesh's first triangle */
  long long* vtx_base;       /* [n_meshes] */
  double** vnormals;         /* [mesh][3*nv] */
  double** fnormals;         /* [mesh][3*nt] */
  /* reference BVH (mybvh.h:100-173 BVHNode pool) */
  long long n_tris;
  tri_ref* tris;             /* triangles_ in leaf order */
  double* cent;              /* centroid per original global triangle id [3*n] */
  int n_alloc, nodes_used;
  double* bmin; double* bmax;
  int* left; int* first; int* count;
  int depth;
  /* GPU-layout replica for OR_MODE_ORDERED */
  int n_g;
  float* gbox;               /* [n_g*12]: x{lo0,hi0,lo1,hi1} y{..} z{..} */
  uint32_t* gref;            /* [n_g*2] */
  unsigned char* tri_last;   /* [n_tris] last triangle of a leaf */
  double delta;
  double root_lo[3], root_hi[3];
};

static const double* vpos(const or_ctx* C, int m, int vi) {
  return C->s->meshes[m].positions + 3 * (long long)vi;
}

/* ------------------------------------------------------------------ */
/* Mesh::compute_normals, mymesh.cpp:103-163                           */
/* ------------------------------------------------------------------ */
static void compute_normals(const rt_mesh* M, double* vn, double* fn) {
  const double eps = 1e-12;
  for (int v = 0; v < M->n_vertices; ++v) { vn[3 * v] = 0.0; vn[3 * v + 1] = 0.0; vn[3 * v + 2] = 0.0; }
  for (int t = 0; t < M->n_triangles; ++t) {   /* face normals, :111-117 */
    const int* ix = M->tri_vertex + 3 * t;
    const double* p0 = M->positions + 3 * ix[0];
    const double* p1 = M->positions + 3 * ix[1];
    const double* p2 = M->positions + 3 * ix[2];
    double a[3], b[3], n[3];
    sub3(p1, p0, a); sub3(p2, p0, b); cross3(a, b, n); normalize3(n);
    fn[3 * t] = n[0]; fn[3 * t + 1] = n[1]; fn[3 * t + 2] = n[2];
  }
  for (int t = 0; t < M->n_triangles; ++t) {   /* angle weights, :120-157 */
    const int* ix = M->tri_vertex + 3 * t;
    const double* p0 = M->positions + 3 * ix[0];
    const double* p1 = M->positions + 3 * ix[1];
    const double* p2 = M->positions + 3 * ix[2];
    double v0[3], v1[3], v2[3], mv0[3], mv1[3], mv2[3];
    sub3(p1, p0, v0); sub3(p2, p1, v1); sub3(p0, p2, v2);
    const double l0 = norm3(v0), l1 = norm3(v1), l2 = norm3(v2);
    for (int k = 0; k < 3; ++k) { mv0[k] = -v0[k]; mv1[k] = -v1[k]; mv2[k] = -v2[k]; }
    const double d0 = dot3(v0, mv2), d1 = dot3(v1, mv0), d2 = dot3(v2, mv1);
    const double w0 = l0 * l2 + d0, w1 = l1 * l0 + d1, w2 = l2 * l1 + d2;
    const double* n = fn + 3 * t;
    if (fabs(w0) > eps) for (int k = 0; k < 3; ++k) vn[3 * ix[0] + k] += n[k] / w0;
    if (fabs(w1) > eps) for (int k = 0; k < 3; ++k) vn[3 * ix[1] + k] += n[k] / w1;
    if (fabs(w2) > eps) for (int k = 0; k < 3; ++k) vn[3 * ix[2] + k] += n[k] / w2;
  }
  for (int v = 0; v < M->n_vertices; ++v) normalize3(vn + 3 * v);
}

/* ------------------------------------------------------------------ */
/* BVH build, mybvh.cpp:44-81 (init), 220-362                          */
/* ------------------------------------------------------------------ */
/* k-th smallest (0-based) by quickselect; equivalent value to nth_element. */
static double select_kth(double* a, int n, int k) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    double pivot = a[lo + (hi - lo) / 2];
    int i = lo, j = hi;
    while (i <= j) {
      while (a[i] < pivot) i++;
      while (a[j] > pivot) j--;
      if (i <= j) { double t = a[i]; a[i] = a[j]; a[j] = t; i++; j--; }
    }
    if (k <= j) hi = j; else if (k >= i) lo = i; else return a[k];
  }
  return a[k];
}

/* BVH::median_inplace, mybvh.cpp:346-362. */
double or_median(double* a, int n) {
  const int mid = n / 2;
  if (n % 2 == 1) return select_kth(a, n, mid);
  const double hi = select_kth(a, n, mid);
  double lo = a[0];                       /* max of the lower part = (mid-1)-th smallest */
  for (int i = 1; i < mid; ++i) if (a[i] > lo) lo = a[i];
  return 0.5 * (lo + hi);
}

static void update_bounds(or_ctx* C, int node) {     /* mybvh.cpp:243-259 */
  double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (int i = C->first[node]; i < C->first[node] + C->count[node]; ++i) {
    const tri_ref tr = C->tris[i];
    const int* ix = C->s->meshes[tr.mesh].tri_vertex + 3 * tr.tri;
    for (int c = 0; c < 3; ++c) {
      const double* p = vpos(C, tr.mesh, ix[c]);
      for (int k = 0; k < 3; ++k) { mn[k] = fmin(mn[k], p[k]); mx[k] = fmax(mx[k], p[k]); }
    }
  }
  memcpy(C->bmin + 3 * node, mn, sizeof mn);
  memcpy(C->bmax + 3 * node, mx, sizeof mx);
}

static double centroid_axis(const or_ctx* C, tri_ref tr, int axis) {
  return C->cent[3 * (C->tri_base[tr.mesh] + tr.tri) + axis];
}

/* BVH::subdivide (mybvh.cpp:266-300) with an explicit LIFO stack that keeps
 * the recursion's node numbering (children allocated when the parent splits,
 * left subtree fully before the right one). */
static int build_bvh(or_ctx* C) {
  const long long N = C->n_tris;
  if (N <= 0) { C->nodes_used = 0; return 0; }
  C->n_alloc = (int)(2 * N - 1);
  C->bmin = (double*)malloc(sizeof(double) * 3 * C->n_alloc);
  C->bmax = (double*)malloc(sizeof(double) * 3 * C->n_alloc);
  C->left = (int*)calloc(C->n_alloc, sizeof(int));
  C->first = (int*)calloc(C->n_alloc, sizeof(int));
  C->count = (int*)calloc(C->n_alloc, sizeof(int));
  int* stack_node = (int*)malloc(sizeof(int) * (C->n_alloc + 1));
  int* stack_depth = (int*)malloc(sizeof(int) * (C->n_alloc + 1));
  double* scratch = (double*)malloc(sizeof(double) * N);
  if (!C->bmin || !C->bmax || !C->left || !C->first || !C->count || !stack_node || !stack_depth || !scratch)
    return -1;
  C->left[0] = 0; C->first[0] = 0; C->count[0] = (int)N;
  C->nodes_used = 1;
  update_bounds(C, 0);
  int sp = 0, maxd = 0;
  stack_node[sp] = 0; stack_depth[sp] = 1; sp++;
  while (sp > 0) {
    --sp;
    const int node = stack_node[sp], depth = stack_depth[sp];
    if (depth - 1 > maxd) maxd = depth - 1;
    if (C->count[node] <= 2) continue;                       /* :270 */
    const int axis = depth % 3;                              /* :273 */
    const int f = C->first[node], n = C->count[node];
    for (int i = 0; i < n; ++i) scratch[i] = centroid_axis(C, C->tris[f + i], axis);
    const double split = or_median(scratch, n);              /* :274, 328-339 */
    int i = f, j = f + n - 1;                                /* :309-320 */
    while (i <= j) {
      if (centroid_axis(C, C->tris[i], axis) < split) i++;
      else { tri_ref t = C->tris[i]; C->tris[i] = C->tris[j]; C->tris[j] = t; j--; }
    }
    const int left_count = i - f;
    if (left_count == 0 || left_count == n) continue;        /* :282 */
    const int l = C->nodes_used, r = l + 1;                  /* :285-293 */
    C->nodes_used += 2;
    C->first[l] = f; C->count[l] = left_count;
    C->first[r] = i; C->count[r] = n - left_count;
    C->left[node] = l; C->count[node] = 0;
    update_bounds(C, l); update_bounds(C, r);
    stack_node[sp] = r; stack_depth[sp] = depth + 1; sp++;   /* right popped after left */
    stack_node[sp] = l; stack_depth[sp] = depth + 1; sp++;
  }
  /* leaves' depth: children of the deepest split */
  C->depth = maxd;
  free(stack_node); free(stack_depth); free(scratch);
  return 0;
}

/* ------------------------------------------------------------------ */
/* GPU-layout replica (conservative fp32 2-wide nodes)  */
/* ------------------------------------------------------------------ */
static float round_down_f(double x) {
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}
static float round_up_f(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, INFINITY);
  return f;
}

static int build_gpu_replica(or_ctx* C) {
  double M = 0.0;
  for (int m = 0; m < C->n_meshes; ++m) {
    const rt_mesh* me = &C->s->meshes[m];
    for (long long k = 0; k < 3LL * me->n_vertices; ++k) {
      double a = fabs(me->positions[k]);
      if (a > M) M = a;
    }
  }
  if (!(M > 0.0)) M = 1.0;
  C->delta = M * 9.5367431640625e-07;   /* 2^-20 */
  if (C->nodes_used == 0) { C->n_g = 0; return 0; }
  for (int k = 0; k < 3; ++k) {
    C->root_lo[k] = C->bmin[k] - C->delta;
    C->root_hi[k] = C->bmax[k] + C->delta;
  }
  int n_internal = 0;
  for (int i = 0; i < C->nodes_used; ++i) if (C->count[i] == 0) n_internal++;
  const int ng = n_internal > 0 ? n_internal : 1;
  C->n_g = ng;
  C->gbox = (float*)malloc(sizeof(float) * 12 * ng);
  C->gref = (uint32_t*)malloc(sizeof(uint32_t) * 2 * ng);
  C->tri_last = (unsigned char*)calloc(C->n_tris, 1);
  int* gidx = (int*)malloc(sizeof(int) * C->nodes_used);
  int* stk = (int*)malloc(sizeof(int) * (C->nodes_used + 1));
  if (!C->gbox || !C->gref || !C->tri_last || !gidx || !stk) return -1;
  for (int i = 0; i < C->nodes_used; ++i) {
    gidx[i] = -1;
    if (C->count[i] > 0) C->tri_last[C->first[i] + C->count[i] - 1] = 1;
  }
  /* child box of reference node c into slot s of g-node g */
#define SET_CHILD(g, s, c)                                                      \
  do {                                                                          \
    for (int k = 0; k < 3; ++k) {                                               \
      C->gbox[12 * (g) + 4 * k + 2 * (s)] = round_down_f(C->bmin[3 * (c) + k] - C->delta); \
      C->gbox[12 * (g) + 4 * k + 2 * (s) + 1] = round_up_f(C->bmax[3 * (c) + k] + C->delta); \
    }                                                                           \
  } while (0)
  if (n_internal == 0) {            /* root is a leaf */
    SET_CHILD(0, 0, 0);
    for (int k = 0; k < 3; ++k) { C->gbox[12 * 0 + 4 * k + 2] = 0.0f; C->gbox[12 * 0 + 4 * k + 3] = 0.0f; }
    C->gref[0] = GREF_LEAF | (uint32_t)C->first[0];
    C->gref[1] = GREF_EMPTY;
  } else {                          /* preorder numbering, left first */
    int sp = 0, next = 0;
    stk[sp++] = 0;
    while (sp > 0) {
      int n = stk[--sp];
      gidx[n] = next++;
      int l = C->left[n], r = l + 1;
      if (C->count[r] == 0) stk[sp++] = r;
      if (C->count[l] == 0) stk[sp++] = l;
    }
    for (int n = 0; n < C->nodes_used; ++n) {
      if (C->count[n] != 0 || gidx[n] < 0) continue;
      int g = gidx[n];
      for (int s = 0; s < 2; ++s) {
        int c = C->left[n] + s;
        SET_CHILD(g, s, c);
        C->gref[2 * g + s] = (C->count[c] == 0) ? (uint32_t)gidx[c] : (GREF_LEAF | (uint32_t)C->first[c]);
      }
    }
  }
#undef SET_CHILD
  free(gidx); free(stk);
  return 0;
}

/* ------------------------------------------------------------------ */
/* prepare / free / exports                                            */
/* ------------------------------------------------------------------ */
or_ctx* or_prepare(const rt_raw_scene* s) {
  or_ctx* C = (or_ctx*)calloc(1, sizeof(or_ctx));
  if (!C) return NULL;
  C->s = s;
  C->n_meshes = s->n_meshes;
  C->tri_base = (long long*)calloc(s->n_meshes + 1, sizeof(long long));
  C->vtx_base = (long long*)calloc(s->n_meshes + 1, sizeof(long long));
  C->vnormals = (double**)calloc(s->n_meshes + 1, sizeof(double*));
  C->fnormals = (double**)calloc(s->n_meshes + 1, sizeof(double*));
  long long nt = 0, nv = 0;
  for (int m = 0; m < s->n_meshes; ++m) {
    const rt_mesh* M = &s->meshes[m];
    if (M->draw_mode != RT_DRAW_FLAT && M->draw_mode != RT_DRAW_PHONG) { or_free(C); return NULL; }
    C->tri_base[m] = nt; C->vtx_base[m] = nv;
    nt += M->n_triangles; nv += M->n_vertices;
    C->vnormals[m] = (double*)malloc(sizeof(double) * 3 * (M->n_vertices + 1));
    C->fnormals[m] = (double*)malloc(sizeof(double) * 3 * (M->n_triangles + 1));
    compute_normals(M, C->vnormals[m], C->fnormals[m]);
  }
  C->n_tris = nt;
  C->tris = (tri_ref*)malloc(sizeof(tri_ref) * (nt + 1));
  C->cent = (double*)malloc(sizeof(double) * 3 * (nt + 1));
  long long g = 0;
  for (int m = 0; m < s->n_meshes; ++m) {          /* BVH::getData, mybvh.cpp:220-237 */
    const rt_mesh* M = &s->meshes[m];
    for (int t = 0; t < M->n_triangles; ++t, ++g) {
      C->tris[g].mesh = m; C->tris[g].tri = t;
      const int* ix = M->tri_vertex + 3 * t;
      const double* p0 = M->positions + 3 * ix[0];
      const double* p1 = M->positions + 3 * ix[1];
      const double* p2 = M->positions + 3 * ix[2];
      for (int k = 0; k < 3; ++k) C->cent[3 * g + k] = (p0[k] + p1[k] + p2[k]) / 3.0;
    }
  }
  if (build_bvh(C) != 0 || build_gpu_replica(C) != 0) { or_free(C); return NULL; }
  return C;
}

void or_free(or_ctx* C) {
  if (!C) return;
  for (int m = 0; m < C->n_meshes; ++m) {
    if (C->vnormals) free(C->vnormals[m]);
    if (C->fnormals) free(C->fnormals[m]);
  }
  free(C->vnormals); free(C->fnormals); free(C->tri_base); free(C->vtx_base);
  free(C->tris); free(C->cent);
  free(C->bmin); free(C->bmax); free(C->left); free(C->first); free(C->count);
  free(C->gbox); free(C->gref); free(C->tri_last);
  free(C);
}

long long or_n_triangles(const or_ctx* C) { return C->n_tris; }
int or_n_nodes(const or_ctx* C) { return C->nodes_used; }
int or_tree_depth(const or_ctx* C) { return C->depth; }

void or_export_bvh(const or_ctx* C, double* bb_min, double* bb_max, int* left, int* first,
                   int* count, int* perm) {
  if (C->nodes_used > 0) {
    memcpy(bb_min, C->bmin, sizeof(double) * 3 * C->nodes_used);
    memcpy(bb_max, C->bmax, sizeof(double) * 3 * C->nodes_used);
    memcpy(left, C->left, sizeof(int) * C->nodes_used);
    memcpy(first, C->first, sizeof(int) * C->nodes_used);
    memcpy(count, C->count, sizeof(int) * C->nodes_used);
  }
  for (long long i = 0; i < C->n_tris; ++i) perm[i] = (int)(C->tri_base[C->tris[i].mesh] + C->tris[i].tri);
}

void or_export_normals(const or_ctx* C, double* vn, double* fn) {
  for (int m = 0; m < C->n_meshes; ++m) {
    const rt_mesh* M = &C->s->meshes[m];
    memcpy(vn + 3 * C->vtx_base[m], C->vnormals[m], sizeof(double) * 3 * M->n_vertices);
    memcpy(fn + 3 * C->tri_base[m], C->fnormals[m], sizeof(double) * 3 * M->n_triangles);
  }
}

/* ------------------------------------------------------------------ */
/* Camera (course framework [ABSENT]; restated)          */
/* ------------------------------------------------------------------ */
void or_camera(const rt_camera_def* def, int width, int height, rt_camera* out) {
  if (width <= 0) width = def->width;
  if (height <= 0) height = def->height;
  double view[3], xd[3], yd[3];
  sub3(def->center, def->eye, view);
  const double dist = norm3(view);
  normalize3(view);
  const double image_height = 2.0 * dist * tan(0.5 * def->fovy / 180.0 * M_PI);
  const double image_width = (double)width / (double)height * image_height;
  cross3(view, def->up, xd); normalize3(xd);
  for (int k = 0; k < 3; ++k) xd[k] = xd[k] * image_width / (double)width;
  cross3(xd, view, yd); normalize3(yd);
  for (int k = 0; k < 3; ++k) yd[k] = yd[k] * image_height / (double)height;
  for (int k = 0; k < 3; ++k) {
    out->eye[k] = def->eye[k];
    out->x_dir[k] = xd[k];
    out->y_dir[k] = yd[k];
    out->lower_left[k] = def->center[k] - 0.5 * (double)width * xd[k] - 0.5 * (double)height * yd[k];
  }
  out->width = width;
  out->height = height;
}

static void primary_ray(const rt_camera* cam, double x, double y, ray_t* r) {
  double d[3];
  for (int k = 0; k < 3; ++k) d[k] = cam->lower_left[k] + x * cam->x_dir[k] + y * cam->y_dir[k] - cam->eye[k];
  make_ray(cam->eye, d, r);
}

/* ------------------------------------------------------------------ */
/* intersections                                                       */
/* ------------------------------------------------------------------ */
/* Mesh::intersect_triangle core, mymesh.cpp:186-215. */
int or_intersect_triangle(const double p0[3], const double p1[3], const double p2[3],
                          const double o[3], const double d[3],
                          double* t_out, double* alpha_out, double* beta_out, double* gamma_out) {
  const double c1[3] = {p0[0] - p2[0], p0[1] - p2[1], p0[2] - p2[2]};
  const double c2[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
  const double c3[3] = {-d[0], -d[1], -d[2]};
  const double c4[3] = {o[0] - p2[0], o[1] - p2[1], o[2] - p2[2]};
  const double S = det3c(c1, c2, c3);
  if (fabs(S) < 1e-10) return 0;                               /* :197 */
  const double alpha = det3c(c4, c2, c3) / S;
  const double beta = det3c(c1, c4, c3) / S;
  const double gamma = (1.0 - alpha - beta);
  const double t = det3c(c1, c2, c4) / S;
  if (t <= 1e-5) return 0;                                     /* :206-208 */
  if (!((0.0 <= alpha && alpha <= 1.0) && (0.0 <= beta && beta <= 1.0) &&
        (0.0 <= gamma && gamma <= 1.0)))
    return 0;
  *t_out = t; *alpha_out = alpha; *beta_out = beta; *gamma_out = gamma;
  return 1;
}

/* BVH::intersectAABB, mybvh.cpp:99-135 (std::max/min semantics, no z in tmin). */
int or_intersect_aabb(const double o[3], const double d[3], const double bmin[3], const double bmax[3]) {
  double tmin = (bmin[0] - o[0]) / d[0];
  double tmax = (bmax[0] - o[0]) / d[0];
  if (tmin > tmax) { double t = tmin; tmin = tmax; tmax = t; }
  double tymin = (bmin[1] - o[1]) / d[1];
  double tymax = (bmax[1] - o[1]) / d[1];
  if (tymin > tymax) { double t = tymin; tymin = tymax; tymax = t; }
  if ((tmin > tymax) || (tymin > tmax)) return 0;
  tmin = std_max(tmin, tymin);
  tmax = std_min(tmax, tymax);
  double tzmin = (bmin[2] - o[2]) / d[2];
  double tzmax = (bmax[2] - o[2]) / d[2];
  if (tzmin > tzmax) { double t = tzmin; tzmin = tzmax; tzmax = t; }
  if ((tmin > tzmax) || (tzmin > tmax)) return 0;
  tmax = std_min(tmax, tzmax);
  return tmax > 1e-5;
}

typedef struct {
  double t;
  double p[3];
  double n[3];
  double diffuse[3];
  const rt_material* mat;
  int tri_id;   /* global original id, -1 analytic */
} hit_t;

/* Triangle attributes at an accepted hit: mymesh.cpp:217-235 + 70-95. */
static void triangle_shade(const or_ctx* C, tri_ref tr, const ray_t* r, double t, double alpha,
                           double beta, double gamma, hit_t* h) {
  const rt_mesh* M = &C->s->meshes[tr.mesh];
  h->t = t;
  for (int k = 0; k < 3; ++k) h->p[k] = r->o[k] + t * r->d[k];
  h->mat = &M->material;
  for (int k = 0; k < 3; ++k) h->diffuse[k] = M->material.diffuse[k];
  if (M->texture.width > 0 && M->tri_uv) {                      /* compute_texture :70-95 */
    const int* iuv = M->tri_uv + 3 * tr.tri;
    double u = alpha * M->u[iuv[0]] + beta * M->u[iuv[1]] + gamma * M->u[iuv[2]];
    double v = alpha * M->v[iuv[0]] + beta * M->v[iuv[1]] + gamma * M->v[iuv[2]];
    u = fmin(fmax(u, 0.0), 1.0);   /* NaN -> 0, as mytracer_gpu.cu:532-533 */
    v = fmin(fmax(v, 0.0), 1.0);
    const unsigned W = (unsigned)M->texture.width, H = (unsigned)M->texture.height;
    const int px = (int)round(u * (W - 1));
    const int py = (int)round((1.0 - v) * (H - 1));
    const unsigned char* tx = M->texture.rgb + 3 * ((long long)py * W + px);
    for (int k = 0; k < 3; ++k) h->diffuse[k] = (double)tx[k] / 255.0;
  }
  if (M->draw_mode == RT_DRAW_FLAT) {
    const double* fn = C->fnormals[tr.mesh] + 3 * tr.tri;
    for (int k = 0; k < 3; ++k) h->n[k] = fn[k];
  } else {
    const int* ix = M->tri_vertex + 3 * tr.tri;
    const double* vn = C->vnormals[tr.mesh];
    for (int k = 0; k < 3; ++k)
      h->n[k] = alpha * vn[3 * ix[0] + k] + beta * vn[3 * ix[1] + k] + gamma * vn[3 * ix[2] + k];
  }
  h->tri_id = (int)(C->tri_base[tr.mesh] + tr.tri);
}

static int test_tri(const or_ctx* C, tri_ref tr, const ray_t* r, double* t, double* a, double* b, double* g) {
  const rt_mesh* M = &C->s->meshes[tr.mesh];
  const int* ix = M->tri_vertex + 3 * tr.tri;
  return or_intersect_triangle(M->positions + 3 * ix[0], M->positions + 3 * ix[1],
                               M->positions + 3 * ix[2], r->o, r->d, t, a, b, g);
}

/* Plane::intersect, myplane.cpp:22-49. */
static int plane_hit(const rt_plane* P, const ray_t* r, double* t_out) {
  const double cosTheta = dot3(P->normal, r->d);
  if (fabs(cosTheta) < 1e-9) return 0;
  const double distance = dot3(P->normal, P->center);
  const double t = (distance - dot3(P->normal, r->o)) / dot3(P->normal, r->d);
  if (t > 1e-5) { *t_out = t; return 1; }
  return 0;
}

/* Sphere::intersect ([ABSENT]; restated). */
static int sphere_hit(const rt_sphere* S, const ray_t* r, double* t_out) {
  double oc[3];
  sub3(r->o, S->center, oc);
  const double a = dot3(r->d, r->d);
  const double b = 2.0 * dot3(r->d, oc);
  const double c = dot3(oc, oc) - S->radius * S->radius;
  const double disc = b * b - 4.0 * a * c;
  if (disc < 0.0) return 0;
  const double sq = sqrt(disc);
  const double t1 = (-b - sq) / (2.0 * a), t2 = (-b + sq) / (2.0 * a);
  double t = DBL_MAX;
  if (t1 > 1e-5 && t1 < t) t = t1;
  if (t2 > 1e-5 && t2 < t) t = t2;
  if (t == DBL_MAX) return 0;
  *t_out = t;
  return 1;
}

/* BVH::intersectBVH, mybvh.cpp:147-210 (recursive, unordered). */
typedef struct { double t; int slot; double a, b, g; } best_t;

static int bvh_ref(const or_ctx* C, const ray_t* r, best_t* best, int node, or_counts* cnt) {
  cnt->box_tests++;
  if (!or_intersect_aabb(r->o, r->d, C->bmin + 3 * node, C->bmax + 3 * node)) return 0;
  if (C->count[node] > 0) {
    for (int i = C->first[node]; i < C->first[node] + C->count[node]; ++i) {
      double t, a, b, g;
      cnt->tri_tests++;
      if (test_tri(C, C->tris[i], r, &t, &a, &b, &g)) {
        if (t < best->t) { best->t = t; best->slot = i; best->a = a; best->b = b; best->g = g; }
      }
    }
    return best->t < DBL_MAX;
  }
  int hl = 0, hr = 0;
  const int l = C->left[node];
  cnt->box_tests++;
  if (or_intersect_aabb(r->o, r->d, C->bmin + 3 * l, C->bmax + 3 * l)) hl = bvh_ref(C, r, best, l, cnt);
  cnt->box_tests++;
  if (or_intersect_aabb(r->o, r->d, C->bmin + 3 * (l + 1), C->bmax + 3 * (l + 1))) hr = bvh_ref(C, r, best, l + 1, cnt);
  return hl || hr;
}

/* ---- ordered, t-culled fp32 traversal (GPU algorithm replica) ---- */
typedef struct {
  float of[3];
  float inv[3];
  double t_off;
  int miss;
} gray_t;

/* Per-ray setup shared with the kernel (rt_kernel.hip: setup_box_ray). */
static void gray_setup(const or_ctx* C, const ray_t* r, gray_t* g) {
  g->miss = 0;
  g->t_off = 0.0;
  int inside = 1;
  for (int k = 0; k < 3; ++k)
    if (!(r->o[k] >= C->root_lo[k] && r->o[k] <= C->root_hi[k])) inside = 0;
  if (!inside) {
    double tn = -DBL_MAX, tf = DBL_MAX;
    for (int k = 0; k < 3; ++k) {
      if (r->d[k] == 0.0) {
        if (r->o[k] < C->root_lo[k] || r->o[k] > C->root_hi[k]) { g->miss = 1; return; }
        continue;
      }
      double t0 = (C->root_lo[k] - r->o[k]) / r->d[k];
      double t1 = (C->root_hi[k] - r->o[k]) / r->d[k];
      if (t0 > t1) { double t = t0; t0 = t1; t1 = t; }
      if (t0 > tn) tn = t0;
      if (t1 < tf) tf = t1;
    }
    if (tn > tf || tf < 0.0) { g->miss = 1; return; }
    g->t_off = tn > 0.0 ? tn : 0.0;
  }
  for (int k = 0; k < 3; ++k) {
    const double ob = r->o[k] + g->t_off * r->d[k];
    g->of[k] = (float)ob;
    float df = (float)r->d[k];
    if (fabsf(df) < 1e-20f) df = signbit(r->d[k]) ? -1e-20f : 1e-20f;
    g->inv[k] = 1.0f / df;
  }
}

static inline void box2(const float* bx, const gray_t* g, float lo_c, float hi_c, int* h0, float* tn0,
                        int* h1, float* tn1) {
  for (int s = 0; s < 2; ++s) {
    const float tx0 = (bx[0 + 2 * s] - g->of[0]) * g->inv[0], tx1 = (bx[1 + 2 * s] - g->of[0]) * g->inv[0];
    const float ty0 = (bx[4 + 2 * s] - g->of[1]) * g->inv[1], ty1 = (bx[5 + 2 * s] - g->of[1]) * g->inv[1];
    const float tz0 = (bx[8 + 2 * s] - g->of[2]) * g->inv[2], tz1 = (bx[9 + 2 * s] - g->of[2]) * g->inv[2];
    const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), lo_c));
    const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), hi_c));
    if (s == 0) { *h0 = tmin <= tmax; *tn0 = tmin; } else { *h1 = tmin <= tmax; *tn1 = tmin; }
  }
}

/* any_hit: terminate at the first valid triangle with t < tmax (shadow rays).
 * Closest-hit ties resolve to the smallest leaf slot (= the reference's
 * left-first visit order with strict <, mybvh.cpp:169).  Returns hit flag. */
static int bvh_ordered(const or_ctx* C, const ray_t* r, best_t* best, int any_hit, double tmax,
                       or_counts* cnt) {
  if (C->n_g == 0) return 0;
  gray_t g;
  gray_setup(C, r, &g);
  if (g.miss) return 0;
  const float lo_c = round_down_f(-g.t_off);
  float hi_c = round_up_f((any_hit ? tmax : best->t) - g.t_off);
  uint32_t* stack = (uint32_t*)alloca(sizeof(uint32_t) * (C->depth + 2));
  int sp = 0;
  uint32_t cur = 0;       /* internal g-node 0 */
  int found = 0;
  for (;;) {
    if (!(cur & GREF_LEAF)) {
      cnt->node_visits++;
      const float* bx = C->gbox + 12 * (size_t)cur;
      const uint32_t r0 = C->gref[2 * cur], r1 = C->gref[2 * cur + 1];
      int h0, h1; float tn0, tn1;
      box2(bx, &g, lo_c, hi_c, &h0, &tn0, &h1, &tn1);
      h1 = h1 && (r1 != GREF_EMPTY);
      if (h0 && h1) {
        if (tn1 < tn0) { stack[sp++] = r0; cur = r1; } else { stack[sp++] = r1; cur = r0; }
        continue;
      }
      if (h0) { cur = r0; continue; }
      if (h1) { cur = r1; continue; }
    } else {
      uint32_t i = cur & ~GREF_LEAF;
      for (;;) {
        double t, a, b, gm;
        cnt->tri_tests++;
        if (test_tri(C, C->tris[i], r, &t, &a, &b, &gm)) {
          if (any_hit) {
            if (t < tmax) { best->t = t; best->slot = (int)i; return 1; }
          } else if (t < best->t || (t == best->t && (int)i < best->slot)) {
            best->t = t; best->slot = (int)i; best->a = a; best->b = b; best->g = gm;
            hi_c = round_up_f(best->t - g.t_off);
            found = 1;
          }
        }
        if (C->tri_last[i]) break;
        ++i;
      }
    }
    if (sp == 0) break;
    cur = stack[--sp];
  }
  return found;
}

/* intersect_scene ([ABSENT]): analytic objects in order
 * (spheres, planes), then the BVH with the running best distance. */
static int intersect_scene(const or_ctx* C, const ray_t* r, int mode, hit_t* h, or_counts* cnt) {
  const rt_raw_scene* s = C->s;
  double tbest = DBL_MAX;
  const rt_material* obj_mat = NULL;
  double obj_n[3] = {0, 0, 0};
  for (int i = 0; i < s->n_spheres; ++i) {
    double t;
    if (sphere_hit(&s->spheres[i], r, &t) && t < tbest) {
      tbest = t; obj_mat = &s->spheres[i].material;
      for (int k = 0; k < 3; ++k) obj_n[k] = (r->o[k] + t * r->d[k] - s->spheres[i].center[k]) / s->spheres[i].radius;
    }
  }
  for (int i = 0; i < s->n_planes; ++i) {
    double t;
    if (plane_hit(&s->planes[i], r, &t) && t < tbest) {
      tbest = t; obj_mat = &s->planes[i].material;
      for (int k = 0; k < 3; ++k) obj_n[k] = s->planes[i].normal[k];
    }
  }
  best_t best = {tbest, obj_mat ? -1 : 0x7fffffff, 0, 0, 0};
  if (C->nodes_used > 0) {
    if (mode == OR_MODE_REFERENCE) bvh_ref(C, r, &best, 0, cnt);
    else bvh_ordered(C, r, &best, 0, 0.0, cnt);
  }
  if (!(best.t < DBL_MAX)) return 0;
  if (best.slot >= 0 && best.slot != 0x7fffffff) {
    triangle_shade(C, C->tris[best.slot], r, best.t, best.a, best.b, best.g, h);
  } else {
    h->t = best.t;
    for (int k = 0; k < 3; ++k) { h->p[k] = r->o[k] + best.t * r->d[k]; h->n[k] = obj_n[k]; h->diffuse[k] = obj_mat->diffuse[k]; }
    h->mat = obj_mat;
    h->tri_id = -1;
  }
  return 1;
}

/* Shadow query: reference = closest hit then t < light_distance
 * (mytracer.cpp:594-599); ordered = analytic objects + any-hit BVH. */
static int shadowed(const or_ctx* C, const ray_t* r, double light_distance, int mode, or_counts* cnt) {
  if (mode == OR_MODE_REFERENCE) {
    hit_t h;
    const int hit = intersect_scene(C, r, mode, &h, cnt);
    return hit && h.t < light_distance && 0.0 < h.t;
  }
  const rt_raw_scene* s = C->s;
  double tb = DBL_MAX;
  for (int i = 0; i < s->n_spheres; ++i) { double t; if (sphere_hit(&s->spheres[i], r, &t) && t < tb) tb = t; }
  for (int i = 0; i < s->n_planes; ++i) { double t; if (plane_hit(&s->planes[i], r, &t) && t < tb) tb = t; }
  if (tb < light_distance) return 1;
  if (C->nodes_used == 0) return 0;
  best_t best = {DBL_MAX, 0x7fffffff, 0, 0, 0};
  return bvh_ordered(C, r, &best, 1, light_distance, cnt);
}

/* ------------------------------------------------------------------ */
/* shading: mytracer.cpp:510-608                                       */
/* ------------------------------------------------------------------ */
static double diffuse_term(const double point[3], const double normal[3], const double lpos[3]) {
  double l[3];
  sub3(lpos, point, l); normalize3(l);
  const double c = dot3(normal, l);
  return std_max(0.0, c);
}

static double reflection_term(const double point[3], const double normal[3], const double view[3],
                              const double lpos[3]) {
  if (diffuse_term(point, normal, lpos) > 0.0) {
    double l[3], rr[3];
    sub3(lpos, point, l); normalize3(l);
    const double s = 2.0 * dot3(normal, l);            /* mirror(l, n) = 2(n.l)n - l */
    for (int k = 0; k < 3; ++k) rr[k] = s * normal[k] - l[k];
    normalize3(rr);
    const double c = dot3(rr, view);
    return std_max(0.0, c);
  }
  return 0.0;
}

static void lighting(const or_ctx* C, const rt_render_params* p, const hit_t* h, const double view[3],
                     int mode, double col[3], or_counts* cnt) {
  const double epsilon = 1e-4;
  const rt_material* mat = h->mat;
  col[0] = 0.0; col[1] = 0.0; col[2] = 0.0;
  for (int k = 0; k < 3; ++k) col[k] += p->ambience[k] * mat->ambient[k];
  for (int li = 0; li < p->n_lights; ++li) {
    const rt_light* L = rt_params_light(p, li);
    const double diff = diffuse_term(h->p, h->n, L->position);
    double refl = reflection_term(h->p, h->n, view, L->position);
    refl = pow(refl, mat->shininess);
    int is_shadow = 0;
    if (mat->shadowable) {
      double ld[3], tmp[3], o[3];
      sub3(L->position, h->p, tmp);
      for (int k = 0; k < 3; ++k) ld[k] = tmp[k];
      normalize3(ld);
      const double light_distance = norm3(tmp);
      for (int k = 0; k < 3; ++k) o[k] = h->p[k] + epsilon * ld[k];
      ray_t sr;
      make_ray(o, ld, &sr);
      cnt->shadow_rays++;
      is_shadow = shadowed(C, &sr, light_distance, mode, cnt);
    }
    for (int k = 0; k < 3; ++k)
      col[k] += L->color[k] * (double)(!is_shadow) * (h->diffuse[k] * diff + mat->specular[k] * refl);
  }
}

/* trace ([ABSENT]) with Raytracer::subtrace (mytracer.cpp:546-555). */
static void trace(const or_ctx* C, const rt_render_params* p, const ray_t* r, int depth, int mode,
                  double out[3], or_counts* cnt) {
  if (depth > p->max_depth) { out[0] = out[1] = out[2] = 0.0; return; }
  if (depth == 0) cnt->primary_rays++; else cnt->reflection_rays++;
  hit_t h;
  if (!intersect_scene(C, r, mode, &h, cnt)) {
    for (int k = 0; k < 3; ++k) out[k] = p->background[k];
    return;
  }
  cnt->closest_hits++;
  const double view[3] = {-r->d[0], -r->d[1], -r->d[2]};
  double col[3];
  lighting(C, p, &h, view, mode, col, cnt);
  double refl[3] = {0.0, 0.0, 0.0};
  const double m = h.mat->mirror;
  if (m > 0.0) {
    const double s = 2.0 * dot3(h.n, r->d);            /* reflect(d, n) = d - 2(n.d)n */
    double v[3], o[3], sub[3];
    for (int k = 0; k < 3; ++k) v[k] = r->d[k] - s * h.n[k];
    for (int k = 0; k < 3; ++k) o[k] = h.p[k] + 1e-4 * v[k];
    ray_t rr;
    make_ray(o, v, &rr);
    trace(C, p, &rr, depth + 1, mode, sub, cnt);
    for (int k = 0; k < 3; ++k) refl[k] = m * sub[k];
  }
  for (int k = 0; k < 3; ++k) out[k] = (1.0 - m) * col[k] + refl[k];
}

/* compute_image for one pixel ([ABSENT]; sample pattern mytracer_gpu.cu:202-224). */
static void render_pixel(const or_ctx* C, const rt_render_params* p, int x, int y, int mode,
                         double out[3], or_counts* cnt) {
  const int n = p->spp_n > 0 ? p->spp_n : 1;
  double color[3] = {0.0, 0.0, 0.0};
  for (int si = 0; si < n; ++si) {
    const double xo = (si) / (double)n - 0.5 + 1.0 / (2.0 * n);
    for (int sj = 0; sj < n; ++sj) {
      const double yo = (sj) / (double)n - 0.5 + 1.0 / (2.0 * n);
      ray_t r;
      primary_ray(&p->camera, (double)x + xo, (double)y + yo, &r);
      double c[3];
      trace(C, p, &r, 0, mode, c, cnt);
      for (int k = 0; k < 3; ++k) color[k] += c[k];
    }
  }
  for (int k = 0; k < 3; ++k) {
    color[k] /= (double)(n * n);
    out[k] = std_min(color[k], 1.0);
  }
  cnt->pixels++;
}

static void add_counts(or_counts* dst, const or_counts* src) {
  dst->primary_rays += src->primary_rays; dst->shadow_rays += src->shadow_rays;
  dst->reflection_rays += src->reflection_rays; dst->node_visits += src->node_visits;
  dst->tri_tests += src->tri_tests; dst->closest_hits += src->closest_hits;
  dst->pixels += src->pixels; dst->box_tests += src->box_tests;
}

int or_render_pixels(or_ctx* C, const rt_render_params* p, int mode, int nthreads, const int* xy,
                     long long n_pixels, double* out, or_counts* counts) {
  if (!C || !p || p->n_lights < 0 || p->n_lights > (p->lights_ext ? RT_LIGHTS_LIMIT : RT_MAX_LIGHTS)) return -1;
  or_counts total;
  memset(&total, 0, sizeof total);
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#else
  nthreads = 1;
#endif
#pragma omp parallel num_threads(nthreads)
  {
    or_counts local;
    memset(&local, 0, sizeof local);
#pragma omp for schedule(dynamic, 16)
    for (long long i = 0; i < n_pixels; ++i) render_pixel(C, p, xy[2 * i], xy[2 * i + 1], mode, out + 3 * i, &local);
#pragma omp critical
    add_counts(&total, &local);
  }
  if (counts) *counts = total;
  return 0;
}

int or_render(or_ctx* C, const rt_render_params* p, int mode, int nthreads, double* out, or_counts* counts) {
  if (!C || !p) return -1;
  const int W = p->camera.width, H = p->camera.height;
  const int rb = p->row_begin < 0 ? 0 : p->row_begin;
  const int re = (p->row_end <= 0 || p->row_end > H) ? H : p->row_end;
  const int sh = p->stripe_height > 0 ? p->stripe_height : 1;
  const int sc = p->stripe_count > 0 ? p->stripe_count : 1;
  long long rows = 0;
  for (int y = rb; y < re; ++y) if ((y / sh) % sc == p->stripe_index) rows++;
  int* xy = (int*)malloc(sizeof(int) * 2 * (rows * W + 1));
  if (!xy) return -1;
  long long k = 0;
  for (int y = rb; y < re; ++y) {
    if ((y / sh) % sc != p->stripe_index) continue;
    for (int x = 0; x < W; ++x) { xy[2 * k] = x; xy[2 * k + 1] = y; ++k; }
  }
  const int rc = or_render_pixels(C, p, mode, nthreads, xy, k, out, counts);
  free(xy);
  return rc;
}

int or_closest_hit(or_ctx* C, const double o[3], const double d[3], int mode, double* t, int* tri_id,
                   double point[3], double normal[3]) {
  ray_t r;
  make_ray(o, d, &r);
  hit_t h;
  or_counts cnt;
  memset(&cnt, 0, sizeof cnt);
  if (!intersect_scene(C, &r, mode, &h, &cnt)) return 0;
  *t = h.t;
  *tri_id = h.tri_id;
  for (int k = 0; k < 3; ++k) { point[k] = h.p[k]; normal[k] = h.n[k]; }
  return 1;
}
