// host_scene.cpp — normals, SoA flattening, median-split BVH, camera and the
// C-ABI of librt_host.so (include/rt_host.h).
//
// Restated (not copied) from the reference host path:
//   Mesh::compute_normals        mymesh.cpp:103-163
//   Raytracer::build_Data        mytracer.cpp:166-296
//   BVH::initSoA + helpers       mybvh.cpp:375-539, median_inplace 346-362
// The tree, node numbering and the in-place permutation of the per-triangle
// arrays are reproduced exactly (tests/test_host_parity.py compares them with
// the oracle bit for bit).
#include "host_scene.hpp"

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <cstdlib>
#include <sched.h>

namespace rt {

namespace {
inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline double norm3(const double* a) { return std::sqrt(dot3(a, a)); }
inline void normalize3(double* v) {
  const double n = norm3(v);
  if (n > 0.0) { v[0] = v[0] / n; v[1] = v[1] / n; v[2] = v[2] / n; }
}
inline void cross3(const double* a, const double* b, double* r) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
}  // namespace

rt_material make_material(double ar, double ag, double ab, double dr, double dg, double db, double sr,
                          double sg, double sb, double shininess, double mirror, int shadowable) {
  rt_material m{};
  m.ambient[0] = ar; m.ambient[1] = ag; m.ambient[2] = ab;
  m.diffuse[0] = dr; m.diffuse[1] = dg; m.diffuse[2] = db;
  m.specular[0] = sr; m.specular[1] = sg; m.specular[2] = sb;
  m.shininess = shininess;
  m.mirror = mirror;
  m.shadowable = shadowable;
  return m;
}

// Angle-weighted vertex normals, mymesh.cpp:103-163: face normal
// normalize(cross(p1-p0, p2-p0)); each corner adds n / (|u||v| + u.v).
void HostMesh::compute_normals() {
  const double eps = 1e-12;
  const int nv = n_vertices(), nt = n_triangles();
  vertex_normals.assign(3 * (size_t)nv, 0.0);
  face_normals.assign(3 * (size_t)nt, 0.0);
  for (int t = 0; t < nt; ++t) {
    const double* p0 = &positions[3 * (size_t)tri_vertex[3 * t]];
    const double* p1 = &positions[3 * (size_t)tri_vertex[3 * t + 1]];
    const double* p2 = &positions[3 * (size_t)tri_vertex[3 * t + 2]];
    const double e1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
    const double e2[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
    double* n = &face_normals[3 * (size_t)t];
    cross3(e1, e2, n);
    normalize3(n);
  }
  for (int t = 0; t < nt; ++t) {
    const int i0 = tri_vertex[3 * t], i1 = tri_vertex[3 * t + 1], i2 = tri_vertex[3 * t + 2];
    const double* p0 = &positions[3 * (size_t)i0];
    const double* p1 = &positions[3 * (size_t)i1];
    const double* p2 = &positions[3 * (size_t)i2];
    const double a[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};   // v0
    const double b[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};   // v1
    const double c[3] = {p0[0] - p2[0], p0[1] - p2[1], p0[2] - p2[2]};   // v2
    const double na[3] = {-a[0], -a[1], -a[2]}, nb[3] = {-b[0], -b[1], -b[2]}, nc[3] = {-c[0], -c[1], -c[2]};
    const double la = norm3(a), lb = norm3(b), lc = norm3(c);
    const double w0 = la * lc + dot3(a, nc);
    const double w1 = lb * la + dot3(b, na);
    const double w2 = lc * lb + dot3(c, nb);
    const double* n = &face_normals[3 * (size_t)t];
    if (std::fabs(w0) > eps) for (int k = 0; k < 3; ++k) vertex_normals[3 * (size_t)i0 + k] += n[k] / w0;
    if (std::fabs(w1) > eps) for (int k = 0; k < 3; ++k) vertex_normals[3 * (size_t)i1 + k] += n[k] / w1;
    if (std::fabs(w2) > eps) for (int k = 0; k < 3; ++k) vertex_normals[3 * (size_t)i2 + k] += n[k] / w2;
  }
  for (int v = 0; v < nv; ++v) normalize3(&vertex_normals[3 * (size_t)v]);
}

long long HostScene::triangle_count() const {
  long long n = 0;
  for (const auto& m : meshes) n += m.n_triangles();
  return n;
}

void HostScene::refresh_raw() {
  raw_meshes.resize(meshes.size());
  for (size_t i = 0; i < meshes.size(); ++i) {
    const HostMesh& m = meshes[i];
    rt_mesh& r = raw_meshes[i];
    std::memset(&r, 0, sizeof r);
    r.n_vertices = m.n_vertices();
    r.positions = m.positions.data();
    r.n_triangles = m.n_triangles();
    r.tri_vertex = m.tri_vertex.data();
    r.n_uv = (int)m.u.size();
    r.u = m.u.data();
    r.v = m.v.data();
    r.tri_uv = m.tri_uv.empty() ? nullptr : m.tri_uv.data();
    r.draw_mode = m.draw_mode;
    r.material = m.material;
    r.texture.width = m.tex_w > 0 ? m.tex_w : 0;
    r.texture.height = m.tex_h > 0 ? m.tex_h : 0;
    r.texture.rgb = m.texels.empty() ? nullptr : m.texels.data();
  }
  std::memset(&raw, 0, sizeof raw);
  raw.camera = camera;
  for (int k = 0; k < 3; ++k) { raw.background[k] = background[k]; raw.ambience[k] = ambience[k]; }
  raw.max_depth = max_depth;
  raw.n_lights = (int)lights.size();
  raw.lights = lights.data();
  raw.n_meshes = (int)raw_meshes.size();
  raw.meshes = raw_meshes.data();
  raw.n_spheres = (int)spheres.size();
  raw.spheres = spheres.data();
  raw.n_planes = (int)planes.size();
  raw.planes = planes.data();
}

// Raytracer::build_Data, mytracer.cpp:166-296: concatenate every mesh into
// global arrays; vertex / uv indices are rebased (vbase, tbase; :246-251),
// per-mesh texture blocks are appended (:261-276), materials per mesh (:282-287).
void build_data(const HostScene& scene, SoA& s) {
  s = SoA();
  s.n_meshes = (int)scene.meshes.size();
  long long nv = 0, nt = 0, nuv = 0, ntex = 0;
  for (const auto& m : scene.meshes) {
    nv += m.n_vertices(); nt += m.n_triangles(); nuv += (long long)m.u.size();
    if (m.tex_w > 0) ntex += (long long)m.tex_w * m.tex_h;
  }
  if (nv > INT32_MAX || 3 * nt > INT32_MAX) throw std::runtime_error("scene too large for 32-bit indices");
  s.n_vertices = (int)nv;
  s.n_vertex_idx = (int)(3 * nt);
  s.n_tex_coords = (int)nuv;
  s.n_texels = ntex;
  s.vertex_mesh_id.resize(nv);
  s.vertex_pos.resize(3 * nv);
  s.vertex_normals.resize(3 * nv);
  s.face_normals.resize(3 * nt);
  s.vertex_idx.resize(3 * nt);
  s.texture_idx.resize(3 * nt);
  s.tex_u.resize(nuv);
  s.tex_v.resize(nuv);
  s.texels.resize(3 * ntex);
  const int M = s.n_meshes;
  s.first_vertex.resize(M); s.vertex_count.resize(M);
  s.first_vertex_idx.resize(M); s.vertex_idx_count.resize(M);
  s.first_tex_coord.resize(M); s.tex_coord_count.resize(M);
  s.mesh_tex_width.resize(M); s.mesh_tex_height.resize(M); s.mesh_tex_offset.resize(M);
  s.mesh_draw_mode.resize(M);
  s.mat_ambient.resize(3 * M); s.mat_diffuse.resize(3 * M); s.mat_specular.resize(3 * M);
  s.mat_shininess.resize(M); s.mat_mirror.resize(M); s.mat_shadowable.resize(M);

  long long vbase = 0, tbase = 0, ibase = 0, texoff = 0;
  for (int mi = 0; mi < M; ++mi) {
    const HostMesh& m = scene.meshes[mi];
    const int mv = m.n_vertices(), mt = m.n_triangles(), mu = (int)m.u.size();
    std::copy(m.positions.begin(), m.positions.end(), s.vertex_pos.begin() + 3 * vbase);
    std::copy(m.vertex_normals.begin(), m.vertex_normals.end(), s.vertex_normals.begin() + 3 * vbase);
    std::fill(s.vertex_mesh_id.begin() + vbase, s.vertex_mesh_id.begin() + vbase + mv, mi);
    s.first_vertex[mi] = (int)vbase; s.vertex_count[mi] = mv;
    std::copy(m.u.begin(), m.u.end(), s.tex_u.begin() + tbase);
    std::copy(m.v.begin(), m.v.end(), s.tex_v.begin() + tbase);
    s.first_tex_coord[mi] = (int)tbase; s.tex_coord_count[mi] = mu;
    for (int t = 0; t < mt; ++t) {
      for (int c = 0; c < 3; ++c) {
        s.vertex_idx[ibase + 3 * t + c] = (int)(vbase + m.tri_vertex[3 * t + c]);
        s.texture_idx[ibase + 3 * t + c] = m.tri_uv.empty() ? -1 : (int)(tbase + m.tri_uv[3 * t + c]);
        s.face_normals[ibase + 3 * t + c] = m.face_normals[3 * t + c];   // normals_[ibase/3 + t]
      }
    }
    s.first_vertex_idx[mi] = (int)ibase; s.vertex_idx_count[mi] = 3 * mt;
    if (m.tex_w > 0) {
      s.mesh_tex_width[mi] = m.tex_w; s.mesh_tex_height[mi] = m.tex_h; s.mesh_tex_offset[mi] = texoff;
      std::copy(m.texels.begin(), m.texels.end(), s.texels.begin() + 3 * texoff);
      texoff += (long long)m.tex_w * m.tex_h;
    } else {
      s.mesh_tex_width[mi] = -1; s.mesh_tex_height[mi] = -1; s.mesh_tex_offset[mi] = -1;
    }
    s.mesh_draw_mode[mi] = m.draw_mode;
    for (int k = 0; k < 3; ++k) {
      s.mat_ambient[3 * mi + k] = m.material.ambient[k];
      s.mat_diffuse[3 * mi + k] = m.material.diffuse[k];
      s.mat_specular[3 * mi + k] = m.material.specular[k];
    }
    s.mat_shininess[mi] = m.material.shininess;
    s.mat_mirror[mi] = m.material.mirror;
    s.mat_shadowable[mi] = m.material.shadowable;
    vbase += mv; ibase += 3 * mt; tbase += mu;
  }
}

// BVH::initSoA / subdivideSoA / inplace_partitionSoA / medianSoA,
// mybvh.cpp:375-539.  Root at depth 1 => the root splits on axis 1 (y).
// The recursion is replaced by a LIFO stack that visits nodes in the same
// order, so children get the same ids (nodesUsed_ at split time, :456-458).
// Triangle centroids ((v0+v1+v2)/3.0, :492/:535) are cached per slot and
// swapped with the slot's data, which leaves every value bit-identical.
// ---------------------------------------------------------------------------
// BVH::initSoA's median-split builder (mybvh.cpp:375-539), parallel.
// Subtrees own disjoint slot ranges, so they are built concurrently (one
// thread per subtree down to a fixed depth), each into its own node arena with
// local ids.  A final pass replays the reference's id allocation -- a node
// allocates ids for its two children when it splits, children are processed
// left first (LIFO, :456-468) -- so ids, bounds and the slot permutation are
// bit-identical to the sequential build (tests/test_host_parity.py).
namespace {

struct FragNode {
  double mn[3], mx[3];
  int first = 0, count = 0;   // count > 0: leaf
  int left = -1, right = -1;  // arena ids (internal)
  int depth = 0;              // reference depth (root = 1), for the axis and the max-depth stat
};

struct BuildCtx {
  SoA& s;
  std::vector<double>& cent;
  int par_levels;   // spawn a thread for the left subtree above this depth
};

void node_bounds(const SoA& s, FragNode& nd) {   // updateNodeBoundsSoA, mybvh.cpp:412-431
  double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (int i = nd.first; i < nd.first + nd.count; ++i)
    for (int c = 0; c < 3; ++c) {
      const double* p = &s.vertex_pos[3 * (size_t)s.vertex_idx[3 * (size_t)i + c]];
      for (int k = 0; k < 3; ++k) { mn[k] = std::fmin(mn[k], p[k]); mx[k] = std::fmax(mx[k], p[k]); }
    }
  for (int k = 0; k < 3; ++k) { nd.mn[k] = mn[k]; nd.mx[k] = mx[k]; }
}

// Splits arena[root] and its descendants (sequential within the subtree unless
// depth < par_levels, where the left child's subtree goes to a new thread).
void build_subtree(BuildCtx& cx, std::vector<FragNode>& arena, int root) {
  std::vector<double> axis_pts;
  std::vector<int> stack = {root};
  while (!stack.empty()) {
    const int node = stack.back();
    stack.pop_back();
    const int n = arena[node].count, f = arena[node].first, depth = arena[node].depth;
    if (n <= 2) continue;                                    // :441
    const int axis = depth % 3;                              // :444
    axis_pts.resize(n);
    for (int i = 0; i < n; ++i) axis_pts[i] = cx.cent[3 * (size_t)(f + i) + axis];
    const size_t mid = (size_t)n / 2;                        // median_inplace, :346-362
    double split;
    std::nth_element(axis_pts.begin(), axis_pts.begin() + mid, axis_pts.end());
    if (n % 2 == 1) {
      split = axis_pts[mid];
    } else {
      const double hi = axis_pts[mid];
      std::nth_element(axis_pts.begin(), axis_pts.begin() + (mid - 1), axis_pts.begin() + mid);
      split = 0.5 * (axis_pts[mid - 1] + hi);
    }
    int i = f, j = f + n - 1;                                // :481-513 (+ cached centroids)
    SoA& s = cx.s;
    while (i <= j) {
      if (cx.cent[3 * (size_t)i + axis] < split) {
        ++i;
      } else {
        for (int k = 0; k < 3; ++k) {
          std::swap(s.face_normals[3 * (size_t)i + k], s.face_normals[3 * (size_t)j + k]);
          std::swap(s.vertex_idx[3 * (size_t)i + k], s.vertex_idx[3 * (size_t)j + k]);
          std::swap(s.texture_idx[3 * (size_t)i + k], s.texture_idx[3 * (size_t)j + k]);
          std::swap(cx.cent[3 * (size_t)i + k], cx.cent[3 * (size_t)j + k]);
        }
        --j;
      }
    }
    const int left_count = i - f;
    if (left_count == 0 || left_count == n) continue;        // :453
    FragNode l, r;
    l.first = f; l.count = left_count; l.depth = depth + 1;
    r.first = i; r.count = n - left_count; r.depth = depth + 1;
    node_bounds(s, l);
    node_bounds(s, r);
    const int li = (int)arena.size();
    arena.push_back(l);
    arena.push_back(r);
    arena[node].left = li;
    arena[node].right = li + 1;
    arena[node].count = 0;
    if (depth < cx.par_levels) {   // left subtree on a new thread, right one here; then graft
      std::vector<FragNode> sub = {arena[li]};
      sub[0].left = sub[0].right = -1;
      std::thread t([&cx, &sub]() { build_subtree(cx, sub, 0); });
      build_subtree(cx, arena, li + 1);
      t.join();
      const int off = (int)arena.size() - 1;   // sub[k] (k >= 1) -> arena[off + k]; sub[0] -> arena[li]
      auto remap = [&](int k) { return k <= 0 ? k : off + k; };
      arena[li] = sub[0];
      arena[li].left = remap(sub[0].left);
      arena[li].right = remap(sub[0].right);
      for (size_t k = 1; k < sub.size(); ++k) {
        FragNode nd = sub[k];
        nd.left = remap(nd.left);
        nd.right = remap(nd.right);
        arena.push_back(nd);
      }
      continue;
    }
    stack.push_back(li + 1);
    stack.push_back(li);
  }
}

// Builder threads: `requested` when > 0, else the CPUs this process may run on -- its affinity
// mask, capped by a cgroup v2 CPU quota (a GPU box's job may use only its share of the node).
// The library reads nothing from the environment (rt_host_prepare_ex).
int build_threads(int requested) {
  int t = requested;
  if (t <= 0) {
    cpu_set_t set;
    t = sched_getaffinity(0, sizeof set, &set) == 0 ? CPU_COUNT(&set) : (int)std::thread::hardware_concurrency();
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long per = 0;
      if (std::fscanf(f, "%31s %lld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
        const long long quota = std::atoll(q);
        if (quota > 0) t = (int)std::min<long long>(t, std::max(1LL, quota / per));
      }
      std::fclose(f);
    }
  }
  return std::max(1, std::min(t, 64));
}

}  // namespace

void build_bvh_soa(SoA& s, BvhSoA& b, int requested_threads) {
  b = BvhSoA();
  const long long N = s.n_vertex_idx / 3;
  if (N <= 0) return;
  std::vector<double> cent(3 * (size_t)N);
  for (long long i = 0; i < N; ++i) {
    const double* p0 = &s.vertex_pos[3 * (size_t)s.vertex_idx[3 * i]];
    const double* p1 = &s.vertex_pos[3 * (size_t)s.vertex_idx[3 * i + 1]];
    const double* p2 = &s.vertex_pos[3 * (size_t)s.vertex_idx[3 * i + 2]];
    for (int k = 0; k < 3; ++k) cent[3 * i + k] = (p0[k] + p1[k] + p2[k]) / 3.0;
  }
  // threads = 2^par_levels; small builds stay sequential
  int levels = 0;
  const int threads = build_threads(requested_threads);
  while ((1 << (levels + 1)) <= threads) ++levels;
  if (N < 200000) levels = 0;
  BuildCtx cx{s, cent, levels + 1};   // root depth is 1: split in parallel while depth <= levels
  std::vector<FragNode> arena(1);
  arena[0].first = 0;
  arena[0].count = (int)N;
  arena[0].depth = 1;
  node_bounds(s, arena[0]);
  build_subtree(cx, arena, 0);

  // replay the reference's id allocation (children numbered at split time, left first)
  const size_t cap = 2 * (size_t)N - 1;
  b.bb_min.assign(3 * cap, 0.0);
  b.bb_max.assign(3 * cap, 0.0);
  b.left_child.assign(cap, 0);
  b.first_tri.assign(cap, 0);
  b.tri_count.assign(cap, 0);
  int nodes_used = 1, maxd = 0;
  std::vector<std::pair<int, int>> st = {{0, 0}};   // (arena id, reference id)
  while (!st.empty()) {
    const auto [a, id] = st.back();
    st.pop_back();
    const FragNode& nd = arena[a];
    for (int k = 0; k < 3; ++k) { b.bb_min[3 * (size_t)id + k] = nd.mn[k]; b.bb_max[3 * (size_t)id + k] = nd.mx[k]; }
    maxd = std::max(maxd, nd.depth - 1);
    if (nd.left < 0) {
      b.first_tri[id] = nd.first;
      b.tri_count[id] = nd.count;
      b.left_child[id] = 0;
      continue;
    }
    const int l = nodes_used, r = l + 1;
    nodes_used += 2;
    b.left_child[id] = l;
    b.first_tri[id] = nd.first;   // the reference keeps firstTri of a split node (:457-464)
    b.tri_count[id] = 0;
    st.emplace_back(nd.right, r);
    st.emplace_back(nd.left, l);
  }
  b.n_nodes = nodes_used;
  b.depth = maxd;
}

// Course Camera (absent from the reference): image plane through
// `center`, height 2*dist*tan(fovy/2), x_dir / y_dir one pixel wide, pixel
// (0,0) at lower_left.
void derive_camera(const rt_camera_def& def, int width, int height, rt_camera& out) {
  if (width <= 0) width = def.width;
  if (height <= 0) height = def.height;
  double view[3] = {def.center[0] - def.eye[0], def.center[1] - def.eye[1], def.center[2] - def.eye[2]};
  const double dist = norm3(view);
  normalize3(view);
  const double image_height = 2.0 * dist * std::tan(0.5 * def.fovy / 180.0 * M_PI);
  const double image_width = (double)width / (double)height * image_height;
  double xd[3], yd[3];
  cross3(view, def.up, xd);
  normalize3(xd);
  for (int k = 0; k < 3; ++k) xd[k] = xd[k] * image_width / (double)width;
  cross3(xd, view, yd);
  normalize3(yd);
  for (int k = 0; k < 3; ++k) yd[k] = yd[k] * image_height / (double)height;
  for (int k = 0; k < 3; ++k) {
    out.eye[k] = def.eye[k];
    out.x_dir[k] = xd[k];
    out.y_dir[k] = yd[k];
    out.lower_left[k] = def.center[k] - 0.5 * (double)width * xd[k] - 0.5 * (double)height * yd[k];
  }
  out.width = width;
  out.height = height;
}

void HostScene::prepare(int threads) {
  if (prepared) return;
  for (auto& m : meshes) {
    if (m.draw_mode != RT_DRAW_FLAT && m.draw_mode != RT_DRAW_PHONG)
      throw std::runtime_error("invalid draw mode in mesh " + m.name);
    m.compute_normals();
  }
  build_data(*this, soa);
  build_bvh_soa(soa, bvh, threads);
  rt_scene_soa& v = soa_view;
  std::memset(&v, 0, sizeof v);
  v.n_meshes = soa.n_meshes;
  v.n_vertices = soa.n_vertices;
  v.n_vertex_idx = soa.n_vertex_idx;
  v.n_tex_coords = soa.n_tex_coords;
  v.n_texels = soa.n_texels;
  v.vertex_mesh_id = soa.vertex_mesh_id.data();
  v.vertex_pos = soa.vertex_pos.data();
  v.vertex_normals = soa.vertex_normals.data();
  v.face_normals = soa.face_normals.data();
  v.vertex_idx = soa.vertex_idx.data();
  v.texture_idx = soa.texture_idx.data();
  v.tex_u = soa.tex_u.data();
  v.tex_v = soa.tex_v.data();
  v.texels = soa.texels.data();
  v.mesh_tex_width = soa.mesh_tex_width.data();
  v.mesh_tex_height = soa.mesh_tex_height.data();
  v.mesh_tex_offset = soa.mesh_tex_offset.data();
  v.mesh_draw_mode = soa.mesh_draw_mode.data();
  v.mat_ambient = soa.mat_ambient.data();
  v.mat_diffuse = soa.mat_diffuse.data();
  v.mat_specular = soa.mat_specular.data();
  v.mat_shininess = soa.mat_shininess.data();
  v.mat_mirror = soa.mat_mirror.data();
  v.mat_shadowable = soa.mat_shadowable.data();
  rt_bvh_soa& bv = bvh_view;
  bv.n_nodes = bvh.n_nodes;
  bv.bb_min = bvh.bb_min.data();
  bv.bb_max = bvh.bb_max.data();
  bv.left_child = bvh.left_child.data();
  bv.first_tri = bvh.first_tri.data();
  bv.tri_count = bvh.tri_count.data();
  prepared = true;
}

}  // namespace rt

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
struct rt_host_scene {
  rt::HostScene scene;
};

namespace {
thread_local std::string g_host_error;
int host_fail(const std::string& msg) {
  g_host_error = msg;
  return RT_ERR_INVALID;
}
}  // namespace

extern "C" {

const char* rt_host_last_error(void) { return g_host_error.c_str(); }

int rt_host_load(const char* sce_path, rt_host_scene** out) {
  if (!sce_path || !out) return host_fail("rt_host_load: null argument");
  try {
    auto* h = new rt_host_scene();
    rt::load_sce(sce_path, h->scene);
    h->scene.refresh_raw();
    *out = h;
    return RT_OK;
  } catch (const std::exception& e) {
    return host_fail(std::string("rt_host_load: ") + e.what());
  }
}

int rt_host_generate(const char* kind, const rt_gen_params* params, rt_host_scene** out) {
  if (!kind || !out) return host_fail("rt_host_generate: null argument");
  rt_gen_params p{};
  p.max_depth = -1;
  if (params) p = *params;
  try {
    auto* h = new rt_host_scene();
    rt::generate_scene(kind, p, h->scene);
    h->scene.refresh_raw();
    *out = h;
    return RT_OK;
  } catch (const std::exception& e) {
    return host_fail(std::string("rt_host_generate: ") + e.what());
  }
}

const rt_raw_scene* rt_host_raw(const rt_host_scene* s) { return s ? &s->scene.raw : nullptr; }

int rt_host_prepare(rt_host_scene* s, double* seconds) { return rt_host_prepare_ex(s, 0, seconds); }

int rt_host_prepare_ex(rt_host_scene* s, int build_threads, double* seconds) {
  if (!s) return host_fail("rt_host_prepare: null scene");
  if (build_threads < 0) return host_fail("rt_host_prepare_ex: build_threads must be >= 0");
  try {
    const auto t0 = std::chrono::steady_clock::now();
    s->scene.prepare(build_threads);
    const auto t1 = std::chrono::steady_clock::now();
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    return RT_OK;
  } catch (const std::exception& e) {
    return host_fail(std::string("rt_host_prepare: ") + e.what());
  }
}

const rt_scene_soa* rt_host_soa(const rt_host_scene* s) {
  return (s && s->scene.prepared) ? &s->scene.soa_view : nullptr;
}
const rt_bvh_soa* rt_host_bvh(const rt_host_scene* s) {
  return (s && s->scene.prepared) ? &s->scene.bvh_view : nullptr;
}

int rt_host_camera(const rt_host_scene* s, int width, int height, rt_camera* out) {
  if (!s || !out) return host_fail("rt_host_camera: null argument");
  rt::derive_camera(s->scene.camera, width, height, *out);
  return RT_OK;
}

int rt_host_render_params(const rt_host_scene* s, int width, int height, int spp_n, rt_render_params* out) {
  if (!s || !out) return host_fail("rt_host_render_params: null argument");
  const rt::HostScene& sc = s->scene;
  if ((long long)sc.lights.size() > RT_LIGHTS_LIMIT) return host_fail("rt_host_render_params: too many lights");
  std::memset(out, 0, sizeof *out);
  rt::derive_camera(sc.camera, width, height, out->camera);
  out->n_lights = (int)sc.lights.size();
  for (int i = 0; i < std::min(out->n_lights, RT_MAX_LIGHTS); ++i) out->lights[i] = sc.lights[i];
  // more than the inline table holds: point at the scene's own list (valid while s lives)
  out->lights_ext = out->n_lights > RT_MAX_LIGHTS ? sc.lights.data() : nullptr;
  for (int k = 0; k < 3; ++k) { out->background[k] = sc.background[k]; out->ambience[k] = sc.ambience[k]; }
  out->max_depth = sc.max_depth;
  out->spp_n = spp_n > 0 ? spp_n : 1;
  out->row_begin = 0;
  out->row_end = out->camera.height;
  out->stripe_height = 16;
  out->stripe_count = 1;
  out->stripe_index = 0;
  out->out_format = RT_OUT_RGB_F32;
  out->flags = 0;
  return RT_OK;
}

int rt_host_save(const rt_host_scene* s, const char* sce_path) {
  if (!s || !sce_path) return host_fail("rt_host_save: null argument");
  try {
    rt::save_sce(s->scene, sce_path);
    return RT_OK;
  } catch (const std::exception& e) {
    return host_fail(std::string("rt_host_save: ") + e.what());
  }
}

int rt_write_ppm(const char* path, const float* rgb, int width, int height) {
  if (!path || !rgb || width <= 0 || height <= 0) return host_fail("rt_write_ppm: bad argument");
  FILE* f = std::fopen(path, "wb");
  if (!f) return host_fail(std::string("rt_write_ppm: cannot open ") + path);
  std::fprintf(f, "P6\n%d %d\n255\n", width, height);
  std::vector<unsigned char> line(3 * (size_t)width);
  for (int y = height - 1; y >= 0; --y) {
    for (int x = 0; x < width; ++x) {
      for (int c = 0; c < 3; ++c) {
        float v = rgb[3 * ((size_t)y * width + x) + c];
        v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
        line[3 * (size_t)x + c] = (unsigned char)std::lround(v * 255.0f);
      }
    }
    std::fwrite(line.data(), 1, line.size(), f);
  }
  std::fclose(f);
  return RT_OK;
}

long long rt_host_triangle_count(const rt_host_scene* s) { return s ? s->scene.triangle_count() : 0; }

int rt_host_bvh_depth(const rt_host_scene* s) {
  return (s && s->scene.prepared) ? s->scene.bvh.depth : -1;
}

void rt_host_free(rt_host_scene* s) { delete s; }

}  // extern "C"
