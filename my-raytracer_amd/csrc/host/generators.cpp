// generators.cpp — procedural stand-in scenes.
//
// The reference's scene files (Office, spheres, ...) are not in the reference
// repository (only their renders, outputs/*.png), so the benchmark configs
// (BASELINE.json) run on labelled, fixed-seed stand-ins:
//   "office"      office_proxy: a room modelled on outputs/o_08_office.png —
//                 window wall with mirroring panes, stadium table, 4 chairs,
//                 cabinet, plant; FLAT + PHONG meshes, 2 lights, depth 5,
//                 1920x1080 (~70k triangles at detail 1)
//   "spheres"     spheres_proxy: 4 spheres + floor plane, 2 lights, depth 3,
//                 640x480 (config 1, CPU path only: analytic primitives)
//   "random_tris" N random triangles in [-1,1]^3, edge e = 3 N^(-1/3),
//                 1 FLAT mesh, 1 light, depth 0, camera (0,0,4) -> origin
//   "cornell"     small parity room: FLAT, PHONG, texture, mirror,
//                 non-shadowable material, 2 lights, depth 3
// All randomness is a fixed-seed splitmix64 stream (platform independent).
#include <cmath>
#include <map>
#include <stdexcept>
#include <tuple>

#include "host_scene.hpp"

namespace rt {

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }   // [0,1)
  double uniform(double a, double b) { return a + (b - a) * uniform(); }
};

struct Builder {
  HostMesh m;
  Builder(const std::string& name, int mode, const rt_material& mat) {
    m.name = name;
    m.draw_mode = mode;
    m.material = mat;
  }
  int vertex(double x, double y, double z) {
    m.positions.push_back(x); m.positions.push_back(y); m.positions.push_back(z);
    return m.n_vertices() - 1;
  }
  void tri(int a, int b, int c) { m.tri_vertex.push_back(a); m.tri_vertex.push_back(b); m.tri_vertex.push_back(c); }
  // Grid on the parallelogram o + s*a + t*b, s,t in [0,1]; normal along a x b.
  void grid(const double o[3], const double a[3], const double b[3], int na, int nb) {
    const int base = m.n_vertices();
    for (int j = 0; j <= nb; ++j)
      for (int i = 0; i <= na; ++i) {
        const double s = (double)i / na, t = (double)j / nb;
        vertex(o[0] + s * a[0] + t * b[0], o[1] + s * a[1] + t * b[1], o[2] + s * a[2] + t * b[2]);
      }
    for (int j = 0; j < nb; ++j)
      for (int i = 0; i < na; ++i) {
        const int v00 = base + j * (na + 1) + i, v10 = v00 + 1, v01 = v00 + na + 1, v11 = v01 + 1;
        tri(v00, v10, v11);
        tri(v00, v11, v01);
      }
  }
  // Axis-aligned box, outward normals, n x n quads per face.
  void box(double x0, double y0, double z0, double x1, double y1, double z1, int n) {
    const double dx = x1 - x0, dy = y1 - y0, dz = z1 - z0;
    { const double o[3] = {x0, y0, z1}, a[3] = {dx, 0, 0}, b[3] = {0, dy, 0}; grid(o, a, b, n, n); }      // +z
    { const double o[3] = {x1, y0, z0}, a[3] = {-dx, 0, 0}, b[3] = {0, dy, 0}; grid(o, a, b, n, n); }     // -z
    { const double o[3] = {x1, y0, z1}, a[3] = {0, 0, -dz}, b[3] = {0, dy, 0}; grid(o, a, b, n, n); }     // +x
    { const double o[3] = {x0, y0, z0}, a[3] = {0, 0, dz}, b[3] = {0, dy, 0}; grid(o, a, b, n, n); }      // -x
    { const double o[3] = {x0, y1, z1}, a[3] = {dx, 0, 0}, b[3] = {0, 0, -dz}; grid(o, a, b, n, n); }     // +y
    { const double o[3] = {x0, y0, z0}, a[3] = {dx, 0, 0}, b[3] = {0, 0, dz}; grid(o, a, b, n, n); }      // -y
  }
  // Rounded box (superellipsoid-like, shared vertices => smooth PHONG normals).
  void rounded_box(double cx, double cy, double cz, double hx, double hy, double hz, int n, double power) {
    std::map<std::tuple<int, int, int>, int> ids;
    auto vid = [&](int i, int j, int k) {
      auto key = std::make_tuple(i, j, k);
      auto it = ids.find(key);
      if (it != ids.end()) return it->second;
      double p[3] = {2.0 * i / n - 1.0, 2.0 * j / n - 1.0, 2.0 * k / n - 1.0};
      const double ln = std::pow(std::pow(std::fabs(p[0]), power) + std::pow(std::fabs(p[1]), power) +
                                     std::pow(std::fabs(p[2]), power), 1.0 / power);
      for (double& c : p) c /= ln;
      const int id = vertex(cx + hx * p[0], cy + hy * p[1], cz + hz * p[2]);
      ids[key] = id;
      return id;
    };
    // 6 faces of the lattice cube [0,n]^3; (u,v) axes chosen for outward winding
    for (int face = 0; face < 6; ++face) {
      for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) {
          int q[4][3];
          const int us[4] = {a, a + 1, a + 1, a}, vs[4] = {b, b, b + 1, b + 1};
          for (int c = 0; c < 4; ++c) {
            const int u = us[c], v = vs[c];
            switch (face) {
              case 0: q[c][0] = n; q[c][1] = v; q[c][2] = n - u; break;   // +x
              case 1: q[c][0] = 0; q[c][1] = v; q[c][2] = u; break;       // -x
              case 2: q[c][0] = u; q[c][1] = n; q[c][2] = n - v; break;   // +y
              case 3: q[c][0] = u; q[c][1] = 0; q[c][2] = v; break;       // -y
              case 4: q[c][0] = u; q[c][1] = v; q[c][2] = n; break;       // +z
              default: q[c][0] = n - u; q[c][1] = v; q[c][2] = 0; break;  // -z
            }
          }
          const int i0 = vid(q[0][0], q[0][1], q[0][2]), i1 = vid(q[1][0], q[1][1], q[1][2]);
          const int i2 = vid(q[2][0], q[2][1], q[2][2]), i3 = vid(q[3][0], q[3][1], q[3][2]);
          tri(i0, i1, i2);
          tri(i0, i2, i3);
        }
    }
  }
  // Vertical cylinder (axis y), side with shared ring vertices, optional caps.
  void cylinder(double cx, double cz, double y0, double y1, double r, int seg, bool caps) {
    const int base = m.n_vertices();
    for (int i = 0; i < seg; ++i) {
      const double a = 2.0 * M_PI * i / seg;
      vertex(cx + r * std::cos(a), y0, cz + r * std::sin(a));
      vertex(cx + r * std::cos(a), y1, cz + r * std::sin(a));
    }
    for (int i = 0; i < seg; ++i) {
      const int j = (i + 1) % seg;
      const int b0 = base + 2 * i, t0 = b0 + 1, b1 = base + 2 * j, t1 = b1 + 1;
      tri(b0, t0, t1);
      tri(b0, t1, b1);
    }
    if (caps) {
      const int ct = vertex(cx, y1, cz), cb = vertex(cx, y0, cz);
      const int rt = m.n_vertices();
      for (int i = 0; i < seg; ++i) {
        const double a = 2.0 * M_PI * i / seg;
        vertex(cx + r * std::cos(a), y1, cz + r * std::sin(a));
        vertex(cx + r * std::cos(a), y0, cz + r * std::sin(a));
      }
      for (int i = 0; i < seg; ++i) {
        const int j = (i + 1) % seg;
        tri(ct, rt + 2 * j, rt + 2 * i);
        tri(cb, rt + 2 * i + 1, rt + 2 * j + 1);
      }
    }
  }
  // UV sphere.
  void sphere(double cx, double cy, double cz, double r, int nu, int nv) {
    const int base = m.n_vertices();
    for (int j = 0; j <= nv; ++j) {
      const double th = M_PI * j / nv;
      for (int i = 0; i < nu; ++i) {
        const double ph = 2.0 * M_PI * i / nu;
        vertex(cx + r * std::sin(th) * std::cos(ph), cy + r * std::cos(th), cz + r * std::sin(th) * std::sin(ph));
      }
    }
    for (int j = 0; j < nv; ++j)
      for (int i = 0; i < nu; ++i) {
        const int i1 = (i + 1) % nu;
        const int a = base + j * nu + i, b = base + j * nu + i1, c = base + (j + 1) * nu + i1, d = base + (j + 1) * nu + i;
        if (j != 0) tri(a, c, b);
        if (j != nv - 1) tri(a, d, c);
      }
  }
  // Prism over a star-shaped outline (x,z) between y0 and y1.
  void extrude(const std::vector<std::pair<double, double>>& outline, double y0, double y1) {
    const int n = (int)outline.size();
    double mx = 0, mz = 0;
    for (auto& p : outline) { mx += p.first; mz += p.second; }
    mx /= n; mz /= n;
    const int ct = vertex(mx, y1, mz), cb = vertex(mx, y0, mz);
    const int top = m.n_vertices();
    for (auto& p : outline) vertex(p.first, y1, p.second);
    const int bot = m.n_vertices();
    for (auto& p : outline) vertex(p.first, y0, p.second);
    const int st = m.n_vertices();
    for (auto& p : outline) { vertex(p.first, y1, p.second); vertex(p.first, y0, p.second); }
    for (int i = 0; i < n; ++i) {
      const int j = (i + 1) % n;
      tri(ct, top + j, top + i);
      tri(cb, bot + i, bot + j);
      tri(st + 2 * i, st + 2 * j, st + 2 * j + 1);
      tri(st + 2 * i, st + 2 * j + 1, st + 2 * i + 1);
    }
  }
};

void set3(double* d, double a, double b, double c) { d[0] = a; d[1] = b; d[2] = c; }

rt_light light(double x, double y, double z, double r, double g, double b) {
  rt_light l{};
  set3(l.position, x, y, z);
  set3(l.color, r, g, b);
  return l;
}

int scaled(int base, int detail) { return std::max(1, base * detail); }

void gen_office(const rt_gen_params& p, HostScene& sc) {
  const int det = p.detail > 0 ? p.detail : 1;
  const double X0 = -2.6, X1 = 2.4, Y1 = 2.9, Z0 = -3.1, Z1 = 2.9;
  sc.camera = rt_camera_def{};
  set3(sc.camera.eye, 0.35, 1.55, 2.6);
  set3(sc.camera.center, -0.15, 1.05, -1.2);
  set3(sc.camera.up, 0.0, 1.0, 0.0);
  sc.camera.fovy = 52.0;
  sc.camera.width = 1920;
  sc.camera.height = 1080;
  sc.max_depth = 5;
  set3(sc.background, 0.02, 0.02, 0.03);
  set3(sc.ambience, 0.25, 0.25, 0.25);
  sc.lights.push_back(light(-0.8, 2.7, 0.55, 0.55, 0.55, 0.55));
  sc.lights.push_back(light(1.15, 2.62, -1.3, 0.5, 0.5, 0.48));

  {  // floor, dark red carpet
    Builder b("floor", RT_DRAW_FLAT, make_material(0.3, 0.05, 0.06, 0.38, 0.06, 0.08, 0.05, 0.05, 0.05, 10.0, 0.0));
    const double o[3] = {X0, 0.0, Z1}, a[3] = {X1 - X0, 0, 0}, c[3] = {0, 0, Z0 - Z1};
    b.grid(o, a, c, 1, 1);
    sc.meshes.push_back(std::move(b.m));
  }
  {  // ceiling + walls, white
    Builder b("walls", RT_DRAW_FLAT, make_material(0.8, 0.8, 0.8, 0.85, 0.85, 0.82, 0.05, 0.05, 0.05, 10.0, 0.0));
    { const double o[3] = {X0, Y1, Z0}, a[3] = {X1 - X0, 0, 0}, c[3] = {0, 0, Z1 - Z0}; b.grid(o, a, c, 1, 1); }
    { const double o[3] = {X0, 0, Z1}, a[3] = {0, 0, Z0 - Z1}, c[3] = {0, Y1, 0}; b.grid(o, a, c, 1, 1); }
    { const double o[3] = {X1, 0, Z0}, a[3] = {0, 0, Z1 - Z0}, c[3] = {0, Y1, 0}; b.grid(o, a, c, 1, 1); }
    { const double o[3] = {X1, 0, Z1}, a[3] = {X0 - X1, 0, 0}, c[3] = {0, Y1, 0}; b.grid(o, a, c, 1, 1); }
    sc.meshes.push_back(std::move(b.m));
  }
  {  // window wall frame, dark grey
    Builder b("window_frame", RT_DRAW_FLAT, make_material(0.12, 0.12, 0.13, 0.2, 0.2, 0.22, 0.2, 0.2, 0.2, 30.0, 0.0));
    const double zb = Z0, zf = Z0 + 0.12;
    const int n = 1;
    b.box(X0, 0.0, zb, X1, 0.62, zf, n);          // parapet
    b.box(X0, 2.55, zb, X1, Y1, zf, n);           // lintel
    b.box(X0, 0.62, zb, -2.3, 2.55, zf, n);       // left jamb
    b.box(2.1, 0.62, zb, X1, 2.55, zf, n);        // right jamb
    b.box(-0.17, 0.62, zb, -0.03, 2.55, zf, n);   // centre mullion
    b.box(-2.3, 1.86, zb, 2.1, 1.98, zf, n);      // transom
    sc.meshes.push_back(std::move(b.m));
  }
  {  // glass panes: mirrors (the office render shows the room reflected)
    Builder b("glass", RT_DRAW_FLAT, make_material(0.02, 0.02, 0.03, 0.1, 0.12, 0.14, 0.6, 0.6, 0.6, 80.0, 0.55));
    const double z = Z0 + 0.06;
    const int n = 1;
    const double panes[4][4] = {{-2.3, 0.62, -0.17, 1.86}, {-0.03, 0.62, 2.1, 1.86},
                                {-2.3, 1.98, -0.17, 2.55}, {-0.03, 1.98, 2.1, 2.55}};
    for (const auto& q : panes) {
      const double o[3] = {q[0], q[1], z}, a[3] = {q[2] - q[0], 0, 0}, c[3] = {0, q[3] - q[1], 0};
      b.grid(o, a, c, n, n);
    }
    sc.meshes.push_back(std::move(b.m));
  }
  {  // cabinet, pale yellow
    Builder b("cabinet", RT_DRAW_FLAT, make_material(0.35, 0.34, 0.18, 0.78, 0.76, 0.42, 0.2, 0.2, 0.2, 20.0, 0.0));
    const int n = 1;
    b.box(1.62, 0.0, -2.05, X1 - 0.01, 2.2, 0.25, n);
    for (int r = 0; r < 2; ++r)
      for (int c = 0; c < 2; ++c) {
        const double y0 = 0.05 + r * 1.08, z0 = -2.0 + c * 1.12;
        b.box(1.58, y0, z0, 1.62, y0 + 1.03, z0 + 1.08, n);
      }
    sc.meshes.push_back(std::move(b.m));
  }
  {  // cabinet handles, black PHONG
    Builder b("handles", RT_DRAW_PHONG, make_material(0.02, 0.02, 0.02, 0.05, 0.05, 0.05, 0.6, 0.6, 0.6, 60.0, 0.0));
    for (int r = 0; r < 2; ++r)
      for (int c = 0; c < 4; ++c) {
        const double y = 0.9 + r * 1.08, z = -1.95 + c * 0.555 + (c % 2 ? -0.04 : 0.04);
        b.cylinder(1.55, z, y, y + 0.16, 0.012, scaled(16, det), true);
      }
    sc.meshes.push_back(std::move(b.m));
  }
  {  // stadium table top, PHONG
    Builder b("table_top", RT_DRAW_PHONG, make_material(0.35, 0.34, 0.15, 0.85, 0.82, 0.42, 0.35, 0.35, 0.3, 40.0, 0.0));
    std::vector<std::pair<double, double>> outline;
    const int seg = scaled(96, det);
    const double cx = -0.2, cz = -0.7, half = 0.85, r = 0.48, ang = 0.32;
    for (int i = 0; i < seg; ++i) {   // right half-disc then left half-disc
      const double a = -M_PI / 2 + M_PI * i / (seg - 1);
      outline.emplace_back(half + r * std::cos(a), r * std::sin(a));
    }
    for (int i = 0; i < seg; ++i) {
      const double a = M_PI / 2 + M_PI * i / (seg - 1);
      outline.emplace_back(-half + 0.7 * r * std::cos(a), 0.7 * r * std::sin(a));
    }
    for (auto& q : outline) {   // rotate and place
      const double x = q.first, z = q.second;
      q.first = cx + x * std::cos(ang) - z * std::sin(ang);
      q.second = cz + x * std::sin(ang) + z * std::cos(ang);
    }
    b.extrude(outline, 0.72, 0.76);
    sc.meshes.push_back(std::move(b.m));
  }
  {  // table pedestals, PHONG grey
    Builder b("table_legs", RT_DRAW_PHONG, make_material(0.2, 0.2, 0.2, 0.45, 0.45, 0.42, 0.4, 0.4, 0.4, 50.0, 0.0));
    b.cylinder(0.35, -0.45, 0.0, 0.72, 0.1, scaled(48, det), true);
    b.cylinder(-0.85, -0.98, 0.0, 0.72, 0.08, scaled(48, det), true);
    b.cylinder(0.35, -0.45, 0.0, 0.03, 0.32, scaled(48, det), true);
    b.cylinder(-0.85, -0.98, 0.0, 0.03, 0.28, scaled(48, det), true);
    sc.meshes.push_back(std::move(b.m));
  }
  {  // 4 chairs, blue PHONG cushions + dark metal frames
    Builder cush("chair_cushions", RT_DRAW_PHONG, make_material(0.05, 0.05, 0.3, 0.12, 0.12, 0.75, 0.3, 0.3, 0.4, 25.0, 0.0));
    Builder metal("chair_frames", RT_DRAW_PHONG, make_material(0.05, 0.05, 0.05, 0.15, 0.15, 0.16, 0.7, 0.7, 0.7, 80.0, 0.0));
    const double chairs[4][3] = {{-1.55, 0.45, 0.12}, {-0.85, 0.55, 0.0}, {0.95, -1.45, 3.3}, {-1.7, -1.2, 1.2}};
    const int n = scaled(20, det);
    for (const auto& c : chairs) {
      const double x = c[0], z = c[1], ang = c[2];
      const double bx = x - 0.26 * std::sin(ang), bz = z + 0.26 * std::cos(ang);
      cush.rounded_box(x, 0.48, z, 0.25, 0.055, 0.25, n, 6.0);
      cush.rounded_box(bx, 0.86, bz, 0.24 * std::fabs(std::cos(ang)) + 0.05 * std::fabs(std::sin(ang)), 0.3,
                       0.05 * std::fabs(std::cos(ang)) + 0.24 * std::fabs(std::sin(ang)), n, 6.0);
      metal.cylinder(x, z, 0.08, 0.43, 0.025, scaled(24, det), true);
      for (int k = 0; k < 5; ++k) {
        const double a = ang + 2.0 * M_PI * k / 5;
        const double ex = x + 0.28 * std::cos(a), ez = z + 0.28 * std::sin(a);
        metal.cylinder(0.5 * (x + ex), 0.5 * (z + ez), 0.06, 0.09, 0.03, scaled(12, det), true);
        metal.sphere(ex, 0.035, ez, 0.035, scaled(16, det), scaled(8, det));
      }
    }
    sc.meshes.push_back(std::move(cush.m));
    sc.meshes.push_back(std::move(metal.m));
  }
  {  // plant: pot + foliage ball + lamp globe
    Builder pot("pot", RT_DRAW_PHONG, make_material(0.25, 0.12, 0.05, 0.55, 0.3, 0.12, 0.2, 0.2, 0.2, 20.0, 0.0));
    pot.cylinder(-2.1, 1.9, 0.0, 0.45, 0.2, scaled(64, det), true);
    sc.meshes.push_back(std::move(pot.m));
    Builder leaf("foliage", RT_DRAW_PHONG, make_material(0.05, 0.2, 0.05, 0.15, 0.55, 0.15, 0.1, 0.2, 0.1, 15.0, 0.0));
    leaf.sphere(-2.1, 0.85, 1.9, 0.42, scaled(64, det), scaled(32, det));
    sc.meshes.push_back(std::move(leaf.m));
    Builder globe("lamp_globe", RT_DRAW_PHONG, make_material(0.4, 0.4, 0.38, 0.9, 0.9, 0.85, 0.9, 0.9, 0.9, 120.0, 0.25, 0));
    globe.sphere(0.2, 2.35, -0.6, 0.22, scaled(96, det), scaled(48, det));
    sc.meshes.push_back(std::move(globe.m));
  }
}

void gen_spheres(const rt_gen_params&, HostScene& sc) {
  sc.camera = rt_camera_def{};
  set3(sc.camera.eye, 0.05, 1.35, 6.2);
  set3(sc.camera.center, 0.0, 0.65, 0.0);
  set3(sc.camera.up, 0.0, 1.0, 0.0);
  sc.camera.fovy = 45.0;
  sc.camera.width = 640;
  sc.camera.height = 480;
  sc.max_depth = 3;
  set3(sc.background, 0.0, 0.0, 0.0);
  set3(sc.ambience, 0.2, 0.2, 0.2);
  sc.lights.push_back(light(-4.0, 5.0, 4.5, 0.6, 0.6, 0.6));
  sc.lights.push_back(light(3.5, 4.0, 3.0, 0.4, 0.4, 0.45));
  const double spheres[4][8] = {
      {-1.6, 0.7, -0.3, 0.7, 0.9, 0.15, 0.1, 0.0},
      {0.05, 0.8, -1.2, 0.8, 0.15, 0.8, 0.2, 0.0},
      {1.55, 0.6, 0.2, 0.6, 0.2, 0.3, 0.9, 0.0},
      {0.2, 0.45, 1.1, 0.45, 0.6, 0.6, 0.6, 0.6}};
  for (const auto& s : spheres) {
    rt_sphere sp{};
    set3(sp.center, s[0], s[1], s[2]);
    sp.radius = s[3];
    sp.material = make_material(s[4] * 0.3, s[5] * 0.3, s[6] * 0.3, s[4], s[5], s[6], 0.8, 0.8, 0.8, 60.0, s[7]);
    sc.spheres.push_back(sp);
  }
  rt_plane pl{};
  set3(pl.center, 0.0, 0.0, 0.0);
  set3(pl.normal, 0.0, 1.0, 0.0);
  pl.material = make_material(0.2, 0.2, 0.2, 0.5, 0.5, 0.5, 0.1, 0.1, 0.1, 10.0, 0.2);
  sc.planes.push_back(pl);
}

void gen_random_tris(const rt_gen_params& p, HostScene& sc) {
  const long long N = p.n_triangles > 0 ? p.n_triangles : 100000;
  if (N > 20000000) throw std::runtime_error("random_tris: n_triangles > 20M");
  Rng rng(p.seed ? p.seed : 1234);
  const double e = 3.0 * std::pow((double)N, -1.0 / 3.0);
  Builder b("random_tris", RT_DRAW_FLAT, make_material(0.1, 0.1, 0.1, 0.7, 0.6, 0.5, 0.3, 0.3, 0.3, 20.0, 0.0));
  b.m.positions.reserve(9 * (size_t)N);
  b.m.tri_vertex.reserve(3 * (size_t)N);
  for (long long t = 0; t < N; ++t) {
    const double c[3] = {rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-1, 1)};
    int v[3];
    for (int k = 0; k < 3; ++k)
      v[k] = b.vertex(c[0] + rng.uniform(-e, e), c[1] + rng.uniform(-e, e), c[2] + rng.uniform(-e, e));
    b.tri(v[0], v[1], v[2]);
  }
  sc.meshes.push_back(std::move(b.m));
  sc.camera = rt_camera_def{};
  set3(sc.camera.eye, 0.0, 0.0, 4.0);
  set3(sc.camera.center, 0.0, 0.0, 0.0);
  set3(sc.camera.up, 0.0, 1.0, 0.0);
  sc.camera.fovy = 45.0;
  sc.camera.width = 1920;
  sc.camera.height = 1080;
  sc.max_depth = 0;
  set3(sc.background, 0.0, 0.0, 0.0);
  set3(sc.ambience, 0.2, 0.2, 0.2);
  sc.lights.push_back(light(2.0, 3.0, 5.0, 0.9, 0.9, 0.9));
}

void gen_cornell(const rt_gen_params& p, HostScene& sc) {
  const int det = p.detail > 0 ? p.detail : 1;
  sc.camera = rt_camera_def{};
  set3(sc.camera.eye, 0.03, 1.02, 3.35);
  set3(sc.camera.center, -0.02, 0.97, 0.0);
  set3(sc.camera.up, 0.0, 1.0, 0.0);
  sc.camera.fovy = 50.0;
  sc.camera.width = 160;
  sc.camera.height = 120;
  sc.max_depth = 3;
  set3(sc.background, 0.1, 0.1, 0.15);
  set3(sc.ambience, 0.2, 0.2, 0.2);
  sc.lights.push_back(light(0.3, 1.85, 0.6, 0.6, 0.6, 0.55));
  sc.lights.push_back(light(-0.6, 1.5, 1.8, 0.35, 0.3, 0.3));
  {
    Builder b("room", RT_DRAW_FLAT, make_material(0.3, 0.3, 0.3, 0.75, 0.75, 0.72, 0.0, 0.0, 0.0, 1.0, 0.0));
    const int n = scaled(6, det);
    { const double o[3] = {-1, 0, 1}, a[3] = {2, 0, 0}, c[3] = {0, 0, -2}; b.grid(o, a, c, n, n); }    // floor
    { const double o[3] = {-1, 2, -1}, a[3] = {2, 0, 0}, c[3] = {0, 0, 2}; b.grid(o, a, c, n, n); }    // ceiling
    { const double o[3] = {-1, 0, -1}, a[3] = {2, 0, 0}, c[3] = {0, 2, 0}; b.grid(o, a, c, n, n); }    // back
    sc.meshes.push_back(std::move(b.m));
  }
  {
    Builder b("red_wall", RT_DRAW_FLAT, make_material(0.3, 0.05, 0.05, 0.75, 0.1, 0.1, 0.1, 0.1, 0.1, 5.0, 0.0));
    const double o[3] = {-1, 0, 1}, a[3] = {0, 0, -2}, c[3] = {0, 2, 0};
    b.grid(o, a, c, scaled(6, det), scaled(6, det));
    sc.meshes.push_back(std::move(b.m));
  }
  {  // right wall is a mirror
    Builder b("mirror_wall", RT_DRAW_FLAT, make_material(0.05, 0.1, 0.05, 0.1, 0.5, 0.1, 0.5, 0.5, 0.5, 50.0, 0.7));
    const double o[3] = {1, 0, -1}, a[3] = {0, 0, 2}, c[3] = {0, 2, 0};
    b.grid(o, a, c, scaled(6, det), scaled(6, det));
    sc.meshes.push_back(std::move(b.m));
  }
  {
    Builder b("phong_ball", RT_DRAW_PHONG, make_material(0.1, 0.1, 0.25, 0.3, 0.35, 0.85, 0.8, 0.8, 0.8, 64.0, 0.0));
    b.sphere(-0.42, 0.36, -0.25, 0.36, scaled(40, det), scaled(20, det));
    sc.meshes.push_back(std::move(b.m));
  }
  {
    Builder b("chrome_ball", RT_DRAW_PHONG, make_material(0.05, 0.05, 0.05, 0.2, 0.2, 0.2, 0.9, 0.9, 0.9, 120.0, 0.6));
    b.sphere(0.45, 0.3, 0.25, 0.3, scaled(32, det), scaled(16, det));
    sc.meshes.push_back(std::move(b.m));
  }
  {  // flat box, not shadowable
    Builder b("box", RT_DRAW_FLAT, make_material(0.25, 0.2, 0.1, 0.7, 0.55, 0.25, 0.2, 0.2, 0.2, 10.0, 0.0, 0));
    b.box(0.15, 0.0, -0.75, 0.6, 0.8, -0.3, scaled(2, det));
    sc.meshes.push_back(std::move(b.m));
  }
  {  // textured poster on the back wall
    Builder b("poster", RT_DRAW_FLAT, make_material(0.2, 0.2, 0.2, 1.0, 1.0, 1.0, 0.1, 0.1, 0.1, 10.0, 0.0));
    const double o[3] = {-0.8, 0.9, -0.99}, a[3] = {0.9, 0, 0}, c[3] = {0, 0.8, 0};
    const int n = 3;
    b.grid(o, a, c, n, n);
    for (int j = 0; j <= n; ++j)
      for (int i = 0; i <= n; ++i) { b.m.u.push_back((double)i / n); b.m.v.push_back((double)j / n); }
    b.m.tri_uv = b.m.tri_vertex;   // grid vertex id == uv id
    b.m.tex_w = 37; b.m.tex_h = 29;
    b.m.texels.resize(3 * 37 * 29);
    for (int y = 0; y < 29; ++y)
      for (int x = 0; x < 37; ++x) {
        const bool chk = ((x / 4) + (y / 4)) % 2;
        unsigned char* t = &b.m.texels[3 * (y * 37 + x)];
        t[0] = (unsigned char)(chk ? 230 : 20 + 6 * x);
        t[1] = (unsigned char)(chk ? 200 : 40 + 7 * y);
        t[2] = (unsigned char)(chk ? 30 : 180);
      }
    sc.meshes.push_back(std::move(b.m));
  }
}

}  // namespace

void generate_scene(const std::string& kind, const rt_gen_params& p, HostScene& sc) {
  sc = HostScene();
  if (kind == "office") gen_office(p, sc);
  else if (kind == "spheres") gen_spheres(p, sc);
  else if (kind == "random_tris") gen_random_tris(p, sc);
  else if (kind == "cornell") gen_cornell(p, sc);
  else throw std::runtime_error("unknown scene kind: " + kind);
  if (p.width > 0) sc.camera.width = p.width;
  if (p.height > 0) sc.camera.height = p.height;
  if (p.max_depth >= 0) sc.max_depth = p.max_depth;
}

}  // namespace rt
