// loader.cpp — .sce / .obj / .mtl scene files and texture images.
//
// The reference's course parser (Raytracer::read_scene, Mesh::read_obj) is
// absent; only its pre-read pass is visible: scene tokens `mesh <file> <mode>`
// with the mesh path taken relative to the scene file (mytracer.cpp:330-344)
// and .obj headers v / vt / vn / mtllib / usemtl / f (mytracer.cpp:447-488).
// The grammar below keeps those tokens and fixes the rest:
//
//   # comment
//   camera     ex ey ez  cx cy cz  ux uy uz  fovy  width height
//   depth      D
//   background r g b
//   ambience   r g b
//   light      x y z  r g b
//   sphere     cx cy cz  radius           MATERIAL
//   plane      cx cy cz  nx ny nz         MATERIAL
//   mesh       file.obj  FLAT|PHONG       MATERIAL
//   MATERIAL := ar ag ab  dr dg db  sr sg sb  shininess  mirror  [shadowable(0|1)]
//
// .obj faces with more than 3 corners are fan-triangulated; `usemtl` selects
// the `map_Kd` texture of the named .mtl material (PPM P3/P6 or 8-bit PNG).
#include <zlib.h>

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>

#include "host_scene.hpp"

namespace rt {

namespace {

std::string dir_of(const std::string& path) {
  const size_t p = path.find_last_of('/');
  return p == std::string::npos ? std::string() : path.substr(0, p + 1);
}

std::string base_of(const std::string& path) {
  const size_t p = path.find_last_of('/');
  return p == std::string::npos ? path : path.substr(p + 1);
}

bool read_file(const std::string& path, std::vector<unsigned char>& data) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  data.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}

// --- PPM (P3 / P6, maxval <= 255) ---
bool read_ppm(const std::vector<unsigned char>& d, int& w, int& h, std::vector<unsigned char>& rgb) {
  size_t pos = 0;
  auto next_token = [&]() -> std::string {
    std::string tok;
    while (pos < d.size()) {
      const char c = (char)d[pos];
      if (c == '#') { while (pos < d.size() && d[pos] != '\n') ++pos; continue; }
      if (std::isspace((unsigned char)c)) { if (!tok.empty()) break; ++pos; continue; }
      tok.push_back(c); ++pos;
    }
    return tok;
  };
  const std::string magic = next_token();
  if (magic != "P6" && magic != "P3") return false;
  w = std::stoi(next_token());
  h = std::stoi(next_token());
  const int maxval = std::stoi(next_token());
  if (w <= 0 || h <= 0 || maxval <= 0 || maxval > 255) return false;
  rgb.resize(3 * (size_t)w * h);
  if (magic == "P6") {
    ++pos;  // single whitespace after maxval
    if (pos + rgb.size() > d.size()) return false;
    std::memcpy(rgb.data(), d.data() + pos, rgb.size());
  } else {
    for (auto& c : rgb) c = (unsigned char)std::stoi(next_token());
  }
  if (maxval != 255)
    for (auto& c : rgb) c = (unsigned char)std::lround(c * 255.0 / maxval);
  return true;
}

// --- PNG: every standard colour type and bit depth (gray 1/2/4/8/16, RGB 8/16,
// palette 1/2/4/8, gray+alpha 8/16, RGBA 8/16), plain or Adam7-interlaced.  Converted
// to RGB8 the way lodepng's RGBA8 decode does (the usual course Image loader): 16-bit
// samples keep their high byte, low-bit gray scales as v*255/(2^depth-1), palette
// indices look up PLTE; alpha is dropped (the texel is used as an RGB colour). ---
uint32_t be32(const unsigned char* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

bool png_unfilter(const unsigned char* src, unsigned char* dst, size_t stride, int rows, int bpp) {
  for (int y = 0; y < rows; ++y) {
    const unsigned char filter = src[y * (stride + 1)];
    const unsigned char* in = &src[y * (stride + 1) + 1];
    unsigned char* out = &dst[y * stride];
    const unsigned char* prev = y > 0 ? &dst[(y - 1) * stride] : nullptr;
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= (size_t)bpp ? out[x - bpp] : 0;
      const int b = prev ? prev[x] : 0;
      const int c = (prev && x >= (size_t)bpp) ? prev[x - bpp] : 0;
      int v = in[x];
      switch (filter) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: { const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                  v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c); break; }
        default: return false;
      }
      out[x] = (unsigned char)v;
    }
  }
  return true;
}

bool read_png(const std::vector<unsigned char>& d, int& w, int& h, std::vector<unsigned char>& rgb) {
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) return false;
  size_t pos = 8;
  int depth = 0, ctype = -1, interlace = 0;
  bool have_ihdr = false;
  std::vector<unsigned char> idat, plte;
  while (pos + 8 <= d.size()) {
    const uint32_t len = be32(&d[pos]);
    const std::string type((const char*)&d[pos + 4], 4);
    if (len > d.size() || pos + 12 + len > d.size()) return false;
    const unsigned char* body = &d[pos + 8];
    if (type == "IHDR") {
      if (len < 13) return false;
      w = (int)be32(body); h = (int)be32(body + 4);
      depth = body[8]; ctype = body[9]; interlace = body[12];
      have_ihdr = true;
    } else if (type == "PLTE") {
      plte.assign(body, body + len);
    } else if (type == "IDAT") {
      idat.insert(idat.end(), body, body + len);
    } else if (type == "IEND") {
      break;
    }
    pos += 12 + len;
  }
  if (!have_ihdr || w <= 0 || h <= 0 || (long long)w * h > (1ll << 28) || interlace > 1) return false;
  int ch;
  switch (ctype) { case 0: ch = 1; break; case 2: ch = 3; break; case 3: ch = 1; break; case 4: ch = 2; break;
                   case 6: ch = 4; break; default: return false; }
  const bool depth_ok = ctype == 0 ? (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)
                      : ctype == 3 ? (depth == 1 || depth == 2 || depth == 4 || depth == 8)
                                   : (depth == 8 || depth == 16);
  if (!depth_ok || (ctype == 3 && (plte.empty() || plte.size() % 3 != 0))) return false;
  const int bits_pp = ch * depth;
  const int bpp = std::max(1, bits_pp / 8);
  // passes: Adam7 (7 sub-images) or one full image
  static const int IX[7] = {0, 4, 0, 2, 0, 1, 0}, IY[7] = {0, 0, 4, 0, 2, 0, 1};
  static const int DX[7] = {8, 8, 4, 4, 2, 2, 1}, DY[7] = {8, 8, 8, 4, 4, 2, 2};
  const int npass = interlace ? 7 : 1;
  int pw[7], ph[7];
  size_t raw_size = 0;
  for (int p = 0; p < npass; ++p) {
    pw[p] = interlace ? (w > IX[p] ? (w - IX[p] + DX[p] - 1) / DX[p] : 0) : w;
    ph[p] = interlace ? (h > IY[p] ? (h - IY[p] + DY[p] - 1) / DY[p] : 0) : h;
    if (pw[p] > 0 && ph[p] > 0) raw_size += (size_t)ph[p] * (1 + ((size_t)pw[p] * bits_pp + 7) / 8);
  }
  std::vector<unsigned char> raw(raw_size);
  uLongf raw_len = raw.size();
  if (uncompress(raw.data(), &raw_len, idat.data(), idat.size()) != Z_OK || raw_len != raw.size()) return false;
  const int maxv = (1 << depth) - 1;
  auto sample = [&](const unsigned char* line, int x, int c) -> int {
    if (depth == 8) return line[(size_t)x * ch + c];
    if (depth == 16) return line[2 * ((size_t)x * ch + c)];   // high byte
    const size_t bit = (size_t)x * depth;                      // ch == 1 for depth < 8
    return (line[bit / 8] >> (8 - depth - (int)(bit % 8))) & maxv;
  };
  rgb.assign(3 * (size_t)w * h, 0);
  size_t off = 0;
  std::vector<unsigned char> img;
  for (int p = 0; p < npass; ++p) {
    if (pw[p] == 0 || ph[p] == 0) continue;
    const size_t stride = ((size_t)pw[p] * bits_pp + 7) / 8;
    img.assign(stride * ph[p], 0);
    if (!png_unfilter(&raw[off], img.data(), stride, ph[p], bpp)) return false;
    off += (stride + 1) * ph[p];
    for (int y = 0; y < ph[p]; ++y) {
      const unsigned char* line = &img[y * stride];
      const int oy = interlace ? IY[p] + y * DY[p] : y;
      for (int x = 0; x < pw[p]; ++x) {
        const int ox = interlace ? IX[p] + x * DX[p] : x;
        unsigned char* o = &rgb[3 * ((size_t)oy * w + ox)];
        if (ctype == 3) {
          const int idx = sample(line, x, 0);
          if (3 * (size_t)idx + 2 >= plte.size()) return false;
          for (int k = 0; k < 3; ++k) o[k] = plte[3 * idx + k];
        } else if (ch >= 3) {
          for (int k = 0; k < 3; ++k) o[k] = (unsigned char)sample(line, x, k);
        } else {
          const int g = sample(line, x, 0);
          const unsigned char v = depth < 8 ? (unsigned char)(g * 255 / maxv) : (unsigned char)g;
          o[0] = o[1] = o[2] = v;
        }
      }
    }
  }
  return true;
}

rt_material parse_material(std::istringstream& ls, const std::string& line) {
  double m[11];
  for (double& x : m)
    if (!(ls >> x)) throw std::runtime_error("material needs 11 numbers: " + line);
  int shadowable = 1;
  int sh;
  if (ls >> sh) shadowable = sh;
  return make_material(m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9], m[10], shadowable);
}

std::map<std::string, std::string> read_mtl(const std::string& path) {
  std::map<std::string, std::string> tex;   // material name -> map_Kd path
  std::ifstream f(path);
  if (!f) return tex;
  std::string line, cur;
  while (std::getline(f, line)) {
    std::istringstream ls(line);
    std::string key;
    if (!(ls >> key)) continue;
    if (key == "newmtl") ls >> cur;
    else if (key == "map_Kd") {   // options (-s u v w, -bm b, ...) precede the file name: take the last token
      std::string fn, t;
      while (ls >> t) fn = t;
      if (!fn.empty()) tex[cur] = dir_of(path) + fn;
    }
  }
  return tex;
}

int parse_index(const std::string& tok, int count) {
  const int i = std::stoi(tok);
  return i > 0 ? i - 1 : count + i;   // 1-based; negative = relative
}

void read_obj(const std::string& path, HostMesh& mesh) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::map<std::string, std::string> mtl_tex;
  std::string texture_file;
  std::string line;
  bool any_uv_face = false;
  while (std::getline(f, line)) {
    const size_t sp = line.find_first_of(" \t");
    const std::string header = line.substr(0, sp);
    std::istringstream ls(sp == std::string::npos ? std::string() : line.substr(sp + 1));
    if (header == "v") {
      double x, y, z;
      ls >> x >> y >> z;
      mesh.positions.push_back(x); mesh.positions.push_back(y); mesh.positions.push_back(z);
    } else if (header == "vt") {
      double u, v;
      ls >> u >> v;
      mesh.u.push_back(u); mesh.v.push_back(v);
    } else if (header == "mtllib") {
      std::string fn; ls >> fn;
      mtl_tex = read_mtl(dir_of(path) + fn);
    } else if (header == "usemtl") {
      std::string name; ls >> name;
      auto it = mtl_tex.find(name);
      if (it != mtl_tex.end() && texture_file.empty()) texture_file = it->second;
    } else if (header == "f") {
      std::vector<int> vi, ti;
      std::string tok;
      while (ls >> tok) {
        const size_t s1 = tok.find('/');
        vi.push_back(parse_index(tok.substr(0, s1), mesh.n_vertices()));
        int t = -1;
        if (s1 != std::string::npos) {
          const size_t s2 = tok.find('/', s1 + 1);
          const std::string ts = tok.substr(s1 + 1, s2 == std::string::npos ? std::string::npos : s2 - s1 - 1);
          if (!ts.empty()) { t = parse_index(ts, (int)mesh.u.size()); any_uv_face = true; }
        }
        ti.push_back(t);
      }
      for (size_t k = 2; k < vi.size(); ++k) {   // fan triangulation
        mesh.tri_vertex.push_back(vi[0]); mesh.tri_vertex.push_back(vi[k - 1]); mesh.tri_vertex.push_back(vi[k]);
        mesh.tri_uv.push_back(ti[0]); mesh.tri_uv.push_back(ti[k - 1]); mesh.tri_uv.push_back(ti[k]);
      }
    }
  }
  for (int idx : mesh.tri_vertex)
    if (idx < 0 || idx >= mesh.n_vertices()) throw std::runtime_error("vertex index out of range in " + path);
  if (!any_uv_face || mesh.u.empty()) {
    mesh.tri_uv.clear();
  } else {
    for (int& t : mesh.tri_uv) {
      if (t < 0) t = 0;
      if (t >= (int)mesh.u.size()) throw std::runtime_error("uv index out of range in " + path);
    }
  }
  if (!texture_file.empty() && !mesh.tri_uv.empty()) {
    if (!read_image(texture_file, mesh.tex_w, mesh.tex_h, mesh.texels))
      throw std::runtime_error("cannot read texture " + texture_file);
  }
  mesh.name = base_of(path);
}

void write_vec(std::ostream& o, const double* v, int n) {
  for (int i = 0; i < n; ++i) o << ' ' << v[i];
}

void write_material(std::ostream& o, const rt_material& m) {
  write_vec(o, m.ambient, 3); write_vec(o, m.diffuse, 3); write_vec(o, m.specular, 3);
  o << ' ' << m.shininess << ' ' << m.mirror << ' ' << m.shadowable;
}

}  // namespace

bool read_image(const std::string& path, int& w, int& h, std::vector<unsigned char>& rgb) {
  std::vector<unsigned char> d;
  if (!read_file(path, d)) return false;
  if (read_png(d, w, h, rgb)) return true;
  return read_ppm(d, w, h, rgb);
}

void load_sce(const std::string& path, HostScene& scene) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open scene " + path);
  scene = HostScene();
  scene.camera.fovy = 45.0;
  scene.camera.width = 640;
  scene.camera.height = 480;
  scene.camera.up[1] = 1.0;
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream ls(line);
    std::string key;
    if (!(ls >> key) || key[0] == '#') continue;
    if (key == "camera") {
      rt_camera_def& c = scene.camera;
      ls >> c.eye[0] >> c.eye[1] >> c.eye[2] >> c.center[0] >> c.center[1] >> c.center[2] >> c.up[0] >>
          c.up[1] >> c.up[2] >> c.fovy >> c.width >> c.height;
      if (!ls) throw std::runtime_error("bad camera line: " + line);
    } else if (key == "depth") {
      ls >> scene.max_depth;
    } else if (key == "background") {
      ls >> scene.background[0] >> scene.background[1] >> scene.background[2];
    } else if (key == "ambience") {
      ls >> scene.ambience[0] >> scene.ambience[1] >> scene.ambience[2];
    } else if (key == "light") {
      rt_light l{};
      ls >> l.position[0] >> l.position[1] >> l.position[2] >> l.color[0] >> l.color[1] >> l.color[2];
      if (!ls) throw std::runtime_error("bad light line: " + line);
      scene.lights.push_back(l);
    } else if (key == "sphere") {
      rt_sphere s{};
      ls >> s.center[0] >> s.center[1] >> s.center[2] >> s.radius;
      s.material = parse_material(ls, line);
      scene.spheres.push_back(s);
    } else if (key == "plane") {
      rt_plane p{};
      ls >> p.center[0] >> p.center[1] >> p.center[2] >> p.normal[0] >> p.normal[1] >> p.normal[2];
      p.material = parse_material(ls, line);
      scene.planes.push_back(p);
    } else if (key == "mesh") {
      std::string fn, mode;
      ls >> fn >> mode;
      HostMesh m;
      if (mode == "FLAT") m.draw_mode = RT_DRAW_FLAT;
      else if (mode == "PHONG") m.draw_mode = RT_DRAW_PHONG;
      else throw std::runtime_error("mesh mode must be FLAT or PHONG: " + line);
      m.material = parse_material(ls, line);
      read_obj(dir_of(path) + fn, m);          // path relative to the scene (mytracer.cpp:337-340)
      scene.meshes.push_back(std::move(m));
    } else {
      throw std::runtime_error("unknown scene statement: " + key);
    }
  }
}

void save_sce(const HostScene& scene, const std::string& path) {
  std::ofstream o(path);
  if (!o) throw std::runtime_error("cannot write " + path);
  o.precision(17);
  const std::string dir = dir_of(path), base = base_of(path);
  const std::string stem = base.substr(0, base.find_last_of('.'));
  const rt_camera_def& c = scene.camera;
  o << "camera";
  write_vec(o, c.eye, 3); write_vec(o, c.center, 3); write_vec(o, c.up, 3);
  o << ' ' << c.fovy << ' ' << c.width << ' ' << c.height << "\n";
  o << "depth " << scene.max_depth << "\n";
  o << "background"; write_vec(o, scene.background, 3); o << "\n";
  o << "ambience"; write_vec(o, scene.ambience, 3); o << "\n";
  for (const auto& l : scene.lights) { o << "light"; write_vec(o, l.position, 3); write_vec(o, l.color, 3); o << "\n"; }
  for (const auto& s : scene.spheres) {
    o << "sphere"; write_vec(o, s.center, 3); o << ' ' << s.radius; write_material(o, s.material); o << "\n";
  }
  for (const auto& p : scene.planes) {
    o << "plane"; write_vec(o, p.center, 3); write_vec(o, p.normal, 3); write_material(o, p.material); o << "\n";
  }
  for (size_t i = 0; i < scene.meshes.size(); ++i) {
    const HostMesh& m = scene.meshes[i];
    const std::string obj = stem + "_mesh" + std::to_string(i) + ".obj";
    std::ofstream ob(dir + obj);
    if (!ob) throw std::runtime_error("cannot write " + dir + obj);
    ob.precision(17);
    if (m.tex_w > 0) {
      const std::string mtl = stem + "_mesh" + std::to_string(i) + ".mtl";
      const std::string ppm = stem + "_mesh" + std::to_string(i) + ".ppm";
      std::ofstream mo(dir + mtl);
      mo << "newmtl tex\nmap_Kd " << ppm << "\n";
      FILE* pf = std::fopen((dir + ppm).c_str(), "wb");
      if (!pf) throw std::runtime_error("cannot write " + dir + ppm);
      std::fprintf(pf, "P6\n%d %d\n255\n", m.tex_w, m.tex_h);
      std::fwrite(m.texels.data(), 1, m.texels.size(), pf);
      std::fclose(pf);
      ob << "mtllib " << mtl << "\nusemtl tex\n";
    }
    for (int v = 0; v < m.n_vertices(); ++v) { ob << "v"; write_vec(ob, &m.positions[3 * (size_t)v], 3); ob << "\n"; }
    for (size_t t = 0; t < m.u.size(); ++t) ob << "vt " << m.u[t] << ' ' << m.v[t] << "\n";
    for (int t = 0; t < m.n_triangles(); ++t) {
      ob << "f";
      for (int k = 0; k < 3; ++k) {
        ob << ' ' << m.tri_vertex[3 * t + k] + 1;
        if (!m.tri_uv.empty()) ob << '/' << m.tri_uv[3 * t + k] + 1;
      }
      ob << "\n";
    }
    o << "mesh " << obj << ' ' << (m.draw_mode == RT_DRAW_PHONG ? "PHONG" : "FLAT");
    write_material(o, m.material);
    o << "\n";
  }
}

}  // namespace rt
