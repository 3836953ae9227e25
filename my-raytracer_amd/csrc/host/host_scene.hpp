// host_scene.hpp — C++ host-side scene model of the MI355X render path.
//
// Mirrors the course types the reference's host code reads (Mesh with
// vertices_/triangles_/u_coordinates_/v_coordinates_/material_/draw_mode_/
// texture_, Raytracer with lights_/camera_/background_/ambience_/max_depth_;
// call sites mytracer.cpp:221-294, mymesh.cpp:103-163) but stores each mesh
// in flat arrays so the raw rt_raw_scene view (include/rt_scene.h) and the
// SoA build can be produced without copies.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/rt_host.h"

namespace rt {

struct HostMesh {
  std::string name;
  std::vector<double> positions;   // 3 * n_vertices
  std::vector<int> tri_vertex;     // 3 * n_triangles (mesh-local)
  std::vector<double> u, v;        // texture coordinates
  std::vector<int> tri_uv;         // 3 * n_triangles or empty
  int draw_mode = RT_DRAW_FLAT;
  rt_material material{};
  int tex_w = 0, tex_h = 0;        // 0: no texture
  std::vector<unsigned char> texels;  // RGB8, row 0 = top
  // derived by compute_normals (mymesh.cpp:103-163)
  std::vector<double> vertex_normals;  // 3 * n_vertices
  std::vector<double> face_normals;    // 3 * n_triangles

  int n_vertices() const { return (int)(positions.size() / 3); }
  int n_triangles() const { return (int)(tri_vertex.size() / 3); }
  void compute_normals();
};

// Struct Data (mydata.h:28-72) as host vectors, packed xyz.
struct SoA {
  int n_meshes = 0, n_vertices = 0, n_vertex_idx = 0, n_tex_coords = 0;
  long long n_texels = 0;
  std::vector<int> vertex_mesh_id;
  std::vector<double> vertex_pos, vertex_normals, face_normals;
  std::vector<int> vertex_idx, texture_idx;
  std::vector<double> tex_u, tex_v;
  std::vector<unsigned char> texels;
  std::vector<int> first_vertex, vertex_count, first_vertex_idx, vertex_idx_count;
  std::vector<int> first_tex_coord, tex_coord_count;
  std::vector<int> mesh_tex_width, mesh_tex_height;
  std::vector<long long> mesh_tex_offset;
  std::vector<int> mesh_draw_mode;
  std::vector<double> mat_ambient, mat_diffuse, mat_specular, mat_shininess, mat_mirror;
  std::vector<int> mat_shadowable;
};

// BVH::BVHNodes_SoA (mybvh.h:49-55) as host vectors.
struct BvhSoA {
  int n_nodes = 0;         // nodesUsed_
  std::vector<double> bb_min, bb_max;   // 3 * allocated
  std::vector<int> left_child, first_tri, tri_count;
  int depth = 0;
};

struct HostScene {
  rt_camera_def camera{};
  double background[3] = {0, 0, 0};
  double ambience[3] = {0, 0, 0};
  int max_depth = 0;
  std::vector<rt_light> lights;
  std::vector<HostMesh> meshes;
  std::vector<rt_sphere> spheres;
  std::vector<rt_plane> planes;

  // views / derived
  std::vector<rt_mesh> raw_meshes;
  rt_raw_scene raw{};
  bool prepared = false;
  SoA soa;
  BvhSoA bvh;
  rt_scene_soa soa_view{};
  rt_bvh_soa bvh_view{};

  void refresh_raw();              // rebuild the rt_raw_scene view
  void prepare(int build_threads = 0);   // compute_normals + build_Data + initSoA (0 threads: usable CPUs)
  long long triangle_count() const;
};

// Steps of Raytracer::init_cuda (mytracer.cpp:54-60), restated.
void build_data(const HostScene& scene, SoA& soa);       // mytracer.cpp:166-296
void build_bvh_soa(SoA& soa, BvhSoA& bvh, int threads = 0);   // mybvh.cpp:375-539
void derive_camera(const rt_camera_def& def, int width, int height, rt_camera& out);

// loader.cpp
void load_sce(const std::string& path, HostScene& scene);  // throws std::runtime_error
void save_sce(const HostScene& scene, const std::string& path);
bool read_image(const std::string& path, int& w, int& h, std::vector<unsigned char>& rgb);

// generators.cpp
void generate_scene(const std::string& kind, const rt_gen_params& p, HostScene& scene);

rt_material make_material(double ar, double ag, double ab, double dr, double dg, double db,
                          double sr, double sg, double sb, double shininess, double mirror,
                          int shadowable = 1);

}  // namespace rt
