// device_image.hpp — host side of rt_scene_upload: turns the reference's Data SoA + median-split
// BVH (BVH::initSoA, mybvh.cpp:375-539; Raytracer::build_Data, mytracer.cpp:166-296) into the
// MI355X device layout (rt_layout.hpp) that librt_hip.so copies to each GPU.
//
// Pure C++ (no HIP): the device hierarchy builders (the reference tree with oversize leaves
// refined, binned SAH, SAH with spatial splits), the 2-wide canonical nodes, the 4-wide
// collapse with its breadth-first LDS treelet prefix, and the fp64 triangle / shading records
// in device leaf order.  Built into librt_hip.so beside the kernel.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/rt_hip.h"
#include "../device/rt_layout.hpp"

namespace rtk {

constexpr int kMaxStackDepth = 4096;   // traversal stack entries (LDS ring + global spill)

// Host-side device layout of a scene: built once (the expensive part: device hierarchy,
// records), then copied to any number of devices.
struct SceneImage {
  std::vector<GNode> nodes;       // 2-wide canonical nodes over the reference tree (preorder)
  std::vector<GNode4> nodes4;     // 4-wide production nodes (first `bfs_top` breadth-first)
  std::vector<GTri> tris;         // triangle records in device leaf order
  std::vector<uint32_t> slot2dev; // reference slot -> first device record
  std::vector<TriShade> shade;
  std::vector<double> tnorm, tu, tv;
  std::vector<unsigned char> texels;
  std::vector<GMat> mats;
  long long n_tris = 0;
  int n_meshes = 0;
  int depth = 0, stack4 = 1;
  double delta = 0.0;
  double root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};
};

// Builds the device layout.  `bfs_top`: how many 4-wide nodes to number breadth-first (the
// treelet the kernel caches in LDS).  Returns RT_OK or an RT_ERR_* code with the message in
// build_image_error().
int build_image(const rt_scene_soa* s, const rt_bvh_soa* b, const rt_upload_options& opt, int bfs_top,
                SceneImage& I);
const std::string& build_image_error();

// Defaults of rt_upload_options (include/rt_hip.h).
void upload_options_defaults(rt_upload_options* opt);

}  // namespace rtk
