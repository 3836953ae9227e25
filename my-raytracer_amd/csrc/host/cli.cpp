// cli.cpp — rt_render: command-line front end of the MI355X render path.
//
// Host-side mirror of the reference's Raytracer flow (mytracer.cpp:54-60 and
// 123-159): init (read/generate scene, compute normals, build_Data, BVH
// initSoA) then compute_image on the GPU and write the image.  Everything goes
// through the two C-ABIs (rt_host.h, rt_hip.h); no HIP headers here.
//
//   rt_render --scene office|cornell|random_tris|spheres|path.sce
//             [--width W --height H --spp N --max-depth D --tris N --seed S
//              --detail K --device I --gpus N --assembly gather|peer --frames F --adaptive
//              --out image.ppm]
// --gpus N renders each frame on GPUs 0..N-1 (row stripes + one RCCL gather, rt_multi.h; with
// --assembly peer every GPU stores its rows straight into device 0's frame instead);
// without it one device (--device) renders through rt_render_to_host.  --adaptive (one device):
// the primary pass followed by the adaptive supersampling pass (subp 4, threshold 0.02), as the
// reference's launch_compute_image_device always runs them (mytracer_gpu.cu:44-113).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/rt_hip.h"
#include "../../../include/rt_host.h"
#include "../../../include/rt_multi.h"

namespace {

class Raytracer {
 public:
  ~Raytracer() {
    rt_multi_free(multi_);
    rt_scene_free(gpu_);
    rt_host_free(host_);
  }
  // Raytracer::init_cuda equivalent; gpus >= 1: every frame sharded over GPUs 0..gpus-1.
  bool init(const std::string& scene, const rt_gen_params& gp, int device, int gpus, bool peer) {
    int rc = (scene.size() > 4 && scene.substr(scene.size() - 4) == ".sce") ? rt_host_load(scene.c_str(), &host_)
                                                                              : rt_host_generate(scene.c_str(), &gp, &host_);
    if (rc != RT_OK) return error(rt_host_last_error());
    double build_s = 0;
    if (rt_host_prepare(host_, &build_s) != RT_OK) return error(rt_host_last_error());
    std::printf("scene %s: %lld triangles, BVH depth %d, host build %.3f s\n", scene.c_str(),
                rt_host_triangle_count(host_), rt_host_bvh_depth(host_), build_s);
    if (gpus >= 1) {
      std::vector<int> devs(gpus);
      for (int g = 0; g < gpus; ++g) devs[g] = g;
      if (rt_multi_create(rt_host_soa(host_), rt_host_bvh(host_), devs.data(), gpus, nullptr, &multi_) != RT_OK)
        return error(rt_multi_last_error());
      if (peer && rt_multi_set_assembly(multi_, RT_MULTI_PEER) != RT_OK) return error(rt_multi_last_error());
      std::printf("uploaded to %d devices (row stripes of %d rows, %s)\n", gpus, kStripe,
                  peer ? "peer stores into device 0's frame" : "RCCL gather to device 0");
      return true;
    }
    if (rt_scene_upload(rt_host_soa(host_), rt_host_bvh(host_), device, &gpu_) != RT_OK) return error(rt_last_error());
    std::printf("uploaded %.1f MB to device %d\n", rt_scene_device_bytes(gpu_) / 1e6, device);
    return true;
  }
  // Raytracer::compute_image_cuda equivalent.
  bool compute_image(int width, int height, int spp, int max_depth, int frames, bool adaptive) {
    if (rt_host_render_params(host_, width, height, spp, &params_) != RT_OK) return error(rt_host_last_error());
    if (max_depth >= 0) params_.max_depth = max_depth;
    image_.assign(3 * (size_t)params_.camera.width * params_.camera.height, 0.f);
    for (int f = 0; f < frames; ++f) {
      rt_stats st;
      float ms = 0;
      if (multi_) {
        double mt = 0;
        if (rt_multi_render_to_host(multi_, &params_, kStripe, image_.data(), &st, &mt) != RT_OK)
          return error(rt_multi_last_error());
        ms = (float)mt;
        if (f == 0)   // (peer stores are kept only if the driver's bit check of the first frame passed)
          std::printf("frame assembly in use: %s\n",
                      rt_multi_assembly(multi_) == RT_MULTI_PEER ? "peer stores" : "RCCL gather");
      } else if (adaptive) {
        rt_stats st1;
        long long n_sel = 0;
        const auto t0 = std::chrono::steady_clock::now();
        if (rt_render_adaptive_to_host(gpu_, &params_, 4, 0.02, image_.data(), &st, &st1, &n_sel) != RT_OK)
          return error(rt_last_error());
        ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::printf("frame %d: adaptive pass re-rendered %lld pixels (rays P %lld S %lld R %lld)\n", f, n_sel,
                    st1.primary_rays, st1.shadow_rays, st1.reflection_rays);
        st.primary_rays += st1.primary_rays;
        st.shadow_rays += st1.shadow_rays;
        st.reflection_rays += st1.reflection_rays;
      } else {
        if (rt_render_to_host(gpu_, &params_, image_.data(), &st) != RT_OK) return error(rt_last_error());
        rt_last_kernel_ms(gpu_, &ms);
      }
      const long long rays = st.primary_rays + st.shadow_rays + st.reflection_rays;
      std::printf("frame %d: %dx%d spp %d  %s %.3f ms  rays %lld (P %lld S %lld R %lld)  %.1f Mrays/s\n", f,
                  params_.camera.width, params_.camera.height, params_.spp_n * params_.spp_n,
                  adaptive ? "call (both passes + copy)" : "kernel", ms, rays,
                  st.primary_rays, st.shadow_rays, st.reflection_rays, rays / (ms * 1e3));
    }
    return true;
  }
  bool write(const std::string& path) {
    if (rt_write_ppm(path.c_str(), image_.data(), params_.camera.width, params_.camera.height) != RT_OK)
      return error(rt_host_last_error());
    std::printf("wrote %s\n", path.c_str());
    return true;
  }

 private:
  bool error(const char* msg) {
    std::fprintf(stderr, "rt_render: %s\n", msg);
    return false;
  }
  static constexpr int kStripe = 16;   // rows per stripe (interleaved over the GPUs)
  rt_host_scene* host_ = nullptr;
  rt_scene* gpu_ = nullptr;
  rt_multi* multi_ = nullptr;
  rt_render_params params_{};
  std::vector<float> image_;
};

}  // namespace

int main(int argc, char** argv) {
  std::string scene = "office", out;
  int width = 0, height = 0, spp = 1, max_depth = -1, device = 0, frames = 1, gpus = 0;
  bool adaptive = false;
  std::string assembly = "gather";
  rt_gen_params gp{};
  gp.max_depth = -1;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
      return argv[++i];
    };
    if (a == "--scene") scene = next();
    else if (a == "--width") width = std::atoi(next());
    else if (a == "--height") height = std::atoi(next());
    else if (a == "--spp") spp = std::atoi(next());
    else if (a == "--max-depth") max_depth = std::atoi(next());
    else if (a == "--tris") gp.n_triangles = std::atoll(next());
    else if (a == "--seed") gp.seed = std::strtoull(next(), nullptr, 10);
    else if (a == "--detail") gp.detail = std::atoi(next());
    else if (a == "--device") device = std::atoi(next());
    else if (a == "--frames") frames = std::atoi(next());
    else if (a == "--gpus") gpus = std::atoi(next());
    else if (a == "--assembly") assembly = next();
    else if (a == "--out") out = next();
    else if (a == "--adaptive") adaptive = true;
    else if (a == "--help" || a == "-h") {
      std::printf("usage: rt_render [--scene office|cornell|random_tris|spheres|FILE.sce] [--width W] [--height H]\n"
                  "                 [--spp N] [--max-depth D] [--tris N] [--seed S] [--detail K] [--device I]\n"
                  "                 [--gpus N [--assembly gather|peer]] [--frames F] [--adaptive] [--out image.ppm]\n");
      return 0;
    }
    else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
  }
  Raytracer rt;
  if (gpus < 0) { std::fprintf(stderr, "--gpus must be >= 1\n"); return 2; }
  if (assembly != "gather" && assembly != "peer") { std::fprintf(stderr, "--assembly must be gather or peer\n"); return 2; }
  if (adaptive && gpus >= 1) { std::fprintf(stderr, "--adaptive renders on one device (no --gpus)\n"); return 2; }
  if (!rt.init(scene, gp, device, gpus, assembly == "peer")) return 1;
  if (!rt.compute_image(width, height, spp, max_depth, frames, adaptive)) return 1;
  if (!out.empty() && !rt.write(out)) return 1;
  return 0;
}
