// rt_multi.hip — single-process multi-GPU driver (include/rt_multi.h): row stripes per GPU,
// one RCCL gather to devices[0], a re-interleave kernel there.  SURVEY §8(e).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/rt_multi.h"

namespace {

thread_local std::string g_error;

int fail(int code, const std::string& msg) {
  g_error = msg;
  return code;
}

#define HIP_TRY(call)                                                                          \
  do {                                                                                         \
    const hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess) return fail(RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCCL_TRY(call)                                                                         \
  do {                                                                                         \
    const ncclResult_t r_ = (call);                                                            \
    if (r_ != ncclSuccess) return fail(RT_ERR_HIP, std::string(#call) + ": " + ncclGetErrorString(r_)); \
  } while (0)

// Shard g renders the rows (y / sh) % n == g packed in increasing y: global row y sits in
// shard (y / sh) % n at local row (y / sh / n) * sh + y % sh.  Shared by the device kernel
// and the host restatement.
__host__ __device__ inline void stripe_source(int y, int sh, int n, int& shard, int& lrow) {
  const int s = y / sh;
  shard = s % n;
  lrow = (s / n) * sh + y % sh;
}

int max_rows_of(int h, int sh, int n) {
  int best = 0;
  for (int g = 0; g < n; ++g) {
    int rows = 0;
    for (int y = 0; y < h; ++y)
      if ((y / sh) % n == g) rows++;
    best = rows > best ? rows : best;
  }
  return best;
}

// One thread per 4-B word of an output row (rows are width x 3 x 4 or 8 bytes, so 4-B
// aligned): row y of the frame comes from its shard's packed buffer in the gathered array
// [n][max_rows][row_bytes].
__global__ void interleave_kernel(const uint32_t* __restrict__ gathered, uint32_t* __restrict__ out, int height,
                                  size_t row_words, int sh, int n, int max_rows) {
  const int y = blockIdx.y;
  int shard, lrow;
  stripe_source(y, sh, n, shard, lrow);
  const uint32_t* src = gathered + ((size_t)shard * max_rows + lrow) * row_words;
  uint32_t* dst = out + (size_t)y * row_words;
  for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < row_words; c += (size_t)gridDim.x * blockDim.x)
    dst[c] = src[c];
}

}  // namespace

struct rt_multi {
  int n = 0;
  std::vector<int> devices;
  std::vector<rt_scene*> scenes;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;
  std::vector<void*> sbuf;     // per device: its packed stripes (max_rows x row_bytes)
  size_t sbuf_bytes = 0;
  void* gbuf = nullptr;        // devices[0]: n x max_rows x row_bytes
  size_t gbuf_bytes = 0;
};

extern "C" {

const char* rt_multi_last_error(void) { return g_error.c_str(); }

int rt_multi_max_rows(int height, int stripe_height, int n) {
  if (height <= 0 || stripe_height < 1 || n < 1) return 0;
  return max_rows_of(height, stripe_height, n);
}

int rt_multi_interleave_host(const void* gathered, void* out, int height, int width, int channels, int elem_bytes,
                             int stripe_height, int n) {
  if (!gathered || !out || height <= 0 || width <= 0 || channels <= 0 || elem_bytes <= 0 || stripe_height < 1 ||
      n < 1)
    return fail(RT_ERR_INVALID, "rt_multi_interleave_host: bad argument");
  const int mr = max_rows_of(height, stripe_height, n);
  const size_t row_bytes = (size_t)width * channels * elem_bytes;
  for (int y = 0; y < height; ++y) {
    int shard, lrow;
    stripe_source(y, stripe_height, n, shard, lrow);
    std::memcpy(static_cast<unsigned char*>(out) + (size_t)y * row_bytes,
                static_cast<const unsigned char*>(gathered) + ((size_t)shard * mr + lrow) * row_bytes, row_bytes);
  }
  return RT_OK;
}

void rt_multi_free(rt_multi* m) {
  if (!m) return;
  for (int g = 0; g < (int)m->devices.size(); ++g) {
    (void)hipSetDevice(m->devices[g]);
    (void)hipDeviceSynchronize();
    if (g < (int)m->sbuf.size() && m->sbuf[g]) (void)hipFree(m->sbuf[g]);
    if (g < (int)m->streams.size() && m->streams[g]) (void)hipStreamDestroy(m->streams[g]);
    if (g < (int)m->comms.size() && m->comms[g]) (void)ncclCommDestroy(m->comms[g]);
    if (g < (int)m->scenes.size()) rt_scene_free(m->scenes[g]);
  }
  if (m->gbuf) {
    (void)hipSetDevice(m->devices[0]);
    (void)hipFree(m->gbuf);
  }
  delete m;
}

int rt_multi_create(const rt_scene_soa* soa, const rt_bvh_soa* bvh, const int* devices, int n_devices,
                    const rt_upload_options* opt, rt_multi** out) {
  if (!out || !devices || n_devices < 1) return fail(RT_ERR_INVALID, "rt_multi_create: bad argument");
  *out = nullptr;
  for (int a = 0; a < n_devices; ++a)
    for (int b = a + 1; b < n_devices; ++b)
      if (devices[a] == devices[b]) return fail(RT_ERR_INVALID, "rt_multi_create: device ids must be distinct");
  auto* m = new rt_multi();
  m->n = n_devices;
  m->devices.assign(devices, devices + n_devices);
  m->scenes.assign(n_devices, nullptr);
  if (rt_scene_upload_multi(soa, bvh, devices, n_devices, opt, m->scenes.data()) != RT_OK) {
    const std::string e = rt_last_error();
    rt_multi_free(m);
    return fail(RT_ERR_HIP, "rt_multi_create: " + e);
  }
  m->comms.assign(n_devices, nullptr);
  m->streams.assign(n_devices, nullptr);
  m->sbuf.assign(n_devices, nullptr);
  for (int g = 0; g < n_devices; ++g) {
    if (hipSetDevice(devices[g]) != hipSuccess ||
        hipStreamCreateWithFlags(&m->streams[g], hipStreamNonBlocking) != hipSuccess) {
      rt_multi_free(m);
      return fail(RT_ERR_HIP, "rt_multi_create: stream creation failed");
    }
  }
  const ncclResult_t r = ncclCommInitAll(m->comms.data(), n_devices, devices);
  if (r != ncclSuccess) {
    m->comms.assign(n_devices, nullptr);
    rt_multi_free(m);
    return fail(RT_ERR_HIP, std::string("rt_multi_create: ncclCommInitAll: ") + ncclGetErrorString(r));
  }
  *out = m;
  return RT_OK;
}

int rt_multi_device_count(const rt_multi* m) { return m ? m->n : 0; }

int rt_multi_render(rt_multi* m, const rt_render_params* p, int stripe_height, void* d_out, rt_stats* stats,
                    double* ms) {
  if (!m || !p || !d_out || stripe_height < 1) return fail(RT_ERR_INVALID, "rt_multi_render: bad argument");
  if (p->out_format != RT_OUT_RGB_F32 && p->out_format != RT_OUT_RGB_F64)
    return fail(RT_ERR_INVALID, "rt_multi_render: bad out_format");
  const int n = m->n, W = p->camera.width, H = p->camera.height;
  if (W <= 0 || H <= 0) return fail(RT_ERR_INVALID, "rt_multi_render: bad image size");
  const int elem = p->out_format == RT_OUT_RGB_F64 ? 8 : 4;
  const int mr = max_rows_of(H, stripe_height, n);
  const size_t row_bytes = (size_t)W * 3 * elem;
  const size_t shard_bytes = (size_t)mr * row_bytes;
  if (shard_bytes > m->sbuf_bytes) {   // (re)allocate the stripe buffers for this frame size
    for (int g = 0; g < n; ++g) {
      HIP_TRY(hipSetDevice(m->devices[g]));
      HIP_TRY(hipDeviceSynchronize());
      if (m->sbuf[g]) HIP_TRY(hipFree(m->sbuf[g]));
      m->sbuf[g] = nullptr;
      HIP_TRY(hipMalloc(&m->sbuf[g], shard_bytes));
    }
    m->sbuf_bytes = shard_bytes;
    HIP_TRY(hipSetDevice(m->devices[0]));
    if (m->gbuf) HIP_TRY(hipFree(m->gbuf));
    m->gbuf = nullptr;
    HIP_TRY(hipMalloc(&m->gbuf, shard_bytes * n));
    m->gbuf_bytes = shard_bytes * n;
  }
  const auto t0 = std::chrono::steady_clock::now();
  // every GPU renders its stripes (asynchronous launches on its own stream)
  for (int g = 0; g < n; ++g) {
    rt_render_params q = *p;
    q.row_begin = 0;
    q.row_end = H;
    q.stripe_height = stripe_height;
    q.stripe_count = n;
    q.stripe_index = g;
    if (rt_launch_compute_image(m->scenes[g], &q, m->sbuf[g], nullptr, m->streams[g]) != RT_OK)
      return fail(RT_ERR_HIP, std::string("rt_multi_render: device ") + std::to_string(m->devices[g]) + ": " +
                                  rt_last_error());
  }
  // ONE gather of the padded stripe buffers to devices[0] (each rank sends on its own link)
  const size_t count = shard_bytes / elem;
  const ncclDataType_t type = elem == 8 ? ncclFloat64 : ncclFloat32;
  NCCL_TRY(ncclGroupStart());
  for (int g = 0; g < n; ++g)
    NCCL_TRY(ncclGather(m->sbuf[g], g == 0 ? m->gbuf : nullptr, count, type, 0, m->comms[g], m->streams[g]));
  NCCL_TRY(ncclGroupEnd());
  // re-interleave the stripes into the frame on devices[0]
  HIP_TRY(hipSetDevice(m->devices[0]));
  const size_t row_words = row_bytes / 4;
  const unsigned bx = (unsigned)std::min<size_t>((row_words + 255) / 256, 64);
  interleave_kernel<<<dim3(bx, (unsigned)H), dim3(256), 0, m->streams[0]>>>(
      static_cast<const uint32_t*>(m->gbuf), static_cast<uint32_t*>(d_out), H, row_words, stripe_height, n, mr);
  HIP_TRY(hipGetLastError());
  for (int g = 0; g < n; ++g) {
    HIP_TRY(hipSetDevice(m->devices[g]));
    HIP_TRY(hipStreamSynchronize(m->streams[g]));
  }
  const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (ms) *ms = t;
  if (stats) {   // raw counter words [8, 11) of each GPU's launch = primary / shadow / reflection rays
    std::memset(stats, 0, sizeof *stats);
    for (int g = 0; g < n; ++g) {
      unsigned long long w[32] = {};
      if (rt_debug_counters(m->scenes[g], w, 32) < 32) return fail(RT_ERR_HIP, "rt_multi_render: counters");
      if (w[31] != 0) return fail(RT_ERR_HIP, "rt_multi_render: persistent-loop watchdog fired (kernel bug)");
      stats->primary_rays += (long long)w[8];
      stats->shadow_rays += (long long)w[9];
      stats->reflection_rays += (long long)w[10];
      stats->pixels += (long long)w[14];
    }
  }
  return RT_OK;
}

int rt_multi_render_to_host(rt_multi* m, const rt_render_params* p, int stripe_height, void* host_out,
                            rt_stats* stats, double* ms) {
  if (!m || !p || !host_out) return fail(RT_ERR_INVALID, "rt_multi_render_to_host: bad argument");
  const size_t bytes = (size_t)p->camera.width * p->camera.height * 3 * (p->out_format == RT_OUT_RGB_F64 ? 8 : 4);
  HIP_TRY(hipSetDevice(m->devices[0]));
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, bytes));
  const int rc = rt_multi_render(m, p, stripe_height, d, stats, ms);
  if (rc == RT_OK) {
    (void)hipSetDevice(m->devices[0]);
    const hipError_t e = hipMemcpy(host_out, d, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("rt_multi_render_to_host: ") + hipGetErrorString(e));
    return RT_OK;
  }
  (void)hipFree(d);
  return rc;
}

}  // extern "C"
