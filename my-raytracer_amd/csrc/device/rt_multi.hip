// rt_multi.hip — single-process multi-GPU driver (include/rt_multi.h): row stripes per GPU,
// one RCCL gather to devices[0], a re-interleave kernel there (or, RT_MULTI_PEER, every GPU storing
// its rows straight into devices[0]'s frames).  SURVEY §8(e).
// Frames go in batches (one rt_launch_frames per GPU per batch, so the per-launch drain is paid
// once per batch), and two batches are in flight: batch i + 1 renders on the other slot's
// streams while batch i's gather and re-interleave drain.
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

// Restores the calling thread's current device when an entry point returns (every return path):
// the driver switches devices internally, the caller's own device stays current.
struct DeviceRestore {
  int dev = -1;
  DeviceRestore() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DeviceRestore() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
};

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
// aligned): row y of frame f = blockIdx.z comes from its shard's packed buffer in the gathered
// array [n][n_frames][max_rows][row_bytes] (each GPU sends its frames' stripes as one block).
__global__ void interleave_kernel(const uint32_t* __restrict__ gathered, uint32_t* const* __restrict__ outs,
                                  int n_frames, size_t row_words, int sh, int n, int max_rows) {
  const int y = blockIdx.y, f = blockIdx.z;
  int shard, lrow;
  stripe_source(y, sh, n, shard, lrow);
  const uint32_t* src = gathered + (((size_t)shard * n_frames + f) * max_rows + lrow) * row_words;
  uint32_t* dst = outs[f] + (size_t)y * row_words;
  for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < row_words; c += (size_t)gridDim.x * blockDim.x)
    dst[c] = src[c];
}

void interleave_host(const void* gathered, void* const* outs, int n_frames, int height, size_t row_bytes, int sh,
                     int n) {
  const int mr = max_rows_of(height, sh, n);
  for (int f = 0; f < n_frames; ++f)
    for (int y = 0; y < height; ++y) {
      int shard, lrow;
      stripe_source(y, sh, n, shard, lrow);
      std::memcpy(static_cast<unsigned char*>(outs[f]) + (size_t)y * row_bytes,
                  static_cast<const unsigned char*>(gathered) + (((size_t)shard * n_frames + f) * mr + lrow) * row_bytes,
                  row_bytes);
    }
}

// A batch in flight: per device its stripe buffers for the batch's frames and the streams its
// launch and gather run on, on devices[0] the gathered array and the output table.  Two slots
// alternate, each with its own communicators, so the collectives of two batches never share a
// communicator across streams.
constexpr int kSlots = 2;
struct Slot {
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;
  std::vector<void*> sbuf;       // per device: [frames][max_rows][row_bytes]
  void* gbuf = nullptr;          // devices[0]: [n][frames][max_rows][row_bytes]
  void** d_outs = nullptr;       // devices[0]: [RT_MAX_FRAMES] output pointers of the batch
  void** h_outs = nullptr;       // pinned staging of the same
  hipEvent_t done = nullptr;     // devices[0]: the batch's re-interleave finished
  bool busy = false;
};

}  // namespace

struct rt_multi {
  int n = 0;
  int assembly = RT_MULTI_GATHER;
  std::vector<int> devices;
  std::vector<rt_scene*> scenes;
  Slot slot[kSlots];
  size_t sbuf_bytes = 0;       // bytes of every slot's per-device stripe buffer
  void* d_host_stage = nullptr;   // rt_multi_render_to_host: the assembled frame on devices[0], kept
  size_t host_stage_bytes = 0;
  // RT_MULTI_PEER guard: before its first peer render the driver renders a corner window of the
  // caller's first frame both ways and keeps peer only if the two frames are bit-identical
  bool peer_checked = false;
  bool peer_refused = false;
  int debug = 0;                  // rt_multi_debug_inject
};

extern "C" {

const char* rt_multi_last_error(void) { return g_error.c_str(); }

int rt_multi_max_rows(int height, int stripe_height, int n) {
  if (height <= 0 || stripe_height < 1 || n < 1) return 0;
  return max_rows_of(height, stripe_height, n);
}

int rt_multi_interleave_host(const void* gathered, void* out, int height, int width, int channels, int elem_bytes,
                             int stripe_height, int n) {
  return rt_multi_interleave_frames_host(gathered, &out, 1, height, width, channels, elem_bytes, stripe_height, n);
}

int rt_multi_interleave_frames_host(const void* gathered, void* const* outs, int n_frames, int height, int width,
                                    int channels, int elem_bytes, int stripe_height, int n) {
  if (!gathered || !outs || n_frames < 1 || height <= 0 || width <= 0 || channels <= 0 || elem_bytes <= 0 ||
      stripe_height < 1 || n < 1)
    return fail(RT_ERR_INVALID, "rt_multi_interleave_host: bad argument");
  for (int f = 0; f < n_frames; ++f)
    if (!outs[f]) return fail(RT_ERR_INVALID, "rt_multi_interleave_host: null output frame");
  interleave_host(gathered, outs, n_frames, height, (size_t)width * channels * elem_bytes, stripe_height, n);
  return RT_OK;
}

void rt_multi_free(rt_multi* m) {
  if (!m) return;
  DeviceRestore keep;
  for (int g = 0; g < (int)m->devices.size(); ++g) {
    (void)hipSetDevice(m->devices[g]);
    (void)hipDeviceSynchronize();
    for (Slot& S : m->slot) {
      if (g < (int)S.sbuf.size() && S.sbuf[g]) (void)hipFree(S.sbuf[g]);
      if (g < (int)S.streams.size() && S.streams[g]) (void)hipStreamDestroy(S.streams[g]);
      if (g < (int)S.comms.size() && S.comms[g]) (void)ncclCommDestroy(S.comms[g]);
    }
    if (g < (int)m->scenes.size()) rt_scene_free(m->scenes[g]);
  }
  if (!m->devices.empty()) {
    (void)hipSetDevice(m->devices[0]);
    for (Slot& S : m->slot) {
      if (S.gbuf) (void)hipFree(S.gbuf);
      if (S.d_outs) (void)hipFree(S.d_outs);
      if (S.h_outs) (void)hipHostFree(S.h_outs);
      if (S.done) (void)hipEventDestroy(S.done);
    }
    if (m->d_host_stage) (void)hipFree(m->d_host_stage);
  }
  delete m;
}

int rt_multi_create(const rt_scene_soa* soa, const rt_bvh_soa* bvh, const int* devices, int n_devices,
                    const rt_upload_options* opt, rt_multi** out) {
  if (!out || !devices || n_devices < 1) return fail(RT_ERR_INVALID, "rt_multi_create: bad argument");
  *out = nullptr;
  DeviceRestore keep;
  for (int a = 0; a < n_devices; ++a)
    for (int b = a + 1; b < n_devices; ++b)
      if (devices[a] == devices[b]) return fail(RT_ERR_INVALID, "rt_multi_create: device ids must be distinct");
  auto* m = new rt_multi();
  m->n = n_devices;
  m->devices.assign(devices, devices + n_devices);
  m->scenes.assign(n_devices, nullptr);
  // reserve_cus is the caller's (default 0): leaving 32 CUs (one XCD's worth) free lets an RCCL gather run
  // beside the next batch's persistent kernel, but costs ~12 % of the render and its
  // gain is unmeasured at N > 1, so it is opt-in (bench.py records both settings at N > 1)
  rt_upload_options o;
  if (opt) o = *opt;
  else rt_upload_options_init(&o);
  if (rt_scene_upload_multi(soa, bvh, devices, n_devices, &o, m->scenes.data()) != RT_OK) {
    const std::string e = rt_last_error();
    rt_multi_free(m);
    return fail(RT_ERR_HIP, "rt_multi_create: " + e);
  }
  for (Slot& S : m->slot) {
    S.comms.assign(n_devices, nullptr);
    S.streams.assign(n_devices, nullptr);
    S.sbuf.assign(n_devices, nullptr);
    for (int g = 0; g < n_devices; ++g) {
      if (hipSetDevice(devices[g]) != hipSuccess ||
          hipStreamCreateWithFlags(&S.streams[g], hipStreamNonBlocking) != hipSuccess) {
        rt_multi_free(m);
        return fail(RT_ERR_HIP, "rt_multi_create: stream creation failed");
      }
    }
    if (hipSetDevice(devices[0]) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&S.d_outs), RT_MAX_FRAMES * sizeof(void*)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&S.h_outs), RT_MAX_FRAMES * sizeof(void*), hipHostMallocDefault) !=
            hipSuccess ||
        hipEventCreateWithFlags(&S.done, hipEventDisableTiming) != hipSuccess) {
      rt_multi_free(m);
      return fail(RT_ERR_HIP, "rt_multi_create: output table allocation failed");
    }
    const ncclResult_t r = ncclCommInitAll(S.comms.data(), n_devices, devices);
    if (r != ncclSuccess) {
      S.comms.assign(n_devices, nullptr);
      rt_multi_free(m);
      return fail(RT_ERR_HIP, std::string("rt_multi_create: ncclCommInitAll: ") + ncclGetErrorString(r));
    }
  }
  *out = m;
  return RT_OK;
}

int rt_multi_device_count(const rt_multi* m) { return m ? m->n : 0; }

int rt_multi_set_assembly(rt_multi* m, int assembly) {
  if (!m || (assembly != RT_MULTI_GATHER && assembly != RT_MULTI_PEER))
    return fail(RT_ERR_INVALID, "rt_multi_set_assembly: bad argument");
  DeviceRestore keep;
  if (assembly == RT_MULTI_PEER)
    for (int g = 1; g < m->n; ++g) {   // kernels on devices[g] store into devices[0]'s frames
      int can = 0;
      HIP_TRY(hipDeviceCanAccessPeer(&can, m->devices[g], m->devices[0]));
      if (!can)
        return fail(RT_ERR_UNSUPPORTED, "rt_multi_set_assembly: device " + std::to_string(m->devices[g]) +
                                            " cannot access device " + std::to_string(m->devices[0]));
      HIP_TRY(hipSetDevice(m->devices[g]));
      const hipError_t e = hipDeviceEnablePeerAccess(m->devices[0], 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
        return fail(RT_ERR_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
      (void)hipGetLastError();
    }
  m->assembly = assembly;
  m->peer_checked = false;   // a peer assembly is verified again before its first render
  m->peer_refused = false;
  return RT_OK;
}

int rt_multi_assembly(const rt_multi* m) {
  if (!m) return fail(RT_ERR_INVALID, "rt_multi_assembly: null driver");
  return m->assembly;
}

int rt_multi_debug_inject(rt_multi* m, int what) {
  if (!m || what < 0) return fail(RT_ERR_INVALID, "rt_multi_debug_inject: bad argument");
  m->debug = what;
  return RT_OK;
}

namespace {
// RT_MULTI_PEER: GPU g renders its stripes of every frame at their global rows of d_outs (devices[0]
// memory) -- launches of up to RT_MAX_FRAMES frames, all GPUs at once; the call returns when every
// GPU's launches have ended (each wave released its stores at system scope before it exited).
int render_frames_peer(rt_multi* m, const rt_render_params* p, int n_frames, int stripe_height, void* const* d_outs,
                       rt_stats* stats) {
  const int n = m->n, H = p->camera.height;
  std::vector<rt_render_params> q(RT_MAX_FRAMES);
  std::vector<void*> outs(RT_MAX_FRAMES);
  for (int f0 = 0; f0 < n_frames; f0 += RT_MAX_FRAMES) {
    const int F = std::min(RT_MAX_FRAMES, n_frames - f0);
    for (int g = 0; g < n; ++g) {
      for (int f = 0; f < F; ++f) {
        q[f] = p[f0 + f];
        q[f].row_begin = 0;
        q[f].row_end = H;
        q[f].stripe_height = stripe_height;
        q[f].stripe_count = n;
        q[f].stripe_index = g;
        q[f].flags |= RT_FLAG_GLOBAL_ROWS;
        outs[f] = d_outs[f0 + f];
      }
      rt_stats st;
      if (rt_launch_frames(m->scenes[g], q.data(), F, outs.data(), stats ? &st : nullptr, m->slot[0].streams[g]) != RT_OK)
        return fail(RT_ERR_HIP, std::string("rt_multi_render_frames: device ") + std::to_string(m->devices[g]) +
                                    ": " + rt_last_error());
      if (stats) {
        stats->primary_rays += st.primary_rays;
        stats->shadow_rays += st.shadow_rays;
        stats->reflection_rays += st.reflection_rays;
        stats->pixels += st.pixels;
      }
    }
  }
  for (int g = 0; g < n; ++g) {
    HIP_TRY(hipSetDevice(m->devices[g]));
    HIP_TRY(hipStreamSynchronize(m->slot[0].streams[g]));
  }
  return RT_OK;
}
}  // namespace

// Largest batch: frames per launch bounded by RT_MAX_FRAMES and by the gathered array on
// devices[0] (n x frames x shard bytes per slot, at most 8 GB of its 288 GB).
static int batch_cap(int n, size_t shard_bytes) {
  const size_t budget = (size_t)8 << 30;
  const size_t per_frame = std::max<size_t>(1, shard_bytes * (size_t)n);
  return (int)std::max<size_t>(1, std::min<size_t>(RT_MAX_FRAMES, budget / per_frame));
}

namespace {
// RT_MULTI_GATHER: batches of frames, every GPU's stripes of a batch in one launch, one grouped
// ncclGather of the batch to devices[0] and one re-interleave kernel there; two batches in flight.
int render_frames_gather(rt_multi* m, const rt_render_params* p, int n_frames, int stripe_height,
                         void* const* d_outs, rt_stats* stats) {
  const int n = m->n, W = p->camera.width, H = p->camera.height;
  const int elem = p->out_format == RT_OUT_RGB_F64 ? 8 : 4;
  const int mr = max_rows_of(H, stripe_height, n);
  const size_t row_bytes = (size_t)W * 3 * elem;
  const size_t shard_bytes = (size_t)mr * row_bytes;
  const int cap = batch_cap(n, shard_bytes);
  // at least two batches when there are two frames, so a gather overlaps the next launch
  const int n_batches = std::max((n_frames + cap - 1) / cap, std::min(n_frames, kSlots));
  const int per = (n_frames + n_batches - 1) / n_batches;
  const size_t need = shard_bytes * (size_t)per;
  if (need > m->sbuf_bytes) {   // (re)allocate every slot's buffers for this batch size
    for (Slot& S : m->slot) {
      for (int g = 0; g < n; ++g) {
        HIP_TRY(hipSetDevice(m->devices[g]));
        HIP_TRY(hipDeviceSynchronize());
        if (S.sbuf[g]) HIP_TRY(hipFree(S.sbuf[g]));
        S.sbuf[g] = nullptr;
        HIP_TRY(hipMalloc(&S.sbuf[g], need));
      }
      HIP_TRY(hipSetDevice(m->devices[0]));
      if (S.gbuf) HIP_TRY(hipFree(S.gbuf));
      S.gbuf = nullptr;
      HIP_TRY(hipMalloc(&S.gbuf, need * n));
      S.busy = false;
    }
    m->sbuf_bytes = need;
  }
  std::vector<rt_render_params> q((size_t)per);
  std::vector<void*> outs((size_t)per);
  for (int b = 0, f0 = 0; f0 < n_frames; ++b, f0 += per) {
    const int F = std::min(per, n_frames - f0);
    Slot& S = m->slot[b % kSlots];
    if (S.busy) {   // batch b - 2 re-interleaved: its buffers and pinned output table are free again
      HIP_TRY(hipSetDevice(m->devices[0]));
      HIP_TRY(hipEventSynchronize(S.done));
    }
    // every GPU renders its stripes of the batch's frames in one launch on the slot's stream
    for (int g = 0; g < n; ++g) {
      for (int f = 0; f < F; ++f) {
        q[f] = p[f0 + f];
        q[f].row_begin = 0;
        q[f].row_end = H;
        q[f].stripe_height = stripe_height;
        q[f].stripe_count = n;
        q[f].stripe_index = g;
        q[f].flags &= ~RT_FLAG_GLOBAL_ROWS;   // the stripe buffers hold packed shard rows
        outs[f] = static_cast<unsigned char*>(S.sbuf[g]) + (size_t)f * shard_bytes;
      }
      rt_stats st;
      if (rt_launch_frames(m->scenes[g], q.data(), F, outs.data(), stats ? &st : nullptr, S.streams[g]) != RT_OK)
        return fail(RT_ERR_HIP, std::string("rt_multi_render_frames: device ") + std::to_string(m->devices[g]) +
                                    ": " + rt_last_error());
      if (stats) {
        stats->primary_rays += st.primary_rays;
        stats->shadow_rays += st.shadow_rays;
        stats->reflection_rays += st.reflection_rays;
        stats->pixels += st.pixels;
      }
    }
    // ONE gather of the batch's padded stripe blocks to devices[0] (each rank sends on its own link)
    const size_t count = shard_bytes * (size_t)F / elem;
    const ncclDataType_t type = elem == 8 ? ncclFloat64 : ncclFloat32;
    NCCL_TRY(ncclGroupStart());
    for (int g = 0; g < n; ++g)
      NCCL_TRY(ncclGather(S.sbuf[g], g == 0 ? S.gbuf : nullptr, count, type, 0, S.comms[g], S.streams[g]));
    NCCL_TRY(ncclGroupEnd());
    // re-interleave the stripes into the batch's frames on devices[0]
    HIP_TRY(hipSetDevice(m->devices[0]));
    for (int f = 0; f < F; ++f) S.h_outs[f] = d_outs[f0 + f];
    HIP_TRY(hipMemcpyAsync(S.d_outs, S.h_outs, (size_t)F * sizeof(void*), hipMemcpyHostToDevice, S.streams[0]));
    const size_t row_words = row_bytes / 4;
    const unsigned bx = (unsigned)std::min<size_t>((row_words + 255) / 256, 64);
    interleave_kernel<<<dim3(bx, (unsigned)H, (unsigned)F), dim3(256), 0, S.streams[0]>>>(
        static_cast<const uint32_t*>(S.gbuf), reinterpret_cast<uint32_t* const*>(S.d_outs), F, row_words,
        stripe_height, n, mr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(S.done, S.streams[0]));
    S.busy = true;
  }
  for (Slot& S : m->slot)
    for (int g = 0; g < n; ++g) {
      HIP_TRY(hipSetDevice(m->devices[g]));
      HIP_TRY(hipStreamSynchronize(S.streams[g]));
    }
  for (Slot& S : m->slot) S.busy = false;
  return RT_OK;
}

// The RT_MULTI_PEER guard.  Peer frames are correct only if every GPU's image stores, written over
// xGMI into devices[0]'s memory, are there once the GPU's launch has ended (each wave's system-scope
// release before it exits; devices[0] reads them after the launches ended).  Before
// its first peer render the driver checks that on this node: a corner window of the caller's first
// frame (the same camera vectors, at most 128 x 2n stripes: every GPU renders rows of it) rendered
// by the gather and by peer stores into two buffers on devices[0], compared bit for bit; *same =
// whether they agree.
int verify_peer(rt_multi* m, const rt_render_params* p, int stripe_height, bool* same) {
  rt_render_params q = *p;
  q.camera.width = std::min(p->camera.width, 128);
  q.camera.height = std::min(p->camera.height, 2 * m->n * stripe_height);
  const size_t bytes = (size_t)q.camera.width * q.camera.height * 3 * (p->out_format == RT_OUT_RGB_F64 ? 8 : 4);
  HIP_TRY(hipSetDevice(m->devices[0]));
  void* a = nullptr;
  void* b = nullptr;
  HIP_TRY(hipMalloc(&a, bytes));
  if (hipMalloc(&b, bytes) != hipSuccess) {
    (void)hipFree(a);
    return fail(RT_ERR_HIP, "rt_multi peer check: hipMalloc failed");
  }
  std::vector<unsigned char> ha(bytes), hb(bytes);
  int rc = RT_OK;
  // different fills: a pixel left unwritten by either assembly shows as a difference
  if (hipMemset(a, 0x00, bytes) != hipSuccess || hipMemset(b, 0xff, bytes) != hipSuccess)
    rc = fail(RT_ERR_HIP, "rt_multi peer check: hipMemset failed");
  if (rc == RT_OK) rc = render_frames_gather(m, &q, 1, stripe_height, &a, nullptr);
  if (rc == RT_OK) rc = render_frames_peer(m, &q, 1, stripe_height, &b, nullptr);
  if (rc == RT_OK && (m->debug & RT_MULTI_DEBUG_PEER_MISMATCH)) {   // test hook: one corrupted word
    (void)hipSetDevice(m->devices[0]);
    if (hipMemset(b, 0x7f, 4) != hipSuccess) rc = fail(RT_ERR_HIP, "rt_multi peer check: hipMemset failed");
  }
  if (rc == RT_OK) {
    (void)hipSetDevice(m->devices[0]);
    if (hipMemcpy(ha.data(), a, bytes, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hb.data(), b, bytes, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(RT_ERR_HIP, "rt_multi peer check: copy failed");
  }
  (void)hipSetDevice(m->devices[0]);
  (void)hipFree(a);
  (void)hipFree(b);
  if (rc == RT_OK) *same = std::memcmp(ha.data(), hb.data(), bytes) == 0;
  return rc;
}
}  // namespace

int rt_multi_render_frames(rt_multi* m, const rt_render_params* p, int n_frames, int stripe_height,
                           void* const* d_outs, rt_stats* stats, double* ms) {
  if (!m || !p || !d_outs || stripe_height < 1 || n_frames < 1)
    return fail(RT_ERR_INVALID, "rt_multi_render_frames: bad argument");
  if (p->out_format != RT_OUT_RGB_F32 && p->out_format != RT_OUT_RGB_F64)
    return fail(RT_ERR_INVALID, "rt_multi_render_frames: bad out_format");
  const int W = p->camera.width, H = p->camera.height;
  if (W <= 0 || H <= 0) return fail(RT_ERR_INVALID, "rt_multi_render_frames: bad image size");
  for (int f = 0; f < n_frames; ++f) {
    if (!d_outs[f]) return fail(RT_ERR_INVALID, "rt_multi_render_frames: null output buffer");
    if (p[f].camera.width != W || p[f].camera.height != H || p[f].out_format != p->out_format)
      return fail(RT_ERR_INVALID, "rt_multi_render_frames: frames must share size and format");
  }
  DeviceRestore keep;
  if (m->assembly == RT_MULTI_PEER && !m->peer_checked) {   // the peer guard (untimed, once)
    bool same = false;
    const int rc = verify_peer(m, p, stripe_height, &same);
    if (rc != RT_OK) return rc;
    m->peer_checked = true;
    if (!same) {   // refused: this driver gathers from now on (rt_multi_assembly reports it)
      m->assembly = RT_MULTI_GATHER;
      m->peer_refused = true;
    }
  }
  if (stats) std::memset(stats, 0, sizeof *stats);
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = m->assembly == RT_MULTI_PEER ? render_frames_peer(m, p, n_frames, stripe_height, d_outs, stats)
                                              : render_frames_gather(m, p, n_frames, stripe_height, d_outs, stats);
  if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

int rt_multi_render(rt_multi* m, const rt_render_params* p, int stripe_height, void* d_out, rt_stats* stats,
                    double* ms) {
  if (!d_out) return fail(RT_ERR_INVALID, "rt_multi_render: bad argument");
  return rt_multi_render_frames(m, p, 1, stripe_height, &d_out, stats, ms);
}

int rt_multi_render_to_host(rt_multi* m, const rt_render_params* p, int stripe_height, void* host_out,
                            rt_stats* stats, double* ms) {
  if (!m || !p || !host_out) return fail(RT_ERR_INVALID, "rt_multi_render_to_host: bad argument");
  DeviceRestore keep;
  const size_t bytes = (size_t)p->camera.width * p->camera.height * 3 * (p->out_format == RT_OUT_RGB_F64 ? 8 : 4);
  HIP_TRY(hipSetDevice(m->devices[0]));
  if (m->host_stage_bytes < bytes) {   // the frame's device buffer, kept between calls (grown as needed)
    if (m->d_host_stage) HIP_TRY(hipFree(m->d_host_stage));
    m->d_host_stage = nullptr;
    m->host_stage_bytes = 0;
    HIP_TRY(hipMalloc(&m->d_host_stage, bytes));
    m->host_stage_bytes = bytes;
  }
  const int rc = rt_multi_render(m, p, stripe_height, m->d_host_stage, stats, ms);
  if (rc != RT_OK) return rc;
  (void)hipSetDevice(m->devices[0]);
  const hipError_t e = hipMemcpy(host_out, m->d_host_stage, bytes, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("rt_multi_render_to_host: ") + hipGetErrorString(e));
  return RT_OK;
}

}  // extern "C"
