/*
 * rt_multi.h — single-process multi-GPU render of one frame on one node (librt_multi.so).
 *
 * image rows shard embarrassingly over the GPUs of a node (pixels are
 * independent, mytracer_gpu.cu:132-159).  GPU g of n renders the interleaved row stripes
 * (y / stripe_height) % n == g, packed in increasing y (rt_render_params rules, the same
 * kernel launch as rt_launch_compute_image); then ONE ncclGather (RCCL over xGMI) of the
 * equal-size, padded stripe buffers to devices[0] and a re-interleave kernel there
 * assemble the frame.  The scene and its device hierarchy are built once on the host and
 * copied to every GPU (rt_scene_upload_multi).
 *
 * The reference renders on device 0 only (launch_compute_image_device,
 * mytracer_gpu.cu:32-113); this is the entry its C++ host side
 * (Raytracer::compute_image_cuda, mytracer.cpp:123-159) would call to use a whole node.
 * One host thread drives every GPU: launches are asynchronous and the collective is one
 * ncclGroupStart/End over the per-device communicators (ncclCommInitAll).
 */
#ifndef RT_MULTI_H
#define RT_MULTI_H

#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_multi rt_multi;   /* opaque: scenes, communicators, streams, stripe buffers */

/* Uploads the scene to devices[0..n_devices) and creates one RCCL communicator per device.
 * n_devices >= 1; device ids must be distinct (RCCL allows one rank per GPU).  opt's reserve_cus
 * (default 0) applies per GPU: 32 leaves one XCD's worth of CUs free for the gathers of the
 * previous batch. */
int rt_multi_create(const rt_scene_soa* soa, const rt_bvh_soa* bvh, const int* devices, int n_devices,
                    const rt_upload_options* opt, rt_multi** out);

/* Number of GPUs of the driver. */
int rt_multi_device_count(const rt_multi* m);

/* Frame assembly of rt_multi_render*: RT_MULTI_GATHER (default) = one grouped ncclGather per
 * batch of frames to devices[0] and a re-interleave kernel there; RT_MULTI_PEER = every GPU's
 * launch writes its stripes straight into the output frames on devices[0] over xGMI
 * (RT_FLAG_GLOBAL_ROWS), with no copy and no re-interleave.  Setting RT_MULTI_PEER checks and
 * enables peer access from every device to devices[0]; it fails (RT_ERR_UNSUPPORTED, the
 * driver unchanged) when a device cannot access it.  Guard: before its first peer render the
 * driver renders a corner window of the caller's first frame (at most 128 x 2n stripes, every GPU
 * rendering rows of it) once by the gather and once by peer stores and keeps the peer assembly
 * only if the two are bit-identical; otherwise it gathers from then on (rt_multi_assembly tells
 * which is in use).  Setting RT_MULTI_PEER again re-arms the check.  The calling thread's current
 * device is left as it was by every rt_multi call. */
enum { RT_MULTI_GATHER = 0, RT_MULTI_PEER = 1 };
int rt_multi_set_assembly(rt_multi* m, int assembly);

/* The frame assembly in use: RT_MULTI_GATHER or RT_MULTI_PEER (RT_MULTI_GATHER after the peer guard
 * refused peer stores). */
int rt_multi_assembly(const rt_multi* m);

/* Test hook: what = RT_MULTI_DEBUG_PEER_MISMATCH corrupts one word of the peer guard's frame, so
 * the guard must refuse the peer assembly; 0 = off. */
enum { RT_MULTI_DEBUG_PEER_MISMATCH = 1 };
int rt_multi_debug_inject(rt_multi* m, int what);

/* Renders one whole frame (rt_multi_render_frames with one frame; p->row_begin / row_end / stripe_* are ignored: every row is
 * rendered, sharded as above with the given stripe_height >= 1) into d_out, a DEVICE
 * buffer on devices[0] holding height x width x 3 values of p->out_format, row-major,
 * row 0 first (the layout of rt_launch_compute_image).  Synchronous.  stats (optional):
 * ray counters summed over the GPUs; ms (optional): wall time from the first launch to
 * the assembled frame (render + gather + re-interleave). */
int rt_multi_render(rt_multi* m, const rt_render_params* p, int stripe_height, void* d_out, rt_stats* stats,
                    double* ms);

/* Renders n_frames whole frames: frame f renders p[f] into d_outs[f] (device buffers on
 * devices[0], layout as rt_multi_render); the frames must share size and out_format (they may
 * differ as rt_launch_frames allows: camera vectors).  Frames go in batches of up to
 * RT_MAX_FRAMES: every GPU renders its stripes of a batch in ONE rt_launch_frames (the
 * per-launch drain is paid once per batch), one ncclGather per batch collects the stripe blocks
 * on devices[0], and one kernel re-interleaves every frame of the batch.  Two batches are in
 * flight on separate streams and communicators (double-buffered stripe buffers), so the gather
 * and re-interleave of batch i proceed while batch i + 1 renders (at least two batches when
 * n_frames >= 2).  Synchronous; results equal n_frames rt_multi_render calls.  stats / ms as
 * rt_multi_render (stats synchronises every launch, so pass NULL when timing).  Replaces the
 * reference's single-device launch_compute_image_device (mytracer_gpu.cu:32-113) for a node. */
int rt_multi_render_frames(rt_multi* m, const rt_render_params* p, int n_frames, int stripe_height,
                           void* const* d_outs, rt_stats* stats, double* ms);

/* rt_multi_render into a HOST buffer (the frame is copied from devices[0] after ms is taken). */
int rt_multi_render_to_host(rt_multi* m, const rt_render_params* p, int stripe_height, void* host_out,
                            rt_stats* stats, double* ms);

/* Rows of the largest shard: the padded stripe-buffer height every GPU sends. */
int rt_multi_max_rows(int height, int stripe_height, int n);

/* Host restatement of the frame assembly (no GPU): gathered holds n shard buffers of
 * rt_multi_max_rows(height, stripe_height, n) x width x channels elements of elem_bytes
 * each, shard g packed as GPU g renders it; out receives the height x width x channels
 * frame.  Same index map as the device kernel. */
int rt_multi_interleave_host(const void* gathered, void* out, int height, int width, int channels, int elem_bytes,
                             int stripe_height, int n);

/* The same for a batch: gathered holds n blocks of n_frames x max_rows x width x channels
 * elements (GPU g's stripes of every frame of the batch, as rt_multi_render_frames gathers them);
 * outs[f] receives frame f. */
int rt_multi_interleave_frames_host(const void* gathered, void* const* outs, int n_frames, int height, int width,
                                    int channels, int elem_bytes, int stripe_height, int n);

void rt_multi_free(rt_multi* m);

/* Thread-local message of the last failing rt_multi_* call. */
const char* rt_multi_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_MULTI_H */
