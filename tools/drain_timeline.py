"""Single-frame launch anatomy (dev tool, under gpurun): kernel time vs image size and
max_depth, and the per-wave timeline (start, last work fetch, end) of one 1080p frame.
usage: python tools/drain_timeline.py"""
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)


def timed(p, reps=7):
    out = torch.zeros((p.camera.height, p.camera.width, 3), device="cuda")
    st = gpu.launch(p, out.data_ptr(), stats=True)
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gpu.launch(p, out.data_ptr())
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms)), st.primary_rays + st.shadow_rays + st.reflection_rays


for w, h in [(64, 64), (480, 270), (960, 540), (1920, 1080), (2715, 1527), (3840, 2160)]:
    for depth in (5, 0):
        p = host.render_params(w, h, 1)
        p.max_depth = depth
        ms, rays = timed(p)
        print(f"{w}x{h} depth {depth}: {ms:.3f} ms, {rays} rays, {rays / ms / 1e3:.0f} Mrays/s", flush=True)

p = host.render_params(1920, 1080, 1)
p.flags = rtamd.RT_FLAG_WIDE_STATS
out = torch.zeros((1080, 1920, 3), device="cuda")
for _ in range(2):
    gpu.launch(p, out.data_ptr(), stats=True)
print(f"STATS variant 1080p: {gpu.last_kernel_ms():.3f} ms")
log = gpu.wave_log().astype(np.int64)
log = log[log[:, 2] >= log[:, 0].max() - 100_000_000]
t0 = log[:, 0].min()
us = (log[:, :3] - t0) / 100.0
start, refill, end, pix = us[:, 0], us[:, 1], us[:, 2], log[:, 3]
print(f"waves {len(log)}, pixels {pix.sum()}")
for name, v in [("start", start), ("last fetch", refill), ("end", end)]:
    q = np.percentile(v, [0, 10, 50, 90, 99, 100])
    print(f"  {name:10s} us: " + "  ".join(f"p{k}={x:.0f}" for k, x in zip([0, 10, 50, 90, 99, 100], q)))
print(f"  drain after last fetch: median {np.median(end - refill):.0f} us, p90 {np.percentile(end - refill, 90):.0f}, "
      f"max {np.max(end - refill):.0f} us")
t = np.linspace(0, end.max(), 26)
print("  waves still running:", " ".join(f"{int((end > x).sum())}" for x in t))
print("  t(us):             ", " ".join(f"{x:.0f}" for x in t))
