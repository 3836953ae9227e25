"""Per-wave timeline of one multi-frame launch (dev tool): start skew, last fetch, drain.
usage: python tools/timeline_frames.py [frames]"""
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 8
host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(1920, 1080, 1)
bufs = [torch.zeros((1080, 1920, 3), device="cuda") for _ in range(F)]
for flags in (0, rtamd.RT_FLAG_WIDE_STATS):
    p.flags = flags
    for _ in range(2):
        gpu.launch_frames(p, [b.data_ptr() for b in bufs], stats=True)
    ms = gpu.last_kernel_ms()
    print(f"F={F} flags={flags}: kernel {ms:.3f} ms ({ms / F:.3f} ms/frame)")
log = gpu.wave_log().astype(np.int64)
log = log[log[:, 2] >= log[:, 0].max() - 100_000_000]
t0 = log[:, 0].min()
us = (log[:, :3] - t0) / 100.0
start, refill, end, pix = us[:, 0], us[:, 1], us[:, 2], log[:, 3]
print(f"waves {len(log)}, pixels {pix.sum()}")
for name, v in [("start", start), ("last fetch", refill), ("end", end)]:
    q = np.percentile(v, [0, 10, 50, 90, 99, 100])
    print(f"  {name:10s} us: " + "  ".join(f"p{k}={x:.0f}" for k, x in zip([0, 10, 50, 90, 99, 100], q)))
print(f"  drain after last fetch: median {np.median(end - refill):.0f} us, max {np.max(end - refill):.0f} us")
t = np.linspace(0, end.max(), 21)
print("  waves still running:", " ".join(f"{int((end > x).sum())}" for x in t))
