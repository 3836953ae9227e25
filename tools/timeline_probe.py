"""Per-wave timeline of one launch (dev tool): when waves run out of work and
how long the drain tail is.  Uses the 4-wide STATS variant (rt_debug_wave_log)."""
import sys

import numpy as np

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

w, h, spp = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (1920, 1080, 1)))
host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(w, h, spp)
p.flags = rtamd.RT_FLAG_WIDE_STATS
gpu.render(p)
gpu.render(p)
ms = gpu.last_kernel_ms()
log = gpu.wave_log().astype(np.int64)
log = log[log[:, 2] >= log[:, 0].max() - 10_000_000]   # this launch's waves (stale words are older)
t0 = log[:, 0].min()
us = (log[:, :3] - t0) / 100.0   # 100 MHz -> microseconds
start, refill, end, pix = us[:, 0], us[:, 1], us[:, 2], log[:, 3]
print(f"{w}x{h} spp{spp*spp}: kernel {ms*1e3:.0f} us (stats variant), waves {len(log)}, pixels {pix.sum()}")
for name, v in [("start", start), ("last fetch", refill), ("end", end)]:
    q = np.percentile(v, [0, 10, 50, 90, 99, 100])
    print(f"  {name:10s} us: " + "  ".join(f"p{k}={x:.0f}" for k, x in zip([0, 10, 50, 90, 99, 100], q)))
print(f"  drain after last fetch (end - last fetch): median {np.median(end - refill):.0f} us, max {np.max(end - refill):.0f} us")
t = np.linspace(0, end.max(), 21)
print("  waves still running:", " ".join(f"{int((end > x).sum())}" for x in t))
