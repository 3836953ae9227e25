"""Where does a multi-frame launch's fixed cost go? (dev tool, GPU)  Office 1080p, orbit views.
1. Production kernel time T(F) for F frames per launch (natural order), fitted T = a + b F.
2. For F = 1, 20, 128 one diagnostic (4-wide stats variant) launch's per-wave log (start, last work
   fetch, end; s_memrealtime, 10-ns ticks): the ramp (first to last wave start), the time the queue
   runs dry (last fetch), and the drain after it (when 50 / 90 / 99 / 100 % of the waves ended).

usage: python tools/launch_shape_probe.py
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "my-raytracer_amd"))
import rtamd  # noqa: E402
from rtamd import abi  # noqa: E402

hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
base = hs.render_params(1920, 1080, 1)
FMAX = 128
cams = [rtamd.camera_orbit(base, 0.12 * (f / 19 - 0.5)) for f in range(FMAX)]
bufs = [torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda") for _ in range(FMAX)]


def launch(F, flags=abi.RT_FLAG_NATURAL_ORDER, stats=False):
    ps = [abi.RenderParams.from_buffer_copy(c) for c in cams[:F]]
    for q in ps:
        q.flags = flags
    if F == 1:
        return dev.launch(ps[0], bufs[0].data_ptr(), stats=stats)
    return dev.launch_frames(ps, [b.data_ptr() for b in bufs[:F]], stats=stats)


fs = [1, 2, 5, 10, 20, 40, 128]
t = {}
for F in fs:
    for _ in range(2):
        launch(F)
    ms = []
    for _ in range(7 if F < 128 else 3):
        launch(F)
        torch.cuda.synchronize()
        ms.append(dev.last_kernel_ms())
    t[F] = float(np.median(ms))
    print(json.dumps({"frames": F, "kernel_ms": round(t[F], 4), "ms_per_frame": round(t[F] / F, 4)}), flush=True)
x = np.array(fs[2:], float)
y = np.array([t[F] for F in fs[2:]])
b, a = np.polyfit(x, y, 1)
print(json.dumps({"fit_F>=5": {"a_ms": round(float(a), 4), "b_ms_per_frame": round(float(b), 4)}}), flush=True)

for F in (1, 20, 128):
    launch(F, abi.RT_FLAG_WIDE_STATS, stats=True)
    torch.cuda.synchronize()
    kms = dev.last_kernel_ms()
    wl = dev.wave_log()
    wl = wl[wl[:, 2] > 0] if len(wl) else wl
    s, f, e = (wl[:, k].astype(np.int64) for k in range(3))
    t0 = s.min()
    dry = f.max() - t0
    ends = np.sort(e - t0)
    n = len(ends)
    q = lambda p: float(ends[min(n - 1, int(p * n))]) / 100.0   # noqa: E731  (ticks -> microseconds)
    print(json.dumps({"frames": F, "stats_kernel_ms": round(kms, 4), "waves": n,
                      "ramp_us_p50_start": float(np.median(s - t0)) / 100.0,
                      "ramp_us_last_start": float((s - t0).max()) / 100.0,
                      "queue_dry_us": float(dry) / 100.0,
                      "end_us_p50": q(0.5), "end_us_p90": q(0.9), "end_us_p99": q(0.99),
                      "end_us_last": float(ends[-1]) / 100.0,
                      "drain_after_dry_us": float(ends[-1] - dry) / 100.0}), flush=True)
