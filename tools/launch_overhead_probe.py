"""Fixed cost of a launch (dev tool, under gpurun): office 1080p kernel time of F-frame launches,
F = 1 .. 64, with one camera for every frame (identical work per frame) and with the bench's
orbit sweep; a least-squares fit T(F) = F * s + X gives the per-frame time s and the per-launch
cost X (ramp-up + drain).  usage: python tools/launch_overhead_probe.py [scene [tris]]"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "office"
gen = {"n_triangles": int(sys.argv[2])} if len(sys.argv) > 2 else {}
host = rtamd.HostScene.generate(scene, **gen)
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(1920, 1080, 1)
FS = [1, 2, 4, 8, 16, 20, 32, 64]
out = [torch.zeros((1080, 1920, 3), device="cuda") for _ in range(max(FS))]
res = {}
for mode in ("same", "sweep"):
    rows = []
    for F in FS:
        if mode == "same" or F == 1:
            cams = [p] * F
        else:
            cams = [rtamd.camera_orbit(p, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
        ptrs = [o.data_ptr() for o in out[:F]]
        for _ in range(2):
            gpu.launch_frames(cams, ptrs)
        t = []
        for _ in range(7):
            gpu.launch_frames(cams, ptrs)
            t.append(gpu.last_kernel_ms())
        rows.append((F, float(np.median(t))))
        print(mode, F, round(rows[-1][1], 4), "ms", round(rows[-1][1] / F, 4), "ms/frame", flush=True)
    F_ = np.array([r[0] for r in rows if r[0] >= 2], dtype=float)
    T_ = np.array([r[1] for r in rows if r[0] >= 2])
    s, X = np.polyfit(F_, T_, 1)
    res[mode] = {"ms": {str(F): round(T, 4) for F, T in rows}, "fit_ms_per_frame": round(float(s), 4),
                 "fit_launch_ms": round(float(X), 4)}
print(json.dumps(res), flush=True)
