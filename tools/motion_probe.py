"""How much could motion compensation of the one-frame cost order gain? (dev tool, under gpurun)

The library orders a one-frame launch by the per-tile costs of the launch two before it on the
stream.  Over an animation those costs are two frames stale.  This probe renders the
driver-shape orbit (0.12 rad over 20 frames, office 1080p) twice:
  stale:   v0, v1, v2, ...        -- view k ordered by the costs of view k-2 (the library's case)
  perfect: v0, v0, v0, v1, v1, v1, ... -- the third launch of each view is ordered by the costs of
           the same view (what an exact motion compensation could at best reach)
and prints the median kernel time of the timed launches of each (the same views in both).
"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(1920, 1080, 1)
out = torch.zeros((1080, 1920, 3), device="cuda")
views = [rtamd.camera_orbit(p, 0.12 * (f / 19 - 0.5)) for f in range(40)]
rounds = {"stale": [], "perfect": []}
for r in range(3):
    for _ in range(4):
        gpu.launch(views[0], out.data_ptr())
    stale = []
    for k, v in enumerate(views):
        gpu.launch(v, out.data_ptr())
        if k >= 4:
            stale.append(gpu.last_kernel_ms())
    perfect = []
    for k, v in enumerate(views):
        for rep in range(3):
            gpu.launch(v, out.data_ptr())
        if k >= 4:
            perfect.append(gpu.last_kernel_ms())
    rounds["stale"].append(float(np.median(stale)))
    rounds["perfect"].append(float(np.median(perfect)))
    print(json.dumps({"round": r, "stale_ms": rounds["stale"][-1], "perfect_ms": rounds["perfect"][-1]}), flush=True)
s, q = float(np.median(rounds["stale"])), float(np.median(rounds["perfect"]))
print(json.dumps({"stale_ms": s, "perfect_ms": q, "gain_bound": round(1 - q / s, 4),
                  "note": "perfect = each view ordered by its own costs: the most a motion-compensated order could "
                          "recover"}), flush=True)
