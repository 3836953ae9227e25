"""Samples of a pixel on one lane vs on neighbouring lanes (dev tool, under gpurun).

The production kernel keeps a pixel on one lane through all n x n samples (the running sum in the
path state); the adaptive pass's list mode (rt_launch_adaptive) runs every (pixel, sample) pair as
its own work item, a pixel's samples on neighbouring lanes, and sums them in (si, sj) order
afterwards.  With threshold -1 every interior pixel is selected, so the list-mode launch renders
the same frame at subp x subp samples: its kernel time per ray against the production launch's at
spp = subp bounds what the neighbouring-lane layout buys in coherence (the sample buffer's writes
included).  Pixels: the interior of the two images must agree bit for bit.

usage: python tools/spp_modes.py [W H SUBP REPS]
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
import rtamd  # noqa: E402

W, H, N, REPS = (int(x) for x in (sys.argv[1:5] if len(sys.argv) >= 5 else (3840, 2160, 4, 3)))
hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
p = hs.render_params(W, H, N)
p.out_format = rtamd.RT_OUT_RGB_F64
p.flags = rtamd.abi.RT_FLAG_NATURAL_ORDER
p1 = hs.render_params(W, H, 1)
p1.out_format = rtamd.RT_OUT_RGB_F64
p1.flags = rtamd.abi.RT_FLAG_NATURAL_ORDER
full = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
prim = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
lst = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
res = {"workload": f"office_proxy {W}x{H} {N * N} spp", "lane_per_pixel_ms": [], "lanes_per_sample_ms": []}
st_full = dev.launch(p, full.data_ptr(), stats=True)
dev.launch(p1, prim.data_ptr(), stats=True)
st_list, nsel = dev.launch_adaptive(p1, prim.data_ptr(), lst.data_ptr(), N, -1.0, stats=True)
for _ in range(REPS):
    dev.launch(p, full.data_ptr())
    res["lane_per_pixel_ms"].append(round(dev.last_kernel_ms(), 3))
    dev.launch_adaptive(p1, prim.data_ptr(), lst.data_ptr(), N, -1.0)
    res["lanes_per_sample_ms"].append(round(dev.last_kernel_ms(), 3))   # the list-mode render launch
torch.cuda.synchronize()
a, b = full.cpu().numpy(), lst.cpu().numpy()
rays = lambda s: s.primary_rays + s.shadow_rays + s.reflection_rays  # noqa: E731
res.update({
    "rays_lane_per_pixel": rays(st_full), "rays_lanes_per_sample": rays(st_list), "pixels_selected": nsel,
    "interior_bit_identical": bool(np.array_equal(a[1:-1, 1:-1], b[1:-1, 1:-1])),
    "grays_lane_per_pixel": round(rays(st_full) / (min(res["lane_per_pixel_ms"]) * 1e-3) / 1e9, 3),
    "grays_lanes_per_sample": round(rays(st_list) / (min(res["lanes_per_sample_ms"]) * 1e-3) / 1e9, 3),
})
print(json.dumps(res), flush=True)
