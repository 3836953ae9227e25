"""Traversal diagnostics per frame against frames per launch (identical views, 4-wide stats
variant), for W H S (dev tool, under gpurun)."""
import json
import sys

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

W, H, S = (int(x) for x in sys.argv[1:4])
host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(W, H, S)
p.flags = rtamd.RT_FLAG_WIDE_STATS
out = [torch.zeros((H, W, 3), device="cuda") for _ in range(16)]
res = {}
for F in (1, 2, 16):
    st = gpu.launch_frames([p] * F, [o.data_ptr() for o in out[:F]], stats=True) if F > 1 else \
        gpu.launch(p, out[0].data_ptr(), stats=True)
    d = gpu.debug_counters()
    keys = ("node_iters", "node_lanes", "leaf_iters", "leaf_lanes", "trav_rounds", "outer_iters")
    r = {k: round(d[k] / F / 1e6, 4) for k in keys if k in d}
    r["node_visits_M"] = round(st.node_visits / F / 1e6, 3)
    r["rays_M"] = round((st.primary_rays + st.shadow_rays + st.reflection_rays) / F / 1e6, 3)
    r["ms_per_frame"] = round(gpu.last_kernel_ms() / F, 3)
    res[F] = r
print(json.dumps(res), flush=True)
