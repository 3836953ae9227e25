"""Does the order the work queue meets the image in change the one-frame time? (dev tool, under
gpurun)  Renders the office frame with the camera as given, flipped vertically and flipped
horizontally (the same rays, met in a different order) and prints median single-frame kernel ms."""
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
out = torch.zeros((1080, 1920, 3), device="cuda")


def flipped(axis):
    q = rtamd.abi.RenderParams.from_buffer_copy(p)
    c = q.camera
    d = c.y_dir if axis == "v" else c.x_dir
    n = c.height if axis == "v" else c.width
    for k in range(3):
        c.lower_left[k] += n * d[k]
        d[k] = -d[k]
    return q


res = {}
for name, q in [("as_given", p), ("flip_v", flipped("v")), ("flip_h", flipped("h"))] * 2:
    for _ in range(3):
        gpu.launch(q, out.data_ptr())
    t = []
    for _ in range(20):
        gpu.launch(q, out.data_ptr())
        t.append(gpu.last_kernel_ms())
    res.setdefault(name, []).append(float(np.median(t)))
print(json.dumps({k: round(float(np.mean(v)), 4) for k, v in res.items()}), flush=True)
