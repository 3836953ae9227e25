"""Config 3 (4K, 4x4 spp): one-frame launches of three views of the bench's camera orbit against
16-frame launches (orbit and identical views), kernel ms per frame (dev tool, under gpurun)."""
import json
import sys

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

W, H, S, F = 3840, 2160, 4, 16
host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(W, H, S)
cams = [rtamd.camera_orbit(p, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
out = [torch.zeros((H, W, 3), device="cuda") for _ in range(F)]
res = {}
for rep in range(2):
    for k in (0, 8, 15):
        gpu.launch(cams[k], out[0].data_ptr())
        res.setdefault(f"single_view{k}", []).append(gpu.last_kernel_ms())
    gpu.launch_frames(cams, [o.data_ptr() for o in out])
    res.setdefault("batch16_orbit", []).append(gpu.last_kernel_ms() / F)
    gpu.launch_frames([cams[0]] * F, [o.data_ptr() for o in out])
    res.setdefault("batch16_view0", []).append(gpu.last_kernel_ms() / F)
print(json.dumps({k: round(min(v), 3) for k, v in res.items()}), flush=True)
