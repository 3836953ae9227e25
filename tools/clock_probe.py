"""Does sustained load lower the clock? (dev tool, under gpurun)  Config 3 (4K, 4x4 spp): 24
one-frame launches back to back, then a 16-frame launch, then 8 more one-frame launches; prints
every kernel time (ms)."""
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
out = [torch.zeros((H, W, 3), device="cuda") for _ in range(F)]
t = []
for _ in range(24):
    gpu.launch(p, out[0].data_ptr())
    t.append(round(gpu.last_kernel_ms(), 2))
gpu.launch_frames([p] * F, [o.data_ptr() for o in out])
b = round(gpu.last_kernel_ms() / F, 2)
t2 = []
for _ in range(8):
    gpu.launch(p, out[0].data_ptr())
    t2.append(round(gpu.last_kernel_ms(), 2))
print(json.dumps({"single_first24": t, "batch16_per_frame": b, "single_after": t2}), flush=True)
