"""Config 3 (4K, 4x4 spp) office, identical views, F frames per launch for 32 frames in total
(dev tool for rocprofv3 --pmc passes under gpurun).  usage: python tools/batch_pmc.py F"""
import sys

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

F = int(sys.argv[1])
W, H, S = 3840, 2160, 4
host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(W, H, S)
out = [torch.zeros((H, W, 3), device="cuda") for _ in range(F)]
ms = 0.0
for _ in range(32 // F):
    if F == 1:
        gpu.launch(p, out[0].data_ptr())
    else:
        gpu.launch_frames([p] * F, [o.data_ptr() for o in out])
    ms += gpu.last_kernel_ms()
print(f"F={F} per-frame {ms / 32:.3f} ms", flush=True)
