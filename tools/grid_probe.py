"""Frame time vs persistent-grid size (dev tool): one frame per launch and 32 frames per
launch, office 1080p, with at most k persistent blocks per CU (blocks_per_cu upload option).
usage: python tools/grid_probe.py k"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
K = int(sys.argv[1]) if len(sys.argv) > 1 else 0
gpu = rtamd.DeviceScene(host, 0, blocks_per_cu=K)
p = host.render_params(1920, 1080, 1)
for F in (1, 32):
    outs = [torch.zeros((1080, 1920, 3), device="cuda") for _ in range(F)]
    gpu.launch_frames(p, [o.data_ptr() for o in outs], stats=True)
    ms = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gpu.launch_frames(p, [o.data_ptr() for o in outs])
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    m = float(np.median(ms))
    print(f"blocks/CU {K or 'max'} F={F}: {m:.3f} ms, {m / F:.4f} ms/frame", flush=True)
