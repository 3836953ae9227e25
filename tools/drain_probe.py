"""Per-launch fixed cost vs path length (dev tool): launch time for 1 and 16 frames per launch on
the office frame at max_depth 5 (mirror chains) and 0 (no reflection rays)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
for depth in (5, 0):
    res = {}
    for F in (1, 16):
        p = host.render_params(1920, 1080, 1)
        p.max_depth = depth
        outs = [torch.zeros((1080, 1920, 3), device="cuda") for _ in range(F)]
        st = gpu.launch_frames(p, [o.data_ptr() for o in outs], stats=True)
        ms = []
        for _ in range(9):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gpu.launch_frames(p, [o.data_ptr() for o in outs])
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        res[F] = float(np.median(ms[2:]))
    per = (res[16] - res[1]) / 15
    print(f"depth {depth}: 1 frame {res[1]:.3f} ms, 16 frames {res[16]:.3f} ms -> {per:.3f} ms/frame + "
          f"{res[1] - per:.3f} ms per launch", flush=True)
