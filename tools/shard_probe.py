"""Per-rank launch time of the N-GPU bench, emulated on one GPU (dev tool).

Rank 0's share of N-way row striping (16-row stripes, stripe s -> rank s mod N), 64 frames per
launch as bench.py does; prints the launch time and the whole-job rate it implies if every
rank ran as fast (the gather is not included)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
FA = sys.argv[1] if len(sys.argv) > 1 else "auto"
for n in (1, 2, 4, 8):
    F = 64 if FA == "auto" else int(FA)
    p = host.render_params(1920, 1080, 1)
    p.stripe_height, p.stripe_count, p.stripe_index = 16, n, 0
    rows = rtamd.rows_in_shard(p)
    outs = [torch.zeros((rows, 1920, 3), device="cuda") for _ in range(F)]
    st = gpu.launch_frames(p, [o.data_ptr() for o in outs], stats=True)
    rays_rank = (st.primary_rays + st.shadow_rays + st.reflection_rays) / F
    ms = []
    for _ in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gpu.launch_frames(p, [o.data_ptr() for o in outs])
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    m = float(np.median(ms[2:]))
    print(f"N={n}: rank-0 rows {rows}, {F} frames/launch {m:.3f} ms = {m / F:.3f} ms/frame, rank rays/frame "
          f"{rays_rank:.0f}; implied whole-job {rays_rank * n * F / m / 1e3:.0f} Mrays/s", flush=True)
