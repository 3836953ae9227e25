"""Config 5 on one GPU (dev tool): office 7680x4320, 64 spp (8x8 stratified), the row shard
rank 0 of 8 renders (16-row stripes), one launch; prints its time and rays/s."""
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(7680, 4320, 8)
p.stripe_height, p.stripe_count, p.stripe_index = 16, 8, 0
rows = rtamd.rows_in_shard(p)
out = torch.zeros((rows, 7680, 3), device="cuda")
st = gpu.launch(p, out.data_ptr(), stats=True)
rays = st.primary_rays + st.shadow_rays + st.reflection_rays
ms = []
for _ in range(3):
    gpu.launch(p, out.data_ptr(), stats=True)
    ms.append(gpu.last_kernel_ms())
m = float(np.median(ms))
print(f"config 5 shard 0/8: rows {rows}, rays {rays}, {m:.1f} ms, {rays / m / 1e3:.0f} Mrays/s "
      f"(x8 GPUs: full 8K 64spp frame in {m:.1f} ms + gather)", flush=True)
