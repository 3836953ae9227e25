"""Kernel time for small frames (dev tool): exposes per-launch fixed costs."""
import sys

import numpy as np

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
for w, h in [(8, 8), (64, 8), (64, 64), (128, 128), (256, 256), (512, 512), (1024, 512), (1920, 1080)]:
    p = host.render_params(w, h, 1)
    _, st = gpu.render(p)
    ms = []
    for _ in range(7):
        gpu.render(p)
        ms.append(gpu.last_kernel_ms())
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    print(f"{w}x{h}: {np.median(ms):.3f} ms (min {min(ms):.3f})  rays {rays}", flush=True)
