"""Kernel time vs reflection depth / light count (dev tool): is the per-launch
fixed cost the longest reflection chain?"""
import sys

import numpy as np

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
for w, h in [(8, 8), (256, 256), (1920, 1080)]:
    for depth in (0, 1, 2, 5):
        for nl in (1, 2):
            p = host.render_params(w, h, 1)
            p.max_depth = depth
            p.n_lights = min(nl, p.n_lights)
            _, st = gpu.render(p)
            ms = []
            for _ in range(5):
                gpu.render(p)
                ms.append(gpu.last_kernel_ms())
            rays = st.primary_rays + st.shadow_rays + st.reflection_rays
            print(f"{w}x{h} depth {depth} lights {p.n_lights}: {np.median(ms):.3f} ms  rays {rays} "
                  f"(refl {st.reflection_rays})  {rays / np.median(ms) / 1e3:.0f} Mrays/s", flush=True)
