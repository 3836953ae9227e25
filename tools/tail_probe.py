"""Kernel time vs work size at fixed coherence (dev tool): renders 1/k of the
office frame as interleaved 16-row stripes and fits T(k) = W/k + tau."""
import sys

import numpy as np

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

w, h, spp = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (1920, 1080, 1)))
host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
res = []
for k in (1, 2, 4, 8, 16):
    p = host.render_params(w, h, spp)
    p.stripe_height, p.stripe_count, p.stripe_index = 16, k, 0
    _, st = gpu.render(p)
    ms = []
    for _ in range(7):
        gpu.render(p)
        ms.append(gpu.last_kernel_ms())
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    m = float(np.median(ms))
    res.append((k, m, rays))
    print(f"{w}x{h} spp{spp*spp} 1/{k}: {m:.3f} ms  rays {rays}  {rays / m / 1e3:.1f} Mrays/s", flush=True)
k = np.array([r[0] for r in res], float)
t = np.array([r[1] for r in res])
A = np.stack([1 / k, np.ones_like(k)], 1)
(W, tau), *_ = np.linalg.lstsq(A, t, rcond=None)
print(f"fit: T = {W:.3f}/k + {tau:.3f} ms  (steady-state {res[0][2] / W / 1e3:.1f} Mrays/s)")
