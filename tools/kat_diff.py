"""Diff map of a KAT scene against its golden image (dev tool)."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, "my-raytracer_amd")
sys.path.insert(0, "tests")
import kat_scenes  # noqa: E402
import rtamd  # noqa: E402

name, spp = sys.argv[1], int(sys.argv[2])
g = np.load(Path("tests/golden") / f"kat_{name}_spp{spp}.npz")
tmp = Path("gpurun_out/kat_tmp")
tmp.mkdir(parents=True, exist_ok=True)
hs = rtamd.HostScene.load(kat_scenes.write(tmp, name))
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
p = hs.render_params(0, 0, spp)
p.out_format = rtamd.RT_OUT_RGB_F64
for rep in range(3):
    img, st = dev.render(p)
    d = np.abs(img - g["image"]).max(axis=2)
    print("rep", rep, "counts", [st.primary_rays, st.shadow_rays, st.reflection_rays], "golden", list(g["counts"]))
    for row in d:
        print(" ".join("X" if v > 1e-9 else "." for v in row))
