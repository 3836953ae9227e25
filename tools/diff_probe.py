"""GPU vs oracle difference map of one frame (dev tool, run under gpurun).
usage: python tools/diff_probe.py [W H]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1080)
hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
orc = pyoracle.Oracle(hs.raw, hs)
p = hs.render_params(W, H, 1)
ref, cnt = orc.render(p, pyoracle.MODE_REFERENCE)
p.out_format = rtamd.RT_OUT_RGB_F64
img, st = dev.render(p)
runs = [dev.render(p)[0] for _ in range(4)]
img2 = runs[0]
d = np.abs(img - ref).max(-1)
for r in runs:
    d = np.maximum(d, np.abs(r - ref).max(-1))
bad = np.argwhere(d > 1e-12)
print("counts gpu", st.primary_rays, st.shadow_rays, st.reflection_rays, "oracle", cnt.primary_rays, cnt.shadow_rays,
      cnt.reflection_rays)
print("bad pixels", len(bad), "max", d.max(), "gpu deterministic", np.array_equal(img, img2),
      "run-to-run diff pixels", int((np.abs(img - img2).max(-1) > 0).sum()))
for y, x in bad[:25]:
    print(f"({x},{y}) gpu {img[y, x]} ref {ref[y, x]}")
if len(bad):
    ys, xs = bad[:, 0], bad[:, 1]
    print("rows", np.unique(ys)[:40], "x range", xs.min(), xs.max())
    print("x%8", np.bincount(xs % 8, minlength=8), "y%8", np.bincount(ys % 8, minlength=8))
