"""Parity over the driver's animation (dev tool, under gpurun): the 20 orbit views of bench.py's
driver shape (office 1080p, 0.12 rad over 20 frames), rendered by the production kernel as ONE
20-frame launch and as 20 consecutive one-frame launches (the library's cost-ordered default), both
fp64, against the CPU oracle's reference-semantics render of every view: pixels within 1e-12, ray
counts exact (summed over the launch).  The oracle is the checker only.

usage: python tools/view_sweep.py [frames] OUT.json
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 2 else 20
out_path = sys.argv[-1]
TOL64 = 1e-12
t0 = time.time()
hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
orc = pyoracle.Oracle(hs.raw, hs)
base = hs.render_params(1920, 1080, 1)
base.out_format = rtamd.RT_OUT_RGB_F64
cams = [rtamd.camera_orbit(base, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
for c in cams:
    c.out_format = rtamd.RT_OUT_RGB_F64
bufs = [torch.zeros((1080, 1920, 3), dtype=torch.float64, device="cuda") for _ in range(F)]
st_multi = dev.launch_frames(cams, [b.data_ptr() for b in bufs], stats=True)
multi = [b.cpu().numpy() for b in bufs]
single, single_counts = [], [0, 0, 0]
for c in cams:   # consecutive one-frame launches on one stream: cost-ordered from the third
    st = dev.launch(c, bufs[0].data_ptr(), stats=True)
    single.append(bufs[0].cpu().numpy())
    single_counts = [a + b for a, b in zip(single_counts, (st.primary_rays, st.shadow_rays, st.reflection_rays))]
rows, ref_counts, worst = [], [0, 0, 0], 0.0
for f, c in enumerate(cams):
    ref, cnt = orc.render(c, pyoracle.MODE_REFERENCE)
    ref_counts = [a + b for a, b in zip(ref_counts, (cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays))]
    em = float(np.abs(multi[f] - ref).max())
    es = float(np.abs(single[f] - ref).max())
    worst = max(worst, em, es)
    rows.append({"view": f, "multi_max_abs_err": em, "single_max_abs_err": es,
                 "multi_equals_single": bool(np.array_equal(multi[f], single[f]))})
    print(json.dumps(rows[-1]), flush=True)
mc = [st_multi.primary_rays, st_multi.shadow_rays, st_multi.reflection_rays]
summary = {"views": F, "worst_max_abs_err": worst, "tolerance": TOL64,
           "counts_oracle": ref_counts, "counts_multi_frame_launch": mc, "counts_one_frame_launches": single_counts,
           "ok": worst <= TOL64 and mc == ref_counts and single_counts == ref_counts and all(r["multi_equals_single"] for r in rows),
           "seconds": round(time.time() - t0, 1)}
Path(out_path).write_text(json.dumps({"summary": summary, "rows": rows}, indent=1))
print(json.dumps(summary), flush=True)
sys.exit(0 if summary["ok"] else 1)
