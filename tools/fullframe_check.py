"""Whole-frame parity records for the large BASELINE configs (dev tool, under gpurun): config 3
(office proxy 3840x2160, 16 spp) compared pixel for pixel over the WHOLE frame with the CPU oracle
(ordered traversal, which equals the reference-semantics render: tests/test_fuzz_oracle.py), ray
counts exact for the whole frame; config 5 (7680x4320, 64 spp) on every 32nd row (the GPU renders
the whole frame; the oracle those 135 rows), counts exact for the same rows through the 1-row
stripe path.  The oracle is the checker only.

usage: python tools/fullframe_check.py OUT.json
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

TOL64 = 1e-12
hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
orc = pyoracle.Oracle(hs.raw, hs)
res = {}

t0 = time.time()
p = hs.render_params(3840, 2160, 4)
p.out_format = rtamd.RT_OUT_RGB_F64
img, st = dev.render(p)
err3, oc3 = 0.0, [0, 0, 0]
for y0 in range(0, 2160, 108):   # chunks of rows, a progress line each (a silent run is taken as hung)
    yk = np.arange(y0, min(2160, y0 + 108))
    xy = np.stack(np.meshgrid(np.arange(3840), yk), -1).reshape(-1, 2).astype(np.int32)
    ref, cnt = orc.render_pixels(p, xy, pyoracle.MODE_ORDERED, threads=0)
    err3 = max(err3, float(np.abs(img[yk].reshape(-1, 3) - ref).max()))
    oc3 = [a + b for a, b in zip(oc3, (cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays))]
    print(json.dumps({"config3_rows_done": int(yk[-1] + 1), "max_abs_err": err3}), flush=True)
res["config3_whole_frame"] = {
    "pixels": 3840 * 2160, "max_abs_err": err3,
    "counts_gpu": [st.primary_rays, st.shadow_rays, st.reflection_rays],
    "counts_oracle": oc3, "seconds": round(time.time() - t0, 1)}
print(json.dumps(res["config3_whole_frame"]), flush=True)

t0 = time.time()
p = hs.render_params(7680, 4320, 8)
p.out_format = rtamd.RT_OUT_RGB_F64
img, st = dev.render(p)
ys = np.arange(3, 4320, 32)
err, oc = 0.0, [0, 0, 0]
for k in range(0, len(ys), 15):   # chunks of rows, a progress line each
    yk = ys[k:k + 15]
    xy = np.stack(np.meshgrid(np.arange(7680), yk), -1).reshape(-1, 2).astype(np.int32)
    ref, cnt = orc.render_pixels(p, xy, pyoracle.MODE_ORDERED, threads=0)
    err = max(err, float(np.abs(img[yk].reshape(-1, 3) - ref).max()))
    oc = [a + b for a, b in zip(oc, (cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays))]
    print(json.dumps({"config5_rows_done": int(k + len(yk)), "max_abs_err": err}), flush=True)
q = rtamd.abi.RenderParams.from_buffer_copy(p)
q.stripe_height, q.stripe_count, q.stripe_index = 1, 32, 3
img32, st32 = dev.render(q)
res["config5_every_32nd_row"] = {
    "rows": len(ys), "pixels": int(len(ys) * 7680), "max_abs_err": err,
    "stripe_rows_equal_whole_frame_rows": bool(np.array_equal(img32, img[ys])),
    "counts_gpu_rows": [st32.primary_rays, st32.shadow_rays, st32.reflection_rays],
    "counts_oracle_rows": oc,
    "primary_whole_frame": st.primary_rays, "seconds": round(time.time() - t0, 1)}
print(json.dumps(res["config5_every_32nd_row"]), flush=True)
ok = all(r["max_abs_err"] <= TOL64 for r in res.values()) and \
    res["config3_whole_frame"]["counts_gpu"] == res["config3_whole_frame"]["counts_oracle"] and \
    res["config5_every_32nd_row"]["counts_gpu_rows"] == res["config5_every_32nd_row"]["counts_oracle_rows"] and \
    res["config5_every_32nd_row"]["stripe_rows_equal_whole_frame_rows"] and \
    res["config5_every_32nd_row"]["primary_whole_frame"] == 7680 * 4320 * 64
res["ok"] = ok
Path(sys.argv[1]).write_text(json.dumps(res, indent=1))
print(json.dumps({"ok": ok}), flush=True)
sys.exit(0 if ok else 1)
