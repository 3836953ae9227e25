"""One kernel library, office 1080p (dev tool, under gpurun; run by tools/ab_frame.py with
RTAMD_HIP_LIB set): median kernel time of single-frame launches and of 64-frame launches
(per frame), printed as one JSON line; single_call_ms: HIP events around the one-frame call.  RTAMD_AB_OPTS: upload options "key=value,..."."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "office"
gen = {"n_triangles": int(sys.argv[2])} if len(sys.argv) > 2 else {}
host = rtamd.HostScene.generate(scene, **gen)
host.prepare()
opts = dict(kv.split("=") for kv in os.environ.get("RTAMD_AB_OPTS", "").split(",") if kv)
gpu = rtamd.DeviceScene(host, 0, **{k: (float(v) if "." in v else int(v)) for k, v in opts.items()})
p = host.render_params(1920, 1080, 1)
out = [torch.zeros((1080, 1920, 3), device="cuda") for _ in range(64)]
for _ in range(5):
    gpu.launch(p, out[0].data_ptr())
single, call = [], []
for _ in range(30):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gpu.launch(p, out[0].data_ptr())
    e1.record()
    single.append(gpu.last_kernel_ms())
    torch.cuda.synchronize()
    call.append(e0.elapsed_time(e1))   # the whole call on the stream: set-up + kernel
# one-frame launches over consecutive views of the driver-shape animation (0.12 rad per 20 frames),
# the library's default cost order (frame i ordered by the costs of frame i - 2)
orbit = []
for f in range(34):
    gpu.launch(rtamd.camera_orbit(p, 0.12 * (f / 19 - 0.5)), out[0].data_ptr())
    if f >= 4:
        orbit.append(gpu.last_kernel_ms())
cams = [rtamd.camera_orbit(p, 0.12 * (f / 63 - 0.5)) for f in range(64)]
gpu.launch_frames(cams, [o.data_ptr() for o in out])
batch = []
for _ in range(3):
    gpu.launch_frames(cams, [o.data_ptr() for o in out])
    batch.append(gpu.last_kernel_ms() / 64)
print(json.dumps({"single_ms": float(np.median(single)), "single_p90": float(np.percentile(single, 90)),
                  "single_call_ms": float(np.median(call)), "single_orbit20_ms": float(np.median(orbit)),
                  "batched_ms_per_frame": float(np.median(batch))}), flush=True)
