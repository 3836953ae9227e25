"""PCIe-inclusive rate of the host-buffer boundary (dev tool, GPU): rt_render_to_host of the office
1080p frame (render + device-to-host copy of the finished fp32 frame, synchronous, no stats),
into pageable (numpy) and pinned (torch pin_memory) host memory, against the device-buffer launch.
Consecutive orbit views, one frame per call (the reference's use, mytracer.cpp:123-159).

usage: python tools/host_rate_probe.py [calls]
"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "my-raytracer_amd"))
import rtamd  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
base = hs.render_params(1920, 1080, 1)
cams = [rtamd.camera_orbit(base, 0.12 * (f / 19 - 0.5)) for f in range(20)]
_, st = dev.render(cams[0])
rays = st.primary_rays + st.shadow_rays + st.reflection_rays
lib = rtamd.hip_lib()
page = np.zeros((1080, 1920, 3), dtype=np.float32)
pinned = torch.empty((1080, 1920, 3), dtype=torch.float32, pin_memory=True)
devbuf = torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda")


def run(kind):
    for i in range(N + 5):
        if i == 5:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        c = cams[i % 20]
        if kind == "device":
            dev.launch(c, devbuf.data_ptr())
        else:
            ptr = page.ctypes.data_as(C.c_void_p) if kind == "pageable" else C.c_void_p(pinned.data_ptr())
            rc = lib.rt_render_to_host(dev._h, C.byref(c), ptr, None)
            assert rc == 0, lib.rt_last_error()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / N * 1e3
    return {"buffer": kind, "ms_per_frame": round(ms, 4), "mrays_s": round(rays / ms / 1e3, 1)}


for kind in ("device", "pageable", "pinned", "device"):
    print(json.dumps(run(kind)), flush=True)
print(json.dumps({"rays_per_frame": rays, "frame_bytes": 1080 * 1920 * 3 * 4}), flush=True)
