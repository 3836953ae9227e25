"""Host-buffer call rate (dev tool, under gpurun): the reference's call pattern -- one synchronous
frame per call, the image back in host memory (Raytracer::compute_image_cuda, mytracer.cpp:123-159)
-- through rt_render_to_host into page-locked and into pageable memory, beside one-frame launches
into a device buffer (launch + synchronise); and the reference's whole launch_compute_image_device
(primary + adaptive pass + copy back) through rt_render_adaptive_to_host.  Office proxy 1080p fp32, consecutive orbit views;
median ms per call over REPS calls.  RTAMD_HIP_LIB selects the library (A/B).

usage: python tools/host_rate.py [REPS]
"""
import ctypes as C
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
import rtamd  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 40
W, H = 1920, 1080
hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
lib = rtamd.hip_lib()
views = [rtamd.camera_orbit(hs.render_params(W, H, 1), 0.004 * k) for k in range(REPS)]
for v in views:
    v.out_format = rtamd.RT_OUT_RGB_F32
d_out = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
pinned = torch.zeros((H, W, 3), dtype=torch.float32).pin_memory()
pageable = np.zeros((H, W, 3), dtype=np.float32)


def timed(call):
    for v in views[:5]:   # warm-up (cost maps, staging buffer)
        call(v)
    torch.cuda.synchronize()
    ms = []
    for v in views:
        t0 = time.perf_counter()
        call(v)
        ms.append((time.perf_counter() - t0) * 1e3)
    return round(statistics.median(ms), 4)


def device(v):
    dev.launch(v, d_out.data_ptr())
    torch.cuda.synchronize()


def host(buf_ptr):
    def f(v):
        rc = lib.rt_render_to_host(dev._h, C.byref(v), C.c_void_p(buf_ptr), None)
        assert rc == 0, rc
    return f


def host_adaptive(buf_ptr):   # the reference's whole call: primary + adaptive pass + copy back
    def f(v):
        rc = lib.rt_render_adaptive_to_host(dev._h, C.byref(v), 4, 0.02, C.c_void_p(buf_ptr), None, None, None)
        assert rc == 0, rc
    return f


def d2h(v):   # the PCIe leg alone: a finished frame copied into page-locked memory
    pinned.copy_(d_out, non_blocking=True)
    torch.cuda.synchronize()


res = {"workload": f"office_proxy {W}x{H} 1 spp fp32, one frame per call", "reps": REPS,
       "lib": os.environ.get("RTAMD_HIP_LIB", "in-tree"),
       "device_buffer_ms": timed(device),
       "pinned_host_ms": timed(host(pinned.data_ptr())),
       "pageable_host_ms": timed(host(pageable.ctypes.data))}
# the host images (the last view) equal the device-buffer image of the same view
dev.launch(views[-1], d_out.data_ptr())
torch.cuda.synchronize()
ref = d_out.cpu().numpy()
res["pinned_equal"] = bool(np.array_equal(pinned.numpy(), ref))
res["pageable_equal"] = bool(np.array_equal(pageable, ref))
res.update({"d2h_copy_pinned_ms": timed(d2h), "frame_MB": round(W * H * 12 / 1e6, 2),
            "adaptive_pinned_host_ms": timed(host_adaptive(pinned.data_ptr())),
            "adaptive_pageable_host_ms": timed(host_adaptive(pageable.ctypes.data))})
print(json.dumps(res), flush=True)
