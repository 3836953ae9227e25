"""Can another kernel run beside the persistent render kernel? (dev tool, under gpurun)  Stream A
renders a 32-frame launch; stream B, enqueued right after, copies 1 GB device to device (a
stand-in for the RCCL gather of the previous launch).  Prints, per grid_spare upload option, when B
ends relative to A's start and end (ms)."""
import json
import os
import sys

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(1920, 1080, 1)
F = 32
out = [torch.zeros((1080, 1920, 3), device="cuda") for _ in range(F)]
cams = [rtamd.camera_orbit(p, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
x = torch.ones(256 * 1024 * 1024, device="cuda")
y = torch.empty_like(x)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
res = {}
for spare in [0, 4, 16, 64, 0, 4, 16, 64]:
    gpu = rtamd.DeviceScene(host, 0, grid_spare=spare)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    with torch.cuda.stream(sa):
        ev[0].record(sa)
        gpu.launch_frames(cams, [o.data_ptr() for o in out], stream=sa.cuda_stream)
        ev[1].record(sa)
    with torch.cuda.stream(sb):
        sb.wait_event(ev[0])
        ev[2].record(sb)
        y.copy_(x)
        ev[3].record(sb)
    torch.cuda.synchronize()
    a_end = ev[0].elapsed_time(ev[1])
    b_end = ev[0].elapsed_time(ev[3])
    # alone: the copy by itself
    with torch.cuda.stream(sb):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sb); y.copy_(x); e1.record(sb)
    torch.cuda.synchronize()
    res.setdefault(spare, []).append((round(a_end, 3), round(b_end, 3), round(e0.elapsed_time(e1), 3)))
print(json.dumps({str(k): v for k, v in res.items()}), flush=True)
