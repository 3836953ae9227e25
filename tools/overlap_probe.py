"""Throughput of back-to-back frames on one stream vs alternating two streams with
two device scenes (independent launch state) -- does the per-launch drain hide? (dev tool)"""
import sys
import time

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

w, h = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (1920, 1080)))
K = 20
host = rtamd.HostScene.generate("office")
host.prepare()
scenes = [rtamd.DeviceScene(host, 0) for _ in range(3)]
p = host.render_params(w, h, 1)
st = scenes[0].launch(p, torch.zeros(h * w * 3, device="cuda").data_ptr(), stats=True)
rays = st.primary_rays + st.shadow_rays + st.reflection_rays
for nstreams in (1, 2, 3):
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    bufs = [torch.zeros(h * w * 3, device="cuda") for _ in range(nstreams)]
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            i = k % nstreams
            scenes[i].launch(p, bufs[i].data_ptr(), stats=False, stream=streams[i].cuda_stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
    print(f"{w}x{h} streams {nstreams}: {dt*1e3:.3f} ms/frame  {rays/dt/1e6:.0f} Mrays/s", flush=True)
