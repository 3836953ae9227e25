"""Host/device timing of the batched adaptive path (dev tool, under gpurun): wall time of the
launch calls vs HIP-event time, per batch size."""
import sys
import time

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

host = rtamd.HostScene.generate("office")
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(1920, 1080, 1)
for F in (1, 8, 32):
    cams = [rtamd.camera_orbit(p, 0.12 * (f / max(F - 1, 1) - 0.5)) for f in range(F)]
    p64 = []
    for c in cams:
        q = rtamd.abi.RenderParams.from_buffer_copy(c)
        q.out_format = rtamd.RT_OUT_RGB_F64
        p64.append(q)
    prim = torch.zeros((F, 1080, 1920, 3), dtype=torch.float64, device="cuda")
    out = torch.zeros((F, 1080, 1920, 3), dtype=torch.float32, device="cuda")
    for it in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        gpu.launch_frames(p64, [prim[f].data_ptr() for f in range(F)])
        e1.record()
        t1 = time.perf_counter()
        gpu.launch_adaptive_frames(cams, [prim[f].data_ptr() for f in range(F)], [out[f].data_ptr() for f in range(F)])
        e2.record()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(f"F={F} it{it}: host primary {1e3*(t1-t0):.2f} ms, host adaptive {1e3*(t2-t1):.2f} ms, wall {1e3*(t3-t0):.2f} ms; "
              f"gpu primary {e0.elapsed_time(e1):.2f} ms, adaptive {e1.elapsed_time(e2):.2f} ms "
              f"({(e0.elapsed_time(e2))/F:.3f} ms/frame)", flush=True)
