"""Can a gather kernel run beside the persistent render kernel? (dev tool, under gpurun)

Stream A renders a 32-frame office 1080p launch; stream B, enqueued right after, runs a stand-in
for RCCL's gather kernel (tools/heavy_copy.hip: 256 VGPRs per wave, 37.6 KB LDS per block, like
ncclDevKernel_Generic on gfx950) copying 96 MB -- 4x the fp32 RGB a rank-0 gather receives per 1080p
frame at N = 8.  Per upload option (grid_spare: block slots left free; reserve_cus: whole CUs left
free through a CU-masked launch stream), prints when B ends relative to A's start, A's own end, and
B's time alone (ms), medians over repeats.  B ending long before A means the gather overlaps the
render."""
import ctypes as C
import json
import statistics
import sys

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

lib = C.CDLL("tools/libheavy_copy.so")
lib.heavy_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
host = rtamd.HostScene.generate("office")
host.prepare()
p = host.render_params(1920, 1080, 1)
F = 32
out = [torch.zeros((1080, 1920, 3), device="cuda") for _ in range(F)]
cams = [rtamd.camera_orbit(p, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
x = torch.ones(24 * 1024 * 1024, device="cuda")
y = torch.empty_like(x)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
res = {}
configs = [("base", {}), ("grid_spare=64", {"grid_spare": 64})] + \
    [(f"reserve_cus={r}", {"reserve_cus": r}) for r in (int(x) for x in (sys.argv[1:] or ["8", "16"]))]
scenes = {name: rtamd.DeviceScene(host, 0, **kw) for name, kw in configs}
for rep in range(3):
    for name, _ in configs:
        gpu = scenes[name]
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        with torch.cuda.stream(sa):
            ev[0].record(sa)
            gpu.launch_frames(cams, [o.data_ptr() for o in out], stream=sa.cuda_stream)
            ev[1].record(sa)
        with torch.cuda.stream(sb):
            sb.wait_event(ev[0])
            lib.heavy_copy(x.data_ptr(), y.data_ptr(), x.numel() * 4, 16, C.c_void_p(sb.cuda_stream))
            ev[3].record(sb)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(sb):
            e0.record(sb)
            lib.heavy_copy(x.data_ptr(), y.data_ptr(), x.numel() * 4, 16, C.c_void_p(sb.cuda_stream))
            e1.record(sb)
        # the render alone
        with torch.cuda.stream(sa):
            ev[2].record(sa)
            gpu.launch_frames(cams, [o.data_ptr() for o in out], stream=sa.cuda_stream)
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record(sa)
        torch.cuda.synchronize()
        r = res.setdefault(name, {"render_with_copy": [], "copy_end": [], "copy_alone": [], "render_alone": []})
        r["render_with_copy"].append(ev[0].elapsed_time(ev[1]))
        r["copy_end"].append(ev[0].elapsed_time(ev[3]))
        r["copy_alone"].append(e0.elapsed_time(e1))
        r["render_alone"].append(ev[2].elapsed_time(e2))
        print(name, rep, {k: round(v[-1], 3) for k, v in r.items()}, flush=True)
print(json.dumps({n: {k: round(statistics.median(v), 3) for k, v in r.items()} for n, r in res.items()}), flush=True)
