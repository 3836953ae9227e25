"""Which CU-mask patterns let a gather-shaped kernel run beside the persistent render grid? (dev
tool, under gpurun).  For each pattern of freed CU-mask bits, the office 32-frame launch runs on a
stream created with that mask (grid shrunk by 4 blocks per freed CU) while a 256-VGPR / 37.6-KB-LDS
copy kernel (tools/heavy_copy.hip, RCCL's resource shape) is enqueued on another stream; prints the
render time and when the copy ended (ms from the render's start; copy alone ~0.5 ms)."""
import ctypes as C
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

hip = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
hip.hipExtStreamCreateWithCUMask.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]
hip.hipExtStreamGetCUMask.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
lib = C.CDLL("tools/libheavy_copy.so")
lib.heavy_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
host = rtamd.HostScene.generate("office")
host.prepare()
p = host.render_params(1920, 1080, 1)
F = 32
out = [torch.zeros((1080, 1920, 3), device="cuda") for _ in range(F)]
cams = [rtamd.camera_orbit(p, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
x = torch.ones(24 * 1024 * 1024, device="cuda")
y = torch.empty_like(x)
sb = torch.cuda.Stream()

patterns = {
    "none": [],
    "bits0-7": list(range(8)),
    "bits0-15": list(range(16)),
    "bits0-31": list(range(32)),
    "stride32": [32 * k + 31 for k in range(8)],
    "stride8_first4": [8 * k for k in range(32)][:16],
    "every8": [8 * k for k in range(32)],
    "bits_mod32_0-1": [32 * k + j for k in range(8) for j in range(2)],
}
res = {}
for name, freed in patterns.items():
    words = [0] * ((n_cu + 31) // 32)
    for c in range(n_cu):
        if c not in freed:
            words[c // 32] |= 1 << (c % 32)
    arr = (C.c_uint32 * len(words))(*words)
    s = C.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(C.byref(s), len(words), arr) == 0
    got = (C.c_uint32 * len(words))()
    hip.hipExtStreamGetCUMask(s, len(words), got)
    sa = torch.cuda.ExternalStream(s.value)
    gpu = rtamd.DeviceScene(host, 0, grid_spare=4 * len(freed))
    r = {"render_with_copy": [], "copy_end": [], "render_alone": []}
    for rep in range(3):
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        ev[0].record(sa)
        gpu.launch_frames(cams, [o.data_ptr() for o in out], stream=s.value)
        ev[1].record(sa)
        sb.wait_event(ev[0])
        lib.heavy_copy(x.data_ptr(), y.data_ptr(), x.numel() * 4, 16, C.c_void_p(sb.cuda_stream))
        ev[2].record(sb)
        torch.cuda.synchronize()
        ev[3].record(sa)
        gpu.launch_frames(cams, [o.data_ptr() for o in out], stream=s.value)
        ev[4].record(sa)
        torch.cuda.synchronize()
        r["render_with_copy"].append(ev[0].elapsed_time(ev[1]))
        r["copy_end"].append(ev[0].elapsed_time(ev[2]))
        r["render_alone"].append(ev[3].elapsed_time(ev[4]))
    res[name] = {k: round(statistics.median(v), 3) for k, v in r.items()}
    res[name]["mask_words"] = [hex(w) for w in got]
    print(name, res[name], flush=True)
    gpu.close()
print(json.dumps(res), flush=True)
