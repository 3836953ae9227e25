"""Per-frame kernel time against frames per launch (identical views), for a workload given as
W H S [scene [tris]] (dev tool, under gpurun).  "shared_out" launches write every frame into the
same buffer (identical frames, so the same bytes): isolates the cost of scattering the output
over F buffers."""
import json
import sys

import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

W, H, S = (int(x) for x in sys.argv[1:4])
scene = sys.argv[4] if len(sys.argv) > 4 else "office"
gen = {"n_triangles": int(sys.argv[5])} if len(sys.argv) > 5 else {}
host = rtamd.HostScene.generate(scene, **gen)
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(W, H, S)
Fs = [int(x) for x in __import__('os').environ.get('FS', '1,2,4,8,16').split(',')]
out = [torch.zeros((H, W, 3), device="cuda") for _ in range(max(Fs))]
res = {}
for rep in range(2):
    for F in Fs:
        if F == 1:
            gpu.launch(p, out[0].data_ptr())
        else:
            gpu.launch_frames([p] * F, [o.data_ptr() for o in out[:F]])
        res.setdefault(F, []).append(gpu.last_kernel_ms() / F)
        if F > 1:
            gpu.launch_frames([p] * F, [out[0].data_ptr()] * F)
            res.setdefault(f"{F}_shared_out", []).append(gpu.last_kernel_ms() / F)
print(json.dumps({str(k): round(min(v), 3) for k, v in res.items()}), flush=True)
