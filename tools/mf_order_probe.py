"""Work order inside a multi-frame launch (dev tool, GPU): the library renders F frames per launch
band-major -- tile row ty of every frame, then ty + 1 (item order (ty, frame, tx)).  This probe
times 20-frame office launches (driver-shape orbit views) with host-built orders through
rt_debug_set_tile_order against the natural order:
  identity   the natural order through the debug order array (control: the array's own cost)
  posmajor   (ty, tx, frame): one tile position of all F frames back to back
  rowpair    (ty // 2, frame, ty % 2, tx): two tile rows of a frame before the next frame
Pixels must not change.

usage: python tools/mf_order_probe.py [F] [reps] [rounds]
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "my-raytracer_amd"))
import rtamd  # noqa: E402
from rtamd import abi  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 20
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ROUNDS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
lib = rtamd.hip_lib()
tw, th = rtamd.tile_shape()
hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
base = hs.render_params(1920, 1080, 1)
cams = [rtamd.camera_orbit(base, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
bufs = [torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda") for _ in range(F)]
TX, TY = -(-1920 // tw), -(-1080 // th)
n = TX * TY * F


def lin(ty, f, tx):
    return (ty * F + f) * TX + tx


ty, f, tx = np.meshgrid(np.arange(TY), np.arange(F), np.arange(TX), indexing="ij")
orders = {"identity": lin(ty, f, tx).reshape(-1)}
ty2, tx2, f2 = np.meshgrid(np.arange(TY), np.arange(TX), np.arange(F), indexing="ij")
orders["posmajor"] = lin(ty2, f2, tx2).reshape(-1)
TYp = -(-TY // 2)
rows = []
for a in range(TYp):
    for fr in range(F):
        for b in range(2):
            y = 2 * a + b
            if y < TY:
                rows.append(lin(y, fr, np.arange(TX)))
orders["rowpair"] = np.concatenate(rows)
for k, o in orders.items():
    assert len(o) == n and len(np.unique(o)) == n, k
    orders[k] = o.astype(np.uint32)


def launch():
    dev.launch_frames(cams, [b.data_ptr() for b in bufs])


def timed():
    ms = []
    for _ in range(REPS):
        launch()
        torch.cuda.synchronize()
        ms.append(dev.last_kernel_ms())
    return float(np.median(ms))


def use(name):
    if name == "natural":
        lib.rt_debug_set_tile_order(dev._h, None, 0)
    else:
        o = orders[name]
        assert lib.rt_debug_set_tile_order(dev._h, o.ctypes.data_as(C.POINTER(C.c_uint)), n) == 0, lib.rt_last_error()
    for _ in range(2):
        launch()


use("natural")
ref = [b.clone() for b in bufs]
res = {k: [] for k in ["natural", *orders]}
for r in range(ROUNDS):
    for k in res:
        use(k)
        res[k].append(timed())
        if k != "natural":
            assert all(torch.equal(a, b) for a, b in zip(ref, bufs)), k
    print(json.dumps({"round": r, **{k: round(v[-1], 4) for k, v in res.items()}}), flush=True)
nat = float(np.median(res["natural"]))
print(json.dumps({k: {"ms": round(float(np.median(v)), 4), "vs_natural": round(float(np.median(v)) / nat - 1, 4)}
                  for k, v in res.items()}), flush=True)
