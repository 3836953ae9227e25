"""Tail-order probe for multi-frame launches (dev tool, GPU): a launch of F frames costs about
0.27 ms more than F x its per-frame rate at 128 frames (T(F) = a + b F fitted on 20 and 128), while a
cost-ordered one-frame launch drains in ~0.09 ms.  Sorting the whole F-frame launch by cost was +4 %
slower in round 3 (the band order's locality is worth more); this probe sorts only the
LAST k % of every work head's range (expensive tiles first, stable), keeping the band order for the
rest, through rt_debug_set_tile_order (host-built permutations; pixels must not change).  Costs: per
tile position, pixel lifetimes of one RT_FLAG_TILE_COST_TIME launch of the same frames.

usage: python tools/tail_order_probe.py [F] [reps]
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
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 15
lib = rtamd.hip_lib()
tw, th = rtamd.tile_shape()

hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
base = hs.render_params(1920, 1080, 1)
cams = [rtamd.camera_orbit(base, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
bufs = [torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda") for _ in range(F)]
tiles_x = -(-1920 // tw)


def launch(flags=0):
    ps = [abi.RenderParams.from_buffer_copy(c) for c in cams]
    for q in ps:
        q.flags = flags
    dev.launch_frames(ps, [b.data_ptr() for b in bufs])


def timed():
    ms = []
    for _ in range(REPS):
        launch()
        torch.cuda.synchronize()
        ms.append(dev.last_kernel_ms())
    return float(np.median(ms))


launch(abi.RT_FLAG_TILE_COST_TIME)
torch.cuda.synchronize()
npos = lib.rt_debug_tile_cost(dev._h, None, 0)
cpos = np.zeros(npos, dtype=np.uint32)
lib.rt_debug_tile_cost(dev._h, cpos.ctypes.data_as(C.POINTER(C.c_uint)), npos)
lin = np.arange(npos * F)                      # band-major linear tiles (ty, frame, tx) -> positions
ty, rem = lin // (F * tiles_x), lin % (F * tiles_x)
cost = cpos[ty * tiles_x + rem % tiles_x].astype(np.int64)
n = len(cost)


def order_tail(k, dilate=0):
    order = np.arange(n, dtype=np.uint32)
    c = cost
    if dilate:   # the largest cost within +-dilate tiles of the row (the library's one-frame window)
        cc = cost.reshape(-1, tiles_x)
        m = cc.copy()
        for d in range(1, dilate + 1):
            m[:, d:] = np.maximum(m[:, d:], cc[:, :-d])
            m[:, :-d] = np.maximum(m[:, :-d], cc[:, d:])
        c = m.reshape(-1)
    for h in range(8):
        t0, t1 = n * h // 8, n * (h + 1) // 8
        s = t1 - max(1, int((t1 - t0) * k / 100))
        seg = np.arange(s, t1)
        order[s:t1] = seg[np.argsort(-c[s:t1], kind="stable")]
    return order


lib.rt_debug_set_tile_order(dev._h, None, 0)
for _ in range(3):
    launch()
ref = [b.clone() for b in bufs]
res = {"frames": F, "natural_ms": timed()}
print(json.dumps(res), flush=True)
for k in (5, 10, 20, 40, 100):
    for dil in (0, 4):
        order = order_tail(k, dil)
        rc = lib.rt_debug_set_tile_order(dev._h, order.ctypes.data_as(C.POINTER(C.c_uint)), n)
        assert rc == 0, lib.rt_last_error()
        for _ in range(2):
            launch()
        t = timed()
        same = all(torch.equal(a, b) for a, b in zip(ref, bufs))
        lib.rt_debug_set_tile_order(dev._h, None, 0)
        for _ in range(2):
            launch()
        t_nat = timed()   # interleaved natural-order reference
        r = {"tail_pct": k, "dilate": dil, "ordered_ms": t, "natural_ms": t_nat,
             "gain": round(1 - t / t_nat, 4), "pixels_identical": same}
        print(json.dumps(r), flush=True)
