"""Tile-order probe (dev tool, GPU): does rendering each work head's expensive tiles first shorten a
launch's drain?  Per-tile costs (bounces per finished sample) come from one launch with
RT_FLAG_TILE_COST; the order sorts every head's tile range by cost, descending (stable), and is
handed to the library with rt_debug_set_tile_order.  Times one-frame launches and F-frame launches
(kernel time, HIP events) with and without the order, and checks the pixels do not change.

usage: python tools/order_probe.py [F] [reps]
"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "my-raytracer_amd"))
import rtamd  # noqa: E402
from rtamd import abi  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 20
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20
lib = rtamd.hip_lib()

hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
base = hs.render_params(1920, 1080, 1)
cams = [rtamd.camera_orbit(base, 0.12 * (f / (F - 1) - 0.5)) for f in range(F)]
bufs = [torch.zeros((1080, 1920, 3), dtype=torch.float32, device="cuda") for _ in range(F)]


def launch(nf, flags=0):
    ps = [abi.RenderParams.from_buffer_copy(c) for c in cams[:nf]]
    for q in ps:
        q.flags = flags
    if nf == 1:
        dev.launch(ps[0], bufs[0].data_ptr())
    else:
        dev.launch_frames(ps, [b.data_ptr() for b in bufs[:nf]])


def timed(nf, reps, flags=0):
    # (kernel time from the library's events; the stream time around the call includes the order kernel)
    ms, wall = [], []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        launch(nf, flags)
        e1.record()
        torch.cuda.synchronize()
        ms.append(dev.last_kernel_ms())
        wall.append(e0.elapsed_time(e1))
    return float(np.median(ms)), float(np.mean(ms)), float(np.median(wall))


def order_from_costs(cost, mode):
    n = len(cost)
    order = np.arange(n, dtype=np.uint32)
    for h in range(8):
        t0, t1 = n * h // 8, n * (h + 1) // 8
        seg = np.arange(t0, t1)
        if mode == "desc":
            seg = seg[np.argsort(-cost[t0:t1].astype(np.int64), kind="stable")]
        elif mode == "asc":
            seg = seg[np.argsort(cost[t0:t1].astype(np.int64), kind="stable")]
        elif mode == "reverse":
            seg = seg[::-1]
        elif mode.startswith("top"):   # the most expensive k % first (in natural order), then the rest
            k = max(1, int(len(seg) * int(mode[3:]) / 100))
            hot = np.zeros(len(seg), bool)
            hot[np.argsort(-cost[t0:t1].astype(np.int64), kind="stable")[:k]] = True
            seg = np.concatenate([seg[hot], seg[~hot]])
        order[t0:t1] = seg
    return order


for nf in (1, F):
    lib.rt_debug_set_tile_order(dev._h, None, 0)
    for _ in range(3):
        launch(nf)
    base_ms = timed(nf, REPS)
    ref = [b.clone() for b in bufs[:nf]]
    print(f"frames/launch {nf}: no order: kernel median {base_ms[0]:.4f} ms mean {base_ms[1]:.4f}", flush=True)
    for cflag, cname in ((abi.RT_FLAG_TILE_COST, "bounces"), (abi.RT_FLAG_TILE_COST_TIME, "time")):
      lib.rt_debug_set_tile_order(dev._h, None, 0)
      launch(nf, cflag)
      torch.cuda.synchronize()
      npos = lib.rt_debug_tile_cost(dev._h, None, 0)
      cpos = np.zeros(npos, dtype=np.uint32)
      lib.rt_debug_tile_cost(dev._h, cpos.ctypes.data_as(C.POINTER(C.c_uint)), npos)
      tx_n = 1920 // 8
      lin = np.arange(npos * nf)                      # band-major linear tiles -> their positions
      ty, rem = lin // (nf * tx_n), lin % (nf * tx_n)
      cost = cpos[ty * tx_n + rem % tx_n]
      n = len(cost)
      print(f" cost {cname}: tiles {n}, per tile mean {cost.mean():.1f} p50 {np.median(cost):.0f} "
            f"p90 {np.percentile(cost, 90):.0f} max {cost.max()}", flush=True)
      for mode in (("desc", "reverse") if cname == "bounces" else ("desc", "top5", "top15", "top30")):
        order = order_from_costs(cost, mode)
        rc = lib.rt_debug_set_tile_order(dev._h, order.ctypes.data_as(C.POINTER(C.c_uint)), n)
        assert rc == 0, lib.rt_last_error()
        for _ in range(2):
            launch(nf)
        t = timed(nf, REPS)
        same = all(torch.equal(a, b) for a, b in zip(ref, bufs[:nf]))
        print(f"  order {cname}/{mode:<8} kernel median {t[0]:.4f} ms mean {t[1]:.4f} "
              f"({(t[0] / base_ms[0] - 1) * 100:+.1f} %), pixels identical: {same}", flush=True)
    lib.rt_debug_set_tile_order(dev._h, None, 0)
    # the library's own cost order (RT_FLAG_COST_ORDER): each launch ordered by the previous one's costs
    for fl, nm in ((abi.RT_FLAG_COST_ORDER, "lifetime"), (abi.RT_FLAG_COST_ORDER | abi.RT_FLAG_TILE_COST, "bounces")):
        for _ in range(3):
            launch(nf, fl)
        t = timed(nf, REPS, fl)
        same = all(torch.equal(a, b) for a, b in zip(ref, bufs[:nf]))
        if nf == 1:   # the library's order against the host's order of the same cost map
            npos = lib.rt_debug_tile_cost(dev._h, None, 0)
            cpos = np.zeros(npos, dtype=np.uint32)
            lib.rt_debug_tile_cost(dev._h, cpos.ctypes.data_as(C.POINTER(C.c_uint)), npos)
            launch(nf, fl)   # builds the order of the next launch from cpos in its drain
            launch(nf, fl)   # ordered by cpos
            torch.cuda.synchronize()
            m = lib.rt_debug_last_tile_order(dev._h, None, 0)
            got = np.zeros(m, dtype=np.uint32)
            lib.rt_debug_last_tile_order(dev._h, got.ctypes.data_as(C.POINTER(C.c_uint)), m)
            # the library sorts 8-bit log-scale cost classes (4 per octave, RT_ORDER_SHIFT 21), stable
            q = np.clip((cpos.astype(np.float32).view(np.uint32) >> 21).astype(np.int64) - ((127 + 8) << 2), 0, 255)
            want = order_from_costs(q.astype(np.uint32), "desc")
            print(f"   library order == host exact order: {np.array_equal(got, want)} "
                  f"(first differences at {np.nonzero(got != want)[0][:5]})", flush=True)
        print(f"  RT_FLAG_COST_ORDER ({nm}) kernel median {t[0]:.4f} ms mean {t[1]:.4f} "
              f"({(t[0] / base_ms[0] - 1) * 100:+.1f} %), stream time {t[2]:.4f} ms (unordered {base_ms[2]:.4f}), "
              f"pixels identical: {same}", flush=True)
