"""Per-round anatomy of single-frame launches (dev tool, under gpurun): the production kernel with
the round timeline (RT_FLAG_TIMELINE, record layout in rt_hip.h rt_debug_timeline), 1080p.
Prints round counts and durations, the time per wave-level iteration by kind (global-memory node,
LDS-treelet node, leaf) in the steady phase and after the work queue emptied, the busy-lane curve
and the slowest rounds.
usage: python tools/round_timeline.py [scene [tris]] [--depth D]"""
import argparse
import sys

import numpy as np
import torch

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("scene", nargs="?", default="office")
ap.add_argument("tris", nargs="?", type=int, default=0)
ap.add_argument("--depth", type=int, default=-1)
ap.add_argument("--order", action="store_true", help="cost-ordered launches (RT_FLAG_COST_ORDER), warmed up")
a = ap.parse_args()
host = rtamd.HostScene.generate(a.scene, **({"n_triangles": a.tris} if a.tris else {}))
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
out = torch.zeros((1080, 1920, 3), device="cuda")


def pct(v, qs=(10, 50, 90, 99)):
    return " ".join(f"p{q}={np.percentile(v, q):.1f}" for q in qs) if len(v) else "-"


p = host.render_params(1920, 1080, 1)
if a.depth >= 0:
    p.max_depth = a.depth
ms = []
base = rtamd.abi.RT_FLAG_COST_ORDER if a.order else rtamd.abi.RT_FLAG_NATURAL_ORDER
p.flags = base
for _ in range(5):
    gpu.launch(p, out.data_ptr())
    ms.append(gpu.last_kernel_ms())
p.flags = rtamd.RT_FLAG_TIMELINE | (rtamd.abi.RT_FLAG_COST_ORDER if a.order else 0)
gpu.launch(p, out.data_ptr())
gpu.launch(p, out.data_ptr())
tl_ms = gpu.last_kernel_ms()
tl = gpu.timeline().astype(np.int64)
used = tl[:, :, 0] > 0
t0 = tl[:, :, 0][used].min()
start = np.where(used, (tl[:, :, 0] - t0) / 100.0, np.nan)   # us
end = np.where(used, (tl[:, :, 1] - t0) / 100.0, np.nan)
dur = end - start
busy = tl[:, :, 2] & 0xFF
queued = (tl[:, :, 2] >> 16) & 1
shadow = (tl[:, :, 2] >> 24) & 0xFF
iters = tl[:, :, 3] & 0xFFFFFFFF
rloop = tl[:, :, 3] >> 32
M40 = (1 << 40) - 1
gsum = {k: (tl[:, :, 3 + i] & M40) / 100.0 for i, k in enumerate(["gnode", "lnode", "leaf"], 1)}   # us
gcnt = {k: tl[:, :, 3 + i] >> 40 for i, k in enumerate(["gnode", "lnode", "leaf"], 1)}
gmax = (tl[:, :, 7] & 0xFFFFFFFF) / 100.0
setup = (tl[:, :, 7] >> 32) / 100.0
witer = sum(gcnt.values())
rounds = used.sum(1)
waves = rounds > 0
print(f"== {a.scene} 1080p depth {p.max_depth}: production {np.median(ms):.3f} ms, timeline variant {tl_ms:.3f} ms; "
      f"waves {waves.sum()}, rounds/wave {pct(rounds[waves])}")
u = used
print(f"  round us {pct(dur[u])}; busy {pct(busy[u])}; lane iters {pct(iters[u])}; wave iters {pct(witer[u])}; "
      f"round loops {pct(rloop[u])}; setup us {pct(setup[u])}; longest iteration us {pct(gmax[u])}")
T = float(np.nanmax(end))
t_end = np.nanmax(end, axis=1)[waves]
print(f"  wave end us {pct(t_end, (0, 10, 50, 90, 100))}")
qd = start[used & (queued == 0)]
print(f"  queue empty from {np.nanmin(qd) if len(qd) else float('nan'):.0f} us (first round that saw no work left) of {T:.0f} us")
# time per wave-level iteration by kind, in time windows (round start)
edges = [0, 100, 200, 300, 400, 500, 600, 700, 10_000]
print("  us per wave-level iteration by kind and round-start window (count):")
for k in gsum:
    row = []
    for lo, hi in zip(edges[:-1], edges[1:]):
        m = used & (start >= lo) & (start < hi)
        c = gcnt[k][m].sum()
        row.append(f"[{lo}-{hi if hi < 10_000 else 'end'}) {gsum[k][m].sum() / max(c, 1):.2f} ({c})")
    print(f"    {k:5s}: " + "  ".join(row))
for name, m in [("rounds <= 50 us", used & (dur <= 50)), ("rounds > 50 us", used & (dur > 50))]:
    print(f"  {name}: {int(m.sum())}; us/iteration " +
          " ".join(f"{k} {gsum[k][m].sum() / max(gcnt[k][m].sum(), 1):.2f} ({gcnt[k][m].sum()})" for k in gsum) +
          f"; wave iters {pct(witer[m])}; busy {pct(busy[m])}; shadow lanes {pct(shadow[m])}")
grid = np.linspace(0, T, 21)
lanes, wv = [], []
for x in grid:
    m = used & (start <= x) & (end >= x)
    lanes.append(int(busy[m].sum()))
    wv.append(int(((np.nanmin(start, 1) <= x) & (np.nanmax(end, 1) >= x)).sum()))
print("  t(us):       " + " ".join(f"{x:6.0f}" for x in grid))
print("  waves alive: " + " ".join(f"{v:6d}" for v in wv))
print("  busy lanes:  " + " ".join(f"{v:6d}" for v in lanes))
flat = np.argsort(-np.nan_to_num(dur, nan=-1).ravel())[:10]
print("  slowest rounds: start+dur us | busy shadow | lane iters, wave iters gnode/lnode/leaf (us each) | longest it")
for f in flat:
    w, r = divmod(int(f), dur.shape[1])
    kinds = " ".join(f"{gcnt[k][w, r]}x{gsum[k][w, r] / max(gcnt[k][w, r], 1):.1f}" for k in gsum)
    print(f"    w{w} r{r}: {start[w, r]:.0f}+{dur[w, r]:.0f} | b{busy[w, r]} s{shadow[w, r]} | i{iters[w, r]} "
          f"W{witer[w, r]} {kinds} | {gmax[w, r]:.1f} q{queued[w, r]}")
sys.stdout.flush()
