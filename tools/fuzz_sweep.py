"""Extended parity sweep (dev tool, under gpurun): the GPU suite's seeded random scenes
(tests/fuzz_scenes.py) over many more seeds than the suite runs, each rendered by the production
kernel and by the CPU oracle (reference CPU semantics, oracle/) and compared -- fp64 pixels within
1e-12, ray counts exact.  Per seed, at an odd image size with n x n spp, n = 1-4 (n = 2, 4:
sample groups, the default since round 6; n = 3: one lane per pixel): the plain mesh scene, the
same scene with spheres and planes (analytic path, CPU intersect_scene semantics) and with a
textured mesh; every 5th seed also on the SAH and refined-reference device trees (bit-identical
to the default SBVH).  The oracle here is the checker, never the thing measured.

usage: python tools/fuzz_sweep.py FIRST_SEED N_SEEDS OUT.json
       python tools/fuzz_sweep.py --deep FIRST_SEED N_SEEDS OUT.json
--deep: generated deep scenes instead -- random-triangle soups of 2^15 .. 2^20 triangles (the
16-entry stack ring and global spills from 2^18 records on) and cornell boxes of random detail,
random depth 0-5, at 96 x 64 with 1x1, 2x2 or 4x4 spp.
"""
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
import fuzz_scenes  # noqa: E402
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

TOL64 = 1e-12


def counts(st):
    return [st.primary_rays, st.shadow_rays, st.reflection_rays]


def check(hs, p, analytic=False, trees=("sbvh",)):
    """Max |GPU - oracle| over the image and whether every tree gave the same bits and counts."""
    orc = pyoracle.Oracle(hs.raw, hs)
    ref, cnt = orc.render(p, pyoracle.MODE_REFERENCE)
    p.out_format = rtamd.RT_OUT_RGB_F64
    first = None
    err, same, rays = 0.0, True, 0
    for tree in trees:
        dev = rtamd.DeviceScene(hs, 0, analytic=analytic, tree=tree)
        img, st = dev.render(p)
        dev.close()
        err = max(err, float(np.abs(img - ref).max()))
        ok_counts = counts(st) == [cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays]
        if first is None:
            first = (img, counts(st))
        else:
            same &= bool(np.array_equal(img, first[0]) and counts(st) == first[1])
        same &= ok_counts
        rays = sum(counts(st))
    return err, same, rays


def deep(s0, n, out):
    rows, worst, fails, t0 = [], 0.0, [], time.time()
    sizes = [1 << 15, 1 << 16, 1 << 17, 1 << 18, 1 << 19, 1 << 20]
    for seed in range(s0, s0 + n):
        kind = "cornell" if seed % 4 == 3 else "random_tris"
        gen = {"detail": 1 + seed % 6} if kind == "cornell" else {"n_triangles": sizes[seed % len(sizes)]}
        hs = rtamd.HostScene.generate(kind, seed=seed, max_depth=seed % 6, **gen)
        hs.prepare()
        p = hs.render_params(96, 64, (1, 2, 4)[seed % 3])   # 2x2 / 4x4: sample groups
        err, same, rays = check(hs, p, False, ("sbvh", "sah") if seed % 3 == 0 else ("sbvh",))
        ok = err <= TOL64 and same
        res = {"seed": seed, "scene": kind, **gen, "depth": seed % 6, "max_abs_err": err,
               "exact_counts_and_trees": same, "rays": rays, "ok": ok}
        worst = max(worst, err)
        if not ok:
            fails.append(seed)
        rows.append(res)
        print(json.dumps(res), flush=True)
    summary = {"deep": True, "seeds": [s0, s0 + n], "scenes": n, "failures": fails, "worst_max_abs_err": worst,
               "tolerance": TOL64, "seconds": round(time.time() - t0, 1)}
    Path(out).write_text(json.dumps({"summary": summary, "rows": rows}, indent=1))
    print(json.dumps(summary), flush=True)
    sys.exit(1 if fails else 0)


def main():
    if sys.argv[1] == "--deep":
        deep(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
    s0, n, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    rows, worst, fails, t0 = [], 0.0, [], time.time()
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td)
        for seed in range(s0, s0 + n):
            w, h = 33 + seed % 40, 21 + (seed * 7) % 31        # odd and even sizes, partial tiles
            spp = 1 + seed % 4
            trees = ("sbvh", "sah", "reference") if seed % 5 == 0 else ("sbvh",)
            res = {"seed": seed, "size": [w, h], "spp": spp}
            for kind, writer, analytic in (("mesh", fuzz_scenes.write, False),
                                           ("analytic", fuzz_scenes.write_analytic, True),
                                           ("textured", fuzz_scenes.write_textured, False)):
                d = tmp / f"{kind}{seed}"
                d.mkdir()
                hs = rtamd.HostScene.load(writer(d, seed, w, h))
                hs.prepare()
                p = hs.render_params(0, 0, spp)
                err, same, rays = check(hs, p, analytic, trees if kind == "mesh" else ("sbvh",))
                ok = err <= TOL64 and same
                res[kind] = {"max_abs_err": err, "exact_counts_and_trees": same, "rays": rays, "ok": ok}
                worst = max(worst, err)
                if not ok:
                    fails.append((seed, kind))
            rows.append(res)
            print(json.dumps(res), flush=True)
    summary = {"seeds": [s0, s0 + n], "scenes": 3 * n, "failures": fails, "worst_max_abs_err": worst,
               "tolerance": TOL64, "seconds": round(time.time() - t0, 1)}
    Path(out).write_text(json.dumps({"summary": summary, "rows": rows}, indent=1))
    print(json.dumps(summary), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
