"""Interleaved A/B of kernel libraries on single-frame and batched frame time (dev tool, under
gpurun).  usage: python tools/ab_frame.py ROUNDS lib1 lib2 ... [-- scene [tris]]
A library entry may carry upload options after '#': lib.so#stack_ring=16,lds_treelet=-1."""
import json
import os
import subprocess
import sys

import numpy as np

args = sys.argv[1:]
extra = []
if "--" in args:
    i = args.index("--")
    args, extra = args[:i], args[i + 1:]
R, libs = int(args[0]), args[1:]
res = {l: [] for l in libs}
for r in range(R):
    for l in libs:
        path, _, opts = l.partition("#")
        env = dict(os.environ, RTAMD_HIP_LIB=os.path.abspath(path), RTAMD_AB_OPTS=opts)
        o = subprocess.run([sys.executable, "tools/frame_probe.py", *extra], env=env, capture_output=True,
                           text=True, timeout=300)
        if o.returncode != 0:
            print(l, "FAILED", o.stderr[-2000:], flush=True)
            sys.exit(1)
        d = json.loads(o.stdout.strip().splitlines()[-1])
        res[l].append(d)
        print(f"{r} {os.path.basename(l)} {d}", flush=True)
for l, v in res.items():
    s = np.median([d["single_ms"] for d in v])
    b = np.median([d["batched_ms_per_frame"] for d in v])
    c = np.median([d.get("single_call_ms", float("nan")) for d in v])
    o = np.median([d.get("single_orbit20_ms", float("nan")) for d in v])
    print(f"{os.path.basename(l):48s} single {s:.4f} ms (call {c:.4f}, orbit-20 views {o:.4f})   "
          f"batched {b:.4f} ms/frame", flush=True)
