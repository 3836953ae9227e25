"""Collects tools/configs_bench.sh's per-config bench lines into one table (dev tool).

usage: python tools/configs_summary.py gpurun_out/configs_TAG OUT.json
Each row: the workload, GPU Mrays/s and ms per frame (whole frames, one GPU), the single-frame
record where measured, the CPU baseline (Mrays/s, threads, whole-frame seconds, extrapolated or
not) and the GPU / CPU ratio.
"""
import json
import sys
from pathlib import Path

NAMES = {"c1": "o_01_spheres proxy 640x480 1spp", "c2": "Office proxy 1920x1080 1spp",
         "c3": "Office proxy 3840x2160 16spp", "c4": "10M random triangles 1920x1080 1spp",
         "c5": "Office proxy 7680x4320 64spp (whole frame on one GPU)"}


def main(src, dst):
    rows = []
    for c in sorted(NAMES):
        p = Path(src) / f"{c}.json"
        if not p.exists():
            continue
        d = json.loads(p.read_text())
        cb = d.get("cpu_baseline") or {}
        sf = d.get("single_frame") or {}
        rows.append({
            "config": c, "name": NAMES[c], "workload": d["config"]["workload"],
            "gpu_mrays_s": d["value"], "gpu_ms_per_frame": d["ms_per_step"],
            "kernel_ms_per_frame": d.get("kernel_ms_per_frame"),
            "frames_per_launch": d["config"]["frames_per_launch"], "rays_per_frame": d["config"]["rays_per_frame"],
            "single_frame_ms": sf.get("ms_per_frame"),
            "single_frame_pipelined_ms": (sf.get("pipelined") or {}).get("ms_per_frame"),
            "roofline_frac": (d.get("roofline") or {}).get("frac"),
            "bound": (d.get("roofline") or {}).get("bound"),
            "cpu_mrays_s": cb.get("value"), "cpu_threads": cb.get("cores"), "cpu_frame_s": cb.get("frame_s"),
            "cpu_frame_s_extrapolated": cb.get("frame_s_extrapolated"), "cpu_sample": cb.get("sample"),
            "gpu_over_cpu": round(d["value"] / cb["value"], 1) if cb.get("value") else None,
        })
    Path(dst).write_text(json.dumps({"rows": rows, "_source": str(src)}, indent=1))
    for r in rows:
        print(f"{r['config']} {r['name']:<52} GPU {r['gpu_mrays_s']:>9.1f} Mrays/s {r['gpu_ms_per_frame']:>9.3f} ms/frame | "
              f"CPU {r['cpu_mrays_s']} Mrays/s x{r['cpu_threads']} ({r['cpu_frame_s']} s/frame"
              f"{', extrapolated' if r['cpu_frame_s_extrapolated'] else ''})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
