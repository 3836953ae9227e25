"""Summarise rocprofv3 --pmc passes of bench.py into one JSON (dev tool).

usage: python tools/pmc_summary.py OUT.json --bench BENCH.json [--calib CALIB.json] DIR [DIR ...]

Each DIR holds one pass's *counter_collection.csv over the command that printed
BENCH.json (the same bench.py command, unprofiled, run just before).  Only the
production render kernel (render_kernel<4, false[, false]>) dispatches count.  Every
counter is summed over those dispatches and divided by the frames they rendered
(BENCH.json config.production_frames_rendered), so the figures are per frame and
apply to any launch shape of the same workload (bench.py multiplies by its own
frames per launch).  HBM bytes (MI355X_MICROARCH.md, HBM section): FETCH_SIZE
and WRITE_SIZE are KB; gfx950 under-reports wide reads, so each is scaled by the
factor measured by tools/hbm_calib.hip for the 16-B-per-lane accesses that make
up the kernel's fabric traffic (CALIB.json, from tools/calib_summary.py;
default read x2, write x1 as the guide states for that width).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def is_production(name):
    # render_kernel<4, false> (round 1) / render_kernel<4, false, false[, RING]> (mangled ...ILi4ELb0ELb0E...)
    return "render_kernel" in name and ("<4, false>" in name or "<4, false, false" in name
                                        or "ILi4ELb0EEE" in name or "ILi4ELb0ELb0E" in name)


def collect(dirs):
    vals = defaultdict(lambda: defaultdict(float))   # counter -> dispatch -> value
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if not is_production(row["Kernel_Name"]):
                        continue
                    vals[row["Counter_Name"]][(path, row["Dispatch_Id"])] += float(row["Counter_Value"])
    return {name: list(per.values()) for name, per in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--bench", required=True)
    ap.add_argument("--calib", default="")
    a = ap.parse_args()
    bench = json.loads(open(a.bench).read().strip().splitlines()[-1])
    frames = bench["config"]["production_frames_rendered"]
    raw = collect(a.dirs)
    read_f, write_f, calib_src = 2.0, 1.0, "MI355X_MICROARCH.md (16-B/lane streaming: read x2, write x1)"
    if a.calib:
        c = json.load(open(a.calib))
        read_f, write_f, calib_src = c["read_b128"]["factor"], c["write_b128"]["factor"], a.calib
    out = {name: {"dispatches": len(v), "sum": sum(v), "per_frame": sum(v) / frames} for name, v in sorted(raw.items())}
    g = lambda k: out.get(k, {}).get("per_frame")
    pf = {}
    if g("FETCH_SIZE") is not None:
        pf["hbm_read_bytes"] = g("FETCH_SIZE") * 1024 * read_f
    if g("WRITE_SIZE") is not None:
        pf["hbm_write_bytes"] = g("WRITE_SIZE") * 1024 * write_f
    d = {}
    if g("TCC_HIT_sum") and g("TCC_MISS_sum") is not None:
        d["l2_hit_rate"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD active cycles = GRBM / 8
    if g("TA_BUSY_avr") and g("GRBM_GUI_ACTIVE"):
        d["ta_busy_frac"] = g("TA_BUSY_avr") / (g("GRBM_GUI_ACTIVE") / 8)
    if g("TD_TD_BUSY_sum") and g("GRBM_GUI_ACTIVE"):
        d["td_busy_frac"] = g("TD_TD_BUSY_sum") / 256 / (g("GRBM_GUI_ACTIVE") / 8)
    if g("TCP_TOTAL_CACHE_ACCESSES_sum") and g("TCP_TCC_READ_REQ_sum") is not None:
        d["l1_miss_to_l2_frac"] = g("TCP_TCC_READ_REQ_sum") / g("TCP_TOTAL_CACHE_ACCESSES_sum")
    out["_per_frame"] = pf
    out["_derived"] = d
    out["_workload"] = bench["config"]["workload_key"]
    out["_frames"] = frames
    out["_calibration"] = {"read_factor": read_f, "write_factor": write_f, "source": calib_src}
    out["_bench"] = {"value": bench["value"], "kernel_ms_avg": bench["roofline"]["kernel_ms_avg"],
                     "frames_per_launch": bench["config"]["frames_per_launch"]}
    out["_note"] = ("rocprofv3 --pmc, one pass per directory ("
                    + ", ".join(os.path.basename(os.path.normpath(x)) for x in a.dirs)
                    + "); production-kernel dispatches only; 'sum' over the run, 'per_frame' = sum / _frames. "
                    "_per_frame HBM bytes = FETCH_SIZE x 1024 x read_factor, WRITE_SIZE x 1024 x write_factor.")
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"_per_frame": pf, "_derived": d}, indent=1))


if __name__ == "__main__":
    main()
