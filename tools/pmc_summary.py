"""Summarise rocprofv3 --pmc passes of bench.py into one JSON (dev tool).

usage: PMC_CMD="<profiled command>" PMC_FRAMES=<frames per launch> \
       python tools/pmc_summary.py OUT.json DIR [DIR ...]
Each DIR holds one pass's pmc_counter_collection.csv.  Only the production
render kernel (render_kernel<4, false>) dispatches are averaged.  Derived
figures follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE / WRITE_SIZE are
KB, and gfx950 FETCH_SIZE under-reports wide streaming reads by 2x.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def is_production(name):
    return "render_kernel" in name and ("<4, false>" in name or "ILi4ELb0E" in name)


def collect(dirs):
    vals = defaultdict(lambda: defaultdict(float))   # counter -> dispatch -> value
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if not is_production(row["Kernel_Name"]):
                        continue
                    vals[row["Counter_Name"]][(path, row["Dispatch_Id"])] += float(row["Counter_Value"])
    out = {}
    for name, per in sorted(vals.items()):
        v = list(per.values())
        out[name] = {"dispatches": len(v), "mean_per_dispatch": sum(v) / len(v)}
    return out


def derive(c):
    g = lambda k: c.get(k, {}).get("mean_per_dispatch")
    d = {}
    if g("FETCH_SIZE") is not None:
        d["hbm_read_bytes_corrected"] = 2 * g("FETCH_SIZE") * 1024
    if g("WRITE_SIZE") is not None:
        d["hbm_write_bytes"] = g("WRITE_SIZE") * 1024
    if g("TCC_HIT_sum") and g("TCC_MISS_sum") is not None:
        d["l2_hit_rate"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD active cycles = GRBM / 8
    if g("TA_BUSY_avr") and g("GRBM_GUI_ACTIVE"):
        d["ta_busy_frac"] = g("TA_BUSY_avr") / (g("GRBM_GUI_ACTIVE") / 8)
    if g("TD_TD_BUSY_sum") and g("GRBM_GUI_ACTIVE"):
        d["td_busy_frac"] = g("TD_TD_BUSY_sum") / 256 / (g("GRBM_GUI_ACTIVE") / 8)
    if g("TCP_TOTAL_CACHE_ACCESSES_sum") and g("TCP_TCC_READ_REQ_sum") is not None:
        d["l1_miss_to_l2_frac"] = g("TCP_TCC_READ_REQ_sum") / g("TCP_TOTAL_CACHE_ACCESSES_sum")
    return d


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    c = collect(dirs)
    c["_derived"] = derive(c)
    cmd = os.environ.get("PMC_CMD", "python bench.py")
    c["_command"] = cmd
    c["_frames_per_launch"] = int(os.environ.get("PMC_FRAMES", "1"))
    c["_note"] = ("rocprofv3 --pmc, one pass per directory ("
                  + ", ".join(os.path.basename(os.path.normpath(d)) for d in dirs)
                  + f") of `{cmd}`; production kernel dispatches only, per dispatch (= per launch). "
                  "FETCH_SIZE/WRITE_SIZE in KB; HBM read bytes = 2*FETCH_SIZE*1024 on gfx950.")
    with open(out, "w") as f:
        json.dump(c, f, indent=1)
    print(json.dumps(c["_derived"], indent=1))


if __name__ == "__main__":
    main()
