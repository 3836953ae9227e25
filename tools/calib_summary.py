"""FETCH_SIZE / WRITE_SIZE calibration from rocprofv3 passes over tools/hbm_calib.bin (dev tool).

usage: python tools/calib_summary.py OUT.json FETCH_DIR WRITE_DIR
Each calibration kernel moves exactly 2 GiB (read_bN: FETCH_SIZE pass, write_bN: WRITE_SIZE
pass); factor = true bytes / (counter KB x 1024).
"""
import csv
import glob
import json
import os
import sys

BYTES = 2 << 30


def values(d, counter):
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                name = row["Kernel_Name"].split("(")[0].strip()
                out[name] = out.get(name, 0.0) + float(row["Counter_Value"])
    return out


def main():
    out_path, fdir, wdir = sys.argv[1:4]
    res = {}
    for name, v in values(fdir, "FETCH_SIZE").items():
        if name.startswith("read_"):
            res[name] = {"counter": "FETCH_SIZE", "kb": v, "factor": BYTES / (v * 1024)}
    for name, v in values(wdir, "WRITE_SIZE").items():
        if name.startswith("write_"):
            res[name] = {"counter": "WRITE_SIZE", "kb": v, "factor": BYTES / (v * 1024)}
    res["_note"] = "tools/hbm_calib.hip: each kernel streams 2 GiB once (coalesced, one width per lane)"
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
