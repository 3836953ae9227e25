"""Per-launch-shape durations of the production kernel from a rocprofv3 --kernel-trace run of
bench.py (dev tool).

usage: python tools/trace_summary.py OUT.json PROF_DIR BENCH.json

bench.py's production-kernel dispatches come in a fixed order: the counting launch of F frames
(plus one of steps % F frames when F does not divide --steps), the counting launch of the NS
single-frame views, the warm-up launches, the timed launches, then three runs of NS one-frame
launches: the natural-order record, an untimed pass in the library's default (cost) order, and
the default-order single-frame record.  The summary averages the timed launches and each
single-frame record separately, so each figure can be set beside the bench's own HIP-event
kernel_ms_avg / single_frame.kernel_ms_avg / single_frame.natural_order.kernel_ms_avg.
"""
import csv
import glob
import json
import os
import sys


def main():
    out, pdir, bench_path = sys.argv[1:4]
    bench = json.loads(open(bench_path).read().strip().splitlines()[-1])
    paths = glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                if any(k in name for k in ("render_kernel<4, false>", "render_kernel<4, false, false",
                                           "ILi4ELb0EEE", "ILi4ELb0ELb0E")):
                    rows.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
    rows.sort()
    dur = [d for _, d in rows]
    steps, warm = bench["steps"], bench["warmup"]
    F = int(bench["config"]["rays_breakdown_rank0_launch"]["frames"])
    n_timed = -(-steps // F)
    n_count = 1 + (1 if steps % F else 0) + 1
    n_warm = -(-warm // F) if warm else 0
    n_single = bench["single_frame"]["frames"] if bench.get("single_frame") else 0
    t0 = n_count + n_warm
    timed = dur[t0:t0 + n_timed]
    natural = dur[t0 + n_timed:t0 + n_timed + n_single]
    single = dur[t0 + n_timed + 2 * n_single:t0 + n_timed + 3 * n_single]
    sf = bench.get("single_frame") or {}
    res = {
        "production_dispatches": len(dur),
        "expected_dispatches": n_count + n_warm + n_timed + 3 * n_single,
        "timed_launches": len(timed),
        "timed_ms_avg": sum(timed) / len(timed) if timed else None,
        "bench_kernel_ms_avg": bench["roofline"]["kernel_ms_avg"],
        "single_frame_launches": len(single),
        "single_ms_avg": sum(single) / len(single) if single else None,
        "bench_single_kernel_ms_avg": sf.get("kernel_ms_avg"),
        "natural_order_launches": len(natural),
        "natural_order_ms_avg": sum(natural) / len(natural) if natural else None,
        "bench_natural_order_kernel_ms_avg": (sf.get("natural_order") or {}).get("kernel_ms_avg"),
        "all_ms": [round(d, 4) for d in dur],
        "source": os.path.normpath(pdir),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "all_ms"}, indent=1))


if __name__ == "__main__":
    main()
