"""bench.py — Mrays/s of the MI355X render path on the Office workload.

Metric (BASELINE.json): Mrays/sec (primary + shadow + reflection), Office
1920x1080 1 spp, on 1/2/4/8 MI355X.  The Office scene files are not in the
reference, so the workload is the fixed-seed office_proxy.

One step = one full frame: every rank renders its interleaved 16-row stripes
(stripe = rank mod N) with one launch of the flattened HIP kernel, then rank 0
gathers the stripes over RCCL (torch.distributed "nccl") and re-interleaves
them into the final image.  Total work per step is fixed => "strong" scaling.
Consecutive frames are rendered --frames at a time (default 128) by ONE launch
of the persistent kernel (rt_launch_frames: the frames share one work queue,
so the drain at the end of a launch is paid once per F frames); every frame
still traces all of its rays.  --streams S > 1 additionally keeps S launches in
flight on separate streams.  Default: 1 on one GPU (launches serial, so the HIP-event
launch duration is the kernel's own duration, as rocprofv3 reports it); 2 on N > 1,
so the RCCL gather of launch i (and the drain of its kernel) overlaps launch i+1.

Rays per frame are the canonical counts returned by the kernel's
counters in an untimed launch.  Roofline: algorithmic bytes per launch =
64*node_visits + 48*tri_tests + 64*closest_hits, from the
instrumented kernel variant (its counters are pinned to the CPU oracle's
replica by tests/test_gpu_parity.py), divided by the kernel duration measured
with HIP events on the launch stream over the timed steps.

cpu_baseline: the CPU oracle (C restatement of the reference's CPU renderer:
recursive unordered fp64 BVH traversal, closest-hit shadow rays, OpenMP) timed
on a deterministic row sample of the same frame, rank 0 / N=1 only.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
import rtamd  # noqa: E402
from rtamd.shard import HaloExchange, StripeGather, max_rows as shard_max_rows  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# The CU's vector-L1 data return (TD): one 64-lane dwordx4 wave-instruction per 16 cycles =
# 64 B/clk/CU (tools/l1_micro.hip) x 256 CUs x 2.4 GHz.
L1_PEAK_GBPS = 64 * 256 * 2.4
STRIPE_H = 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=128)
    ap.add_argument("--scene", default="office")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1, help="n: n*n stratified samples per pixel")
    ap.add_argument("--tris", type=int, default=0, help="random_tris triangle count")
    ap.add_argument("--cpu-row-stride", type=int, default=1, help="cpu_baseline renders every k-th row")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="cpu_baseline: minimum timed CPU work")
    ap.add_argument("--save", default="", help="rank 0: save the gathered image (.npy)")
    ap.add_argument("--frames", type=int, default=0,
                    help="frames per launch (rt_launch_frames, <= RT_MAX_FRAMES = 128; default 128): one persistent-kernel "
                         "launch renders F consecutive frames from one work queue, so the per-launch drain is "
                         "paid once per F")
    ap.add_argument("--streams", type=int, default=0,
                    help="launches in flight on separate streams (1 = launches strictly serial; default 1 on "
                         "one GPU, 2 on N > 1 so the RCCL gather of one launch overlaps the next launch)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: nccl (RCCL over xGMI, the measured path) or gloo (host-staged rehearsal)")
    ap.add_argument("--tree", choices=["sah", "sbvh", "reference"], default=os.environ.get("RT_BENCH_TREE", "sbvh"),
                    help="device traversal hierarchy (pixels identical either way; DESIGN.md §4)")
    ap.add_argument("--analytic", action="store_true",
                    help="also trace the scene's spheres/planes (always on for --scene spheres)")
    ap.add_argument("--adaptive", action="store_true",
                    help="each frame = primary pass + adaptive supersampling pass (subp 4, threshold 0.02, "
                         "mytracer_gpu.cu:83-109); N > 1: stripe-edge halo rows exchanged by one all_gather per frame")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    n = world
    # rehearsal of the N-rank path on fewer GPUs (dev only): --dist-backend gloo stages the
    # collectives through host memory and RT_BENCH_DEVICE pins every rank to one device
    dev = int(os.environ.get("RT_BENCH_DEVICE", local))
    torch.cuda.set_device(dev)
    if n > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    host_staged = a.dist_backend == "gloo"

    # ---- host side: scene, normals, SoA, median-split BVH (untimed) ----
    gen = {"n_triangles": a.tris} if a.scene == "random_tris" and a.tris else {}
    host = rtamd.HostScene.generate(a.scene, **gen)
    build_s = host.prepare()
    gpu = rtamd.DeviceScene(host, device=dev, analytic=a.analytic or a.scene == "spheres",
                             tree=a.tree)
    params = host.render_params(a.width, a.height, a.spp)
    params.stripe_height = STRIPE_H
    params.stripe_count = n
    params.stripe_index = rank
    W = a.width
    # librt_hip keeps 8 launch contexts per scene; the halo exchange of --adaptive is single-stream
    S = 1 if a.adaptive else max(1, min(a.streams or (1 if n == 1 else 2), 8))
    F = 1 if a.adaptive else max(1, min(a.frames or 128, rtamd.abi.RT_MAX_FRAMES))
    # per stream: the F frames of one launch, contiguous, so one collective gathers them
    fbufs = [torch.zeros((F, shard_max_rows(a.height, STRIPE_H, n), W, 3), dtype=torch.float32, device="cuda")
             for _ in range(S)]
    bufs = [fb[f] for fb in fbufs for f in range(F)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(S - 1)]
    buf = bufs[0]
    stream = streams[0].cuda_stream
    rows_local = rtamd.rows_in_shard(params)
    prims = [torch.zeros((shard_max_rows(a.height, STRIPE_H, n), W, 3), dtype=torch.float64, device="cuda")
             for _ in range(S)] if a.adaptive else []
    # N > 1: the neighbour test of a stripe's edge rows needs the rows the neighbouring ranks
    # rendered -- ONE all_gather of every rank's stripe-edge rows per frame (rtamd.shard.HaloExchange)
    halo_x = HaloExchange(a.height, W, STRIPE_H, n, rank, rtamd.adaptive_halo_rows(params), device="cuda",
                          host_staged=host_staged) \
        if a.adaptive and n > 1 else None

    def adaptive_pass(prim, out, stats, stream_):
        if halo_x is None:
            return gpu.launch_adaptive(params, prim.data_ptr(), out.data_ptr(), 4, 0.02, stats=stats, stream=stream_)
        halo = halo_x(prim[:rows_local])
        return gpu.launch_adaptive_shard(params, prim.data_ptr(), halo.data_ptr(), out.data_ptr(), 4, 0.02,
                                         stats=stats, stream=stream_)

    # ---- counters: canonical rays + algorithmic bytes (untimed launches) ----
    if F > 1:   # same launch shape as the timed ones (identical frames: counts / F are exact)
        st = gpu.launch_frames(params, [b.data_ptr() for b in bufs[:F]], stats=True, stream=stream)
        for f in ("primary_rays", "shadow_rays", "reflection_rays", "node_visits", "tri_tests", "closest_hits",
                  "pixels"):
            setattr(st, f, getattr(st, f) // F)
    else:
        st = gpu.launch(params, buf.data_ptr(), stats=True, stream=stream)
    params.flags = rtamd.RT_FLAG_TRAVERSAL_STATS
    tst = gpu.launch(params, buf.data_ptr(), stats=True, stream=stream)
    params.flags = rtamd.RT_FLAG_WIDE_STATS   # the production kernel's own node / triangle fetches
    wst = gpu.launch(params, buf.data_ptr(), stats=True, stream=stream)
    params.flags = 0
    rays_local = st.primary_rays + st.shadow_rays + st.reflection_rays
    adaptive_info = None
    if a.adaptive:   # untimed: rays of the adaptive pass (selection depends on the primary image)
        p64 = rtamd.abi.RenderParams.from_buffer_copy(params)
        p64.out_format = rtamd.RT_OUT_RGB_F64
        gpu.launch(p64, prims[0].data_ptr(), stats=True, stream=stream)
        ast, nsel = adaptive_pass(prims[0], buf, True, stream)
        rays_local += ast.primary_rays + ast.shadow_rays + ast.reflection_rays
        adaptive_info = {("pixels_supersampled" if n == 1 else "pixels_supersampled_rank0"): nsel, "subp": 4, "threshold": 0.02,
                         "rays": ast.primary_rays + ast.shadow_rays + ast.reflection_rays}
    alg_bytes_local = 64 * tst.node_visits + 48 * tst.tri_tests + 64 * tst.closest_hits
    # bytes the production kernel requests from L1: 128-B GNode4, 80-B GTri, 96-B normal record per hit
    fetch_bytes_local = 128 * wst.node_visits + 80 * wst.tri_tests + 96 * wst.closest_hits

    gathers = [StripeGather(a.height, W, STRIPE_H, n, rank, device="cuda", frames=F, host_staged=host_staged)
               for _ in range(S)]
    image = None

    starts, ends, launch_frames = [], [], []

    def launch(li, nf, timed):
        """Launch li renders nf frames (steps); each frame is then gathered to rank 0."""
        nonlocal image
        s = streams[li % S]
        bs = bufs[(li % S) * F:(li % S) * F + nf]
        with torch.cuda.stream(s):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
            if a.adaptive:
                gpu.launch(p64, prims[li % S].data_ptr(), stats=False, stream=s.cuda_stream)
                adaptive_pass(prims[li % S], bs[0], False, s.cuda_stream)
            elif nf == 1:
                gpu.launch(params, bs[0].data_ptr(), stats=False, stream=s.cuda_stream)
            else:
                gpu.launch_frames(params, [b.data_ptr() for b in bs], stats=False, stream=s.cuda_stream)
            if timed:
                e1.record(s)
                starts.append(e0)
                ends.append(e1)
                launch_frames.append(nf)
            image = gathers[li % S](fbufs[li % S])   # N>1: ONE RCCL gather of the F frames' stripes + re-interleave

    def run(steps, timed):
        li, done = 0, 0
        while done < steps:
            nf = min(F, steps - done)
            launch(li, nf, timed)
            li += 1
            done += nf

    run(a.warmup, False)
    torch.cuda.synchronize()
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps, True)
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    kernel_ms_avg = float(np.mean(kernel_ms))
    frames_per_launch = float(np.mean(launch_frames))

    tot = torch.tensor([rays_local, alg_bytes_local], dtype=torch.float64, device="cuda")
    tmax = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if n > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    rays_total = float(tot[0])
    elapsed = float(tmax[0])

    if rank == 0:
        traffic = pmc_traffic(a, n, F)
        if a.save:
            np.save(a.save, (image[0] if image.dim() == 4 else image).float().cpu().numpy())
        ms_per_step = elapsed / a.steps * 1e3
        mrays = rays_total * a.steps / elapsed / 1e6
        achieved = alg_bytes_local * frames_per_launch / (kernel_ms_avg * 1e-3) / 1e9
        achieved_interval = alg_bytes_local / (elapsed / a.steps) / 1e9
        out = {
            "metric": "Mrays/sec (primary+shadow+reflect), Office 1920x1080 1spp",
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic: fixed-seed office_proxy stand-in (reference Office scene files are absent)"
                     if a.scene == "office" else f"synthetic: fixed-seed {a.scene} scene generator"),
            "config": {
                "workload": f"{a.scene}_proxy {a.width}x{a.height} spp={a.spp * a.spp} depth={params.max_depth} "
                            f"lights={params.n_lights}",
                "triangles": host.triangle_count,
                "bvh": f"host: reference median split, depth {host.bvh_depth}; device: "
                       + {"sah": "binned-SAH hierarchy, 4-wide", "sbvh": "binned SAH with spatial splits, 4-wide",
                          "reference": "reference tree refined, 4-wide"}[a.tree],
                "rays_per_frame": int(rays_total),
                "rays_breakdown_rank0": {"primary": st.primary_rays, "shadow": st.shadow_rays,
                                         "reflection": st.reflection_rays},
                "parallelism": f"row-stripes x{n} (16-row interleave) + RCCL gather" if n > 1 else "single GPU",
                "frames_per_launch": F,
                "launches_in_flight": S,
                "adaptive_pass": adaptive_info,
                "analytic_prims": bool(gpu.analytic),
                "host_bvh_build_s": round(build_s, 4),
                "device_scene_MB": round(gpu.device_bytes / 1e6, 1),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic["bytes_per_launch"] if traffic else None,
                "traffic_detail": traffic,
                "kernel_ms_avg": round(kernel_ms_avg, 4),
                "achieved_per_frame_interval": round(achieved_interval, 1),
                "note": "achieved = alg bytes per launch (frames_per_launch frames) / mean launch duration "
                        "(HIP events on the launch stream); achieved_per_frame_interval = alg bytes per frame / "
                        "(elapsed / steps)",
                "alg_bytes_per_frame": int(alg_bytes_local),
                "alg_bytes_per_launch": int(alg_bytes_local * frames_per_launch),
                "alg_bytes_def": "64*node_visits + 48*tri_tests + 64*closest_hits (rank-0 frame, canonical 2-wide "
                                 "traversal of the reference tree)",
                # The scene (nodes + triangles, a few MB) stays cache-resident: the canonical
                # stream is served by L1 (98 % hits) and L2, so frac vs HBM exceeds 1 (SURVEY §8d
                # caveat).  The binding roof is the CU's L1 data path; it is priced with the
                # bytes the production kernel actually fetches.
                "l1_roof": {"peak": round(L1_PEAK_GBPS, 1), "unit": "GB/s",
                            "fetch_bytes_per_launch": int(fetch_bytes_local * frames_per_launch),
                            "achieved": round(fetch_bytes_local * frames_per_launch / (kernel_ms_avg * 1e-3) / 1e9, 1),
                            "frac": round(fetch_bytes_local * frames_per_launch / (kernel_ms_avg * 1e-3) / 1e9
                                          / L1_PEAK_GBPS, 4),
                            "achieved_per_frame_interval": round(fetch_bytes_local / (elapsed / a.steps) / 1e9, 1),
                            "frac_per_frame_interval": round(fetch_bytes_local / (elapsed / a.steps) / 1e9
                                                             / L1_PEAK_GBPS, 4),
                            "def": "128*wide_node_visits + 80*tri_tests + 96*closest_hits (production kernel)"},
            },
            "cpu_baseline": None,
        }
        if n == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(host, params, a)
        print(json.dumps(out), flush=True)
    if n > 1:
        dist.barrier()
        dist.destroy_process_group()


def pmc_traffic(a, n, F):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary of this exact launch
    shape (profiles/r*/pmc_office1080.json: FETCH_SIZE x 2 (gfx950) + WRITE_SIZE, in bytes,
    production kernel dispatches), or None when this run's shape was not profiled."""
    default = (a.scene == "office" and a.width == 1920 and a.height == 1080 and a.spp == 1 and n == 1
               and not a.adaptive and a.tree == "sbvh")
    if not default:
        return None
    found = sorted(ROOT.glob("profiles/r*/pmc_office1080.json"))
    if not found:
        return None
    d = json.loads(found[-1].read_text())
    if d.get("_frames_per_launch") != F:
        return None
    der = d.get("_derived", {})
    if "hbm_read_bytes_corrected" not in der or "hbm_write_bytes" not in der:
        return None
    return {"bytes_per_launch": int(der["hbm_read_bytes_corrected"] + der["hbm_write_bytes"]),
            "read": int(der["hbm_read_bytes_corrected"]), "write": int(der["hbm_write_bytes"]),
            "source": str(found[-1].relative_to(ROOT))}


def cpu_baseline(host, params, a):
    """CPU oracle (reference CPU renderer restated in C, OpenMP): whole frames of the
    same workload, repeated until --cpu-seconds of CPU work have been timed."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    orc = pyoracle.Oracle(host.raw, host)
    ys = np.arange(0, a.height, a.cpu_row_stride)
    xs = np.arange(a.width)
    xy = np.stack(np.meshgrid(xs, ys), -1).reshape(-1, 2)
    p = host.render_params(a.width, a.height, a.spp)
    rays, frames = 0, 0
    t0 = time.perf_counter()
    while True:
        _, cnt = orc.render_pixels(p, xy, pyoracle.MODE_REFERENCE, threads)
        rays += cnt.primary_rays + cnt.shadow_rays + cnt.reflection_rays
        frames += 1
        dt = time.perf_counter() - t0
        if dt >= a.cpu_seconds:
            break
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(rays / dt / 1e6, 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{frames} x (every {a.cpu_row_stride}th row of the frame: {len(xy)} pixels), {rays} rays, "
                  f"{dt:.2f} s; reference-CPU-semantics oracle (recursive unordered fp64 BVH, "
                  f"closest-hit shadows, OpenMP over pixels)",
        "cpu_model": cpu_model,
        "nproc": os.cpu_count(),
        "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
    }


if __name__ == "__main__":
    main()
