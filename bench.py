"""bench.py — Mrays/s of the MI355X render path on the Office workload.

Metric (BASELINE.json): Mrays/sec (primary + shadow + reflection), Office
1920x1080 1 spp, on 1/2/4/8 MI355X.  The Office scene files are not in the
reference, so the workload is the fixed-seed office_proxy.

One step = one full frame: every rank renders its interleaved 16-row stripes
(stripe = rank mod N) with one launch of the flattened HIP kernel, then rank 0
gathers the stripes over RCCL (torch.distributed "nccl") and re-interleaves
them into the final image.  Total work per step is fixed => "strong" scaling.
Consecutive frames are rendered --frames at a time (default 128, at most --steps; at N > 1
at most half of --steps, so the timed run has two launches or more and each gather overlaps the
next launch) by ONE launch of the persistent kernel (rt_launch_frames: the frames share one
work queue, so the drain at the end of a launch is paid once per F frames).  The
F frames of a launch follow an animation path (rtamd.camera_orbit, --sweep): they
are distinct views, and every frame traces all of its rays.  A single_frame record
(one frame per launch, the reference's use, mytracer_gpu.cu:59-81; consecutive views of
the orbit) is timed after the main run with the library's default for such launches on one
stream -- cost-ordered work (each launch's work heads take first the tiles that took longest
two launches before, shortening the drain) -- and beside it
single_frame.natural_order: the same launches with RT_FLAG_NATURAL_ORDER; single_frame.pipelined: the
same one-frame launches with --pipeline (3) of them in flight on streams of their own (the throughput
of the reference's call shape for a caller that keeps frames in flight).  --streams S > 1 keeps S launches in flight on separate streams
(default 1 on one GPU: launches serial, so the HIP-event launch duration is the
kernel's own duration, as rocprofv3 reports it; 2 on N > 1, so the RCCL gather of
launch i overlaps launch i+1).

Rays are the canonical counts returned by the kernel's counters in
untimed launches of exactly the timed launch shapes.  Roofline:
`traffic` = HBM bytes per launch from the committed rocprofv3 --pmc summary of
this workload (FETCH_SIZE/WRITE_SIZE per frame x frames per launch), `achieved`
= traffic / the HIP-event launch duration, `frac` = achieved / 8 TB/s.  The
canonical SURVEY §8d bytes (64*node_visits + 48*tri_tests + 64*closest_hits over
the reference tree) are reported as `work_bytes_per_frame`, and `l1_roof` prices
the production kernel's own fetches against the CU vector-L1 data path, the
binding resource.

cpu_baseline: the CPU oracle (C restatement of the reference's CPU renderer:
recursive unordered fp64 BVH traversal, closest-hit shadow rays, OpenMP on every
CPU this process may use) timed on whole frames of the same workload, rank 0 /
N=1 only.

N > 1 (one process per GPU): under a launcher (torch.distributed.run sets WORLD_SIZE, which must
equal --gpus), or without one: `python bench.py --gpus N` then starts the N ranks itself as child
processes (torch.distributed.run, 127.0.0.1) before it makes any GPU call, and exits with their
status; rank 0 prints the JSON line.  The N > 1 line carries a multi_gpu record: the render and
gather time of each launch (HIP events on the launch stream, max over ranks) and the same run with
the other reserve_cus setting (0 / 32 CUs left free for the gather).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
import rtamd  # noqa: E402
from rtamd.shard import HaloExchange, PeerFrames, StripeGather, max_rows as shard_max_rows  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# The CU's vector-L1 data return (TD): one 64-lane dwordx4 wave-instruction per 16 cycles =
# 64 B/clk/CU (tools/l1_micro.hip) x 256 CUs x 2.4 GHz.
L1_PEAK_GBPS = 64 * 256 * 2.4
L1_PEAK_SOURCE = ("measured, not a datasheet figure (MI355X_MICROARCH.md gives none): tools/l1_micro.hip, an "
                  "L1-resident dependent gather, 16 cycles of a CU's TD per 64-lane dwordx4 wave-instruction "
                  "touching <= 16 lines = 64 B/clk/CU (profiles/r05/l1_micro_r05.txt)")
# roofline.bound vocabulary: the resource whose measured fraction of its peak is at least
# BOUND_FRAC ("hbm": HBM bytes, "l1": vector-L1 data return, "valu": VALU issue); none of them, with
# the HBM and VALU fractions both measured -> "latency" (each wave's dependent chain of fetches and
# ALU at 4 waves per SIMD); none of them and one of those two not measured (no
# committed PMC summary for the workload) -> "unmeasured"
BOUND_FRAC = 0.8
BOUND_VOCAB = ("hbm", "l1", "valu", "latency", "unmeasured")
# VALU issue (MI355X_MICROARCH.md, "Per-instruction cycle constants"): a SIMD-32 issues a 32-bit
# wave64 VALU instruction in 2 cycles (4 cycles is what ONE wave alone sustains), an fp64 one in 4
# (16 lanes per cycle: 78.6 TF fp64 = half the fp32 rate), a transcendental in 8 (the issue-cost
# row); 1024 SIMDs at 2.4 GHz.  valu_roof prices each class by its own cycles.
VALU_SIMDS = 256 * 4
VALU_CLOCK_GHZ = 2.4
VALU_CYCLES = {"b32": 2, "f64": 4, "trans64": 8}
STRIPE_H = 16
PIPE_REPS = 4   # single_frame.pipelined: passes over the single-frame views


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
    ap.add_argument("--cpu-row-stride", type=int, default=0,
                    help="cpu_baseline renders every k-th row (default: 1, or 16 when one whole frame would take "
                         "longer than --cpu-seconds on this host, e.g. BASELINE configs 3-5; the frame time is then "
                         "extrapolated from the sample)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="cpu_baseline: minimum timed CPU work")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="cpu_baseline threads (default: every CPU this process may run on, see usable_cpus)")
    ap.add_argument("--save", default="", help="rank 0: save the gathered image of the last frame (.npy)")
    ap.add_argument("--frames", type=int, default=0,
                    help="frames per launch (rt_launch_frames, <= RT_MAX_FRAMES = 128, <= --steps; default: "
                         "default_frames(), 128 at 1 spp): one persistent-kernel launch renders F consecutive "
                         "frames from one work queue, so the per-launch drain is paid once per F")
    ap.add_argument("--sweep", type=float, default=0.12,
                    help="animation path: frame f of a launch turns the camera by sweep*(f/(F-1) - 1/2) radians "
                         "about the image's vertical axis (rtamd.camera_orbit), so the batched frames are distinct "
                         "views; 0 = every frame the same camera")
    ap.add_argument("--single-frames", type=int, default=16,
                    help="after the timed run: this many one-frame launches, timed the same way (single_frame record)")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="one GPU: after the single-frame records, the same one-frame launches with this many in "
                         "flight on streams of their own (single_frame.pipelined); <= 1 = off")
    ap.add_argument("--frame-budget-gb", type=float, default=8.0,
                    help="device memory for one stream's frame buffers; caps frames per launch at large sizes")
    ap.add_argument("--streams", type=int, default=0,
                    help="launches in flight on separate streams (1 = launches strictly serial; default 1 on "
                         "one GPU, 2 on N > 1 so the RCCL gather of one launch overlaps the next launch)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: nccl (RCCL over xGMI, the measured path) or gloo (host-staged rehearsal)")
    ap.add_argument("--tree", choices=["sah", "sbvh", "reference"], default=os.environ.get("RT_BENCH_TREE", "sbvh"),
                    help="device traversal hierarchy (pixels identical either way; DESIGN.md §4)")
    ap.add_argument("--tree-record", choices=["auto", "on", "off"], default="auto",
                    help="after the timed run, time the same run shape on other device hierarchies (the "
                         "reference median-split tree of BASELINE config 2, mybvh.cpp:375-539, and the SAH tree) "
                         "and report each with its upload / build seconds (tree_records); auto = on for one GPU, "
                         "scenes below 2^20 triangles, no --adaptive")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="rt_upload_options.reserve_cus: CUs each render launch leaves free (its grid on an internal "
                         "CU-masked stream), so the RCCL gather of the previous launch can run beside it instead of "
                         "after it (DESIGN.md §8); default 0 (32 = one XCD's worth costs ~12 %% of the render)")
    ap.add_argument("--reserve-ab", choices=["auto", "on", "off"], default="auto",
                    help="N > 1: after the timed run, time the same run again with the other reserve_cus setting "
                         "(32 if the run used 0, else 0) and report both (multi_gpu.reserve_cus_ab); auto = on at N > 1")
    ap.add_argument("--assembly", choices=["auto", "gather", "peer"], default="auto",
                    help="N > 1 frame assembly on rank 0: gather = one RCCL gather of every launch's stripes + "
                         "re-interleave; peer = every rank's render writes its stripes straight into rank 0's frame "
                         "over xGMI (RT_FLAG_GLOBAL_ROWS, IPC-mapped buffers) and one RCCL all_reduce per launch "
                         "fences it (rtamd.shard.PeerFrames); auto (default) = before the warm-up, two untimed "
                         "launches in each, the faster one if both assembled bit-identical frames, else gather "
                         "(multi_gpu.assembly_choice)")
    ap.add_argument("--assembly-ab", choices=["auto", "on", "off"], default="auto",
                    help="N > 1: after the timed run, time the same run with the other assembly and check that both "
                         "assemble bit-identical frames (multi_gpu.assembly_ab); auto = on at N > 1 without --adaptive")
    ap.add_argument("--rank-shape", type=int, default=0, metavar="N",
                    help="one process, one GPU: render exactly what rank 0 of an N-GPU run renders (its 16-row "
                         "stripes of every frame, the N > 1 launch shape: frames per launch of the RCCL gather "
                         "assembly, two launches in flight) with no collective, so rocprofv3 can profile the N-GPU "
                         "rank shape on one GPU; the line's workload_key carries n_gpus = N, so an N-GPU run finds "
                         "the PMC summary of this shape (roofline at N > 1).  value = this shard's rays/s")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks (--gpus N), join a gloo process group, check its size, print one JSON line "
                         "and exit before any GPU call (a dry run of the N-rank launch)")
    ap.add_argument("--opt", action="append", default=[], metavar="FIELD=VALUE",
                    help="dev A/B: an rt_upload_options field (e.g. lds_treelet=9); pixels are identical")
    ap.add_argument("--analytic", action="store_true",
                    help="also trace the scene's spheres/planes (always on for --scene spheres)")
    ap.add_argument("--adaptive", action="store_true",
                    help="each frame = primary pass + adaptive supersampling pass (subp 4, threshold 0.02, "
                         "mytracer_gpu.cu:83-109); N > 1: stripe-edge halo rows exchanged by one all_gather per frame")
    return ap.parse_args()


def workload_key(a, n):
    """Identity of the profiled workload: the PMC summary of a run applies to runs with the same key."""
    return {"scene": a.scene, "tris": a.tris, "width": a.width, "height": a.height, "spp": a.spp, "tree": a.tree,
            "sweep": a.sweep if (not a.adaptive or n == 1) else 0.0, "adaptive": bool(a.adaptive),
            "analytic": bool(a.analytic or a.scene == "spheres"), "n_gpus": n}


def free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(a):
    """--gpus N > 1 without a launcher: start the N ranks as children of this process
    (python -m torch.distributed.run, rendezvous on 127.0.0.1) and return their exit status.
    Called before this process makes any GPU call (torch.cuda.device_count() does not initialise
    the GPU on this image), and the ranks are child processes, not an exec of this one.  Rank 0's
    JSON line reaches this process's stdout.  Fewer visible GPUs than N is an error (exit 2),
    unless RT_BENCH_DEVICE pins every rank to one device (dev rehearsal with --dist-backend gloo)."""
    if "RT_BENCH_DEVICE" not in os.environ and not a.launch_check:
        have = torch.cuda.device_count()
        if have < a.gpus:
            print(f"bench.py: --gpus {a.gpus} but {have} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(Path(__file__).resolve()),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL across processes)
    env.setdefault("OMP_NUM_THREADS", str(max(1, usable_cpus() // a.gpus)))
    return subprocess.run(cmd, env=env).returncode


def launch_check(a, n, rank):
    """--launch-check: the ranks exist and agree on the world size; no GPU call."""
    ws = 1
    if n > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
        ws = dist.get_world_size()
        ranks = [None] * ws
        dist.all_gather_object(ranks, (rank, os.getpid()))
    else:
        ranks = [(0, os.getpid())]
    if ws != a.gpus:
        raise SystemExit(f"bench.py: world size {ws} but --gpus {a.gpus}")
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": ws, "ranks": sorted(r for r, _ in ranks),
                          "distinct_pids": len({p for _, p in ranks}), "parent_pid": os.getppid()}), flush=True)
    if n > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    if "WORLD_SIZE" in os.environ:   # under a launcher: one process per GPU
        world = int(os.environ["WORLD_SIZE"])
        if world != a.gpus:
            raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}")
    elif a.gpus > 1:                 # no launcher: start the ranks, before any GPU call
        sys.exit(spawn_ranks(a))
    else:
        world = 1
    if a.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = world
    if a.launch_check:
        return launch_check(a, n, rank)
    if a.rank_shape and (n > 1 or a.rank_shape < 2 or a.adaptive):
        raise SystemExit("bench.py: --rank-shape N (N >= 2) is a one-process run without --adaptive")
    # the stripe partition and launch shape of this process: N > 1 ranks, or rank 0 of --rank-shape N
    shape_n = a.rank_shape or n
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
        if dist.get_world_size() != a.gpus:
            raise SystemExit(f"bench.py: process group of {dist.get_world_size()} ranks but --gpus {a.gpus}")
    host_staged = a.dist_backend == "gloo"

    # ---- host side: scene, normals, SoA, median-split BVH (untimed) ----
    gen = {"n_triangles": a.tris} if a.scene == "random_tris" and a.tris else {}
    host = rtamd.HostScene.generate(a.scene, **gen)
    build_s = host.prepare()
    upload_opts = upload_options_for(a, n)
    t_up = time.perf_counter()
    gpu = rtamd.DeviceScene(host, device=dev, analytic=a.analytic or a.scene == "spheres",
                             tree=a.tree, **upload_opts)
    upload_wall_s = time.perf_counter() - t_up
    dev_build_s, dev_copy_s = gpu.upload_seconds
    params = host.render_params(a.width, a.height, a.spp)
    params.stripe_height = STRIPE_H
    params.stripe_count = shape_n
    params.stripe_index = rank
    W = a.width
    rows_max = shard_max_rows(a.height, STRIPE_H, shape_n)
    # librt_hip keeps 8 launch contexts per scene; the halo exchange of --adaptive is single-stream
    S = 1 if a.adaptive else max(1, min(a.streams or (1 if shape_n == 1 else 2), 8))
    # --adaptive on one GPU: F frames per launch for both passes (rt_launch_frames for the fp64
    # primary images, rt_launch_adaptive_frames for the supersampling of all F frames); on N > 1
    # one frame per launch (the halo exchange is per frame)
    batched_adaptive = a.adaptive and n == 1
    frame_bytes = rows_max * W * 3 * (4 + (8 if a.adaptive else 0))
    F = 1 if (a.adaptive and not batched_adaptive) else max(1, min(a.frames or default_frames(a), rtamd.abi.RT_MAX_FRAMES,
                                                                   a.steps,
                                                                   int(a.frame_budget_gb * 1e9 // frame_bytes)))

    def per_launch_of(mode):
        """Frames per launch of the timed run.  N > 1 with the RCCL gather: at most half the steps,
        so the run has two launches and the gather of one can overlap the next launch; the peer
        assembly has nothing to overlap, so its frames go in launches of F (one drain per F)."""
        if shape_n > 1 and mode == "gather" and not a.frames and not a.adaptive:
            return min(F, max(1, (a.steps + 1) // 2))
        return F
    # the animation path: frame f of every launch (the batched frames are distinct views)
    if F > 1 and a.sweep != 0.0:
        cams = [rtamd.camera_orbit(params, a.sweep * (f / (F - 1) - 0.5)) for f in range(F)]
    else:
        cams = [params] * F
    # per stream: the F frames of one launch, contiguous, so one collective gathers them
    fbufs = [torch.zeros((F, rows_max, W, 3), dtype=torch.float32, device="cuda") for _ in range(S)]
    bufs = [fb[f] for fb in fbufs for f in range(F)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(S - 1)]
    stream = streams[0].cuda_stream
    rows_local = rtamd.rows_in_shard(params)
    prims = [torch.zeros((F, rows_max, W, 3), dtype=torch.float64, device="cuda")
             for _ in range(S)] if a.adaptive else []
    p64s = []   # the primary pass of --adaptive renders fp64 images (the selection reads fp64 colours)
    for c in cams:
        q = rtamd.abi.RenderParams.from_buffer_copy(c)
        q.out_format = rtamd.RT_OUT_RGB_F64
        p64s.append(q)
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

    def adaptive_frames(prim, outs, nf, stats, stream_):
        """One GPU: the primary passes of nf frames (fp64, one launch), then their adaptive passes
        (one launch); returns (Stats of the adaptive pass, pixels supersampled)."""
        gpu.launch_frames(p64s[:nf], [prim[f].data_ptr() for f in range(nf)], stats=False, stream=stream_)
        return gpu.launch_adaptive_frames(cams[:nf], [prim[f].data_ptr() for f in range(nf)],
                                          [o.data_ptr() for o in outs[:nf]], 4, 0.02, stats=stats, stream=stream_)

    # ---- counters (untimed launches of exactly the timed launch shapes) ----
    # rays of one launch of nf frames (frames cams[:nf]); the timed run is full launches of F frames
    # plus one of steps % F frames
    def launch_counts(nf, flags=0):
        ps = [rtamd.abi.RenderParams.from_buffer_copy(c) for c in cams[:nf]]
        for q in ps:
            q.flags = flags
        if nf == 1:
            return gpu.launch(ps[0], bufs[0].data_ptr(), stats=True, stream=stream)
        return gpu.launch_frames(ps, [b.data_ptr() for b in bufs[:nf]], stats=True, stream=stream)

    def rays_of(st):
        return st.primary_rays + st.shadow_rays + st.reflection_rays

    n_full, rem = divmod(a.steps, F)
    st = launch_counts(F)
    rays_cache = {}
    counts_cache = {F: st}   # ray counts of a launch of nf frames (deterministic): one counting launch per shape

    def counts_of(nf):
        if nf not in counts_cache:
            counts_cache[nf] = launch_counts(nf)
        return counts_cache[nf]

    def rays_timed_for(pl):
        """This rank's rays in a.steps frames rendered pl at a time (launches of frames cams[:pl])
        -- from untimed counting launches of exactly those shapes."""
        if pl not in rays_cache:
            nf_, rm_ = divmod(a.steps, pl)
            rays_cache[pl] = nf_ * rays_of(counts_of(pl)) + (rays_of(counts_of(rm_)) if rm_ else 0)
        return rays_cache[pl]
    rays_adaptive_local = 0
    # the single-frame records render frames cams[0 .. NS) one per launch (an animation: distinct views)
    NS = max(1, min(a.single_frames, F))
    rays_frame0_local = rays_of(counts_of(NS)) / NS  # rays per frame of those frames
    tst = launch_counts(F, rtamd.RT_FLAG_TRAVERSAL_STATS)   # canonical 2-wide walk of the reference tree
    wst = launch_counts(F, rtamd.RT_FLAG_WIDE_STATS)        # the production kernel's own fetches
    adaptive_info = None
    if batched_adaptive:   # untimed: rays of the adaptive passes (selection depends on the primary images)
        ast, nsel = adaptive_frames(prims[0], bufs, F, True, stream)
        rays_adaptive_local += n_full * rays_of(ast) + (rays_of(adaptive_frames(prims[0], bufs, rem, True, stream)[0])
                                                        if rem else 0)
        rays_frame0_local += rays_of(adaptive_frames(prims[0], bufs, 1, True, stream)[0])
        adaptive_info = {"pixels_supersampled_per_frame": round(nsel / F, 1), "subp": 4, "threshold": 0.02,
                         "rays_per_frame": round(rays_of(ast) / F, 1), "frames_per_launch": F}
    elif a.adaptive:
        gpu.launch(p64s[0], prims[0][0].data_ptr(), stats=True, stream=stream)
        ast, nsel = adaptive_pass(prims[0][0], bufs[0], True, stream)
        rays_adaptive_local += a.steps * rays_of(ast)
        rays_frame0_local += rays_of(ast)
        adaptive_info = {("pixels_supersampled" if n == 1 else "pixels_supersampled_rank0"): nsel, "subp": 4,
                         "threshold": 0.02, "rays": rays_of(ast)}
    # per frame, averaged over the F frames of a launch
    work_bytes_frame = (64 * tst.node_visits + 48 * tst.tri_tests + 64 * tst.closest_hits) / F
    fetch_bytes_frame = (128 * wst.node_visits + 80 * wst.tri_tests + 96 * wst.closest_hits) / F

    if a.rank_shape:   # rank 0's stripes stay where they are rendered: no collective in this shape
        gathers = [lambda b: b] * S
    else:
        gathers = [StripeGather(a.height, W, STRIPE_H, n, rank, device="cuda", frames=F, host_staged=host_staged)
                   for _ in range(S)]
    image = None
    # N > 1 assembly by peer stores (--assembly peer): rank 0's whole frames, mapped by every rank;
    # the launches write global rows (RT_FLAG_GLOBAL_ROWS)
    if a.adaptive and a.assembly == "peer":
        raise SystemExit("bench.py: --assembly peer does not support --adaptive")
    assembly = a.assembly if n > 1 and not a.adaptive else "gather"
    peer = None

    def peer_frames():
        nonlocal peer
        if peer is None:
            peer = PeerFrames(a.height, W, n, rank, device="cuda", frames=F, slots=S)
        return peer

    def global_rows(c):
        q = rtamd.abi.RenderParams.from_buffer_copy(c)
        q.flags |= rtamd.abi.RT_FLAG_GLOBAL_ROWS
        return q
    cams_g = [global_rows(c) for c in cams]

    starts, ends, launch_frames = [], [], []
    gstarts, gends = [], []   # N > 1: HIP events around each launch's gather + re-interleave

    warmed = set()   # streams that have carried a launch (a stream's first launch pays set-up)

    def launch(li, nf, timed, flags=0):
        """Launch li renders nf frames (steps); their stripes are then gathered to rank 0 (or, with
        the peer assembly, written there by the render itself and fenced).  A one-frame launch
        renders view cams[li % F] (the single-frame records: consecutive frames of the orbit)."""
        nonlocal image
        s = streams[li % S]
        warmed.add(li % S)
        bs = [fbufs[li % S][f] for f in range(nf)]
        if assembly == "peer":
            outs = peer_frames().outs(li % S, nf)
            with torch.cuda.stream(s):
                if timed:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                if nf == 1:
                    c1 = cams_g[li % len(cams_g)]
                    if flags:
                        c1 = rtamd.abi.RenderParams.from_buffer_copy(c1)
                        c1.flags = flags | rtamd.abi.RT_FLAG_GLOBAL_ROWS
                    gpu.launch(c1, outs[0], stats=False, stream=s.cuda_stream)
                else:
                    gpu.launch_frames(cams_g[:nf], outs, stats=False, stream=s.cuda_stream)
                if timed:
                    e1.record(s)
                    starts.append(e0)
                    ends.append(e1)
                    launch_frames.append(nf)
                    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    g0.record(s)
                peer.fence()   # the frames are whole on rank 0 once every rank's render has ended
                if timed:
                    g1.record(s)
                    gstarts.append(g0)
                    gends.append(g1)
                img = peer.image(li % S)
                image = img[:nf] if img is not None else None
            return
        with torch.cuda.stream(s):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
            if batched_adaptive:
                adaptive_frames(prims[li % S], bs, nf, False, s.cuda_stream)
            elif a.adaptive:
                gpu.launch(p64s[0], prims[li % S][0].data_ptr(), stats=False, stream=s.cuda_stream)
                adaptive_pass(prims[li % S][0], bs[0], False, s.cuda_stream)
            elif nf == 1:
                c1 = cams[li % len(cams)]
                if flags:
                    c1 = rtamd.abi.RenderParams.from_buffer_copy(c1)
                    c1.flags = flags
                gpu.launch(c1, bs[0].data_ptr(), stats=False, stream=s.cuda_stream)
            else:
                gpu.launch_frames(cams[:nf], [b.data_ptr() for b in bs], stats=False, stream=s.cuda_stream)
            if timed:
                e1.record(s)
                starts.append(e0)
                ends.append(e1)
                launch_frames.append(nf)
            # N>1: ONE RCCL gather of the nf frames' stripes + re-interleave
            if timed and n > 1:
                g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                g0.record(s)
            image = gathers[li % S](fbufs[li % S][:nf])
            if timed and n > 1:
                g1.record(s)   # the gather's end: the stream waits for the collective (and rank 0's copies)
                gstarts.append(g0)
                gends.append(g1)

    def run(steps, timed, per_launch=None, flags=0):
        per_launch = per_launch or per_launch_of(assembly)
        li, done = 0, 0
        while done < steps:
            nf = min(per_launch, steps - done)
            launch(li, nf, timed, flags)
            li += 1
            done += nf

    def timed_region(fn):
        torch.cuda.synchronize()
        if n > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if n > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tmax = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        if n > 1:
            dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        return float(tmax[0])

    stream_warm_frames = 0   # one-frame launches that only warmed a stream (counted below)

    def timed_run(warm):
        """warm-up frames, then the timed run of a.steps frames: (seconds (max over ranks), mean
        launch ms, mean gather ms); the per-launch event lists are refilled."""
        nonlocal stream_warm_frames
        for lst in (starts, ends, launch_frames, gstarts, gends):
            lst.clear()
        run(warm, False)
        # every stream the timed run uses has carried a launch before it: a stream's first launch
        # pays its hardware queue's set-up (r05zv: two 10-frame launches on two streams, the second
        # stream new, 10.1 ms against 8.0 ms of launch time)
        for i in range(min(S, -(-a.steps // per_launch_of(assembly)))):
            if i not in warmed:
                launch(i, 1, False)
                stream_warm_frames += 1
        el = timed_region(lambda: run(a.steps, True))
        k_ms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in zip(starts, ends)]))
        g_ms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in zip(gstarts, gends)])) if gstarts else 0.0
        return el, k_ms, g_ms

    def same_frames(x, y):
        """Bitwise equality of two assembled launches' frames (rank 0), over the frames both
        rendered: a launch of nf frames renders views cams[:nf]."""
        k = min(x.shape[0], y.shape[0])
        return torch.equal(x[:k], y[:k])

    def choose_assembly():
        """--assembly auto (N > 1): both assemblies render the same two launches of F frames (after one
        warm-up launch each, untimed for the result); peer wins if it was faster and its frames equal the
        gather's bit for bit on rank 0.  A rank that cannot map rank 0's frames makes it gather."""
        nonlocal assembly
        err = ""
        try:
            peer_frames()
        except Exception as e:   # IPC mapping refused on this rank
            err = repr(e)
        ok = torch.tensor([0.0 if err else 1.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok[0] < 1.0:
            return "gather", {"chosen": "gather", "reason": "peer mapping failed" + (f" here: {err}" if err else
                                                                                       " on another rank")}
        secs, frames = {}, {}
        for mode in ("gather", "peer"):
            assembly = mode
            run(F, False)
            secs[mode] = timed_region(lambda: run(2 * F, False))
            frames[mode] = image.clone() if rank == 0 else None
        same = torch.tensor([float(same_frames(frames["gather"], frames["peer"])) if rank == 0 else 0.0],
                            dtype=torch.float64, device="cuda")
        dist.broadcast(same, src=0)
        identical = bool(same[0] == 1.0)
        chosen = "peer" if identical and secs["peer"] < secs["gather"] else "gather"
        return chosen, {"chosen": chosen, "frames_identical": identical,
                        "calibration_ms_per_frame": {k: round(v / (2 * F) * 1e3, 4) for k, v in secs.items()},
                        "rule": "two untimed launches of F frames in each assembly; peer if faster and bit-identical"}

    assembly_choice = None
    if assembly == "auto":
        assembly, assembly_choice = choose_assembly()
    rays_timed_local = rays_timed_for(per_launch_of(assembly)) + rays_adaptive_local
    elapsed, kernel_ms_avg, gather_ms_avg = timed_run(a.warmup)
    frames_per_launch = float(np.mean(launch_frames))
    last_image = image

    def over_ranks(vals):
        """[max over ranks, rank 0's] of each value (N > 1)."""
        t = torch.tensor(vals, dtype=torch.float64, device="cuda")
        r0 = t.clone()
        if n > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.broadcast(r0, src=0)
        return [(float(x), float(y)) for x, y in zip(t, r0)]

    multi = None
    if n > 1:
        (k_max, k_r0), (g_max, g_r0) = over_ranks([kernel_ms_avg, gather_ms_avg])
        multi = {"render_ms_per_launch_max": round(k_max, 4), "render_ms_per_launch_rank0": round(k_r0, 4),
                 "gather_ms_per_launch_rank0": round(g_r0, 4), "gather_ms_per_launch_max": round(g_max, 4),
                 "frames_per_launch": frames_per_launch,
                 "gather_MB_per_launch_into_rank0": round((n - 1) * frames_per_launch * rows_max * W * 3 * 4 / 1e6, 2),
                 "reserve_cus": int(upload_opts.get("reserve_cus", 0)),
                 "assembly": assembly,
                 "assembly_choice": assembly_choice,
                 "def": "render = HIP events around each launch on its stream; gather = HIP events around the "
                        "collective of its frames' stripes + rank 0's re-interleave (peer assembly: around the "
                        "fence all_reduce) -- includes waiting for the slowest rank's render; means over the "
                        "timed launches, then max over ranks"}
        main_frames = last_image.clone() if rank == 0 else None   # for the assembly A/B's bit check

    # single-frame record: the reference's use, one frame per launch (mytracer_gpu.cu:59-81)
    # (NS consecutive views of the orbit, one per launch) in the natural tile order, then with the
    # library's default for consecutive one-frame launches on a stream: each launch ordered by the
    # per-tile costs of the launch two before (one untimed pass of the NS views first)
    single = None
    if a.single_frames > 0 and not a.adaptive:
        def single_record(flags):
            for lst in (starts, ends, launch_frames, gstarts, gends):
                lst.clear()
            el = timed_region(lambda: run(NS, True, per_launch=1, flags=flags))
            return {"frames": NS, "rays_per_frame": None, "ms_per_frame": round(el / NS * 1e3, 4),
                    "kernel_ms_avg": round(float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)])), 4)}
        natural = single_record(rtamd.abi.RT_FLAG_NATURAL_ORDER)
        run(NS, False, per_launch=1)
        single = single_record(0)
        single["order"] = ("cost-ordered (library default on one stream)" if S == 1 else
                           "natural (launches alternate streams)")
        single["natural_order"] = natural
        single["views"] = "consecutive camera-orbit views, one per launch"
        # the same call shape with a.pipeline launches in flight (one stream each, round robin): a
        # caller that keeps frames in flight lets launch i+1's waves fill launch i's drain, which
        # serial one-frame launches pay in full (r05zv: 0.417 ms -> 0.349 / 0.338 ms per frame at
        # 2 / 3 in flight).  The streams are not the cost maps' stream, so the order is natural
        if n == 1 and S == 1 and a.pipeline > 1:
            pst = [torch.cuda.Stream() for _ in range(a.pipeline)]
            pbuf = [torch.empty((rows_max, W, 3), dtype=torch.float32, device="cuda") for _ in range(a.pipeline)]

            def pipelined():
                for li in range(PIPE_REPS * NS):
                    gpu.launch(cams[li % NS], pbuf[li % a.pipeline].data_ptr(), stats=False,
                               stream=pst[li % a.pipeline].cuda_stream)
            pipelined()
            el = timed_region(pipelined)
            single["pipelined"] = {"launches_in_flight": a.pipeline, "frames": PIPE_REPS * NS,
                                   "ms_per_frame": round(el / (PIPE_REPS * NS) * 1e3, 4),
                                   "order": "natural (streams other than the cost maps' stream)",
                                   "views": f"the {NS} views above, {PIPE_REPS} times"}

    # other device hierarchies over the same records (pixels and ray counts are identical for every
    # tree, tests/test_gpu_parity.py::test_device_tree_changes_no_pixel): the same run shape, timed the
    # same way, with each tree's upload / build seconds -- BASELINE config 2 names the reference's
    # median-split tree (mybvh.cpp:375-539, walked by intersectBVH_device, mytracer_gpu.cu:340-424)
    tree_records = None
    if a.tree_record == "on" or (a.tree_record == "auto" and n == 1 and not a.adaptive
                                 and host.triangle_count < (1 << 20)):
        tree_records = {}
        for tree in [t for t in ("reference", "sah", "sbvh") if t != a.tree]:
            tree_records[tree] = tree_record(host, dev, a, upload_opts, tree, cams, F, fbufs[0], stream,
                                             rays_of(st), timed_region)
    tot = torch.tensor([rays_timed_local, rays_frame0_local, work_bytes_frame], dtype=torch.float64, device="cuda")
    if n > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    rays_total, rays_frame0 = float(tot[0]), float(tot[1])

    # N > 1: the same run with the other frame assembly (RCCL gather <-> peer stores + fence), and
    # the last launch's assembled frames compared bit for bit with the main run's (same views)
    peer_failed = bool(assembly_choice and assembly_choice.get("reason"))
    if peer_failed:
        multi["assembly_ab"] = {"skipped": assembly_choice["reason"]}
    elif multi is not None and (a.assembly_ab == "on" or (a.assembly_ab == "auto" and not a.adaptive)):
        main_as = assembly
        assembly = "peer" if main_as == "gather" else "gather"
        el2, k2, g2 = timed_run(min(a.warmup, F))
        (el2_max, _), (k2_max, _), (g2_max, g2_r0) = over_ranks([el2, k2, g2])
        same = torch.tensor([1.0 if rank != 0 else float(same_frames(image, main_frames)),
                             rays_timed_for(per_launch_of(assembly))], dtype=torch.float64, device="cuda")
        if n > 1:
            dist.broadcast(same[:1], src=0)
            dist.all_reduce(same[1:], op=dist.ReduceOp.SUM)
        rays_other = float(same[1])
        multi["assembly_ab"] = {
            main_as: {"value": round(rays_total / elapsed / 1e6, 2), "ms_per_step": round(elapsed / a.steps * 1e3, 4),
                      "render_ms_per_launch_max": multi["render_ms_per_launch_max"],
                      "gather_ms_per_launch_rank0": multi["gather_ms_per_launch_rank0"]},
            assembly: {"value": round(rays_other / el2_max / 1e6, 2), "ms_per_step": round(el2_max / a.steps * 1e3, 4),
                       "frames_per_launch": per_launch_of(assembly),
                       "render_ms_per_launch_max": round(k2_max, 4), "gather_ms_per_launch_rank0": round(g2_r0, 4)},
            "frames_identical": bool(same[0] == 1.0)}
        assembly = main_as
        main_frames = None

    # N > 1: the same run with the other reserve_cus setting (0 <-> 32 CUs left free for the
    # gather), so every N > 1 line measures what the reservation costs the render and what it
    # gains the gather overlap -- same scene, same launches, pixels identical
    if multi is not None and (a.reserve_ab == "on" or (a.reserve_ab == "auto" and not a.adaptive)):
        main_r = multi["reserve_cus"]
        other = 32 if main_r <= 0 else 0
        gpu.close()
        err = ""
        try:   # the CU-masked streams are created (and their masks read back) at the first launch
            gpu = rtamd.DeviceScene(host, device=dev, analytic=a.analytic or a.scene == "spheres", tree=a.tree,
                                    **dict(upload_opts, reserve_cus=other))
            gpu.launch(cams[0], bufs[0].data_ptr(), stats=False, stream=stream)
            torch.cuda.synchronize()
        except Exception as e:   # every rank learns of it before any further collective
            err = repr(e)
        ok = torch.tensor([0.0 if err else 1.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok[0] < 1.0:
            multi["reserve_cus_ab"] = {"skipped": f"reserve_cus {other} failed" +
                                                  (f" here: {err}" if err else " on another rank")}
        else:
            el2, k2, g2 = timed_run(min(a.warmup, F))
            (el2_max, _), (k2_max, _), (g2_max, g2_r0) = over_ranks([el2, k2, g2])
            multi["reserve_cus_ab"] = {
                str(main_r): {"value": round(rays_total / elapsed / 1e6, 2), "ms_per_step": round(elapsed / a.steps * 1e3, 4),
                              "render_ms_per_launch_max": multi["render_ms_per_launch_max"],
                              "gather_ms_per_launch_rank0": multi["gather_ms_per_launch_rank0"]},
                str(other): {"value": round(rays_total / el2_max / 1e6, 2),
                             "ms_per_step": round(el2_max / a.steps * 1e3, 4),
                             "render_ms_per_launch_max": round(k2_max, 4), "gather_ms_per_launch_rank0": round(g2_r0, 4)}}

    if rank == 0:
        if a.save:
            img = last_image[-1] if last_image.dim() == 4 else last_image
            np.save(a.save, img.float().cpu().numpy())
        ms_per_step = elapsed / a.steps * 1e3
        mrays = rays_total / elapsed / 1e6
        if single is not None:
            for rec in (single, single["natural_order"]) + ((single["pipelined"],) if "pipelined" in single else ()):
                rec["rays_per_frame"] = int(rays_frame0)
                rec["value"] = round(rays_frame0 / (rec["ms_per_frame"] * 1e-3) / 1e6, 2)
                rec["unit"] = "Mrays/s"
        # (N > 1: the PMC summary of the rank shape -- rank 0's launches profiled on one GPU with
        # --rank-shape N -- so the fractions are per GPU, of rank 0's kernel)
        key = workload_key(a, shape_n)
        pmc = pmc_per_frame(key, frames_per_launch)
        kernel_s = kernel_ms_avg * 1e-3
        roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": None,
                "traffic": None}
        if pmc is not None:
            traffic = (pmc["read"] + pmc["write"]) * frames_per_launch
            roof["traffic"] = int(traffic)
            roof["achieved"] = round(traffic / kernel_s / 1e9, 1)
            roof["frac"] = round(traffic / kernel_s / 1e9 / HBM_PEAK_GBPS, 4)
            roof["traffic_detail"] = {"read_per_frame": int(pmc["read"]), "write_per_frame": int(pmc["write"]),
                                      "source": pmc["source"]}
        roof.update({
            "kernel_ms_avg": round(kernel_ms_avg, 4),
            "frames_per_launch": frames_per_launch,
            "note": "achieved = HBM bytes per launch (rocprofv3 FETCH_SIZE/WRITE_SIZE of this workload, per frame, "
                    "x frames per launch; traffic) / mean launch duration (HIP events on the launch stream); "
                    "frac = achieved / 8 TB/s (the HBM fraction).  `bound` names the binding resource measured "
                    "(binding_resource): the scene is cache-resident, and each wave is bound by its own dependent "
                    "chain (node fetch, box test, stack pop) at 4 waves per SIMD (wave_cycles; DESIGN.md §4-5)",
            # SURVEY §8d canonical work: 64 B per 2-wide node + 48 B per triangle test + 64 B per hit,
            # counted over the REFERENCE median-split tree (the canonical 2-wide walk), not over the
            # timed device tree -- a measure of work, served from L1/L2/LDS, not HBM bytes
            "work_bytes_per_frame": int(work_bytes_frame),
            "work_bytes_tree": "reference median-split tree (mybvh.cpp:375-539; SURVEY §8d canonical 2-wide walk), "
                               "not the timed device tree",
            "work_rate_GBps": round(work_bytes_frame * frames_per_launch / kernel_s / 1e9, 1),
            "l1_roof": {"peak": round(L1_PEAK_GBPS, 1), "unit": "GB/s",
                        "fetch_bytes_per_frame": int(fetch_bytes_frame),
                        "achieved": round(fetch_bytes_frame * frames_per_launch / kernel_s / 1e9, 1),
                        "frac": round(fetch_bytes_frame * frames_per_launch / kernel_s / 1e9 / L1_PEAK_GBPS, 4),
                        "td_busy_frac": pmc.get("td_busy_frac") if pmc else None,
                        "def": "128*wide_node_visits + 80*tri_tests + 96*closest_hits (production kernel's "
                               "4-wide diagnostic variant) / (64 B/clk x 256 CUs x 2.4 GHz)",
                        "peak_source": L1_PEAK_SOURCE},
            "wave_cycles": pmc_wave_mix(key, frames_per_launch),
            "valu_roof": pmc_valu_roof(key, frames_per_launch, kernel_s / frames_per_launch),
        })
        roof["bound"], roof["bound_basis"] = binding_resource(roof)
        out = {
            "metric": f"Mrays/sec (primary+shadow+reflect), {workload_label(a, host.triangle_count)}",
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            # the render kernel's own time per frame (HIP events around each launch / its frames)
            "kernel_ms_per_frame": round(kernel_ms_avg / frames_per_launch, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic: fixed-seed office_proxy stand-in (reference Office scene files are absent)"
                     if a.scene == "office" else f"synthetic: fixed-seed {a.scene} scene generator"),
            "config": {
                "workload": f"{a.scene}_proxy {a.width}x{a.height} spp={a.spp * a.spp} depth={params.max_depth} "
                            f"lights={params.n_lights}",
                "workload_key": workload_key(a, shape_n),
                "triangles": host.triangle_count,
                "bvh": f"host: reference median split, depth {host.bvh_depth}; device: "
                       + {"sah": "binned-SAH hierarchy, 4-wide", "sbvh": "binned SAH with spatial splits, 4-wide",
                          "reference": "reference tree refined, 4-wide"}[a.tree],
                "rays_per_frame": int(rays_total / a.steps),
                "rays_breakdown_rank0_launch": {"primary": st.primary_rays, "shadow": st.shadow_rays,
                                                "reflection": st.reflection_rays, "frames": F},
                "parallelism": (f"row-stripes x{n} (16-row interleave) + RCCL gather" if n > 1 else
                                f"rank 0 of row-stripes x{shape_n}, alone on one GPU" if a.rank_shape else "single GPU"),
                "frames_per_launch": frames_per_launch,
                "animation": (f"camera orbit, {a.sweep} rad over each launch's {F} frames (distinct views)"
                              if F > 1 and a.sweep != 0.0 else "none (identical frames)"),
                "launches_in_flight": S,
                "adaptive_pass": adaptive_info,
                "analytic_prims": bool(gpu.analytic),
                "host_bvh_build_s": round(build_s, 4),
                # rt_scene_upload: the device layout built on the host (hierarchy, wide collapse,
                # records), then allocation + H2D copies (rt_scene_upload_seconds); excluded from value
                "device_tree_build_s": round(dev_build_s, 4),
                "upload_copy_s": round(dev_copy_s, 4),
                "upload_wall_s": round(upload_wall_s, 4),
                # frames the production kernel rendered in this process (counting launches, warm-up,
                # timed run, single-frame run): the divisor tools/pmc_summary.py uses for per-frame bytes
                "production_frames_rendered": (F + rem + NS + a.warmup + a.steps + stream_warm_frames
                                               + (3 * NS if single else 0)
                                               + (2 * PIPE_REPS * NS if single and "pipelined" in single else 0)
                                               if not a.adaptive else None),
                "device_scene_MB": round(gpu.device_bytes / 1e6, 1),
                **({"upload_options": upload_opts} if upload_opts else {}),
            },
            "single_frame": single,
            "multi_gpu": multi,
            "rank_shape": ({"n_gpus": shape_n, "stripe_index": 0, "rows_per_frame": rows_local,
                            "def": f"rank 0's share of a {shape_n}-GPU run (its {STRIPE_H}-row stripes of every "
                                   "frame, the N > 1 launch shape) rendered alone on one GPU, no collective: the "
                                   "shape whose rocprofv3 counters give the roofline of N > 1 lines; value = "
                                   "this shard's rays/s, not a whole-job rate"} if a.rank_shape else None),
            "tree_records": tree_records,
            "roofline": roof,
            "cpu_baseline": None,
        }
        if n == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(host, params, a)
        print(json.dumps(out), flush=True)
    if n > 1:
        dist.barrier()   # every rank's work on rank 0's frames has ended before any mapping goes
        if peer is not None:
            peer.close()
        dist.barrier()
        dist.destroy_process_group()


def upload_options_for(a, n):
    """rt_upload_options fields of this run: --opt FIELD=VALUE (dev A/B), and --reserve-cus (default
    0 at any N: reserving 32 CUs slows the render by ~12 %, r04e_cumask.txt, and what it buys at
    N > 1 -- the gather beside the next launch -- is measured by the multi_gpu.reserve_cus_ab
    record of every N > 1 run, not assumed)."""
    opts = {k: (float(v) if "." in v else int(v)) for k, v in (o.split("=", 1) for o in a.opt)}
    if "reserve_cus" not in opts and a.reserve_cus > 0:
        opts["reserve_cus"] = a.reserve_cus
    return opts


def binding_resource(roof):
    """(bound, basis) from the measured fractions in a roofline record: HBM (roof.frac), the
    vector-L1 data path (l1_roof.frac: useful fetch bytes / data-return peak) and VALU issue
    (valu_roof.frac).  The largest fraction names the bound when it reaches BOUND_FRAC; else no
    throughput roof binds and the kernel is latency-bound (per-wave dependent chains, wave_cycles) --
    a claim that needs the HBM and VALU fractions measured: without either, "unmeasured".
    TD busy is not used: it counts cycles the TD holds requests waiting on L2."""
    fr = {"hbm": roof.get("frac"), "l1": (roof.get("l1_roof") or {}).get("frac"),
          "valu": (roof.get("valu_roof") or {}).get("frac")}
    known = {k: v for k, v in fr.items() if v is not None}
    basis = {f"{k}_frac": v for k, v in fr.items()}
    wc = roof.get("wave_cycles")
    if wc:
        basis["wave_mem_wait_frac"] = wc.get("mem_wait_frac")
        basis["wave_issue_frac"] = wc.get("issue_frac")
    basis["rule"] = (f"largest measured fraction >= {BOUND_FRAC} names the roof, else latency if the hbm and valu "
                     "fractions are both measured, else unmeasured")
    if known:
        k, v = max(known.items(), key=lambda kv: kv[1])
        if v >= BOUND_FRAC:
            return k, basis
    if fr["hbm"] is None or fr["valu"] is None:
        return "unmeasured", basis
    return "latency", basis


def tree_record(host, dev, a, upload_opts, tree, cams, F, fbuf, stream, rays_launch, timed_region):
    """Uploads the scene with device hierarchy `tree` and times a.steps frames in launches of F
    (after min(a.warmup, F) warm-up frames), as the main run; returns Mrays/s, ms per frame and the
    upload seconds.  Rays per launch are counted again and must equal the main tree's."""
    t0 = time.perf_counter()
    g = rtamd.DeviceScene(host, device=dev, analytic=a.analytic or a.scene == "spheres", tree=tree, **upload_opts)
    wall = time.perf_counter() - t0
    b_s, c_s = g.upload_seconds
    outs = [fbuf[f].data_ptr() for f in range(F)]
    stt = g.launch_frames(cams[:F], outs, stats=True, stream=stream) if F > 1 else \
        g.launch(cams[0], outs[0], stats=True, stream=stream)
    rays = stt.primary_rays + stt.shadow_rays + stt.reflection_rays
    if rays != rays_launch:
        raise RuntimeError(f"tree {tree}: {rays} rays per launch, main tree {rays_launch}")
    ev = []

    def run(frames, timed):
        done = 0
        while done < frames:
            nf = min(F, frames - done)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if nf > 1:
                g.launch_frames(cams[:nf], outs[:nf], stats=False, stream=stream)
            else:
                g.launch(cams[0], outs[0], stats=False, stream=stream)
            e1.record()
            if timed:
                ev.append((e0, e1, nf))
            done += nf

    n_full, rem = divmod(a.steps, F)
    total_rays = n_full * rays_launch
    if rem:
        sr = g.launch_frames(cams[:rem], outs[:rem], stats=True, stream=stream) if rem > 1 else \
            g.launch(cams[0], outs[0], stats=True, stream=stream)
        total_rays += sr.primary_rays + sr.shadow_rays + sr.reflection_rays
    run(min(a.warmup, F), False)
    el = timed_region(lambda: run(a.steps, True))
    kern = sum(e0.elapsed_time(e1) for e0, e1, _ in ev) / a.steps
    g.close()
    return {"value": round(total_rays / el / 1e6, 2), "unit": "Mrays/s", "ms_per_frame": round(el / a.steps * 1e3, 4),
            "kernel_ms_per_frame": round(kern, 4), "frames_per_launch": F, "rays_identical": True,
            "device_tree_build_s": round(b_s, 4), "upload_copy_s": round(c_s, 4), "upload_wall_s": round(wall, 4),
            "tree": {"reference": "reference median-split tree (mybvh.cpp:375-539), oversize leaves refined, 4-wide",
                     "sah": "binned-SAH hierarchy, 4-wide", "sbvh": "binned SAH with spatial splits, 4-wide"}[tree]}


def workload_label(a, n_tris):
    """The metric's workload name: BASELINE.json's own wording for the Office config ("Office
    1920x1080 1spp"; the office_proxy stand-in), else the scene actually rendered."""
    name = {"office": "Office", "spheres": "o_01_spheres", "cornell": "cornell"}.get(a.scene, a.scene)
    if a.scene == "random_tris":
        name = f"random_tris {n_tris / 1e6:g}M" if n_tris >= 1e6 else f"random_tris {n_tris}"
    return f"{name} {a.width}x{a.height} {a.spp * a.spp}spp" + (" + adaptive pass" if a.adaptive else "")


def default_frames(a):
    """Frames per launch when --frames is not given: about 2.6e8 samples per launch (a power of
    two, 1..128).  One frame of many samples is already a long launch with a negligible drain.
    (Measured in round 3 with one lane per pixel, its n*n samples in sequence: batching such frames
    cost coherence, the waves' lanes drifting apart -- 4K 4x4 spp 24.3 ms per frame at 2 frames per
    launch, 28.4 at 16; HISTORY §4.  Round 6's sample groups keep a pixel's samples on neighbouring
    lanes)  At 1 spp more frames only help."""
    samples = a.width * a.height * a.spp * a.spp
    return int(min(128, max(1, 2 ** round(math.log2(max(1.0, 2.6e8 / samples))))))


def _profile_tag(path):
    """Profiling round of a committed summary, from its name (pmc_office1080_r02u_f20.json -> "r02u",
    pmc_rt10m_r03c.json -> "r03c"): later rounds and later letters sort higher."""
    import re
    m = re.search(r"_(r\d\d[a-z]*)(?:_|\.json$)", path.name)
    return m.group(1) if m else ""


def _newest_first(key):
    """Committed PMC summaries of this workload, newest profiling round first."""
    found = []
    for path in ROOT.glob("profiles/r*/pmc_*.json"):
        try:
            d = json.loads(path.read_text())
        except (OSError, ValueError):
            continue
        if d.get("_workload") == key:
            found.append((_profile_tag(path), str(path), d))
    found.sort(reverse=True)
    return [(Path(p), d) for _, p, d in found]


def pmc_per_frame(key, frames_per_launch=None):
    """HBM bytes per frame of this workload from the newest committed rocprofv3 --pmc summary
    (profiles/r*/pmc_*.json, tools/pmc_summary.py: production-kernel FETCH_SIZE / WRITE_SIZE summed
    over the profiled run's dispatches, divided by the frames they rendered, with the access-width
    corrections of profiles/r*/hbm_calib.json).  Among the summaries of the newest profiling round
    that has one, a summary profiled at the same frames per launch wins (fewer frames per launch
    read more per frame: the L2 starts cold each launch); None when this workload was not
    profiled."""
    cands = []
    for path, d in _newest_first(key):
        pf = d.get("_per_frame", {})
        if "hbm_read_bytes" in pf and "hbm_write_bytes" in pf:
            cands.append((_profile_tag(path), path, d, pf))
    if not cands:
        return None
    newest = cands[0][0]
    same_round = [c for c in cands if c[0] == newest]
    pick = next((c for c in same_round if frames_per_launch is not None
                 and c[2].get("_bench", {}).get("frames_per_launch") == frames_per_launch), same_round[0])
    _, path, d, pf = pick
    return {"read": pf["hbm_read_bytes"], "write": pf["hbm_write_bytes"],
            "td_busy_frac": d.get("_derived", {}).get("td_busy_frac"), "source": str(path.relative_to(ROOT))}


def pmc_wave_mix(key, frames_per_launch=None):
    """Where a wave's cycles go (rocprofv3 SQ counters of this workload, newest committed summary;
    within that round the one profiled at the same frames per launch, as pmc_per_frame picks):
    issuing an instruction, waiting on a memory counter, the rest (ready behind the SIMD's other
    waves); None when no such pass was committed."""
    cands = []
    for path, d in _newest_first(key):
        try:
            wc = d["SQ_WAVE_CYCLES"]["sum"]
            issue, wait = d["SQ_ACTIVE_INST_ANY"]["sum"] / wc, d["SQ_WAIT_ANY"]["sum"] / wc
        except (KeyError, TypeError, ZeroDivisionError):
            continue
        cands.append((_profile_tag(path), path, d, issue, wait))
    if not cands:
        return None
    same_round = [c for c in cands if c[0] == cands[0][0]]
    _, path, d, issue, wait = next((c for c in same_round if frames_per_launch is not None
                                    and c[2].get("_bench", {}).get("frames_per_launch") == frames_per_launch),
                                   same_round[0])
    return {"issue_frac": round(issue, 3), "mem_wait_frac": round(wait, 3),
            "other_frac": round(1.0 - issue - wait, 3), "source": str(path.relative_to(ROOT))}


def valu_issue_cycles(d):
    """SIMD cycles of VALU issue per frame from a PMC summary's instruction classes: fp64 add / mul /
    fma at 4 cycles, fp64 transcendentals at 8, every other wave64 VALU instruction at 2
    (VALU_CYCLES); None without the class counters."""
    try:
        total = d["SQ_INSTS_VALU"]["per_frame"]
        f64 = sum(d[f"SQ_INSTS_VALU_{c}_F64"]["per_frame"] for c in ("ADD", "MUL", "FMA"))
        trans = d["SQ_INSTS_VALU_TRANS_F64"]["per_frame"]
    except (KeyError, TypeError):
        return None
    b32 = total - f64 - trans
    return {"cycles": VALU_CYCLES["b32"] * b32 + VALU_CYCLES["f64"] * f64 + VALU_CYCLES["trans64"] * trans,
            "insts": total, "b32": b32, "f64": f64, "trans64": trans}


def pmc_valu_roof(key, frames_per_launch, kernel_s_per_frame):
    """VALU issue against the SIMDs' issue capacity: the SIMD cycles the frame's VALU
    instructions need (valu_issue_cycles: each class at its own cost, from the newest committed
    summary of this workload, picked as pmc_per_frame picks it) / the cycles 1024 SIMDs offer at
    2.4 GHz in this run's kernel time per frame.  Not the binding resource (frac ~0.5 on the office):
    each wave's dependent chain is -- see wave_cycles.  None when no such pass was committed."""
    cands = []
    for path, d in _newest_first(key):
        v = valu_issue_cycles(d)
        if v is not None:
            cands.append((_profile_tag(path), path, d, v))
    if not cands:
        return None
    same_round = [c for c in cands if c[0] == cands[0][0]]
    _, path, d, v = next((c for c in same_round if frames_per_launch is not None
                          and c[2].get("_bench", {}).get("frames_per_launch") == frames_per_launch), same_round[0])
    avail = VALU_SIMDS * VALU_CLOCK_GHZ * 1e9 * kernel_s_per_frame
    return {"unit": "SIMD-cycles/frame", "achieved": int(v["cycles"]), "peak": int(avail),
            "frac": round(v["cycles"] / avail, 4), "valu_insts_per_frame": int(v["insts"]),
            "insts_b32": int(v["b32"]), "insts_f64": int(v["f64"]), "insts_trans_f64": int(v["trans64"]),
            "pricing": "2 cycles per 32-bit wave64 VALU instruction per SIMD-32, 4 per fp64, 8 per fp64 "
                       "transcendental (MI355X_MICROARCH.md cycle constants); 1024 SIMDs x 2.4 GHz",
            "source": str(path.relative_to(ROOT))}


def usable_cpus():
    """CPUs this process may actually use: its affinity mask, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(host, params, a):
    """CPU oracle (reference CPU renderer restated in C, OpenMP): whole frames of the
    same workload, repeated until --cpu-seconds of CPU work have been timed."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    # every CPU this process may use (the reference CPU path is OpenMP over all host cores,
    # README.md:10); on the GPU box that is the job's share of the node, not the node's nproc
    threads = a.cpu_threads or usable_cpus()
    orc = pyoracle.Oracle(host.raw, host)
    p = host.render_params(a.width, a.height, a.spp)
    stride = a.cpu_row_stride
    if stride <= 0:
        # probe: one 64th of the rows; a whole frame that would exceed --cpu-seconds is sampled
        # every 16th row (configs 3-5 on a 1/16-row subsample, frame time extrapolated)
        ys = np.arange(0, a.height, 64)
        xy = np.stack(np.meshgrid(np.arange(a.width), ys), -1).reshape(-1, 2)
        t = time.perf_counter()
        orc.render_pixels(p, xy, pyoracle.MODE_REFERENCE, threads)
        stride = 16 if (time.perf_counter() - t) * 64 > a.cpu_seconds else 1
    ys = np.arange(0, a.height, stride)
    xs = np.arange(a.width)
    xy = np.stack(np.meshgrid(xs, ys), -1).reshape(-1, 2)
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
        "sample": f"{frames} x (every {stride}th row of the frame: {len(xy)} pixels), {rays} rays, "
                  f"{dt:.2f} s; reference-CPU-semantics oracle (recursive unordered fp64 BVH, "
                  f"closest-hit shadows, OpenMP over pixels)",
        "workload": f"{a.scene} {a.width}x{a.height} spp={a.spp * a.spp}" + (f" tris={a.tris}" if a.tris else ""),
        "row_stride": stride,
        # seconds per whole frame at this rate: measured when the sample is whole frames, else
        # extrapolated from the 1/stride-row sample (rays per frame ~ stride x sample rays)
        "frame_s": round(dt / frames * stride, 3),
        "frame_s_extrapolated": stride > 1,
        "cpu_model": cpu_model,
        "nproc": os.cpu_count(),
        "usable_cpus": usable_cpus(),
        "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
        "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
    }


if __name__ == "__main__":
    main()
