"""bench.py end to end on one MI355X (short run): the JSON contract and the frame it renders."""
import json
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import rtamd

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(autouse=True)
def _gpu(gpu_available):
    return gpu_available


SWEEP = 0.12


def expected_frames(w, h, frames, upto=None):
    """The bench's animation path (rtamd.camera_orbit over the F = `frames` views of a launch): the
    last frame of a launch of the first `upto` views (default all) -- the frame it saves -- and the
    mean rays per frame of that launch, rendered here directly."""
    hs = rtamd.HostScene.generate("office")
    hs.prepare()
    dev = rtamd.DeviceScene(hs, 0)
    p = hs.render_params(w, h, 1)
    cams = [rtamd.camera_orbit(p, SWEEP * (f / (frames - 1) - 0.5)) for f in range(frames)] if frames > 1 else [p]
    cams = cams[:upto or len(cams)]
    rays, img = 0, None
    for c in cams:
        img, st = dev.render(c)
        rays += st.primary_rays + st.shadow_rays + st.reflection_rays
    return img, rays // len(cams)


@pytest.mark.parametrize("frames", [1, 8])
def test_bench_json_contract_and_saved_frame(tmp_path, frames):
    out = tmp_path / "frame.npy"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "8", "--warmup", "8", "--width", "320",
                        "--height", "180", "--frames", str(frames), "--no-cpu-baseline", "--save", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 8 and d["value"] > 0
    assert d["config"]["frames_per_launch"] == frames
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "l1", "valu", "latency", "unmeasured") and rf["peak"] == 8000.0 and rf["kernel_ms_avg"] > 0
    # (no PMC summary of this small workload is committed: without its basis the bound is not claimed)
    assert rf["bound"] == "unmeasured" if rf["frac"] is None else rf["bound"] != "unmeasured"
    assert rf["bound_basis"]["rule"] and "reference median-split" in rf["work_bytes_tree"]
    assert "l1_micro" in rf["l1_roof"]["peak_source"]
    assert d["multi_gpu"] is None
    assert rf["frac"] is None or 0.0 < rf["frac"] <= 1.0
    sf = d["single_frame"]
    assert sf["frames"] == min(16, frames) and sf["ms_per_frame"] > 0 and sf["value"] > 0
    co = sf["natural_order"]
    assert co["frames"] == sf["frames"] and co["ms_per_frame"] > 0 and co["rays_per_frame"] == sf["rays_per_frame"]
    pl = sf["pipelined"]   # the same one-frame launches, 3 in flight
    assert pl["launches_in_flight"] == 3 and pl["frames"] == 4 * sf["frames"] and pl["ms_per_frame"] > 0
    assert pl["rays_per_frame"] == sf["rays_per_frame"] and pl["value"] > 0
    ref, rays = expected_frames(320, 180, frames)
    assert np.array_equal(np.load(out), ref)
    assert d["config"]["rays_per_frame"] == rays


def test_bench_adaptive_pass_runs():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1", "--width", "320",
                        "--height", "180", "--adaptive", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    ad = d["config"]["adaptive_pass"]   # one GPU: the 3 frames' passes batched (rt_launch_adaptive_frames)
    assert ad["frames_per_launch"] == 3 and d["config"]["frames_per_launch"] == 3
    assert ad["pixels_supersampled_per_frame"] > 0 and ad["rays_per_frame"] > 0 and d["value"] > 0


def test_bench_two_ranks_rehearsal(tmp_path):
    # bench.py's N-rank path (row stripes, frames per launch, two launches in flight, the
    # per-launch gather and re-interleave) with 2 ranks on this one GPU: gloo stages the
    # collectives through the host (RCCL refuses two ranks on one device); the assembled frame
    # must equal the single-GPU render bit for bit.
    import os
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "frame2.npy"
    env = dict(os.environ, RT_BENCH_DEVICE="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                        "--gpus", "2", "--dist-backend", "gloo", "--steps", "16", "--warmup", "8", "--frames", "8",
                        "--width", "320", "--height", "180", "--no-cpu-baseline", "--save", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["config"]["launches_in_flight"] == 2 and d["value"] > 0
    ref, rays = expected_frames(320, 180, 8)
    assert np.array_equal(np.load(out), ref)
    assert d["config"]["rays_per_frame"] == rays


def test_bench_gpus_two_without_launcher(tmp_path):
    # `bench.py --gpus 2` with no launcher starts its two ranks itself (before any GPU call in the
    # parent) and prints rank 0's line with n_gpus 2; both ranks on this one GPU over gloo
    # (RT_BENCH_DEVICE=0); the assembled frame equals the single-GPU render bit for bit
    import os

    out = tmp_path / "frame2s.npy"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RT_BENCH_DEVICE"] = "0"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "16", "--warmup", "8", "--frames", "8", "--width", "320", "--height", "180",
                        "--no-cpu-baseline", "--save", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["value"] > 0
    ref, rays = expected_frames(320, 180, 8)
    assert np.array_equal(np.load(out), ref)
    assert d["config"]["rays_per_frame"] == rays


def test_bench_peer_assembly_two_ranks(tmp_path):
    # --assembly peer: rank 1 maps rank 0's frame buffers (IPC) and its launches write their stripes
    # there at their global rows; here both ranks share this one GPU (gloo fences); the assembled
    # frame equals the single-GPU render bit for bit, as does the gather A/B run's
    import os

    out = tmp_path / "framep.npy"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RT_BENCH_DEVICE"] = "0"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--assembly", "peer", "--reserve-ab", "off", "--steps", "16", "--warmup", "8", "--frames", "8",
                        "--width", "320", "--height", "180", "--no-cpu-baseline", "--save", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    m = d["multi_gpu"]
    assert d["n_gpus"] == 2 and m["assembly"] == "peer" and m["assembly_ab"]["frames_identical"] is True
    assert "reserve_cus_ab" not in m and m["assembly_choice"] is None   # given, not chosen
    ref, rays = expected_frames(320, 180, 8)
    assert np.array_equal(np.load(out), ref)
    assert d["config"]["rays_per_frame"] == rays


def test_bench_four_ranks_driver_shape(tmp_path):
    # the driver's command shape (--steps 20 --warmup 5, default frames per launch: 10 per rank
    # launch, two launches in flight) with 4 ranks on this one GPU over gloo: stripes of 16 rows
    # interleaved over 4 ranks, band-major frames inside each rank's launch; the assembled last
    # frame equals the single-GPU render bit for bit
    import os
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "frame4.npy"
    env = dict(os.environ, RT_BENCH_DEVICE="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                        "--gpus", "4", "--dist-backend", "gloo", "--steps", "20", "--warmup", "5",
                        "--width", "320", "--height", "180", "--no-cpu-baseline", "--save", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    # the orbit spans F = 20 views; the gather renders them 10 per launch (two launches), the peer
    # assembly 20 per launch (one)
    fpl = d["config"]["frames_per_launch"]
    assert d["n_gpus"] == 4 and d["steps"] == 20 and fpl == (10 if d["multi_gpu"]["assembly"] == "gather" else 20)
    # the N > 1 instrumentation: render and gather time per launch (max over ranks), and the run
    # again with 32 CUs reserved for the gather (reserve_cus 0 is the default)
    m = d["multi_gpu"]
    assert m["render_ms_per_launch_max"] >= m["render_ms_per_launch_rank0"] > 0
    assert m["gather_ms_per_launch_max"] >= m["gather_ms_per_launch_rank0"] > 0
    assert m["reserve_cus"] == 0 and m["gather_MB_per_launch_into_rank0"] > 0
    ab = m["reserve_cus_ab"]
    assert set(ab) == {"0", "32"} and ab["0"]["value"] == d["value"]
    for rec in ab.values():
        assert rec["value"] > 0 and rec["render_ms_per_launch_max"] > 0 and rec["gather_ms_per_launch_rank0"] > 0
    # assembly auto: both assemblies calibrated on the same launches, bit-identical frames; the other
    # one timed as well (assembly_ab), its frames bit-identical too
    ch = m["assembly_choice"]
    assert ch["frames_identical"] is True and ch["chosen"] == m["assembly"] in ("gather", "peer")
    assert set(ch["calibration_ms_per_frame"]) == {"gather", "peer"}
    asm = m["assembly_ab"]
    other = "peer" if m["assembly"] == "gather" else "gather"
    assert asm["frames_identical"] is True and asm[m["assembly"]]["value"] == d["value"] and asm[other]["value"] > 0
    assert asm[other]["frames_per_launch"] == (10 if other == "gather" else 20)
    ref, rays = expected_frames(320, 180, 20, upto=int(fpl))
    assert np.array_equal(np.load(out), ref)
    assert d["config"]["rays_per_frame"] == rays
    # the roofline of an N > 1 line: rank 0's launches, priced from the committed PMC summary of this
    # workload's rank shape (profiled on one GPU with --rank-shape 4), so the HBM fraction is numeric
    # and the bound is named from measured fractions
    rf = d["roofline"]
    assert rf["traffic"] > 0 and 0.0 < rf["frac"] <= 1.0, rf
    assert rf["valu_roof"]["frac"] > 0 and rf["wave_cycles"]["mem_wait_frac"] > 0
    assert rf["bound"] in ("hbm", "l1", "valu", "latency") and rf["bound_basis"]["hbm_frac"] == rf["frac"]
    assert d["config"]["workload_key"]["n_gpus"] == 4


def test_bench_rank_shape_is_rank0_of_n(tmp_path):
    # --rank-shape N: one process renders exactly rank 0's stripes of an N-GPU run in the N > 1 launch
    # shape (frames per launch of the gather assembly, two launches in flight) -- the shape profiled
    # for the N > 1 roofline; the rays equal rank 0's share of the frames
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--rank-shape", "4", "--steps", "20", "--warmup", "5",
                        "--width", "320", "--height", "180", "--no-cpu-baseline", "--tree-record", "off"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["rank_shape"]["n_gpus"] == 4 and d["config"]["workload_key"]["n_gpus"] == 4
    assert d["config"]["frames_per_launch"] == 10 and d["config"]["launches_in_flight"] == 2
    hs = rtamd.HostScene.generate("office")
    hs.prepare()
    dev = rtamd.DeviceScene(hs, 0)
    base = hs.render_params(320, 180, 1)
    rays = 0
    for f in range(10):   # the orbit spans F = 20 views; launches of 10 render views 0..9
        p = rtamd.camera_orbit(base, SWEEP * (f / 19 - 0.5))
        p.stripe_height, p.stripe_count, p.stripe_index = 16, 4, 0
        _, st = dev.render(p)
        rays += st.primary_rays + st.shadow_rays + st.reflection_rays
    assert d["config"]["rays_per_frame"] == rays // 10
    assert d["rank_shape"]["rows_per_frame"] == rtamd.rows_in_shard(p)
