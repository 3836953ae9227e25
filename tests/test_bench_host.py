"""bench.py host-side choices (no GPU): frames per launch by samples per frame."""
import importlib.util
import types
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_default_frames_per_launch():
    b = _bench()
    f = lambda w, h, s: b.default_frames(types.SimpleNamespace(width=w, height=h, spp=s))  # noqa: E731
    assert f(1920, 1080, 1) == 128      # the headline: 1 spp, batching only helps
    assert f(640, 480, 1) == 128
    assert f(1920, 1080, 4) == 8        # 16 spp
    assert f(3840, 2160, 4) == 2        # config 3
    assert f(7680, 4320, 8) == 1        # config 5


def test_valu_roof_from_committed_summary():
    """The VALU-issue roof is read from the committed SQ counters of the workload and priced per
    class (MI355X_MICROARCH.md: 2 SIMD cycles per 32-bit wave64 instruction, 4 per fp64, 8 per fp64
    transcendental) against 1024 SIMDs x 2.4 GHz x the kernel time per frame."""
    b = _bench()
    key = {"scene": "office", "tris": 0, "width": 1920, "height": 1080, "spp": 1, "tree": "sbvh",
           "sweep": 0.12, "adaptive": False, "analytic": False, "n_gpus": 1}
    r = b.pmc_valu_roof(key, 20, 0.3408e-3)
    assert r is not None and r["source"].startswith("profiles/")
    cycles = 2 * r["insts_b32"] + 4 * r["insts_f64"] + 8 * r["insts_trans_f64"]
    assert abs(r["insts_b32"] + r["insts_f64"] + r["insts_trans_f64"] - r["valu_insts_per_frame"]) <= 3
    assert abs(r["frac"] - cycles / (1024 * 2.4e9 * 0.3408e-3)) < 1e-3
    assert 0.3 < r["frac"] < 0.7   # the office at the driver's shape: about half the issue capacity
    assert b.pmc_valu_roof(dict(key, scene="nonexistent"), 128, 0.36e-3) is None


def test_metric_names_the_workload():
    b = _bench()
    a = types.SimpleNamespace(scene="office", width=1920, height=1080, spp=1, adaptive=False)
    assert b.workload_label(a, 59670) == "Office 1920x1080 1spp"   # BASELINE.json's wording
    a = types.SimpleNamespace(scene="random_tris", width=1920, height=1080, spp=1, adaptive=False)
    assert b.workload_label(a, 10_000_000) == "random_tris 10M 1920x1080 1spp"
    a = types.SimpleNamespace(scene="office", width=3840, height=2160, spp=4, adaptive=False)
    assert b.workload_label(a, 59670) == "Office 3840x2160 16spp"


def test_reserve_cus_is_opt_in():
    # reserving CUs for the gather costs the render ~12 % (r04e_cumask.txt) and its gain at N > 1 is
    # measured by multi_gpu.reserve_cus_ab, so no run reserves CUs unless asked
    b = _bench()
    a = types.SimpleNamespace(opt=[], reserve_cus=0)
    assert b.upload_options_for(a, 1) == {}
    assert b.upload_options_for(a, 8) == {}
    assert b.upload_options_for(types.SimpleNamespace(opt=[], reserve_cus=32), 8) == {"reserve_cus": 32}
    assert b.upload_options_for(types.SimpleNamespace(opt=["reserve_cus=4", "lds_treelet=9"], reserve_cus=0), 8) == \
        {"reserve_cus": 4, "lds_treelet": 9}


def test_binding_resource_vocabulary():
    b = _bench()
    # the office at the driver's shape (BENCH_r04): no roof near its peak -> latency-bound
    roof = {"frac": 0.03, "l1_roof": {"frac": 0.681}, "valu_roof": {"frac": 0.498},
            "wave_cycles": {"mem_wait_frac": 0.455, "issue_frac": 0.375}}
    bound, basis = b.binding_resource(roof)
    assert bound == "latency" and basis["l1_frac"] == 0.681 and basis["wave_mem_wait_frac"] == 0.455
    assert b.binding_resource({"frac": 0.85, "l1_roof": {"frac": 0.3}})[0] == "hbm"
    assert b.binding_resource({"frac": 0.1, "l1_roof": {"frac": 0.9}, "valu_roof": {"frac": 0.5}})[0] == "l1"
    assert b.binding_resource({"frac": None, "l1_roof": None, "valu_roof": {"frac": 0.95}})[0] == "valu"
    assert set(b.BOUND_VOCAB) == {"hbm", "l1", "valu", "latency", "unmeasured"}


def test_binding_resource_unmeasured_without_its_basis():
    # "latency" is a claim about measured fractions: with the HBM or the VALU fraction missing (an
    # N > 1 line of a workload whose rank shape was never profiled) the bound is "unmeasured"
    b = _bench()
    assert b.binding_resource({})[0] == "unmeasured"
    assert b.binding_resource({"frac": None, "l1_roof": {"frac": 0.7}, "valu_roof": {"frac": 0.5}})[0] == "unmeasured"
    assert b.binding_resource({"frac": 0.03, "l1_roof": {"frac": 0.7}, "valu_roof": None})[0] == "unmeasured"
    assert b.binding_resource({"frac": 0.03, "l1_roof": None, "valu_roof": {"frac": 0.5}})[0] == "latency"
    bound, basis = b.binding_resource({"frac": None, "l1_roof": {"frac": 0.9}, "valu_roof": None})
    assert bound == "l1" and basis["hbm_frac"] is None   # a measured roof at >= 0.8 still names itself


def test_rank_shape_profiles_feed_n_gpu_lines():
    # every N > 1 line of the driver's office shape finds the PMC summary of its rank shape (rank 0's
    # launches profiled on one GPU with --rank-shape N): a numeric HBM fraction and a VALU roof
    b = _bench()
    key = {"scene": "office", "tris": 0, "width": 1920, "height": 1080, "spp": 1, "tree": "sbvh",
           "sweep": 0.12, "adaptive": False, "analytic": False}
    for n in (2, 4, 8):
        for fpl in (10.0, 20.0):
            pmc = b.pmc_per_frame(dict(key, n_gpus=n), fpl)
            assert pmc is not None and pmc["read"] > 0 and pmc["write"] > 0, (n, fpl)
            assert b.pmc_valu_roof(dict(key, n_gpus=n), fpl, 0.1e-3) is not None, n
            assert b.pmc_wave_mix(dict(key, n_gpus=n), fpl) is not None, n
            # the gather's shape (10 frames per launch) and the peer assembly's (20) each find the
            # summary profiled at their own frames per launch
            assert pmc["source"].endswith("_f20.json") == (fpl == 20.0), (n, fpl, pmc["source"])


def _launch(args, env_extra=None, timeout=240):
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=env)


def test_gpus_n_starts_n_ranks_without_a_launcher():
    # `python bench.py --gpus N` with no launcher (no WORLD_SIZE) starts N child ranks itself, before
    # any GPU call; --launch-check stops them after they joined a process group of N (no GPU here)
    import json
    for n in (2, 3):
        r = _launch(["--gpus", str(n), "--launch-check"])
        assert r.returncode == 0, r.stderr[-2000:]
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["launch_check"] and d["n_gpus"] == n and d["ranks"] == list(range(n)) and d["distinct_pids"] == n


def test_gpus_mismatch_with_launcher_fails():
    r = _launch(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_gpus_beyond_visible_devices_fails():
    # no launcher, more GPUs asked than visible (none in this container): exit 2 before any rank starts
    import torch
    if torch.cuda.device_count() >= 2:
        return
    r = _launch(["--gpus", "2", "--steps", "1"])
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr
