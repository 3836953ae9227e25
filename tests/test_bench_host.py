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


def test_reserve_cus_at_n_above_one():
    # N > 1: the render launches leave 32 CUs free for the RCCL gather; one GPU: none
    b = _bench()
    a = types.SimpleNamespace(opt=[], reserve_cus=-2)
    assert b.upload_options_for(a, 1) == {}
    assert b.upload_options_for(a, 8) == {"reserve_cus": 32}
    assert b.upload_options_for(types.SimpleNamespace(opt=[], reserve_cus=0), 8) == {}
    assert b.upload_options_for(types.SimpleNamespace(opt=["reserve_cus=4", "lds_treelet=9"], reserve_cus=-2), 8) == \
        {"reserve_cus": 4, "lds_treelet": 9}
