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
    """The VALU-issue roof is read from the committed SQ counters of the workload: the office
    summaries carry SQ_INSTS_VALU, and the fraction is instructions / kernel time / peak."""
    b = _bench()
    key = {"scene": "office", "tris": 0, "width": 1920, "height": 1080, "spp": 1, "tree": "sbvh",
           "sweep": 0.12, "adaptive": False, "analytic": False, "n_gpus": 1}
    r = b.pmc_valu_roof(key, 128, 0.36e-3)
    assert r is not None and r["source"].startswith("profiles/")
    assert abs(r["frac"] - r["valu_insts_per_frame"] / 0.36e-3 / 1e9 / b.VALU_PEAK_GINSTS) < 1e-3
    assert 0.0 < r["frac"] < 1.2 and (r["busy_frac"] is None or 0.0 < r["busy_frac"] < 1.1)
    assert b.pmc_valu_roof(dict(key, scene="nonexistent"), 128, 0.36e-3) is None
