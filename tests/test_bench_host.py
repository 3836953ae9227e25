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
