"""Adaptive supersampling pass (mytracer_gpu.cu:162-229) on the CPU:
the oracle's restatement against an independent pure-Python one (tests/minirt.py)."""
import numpy as np

import kat_scenes
import pyoracle
import rtamd


def reference_selection(prim, threshold):
    """Literal per-pixel loop of mytracer_gpu.cu:183-198 (normSq over xyz)."""
    H, W = prim.shape[:2]
    sel = np.zeros((H, W), dtype=bool)

    def nsq(a, b):
        dx, dy, dz = a[0] - b[0], a[1] - b[1], a[2] - b[2]
        return dx * dx + dy * dy + dz * dz

    for y in range(1, H - 1):
        for x in range(1, W - 1):
            c = prim[y, x]
            n = nsq(c, prim[y, x + 1]) + nsq(c, prim[y + 1, x]) + nsq(c, prim[y, x - 1]) + nsq(c, prim[y - 1, x])
            sel[y, x] = n > threshold
    return sel


def test_selection_matches_literal_loop():
    rng = np.random.default_rng(5)
    prim = np.minimum(rng.random((13, 17, 3)) * rng.random((13, 17, 1)), 1.0)
    for thr in (0.0, 0.02, 0.3, 5.0):
        assert np.array_equal(pyoracle.adaptive_selection(prim, thr), reference_selection(prim, thr))
    assert not pyoracle.adaptive_selection(prim[:2], 0.0).any()   # no interior pixels


def test_adaptive_pass_matches_python_restatement(tmp_path):
    name = "mirror"
    hs = rtamd.HostScene.load(kat_scenes.write(tmp_path, name))
    hs.prepare()
    orc = pyoracle.Oracle(hs.raw, hs)
    p = hs.render_params(0, 0, 1)
    prim, _ = orc.render(p)
    img, cnt, sel = orc.adaptive(p, prim, subp=4, threshold=0.02)
    mini = kat_scenes.mini(name)
    mprim = np.array(mini.render(1))
    assert np.abs(mprim - prim).max() <= 1e-12
    assert np.array_equal(sel, reference_selection(mprim, 0.02))
    assert sel.sum() > 0 and not sel.all()
    m4 = np.array(mini.render(4))                     # 4x4 samples everywhere, used where selected
    ref = np.where(sel[..., None], m4, mprim)
    assert np.abs(img - ref).max() <= 1e-12
    assert cnt.primary_rays == 16 * sel.sum()
