"""Oracle self-consistency (CPU): the reference-semantics traversal and the
replica of the GPU algorithm give identical images and ray sets; config 1
(spheres_proxy, analytic primitives, CPU path only) renders."""
import numpy as np
import pytest

import pyoracle
import rtamd


@pytest.mark.parametrize("kind,kw,w,h", [("cornell", {}, 80, 60), ("office", {}, 96, 54),
                                         ("random_tris", {"n_triangles": 8000}, 64, 36)])
def test_reference_and_ordered_modes_agree(kind, kw, w, h):
    hs = rtamd.HostScene.generate(kind, **kw)
    hs.prepare()
    orc = pyoracle.Oracle(hs.raw, hs)
    p = hs.render_params(w, h, 1)
    a, ca = orc.render(p, pyoracle.MODE_REFERENCE)
    b, cb = orc.render(p, pyoracle.MODE_ORDERED)
    assert np.array_equal(a, b)
    for k in ("primary_rays", "shadow_rays", "reflection_rays", "closest_hits"):
        assert getattr(ca, k) == getattr(cb, k), k
    assert cb.tri_tests < ca.tri_tests       # ordered + t-culled + any-hit does less work
    assert cb.node_visits > 0 and ca.box_tests > 0


def test_spheres_proxy_config1_cpu_path():
    # BASELINE config 1: o_01_spheres stand-in, 640x480 1spp on the CPU path (no BVH)
    hs = rtamd.HostScene.generate("spheres")
    hs.prepare()
    assert hs.triangle_count == 0
    orc = pyoracle.Oracle(hs.raw, hs)
    p = hs.render_params(640, 480, 1)
    img, cnt = orc.render(p)
    assert img.shape == (480, 640, 3)
    assert cnt.primary_rays == 640 * 480
    assert cnt.shadow_rays > 0 and cnt.reflection_rays > 0   # plane and one sphere are mirrors
    assert (img.sum(-1) > 0).mean() > 0.5                       # floor plane + spheres cover the view
    assert 0.0 <= img.min() and img.max() <= 1.0


def test_closest_hit_api():
    hs = rtamd.HostScene.generate("cornell")
    hs.prepare()
    orc = pyoracle.Oracle(hs.raw, hs)
    h = orc.closest_hit((0.0, 1.0, 3.0), (0.0, 0.0, -1.0))
    assert h is not None and abs(h["point"][2] - (-0.99)) < 1e-9    # the textured poster at z = -0.99
    h2 = orc.closest_hit((0.0, 1.0, 3.0), (0.0, 0.0, -1.0), pyoracle.MODE_ORDERED)
    assert h2["t"] == h["t"] and h2["tri"] == h["tri"]
    assert orc.closest_hit((0.0, 1.0, 3.0), (0.0, 0.0, 1.0)) is None   # looking out of the open front
