"""Known inputs where the reference CPU renderer and a brute-force renderer disagree, pinned.

The reference's fp64 slab test (BVH::intersectAABB, mybvh.cpp:99-135) is not conservative: a ray
that meets a triangle exactly on the boundary of its leaf box can lose a hit the triangle test
(mymesh.cpp:190-215, inclusive barycentrics) accepts.  DESIGN.md §3 documents two such inputs:

  * edge_exact: 64x48, 2x2 spp, the floor's edge at x = -3: one sample of pixel (14, 3);
  * nan_max_plane: a ray with d.x == 0 exactly on a leaf box's max-x plane (0/0 = NaN carried into
    tmax by std::min): the 17 centre-column pixels that see the panel.

The kernel's boxes are conservative, so it keeps those hits, as tests/minirt.py (no boxes) does.
These tests enumerate the divergence exactly -- the reference (oracle MODE_REFERENCE) differs from
the brute force at exactly the listed pixels and by exactly the listed shadow-ray count, the
oracle's GPU-semantics mode and the kernel equal the brute force everywhere -- so a change that
widens it (a looser fp32 delta, a non-conservative slab) fails here instead of going unseen.
"""
import numpy as np
import pytest

import kat_scenes
import pyoracle
import rtamd

TOL64 = 1e-12
CASES = sorted(kat_scenes.divergence_scenes())


def _setup(tmp_path, name):
    case = kat_scenes.divergence_scenes()[name]
    spp, pixels, (d_shadow, d_refl) = case[6], case[7], case[8]
    hs = rtamd.HostScene.load(kat_scenes.write_divergence(tmp_path, name))
    hs.prepare()
    mini = kat_scenes.mini_divergence(name)
    brute = np.array(mini.render(spp))
    return hs, spp, pixels, (d_shadow, d_refl), brute, mini.counts


def _diff_pixels(a, b):
    return sorted(map(tuple, np.argwhere(np.abs(a - b).max(axis=2) > TOL64).tolist()))


@pytest.mark.parametrize("name", CASES)
def test_reference_diverges_exactly_at_the_documented_pixels(tmp_path, name):
    hs, spp, pixels, (d_shadow, d_refl), brute, bc = _setup(tmp_path, name)
    orc = pyoracle.Oracle(hs.raw, hs)
    p = hs.render_params(0, 0, spp)
    ref, cnt = orc.render(p, pyoracle.MODE_REFERENCE)
    assert _diff_pixels(ref, brute) == sorted(pixels)
    assert bc["primary"] == cnt.primary_rays
    assert (bc["shadow"] - cnt.shadow_rays, bc["reflection"] - cnt.reflection_rays) == (d_shadow, d_refl)
    # the oracle's GPU-semantics mode (ordered, conservative fp32 boxes) keeps every hit
    ordm, c2 = orc.render(p, pyoracle.MODE_ORDERED)
    assert np.abs(ordm - brute).max() <= TOL64
    assert [c2.primary_rays, c2.shadow_rays, c2.reflection_rays] == [bc["primary"], bc["shadow"], bc["reflection"]]


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("tree", [None, "reference"])
def test_kernel_keeps_the_hits_the_reference_loses(gpu_available, tmp_path, name, tree):
    hs, spp, pixels, _, brute, bc = _setup(tmp_path, name)
    dev = rtamd.DeviceScene(hs, 0, tree=tree)
    p = hs.render_params(0, 0, spp)
    p.out_format = rtamd.RT_OUT_RGB_F64
    for flags in (0, rtamd.RT_FLAG_TRAVERSAL_STATS):   # production 4-wide, canonical 2-wide
        p.flags = flags
        img, st = dev.render(p)
        assert np.abs(img - brute).max() <= TOL64, flags
        assert [st.primary_rays, st.shadow_rays, st.reflection_rays] == \
            [bc["primary"], bc["shadow"], bc["reflection"]], flags
    # ... and so differs from the reference CPU renderer at exactly the documented pixels
    ref, _ = pyoracle.Oracle(hs.raw, hs).render(p, pyoracle.MODE_REFERENCE)
    assert _diff_pixels(img, ref) == sorted(pixels)
    dev.close()
