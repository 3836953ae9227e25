"""Seeded random scenes (tests/fuzz_scenes.py): the CPU oracle against the independent pure-Python
restatement (tests/minirt.py, brute force, no BVH), in both oracle traversal modes.  Pixels within
1e-12, ray counts exact.  The GPU side of the same scenes is tests/test_gpu_parity.py::test_fuzz_*."""
import numpy as np
import pytest

import fuzz_scenes
import pyoracle
import rtamd

SEEDS = range(40)


@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_scene_oracle_matches_python(tmp_path, seed):
    hs = rtamd.HostScene.load(fuzz_scenes.write(tmp_path, seed))
    hs.prepare()
    orc = pyoracle.Oracle(hs.raw, hs)
    spp = 2 if seed % 4 == 3 else 1
    p = hs.render_params(0, 0, spp)
    img, cnt = orc.render(p, pyoracle.MODE_REFERENCE)
    mini = fuzz_scenes.mini(seed)
    ref = np.array(mini.render(spp))
    assert img.shape == ref.shape
    assert np.abs(img - ref).max() <= 1e-12, np.abs(img - ref).max()
    assert [cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays] == \
        [mini.counts["primary"], mini.counts["shadow"], mini.counts["reflection"]]
    img2, cnt2 = orc.render(p, pyoracle.MODE_ORDERED)
    assert np.abs(img2 - img).max() <= 1e-12
    assert [cnt2.primary_rays, cnt2.shadow_rays, cnt2.reflection_rays] == \
        [cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays]


def test_fuzz_scenes_cover_the_cases():
    # across the seeds: mirrors, non-shadowable materials, PHONG meshes, > RT_MAX_LIGHTS lights
    # (> 32: more than one shadow batch), depth 0 and depth >= 3
    seen = set()
    for s in SEEDS:
        meshes, lights, _, _, _, depth = fuzz_scenes.scene(s)
        seen |= {("mirror" if m.mat[4] > 0 else "matte") for m in meshes}
        seen |= {("noshadow" if m.mat[5] == 0 else "shadow") for m in meshes}
        seen |= {m.mode for m in meshes}
        seen.add("lights>16" if len(lights) > rtamd.abi.RT_MAX_LIGHTS else "lights<=16")
        seen.add("lights>32" if len(lights) > 32 else "lights<=32")
        seen.add("depth0" if depth == 0 else ("deep" if depth >= 3 else "shallow"))
    assert {"mirror", "matte", "noshadow", "shadow", "FLAT", "PHONG", "lights>16", "lights<=16",
            "lights>32", "depth0", "deep"} <= seen, seen
