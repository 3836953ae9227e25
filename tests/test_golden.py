"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py):
the oracle and the host builder must reproduce them exactly."""
from pathlib import Path

import numpy as np
import pytest

import kat_scenes
import pyoracle
import rtamd

GOLD = Path(__file__).resolve().parent / "golden"
SCENE_CASES = {
    "scene_cornell_40x30": ("cornell", {}, 40, 30, 1),
    "scene_office_48x27": ("office", {}, 48, 27, 1),
    "scene_office_24x14_spp2": ("office", {}, 24, 14, 2),
    "scene_random_tris_32x18": ("random_tris", {"n_triangles": 3000, "seed": 1234}, 32, 18, 1),
}


@pytest.mark.parametrize("name", sorted(kat_scenes.scenes()))
@pytest.mark.parametrize("spp", [1, 2])
def test_oracle_matches_kat_golden(tmp_path, name, spp):
    g = np.load(GOLD / f"kat_{name}_spp{spp}.npz")
    hs = rtamd.HostScene.load(kat_scenes.write(tmp_path, name))
    hs.prepare()
    img, cnt = pyoracle.Oracle(hs.raw, hs).render(hs.render_params(0, 0, spp))
    assert np.abs(img - g["image"]).max() <= 1e-12
    assert [cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays] == list(g["counts"])


@pytest.mark.parametrize("fname", sorted(SCENE_CASES))
def test_oracle_and_host_match_scene_golden(fname):
    kind, kw, w, h, spp = SCENE_CASES[fname]
    g = np.load(GOLD / f"{fname}.npz")
    hs = rtamd.HostScene.generate(kind, **kw)
    hs.prepare()
    hb = hs.bvh_arrays()
    for k in ("left_child", "first_tri", "tri_count"):
        assert np.array_equal(hb[k], g[k]), k
    img, cnt = pyoracle.Oracle(hs.raw, hs).render(hs.render_params(w, h, spp))
    assert np.array_equal(img, g["image"])
    assert [cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays] == list(g["counts"])
