"""Generates tests/golden/*.npz (run from the repo root: python tests/golden/make_golden.py).

Golden vectors for the render path.  The reference ships none and
cannot be built here, so they come from
  * the pure-Python restatement (tests/minirt.py) for the tiny KAT scenes
    ("kat_*": independent of both the oracle and the product), and
  * the C oracle in reference mode for the procedural scenes at small sizes
    ("scene_*": regression pins of the oracle; parity unpinned vs the
    reference's own outputs).
Each file holds the fp64 image (rows bottom-up), the canonical ray counts and,
for the scene files, the reference-order BVH arrays.
"""
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
import kat_scenes  # noqa: E402
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

OUT = Path(__file__).resolve().parent

SCENE_CASES = {
    "scene_cornell_40x30": ("cornell", {}, 40, 30, 1),
    "scene_office_48x27": ("office", {}, 48, 27, 1),
    "scene_office_24x14_spp2": ("office", {}, 24, 14, 2),
    "scene_random_tris_32x18": ("random_tris", {"n_triangles": 3000, "seed": 1234}, 32, 18, 1),
}


def main(only=()):
    """only: regenerate just these KAT scene names (the other files stay untouched)."""
    for name in kat_scenes.scenes():
        if only and name not in only:
            continue
        for spp in (1, 2):
            mini = kat_scenes.mini(name)
            img = np.array(mini.render(spp))
            np.savez_compressed(OUT / f"kat_{name}_spp{spp}.npz", image=img,
                                counts=np.array([mini.counts["primary"], mini.counts["shadow"],
                                                 mini.counts["reflection"]]))
    for fname, (kind, kw, w, h, spp) in SCENE_CASES.items():
        if only:
            break
        hs = rtamd.HostScene.generate(kind, **kw)
        hs.prepare()
        orc = pyoracle.Oracle(hs.raw, hs)
        p = hs.render_params(w, h, spp)
        img, cnt = orc.render(p, pyoracle.MODE_REFERENCE)
        b = orc.bvh()
        np.savez_compressed(OUT / f"{fname}.npz", image=img,
                            counts=np.array([cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays]),
                            left_child=b["left_child"], first_tri=b["first_tri"], tri_count=b["tri_count"],
                            perm=b["perm"])
    print("\n".join(sorted(p.name for p in OUT.glob("*.npz"))))


if __name__ == "__main__":
    with tempfile.TemporaryDirectory():
        main(tuple(sys.argv[1:]))
