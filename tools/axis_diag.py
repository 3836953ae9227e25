"""Axis-aligned scene (tests/test_gpu_parity.py::test_axis_aligned_scene_exact_zero_components):
where the GPU render differs from the oracle, with the production and the 2-wide canonical kernel
(dev tool, under gpurun; RTAMD_HIP_LIB selects the library)."""
import pathlib
import sys
import tempfile

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
sys.path.insert(0, "my-raytracer_amd")
import kat_scenes  # noqa: E402
import minirt  # noqa: E402
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

box_top = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
box_z = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
t = pathlib.Path(tempfile.mkdtemp())
floor_v, floor_t = [(-3.0, -1.0, 3.0), (3.0, -1.0, 3.0), (3.0, -1.0, -3.0), (-3.0, -1.0, -3.0)], [(0, 1, 2), (0, 2, 3)]
wall_v, wall_t = kat_scenes.quad(-3.0, 3.0, -1.0, 3.0, -2.0)
box_v = [(-0.5, -1.0, box_z), (0.5, -1.0, box_z), (0.5, box_top, box_z), (-0.5, box_top, box_z)]
meshes = [minirt.Mesh(floor_v, floor_t, "FLAT", kat_scenes.FLAT_MAT),
          minirt.Mesh(wall_v, wall_t, "FLAT", kat_scenes.MIRROR_MAT),
          minirt.Mesh(box_v, [(0, 1, 2), (0, 2, 3)], "FLAT", kat_scenes.FLAT_MAT)]
lights = [((0.0, 2.5, 0.0), (0.7, 0.7, 0.7)), ((0.0, 0.0, 3.0), (0.3, 0.3, 0.3))]
for w, h in [(16, 12), (64, 48)]:
    path = t / f"axis_{w}.sce"
    minirt.write_sce(path, meshes, lights, ((0.0, 0.0, 4.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 50.0, w, h),
                     (0.05, 0.1, 0.2), (0.2, 0.2, 0.2), 3)
    hs = rtamd.HostScene.load(path)
    hs.prepare()
    orc = pyoracle.Oracle(hs.raw, hs)
    p = hs.render_params(0, 0, int(sys.argv[3]) if len(sys.argv) > 3 else 1)
    ref, cnt = orc.render(p, pyoracle.MODE_REFERENCE)
    p.out_format = rtamd.RT_OUT_RGB_F64
    for flags, name in [(0, "4-wide production"), (rtamd.RT_FLAG_TRAVERSAL_STATS, "2-wide canonical")]:
        p.flags = flags
        dev = rtamd.DeviceScene(hs, 0)
        img, st = dev.render(p)
        d = np.abs(img - ref).max(axis=2)
        bad = np.argwhere(d > 1e-12)
        print(f"{w}x{h} {name}: max {d.max():.3e}, {len(bad)} pixels, counts gpu "
              f"{[st.primary_rays, st.shadow_rays, st.reflection_rays]} oracle "
              f"{[cnt.primary_rays, cnt.shadow_rays, cnt.reflection_rays]}; rows,cols {bad[:12].tolist()}", flush=True)
        for (y, x) in bad[:3]:
            print("   ", y, x, img[y, x], ref[y, x])
        dev.close()
