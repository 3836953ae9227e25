"""Path-state parity check of one librt_hip build (dev tool, under gpurun): office 3840x2160
4x4 spp (config 3; the pixel sum across samples lives in path state) and office 1080p 1 spp
(mirror chains: colour and weight across bounces), fp64, GPU vs oracle on a band of rows.
usage: [RTAMD_HIP_LIB=path] python tools/repro_pathstate.py [label]"""
import os
import sys

import numpy as np

sys.path.insert(0, "my-raytracer_amd")
sys.path.insert(0, "oracle")
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("RTAMD_HIP_LIB", "default")
hs = rtamd.HostScene.generate("office")
hs.prepare()
dev = rtamd.DeviceScene(hs, 0)
orc = pyoracle.Oracle(hs.raw, hs)
for w, h, spp, rows in ((3840, 2160, 4, np.arange(1048, 1080)), (1920, 1080, 1, np.arange(0, 1080, 9))):
    p = hs.render_params(w, h, spp)
    p.out_format = rtamd.RT_OUT_RGB_F64
    bad = 0
    for rep in range(3):
        img, st = dev.render(p)
        nanpx = np.isnan(img).any(-1)
        bad = max(bad, int(nanpx.sum()))
    if nanpx.any():
        ys, xs = np.nonzero(nanpx)
        tiles = np.unique((ys // 8) * 10000 + xs // 8)
        per_tile = np.bincount(((ys // 8) * ((w + 7) // 8) + xs // 8))
        per_tile = per_tile[per_tile > 0]
        chan = np.isnan(img[nanpx]).sum(0)
        print(f"  NaN rows {ys.min()}..{ys.max()} ({len(np.unique(ys))} distinct), cols {xs.min()}..{xs.max()}, "
              f"{len(tiles)} 8x8 tiles, NaN pixels per hit tile: mean {per_tile.mean():.1f} max {per_tile.max()}; "
              f"NaN channels r/g/b {chan.tolist()}; row histogram /256: "
              f"{np.bincount(ys // 256, minlength=(h + 255) // 256).tolist()}", flush=True)
    xy = np.stack(np.meshgrid(np.arange(w), rows), -1).reshape(-1, 2).astype(np.int32)
    ref, _ = orc.render_pixels(p, xy, pyoracle.MODE_ORDERED, threads=0)
    got = img[rows].reshape(-1, 3)
    err = np.abs(got - ref)
    wrong = int((err.max(-1) > 1e-12).sum())
    print(f"{label}: {w}x{h} spp={spp * spp}: NaN pixels (max of 3 renders) {bad}, "
          f"wrong pixels in {len(rows)} checked rows {wrong} of {len(xy)}, max err {np.nanmax(err):.3g}", flush=True)
