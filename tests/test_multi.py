"""Single-process multi-GPU driver (include/rt_multi.h, librt_multi.so).

CPU: the row partition and the frame assembly.  Every shard of n is rendered by the CPU
oracle with the same stripe parameters the driver gives GPU g, padded to the common
height as ncclGather receives them, and re-interleaved by the library's host restatement
of the assembly kernel (same index map); the result must equal the oracle's full frame
bit for bit.  GPU: the driver itself through RCCL on the one device of the box (a one-rank
ncclGather; RCCL refuses two ranks on one GPU, so N > 1 runs only on a multi-GPU node)
against the single-device launch, and the CLI's --gpus path.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

import pyoracle
import rtamd

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def office():
    hs = rtamd.HostScene.generate("office")
    hs.prepare()
    return hs, pyoracle.Oracle(hs.raw, hs)


@pytest.mark.parametrize("h,sh,n", [(1080, 16, 8), (37, 16, 8), (45, 4, 3), (27, 1, 2), (20, 16, 1), (9, 2, 4)])
def test_max_rows_matches_partition(h, sh, n):
    rows = [len(rtamd.shard_rows(h, sh, n, g)) for g in range(n)]
    assert rtamd.multi_lib().rt_multi_max_rows(h, sh, n) == max(rows)
    assert sum(rows) == h


@pytest.mark.parametrize("w,h,sh,n", [(48, 27, 4, 3), (40, 23, 1, 2), (32, 18, 16, 8), (24, 14, 2, 1)])
def test_stripes_gathered_and_interleaved_equal_full_frame(office, w, h, sh, n):
    hs, orc = office
    full, cnt = orc.render(hs.render_params(w, h, 1), pyoracle.MODE_REFERENCE)
    mr = rtamd.multi_lib().rt_multi_max_rows(h, sh, n)
    gathered = np.full((n, mr, w, 3), np.nan)   # padding rows must never reach the frame
    rays = 0
    for g in range(n):
        p = hs.render_params(w, h, 1)
        p.stripe_height, p.stripe_count, p.stripe_index = sh, n, g
        shard, c = orc.render(p, pyoracle.MODE_REFERENCE)
        gathered[g, :shard.shape[0]] = shard
        rays += c.primary_rays + c.shadow_rays + c.reflection_rays
    img = rtamd.multi_interleave_host(gathered, h, sh, n)
    assert np.array_equal(img, full)
    assert rays == cnt.primary_rays + cnt.shadow_rays + cnt.reflection_rays


@pytest.mark.parametrize("w,h,sh,n,nf", [(40, 23, 4, 3, 3), (32, 18, 16, 8, 2), (24, 14, 2, 2, 4)])
def test_batched_stripes_gathered_and_interleaved_equal_frames(office, w, h, sh, n, nf):
    # rt_multi_render_frames: GPU g renders its stripes of every frame of a batch (distinct
    # cameras: an orbit) into one [frames][max_rows] block, one gather stacks the n blocks, and the
    # batch's assembly kernel (host restatement: same index map) must give every frame exactly.
    hs, orc = office
    base = hs.render_params(w, h, 1)
    cams = [rtamd.camera_orbit(base, 0.1 * f) for f in range(nf)]
    mr = rtamd.multi_lib().rt_multi_max_rows(h, sh, n)
    gathered = np.full((n, nf, mr, w, 3), np.nan)   # padding rows must never reach a frame
    for g in range(n):
        for f, cam in enumerate(cams):
            p = rtamd.abi.RenderParams.from_buffer_copy(cam)
            p.stripe_height, p.stripe_count, p.stripe_index = sh, n, g
            shard, _ = orc.render(p, pyoracle.MODE_REFERENCE)
            gathered[g, f, :shard.shape[0]] = shard
    frames = rtamd.multi_interleave_frames_host(gathered, h, sh, n)
    for f, cam in enumerate(cams):
        full, _ = orc.render(cam, pyoracle.MODE_REFERENCE)
        assert np.array_equal(frames[f], full), f


def test_interleave_rejects_bad_arguments():
    g = np.zeros((2, 3, 4, 3), np.float32)
    with pytest.raises(rtamd.RtError):
        rtamd.multi_interleave_host(g, 5, 0, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [rtamd.RT_OUT_RGB_F64, rtamd.RT_OUT_RGB_F32])
def test_multi_driver_one_gpu_equals_single_launch(gpu_available, office, fmt):
    hs, _ = office
    m = rtamd.MultiScene(hs, devices=(0,))
    dev = rtamd.DeviceScene(hs, 0)
    for w, h, sh in [(320, 180, 16), (97, 61, 4)]:
        p = hs.render_params(w, h, 1)
        p.out_format = fmt
        img, st, ms = m.render(p, stripe_height=sh)
        ref, rst = dev.render(p)
        assert np.array_equal(img, ref)
        assert [st.primary_rays, st.shadow_rays, st.reflection_rays] == \
            [rst.primary_rays, rst.shadow_rays, rst.reflection_rays]
        assert ms > 0
    m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("assembly", ["gather", "peer"])
@pytest.mark.parametrize("nf,w,h,sh", [(5, 320, 180, 16), (2, 97, 61, 4), (1, 64, 48, 8)])
def test_multi_driver_frames_equal_single_launches(gpu_available, office, nf, w, h, sh, assembly):
    # Batched multi-GPU entry on the box's one GPU (one RCCL rank): batches of frames, two in
    # flight on separate streams / communicators (gather), or the GPU's rows stored straight into
    # the output frames (peer), every frame equal to its own single launch.
    import torch
    hs, _ = office
    m = rtamd.MultiScene(hs, devices=(0,), assembly=assembly)
    dev = rtamd.DeviceScene(hs, 0)
    base = hs.render_params(w, h, 1)
    base.out_format = rtamd.RT_OUT_RGB_F64
    cams = [rtamd.camera_orbit(base, 0.05 * f) for f in range(nf)]
    outs = [torch.full((h, w, 3), float("nan"), dtype=torch.float64, device="cuda") for _ in range(nf)]
    st, ms = m.render_frames(cams, [o.data_ptr() for o in outs], stripe_height=sh, stats=True)
    rays = 0
    for f, cam in enumerate(cams):
        ref, rst = dev.render(cam)
        assert np.array_equal(outs[f].cpu().numpy(), ref), f
        rays += rst.primary_rays + rst.shadow_rays + rst.reflection_rays
    assert st.primary_rays + st.shadow_rays + st.reflection_rays == rays
    assert st.pixels == nf * w * h and ms > 0
    m.close()


@pytest.mark.gpu
def test_multi_driver_frames_async_three_batches(gpu_available, office):
    # The timed path: stats=NULL (launches asynchronous, batch i + 1 renders while batch i is
    # gathered and re-interleaved), more than two batches so every slot is reused after
    # hipEventSynchronize(done) and its pinned output table is rewritten while later batches are in
    # flight.  Batches hold at most RT_MAX_FRAMES (128) frames, so 2 x 128 + 5 frames give 3.
    import torch
    hs, _ = office
    m = rtamd.MultiScene(hs, devices=(0,))
    dev = rtamd.DeviceScene(hs, 0)
    w, h, nf = 40, 24, 2 * rtamd.abi.RT_MAX_FRAMES + 5
    base = hs.render_params(w, h, 1)
    base.out_format = rtamd.RT_OUT_RGB_F64
    cams = [rtamd.camera_orbit(base, 0.004 * f) for f in range(nf)]
    outs = torch.full((nf, h, w, 3), float("nan"), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    st, ms = m.render_frames(cams, [outs[f].data_ptr() for f in range(nf)], stripe_height=4, stats=False)
    assert st is None and ms > 0
    got = outs.cpu().numpy()
    for f, cam in enumerate(cams):
        ref, _ = dev.render(_natural(cam))
        assert np.array_equal(got[f], ref), f
    m.close()


def _natural(p):
    q = rtamd.abi.RenderParams.from_buffer_copy(p)
    q.flags = rtamd.abi.RT_FLAG_NATURAL_ORDER
    return q


@pytest.mark.gpu
@pytest.mark.parametrize("assembly", ["gather", "peer"])
@pytest.mark.parametrize("nf", [1, 3])
def test_multi_driver_two_gpus_equal_single_launch(gpu_available, office, nf, assembly):
    # The N > 1 path proper: grouped ncclGather of several GPUs' padded stripe buffers,
    # per-device streams, re-interleave on devices[0].  Needs a multi-GPU node (the one-GPU
    # box skips it; INTEGRATION.md "Verification status of the N > 1 path").
    import torch
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs")
    hs, _ = office
    devs = tuple(range(min(n, 8)))
    m = rtamd.MultiScene(hs, devices=devs, assembly=assembly)
    dev = rtamd.DeviceScene(hs, 0)
    base = hs.render_params(160, 97, 1)
    base.out_format = rtamd.RT_OUT_RGB_F64
    cams = [rtamd.camera_orbit(base, 0.05 * f) for f in range(nf)]
    outs = [torch.full((97, 160, 3), float("nan"), dtype=torch.float64, device="cuda:0") for _ in range(nf)]
    st, ms = m.render_frames(cams, [o.data_ptr() for o in outs], stripe_height=4, stats=True)
    rays = 0
    for f, cam in enumerate(cams):
        ref, rst = dev.render(cam)
        assert np.array_equal(outs[f].cpu().numpy(), ref), f
        rays += rst.primary_rays + rst.shadow_rays + rst.reflection_rays
    assert st.primary_rays + st.shadow_rays + st.reflection_rays == rays
    assert st.pixels == nf * 160 * 97 and ms > 0
    m.close()


@pytest.mark.gpu
def test_multi_driver_rejects_unknown_assembly(gpu_available, office):
    hs, _ = office
    with pytest.raises(ValueError):
        rtamd.MultiScene(hs, devices=(0,), assembly="scatter")


@pytest.mark.gpu
def test_multi_driver_rejects_duplicate_devices(gpu_available, office):
    hs, _ = office
    with pytest.raises(rtamd.RtError, match="distinct"):
        rtamd.MultiScene(hs, devices=(0, 0))


@pytest.mark.gpu
@pytest.mark.parametrize("assembly", ["gather", "peer"])
def test_cli_gpus_path_pixels(gpu_available, tmp_path, office, assembly):
    hs, orc = office
    out = tmp_path / "m.ppm"
    r = subprocess.run([str(ROOT / "my-raytracer_amd/bin/rt_render"), "--scene", "office", "--width", "96",
                        "--height", "54", "--gpus", "1", "--assembly", assembly, "--out", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert ("RCCL gather" if assembly == "gather" else "peer stores") in r.stdout and "Mrays/s" in r.stdout
    data = out.read_bytes()
    head = b"P6\n96 54\n255\n"
    assert data.startswith(head)
    got = np.frombuffer(data[len(head):], np.uint8).reshape(54, 96, 3).astype(int)
    ref, _ = orc.render(hs.render_params(96, 54, 1), pyoracle.MODE_REFERENCE)
    want = np.floor(np.clip(ref[::-1].astype(np.float32), 0, 1) * np.float32(255) + 0.5).astype(int)
    diff = np.abs(got - want)
    assert diff.max() <= 1 and (diff == 0).mean() >= 0.999
