"""Launch-runtime behaviour of the C-ABI on one MI355X: the kernel watchdog reported without stats,
light tables staged per launch (no device synchronisation), the half grid of overlapped one-frame
launches, argument checks of the host-buffer path, and the multi-GPU driver's peer guard and
gather flags.  Every rendered result is compared bit for bit with a serial single launch."""
import ctypes as C

import numpy as np
import pytest

import rtamd

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(gpu_available):
    return gpu_available


@pytest.fixture(scope="module")
def office():
    hs = rtamd.HostScene.generate("office")
    hs.prepare()
    return hs, rtamd.DeviceScene(hs, 0)


def _natural(p, fmt=None):
    q = rtamd.abi.RenderParams.from_buffer_copy(p)
    q.flags |= rtamd.abi.RT_FLAG_NATURAL_ORDER
    if fmt is not None:
        q.out_format = fmt
    return q


def test_watchdog_reported_by_launch_without_stats(office):
    # A cyclic hierarchy (rt_debug_corrupt_hierarchy: node 0's only child is node 0) makes every
    # traversal loop until the kernel's watchdog ends it.  A launch WITHOUT stats (the production
    # call shape) returns RT_OK asynchronously; its watchdog must then surface: rt_last_kernel_ms,
    # rt_scene_status and every later launch on the scene return RT_ERR_HIP (common/common.h:6-15
    # printed and continued).
    import torch

    hs, _ = office
    bad = rtamd.DeviceScene(hs, 0)
    p = hs.render_params(64, 48, 1)
    buf = torch.zeros((48, 64, 3), dtype=torch.float32, device="cuda")
    bad.launch(p, buf.data_ptr(), stats=False)   # healthy first
    assert bad.last_kernel_ms() > 0 and bad.status() == rtamd.RT_OK
    bad.debug_corrupt_hierarchy()
    bad.launch(p, buf.data_ptr(), stats=False)   # asynchronous: no error yet
    with pytest.raises(rtamd.RtError, match="watchdog"):
        bad.last_kernel_ms()                      # waits for the launch, then reports it
    assert bad.status() == rtamd.abi.RT_ERR_HIP
    assert b"watchdog" in rtamd.hip_lib().rt_last_error()
    with pytest.raises(rtamd.RtError, match="watchdog"):
        bad.launch(p, buf.data_ptr(), stats=False)
    bad.close()
    # another scene of the same process is unaffected
    _, good = office
    img, _ = good.render(p)
    assert np.isfinite(img).all() and good.status() == rtamd.RT_OK


def test_lights_change_per_call_on_three_streams(office):
    # Every launch stages its own light table (the reference copies lights per call,
    # mytracer.cpp:105-118): launches on 3 streams, lights different in every call (inline tables
    # and lights_ext beyond RT_MAX_LIGHTS), nothing synchronised in between -- each result equals
    # its serial render bit for bit.
    import torch

    hs, dev = office
    jobs = []
    for k in range(9):
        p = _natural(hs.render_params(160, 90, 1), rtamd.RT_OUT_RGB_F64)
        n = (2, 20, 400)[k % 3]   # 400 lights (lights_ext) outgrow a context's control block: it grows
        lights = []
        for i in range(n):
            a = 0.7 * k + 2.0 * np.pi * i / n
            lights.append(((1.5 * np.cos(a), 2.0 + 0.1 * k, 1.5 * np.sin(a)), (0.5 / n + 0.03 * (i % 3),) * 3))
        p.set_lights(lights)
        jobs.append(p)
    serial = [dev.render(p)[0] for p in jobs]
    for a in range(len(serial)):
        for b in range(a):
            assert not np.array_equal(serial[a], serial[b])   # the lights do change the image
    streams = [torch.cuda.Stream() for _ in range(3)]
    bufs = [torch.zeros(s_.shape, dtype=torch.float64, device="cuda") for s_ in serial]
    torch.cuda.synchronize()
    for k, p in enumerate(jobs):
        s = streams[k % 3]
        with torch.cuda.stream(s):
            dev.launch(p, bufs[k].data_ptr(), stats=False, stream=s.cuda_stream)
    torch.cuda.synchronize()
    for k in range(len(jobs)):
        assert np.array_equal(bufs[k].cpu().numpy(), serial[k]), k


def test_overlapped_one_frame_launch_takes_half_grid(office):
    # A one-frame launch issued while the scene's previous launch (another stream) still runs takes
    # half the block slots (rt_debug_last_grid records it); pixels do not depend on the grid: both
    # launches equal their serial renders bit for bit.
    import torch

    hs, dev = office
    base = hs.render_params(1920, 1080, 1)
    cams = [_natural(rtamd.camera_orbit(base, 0.01 * f), rtamd.RT_OUT_RGB_F32) for f in range(8)]
    one = _natural(hs.render_params(640, 480, 1), rtamd.RT_OUT_RGB_F32)   # 4800 tiles: more than half a grid
    want_one, _ = dev.render(one)
    b_full = dev.last_grid()
    want_big = []
    for c in cams:
        want_big.append(dev.render(c)[0])
    big = torch.zeros((8, 1080, 1920, 3), dtype=torch.float32, device="cuda")
    small = torch.zeros((480, 640, 3), dtype=torch.float32, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        dev.launch_frames(cams, [big[f].data_ptr() for f in range(8)], stats=False, stream=s1.cuda_stream)
    with torch.cuda.stream(s2):
        dev.launch(one, small.data_ptr(), stats=False, stream=s2.cuda_stream)
    blocks, full = dev.last_grid()
    torch.cuda.synchronize()
    assert full == b_full[1] and 2 * blocks <= full   # 8 frames of 1080p are still running: half grid
    assert np.array_equal(small.cpu().numpy(), want_one)
    for f in range(8):
        assert np.array_equal(big[f].cpu().numpy(), want_big[f]), f
    dev.render(one)
    assert dev.last_grid()[0] == dev.last_grid()[1]   # alone again: the whole grid


def test_render_to_host_rejects_global_rows(office):
    # the host buffer holds the packed shard: a frame-layout flag would overrun it
    hs, dev = office
    p = hs.render_params(64, 48, 1)
    p.stripe_height, p.stripe_count, p.stripe_index = 8, 2, 1
    p.flags |= rtamd.abi.RT_FLAG_GLOBAL_ROWS
    host = np.zeros((rtamd.rows_in_shard(p), 64, 3), np.float32)
    rc = rtamd.hip_lib().rt_render_to_host(dev._h, C.byref(p), host.ctypes.data_as(C.c_void_p), None)
    assert rc == rtamd.abi.RT_ERR_INVALID and b"GLOBAL_ROWS" in rtamd.hip_lib().rt_last_error()


def test_multi_gather_clears_global_rows_flag(office):
    # the gather assembly renders packed stripes whatever flags the caller's params carry (a params
    # block reused from the peer path keeps RT_FLAG_GLOBAL_ROWS): frames equal the single launch
    import torch

    hs, dev = office
    m = rtamd.MultiScene(hs, devices=(0,), assembly="gather")
    p = _natural(hs.render_params(97, 61, 1), rtamd.RT_OUT_RGB_F64)
    p.flags |= rtamd.abi.RT_FLAG_GLOBAL_ROWS
    outs = [torch.full((61, 97, 3), float("nan"), dtype=torch.float64, device="cuda") for _ in range(3)]
    m.render_frames([p] * 3, [o.data_ptr() for o in outs], stripe_height=4)
    q = _natural(hs.render_params(97, 61, 1), rtamd.RT_OUT_RGB_F64)
    ref, _ = dev.render(q)
    for o in outs:
        assert np.array_equal(o.cpu().numpy(), ref)
    m.close()


@pytest.mark.parametrize("inject", [False, True])
def test_multi_peer_guard(office, inject):
    # RT_MULTI_PEER is kept only if the guard's check frame (a corner window of the first frame,
    # rendered by the gather and by peer stores) is bit-identical; an injected mismatch
    # (rt_multi_debug_inject) makes the driver gather instead.  Either way the frames are right.
    import torch

    hs, dev = office
    m = rtamd.MultiScene(hs, devices=(0,), assembly="peer")
    if inject:
        m.debug_inject(rtamd.abi.RT_MULTI_DEBUG_PEER_MISMATCH)
    assert m.assembly_in_use == "peer"   # not checked before the first render
    p = _natural(hs.render_params(160, 97, 1), rtamd.RT_OUT_RGB_F64)
    cams = [rtamd.camera_orbit(p, 0.04 * f) for f in range(2)]
    outs = [torch.full((97, 160, 3), float("nan"), dtype=torch.float64, device="cuda") for _ in range(2)]
    m.render_frames(cams, [o.data_ptr() for o in outs], stripe_height=4)
    assert m.assembly_in_use == ("gather" if inject else "peer")
    for f, c in enumerate(cams):
        ref, _ = dev.render(c)
        assert np.array_equal(outs[f].cpu().numpy(), ref), f
    m.close()


def test_multi_calls_keep_the_current_device(office):
    # every rt_multi entry point leaves the calling thread's current device as it was
    import torch

    hs, _ = office
    before = torch.cuda.current_device()
    m = rtamd.MultiScene(hs, devices=(torch.cuda.device_count() - 1,), assembly="peer")
    assert torch.cuda.current_device() == before
    img, _, _ = m.render(hs.render_params(32, 24, 1))
    assert torch.cuda.current_device() == before and img.shape == (24, 32, 3)
    m.close()
    assert torch.cuda.current_device() == before


@pytest.mark.parametrize("n", [2, 3, 4, 8, 16])
def test_sample_groups_equal_lane_per_pixel(office, n):
    # spp_lanes = 1: a pixel's n x n samples run on neighbouring lanes of one wave (groups of
    # min(n^2, 32) lanes; n^2 = 64, 256: two / eight chunks of 32 with the running sum in the path state) and are
    # summed in sample order on chip; n = 3 (9 samples, not a power of two) keeps one lane per pixel.
    # Pixels and ray counts equal the lane-per-pixel render bit for bit -- one frame, several frames
    # in one launch, a striped shard -- and the oracle within the fp64 tolerance.
    import torch
    import pyoracle

    hs, _ = office
    on, off = rtamd.DeviceScene(hs, 0, spp_lanes=1), rtamd.DeviceScene(hs, 0, spp_lanes=-1)
    w, h = (64, 40) if n <= 8 else (24, 16)
    p = hs.render_params(w, h, n)
    p.out_format = rtamd.RT_OUT_RGB_F64
    a, sa = on.render(p)
    b, sb = off.render(p)
    assert np.array_equal(a, b) and [sa.primary_rays, sa.shadow_rays, sa.reflection_rays] == \
        [sb.primary_rays, sb.shadow_rays, sb.reflection_rays]
    if n == 4:
        ref, cnt = pyoracle.Oracle(hs.raw, hs).render(p, pyoracle.MODE_REFERENCE)
        assert np.abs(a - ref).max() <= 1e-12 and sa.primary_rays == cnt.primary_rays
    cams = []
    for f in range(3):
        c = rtamd.camera_orbit(p, 0.05 * f)
        c.stripe_height, c.stripe_count, c.stripe_index = 4, 3, 1
        cams.append(c)
    rows = rtamd.rows_in_shard(cams[0])
    outs = {k: [torch.full((rows, w, 3), float("nan"), dtype=torch.float64, device="cuda") for _ in cams]
            for k in ("on", "off")}
    st_on = on.launch_frames(cams, [o.data_ptr() for o in outs["on"]], stats=True)
    st_off = off.launch_frames(cams, [o.data_ptr() for o in outs["off"]], stats=True)
    for x, y in zip(outs["on"], outs["off"]):
        assert torch.equal(x, y)
    assert st_on.primary_rays + st_on.shadow_rays + st_on.reflection_rays == \
        st_off.primary_rays + st_off.shadow_rays + st_off.reflection_rays
    on.close()
    off.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,cap", [(4, 4), (8, 16), (8, 2), (16, 32)])
def test_sample_group_size_cap_changes_no_pixel(office, n, cap):
    # rt_upload_options.spp_lanes = 2..64 caps the group at that many lanes: the n^2 samples then
    # run in n^2 / cap chunks (the running sum in the path state between chunks), in sample order
    import torch

    hs, _ = office
    capd, off = rtamd.DeviceScene(hs, 0, spp_lanes=cap), rtamd.DeviceScene(hs, 0, spp_lanes=-1)
    w, h = (48, 32) if n <= 8 else (20, 12)
    p = hs.render_params(w, h, n)
    p.out_format = rtamd.RT_OUT_RGB_F64
    a, sa = capd.render(p)
    b, sb = off.render(p)
    assert np.array_equal(a, b)
    assert [sa.primary_rays, sa.shadow_rays, sa.reflection_rays] == [sb.primary_rays, sb.shadow_rays, sb.reflection_rays]
    p1 = hs.render_params(w, h, 1)
    p1.out_format = rtamd.RT_OUT_RGB_F64
    prim = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda")
    capd.launch(p1, prim.data_ptr())
    outs = [torch.full((h, w, 3), float("nan"), dtype=torch.float64, device="cuda") for _ in range(2)]
    _, n1 = capd.launch_adaptive(p1, prim.data_ptr(), outs[0].data_ptr(), n, -1.0, stats=True)
    _, n2 = off.launch_adaptive(p1, prim.data_ptr(), outs[1].data_ptr(), n, -1.0, stats=True)
    torch.cuda.synchronize()
    assert n1 == n2 and torch.equal(outs[0], outs[1])
    capd.close()
    off.close()
    for bad in (-2, 3, 6, 128):   # -1, 0, 1 or a power of two <= 64
        with pytest.raises(RuntimeError):
            rtamd.DeviceScene(hs, 0, spp_lanes=bad)


@pytest.mark.gpu
@pytest.mark.parametrize("subp", [2, 3, 4, 8, 16])
def test_adaptive_sample_groups_equal_sample_buffer(office, subp):
    # The adaptive pass with sample groups (a selected pixel's subp^2 samples on neighbouring lanes,
    # summed in (si, sj) order by the render kernel: no sample buffer, no reduce kernel, no
    # read-back of the selection count) against the sample-buffer path (spp_lanes = -1): the same
    # pixels bit for bit, the same selection and ray counts -- one frame, several frames in one
    # launch, a row shard with its halo, every interior pixel selected (threshold -1).
    import torch

    hs, _ = office
    on, off = rtamd.DeviceScene(hs, 0, spp_lanes=1), rtamd.DeviceScene(hs, 0, spp_lanes=-1)
    w, h = (64, 40) if subp <= 8 else (24, 16)
    p = hs.render_params(w, h, 1)
    p.out_format = rtamd.RT_OUT_RGB_F64
    rays = lambda s: (s.primary_rays, s.shadow_rays, s.reflection_rays)  # noqa: E731
    cams = [rtamd.camera_orbit(p, 0.05 * f) for f in range(3)]
    prims = [torch.zeros((h, w, 3), dtype=torch.float64, device="cuda") for _ in cams]
    on.launch_frames(cams, [x.data_ptr() for x in prims])
    for thr in (0.02, -1.0):
        res = {}
        for k, d in (("on", on), ("off", off)):
            outs = [torch.full((h, w, 3), float("nan"), dtype=torch.float64, device="cuda") for _ in cams]
            one = torch.full((h, w, 3), float("nan"), dtype=torch.float64, device="cuda")
            s1, n1 = d.launch_adaptive(cams[1], prims[1].data_ptr(), one.data_ptr(), subp, thr, stats=True)
            sf, nf = d.launch_adaptive_frames(cams, [x.data_ptr() for x in prims], [o.data_ptr() for o in outs],
                                              subp, thr, stats=True)
            torch.cuda.synchronize()
            res[k] = (one.cpu().numpy(), rays(s1), n1, [o.cpu().numpy() for o in outs], rays(sf), nf)
        a, b = res["on"], res["off"]
        assert a[2] == b[2] and a[5] == b[5] and a[2] > 0
        assert a[1] == b[1] and a[4] == b[4]
        assert np.array_equal(a[0], b[0], equal_nan=True)
        for x, y in zip(a[3], b[3]):
            assert np.array_equal(x, y, equal_nan=True)
    on.close()
    off.close()
