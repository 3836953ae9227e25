"""rtamd — Python host mirror of the MI355X render path.

Thin ctypes layer over the two C-ABIs built in-tree:
  lib/librt_host.so  (include/rt_host.h)  scene load / generate, normals,
                     SoA flattening, median-split BVH  (C++)
  lib/librt_hip.so   (include/rt_hip.h)   device upload + the flattened HIP
                     render kernel for gfx950
The classes mirror the reference's host flow (Raytracer::init_cuda,
mytracer.cpp:54-60; Raytracer::compute_image_cuda, mytracer.cpp:123-159).
There is no CPU fallback: if a library is missing every call fails loudly.
"""
import ctypes as C
import os
from pathlib import Path

import numpy as np

from . import abi
from .abi import RT_OK, RT_OUT_RGB_F32, RT_OUT_RGB_F64, RT_FLAG_TRAVERSAL_STATS, RT_FLAG_WIDE_STATS, RT_FLAG_TIMELINE  # noqa: F401

PKG_ROOT = Path(__file__).resolve().parent.parent
LIB_DIR = PKG_ROOT / "lib"
HOST_LIB = LIB_DIR / "librt_host.so"
HIP_LIB = Path(os.environ.get("RTAMD_HIP_LIB", LIB_DIR / "librt_hip.so"))   # override: kernel variants
MULTI_LIB = LIB_DIR / "librt_multi.so"

_host = None
_hip = None
_multi = None


class RtError(RuntimeError):
    pass


def host_lib():
    global _host
    if _host is None:
        if not HOST_LIB.exists():
            raise RtError(f"{HOST_LIB} not built: run `make -C my-raytracer_amd` or __graft_entry__.build()")
        _host = abi.bind(C.CDLL(str(HOST_LIB)), abi.HOST_SYMBOLS)
    return _host


def _one_hip_runtime():
    """PyTorch-ROCm ships its own HIP runtime (torch/lib/libamdhip64.so).  Load it before our
    libraries so that they bind to it: a process holding both that copy and /opt/rocm's
    (ours loaded first, torch imported later) sees no devices in one of them."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def hip_lib():
    global _hip
    if _hip is None:
        _one_hip_runtime()
        if not HIP_LIB.exists():
            raise RtError(f"{HIP_LIB} not built: run `make -C my-raytracer_amd` or __graft_entry__.build()")
        _hip = abi.bind(C.CDLL(str(HIP_LIB)), abi.HIP_SYMBOLS, partial="RTAMD_HIP_LIB" in os.environ)
    return _hip


def multi_lib():
    """librt_multi.so (include/rt_multi.h): the single-process multi-GPU driver (RCCL)."""
    global _multi
    if _multi is None:
        if not MULTI_LIB.exists():
            raise RtError(f"{MULTI_LIB} not built: run `make -C my-raytracer_amd` or __graft_entry__.build()")
        hip_lib()   # librt_multi links librt_hip: load the same copy first
        _multi = abi.bind(C.CDLL(str(MULTI_LIB)), abi.MULTI_SYMBOLS)
    return _multi


def _check_host(rc, what):
    if rc != RT_OK:
        raise RtError(f"{what}: {host_lib().rt_host_last_error().decode()}")


def _check_hip(rc, what):
    if rc != RT_OK:
        raise RtError(f"{what}: {hip_lib().rt_last_error().decode()}")


def usable_cpus():
    """CPUs this process may run on: the affinity mask, bounded by a cgroup CPU quota (the GPU
    box grants 16 CPUs of a 256-thread host per GPU)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


_TREES = {"sah": abi.RT_TREE_SAH, "reference": abi.RT_TREE_REFERENCE, "sbvh": abi.RT_TREE_SBVH}


def upload_options(tree=None, **fields):
    """rt_upload_options with the library defaults (rt_upload_options_init), the device tree
    (None = default, or "sbvh" / "sah" / "reference") and any other fields set.  build_threads
    defaults to usable_cpus() (the library would use every hardware thread)."""
    opt = abi.UploadOptions()
    hip_lib().rt_upload_options_init(C.byref(opt))
    opt.build_threads = usable_cpus()
    if tree is not None:
        if tree not in _TREES:
            raise ValueError(f"tree must be one of {sorted(_TREES)}")
        opt.device_tree = _TREES[tree]
    names = {n for n, _ in abi.UploadOptions._fields_ if n != "reserved_"}
    for k, v in fields.items():
        if k not in names:
            raise ValueError(f"unknown upload option {k!r}")
        setattr(opt, k, v)
    return opt


def _np(ptr, count, dtype):
    if count == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(count,)).view(dtype)


class HostScene:
    """Host-resident scene (rt_host_scene*)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def generate(cls, kind, width=0, height=0, n_triangles=0, seed=0, max_depth=-1, detail=0):
        gp = abi.GenParams(width=width, height=height, n_triangles=n_triangles, seed=seed,
                           max_depth=max_depth, detail=detail)
        h = C.c_void_p()
        _check_host(host_lib().rt_host_generate(kind.encode(), C.byref(gp), C.byref(h)), f"generate {kind}")
        return cls(h)

    @classmethod
    def load(cls, path):
        h = C.c_void_p()
        _check_host(host_lib().rt_host_load(str(path).encode(), C.byref(h)), f"load {path}")
        return cls(h)

    @property
    def handle(self):
        if self._h is None:
            raise RtError("scene closed")
        return self._h

    def close(self):
        if self._h is not None:
            host_lib().rt_host_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def prepare(self, build_threads=0):
        """compute_normals + build_Data + BVH::initSoA; build_threads 0 = the usable CPUs."""
        secs = C.c_double(0.0)
        _check_host(host_lib().rt_host_prepare_ex(self.handle, int(build_threads), C.byref(secs)), "prepare")
        return secs.value

    @property
    def raw(self):
        return host_lib().rt_host_raw(self.handle)

    @property
    def soa(self):
        p = host_lib().rt_host_soa(self.handle)
        if not p:
            raise RtError("scene not prepared")
        return p

    @property
    def bvh(self):
        p = host_lib().rt_host_bvh(self.handle)
        if not p:
            raise RtError("scene not prepared")
        return p

    def soa_arrays(self):
        s = self.soa.contents
        nt = s.n_vertex_idx // 3
        return {
            "vertex_pos": _np(s.vertex_pos, 3 * s.n_vertices, np.float64).reshape(-1, 3),
            "vertex_normals": _np(s.vertex_normals, 3 * s.n_vertices, np.float64).reshape(-1, 3),
            "vertex_mesh_id": _np(s.vertex_mesh_id, s.n_vertices, np.int32),
            "face_normals": _np(s.face_normals, 3 * nt, np.float64).reshape(-1, 3),
            "vertex_idx": _np(s.vertex_idx, s.n_vertex_idx, np.int32).reshape(-1, 3),
            "texture_idx": _np(s.texture_idx, s.n_vertex_idx, np.int32).reshape(-1, 3),
        }

    def bvh_arrays(self):
        b = self.bvh.contents
        n = b.n_nodes
        return {
            "bb_min": _np(b.bb_min, 3 * n, np.float64).reshape(-1, 3),
            "bb_max": _np(b.bb_max, 3 * n, np.float64).reshape(-1, 3),
            "left_child": _np(b.left_child, n, np.int32),
            "first_tri": _np(b.first_tri, n, np.int32),
            "tri_count": _np(b.tri_count, n, np.int32),
        }

    def camera(self, width=0, height=0):
        cam = abi.Camera()
        _check_host(host_lib().rt_host_camera(self.handle, width, height, C.byref(cam)), "camera")
        return cam

    def render_params(self, width=0, height=0, spp_n=1):
        p = abi.RenderParams()
        _check_host(host_lib().rt_host_render_params(self.handle, width, height, spp_n, C.byref(p)),
                    "render_params")
        return p

    def save(self, path):
        _check_host(host_lib().rt_host_save(self.handle, str(path).encode()), f"save {path}")

    @property
    def triangle_count(self):
        return int(host_lib().rt_host_triangle_count(self.handle))

    @property
    def bvh_depth(self):
        return int(host_lib().rt_host_bvh_depth(self.handle))


class DeviceScene:
    """Scene resident on one MI355X (rt_scene*), uploaded from a prepared HostScene."""

    def __init__(self, host_scene, device=0, analytic=False, tree=None, **options):
        """analytic=True also uploads the raw scene's spheres and planes (rt_scene_set_analytic,
        CPU intersect_scene semantics); the default traces meshes only, like the reference GPU
        path (mytracer_gpu.cu:314-328).  tree: None (library default, "sbvh": SAH with
        spatial splits), "sbvh", "sah" (object splits only) or "reference" -- the device
        traversal hierarchy (pixels and ray counts do not depend on it).  options: other
        rt_upload_options fields (stack_ring=16, lds_treelet=-1 (none), sbvh_leaf_max=1, ...)."""
        self._h = C.c_void_p()
        self.device = device
        opt = upload_options(tree, **options)
        _check_hip(hip_lib().rt_scene_upload_ex(host_scene.soa, host_scene.bvh, device, C.byref(opt),
                                                C.byref(self._h)), "rt_scene_upload_ex")
        self.tree = tree
        self.analytic = False
        if analytic:
            r = host_scene.raw.contents
            self.set_analytic(r.spheres, r.n_spheres, r.planes, r.n_planes)

    def set_analytic(self, spheres, n_spheres, planes, n_planes):
        """Replaces the analytic primitives (ctypes arrays/pointers of abi.Sphere / abi.Plane)."""
        _check_hip(hip_lib().rt_scene_set_analytic(self._h, spheres, n_spheres, planes, n_planes),
                   "rt_scene_set_analytic")
        self.analytic = (n_spheres + n_planes) > 0

    def close(self):
        if self._h:
            hip_lib().rt_scene_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def device_bytes(self):
        return int(hip_lib().rt_scene_device_bytes(self._h))

    @property
    def upload_seconds(self):
        """(build_s, copy_s) of rt_scene_upload: the device layout built on the host (hierarchy,
        collapse, records), then device allocation + H2D copies (rt_scene_upload_seconds)."""
        b, c = C.c_double(), C.c_double()
        _check_hip(hip_lib().rt_scene_upload_seconds(self._h, C.byref(b), C.byref(c)), "rt_scene_upload_seconds")
        return b.value, c.value

    def launch(self, params, d_out, stats=False, stream=None):
        """Asynchronous render into a device buffer (int pointer); returns Stats if stats=True."""
        st = abi.Stats() if stats else None
        _check_hip(hip_lib().rt_launch_compute_image(self._h, C.byref(params), C.c_void_p(d_out),
                                                     C.byref(st) if st is not None else None,
                                                     C.c_void_p(stream) if stream else None),
                   "rt_launch_compute_image")
        return st

    def launch_frames(self, params, d_outs, stats=False, stream=None):
        """Asynchronous render of len(d_outs) frames in ONE launch (rt_launch_frames); params is
        one RenderParams (every frame the same) or a list of them differing only in their camera
        vectors.  Returns Stats summed over the frames if stats=True."""
        n = len(d_outs)
        plist = params if isinstance(params, (list, tuple)) else [params] * n
        if len(plist) != n:
            raise ValueError("one params per output buffer")
        parr = (abi.RenderParams * n)(*plist)
        oarr = (C.c_void_p * n)(*[C.c_void_p(d) for d in d_outs])
        st = abi.Stats() if stats else None
        _check_hip(hip_lib().rt_launch_frames(self._h, parr, n, oarr, C.byref(st) if st is not None else None,
                                              C.c_void_p(stream) if stream else None), "rt_launch_frames")
        return st

    def launch_adaptive(self, params, d_primary, d_out, subp=4, threshold=0.02, stats=False, stream=None):
        """Adaptive supersampling pass (rt_launch_adaptive) over device buffers (int pointers);
        returns (Stats or None, number of re-rendered pixels)."""
        st = abi.Stats() if stats else None
        nsel = C.c_longlong(-1)   # only requested with stats (reading it synchronises)
        _check_hip(hip_lib().rt_launch_adaptive(self._h, C.byref(params), C.c_void_p(d_primary), C.c_void_p(d_out),
                                                subp, threshold, C.byref(st) if st is not None else None,
                                                C.byref(nsel) if stats else None,
                                                C.c_void_p(stream) if stream else None),
                   "rt_launch_adaptive")
        return st, int(nsel.value)

    def launch_adaptive_frames(self, params, d_primaries, d_outs, subp=4, threshold=0.02, stats=False, stream=None):
        """Adaptive pass over len(d_outs) full frames in one render launch (rt_launch_adaptive_frames);
        params as launch_frames.  Returns (Stats or None, re-rendered pixels over all frames)."""
        n = len(d_outs)
        plist = params if isinstance(params, (list, tuple)) else [params] * n
        if len(plist) != n or len(d_primaries) != n:
            raise ValueError("one params and one primary image per output buffer")
        parr = (abi.RenderParams * n)(*plist)
        parr_p = (C.c_void_p * n)(*[C.c_void_p(d) for d in d_primaries])
        oarr = (C.c_void_p * n)(*[C.c_void_p(d) for d in d_outs])
        st = abi.Stats() if stats else None
        nsel = C.c_longlong(-1)
        _check_hip(hip_lib().rt_launch_adaptive_frames(self._h, parr, n, parr_p, oarr, subp, threshold,
                                                       C.byref(st) if st is not None else None,
                                                       C.byref(nsel) if stats else None,
                                                       C.c_void_p(stream) if stream else None),
                   "rt_launch_adaptive_frames")
        return st, int(nsel.value)

    def launch_adaptive_shard(self, params, d_primary, d_halo, d_out, subp=4, threshold=0.02, stats=False,
                              stream=None):
        """Adaptive pass over a row shard (rt_launch_adaptive_shard): d_primary / d_out are the
        shard's packed rows, d_halo the rows adaptive_halo_rows(params) lists (0: none needed)."""
        st = abi.Stats() if stats else None
        nsel = C.c_longlong(-1)
        _check_hip(hip_lib().rt_launch_adaptive_shard(self._h, C.byref(params), C.c_void_p(d_primary),
                                                      C.c_void_p(d_halo) if d_halo else None, C.c_void_p(d_out),
                                                      subp, threshold, C.byref(st) if st is not None else None,
                                                      C.byref(nsel) if stats else None,
                                                      C.c_void_p(stream) if stream else None),
                   "rt_launch_adaptive_shard")
        return st, int(nsel.value)

    def render_adaptive(self, params, subp=4, threshold=0.02):
        """Primary pass (fp64) + adaptive pass, the reference's launch_compute_image_device
        (mytracer_gpu.cu:44-113); returns (image[H, W, 3], primary Stats, adaptive Stats, n_selected)."""
        import torch

        H, W = params.camera.height, params.camera.width
        prim = torch.zeros((H, W, 3), dtype=torch.float64, device=f"cuda:{self.device}")
        dtype = torch.float64 if params.out_format == RT_OUT_RGB_F64 else torch.float32
        out = torch.zeros((H, W, 3), dtype=dtype, device=f"cuda:{self.device}")
        q = abi.RenderParams.from_buffer_copy(params)
        q.out_format = RT_OUT_RGB_F64
        st0 = self.launch(q, prim.data_ptr(), stats=True)
        st1, nsel = self.launch_adaptive(params, prim.data_ptr(), out.data_ptr(), subp, threshold, stats=True)
        return out.cpu().numpy(), st0, st1, nsel

    def render_adaptive_to_host(self, params, subp=4, threshold=0.02, out=None):
        """rt_render_adaptive_to_host: primary + adaptive pass + copy in one synchronous call (the
        reference's launch_compute_image_device); out: a host array [H, W, 3] of params.out_format
        (numpy, or a pinned torch tensor's numpy view).  Returns (image, primary Stats, adaptive
        Stats, n_selected)."""
        H, W = params.camera.height, params.camera.width
        dtype = np.float64 if params.out_format == RT_OUT_RGB_F64 else np.float32
        img = np.zeros((H, W, 3), dtype=dtype) if out is None else out
        if img.shape != (H, W, 3) or img.dtype != dtype or not img.flags["C_CONTIGUOUS"]:
            raise ValueError("out must be a C-contiguous [H, W, 3] array of the output format")
        st0, st1, nsel = abi.Stats(), abi.Stats(), C.c_longlong(-1)
        _check_hip(hip_lib().rt_render_adaptive_to_host(self._h, C.byref(params), subp, threshold,
                                                        img.ctypes.data_as(C.c_void_p), C.byref(st0), C.byref(st1),
                                                        C.byref(nsel)), "rt_render_adaptive_to_host")
        return img, st0, st1, int(nsel.value)

    def render(self, params):
        """Synchronous render to host; returns (image[rows, W, 3], Stats)."""
        rows = rows_in_shard(params)
        dtype = np.float64 if params.out_format == RT_OUT_RGB_F64 else np.float32
        img = np.zeros((rows, params.camera.width, 3), dtype=dtype)
        st = abi.Stats()
        _check_hip(hip_lib().rt_render_to_host(self._h, C.byref(params), img.ctypes.data_as(C.c_void_p),
                                               C.byref(st)), "rt_render_to_host")
        return img, st

    def debug_counters(self):
        """Raw counter words of the last launch (see rt_debug_counters in rt_hip.h)."""
        buf = (C.c_ulonglong * 40)()
        n = hip_lib().rt_debug_counters(self._h, buf, 40)
        if n < 0:
            _check_hip(n, "rt_debug_counters")
        names = {16: "node_iters", 17: "node_lanes", 18: "leaf_iters", 19: "leaf_lanes", 20: "trav_cycles",
                 21: "shade_cycles", 22: "fetch_cycles", 23: "outer_iters", 24: "trav_rounds", 25: "trav_round_lanes",
                 26: "stack_spills", 27: "node_lines", 28: "leaf_lines", 29: "big_leaf_tests",
                 30: "node_lds_iters", 32: "gnode_uniform_iters", 33: "gnode_distinct", 34: "leaf_uniform_iters",
                 35: "anyhit_tri_tests", 36: "anyhit_own_record_tests"}
        return {v: int(buf[k]) for k, v in names.items()}

    def wave_log(self, max_waves=1 << 16):
        """Per-wave {start, last fetch, end, pixels} of the last STATS launch (rt_debug_wave_log)."""
        buf = np.zeros(4 * max_waves, dtype=np.uint64)
        n = hip_lib().rt_debug_wave_log(self._h, buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), len(buf))
        if n < 0:
            _check_hip(int(n), "rt_debug_wave_log")
        return buf[:n].reshape(-1, 4)

    def timeline(self, max_waves=1 << 14):
        """Per-round records [wave, round, 4] of the last RT_FLAG_TIMELINE launch (rt_debug_timeline)."""
        buf = np.zeros(8 * 256 * max_waves, dtype=np.uint64)
        n = hip_lib().rt_debug_timeline(self._h, buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), len(buf))
        if n < 0:
            _check_hip(int(n), "rt_debug_timeline")
        return buf[:n].reshape(-1, 256, 8)

    def last_kernel_ms(self):
        ms = C.c_float(0.0)
        _check_hip(hip_lib().rt_last_kernel_ms(self._h, C.byref(ms)), "rt_last_kernel_ms")
        return ms.value

    def status(self):
        """rt_scene_status: RT_OK, or RT_ERR_HIP once a finished launch tripped the kernel watchdog."""
        return int(hip_lib().rt_scene_status(self._h))

    def last_grid(self):
        """(blocks, full_blocks) of the last launch's persistent grid (rt_debug_last_grid)."""
        b, f = C.c_longlong(0), C.c_longlong(0)
        _check_hip(hip_lib().rt_debug_last_grid(self._h, C.byref(b), C.byref(f)), "rt_debug_last_grid")
        return b.value, f.value

    def debug_corrupt_hierarchy(self):
        """Test hook (rt_debug_corrupt_hierarchy): the first 4-wide node becomes a cycle."""
        _check_hip(hip_lib().rt_debug_corrupt_hierarchy(self._h), "rt_debug_corrupt_hierarchy")


def tile_shape():
    """(width, height) of the render kernel's work tile (rt_tile_shape)."""
    w, h = C.c_int(0), C.c_int(0)
    _check_hip(hip_lib().rt_tile_shape(C.byref(w), C.byref(h)), "rt_tile_shape")
    return w.value, h.value


def ipc_handle(d_ptr):
    """(handle bytes, offset) exporting the device allocation that holds d_ptr to other
    processes (rt_ipc_get_handle)."""
    h = C.create_string_buffer(abi.RT_IPC_HANDLE_BYTES)
    off = C.c_ulonglong(0)
    _check_hip(hip_lib().rt_ipc_get_handle(C.c_void_p(d_ptr), h, C.byref(off)), "rt_ipc_get_handle")
    return h.raw, off.value


def ipc_open(handle, offset, device, owner_device=-1):
    """Device pointer in this process (device `device` current) to the bytes another process
    exported with ipc_handle from its device `owner_device` (this process's numbering; -1 =
    unknown), with peer access from device to owner enabled (rt_ipc_open)."""
    if len(handle) != abi.RT_IPC_HANDLE_BYTES:
        raise ValueError("IPC handle must be RT_IPC_HANDLE_BYTES bytes")
    p = C.c_void_p(0)
    _check_hip(hip_lib().rt_ipc_open(handle, C.c_ulonglong(offset), int(device), int(owner_device), C.byref(p)),
               "rt_ipc_open")
    return int(p.value)


def ipc_close(d_ptr, offset):
    _check_hip(hip_lib().rt_ipc_close(C.c_void_p(d_ptr), C.c_ulonglong(offset)), "rt_ipc_close")


def rows_in_shard(params):
    return int(hip_lib().rt_rows_in_shard(C.byref(params)))


def adaptive_halo_rows(params):
    """Global rows rt_launch_adaptive_shard's halo must hold ([2s] below / [2s+1] above
    segment s; -1 = outside the frame), from the library itself (no GPU needed)."""
    n = int(hip_lib().rt_adaptive_halo_rows(C.byref(params), None, 0))
    _check_hip(min(n, 0), "rt_adaptive_halo_rows")
    buf = (C.c_int * max(1, n))()
    _check_hip(min(0, int(hip_lib().rt_adaptive_halo_rows(C.byref(params), buf, n))), "rt_adaptive_halo_rows")
    return np.array(buf[:n], dtype=np.int64)


def shard_rows(height, stripe_height, stripe_count, stripe_index):
    """Global row ids a shard renders, in output order (rt_render_params rules)."""
    y = np.arange(height)
    return y[(y // stripe_height) % stripe_count == stripe_index]


def camera_orbit(params, angle):
    """Copy of params whose camera is turned rigidly by `angle` radians about the image's
    vertical axis (y_dir) through the point the image centre looks at (lower_left +
    W/2 x_dir + H/2 y_dir): eye, lower_left, x_dir and y_dir rotate together, so every frame
    is a valid pinhole camera of the same scene.  Frames of an animation path for
    rt_launch_frames, which lets frames differ only in these four vectors."""
    q = abi.RenderParams.from_buffer_copy(params)
    cam = q.camera
    eye, ll = np.array(cam.eye[:]), np.array(cam.lower_left[:])
    xd, yd = np.array(cam.x_dir[:]), np.array(cam.y_dir[:])
    c = ll + 0.5 * cam.width * xd + 0.5 * cam.height * yd
    k = yd / np.linalg.norm(yd)
    kx = np.array([[0.0, -k[2], k[1]], [k[2], 0.0, -k[0]], [-k[1], k[0], 0.0]])
    R = np.eye(3) + np.sin(angle) * kx + (1.0 - np.cos(angle)) * (kx @ kx)   # Rodrigues
    for name, v in (("eye", c + R @ (eye - c)), ("lower_left", c + R @ (ll - c)), ("x_dir", R @ xd),
                    ("y_dir", R @ yd)):
        getattr(cam, name)[:] = [float(x) for x in v]
    return q


def write_ppm(path, img):
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w, _ = img.shape
    _check_host(host_lib().rt_write_ppm(str(path).encode(), img.ctypes.data_as(C.POINTER(C.c_float)), w, h),
                "rt_write_ppm")


class MultiScene:
    """One scene on several GPUs of this node, one process (rt_multi.h): every frame is cut
    into interleaved row stripes per GPU and assembled on devices[0] by one RCCL gather
    (assembly="gather") or by every GPU storing its rows into devices[0]'s frames ("peer")."""

    def __init__(self, host_scene, devices=(0,), tree=None, assembly="gather", **options):
        self._h = C.c_void_p()
        devs = (C.c_int * len(devices))(*devices)
        opt = upload_options(tree, **options)
        rc = multi_lib().rt_multi_create(host_scene.soa, host_scene.bvh, devs, len(devices), C.byref(opt),
                                         C.byref(self._h))
        if rc != RT_OK:
            raise RtError(f"rt_multi_create: {multi_lib().rt_multi_last_error().decode()}")
        self.devices = tuple(devices)
        modes = {"gather": abi.RT_MULTI_GATHER, "peer": abi.RT_MULTI_PEER}
        if assembly not in modes:
            self.close()
            raise ValueError(f"assembly must be one of {sorted(modes)}")
        if multi_lib().rt_multi_set_assembly(self._h, modes[assembly]) != RT_OK:
            err = multi_lib().rt_multi_last_error().decode()
            self.close()
            raise RtError(f"rt_multi_set_assembly: {err}")
        self.assembly = assembly

    @property
    def assembly_in_use(self):
        """"gather" or "peer": the assembly rt_multi_render* use now (the peer guard falls back to
        the gather when the peer stores did not assemble a bit-identical check frame)."""
        a = multi_lib().rt_multi_assembly(self._h)
        if a < 0:
            raise RtError(f"rt_multi_assembly: {multi_lib().rt_multi_last_error().decode()}")
        return "peer" if a == abi.RT_MULTI_PEER else "gather"

    def debug_inject(self, what):
        """Test hook (rt_multi_debug_inject): abi.RT_MULTI_DEBUG_PEER_MISMATCH, or 0."""
        if multi_lib().rt_multi_debug_inject(self._h, int(what)) != RT_OK:
            raise RtError(f"rt_multi_debug_inject: {multi_lib().rt_multi_last_error().decode()}")

    def render(self, params, stripe_height=16):
        """Synchronous render of the whole frame to host memory -> (image [H, W, 3], Stats, ms)."""
        dt = np.float64 if params.out_format == RT_OUT_RGB_F64 else np.float32
        img = np.zeros((params.camera.height, params.camera.width, 3), dtype=dt)
        st, ms = abi.Stats(), C.c_double()
        rc = multi_lib().rt_multi_render_to_host(self._h, C.byref(params), stripe_height, img.ctypes.data_as(C.c_void_p),
                                                 C.byref(st), C.byref(ms))
        if rc != RT_OK:
            raise RtError(f"rt_multi_render: {multi_lib().rt_multi_last_error().decode()}")
        return img, st, ms.value

    def render_frames(self, params, d_outs, stripe_height=16, stats=False):
        """Renders len(d_outs) frames into device buffers on devices[0] (int pointers) with
        rt_multi_render_frames (batched launches, two batches in flight); params: one
        RenderParams or one per frame.  Returns (Stats or None, wall ms)."""
        n = len(d_outs)
        plist = params if isinstance(params, (list, tuple)) else [params] * n
        if len(plist) != n:
            raise ValueError("one params per output buffer")
        parr = (abi.RenderParams * n)(*plist)
        oarr = (C.c_void_p * n)(*[C.c_void_p(d) for d in d_outs])
        st, ms = (abi.Stats() if stats else None), C.c_double()
        rc = multi_lib().rt_multi_render_frames(self._h, parr, n, stripe_height, oarr,
                                                C.byref(st) if st is not None else None, C.byref(ms))
        if rc != RT_OK:
            raise RtError(f"rt_multi_render_frames: {multi_lib().rt_multi_last_error().decode()}")
        return st, ms.value

    def close(self):
        if self._h:
            multi_lib().rt_multi_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def multi_interleave_frames_host(gathered, height, stripe_height, n):
    """Host restatement of rt_multi's batched assembly: gathered [n, frames, max_rows, W, C] ->
    [frames, H, W, C]."""
    g = np.ascontiguousarray(gathered)
    nf = g.shape[1]
    out = np.empty((nf, height) + g.shape[3:], dtype=g.dtype)
    ptrs = (C.c_void_p * nf)(*[C.c_void_p(out[f].ctypes.data) for f in range(nf)])
    rc = multi_lib().rt_multi_interleave_frames_host(g.ctypes.data_as(C.c_void_p), ptrs, nf, height, g.shape[3],
                                                     g.shape[4], g.itemsize, stripe_height, n)
    if rc != RT_OK:
        raise RtError(f"rt_multi_interleave_frames_host: {multi_lib().rt_multi_last_error().decode()}")
    return out


def multi_interleave_host(gathered, height, stripe_height, n):
    """Host restatement of rt_multi's frame assembly: gathered [n, max_rows, W, C] -> [H, W, C]."""
    g = np.ascontiguousarray(gathered)
    out = np.empty((height,) + g.shape[2:], dtype=g.dtype)
    rc = multi_lib().rt_multi_interleave_host(g.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p), height,
                                              g.shape[2], g.shape[3], g.itemsize, stripe_height, n)
    if rc != RT_OK:
        raise RtError(f"rt_multi_interleave_host: {multi_lib().rt_multi_last_error().decode()}")
    return out


class Raytracer:
    """Mirror of the reference's Raytracer host flow on the MI355X path."""

    def __init__(self, scene="office", device=0, **gen):
        if str(scene).endswith(".sce") or os.path.sep in str(scene):
            self.host = HostScene.load(scene)
        else:
            self.host = HostScene.generate(scene, **gen)
        self.build_seconds = self.host.prepare()
        self.gpu = DeviceScene(self.host, device)

    def compute_image(self, width=0, height=0, spp_n=1, out_format=RT_OUT_RGB_F32):
        p = self.host.render_params(width, height, spp_n)
        p.out_format = out_format
        return self.gpu.render(p)
