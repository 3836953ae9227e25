"""ctypes wrapper of the CPU ORACLE (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker / baseline, never as the
product path.  See oracle/rt_oracle.h for the parity status ("parity
unpinned" against reference outputs; pinned by hand-derived known answers).
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
LIB = ROOT / "_build" / "liboracle.so"
sys.path.insert(0, str(ROOT.parent / "my-raytracer_amd"))
from rtamd import abi  # noqa: E402  (struct layouts shared with the headers)

MODE_REFERENCE = 0
MODE_ORDERED = 1


class Counts(C.Structure):
    _fields_ = [("primary_rays", C.c_longlong), ("shadow_rays", C.c_longlong),
                ("reflection_rays", C.c_longlong), ("node_visits", C.c_longlong),
                ("tri_tests", C.c_longlong), ("closest_hits", C.c_longlong),
                ("pixels", C.c_longlong), ("box_tests", C.c_longlong)]

    def as_dict(self):
        return {name: int(getattr(self, name)) for name, _ in self._fields_}


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(ROOT)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        P = C.POINTER
        L.or_prepare.restype = C.c_void_p
        L.or_prepare.argtypes = [P(abi.RawScene)]
        L.or_free.argtypes = [C.c_void_p]
        L.or_camera.argtypes = [P(abi.CameraDef), C.c_int, C.c_int, P(abi.Camera)]
        L.or_render.restype = C.c_int
        L.or_render.argtypes = [C.c_void_p, P(abi.RenderParams), C.c_int, C.c_int, P(C.c_double), P(Counts)]
        L.or_render_pixels.restype = C.c_int
        L.or_render_pixels.argtypes = [C.c_void_p, P(abi.RenderParams), C.c_int, C.c_int, P(C.c_int),
                                       C.c_longlong, P(C.c_double), P(Counts)]
        L.or_n_triangles.restype = C.c_longlong
        L.or_n_triangles.argtypes = [C.c_void_p]
        L.or_n_nodes.restype = C.c_int
        L.or_n_nodes.argtypes = [C.c_void_p]
        L.or_tree_depth.restype = C.c_int
        L.or_tree_depth.argtypes = [C.c_void_p]
        L.or_export_bvh.argtypes = [C.c_void_p, P(C.c_double), P(C.c_double), P(C.c_int), P(C.c_int),
                                    P(C.c_int), P(C.c_int)]
        L.or_export_normals.argtypes = [C.c_void_p, P(C.c_double), P(C.c_double)]
        L.or_closest_hit.restype = C.c_int
        L.or_closest_hit.argtypes = [C.c_void_p, P(C.c_double), P(C.c_double), C.c_int, P(C.c_double),
                                     P(C.c_int), P(C.c_double), P(C.c_double)]
        L.or_intersect_triangle.restype = C.c_int
        L.or_intersect_triangle.argtypes = [P(C.c_double)] * 5 + [P(C.c_double)] * 4
        L.or_intersect_aabb.restype = C.c_int
        L.or_intersect_aabb.argtypes = [P(C.c_double)] * 4
        L.or_median.restype = C.c_double
        L.or_median.argtypes = [P(C.c_double), C.c_int]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


class Oracle:
    """CPU restatement of the reference renderer over a raw scene (rt_raw_scene*)."""

    def __init__(self, raw_ptr, keepalive=None):
        self._keep = keepalive   # the object owning raw_ptr's memory
        self._raw = raw_ptr
        self._h = lib().or_prepare(raw_ptr)
        if not self._h:
            raise RuntimeError("or_prepare failed")

    def close(self):
        if self._h:
            lib().or_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n_triangles(self):
        return int(lib().or_n_triangles(self._h))

    @property
    def n_nodes(self):
        return int(lib().or_n_nodes(self._h))

    @property
    def depth(self):
        return int(lib().or_tree_depth(self._h))

    def camera(self, width=0, height=0):
        cam = abi.Camera()
        lib().or_camera(C.byref(self._raw.contents.camera), width, height, C.byref(cam))
        return cam

    def bvh(self):
        n, nt = self.n_nodes, self.n_triangles
        out = {"bb_min": np.zeros((n, 3)), "bb_max": np.zeros((n, 3)), "left_child": np.zeros(n, np.int32),
               "first_tri": np.zeros(n, np.int32), "tri_count": np.zeros(n, np.int32),
               "perm": np.zeros(nt, np.int32)}
        lib().or_export_bvh(self._h, _dp(out["bb_min"]), _dp(out["bb_max"]), _ip(out["left_child"]),
                            _ip(out["first_tri"]), _ip(out["tri_count"]), _ip(out["perm"]))
        return out

    def normals(self, n_vertices):
        vn = np.zeros((n_vertices, 3))
        fn = np.zeros((self.n_triangles, 3))
        lib().or_export_normals(self._h, _dp(vn), _dp(fn))
        return vn, fn

    def render(self, params, mode=MODE_REFERENCE, threads=0):
        import rtamd
        rows = rtamd.rows_in_shard(params) if rtamd.HIP_LIB.exists() else _rows(params)
        img = np.zeros((rows, params.camera.width, 3))
        cnt = Counts()
        rc = lib().or_render(self._h, C.byref(params), mode, threads, _dp(img), C.byref(cnt))
        if rc != 0:
            raise RuntimeError("or_render failed")
        return img, cnt

    def render_pixels(self, params, xy, mode=MODE_REFERENCE, threads=0):
        xy = np.ascontiguousarray(xy, dtype=np.int32)
        out = np.zeros((len(xy), 3))
        cnt = Counts()
        rc = lib().or_render_pixels(self._h, C.byref(params), mode, threads, _ip(xy), len(xy), _dp(out),
                                    C.byref(cnt))
        if rc != 0:
            raise RuntimeError("or_render_pixels failed")
        return out, cnt

    def adaptive(self, params, primary, subp=4, threshold=0.02, mode=MODE_REFERENCE, threads=0):
        """adaptive_supersampling_device (mytracer_gpu.cu:162-229) on the CPU: `primary` is the
        fp64 primary image [H, W, 3] of `params` (1 ray per pixel).  Returns (image, Counts of the
        supersampled rays, selection mask)."""
        prim = np.ascontiguousarray(primary, dtype=np.float64)
        H, W = prim.shape[:2]
        sel = adaptive_selection(prim, threshold)
        ys, xs = np.nonzero(sel)
        img = prim.copy()
        cnt = Counts()
        if len(xs):
            q = type(params).from_buffer_copy(params)
            q.spp_n = subp
            vals, cnt = self.render_pixels(q, np.stack([xs, ys], 1), mode, threads)
            img[ys, xs] = vals
        return img, cnt, sel

    def closest_hit(self, o, d, mode=MODE_REFERENCE):
        o = np.ascontiguousarray(o, dtype=np.float64)
        d = np.ascontiguousarray(d, dtype=np.float64)
        t = C.c_double()
        tri = C.c_int()
        p = np.zeros(3)
        n = np.zeros(3)
        hit = lib().or_closest_hit(self._h, _dp(o), _dp(d), mode, C.byref(t), C.byref(tri), _dp(p), _dp(n))
        if not hit:
            return None
        return {"t": t.value, "tri": tri.value, "point": p, "normal": n}


def _rows(params):
    h = params.camera.height
    if params.stripe_count <= 1:
        rb = max(0, params.row_begin)
        re = h if params.row_end <= 0 or params.row_end > h else params.row_end
        return max(0, re - rb)
    y = np.arange(h)
    return int(np.sum((y // max(1, params.stripe_height)) % params.stripe_count == params.stripe_index))


def intersect_triangle(p0, p1, p2, o, d):
    vals = [np.ascontiguousarray(v, dtype=np.float64) for v in (p0, p1, p2, o, d)]
    outs = [C.c_double() for _ in range(4)]
    ok = lib().or_intersect_triangle(*[_dp(v) for v in vals], *[C.byref(x) for x in outs])
    if not ok:
        return None
    return tuple(x.value for x in outs)   # t, alpha, beta, gamma


def intersect_aabb(o, d, bmin, bmax):
    vals = [np.ascontiguousarray(v, dtype=np.float64) for v in (o, d, bmin, bmax)]
    return bool(lib().or_intersect_aabb(*[_dp(v) for v in vals]))


def median(values):
    a = np.ascontiguousarray(values, dtype=np.float64).copy()
    return float(lib().or_median(_dp(a), len(a)))


def adaptive_selection(prim, threshold):
    """Pixels adaptive_supersampling_device re-renders (mytracer_gpu.cu:183-198): interior pixels
    whose squared colour distances to the neighbours (x+1, y+1, x-1, y-1) sum above threshold.
    Same operation order as the reference: normSq = dx*dx + dy*dy + dz*dz, summed left to right."""
    def nsq(a, b):
        d = a - b
        return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]

    H, W = prim.shape[:2]
    sel = np.zeros((H, W), dtype=bool)
    if H < 3 or W < 3:
        return sel
    c = prim[1:-1, 1:-1]
    n = ((nsq(c, prim[1:-1, 2:]) + nsq(c, prim[2:, 1:-1])) + nsq(c, prim[1:-1, :-2])) + nsq(c, prim[:-2, 1:-1])
    sel[1:-1, 1:-1] = n > threshold
    return sel
