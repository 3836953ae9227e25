"""ctypes mirror of include/rt_scene.h, include/rt_hip.h and include/rt_host.h.

These structs are the plain-C boundary of the MI355X render path; keep them in
lock-step with the headers (tests/test_abi.py checks sizes and symbols).
"""
import ctypes as C

c_double3 = C.c_double * 3

RT_OK = 0
RT_ERR_INVALID = -1
RT_ERR_HIP = -2
RT_ERR_UNSUPPORTED = -3
RT_MAX_LIGHTS = 16
RT_LIGHTS_LIMIT = 1 << 20
RT_MAX_FRAMES = 128
RT_DRAW_FLAT = 0
RT_DRAW_PHONG = 1
RT_OUT_RGB_F32 = 0
RT_OUT_RGB_F64 = 1
RT_FLAG_TRAVERSAL_STATS = 1
RT_FLAG_WIDE_STATS = 2
RT_FLAG_TIMELINE = 4
RT_FLAG_TILE_COST = 8
RT_FLAG_TILE_COST_TIME = 16
RT_FLAG_COST_ORDER = 32
RT_FLAG_NATURAL_ORDER = 64
RT_FLAG_GLOBAL_ROWS = 128
RT_IPC_HANDLE_BYTES = 64
RT_MULTI_GATHER = 0
RT_MULTI_PEER = 1
RT_MULTI_DEBUG_PEER_MISMATCH = 1


class Material(C.Structure):
    _fields_ = [("ambient", c_double3), ("diffuse", c_double3), ("specular", c_double3),
                ("shininess", C.c_double), ("mirror", C.c_double), ("shadowable", C.c_int),
                ("pad_", C.c_int)]


class Texture(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("rgb", C.POINTER(C.c_ubyte))]


class Mesh(C.Structure):
    _fields_ = [("n_vertices", C.c_int), ("positions", C.POINTER(C.c_double)),
                ("n_triangles", C.c_int), ("tri_vertex", C.POINTER(C.c_int)),
                ("n_uv", C.c_int), ("u", C.POINTER(C.c_double)), ("v", C.POINTER(C.c_double)),
                ("tri_uv", C.POINTER(C.c_int)), ("draw_mode", C.c_int), ("pad_", C.c_int),
                ("material", Material), ("texture", Texture)]


class Sphere(C.Structure):
    _fields_ = [("center", c_double3), ("radius", C.c_double), ("material", Material)]


class Plane(C.Structure):
    _fields_ = [("center", c_double3), ("normal", c_double3), ("material", Material)]


class Light(C.Structure):
    _fields_ = [("position", c_double3), ("color", c_double3)]


class CameraDef(C.Structure):
    _fields_ = [("eye", c_double3), ("center", c_double3), ("up", c_double3),
                ("fovy", C.c_double), ("width", C.c_int), ("height", C.c_int)]


class Camera(C.Structure):
    _fields_ = [("eye", c_double3), ("lower_left", c_double3), ("x_dir", c_double3),
                ("y_dir", c_double3), ("width", C.c_int), ("height", C.c_int)]


class RawScene(C.Structure):
    _fields_ = [("camera", CameraDef), ("background", c_double3), ("ambience", c_double3),
                ("max_depth", C.c_int), ("n_lights", C.c_int), ("lights", C.POINTER(Light)),
                ("n_meshes", C.c_int), ("meshes", C.POINTER(Mesh)),
                ("n_spheres", C.c_int), ("spheres", C.POINTER(Sphere)),
                ("n_planes", C.c_int), ("planes", C.POINTER(Plane))]


class SceneSoA(C.Structure):
    _fields_ = [("n_meshes", C.c_int), ("n_vertices", C.c_int), ("n_vertex_idx", C.c_int),
                ("n_tex_coords", C.c_int), ("n_texels", C.c_longlong),
                ("vertex_mesh_id", C.POINTER(C.c_int)), ("vertex_pos", C.POINTER(C.c_double)),
                ("vertex_normals", C.POINTER(C.c_double)), ("face_normals", C.POINTER(C.c_double)),
                ("vertex_idx", C.POINTER(C.c_int)), ("texture_idx", C.POINTER(C.c_int)),
                ("tex_u", C.POINTER(C.c_double)), ("tex_v", C.POINTER(C.c_double)),
                ("texels", C.POINTER(C.c_ubyte)), ("mesh_tex_width", C.POINTER(C.c_int)),
                ("mesh_tex_height", C.POINTER(C.c_int)), ("mesh_tex_offset", C.POINTER(C.c_longlong)),
                ("mesh_draw_mode", C.POINTER(C.c_int)), ("mat_ambient", C.POINTER(C.c_double)),
                ("mat_diffuse", C.POINTER(C.c_double)), ("mat_specular", C.POINTER(C.c_double)),
                ("mat_shininess", C.POINTER(C.c_double)), ("mat_mirror", C.POINTER(C.c_double)),
                ("mat_shadowable", C.POINTER(C.c_int))]


class BvhSoA(C.Structure):
    _fields_ = [("n_nodes", C.c_int), ("bb_min", C.POINTER(C.c_double)),
                ("bb_max", C.POINTER(C.c_double)), ("left_child", C.POINTER(C.c_int)),
                ("first_tri", C.POINTER(C.c_int)), ("tri_count", C.POINTER(C.c_int))]


class RenderParams(C.Structure):
    _fields_ = [("camera", Camera), ("n_lights", C.c_int), ("max_depth", C.c_int),
                ("lights", Light * RT_MAX_LIGHTS), ("background", c_double3),
                ("ambience", c_double3), ("spp_n", C.c_int), ("row_begin", C.c_int),
                ("row_end", C.c_int), ("stripe_height", C.c_int), ("stripe_count", C.c_int),
                ("stripe_index", C.c_int), ("out_format", C.c_int), ("flags", C.c_int),
                ("lights_ext", C.POINTER(Light))]

    def set_lights(self, lights):
        """Sets the light list; more than RT_MAX_LIGHTS go through lights_ext (the array is
        kept alive on this object)."""
        n = len(lights)
        self.n_lights = n
        if n <= RT_MAX_LIGHTS:
            self.lights_ext = None
            arr = self.lights
        else:
            arr = (Light * n)()
            self._lights_keep = arr
            self.lights_ext = C.cast(arr, C.POINTER(Light))
        for i, (pos, col) in enumerate(lights):
            for k in range(3):
                arr[i].position[k] = pos[k]
                arr[i].color[k] = col[k]


class Stats(C.Structure):
    _fields_ = [("primary_rays", C.c_longlong), ("shadow_rays", C.c_longlong),
                ("reflection_rays", C.c_longlong), ("node_visits", C.c_longlong),
                ("tri_tests", C.c_longlong), ("closest_hits", C.c_longlong),
                ("pixels", C.c_longlong), ("reserved_", C.c_longlong)]

    def as_dict(self):
        return {name: int(getattr(self, name)) for name, _ in self._fields_ if name != "reserved_"}


class GenParams(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("n_triangles", C.c_longlong),
                ("seed", C.c_ulonglong), ("max_depth", C.c_int), ("detail", C.c_int)]


class UploadOptions(C.Structure):
    """rt_upload_options (include/rt_hip.h); make one with upload_options(**fields)."""
    _fields_ = [("device_tree", C.c_int), ("build_threads", C.c_int), ("stack_ring", C.c_int),
                ("lds_treelet", C.c_int), ("collapse", C.c_int), ("sbvh_leaf_max", C.c_int),
                ("sbvh_bins", C.c_int), ("blocks_per_cu", C.c_int), ("grid_spare", C.c_int),
                ("verbose", C.c_int), ("sbvh_alpha", C.c_double), ("sbvh_budget", C.c_double),
                ("sbvh_c_trav", C.c_double), ("collapse_c_tri", C.c_double), ("reserve_cus", C.c_int),
                ("order_window", C.c_int), ("spp_lanes", C.c_int),
                ("reserved_", C.c_int * 5)]


RT_TREE_SAH, RT_TREE_REFERENCE, RT_TREE_SBVH = 0, 1, 2
RT_COLLAPSE_GREEDY, RT_COLLAPSE_SAH, RT_COLLAPSE_BY_SIZE = 0, 1, 2

# Symbols each library must export (declared in include/*.h).
HIP_SYMBOLS = {
    "rt_scene_upload": (C.c_int, [C.POINTER(SceneSoA), C.POINTER(BvhSoA), C.c_int, C.POINTER(C.c_void_p)]),
    "rt_upload_options_init": (None, [C.POINTER(UploadOptions)]),
    "rt_scene_upload_ex": (C.c_int, [C.POINTER(SceneSoA), C.POINTER(BvhSoA), C.c_int, C.POINTER(UploadOptions),
                                     C.POINTER(C.c_void_p)]),
    "rt_scene_upload_multi": (C.c_int, [C.POINTER(SceneSoA), C.POINTER(BvhSoA), C.POINTER(C.c_int), C.c_int,
                                        C.POINTER(UploadOptions), C.POINTER(C.c_void_p)]),
    "rt_scene_set_analytic": (C.c_int, [C.c_void_p, C.POINTER(Sphere), C.c_int, C.POINTER(Plane), C.c_int]),
    "rt_scene_device_bytes": (C.c_longlong, [C.c_void_p]),
    "rt_scene_upload_seconds": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "rt_rows_in_shard": (C.c_int, [C.POINTER(RenderParams)]),
    "rt_launch_compute_image": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_void_p,
                                          C.POINTER(Stats), C.c_void_p]),
    "rt_launch_frames": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_int, C.POINTER(C.c_void_p),
                                   C.POINTER(Stats), C.c_void_p]),
    "rt_launch_adaptive": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_void_p, C.c_void_p, C.c_int,
                                     C.c_double, C.POINTER(Stats), C.POINTER(C.c_longlong), C.c_void_p]),
    "rt_launch_adaptive_shard": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_int, C.c_double, C.POINTER(Stats),
                                           C.POINTER(C.c_longlong), C.c_void_p]),
    "rt_launch_adaptive_frames": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_int, C.POINTER(C.c_void_p),
                                            C.POINTER(C.c_void_p), C.c_int, C.c_double, C.POINTER(Stats),
                                            C.POINTER(C.c_longlong), C.c_void_p]),
    "rt_adaptive_halo_rows": (C.c_int, [C.POINTER(RenderParams), C.POINTER(C.c_int), C.c_int]),
    "rt_render_to_host": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_void_p, C.POINTER(Stats)]),
    "rt_render_adaptive_to_host": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_int, C.c_double, C.c_void_p,
                                             C.POINTER(Stats), C.POINTER(Stats), C.POINTER(C.c_longlong)]),
    "rt_last_kernel_ms": (C.c_int, [C.c_void_p, C.POINTER(C.c_float)]),
    "rt_tile_shape": (C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "rt_ipc_get_handle": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_ulonglong)]),
    "rt_ipc_open": (C.c_int, [C.c_char_p, C.c_ulonglong, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "rt_ipc_close": (C.c_int, [C.c_void_p, C.c_ulonglong]),
    "rt_debug_counters": (C.c_int, [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]),
    "rt_debug_wave_log": (C.c_longlong, [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_longlong]),
    "rt_debug_timeline": (C.c_longlong, [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_longlong]),
    "rt_debug_tile_cost": (C.c_longlong, [C.c_void_p, C.POINTER(C.c_uint), C.c_longlong]),
    "rt_debug_set_tile_order": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint), C.c_longlong]),
    "rt_debug_last_tile_order": (C.c_longlong, [C.c_void_p, C.POINTER(C.c_uint), C.c_longlong]),
    "rt_debug_blocks_per_cu": (C.c_int, [C.c_void_p, C.c_int]),
    "rt_debug_last_grid": (C.c_int, [C.c_void_p, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    "rt_debug_corrupt_hierarchy": (C.c_int, [C.c_void_p]),
    "rt_scene_status": (C.c_int, [C.c_void_p]),
    "rt_scene_free": (None, [C.c_void_p]),
    "rt_last_error": (C.c_char_p, []),
    "rt_build_info": (C.c_char_p, []),
}

HOST_SYMBOLS = {
    "rt_host_load": (C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    "rt_host_generate": (C.c_int, [C.c_char_p, C.POINTER(GenParams), C.POINTER(C.c_void_p)]),
    "rt_host_raw": (C.POINTER(RawScene), [C.c_void_p]),
    "rt_host_prepare": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "rt_host_prepare_ex": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_double)]),
    "rt_host_soa": (C.POINTER(SceneSoA), [C.c_void_p]),
    "rt_host_bvh": (C.POINTER(BvhSoA), [C.c_void_p]),
    "rt_host_camera": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(Camera)]),
    "rt_host_render_params": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(RenderParams)]),
    "rt_host_save": (C.c_int, [C.c_void_p, C.c_char_p]),
    "rt_write_ppm": (C.c_int, [C.c_char_p, C.POINTER(C.c_float), C.c_int, C.c_int]),
    "rt_host_triangle_count": (C.c_longlong, [C.c_void_p]),
    "rt_host_bvh_depth": (C.c_int, [C.c_void_p]),
    "rt_host_free": (None, [C.c_void_p]),
    "rt_host_last_error": (C.c_char_p, []),
}


MULTI_SYMBOLS = {
    "rt_multi_create": (C.c_int, [C.POINTER(SceneSoA), C.POINTER(BvhSoA), C.POINTER(C.c_int), C.c_int,
                                  C.POINTER(UploadOptions), C.POINTER(C.c_void_p)]),
    "rt_multi_device_count": (C.c_int, [C.c_void_p]),
    "rt_multi_set_assembly": (C.c_int, [C.c_void_p, C.c_int]),
    "rt_multi_assembly": (C.c_int, [C.c_void_p]),
    "rt_multi_debug_inject": (C.c_int, [C.c_void_p, C.c_int]),
    "rt_multi_render": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_int, C.c_void_p, C.POINTER(Stats),
                                  C.POINTER(C.c_double)]),
    "rt_multi_render_frames": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_int, C.c_int,
                                         C.POINTER(C.c_void_p), C.POINTER(Stats), C.POINTER(C.c_double)]),
    "rt_multi_render_to_host": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_int, C.c_void_p,
                                          C.POINTER(Stats), C.POINTER(C.c_double)]),
    "rt_multi_max_rows": (C.c_int, [C.c_int, C.c_int, C.c_int]),
    "rt_multi_interleave_host": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.c_int]),
    "rt_multi_interleave_frames_host": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int,
                                                  C.c_int, C.c_int, C.c_int, C.c_int]),
    "rt_multi_free": (None, [C.c_void_p]),
    "rt_multi_last_error": (C.c_char_p, []),
}


def bind(lib, table, partial=False):
    for name, (res, args) in table.items():
        if (partial or name.startswith("rt_debug_")) and not hasattr(lib, name):
            continue   # entry points a kernel variant built from an older source lacks (A/B tools)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
