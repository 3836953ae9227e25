"""The C-ABI libraries load on CPU and export every symbol include/*.h declares;
the ctypes mirror (rtamd/abi.py) matches the C struct layouts."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

import rtamd
from rtamd import abi

ROOT = Path(__file__).resolve().parents[1]


def declared(header):
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"static inline[^{]*\{.*?\n\}", "", text, flags=re.S)   # header-only helpers
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.split()}


@pytest.mark.parametrize("header,lib", [("rt_hip.h", rtamd.HIP_LIB), ("rt_host.h", rtamd.HOST_LIB),
                                        ("rt_multi.h", rtamd.MULTI_LIB)])
def test_every_declared_symbol_exported(header, lib):
    syms = declared(header)
    assert syms, header
    missing = [s for s in syms if s not in exported(lib)]
    assert not missing, missing


def test_ctypes_tables_cover_headers():
    assert set(declared("rt_hip.h")) == set(abi.HIP_SYMBOLS)
    assert set(declared("rt_host.h")) == set(abi.HOST_SYMBOLS)
    assert set(declared("rt_multi.h")) == set(abi.MULTI_SYMBOLS)
    rtamd.multi_lib()   # loads (and binds every symbol) without a GPU


def test_libraries_load_and_report():
    assert b"gfx950" in rtamd.hip_lib().rt_build_info()
    assert rtamd.host_lib().rt_host_last_error() is not None


def test_struct_layouts_match_c(tmp_path):
    structs = {"rt_material": abi.Material, "rt_texture": abi.Texture, "rt_mesh": abi.Mesh,
               "rt_sphere": abi.Sphere, "rt_plane": abi.Plane, "rt_light": abi.Light,
               "rt_camera_def": abi.CameraDef, "rt_camera": abi.Camera, "rt_raw_scene": abi.RawScene,
               "rt_scene_soa": abi.SceneSoA, "rt_bvh_soa": abi.BvhSoA, "rt_render_params": abi.RenderParams,
               "rt_stats": abi.Stats, "rt_gen_params": abi.GenParams, "rt_upload_options": abi.UploadOptions}
    src = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{ROOT}/include/rt_host.h"',
           f'#include "{ROOT}/include/rt_hip.h"', "int main(void){"]
    for name in structs:
        src.append(f'printf("{name} %zu\\n", sizeof({name}));')
    src.append('printf("params.out_format %zu\\n", offsetof(rt_render_params, out_format));')
    src.append('printf("soa.mat_shadowable %zu\\n", offsetof(rt_scene_soa, mat_shadowable));')
    src.append('printf("params.lights_ext %zu\\n", offsetof(rt_render_params, lights_ext));')
    src.append('printf("opt.sbvh_alpha %zu\\n", offsetof(rt_upload_options, sbvh_alpha));')
    src.append('printf("opt.collapse_c_tri %zu\\n", offsetof(rt_upload_options, collapse_c_tri));')
    src.append("return 0;}")
    (tmp_path / "sizes.c").write_text("\n".join(src))
    subprocess.run(["gcc", "-o", str(tmp_path / "sizes"), str(tmp_path / "sizes.c")], check=True)
    out = subprocess.run([str(tmp_path / "sizes")], capture_output=True, text=True, check=True).stdout
    got = dict(line.split() for line in out.splitlines())
    for name, cls in structs.items():
        assert int(got[name]) == C.sizeof(cls), name
    assert int(got["params.out_format"]) == abi.RenderParams.out_format.offset
    assert int(got["soa.mat_shadowable"]) == abi.SceneSoA.mat_shadowable.offset
    assert int(got["params.lights_ext"]) == abi.RenderParams.lights_ext.offset
    assert int(got["opt.sbvh_alpha"]) == abi.UploadOptions.sbvh_alpha.offset
    assert int(got["opt.collapse_c_tri"]) == abi.UploadOptions.collapse_c_tri.offset


def test_upload_options_defaults_and_validation():
    # The library reads no environment: every build / layout choice is an rt_upload_options field.
    o = abi.UploadOptions()
    rtamd.hip_lib().rt_upload_options_init(C.byref(o))
    assert (o.device_tree, o.stack_ring, o.lds_treelet, o.collapse) == (abi.RT_TREE_SBVH, 0, 0, abi.RT_COLLAPSE_SAH)
    assert (o.sbvh_leaf_max, o.sbvh_bins, o.blocks_per_cu, o.grid_spare, o.verbose) == (0, 32, 0, 0, 0)
    assert (o.sbvh_alpha, o.sbvh_budget, o.sbvh_c_trav, o.collapse_c_tri) == (-1.0, -1.0, 1.0, 1.0)
    assert (o.reserve_cus, o.order_window) == (0, 0)
    hs = rtamd.HostScene.generate("cornell")
    hs.prepare()
    lib = rtamd.hip_lib()
    for field, bad in (("stack_ring", 12), ("blocks_per_cu", -1), ("sbvh_bins", 1), ("sbvh_leaf_max", 9), ("sbvh_leaf_max", -1),
                       ("device_tree", 7), ("collapse", 3), ("sbvh_alpha", float("nan")), ("sbvh_budget", float("nan")),
                       ("lds_treelet", -2), ("sbvh_c_trav", -1.0), ("order_window", -2), ("order_window", 65)):
        q = rtamd.upload_options(**{field: bad})
        rc = lib.rt_scene_upload_ex(hs.soa, hs.bvh, 0, C.byref(q), C.byref(C.c_void_p()))
        assert rc == abi.RT_ERR_INVALID, (field, rc)
        assert lib.rt_last_error(), field
    with pytest.raises(ValueError):
        rtamd.upload_options(no_such_field=1)


def test_hip_entry_points_reject_bad_arguments():
    lib = rtamd.hip_lib()
    assert lib.rt_scene_upload(None, None, 0, C.byref(C.c_void_p())) == abi.RT_ERR_INVALID
    assert b"null" in lib.rt_last_error()
    assert lib.rt_launch_compute_image(None, None, None, None, None) == abi.RT_ERR_INVALID
    p = abi.RenderParams()
    p.camera.height = 100
    p.stripe_height, p.stripe_count, p.stripe_index = 16, 3, 1
    assert lib.rt_rows_in_shard(C.byref(p)) == len(rtamd.shard_rows(100, 16, 3, 1))


def test_tile_shape_and_ipc_argument_checks():
    # no GPU needed: the work tile is a compile-time shape (8 x 8: one wave's 64 pixels), and the
    # IPC entry points reject null arguments before any HIP call
    assert rtamd.tile_shape() == (8, 8)
    lib = rtamd.hip_lib()
    assert lib.rt_tile_shape(None, None) == abi.RT_ERR_INVALID
    off = C.c_ulonglong(0)
    assert lib.rt_ipc_get_handle(None, None, C.byref(off)) == abi.RT_ERR_INVALID
    assert lib.rt_ipc_open(None, 0, 0, -1, None) == abi.RT_ERR_INVALID
    assert lib.rt_ipc_close(None, 0) == abi.RT_ERR_INVALID
    with pytest.raises(ValueError):
        rtamd.ipc_open(b"short", 0, 0)


def test_multi_set_assembly_rejects_bad_arguments():
    lib = rtamd.multi_lib()
    assert lib.rt_multi_set_assembly(None, abi.RT_MULTI_PEER) == abi.RT_ERR_INVALID


def test_shard_rows_partition_the_image():
    for h, sh, n in [(1080, 16, 8), (1080, 16, 3), (17, 4, 2), (5, 16, 8)]:
        rows = sorted(sum((list(rtamd.shard_rows(h, sh, n, r)) for r in range(n)), []))
        assert rows == list(range(h))


def test_zero_initialised_upload_options_are_valid():
    # A C caller's zero-initialised rt_upload_options (`= {0}`, or a designated initialiser naming one
    # field) must pass validation: zero sbvh_bins / sbvh_c_trav / collapse_c_tri / lds_treelet mean
    # their defaults.  (No GPU here: the upload then fails at the HIP step, never as RT_ERR_INVALID.)
    hs = rtamd.HostScene.generate("cornell")
    hs.prepare()
    lib = rtamd.hip_lib()
    for tree in (abi.RT_TREE_SAH, abi.RT_TREE_SBVH, abi.RT_TREE_REFERENCE):
        z = abi.UploadOptions()
        z.device_tree = tree
        h = C.c_void_p()
        rc = lib.rt_scene_upload_ex(hs.soa, hs.bvh, 0, C.byref(z), C.byref(h))
        assert rc != abi.RT_ERR_INVALID, lib.rt_last_error()
        if rc == abi.RT_OK:
            lib.rt_scene_free(h)
