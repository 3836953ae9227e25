"""C++ host side vs the C oracle, bit for bit (CPU only).

The product host (librt_host.so: compute_normals, build_Data, BVH::initSoA
restated in C++) and the oracle (independent C restatement of the AoS build,
mybvh.cpp:44-362) must produce the same tree, node numbering, leaf
permutation, normals and camera.
"""
import numpy as np
import pytest

import pyoracle
import rtamd

SCENES = [("cornell", {}), ("office", {}), ("random_tris", {"n_triangles": 30000, "seed": 99}),
          ("office", {"detail": 2})]


@pytest.fixture(scope="module", params=SCENES, ids=lambda s: f"{s[0]}-{s[1]}")
def pair(request):
    kind, kw = request.param
    hs = rtamd.HostScene.generate(kind, **kw)
    hs.prepare()
    return hs, pyoracle.Oracle(hs.raw, hs)


def test_tree_identical(pair):
    hs, orc = pair
    hb, ob = hs.bvh_arrays(), orc.bvh()
    n = orc.n_nodes
    assert len(hb["left_child"]) == n
    for k in ("bb_min", "bb_max", "left_child", "first_tri", "tri_count"):
        assert np.array_equal(hb[k], ob[k]), k
    assert hs.bvh_depth == orc.depth


def test_leaf_permutation_identical(pair):
    hs, orc = pair
    sa = hs.soa_arrays()
    perm = orc.bvh()["perm"]
    # rebuild the global vertex ids of every triangle in original order from the raw scene
    raw = hs.raw.contents
    tv, base = [], 0
    for m in range(raw.n_meshes):
        mesh = raw.meshes[m]
        t = np.ctypeslib.as_array(mesh.tri_vertex, shape=(3 * mesh.n_triangles,)).reshape(-1, 3) + base
        tv.append(t)
        base += mesh.n_vertices
    tv = np.concatenate(tv)
    assert np.array_equal(sa["vertex_idx"], tv[perm])


def test_normals_identical(pair):
    hs, orc = pair
    sa = hs.soa_arrays()
    vn, fn = orc.normals(len(sa["vertex_pos"]))
    perm = orc.bvh()["perm"]
    assert np.array_equal(vn, sa["vertex_normals"], equal_nan=True)
    assert np.array_equal(fn[perm], sa["face_normals"], equal_nan=True)


def test_camera_identical(pair):
    hs, orc = pair
    for w, h in [(0, 0), (1920, 1080), (37, 23)]:
        assert bytes(hs.camera(w, h)) == bytes(orc.camera(w, h))


def test_every_leaf_small_or_unsplittable(pair):
    # mybvh.cpp:441/453: a node stays a leaf iff it has <= 2 triangles or the
    # median split on axis depth % 3 (root depth 1) leaves one side empty.
    hs, _ = pair
    b = hs.bvh_arrays()
    sa = hs.soa_arrays()
    cent = (sa["vertex_pos"][sa["vertex_idx"][:, 0]] + sa["vertex_pos"][sa["vertex_idx"][:, 1]]
            + sa["vertex_pos"][sa["vertex_idx"][:, 2]]) / 3.0
    depth = np.zeros(len(b["tri_count"]), np.int64)
    depth[0] = 1
    for n in range(len(b["tri_count"])):          # children are numbered after their parent
        if b["tri_count"][n] == 0:
            depth[b["left_child"][n]] = depth[n] + 1
            depth[b["left_child"][n] + 1] = depth[n] + 1
    for node in np.nonzero(b["tri_count"] > 2)[0]:
        f, c = b["first_tri"][node], b["tri_count"][node]
        v = cent[f:f + c, depth[node] % 3]
        s = np.sort(v)
        med = s[c // 2] if c % 2 else 0.5 * (s[c // 2 - 1] + s[c // 2])
        left = int(np.sum(v < med))
        assert left == 0 or left == c, (node, c, left)


def test_save_load_roundtrip(tmp_path):
    hs = rtamd.HostScene.generate("cornell")
    hs.save(tmp_path / "cornell.sce")
    back = rtamd.HostScene.load(tmp_path / "cornell.sce")
    hs.prepare()
    back.prepare()
    for k, v in hs.bvh_arrays().items():
        assert np.array_equal(v, back.bvh_arrays()[k]), k
    a, b = hs.soa_arrays(), back.soa_arrays()
    for k in a:
        assert np.array_equal(a[k], b[k], equal_nan=True), k
    assert bytes(hs.camera()) == bytes(back.camera())
    assert (tmp_path / "cornell_mesh6.ppm").exists()   # textured poster travels as PPM


def test_generators_deterministic():
    a = rtamd.HostScene.generate("random_tris", n_triangles=5000, seed=5)
    b = rtamd.HostScene.generate("random_tris", n_triangles=5000, seed=5)
    c = rtamd.HostScene.generate("random_tris", n_triangles=5000, seed=6)
    a.prepare(), b.prepare(), c.prepare()
    assert np.array_equal(a.soa_arrays()["vertex_pos"], b.soa_arrays()["vertex_pos"])
    assert not np.array_equal(a.soa_arrays()["vertex_pos"], c.soa_arrays()["vertex_pos"])


def test_office_proxy_in_spec():
    hs = rtamd.HostScene.generate("office")
    assert 50000 <= hs.triangle_count <= 100000   # 50k-100k triangles
    p = hs.render_params()
    assert (p.camera.width, p.camera.height, p.max_depth, p.n_lights) == (1920, 1080, 5, 2)
    raw = hs.raw.contents
    mirrors = [raw.meshes[i].material.mirror for i in range(raw.n_meshes)]
    modes = {raw.meshes[i].draw_mode for i in range(raw.n_meshes)}
    assert any(m > 0 for m in mirrors) and modes == {0, 1}


def test_bad_inputs_raise(tmp_path):
    with pytest.raises(rtamd.RtError):
        rtamd.HostScene.generate("no_such_scene")
    with pytest.raises(rtamd.RtError):
        rtamd.HostScene.load(tmp_path / "missing.sce")
    bad = tmp_path / "bad.sce"
    bad.write_text("mesh x.obj WIREFRAME 0 0 0 0 0 0 0 0 0 1 0\n")
    with pytest.raises(rtamd.RtError):
        rtamd.HostScene.load(bad)


def test_parallel_builder_is_bit_identical_to_sequential():
    # The median-split builder splits subtrees on threads and replays the reference's
    # id allocation afterwards (host_scene.cpp build_bvh_soa): same tree, same permutation.
    out = []
    for threads in (1, 8):
        hs = rtamd.HostScene.generate("random_tris", n_triangles=300_000, seed=7)
        hs.prepare(build_threads=threads)
        out.append((hs.bvh_arrays(), hs.soa_arrays(), hs.bvh_depth, hs))
    (b1, s1, d1, _), (b8, s8, d8, _) = out
    assert d1 == d8
    for k in b1:
        assert np.array_equal(b1[k], b8[k]), k
    for k in ("vertex_idx", "face_normals", "texture_idx"):
        assert np.array_equal(s1[k], s8[k]), k
