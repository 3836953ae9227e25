"""Scene / mesh / texture loader fidelity (CPU only).

The course parser (Raytracer::read_scene, Mesh::read_obj, Image) is absent from the
reference; what is visible is the pre-read pass (mytracer.cpp:302-350, 424-500): scene
tokens `mesh <file> <mode>` with the path relative to the scene file, `#` comments, and
OBJ headers v / vt / vn / mtllib / usemtl / f where every `f` line is one triangle.  The
loader (my-raytracer_amd/csrc/host/loader.cpp) accepts that subset and the common OBJ
variants around it; these tests pin its behaviour on hand-made files whose expected
contents are written out here.  Polygons with more than 3 corners are fan-triangulated
(a superset: the reference pre-read would under-allocate for them).
"""
import struct
import zlib

import numpy as np
import pytest

import rtamd

MAT = "0.1 0.1 0.1  0.7 0.6 0.5  0.3 0.3 0.3  20  0.0"


def load_mesh(tmp_path, obj_text, extra_files=(), newline="\n", scene_extra=""):
    (tmp_path / "m.obj").write_bytes(obj_text.replace("\n", newline).encode())
    for name, data in extra_files:
        (tmp_path / name).write_bytes(data if isinstance(data, bytes) else data.encode())
    sce = f"# test scene{newline}camera 0 0 4  0 0 0  0 1 0  40  8 6{newline}light 0 1 3  1 1 1{newline}" \
          f"mesh m.obj FLAT {MAT}{newline}{scene_extra}"
    (tmp_path / "s.sce").write_bytes(sce.encode())
    hs = rtamd.HostScene.load(tmp_path / "s.sce")
    return hs, hs.raw.contents.meshes[0]


def tris(m):
    return np.ctypeslib.as_array(m.tri_vertex, (3 * m.n_triangles,)).reshape(-1, 3).tolist()


def uvs(m):
    if not m.tri_uv:
        return None
    return np.ctypeslib.as_array(m.tri_uv, (3 * m.n_triangles,)).reshape(-1, 3).tolist()


QUADS = "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0.5 1.5 0\nvt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\nvt 0.5 1\n"


@pytest.mark.parametrize("newline", ["\n", "\r\n"])
def test_obj_face_forms_and_fan_triangulation(tmp_path, newline):
    obj = ("# header comment\no thing\ng group\ns off\n" + QUADS + "vn 0 0 1\n"
           "f 1 2 3\n"                  # plain
           "f 1/1 3/3 4/4\n"            # v/vt
           "f 1/1/1 2/2/1 3/3/1\n"      # v/vt/vn
           "f 1//1 3//1 4//1\n"         # v//vn (no uv for this face)
           "f -5/-5 -4/-4 -3/-3 -2/-2\n"  # negative (relative) indices, quad
           "f\t1/1\t2/2\t3/3\t5/5\t4/4\n")  # tabs, pentagon
    hs, m = load_mesh(tmp_path, obj, newline=newline)
    assert m.n_vertices == 5 and m.n_uv == 5
    assert tris(m) == [[0, 1, 2], [0, 2, 3], [0, 1, 2], [0, 2, 3], [0, 1, 2], [0, 2, 3],
                       [0, 1, 2], [0, 2, 4], [0, 4, 3]]
    # faces without uv get uv 0 once any face has uvs
    assert uvs(m) == [[0, 0, 0], [0, 2, 3], [0, 1, 2], [0, 0, 0], [0, 1, 2], [0, 2, 3],
                      [0, 1, 2], [0, 2, 4], [0, 4, 3]]
    pos = np.ctypeslib.as_array(m.positions, (15,)).reshape(5, 3)
    assert np.array_equal(pos[4], [0.5, 1.5, 0.0])


def test_obj_without_uv_faces_has_no_uv_table(tmp_path):
    _, m = load_mesh(tmp_path, QUADS + "f 1 2 3\nf 1 3 4\n")
    assert not m.tri_uv and m.n_triangles == 2


@pytest.mark.parametrize("face", ["f 1 2 9", "f 0 1 2", "f 1/9 2/1 3/1"])
def test_obj_index_out_of_range_raises(tmp_path, face):
    with pytest.raises(rtamd.RtError):
        load_mesh(tmp_path, QUADS + face + "\n")


def test_scene_tokens_and_relative_paths(tmp_path):
    sub = tmp_path / "scenes"
    (sub / "meshes").mkdir(parents=True)
    (sub / "meshes" / "a.obj").write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    (sub / "s.sce").write_text(
        "# comment line\n\n"
        "camera 0 0 4  0 0 0  0 1 0  40  8 6   # trailing comment is ignored\n"
        "depth 4\nbackground 0.1 0.2 0.3\nambience 0.3 0.3 0.3\n"
        "light 0 1 3  1 0.5 0.25\n"
        f"mesh meshes/a.obj PHONG {MAT} 0\n"
        f"sphere 0 0 -1  0.5  {MAT}\n"
        f"plane 0 -1 0  0 1 0  {MAT} 1\n")
    hs = rtamd.HostScene.load(sub / "s.sce")
    r = hs.raw.contents
    assert (r.n_meshes, r.n_spheres, r.n_planes, r.n_lights, r.max_depth) == (1, 1, 1, 1, 4)
    assert list(r.background) == [0.1, 0.2, 0.3]
    assert r.meshes[0].draw_mode == 1   # RT_DRAW_PHONG
    assert r.meshes[0].material.shadowable == 0          # explicit 0
    assert r.spheres[0].material.shadowable == 1         # default
    assert r.camera.width == 8 and r.camera.height == 6 and r.camera.fovy == 40.0


# ---------------- textures: PPM and PNG (every colour type / depth, Adam7) ----------------
def _png_chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xffffffff)


def _filter_rows(rows, bpp):
    """Applies filter type (y % 5) to each packed row (exercises all five filters)."""
    out, prev = b"", bytes(len(rows[0])) if rows else b""
    for y, row in enumerate(rows):
        f = y % 5
        enc = bytearray(len(row))
        for x in range(len(row)):
            a = row[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            if f == 0:
                pred = 0
            elif f == 1:
                pred = a
            elif f == 2:
                pred = b
            elif f == 3:
                pred = (a + b) // 2
            else:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            enc[x] = (row[x] - pred) & 0xff
        out += bytes([f]) + bytes(enc)
        prev = row
    return out


def _pack_row(samples, depth):
    if depth == 8:
        return bytes(samples)
    if depth == 16:
        return b"".join(struct.pack(">H", s) for s in samples)
    bits, out, acc, n = depth, bytearray(), 0, 0
    for s in samples:
        acc = (acc << bits) | s
        n += bits
        if n == 8:
            out.append(acc)
            acc, n = 0, 0
    if n:
        out.append(acc << (8 - n))
    return bytes(out)


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def make_png(samples, ctype, depth, palette=None, interlace=False):
    """samples: int array [H, W, ch] of raw sample values."""
    h, w, ch = samples.shape
    bpp = max(1, ch * depth // 8)
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    data = b""
    for ix, iy, dx, dy in passes:
        sub = samples[iy::dy, ix::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        rows = [_pack_row(sub[y].reshape(-1).tolist(), depth) for y in range(sub.shape[0])]
        data += _filter_rows(rows, bpp)
    png = b"\x89PNG\r\n\x1a\n" + _png_chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0,
                                                                    1 if interlace else 0))
    if palette is not None:
        png += _png_chunk(b"PLTE", bytes(np.asarray(palette, dtype=np.uint8).reshape(-1)))
    half = len(data) // 2
    comp = zlib.compress(data)
    png += _png_chunk(b"IDAT", comp[:len(comp) // 2]) + _png_chunk(b"IDAT", comp[len(comp) // 2:])
    return png + _png_chunk(b"IEND", b"")


def expected_rgb(samples, ctype, depth, palette=None):
    s = samples.astype(np.int64)
    if ctype == 3:
        return np.asarray(palette, dtype=np.uint8)[s[..., 0]]
    if depth == 16:
        s = s >> 8
    elif depth < 8:
        s = s * 255 // ((1 << depth) - 1)
    if ctype in (0, 4):
        return np.repeat(s[..., :1], 3, axis=2).astype(np.uint8)
    return s[..., :3].astype(np.uint8)


TEX_OBJ = ("mtllib m.mtl\n" + QUADS + "usemtl tex\nf 1/1 2/2 3/3\nf 1/1 3/3 4/4\n")


def load_texture(tmp_path, name, data, mtl_line=None):
    mtl = f"newmtl other\nKd 1 1 1\nnewmtl tex\n{mtl_line or 'map_Kd ' + name}\n"
    _, m = load_mesh(tmp_path, TEX_OBJ, extra_files=[("m.mtl", mtl), (name, data)])
    t = m.texture
    return np.ctypeslib.as_array(t.rgb, (t.height, t.width, 3)).copy()


CASES = [(0, 1), (0, 2), (0, 4), (0, 8), (0, 16), (2, 8), (2, 16), (3, 1), (3, 2), (3, 4), (3, 8),
         (4, 8), (4, 16), (6, 8), (6, 16)]


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("ctype,depth", CASES)
def test_png_colour_types_depths_and_interlace(tmp_path, ctype, depth, interlace):
    rng = np.random.default_rng(ctype * 100 + depth)
    h, w = 11, 13                           # odd sizes: partial Adam7 passes and bit-packed row tails
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    palette = None
    if ctype == 3:
        npal = min(1 << depth, 200)
        palette = rng.integers(0, 256, (npal, 3))
        samples = rng.integers(0, npal, (h, w, 1))
    else:
        samples = rng.integers(0, 1 << depth, (h, w, ch))
    png = make_png(samples, ctype, depth, palette, interlace)
    got = load_texture(tmp_path, "t.png", png)
    assert got.shape == (h, w, 3)
    assert np.array_equal(got, expected_rgb(samples, ctype, depth, palette))


@pytest.mark.parametrize("magic", ["P3", "P6"])
def test_ppm_textures_and_map_kd_options(tmp_path, magic):
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, (5, 4, 3), dtype=np.uint8)
    head = f"{magic}\n# a comment\n4 5\n255\n".encode()
    body = img.tobytes() if magic == "P6" else " ".join(str(v) for v in img.reshape(-1)).encode()
    got = load_texture(tmp_path, "t.ppm", head + body, mtl_line="map_Kd -s 1 1 1 -bm 1 t.ppm")
    assert np.array_equal(got, img)


def test_ppm_maxval_rescale_and_bad_texture_raises(tmp_path):
    img = np.array([[[0, 7, 15], [3, 8, 1]]], dtype=np.uint8)
    got = load_texture(tmp_path, "t.ppm", b"P6 2 1 15\n" + img.tobytes())
    assert np.array_equal(got, np.rint(img * 255.0 / 15).astype(np.uint8))
    with pytest.raises(rtamd.RtError):
        load_texture(tmp_path / ".." / tmp_path.name, "bad.png", b"\x89PNG\r\n\x1a\nnot really")
