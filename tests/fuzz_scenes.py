"""Seeded random scenes for parity fuzzing, written as .sce/.obj and loaded through the product
loader (rt_host_load), so the CPU oracle, the pure-Python restatement (tests/minirt.py) and the
GPU kernel all see the same bytes.

Each seed draws: a floor quad, 1-4 meshes (random triangle blobs, FLAT or PHONG, and shared-vertex
height-field strips whose PHONG normals interpolate), random materials (mirrors, non-shadowable
materials, shininess 1-120), 1-33 lights (more than RT_MAX_LIGHTS and more than one 32-light shadow
batch on some seeds), reflection depth 0-5, and a camera looking into the cluster."""
import math
import random

import minirt


def _mat(rng):
    ka = tuple(rng.uniform(0.0, 0.3) for _ in range(3))
    kd = tuple(rng.uniform(0.1, 0.9) for _ in range(3))
    ks = tuple(rng.uniform(0.0, 0.8) for _ in range(3))
    shin = rng.choice([1.0, 5.0, 20.0, 64.0, rng.uniform(1.0, 120.0)])
    mirror = rng.uniform(0.1, 0.8) if rng.random() < 0.4 else 0.0
    shadowable = 1 if rng.random() < 0.8 else 0
    return (ka, kd, ks, shin, mirror, shadowable)


def _blob(rng, n):
    """n independent triangles scattered around a random centre."""
    c = [rng.uniform(-1.0, 1.0), rng.uniform(-0.6, 1.0), rng.uniform(-1.0, 1.0)]
    s = rng.uniform(0.25, 0.9)
    verts, tris = [], []
    for i in range(n):
        base = [c[k] + rng.uniform(-s, s) for k in range(3)]
        for _ in range(3):
            verts.append(tuple(base[k] + rng.uniform(-0.45 * s, 0.45 * s) for k in range(3)))
        tris.append((3 * i, 3 * i + 1, 3 * i + 2))
    return verts, tris


def _strip(rng, nx, nz):
    """A bumpy (nx+1) x (nz+1) height field with shared vertices."""
    x0, z0 = rng.uniform(-1.5, 0.0), rng.uniform(-1.5, 0.0)
    dx, dz = rng.uniform(0.2, 0.5), rng.uniform(0.2, 0.5)
    y0, amp = rng.uniform(-0.8, 0.8), rng.uniform(0.05, 0.4)
    ph = rng.uniform(0.0, 2.0 * math.pi)
    verts = [(x0 + i * dx, y0 + amp * math.sin(ph + 1.7 * i + 0.9 * j), z0 + j * dz)
             for j in range(nz + 1) for i in range(nx + 1)]
    tris = []
    for j in range(nz):
        for i in range(nx):
            a = j * (nx + 1) + i
            b, c, d = a + 1, a + nx + 1, a + nx + 2
            tris += [(a, c, b), (b, c, d)]
    return verts, tris


def scene(seed, width=9, height=7):
    """-> (meshes, lights, cam_def, background, ambience, max_depth)."""
    rng = random.Random(seed)
    fy = rng.uniform(-1.4, -0.9)
    floor_v = [(-3.0, fy, -3.0), (3.1, fy, -3.0), (3.0, fy, 3.2), (-3.1, fy, 3.0)]
    meshes = [minirt.Mesh(floor_v, [(0, 2, 1), (0, 3, 2)], "FLAT", _mat(rng))]
    for _ in range(rng.randint(1, 4)):
        if rng.random() < 0.55:
            v, t = _blob(rng, rng.randint(2, 30))
            mode = rng.choice(["FLAT", "PHONG"])
        else:
            v, t = _strip(rng, rng.randint(1, 5), rng.randint(1, 5))
            mode = "PHONG"
        meshes.append(minirt.Mesh(v, t, mode, _mat(rng)))
    n_lights = rng.choice([1, 1, 2, 2, 3, 5, 17, 33])
    scale = 1.0 / math.sqrt(n_lights)
    lights = [((rng.uniform(-3.0, 3.0), rng.uniform(0.5, 4.0), rng.uniform(-2.0, 4.0)),
               tuple(scale * rng.uniform(0.2, 1.0) for _ in range(3))) for _ in range(n_lights)]
    eye = (rng.uniform(-1.0, 1.0), rng.uniform(0.0, 1.5), rng.uniform(3.0, 5.0))
    center = (rng.uniform(-0.3, 0.3), rng.uniform(-0.3, 0.3), rng.uniform(-0.3, 0.3))
    cam = (eye, center, (0.0, 1.0, 0.0), rng.uniform(35.0, 60.0), width, height)
    bg = tuple(rng.uniform(0.0, 0.4) for _ in range(3))
    amb = tuple(rng.uniform(0.0, 0.3) for _ in range(3))
    return meshes, lights, cam, bg, amb, rng.randint(0, 5)


def write(tmpdir, seed, width=9, height=7):
    meshes, lights, cam, bg, amb, depth = scene(seed, width, height)
    path = tmpdir / f"fuzz{seed}.sce"
    minirt.write_sce(path, meshes, lights, cam, bg, amb, depth)
    return path


def mini(seed, width=9, height=7):
    meshes, lights, cam, bg, amb, depth = scene(seed, width, height)
    eye, center, up, fovy, w, h = cam
    return minirt.Scene(meshes, lights, minirt.camera(eye, center, up, fovy, w, h), bg, amb, depth)


def write_analytic(tmpdir, seed, width=64, height=48):
    """The seed's mesh scene plus 1-4 spheres and 0-2 planes (opt-in GPU analytic path): spheres
    cutting through meshes, mirror spheres, a tilted reflective plane."""
    path = write(tmpdir, seed, width, height)
    rng = random.Random(10_000 + seed)
    r = lambda v: " ".join(repr(float(x)) for x in v)  # noqa: E731

    def mat():
        ka, kd, ks, shin, mirror, sh = _mat(rng)
        return f"{r(ka)}  {r(kd)}  {r(ks)}  {float(shin)!r}  {float(mirror)!r}  {int(sh)}"

    lines = [f"sphere {r([rng.uniform(-1.2, 1.2), rng.uniform(-0.8, 1.0), rng.uniform(-1.2, 1.2)])}  "
             f"{rng.uniform(0.15, 0.7)!r}  {mat()}" for _ in range(rng.randint(1, 4))]
    for _ in range(rng.randint(0, 2)):
        n = [rng.uniform(-0.3, 0.3), 1.0, rng.uniform(-0.3, 0.3)] if rng.random() < 0.5 else \
            [rng.uniform(-1, 1), rng.uniform(-0.2, 0.2), -1.0]
        ln = math.sqrt(sum(c * c for c in n))
        n = [c / ln for c in n]
        q = [rng.uniform(-0.5, 0.5), rng.uniform(-1.6, -1.0), rng.uniform(-3.5, -2.0)]
        lines.append(f"plane {r(q)}  {r(n)}  {mat()}")
    with open(path, "a") as f:
        f.write("\n".join(lines) + "\n")
    return path


def write_textured(tmpdir, seed, width=64, height=48):
    """The seed's mesh scene plus a textured height field (OBJ vt coordinates, some outside [0, 1]
    so the lookup clamps, mtllib / usemtl / map_Kd to a random P6 texture of odd size)."""
    path = write(tmpdir, seed, width, height)
    rng = random.Random(20_000 + seed)
    r = lambda v: " ".join(repr(float(x)) for x in v)  # noqa: E731
    nx, nz = rng.randint(1, 5), rng.randint(1, 5)
    verts, tris = _strip(rng, nx, nz)
    uv = [(rng.uniform(-0.2, 1.2), rng.uniform(-0.2, 1.2)) for _ in verts]
    tw, th = rng.randint(1, 40), rng.randint(1, 30)
    tex = bytes(rng.randrange(256) for _ in range(tw * th * 3))
    (tmpdir / f"fuzz{seed}_tex.ppm").write_bytes(f"P6\n{tw} {th}\n255\n".encode() + tex)
    (tmpdir / f"fuzz{seed}_tex.mtl").write_text(f"newmtl tex\nKd 1 1 1\nmap_Kd fuzz{seed}_tex.ppm\n")
    obj = tmpdir / f"fuzz{seed}_tex.obj"
    lines = [f"mtllib fuzz{seed}_tex.mtl"] + [f"v {r(v)}" for v in verts] + [f"vt {r(t)}" for t in uv]
    lines += ["usemtl tex"] + ["f " + " ".join(f"{k + 1}/{k + 1}" for k in t) for t in tris]
    obj.write_text("\n".join(lines) + "\n")
    ka, kd, ks, shin, mirror, sh = _mat(rng)
    mode = rng.choice(["FLAT", "PHONG"])
    with open(path, "a") as f:
        f.write(f"mesh {obj.name} {mode} {r(ka)} {r(kd)} {r(ks)} {float(shin)!r} {float(mirror)!r} {int(sh)}\n")
    return path
