"""Pure-Python mini ray tracer for tiny known-answer scenes (test infrastructure).

A third, independent restatement of the reference CPU renderer's semantics
(mymesh.cpp:176-236 triangle test, mytracer.cpp:510-608 lighting and
subtrace, mytracer_gpu.cu:202-224 samples; Camera/trace/intersect_scene as
fixed in DESIGN.md §2), written with Python floats (IEEE fp64, no FMA) and a
brute-force closest hit over all triangles (no BVH).  Used only on scenes of a
few triangles and images of a few pixels, where it pins both the C oracle and
the HIP kernel.  Scenes must avoid exact t-ties between triangles (brute force
breaks ties by input order, the BVH by leaf order).

Also writes .sce/.obj files so KAT scenes go through the product loader.
"""
import math
from pathlib import Path


def dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def normalize(v):
    n = math.sqrt(dot(v, v))
    return (v[0] / n, v[1] / n, v[2] / n) if n > 0.0 else v


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def det3(v1, v2, v3):
    return (v1[0] * (v2[1] * v3[2] - v3[1] * v2[2]) - v2[0] * (v1[1] * v3[2] - v3[1] * v1[2])
            + v3[0] * (v1[1] * v2[2] - v2[1] * v1[2]))


def intersect_triangle(p0, p1, p2, o, d):
    c1 = sub(p0, p2)
    c2 = sub(p1, p2)
    c3 = (-d[0], -d[1], -d[2])
    c4 = sub(o, p2)
    S = det3(c1, c2, c3)
    if abs(S) < 1e-10:
        return None
    alpha = det3(c4, c2, c3) / S
    beta = det3(c1, c4, c3) / S
    gamma = 1.0 - alpha - beta
    t = det3(c1, c2, c4) / S
    if t <= 1e-5:
        return None
    if not (0.0 <= alpha <= 1.0 and 0.0 <= beta <= 1.0 and 0.0 <= gamma <= 1.0):
        return None
    return t, alpha, beta, gamma


def camera(eye, center, up, fovy, width, height):
    view = sub(center, eye)
    dist = math.sqrt(dot(view, view))
    view = normalize(view)
    ih = 2.0 * dist * math.tan(0.5 * fovy / 180.0 * math.pi)
    iw = width / height * ih
    xd = normalize(cross(view, up))
    xd = tuple(c * iw / width for c in xd)
    yd = normalize(cross(xd, view))
    yd = tuple(c * ih / height for c in yd)
    ll = tuple(center[k] - 0.5 * width * xd[k] - 0.5 * height * yd[k] for k in range(3))
    return {"eye": tuple(eye), "ll": ll, "xd": xd, "yd": yd, "w": width, "h": height}


class Mesh:
    def __init__(self, verts, tris, mode="FLAT", material=None):
        self.verts = [tuple(map(float, v)) for v in verts]
        self.tris = [tuple(t) for t in tris]
        self.mode = mode
        # ambient, diffuse, specular, shininess, mirror, shadowable
        self.mat = material or ((0.1, 0.1, 0.1), (0.7, 0.6, 0.5), (0.3, 0.3, 0.3), 20.0, 0.0, 1)
        self.face_n = [normalize(cross(sub(self.verts[b], self.verts[a]), sub(self.verts[c], self.verts[a])))
                       for a, b, c in self.tris]
        self.vert_n = self._vertex_normals()

    def _vertex_normals(self):   # mymesh.cpp:103-163
        vn = [(0.0, 0.0, 0.0)] * len(self.verts)
        for (i0, i1, i2), n in zip(self.tris, self.face_n):
            p0, p1, p2 = self.verts[i0], self.verts[i1], self.verts[i2]
            v0, v1, v2 = sub(p1, p0), sub(p2, p1), sub(p0, p2)
            l0, l1, l2 = (math.sqrt(dot(v, v)) for v in (v0, v1, v2))
            neg = lambda v: (-v[0], -v[1], -v[2])  # noqa: E731
            w = (l0 * l2 + dot(v0, neg(v2)), l1 * l0 + dot(v1, neg(v0)), l2 * l1 + dot(v2, neg(v1)))
            for i, wi in zip((i0, i1, i2), w):
                if abs(wi) > 1e-12:
                    vn[i] = (vn[i][0] + n[0] / wi, vn[i][1] + n[1] / wi, vn[i][2] + n[2] / wi)
        return [normalize(v) for v in vn]


class Scene:
    def __init__(self, meshes, lights, cam, background=(0.0, 0.0, 0.0), ambience=(0.2, 0.2, 0.2), max_depth=2):
        self.meshes, self.lights, self.cam = meshes, lights, cam
        self.bg, self.amb, self.max_depth = background, ambience, max_depth
        self.counts = {"primary": 0, "shadow": 0, "reflection": 0}

    def closest(self, o, d):
        best = None
        for m in self.meshes:
            for ti, (i0, i1, i2) in enumerate(m.tris):
                r = intersect_triangle(m.verts[i0], m.verts[i1], m.verts[i2], o, d)
                if r is not None and (best is None or r[0] < best[0]):
                    best = (r[0], r[1], r[2], r[3], m, ti)
        return best

    def lighting(self, p, n, view, m, diffuse):
        ka, _, ks, shin, _, shadowable = m.mat
        col = [0.0 + self.amb[k] * ka[k] for k in range(3)]
        for lpos, lcol in self.lights:
            to_l = sub(lpos, p)
            l = normalize(to_l)
            c0 = dot(n, l)
            diff = c0 if 0.0 < c0 else 0.0
            refl = 0.0
            if diff > 0.0:
                s = 2.0 * dot(n, l)
                r = normalize(tuple(s * n[k] - l[k] for k in range(3)))
                c = dot(r, view)
                refl = c if 0.0 < c else 0.0
            refl = math.pow(refl, shin)
            shadow = False
            if shadowable:
                dist = math.sqrt(dot(to_l, to_l))
                o = tuple(p[k] + 1e-4 * l[k] for k in range(3))
                self.counts["shadow"] += 1
                h = self.closest(o, normalize(l))
                shadow = h is not None and h[0] < dist and 0.0 < h[0]
            for k in range(3):
                col[k] += lcol[k] * float(not shadow) * (diffuse[k] * diff + ks[k] * refl)
        return col

    def trace(self, o, d, depth):
        if depth > self.max_depth:
            return [0.0, 0.0, 0.0]
        self.counts["primary" if depth == 0 else "reflection"] += 1
        h = self.closest(o, d)
        if h is None:
            return list(self.bg)
        t, a, b, g, m, ti = h
        p = tuple(o[k] + t * d[k] for k in range(3))
        i0, i1, i2 = m.tris[ti]
        if m.mode == "FLAT":
            n = m.face_n[ti]
        else:
            n = tuple(a * m.vert_n[i0][k] + b * m.vert_n[i1][k] + g * m.vert_n[i2][k] for k in range(3))
        col = self.lighting(p, n, (-d[0], -d[1], -d[2]), m, m.mat[1])
        mirror = m.mat[4]
        refl = [0.0, 0.0, 0.0]
        if mirror > 0.0:
            s = 2.0 * dot(n, d)
            v = tuple(d[k] - s * n[k] for k in range(3))
            sub_c = self.trace(tuple(p[k] + 1e-4 * v[k] for k in range(3)), normalize(v), depth + 1)
            refl = [mirror * c for c in sub_c]
        return [(1.0 - mirror) * col[k] + refl[k] for k in range(3)]

    def render(self, spp_n=1):
        c = self.cam
        img = [[None] * c["w"] for _ in range(c["h"])]
        for y in range(c["h"]):
            for x in range(c["w"]):
                acc = [0.0, 0.0, 0.0]
                for si in range(spp_n):
                    xo = si / spp_n - 0.5 + 1.0 / (2.0 * spp_n)
                    for sj in range(spp_n):
                        yo = sj / spp_n - 0.5 + 1.0 / (2.0 * spp_n)
                        X, Y = x + xo, y + yo
                        d = tuple(c["ll"][k] + X * c["xd"][k] + Y * c["yd"][k] - c["eye"][k] for k in range(3))
                        col = self.trace(c["eye"], normalize(d), 0)
                        acc = [acc[k] + col[k] for k in range(3)]
                img[y][x] = [min(acc[k] / (spp_n * spp_n), 1.0) for k in range(3)]
        return img


def write_sce(path, meshes, lights, cam_def, background=(0, 0, 0), ambience=(0.2, 0.2, 0.2), max_depth=2):
    """cam_def = (eye, center, up, fovy, width, height); writes .sce + one .obj per mesh."""
    path = Path(path)
    eye, center, up, fovy, w, h = cam_def
    r = lambda v: " ".join(repr(float(x)) for x in v)  # noqa: E731
    lines = [f"camera {r(eye)} {r(center)} {r(up)} {float(fovy)!r} {w} {h}", f"depth {max_depth}",
             f"background {r(background)}", f"ambience {r(ambience)}"]
    for lp, lc in lights:
        lines.append(f"light {r(lp)} {r(lc)}")
    for i, m in enumerate(meshes):
        obj = path.with_name(f"{path.stem}_m{i}.obj")
        with open(obj, "w") as f:
            for v in m.verts:
                f.write(f"v {r(v)}\n")
            for t in m.tris:
                f.write("f " + " ".join(str(k + 1) for k in t) + "\n")
        ka, kd, ks, shin, mirror, sh = m.mat
        lines.append(f"mesh {obj.name} {m.mode} {r(ka)} {r(kd)} {r(ks)} {float(shin)!r} {float(mirror)!r} {int(sh)}")
    path.write_text("\n".join(lines) + "\n")
