"""Known-answer scenes shared by the CPU and GPU tests (written as .sce/.obj
and loaded through the product loader, rt_host_load)."""
import minirt

FLAT_MAT = ((0.1, 0.1, 0.1), (0.7, 0.6, 0.5), (0.3, 0.3, 0.3), 20.0, 0.0, 1)
MIRROR_MAT = ((0.05, 0.05, 0.05), (0.2, 0.3, 0.2), (0.5, 0.5, 0.5), 40.0, 0.6, 1)
NOSHADOW_MAT = ((0.2, 0.1, 0.1), (0.8, 0.2, 0.2), (0.1, 0.1, 0.1), 10.0, 0.0, 0)


def quad(x0, x1, y0, y1, z):
    return [(x0, y0, z), (x1, y0, z), (x1, y1, z), (x0, y1, z)], [(0, 1, 2), (0, 2, 3)]


def scenes():
    """name -> (meshes, lights, cam_def, background, ambience, max_depth)."""
    cam = ((0.013, 0.021, 4.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 40.0, 9, 7)
    out = {}
    # single triangle facing the camera, one light
    out["one_tri"] = ([minirt.Mesh([(-1.1, -0.9, 0.0), (1.2, -1.0, 0.0), (0.05, 1.1, 0.0)], [(0, 1, 2)], "FLAT", FLAT_MAT)],
                      [((0.5, 0.7, 3.0), (0.9, 0.9, 0.9))], cam, (0.1, 0.2, 0.3), (0.2, 0.2, 0.2), 2)
    # occluder casting a shadow onto a back wall, 2 lights, one material not shadowable
    wv, wt = quad(-2.0, 2.1, -1.9, 2.2, -0.5)
    ov, ot = quad(-0.45, 0.4, -0.35, 0.5, 0.6)
    out["shadow"] = ([minirt.Mesh(wv, wt, "FLAT", FLAT_MAT), minirt.Mesh(ov, ot, "FLAT", NOSHADOW_MAT)],
                     [((0.1, 0.2, 3.5), (0.7, 0.7, 0.7)), ((-1.5, 1.0, 2.0), (0.3, 0.3, 0.4))], cam,
                     (0.0, 0.0, 0.0), (0.2, 0.2, 0.2), 2)
    # tilted mirror reflecting a coloured quad, depth 3
    mv = [(-1.5, -1.2, -0.8), (1.6, -1.1, -0.5), (1.5, 1.3, -1.2), (-1.4, 1.2, -1.4)]
    tv, tt = quad(-0.7, 0.8, -0.6, 0.9, 1.5)
    out["mirror"] = ([minirt.Mesh(mv, [(0, 1, 2), (0, 2, 3)], "FLAT", MIRROR_MAT),
                      minirt.Mesh(tv, [(0, 2, 1), (0, 3, 2)], "FLAT", FLAT_MAT)],
                     [((0.3, 2.0, 3.0), (0.8, 0.8, 0.8))], cam, (0.05, 0.1, 0.2), (0.2, 0.2, 0.2), 3)
    # PHONG-shaded bent strip (shared vertices => interpolated normals)
    pv = [(-1.2, -1.0, 0.0), (-1.2, 1.0, 0.0), (0.0, -1.0, 0.35), (0.0, 1.0, 0.35), (1.25, -1.0, 0.05), (1.25, 1.0, 0.05)]
    pt = [(0, 2, 3), (0, 3, 1), (2, 4, 5), (2, 5, 3)]
    out["phong"] = ([minirt.Mesh(pv, pt, "PHONG", FLAT_MAT)], [((0.6, 0.8, 3.0), (0.9, 0.85, 0.8))], cam,
                    (0.0, 0.0, 0.0), (0.25, 0.25, 0.25), 1)
    # 40 lights around an occluder over a mirror: more lights than the inline table
    # (RT_MAX_LIGHTS = 16, so they travel through lights_ext) and more than one shadow batch
    # per bounce (1 + 31 lights), with occlusion bits on both sides of the batch boundary
    many = [((1.8 * ((i * 37) % 19 - 9) / 9.0, 0.4 + 0.05 * (i % 7), 1.2 + 0.06 * i),
             (0.02 + 0.001 * (i % 11), 0.025, 0.03 - 0.0005 * (i % 5))) for i in range(40)]
    out["many_lights"] = ([minirt.Mesh(mv, [(0, 1, 2), (0, 2, 3)], "FLAT", MIRROR_MAT),
                           minirt.Mesh(ov, ot, "FLAT", FLAT_MAT)],
                          many, cam, (0.05, 0.1, 0.2), (0.2, 0.2, 0.2), 2)
    return out


def write(tmpdir, name):
    meshes, lights, cam_def, bg, amb, depth = scenes()[name]
    path = tmpdir / f"{name}.sce"
    minirt.write_sce(path, meshes, lights, cam_def, bg, amb, depth)
    return path


def mini(name):
    meshes, lights, cam_def, bg, amb, depth = scenes()[name]
    eye, center, up, fovy, w, h = cam_def
    return minirt.Scene(meshes, lights, minirt.camera(eye, center, up, fovy, w, h), bg, amb, depth)
