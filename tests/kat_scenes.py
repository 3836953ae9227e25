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


# ---- inputs where the reference CPU renderer and a brute-force renderer differ ----
# The reference's fp64 slab test (BVH::intersectAABB, mybvh.cpp:99-135) is not conservative, so a
# ray that meets a triangle exactly on the boundary of its leaf box can lose the hit that the
# triangle test (Mesh::intersect_triangle, mymesh.cpp:190-215, inclusive barycentrics) accepts.  The
# kernel's boxes are conservative (outward-rounded fp32, grown by delta), so it keeps the hit, as
# tests/minirt.py (no boxes at all) does.  Each case lists exactly the (row, col) pixels where the
# reference differs; everywhere else all three agree.
AXIS_CAM = ((0.0, 0.0, 4.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 50.0, 64, 48)
AXIS_LIGHTS = [((0.0, 2.5, 0.0), (0.7, 0.7, 0.7)), ((0.0, 0.0, 3.0), (0.3, 0.3, 0.3))]


def divergence_scenes():
    """name -> (meshes, lights, cam_def, background, ambience, max_depth, spp_n,
    expected divergent pixels [(row, col)], expected (shadow, reflection) ray-count difference
    minirt - reference)."""
    floor_v = [(-3.0, -1.0, 3.0), (3.0, -1.0, 3.0), (3.0, -1.0, -3.0), (-3.0, -1.0, -3.0)]   # y = -1
    floor_t = [(0, 1, 2), (0, 2, 3)]
    wall_v, wall_t = quad(-3.0, 3.0, -1.0, 3.0, -2.0)
    box_v = [(-0.5, -1.0, 0.0), (0.5, -1.0, 0.0), (0.5, 0.1, 0.0), (-0.5, 0.1, 0.0)]
    out = {}
    # 1. edge-exact hit: at round extents one 2x2-spp sample ray of the 64x48 image meets the floor
    #    exactly on its edge x = -3 (a face of the floor's leaf box); the reference's slabs round the
    #    box out by an ulp and reject it, the triangle test accepts the edge point
    out["edge_exact"] = ([minirt.Mesh(floor_v, floor_t, "FLAT", FLAT_MAT),
                          minirt.Mesh(wall_v, wall_t, "FLAT", MIRROR_MAT),
                          minirt.Mesh(box_v, [(0, 1, 2), (0, 2, 3)], "FLAT", FLAT_MAT)],
                         AXIS_LIGHTS, AXIS_CAM, (0.05, 0.1, 0.2), (0.2, 0.2, 0.2), 3, 2, [(14, 3)], (2, 0))
    # 2. NaN max plane: a panel x in [-1, 0] alone; the centre column's primary rays have d.x == 0
    #    exactly and o.x == 0 == the leaf box's max x, where the reference's slab computes
    #    (0 - 0) / 0 = NaN and std::min carries it into tmax (the min-plane side keeps it out):
    #    the box is rejected, the panel's edge x = 0 is missed
    pan_v, pan_t = quad(-1.0, 0.0, -0.5, 0.5, 1.0)
    out["nan_max_plane"] = ([minirt.Mesh(pan_v, pan_t, "FLAT", FLAT_MAT)], AXIS_LIGHTS, AXIS_CAM,
                            (0.05, 0.1, 0.2), (0.2, 0.2, 0.2), 3, 1, [(r, 32) for r in range(16, 33)], (34, 0))
    return out


def write_divergence(tmpdir, name):
    meshes, lights, cam_def, bg, amb, depth = divergence_scenes()[name][:6]
    path = tmpdir / f"{name}.sce"
    minirt.write_sce(path, meshes, lights, cam_def, bg, amb, depth)
    return path


def mini_divergence(name):
    meshes, lights, cam_def, bg, amb, depth = divergence_scenes()[name][:6]
    eye, center, up, fovy, w, h = cam_def
    return minirt.Scene(meshes, lights, minirt.camera(eye, center, up, fovy, w, h), bg, amb, depth)
