import sys, time, numpy as np
sys.path.insert(0, 'my-raytracer_amd'); sys.path.insert(0, 'oracle')
import rtamd, pyoracle
for kind, kw, W, H in [("cornell", {}, 160, 120), ("office", {}, 192, 108), ("random_tris", {"n_triangles": 20000}, 160, 90)]:
    host = rtamd.HostScene.generate(kind, **kw); host.prepare()
    gpu = rtamd.DeviceScene(host, 0)
    p = host.render_params(W, H, 1); p.out_format = rtamd.RT_OUT_RGB_F64
    img, st = gpu.render(p)
    orc = pyoracle.Oracle(host.raw, host)
    ref, cnt = orc.render(p, pyoracle.MODE_REFERENCE)
    d = np.abs(img - ref)
    print(kind, "maxdiff", d.max(), "bad px", int((d.max(-1) > 1e-9).sum()), "gpu", st.as_dict(), "cpu", {k: v for k, v in cnt.as_dict().items() if k in ("primary_rays","shadow_rays","reflection_rays")}, flush=True)
    p.flags = rtamd.RT_FLAG_TRAVERSAL_STATS
    img2, st2 = gpu.render(p)
    _, cnt2 = orc.render(p, pyoracle.MODE_ORDERED)
    print("   stats gpu", st2.node_visits, st2.tri_tests, st2.closest_hits, " oracle", cnt2.node_visits, cnt2.tri_tests, cnt2.closest_hits, flush=True)
# timing office 1080p
host = rtamd.HostScene.generate("office"); host.prepare(); gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(1920, 1080, 1)
for i in range(3):
    img, st = gpu.render(p); ms = gpu.last_kernel_ms()
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    print("office 1080p kernel ms", round(ms, 3), "rays", rays, "Mrays/s", round(rays / ms / 1e3, 1), flush=True)
np.save('gpurun_out/office1080.npy', img.astype(np.float32))
