import sys
sys.path.insert(0, "my-raytracer_amd")
import rtamd
for kind, kw in [("office", {}), ("random_tris", {"n_triangles": 1000000})]:
    host = rtamd.HostScene.generate(kind, **kw)
    host.prepare()
    gpu = rtamd.DeviceScene(host, 0)
    p = host.render_params(1920, 1080, 1)
    p.flags = rtamd.RT_FLAG_WIDE_STATS
    _, st = gpu.render(p)
    d = gpu.debug_counters()
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    print(kind, "spills/ray", d["stack_spills"] / rays, "node iters", d["node_iters"], "lds", d["node_lds_iters"], "leaf iters", d["leaf_iters"], flush=True)
