"""Quick timing of the production kernel on several workloads (dev tool)."""
import sys
import time

import numpy as np

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

CASES = [("office", {}, 1920, 1080, 1), ("office", {}, 3840, 2160, 4), ("random_tris", {"n_triangles": 1000000}, 1920, 1080, 1)]
if len(sys.argv) > 1 and sys.argv[1] == "quick":
    CASES = CASES[:1]
elif len(sys.argv) > 1 and sys.argv[1] != "all":   # kind:WxH:spp_n[:n_triangles] ...
    CASES = []
    for spec in sys.argv[1:]:
        f = spec.split(":")
        w, h = map(int, f[1].split("x"))
        CASES.append((f[0], {"n_triangles": int(f[3])} if len(f) > 3 else {}, w, h, int(f[2])))
for kind, kw, w, h, spp in CASES:
    t0 = time.time()
    host = rtamd.HostScene.generate(kind, **kw)
    bs = host.prepare()
    gpu = rtamd.DeviceScene(host, 0)
    p = host.render_params(w, h, spp)
    img, st = gpu.render(p)
    ms = []
    for _ in range(5):
        gpu.render(p)
        ms.append(gpu.last_kernel_ms())
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    p.flags = rtamd.RT_FLAG_WIDE_STATS
    _, ws = gpu.render(p)
    dc = gpu.debug_counters()
    spills = dc["stack_spills"]
    diag = (f"  node: simd {dc['node_lanes']/max(1,dc['node_iters']):.1f} lanes, {dc['node_lines']/max(1,dc['node_iters']):.1f} lines"
            f" | leaf: simd {dc['leaf_lanes']/max(1,dc['leaf_iters']):.1f}, {dc['leaf_lines']/max(1,dc['leaf_iters']):.1f} lines"
            f" | big-leaf tests {dc['big_leaf_tests']/max(1,ws.tri_tests):.2f} | iters/ray node {dc['node_iters']*64/rays:.1f} leaf {dc['leaf_iters']*64/rays:.1f}"
            f"\n     cycles: trav {dc['trav_cycles']/max(1,dc['trav_cycles']+dc['shade_cycles']+dc['fetch_cycles']):.2f}"
            f" shade {dc['shade_cycles']/max(1,dc['trav_cycles']+dc['shade_cycles']+dc['fetch_cycles']):.2f}"
            f" fetch {dc['fetch_cycles']/max(1,dc['trav_cycles']+dc['shade_cycles']+dc['fetch_cycles']):.2f}"
            f" | rounds/ray {dc['trav_rounds']*64/rays:.2f} lanes/round {dc['trav_round_lanes']/max(1,dc['trav_rounds']):.1f}")
    p.flags = rtamd.RT_FLAG_TRAVERSAL_STATS
    _, cs = gpu.render(p)
    m = float(np.median(ms))
    print(f"{kind} {w}x{h} spp{spp*spp}: build {bs:.2f}s  kernel {m:.3f} ms  rays {rays}  {rays/m/1e3:.1f} Mrays/s  "
          f"per-ray: wide nodes {ws.node_visits/rays:.1f} tris {ws.tri_tests/rays:.1f} | 2-wide nodes {cs.node_visits/rays:.1f} "
          f"tris {cs.tri_tests/rays:.1f}  spills/ray {spills/rays:.4f}  (total {time.time()-t0:.1f}s)\n   {diag}", flush=True)
