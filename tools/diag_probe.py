"""Diagnostic counters of the 4-wide traversal (dev tool): SIMD efficiency and phase cycle shares."""
import sys

sys.path.insert(0, "my-raytracer_amd")
import rtamd  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "office"
w, h, spp = (int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1920, 1080, 1)
kw = {"n_triangles": int(sys.argv[5]) if len(sys.argv) > 5 else 1000000} if kind == "random_tris" else {}
host = rtamd.HostScene.generate(kind, **kw)
host.prepare()
gpu = rtamd.DeviceScene(host, 0)
p = host.render_params(w, h, spp)
for flags, name in [(rtamd.RT_FLAG_WIDE_STATS, "4-wide"), (rtamd.RT_FLAG_TRAVERSAL_STATS, "2-wide")]:
    p.flags = flags
    _, st = gpu.render(p)
    d = gpu.debug_counters()
    rays = st.primary_rays + st.shadow_rays + st.reflection_rays
    tot = d["trav_cycles"] + d["shade_cycles"] + d["fetch_cycles"]
    print(f"{kind} {w}x{h} {name}: rays {rays}  nodes/ray {st.node_visits/rays:.1f} tris/ray {st.tri_tests/rays:.1f}")
    print(f"  node loop: {d['node_iters']} wave-iters, SIMD eff {d['node_lanes']/(64*max(1,d['node_iters'])):.3f}, "
          f"from the LDS treelet {d['node_lds_iters']/max(1,d['node_iters']):.3f}")
    g = max(1, d['node_iters'] - d['node_lds_iters'])
    print(f"  global node iters: {g}, one node for the wave {d['gnode_uniform_iters']/g:.3f}, distinct nodes {d['gnode_distinct']/g:.2f}; "
          f"leaf iters with one record {d['leaf_uniform_iters']/max(1,d['leaf_iters']):.3f}")
    print(f"  leaf loop: {d['leaf_iters']} wave-iters, SIMD eff {d['leaf_lanes']/(64*max(1,d['leaf_iters'])):.3f}")
    print(f"  trav rounds: {d['trav_rounds']}, lanes active {d['trav_round_lanes']/(64*max(1,d['trav_rounds'])):.3f}; outer iters {d['outer_iters']}")
    print(f"  cycles: trav {d['trav_cycles']/tot:.3f} shade {d['shade_cycles']/tot:.3f} fetch {d['fetch_cycles']/tot:.3f} (total wave-cycles {tot:.3e})")
    print(f"  stack spills {d['stack_spills']} ({d['stack_spills']/rays:.3f} per ray)")
    print(f"  per ray: node wave-iters {d['node_iters']*64/rays:.1f}  leaf wave-iters {d['leaf_iters']*64/rays:.1f}")
    it = d['node_iters'] + d['leaf_iters']
    print(f"  trav cycles per wave-iteration {d['trav_cycles']/max(1,it):.0f}; trav rounds {d['trav_rounds']}, "
          f"wave-iters per round {it/max(1,d['trav_rounds']):.1f}; kernel {gpu.last_kernel_ms():.3f} ms")
