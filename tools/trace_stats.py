"""GPU box: traversal statistics of the walk (k_rootwalk / k_spill) per bench iteration (diagnostic)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "synthetic"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
sc = scenes.BUILDERS[name](n=n, seed=7)
e = Engine(0)
e.upload_meshes(sc.meshes)
o = np.asarray(sc.sources[0].rays_origin, np.float32)
d = np.asarray(sc.sources[0].rays_dir, np.float32)
p = np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1)
e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
thr = (1.0 - sc.tau) * float(np.sum(p, dtype=np.float64))
for counters in (False, True):
    e.reset()
    e.prof_enable(True, counters=counters)
    e.prof_read(reset=True)
    for it in range(sc.iterations):
        nin = e.population()
        t = time.perf_counter()
        st, _ = e.iterate()
        dt = time.perf_counter() - t
        pr = e.prof_read(reset=True)
        waves = max(pr["wave_traversals"], 1)
        print(f"{name} it{it} rays {nin:8d} wall {dt*1e3:7.3f} ms  isect {pr['intersect_ms']:7.3f} ms "
              f"rest {pr['shade_ms']:6.3f} ms  nodes/traversal {pr['node_visits']/max(pr['wave_traversals'],1):7.1f} "
              f"sliver tests/packet {pr['group_tests']/max(nin/128,1):7.1f} exact/ray {pr['exact_tests']/max(nin,1):6.2f} "
              f"waves {pr['wave_traversals']}", flush=True)
        if counters:
            h = pr["wave_hist"]
            nz = [(b, c) for b, c in enumerate(h) if c]
            print("    wave time histogram (us >= : waves): " +
                  ", ".join(f"{(1 << b) / 100:.2f}: {c}" for b, c in nz) +
                  f"  | heaviest piece {pr['heavy_piece']} = "
                  f"{100.0 * pr['heavy_piece_ticks'] / max(pr['piece_ticks'], 1):.1f}% of wave time", flush=True)
            wc = max(pr["walk_cycles"], 1)
            print(f"    walk items: {pr['walk_cycles'] / waves:.0f} shader cycles each, "
                  f"{100.0 * pr['drain_cycles'] / wc:.1f}% in exact-test drains; "
                  f"{(pr['walk_cycles'] - pr['drain_cycles']) / max(pr['node_visits'], 1):.0f} cycles per node visit "
                  f"outside drains, {pr['drain_cycles'] / max(pr['exact_tests'], 1):.1f} drain cycles per exact test; "
                  f"{100.0 * pr['fan_exact'] / max(pr['exact_tests'], 1):.1f}% of exact tests on fan triangles "
                  f"({pr['fan_exact'] / max(nin, 1):.1f} per ray); {100.0 * pr['behind_exact'] / max(pr['exact_tests'], 1):.1f}% "
                  f"wholly behind the origin, {100.0 * pr['hit_exact'] / max(pr['exact_tests'], 1):.1f}% accepted", flush=True)
            tw = max(pr["tail_waves"], 1)
            print(f"    tail waves {pr['tail_waves']}: nodes/wave {pr['tail_nodes']/tw:.0f} "
                  f"spread {pr['tail_spread_urad']/tw/1e6:.4f} rad exact/wave {pr['tail_exact']/tw:.0f}; "
                  f"all waves: nodes/wave {pr['node_visits']/max(pr['wave_traversals'],1):.1f}", flush=True)
        if st.n_reflect + st.n_refract == 0 or st.power_next < thr:   # iterative_tracer.py:383-391
            break
    print("counters" if counters else "timing only")
