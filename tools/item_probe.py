"""GPU box: per-item records of the work-queue traversal (k_trav) for each
iteration of one synthetic trace: item durations, wait before the walk,
concurrency over time, node visits and exact tests per item.

    python tools/item_probe.py [scene] [rays]
"""
import os
import sys

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
e.reset()
e.prof_enable(True, items=True)
for it in range(3):
    nin = e.population()
    st, _ = e.iterate()
    r = e.prof_items().astype(np.int64)
    if len(r) == 0:
        print("no records"); break
    t_claim = r[:, 4]; t_walk = r[:, 5]; dur = r[:, 0]
    # unwrap 32-bit clock relative to the earliest record
    base = t_claim.min()
    t0 = (t_claim - base) & 0xffffffff
    tw = (t_walk - base) & 0xffffffff
    te = tw + dur
    span = te.max() - t0.min()
    ph = r[:, 7] >> 8
    xcc = r[:, 7] & 0xff
    print(f"{name} it{it} rays {nin} items {len(r)} (root {np.sum(ph == 1)}, handed over {np.sum(ph == 2)}) "
          f"span {span / 100:.1f} us")
    for lab, m in (("root", ph == 1), ("hand", ph == 2)):
        if m.sum() == 0:
            continue
        dd = dur[m] / 100.0
        wt = (tw[m] - t0[m]) / 100.0
        print(f"  {lab}: walk us p50 {np.percentile(dd, 50):.1f} p90 {np.percentile(dd, 90):.1f} "
              f"max {dd.max():.1f} | wait us p50 {np.percentile(wt, 50):.1f} p90 {np.percentile(wt, 90):.1f} "
              f"| nodes p50 {np.percentile(r[m, 1], 50):.0f} mean {r[m, 1].mean():.1f} | exact mean {r[m, 2].mean():.0f}"
              f" | us/node {np.sum(dd) / max(1, r[m, 1].sum()):.3f}")
    # concurrency: items walking at each 1% of the span
    edges = np.linspace(0, span, 21)
    conc = [int(np.sum((tw <= x) & (te > x))) for x in edges[:-1]]
    print("  walking items over time (5% steps):", conc)
    tot_walk = dur.sum() / 100.0
    print(f"  sum walk {tot_walk:.0f} item-us = {tot_walk / max(span / 100.0, 1e-9):.0f} walking on average; "
          f"per XCC items {np.bincount(xcc, minlength=8)[:8].tolist()}")
    if st.n_reflect + st.n_refract == 0:
        break
