"""GPU box: the drop-in's default results mode end to end, as the reference's
examples time it (example_directivity_parabolic_mirror.py:88-102: time() around
CL_Tracer.iterative_tracer, ray-bounces = sum of the results tuples' lengths),
with a per-phase breakdown of the host loop.

    python tools/results_mode.py [scene] [rays] [reps]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.iterative_tracer import CL_Tracer  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "parabolic"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
sc = scenes.BUILDERS[name](n=n, seed=7, iterations=4 if name == "parabolic" else 8)
tr = CL_Tracer(device=0)
tr.iterative_tracer(sc.sources, sc.meshes, trace_iterations=sc.iterations, max_ray_len=sc.max_ray_len)
times = []
for _ in range(reps):
    t = time.perf_counter()
    res = tr.iterative_tracer(sc.sources, sc.meshes, trace_iterations=sc.iterations, max_ray_len=sc.max_ray_len)
    times.append(time.perf_counter() - t)
bounces = sum(len(r[3]) for r in res)
dt = min(times)
print(json.dumps(dict(scene=name, rays=n, iterations=len(res), ray_bounces=bounces, s_per_trace=times,
                      ray_bounces_per_s=bounces / dt, phases={k: (round(v * 1e3, 3) if not isinstance(v, list) else [round(x * 1e3, 3) for x in v])
                              for k, v in getattr(tr, "phase_s", {}).items()},
                      pinned_allocs=__import__("lightpycl_amd.pinned", fromlist=["POOL"]).POOL.allocated,
                      measured_power=float(np.sum(tr.get_measured_rays()[1], dtype=np.float64)))), flush=True)
