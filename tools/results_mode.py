"""GPU box: the drop-in's default results mode end to end, as the reference's
examples time it (example_directivity_parabolic_mirror.py:88-102: time() around
CL_Tracer.iterative_tracer, ray-bounces = sum of the results tuples' lengths),
with a per-phase breakdown of every call (the caller keeps the previous call's
results alive, as a script that compares or stores them does).

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
from lightpycl_amd.pinned import POOL  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "parabolic"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
sc = scenes.BUILDERS[name](n=n, seed=7, iterations=4 if name == "parabolic" else 8)
if os.environ.get("RM_GC") == "0":
    import gc
    gc.disable()
tr = CL_Tracer(device=0)
res = None
for k in range(reps + 1):
    a0 = POOL.allocated
    t = time.perf_counter()
    res = tr.iterative_tracer(sc.sources, sc.meshes, trace_iterations=sc.iterations, max_ray_len=sc.max_ray_len)
    dt = time.perf_counter() - t
    ph = {k2: (round(v * 1e3, 3) if not isinstance(v, list) else [round(x * 1e3, 3) for x in v])
          for k2, v in getattr(tr, "phase_s", {}).items()}
    print(json.dumps(dict(call=k, ms=round(dt * 1e3, 3), pinned_allocs=POOL.allocated - a0,
                          bounces=int(sum(len(r[3]) for r in res)), phases=ph)), flush=True)
