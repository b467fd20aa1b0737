"""GPU box: one warm-up trace, then `reps` timed traces of a BASELINE config
scene (inputs resident, as bench.py's configs leg), for kernel traces under
rocprofv3.  Prints per-iteration populations and ray-bounces/s.

    python tools/cfg_trace.py scene rays [depth] [reps]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.distributed import ShardedTrace  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

name = sys.argv[1]
n = int(sys.argv[2])
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 16
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
sc = scenes.BUILDERS[name](n=n, seed=7, iterations=depth)
o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
e = Engine(0)
e.upload_meshes(sc.meshes)
e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
in_pow = float(np.sum(p, dtype=np.float64))
run = ShardedTrace(e)
for _ in range(2):          # two warm-up traces: the second runs with the first's prediction (speculative
    e.reset()               # iterations' allocations happen before the timed traces)
    run.run(depth, sc.tau, in_pow)
e.sync()
t = time.perf_counter()
for _ in range(reps):
    e.reset()
    r = run.run(depth, sc.tau, in_pow, wait=False)
e.sync()
dt = (time.perf_counter() - t) / reps
print(json.dumps(dict(scene=name, rays=n, triangles=int(e.tri_count), iterations=int(r["iterations"]),
                      populations=[int(x) for x in r["global_counts"]], ms_per_trace=dt * 1e3,
                      ray_bounces_per_s=int(r["bounces"]) / dt)), flush=True)
e.close()
