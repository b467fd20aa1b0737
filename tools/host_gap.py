"""Host time between back-to-back headline traces (the bench's step loop):
run with LPC_HOSTPROF=1 so the library prints, per trace, the caller's time
since the last trace ("trace enter"), each iteration's launch/wait and the
trace's own tail ("trace leave"); this script adds the Python side of a step.

    LPC_HOSTPROF=1 python tools/host_gap.py [steps] 2> host.log
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bench import rays_of  # noqa: E402
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.distributed import ShardedTrace  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sc = scenes.synthetic(n=1_000_000, seed=7)
eng = Engine(0)
eng.upload_meshes(sc.meshes)
o, d, p = rays_of(sc)
eng.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
in_pow = float(np.sum(p, dtype=np.float64))
runner = ShardedTrace(eng, None)
for _ in range(5):
    eng.reset()
    runner.run(sc.iterations, sc.tau, in_pow, wait=False, input_power_global=in_pow)
eng.sync()
py = []
t_prev = time.perf_counter()
for _ in range(steps):
    t0 = time.perf_counter()
    eng.reset()
    r = runner.run(sc.iterations, sc.tau, in_pow, wait=False, input_power_global=in_pow)
    t1 = time.perf_counter()
    py.append((t0 - t_prev, t1 - t0))
    t_prev = t1
eng.sync()
step_us = [1e6 * (a + b) for a, b in py[1:]]
print(f"steps {steps}  mean step {np.mean(step_us):.1f} us  "
      f"python between steps {1e6 * np.mean([a for a, _ in py[1:]]):.1f} us", flush=True)
