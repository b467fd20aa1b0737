"""GPU box: A/B sweep of liblpc launch policies (LPC_* environment knobs read at
lpc_open) on one scene.  Every configuration must give the identical trace
(per-iteration ray counts, measured count, per-mesh measured power): the
policies change only speed.

    python tools/sweep.py [scene] [rays] [steps] 'FLAT=0' 'FLAT=5,KEY=3' ...
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.distributed import ShardedTrace  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "synthetic"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
configs = sys.argv[4:] or ["FLAT=0", "KEY=0"]
sc = scenes.BUILDERS[name](n=n, seed=7)
o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
in_pow = float(np.sum(p, dtype=np.float64))
ref = None
for cfg in configs:
    env = dict(kv.split("=") for kv in cfg.split(",") if kv)
    for k in ("KEY", "FLAT", "TARGET_BLOCKS", "SORT", "BUDGET", "SPILL_CAP", "SPILL_BLOCKS", "LOOP"):
        os.environ.pop("LPC_" + k, None)
    for k, v in env.items():
        os.environ["LPC_" + k] = v
    e = Engine(0)
    e.upload_meshes(sc.meshes)
    e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
    run = ShardedTrace(e)
    e.reset()
    r = run.run(sc.iterations, sc.tau, in_pow)
    got = (tuple(r["global_counts"]), e.measured()[0], tuple(np.asarray(r["mesh_power"]).tolist()))
    same = "REF" if ref is None else ("same" if got == ref else "DIFFERENT")
    ref = ref or got
    # per-iteration intersect time (HIP events around the intersect stage)
    e.prof_enable(True)
    e.reset()
    e.prof_read(reset=True)
    its = []
    while True:
        st, _ = e.iterate()
        pr = e.prof_read(reset=True)
        its.append((st.n_in, pr["intersect_ms"], pr["shade_ms"]))
        if len(its) >= len(got[0]):
            break
    e.prof_enable(False)
    ts = []
    for _ in range(steps):
        e.reset()
        t = time.perf_counter()
        run.run(sc.iterations, sc.tau, in_pow)
        ts.append(time.perf_counter() - t)
    bounces = sum(got[0])
    ms = 1e3 * float(np.median(ts))
    print(f"{cfg:28s} {ms:7.3f} ms/step  {bounces / (ms * 1e-3) / 1e6:8.1f} M bounces/s  [{same}] "
          f"isect/it: " + " ".join(f"{a}:{b:.3f}" for a, b, _ in its), flush=True)
    e.close()
