"""GPU box: A/B sweep of liblpc launch policies (LPC_* environment knobs read at
lpc_open) on one scene.  Every configuration must give the identical trace
(per-iteration ray counts, measured count, per-mesh measured power): the
policies change only speed.  All engines stay open and are timed round-robin
(rounds x steps), so clock drift and warm-up hit every configuration alike.

    python tools/sweep.py [scene] [rays] [rounds] 'FLAT=0' 'FLAT=5,KEY=3' ...
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.distributed import ShardedTrace  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

KNOBS = ("KEY", "LARGE_PER_TRI", "BUDGET_LARGE", "LARGE_N", "FLAT", "TARGET_BLOCKS", "SORT", "BUDGET", "SPILL_CAP", "SPILL_BLOCKS", "LOOP", "SLIVER_WAVES",
         "SLIVER_PPW", "NODE_W", "SPILL_LEVELS", "PAIR_SHIFT", "SORT_MIN", "LOOP_MIN", "GATHER_AOS", "SLIVER_RAYS", "WAVE_TARGET", "SLIVER_CULL", "SPILL_SHRINK", "SPILL_MIN_BLOCKS", "LANE_MAX", "LANE_G", "ISECT_MINB", "ONESWEEP_MIN", "SPILL_LEVELS_SMALL", "FUSE_SHADE", "XCD_ROWS", "CHAIN", "CHUNK", "QUEUE", "TRACED", "TRACED_SORT", "Q_TARGET", "Q_WALK_BLOCKS", "Q_WALK_WPB",
         "SPILL_WPB", "SIDE_STREAM", "EARLY_ACC", "DBG", "FUSE_COMPACT", "SLIVER_LATE", "WALK_WAVES", "HALF", "SHADE_KU", "ROOTS_S", "XCD_WALK", "ROOTS_TASKS", "EV_SYSFENCE", "FORK_LATE", "SHADE_CFIRST")
name = sys.argv[1] if len(sys.argv) > 1 else "synthetic"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
configs = sys.argv[4:] or ["KEY=0"]
steps = int(os.environ.get("SWEEP_STEPS", "3"))
sc = scenes.BUILDERS[name](n=n, seed=7)
o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
in_pow = float(np.sum(p, dtype=np.float64))
ref = None
engs = []
for cfg in configs:
    env = dict(kv.split("=") for kv in cfg.split(",") if kv)
    for k in KNOBS:
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
    engs.append((cfg, e, run, same, len(got[0])))
for k in KNOBS:
    os.environ.pop("LPC_" + k, None)
ms = {cfg: [] for cfg, *_ in engs}
isect = {cfg: [] for cfg, *_ in engs}
for _ in range(rounds):
    for cfg, e, run, _, nit in engs:
        if os.environ.get("SWEEP_ASYNC"):     # back-to-back async traces (bench.py's steps), one sync
            e.sync()
            t = time.perf_counter()
            for _ in range(steps):
                e.reset()
                run.run(sc.iterations, sc.tau, in_pow, wait=False)
            e.sync()
            ms[cfg].append(1e3 * (time.perf_counter() - t) / steps)
        else:
            for _ in range(steps):
                e.reset()
                t = time.perf_counter()
                run.run(sc.iterations, sc.tau, in_pow)
                ms[cfg].append(1e3 * (time.perf_counter() - t))
        # per-iteration intersect stage time (HIP events)
        e.prof_enable(True)
        e.reset()
        e.prof_read(reset=True)
        its = []
        for _ in range(nit):
            st, _ = e.iterate()
            its.append(e.prof_read(reset=True)["intersect_ms"])
        e.prof_enable(False)
        isect[cfg].append(its)
bounces = sum(ref[0])
for cfg, e, run, same, nit in engs:
    m = float(np.median(ms[cfg]))
    it = np.median(np.asarray(isect[cfg]), axis=0)
    print(f"{cfg:34s} {m:7.3f} ms/step (min {min(ms[cfg]):.3f})  {bounces / (m * 1e-3) / 1e6:7.1f} M bounces/s "
          f"[{same}] isect/it: " + " ".join(f"{c}:{t:.3f}" for c, t in zip(ref[0], it)), flush=True)
    e.close()
