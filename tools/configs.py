"""GPU box: BASELINE.json configs 2-4 (and the synthetic headline scene) at full
size on one MI355X: ray-bounces/s of a whole trace (inputs resident, as bench.py)
and the ray-sharding property -- two engines tracing the two halves of the rays
in lockstep with the reference's global termination give the single engine's
per-iteration counts and measured count exactly, and its per-mesh measured power
to float64 summation order.

    python tools/configs.py [name ...]      (default: parabolic lens eye)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.distributed import ShardedTrace, shard_bounds  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

CONFIGS = {   # BASELINE.json configs: rays, depth
    "parabolic": (1_000_000, 4),
    "lens": (10_000_000, 8),
    "eye": (10_000_000, 16),
    "synthetic": (1_000_000, 16),
    "synthetic_shard": (12_500_000, 16),   # config 5: one GPU's shard of 100 M rays over 8
}
SCENE = {"synthetic_shard": "synthetic"}


def rays(sc):
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
    return o, d, p


def lockstep(engines, iterations, thr):
    counts = []
    for _ in range(iterations):
        sts = [e.iterate()[0] for e in engines]
        counts.append(sum(int(s.n_in) for s in sts))
        if sum(float(s.power_next) for s in sts) < thr:
            break
        if sum(int(s.n_reflect + s.n_refract) for s in sts) == 0:
            break
    cnt = sum(e.measured()[0] for e in engines)
    mp = np.sum([e.measured()[1] for e in engines], axis=0)
    return counts, cnt, mp


def main():
    names = sys.argv[1:] or ["parabolic", "lens", "eye"]
    for name in names:
        n, depth = CONFIGS[name]
        t0 = time.perf_counter()
        sc = scenes.BUILDERS[SCENE.get(name, name)](n=n, seed=7, iterations=depth)
        o, d, p = rays(sc)
        gen_s = time.perf_counter() - t0
        in_pow = float(np.sum(p, dtype=np.float64))
        e = Engine(0)
        e.upload_meshes(sc.meshes)
        e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
        run = ShardedTrace(e)
        e.reset()
        r = run.run(depth, sc.tau, in_pow)                 # warm-up (allocations)
        ts = []
        for _ in range(3):
            e.reset()
            t = time.perf_counter()
            r = run.run(depth, sc.tau, in_pow)
            ts.append(time.perf_counter() - t)
        full = (r["global_counts"], e.measured()[0], np.asarray(r["mesh_power"]))
        e.close()
        # the two halves in lockstep (ray sharding, global termination)
        halves = []
        for k in range(2):
            lo, hi = shard_bounds(len(p), k, 2)
            h = Engine(0)
            h.upload_meshes(sc.meshes)
            h.set_rays(o[lo:hi], d[lo:hi], p[lo:hi], sc.max_ray_len, sc.ior_env)
            h.reset()
            halves.append(h)
        counts, cnt, mp = lockstep(halves, depth, (1.0 - sc.tau) * in_pow)
        for h in halves:
            h.close()
        ok = counts == full[0] and cnt == full[1] and np.allclose(mp, full[2], rtol=1e-9, atol=0.0)
        t = float(np.median(ts))
        bounces = sum(full[0])
        print(json.dumps(dict(config=name, rays=n, depth=depth, triangles=int(sum(len(m.tribuf()[0]) for m in sc.meshes)),
                              iterations=len(full[0]), bounces=bounces, seconds=t,
                              ray_bounces_per_s=bounces / t, measured=int(full[1]),
                              measured_power=float(np.sum(full[2])), input_power=in_pow,
                              halves_match=bool(ok), host_generation_s=gen_s)), flush=True)
        if not ok:
            print("halves:", counts, cnt, mp.tolist(), "full:", full[0], full[1], full[2].tolist(), flush=True)


if __name__ == "__main__":
    main()
