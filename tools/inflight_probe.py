"""Traces in flight: E engines (handles, each its own stream and copy of the
scene; with E > 1 TracePool's walk grid) on one GPU, each re-tracing the
headline's 1 M rays from its own host thread, against one engine alone.  Prints one JSON line per E: total
ray-bounces/s and the per-trace time seen by each thread.

    python tools/inflight_probe.py [traces per engine] [E ...]
"""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import Engine
    from lightpycl_amd.pool import INFLIGHT_WALK_GRID
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    Es = [int(a) for a in sys.argv[2:]] or [1, 2, 3]
    sc = scenes.synthetic(n=1_000_000, seed=7)
    s = sc.sources[0]
    o = np.asarray(s.rays_origin, np.float32)
    d = np.asarray(s.rays_dir, np.float32)
    p = np.asarray(s.rays_power, np.float32).reshape(-1)
    thr = (1.0 - sc.tau) * float(np.sum(p, dtype=np.float64))
    for E in Es:
        engines = []
        for _ in range(E):
            e = Engine(0)
            e.upload_meshes(sc.meshes)
            e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
            if E > 1:
                e.set_walk_grid(INFLIGHT_WALK_GRID)     # as TracePool does
            engines.append(e)
        bounces = []
        for e in engines:                       # warm-up, and the bounces of one trace
            for _ in range(5):
                st, _ = e.run_local(sc.iterations, thr, wait=False, reset=True)
            e.sync()
            bounces.append(sum(int(x.n_in) for x in st))
        per = [0.0] * E

        def worker(i):
            e = engines[i]
            t0 = time.perf_counter()
            for _ in range(K):
                e.run_local(sc.iterations, thr, wait=False, reset=True)
            e.sync()
            per[i] = (time.perf_counter() - t0) / K

        th = [threading.Thread(target=worker, args=(i,)) for i in range(E)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        total = K * sum(bounces)
        print(json.dumps(dict(engines=E, traces=K * E, seconds=dt, ray_bounces_per_s=total / dt,
                              ms_per_trace_amortized=1e3 * dt / (K * E),
                              ms_per_trace_per_thread=[1e3 * x for x in per], bounces_per_trace=bounces)),
              flush=True)
        for e in engines:
            e.close()


if __name__ == "__main__":
    main()
