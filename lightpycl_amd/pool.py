"""Several traces in flight on one GPU (round 6).

A trace of 1 M rays leaves much of the MI355X idle: its small chained
populations and the tails of its hierarchy walks hold a few thousand waves at a
time.  Independent batches -- the reference's partitions
(iterative_tracer.py:246-271) or a caller's stream of light sources -- can share
the chip: a :class:`TracePool` keeps ``engines`` liblpc handles on the device,
each with its own HIP stream, scene records and population buffers, and one host
thread per handle (ctypes releases the GIL inside the library calls), so up to
``engines`` traces run at once.  Each batch is traced exactly as by one engine
alone (the same kernels on the same rays: counts, per-mesh power and measured
rays identical; tests/test_gpu_pool.py); with three in flight the headline
workload runs 1.52x the ray-bounces/s of back-to-back traces (bench.py
``inflight``).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import queue
import threading

import numpy as np

from .engine import Engine

# Walk grid of engines that trace side by side: 16 384 single-wave blocks ran the
# headline 2.4 % faster than the default 65 536 with three in flight, and one
# trace alone 7-15 % slower on the larger configs.
# LPC_INFLIGHT_WALK_GRID overrides it (A/B runs).
INFLIGHT_WALK_GRID = int(os.environ.get("LPC_INFLIGHT_WALK_GRID", "16384"))


class TracePool:
    """``submit`` batches; each future gives the batch's per-iteration counts,
    ray-bounces, measured count and per-mesh measured power (and, with
    ``measured=True``, the measured rows).  Batches go to the engines in turn;
    an engine traces its batches in submission order."""

    def __init__(self, meshes, device=0, engines=3):
        self.engines = [Engine(device) for _ in range(max(1, int(engines)))]
        for e in self.engines:
            e.upload_meshes(meshes)
            if len(self.engines) > 1:
                e.set_walk_grid(INFLIGHT_WALK_GRID)
        self._q = [queue.Queue() for _ in self.engines]
        self._next = 0
        self._lock = threading.Lock()
        self._th = [threading.Thread(target=self._worker, args=(j,), daemon=True) for j in range(len(self.engines))]
        for t in self._th:
            t.start()

    def _worker(self, j):
        e = self.engines[j]
        while True:
            job = self._q[j].get()
            if job is None:
                return
            fut, args = job
            if not fut.set_running_or_notify_cancel():
                continue
            try:
                fut.set_result(self._trace(e, *args))
            except BaseException as ex:
                fut.set_exception(ex)

    @staticmethod
    def _trace(e, origin, direction, power, max_ray_len, ior_env, iterations, tau, measured):
        p = np.asarray(power, np.float32).reshape(-1)
        e.set_rays(origin, direction, p, max_ray_len, ior_env)
        thr = (1.0 - float(tau)) * float(np.sum(p, dtype=np.float64))
        stats, (count, mesh_power) = e.run_local(int(iterations), thr)
        out = {"counts": [int(s.n_in) for s in stats], "ray_bounces": int(sum(int(s.n_in) for s in stats)),
               "measured_count": int(count), "mesh_power": np.asarray(mesh_power, np.float64)}
        if measured:
            out["measured"] = e.fetch_measured()
        return out

    def submit(self, origin, direction, power, max_ray_len=1e3, ior_env=1.0, iterations=16, tau=0.99,
               measured=False):
        """Queue one batch (origin/direction (n,4) float32 rows, power (n,)):
        traced to the reference's termination (``iterations``, dissipated
        fraction ``tau``, iterative_tracer.py:383-391).  Returns a Future."""
        fut = cf.Future()
        with self._lock:
            j = self._next
            self._next = (self._next + 1) % len(self.engines)
        self._q[j].put((fut, (origin, direction, power, max_ray_len, ior_env, iterations, tau, measured)))
        return fut

    def close(self):
        for q in self._q:
            q.put(None)
        for t in self._th:
            t.join()
        for e in self.engines:
            e.close()
        self.engines = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
