"""Ray-sharded multi-GPU trace: one process per GPU, scene replicated, rays split.

The reference traces every ray independently within an iteration
(``kernel_reflect_refract_intersect.cl`` indexes only its own ray), so a shard of
rays is traced to completion on its own GPU with no data-path exchange.  The only
real exchange steps are the reference's global decisions and outputs:

* per iteration, the termination test ``power_in_scene < (1-tau) * input_power``
  and ``ray_count == 0`` (``iterative_tracer.py:372-391``) are taken on the
  all-reduced (power left, live rays) pair, so every rank stops at the same
  iteration as a single-device trace of all rays would;
* at trace end, the per-mesh measured power (and, if requested, the angular
  histogram) are all-reduced.

All messages are a few doubles: latency-bound, one RCCL all-reduce each.  On CPU
(tests) the same code runs over gloo with any engine object exposing
``iterate() -> (stats, _)`` and ``measured() -> (count, mesh_power)``.
"""
from __future__ import annotations

import ctypes
import os
import socket
import weakref

import numpy as np


class TorchComm:
    """All-reduce of small float64 vectors over torch.distributed (RCCL on GPU,
    gloo on CPU)."""

    def __init__(self, dist, local_rank=0, device=None):
        import torch
        self.torch = torch
        self.dist = dist
        if device is None:
            device = f"cuda:{local_rank}" if dist.get_backend() == "nccl" else "cpu"
        self.device = device

    def allreduce_sum(self, values):
        v = np.asarray(values, dtype=np.float64).reshape(-1)
        if self.device == "cpu":
            t = self.torch.from_numpy(v.copy())
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
            return t.numpy()
        # GPU (RCCL): persistent device and pinned host buffers, no per-call allocation
        n = v.shape[0]
        if getattr(self, "_dev", None) is None or self._dev.shape[0] < n:
            m = max(n, 64)
            self._dev = self.torch.zeros(m, dtype=self.torch.float64, device=self.device)
            self._host = self.torch.zeros(m, dtype=self.torch.float64).pin_memory()
        h, d = self._host[:n], self._dev[:n]
        h.copy_(self.torch.from_numpy(v))
        d.copy_(h, non_blocking=True)
        self.dist.all_reduce(d, op=self.dist.ReduceOp.SUM)
        h.copy_(d)
        return h.numpy().copy()

    @property
    def rank(self):
        return self.dist.get_rank()

    @property
    def world(self):
        return self.dist.get_world_size()


class ShmComm:
    """The library's intra-node all-reduce (lpc_shm_comm_*, POSIX shared memory):
    rank-order sums, identical bits on every rank, ~1 us per exchange.  Installed
    in an engine it runs inside lpc_trace_run's loop with no Python in between
    (``native_hook``); ``allreduce_sum`` calls it from Python."""

    def __init__(self, name, rank, world, create):
        from . import _lib
        self._lib = _lib
        self.L = _lib.load()
        self.rank = int(rank)
        self.world = int(world)
        c = ctypes.c_void_p()
        _lib.check(self.L.lpc_shm_comm_open(name.encode(), self.rank, self.world, 1 if create else 0,
                                            ctypes.byref(c)))
        self.c = c
        self._engines = weakref.WeakSet()     # engines whose loop calls this comm (native_hook)

    @staticmethod
    def single_node(dist):
        """True when every rank of the job runs on this host (POSIX shared memory
        reaches only the ranks of one node): the hostnames all-gathered."""
        names = [None] * dist.get_world_size()
        dist.all_gather_object(names, socket.gethostname())
        return len(set(names)) == 1

    @classmethod
    def from_dist(cls, dist, fallback=None):
        """One segment per torch.distributed job: rank 0 names and creates it, the
        others open it, then the name is unlinked (nothing is left in /dev/shm).
        On a multi-node job the segment cannot reach every rank: returns
        ``fallback`` (e.g. a :class:`TorchComm`, called through the hook) instead."""
        import secrets
        if not cls.single_node(dist):
            return fallback
        rank, world = dist.get_rank(), dist.get_world_size()
        box = [f"lpc_{os.getpid()}_{secrets.token_hex(6)}" if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        comm = cls(box[0], rank, world, create=(rank == 0))
        dist.barrier()
        comm.unlink()
        return comm

    def native_hook(self, engine=None):
        if not self.c:
            raise RuntimeError("ShmComm is closed")
        if engine is not None:
            self._engines.add(engine)
        fn = ctypes.cast(self.L.lpc_shm_allreduce, ctypes.c_void_p)
        return fn, self.c

    def abort(self):
        """Break the comm (lpc_shm_comm_abort): later exchanges fail here, and the
        peers' current waits fail instead of running to the 300 s timeout."""
        if self.c:
            self.L.lpc_shm_comm_abort(self.c)

    def allreduce_sum(self, values):
        v = np.ascontiguousarray(np.asarray(values, dtype=np.float64).reshape(-1)).copy()
        self._lib.check(self.L.lpc_shm_allreduce(self.c, v.ctypes.data_as(ctypes.c_void_p), v.shape[0]))
        return v

    def unlink(self):
        if self.c:
            self.L.lpc_shm_comm_unlink(self.c)

    def close(self):
        """Unmap the segment.  The hook is removed first from every engine that
        still has it installed, so no later trace calls into freed memory."""
        if getattr(self, "c", None):
            for e in list(getattr(self, "_engines", ())):
                if getattr(e, "_xchg", None) is not None and e._xchg[0] is self and getattr(e, "h", None):
                    e.set_allreduce(None)
            self.L.lpc_shm_comm_close(self.c)
            self.c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_bounds(n, rank, world):
    """Contiguous shard [lo, hi) of n rays for `rank` (sizes differ by at most 1)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


class ShardedTrace:
    """Drive one rank's engine through the reference's iteration loop with global
    termination decisions.

    A liblpc engine runs the loop inside the library (lpc_trace_run(_async));
    with a comm the per-iteration all-reduce is the library's hook
    (``iter_comm``: the native shared-memory comm when given, else ``comm``
    through a ctypes callback), so N > 1 adds one tiny exchange per iteration
    and keeps the single-GPU pipelining.  The trace-end histogram is all-reduced
    over ``comm`` (RCCL on GPU ranks).  Engines without ``run_local`` (the CPU
    tests' OracleEngine) run the same loop here in Python."""

    def __init__(self, engine, comm=None, iter_comm=None):
        self.engine = engine
        self.comm = comm
        self.iter_comm = iter_comm if iter_comm is not None else comm
        self._installed = None

    def close(self):
        """Remove the per-iteration hook from the engine (before its comm closes)."""
        if self._installed is not None and hasattr(self.engine, "set_allreduce") and getattr(self.engine, "h", None):
            self.engine.set_allreduce(None)
        self._installed = None

    def _sum(self, vals):
        if self.comm is None:
            return np.asarray(vals, dtype=np.float64)
        return self.comm.allreduce_sum(vals)

    def run(self, iterations, tau, input_power_local, hist=None, wait=True, input_power_global=None, reset=False):
        """Trace to the reference's termination.  hist=(limits, points): also bin
        the measured rays (get_binned_data_angular) on every rank and all-reduce
        the histogram (float64, bin counts are additive).  wait=False: return once
        the outputs are final, without waiting for the last rows to move on the
        device (engine.sync() waits).  input_power_global: the all-ranks input power
        if already known (no all-reduce for it).  reset=True: trace the engine's
        emitted rays again from the start (engine.reset() first; one library call
        with the trace for a liblpc engine)."""
        in_pow = (float(input_power_global) if input_power_global is not None
                  else float(self._sum([input_power_local])[0]))
        thr = (1.0 - tau) * in_pow
        bounces = 0
        iters = 0
        counts = []
        if hasattr(self.engine, "run_local"):
            if self.iter_comm is not None and self._installed is not self.iter_comm:
                self.engine.set_allreduce(self.iter_comm)
                self._installed = self.iter_comm
            stats, (_, mesh_pow) = self.engine.run_local(int(iterations), thr, wait=wait or hist is not None,
                                                         reset=reset)
            glob = self.engine.global_stats() if self.iter_comm is not None else stats
            bounces = sum(int(st.n_in) for st in stats)
            iters = len(stats)
            counts = [int(st.n_in) for st in glob]
            mesh_pow = np.asarray(mesh_pow, dtype=np.float64)
        else:
            if reset:
                self.engine.reset()
            for _ in range(int(iterations)):
                st, _ = self.engine.iterate()
                bounces += int(st.n_in)
                iters += 1
                tot = self._sum([st.n_in, st.power_next, st.n_reflect + st.n_refract])
                counts.append(int(tot[0]))
                if tot[1] < thr:
                    break
                if tot[2] == 0:
                    break
            _, mesh_pow = self.engine.measured()
            mesh_pow = self._sum(np.asarray(mesh_pow, dtype=np.float64))
        out = dict(bounces=bounces, iterations=iters, global_counts=counts, mesh_power=mesh_pow)
        if hist is not None:
            limits, points = hist
            H, xe, ye = self.engine.project_hist(None, None, limits, points)[:3]
            out["hist"] = (self._sum(np.asarray(H, np.float64).ravel()).reshape(H.shape), xe, ye)
        return out
