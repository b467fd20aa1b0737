"""Multi-process (world_size 2, gloo, CPU) run of the sharded trace driver
(lightpycl_amd.distributed): each rank traces its contiguous shard of the rays
and all ranks take the reference's global termination decision from all-reduced
(live rays, power left).  The global per-iteration ray counts, the summed
per-mesh measured power and the all-reduced angular histogram must equal a
single-process trace of all rays."""
import json
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
HIST_LIMITS = ((-np.pi / 2, np.pi / 2), (-np.pi / 2, np.pi / 2))
HIST_POINTS = 30


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, n, out_path):
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lightpycl_amd import scenes
    from lightpycl_amd.distributed import ShardedTrace, TorchComm, shard_bounds
    from oracle_engine import OracleEngine
    sc = scenes.BUILDERS[name](n=n, seed=2)
    o = np.asarray(sc.sources[0].rays_origin, np.float32)
    d = np.asarray(sc.sources[0].rays_dir, np.float32)
    p = np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1)
    lo, hi = shard_bounds(len(p), rank, world)
    eng = OracleEngine(sc.meshes, o[lo:hi], d[lo:hi], p[lo:hi], sc.max_ray_len, sc.ior_env)
    r = ShardedTrace(eng, TorchComm(dist)).run(sc.iterations, sc.tau, float(np.sum(p[lo:hi], dtype=np.float64)),
                                               hist=(HIST_LIMITS, HIST_POINTS))
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(dict(counts=r["global_counts"], mesh_power=list(map(float, r["mesh_power"])),
                           hist=r["hist"][0].tolist()), f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,n", [("lens", 3000), ("parabolic", 2001)])
def test_sharded_trace_matches_single_process(oracle_mod, tmp_path, name, n):
    from lightpycl_amd import scenes
    out = str(tmp_path / "r.json")
    mp.spawn(_worker, args=(2, _free_port(), name, n, out), nprocs=2, join=True)
    got = json.load(open(out))
    sc = scenes.BUILDERS[name](n=n, seed=2)
    res, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env)
    assert got["counts"] == info["counts"]
    np.testing.assert_allclose(got["mesh_power"], info["mesh_power"], rtol=1e-12, atol=1e-12)
    # angular histogram of the measured rays: per-rank bins all-reduced (float64;
    # only the summation order differs from the single-process binning)
    pos, pwr = oracle_mod.measured_rays(res)
    H = oracle_mod.binned_angular(pos, pwr, HIST_LIMITS, HIST_POINTS)[0]
    assert np.sum(H) > 0
    np.testing.assert_allclose(np.asarray(got["hist"]), H, rtol=1e-12, atol=1e-9 * float(np.max(H)))


def test_shard_bounds_cover():
    from lightpycl_amd.distributed import shard_bounds
    for n in (0, 1, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            parts = [shard_bounds(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1


# -- the library's intra-node all-reduce (lpc_shm_comm_*), CPU only ------------------
def _shm_worker(rank, world, name, out_dir):
    sys.path.insert(0, os.path.dirname(HERE))
    from lightpycl_amd.distributed import ShmComm
    c = ShmComm(name, rank, world, create=(rank == 0))
    rng = np.random.default_rng(rank)
    res = {}
    for n in (0, 1, 5, 8192, 20000):            # 20000 > one exchange chunk (8192 doubles)
        v = rng.normal(size=n)
        res[n] = (v, c.allreduce_sum(v))
    for rep in range(200):                      # many back-to-back exchanges (buffer parity reuse)
        x = c.allreduce_sum([rank + rep, 1.0])
        assert x[0] == sum(r + rep for r in range(world)) and x[1] == world
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **{f"in{n}": a for n, (a, _) in res.items()},
             **{f"out{n}": b for n, (_, b) in res.items()})
    c.close()


@pytest.mark.parametrize("world", [2, 4])
def test_shm_allreduce_identical_bits(tmp_path, world):
    """lpc_shm_allreduce: every rank receives the rank-order sum, bit for bit
    (so every rank takes the identical termination decision)."""
    import secrets
    name = f"lpc_test_{os.getpid()}_{secrets.token_hex(4)}"
    mp.spawn(_shm_worker, args=(world, name, str(tmp_path)), nprocs=world, join=True)
    got = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    for n in (0, 1, 5, 8192, 20000):
        want = got[0][f"in{n}"].copy()
        for r in range(1, world):
            want = want + got[r][f"in{n}"]
        for r in range(world):
            np.testing.assert_array_equal(got[r][f"out{n}"], want)
    assert not os.path.exists(f"/dev/shm/{name}")


def test_shm_comm_errors():
    sys.path.insert(0, os.path.dirname(HERE))
    from lightpycl_amd import _lib
    from lightpycl_amd.distributed import ShmComm
    with pytest.raises(_lib.LpcError):
        ShmComm("x", 3, 2, create=True)         # rank out of range
    c = ShmComm(f"lpc_single_{os.getpid()}", 0, 1, create=True)
    np.testing.assert_array_equal(c.allreduce_sum([1.5, 2.0]), [1.5, 2.0])
    c.close()


def _worker_shm(rank, world, port, name, n, out_path):
    """The sharded driver with the library's shared-memory comm for the
    per-iteration decisions and gloo for the trace-end histogram."""
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lightpycl_amd import scenes
    from lightpycl_amd.distributed import ShardedTrace, ShmComm, TorchComm, shard_bounds
    from oracle_engine import OracleEngine
    shm = ShmComm.from_dist(dist)
    sc = scenes.BUILDERS[name](n=n, seed=2)
    o = np.asarray(sc.sources[0].rays_origin, np.float32)
    d = np.asarray(sc.sources[0].rays_dir, np.float32)
    p = np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1)
    lo, hi = shard_bounds(len(p), rank, world)
    eng = OracleEngine(sc.meshes, o[lo:hi], d[lo:hi], p[lo:hi], sc.max_ray_len, sc.ior_env)
    r = ShardedTrace(eng, shm).run(sc.iterations, sc.tau, float(np.sum(p[lo:hi], dtype=np.float64)),
                                   hist=(HIST_LIMITS, HIST_POINTS))
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(dict(counts=r["global_counts"], mesh_power=list(map(float, r["mesh_power"]))), f)
    shm.close()
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_trace_world8(oracle_mod, tmp_path):
    """The N = 8 split rehearsed on the CPU (the 8-GPU node is the driver's): eight
    gloo ranks, each tracing its contiguous shard through the sharded driver with
    the library's shared-memory per-iteration exchange, give the single-process
    trace's global per-iteration counts and per-mesh power (the partition loop
    this replaces: iterative_tracer.py:246-271, 383-391)."""
    from lightpycl_amd import scenes
    out = str(tmp_path / "r.json")
    mp.spawn(_worker_shm, args=(8, _free_port(), "lens", 2403, out), nprocs=8, join=True)
    got = json.load(open(out))
    sc = scenes.lens(n=2403, seed=2)
    _, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                               keep_results=False)
    assert got["counts"] == info["counts"] and len(info["counts"]) >= 4
    np.testing.assert_allclose(got["mesh_power"], info["mesh_power"], rtol=1e-12, atol=1e-12)


def test_config5_split_covers_blocks():
    """bench.py's config-5 ray set (8 fixed blocks) split over 1, 2, 4, 8 and 16
    ranks: the ranks' shards, concatenated in rank order, are the whole set in
    order (world == 8: one block per rank; world > 8: blocks split by rays)."""
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    from lightpycl_amd import scenes
    total = 8 * 96
    whole = bench.config5_rays(scenes, 0, 1, total)
    for world in (2, 4, 8, 16):
        parts = [bench.config5_rays(scenes, r, world, total) for r in range(world)]
        assert [len(q[2]) for q in parts] == [total // world] * world
        for k in range(3):
            np.testing.assert_array_equal(np.concatenate([q[k] for q in parts]), whole[k])


def test_sharded_trace_shm_comm(oracle_mod, tmp_path):
    from lightpycl_amd import scenes
    out = str(tmp_path / "r.json")
    mp.spawn(_worker_shm, args=(3, _free_port(), "lens", 2500, out), nprocs=3, join=True)
    got = json.load(open(out))
    sc = scenes.lens(n=2500, seed=2)
    _, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                               keep_results=False)
    assert got["counts"] == info["counts"]
    np.testing.assert_allclose(got["mesh_power"], info["mesh_power"], rtol=1e-12, atol=1e-12)


def _abort_worker(rank, world, name, out_dir):
    """Rank 1 exchanges once, then gives up (lpc_shm_comm_abort); rank 0's next
    exchange must fail at once (not after the 300 s timeout), and every later
    exchange on the broken comm too."""
    import time
    sys.path.insert(0, os.path.dirname(HERE))
    from lightpycl_amd import _lib
    from lightpycl_amd.distributed import ShmComm
    c = ShmComm(name, rank, world, create=(rank == 0))
    assert list(c.allreduce_sum([1.0])) == [float(world)]
    res = {}
    if rank == 1:
        c.abort()
        with pytest.raises(_lib.LpcError):
            c.allreduce_sum([1.0])
    else:
        t = time.perf_counter()
        try:
            c.allreduce_sum([2.0])
            res["first"] = "ok"
        except _lib.LpcError as e:
            res["first"] = str(e)
        res["wait_s"] = time.perf_counter() - t
        try:
            c.allreduce_sum([3.0])
            res["second"] = "ok"
        except _lib.LpcError as e:
            res["second"] = str(e)
        with open(os.path.join(out_dir, "abort.json"), "w") as f:
            json.dump(res, f)
    c.close()


def test_shm_comm_abort_fails_peers_fast(tmp_path):
    import secrets
    name = f"lpc_abort_{os.getpid()}_{secrets.token_hex(4)}"
    mp.spawn(_abort_worker, args=(2, name, str(tmp_path)), nprocs=2, join=True)
    got = json.load(open(tmp_path / "abort.json"))
    assert "aborted" in got["first"], got
    assert got["wait_s"] < 30.0, got
    assert got["second"] != "ok", got          # the comm stays broken


def test_shm_close_removes_installed_hook():
    """Closing a ShmComm takes its hook out of every engine it was installed in
    (an engine must not keep a pointer into the unmapped segment)."""
    sys.path.insert(0, os.path.dirname(HERE))
    from lightpycl_amd.distributed import ShmComm

    class FakeEngine:
        h = 1

        def __init__(self):
            self._xchg = None
            self.calls = []

        def set_allreduce(self, comm):
            if comm is None:
                self._xchg = None
            else:
                fn, _ = comm.native_hook(self)
                self._xchg = (comm, fn)
            self.calls.append(comm)

    c = ShmComm(f"lpc_hook_{os.getpid()}", 0, 1, create=True)
    e = FakeEngine()
    e.set_allreduce(c)
    c.close()
    assert e._xchg is None and e.calls[-1] is None
    with pytest.raises(RuntimeError):
        c.native_hook()
