"""BASELINE.json configs 2-4 on the GPU at reduced ray counts (full sizes:
tools/configs.py, results in DESIGN.md section 7): size-independent properties
of the whole trace.

* parabolic mirror + hemisphere, depth 4: every emitted ray reaches the mirror
  and then the hemisphere, so the trace has 2 iterations of (almost) n rays and
  the measured power is (almost) the input power;
* ray sharding: two engines tracing the two halves of the rays in lockstep with
  the reference's global termination (the multi-GPU scheme of
  lightpycl_amd.distributed) reproduce the single engine's per-iteration counts
  and measured count exactly and its per-mesh measured power to float64
  summation order."""
import numpy as np
import pytest

from lightpycl_amd import scenes
from lightpycl_amd.distributed import ShardedTrace, shard_bounds


def _rays(sc):
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
    return o, d, p


def _engine(sc, o, d, p):
    from lightpycl_amd.engine import Engine
    e = Engine(0)
    e.upload_meshes(sc.meshes)
    e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
    e.reset()
    return e


@pytest.mark.gpu
def test_parabolic_two_bounces():
    n = 200_000
    sc = scenes.BUILDERS["parabolic"](n=n, seed=7, iterations=4)
    o, d, p = _rays(sc)
    e = _engine(sc, o, d, p)
    in_pow = float(np.sum(p, dtype=np.float64))
    r = ShardedTrace(e).run(4, sc.tau, in_pow)
    cnt, mp = e.measured()
    e.close()
    assert len(r["global_counts"]) == 2 and r["global_counts"][0] == n
    assert r["global_counts"][1] >= n - n // 1000
    assert cnt >= n - n // 1000
    assert abs(float(np.sum(mp)) - in_pow) <= 1e-3 * in_pow


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,depth", [("lens", 300_000, 8), ("eye", 40_000, 16), ("synthetic", 200_000, 16)])
def test_ray_sharded_halves_match(name, n, depth):
    sc = scenes.BUILDERS[name](n=n, seed=7, iterations=depth)
    o, d, p = _rays(sc)
    in_pow = float(np.sum(p, dtype=np.float64))
    e = _engine(sc, o, d, p)
    r = ShardedTrace(e).run(depth, sc.tau, in_pow)
    full_cnt, full_mp = e.measured()
    e.close()
    halves = []
    for k in range(2):
        lo, hi = shard_bounds(len(p), k, 2)
        halves.append(_engine(sc, o[lo:hi], d[lo:hi], p[lo:hi]))
    thr = (1.0 - sc.tau) * in_pow
    counts = []
    for _ in range(depth):
        sts = [h.iterate()[0] for h in halves]
        counts.append(sum(int(s.n_in) for s in sts))
        if sum(float(s.power_next) for s in sts) < thr:
            break
        if sum(int(s.n_reflect + s.n_refract) for s in sts) == 0:
            break
    cnt = sum(h.measured()[0] for h in halves)
    mp = np.sum([h.measured()[1] for h in halves], axis=0)
    for h in halves:
        h.close()
    assert counts == r["global_counts"]
    assert cnt == full_cnt
    np.testing.assert_allclose(mp, full_mp, rtol=1e-9, atol=0.0)


@pytest.mark.gpu
def test_rccl_comm_single_rank():
    """The RCCL code path of TorchComm (device + pinned host buffers) on a
    one-rank process group: the all-reduced trace equals the local trace."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    from lightpycl_amd.distributed import TorchComm
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        comm = TorchComm(dist, 0)
        np.testing.assert_array_equal(comm.allreduce_sum([1.0, 2.5, 3.0]), [1.0, 2.5, 3.0])
        np.testing.assert_array_equal(comm.allreduce_sum(np.arange(100.0)), np.arange(100.0))
        sc = scenes.BUILDERS["lens"](n=20_000, seed=7, iterations=8)
        o, d, p = _rays(sc)
        in_pow = float(np.sum(p, dtype=np.float64))
        e = _engine(sc, o, d, p)
        r_comm = ShardedTrace(e, comm).run(8, sc.tau, in_pow)
        e.reset()
        r_loc = ShardedTrace(e).run(8, sc.tau, in_pow)
        e.close()
        assert r_comm["global_counts"] == r_loc["global_counts"]
        np.testing.assert_allclose(r_comm["mesh_power"], r_loc["mesh_power"], rtol=1e-12, atol=0.0)
    finally:
        dist.destroy_process_group()
