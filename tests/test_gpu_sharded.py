"""Config 5's path on the HIP engine: a ray-sharded trace over two processes, each
with its own liblpc handle on the GPU (the one GPU of the test box; one process
per GPU on an 8-GPU node), the per-iteration termination decisions taken inside
the library's loop (lpc_trace_run_async + the all-reduce hook,
iterative_tracer.py:383-391) and the trace-end angular histogram all-reduced.

The parent spawns fresh child processes (torch.multiprocessing, spawn) and never
replaces itself.  The global per-iteration counts, per-mesh measured power and
histogram must equal the single-process trace of all rays by the reference's own
kernels (the `checker` fixture; the CPU oracle without oracle/_ref).
"""
import json
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIMITS = ((-np.pi / 2, np.pi / 2), (-np.pi / 2, np.pi / 2))
POINTS = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(name, n):
    """The named scene; "neg_mirror": cube_field's mirrors with reflectivity -0.5
    (the reference's mirror child carries P * R, .cl:443: a negative R flips the
    sign, so a rank's power left can grow from one iteration to the next -- the
    sharded trace must not stop a rank on a local bound then)."""
    from lightpycl_amd import scenes
    if name == "neg_mirror":
        sc = scenes.cube_field(n=n, seed=2, count=150)
        for m in sc.meshes[1:]:
            if m.getMaterialBuf()["type"] == 1:
                m.reflectivity = -0.5
        return sc
    return scenes.BUILDERS[name](n=n, seed=2)


def _child(rank, world, port, name, n, hook, out_path):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lightpycl_amd.distributed import ShardedTrace, ShmComm, TorchComm, shard_bounds
    from lightpycl_amd.engine import Engine
    sc = _scene(name, n)
    o = np.asarray(sc.sources[0].rays_origin, np.float32)
    d = np.asarray(sc.sources[0].rays_dir, np.float32)
    p = np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1)
    lo, hi = shard_bounds(len(p), rank, world)
    eng = Engine(0)
    eng.upload_meshes(sc.meshes)
    eng.set_rays(o[lo:hi], d[lo:hi], p[lo:hi], sc.max_ray_len, sc.ior_env)
    comm = TorchComm(dist)                      # gloo: trace-end histogram, input power
    iter_comm = ShmComm.from_dist(dist) if hook == "shm" else comm
    tr = ShardedTrace(eng, comm, iter_comm=iter_comm)
    in_pow = float(np.sum(p[lo:hi], dtype=np.float64))
    runs = []
    # a trace to a lower threshold first: the next trace's prediction (speculative
    # device-sized iterations, kept in sharded traces) then runs past the ranks'
    # global stop, and the dropped iteration must leave no trace in the results
    eng.reset()
    tr.run(sc.iterations, 1.0 - (1.0 - sc.tau) * 1e-3, in_pow, wait=False)
    eng.prof_read(reset=True)
    for rep in range(3):                        # back-to-back asynchronous traces (the bench's step)
        eng.reset()
        r = tr.run(sc.iterations, sc.tau, in_pow, wait=False)
        runs.append((r["global_counts"], list(map(float, r["mesh_power"])), r["bounces"]))
    eng.sync()
    pr = eng.prof_read(reset=True)              # host time inside the per-iteration all-reduce hook
    eng.reset()
    r = tr.run(sc.iterations, sc.tau, in_pow, hist=(LIMITS, POINTS))
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(dict(counts=r["global_counts"], mesh_power=list(map(float, r["mesh_power"])),
                           hist=r["hist"][0].tolist(), runs=runs, xchg_us=pr["xchg_us"],
                           xchg_calls=pr["xchg_calls"]), f)
    if hook == "shm":
        iter_comm.close()
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,n,hook", [("synthetic", 20000, "shm"), ("lens", 20000, "shm"),
                                         ("lens", 9000, "gloo"), ("neg_mirror", 12000, "shm")])
def test_sharded_trace_two_processes(oracle_mod, checker, tmp_path, name, n, hook):
    import torch.multiprocessing as mp
    from lightpycl_amd import scenes
    out = str(tmp_path / "r.json")
    mp.spawn(_child, args=(2, _free_port(), name, n, hook, out), nprocs=2, join=True)
    got = json.load(open(out))
    # the exchange cost per iteration, kept with the GPU run's outputs
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "sharded.jsonl"), "a") as f:
        f.write(json.dumps(dict(scene=name, n=n, hook=hook, calls=got["xchg_calls"],
                                us_per_exchange=got["xchg_us"] / max(got["xchg_calls"], 1))) + "\n")
    sc = _scene(name, n)
    res, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                                 bounce_fn=checker[0])
    assert got["counts"] == info["counts"]
    np.testing.assert_allclose(got["mesh_power"], info["mesh_power"], rtol=1e-12, atol=1e-12)
    for counts, mpow, _ in got["runs"]:
        assert counts == got["counts"]
        np.testing.assert_array_equal(mpow, got["mesh_power"])
    pos, pwr = oracle_mod.measured_rays(res)
    H = oracle_mod.binned_angular(pos, pwr, LIMITS, POINTS)[0]
    l1 = np.abs(np.asarray(got["hist"]) - H).sum() / np.abs(H).sum()
    assert l1 <= 1e-5, l1
