"""Streamed batches of new rays (lpc_trace_stage_rays / lpc_trace_run_staged_async):
the next batch is copied to the device by a helper thread on a copy stream while
the engine traces the batch before it.  Each staged trace must equal the same
batch traced after lpc_trace_set_rays (itself bit-exact against the reference's
kernels, tests/test_gpu_parity.py): per-iteration counts, per-mesh measured power
bits and the measured rays as a set.  The reference uploads each partition's
rays inside its loop (iterative_tracer.py:280-284)."""
import numpy as np
import pytest

from lightpycl_amd import scenes

pytestmark = pytest.mark.gpu


def _batch(n, seed):
    ls = scenes.synthetic_rays(n=n, seed=seed)
    return (np.asarray(ls.rays_origin, np.float32), np.asarray(ls.rays_dir, np.float32),
            np.asarray(ls.rays_power, np.float32).reshape(-1))


def _measured(e):
    from parity_util import measured_rows
    return measured_rows(*e.fetch_measured())


@pytest.mark.parametrize("name,n", [("synthetic", 150000), ("synthetic_dense", 40000)])
def test_staged_batches_equal_set_rays(name, n):
    from lightpycl_amd.engine import Engine
    sc = scenes.BUILDERS[name](n=64, seed=7)
    batches = [_batch(n, 500 + b) for b in range(4)] + [_batch(n // 3, 600)]   # a smaller last batch
    thr = [(1.0 - sc.tau) * float(np.sum(b[2], dtype=np.float64)) for b in batches]
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        ref = []
        for b, t in zip(batches, thr):
            e.set_rays(*b, sc.max_ray_len, sc.ior_env)
            st, (c, mp) = e.run_local(sc.iterations, t)
            ref.append(([int(s.n_in) for s in st], c, mp.tolist(), _measured(e)))
        # pipelined: batch k + 1 staged before batch k is traced; twice over, so
        # the second pass runs with the first's speculation predictions
        for rep in range(2):
            e.stage_rays(*batches[0], sc.max_ray_len, sc.ior_env)
            for k in range(len(batches)):
                if k + 1 < len(batches):
                    e.stage_rays(*batches[k + 1], sc.max_ray_len, sc.ior_env)
                st, (c, mp) = e.run_staged(sc.iterations, thr[k])
                got = ([int(s.n_in) for s in st], c, mp.tolist())
                assert got == tuple(ref[k][:3]), (rep, k, got[:2], ref[k][:2])
                np.testing.assert_array_equal(_measured(e), ref[k][3], err_msg=f"pass {rep} batch {k}")
        # the staged batch is the emitted population: a reset re-traces it
        e.reset()
        st, (c, mp) = e.run_local(sc.iterations, thr[-1])
        assert [int(s.n_in) for s in st] == ref[-1][0] and mp.tolist() == ref[-1][2]
    finally:
        e.close()


def test_stage_errors_and_scene_upload(engine):
    from lightpycl_amd import _lib
    sc = scenes.synthetic(n=64, seed=7)
    engine.upload_meshes(sc.meshes)
    b = _batch(5000, 9)
    with pytest.raises(_lib.LpcError, match="no batch staged"):
        engine.run_staged(4, 0.0)
    engine.stage_rays(*b, sc.max_ray_len, sc.ior_env)
    engine.stage_rays(*b, sc.max_ray_len, sc.ior_env)
    with pytest.raises(_lib.LpcError, match="two batches"):
        engine.stage_rays(*b, sc.max_ray_len, sc.ior_env)
    st, _ = engine.run_staged(sc.iterations, 0.0)
    assert int(st[0].n_in) == 5000
    # a batch staged under one scene and traced under another: its analysis (keyed
    # to the scene box) is redone, and the trace equals set_rays under the new scene
    lens = scenes.lens(n=64, seed=1)
    engine.upload_meshes(lens.meshes)
    st, (c, mp) = engine.run_staged(lens.iterations, 1.0)
    got = ([int(x.n_in) for x in st], c, mp.tolist(), _measured(engine))
    engine.set_rays(*b, sc.max_ray_len, sc.ior_env)
    st, (c, mp) = engine.run_local(lens.iterations, 1.0)
    assert got[:3] == ([int(x.n_in) for x in st], c, mp.tolist())
    np.testing.assert_array_equal(got[3], _measured(engine))


def test_stage_before_scene():
    """The drop-in's aggregate mode stages its rays before it builds the scene
    records: the batch traced after the upload equals set_rays after it."""
    from lightpycl_amd.engine import Engine
    sc = scenes.eye(n=20000, seed=3)
    o, d, p = (np.asarray(sc.sources[0].rays_origin, np.float32), np.asarray(sc.sources[0].rays_dir, np.float32),
               np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1))
    thr = (1.0 - sc.tau) * float(np.sum(p, dtype=np.float64))
    e = Engine(0)
    try:
        e.stage_rays(o, d, p, sc.max_ray_len, sc.ior_env)
        e.upload_meshes(sc.meshes)
        st, (c, mp) = e.run_staged(sc.iterations, thr)
        got = ([int(x.n_in) for x in st], c, mp.tolist(), _measured(e))
        e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
        st, (c, mp) = e.run_local(sc.iterations, thr)
        assert got[:3] == ([int(x.n_in) for x in st], c, mp.tolist())
        np.testing.assert_array_equal(got[3], _measured(e))
    finally:
        e.close()
