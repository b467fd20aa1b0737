"""Traces in flight (lightpycl_amd.pool.TracePool): several engines on one GPU,
each tracing its batches from its own host thread while the others run.  Every
batch must come out exactly as one engine alone traces it -- per-iteration
counts, measured count, per-mesh power bits and the measured rays as a set --
and the one engine's traces are the reference kernels' (tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from lightpycl_amd import scenes

pytestmark = pytest.mark.gpu


def _batches(sc_name, n, k):
    out = []
    for b in range(k):
        ls = scenes.BUILDERS[sc_name](n=n, seed=40 + b).sources[0]
        out.append((np.asarray(ls.rays_origin, np.float32), np.asarray(ls.rays_dir, np.float32),
                    np.asarray(ls.rays_power, np.float32).reshape(-1)))
    return out


@pytest.mark.parametrize("name,n,k,engines", [("synthetic", 100000, 7, 3), ("lens", 20000, 5, 2)])
def test_pool_batches_equal_one_engine(name, n, k, engines):
    from lightpycl_amd.engine import Engine
    from lightpycl_amd.pool import TracePool
    from parity_util import measured_rows
    sc = scenes.BUILDERS[name](n=64, seed=1)
    batches = _batches(name, n, k)
    e = Engine(0)
    ref = []
    try:
        e.upload_meshes(sc.meshes)
        for o, d, p in batches:
            e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
            thr = (1.0 - sc.tau) * float(np.sum(p, dtype=np.float64))
            st, (c, mp) = e.run_local(sc.iterations, thr)
            ref.append(([int(s.n_in) for s in st], int(c), mp.tolist(), measured_rows(*e.fetch_measured())))
    finally:
        e.close()
    with TracePool(sc.meshes, engines=engines) as pool:
        futs = [pool.submit(o, d, p, sc.max_ray_len, sc.ior_env, sc.iterations, sc.tau, measured=True)
                for o, d, p in batches]
        got = [f.result(timeout=120) for f in futs]
    for b, (r, g) in enumerate(zip(ref, got)):
        assert g["counts"] == r[0], b
        assert g["measured_count"] == r[1], b
        assert g["mesh_power"].tolist() == r[2], b
        np.testing.assert_array_equal(measured_rows(*g["measured"]), r[3], err_msg=f"batch {b}")


def test_walk_grid_results_unchanged():
    """lpc_set_walk_grid is a launch policy: a trace under walk grids of 64,
    16 384 (TracePool's) and the default gives the same per-iteration counts,
    per-mesh power bits and measured rays; out-of-range grids are refused."""
    from lightpycl_amd._lib import LpcError
    from lightpycl_amd.engine import Engine
    from parity_util import measured_rows
    sc = scenes.BUILDERS["synthetic"](n=50000, seed=3)
    ls = sc.sources[0]
    o, d = np.asarray(ls.rays_origin, np.float32), np.asarray(ls.rays_dir, np.float32)
    p = np.asarray(ls.rays_power, np.float32).reshape(-1)
    thr = (1.0 - sc.tau) * float(np.sum(p, dtype=np.float64))
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        for bad in (-1, 63, (1 << 22) + 1):
            with pytest.raises(LpcError):
                e.set_walk_grid(bad)
        got = []
        for g in (0, 64, 16384, 0):
            e.set_walk_grid(g)
            e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
            st, (c, mp) = e.run_local(sc.iterations, thr)
            got.append(([int(x.n_in) for x in st], int(c), mp.tolist(), measured_rows(*e.fetch_measured())))
    finally:
        e.close()
    for g in got[1:]:
        assert g[0] == got[0][0] and g[1] == got[0][1] and g[2] == got[0][2]
        np.testing.assert_array_equal(g[3], got[0][3])
