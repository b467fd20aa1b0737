"""The conservative filter's superset property on the code the GPU runs.

tests/test_filter_superset.py checks it on a host (g++) build of lpc_math.hpp;
here the same adversarial (ray, record) pairs go through the device's own filter
paths (lpc_filter_eval -> k_filter_eval): the scalar test of the root-test
kernels, the packed-FP32 child tests of the walk (filter_test2, v_pk_fma_f32),
the packed test with the half-line cull (LPC_HALF 1/2) and the piece-root
half-line cull of k_roots* (LPC_HALF 3, the default).  Every pair the exact
Moller-Trumbore test accepts with t > eps must pass (d <= 0).

A trace with grazing secondaries -- reflected children that leave a flat cube
face almost along it, the class DESIGN.md section 3 names as the filter proof's
edge -- is compared with the reference's own kernels.
"""
import ctypes

import numpy as np
import pytest

from test_filter_superset import SO, adversarial

pytestmark = pytest.mark.gpu

MODES = {0: "filter_test", 1: "filter_test2 (packed)", 2: "filter_test2h (packed, half-line)",
         3: "filter_testh (piece-root half-line cull)"}


@pytest.fixture(scope="module")
def recs(harness):                       # harness fixture (test_filter_superset) builds the .so
    L = ctypes.CDLL(SO)
    P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    L.filt_records.argtypes = [ctypes.c_int, P, ctypes.c_double, ctypes.c_double, P]
    L.filt_records.restype = None
    L.node_rec.argtypes = [ctypes.c_int, P, ctypes.c_double, P]
    L.node_rec.restype = None

    def tri(V, S, dcap=16.0):
        out = np.zeros((V.shape[0], 5), np.float32)
        L.filt_records(V.shape[0], np.ascontiguousarray(V, np.float32), dcap, S, out)
        return out

    def node(V, S):
        out = np.zeros(5, np.float32)
        L.node_rec(V.shape[0], np.ascontiguousarray(V, np.float32), S, out)
        return out
    return tri, node


from test_filter_superset import harness  # noqa: E402,F401  (fixture)


def device_eval(engine, O, D, R, mode):
    n = O.shape[0]
    out = np.zeros(n, np.float32)
    p = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(ctypes.c_void_p)
    Oc, Dc, Rc = (np.ascontiguousarray(a, np.float32) for a in (O, D, R))
    engine._c(engine.L.lpc_filter_eval(engine.h, n, p(Oc), p(Dc), p(Rc), mode,
                                       out.ctypes.data_as(ctypes.c_void_p)))
    return out


@pytest.mark.parametrize("scale,dist,aspect,graze", [
    (1.0, 10.0, 1.0, 0.0), (1.0, 1000.0, 1.0, 0.0), (0.01, 100.0, 1.0, 0.0), (50.0, 1000.0, 1.0, 0.5),
    (1.0, 10.0, 100.0, 0.0), (1.0, 10.0, 1.0, 0.999), (1.0, 300.0, 30.0, 0.99), (0.02, 1.0, 10.0, 0.9),
    (0.05, 0.5, 3.0, 0.0), (1.0, 1e4, 1.0, 0.0)])
def test_device_filter_superset_triangles(engine, harness, recs, scale, dist, aspect, graze):
    rng = np.random.default_rng(int(scale * 1000 + dist + aspect * 7 + graze * 100) + 1)
    O, D, V = adversarial(rng, 200_000, scale, dist, aspect, graze, tiny_shift=1e-6)
    for S in (dist, 1e5):
        _, hit, _ = harness(O, D, V, eps=1e-6 * dist, S=S)
        assert hit.sum() > 1000
        R = recs[0](V, S)
        for mode in MODES:
            d = device_eval(engine, O, D, R, mode)
            lost = hit & ~(d <= 0)
            assert not lost.any(), f"{MODES[mode]} S={S}: {lost.sum()} exact hits rejected on the device"


@pytest.mark.parametrize("name", ["lens", "eye", "synthetic", "parabolic"])
def test_device_node_superset(engine, harness, recs, name):
    """Node / piece-root records (node_record of 64 consecutive triangles of the
    real meshes) on the device: a ray the exact test accepts against any of the
    node's triangles passes the node's test, in every mode."""
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import flatten_meshes
    sc = scenes.BUILDERS[name](n=8, seed=1)
    v0, v1, v2, *_ = flatten_meshes(sc.meshes)
    rng = np.random.default_rng(17)
    checked = 0
    for start in rng.choice(len(v0) - 64, 25, replace=False):
        V = np.concatenate([v0[start:start + 64, :3], v1[start:start + 64, :3], v2[start:start + 64, :3]], 1)
        V = V.astype(np.float32)
        j = rng.integers(0, 64, 4000)
        bu, bv = rng.random(4000), rng.random(4000)
        flip = bu + bv > 1
        bu[flip], bv[flip] = 1 - bu[flip], 1 - bv[flip]
        edge = rng.random(4000) < 0.3
        bv[edge] = 1 - bu[edge]
        tgt = V[j, :3] + bu[:, None] * (V[j, 3:6] - V[j, :3]) + bv[:, None] * (V[j, 6:9] - V[j, :3])
        O = (tgt + rng.normal(size=tgt.shape) * rng.choice([1e-2, 1.0, 1e2, 1e3], (4000, 1))).astype(np.float32)
        D = tgt - O
        D = (D / np.linalg.norm(D, axis=1, keepdims=True)).astype(np.float32)
        # exact acceptance (t > eps) of the aimed-at triangle, host build of the same arithmetic
        _, hit, _ = harness(O, D, V[j], eps=1e-6)
        for S in (1.0, 1e3):
            R = np.tile(recs[1](V, S), (len(O), 1))
            for mode in MODES:
                d = device_eval(engine, O, D, R, mode)
                assert not (hit & ~(d <= 0)).any(), (name, MODES[mode], S)
            checked += int(hit.sum())
    assert checked > 10000


def test_grazing_secondaries_match_reference(oracle_mod, exact_ref, monkeypatch):
    """Rays that meet the dissipative cube's bottom face (z = 15) at 1e-6 .. 1e-2
    rad: their reflected children start on the face and leave it almost along it.
    The drop-in trace (default LPC_HALF=3 root cull, hierarchy filters) gives the
    reference kernels' results tuples bit for bit, and so does LPC_HALF=0."""
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    from lightpycl_amd import scenes
    from lightpycl_amd.iterative_tracer import CL_Tracer
    sc = scenes.cube(n=8, seed=1)
    rng = np.random.default_rng(3)
    n = 20000
    eps_ang = 10.0 ** rng.uniform(-6, -2, n)
    hit_x = rng.uniform(-4.9, 4.9, n)
    hit_y = rng.uniform(-4.9, 4.9, n)
    back = rng.uniform(0.5, 30.0, n)                   # distance travelled before the face
    d = np.stack([np.ones(n), rng.normal(size=n) * 0.3, eps_ang], 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tgt = np.stack([hit_x, hit_y, np.full(n, 15.0)], 1)
    o = tgt - d * back[:, None]
    src = sc.sources[0]
    src.rays_origin = np.concatenate([o, np.zeros((n, 1))], 1).astype(np.float32)
    src.rays_dir = np.concatenate([d, np.zeros((n, 1))], 1).astype(np.float32)
    src.rays_power = np.full((n, 1), 1.0 / n, np.float32)
    want, info = oracle_mod.trace([src], sc.meshes, 6, sc.tau, sc.max_ray_len, sc.ior_env,
                                  bounce_fn=exact_ref.bounce)
    assert len(want) >= 2 and len(want[1][3]) > 1000      # grazing children were traced
    for half in ("3", "0"):
        monkeypatch.setenv("LPC_HALF", half)
        tr = CL_Tracer(device=0)
        got = tr.iterative_tracer(light_source=[src], meshes=sc.meshes, trace_iterations=6,
                                  trace_until_dissipated=sc.tau, max_ray_len=sc.max_ray_len, ior_env=sc.ior_env)
        assert [len(r[3]) for r in got] == info["counts"], half
        for it, (a, b) in enumerate(zip(got, want)):
            for k in range(4):
                x = a[k][:, :3] if a[k].ndim == 2 and a[k].shape[-1] == 4 else a[k]
                y = b[k][:, :3] if b[k].ndim == 2 and b[k].shape[-1] == 4 else b[k]
                np.testing.assert_array_equal(x, y, err_msg=f"LPC_HALF={half} it{it} field{k}")
