"""The hot loop only runs the exact Moller-Trumbore test on pairs its bounding-sphere
filter accepts, so the filter must accept EVERY pair the exact test accepts (else a
hit would be lost).  This checks that superset property on adversarial inputs --
edge/vertex grazing hits, nearly parallel rays, far origins, slivers, large and
tiny triangles -- with the filter evaluated from the same header the kernel uses
(lightpycl_amd/csrc/lpc_math.hpp) compiled for the host."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "csrc", "_build", "libfilter_harness.so")


@pytest.fixture(scope="module")
def harness():
    src = os.path.join(ROOT, "tests", "csrc", "filter_harness.cpp")
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(
            os.path.getmtime(src), os.path.getmtime(os.path.join(ROOT, "lightpycl_amd", "csrc", "lpc_math.hpp"))):
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "lightpycl_amd", "csrc"), src, "-o", SO], check=True)
    L = ctypes.CDLL(SO)
    P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
    L.filt_eval.argtypes = [ctypes.c_int, P, P, P, ctypes.c_float, ctypes.c_double, P, I, P]
    L.filt_eval.restype = None

    def run(O, D, V, eps, dcap=16.0):
        n = O.shape[0]
        d = np.zeros(n, np.float32)
        h = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        L.filt_eval(n, np.ascontiguousarray(O, np.float32), np.ascontiguousarray(D, np.float32),
                    np.ascontiguousarray(V, np.float32), np.float32(eps), dcap, d, h, t)
        return d, h.astype(bool), t
    return run


def adversarial(rng, n, scale, dist, aspect, graze, tiny_shift):
    """Triangles of size `scale` (aspect = sliver factor) at distance `dist` from the ray
    origin; rays aimed at points on/near the triangle boundary; `graze` tilts the ray
    toward the triangle plane."""
    c = rng.normal(size=(n, 3)) * dist
    e1 = rng.normal(size=(n, 3))
    e1 /= np.linalg.norm(e1, axis=1, keepdims=True)
    nrm = rng.normal(size=(n, 3))
    nrm -= (nrm * e1).sum(1, keepdims=True) * e1
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    e2 = np.cross(nrm, e1)
    a = scale * (0.2 + rng.random((n, 1)))
    b = a / aspect
    v0 = c
    v1 = c + a * e1
    v2 = c + b * e2 + a * rng.random((n, 1)) * e1
    # target: barycentric point on an edge or a vertex, jittered by ~tiny_shift
    u = rng.random((n, 1))
    w = rng.random((n, 1))
    pick = rng.integers(0, 4, (n, 1))
    bu = np.where(pick == 0, u, np.where(pick == 1, 0.0, np.where(pick == 2, 1 - w, w * 0.0 + u)))
    bv = np.where(pick == 0, 0.0, np.where(pick == 1, u, np.where(pick == 2, w, 1 - u)))
    tgt = v0 + bu * (v1 - v0) + bv * (v2 - v0) + rng.normal(size=(n, 3)) * tiny_shift * scale
    # direction: mostly toward the target, optionally tilted into the plane (grazing)
    o = tgt - rng.normal(size=(n, 3)) * 0 - (nrm * rng.choice([-1, 1], (n, 1)) * (1 - graze) +
                                              e1 * graze + e2 * graze * rng.normal(size=(n, 1))) * dist
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    V = np.concatenate([v0, v1, v2], axis=1)
    return o.astype(np.float32), d.astype(np.float32), V.astype(np.float32)


@pytest.mark.parametrize("scale,dist,aspect,graze", [
    (1.0, 10.0, 1.0, 0.0), (1.0, 1000.0, 1.0, 0.0), (0.01, 100.0, 1.0, 0.0), (50.0, 1000.0, 1.0, 0.5),
    (1.0, 10.0, 100.0, 0.0), (1.0, 10.0, 1.0, 0.999), (1.0, 300.0, 30.0, 0.99), (0.02, 1.0, 10.0, 0.9), (0.05, 0.5, 3.0, 0.0),
    (1.0, 1e4, 1.0, 0.0)])
def test_filter_is_superset_of_exact(harness, scale, dist, aspect, graze):
    rng = np.random.default_rng(int(scale * 1000 + dist + aspect * 7 + graze * 100))
    O, D, V = adversarial(rng, 200_000, scale, dist, aspect, graze, tiny_shift=1e-6)
    d, hit, t = harness(O, D, V, eps=1e-6 * dist)
    assert hit.sum() > 1000                     # the cases do exercise accepted hits
    lost = hit & ~(d <= 0)
    assert not lost.any(), f"{lost.sum()} exact hits rejected by the filter"


def test_filter_rejects_most_far_misses(harness):
    """Sanity: the margin is not so large that the filter accepts everything."""
    rng = np.random.default_rng(1)
    O, D, V = adversarial(rng, 50_000, 1.0, 100.0, 1.0, 0.0, tiny_shift=20.0)
    d, hit, _ = harness(O, D, V, eps=1e-3)
    assert (d <= 0).mean() < 0.5


def test_degenerate_triangles_never_candidates(harness):
    """Zero-edge triangles (revolve_curve poles) can never be hit and are culled."""
    rng = np.random.default_rng(2)
    n = 10_000
    p = rng.normal(size=(n, 3)).astype(np.float32)
    q = rng.normal(size=(n, 3)).astype(np.float32)
    V = np.concatenate([p, q, p], axis=1)      # E2 == 0
    O = np.zeros((n, 3), np.float32)
    D = (p / np.linalg.norm(p, axis=1, keepdims=True)).astype(np.float32)
    d, hit, _ = harness(O, D, V, eps=1e-3)
    assert not hit.any() and (d > 0).all()


@pytest.fixture(scope="module")
def cluster_harness(harness):
    L = ctypes.CDLL(SO)
    P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    L.cluster_eval.argtypes = [ctypes.c_int, P, P, ctypes.c_int, P, ctypes.c_double, P, P]
    L.cluster_eval.restype = None

    def run(O, D, V, dcap=16.0):
        n, m = O.shape[0], V.shape[0]
        dt = np.zeros(n * m, np.float32)
        dc = np.zeros(n, np.float32)
        L.cluster_eval(n, np.ascontiguousarray(O, np.float32), np.ascontiguousarray(D, np.float32), m,
                       np.ascontiguousarray(V, np.float32), dcap, dt, dc)
        return dt.reshape(n, m), dc
    return run


@pytest.mark.parametrize("name", ["lens", "eye", "synthetic", "parabolic"])
def test_cluster_test_implied_by_member_tests(cluster_harness, name):
    """Every ray whose test passes for some triangle of a 64-triangle cluster must
    pass the cluster's test (k_intersect skips the cluster's triangles otherwise).
    Clusters are consecutive triangles of the real scenes' meshes; rays are aimed
    at those triangles from near and far origins."""
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import flatten_meshes
    sc = scenes.BUILDERS[name](n=8, seed=1)
    v0, v1, v2, mid, *_ = flatten_meshes(sc.meshes)
    rng = np.random.default_rng(7)
    checked = 0
    for start in rng.choice(len(v0) - 64, 40, replace=False):
        V = np.concatenate([v0[start:start + 64, :3], v1[start:start + 64, :3], v2[start:start + 64, :3]], 1)
        j = rng.integers(0, 64, 2000)
        bu, bv = rng.random(2000), rng.random(2000)
        flip = bu + bv > 1
        bu[flip], bv[flip] = 1 - bu[flip], 1 - bv[flip]
        tgt = V[j, :3] + bu[:, None] * (V[j, 3:6] - V[j, :3]) + bv[:, None] * (V[j, 6:9] - V[j, :3])
        tgt += rng.normal(size=tgt.shape) * np.abs(V).max() * 1e-3
        O = (tgt + rng.normal(size=tgt.shape) * rng.choice([1e-2, 1.0, 1e2, 1e3], (2000, 1))).astype(np.float32)
        D = (tgt - O)
        D /= np.linalg.norm(D, axis=1, keepdims=True)
        dt, dc = cluster_harness(O, D.astype(np.float32), V.astype(np.float32))
        tri_pass = (dt <= 0).any(axis=1)
        assert not (tri_pass & ~(dc <= 0)).any()
        checked += int(tri_pass.sum())
    assert checked > 10000
