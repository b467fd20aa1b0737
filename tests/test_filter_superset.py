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
    L.filt_eval.argtypes = [ctypes.c_int, P, P, P, ctypes.c_float, ctypes.c_double, ctypes.c_double, P, I, P]
    L.filt_eval.restype = None

    def run(O, D, V, eps, dcap=16.0, S=1000.0):
        n = O.shape[0]
        d = np.zeros(n, np.float32)
        h = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        L.filt_eval(n, np.ascontiguousarray(O, np.float32), np.ascontiguousarray(D, np.float32),
                    np.ascontiguousarray(V, np.float32), np.float32(eps), dcap, S, d, h, t)
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
    # the per-record split h depends on the assumed scene scale S; every S must hold
    for S in (dist, 1.0, 1e5):
        d, hit, t = harness(O, D, V, eps=1e-6 * dist, S=S)
        assert hit.sum() > 1000                 # the cases do exercise accepted hits
        lost = hit & ~(d <= 0)
        assert not lost.any(), f"S={S}: {lost.sum()} exact hits rejected by the filter"


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
    I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
    L.cluster_eval.argtypes = [ctypes.c_int, P, P, ctypes.c_int, P, ctypes.c_float, ctypes.c_double, I, P]
    L.cluster_eval.restype = None

    def run(O, D, V, eps, S=1000.0):
        n, m = O.shape[0], V.shape[0]
        ht = np.zeros(n * m, np.int32)
        dc = np.zeros(n, np.float32)
        L.cluster_eval(n, np.ascontiguousarray(O, np.float32), np.ascontiguousarray(D, np.float32), m,
                       np.ascontiguousarray(V, np.float32), np.float32(eps), S, ht, dc)
        return ht.reshape(n, m).astype(bool), dc
    return run


@pytest.mark.parametrize("name", ["lens", "eye", "synthetic", "parabolic"])
def test_node_test_passes_for_every_accepted_triangle(cluster_harness, name):
    """Every ray whose line the exact test accepts against some triangle of a
    64-triangle node must pass the node's test (the walk skips the node's
    triangles otherwise).  Nodes are consecutive triangles of the real scenes'
    meshes; rays are aimed at those triangles (and their edges) from near and far
    origins, including grazing ones."""
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
        edge = rng.random(2000) < 0.3
        bv[edge] = 1 - bu[edge]                    # on the far edge
        tgt = V[j, :3] + bu[:, None] * (V[j, 3:6] - V[j, :3]) + bv[:, None] * (V[j, 6:9] - V[j, :3])
        O = (tgt + rng.normal(size=tgt.shape) * rng.choice([1e-2, 1.0, 1e2, 1e3], (2000, 1))).astype(np.float32)
        D = (tgt - O)
        D /= np.linalg.norm(D, axis=1, keepdims=True)
        for S in (1.0, 1e3):
            ht, dc = cluster_harness(O, D.astype(np.float32), V.astype(np.float32), 1e-6, S=S)
            acc = ht.any(axis=1)
            assert not (acc & ~(dc <= 0)).any()
            checked += int(acc.sum())
    assert checked > 10000


@pytest.fixture(scope="module")
def sliver_harness(harness):
    L = ctypes.CDLL(SO)
    P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
    L.sliver_eval.argtypes = [ctypes.c_int, P, P, P, ctypes.c_float, ctypes.c_int, P, I, P]
    L.sliver_eval.restype = None
    L.filt_class.argtypes = [ctypes.c_int, P, ctypes.c_double, ctypes.c_double, I]
    L.filt_class.restype = None

    def run(O, D, V, eps, fused):
        n = O.shape[0]
        d = np.zeros(n, np.float32)
        h = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        L.sliver_eval(n, np.ascontiguousarray(O, np.float32), np.ascontiguousarray(D, np.float32),
                      np.ascontiguousarray(V, np.float32), np.float32(eps), int(fused), d, h, t)
        return d, h.astype(bool), t

    def classify(V, dcap=16.0, S=1000.0):
        c = np.zeros(V.shape[0], np.int32)
        L.filt_class(V.shape[0], np.ascontiguousarray(V, np.float32), dcap, S, c)
        return c
    run.classify = classify
    return run


def _scene_slivers(sliver_harness, name):
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import flatten_meshes
    sc = scenes.BUILDERS[name](n=8, seed=1)
    v0, v1, v2, *_ = flatten_meshes(sc.meshes)
    V = np.concatenate([v0[:, :3], v1[:, :3], v2[:, :3]], 1).astype(np.float32)
    return V[sliver_harness.classify(V) == 2]


def _rays_at_lines(rng, V, n, dist):
    """Rays aimed at points on (or 1e-7 relative off) the infinite line through V0
    along E2 -- where Moller-Trumbore's rounding noise accepts pairs of a sliver."""
    j = rng.integers(0, V.shape[0], n)
    v0 = V[j, :3].astype(np.float64)
    e2 = V[j, 6:9].astype(np.float64) - v0
    s = rng.uniform(-3, 3, (n, 1))
    tgt = v0 + s * e2 + rng.normal(size=(n, 3)) * 1e-7 * np.abs(V[j]).max(1, keepdims=True)
    o = tgt + rng.normal(size=(n, 3)) * dist[:, None]
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o.astype(np.float32), d.astype(np.float32), V[j]


@pytest.mark.parametrize("name", ["synthetic", "eye", "lens"])
@pytest.mark.parametrize("fused", [0, 1])
def test_sliver_line_filter_is_superset(sliver_harness, name, fused):
    """Triangles whose sphere test degenerates (revolve_curve's pole slivers: two
    vertices ~1e-11 apart) are tested with the line filter; every pair the exact test
    accepts -- including rounding-noise accepts anywhere along the sliver's line --
    must pass it."""
    V = _scene_slivers(sliver_harness, name)
    if V.shape[0] == 0:
        pytest.skip("scene has no slivers")
    rng = np.random.default_rng(11 + fused)
    n = 400_000
    dist = rng.choice([1e-2, 1.0, 30.0, 1e3], n)
    O, D, Vj = _rays_at_lines(rng, V, n, dist)
    d, hit, _ = sliver_harness(O, D, Vj, 1e-3, fused)
    if name == "synthetic" and fused == 0:
        # noise accepts do occur (r = 1000 pole slivers; rarer with the OpenCL
        # library's fused dot/cross than with unfused products, but present)
        assert hit.sum() > 0
    assert not (hit & ~(d <= 0)).any()
    # random directions from the same origins: the line filter rejects nearly all
    Dr = rng.normal(size=D.shape).astype(np.float32)
    d2, hit2, _ = sliver_harness(O, Dr, Vj, 1e-3, fused)
    assert not (hit2 & ~(d2 <= 0)).any()
    assert (d2 <= 0).mean() < 0.05                # and the filter still rejects pairs


def test_sliver_line_filter_synthetic_thin(sliver_harness):
    """Random thin triangles (aspect 1e4 .. 1e12) that filter_record routes to the
    sliver list; rays aimed along their lines and at their interiors."""
    rng = np.random.default_rng(5)
    m = 5000
    v0 = rng.normal(size=(m, 3)) * 100
    e = rng.normal(size=(m, 3))
    e /= np.linalg.norm(e, axis=1, keepdims=True)
    perp = np.cross(e, rng.normal(size=(m, 3)))
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    L = rng.uniform(0.1, 100, (m, 1))
    h = L * 10.0 ** rng.uniform(-12, -4, (m, 1))
    v1 = v0 + L * e
    v2 = v0 + L * e * rng.uniform(0, 1, (m, 1)) + h * perp
    V = np.concatenate([v0, v1, v2], 1).astype(np.float32)
    V = V[sliver_harness.classify(V) == 2]
    assert V.shape[0] > 1000
    n = 400_000
    dist = rng.choice([1e-1, 10.0, 1e3], n)
    O, D, Vj = _rays_at_lines(rng, V, n, dist)
    for fused in (0, 1):
        d, hit, _ = sliver_harness(O, D, Vj, 1e-3, fused)
        assert hit.sum() > 100
        assert not (hit & ~(d <= 0)).any()


@pytest.fixture(scope="module")
def thin_harness(harness):
    L = ctypes.CDLL(SO)
    P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
    L.sliver_eval_axis.argtypes = [ctypes.c_int, P, P, P, ctypes.c_float, ctypes.c_int, ctypes.c_int, P, I]
    L.sliver_eval_axis.restype = None
    L.thin_class.argtypes = [ctypes.c_int, P, ctypes.c_double, ctypes.c_double, ctypes.c_double, I]
    L.thin_class.restype = None

    def run(O, D, V, eps, fused, ax1):
        n = O.shape[0]
        d = np.zeros(n, np.float32)
        h = np.zeros(n, np.int32)
        L.sliver_eval_axis(n, np.ascontiguousarray(O, np.float32), np.ascontiguousarray(D, np.float32),
                           np.ascontiguousarray(V, np.float32), np.float32(eps), int(fused), int(ax1), d, h)
        return d, h.astype(bool)

    def classify(V, S, k=1.0, dcap=16.0):
        c = np.zeros(V.shape[0], np.int32)
        L.thin_class(V.shape[0], np.ascontiguousarray(V, np.float32), dcap, S, k, c)
        return c
    run.classify = classify
    return run


def _scene_box_half_diag(V):
    P = V.reshape(-1, 3).astype(np.float64)
    return 0.5 * float(np.linalg.norm(P.max(0) - P.min(0)))


def test_thin_rule_picks_the_lens_discs_only(thin_harness):
    """LPC_THIN: the eye's crystalline lens holds a disc of 144 long thin triangles
    through the optical axis (its two arcs are joined across the axis), whose
    bounding spheres every axial ray passes; those take the line filter.  The
    sphere meshes of the synthetic, parabolic and lens scenes keep their sphere
    tests."""
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import flatten_meshes
    for name, lo, hi in (("eye", 144, 400), ("synthetic", 0, 0), ("parabolic", 0, 0), ("lens", 0, 0)):
        sc = scenes.BUILDERS[name](n=8, seed=1)
        v0, v1, v2, mid, *_ = flatten_meshes(sc.meshes)
        V = np.concatenate([v0[:, :3], v1[:, :3], v2[:, :3]], 1).astype(np.float32)
        c = thin_harness.classify(V, _scene_box_half_diag(V))
        n_thin = int((c > 0).sum())
        assert lo <= n_thin <= hi, (name, n_thin)
        if name == "eye":
            assert ((c > 0) & (mid == 2)).sum() >= 144


def _rays_at_triangles(rng, V, n, dist, graze=0.0):
    """Rays aimed at points inside / on the edges of the triangles V (rows), from
    origins ~dist away, optionally tilted toward the triangle plane."""
    j = rng.integers(0, V.shape[0], n)
    v0, v1, v2 = (V[j, 3 * k:3 * k + 3].astype(np.float64) for k in range(3))
    bu, bv = rng.random((2, n, 1))
    f = bu + bv > 1
    bu[f], bv[f] = 1 - bu[f], 1 - bv[f]
    edge = rng.random((n, 1)) < 0.3
    bv = np.where(edge, 0.0, bv)
    # 20 %: a vertex (the far vertex lies exactly at the line filter's width),
    # jittered by a few ulps of the coordinates
    vert = rng.random((n, 1)) < 0.2
    k = rng.integers(0, 3, (n, 1))
    bu = np.where(vert, (k == 1).astype(float), bu)
    bv = np.where(vert, (k == 2).astype(float), bv)
    tgt = v0 + bu * (v1 - v0) + bv * (v2 - v0)
    tgt = tgt + np.where(vert, rng.normal(size=(n, 3)) * 1e-7 * np.abs(v0).max(1, keepdims=True), 0.0)
    nrm = np.cross(v1 - v0, v2 - v0)
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-300)
    tang = (v1 - v0) / np.maximum(np.linalg.norm(v1 - v0, axis=1, keepdims=True), 1e-300)
    o = tgt + (nrm * (1 - graze) + tang * graze * rng.normal(size=(n, 1)) +
               rng.normal(size=(n, 3)) * 0.3) * dist[:, None]
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o.astype(np.float32), d.astype(np.float32), V[j]


@pytest.mark.parametrize("fused", [0, 1])
def test_thin_line_filter_is_superset(thin_harness, fused):
    """Every pair Moller-Trumbore accepts passes the line filter about the edge the
    thin rule picks (E1 via the v-test, E2 via the u-test): the eye's thin triangles
    and random thin triangles (aspect 3 .. 1e4, long edge as E1 or E2), rays at their
    interiors, edges and at grazing angles."""
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import flatten_meshes
    rng = np.random.default_rng(21 + fused)
    sc = scenes.eye(n=8, seed=1)
    v0, v1, v2, *_ = flatten_meshes(sc.meshes)
    Ve = np.concatenate([v0[:, :3], v1[:, :3], v2[:, :3]], 1).astype(np.float32)
    ce = thin_harness.classify(Ve, _scene_box_half_diag(Ve))
    m = 6000
    p0 = rng.normal(size=(m, 3)) * 50
    e = rng.normal(size=(m, 3))
    e /= np.linalg.norm(e, axis=1, keepdims=True)
    perp = np.cross(e, rng.normal(size=(m, 3)))
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    L = rng.uniform(0.01, 100, (m, 1))
    w = L / 10.0 ** rng.uniform(0.5, 4, (m, 1))
    pa, pb = p0 + L * e, p0 + L * e * rng.uniform(0, 1, (m, 1)) + w * perp
    long1 = rng.random(m) < 0.5                 # long edge = E1 (v1 - v0) or E2 (v2 - v0)
    Vr = np.where(long1[:, None], np.concatenate([p0, pa, pb], 1), np.concatenate([p0, pb, pa], 1))
    for V, ax in ((Ve[ce > 0], ce[ce > 0]), (Vr.astype(np.float32), np.where(long1, 2, 1))):
        for k in (1, 2):
            Vk = V[ax == k]
            if len(Vk) == 0:
                continue
            for graze in (0.0, 0.9, 0.999):
                n = 200_000
                dist = rng.choice([1e-2, 1.0, 30.0, 1e3], n)
                O, D, Vj = _rays_at_triangles(rng, Vk, n, dist, graze)
                d, hit = thin_harness(O, D, Vj, 1e-6, fused, k == 2)
                assert hit.sum() > 1000
                assert not (hit & ~(d <= 0)).any(), (k, graze)


@pytest.fixture(scope="module")
def packet_harness(harness):
    L = ctypes.CDLL(SO)
    P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    Q = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
    L.packet_eval.argtypes = [ctypes.c_int, P, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, ctypes.c_double,
                              ctypes.c_double, Q]
    L.packet_eval.restype = None

    def run(O, D, V, kind, pk=128, dcap=16.0, S=1000.0):
        out = np.zeros(4, np.int64)
        L.packet_eval(O.shape[0], np.ascontiguousarray(O, np.float32), np.ascontiguousarray(D, np.float32), pk,
                      V.shape[0], np.ascontiguousarray(V, np.float32), kind, dcap, S, out)
        return dict(violations=int(out[0]), packet_pass=int(out[1]), ray_pass=int(out[2]), incoherent=int(out[3]))
    return run


def _packets(rng, V, npk, ball, dist, spread, line=False):
    """npk packets of 128 rays: origins in a ball of radius `ball` around a point at
    ~`dist` from a target triangle (or sliver line), directions toward points on /
    near it with angular jitter `spread`."""
    O, D = [], []
    for _ in range(npk):
        j = rng.integers(0, V.shape[0])
        v0, v1, v2 = (V[j, 3 * k:3 * k + 3].astype(np.float64) for k in range(3))
        if line:
            tgt = v0 + rng.uniform(-3, 3, (128, 1)) * (v2 - v0)
        else:
            bu, bv = rng.random((2, 128, 1))
            f = bu + bv > 1
            bu[f], bv[f] = 1 - bu[f], 1 - bv[f]
            tgt = v0 + bu * (v1 - v0) + bv * (v2 - v0)
        c = tgt.mean(0) + rng.normal(size=3) * dist
        o = c + rng.normal(size=(128, 3)) * ball
        d = tgt - o
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        d += rng.normal(size=d.shape) * spread
        O.append(o)
        D.append(d)
    return np.concatenate(O).astype(np.float32), np.concatenate(D).astype(np.float32)


@pytest.mark.parametrize("name", ["lens", "synthetic", "eye"])
@pytest.mark.parametrize("ball,dist,spread", [(0.0, 100.0, 1e-3), (1e-3, 30.0, 1e-2), (1.0, 10.0, 0.05),
                                              (30.0, 500.0, 1e-4), (0.0, 1e3, 0.0), (5.0, 2.0, 0.3)])
def test_packet_tests_are_sound(packet_harness, sliver_harness, name, ball, dist, spread):
    """The sliver tests skip a cluster / triangle / sliver for a whole wave when the
    packet bound of its 128 rays (origin ball + direction cone, k_packet) fails the
    record's packet test; that must never happen while some ray of the packet passes
    the record's per-ray test."""
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import flatten_meshes
    sc = scenes.BUILDERS[name](n=8, seed=1)
    v0, v1, v2, *_ = flatten_meshes(sc.meshes)
    V = np.concatenate([v0[:, :3], v1[:, :3], v2[:, :3]], 1).astype(np.float32)
    cls = sliver_harness.classify(V)
    rng = np.random.default_rng(int(ball * 7 + dist + spread * 1000))
    start = rng.integers(0, max(1, V.shape[0] - 4096))
    Vn = V[start:start + 4096][cls[start:start + 4096] == 0]
    O, D = _packets(rng, Vn, 60, ball, dist, spread)
    for kind in (0, 1):
        r = packet_harness(O, D, Vn, kind)
        assert r["violations"] == 0, r
        assert r["ray_pass"] > 0
        if kind == 0 and ball <= 1e-3:                 # the packet test does cull
            assert r["packet_pass"] < max(2 * r["ray_pass"], 0.5 * len(Vn) * 60), r
    Vs = V[cls == 2]
    if len(Vs):
        O, D = _packets(rng, Vs, 60, ball, dist, spread, line=True)
        r = packet_harness(O, D, Vs, 2)
        assert r["violations"] == 0, r


@pytest.mark.parametrize("name", ["synthetic", "eye", "lens", "parabolic"])
def test_sliver_dmin_bounds_den(harness, sliver_harness, name):
    """SliverRec::dmin: below it |D| is too short for Moller-Trumbore's float DEN
    (plain or FMA-contracted) to reach the 1e-6 threshold, so a launch whose rays
    are all shorter skips the sliver (k_slivers).  Random directions scaled to just
    under dmin never reach it; the bound is within a small factor of the real noise."""
    V = _scene_slivers(sliver_harness, name)
    if V.shape[0] == 0:
        pytest.skip("scene has no slivers")
    L = ctypes.CDLL(SO)
    P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    L.sliver_den.argtypes = [ctypes.c_int, P, P, P, P, P]
    L.sliver_den.restype = None
    rng = np.random.default_rng(17)
    n = 300_000
    j = rng.integers(0, V.shape[0], n)
    Vj = np.ascontiguousarray(V[j], np.float32)
    D = rng.normal(size=(n, 3))
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    dmin = np.zeros(n, np.float32)
    a = np.zeros(n, np.float32)
    b = np.zeros(n, np.float32)
    L.sliver_den(n, np.ascontiguousarray(D, np.float32), Vj, dmin, a, b)   # dmin per row
    fin = np.isfinite(dmin)
    assert fin.any()
    Ds = np.ascontiguousarray(D * (np.where(fin, dmin, 1.0) * 0.9999)[:, None], np.float32)
    L.sliver_den(n, Ds, Vj, dmin, a, b)
    eps6 = np.float32(0.000001)
    assert not (fin & ((np.abs(a) >= eps6) | (np.abs(b) >= eps6))).any()
    # the noise at dmin is a real fraction of the threshold (the bound is not vacuous)
    assert np.max(np.abs(np.concatenate([a[fin], b[fin]]))) > 1e-3 * eps6
