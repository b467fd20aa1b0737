"""CPU tests of the drop-in host API (light_source, geo_optical_elements,
iterative_tracer helpers) and of the C-ABI library surface (loads and exports
every symbol of include/lpc.h; no compute without a GPU)."""
import os
import re

import numpy as np
import pytest

from lightpycl_amd import geo_optical_elements as goe
from lightpycl_amd import light_source as lsrc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# -- light_source.py -----------------------------------------------------------
def test_random_rays_layout_and_rng_sequence():
    np.random.seed(123)
    ls = lsrc.light_source(center=np.array([1, 2, 3, 0], np.float32), direction=(0, 0, 1), power=5.0,
                           ray_count=1000)
    nxt = np.random.rand()
    np.random.seed(123)
    draws = np.random.rand(2001)
    assert nxt == draws[2000]                       # constructor draws u then v, N each
    assert np.asarray(ls.rays_origin).shape == (1000, 4) and np.asarray(ls.rays_origin).dtype == np.float32
    d = np.asarray(ls.rays_dir)
    assert d.shape == (1000, 4) and d.dtype == np.float32
    np.testing.assert_allclose(np.linalg.norm(d[:, :3], axis=1), 1.0, rtol=1e-6)
    assert np.all(d[:, 2] >= 0)                     # +z hemisphere
    assert np.isclose(np.sum(np.asarray(ls.rays_power, np.float64)), 5.0, rtol=1e-5)
    np.testing.assert_array_equal(np.asarray(ls.rays_origin)[0], np.float32([1, 2, 3, 0]))
    # directions are arccos(u) elevation, 2 pi v azimuth
    u, v = draws[:1000], draws[1000:2000]
    np.testing.assert_allclose(d[:, 2], np.cos(np.arccos(u)), atol=1e-6)


def test_direction_rotation():
    np.random.seed(0)
    ls = lsrc.light_source(direction=(0, 0, -1), ray_count=500)
    assert np.all(np.asarray(ls.rays_dir)[:, 2] <= 1e-6)
    np.random.seed(0)
    ls = lsrc.light_source(direction=(1, 0, 0), ray_count=500)
    # the reference rotates row vectors by Rx(elevation) then Rz(azimuth)
    # (light_source.py:136-137): with azimuth 0 the +z beam axis lands on +y
    assert np.all(np.asarray(ls.rays_dir)[:, 1] >= -1e-6)


def test_collimated_rays():
    np.random.seed(5)
    ls = lsrc.light_source(center=np.array([0, 0, -10, 0], np.float32), direction=(0, 0.01, 1),
                           directivity=lambda x, y: 1.0 + 0.0 * np.cos(y), power=1000., ray_count=400)
    ls.random_collimated_rays(diameter=5.0)
    o = np.asarray(ls.rays_origin)
    d = np.asarray(ls.rays_dir)
    assert o.shape == (400, 4) and o.dtype == np.float32 and d.dtype == np.float32
    assert np.allclose(d, d[0])                     # parallel
    assert np.ptp(o[:, 0]) <= 5.0 + 1e-4
    assert np.asarray(ls.rays_power).shape == (400,)
    assert np.isclose(np.sum(ls.rays_power, dtype=np.float64), 1000.0, rtol=1e-6)


# -- geo_optical_elements.py ---------------------------------------------------
def test_generators_triangle_counts_and_materials():
    oe = goe.optical_elements()
    h = oe.hemisphere(center=[0, 0, 0, 0], radius=10.0)
    assert len(h.triangles) == 2 * 71 * 73
    s = oe.sphere(center=[0, 0, 0, 0], radius=1.0)
    assert len(s.triangles) == 2 * 71 * 73
    c = oe.cube(center=(0, 0, 0, 0), size=[2, 2, 2, 0])
    assert len(c.triangles) == 12
    m = oe.parabolic_mirror(reflectivity=0.5)
    assert m.getMaterialBuf() == {"type": 1, "IOR": 1.0, "R": 1.0, "dissipation": 0.0}   # reference quirk
    c.setMaterial(mat_type="refractive", IOR=1.7, dissipation=0.5)
    assert c.getMaterialBuf() == {"type": 0, "IOR": 1.7, "R": 1.0, "dissipation": 0.5}
    c.setMaterial(mat_type="nonsense")
    assert c.getMaterialBuf()["type"] == 0


def test_tribuf_translate_rotate():
    oe = goe.optical_elements()
    c = oe.cube(center=(0, 0, 0, 0), size=[2, 2, 2, 0])
    v0, v1, v2 = c.tribuf()
    assert len(v0) == 12 and np.asarray(v0).shape == (12, 4)
    c.translate([1, 0, 0, 0])
    assert np.isclose(np.asarray(c.vertices)[:, 0].mean(), 1.0)
    c.rotate(axis="z", angle=np.pi / 2, pivot=(0, 0, 0, 0))
    vv = np.asarray(c.vertices)
    assert vv.dtype == np.float64 or vv.dtype == np.float32
    assert np.allclose(vv[:, 1].mean(), 1.0, atol=1e-6)         # x -> y
    assert np.all(vv[:, 3] == 0)


def test_flatten_matches_oracle_scene(oracle_mod):
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import flatten_meshes
    sc = scenes.eye(n=8, seed=1)
    v0, v1, v2, mid, mt, ior, refl, diss = flatten_meshes(sc.meshes)
    S = oracle_mod.Scene(sc.meshes)
    for a, b in ((v0, S.v0), (v1, S.v1), (v2, S.v2), (mid, S.mesh_id), (mt, S.mat_type), (ior, S.ior),
                 (refl, S.refl), (diss, S.diss)):
        np.testing.assert_array_equal(a, b)
    with pytest.raises(ValueError):
        flatten_meshes([])


# -- iterative_tracer host helpers -------------------------------------------------
def test_f32_sorted_sum_semantics():
    from lightpycl_amd.iterative_tracer import f32_sorted_sum
    rng = np.random.default_rng(0)
    a = rng.random(1000).astype(np.float32) * np.float32(1e3)
    ref = 0
    for x in np.sort(a):                        # builtin sum(np.sort(a)), as :372
        ref = ref + x
    assert f32_sorted_sum(a) == ref and np.asarray(ref).dtype == np.float32
    a2 = a.reshape(-1, 1)                        # (N,1): np.sort per row -> original order (:115)
    ref2 = 0
    for x in np.sort(a2):
        ref2 = ref2 + x
    assert f32_sorted_sum(a2) == ref2[0]
    assert f32_sorted_sum(np.zeros(0, np.float32)) == 0


# -- C ABI surface ---------------------------------------------------------------
def test_c_abi_exports_every_header_symbol():
    from lightpycl_amd import _lib
    from lightpycl_amd.build import build
    build(verbose=False)
    hdr = open(os.path.join(ROOT, "include", "lpc.h")).read()
    declared = set(re.findall(r"^(?:int|const char \*)\s*(lpc_\w+)\(", hdr, flags=re.M))
    assert len(declared) >= 20
    assert declared == set(_lib.EXPORTED)
    L = _lib.load()
    for name in declared:
        assert getattr(L, name) is not None
    assert L.lpc_abi_version() == 4


def test_c_abi_errors_without_device():
    import ctypes
    from lightpycl_amd import _lib
    L = _lib.load()
    if _lib.device_count() > 0:
        pytest.skip("a HIP device is present")
    h = ctypes.c_void_p()
    rc = L.lpc_open(0, ctypes.byref(h))
    assert rc != 0 and not h.value
    assert L.lpc_last_error(None)                 # message for the failed open
    assert L.lpc_close(None) == 0
    assert L.lpc_trace_reset(None) != 0


def test_pickle_results_protocol1_and_reference_module_names(tmp_path):
    """pickle_results writes (results, meshes) with protocol 1 as the reference
    (iterative_tracer.py:711-733); load_pickle_results reads it back and also a
    file naming the reference's own modules (geo_optical_elements, as a pickle
    written by the reference's Python 2 code does)."""
    import pickle

    import numpy as np
    from lightpycl_amd import scenes
    from lightpycl_amd.iterative_tracer import CL_Tracer
    sc = scenes.cube(n=16, seed=1)
    rng = np.random.default_rng(0)
    results = [(rng.random((16, 4)).astype(np.float32), rng.random((16, 4)).astype(np.float32),
                rng.random((16, 1)).astype(np.float32), rng.integers(-1, 2, 16).astype(np.int32))]
    tr = CL_Tracer.__new__(CL_Tracer)          # no GPU needed for the file format
    tr.results, tr.meshes, tr._aggregate = results, sc.meshes, False
    fname = tr.pickle_results(str(tmp_path / "r.txt"))
    raw = open(fname, "rb").read()
    assert raw[:1] != b"\x80"                   # protocol 1 has no PROTO opcode
    tr2 = CL_Tracer.__new__(CL_Tracer)
    tr2.load_pickle_results(fname)
    for a, b in zip(tr2.results[0], results[0]):
        np.testing.assert_array_equal(a, b)
    assert [len(m.tribuf()[0]) for m in tr2.meshes] == [len(m.tribuf()[0]) for m in sc.meshes]
    # the reference's module name in the GLOBAL opcodes
    ref_raw = raw.replace(b"clightpycl_amd.geo_optical_elements\n", b"cgeo_optical_elements\n")
    assert ref_raw != raw
    p2 = tmp_path / "ref.txt"
    p2.write_bytes(ref_raw)
    tr3 = CL_Tracer.__new__(CL_Tracer)
    tr3.load_pickle_results(str(p2))
    assert type(tr3.meshes[0]).__name__ == "GeoObject"
    with pytest.raises(Exception):
        pickle.loads(ref_raw)                   # a plain loader cannot resolve the reference's module
    # an aggregate-mode trace kept no per-ray results: no empty record is written
    tr4 = CL_Tracer.__new__(CL_Tracer)
    tr4.results, tr4.meshes, tr4._aggregate = [], sc.meshes, True
    with pytest.raises(ValueError):
        tr4.pickle_results(str(tmp_path / "agg.txt"))
    assert not (tmp_path / "agg.txt").exists()


def test_select_device_by_name(monkeypatch):
    """CL_Tracer(device_name=...) picks the HIP device as the reference's loop
    picks its OpenCL device (iterative_tracer.py:50-55): ordinal, substring of the
    name or gfx architecture (last match wins), no match -> the default device."""
    from lightpycl_amd.engine import select_device
    names = [("AMD Instinct MI355X", "gfx950:sramecc+:xnack-", 256)] * 4 + [("Other GPU", "gfx1100", 48)]
    monkeypatch.delenv("LPC_DEVICE", raising=False)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    assert select_device(3, names) == 3
    assert select_device("2", names) == 2
    assert select_device("770", names) == 0            # the reference's default string: no match
    assert select_device("gfx1100", names) == 4
    assert select_device("Other", names) == 4
    assert select_device("MI355", names) == 0         # the default device is among the matches
    monkeypatch.setenv("LOCAL_RANK", "2")
    assert select_device("MI355", names) == 2         # one process per GPU keeps its own
    assert select_device("Other", names) == 4
    monkeypatch.setenv("LOCAL_RANK", "4")
    assert select_device("gfx950", names) == 3        # default not among the matches: last match


def test_power_decision_bound():
    """The results-mode stop test (iterative_tracer.py:372, :383) decided from the
    device's float64 sum when the float32 sorted sum's error bound cannot cross
    the threshold; the bound holds on adversarial non-negative data."""
    import numpy as np
    from lightpycl_amd.iterative_tracer import CL_Tracer, f32_sorted_sum
    rng = np.random.default_rng(5)
    U = CL_Tracer._U32
    for n in (1, 10, 1000, 100000, 1000000):
        for kind in range(3):
            if kind == 0:
                x = rng.random(n).astype(np.float32)
            elif kind == 1:
                x = (rng.random(n) ** 8).astype(np.float32) * np.float32(1e-3)
            else:
                x = np.full(n, np.float32(1.0 + 2.0 ** -23))
            exact = float(np.sum(x, dtype=np.float64))
            f32 = float(f32_sorted_sum(x))
            if n * U <= 0.1:
                B = 1.2 * U * exact * (n + 1) / 2.0
                assert abs(f32 - exact) <= B, (n, kind, f32, exact, B)

    class St:
        pass

    class Eng:
        def __init__(self, p):
            self.p = p
            self.fetched = 0

        def population_power(self):
            self.fetched += 1
            return self.p

    p = rng.random(200000).astype(np.float32)
    S = float(np.sum(p, dtype=np.float64))
    tr = CL_Tracer.__new__(CL_Tracer)
    tr.engine = Eng(p)
    st = St()
    st.n_reflect, st.n_refract, st.power_next, st.power_nonneg = 150000, 50000, S, 1
    for thr in (np.float32(S * 0.5), np.float32(S * 1.5)):                  # far: no fetch
        v, stop = tr._power_decision(st, thr)
        assert stop == (f32_sorted_sum(p) < thr) and tr.engine.fetched == 0
    v, stop = tr._power_decision(st, np.float32(S))                          # near: exact, as the reference
    assert tr.engine.fetched == 1 and v == f32_sorted_sum(p) and stop == (v < np.float32(S))
    st.power_nonneg = 0                                                      # negative powers: always exact
    tr._power_decision(st, np.float32(S * 0.5))
    assert tr.engine.fetched == 2


def test_flatten_meshes_equals_tribuf_rows():
    """The drop-in's mesh flattening (iterative_tracer.py:121-151) gathers the
    triangles' vertex rows at once; bit for bit the rows of tribuf() converted to
    float32 as the reference does, on every scene builder's meshes."""
    import numpy as np
    from lightpycl_amd import engine, scenes
    for name, build in scenes.BUILDERS.items():
        sc = build(n=4)
        v0, v1, v2, mid, *_ = engine.flatten_meshes(sc.meshes)
        ref = [[], [], []]
        ids = []
        for j, m in enumerate(sc.meshes):
            tb = m.tribuf()
            for k in range(3):
                ref[k].append(np.array(tb[k], dtype=np.float32).reshape(-1, 4))
            ids.append(np.full(len(tb[0]), j, np.int32))
        for got, want in zip((v0, v1, v2), ref):
            want = np.concatenate(want)
            assert got.dtype == want.dtype and got.shape == want.shape, name
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), name
        assert np.array_equal(mid, np.concatenate(ids)), name


def test_pinned_pool_recycles_blocks(monkeypatch):
    """The results export's page-locked blocks (lightpycl_amd/pinned.py) return
    to the pool as soon as no numpy view of them is left (reference counting, no
    cyclic-GC pass needed), so repeated traces reuse them instead of pinning new
    memory."""
    import ctypes
    import gc

    import numpy as np
    from lightpycl_amd import _lib, pinned
    libc = ctypes.CDLL("libc.so.6")
    libc.malloc.restype = ctypes.c_void_p
    libc.free.argtypes = [ctypes.c_void_p]

    class FakeL:
        def lpc_host_alloc(self, size, pp):
            ctypes.cast(pp, ctypes.POINTER(ctypes.c_void_p))[0] = libc.malloc(size)
            return 0

        def lpc_host_free(self, p):
            libc.free(p)
            return 0

    monkeypatch.setattr(_lib, "load", lambda: FakeL())
    monkeypatch.setattr(_lib, "check", lambda rc, h: None)
    pool = pinned.PinnedPool()
    gc.disable()
    try:
        def trace():
            out = []
            for size in (24_000_000, 40_000_000):
                blk = pool.block(size)
                _ = ctypes.c_void_p(ctypes.addressof(blk))       # what the engine passes to the library
                out.append(pool.views(blk, [(np.float32, (1000, 4)), (np.int32, (1000,))]))
            return out
        res = trace()
        for _ in range(5):
            res = trace()
        assert pool.allocated == 4, pool.allocated              # two traces' blocks, then reuse
        assert res[1][0].shape == (1000, 4) and res[1][1].dtype == np.int32
    finally:
        gc.enable()


def test_tracer_flatten_cache_follows_the_meshes():
    """CL_Tracer reuses its last flatten only while the same mesh objects hold the
    same vertex / triangle bits and materials; any change flattens again."""
    import numpy as np
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import flatten_meshes
    from lightpycl_amd.iterative_tracer import CL_Tracer
    sc = scenes.parabolic(n=10)
    tr = CL_Tracer.__new__(CL_Tracer)
    a = tr._flatten(sc.meshes)
    assert tr._flatten(sc.meshes) is a

    def fresh_equal(x):
        return all(np.array_equal(p, q) and p.dtype == q.dtype for p, q in zip(x, flatten_meshes(sc.meshes)))
    sc.meshes[1].translate([0, 0, 1e-3, 0])                 # new vertex table
    b = tr._flatten(sc.meshes)
    assert b is not a and fresh_equal(b)
    v = sc.meshes[1].vertices
    v[0, 0] = np.nextafter(v[0, 0], np.inf)                 # in place, one ulp
    c = tr._flatten(sc.meshes)
    assert c is not b and fresh_equal(c)
    sc.meshes[1].setMaterial(mat_type="refractive", IOR=1.7)   # (a mirror keeps its reflectivity: the quirk)
    d = tr._flatten(sc.meshes)
    assert d is not c and fresh_equal(d)
    e = tr._flatten(sc.meshes[::-1])                        # other order
    assert e is not d
    assert all(np.array_equal(p, q) for p, q in zip(e, flatten_meshes(sc.meshes[::-1])))

