"""The drop-in's default results mode (iterative_tracer.py:335-355, :711-751):
per-iteration results tuples exported asynchronously into pinned host blocks
(lpc_trace_iterate_export), the stop test decided from the device's float64 sum
when the float32 sorted sum's bound allows (CL_Tracer._power_decision).

* the asynchronous export equals the synchronous one (lpc_trace_iterate with
  host pointers) bit for bit, in one chunk and in several;
* a tracer's earlier results stay intact while later traces reuse pinned blocks;
* a traced scene pickles and reloads bit for bit (pickle_results protocol 1).
Whole traces against the reference's own kernels: tests/test_ref_parity.py
(test_trace_vs_reference runs CL_Tracer in this mode)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rays(sc):
    o = np.asarray(sc.sources[0].rays_origin, np.float32)
    d = np.asarray(sc.sources[0].rays_dir, np.float32)
    p = np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1)
    return o, d, p


@pytest.mark.parametrize("chunk", [0, 7000])
def test_async_export_equals_sync_export(chunk):
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import Engine
    sc = scenes.lens(n=20000, seed=3)
    o, d, p = _rays(sc)
    outs = []
    for mode in ("sync", "async"):
        e = Engine(0)
        e.upload_meshes(sc.meshes)
        if chunk:
            e.set_chunk(chunk)
        e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
        its = []
        for i in range(6):
            if e.population() == 0:
                break
            if mode == "sync":
                st, ex = e.iterate(export=True)
            else:
                st, ex = e.iterate_export(with_origin=True)
            its.append((st.n_in, st.n_reflect, st.n_refract, st.power_next, ex))
        e.sync()
        outs.append([(a, b, c, pw, {k: np.array(v) for k, v in ex.items() if k != "next_pow"})
                     for a, b, c, pw, ex in its])
        e.close()
    s, a = outs
    assert len(s) == len(a) >= 3
    for (n0, r0, t0, p0, x0), (n1, r1, t1, p1, x1) in zip(s, a):
        assert (n0, r0, t0) == (n1, r1, t1)
        assert p0 == p1
        for k in ("origin", "dest", "pow", "meas"):
            np.testing.assert_array_equal(x0[k], x1[k], err_msg=k)


def test_results_survive_later_traces():
    from lightpycl_amd import scenes
    from lightpycl_amd.iterative_tracer import CL_Tracer
    sc = scenes.parabolic(n=30000, seed=2)
    tr = CL_Tracer(device=0)
    r1 = tr.iterative_tracer(sc.sources, sc.meshes, trace_iterations=4, max_ray_len=sc.max_ray_len)
    copy1 = [tuple(np.array(a) for a in t) for t in r1]
    for _ in range(3):                          # later traces recycle the pinned blocks no one holds
        tr.iterative_tracer(sc.sources, sc.meshes, trace_iterations=4, max_ray_len=sc.max_ray_len)
    for t, c in zip(r1, copy1):
        for a, b in zip(t, c):
            np.testing.assert_array_equal(a, b)
    assert [len(t[3]) for t in r1] == [len(t[3]) for t in tr.results]


def test_pickle_traced_scene_roundtrip(tmp_path):
    from lightpycl_amd import scenes
    from lightpycl_amd.iterative_tracer import CL_Tracer
    sc = scenes.lens(n=3000, seed=4)
    tr = CL_Tracer(device=0)
    res = tr.iterative_tracer(sc.sources, sc.meshes, trace_iterations=sc.iterations, max_ray_len=sc.max_ray_len)
    fname = tr.pickle_results(str(tmp_path / "traced.txt"))
    assert fname is not None
    tr2 = CL_Tracer.__new__(CL_Tracer)
    got = tr2.load_pickle_results(fname)
    assert len(got) == len(res)
    for a, b in zip(got, res):
        for x, y in zip(a, b):
            assert x.dtype == y.dtype and x.shape == y.shape
            np.testing.assert_array_equal(x, y)
    # the reloaded record gives the same measured rays
    tr2.results = got
    tr2._aggregate = False
    p0, w0 = tr.get_measured_rays()
    p1, w1 = tr2.get_measured_rays()
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(w0, w1)


def test_scene_upload_skipped_only_for_identical_bits():
    """A tracer called again on its meshes keeps the device scene (Engine.
    upload_arrays compares bit for bit with the last upload); a moved mesh, or a
    vertex whose only change is the sign of a zero, is uploaded again."""
    from lightpycl_amd import scenes
    from lightpycl_amd.engine import Engine, flatten_meshes
    sc = scenes.lens(n=4000, seed=5)
    o, d, p = _rays(sc)
    arrs = [np.array(a) for a in flatten_meshes(sc.meshes)]
    e = Engine(0)

    def trace(a):
        e.upload_arrays(*a)
        e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
        out = []
        while e.population() and len(out) < 4:
            st, ex = e.iterate(export=True)
            out.append((st.n_reflect, st.n_refract, ex["dest"].copy()))
        return out

    base = trace(arrs)
    kept = e._scene_last
    assert trace([a.copy() for a in arrs]) and e._scene_last is kept      # identical bits: no upload
    moved = [a.copy() for a in arrs]
    for k in range(3):
        moved[k][:, 0] += np.float32(0.25)
    got = trace(moved)
    assert e._scene_last is not kept
    assert any(not np.array_equal(x[2], y[2]) for x, y in zip(base, got))
    z = [a.copy() for a in arrs]
    zero = np.flatnonzero(z[0][:, 3] == 0)[0]
    z[0][zero, 3] = -0.0                                        # w: bits differ, value equal
    kept = e._scene_last
    trace(z)
    assert e._scene_last is not kept
    back = trace(arrs)
    for x, y in zip(base, back):
        assert x[:2] == y[:2]
        np.testing.assert_array_equal(x[2], y[2])
    e.close()
