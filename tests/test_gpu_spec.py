"""Speculative trace iterations (lpc_trace_run, LPC_SPEC): iteration i + 1 is
enqueued device-sized -- its population size and the termination rule of
iterative_tracer.py:383-391 evaluated on the device by iteration i's
k_stage_move -- before the host reads iteration i's counters.  The prediction
(which iterations a trace reaches, their sizes) comes from the handle's
previous trace; whatever it predicts, the trace must be the host-sized trace
(LPC_SPEC=0) bit for bit: per-iteration counts and power, per-mesh power and
the measured record element by element.  Covered: repeated traces (the
speculation taken), a prediction of more iterations than the trace has (an
iteration that runs empty and is dropped), of fewer, and a Dcap overflow inside
a trace (the filter records are rebuilt and the speculative iteration re-runs
host-sized)."""
import numpy as np
import pytest

from lightpycl_amd import scenes

pytestmark = pytest.mark.gpu


def _rays(sc, flip=False, dscale=1.0):
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
    d = d.copy()
    if flip:
        d[:, :3] = -d[:, :3]
    if dscale != 1.0:
        d[:, :3] *= np.float32(dscale)
    return o, d, p


def _trace(e, sc, rays):
    o4, d4, pw = rays
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    e.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
    stats, (cnt, mp) = e.run_local(sc.iterations, thr)
    rec = e.fetch_measured()
    return ([(s.n_in, s.n_reflect, s.n_refract, s.n_measured, s.power_next) for s in stats], cnt, mp.tolist(), rec)


def _same(got, want):
    assert got[0] == want[0]
    assert got[1] == want[1]
    assert got[2] == want[2]
    for x, y in zip(got[3], want[3]):
        np.testing.assert_array_equal(x, y)


def _engine(monkeypatch, spec, sc):
    from lightpycl_amd.engine import Engine
    monkeypatch.setenv("LPC_SPEC", spec)
    e = Engine(0)
    e.upload_meshes(sc.meshes)
    return e


@pytest.mark.parametrize("name,n", [("synthetic", 100000), ("lens", 30000), ("eye", 4000), ("cube", 3000),
                                    ("nested_cubes", 2000), ("parabolic", 20000)])
def test_speculative_trace_equals_host_sized(monkeypatch, name, n):
    sc = scenes.BUILDERS[name](n=n, seed=51)
    rays = _rays(sc)
    a = _engine(monkeypatch, "0", sc)
    b = _engine(monkeypatch, "1", sc)
    try:
        want = _trace(a, sc, rays)
        assert len(want[0]) >= 2, "a multi-iteration trace"
        for _ in range(3):                 # the first builds the prediction, the others speculate
            _same(_trace(b, sc, rays), want)
    finally:
        a.close()
        b.close()


def test_speculation_mispredicted(monkeypatch):
    """Predicted more iterations than the trace has (rays leaving the scene end
    after one iteration) and fewer (the full trace after the short one)."""
    sc = scenes.synthetic(n=30000, seed=52)
    full, away = _rays(sc), _rays(sc, flip=True)
    a = _engine(monkeypatch, "0", sc)
    b = _engine(monkeypatch, "1", sc)
    try:
        want_full, want_away = _trace(a, sc, full), _trace(a, sc, away)
        assert len(want_away[0]) < len(want_full[0])
        for r, w in ((full, want_full), (full, want_full), (away, want_away), (full, want_full), (full, want_full),
                     (away, want_away)):
            _same(_trace(b, sc, r), w)
    finally:
        a.close()
        b.close()


def test_speculation_dcap_rebuild(monkeypatch):
    """Emitted directions of length 0.5 under a Dcap of 0.6 (LPC_DCAP_MILLI): the
    refracted children are longer, the records are rebuilt inside the trace while
    the next iteration is already queued (it runs empty and re-runs host-sized)."""
    monkeypatch.setenv("LPC_DCAP_MILLI", "600")
    sc = scenes.lens(n=20000, seed=53)
    rays = _rays(sc, dscale=0.5)
    a = _engine(monkeypatch, "0", sc)
    b = _engine(monkeypatch, "1", sc)
    try:
        want = _trace(a, sc, rays)
        assert len(want[0]) >= 3
        for _ in range(2):
            b.upload_meshes(sc.meshes)     # Dcap back to 0.6 (the trace before rebuilt the records)
            _same(_trace(b, sc, rays), want)
    finally:
        a.close()
        b.close()


def test_speculation_dcap_overflow_in_an_earlier_chunk(monkeypatch):
    """A chunked traced iteration whose kept children exceed Dcap only in a chunk
    before the last (the sphere hitters ordered first, 5 000-ray chunks), with the
    next iteration speculated device-sized: the device must stop that iteration
    on the whole iteration's max |D| (not the last chunk's), and a discarded
    iteration's measured power must not count.  The trace equals the host-sized
    one bit for bit."""
    from lightpycl_amd.engine import Engine
    monkeypatch.setenv("LPC_DCAP_MILLI", "600")
    sc = scenes.synthetic(n=60000, seed=54)
    o4, d4, pw = _rays(sc, dscale=0.5)
    probe = Engine(0)
    try:
        probe.upload_meshes(sc.meshes)
        z = np.zeros(len(pw), np.int32)
        g = probe.bounce(o4, d4, pw, z, np.full(len(pw), -2, np.int32), sc.max_ray_len, sc.ior_env)
    finally:
        probe.close()
    hits = np.asarray(g["isect_mid"]) > 0                 # a sphere (mesh 0 is the measure hemisphere)
    order = np.concatenate([np.where(hits)[0], np.where(~hits)[0]])
    assert 0 < hits.sum() < 5000
    rays = (o4[order], d4[order], pw[order])
    a = _engine(monkeypatch, "0", sc)
    b = _engine(monkeypatch, "1", sc)
    try:
        a.set_chunk(5000)
        b.set_chunk(5000)
        want = _trace(a, sc, rays)
        assert len(want[0]) >= 2
        for _ in range(3):                 # the first builds the prediction, the others speculate
            b.upload_meshes(sc.meshes)     # Dcap back to 0.6
            _same(_trace(b, sc, rays), want)
    finally:
        a.close()
        b.close()
