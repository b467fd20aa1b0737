"""GPU parity: liblpc (HIP, gfx950) against the reference's OWN kernels
(kernel_reflect_refract_intersect.cl compiled for gfx950, oracle/_ref, launched
by tests/ref_gpu.py; the `checker` fixture) on the same seeded inputs.

Bar (DESIGN.md "Parity"): every intersection decision, index, destination,
Fresnel child and power is BIT-EXACT against the reference kernels, and whole
traces (results tuples, counts, measured power) are identical.  Without the
reference code object the checker falls back to the CPU oracle, which differs
from the hardware only in gfx950's rsqrt / sqrt (<= 1 ulp, tools/rsq_check.py)
and the C library's exp / acos / atan2 / sin / cos: children directions and
powers then within a few ulp, decisions and destinations still exact.
"""
import ctypes
import json
import os

import numpy as np
import pytest

from lightpycl_amd import scenes

pytestmark = pytest.mark.gpu

# n >= 4096 runs the coherence-sorted path (k_raykey + radix sort + k_gather) and
# the work-list traversal on sorted packets; smaller n the unsorted packets.
SCENES = [("parabolic", 2000), ("lens", 2000), ("eye", 600), ("cube", 2000), ("nested_cubes", 10),
          ("synthetic", 700), ("synthetic", 20000), ("lens", 30000), ("eye", 12000), ("parabolic", 25000)]


def rays_of(sc):
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
    return o, d, p


def _ulps(a, b):
    a = np.asarray(a, np.float32).reshape(-1)
    b = np.asarray(b, np.float32).reshape(-1)
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7fffffff), ia)
    ib = np.where(ib < 0, -(ib & 0x7fffffff), ib)
    return np.abs(ia - ib)


def _cmp_bounce(g, o, exact=True):
    """exact: bit for bit (the reference kernels).  Otherwise (the CPU oracle):
    decisions and destinations bit for bit, children within the hardware
    rsqrt's ulp as it propagates through the Fresnel formulas."""
    for k in ("isect_mid", "n1", "n2", "r_meas", "t_meas", "meas"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    np.testing.assert_array_equal(g["isect_idx"], o["isect_idx"], err_msg="isect_idx")
    # no hit: the reference leaves its zeroed buffer (iterative_tracer.py:230), liblpc writes 0
    np.testing.assert_array_equal(g["entering"], o["entering"], err_msg="entering")
    np.testing.assert_array_equal(g["dest"][:, :3], o["dest"][:, :3], err_msg="dest")
    for k in ("r_dir", "t_dir", "pow", "r_pow", "t_pow"):
        a = g[k][:, :3] if g[k].ndim == 2 else g[k]
        b = o[k][:, :3] if o[k].ndim == 2 else o[k]
        if exact:
            np.testing.assert_array_equal(a, b, err_msg=k)
        else:
            assert np.all((_ulps(a, b) <= 64) | (np.abs(np.float64(a) - b) <= 1e-6 * np.abs(b).max())), k


@pytest.mark.parametrize("name,n", SCENES)
def test_bounce_bitexact_two_levels(engine, oracle_mod, checker, name, n):
    ref_bounce, exact = checker
    sc = scenes.BUILDERS[name](n=n, seed=3)
    o4, d4, pw = rays_of(sc)
    engine.upload_meshes(sc.meshes)
    S = oracle_mod.Scene(sc.meshes)
    meas = np.zeros(len(pw), np.int32)
    prev = np.full(len(pw), -2, np.int32)
    g = engine.bounce(o4, d4, pw, meas, prev, sc.max_ray_len, sc.ior_env)
    o = ref_bounce(S, o4, d4, pw, meas, prev, sc.max_ray_len, sc.ior_env)
    _cmp_bounce(g, o, exact)
    # second level: the oracle's kept children (prev_mid >= 0 exercises n1/n2 hand-over)
    keep = np.where(np.concatenate((o["r_meas"], o["t_meas"])) == 0)[0]
    if keep.size == 0:
        return
    o2 = np.concatenate((o["r_origin"], o["t_origin"]))[keep]
    d2 = np.concatenate((o["r_dir"], o["t_dir"]))[keep]
    p2 = np.concatenate((o["r_pow"], o["t_pow"]))[keep]
    m2 = np.concatenate((o["isect_mid"], o["isect_mid"]))[keep]
    z = np.zeros(keep.size, np.int32)
    g2 = engine.bounce(o2, d2, p2, z, m2, sc.max_ray_len, sc.ior_env)
    r2 = ref_bounce(S, o2, d2, p2, z, m2, sc.max_ray_len, sc.ior_env)
    _cmp_bounce(g2, r2, exact)


_POLICIES = [
    # the piece-root half-line cull off (LPC_HALF 0; 3 is the default)
    dict(LPC_HALF="0"),
    # work hand-over: budgets, queues that overflow (the wave carries on itself)
    dict(LPC_BUDGET="4"), dict(LPC_BUDGET="2", LPC_SPILL_CAP="100"), dict(LPC_BUDGET="0"),
    dict(LPC_BUDGET="0", LPC_HALF="0"), dict(LPC_BUDGET="3", LPC_SPILL_CAP="3000"),
    # no hand-over from 0 rays per triangle (always) / hand-over at every size
    dict(LPC_LARGE_PER_TRI="0"), dict(LPC_LARGE_PER_TRI="1000000", LPC_BUDGET="3"),
    # slivers on the side stream (k_slivers beside the walk) at every size; below
    # 4 M rays only; the default runs them in the walk's grid at every size
    dict(LPC_SLIVER_MERGE="-1"), dict(LPC_SLIVER_MERGE="-1", LPC_BUDGET="2", LPC_SPILL_CAP="100"),
    dict(LPC_SLIVER_MERGE="4000000"),
    # a filter-record rebuild below the emitted |D| (Dcap 0.5: unit directions exceed it)
    dict(LPC_DCAP_MILLI="500"),
]
@pytest.mark.parametrize("cfg", _POLICIES)
def test_launch_policies_bitexact(oracle_mod, checker, monkeypatch, cfg):
    """The size switches and test hooks that remain (the half-line cull,
    hand-over budgets and queues that overflow, merged sliver units, a record
    rebuild) change only speed: every bounce is bit-exact against the reference's
    kernels."""
    from lightpycl_amd.engine import Engine
    for k, v in cfg.items():
        monkeypatch.setenv(k, v)
    sc = scenes.synthetic(n=9000, seed=8)
    o4, d4, pw = rays_of(sc)
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        S = oracle_mod.Scene(sc.meshes)
        z = np.zeros(len(pw), np.int32)
        pm = np.full(len(pw), -2, np.int32)
        g = e.bounce(o4, d4, pw, z, pm, sc.max_ray_len, sc.ior_env)
        o = checker[0](S, o4, d4, pw, z, pm, sc.max_ray_len, sc.ior_env)
        _cmp_bounce(g, o, checker[1])
    finally:
        e.close()


@pytest.mark.parametrize("name,n", [("parabolic", 3000), ("lens", 3000), ("eye", 300), ("cube", 3000),
                                    ("nested_cubes", 10)])
def test_trace_results_match_reference(oracle_mod, exact_ref, name, n):
    """Whole traces, results tuples element for element: the drop-in CL_Tracer
    against the reference's host loop over the reference's kernels."""
    from lightpycl_amd.iterative_tracer import CL_Tracer
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    sc = scenes.BUILDERS[name](n=n, seed=5)
    ref, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                                 bounce_fn=exact_ref.bounce)
    tr = CL_Tracer(device=0)
    res = tr.iterative_tracer(light_source=sc.sources, meshes=sc.meshes, trace_iterations=sc.iterations,
                              trace_until_dissipated=sc.tau, max_ray_len=sc.max_ray_len, ior_env=sc.ior_env)
    assert [len(r[3]) for r in res] == info["counts"]
    assert tr.tri_count == info["tri_count"]
    for it, (a, b) in enumerate(zip(res, ref)):
        np.testing.assert_array_equal(a[0][:, :3], b[0][:, :3], err_msg=f"origin it{it}")
        np.testing.assert_array_equal(a[1][:, :3], b[1][:, :3], err_msg=f"dest it{it}")
        assert a[2].shape == b[2].shape and a[3].dtype == np.int32
        np.testing.assert_array_equal(a[3], b[3], err_msg=f"meas it{it}")
        np.testing.assert_array_equal(a[2], b[2], err_msg=f"pow it{it}")
    pos, pwr = tr.get_measured_rays()
    rpos, rpwr = oracle_mod.measured_rays(ref)
    np.testing.assert_array_equal(pos[:, :3], rpos[:, :3])
    np.testing.assert_array_equal(np.asarray(pwr).reshape(-1), np.asarray(rpwr).reshape(-1))


@pytest.mark.parametrize("name,n", [("parabolic", 4000), ("lens", 4000), ("synthetic", 1000)])
def test_aggregate_mode_and_histogram(oracle_mod, checker, exact_ref, name, n):
    from lightpycl_amd.iterative_tracer import CL_Tracer
    sc = scenes.BUILDERS[name](n=n, seed=11)
    ref, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                                 bounce_fn=checker[0])
    tr = CL_Tracer(device=0)
    tr.iterative_tracer(light_source=sc.sources, meshes=sc.meshes, trace_iterations=sc.iterations,
                        trace_until_dissipated=sc.tau, max_ray_len=sc.max_ray_len, ior_env=sc.ior_env,
                        keep_results=False)
    assert tr.iteration_counts == info["counts"]
    pos, pwr = tr.get_measured_rays()
    rpos, rpwr = oracle_mod.measured_rays(ref)
    # aggregate mode keeps each iteration's rays in the launch's coherence order
    # (DESIGN.md "traced order"): the same measured rays, bit for bit, as a set
    rpwr = np.asarray(rpwr).reshape(-1)

    def rows(p, w):
        r = np.concatenate([p[:, :3], w.reshape(-1, 1)], axis=1)
        return r[np.lexsort(r.T[::-1])]
    if checker[1]:
        np.testing.assert_array_equal(rows(pos, pwr), rows(np.asarray(rpos), rpwr))
    np.testing.assert_allclose(tr.measured_power(), info["mesh_power"], rtol=1e-12 if checker[1] else 1e-6)
    H, xe, ye = tr.get_binned_data_angular(limits=sc.hist_limits, points=sc.hist_points)
    if exact_ref is not None:       # the reference's angular_project kernel: identical bins
        Hr, xr, yr = exact_ref.binned_angular(rpos, rpwr, sc.hist_limits, sc.hist_points)
    else:
        Hr, xr, yr = oracle_mod.binned_angular(rpos, rpwr, limits=sc.hist_limits, points=sc.hist_points)
    np.testing.assert_array_equal(xe, xr)
    np.testing.assert_array_equal(ye, yr)
    l1 = np.abs(H - Hr).sum() / np.abs(Hr).sum()
    assert l1 <= (1e-12 if exact_ref is not None else 1e-5), l1


def test_chunked_trace_equals_unchunked(oracle_mod):
    from lightpycl_amd.engine import Engine
    sc = scenes.lens(n=5000, seed=2)
    o4, d4, pw = rays_of(sc)
    out = []
    for chunk in (0, 777):
        e = Engine(0)
        e.upload_meshes(sc.meshes)
        e.set_chunk(chunk)
        e.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
        its = []
        for _ in range(6):
            st, ex = e.iterate(export=True)
            its.append(ex)
        out.append((its, e.measured()))
        e.close()
    for a, b in zip(out[0][0], out[1][0]):
        for k in ("origin", "dest", "pow", "meas", "next_pow"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert out[0][1][0] == out[1][1][0]


def test_edge_cases(engine, oracle_mod, checker):
    sc = scenes.parabolic(n=1000, seed=4)
    engine.upload_meshes(sc.meshes)
    S = oracle_mod.Scene(sc.meshes)
    # empty population
    g = engine.bounce(np.zeros((0, 4), np.float32), np.zeros((0, 4), np.float32), np.zeros(0, np.float32),
                      np.zeros(0, np.int32), np.zeros(0, np.int32))
    assert g["dest"].shape == (0, 4)
    # single ray, ray along the axis, ray pointing away from every surface (no hit)
    o4 = np.array([[0, 0, 0, 0], [0, 0, 0, 0], [1e4, 1e4, 1e4, 0]], np.float32)
    d4 = np.array([[0, 0, -1, 0], [0.6, 0.0, 0.8, 0], [1, 0, 0, 0]], np.float32)
    pw = np.ones(3, np.float32)
    z = np.zeros(3, np.int32)
    pm = np.full(3, -2, np.int32)
    g = engine.bounce(o4, d4, pw, z, pm, sc.max_ray_len, sc.ior_env)
    o = checker[0](S, o4, d4, pw, z, pm, sc.max_ray_len, sc.ior_env)
    _cmp_bounce(g, o, checker[1])
    assert g["isect_mid"][2] == -1 and g["meas"][2] == -1
    # ragged count (not a multiple of the 512-ray block) and already-measured input rays
    rng = np.random.default_rng(0)
    n = 1237
    o4, d4, pw = rays_of(scenes.parabolic(n=n, seed=9))
    meas = rng.integers(-1, 2, n).astype(np.int32)
    pm = rng.integers(-2, 2, n).astype(np.int32)
    g = engine.bounce(o4, d4, pw, meas, pm, sc.max_ray_len, sc.ior_env)
    o = checker[0](S, o4, d4, pw, meas, pm, sc.max_ray_len, sc.ior_env)
    _cmp_bounce(g, o, checker[1])


def test_dropin_device_kernels(engine, oracle_mod, exact_ref):
    """lpc_intersect / lpc_intersect_postproc / lpc_reflect_refract_rays on device
    buffers in the reference's (n,4) and [ray][mesh] layouts."""
    torch = pytest.importorskip("torch")
    sc = scenes.eye(n=500, seed=6)
    engine.upload_meshes(sc.meshes)
    S = oracle_mod.Scene(sc.meshes)
    o4, d4, pw = rays_of(sc)
    n, K = len(pw), S.mesh_count
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    ref = exact_ref.bounce(S, o4, d4, pw, np.zeros(n, np.int32), np.full(n, -2, np.int32),
                           sc.max_ray_len, sc.ior_env)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    to, td = T(o4), T(d4)
    tmin = torch.full((n, K), float(sc.max_ray_len), dtype=torch.float32, device=dev)
    cnt = torch.zeros((n, K), dtype=torch.int32, device=dev)
    itmp = torch.zeros((n, K), dtype=torch.int32, device=dev)
    L, h = engine.L, engine.h
    P = lambda t: t.data_ptr()
    torch.cuda.synchronize()
    engine._c(L.lpc_intersect(h, n, P(to), P(td), np.float32(sc.max_ray_len), P(tmin), P(cnt), P(itmp)))
    np.testing.assert_array_equal(tmin.cpu().numpy(), ref["isect_min_ray_len"])
    np.testing.assert_array_equal(cnt.cpu().numpy(), ref["isects_count"])
    np.testing.assert_array_equal(itmp.cpu().numpy(), ref["isect_idx_tmp"])
    dest = torch.zeros((n, 4), dtype=torch.float32, device=dev)
    I = lambda: torch.zeros(n, dtype=torch.int32, device=dev)
    prev = T(np.full(n, -2, np.int32))
    n1, n2, ent, imid, iidx = I(), I(), I(), I(), I()
    engine._c(L.lpc_intersect_postproc(h, n, P(to), P(td), P(dest), P(prev), P(n1), P(n2), P(ent), P(imid),
                                       P(iidx), P(tmin), P(cnt), P(itmp), np.float32(sc.max_ray_len)))
    np.testing.assert_array_equal(dest.cpu().numpy()[:, :3], ref["dest"][:, :3])
    np.testing.assert_array_equal(imid.cpu().numpy(), ref["isect_mid"])
    tp, tm = T(pw.copy()), I()
    F4 = lambda: torch.zeros((n, 4), dtype=torch.float32, device=dev)
    ro, rd, to2, td2 = F4(), F4(), F4(), F4()
    rp, tpw = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    rm, tmm = I(), I()
    engine._c(L.lpc_reflect_refract_rays(h, n, P(to), P(dest), P(td), P(tp), P(tm), P(n1), P(n2), P(ro), P(rd),
                                         P(rp), P(rm), P(to2), P(td2), P(tpw), P(tmm), P(imid), P(iidx),
                                         np.float32(sc.ior_env)))
    np.testing.assert_array_equal(rd.cpu().numpy()[:, :3], ref["r_dir"][:, :3])
    np.testing.assert_array_equal(td2.cpu().numpy()[:, :3], ref["t_dir"][:, :3])
    np.testing.assert_array_equal(rp.cpu().numpy(), ref["r_pow"])
    np.testing.assert_array_equal(tm.cpu().numpy(), ref["meas"])


@pytest.mark.gpu
def test_trace_run_matches_host_loop(oracle_mod, checker):
    """lpc_trace_run (the loop in the library) gives the host loop's iterations,
    counts and measured power, and both match the oracle's trace."""
    from lightpycl_amd import scenes
    from lightpycl_amd.distributed import ShardedTrace
    from lightpycl_amd.engine import Engine
    sc = scenes.BUILDERS["lens"](n=6000, seed=3)
    o = np.asarray(sc.sources[0].rays_origin, np.float32)
    d = np.asarray(sc.sources[0].rays_dir, np.float32)
    p = np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1)
    in_pow = float(np.sum(p, dtype=np.float64))
    e = Engine(0)
    e.upload_meshes(sc.meshes)
    e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
    fast = ShardedTrace(e).run(sc.iterations, sc.tau, in_pow)
    fast_meas = e.measured()
    e.reset()

    class NoFast:                      # the same engine without run_local: host loop
        def __init__(self, eng):
            self.eng = eng

        def iterate(self):
            return self.eng.iterate()

        def measured(self):
            return self.eng.measured()

    slow = ShardedTrace(NoFast(e)).run(sc.iterations, sc.tau, in_pow)
    slow_meas = e.measured()
    assert fast["global_counts"] == slow["global_counts"]
    assert fast_meas[0] == slow_meas[0]
    np.testing.assert_array_equal(fast_meas[1], slow_meas[1])
    _, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                               keep_results=False, bounce_fn=checker[0])
    assert fast["global_counts"] == info["counts"]
    e.close()


@pytest.mark.parametrize("name,n,chunk", [("synthetic", 20000, 0), ("lens", 20000, 0), ("eye", 3000, 0),
                                          ("lens", 20000, 7000), ("eye", 6000, 5000), ("synthetic", 30000, 6000)])
def test_aggregate_trace_matches_reference_kernels(oracle_mod, exact_ref, name, n, chunk):
    """Aggregate iterations (traced order: the launch's coherence order, the
    default without per-ray export) against the reference's host loop over the
    reference's own kernels: identical per-iteration counts, per-mesh power to
    float64 summation order, the measured rays bit for bit as a set.  With a
    chunk size below the population the traced iterations run chunk by chunk
    (k_shade_stage + k_stage_move per chunk, running row bases, k_append of the
    staged refracted block)."""
    from parity_util import assert_aggregate_equal, lib_aggregate, ref_aggregate
    from lightpycl_amd.engine import Engine
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    sc = scenes.BUILDERS[name](n=n, seed=21)
    o4, d4, pw = rays_of(sc)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        e.set_chunk(chunk)
        e.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
        lib = lib_aggregate(e, sc.iterations, thr, reps=2)
    finally:
        e.close()
    ref = ref_aggregate(oracle_mod, exact_ref.bounce, sc.meshes, o4, d4, pw, sc.iterations, sc.tau, sc.max_ray_len,
                        sc.ior_env)
    assert_aggregate_equal(lib, ref, f"{name} {n} chunk {chunk}")


def test_clean_slots_across_paths(oracle_mod):
    """Traced iterations leave the slot arrays clean instead of resetting them;
    traces after a per-ray export (which dirties them), a bounce on the same
    handle and a new max_ray_len must still match a fresh handle's trace."""
    from lightpycl_amd.engine import Engine
    sc = scenes.lens(n=20000, seed=31)
    o4, d4, pw = rays_of(sc)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))

    def trace(e, mrl):
        e.set_rays(o4, d4, pw, mrl, sc.ior_env)
        stats, (cnt, mp) = e.run_local(sc.iterations, thr)
        return [(s.n_in, s.n_reflect, s.n_refract, s.n_measured) for s in stats], cnt, mp

    fresh = []
    for mrl in (sc.max_ray_len, np.float32(sc.max_ray_len * 0.75)):
        e = Engine(0)
        e.upload_meshes(sc.meshes)
        fresh.append(trace(e, mrl))
        e.close()
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        a = trace(e, sc.max_ray_len)
        e.reset()
        e.iterate(export=True)                      # reference-order iteration (slots dirty)
        e.iterate()
        b = trace(e, sc.max_ray_len)
        z = np.zeros(len(pw), np.int32)
        e.bounce(o4, d4, pw, z, np.full(len(pw), -2, np.int32), sc.max_ray_len, sc.ior_env)
        c = trace(e, np.float32(sc.max_ray_len * 0.75))
        d = trace(e, sc.max_ray_len)
    finally:
        e.close()
    for got, want in ((a, fresh[0]), (b, fresh[0]), (c, fresh[1]), (d, fresh[0])):
        assert got[0] == want[0] and got[1] == want[1]
        np.testing.assert_array_equal(got[2], want[2])


@pytest.mark.parametrize("name,n", [("synthetic", 100000), ("lens", 30000)])
def test_async_trace_run_equals_sync(name, n):
    """lpc_trace_run_async returns once the trace's outputs are final and lets
    the next trace queue behind its last row moves: back-to-back async traces
    give the synchronous trace's stats and per-mesh power, and the measured
    record read afterwards (the entry point waits for the stream) is the same
    element for element, also through the power-only copy."""
    from lightpycl_amd.engine import Engine
    sc = scenes.BUILDERS[name](n=n, seed=41)
    o4, d4, pw = rays_of(sc)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        e.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
        stats, (cnt, mp) = e.run_local(sc.iterations, thr)
        want = ([(s.n_in, s.n_reflect, s.n_refract, s.n_measured, s.power_next) for s in stats], cnt, mp.tolist())
        rec = e.fetch_measured()
        for rep in range(3):
            e.reset()
            stats, (cnt, mp) = e.run_local(sc.iterations, thr, wait=False)
            got = ([(s.n_in, s.n_reflect, s.n_refract, s.n_measured, s.power_next) for s in stats], cnt, mp.tolist())
            assert got == want
        p = np.zeros(cnt, np.float32)
        e._c(e.L.lpc_trace_fetch_measured(e.h, None, p.ctypes.data_as(ctypes.c_void_p), None))
        np.testing.assert_array_equal(p, rec[1])
        e.reset()
        e.run_local(sc.iterations, thr, wait=False)
        for x, y in zip(e.fetch_measured(), rec):
            np.testing.assert_array_equal(x, y)
        # lpc_trace_rerun_async: the reset and the asynchronous trace in one call
        for rep in range(3):
            stats, (cnt, mp) = e.run_local(sc.iterations, thr, wait=False, reset=True)
            got = ([(s.n_in, s.n_reflect, s.n_refract, s.n_measured, s.power_next) for s in stats], cnt, mp.tolist())
            assert got == want
        for x, y in zip(e.fetch_measured(), rec):
            np.testing.assert_array_equal(x, y)
        e.sync()
    finally:
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,n", [("synthetic", 200000), ("lens", 50000), ("eye", 30000), ("same", 5000),
                                    ("beam", 60000)])
def test_emitted_sort_paths_match_reference(oracle_mod, exact_ref, name, n):
    """The emitted rays' coherence sort takes the counting sort (k_bkey /
    k_bprefix / k_bscatter / k_bsort2, key windows of <= 16 bits: a point source's
    16 direction bits, a collimated beam's 15 origin-cell bits, one 8-bit level
    when nothing varies) or rocPRIM's radix sort (a narrow beam's few origin
    cells): either way the trace equals the reference kernels' (counts, per-mesh
    power, measured rays as a set), twice back to back (the digit counts of the
    first trace must not leak into the second)."""
    from parity_util import assert_aggregate_equal, lib_aggregate, ref_aggregate
    from lightpycl_amd.engine import Engine
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    if name == "same":                      # every ray identical: one 8-bit level
        sc = scenes.lens(n=10, seed=3)
        o4, d4, pw = rays_of(sc)
        o4 = np.repeat(o4[:1], n, axis=0)
        d4 = np.repeat(d4[:1], n, axis=0)
        pw = np.repeat(pw[:1], n)
    elif name == "beam":                    # one direction, origins all over the scene box: 15 origin bits
        sc = scenes.lens(n=10, seed=3)
        v = np.concatenate([np.asarray(m.vertices, np.float32).reshape(-1, 4)[:, :3] for m in sc.meshes])
        rng = np.random.default_rng(5)
        o4 = np.zeros((n, 4), np.float32)
        o4[:, :3] = rng.uniform(v.min(0), v.max(0), (n, 3)).astype(np.float32)
        d4 = np.tile(np.array([[0.0, 0.0, 1.0, 0.0]], np.float32), (n, 1))
        pw = np.ones(n, np.float32)
    else:
        sc = scenes.BUILDERS[name](n=n, seed=29)
        o4, d4, pw = rays_of(sc)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        e.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
        lib = lib_aggregate(e, sc.iterations, thr, reps=2)
    finally:
        e.close()
    ref = ref_aggregate(oracle_mod, exact_ref.bounce, sc.meshes, o4, d4, pw, sc.iterations, sc.tau, sc.max_ray_len,
                        sc.ior_env)
    assert_aggregate_equal(lib, ref, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,env", [
    # chained populations re-sorted (LPC_RESORT_MIN lowered from 2 M rays) against
    # kept in their parents' traced order (re-sort off)
    ("lens", 30000, dict(LPC_RESORT_MIN="1000")), ("eye", 3000, dict(LPC_RESORT_MIN="1000")),
    ("lens", 30000, dict(LPC_RESORT_MIN="1000000000000")), ("eye", 3000, dict(LPC_RESORT_MIN="1000000000000")),
    # every iteration of the dense scene re-sorted and keyed in its population's box
    ("synthetic_dense", 20000, dict(LPC_RESORT_MIN="4096")),
    # the gather with the root tests fused in, on re-sorted populations too
    ("synthetic", 200000, dict(LPC_RESORT_MIN="20000")), ("eye", 30000, dict(LPC_RESORT_MIN="20000")),
    ("synthetic_dense", 60000, dict(LPC_RESORT_MIN="20000")),
    # written-slot masks over K = 10 and K = 12 meshes, three traces back to back
    ("synthetic", 50000, dict()), ("nested_cubes", 2000, dict()),
])
def test_population_paths_match_reference(oracle_mod, exact_ref, monkeypatch, name, n, env):
    """The population paths (re-sort of chained populations and its 5-D Morton
    key in the population's own box, k_gather_roots, written-slot masks across
    back-to-back traces) against the reference kernels' trace: identical counts,
    per-mesh power to float64 summation order, measured rays as a set."""
    from parity_util import assert_aggregate_equal, lib_aggregate, ref_aggregate
    from lightpycl_amd.engine import Engine
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    kw = dict(iterations=8) if name == "synthetic_dense" else {}
    sc = scenes.BUILDERS[name](n=n, seed=31, **kw)
    o4, d4, pw = rays_of(sc)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        e.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
        lib = lib_aggregate(e, sc.iterations, thr, reps=3)
    finally:
        e.close()
    ref = ref_aggregate(oracle_mod, exact_ref.bounce, sc.meshes, o4, d4, pw, sc.iterations, sc.tau, sc.max_ray_len,
                        sc.ior_env)
    assert len(ref[0]) >= 3
    assert_aggregate_equal(lib, ref, f"{name} {env}")


@pytest.mark.parametrize("cfg", [dict(), dict(LPC_SLIVER_MERGE="4000000"), dict(LPC_SLIVER_MERGE="-1"),
                                 dict(LPC_SLIVER_MERGE="-1", LPC_RESORT_MIN="4096"), dict(LPC_RESORT_MIN="4096")])
def test_eye_results_mode_policies_match_reference(oracle_mod, exact_ref, monkeypatch, cfg):
    """The eye (thin triangles on the sliver path), results mode: every results
    tuple element for element equals the reference host loop over the
    reference's kernels, with the sliver units merged into the walk's grid at
    every size (the default) / from 4 M rays / never, and re-sorted chained
    populations."""
    from lightpycl_amd.iterative_tracer import CL_Tracer
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    for k, v in cfg.items():
        monkeypatch.setenv(k, v)
    sc = scenes.eye(n=3000, seed=6)
    ref, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                                 bounce_fn=exact_ref.bounce)
    tr = CL_Tracer(device=0)
    res = tr.iterative_tracer(light_source=sc.sources, meshes=sc.meshes, trace_iterations=sc.iterations,
                              trace_until_dissipated=sc.tau, max_ray_len=sc.max_ray_len, ior_env=sc.ior_env)
    assert [len(r[3]) for r in res] == info["counts"] and len(res) >= 3
    for it, (a, b) in enumerate(zip(res, ref)):
        for k, (x, y) in enumerate(zip(a, b)):
            x, y = np.asarray(x), np.asarray(y)
            if x.ndim == 2 and x.shape[1] == 4:
                x, y = x[:, :3], y[:, :3]
            np.testing.assert_array_equal(x, y, err_msg=f"it{it} field{k} {cfg}")


# The default paths that switch on only for large populations, whole traces
# under the DEFAULT policy (no threshold overrides) against the reference host
# loop over the reference's own kernels (iterative_tracer.py:241-391,
# .cl:243-474): the eye's populations pass 2 M (re-sort, k_gather_roots on
# re-sorted populations) and 4 M rays (merged sliver units) and 16 rays per
# triangle (no hand-over); the dense synthetic layout is the scene the
# population-box key was tuned on; a chunk size below the population runs the
# multi-chunk traced compaction (k_stage_move per chunk, k_append).
@pytest.mark.gpu
@pytest.mark.parametrize("name,n,chunk", [("eye", 100000, 0), ("synthetic_dense", 300000, 0),
                                          ("eye", 30000, 1000000), ("synthetic_dense", 100000, 700000)])
def test_large_population_defaults_match_reference(oracle_mod, exact_ref, name, n, chunk):
    from parity_util import assert_aggregate_equal, lib_aggregate, ref_aggregate
    from lightpycl_amd.engine import Engine
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    sc = scenes.BUILDERS[name](n=n, seed=43)
    o4, d4, pw = rays_of(sc)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    e = Engine(0)
    try:
        e.upload_meshes(sc.meshes)
        e.set_chunk(chunk)
        e.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
        lib = lib_aggregate(e, sc.iterations, thr, reps=1)
    finally:
        e.close()
    ref = ref_aggregate(oracle_mod, exact_ref.bounce, sc.meshes, o4, d4, pw, sc.iterations, sc.tau, sc.max_ray_len,
                        sc.ior_env)
    pops = ref[0]
    if chunk == 0 and name == "eye":
        assert max(pops) > 4_000_000, pops          # re-sort (2 M) and merged sliver units (4 M) engaged
    if chunk:
        assert max(pops) > chunk, pops              # some iteration ran in several chunks
    with open(os.path.join(os.environ.get("LPC_TEST_OUT", "/tmp"), "large_population_parity.jsonl"), "a") as f:
        f.write(json.dumps(dict(scene=name, rays=n, chunk=chunk, populations=pops, bounces=int(sum(pops)),
                                measured=int(len(ref[2])), mesh_power=[float(x) for x in ref[1]],
                                identical=True)) + "\n")
    assert_aggregate_equal(lib, ref, f"{name} {n} chunk {chunk}")
