"""Parity against the REFERENCE's own kernels, run on the GPU.

``oracle/_ref/lpc_ref_{ieee,stock}.co`` is the unmodified
``/root/reference/kernel_reflect_refract_intersect.cl`` compiled for gfx950 with
ROCm's OpenCL C front end and device libraries (``oracle/Makefile`` target
``ref``); ``tests/ref_gpu.py`` launches it with the reference host's argument
lists (``iterative_tracer.py:288-326, 546``) and :func:`oracle.trace` drives it
with the reference's host loop (``:241-391``).

* ``ieee`` build (IEEE divide/sqrt, no contraction in the kernel's own
  expressions -- DESIGN.md section 2): liblpc is held BIT-EXACT, per ray at two
  bounce levels, whole traces (results tuples, counts, measured power),
  projections, and the bench's 1M-ray workload.  The CPU oracle is held to
  SURVEY.md section 8c's tolerance (it computes the hardware's rsqrt/sqrt
  correctly rounded and the C library's exp).
* ``stock`` build (OpenCL's default fp options: what PyOpenCL's
  ``Program(...).build()`` runs on an AMD GPU -- approximate divide, contracted
  multiply-adds): liblpc and the oracle within SURVEY.md section 8c's
  tolerances (``tests/parity_util.py``).

``LPC_REF_REPORT=path`` appends one JSON line per case (exact-match fractions).
"""
import json
import os

import numpy as np
import pytest

import ref_gpu
from parity_util import (HIST_L1, POWER_RTOL, assert_bounce_within, bounce_stats, counts_within, hist_l1, rel)
from lightpycl_amd import scenes

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not ref_gpu.available("stock"),
                                 reason="oracle/_ref not built (make -C oracle ref needs /root/reference)")]


def report(case, **kw):
    path = os.environ.get("LPC_REF_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(dict(case=case, **kw), default=float) + "\n")


@pytest.fixture(scope="module", params=ref_gpu.VARIANTS)
def ref(request):
    if not ref_gpu.available(request.param):
        pytest.skip(f"lpc_ref_{request.param}.co not built")
    r = ref_gpu.RefKernels(request.param)
    yield r
    r.close()


def rays_of(sc):
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
    return o, d, p


BOUNCE_SCENES = [("parabolic", 2000), ("lens", 2000), ("eye", 2000), ("cube", 2000), ("nested_cubes", 10),
                 ("synthetic", 4000)]


@pytest.mark.parametrize("name,n", BOUNCE_SCENES)
def test_bounce_two_levels_vs_reference(engine, oracle_mod, ref, name, n):
    """Per-ray outputs of one bounce (emitted rays) and of a second bounce (the
    reference's kept children, prev_mid >= 0): liblpc (exact against the ieee
    build) and the oracle against the reference kernels."""
    sc = scenes.BUILDERS[name](n=n, seed=3)
    o4, d4, pw = rays_of(sc)
    engine.upload_meshes(sc.meshes)
    S = oracle_mod.Scene(sc.meshes)
    meas = np.zeros(len(pw), np.int32)
    prev = np.full(len(pw), -2, np.int32)
    for level in (0, 1):
        r = ref.bounce(S, o4, d4, pw, meas, prev, sc.max_ray_len, sc.ior_env)
        g = engine.bounce(o4, d4, pw, meas, prev, sc.max_ray_len, sc.ior_env)
        c = oracle_mod.bounce(S, o4, d4, pw, meas, prev, sc.max_ray_len, sc.ior_env)
        for who, x in (("liblpc", g), ("oracle", c)):
            st = bounce_stats(x, r, sc.max_ray_len)
            report("bounce", scene=name, level=level, variant=ref.variant, who=who, **st)
            if who == "liblpc" and ref.variant == "ieee":
                assert st["all_exact"], (name, level, st)
            assert_bounce_within(st, f"{who} {name} level {level} {ref.variant}")
        keep = np.where(np.concatenate((r["r_meas"], r["t_meas"])) == 0)[0]
        if keep.size == 0:
            break
        o4 = np.concatenate((r["r_origin"], r["t_origin"]))[keep]
        d4 = np.concatenate((r["r_dir"], r["t_dir"]))[keep]
        pw = np.concatenate((r["r_pow"], r["t_pow"]))[keep]
        prev = np.concatenate((r["isect_mid"], r["isect_mid"]))[keep]
        meas = np.zeros(keep.size, np.int32)


TRACE_SCENES = [("parabolic", 3000), ("lens", 3000), ("eye", 3000), ("cube", 3000), ("nested_cubes", 10),
                ("synthetic", 5000)]


@pytest.mark.parametrize("name,n", TRACE_SCENES)
def test_trace_vs_reference(oracle_mod, ref, name, n):
    """Whole traces: the reference's host loop over the reference's kernels against
    the drop-in CL_Tracer (liblpc): the results tuples of every iteration,
    per-iteration ray counts, total measured power and the measured rays'
    angular histogram (the reference's angular_project kernel + np.histogram2d)."""
    from lightpycl_amd.iterative_tracer import CL_Tracer
    sc = scenes.BUILDERS[name](n=n, seed=5)
    want, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                                  bounce_fn=ref.bounce)
    tr = CL_Tracer(device=0)
    got = tr.iterative_tracer(light_source=sc.sources, meshes=sc.meshes, trace_iterations=sc.iterations,
                              trace_until_dissipated=sc.tau, max_ray_len=sc.max_ray_len, ior_env=sc.ior_env)
    gc = [len(r[3]) for r in got]
    pos, pwr = tr.get_measured_rays()
    rpos, rpwr = oracle_mod.measured_rays(want)
    P = float(np.sum(np.float64(pwr)))
    Pr = float(np.sum(np.float64(rpwr))) if rpwr is not None else 0.0
    l1 = 0.0
    if rpos is not None and len(rpwr):
        H = tr.get_binned_data_angular(limits=sc.hist_limits, points=sc.hist_points)[0]
        Hr = ref.binned_angular(rpos, rpwr, sc.hist_limits, sc.hist_points)[0]
        l1 = hist_l1(H, Hr)
    # per-iteration results tuples (origin, dest, pow, meas)
    same_iters = 0
    for a, b in zip(got, want):
        if (a[0].shape == b[0].shape and np.array_equal(a[0][:, :3], b[0][:, :3]) and
                np.array_equal(a[1][:, :3], b[1][:, :3]) and np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])):
            same_iters += 1
    o0, d0, p0, m0 = got[0]
    ro0, rd0, rp0, rm0 = want[0]
    meas_mis = int(np.sum(m0 != rm0))
    same = m0 == rm0
    dmax = float(np.max(np.abs(d0[same, :3].astype(np.float64) - rd0[same, :3]))) if same.any() else 0.0
    report("trace", scene=name, n=n, variant=ref.variant, counts=gc, ref_counts=info["counts"],
           power=P, ref_power=Pr, power_rel=rel(P, Pr) if Pr else abs(P), hist_l1=l1, it0_meas_mismatch=meas_mis,
           it0_dest_maxabs=dmax, identical_iterations=same_iters, iterations=len(want))
    if ref.variant == "ieee":                     # bit-exact: every results tuple, the measured rays
        assert gc == info["counts"]
        assert same_iters == len(want) == len(got)
        if rpos is not None:
            np.testing.assert_array_equal(pos[:, :3], rpos[:, :3])
            np.testing.assert_array_equal(np.asarray(pwr).reshape(-1), np.asarray(rpwr).reshape(-1))
        assert l1 <= 1e-12, l1
        return
    # the stock build: SURVEY.md section 8c tolerances.  The termination rule is a
    # threshold on the power left, so builds whose powers differ in the last bits
    # may stop one iteration apart (the eye, whose power left crosses 1 % between
    # iterations 10 and 11): counts are compared on the common prefix, and the
    # trace-end aggregates only when both stopped at the same iteration.
    k = min(len(gc), len(info["counts"]))
    assert abs(len(gc) - len(info["counts"])) <= 1, (gc, info["counts"])
    assert counts_within(gc[:k], info["counts"][:k]), (gc, info["counts"])
    if len(gc) == len(info["counts"]):
        if Pr:
            assert rel(P, Pr) <= POWER_RTOL, (P, Pr)
        else:
            assert P == 0.0
        assert l1 <= HIST_L1, l1
    assert meas_mis <= 1e-3 * len(m0)
    assert dmax <= 1e-6 * float(sc.max_ray_len)


def test_headline_workload_vs_reference(engine, oracle_mod, ref):
    """The bench's own workload at full size: 1M rays of scenes.synthetic(seed=7)
    over 103,660 triangles.  First bounce per ray (liblpc vs the reference
    kernels), then the whole trace's per-iteration counts and measured power
    (liblpc's device loop vs the reference's host loop over its kernels)."""
    sc = scenes.synthetic(n=1_000_000, seed=7)
    o4, d4, pw = rays_of(sc)
    engine.upload_meshes(sc.meshes)
    S = oracle_mod.Scene(sc.meshes)
    z = np.zeros(len(pw), np.int32)
    pm = np.full(len(pw), -2, np.int32)
    r = ref.bounce(S, o4, d4, pw, z, pm, sc.max_ray_len, sc.ior_env)
    g = engine.bounce(o4, d4, pw, z, pm, sc.max_ray_len, sc.ior_env)
    st = bounce_stats(g, r, sc.max_ray_len)
    report("headline_bounce", scene="synthetic", variant=ref.variant, who="liblpc", **st)
    if ref.variant == "ieee":
        assert st["all_exact"], st
    assert_bounce_within(st, "headline first bounce")
    _, info = oracle_mod.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                               keep_results=False, bounce_fn=ref.bounce)
    engine.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    stats, (cnt, mp) = engine.run_local(sc.iterations, thr)
    gc = [int(s.n_in) for s in stats]
    report("headline_trace", scene="synthetic", n=len(pw), variant=ref.variant, counts=gc,
           ref_counts=info["counts"], mesh_power=list(mp), ref_mesh_power=list(info["mesh_power"]))
    if ref.variant == "ieee":
        assert gc == info["counts"]
        np.testing.assert_allclose(mp, info["mesh_power"], rtol=1e-12)   # float64 summation order only
    assert counts_within(gc, info["counts"]), (gc, info["counts"])
    assert rel(mp.sum(), info["mesh_power"].sum()) <= POWER_RTOL


@pytest.mark.parametrize("mode", [0, 1])
def test_projection_vs_reference(engine, ref, mode):
    """angular_project / stereograph_project (.cl:488-538): liblpc's projection of
    measured-like points against the reference kernels, point by point (exact
    against the ieee build; the stock build's approximate divide moves points
    near the pole by up to ~1e-5 rad), and the binned histograms."""
    rng = np.random.default_rng(5)
    n = 20000
    v = rng.normal(size=(n, 3))
    v[:, 2] = np.abs(v[:, 2])
    v = v / np.linalg.norm(v, axis=1, keepdims=True) * 1000.0
    pos = np.zeros((n, 4), np.float32)
    pos[:, :3] = v
    pw = rng.random(n).astype(np.float32)
    lim = ((-np.pi / 2, np.pi / 2), (-np.pi / 2, np.pi / 2)) if mode == 0 else ((-1, 1), (-1, 1))
    H, xe, ye, x, y, pc = engine.project_hist(pos, pw, lim, 50, mode=mode, want_xy=True)
    rx, ry, rpc = ref.project(pos, pw, "angular" if mode == 0 else "stereo")
    report("project", mode=mode, variant=ref.variant, x_maxabs=float(np.max(np.abs(x - rx))),
           y_maxabs=float(np.max(np.abs(y - ry))), pc_maxrel=float(np.max(np.abs(pc - rpc) / np.abs(rpc))),
           x_exact=float(np.mean(x == rx)))
    if ref.variant == "ieee":
        np.testing.assert_array_equal(x, rx)
        np.testing.assert_array_equal(y, ry)
        np.testing.assert_array_equal(pc, rpc)
    else:
        np.testing.assert_allclose(x, rx, rtol=0, atol=1e-4)
        np.testing.assert_allclose(y, ry, rtol=0, atol=1e-4)
        np.testing.assert_allclose(pc, rpc, rtol=1e-5, atol=0)
    dx = np.float64(lim[0][1] - lim[0][0]) / 50
    Hr = np.histogram2d(rx, ry, bins=50, range=lim, weights=np.float64(rpc) / (dx * dx))[0]
    assert hist_l1(H, Hr) <= (1e-12 if ref.variant == "ieee" else HIST_L1)
