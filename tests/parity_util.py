"""Shared comparison helpers for the parity tests (test infrastructure).

SURVEY.md section 8c states the fp32 tolerance of "matches the reference":
  * iteration 0-1, per ray: |dest diff|_inf <= 1e-6 * max_ray_len,
    |pow diff| / pow <= 1e-5, meas / isect-id mismatch <= 0.1 % of rays;
  * deeper iterations: per-iteration ray count relative diff <= 1e-3;
  * total measured power relative diff <= 1e-4;
  * angular histogram L1 relative diff <= 1e-3.
"""
from __future__ import annotations

import numpy as np

ID_MISMATCH = 1e-3
POW_RTOL = 1e-5
COUNT_RTOL = 1e-3
POWER_RTOL = 1e-4
HIST_L1 = 1e-3


def bounce_stats(a, b, max_ray_len):
    """Per-ray differences between two bounce output dicts (oracle.bounce layout).
    Discrete outputs are counted as mismatches; continuous ones are compared on the
    rays whose discrete outputs agree."""
    n = len(a["isect_mid"])
    disc = np.zeros(n, bool)
    for k in ("isect_mid", "isect_idx", "meas", "r_meas", "t_meas", "n1", "n2", "entering"):
        disc |= np.asarray(a[k]).reshape(-1) != np.asarray(b[k]).reshape(-1)
    same = ~disc
    out = dict(n=n, id_mismatch=int(disc.sum()))
    for k in ("dest", "r_dir", "t_dir"):
        x = np.asarray(a[k], np.float32)[same, :3]
        y = np.asarray(b[k], np.float32)[same, :3]
        out[k + "_maxabs"] = float(np.max(np.abs(x.astype(np.float64) - y))) if x.size else 0.0
        out[k + "_exact"] = float(np.mean(np.all(x == y, axis=1))) if x.size else 1.0
    # powers relative to the ray's own (post-dissipation) power, so that a child
    # carrying a near-zero share (R ~ 0) is not judged by its own tiny magnitude
    ref_pow = np.abs(np.asarray(b["pow"], np.float64).reshape(-1)[same])
    for k in ("pow", "r_pow", "t_pow"):
        x = np.asarray(a[k], np.float64).reshape(-1)[same]
        y = np.asarray(b[k], np.float64).reshape(-1)[same]
        den = np.maximum(np.maximum(np.abs(y), ref_pow), 1e-30)
        rel = np.abs(x - y) / den
        out[k + "_maxrel"] = float(rel.max()) if rel.size else 0.0
        out[k + "_exact"] = float(np.mean(x == y)) if x.size else 1.0
    out["all_exact"] = bool(out["id_mismatch"] == 0 and all(out[k] == 1.0 for k in out if k.endswith("_exact")))
    out["max_ray_len"] = float(max_ray_len)
    return out


def assert_bounce_within(st, what=""):
    """SURVEY.md section 8c per-ray tolerance."""
    tol = 1e-6 * st["max_ray_len"]
    assert st["id_mismatch"] <= ID_MISMATCH * st["n"], (what, st)
    assert st["dest_maxabs"] <= tol, (what, st)
    for k in ("pow_maxrel", "r_pow_maxrel", "t_pow_maxrel"):
        assert st[k] <= POW_RTOL, (what, k, st)
    # unit directions: the same 1e-5 relative bound as powers
    for k in ("r_dir_maxabs", "t_dir_maxabs"):
        assert st[k] <= 1e-5, (what, k, st)


def counts_within(a, b):
    if len(a) != len(b):
        return False
    return all(abs(x - y) <= COUNT_RTOL * max(y, 1) for x, y in zip(a, b))


def rel(a, b):
    a = float(a)
    b = float(b)
    return abs(a - b) / max(abs(b), 1e-300)


def hist_l1(H, Hr):
    H = np.asarray(H, np.float64)
    Hr = np.asarray(Hr, np.float64)
    return float(np.abs(H - Hr).sum() / max(np.abs(Hr).sum(), 1e-300))


def measured_rows(pos, pw, mesh):
    """Measured rays (x, y, z, power, hit mesh) as lexicographically sorted float64
    rows: aggregate mode keeps each iteration's rays in its coherence order, so
    the measured record is compared as a set, bit for bit."""
    r = np.concatenate([np.asarray(pos, np.float32)[:, :3].astype(np.float64),
                        np.asarray(pw, np.float32).reshape(-1, 1).astype(np.float64),
                        np.asarray(mesh).reshape(-1, 1).astype(np.float64)], axis=1)
    return r[np.lexsort(r.T[::-1])] if len(r) else r


def ref_aggregate(oracle_mod, bounce_fn, meshes, o4, d4, pw, iterations, tau, max_ray_len, ior_env):
    """The reference's host loop (oracle.trace_rays, iterative_tracer.py:241-391)
    over ``bounce_fn`` (the reference's own kernels, tests/ref_gpu.py):
    per-iteration populations, per-mesh measured power, measured rows."""
    meas = []
    _, info = oracle_mod.trace_rays(o4, d4, pw, meshes, iterations, tau, max_ray_len, ior_env,
                                    keep_results=False, bounce_fn=bounce_fn, measured_out=meas)
    if meas:
        pos = np.concatenate([m[0] for m in meas])
        p = np.concatenate([m[1] for m in meas])
        mm = np.concatenate([m[2] for m in meas])
    else:
        pos, p, mm = np.zeros((0, 4), np.float32), np.zeros(0, np.float32), np.zeros(0, np.int32)
    return list(info["counts"]), np.asarray(info["mesh_power"]), measured_rows(pos, p, mm)


def lib_aggregate(engine, iterations, threshold, reps=1):
    """liblpc's aggregate trace (lpc_trace_run, the bench's path) on the rays set
    on ``engine``: ``reps`` back-to-back traces (the last one's record), each
    required to give the same counts and per-mesh power bits."""
    first = None
    for _ in range(reps):
        engine.reset()
        stats, (cnt, mp) = engine.run_local(iterations, threshold)
        got = ([int(s.n_in) for s in stats], int(cnt), [float(x) for x in mp])
        assert first is None or got == first, "back-to-back traces differ"
        first = got
    pos, p, mm = engine.fetch_measured()
    assert first[1] == len(p)
    return first[0], np.asarray(first[2]), measured_rows(pos, p, mm)


def assert_aggregate_equal(lib, ref, what=""):
    """Bar for the aggregate paths: per-iteration counts identical; the measured
    rays bit for bit as a set (so their exactly rounded per-mesh sums,
    math.fsum, are identical too); per-mesh power within rtol 1e-12, or, for a
    mesh with more measured rays than 1e-12 / u = 9 007 terms, within the float64
    summation bound (n - 1) u of non-negative terms summed in another order
    (liblpc sums per 256-ray tile in traced order, the reference host loop in ray
    order): 4 M terms may differ by ~1e-12 relative by rounding alone."""
    import math
    assert lib[0] == ref[0], (what, lib[0], ref[0])
    assert lib[2].shape == ref[2].shape, (what, lib[2].shape, ref[2].shape)
    np.testing.assert_array_equal(lib[2], ref[2], err_msg=f"measured rays {what}")
    u = 2.0 ** -53
    mesh = ref[2][:, 4] if len(ref[2]) else np.zeros(0)
    for j in range(len(ref[1])):
        sel = ref[2][mesh == j, 3] if len(ref[2]) else np.zeros(0)
        exact = math.fsum(sel.tolist())
        nonneg = bool(np.all(sel >= 0))
        tol = max(1e-12, (len(sel) - 1) * u) if nonneg else 1e-12
        for name, v in (("liblpc", lib[1][j]), ("reference", ref[1][j])):
            assert abs(v - exact) <= tol * abs(exact) + 1e-300, (what, name, j, v, exact, len(sel))
        assert abs(lib[1][j] - ref[1][j]) <= 2 * tol * abs(exact) + 1e-300, (what, j, lib[1][j], ref[1][j])
