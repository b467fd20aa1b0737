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
