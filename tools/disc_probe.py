"""Plane-test probe (tools/disc_probe.cpp): on the chained populations of the
bench scenes (made by the CPU oracle's bounce, iterative_tracer.py:267-348),
how many of the sphere filter's candidate pairs a per-triangle plane test
(disc + behind-origin) removes, and whether it keeps every pair the exact
Moller-Trumbore test accepts.

    python tools/disc_probe.py [scene ...]     (synthetic synthetic_dense eye lens)
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
SO = os.path.join(ROOT, "tools", "_disc_probe.so")


def lib():
    src = os.path.join(ROOT, "tools", "disc_probe.cpp")
    hdr = os.path.join(ROOT, "lightpycl_amd", "csrc", "lpc_math.hpp")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.run(["g++", "-O2", "-fopenmp", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "lightpycl_amd", "csrc"), src, "-o", SO], check=True)
    L = ctypes.CDLL(SO)
    P = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    L.disc_probe.argtypes = [ctypes.c_int, P, P, ctypes.c_int, P, ctypes.c_float, ctypes.c_double,
                             ctypes.c_double, np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS"),
                             np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")]
    return L


def populations(name, n0, depth, cap, seed=3):
    import oracle
    from lightpycl_amd import scenes
    sc = scenes.BUILDERS[name](n=n0, seed=seed)
    S = oracle.Scene(sc.meshes)
    src = sc.sources[0]
    o = np.asarray(src.rays_origin, np.float32)[:, :3]
    d = np.asarray(src.rays_dir, np.float32)[:, :3]
    p = np.asarray(src.rays_power, np.float32).reshape(-1)
    pm = np.full(len(p), -2, np.int32)
    rng = np.random.default_rng(seed)
    pops = []
    for it in range(depth):
        if len(p) > cap:
            k = rng.choice(len(p), cap, replace=False)
            o, d, p, pm = o[k], d[k], p[k], pm[k]
        pops.append((it, o.copy(), d.copy()))
        z = np.zeros((len(p), 1), np.float32)
        b = oracle.bounce(S, np.hstack([o, z]), np.hstack([d, z]), p, np.zeros(len(p), np.int32), pm,
                          sc.max_ray_len, sc.ior_env)
        kr = b["r_meas"] == 0
        kt = b["t_meas"] == 0
        dest = b["dest"][:, :3]
        o = np.concatenate([dest[kr], dest[kt]]).astype(np.float32)
        d = np.concatenate([b["r_dir"][kr, :3], b["t_dir"][kt, :3]]).astype(np.float32)
        p = np.concatenate([b["r_pow"][kr], b["t_pow"][kt]]).astype(np.float32)
        pm = np.concatenate([b["isect_mid"][kr], b["isect_mid"][kt]]).astype(np.int32)
        if len(p) == 0:
            break
    V = np.concatenate([S.v0[:, :3], S.v1[:, :3], S.v2[:, :3]], axis=1).astype(np.float32)
    return sc, V, pops


def main():
    names = sys.argv[1:] or ["synthetic", "synthetic_dense", "eye", "lens"]
    L = lib()
    cfg = dict(synthetic=(20000, 3, 3000), synthetic_dense=(4000, 4, 2000), eye=(3000, 6, 1500),
               lens=(3000, 4, 1500))
    for name in names:
        n0, depth, cap = cfg[name]
        sc, V, pops = populations(name, n0, depth, cap)
        lo, hi = V.reshape(-1, 3).min(0), V.reshape(-1, 3).max(0)
        S = float(np.linalg.norm(hi - lo) / 2)
        eps = np.float32(1e-6) * np.float32(sc.max_ray_len)
        for it, o, d in pops:
            out = np.zeros(7, np.int64)
            vi = np.zeros(32, np.int32)
            L.disc_probe(len(o), np.ascontiguousarray(o), np.ascontiguousarray(d), V.shape[0],
                         np.ascontiguousarray(V), eps, 16.0, S, out, vi)
            c = out.tolist()
            print(f"{name} it{it} rays {len(o):6d}  sphere cand/ray {c[0] / len(o):7.2f}  plane keeps "
                  f"{c[1] / max(c[0], 1):.3f} (behind {c[2] / max(c[0], 1):.3f}, disc {c[3] / max(c[0], 1):.3f})"
                  f"  MT acc/cand {c[4] / max(c[0], 1):.3f} -> {c[4] / max(c[1], 1):.3f}  sphere misses {c[5]}"
                  f"  PLANE MISSES {c[6]}", flush=True)


if __name__ == "__main__":
    main()
