"""Capacity and ABI-contract cases on the GPU, against the reference's own kernels
(oracle/_ref via tests/ref_gpu.py: the `exact_ref` / `checker` fixtures).

* mesh_power capacity (ABI 4, include/lpc.h lpc_trace_run): the library writes
  one double per mesh of the CURRENT scene and refuses a smaller buffer with
  LPC_E_ARG instead of overrunning it; one engine traced over scenes of 2, 5 and
  2 meshes through run_local gives the reference's per-mesh power each time.
* many meshes: the reference has no mesh-count limit (.cl:243-289 loops over
  any mesh_id sequence); above 128 live runs every packet's root tests take >= 3
  tasks (k_roots_s S >= 3, one packet per block), above 1 024 the piece table
  goes to k_roots_s in batches.  Bounces bit-exact, whole traces identical.
"""
import ctypes

import numpy as np
import pytest

from lightpycl_amd import scenes

pytestmark = pytest.mark.gpu


def rays_of(sc):
    o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
    d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
    p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
    return o, d, p


def test_mesh_power_capacity_refused(engine):
    """A mesh_power buffer below the scene's mesh count: LPC_E_ARG, nothing written."""
    from lightpycl_amd import _lib
    sc = scenes.eye(n=500, seed=2)                         # K = 5
    o4, d4, pw = rays_of(sc)
    engine.upload_meshes(sc.meshes)
    engine.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
    L = engine.L
    arr = (_lib.IterStats * 16)()
    k, c = ctypes.c_int32(0), ctypes.c_int64(0)
    mp = np.full(8, -7.0, np.float64)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    for fn in (L.lpc_trace_run, L.lpc_trace_run_async, L.lpc_trace_rerun_async):
        rc = fn(engine.h, 16, thr, arr, ctypes.byref(k), ctypes.byref(c), mp.ctypes.data_as(ctypes.c_void_p), 4)
        assert rc == -1, rc                                 # LPC_E_ARG
        assert b"capacity" in L.lpc_last_error(engine.h)
        assert np.all(mp == -7.0)
    rc = L.lpc_trace_measured(engine.h, ctypes.byref(c), mp.ctypes.data_as(ctypes.c_void_p), 4)
    assert rc == -1 and np.all(mp == -7.0)
    # the exact capacity is accepted; NULL mesh_power needs none
    engine.reset()
    assert fn(engine.h, 16, thr, arr, ctypes.byref(k), ctypes.byref(c), mp.ctypes.data_as(ctypes.c_void_p), 5) == 0
    engine.sync()
    assert np.all(mp[5:] == -7.0)
    assert L.lpc_trace_rerun_async(engine.h, 16, thr, arr, ctypes.byref(k), ctypes.byref(c), None, 0) == 0
    engine.sync()


def test_mesh_count_switch_on_one_engine(oracle_mod, exact_ref):
    """K = 2, then the K = 5 eye, then K = 2 again on ONE engine through run_local
    (the sequence behind round 5's heap abort): per-mesh power and counts equal
    the reference host loop over the reference's kernels each time."""
    from parity_util import assert_aggregate_equal, lib_aggregate, ref_aggregate
    from lightpycl_amd.engine import Engine
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    e = Engine(0)
    try:
        for name, n in (("parabolic", 3000), ("eye", 2000), ("lens", 3000)):
            sc = scenes.BUILDERS[name](n=n, seed=17)
            o4, d4, pw = rays_of(sc)
            e.upload_meshes(sc.meshes)
            assert e.mesh_count == len(sc.meshes)
            e.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
            thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
            lib = lib_aggregate(e, sc.iterations, thr, reps=2)
            assert len(lib[1]) == len(sc.meshes)
            ref = ref_aggregate(oracle_mod, exact_ref.bounce, sc.meshes, o4, d4, pw, sc.iterations, sc.tau,
                                sc.max_ray_len, sc.ior_env)
            assert_aggregate_equal(lib, ref, name)
    finally:
        e.close()


@pytest.mark.parametrize("count", [200, 1100])
def test_many_meshes_match_reference(engine, oracle_mod, checker, exact_ref, count):
    """Scenes of 201 and 1 101 meshes: first bounce bit-exact against the
    reference kernels, and the whole aggregate trace identical to the reference
    host loop over them."""
    from parity_util import assert_aggregate_equal, lib_aggregate, ref_aggregate
    sc = scenes.cube_field(n=6000, seed=4, count=count)
    o4, d4, pw = rays_of(sc)
    engine.upload_meshes(sc.meshes)
    assert engine.mesh_count == count + 1
    S = oracle_mod.Scene(sc.meshes)
    z = np.zeros(len(pw), np.int32)
    pm = np.full(len(pw), -2, np.int32)
    g = engine.bounce(o4, d4, pw, z, pm, sc.max_ray_len, sc.ior_env)
    r = checker[0](S, o4, d4, pw, z, pm, sc.max_ray_len, sc.ior_env)
    for k in ("isect_mid", "isect_idx", "n1", "n2", "meas", "r_meas", "t_meas", "entering"):
        np.testing.assert_array_equal(g[k], r[k], err_msg=k)
    np.testing.assert_array_equal(g["dest"][:, :3], r["dest"][:, :3])
    if checker[1]:
        for k in ("r_dir", "t_dir"):
            np.testing.assert_array_equal(g[k][:, :3], r[k][:, :3], err_msg=k)
        for k in ("pow", "r_pow", "t_pow"):
            np.testing.assert_array_equal(g[k], r[k], err_msg=k)
    assert np.unique(g["isect_mid"]).size > min(count, 150)     # many meshes are hit
    if exact_ref is None:
        return
    engine.set_rays(o4, d4, pw, sc.max_ray_len, sc.ior_env)
    thr = (1.0 - sc.tau) * float(np.sum(pw, dtype=np.float64))
    lib = lib_aggregate(engine, sc.iterations, thr, reps=2)
    ref = ref_aggregate(oracle_mod, exact_ref.bounce, sc.meshes, o4, d4, pw, sc.iterations, sc.tau,
                        sc.max_ray_len, sc.ior_env)
    assert len(ref[0]) >= 3
    assert_aggregate_equal(lib, ref, f"cube_field {count}")
