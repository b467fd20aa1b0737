"""CPU ORACLE for the LightPyCL per-bounce path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker (or the timed CPU
baseline).  The product package ``lightpycl_amd`` never imports it.

It is a restatement of the reference:

* the four OpenCL kernels -> ``lpc_oracle.c`` (built by ``oracle/Makefile``),
  called here through ctypes with the reference's own (n,4) buffer layouts;
* the host loop of ``CL_Tracer.iterative_tracer``
  (``/root/reference/iterative_tracer.py:77-393``) -> :func:`trace`;
* ``get_measured_rays`` (``iterative_tracer.py:395-411``) and
  ``get_binned_data_angular`` (``iterative_tracer.py:534-562``).

Parity status: pinned against the reference's OWN kernels -- the unmodified
``kernel_reflect_refract_intersect.cl`` compiled for gfx950 with ROCm's OpenCL
device libraries (``oracle/Makefile`` target ``ref`` -> ``oracle/_ref/``,
launched by ``tests/ref_gpu.py``) -- within SURVEY.md section 8c's fp32
tolerances (``tests/test_ref_parity.py``, on the GPU), and on the CPU by the
SURVEY.md section-4 known-answer rows and the reference-scene counts
(``tests/test_oracle_pins.py``).  The reference's Python-2 host loop cannot be
imported; :func:`trace` restates it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liblpc_oracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_f32 = ctypes.c_float


def build():
    """Compile ``lpc_oracle.c`` (idempotent)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.orc_intersect.argtypes = [_i64, _f32p, _f32p, _f32p, _f32p, _f32p, _i32p, _i32, _i32,
                                    _f32, _f32p, _i32p, _i32p]
        L.orc_intersect_postproc.argtypes = [_i64, _f32p, _f32p, _f32p, _i32p, _i32p, _i32p,
                                             _i32p, _i32p, _i32p, _i32p, _f32p, _i32p, _i32p,
                                             _i32, _f32]
        L.orc_reflect_refract_rays.argtypes = [_i64, _f32p, _f32p, _f32p, _f32p, _i32p, _i32p,
                                               _i32p, _f32p, _f32p, _f32p, _i32p, _f32p, _f32p,
                                               _f32p, _i32p, _i32p, _i32p, _f32p, _f32p, _f32p,
                                               _i32p, _f32p, _f32p, _f32p, _f32]
        L.orc_angular_project.argtypes = [_i64, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
        L.orc_stereograph_project.argtypes = [_i64, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                              _f32p]
        L.orc_set_threads.argtypes = [_i32]
        L.orc_set_threads.restype = _i32
        for fn in (L.orc_intersect, L.orc_intersect_postproc, L.orc_reflect_refract_rays,
                   L.orc_angular_project, L.orc_stereograph_project):
            fn.restype = None
        _lib = L
    return _lib


def set_threads(n: int) -> int:
    """OpenMP team size for the kernels above (n <= 0: leave it); returns the
    team size in effect."""
    return int(lib().orc_set_threads(int(n)))


def _v4(a, n=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1, 4))
    if n is not None:
        assert a.shape[0] == n
    return a


class Scene:
    """Flattened scene exactly as iterative_tracer.py:121-151 builds it."""

    def __init__(self, meshes):
        K = len(meshes)
        self.mesh_count = K
        self.mat_type = np.zeros(K, np.int32)
        self.ior = np.zeros(K, np.float32)
        self.refl = np.zeros(K, np.float32)
        self.diss = np.zeros(K, np.float32)
        v0s, v1s, v2s, ids = [], [], [], []
        for j, m in enumerate(meshes):
            mat = m.getMaterialBuf()
            self.mat_type[j] = np.int32(mat.get("type"))
            self.ior[j] = np.float32(mat.get("IOR"))
            self.refl[j] = np.float32(mat.get("R"))
            self.diss[j] = np.float32(mat.get("dissipation"))
            tb = m.tribuf()
            v0s.append(np.array(tb[0], dtype=np.float32).reshape(-1, 4))
            v1s.append(np.array(tb[1], dtype=np.float32).reshape(-1, 4))
            v2s.append(np.array(tb[2], dtype=np.float32).reshape(-1, 4))
            ids.append(np.zeros(len(tb[0]), np.int32) + j)
        self.v0 = np.ascontiguousarray(np.concatenate(v0s).astype(np.float32))
        self.v1 = np.ascontiguousarray(np.concatenate(v1s).astype(np.float32))
        self.v2 = np.ascontiguousarray(np.concatenate(v2s).astype(np.float32))
        self.mesh_id = np.ascontiguousarray(np.concatenate(ids).astype(np.int32))
        self.tri_count = int(self.v0.shape[0])


def bounce(scene: Scene, origin, direction, power, meas, prev_mid, max_ray_len=1e3, ior_env=1.0):
    """One pass of the partition-loop body (iterative_tracer.py:267-348): the three
    kernels on the CPU.  Returns a dict of every per-ray output buffer."""
    L = lib()
    n = int(np.asarray(prev_mid).shape[0])
    K = scene.mesh_count
    mrl = np.float32(max_ray_len)
    o = _v4(origin, n)
    d = _v4(direction, n)
    pw = np.ascontiguousarray(np.asarray(power, np.float32).reshape(-1).copy())
    ms = np.ascontiguousarray(np.asarray(meas, np.int32).reshape(-1).copy())
    pm = np.ascontiguousarray(np.asarray(prev_mid, np.int32).reshape(-1))
    tmin = np.zeros(n * K, np.float32) + mrl           # iterative_tracer.py:267
    cnt = np.zeros(n * K, np.int32)                    # :236 (zeros; never-written slots stay 0)
    itmp = np.zeros(n * K, np.int32)                   # :237
    L.orc_intersect(n, o, d, scene.v0, scene.v1, scene.v2, scene.mesh_id, K, scene.tri_count,
                    mrl, tmin, cnt, itmp)
    dest = np.zeros((n, 4), np.float32)
    n1 = np.zeros(n, np.int32)
    n2 = np.zeros(n, np.int32)
    ent = np.zeros(n, np.int32)
    imid = np.zeros(n, np.int32)
    iidx = np.zeros(n, np.int32)
    L.orc_intersect_postproc(n, o, d, dest, pm, n1, n2, ent, imid, iidx, scene.mat_type,
                             tmin, cnt, itmp, K, mrl)
    ro = np.zeros((n, 4), np.float32)
    rd = np.zeros((n, 4), np.float32)
    rp = np.zeros(n, np.float32)
    rm = np.zeros(n, np.int32)
    to = np.zeros((n, 4), np.float32)
    td = np.zeros((n, 4), np.float32)
    tp = np.zeros(n, np.float32)
    tm = np.zeros(n, np.int32)
    L.orc_reflect_refract_rays(n, o, dest, d, pw, ms, n1, n2, ro, rd, rp, rm, to, td, tp, tm,
                               imid, iidx, scene.v0, scene.v1, scene.v2, scene.mat_type,
                               scene.ior, scene.refl, scene.diss, np.float32(ior_env))
    return dict(dest=dest, pow=pw, meas=ms, isect_mid=imid, isect_idx=iidx, n1=n1, n2=n2,
                entering=ent, r_origin=ro, r_dir=rd, r_pow=rp, r_meas=rm, t_origin=to,
                t_dir=td, t_pow=tp, t_meas=tm, isect_min_ray_len=tmin.reshape(n, K),
                isects_count=cnt.reshape(n, K), isect_idx_tmp=itmp.reshape(n, K))


def f32_sorted_sum(a):
    """``sum(np.sort(a))`` as iterative_tracer.py:115/372 evaluates it: Python's builtin
    sum over np.sort along the LAST axis, i.e. a sequential float32 accumulation."""
    s = np.sort(np.asarray(a), axis=-1)
    flat = s.reshape(-1).astype(np.float32)
    if flat.size == 0:
        return np.float32(0.0)
    return np.add.accumulate(flat, dtype=np.float32)[-1]


def trace(light_source, meshes, trace_iterations=100, trace_until_dissipated=0.99,
          max_ray_len=np.float32(1e3), ior_env=np.float32(1.0), keep_results=True, bounce_fn=None,
          measured_out=None):
    """Restatement of CL_Tracer.iterative_tracer (iterative_tracer.py:77-393).

    Returns (results, info) where results is the list of per-iteration tuples
    (rays_origin, rays_dest, rays_pow, rays_meas) and info holds the per-iteration
    ray counts and the per-mesh measured power (float64).  ``bounce_fn`` replaces
    the three kernels (default: :func:`bounce`, the C restatement); the GPU tests
    pass the reference's own kernels (``tests/ref_gpu.py``) here.
    ``measured_out`` (a list): each iteration's measured rays are appended as
    (dest (m,4), pow (m,), hit mesh (m,)) -- get_measured_rays' rows plus the
    mesh, without keeping the whole results tuples (large traces)."""
    origin = dirs = power = None
    for k, light in enumerate(light_source):                       # :99-113
        if k == 0:
            origin = np.float32(light.rays_origin)
            dirs = np.float32(light.rays_dir)
            power = np.float32(light.rays_power)
        else:
            origin = np.append(origin, light.rays_origin, axis=0).astype(np.float32)
            dirs = np.append(dirs, light.rays_dir, axis=0).astype(np.float32)
            power = np.append(power, light.rays_power, axis=0).astype(np.float32)
    return trace_rays(origin, dirs, power, meshes, trace_iterations, trace_until_dissipated, max_ray_len,
                      ior_env, keep_results, bounce_fn, measured_out)


def trace_rays(origin, dirs, power, meshes, trace_iterations=100, trace_until_dissipated=0.99,
               max_ray_len=np.float32(1e3), ior_env=np.float32(1.0), keep_results=True, bounce_fn=None,
               measured_out=None):
    """:func:`trace` from the concatenated emitted rays (iterative_tracer.py:99-113's
    arrays: origin (N,4), dirs (N,4), power (N,1) or (N,)) instead of light sources."""
    bounce_fn = bounce if bounce_fn is None else bounce_fn
    max_ray_len = np.float32(max_ray_len)
    ior_env = np.float32(ior_env)
    origin = np.asarray(origin, np.float32)
    dirs = np.asarray(dirs, np.float32)
    power = np.asarray(power, np.float32)
    ray_count = origin.shape[0]
    input_power = f32_sorted_sum(power)                            # :115
    rays_pow = np.array(power, dtype=np.float32)                   # :116
    rays_meas = np.zeros(ray_count, np.int32)                      # :117
    cur_mid = np.zeros(ray_count, np.int32) - 2                    # :118
    scene = Scene(meshes)
    results = []
    counts = []
    mesh_power = np.zeros(scene.mesh_count, np.float64)
    for _ in range(int(trace_iterations)):                         # :241
        counts.append(ray_count)
        out = bounce_fn(scene, origin, dirs, rays_pow, rays_meas, cur_mid, max_ray_len, ior_env)
        rays_dest = out["dest"]
        rays_pow = out["pow"].reshape(np.shape(rays_pow))           # :347 keeps the input shape
        rays_meas = out["meas"]
        m = rays_meas >= 0.9
        np.add.at(mesh_power, out["isect_mid"][m], rays_pow.reshape(-1)[m].astype(np.float64))
        if measured_out is not None:
            measured_out.append((rays_dest[m], rays_pow.reshape(-1)[m], out["isect_mid"][m]))
        if keep_results:
            results.append((origin, rays_dest, rays_pow, rays_meas))   # :355
        keep = np.where(np.concatenate((out["r_meas"], out["t_meas"])) == 0)[0]   # :366
        origin = np.append(out["r_origin"], out["t_origin"], axis=0).astype(np.float32)[keep]
        dirs = np.append(out["r_dir"], out["t_dir"], axis=0).astype(np.float32)[keep]
        rays_pow = np.append(out["r_pow"], out["t_pow"], axis=0).astype(np.float32)[keep]
        rays_meas = np.append(out["r_meas"], out["t_meas"], axis=0).astype(np.int32)[keep]
        power_in_scene = f32_sorted_sum(rays_pow)                  # :372
        cur_mid = np.append(out["isect_mid"], out["isect_mid"], axis=0).astype(np.int32)[keep]
        ray_count = origin.shape[0]
        if power_in_scene < (1.0 - trace_until_dissipated) * input_power:   # :383
            break
        if ray_count == 0:                                         # :389
            break
    info = dict(counts=counts, mesh_power=mesh_power, input_power=input_power,
                tri_count=scene.tri_count)
    return results, info


def measured_rays(results):
    """get_measured_rays, iterative_tracer.py:395-411."""
    pos = pwr = None
    for k, (_o, dest, pw, ms) in enumerate(results):
        idx = np.where(ms >= .9)[0]
        if k == 0:
            pos, pwr = dest[idx], pw[idx]
        else:
            pos = np.concatenate((pos, dest[idx]), axis=0)
            pwr = np.concatenate((pwr.flatten(), pw[idx].flatten()), axis=0)
    return pos, pwr


_IDENT = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 0]], np.float32)
_ZERO4 = np.zeros(4, np.float32)


def angular_project(pos, pwr, rot=_IDENT, pivot=_ZERO4):
    """__kernel angular_project on the CPU (.cl:509-538)."""
    pos = _v4(pos)
    pwr = np.ascontiguousarray(np.asarray(pwr, np.float32).reshape(-1))
    n = pos.shape[0]
    x = np.zeros(n, np.float32)
    y = np.zeros(n, np.float32)
    pc = np.zeros(n, np.float32)
    lib().orc_angular_project(n, pos, pwr, np.ascontiguousarray(rot, np.float32).reshape(-1),
                              np.ascontiguousarray(pivot, np.float32).reshape(-1), x, y, pc)
    return x, y, pc


def stereograph_project(pos, pwr, rot=_IDENT, pivot=_ZERO4):
    """__kernel stereograph_project on the CPU (.cl:488-506)."""
    pos = _v4(pos)
    pwr = np.ascontiguousarray(np.asarray(pwr, np.float32).reshape(-1))
    n = pos.shape[0]
    x = np.zeros(n, np.float32)
    y = np.zeros(n, np.float32)
    pc = np.zeros(n, np.float32)
    lib().orc_stereograph_project(n, pos, pwr, np.ascontiguousarray(rot, np.float32).reshape(-1),
                                  np.ascontiguousarray(pivot, np.float32).reshape(-1), x, y, pc)
    return x, y, pc


def binned_angular(pos, pwr, limits=((-1, 1), (-1, 1)), points=500):
    """get_binned_data_angular, iterative_tracer.py:534-562."""
    x, y, pc = angular_project(pos, pwr)
    pw = np.float64(pc)
    dx = np.float64(limits[0][1] - limits[0][0]) / np.float64(points)
    dy = np.float64(limits[1][1] - limits[1][0]) / np.float64(points)
    pw = pw / (dx * dy)
    return np.histogram2d(x=x.flatten(), y=y.flatten(), bins=points, range=limits,
                          weights=pw.flatten())
