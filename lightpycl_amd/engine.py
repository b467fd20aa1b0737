"""Python front of liblpc: one :class:`Engine` per GPU.

Flattens LightPyCL meshes exactly as ``CL_Tracer.iterative_tracer`` does
(``/root/reference/iterative_tracer.py:121-158``), uploads them, and exposes the
per-bounce entry points of ``include/lpc.h`` with numpy arrays.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check, f32, i32, ptr


def _rows(x, w):
    """x as an (n, w) ndarray without changing a value (an ndarray as is, a list of
    rows through np.asarray), or None when it is not such a table."""
    if type(x) is list:
        try:
            x = np.asarray(x)
        except Exception:
            return None
    if type(x) is not np.ndarray or x.ndim != 2 or x.shape[1] != w or x.dtype.kind not in "fiu":
        return None
    return x


def _tri_tables(mesh):
    """(V as float32 (nv,4), T (n,3) integer) when the mesh holds an ndarray of
    vertex rows and integer triangles (the generators' meshes), else None (the
    caller uses tribuf()).  Gathering rows of float32(V) gives the same rows,
    rounded to float32 the same way, as np.array(tribuf()[k], dtype=np.float32)."""
    V, T = _rows(getattr(mesh, "vertices", None), 4), _rows(getattr(mesh, "triangles", None), 3)
    if V is None or T is None or V.dtype.kind != "f":
        return None
    if T.ndim != 2 or T.shape[1] != 3 or T.dtype.kind not in "iu":
        return None
    if len(T) and (T.min() < -len(V) or T.max() >= len(V)):
        return None
    return np.ascontiguousarray(V, dtype=np.float32), T


def flatten_meshes(meshes):
    """(v0, v1, v2, mesh_id, mat_type, ior, refl, diss) as iterative_tracer.py:121-151 builds
    them: per-mesh material records and the concatenated tribuf() vertex rows
    (gathered straight into the float32 outputs)."""
    K = len(meshes)
    if K == 0:
        raise ValueError("iterative_tracer needs at least one mesh")
    mat_type = np.zeros(K, np.int32)
    ior = np.zeros(K, np.float32)
    refl = np.zeros(K, np.float32)
    diss = np.zeros(K, np.float32)
    parts = []
    for j, mesh in enumerate(meshes):
        mat = mesh.getMaterialBuf()
        mat_type[j] = np.int32(mat.get("type"))
        ior[j] = np.float32(mat.get("IOR"))
        refl[j] = np.float32(mat.get("R"))
        diss[j] = np.float32(mat.get("dissipation"))
        tt = _tri_tables(mesh)
        if tt is None:                          # general vertex containers: the reference's tribuf() lists
            tb = mesh.tribuf()
            tt = [np.array(tb[k], dtype=np.float32).reshape(-1, 4) for k in range(3)]
        parts.append(tt)
    counts = [len(p[1]) if len(p) == 2 else len(p[0]) for p in parts]
    M = int(sum(counts))
    v0, v1, v2 = (np.empty((M, 4), np.float32) for _ in range(3))
    lo = 0
    for p, c in zip(parts, counts):
        for k, out in enumerate((v0, v1, v2)):
            if len(p) == 2:
                np.take(p[0], p[1][:, k], axis=0, out=out[lo:lo + c])
            else:
                out[lo:lo + c] = p[k]
        lo += c
    mesh_id = np.repeat(np.arange(K, dtype=np.int32), counts)
    return v0, v1, v2, mesh_id, mat_type, ior, refl, diss


def array_digest(a):
    """A 128-bit digest of an array's bytes, shape and dtype (xxh3; without the
    xxhash module, a copy of the array stands in for it): the scene and mesh
    caches compare these instead of keeping copies of the arrays."""
    a = np.ascontiguousarray(a)
    try:
        import xxhash
    except ImportError:
        return (a.shape, a.dtype.str, a.copy())
    return (a.shape, a.dtype.str, xxhash.xxh3_128_digest(a.view(np.uint8).reshape(-1)))


def _same_digest(x, y):
    if x[0] != y[0] or x[1] != y[1]:
        return False
    return np.array_equal(x[2], y[2]) if isinstance(x[2], np.ndarray) else x[2] == y[2]


def default_device() -> int:
    for key in ("LPC_DEVICE", "LOCAL_RANK"):
        if os.environ.get(key, "") != "":
            return int(os.environ[key])
    return 0


def device_names():
    """[(name, gcnArchName, CUs)] of the visible HIP devices (lpc_device_query)."""
    L = _lib.load()
    c = ctypes.c_int(0)
    check(L.lpc_device_count(ctypes.byref(c)), None)
    out = []
    for k in range(c.value):
        name, arch, cu = ctypes.create_string_buffer(256), ctypes.create_string_buffer(64), ctypes.c_int(0)
        check(L.lpc_device_query(k, name, 256, arch, 64, ctypes.byref(cu)), None)
        out.append((name.value.decode(errors="replace"), arch.value.decode(errors="replace"), cu.value))
    return out


def select_device(device_name=None, names=None) -> int:
    """The HIP device for ``CL_Tracer(device_name=...)``, as the reference picks
    its OpenCL device (iterative_tracer.py:50-55): an int is an ordinal; a string
    is a substring of the device's name or architecture, and the LAST matching
    device wins, as in the reference's loop (a string of digits that matches no
    name is an ordinal if that device exists); no match -> the default device (``$LPC_DEVICE``, ``$LOCAL_RANK`` or 0), as
    the reference falls back to its first device.  When several devices match
    and the default one is among them, the default is kept (one process per GPU:
    every rank asks for "MI355" and keeps its own)."""
    dflt = default_device()
    if device_name is None:
        return dflt
    if isinstance(device_name, (int, np.integer)):
        return int(device_name)
    names = device_names() if names is None else names
    key = str(device_name)
    hits = [k for k, (nm, arch, _) in enumerate(names) if key in nm or key in arch]
    if hits:
        return dflt if dflt in hits else hits[-1]
    # a string of digits that names no device: an ordinal when there is such a
    # device (the reference's default "770" is neither: default device)
    if key.strip().isdigit() and int(key) < len(names):
        return int(key)
    return dflt


class Engine:
    """A liblpc handle on one GPU (HIP device ordinal ``device``)."""

    def __init__(self, device=None):
        self.L = _lib.load()
        self.device = default_device() if device is None else int(device)
        h = ctypes.c_void_p()
        check(self.L.lpc_open(self.device, ctypes.byref(h)), None)
        self.h = h
        self.tri_count = 0
        self.mesh_count = 0

    # -- lifecycle -----------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.L.lpc_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, rc):
        check(rc, self.h)

    def info(self):
        buf = ctypes.create_string_buffer(256)
        cu = ctypes.c_int(0)
        self._c(self.L.lpc_device_info(self.h, buf, 256, ctypes.byref(cu)))
        return buf.value.decode(), cu.value

    # -- scene ---------------------------------------------------------------
    def upload_arrays(self, v0, v1, v2, mesh_id, mat_type, ior, refl, diss):
        v0, v1, v2 = f32(v0, (-1, 4)), f32(v1, (-1, 4)), f32(v2, (-1, 4))
        mesh_id, mat_type = i32(mesh_id), i32(mat_type)
        ior, refl, diss = f32(ior), f32(refl), f32(diss)
        M, K = v0.shape[0], mat_type.shape[0]
        # the same scene as the last upload (a tracer called again on its meshes,
        # as the reference's examples do): keep the device records, skip the
        # rebuild (the filter hierarchy is built on the host at every upload).
        # Compared by a digest of the bytes (-0.0 is not 0.0).
        arrs = (v0, v1, v2, mesh_id, mat_type, ior, refl, diss)
        digest = tuple(array_digest(a) for a in arrs)
        last = getattr(self, "_scene_last", None)
        if last is not None and all(_same_digest(a, b) for a, b in zip(digest, last)):
            return
        self._scene_last = None
        self._c(self.L.lpc_scene_upload(self.h, M, ptr(v0), ptr(v1), ptr(v2), ptr(mesh_id), K,
                                        ptr(mat_type), ptr(ior), ptr(refl), ptr(diss)))
        self.tri_count, self.mesh_count = M, K
        self.mat_type = mat_type
        self._scene_last = digest

    def upload_meshes(self, meshes):
        arrs = flatten_meshes(meshes)
        self.upload_arrays(*arrs)
        return arrs

    # -- one bounce on host arrays (partition-loop body) ------------------------
    def bounce(self, origin4, dir4, pow_, meas, prev_mid, max_ray_len=1e3, ior_env=1.0):
        o, d = f32(origin4, (-1, 4)), f32(dir4, (-1, 4))
        n = o.shape[0]
        pw = f32(pow_).reshape(-1).copy()
        ms = i32(meas).reshape(-1).copy()
        pm = i32(prev_mid).reshape(-1)
        out = {k: np.zeros((n, 4), np.float32) for k in ("dest", "r_dir", "t_dir")}
        for k in ("r_pow", "t_pow"):
            out[k] = np.zeros(n, np.float32)
        for k in ("isect_mid", "r_meas", "t_meas", "n1", "n2", "entering", "isect_idx"):
            out[k] = np.zeros(n, np.int32)
        self._c(self.L.lpc_bounce_host(
            self.h, n, ptr(o), ptr(d), ptr(pw), ptr(ms), ptr(pm), np.float32(max_ray_len),
            np.float32(ior_env), ptr(out["dest"]), ptr(out["isect_mid"]), ptr(out["r_dir"]),
            ptr(out["r_pow"]), ptr(out["r_meas"]), ptr(out["t_dir"]), ptr(out["t_pow"]),
            ptr(out["t_meas"]), ptr(out["n1"]), ptr(out["n2"]), ptr(out["entering"]),
            ptr(out["isect_idx"])))
        out["pow"] = pw
        out["meas"] = ms
        return out

    # -- device-resident trace -----------------------------------------------
    def set_chunk(self, rays):
        self._c(self.L.lpc_set_chunk(self.h, int(rays)))

    def set_walk_grid(self, blocks):
        """Hierarchy-walk grid in single-wave blocks (0: the library default);
        a launch policy, results unchanged (lpc_set_walk_grid)."""
        self._c(self.L.lpc_set_walk_grid(self.h, int(blocks)))

    def set_rays(self, origin4, dir4, pow_, max_ray_len=1e3, ior_env=1.0):
        o, d = f32(origin4, (-1, 4)), f32(dir4, (-1, 4))
        pw = f32(pow_).reshape(-1)
        n = o.shape[0]
        if d.shape[0] != n or pw.shape[0] != n:
            raise ValueError("origin, direction and power must have the same ray count")
        self._c(self.L.lpc_trace_set_rays(self.h, n, ptr(o), ptr(d), ptr(pw),
                                          np.float32(max_ray_len), np.float32(ior_env)))
        return n

    def stage_rays(self, origin4, dir4, pow_, max_ray_len=1e3, ior_env=1.0):
        """lpc_trace_stage_rays: queue a batch of new rays (at most two staged),
        copied to the device by a helper thread while the engine traces the batch
        before it.  The arrays are kept alive here until :meth:`run_staged`
        traces the batch."""
        o, d = f32(origin4, (-1, 4)), f32(dir4, (-1, 4))
        pw = f32(pow_).reshape(-1)
        n = o.shape[0]
        if d.shape[0] != n or pw.shape[0] != n:
            raise ValueError("origin, direction and power must have the same ray count")
        self._c(self.L.lpc_trace_stage_rays(self.h, n, ptr(o), ptr(d), ptr(pw), np.float32(max_ray_len),
                                            np.float32(ior_env)))
        self.__dict__.setdefault("_staged", []).append((o, d, pw))
        return n

    def run_staged(self, iterations, power_threshold):
        """lpc_trace_run_staged_async: trace the oldest staged batch (it becomes
        the emitted rays, as set_rays) to the reference's termination.  Returns
        what :meth:`run_local` returns; the outputs are final, the last rows may
        still move (:meth:`sync`)."""
        arr, k, c, mp, pk, pc, pmp, mcap = self._bufs(iterations)
        try:
            self._c(self.L.lpc_trace_run_staged_async(self.h, max(int(iterations), 0), float(power_threshold), arr,
                                                      pk, pc, pmp, mcap))
        finally:
            staged = getattr(self, "_staged", [])
            if staged:
                staged.pop(0)               # the helper has copied it (joined in the call)
        return type(arr).from_buffer_copy(arr)[:k.value], (c.value, mp[: self.mesh_count].copy())

    def reset(self):
        self._c(self.L.lpc_trace_reset(self.h))

    def population(self):
        n = ctypes.c_int64(0)
        self._c(self.L.lpc_trace_population(self.h, ctypes.byref(n)))
        return n.value

    def iterate(self, export=False):
        """One iteration over the device population.  With ``export`` returns the
        reference's results tuple arrays and the next population's powers."""
        st = _lib.IterStats()
        if not export:
            self._c(self.L.lpc_trace_iterate(self.h, None, None, None, None, None, ctypes.byref(st)))
            return st, None
        n = self.population()
        org = np.empty((n, 4), np.float32)
        dst = np.empty((n, 4), np.float32)
        pw = np.empty(n, np.float32)
        ms = np.empty(n, np.int32)
        nxt = np.empty(max(2 * n, 1), np.float32)
        self._c(self.L.lpc_trace_iterate(self.h, ptr(org), ptr(dst), ptr(pw), ptr(ms), ptr(nxt),
                                         ctypes.byref(st)))
        return st, dict(origin=org, dest=dst, pow=pw, meas=ms,
                        next_pow=nxt[: st.n_reflect + st.n_refract])

    def iterate_export(self, with_origin=True):
        """One iteration with its results tuple exported asynchronously
        (lpc_trace_iterate_export) into a pinned block: returns (stats, dict of
        origin (N,4) [if with_origin], dest (N,4), pow (N,), meas (N,) numpy views).
        The arrays are complete after :meth:`sync` (the copy overlaps the next
        iteration's kernels)."""
        from .pinned import POOL
        n = self.population()
        st = _lib.IterStats()
        if n == 0:
            self._c(self.L.lpc_trace_iterate(self.h, None, None, None, None, None, ctypes.byref(st)))
            z = np.zeros((0, 4), np.float32)
            return st, dict(origin=z, dest=z.copy(), pow=np.zeros(0, np.float32), meas=np.zeros(0, np.int32))
        layout = ([(np.float32, (n, 4))] if with_origin else []) + [(np.float32, (n, 4)), (np.float32, (n,)),
                                                                     (np.int32, (n,))]
        import time as _t
        t0 = _t.perf_counter()
        blk = POOL.block(n * ((16 if with_origin else 0) + 24))
        t1 = _t.perf_counter()
        # the block's address as a plain integer: ctypes.cast would tie the block and
        # the cast result into a reference cycle, and the block would return to the
        # pool only when the cyclic GC happens to run
        self._c(self.L.lpc_trace_iterate_export(self.h, ctypes.c_void_p(ctypes.addressof(blk)),
                                                1 if with_origin else 0, ctypes.byref(st)))
        self.export_times = (t1 - t0, _t.perf_counter() - t1)
        v = POOL.views(blk, layout)
        if not with_origin:
            v = [None] + v
        return st, dict(origin=v[0], dest=v[1], pow=v[2], meas=v[3])

    def population_power(self):
        """The current population's power (lpc_trace_population_power)."""
        n = self.population()
        out = np.empty(n, np.float32)
        if n:
            self._c(self.L.lpc_trace_population_power(self.h, ptr(out)))
        return out

    def sync(self):
        """lpc_sync: wait for every kernel queued on the engine's stream."""
        self._c(self.L.lpc_sync(self.h))

    def _bufs(self, iterations):
        """Output buffers and argument objects of the trace calls, kept per
        (iteration cap, mesh count): the library writes one power per mesh of the
        CURRENT scene into mp, and refuses a buffer below that count (its capacity
        travels with the call)."""
        cap = max(int(iterations), 0)
        key = (cap, int(self.mesh_count))
        bufs = self._run_bufs.get(key) if hasattr(self, "_run_bufs") else None
        if bufs is None:
            arr, k, c = (_lib.IterStats * max(cap, 1))(), ctypes.c_int32(0), ctypes.c_int64(0)
            mp = np.zeros(max(key[1], 1), np.float64)
            bufs = (arr, k, c, mp, ctypes.byref(k), ctypes.byref(c), mp.ctypes.data_as(ctypes.c_void_p),
                    ctypes.c_int32(mp.size))
            self.__dict__.setdefault("_run_bufs", {})[key] = bufs
        return bufs

    def run_local(self, iterations, power_threshold, wait=True, reset=False):
        """lpc_trace_run: iterate until the next population's power is below
        power_threshold or no ray is kept (at most `iterations`).  Returns the
        per-iteration stats and the measured (count, per-mesh power).
        reset=True (with wait=False): lpc_trace_rerun_async, the reset and the
        trace in one call (the bench's back-to-back batches)."""
        cap = max(int(iterations), 0)
        arr, k, c, mp, pk, pc, pmp, mcap = self._bufs(cap)
        # wait=False: lpc_trace_run_async (the outputs are final; the last rows may
        # still move on the device and the next batch's launches queue behind them)
        if reset and not wait:
            fn = self.L.lpc_trace_rerun_async
        else:
            if reset:
                self.reset()
            fn = self.L.lpc_trace_run if wait else self.L.lpc_trace_run_async
        self._c(fn(self.h, cap, float(power_threshold), arr, pk, pc, pmp, mcap))
        # one copy of the stats block (the buffers are reused by the next call)
        return type(arr).from_buffer_copy(arr)[:k.value], (c.value, mp[: self.mesh_count].copy())

    # -- ray-sharded trace --------------------------------------------------------
    def set_allreduce(self, comm):
        """Install the all-reduce hook of lpc_trace_run's loop (lpc_set_allreduce):
        the library's shared-memory comm (:class:`distributed.ShmComm`, native, no
        Python in the loop) or any object with ``allreduce_sum(values) -> array``
        (called back through ctypes).  None removes it."""
        if comm is None:
            self._xchg = None
            self._c(self.L.lpc_set_allreduce(self.h, None, None))
            return
        native = getattr(comm, "native_hook", None)
        if native is not None:
            fn, ctx = native(self)
            self._xchg = (comm, fn)
            self._c(self.L.lpc_set_allreduce(self.h, fn, ctx))
            return

        def cb(_ctx, vals, n):
            try:
                v = np.ctypeslib.as_array(vals, shape=(n,))
                v[:] = np.asarray(comm.allreduce_sum(v.copy()), dtype=np.float64).reshape(-1)
                return 0
            except Exception:           # an exception must not cross the C frame
                return -1
        fn = _lib.ALLREDUCE_FN(cb)
        self._xchg = (comm, fn)         # keep the callback alive while installed
        self._c(self.L.lpc_set_allreduce(self.h, ctypes.cast(fn, ctypes.c_void_p), None))

    def global_stats(self):
        """All-reduced per-iteration stats of the last run_local (lpc_trace_global_stats)."""
        n = ctypes.c_int32(0)
        self._c(self.L.lpc_trace_global_stats(self.h, None, 0, ctypes.byref(n)))
        arr = (_lib.IterStats * max(n.value, 1))()
        self._c(self.L.lpc_trace_global_stats(self.h, arr, n.value, ctypes.byref(n)))
        return [_lib.IterStats.from_buffer_copy(arr[i]) for i in range(n.value)]

    def measured(self):
        """(count, per-mesh measured power float64[K])."""
        c = ctypes.c_int64(0)
        mp = np.zeros(max(self.mesh_count, 1), np.float64)
        self._c(self.L.lpc_trace_measured(self.h, ctypes.byref(c), ptr(mp), mp.size))
        return c.value, mp[: self.mesh_count]

    def fetch_measured(self):
        """Measured record: pos (Nm,4) float32, pwr (Nm,) float32, mesh (Nm,) int32."""
        c = ctypes.c_int64(0)
        self._c(self.L.lpc_trace_measured(self.h, ctypes.byref(c), None, 0))
        n = c.value
        pos = np.zeros((n, 4), np.float32)
        pw = np.zeros(n, np.float32)
        mm = np.zeros(n, np.int32)
        if n:
            self._c(self.L.lpc_trace_fetch_measured(self.h, ptr(pos), ptr(pw), ptr(mm)))
        return pos, pw, mm

    # -- projection + histogram ---------------------------------------------
    def project_hist(self, pos4, pwr, limits, points, mode=0, rot=None, pivot=None,
                     want_xy=False):
        """angular (mode 0) / stereographic (1) projection + np.histogram2d binning of
        pwr_cor / (dx*dy).  pos4=None bins the device-resident measured record."""
        _, xe, ye = np.histogram2d(np.zeros(0), np.zeros(0), bins=points, range=limits)
        xe = np.ascontiguousarray(xe, np.float64)
        ye = np.ascontiguousarray(ye, np.float64)
        nx, ny = xe.size - 1, ye.size - 1
        dx = np.float64(limits[0][1] - limits[0][0]) / np.float64(points)
        dy = np.float64(limits[1][1] - limits[1][0]) / np.float64(points)
        # rotation rows as the reference's R_dev (iterative_tracer.py:545); only rows 0-2
        # (xyz) are read by the kernel
        rot = f32(np.eye(4, dtype=np.float32) if rot is None else rot, (4, 4))
        piv = f32(np.zeros(4, np.float32) if pivot is None else pivot).reshape(4)
        H = np.zeros((nx, ny), np.float64)
        if pos4 is None:
            n = 0
            p4 = pw = None
        else:
            p4 = f32(pos4, (-1, 4))
            pw = f32(pwr).reshape(-1)
            n = p4.shape[0]
        x = y = pc = None
        if want_xy:
            cnt = n if pos4 is not None else self.measured()[0]
            x, y, pc = (np.zeros(cnt, np.float32) for _ in range(3))
        self._c(self.L.lpc_project_hist(self.h, int(mode), n, ptr(p4), ptr(pw), ptr(rot), ptr(piv),
                                        ptr(xe), nx, ptr(ye), ny, float(dx * dy), ptr(H), ptr(x),
                                        ptr(y), ptr(pc)))
        return (H, xe, ye) if not want_xy else (H, xe, ye, x, y, pc)

    # -- profiling -------------------------------------------------------------
    def prof_enable(self, on=True, counters=False, light=False, every=1):
        """light: HIP events on the walk kernel's launches only, on every
        `every`-th one (lpc_prof_enable's 4 + 256 k)."""
        level = ((4 + 256 * max(int(every), 1)) if light else 2 if counters else 1) if on else 0
        self._c(self.L.lpc_prof_enable(self.h, level))

    def prof_read(self, reset=True):
        p = _lib.Prof()
        self._c(self.L.lpc_prof_read(self.h, ctypes.byref(p), 1 if reset else 0))
        return dict(intersect_ms=p.intersect_ms, shade_ms=p.shade_ms,
                    intersect_launches=p.intersect_launches, pairs=p.pairs, node_visits=p.node_visits,
                    group_tests=p.group_tests, wave_traversals=p.wave_traversals, exact_tests=p.exact_tests,
                    wave_hist=list(p.wave_hist), heavy_piece=p.heavy_piece, heavy_piece_ticks=p.heavy_piece_ticks,
                    piece_ticks=p.piece_ticks, tail_waves=p.tail_waves, tail_nodes=p.tail_nodes,
                    tail_spread_urad=p.tail_spread_urad, tail_exact=p.tail_exact, kernel_ms=p.kernel_ms,
                    xchg_us=p.xchg_us, xchg_calls=p.xchg_calls, walk_cycles=p.walk_cycles,
                    drain_cycles=p.drain_cycles, fan_exact=p.fan_exact,
                    behind_exact=p.behind_exact, hit_exact=p.hit_exact)
