"""``CL_Tracer`` -- drop-in for LightPyCL's ``iterative_tracer`` module, running the
per-bounce hot path on an MI355X through liblpc (HIP, gfx950).

Mirrors ``/root/reference/iterative_tracer.py``:
  * ``CL_Tracer(platform_name, device_name, debug)`` (:36-74): ``device_name``
    picks the HIP device as the reference picks its OpenCL device (an ordinal, or
    a substring of the device name / gfx architecture, last match wins, no match
    -> ``$LPC_DEVICE``, ``$LOCAL_RANK`` or 0); ``device=`` (an ordinal) overrides;
  * ``iterative_tracer(light_source, meshes, trace_iterations, trace_until_dissipated,
    max_ray_len, ior_env)`` (:77-393) -> ``self.results``, a list of per-iteration
    tuples ``(rays_origin (N,4) f32, rays_dest (N,4) f32, rays_pow, rays_meas (N,) i32)``
    in the reference's ray order and shapes;
  * ``get_measured_rays`` (:395-411), the binning / beam-width analyses (:413-709),
    ``pickle_results`` / ``load_pickle_results`` (:711-751), ``save_traced_scene``.

Extra keyword ``keep_results=False`` selects the aggregate mode: no per-ray results
cross PCIe; measured rays and per-mesh measured power stay on the device
(``get_measured_rays`` / ``measured_power`` / the binning calls read them there).
In that mode the measured rays of an iteration come in the device's coherence
(traced) order, not the reference's ray order: the same rays bit for bit as a
set, so order-dependent reductions over them (a float32 ``np.sum``, the stable
sort behind ``get_beam_width_half_power``'s tie-breaking) can differ from the
reference in the last bits.  ``keep_results=True`` (the default) keeps the
reference's order (iteration, then ray).
"""
from __future__ import annotations

import ctypes
import pickle
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _lib
from .engine import Engine, _same_digest, array_digest, flatten_meshes, select_device


def f32_sorted_sum(a):
    """``sum(np.sort(a))`` as the reference evaluates it (:115, :372): np.sort along the
    last axis, then a sequential float32 accumulation (liblpc's host loop: the
    same adds in the same order as np.add.accumulate, without its output array)."""
    a = np.asarray(a)
    flat = (a if a.ndim == 2 and a.shape[-1] == 1 else np.sort(a, axis=-1)).reshape(-1)
    flat = np.ascontiguousarray(flat, dtype=np.float32)
    if flat.size == 0:
        return np.float32(0.0)
    out = ctypes.c_float(0.0)
    _lib.check(_lib.load().lpc_host_seq_sum_f32(flat.ctypes.data_as(ctypes.c_void_p), flat.size, ctypes.byref(out)))
    return np.float32(out.value)


# the tracer's helper thread (created with the module, started on first use)
_SUM_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="lpc-sum")


def _background(fn, *args):
    """Run fn(*args) on the tracer's helper thread (numpy's sort and the ctypes
    call release the GIL): the input-power sum overlaps the scene and ray upload."""
    return _SUM_POOL.submit(fn, *args)


def _rot(axis):
    if axis in ("y", "Y"):
        return lambda x: np.matrix([[np.cos(x), 0, np.sin(x), 0], [0, 1, 0, 0], [-np.sin(x), 0, np.cos(x), 0],
                                    [0, 0, 0, 0]])
    if axis in ("z", "Z"):
        return lambda x: np.matrix([[np.cos(x), -np.sin(x), 0, 0], [np.sin(x), np.cos(x), 0, 0], [0, 0, 1, 0],
                                    [0, 0, 0, 0]])
    return lambda x: np.matrix([[1, 0, 0, 0], [0, np.cos(x), -np.sin(x), 0], [0, np.sin(x), np.cos(x), 0],
                                [0, 0, 0, 0]])


class CL_Tracer:
    """Iterative optical ray tracer (reference class ``CL_Tracer``)."""

    results = None
    geometry = None

    def __init__(self, platform_name="NVIDIA", device_name="770", debug=False, device=None,
                 verbose=False):
        self.debug = debug
        self.verbose = verbose
        self.platform_name, self.device_name = platform_name, device_name
        # device= (HIP ordinal) wins; else device_name selects as the reference's
        # substring loop does (:50-55); the platform is always HIP (the reference
        # falls back to its first platform when platform_name matches none)
        self.engine = Engine(device if device is not None else select_device(device_name))
        name, cus = self.engine.info()
        self.device_label = f"{name} ({cus} CUs)"
        if self.verbose:
            print("Using HIP device:", self.device_label)
        self.meshes = None
        self.tri_count = 0
        self.iteration_counts = []
        self.power_left = []
        self._aggregate = False
        self.hist_data = None

    # ------------------------------------------------------------------------
    def _flatten(self, meshes):
        """flatten_meshes(meshes), reused when this tracer last flattened the same
        mesh objects and their vertex / triangle tables and materials still hold
        the same bits (compared by digests of the tables); meshes whose tables are
        not numpy arrays are flattened every time."""
        def bits(a):
            a = np.ascontiguousarray(a)
            return array_digest(a) if a.dtype.kind in "fiu" and a.itemsize in (1, 2, 4, 8) else None

        def mat(m):
            b = m.getMaterialBuf()
            return tuple(float(np.float32(b.get(k))) for k in ("type", "IOR", "R", "dissipation"))

        cache = getattr(self, "_flat_cache", None)
        if cache is not None and len(cache[0]) == len(meshes):
            same = True
            for m, (mid, v, t, mt) in zip(meshes, cache[0]):
                V, T = getattr(m, "vertices", None), getattr(m, "triangles", None)
                if (id(m) != mid or type(V) is not np.ndarray or type(T) is not np.ndarray or
                        V.shape != v[0] or T.shape != t[0] or mat(m) != mt):
                    same = False
                    break
                bv, bt = bits(V), bits(T)
                if bv is None or bt is None or not _same_digest(bv, v) or not _same_digest(bt, t):
                    same = False
                    break
            if same:
                return cache[1]
        arrs = flatten_meshes(meshes)
        keep = []
        for m in meshes:
            V, T = getattr(m, "vertices", None), getattr(m, "triangles", None)
            bv = bits(V) if type(V) is np.ndarray else None
            bt = bits(T) if type(T) is np.ndarray else None
            if bv is None or bt is None:
                keep = None
                break
            keep.append((id(m), bv, bt, mat(m)))
        self._flat_cache = (keep, arrs) if keep is not None else None
        return arrs

    def iterative_tracer(self, light_source, meshes, trace_iterations=100, trace_until_dissipated=0.99,
                         max_ray_len=np.float32(1e3), ior_env=np.float32(1.0), keep_results=True):
        """Trace until ``trace_iterations`` bounces, until less than
        (1 - trace_until_dissipated) of the input power is left, or until no ray is
        left (iterative_tracer.py:241-391).  Returns ``self.results``."""
        max_ray_len = np.float32(max_ray_len)
        ior_env = np.float32(ior_env)
        clk = time.perf_counter
        ph = {}                                 # host-side phases of this call (self.phase_s)
        t_ph = clk()
        origin = dirs = power = None
        # results mode keeps iteration 0's origins in its results tuple: a copy, as
        # the reference's np.float32(...) is; aggregate mode only reads them
        conv = np.float32 if keep_results else (lambda a: np.asarray(a, dtype=np.float32))
        for k, light in enumerate(light_source):                       # :99-113
            if k == 0:
                origin = conv(light.rays_origin)
                dirs = conv(light.rays_dir)
                power = conv(light.rays_power)
            else:
                origin = np.append(origin, light.rays_origin, axis=0).astype(np.float32)
                dirs = np.append(dirs, light.rays_dir, axis=0).astype(np.float32)
                power = np.append(power, light.rays_power, axis=0).astype(np.float32)
        origin = np.asarray(origin, dtype=np.float32)
        dirs = np.asarray(dirs, dtype=np.float32)
        power = np.asarray(power, dtype=np.float32)
        in_pow = _background(f32_sorted_sum, power)                    # :115, beside the uploads
        pow_shape0 = power.shape
        if not keep_results:
            # aggregate mode: the rays go to the device on the engine's helper thread
            # (lpc_trace_stage_rays) while the scene records are built below
            n = self.engine.stage_rays(origin, dirs, power.reshape(-1), max_ray_len, ior_env)
        ph["sources"] = clk() - t_ph
        t_ph = clk()
        arrs = self._flatten(meshes)                                   # :121-151
        ph["flatten"] = clk() - t_ph
        t_ph = clk()
        self.engine.upload_arrays(*arrs)                                # skipped for an unchanged scene
        self.tri_count = np.int32(arrs[0].shape[0])
        self.meshes = meshes
        self.geometry = (arrs[0], arrs[1], arrs[2])
        ph["scene"] = clk() - t_ph
        t_ph = clk()
        if keep_results:
            n = self.engine.set_rays(origin, dirs, power.reshape(-1), max_ray_len, ior_env)
        ph["set_rays"] = clk() - t_ph
        t_ph = clk()
        input_power = in_pow.result()
        ph["input_power_wait"] = clk() - t_ph
        t_ph = clk()

        self.results = []
        self.iteration_counts = []
        self.power_left = []
        self._aggregate = not keep_results
        self.exact_sums = 0                     # stop tests that needed the powers (_power_decision)
        thr = (1.0 - trace_until_dissipated) * input_power              # :383
        t0 = time.time()
        try:
            if not keep_results:
                # the whole loop (:241-391) in the library: the same stop rules on the
                # device's float64 power sums, iteration i + 1 enqueued before
                # iteration i's counters arrive
                stats, _ = self.engine.run_staged(int(trace_iterations), float(thr))
                for t_iter, st in enumerate(stats):
                    self.iteration_counts.append(int(st.n_in))
                    self.power_left.append(float(st.power_next) / float(input_power) if input_power else 0.0)
                    if self.verbose:
                        print(f"iteration {t_iter + 1}: {st.n_in} rays, {st.n_reflect + st.n_refract} children "
                              f"kept, {100.0 * self.power_left[-1]:.4f} % power left")
                trace_iterations = 0                                    # the host loop below has nothing left
            for t_iter in range(int(trace_iterations)):                 # :241 (results mode)
                self.iteration_counts.append(n)
                # the results tuple (:335-355) copied to pinned host arrays on the
                # export stream while the next iterations run (complete after the
                # sync below); iteration 0's origins are the host's
                t_it = clk()
                st, ex = self.engine.iterate_export(with_origin=t_iter > 0)
                ph.setdefault("iterate_export", []).append(clk() - t_it)
                ph.setdefault("export_pool_call", []).extend(getattr(self.engine, "export_times", ()))
                org = origin if t_iter == 0 else ex["origin"]
                pw = ex["pow"].reshape(pow_shape0) if t_iter == 0 else ex["pow"]
                self.results.append((org, ex["dest"], pw, ex["meas"]))  # :355
                power_in_scene, below = self._power_decision(st, thr)    # :372, :383
                n = st.n_reflect + st.n_refract
                self.power_left.append(float(power_in_scene) / float(input_power) if input_power else 0.0)
                if self.verbose:
                    print(f"iteration {t_iter + 1}: {st.n_in} rays, {n} children kept, "
                          f"{100.0 * self.power_left[-1]:.4f} % power left")
                if below:
                    break
                if n == 0:
                    break
            ph["loop"] = clk() - t_ph
            t_ph = clk()
        finally:
            self.engine.sync()                  # the exported results arrays are complete
        ph["sync"] = clk() - t_ph
        self.phase_s = ph
        self.sim_time = time.time() - t0
        return self.results

    # float32 unit roundoff; a sequential float32 sum of n non-negative values in
    # ascending order is within 1.2 * u * S * (n + 1) / 2 of the exact sum S when
    # n * u <= 0.1 (each partial sum s_k <= k S / n, first-order error u * sum s_k,
    # the factor covers the higher-order terms)
    _U32 = 2.0 ** -24

    def _power_decision(self, st, thr):
        """The reference's stop test ``sum(np.sort(rays_pow)) < thr`` (:372, :383)
        on the next population, decided without copying its powers when the
        device's float64 sum S is farther from thr than the float32 sorted sum's
        error bound allows; otherwise the powers are fetched and summed exactly
        as the reference does.  Returns (power left, stop)."""
        n = int(st.n_reflect + st.n_refract)
        S = float(st.power_next)
        if n == 0:
            return np.float32(0.0), np.float32(0.0) < thr
        if st.power_nonneg == 1 and n * self._U32 <= 0.1:
            B = 1.2 * self._U32 * abs(S) * (n + 1) / 2.0
            if S + B < float(thr):
                return S, True
            if S - B >= float(thr):
                return S, False
        v = f32_sorted_sum(self.engine.population_power())
        self.exact_sums = getattr(self, "exact_sums", 0) + 1
        return v, v < thr

    # ------------------------------------------------------------------------
    def ray_bounces(self):
        """Rays processed over all iterations (the examples' proc_ray_count)."""
        return int(sum(self.iteration_counts))

    def measured_power(self):
        """Per-mesh measured power (float64[K]) accumulated on the device."""
        return self.engine.measured()[1]

    def get_measured_rays(self):
        """End points and powers of every ray that hit a measure surface (:395-411),
        in the reference's order; in aggregate mode (``keep_results=False``) per
        iteration in the device's traced order (see the module docstring)."""
        if self._aggregate:
            pos, pw, _ = self.engine.fetch_measured()
            return pos, pw
        pos = pwr = None
        for k, (_o, dest, pw, ms) in enumerate(self.results):
            idx = np.where(ms >= .9)[0]
            if k == 0:
                pos, pwr = dest[idx], pw[idx]
            else:
                pos = np.concatenate((pos, dest[idx]), axis=0)
                pwr = np.concatenate((pwr.flatten(), pw[idx].flatten()), axis=0)
        return pos, pwr

    def get_binned_data(self, limits=((-10, 10), (-10, 10)), points=500):
        (pos, pwr) = self.get_measured_rays()
        self.hist_data = np.histogram2d(x=pos[:, 0], y=pos[:, 1], bins=points, range=limits, weights=pwr)
        return self.hist_data

    def _project(self, mode, limits, points, rot=None, want_xy=False):
        if self._aggregate:
            return self.engine.project_hist(None, None, limits, points, mode=mode, rot=rot, want_xy=want_xy)
        pos, pwr = self.get_measured_rays()
        return self.engine.project_hist(pos, np.asarray(pwr).reshape(-1), limits, points, mode=mode, rot=rot,
                                        want_xy=want_xy)

    def get_binned_data_angular(self, limits=((-1, 1), (-1, 1)), points=500):
        """angular_project on the GPU + histogram2d binning on the GPU (:534-562)."""
        self.hist_data = tuple(self._project(0, limits, points))
        return self.hist_data

    def get_binned_data_stereographic(self, limits=((-1, 1), (-1, 1)), points=500):
        """stereograph_project on the GPU + binning (:503-531)."""
        self.hist_data = tuple(self._project(1, limits, points))
        return self.hist_data

    def replicate_lightsources_and_plot(self, limits=((-10, 10), (-10, 10)), points=500, axis="z", sources=36,
                                        use_3D=True, plot=True):
        """Emulate ``sources`` rotated copies of the source by rotating the measured rays
        (:564-657): angular_project on the GPU per rotation (R(ang) rows as the
        reference's R_dev, :601), the projected points of all rotations
        concatenated and binned once with np.histogram2d, as the reference does
        (:608-627)."""
        R = _rot(axis)
        xs, ys, ps = [], [], []
        for k in np.arange(sources):
            ang = k * 2.0 * np.pi / sources
            _, _, _, x, y, pc = self._project(0, limits, points, rot=np.asarray(R(ang), dtype=np.float32),
                                              want_xy=True)
            xs.append(x)
            ys.append(y)
            ps.append(np.float64(pc))
        x = np.concatenate(xs) if xs else np.zeros(0, np.float32)
        y = np.concatenate(ys) if ys else np.zeros(0, np.float32)
        pwr = np.concatenate(ps) if ps else np.zeros(0, np.float64)
        dx = np.float64(limits[0][1] - limits[0][0]) / np.float64(points)
        dy = np.float64(limits[1][1] - limits[1][0]) / np.float64(points)
        pwr = pwr / (dx * dy)                                           # :622-624
        H, xe, ye = np.histogram2d(x=x.flatten(), y=y.flatten(), bins=points, range=limits,
                                   weights=pwr.flatten())              # :627
        self.hist_data = (H, xe, ye)
        if plot:
            self._plot(H, xe * 180.0 / np.pi, ye * 180.0 / np.pi, use_3D, "replicated_sources")
        return self.hist_data

    def plot_binned_data(self, limits=((-10, 10), (-10, 10)), points=500, use_3d=True, use_angular=False,
                         hist_data=None):
        if hist_data is None:
            if use_angular:
                self.get_binned_data_angular(limits=limits, points=points)
            else:
                (pos, pwr) = self.get_measured_rays()
                H, xc, yc = np.histogram2d(x=np.array(pos[:, 0].flatten()), y=np.array(pos[:, 1].flatten()),
                                           bins=points, range=limits, weights=np.array(np.float64(pwr).flatten()))
                self.hist_data = (H.astype(np.float64), xc, yc)
        else:
            self.hist_data = hist_data
        H, xe, ye = self.hist_data
        self._plot(H, xe, ye, use_3d, "binned")

    @staticmethod
    def _plot(H, xe, ye, use_3d, tag):
        import matplotlib.pyplot as plt  # optional dependency
        fig = plt.figure()
        if use_3d:
            ax = fig.add_subplot(projection="3d")
            X, Y = np.meshgrid(xe[0:-1], ye[0:-1])
            ax.plot_surface(X, Y, H, rstride=1, cstride=1, linewidth=0, antialiased=False)
        else:
            plt.imshow(np.log10(H), extent=[xe[0], xe[-1], ye[0], ye[-1]], interpolation="nearest", origin="lower")
            plt.colorbar()
        plt.savefig(f"./{tag}_{'3D' if use_3d else '2D'}_data.pdf")

    def plot_elevation_histogram(self, points=500, pole=[0, 0, 1, 0]):
        (pos, pwr) = self.get_measured_rays()
        pos0 = np.array(np.divide(pos, np.matrix(np.linalg.norm(pos, axis=1)).T))
        pwr = np.float64(pwr).flatten()
        elevation = np.arccos(np.dot(pos0, pole)).flatten()
        (H, x) = np.histogram(elevation, bins=points, weights=pwr)
        x = (x[0:-1] + x[1:]) / 2.0
        dx = x[1] - x[0]
        H = H / (np.sin(x) * dx)
        import matplotlib.pyplot as plt  # optional dependency
        plt.plot(x * 180.0 / np.pi, H)
        plt.savefig("./elevation_power_distribution.pdf")
        return H, x

    def get_beam_width_half_power(self, points=500, pole=[0, 0, 1, 0]):
        """Elevation at which the cumulative measured power reaches half (:443-466)."""
        (pos, pwr0) = self.get_measured_rays()
        pos0 = np.array(np.divide(pos, np.matrix(np.linalg.norm(pos, axis=1)).T))
        pwr0 = np.float64(pwr0).reshape(-1)
        elevation0 = np.arccos(np.dot(pos0, pole)).reshape(-1)
        order = np.argsort(elevation0, kind="stable")
        elevation = elevation0[order]
        cums = np.cumsum(pwr0[order])
        half = cums[-1] / 2.0
        idx = np.where(np.absolute(cums - half) == min(np.absolute(cums - half)))
        return cums[-1], elevation[idx] / np.pi * 180.0, cums[idx] / cums[-1] * 100.0

    def get_beam_HWHM(self, points=500, pole=[0, 0, 1, 0]):
        """Half-width at half-maximum of the elevation intensity (:468-501)."""
        (pos, pwr0) = self.get_measured_rays()
        pos0 = np.array(np.divide(pos, np.matrix(np.linalg.norm(pos, axis=1)).T))
        pwr0 = np.float64(pwr0).reshape(-1)
        elevation0 = np.arccos(np.dot(pos0, pole)).reshape(-1)
        order = np.argsort(elevation0, kind="stable")
        (H, x) = np.histogram(a=elevation0[order], bins=points, weights=pwr0[order])
        x = (x[0:-1] + x[1:]) / 2.0
        H = (H.T / np.sin(x)).flatten()
        hmax = max(H) / 2.0
        idx = np.where(np.absolute(H - hmax) == min(np.absolute(H - hmax)))[0]
        el = x[idx]
        within = np.sum(pwr0[np.where(elevation0 < el)])
        return sum(pwr0), el / np.pi * 180.0, within / sum(pwr0) * 100.0

    def pickle_results(self, fname=None):
        """Pickle (results, meshes) with protocol 1 to ./<timestamp>-tracer_results.txt,
        as the reference writes them (``pickle.dumps((results, meshes), 1)``, :711-733).
        An aggregate-mode trace (``keep_results=False``) kept no per-ray results
        on the host or the device, so there is nothing the reference's loader
        could read: it raises ValueError instead of writing an empty record."""
        if self._aggregate:
            raise ValueError("pickle_results: this trace ran with keep_results=False and kept no per-ray "
                             "results; trace with keep_results=True (the reference's mode) to pickle them")
        if fname is None:
            fname = "./{0}-tracer_results.txt".format(time.strftime("%Y.%m.%d.%H.%M.%S"))
        try:
            data = pickle.dumps((self.results, self.meshes), 1)
            with open(fname, "wb") as f:
                f.write(data)
        except Exception:
            print("Pickling results failed.")
            return None
        return fname

    def load_pickle_results(self, path):
        """Load a results file written by :meth:`pickle_results` or by the reference
        (Python 2 cPickle, :735-751): byte strings decoded as latin-1 (numpy arrays of
        Python-2 pickles), the reference's module names (``geo_optical_elements``,
        ``light_source``) mapped to this package's.  Unpickling runs code named in
        the file: only load files you (or your reference runs) wrote."""
        with open(path, "rb") as f:
            (self.results, self.meshes) = _RefUnpickler(f, encoding="latin1").load()
        self._aggregate = False
        return self.results

    def save_traced_scene(self, dxf_file):
        """DXF export of rays and facets; needs the optional ``dxfwrite`` package."""
        from dxfwrite import DXFEngine as dxf  # noqa: optional dependency
        drawing = dxf.drawing(dxf_file)
        drawing.add_layer('Rays', color=3)
        drawing.add_layer('Geometry', color=5)
        for res in self.results:
            for r0, rd in zip(res[0], res[1]):
                drawing.add(dxf.face3d([r0[0:3], rd[0:3], rd[0:3]], layer="Rays"))
        for t0, t1, t2 in zip(*self.geometry):
            drawing.add(dxf.face3d([t0[0:3], t1[0:3], t2[0:3]], layer="Geometry"))
        drawing.save()


class _RefUnpickler(pickle.Unpickler):
    """Maps the reference's top-level module names to this package's modules."""
    _MAP = {"geo_optical_elements": "lightpycl_amd.geo_optical_elements",
            "light_source": "lightpycl_amd.light_source",
            "iterative_tracer": "lightpycl_amd.iterative_tracer"}

    def find_class(self, module, name):
        return super().find_class(self._MAP.get(module, module), name)


# alias with the north star's spelling
CLTracer = CL_Tracer
