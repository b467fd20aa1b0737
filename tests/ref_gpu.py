"""The REFERENCE's own OpenCL kernels on the GPU -- TEST INFRASTRUCTURE ONLY.

``oracle/Makefile`` (target ``ref``) compiles the unmodified
``/root/reference/kernel_reflect_refract_intersect.cl`` for gfx950 with ROCm's
OpenCL C front end and ROCm's own OpenCL device libraries into
``oracle/_ref/lpc_ref_{stock,ieee}.co``.  This module loads such a code object
with ``hipModuleLoad`` and launches its kernels with exactly the argument lists
the reference's host passes (``/root/reference/iterative_tracer.py:288-326``
for the three per-bounce kernels, ``:546`` for ``angular_project``), on device
buffers in the reference's layouts: float3 arrays as 16-byte ``(n,4)`` rows,
per-(ray, mesh) scratch as ``[ray][mesh]``.

It is the parity pin of DESIGN.md section 3: the product (``lightpycl_amd``)
never loads it; tests compare liblpc and the CPU oracle against it.

The reference launches ``(n,)`` work-items with no bounds check in the kernels
(``.cl:114,247,360``); here every per-ray buffer is padded to a whole number of
64-lane blocks and the padding rows are dropped from the outputs.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")
VARIANTS = ("stock", "ieee")
BLOCK = 64


def code_object(variant="stock"):
    return os.path.join(REF_DIR, f"lpc_ref_{variant}.co")


def available(variant="stock"):
    return os.path.exists(code_object(variant))


def _hip():
    """The HIP runtime torch already uses (one runtime per process, as liblpc)."""
    import torch  # noqa: F401  (loads torch/lib/libamdhip64.so)
    cand = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    L = ctypes.CDLL(cand if os.path.exists(cand) else "libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    L.hipModuleLoad.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    L.hipModuleGetFunction.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p]
    L.hipModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint] * 6 + [
        ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.hipModuleUnload.argtypes = [ctypes.c_void_p]
    L.hipDeviceSynchronize.argtypes = []
    L.hipGetErrorString.restype = ctypes.c_char_p
    return L


def _ok(L, rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc} {L.hipGetErrorString(rc).decode()}")


class RefKernels:
    """One loaded reference code object (``variant`` stock or ieee) on cuda:0."""

    def __init__(self, variant="stock", device=0):
        import torch
        self.torch = torch
        self.dev = torch.device("cuda", device)
        torch.cuda.set_device(device)
        torch.zeros(1, device=self.dev)              # context up before hipModuleLoad
        self.L = _hip()
        self.mod = ctypes.c_void_p()
        _ok(self.L, self.L.hipModuleLoad(ctypes.byref(self.mod), code_object(variant).encode()),
            "hipModuleLoad")
        self.fn = {}
        for name in ("intersect", "intersect_postproc", "reflect_refract_rays", "angular_project",
                     "stereograph_project"):
            f = ctypes.c_void_p()
            _ok(self.L, self.L.hipModuleGetFunction(ctypes.byref(f), self.mod, name.encode()), name)
            self.fn[name] = f
        self.variant = variant

    # -- plumbing ---------------------------------------------------------------
    def _launch(self, name, n_pad, args):
        """args: list of ('p', tensor) | ('i', int) | ('f', float) in kernel order."""
        keep = []
        ptrs = (ctypes.c_void_p * len(args))()
        for i, (kind, v) in enumerate(args):
            if kind == "p":
                c = ctypes.c_void_p(v.data_ptr())
            elif kind == "i":
                c = ctypes.c_int32(int(v))
            else:
                c = ctypes.c_float(float(v))
            keep.append(c)
            ptrs[i] = ctypes.cast(ctypes.byref(c), ctypes.c_void_p)
        grid = n_pad // BLOCK
        self.torch.cuda.synchronize(self.dev)
        _ok(self.L, self.L.hipModuleLaunchKernel(self.fn[name], grid, 1, 1, BLOCK, 1, 1, 0, None,
                                                 ptrs, None), name)
        _ok(self.L, self.L.hipDeviceSynchronize(), name + " (sync)")

    def _dev(self, a, n_pad=None, fill=0):
        a = np.ascontiguousarray(a)
        if n_pad is not None and a.shape[0] < n_pad:
            pad = np.full((n_pad - a.shape[0],) + a.shape[1:], fill, a.dtype)
            a = np.concatenate([a, pad])
        return self.torch.from_numpy(a).to(self.dev)

    def _zeros(self, shape, dtype):
        t = {np.float32: self.torch.float32, np.int32: self.torch.int32}[dtype]
        return self.torch.zeros(shape, dtype=t, device=self.dev)

    def upload_scene(self, scene):
        """oracle.Scene (the reference's flattened arrays, iterative_tracer.py:121-169)."""
        self.scene = scene
        self.v0, self.v1, self.v2 = (self._dev(np.asarray(a, np.float32).reshape(-1, 4))
                                     for a in (scene.v0, scene.v1, scene.v2))
        self.mid = self._dev(np.asarray(scene.mesh_id, np.int32))
        self.typ = self._dev(np.asarray(scene.mat_type, np.int32))
        self.ior = self._dev(np.asarray(scene.ior, np.float32))
        self.refl = self._dev(np.asarray(scene.refl, np.float32))
        self.diss = self._dev(np.asarray(scene.diss, np.float32))

    # -- the partition-loop body, iterative_tracer.py:267-348 --------------------
    def bounce(self, scene, origin, direction, power, meas, prev_mid, max_ray_len=1e3, ior_env=1.0):
        """Same signature and outputs as ``oracle.bounce``."""
        if getattr(self, "scene", None) is not scene:
            self.upload_scene(scene)
        n = int(np.asarray(prev_mid).shape[0])
        K = int(scene.mesh_count)
        M = int(scene.tri_count)
        mrl = np.float32(max_ray_len)
        if n == 0:
            z4 = np.zeros((0, 4), np.float32)
            zi = np.zeros(0, np.int32)
            zf = np.zeros(0, np.float32)
            return dict(dest=z4, pow=zf, meas=zi, isect_mid=zi, isect_idx=zi, n1=zi, n2=zi, entering=zi,
                        r_origin=z4, r_dir=z4, r_pow=zf, r_meas=zi, t_origin=z4, t_dir=z4, t_pow=zf,
                        t_meas=zi, isect_min_ray_len=np.zeros((0, K), np.float32),
                        isects_count=np.zeros((0, K), np.int32), isect_idx_tmp=np.zeros((0, K), np.int32))
        n_pad = -(-n // BLOCK) * BLOCK
        F, I = np.float32, np.int32
        o = self._dev(np.asarray(origin, F).reshape(-1, 4), n_pad)
        d = self._dev(np.asarray(direction, F).reshape(-1, 4), n_pad)
        pw = self._dev(np.asarray(power, F).reshape(-1), n_pad)
        ms = self._dev(np.asarray(meas, I).reshape(-1), n_pad)
        pm = self._dev(np.asarray(prev_mid, I).reshape(-1), n_pad, fill=-2)
        dest = self._zeros((n_pad, 4), F)
        ent, imid, iidx, n1, n2 = (self._zeros(n_pad, I) for _ in range(5))
        tmin = self._zeros((n_pad, K), F) + float(mrl)                 # :267
        cnt = self._zeros((n_pad, K), I)                               # :236
        itmp = self._zeros((n_pad, K), I)                              # :237
        # prg.intersect, :288-294
        self._launch("intersect", n_pad, [
            ("p", o), ("p", d), ("p", dest), ("p", ent), ("p", imid), ("p", iidx), ("p", self.v0),
            ("p", self.v1), ("p", self.v2), ("p", self.mid), ("p", tmin), ("p", cnt), ("p", itmp),
            ("i", K), ("i", M), ("i", n), ("f", mrl)])
        # prg.intersect_postproc, :303-309
        self._launch("intersect_postproc", n_pad, [
            ("p", o), ("p", d), ("p", dest), ("p", pm), ("p", n1), ("p", n2), ("p", ent), ("p", imid),
            ("p", iidx), ("p", self.v0), ("p", self.v1), ("p", self.v2), ("p", self.mid), ("p", self.typ),
            ("p", tmin), ("p", cnt), ("p", itmp), ("i", K), ("i", n), ("f", mrl)])
        ro, rd, to, td = (self._zeros((n_pad, 4), F) for _ in range(4))
        rp, tp = self._zeros(n_pad, F), self._zeros(n_pad, F)
        rm, tm = self._zeros(n_pad, I), self._zeros(n_pad, I)
        # prg.reflect_refract_rays, :318-325
        self._launch("reflect_refract_rays", n_pad, [
            ("p", o), ("p", dest), ("p", d), ("p", pw), ("p", ms), ("p", ent), ("p", n1), ("p", n2),
            ("p", ro), ("p", rd), ("p", rp), ("p", rm), ("p", to), ("p", td), ("p", tp), ("p", tm),
            ("p", imid), ("p", iidx), ("p", self.v0), ("p", self.v1), ("p", self.v2), ("p", self.mid),
            ("p", self.typ), ("p", self.ior), ("p", self.refl), ("p", self.diss), ("f", ior_env),
            ("i", K), ("i", n), ("f", mrl)])
        h = lambda t: t.cpu().numpy()[:n]
        return dict(dest=h(dest), pow=h(pw), meas=h(ms), isect_mid=h(imid), isect_idx=h(iidx), n1=h(n1),
                    n2=h(n2), entering=h(ent), r_origin=h(ro), r_dir=h(rd), r_pow=h(rp), r_meas=h(rm),
                    t_origin=h(to), t_dir=h(td), t_pow=h(tp), t_meas=h(tm), isect_min_ray_len=h(tmin),
                    isects_count=h(cnt), isect_idx_tmp=h(itmp))

    # -- projections, iterative_tracer.py:503-562 --------------------------------
    def project(self, pos, pwr, mode="angular", rot=None, pivot=None):
        n = int(np.asarray(pwr).reshape(-1).shape[0])
        if n == 0:
            z = np.zeros(0, np.float32)
            return z, z, z
        n_pad = -(-n // BLOCK) * BLOCK
        # R_dev rows as iterative_tracer.py:514/545 uploads them (row 3 = 0)
        if rot is None:
            rot = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 0]], np.float32)
        rot = np.ascontiguousarray(np.asarray(rot, np.float32).reshape(4, 4))
        piv = np.zeros((1, 4), np.float32) if pivot is None else np.asarray(pivot, np.float32).reshape(1, 4)
        p = self._dev(np.asarray(pos, np.float32).reshape(-1, 4), n_pad)
        w = self._dev(np.asarray(pwr, np.float32).reshape(-1), n_pad)
        R = self._dev(rot)
        P = self._dev(piv)
        x, y, pc = (self._zeros(n_pad, np.float32) for _ in range(3))
        name = "angular_project" if mode == "angular" else "stereograph_project"
        self._launch(name, n_pad, [("p", p), ("p", w), ("p", R), ("p", P), ("p", x), ("p", y), ("p", pc)])
        return tuple(t.cpu().numpy()[:n] for t in (x, y, pc))

    def binned_angular(self, pos, pwr, limits, points):
        """get_binned_data_angular (iterative_tracer.py:534-562) with the reference's
        angular_project kernel."""
        x, y, pc = self.project(pos, pwr)
        pw = np.float64(pc)
        dx = np.float64(limits[0][1] - limits[0][0]) / np.float64(points)
        dy = np.float64(limits[1][1] - limits[1][0]) / np.float64(points)
        return np.histogram2d(x=x, y=y, bins=points, range=limits, weights=pw / (dx * dy))

    def close(self):
        if getattr(self, "mod", None):
            self.L.hipModuleUnload(self.mod)
            self.mod = None
