"""Test double: an engine with the lightpycl_amd.engine.Engine trace interface
(iterate / measured) whose bounce is the CPU oracle.  TEST INFRASTRUCTURE ONLY --
used to exercise the sharded multi-process driver over gloo on CPU."""
from types import SimpleNamespace

import numpy as np

import oracle


class OracleEngine:
    def __init__(self, meshes, origin4, dir4, power, max_ray_len, ior_env):
        self.S = oracle.Scene(meshes)
        self.o = np.ascontiguousarray(origin4, np.float32)
        self.d = np.ascontiguousarray(dir4, np.float32)
        self.p = np.ascontiguousarray(power, np.float32).reshape(-1)
        self.pm = np.full(self.p.shape[0], -2, np.int32)
        self.mrl, self.ior = np.float32(max_ray_len), np.float32(ior_env)
        self.mesh_power = np.zeros(self.S.mesh_count, np.float64)
        self.count = 0
        self.pos, self.pwr = [], []

    def iterate(self):
        n = self.p.shape[0]
        if n == 0:
            return SimpleNamespace(n_in=0, n_reflect=0, n_refract=0, n_measured=0, power_next=0.0), None
        out = oracle.bounce(self.S, self.o, self.d, self.p, np.zeros(n, np.int32), self.pm, self.mrl, self.ior)
        m = out["meas"] == 1
        np.add.at(self.mesh_power, out["isect_mid"][m], out["pow"][m].astype(np.float64))
        self.count += int(m.sum())
        self.pos.append(out["dest"][m])
        self.pwr.append(out["pow"][m])
        kr, kt = out["r_meas"] == 0, out["t_meas"] == 0
        self.o = np.concatenate((out["r_origin"][kr], out["t_origin"][kt]))
        self.d = np.concatenate((out["r_dir"][kr], out["t_dir"][kt]))
        self.p = np.concatenate((out["r_pow"][kr], out["t_pow"][kt]))
        self.pm = np.concatenate((out["isect_mid"][kr], out["isect_mid"][kt]))
        st = SimpleNamespace(n_in=n, n_reflect=int(kr.sum()), n_refract=int(kt.sum()), n_measured=int(m.sum()),
                             power_next=float(np.sum(self.p, dtype=np.float64)))
        return st, None

    def measured(self):
        return self.count, self.mesh_power

    def project_hist(self, pos4, pwr, limits, points):
        """get_binned_data_angular over the measured record (pos4=None) or the given rays."""
        if pos4 is None:
            pos4 = np.concatenate(self.pos) if self.pos else np.zeros((0, 4), np.float32)
            pwr = np.concatenate(self.pwr) if self.pwr else np.zeros(0, np.float32)
        return oracle.binned_angular(pos4, pwr, limits, points)
