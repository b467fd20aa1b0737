"""Run tools/rsq_probe (gfx950 v_rsq_f32 / v_sqrt_f32 over every float in [1, 4))
into a scratch file and compare with correctly rounded 1/sqrt(x) and sqrt(x).
Prints one JSON line: mismatch counts and the first few mismatching inputs."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
with tempfile.TemporaryDirectory() as d:
    f = os.path.join(d, "p.bin")
    subprocess.run([os.path.join(here, "rsq_probe"), f], check=True, timeout=60)
    raw = np.fromfile(f, dtype=np.uint32)
n = 1 << 24
rsq = raw[:n].view(np.float32)
sq = raw[n:].view(np.float32)
x = (np.uint32(0x3f800000) + np.arange(n, dtype=np.uint32)).view(np.float32)
xd = x.astype(np.float64)
# correctly rounded references: float64 has 29 spare bits, so rounding the
# float64 result to float32 is wrong only within 2^-29 ulp of a midpoint
r_ref = (1.0 / np.sqrt(xd)).astype(np.float32)
s_ref = np.sqrt(x)                      # IEEE float32 sqrt
def near_mid(v64):
    f = v64.astype(np.float32).astype(np.float64)
    u = np.spacing(v64.astype(np.float32)).astype(np.float64)
    frac = np.abs(v64 - f) / u
    return np.abs(frac - 0.5) < 1e-6
amb_r = int(np.sum(near_mid(1.0 / np.sqrt(xd))))
bad_r = np.nonzero(rsq != r_ref)[0]
bad_s = np.nonzero(sq != s_ref)[0]
ulp_r = np.abs(rsq.view(np.int32).astype(np.int64) - r_ref.view(np.int32).astype(np.int64))
print(json.dumps(dict(inputs=n, rsq_mismatch=int(bad_r.size), rsq_max_ulp=int(ulp_r.max()),
                      rsq_ambiguous=amb_r, sqrt_mismatch=int(bad_s.size),
                      rsq_examples=[[float(x[i]), float(rsq[i]), float(r_ref[i])] for i in bad_r[:5]],
                      sqrt_examples=[[float(x[i]), float(sq[i]), float(s_ref[i])] for i in bad_s[:5]])))
