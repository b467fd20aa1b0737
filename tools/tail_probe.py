"""GPU box: where does the intersect stage's fixed cost come from?  Bounces
subsets of the synthetic scene's primary rays (elevation bands, rays that pass
near a sphere vs. not) and prints the intersect-stage time of each subset."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
sc = scenes.synthetic(n=n, seed=7)
o = np.asarray(sc.sources[0].rays_origin, np.float32)
d = np.asarray(sc.sources[0].rays_dir, np.float32)
p = np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1)
e = Engine(0)
e.upload_meshes(sc.meshes)
e.prof_enable(True)


def run(mask, label):
    idx = np.where(mask)[0]
    if idx.size == 0:
        return
    z = np.zeros(idx.size, np.int32)
    pm = np.full(idx.size, -2, np.int32)
    best = None
    for _ in range(3):
        e.prof_read(reset=True)
        e.bounce(o[idx], d[idx], p[idx], z, pm, sc.max_ray_len, sc.ior_env)
        t = e.prof_read(reset=True)["intersect_ms"]
        best = t if best is None else min(best, t)
    print(f"{label:40s} rays {idx.size:8d}  intersect {best:7.3f} ms", flush=True)


run(np.ones(n, bool), "all")
th = np.degrees(np.arccos(np.clip(d[:, 2] / np.linalg.norm(d[:, :3], axis=1), -1, 1)))
for a, b in ((0, 5), (5, 10), (10, 20), (20, 30), (30, 45), (45, 60), (60, 75), (75, 90)):
    run((th >= a) & (th < b), f"elevation from +z in [{a},{b}) deg")
# rays whose line passes within 12 units of a sphere centre (they meet a sphere)
near = np.zeros(n, bool)
u = d[:, :3] / np.linalg.norm(d[:, :3], axis=1, keepdims=True)
for m in sc.meshes[1:]:
    v = np.asarray(m.tribuf()[0], np.float32).reshape(-1, 4)[:, :3]
    c = v.mean(0)
    tc = u @ c
    dist = np.linalg.norm(c[None, :] - tc[:, None] * u, axis=1)
    near |= (dist < 12.0) & (tc > 0)
run(near, "near a sphere")
run(~near, "not near a sphere")
for w in (64, 256, 1024, 4096):
    run(np.arange(n) < w, f"first {w} rays")
