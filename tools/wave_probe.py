"""GPU box: per-wave cost of the grid traversal (k_intersect, prof level 3) on
one bounce of a scene: distribution of wave durations, the heaviest waves and
what they did (nodes visited, exact tests), and time per piece."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightpycl_amd import scenes  # noqa: E402
from lightpycl_amd.engine import Engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "synthetic"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
level = int(sys.argv[3]) if len(sys.argv) > 3 else 0      # 0 primaries; k: k-th bounce population
sc = scenes.BUILDERS[name](n=n, seed=7)
o = np.concatenate([np.asarray(s.rays_origin, np.float32) for s in sc.sources])
d = np.concatenate([np.asarray(s.rays_dir, np.float32) for s in sc.sources])
p = np.concatenate([np.asarray(s.rays_power, np.float32).reshape(-1) for s in sc.sources])
e = Engine(0)
e.upload_meshes(sc.meshes)
e.set_rays(o, d, p, sc.max_ray_len, sc.ior_env)
for it in range(level + 1):
    e.prof_enable(True, waves=(it == level))
    e.prof_read(reset=True)
    nin = e.population()
    st, _ = e.iterate()
    pr = e.prof_read(reset=True)
rec = e.prof_waves().astype(np.int64)
us = rec[:, 0] / 100.0
live = rec[:, 1] > 0
print(f"{name} level {level}: {nin} rays, intersect stage {pr['intersect_ms']:.3f} ms, "
      f"{rec.shape[0]} (piece, packet) waves, {live.sum()} past the root")
q = np.percentile(us[live], [50, 90, 99, 99.9, 100]) if live.any() else []
print("wave us p50/p90/p99/p99.9/max:", " ".join(f"{v:.1f}" for v in q))
print(f"sum of wave time {us.sum() / 1e3:.2f} ms; nodes {rec[:, 1].sum()}, exact {rec[:, 2].sum()}; "
      f"sum / 7168 resident waves = {us.sum() / 7168 / 1e3:.3f} ms; "
      f"us per node (waves without exact tests) {np.median(us[live & (rec[:, 2] == 0)] / np.maximum(rec[live & (rec[:, 2] == 0), 1], 1)) if (live & (rec[:, 2] == 0)).any() else 0:.2f}")
big = live & (rec[:, 2] > 0)
if big.any():
    A = np.stack([rec[big, 1], rec[big, 2], np.ones(big.sum())], 1).astype(np.float64)
    coef = np.linalg.lstsq(A, us[big], rcond=None)[0]
    print(f"fit wave us = {coef[0]:.3f}*nodes + {coef[1]:.4f}*exact + {coef[2]:.2f}")
order = np.argsort(-us)[:15]
for i in order:
    print(f"  piece {rec[i, 3]:4d} packet {i % max(1, (nin + 63) // 64):7d}: {us[i]:8.1f} us  "
          f"nodes {rec[i, 1]:5d}  exact {rec[i, 2]:6d}")
pieces = np.unique(rec[:, 3])
per = [(us[rec[:, 3] == k].sum(), us[rec[:, 3] == k].max(), k) for k in pieces]
for tot, mx, k in sorted(per, reverse=True)[:12]:
    print(f"  piece {k:4d}: sum {tot / 1e3:7.2f} ms  max {mx:8.1f} us")

if level == 0 and name == "synthetic":
    # reproduce the coherence order on the host (k_raykey, key mode 0; the radix
    # sort is stable) and locate the heaviest packets on their sphere
    def spread2(x):
        x = x & 0xff
        x = (x | (x << 4)) & 0x0f0f
        x = (x | (x << 2)) & 0x3333
        return (x | (x << 1)) & 0x5555
    dd = d[:, :3].astype(np.float32)
    l1 = np.abs(dd).sum(1)
    px, py = dd[:, 0] / l1, dd[:, 1] / l1
    neg = dd[:, 2] < 0
    tx = (1 - np.abs(py)) * np.where(px >= 0, 1, -1)
    ty = (1 - np.abs(px)) * np.where(py >= 0, 1, -1)
    px, py = np.where(neg, tx, px), np.where(neg, ty, py)
    du = np.clip((px * 0.5 + 0.5) * 256, 0, 255).astype(np.uint32)
    dv = np.clip((py * 0.5 + 0.5) * 256, 0, 255).astype(np.uint32)
    key = spread2(du) | (spread2(dv) << 1)
    perm = np.argsort(key, kind="stable")
    npk = (nin + 63) // 64
    for i in order[:10]:
        w, piece = i % npk, rec[i, 3]
        rays = perm[w * 64:(w + 1) * 64]
        u = dd[rays] / np.linalg.norm(dd[rays], axis=1, keepdims=True)
        m = sc.meshes[piece] if piece < len(sc.meshes) else None
        ctr = np.asarray(m.tribuf()[0], np.float32).reshape(-1, 4)[:, :3].mean(0) if m is not None else np.zeros(3)
        tc = u @ ctr
        miss = np.linalg.norm(ctr[None] - tc[:, None] * u, axis=1)
        ang = np.degrees(np.arccos(np.clip(u @ u.mean(0) / np.linalg.norm(u.mean(0)), -1, 1))).max()
        # closest approach point relative to the sphere centre (x axis = revolve axis)
        rel = tc[:, None] * u - ctr[None]
        print(f"  heavy piece {piece} packet {w}: spread {ang:.3f} deg, line-centre distance "
              f"{miss.min():.2f}..{miss.max():.2f}, rel mean {np.round(rel.mean(0), 2)}")
