"""Generate tests/golden/*.npz: small seeded cases of the per-bounce path whose
outputs come from the REFERENCE's own kernels -- the unmodified
kernel_reflect_refract_intersect.cl compiled for gfx950 (oracle/_ref, built by
`make -C oracle ref`), launched with the reference host's argument lists
(tests/ref_gpu.py) and driven by the reference's host loop restated in
oracle.trace.  Needs a GPU (run on the GPU box):

    python tests/golden/make_golden.py            # reference kernels, ieee build
    python tests/golden/make_golden.py --oracle   # the CPU oracle instead (no GPU)

Each fixture holds the inputs (so a test can run from the fixture alone), the
first-bounce outputs, the trace's per-iteration ray counts and the per-mesh
measured power, plus the stock build's counts and power (`stock_*`: the same
source built with OpenCL's default fp options, what PyOpenCL would run).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.dirname(HERE)]

import oracle  # noqa: E402
from lightpycl_amd import scenes  # noqa: E402

CASES = [("parabolic", 1500, 21), ("lens", 1500, 22), ("eye", 400, 23), ("cube", 1500, 24),
         ("nested_cubes", 10, 25), ("synthetic", 300, 26)]
BOUNCE_KEYS = ("dest", "pow", "meas", "isect_mid", "isect_idx", "n1", "n2", "r_dir", "r_pow", "r_meas", "t_dir",
               "t_pow", "t_meas")


def make(name, n, seed, bounce, extra=None):
    sc = scenes.BUILDERS[name](n=n, seed=seed)
    o = np.asarray(sc.sources[0].rays_origin, np.float32)
    d = np.asarray(sc.sources[0].rays_dir, np.float32)
    p = np.asarray(sc.sources[0].rays_power, np.float32).reshape(-1)
    S = oracle.Scene(sc.meshes)
    b = bounce(S, o, d, p, np.zeros(n, np.int32), np.full(n, -2, np.int32), sc.max_ray_len, sc.ior_env)
    _, info = oracle.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                           keep_results=False, bounce_fn=bounce)
    arrs = dict(origin=o, dir=d, pow_in=p, max_ray_len=np.float32(sc.max_ray_len), ior_env=np.float32(sc.ior_env),
                counts=np.asarray(info["counts"], np.int64), mesh_power=info["mesh_power"],
                tri_count=np.int64(S.tri_count))
    for k in BOUNCE_KEYS:
        v = b[k]
        arrs["b_" + k] = v[:, :3] if v.ndim == 2 and v.shape[1] == 4 else v
    if extra is not None:
        _, info2 = oracle.trace(sc.sources, sc.meshes, sc.iterations, sc.tau, sc.max_ray_len, sc.ior_env,
                                keep_results=False, bounce_fn=extra)
        arrs["stock_counts"] = np.asarray(info2["counts"], np.int64)
        arrs["stock_mesh_power"] = info2["mesh_power"]
    return arrs


if __name__ == "__main__":
    oracle.build()
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else HERE
    os.makedirs(out, exist_ok=True)
    if "--oracle" in sys.argv:
        bounce, extra, source = oracle.bounce, None, "oracle"
    else:
        import ref_gpu
        ieee, stock = ref_gpu.RefKernels("ieee"), ref_gpu.RefKernels("stock")
        bounce, extra, source = ieee.bounce, stock.bounce, "reference kernels (gfx950, ieee build)"
    for name, n, seed in CASES:
        np.savez_compressed(os.path.join(out, f"{name}.npz"), seed=seed, n=n, source=source,
                            **make(name, n, seed, bounce, extra))
        print("wrote", name, "from", source)
