"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from
the pinned oracle).  CPU: the seeded scene builders and the oracle still
reproduce them.  GPU: liblpc reproduces the first bounce bit-exactly (powers of
rays leaving a dissipative medium within 2 ulp: exp() differs between libm and
the device library) and the trace's ray counts / measured power."""
import glob
import os

import numpy as np
import pytest

from lightpycl_amd import scenes

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))
NAMES = [os.path.basename(f)[:-4] for f in FIX]
KEYS = ("dest", "pow", "meas", "isect_mid", "isect_idx", "n1", "n2", "r_dir", "r_pow", "r_meas", "t_dir",
        "t_pow", "t_meas")


def load(name):
    return dict(np.load(os.path.join(HERE, "golden", name + ".npz")))


def _compare(got, g, name):
    for k in KEYS:
        a = got[k][:, :3] if got[k].ndim == 2 and got[k].shape[1] == 4 else got[k]
        b = g["b_" + k]
        if name == "cube" and k in ("pow", "r_pow", "t_pow"):
            np.testing.assert_allclose(a, b, rtol=4e-7, atol=0, err_msg=k)
        else:
            np.testing.assert_array_equal(a, b, err_msg=f"{name}:{k}")


@pytest.mark.parametrize("name", NAMES)
def test_builders_and_oracle_reproduce_fixture(oracle_mod, name):
    g = load(name)
    n, seed = int(g["n"]), int(g["seed"])
    sc = scenes.BUILDERS[name](n=n, seed=seed)
    np.testing.assert_array_equal(np.asarray(sc.sources[0].rays_origin, np.float32), g["origin"])
    np.testing.assert_array_equal(np.asarray(sc.sources[0].rays_dir, np.float32), g["dir"])
    S = oracle_mod.Scene(sc.meshes)
    assert S.tri_count == int(g["tri_count"])
    b = oracle_mod.bounce(S, g["origin"], g["dir"], g["pow_in"], np.zeros(n, np.int32), np.full(n, -2, np.int32),
                          g["max_ray_len"], g["ior_env"])
    _compare(b, g, "oracle")


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_fixture(engine, name):
    g = load(name)
    n, seed = int(g["n"]), int(g["seed"])
    sc = scenes.BUILDERS[name](n=n, seed=seed)
    engine.upload_meshes(sc.meshes)
    b = engine.bounce(g["origin"], g["dir"], g["pow_in"], np.zeros(n, np.int32), np.full(n, -2, np.int32),
                      g["max_ray_len"], g["ior_env"])
    _compare(b, g, name)
    engine.set_rays(g["origin"], g["dir"], g["pow_in"], g["max_ray_len"], g["ior_env"])
    from lightpycl_amd.distributed import ShardedTrace
    r = ShardedTrace(engine).run(sc.iterations, sc.tau, float(np.sum(g["pow_in"], dtype=np.float64)))
    assert r["global_counts"] == list(g["counts"])
    np.testing.assert_allclose(r["mesh_power"], g["mesh_power"], rtol=1e-6 if name == "cube" else 1e-12)
