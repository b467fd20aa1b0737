"""Trace-end post-processing on the GPU against the reference's own kernels
(SURVEY.md section 8 row f3): get_binned_data_stereographic
(iterative_tracer.py:503-531, stereograph_project .cl:488-506) and
replicate_lightsources_and_plot (:564-628: 36 rotated angular_project passes,
points concatenated, binned once)."""
import numpy as np
import pytest

from lightpycl_amd import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def traced(exact_ref):
    if exact_ref is None:
        pytest.skip("oracle/_ref not built")
    from lightpycl_amd.iterative_tracer import CL_Tracer
    sc = scenes.lens(n=4000, seed=9)
    out = {}
    for keep in (True, False):
        tr = CL_Tracer(device=0)
        tr.iterative_tracer(sc.sources, sc.meshes, trace_iterations=sc.iterations, trace_until_dissipated=sc.tau,
                            max_ray_len=sc.max_ray_len, ior_env=sc.ior_env, keep_results=keep)
        out[keep] = tr
    return out


@pytest.mark.parametrize("keep", [True, False])
def test_stereographic_binning_vs_reference(traced, exact_ref, keep):
    tr = traced[keep]
    lim, pts = ((-1.0, 1.0), (-1.0, 1.0)), 40
    H, xe, ye = tr.get_binned_data_stereographic(limits=lim, points=pts)
    pos, pwr = tr.get_measured_rays()
    x, y, pc = exact_ref.project(pos, np.asarray(pwr).reshape(-1), "stereo")
    dx = np.float64(lim[0][1] - lim[0][0]) / np.float64(pts)
    dy = np.float64(lim[1][1] - lim[1][0]) / np.float64(pts)
    Hr, xr, yr = np.histogram2d(x=x, y=y, bins=pts, range=lim, weights=np.float64(pc) / (dx * dy))
    np.testing.assert_array_equal(xe, xr)
    np.testing.assert_array_equal(ye, yr)
    assert Hr.sum() > 0
    # device binning: float64 atomics (summation order only)
    np.testing.assert_allclose(H, Hr, rtol=1e-12, atol=1e-12 * np.abs(Hr).max())


@pytest.mark.parametrize("keep,axis,sources", [(True, "z", 36), (False, "z", 12), (True, "x", 7)])
def test_replicated_sources_vs_reference(traced, exact_ref, keep, axis, sources):
    from lightpycl_amd.iterative_tracer import _rot
    tr = traced[keep]
    lim, pts = ((-np.pi / 2, np.pi / 2), (-np.pi / 2, np.pi / 2)), 30
    H, xe, ye = tr.replicate_lightsources_and_plot(limits=lim, points=pts, axis=axis, sources=sources, plot=False)
    pos, pwr = tr.get_measured_rays()
    R = _rot(axis)
    xs, ys, ps = [], [], []
    for k in np.arange(sources):                       # the reference's loop, :598-615
        ang = k * 2.0 * np.pi / sources
        x, y, pc = exact_ref.project(pos, np.asarray(pwr).reshape(-1), "angular",
                                     rot=np.asarray(R(ang), dtype=np.float32))
        xs.append(x)
        ys.append(y)
        ps.append(np.float64(pc))
    dx = np.float64(lim[0][1] - lim[0][0]) / np.float64(pts)
    dy = np.float64(lim[1][1] - lim[1][0]) / np.float64(pts)
    pw = np.concatenate(ps) / (dx * dy)
    Hr, xr, yr = np.histogram2d(x=np.concatenate(xs), y=np.concatenate(ys), bins=pts, range=lim, weights=pw)
    assert Hr.sum() > 0
    np.testing.assert_array_equal(H, Hr)               # same points, same binning: bit for bit
    np.testing.assert_array_equal(xe, xr)
