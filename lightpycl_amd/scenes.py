"""Workload scenes: the reference's example scenes (BASELINE.json configs) and the
synthetic ~100k-triangle benchmark scene, built only through the drop-in
light_source / geo_optical_elements API.

Each builder seeds numpy (``np.random.seed(seed)``) before creating its light
source, exactly as the SURVEY.md probes did, and returns a :class:`SceneSpec`.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import geo_optical_elements as goe
from . import light_source as lsrc


@dataclass
class SceneSpec:
    name: str
    sources: list
    meshes: list
    max_ray_len: np.float32
    ior_env: np.float32 = np.float32(1.0)
    iterations: int = 16
    tau: float = 0.99
    hist_limits: tuple = ((-np.pi / 2, np.pi / 2), (-np.pi / 2, np.pi / 2))
    hist_points: int = 30
    meta: dict = field(default_factory=dict)


def parabolic(n=10000, seed=1, iterations=16):
    """example_directivity_parabolic_mirror.py:41-91 (BASELINE configs 1-2)."""
    np.random.seed(seed)
    oe = goe.optical_elements()
    ls0 = lsrc.light_source(center=np.array([0, 0, 0, 0], dtype=np.float32), direction=(0, 0, -1),
                            directivity=lambda x, y: np.cos(y), power=1.0, ray_count=n)
    ms = oe.hemisphere(center=[0, 0, 0, 0], radius=500.0)
    ms.setMaterial(mat_type="measure")
    m2 = oe.parabolic_mirror(focus=(0, 0, 0), focal_length=5.0, diameter=20.0, reflectivity=0.98)
    m2.rotate(axis="y", angle=-np.pi / 2, pivot=(0, 0, 0, 0))
    return SceneSpec("parabolic", [ls0], [ms, m2], np.float32(1e3), iterations=iterations,
                     hist_limits=((-np.pi / 2.0, np.pi / 2.0), (-np.pi / 2.0, np.pi / 2.0)),
                     hist_points=100)


def lens(n=10000, seed=1, iterations=16):
    """example_directivity_lens.py:167-195 (BASELINE config 3)."""
    np.random.seed(seed)
    oe = goe.optical_elements()
    ls0 = lsrc.light_source(center=np.array([0, 0, 0, 0], dtype=np.float32), direction=(0, 0, 1),
                            directivity=lambda x, y: np.cos(y), power=1000., ray_count=n)
    ms = oe.hemisphere(center=[0, 0, 0, 0], radius=1000.0)
    ms.setMaterial(mat_type="measure")
    m2 = oe.lens_spherical_biconcave(focus=(0, 0, 0), r1=60., r2=6000., diameter=50.0, IOR=2.5)
    m2.rotate(axis="y", angle=-np.pi / 2.0, pivot=(0, 0, 0, 0))
    return SceneSpec("lens", [ls0], [ms, m2], np.float32(2e3), iterations=iterations,
                     hist_points=30)


def eye(n=10000, seed=1, iterations=16):
    """example_human_eye.py:278-341 (BASELINE config 4): collimated source, nested
    refractive media (cornea, lens, aqueous and vitreous humour), retina = measure."""
    np.random.seed(seed)
    oe = goe.optical_elements()
    ls0 = lsrc.light_source(center=np.array([0, 0, -10, 0], dtype=np.float32), direction=(0, 0.01, 1),
                            directivity=lambda x, y: 1.0 + 0.0 * np.cos(y), power=1000., ray_count=n)
    ls0.random_collimated_rays(diameter=5.0)
    r_cornea = r_lens = 5.0
    r_ac, d_ac, r_pc, d_pc = 7.8, 0.0, 6.5, 0.55
    r_al, d_al, r_pl, d_pl = 10.2, 3.6, -6.0, 7.6
    r_r, d_r = -12.1, 24.2
    retina = oe.hemisphere(center=[0, 0, d_r / 2.0, 0], radius=-r_r * (1.0 - 1e-3))
    retina.setMaterial(mat_type="measure")
    meshes = [retina]
    cornea = oe.spherical_lens_nofoc(r1=r_ac, r2=r_pc, x1=d_ac, x2=d_pc, d=r_cornea)
    cornea.setMaterial(mat_type="refractive", IOR=1.3771)
    meshes.append(cornea)
    lns = oe.spherical_lens_nofoc(r1=r_al, r2=r_pl, x1=d_al, x2=d_pl, d=r_lens)
    lns.setMaterial(mat_type="refractive", IOR=1.4200)
    meshes.append(lns)
    aqu = oe.spherical_lens_nofoc(r1=r_pc, r2=r_al, x1=d_pc * (1.0 + 1e-6), x2=d_al * (1.0 - 1e-6),
                                  d=r_cornea, d2=r_lens)
    aqu.setMaterial(mat_type="refractive", IOR=1.3374)
    meshes.append(aqu)
    vit = oe.spherical_lens_nofoc(r1=r_pl, r2=r_r * (1.0 + 1e-6), x1=d_pl * (1.0 + 1e-6), x2=d_r,
                                  d=r_lens, d2=r_lens, sign2_arcsin=-1.0)
    vit.setMaterial(mat_type="refractive", IOR=1.336)
    meshes.append(vit)
    return SceneSpec("eye", [ls0], meshes, np.float32(4e1), iterations=iterations, hist_points=90)


def cube(n=10000, seed=1, iterations=16):
    """example_directivity_dissipative_cube.py:47-67: dissipative (Beer-Lambert) cube."""
    np.random.seed(seed)
    oe = goe.optical_elements()
    ls0 = lsrc.light_source(center=np.array([0, 0, 0, 0], dtype=np.float32), direction=(0, 0, 1),
                            directivity=lambda x, y: np.cos(y), power=1000., ray_count=n)
    ms = oe.hemisphere(center=[0, 0, 0, 0], radius=1000.0)
    ms.setMaterial(mat_type="measure")
    m2 = oe.cube(center=(0, 0, 20, 0), size=[10, 10, 10, 0])
    m2.setMaterial(mat_type="refractive", IOR=1.0, dissipation=1.0)
    return SceneSpec("cube", [ls0], [ms, m2], np.float32(2e3), iterations=iterations)


def nested_cubes(n=10, seed=1, iterations=16):
    """example_nested_cubes_refraction.py:439-473: overlapping cubes, negative IOR, no
    measure surface (rays leave through max_ray_len)."""
    np.random.seed(seed)
    oe = goe.optical_elements()
    ls0 = lsrc.light_source(center=np.array([0, 0, 0, 0], dtype=np.float32), direction=(0, 0, 1),
                            directivity=lambda x, y: np.cos(y), power=1000., ray_count=n)
    meshes = []
    for ctr, size, ior in (((0, 0, 20, 0), [100, 100, 10, 0], 1.5),
                           ((-20, 0, 22.5 * (1.0 - 1e-6), 0), [30, 30, 5, 0], -2.0),
                           ((-20, 0, 27.5 * (1.0 + 1e-6), 0), [30, 30, 5, 0], -2.0),
                           ((20, 0, 20, 0), [30, 30, 5, 0], -2.0)):
        m = oe.cube(center=ctr, size=size)
        m.setMaterial(mat_type="refractive", IOR=ior)
        meshes.append(m)
    return SceneSpec("nested_cubes", [ls0], meshes, np.float32(2e2), iterations=iterations)


def synthetic(n=1_000_000, seed=7, iterations=16, grid=3, spacing=30.0, radius=10.0, z=100.0):
    """Synthetic benchmark scene: a measure hemisphere
    (r = 1000) plus grid x grid refractive spheres (r = 10, IOR 1.5) at z = 100 on a
    30-unit grid.  Each sphere/hemisphere is 10,366 triangles -> 103,660 at grid 3."""
    np.random.seed(seed)
    oe = goe.optical_elements()
    ms = oe.hemisphere(center=[0, 0, 0, 0], radius=1000.0)
    ms.setMaterial(mat_type="measure")
    meshes = [ms]
    for i in range(grid * grid):
        s = oe.sphere(center=[(i % grid - (grid - 1) / 2) * spacing, (i // grid - (grid - 1) / 2) * spacing,
                              z, 0], radius=radius)
        s.setMaterial(mat_type="refractive", IOR=1.5)
        meshes.append(s)
    ls0 = lsrc.light_source(center=np.array([0, 0, 0, 0], dtype=np.float32), direction=(0, 0, 1),
                            directivity=lambda x, y: np.cos(y), power=1.0, ray_count=n)
    return SceneSpec("synthetic", [ls0], meshes, np.float32(2e3), iterations=iterations,
                     hist_points=100)


def synthetic_rays(n=1_000_000, seed=7):
    """The emitted rays of :func:`synthetic` alone (the same RNG draws: the mesh
    generators draw nothing), without building its 103,660 triangles."""
    np.random.seed(seed)
    return lsrc.light_source(center=np.array([0, 0, 0, 0], dtype=np.float32), direction=(0, 0, 1),
                             directivity=lambda x, y: np.cos(y), power=1.0, ray_count=n)


def synthetic_dense(n=1_000_000, seed=7, iterations=16):
    """The synthetic generator with the nine spheres packed in front of the source
    (21-unit grid at z = 13, the central sphere subtending 50 degrees): ~79 % of
    the emitted rays enter a refractive sphere (measured on 20 k rays with the
    oracle), so bounces/s covers the secondaries, not only iteration 1
    ("place the objects so most rays hit refractive
    surfaces").  Same 103,660 triangles."""
    sc = synthetic(n=n, seed=seed, iterations=iterations, spacing=21.0, z=13.0)
    sc.name = "synthetic_dense"
    return sc


def cube_field(n=2000, seed=1, iterations=8, count=1100):
    """Many meshes (a capability case, not a BASELINE config): a measure hemisphere
    (r = 1000) plus `count` small cubes (12 triangles each) on a square grid at
    z = 40 in front of a point source pointing +z, every 7th a mirror, the rest
    refractive (IOR 1.5, every 5th dissipative).  Above 1 024 live mesh runs the
    root tests run in batches of pieces; above 128 each packet takes >= 3 tasks."""
    np.random.seed(seed)
    oe = goe.optical_elements()
    ms = oe.hemisphere(center=[0, 0, 0, 0], radius=1000.0)
    ms.setMaterial(mat_type="measure")
    meshes = [ms]
    side = int(np.ceil(np.sqrt(count)))
    for i in range(count):
        cx = (i % side - (side - 1) / 2.0) * 2.5
        cy = (i // side - (side - 1) / 2.0) * 2.5
        m = oe.cube(center=(cx, cy, 40.0 + 0.3 * (i % 3), 0), size=[1.5, 1.5, 1.5, 0])
        if i % 7 == 0:
            m.setMaterial(mat_type="mirror")
        else:
            m.setMaterial(mat_type="refractive", IOR=1.5, dissipation=0.05 if i % 5 == 0 else 0.0)
        meshes.append(m)
    ls0 = lsrc.light_source(center=np.array([0, 0, 0, 0], dtype=np.float32), direction=(0, 0, 1),
                            directivity=lambda x, y: np.cos(y), power=1.0, ray_count=n)
    return SceneSpec("cube_field", [ls0], meshes, np.float32(2e3), iterations=iterations)


BUILDERS = dict(parabolic=parabolic, lens=lens, eye=eye, cube=cube, nested_cubes=nested_cubes,
                synthetic=synthetic, synthetic_dense=synthetic_dense, cube_field=cube_field)
