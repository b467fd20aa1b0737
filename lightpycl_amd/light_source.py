"""Ray sources -- drop-in for LightPyCL's ``light_source`` module.

Mirrors ``/root/reference/light_source.py`` (class ``light_source``, :28-204):
same constructor signature, same attributes (``rays_origin`` (N,4) f32,
``rays_dir`` (N,4) f32, ``rays_power``), and the same numpy RNG draw sequence,
so ``np.random.seed(s)`` before construction yields the same rays as the
reference.  Host-side numpy only: ray generation is not on the hot path.
"""
from __future__ import annotations

import numpy as np
import numpy.linalg as la


def _rot(axis):
    """4x4 homogeneous rotation builders with a zero [3][3] entry, as every
    reference module defines them (light_source.py:64-66, 115-117, ...)."""
    if axis in ("x", "X"):
        return lambda a: np.matrix([[1, 0, 0, 0], [0, np.cos(a), -np.sin(a), 0],
                                    [0, np.sin(a), np.cos(a), 0], [0, 0, 0, 0]])
    if axis in ("y", "Y"):
        return lambda a: np.matrix([[np.cos(a), 0, np.sin(a), 0], [0, 1, 0, 0],
                                    [-np.sin(a), 0, np.cos(a), 0], [0, 0, 0, 0]])
    if axis in ("z", "Z"):
        return lambda a: np.matrix([[np.cos(a), -np.sin(a), 0, 0], [np.sin(a), np.cos(a), 0, 0],
                                    [0, 0, 1, 0], [0, 0, 0, 0]])
    return _rot("x")


_Rx, _Rz = _rot("x"), _rot("z")


def _pointing(direction, use_arctan2_always):
    """Elevation/azimuth of the beam axis (light_source.py:106-113 and :146-147)."""
    elev = np.arccos(direction[2] / la.norm(direction))
    if use_arctan2_always:
        return elev, np.arctan2(direction[1], direction[0])
    if direction[0] == 0:
        az = np.pi / 2.0 if direction[1] >= 0 else -np.pi / 2.0
    else:
        az = np.arctan2(direction[1], direction[0])
    return elev, az


class light_source:
    """A point (or collimated-disc) source of ``ray_count`` rays.

    Constructing one draws random hemisphere rays immediately, exactly like the
    reference constructor (light_source.py:37-43)."""

    center = None
    direction = None
    directivity = None
    power = 1
    ray_count = None
    rays_origin = None
    rays_dir = None

    def __init__(self, center=np.array([0, 0, 0, 0], dtype=np.float32), direction=(0, 0, 1),
                 directivity=lambda x, y: np.cos(y), power=1, ray_count=500):
        self.center = center
        self.direction = direction
        self.directivity = directivity
        self.power = power
        self.ray_count = ray_count
        self.random_rays()

    # -- light_source.py:98-137 -------------------------------------------
    def random_rays(self):
        """Random directions over the +z hemisphere (u -> elevation = arccos(u),
        v -> azimuth = 2 pi v), power weighted by ``directivity`` and normalised to
        ``power``, then rotated onto ``direction``."""
        n = self.ray_count
        self.rays_origin = np.zeros((n, 4)).astype(np.float32) + self.center
        self.rays_dest = np.zeros((n, 4)).astype(np.float32)
        elev0, az0 = _pointing(self.direction, use_arctan2_always=False)
        u = np.random.rand(n, 1)
        v = np.random.rand(n, 1)
        pad = np.zeros((n, 1))
        elevation = np.arccos(u)
        azimuth = 2.0 * np.pi * v
        xs = np.sin(elevation) * np.cos(azimuth)
        ys = np.sin(elevation) * np.sin(azimuth)
        zs = np.cos(elevation)
        dirs = np.concatenate((xs, ys, zs, pad), axis=1)
        pw = np.float32(self.directivity(azimuth, elevation))
        self.rays_power = pw * self.power / np.sum(pw)
        dirs = np.dot(dirs, _Rx(elev0))
        self.rays_dir = np.dot(dirs, _Rz(az0)).astype(np.float32)

    # -- light_source.py:45-95 --------------------------------------------
    def grid_rays(self):
        """Regular elevation x azimuth grid of floor(sqrt(N))**2 rays.  (The
        reference's ``np.float`` / float ``linspace`` count no longer run under
        numpy 2; this keeps its arithmetic with integer counts.)"""
        self.rays_origin = np.zeros((self.ray_count, 4)).astype(np.float32) + self.center
        self.rays_dest = np.zeros((self.ray_count, 4)).astype(np.float32)
        side = int(np.floor(np.sqrt(self.ray_count)))
        self.ray_count = np.floor(np.sqrt(self.ray_count)) ** 2
        elev0 = np.arccos(self.direction[2] / la.norm(self.direction))
        if self.direction[0] == 0:
            az0 = np.pi / 2.0 if self.direction[1] >= 0 else -np.pi / 2.0
        else:
            az0 = np.arctan(self.direction[1] / self.direction[0])
        el_col = np.transpose(np.matrix(np.linspace(0.0, np.pi / 2.0, side)))
        az_col = np.transpose(np.matrix(np.linspace(0.0, 2.0 * np.pi, side)))
        elevation = azimuth = None
        for k in range(side):
            if k == 0:
                elevation, azimuth = el_col, az_col
            else:
                elevation = np.concatenate((elevation, el_col), axis=0)
                azimuth = np.concatenate((azimuth, 0.0 * az_col + float(az_col[k])), axis=0)
        sa, ca = np.sin(azimuth), np.cos(azimuth)
        se, ce = np.sin(elevation), np.cos(elevation)
        self.rays_power = np.array(self.directivity(azimuth, elevation), dtype=np.float32) * self.power
        cnt = int(self.ray_count)
        dirs = np.array(np.append(np.append(np.append(np.multiply(se, ca), np.multiply(se, sa), axis=1),
                                            ce, axis=1), np.zeros((cnt, 1)), axis=1), dtype=np.float32)
        dirs = np.dot(dirs, _Rx(elev0))
        self.rays_dir = np.dot(dirs, _Rz(az0))

    # -- light_source.py:139-170 ------------------------------------------
    def random_collimated_rays(self, diameter=1.0):
        """Parallel rays (+z before rotation) with origins uniform in a
        ``diameter`` square, equal power.  Draws x then y after the
        constructor's own draws, as the reference does."""
        n = self.ray_count
        self.rays_dest = np.zeros((n, 4)).astype(np.float32)
        elev0, az0 = _pointing(self.direction, use_arctan2_always=True)
        x = (np.random.rand(n, 1) - 0.5) * diameter
        y = (np.random.rand(n, 1) - 0.5) * diameter
        z = np.zeros((n, 1))
        pad = np.zeros((n, 1))
        org = np.concatenate((x, y, z, pad), axis=1)
        dirs = np.zeros((n, 4)).astype(np.float32)
        dirs[:, 2] = 1.0
        pw = np.ones(n).astype(np.float32)
        self.rays_power = pw * self.power / np.sum(pw)
        org = np.dot(org, _Rx(elev0))
        self.rays_origin = np.array(np.dot(org, _Rz(az0)).astype(np.float32) + self.center).astype(np.float32)
        dirs = np.dot(dirs, _Rx(elev0))
        self.rays_dir = np.array(np.dot(dirs, _Rz(az0))).astype(np.float32)

    # -- light_source.py:173-188 ------------------------------------------
    def rotate_rays(self, axis="z", pivot=[0, 0, 0, 0], ang=np.pi / 2.0):
        R = _rot(axis)
        piv = np.array(pivot)
        self.rays_origin = np.array(np.add(np.dot(np.subtract(self.rays_origin, piv), R(ang)), piv)).astype(np.float32)
        self.rays_dir = np.array(np.dot(self.rays_dir, R(ang))).astype(np.float32)

    # -- light_source.py:191-204 ------------------------------------------
    def save_dxf(self, dxf_file):
        """DXF export needs the optional ``dxfwrite`` package (not part of the hot path)."""
        from dxfwrite import DXFEngine as dxf  # noqa: optional dependency, raises if absent
        drawing = dxf.drawing(dxf_file)
        drawing.add_layer('Rays', color=3)
        for r0, rd in zip(self.rays_origin, self.rays_origin + self.rays_dir):
            drawing.add(dxf.face3d([r0[0:3], rd[0:3], rd[0:3]], layer="Rays"))
        drawing.save()
