"""Meshes and optical-element generators -- drop-in for LightPyCL's
``geo_optical_elements`` module (``/root/reference/geo_optical_elements.py``).

``GeoObject`` (:25-148) holds vertices ((n,4) rows, w = 0), triangles (index
triples) and a material; ``optical_elements`` (:150-504) builds the standard
elements by revolving 2-D curves.  Vertex arithmetic follows the reference
operation for operation (same numpy calls, same float32/float64 casts), so
scenes built here are the scenes the reference builds.  Host-side numpy only.

Reference quirk kept on purpose: ``setMaterial(mat_type="mirror",
reflectivity=r)`` does NOT store ``r`` (the reference's second branch tests
"refractive" twice, :59-60), so mirrors keep the class default R = 1.0.
"""
from __future__ import annotations

import numpy as np


def _rot4(axis):
    if axis in ("y", "Y"):
        return lambda a: np.matrix([[np.cos(a), 0, np.sin(a), 0], [0, 1, 0, 0],
                                    [-np.sin(a), 0, np.cos(a), 0], [0, 0, 0, 0]])
    if axis in ("z", "Z"):
        return lambda a: np.matrix([[np.cos(a), -np.sin(a), 0, 0], [np.sin(a), np.cos(a), 0, 0],
                                    [0, 0, 1, 0], [0, 0, 0, 0]])
    return lambda a: np.matrix([[1, 0, 0, 0], [0, np.cos(a), -np.sin(a), 0],
                                [0, np.sin(a), np.cos(a), 0], [0, 0, 0, 0]])


def _rot3(axis):
    if axis in ("y", "Y"):
        return lambda a: np.matrix([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    if axis in ("z", "Z"):
        return lambda a: np.matrix([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    return lambda a: np.matrix([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])


class GeoObject:
    """A triangle mesh plus its optical material (geo_optical_elements.py:25-148)."""

    vertices = None
    triangles = None
    IOR = 1.0
    reflectivity = 1.0
    dissipation = 0.0      # 1/length unit (Beer-Lambert)
    AR_IOR = 1.0
    AR_thickness = 0.0
    anisotropy = None

    matTypes = {"refractive": 0, "mirror": 1, "terminator": 2, "measure": 3, "refractive_anisotropic": 4}
    matType = "refractive"

    def __init__(self, verts, tris, mat_type="refractive", IOR=1.0, reflectivity=1.0, dissipation=0.0,
                 AR_IOR=1.0, AR_thickness=0.0, anisotropy=None):
        self.vertices = verts
        self.triangles = tris
        self.setMaterial(mat_type, IOR, reflectivity, dissipation, AR_IOR, AR_thickness, anisotropy)

    def setMaterial(self, mat_type="refractive", IOR=1.0, reflectivity=1.0, dissipation=0.0, AR_IOR=1.0,
                    AR_thickness=0.0, anisotropy=None):
        """:46-62.  Unknown types fall back to "refractive".  Only the refractive
        branch stores parameters (the mirror quirk, see module docstring)."""
        if mat_type in self.matTypes:
            self.matType = mat_type
        else:
            print("Warning: material", mat_type, "unknown. Setting material as ", "refractive")
            self.matType = "refractive"
        if self.matType == "refractive":
            self.IOR = IOR
            self.dissipation = dissipation
            self.AR_IOR = AR_IOR
            self.AR_thickness = AR_thickness
        elif self.matType == "refractive_anisotropic":
            print("Warning: anisotropic materials are not yet supported.")

    def getMaterialBuf(self):
        """:64-66 -- the per-mesh material record the tracer flattens."""
        return {"type": self.matTypes.get(self.matType), "IOR": self.IOR, "R": self.reflectivity,
                "dissipation": self.dissipation}

    def translate(self, vec):
        self.vertices = self.vertices + np.array(vec)

    def rotate(self, axis="x", angle=np.pi / 2, pivot=(0, 0, 0, 0)):
        """:72-93: rotate every vertex about ``pivot``; rows are rewritten as float32 with w = 0."""
        R = _rot4(axis)
        moved = np.transpose(R(angle) * np.transpose(np.array(self.vertices) - np.array(pivot))) + np.array(pivot)
        for i, row in enumerate(list(moved)):
            r = np.array(row)
            self.vertices[i] = np.array([r[0][0], r[0][1], r[0][2], 0], dtype=np.float32)

    def trimesh(self):
        return [[self.vertices[idx] for idx in tri] for tri in self.triangles]

    def trimesh_to_geoObject(self, trimesh):
        verts, tris, k = [], [], 0
        for tri in trimesh:
            this = []
            for v in tri:
                verts.append(v)
                this.append(k)
                k += 1
            tris.append(this)
        self.vertices = verts
        self.triangles = tris

    def tribuf(self):
        """:121-132 -- three parallel vertex lists (v0[i], v1[i], v2[i]) = triangle i."""
        m_v0, m_v1, m_v2 = [], [], []
        for tri in self.triangles:
            m_v0.append(self.vertices[tri[0]])
            m_v1.append(self.vertices[tri[1]])
            m_v2.append(self.vertices[tri[2]])
        return (m_v0, m_v1, m_v2)

    def append(self, verts, tris):
        self.triangles = np.append(self.triangles, np.array(tris).astype(np.int32) + len(self.vertices), axis=0)
        self.vertices = np.append(self.vertices, verts, axis=0)

    def write_dxf(self, dxf_file):
        """DXF export needs the optional ``dxfwrite`` package."""
        from dxfwrite import DXFEngine as dxf  # noqa: optional dependency, raises if absent
        drawing = dxf.drawing(dxf_file)
        drawing.add_layer('0', color=2)
        for tri in self.triangles:
            drawing.add(dxf.face3d([self.vertices[tri[0]][0:3], self.vertices[tri[1]][0:3],
                                    self.vertices[tri[2]][0:3]], layer="0"))
        drawing.save()


class optical_elements:
    """Generators for standard optical elements (geo_optical_elements.py:150-504)."""

    def cube(self, center, size):
        corners = np.array([[-1, -1, -1, 0], [1, -1, -1, 0], [-1, 1, -1, 0], [1, 1, -1, 0],
                            [-1, -1, 1, 0], [1, -1, 1, 0], [-1, 1, 1, 0], [1, 1, 1, 0]],
                           dtype=np.float32) / 2.0 * size + center
        faces = [[0, 1, 2], [2, 3, 1], [4, 5, 6], [6, 7, 5], [0, 1, 4], [4, 5, 1],
                 [2, 3, 6], [6, 7, 3], [0, 2, 4], [4, 6, 2], [1, 3, 5], [5, 7, 3]]
        return GeoObject(corners, faces)

    def spherical_lens_nofoc(self, r1, r2, x1, x2, d, d2=None, sign1_arcsin=1.0, sign2_arcsin=1.0):
        """:172-200 -- a two-surface lens body made by revolving two arcs about x."""
        N = 50
        if d2 is None:
            d2 = d
        z1, z2 = r1 + x1, r2 + x2
        dphi1 = np.pi / 2.0 if sign1_arcsin < 0 else 0.0
        dphi2 = np.pi / 2.0 if sign2_arcsin < 0 else 0.0
        phi1 = np.linspace(0.0, np.absolute(np.arcsin(d / r1)) + dphi1, N)
        phi2 = np.linspace(np.absolute(np.arcsin(d2 / r2)) + dphi2, 0.0, N)
        xs = np.append(z1 - r1 * np.cos(phi1), z2 - r2 * np.cos(phi2))
        ys = np.append(r1 * np.sin(phi1), r2 * np.sin(phi2))
        mesh = self.revolve_curve([[a, b] for a, b in zip(xs, ys)], axis="x", ang=2.0 * np.pi, ang_pts=72)
        mesh.rotate(axis="y", angle=-np.pi / 2.0, pivot=(0, 0, 0, 0))
        return mesh

    def sphere(self, center, radius):
        N = 72
        phi = np.linspace(0.0, 2.0 * np.pi, N)
        mesh = self.revolve_curve([[a, b] for a, b in zip(np.cos(phi) * radius, np.sin(phi) * radius)],
                                  axis="x", ang=np.pi, ang_pts=N + 1)
        mesh.translate(center)
        return mesh

    def hemisphere(self, center, radius):
        N = 72
        phi = np.linspace(0.0, np.pi, N)
        mesh = self.revolve_curve([[a, b] for a, b in zip(np.cos(phi) * radius, np.sin(phi) * radius)],
                                  axis="x", ang=np.pi, ang_pts=N + 1)
        mesh.translate(center)
        return mesh

    def parabolic_mirror(self, focus=(0, 0, 0), focal_length=5.0, diameter=20.0, reflectivity=0.98):
        N, M = 72, 200
        yn = np.linspace(0.0, diameter / 2.0, M)
        xn = yn ** 2 / (4.0 * focal_length) - focal_length
        curve = [[a, b] for a, b in zip(focus[0] + xn, focus[1] + yn)]
        mesh = self.revolve_curve(curve, axis="x", ang=2. * np.pi, ang_pts=N + 1)
        mesh.setMaterial(mat_type="mirror", reflectivity=reflectivity)
        return mesh

    def topless_cylinder(self, center=(0, 0, 0), diameter=20.0, height=10.0):
        N = 72
        xs = np.array([0.0, 0.0, 1.0]) * height + center[1]
        ys = np.array([0.0, .5, .5]) * diameter + center[0]
        return self.revolve_curve([[a, b] for a, b in zip(xs, ys)], axis="x", ang=2. * np.pi, ang_pts=N + 1)

    def revolve_curve(self, curve, axis="x", ang=2 * np.pi, ang_pts=36):
        """:259-302 -- sweep a 2-D polyline (z = 0) around ``axis``.  Every
        (angle step, curve segment) quad becomes four fresh float32 vertices and
        two triangles [0,1,2], [2,3,1]; the last step slightly overlaps the first
        (angle step ang/(ang_pts-1) taken ang_pts times)."""
        R = _rot3(axis)
        cols = [[[xy[0]], [xy[1]], [0]] for xy in curve]
        step = ang / (ang_pts - 1.0)
        angs = np.linspace(0.0, ang - step, ang_pts)
        nseg = len(cols) - 1
        verts, tris = [], []
        for k, (phi1, phi2) in enumerate(zip(angs, angs + step)):
            Ra, Rb = R(phi1), R(phi2)
            for i in np.arange(nseg):
                for m in (Ra * cols[i], Ra * cols[i + 1], Rb * cols[i], Rb * cols[i + 1]):
                    verts.append(np.array([m[0, 0], m[1, 0], m[2, 0], 0], dtype=np.float32))
                base = i * 4 + 4 * k * nseg
                tris.append([0, 1, 2] + base)
                tris.append([2, 3, 1] + base)
        # one (n, 4) float32 table (the same rows as a list of them) so that
        # flattening a scene is one gather, not a pass over Python rows
        return GeoObject(np.array(verts, dtype=np.float32).reshape(-1, 4),
                         np.array(tris, dtype=np.int64).reshape(-1, 3))

    def extrude_by_vector(self, curve, vector, capped=True):
        verts, tris = [], []
        z0 = 0.0
        for k, xy in enumerate(curve):
            verts.append(np.array([xy[0], xy[1], z0, 0], dtype=np.float32))
            verts.append(np.array([xy[0] + vector[0], xy[1] + vector[1], z0 + vector[2], 0], dtype=np.float32))
            if k < len(curve) - 1:
                tris.append([2 * k + 0, 2 * k + 1, 2 * k + 2])
                tris.append([2 * k + 2, 2 * k + 3, 2 * k + 1])
        gobj = GeoObject(np.array(verts, dtype=np.float32).reshape(-1, 4),
                         np.array(tris, dtype=np.int64).reshape(-1, 3))
        if capped:
            cap = self.curve_to_mesh(curve)
            gobj.append(cap.vertices, cap.triangles)
            gobj.append(cap.vertices + vector, cap.triangles)
        return gobj

    def curve_to_mesh(self, curve):
        """Needs Shewchuk's ``triangle`` bindings (optional; not in this image)."""
        import triangle  # noqa: optional dependency, raises ImportError if absent
        M = len(curve)
        segs = np.zeros((M, 2)).astype(np.int32)
        segs[:, 0] = np.linspace(0, M - 1, M).astype(np.int32)
        segs[:, 1] = segs[:, 0] + 1
        segs[-1, -1] = 0
        tri = triangle.triangulate({"vertices": np.array(curve).astype(np.float32),
                                    "segments": np.array(segs).astype(np.int32)}, 'pq10')
        v2, t2 = tri["vertices"], tri["triangles"]
        verts = np.zeros((len(v2), 4), dtype=np.float32)
        tris = np.zeros((len(t2), 3), dtype=np.float32)
        verts[:, 0], verts[:, 1] = v2[:, 0], v2[:, 1]
        tris[:, 0], tris[:, 1], tris[:, 2] = t2[:, 0], t2[:, 1], t2[:, 2]
        return GeoObject(verts=verts, tris=tris)

    def lens_spherical_biconcave(self, focus, r1, r2, diameter, IOR):
        mesh = self.revolve_curve(self.lens_spherical_2r(focus, r1, r2, diameter, 1, IOR), axis="x",
                                  ang=np.pi, ang_pts=36)
        mesh.setMaterial(mat_type="refractive", IOR=IOR)
        return mesh

    def curve_lens_spherical_biconcave(self, focus, r1, r2, d, diameter, axis, IOR):
        n = IOR
        f1 = np.absolute(1 / ((n - 1) * (1 / r1)))
        f2 = np.absolute(1 / ((n - 1) * (1 / r2)))
        f0 = 1 / (1 / f1 + 1 / f2)
        fx0, fy0 = focus[0], focus[1]
        (poly1, f1, _d1) = self.curve_lens_spherical((fx0 + f1 + f0, fy0), r1, diameter, -1, -1, IOR)
        (poly2, f2, _d2) = self.curve_lens_spherical((fx0 + d - f1 + f0, fy0), r2, diameter, 1, -1, IOR)
        curve = poly1[0:-3]
        curve.extend(poly2[0:-3])
        curve.extend([poly1[1]])
        return (curve, f0, d)

    def lens_spherical_2r(self, focus, r1, r2, diameter, lens_sign, n):
        """:366-401 -- closed 2-D outline of a lens from two circular arcs."""
        N = 60
        fx0, fy0 = focus[0], focus[1]
        ab = np.absolute
        x = np.zeros(2 * N + 1)
        y = np.zeros(2 * N + 1)
        phi_r1 = np.arcsin(diameter / r1)
        phi_r2 = np.arcsin(diameter / r2)
        d = ab(r1 - r1 * np.cos(phi_r1)) + ab(r2 - r2 * np.cos(phi_r2))
        f = ab(1 / ((n - 1) * (1 / r1 - 1 / r2 + (n - 1) * d / (n * r1 * r2))))
        q = (f - r1)
        r1x0, r1y0 = fx0 + q, fy0
        r2x0, r2y0 = fx0 + q + r1 - lens_sign * d + r2, fy0
        i = 0
        for phi in np.linspace(np.pi - ab(phi_r2), np.pi + ab(phi_r2), N):
            x[i] = r2x0 + r2 * np.cos(phi)
            y[i] = r2y0 + r2 * np.sin(phi)
            i += 1
        for phi in np.linspace(-ab(phi_r1), ab(phi_r1), N):
            x[i] = r1x0 + r1 * np.cos(phi)
            y[i] = r1y0 + r1 * np.sin(phi)
            i += 1
        x[i], y[i] = x[0], y[0]
        return [[a, b] for a, b in zip(x, y)]

    def curve_lens_spherical(self, focus, r1, diameter, lens_direction, lens_sign, IOR):
        N = 20
        n = IOR
        ab = np.absolute
        x = np.zeros(N + 3)
        y = np.zeros(N + 3)
        phi_r1 = np.arcsin(diameter / (2 * r1))
        d = ab(r1 - r1 * np.cos(phi_r1))
        f = ab(1 / ((n - 1) * (1 / r1)))
        q = f + r1
        fx0, fy0 = focus[0], focus[1]
        off = 0 if lens_sign > 0 else -np.pi
        if lens_direction >= 0:
            r1x0, r1y0 = fx0 - lens_sign * q, fy0
            angles = np.linspace(off - lens_sign * ab(phi_r1), off + lens_sign * ab(phi_r1), N)
        else:
            r1x0, r1y0 = fx0 + lens_sign * q, fy0
            angles = np.linspace(off + np.pi - lens_sign * ab(phi_r1), off + np.pi + lens_sign * ab(phi_r1), N)
        i = 0
        for phi in angles:
            x[i] = r1x0 + r1 * np.cos(phi)
            y[i] = r1y0 + r1 * np.sin(phi)
            i += 1
        if lens_sign < 0:
            x[i], y[i] = x[i - 1] + lens_direction * d, y[i - 1]
            i += 1
            x[i], y[i] = x[i - 2] + lens_direction * d, y[0]
            i += 1
        x[i], y[i] = x[0], y[0]
        return ([[a, b] for a, b in zip(x, y)], f, d)
