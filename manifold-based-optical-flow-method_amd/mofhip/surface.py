"""The S3 surface without pyvista (C ABI mof_ply_* /
mof_point_normals / mof_cell_areas).

``read_surface(path)`` returns a small PolyData-like object carrying exactly
what S3 takes from ``pv.read(surface_path)`` (S3…py:75-84): ``points``
(N,3) float32, ``faces`` (flat ``[3, a, b, c, ...]`` int64 as pyvista),
``point_normals`` (N,3) float32 and ``compute_cell_sizes(...)['Area']``
(M,) float64. VTK is not available to check against: the normals and areas
restate vtkPolyDataNormals / the triangle area (parity unpinned).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib as L


def _path(p) -> bytes:
    return os.fsencode(os.fspath(p))


def point_normals(points, triangles) -> np.ndarray:
    P = np.ascontiguousarray(points, dtype=np.float32)
    T = np.ascontiguousarray(triangles, dtype=np.int64).reshape(-1, 3)
    out = np.empty((len(P), 3), dtype=np.float32)
    L.check(L.lib().mof_point_normals(L.ptr(P), L.ptr(T), len(P), len(T), L.ptr(out)))
    return out


def cell_areas(points, triangles) -> np.ndarray:
    P = np.ascontiguousarray(points, dtype=np.float32)
    T = np.ascontiguousarray(triangles, dtype=np.int64).reshape(-1, 3)
    out = np.empty(len(T), dtype=np.float64)
    L.check(L.lib().mof_cell_areas(L.ptr(P), L.ptr(T), len(P), len(T), L.ptr(out)))
    return out


class Surface:
    """The pyvista.PolyData attributes S3 uses."""

    def __init__(self, points, triangles, normals=None):
        self.points = np.ascontiguousarray(points, dtype=np.float32)
        self.triangles = np.ascontiguousarray(triangles, dtype=np.int64).reshape(-1, 3)
        self._normals = None if normals is None else np.asarray(normals, dtype=np.float32)

    @property
    def n_points(self) -> int:
        return len(self.points)

    @property
    def n_cells(self) -> int:
        return len(self.triangles)

    @property
    def faces(self) -> np.ndarray:
        f = np.empty((self.n_cells, 4), dtype=np.int64)
        f[:, 0] = 3
        f[:, 1:] = self.triangles
        return f.reshape(-1)

    @property
    def point_normals(self) -> np.ndarray:
        if self._normals is None:
            self._normals = point_normals(self.points, self.triangles)
        return self._normals

    def compute_cell_sizes(self, length=True, area=True, volume=True):
        out = {}
        if area:
            out["Area"] = cell_areas(self.points, self.triangles)
        return out


def read_surface(path) -> Surface:
    n, m, hn = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_uint32(0)
    L.check(L.lib().mof_ply_info(_path(path), ctypes.byref(n), ctypes.byref(m), ctypes.byref(hn)))
    P = np.empty((n.value, 3), dtype=np.float32)
    T = np.empty((m.value, 3), dtype=np.int64)
    Nrm = np.empty((n.value, 3), dtype=np.float32) if hn.value else None
    L.check(L.lib().mof_ply_read(_path(path), L.ptr(P), L.ptr(T), None if Nrm is None else L.ptr(Nrm)))
    return Surface(P, T, Nrm)


def write_ply(path, points, triangles, binary=True, normals=None) -> None:
    """Minimal PLY writer (float32 x y z [nx ny nz], uchar/int faces), for
    tests and for surfaces built without VTK."""
    P = np.asarray(points, dtype=np.float32)
    T = np.asarray(triangles, dtype=np.int64).reshape(-1, 3)
    fmt = "binary_little_endian" if binary else "ascii"
    head = ["ply", "format %s 1.0" % fmt, "element vertex %d" % len(P),
            "property float x", "property float y", "property float z"]
    if normals is not None:
        head += ["property float nx", "property float ny", "property float nz"]
    head += ["element face %d" % len(T), "property list uchar int vertex_indices", "end_header"]
    V = P if normals is None else np.hstack([P, np.asarray(normals, dtype=np.float32)])
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode())
        if binary:
            f.write(np.ascontiguousarray(V, dtype="<f4").tobytes())
            rec = np.zeros(len(T), dtype=[("n", "u1"), ("v", "<i4", 3)])
            rec["n"] = 3
            rec["v"] = T
            f.write(rec.tobytes())
        else:
            for row in V:
                f.write((" ".join(repr(float(x)) for x in row) + "\n").encode())
            for t in T:
                f.write(("3 %d %d %d\n" % tuple(t)).encode())
