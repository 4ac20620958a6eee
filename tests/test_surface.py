"""the S3 surface without pyvista (libmofhip host code).

VTK/pyvista are absent, so nothing here is pinned to VTK output ("parity
unpinned"): the PLY reader is checked by write/read round trips
(ascii, binary little- and big-endian, float and double vertex properties,
extra properties), the normals and areas against a numpy restatement of the
same formulas (vtkPolyDataNormals: normalised per-triangle normals summed per
point in triangle order, normalised, float32; area = |cross| / 2), and the
areas of the synthetic meshes against mofhip.synth's.
"""
import numpy as np
import pytest

from mofhip import surface, synth
from mofhip._lib import MofError


def np_normals(P, T):
    P = P.astype(np.float64)
    p0, p1, p2 = P[T[:, 0]], P[T[:, 1]], P[T[:, 2]]
    a, b = p2 - p1, p0 - p1
    n = np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                  a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], axis=1)
    ln = np.sqrt(n[:, 0] * n[:, 0] + n[:, 1] * n[:, 1] + n[:, 2] * n[:, 2])
    n = np.where(ln[:, None] != 0, n / np.where(ln == 0, 1, ln)[:, None], n)
    acc = np.zeros((len(P), 3))
    for k in range(3):  # triangle order per point: np.add.at is sequential
        np.add.at(acc, T[:, k], n)
    ln = np.sqrt(acc[:, 0] * acc[:, 0] + acc[:, 1] * acc[:, 1] + acc[:, 2] * acc[:, 2])
    acc = np.where(ln[:, None] != 0, acc / np.where(ln == 0, 1, ln)[:, None], acc)
    return acc.astype(np.float32)


def mesh():
    p, t = synth.icosphere(6, 10.0, jitter=0.01)
    return p.astype(np.float32), t.astype(np.int64)


@pytest.mark.parametrize("binary", [True, False])
def test_ply_round_trip(tmp_path, binary):
    P, T = mesh()
    f = tmp_path / "s.ply"
    surface.write_ply(f, P, T, binary=binary)
    s = surface.read_surface(f)
    assert s.points.dtype == np.float32 and np.array_equal(s.points, P)
    assert np.array_equal(s.faces.reshape(-1, 4)[:, 1:], T)  # S3…py:80
    assert np.all(s.faces.reshape(-1, 4)[:, 0] == 3)
    assert s.n_points == len(P) and s.n_cells == len(T)


def test_ply_big_endian_double_and_extra_props(tmp_path):
    P, T = mesh()
    head = ("ply\nformat binary_big_endian 1.0\ncomment made by test\nelement vertex %d\n"
            "property double x\nproperty double y\nproperty double z\nproperty uchar red\n"
            "element face %d\nproperty list uchar uint vertex_indices\nproperty float quality\n"
            "element edge 0\nproperty int vertex1\nend_header\n" % (len(P), len(T)))
    vrec = np.zeros(len(P), dtype=[("x", ">f8"), ("y", ">f8"), ("z", ">f8"), ("r", "u1")])
    vrec["x"], vrec["y"], vrec["z"] = P[:, 0], P[:, 1], P[:, 2]
    frec = np.zeros(len(T), dtype=[("n", "u1"), ("v", ">u4", 3), ("q", ">f4")])
    frec["n"], frec["v"] = 3, T
    f = tmp_path / "be.ply"
    f.write_bytes(head.encode() + vrec.tobytes() + frec.tobytes())
    s = surface.read_surface(f)
    assert np.array_equal(s.points, P) and np.array_equal(s.triangles, T)


def test_file_normals_are_returned(tmp_path):
    P, T = mesh()
    N = np.random.default_rng(0).standard_normal(P.shape).astype(np.float32)
    f = tmp_path / "n.ply"
    surface.write_ply(f, P, T, normals=N)
    assert np.array_equal(surface.read_surface(f).point_normals, N)


def test_normals_and_areas_restatement():
    P, T = mesh()
    n = surface.point_normals(P, T)
    assert n.dtype == np.float32 and np.array_equal(n, np_normals(P, T))
    # outward on a sphere, unit length
    assert np.all(np.sum(n * P, axis=1) > 0)
    assert np.allclose(np.linalg.norm(n.astype(np.float64), axis=1), 1.0, atol=1e-6)
    a = surface.cell_areas(P, T)
    assert a.dtype == np.float64
    assert np.array_equal(a, synth.triangle_areas(P.astype(np.float64), T))
    s = surface.Surface(P, T)
    assert np.array_equal(s.compute_cell_sizes(length=False, volume=False)["Area"], a)


def test_drop_in_load_surface_and_errors(tmp_path):
    from utils import compute_optical_flow as cof
    P, T = mesh()
    f = tmp_path / "s.ply"
    surface.write_ply(f, P, T)
    s = cof.load_surface(str(f))
    assert np.array_equal(s.points, P)
    quad = tmp_path / "q.ply"
    quad.write_text("ply\nformat ascii 1.0\nelement vertex 4\nproperty float x\nproperty float y\n"
                    "property float z\nelement face 1\nproperty list uchar int vertex_indices\n"
                    "end_header\n0 0 0\n1 0 0\n1 1 0\n0 1 0\n4 0 1 2 3\n")
    with pytest.raises(MofError):
        surface.read_surface(quad)
    with pytest.raises(MofError):
        surface.read_surface(tmp_path / "missing.ply")
    with pytest.raises(MofError):
        surface.point_normals(P, np.array([[0, 1, len(P)]]))
