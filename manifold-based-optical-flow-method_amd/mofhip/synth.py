"""Synthetic inputs for the manifold optical-flow path.

The reference reads a PLY surface and a potentials CSV
(`S3_compute_v_and_detection_singularity.py:75-89`). Neither ships, so every
parity case and benchmark runs on generated inputs of the same shapes:

* a geodesic icosphere of frequency ``n`` (V = 10 n^2 + 2 vertices,
  M = 20 n^2 triangles), optionally with seeded radial jitter, or an open
  spherical cap cut from one;
* VTK-like per-vertex normals (normalised sum of unit face normals) and
  triangle areas (half the cross-product norm), the attributes S3 takes from
  pyvista (`S3…py:83-84`);
* a travelling wave ``I_k(x) = sin(kappa * phi(x) - omega * k)``.

All arrays are float64 / int32 unless a caller asks otherwise.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "icosphere",
    "random_sphere",
    "permute_vertices",
    "spherical_cap",
    "vertex_normals",
    "triangle_areas",
    "travelling_wave",
    "electrode_surface",
    "folded_sphere",
    "mesh_for_config",
    "wave_phase",
    "config_wave",
    "CONFIG_FREQ",
]

# frequency n of the configs in SURVEY.md §8d (V = 10 n^2 + 2)
CONFIG_FREQ = {"C1": 8, "C2": 57, "C3": 128, "C5": 253}


def _icosahedron():
    t = (1.0 + 5.0 ** 0.5) / 2.0
    v = np.array(
        [[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0],
         [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
         [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], dtype=np.float64)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    f = np.array(
        [[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11],
         [1, 5, 9], [5, 11, 4], [11, 10, 2], [10, 7, 6], [7, 1, 8],
         [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9],
         [4, 9, 5], [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]],
        dtype=np.int64)
    return v, f


def icosphere(n: int, radius: float = 10.0, jitter: float = 0.0, seed: int = 0):
    """Geodesic icosphere of frequency ``n`` (class-I subdivision of each face
    into n^2 triangles, projected to the sphere).

    Returns ``(points (V,3) f64, triangles (M,3) int32)`` with outward,
    consistently oriented triangles. ``jitter`` scales each radius by
    ``1 + jitter * U(-1, 1)`` drawn from ``numpy.random.default_rng(seed)``.
    """
    if n < 1:
        raise ValueError("frequency n must be >= 1")
    cv, cf = _icosahedron()
    nv = len(cv)
    # canonical edge ids
    edges = {}
    for f in cf:
        for a, b in ((f[0], f[1]), (f[1], f[2]), (f[2], f[0])):
            key = (min(a, b), max(a, b))
            if key not in edges:
                edges[key] = len(edges)
    ne = len(edges)
    n_edge_pts = n - 1
    n_face_pts = (n - 1) * (n - 2) // 2
    total = nv + ne * n_edge_pts + len(cf) * n_face_pts

    pts = np.empty((total, 3), dtype=np.float64)
    pts[:nv] = cv
    # lattice index -> vertex id, built per face
    tris = []
    for fi, (a, b, c) in enumerate(cf):
        A, Bv, C = cv[a], cv[b], cv[c]
        idx = -np.ones((n + 1, n + 1), dtype=np.int64)  # idx[i, j]: i along a->b, j along a->c

        def edge_vertex(p, q, s):
            # s-th interior point (1..n-1) from p towards q
            key = (min(p, q), max(p, q))
            eid = edges[key]
            pos = s if p < q else n - s
            return nv + eid * n_edge_pts + (pos - 1)

        face_base = nv + ne * n_edge_pts + fi * n_face_pts
        fcount = 0
        for i in range(n + 1):
            for j in range(n + 1 - i):
                k = n - i - j  # weight of a
                if i == 0 and j == 0:
                    vid = a
                elif i == n:
                    vid = b
                elif j == n:
                    vid = c
                elif j == 0:
                    vid = edge_vertex(a, b, i)
                elif i == 0:
                    vid = edge_vertex(a, c, j)
                elif k == 0:
                    vid = edge_vertex(b, c, j)
                else:
                    vid = face_base + fcount
                    fcount += 1
                idx[i, j] = vid
                pts[vid] = (k * A + i * Bv + j * C) / n
        for i in range(n):
            for j in range(n - i):
                tris.append((idx[i, j], idx[i + 1, j], idx[i, j + 1]))
                if i + j < n - 1:
                    tris.append((idx[i + 1, j], idx[i + 1, j + 1], idx[i, j + 1]))
    tri = np.asarray(tris, dtype=np.int64)
    pts /= np.linalg.norm(pts, axis=1, keepdims=True)
    r = np.full(total, float(radius))
    if jitter:
        rng = np.random.default_rng(seed)
        r = r * (1.0 + jitter * rng.uniform(-1.0, 1.0, size=total))
    pts *= r[:, None]
    return pts, tri.astype(np.int32)


def random_sphere(n_points: int, radius: float = 10.0, seed: int = 0):
    """Irregular closed mesh: convex hull of uniformly random points on a
    sphere (valence varies, vertex order is random), outward oriented.
    Stands in for reconstructed cortical surfaces, whose valence and vertex
    order are not the icosphere's."""
    from scipy.spatial import ConvexHull
    rng = np.random.default_rng(seed)
    p = rng.normal(size=(n_points, 3))
    p /= np.linalg.norm(p, axis=1, keepdims=True)
    hull = ConvexHull(p)
    t = hull.simplices.astype(np.int64)
    c = np.cross(p[t[:, 1]] - p[t[:, 0]], p[t[:, 2]] - p[t[:, 0]])
    flip = (c * p[t].mean(axis=1)).sum(axis=1) < 0
    t[flip] = t[flip][:, [0, 2, 1]]
    return p * radius, t.astype(np.int32)


def permute_vertices(points, triangles, seed: int = 0):
    """The same mesh with its vertices relabelled by a random permutation
    (locality stress test). Returns (points, triangles, perm) with
    new_points[perm[i]] = points[i]."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(len(points))
    out = np.empty_like(points)
    out[perm] = points
    return out, perm[np.asarray(triangles)].astype(np.int32), perm


def spherical_cap(n: int = 16, radius: float = 10.0, zcut: float = 0.5):
    """Open cap: the triangles of ``icosphere(n)`` whose three vertices all have
    z > zcut * radius, re-indexed (the G2 boundary case)."""
    p, t = icosphere(n, radius)
    keep_v = p[:, 2] > zcut * radius
    keep_t = keep_v[t].all(axis=1)
    t = t[keep_t]
    used = np.unique(t)
    remap = -np.ones(len(p), dtype=np.int64)
    remap[used] = np.arange(len(used))
    return p[used].copy(), remap[t].astype(np.int32)


def _edges_with_opposites(tri):
    """{(a, b) a < b: [opposite vertices]} in first-seen order."""
    opp = {}
    for a, b, c in tri.tolist():
        for u, v, w in ((a, b, c), (b, c, a), (c, a, b)):
            opp.setdefault((u, v) if u < v else (v, u), []).append(w)
    return opp


def _laplacian_smooth(p, tri, n_iter=100, relax=0.01):
    """vtkSmoothPolyDataFilter-like (pyvista ``smooth``): n_iter Laplacian
    steps p += relax (mean of neighbours - p); boundary vertices move along
    the boundary (their boundary-edge neighbours only)."""
    opp = _edges_with_opposites(tri)
    nbr = [[] for _ in range(len(p))]
    bnb = [[] for _ in range(len(p))]
    for (a, b), o in opp.items():
        nbr[a].append(b)
        nbr[b].append(a)
        if len(o) == 1:
            bnb[a].append(b)
            bnb[b].append(a)
    src, dst = [], []
    for i in range(len(p)):
        ns = bnb[i] if bnb[i] else nbr[i]
        src.extend(ns)
        dst.extend([i] * len(ns))
    src, dst = np.asarray(src), np.asarray(dst)
    cnt = np.bincount(dst, minlength=len(p)).astype(np.float64)[:, None]
    p = p.copy()
    for _ in range(n_iter):
        acc = np.zeros_like(p)
        np.add.at(acc, dst, p[src])
        p += relax * (acc / cnt - p)
    return p


def _butterfly(p, tri):
    """One butterfly subdivision step (vtkButterflySubdivisionFilter-like):
    every triangle splits in four; an interior edge (a, b) with opposite
    vertices c, d gets 1/2 (a + b) + 1/8 (c + d) - 1/16 (the four wing
    vertices opposite the edges a-c, b-c, a-d, b-d), a boundary edge the
    four-point rule 9/16 (a + b) - 1/16 (its boundary neighbours); a missing
    wing falls back to the edge's far corner. New vertices follow the old
    ones in edge order."""
    opp = _edges_with_opposites(tri)
    bnext = {}
    for (a, b), o in opp.items():
        if len(o) == 1:
            bnext.setdefault(a, []).append(b)
            bnext.setdefault(b, []).append(a)

    def wing(u, v, notw):
        o = opp[(u, v) if u < v else (v, u)]
        for w in o:
            if w != notw:
                return w
        return None

    eid = {}
    new = []
    N = len(p)
    for (a, b), o in opp.items():
        if len(o) == 2:
            c, d = o
            q = 0.5 * (p[a] + p[b]) + 0.125 * (p[c] + p[d])
            for u, v, far in ((a, c, b), (b, c, a), (a, d, b), (b, d, a)):
                w = wing(u, v, far)
                q -= 0.0625 * p[w if w is not None else far]
        else:
            pa = [x for x in bnext.get(a, []) if x != b]
            pb = [x for x in bnext.get(b, []) if x != a]
            qa = p[pa[0]] if pa else p[a]
            qb = p[pb[0]] if pb else p[b]
            q = 0.5625 * (p[a] + p[b]) - 0.0625 * (qa + qb)
        eid[(a, b)] = N + len(new)
        new.append(q)
    e = lambda u, v: eid[(u, v) if u < v else (v, u)]  # noqa: E731
    out = []
    for a, b, c in tri.tolist():
        ab, bc, ca = e(a, b), e(b, c), e(c, a)
        out += [(a, ab, ca), (ab, b, bc), (ca, bc, c), (ab, bc, ca)]
    return np.vstack([p, np.asarray(new)]), np.asarray(out, dtype=np.int64)


def electrode_surface(n_side: int, spacing: float = 10.0, jitter: float = 0.15, radius: float = 70.0,
                      subdivisions: int = 3, seed: int = 0):
    """S1-like reconstructed cortical patch (S1_reconstruct_surface.py:82-97):
    an ``n_side`` x ``n_side`` ECoG electrode grid (``spacing`` mm, positions
    jittered by ``jitter`` x spacing) lying on a sphere of ``radius`` mm (the
    cortex's curvature), a 2-D Delaunay triangulation of it (pyvista
    ``delaunay_2d``), 100 Laplacian smoothing steps, ``subdivisions``
    butterfly subdivision steps, and 100 more smoothing steps. An open,
    mostly valence-6 surface whose original grid vertices keep the
    Delaunay valences (4-8). Returns (points (V,3) f64, triangles (M,3) int32)
    with consistently oriented triangles (normals towards +z)."""
    from scipy.spatial import Delaunay
    half = 0.5 * (n_side - 1) * spacing * (1.0 + jitter)
    if half * 2 ** 0.5 > 0.9 * radius:
        raise ValueError("the grid (half-width %.1f) must lie well inside the sphere (radius %.1f)" % (half, radius))
    rng = np.random.default_rng(seed)
    g = (np.arange(n_side) - 0.5 * (n_side - 1)) * spacing
    x, y = np.meshgrid(g, g, indexing="ij")
    xy = np.stack([x.ravel(), y.ravel()], axis=1)
    xy += jitter * spacing * rng.uniform(-1.0, 1.0, size=xy.shape)
    z = np.sqrt(np.maximum(radius ** 2 - (xy ** 2).sum(axis=1), 0.0)) - radius
    p = np.column_stack([xy, z])
    tri = Delaunay(xy).simplices.astype(np.int64)
    # the hull of a jittered grid closes with slivers over nearly collinear
    # boundary electrodes, which the smoothing folds over: peel boundary
    # triangles with an angle under 20 degrees
    while True:
        opp = _edges_with_opposites(tri)
        bd = {e for e, o in opp.items() if len(o) == 1}
        e0 = xy[tri[:, 1]] - xy[tri[:, 0]]
        e1 = xy[tri[:, 2]] - xy[tri[:, 1]]
        e2 = xy[tri[:, 0]] - xy[tri[:, 2]]

        def angle(u, v):
            return np.degrees(np.arccos(np.clip(-(u * v).sum(1) / np.linalg.norm(u, axis=1)
                                                / np.linalg.norm(v, axis=1), -1.0, 1.0)))
        amin = np.minimum(np.minimum(angle(e2, e0), angle(e0, e1)), angle(e1, e2))
        onb = np.array([any(((min(u, v), max(u, v)) in bd) for u, v in ((a, b), (b, c), (c, a)))
                        for a, b, c in tri.tolist()])
        drop = onb & (amin < 20.0)
        if not drop.any():
            break
        tri = tri[~drop]
    used = np.unique(tri)
    remap = -np.ones(len(p), dtype=np.int64)
    remap[used] = np.arange(len(used))
    p, tri = p[used], remap[tri]
    c = np.cross(p[tri[:, 1]] - p[tri[:, 0]], p[tri[:, 2]] - p[tri[:, 0]])
    flip = c[:, 2] < 0
    tri[flip] = tri[flip][:, [0, 2, 1]]
    p = _laplacian_smooth(p, tri)
    for _ in range(subdivisions):
        p, tri = _butterfly(p, tri)
    p = _laplacian_smooth(p, tri)
    return p, tri.astype(np.int32)


def folded_sphere(n: int = 128, radius: float = 10.0, depth: float = 0.3, kmin: float = 16.0,
                  kmax: float = 28.0, waves: int = 64, seed: int = 0):
    """Folded cortex-like closed surface: ``icosphere(n)`` (n = 128: the
    163,842-vertex order-7 icosahedral topology of FreeSurfer's fsaverage)
    with each vertex moved along its ray by a seeded band-limited field,
    r = radius (1 + depth/2 g(x)), g in [-1, 1]: ``waves`` plane waves
    cos(k (u . x) + phase) of random directions u and angular wavenumbers k in
    [kmin, kmax] restricted to the unit sphere -- gyri and sulci about
    2 pi radius / k apart (kmin 16 .. kmax 28 at radius 70 mm: 16-27 mm, the
    gyral period of a human cortex) with a peak-to-trough sulcal depth of
    ``depth`` x radius (0.3: an amplitude of 15 % of the radius, 21 mm
    peak-to-trough at 70 mm). A radial graph over the sphere cannot fold over
    itself, so every triangle keeps its outward orientation; at depth 0.3 the
    sulcal walls tilt the surface up to 64 degrees from the sphere, the area
    grows 1.20x and 1 % of the triangles turn obtuse (angles 28-104 degrees)
    -- the curvature and the stretched elements a reconstructed pial surface
    brings to its FEM operator (S1_reconstruct_surface.py:85-97 builds the
    reference's surfaces)."""
    p, t = icosphere(n, 1.0)
    rng = np.random.default_rng(seed)
    u = rng.normal(size=(waves, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    k = rng.uniform(kmin, kmax, size=waves)
    ph = rng.uniform(0.0, 2.0 * np.pi, size=waves)
    g = np.zeros(len(p))
    for j in range(waves):
        g += np.cos(k[j] * (p @ u[j]) + ph[j])
    g = 2.0 * (g - g.min()) / (g.max() - g.min()) - 1.0
    return p * (radius * (1.0 + 0.5 * depth * g))[:, None], t


def vertex_normals(points: np.ndarray, triangles: np.ndarray) -> np.ndarray:
    """VTK-like point normals: normalised sum of the unit normals of the
    incident faces."""
    p = np.asarray(points, dtype=np.float64)
    t = np.asarray(triangles, dtype=np.int64)
    fn = np.cross(p[t[:, 1]] - p[t[:, 0]], p[t[:, 2]] - p[t[:, 0]])
    fn /= np.linalg.norm(fn, axis=1, keepdims=True)
    vn = np.zeros_like(p)
    for l in range(3):
        np.add.at(vn, t[:, l], fn)
    vn /= np.linalg.norm(vn, axis=1, keepdims=True)
    return vn


def triangle_areas(points: np.ndarray, triangles: np.ndarray) -> np.ndarray:
    p = np.asarray(points, dtype=np.float64)
    t = np.asarray(triangles, dtype=np.int64)
    return 0.5 * np.linalg.norm(
        np.cross(p[t[:, 1]] - p[t[:, 0]], p[t[:, 2]] - p[t[:, 0]]), axis=1)


def travelling_wave(points: np.ndarray, T: int, kappa: float = 3.0,
                    omega: float = 0.3) -> np.ndarray:
    """``I[k, x] = sin(kappa * atan2(y, x) - omega * k)``, shape (T, N) f64."""
    phi = np.arctan2(points[:, 1], points[:, 0])
    k = np.arange(T, dtype=np.float64)[:, None]
    return np.sin(kappa * phi[None, :] - omega * k)


def wave_phase(name: str, points: np.ndarray):
    """(phase (N,), kappa) of the bench signal I_k = sin(kappa phase - 0.3 k)
    on config ``name``'s mesh: on the spheres the azimuth about the z axis
    (kappa 3: a pattern rotating around the sphere); on the S1-like patches
    (centred on the z axis, curvature centre (0, 0, -70 mm)) the angle about
    the x axis through the curvature centre, kappa 30 -- a wave travelling
    across the electrode grid (about 3 wavelengths over it) instead of a
    pinwheel whose unbounded gradient would sit at the patch centre."""
    p = np.asarray(points, dtype=np.float64)
    if name in ("S1", "S1s", "S1m"):
        return np.arctan2(p[:, 2] + 70.0, p[:, 1]), 30.0
    return np.arctan2(p[:, 1], p[:, 0]), 3.0


def config_wave(name: str, points: np.ndarray, T: int, omega: float = 0.3) -> np.ndarray:
    """The bench signal of config ``name`` (wave_phase), shape (T, N) f64."""
    phi, kappa = wave_phase(name, points)
    k = np.arange(T, dtype=np.float64)[:, None]
    return np.sin(kappa * phi[None, :] - omega * k)


def mesh_for_config(name: str):
    """(points, triangles, normals, areas) of a SURVEY.md §8d config mesh.

    C1 has no jitter; the >=32k meshes get 0.5 % radial jitter, seed 0.
    R3 is an irregular 163,842-vertex random-hull sphere, P3 the C3 mesh
    with randomly relabelled vertices (locality stress cases), F3 the folded
    cortex-like surface on the same 163,842-vertex topology (folded_sphere)."""
    if name == "F3":
        p, t = folded_sphere(128)
        return p, t, vertex_normals(p, t), triangle_areas(p, t)
    if name == "R3":
        p, t = random_sphere(163842, 10.0, seed=0)
        return p, t, vertex_normals(p, t), triangle_areas(p, t)
    if name in ("S1", "S1s", "S1m"):
        # S1-like surfaces (electrode_surface): S1s = an 8 x 8 grid at 10 mm
        # (a clinical ECoG grid, 70 mm across; 3,249 vertices, the size of the
        # reference's real surfaces, find_singularity_point.py:19-20), S1 = a
        # 51 x 51 high-density grid at 1.5 mm over the same 75 mm (160,801
        # vertices, the 160k class), S1m = a 26 x 26 grid at 3 mm (40,401
        # vertices: the smallest of the class whose multigrid level 1 is a
        # separate level, for tests of the coarse-level cycle)
        p, t = {"S1": lambda: electrode_surface(51, spacing=1.5), "S1s": lambda: electrode_surface(8, spacing=10.0),
                "S1m": lambda: electrode_surface(26, spacing=3.0)}[name]()
        return p, t, vertex_normals(p, t), triangle_areas(p, t)
    if name == "P3":
        p, t, _, _ = mesh_for_config("C3")
        p, t, _ = permute_vertices(p, t, seed=1)
        return p, t, vertex_normals(p, t), triangle_areas(p, t)
    n = CONFIG_FREQ[name]
    jitter = 0.0 if name == "C1" else 0.005
    p, t = icosphere(n, 10.0, jitter=jitter, seed=0)
    return p, t, vertex_normals(p, t), triangle_areas(p, t)
