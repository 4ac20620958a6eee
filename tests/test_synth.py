"""Synthetic meshes of the bench configurations (CPU): the S1-like
reconstructed patch (mofhip.synth.electrode_surface, after
S1_reconstruct_surface.py:82-97) is a consistently oriented open 2-manifold
without folds, of the stated sizes; the icosphere counts of SURVEY.md §8d."""
import numpy as np
import pytest

from mofhip import synth


def _check_manifold(p, t):
    directed = {}
    for a, b, c in t.tolist():
        for u, v in ((a, b), (b, c), (c, a)):
            assert (u, v) not in directed, "edge used twice in one direction: inconsistent orientation"
            directed[(u, v)] = True
    und = {}
    for u, v in directed:
        und[(min(u, v), max(u, v))] = und.get((min(u, v), max(u, v)), 0) + 1
    assert max(und.values()) <= 2
    return sum(1 for c in und.values() if c == 1)


@pytest.mark.parametrize("n_side,nv", [(8, 3249), (5, None)])
def test_electrode_surface(n_side, nv):
    p, t = synth.electrode_surface(n_side)
    if nv is not None:
        assert len(p) == nv
    assert t.dtype == np.int32 and t.min() == 0 and t.max() == len(p) - 1
    nb = _check_manifold(p, t)
    assert nb > 0  # an open patch
    fn = np.cross(p[t[:, 1]] - p[t[:, 0]], p[t[:, 2]] - p[t[:, 0]])
    assert (fn[:, 2] > 0).all()  # no fold: every face towards +z
    assert synth.triangle_areas(p, t).min() > 0
    n = synth.vertex_normals(p, t)
    assert np.isfinite(n).all() and n[:, 2].min() > 0.5
    # mostly regular: butterfly vertices have valence 6
    inc = np.bincount(t.ravel(), minlength=len(p))
    assert (inc == 6).mean() > 0.85  # boundary vertices have fewer
    # deterministic
    p2, t2 = synth.electrode_surface(n_side)
    assert np.array_equal(p, p2) and np.array_equal(t, t2)


def test_icosphere_counts():
    for n in (1, 2, 8):
        p, t = synth.icosphere(n)
        assert len(p) == 10 * n * n + 2 and len(t) == 20 * n * n
        assert _check_manifold(p, t) == 0


def test_folded_sphere():
    """F3's folded cortex-like surface (synth.folded_sphere) on a small
    topology: the icosphere's counts, every triangle outward (a radial graph
    cannot fold), the configured peak-to-trough depth, seeded."""
    p, t = synth.folded_sphere(16, radius=10.0, depth=0.3)
    assert p.shape == (10 * 16 ** 2 + 2, 3) and t.shape == (20 * 16 ** 2, 3)
    r = np.linalg.norm(p, axis=1)
    assert abs(r.min() - 8.5) < 1e-9 and abs(r.max() - 11.5) < 1e-9
    c = np.cross(p[t[:, 1]] - p[t[:, 0]], p[t[:, 2]] - p[t[:, 0]])
    assert ((c * p[t].mean(axis=1)).sum(axis=1) > 0).all()
    p2, _ = synth.folded_sphere(16, radius=10.0, depth=0.3)
    assert np.array_equal(p, p2)
