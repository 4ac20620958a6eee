"""critical points (find_singularity_point.py:140-189).

Pinning: tests/golden/G7 holds the reference's own find_singularity_points
results on the 642-vertex mesh (float64 and float32 points), 18 fields, two
eps. The oracle (numpy, same operations) must reproduce them bit for bit; the
GPU kernel must reproduce v_length_max and the zero-vertex flags bit for bit
and the triangle flags / (lam, mu) to rounding: np.linalg.lstsq (LAPACK
dgelsd) is restated by QR + 2x2 SVD, so a triangle may only differ when lam,
mu or 1 - lam - mu is within 1e-9 of 0 (excluded band, counted).
"""
import io
import contextlib

import numpy as np
import pytest

import oracle
from conftest import load_golden

CASES = [("f64", 0), ("f64", 1), ("f32", 0), ("f32", 1)]


@pytest.mark.parametrize("tag,ei", CASES)
def test_oracle_matches_reference_golden(tag, ei):
    g = load_golden("G7_singularities")
    coords, tri, V, eps = g["coords_" + tag], g["triangles"], g["V"], g["eps"][ei]
    key = "%s_e%d" % (tag, ei)
    for k in range(len(V)):
        vmax, vf, tf, lm = oracle.singularities(coords, tri, V[k], eps)
        assert vmax == g["vmax_" + key][k]
        assert np.array_equal(vf, g["vflag_" + key][k])
        assert np.array_equal(tf, g["tflag_" + key][k])
        assert np.array_equal(lm, g["lam_mu_" + key][k])


def ambiguous(lm, tol=1e-9):
    lam, mu = lm[..., 0], lm[..., 1]
    return np.minimum(np.minimum(np.abs(lam), np.abs(mu)), np.abs(1 - lam - mu)) < tol


@pytest.mark.gpu
@pytest.mark.parametrize("tag,ei", CASES)
def test_gpu_matches_reference_golden(tag, ei):
    from mofhip import singular
    g = load_golden("G7_singularities")
    coords, tri, V, eps = g["coords_" + tag], g["triangles"], g["V"], g["eps"][ei]
    key = "%s_e%d" % (tag, ei)
    vmax, vf, tf, lm = singular.singularity_flags(coords, tri, V, eps)
    assert np.array_equal(vmax, g["vmax_" + key])
    assert np.array_equal(vf, g["vflag_" + key])
    ref_tf, ref_lm = g["tflag_" + key], g["lam_mu_" + key]
    # a triangle flagged on one side only must sit on the inside/outside
    # boundary (its lam, mu or 1 - lam - mu within 1e-9 of 0) -- and be rare
    diff = tf != ref_tf
    assert np.all(ambiguous(np.where(tf[..., None], lm, ref_lm))[diff])
    assert diff.sum() <= 2
    assert ref_tf.sum() > 0
    both = tf & ref_tf
    assert np.abs(lm[both] - ref_lm[both]).max() < 1e-9


@pytest.mark.gpu
def test_gpu_drop_in_lists():
    """The drop-in's list structure (find_singularity_point.py:176-187)."""
    from utils import find_singularity_point as fsp
    g = load_golden("G7_singularities")
    coords, tri, V = g["coords_f64"], g["triangles"], g["V"]
    sv, si, vm = fsp.find_singularity_points(coords, tri, V[15], 1e-3)
    assert vm == g["vmax_f64_e0"][15]
    assert [i for i, _ in sv] == list(np.flatnonzero(g["vflag_f64_e0"][15]))
    assert [r[0] for r in si] == list(np.flatnonzero(g["tflag_f64_e0"][15]))
    for i, P, t, bary, corners in si:
        lam, mu, nu = bary
        assert np.array_equal(t, tri[i]) and abs(lam + mu + nu - 1) < 1e-12
        assert np.allclose(P, lam * coords[t[0]] + mu * coords[t[1]] + nu * coords[t[2]])
    with contextlib.redirect_stdout(io.StringIO()) as out:
        pts = fsp.find_singularity_points_for_all_Vk(V, coords, tri, 1e-3)
    assert len(pts) == len(V) and "临界点个数" in out.getvalue()
    assert len(pts[15]) == len(sv) + len(si)


@pytest.mark.gpu
@pytest.mark.slow
def test_gpu_160k_vs_oracle_sample():
    """C3-size mesh: GPU vs the oracle on one field (vertex flags exact)."""
    from mofhip import singular, synth
    p, t, n, a = synth.mesh_for_config("C3")
    rng = np.random.default_rng(0)
    nn = p / np.linalg.norm(p, axis=1, keepdims=True)
    amb = np.stack([np.sin(0.3 * p[:, 1]), np.cos(0.4 * p[:, 2]), np.sin(0.5 * p[:, 0] + 1)], axis=1)
    V = amb - np.sum(amb * nn, axis=1, keepdims=True) * nn + 1e-3 * rng.standard_normal(p.shape)
    vmax, vf, tf, lm = singular.singularity_flags(p, t, V, 5e-3)
    # the oracle's Python loop over 327k triangles takes minutes: check a slice
    sel = np.arange(0, len(t), 97)
    ovmax, ovf, _, _ = oracle.singularities(p, t[:1], V, 5e-3)
    assert vmax[0] == ovmax and np.array_equal(vf[0], ovf)
    _, _, otf, olm = oracle.singularities(p, t[sel], V, 5e-3)
    g_tf, g_lm = tf[0][sel], lm[0][sel]
    diff = g_tf != otf
    assert np.all(ambiguous(np.where(g_tf[:, None], g_lm, olm))[diff]) and diff.sum() <= 2


@pytest.mark.gpu
@pytest.mark.parametrize("tag,ei", CASES)
def test_gpu_compact_lists_equal_dense_flags(tag, ei):
    """mof_singularities_compact returns exactly the dense path's flagged
    vertices and triangles (and their lam, mu), field by field, also when the
    first capacity is too small (the wrapper re-sizes from the totals)."""
    from mofhip import singular
    g = load_golden("G7_singularities")
    coords, tri, V, eps = g["coords_" + tag], g["triangles"], g["V"], g["eps"][ei]
    vmax, vf, tf, lm = singular.singularity_flags(coords, tri, V, eps)
    for cap in (0, 1):
        vmax2, verts, tris = singular.singularity_lists(coords, tri, V, eps, cap=cap)
        assert np.array_equal(vmax, vmax2)
        for k in range(len(V)):
            assert np.array_equal(verts[k], np.flatnonzero(vf[k]))
            tids, lms = tris[k]
            assert np.array_equal(tids, np.flatnonzero(tf[k]))
            assert np.array_equal(lms, lm[k][tids])
