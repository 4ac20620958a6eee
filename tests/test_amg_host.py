"""The multigrid's host setup (csrc/mof_amg_host.cpp) on the CPU, through
the host-only diagnostic entry point mof_amg_probe (no device needed):
coarsening ratios, coarsest size bound, orthonormal tentative prolongators,
determinism, and the tiny-mesh case that keeps block Jacobi."""
import ctypes

import numpy as np
import pytest

import oracle
from mofhip import _lib as L
from mofhip import synth


def probe(p, t):
    n = synth.vertex_normals(p, t)
    a = synth.triangle_areas(p, t)
    _, _, e, _ = oracle.geometry(p, n, t, a)
    T = np.ascontiguousarray(t, dtype=np.int32)
    E = np.ascontiguousarray(e, dtype=np.float64)
    nl = ctypes.c_int32(0)
    sizes = np.zeros(16, dtype=np.int32)
    err = ctypes.c_double(0.0)
    curl = ctypes.c_double(0.0)
    L.check(L.lib().mof_amg_probe(L.ptr(T), L.ptr(E), len(p), len(t), ctypes.byref(nl), L.ptr(sizes),
                                  ctypes.byref(err), ctypes.byref(curl)))
    probe.curl = curl.value
    return list(sizes[:nl.value]), err.value


@pytest.mark.parametrize("mesh", ["ico", "random", "cap"])
def test_hierarchy_shape(mesh):
    if mesh == "ico":
        p, t = synth.icosphere(24, 10.0, jitter=0.005)
    elif mesh == "random":
        p, t = synth.random_sphere(4000, 10.0, seed=1)
    else:
        p, t = synth.spherical_cap(30, 10.0, 0.6)
    sizes, err = probe(p, t)
    assert sizes[0] == len(p)
    assert len(sizes) >= 2
    for a, b in zip(sizes, sizes[1:]):
        assert b < a / 3  # aggregates of several vertices
    assert 3 * sizes[-1] <= 128  # coarsest solved densely (<= 128 dofs)
    assert err < 1e-5  # fp32 Q rows, orthonormal columns per aggregate


def test_hierarchy_deterministic_and_tiny():
    p, t = synth.icosphere(12, 10.0)
    assert probe(p, t) == probe(p, t)
    p1, t1 = synth.icosphere(1, 10.0)  # 12 vertices, 24 dofs: does not coarsen
    sizes, _ = probe(p1, t1)
    assert sizes == [len(p1)]


def test_fold_criterion_separates_folded_from_spheres():
    """The multigrid's fold choice (amg_build, kFoldCurl = 0.35: level 1's
    prolongator smoothed on closed folded surfaces): the median
    turn of the tangent planes inside the coarse aggregates (sigma_3 /
    sigma_1 of their near-null blocks) is large on a folded surface (the
    F3 class, synth.folded_sphere) and stays small on jittered and random
    spheres, at any resolution (round 5: F3 0.46, C3 0.24, R3 0.09 at 163,842
    vertices)."""
    p, t = synth.folded_sphere(64)
    probe(p, t)
    folded = probe.curl
    p, t = synth.icosphere(64, 10.0, jitter=0.005)
    probe(p, t)
    sphere = probe.curl
    p, t = synth.random_sphere(40962, 10.0, seed=0)
    probe(p, t)
    hull = probe.curl
    assert folded >= 0.35 > max(sphere, hull), (folded, sphere, hull)


def test_probe_rejects_bad_input():
    p, t = synth.icosphere(2, 10.0)
    bad = np.ascontiguousarray(t, dtype=np.int32)
    bad[0, 0] = len(p)
    E = np.zeros((len(p), 2, 3))
    nl, sizes = ctypes.c_int32(0), np.zeros(16, dtype=np.int32)
    rc = L.lib().mof_amg_probe(L.ptr(bad), L.ptr(E), len(p), len(t), ctypes.byref(nl), L.ptr(sizes), None, None)
    with pytest.raises(L.MofError):
        L.check(rc)


@pytest.mark.parametrize("nblk", [1, 7, 8, 9, 160, 641])
@pytest.mark.parametrize("batch", [1, 3, 8, 15, 41, 256])
@pytest.mark.parametrize("group", [0, 1, 8, 32])
def test_xcd_order_visits_every_pair_once(nblk, batch, group):
    """The XCD-aware workgroup order of the row kernels (system groups of
    8 / 32 / all) covers every (row block, system) pair exactly once, also
    with partial groups and row-block counts not divisible by 8."""
    L.check(L.lib().mof_xcd_map_check(nblk, batch, group))


def test_xcd_grid_past_dispatch_limit_fails_loudly():
    """A row-kernel grid past 2^32 - 1 work-items (a dispatch would run only
    part of its workgroups) is refused with an error, never launched."""
    # 40,000 row blocks x 1024 systems in groups of 8: 41 M workgroups of 256
    with pytest.raises(L.MofError):
        L.check(L.lib().mof_xcd_map_check(40000, 1024, 8))
    L.check(L.lib().mof_xcd_map_check(641, 1024, 8))  # C3's size: fine


def test_batch_cap_keeps_every_grid_within_dispatch_limit():
    """The batch the library never passes (mof_mesh_info.max_batch: the
    auto and explicit batches are clamped to it) is the largest whose
    XCD-ordered grid fits 2^32 - 1 work-items: one more system is refused.
    40,000 blocks per system is a 10 M-slot operator (the block assembly's
    grid at ~1.4 M vertices); 4,608 is C3's (1.18 M SELL slots)."""
    for nblk, grp in ((40000, 8), (4608, 8), (641, 8), (12345, 0)):
        cap = ctypes.c_int32(0)
        L.check(L.lib().mof_xcd_batch_cap(nblk, grp, ctypes.byref(cap)))
        assert cap.value >= 1
        if nblk * cap.value < 2 ** 31:  # mof_xcd_map_check walks every workgroup: small grids only
            L.check(L.lib().mof_xcd_map_check(nblk, cap.value, grp))
        with pytest.raises(L.MofError):
            L.check(L.lib().mof_xcd_map_check(nblk, cap.value + 8, grp))
    cap = ctypes.c_int32(0)
    L.check(L.lib().mof_xcd_batch_cap(4608, 8, ctypes.byref(cap)))
    assert 3000 < cap.value < 3700  # C3: B = 1024 fits, ~3.6 k would not
