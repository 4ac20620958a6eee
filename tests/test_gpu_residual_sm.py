"""The system-major fp64 residual of the mixed path (csrc/mof_pcg.hip
k_residual_sm: one SELL slice per wave, one system per lane, x64 and the I
rows read from system-interleaved copies) against the row-major
k_residual_rcn it replaces (MOF_RES_SM=0). The residual r64 = f - A x64 of
the refinement (compute_optical_flow.py:147's system) keeps
its arithmetic per (row, system) and the partial |r|^2 / |f|^2 records keep
their summation tree, so V, the iteration counts and the residuals must be
bit-identical -- on full and partial 64-system groups, ragged batches, an
open surface, a vertex order scattered by a random relabelling, and the
recovery passes that re-solve failed systems."""
import numpy as np
import pytest

from mofhip import DeviceMesh, synth

pytestmark = pytest.mark.gpu

_KEYS = ("iterations", "max_iterations", "failed", "recovered", "outer_steps", "max_rel_residual")


def _mesh(p, t, **kw):
    return DeviceMesh(p, synth.vertex_normals(p, t), t, synth.triangle_areas(p, t), **kw)


def _both(monkeypatch, m, I, **opts):
    tk = np.arange(len(I), dtype=np.float64)
    out = []
    for v in ("0", "1"):
        monkeypatch.setenv("MOF_RES_SM", v)
        out.append(m.solve_range(I, tk, 0, len(I) - 1, 0.01, **opts))
    return out


@pytest.mark.parametrize("case,opts", [
    ("ico", dict(precision="mixed", precond="amg", batch=0)),       # 70 systems: 64 + 6 lanes
    ("ico", dict(precision="mixed", precond="jacobi", batch=33)),   # ragged batches 33, 33, 4
    ("S1s", dict(precision="mixed", precond="amg", batch=0)),       # open surface
    ("perm", dict(precision="mixed", precond="jacobi", batch=0)),   # scattered vertex order
])
def test_residual_sm_bit_identical(case, opts, monkeypatch):
    if case == "S1s":
        p, t, _, _ = synth.mesh_for_config("S1s")
        I = synth.config_wave("S1s", p, 71)
    else:
        p, t = synth.icosphere(32, jitter=0.005)
        if case == "perm":
            p, t, _ = synth.permute_vertices(p, t, seed=3)
        I = synth.travelling_wave(p, 71)
    # perm: the internal order is the random one (no RCM), so every gather scatters
    m = _mesh(p, t, reorder=case != "perm")
    (V0, s0), (V1, s1) = _both(monkeypatch, m, I, **opts)
    assert s1["failed"] == 0 and s1["max_rel_residual"] <= 1e-8
    assert np.array_equal(V0, V1)
    for k in _KEYS:
        assert s0[k] == s1[k], k


def test_residual_sm_recovery_passes(monkeypatch):
    """Inner solves cut at 3 iterations with one refinement step: every
    system fails the multigrid solve and is re-solved by the recovery passes
    (the damped multigrid and mixed block-Jacobi passes run the system-major
    residual on the selected systems only; the others keep x64)."""
    p, t = synth.icosphere(16, jitter=0.005)
    m = _mesh(p, t)
    I = synth.travelling_wave(p, 20)
    (V0, s0), (V1, s1) = _both(monkeypatch, m, I, precision="mixed", precond="amg", max_iter=3, max_outer=1)
    assert s0["recovered"] > 0 and s1["failed"] == 0
    assert np.array_equal(V0, V1)
    for k in _KEYS:
        assert s0[k] == s1[k], k
