"""The system-major fp64 residual of the mixed path (csrc/mof_pcg.hip
k_residual_x3sm: one SELL slice per wave, one system per lane, the operator
applied in ambient 3-D from system-interleaved X = E x and I copies) against
the row-major tangent-frame k_residual_rcn it replaces (MOF_RES_SM=0). Both
apply the reference's A_k (compute_optical_flow.py:100-146) in fp64 --
tests/test_operator_3d.py checks the 3-D identity on the CPU -- so the
refinement converges to the same V within its tolerance (rtol 1e-8), with
the same refinement steps; on full and partial 64-system groups, ragged
batches, an open surface, a vertex order scattered by a random relabelling,
and the recovery passes that re-solve failed systems. The kernel's partial
|r|^2 records follow block_sum's tree, and a system's bits do not depend on
its lane: a batch split leaves V bit-identical."""
import numpy as np
import pytest

from mofhip import DeviceMesh, synth

pytestmark = pytest.mark.gpu

_KEYS = ("failed", "recovered", "outer_steps")


def _close(V0, V1, s0, s1):
    assert s1["failed"] == 0 and s1["max_rel_residual"] <= 1e-8
    # two solutions within rtol 1e-8 of the same system: |V1 - V0| is of the
    # order of either's distance from spsolve (3-9e-8 on these meshes)
    scale = float(np.abs(V0).max())
    assert np.abs(V1 - V0).max() <= 2e-7 * scale
    for k in _KEYS:
        assert s0[k] == s1[k], k
    assert abs(s0["iterations"] - s1["iterations"]) <= 0.02 * s0["iterations"] + 2


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
    _close(V0, V1, s0, s1)


def test_residual_sm_recovery_passes(monkeypatch):
    """Inner solves cut at 3 iterations with one refinement step: every
    system fails the multigrid solve and is re-solved by the recovery passes
    (the damped multigrid and mixed block-Jacobi passes run the system-major
    residual on the selected systems only; the others keep x64)."""
    p, t = synth.icosphere(16, jitter=0.005)
    m = _mesh(p, t)
    I = synth.travelling_wave(p, 20)
    (V0, s0), (V1, s1) = _both(monkeypatch, m, I, precision="mixed", precond="amg", max_iter=3, max_outer=1)
    assert s0["recovered"] > 0
    _close(V0, V1, s0, s1)


def test_residual_sm_batch_split_bit_identical(monkeypatch):
    """A system's bits do not depend on its lane or 64-system group: the
    same timesteps solved as one batch of 70 and as batches of 33 / 33 / 4
    (different lanes, groups and partial groups) give the same V."""
    monkeypatch.setenv("MOF_RES_SM", "1")
    p, t = synth.icosphere(32, jitter=0.005)
    m = _mesh(p, t)
    I = synth.travelling_wave(p, 71)
    tk = np.arange(71, dtype=np.float64)
    Va, sa = m.solve_range(I, tk, 0, 70, 0.01, precision="mixed", precond="jacobi", batch=0)
    Vb, sb = m.solve_range(I, tk, 0, 70, 0.01, precision="mixed", precond="jacobi", batch=33)
    assert sa["failed"] == sb["failed"] == 0
    assert np.array_equal(Va, Vb)
