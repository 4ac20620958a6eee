"""The re-forming fp64 residual of the mixed path reads each incident
triangle's geometry (hat gradients, the other corners' tangent bases, A_T/12)
from the mesh's incidence-ordered planes (csrc/mof_pcg.hip
residual_geometry / apply_row_rcn_soa) instead of gathering it per lane
(MOF_RES_GATHER=1). The values and the arithmetic are the same, so V, the
iteration counts and the residuals are bit-identical -- on a regular mesh
with ragged batches, an open surface, a scattered vertex order and the
recovery passes (the residual r64 = f - A x64 of the
refinement; compute_optical_flow.py:100-147's system)."""
import numpy as np
import pytest

from mofhip import DeviceMesh, synth

pytestmark = pytest.mark.gpu

_KEYS = ("iterations", "max_iterations", "failed", "recovered", "outer_steps", "max_rel_residual")


def _mesh(p, t, **kw):
    return DeviceMesh(p, synth.vertex_normals(p, t), t, synth.triangle_areas(p, t), **kw)


def _both(monkeypatch, make, I, **opts):
    tk = np.arange(len(I), dtype=np.float64)
    out = []
    for v in ("1", "0"):
        monkeypatch.setenv("MOF_RES_GATHER", v)
        m = make()  # a fresh handle: the planes are built on its first residual
        out.append(m.solve_range(I, tk, 0, len(I) - 1, 0.01, **opts))
        m.close()
    return out


@pytest.mark.parametrize("case,opts", [
    ("ico", dict(precision="mixed", precond="amg", batch=0)),
    ("ico", dict(precision="mixed", precond="jacobi", batch=33)),
    ("S1s", dict(precision="mixed", precond="amg", batch=0)),
    ("perm", dict(precision="mixed", precond="jacobi", batch=0)),
    ("recovery", dict(precision="mixed", precond="amg", max_iter=3, max_outer=1)),
])
def test_residual_geometry_planes_bit_identical(case, opts, monkeypatch):
    if case == "S1s":
        p, t, _, _ = synth.mesh_for_config("S1s")
        I = synth.config_wave("S1s", p, 71)
    else:
        p, t = synth.icosphere(32 if case != "recovery" else 16, jitter=0.005)
        if case == "perm":
            p, t, _ = synth.permute_vertices(p, t, seed=3)
        I = synth.travelling_wave(p, 71 if case != "recovery" else 20)
    (V0, s0), (V1, s1) = _both(monkeypatch, lambda: _mesh(p, t, reorder=case != "perm"), I, **opts)
    assert s1["failed"] == 0 and s1["max_rel_residual"] <= 1e-8
    if case == "recovery":
        assert s1["recovered"] > 0
    assert np.array_equal(V0, V1)
    for k in _KEYS:
        assert s0[k] == s1[k], k
