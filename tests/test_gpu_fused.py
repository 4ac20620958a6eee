"""The fused small-mesh solve (MOF_SOLVE_FUSED, csrc/mof_pcg.hip
k_solve_fused): the whole fp64 block-Jacobi solve of a batch in one launch,
one workgroup per system running the eager kernels' bodies row block by row
block. It must give the eager path's bits: V, the convergence / failure
flags and the iteration counts (small meshes), and V within
the north-star bar of spsolve (compute_optical_flow.py:147) through the
reference-captured goldens."""
import numpy as np
import pytest

from conftest import load_golden
from mofhip import DeviceMesh, synth

pytestmark = pytest.mark.gpu


def _solve(m, I, tk, fused, **kw):
    opts = dict(precision="f64", precond="jacobi", time_spmv=True)
    opts.update(kw)
    return m.solve_range(I, tk, 0, len(I) - 1, 0.01, fused=fused, **opts)


def _mesh(p, t):
    return DeviceMesh(p, synth.vertex_normals(p, t), t, synth.triangle_areas(p, t))


@pytest.mark.parametrize("n,jitter,T,batch", [
    (8, 0.0, 16, 0),        # C1: 642 vertices, the reference's parity case
    (8, 0.0, 16, 4),        # ragged batches (4, 4, 4, 3)
    (17, 0.005, 12, 0),     # 2,892 vertices: the reference's real mesh size (~3,101)
    (32, 0.005, 6, 0),      # 10,242 vertices, 40 row blocks (fused forced)
])
def test_fused_bit_identical_to_eager(n, jitter, T, batch):
    p, t = synth.icosphere(n, jitter=jitter)
    m = _mesh(p, t)
    I = synth.travelling_wave(p, T)
    tk = np.arange(T, dtype=np.float64)
    Ve, se = _solve(m, I, tk, False, batch=batch)
    Vf, sf = _solve(m, I, tk, True, batch=batch)
    assert se["fused_launches"] == 0 and sf["fused_launches"] == sf["batches"] > 0
    assert np.array_equal(Ve, Vf)
    for k in ("iterations", "max_iterations", "failed", "outer_steps", "max_rel_residual"):
        assert se[k] == sf[k], k
    assert sf["failed"] == sf["recovered"] == 0 and sf["max_rel_residual"] <= 1e-8


def test_fused_is_the_small_mesh_default():
    p, t = synth.icosphere(8)
    m = _mesh(p, t)
    I = synth.travelling_wave(p, 6)
    tk = np.arange(6, dtype=np.float64)
    _, s_auto = _solve(m, I, tk, None)
    assert s_auto["fused_launches"] == s_auto["batches"] == 1
    p2, t2 = synth.icosphere(32, jitter=0.005)  # 40 row blocks: eager unless asked
    _, s_big = _solve(_mesh(p2, t2), synth.travelling_wave(p2, 3), np.arange(3.0), None)
    assert s_big["fused_launches"] == 0


def test_fused_failures_match_eager():
    """Systems stopped at max_iter: the same systems fail with the same flags
    (no recovery), and with recovery (eager re-solves) the same V."""
    p, t = synth.icosphere(8)
    m = _mesh(p, t)
    I = synth.travelling_wave(p, 8)
    tk = np.arange(8, dtype=np.float64)
    Ve, se = _solve(m, I, tk, False, max_iter=5, max_outer=2, recovery=False)
    Vf, sf = _solve(m, I, tk, True, max_iter=5, max_outer=2, recovery=False)
    assert se["failed"] == sf["failed"] == 7
    assert np.isnan(Ve).all() and np.isnan(Vf).all()
    assert se["iterations"] == sf["iterations"] and se["max_iterations"] == sf["max_iterations"]
    Ve, se = _solve(m, I, tk, False, max_iter=5, max_outer=2)
    Vf, sf = _solve(m, I, tk, True, max_iter=5, max_outer=2)
    assert se["failed"] == sf["failed"] == 0 and se["recovered"] == sf["recovered"] == 7
    assert np.array_equal(Ve, Vf)


@pytest.mark.parametrize("case", ["G1_ico642", "G2_cap641", "G5_dt512"])
def test_fused_vs_golden_spsolve(case):
    g = load_golden(case)
    m = DeviceMesh(g["coordinates"], g["normals"], g["triangles"], g["areas"])
    I, tk = g["I"], g["t_k"]
    V, st = m.solve_range(I, tk, 0, len(I) - 1, float(g["lambda_"]), precision="f64", precond="jacobi",
                          fused=True, time_spmv=True)
    assert st["fused_launches"] >= 1 and st["failed"] == st["recovered"] == 0
    ref = g["V_k"]
    scale = max(1.0, float(np.abs(ref).max()))  # dt = 1/512 (G5): |V| ~ 600
    assert np.abs(V - ref).max() < 1e-6 * scale
