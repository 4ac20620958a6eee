"""The 3-D form of the system operator that the re-forming fp64 residual
applies (csrc/mof_pcg.hip k_residual_x3sm), checked on the CPU
against the reference's assembled A_k (oracle.step_system, bit-exact with
compute_optical_flow.py:100-146):

    (A x)_i = E_i [ sum_j lambda L_ij X_j + sum_{T ni i} (A_T / 12) (gI_T . Y_T) gI_T ],
    X_v = E_v^T x_v,  Y_T = 2 X_i + X_j + X_k,  L_ij = sum_T A_T grad w_i . grad w_j

with E_v = [e_v^0; e_v^1] (2 x 3) and gI_T = sum_a I_k[T_a] grad w_a."""
import numpy as np

import oracle
from mofhip import synth


def test_operator_3d_matches_reference_assembly():
    p, t = synth.icosphere(6, jitter=0.01)
    n, a = synth.vertex_normals(p, t), synth.triangle_areas(p, t)
    N = len(p)
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    I = synth.travelling_wave(p, 2)
    lam = 0.01
    A, _ = oracle.step_system(a2, gw, e, iw, t, a, lam, I[0], I[1], 1.0)
    x = np.random.default_rng(3).standard_normal(2 * N)
    ref = A @ x
    # X_v = E_v^T x_v (planar x: x[v] and x[v + N])
    X = e[:, 0, :] * x[:N, None] + e[:, 1, :] * x[N:, None]
    acc = np.zeros((N, 3))
    gw = gw.reshape(-1, 3, 3)
    for T, (i0, i1, i2) in enumerate(t):
        vs = (i0, i1, i2)
        gI = I[0][i0] * gw[T, 0] + I[0][i1] * gw[T, 1] + I[0][i2] * gw[T, 2]
        w12 = a[T] / 12
        for c in range(3):
            i, j, k = vs[c], vs[(c + 1) % 3], vs[(c + 2) % 3]
            Y = 2 * X[i] + X[j] + X[k]
            acc[i] += w12 * (gI @ Y) * gI
            # lambda L: the triangle's contribution to L_ii, L_ij, L_ik
            for d in range(3):
                acc[i] += lam * a[T] * (gw[T, c] @ gw[T, d]) * X[vs[d]]
    y = np.concatenate([(e[:, 0, :] * acc).sum(1), (e[:, 1, :] * acc).sum(1)])
    assert np.abs(y - ref).max() <= 1e-12 * np.abs(ref).max()
