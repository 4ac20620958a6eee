"""Warm start from the previous timestep's V, measured on the CPU (design tool;
verdict round 2 item 8).

    python tools/warm_start.py CONFIG [K] [omega ...]

For K consecutive timesteps of the travelling wave I_k = sin(3 phi - omega k)
(the bench's signal has omega = 0.3 rad per step), each system (the oracle's
A_k, f_k, RCM order as the library) is solved the way the library's mixed
solve does -- refinement steps of an inner multigrid-PCG (amg_proto's cycle,
the library's V(1,1)) to 1e-4 of the step's residual, later steps to the
adaptive tolerance 0.3 rtol |f| / |r| clamped to [1e-4, 0.5], until
|f - A x| <= 1e-8 |f| -- from x0 = 0 and from x0 = V_{k-1}. Prints the inner
iterations per timestep of both and the start residual |f - A V_{k-1}| / |f|.
The time step dt scales f (and V) only, not A: t_k = i/512 (S3's
convention) gives the same iteration counts as dt = 1.
"""
import os
import sys

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as ap  # noqa: E402

import oracle  # noqa: E402  (amg_proto put oracle/ on sys.path)
from mofhip import synth  # noqa: E402


def systems(cfg, K, omega):
    p, t, n, a = synth.mesh_for_config(cfg)
    N = len(p)
    phi = np.arctan2(p[:, 1], p[:, 0])
    I = np.array([np.sin(3.0 * phi - omega * k) for k in range(K + 1)])
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    r = np.concatenate([t[:, 0], t[:, 1], t[:, 2], t[:, 1], t[:, 2], t[:, 0]])
    c = np.concatenate([t[:, 1], t[:, 2], t[:, 0], t[:, 0], t[:, 1], t[:, 2]])
    G = sp.csr_matrix((np.ones(len(r)), (r, c)), shape=(N, N))
    order = reverse_cuthill_mckee(G.tocsr(), symmetric_mode=True)
    dof = np.empty(2 * N, dtype=np.int64)
    dof[0::2] = order
    dof[1::2] = order + N
    a2m = sp.csr_matrix(0.01 * a2)[dof][:, dof].tocsr()
    out = []
    for k in range(K):
        A, f = oracle.step_system(a2, gw, e, iw, t, a, 0.01, I[k], I[k + 1], 1.0)
        out.append((sp.csr_matrix(A)[dof][:, dof].tocsr(), f[dof]))
    return out, a2m, e[order]


def pcg_x(A, b, M, tol):
    """amg_proto.pcg on the correction A d = b, relative to |b|."""
    return ap.pcg(A, b, M, tol=tol)


def refine(A, f, M, x0, rtol=1e-8, inner=1e-4):
    """The library's mixed solve: returns (x, inner iterations, steps)."""
    x = x0.copy()
    nf = np.linalg.norm(f)
    its = steps = 0
    for o in range(10):
        r = f - A @ x
        nr = np.linalg.norm(r)
        if nr <= rtol * nf:
            break
        tol = inner if o == 0 else min(0.5, max(inner, 0.3 * rtol * nf / nr))
        d, n = pcg_d(A, r, M, tol)
        x += d
        its += n
        steps += 1
    return x, its, steps


def pcg_d(A, b, M, tol, maxit=2000):
    x = np.zeros_like(b)
    r = b.copy()
    z = M(r)
    p = z.copy()
    rz = r @ z
    nb = np.linalg.norm(b)
    for it in range(1, maxit + 1):
        q = A @ p
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        if np.linalg.norm(r) <= tol * nb:
            return x, it
        z = M(r)
        rz2 = r @ z
        p = z + (rz2 / rz) * p
        rz = rz2
    return x, maxit


def main():
    cfg = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    omegas = [float(v) for v in sys.argv[3:]] or [0.3]
    for om in omegas:
        sysl, a2m, e = systems(cfg, K, om)
        cold = warm = 0
        prev = None
        eps = []
        for k, (A, f) in enumerate(sysl):
            levels = ap.build(A, a2m, e, {})
            M = lambda r, lv=levels: ap.vcycle(lv, 0, r, {})  # noqa: E731
            x, n0, _ = refine(A, f, M, np.zeros_like(f))
            if k > 0:  # warm start from the previous timestep's solution
                eps.append(np.linalg.norm(f - A @ prev) / np.linalg.norm(f))
                _, n1, _ = refine(A, f, M, prev)
                cold += n0
                warm += n1
            prev = x
        print("%s omega %.3f: %d timesteps, PCG its/timestep cold %.2f warm %.2f (%.1f %%), "
              "start residual |f - A V_k-1| / |f| = %.3f" % (cfg, om, K - 1, cold / (K - 1), warm / (K - 1),
                                                            100.0 * (cold - warm) / cold, float(np.mean(eps))),
              flush=True)


if __name__ == "__main__":
    main()
