"""Deflated PCG on the open S1-like patches (round-5 verdict, item 1a): is a
per-mesh set of slow modes worth building into the inner solve?

    python tools/deflation_study.py [CONFIG] [k ...]

One timestep's system (oracle, RCM order; tools/amg_proto.py) with the
library's multigrid V-cycle M (open-patch options as tools/wcycle_study.py).
The slowest modes of M A are found by Lanczos (A-inner product, full
reorthogonalisation); then the PCG iterations to 1e-4 (the mixed solve's
first inner tolerance) and to 1e-8 are counted for

  * plain PCG (the library's inner solve),
  * deflated PCG (Saad et al. 2000: x0 with W^T r0 = 0, search directions
    A-orthogonal to W) with W = the k slowest Ritz vectors of THIS system
    (the upper bound of the lever),
  * W from ANOTHER timestep of the same mesh (what a per-mesh basis built
    once could give every timestep),
  * W from the mesh alone: the k slowest modes of M_a A_a, A_a = lambda a2
    plus a small multiple of the mass-like diagonal (no signal), M_a its
    own V-cycle.

A design tool, never part of the product path.
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as P  # noqa: E402
from wcycle_study import BASE  # noqa: E402


def slow_modes(A, M, n, k, steps=240, seed=0):
    """The k smallest Ritz pairs of M A (A-orthonormal Ritz vectors)."""
    rng = np.random.default_rng(seed)
    v = M(rng.standard_normal(n))
    v /= np.sqrt(v @ (A @ v))
    V, al, be = [v], [], []
    AV = [A @ v]
    for j in range(steps):
        w = M(AV[-1])
        for u, Au in zip(V, AV):  # full reorthogonalisation, A-inner product
            w -= (w @ Au) * u
        for u, Au in zip(V, AV):
            w -= (w @ Au) * u
        Aw = A @ w
        b = np.sqrt(max(w @ Aw, 0.0))
        if b < 1e-12:
            break
        V.append(w / b)
        AV.append(Aw / b)
    Vm = np.column_stack(V)
    AVm = np.column_stack(AV)
    # Rayleigh-Ritz of M A in the A-inner product: T = V^T A M A V
    MAV = np.column_stack([M(c) for c in AVm.T])
    T = AVm.T @ MAV
    T = 0.5 * (T + T.T)
    ev, S = np.linalg.eigh(T)
    W = Vm @ S[:, :k]
    return ev[:k], W


def pcg(A, f, M, tol, W=None, maxit=3000):
    """PCG (W None) or deflated PCG with basis W (columns)."""
    if W is not None:
        AW = A @ W
        E = W.T @ AW
        Einv = np.linalg.inv(E)
        x = W @ (Einv @ (W.T @ f))
    else:
        x = np.zeros_like(f)
    r = f - A @ x
    z = M(r)
    if W is not None:
        z_p = z - W @ (Einv @ (AW.T @ z))
    else:
        z_p = z
    p = z_p.copy()
    rz = r @ z
    nf = np.linalg.norm(f)
    for it in range(1, maxit + 1):
        q = A @ p
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        if np.linalg.norm(r) <= tol * nf:
            return it
        z = M(r)
        rz2 = r @ z
        if W is not None:
            z_p = z - W @ (Einv @ (AW.T @ z))
        else:
            z_p = z
        p = z_p + (rz2 / rz) * p
        rz = rz2
    return maxit


def refine(A, f, M, W=None, first=1e-5, later=1e-3, rtol=1e-8, additive=False):
    """The mixed solve's refinement as the library runs it (fp64 outer,
    inner PCG to `first`, then to `later` on each new residual) -- inner
    iterations summed until the outer relative residual meets rtol."""
    x = np.zeros_like(f)
    r = f.copy()
    tot = 0
    nf = np.linalg.norm(f)
    Mw = M
    if additive and W is not None:
        E = np.linalg.inv(W.T @ (A @ W))

        def Mw(v):
            return M(v) + W @ (E @ (W.T @ v))
    for step in range(10):
        d, its = pcg_x(A, r, Mw, first if step == 0 else later, None if additive else W)
        tot += its
        x += d
        r = f - A @ x
        if np.linalg.norm(r) <= rtol * nf:
            return tot, step + 1
    return tot, 10


def pcg_x(A, f, M, tol, W=None, maxit=3000):
    """pcg() returning the solution too."""
    if W is not None:
        AW = A @ W
        Einv = np.linalg.inv(W.T @ AW)
        x = W @ (Einv @ (W.T @ f))
    else:
        x = np.zeros_like(f)
    r = f - A @ x
    z = M(r)
    z_p = z - W @ (Einv @ (AW.T @ z)) if W is not None else z
    p = z_p.copy()
    rz = r @ z
    nf = np.linalg.norm(f)
    for it in range(1, maxit + 1):
        q = A @ p
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        if np.linalg.norm(r) <= tol * nf:
            return x, it
        z = M(r)
        rz2 = r @ z
        z_p = z - W @ (Einv @ (AW.T @ z)) if W is not None else z
        p = z_p + (rz2 / rz) * p
        rz = rz2
    return x, maxit


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "S1m"
    ks = [int(v) for v in sys.argv[2:]] or [8, 16, 32]
    A, a2m, f, e, N = P.system(cfg, k=0)
    A1, _, f1, _, _ = P.system(cfg, k=12)
    n = A.shape[0]
    o = dict(BASE)
    lev = P.build(A, a2m, e, o)
    lev1 = P.build(A1, a2m, e, o)

    def M(r):
        return P.vcycle(lev, 0, r, o)

    def M1(r):
        return P.vcycle(lev1, 0, r, o)

    # the mesh-only operator: lambda a2 + a small diagonal shift (the data
    # term's average weight), with its own cycle
    d = A.diagonal() - a2m.diagonal()
    Aa = (a2m + sp.diags(np.full(n, max(d.mean(), 1e-12)))).tocsr()
    leva = P.build(Aa, a2m, e, o)

    def Ma(r):
        return P.vcycle(leva, 0, r, o)

    kmax = max(ks)
    ev, W = slow_modes(A, M, n, kmax)
    ev1, W1 = slow_modes(A1, M1, n, kmax)
    eva, Wa = slow_modes(Aa, Ma, n, kmax)
    print("%s: %d dofs; slowest eigenvalues of M A: %s" % (cfg, n, np.array2string(ev[:8], precision=4)))
    # where the slow modes live: share of their A-energy on the boundary rows
    bnd = np.repeat(P.system.boundary, 2)
    sh = [float((W[bnd, j] ** 2).sum() / (W[:, j] ** 2).sum()) for j in range(min(8, kmax))]
    print("  boundary rows: %.1f %% of the dofs; share of the slow modes' norm there: %s" %
          (100 * bnd.mean(), " ".join("%.2f" % s for s in sh)))
    for tol in (1e-4, 1e-8):
        base = pcg(A, f, M, tol)
        row = ["tol %.0e: plain %d" % (tol, base)]
        for k in ks:
            row.append("k=%d own %d other-timestep %d mesh-only %d" %
                       (k, pcg(A, f, M, tol, W[:, :k]), pcg(A, f, M, tol, W1[:, :k]),
                        pcg(A, f, M, tol, Wa[:, :k])))
        print("  " + " | ".join(row), flush=True)
    # the library's mixed refinement (first inner solve to 1e-5, later ones
    # to 1e-3, until 1e-8): inner iterations summed
    base, st = refine(A, f, M)
    row = ["refinement: plain %d its (%d steps)" % (base, st)]
    for k in ks:
        row.append("k=%d deflated %d/%d additive %d/%d" % ((k,) + refine(A, f, M, Wa[:, :k]) +
                                                           refine(A, f, M, Wa[:, :k], additive=True)))
    print("  " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
