"""Coarse-space study for folded surfaces (design tool, CPU): PCG iterations
to a 1e-4 relative residual of one timestep's oracle system with an
aggregation V-cycle whose tentative prolongator interpolates k near-null
vectors per aggregate:

  k = 3   the library's: the three ambient directions c seen in each
          vertex's tangent frame, v_i = E_i c (E_i = [e_i^0; e_i^1], 2x3)
  k = 6   plus the rotations about the three axes through the aggregate's
          centroid, v_i = E_i (w x (x_i - x_I)): the tangent fields of a
          rigid motion, the other smooth modes of the ambient-projected
          vector Laplacian on a curved surface

Coarse levels carry k dofs per node (the library's GPU levels are 3x3
blocks). Aggregation, smoother (damped block Jacobi, V(1,1)), dense
coarsest solve as tools/amg_proto.py.

    python tools/nullspace_study.py CONFIG [k ...] [w2]

The oracle is test infrastructure; this script is a design tool, never part
of the product path.
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as ap  # noqa: E402
from scipy.sparse.csgraph import reverse_cuthill_mckee  # noqa: E402


def positions_rcm(cfg):
    """Vertex positions in the RCM order ap.system uses."""
    p, t, n, a = ap.synth.mesh_for_config(cfg)
    N = len(p)
    r = np.concatenate([t[:, 0], t[:, 1], t[:, 2], t[:, 1], t[:, 2], t[:, 0]])
    c = np.concatenate([t[:, 1], t[:, 2], t[:, 0], t[:, 0], t[:, 1], t[:, 2]])
    G = sp.csr_matrix((np.ones(len(r)), (r, c)), shape=(N, N))
    order = reverse_cuthill_mckee(G.tocsr(), symmetric_mode=True)
    return p[order]


def tentative_k(agg, na, Bnull, bs):
    """Per-aggregate QR of the stacked (bs*m x k) near-null block (MGS twice,
    dead columns dropped): P (n*bs x k*na), coarse near-null (na, k, k)."""
    n, k = len(agg), Bnull.shape[2]
    order = np.argsort(agg, kind="stable")
    bounds = np.searchsorted(agg[order], np.arange(na + 1))
    rows, cols, vals = [], [], []
    Bc = np.zeros((na, k, k))
    for I in range(na):
        mem = order[bounds[I]:bounds[I + 1]]
        Bm = Bnull[mem].reshape(-1, k)
        Q = Bm.copy()
        R = np.zeros((k, k))
        cmax = np.sqrt((Bm ** 2).sum(0)).max()
        dead = [False] * k
        for c in range(k):
            for _ in range(2):
                for pp in range(c):
                    if dead[pp]:
                        continue
                    d = Q[:, pp] @ Q[:, c]
                    R[pp, c] += d
                    Q[:, c] -= d * Q[:, pp]
            s = np.sqrt(Q[:, c] @ Q[:, c])
            dead[c] = not (s > 1e-6 * cmax) or Bm.shape[0] < c + 1
            if dead[c]:
                Q[:, c] = 0
                R[:, c] = 0
                continue
            R[c, c] = s
            Q[:, c] /= s
        Bc[I] = R
        dofs = (mem[:, None] * bs + np.arange(bs)).ravel()
        for c in range(k):
            if not dead[c]:
                rows.append(dofs)
                cols.append(np.full(len(dofs), k * I + c))
                vals.append(Q[:, c])
    P = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(n * bs, k * na))
    return P, Bc


def near_null(e, x, agg, k):
    """(n, 2, k): the ambient directions in each tangent frame, and with
    k = 6 the rotations about the aggregate centroids."""
    n = len(e)
    B = np.zeros((n, 2, k))
    B[:, :, :3] = e
    if k == 6:
        na = agg.max() + 1
        cen = np.zeros((na, 3))
        np.add.at(cen, agg, x)
        cen /= np.bincount(agg, minlength=na)[:, None]
        d = x - cen[agg]
        for a in range(3):
            w = np.zeros(3)
            w[a] = 1.0
            B[:, :, 3 + a] = np.einsum("nij,nj->ni", e, np.cross(w, d))
    return B


def build(A, e, x, k, om=(0.85, 1.05), w2=False):
    levels = []
    bs = 2
    Acur = A
    Bnull = None
    lvl = 0
    while True:
        L = ap.Level()
        L.A, L.bs = Acur, bs
        L.D, L.Dinv = ap.block_diag_inv(Acur, bs)
        L.om = om[0 if lvl == 0 else 1]
        levels.append(L)
        n = Acur.shape[0] // bs
        if n * bs <= 128 or n * k <= 128:
            L.coarse = np.linalg.inv(Acur.toarray() + np.diag((np.abs(Acur).sum(1).A1 == 0) * 1.0))
            break
        G = ap.block_graph(Acur, bs)
        G = (G + sp.eye(G.shape[0])).tocsr()
        G.sort_indices()
        agg, na = ap.aggregate(G)
        if na >= n:
            L.coarse = np.linalg.inv(Acur.toarray())
            break
        if lvl == 0:
            Bnull = near_null(e, x, agg, k)
        P, Bc = tentative_k(agg, na, Bnull, bs)
        L.P = P
        Ac = (P.T @ Acur @ P).tocsr()
        dead = np.abs(Ac).sum(1).A1 == 0
        Acur = (Ac + sp.diags(dead * 1.0)).tocsr()
        Bnull = Bc
        bs = k
        lvl += 1
    return levels


def main():
    cfg = sys.argv[1]
    args = sys.argv[2:] or ["3", "6"]
    w2 = "w2" in args
    ks = [int(a) for a in args if a != "w2"]
    A, a2m, f, e, N = ap.system(cfg)
    x = positions_rcm(cfg)
    opts = {"w2": True} if w2 else {}
    for k in ks:
        levels = build(A, e, x, k)
        sizes = [lv.A.shape[0] // lv.bs for lv in levels]
        nnz = sum(lv.A.nnz for lv in levels)
        its = ap.pcg(A, f, lambda r: ap.vcycle(levels, 0, r, opts))
        print("%s k=%d%s its(1e-4) %4d rho %.4f levels %s op complexity %.2f"
              % (cfg, k, " w2" if w2 else "", its, ap.pcg.rho, sizes, nnz / A.nnz), flush=True)


if __name__ == "__main__":
    main()
