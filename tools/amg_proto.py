"""CPU prototype of the inner solve's multigrid preconditioner (research tool).

    python tools/amg_proto.py CONFIG [variant ...]

Builds one timestep's system with the oracle (fp64, caller order), renumbers
it by reverse Cuthill-McKee like the library, and counts the PCG iterations
(fp64) to a 1e-4 relative residual -- the first refinement step of the
mixed solve -- for aggregation-multigrid variants:

  base        the library's cycle: greedy aggregation on the block graph,
              tentative prolongator from the tangent-frame near-null space,
              V(1,1) damped block Jacobi (omega 0.85 / 1.05), dense coarsest
  theta=X     level-0 aggregation on strong couplings only
              (||A_ij||_F >= X sqrt(||A_ii||_F ||A_jj||_F))
  theta2=X    the same with the strength measured on lambda*a2 (per mesh)
  om=X,Y      smoother damping (fine, coarse)
  omb=X       level-0 damping X on the boundary rows (open surfaces) only
  sgn=1       level-0 aggregation on the negative couplings of lambda*a2 only
  amax1=K     coarse-level aggregates of at most K nodes
  theta1=X    coarse-level aggregation on strong couplings only
  theta1only=X  the same at level 1 only
  theta1a2=X  level 1 only, the strength from P^T (lambda a2) P (mesh-only)
  l1          l1 block-Jacobi smoother (D + sum_j ||A_ij|| I), undamped
  sa=X        smoothed prolongator P = (I - X D^-1 A) P_tent at level 0,
              with the system's own A (per timestep)
  sa2=X       the same with lambda*a2 only (a per-mesh, timestep-free P)
  sa1=X       smoothed P at the coarse levels (>= 1), with the level's own A
  sa1a2=X     the same with the coarse levels' Galerkin image of lambda*a2 (per mesh)
  sa1only=1   sa1 / sa1a2 at level 1 only (the transition 1 -> 2)
  w2          two coarse-grid visits per level-1 cycle (W-cycle at level 1)
  kcyc=K      K-cycle at level 1: level 2's problem by K flexible-CG steps
              preconditioned by level 2's cycle (the outer PCG turns flexible)
  nu1=K       K pre- and K post-smoothing sweeps at the coarse levels (V(K,K))
  q1=F        the sweeps at levels >= 1 on a stored copy of the operator: 1 bf16,
              2 int8 + one scale per block, 3 fp8 e4m3 + one scale per block,
              4 int8 + one scale per row
  q0=F        the same for the level-0 sweeps (the PCG operator stays exact)
              (formats 5: D^-1/2 A D^-1/2 with D = diag(A), entries in
              [-1, 1] as int8 with the one fixed scale 1/127, rescaled)
  amax=K      level-0 aggregates of at most K nodes (root + K-1 free
              neighbours; design study)
  cheb=K      level 0 smoothed by degree-K Chebyshev in D^-1 A on both sides
              (pre from x = 0); chebpost=K after the coarse correction only
              (pre stays om D^-1 b); cr=X the interval [lmax / X, lmax]
  mcgs=1      level 0 smoothed by multicolour block Gauss-Seidel (forward
              before, backward after; gsom=X damping)
  bsw=K       K extra block-Jacobi sweeps on the boundary rows (open
              surfaces) and bring=R rings of neighbours (bom=X damping), after
              the pre- and before the post-smoothing (the library's k_bsweep)
  exact=L     an exact (sparse LU) solve from level L down: the two-grid
              bound at L = 1
  galq=1      with q1: the coarse Galerkin products from the stored copy
  f32gal=1    the Galerkin products in fp32 (fp32 operands and sums, as the
              GPU's k_galerkin* kernels)
  s0=F        level 0 as the GPU runs it: the sweeps, the smoother's D
              (from the copy's diagonal blocks) and the level-0 Galerkin
              product all on the stored copy in format F (1 = bf16, today)

The oracle is test infrastructure; this script is a design tool, never part
of the product path.
"""
import sys
import os

import numpy as np
import scipy.sparse as sp
import scipy.linalg as sla
import scipy.sparse.linalg as sla_sparse
from scipy.sparse.csgraph import reverse_cuthill_mckee

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))
import oracle  # noqa: E402
from mofhip import synth  # noqa: E402


def system(cfg, k=0):
    if cfg.startswith("ico"):
        p, t = synth.icosphere(int(cfg[3:]), 0.005)
        n, a = synth.vertex_normals(p, t), synth.triangle_areas(p, t)
    else:
        p, t, n, a = synth.mesh_for_config(cfg)
    # the bench's signal for the config (synth.config_wave: on the S1-like
    # patches a wave across the grid), PROTO_PINWHEEL=1: the atan2 pinwheel
    if os.environ.get("PROTO_PINWHEEL") == "1" or cfg.startswith("ico"):
        I = synth.travelling_wave(p, k + 2)
    else:
        I = synth.config_wave(cfg, p, k + 2)
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    A, f = oracle.step_system(a2, gw, e, iw, t, a, 0.01, I[k], I[k + 1], 1.0)
    N = len(p)
    lam_a2 = 0.01 * a2
    # planar [V0, V1] -> interleaved (vertex-major) dofs, vertices in RCM order
    r = np.concatenate([t[:, 0], t[:, 1], t[:, 2], t[:, 1], t[:, 2], t[:, 0]])
    c = np.concatenate([t[:, 1], t[:, 2], t[:, 0], t[:, 0], t[:, 1], t[:, 2]])
    G = sp.csr_matrix((np.ones(len(r)), (r, c)), shape=(N, N))
    order = reverse_cuthill_mckee(G.tocsr(), symmetric_mode=True)  # new -> old
    dof = np.empty(2 * N, dtype=np.int64)
    dof[0::2] = order
    dof[1::2] = order + N
    # boundary vertices (on an edge of one triangle), in the RCM order: the
    # omb=X option's rows
    ed = np.sort(np.concatenate([t[:, [0, 1]], t[:, [1, 2]], t[:, [2, 0]]]), axis=1)
    u, cnt = np.unique(ed, axis=0, return_counts=True)
    bnd = np.zeros(N, dtype=bool)
    bnd[u[cnt == 1].ravel()] = True
    system.boundary = bnd[order]
    A = sp.csr_matrix(A)[dof][:, dof].tocsr()
    a2m = sp.csr_matrix(lam_a2)[dof][:, dof].tocsr()
    f = f[dof]
    e = e[order]  # (N, 2, 3)
    return A, a2m, f, e, N


def block_diag_inv(A, bs):
    n = A.shape[0] // bs
    D = np.zeros((n, bs, bs))
    Acoo = A.tocoo()
    m = (Acoo.row // bs) == (Acoo.col // bs)
    D[Acoo.row[m] // bs, Acoo.row[m] % bs, Acoo.col[m] % bs] += Acoo.data[m]
    return D, np.linalg.inv(D)


def bsr_apply(Dinv, v, bs):
    return np.einsum("nij,nj->ni", Dinv, v.reshape(-1, bs)).ravel()


def block_graph(A, bs):
    n = A.shape[0] // bs
    Acoo = A.tocoo()
    Bg = sp.csr_matrix((np.abs(Acoo.data), (Acoo.row // bs, Acoo.col // bs)), shape=(n, n))
    Bg.sum_duplicates()
    return Bg


def aggregate(G, amax=0):
    """The library's greedy aggregation (mof_amg_host.cpp aggregate) on CSR
    adjacency with self loops. amax > 0 (design study): a root takes at most
    amax - 1 of its free neighbours (smaller aggregates, more coarse nodes)."""
    n = G.shape[0]
    ptr, col = G.indptr, G.indices
    agg = -np.ones(n, dtype=np.int64)
    na = 0
    for i in range(n):
        nb = col[ptr[i]:ptr[i + 1]]
        if amax > 0:
            if agg[i] >= 0:
                continue
            free = nb[(agg[nb] < 0) & (nb != i)]
            if len(free) < amax - 1:
                continue
            agg[i] = na
            agg[free[:amax - 1]] = na
            na += 1
            continue
        if (agg[nb] < 0).all():
            agg[nb] = na
            na += 1
    for i in range(n):
        if agg[i] >= 0:
            continue
        nb = agg[col[ptr[i]:ptr[i + 1]]]
        nb = nb[nb >= 0]
        if len(nb) == 0:
            agg[i] = na
            na += 1
            continue
        vals, cnt = np.unique(nb, return_counts=True)
        agg[i] = vals[np.argmax(cnt)]
    return agg, na


def strength_graph(A, bs, theta):
    Acoo = A.tocoo()
    n = A.shape[0] // bs
    F = sp.csr_matrix((Acoo.data ** 2, (Acoo.row // bs, Acoo.col // bs)), shape=(n, n))
    F.sum_duplicates()
    F.data = np.sqrt(F.data)
    d = F.diagonal()
    Fc = F.tocoo()
    keep = (Fc.row == Fc.col) | (Fc.data >= theta * np.sqrt(d[Fc.row] * d[Fc.col]))
    return sp.csr_matrix((np.ones(keep.sum()), (Fc.row[keep], Fc.col[keep])), shape=(n, n))


def sign_graph(A, bs):
    """Couplings whose 2x2 block has a negative trace (the cotangent weight's
    sign in lambda*a2: an obtuse triangle's opposite edge couples positively)."""
    Acoo = A.tocoo()
    n = A.shape[0] // bs
    diag_entry = (Acoo.row % bs) == (Acoo.col % bs)
    T = sp.csr_matrix((Acoo.data * diag_entry, (Acoo.row // bs, Acoo.col // bs)), shape=(n, n))
    T.sum_duplicates()
    Tc = T.tocoo()
    keep = (Tc.row == Tc.col) | (Tc.data < 0)
    return sp.csr_matrix((np.ones(keep.sum()), (Tc.row[keep], Tc.col[keep])), shape=(n, n))


def tentative(agg, na, Bnull, bs):
    """Per aggregate QR of the stacked near-null space (MGS twice, dead
    columns dropped) -> P (n*bs x 3*na), coarse near-null (na, 3, 3)."""
    n = len(agg)
    order = np.argsort(agg, kind="stable")
    bounds = np.searchsorted(agg[order], np.arange(na + 1))
    rows, cols, vals = [], [], []
    Bc = np.zeros((na, 3, 3))
    for I in range(na):
        mem = order[bounds[I]:bounds[I + 1]]
        Bm = Bnull[mem].reshape(-1, 3)
        Q = Bm.copy()
        R = np.zeros((3, 3))
        cmax = np.sqrt((Bm ** 2).sum(0)).max()
        dead = [False] * 3
        for c in range(3):
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
        for c in range(3):
            if dead[c]:
                continue
            rows.append(dofs)
            cols.append(np.full(len(dofs), 3 * I + c))
            vals.append(Q[:, c])
    P = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(n * bs, 3 * na))
    return P, Bc


class Level:
    pass


def build(A, a2m, e, opts):
    levels = []
    bs = 2
    Bnull = e.reshape(-1, bs, 3)
    Acur = A
    a2cur = a2m
    lvl = 0
    while True:
        L = Level()
        L.A, L.bs = Acur, bs
        L.D, L.Dinv = block_diag_inv(Acur, bs)
        if lvl == 0 and "s0" in opts:  # the GPU's level 0: everything on the stored copy
            L.Aq = quantize(Acur, bs, int(opts["s0"]))
            L.D, L.Dinv = block_diag_inv(L.Aq, bs)
        if opts.get("l1"):
            G = block_graph(Acur, bs)  # |entries| summed per block
            Fr = sp.csr_matrix((Acur.tocoo().data ** 2, (Acur.tocoo().row // bs, Acur.tocoo().col // bs)),
                               shape=G.shape)
            Fr.sum_duplicates()
            Fr.data = np.sqrt(Fr.data)
            off = np.asarray(Fr.sum(1)).ravel() - Fr.diagonal()
            L.Dinv = np.linalg.inv(L.D + off[:, None, None] * np.eye(bs)[None])
            L.om = 1.0
        else:
            L.om = opts.get("om", (0.85, 1.05))[0 if lvl == 0 else 1]
            if lvl == 0 and "omb" in opts:  # per-row damping: boundary rows omb
                om = np.where(system.boundary, opts["omb"], L.om)
                L.om = np.repeat(om, bs)
        if lvl >= 1 and opts.get("galq") and opts.get("q1"):
            # the coarse Galerkin products from the sweeps' stored copy (the
            # operator the level's residual applies), not the exact one
            L.Aq = quantize(Acur, bs, int(opts["q1"]))
        levels.append(L)
        n = Acur.shape[0] // bs
        if n * bs <= 128 or n * 3 <= 128:
            L.coarse = np.linalg.inv(Acur.toarray() + np.diag((np.abs(Acur).sum(1).A1 == 0) * 1.0))
            break
        G = block_graph(Acur, bs)
        if lvl == 0 and "theta" in opts:
            G = strength_graph(Acur, bs, opts["theta"])
        if lvl == 0 and "theta2" in opts:  # strength from lambda*a2 (per mesh)
            G = strength_graph(a2m, bs, opts["theta2"])
        if lvl == 0 and "sgn" in opts:  # negative couplings of lambda*a2 only
            G = sign_graph(a2m, bs)
        if lvl >= 1 and "theta1" in opts:  # coarse levels: strong couplings only
            G = strength_graph(Acur, bs, opts["theta1"])
        if lvl == 1 and "theta1only" in opts:  # level 1 only
            G = strength_graph(Acur, bs, opts["theta1only"])
        if lvl == 1 and "theta1a2" in opts:  # level 1, strength from P^T (lambda a2) P (per mesh)
            G = strength_graph(a2cur, bs, opts["theta1a2"])
        G = (G + sp.eye(G.shape[0])).tocsr()
        G.sort_indices()
        agg, na = aggregate(G, int(opts.get("amax", 0)) if lvl == 0 else int(opts.get("amax1", 0)))
        if na >= n:
            L.coarse = np.linalg.inv(Acur.toarray())
            break
        P, Bc = tentative(agg, na, Bnull, bs)
        if lvl >= 1 and ("sa1" in opts or "sa1a2" in opts) and (lvl == 1 or "sa1only" not in opts):
            # sa1: with the level's own A (per timestep); sa1a2: with the
            # Galerkin image of lambda*a2 (per mesh)
            Asm = Acur if "sa1" in opts else a2cur
            _, Dinv_s = block_diag_inv(Asm, bs)
            Dbsr = sp.block_diag([Dinv_s[i] for i in range(n)], format="csr")
            P = (P - opts.get("sa1", opts.get("sa1a2")) * (Dbsr @ (Asm @ P))).tocsr()
        if lvl == 0 and ("sa" in opts or "sa2" in opts):
            Asm = Acur if "sa" in opts else a2m
            w = opts.get("sa", opts.get("sa2"))
            _, Dinv_s = block_diag_inv(Asm, bs)
            Dbsr = sp.block_diag([Dinv_s[i] for i in range(n)], format="csr")
            P = (P - w * (Dbsr @ (Asm @ P))).tocsr()
            if "trunc" in opts:  # drop the 2x3 blocks of P below trunc x the row's largest
                Pb = P.tobsr(blocksize=(2, 3))
                nb = np.sqrt((Pb.data ** 2).sum(axis=(1, 2)))
                rowmax = np.zeros(Pb.shape[0] // 2)
                rows = np.repeat(np.arange(Pb.shape[0] // 2), np.diff(Pb.indptr))
                np.maximum.at(rowmax, rows, nb)
                keep = nb >= opts["trunc"] * rowmax[rows]
                Pb.data[~keep] = 0
                P = Pb.tocsr()
                P.eliminate_zeros()
        Pb = P.tobsr(blocksize=(bs, 3))
        L.p_blocks = Pb.nnz / (bs * 3) / (P.shape[0] / bs)
        L.P = P
        Ab = Acur.tobsr(blocksize=(bs, bs))
        # Galerkin terms: sum over fine blocks (i, j) of |P_i| |P_j| (blocks)
        pc = np.diff(Pb.indptr)
        rows = np.repeat(np.arange(Ab.shape[0] // bs), np.diff(Ab.indptr))
        L.gal_terms = int((pc[rows] * pc[Ab.indices]).sum())
        if opts.get("f32gal"):  # the GPU's fp32 Galerkin product: fp32 operands, fp32 sums
            P32 = P.astype(np.float32)
            Ac = (P32.T @ (L.Aq if hasattr(L, "Aq") else Acur).astype(np.float32) @ P32).astype(np.float64).tocsr()
        else:
            Ac = (P.T @ (L.Aq if hasattr(L, "Aq") else Acur) @ P).tocsr()
        a2cur = (P.T @ (a2m if lvl == 0 else a2cur) @ P).tocsr()
        dead = np.abs(Ac).sum(1).A1 == 0
        Ac = (Ac + sp.diags(dead * 1.0)).tocsr()
        Acur, bs, Bnull = Ac, 3, Bc
        lvl += 1
    return levels


def quantize(A, bs, fmt):
    """The sweep copy of a coarse operator in a storage format (emulated)."""
    Ab = A.tobsr(blocksize=(bs, bs)).copy()
    d = Ab.data.astype(np.float64)
    if fmt == 1:  # bf16 (round to nearest even on the fp32 bits)
        u = d.astype(np.float32).view(np.uint32).astype(np.uint64)
        u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
        d = u.astype(np.uint32).view(np.float32).astype(np.float64)
    elif fmt == 2:  # int8 with one scale per block
        m = np.abs(d).max(axis=(1, 2), keepdims=True)
        sc = np.where(m > 0, m / 127.0, 1.0)
        d = np.round(d / sc) * sc
    elif fmt == 3:  # fp8 e4m3 with one scale per block (3 mantissa bits)
        m = np.abs(d).max(axis=(1, 2), keepdims=True)
        sc = np.where(m > 0, m / 448.0, 1.0)
        v = d / sc
        ex = np.floor(np.log2(np.maximum(np.abs(v), 2.0 ** -6)))
        q = 2.0 ** (ex - 3)
        d = np.round(v / q) * q * sc
    elif fmt == 5:  # symmetric diagonal scaling, int8 with one global scale
        s = np.sqrt(np.abs(A.diagonal()))
        S = sp.diags(1.0 / s) @ A @ sp.diags(1.0 / s)
        S = S.tocsr()
        S.data = np.clip(np.round(S.data * 127.0), -127, 127) / 127.0
        return (sp.diags(s) @ S @ sp.diags(s)).tocsr()
    elif fmt in (6, 7):  # 6: diagonal blocks bf16, off-diagonal blocks of the equilibrated
        # Q = T^-1 D^-1/2 A D^-1/2 T^-1 (t_i^2 = the row's largest |off-diagonal|, so
        # |Q| <= 1) as int8 with the one scale 1/127; 7: the same with fp8 e4m3 codes
        s = np.sqrt(np.abs(A.diagonal()))
        S = (sp.diags(1.0 / s) @ A @ sp.diags(1.0 / s)).tocoo()
        same = (S.row // bs) == (S.col // bs)
        m = np.zeros(A.shape[0])
        np.maximum.at(m, S.row[~same], np.abs(S.data[~same]))
        t = np.sqrt(np.where(m > 0, m, 1.0))
        d = S.data.copy()
        qv = d[~same] / (t[S.row[~same]] * t[S.col[~same]])
        if fmt == 6:
            qv = np.clip(np.round(qv * 127.0), -127, 127) / 127.0
        else:
            ex = np.floor(np.log2(np.maximum(np.abs(qv), 2.0 ** -6)))
            q = 2.0 ** (ex - 3)
            qv = np.round(qv / q) * q
        d[~same] = qv * t[S.row[~same]] * t[S.col[~same]]
        u = d[same].astype(np.float32).view(np.uint32).astype(np.uint64)
        u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
        d[same] = u.astype(np.uint32).view(np.float32).astype(np.float64)
        Sq = sp.csr_matrix((d, (S.row, S.col)), shape=A.shape)
        return (sp.diags(s) @ Sq @ sp.diags(s)).tocsr()
    elif fmt == 4:  # int8 with one scale per row block (row of blocks)
        rows = np.repeat(np.arange(Ab.shape[0] // bs), np.diff(Ab.indptr))
        m = np.zeros(Ab.shape[0] // bs)
        np.maximum.at(m, rows, np.abs(d).max(axis=(1, 2)))
        sc = np.where(m > 0, m / 127.0, 1.0)[rows][:, None, None]
        d = np.round(d / sc) * sc
    Ab.data = d
    return Ab.tocsr()


def vcycle(levels, l, b, opts):
    L = levels[l]
    if hasattr(L, "coarse"):
        return L.coarse @ b
    if l == int(opts.get("exact", -1)):  # an exact solve from this level down (two-grid bound)
        if not hasattr(L, "lu"):
            L.lu = sla_sparse.splu(L.A.tocsc())
        return L.lu.solve(b)
    Aw = L.A
    qf = opts.get("q1") if l >= 1 else opts.get("q0")
    if hasattr(L, "Aq"):
        Aw = L.Aq
    elif qf:
        if not hasattr(L, "Aq"):
            L.Aq = quantize(L.A, L.bs, int(qf))
        Aw = L.Aq
    nu = int(opts.get("nu1", 1)) if l >= 1 else int(opts.get("nu0", 1))  # sweeps per side
    if l == 0 and (opts.get("cheb") or opts.get("chebpost")):
        return _cheb_vcycle(levels, L, Aw, b, opts)
    if l == 0 and opts.get("mcgs"):
        return _mcgs_vcycle(levels, L, Aw, b, opts)
    if l == 0 and opts.get("bsw"):
        return _bsw_vcycle(levels, L, Aw, b, opts)
    x = L.om * bsr_apply(L.Dinv, b, L.bs)
    for _ in range(nu - 1):
        x = x + L.om * bsr_apply(L.Dinv, b - Aw @ x, L.bs)
    cyc = 2 if (opts.get("w2") and l == 1) else 1
    for _ in range(cyc):
        r = b - Aw @ x
        if opts.get("kcyc") and l == 1:  # K-cycle: the level-2 problem by kcyc FCG steps
            y = _kcycle(levels, l + 1, L.P.T @ r, opts, int(opts["kcyc"]))
        else:
            y = vcycle(levels, l + 1, L.P.T @ r, opts)
        x = x + L.P @ y
        for _ in range(nu):
            x = x + L.om * bsr_apply(L.Dinv, b - Aw @ x, L.bs)
    return x


def _kcycle(levels, l, b, opts, steps):
    """Notay's K-cycle at level l: `steps` flexible-CG iterations on the
    level's operator (the copy its cycle applies), preconditioned by the
    level's own cycle, from x = 0."""
    L = levels[l]
    Aw = getattr(L, "Aq", L.A)
    x = np.zeros_like(b)
    r = b.copy()
    d_prev = q_prev = None
    for _ in range(steps):
        z = vcycle(levels, l, r, opts)
        d = z
        if d_prev is not None:  # A-orthogonal to the previous direction
            d = z - (z @ q_prev) / (d_prev @ q_prev) * d_prev
        q = Aw @ d
        a = (d @ r) / (d @ q)
        x = x + a * d
        r = r - a * q
        d_prev, q_prev = d, q
    return x


def _cheb(L, Aw, b, x, deg, ratio):
    """Degree-deg Chebyshev smoothing of Aw x = b in D^-1 Aw over
    [lmax / ratio, lmax] (lmax: 1.1 x a 20-step power estimate, cached)."""
    if not hasattr(L, "lmax"):
        v = np.random.default_rng(0).standard_normal(Aw.shape[0])
        for _ in range(20):
            v = bsr_apply(L.Dinv, Aw @ v, L.bs)
            lm = np.linalg.norm(v)
            v /= lm
        L.lmax = 1.1 * lm
    hi, lo = L.lmax, L.lmax / ratio
    theta, delta = 0.5 * (hi + lo), 0.5 * (hi - lo)
    sigma = theta / delta
    rho = 1.0 / sigma
    r = bsr_apply(L.Dinv, b - Aw @ x if x is not None else b, L.bs)
    x = np.zeros_like(b) if x is None else x
    d = r / theta
    for k in range(deg):
        x = x + d
        if k == deg - 1:
            break
        r = r - bsr_apply(L.Dinv, Aw @ d, L.bs)
        rho1 = 1.0 / (2.0 * sigma - rho)
        d = rho1 * rho * d + (2.0 * rho1 / delta) * r
        rho = rho1
    return x


def _cheb_vcycle(levels, L, Aw, b, opts):
    """Level 0 with Chebyshev smoothing: cheb=k both sides (pre from x = 0),
    chebpost=k the post side only (pre stays om D^-1 b); cr = the ratio."""
    ratio = float(opts.get("cr", 30.0))
    kpre = int(opts.get("cheb", 0))
    kpost = int(opts.get("chebpost", 0)) or kpre
    x = _cheb(L, Aw, b, None, kpre, ratio) if kpre else L.om * bsr_apply(L.Dinv, b, L.bs)
    r = b - Aw @ x
    y = vcycle(levels, 1, L.P.T @ r, opts)
    x = x + L.P @ y
    return _cheb(L, Aw, b, x, kpost, ratio)


def _colors(L):
    """Greedy colouring of the level's block graph (node order)."""
    if not hasattr(L, "color"):
        G = block_graph(L.A, L.bs).tocsr()
        n = G.shape[0]
        col = -np.ones(n, dtype=np.int64)
        for i in range(n):
            used = set(col[G.indices[G.indptr[i]:G.indptr[i + 1]]].tolist())
            c = 0
            while c in used:
                c += 1
            col[i] = c
        L.color = col
        L.ncolor = int(col.max()) + 1
    return L.color, L.ncolor


def _mcgs(L, Aw, b, x, order, om):
    """Block Gauss-Seidel by colour (the colours in `order`), damped by om."""
    col, _ = _colors(L)
    x = x.copy()
    for c in order:
        rows = np.flatnonzero(col == c)
        dof = (rows[:, None] * L.bs + np.arange(L.bs)[None]).ravel()
        r = (b[dof] - Aw[dof] @ x).reshape(-1, L.bs)
        x[dof] += om * np.einsum("nij,nj->ni", L.Dinv[rows], r).ravel()
    return x


def _mcgs_vcycle(levels, L, Aw, b, opts):
    """Level 0 with multicolour block Gauss-Seidel: mcgs=1 forward before,
    backward after (symmetric); om damping from gsom= (default 1)."""
    _, nc = _colors(L)
    om = float(opts.get("gsom", 1.0))
    x = _mcgs(L, Aw, b, np.zeros_like(b), range(nc), om)
    r = b - Aw @ x
    y = vcycle(levels, 1, L.P.T @ r, opts)
    x = x + L.P @ y
    return _mcgs(L, Aw, b, x, range(nc - 1, -1, -1), om)


def _bsw(L, Aw, b, x, k, om, ring):
    """k block-Jacobi sweeps (damping om) on the boundary rows and their
    `ring`-neighbourhood only."""
    if not hasattr(L, "bdof"):
        rows = np.flatnonzero(system.boundary)
        G = block_graph(L.A, L.bs).tocsr()
        sel = np.zeros(G.shape[0], dtype=bool)
        sel[rows] = True
        for _ in range(ring):
            sel = sel | (G @ sel.astype(np.float64) > 0)
        L.brows = np.flatnonzero(sel)
        L.bdof = (L.brows[:, None] * L.bs + np.arange(L.bs)[None]).ravel()
        L.Ab = Aw[L.bdof].tocsr()
    x = x.copy()
    for _ in range(k):
        r = (b[L.bdof] - L.Ab @ x).reshape(-1, L.bs)
        x[L.bdof] += om * np.einsum("nij,nj->ni", L.Dinv[L.brows], r).ravel()
    return x


def _bsw_vcycle(levels, L, Aw, b, opts):
    """Level 0 as the library's, plus bsw=K sweeps on the boundary rows
    (bring=R neighbour rings, bom=X damping) after the pre- and before the
    post-smoothing (symmetric)."""
    k, ring, om = int(opts["bsw"]), int(opts.get("bring", 1)), float(opts.get("bom", 0.7))
    x = L.om * bsr_apply(L.Dinv, b, L.bs)
    x = _bsw(L, Aw, b, x, k, om, ring)
    r = b - Aw @ x
    y = vcycle(levels, 1, L.P.T @ r, opts)
    x = x + L.P @ y
    x = _bsw(L, Aw, b, x, k, om, ring)
    return x + L.om * bsr_apply(L.Dinv, b - Aw @ x, L.bs)


def pcg(A, f, M, tol=1e-4, maxit=2000, flexible=False):
    """PCG; flexible: Polak-Ribiere beta (flexible CG, for a nonlinear
    preconditioner such as the K-cycle)."""
    x = np.zeros_like(f)
    r = f.copy()
    z = M(r)
    p = z.copy()
    rz = r @ z
    nf = np.linalg.norm(f)
    for it in range(1, maxit + 1):
        q = A @ p
        a = rz / (p @ q)
        x += a * p
        r_old = r.copy() if flexible else None
        r -= a * q
        if np.linalg.norm(r) <= tol * nf:
            pcg.rho = (np.linalg.norm(r) / nf) ** (1.0 / it)
            return it
        z = M(r)
        rz2 = r @ z
        beta = (z @ (r - r_old)) / rz if flexible else rz2 / rz
        p = z + beta * p
        rz = rz2
    return maxit


def parse(args):
    opts = {}
    for a in args:
        if a == "base":
            continue
        if a in ("l1", "w2"):
            opts[a] = True
        elif a.startswith("om="):
            opts["om"] = tuple(float(v) for v in a[3:].split(","))
        else:
            k, v = a.split("=")
            opts[k] = float(v)
    return opts


def main():
    cfg = sys.argv[1]
    A, a2m, f, e, N = system(cfg)
    for spec in sys.argv[2:] or ["base"]:
        opts = parse(spec.split("+"))
        levels = build(A, a2m, e, opts)
        sizes = [lv.A.shape[0] // lv.bs for lv in levels]
        nnz = sum(lv.A.nnz for lv in levels)
        its = pcg(A, f, lambda r: vcycle(levels, 0, r, opts), flexible=bool(opts.get("kcyc")))
        blk = [round(lv.A.nnz / lv.bs ** 2 / (lv.A.shape[0] / lv.bs), 1) for lv in levels]
        pb = [round(lv.p_blocks, 2) for lv in levels if hasattr(lv, "p_blocks")]
        gal = [getattr(lv, "gal_terms", 0) for lv in levels]
        print("%s %-24s its(1e-4) %4d  rho %.4f  levels %s  op complexity %.2f  blocks/row %s  P blocks/row %s  "
              "Galerkin terms %s" % (cfg, spec, its, pcg.rho, sizes, nnz / A.nnz, blk, pb, gal), flush=True)


if __name__ == "__main__":
    main()
