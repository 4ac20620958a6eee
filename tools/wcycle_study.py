"""Why the level-1 W-cycle breaks PCG down on the open S1-like patches
(round-5 verdict, weak #1 / item 2): a CPU study of the library's cycle.

    python tools/wcycle_study.py [CONFIG] [variant ...]

Builds one timestep's system (oracle, RCM order; tools/amg_proto.py) and the
library's hierarchy for an open patch -- level 0 and level 1 prolongators
smoothed with the (Galerkin image of) a2 (w = 0.66), damping 0.7 fine / 1.05
coarse, the level-0 sweeps and residual on a bf16 copy, the coarse ones on
the int8 + scale copy, every Galerkin product from the unquantised operator
(mof_amg.hip amg_build / amg_setup_batch) -- and reports, for the V-cycle
and the level-1 W-cycle (S C S C S):

  * symmetry of the preconditioner M: max |u.Mv - v.Mu| / (|u| |Mv|);
  * the extreme eigenvalues of M A (Lanczos on A^1/2 M A^1/2 through the
    A-inner product): M is SPD iff lambda_min(M A) > 0;
  * the spectrum of the cycle below level 1 as a solver for level 2's
    operator, B2 A2: the W-cycle's coarse correction C = I - P B2 P^T A1 has
    eigenvalues in (-1, 1] only if lambda(B2 A2) lies in (0, 2);
  * the PCG iterations to 1e-4 and the smallest p.q / r.z ratios seen.

Variants: "v" (library V-cycle), "w" (W-cycle), "wq" (W with the coarse
residual on the same copy as the Galerkin product, i.e. q1 off), "w_om1=X"
(W with coarse damping X). A design tool, never part of the product path.
"""
import os
import sys

import numpy as np
import scipy.sparse.linalg as sla

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as P  # noqa: E402

BASE = {"om": (0.7, 1.05), "sa2": 0.66, "sa1a2": 0.66, "sa1only": 1.0, "q0": 1.0, "q1": 2.0}


def opts_for(spec):
    o = dict(BASE)
    for part in spec.split("+"):
        if part == "v":
            continue
        if part == "w":
            o["w2"] = True
        elif part == "wq":
            o["w2"] = True
            o.pop("q1")
        elif part.startswith("om1="):
            o["om"] = (o["om"][0], float(part[4:]))
        elif part.startswith("om0="):
            o["om"] = (float(part[4:]), o["om"][1])
        else:
            k, v = part.split("=")
            o[k] = float(v)
    return o


def lanczos_extremes(A, M, n, steps=120, seed=0):
    """Extreme eigenvalues of M A (A, M symmetric, A SPD) by Lanczos on M A
    in the A-inner product (the PCG's own Krylov space)."""
    rng = np.random.default_rng(seed)
    v = rng.standard_normal(n)
    v /= np.sqrt(v @ (A @ v))
    vs, al, be = [v], [], []
    w_prev = np.zeros(n)
    b_prev = 0.0
    for j in range(steps):
        w = M(A @ vs[-1])
        a = w @ (A @ vs[-1])
        w = w - a * vs[-1] - b_prev * w_prev
        for u in vs:  # full reorthogonalisation (A-inner product)
            w -= (w @ (A @ u)) * u
        b = np.sqrt(max(w @ (A @ w), 0.0))
        al.append(a)
        if b < 1e-14 or j == steps - 1:
            break
        be.append(b)
        w_prev, b_prev = vs[-1], b
        vs.append(w / b)
    T = np.diag(al) + np.diag(be[:len(al) - 1], 1) + np.diag(be[:len(al) - 1], -1)
    ev = np.linalg.eigvalsh(T)
    return ev[0], ev[-1]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "S1m"
    specs = sys.argv[2:] or ["v", "w"]
    A, a2m, f, e, N = P.system(cfg)
    n = A.shape[0]
    print("%s: %d dofs, nnz %d" % (cfg, n, A.nnz), flush=True)
    for spec in specs:
        o = opts_for(spec)
        levels = P.build(A, a2m, e, o)
        sizes = [lv.A.shape[0] // lv.bs for lv in levels]

        def M(r, o=o, levels=levels):
            return P.vcycle(levels, 0, r, o)

        rng = np.random.default_rng(1)
        asym = 0.0
        for _ in range(3):
            u, v = rng.standard_normal(n), rng.standard_normal(n)
            Mv, Mu = M(v), M(u)
            asym = max(asym, abs(u @ Mv - v @ Mu) / (np.linalg.norm(u) * np.linalg.norm(Mv)))
        lo, hi = lanczos_extremes(A, M, n)
        # the cycle below level 1 as a solver of level 2's operator (the
        # operator the level-1 coarse correction inverts)
        b2 = ""
        if len(levels) > 2 and not hasattr(levels[2], "coarse"):
            A2 = levels[2].A
            n2 = A2.shape[0]
            live = np.abs(A2).sum(1).A1 > 0
            lo2, hi2 = lanczos_extremes(A2, lambda r: P.vcycle(levels, 2, r, o), n2, steps=80)
            b2 = "  B2 A2 in [%.4f, %.4f] (%d dofs, %d live)" % (lo2, hi2, n2, live.sum())
        # dense: the level-2 cycle B2 against level 2's Galerkin operator A2
        # and against the operator level 1's coarse correction actually
        # inverts, P1^T A1q P1 (A1q: the level-1 residual's stored copy)
        if len(levels) > 2 and not hasattr(levels[2], "coarse") and levels[2].A.shape[0] <= 6000:
            n2 = levels[2].A.shape[0]
            B2 = np.column_stack([P.vcycle(levels, 2, col, o) for col in np.eye(n2)])
            B2 = 0.5 * (B2 + B2.T)
            A1w = getattr(levels[1], "Aq", levels[1].A)
            A2e = (levels[1].P.T @ A1w @ levels[1].P).toarray()
            A2e += np.diag((np.abs(A2e).sum(1) == 0) * 1.0)
            import scipy.linalg as sl
            Lb = np.linalg.cholesky(B2)
            for nm, Am in (("A2", levels[2].A.toarray()), ("P1'A1q P1", A2e)):
                ev = np.linalg.eigvalsh(Lb.T @ Am @ Lb)
                print("   eig(B2 %s) in [%.4f, %.4f]  (lambda_min(%s) %.3e)" %
                      (nm, ev[0], ev[-1], nm, np.linalg.eigvalsh(Am)[0]), flush=True)
        # smallest eigenvalues of the coarse operators (the Galerkin products
        # the cycle inverts): dense below 4k dofs, else shift-invert near 0
        lmin = []
        for lv in levels[1:]:
            Al = lv.A
            if Al.shape[0] <= 4000:
                ev = np.linalg.eigvalsh(Al.toarray())
                lmin.append("%.2e/%.2e" % (ev[0], ev[-1]))
            else:
                ev = sla.eigsh(Al.tocsc(), k=2, sigma=0.0, which="LM", return_eigenvectors=False)
                lmin.append("%.2e" % ev.min())
        print("   coarse lambda_min[/max]: %s" % " ".join(lmin), flush=True)
        its = P.pcg(A, f, M, flexible=bool(o.get("kcyc")))
        its_tight = P.pcg(A, f, M, tol=1e-8, flexible=bool(o.get("kcyc")))
        print("%-14s levels %s  asym %.2e  M A in [%.4f, %.4f]%s  its(1e-4) %d  its(1e-8) %d" %
              (spec, sizes, asym, lo, hi, b2, its, its_tight), flush=True)


if __name__ == "__main__":
    main()
