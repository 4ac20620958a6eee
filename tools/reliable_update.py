"""Restarted iterative refinement vs reliable updates, on the CPU (design tool).

    python tools/reliable_update.py CONFIG [K] [delta ...]

The library's mixed solve restarts the inner fp32 PCG after each fp64
residual refresh (refinement steps: inner to 1e-4 of the step's residual,
later steps to 0.3 rtol |f| / |r| clamped to [1e-4, 0.5], until
|f - A x| <= 1e-8 |f|). A reliable update (the mixed-precision Krylov
scheme of lattice QCD solvers) refreshes the residual the same way -- fold
the fp32 iterate into x64, r = f - A64 x64 in fp64 -- but keeps the search
direction p and q = A32 p and continues the recurrence (beta from the new
r.z over the old one), so the Krylov space is not thrown away.

Emulates the GPU's arithmetic: A32 = fl32(A), fp32 vectors, fp64 dot
products, the multigrid output z rounded to bf16 (regular meshes), the
V(1,1) cycle of tools/amg_proto.py. For K timesteps of the bench signal,
prints PCG iterations and residual refreshes per timestep for the restarted
scheme and for reliable updates at each delta (refresh when the recursive
|r| falls below delta times |r| at the last refresh).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import warm_start as ws  # noqa: E402
import amg_proto as ap  # noqa: E402


def bf16(v):
    u = np.ascontiguousarray(v, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32)


class Inner:
    """fp32 operator and preconditioner of one system."""

    def __init__(self, A, M):
        self.A64 = A
        self.A32 = A.astype(np.float32)
        self.M = M

    def prec(self, r32):
        return bf16(self.M(r32.astype(np.float64)).astype(np.float32))


def restarted(S, f, rtol=1e-8, inner=1e-4, maxit=500):
    nf = np.linalg.norm(f)
    x64 = np.zeros_like(f)
    its = steps = 0
    for o in range(10):
        r64 = f - S.A64 @ x64
        nr = np.linalg.norm(r64)
        if nr <= rtol * nf:
            break
        tol = inner if o == 0 else min(0.5, max(inner, 0.3 * rtol * nf / nr))
        r = r64.astype(np.float32)
        x = np.zeros_like(r)
        z = S.prec(r)
        p = z.copy()
        rz = float(r.astype(np.float64) @ z.astype(np.float64))
        nb = float(np.linalg.norm(r.astype(np.float64)))
        for it in range(maxit):
            q = (S.A32 @ p).astype(np.float32)
            a = rz / float(p.astype(np.float64) @ q.astype(np.float64))
            x = (x + np.float32(a) * p).astype(np.float32)
            r = (r - np.float32(a) * q).astype(np.float32)
            its += 1
            if np.linalg.norm(r.astype(np.float64)) <= tol * nb:
                break
            z = S.prec(r)
            rz2 = float(r.astype(np.float64) @ z.astype(np.float64))
            p = (z + np.float32(rz2 / rz) * p).astype(np.float32)
            rz = rz2
        x64 += x.astype(np.float64)
        steps += 1
    return x64, its, steps


def reliable(S, f, delta, rtol=1e-8, maxit=500):
    nf = np.linalg.norm(f)
    x64 = np.zeros_like(f)
    r = f.astype(np.float32)
    x = np.zeros_like(r)
    z = S.prec(r)
    p = z.copy()
    q = (S.A32 @ p).astype(np.float32)
    rz = float(r.astype(np.float64) @ z.astype(np.float64))
    rmax = nf  # |r| at the last refresh
    its = refreshes = 0
    for it in range(maxit):
        a = rz / float(p.astype(np.float64) @ q.astype(np.float64))
        x = (x + np.float32(a) * p).astype(np.float32)
        r = (r - np.float32(a) * q).astype(np.float32)
        its += 1
        nr = float(np.linalg.norm(r.astype(np.float64)))
        if nr <= delta * rmax or nr <= rtol * nf:
            x64 += x.astype(np.float64)
            x[:] = 0
            r64 = f - S.A64 @ x64
            refreshes += 1
            nr = float(np.linalg.norm(r64))
            if nr <= rtol * nf:
                break
            r = r64.astype(np.float32)
            rmax = nr
        z = S.prec(r)
        rz2 = float(r.astype(np.float64) @ z.astype(np.float64))
        b = np.float32(rz2 / rz)
        p = (z + b * p).astype(np.float32)
        q = ((S.A32 @ z).astype(np.float32) + b * q).astype(np.float32)  # the GPU's q = A z + beta q
        rz = rz2
    return x64, its, refreshes


def main():
    cfg = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    deltas = [float(v) for v in sys.argv[3:]] or [1e-4, 1e-2, 1e-1]
    sysl, a2m, e = ws.systems(cfg, K, 0.3)
    tot = {"restart": [0, 0]}
    for d in deltas:
        tot[d] = [0, 0]
    err = {}
    for k, (A, f) in enumerate(sysl):
        levels = ap.build(A, a2m, e, {})
        S = Inner(A, lambda r, lv=levels: ap.vcycle(lv, 0, r, {}))
        x0, n0, s0 = restarted(S, f)
        tot["restart"][0] += n0
        tot["restart"][1] += s0
        for d in deltas:
            x1, n1, s1 = reliable(S, f, d)
            tot[d][0] += n1
            tot[d][1] += s1
            err[d] = max(err.get(d, 0.0), float(np.abs(x1 - x0).max()))
            rr = np.linalg.norm(f - A @ x1) / np.linalg.norm(f)
            assert rr <= 1e-8, (d, rr)
    for key, (n, s) in tot.items():
        print("%s %-8s PCG its/timestep %.2f  residual refreshes %.2f  max|dV| vs restart %s"
              % (cfg, key, n / K, s / K, "-" if key == "restart" else "%.1e" % err[key]), flush=True)


if __name__ == "__main__":
    main()
