"""Error control of the mixed-precision refinement (design tool, CPU).

Emulates the library's mixed solve on one timestep's oracle system: inner
PCG in fp32 (fp32 operator and vectors, fp64 dot products) preconditioned by
the prototype V-cycle, fp64 refinement x += d, r = f - A x (fp64), the
first inner solve to 1e-4 and later ones to the adaptive tolerance
clamp(0.3 rtol |f| / |r|, 1e-4, 0.5). After every refinement step it prints
the true error max|x - x*| (x* = spsolve), the residual and the error
estimate the library's stop rule uses,

    E_{k+1} = max|d_k| * |r_{k+1}|_2 / |r_k|_2,

the last correction scaled by the step's residual reduction: from the second
step on, r_k lies in the slow modes the next residual also lies in, so the
gain |d_k| / |r_k| of A^-1 along r_k is the gain along r_{k+1}.

    python tools/error_control_study.py CONFIG [spec] [timesteps...]

The oracle is test infrastructure; this script is a design tool, never part
of the product path.
"""
import os
import sys

import numpy as np
import scipy.sparse.linalg as sla

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as ap  # noqa: E402


def pcg32(A32, f, M, tol, maxit=3000):
    f = f.astype(np.float32)
    x = np.zeros_like(f)
    r = f.copy()
    z = M(r.astype(np.float64)).astype(np.float32)
    p = z.copy()
    rz = float(r.astype(np.float64) @ z.astype(np.float64))
    nf = float(np.linalg.norm(f.astype(np.float64)))
    for it in range(1, maxit + 1):
        q = (A32 @ p).astype(np.float32)
        a = rz / float(p.astype(np.float64) @ q.astype(np.float64))
        x = (x + np.float32(a) * p).astype(np.float32)
        r = (r - np.float32(a) * q).astype(np.float32)
        if np.linalg.norm(r.astype(np.float64)) <= tol * nf:
            return x.astype(np.float64), it
        z = M(r.astype(np.float64)).astype(np.float32)
        rz2 = float(r.astype(np.float64) @ z.astype(np.float64))
        p = (z + np.float32(rz2 / rz) * p).astype(np.float32)
        rz = rz2
    return x.astype(np.float64), maxit


def main():
    cfg = sys.argv[1]
    spec = sys.argv[2] if len(sys.argv) > 2 else "sa2=0.66+om=0.7,1.05"
    ks = [int(v) for v in sys.argv[3:]] or [0]
    rtol, inner = 1e-8, 1e-4
    for k in ks:
        A, a2m, f, e, N = ap.system(cfg, k)
        xs = sla.spsolve(A.tocsc(), f)
        opts = ap.parse(spec.split("+"))
        levels = ap.build(A, a2m, e, opts)
        M = lambda r: ap.vcycle(levels, 0, r, opts)  # noqa: E731
        A32 = A.astype(np.float32)
        nf = np.linalg.norm(f)
        x = np.zeros_like(f)
        r = f.copy()
        xmax = np.abs(xs).max()
        print("%s k=%d N=%d max|x*| %.3e" % (cfg, k, N, xmax))
        tau = float(os.environ.get("TAU", "1e-7"))
        est = None
        tot = 0
        for o in range(8):
            rel = np.linalg.norm(r) / nf
            need = 0.3 * rtol / rel
            if est is not None and os.environ.get("ERRTOL", "1") == "1":
                need = min(need, float(os.environ.get("NEEDF", "0.3")) * tau * np.abs(x).max() / (2 * est))
            t = inner if o == 0 else max(inner, min(0.5, need))
            d, its = pcg32(A32, r, M, t)
            tot += its
            x = x + d
            rn = f - A @ x
            est = np.abs(d).max() * np.linalg.norm(rn) / np.linalg.norm(r)
            err = np.abs(x - xs).max()
            print("  step %d: %4d its  rel res %.2e  err %.2e (rel %.2e)  est %.2e  est/err %.2f"
                  % (o, its, np.linalg.norm(rn) / nf, err, err / xmax, est, est / err), flush=True)
            r = rn
            if np.linalg.norm(r) / nf <= rtol and 2 * est <= tau * np.abs(x).max():
                break
        print("  total %d its, %d steps" % (tot, o + 1))


if __name__ == "__main__":
    main()
