"""Iterative-refinement schedule study (design tool, CPU): PCG iterations of
the inner solves when the first refinement step stops at inner tolerance t1
and later steps at max(1e-4, 0.3 rtol |f| / |r|) (the library's adaptive
rule), against one PCG to rtol. The inner solve here is fp64 (the GPU's is
fp32 with fp64 dots): the study isolates the restart cost -- a later step's
right-hand side is the residual the first solve left, without its easy modes.

    python tools/refine_study.py CONFIG [variant] [t1 ...]
"""
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as ap  # noqa: E402


def pcg_x(A, f, M, tol, maxit=3000):
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
        r -= a * q
        if np.linalg.norm(r) <= tol * nf:
            return x, it
        z = M(r)
        rz2 = r @ z
        p = z + (rz2 / rz) * p
        rz = rz2
    return x, maxit


def main():
    cfg = sys.argv[1]
    spec = sys.argv[2] if len(sys.argv) > 2 else "base"
    t1s = [float(v) for v in sys.argv[3:]] or [1e-4, 1e-5, 1e-6]
    A, a2m, f, e, N = ap.system(cfg)
    opts = ap.parse(spec.split("+"))
    levels = ap.build(A, a2m, e, opts)
    M = lambda r: ap.vcycle(levels, 0, r, opts)  # noqa: E731
    rtol = 1e-8
    _, one = pcg_x(A, f, M, rtol)
    print("%s %s one PCG to 1e-8: %d its" % (cfg, spec, one), flush=True)
    nf = np.linalg.norm(f)
    for t1 in t1s:
        x = np.zeros_like(f)
        steps = []
        for o in range(6):
            r = f - A @ x
            rel = np.linalg.norm(r) / nf
            if rel <= rtol:
                break
            t = t1 if o == 0 else max(1e-4, min(0.5, 0.3 * rtol / rel))
            d, its = pcg_x(A, r, M, t)
            x = x + d
            steps.append(its)
        print("%s %s first step to %.0e: steps %s = %d its (final rel %.2e)"
              % (cfg, spec, t1, steps, sum(steps), np.linalg.norm(f - A @ x) / nf), flush=True)


if __name__ == "__main__":
    main()
