"""Inner operator precision study (design tool, CPU; DESIGN.md §4 "Rejected
on paper"): iterative refinement in fp64 around an inner PCG whose operator
is A rounded to fp32 (the library), to fp16 after symmetric diagonal
scaling (D^-1/2 A D^-1/2, every entry <= 1, so fp16's 2^-11 holds for the
large ones), or to bf16. The preconditioner is the same V-cycle in every
case; the inner solves stop at the library's rule (first step 7e-5, later
steps max(1e-4, 0.3 rtol |f| / |r|)). Reports outer steps, total inner
iterations and the final relative residual.

    python tools/half_a_study.py CONFIG [variant]
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as ap  # noqa: E402
from refine_study import pcg_x  # noqa: E402


def rounded(A, kind):
    A = sp.csr_matrix(A)
    if kind == "fp32":
        return A.astype(np.float32).astype(np.float64)
    if kind == "bf16":
        d = A.data.astype(np.float32).view(np.uint32)
        d = ((d + 0x7FFF + ((d >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
        B = A.copy()
        B.data = d.view(np.float32).astype(np.float64)
        return B
    if kind == "fp16s":
        s = 1.0 / np.sqrt(A.diagonal())
        S = sp.diags(s)
        As = (S @ A @ S).tocsr()
        As.data = As.data.astype(np.float16).astype(np.float64)
        Si = sp.diags(1.0 / s)
        return (Si @ As @ Si).tocsr()
    raise ValueError(kind)


def main():
    cfg = sys.argv[1]
    spec = sys.argv[2] if len(sys.argv) > 2 else "base"
    A, a2m, f, e, N = ap.system(cfg)
    opts = ap.parse(spec.split("+"))
    levels = ap.build(A, a2m, e, opts)
    M = lambda r: ap.vcycle(levels, 0, r, opts)  # noqa: E731
    rtol = float(os.environ.get("RTOL", "1e-6"))
    nf = np.linalg.norm(f)
    xs = sp.linalg.spsolve(A.tocsc(), f)
    for kind in ("fp32", "fp16s", "bf16"):
        At = rounded(A, kind)
        x = np.zeros_like(f)
        steps = []
        for o in range(12):
            r = f - A @ x
            rel = np.linalg.norm(r) / nf
            if rel <= rtol and o >= 2:
                break
            t = 7e-5 if o == 0 else max(1e-4, min(0.5, 0.3 * rtol / rel))
            d, its = pcg_x(At, r, M, t)
            x = x + d
            steps.append(its)
        err = np.abs(x - xs).max() / np.abs(xs).max()
        print("%s %s inner A in %-5s: steps %s = %d its, final rel %.2e, max err / max|x| %.2e"
              % (cfg, spec, kind, steps, sum(steps), np.linalg.norm(f - A @ x) / nf, err), flush=True)


if __name__ == "__main__":
    main()
