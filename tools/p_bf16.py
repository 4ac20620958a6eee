"""bf16 storage of the PCG search direction p, on the CPU (design tool; the
verdict of round 3, item 4).

    python tools/p_bf16.py CONFIG [K]

The GPU's inner recurrence (k_pcg_spmv / k_pcg_update): q = A32 z + beta q,
p = z + beta p, x += alpha p (deferred), r -= alpha q, z = bf16(M r), fp64
dot products, restarted refinement to |f - A x| <= 1e-8 |f|. With p stored
as bf16 (fp32 arithmetic), x is updated with the rounded p while q still
carries A times the unrounded one, so the recursive r and the true f - A x
part by the rounding of every step: the inner solve's true residual stalls
near the bf16 unit (~4e-3), and the refinement needs more steps. Prints PCG
iterations and refinement steps per timestep for both, emulating the GPU's
arithmetic (tools/reliable_update.py's Inner: fp32 A, bf16 z, the V(1,1)
cycle of tools/amg_proto.py).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as ap  # noqa: E402
import warm_start as ws  # noqa: E402
from reliable_update import Inner, bf16  # noqa: E402


def solve(S, f, p_bf16, rtol=1e-8, inner=1e-4, maxit=500):
    nf = np.linalg.norm(f)
    x64 = np.zeros_like(f)
    its = steps = 0
    for o in range(12):
        r64 = f - S.A64 @ x64
        nr = np.linalg.norm(r64)
        if nr <= rtol * nf:
            break
        tol = inner if o == 0 else min(0.5, max(inner, 0.3 * rtol * nf / nr))
        r = r64.astype(np.float32)
        x = np.zeros_like(r)
        z = S.prec(r)
        p = bf16(z) if p_bf16 else z.copy()
        q = (S.A32 @ z).astype(np.float32)
        rz = float(r.astype(np.float64) @ z.astype(np.float64))
        nb = float(np.linalg.norm(r.astype(np.float64)))
        for it in range(maxit):
            a = rz / float(p.astype(np.float64) @ q.astype(np.float64))
            x = (x + np.float32(a) * p).astype(np.float32)
            r = (r - np.float32(a) * q).astype(np.float32)
            its += 1
            if np.linalg.norm(r.astype(np.float64)) <= tol * nb:
                break
            z = S.prec(r)
            rz2 = float(r.astype(np.float64) @ z.astype(np.float64))
            b = np.float32(rz2 / rz)
            pn = (z + b * p).astype(np.float32)
            p = bf16(pn) if p_bf16 else pn
            q = ((S.A32 @ z).astype(np.float32) + b * q).astype(np.float32)
            rz = rz2
        x64 += x.astype(np.float64)
        steps += 1
    return x64, its, steps, float(np.linalg.norm(f - S.A64 @ x64) / nf)


def main():
    cfg = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    sysl, a2m, e = ws.systems(cfg, K, 0.3)
    tot = {False: [0, 0, 0.0], True: [0, 0, 0.0]}
    for A, f in sysl:
        levels = ap.build(A, a2m, e, {})
        S = Inner(A, lambda r, lv=levels: ap.vcycle(lv, 0, r, {}))
        for pb in (False, True):
            _, n, s, rr = solve(S, f, pb)
            tot[pb][0] += n
            tot[pb][1] += s
            tot[pb][2] = max(tot[pb][2], rr)
    for pb, (n, s, rr) in tot.items():
        print("%s p %-5s PCG its/timestep %.2f  refinement steps %.2f  max rel residual %.1e"
              % (cfg, "bf16" if pb else "fp32", n / K, s / K, rr), flush=True)


if __name__ == "__main__":
    main()
