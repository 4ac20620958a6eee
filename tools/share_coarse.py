"""Design study (CPU): the coarse levels of timestep 0's hierarchy reused for
the next timesteps (level 0 keeps each system's own operator and smoother):

    python tools/share_coarse.py CONFIG K OMEGA
"""
import sys, copy
sys.path.insert(0, 'tools')
import numpy as np
import warm_start as ws
import amg_proto as ap
cfg = sys.argv[1]; K = int(sys.argv[2]); om = float(sys.argv[3])
sysl, a2m, e = ws.systems(cfg, K, om)
base = ap.build(sysl[0][0], a2m, e, {})
for k, (A, f) in enumerate(sysl):
    own = ap.build(A, a2m, e, {})
    M = lambda r, lv=own: ap.vcycle(lv, 0, r, {})
    _, n_own, _ = ws.refine(A, f, M, np.zeros_like(f))
    sh = copy.copy(base)
    L0 = copy.copy(base[0]); L0.A = A; L0.D, L0.Dinv = ap.block_diag_inv(A, L0.bs)
    for a in ('Aq',):
        if hasattr(L0, a): delattr(L0, a)
    sh = [L0] + base[1:]
    M2 = lambda r, lv=sh: ap.vcycle(lv, 0, r, {})
    _, n_sh, _ = ws.refine(A, f, M2, np.zeros_like(f))
    print("%s om %.2f k=%d: own hierarchy %d its, coarse levels from k=0: %d its" % (cfg, om, k, n_own, n_sh), flush=True)
