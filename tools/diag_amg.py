"""Multigrid failure diagnosis on one mesh (design tool, GPU).

    python tools/diag_amg.py CONFIG [K] [ENV=VAL ...]

Solves K timesteps (mixed + multigrid) with recovery off and MOF_VERBOSE
set, so the library prints per refinement step the inner iterations and why
the first solve's failed systems failed; the environment assignments (e.g.
MOF_AMG_SMOOTH=0, MOF_AMG_OMEGA=...) select the variant. The
signal is the bench's for CONFIG (synth.config_wave; DIAG_PINWHEEL=1: the
atan2 pinwheel of synth.travelling_wave).
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))


def main():
    cfg = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 and "=" not in sys.argv[2] else 8
    for kv in sys.argv[2:]:
        if "=" in kv:
            k, v = kv.split("=", 1)
            os.environ[k] = v
    os.environ["MOF_VERBOSE"] = "1"
    from mofhip import DeviceMesh, synth
    p, t, n, a = synth.mesh_for_config(cfg)
    m = DeviceMesh(p, n, t, a)
    I = synth.config_wave(cfg, p, K + 1) if os.environ.get("DIAG_PINWHEEL") != "1" else synth.travelling_wave(p, K + 1)
    tk = np.arange(K + 1, dtype=np.float64)
    out = {"config": cfg, "env": [kv for kv in sys.argv[2:] if "=" in kv]}
    for rec in (False, True):
        V, st = m.solve_range(I, tk, 0, K, 0.01, precision="mixed", precond="amg", recovery=rec)
        out["recovery" if rec else "no_recovery"] = {k: st[k] for k in ("iterations", "failed", "recovered",
                                                                        "max_rel_residual", "outer_steps")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
