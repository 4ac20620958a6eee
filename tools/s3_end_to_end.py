"""The reference's real workload through the drop-in, end to end (design /
measurement tool, GPU): one S3-style call sequence on a fresh process --
import, runtime start, compute_geometrical_quantities (the mesh build),
compute_velocity_field (the reference's own timer, compute_optical_flow.py:
160-182, covers only this call's solve) -- for the small configs whose whole
job is one call (S1s: 3,249 vertices x 97 solves, the reference's mesh size
and time_steps; C1: 642 x 15). The first call carries the one-time costs
(workspace, multigrid hierarchy, code-object load); the second call on the
same mesh is the steady state.

    python tools/s3_end_to_end.py [CONFIG ...]
"""
import json
import os
import sys
import time

t_start = time.perf_counter()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))

import numpy as np  # noqa: E402

from mofhip import device_count, synth  # noqa: E402
from utils import compute_optical_flow as cof  # noqa: E402

T_OF = {"S1s": 98, "C1": 16}


def run(cfg):
    t0 = time.perf_counter()
    p, t, n, a = synth.mesh_for_config(cfg)
    T = T_OF[cfg]
    I = synth.config_wave(cfg, p, T)
    tk = np.arange(T, dtype=np.float64)
    t_inputs = time.perf_counter() - t0
    t0 = time.perf_counter()
    a2, gw, e, iw, geo_s = cof.compute_geometrical_quantities(p, n, t, a)
    t_geo = time.perf_counter() - t0
    out = {"config": cfg, "N": len(p), "timesteps": T - 1, "geometry_wall_s": round(t_geo, 4),
           "geometry_reported_s": round(geo_s, 4), "inputs_s": round(t_inputs, 3)}
    for rep in ("first", "second"):
        t0 = time.perf_counter()
        V, ex = cof.compute_velocity_field(1, T, a2, gw, e, iw, t, tk, a, 0.01, I, I)
        wall = time.perf_counter() - t0
        assert len(V) == T - 1 and all(np.isfinite(v).all() for v in V)
        out[rep + "_call_wall_s"] = round(wall, 4)
        out[rep + "_call_reference_timer_s"] = round(ex, 4)
    return out


def main():
    t0 = time.perf_counter()
    n = device_count()
    runtime_s = time.perf_counter() - t0
    res = {"process_to_import_s": round(t0 - t_start, 3), "runtime_start_s": round(runtime_s, 3), "devices": n,
           "precision": cof.SOLVER_OPTIONS.get("precision")}
    for cfg in sys.argv[1:] or ["S1s", "C1"]:
        res[cfg] = run(cfg)
    res["process_total_s"] = round(time.perf_counter() - t_start, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
