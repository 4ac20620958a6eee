"""Calibrate oracle/reference_clone.py against the real reference (container-only).

Times the reference's ``compute_velocity_field`` (imported from
/root/reference as in make_golden.py) and the clone's ``pool_timesteps`` on
the same inputs and pool size, checks the clone's V is bit-identical, and
writes tests/golden/cpu_clone_calibration.json with the time ratio
(reference / clone; >= 0.9 means the clone is not slower).

Run:  python tests/golden/calibrate_clone.py
"""
from __future__ import annotations

import io
import json
import os
import sys
import contextlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))

from make_golden import load_reference  # noqa: E402
from mofhip import synth  # noqa: E402
import oracle  # noqa: E402
import reference_clone as clone  # noqa: E402


def main():
    ref = load_reference()
    out = {"processes": 8, "cases": []}
    for n, T in ((8, 16), (32, 9)):
        p, t = synth.icosphere(n, 10.0)
        nrm, a = synth.vertex_normals(p, t), synth.triangle_areas(p, t)
        I = synth.travelling_wave(p, T)
        tk = list(range(T))
        a2, gw, e, iw, _ = ref.compute_geometrical_quantities(p, nrm, t, a)
        with contextlib.redirect_stdout(io.StringIO()):
            Vr, t_ref = ref.compute_velocity_field(8, T, a2, gw, e, iw, t, tk, a, 0.01, I, I)
        res, t_clone = clone.pool_timesteps(range(T - 1), a2, gw, e, iw, t, tk, a, 0.01, I, I, 8)
        Vc = np.array([r[0] for r in res])
        case = {"N": len(p), "T": T, "ref_wall_s": t_ref, "clone_wall_s": t_clone,
                "ratio_ref_over_clone": t_ref / t_clone,
                "V_bit_identical": bool(np.array_equal(Vc, np.array(Vr)))}
        print(case)
        out["cases"].append(case)
    with open(os.path.join(HERE, "cpu_clone_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
