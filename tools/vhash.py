"""SHA-256 of V (and the iteration count) of one mixed multigrid solve on a
config mesh, for bit-identity checks between two builds (MOFHIP_LIB).

    python3 tools/vhash.py S1s 97 [batch]"""
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))

import numpy as np  # noqa: E402

from mofhip import synth  # noqa: E402
from mofhip.mesh import DeviceMesh  # noqa: E402

name = sys.argv[1]
T = int(sys.argv[2])
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 0
p, t, n, a = synth.mesh_for_config(name)
I = synth.config_wave(name, p, T)
m = DeviceMesh(p, n, t, a)
kw = {"batch": batch} if batch else {}
V, st = m.solve_range(I, np.arange(float(T)), 0, T - 1, 0.01, precision="mixed", precond="amg", **kw)
print(json.dumps({"config": name, "T": T, "batch": batch, "sha256": hashlib.sha256(np.ascontiguousarray(V).tobytes()).hexdigest(),
                  "iterations": st["iterations"], "failed": st["failed"], "lib": os.environ.get("MOFHIP_LIB", "in-tree")}))
