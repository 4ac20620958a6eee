"""Two solves in flight on one GPU (design measurement).

    python tools/streams2.py [CONFIG] [B] [STEPS]

Each mesh handle owns a HIP stream; two handles of the same mesh on one GPU,
driven from two host threads (ctypes releases the GIL), run two batches at
once, so one batch's latency-bound setup kernels (assembly, fp64 residual,
Galerkin products) can overlap the other's bandwidth-bound PCG iterations.
Prints timesteps/s for STEPS batches of B solved one after the other on one
handle, and the same batches split alternately over two handles solving
concurrently (device-resident I and V, as bench.py's default).
"""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))
from mofhip import DeviceMesh, synth  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    p, t, n, a = synth.mesh_for_config(cfg)
    N = len(p)
    meshes = [DeviceMesh(p, n, t, a, device=0) for _ in range(2)]
    K = (2 + steps) * B
    dev = torch.device("cuda", 0)
    phi = torch.atan2(torch.from_numpy(p[:, 1].copy()).to(dev), torch.from_numpy(p[:, 0].copy()).to(dev))
    I_dev = torch.empty((K + 1, N), dtype=torch.float64, device=dev)
    for r0 in range(0, K + 1, 256):
        r1 = min(K + 1, r0 + 256)
        kk = torch.arange(r0, r1, dtype=torch.float64, device=dev)
        I_dev[r0:r1] = torch.sin(3.0 * phi[None, :] - 0.3 * kk[:, None])
    V = [torch.empty((B, 2 * N), dtype=torch.float64, device=dev) for _ in range(2)]
    tk = np.arange(K + 1, dtype=np.float64)
    opts = dict(precision="mixed", batch=B, rtol=1e-8, precond="amg")
    iters = [0, 0]

    def solve(j, k0):
        st = meshes[j].solve_range_device(I_dev.data_ptr(), I_dev.data_ptr(), K + 1, tk, k0, k0 + B, 0.01,
                                          V[j].data_ptr(), device=0, **opts)
        assert st["failed"] == 0
        iters[j] += st["iterations"]

    solve(0, 0)
    solve(1, B)
    torch.cuda.synchronize(dev)
    out = {"config": cfg, "batch": B, "steps": steps}
    for rep in range(2):
        t0 = time.perf_counter()
        for s in range(steps):
            solve(0, (2 + s) * B)
        torch.cuda.synchronize(dev)
        out["sequential_%d" % rep] = round(steps * B / (time.perf_counter() - t0), 1)

        def run(j):
            for s in range(j, steps, 2):
                solve(j, (2 + s) * B)

        t0 = time.perf_counter()
        th = [threading.Thread(target=run, args=(j,)) for j in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        torch.cuda.synchronize(dev)
        out["concurrent_%d" % rep] = round(steps * B / (time.perf_counter() - t0), 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
