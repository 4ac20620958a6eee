#!/usr/bin/env python3
"""bench_dd.py -- the domain-decomposed stretch config (BASELINE.json
configs[4]): one timestep's system split over P vertex
parts (RCB), PCG in lockstep with a halo exchange per iteration.

    python bench_dd.py [--parts P] [--config C5] [--batch B] [--steps K]
    torchrun --nproc-per-node N bench_dd.py      # RCCL: one part per rank/GPU

Without torchrun all P parts run in this process on GPU 0 (in-process
transport); the line then also times the single-domain solve of the same
systems with the same solver (mixed precision; multigrid or 2x2 block-Jacobi PCG) on the
same GPU, so ``dd_overhead`` is the cost of the decomposition itself (more,
smaller launches + the halo gathers; with ``--precond amg`` also the weaker
block-Jacobi-over-parts multigrid against the single-domain one). Under torchrun each rank drives its own
part on its own GPU and the halo / CG scalars travel over RCCL.

One step = B timesteps (assembly, PCG to 1e-8, V in HBM), inputs resident in
HBM. Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--config", default="C5", choices=["C2", "C3", "C5"])
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--precision", default="mixed", choices=["mixed", "f64"])
    ap.add_argument("--precond", default="jacobi", choices=["jacobi", "amg"],
                    help="amg: a V-cycle per part (mixed precision only; fewer iterations, "
                         "more launches per iteration)")
    ap.add_argument("--no-single", action="store_true", help="skip the single-domain reference")
    args = ap.parse_args()
    from mofhip.dist import rank_env
    rank, world, local = rank_env()
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend="gloo")  # id broadcast + timing only; data over RCCL
    dev = torch.device("cuda", local)
    torch.cuda.init()
    from mofhip import DecomposedMesh, DeviceMesh, synth

    p, t, n, a = synth.mesh_for_config(args.config)
    N = len(p)
    P = world if world > 1 else args.parts
    t0 = time.perf_counter()
    dd = DecomposedMesh(p, n, t, a, P, device=local, group=dist.group.WORLD if dist else None)
    setup_s = time.perf_counter() - t0
    info = dd.info()
    B = args.batch
    total = args.warmup + args.steps
    I_host = np.sin(3.0 * np.arctan2(p[:, 1], p[:, 0])[None, :]
                    - 0.3 * np.arange(total * B + 1, dtype=np.float64)[:, None])
    I_dev = torch.from_numpy(I_host).to(dev)
    V_dev = torch.empty((B, 2 * N), dtype=torch.float64, device=dev)
    tk = np.arange(total * B + 1, dtype=np.float64)
    opts = dict(precision=args.precision, batch=B, precond=args.precond)

    def run(solver, s):
        return solver.solve_range_device(I_dev.data_ptr(), I_dev.data_ptr(), total * B + 1, tk, s * B,
                                         (s + 1) * B, 0.01, V_dev.data_ptr(), **opts)

    def timed(solver):
        for s in range(args.warmup):
            run(solver, s)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        its = 0
        fails = 0
        for s in range(args.warmup, total):
            st = run(solver, s)
            its += st["iterations"]
            fails += st["failed"]
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if dist:
            x = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(x, op=dist.ReduceOp.MAX)
            el = float(x[0])
        return el, its, fails

    el, its, fails = timed(dd)
    V_dd = V_dev.cpu().numpy().copy()
    single = None
    if world == 1 and not args.no_single:
        mesh = DeviceMesh(p, n, t, a, device=local)
        el1, its1, _ = timed(mesh)
        diff = float(np.abs(V_dev.cpu().numpy() - V_dd).max())
        single = {"timesteps_per_s": round(args.steps * B / el1, 2),
                  "pcg_iterations_per_timestep": round(its1 / (args.steps * B), 1),
                  "max_abs_diff_V_vs_decomposed": diff}
        mesh.close()
    if rank == 0:
        line = {
            "metric": "flow timesteps/sec, one timestep decomposed over %d vertex parts (%s)"
                      % (P, args.config),
            "value": round(args.steps * B / el, 2), "unit": "timesteps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 2),
            "higher_is_better": True, "scaling": "strong", "dtype": "f32" if args.precision == "mixed" else "f64",
            "data": "synthetic travelling wave sin(3 phi - 0.3 k), dt = 1, lambda = 0.01",
            "config": {"workload": "%s, %d vertices, %d parts (RCB), %s" % (
                args.config, N, P, "RCCL, one part per GPU" if world > 1 else "in-process on 1 GPU"),
                "timesteps_per_step": B, "precision": args.precision,
                "precond": "multigrid per part" if args.precond == "amg" else "block jacobi"},
            "decomposition": {"max_owned": info["max_owned"], "ghost_rows": info["ghost_rows"],
                              "halo_fraction": round(info["ghost_rows"] / N, 4),
                              "max_neighbours": info["max_neighbours"], "setup_s": round(setup_s, 2)},
            "solver": {"pcg_iterations_per_timestep": round(its / (args.steps * B), 1), "failed": fails},
            "single_domain": single,
        }
        if single:
            line["dd_overhead"] = round(single["timesteps_per_s"] / line["value"], 3)
        print(json.dumps(line), flush=True)
    dd.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
