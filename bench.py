#!/usr/bin/env python3
"""bench.py -- flow timesteps/s of the manifold optical-flow solve on MI355X.

Metric (BASELINE.json): flow timesteps/sec on the 160k-vertex mesh
(configs[2]: 163,842-vertex icosphere, fp32-inner PCG with fp64 refinement,
aggregation-multigrid preconditioner, 1 x MI355X), plus the SpMV's achieved GB/s against the HBM roofline.

One "step" = one batch of B consecutive timesteps (assembly of a1/f + A for
every timestep, batched PCG to ||f - A V|| <= 1e-8 ||f||, planar V written
to HBM), inputs resident in HBM before the timed region. With N GPUs (one
process per GPU, torchrun) each rank solves its own contiguous timesteps
(weak scaling, no collective on the data path); value = all timesteps / the
max-over-ranks wall time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                    [--config C3] [--precision mixed|f64] [--precond amg|jacobi]
                    [--no-cpu-baseline]
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
sys.path.insert(0, os.path.join(REPO, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
CONFIG_NAMES = {
    "C2": "32k-vertex jittered icosphere (n=57, 32,492 vertices), fp64 Jacobi-PCG",
    "C3": "160k-vertex jittered icosphere (n=128, 163,842 vertices), fp32 PCG + fp64 refinement",
    "C5": "640k-vertex jittered icosphere (n=253, 640,092 vertices)",
    "R3": "163,842-vertex irregular random-hull sphere (valence 3-14, random vertex order)",
    "P3": "C3 mesh with randomly relabelled vertices (no index locality)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256, help="timesteps per step")
    ap.add_argument("--config", default="C3", choices=sorted(CONFIG_NAMES))
    ap.add_argument("--precision", default=None, choices=["mixed", "f64"])
    ap.add_argument("--precond", default=None, choices=["jacobi", "amg"],
                    help="inner preconditioner (default: amg for mixed, jacobi for f64)")
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--inner-rtol", type=float, default=0.0,
                    help="mixed precision: inner PCG tolerance per refinement step (0: the library's 1e-4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-frac", type=float, default=1.0 / 64,
                    help="fraction of the triangle loop the CPU baseline times")
    ap.add_argument("--lambda_", type=float, default=0.01)
    return ap.parse_args()


def pmc_traffic(key, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json, made by profiles/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes of this bench at the same
    config; read bytes = 2 x FETCH_SIZE on gfx950). None if not measured."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        entry = json.load(open(path))[key]
        return round(entry["kernels"][kernel]["hbm_bytes_per_launch"]), entry["source"][0]
    except (OSError, ValueError, KeyError):
        return None, None


def cpu_baseline(p, t, n, a, lam, frac):
    """The reference CPU path (lil assembly + spsolve on a Pool), timed on this
    host on a bounded sample: Pool(C) runs C timesteps; each assembles the
    first `frac` of the triangles with the reference's scalar loop and then
    runs spsolve on the full-size system. Per-timestep time is extrapolated
    linearly in the triangle count."""
    import oracle
    import reference_clone as clone
    C = clone.default_cores()
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    a2l = clone.as_lil(a2)
    T = C + 1
    from mofhip import synth
    I = synth.travelling_wave(p, T)
    tk = list(range(T))
    M = len(t)
    S = max(1, int(M * frac))
    res, wall = clone.pool_timesteps(range(C), a2l, gw, e, iw, t, tk, a, lam, I, I, C,
                                     sample_tris=S)
    loop = float(np.mean([r[1] for r in res]))
    solve = float(np.mean([r[2] for r in res]))
    full_wall = wall + loop * (M / S - 1.0)
    value = C / full_wall
    return {
        "value": value, "unit": "timesteps/s", "cores": C, "kind": "port",
        "sample": ("Pool(%d) x %d timesteps of the reference algorithm (lil scalar assembly, csr, "
                   "spsolve; oracle/reference_clone.py, calibrated vs the reference) on the %d-vertex "
                   "mesh; triangle loop timed on %d of %d triangles (%.1f s/step measured, "
                   "extrapolated x%.0f), spsolve on the full system (%.1f s/step); pool wall %.1f s"
                   % (C, C, len(p), S, M, loop, M / S, solve, wall)),
    }


def main():
    args = parse()
    from mofhip.dist import max_over_ranks, rank_env, rank_k_range, sum_over_ranks
    rank, world, local = rank_env()
    # MOF_BENCH_REHEARSE=1: every rank on GPU 0 over gloo -- exercises the
    # N-rank path on a 1-GPU box (RCCL refuses two ranks on one GPU)
    rehearse = os.environ.get("MOF_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    precision = args.precision or ("f64" if args.config == "C2" else "mixed")

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group(backend="gloo")
        else:
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    from mofhip import DeviceMesh, synth

    # --- one-time mesh build (reported separately, outside the metric) -----
    p, t, n, a = synth.mesh_for_config(args.config)
    N = len(p)
    t0 = time.perf_counter()
    mesh = DeviceMesh(p, n, t, a, device=local)
    info = mesh.info()
    mesh_s = time.perf_counter() - t0

    # --- this rank's synthetic signal, resident in HBM ----------------------
    B = args.batch
    steps_total = args.warmup + args.steps
    K_rank = steps_total * B
    k_off, _ = rank_k_range(rank, world, 0, world * K_rank)  # this rank's timesteps
    # generated on the device: (K_rank + 1) x N f64 is 7.4 GB per rank at the
    # default C3 sizes, which 8 ranks would otherwise hold in host memory
    dev = torch.device("cuda", local)
    pts = torch.from_numpy(np.ascontiguousarray(p[:, :2])).to(dev)
    phi = torch.atan2(pts[:, 1], pts[:, 0])
    kk = k_off + torch.arange(K_rank + 1, dtype=torch.float64, device=dev)
    I_dev = torch.empty((K_rank + 1, N), dtype=torch.float64, device=dev)
    for r0 in range(0, K_rank + 1, 256):
        r1 = min(K_rank + 1, r0 + 256)
        I_dev[r0:r1] = torch.sin(3.0 * phi[None, :] - 0.3 * kk[r0:r1, None])
    del pts, phi, kk
    V_dev = torch.empty((B, 2 * N), dtype=torch.float64, device=dev)
    tk = np.arange(K_rank + 1, dtype=np.float64)
    torch.cuda.synchronize(dev)
    precond = (args.precond or "amg") if precision == "mixed" else "jacobi"
    opts = dict(precision=precision, batch=B, rtol=args.rtol, precond=precond, inner_rtol=args.inner_rtol)

    def step(s, timed):
        return mesh.solve_range_device(I_dev.data_ptr(), I_dev.data_ptr(), K_rank + 1, tk, s * B,
                                       (s + 1) * B, args.lambda_, V_dev.data_ptr(), device=local,
                                       time_spmv=timed, **opts)

    for s in range(args.warmup):
        step(s, False)

    # --- timed region -------------------------------------------------------
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    agg = {"iterations": 0, "failed": 0, "ms_spmv": 0.0, "spmv_bytes": 0.0, "spmv_launches": 0,
           "max_rel_residual": 0.0, "ms_assembly": 0.0, "ms_solve": 0.0}
    for s in range(args.warmup, steps_total):
        st = step(s, True)
        for k in ("iterations", "failed", "ms_spmv", "spmv_bytes", "spmv_launches", "ms_assembly",
                  "ms_solve"):
            agg[k] += st[k]
        agg["max_rel_residual"] = max(agg["max_rel_residual"], st["max_rel_residual"])
        agg["max_outer_steps"] = max(agg.get("max_outer_steps", 0), st["outer_steps"])
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    cdev = torch.device("cpu") if rehearse else dev
    elapsed = max_over_ranks(elapsed, dist, cdev)
    agg["failed"] = int(sum_over_ranks(agg["failed"], dist, cdev))
    n_ts = world * args.steps * B
    value = n_ts / elapsed

    # roofline of the dominant kernel (k_pcg_spmv), live over the timed region
    achieved = agg["spmv_bytes"] / (agg["ms_spmv"] * 1e-3) / 1e9 if agg["ms_spmv"] > 0 else 0.0
    kname = "k_pcg_spmv<%s, false>" % ("float" if precision == "mixed" else "double")
    traffic, traffic_src = pmc_traffic("%s/%s/%s/B%d" % (args.config, precision, precond, B), kname)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": traffic_src, "kernel": kname,
                "bytes_per_launch": round(agg["spmv_bytes"] / max(1, agg["spmv_launches"])),
                "us_per_launch": round(1e3 * agg["ms_spmv"] / max(1, agg["spmv_launches"]), 2),
                "launches": agg["spmv_launches"]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(p, t, n, a, args.lambda_, args.cpu_sample_frac)

    if rank == 0:
        line = {
            "metric": "flow timesteps/sec on 160k-vertex mesh" if args.config == "C3"
                      else "flow timesteps/sec (%s)" % args.config,
            "value": round(value, 3), "unit": "timesteps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" if precision == "mixed" else "f64",
            "data": "synthetic travelling wave sin(3 phi - 0.3 k), dt = 1, lambda = 0.01",
            "config": {"workload": CONFIG_NAMES[args.config], "vertices": N, "triangles": len(t),
                       "timesteps_per_step": B, "timesteps_timed": n_ts, "precision": precision,
                       "precond": opts["precond"],
                       "rtol": args.rtol, "parallelism": "timestep shards x%d" % world},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "solver": {"pcg_iterations_per_timestep": round(agg["iterations"] / (args.steps * B), 1),
                       "failed": agg["failed"], "max_rel_residual": agg["max_rel_residual"],
                       "max_refinement_steps": agg.get("max_outer_steps", 0),
                       "ms_assembly_per_timestep": round(agg["ms_assembly"] / (args.steps * B), 4),
                       "ms_solve_per_timestep": round(agg["ms_solve"] / (args.steps * B), 4),
                       "mesh_build_s": round(mesh_s, 3), "mesh_geometry_ms": round(info["ms_geometry"], 3),
                       "mesh_pattern_ms": round(info["ms_pattern"], 3)},
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
