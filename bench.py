#!/usr/bin/env python3
"""bench.py -- flow timesteps/s of the manifold optical-flow solve on MI355X.

Metric (BASELINE.json): flow timesteps/sec on the 160k-vertex mesh
(configs[2]: 163,842-vertex icosphere, fp32-inner PCG with fp64 refinement,
aggregation-multigrid preconditioner, 1 x MI355X), plus the SpMV's achieved GB/s against the HBM roofline.

One "step" = one batch of B consecutive timesteps (assembly of a1/f + A for
every timestep, batched PCG to ||f - A V|| <= 1e-8 ||f||, planar V written
to HBM), inputs resident in HBM before the timed region. With N GPUs (one
process per GPU) each rank solves its own contiguous timesteps (no
collective on the data path); value = all timesteps / the max-over-ranks
wall time.

  * weak scaling (default): every rank solves K batches of B timesteps;
  * --fixed-timesteps T (strong scaling, config C4): one step = the whole
    T-timestep job (5000 in BASELINE configs[3]) split into contiguous
    k-ranges over the N ranks, as the reference's Pool splits it
    (compute_optical_flow.py:157-177);
  * --io host: the drop-in's path -- I in pageable host memory, V back into
    host memory, one mof_solve_range call over all timed timesteps (the
    PCIe-inclusive rate; value is never this line's unless asked for).

--gpus N without a torchrun environment starts N local worker processes
itself (torch.distributed.run, 127.0.0.1) before anything touches a GPU;
under torchrun --gpus must equal WORLD_SIZE.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                    [--config C3] [--precision mixed|f64] [--precond amg|jacobi]
                    [--fixed-timesteps T] [--io device|host] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
CONFIG_NAMES = {
    "C1": "642-vertex icosphere (n=8), T=16 (15 solves), the reference S3 path's parity case",
    "C2": "32k-vertex jittered icosphere (n=57, 32,492 vertices), fp64 Jacobi-PCG",
    "C3": "160k-vertex jittered icosphere (n=128, 163,842 vertices), fp32 PCG + fp64 refinement",
    "C5": "640k-vertex jittered icosphere (n=253, 640,092 vertices)",
    "R3": "163,842-vertex irregular random-hull sphere (valence 3-14, random vertex order)",
    "P3": "C3 mesh with randomly relabelled vertices (no index locality)",
    "F3": "163,842-vertex folded cortex-like surface (fsaverage's order-7 icosahedral topology, radially folded "
          "by a seeded band-limited field: gyral period 16-27 mm at 70 mm radius, sulcal amplitude 15 % of the "
          "radius; synth.folded_sphere)",
    "S1": "160,801-vertex S1-like reconstructed patch (51 x 51 electrode grid, Delaunay, butterfly x3, smoothed)",
    "S1m": "40,401-vertex S1-like reconstructed patch (26 x 26 electrode grid at 3 mm)",
    "S1s": "3,249-vertex S1-like reconstructed patch (8 x 8 electrode grid), T=98 (97 solves), the reference's "
           "real workload size (config.yaml:5, find_singularity_point.py:19-20)",
}
# small jobs timed whole: one step = every timestep of the job (one batch)
SMALL_JOBS = {"C1": 15, "S1s": 97}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    # 1536 timesteps per step: +1-2 % over 1024 on one box (round 5,
    # profiles/r05_ab/batch/: 3710 vs 3626-3675 timesteps/s at C3), which was
    # +1-4 % over 512 (round 4: the setup kernels and the small multigrid
    # levels hide more latency per launch); ~235 GB of HBM at C3 with the
    # driver's 25 steps of signal rows, else the largest of 1024, 512, ...
    # that fits
    ap.add_argument("--batch", type=int, default=1536, help="timesteps per step")
    ap.add_argument("--config", default="C3", choices=sorted(CONFIG_NAMES))
    ap.add_argument("--precision", default=None, choices=["mixed", "f64"])
    ap.add_argument("--precond", default=None, choices=["jacobi", "amg"],
                    help="inner preconditioner (default: amg for mixed, jacobi for f64)")
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--inner-rtol", type=float, default=0.0,
                    help="mixed precision: inner PCG tolerance per refinement step (0: the library's 1e-4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-frac", type=float, default=1.0 / 4,
                    help="fraction of the triangle loop the CPU baseline times")
    ap.add_argument("--cpu-timesteps-per-core", type=int, default=2,
                    help="CPU baseline: timesteps per pool process (SURVEY.md 8(d): 2 per core)")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="CPU baseline pool size (0: the box's CPU share per GPU, 16; BASELINE.md names "
                         "os.cpu_count(), which a larger pool approaches)")
    ap.add_argument("--lambda_", type=float, default=0.01)
    ap.add_argument("--fixed-timesteps", type=int, default=0,
                    help="strong scaling: one step = this many timesteps split over the ranks")
    ap.add_argument("--io", default="device", choices=["device", "host"],
                    help="device: I/V resident in HBM; host: pageable numpy in and out (drop-in path)")
    ap.add_argument("--parity-samples", type=int, default=2,
                    help="timesteps of the last timed batch checked against the oracle + spsolve (0: none)")
    ap.add_argument("--fused", default="auto", choices=["auto", "on", "off"],
                    help="fp64: the one-launch fused solve per batch (auto: the library's choice, small meshes)")
    ap.add_argument("--allow-recovery", action="store_true",
                    help="do not treat recovered systems as a defect (experiments that force a failing solver)")
    ap.add_argument("--etol", type=float, default=0.0,
                    help="the refinement's error control: estimated error <= etol max|V| (0: the library's "
                         "1e-7, < 0: the residual test alone)")
    ap.add_argument("--legs", default="auto",
                    help="comma-separated extra configurations timed after the main line on the same GPU, "
                         "each with its iterations, parity and SpMV roofline (auto: F3,S1s,S1 -- the "
                         "reference's mesh class -- for a 1-GPU C3 line; none: no legs)")
    ap.add_argument("--host-batches", type=int, default=4,
                    help="--io device: batches of the host-to-host leg (SURVEY.md 8(d)'s metric) timed after "
                         "the device-resident region (0: none)")
    return ap.parse_args()


def self_launch(args):
    """--gpus N > 1 outside torchrun: run N local ranks through
    torch.distributed.run as a child process (this process never initialises
    the GPU; nothing is re-exec'ed) and exit with its status. Under torchrun,
    --gpus must match WORLD_SIZE."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s" % (args.gpus, world))
        return
    if args.gpus <= 1:
        return
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % args.gpus, "--master-addr=127.0.0.1",
           "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def pmc_traffic(key, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json, made by profiles/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes of this bench at the same
    config; read bytes = 2 x FETCH_SIZE on gfx950). None if not measured."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        entry = json.load(open(path))[key]
        # the instance name may carry more template arguments (e.g. the bf16-z
        # flag: k_pcg_spmv<float, false, true>); the largest matching instance
        names = [k for k in entry["kernels"] if k == kernel or k.startswith(kernel[:-1] + ",")]
        best = max(names, key=lambda k: entry["kernels"][k]["hbm_bytes_per_launch"])
        return round(entry["kernels"][best]["hbm_bytes_per_launch"]), entry["source"][0]
    except (OSError, ValueError, KeyError):
        return None, None


def step_traffic(key, value):
    """Whole-step HBM traffic from the committed PMC passes of this
    configuration: every dispatch's FETCH_SIZE (x2) + WRITE_SIZE summed over
    the profiled run, per timestep; at this line's rate that is the achieved
    whole-step bandwidth (all kernels, not only the SpMV)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        run = json.load(open(path))[key]["run"]
    except (OSError, ValueError, KeyError):
        return None
    bw = run["hbm_bytes_per_timestep"] * value / 1e9
    return {"hbm_bytes_per_timestep": round(run["hbm_bytes_per_timestep"]), "achieved": round(bw, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(bw / HBM_PEAK_GBS, 4),
            "source": "profiles/pmc_traffic.json[%s] (PMC run of %d timesteps)" % (key, run["timesteps"])}


def parity_checks(jobs):
    """Parity in the measured run: for each sampled timestep of a line's last
    timed batch, the reference's system (oracle.step_system: the bit-exact
    restatement of worker's assembly, compute_optical_flow.py:100-146) solved
    by the reference's own solver, scipy's spsolve (:147), against the V the
    timed GPU solve returned. jobs: [(geometry, triangles, areas, lambda,
    samples)], one per line (the main line and its legs); every sample of
    every job runs in one pool of host threads (the C oracle and SuperLU
    release the GIL). Returns one parity dict per job."""
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    from scipy.sparse.linalg import spsolve

    def one(item):
        (a2, gw, e, iw), t, a, lam, (k, I0, I1, dt, V) = item
        A, f = oracle.step_system(a2, gw, e, iw, t, a, lam, I0, I1, dt)
        Vo = spsolve(A.tocsc(), f)
        return k, float(np.abs(V - Vo).max()), float(np.abs(Vo).max()), \
            float(np.linalg.norm(f - A @ V) / np.linalg.norm(f))

    items = [((geom, t, a, lam, smp), j) for j, (geom, t, a, lam, samples) in enumerate(jobs) for smp in samples]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max(1, min(16, len(items)))) as ex:
        res = list(ex.map(one, [it for it, _ in items]))
    secs = round(time.perf_counter() - t0, 1)
    out = []
    for j in range(len(jobs)):
        rj = [r for r, (_, jj) in zip(res, items) if jj == j]
        out.append({"max_abs_err": max(r[1] for r in rj), "timesteps": [r[0] for r in rj],
                    "per_timestep_max_abs_err": [r[1] for r in rj], "max_abs_V": max(r[2] for r in rj),
                    "rel_residual_oracle_A": max(r[3] for r in rj), "bar": 1e-6,
                    "reference": "oracle.step_system (bit-exact A_k, f_k of compute_optical_flow.py:100-146) + "
                                 "scipy spsolve (:147), on timesteps of the last timed batch",
                    "seconds": secs} if rj else None)
    return out


# extra lines after the main one (--legs): (batch, timed steps, warmup steps);
# the small jobs time their whole job per step (SMALL_JOBS)
LEGS = {"F3": (1536, 5, 1), "S1s": (97, 20, 2), "S1": (1536, 3, 1), "R3": (1536, 3, 1), "C2": (1536, 5, 1)}


def run_leg(name, args, torch, local):
    """One extra configuration on this GPU, device-resident like the main
    line (mixed precision, multigrid): its timesteps/s, PCG iterations, SpMV
    roofline and parity samples (checked by parity_checks with the main
    line's). The mesh and its signal rows are freed before returning."""
    from mofhip import DeviceMesh, synth
    p, t, n, a = synth.mesh_for_config(name)
    N = len(p)
    dev = torch.device("cuda", local)
    t0 = time.perf_counter()
    mesh = DeviceMesh(p, n, t, a, device=local)
    info = mesh.info()
    build_s = time.perf_counter() - t0
    B, steps, warmup = LEGS[name]
    if name in SMALL_JOBS:
        B = SMALL_JOBS[name]
        calls = [(0, B)] * (warmup + steps)
        rows = B + 1
    else:
        B = min(B, int(info.get("max_batch") or B))
        calls = [(s_ * B, (s_ + 1) * B) for s_ in range(warmup + steps)]
        rows = (warmup + steps) * B + 1
    phase, kappa = synth.wave_phase(name, p)
    phi = torch.from_numpy(np.ascontiguousarray(phase)).to(dev)
    I_dev = torch.empty((rows, N), dtype=torch.float64, device=dev)
    for r0 in range(0, rows, 256):
        r1 = min(rows, r0 + 256)
        kk = torch.arange(r0, r1, dtype=torch.float64, device=dev)
        I_dev[r0:r1] = torch.sin(kappa * phi[None, :] - 0.3 * kk[:, None])
    V_dev = torch.empty((B, 2 * N), dtype=torch.float64, device=dev)
    tk = np.arange(rows, dtype=np.float64)
    opts = dict(precision="mixed", batch=B, rtol=args.rtol, precond="amg", etol=args.etol)

    def solve(a_, b_, timed):
        return mesh.solve_range_device(I_dev.data_ptr(), I_dev.data_ptr(), rows, tk, a_, b_, args.lambda_,
                                       V_dev.data_ptr(), device=local, time_spmv=timed, **opts)

    for a_, b_ in calls[:warmup]:
        solve(a_, b_, False)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    agg = {}
    for a_, b_ in calls[warmup:]:
        st = solve(a_, b_, True)
        for k, v in st.items():
            agg[k] = max(agg.get(k, 0), v) if k.startswith("max_") else agg.get(k, 0) + v
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    a_, b_ = calls[-1]
    samples = []
    for k in sorted({a_, b_ - 1}):
        samples.append((k, I_dev[k].cpu().numpy(), I_dev[k + 1].cpu().numpy(), float(tk[k + 1] - tk[k]),
                        V_dev[k - a_].cpu().numpy()))
    del I_dev, V_dev, phi
    mesh.close()
    torch.cuda.empty_cache()
    n_ts = agg["systems"]
    leg = {"config": name, "workload": CONFIG_NAMES[name], "vertices": N, "batch": B,
           "value": round(n_ts / elapsed, 3), "unit": "timesteps/s", "steps": steps, "warmup": warmup,
           "timesteps_timed": n_ts, "ms_per_step": round(1e3 * elapsed / steps, 3),
           "precision": "mixed", "precond": "amg",
           "roofline": spmv_roofline(agg, info, N, "mixed", "amg", B, name),
           "solver": {"pcg_iterations_per_timestep": round(agg["iterations"] / max(1, n_ts), 1),
                      "failed": agg["failed"], "recovered": agg["recovered"],
                      "max_rel_residual": agg["max_rel_residual"], "max_err_est": agg["max_err_est"],
                      "mesh_build_s": round(build_s, 3)}}
    return leg, (p, t, n, a), samples


def size_batch(B, N, free_b, max_batch, rows_of):
    """The batch this rank can run: a batch whose workspace (~720 B per
    vertex and timestep with the multigrid levels, the library's own
    estimate) and signal rows (rows_of(b) rows of N f64) do not fit 85 % of
    the GPU's free HBM is reduced -- to the largest multiple of 256 that
    fits, then halved below 256 -- and said so, rather than failing an
    allocation mid-run; then clamped to the library's largest batch whose
    launch grids fit 2^32 work-items (mof_mesh_info.max_batch). Returns
    (batch, note or None)."""
    def need(b):
        return 720.0 * N * b + 8.0 * N * rows_of(b) + 16.0 * N * b

    note = None
    B0 = B
    if need(B) > 0.85 * free_b and B > 256:
        B = B // 256 * 256
        while B > 256 and need(B) > 0.85 * free_b:
            B -= 256
    while B > 64 and need(B) > 0.85 * free_b:
        B //= 2
    if B != B0:
        note = "batch %d reduced to %d: %.0f GB of HBM free" % (B0, B, free_b / 1e9)
    if max_batch and B > max_batch:
        B1, B = B, int(max_batch)
        note = (note + "; " if note else "") + "batch %d reduced to %d: launch grids past 2^32 work-items" % (B1, B)
    return B, note


def spmv_roofline(agg, info, N, precision, precond, B, config):
    """The SpMV roofline of a timed region (the dominant kernel, k_pcg_spmv)."""
    # roofline of the dominant kernel (k_pcg_spmv), live over the timed region:
    # every timed launch is charged with the systems it processed, in
    # SURVEY.md 8(d)'s algorithmic bytes of a batched CSR SpMV
    #   B nnz s_v + 4 nnz + 4 (R + 1) + B R (s_x + s_y)   (nnz = 4 nblocks, R = 2N)
    achieved = agg["spmv_bytes"] / (agg["ms_spmv"] * 1e-3) / 1e9 if agg["ms_spmv"] > 0 else 0.0
    kname = "k_pcg_spmv<%s, false>" % ("float" if precision == "mixed" else "double")
    traffic, traffic_src = pmc_traffic("%s/%s/%s/B%d" % (config, precision, precond, B), kname)
    sv = 4 if precision == "mixed" else 8
    nnz, R = 4 * info["nblocks"], 2 * N
    per_sys = nnz * sv + R * 2 * sv
    shared = 4 * nnz + 4 * (R + 1)
    nl = max(1, agg["spmv_launches"])
    nfull = max(1, agg["spmv_full_launches"])
    t_full = agg["ms_spmv_full"] / nfull * 1e-3 if agg["ms_spmv_full"] > 0 else 0.0
    # launches that did work (the shared bytes are charged once each)
    n_work = round((agg["spmv_bytes"] - agg["spmv_systems"] * per_sys) / shared) if agg["spmv_bytes"] else 0
    # the kernel's own traffic: the fp32 operator's diagonal + upper blocks
    # (lower ones read as transposes through the shared mirror table), z
    # gathered, q, p and x read and written; shared column indices (+ mirror)
    nread = info.get("blocks_read", info["nblocks"]) if precision == "mixed" else info["nblocks"]
    k_sys = nread * 4 * sv + N * 2 * sv * 7
    k_shared = info["nblocks"] * 4 * (2 if nread < info["nblocks"] else 1)
    k_bytes = agg["spmv_systems"] * k_sys + n_work * k_shared
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": traffic_src, "kernel": kname,
                "bytes_formula": "SURVEY.md 8(d): B*nnz*s_v + 4*nnz + 4*(R+1) + B*R*(s_x+s_y)",
                "bytes_per_launch": round(agg["spmv_bytes"] / nl),
                "bytes_per_system": per_sys, "shared_bytes_per_launch": shared,
                "systems_per_launch": round(agg["spmv_systems"] / nl, 2),
                "us_per_launch": round(1e3 * agg["ms_spmv"] / nl, 2),
                "launches": agg["spmv_launches"],
                "full_launches": agg["spmv_full_launches"],
                "us_per_full_launch": round(1e6 * t_full, 2),
                "full_launch_frac": round((B * per_sys + shared) / t_full / 1e9 / HBM_PEAK_GBS, 4)
                if t_full > 0 else None,
                "symmetric_reads": nread < info["nblocks"],
                # context: what this fused kernel itself must move
                "kernel_bytes_per_system": k_sys, "kernel_shared_bytes_per_launch": k_shared,
                "kernel_frac": round(k_bytes / (agg["ms_spmv"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                if agg["ms_spmv"] > 0 else None,
                "kernel_full_launch_frac": round((B * k_sys + k_shared) / t_full / 1e9 / HBM_PEAK_GBS, 4)
                if t_full > 0 else None}

    if agg["spmv_launches"] == 0 and agg["fused_launches"] > 0:
        # the fused one-launch solve (small meshes) runs its SpMV inside one
        # kernel per batch with no per-SpMV timing: no SpMV roofline is
        # measured, and the line says so instead of reporting 0 GB/s
        roofline = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                    "traffic": None, "kernel": "k_solve_fused (the whole fp64 solve of a batch in one launch)",
                    "us_per_launch": round(1e3 * agg["ms_fused"] / agg["fused_launches"], 2),
                    "launches": agg["fused_launches"],
                    "note": "no per-SpMV timing inside the fused launch: the SpMV roofline is not measured"}
    return roofline


def cpu_baseline(p, t, n, a, lam, frac, per_core=2, geom=None, full_timesteps=0, cores=0, config="C3"):
    """The reference CPU path (lil assembly + spsolve on a Pool), timed on this
    host on a bounded sample: Pool(C) runs per_core * C timesteps (SURVEY.md
    §8(d): 2 C); each assembles the first `frac` of the triangles with the
    reference's scalar loop and then runs spsolve on the full-size system.
    Every core runs per_core timesteps back to back, so the pool's wall
    misses per_core x the unsampled part of the loop; per-timestep loop time
    is extrapolated linearly in the triangle count."""
    import oracle
    import reference_clone as clone
    C = int(cores) if cores and cores > 0 else clone.default_cores()
    K = per_core * C
    if full_timesteps:  # C1 is timed in full (every timestep, the whole triangle loop)
        K, frac = full_timesteps, 1.0
        C = min(C, K)
    a2, gw, e, iw = geom if geom is not None else oracle.geometry(p, n, t, a)
    a2l = clone.as_lil(a2)
    T = K + 1
    from mofhip import synth
    I = synth.config_wave(config, p, T)
    tk = list(range(T))
    M = len(t)
    S = max(1, int(M * frac))
    res, wall = clone.pool_timesteps(range(K), a2l, gw, e, iw, t, tk, a, lam, I, I, C,
                                     sample_tris=S)
    loop = float(np.mean([r[1] for r in res]))
    solve = float(np.mean([r[2] for r in res]))
    full_wall = wall + per_core * loop * (M / S - 1.0)
    value = K / full_wall
    return {
        "value": value, "unit": "timesteps/s", "cores": C, "kind": "port",
        "host_cpu_count": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
        "cores_reason": ("--cpu-cores %d: a pool larger than the box's 16-core share per GPU, to measure "
                         "the baseline's scaling towards os.cpu_count()" % C) if cores and cores > 0 else
                        "the GPU box's CPU share is 16 cores per GPU (OMP_NUM_THREADS=16 there); "
                        "os.cpu_count() reports the whole machine",
        "sample": ("Pool(%d) x %d timesteps of the reference algorithm (lil scalar assembly, csr, "
                   "spsolve; oracle/reference_clone.py, calibrated vs the reference) on the %d-vertex "
                   "mesh; triangle loop timed on %d of %d triangles (%.1f s/step measured, "
                   "extrapolated x%.0f), spsolve on the full system (%.1f s/step); pool wall %.1f s"
                   % (C, K, len(p), S, M, loop, M / S, solve, wall)),
    }


def main():
    args = parse()
    if args.config in SMALL_JOBS:  # the whole job is one step (one batch: C1 15, S1s 97 timesteps)
        args.fixed_timesteps = args.fixed_timesteps or SMALL_JOBS[args.config]
        args.batch = min(args.batch, args.fixed_timesteps)
    self_launch(args)
    from mofhip.dist import max_over_ranks, rank_env, rank_k_range, sum_over_ranks
    rank, world, local = rank_env()
    # MOF_BENCH_REHEARSE=1: every rank on GPU 0 over gloo -- exercises the
    # N-rank path on a 1-GPU box (RCCL refuses two ranks on one GPU)
    rehearse = os.environ.get("MOF_BENCH_REHEARSE") == "1"
    # MOF_BENCH_DRYRUN=1 (CPU tests of the launcher / partition / reduction
    # path only): no GPU, no solve -- each call returns empty statistics and
    # the line says "dry_run"; never a measurement
    dry = os.environ.get("MOF_BENCH_DRYRUN") == "1"
    if rehearse:
        local = 0
    # C2 is configured fp64 (BASELINE configs[1]); C1, the 642-vertex job, runs
    # fastest as the fused one-launch fp64 solve (round 4: 0.54 vs 1.11 ms per
    # 15-timestep step for the eager mixed multigrid path)
    precision = args.precision or ("f64" if args.config in ("C1", "C2") else "mixed")

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse or dry:
            dist.init_process_group(backend="gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    from mofhip import synth

    # --- one-time mesh build (reported separately, outside the metric) -----
    p, t, n, a = synth.mesh_for_config(args.config)
    N = len(p)
    runtime_s = 0.0
    t0 = time.perf_counter()
    if dry:
        mesh, info = None, {"nblocks": 0, "ms_geometry": 0.0, "ms_pattern": 0.0}
    else:
        from mofhip import DeviceMesh, device_count
        device_count()  # the library's HIP runtime comes up once per process
        runtime_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        mesh = DeviceMesh(p, n, t, a, device=local)
        info = mesh.info()
    mesh_s = time.perf_counter() - t0

    def sync():
        if not dry:
            torch.cuda.synchronize(dev)

    # --- this rank's timesteps --------------------------------------------
    strong = args.fixed_timesteps > 0
    if strong:
        # the fixed job, split over the ranks; a step solves all of it
        k_off, k_end = rank_k_range(rank, world, 0, args.fixed_timesteps)
        K_strong = k_end - k_off
    if dry:
        # dry runs size the batch as a GPU run would, against this rank's
        # simulated free HBM (MOF_BENCH_DRYRUN_FREE_GB: one value, or one
        # per rank; default the MI355X's 288 GB) and no grid cap
        fg = os.environ.get("MOF_BENCH_DRYRUN_FREE_GB", "288").split(",")
        free_b, max_batch = float(fg[min(rank, len(fg) - 1)]) * 1e9, None
    else:
        free_b, _ = torch.cuda.mem_get_info(local)
        max_batch = info.get("max_batch")
    B, batch_note = size_batch(args.batch, N, free_b, max_batch,
                               (lambda b: K_strong + 1) if strong else
                               (lambda b: (args.warmup + args.steps) * b + 1))
    # every rank runs the smallest rank's batch, so the line rank 0 prints
    # (batch, timesteps per step) holds for every rank
    cdev = torch.device("cpu") if (rehearse or dry) else torch.device("cuda", local)
    B_rank = B
    B = int(-max_over_ranks(-B, dist, cdev))
    if B != B_rank:
        batch_note = (batch_note + "; " if batch_note else "") + \
            "batch %d reduced to %d: the smallest rank's batch" % (B_rank, B)
    if batch_note and rank == 0:
        print("[bench] " + batch_note, file=sys.stderr, flush=True)
    if strong:
        K_rank = K_strong
    else:
        K_rank = (args.warmup + args.steps) * B
        k_off, _ = rank_k_range(rank, world, 0, world * K_rank)
    # synthetic signal rows k_off .. k_off + K_rank, generated on the device:
    # (K_rank + 1) x N f64 is 7.4 GB per rank at the default C3 sizes, which
    # 8 ranks would otherwise hold in host memory
    dev = torch.device("cpu") if dry else torch.device("cuda", local)
    # the config's travelling wave (synth.wave_phase): sin(kappa phase - 0.3 k)
    phase, kappa = synth.wave_phase(args.config, p)
    phi = torch.from_numpy(np.ascontiguousarray(phase)).to(dev)
    kk = k_off + torch.arange(K_rank + 1, dtype=torch.float64, device=dev)
    I_dev = torch.empty((K_rank + 1, N), dtype=torch.float64, device=dev)
    for r0 in range(0, (K_rank + 1) if not dry else 0, 256):
        r1 = min(K_rank + 1, r0 + 256)
        I_dev[r0:r1] = torch.sin(kappa * phi[None, :] - 0.3 * kk[r0:r1, None])
    del phi, kk
    host_io = args.io == "host"
    I_host = V_host = None
    if host_io:
        I_host = I_dev.cpu().numpy()  # pageable, as S3's numpy array
        del I_dev
        I_dev = None
    else:
        V_dev = torch.empty((B, 2 * N), dtype=torch.float64, device=dev)
    tk = np.arange(K_rank + 1, dtype=np.float64)
    sync()
    precond = (args.precond or "amg") if precision == "mixed" else "jacobi"
    opts = dict(precision=precision, batch=B, rtol=args.rtol, precond=precond, inner_rtol=args.inner_rtol,
                fused={"auto": None, "on": True, "off": False}[args.fused], etol=args.etol)

    kept = []  # host V of the timed calls, freed after the clock stops (the caller keeps its result)

    def solve(a, b, timed):
        """timesteps [a, b) of this rank's rows"""
        if dry:
            return dict.fromkeys(("iterations", "failed", "recovered", "ms_spmv", "spmv_bytes", "spmv_launches",
                                  "spmv_systems", "spmv_full_launches", "ms_spmv_full", "ms_assembly",
                                  "ms_solve", "max_rel_residual", "outer_steps", "fused_launches",
                                  "ms_fused", "max_err_est"), 0) | {"systems": b - a}
        if host_io:
            V, st = mesh.solve_range(I_host, tk, a, b, args.lambda_, device=local, time_spmv=timed, **opts)
            if timed:
                kept.append(V)
            return st
        return mesh.solve_range_device(I_dev.data_ptr(), I_dev.data_ptr(), K_rank + 1, tk, a, b, args.lambda_,
                                       V_dev.data_ptr(), device=local, time_spmv=timed, **opts)

    if strong:
        # balanced batches: 625 timesteps per rank at N = 8 run as 2 x 313,
        # not 512 + 113 (a narrow tail batch pays the whole setup and
        # iteration sequence at a fraction of the width)
        nbat = max(1, -(-K_rank // B))
        B_eff = max(1, -(-K_rank // nbat))
        opts["batch"] = B_eff
        batches = [(a, min(a + B_eff, K_rank)) for a in range(0, K_rank, B_eff)]
        warm = batches[:max(1, args.warmup)] if batches else []
        if host_io:
            step_calls = [(0, K_rank)]
        else:
            step_calls = batches
        timed_calls = step_calls * args.steps
    else:
        warm = [(s * B, (s + 1) * B) for s in range(args.warmup)]
        timed = [(s * B, (s + 1) * B) for s in range(args.warmup, args.warmup + args.steps)]
        timed_calls = [(timed[0][0], timed[-1][1])] if host_io else timed
        if host_io and warm:
            warm = [(warm[0][0], warm[-1][1])]
    for a_, b_ in warm:
        solve(a_, b_, False)

    # --- timed region -------------------------------------------------------
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    agg = {"iterations": 0, "failed": 0, "recovered": 0, "ms_spmv": 0.0, "spmv_bytes": 0.0, "spmv_launches": 0,
           "spmv_systems": 0, "spmv_full_launches": 0, "ms_spmv_full": 0.0, "max_rel_residual": 0.0,
           "ms_assembly": 0.0, "ms_solve": 0.0, "systems": 0, "fused_launches": 0, "ms_fused": 0.0,
           "max_err_est": 0.0}
    for a_, b_ in timed_calls:
        st = solve(a_, b_, True)
        for k in ("iterations", "failed", "recovered", "ms_spmv", "spmv_bytes", "spmv_launches", "spmv_systems",
                  "spmv_full_launches", "ms_spmv_full", "ms_assembly", "ms_solve", "systems", "fused_launches",
                  "ms_fused"):
            agg[k] += st[k]
        agg["max_rel_residual"] = max(agg["max_rel_residual"], st["max_rel_residual"])
        agg["max_err_est"] = max(agg["max_err_est"], st["max_err_est"])
        agg["max_outer_steps"] = max(agg.get("max_outer_steps", 0), st["outer_steps"])
    sync()
    elapsed = time.perf_counter() - t0
    # parity samples: timesteps of the last timed call, its V as the timed
    # solve returned it (V_dev holds the last call's batch; host io: kept[-1])
    samples = []
    if rank == 0 and args.parity_samples > 0 and not dry and timed_calls:
        a_, b_ = timed_calls[-1]
        ks = sorted({a_ + round(q * (b_ - a_ - 1) / max(1, args.parity_samples - 1))
                     for q in range(args.parity_samples)})
        for k in ks:
            if host_io:
                Vk, I0k, I1k = kept[-1][k - a_], I_host[k], I_host[k + 1]
            else:
                Vk = V_dev[k - a_].cpu().numpy()
                I0k, I1k = I_dev[k].cpu().numpy(), I_dev[k + 1].cpu().numpy()
            samples.append((k_off + k, I0k, I1k, float(tk[k + 1] - tk[k]), Vk))
    kept.clear()
    elapsed = max_over_ranks(elapsed, dist, cdev)
    agg["failed"] = int(sum_over_ranks(agg["failed"], dist, cdev))
    agg["recovered"] = int(sum_over_ranks(agg["recovered"], dist, cdev))
    n_ts = int(sum_over_ranks(agg["systems"], dist, cdev))
    value = n_ts / elapsed
    n_local = max(1, agg["systems"])
    rank_ranges = None
    if dry and dist:
        got = [None] * world
        dist.all_gather_object(got, [k_off, k_off + K_rank, agg["systems"], B_rank, opts["batch"]])
        rank_ranges = got
    elif dry:
        rank_ranges = [[k_off, k_off + K_rank, agg["systems"], B_rank, opts["batch"]]]

    roofline = spmv_roofline(agg, info, N, precision, precond, B, args.config)

    # host-to-host leg (SURVEY.md 8(d)'s metric: host I -> host V_k, the
    # reference's submit -> join, compute_optical_flow.py:160-182), measured in
    # this invocation after the device-resident region: pageable numpy I in,
    # V into a numpy array, one mof_solve_range call per rank over
    # --host-batches batches (the drop-in's pipelined path)
    host_leg = None
    if not host_io and not dry and args.host_batches > 0:
        R = min(K_rank, args.host_batches * B)
        I_h = I_dev[:R + 1].cpu().numpy()
        mesh.solve_range(I_h, tk, 0, min(R, B), args.lambda_, device=local, **opts)  # pinned ring, slots
        if dist:
            dist.barrier()
        sync()
        th = time.perf_counter()
        Vh, sh = mesh.solve_range(I_h, tk, 0, R, args.lambda_, device=local, **opts)
        th = time.perf_counter() - th
        th = max_over_ranks(th, dist, cdev)
        nh = int(sum_over_ranks(sh["systems"], dist, cdev))
        host_leg = {"value": round(nh / th, 3), "unit": "timesteps/s", "timesteps": nh,
                    "seconds": round(th, 4), "failed": int(sum_over_ranks(sh["failed"], dist, cdev)),
                    "io": "host: pageable numpy I (T, N) in, numpy V (T-1, 2N) out, PCIe inclusive "
                          "(SURVEY.md 8(d) metric; reference timer compute_optical_flow.py:160-182)"}
        del Vh, I_h

    # extra configurations on this GPU (--legs; a 1-GPU C3 line by default:
    # F3, S1s and S1, the reference's mesh class), after the main mesh is freed
    legs, leg_jobs = [], []
    leg_names = ([] if args.legs == "none" else
                 (["F3", "S1s", "S1"] if args.config == "C3" else []) if args.legs == "auto" else
                 [x for x in args.legs.split(",") if x])
    if world > 1 or dry or host_io:
        leg_names = []
    if leg_names:
        del I_dev, V_dev
        mesh.close()
        torch.cuda.empty_cache()
        for name in leg_names:
            if name not in LEGS:
                raise SystemExit("bench.py: --legs knows %s" % ",".join(sorted(LEGS)))
            leg, mesh_l, smp = run_leg(name, args, torch, local)
            legs.append(leg)
            leg_jobs.append((mesh_l, smp))

    cpu = geom = None
    if rank == 0 and not dry and (not args.no_cpu_baseline or samples):
        import oracle
        geom = oracle.geometry(p, n, t, a)
    jobs = [(geom, t, a, args.lambda_, samples)] if samples else []
    if leg_jobs and args.parity_samples > 0:
        import oracle
        for (pl, tl, nl_, al), smp in leg_jobs:
            jobs.append((oracle.geometry(pl, nl_, tl, al), tl, al, args.lambda_, smp))
    par = parity_checks(jobs) if jobs else []
    parity = par[0] if samples else None
    for i, leg in enumerate(legs):
        leg["parity"] = par[i + (1 if samples else 0)] if args.parity_samples > 0 else None
    if rank == 0 and not args.no_cpu_baseline and not dry:
        cpu = cpu_baseline(p, t, n, a, args.lambda_, args.cpu_sample_frac, args.cpu_timesteps_per_core, geom=geom,
                           full_timesteps=args.fixed_timesteps if args.config in SMALL_JOBS else 0,
                           cores=args.cpu_cores, config=args.config)

    if rank == 0:
        line = {
            "metric": "flow timesteps/sec on 160k-vertex mesh" if args.config == "C3"
                      else "flow timesteps/sec (%s)" % args.config,
            "value": round(value, 3), "unit": "timesteps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "f32" if precision == "mixed" else "f64",
            "data": "synthetic travelling wave sin(%g phi - 0.3 k) (synth.wave_phase), dt = 1, lambda = 0.01"
                    % synth.wave_phase(args.config, p[:1])[1],
            "config": {"workload": CONFIG_NAMES[args.config], "vertices": N, "triangles": len(t),
                       "timesteps_per_step": args.fixed_timesteps if strong else world * B,
                       "timesteps_timed": n_ts, "batch": B, **({"batch_note": batch_note} if batch_note else {}),
                       "precision": precision,
                       "batch_effective": opts["batch"],
                       "precond": opts["precond"], "rtol": args.rtol,
                       "io": "host (pageable numpy I in, numpy V out; PCIe inclusive)" if host_io
                             else "device (I and V resident in HBM)",
                       "parallelism": "timestep shards x%d" % world},
            "roofline": roofline,
            "step_traffic": step_traffic("%s/%s/%s/B%d" % (args.config, precision, precond, B), value),
            "host_io": host_leg,
            "parity": parity,
            "legs": legs or None,
            "cpu_baseline": cpu,
            "solver": {"pcg_iterations_per_timestep": round(agg["iterations"] / n_local, 1),
                       "failed": agg["failed"], "recovered": agg["recovered"],
                       "max_rel_residual": agg["max_rel_residual"],
                       # the refinement's error estimate, max|d_k| |r_k+1| / |r_k|
                       # over max|V| (the stop rule's)
                       "max_err_est": agg["max_err_est"],
                       "max_refinement_steps": agg.get("max_outer_steps", 0),
                       "ms_assembly_per_timestep": round(agg["ms_assembly"] / n_local, 4),
                       "ms_solve_per_timestep": round(agg["ms_solve"] / n_local, 4),
                       "mesh_build_s": round(mesh_s, 3), "library_init_s": round(runtime_s, 3), "mesh_geometry_ms": round(info["ms_geometry"], 3),
                       "mesh_pattern_ms": round(info["ms_pattern"], 3),
                       # the one-launch fp64 solve per batch (small meshes): its
                       # launches and kernel time (no per-SpMV timing there)
                       "fused_launches": agg["fused_launches"],
                       "ms_fused_per_launch": round(agg["ms_fused"] / agg["fused_launches"], 4)
                       if agg["fused_launches"] else None},
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        # a system the first solve failed and a recovery pass repaired is a
        # solver defect on these healthy configurations (round 4: a launch that
        # skipped workgroups was hidden by the recovery) -- marked, and the run
        # exits non-zero unless --allow-recovery
        defect = None
        if agg["recovered"] > 0 or agg["failed"] > 0:
            defect = {"recovered": agg["recovered"], "failed": agg["failed"],
                      "why": "the first solve failed on systems of a healthy configuration"}
            line["defect"] = defect
        if parity is not None and parity["max_abs_err"] > parity["bar"] * max(1.0, parity["max_abs_V"]):
            line["defect"] = dict(defect or {}, parity=parity["max_abs_err"])
        for leg in legs:  # the legs' solver defects and parity, as the main line's
            lp, ls = leg.get("parity"), leg["solver"]
            bad = {}
            if ls["recovered"] or ls["failed"]:
                bad.update(recovered=ls["recovered"], failed=ls["failed"])
            if lp is not None and lp["max_abs_err"] > lp["bar"] * max(1.0, lp["max_abs_V"]):
                bad["parity"] = lp["max_abs_err"]
            if bad:
                line["defect"] = dict(line.get("defect") or {}, **{leg["config"]: bad})
        if dry:
            line["dry_run"] = True
            line["rank_ranges"] = rank_ranges
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    parity_bad = rank == 0 and "defect" in line and (
        "parity" in line["defect"] or any(isinstance(v, dict) and "parity" in v for v in line["defect"].values()))
    if rank == 0 and "defect" in line and not (args.allow_recovery and not parity_bad):
        print("[bench] defect: %s" % json.dumps(line["defect"]), file=sys.stderr, flush=True)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
