#!/usr/bin/env python3
"""bench_rows.py -- measurement of the SURVEY.md §8(f) rows on MI355X.

One JSON line per row, each on the C3 mesh (163,842 vertices, 327,680
triangles) with a CPU baseline of the reference's own path timed on a
bounded sample and scaled:

  epilogue       process_V_k + speed (find_singularity_point.py:28-69,
                 S3…py:130-132): mof_velocity_vectors on K fields resident
                 in HBM vs the reference's Python loops (oracle.process_V_k);
  csv            V_k CSV write (reshape_and_save_data) / potentials CSV read
                 (load_potentials): libmofhip's threaded host code vs pandas,
                 bytes / values checked identical;
  singularities  find_singularity_points for K fields (mof_singularities)
                 vs the reference's per-triangle loop (oracle.singularities).

    python bench_rows.py [--rows epilogue,csv,singularities] [--K 64]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "manifold-based-optical-flow-method_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
HBM_PEAK_GBS = 8000.0


def c3():
    from mofhip import synth
    p, t, n, a = synth.mesh_for_config("C3")
    return p, t


def tangent_fields(p, K, seed=0):
    rng = np.random.default_rng(seed)
    nn = p / np.linalg.norm(p, axis=1, keepdims=True)
    out = np.empty((K, len(p), 3))
    for k in range(K):
        f, ph = rng.uniform(0.2, 0.6, 3), rng.uniform(0, 6.28, 3)
        amb = np.stack([np.sin(f[0] * p[:, 1] + ph[0]), np.cos(f[1] * p[:, 2] + ph[1]),
                        np.sin(f[2] * p[:, 0] + ph[2])], axis=1)
        out[k] = amb - np.sum(amb * nn, axis=1, keepdims=True) * nn
    return out


def row_epilogue(K, reps=20):
    import torch
    import oracle
    from mofhip.epilogue import velocity_vectors_device
    p, t = c3()
    N = len(p)
    rng = np.random.default_rng(1)
    e = rng.standard_normal((N, 2, 3))
    V = rng.standard_normal((K, 2 * N))
    dev = torch.device("cuda", 0)
    de, dV = torch.from_numpy(e).to(dev), torch.from_numpy(V).to(dev)
    dc = torch.empty((K, N, 3), dtype=torch.float64, device=dev)
    ds = torch.empty((K, N), dtype=torch.float64, device=dev)
    run = lambda: velocity_vectors_device(de.data_ptr(), dV.data_ptr(), N, K, dc.data_ptr(), ds.data_ptr())
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    nbytes = K * N * (16 + 24 + 8) + N * 48  # V in, V_coord + speed out, e once
    # correctness on two fields against the reference loop restatement
    sub = 2000
    t0 = time.perf_counter()
    ref = oracle.process_V_k(np.concatenate([V[:2, :sub], V[:2, N:N + sub]], axis=1), e[:sub])
    cpu_s = (time.perf_counter() - t0) / (2 * sub) * N  # per field, scaled to N vertices
    same = np.array_equal(dc[:2, :sub].cpu().numpy(), ref)
    return {"row": "(f)1 epilogue process_V_k + V_c", "K": K, "N": N,
            "value": round(K / dt, 1), "unit": "fields/s", "ms_per_launch": round(dt * 1e3, 4),
            "roofline": {"bound": "hbm", "achieved": round(nbytes / dt / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(nbytes / dt / 1e9 / HBM_PEAK_GBS, 3)},
            "bit_identical_to_reference_loop": bool(same),
            "cpu_baseline": {"value": round(1.0 / cpu_s, 4), "unit": "fields/s", "cores": 1, "kind": "port",
                             "sample": "reference loop (oracle.process_V_k) on 2 fields x %d vertices, "
                                       "scaled to %d" % (sub, N)}}


def row_csv(rows=64, threads=0, sample=4):
    import pandas as pd
    from mofhip import csvio
    p, t = c3()
    cols = 2 * len(p)
    V = np.random.default_rng(0).standard_normal((rows, cols)) * 0.7
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as d:
        ours, theirs = os.path.join(d, "mof.csv"), os.path.join(d, "pd.csv")
        t0 = time.perf_counter()
        csvio.write_csv(ours, V, threads=threads)
        t_w = time.perf_counter() - t0
        size = os.path.getsize(ours)
        t0 = time.perf_counter()
        pd.DataFrame(V[:sample]).to_csv(theirs)
        t_pw = (time.perf_counter() - t0) * rows / sample
        with open(ours, "rb") as f:
            same_bytes = f.read(os.path.getsize(theirs)) == open(theirs, "rb").read()
        t0 = time.perf_counter()
        back = csvio.read_csv(ours, threads=threads)
        t_r = time.perf_counter() - t0
        t0 = time.perf_counter()
        ref = pd.read_csv(theirs, sep=",", header="infer", index_col=0).values
        t_pr = (time.perf_counter() - t0) * rows / sample
        same_vals = np.array_equal(back[:sample].view(np.int64), ref.view(np.int64))
    nth = threads or int(os.environ.get("MOF_IO_THREADS") or os.environ.get("OMP_NUM_THREADS") or os.cpu_count())
    return {"row": "(f)2 S3 CSV I/O", "rows": rows, "cols": cols, "csv_bytes": size, "threads": min(nth, 64),
            "unit": "MB/s of CSV text",
            "write": {"value": round(size / t_w / 1e6, 1), "s": round(t_w, 3), "speedup_vs_pandas": round(t_pw / t_w, 1),
                      "bytes_identical_to_pandas": bool(same_bytes)},
            "read": {"value": round(size / t_r / 1e6, 1), "s": round(t_r, 3), "speedup_vs_pandas": round(t_pr / t_r, 1),
                     "values_identical_to_pandas": bool(same_vals)},
            "cpu_baseline": {"write_s": round(t_pw, 2), "read_s": round(t_pr, 2), "cores": 1, "kind": "reference",
                             "sample": "pandas to_csv / read_csv (the reference's calls) on %d rows, scaled" % sample}}


def row_singularities(K, reps=5, eps=5e-3):
    import torch
    import oracle
    from mofhip import singular
    p, t = c3()
    V = tangent_fields(p, K) + 1e-3 * np.random.default_rng(2).standard_normal((K, len(p), 3))
    singular.singularity_lists(p, t, V[:1], eps)  # warm
    t0 = time.perf_counter()
    for _ in range(reps):
        vmax, verts, tris = singular.singularity_lists(p, t, V, eps)
    dt = (time.perf_counter() - t0) / reps  # includes host<->device copies
    sel = np.arange(0, len(t), 331)
    t0 = time.perf_counter()
    ovmax, ovf, otf, olm = oracle.singularities(p, t[sel], V[0], eps)
    cpu_s = (time.perf_counter() - t0)
    cpu_field_s = cpu_s / len(sel) * len(t)  # the per-triangle loop dominates
    tf0 = np.zeros(len(t), bool)
    tf0[tris[0][0]] = True
    agree = bool(vmax[0] == ovmax and np.array_equal(verts[0], np.flatnonzero(ovf)) and
                 (tf0[sel] != otf).sum() <= 2)
    return {"row": "(f)4 find_singularity_points", "K": K, "N": len(p), "M": len(t), "eps": eps,
            "value": round(K / dt, 2),
            "unit": "fields/s (host V in, the reference's lists out: device-compacted, PCIe included)",
            "zeros_found_per_field": round(float(sum(len(v) for v in verts) + sum(len(x[0]) for x in tris)) / K, 1),
            "agrees_with_oracle_on_sample": agree,
            "cpu_baseline": {"value": round(1.0 / cpu_field_s, 5), "unit": "fields/s", "cores": 1, "kind": "port",
                             "sample": "oracle.singularities (the reference's per-triangle loop with "
                                       "np.linalg.lstsq) on %d of %d triangles, scaled" % (len(sel), len(t))}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="epilogue,csv,singularities")
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    for r in args.rows.split(","):
        if r == "epilogue":
            print(json.dumps(row_epilogue(args.K)), flush=True)
        elif r == "csv":
            print(json.dumps(row_csv(threads=args.threads)), flush=True)
        elif r == "singularities":
            print(json.dumps(row_singularities(min(args.K, 32))), flush=True)
        else:
            raise SystemExit("unknown row " + r)


if __name__ == "__main__":
    main()
