#!/usr/bin/env python3
"""bench_io.py -- SURVEY.md §8(f)2: the S3 CSV files, libmofhip vs pandas.

Writes a V_k block of the C3 run (B timesteps x 2N = 327,684 planar values,
synthetic travelling-wave magnitudes) the way S3 does
(``reshape_and_save_data`` -> ``pd.DataFrame(...).to_csv``,
compute_optical_flow.py:314-320) and reads a potentials file the way
``load_potentials`` does (``pd.read_csv(..., index_col=0).values``,
:203-207), with libmofhip's threaded writer/reader and with pandas (timed
on a row sample and scaled). Checks the bytes / values are identical and
prints one JSON line: MB/s of CSV text and the speedup over pandas.

    python bench_io.py [--rows 64] [--cols 327684] [--threads 0] [--sample 4]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--cols", type=int, default=2 * 163842)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--sample", type=int, default=4, help="rows pandas is timed on")
    args = ap.parse_args()
    import pandas as pd
    from mofhip import csvio

    rng = np.random.default_rng(0)
    V = rng.standard_normal((args.rows, args.cols)) * 0.7
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as d:
        ours, theirs = os.path.join(d, "mof.csv"), os.path.join(d, "pd.csv")
        t0 = time.perf_counter()
        csvio.write_csv(ours, V, threads=args.threads)
        t_w = time.perf_counter() - t0
        size = os.path.getsize(ours)
        s = min(args.sample, args.rows)
        t0 = time.perf_counter()
        pd.DataFrame(V[:s]).to_csv(theirs)
        t_pw = (time.perf_counter() - t0) * args.rows / s
        # bytes identical on the sampled rows (header + first s rows)
        with open(ours, "rb") as f:
            head = f.read(os.path.getsize(theirs))
        same_bytes = head == open(theirs, "rb").read()

        t0 = time.perf_counter()
        back = csvio.read_csv(ours, threads=args.threads)
        t_r = time.perf_counter() - t0
        t0 = time.perf_counter()
        ref = pd.read_csv(theirs, sep=",", header="infer", index_col=0).values
        t_pr = (time.perf_counter() - t0) * args.rows / s
        same_vals = np.array_equal(back[:s].view(np.int64), ref.view(np.int64))
    threads = args.threads or int(os.environ.get("MOF_IO_THREADS") or os.environ.get("OMP_NUM_THREADS")
                                  or os.cpu_count())
    print(json.dumps({
        "metric": "S3 V_k CSV write / potentials CSV read throughput",
        "unit": "MB/s of CSV text", "rows": args.rows, "cols": args.cols,
        "csv_bytes": size, "threads": min(threads, 64),
        "write": {"value": round(size / t_w / 1e6, 1), "s": round(t_w, 3),
                  "pandas_s_extrapolated": round(t_pw, 2), "speedup": round(t_pw / t_w, 1),
                  "bytes_identical_to_pandas": bool(same_bytes)},
        "read": {"value": round(size / t_r / 1e6, 1), "s": round(t_r, 3),
                 "pandas_s_extrapolated": round(t_pr, 2), "speedup": round(t_pr / t_r, 1),
                 "values_identical_to_pandas": bool(same_vals)},
        "pandas_sample_rows": s,
    }))


if __name__ == "__main__":
    main()
