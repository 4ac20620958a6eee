"""Recompute a bench line's SpMV roofline from a rocprofv3 kernel summary.

    python profiles/roofline_check.py <bench_line.json> <kernel_trace.csv|kernel_stats.csv> [pmc key]

bench.py charges every timed launch of k_pcg_spmv with the systems it
processed (bytes_per_launch = bytes_per_system x systems_per_launch +
the shared column indices of every launch with work, averaged over the
timed launches) and times each launch with events stamped by the kernel's
own dispatch packet. This script divides the same bytes by rocprof's
average duration of the same launches -- from a kernel trace, the SpMV
launches of the timed region: every batch starts with one `k_gather_I`
launch, so the timed batches are those from batch `warmup * b` to batch
`(warmup + steps) * b` (b batches per step), and the SpMV launches between
those two `k_gather_I` starts are the timed ones (the host-IO leg and the
parity solves after the clock are excluded); from a kernel summary, all
SpMV launches (both template instances) -- and prints both fractions of the
8 TB/s peak, and the full-launch durations side by side.
Since round 5's early convergence mark, a refinement step whose systems were
marked by its last queued iteration ends with one more SpMV launch that the
bench does not time (the deferred x += alpha p only, every system retired
from the SpMV work): in a trace those are the region's shortest SpMV
launches beyond the line's `launches`, and they are left out (reported as
`untimed_x_update_launches`).
With a pmc_traffic.json key it also prints measured HBM bytes per launch
(PMC, gfx950 FETCH_SIZE doubled) next to the algorithmic bytes.
"""
import csv
import json
import sys

PEAK_GBS = 8000.0


def timed_launches(rows, line, prefix):
    """Durations (us) of the SpMV launches inside the bench line's timed
    region of a rocprofv3 kernel trace, bounded by the batches' k_gather_I
    launches (see the module docstring)."""
    cfg = line["config"]
    per_step = -(-int(cfg["timesteps_per_step"]) // int(cfg.get("batch_effective") or cfg["batch"]))
    first, last = line["warmup"] * per_step, (line["warmup"] + line["steps"]) * per_step
    marks = sorted(int(r["Start_Timestamp"]) for r in rows if "k_gather_I(" in r["Kernel_Name"])
    if len(marks) < last:
        raise SystemExit("trace holds %d batches, the line's timed region ends at batch %d" % (len(marks), last))
    t0 = marks[first]
    t1 = marks[last] if len(marks) > last else float("inf")
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
            if prefix in r["Kernel_Name"] and t0 <= int(r["Start_Timestamp"]) < t1]


def main():
    line = json.loads(open(sys.argv[1]).readline())
    rl = line["roofline"]
    prefix = "k_pcg_spmv<%s" % ("float" if line["dtype"] == "f32" else "double")  # both instances: the last launches
    rows = list(csv.DictReader(open(sys.argv[2])))
    full_us = None
    if rows and "Start_Timestamp" in rows[0]:
        d = timed_launches(rows, line, prefix)
        extra = max(0, len(d) - int(rl.get("launches") or len(d)))
        d = sorted(d)[extra:]
        n, us = len(d), sum(d) / len(d)
        full = sorted(d)[-rl["full_launches"]:] if rl.get("full_launches") else []
        full_us = sum(full) / len(full) if full else None
    else:
        n = tot = 0.0
        for r in rows:
            if prefix in r["Name"]:
                n += float(r["Calls"])
                tot += float(r["TotalDurationNs"])
        us = tot / n / 1e3
    frac = rl["bytes_per_launch"] / (us * 1e-6) / 1e9 / PEAK_GBS
    out = {"bench_frac": rl["frac"], "bench_us_per_launch": rl["us_per_launch"],
           "rocprof_us_per_launch": round(us, 2), "rocprof_launches": int(n),
           "rocprof_frac": round(frac, 4), "rel_diff": round(frac / rl["frac"] - 1.0, 4),
           "bytes_per_launch": rl["bytes_per_launch"], "systems_per_launch": rl["systems_per_launch"],
           "bytes_per_system": rl["bytes_per_system"],
           "bench_us_per_full_launch": rl.get("us_per_full_launch"),
           "rocprof_us_per_full_launch": round(full_us, 2) if full_us else None}
    if rows and "Start_Timestamp" in rows[0]:
        out["untimed_x_update_launches"] = extra
    if len(sys.argv) > 3:
        key = sys.argv[3]
        ent = json.load(open(sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_traffic.json"))[key]
        base = "k_pcg_spmv<float, false" if line["dtype"] == "f32" else "k_pcg_spmv<double, false"
        names = [n for n in ent["kernels"] if n.startswith(base)]  # + template flags (bf16 z)
        out["pmc_hbm_bytes_median_launch"] = max(ent["kernels"][n]["hbm_bytes_per_launch"] for n in names)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
