"""Per-kernel HBM rates of full launches, from a rocprofv3 kernel trace and
the FETCH_SIZE / WRITE_SIZE passes of the same bench configuration.

    python profiles/kernel_rates.py TRACE.csv FETCH.csv WRITE.csv [top]

A batch's late launches cover fewer systems (converged systems exit, the
tail runs compacted), so a kernel's mean launch mixes full and partial
work. For each kernel this takes its *full* launches on both sides:

  * bytes: the median over the PMC dispatches whose bytes (2 x FETCH_SIZE +
    WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction) are >= 0.9 x the
    kernel's largest;
  * time: the median over the trace's dispatches whose duration is >= 0.9 x
    the kernel's 95th percentile,

and reports bytes / time against the 8 TB/s HBM3E peak, with each kernel's
share of the trace's GPU time. (The PMC passes run their own bench command,
so dispatches are matched by kernel, not one by one; the PMC run's own
timestamps give a second, counter-perturbed time column.)
"""
import csv
import re
import statistics
import sys
from collections import defaultdict

PEAK = 8.0e12


def kname(raw):
    m = re.search(r"(k_\w+(<[^>]*>)?)", raw)
    return m.group(1) if m else raw[:40]


def pmc(path, counter, scale):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out[kname(r["Kernel_Name"])].append(
                (float(r["Counter_Value"]) * 1024.0 * scale, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
    return out


def main():
    trace, fetch, write = sys.argv[1:4]
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    dur = defaultdict(list)
    for r in csv.DictReader(open(trace)):
        dur[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    total = sum(sum(v) for v in dur.values())
    f, w = pmc(fetch, "FETCH_SIZE", 2.0), pmc(write, "WRITE_SIZE", 1.0)
    rows = []
    for k, ds in dur.items():
        if k not in f:
            continue
        fb = [b for b, _ in f[k]]
        wb = [b for b, _ in w.get(k, [])] or [0.0] * len(fb)
        n = min(len(fb), len(wb))
        tot = [fb[i] + wb[i] for i in range(n)]
        big = max(tot)
        full_i = [i for i in range(n) if tot[i] >= 0.9 * big]
        bytes_full = statistics.median(tot[i] for i in full_i)
        t_pmc = statistics.median(f[k][i][1] for i in full_i)
        p95 = sorted(ds)[int(0.95 * (len(ds) - 1))]
        t_full = statistics.median(d for d in ds if d >= 0.9 * p95)
        rows.append((sum(ds) / total, k, len(ds), t_full, bytes_full, bytes_full / t_full, t_pmc))
    rows.sort(reverse=True)
    print("| kernel | share of GPU time | launches | full launch (trace) | HBM bytes (PMC, full) | TB/s | of 8 TB/s | PMC-run time |")
    print("|---|---|---|---|---|---|---|---|")
    for share, k, n, t, b, rate, tp in rows[:top]:
        print("| `%s` | %.1f %% | %d | %.0f µs | %.2f GB | %.2f | %.2f | %.0f µs |"
              % (k, 100 * share, n, t * 1e6, b / 1e9, rate / 1e12, rate / PEAK, tp * 1e6))


if __name__ == "__main__":
    main()
