"""Per-kernel totals from a rocprofv3 rocpd database (the default output
format: run_results.db): name, calls, total ms, mean us, share.

    python tools/rocpd_stats.py DIR_OR_DB [top] [filter]"""
import collections
import os
import re
import sqlite3
import sys


def kname(raw):
    m = re.search(r"(k_\w+(<[^>]*>)?|__amd_\w+)", raw)
    return m.group(1) if m else raw[:40]


def load(path):
    db = os.path.join(path, "run_results.db") if os.path.isdir(path) else path
    c = sqlite3.connect(db)
    acc = collections.defaultdict(list)
    for name, dur in c.execute("select name, duration from kernels"):
        acc[kname(name)].append(dur * 1e-3)  # us
    return acc


def main():
    acc = load(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    flt = sys.argv[3] if len(sys.argv) > 3 else ""
    tot = sum(sum(v) for v in acc.values())
    rows = sorted(((sum(v), k, len(v)) for k, v in acc.items() if flt in k), reverse=True)
    for s, k, n in rows[:top]:
        print("%-40s %6d calls %10.2f ms  mean %9.1f us  %5.1f %%" % (k, n, s / 1e3, s / n, 100 * s / tot))


if __name__ == "__main__":
    main()
