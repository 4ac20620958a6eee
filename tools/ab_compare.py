"""Compare per-kernel average durations across ab_prof.sh runs:
    python tools/ab_compare.py gpurun_out/abprof_TAG [kernel substrings...]"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
pats = sys.argv[2:]
runs = {}
for d in sorted(glob.glob(os.path.join(root, "*"))):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        continue
    rows = {r["Name"]: r for r in csv.DictReader(open(f[0]))}
    try:
        line = json.loads(open(os.path.join(d, "bench.json")).readline())
        val = line["value"]
    except Exception:
        val = None
    runs[os.path.basename(d)] = (rows, val)
names = sorted({n for rows, _ in runs.values() for n in rows})
print("%-44s" % "kernel" + "".join("%14s" % k for k in runs))
print("%-44s" % "value (ts/s)" + "".join("%14s" % (v if v else "-") for _, v in runs.values()))
for n in names:
    short = n.replace("void mof::(anonymous namespace)::", "").replace("mof::(anonymous namespace)::", "")
    if pats and not any(p in short for p in pats):
        continue
    vals = []
    for rows, _ in runs.values():
        r = rows.get(n)
        vals.append("%14.1f" % (float(r["AverageNs"]) / 1e3) if r else "%14s" % "-")
    print("%-44s" % short[:44] + "".join(vals))
