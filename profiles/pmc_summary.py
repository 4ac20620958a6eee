"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

    python profiles/pmc_summary.py <fetch_csv> <write_csv> <out.json> <key> [timesteps]

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE;
WRITE_SIZE is exact for 16-B-per-lane stores. Both counters are in KiB.
The two counters come from separate rocprofv3 --pmc passes of the same
bench command. `key` names the bench configuration the passes ran
(bench.py reads the entry whose key matches its own run). With the number
of timesteps the profiled run solved, the entry also records the whole
run's HBM bytes per timestep (every dispatch's counters summed) and their
rate over the summed kernel time.
"""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        vals[m.group(1) if m else r["Kernel_Name"][:40]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: statistics.median(v) for k, v in vals.items()}


def main():
    fetch_csv, write_csv, out, key = sys.argv[1:5]
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        rd = 2.0 * f.get(k, 0.0)
        kernels[k] = {"fetch_size_bytes": f.get(k), "read_bytes_corrected": rd,
                      "write_bytes": w.get(k), "hbm_bytes_per_launch": rd + w.get(k, 0.0)}
    try:
        data = json.load(open(out))
    except (OSError, ValueError):
        data = {}
    data[key] = {"source": [fetch_csv, write_csv], "kernels": kernels}
    if len(sys.argv) > 5:
        tot_b = tot_t = 0.0
        for path, counter, scale in ((fetch_csv, "FETCH_SIZE", 2.0), (write_csv, "WRITE_SIZE", 1.0)):
            for r in csv.DictReader(open(path)):
                if r["Counter_Name"] == counter:
                    tot_b += float(r["Counter_Value"]) * 1024.0 * scale
                    tot_t += 0.5 * (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        ts = int(sys.argv[5])
        data[key]["run"] = {"timesteps": ts, "hbm_bytes": tot_b, "kernel_s": tot_t,
                            "hbm_bytes_per_timestep": tot_b / ts, "tb_per_s": tot_b / tot_t / 1e12}
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 2) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
