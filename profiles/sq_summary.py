"""Summarise one rocprofv3 SQ-counter pass (tools/pmc_issue.sh) per kernel.

    python profiles/sq_summary.py <run_counter_collection.csv> <out.csv>

Per kernel: the counters summed over its dispatches, VALU instructions per
wave, and the shares of the summed wave cycles spent issuing VALU / any
instruction, waiting on an instruction dependency (SQ_WAIT_INST_ANY) and
waiting on anything (memory, barriers: SQ_WAIT_ANY).
"""
import csv
import re
import sys
from collections import defaultdict

C = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
     "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"]


def main():
    src, out = sys.argv[1:3]
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(src)):
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    rows = sorted(tot, key=lambda k: -tot[k]["SQ_WAVE_CYCLES"])
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches"] + C + ["valu_insts_per_wave", "active_valu_pct", "active_any_pct",
                                                  "wait_inst_any_pct", "wait_any_pct"])
        for k in rows:
            t = tot[k]
            wc = t["SQ_WAVE_CYCLES"] or 1.0
            w.writerow([k, len(disp[k])] + [int(t[c]) for c in C] + [
                round(t["SQ_INSTS_VALU"] / max(t["SQ_WAVES"], 1.0), 1),
                round(100 * t["SQ_ACTIVE_INST_VALU"] / wc, 2), round(100 * t["SQ_ACTIVE_INST_ANY"] / wc, 2),
                round(100 * t["SQ_WAIT_INST_ANY"] / wc, 2), round(100 * t["SQ_WAIT_ANY"] / wc, 2)])


if __name__ == "__main__":
    main()
