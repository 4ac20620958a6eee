"""Print a rocprofv3 kernel_stats CSV as a per-kernel table (time per call,
share of GPU time), kernels in descending total time.

    python profiles/stats_table.py <run_kernel_stats.csv> [top]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = r["Name"].replace("mof::(anonymous namespace)::", "").replace("void ", "")
        print("%-44s %6s %10.1f us %5.1f%%" % (name[:44], r["Calls"], float(r["AverageNs"]) / 1e3,
                                              100 * float(r["TotalDurationNs"]) / tot))
    print("total %.1f ms" % (tot / 1e6))


if __name__ == "__main__":
    main()
