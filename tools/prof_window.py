#!/usr/bin/env python3
"""Kernel statistics of the LAST N launches of each kernel matching a pattern in a rocprofv3 kernel trace (the timed
steps of a bench run, without its warm-up launches), in run_kernel_stats.csv's columns.

  tools/prof_window.py gpurun_out/prof_driver/run_kernel_trace.csv k_fused 20 > profiles/r05_kernel_stats_timed.csv
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path, pattern, last = sys.argv[1], sys.argv[2], int(sys.argv[3])
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if pattern in r["Kernel_Name"]:
            per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev"])
    for name, d in per.items():
        d = d[-last:]
        w.writerow([name, len(d), sum(d), sum(d) / len(d), min(d), max(d), statistics.pstdev(d)])


if __name__ == "__main__":
    main()
