#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats run: name, calls, total ms, average us."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
rows = list(csv.DictReader(open(path)))
print("total kernel ms %.3f" % (sum(float(r["TotalDurationNs"]) for r in rows) / 1e6))
for r in rows[:top]:
    print("%-78s %5s %9.3f %9.1f" % (r["Name"][:78], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
                                     float(r["AverageNs"]) / 1e3))
