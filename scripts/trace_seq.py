#!/usr/bin/env python3
"""Print a rocprofv3 kernel trace as a timeline: per dispatch the start
offset, duration and the gap since the previous dispatch ended (us).
    python scripts/trace_seq.py run_kernel_trace.csv [first] [count]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows)
t0 = int(rows[first]["Start_Timestamp"]) if rows else 0
prev = None
for r in rows[first:first + count]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"orcg::\(anonymous namespace\)::", "", r["Kernel_Name"])
    name = re.sub(r"\(.*", "", name)[:60]
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print("%9.1f %8.1f %8.1f  %-60s grid %s wg %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, name, r["Grid_Size_X"],
                                                      r["Workgroup_Size_X"]))
    prev = e
