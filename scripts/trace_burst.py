#!/usr/bin/env python3
"""One decode burst of a rocprofv3 kernel trace as a timeline (start, duration,
queue, kernel, grid): bursts are separated by > 1 ms of GPU idle time.
    python scripts/trace_burst.py run_kernel_trace.csv [burst index, default -2]"""
import csv
import re
import sys

r = list(csv.DictReader(open(sys.argv[1])))
ev = sorted(r, key=lambda x: int(x["Start_Timestamp"]))
bursts, cur = [], [ev[0]]
for e in ev[1:]:
    if int(e["Start_Timestamp"]) - max(int(c["End_Timestamp"]) for c in cur) > 1_000_000:
        bursts.append(cur)
        cur = [e]
    else:
        cur.append(e)
bursts.append(cur)
b = bursts[int(sys.argv[2]) if len(sys.argv) > 2 else -2]
t0 = int(b[0]["Start_Timestamp"])
for x in b:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    n = re.sub(r"orcg::\(anonymous namespace\)::", "", x["Kernel_Name"])
    n = re.sub(r"\(.*", "", n)[:50]
    print("%8.1f %7.1f q%s %-50s %s" % ((s - t0) / 1e3, (e - s) / 1e3, x["Queue_Id"], n, x["Grid_Size_X"]))
