#!/usr/bin/env python3
"""Print the results a gpu_session / bench run left under gpurun_out/: the
pytest tail, sweep rows (variant, ms, GB/s) and file-bench lines."""
import glob
import json
import os
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"


def lines(p):
    try:
        with open(p) as f:
            return f.read().splitlines()
    except OSError:
        return []


for p in sorted(glob.glob(os.path.join(OUT, "pt*.log"))):
    print(p, *lines(p)[-2:], sep="\n  ")
for p in sorted(glob.glob(os.path.join(OUT, "sw_*.log"))):
    rows = []
    for ln in lines(p):
        if ln.startswith("{"):
            d = json.loads(ln)
            rows.append("%s:%.4f/%.0f" % (d["variant"], d["ms_median"], d["GBps"]))
    print(os.path.basename(p)[3:-4].ljust(16), " ".join(rows))
for p in sorted(glob.glob(os.path.join(OUT, "*.log"))):
    for ln in lines(p):
        if ln.startswith("{") and '"workload"' in ln:
            d = json.loads(ln)
            if "phases_s_summed_over_stripes" in d:
                print(os.path.basename(p), "wall", d["wall_s"], d["phases_s_summed_over_stripes"], d["rle_streams"])
            else:
                print(os.path.basename(p), ln[:400])
