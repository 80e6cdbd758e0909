#!/usr/bin/env python3
"""Markdown table of a gpu_session.sh `sweep2` run (gpurun_out/sw_*.log):
per stream shape, the default's time and algorithmic GB/s, every pinned
instance's GB/s and the copy references."""
import glob
import json
import os
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
ORDER = ["random_64", "random_48", "random_13", "random_8", "random_1", "delta_12", "patched_12", "repeat_12",
         "repeat_40", "repeat_64", "shortdirect_16", "shortdirect_64", "shortmix_32"]
rows, cols = {}, []
for p in glob.glob(os.path.join(OUT, "sw_*.log")):
    name = os.path.basename(p)[3:-4]
    d = {}
    for ln in open(p):
        if ln.startswith("{"):
            j = json.loads(ln)
            d[str(j["variant"])] = j
            if str(j["variant"]) not in cols:
                cols.append(str(j["variant"]))
    rows[name] = d
var = sorted([c for c in cols if c.isdigit() and c != "0"], key=int)
refs = [c for c in cols if not c.isdigit()]
print("| data | W | stream B/value | v0 ms | v0 GB/s | " + " | ".join("v%s GB/s" % c for c in var) + " | "
      + " | ".join("%s GB/s" % c for c in refs) + " |")
print("|" + "---|" * (5 + len(var) + len(refs)))
for name in ORDER + sorted(set(rows) - set(ORDER)):
    if name not in rows:
        continue
    d = rows[name]
    kind, bits = name.rsplit("_", 1)
    any_row = next(iter(d.values()))
    cells = [kind, bits, "%.3f" % any_row["stream_B_per_value"]]
    v0 = d.get("0")
    cells += ["%.4f" % v0["ms_median"], "%.0f" % v0["GBps"]] if v0 else ["", ""]
    cells += ["%.0f" % d[c]["GBps"] if c in d else "" for c in var + refs]
    print("| " + " | ".join(cells) + " |")
