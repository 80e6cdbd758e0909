#!/usr/bin/env python3
"""Copy a measurement pass (gpurun_out of scripts/gpu_r4_final_[ab].sh) into
profiles/<round>/ under stable names: the bench line, rocprof kernel stats of
bench.py and of the file workloads, the PMC passes, bench_file JSON lines,
per-stream phase profiles and the sweep table.
    python scripts/collect_profiles.py SRC_DIR profiles/r04"""
import glob
import json
import os
import shutil
import subprocess
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)


def last_json(path):
    for ln in reversed(open(path).read().splitlines()):
        if ln.startswith("{"):
            return ln
    return None


def cp(a, b):
    if os.path.exists(os.path.join(src, a)):
        shutil.copy(os.path.join(src, a), os.path.join(dst, b))
        print("copied", a, "->", b)


if os.path.exists(os.path.join(src, "bench.log")):
    ln = last_json(os.path.join(src, "bench.log"))
    if ln:
        open(os.path.join(dst, "bench_line.json"), "w").write(ln + "\n")
cp("prof/run_kernel_stats.csv", "rocprof_kernel_stats_bench.csv")
cp("pmc_fetch/run_counter_collection.csv", "rocprof_pmc_fetch_size.csv")
cp("pmc_write/run_counter_collection.csv", "rocprof_pmc_write_size.csv")
cp("tr_c5/run_kernel_stats.csv", "rocprof_kernel_stats_c5.csv")
cp("tr_c4/run_kernel_stats.csv", "rocprof_kernel_stats_c4.csv")
cp("t_all.log", "pytest_gpu_final.log")
for w in ("c1", "c4", "c5", "c4_125m"):
    p = os.path.join(src, "bf_%s.log" % w)
    if os.path.exists(p):
        ln = last_json(p)
        if ln:
            open(os.path.join(dst, "bench_file_%s.json" % w), "w").write(ln + "\n")
for w in ("c5",):
    p = os.path.join(src, "wl_%s.log" % w)
    if os.path.exists(p):
        ln = last_json(p)
        if ln:
            open(os.path.join(dst, "bench_workload_%s.json" % w), "w").write(ln + "\n")
for p in glob.glob(os.path.join(src, "ph_*.log")):
    rows = [ln for ln in open(p).read().splitlines() if ln.startswith("{")]
    if rows:
        open(os.path.join(dst, os.path.basename(p)[:-4] + ".jsonl"), "w").write("\n".join(rows) + "\n")
if glob.glob(os.path.join(src, "sw_*.log")):
    here = os.path.dirname(os.path.abspath(__file__))
    md = subprocess.check_output([sys.executable, os.path.join(here, "sweep_table.py"), src], text=True)
    open(os.path.join(dst, "sweep.md"), "w").write(md)
print(json.dumps(sorted(os.listdir(dst))))
