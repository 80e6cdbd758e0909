#!/usr/bin/env python3
"""Fold a gpu_session.sh `prof pmc` run (gpurun_out/) into committed
artifacts: profiles/<round>/ copies of the rocprofv3 --stats summaries and
profiles/pmc_rlev2_decode.json (per-launch HBM bytes that bench.py reports as
roofline.traffic).

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are in KB; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced streaming read (the decoder's `buffer_load ... lds`), so it is
doubled; WRITE_SIZE is taken as is (the decoder writes 8 B/lane; the
per-launch figure agrees with the 8N algorithmic bytes exactly).
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "rlev2_tiled_kernel"


def counter(path, name, kernel):
    """Per-launch values of the full-column launches (the copy-inclusive leg
    also launches the kernel on row-group chunks, a tenth of the bytes each)."""
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Kernel_Name"] == kernel and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    top = max(vals)
    return [v for v in vals if v >= 0.5 * top]


def dominant(stats_csv):
    """The rlev2_tiled_kernel instance with the most time (the default
    launches a serial instance and the queue drain)."""
    best = None
    with open(stats_csv) as f:
        for row in csv.DictReader(f):
            if KERNEL in row["Name"] and (best is None or float(row["TotalDurationNs"]) > float(best["TotalDurationNs"])):
                best = row
    return best


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    if not (rnd.startswith("r") and rnd[1:].isdigit()):
        sys.exit("usage: summarize_profiles.py rNN   (folds gpurun_out/{prof,pmc_fetch,pmc_write} into profiles/rNN)")
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for sub, name in [("prof/run_kernel_stats.csv", "rocprof_kernel_stats_bench.csv"),
                      ("pmc_fetch/run_counter_collection.csv", "rocprof_pmc_fetch_size.csv"),
                      ("pmc_write/run_counter_collection.csv", "rocprof_pmc_write_size.csv")]:
        p = os.path.join(src, sub)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, name))
    row = dominant(os.path.join(src, "prof/run_kernel_stats.csv"))
    kernel = row["Name"]
    fetch = counter(os.path.join(src, "pmc_fetch/run_counter_collection.csv"), "FETCH_SIZE", kernel)
    write = counter(os.path.join(src, "pmc_write/run_counter_collection.csv"), "WRITE_SIZE", kernel)
    f_kb, w_kb = statistics.median(fetch), statistics.median(write)
    read_b = 2 * f_kb * 1024
    write_b = w_kb * 1024
    stats = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
             "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}
    out = {
        "kernel": kernel,
        "command": "python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify (C2: 1e8 rows W=64)",
        "launches": len(fetch),
        "FETCH_SIZE_KB_median": f_kb,
        "WRITE_SIZE_KB_median": w_kb,
        "read_bytes_per_launch": int(read_b),
        "write_bytes_per_launch": int(write_b),
        "hbm_bytes_per_launch": int(read_b + write_b),
        "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KB x1024",
        "kernel_stats": stats,
        "round": rnd,
    }
    with open(os.path.join(ROOT, "profiles", "pmc_rlev2_decode.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
