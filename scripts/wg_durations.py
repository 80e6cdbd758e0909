#!/usr/bin/env python3
"""Per-workgroup durations of the union RLEv2 instance on one stripe of a
workload file (profiling build: ORCG_LIB=liborcgpu_prof.so, built with
ORCG_PHASE_PROF=1 python -m orc_amd.build). Prints the distribution of
workgroup wall-clock times (100 MHz ticks -> us) of the stripe's last union
launch, with the dense / serial pass counts of the slowest ones.

    ORCG_LIB=liborcgpu_prof.so python scripts/wg_durations.py --workload c4
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4", choices=["c4", "c5"])
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--stripe", type=int, default=0)
    args = ap.parse_args()
    from workload_files import make_c4, make_c5

    path = "/tmp/orcg_wg_%s_%d.orc" % (args.workload, args.rows)
    if not os.path.exists(path):
        (make_c4 if args.workload == "c4" else make_c5)(path + ".tmp", args.rows, 64, compression="zstd")
        os.replace(path + ".tmp", path)
    import orc_amd

    L = orc_amd._lib.load()
    f = L.orcg_debug_wg_durations
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = 2 * 16384
    r = orc_amd.Reader(path, orc_amd.Context(0))
    xp = getattr(L, "orcg_debug_expand_phases", None)
    xb = (ctypes.c_ulonglong * 8)()
    for _ in range(3):
        buf = (ctypes.c_ulonglong * n)()
        ctypes.memset(buf, 0, n * 8)
        if xp is not None:
            xp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            xp(xb, 8, 1)
        r.read_stripe_device(args.stripe)
    f(buf, n)
    if xp is not None:
        xp(xb, 8, 0)
        nwg = max(int(xb[7]), 1)
        names = ["hdr_job", "entries_headers", "parse", "fill_scan", "patch_store"]
        print(json.dumps({"expand_workgroups": nwg,
                          "expand_us_per_wg": {nm: round(xb[k] * 0.01 / nwg, 2) for k, nm in enumerate(names)}}))
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2)
    used = a[:, 0] > 0
    dur = a[used, 0].astype(np.float64) * 0.01  # us
    dense = (a[used, 1] & 0xffffffff).astype(np.int64)
    serial = (a[used, 1] >> 32).astype(np.int64)
    idx = np.flatnonzero(used)
    order = np.argsort(-dur)
    print(json.dumps({"workgroups": int(dur.size), "mean_us": round(float(dur.mean()), 1),
                      "p50": round(float(np.percentile(dur, 50)), 1), "p90": round(float(np.percentile(dur, 90)), 1),
                      "p99": round(float(np.percentile(dur, 99)), 1), "max": round(float(dur.max()), 1),
                      "dense_passes_mean": round(float(dense.mean()), 2),
                      "serial_passes_mean": round(float(serial.mean()), 2)}))
    for k in order[:25]:
        print(json.dumps({"wg": int(idx[k]), "us": round(float(dur[k]), 1), "dense": int(dense[k]),
                          "serial": int(serial[k])}))
    hist, edges = np.histogram(dur, bins=20)
    print(json.dumps({"hist": hist.tolist(), "edges_us": [round(float(e), 1) for e in edges]}))


if __name__ == "__main__":
    main()
