#!/usr/bin/env python3
"""RLEv1 phase split inside the file path (configs[0], demo-11): reads every
stripe through the product reader on the phase-profiling build
(ORCG_LIB=liborcgpu_prof.so) and prints the kernel's per-workgroup phase
times (scripts/ab_rlev1.py --phases gives the same for synthetic streams)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ORCG_LIB", "liborcgpu_prof.so")


def main():
    import orc_amd
    L = orc_amd._lib.load()
    f = L.orcg_debug_rlev1_phases
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    ctx = orc_amd.Context(0)
    path = os.path.join(ROOT, "tests", "golden", "files", "demo-11-zlib.orc")
    r = orc_amd.Reader(path, ctx)
    n = r.num_stripes
    r.read_stripes_device(0, n)  # warm-up
    pb = (ctypes.c_ulonglong * 10)()
    f(pb, 10, 1)
    r.read_stripes_device(0, n)
    f(pb, 10, 1)
    names = ["setup", "window", "bitmap", "exits", "chain", "groups", "table", "literals", "runs"]
    wgs = int(sys.argv[1]) if len(sys.argv) > 1 else 22 * n
    print(json.dumps({"stripes": n, "workgroups": wgs,
                      "phases_us_per_wg": {nm: round(pb[k] * 0.01 / wgs, 3) for k, nm in enumerate(names)},
                      "slowest_window_us": round(pb[9] * 0.01, 3)}))


if __name__ == "__main__":
    main()
