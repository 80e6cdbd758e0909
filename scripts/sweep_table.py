#!/usr/bin/env python3
"""Fold the `gpu_session.sh sweep` logs (gpurun_out/sweep_*.log, one JSON
line per variant / reference copy from scripts/ab_rlev2.py) into the
markdown table profiles/<round>/sweep.md.

    python scripts/sweep_table.py r01
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

VARIANTS = {
    0: "default (density-adaptive)",
    1: "wave-walk (rlev2_kernels.hip)",
    8: "tiled 21 KB + full-run fast path",
    9: "tiled 33 KB, LDS-DMA fill",
    10: "dense-capable 20.5 KB",
    11: "dense-capable 12.5 KB",
    14: "tiled 33 KB, register fill",
    15: "dense-capable 8.5 KB (6 WG/CU)",
    16: "8 + DELTA varint ends from terminator nibbles (T4)",
    17: "14 + T4",
    18: "11 + T4",
    19: "15 + T4",
}
REFS = {
    "copy": "torch copy",
    "probe2": "copy 8 B/lane NT (grid-stride)",
    "probe5": "copy 16 B/lane x4 NT (one-shot)",
    "probe7": "copy through 32 KB LDS-DMA windows",
    "probe11": "copy through 32 KB register-filled LDS windows",
}


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    if not (rnd.startswith("r") and rnd[1:].isdigit()):
        sys.exit("usage: sweep_table.py rNN")
    rows = []
    for path in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "sweep_*.log"))):
        recs = {}
        for line in open(path):
            line = line.strip()
            if not line.startswith("{"):
                continue
            r = json.loads(line)
            if "GBps" in r:
                recs[r["variant"]] = r
        if 0 not in recs:
            continue
        r0 = recs[0]
        rows.append((r0["data"], r0["bits"], r0["stream_B_per_value"], recs))
    rows.sort(key=lambda t: (t[0] != "random", t[0], t[1]))
    var_cols = [v for v in VARIANTS if any(v in r[3] for r in rows)]
    ref_cols = [v for v in REFS if any(v in r[3] for r in rows)]
    out = ["# RLEv2 decode sweep (%s, one MI355X, scripts/ab_rlev2.py, 1e8 values, stride 10000)" % rnd, "",
           "GB/s = (stream bytes + 8 B/value) / median kernel time (interleaved rounds, one process); "
           "copy columns move 16 B/value (800 MB read + 800 MB write) on the same box.", ""]
    out.append("Variants: " + "; ".join("%d = %s" % (v, VARIANTS[v]) for v in var_cols) + ".")
    out.append("References: " + "; ".join("%s = %s" % (v, REFS[v]) for v in ref_cols) + ".")
    out.append("")
    head = ["data", "W", "stream B/value", "v0 ms"] + ["v%d GB/s" % v for v in var_cols] + \
           ["%s GB/s" % v for v in ref_cols]
    out.append("| " + " | ".join(head) + " |")
    out.append("|" + "---|" * len(head))
    for data, bits, bpv, recs in rows:
        cells = [data, str(bits), "%.3f" % bpv, "%.4f" % recs[0]["ms_median"]]
        cells += ["%.0f" % recs[v]["GBps"] if v in recs else "-" for v in var_cols]
        cells += ["%.0f" % recs[v]["GBps"] if v in recs else "-" for v in ref_cols]
        out.append("| " + " | ".join(cells) + " |")
    dst = os.path.join(ROOT, "profiles", rnd, "sweep.md")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        f.write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main()
