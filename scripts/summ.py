#!/usr/bin/env python3
"""One line per bench_file JSON log: workload, value, device decode, row reader rates."""
import json
import sys

for p in sys.argv[1:]:
    try:
        d = [json.loads(l) for l in open(p) if l.startswith("{")][-1]
    except Exception as e:  # noqa: BLE001
        print(p, "no json", e)
        continue
    rr = d.get("row_reader") or {}
    cb = d.get("cpu_baseline") or {}
    print("%s: %s Mrows/s, device %.4f s (steady %s), x roofline %s, rr1024 %s rr16k %s, cpu %s, check %s" % (
        d.get("workload"), d.get("value"), d["phases_s_summed_over_stripes"]["device_decode"],
        (d.get("device_decode_steady") or {}).get("device_decode_s"), d.get("device_vs_roofline"),
        (rr.get("batch_1024") or {}).get("mrows_per_s"), (rr.get("batch_16384") or {}).get("mrows_per_s"),
        cb.get("value"), (d.get("check") or "")[:40]))
