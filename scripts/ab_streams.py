#!/usr/bin/env python3
"""Per-stream kernel timing on real column shapes: writes a C4 / C5 workload
file uncompressed (same generator as bench_file.py), takes stripe 0's RLE
streams (scripts/file_streams.py) and decodes each one alone on the GPU at
several segment counts (host plans with at most values/G values per
segment, G = the stripe's row groups x factor), with each requested RLEv2
variant. One JSON line per (stream, segments, variant): median kernel ms
over --iters launches, values/s and (stream bytes + output bytes)/s.

    python scripts/ab_streams.py --workload c5 --rows 2600000 --factors 1,4,16
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5", choices=["c4", "c5"])
    ap.add_argument("--rows", type=int, default=2_600_000)
    ap.add_argument("--factors", default="1,4,16")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--min-bytes", type=int, default=64 << 10, help="skip streams smaller than this")
    ap.add_argument("--kinds", default="PRESENT,DATA,LENGTH")
    ap.add_argument("--phases", action="store_true",
                    help="byte RLE phase split (ORCG_LIB=liborcgpu_prof.so, a -DORCG_PHASE_PROF build)")
    args = ap.parse_args()
    from workload_files import make_c4, make_c5
    from file_streams import stripe_streams

    path = "/tmp/orcg_ab_%s_%d_none.orc" % (args.workload, args.rows)
    if not os.path.exists(path):
        (make_c4 if args.workload == "c4" else make_c5)(path + ".tmp", args.rows, 256, compression="uncompressed")
        os.replace(path + ".tmp", path)
    streams, enc, nrows = stripe_streams(path, 0)
    groups = (nrows + 9999) // 10000
    import torch

    import orc_amd

    L = orc_amd._lib.load()
    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(0, stream=stream)
    variants = [int(x) for x in args.variants.split(",")]
    factors = [int(x) for x in args.factors.split(",")]
    for col, kind, data in streams:
        if kind not in args.kinds.split(",") or data.size < args.min_bytes:
            continue
        ek = enc[col][0] if col < len(enc) else 0
        byte_rle = kind == "PRESENT"
        if not byte_rle and ek not in (2, 3):  # RLEv2 streams only (DIRECT_V2 / DICTIONARY_V2 columns)
            continue
        if kind == "DATA" and ek == 2 and data.size > 8 * 10_000_000:
            continue
        # DATA of a DIRECT_V2 int column is signed; dictionary indices and lengths are not
        signed = kind == "DATA" and ek == 2
        with torch.cuda.stream(stream):
            d_src = torch.from_numpy(data).cuda()
        ref = None
        for f in factors:
            G = groups * f
            if byte_rle:
                p0 = orc_amd.BytePlan(data, 1 << 30, 1 << 40)
                nvals = p0.values * 8
                plan = orc_amd.BytePlan(data, 1 << 30, max(1, -(-p0.values // G)))
            else:
                p0 = orc_amd.Plan(data, 1 << 30, 1 << 40)
                nvals = p0.values
                plan = orc_amd.Plan(data, 1 << 30, max(1, -(-nvals // G)))
            segs = plan.segments()
            with torch.cuda.stream(stream):
                d_seg = torch.from_numpy(segs.view(np.int64)).cuda()
                out = torch.empty(nvals + 8, dtype=torch.uint8 if byte_rle else torch.int64, device="cuda")
            for var in ([0] if byte_rle else variants):
                ctx.set_rlev2_variant(var)

                def run():
                    if byte_rle:
                        orc_amd.byterle_decode_device(ctx, d_src, d_seg, nvals, out, boolean=True)
                    else:
                        orc_amd.decode_device(ctx, d_src, d_seg, nvals, signed, out)

                run()
                ctx.synchronize()
                got = out[:nvals].clone()
                if ref is None:
                    ref = got
                elif not torch.equal(ref, got):
                    print(json.dumps({"col": col, "kind": kind, "segments": int(segs.shape[0]), "variant": var,
                                      "mismatch": True}), flush=True)
                    continue
                ts = []
                for _ in range(3):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.iters):
                        run()
                    e1.record(stream)
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) / args.iters)
                ms = float(np.median(ts))
                phases = None
                if args.phases and not byte_rle:
                    import ctypes
                    f = L.orcg_debug_phase_counters
                    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
                    buf = (ctypes.c_ulonglong * 16)()
                    f(buf, 16, 1)
                    for _ in range(args.iters):
                        run()
                    ctx.synchronize()
                    f(buf, 16, 1)
                    nwg = int(segs.shape[0]) * args.iters
                    names = ["fill", "serial_walk", "serial_expand", "dense_dp", "dense_chain", "dense_emit",
                             "dense_expand"]
                    phases = {nm: round(buf[k] * 0.01 / nwg, 3) for k, nm in enumerate(names)}
                    phases["runs_walked_per_wg"] = round(buf[8] / nwg, 1)
                    phases["serial_passes_per_wg"] = round(buf[9] / nwg, 2)
                if args.phases and byte_rle:
                    import ctypes
                    f = L.orcg_debug_byterle_phases
                    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
                    buf = (ctypes.c_ulonglong * 8)()
                    f(buf, 8, 1)
                    for _ in range(args.iters):
                        run()
                    ctx.synchronize()
                    f(buf, 8, 1)
                    # wall-clock ticks (100 MHz) summed over workgroups -> us per workgroup
                    nwg = int(segs.shape[0]) * args.iters
                    phases = [round(buf[k] * 0.01 / nwg, 3) for k in range(8)]
                out_b = nvals * (1 if byte_rle else 8)
                print(json.dumps({"col": col, "kind": kind, "enc": ek, "bytes": int(data.size), "values": int(nvals),
                                  "B_per_value": round(data.size / max(nvals, 1), 3),
                                  "segments": int(segs.shape[0]), "variant": var, "ms": round(ms, 4),
                                  "Gvalues_s": round(nvals / ms / 1e6, 1),
                                  "GBps": round((data.size + out_b) / ms / 1e6, 1), "phases_us_per_wg": phases}),
                      flush=True)
        ctx.set_rlev2_variant(0)


if __name__ == "__main__":
    main()
