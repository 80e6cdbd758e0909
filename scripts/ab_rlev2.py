#!/usr/bin/env python3
"""Interleaved A/B of the RLEv2 kernel variants in ONE process (guide rule:
perf deltas come from interleaved rounds), next to a device copy of the same
byte count as the roofline reference. Prints one JSON line per variant."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the A/B build carries every tuning instance and the copy probes
os.environ.setdefault("ORCG_LIB", "liborcgpu_ab.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--bits", type=int, default=64)
    ap.add_argument("--variants", default="0,1,2,3,4,5,6")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--stride", type=int, default=10_000)
    ap.add_argument("--data", default="random", choices=["random", "delta", "repeat", "patched", "shortdirect", "shortmix"])
    ap.add_argument("--refs", default="copy,probe2,probe5,probe7,probe11",
                    help="reference copies timed beside the decoder (copy = torch, probeN = orcg_probe_copy mode N)")
    ap.add_argument("--timing-only", default="", help="variants timed even when their output mismatches (debug instances)")
    args = ap.parse_args()
    import torch

    import orc_amd

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from streams import make

    v, data, pos = make(args.data, args.bits, args.rows, args.stride)
    n = int(v.size)
    S = data.size
    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(0, stream=stream)
    with torch.cuda.stream(stream):
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        d_out = torch.empty(n, dtype=torch.int64, device="cuda")
        d_vals = torch.from_numpy(v).cuda()
        d_copy = torch.empty_like(d_vals)
    stream.synchronize()
    variants = [int(x) for x in args.variants.split(",")]

    L = orc_amd._lib.load()

    def run(var):
        if var == "copy":
            with torch.cuda.stream(stream):
                d_copy.copy_(d_vals)
        elif isinstance(var, str) and var.startswith("probe"):
            # the probes copy whole KBs: the copy covers the values up to the last full KB
            orc_amd._lib.check(L.orcg_probe_copy(ctx.handle, orc_amd.rle._tensor_ptr(d_vals),
                                                 orc_amd.rle._tensor_ptr(d_copy), (8 * n) & ~1023, int(var[5:])))
        else:
            ctx.set_rlev2_variant(var)
            orc_amd.decode_positions_device(ctx, d_src, d_pos, args.stride, n, True, d_out)

    # verify every variant once; a mismatching variant is reported and dropped
    bad = []
    for var in variants:
        with torch.cuda.stream(stream):  # same stream as the decode (torch streams do not sync)
            d_out.zero_()
        run(var)
        ctx.synchronize()
        if not torch.equal(d_out, d_vals):
            idx = torch.nonzero(d_out != d_vals).flatten()
            i0 = int(idx[0])
            print(json.dumps({"variant": var, "mismatch": int(idx.numel()), "first": i0,
                              "group": i0 // args.stride, "in_group": i0 % args.stride,
                              "expected": d_vals[i0:i0 + 4].tolist(), "got": d_out[i0:i0 + 4].tolist(),
                              "last": int(idx[-1])}), flush=True)
            bad.append(var)
    keep = {int(x) for x in args.timing_only.split(",") if x}
    variants = [v for v in variants if v not in bad or v in keep]
    refs = [r for r in args.refs.split(",") if r]
    for var in [r for r in refs if r.startswith("probe")]:
        with torch.cuda.stream(stream):
            d_copy.zero_()
        run(var)
        ctx.synchronize()
        m = ((8 * n) & ~1023) // 8
        if not torch.equal(d_copy[:m], d_vals[:m]):
            print(json.dumps({"variant": var, "mismatch": int((d_copy[:m] != d_vals[:m]).sum())}), flush=True)
    times = {var: [] for var in refs + variants}
    for _ in range(args.rounds):
        for var in refs + variants:
            for _ in range(2):
                run(var)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                run(var)
            e1.record(stream)
            e1.synchronize()
            times[var].append(e0.elapsed_time(e1) / args.iters)
    for var, ts in times.items():
        ms = float(np.median(ts))
        byts = 16 * n if isinstance(var, str) else S + 8 * n
        print(json.dumps({"variant": var, "bits": args.bits, "data": args.data, "stream_B_per_value": round(S / n, 3), "ms_median": round(ms, 4),
                          "ms_min": round(float(np.min(ts)), 4),
                          "GBps": round(byts / ms / 1e6, 1), "bytes": int(byts)}), flush=True)
    if set(bad) - keep:
        sys.exit(3)


if __name__ == "__main__":
    main()
