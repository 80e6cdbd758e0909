#!/usr/bin/env python3
"""Where a tiled RLEv2 launch spends its time, per phase, from the kernel's
own cycle counters (orc_amd/csrc/rlev2_tiled.hip PROF_MARK; build with
ORCG_PHASE_PROF=1 python -m orc_amd.build, which writes liborcgpu_prof.so).
Thread 0 of every workgroup adds the wall-clock ticks (100 MHz) between
consecutive phase marks; the script prints each phase's share and its
workgroup-microseconds per launch.

    ORCG_LIB=liborcgpu_prof.so python scripts/phase_prof.py --data repeat --bits 12
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ORCG_LIB", "liborcgpu_prof.so")

PHASES = ["fill", "serial_walk", "serial_expand", "dense_dp", "dense_chain", "dense_emit", "dense_expand"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--bits", type=int, default=12)
    ap.add_argument("--data", default="repeat")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--stride", type=int, default=10_000)
    args = ap.parse_args()
    import torch

    import orc_amd

    L = orc_amd._lib.load()
    L.orcg_debug_phase_counters.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from streams import make

    v, data, pos = make(args.data, args.bits, args.rows, args.stride)
    n = int(v.size)
    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(0, stream=stream)
    with torch.cuda.stream(stream):
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        d_out = torch.empty(n, dtype=torch.int64, device="cuda")
    stream.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    for var in [int(x) for x in args.variants.split(",")]:
        ctx.set_rlev2_variant(var)
        orc_amd.decode_positions_device(ctx, d_src, d_pos, args.stride, n, True, d_out)
        ctx.synchronize()
        assert np.array_equal(d_out.cpu().numpy(), v), "decode mismatch"
        L.orcg_debug_phase_counters(buf, 16, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.iters):
            orc_amd.decode_positions_device(ctx, d_src, d_pos, args.stride, n, True, d_out)
        e1.record(stream)
        ctx.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        L.orcg_debug_phase_counters(buf, 16, 1)
        ticks = np.array(buf[: len(PHASES)], dtype=np.float64) / args.iters
        tot = ticks.sum()
        print(json.dumps({"variant": var, "data": args.data, "bits": args.bits, "rows": n,
                          "stream_B_per_value": round(data.size / n, 3), "ms": round(ms, 4),
                          "wg_us_per_launch": {p: round(t / 100.0, 1) for p, t in zip(PHASES, ticks)},
                          "share": {p: round(t / tot, 3) for p, t in zip(PHASES, ticks) if tot}}), flush=True)


if __name__ == "__main__":
    main()
