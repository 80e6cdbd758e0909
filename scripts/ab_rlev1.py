#!/usr/bin/env python3
"""RLEv1 kernel timing on synthetic stream shapes (tests/rlev1_writer.py):
configs[0]'s shapes (demo-11: dictionary indices as literal groups of 1-byte
varints, a sequential column as runs of 130) and larger streams cut by host
plans. Each shape is decoded through orcg_rlev1_decode_device, checked
against the writer's values, then timed with HIP events on the context's
stream (median of 3 x --iters launches). --phases reads the kernel's phase
counters (ORCG_LIB=orc_amd/liborcgpu_prof.so, a -DORCG_PHASE_PROF build).

    python scripts/ab_rlev1.py --shapes dict7,seq,rand14,mix
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

from rlev1_writer import encode, random_groups  # noqa: E402


def shape(name, n, rng):
    if name == "dict7":  # demo-11 dictionary indices: literal groups of 128 1-byte varints
        v = rng.integers(0, 7, size=n)
        return encode([("lit", [int(x) for x in v[i:i + 128]]) for i in range(0, n, 128)], False)
    if name == "seq":  # a sequential key column: runs of 130, delta 1
        gs, b = [], 1
        for i in range(0, n, 130):
            k = min(130, n - i)
            gs.append(("run", b, 1, k) if k >= 3 else ("lit", list(range(b, b + k))))
            b += k
        return encode(gs, True)
    if name == "rand14":  # literal groups of 2-byte varints
        v = rng.integers(-(1 << 13), 1 << 13, size=n)
        return encode([("lit", [int(x) for x in v[i:i + 128]]) for i in range(0, n, 128)], True)
    if name == "mix":
        return encode(random_groups(rng, n, True, 35), True)
    raise SystemExit("unknown shape " + name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="dict7,seq,rand14,mix")
    ap.add_argument("--sizes", default="5000,1000000", help="values per stream")
    ap.add_argument("--seg-bytes", type=int, default=16 << 10, help="host plan segment bytes")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--phases", action="store_true")
    ap.add_argument("--interleave", action="store_true",
                    help="also time each launch bracketed by events with a different kernel (the wide instance on "
                         "the same stream) between launches: the file path's situation (cold instruction cache)")
    args = ap.parse_args()
    import torch

    import orc_amd

    L = orc_amd._lib.load()
    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(0, stream=stream)
    rng = np.random.default_rng(5)
    for name in args.shapes.split(","):
        for n in [int(x) for x in args.sizes.split(",")]:
            data, vals = shape(name, n, rng)
            buf = np.frombuffer(bytes(data), dtype=np.uint8)
            h = ctypes.c_void_p()
            orc_amd.rle.check(L.orcg_rlev1_plan_create(buf.ctypes.data_as(ctypes.c_void_p), buf.size, args.seg_bytes,
                                                       1 << 40, ctypes.byref(h)))
            segp = ctypes.c_void_p()
            nseg = L.orcg_rlev2_plan_segments(h, ctypes.byref(segp))
            segs = np.ctypeslib.as_array(ctypes.cast(segp, ctypes.POINTER(ctypes.c_uint64)), shape=(nseg * 2,)).copy()
            L.orcg_rlev2_plan_destroy(h)
            with torch.cuda.stream(stream):
                d_src = torch.from_numpy(buf.copy()).cuda()
                d_seg = torch.from_numpy(segs.view(np.int64)).cuda()
                out = torch.zeros(vals.size, dtype=torch.int64, device="cuda")
            stream.synchronize()

            def run():
                orc_amd.rle.check(L.orcg_rlev1_decode_device(ctx.handle, d_src.data_ptr(), buf.size, 1 if name in (
                    "seq", "rand14", "mix") else 0, d_seg.data_ptr(), nseg, 0, vals.size, out.data_ptr(), 8),
                    ctx.last_error)

            run()
            ctx.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), vals)
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
            cold_us = None
            if args.interleave:
                h2 = ctypes.c_void_p()
                orc_amd.rle.check(L.orcg_rlev1_plan_create(buf.ctypes.data_as(ctypes.c_void_p), buf.size, 1 << 20,
                                                           1 << 40, ctypes.byref(h2)))
                sp2 = ctypes.c_void_p()
                ns2 = L.orcg_rlev2_plan_segments(h2, ctypes.byref(sp2))
                s2 = np.ctypeslib.as_array(ctypes.cast(sp2, ctypes.POINTER(ctypes.c_uint64)), shape=(ns2 * 2,)).copy()
                L.orcg_rlev2_plan_destroy(h2)
                with torch.cuda.stream(stream):
                    d_seg2 = torch.from_numpy(s2.view(np.int64)).cuda()
                    out2 = torch.zeros(vals.size, dtype=torch.int64, device="cuda")

                def other():
                    orc_amd.rle.check(L.orcg_rlev1_decode_device(ctx.handle, d_src.data_ptr(), buf.size, 1 if name in (
                        "seq", "rand14", "mix") else 0, d_seg2.data_ptr(), ns2, 0, vals.size, out2.data_ptr(), 8),
                        ctx.last_error)

                pairs = []
                for _ in range(args.iters):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    run()
                    e1.record(stream)
                    other()
                    pairs.append((e0, e1))
                stream.synchronize()
                cold_us = round(float(np.median([a.elapsed_time(b) for a, b in pairs])) * 1e3, 2)
            phases = None
            if args.phases:
                f = L.orcg_debug_rlev1_phases
                f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
                pb = (ctypes.c_ulonglong * 10)()
                f(pb, 10, 1)
                for _ in range(args.iters):
                    run()
                ctx.synchronize()
                f(pb, 10, 1)
                nwg = nseg * args.iters
                names = ["setup", "window", "bitmap", "exits", "chain", "groups", "owner", "literals", "runs"]
                phases = {nm: round(pb[k] * 0.01 / nwg, 3) for k, nm in enumerate(names)}
            print(json.dumps({"shape": name, "values": int(vals.size), "bytes": int(buf.size), "segments": int(nseg),
                              "us": round(ms * 1e3, 2), "GBps": round((buf.size + 8 * vals.size) / ms / 1e6, 1),
                              "Mvalues_s": round(vals.size / ms / 1e3, 1), "interleaved_us": cold_us,
                              "phases_us_per_wg": phases}), flush=True)


if __name__ == "__main__":
    main()
