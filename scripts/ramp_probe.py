#!/usr/bin/env python3
"""How long the C2 decode takes launch by launch after the GPU has been idle:
per-launch HIP-event times of the first 60 launches after a 1.5 s host-side
idle, preceded by nothing, by 5 launches, or by a ~100 ms busy phase (the
copy-inclusive pipeline of bench.py). Prints one JSON line per case."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import orc_amd

    values, data, pos = bench.make_stream(100_000_000, 10_000)
    N = values.size
    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(0, stream=stream)
    with torch.cuda.stream(stream):
        d_src = torch.from_numpy(data).to("cuda")
        d_pos = torch.from_numpy(pos.view(np.int64)).to("cuda")
        d_out = torch.empty(N, dtype=torch.int64, device="cuda")
    stream.synchronize()
    h_src = torch.from_numpy(data).pin_memory()
    h_out = torch.empty(N, dtype=torch.int64).pin_memory()
    pipe = bench.copy_pipeline(ctx, stream, h_src, d_src, h_out, d_out, pos, 10_000, N, 10)

    def step():
        orc_amd.decode_positions_device(ctx, d_src, d_pos, 10_000, N, True, d_out)

    def timed(k):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
        evs[0].record(stream)
        for i in range(k):
            step()
            evs[i + 1].record(stream)
        stream.synchronize()
        return [round(evs[i].elapsed_time(evs[i + 1]), 4) for i in range(k)]

    for case in ("idle", "warm5", "copy_pipeline", "warm100", "idle", "copy_pipeline"):
        time.sleep(1.5)
        t0 = time.perf_counter()
        if case == "warm5":
            for _ in range(5):
                step()
        elif case == "warm100":
            for _ in range(100):
                step()
        elif case == "copy_pipeline":
            for _ in range(4):
                pipe()
        stream.synchronize()
        pre = time.perf_counter() - t0
        t = timed(60)
        print(json.dumps({"case": case, "pre_s": round(pre, 4), "first20_mean": round(float(np.mean(t[:20])), 4),
                          "last20_mean": round(float(np.mean(t[40:])), 4), "ms": t}), flush=True)


if __name__ == "__main__":
    main()
