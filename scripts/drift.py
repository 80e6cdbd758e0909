#!/usr/bin/env python3
"""Per-launch time series of the decoder and a copy probe run back to back
(does sustained load lower the clock?)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the A/B build carries every tuning instance and the copy probes
os.environ.setdefault("ORCG_LIB", "liborcgpu_ab.so")


def main():
    import torch

    import orc_amd

    n = 100_000_000
    rng = np.random.default_rng(42)
    v = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64, endpoint=True)
    data, pos = orc_amd.encode_direct(v, True, aligned=True, rows_per_group=10_000)
    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(0, stream=stream)
    L = orc_amd._lib.load()
    with torch.cuda.stream(stream):
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        d_out = torch.empty(n, dtype=torch.int64, device="cuda")
        d_vals = torch.from_numpy(v).cuda()
        d_copy = torch.empty_like(d_vals)
    stream.synchronize()

    def dec():
        orc_amd.decode_positions_device(ctx, d_src, d_pos, 10_000, n, True, d_out)

    def cpy():
        L.orcg_probe_copy(ctx.handle, orc_amd.rle._tensor_ptr(d_vals), orc_amd.rle._tensor_ptr(d_copy), 8 * n, 2)

    for name, fn in [("decode", dec), ("copy8nt", cpy), ("decode", dec), ("copy8nt", cpy)]:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(201)]
        ev[0].record(stream)
        for i in range(200):
            fn()
            ev[i + 1].record(stream)
        ev[-1].synchronize()
        ts = [ev[i].elapsed_time(ev[i + 1]) * 1000 for i in range(200)]
        print(json.dumps({"kernel": name, "us": [round(t, 1) for t in ts]}), flush=True)


if __name__ == "__main__":
    main()
