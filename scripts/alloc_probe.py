#!/usr/bin/env python3
"""Does the output buffer's placement change the decoder's time? Decodes the
bench stream into two output columns, one allocated right after the stream
(bench.py's order) and one allocated after 1.6 GB of other buffers
(scripts/ab_rlev2.py's order), alternating blocks of 50 back-to-back
launches between two HIP events."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import orc_amd

    n = 100_000_000
    rng = np.random.default_rng(42)
    v = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64, endpoint=True)
    data, pos = orc_amd.encode_direct(v, True, aligned=True, rows_per_group=10_000)
    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(0, stream=stream)
    with torch.cuda.stream(stream):
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        out1 = torch.empty(n, dtype=torch.int64, device="cuda")
        pad = torch.empty(2 * n, dtype=torch.int64, device="cuda")
        out2 = torch.empty(n, dtype=torch.int64, device="cuda")
    stream.synchronize()
    addrs = {"src": d_src.data_ptr(), "out1": out1.data_ptr(), "pad": pad.data_ptr(), "out2": out2.data_ptr()}
    print(json.dumps({k: hex(a) for k, a in addrs.items()}), flush=True)

    def block(out):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(50):
            orc_amd.decode_positions_device(ctx, d_src, d_pos, 10_000, n, True, out)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1000 / 50

    for out in (out1, out2):
        block(out)
    res = {"out1": [], "out2": []}
    for _ in range(6):
        res["out1"].append(round(block(out1), 1))
        res["out2"].append(round(block(out2), 1))
    ctx.synchronize()
    assert torch.equal(out1.cpu(), torch.from_numpy(v)) and torch.equal(out2.cpu(), torch.from_numpy(v))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
