#!/usr/bin/env python3
"""Repeat one dense-instance parity case (tests/test_gpu_dense.py's
[40-False] stream at stride 777) many times in one process and report how
often and where the output differs (diagnosing an intermittent mismatch)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import orc_amd
    from test_gpu_dense import _encode_with_positions, _short_run_stream

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    variants = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "5,4,3,2,0").split(",")]
    rng = np.random.default_rng(5 + 40)
    v, kinds, lens = _short_run_stream(rng, False, 400_000, 40)
    ctx = orc_amd.default_context(0)
    for stride in (777, 10_000):
        data, pos = _encode_with_positions(orc_amd, v, False, kinds, lens, stride)
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        for variant in variants:
            ctx.set_rlev2_variant(variant)
            bad_runs = 0
            for r in range(reps):
                out = torch.zeros(v.size, dtype=torch.int64, device="cuda")
                try:
                    orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v.size, False, out)
                    ctx.synchronize()
                except Exception as e:  # a debug build's coverage check (ORCG_DEBUG_COVER)
                    print("variant %d stride %d rep %d: device error %s" % (variant, stride, r, e), flush=True)
                got = out.cpu().numpy()
                if not np.array_equal(got, v):
                    bad = np.flatnonzero(got != v)
                    i = int(bad[0])
                    bad_runs += 1
                    if bad_runs <= 3:
                        print("variant %d stride %d rep %d: %d bad, first %d (segment %d) got %s want %s" % (
                            variant, stride, r, bad.size, i, i // stride, got[i - 2:i + 8].tolist(),
                            v[i - 2:i + 8].tolist()), flush=True)
            print("variant %d stride %d: %d of %d runs differ" % (variant, stride, bad_runs, reps), flush=True)


if __name__ == "__main__":
    main()
