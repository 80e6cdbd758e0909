#!/usr/bin/env python3
"""Sustained-load behaviour: run the decoder, then a copy probe of the same
byte count, back to back for a few seconds each while a thread samples
`rocm-smi` (socket power, shader / fabric / memory clocks). Prints one JSON
line per phase: per-launch time (first / last second) and the samples.
Question answered: does the decoder lose clock under sustained load where a
plain copy does not (power cap), or is the gap elsewhere?"""
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the A/B build carries every tuning instance and the copy probes
os.environ.setdefault("ORCG_LIB", "liborcgpu_ab.so")


def smi_sample():
    try:
        out = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--json"], capture_output=True,
                             text=True, timeout=10).stdout
        d = json.loads(out)
        card = d[sorted(d)[0]]
        keep = {}
        for k, v in card.items():
            kl = k.lower()
            if "power" in kl or "sclk" in kl or "fclk" in kl or "mclk" in kl or "socclk" in kl:
                keep[k] = v
        return keep
    except Exception as e:  # noqa: BLE001 - sampling is best effort
        return {"error": str(e)[:200]}


def main():
    import torch

    import orc_amd

    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
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
        L.orcg_probe_copy(ctx.handle, orc_amd.rle._tensor_ptr(d_vals), orc_amd.rle._tensor_ptr(d_copy), 8 * n, 5)

    print(json.dumps({"phase": "idle", "smi": smi_sample()}), flush=True)
    for name, fn in [("decode", dec), ("copy16x4nt", cpy), ("decode", dec)]:
        samples = []
        stop = threading.Event()

        def sampler():
            while not stop.is_set():
                samples.append(smi_sample())
                time.sleep(0.2)

        th = threading.Thread(target=sampler)
        th.start()
        t_end = time.time() + secs
        blocks = []
        while time.time() < t_end:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(50):
                fn()
            e1.record(stream)
            e1.synchronize()
            blocks.append(round(e0.elapsed_time(e1) * 1000 / 50, 1))
        stop.set()
        th.join()
        print(json.dumps({"phase": name, "us_per_launch_blocks_of_50": blocks, "smi": samples[:3] + samples[-3:]}),
              flush=True)


if __name__ == "__main__":
    main()
