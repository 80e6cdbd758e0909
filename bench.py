#!/usr/bin/env python3
"""Benchmark: device-resident RLEv2 int64 decode (BASELINE.json configs[1]).

Workload (the configuration BASELINE.json's metric is quoted on): one int64
column of 10^8 rows, full-range signed values (seed 42) encoded as RLEv2
DIRECT runs of 512 at W=64 (the reference writer's aligned widths), the
uncompressed DATA stream and its ROW_INDEX positions (stride 10,000) resident
in HBM. One step = one decode of the whole stream into an int64 column in HBM.

Multi-GPU (torch.distributed.run, one rank per GPU): stripes shard across
ranks, each rank decodes its own 10^8-row stripe, no collective in the timed
region ("scaling": "weak"); value = all rows decoded / max-over-ranks time.

The JSON line also carries
  roofline     achieved algorithmic bytes (S + 8N per launch) / the kernel's
               HIP-event duration on its own stream, vs 8 TB/s HBM3E peak;
  cpu_baseline the CPU oracle (oracle/orc_oracle.c, a scalar restatement of
               RleDecoderV2) timed on this host on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "decoded GB/s + Mvalues/s device-resident, RLEv2 int64 column at 1/2/4/8 GPU"


def make_stream(rows, stride, seed=42):
    import orc_amd

    rng = np.random.default_rng(seed)
    v = rng.integers(-(1 << 63), (1 << 63) - 1, size=rows, dtype=np.int64, endpoint=True)
    data, pos = orc_amd.encode_direct(v, True, aligned=True, rows_per_group=stride)
    return v, data, pos


def cpu_baseline(data, rows, budget_s):
    """Scalar C oracle, 1 thread, on a bounded sample of the same stream:
    the first `sample` rows, repeated until ~budget_s of CPU work."""
    from oracle import oracle

    sample = min(rows, 20_000_000)
    # the sample's stream prefix ends at the first run boundary after `sample`
    buf = data.tobytes()
    out = np.empty(sample, dtype=np.int64)
    lib = oracle.lib()
    src = np.frombuffer(buf, dtype=np.uint8)
    reps, t_total = 0, 0.0
    while t_total < budget_s or reps == 0:
        t0 = time.perf_counter()
        rc = lib.orco_rlev2_decode_i64(src.ctypes.data, src.size, 1, out.ctypes.data, sample)
        t_total += time.perf_counter() - t0
        reps += 1
        if rc != 0:
            raise RuntimeError("oracle decode failed")
    vps = sample * reps / t_total
    return {
        "value": round(vps * 8 / 1e9, 3),
        "unit": "GB/s",
        "mvalues_per_s": round(vps / 1e6, 1),
        "cores": 1,
        "kind": "port",
        "sample": "first %d rows of the same W=64 DIRECT stream, decoded %d times (%.1f s)"
                  % (sample, reps, t_total),
    }


def load_traffic():
    """Per-launch HBM bytes from the committed rocprofv3 --pmc summary, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_rlev2_decode.json")
    if os.path.exists(p):
        try:
            with open(p) as f:
                return json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    # 100 warm-up launches (~30 ms): after the ~1 s idle of the verification
    # the clocks need that long to ramp; 10 left the first timed launches
    # ~4 % slow (measured 0.300 vs 0.289 ms per launch)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--stride", type=int, default=10_000)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--variant", type=int, default=0, help="0 tiled (default), 1 wave-walk")
    ap.add_argument("--copy-inclusive", type=int, default=3,
                    help="steps of the PCIe-inclusive pipeline to time (host bytes -> host values); 0 = skip")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import orc_amd

    # each rank owns its own stripe (different seed = different data)
    values, data, pos = make_stream(args.rows, args.stride, seed=42 + rank)
    S = int(data.size)
    N = args.rows

    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(local_rank, stream=stream)
    ctx.set_rlev2_variant(args.variant)
    with torch.cuda.stream(stream):
        d_src = torch.from_numpy(data).to("cuda")
        d_pos = torch.from_numpy(pos.view(np.int64)).to("cuda")
        d_out = torch.empty(N, dtype=torch.int64, device="cuda")
    stream.synchronize()

    def step():
        orc_amd.decode_positions_device(ctx, d_src, d_pos, args.stride, N, True, d_out)

    # verify one decode first, then warm up: the host-side compare leaves the
    # GPU idle for ~1 s, and the timed steps must not start from idle clocks
    if not args.no_verify:
        step()
        ctx.synchronize()
        ok = torch.equal(d_out.cpu(), torch.from_numpy(values))
        if not ok:
            raise SystemExit("decode mismatch on rank %d" % rank)
    for _ in range(args.warmup):
        step()
    ctx.synchronize()

    # the timed region: K back-to-back launches on the decode stream between
    # two HIP events (the kernel's average launch duration, gaps included)
    e_start = torch.cuda.Event(enable_timing=True)
    e_end = torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e_start.record(stream)
    for i in range(args.steps):
        step()
    e_end.record(stream)
    stream.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ctx.synchronize()  # surfaces any device-side decode error
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    kern_ms = e_start.elapsed_time(e_end) / args.steps
    # outside the timed region: the same K launches with an event after each
    # one (per-launch durations, as rocprofv3 --kernel-trace timestamps every
    # dispatch): mean within ~1 % of the back-to-back figure, plus the spread
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    evs[0].record(stream)
    for i in range(args.steps):
        step()
        evs[i + 1].record(stream)
    stream.synchronize()
    ctx.synchronize()
    per_launch = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]

    copy_incl = None
    if args.copy_inclusive and rank == 0:
        # host stream bytes (pinned) -> H2D -> decode -> D2H into a pinned
        # host column: the rate a host-memory caller sees
        h_src = torch.from_numpy(data).pin_memory()
        h_out = torch.empty(N, dtype=torch.int64).pin_memory()
        ts = []
        for _ in range(args.copy_inclusive + 1):
            torch.cuda.synchronize()
            c0 = time.perf_counter()
            with torch.cuda.stream(stream):
                d_src.copy_(h_src, non_blocking=True)
                step()
                h_out.copy_(d_out, non_blocking=True)
            stream.synchronize()
            ts.append(time.perf_counter() - c0)
        t_ci = float(np.median(ts[1:]))
        copy_incl = {"GBps_decoded": round(8 * N / t_ci / 1e9, 2), "ms": round(t_ci * 1e3, 3),
                     "h2d_bytes": S, "d2h_bytes": 8 * N}
        if not args.no_verify and not torch.equal(h_out, torch.from_numpy(values)):
            raise SystemExit("copy-inclusive decode mismatch")

    if rank == 0:
        rows_total = N * world
        ms_per_step = elapsed * 1e3 / args.steps
        value = rows_total * 8 / (elapsed / args.steps) / 1e9
        algo_bytes = S + 8 * N
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic()
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "mvalues_per_s": round(rows_total / (elapsed / args.steps) / 1e6, 1),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {
                "workload": "configs[1]: single int64 RLEv2-direct column, 10^8 rows, uncompressed "
                            "stream resident in HBM, 1 MI355X per stripe",
                "rows_per_gpu": N,
                "encoding": "RLEv2 DIRECT, W=64 (aligned), 512-value runs, signed (zigzag)",
                "stream_bytes": S,
                "row_index_stride": args.stride,
                "parallelism": "stripe-sharded x%d" % world,
                "kernel": ["rlev2_tiled_kernel", "rlev2_decode_kernel"][args.variant],
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel_ms": round(kern_ms, 4),
                "kernel_ms_timestamped": {"mean": round(float(np.mean(per_launch)), 4),
                                          "min": round(float(np.min(per_launch)), 4),
                                          "max": round(float(np.max(per_launch)), 4)},
                "algorithmic_bytes_per_launch": algo_bytes,
            },
        }
        if copy_incl:
            line["copy_inclusive"] = copy_incl
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(data, N, args.cpu_budget)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
