#!/usr/bin/env python3
"""Benchmark: device-resident RLEv2 int64 decode (BASELINE.json configs[1]).

Workload (the configuration BASELINE.json's metric is quoted on): one int64
column of 10^8 rows, full-range signed values (seed 42) encoded as RLEv2
DIRECT runs of 512 at W=64 (the reference writer's aligned widths), the
uncompressed DATA stream and its ROW_INDEX positions (stride 10,000) resident
in HBM. One step = one decode of the whole stream into an int64 column in HBM.

Multi-GPU: `--gpus N` (N > 1) run without torch.distributed.run's environment
starts N ranks itself (a child `python -m torch.distributed.run`, spawned
before this process touches the GPU); under torch.distributed.run each rank
owns one GPU. Stripes shard across ranks as RowReaderOptions::range does
(c++/src/Reader.cc:337-345): each rank decodes its own 10^8-row stripe, no
collective in the timed region ("scaling": "weak"); value = all rows decoded
/ max-over-ranks time. Outside the timed region the final row-batch concat
is measured both ways SURVEY.md §8(e) names: every rank D2H's its rows into
its own slice of one shared host batch (no collective), and an RCCL
point-to-point gather of the device columns to rank 0 over xGMI.

Before the W warm-up steps, `--settle-ms` (default 60) of back-to-back
decodes take the GPU out of its idle power state: after the host-side stream
generation the first ~100 launches run 5-7 % slow (scripts/ramp_probe.py,
DESIGN.md §4). The JSON line reports them as `settle`; `--settle-ms 0` turns
them off.

The JSON line also carries
  roofline     achieved algorithmic bytes (S + 8N per launch) / the kernel's
               HIP-event duration on its own stream, vs 8 TB/s HBM3E peak;
  cpu_baseline the reference's own C++ decoder as pyarrow bundles it (Apache
               ORC C++ 2.2.2, a build of c++/src) reading a C2-shaped file
               stripe by stripe on every usable core (value) and on 1 core;
               beside it the CPU oracle (oracle/orc_oracle.c, the scalar
               restatement of RleDecoderV2) on the same host, and the
               reference's AVX-512 figures from BASELINE.md as context.

`--workload c4|c5` runs the file configs north_star shards over GPUs
(configs[3] / configs[4]) under the same contract: each rank reads a
contiguous, byte-balanced stripe range of one file (RowReaderOptions::range,
c++/src/Reader.cc:337-345) end to end (host decompression -> H2D -> GPU
decode into HBM, scripts/bench_file.py's pipeline); one step = one pass over
the rank's stripes; value = all ranks' rows / max-over-ranks step time.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "decoded GB/s + Mvalues/s device-resident, RLEv2 int64 column at 1/2/4/8 GPU"
# The reference's RleDecoderV2 on the survey container's Xeon (BASELINE.md §2,
# W=64, N=10^8): quoted for context, not measured here (the reference source
# does not travel to the GPU host)
REFERENCE_CPU = {"source": "BASELINE.md §2 (reference RleDecoderV2, survey container: 8 vCPU Xeon, not this host)",
                 "w64_1core_none_mvalues_per_s": 413.7, "w64_1core_avx512_mvalues_per_s": 473.2,
                 "w64_8core_avx512_mvalues_per_s": 3895.0}


def make_stream(rows, stride, seed=42):
    import orc_amd

    rng = np.random.default_rng(seed)
    v = rng.integers(-(1 << 63), (1 << 63) - 1, size=rows, dtype=np.int64, endpoint=True)
    data, pos = orc_amd.encode_direct(v, True, aligned=True, rows_per_group=stride)
    return v, data, pos


def usable_cores():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    # the GPU box's share is 16 CPUs whatever nproc shows
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16))


def cpu_baseline(data, rows, budget_s):
    """Scalar C oracle on a bounded sample of the same stream: the first
    `sample` rows (a run-aligned stream prefix), decoded repeatedly, on one
    core and then on every usable core at once (one independent stream per
    thread; ctypes releases the GIL around the C call)."""
    from oracle import oracle

    lib = oracle.lib()
    src = np.frombuffer(data.tobytes(), dtype=np.uint8)

    def leg(threads, sample, seconds):
        outs = [np.empty(sample, dtype=np.int64) for _ in range(threads)]
        done = [0] * threads
        err = []
        stop = time.perf_counter() + seconds

        def work(t):
            while True:
                rc = lib.orco_rlev2_decode_i64(src.ctypes.data, src.size, 1, outs[t].ctypes.data, sample)
                if rc != 0:
                    err.append(rc)
                    return
                done[t] += 1
                if time.perf_counter() >= stop:
                    return

        t0 = time.perf_counter()
        ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        el = time.perf_counter() - t0
        if err:
            raise RuntimeError("oracle decode failed")
        return sample * sum(done) / el, sum(done), el

    cores = usable_cores()
    s1 = min(rows, 20_000_000)
    v1, reps1, el1 = leg(1, s1, budget_s / 2)
    sn = min(rows, 5_000_000)
    vn, repsn, eln = leg(cores, sn, budget_s / 2)
    return {
        "value": round(vn * 8 / 1e9, 3),
        "unit": "GB/s",
        "mvalues_per_s": round(vn / 1e6, 1),
        "cores": cores,
        "kind": "port",
        "sample": "%d threads x first %d rows of the same W=64 DIRECT stream (independent streams), %d decodes "
                  "in %.1f s" % (cores, sn, repsn, eln),
        "one_core": {"value": round(v1 * 8 / 1e9, 3), "mvalues_per_s": round(v1 / 1e6, 1), "cores": 1,
                     "sample": "first %d rows decoded %d times (%.1f s)" % (s1, reps1, el1)},
        "reference_context": REFERENCE_CPU,
    }


def pyarrow_baseline(values, budget_s):
    """The reference's own C++ reader as pyarrow bundles it (Apache ORC C++
    2.2.2) on a C2-shaped file: the same full-range int64 values (a bounded
    prefix) written uncompressed by pyarrow's ORC writer (RLEv2 DIRECT runs of
    512 at W=64, 1 M-row stripes), read back stripe by stripe like
    tools/src/FileScan.cc's scan loop, on 1 thread and on every usable core
    (one stripe per task). Decoded GB/s = 8 B per value."""
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    try:
        import pyarrow as pa
        import pyarrow.orc as po
    except ImportError:
        return None
    n = min(values.size, 20_000_000)
    fd, path = tempfile.mkstemp(suffix=".orc", dir=os.environ.get("TMPDIR", "/tmp"))
    os.close(fd)
    try:
        po.write_table(pa.table({"v": pa.array(values[:n])}), path, compression="uncompressed",
                       stripe_size=8 << 20, row_index_stride=10000)
        nst = po.ORCFile(path).nstripes

        def leg(threads, seconds):
            # every thread reads its own stripes (k, k + threads, ...) with
            # its own ORCFile, over and over, until the time is up
            pa.set_cpu_count(threads)
            t0 = time.perf_counter()
            stop = t0 + seconds

            def work(t):
                f = po.ORCFile(path)
                rows, k = 0, t % nst
                while True:
                    rows += f.read_stripe(k).num_rows
                    k = (k + threads) % nst
                    if time.perf_counter() >= stop:
                        return rows

            with ThreadPoolExecutor(threads) as ex:
                done = sum(ex.map(work, range(threads)))
            el = time.perf_counter() - t0
            return done / el, done, el

        cores = usable_cores()
        v1, d1, e1 = leg(1, budget_s / 2)
        vn, dn, en = leg(cores, budget_s / 2)
        pa.set_cpu_count(cores)
        return {"kind": "pyarrow ORC C++ (pyarrow %s)" % pa.__version__,
                "sample": "first %d of the same values written uncompressed by pyarrow (%d stripes), read stripe "
                          "by stripe" % (n, nst),
                "one_core": {"value": round(v1 * 8 / 1e9, 3), "mvalues_per_s": round(v1 / 1e6, 1), "cores": 1,
                             "rows_read": d1, "seconds": round(e1, 2)},
                "all_cores": {"value": round(vn * 8 / 1e9, 3), "mvalues_per_s": round(vn / 1e6, 1), "cores": cores,
                              "rows_read": dn, "seconds": round(en, 2)}}
    finally:
        os.unlink(path)


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


def copy_pipeline(ctx, dec_stream, h_src, d_src, h_out, d_out, pos, stride, N, chunks):
    """Copy-inclusive decode as a pipeline: the stream is cut into `chunks`
    ranges of whole row groups (byte ranges from the row-index positions);
    chunk k's H2D, decode (value range of its row groups) and D2H run on
    three streams ordered by events, so chunk k + 1's H2D and chunk k - 1's
    D2H overlap chunk k's decode."""
    import torch

    import orc_amd

    G = pos.shape[0]
    S = int(d_src.numel())
    cuts = np.linspace(0, G, chunks + 1).astype(np.int64)
    ranges = []
    for k in range(chunks):
        g0, g1 = int(cuts[k]), int(cuts[k + 1])
        if g1 <= g0:
            continue
        b0 = 0 if g0 == 0 else int(pos[g0, 0])
        b1 = S if g1 >= G else int(pos[g1, 0])
        v0, v1 = g0 * stride, min(N, g1 * stride)
        ranges.append((b0, b1, v0, v1))
    d_pos = torch.from_numpy(pos.view(np.int64)).to("cuda")
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()

    def run():
        evs_in = [torch.cuda.Event() for _ in ranges]
        evs_dec = [torch.cuda.Event() for _ in ranges]
        for k, (b0, b1, v0, v1) in enumerate(ranges):
            with torch.cuda.stream(s_in):
                d_src[b0:b1].copy_(h_src[b0:b1], non_blocking=True)
                evs_in[k].record(s_in)
            dec_stream.wait_event(evs_in[k])
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v1 - v0, True, d_out[v0:v1], value_begin=v0)
            evs_dec[k].record(dec_stream)
            s_out.wait_event(evs_dec[k])
            with torch.cuda.stream(s_out):
                h_out[v0:v1].copy_(d_out[v0:v1], non_blocking=True)
        s_out.synchronize()

    return run


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nproc):
    """Start `nproc` ranks of this script under torch.distributed.run as a
    child process (this process has not touched the GPU) and return its exit
    code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % nproc,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def concat_legs(dist, d_out, N, world, rank, stream):
    """The final row-batch concat, timed outside the decode region:
    host  -- each rank copies its rows into its own slice of one shared host
             batch (a /dev/shm file every rank maps; offsets from an
             all-gather of the row counts): no collective on the data;
    rccl  -- point-to-point gather of the device columns to rank 0
             (orc_amd.shard.gather_to_root: RCCL send/recv over xGMI)."""
    import torch

    from orc_amd.shard import gather_to_root, write_rows_to_shared_host

    res = {}
    # the shared batch lives in /dev/shm when it fits there, else in TMPDIR
    need = 8 * N * world + (64 << 20)
    base = "/dev/shm"
    try:
        st = os.statvfs(base)
        if st.f_bavail * st.f_frsize < need:
            base = os.environ.get("TMPDIR", "/tmp")
    except OSError:
        base = os.environ.get("TMPDIR", "/tmp")
    path = os.path.join(base, "orcg_bench_concat_%s" % os.environ.get("MASTER_PORT", "0"))
    try:
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        write_rows_to_shared_host(dist, d_out, path, create=(rank == 0))
        torch.cuda.synchronize()
        dist.barrier()
        el = time.perf_counter() - t0
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        res["host"] = {"ms": round(el * 1e3, 3), "GBps": round(8 * N * world / el / 1e9, 2),
                       "bytes": 8 * N * world}
    except Exception as e:  # reported, never fatal to the decode measurement
        res["host"] = {"error": str(e)[:200]}
    finally:
        dist.barrier()
        if rank == 0 and os.path.exists(path):
            os.unlink(path)
    try:
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            full = gather_to_root(dist, d_out)
        torch.cuda.synchronize()
        dist.barrier()
        el = time.perf_counter() - t0
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        ok = True
        if rank == 0:
            ok = full is not None and full.numel() == N * world and torch.equal(full[:N], d_out)
        res["rccl"] = {"ms": round(el * 1e3, 3), "GBps": round(8 * N * (world - 1) / el / 1e9, 2),
                       "bytes_moved": 8 * N * (world - 1), "root_check": bool(ok)}
        del full
    except Exception as e:
        res["rccl"] = {"error": str(e)[:200]}
    return res


FILE_METRIC = "file decode Mrows/s (host decompress -> H2D -> GPU decode into HBM), stripes sharded over GPUs"


def run_file_workload(args, dist, world, rank, device):
    """configs[3] (C4) / configs[4] (C5) under the bench contract: one file of
    rows_per_gpu x world rows (written once by rank 0 with the generators of
    scripts/bench_file.py), each rank's stripe range from
    orc_amd.shard.reader_ranges (byte-balanced contiguous ranges, as
    RowReaderOptions::range selects stripes), one step = read_stripes_device
    over that range (pipelined host decompression, H2D, GPU decode)."""
    import torch

    import orc_amd
    from orc_amd.shard import reader_ranges

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from workload_files import make_c4, make_c5

    rows_per_gpu = args.file_rows
    total = rows_per_gpu * world
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "orcg_bench_%s_%d.orc" % (args.workload, total))
    t0 = time.time()
    if rank == 0 and not os.path.exists(path):
        print("[bench] writing %s (%d rows)" % (path, total), file=sys.stderr, flush=True)
        (make_c4 if args.workload == "c4" else make_c5)(path + ".tmp", total, 64)
        os.replace(path + ".tmp", path)
    make_s = time.time() - t0
    if dist:
        dist.barrier()
    ctx = orc_amd.Context(device)
    r = orc_amd.Reader(path, ctx)
    ranges, stripe_rows = reader_ranges(r, world)
    first, last = ranges[rank]
    my_rows = int(sum(stripe_rows[first:last]))

    def step():
        if last > first:
            r.read_stripes_device(first, last - first)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    dev_s = 0.0
    for _ in range(args.steps):
        step()
        dev_s += r.last_timings()["device_decode_s"]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = r.last_stream_stats()
    if dist:
        dev_t = "cuda" if args.backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rows_all = torch.tensor([float(my_rows)], dtype=torch.float64, device=dev_t)
        dist.all_reduce(rows_all)
        elapsed = float(t.item())
        rows_all = int(rows_all.item())
    else:
        rows_all = my_rows
    check = None
    if not args.no_verify and last > first:
        # outside the timed region: the rank's first stripe against pyarrow
        # (the reference's C++ reader)
        import pyarrow.orc as po

        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from arrow_parity import first_difference_arrow

        pf = po.ORCFile(path)
        for s in range(first, last):
            diff = first_difference_arrow(pf.read_stripe(s), r.read_stripe(s), r)
            if diff:
                raise SystemExit("%s stripe %d mismatch against pyarrow on rank %d: %s" % (args.workload, s, rank, diff))
        check = "every stripe of every rank equal to pyarrow (value buffers, tests/arrow_parity.py)"
    if rank == 0:
        step_s = elapsed / args.steps
        dev = dev_s / args.steps
        line = {
            "metric": FILE_METRIC,
            "value": round(rows_all / step_s / 1e6, 2),
            "unit": "Mrows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {"workload": ("configs[3]: TPC-H lineitem-like 16 columns" if args.workload == "c4" else
                                    "configs[4]: struct<list<int>, map<string,int>>, 10%% nulls") +
                                   ", %d rows per GPU (%d in the file), zstd, 64 MB stripes" % (rows_per_gpu, total),
                       "stripes": r.num_stripes, "rank0_stripes": [first, last],
                       "parallelism": "stripe-sharded x%d" % world, "file_s": round(make_s, 1)},
            "device_decode_ms_per_step_rank0": round(dev * 1e3, 3),
            "rle_streams": stats,
            "check": check,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--stride", type=int, default=10_000)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--settle-ms", type=float, default=60.0,
                    help="decode launches before the warm-up until this much GPU time has passed: the GPU leaves "
                         "its idle power state (the first ~100 launches after an idle second run 5-7 %% slow, "
                         "DESIGN.md §4); reported in the JSON line as `settle`; 0 = none")
    ap.add_argument("--variant", type=int, default=0, help="RLEv2 kernel variant (0 default, 1 wave-walk, ...)")
    ap.add_argument("--copy-inclusive", type=int, default=3,
                    help="steps of the PCIe-inclusive pipeline to time (host bytes -> host values); 0 = skip")
    ap.add_argument("--chunks", type=int, default=10, help="row-group chunks of the pipelined copy-inclusive leg")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--no-concat", action="store_true", help="skip the N > 1 concat legs")
    ap.add_argument("--workload", default="c2", choices=["c2", "c4", "c5"],
                    help="c2 = configs[1] device-resident column (the headline); c4 / c5 = configs[3] / [4] files, "
                         "stripes sharded over the GPUs")
    ap.add_argument("--file-rows", type=int, default=10_000_000, help="rows per GPU of the c4 / c5 file")
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's RANK / LOCAL_RANK / WORLD_SIZE and exit before touching the GPU")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world_size": world, "gpus": args.gpus}),
              flush=True)
        return

    import torch

    # one GPU per rank; on a box with fewer GPUs than ranks (the gloo
    # rehearsal of the N > 1 path on one GPU) ranks share devices round robin
    ndev = torch.cuda.device_count()
    device = local_rank % ndev if ndev else local_rank
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.backend)
        world = dist.get_world_size()

    if args.workload != "c2":
        return run_file_workload(args, dist, world, rank, device)

    import orc_amd

    # each rank owns its own stripe (different seed = different data)
    values, data, pos = make_stream(args.rows, args.stride, seed=42 + rank)
    S = int(data.size)
    N = args.rows

    stream = torch.cuda.Stream()
    ctx = orc_amd.Context(device, stream=stream)
    ctx.set_rlev2_variant(args.variant)
    with torch.cuda.stream(stream):
        d_src = torch.from_numpy(data).to("cuda")
        d_pos = torch.from_numpy(pos.view(np.int64)).to("cuda")
        d_out = torch.empty(N, dtype=torch.int64, device="cuda")
    stream.synchronize()

    def step():
        orc_amd.decode_positions_device(ctx, d_src, d_pos, args.stride, N, True, d_out)

    # verify one decode first (every value, compared on the device against the
    # generated values uploaded beforehand, so no host round trip leaves the
    # GPU idle between the check and the warm-up), then warm up
    if not args.no_verify:
        with torch.cuda.stream(stream):
            d_want = torch.from_numpy(values).to("cuda")
        stream.synchronize()
        step()
        with torch.cuda.stream(stream):
            ok = bool(torch.equal(d_out, d_want))
        ctx.synchronize()
        del d_want
        if not ok:
            raise SystemExit("decode mismatch on rank %d" % rank)
    # settle: back-to-back decodes until --settle-ms of GPU time has passed
    # (measured on the decode stream), then the W warm-up steps proper
    settle = {"launches": 0, "ms": 0.0}
    if args.settle_ms > 0:
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record(stream)
        while True:
            for _ in range(10):
                step()
            settle["launches"] += 10
            s1.record(stream)
            s1.synchronize()
            settle["ms"] = round(s0.elapsed_time(s1), 2)
            if settle["ms"] >= args.settle_ms or settle["launches"] >= 2000:
                break
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
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    ctx.synchronize()  # surfaces any device-side decode error
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
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

    concat = None
    if dist and not args.no_concat:
        concat = concat_legs(dist, d_out, N, world, rank, stream)

    copy_incl = None
    if args.copy_inclusive and rank == 0:
        # host stream bytes (pinned) -> H2D -> decode -> D2H into a pinned
        # host column: the rate a host-memory caller sees,
        # serial (one stream) and pipelined (row-group chunks over an H2D, a
        # decode and a D2H stream, so both PCIe directions and the decode
        # overlap)
        h_src = torch.from_numpy(data).pin_memory()
        h_out = torch.empty(N, dtype=torch.int64).pin_memory()

        def serial():
            with torch.cuda.stream(stream):
                d_src.copy_(h_src, non_blocking=True)
                step()
                h_out.copy_(d_out, non_blocking=True)
            stream.synchronize()

        pipelined = copy_pipeline(ctx, stream, h_src, d_src, h_out, d_out, pos, args.stride, N, args.chunks)
        res = {}
        for name, fn in (("serial", serial), ("pipelined", pipelined)):
            ts = []
            for _ in range(args.copy_inclusive + 1):
                h_out.zero_()
                torch.cuda.synchronize()
                c0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - c0)
            if not args.no_verify and not torch.equal(h_out, torch.from_numpy(values)):
                raise SystemExit("copy-inclusive (%s) decode mismatch" % name)
            t_ci = float(np.median(ts[1:]))
            res[name] = {"GBps_decoded": round(8 * N / t_ci / 1e9, 2), "ms": round(t_ci * 1e3, 3)}
        copy_incl = dict(res["pipelined"], h2d_bytes=S, d2h_bytes=8 * N,
                         pipeline="%d row-group chunks over H2D / decode / D2H streams" % args.chunks,
                         serial=res["serial"])

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
            "settle": settle,
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
                "kernel": "rlev2_decode_kernel" if args.variant == 1 else "rlev2_tiled_kernel",
                "variant": args.variant,
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
        if concat:
            line["concat"] = concat
        if copy_incl:
            line["copy_inclusive"] = copy_incl
        if not args.no_cpu_baseline:
            port = cpu_baseline(data, N, args.cpu_budget)
            ref = pyarrow_baseline(values, args.cpu_budget)
            if ref is not None:
                # the stated baseline is the reference's own C++ decoder (pyarrow's
                # build of it) on every usable core; the port is a secondary leg
                line["cpu_baseline"] = {
                    "value": ref["all_cores"]["value"], "unit": "GB/s",
                    "mvalues_per_s": ref["all_cores"]["mvalues_per_s"], "cores": ref["all_cores"]["cores"],
                    "kind": "reference",
                    "implementation": ref["kind"] + ": the reference's C++ RleDecoderV2 / IntegerColumnReader as "
                                                    "pyarrow builds it (c++/src, scalar unpack)",
                    "sample": ref["sample"] + ", %d threads (one stripe per task), %d rows in %.1f s" % (
                        ref["all_cores"]["cores"], ref["all_cores"]["rows_read"], ref["all_cores"]["seconds"]),
                    "one_core": ref["one_core"],
                    "port": port,
                    "reference_context": port.pop("reference_context"),
                }
            else:
                line["cpu_baseline"] = port
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
