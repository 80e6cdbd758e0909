#!/usr/bin/env python3
"""File-path benchmarks (BASELINE.json configs[2..4]): ORC file bytes in host
memory -> host block decompression + stripe / row-index parse -> one H2D per
stripe -> GPU decode of every column into HBM (stripe i+1 prepared on the
host while stripe i decodes), next to pyarrow's ORC C++ reader (1 thread) on
the same file.

Workloads (--workload):
  c3  demo-12-zlib schema at ~10^8 rows: the example's 1,920,800 rows tiled
      52x (_col0 offset per tile), zlib, 64 MB stripes, dictionary strings.
  c4  TPC-H lineitem-like, 16 columns (sorted orderkey with 1-7 repeats,
      uniform part/suppkey, linenumber, 4 decimal(15,2), 3 dates, 4
      low-cardinality dictionary strings, direct comment strings), zstd.
  c5  struct<a:list<int>, m:map<string,int>> with 10 % nulls at every level,
      list / map lengths U[0, 8], 16 map keys, zstd.

Multi-GPU: under torch.distributed.run each rank decodes a contiguous stripe
range (RowReaderOptions::range; orc_amd.shard.partition_stripes) with no
collective in the timed region; value = all rows / max-over-ranks time.

    python scripts/bench_file.py --workload c4 [--rows 10000000] [--iters 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from workload_files import make_c3, make_c4, make_c5  # noqa: E402


WORKLOADS = {
    "c3": (make_c3, 52 * 1920800, "configs[2]: demo-12-zlib schema at %d rows, zlib, %d MB stripes"),
    "c4": (make_c4, 10_000_000, "configs[3] schema (TPC-H lineitem-like 16 columns) at %d rows (one GPU's share of "
                                "configs[3] is 1.25 * 10^8), zstd, %d MB stripes"),
    "c5": (make_c5, 10_000_000, "configs[4] schema (struct<list<int>, map<string,int>>, 10%% nulls) at %d rows (one "
                                "GPU's share of configs[4] is 1.25 * 10^7), zstd, %d MB stripes"),
    "c1": (None, 0, "configs[0] substitute: examples/demo-11-zlib.orc (demo-11-none.orc is not in the reference), "
                    "%d rows, full scan, %s"),
}



HBM_PEAK = 8.0e12      # B/s, MI355X HBM3E peak (the roofline denominator everywhere)
COPY_CEILING = 6.0e12  # B/s, the best measured device copy on these boxes (profiles/r03, probe5)

def view_bytes(v, kind, precision):
    """Device bytes of one decoded column view (the batch layout of
    include/orcg_reader.h)."""
    n = v.num_elements
    b = n if v.has_nulls else 0
    if kind in (7, 8, 16, 17):  # strings: start + length
        b += 16 * n
    elif kind in (10, 11):  # list / map offsets
        b += 8 * (n + 1)
    elif kind == 14:
        b += (16 if precision > 18 else 8) * n
    elif kind in (9, 18):
        b += 16 * n
    elif kind != 12:
        b += 8 * n
    return b


def progress(msg):
    """A line on stderr per phase (long silent phases look hung to the runner)."""
    print("[bench_file %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def concat_leg(dist, r, path, first, last, rank):
    """The N > 1 final concat, timed apart from the decode: every rank copies
    its stripes' rows of the first integer column out of HBM into its own
    slice of one shared host batch (orc_amd.shard.write_rows_to_shared_host,
    no data collective); rank 0 checks the assembled column against
    pyarrow."""
    import torch

    from orc_amd.shard import write_rows_to_shared_host

    root = r.types[0]
    fields = [(n, t) for n, t in zip(root.field_names, root.subtypes) if r.types[t].kind in (2, 3, 4)]
    if not fields:
        return None
    name, tid = fields[0]
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else os.environ.get("TMPDIR", "/tmp")
    fpath = os.path.join(shm, "orcg_bench_file_concat_%s" % os.environ.get("MASTER_PORT", "0"))
    dist.barrier()
    t = time.perf_counter()
    parts = []
    for k in range(last - first):
        v = r.stripe_column_view(k, tid)
        parts.append(r._host(v.data, 8 * v.num_elements, np.int64))
    local = torch.from_numpy(np.concatenate(parts) if parts else np.zeros(0, np.int64))
    host = write_rows_to_shared_host(dist, local, fpath, create=(rank == 0))
    el = time.perf_counter() - t
    tt = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    ok = None
    if rank == 0:
        import pyarrow.orc as po
        col = po.ORCFile(path).read(columns=[name]).column(0)
        want = np.array([0 if x is None else x for x in col.to_pylist()], dtype=np.int64)
        ok = bool(np.array_equal(host.numpy(), want))
        if not ok:
            raise SystemExit("concatenated %s differs from pyarrow" % name)
    dist.barrier()
    if rank == 0 and os.path.exists(fpath):
        os.unlink(fpath)
    n = int(host.numel())
    return {"column": name, "rows": n, "ms": round(float(tt.item()) * 1e3, 3),
            "GBps": round(8 * n / float(tt.item()) / 1e9, 2), "mode": "D2H into a shared host batch",
            "checked_against_pyarrow": ok}


def row_reader_leg(path, nrows, stripes_wall):
    """The reference caller's path: orc::RowReader::next(batch) at capacity
    1024 (the reference's default batch) and 16384 through the C++ adapter (orc_amd/csrc/GpuRowReader.hh), every batch
    filled into host ColumnVectorBatches; a compiled program
    (tests/cxx/reader_test.cpp --bench), timed from the first next() to the
    last."""
    import subprocess

    src = os.path.join(ROOT, "tests", "cxx", "reader_test.cpp")
    exe = os.path.join(ROOT, "tests", "cxx", "build", "reader_test")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    hdr = os.path.join(ROOT, "orc_amd", "csrc", "GpuRowReader.hh")
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", src, "-o",
                               exe, "-L" + os.path.join(ROOT, "orc_amd"), "-lorcgpu",
                               "-Wl,-rpath," + os.path.join(ROOT, "orc_amd"), "-Wl,-rpath,/opt/rocm/lib"])
    out = {}
    for cap, extra in ((1024, []), (16384, []), (1024, ["--pinned"])):
        r = subprocess.run([exe, path, "--bench", "--batch", str(cap)] + extra, capture_output=True, text=True,
                           timeout=600)
        if r.returncode != 0:
            raise SystemExit("row reader bench failed: %s" % r.stderr[-500:])
        if "rowreader" in os.environ.get("ORCG_DEBUG", ""):
            sys.stderr.write("batch %d%s:\n%s" % (cap, " pinned" if extra else "", r.stderr))
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d["vs_read_stripes_wall"] = round(d["seconds"] / max(stripes_wall, 1e-9), 2)
        out["batch_%d%s" % (cap, "_pinned_pool" if extra else "")] = d
    return out


def multi_reader_leg(path, k, first, last, stripe_rows, iters, device):
    """k Readers, each with its own Context (stream), read contiguous stripe
    ranges of [first, last) from k threads (ctypes drops the GIL in the
    library calls); the decoded batches stay in HBM as in the single-reader
    pass (checked by check_multi, outside the timed region)."""
    import threading

    import orc_amd

    bounds = np.linspace(first, last, k + 1).round().astype(int)
    parts = [(int(a), int(b)) for a, b in zip(bounds[:-1], bounds[1:]) if b > a]
    readers = [orc_amd.Reader(path, orc_amd.Context(device)) for _ in parts]
    errs = []

    def one(rd, a, b):
        try:
            rd.read_stripes_device(a, b - a)
        except Exception as e:  # surfaced after the join
            errs.append(e)

    def scan():
        ts = [threading.Thread(target=one, args=(rd, a, b)) for rd, (a, b) in zip(readers, parts)]
        t = time.perf_counter()
        for th in ts:
            th.start()
        for th in ts:
            th.join()
        dt = time.perf_counter() - t
        if errs:
            raise errs[0]
        return dt

    scan()  # warm-up (allocations)
    wall = min(scan() for _ in range(max(iters, 1)))
    rows = int(sum(stripe_rows[first:last]))
    return {"readers": len(parts), "wall_s": round(wall, 4), "mrows_per_s": round(rows / wall / 1e6, 2),
            "ranges": parts if len(parts) <= 16 else len(parts)}, readers, parts


def check_multi(readers, parts, r, first):
    """The concurrent scan's resident batches (every stripe, every column)
    against the single reader's batches of the same stripes."""
    for rd, (a, b) in zip(readers, parts):
        for s in range(a, b):
            for t in r.types:
                v1, v0 = rd.stripe_column_view(s - a, t.id), r.stripe_column_view(s - first, t.id)
                if v1.decoded != v0.decoded:
                    return "stripe %d column %d: decoded flag differs" % (s, t.id)
                if v0.decoded and not _same(vars(rd._column(v1, t)), vars(r._column(v0, t))):
                    return "stripe %d column %d differs" % (s, t.id)
    return None


def _same(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return np.array_equal(np.asarray(a), np.asarray(b))
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(_same(a[x], b[x]) for x in a)
    return a == b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS),
                    help="c1 = configs[0]'s scan of demo-11 (the zlib copy: demo-11-none.orc is not in the "
                         "reference), RLEv1 streams; c3 / c4 / c5 = configs[2..4]")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--stripe-mb", type=int, default=64)
    ap.add_argument("--path", default=None)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-copy", action="store_true", help="also time decode + D2H into host batches")
    ap.add_argument("--no-batch", action="store_true", help="one RLEv2 launch per stream (no multi-stream launches)")
    ap.add_argument("--row-reader", action="store_true",
                    help="also time the C++ RowReader scan loop (tests/cxx/reader_test --bench, batch 1024)")
    ap.add_argument("--cpu-threads", default="1,16", help="pyarrow ORC reader thread counts for the CPU legs")
    ap.add_argument("--steady", type=int, default=10,
                    help="also decode each prepared stripe this many times back to back (GPU never waiting for the "
                         "host): device decode at steady clocks; 0 = skip")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL; gloo lets "
                                                      "ranks share one GPU)")
    ap.add_argument("--variant", type=int, default=0, help="pinned RLEv2 kernel variant (0 = per-stream default)")
    ap.add_argument("--readers", type=int, default=0,
                    help="also time a scan by this many Readers (each its own Context and stream) on contiguous "
                         "stripe ranges (RowReaderOptions::range), driven from as many host threads: small "
                         "stripes' fixed costs overlap on one GPU")
    ap.add_argument("--check", default="all", choices=["all", "first", "none"],
                    help="stripes of this rank checked against pyarrow outside the timed region (numpy on the "
                         "value buffers, tests/arrow_parity.py)")
    args = ap.parse_args()
    maker, default_rows, desc = WORKLOADS[args.workload]
    rows = args.rows or default_rows
    path = args.path or "/tmp/orcg_%s_%d.orc" % (args.workload, rows)
    if args.workload == "c1":
        path = args.path or os.path.join(ROOT, "tests", "golden", "files", "demo-11-zlib.orc")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    t0 = time.time()
    if rank == 0 and maker is not None and not os.path.exists(path):
        progress("writing %s (%d rows)" % (path, rows))
        import threading

        w = threading.Thread(target=maker, args=(path + ".tmp", rows, args.stripe_mb))
        w.start()
        while w.is_alive():  # a line every 30 s: a 10^8-row file takes minutes to write
            w.join(30)
            if w.is_alive():
                progress("still writing %s" % path)
        if not os.path.exists(path + ".tmp"):
            raise SystemExit("writing %s failed" % path)
        os.replace(path + ".tmp", path)
    t_make = time.time() - t0

    import torch

    torch.cuda.set_device(local_rank % max(torch.cuda.device_count(), 1))
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(args.backend)
        dist.barrier()  # the file exists

    import orc_amd
    from orc_amd.shard import reader_ranges

    ctx = orc_amd.Context(local_rank % max(torch.cuda.device_count(), 1))
    if args.variant:
        ctx.set_rlev2_variant(args.variant)
    r = orc_amd.Reader(path, ctx)
    if args.no_batch:
        r.set_stream_batching(False)
    nrows = r.num_rows
    fsize = os.path.getsize(path)
    ranges, stripe_rows = reader_ranges(r, world)
    first, last = ranges[rank]
    my_rows = int(sum(stripe_rows[first:last]))

    def full_pass():
        t = time.perf_counter()
        if last > first:
            r.read_stripes_device(first, last - first)
        wall = time.perf_counter() - t
        tm = r.last_timings()
        return wall, np.array([tm["host_parse_s"], tm["host_decompress_s"], tm["host_plan_s"], tm["h2d_s"],
                               tm["device_decode_s"]])

    progress("file ready (%.1f s); decoding" % t_make)
    full_pass()  # warm-up (allocations, page cache)
    if dist:
        dist.barrier()
    runs = [full_pass() for _ in range(args.iters)]
    wall, ph = min(runs, key=lambda x: x[0])
    if dist:
        t = torch.tensor([wall], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    stats = r.last_stream_stats()

    # steady state: each stripe prepared once and decoded back to back, so
    # the kernels run at the clocks of a busy GPU (the pipelined read leaves
    # the GPU idle while the host decompresses, and its kernels then run at
    # idle clocks)
    steady = None
    if args.steady and last > first:
        import ctypes
        dec, h2d = ctypes.c_double(), ctypes.c_double()
        tot_dec = tot_h2d = 0.0
        for s in range(first, last):
            orc_amd._lib.check(r._L.orcg_reader_bench_stripe_decode(r._h, s, args.steady, ctypes.byref(dec),
                                                                    ctypes.byref(h2d)), r._err)
            tot_dec += dec.value
            tot_h2d += h2d.value
        steady = {"device_decode_s": round(tot_dec, 5), "h2d_s": round(tot_h2d, 5), "iters_per_stripe": args.steady}
        r.read_stripes_device(first, last - first)  # the views below describe the full read again

    # decoded bytes (device batch layout) of this rank's stripes
    dec_bytes = 0
    for k in range(last - first):
        for t in r.types:
            v = r.stripe_column_view(k, t.id)
            if v.decoded:
                dec_bytes += view_bytes(v, t.kind, t.precision)

    multi = None
    if args.readers > 1 and rank == 0:
        multi, mreaders, mparts = multi_reader_leg(path, args.readers, first, last, stripe_rows, args.iters,
                                                   ctx.device)
        diff = check_multi(mreaders, mparts, r, first)
        if diff:
            raise SystemExit("multi-reader scan differs from the single reader: " + diff)
        multi["check"] = "every stripe and column equal to the single reader's resident batches"
        del mreaders

    concat = None
    if dist:
        concat = concat_leg(dist, r, path, first, last, rank)

    check = None
    if last > first and args.check != "none":
        # correctness check on every rank, outside the timed region: its
        # stripes (all, or the first) against pyarrow (the reference's C++
        # reader), compared buffer by buffer (tests/arrow_parity.py)
        import pyarrow.orc as po
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from arrow_parity import first_difference_arrow

        pf = po.ORCFile(path)
        todo = range(first, last) if args.check == "all" else range(first, first + 1)
        checked = 0
        for s in todo:
            progress("rank %d: checking stripe %d against pyarrow" % (rank, s))
            diff = first_difference_arrow(pf.read_stripe(s), r.read_stripe(s), r)
            if diff:
                raise SystemExit("%s stripe %d decode mismatch against pyarrow on rank %d: %s"
                                 % (args.workload, s, rank, diff))
            checked += int(stripe_rows[s])
        check = "%s: stripes %d-%d (%d rows) equal to pyarrow (value buffers)" % (
            "every stripe" if args.check == "all" else "first stripe", first, first + len(todo) - 1, checked)

    host = None
    if args.host_copy and rank == 0:
        t = time.perf_counter()
        for s in range(first, last):
            r.read_stripe(s)
        host = time.perf_counter() - t

    rowreader = None
    if args.row_reader and rank == 0:
        progress("RowReader scan leg")
        rowreader = row_reader_leg(path, nrows, wall)

    cpu = None
    if not args.no_cpu_baseline and rank == 0:
        # the reference's C++ reader as pyarrow bundles it (ORC C++ 2.2.2):
        # a full read of the same file to Arrow, like tools/src/FileScan.cc's
        # scan loop (c++ ColumnVectorBatch -> Arrow arrays), on 1 and N threads
        import pyarrow as pa
        import pyarrow.orc as po
        legs = []
        progress("pyarrow CPU legs")
        reps = 5 if args.workload == "c1" else 1  # demo-11 reads in ~0.1 s: five reads per leg
        for th in [int(x) for x in args.cpu_threads.split(",") if x]:
            pa.set_cpu_count(th)
            t = time.perf_counter()
            for _ in range(reps):
                po.ORCFile(path).read()
            tc = (time.perf_counter() - t) / reps
            legs.append({"value": round(nrows / tc / 1e6, 2), "unit": "Mrows/s", "cores": th,
                         "kind": "pyarrow ORC C++ %s" % pa.__version__,
                         "sample": "full read of the same file to Arrow (pyarrow.orc.ORCFile.read), "
                                   "pa.set_cpu_count(%d), %.2f s" % (th, tc)})
        cpu = dict(legs[0], all_legs=legs) if legs else None

    if rank == 0:
        line = {
            "metric": "file decode Mrows/s (host decompress -> H2D -> GPU decode into HBM)",
            "workload": args.workload,
            "config": {"workload": desc % (nrows, "zlib, 385 stripes" if args.workload == "c1" else args.stripe_mb),
                       "stripes": r.num_stripes, "file_bytes": fsize,
                       "n_gpus": world, "host_threads": int(os.environ.get("ORCG_HOST_THREADS", "0"))
                       or min(16, os.cpu_count() or 1)},
            "value": round(nrows / wall / 1e6, 2),
            "unit": "Mrows/s",
            "decoded_GBps": round(dec_bytes * world / wall / 1e9, 2),
            "decoded_bytes_per_row": round(dec_bytes / max(my_rows, 1), 1),
            "wall_s": round(wall, 4),
            "phases_s_summed_over_stripes": {"host_parse": round(ph[0], 4), "host_decompress": round(ph[1], 4),
                                             "host_plan_and_row_index": round(ph[2], 4), "h2d": round(ph[3], 4),
                                             "device_decode": round(ph[4], 4)},
            "device_decode_Mrows_per_s": round(my_rows / max(ph[4], 1e-9) / 1e6, 1),
            # roofline: (uploaded stream bytes + decoded bytes) at the MI355X HBM peak
            # (8 TB/s, MI355X_MICROARCH.md); the measured device copy (~6 TB/s) is a
            # second column, never the denominator
            "device_roofline_s": round((stats["stage_bytes"] + dec_bytes) / HBM_PEAK, 6),
            "device_vs_roofline": round(ph[4] / max((stats["stage_bytes"] + dec_bytes) / HBM_PEAK, 1e-12), 1),
            "device_vs_copy_ceiling": round(ph[4] / max((stats["stage_bytes"] + dec_bytes) / COPY_CEILING, 1e-12), 1),
            "rle_streams": stats,
            "device_decode_steady": None if steady is None else dict(
                steady, Mrows_per_s=round(my_rows / max(steady["device_decode_s"], 1e-9) / 1e6, 1),
                vs_roofline=round(steady["device_decode_s"] / max((stats["stage_bytes"] + dec_bytes) / HBM_PEAK,
                                                                  1e-12), 1)),
            "host_batch_copy_s": None if host is None else round(host, 3),
            "concat": concat,
            "multi_reader": multi,
            "row_reader": rowreader,
            "check": check,
            "cpu_baseline": cpu,
            "make_file_s": round(t_make, 1),
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
