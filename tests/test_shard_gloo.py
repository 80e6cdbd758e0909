"""Multi-process (world_size 2, gloo over 127.0.0.1) tests of the stripe
sharding path: every rank computes the same contiguous stripe ranges, row
offsets agree with an all-gather of counts, and the final concat reassembles
the column in rank order. The GPU variant decodes each rank's stripes on
cuda:0 and checks the gathered column against pyarrow."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT
from orc_amd.shard import gather_to_root, partition_stripes, row_offsets


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_partition_is_contiguous_and_balanced():
    rng = np.random.default_rng(0)
    sizes = rng.integers(1, 1000, size=385)
    for world in (1, 2, 3, 4, 8):
        ranges = partition_stripes(sizes, world)
        assert ranges[0][0] == 0 and ranges[-1][1] == len(sizes)
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
        per = [sizes[b:e].sum() for b, e in ranges]
        assert max(per) - min(per) <= 2 * sizes.max() + 1
    assert partition_stripes([], 4) == [(0, 0)] * 4
    assert partition_stripes([10], 2) in ([(0, 0), (0, 1)], [(0, 1), (1, 1)])


def _worker(rank, world, port, path, out_dir, use_gpu):
    import torch
    import torch.distributed as dist

    import orc_amd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = orc_amd.Context(0) if use_gpu else None
        r = orc_amd.Reader(path, ctx)
        from orc_amd.shard import reader_ranges
        ranges, rows = reader_ranges(r, world)
        offs, sizes = row_offsets(rows, ranges)
        # every rank derived the same plan
        mine = torch.tensor([ranges[rank][0], ranges[rank][1], offs[rank]], dtype=torch.int64)
        allp = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allp, mine)
        for q, t in enumerate(allp):
            assert t.tolist() == [ranges[q][0], ranges[q][1], offs[q]]
        b, e = ranges[rank]
        if use_gpu:
            col = r.types[0].subtypes[0]  # first top-level column (int)
            r.select([col])
            parts = [r.read_stripe(s).columns[col].data for s in range(b, e)]
            local = torch.from_numpy(np.concatenate(parts) if parts else np.zeros(0, np.int64))
        else:
            local = torch.arange(offs[rank], offs[rank] + sizes[rank], dtype=torch.int64)
        full = gather_to_root(dist, local)
        if rank == 0:
            np.save(os.path.join(out_dir, "full.npy"), full.numpy())
    finally:
        dist.destroy_process_group()


def _run(tmp_path, use_gpu, name="demo-11-zlib.orc"):
    path = os.path.join(ROOT, "tests", "golden", "files", name)
    mp.start_processes(_worker, args=(2, _free_port(), path, str(tmp_path), use_gpu), nprocs=2, join=True,
                       start_method="spawn")
    return np.load(os.path.join(tmp_path, "full.npy")), path


def test_gloo_world2_plan_and_concat(tmp_path):
    full, path = _run(tmp_path, use_gpu=False)
    import orc_amd
    n = orc_amd.Reader(path).num_rows
    np.testing.assert_array_equal(full, np.arange(n))


@pytest.mark.gpu
def test_gloo_world2_sharded_decode_matches_pyarrow(tmp_path):
    pa = pytest.importorskip("pyarrow.orc")
    full, path = _run(tmp_path, use_gpu=True)
    want = pa.ORCFile(path).read(columns=["_col0"]).column(0).to_numpy(zero_copy_only=False)
    np.testing.assert_array_equal(full, want.astype(np.int64))


def _host_concat_worker(rank, world, port, path, out_dir):
    import torch
    import torch.distributed as dist

    from orc_amd.shard import write_rows_to_shared_host

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # ragged shards (rank r holds 1000 + 37 r rows, rank 2 of 3 none)
        n = 0 if (world == 3 and rank == 2) else 1000 + 37 * rank
        start = sum(0 if (world == 3 and q == 2) else 1000 + 37 * q for q in range(rank))
        local = torch.arange(start, start + n, dtype=torch.int64)
        host = write_rows_to_shared_host(dist, local, path, create=(rank == 0))
        if rank == 0:
            np.save(os.path.join(out_dir, "host.npy"), host.numpy().copy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_concat_into_shared_host_batch(tmp_path, world):
    """DESIGN §5 option 2: each rank writes its rows into its own slice of one
    shared host batch (offsets from an all-gather of counts), no data
    collective."""
    shm = os.path.join(str(tmp_path), "batch.bin")
    mp.start_processes(_host_concat_worker, args=(world, _free_port(), shm, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(os.path.join(tmp_path, "host.npy"))
    n = sum(0 if (world == 3 and q == 2) else 1000 + 37 * q for q in range(world))
    np.testing.assert_array_equal(got, np.arange(n))


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` starts two ranks itself (torch.distributed.run as a
    child, before any GPU use); --dry-run makes each rank report its
    environment and exit."""
    import json
    import subprocess
    import sys

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted((d["rank"], d["local_rank"], d["world_size"]) for d in lines) == [(0, 0, 2), (1, 1, 2)]


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu_with_gloo():
    """The N > 1 bench path end to end on one GPU (both ranks share cuda:0;
    gloo instead of RCCL, which needs one GPU per rank): per-rank decode,
    max-over-ranks timing, the shared-host concat; one JSON line from rank 0."""
    import json
    import subprocess
    import sys

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                          "--rows", "2000000", "--steps", "3", "--warmup", "2", "--no-cpu-baseline",
                          "--copy-inclusive", "0"], capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "ms" in d["concat"]["host"], d["concat"]


@pytest.mark.gpu
def test_bench_file_two_ranks_sharded_c4():
    """configs[3] sharded over two ranks (both on cuda:0, gloo): each rank
    decodes its contiguous stripe range (RowReaderOptions::range,
    c++/src/Reader.cc:337-345) and checks its first and last stripe against
    pyarrow; the timed concat assembles l_orderkey in one shared host batch
    that rank 0 checks against pyarrow; the JSON line reports the decode and
    the concat separately."""
    import json
    import subprocess
    import sys

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    path = os.path.join("/tmp", "orcg_test_c4_2m_%d.orc" % os.getpid())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "scripts", "bench_file.py"),
           "--workload", "c4", "--rows", "2000000", "--stripe-mb", "4", "--iters", "1", "--backend", "gloo",
           "--no-cpu-baseline", "--path", path]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = lines[0]
    assert d["config"]["n_gpus"] == 2 and d["config"]["stripes"] >= 4
    assert d["concat"]["checked_against_pyarrow"] and d["concat"]["rows"] == 2_000_000
    assert d["wall_s"] > 0 and d["concat"]["ms"] > 0
