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
