"""Stripe sharding across GPUs (one process per GPU).

ORC stripes decode independently (site/_docs/index.md:33-35), so a file is
split into contiguous stripe ranges balanced by stripe bytes, the way
RowReaderOptions::range selects the stripes whose start falls in a byte range
(c++/src/Reader.cc:337-345). Each rank decodes its range with no data-path
collective. The only exchange is the final concat of a column
(SURVEY.md §8e): either each rank copies its rows into its own slice of one
host batch (no collective; offsets from an all-gather of row counts), or the
shards are gathered to a root rank over RCCL point-to-point send/recv
(xGMI links), which `gather_to_root` does. `write_rows_to_shared_host` is
the first: one host batch in shared memory that every rank maps and fills
with a D2H copy of its own rows (pinned with hipHostRegister for the copy).
"""
import os

import numpy as np


def partition_stripes(stripe_bytes, world):
    """Contiguous [begin, end) stripe ranges, one per rank, with cut points
    at the stripe boundaries closest to k * total / world."""
    n = len(stripe_bytes)
    if world <= 0:
        raise ValueError("world must be positive")
    if n == 0:
        return [(0, 0)] * world
    cum = np.concatenate([[0], np.cumsum(np.asarray(stripe_bytes, dtype=np.float64))])
    total = cum[-1]
    cuts = [0]
    for k in range(1, world):
        target = total * k / world
        j = int(np.argmin(np.abs(cum - target)))
        j = max(j, cuts[-1])
        cuts.append(min(j, n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def range_rows(stripe_rows, rng):
    b, e = rng
    return int(sum(stripe_rows[b:e]))


def row_offsets(stripe_rows, ranges):
    """Global index of each rank's first row (exclusive scan of range rows)."""
    sizes = [range_rows(stripe_rows, r) for r in ranges]
    return [int(x) for x in np.concatenate([[0], np.cumsum(sizes)[:-1]])], sizes


def reader_ranges(reader, world):
    """partition_stripes over an orc_amd.Reader's stripes (index + data + footer bytes)."""
    sb, rows = [], []
    for s in range(reader.num_stripes):
        st = reader.stripe(s)
        sb.append(st["index_length"] + st["data_length"] + st["footer_length"])
        rows.append(st["num_rows"])
    return partition_stripes(sb, world), rows


def _count_device(dist, tensor):
    """Where small control tensors live for this backend (RCCL needs device
    tensors, gloo takes host ones)."""
    import torch

    if dist.get_backend() == "nccl":
        return tensor.device if tensor.is_cuda else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_row_counts(dist, tensor):
    """Every rank's row count, in rank order (one all-gather of a scalar)."""
    import torch

    dev = _count_device(dist, tensor)
    n = torch.tensor([tensor.numel()], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
    dist.all_gather(counts, n)
    return [int(c.item()) for c in counts]


def write_rows_to_shared_host(dist, tensor, path, create):
    """Concat without a data collective: every rank copies its 1-D `tensor`
    (device or host) into its own slice [offset, offset + n) of one host
    batch backed by the shared-memory file `path` (created and sized by the
    rank with `create`); offsets come from an all-gather of the row counts.
    Returns the whole batch (a host tensor over the shared mapping) once
    every rank's slice has landed."""
    import torch

    counts = all_row_counts(dist, tensor)
    rank = dist.get_rank()
    total = sum(counts)
    itemsize = tensor.element_size()
    if create:
        with open(path, "wb") as f:
            f.truncate(max(total * itemsize, 1))
    dist.barrier()
    host = torch.from_file(path, shared=True, size=max(total, 1), dtype=tensor.dtype)[:total]
    off = int(sum(counts[:rank]))
    view = host[off:off + counts[rank]]
    if counts[rank]:
        if tensor.is_cuda:
            from . import _lib

            L = _lib.load()
            nbytes = counts[rank] * itemsize
            pinned = L.orcg_host_register(view.data_ptr(), nbytes) == 0
            try:
                view.copy_(tensor, non_blocking=pinned)
                torch.cuda.current_stream().synchronize()
            finally:
                if pinned:
                    L.orcg_host_unregister(view.data_ptr())
        else:
            view.copy_(tensor)
    dist.barrier()
    return host


def gather_to_root(dist, tensor, root=0):
    """Concatenate each rank's 1-D `tensor` on `root` in rank order with
    point-to-point send/recv (RCCL over xGMI for CUDA tensors, gloo on CPU).
    Returns the concatenation on root, None elsewhere."""
    import torch

    world = dist.get_world_size()
    rank = dist.get_rank()
    counts = all_row_counts(dist, tensor)
    if rank != root:
        if tensor.numel():
            dist.send(tensor.contiguous(), dst=root)
        return None
    out = torch.empty(sum(counts), dtype=tensor.dtype, device=tensor.device)
    offs = np.concatenate([[0], np.cumsum(counts)])
    reqs = []
    for r in range(world):
        view = out[int(offs[r]):int(offs[r + 1])]
        if r == root:
            view.copy_(tensor)
        elif counts[r]:
            reqs.append(dist.irecv(view, src=r))
    for q in reqs:
        q.wait()
    return out
