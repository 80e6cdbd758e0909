"""Synthetic RLEv2 streams for the A/B and profiling scripts: random values
DIRECT-encoded at a width, or structured columns through the explicit run
builder (orc_amd.encode_runs), with row-index positions every `stride`
values (run-aligned byte offset + values to skip)."""
import numpy as np

KINDS = ["random", "delta", "repeat", "patched", "shortdirect", "shortmix"]


def make(kind, bits, n, stride, seed=42):
    """Returns (values int64[n'], stream bytes uint8, positions uint64[G, 2])."""
    import orc_amd

    rng = np.random.default_rng(seed)
    if kind == "random":
        if bits == 64:
            v = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64, endpoint=True)
        else:
            v = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), size=n, dtype=np.int64)
        data, pos = orc_amd.encode_direct(v, True, aligned=True, rows_per_group=stride)
    else:
        # structured columns through the run builder: sorted keys (DELTA
        # runs of 512), low-cardinality repeats (SHORT_REPEAT runs of 3-10),
        # small values with outliers (PATCHED_BASE runs of 512)
        if kind == "delta":
            lens = np.full(n // 512, 512, dtype=np.uint32)
            kinds = np.full(lens.size, 3, dtype=np.uint8)
            v = np.cumsum(rng.integers(0, 1 << bits, size=n, dtype=np.int64)) + 1_000_000
        elif kind == "repeat":
            lens = rng.integers(3, 11, size=n // 6 + 16).astype(np.uint32)
            lens = lens[: np.searchsorted(np.cumsum(lens), n) + 1]
            lens[-1] -= np.cumsum(lens)[-1] - n
            if lens[-1] < 3:
                lens = lens[:-1]
                n = int(lens.sum())
            kinds = np.zeros(lens.size, dtype=np.uint8)
            v = np.repeat(rng.integers(-(1 << (bits - 1)), (1 << (bits - 1)) - 1, size=lens.size,
                                       dtype=np.int64, endpoint=True), lens)
        elif kind == "shortdirect":
            # short DIRECT runs (1-10 values) of --bits-wide values: the shape
            # a writer emits between repeats of a high-cardinality column
            lens = rng.integers(1, 11, size=n // 5 + 16).astype(np.uint32)
            lens = lens[: np.searchsorted(np.cumsum(lens), n)]
            kinds = np.ones(lens.size, dtype=np.uint8)
            n = int(lens.sum())
            if bits == 64:
                v = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64, endpoint=True)
            else:
                v = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), size=n, dtype=np.int64)
        elif kind == "shortmix":
            # alternating SHORT_REPEAT (3-10) and short DIRECT (1-10) runs
            nr = n // 6 + 16
            kinds = (np.arange(nr) % 2).astype(np.uint8)
            lens = np.where(kinds == 0, rng.integers(3, 11, size=nr), rng.integers(1, 11, size=nr)).astype(np.uint32)
            cut = np.searchsorted(np.cumsum(lens), n)
            lens, kinds = lens[:cut], kinds[:cut]
            n = int(lens.sum())
            lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
            rv = rng.integers(lo, hi, size=lens.size, dtype=np.int64, endpoint=True)
            v = np.repeat(rv, lens)
            dmask = np.repeat(kinds == 1, lens)
            v[dmask] = rng.integers(lo, hi, size=int(dmask.sum()), dtype=np.int64, endpoint=True)
        else:
            lens = np.full(n // 512, 512, dtype=np.uint32)
            kinds = np.full(lens.size, 2, dtype=np.uint8)
            v = rng.integers(0, 1 << bits, size=n, dtype=np.int64)
            out = rng.random(n) < 0.004
            v[out] += rng.integers(1 << 40, 1 << 44, size=int(out.sum()))
            v[::512] = 0  # keep a small base per run
            v[100::512] += 1 << 41  # and at least one patch (pl == 0 is corrupt)
        n = int(lens.sum())
        v = v[:n].astype(np.int64)
        data, offs = orc_amd.encode_runs(v, True, kinds, lens)
        # positions: first run of every row group (stride-aligned run starts)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        g = np.arange(0, n, stride)
        ri = np.searchsorted(starts, g, side="right") - 1
        pos = np.stack([offs[ri].astype(np.uint64), (g - starts[ri]).astype(np.uint64)], axis=1)
    return v, data, pos
