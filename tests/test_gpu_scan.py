"""The reader's int64 exclusive scan (list / map lengths -> offsets,
ListColumnReader::nextInternal, c++/src/ColumnReader.cc:960-993; direct string
lengths -> starts, :725-793): the single-pass decoupled look-back kernel
against numpy at tile edges and large sizes (4,096 values a tile), and the
one-workgroup path below 8,192 values."""
import ctypes

import numpy as np
import pytest

import orc_amd

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 4095, 8192, 8193, 4096 * 3, 4096 * 3 + 1, 1_000_003, 2_634_752])
def test_exclusive_scan_matches_numpy(n):
    import torch

    L = orc_amd._lib.load()
    f = L.orcg_debug_exclusive_scan
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    ctx = orc_amd.Context(0)
    rng = np.random.default_rng(n)
    x = rng.integers(0, 1 << 20, size=n, dtype=np.int64)
    if n > 10:
        x[rng.integers(0, n, size=3)] = 1 << 40  # large lengths carry across tiles
    d_in = torch.from_numpy(x).cuda()
    d_out = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for _ in range(2):  # the status words are reset per launch
        orc_amd.rle.check(f(ctx.handle, d_in.data_ptr() if n else None, n, d_out.data_ptr()), ctx.last_error)
        ctx.synchronize()
        want = np.concatenate([[0], np.cumsum(x)]).astype(np.int64)
        np.testing.assert_array_equal(d_out.cpu().numpy(), want)


def _scan(ctx, x):
    import torch

    L = orc_amd._lib.load()
    f = L.orcg_debug_exclusive_scan
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    n = x.size
    d_in = torch.from_numpy(x).cuda()
    d_out = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    orc_amd.rle.check(f(ctx.handle, d_in.data_ptr(), n, d_out.data_ptr()), ctx.last_error)
    ctx.synchronize()
    return d_out.cpu().numpy()


@pytest.mark.parametrize("big", [(1 << 46) + 5, (1 << 47) - 3, (1 << 62) + 11, -(1 << 50), (1 << 63) - 1])
def test_exclusive_scan_exact_for_any_int64(big):
    """The look-back status carries the whole 64-bit value (two tagged words
    per tile): a length of 2^46 or more in an early tile, a negative one
    (a corrupt unsigned length read as int64) and a sum that wraps past
    2^63 all reach the later tiles exactly, equal to numpy's wrapping int64
    cumsum (the reference sums int64, ColumnReader.cc:960-993)."""
    ctx = orc_amd.Context(0)
    n = 4096 * 40 + 17
    rng = np.random.default_rng(abs(big) % 1000)
    x = rng.integers(0, 1 << 20, size=n, dtype=np.int64)
    x[4096 * 2 + 7] = big  # a non-final tile
    x[4096 * 9 + 1] = big
    x[4096 * 33] = (1 << 45) + 1
    with np.errstate(over="ignore"):
        want = np.concatenate([[0], np.cumsum(x)]).astype(np.int64)
    np.testing.assert_array_equal(_scan(ctx, x), want)


def test_exclusive_scan_epoch_wrap():
    """The look-back status words carry a 16-bit launch epoch (no clearing
    launch); past 65,535 launches on one context the buffer is cleared once
    and the epochs restart: results stay exact across the wrap (the test
    hook starts the context's epochs just below the wrap)."""
    L = orc_amd._lib.load()
    L.orcg_debug_set_lb_epoch.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    ctx = orc_amd.Context(0)
    n = 3 * 4096 + 5
    x = np.arange(n, dtype=np.int64) % 7
    want = np.concatenate([[0], np.cumsum(x)]).astype(np.int64)
    np.testing.assert_array_equal(_scan(ctx, x), want)  # allocates the status words
    assert L.orcg_debug_set_lb_epoch(ctx.handle, 0xfffc) == 0
    for i in range(8):  # epochs 0xfffd .. 0xffff, the clear, then 1 .. 4
        np.testing.assert_array_equal(_scan(ctx, x + i), np.concatenate([[0], np.cumsum(x + i)]).astype(np.int64))
