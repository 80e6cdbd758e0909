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


def test_exclusive_scan_epoch_wrap():
    """The look-back status words carry a 16-bit launch epoch (no clearing
    launch); past 65,535 launches on one context the buffer is cleared once
    and the epochs restart: results stay exact across the wrap."""
    import torch

    L = orc_amd._lib.load()
    f = L.orcg_debug_exclusive_scan
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    ctx = orc_amd.Context(0)
    n = 3 * 4096 + 5
    x = np.arange(n, dtype=np.int64) % 7
    d_in = torch.from_numpy(x).cuda()
    d_out = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    want = np.concatenate([[0], np.cumsum(x)]).astype(np.int64)
    for i in range(66_000):
        rc = f(ctx.handle, d_in.data_ptr(), n, d_out.data_ptr())
        assert rc == 0, ctx.last_error
        if i in (0, 65_533, 65_534, 65_535, 65_999):
            ctx.synchronize()
            np.testing.assert_array_equal(d_out.cpu().numpy(), want)
