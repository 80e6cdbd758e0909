"""Stream ordering of the C ABI's *_device entries (include/orcg.h, the
contract under orcg_ctx_set_stream), exercised through the raw C calls
rather than the Python wrappers, which add their own ordering
(Context.after_torch):

  * with the producer's stream handed to orcg_ctx_set_stream, the decode is
    queued behind a slow producer chain that writes its output buffer, and a
    consumer queued on the same stream sees the decoded values;
  * with the context's own (non-blocking) stream, a caller that records an
    event on its producer stream and makes orcg_ctx_stream() wait on it gets
    the same result.

The producer's last step overwrites every output slot with garbage, so a
decode that overtook it would leave garbage behind.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, STRIDE = 4_000_000, 10_000


def _producer(torch, out, s):
    """Queue ~ms of work on s that ends by filling `out` with garbage."""
    with torch.cuda.stream(s):
        a = torch.randn(2048, 2048, device="cuda")
        for _ in range(24):
            a = torch.tanh(a @ a)
        out.fill_(-7)
        out.add_((a[0, 0] * 0).to(torch.int64))  # depends on the chain


def _decode_raw(L, ctx, src, pos, out):
    rc = L.orcg_rlev2_decode_positions_device(ctx.handle, ctypes.c_void_p(src.data_ptr()), src.numel(), 1,
                                              ctypes.c_void_p(pos.data_ptr()), pos.shape[0], STRIDE, 0, N,
                                              ctypes.c_void_p(out.data_ptr()), 8)
    assert rc == 0


@pytest.fixture(scope="module")
def stream_case():
    import torch

    import orc_amd

    rng = np.random.default_rng(7)
    v = rng.integers(-(1 << 40), 1 << 40, size=N, dtype=np.int64)
    data, pos = orc_amd.encode_direct(v, True, aligned=True, rows_per_group=STRIDE)
    return (torch.from_numpy(v).cuda(), torch.from_numpy(data).cuda(),
            torch.from_numpy(pos.view(np.int64)).cuda())


def test_external_stream_orders_decode_after_producer(stream_case):
    import torch

    import orc_amd
    from orc_amd import _lib

    L = _lib.load()
    v, src, pos = stream_case
    torch.cuda.synchronize()
    ctx = orc_amd.Context(0)
    s = torch.cuda.Stream()
    try:
        assert L.orcg_ctx_set_stream(ctx.handle, ctypes.c_void_p(s.cuda_stream)) == 0
        assert ctx.stream_ptr() == s.cuda_stream
        out = torch.empty(N, dtype=torch.int64, device="cuda")
        for _ in range(3):
            _producer(torch, out, s)
            _decode_raw(L, ctx, src, pos, out)
            with torch.cuda.stream(s):
                eq = torch.equal(out, v)  # consumer on the same stream
            assert eq
        assert L.orcg_ctx_synchronize(ctx.handle) == 0
    finally:
        L.orcg_ctx_set_stream(ctx.handle, None)
        ctx.close()


def test_own_stream_ordered_by_event_wait(stream_case):
    import torch

    import orc_amd
    from orc_amd import _lib

    L = _lib.load()
    v, src, pos = stream_case
    torch.cuda.synchronize()
    ctx = orc_amd.Context(0)
    s = torch.cuda.Stream()
    try:
        own = ctx.stream_ptr()
        assert own and own != s.cuda_stream
        ext = torch.cuda.ExternalStream(own)
        out = torch.empty(N, dtype=torch.int64, device="cuda")
        for _ in range(3):
            _producer(torch, out, s)
            ev = torch.cuda.Event()
            ev.record(s)
            ext.wait_event(ev)  # hipStreamWaitEvent(orcg_ctx_stream(ctx), ev, 0)
            _decode_raw(L, ctx, src, pos, out)
            assert L.orcg_ctx_synchronize(ctx.handle) == 0
            assert torch.equal(out, v)
    finally:
        ctx.close()
