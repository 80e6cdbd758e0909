"""RLEv1 on the GPU (rlev1_kernel through orcg_rlev1_*): the reference's
RLEv1 known-answer tests (c++/test/TestRleDecoder.cc, TEST(RLEv1, ...)),
random run/literal mixes checked bit-exactly against the oracle
(oracle/orc_oracle.c, RLEv1.cc:140-300 restated), device row ranges and the
reference's truncation error."""
import numpy as np
import pytest

import orc_amd
from conftest import load_golden
from oracle import oracle
from rlev1_writer import encode, random_groups

pytestmark = pytest.mark.gpu

RLEV1 = load_golden("kat_rlev1.json")


@pytest.fixture(scope="module")
def ctx():
    return orc_amd.Context(0)


@pytest.mark.parametrize("fx", RLEV1, ids=[f["name"] for f in RLEV1])
def test_rlev1_kat(ctx, fx):
    data = bytes.fromhex(fx["data"])
    exp = fx["expected"]
    nn = fx.get("not_null")
    nnv = None if nn is None else np.array(nn, dtype=np.uint8)
    got = orc_amd.rlev1_decode(data, len(exp), fx["signed"], not_null=nnv, ctx=ctx)
    for i, e in enumerate(exp):
        if e is not None:
            assert int(got[i]) == e, "%s at %d" % (fx["name"], i)
    for sk in fx.get("seeks", []):
        off, skip = sk["position"]
        k = skip + len(sk["expected"])
        got = orc_amd.rlev1_decode(data[off:], k, fx["signed"], ctx=ctx)
        assert list(int(x) for x in got[skip:]) == sk["expected"]


@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("max_bits", [7, 14, 35, 64])
def test_rlev1_random_vs_oracle(ctx, signed, max_bits):
    rng = np.random.default_rng(1000 + max_bits + int(signed))
    data, vals = encode(random_groups(rng, 200_000, signed, max_bits), signed)
    want = oracle.RleDecoderV1(data, signed).next(vals.size)
    np.testing.assert_array_equal(want, vals)
    got = orc_amd.rlev1_decode(data, vals.size, signed, ctx=ctx)
    np.testing.assert_array_equal(got, want)
    # with nulls: values land on the non-null rows, null slots untouched (0)
    nn = (rng.random(vals.size * 2) < 0.5).astype(np.uint8)
    nn[np.flatnonzero(nn)[vals.size:]] = 0
    k = int(nn.sum())
    got = orc_amd.rlev1_decode(data, nn.size, signed, not_null=nn, ctx=ctx)
    np.testing.assert_array_equal(got[nn.astype(bool)], want[:k])
    assert not got[~nn.astype(bool)].any()


def test_rlev1_long_literal_groups(ctx):
    # 128 ten-byte varints per group: literal chunks span many 64-byte windows
    rng = np.random.default_rng(7)
    groups = [("lit", [int(x) for x in rng.integers(-(1 << 63), (1 << 63) - 1, size=128, dtype=np.int64)])
              for _ in range(300)]
    data, vals = encode(groups, True)
    got = orc_amd.rlev1_decode(data, vals.size, True, ctx=ctx)
    np.testing.assert_array_equal(got, vals)


def test_rlev1_device_ranges(ctx):
    import torch
    rng = np.random.default_rng(3)
    data, vals = encode(random_groups(rng, 100_000, True, 40), True)
    plan_h = orc_amd.rle._lib.load()
    import ctypes
    h = ctypes.c_void_p()
    buf = np.frombuffer(data, dtype=np.uint8)
    orc_amd.rle.check(plan_h.orcg_rlev1_plan_create(buf.ctypes.data_as(ctypes.c_void_p), buf.size, 2048, 1000,
                                                    ctypes.byref(h)))
    segp = ctypes.c_void_p()
    nseg = plan_h.orcg_rlev2_plan_segments(h, ctypes.byref(segp))
    assert plan_h.orcg_rlev2_plan_values(h) == vals.size and nseg > 10
    segs = np.ctypeslib.as_array(ctypes.cast(segp, ctypes.POINTER(ctypes.c_uint64)), shape=(nseg * 2,)).copy()
    plan_h.orcg_rlev2_plan_destroy(h)
    d_src = torch.from_numpy(buf.copy()).cuda()
    d_seg = torch.from_numpy(segs.view(np.int64)).cuda()
    for begin, count in [(0, vals.size), (12345, 777), (vals.size - 5, 5), (999, 1)]:
        out = torch.zeros(count, dtype=torch.int64, device="cuda")
        orc_amd.rle.check(plan_h.orcg_rlev1_decode_device(ctx.handle, d_src.data_ptr(), buf.size, 1, d_seg.data_ptr(),
                                                          nseg, begin, count, out.data_ptr(), 8), ctx.last_error)
        ctx.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), vals[begin:begin + count])


def test_rlev1_truncated_stream_raises_reference_error(ctx):
    data, vals = encode([("lit", [1 << 40] * 10), ("run", 5, 1, 10)], False)
    with pytest.raises(orc_amd.ParseError, match="bad read in readByte"):
        orc_amd.rlev1_decode(data[:-1], vals.size, False, ctx=ctx)
    # values before the corrupt run still decode
    got = orc_amd.rlev1_decode(data[:-1], 10, False, ctx=ctx)
    np.testing.assert_array_equal(got, vals[:10])
