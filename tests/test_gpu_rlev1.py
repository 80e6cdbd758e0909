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


def _padded_varint(u, nbytes):
    """A base-128 varint of exactly nbytes bytes (continuation bytes past the
    value's own carry zeros): legal for readLong (RLEv1.cc:154-170), which
    keeps reading until a byte below 0x80; bits past 64 are dropped."""
    out = []
    for i in range(nbytes):
        b = (u >> (7 * i)) & 0x7F if 7 * i < 64 else 0
        out.append(b | (0x80 if i + 1 < nbytes else 0))
    return out


@pytest.mark.parametrize("nbytes", [11, 16, 40])
def test_rlev1_overlong_varints_vs_oracle(ctx, nbytes):
    # literal groups whose varints run past 10 bytes: 128 x 40 bytes is longer
    # than a whole LDS window (the kernel's serial fallback), 11 / 16 bytes
    # cross the window tail and the chunk prologue
    rng = np.random.default_rng(nbytes)
    data = bytearray()
    for g in range(6):
        k = 128 if g % 2 == 0 else int(rng.integers(1, 128))
        data.append(256 - k)
        for _ in range(k):
            data += bytes(_padded_varint(int(rng.integers(0, 1 << 62)), nbytes if rng.random() < 0.7 else 2))
        data += bytes([5, 3, 7])  # a run of 8: base 7, delta 3
    data = bytes(data)
    total = 0
    probe = oracle.RleDecoderV1(data, False)
    # count the values by decoding until the stream ends
    while True:
        try:
            probe.next(1)
            total += 1
        except Exception:
            break
    want = oracle.RleDecoderV1(data, False).next(total)
    got = orc_amd.rlev1_decode(data, total, False, ctx=ctx)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("cut", [4000, 4097, 5000, 9000, 12001])
def test_rlev1_truncated_in_a_later_window(ctx, cut):
    # a stream cut at `cut` bytes: every whole value before the cut decodes,
    # the first value the cut makes unreadable raises the reference's error
    rng = np.random.default_rng(cut)
    data, vals = encode(random_groups(rng, 20_000, True, 30), True)
    data = data[:cut]
    dec = oracle.RleDecoderV1(data, True)
    ok = 0
    while True:
        try:
            dec.next(1)
            ok += 1
        except Exception:
            break
    got = orc_amd.rlev1_decode(data, ok, True, ctx=ctx)
    np.testing.assert_array_equal(got, vals[:ok])
    with pytest.raises(orc_amd.ParseError, match="bad read in readByte"):
        orc_amd.rlev1_decode(data, ok + 1, True, ctx=ctx)


@pytest.mark.parametrize("shape", ["dict", "runs", "wide"])
@pytest.mark.parametrize("seg_bytes", [64, 1000, 4096, 5000, 1 << 20])
def test_rlev1_segment_sizes(ctx, shape, seg_bytes):
    # host plans cut the stream into segments of every size around the
    # kernel's 4 KB window: each workgroup's windows, chunk prologues and
    # run / literal splits must agree with one serial decode
    import ctypes
    import torch
    rng = np.random.default_rng(len(shape) * 7 + seg_bytes)
    if shape == "dict":
        v = rng.integers(0, 7, size=30_000)
        groups = [("lit", [int(x) for x in v[i:i + 128]]) for i in range(0, v.size, 128)]
    elif shape == "runs":
        groups = [("run", int(rng.integers(0, 1 << 40)), int(rng.integers(-128, 128)), int(rng.integers(3, 131)))
                  for _ in range(800)]
    else:
        groups = random_groups(rng, 30_000, True, 64)
    data, vals = encode(groups, True)
    L = orc_amd.rle._lib.load()
    buf = np.frombuffer(data, dtype=np.uint8)
    h = ctypes.c_void_p()
    orc_amd.rle.check(L.orcg_rlev1_plan_create(buf.ctypes.data_as(ctypes.c_void_p), buf.size, seg_bytes, 1 << 40,
                                               ctypes.byref(h)))
    segp = ctypes.c_void_p()
    nseg = L.orcg_rlev2_plan_segments(h, ctypes.byref(segp))
    segs = np.ctypeslib.as_array(ctypes.cast(segp, ctypes.POINTER(ctypes.c_uint64)), shape=(nseg * 2,)).copy()
    L.orcg_rlev2_plan_destroy(h)
    d_src = torch.from_numpy(buf.copy()).cuda()
    d_seg = torch.from_numpy(segs.view(np.int64)).cuda()
    out = torch.zeros(vals.size, dtype=torch.int64, device="cuda")
    orc_amd.rle.check(L.orcg_rlev1_decode_device(ctx.handle, d_src.data_ptr(), buf.size, 1, d_seg.data_ptr(), nseg,
                                                 0, vals.size, out.data_ptr(), 8), ctx.last_error)
    ctx.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), vals)
