"""GPU parity for byte / boolean RLE (PRESENT streams), the null scatter and
the string-dictionary gather, against the reference's KATs and the oracle."""
import numpy as np
import pytest

from conftest import assert_matches, decode_batches, load_golden
from oracle import oracle

pytestmark = pytest.mark.gpu

BYTE = load_golden("kat_byterle.json")
BOOL = load_golden("kat_boolrle.json")


@pytest.fixture(scope="module")
def orc():
    import orc_amd

    orc_amd.default_context(0)
    return orc_amd


def byte_rle_encode(data, rng):
    """Writer-side helper (ORCv1.md:672-687): random split into runs/literals."""
    out = bytearray()
    i, n = 0, len(data)
    while i < n:
        j = i
        while j < n and j - i < 130 and data[j] == data[i]:
            j += 1
        if j - i >= 3:
            out += bytes([j - i - 3, data[i]])
            i = j
            continue
        k = min(n - i, int(rng.integers(1, 129)))
        # stop a literal before a run of 3
        m = i
        while m < i + k:
            if m + 2 < n and data[m] == data[m + 1] == data[m + 2]:
                break
            m += 1
        if m == i:
            m = i + 1
        out += bytes([256 - (m - i)]) + bytes(data[i:m])
        i = m
    return bytes(out)


def random_bytes(rng, n):
    parts = []
    while sum(len(p) for p in parts) < n:
        if rng.random() < 0.5:
            parts.append(bytes([int(rng.integers(0, 256))]) * int(rng.integers(3, 300)))
        else:
            parts.append(rng.integers(0, 256, size=int(rng.integers(1, 300)), dtype=np.uint8).tobytes())
    return b"".join(parts)[:n]


@pytest.mark.parametrize("fx", BYTE, ids=[f["name"] for f in BYTE])
def test_byterle_kat(orc, fx):
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    for b in fx["batches"]:
        dec = orc.create_byte_rle_decoder(data)
        got = decode_batches(dec.next, fx["expected"], b, nn)
        assert_matches(fx["expected"], got, nn, fx["name"])


@pytest.mark.parametrize("fx", BOOL, ids=[f["name"] for f in BOOL])
def test_boolrle_kat(orc, fx):
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    for b in fx["batches"]:
        dec = orc.create_boolean_rle_decoder(data)
        got = decode_batches(dec.next, fx["expected"], b, nn)
        assert_matches(fx["expected"], got, nn, fx["name"])


@pytest.mark.parametrize("boolean", [False, True])
@pytest.mark.parametrize("seed", range(4))
def test_random_streams_vs_oracle(orc, boolean, seed):
    rng = np.random.default_rng(seed)
    raw = random_bytes(rng, 50_000)
    enc = byte_rle_encode(raw, rng)
    units = len(raw) * (8 if boolean else 1)
    # random nulls, random batch sizes, with skips
    od = oracle.ByteRleDecoder(enc, boolean=boolean)
    gd = orc.ByteRleDecoder(enc, boolean=boolean)
    consumed = 0
    while consumed < units - 2000:
        k = int(rng.integers(1, 1500))
        if rng.random() < 0.1:
            s = int(rng.integers(0, 100))
            od.skip(s)
            gd.skip(s)
            consumed += s
            continue
        nn = (rng.random(k) > 0.3).astype(np.uint8)
        w = od.next(k, nn)
        g = gd.next(k, nn)
        if boolean:
            np.testing.assert_array_equal(g, w)  # null slots are 0 in both
        else:
            np.testing.assert_array_equal(g[nn == 1], w[nn == 1])
        consumed += int(nn.sum())


def test_seek_matches_oracle(orc):
    rng = np.random.default_rng(9)
    raw = random_bytes(rng, 20_000)
    enc = byte_rle_encode(raw, rng)
    plan = orc.BytePlan(enc, max_segment_bytes=200, max_segment_values=500)
    segs = plan.segments()
    for boolean in (False, True):
        for b, vi in segs[:: max(1, len(segs) // 15)]:
            for skip in (0, 3):
                pos = [int(b), skip] + ([5] if boolean else [])
                od = oracle.ByteRleDecoder(enc, boolean=boolean)
                gd = orc.ByteRleDecoder(enc, boolean=boolean)
                od.seek(*pos)
                gd.seek(*pos)
                np.testing.assert_array_equal(gd.next(100), od.next(100))


@pytest.mark.parametrize("boolean", [False, True])
def test_device_decode_ranges(orc, boolean):
    import torch

    rng = np.random.default_rng(4)
    raw = random_bytes(rng, 300_000)
    enc = byte_rle_encode(raw, rng)
    plan = orc.BytePlan(enc, max_segment_bytes=4096, max_segment_values=8192)
    segs = torch.from_numpy(plan.segments().view(np.int64)).cuda()
    src = torch.from_numpy(np.frombuffer(enc, dtype=np.uint8).copy()).cuda()
    ctx = orc.default_context(0)
    raw_np = np.frombuffer(raw, dtype=np.uint8)
    full = np.unpackbits(raw_np) if boolean else raw_np
    for a, b in [(0, full.size), (1, 12_345), (full.size - 77, full.size), (8_191, 8_203)]:
        out = torch.zeros(b - a, dtype=torch.uint8, device="cuda")
        orc.byterle_decode_device(ctx, src, segs, b - a, out, value_begin=a, boolean=boolean)
        ctx.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), full[a:b])


@pytest.mark.parametrize("width,dtype", [(8, "int64"), (4, "int32"), (2, "int16"), (1, "int8")])
def test_scatter_not_null(orc, width, dtype):
    import torch

    rng = np.random.default_rng(width)
    n = 1_000_003
    nn = (rng.random(n) > 0.37).astype(np.uint8)
    k = int(nn.sum())
    dense = rng.integers(-100, 100, size=k).astype(dtype)
    ctx = orc.default_context(0)
    sentinel = np.full(n, 55, dtype=dtype)
    out = torch.from_numpy(sentinel.copy()).cuda()
    orc.scatter_not_null_device(ctx, torch.from_numpy(dense).cuda(), torch.from_numpy(nn).cuda(), out)
    ctx.synchronize()
    want = sentinel.copy()
    want[nn == 1] = dense
    np.testing.assert_array_equal(out.cpu().numpy(), want)
    orc.scatter_not_null_device(ctx, torch.from_numpy(dense).cuda(), torch.from_numpy(nn).cuda(), out, fill=1)
    ctx.synchronize()
    want[nn == 0] = 1
    np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_dictionary_gather(orc):
    import torch

    rng = np.random.default_rng(5)
    lengths = rng.integers(0, 40, size=5000).astype(np.int64)
    n = 200_000
    idx = rng.integers(0, lengths.size, size=n).astype(np.int64)
    nn = (rng.random(n) > 0.2).astype(np.uint8)
    ws, wl = oracle.dict_gather(idx, lengths, nn)
    ctx = orc.default_context(0)
    d_len = torch.from_numpy(lengths).cuda()
    d_off = torch.empty(lengths.size + 1, dtype=torch.int64, device="cuda")
    orc.dict_offsets_device(ctx, d_len, d_off)
    start = torch.zeros(n, dtype=torch.int64, device="cuda")
    length = torch.zeros(n, dtype=torch.int64, device="cuda")
    orc.dict_gather_device(ctx, torch.from_numpy(idx).cuda(), d_off, start, length,
                           not_null=torch.from_numpy(nn).cuda())
    ctx.synchronize()
    m = nn == 1
    np.testing.assert_array_equal(start.cpu().numpy()[m], ws[m])
    np.testing.assert_array_equal(length.cpu().numpy()[m], wl[m])
    # out-of-range index: the reference's error (ColumnReader.cc:578)
    bad = idx.copy()
    bad[123] = lengths.size
    orc.dict_gather_device(ctx, torch.from_numpy(bad).cuda(), d_off, start, length)
    with pytest.raises(orc.ParseError, match="Entry index out of range in StringDictionaryColumn"):
        ctx.synchronize()


def test_integer_column_with_present(orc):
    rng = np.random.default_rng(6)
    n = 100_000
    nn = (rng.random(n) > 0.1).astype(np.uint8)
    vals = rng.integers(-(1 << 40), 1 << 40, size=int(nn.sum()))
    data, _ = orc.encode_direct(vals, True, aligned=False)
    present = byte_rle_encode(np.packbits(nn).tobytes(), rng)
    # oracle: boolean decoder for PRESENT, then RLEv2 with notNull
    onn = oracle.ByteRleDecoder(present, boolean=True).next(n)
    ovals = oracle.RleDecoderV2(data.tobytes(), True).next(n, onn)
    got, gnn = orc.decode_integer_column(present, data.tobytes(), n, True)
    np.testing.assert_array_equal(gnn, onn)
    np.testing.assert_array_equal(got[gnn == 1], ovals[onn == 1])
    assert np.all(got[gnn == 0] == 0)  # untouched (zero-initialised) slots


def _present_like(rng, nrows, null_frac):
    """PRESENT-shaped bits (the reference writer's byte RLE of them): random
    nulls at `null_frac`, so most groups are short runs of 0xFF and short
    literals (~4-5 stream bytes per group at 10 %)."""
    bits = (rng.random(nrows) >= null_frac).astype(np.uint8)
    return bits, np.packbits(bits).tobytes()


@pytest.mark.parametrize("null_frac", [0.0, 0.01, 0.1, 0.5, 0.97])
@pytest.mark.parametrize("seg_bytes", [300, 4096, 20000, 1 << 30])
def test_boolean_segments_of_every_size(orc, null_frac, seg_bytes):
    """The parallel group discovery over windows of every fill (segments
    shorter than a window, several windows per segment, one segment for the
    whole stream) on PRESENT-shaped data, plus the set-row count the file
    reader takes its non-null counts from."""
    import ctypes

    import torch

    rng = np.random.default_rng(int(null_frac * 100) + seg_bytes % 97)
    bits, raw = _present_like(rng, 400_003, null_frac)
    enc = byte_rle_encode(raw, rng)
    plan = orc.BytePlan(enc, max_segment_bytes=seg_bytes, max_segment_values=1 << 40)
    segs = torch.from_numpy(plan.segments().view(np.int64)).cuda()
    src = torch.from_numpy(np.frombuffer(enc, dtype=np.uint8).copy()).cuda()
    ctx = orc.default_context(0)
    full = np.unpackbits(np.frombuffer(raw, dtype=np.uint8))
    n = bits.size
    out = torch.zeros(n, dtype=torch.uint8, device="cuda")
    orc.byterle_decode_device(ctx, src, segs, n, out, boolean=True)
    ctx.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), full[:n])
    # decoded bytes (non-boolean) at an offset range
    outb = torch.zeros(len(raw) - 5, dtype=torch.uint8, device="cuda")
    orc.byterle_decode_device(ctx, src, segs, len(raw) - 5, outb, value_begin=5)
    ctx.synchronize()
    np.testing.assert_array_equal(outb.cpu().numpy(), np.frombuffer(raw, dtype=np.uint8)[5:])
    del ctypes


def test_truncated_stream_reports_first_bad_group(orc):
    """A stream cut inside a literal group: the reference's "bad read in
    nextBuffer" is raised for the first value of that group, whichever
    thread of the window finds it."""
    rng = np.random.default_rng(3)
    raw = random_bytes(rng, 30_000)
    enc = byte_rle_encode(raw, rng)
    for cut in (len(enc) - 1, len(enc) // 2 + 7, 4097, 130):
        bad = enc[:cut]
        od = oracle.ByteRleDecoder(bad, boolean=False)
        gd = orc.ByteRleDecoder(bad, boolean=False)
        with pytest.raises(Exception) as we:
            od.next(len(raw))
        with pytest.raises(orc.ParseError) as ge:
            gd.next(len(raw))
        assert "bad read in nextBuffer" in str(ge.value) and str(we.value) in str(ge.value)


@pytest.mark.parametrize("n,p_null", [(1, 0.0), (4095, 0.5), (4097, 1.0), (1_000_003, 0.0), (9_000_011, 0.37),
                                      (9_000_011, 0.999)])
def test_scatter_lookback_sizes(orc, n, p_null):
    """The placement's single launch: each 4,096-row tile's first dense index
    from a decoupled look-back over the tiles' non-null counts (one tile,
    tile edges, all-null tiles, ~2,200 tiles), repeated launches on one
    context (a new look-back epoch each), against numpy's placement."""
    import torch

    rng = np.random.default_rng(n)
    nn = (rng.random(n) >= p_null).astype(np.uint8)
    k = int(nn.sum())
    dense = rng.integers(-(1 << 62), 1 << 62, size=k).astype(np.int64)
    ctx = orc.default_context(0)
    # (an all-null column still hands the C ABI a dense buffer: it checks for one)
    d_dense = torch.from_numpy(dense if k else np.zeros(1, dtype=np.int64)).cuda()
    d_nn = torch.from_numpy(nn).cuda()
    want = np.full(n, -9, dtype=np.int64)
    want[nn == 1] = dense
    for _ in range(3):
        out = torch.full((n,), 7, dtype=torch.int64, device="cuda")
        orc.scatter_not_null_device(ctx, d_dense, d_nn, out, fill=-9)
        ctx.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), want)
