"""GPU parity tests: the HIP RLEv2 decoder (through the C ABI) against the
reference's known answers and the CPU oracle. Bit-exact throughout.

Needs a real MI355X: run with `pytest -m gpu`.
"""
import numpy as np
import pytest

from conftest import assert_matches, decode_batches, load_golden
from oracle import oracle

pytestmark = pytest.mark.gpu

RLEV2 = load_golden("kat_rlev2.json")


@pytest.fixture(scope="module", params=[0, 1], ids=["tiled", "wavewalk"])
def orc(request):
    """Every parity test runs against both RLEv2 kernels (ORCG_RLEV2_TILED,
    ORCG_RLEV2_WAVE_WALK)."""
    import orc_amd

    ctx = orc_amd.default_context(0)
    ctx.set_rlev2_variant(request.param)
    yield orc_amd
    ctx.set_rlev2_variant(0)


@pytest.mark.parametrize("fx", RLEV2, ids=[f["name"] for f in RLEV2])
def test_kat_stateful(orc, fx):
    """Same reads as the reference test: batches 1, 3, 7 and all at once,
    with its notNull mask (c++/test/TestRleDecoder.cc)."""
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    for b in fx["batches"]:
        dec = orc.create_rle_decoder(data, fx["signed"])
        got = decode_batches(dec.next, fx["expected"], b, nn)
        assert_matches(fx["expected"], got, nn, "%s batch=%s" % (fx["name"], b))
    if "seek" in fx:
        dec = orc.create_rle_decoder(data, fx["signed"])
        dec.seek(*fx["seek"]["position"])
        got = list(dec.next(3)) + list(dec.next(3)) + list(dec.next(1))
        assert got == fx["seek"]["expected"]


@pytest.mark.parametrize("fx", RLEV2, ids=[f["name"] for f in RLEV2])
def test_kat_narrow_matches_oracle(orc, fx):
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    n = len(fx["expected"])
    nnarr = None if nn is None else np.array(nn, dtype=np.uint8)
    for dt in (np.int64, np.int32, np.int16):
        want = oracle.RleDecoderV2(data, fx["signed"]).next(n, nnarr, dtype=dt)
        got = orc.rlev2_decode(data, n, fx["signed"], not_null=nnarr, dtype=dt)
        keep = np.ones(n, bool) if nn is None else nnarr.astype(bool)
        np.testing.assert_array_equal(got[keep], want[keep])


def _mixed(rng, signed, nruns):
    from test_host_cpu import _mixed_stream

    return _mixed_stream(rng, signed, nruns)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("signed", [True, False])
def test_mixed_runs_vs_oracle(orc, seed, signed):
    rng = np.random.default_rng(100 + seed)
    for _ in range(20):
        v, kinds, lens = _mixed(rng, signed, 300)
        try:
            data, _ = orc.encode_runs(v, signed, kinds, lens)
            break
        except orc.OrcError:
            continue
    want = oracle.rlev2_decode(data.tobytes(), v.size, signed)
    np.testing.assert_array_equal(want, v)
    got = orc.rlev2_decode(data.tobytes(), v.size, signed)
    np.testing.assert_array_equal(got, want)
    # batched reads with a random null mask through the stateful decoder
    nn = (rng.random(v.size + v.size // 3) > 0.25).astype(np.uint8)
    nn[np.cumsum(nn) > v.size] = 0
    nd = nn.size
    odec = oracle.RleDecoderV2(data.tobytes(), signed)
    gdec = orc.create_rle_decoder(data.tobytes(), signed)
    i = 0
    while i < nd:
        k = int(min(rng.integers(1, 2000), nd - i))
        w = odec.next(k, nn[i:i + k])
        g = gdec.next(k, nn[i:i + k])
        m = nn[i:i + k].astype(bool)
        np.testing.assert_array_equal(g[m], w[m])
        i += k


@pytest.mark.parametrize("bits", [1, 2, 3, 4, 5, 7, 8, 11, 13, 16, 17, 24, 26, 28, 30, 32, 40, 48, 56, 64])
@pytest.mark.parametrize("signed", [True, False])
def test_direct_every_width(orc, bits, signed):
    rng = np.random.default_rng(bits)
    n = 70001
    if bits == 64:
        v = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64, endpoint=True)
    elif signed:
        v = rng.integers(-(1 << (bits - 1)), (1 << (bits - 1)), size=n, dtype=np.int64)
    else:
        v = rng.integers(0, (1 << bits) - 1, size=n, dtype=np.int64, endpoint=True)
    for aligned in (False, True):
        data, _ = orc.encode_direct(v, signed, aligned=aligned)
        got = orc.rlev2_decode(data.tobytes(), n, signed)
        np.testing.assert_array_equal(got, v)


def test_device_positions_decode_and_subranges(orc):
    import torch

    rng = np.random.default_rng(7)
    n, stride = 1_000_003, 10_000
    v = rng.integers(-(1 << 40), 1 << 40, size=n, dtype=np.int64)
    data, pos = orc.encode_direct(v, True, aligned=True, rows_per_group=stride)
    ctx = orc.default_context(0)
    d_src = torch.from_numpy(data).cuda()
    d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    orc.decode_positions_device(ctx, d_src, d_pos, stride, n, True, out)
    ctx.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), v)
    # row range [a, b) as RowReaderOptions::range would request
    for a, b in [(0, 1), (12345, 54321), (n - 7, n), (9_999, 10_001)]:
        o2 = torch.zeros(b - a, dtype=torch.int64, device="cuda")
        orc.decode_positions_device(ctx, d_src, d_pos, stride, b - a, True, o2, value_begin=a)
        ctx.synchronize()
        np.testing.assert_array_equal(o2.cpu().numpy(), v[a:b])
    # int32 narrowing on device
    o3 = torch.empty(n, dtype=torch.int32, device="cuda")
    orc.decode_positions_device(ctx, d_src, d_pos, stride, n, True, o3)
    ctx.synchronize()
    np.testing.assert_array_equal(o3.cpu().numpy(), v.astype(np.int32))


def test_device_segments_mixed(orc):
    import torch

    rng = np.random.default_rng(11)
    v, kinds, lens = _mixed(rng, True, 2000)
    data, offs = orc.encode_runs(v, True, kinds, lens)
    plan = orc.Plan(data.tobytes(), max_segment_bytes=1024, max_segment_values=1000)
    segs = plan.segments()
    ctx = orc.default_context(0)
    out = torch.empty(v.size, dtype=torch.int64, device="cuda")
    orc.decode_device(ctx, torch.from_numpy(data).cuda(), torch.from_numpy(segs.view(np.int64)).cuda(),
                      v.size, True, out)
    ctx.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), v)


@pytest.mark.parametrize("case", ["pl0", "pgw", "delta_len", "truncated"])
def test_errors_match_reference(orc, case):
    good, _ = orc.encode_direct(np.arange(700, dtype=np.int64), False)
    g = good.tobytes()
    tail = {
        "pl0": bytes([0x8E, 0x09, 0x2B, 0x20, 0x07, 0xD0]),
        "pgw": bytes([0x8E, 0x09, 0x3F, 0xE1, 0x07]) + bytes(64),  # pw 64 + pgw 8 > 64
        "delta_len": bytes([0xC2, 0x00, 0x02, 0x02]),
        "truncated": bytes([0x5E, 0x03, 0x5C]),
    }[case]
    data = g + tail
    # values before the corrupt run decode fine, the next read raises the
    # reference's message (RleDecoderV2.cc:38, :307, :328-330, :412-415)
    with pytest.raises(oracle.OracleError) as want:
        oracle.RleDecoderV2(data, False).next(701)
    dec = orc.create_rle_decoder(data, False)
    np.testing.assert_array_equal(dec.next(700), np.arange(700))
    with pytest.raises(orc.ParseError) as got:
        dec.next(1)
    assert str(got.value) == str(want.value)


def test_large_roundtrip_property(orc):
    """Full-range int64 at 2e7 rows: decode(encode(v)) == v (size-independent
    round-trip property; the oracle is checked on the small cases)."""
    import torch

    n = 20_000_000
    g = torch.Generator(device="cuda").manual_seed(42)
    v = torch.randint(-(1 << 63), (1 << 63) - 1, (n,), dtype=torch.int64, device="cuda", generator=g)
    vh = v.cpu().numpy()
    data, pos = orc.encode_direct(vh, True, aligned=True, rows_per_group=10_000)
    ctx = orc.default_context(0)
    out = torch.empty_like(v)
    orc.decode_positions_device(ctx, torch.from_numpy(data).cuda(), torch.from_numpy(pos.view(np.int64)).cuda(),
                                10_000, n, True, out)
    ctx.synchronize()
    assert torch.equal(out, v)


def _stream_with_positions(orc, rng, kind, n, stride, bits=12):
    if kind == "repeat":
        lens = rng.integers(3, 11, size=n // 3).astype(np.uint32)
        lens = lens[: np.searchsorted(np.cumsum(lens), n)]
        kinds = np.zeros(lens.size, dtype=np.uint8)
        v = np.repeat(rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), size=lens.size), lens)
    elif kind == "delta":
        lens = np.full(n // 512, 512, dtype=np.uint32)
        lens[::7] = 300  # ragged runs too
        kinds = np.full(lens.size, 3, dtype=np.uint8)
        v = np.cumsum(rng.integers(0, 1 << bits, size=int(lens.sum()), dtype=np.int64))
        sgn = np.repeat(np.where(np.arange(lens.size) % 2 == 0, 1, -1), lens)
        v = v * sgn  # alternate increasing / decreasing runs
        # each run must be monotone in its own direction: rebuild per run
        out, at = [], 0
        for L, s in zip(lens, np.where(np.arange(lens.size) % 2 == 0, 1, -1)):
            base = int(rng.integers(-(1 << 40), 1 << 40))
            out.append(base + s * np.cumsum(rng.integers(1, 1 << bits, size=int(L))))
        v = np.concatenate(out)
    elif kind == "wide":
        # >= 5 stream bytes per value, so variant 0 picks the 33 KB
        # register-fill instance with the full-run fast paths: DIRECT runs of
        # 47-bit values alternating with DELTA runs of 40-bit deltas, some
        # ragged (300 values)
        lens = np.full(n // 512, 512, dtype=np.uint32)
        lens[::5] = 300
        kinds = np.where(np.arange(lens.size) % 2 == 0, 1, 3).astype(np.uint8)
        out = []
        for L, k in zip(lens, kinds):
            if k == 1:
                out.append(rng.integers(-(1 << 46), 1 << 46, size=int(L)))
            else:
                s = 1 if rng.integers(0, 2) else -1
                base = int(rng.integers(-(1 << 50), 1 << 50))
                out.append(base + s * np.cumsum(rng.integers(1 << 38, 1 << 40, size=int(L))))
        v = np.concatenate(out)
    else:  # patched
        lens = np.full(n // 512, 512, dtype=np.uint32)
        kinds = np.full(lens.size, 2, dtype=np.uint8)
        v = rng.integers(0, 1 << bits, size=int(lens.sum()), dtype=np.int64)
        hot = rng.random(v.size) < 0.01
        v[hot] += rng.integers(1 << 30, 1 << 50, size=int(hot.sum()))
        v[100::512] += 1 << 33
        v[::512] = 0
    n = int(lens.sum())
    v = v[:n].astype(np.int64)
    data, offs = orc.encode_runs(v, True, kinds, lens)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    g = np.arange(0, n, stride)
    ri = np.searchsorted(starts, g, side="right") - 1
    pos = np.stack([offs[ri].astype(np.uint64), (g - starts[ri]).astype(np.uint64)], axis=1)
    return v, data, pos


@pytest.mark.parametrize("kind", ["repeat", "delta", "patched", "wide"])
def test_structured_streams_every_variant(kind):
    """Every kernel variant (ORCG_RLEV2_* and the tuning variants) is
    bit-exact on SR-heavy (run tables that fill up), DELTA-heavy and
    PATCHED-heavy streams, with one huge segment and with row groups."""
    import torch

    import orc_amd

    rng = np.random.default_rng({"repeat": 1, "delta": 2, "patched": 3, "wide": 4}[kind])
    ctx = orc_amd.default_context(0)
    for stride in (10_000, 1 << 30):
        v, data, pos = _stream_with_positions(orc_amd, rng, kind, 300_000, stride)
        want = oracle.rlev2_decode(data.tobytes(), v.size, True)
        np.testing.assert_array_equal(want, v)
        if kind == "wide":
            assert data.size >= 5 * v.size  # reaches the >= 5 B/value default instance
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        for variant in orc_amd.rlev2_variants():
            ctx.set_rlev2_variant(variant)
            out = torch.zeros(v.size, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v.size, True, out)
            ctx.synchronize()
            got = out.cpu().numpy()
            assert np.array_equal(got, want), "variant %d stride %d: first mismatch at %d" % (
                variant, stride, int(np.argmax(got != want)))
    ctx.set_rlev2_variant(0)


@pytest.mark.parametrize("layout", ["edges", "same_chunk", "escape_gaps", "max_patches"])
def test_patched_full_runs_patch_layouts(layout):
    """Full 512-value PATCHED_BASE runs (the predicate-free path) with patches
    at chunk edges (0, 63, 64, 511), several in one 64-value chunk, gaps past
    255 (escape entries, RleDecoderV2.cc:250-271) and the 31-entry maximum,
    against the oracle, with row groups aligned to the runs and not."""
    import torch

    import orc_amd

    pos_sets = {
        "edges": [0, 1, 63, 64, 65, 127, 128, 300, 510, 511],
        "same_chunk": [200, 201, 203, 210, 230, 255],
        "escape_gaps": [5, 400, 511],
        "max_patches": list(range(0, 512, 17))[:31],
    }[layout]
    rng = np.random.default_rng(7)
    runs = 40
    v = rng.integers(0, 1 << 10, size=runs * 512, dtype=np.int64)
    for r in range(runs):
        for p in pos_sets:
            v[r * 512 + p] += int(rng.integers(1 << 20, 1 << 40)) << 10
        v[r * 512 + 7] = 0  # a small base
    data, offs = orc_amd.encode_runs(v, True, np.full(runs, 2, dtype=np.uint8), np.full(runs, 512, dtype=np.uint32))
    want = oracle.rlev2_decode(data.tobytes(), v.size, True)
    np.testing.assert_array_equal(want, v)
    ctx = orc_amd.default_context(0)
    d_src = torch.from_numpy(data).cuda()
    starts = np.arange(runs, dtype=np.int64) * 512
    for stride in (1024, 1000):
        g = np.arange(0, v.size, stride)
        ri = np.searchsorted(starts, g, side="right") - 1
        pos = np.stack([offs[ri].astype(np.uint64), (g - starts[ri]).astype(np.uint64)], axis=1)
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        for variant in orc_amd.rlev2_variants():
            ctx.set_rlev2_variant(variant)
            out = torch.zeros(v.size, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v.size, True, out)
            ctx.synchronize()
            got = out.cpu().numpy()
            assert np.array_equal(got, want), "variant %d stride %d: first mismatch at %d" % (
                variant, stride, int(np.argmax(got != want)))
    ctx.set_rlev2_variant(0)


def _mixed_segments(orc, rng, nseg, stride):
    """Row groups alternating between long DIRECT runs of 64-bit values and
    short SHORT_REPEAT / short DIRECT runs of wide values: overall >= 1.25
    stream bytes per value (the default picks a serial-walk instance), with
    every other segment made of short runs (queued for the dense instance)."""
    vals, kinds, lens = [], [], []
    for s in range(nseg):
        left = stride
        if s % 2 == 0:
            while left:
                L = min(512, left)
                vals.append(rng.integers(-(1 << 62), 1 << 62, size=L))
                kinds.append(1)
                lens.append(L)
                left -= L
        else:
            while left:
                if rng.random() < 0.5 and left >= 3:
                    L = int(min(rng.integers(3, 11), left))
                    vals.append(np.full(L, int(rng.integers(-(1 << 50), 1 << 50))))
                    kinds.append(0)
                else:
                    L = int(min(rng.integers(1, 9), left))
                    vals.append(rng.integers(-(1 << 40), 1 << 40, size=L))
                    kinds.append(1)
                lens.append(L)
                left -= L
    v = np.concatenate(vals).astype(np.int64)
    lens = np.array(lens, dtype=np.uint32)
    data, offs = orc.encode_runs(v, True, np.array(kinds, np.uint8), lens)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    g = np.arange(0, v.size, stride)
    ri = np.searchsorted(starts, g, side="right") - 1
    pos = np.stack([offs[ri].astype(np.uint64), (g - starts[ri]).astype(np.uint64)], axis=1)
    return v, data, pos


def test_short_run_segments_are_queued_for_the_dense_instance():
    """The serial-walk instances queue short-run segments and the dense
    instance drains the queue in the same decode: bit-exact against the
    oracle for every instance the default launches, for value sub-ranges,
    and across repeated launches (the queue resets itself)."""
    import torch

    import orc_amd

    rng = np.random.default_rng(21)
    ctx = orc_amd.default_context(0)
    stride = 5000
    v, data, pos = _mixed_segments(orc_amd, rng, 40, stride)
    want = oracle.rlev2_decode(data.tobytes(), v.size, True)
    np.testing.assert_array_equal(want, v)
    assert data.size >= 1.25 * v.size
    d_src = torch.from_numpy(data).cuda()
    d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
    for variant in orc_amd.rlev2_variants():
        ctx.set_rlev2_variant(variant)
        for _ in range(3):
            out = torch.zeros(v.size, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v.size, True, out)
            ctx.synchronize()
            got = out.cpu().numpy()
            assert np.array_equal(got, want), "variant %d: first mismatch at %d" % (variant, int(np.argmax(got != want)))
        for a, b in [(7_001, 7_002), (4_999, 15_001), (100_000, 200_000 - 3)]:
            o2 = torch.zeros(b - a, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, b - a, True, o2, value_begin=a)
            ctx.synchronize()
            np.testing.assert_array_equal(o2.cpu().numpy(), want[a:b])
    ctx.set_rlev2_variant(0)


def test_queued_segment_reports_truncation():
    """A short-run segment that runs into a truncated run: the dense instance
    draining the queue reports the reference's error at the first missing
    value, like the serial walk."""
    import orc_amd

    rng = np.random.default_rng(3)
    v = np.repeat(rng.integers(-(1 << 60), 1 << 60, size=3000), 5)
    data, _ = orc_amd.encode_runs(v, True, np.zeros(3000, np.uint8), np.full(3000, 5, np.uint32))
    bad = data.tobytes() + bytes([0x5E, 0x03, 0x5C])  # a DIRECT header whose data is missing
    with pytest.raises(oracle.OracleError) as want:
        oracle.RleDecoderV2(bad, True).next(v.size + 1)
    ctx = orc_amd.default_context(0)
    for variant in orc_amd.rlev2_variants():
        if variant == 1:
            continue
        ctx.set_rlev2_variant(variant)
        with pytest.raises(orc_amd.ParseError) as got:
            orc_amd.rlev2_decode(bad, v.size + 1, True)
        assert str(got.value) == str(want.value), variant
    ctx.set_rlev2_variant(0)


@pytest.mark.parametrize("kind", ["repeat", "delta", "patched", "wide"])
def test_split_launches_every_variant(kind):
    """Few large segments (a file's child-column row groups), every pinned
    instance, full range and value windows whose ends fall inside runs,
    against the generated values (the encoder's input, checked against the
    oracle below). With ORCG_SPLIT=k (k > 1) in the environment the launches
    split each segment's values over k workgroups (rlev2_tiled.hip
    auto_split), each one walking the runs before its share: the same test
    covers that path."""
    import torch

    import orc_amd as orc
    from oracle import oracle

    rng = np.random.default_rng(11)
    v, data, _ = _stream_with_positions(orc, rng, kind, 600_000, 10_000)
    n = v.size
    assert np.array_equal(oracle.rlev2_decode(data.tobytes(), n, True), v)
    ctx = orc.default_context(0)
    d_src = torch.from_numpy(data).cuda()
    for seg_values in (40_000, 150_000):  # 15 / 4 segments: split 8 / 8
        plan = orc.Plan(data, 1 << 30, seg_values)
        segs = torch.from_numpy(plan.segments().view(np.int64)).cuda()
        try:
            for variant in orc.rlev2_variants():
                ctx.set_rlev2_variant(variant)
                for a, b in [(0, n), (1, n - 1), (12_345, 333_333), (n - 513, n)]:
                    out = torch.zeros(b - a, dtype=torch.int64, device="cuda")
                    orc.decode_device(ctx, d_src, segs, b - a, True, out, value_begin=a)
                    ctx.synchronize()
                    got = out.cpu().numpy()
                    assert np.array_equal(got, v[a:b]), "variant %d segs %d range %d-%d: first mismatch at %d" % (
                        variant, segs.shape[0], a, b, a + int(np.argmax(got != v[a:b])))
        finally:
            ctx.set_rlev2_variant(0)
