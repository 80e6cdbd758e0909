"""GPU parity tests for the tiled kernel's dense (short-run) mode: parallel
run discovery over slabs and lane-per-run expansion through the LDS stage
(orc_amd/csrc/rlev2_tiled.hip). Streams are made of short
runs (SHORT_REPEAT-heavy low-cardinality columns, short DIRECT / DELTA runs)
with long and PATCHED_BASE runs mixed in, so a window switches between the
serial walk and dense mode. Bit-exact against the CPU oracle.
"""
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

# default (three density tiers: 33 KB serial, 21 KB serial + queue, union), the 33 KB serial instance,
# the 21 KB serial instance that queues short-run segments, the dense
# instances (8.5 KB, 12.5 KB), the union instance (8.5 KB dense / 16.75 KB
# serial windows) in two passes (its dense passes table their runs, the
# expansion kernel expands them by value slices), the 33 KB serial instance
# that queues, the union instance in one pass
DENSE_VARIANTS = [0, 2, 3, 4, 5, 6, 7, 8]
# A/B instances of the tuning build (ORCG_LIB=liborcgpu_ab.so), e.g.
# ORCG_TEST_EXTRA_VARIANTS=34,35
DENSE_VARIANTS += [int(v) for v in os.environ.get("ORCG_TEST_EXTRA_VARIANTS", "").split(",") if v]


def _short_run_stream(rng, signed, n_target, long_every=0, phase=0):
    """Run kinds / lengths / values of a stream dominated by short runs
    (phase > 0: alternately `phase` short runs and `phase // 8` long runs, so
    a segment's windows switch between dense and serial mode)."""
    vals, kinds, lens = [], [], []
    total = 0
    i = 0
    while total < n_target:
        i += 1
        r = rng.random()
        in_long = phase and (i % (phase + phase // 8)) >= phase
        if (long_every and i % long_every == 0) or in_long:
            k = int(rng.choice([1, 2, 3]))
            L = int(rng.integers(100, 513))
        elif r < 0.7:
            k, L = 0, int(rng.integers(3, 11))
        elif r < 0.8:
            k, L = 1, int(rng.integers(1, 17))
        elif r < 0.9:
            k, L = 3, int(rng.integers(1, 17))
        else:
            k, L = 3, int(rng.integers(11, 100))  # fixed-delta repeats (W = 0)
        if k == 0:
            x = int(rng.integers(-300, 300)) if signed else int(rng.integers(0, 1 << 20))
            v = [x] * L
        elif k == 1:
            w = int(rng.integers(1, 40))
            lo = -(1 << (w - 1)) if signed else 0
            v = list(rng.integers(lo, 1 << (w - 1), size=L))
        elif k == 2:
            base = int(rng.integers(0, 5000))
            x = base + rng.integers(0, 200, size=L)
            npatch = int(rng.integers(1, 6))
            idx = rng.choice(L, size=npatch, replace=False)
            x[idx] += rng.integers(1 << 20, 1 << 30, size=npatch)
            v = list(x)
        else:
            start = int(rng.integers(-10 ** 6, 10 ** 6)) if signed else int(rng.integers(10 ** 6, 2 * 10 ** 6))
            if r >= 0.9 or rng.integers(0, 2):
                step = 0 if r >= 0.9 else int(rng.integers(-50, 50))
                x = start + step * np.arange(L)
            else:
                d = rng.integers(1, 1000, size=L)
                d[0] = 0
                x = start + np.cumsum(d) * (1 if rng.integers(0, 2) else -1)
            v = list(x)
        vals += v
        kinds.append(k)
        lens.append(L)
        total += L
    return np.array(vals, dtype=np.int64), np.array(kinds, dtype=np.uint8), np.array(lens, dtype=np.uint32)


def _encode_with_positions(orc, v, signed, kinds, lens, stride):
    data, offs = orc.encode_runs(v, signed, kinds, lens)
    n = v.size
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    g = np.arange(0, n, stride)
    ri = np.searchsorted(starts, g, side="right") - 1
    pos = np.stack([offs[ri].astype(np.uint64), (g - starts[ri]).astype(np.uint64)], axis=1)
    return data, pos


@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("long_every", [0, 40])
def test_dense_streams_vs_oracle(signed, long_every):
    import torch

    import orc_amd

    rng = np.random.default_rng(5 + long_every + int(signed))
    v, kinds, lens = _short_run_stream(rng, signed, 400_000, long_every)
    ctx = orc_amd.default_context(0)
    for stride in (10_000, 777, 1 << 30):
        data, pos = _encode_with_positions(orc_amd, v, signed, kinds, lens, stride)
        if stride == 10_000:
            want = oracle.rlev2_decode(data.tobytes(), v.size, signed)
            np.testing.assert_array_equal(want, v)
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        for variant in DENSE_VARIANTS + [1]:
            ctx.set_rlev2_variant(variant)
            out = torch.zeros(v.size, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v.size, signed, out)
            ctx.synchronize()
            got = out.cpu().numpy()
            if not np.array_equal(got, v):
                bad = np.flatnonzero(got != v)
                i = int(bad[0])
                raise AssertionError("variant %d stride %d: %d mismatches, first at %d; got %s want %s" % (
                    variant, stride, bad.size, i, got[max(0, i - 4):i + 12].tolist(),
                    v[max(0, i - 4):i + 12].tolist()))
    ctx.set_rlev2_variant(0)


@pytest.mark.parametrize("phase", [300, 2000])
def test_window_mode_switches_vs_oracle(phase):
    """Stretches of short runs and of long runs inside one segment: the
    union instance (variant 6, the default's below 5 B/value) moves between
    8.5 KB dense windows and 16.75 KB serial windows; whole streams and value
    windows against the oracle."""
    import torch

    import orc_amd

    rng = np.random.default_rng(phase)
    v, kinds, lens = _short_run_stream(rng, True, 600_000, 0, phase)
    ctx = orc_amd.default_context(0)
    n = v.size
    for stride in (50_000, 10_000, 1 << 30):
        data, pos = _encode_with_positions(orc_amd, v, True, kinds, lens, stride)
        if stride == 10_000:
            np.testing.assert_array_equal(oracle.rlev2_decode(data.tobytes(), n, True), v)
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        for variant in DENSE_VARIANTS:
            ctx.set_rlev2_variant(variant)
            for a, b in [(0, n), (7, n - 11), (123_457, 400_001)]:
                o = torch.full((b - a,), -7, dtype=torch.int64, device="cuda")
                orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, b - a, True, o, value_begin=a)
                ctx.synchronize()
                got = o.cpu().numpy()
                if not np.array_equal(got, v[a:b]):
                    i = int(np.argmax(got != v[a:b]))
                    raise AssertionError("variant %d stride %d range %d-%d: first mismatch at %d" % (
                        variant, stride, a, b, a + i))
    ctx.set_rlev2_variant(0)


def test_dense_subranges_and_narrow_types():
    import torch

    import orc_amd

    rng = np.random.default_rng(99)
    v, kinds, lens = _short_run_stream(rng, True, 300_000, 25)
    stride = 10_000
    data, pos = _encode_with_positions(orc_amd, v, True, kinds, lens, stride)
    ctx = orc_amd.default_context(0)
    d_src = torch.from_numpy(data).cuda()
    d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
    n = v.size
    for variant in DENSE_VARIANTS:
        ctx.set_rlev2_variant(variant)
        for a, b in [(0, 1), (12345, 54321), (n - 7, n), (9_999, 10_001), (3, n - 3)]:
            o = torch.full((b - a,), -7, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, b - a, True, o, value_begin=a)
            ctx.synchronize()
            np.testing.assert_array_equal(o.cpu().numpy(), v[a:b])
        for dt, tdt in ((np.int32, torch.int32), (np.int16, torch.int16)):
            o = torch.empty(n, dtype=tdt, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, n, True, o)
            ctx.synchronize()
            np.testing.assert_array_equal(o.cpu().numpy(), v.astype(dt))
    ctx.set_rlev2_variant(0)


@pytest.mark.parametrize("case", ["pl0", "pgw", "delta_len", "truncated"])
@pytest.mark.parametrize("variant", DENSE_VARIANTS)
def test_dense_errors_match_reference(case, variant):
    """A corrupt run after thousands of SHORT_REPEAT runs (dense mode is on
    when the walk reaches it): the values before it decode, the next read
    raises the reference's message."""
    import orc_amd

    rng = np.random.default_rng(3)
    lens = rng.integers(3, 11, size=3000).astype(np.uint32)
    v = np.repeat(rng.integers(0, 100, size=lens.size), lens).astype(np.int64)
    good, _ = orc_amd.encode_runs(v, False, np.zeros(lens.size, np.uint8), lens)
    tail = {
        "pl0": bytes([0x8E, 0x09, 0x2B, 0x20, 0x07, 0xD0]),
        "pgw": bytes([0x8E, 0x09, 0x3F, 0xE1, 0x07]) + bytes(64),
        "delta_len": bytes([0xC2, 0x00, 0x02, 0x02]),
        "truncated": bytes([0x5E, 0x03, 0x5C]),
    }[case]
    data = good.tobytes() + tail
    n = v.size
    with pytest.raises(oracle.OracleError) as want:
        oracle.RleDecoderV2(data, False).next(n + 1)
    ctx = orc_amd.default_context(0)
    ctx.set_rlev2_variant(variant)
    try:
        dec = orc_amd.create_rle_decoder(data, False)
        np.testing.assert_array_equal(dec.next(n), v)
        with pytest.raises(orc_amd.ParseError) as got:
            dec.next(1)
        assert str(got.value) == str(want.value)
    finally:
        ctx.set_rlev2_variant(0)


def _wide_short_stream(rng, n_target):
    """Short runs (1-10 values) of wide values (>= 5 stream bytes per value):
    the serial instances queue such segments by values per run, and the
    drain walks them serially with staged (coalesced) group expansion."""
    vals, kinds, lens = [], [], []
    total = 0
    while total < n_target:
        r = rng.random()
        L = int(rng.integers(1, 11))
        if r < 0.6:
            k = 1
            w = int(rng.integers(40, 65))
            hi = (1 << (w - 1)) - 1
            v = list(rng.integers(-hi - 1, hi, size=L, endpoint=True))
        elif r < 0.8:
            k, L = 0, max(L, 3)
            v = [int(rng.integers(-(1 << 62), 1 << 62))] * L
        else:
            k = 3
            start = int(rng.integers(-(1 << 60), 1 << 60))
            d = rng.integers(1 << 30, 1 << 40, size=L)
            d[0] = 0
            v = list(start + np.cumsum(d))
        vals += v
        kinds.append(k)
        lens.append(L)
        total += L
    return np.array(vals, dtype=np.int64), np.array(kinds, dtype=np.uint8), np.array(lens, dtype=np.uint32)


def test_wide_short_runs_vs_oracle():
    import torch

    import orc_amd

    rng = np.random.default_rng(2026)
    v, kinds, lens = _wide_short_stream(rng, 300_000)
    ctx = orc_amd.default_context(0)
    n = v.size
    for stride in (10_000, 777):
        data, pos = _encode_with_positions(orc_amd, v, True, kinds, lens, stride)
        assert data.size >= 5 * n  # the >= 5 B/value instance under variant 0
        if stride == 10_000:
            np.testing.assert_array_equal(oracle.rlev2_decode(data.tobytes(), n, True), v)
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        for variant in orc_amd.rlev2_variants():
            ctx.set_rlev2_variant(variant)
            out = torch.zeros(n, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, n, True, out)
            ctx.synchronize()
            got = out.cpu().numpy()
            assert np.array_equal(got, v), "variant %d stride %d: first mismatch at %d" % (
                variant, stride, int(np.argmax(got != v)))
            for a, b in [(12345, 54321), (n - 7, n)]:
                o = torch.full((b - a,), -7, dtype=torch.int64, device="cuda")
                orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, b - a, True, o, value_begin=a)
                ctx.synchronize()
                np.testing.assert_array_equal(o.cpu().numpy(), v[a:b])
    ctx.set_rlev2_variant(0)


@pytest.mark.parametrize("signed", [True, False])
def test_short_wide_direct_default_routing_vs_oracle(signed):
    """Short DIRECT runs (1-12 values) of full 64-bit values: more than 8.1
    stream bytes a value, which variant 0 sends to the two-pass union instead
    of the serial walk (launch_rlev2_tiled). Row-index positions (one row
    group, many, and a stride that cuts runs) and value windows, against the
    oracle's RleDecoderV2 restatement."""
    import torch

    import orc_amd

    rng = np.random.default_rng(64 + int(signed))
    lens = rng.integers(1, 13, size=40_000).astype(np.uint32)
    n = int(lens.sum())
    lo, hi = (-(1 << 63), (1 << 63) - 1) if signed else (0, (1 << 64) - 1)
    v = rng.integers(lo, hi, size=n, endpoint=True, dtype=np.int64 if signed else np.uint64).view(np.int64)
    kinds = np.ones(lens.size, dtype=np.uint8)
    want = oracle.rlev2_decode(orc_amd.encode_runs(v, signed, kinds, lens)[0].tobytes(), n, signed)
    np.testing.assert_array_equal(want, v)
    ctx = orc_amd.default_context(0)
    ctx.set_rlev2_variant(0)
    for stride in (10_000, 777, 1 << 30):
        data, pos = _encode_with_positions(orc_amd, v, signed, kinds, lens, stride)
        assert 10 * data.size > 81 * n  # the rule's side of 8.1 B/value
        d_src = torch.from_numpy(data).cuda()
        d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
        out = torch.full((n,), -7, dtype=torch.int64, device="cuda")
        orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, n, signed, out)
        ctx.synchronize()
        got = out.cpu().numpy()
        assert np.array_equal(got, want), "stride %d: first mismatch at %d" % (stride, int(np.argmax(got != want)))
        for a, b in [(12345, 54321), (n - 7, n)]:
            o = torch.full((b - a,), -7, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, b - a, signed, o, value_begin=a)
            ctx.synchronize()
            np.testing.assert_array_equal(o.cpu().numpy(), want[a:b])


@pytest.mark.parametrize("bits", [7, 33, 64])
@pytest.mark.parametrize("signed", [True, False])
def test_value_parallel_expansion_vs_oracle(bits, signed):
    """The dense expansion's value-parallel path (rlev2_tiled.hip dense_expand:
    SHORT_REPEAT / DIRECT / constant-step DELTA runs of 17-256 values inside
    dense segments, each value found by a binary search over the runs' first
    values): short-run segments (SHORT_REPEAT runs of 3-10 values) with DIRECT
    runs of 17-99 values of `bits`-bit values and constant-step DELTA runs
    (11-99 values) interleaved, on every pinned variant, bit-exact against
    the oracle (RleDecoderV2.cc:184-248, 372-435)."""
    import torch

    import orc_amd

    rng = np.random.default_rng(17 * bits + int(signed))
    vals, kinds, lens = [], [], []
    total = 0
    while total < 300_000:
        r = rng.random()
        if r < 0.6:
            k, L = 0, int(rng.integers(3, 11))
            x = int(rng.integers(-300, 300)) if signed else int(rng.integers(0, 1 << 12))
            v = [x] * L
        elif r < 0.85:
            k, L = 1, int(rng.integers(17, 100))
            if bits == 64:
                v = [int(x) for x in rng.integers(-(1 << 63), (1 << 63) - 1, size=L, dtype=np.int64)]
                if not signed:
                    v = [x & ((1 << 63) - 1) for x in v]
            else:
                hi = 1 << (bits - 1 if signed else bits)
                v = [int(x) for x in rng.integers(-hi if signed else 0, hi, size=L)]
        else:
            k, L = 3, int(rng.integers(11, 100))
            start = int(rng.integers(-10 ** 6, 10 ** 6)) if signed else int(rng.integers(10 ** 6, 2 * 10 ** 6))
            step = int(rng.integers(-50, 50)) if signed else int(rng.integers(0, 50))
            v = [start + step * i for i in range(L)]
        vals += v
        kinds.append(k)
        lens.append(L)
        total += L
    v = np.array(vals, dtype=np.int64)
    kinds = np.array(kinds, dtype=np.uint8)
    lens = np.array(lens, dtype=np.uint32)
    stride = 10_000
    data, pos = _encode_with_positions(orc_amd, v, signed, kinds, lens, stride)
    want = oracle.rlev2_decode(data.tobytes(), v.size, signed)
    np.testing.assert_array_equal(want, v)
    ctx = orc_amd.default_context(0)
    d_src = torch.from_numpy(data).cuda()
    d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
    try:
        for variant in DENSE_VARIANTS + [1]:
            ctx.set_rlev2_variant(variant)
            out = torch.zeros(v.size, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v.size, signed, out)
            ctx.synchronize()
            got = out.cpu().numpy()
            if not np.array_equal(got, want):
                i = int(np.flatnonzero(got != want)[0])
                raise AssertionError("variant %d: first mismatch at %d: got %s want %s" % (
                    variant, i, got[max(0, i - 4):i + 8].tolist(), want[max(0, i - 4):i + 8].tolist()))
    finally:
        ctx.set_rlev2_variant(0)


def _skew_stream(rng, signed, n_target, long_kind, every):
    """Short-run row groups (SHORT_REPEAT runs of 3 values) with one long run
    of `long_kind` every `every` short runs: DIRECT runs of 512 values, DELTA
    runs of 200-512 values with variable deltas, or PATCHED_BASE runs of
    100-512 values. The stream stays dense (few bytes per run on average), so
    the long runs land in tabled dense passes and cross value slices."""
    vals, kinds, lens = [], [], []
    total, i = 0, 0
    while total < n_target:
        i += 1
        if i % every == 0:
            if long_kind == "direct":
                k, L = 1, 512
                hi = 1 << 6
                v = [int(x) for x in rng.integers(-hi if signed else 0, hi, size=L)]
            elif long_kind == "delta":
                k, L = 3, int(rng.integers(200, 513))
                start = int(rng.integers(-10 ** 6, 10 ** 6)) if signed else int(rng.integers(10 ** 7, 2 * 10 ** 7))
                d = rng.integers(0, 100, size=L)
                d[0] = 0
                sgn = -1 if (signed and rng.integers(0, 2)) else 1
                if not signed:
                    sgn = 1 if rng.integers(0, 2) else -1
                d[1] = max(int(d[1]), 1)
                v = [int(x) for x in start + sgn * np.cumsum(d)]
            else:
                k, L = 2, int(rng.integers(100, 513))
                base = int(rng.integers(0, 5000))
                x = base + rng.integers(0, 200, size=L)
                npatch = int(rng.integers(1, 6))
                idx = rng.choice(L, size=npatch, replace=False)
                x[idx] += rng.integers(1 << 20, 1 << 30, size=npatch)
                v = [int(y) for y in x]
        else:
            k, L = 0, 3
            x = int(rng.integers(-300, 300)) if signed else int(rng.integers(0, 1 << 12))
            v = [x] * L
        vals += v
        kinds.append(k)
        lens.append(L)
        total += L
    return np.array(vals, dtype=np.int64), np.array(kinds, dtype=np.uint8), np.array(lens, dtype=np.uint32)


@pytest.mark.parametrize("long_kind", ["direct", "delta", "patched"])
@pytest.mark.parametrize("signed", [True, False])
def test_two_pass_skew_vs_oracle(long_kind, signed):
    """The two-pass union decode (variant 6; rlev2_tiled.hip kOptTable +
    rlev2_expand.hip) on row groups that mix 3-value SHORT_REPEAT runs with
    long DIRECT / variable-width DELTA / PATCHED_BASE runs: the long runs sit
    in tabled dense passes and straddle value slices (a DELTA run begun before
    its slice is resumed from its running sum), at row-group strides that cut
    segments mid-run and with row ranges; bit-exact against the oracle
    (RleDecoderV2.cc:184-248, 250-370, 372-435) and against the one-pass
    union instance (variant 8)."""
    import torch

    import orc_amd

    rng = np.random.default_rng(101 + 7 * len(long_kind) + int(signed))
    every = 60 if long_kind == "direct" else 25
    v, kinds, lens = _skew_stream(rng, signed, 500_000, long_kind, every)
    ctx = orc_amd.default_context(0)
    try:
        for stride in (10_000, 3_333, 50_000):
            data, pos = _encode_with_positions(orc_amd, v, signed, kinds, lens, stride)
            assert data.size < 1.25 * v.size  # the default's union tier
            if stride == 10_000:
                want = oracle.rlev2_decode(data.tobytes(), v.size, signed)
                np.testing.assert_array_equal(want, v)
            d_src = torch.from_numpy(data).cuda()
            d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
            for variant in (0, 6, 8):
                ctx.set_rlev2_variant(variant)
                out = torch.zeros(v.size, dtype=torch.int64, device="cuda")
                orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v.size, signed, out)
                ctx.synchronize()
                got = out.cpu().numpy()
                if not np.array_equal(got, v):
                    i = int(np.flatnonzero(got != v)[0])
                    raise AssertionError("variant %d stride %d: first mismatch at %d: got %s want %s" % (
                        variant, stride, i, got[max(0, i - 4):i + 8].tolist(), v[max(0, i - 4):i + 8].tolist()))
        # segment tables (host plans) and a row range inside the stream
        data, _ = orc_amd.encode_runs(v, signed, kinds, lens)
        d_src = torch.from_numpy(data).cuda()
        plan = orc_amd.Plan(data, 8 << 10, 8192)
        d_seg = torch.from_numpy(plan.segments().view(np.int64)).cuda()
        for variant in (6, 8):
            ctx.set_rlev2_variant(variant)
            for a, b in ((0, v.size), (12_345, 400_001)):
                out = torch.zeros(b - a, dtype=torch.int64, device="cuda")
                orc_amd.decode_device(ctx, d_src, d_seg, b - a, signed, out, value_begin=a)
                ctx.synchronize()
                got = out.cpu().numpy()
                if not np.array_equal(got, v[a:b]):
                    i = int(np.flatnonzero(got != v[a:b])[0])
                    raise AssertionError("variant %d plan range %d-%d: first mismatch at %d" % (variant, a, b, a + i))
    finally:
        ctx.set_rlev2_variant(0)


@pytest.mark.parametrize("signed", [True, False])
def test_two_pass_many_runs_per_slice(signed):
    """Value slices holding more runs than one expansion round takes
    (rlev2_expand.hip kRound): one-value DIRECT runs and 3-value
    SHORT_REPEAT runs (up to ~1,000 runs per 1,024-value slice), with
    variable-width DELTA runs between them; variant 6 (two passes) against
    the oracle and variant 8 (one pass)."""
    import torch

    import orc_amd

    rng = np.random.default_rng(303 + int(signed))
    vals, kinds, lens = [], [], []
    total = 0
    while total < 200_000:
        r = rng.random()
        if r < 0.6:
            k, L = 1, 1
            v = [int(rng.integers(-8, 8)) if signed else int(rng.integers(0, 16))]
        elif r < 0.97:
            k, L = 0, 3
            v = [int(rng.integers(-50, 50)) if signed else int(rng.integers(0, 100))] * 3
        else:
            k, L = 3, int(rng.integers(20, 200))
            d = rng.integers(0, 30, size=L)
            d[0], d[1] = 0, max(int(d[1]), 1)
            start = int(rng.integers(-1000, 1000)) if signed else int(rng.integers(10 ** 6, 2 * 10 ** 6))
            v = [int(x) for x in start + np.cumsum(d)]
        vals += v
        kinds.append(k)
        lens.append(L)
        total += L
    v = np.array(vals, dtype=np.int64)
    kinds = np.array(kinds, dtype=np.uint8)
    lens = np.array(lens, dtype=np.uint32)
    stride = 10_000
    data, pos = _encode_with_positions(orc_amd, v, signed, kinds, lens, stride)
    want = oracle.rlev2_decode(data.tobytes(), v.size, signed)
    np.testing.assert_array_equal(want, v)
    ctx = orc_amd.default_context(0)
    d_src = torch.from_numpy(data).cuda()
    d_pos = torch.from_numpy(pos.view(np.int64)).cuda()
    try:
        for variant in (0, 6, 8):
            ctx.set_rlev2_variant(variant)
            out = torch.zeros(v.size, dtype=torch.int64, device="cuda")
            orc_amd.decode_positions_device(ctx, d_src, d_pos, stride, v.size, signed, out)
            ctx.synchronize()
            got = out.cpu().numpy()
            if not np.array_equal(got, v):
                i = int(np.flatnonzero(got != v)[0])
                raise AssertionError("variant %d: first mismatch at %d: got %s want %s" % (
                    variant, i, got[max(0, i - 4):i + 8].tolist(), v[max(0, i - 4):i + 8].tolist()))
    finally:
        ctx.set_rlev2_variant(0)
