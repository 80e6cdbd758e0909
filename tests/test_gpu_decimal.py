"""GPU parity for DECIMAL and TIMESTAMP columns (decimal_kernels.hip through
the C ABI): the reference's TestColumnReader known answers, random varint
streams with per-value scales against the CPU oracle (rescale up / down,
"Decimal scale out of range", Decimal128 wrap and truncation), and files:
examples/decimal.orc (+ its expected ColumnPrinter output), the ORCv2
Decimal64V2 examples, and pyarrow-written files with nulls and timestamps.
"""
import decimal
import os

import numpy as np
import pytest

from conftest import load_golden
from oracle import oracle

pytestmark = pytest.mark.gpu

DECIMAL = load_golden("kat_decimal.json")
M64 = (1 << 64) - 1


def _zz_varints(vals):
    out = bytearray()
    for v in vals:
        u = v << 1 if v >= 0 else ((-v) << 1) - 1  # zigzag of an arbitrary-width int
        while True:
            b = u & 0x7F
            u >>= 7
            if u:
                out.append(b | 0x80)
            else:
                out.append(b)
                break
    return bytes(out)


def _to_int128(pairs):
    res = []
    for h, lo in np.asarray(pairs).reshape(-1, 2):
        v = ((int(h) & M64) << 64) | (int(lo) & M64)
        res.append(v - (1 << 128) if v >> 127 else v)
    return res


def _device_decimal(data, scales, n, precision, scale):
    import torch

    import orc_amd

    ctx = orc_amd.default_context(0)
    d_src = torch.frombuffer(bytearray(data) or bytearray(1), dtype=torch.uint8).cuda()
    d_sc = torch.from_numpy(np.ascontiguousarray(scales, dtype=np.int64)).cuda()
    out = torch.zeros((n, 2) if precision > 18 or precision == 0 else n, dtype=torch.int64, device="cuda")
    orc_amd.decimal_decode_device(ctx, d_src, d_sc, n, precision, scale, out, src_len=len(data))
    return out.cpu().numpy()


def _device_hive11_keep(data, scales, n, scale):
    """orcg_hive11_decimal_decode_device with throw_on_overflow = 0."""
    import torch

    import orc_amd

    ctx = orc_amd.default_context(0)
    L = orc_amd._lib.load()
    d_src = torch.frombuffer(bytearray(data) or bytearray(1), dtype=torch.uint8).cuda()
    d_sc = torch.from_numpy(np.ascontiguousarray(scales, dtype=np.int64)).cuda()
    out = torch.full((n, 2), 7, dtype=torch.int64, device="cuda")
    keep = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    ctx.after_torch()
    orc_amd._lib.check(L.orcg_hive11_decimal_decode_device(ctx.handle, d_src.data_ptr(), len(data), d_sc.data_ptr(), n,
                                                           scale, 0, out.data_ptr(), keep.data_ptr()), ctx.last_error)
    return out.cpu().numpy(), keep.cpu().numpy()


@pytest.mark.parametrize("fx", DECIMAL, ids=[f["name"] for f in DECIMAL])
def test_decimal_timestamp_kat_on_device(fx):
    import torch

    import orc_amd

    n = len(fx["expected"])
    sec = bytes.fromhex(fx["secondary"])
    data = bytes.fromhex(fx["data"])
    if fx["kind"] == "decimal":
        scales = orc_amd.rlev1_decode(sec, n, True)
        if fx.get("error"):  # Hive 0.11 overflow (throwOnHive11DecimalOverflow)
            with pytest.raises(orc_amd.ParseError, match=fx["error"]):
                _device_decimal(data, scales, n, fx["precision"], fx["scale"])
            return
        if fx.get("throw_on_overflow") is False:  # overflowing values -> NULL
            got, keep = _device_hive11_keep(data, scales, n, fx["scale"])
            vals = [v if k else None for v, k in zip(_to_int128(got), keep)]
            assert vals == fx["expected"]
            with pytest.raises(orc_amd.ParseError, match="more than 38 digits"):
                _device_decimal(data, scales, n, 0, fx["scale"])
            return
        got = _device_decimal(data, scales, n, fx["precision"], fx["scale"])
        vals = _to_int128(got) if fx["precision"] > 18 or fx["precision"] == 0 else [int(v) for v in got]
        assert vals == fx["expected"]
    else:
        secs = torch.from_numpy(orc_amd.rlev1_decode(data, n, True)).cuda()
        nanos = torch.from_numpy(orc_amd.rlev1_decode(sec, n, False)).cuda()
        orc_amd.timestamp_decode_device(orc_amd.default_context(0), secs, nanos)
        assert secs.cpu().tolist() == fx["expected"]
        assert nanos.cpu().tolist() == fx["expected_nanos"]


@pytest.mark.parametrize("precision", [10, 18, 30, 38])
@pytest.mark.parametrize("seed", range(3))
def test_random_decimals_vs_oracle(precision, seed):
    """~100k values across many 16 KB tiles (varints that straddle tiles and
    threads), scales spread around the column's so values are multiplied,
    divided (truncation toward zero) or kept."""
    rng = np.random.default_rng(seed * 100 + precision)
    n = 100_003
    bits = 62 if precision <= 18 else 126
    mags = [int(x) for x in rng.integers(0, 1 << 62, size=n, dtype=np.int64)]
    if bits > 62:
        mags = [(m << int(rng.integers(0, 64))) | int(rng.integers(0, 1 << 62)) for m in mags]
    vals = [-m if rng.random() < 0.5 else m for m in mags]
    vals[:5] = [0, -1, 1, (1 << (bits - 1)) - 1, -(1 << (bits - 1))]
    col_scale = int(rng.integers(0, min(precision, 18) + 1))
    scales = np.clip(col_scale + rng.integers(-18, 19, size=n), 0, 60).astype(np.int64)
    data = _zz_varints(vals)
    want = oracle.decimal_decode(data, scales, n, col_scale, precision > 18)
    got = _device_decimal(data, scales, n, precision, col_scale)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("seed", range(2))
def test_random_hive11_decimals_vs_oracle(seed):
    """Hive 0.11 decimals (precision 0) at forced scales: values up to 38
    digits rescaled up and down, against the oracle; then one value past
    10^38 - 1 and one varint past 128 bits raise the reference's error."""
    import orc_amd

    rng = np.random.default_rng(seed)
    n = 50_001
    forced = int(rng.integers(0, 12))
    scales = rng.integers(0, 24, size=n).astype(np.int64)
    vals = []
    for s in scales:
        # keep |v| * 10^(forced - s) within 38 digits
        digits = int(rng.integers(0, 39 - max(0, forced - int(s))))
        m = int(rng.integers(0, 10 ** min(digits, 18))) * 10 ** max(0, digits - 18)
        vals.append(-m if rng.random() < 0.5 else m)
    data = _zz_varints(vals)
    want = oracle.decimal_decode(data, scales, n, forced, 2)
    np.testing.assert_array_equal(_device_decimal(data, scales, n, 0, forced), want)
    with pytest.raises(orc_amd.ParseError, match="Hive 0.11 decimal was more than 38 digits"):
        _device_decimal(_zz_varints([1, 10 ** 38, 2]), [0, 0, 0], 3, 0, 0)
    with pytest.raises(orc_amd.ParseError, match="Hive 0.11 decimal was more than 38 digits"):
        _device_decimal(_zz_varints([5]) + bytes([0x80] * 19 + [0x01]), [0, 0], 2, 0, 0)


def test_decimal_errors_match_reference():
    import orc_amd

    data = _zz_varints([5, 7, 9])
    with pytest.raises(orc_amd.ParseError, match="Read past end of stream in Decimal64ColumnReader"):
        _device_decimal(data, [2, 2, 2, 2], 4, 12, 2)
    with pytest.raises(orc_amd.ParseError, match="Decimal scale out of range"):
        _device_decimal(data, [2, 30, 2], 3, 12, 2)
    # Decimal128 never raises on scale: 10^-28 of 7 truncates to 0
    assert _to_int128(_device_decimal(data, [2, 30, 2], 3, 30, 2)) == [5, 0, 9]


def test_random_timestamps_vs_oracle():
    import torch

    import orc_amd

    rng = np.random.default_rng(4)
    n = 200_000
    secs = rng.integers(-(1 << 40), 1 << 40, size=n, dtype=np.int64)
    secs[:3] = [-1420070401, -1420070400, 0]
    z = rng.integers(0, 8, size=n)
    base = rng.integers(0, 1_000_000, size=n)
    nanos = (base << 3) | z
    nanos[:3] = [(999_999_9 << 3) | 1, 5, 0]
    ws, wn = oracle.timestamp(secs, nanos)
    ds, dn = torch.from_numpy(secs.copy()).cuda(), torch.from_numpy(nanos.astype(np.int64)).cuda()
    orc_amd.timestamp_decode_device(orc_amd.default_context(0), ds, dn)
    np.testing.assert_array_equal(ds.cpu().numpy(), ws)
    np.testing.assert_array_equal(dn.cpu().numpy(), wn)


# ---- files ---------------------------------------------------------------

def _rows(path, fields=None):
    import orc_amd

    r = orc_amd.Reader(path, orc_amd.default_context(0))
    rows = []
    for s in range(r.num_stripes):
        rows.extend(r.read_stripe(s).to_pylist(fields))
    return rows


@pytest.mark.parametrize("name", ["decimal.orc", "decimal64_v2.orc", "decimal64_v2_cplusplus.orc"])
def test_decimal_files_match_pyarrow(name):
    po = pytest.importorskip("pyarrow.orc")
    from file_parity import path

    got = _rows(path(name))
    want = po.ORCFile(path(name)).read().to_pylist()
    assert got == want


def test_decimal_file_matches_reference_expected_output():
    """examples/expected/decimal.jsn.gz (ColumnPrinter output of the
    reference), decimals parsed exactly."""
    import gzip
    import json

    from file_parity import FILES, path

    with gzip.open(os.path.join(FILES, "decimal.jsn.gz"), "rt") as f:
        want = [json.loads(line, parse_float=decimal.Decimal) for line in f if line.strip()]
    got = _rows(path("decimal.orc"))
    assert len(got) == len(want) == 6000
    for i, (w, g) in enumerate(zip(want, got)):
        ew = w["_col0"]
        assert (ew is None and g["_col0"] is None) or decimal.Decimal(ew) == g["_col0"], i


def test_pyarrow_written_decimals_and_timestamps(tmp_path):
    pa = pytest.importorskip("pyarrow")
    from utc_zones import utc_tzdir

    os.environ["TZDIR"] = utc_tzdir()
    import pyarrow.orc as po

    import random

    rng = np.random.default_rng(9)
    prng = random.Random(9)
    n = 50_000
    null = rng.random(n) < 0.1

    def dec(p, s):
        vals = []
        for i in range(n):
            if null[i]:
                vals.append(None)
            else:
                m = prng.randrange(10 ** prng.randint(1, p))
                vals.append(decimal.Decimal(m if prng.random() < 0.5 else -m).scaleb(-s))
        return pa.array(vals, type=pa.decimal128(p, s))

    ts = rng.integers(-(1 << 61), 1 << 61, size=n, dtype=np.int64)
    ts[:4] = [0, -1, 1_500_000_000_123_456_789, -1_500_000_000_000_000_001]
    t = pa.table({"d": dec(15, 2), "w": dec(38, 10), "e": dec(18, 0),
                  "t": pa.array(ts, type=pa.timestamp("ns"), mask=null)})
    p = str(tmp_path / "dec_ts.orc")
    po.write_table(t, p, stripe_size=1 << 20)
    got = _rows(p)
    want = po.ORCFile(p).read()
    want_ns = want.column("t").cast(pa.int64()).to_pylist()
    want_rows = want.drop_columns(["t"]).to_pylist()
    for i, (g, w) in enumerate(zip(got, want_rows)):
        assert {k: g[k] for k in ("d", "w", "e")} == w, i
        gt = g["t"]
        assert (gt is None and want_ns[i] is None) or int(gt.astype(np.int64)) == want_ns[i], i
    assert len(got) == n


def test_hive11_file_non_throwing_mode_matches_throwing():
    """orc-file-11-format.orc (Hive 0.11 decimals) read with
    throwOnHive11DecimalOverflow(false): no value overflows, so every batch
    equals the throwing mode's (the nulling path runs and keeps hasNulls as
    the PRESENT stream has it)."""
    import orc_amd
    from file_parity import path

    r = orc_amd.Reader(path("orc-file-11-format.orc"), orc_amd.default_context(0))
    # every field but `ts` (a non-UTC writer zone's timestamps, not decoded)
    fields = [f for f in r.types[0].field_names if f != "ts"]
    want = r.read(fields)
    assert all(row["decimal1"] is not None for row in want[:10])
    r.set_hive11_decimal(6, throw_on_overflow=False)
    got = r.read(fields)
    assert got == want
