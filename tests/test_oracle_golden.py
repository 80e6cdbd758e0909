"""Pin the CPU oracle against the reference's own known-answer vectors.

Fixtures: tests/golden/kat_*.json (make_kat_fixtures.py) — byte strings and
asserted values from c++/test/TestRleDecoder.cc, c++/test/TestByteRle.cc and
site/specification/ORCv1.md. Runs on CPU only.
"""
import numpy as np
import pytest

from conftest import assert_matches, decode_batches, load_golden
from oracle import oracle

RLEV2 = load_golden("kat_rlev2.json")
BYTE = load_golden("kat_byterle.json")
BOOL = load_golden("kat_boolrle.json")
RLEV1 = load_golden("kat_rlev1.json")


def _batches(fx):
    return fx["batches"]


@pytest.mark.parametrize("fx", RLEV2, ids=[f["name"] for f in RLEV2])
def test_rlev2_kat(fx):
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    for b in _batches(fx):
        dec = oracle.RleDecoderV2(data, fx["signed"])
        got = decode_batches(dec.next, fx["expected"], b, nn)
        assert_matches(fx["expected"], got, nn, "%s batch=%s" % (fx["name"], b))
    if "seek" in fx:
        dec = oracle.RleDecoderV2(data, fx["signed"])
        dec.seek(*fx["seek"]["position"])
        exp = fx["seek"]["expected"]
        got = list(dec.next(3)) + list(dec.next(3)) + list(dec.next(1))
        assert got == exp


@pytest.mark.parametrize("fx", RLEV2, ids=[f["name"] for f in RLEV2])
def test_rlev2_kat_narrow(fx):
    """int32 / int16 outputs are static_cast narrowings (RleDecoderV2.cc:172-182)."""
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    n = len(fx["expected"])
    for dt, bits in ((np.int32, 32), (np.int16, 16)):
        dec = oracle.RleDecoderV2(data, fx["signed"])
        got = dec.next(n, nn, dtype=dt)
        for i, e in enumerate(fx["expected"]):
            if e is None or (nn is not None and not nn[i]):
                continue
            m = e & ((1 << bits) - 1)
            if m >> (bits - 1):
                m -= 1 << bits
            assert int(got[i]) == m


@pytest.mark.parametrize("fx", BYTE, ids=[f["name"] for f in BYTE])
def test_byterle_kat(fx):
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    for b in _batches(fx):
        dec = oracle.ByteRleDecoder(data)
        got = decode_batches(dec.next, fx["expected"], b, nn)
        assert_matches(fx["expected"], got, nn, fx["name"])


@pytest.mark.parametrize("fx", BOOL, ids=[f["name"] for f in BOOL])
def test_boolrle_kat(fx):
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    for b in _batches(fx):
        dec = oracle.ByteRleDecoder(data, boolean=True)
        got = decode_batches(dec.next, fx["expected"], b, nn)
        assert_matches(fx["expected"], got, nn, fx["name"])


@pytest.mark.parametrize("fx", RLEV1, ids=[f["name"] for f in RLEV1])
def test_rlev1_kat(fx):
    data = bytes.fromhex(fx["data"])
    nn = fx.get("not_null")
    for b in _batches(fx):
        dec = oracle.RleDecoderV1(data, fx["signed"])
        got = decode_batches(dec.next, fx["expected"], b, nn)
        assert_matches(fx["expected"], got, nn, "%s batch=%s" % (fx["name"], b))
    for sk in fx.get("seeks", []):
        dec = oracle.RleDecoderV1(data, fx["signed"])
        dec.seek(*sk["position"])
        assert list(dec.next(len(sk["expected"]))) == sk["expected"]


def test_rlev2_errors_match_reference_messages():
    # PATCHED_BASE with pl == 0 (RleDecoderV2.cc:306-308)
    with pytest.raises(oracle.OracleError, match=r"pl==0"):
        oracle.RleDecoderV2(bytes([0x8E, 0x09, 0x2B, 0x20, 0x07, 0xD0]), False).next(10)
    # DELTA with W != 0 and L < 2 (:411-415)
    with pytest.raises(oracle.OracleError, match="Illegal run length for delta encoding: 1"):
        oracle.RleDecoderV2(bytes([0xC2, 0x00, 0x02, 0x02]), False).next(1)
    # truncated stream (:38)
    with pytest.raises(oracle.OracleError, match="bad read in RleDecoderV2::readByte"):
        oracle.RleDecoderV2(bytes([0x5E, 0x03, 0x5C]), False).next(4)


def test_byterle_bad_read():
    with pytest.raises(oracle.OracleError, match="bad read"):
        oracle.ByteRleDecoder(bytes([0xFE, 0x01])).next(2)


def test_dict_gather_bounds():
    start, ln = oracle.dict_gather([0, 2, 1], [3, 0, 5])
    assert list(start) == [0, 3, 3] and list(ln) == [3, 5, 0]
    with pytest.raises(oracle.OracleError, match="Entry index out of range"):
        oracle.dict_gather([3], [1, 2, 3])


DECIMAL = load_golden("kat_decimal.json")


def _kat_nonnull(fx):
    if not fx.get("present"):
        return len(fx["expected"])
    dec = oracle.ByteRleDecoder(bytes.fromhex(fx["present"]), boolean=True)
    return int(np.count_nonzero(dec.next(len(fx["expected"]) * 2 + 64)[: 10 ** 6]))


def _i128(h, lo):
    v = ((int(h) & ((1 << 64) - 1)) << 64) | (int(lo) & ((1 << 64) - 1))
    return v - (1 << 128) if v >> 127 else v


@pytest.mark.parametrize("fx", DECIMAL, ids=[f["name"] for f in DECIMAL])
def test_decimal_timestamp_kat(fx):
    """Decimal64/128 and timestamp known answers of TestColumnReader.cc: the
    SECONDARY stream through the RLEv1 oracle, then the value construction."""
    n = len(fx["expected"])
    sec = bytes.fromhex(fx["secondary"])
    data = bytes.fromhex(fx["data"])
    if fx["kind"] == "decimal":
        scales = oracle.RleDecoderV1(sec, True).next(n)
        wide = 2 if fx["precision"] == 0 else fx["precision"] > 18  # 2: Hive 0.11 (forced scale)
        if fx.get("error"):
            with pytest.raises(oracle.OracleError, match=fx["error"]):
                oracle.decimal_decode(data, scales, n, fx["scale"], wide)
            return
        if fx.get("throw_on_overflow") is False:
            # throwOnHive11DecimalOverflow(false): overflow -> NULL (None)
            got, keep = oracle.decimal_decode_keep(data, scales, n, fx["scale"])
            vals = [_i128(h, lo) if k else None for (h, lo), k in zip(got, keep)]
            assert vals == fx["expected"]
            with pytest.raises(oracle.OracleError, match="more than 38 digits"):
                oracle.decimal_decode(data, scales, n, fx["scale"], wide)
            return
        got = oracle.decimal_decode(data, scales, n, fx["scale"], wide)
        if wide:
            vals = [(((int(h) & ((1 << 64) - 1)) << 64) | (int(lo) & ((1 << 64) - 1))) for h, lo in got]
            vals = [v - (1 << 128) if v >> 127 else v for v in vals]
        else:
            vals = [int(v) for v in got]
        assert vals == fx["expected"]
    else:
        secs = oracle.RleDecoderV1(data, True).next(n)
        nanos = oracle.RleDecoderV1(sec, False).next(n)
        s, ns = oracle.timestamp(secs, nanos)
        assert list(s) == fx["expected"]
        assert list(ns) == fx["expected_nanos"]


def test_decimal_errors():
    # varint stream ends early; scale 20 digits away from the column's
    with pytest.raises(oracle.OracleError, match="Read past end of stream in Decimal64ColumnReader"):
        oracle.decimal_decode(bytes([6, 0x80]), [2, 2], 2, 2, False)
    with pytest.raises(oracle.OracleError, match="Decimal scale out of range"):
        oracle.decimal_decode(bytes([6]), [22], 1, 2, False)
    # Decimal128 has no range error: 10^-20 of 3 truncates to 0
    assert oracle.decimal_decode(bytes([6]), [22], 1, 2, True).tolist() == [[0, 0]]
