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
