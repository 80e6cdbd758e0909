"""throwOnHive11DecimalOverflow(false) through the file reader and the
RowReader on a value that really overflows.

DecimalHive11ColumnReader::next (c++/src/ColumnReader.cc:1627-1687): a value
whose varint runs past 128 bits or whose magnitude exceeds 10^38 - 1 either
raises "Hive 0.11 decimal was more than 38 digits." or, with
throwOnHive11DecimalOverflow(false), becomes NULL: notNull[i] = 0 and
hasNulls = true (:1650-1677), the other values kept and rescaled to the
forced scale. The stripe is hand-built (tests/orc_craft.py wire helpers): a
struct<d:decimal> whose decimal has precision 0 (Hive 0.11), with and
without a PRESENT stream."""
import decimal

import numpy as np
import pytest

import orc_amd
from orc_craft import field_bytes, field_varint, orc_file, stripe_info, type_msg, varint

pytestmark = pytest.mark.gpu


def _zigzag_varint(v):
    z = (v << 1) if v >= 0 else ((-v) << 1) - 1
    out = bytearray()
    while True:
        b = z & 0x7F
        z >>= 7
        if z:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _bool_rle(bits):
    """Boolean RLE: bits MSB first into bytes, as literal groups (ORCv1.md)."""
    padded = list(bits) + [0] * (-len(bits) % 8)
    by = bytes(int("".join(str(b) for b in padded[i:i + 8]), 2) for i in range(0, len(padded), 8))
    out = bytearray()
    for i in range(0, len(by), 128):
        chunk = by[i:i + 128]
        out.append(256 - len(chunk))
        out += chunk
    return bytes(out)


def _hive11_file(values, scales, present):
    """struct<d:decimal(0,0)> (type ids 0, 1), one stripe, no row index."""
    data = b"".join(_zigzag_varint(v) for v in values)
    sec, _ = orc_amd.encode_direct(np.asarray(scales, dtype=np.int64), True, aligned=True)
    streams = []  # (kind, column, bytes): PRESENT 0, DATA 1, SECONDARY 5
    if present is not None:
        streams.append((0, 1, _bool_rle(present)))
    streams += [(1, 1, data), (5, 1, sec.tobytes())]
    body = b"".join(s[2] for s in streams)
    sf = b"".join(field_bytes(1, field_varint(1, k) + field_varint(2, c) + field_varint(3, len(b)))
                  for k, c, b in streams)
    sf += field_bytes(2, field_varint(1, 0)) + field_bytes(2, field_varint(1, 2))  # DIRECT, DIRECT_V2
    n = len(present) if present is not None else len(values)
    info = stripe_info(3, 0, len(body), len(sf), n)
    types = [type_msg(12, [1], ["d"]), type_msg(14) + field_varint(5, 0) + field_varint(6, 0)]
    return orc_file(body + sf, [info], types, n)


def _expect(values, scales, present, forced=6):
    out, k = [], 0
    for r in range(len(present) if present is not None else len(values)):
        if present is not None and not present[r]:
            out.append(None)
            continue
        v, s = values[k], scales[k]
        k += 1
        u = v * 10 ** (forced - s) if s <= forced else v // 10 ** (s - forced)
        out.append(None if abs(v) >= 10 ** 38 or abs(u) >= 10 ** 38 else decimal.Decimal(u).scaleb(-forced))
    return out


BIG = 10 ** 39 + 7  # 40 digits: more than 38


@pytest.mark.parametrize("with_present", [True, False])
def test_hive11_overflow_becomes_null(tmp_path, with_present):
    # BIG runs past 128 bits (readInt128's varint check); 15 * 10^31 at scale 0
    # is 1.5 * 10^38 at the forced scale 6: in 128 bits, above 10^38 - 1.
    # (scaleInt128's multiply wraps at 128 bits in the reference, so no
    # value here is scaled past 2^127.)
    values = [12345, -7, BIG, 99, -(10 ** 31), 0, BIG * 3, 15 * 10 ** 31, 42]
    scales = [2, 0, 1, 3, 1, 0, 2, 0, 6]
    present = [1, 1, 0, 1, 1, 1, 0, 1, 1, 1, 1] if with_present else None
    p = tmp_path / ("h11_%d.orc" % with_present)
    p.write_bytes(_hive11_file(values, scales, present))
    want = _expect(values, scales, present)
    assert any(w is None for w in want)

    r = orc_amd.Reader(str(p), orc_amd.default_context(0))
    # throwing mode (the default): the reference's ParseError
    with pytest.raises(orc_amd.ParseError, match="Hive 0.11 decimal was more than 38 digits"):
        r.read_stripe(0)
    r.set_hive11_decimal(6, throw_on_overflow=False)
    b = r.read_stripe(0)
    got = [row["d"] for row in b.to_pylist()]
    assert got == want
    c = b.columns[1]
    assert c.not_null is not None, "hasNulls must be set when a value overflowed"
    assert [bool(x) for x in c.not_null[:len(want)]] == [w is not None for w in want]

    # the RowReader (its pinned slab and batch views) at two capacities
    for cap in (3, 1024):
        rr = r.create_row_reader()
        batch = rr.create_row_batch(cap)
        rows = []
        while rr.next(batch):
            rows += [row["d"] for row in batch.to_pylist()]
        assert rows == want, cap


def _hive11_multi_file(cols):
    """struct<d0, d1, ...: decimal(0,0)> (type ids 0 .. k), one stripe, no row
    index; cols = [(values, scales, present or None)], same row count."""
    body, sf, n = b"", b"", None
    for ci, (values, scales, present) in enumerate(cols, start=1):
        sec, _ = orc_amd.encode_direct(np.asarray(scales, dtype=np.int64), True, aligned=True)
        streams = []
        if present is not None:
            streams.append((0, ci, _bool_rle(present)))
        streams += [(1, ci, b"".join(_zigzag_varint(v) for v in values)), (5, ci, sec.tobytes())]
        for k, c, b in streams:
            body += b
            sf += field_bytes(1, field_varint(1, k) + field_varint(2, c) + field_varint(3, len(b)))
        rows = len(present) if present is not None else len(values)
        assert n is None or n == rows
        n = rows
    sf += field_bytes(2, field_varint(1, 0))  # root: DIRECT
    sf += b"".join(field_bytes(2, field_varint(1, 2)) for _ in cols)  # decimals: DIRECT_V2
    info = stripe_info(3, 0, len(body), len(sf), n)
    types = [type_msg(12, list(range(1, len(cols) + 1)), ["d%d" % i for i in range(len(cols))])]
    types += [type_msg(14) + field_varint(5, 0) + field_varint(6, 0) for _ in cols]
    return orc_file(body + sf, [info], types, n)


def test_hive11_overflow_sibling_columns(tmp_path):
    """Sibling Hive 0.11 columns under the root struct decode on different
    side streams (ORCG_LANES): each keeps its own overflow count and null
    mask (a shared count word let one column read
    another's)."""
    rows = 11
    vals_ok = [1, -2, 3, 4, 5, -6, 7, 8, 9, 10, 11]
    vals_a = [12345, BIG, -7, 99, BIG * 5, 0, 15 * 10 ** 31, 42, 1, 2, 3]
    vals_b = [5, 6, BIG, 8, 9, 10, 11]
    pres_b = [1, 0, 1, 1, 0, 1, 1, 0, 1, 0, 1]
    cols = [(vals_ok, [0] * rows, None), (vals_a, [2, 0, 0, 3, 1, 0, 0, 6, 1, 1, 1], None),
            (vals_b, [1, 1, 1, 1, 1, 1, 1], pres_b), (list(reversed(vals_a)), [0] * rows, None)]
    p = tmp_path / "h11_multi.orc"
    p.write_bytes(_hive11_multi_file(cols))
    want = [_expect(v, s, pr) for v, s, pr in cols]
    r = orc_amd.Reader(str(p), orc_amd.default_context(0))
    r.set_hive11_decimal(6, throw_on_overflow=False)
    for _ in range(3):  # repeated stripe reads: each reuses the stripe's read-back block
        b = r.read_stripe(0)
        got = b.to_pylist()
        for ci, w in enumerate(want):
            assert [row["d%d" % ci] for row in got] == w, ci
            c = b.columns[ci + 1]
            if all(x is not None for x in w):
                assert c.not_null is None or all(bool(x) for x in c.not_null[:rows]), ci
            else:
                assert c.not_null is not None, ci
                assert [bool(x) for x in c.not_null[:rows]] == [x is not None for x in w], ci
