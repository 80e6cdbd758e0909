"""StringDirectColumnReader's length checks (c++/src/ColumnReader.cc:694-710
computeSize, then the blob read at :739-757) on hand-built stripes
(tests/orc_craft.py): a negative length (an unsigned LENGTH value of 2^63
or more read as int64), a total that overflows, and a blob shorter than the
lengths, each raised with the reference's ParseError text by the file reader
and by the row reader."""
import numpy as np
import pytest

import orc_amd
from orc_craft import field_bytes, field_varint, orc_file, stripe_info, type_msg

pytestmark = pytest.mark.gpu


def _string_file(lengths, blob):
    """struct<s:string> (type ids 0, 1), DIRECT_V2, one stripe, no row index."""
    ln, _ = orc_amd.encode_direct(np.asarray(lengths, dtype=np.int64), False, aligned=True)
    streams = [(2, 1, ln.tobytes()), (1, 1, bytes(blob))]  # LENGTH, DATA
    body = b"".join(s[2] for s in streams)
    sf = b"".join(field_bytes(1, field_varint(1, k) + field_varint(2, c) + field_varint(3, len(b)))
                  for k, c, b in streams)
    sf += field_bytes(2, field_varint(1, 0)) + field_bytes(2, field_varint(1, 2))  # DIRECT, DIRECT_V2
    n = len(lengths)
    info = stripe_info(3, 0, len(body), len(sf), n)
    types = [type_msg(12, [1], ["s"]), type_msg(7)]
    return orc_file(body + sf, [info], types, n)


CASES = [
    ("negative", [3, -5, 2, 4], b"abcdefghij", "Negative string length in StringDirectColumnReader for column 1"),
    ("overflow", [3, (1 << 63) - 1, (1 << 63) - 1, 4], b"abcdefghij",
     "String length overflow in StringDirectColumnReader for column 1"),
    ("short_blob", [3, 100, 2], b"abcdefghij", "failed to read in StringDirectColumnReader.next"),
]


@pytest.mark.parametrize("name,lengths,blob,msg", CASES, ids=[c[0] for c in CASES])
def test_direct_string_length_checks(tmp_path, name, lengths, blob, msg):
    p = tmp_path / ("sd_%s.orc" % name)
    p.write_bytes(_string_file(lengths, blob))
    r = orc_amd.Reader(str(p), orc_amd.default_context(0))
    with pytest.raises(orc_amd.ParseError, match=msg):
        r.read_stripe(0)
    rr = r.create_row_reader()
    with pytest.raises(orc_amd.ParseError, match=msg):
        rr.next(rr.create_row_batch(1024))


def test_direct_string_good(tmp_path):
    """The same stripe shape with good lengths decodes (the checks pass)."""
    lengths = [3, 0, 5, 2]
    blob = b"abcdefghij"
    p = tmp_path / "sd_good.orc"
    p.write_bytes(_string_file(lengths, blob))
    r = orc_amd.Reader(str(p), orc_amd.default_context(0))
    rows = [row["s"] for row in r.read_stripe(0).to_pylist()]
    assert rows == ["abc", "", "defgh", "ij"]
