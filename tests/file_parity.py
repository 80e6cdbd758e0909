"""Helpers for file-level parity: the example ORC files the reference's own
tests read (examples/*.orc, copied as data fixtures into tests/golden/files),
checked against pyarrow's ORC reader (Apache ORC C++ linked into pyarrow —
the reference implementation, used here only as the checker) and against the
reference's expected ColumnPrinter output (examples/expected/*.jsn.gz) where
it exists."""
import gzip
import json
import math
import os

from conftest import GOLDEN

FILES = os.path.join(GOLDEN, "files")

# (file, expected rows) — every example readable end to end by the GPU path
# for its supported columns. Timestamp / decimal / union columns are skipped
# by the comparison (not decoded this round).
PARITY_FILES = [
    "demo-12-zlib.orc",
    "demo-11-zlib.orc",
    "TestOrcFile.test1.orc",
    "nulls-at-end-snappy.orc",
    "orc_index_int_string.orc",
    "TestStringDictionary.testRowIndex.orc",
    "TestOrcFile.testSnappy.orc",
    "TestOrcFile.testWithoutIndex.orc",
    "TestVectorOrcFile.testLz4.orc",
    "TestVectorOrcFile.testZstd.0.12.orc",
    "orc-file-11-format.orc",
    "orc_no_format.orc",
    "complextypes_iceberg.orc",
    "TestOrcFile.testMemoryManagementV11.orc",
    "TestOrcFile.testMemoryManagementV12.orc",
    "TestOrcFile.columnProjection.orc",
    "over1k_bloom.orc",
    "TestOrcFile.emptyFile.orc",
    "bad_bloom_filter_1.6.11.orc",
    "TestOrcFile.testDate1900.orc",
    "orc_split_elim_cpp.orc",
    "TestOrcFile.metaData.orc",
    "TestOrcFile.testPredicatePushdown.orc",
    "TestOrcFile.testStringAndBinaryStatistics.orc",
    "TestOrcFile.testStripeLevelStats.orc",
    "TestOrcFile.testSargSkipPickupGroupWithoutIndexJava.orc",
    "TestOrcFile.testUnionAndTimestamp.orc",
    "version1999.orc",
]

# reference error texts (tools/test/TestFileScan.cc:226-236)
CORRUPT_FILES = [
    ("stripe_footer_bad_column_encodings.orc",
     ("bad number of ColumnEncodings in StripeFooter: expected=6, actual=0", "bad StripeFooter from zlib")),
    ("negative_dict_entry_lengths.orc", ("Negative dictionary entry length",)),
    ("missing_length_stream_in_string_dict.orc", ("LENGTH stream not found in StringDictionaryColumn",)),
    ("missing_blob_stream_in_string_dict.orc", ("DICTIONARY_DATA stream not found in StringDictionaryColumn",)),
]

UNSUPPORTED = set()  # every kind decodes (TIMESTAMP columns of non-UTC writers and Hive 0.11
# decimals are skipped via `decoded`)


def path(name):
    return os.path.join(FILES, name)


def supported_fields(reader, decoded=None):
    """Top-level fields whose whole subtree the GPU path decodes (`decoded`:
    the type ids a read actually decoded, e.g. without the TIMESTAMP columns
    of a writer zone other than UTC)."""
    def ok(tid):
        t = reader.types[tid]
        if decoded is not None and tid not in decoded:
            return False
        return t.kind not in UNSUPPORTED and all(ok(s) for s in t.subtypes)
    root = reader.types[0]
    if root.kind != 12:
        return []
    return [n for n, s in zip(root.field_names, root.subtypes) if ok(s)]


def pyarrow_rows(name, fields):
    import pyarrow.orc as po
    t = po.ORCFile(path(name)).read(columns=fields) if fields else None
    return [] if t is None else t.to_pylist()


def _ts_ns(x):
    """Timestamps as int nanoseconds: pyarrow gives pandas Timestamps (or
    datetimes), this reader numpy datetime64[ns]."""
    import datetime

    import numpy as np
    if isinstance(x, np.datetime64):
        return int(x.astype("datetime64[ns]").astype(np.int64))
    if hasattr(x, "value") and hasattr(x, "nanosecond"):  # pandas.Timestamp
        return int(x.value)
    if isinstance(x, datetime.datetime):
        d = x - datetime.datetime(1970, 1, 1, tzinfo=x.tzinfo)
        return (d.days * 86400 + d.seconds) * 10 ** 9 + d.microseconds * 1000
    return None


def same(a, b):
    """Deep equality with NaN == NaN and float32-widened floats; a UNION row
    (tag, value) equals pyarrow's bare value."""
    from orc_amd import UnionValue
    if isinstance(a, UnionValue) and not isinstance(b, UnionValue):
        return same(a.value, b)
    if isinstance(b, UnionValue) and not isinstance(a, UnionValue):
        return same(a, b.value)
    ta, tb = _ts_ns(a), _ts_ns(b)
    if ta is not None or tb is not None:
        return ta == tb
    if isinstance(a, float) and isinstance(b, float):
        return (math.isnan(a) and math.isnan(b)) or a == b
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(same(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    return a == b


def first_difference(want, got):
    if len(want) != len(got):
        return "row count %d != %d" % (len(want), len(got))
    for i, (w, g) in enumerate(zip(want, got)):
        if not same(w, g):
            return "row %d: expected %r got %r" % (i, w, g)
    return None


def expected_json(name):
    """examples/expected/<name>.jsn.gz rows (ColumnPrinter output), or None."""
    p = os.path.join(FILES, name.replace(".orc", ".jsn.gz"))
    if not os.path.exists(p):
        return None
    import decimal
    with gzip.open(p, "rt") as f:
        # decimals exact (ColumnPrinter prints them with every scale digit)
        return [json.loads(line, parse_float=decimal.Decimal) for line in f if line.strip()]


def printer_timestamp(x):
    """TimestampColumnPrinter::printRow (c++/src/ColumnPrinter.cc:668-700):
    gmtime seconds, '.', nanoseconds without trailing zeros (at least one
    digit)."""
    import datetime

    import numpy as np
    ns = int(x.astype("datetime64[ns]").astype(np.int64))
    secs, nanos = divmod(ns, 10 ** 9)
    t = datetime.datetime(1970, 1, 1) + datetime.timedelta(seconds=secs)
    frac = ("%09d" % nanos).rstrip("0") or "0"
    return t.strftime("%Y-%m-%d %H:%M:%S") + "." + frac


def to_printer_form(v):
    """Our / pyarrow row values in ColumnPrinter's JSON shape: binary as a
    list of byte values, maps as [{"key", "value"}], dates as ISO strings."""
    import datetime

    import numpy as np

    from orc_amd import UnionValue
    if isinstance(v, UnionValue):
        return {"tag": v.tag, "value": to_printer_form(v.value)}
    if isinstance(v, np.datetime64):
        return printer_timestamp(v)
    if isinstance(v, bytes):
        return list(v)
    if isinstance(v, datetime.date):
        return v.isoformat()
    if isinstance(v, dict):
        return {k: to_printer_form(x) for k, x in v.items()}
    if isinstance(v, list):
        return [{"key": to_printer_form(x[0]), "value": to_printer_form(x[1])} if isinstance(x, tuple)
                else to_printer_form(x) for x in v]
    return v


def printer_equal(expect, got):
    import decimal
    if isinstance(got, decimal.Decimal):  # decimal columns: exact
        return expect is not None and not isinstance(expect, bool) and decimal.Decimal(expect) == got
    if isinstance(expect, (float, decimal.Decimal)) or isinstance(got, float):
        if expect is None or got is None:
            return expect is got
        # ColumnPrinter prints floats with limited digits
        return math.isclose(float(expect), float(got), rel_tol=1e-6, abs_tol=1e-6)
    if isinstance(expect, dict):
        return isinstance(got, dict) and expect.keys() == got.keys() and all(
            printer_equal(expect[k], got[k]) for k in expect)
    if isinstance(expect, list):
        return isinstance(got, list) and len(expect) == len(got) and all(
            printer_equal(a, b) for a, b in zip(expect, got))
    return expect == got


# ---- columnar comparison (large files) -------------------------------------
# Row-by-row to_pylist comparison is too slow for millions of rows; these
# helpers compare one decoded stripe with pyarrow's Arrow arrays column by
# column with numpy, recursively through struct / list / map, at the
# non-null slots (the null masks are compared first).

def _ranges(starts, lens):
    """Concatenation of [starts[i], starts[i] + lens[i]) as one index array."""
    import numpy as np
    lens = np.asarray(lens, dtype=np.int64)
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, dtype=np.int64)
    first = np.repeat(np.cumsum(lens) - lens, lens)
    return np.repeat(np.asarray(starts, dtype=np.int64), lens) + (np.arange(total, dtype=np.int64) - first)


def _arrow_offsets(arr):
    import numpy as np
    off = np.frombuffer(arr.buffers()[1], dtype=np.int32 if arr.type.id in _SMALL_OFFSET_IDS() else np.int64)
    return off[arr.offset:arr.offset + len(arr) + 1].astype(np.int64)


def _SMALL_OFFSET_IDS():
    import pyarrow as pa
    return {pa.string().id, pa.binary().id, pa.list_(pa.int32()).id, pa.map_(pa.string(), pa.int32()).id}


def compare_column(reader, batch, tid, arr, ours_idx, theirs_idx, where=""):
    """Assert the decoded column `tid` of `batch` at rows `ours_idx` equals the
    Arrow array `arr` at `theirs_idx` (same length)."""
    import numpy as np
    import pyarrow as pa
    import pyarrow.compute as pc

    t = reader.types[tid]
    c = batch.columns.get(tid)
    assert c is not None, "%s: column %d not decoded" % (where, tid)
    n = len(ours_idx)
    valid_t = np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), dtype=bool)[theirs_idx] if n else \
        np.zeros(0, bool)
    valid_o = np.ones(n, bool) if c.not_null is None else c.not_null[ours_idx].astype(bool)
    assert np.array_equal(valid_o, valid_t), "%s col %d: null masks differ at %d" % (
        where, tid, int(np.argmax(valid_o != valid_t)))
    oi, ti = ours_idx[valid_o], theirs_idx[valid_o]
    k = t.kind
    if k in (0, 1, 2, 3, 4):  # boolean / byte / short / int / long
        want = np.asarray(arr.to_numpy(zero_copy_only=False))[ti].astype(np.int64)
        got = c.data[oi]
        assert np.array_equal(got, want), "%s col %d: first difference at row %d" % (
            where, tid, int(oi[np.argmax(got != want)]))
    elif k == 15:  # date: days since the epoch
        want = np.asarray(arr.cast(pa.int32()).to_numpy(zero_copy_only=False))[ti].astype(np.int64)
        assert np.array_equal(c.data[oi], want), "%s col %d (date) differs" % (where, tid)
    elif k in (5, 6):
        want = np.asarray(arr.cast(pa.float64()).to_numpy(zero_copy_only=False))[ti]
        got = c.data[oi]
        assert np.array_equal(got.view(np.int64), want.view(np.int64)) or np.array_equal(got, want, equal_nan=True), \
            "%s col %d (float) differs" % (where, tid)
    elif k == 14:  # decimal: unscaled values (int64, or [hi, lo] pairs past 18 digits)
        words = np.frombuffer(arr.buffers()[1], dtype=np.int64).reshape(-1, 2)[arr.offset:arr.offset + len(arr)]
        if t.precision > 18 or t.precision == 0:  # (0: Hive 0.11, Decimal128 at the forced scale)
            got = c.data.reshape(-1, 2)[oi]
            assert np.array_equal(got[:, 1], words[ti, 0]) and np.array_equal(got[:, 0], words[ti, 1]), \
                "%s col %d (decimal128) differs" % (where, tid)
        else:
            assert np.array_equal(c.data[oi], words[ti, 0]), "%s col %d (decimal64) differs" % (where, tid)
            assert np.array_equal(words[ti, 1], words[ti, 0] >> 63), "%s col %d: value past int64" % (where, tid)
    elif k in (7, 8, 16, 17):  # string / binary / varchar / char
        if arr.type != pa.binary() and arr.type != pa.string():
            arr = arr.cast(pa.string() if k != 8 else pa.binary())
        off = _arrow_offsets(arr)
        data = np.frombuffer(arr.buffers()[2], dtype=np.uint8) if arr.buffers()[2] is not None else \
            np.zeros(0, np.uint8)
        want_len = (off[1:] - off[:-1])[ti]
        got_len = c.length[oi]
        assert np.array_equal(got_len, want_len), "%s col %d: string lengths differ at row %d" % (
            where, tid, int(oi[np.argmax(got_len != want_len)]))
        blob = np.frombuffer(c.blob, dtype=np.uint8)
        got_b = blob[_ranges(c.data[oi], got_len)]
        want_b = data[_ranges(off[:-1][ti], want_len)]
        assert np.array_equal(got_b, want_b), "%s col %d: string bytes differ" % (where, tid)
    elif k in (10, 11):  # list / map
        off = _arrow_offsets(arr)
        want_len = (off[1:] - off[:-1])[ti]
        got_len = (c.offsets[1:] - c.offsets[:-1])[oi]
        assert np.array_equal(got_len, want_len), "%s col %d: lengths differ at row %d" % (
            where, tid, int(oi[np.argmax(got_len != want_len)]))
        co = _ranges(c.offsets[:-1][oi], got_len)
        ct = _ranges(off[:-1][ti], want_len)
        if k == 10:
            compare_column(reader, batch, t.subtypes[0], arr.values, co, ct, where)
        else:
            compare_column(reader, batch, t.subtypes[0], arr.keys, co, ct, where)
            compare_column(reader, batch, t.subtypes[1], arr.items, co, ct, where)
    elif k == 12:
        for i, st in enumerate(t.subtypes):
            compare_column(reader, batch, st, arr.field(i), ours_idx, theirs_idx, where)
    else:
        raise AssertionError("%s col %d: kind %d not compared" % (where, tid, k))
    del pc


def compare_stripe(reader, batch, record_batch, where=""):
    """Every top-level column of a decoded stripe against pyarrow's
    RecordBatch of the same stripe."""
    import numpy as np
    root = reader.types[0]
    n = record_batch.num_rows
    assert batch.num_rows == n, "%s: %d rows decoded, %d expected" % (where, batch.num_rows, n)
    idx = np.arange(n, dtype=np.int64)
    for i, (name, st) in enumerate(zip(root.field_names, root.subtypes)):
        compare_column(reader, batch, st, record_batch.column(i), idx, idx, "%s field %s" % (where, name))
