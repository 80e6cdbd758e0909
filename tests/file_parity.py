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

UNSUPPORTED = {13}  # UNION (TIMESTAMP columns of non-UTC writers are skipped via `decoded`)


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
    """Deep equality with NaN == NaN and float32-widened floats."""
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
    with gzip.open(p, "rt") as f:
        return [json.loads(line) for line in f if line.strip()]


def to_printer_form(v):
    """Our / pyarrow row values in ColumnPrinter's JSON shape: binary as a
    list of byte values, maps as [{"key", "value"}], dates as ISO strings."""
    import datetime
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
    if isinstance(expect, float) or isinstance(got, float):
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
