"""CPU tests of the file-level host logic (tail / footer parsing, schema,
reference error texts) and of the parity checker itself: pyarrow's ORC
reader against the reference's expected ColumnPrinter output
(examples/expected/*.jsn.gz, tools/test/TestMatch.cc:124-151). No GPU."""
import os

import pytest

import orc_amd
from file_parity import (CORRUPT_FILES, PARITY_FILES, expected_json, path, printer_equal, pyarrow_rows,
                         supported_fields, to_printer_form)


def _pa():
    return pytest.importorskip("pyarrow.orc")


@pytest.mark.parametrize("name", PARITY_FILES)
def test_tail_matches_pyarrow(name):
    po = _pa()
    r = orc_amd.Reader(path(name))  # metadata only: no device context
    try:
        f = po.ORCFile(path(name))
    except Exception:
        pytest.skip("pyarrow cannot open %s" % name)
    assert r.num_rows == f.nrows
    assert r.num_stripes == f.nstripes
    if r.types[0].kind == 12:
        assert r.types[0].field_names == [fld.name for fld in f.schema]
    comp = {"UNCOMPRESSED": "NONE"}.get(f.compression, f.compression)
    assert r.compression == comp
    rows = sum(r.stripe(i)["num_rows"] for i in range(r.num_stripes))
    assert rows == r.num_rows


def test_tail_errors_use_reference_texts():
    with pytest.raises(orc_amd.ParseError, match="File size too small"):
        orc_amd.Reader(path("zero.orc"))
    with pytest.raises(orc_amd.ParseError, match="Not an ORC file"):
        orc_amd.Reader(b"XYZ" + bytes(100) + b"\x03")
    with pytest.raises(orc_amd.InvalidArgument):
        orc_amd.Reader(path("no_such_file.orc"))


def test_stripe_read_needs_a_device_context():
    r = orc_amd.Reader(path("TestOrcFile.test1.orc"))
    with pytest.raises(orc_amd.InvalidArgument):
        r.read_stripe(0)


def test_type_strings():
    r = orc_amd.Reader(path("TestOrcFile.test1.orc"))
    assert r.type_string() == (
        "struct<boolean1:boolean,byte1:tinyint,short1:smallint,int1:int,long1:bigint,float1:float,"
        "double1:double,bytes1:binary,string1:string,middle:struct<list:array<struct<int1:int,string1:string>>>,"
        "list:array<struct<int1:int,string1:string>>,map:map<string,struct<int1:int,string1:string>>>")
    r = orc_amd.Reader(path("orc_index_int_string.orc"))
    assert r.type_string() == "struct<_col0:int,_col1:varchar(4)>"


@pytest.mark.parametrize("name", ["TestOrcFile.test1.orc", "nulls-at-end-snappy.orc", "orc_index_int_string.orc",
                                  "TestStringDictionary.testRowIndex.orc"])
def test_checker_pinned_to_reference_expected_output(name):
    """pyarrow (the checker the GPU parity tests use) reproduces the
    reference's own expected rows for these files."""
    _pa()
    want = expected_json(name)
    assert want is not None
    r = orc_amd.Reader(path(name))
    fields = supported_fields(r)
    got = [to_printer_form(row) for row in pyarrow_rows(name, fields)]
    assert len(got) == len(want)
    for i, (w, g) in enumerate(zip(want, got)):
        w = {k: w[k] for k in fields}
        assert printer_equal(w, g), "row %d: %r vs %r" % (i, w, g)


def test_corrupt_fixtures_present():
    for name, _ in CORRUPT_FILES:
        assert os.path.exists(path(name))


def test_tail_with_wrapping_footer_length_is_rejected():
    """A PostScript footer length near 2^64 must not wrap the tail-size check
    (Reader.cc readPostscript / the tail bounds)."""
    from orc_craft import orc_file, type_msg

    good = orc_file(b"", [], [type_msg(12)], 0)
    assert orc_amd.Reader(good).num_rows == 0
    for flen in ((1 << 64) - 1, (1 << 64) - 5, 1 << 63, 10 ** 9):
        bad = orc_file(b"", [], [type_msg(12)], 0, footer_length_override=flen)
        with pytest.raises(orc_amd.ParseError, match="Invalid tail size"):
            orc_amd.Reader(bad)


@pytest.mark.parametrize("name", ["c4", "c5"])
def test_workload_files_have_the_configured_shape(tmp_path, name):
    """The configs[3] / configs[4] writers produce >= 3 stripes with a row
    index and the encodings the parity tests rely on (RLEv2, dictionaries,
    PRESENT streams); metadata only, no GPU."""
    _pa()
    from workload_files import make_c4, make_c5

    p = str(tmp_path / (name + ".orc"))
    {"c4": make_c4, "c5": make_c5}[name](p, 200_000, 1)
    r = orc_amd.Reader(p)
    assert r.num_rows == 200_000 and r.num_stripes >= 3 and r.row_index_stride == 10000
    assert r.compression == "ZSTD"
    kinds = [t.kind for t in r.types]
    if name == "c4":
        assert len(r.types[0].subtypes) == 16 and kinds.count(14) == 4 and kinds.count(15) == 3
    else:
        assert r.type_string() == "struct<s:struct<a:array<int>,m:map<string,int>>>"


def _testmatch():
    from conftest import load_golden
    return [d for d in load_golden("testmatch.json") if os.path.exists(path(d["file"]))]


@pytest.mark.parametrize("d", _testmatch(), ids=lambda d: d["file"])
def test_metadata_matches_reference_testmatch(d):
    """Reader metadata against the reference's TestMatch expectations
    (tools/test/TestMatch.cc:98-121 Metadata: compression, compression size,
    stripe count, row count, row index stride, content length, format
    version, software version, user metadata, type string); no GPU."""
    r = orc_amd.Reader(path(d["file"]))
    assert r.compression == d["compression"]
    assert r.compression_block_size == d["compression_size"]
    assert r.num_stripes == d["stripes"]
    assert r.num_rows == d["rows"]
    assert r.row_index_stride == d["row_index_stride"]
    assert r.content_length == d["content_length"]
    assert r.format_version == d["format_version"]
    assert r.software_version == d["software_version"]
    assert r.type_string() == d["type"]
    meta = r.metadata
    assert set(meta) == set(d["metadata"])
    for k, v in d["metadata"].items():
        assert meta[k] == bytes.fromhex(v), k
    assert "foo" not in meta


def test_hive11_decimal_options():
    """RowReaderOptions::forcedScaleOnHive11Decimal (default 6, Reader.hh:258-271)
    and throwOnHive11DecimalOverflow on a Hive 0.11 file (decimal1 has
    precision 0). No GPU."""
    r = orc_amd.Reader(path("orc-file-11-format.orc"))
    dec = [t for t in r.types if t.kind == 14]
    assert dec and all(t.precision == 0 for t in dec)
    assert r.hive11_scale == 6
    r.set_hive11_decimal(3)
    assert r.hive11_scale == 3
    r.set_hive11_decimal(4, throw_on_overflow=False)
    assert r.hive11_scale == 4
    with pytest.raises(orc_amd.OrcError):
        r.set_hive11_decimal(39)
    assert r.hive11_scale == 4
