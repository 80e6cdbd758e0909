"""The C++ adapter (orc_amd/csrc/GpuRleDecoder.hh) compiled as a reference-
style host program: compiles on CPU; runs the KATs through it on the GPU."""
import os
import subprocess

import pytest

from conftest import ROOT, load_golden

SRC = os.path.join(ROOT, "tests", "cxx", "adapter_test.cpp")
OUT = os.path.join(ROOT, "tests", "cxx", "build", "adapter_test")


def build_adapter_test():
    from orc_amd import build as orc_build

    orc_build.build()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.check_call([
        "g++", "-std=c++17", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", SRC, "-o", OUT,
        "-L" + os.path.join(ROOT, "orc_amd"), "-lorcgpu", "-Wl,-rpath," + os.path.join(ROOT, "orc_amd"),
        "-Wl,-rpath,/opt/rocm/lib",
    ])
    return OUT


def test_adapter_compiles_and_links():
    assert os.access(build_adapter_test(), os.X_OK)


def _fixture_lines():
    lines = []
    for fx in load_golden("kat_rlev2.json"):
        if "not_null" in fx:
            continue
        exp = ["x" if e is None else str(e) for e in fx["expected"]]
        lines.append("rlev2 %d %s %d %s" % (int(fx["signed"]), fx["data"], len(exp), " ".join(exp)))
    for name, kind in (("kat_byterle.json", "byte"), ("kat_boolrle.json", "bool")):
        for fx in load_golden(name):
            if "not_null" in fx:
                continue
            exp = ["x" if e is None else str(e) for e in fx["expected"]]
            lines.append("%s 0 %s %d %s" % (kind, fx["data"], len(exp), " ".join(exp)))
    return lines


@pytest.mark.gpu
def test_adapter_kats_on_gpu(tmp_path):
    exe = build_adapter_test()
    f = tmp_path / "kats.txt"
    f.write_text("\n".join(_fixture_lines()) + "\n")
    r = subprocess.run([exe, str(f)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK")


READER_SRC = os.path.join(ROOT, "tests", "cxx", "reader_test.cpp")
READER_OUT = os.path.join(ROOT, "tests", "cxx", "build", "reader_test")


def build_reader_test():
    from orc_amd import build as orc_build

    orc_build.build()
    os.makedirs(os.path.dirname(READER_OUT), exist_ok=True)
    subprocess.check_call([
        "g++", "-std=c++17", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", READER_SRC, "-o",
        READER_OUT, "-L" + os.path.join(ROOT, "orc_amd"), "-lorcgpu",
        "-Wl,-rpath," + os.path.join(ROOT, "orc_amd"), "-Wl,-rpath,/opt/rocm/lib",
    ])
    return READER_OUT


def test_row_reader_adapter_compiles_and_links():
    assert os.access(build_reader_test(), os.X_OK)


def _run_reader(name, *args):
    import json
    import decimal

    from file_parity import path

    exe = build_reader_test()
    r = subprocess.run([exe, path(name)] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    out = []
    for line in r.stdout.splitlines():
        if line.startswith("#"):
            out.append(line.split())
        elif line.strip():
            out.append(json.loads(line, parse_float=decimal.Decimal))
    return out


def _include(name):
    """Top-level columns the GPU path decodes in this file (timestamps of
    non-UTC writer zones and Hive 0.11 decimals are not): their type ids, and
    the expected rows restricted to them."""
    import orc_amd
    from file_parity import expected_json, path

    r = orc_amd.Reader(path(name), orc_amd.default_context(0))
    root = r.types[0]
    decoded = set(r.read_stripe(0).columns) if r.num_stripes else set()

    def ok(t):
        return t in decoded and all(ok(s) for s in r.types[t].subtypes)
    fields = [(n, s) for n, s in zip(root.field_names, root.subtypes) if ok(s)]
    want = [{k: w[k] for k, _ in fields} for w in expected_json(name)]
    return ",".join(str(s) for _, s in fields), want


CXX_FILES = ["TestOrcFile.test1.orc", "decimal.orc", "nulls-at-end-snappy.orc", "orc_index_int_string.orc",
             "TestOrcFile.testSnappy.orc", "TestOrcFile.testSeek.orc", "TestOrcFile.testUnionAndTimestamp.orc",
             "over1k_bloom.orc", "TestStringDictionary.testRowIndex.orc"]


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 1000, 1024, 5000])
@pytest.mark.parametrize("name", CXX_FILES)
def test_row_reader_adapter_matches_expected_output(name, batch):
    """orc::Reader / RowReader::createRowBatch(capacity) / next(batch) /
    getRowNumber through the C++ adapter (GpuRowReader.hh), every row against
    the reference's expected ColumnPrinter output (tools/test/TestMatch.cc
    Contents); reader_test itself checks numElements <= capacity and
    getRowNumber() == the batch's first row."""
    from file_parity import printer_equal

    if batch == 1 and name == "TestOrcFile.testSeek.orc":
        pytest.skip("32,768 single-row batches: covered at the other capacities")
    inc, want = _include(name)
    got = _run_reader(name, "--batch", batch, "--include", inc)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert printer_equal(w, g), (name, i, w, g)


@pytest.mark.gpu
def test_row_reader_adapter_seek_to_row():
    """seekToRow at row-group (stride 1,000) and stripe edges of testSeek.orc."""
    import numpy as np

    import orc_amd
    from file_parity import path, printer_equal

    name = "TestOrcFile.testSeek.orc"
    inc, want = _include(name)
    r = orc_amd.Reader(path(name))
    firsts = np.cumsum([0] + [r.stripe(s)["num_rows"] for s in range(r.num_stripes)])
    targets = [0, 999, 1000, 1001, 12345, int(firsts[1]), int(firsts[1]) - 1, int(firsts[3]), r.num_rows - 1]
    out = _run_reader(name, "--batch", 50, "--include", inc, "--seek", ",".join(map(str, targets)))
    i = 0
    for t in targets:
        tag = out[i]
        assert tag[0] == "#seek" and int(tag[1]) == t and int(tag[2]) == t
        n = int(tag[3])
        s = int(np.searchsorted(firsts, t, side="right") - 1)
        assert n == min(50, int(firsts[s + 1]) - t)
        for k in range(n):
            assert printer_equal(want[t + k], out[i + 1 + k]), (t, k)
        i += 1 + n
    assert i == len(out)


@pytest.mark.gpu
def test_row_reader_adapter_range_and_lazy_decoding():
    """RowReaderOptions::range (stripes 2..4 of testSeek.orc by byte offset)
    and setEnableLazyDecoding (EncodedStringVectorBatch index + dictionary)."""
    import numpy as np

    import orc_amd
    from file_parity import path, printer_equal

    name = "TestOrcFile.testSeek.orc"
    inc, want = _include(name)
    r = orc_amd.Reader(path(name))
    st = [r.stripe(s) for s in range(r.num_stripes)]
    firsts = np.cumsum([0] + [x["num_rows"] for x in st])
    off = st[2]["offset"]
    length = st[4]["offset"] - off + 1
    out = _run_reader(name, "--batch", 3000, "--include", inc, "--range", off, length, "--lazy")
    assert out[0] == ["#first", str(int(firsts[2]))]
    rows = out[1:]
    assert len(rows) == firsts[5] - firsts[2]
    for k, g in enumerate(rows):
        assert printer_equal(want[int(firsts[2]) + k], g), k


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["TestOrcFile.test1.orc", "over1k_bloom.orc", "TestOrcFile.testSeek.orc"])
def test_row_reader_adapter_tight_numeric_vectors(name):
    """RowReaderOptions::setUseTightNumericVector (Reader.hh:375): BOOLEAN /
    BYTE -> ByteVectorBatch, SHORT -> ShortVectorBatch, INT ->
    IntVectorBatch, FLOAT -> FloatVectorBatch (ColumnReader.cc:1703-1790);
    the rows print exactly as the reference's expected output."""
    from file_parity import printer_equal

    inc, want = _include(name)
    got = _run_reader(name, "--batch", 777, "--include", inc, "--tight")
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert printer_equal(w, g), (name, i, w, g)


@pytest.mark.gpu
def test_two_row_readers_keep_their_own_options():
    """Each RowReader keeps its RowReaderOptions (include, lazy decoding):
    interleaving two of them, and a stripe read on the reader itself, changes
    neither one's batches (options used to live on the reader)."""
    import numpy as np

    import orc_amd
    from file_parity import path

    r = orc_amd.Reader(path("TestOrcFile.testSeek.orc"), orc_amd.default_context(0))
    root = r.types[0]
    ids = dict(zip(root.field_names, root.subtypes))
    a = r.create_row_reader(include=["int1", "string1"], lazy_dictionary=True)
    b = r.create_row_reader(include=["long1"])
    ba, bb = a.create_row_batch(3000), b.create_row_batch(2000)
    rows_a, rows_b = [], []
    more_a = more_b = True
    k = 0
    while more_a or more_b:
        if more_a:
            more_a = a.next(ba)
            if more_a:
                assert set(ba.columns) == {0, ids["int1"], ids["string1"]}
                assert ba.columns[ids["string1"]].index is not None  # lazy: index + dictionary
                rows_a.extend(ba.to_pylist(["int1", "string1"]))
        if more_b:
            more_b = b.next(bb)
            if more_b:
                assert set(bb.columns) == {0, ids["long1"]}
                rows_b.extend(bb.to_pylist(["long1"]))
        if k % 3 == 0:
            r.read_stripe(k % r.num_stripes)  # the reader's own read in between
        k += 1
    assert len(rows_a) == len(rows_b) == r.num_rows
    full = r.read()
    assert rows_a == [{"int1": x["int1"], "string1": x["string1"]} for x in full]
    assert rows_b == [{"long1": x["long1"]} for x in full]
    assert a.is_selected(ids["int1"]) and not a.is_selected(ids["long1"])
    assert np.all([b.is_selected(ids["long1"]), not b.is_selected(ids["int1"])])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["TestOrcFile.testSeek.orc", "TestOrcFile.testUnionAndTimestamp.orc",
                                  "TestStringDictionary.testRowIndex.orc"])
def test_row_reader_adapter_pinned_memory_pool(name):
    """ReaderOptions::setMemoryPool (Reader.hh:123, MemoryPool.hh:27-33): the
    batches and dictionaries allocated from the caller's pool, here
    PinnedMemoryPool (page-locked memory from orcg_host_alloc); every row
    against the reference's expected output, capacities 1000 and 1024, with
    the batch copies spread over the copy pool's helper threads."""
    from file_parity import printer_equal

    inc, want = _include(name)
    for batch in (1000, 1024):
        got = _run_reader(name, "--batch", batch, "--include", inc, "--pinned")
        assert len(got) == len(want)
        for i, (g, w) in enumerate(zip(got, want)):
            assert printer_equal(w, g), (name, batch, i, w, g)
