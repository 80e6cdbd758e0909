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


def _canon(v):
    """pyarrow row values and the adapter's JSON in one comparable shape."""
    import datetime
    import decimal
    import math

    from file_parity import _ts_ns
    if v is None or isinstance(v, bool):
        return v
    ts = _ts_ns(v)
    if ts is not None:
        return ("ts", ts)
    if isinstance(v, datetime.date):
        return (v - datetime.date(1970, 1, 1)).days
    if isinstance(v, decimal.Decimal):
        return ("dec", v)
    if isinstance(v, float):
        return "nan" if math.isnan(v) else v
    if isinstance(v, bytes):
        return list(v)
    if isinstance(v, dict):
        return [_canon(x) for x in v.values()]
    if isinstance(v, (list, tuple)):
        return [_canon(x) for x in v]
    return v


def _canon_json(v, t, reader):
    """The adapter's printed value for type id t (DECIMAL strings, TIMESTAMP [s, ns])."""
    import decimal

    k = reader.types[t].kind
    if v is None:
        return None
    if k == 14:
        return ("dec", decimal.Decimal(v))
    if k in (9, 18):
        return ("ts", v[0] * 10 ** 9 + v[1])
    if k in (5, 6):
        return "nan" if v != v else float(v)
    if k == 10:
        return [_canon_json(x, reader.types[t].subtypes[0], reader) for x in v]
    if k == 11:
        ks, vs = reader.types[t].subtypes
        return [[_canon_json(a, ks, reader), _canon_json(b, vs, reader)] for a, b in v]
    if k == 12:
        return [_canon_json(x, st, reader) for x, st in zip(v, reader.types[t].subtypes)]
    return v


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["TestOrcFile.test1.orc", "decimal.orc", "nulls-at-end-snappy.orc",
                                  "complextypes_iceberg.orc", "orc_index_int_string.orc",
                                  "TestOrcFile.testSnappy.orc", "decimal64_v2.orc"])
def test_row_reader_adapter_matches_pyarrow(name):
    """orc::Reader / RowReader::next(ColumnVectorBatch&) through the C++
    adapter (GpuRowReader.hh) against pyarrow, row by row."""
    import json

    po = pytest.importorskip("pyarrow.orc")
    import orc_amd
    from file_parity import path

    exe = build_reader_test()
    r = subprocess.run([exe, path(name)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    meta = orc_amd.Reader(path(name))
    root = meta.types[0]
    got = [json.loads(line) for line in r.stdout.splitlines() if line.strip()]
    want = po.ORCFile(path(name)).read().to_pylist()
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        for fname, st in zip(root.field_names, root.subtypes):
            assert _canon_json(g[fname], st, meta) == _canon(w[fname]), (name, i, fname, g[fname], w[fname])
