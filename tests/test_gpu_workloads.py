"""GPU parity at the file-level configurations (BASELINE.json configs[3] and
configs[4]) at a size the checker reads in seconds: every stripe and every
column decoded by the HIP path compared with pyarrow's ORC reader (Apache
ORC C++, the file-level checker), column by column with numpy.

  configs[3]: TPC-H lineitem-like 16 columns (sorted orderkey DELTA /
      SHORT_REPEAT runs, Decimal64 decimal(15,2) columns, dates, dictionary
      and direct strings), zstd, row index on, >= 3 stripes.
      Reference readers: IntegerColumnReader / Decimal64ColumnReader /
      StringDictionaryColumnReader / StringDirectColumnReader
      (c++/src/ColumnReader.cc:224-258, :1384-1527, :509-607, :615-793).
  configs[2]: demo-12's schema tiled to ~7.7 M rows (4 tiles of its 1.92 M),
      zlib, 4 MB stripes (>= 3 stripes): DELTA / DIRECT / SHORT_REPEAT
      integer streams and DICTIONARY_V2 strings, every stripe compared
      (TestMatch.cc:262-275 reads demo-12 whole).
  configs[4]: struct<a:list<int>, m:map<string,int>> with 10 % nulls at every
      level, zstd, row index on, >= 3 stripes. Reference readers:
      StructColumnReader / ListColumnReader / MapColumnReader
      (c++/src/ColumnReader.cc:795-1157).
"""
import os

import pytest

import orc_amd
from file_parity import compare_stripe
from workload_files import make_c3, make_c4, make_c5

pytestmark = pytest.mark.gpu

ROWS = 2_000_000
C3_ROWS = 4 * 1_920_800  # make_c3 tiles demo-12's 1,920,800 rows


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    pytest.importorskip("pyarrow.orc")
    d = tmp_path_factory.mktemp("workloads")
    out = {}
    for name, maker in (("c4", make_c4), ("c5", make_c5)):
        p = os.path.join(str(d), name + ".orc")
        maker(p, ROWS, 8)
        out[name] = p
    p = os.path.join(str(d), "c3.orc")
    make_c3(p, C3_ROWS, 4)
    out["c3"] = p
    return out


@pytest.fixture(scope="module")
def ctx():
    return orc_amd.Context(0)


@pytest.mark.parametrize("name", ["c3", "c4", "c5"])
def test_workload_every_stripe_matches_pyarrow(ctx, files, name):
    import pyarrow.orc as po

    path = files[name]
    r = orc_amd.Reader(path, ctx)
    f = po.ORCFile(path)
    assert r.num_rows == (C3_ROWS if name == "c3" else ROWS) and r.num_stripes >= 3, (r.num_rows, r.num_stripes)
    for s in range(r.num_stripes):
        b = r.read_stripe(s)
        compare_stripe(r, b, f.read_stripe(s), "%s stripe %d" % (name, s))
    # the row index cut the streams (no host header walk)
    assert r.last_stream_stats()["row_index"] > 0


@pytest.mark.parametrize("name", ["c4", "c5"])
def test_workload_pipelined_read_matches_single_stripe_reads(ctx, files, name):
    """read_stripes (host prepares stripe i+1 while the GPU decodes stripe i)
    leaves every stripe resident and equal to the one-stripe reads."""
    import numpy as np

    r = orc_amd.Reader(files[name], ctx)
    r.read_stripes_device()
    r2 = orc_amd.Reader(files[name], ctx)
    for s in range(r.num_stripes):
        one = r2.read_stripe(s)
        for tid, col in one.columns.items():
            v = r.stripe_column_view(s, tid)
            assert v.decoded and v.num_elements == col.num_elements
            if col.data is not None and r.types[tid].kind not in (5, 6):
                got = r._host(v.data, col.data.nbytes, col.data.dtype)
                if col.not_null is not None:
                    m = col.not_null.astype(bool)
                    if col.data.size == m.size:
                        np.testing.assert_array_equal(got[m], col.data[m])
                else:
                    np.testing.assert_array_equal(got, col.data)


@pytest.mark.parametrize("name", ["c4", "c5"])
def test_workload_stream_batching(ctx, files, name):
    """A stripe's host-countable RLEv2 streams go through multi-stream
    launches (one per kernel instance); the per-stream path (batching off)
    decodes the same file to the same values."""
    import pyarrow.orc as po

    path = files[name]
    f = po.ORCFile(path)
    on = orc_amd.Reader(path, ctx)
    off = orc_amd.Reader(path, ctx)
    off.set_stream_batching(False)
    last = on.num_stripes - 1
    for s in (0, last):
        compare_stripe(on, on.read_stripe(s), f.read_stripe(s), "%s stripe %d (batched)" % (name, s))
        # c5: every column under the root has a PRESENT stream (its value
        # counts come from the device), so only the map keys' dictionary
        # LENGTH stream is batched (its count is the footer's dictionary size)
        if name == "c4":
            assert on.last_stream_stats()["batched"] > 0
        else:
            assert on.last_stream_stats()["batched"] == 1
        compare_stripe(off, off.read_stripe(s), f.read_stripe(s), "%s stripe %d (per stream)" % (name, s))
        assert off.last_stream_stats()["batched"] == 0
    if name == "c4":
        # every integer / length / dictionary stream of the flat schema
        on.read_stripes_device(0, 1)
        assert on.last_stream_stats()["batched"] >= 12


def test_nested_dictionary_lazy_matches_eager(ctx, files):
    """configs[4]'s map keys: a dictionary under a nullable struct and a map,
    whose LENGTH stream and entry offsets ride the stripe's batch while the
    keys themselves wait for the map's element count. The lazy row reader
    (nextEncoded: index + dictionary) resolves to the eager strings."""
    r1 = orc_amd.Reader(files["c5"], ctx)
    r2 = orc_amd.Reader(files["c5"], ctx)
    a = r1.create_row_reader()
    e = r2.create_row_reader(lazy_dictionary=True)
    ba, be = a.create_row_batch(3000), e.create_row_batch(3000)
    for _ in range(3):
        assert a.next(ba) and e.next(be) and be.num_elements == ba.num_elements
        assert any(c.index is not None and c.data is None for c in be.columns.values())
        assert ba.to_pylist() == be.to_pylist()
