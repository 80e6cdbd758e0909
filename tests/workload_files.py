"""ORC files for the file-level configurations (BASELINE.json configs[2..4]),
written with pyarrow (Apache ORC C++ writer): shared by the parity tests
(tests/test_gpu_workloads.py, every stripe and column against pyarrow) and
the file benchmarks (scripts/bench_file.py).

  make_c3  demo-12-zlib schema, the example's 1,920,800 rows tiled (_col0
           offset per tile), zlib, dictionary strings.
  make_c4  TPC-H lineitem-like, 16 columns: sorted orderkey with 1-7 repeats
           (DELTA / SHORT_REPEAT runs), uniform part/suppkey, linenumber,
           quantity / extendedprice / discount / tax as decimal(15,2),
           ship / commit / receipt dates, returnflag / linestatus /
           shipinstruct / shipmode dictionaries, direct comment strings; zstd.
  make_c5  struct<a:list<int>, m:map<string,int>> with 10 % nulls at every
           level (struct, list, list elements, map, map values), list / map
           lengths U[0, 8], 16 dictionary map keys; zstd.
Every writer takes `row_index_stride` (10,000 by default, the reference
writer's) and `stripe_mb` (pyarrow's stripe size target).
"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO12 = os.path.join(ROOT, "tests", "golden", "files", "demo-12-zlib.orc")


def make_c3(path, rows, stripe_mb, row_index_stride=10000):
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.orc as po

    base = po.ORCFile(DEMO12).read()
    n0 = base.num_rows
    tiles = max(1, rows // n0)
    parts = []
    for t in range(tiles):
        cols = []
        for name in base.column_names:
            c = base.column(name)
            if name == "_col0":
                c = pc.add(c, pa.scalar(t * n0, pa.int32()))
            cols.append(c)
        parts.append(pa.table(cols, names=base.column_names))
    table = pa.concat_tables(parts)
    po.write_table(table, path, compression="zlib", stripe_size=stripe_mb << 20,
                   dictionary_key_size_threshold=1.0, row_index_stride=row_index_stride)


def _decimal(pa, cents, precision, scale):
    """decimal128(precision, scale) array of the int64 unscaled values."""
    v = np.ascontiguousarray(cents, dtype=np.int64)
    buf = np.empty((v.size, 2), dtype=np.int64)
    buf[:, 0] = v
    buf[:, 1] = v >> 63
    return pa.Array.from_buffers(pa.decimal128(precision, scale), v.size, [None, pa.py_buffer(buf.tobytes())])


def _dict_strings(pa, rng, words, n):
    idx = pa.array(rng.integers(0, len(words), size=n).astype(np.int32))
    return pa.DictionaryArray.from_arrays(idx, pa.array(words)).cast(pa.string())


def make_c4(path, rows, stripe_mb, row_index_stride=10000, compression="zstd"):
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.orc as po

    rng = np.random.default_rng(4)
    reps = rng.integers(1, 8, size=rows // 2 + 8)
    reps = reps[: np.searchsorted(np.cumsum(reps), rows) + 1]
    okey = np.repeat(np.arange(1, reps.size + 1, dtype=np.int64) * 4, reps)[:rows]
    line = (np.arange(okey.size) - np.repeat(np.cumsum(reps) - reps, reps)[:rows] + 1).astype(np.int32)
    qty = rng.integers(1, 51, size=rows)
    price = qty * rng.integers(90_000, 210_000, size=rows) // 100
    ship = rng.integers(8036, 10561, size=rows).astype(np.int32)  # 1992-01-02 .. 1998-12-01
    pool = pa.array(["".join(chr(97 + c) for c in rng.integers(0, 26, size=int(rng.integers(5, 22))))
                     for _ in range(4096)])
    i1 = rng.integers(0, 4096, size=rows)
    i2 = rng.integers(0, 4096, size=rows)
    # l_comment in chunks of 8M rows: an Arrow string array holds < 2 GiB
    # (configs[3]'s 1.25 * 10^8 rows per GPU make ~3.4 GB of comments)
    step = 1 << 23
    comment = pa.chunked_array([pc.binary_join_element_wise(pc.take(pool, pa.array(i1[a:a + step])),
                                                            pc.take(pool, pa.array(i2[a:a + step])), " ")
                                for a in range(0, rows, step)], type=pa.string())
    table = pa.table({
        "l_orderkey": pa.array(okey),
        "l_partkey": pa.array(rng.integers(1, 20_000_001, size=rows)),
        "l_suppkey": pa.array(rng.integers(1, 1_000_001, size=rows)),
        "l_linenumber": pa.array(line),
        "l_quantity": _decimal(pa, qty * 100, 15, 2),
        "l_extendedprice": _decimal(pa, price, 15, 2),
        "l_discount": _decimal(pa, rng.integers(0, 11, size=rows), 15, 2),
        "l_tax": _decimal(pa, rng.integers(0, 9, size=rows), 15, 2),
        "l_returnflag": _dict_strings(pa, rng, ["A", "N", "R"], rows),
        "l_linestatus": _dict_strings(pa, rng, ["O", "F"], rows),
        "l_shipdate": pa.array(ship, type=pa.date32()),
        "l_commitdate": pa.array(ship + rng.integers(-60, 60, size=rows).astype(np.int32), type=pa.date32()),
        "l_receiptdate": pa.array(ship + rng.integers(1, 31, size=rows).astype(np.int32), type=pa.date32()),
        "l_shipinstruct": _dict_strings(pa, rng, ["DELIVER IN PERSON", "COLLECT COD", "NONE",
                                                  "TAKE BACK RETURN"], rows),
        "l_shipmode": _dict_strings(pa, rng, ["REG AIR", "AIR", "RAIL", "SHIP", "TRUCK", "MAIL", "FOB"], rows),
        "l_comment": comment,
    })
    po.write_table(table, path, compression=compression, stripe_size=stripe_mb << 20,
                   dictionary_key_size_threshold=0.5, row_index_stride=row_index_stride)


def make_c5(path, rows, stripe_mb, row_index_stride=10000, compression="zstd"):
    import pyarrow as pa
    import pyarrow.orc as po

    rng = np.random.default_rng(5)

    def lengths(n):
        ln = rng.integers(0, 9, size=n)
        null = rng.random(n) < 0.1
        ln[null] = 0
        off = np.concatenate([[0], np.cumsum(ln)]).astype(np.int32)
        return off, null

    off_a, null_a = lengths(rows)
    na = int(off_a[-1])
    vals = pa.array(rng.integers(-(1 << 31), 1 << 31, size=na).astype(np.int32), mask=rng.random(na) < 0.1)
    a = pa.ListArray.from_arrays(pa.array(off_a), vals, mask=pa.array(null_a))
    off_m, null_m = lengths(rows)
    nm = int(off_m[-1])
    keys = pa.DictionaryArray.from_arrays(pa.array(rng.integers(0, 16, size=nm).astype(np.int32)),
                                          pa.array(["key%02d" % i for i in range(16)])).cast(pa.string())
    items = pa.array(rng.integers(0, 1 << 20, size=nm).astype(np.int32), mask=rng.random(nm) < 0.1)
    m = pa.MapArray.from_arrays(pa.array(off_m), keys, items, mask=pa.array(null_m))
    s = pa.StructArray.from_arrays([a, m], names=["a", "m"], mask=pa.array(rng.random(rows) < 0.1))
    po.write_table(pa.table({"s": s}), path, compression=compression, stripe_size=stripe_mb << 20,
                   dictionary_key_size_threshold=1.0, row_index_stride=row_index_stride)
