"""Whole-stripe parity against pyarrow (the reference's C++ reader as pyarrow
bundles it) without Python row objects: a pyarrow RecordBatch of one stripe
(pyarrow.orc.ORCFile.read_stripe) is compared column by column with the GPU
reader's host batch (orc_amd.Reader.read_stripe) using numpy on the value
buffers, so multi-million-row stripes (configs[3] at 1.25 * 10^8 rows per
GPU) are checked in seconds. Validity, values, string bytes, list / map
offsets and children, struct fields; first difference reported as text.

Test / bench infrastructure only (the checker, never the thing measured)."""
import numpy as np

BOOLEAN, BYTE, SHORT, INT, LONG, FLOAT, DOUBLE, STRING, BINARY, TIMESTAMP, LIST, MAP, STRUCT, UNION, DECIMAL, DATE, \
    VARCHAR, CHAR, TIMESTAMP_INSTANT = range(19)
STRING_KINDS = (STRING, BINARY, VARCHAR, CHAR)


def _first(mask):
    return int(np.argmax(mask))


def _validity(arr):
    import pyarrow.compute as pc

    if arr.null_count == 0:
        return np.ones(len(arr), dtype=bool)
    return pc.is_valid(arr).to_numpy(zero_copy_only=False)


def _strings(arr):
    """(lengths int64[n], bytes of the valid rows in row order) of a pyarrow
    string / binary array."""
    import pyarrow as pa

    if pa.types.is_large_string(arr.type) or pa.types.is_large_binary(arr.type):
        otype = np.int64
    else:
        otype = np.int32
    bufs = arr.buffers()
    offs = np.frombuffer(bufs[1], dtype=otype)[arr.offset:arr.offset + len(arr) + 1].astype(np.int64)
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
    lens = np.diff(offs)
    return lens, data[offs[0]:offs[-1]], offs - offs[0]


def _gather_spans(blob, starts, lens):
    """Concatenation of blob[starts[i] : starts[i] + lens[i]]."""
    lens = lens.astype(np.int64)
    tot = int(lens.sum())
    if tot == 0:
        return np.zeros(0, np.uint8)
    out_off = np.concatenate([[0], np.cumsum(lens)[:-1]])
    idx = np.repeat(starts.astype(np.int64) - out_off, lens) + np.arange(tot, dtype=np.int64)
    return np.frombuffer(blob, dtype=np.uint8)[idx] if isinstance(blob, (bytes, bytearray)) else blob[idx]


def _cmp(arr, batch, reader, tid, path):
    import pyarrow as pa
    import pyarrow.compute as pc

    t = reader.types[tid]
    c = batch.columns.get(tid)
    if c is None:
        return "%s: column %d not decoded" % (path, tid)
    n = len(arr)
    if c.num_elements != n:
        return "%s: %d rows, pyarrow %d" % (path, c.num_elements, n)
    pv = _validity(arr)
    ov = c.not_null.astype(bool) if c.not_null is not None else np.ones(n, dtype=bool)
    if not np.array_equal(pv, ov):
        i = _first(pv != ov)
        return "%s row %d: valid %s, pyarrow %s" % (path, i, bool(ov[i]), bool(pv[i]))
    k = t.kind
    if k in (BOOLEAN, BYTE, SHORT, INT, LONG, DATE):
        a = arr.cast(pa.int32()) if k == DATE else (arr.cast(pa.int8()) if k == BOOLEAN else arr)
        want = pc.fill_null(a, 0).to_numpy(zero_copy_only=False).astype(np.int64)
        got = np.where(pv, c.data, 0)
        if not np.array_equal(np.where(pv, want, 0), got):
            i = _first(np.where(pv, want, 0) != got)
            return "%s row %d: %d, pyarrow %d" % (path, i, int(got[i]), int(want[i]))
        return None
    if k in (FLOAT, DOUBLE):
        want = pc.fill_null(arr.cast(pa.float64()), 0.0).to_numpy(zero_copy_only=False)
        got = np.where(pv, c.data, 0.0)
        want = np.where(pv, want, 0.0)
        if not np.array_equal(want, got, equal_nan=True):
            i = _first(~((want == got) | (np.isnan(want) & np.isnan(got))))
            return "%s row %d: %r, pyarrow %r" % (path, i, float(got[i]), float(want[i]))
        return None
    if k == DECIMAL:
        raw = np.frombuffer(arr.buffers()[1], dtype="<i8").reshape(-1, 2)[arr.offset:arr.offset + n]
        lo, hi = raw[:, 0], raw[:, 1]
        if t.precision > 18 or t.precision == 0:
            pairs = c.data.reshape(-1, 2)
            ghi, glo = pairs[:, 0], pairs[:, 1]
        else:
            glo = c.data
            ghi = np.where(c.data < 0, -1, 0)
        # pyarrow's decimals are at the type's scale (Hive 0.11: compare at ours)
        bad = pv & ((glo != lo) | (ghi != hi))
        if bad.any():
            i = _first(bad)
            return "%s row %d: (%d, %d), pyarrow (%d, %d)" % (path, i, int(ghi[i]), int(glo[i]), int(hi[i]), int(lo[i]))
        return None
    if k in STRING_KINDS:
        wl, wbytes, _ = _strings(arr)
        if c.index is not None and c.data is None:  # lazy dictionary
            starts = c.dict_offsets[c.index]
            lens = c.dict_offsets[c.index + 1] - starts
        else:
            starts, lens = c.data, c.length
        lens = np.where(pv, lens, 0)
        wl = np.where(pv, wl, 0)
        if not np.array_equal(lens, wl):
            i = _first(lens != wl)
            return "%s row %d: length %d, pyarrow %d" % (path, i, int(lens[i]), int(wl[i]))
        got = _gather_spans(c.blob, np.where(pv, starts, 0), lens)
        want = _gather_spans(wbytes, np.where(pv, (np.cumsum(wl) - wl), 0), wl)
        if not np.array_equal(got, want):
            j = _first(got != want)
            i = int(np.searchsorted(np.cumsum(lens), j, side="right"))
            return "%s row %d: string bytes differ" % (path, i)
        return None
    if k in (LIST, MAP):
        offs = np.frombuffer(arr.buffers()[1], dtype=np.int32)[arr.offset:arr.offset + n + 1].astype(np.int64)
        base = int(offs[0]) if offs.size else 0
        woff = offs - base
        if not np.array_equal(c.offsets, woff):
            i = _first(c.offsets != woff)
            return "%s offset %d: %d, pyarrow %d" % (path, i, int(c.offsets[i]), int(woff[i]))
        m = int(woff[-1]) if woff.size else 0
        if k == LIST:
            kids = [(arr.values.slice(base, m), t.subtypes[0], path + ".item")]
        else:
            kids = [(arr.keys.slice(base, m), t.subtypes[0], path + ".key"),
                    (arr.items.slice(base, m), t.subtypes[1], path + ".value")]
        for ka, kt, kp in kids:
            d = _cmp(ka, batch, reader, kt, kp)
            if d:
                return d
        return None
    if k == STRUCT:
        # flatten(): the fields with the struct's nulls merged in (the
        # reference's children of a null struct row are null too)
        fields = arr.flatten()
        for j, (name, st) in enumerate(zip(t.field_names, t.subtypes)):
            if st not in batch.columns:
                continue
            d = _cmp(fields[j], batch, reader, st, path + "." + name)
            if d:
                return d
        return None
    if k in (TIMESTAMP, TIMESTAMP_INSTANT):
        want = pc.fill_null(arr.cast(pa.int64()), 0).to_numpy(zero_copy_only=False)
        got = c.data * 1_000_000_000 + c.secondary
        bad = pv & (want != got)
        if bad.any():
            i = _first(bad)
            return "%s row %d: %d ns, pyarrow %d" % (path, i, int(got[i]), int(want[i]))
        return None
    return "%s: kind %d not compared" % (path, k)


def first_difference_arrow(pa_batch, batch, reader):
    """None when the GPU reader's host batch of a stripe equals pyarrow's
    RecordBatch of the same stripe, else the first difference."""
    root = reader.types[0]
    if batch.num_rows != pa_batch.num_rows:
        return "rows: %d, pyarrow %d" % (batch.num_rows, pa_batch.num_rows)
    for j, (name, st) in enumerate(zip(root.field_names, root.subtypes)):
        if st not in batch.columns:
            continue
        d = _cmp(pa_batch.column(j), batch, reader, st, name)
        if d:
            return d
    return None
