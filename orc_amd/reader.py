"""File-level reader over include/orcg_reader.h.

Mirrors the reference's reader surface for the decode path
(c++/include/orc/Reader.hh: createReader, getNumberOfRows,
getNumberOfStripes, getType, RowReader::next) with one stripe per read:
the host parses the tail and stripe footers and decompresses, the GPU decodes
every selected column into device batches (LongVectorBatch / DoubleVectorBatch
/ StringVectorBatch / ListVectorBatch / MapVectorBatch / StructVectorBatch
layouts, c++/include/orc/Vector.hh:46-330). `Batch.to_pylist()` renders rows
the way the reference's ColumnPrinter / pyarrow's to_pylist do, for parity
tests.
"""
import ctypes
import datetime
import decimal

import numpy as np

from . import _lib
from ._lib import check
from .rle import Context, default_context

BOOLEAN, BYTE, SHORT, INT, LONG, FLOAT, DOUBLE, STRING, BINARY, TIMESTAMP, LIST, MAP, STRUCT, UNION, \
    DECIMAL, DATE, VARCHAR, CHAR, TIMESTAMP_INSTANT = range(19)
KIND_NAMES = ["boolean", "tinyint", "smallint", "int", "bigint", "float", "double", "string", "binary",
              "timestamp", "array", "map", "struct", "uniontype", "decimal", "date", "varchar", "char",
              "timestamp with local time zone"]
COMPRESSION_NAMES = ["NONE", "ZLIB", "SNAPPY", "LZO", "LZ4", "ZSTD"]
SUPPORTED = {BOOLEAN, BYTE, SHORT, INT, LONG, FLOAT, DOUBLE, STRING, BINARY, LIST, MAP, STRUCT, DATE, VARCHAR,
             CHAR}
_EPOCH = datetime.date(1970, 1, 1)


class Type:
    """orc::Type (c++/include/orc/Type.hh): id, kind, children, field names."""

    def __init__(self, tid, kind, subtypes, field_names, maximum_length, precision, scale):
        self.id = tid
        self.kind = kind
        self.subtypes = subtypes
        self.field_names = field_names
        self.maximum_length = maximum_length
        self.precision = precision
        self.scale = scale

    def __repr__(self):
        return "Type(%d, %s)" % (self.id, KIND_NAMES[self.kind])


class ColumnBatch:
    """Host copy of one column's device batch."""

    def __init__(self, kind, n, not_null, data, length, offsets, blob, encoding, secondary=None):
        self.kind = kind
        self.secondary = secondary  # np.int64[n] TIMESTAMP nanoseconds
        self.num_elements = n
        self.not_null = not_null  # np.uint8[n] or None
        self.data = data          # np.int64 / np.float64 [n] (string starts for string kinds)
        self.length = length      # np.int64[n] for string kinds
        self.offsets = offsets    # np.int64[n + 1] for list / map
        self.blob = blob          # bytes for string kinds
        self.encoding = encoding


class Batch:
    """One stripe of decoded columns, keyed by type id."""

    def __init__(self, reader, columns):
        self.reader = reader
        self.columns = columns

    @property
    def num_rows(self):
        return self.columns[0].num_elements

    def value(self, tid, i):
        t = self.reader.types[tid]
        c = self.columns.get(tid)
        if c is None:
            raise KeyError("column %d (%s) was not decoded" % (tid, KIND_NAMES[t.kind]))
        if c.not_null is not None and not c.not_null[i]:
            return None
        k = t.kind
        if k == BOOLEAN:
            return bool(c.data[i])
        if k in (BYTE, SHORT, INT, LONG):
            return int(c.data[i])
        if k == DATE:
            return _EPOCH + datetime.timedelta(days=int(c.data[i]))
        if k in (FLOAT, DOUBLE):
            return float(c.data[i])
        if k == DECIMAL:
            # Decimal64VectorBatch int64 / Decimal128VectorBatch [hi, lo]
            if t.precision > 18:
                hi, lo = int(c.data[2 * i]), int(c.data[2 * i + 1]) & ((1 << 64) - 1)
                u = (hi << 64) | lo
            else:
                u = int(c.data[i])
            return decimal.Decimal(u).scaleb(-t.scale)
        if k in (TIMESTAMP, TIMESTAMP_INSTANT):
            # TimestampVectorBatch seconds + nanoseconds, as numpy datetime64[ns]
            return np.datetime64(int(c.data[i]) * 1_000_000_000 + int(c.secondary[i]), "ns")
        if k in (STRING, VARCHAR, CHAR, BINARY):
            s, ln = int(c.data[i]), int(c.length[i])
            raw = c.blob[s:s + ln]
            return raw if k == BINARY else raw.decode("utf-8", errors="replace")
        if k == LIST:
            a, b = int(c.offsets[i]), int(c.offsets[i + 1])
            return [self.value(t.subtypes[0], j) for j in range(a, b)]
        if k == MAP:
            a, b = int(c.offsets[i]), int(c.offsets[i + 1])
            return [(self.value(t.subtypes[0], j), self.value(t.subtypes[1], j)) for j in range(a, b)]
        if k == STRUCT:
            return {name: self.value(st, i) for name, st in zip(t.field_names, t.subtypes)}
        raise KeyError("type %s not decoded" % KIND_NAMES[k])

    def to_pylist(self, fields=None):
        """Rows of the root struct as dicts (pyarrow Table.to_pylist shape)."""
        root = self.reader.types[0]
        names = [n for n in root.field_names if fields is None or n in fields]
        ids = {n: st for n, st in zip(root.field_names, root.subtypes)}
        return [{n: self.value(ids[n], i) for n in names} for i in range(self.num_rows)]


class Reader:
    """orc::Reader over liborcgpu (include/orcg_reader.h)."""

    def __init__(self, source, ctx=None):
        self._L = _lib.load()
        self._ctx = ctx
        h = ctypes.c_void_p()
        ch = ctx.handle if ctx is not None else None
        if isinstance(source, (bytes, bytearray, memoryview)):
            self._buf = np.frombuffer(bytes(source), dtype=np.uint8)
            rc = self._L.orcg_reader_open(ch, self._buf.ctypes.data_as(ctypes.c_void_p), self._buf.size,
                                          ctypes.byref(h))
        else:
            self._buf = None
            rc = self._L.orcg_reader_open_file(ch, str(source).encode(), ctypes.byref(h))
        if rc:
            msg = self._L.orcg_reader_open_error()
            check(rc, lambda: msg)
        self._h = h
        self.types = [self._type(i) for i in range(self._L.orcg_reader_num_types(h))]

    def _type(self, i):
        ti = _lib.TypeInfo()
        check(self._L.orcg_reader_type(self._h, i, ctypes.byref(ti)))
        subs = (ctypes.c_uint32 * max(ti.num_subtypes, 1))()
        check(self._L.orcg_reader_subtypes(self._h, i, subs, ti.num_subtypes))
        names = []
        for j in range(ti.num_subtypes):
            nm = self._L.orcg_reader_field_name(self._h, i, j)
            if nm is not None:
                names.append(nm.decode())
        return Type(i, ti.kind, list(subs[:ti.num_subtypes]), names, ti.maximum_length, ti.precision, ti.scale)

    def close(self):
        if getattr(self, "_h", None):
            self._L.orcg_reader_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _err(self):
        return self._L.orcg_reader_last_error(self._h)

    @property
    def num_rows(self):
        return self._L.orcg_reader_num_rows(self._h)

    @property
    def num_stripes(self):
        return self._L.orcg_reader_num_stripes(self._h)

    @property
    def row_index_stride(self):
        return self._L.orcg_reader_row_index_stride(self._h)

    @property
    def compression(self):
        return COMPRESSION_NAMES[self._L.orcg_reader_compression(self._h)]

    @property
    def compression_block_size(self):
        return self._L.orcg_reader_compression_block_size(self._h)

    @property
    def format_version(self):
        a, b = ctypes.c_uint32(), ctypes.c_uint32()
        check(self._L.orcg_reader_format_version(self._h, ctypes.byref(a), ctypes.byref(b)))
        return "%d.%d" % (a.value, b.value)

    def stripe(self, i):
        si = _lib.StripeInfo()
        check(self._L.orcg_reader_stripe(self._h, i, ctypes.byref(si)), self._err)
        return {"offset": si.offset, "index_length": si.index_length, "data_length": si.data_length,
                "footer_length": si.footer_length, "num_rows": si.num_rows}

    def type_string(self, tid=0):
        """orc::Type::toString (c++/src/TypeImpl.cc)."""
        t = self.types[tid]
        k = t.kind
        if k == STRUCT:
            return "struct<%s>" % ",".join("%s:%s" % (n, self.type_string(s)) for n, s in zip(t.field_names, t.subtypes))
        if k == LIST:
            return "array<%s>" % self.type_string(t.subtypes[0])
        if k == MAP:
            return "map<%s,%s>" % (self.type_string(t.subtypes[0]), self.type_string(t.subtypes[1]))
        if k == UNION:
            return "uniontype<%s>" % ",".join(self.type_string(s) for s in t.subtypes)
        if k == DECIMAL:
            return "decimal(%d,%d)" % (t.precision, t.scale)
        if k in (VARCHAR, CHAR):
            return "%s(%d)" % (KIND_NAMES[k], t.maximum_length)
        return KIND_NAMES[k]

    def select(self, type_ids=None):
        """RowReaderOptions::include by type id (None = every column)."""
        if type_ids is None:
            check(self._L.orcg_reader_select(self._h, None, 0), self._err)
            return
        inc = np.zeros(len(self.types), dtype=np.uint8)
        inc[list(type_ids)] = 1
        check(self._L.orcg_reader_select(self._h, inc.ctypes.data_as(ctypes.c_void_p), inc.size), self._err)

    def _host(self, ptr, nbytes, dtype):
        out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype=dtype)
        if nbytes:
            check(self._L.orcg_reader_copy_to_host(self._h, out.ctypes.data_as(ctypes.c_void_p), ptr, nbytes),
                  self._err)
        return out

    def read_stripe_device(self, i):
        """Decode stripe i on the GPU; the batches stay in HBM (column_view)."""
        if self._ctx is None:
            raise _lib.InvalidArgument("reader was opened without a device context")
        check(self._L.orcg_reader_read_stripe(self._h, i), self._err)

    def read_stripes_device(self, first=0, count=None):
        """Decode stripes [first, first + count) into HBM with the host
        decompressing stripe i + 1 while the GPU decodes stripe i; every
        stripe's batches stay resident (stripe_column_view)."""
        if self._ctx is None:
            raise _lib.InvalidArgument("reader was opened without a device context")
        if count is None:
            count = self.num_stripes - first
        check(self._L.orcg_reader_read_stripes(self._h, first, count), self._err)

    def column_view(self, tid):
        v = _lib.ColumnView()
        check(self._L.orcg_reader_column(self._h, tid, ctypes.byref(v)), self._err)
        return v

    def stripe_column_view(self, k, tid):
        v = _lib.ColumnView()
        check(self._L.orcg_reader_stripe_column(self._h, k, tid, ctypes.byref(v)), self._err)
        return v

    def read_stripe(self, i):
        """Decode stripe i on the GPU and copy the selected columns to host."""
        self.read_stripe_device(i)
        cols = {}
        for t in self.types:
            v = _lib.ColumnView()
            if self._L.orcg_reader_column(self._h, t.id, ctypes.byref(v)) != 0 or not v.decoded:
                continue
            n = v.num_elements
            nn = self._host(v.not_null, n, np.uint8) if v.has_nulls else None
            data = length = offsets = None
            blob = b""
            k = t.kind
            if k in (FLOAT, DOUBLE):
                data = self._host(v.data, 8 * n, np.float64)
            elif k in (BOOLEAN, BYTE, SHORT, INT, LONG, DATE):
                data = self._host(v.data, 8 * n, np.int64)
            elif k in (STRING, VARCHAR, CHAR, BINARY):
                data = self._host(v.data, 8 * n, np.int64)
                length = self._host(v.length, 8 * n, np.int64)
                blob = self._host(v.blob, v.blob_len, np.uint8).tobytes()
            elif k in (LIST, MAP):
                offsets = self._host(v.offsets, 8 * (n + 1), np.int64)
            secondary = None
            if k == DECIMAL:
                data = self._host(v.data, (16 if t.precision > 18 else 8) * n, np.int64)
            elif k in (TIMESTAMP, TIMESTAMP_INSTANT):
                data = self._host(v.data, 8 * n, np.int64)
                secondary = self._host(v.secondary, 8 * n, np.int64)
            cols[t.id] = ColumnBatch(k, n, nn, data, length, offsets, blob, v.encoding, secondary)
        return Batch(self, cols)

    def last_timings(self):
        t = (ctypes.c_double * 5)()
        check(self._L.orcg_reader_last_timings(self._h, t))
        return {"host_parse_s": t[0], "host_decompress_s": t[1], "host_plan_s": t[2], "h2d_s": t[3],
                "device_decode_s": t[4]}

    def last_stream_stats(self):
        """RLE streams of the last read cut by the row index / by host plans."""
        t = (ctypes.c_uint64 * 2)()
        check(self._L.orcg_reader_last_stream_stats(self._h, t))
        return {"row_index": t[0], "host_plan": t[1]}

    def read(self, fields=None):
        """All rows as dicts of the root struct's fields (pyarrow to_pylist shape)."""
        rows = []
        for s in range(self.num_stripes):
            rows.extend(self.read_stripe(s).to_pylist(fields))
        return rows


def open_reader(source, ctx=None, device=True):
    """createReader: `device=False` opens for metadata only (no GPU)."""
    if device and ctx is None:
        ctx = default_context()
    return Reader(source, ctx)


__all__ = ["Reader", "Batch", "ColumnBatch", "Type", "open_reader", "Context"]
