"""File-level reader over include/orcg_reader.h.

Mirrors the reference's reader surface for the decode path
(c++/include/orc/Reader.hh: createReader, getNumberOfRows,
getNumberOfStripes, getType, getContentLength, getSoftwareVersion,
getMetadataKeys / getMetadataValue; RowReader createRowBatch(capacity),
next(batch), getRowNumber, seekToRow; RowReaderOptions include / range /
setEnableLazyDecoding): the host parses the tail and stripe footers and
decompresses, the GPU decodes every selected column of a stripe into device
batches (LongVectorBatch / DoubleVectorBatch / StringVectorBatch /
EncodedStringVectorBatch / ListVectorBatch / MapVectorBatch /
StructVectorBatch / UnionVectorBatch layouts, c++/include/orc/Vector.hh:
46-352), and RowReader batches are row ranges of that stripe copied to host.
`Batch.to_pylist()` renders rows the way the reference's ColumnPrinter /
pyarrow's to_pylist do, for parity tests.
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
             CHAR, UNION}
STRING_KINDS = (STRING, VARCHAR, CHAR, BINARY)
_EPOCH = datetime.date(1970, 1, 1)


class UnionValue(tuple):
    """One UNION row: (tag, value) — UnionVectorBatch tags / offsets resolved."""

    __slots__ = ()

    def __new__(cls, tag, value):
        return tuple.__new__(cls, (tag, value))

    @property
    def tag(self):
        return self[0]

    @property
    def value(self):
        return self[1]


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

    def __init__(self, kind, n, not_null, data, length, offsets, blob, encoding, secondary=None, tags=None,
                 index=None, dict_offsets=None, scale=None):
        self.kind = kind
        self.scale = scale          # DECIMAL: the scale the values were decoded at
        self.secondary = secondary  # np.int64[n] TIMESTAMP nanoseconds
        self.num_elements = n
        self.not_null = not_null  # np.uint8[n] or None
        self.data = data          # np.int64 / np.float64 [n] (string starts for string kinds)
        self.length = length      # np.int64[n] for string kinds
        self.offsets = offsets    # np.int64[n + 1] for list / map; np.int64[n] child offsets for union
        self.blob = blob          # bytes for string kinds
        self.encoding = encoding
        self.tags = tags          # np.uint8[n] UNION child per row
        self.index = index        # np.int64[n] dictionary entry per row (EncodedStringVectorBatch::index)
        self.dict_offsets = dict_offsets  # np.int64[dict_size + 1] into blob (StringDictionary)


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
            # (Hive 0.11 precision-0 decimals: Decimal128 at the forced scale)
            if t.precision > 18 or t.precision == 0:
                hi, lo = int(c.data[2 * i]), int(c.data[2 * i + 1]) & ((1 << 64) - 1)
                u = (hi << 64) | lo
            else:
                u = int(c.data[i])
            return decimal.Decimal(u).scaleb(-(c.scale if c.scale is not None else t.scale))
        if k in (TIMESTAMP, TIMESTAMP_INSTANT):
            # TimestampVectorBatch seconds + nanoseconds, as numpy datetime64[ns]
            return np.datetime64(int(c.data[i]) * 1_000_000_000 + int(c.secondary[i]), "ns")
        if k in STRING_KINDS:
            if c.data is None:  # lazy dictionary: index + dictionary
                e = int(c.index[i])
                s, ln = int(c.dict_offsets[e]), int(c.dict_offsets[e + 1] - c.dict_offsets[e])
            else:
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
        if k == UNION:
            tag = int(c.tags[i])
            return UnionValue(tag, self.value(t.subtypes[tag], int(c.offsets[i])))
        raise KeyError("type %s not decoded" % KIND_NAMES[k])

    def to_pylist(self, fields=None):
        """Rows of the root struct as dicts (pyarrow Table.to_pylist shape);
        a non-struct root gives its values."""
        root = self.reader.types[0]
        if root.kind != STRUCT:
            return [self.value(0, i) for i in range(self.num_rows)]
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

    def _host(self, ptr, nbytes, dtype, from_host=False):
        """Copy `nbytes` at `ptr` (device memory, or with from_host a row
        reader's pinned host slab) into a new array."""
        out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype=dtype)
        if nbytes:
            if from_host:
                ctypes.memmove(out.ctypes.data, ptr, nbytes)
            else:
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

    def _column(self, v, t, begin=0, count=None, from_host=False, dict_cache=None, lookup=False):
        """Host copy of elements [begin, begin + count) of a column view (the
        whole column by default; device pointers, or with from_host a row
        reader's host slab): offsets rebased to 0 (the reference's batch
        layout), string starts relative to the copied blob (the dictionary,
        or the span of direct strings the range covers). dict_cache (a dict)
        keeps a dictionary's host copy for the next batches of the stripe.
        lookup: a dictionary column given as entries only (a row reader's
        slab) gets its starts and lengths from the dictionary, as
        StringDictionaryColumnReader::next does (ColumnReader.cc:561-594)."""
        n = v.num_elements if count is None else count
        k = t.kind

        def host(ptr, itemsize, dtype, cnt, first=begin):
            if not ptr or cnt <= 0:
                return np.zeros(max(cnt, 0), dtype=dtype)
            return self._host(ptr + first * itemsize, cnt * itemsize, dtype, from_host)

        nn = host(v.not_null, 1, np.uint8, n) if v.has_nulls else None
        data = length = offsets = tags = index = dict_offsets = secondary = None
        blob = b""
        if k in (FLOAT, DOUBLE):
            data = host(v.data, 8, np.float64, n)
        elif k in (BOOLEAN, BYTE, SHORT, INT, LONG, DATE):
            data = host(v.data, 8, np.int64, n)
        elif k in STRING_KINDS:
            key = (t.id, v.dict_offsets, v.blob, v.dict_size, v.blob_len)
            cached = dict_cache.get(key) if dict_cache is not None and v.index else None
            if v.index:
                index = host(v.index, 8, np.int64, n)
                dict_offsets = cached[0] if cached else \
                    self._host(v.dict_offsets, 8 * (v.dict_size + 1), np.int64, from_host)
            if v.data:
                data = host(v.data, 8, np.int64, n)
                length = host(v.length, 8, np.int64, n)
            if v.index and v.dict_offsets:
                # the dictionary
                blob = cached[1] if cached else self._host(v.blob, v.blob_len, np.uint8, from_host).tobytes()
                if dict_cache is not None and not cached:
                    dict_cache[key] = (dict_offsets, blob)
                if lookup and data is None:
                    data = np.zeros(n, np.int64)
                    length = np.zeros(n, np.int64)
                    m = slice(None) if nn is None else nn != 0
                    e = index[m]
                    data[m] = dict_offsets[e]
                    length[m] = dict_offsets[e + 1] - dict_offsets[e]
            elif data is not None and n:
                live = length > 0
                lo = int(data[live].min()) if live.any() else 0
                hi = int((data + length)[live].max()) if live.any() else 0
                blob = host(v.blob, 1, np.uint8, hi - lo, first=lo).tobytes()
                data = np.where(live, data - lo, 0)
        elif k in (LIST, MAP):
            offsets = host(v.offsets, 8, np.int64, n + 1)
            offsets = offsets - offsets[0] if offsets.size else offsets
        elif k == UNION:
            tags = host(v.tags, 1, np.uint8, n)
            offsets = host(v.offsets, 8, np.int64, n)
        if k == DECIMAL:
            w = 16 if t.precision > 18 or t.precision == 0 else 8
            data = host(v.data, w, np.int64, n).reshape(-1) if w == 8 else \
                self._host(v.data + begin * 16, 16 * n, np.int64, from_host) if n else np.zeros(0, np.int64)
        elif k in (TIMESTAMP, TIMESTAMP_INSTANT):
            data = host(v.data, 8, np.int64, n)
            secondary = host(v.secondary, 8, np.int64, n)
        # Hive 0.11 decimals are decoded at the forced scale in effect now
        scale = (t.scale if t.precision else self.hive11_scale) if k == DECIMAL else None
        return ColumnBatch(k, n, nn, data, length, offsets, blob, v.encoding, secondary, tags, index, dict_offsets,
                           scale)

    def read_stripe(self, i):
        """Decode stripe i on the GPU and copy the selected columns to host."""
        self.read_stripe_device(i)
        cols = {}
        for t in self.types:
            v = _lib.ColumnView()
            if self._L.orcg_reader_column(self._h, t.id, ctypes.byref(v)) != 0 or not v.decoded:
                continue
            cols[t.id] = self._column(v, t)
        return Batch(self, cols)

    @property
    def content_length(self):
        """Reader::getContentLength (Footer.contentLength)."""
        return self._L.orcg_reader_content_length(self._h)

    @property
    def software_version(self):
        """Reader::getSoftwareVersion: writer id name [+ softwareVersion]."""
        return self._L.orcg_reader_software_version(self._h).decode()

    @property
    def metadata(self):
        """User metadata (Reader::getMetadataKeys / getMetadataValue) as bytes values."""
        out = {}
        for i in range(self._L.orcg_reader_num_metadata(self._h)):
            key = self._L.orcg_reader_metadata_key(self._h, i).decode()
            ln = ctypes.c_uint64()
            p = self._L.orcg_reader_metadata_value(self._h, i, ctypes.byref(ln))
            out[key] = ctypes.string_at(p, ln.value) if p and ln.value else b""
        return out

    def set_hive11_decimal(self, forced_scale=6, throw_on_overflow=True):
        """RowReaderOptions::forcedScaleOnHive11Decimal /
        throwOnHive11DecimalOverflow (c++/include/orc/Reader.hh:258-271):
        with throw_on_overflow=False a value past 38 digits reads as NULL."""
        check(self._L.orcg_reader_set_hive11_decimal(self._h, int(forced_scale), int(bool(throw_on_overflow))),
              self._err)

    @property
    def hive11_scale(self):
        return int(self._L.orcg_reader_hive11_scale(self._h))

    def set_lazy_dictionary(self, on=True):
        """RowReaderOptions::setEnableLazyDecoding for stripe reads."""
        check(self._L.orcg_reader_set_lazy_dictionary(self._h, int(bool(on))), self._err)

    def create_row_reader(self, include=None, offset=0, length=None, lazy_dictionary=False, tight_numeric=False):
        """Reader::createRowReader(RowReaderOptions): `include` type ids (or
        top-level field names), range(offset, length) in file bytes,
        setEnableLazyDecoding, setUseTightNumericVector."""
        return RowReader(self, include=include, offset=offset, length=length, lazy_dictionary=lazy_dictionary,
                         tight_numeric=tight_numeric)

    def last_timings(self):
        t = (ctypes.c_double * 5)()
        check(self._L.orcg_reader_last_timings(self._h, t))
        return {"host_parse_s": t[0], "host_decompress_s": t[1], "host_plan_s": t[2], "h2d_s": t[3],
                "device_decode_s": t[4]}

    def last_stream_stats(self):
        """RLE streams of the last read cut by the row index / by host plans."""
        t = (ctypes.c_uint64 * 2)()
        check(self._L.orcg_reader_last_stream_stats(self._h, t))
        return {"row_index": t[0], "host_plan": t[1],
                "batched": int(self._L.orcg_reader_last_batched_streams(self._h)),
                "stage_bytes": int(self._L.orcg_reader_last_stage_bytes(self._h))}

    METRIC_NAMES = ("ReaderCall", "ReaderInclusiveLatencyUs", "DecompressionCall", "DecompressionLatencyUs",
                    "DecodingCall", "DecodingLatencyUs", "ByteDecodingCall", "ByteDecodingLatencyUs", "IOCount",
                    "IOBlockingLatencyUs", "SelectedRowGroupCount", "EvaluatedRowGroupCount",
                    "ReadRangeCacheHits", "ReadRangeCacheMisses")

    def metrics(self, reset=False):
        """ReaderMetrics (c++/include/orc/Reader.hh:59-76) accumulated over the
        reader's life, keyed by the reference's member names
        (orcg_reader_get_metrics); reset=True zeroes them afterwards."""
        t = (ctypes.c_uint64 * len(self.METRIC_NAMES))()
        check(self._L.orcg_reader_get_metrics(self._h, t))
        if reset:
            check(self._L.orcg_reader_reset_metrics(self._h))
        return dict(zip(self.METRIC_NAMES, (int(x) for x in t)))

    def set_metrics_timing(self, on=True):
        """Time the integer-RLE and byte-RLE launches with HIP events
        (DecodingLatencyUs / ByteDecodingLatencyUs; the reference fills its
        metrics only when built with BUILD_CPP_ENABLE_METRICS)."""
        check(self._L.orcg_reader_set_metrics_timing(self._h, int(bool(on))), self._err)

    def set_stream_batching(self, on=True):
        """Decode a stripe's host-countable RLEv2 streams with one launch per
        kernel instance (default) or one launch per stream."""
        check(self._L.orcg_reader_set_stream_batching(self._h, int(bool(on))), self._err)

    def read(self, fields=None):
        """All rows as dicts of the root struct's fields (pyarrow to_pylist shape)."""
        rows = []
        for s in range(self.num_stripes):
            rows.extend(self.read_stripe(s).to_pylist(fields))
        return rows


# setUseTightNumericVector batch element types (c++/src/ColumnReader.cc:1703-1790,
# c++/src/TypeImpl.cc createRowBatch)
_TIGHT = {BOOLEAN: np.int8, BYTE: np.int8, SHORT: np.int16, INT: np.int32, FLOAT: np.float32}


class RowBatch(Batch):
    """A batch of at most `capacity` rows (RowReader::createRowBatch)."""

    def __init__(self, reader, capacity):
        super().__init__(reader, {})
        self.capacity = capacity
        self.num_elements = 0

    @property
    def num_rows(self):
        return self.num_elements


class RowReader:
    """orc::RowReader (c++/include/orc/Reader.hh:640-790) over the GPU stripe
    decode (include/orcg_reader.h orcg_row_reader_*): next(batch) fills at
    most batch.capacity rows and never crosses a stripe
    (RowReaderImpl::next, c++/src/Reader.cc:1392-1442); get_row_number /
    seek_to_row follow RowReaderImpl (:424-499); range(offset, length)
    selects the stripes whose offset falls in the byte range (:337-345)."""

    def __init__(self, reader, include=None, offset=0, length=None, lazy_dictionary=False, tight_numeric=False):
        if reader._ctx is None:
            raise _lib.InvalidArgument("reader was opened without a device context")
        self.reader = reader
        self._L = reader._L
        opts = _lib.RowReaderOptions()
        opts.offset = offset
        opts.length = (1 << 64) - 1 if length is None else length
        self._inc = None
        if include is not None:
            root = reader.types[0]
            ids = [root.subtypes[root.field_names.index(x)] if isinstance(x, str) else int(x) for x in include]
            self._inc = np.zeros(len(reader.types), dtype=np.uint8)
            self._inc[ids] = 1
            opts.include = self._inc.ctypes.data_as(ctypes.c_void_p)
            opts.include_len = self._inc.size
        opts.lazy_dictionary = int(bool(lazy_dictionary))
        h = ctypes.c_void_p()
        check(self._L.orcg_row_reader_create(reader._h, ctypes.byref(opts), ctypes.byref(h)), reader._err)
        self._h = h
        self.tight_numeric = tight_numeric
        self.lazy_dictionary = bool(lazy_dictionary)
        self._dicts = {}  # the current stripe's dictionaries (host copies)
        self._dict_stripe = None

    def _err(self):
        return self._L.orcg_row_reader_last_error(self._h)

    def is_selected(self, tid):
        """RowReader::getSelectedColumns()[tid]."""
        return bool(self._L.orcg_row_reader_is_selected(self._h, tid))

    def close(self):
        if getattr(self, "_h", None):
            self._L.orcg_row_reader_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def create_row_batch(self, capacity):
        return RowBatch(self.reader, int(capacity))

    def next(self, batch):
        """RowReader::next: True with batch.num_elements rows, False at the end."""
        rows = ctypes.c_uint64()
        check(self._L.orcg_row_reader_next(self._h, batch.capacity, ctypes.byref(rows)), self._err)
        batch.num_elements = rows.value
        batch.columns = {}
        if rows.value == 0:
            return False
        stripe = self._L.orcg_row_reader_stripe(self._h)
        if stripe != self._dict_stripe:
            self._dicts, self._dict_stripe = {}, stripe
        begins = {}
        for t in self.reader.types:
            v = _lib.ColumnView()
            b, c = ctypes.c_uint64(), ctypes.c_uint64()
            check(self._L.orcg_row_reader_column(self._h, t.id, ctypes.byref(v), ctypes.byref(b), ctypes.byref(c)),
                  self.reader._err)
            if v.decoded:
                col = self.reader._column(v, t, b.value, c.value, from_host=True, dict_cache=self._dicts,
                                          lookup=not self.lazy_dictionary)
                if self.tight_numeric and t.kind in _TIGHT:
                    # RowReaderOptions::setUseTightNumericVector: Byte / Short /
                    # Int / FloatVectorBatch (ColumnReader.cc:1703-1790)
                    col.data = col.data.astype(_TIGHT[t.kind])
                batch.columns[t.id] = col
                begins[t.id] = b.value
        # union offsets index the stripe's child rows: make them batch-relative
        for tid, col in batch.columns.items():
            t = self.reader.types[tid]
            if t.kind == UNION and col.num_elements:
                offs = col.offsets.copy()
                for k, st in enumerate(t.subtypes):
                    m = col.tags == k
                    offs[m] -= begins.get(st, 0)
                if col.not_null is not None:
                    offs[col.not_null == 0] = 0
                col.offsets = offs
        return True

    def get_row_number(self):
        """RowReader::getRowNumber: first row of the last batch."""
        return self._L.orcg_row_reader_row_number(self._h)

    def seek_to_row(self, row):
        """RowReader::seekToRow: the next batch starts at `row`."""
        check(self._L.orcg_row_reader_seek_to_row(self._h, int(row)), self._err)


def open_reader(source, ctx=None, device=True):
    """createReader: `device=False` opens for metadata only (no GPU)."""
    if device and ctx is None:
        ctx = default_context()
    return Reader(source, ctx)


__all__ = ["Reader", "RowReader", "RowBatch", "Batch", "ColumnBatch", "Type", "UnionValue", "open_reader", "Context"]
