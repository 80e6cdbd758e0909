"""Host-side mirror of the reference's RLE decoder interface, backed by the
HIP decoder in liborcgpu (include/orcg.h).

Reference surface mirrored:
  * ``createRleDecoder(stream, isSigned, RleVersion, pool, metrics)``
    (c++/src/RLE.hh:163, c++/src/RLE.cc:48-60)  ->  :func:`create_rle_decoder`
  * ``RleDecoder::{seek, skip, next}`` (c++/src/RLE.hh:109-141)
    ->  :class:`RleDecoderV2`
  * Java ``IntegerReader.nextVector`` (java/core/.../RunLengthIntegerReaderV2.java:
    371-396)  ->  :meth:`RleDecoderV2.next_vector_java`
Errors are raised as :class:`ParseError` / :class:`InvalidArgument` with the
reference's messages.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import InvalidArgument, OrcError, ParseError, check  # noqa: F401

RleVersion_1 = 1
RleVersion_2 = 2


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


class Context:
    """One orcg_ctx: device scratch + a HIP stream (one per reader thread)."""

    def __init__(self, device=0, stream=None):
        self._L = _lib.load()
        n = self._L.orcg_device_count()
        if n <= device:
            raise _lib.DeviceError("no HIP device %d visible (orcg_device_count() = %d); the "
                                   "orc_amd decoder has no CPU fallback" % (device, n))
        h = ctypes.c_void_p()
        check(self._L.orcg_ctx_create(device, ctypes.byref(h)), lambda: b"orcg_ctx_create failed")
        self._h = h
        self.device = device
        if stream is not None:
            self.set_stream(stream)

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream):
        """stream: a raw hipStream_t (int) or a torch.cuda.Stream."""
        raw = getattr(stream, "cuda_stream", stream)
        check(self._L.orcg_ctx_set_stream(self._h, ctypes.c_void_p(raw)))

    def stream_ptr(self):
        """The context's hipStream_t (its own non-blocking stream, or the one
        set_stream gave it)."""
        return int(self._L.orcg_ctx_stream(self._h) or 0)

    def after_torch(self):
        """Order the context stream after torch's current stream: kernels
        launched next see every tensor op queued there (allocations, fills,
        copies). The *_device wrappers below call it; the context's own
        stream is non-blocking, so without it a kernel could overtake e.g.
        the torch.zeros fill of its output."""
        import torch

        cur = torch.cuda.current_stream(self.device)
        raw = self.stream_ptr()
        if raw == cur.cuda_stream:
            return
        ev = torch.cuda.Event()
        ev.record(cur)
        torch.cuda.ExternalStream(raw, device=self.device).wait_event(ev)

    def set_rlev2_variant(self, variant):
        """0 = tiled LDS kernel (default), 1 = one-wave-per-segment walk."""
        check(self._L.orcg_ctx_set_rlev2_variant(self._h, int(variant)))

    def synchronize(self):
        check(self._L.orcg_ctx_synchronize(self._h), self.last_error)

    def last_error(self):
        return self._L.orcg_ctx_last_error(self._h)

    def close(self):
        if getattr(self, "_h", None):
            self._L.orcg_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}


def default_context(device=0):
    ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = _default_ctx[device] = Context(device)
    return ctx


class RleDecoderV2:
    """Drop-in for orc::RleDecoderV2 over an uncompressed stream held in host
    memory: the whole stream is decoded on the GPU at construction and
    next()/skip()/seek() serve it with the reference's run-state semantics."""

    def __init__(self, data, is_signed, ctx=None, version=RleVersion_2, java=None):
        """java=None: the C++ reader's rules; java=False / True: Java's
        RunLengthIntegerReaderV2 with skipCorrupt off / on
        (orcg_rle_decoder_create_java)."""
        self._L = _lib.load()
        self.ctx = ctx or default_context()
        self._buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        h = ctypes.c_void_p()
        if java is None:
            rc = self._L.orcg_rle_decoder_create(self.ctx.handle, _ptr(self._buf), self._buf.size,
                                                int(bool(is_signed)), version, ctypes.byref(h))
        else:
            rc = self._L.orcg_rle_decoder_create_java(self.ctx.handle, _ptr(self._buf), self._buf.size,
                                                     int(bool(is_signed)), int(bool(java)), ctypes.byref(h))
        check(rc, self.ctx.last_error)
        self._h = h

    def _err(self):
        return self._L.orcg_rle_decoder_last_error(self._h)

    def next(self, n, not_null=None, dtype=np.int64, out=None):
        if out is None:
            out = np.zeros(n, dtype=dtype)
        nn = None if not_null is None else np.ascontiguousarray(not_null, dtype=np.uint8)
        fn = {8: self._L.orcg_rle_decoder_next_i64, 4: self._L.orcg_rle_decoder_next_i32,
              2: self._L.orcg_rle_decoder_next_i16}[out.dtype.itemsize]
        check(fn(self._h, _ptr(out), n, _ptr(nn)), self._err)
        return out

    def skip(self, n):
        check(self._L.orcg_rle_decoder_skip(self._h, n), self._err)

    def seek(self, *positions):
        """PositionProvider for an uncompressed stream: (byte offset, values to skip)."""
        p = np.asarray(positions, dtype=np.uint64)
        check(self._L.orcg_rle_decoder_seek(self._h, _ptr(p), p.size), self._err)

    def next_vector_java(self, n, is_null=None, is_repeating=False, out=None):
        """IntegerReader.nextVector(ColumnVector, long[], int)
        (RunLengthIntegerReaderV2.java:371-396): `is_null` None = noNulls;
        null slots get 1; returns (vector, isRepeating). `out` is the
        caller's long[] (left untouched by the all-null repeating early-out)."""
        if out is None:
            out = np.zeros(n, dtype=np.int64)
        isn = None if is_null is None else np.ascontiguousarray(is_null, dtype=np.uint8)
        rep = ctypes.c_int(1 if is_repeating else 0)
        check(self._L.orcg_rle_decoder_next_vector_java(self._h, _ptr(out), _ptr(isn), n,
                                                         ctypes.byref(rep)), self._err)
        return out, bool(rep.value)

    def next_vector_java_int(self, n, is_null=None, is_repeating=False, out=None):
        """IntegerReader.nextVector(ColumnVector, int[], int)
        (RunLengthIntegerReaderV2.java:399-411): (int) narrowing, null slots
        1; isRepeating is read, not computed."""
        if out is None:
            out = np.zeros(n, dtype=np.int32)
        isn = None if is_null is None else np.ascontiguousarray(is_null, dtype=np.uint8)
        check(self._L.orcg_rle_decoder_next_vector_java_int(self._h, _ptr(out), _ptr(isn), n,
                                                             1 if is_repeating else 0), self._err)
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._L.orcg_rle_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rlev2_variants():
    """RLEv2 kernel variants the library accepts (Context.set_rlev2_variant):
    0 = default, 1 = wave-walk, the rest pin one tiled instance."""
    L = _lib.load()
    n = L.orcg_rlev2_variants(None, 0)
    out = (ctypes.c_int * max(n, 1))()
    L.orcg_rlev2_variants(out, n)
    return list(out[:n])


def create_java_rle_decoder(data, is_signed, skip_corrupt=False, ctx=None):
    """new RunLengthIntegerReaderV2(input, signed, skipCorrupt)
    (java/core/src/java/org/apache/orc/impl/RunLengthIntegerReaderV2.java:47-52)
    over the GPU decode: the Java face's decoder, with Java's checks."""
    return RleDecoderV2(data, is_signed, ctx=ctx, java=bool(skip_corrupt))


def create_rle_decoder(data, is_signed, version=RleVersion_2, ctx=None):
    """createRleDecoder (c++/src/RLE.cc:48-60)."""
    if version != RleVersion_2:
        raise InvalidArgument("only RleVersion_2 streams decode on the GPU")
    return RleDecoderV2(data, is_signed, ctx=ctx, version=version)


def rlev2_decode(data, n, is_signed, not_null=None, dtype=np.int64, ctx=None, out=None):
    """orcg_rlev2_decode_{i64,i32,i16}: one-shot host-buffer decode."""
    L = _lib.load()
    ctx = ctx or default_context()
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    if out is None:
        out = np.zeros(n, dtype=dtype)
    nn = None if not_null is None else np.ascontiguousarray(not_null, dtype=np.uint8)
    fn = {8: L.orcg_rlev2_decode_i64, 4: L.orcg_rlev2_decode_i32, 2: L.orcg_rlev2_decode_i16}
    check(fn[out.dtype.itemsize](ctx.handle, _ptr(buf), buf.size, int(bool(is_signed)), _ptr(nn), n,
                                 _ptr(out)), ctx.last_error)
    return out


def rlev1_decode(data, n, is_signed, not_null=None, dtype=np.int64, ctx=None, out=None):
    """orcg_rlev1_decode_{i64,i32}: one-shot host-buffer RLEv1 decode
    (RleDecoderV1::next, c++/src/RLEv1.cc:234-300)."""
    L = _lib.load()
    ctx = ctx or default_context()
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    if out is None:
        out = np.zeros(n, dtype=dtype)
    nn = None if not_null is None else np.ascontiguousarray(not_null, dtype=np.uint8)
    fn = {8: L.orcg_rlev1_decode_i64, 4: L.orcg_rlev1_decode_i32}
    check(fn[out.dtype.itemsize](ctx.handle, _ptr(buf), buf.size, int(bool(is_signed)), _ptr(nn), n,
                                 _ptr(out)), ctx.last_error)
    return out


class Plan:
    """orcg_rlev2_plan: host run walk -> segments (+ first corrupt run)."""

    def __init__(self, data, max_segment_bytes=16 << 10, max_segment_values=8192):
        self._L = _lib.load()
        self._buf = np.frombuffer(bytes(data), dtype=np.uint8)
        h = ctypes.c_void_p()
        check(self._L.orcg_rlev2_plan_create(_ptr(self._buf), self._buf.size, max_segment_bytes,
                                             max_segment_values, ctypes.byref(h)))
        self._h = h

    @property
    def values(self):
        return int(self._L.orcg_rlev2_plan_values(self._h))

    def segments(self):
        p = ctypes.c_void_p()
        n = int(self._L.orcg_rlev2_plan_segments(self._h, ctypes.byref(p)))
        if n == 0:
            return np.zeros((0, 2), dtype=np.uint64)
        arr = (ctypes.c_uint64 * (2 * n)).from_address(p.value)
        return np.frombuffer(arr, dtype=np.uint64).reshape(n, 2).copy()

    def error(self):
        at = ctypes.c_uint64()
        msg = ctypes.c_char_p()
        rc = self._L.orcg_rlev2_plan_error(self._h, ctypes.byref(at), ctypes.byref(msg))
        if rc == 0:
            return None
        return rc, int(at.value), msg.value.decode()

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orcg_rlev2_plan_destroy(self._h)
            self._h = None


def _tensor_ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def decode_device(ctx, src, segments, nvalues, is_signed, out, value_begin=0):
    """Device-resident decode with a segment table (torch tensors on the
    context's device; asynchronous on the context stream)."""
    L = _lib.load()
    ctx.after_torch()
    check(L.orcg_rlev2_decode_device(ctx.handle, _tensor_ptr(src), src.numel(), int(bool(is_signed)),
                                     _tensor_ptr(segments), segments.shape[0], value_begin, nvalues,
                                     _tensor_ptr(out), out.element_size()), ctx.last_error)
    return out


def decode_positions_device(ctx, src, positions, rows_per_group, nvalues, is_signed, out,
                            value_begin=0, src_len=None):
    """Device-resident decode driven by the column's row-index positions."""
    L = _lib.load()
    n = src.numel() if src_len is None else src_len
    ctx.after_torch()
    check(L.orcg_rlev2_decode_positions_device(ctx.handle, _tensor_ptr(src), n, int(bool(is_signed)),
                                               _tensor_ptr(positions), positions.shape[0],
                                               rows_per_group, value_begin, nvalues,
                                               _tensor_ptr(out), out.element_size()),
          ctx.last_error)
    return out


# ---- writer side (synthetic streams) --------------------------------------
def encode_direct(values, is_signed, aligned=True, rows_per_group=0):
    """DIRECT-only RLEv2 stream; returns (bytes ndarray, positions [G,2] or None)."""
    L = _lib.load()
    v = np.ascontiguousarray(values, dtype=np.int64)
    cap = v.size * 8 + (v.size // 512 + 1) * 2 + 16
    dst = np.empty(cap, dtype=np.uint8)
    out_len = ctypes.c_uint64()
    pos = None
    if rows_per_group:
        ng = (v.size + rows_per_group - 1) // rows_per_group
        pos = np.zeros((ng, 2), dtype=np.uint64)
    check(L.orcg_rlev2_encode_direct(_ptr(v), v.size, int(bool(is_signed)), int(bool(aligned)),
                                     _ptr(dst), cap, ctypes.byref(out_len), rows_per_group,
                                     _ptr(pos)), lambda: b"encode failed")
    return dst[: out_len.value].copy(), pos


KIND = {"short_repeat": 0, "direct": 1, "patched_base": 2, "delta": 3}


def encode_runs(values, is_signed, kinds, lengths):
    """Explicit run builder; returns (bytes ndarray, run byte offsets)."""
    L = _lib.load()
    v = np.ascontiguousarray(values, dtype=np.int64)
    k = np.ascontiguousarray([KIND.get(x, x) for x in kinds], dtype=np.uint8)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    cap = v.size * 9 + k.size * 64 + 64
    dst = np.empty(cap, dtype=np.uint8)
    offs = np.zeros(k.size, dtype=np.uint64)
    out_len = ctypes.c_uint64()
    check(L.orcg_rlev2_encode_runs(_ptr(v), v.size, int(bool(is_signed)), _ptr(k), _ptr(ln), k.size,
                                   _ptr(dst), cap, ctypes.byref(out_len), _ptr(offs)),
          lambda: b"values not representable with the requested run kinds")
    return dst[: out_len.value].copy(), offs


# ---- byte / boolean RLE ------------------------------------------------------
class ByteRleDecoder:
    """Drop-in for orc::ByteRleDecoder (createByteRleDecoder /
    createBooleanRleDecoder, c++/src/ByteRLE.hh:114,126): bulk GPU decode at
    construction, then next(n, notNull) / skip(n) / seek(positions)."""

    def __init__(self, data, boolean=False, ctx=None):
        self._L = _lib.load()
        self.ctx = ctx or default_context()
        self.boolean = boolean
        self._buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        h = ctypes.c_void_p()
        check(self._L.orcg_byte_rle_decoder_create(self.ctx.handle, _ptr(self._buf), self._buf.size,
                                                   int(bool(boolean)), ctypes.byref(h)), self.ctx.last_error)
        self._h = h

    def _err(self):
        return self._L.orcg_byte_rle_decoder_last_error(self._h)

    def next(self, n, not_null=None, out=None):
        if out is None:
            out = np.zeros(n, dtype=np.uint8)
        nn = None if not_null is None else np.ascontiguousarray(not_null, dtype=np.uint8)
        check(self._L.orcg_byte_rle_decoder_next(self._h, _ptr(out), n, _ptr(nn)), self._err)
        return out

    def skip(self, n):
        check(self._L.orcg_byte_rle_decoder_skip(self._h, n), self._err)

    def seek(self, *positions):
        p = np.asarray(positions, dtype=np.uint64)
        check(self._L.orcg_byte_rle_decoder_seek(self._h, _ptr(p), p.size), self._err)

    def close(self):
        if getattr(self, "_h", None):
            self._L.orcg_byte_rle_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def java_tree_present_next(present, batch, parent_is_null=None, is_repeating=False):
    """TreeReader.nextVector (TreeReaderFactory.java:405-441) through the C
    ABI: `present` a boolean ByteRleDecoder (BitFieldReader) or None; returns
    (isNull bytes, noNulls, isRepeating)."""
    L = _lib.load()
    isn = np.zeros(batch, dtype=np.uint8)
    par = None if parent_is_null is None else np.ascontiguousarray(parent_is_null, dtype=np.uint8)
    nn, rep = ctypes.c_int(0), ctypes.c_int(1 if is_repeating else 0)
    check(L.orcg_java_tree_present_next(present._h if present is not None else None, _ptr(par), batch, _ptr(isn),
                                        ctypes.byref(nn), ctypes.byref(rep)), L.orcg_java_last_error)
    return isn, bool(nn.value), bool(rep.value)


def java_dictionary_next(data, dict_offsets, buffer_len, is_null, no_nulls, is_repeating, scratch,
                         has_buffer=True, start=None, length=None):
    """StringDictionaryTreeReader.readDictionaryByteArray
    (TreeReaderFactory.java:2396-2478): `data` the DATA RleDecoderV2
    (unsigned), dict_offsets the int[] dictionaryOffsets (None = null),
    is_null / no_nulls / is_repeating from java_tree_present_next (is_null is
    updated in place), scratch the persistent scratchlcv.vector (int64).
    Returns (start, length, noNulls, isRepeating): the setRef arguments."""
    L = _lib.load()
    batch = is_null.size
    offs = None if dict_offsets is None else np.ascontiguousarray(dict_offsets, dtype=np.int32)
    if start is None:
        start = np.zeros(batch, dtype=np.int32)
    if length is None:
        length = np.zeros(batch, dtype=np.int32)
    nn, rep = ctypes.c_int(1 if no_nulls else 0), ctypes.c_int(1 if is_repeating else 0)
    check(L.orcg_java_dictionary_next(data._h if data is not None else None, _ptr(offs),
                                      0 if offs is None else offs.size, 1 if has_buffer else 0, int(buffer_len),
                                      _ptr(is_null), ctypes.byref(nn), ctypes.byref(rep), batch, _ptr(scratch),
                                      _ptr(start), _ptr(length)), L.orcg_java_last_error)
    return start, length, bool(nn.value), bool(rep.value)


def create_byte_rle_decoder(data, ctx=None):
    return ByteRleDecoder(data, boolean=False, ctx=ctx)


def create_boolean_rle_decoder(data, ctx=None):
    return ByteRleDecoder(data, boolean=True, ctx=ctx)


class BytePlan(Plan):
    """orcg_byterle_plan_create: control-byte walk -> segments."""

    def __init__(self, data, max_segment_bytes=16 << 10, max_segment_values=16384):
        self._L = _lib.load()
        self._buf = np.frombuffer(bytes(data), dtype=np.uint8)
        h = ctypes.c_void_p()
        check(self._L.orcg_byterle_plan_create(_ptr(self._buf), self._buf.size, max_segment_bytes,
                                               max_segment_values, ctypes.byref(h)))
        self._h = h


def byterle_decode_device(ctx, src, segments, nvalues, out, value_begin=0, boolean=False):
    """Device-resident byte RLE (decoded bytes) or boolean RLE (one 0/1 char
    per row) decode; torch tensors, asynchronous on the context stream."""
    L = _lib.load()
    fn = L.orcg_boolrle_decode_device if boolean else L.orcg_byterle_decode_device
    ctx.after_torch()
    check(fn(ctx.handle, _tensor_ptr(src), src.numel(), _tensor_ptr(segments), segments.shape[0], value_begin,
             nvalues, _tensor_ptr(out)), ctx.last_error)
    return out


def scatter_not_null_device(ctx, dense, not_null, out, fill=None):
    """dense values -> non-null rows of out (null slots untouched, or `fill`)."""
    L = _lib.load()
    ctx.after_torch()
    check(L.orcg_scatter_not_null_device(ctx.handle, _tensor_ptr(dense), _tensor_ptr(not_null), not_null.numel(),
                                         _tensor_ptr(out), out.element_size(), 0 if fill is None else 1,
                                         0 if fill is None else int(fill)), ctx.last_error)
    return out


def dict_offsets_device(ctx, lengths, offsets):
    L = _lib.load()
    ctx.after_torch()
    check(L.orcg_dict_offsets_device(ctx.handle, _tensor_ptr(lengths), lengths.numel(), _tensor_ptr(offsets)),
          ctx.last_error)
    return offsets


def dict_gather_device(ctx, indices, offsets, start, length, not_null=None):
    L = _lib.load()
    nn = None if not_null is None else _tensor_ptr(not_null)
    ctx.after_torch()
    check(L.orcg_dict_gather_device(ctx.handle, _tensor_ptr(indices), indices.element_size(), nn, indices.numel(),
                                    _tensor_ptr(offsets), offsets.numel() - 1, _tensor_ptr(start),
                                    _tensor_ptr(length)), ctx.last_error)
    return start, length


def decimal_decode_device(ctx, src, scales, nvalues, precision, scale, out, src_len=None):
    """Decimal64/128ColumnReader value decode of a device varint stream:
    `out` int64[nvalues] (precision <= 18) or int64[nvalues, 2] [hi, lo]."""
    L = _lib.load()
    n = src.numel() if src_len is None else src_len
    ctx.after_torch()
    check(L.orcg_decimal_decode_device(ctx.handle, _tensor_ptr(src), n, _tensor_ptr(scales), nvalues, precision,
                                       scale, _tensor_ptr(out)), ctx.last_error)
    return out


def timestamp_decode_device(ctx, seconds, nanos, epoch=1420070400):
    """TimestampColumnReader value construction on device tensors, in place."""
    L = _lib.load()
    ctx.after_torch()
    check(L.orcg_timestamp_decode_device(ctx.handle, _tensor_ptr(seconds), _tensor_ptr(nanos), seconds.numel(),
                                         int(epoch)), ctx.last_error)
    return seconds, nanos


def decode_integer_column(present, data, n, is_signed=True, ctx=None):
    """IntegerColumnReader::next over a stripe column: (values, not_null);
    null slots of `values` stay 0 (untouched)."""
    L = _lib.load()
    ctx = ctx or default_context()
    pb = None if present is None else np.frombuffer(bytes(present), dtype=np.uint8)
    db = np.frombuffer(bytes(data), dtype=np.uint8)
    out = np.zeros(n, dtype=np.int64)
    nn = np.zeros(n, dtype=np.uint8)
    check(L.orcg_decode_integer_column(ctx.handle, _ptr(pb), 0 if pb is None else pb.size, _ptr(db), db.size,
                                       int(bool(is_signed)), n, _ptr(out), _ptr(nn)), ctx.last_error)
    return out, nn
