"""ctypes binding for the CPU oracle (oracle/orc_oracle.c).

TEST INFRASTRUCTURE ONLY. Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the orc_amd product path.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


class OracleError(RuntimeError):
    """Mirrors orc::ParseError raised by the reference decoders."""


def build(force=False):
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "orc_oracle.c"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, u64, i32, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t
        L.orco_last_error.restype = ctypes.c_char_p
        for name, args, res in [
            ("orco_rlev2_new", [vp, sz, i32], vp),
            ("orco_rlev2_free", [vp], None),
            ("orco_rlev2_next_i64", [vp, vp, u64, vp], i32),
            ("orco_rlev2_next_i32", [vp, vp, u64, vp], i32),
            ("orco_rlev2_next_i16", [vp, vp, u64, vp], i32),
            ("orco_rlev2_skip", [vp, u64], i32),
            ("orco_rlev2_seek", [vp, u64, u64], i32),
            ("orco_rlev2_decode_i64", [vp, sz, i32, vp, u64], i32),
            ("orco_rlev2_count", [vp, sz, i32, vp], i32),
            ("orco_byterle_new", [vp, sz], vp),
            ("orco_byterle_free", [vp], None),
            ("orco_byterle_next", [vp, vp, u64, vp], i32),
            ("orco_byterle_skip", [vp, u64], i32),
            ("orco_byterle_seek", [vp, u64, u64], i32),
            ("orco_boolrle_next", [vp, vp, u64, vp], i32),
            ("orco_boolrle_skip", [vp, u64], i32),
            ("orco_boolrle_seek", [vp, u64, u64, u64], i32),
            ("orco_rlev1_new", [vp, sz, i32], vp),
            ("orco_rlev1_free", [vp], None),
            ("orco_rlev1_next_i64", [vp, vp, u64, vp], i32),
            ("orco_rlev1_skip", [vp, u64], i32),
            ("orco_rlev1_seek", [vp, u64, u64], i32),
            ("orco_dict_offsets", [vp, u64, vp], None),
            ("orco_dict_gather", [vp, u64, vp, vp, u64, vp, vp], i32),
            ("orco_decimal_decode", [vp, sz, vp, u64, i32, i32, vp], i32),
            ("orco_decimal_decode_keep", [vp, sz, vp, u64, i32, vp, vp], i32),
            ("orco_timestamp", [vp, vp, u64, ctypes.c_int64], None),
        ]:
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise OracleError(lib().orco_last_error().decode())


def _ptr(a):
    return None if a is None else a.ctypes.data


class _Stream:
    def __init__(self, data):
        self._buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()


class RleDecoderV2(_Stream):
    """Stateful mirror of orc::RleDecoderV2 (c++/src/RleDecoderV2.cc)."""

    def __init__(self, data, is_signed):
        super().__init__(data)
        self._h = lib().orco_rlev2_new(_ptr(self._buf), self._buf.size, int(bool(is_signed)))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orco_rlev2_free(self._h)
            self._h = None

    def next(self, n, not_null=None, dtype=np.int64, out=None):
        if out is None:
            out = np.zeros(n, dtype=dtype)
        nn = None if not_null is None else np.ascontiguousarray(not_null, dtype=np.uint8)
        fn = {8: lib().orco_rlev2_next_i64, 4: lib().orco_rlev2_next_i32, 2: lib().orco_rlev2_next_i16}
        _check(fn[out.dtype.itemsize](self._h, _ptr(out), n, _ptr(nn)))
        return out

    def skip(self, n):
        _check(lib().orco_rlev2_skip(self._h, n))

    def seek(self, byte_offset, values_to_skip):
        _check(lib().orco_rlev2_seek(self._h, byte_offset, values_to_skip))


class RleDecoderV1(_Stream):
    """Stateful mirror of orc::RleDecoderV1 (c++/src/RLEv1.cc)."""

    def __init__(self, data, is_signed):
        super().__init__(data)
        self._h = lib().orco_rlev1_new(_ptr(self._buf), self._buf.size, int(bool(is_signed)))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orco_rlev1_free(self._h)
            self._h = None

    def next(self, n, not_null=None, out=None):
        if out is None:
            out = np.zeros(n, dtype=np.int64)
        nn = None if not_null is None else np.ascontiguousarray(not_null, dtype=np.uint8)
        _check(lib().orco_rlev1_next_i64(self._h, _ptr(out), n, _ptr(nn)))
        return out

    def skip(self, n):
        _check(lib().orco_rlev1_skip(self._h, n))

    def seek(self, byte_offset, values_to_skip):
        _check(lib().orco_rlev1_seek(self._h, byte_offset, values_to_skip))


class ByteRleDecoder(_Stream):
    """Mirror of orc::ByteRleDecoderImpl / BooleanRleDecoderImpl (c++/src/ByteRLE.cc)."""

    def __init__(self, data, boolean=False):
        super().__init__(data)
        self.boolean = boolean
        self._h = lib().orco_byterle_new(_ptr(self._buf), self._buf.size)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orco_byterle_free(self._h)
            self._h = None

    def next(self, n, not_null=None, out=None):
        if out is None:
            out = np.zeros(n, dtype=np.uint8)
        nn = None if not_null is None else np.ascontiguousarray(not_null, dtype=np.uint8)
        f = lib().orco_boolrle_next if self.boolean else lib().orco_byterle_next
        _check(f(self._h, _ptr(out), n, _ptr(nn)))
        return out

    def skip(self, n):
        _check((lib().orco_boolrle_skip if self.boolean else lib().orco_byterle_skip)(self._h, n))

    def seek(self, *position):
        if self.boolean:
            _check(lib().orco_boolrle_seek(self._h, *position))
        else:
            _check(lib().orco_byterle_seek(self._h, *position))


def rlev2_decode(data, n, is_signed):
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    out = np.empty(n, dtype=np.int64)
    _check(lib().orco_rlev2_decode_i64(_ptr(buf), buf.size, int(bool(is_signed)), _ptr(out), n))
    return out


def rlev2_count(data, is_signed):
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    c = np.zeros(1, dtype=np.uint64)
    _check(lib().orco_rlev2_count(_ptr(buf), buf.size, int(bool(is_signed)), _ptr(c)))
    return int(c[0])


def dict_gather(indices, lengths, not_null=None):
    """(start, length) per row for a string dictionary column."""
    indices = np.ascontiguousarray(indices, dtype=np.int64)
    lengths = np.ascontiguousarray(lengths, dtype=np.int64)
    offs = np.zeros(lengths.size + 1, dtype=np.int64)
    lib().orco_dict_offsets(_ptr(lengths), lengths.size, _ptr(offs))
    start = np.zeros(indices.size, dtype=np.int64)
    ln = np.zeros(indices.size, dtype=np.int64)
    nn = None if not_null is None else np.ascontiguousarray(not_null, dtype=np.uint8)
    _check(lib().orco_dict_gather(_ptr(indices), indices.size, _ptr(nn), _ptr(offs), lengths.size,
                                  _ptr(start), _ptr(ln)))
    return start, ln


def decimal_decode(data, scales, n, scale, wide):
    """Decimal64/128ColumnReader value decode (orco_decimal_decode): int64[n],
    or int64[n, 2] of [hi, lo] when wide (wide=2: Hive 0.11 decimals, with the
    38-digit check)."""
    L = lib()
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    sc = np.ascontiguousarray(scales, dtype=np.int64)
    out = np.zeros((n, 2) if wide else n, dtype=np.int64)
    if L.orco_decimal_decode(buf.ctypes.data, buf.size, sc.ctypes.data, n, int(scale), 2 if wide == 2 else int(bool(wide)),
                             out.ctypes.data) != 0:
        raise OracleError(L.orco_last_error().decode())
    return out


def decimal_decode_keep(data, scales, n, scale):
    """Hive 0.11 decimals with throwOnHive11DecimalOverflow(false)
    (orco_decimal_decode_keep): ([hi, lo] int64[n, 2], keep uint8[n]); an
    overflowing value reads 0 with keep 0."""
    L = lib()
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    sc = np.ascontiguousarray(scales, dtype=np.int64)
    out = np.zeros((n, 2), dtype=np.int64)
    keep = np.zeros(n, dtype=np.uint8)
    if L.orco_decimal_decode_keep(buf.ctypes.data, buf.size, sc.ctypes.data, n, int(scale), out.ctypes.data,
                                  keep.ctypes.data) != 0:
        raise OracleError(L.orco_last_error().decode())
    return out, keep


def timestamp(secs, nanos, epoch=1420070400):
    """TimestampColumnReader value construction (orco_timestamp): (seconds, nanoseconds)."""
    L = lib()
    s = np.array(secs, dtype=np.int64)
    ns = np.array(nanos, dtype=np.int64)
    L.orco_timestamp(s.ctypes.data, ns.ctypes.data, s.size, int(epoch))
    return s, ns
