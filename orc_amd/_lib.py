"""ctypes binding of liborcgpu.so (include/orcg.h).

The product path has no CPU fallback: if the shared library is missing or no
HIP device is usable, every decode raises instead of silently computing on
the host.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ORCG_LIB selects another in-tree build (e.g. liborcgpu_prof.so, the
# phase-profiling variant used by scripts/phase_prof.py)
LIB_PATH = os.path.join(HERE, os.environ.get("ORCG_LIB", "liborcgpu.so"))

ORCG_OK = 0
ORCG_PARSE_ERROR = 1
ORCG_INVALID_ARGUMENT = 2
ORCG_DEVICE_ERROR = 3
ORCG_OUT_OF_MEMORY = 4


class OrcError(RuntimeError):
    status = None


class ParseError(OrcError):
    """orc::ParseError (c++/include/orc/Exceptions.hh:40)."""

    status = ORCG_PARSE_ERROR


class InvalidArgument(OrcError):
    """orc::InvalidArgument (c++/include/orc/Exceptions.hh:52)."""

    status = ORCG_INVALID_ARGUMENT


class DeviceError(OrcError):
    status = ORCG_DEVICE_ERROR


_EXC = {ORCG_PARSE_ERROR: ParseError, ORCG_INVALID_ARGUMENT: InvalidArgument,
        ORCG_DEVICE_ERROR: DeviceError, ORCG_OUT_OF_MEMORY: DeviceError}

vp, u64, i32, sz, cp = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t, ctypes.c_char_p

# (name, argtypes, restype): every symbol include/orcg.h declares.
SIGNATURES = [
    ("orcg_ctx_create", [i32, ctypes.POINTER(vp)], i32),
    ("orcg_ctx_destroy", [vp], None),
    ("orcg_ctx_set_stream", [vp, vp], i32),
    ("orcg_ctx_stream", [vp], vp),
    ("orcg_ctx_synchronize", [vp], i32),
    ("orcg_ctx_last_error", [vp], cp),
    ("orcg_ctx_set_rlev2_variant", [vp, i32], i32),
    ("orcg_rlev2_variants", [vp, i32], i32),
    ("orcg_version", [], cp),
    ("orcg_device_count", [], i32),
    ("orcg_host_register", [vp, u64], i32),
    ("orcg_host_unregister", [vp], i32),
    ("orcg_rlev2_plan_create", [vp, u64, u64, u64, ctypes.POINTER(vp)], i32),
    ("orcg_rlev2_plan_destroy", [vp], None),
    ("orcg_rlev2_plan_values", [vp], u64),
    ("orcg_rlev2_plan_segments", [vp, ctypes.POINTER(vp)], u64),
    ("orcg_rlev2_plan_error", [vp, ctypes.POINTER(u64), ctypes.POINTER(cp)], i32),
    ("orcg_rlev2_decode_device", [vp, vp, u64, i32, vp, u64, u64, u64, vp, i32], i32),
    ("orcg_rlev2_decode_positions_device", [vp, vp, u64, i32, vp, u64, u64, u64, u64, vp, i32], i32),
    ("orcg_rlev2_decode_i64", [vp, vp, u64, i32, vp, u64, vp], i32),
    ("orcg_rlev2_decode_i32", [vp, vp, u64, i32, vp, u64, vp], i32),
    ("orcg_rlev2_decode_i16", [vp, vp, u64, i32, vp, u64, vp], i32),
    ("orcg_rle_decoder_create", [vp, vp, u64, i32, i32, ctypes.POINTER(vp)], i32),
    ("orcg_rle_decoder_create_java", [vp, vp, u64, i32, i32, ctypes.POINTER(vp)], i32),
    ("orcg_rle_decoder_destroy", [vp], None),
    ("orcg_rle_decoder_next_i64", [vp, vp, u64, vp], i32),
    ("orcg_rle_decoder_next_i32", [vp, vp, u64, vp], i32),
    ("orcg_rle_decoder_next_i16", [vp, vp, u64, vp], i32),
    ("orcg_rle_decoder_skip", [vp, u64], i32),
    ("orcg_rle_decoder_seek", [vp, vp, u64], i32),
    ("orcg_rle_decoder_next_vector_java", [vp, vp, vp, u64, ctypes.POINTER(i32)], i32),
    ("orcg_rle_decoder_next_vector_java_int", [vp, vp, vp, u64, i32], i32),
    ("orcg_rle_decoder_last_error", [vp], cp),
    ("orcg_rlev1_plan_create", [vp, u64, u64, u64, ctypes.POINTER(vp)], i32),
    ("orcg_rlev1_decode_device", [vp, vp, u64, i32, vp, u64, u64, u64, vp, i32], i32),
    ("orcg_rlev1_decode_i64", [vp, vp, u64, i32, vp, u64, vp], i32),
    ("orcg_rlev1_decode_i32", [vp, vp, u64, i32, vp, u64, vp], i32),
    ("orcg_byterle_plan_create", [vp, u64, u64, u64, ctypes.POINTER(vp)], i32),
    ("orcg_byterle_decode_device", [vp, vp, u64, vp, u64, u64, u64, vp], i32),
    ("orcg_boolrle_decode_device", [vp, vp, u64, vp, u64, u64, u64, vp], i32),
    ("orcg_byte_rle_decoder_create", [vp, vp, u64, i32, ctypes.POINTER(vp)], i32),
    ("orcg_byte_rle_decoder_destroy", [vp], None),
    ("orcg_byte_rle_decoder_next", [vp, vp, u64, vp], i32),
    ("orcg_byte_rle_decoder_skip", [vp, u64], i32),
    ("orcg_byte_rle_decoder_seek", [vp, vp, u64], i32),
    ("orcg_byte_rle_decoder_last_error", [vp], cp),
    ("orcg_scatter_not_null_device", [vp, vp, vp, u64, vp, i32, i32, ctypes.c_int64], i32),
    ("orcg_dict_offsets_device", [vp, vp, u64, vp], i32),
    ("orcg_dict_gather_device", [vp, vp, i32, vp, u64, vp, u64, vp, vp], i32),
    ("orcg_decimal_decode_device", [vp, vp, u64, vp, u64, ctypes.c_uint32, i32, vp], i32),
    ("orcg_hive11_decimal_decode_device", [vp, vp, u64, vp, u64, i32, i32, vp, vp], i32),
    ("orcg_timestamp_decode_device", [vp, vp, vp, u64, ctypes.c_int64], i32),
    ("orcg_decode_integer_column", [vp, vp, u64, vp, u64, i32, u64, vp, vp], i32),
    ("orcg_java_last_error", [], cp),
    ("orcg_java_tree_present_next", [vp, vp, u64, vp, ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
    ("orcg_java_dictionary_next", [vp, vp, u64, i32, ctypes.c_int64, vp, ctypes.POINTER(i32), ctypes.POINTER(i32),
                                   u64, vp, vp, vp], i32),
    ("orcg_rlev2_encode_direct", [vp, u64, i32, i32, vp, u64, ctypes.POINTER(u64), u64, vp], i32),
    ("orcg_rlev2_encode_runs", [vp, u64, i32, vp, vp, u64, vp, u64, ctypes.POINTER(u64), vp], i32),
]

# symbols of the A/B build (liborcgpu_ab.so, ORCG_LIB) only
AB_SIGNATURES = [("orcg_probe_copy", [vp, vp, vp, u64, i32], i32)]

_lib = None



class TypeInfo(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("num_subtypes", ctypes.c_uint32), ("maximum_length", ctypes.c_uint32),
                ("precision", ctypes.c_uint32), ("scale", ctypes.c_uint32)]


class StripeInfo(ctypes.Structure):
    _fields_ = [("offset", u64), ("index_length", u64), ("data_length", u64), ("footer_length", u64),
                ("num_rows", u64)]


class ColumnView(ctypes.Structure):
    _fields_ = [("type_id", ctypes.c_uint32), ("kind", ctypes.c_uint32), ("encoding", ctypes.c_uint32),
                ("decoded", ctypes.c_uint32), ("num_elements", u64), ("has_nulls", i32), ("not_null", vp),
                ("data", vp), ("length", vp), ("offsets", vp), ("blob", vp), ("blob_len", u64),
                ("secondary", vp), ("tags", vp), ("index", vp), ("dict_offsets", vp), ("dict_size", u64)]


class RowReaderOptions(ctypes.Structure):
    _fields_ = [("offset", u64), ("length", u64), ("include", vp), ("include_len", ctypes.c_uint32),
                ("lazy_dictionary", i32)]


u32 = ctypes.c_uint32
# include/orcg_reader.h
SIGNATURES += [
    ("orcg_reader_open", [vp, vp, u64, ctypes.POINTER(vp)], i32),
    ("orcg_reader_open_file", [vp, cp, ctypes.POINTER(vp)], i32),
    ("orcg_reader_open_error", [], cp),
    ("orcg_reader_destroy", [vp], None),
    ("orcg_reader_last_error", [vp], cp),
    ("orcg_reader_num_rows", [vp], u64),
    ("orcg_reader_num_stripes", [vp], u64),
    ("orcg_reader_row_index_stride", [vp], u32),
    ("orcg_reader_compression", [vp], u32),
    ("orcg_reader_compression_block_size", [vp], u64),
    ("orcg_reader_format_version", [vp, ctypes.POINTER(u32), ctypes.POINTER(u32)], i32),
    ("orcg_reader_writer_version", [vp], u32),
    ("orcg_reader_num_types", [vp], u32),
    ("orcg_reader_type", [vp, u32, ctypes.POINTER(TypeInfo)], i32),
    ("orcg_reader_subtypes", [vp, u32, ctypes.POINTER(u32), u32], i32),
    ("orcg_reader_field_name", [vp, u32, u32], cp),
    ("orcg_reader_stripe", [vp, u64, ctypes.POINTER(StripeInfo)], i32),
    ("orcg_reader_select", [vp, vp, u32], i32),
    ("orcg_reader_read_stripe", [vp, u64], i32),
    ("orcg_reader_column", [vp, u32, ctypes.POINTER(ColumnView)], i32),
    ("orcg_reader_read_stripes", [vp, u64, u64], i32),
    ("orcg_reader_bench_stripe_decode", [vp, u64, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double)], i32),
    ("orcg_reader_stripe_column", [vp, u64, u32, ctypes.POINTER(ColumnView)], i32),
    ("orcg_reader_copy_to_host", [vp, vp, vp, u64], i32),
    ("orcg_reader_last_timings", [vp, ctypes.POINTER(ctypes.c_double)], i32),
    ("orcg_reader_last_stream_stats", [vp, ctypes.POINTER(u64)], i32),
    ("orcg_reader_get_metrics", [vp, ctypes.POINTER(u64)], i32),
    ("orcg_reader_reset_metrics", [vp], i32),
    ("orcg_reader_set_metrics_timing", [vp, i32], i32),
    ("orcg_reader_content_length", [vp], u64),
    ("orcg_reader_software_version", [vp], cp),
    ("orcg_reader_num_metadata", [vp], u32),
    ("orcg_reader_metadata_key", [vp, u32], cp),
    ("orcg_reader_metadata_value", [vp, u32, ctypes.POINTER(u64)], vp),
    ("orcg_reader_set_lazy_dictionary", [vp, i32], i32),
    ("orcg_reader_set_hive11_decimal", [vp, i32, i32], i32),
    ("orcg_reader_hive11_scale", [vp], i32),
    ("orcg_reader_last_batched_streams", [vp], u64),
    ("orcg_reader_last_stage_bytes", [vp], u64),
    ("orcg_reader_set_stream_batching", [vp, i32], i32),
    ("orcg_reader_is_selected", [vp, u32], i32),
    ("orcg_row_reader_create", [vp, ctypes.POINTER(RowReaderOptions), ctypes.POINTER(vp)], i32),
    ("orcg_row_reader_destroy", [vp], None),
    ("orcg_row_reader_next", [vp, u64, ctypes.POINTER(u64)], i32),
    ("orcg_row_reader_is_selected", [vp, u32], i32),
    ("orcg_row_reader_stripe", [vp], u64),
    ("orcg_row_reader_row_number", [vp], u64),
    ("orcg_host_alloc", [u64], vp),
    ("orcg_host_free", [vp], None),
    ("orcg_row_reader_last_error", [vp], cp),
    ("orcg_row_reader_timings", [vp, ctypes.POINTER(ctypes.c_double)], i32),
    ("orcg_row_reader_seek_to_row", [vp, u64], i32),
    ("orcg_row_reader_column", [vp, u32, ctypes.POINTER(ColumnView), ctypes.POINTER(u64), ctypes.POINTER(u64)],
     i32),
]


def load():
    """Load liborcgpu.so (building it first if absent). torch is imported
    first so that the library binds to the HIP runtime torch already loaded
    (both carry SONAME libamdhip64.so.7)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (shares its libamdhip64 with us)
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        from . import build as _build
        _build.build()
    L = ctypes.CDLL(LIB_PATH)
    for name, args, res in SIGNATURES:
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    for name, args, res in AB_SIGNATURES:  # present in the A/B build only
        f = getattr(L, name, None)
        if f is not None:
            f.argtypes = args
            f.restype = res
    _lib = L
    return L


def check(rc, msg_fn=None):
    if rc == ORCG_OK:
        return
    msg = msg_fn() if msg_fn else ""
    if isinstance(msg, bytes):
        msg = msg.decode(errors="replace")
    raise _EXC.get(rc, OrcError)(msg or "orcg status %d" % rc)
