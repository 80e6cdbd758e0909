"""orc_amd — MI355X-native decoder for Apache ORC column streams.

The hot path (RLEv2 integer streams; byte/boolean RLE; string-dictionary
gather) runs as hand-written HIP kernels for gfx950 in liborcgpu.so, reached
through the C ABI in include/orcg.h. This package is the thin host-side
mirror of the reference's decoder interface (c++/src/RLE.hh) over that ABI.
"""
from ._lib import DeviceError, InvalidArgument, OrcError, ParseError  # noqa: F401
from .rle import (  # noqa: F401
    BytePlan,
    ByteRleDecoder,
    Context,
    Plan,
    RleDecoderV2,
    RleVersion_1,
    RleVersion_2,
    byterle_decode_device,
    create_boolean_rle_decoder,
    create_byte_rle_decoder,
    create_java_rle_decoder,
    create_rle_decoder,
    decimal_decode_device,
    decode_integer_column,
    dict_gather_device,
    dict_offsets_device,
    decode_device,
    decode_positions_device,
    default_context,
    encode_direct,
    encode_runs,
    java_dictionary_next,
    java_tree_present_next,
    rlev1_decode,
    rlev2_decode,
    rlev2_variants,
    scatter_not_null_device,
    timestamp_decode_device,
)

from .reader import Reader, RowReader, UnionValue, open_reader  # noqa: F401,E402

__version__ = "0.1.0"
