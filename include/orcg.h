/*
 * orcg.h — C ABI of the MI355X-native ORC column-stream decoder (liborcgpu).
 *
 * This is the drop-in boundary for the reference's stream-decoder hot path.
 * Every entry point is plain C (pointers + sizes, no torch / HIP C++ types);
 * hipStream_t travels as void*. The reference interfaces each group replaces
 * are cited inline (paths relative to the apache/orc checkout). No exceptions
 * cross this ABI: every call returns an ORCG_* status and the message is
 * available from orcg_ctx_last_error() / orcg_*_last_error(). The C++ adapter
 * (orc_amd/csrc/GpuRleDecoder.hh) rethrows them as orc::ParseError /
 * orc::InvalidArgument with the reference's messages
 * (c++/include/orc/Exceptions.hh:40-60); the JNI shim in INTEGRATION.md throws
 * java.io.IOException.
 *
 * Memory ownership: the caller owns every src/dst buffer and
 * the library never frees caller memory. Device scratch lives in an orcg_ctx,
 * one per reader thread (reentrant; contexts are not shared between threads).
 *
 * Value semantics are those of orc::RleDecoderV2 (c++/src/RleDecoderV2.cc):
 * zigzag for signed streams, int64 wraparound, static_cast narrowing for
 * int32/int16 outputs, and null slots (not_null[i] == 0) left untouched.
 */
#ifndef ORCG_H
#define ORCG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status ------------------------------------------------------------ */
enum {
  ORCG_OK = 0,
  ORCG_PARSE_ERROR = 1,      /* orc::ParseError (corrupt / truncated stream) */
  ORCG_INVALID_ARGUMENT = 2, /* orc::InvalidArgument (bad call, bad position) */
  ORCG_DEVICE_ERROR = 3,     /* HIP runtime failure or no usable device */
  ORCG_OUT_OF_MEMORY = 4
};

/* ---- context (one per reader thread) ------------------------------------ */
typedef struct orcg_ctx orcg_ctx;

/* Create a context bound to HIP device `device`, with its own non-blocking
 * stream. Replaces nothing in the reference (the reference has no device);
 * it is the owner of device scratch that MemoryPool (c++/include/orc/
 * MemoryPool.hh:27-33) plays for host buffers. */
int orcg_ctx_create(int device, orcg_ctx** out);
void orcg_ctx_destroy(orcg_ctx* ctx);

/* Pinned (page-locked) host memory, the allocator of the C++ adapter's
 * PinnedMemoryPool (an orc::MemoryPool, c++/include/orc/MemoryPool.hh:27-33):
 * batches in pinned memory can be DMA'd to a device without a staging copy.
 * NULL on failure. */
void* orcg_host_alloc(uint64_t bytes);
void orcg_host_free(void* p);
/* Use an external stream (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the context's own stream.
 * Ordering contract of every *_device entry: the launch is queued on the
 * context stream and nothing else. The context's own stream is
 * non-blocking, so it is NOT ordered after work on the legacy NULL stream or
 * any other stream: a caller that fills or copies d_src / d_segs / d_dst on
 * stream P must either pass P here, or make the context stream wait on an
 * event recorded on P (hipStreamWaitEvent(orcg_ctx_stream(ctx), ev, 0))
 * before the call. Consumers of d_dst order after the context stream the
 * same way (tests/test_gpu_stream_order.py). */
int orcg_ctx_set_stream(orcg_ctx* ctx, void* hip_stream);
void* orcg_ctx_stream(orcg_ctx* ctx);
/* Wait for the context stream and collect any device-side decode error of
 * the launches issued since the last call (first error in value order). */
int orcg_ctx_synchronize(orcg_ctx* ctx);
const char* orcg_ctx_last_error(const orcg_ctx* ctx);

/* Kernel selection for RLEv2 decode (tuning / A-B measurement). TILED (the
 * default) stages segment chunks through LDS by LDS-DMA and walks headers in
 * LDS; WAVE_WALK is one wavefront per segment reading HBM directly. Both are
 * bit-identical. */
enum { ORCG_RLEV2_TILED = 0, ORCG_RLEV2_WAVE_WALK = 1 };
/* Other accepted values pin one instance of the tiled kernel (used by the
 * parity tests to cover every instance the default may pick, and by A/B
 * timing); orcg_rlev2_variants lists them. Unknown values: INVALID_ARGUMENT. */
int orcg_ctx_set_rlev2_variant(orcg_ctx* ctx, int variant);
/* Writes up to `cap` accepted variant ids to `out`; returns how many exist. */
int orcg_rlev2_variants(int* out, int cap);

const char* orcg_version(void);
/* Number of visible HIP devices (0 when none; never aborts). */
int orcg_device_count(void);
/* Page-lock / release caller host memory for asynchronous D2H copies (e.g.
 * each rank's slice of a shared host batch, orc_amd/shard.py). */
int orcg_host_register(void* host, uint64_t bytes);
int orcg_host_unregister(void* host);

/* ---- segments: the ORC-native parallel sync points ----------------------
 * A segment is a run-aligned byte offset in an uncompressed (or already
 * decompressed) stream plus the index of the first value of the run that
 * starts there. Row-index positions (site/specification/ORCv1.md:1266-1272;
 * recorded by RleEncoderV2::recordPosition) are exactly this: (byte offset of
 * the run start, values of that run to skip). Segment k covers every run
 * whose first byte lies in [segs[k].byte_offset, segs[k+1].byte_offset)
 * (the last one runs to the end of the stream). */
typedef struct orcg_segment {
  uint64_t byte_offset;
  uint64_t value_index;
} orcg_segment;

/* ---- RLEv2 integer streams ----------------------------------------------
 * Replaces the run loop of orc::RleDecoderV2::next<T>
 * (c++/src/RleDecoderV2.cc:132-453) and its bit unpackers
 * BitUnpackDefault/BitUnpackAVX512::readLongs (c++/src/BpackingDefault.cc:
 * 330-366, c++/src/BpackingAvx512.cc:2443-2586) for a whole stream or a
 * row-group range at once. */

/* Host run walk: reads only run headers (the host holds the bytes after
 * decompression) and cuts the stream into segments of at most
 * ~max_segment_bytes / max_segment_values. It also finds the first corrupt
 * run, reported lazily by the decoders exactly where the reference would
 * throw (RleDecoderV2.cc:38, :307, :328-330, :412-415). */
typedef struct orcg_rlev2_plan orcg_rlev2_plan;
int orcg_rlev2_plan_create(const uint8_t* src, uint64_t src_len, uint64_t max_segment_bytes,
                           uint64_t max_segment_values, orcg_rlev2_plan** out);
void orcg_rlev2_plan_destroy(orcg_rlev2_plan* plan);
/* values decodable before the first corrupt run (all values if none) */
uint64_t orcg_rlev2_plan_values(const orcg_rlev2_plan* plan);
uint64_t orcg_rlev2_plan_segments(const orcg_rlev2_plan* plan, const orcg_segment** segs);
/* ORCG_OK, or the status of the first corrupt run (*at_value = its first
 * value index, *msg = the reference's ParseError text). */
int orcg_rlev2_plan_error(const orcg_rlev2_plan* plan, uint64_t* at_value, const char** msg);

/* Device-resident decode (asynchronous on the context stream).
 * d_src: stream bytes in HBM; d_segs: segment table in HBM (nsegs entries);
 * values with index v in [value_begin, value_begin + nvalues) are written
 * dense to d_dst[v - value_begin] as int64/int32/int16 (dst_bytes 8/4/2).
 * Corrupt runs set the context's device error record (see
 * orcg_ctx_synchronize). */
int orcg_rlev2_decode_device(orcg_ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                             const orcg_segment* d_segs, uint64_t nsegs, uint64_t value_begin,
                             uint64_t nvalues, void* d_dst, int dst_bytes);

/* Same, but the segment table is the column's ROW_INDEX positions as the
 * writer records them: d_positions[2*g] = byte offset of the run holding row
 * g*rows_per_group, d_positions[2*g+1] = values of that run to skip
 * (ORCv1.md:1266-1272; RleDecoderV2::seek, RleDecoderV2.cc:109-117). The
 * first value of segment g is g*rows_per_group - skip. No host work. */
int orcg_rlev2_decode_positions_device(orcg_ctx* ctx, const uint8_t* d_src, uint64_t src_len,
                                       int is_signed, const uint64_t* d_positions,
                                       uint64_t ngroups, uint64_t rows_per_group,
                                       uint64_t value_begin, uint64_t nvalues, void* d_dst,
                                       int dst_bytes);

/* Host-buffer decode (the SURVEY.md §8b sketch): H2D, decode, D2H; with a
 * not_null mask the n positions receive values in order and null slots are
 * left untouched (RleDecoderV2::copyDataFromBuffer, :437-453). Synchronous. */
int orcg_rlev2_decode_i64(orcg_ctx* ctx, const uint8_t* src, uint64_t src_len, int is_signed,
                          const char* not_null, uint64_t n, int64_t* dst);
int orcg_rlev2_decode_i32(orcg_ctx* ctx, const uint8_t* src, uint64_t src_len, int is_signed,
                          const char* not_null, uint64_t n, int32_t* dst);
int orcg_rlev2_decode_i16(orcg_ctx* ctx, const uint8_t* src, uint64_t src_len, int is_signed,
                          const char* not_null, uint64_t n, int16_t* dst);

/* ---- stateful decoder: drop-in for orc::RleDecoder ----------------------
 * Mirrors class RleDecoder (c++/src/RLE.hh:109-141) as created by
 * createRleDecoder(stream, isSigned, RleVersion_2, pool, metrics)
 * (c++/src/RLE.hh:163, c++/src/RLE.cc:48-60): the stream is bulk-decoded on
 * the device on creation and next()/skip()/seek() serve slices, so run state
 * persists across calls of any size and errors surface at the same value as
 * in the reference. */
typedef struct orcg_rle_decoder orcg_rle_decoder;
int orcg_rle_decoder_create(orcg_ctx* ctx, const uint8_t* src, uint64_t src_len, int is_signed,
                            int rle_version, orcg_rle_decoder** out);
void orcg_rle_decoder_destroy(orcg_rle_decoder* dec);
int orcg_rle_decoder_next_i64(orcg_rle_decoder* dec, int64_t* data, uint64_t n, const char* not_null);
int orcg_rle_decoder_next_i32(orcg_rle_decoder* dec, int32_t* data, uint64_t n, const char* not_null);
int orcg_rle_decoder_next_i16(orcg_rle_decoder* dec, int16_t* data, uint64_t n, const char* not_null);
/* RleDecoder::skip (RleDecoderV2.cc:119-130) */
int orcg_rle_decoder_skip(orcg_rle_decoder* dec, uint64_t n);
/* RleDecoder::seek(PositionProvider&) (RleDecoderV2.cc:109-117) for an
 * uncompressed stream: positions = {byte offset, values to skip}. */
int orcg_rle_decoder_seek(orcg_rle_decoder* dec, const uint64_t* positions, uint64_t npositions);
/* Java face (java/core/src/java/org/apache/orc/impl/
 * RunLengthIntegerReaderV2.java:371-396, nextVector): null slots get 1 and
 * *is_repeating reports whether every slot holds the same value. is_null may
 * be NULL (no nulls). */
int orcg_rle_decoder_next_vector_java(orcg_rle_decoder* dec, int64_t* vector, const uint8_t* is_null,
                                      uint64_t n, int* is_repeating);
/* The int[] overload (RunLengthIntegerReaderV2.java:399-411): values narrowed
 * to int32 ((int) next()), null slots 1; with a null mask, a vector that is
 * repeating with isNull[0] is left untouched; isRepeating is an input only. */
int orcg_rle_decoder_next_vector_java_int(orcg_rle_decoder* dec, int32_t* vector, const uint8_t* is_null, uint64_t n,
                                          int is_repeating);
const char* orcg_rle_decoder_last_error(const orcg_rle_decoder* dec);
/* A decoder with Java's rules: new RunLengthIntegerReaderV2(input, signed,
 * skipCorrupt) (java/core/src/java/org/apache/orc/impl/
 * RunLengthIntegerReaderV2.java:47-52), for the Java faces above. Where the
 * Java reader differs from the C++ one (it checks less):
 *  - a DELTA run with a bit width and one value (length byte 0) is not an
 *    error: Java emits the first value and first + deltaBase (:125-145);
 *  - PATCHED_BASE with pw + pgw > 64 fails with Java's IOException text
 *    ("Corruption in ORC data encountered. To skip reading corrupted data,
 *    set hive.exec.orc.skip.corrupt.data to true", ORCG_PARSE_ERROR) unless
 *    skip_corrupt, which decodes it reading the patch list at
 *    getClosestFixedBits(pw + pgw) bits an entry with Java's shift semantics
 *    (:196-260: pw = 64 leaves no patch bits, so the values are base + the
 *    packed literals);
 *  - PATCHED_BASE with pl == 0 fails as Java's unpackedPatch[0] does
 *    (ArrayIndexOutOfBoundsException "Index 0 out of bounds for length 0",
 *    ORCG_PARSE_ERROR), after the run's bytes are read.
 * Truncated runs keep the C++ reader's "bad read" errors (Java's InStream
 * returns -1 bytes there instead of failing). Decoded by the wave-walk
 * kernel (ORCG_RLEV2_WAVE_WALK). */
int orcg_rle_decoder_create_java(orcg_ctx* ctx, const uint8_t* src, uint64_t src_len, int is_signed,
                                 int skip_corrupt, orcg_rle_decoder** out);

/* ---- byte RLE / boolean RLE (PRESENT, BOOLEAN, BYTE streams) -------------
 * Replaces ByteRleDecoderImpl / BooleanRleDecoderImpl (c++/src/ByteRLE.hh:
 * 71-126, ByteRLE.cc:359-643). Segments index decoded BYTES; byte-RLE
 * row-index positions are (byte offset, bytes to skip) and boolean ones add
 * the bits consumed of the next byte (ByteRLE.cc:409-417, :549-560). The
 * plan accessors above (orcg_rlev2_plan_*) apply to byte plans too. */
int orcg_byterle_plan_create(const uint8_t* src, uint64_t src_len, uint64_t max_segment_bytes,
                             uint64_t max_segment_values, orcg_rlev2_plan** out);
/* decoded bytes [value_begin, value_begin + nvalues) -> d_dst */
int orcg_byterle_decode_device(orcg_ctx* ctx, const uint8_t* d_src, uint64_t src_len,
                               const orcg_segment* d_segs, uint64_t nsegs, uint64_t value_begin,
                               uint64_t nvalues, uint8_t* d_dst);
/* rows (bits, MSB first) [row_begin, row_begin + nrows) -> one char 0/1 per row */
int orcg_boolrle_decode_device(orcg_ctx* ctx, const uint8_t* d_src, uint64_t src_len,
                               const orcg_segment* d_segs, uint64_t nsegs, uint64_t row_begin,
                               uint64_t nrows, uint8_t* d_dst);

/* Stateful drop-in for orc::ByteRleDecoder as created by
 * createByteRleDecoder / createBooleanRleDecoder (c++/src/ByteRLE.hh:114,126):
 * next(data, n, notNull) leaves null slots untouched (byte) or writes 0
 * (boolean); seek takes 2 (byte) or 3 (boolean) position values. */
typedef struct orcg_byte_rle_decoder orcg_byte_rle_decoder;
int orcg_byte_rle_decoder_create(orcg_ctx* ctx, const uint8_t* src, uint64_t src_len, int boolean,
                                 orcg_byte_rle_decoder** out);
void orcg_byte_rle_decoder_destroy(orcg_byte_rle_decoder* dec);
int orcg_byte_rle_decoder_next(orcg_byte_rle_decoder* dec, char* data, uint64_t n, const char* not_null);
int orcg_byte_rle_decoder_skip(orcg_byte_rle_decoder* dec, uint64_t n);
int orcg_byte_rle_decoder_seek(orcg_byte_rle_decoder* dec, const uint64_t* positions, uint64_t npositions);
const char* orcg_byte_rle_decoder_last_error(const orcg_byte_rle_decoder* dec);

/* ---- Java TreeReader face (java/core/src/java/org/apache/orc/impl/
 * TreeReaderFactory.java): the ColumnVector fields a JNI shim fills, built
 * from the GPU-decoded streams of the stateful decoders above. Java boolean[]
 * travels as one byte per row (1 = true). Errors: the status, and the message
 * from orcg_java_last_error() (this thread's last failure). */
const char* orcg_java_last_error(void);
/* TreeReader.nextVector (TreeReaderFactory.java:405-441): `present` is the
 * column's PRESENT stream as a boolean decoder (BitFieldReader,
 * BitFieldReader.java:30-57; NULL = no PRESENT stream), parent_is_null the
 * parent's isNull (NULL = none). Writes is_null[batch] and *no_nulls; with a
 * PRESENT stream or a parent mask *is_repeating = !noNulls && every row null,
 * otherwise *is_repeating is left unchanged (as the reference leaves it). */
int orcg_java_tree_present_next(orcg_byte_rle_decoder* present, const uint8_t* parent_is_null, uint64_t batch,
                                uint8_t* is_null, int* no_nulls, int* is_repeating);
/* StringDictionaryTreeReader.nextVector's readDictionaryByteArray
 * (TreeReaderFactory.java:2396-2478), no filter context: the DATA indices
 * through RunLengthIntegerReaderV2.nextVector (`data`, unsigned; scratch =
 * the reader's scratchlcv.vector, kept by the caller across batches), then
 * BytesColumnVector.setRef(i, dictionaryBuffer, start[i], length[i]) per row:
 * start = dictionaryOffsets[idx], length = the next offset - start, or
 * buffer_len - start for the last array entry (getDictionaryEntryLength);
 * null rows (0, 0); a repeating index vector sets row 0 only and returns
 * *is_repeating = 1. is_null / *no_nulls / *is_repeating come in from
 * orcg_java_tree_present_next (the result vector's fields). has_buffer = 0
 * (dictionaryBuffer == null): non-null rows get the empty string, or with
 * dict_offsets NULL too the batch becomes one repeating null. An index
 * outside the offsets array: ORCG_PARSE_ERROR with Java's
 * "Index i out of bounds for length n". */
int orcg_java_dictionary_next(orcg_rle_decoder* data, const int32_t* dict_offsets, uint64_t dict_offsets_len,
                              int has_buffer, int64_t buffer_len, uint8_t* is_null, int* no_nulls, int* is_repeating,
                              uint64_t batch, int64_t* scratch, int32_t* start, int32_t* length);

/* ---- RLEv1 (DIRECT / DICTIONARY encodings, format 0.11 files) ------------
 * Replaces RleDecoderV1 (c++/src/RLEv1.hh:51-96, RLEv1.cc:140-300) as chosen
 * by createRleDecoder for RleVersion_1 (c++/src/RLE.cc:48-60). Plans cut the
 * stream at control bytes; the plan accessors (orcg_rlev2_plan_*) apply.
 * Truncated streams raise "bad read in readByte" (RLEv1.cc:141-146). */
int orcg_rlev1_plan_create(const uint8_t* src, uint64_t src_len, uint64_t max_segment_bytes,
                           uint64_t max_segment_values, orcg_rlev2_plan** out);
int orcg_rlev1_decode_device(orcg_ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                             const orcg_segment* d_segs, uint64_t nsegs, uint64_t value_begin,
                             uint64_t nvalues, void* d_dst, int dst_bytes);
/* RleDecoderV1::next<T>(data, n, notNull) over a whole host stream. */
int orcg_rlev1_decode_i64(orcg_ctx* ctx, const uint8_t* src, uint64_t src_len, int is_signed,
                          const char* not_null, uint64_t n, int64_t* data);
int orcg_rlev1_decode_i32(orcg_ctx* ctx, const uint8_t* src, uint64_t src_len, int is_signed,
                          const char* not_null, uint64_t n, int32_t* data);

/* ---- nullable columns and string dictionaries ----------------------------
 * Null scatter (RleDecoderV2::copyDataFromBuffer with notNull,
 * RleDecoderV2.cc:437-453): dense values -> the non-null rows of d_out
 * (width 8/4/2/1 bytes). fill_nulls = 0 leaves null slots untouched (C++);
 * 1 writes fill_value there (Java's 1, RunLengthIntegerReaderV2.java:371-396). */
int orcg_scatter_not_null_device(orcg_ctx* ctx, const void* d_dense, const uint8_t* d_not_null,
                                 uint64_t n, void* d_out, int width, int fill_nulls,
                                 int64_t fill_value);
/* Dictionary LENGTH values -> offsets[dict_size + 1] (loadStringDictionary,
 * c++/src/DictionaryLoader.cc:69-80). */
int orcg_dict_offsets_device(orcg_ctx* ctx, const int64_t* d_lengths, uint64_t dict_size,
                             int64_t* d_offsets);
/* Per non-null row: start = offsets[idx], length = offsets[idx+1] -
 * offsets[idx]; idx >= dict_size raises "Entry index out of range in
 * StringDictionaryColumn" (StringDictionaryColumnReader::next,
 * c++/src/ColumnReader.cc:561-594). Starts are blob-relative: the C++ adapter
 * adds the host blob base after D2H. index_width 8 or 4. */
int orcg_dict_gather_device(orcg_ctx* ctx, const void* d_indices, int index_width,
                            const uint8_t* d_not_null, uint64_t n, const int64_t* d_offsets,
                            uint64_t dict_size, int64_t* d_start, int64_t* d_length);
/* Decimal64ColumnReader / Decimal128ColumnReader::next value decode
 * (c++/src/ColumnReader.cc:1300-1527) over a device-resident DATA stream of
 * zigzag varints and the values' scales (the decoded SECONDARY stream):
 * nvalues values rescaled to `scale`. precision <= 18: int64 d_out[nvalues]
 * ("Decimal scale out of range" past 18 digits, readInt64 :1342-1349);
 * precision > 18: int64 d_out[2 * nvalues], [hi, lo] per value (orc::Int128).
 * precision == 0: Hive 0.11 decimals (DecimalHive11ColumnReader, :1578-1692),
 * Int128 layout rescaled to `scale` (the forced scale, RowReaderOptions::
 * forcedScaleOnHive11Decimal, 6 by default); a value past 128 bits or 38
 * digits is "Hive 0.11 decimal was more than 38 digits." (the reference's
 * default throwOnHive11DecimalOverflow). Fewer varints than nvalues: "Read past end of stream in
 * Decimal64ColumnReader". Synchronous. */
int orcg_decimal_decode_device(orcg_ctx* ctx, const uint8_t* d_src, uint64_t src_len, const int64_t* d_scales,
                               uint64_t nvalues, uint32_t precision, int32_t scale, void* d_out);
/* Hive 0.11 decimals (precision 0) under RowReaderOptions::
 * throwOnHive11DecimalOverflow (c++/include/orc/Reader.hh:258-271;
 * DecimalHive11ColumnReader::next, c++/src/ColumnReader.cc:1638-1680): 1 is
 * orcg_decimal_decode_device(precision 0); 0 replaces every value past 128
 * bits or 38 digits by NULL instead of raising: d_keep[k] (nvalues bytes) is 0
 * for such a value (its slot holds 0) and 1 otherwise. Synchronous. */
int orcg_hive11_decimal_decode_device(orcg_ctx* ctx, const uint8_t* d_src, uint64_t src_len, const int64_t* d_scales,
                                      uint64_t nvalues, int32_t scale, int throw_on_overflow, void* d_out,
                                      uint8_t* d_keep);
/* TimestampColumnReader::next value construction (c++/src/ColumnReader.cc
 * :318-347) in place: seconds += epoch (1420070400 for UTC writers), nanos
 * from the trailing-zero code; writer and reader zones with equal rules. */
int orcg_timestamp_decode_device(orcg_ctx* ctx, int64_t* d_seconds, int64_t* d_nanos, uint64_t n, int64_t epoch);

/* IntegerColumnReader<LongVectorBatch>::next for a whole stripe column
 * (c++/src/ColumnReader.cc:81-104, 224-258): PRESENT (boolean RLE; NULL/0 if
 * the column has no nulls) + DATA (RLEv2) host streams -> not_null[n] and
 * data[n] with null slots untouched. */
int orcg_decode_integer_column(orcg_ctx* ctx, const uint8_t* present, uint64_t present_len,
                               const uint8_t* data, uint64_t data_len, int is_signed, uint64_t n,
                               int64_t* out, char* not_null);

/* ---- synthetic streams (writer side, for benchmarks and tests) ----------
 * A minimal RLEv2 writer: DIRECT runs of up to 512 values at the smallest
 * width from the 5-bit table (aligned = round the width up to the
 * byte-aligned set, as RleEncoderV2's SPEED strategy does,
 * c++/src/RleEncoderV2.cc). Optionally records row-index positions
 * ({byte offset, values to skip} per rows_per_group) the way
 * RleEncoderV2::recordPosition does. */
int orcg_rlev2_encode_direct(const int64_t* values, uint64_t n, int is_signed, int aligned,
                             uint8_t* dst, uint64_t dst_cap, uint64_t* out_len,
                             uint64_t rows_per_group, uint64_t* positions);
/* General run builder: run i encodes the next lengths[i] values with
 * kinds[i] (0 SHORT_REPEAT, 1 DIRECT, 2 PATCHED_BASE, 3 DELTA); fails with
 * ORCG_INVALID_ARGUMENT if the values are not representable that way.
 * run_offsets (optional, nruns entries) receives each run's byte offset. */
int orcg_rlev2_encode_runs(const int64_t* values, uint64_t n, int is_signed, const uint8_t* kinds,
                           const uint32_t* lengths, uint64_t nruns, uint8_t* dst, uint64_t dst_cap,
                           uint64_t* out_len, uint64_t* run_offsets);

/* (Roofline calibration copies, orcg_probe_copy, live only in the A/B build
 * liborcgpu_ab.so: orc_amd/csrc/probe_kernels.hip.) */

#ifdef __cplusplus
}
#endif
#endif /* ORCG_H */
