/*
 * orcg_reader.h — file-level C ABI of liborcgpu: ORC file bytes -> decoded
 * column batches in HBM (and, on request, in host memory).
 *
 * Mirrors the reference's reader surface for the decode path:
 *   orc::createReader / ReaderImpl            c++/include/orc/OrcFile.hh, c++/src/Reader.cc:1517-1700
 *   Reader::getNumberOfRows/Stripes, getType  c++/include/orc/Reader.hh:460,529,620
 *   RowReader::next(ColumnVectorBatch&)       c++/include/orc/Reader.hh:764 (one stripe per call here)
 *   ColumnVectorBatch family                  c++/include/orc/Vector.hh:46-330
 *   column readers (PRESENT / DATA / LENGTH / DICTIONARY_DATA per type)
 *                                             c++/src/ColumnReader.cc:81-1160
 *
 * The host parses the tail and stripe footers and decompresses streams
 * (zlib / snappy / lz4 / zstd stay on the CPU, as in the reference, which
 * links those libraries); one H2D copy per stripe moves the stream bytes to
 * HBM, where every integer, boolean, byte, length and dictionary stream is
 * decoded by the HIP kernels of orcg.h. Batch layout per column (type id):
 *   not_null : char[n], 1 = value present (NULL when the column has no nulls)
 *   BOOLEAN, BYTE, SHORT, INT, LONG, DATE : int64 data[n]  (LongVectorBatch)
 *   FLOAT, DOUBLE                         : double data[n] (DoubleVectorBatch)
 *   STRING, VARCHAR, CHAR, BINARY         : int64 start[n] (blob-relative), int64 length[n],
 *                                           blob = DATA (direct) or DICTIONARY_DATA bytes
 *   DECIMAL, precision <= 18              : int64 data[n], unscaled at the type's scale
 *                                           (Decimal64VectorBatch::values)
 *   DECIMAL, precision > 18               : int64 data[2n], [hi, lo] per value (orc::Int128 layout,
 *                                           Decimal128VectorBatch::values)
 *   DECIMAL, precision 0 (Hive 0.11)      : as precision > 18, at orcg_reader_hive11_scale()
 *   TIMESTAMP, TIMESTAMP_INSTANT          : int64 data[n] seconds (UTC), int64 secondary[n] nanoseconds
 *                                           (TimestampVectorBatch::data / nanoseconds)
 *   LIST, MAP                             : int64 offsets[n + 1] (ListVectorBatch::offsets);
 *                                           children hold offsets[n] rows
 *   STRUCT                                : not_null only; children hold n rows
 *   UNION                                 : uint8 tags[n], int64 offsets[n] (UnionVectorBatch::tags /
 *                                           offsets: the row's index in child tags[i])
 * Dictionary-encoded strings also expose int64 index[n] (the entry of each
 * row, EncodedStringVectorBatch::index) and int64 dict_offsets[dict_size + 1]
 * into blob (StringDictionary::dictionaryOffset); with lazy dictionary
 * decoding (orcg_reader_set_lazy_dictionary, RowReaderOptions::
 * setEnableLazyDecoding) only those are produced (data / length are NULL).
 * Null slots hold 0 (the reference leaves them unspecified). Not decoded
 * (view.decoded == 0): TIMESTAMP columns
 * whose writer time zone is not UTC (the reference converts those with the
 * IANA zone rules, Timezone.cc).
 */
#ifndef ORCG_READER_H
#define ORCG_READER_H

#include "orcg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Type.Kind (ORCv1.md "Type Information") */
enum {
  ORCG_TYPE_BOOLEAN = 0, ORCG_TYPE_BYTE = 1, ORCG_TYPE_SHORT = 2, ORCG_TYPE_INT = 3, ORCG_TYPE_LONG = 4,
  ORCG_TYPE_FLOAT = 5, ORCG_TYPE_DOUBLE = 6, ORCG_TYPE_STRING = 7, ORCG_TYPE_BINARY = 8,
  ORCG_TYPE_TIMESTAMP = 9, ORCG_TYPE_LIST = 10, ORCG_TYPE_MAP = 11, ORCG_TYPE_STRUCT = 12,
  ORCG_TYPE_UNION = 13, ORCG_TYPE_DECIMAL = 14, ORCG_TYPE_DATE = 15, ORCG_TYPE_VARCHAR = 16,
  ORCG_TYPE_CHAR = 17, ORCG_TYPE_TIMESTAMP_INSTANT = 18
};
/* CompressionKind */
enum { ORCG_COMPRESSION_NONE = 0, ORCG_COMPRESSION_ZLIB = 1, ORCG_COMPRESSION_SNAPPY = 2,
       ORCG_COMPRESSION_LZO = 3, ORCG_COMPRESSION_LZ4 = 4, ORCG_COMPRESSION_ZSTD = 5 };

typedef struct orcg_reader orcg_reader;

typedef struct {
  uint32_t kind;
  uint32_t num_subtypes;
  uint32_t maximum_length;
  uint32_t precision;
  uint32_t scale;
} orcg_type_info;

typedef struct {
  uint64_t offset, index_length, data_length, footer_length, num_rows;
} orcg_stripe_info;

typedef struct {
  uint32_t type_id;
  uint32_t kind;          /* ORCG_TYPE_* */
  uint32_t encoding;      /* ColumnEncoding.Kind of this stripe (DIRECT=0 .. DICTIONARY_V2=3) */
  uint32_t decoded;       /* 1 if the column was decoded */
  uint64_t num_elements;
  int has_nulls;
  const uint8_t* not_null; /* device */
  const void* data;        /* device: int64 / double / int64 starts */
  const int64_t* length;   /* device: string lengths */
  const int64_t* offsets;  /* device: list / map offsets (n + 1) */
  const uint8_t* blob;     /* device: string bytes */
  uint64_t blob_len;
  const int64_t* secondary; /* device: TIMESTAMP nanoseconds (TimestampVectorBatch::nanoseconds) */
  const uint8_t* tags;      /* device: UNION child per row */
  const int64_t* index;     /* device: dictionary entry per row (dictionary-encoded strings) */
  const int64_t* dict_offsets; /* device: dict_size + 1 entry offsets into blob */
  uint64_t dict_size;
} orcg_column_view;

/* Open an ORC file held in host memory (the caller keeps `file` alive until
 * orcg_reader_destroy) or on disk (memory-mapped). Parses PostScript and
 * Footer; raises the reference's ParseError texts ("File size too small",
 * "Invalid ORC postscript length", "Not an ORC file", ...). `ctx` may be
 * NULL for metadata-only use (no GPU needed until a stripe is read). */
int orcg_reader_open(orcg_ctx* ctx, const uint8_t* file, uint64_t file_len, orcg_reader** out);
int orcg_reader_open_file(orcg_ctx* ctx, const char* path, orcg_reader** out);
/* Message of this thread's last failed open (also in ctx's last error). */
const char* orcg_reader_open_error(void);
void orcg_reader_destroy(orcg_reader* r);
const char* orcg_reader_last_error(const orcg_reader* r);

uint64_t orcg_reader_num_rows(const orcg_reader* r);
uint64_t orcg_reader_num_stripes(const orcg_reader* r);
uint32_t orcg_reader_row_index_stride(const orcg_reader* r);
uint32_t orcg_reader_compression(const orcg_reader* r);
uint64_t orcg_reader_compression_block_size(const orcg_reader* r);
/* file version [major, minor] (PostScript.version) */
int orcg_reader_format_version(const orcg_reader* r, uint32_t* major, uint32_t* minor);
uint32_t orcg_reader_writer_version(const orcg_reader* r);
/* Footer.contentLength (Reader::getContentLength, Reader.cc:755) */
uint64_t orcg_reader_content_length(const orcg_reader* r);
/* Reader::getSoftwareVersion (Reader.cc:742-749): writer id name, then the
 * footer's softwareVersion when present ("ORC Java", "ORC C++ 1.8.0", ...) */
const char* orcg_reader_software_version(const orcg_reader* r);
/* User metadata (Reader::getMetadataKeys / getMetadataValue, Reader.cc:783-798):
 * key i and its value bytes (NULL past the end). */
uint32_t orcg_reader_num_metadata(const orcg_reader* r);
const char* orcg_reader_metadata_key(const orcg_reader* r, uint32_t i);
const uint8_t* orcg_reader_metadata_value(const orcg_reader* r, uint32_t i, uint64_t* len);
uint32_t orcg_reader_num_types(const orcg_reader* r);
int orcg_reader_type(const orcg_reader* r, uint32_t type_id, orcg_type_info* out);
int orcg_reader_subtypes(const orcg_reader* r, uint32_t type_id, uint32_t* out, uint32_t cap);
const char* orcg_reader_field_name(const orcg_reader* r, uint32_t type_id, uint32_t i);
int orcg_reader_stripe(const orcg_reader* r, uint64_t stripe, orcg_stripe_info* out);

/* Column selection by type id (RowReaderOptions::include; NULL = all). A
 * selected column's ancestors are read too. */
int orcg_reader_select(orcg_reader* r, const uint8_t* include, uint32_t ntypes);
/* 1 if the type id is read under the current selection (RowReader::getSelectedColumns) */
int orcg_reader_is_selected(const orcg_reader* r, uint32_t type_id);
/* RowReaderOptions::setEnableLazyDecoding: dictionary string columns decode to
 * index + dictionary only (StringDictionaryColumnReader::nextEncoded). */
int orcg_reader_set_lazy_dictionary(orcg_reader* r, int on);
/* RowReaderOptions::forcedScaleOnHive11Decimal / throwOnHive11DecimalOverflow
 * (c++/include/orc/Reader.hh:258-271): Hive 0.11 decimals (precision 0) decode
 * as Decimal128 [hi, lo] values at forced_scale (default 6); a value past 38
 * digits raises "Hive 0.11 decimal was more than 38 digits." Only
 * throw_on_overflow = 1 (the reference's default) is supported. */
int orcg_reader_set_hive11_decimal(orcg_reader* r, int32_t forced_scale, int throw_on_overflow);
int32_t orcg_reader_hive11_scale(const orcg_reader* r);

/* Decode one stripe of the selected columns into device batches owned by the
 * reader (valid until the next read or destroy). Synchronous. */
int orcg_reader_read_stripe(orcg_reader* r, uint64_t stripe);
int orcg_reader_column(const orcg_reader* r, uint32_t type_id, orcg_column_view* out);
/* Stripes [first, first + count) into HBM, all kept resident: the host
 * decompresses and plans stripe i + 1 on a worker thread while the GPU
 * decodes stripe i. orcg_reader_stripe_column(r, k, ...) views the k-th. */
int orcg_reader_read_stripes(orcg_reader* r, uint64_t first, uint64_t count);
int orcg_reader_stripe_column(const orcg_reader* r, uint64_t k, uint32_t type_id, orcg_column_view* out);
/* Measurement helper (no reference counterpart): prepare stripe `stripe`
 * once (host decompression, plans), then decode it `iters` times back to
 * back; *decode_s / *h2d_s = average device-decode / upload seconds per
 * decode. Separates kernel time from the idle gaps of a host-bound read. */
int orcg_reader_bench_stripe_decode(orcg_reader* r, uint64_t stripe, uint32_t iters, double* decode_s,
                                    double* h2d_s);

/* ---- RowReader (c++/include/orc/Reader.hh:640-790; c++/src/Reader.cc
 * RowReaderImpl) over the GPU stripe decode. Batches hold at most `capacity`
 * rows and never span two stripes (RowReaderImpl::next, Reader.cc:1402-1403).
 * Each stripe is decoded in HBM and copied once into a pinned host slab owned
 * by the row reader; a worker thread decodes stripe s + 1 (and decompresses
 * s + 2) while the caller reads stripe s (startNextStripe's prefetch,
 * Reader.cc:1336-1360), so next() waits only for the slab of a new stripe.
 * Per column, orcg_row_reader_column gives the stripe's column view with
 * HOST pointers into that slab (valid until the next orcg_row_reader_next /
 * seek / destroy) plus the element range [begin, begin + count) of the batch
 * (through list / map offsets and union tags). In a row reader's views a
 * dictionary-encoded string column has index + dict_offsets + blob only
 * (data / length NULL, as with lazy decoding): the slab carries 8 bytes a row
 * instead of 24, and the caller looks each row up in the dictionary
 * (StringDictionaryColumnReader::next, ColumnReader.cc:561-594). A row
 * reader keeps its own
 * RowReaderOptions (include, lazy decoding) and device memory; it borrows
 * the reader (destroy row readers first), whose decodes it takes turns with. */
typedef struct orcg_row_reader orcg_row_reader;
typedef struct {
  uint64_t offset, length;   /* RowReaderOptions::range: stripes whose offset lies in [offset, offset + length) */
  const uint8_t* include;    /* RowReaderOptions::include by type id (NULL = every column) */
  uint32_t include_len;
  int lazy_dictionary;       /* RowReaderOptions::setEnableLazyDecoding */
} orcg_row_reader_options;
/* opts NULL = the whole file, every column */
int orcg_row_reader_create(orcg_reader* r, const orcg_row_reader_options* opts, orcg_row_reader** out);
void orcg_row_reader_destroy(orcg_row_reader* rr);
/* 1 if the type id is read by this row reader (RowReader::getSelectedColumns) */
int orcg_row_reader_is_selected(const orcg_row_reader* rr, uint32_t type_id);
/* RowReader::next: *rows = rows in the new batch (0 at the end) */
int orcg_row_reader_next(orcg_row_reader* rr, uint64_t capacity, uint64_t* rows);
/* RowReader::getRowNumber: first row of the last batch (UINT64_MAX before the first) */
uint64_t orcg_row_reader_row_number(const orcg_row_reader* rr);
/* stripe of the last batch (UINT64_MAX before the first) */
uint64_t orcg_row_reader_stripe(const orcg_row_reader* rr);
/* RowReader::seekToRow: the next batch starts at `row` */
int orcg_row_reader_seek_to_row(orcg_row_reader* rr, uint64_t row);
/* this row reader's last failure (a prefetched stripe's error, surfaced by
 * next / seek); the reader's orcg_reader_last_error also carries it, but is
 * shared with every row reader of that reader */
const char* orcg_row_reader_last_error(const orcg_row_reader* rr);
// Seconds this row reader spent so far: out6[0] host preparation (decompression)
// inside a stripe's decode job, [1] upload + GPU decode, [2] D2H into the
// pinned slab, [3] slab allocation, [4] look-ahead preparation of the next
// stripe (worker thread); [5] the caller's waits for a stripe's slab in
// next() / seekToRow(). Diagnostics; no reference counterpart.
int orcg_row_reader_timings(orcg_row_reader* rr, double* out6);
/* the last batch's view of column type_id (host pointers, see above) */
int orcg_row_reader_column(const orcg_row_reader* rr, uint32_t type_id, orcg_column_view* view, uint64_t* begin,
                           uint64_t* count);

/* Device -> host copy on the reader's context stream (synchronous). */
int orcg_reader_copy_to_host(orcg_reader* r, void* host_dst, const void* device_src, uint64_t bytes);

/* Time split of the last read, in seconds, summed over its stripes:
 * [0] stripe footer + chunk split, [1] decompression, [2] run plans (host
 * threads), [3] H2D, [4] device decode. With read_stripes, [0..2] of
 * stripe i + 1 overlap [3..4] of stripe i. */
int orcg_reader_last_timings(const orcg_reader* r, double* out5);
/* RLE streams of the last read cut at row groups by the ROW_INDEX positions
 * (ColumnReader::seekToRowGroup's PositionProvider, no host work) [0] and by
 * a host header walk (files without a row index) [1]. */
int orcg_reader_last_stream_stats(const orcg_reader* r, uint64_t* out2);
/* ReaderMetrics (c++/include/orc/Reader.hh:59-76; ReaderOptions::setReaderMetrics),
 * accumulated over the reader's life by every decode (read_stripe,
 * read_stripes, row readers). One "reader call" / "I/O" is one stripe read
 * (its byte range of the file); decompression counts compression chunks and
 * their host time; decoding counts RLE streams (RLEv1 / RLEv2 launches and
 * multi-stream jobs) with the device decode phase as its latency; byte decoding
 * counts byte / boolean RLE streams, whose kernels run inside that phase (their
 * latency is not split out: 0). Row groups: selected = the decoded stripes'
 * row groups (no search arguments, so evaluated stays 0), as do the read-range
 * cache counters. */
typedef struct orcg_reader_metrics {
  uint64_t reader_call;
  uint64_t reader_inclusive_latency_us;
  uint64_t decompression_call;
  uint64_t decompression_latency_us;
  uint64_t decoding_call;
  uint64_t decoding_latency_us;
  uint64_t byte_decoding_call;
  uint64_t byte_decoding_latency_us;
  uint64_t io_count;
  uint64_t io_blocking_latency_us;
  uint64_t selected_row_group_count;
  uint64_t evaluated_row_group_count;
  uint64_t read_range_cache_hits;
  uint64_t read_range_cache_misses;
} orcg_reader_metrics;
/* Semantics (ReaderMetrics, c++/include/orc/Reader.hh:59-76; the reference
 * fills them only when built with BUILD_CPP_ENABLE_METRICS):
 *  - ReaderCall / ReaderInclusiveLatencyUs: per caller-facing call
 *    (orcg_reader_read_stripe[s], orcg_row_reader_next), as the reference
 *    times RowReaderImpl::next (Reader.cc:1393); a row reader's prefetch
 *    decodes run inside them or ahead of them;
 *  - DecompressionCall / DecompressionLatencyUs: chunks inflated and host time;
 *  - DecodingCall / ByteDecodingCall: integer-RLE / byte-RLE streams decoded
 *    (one stream decode = one call, the reference counts next() calls);
 *  - DecodingLatencyUs / ByteDecodingLatencyUs: with metrics timing on
 *    (orcg_reader_set_metrics_timing), device time of the integer-RLE and
 *    byte-RLE launches from HIP events; off: DecodingLatencyUs is each
 *    stripe's device decode phase and ByteDecodingLatencyUs stays 0;
 *  - IOCount / IOBlockingLatencyUs: stream reads and their page-in time (the
 *    file is mapped; the reference preads each stream);
 *  - Selected/EvaluatedRowGroupCount: 0 (no search arguments), as the
 *    reference without SargsApplier; ReadRangeCacheHits/Misses: 0 (no
 *    read-range cache). */
int orcg_reader_get_metrics(orcg_reader* r, orcg_reader_metrics* out);
int orcg_reader_reset_metrics(orcg_reader* r);
int orcg_reader_set_metrics_timing(orcg_reader* r, int on);
/* RLEv2 streams of the last read decoded by a stripe's multi-stream launches
 * (every stream whose value count is known on the host: one launch per
 * kernel instance per stripe instead of one per stream). */
uint64_t orcg_reader_last_batched_streams(const orcg_reader* r);
/* Bytes the last read uploaded: decompressed stream bytes plus row-index /
 * plan tables, summed over its stripes. */
uint64_t orcg_reader_last_stage_bytes(const orcg_reader* r);
/* Multi-stream batching on (default) / off (one launch per stream; A/B). */
int orcg_reader_set_stream_batching(orcg_reader* r, int on);

#ifdef __cplusplus
}
#endif
#endif /* ORCG_READER_H */
