// ORC file tail / stripe footer parsing and block decompression (host side).
//
// The file-level pieces the decoder needs to get from file bytes to stream
// bytes in HBM: the protobuf messages of the tail (PostScript, Footer,
// StripeInformation, Type; site/specification/ORCv1.md:76-270) and of the
// stripe footer (StripeFooter, Stream, ColumnEncoding; :940-1030), read
// with a small protobuf wire-format reader (the reference links libprotobuf
// and generated orc_proto classes; only the wire format is restated here),
// and ORC's chunked block compression (ORCv1.md:600-632; Compression.cc).
// Reading follows ReaderImpl (c++/src/Reader.cc:1517-1627, 1650-1700) and
// StripeStreamsImpl::getStream (c++/src/StripeStream.cc:82-125).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace orcg {
namespace file {

enum Compression { kNone = 0, kZlib = 1, kSnappy = 2, kLzo = 3, kLz4 = 4, kZstd = 5 };

struct PostScript {
  uint64_t footer_length = 0;
  uint32_t compression = kNone;
  uint64_t block_size = 256 * 1024;
  std::vector<uint32_t> version;
  uint64_t metadata_length = 0;
  uint32_t writer_version = 0;
  std::string magic;
};

struct StripeInfo {
  uint64_t offset = 0, index_length = 0, data_length = 0, footer_length = 0, num_rows = 0;
};

struct TypeInfo {
  uint32_t kind = 0;
  std::vector<uint32_t> subtypes;
  std::vector<std::string> field_names;
  uint32_t maximum_length = 0, precision = 0, scale = 0;
};

struct Footer {
  uint64_t header_length = 0, content_length = 0, num_rows = 0;
  std::vector<StripeInfo> stripes;
  std::vector<TypeInfo> types;
  uint32_t row_index_stride = 0;
  uint32_t writer = 0;          // Footer.writer (WriterId), ORC Java when absent
  bool has_software_version = false;
  std::string software_version;  // Footer.softwareVersion
  std::vector<std::pair<std::string, std::string>> metadata;  // Footer.metadata (UserMetadataItem name, value)
};

enum StreamKind {
  kPresent = 0,
  kData = 1,
  kLength = 2,
  kDictionaryData = 3,
  kDictionaryCount = 4,
  kSecondary = 5,
  kRowIndex = 6,
};

struct StreamInfo {
  uint32_t kind = 0, column = 0;
  uint64_t length = 0;
  uint64_t offset = 0;  // absolute file offset (sum of the preceding streams)
};

enum EncodingKind { kDirect = 0, kDictionary = 1, kDirectV2 = 2, kDictionaryV2 = 3 };

struct ColumnEncoding {
  uint32_t kind = kDirect;
  uint32_t dictionary_size = 0;
};

struct StripeFooter {
  std::vector<StreamInfo> streams;
  std::vector<ColumnEncoding> encodings;
  std::string writer_timezone;
};

// A compressed (or raw) byte range of the file split into its chunks.
struct Chunk {
  uint64_t src_off = 0, src_len = 0;  // file bytes of the chunk body
  bool original = true;               // stored uncompressed
  uint64_t dst_off = 0, dst_len = 0;  // output placement (dst_len filled by decompress)
};

bool parse_postscript(const uint8_t* p, uint64_t n, PostScript& ps);
bool parse_footer(const uint8_t* p, uint64_t n, Footer& f);
bool parse_stripe_footer(const uint8_t* p, uint64_t n, uint64_t stripe_offset, StripeFooter& sf);
// RowIndex (orc_proto.proto; ORCv1.md "Indexes"): the positions list of every
// RowIndexEntry, one per row group.
bool parse_row_index(const uint8_t* p, uint64_t n, std::vector<std::vector<uint64_t>>& entries);

// Split [off, off + len) of the file into compression chunks (3-byte
// headers); NONE yields one original chunk. False on a malformed header.
bool split_chunks(const uint8_t* file, uint64_t off, uint64_t len, uint32_t compression, std::vector<Chunk>& out,
                  std::string& err);
// Decompress one chunk into dst (capacity cap); sets c.dst_len.
bool decompress_chunk(uint32_t compression, const uint8_t* file, Chunk& c, uint8_t* dst, uint64_t cap,
                      std::string& err);
// Whole-range convenience (metadata: footers).
bool read_range(const uint8_t* file, uint64_t off, uint64_t len, uint32_t compression, uint64_t block_size,
                std::vector<uint8_t>& out, std::string& err);

const char* compression_name(uint32_t c);

}  // namespace file
}  // namespace orcg
