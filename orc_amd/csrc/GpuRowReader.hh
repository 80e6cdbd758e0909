// C++ adapter: the reference's Reader / RowReader -> ColumnVectorBatch surface
// over the liborcgpu file reader (include/orcg_reader.h). Header-only; host
// code only.
//
// Reference interfaces mirrored (apache/orc):
//   orc::createReader, Reader::getNumberOfRows / getNumberOfStripes / getType
//       c++/include/orc/OrcFile.hh, c++/include/orc/Reader.hh:460-633
//   RowReader::createRowBatch / next(ColumnVectorBatch&)  Reader.hh:754-764
//   ColumnVectorBatch family (numElements, notNull, hasNulls; LongVectorBatch
//   data, DoubleVectorBatch data, StringVectorBatch data/length,
//   Decimal64VectorBatch values/precision/scale, Decimal128VectorBatch
//   values (Int128 = {highbits, lowbits}), TimestampVectorBatch data /
//   nanoseconds, ListVectorBatch / MapVectorBatch offsets + children,
//   StructVectorBatch fields)                           c++/include/orc/Vector.hh:46-330
//
// Each next() decodes one stripe on the GPU (host decompression, one H2D,
// HIP kernels) and copies the selected columns into the batch's host
// buffers; string data pointers point into the batch's host copy of the
// stripe's string bytes (the reference's dictionary blob / direct blob).
// Inside the reference build these stand-in batch classes are the
// orc::*VectorBatch classes themselves (same member names).
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/orcg_reader.h"
#include "GpuRleDecoder.hh"

namespace orcg {
namespace cxx {

struct Int128 {  // orc::Int128 member order (c++/include/orc/Int128.hh:325-326)
  int64_t highbits = 0;
  uint64_t lowbits = 0;
};

struct ColumnVectorBatch {
  explicit ColumnVectorBatch(uint32_t kind_) : kind(kind_) {}
  virtual ~ColumnVectorBatch() = default;
  uint32_t kind;  // orc::TypeKind
  uint64_t numElements = 0;
  std::vector<char> notNull;
  bool hasNulls = false;
};
struct LongVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<int64_t> data;
};
struct DoubleVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<double> data;
};
struct StringVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<char*> data;
  std::vector<int64_t> length;
  std::vector<char> blob;  // host copy of the stripe's string bytes
};
struct Decimal64VectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  int32_t precision = 0, scale = 0;
  std::vector<int64_t> values;
};
struct Decimal128VectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  int32_t precision = 0, scale = 0;
  std::vector<Int128> values;
};
struct TimestampVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<int64_t> data, nanoseconds;
};
struct ListVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<int64_t> offsets;
  std::unique_ptr<ColumnVectorBatch> elements;
};
struct MapVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<int64_t> offsets;
  std::unique_ptr<ColumnVectorBatch> keys, elements;
};
struct StructVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<std::unique_ptr<ColumnVectorBatch>> fields;
};

class Reader;

// orc::RowReader: next() = the next stripe (RowReaderOptions::range selects
// stripes [first, last)).
class RowReader {
 public:
  RowReader(Reader& r, uint64_t first, uint64_t last) : r_(r), next_(first), last_(last) {}
  std::unique_ptr<ColumnVectorBatch> createRowBatch() const;
  bool next(ColumnVectorBatch& batch);

 private:
  void fill(uint32_t id, ColumnVectorBatch& b);
  Reader& r_;
  uint64_t next_, last_;
};

class Reader {
 public:
  Reader(Context& ctx, const std::string& path) : ctx_(ctx) {
    if (orcg_reader_open_file(ctx.get(), path.c_str(), &r_) != ORCG_OK) {
      const std::string m = orcg_reader_open_error();
      throw ParseError(m);
    }
  }
  ~Reader() { orcg_reader_destroy(r_); }
  Reader(const Reader&) = delete;
  Reader& operator=(const Reader&) = delete;
  uint64_t getNumberOfRows() const { return orcg_reader_num_rows(r_); }
  uint64_t getNumberOfStripes() const { return orcg_reader_num_stripes(r_); }
  orcg_type_info getType(uint32_t id) const {
    orcg_type_info t;
    check(orcg_reader_type(r_, id, &t));
    return t;
  }
  std::vector<uint32_t> getSubtypes(uint32_t id) const {
    std::vector<uint32_t> s(getType(id).num_subtypes);
    if (!s.empty()) check(orcg_reader_subtypes(r_, id, s.data(), (uint32_t)s.size()));
    return s;
  }
  std::string getFieldName(uint32_t id, uint32_t i) const { return orcg_reader_field_name(r_, id, i); }
  std::unique_ptr<RowReader> createRowReader() { return std::make_unique<RowReader>(*this, 0, getNumberOfStripes()); }
  std::unique_ptr<RowReader> createRowReader(uint64_t first_stripe, uint64_t last_stripe) {
    return std::make_unique<RowReader>(*this, first_stripe, last_stripe);
  }

  // internals for RowReader
  void check(int rc) const {
    if (rc != ORCG_OK) {
      const char* m = orcg_reader_last_error(r_);
      throwOnError(rc, m ? m : "orcg reader error");
    }
  }
  orcg_reader* get() const { return r_; }
  template <typename T>
  void copy(std::vector<T>& dst, const void* src, uint64_t count) {
    dst.resize(count);
    if (count) check(orcg_reader_copy_to_host(r_, dst.data(), src, count * sizeof(T)));
  }

 private:
  Context& ctx_;
  orcg_reader* r_ = nullptr;
};

inline std::unique_ptr<ColumnVectorBatch> make_batch(const Reader& r, uint32_t id) {
  const orcg_type_info t = r.getType(id);
  switch (t.kind) {
    case ORCG_TYPE_FLOAT:
    case ORCG_TYPE_DOUBLE: return std::make_unique<DoubleVectorBatch>(t.kind);
    case ORCG_TYPE_STRING:
    case ORCG_TYPE_BINARY:
    case ORCG_TYPE_VARCHAR:
    case ORCG_TYPE_CHAR: return std::make_unique<StringVectorBatch>(t.kind);
    case ORCG_TYPE_DECIMAL:
      if (t.precision > 18 || t.precision == 0) return std::make_unique<Decimal128VectorBatch>(t.kind);
      return std::make_unique<Decimal64VectorBatch>(t.kind);
    case ORCG_TYPE_TIMESTAMP:
    case ORCG_TYPE_TIMESTAMP_INSTANT: return std::make_unique<TimestampVectorBatch>(t.kind);
    case ORCG_TYPE_LIST: {
      auto b = std::make_unique<ListVectorBatch>(t.kind);
      b->elements = make_batch(r, r.getSubtypes(id)[0]);
      return b;
    }
    case ORCG_TYPE_MAP: {
      auto b = std::make_unique<MapVectorBatch>(t.kind);
      const auto s = r.getSubtypes(id);
      b->keys = make_batch(r, s[0]);
      b->elements = make_batch(r, s[1]);
      return b;
    }
    case ORCG_TYPE_STRUCT: {
      auto b = std::make_unique<StructVectorBatch>(t.kind);
      for (uint32_t s : r.getSubtypes(id)) b->fields.push_back(make_batch(r, s));
      return b;
    }
    default: return std::make_unique<LongVectorBatch>(t.kind);
  }
}

inline std::unique_ptr<ColumnVectorBatch> RowReader::createRowBatch() const { return make_batch(r_, 0); }

inline bool RowReader::next(ColumnVectorBatch& batch) {
  if (next_ >= last_) {
    batch.numElements = 0;
    return false;
  }
  r_.check(orcg_reader_read_stripe(r_.get(), next_));
  ++next_;
  fill(0, batch);
  return true;
}

inline void RowReader::fill(uint32_t id, ColumnVectorBatch& b) {
  orcg_column_view v;
  r_.check(orcg_reader_column(r_.get(), id, &v));
  if (!v.decoded) throw InvalidArgument("column " + std::to_string(id) + " is not decoded by the GPU reader");
  const uint64_t n = v.num_elements;
  b.numElements = n;
  b.hasNulls = v.has_nulls != 0;
  if (b.hasNulls) {
    r_.copy(b.notNull, v.not_null, n);
  } else {
    b.notNull.assign(n, 1);
  }
  const std::vector<uint32_t> subs = r_.getSubtypes(id);
  if (auto* l = dynamic_cast<LongVectorBatch*>(&b)) {
    r_.copy(l->data, v.data, n);
  } else if (auto* d = dynamic_cast<DoubleVectorBatch*>(&b)) {
    r_.copy(d->data, v.data, n);
  } else if (auto* s = dynamic_cast<StringVectorBatch*>(&b)) {
    std::vector<int64_t> start;
    r_.copy(start, v.data, n);
    r_.copy(s->length, v.length, n);
    r_.copy(s->blob, v.blob, v.blob_len);
    s->data.resize(n);
    for (uint64_t i = 0; i < n; ++i) s->data[i] = s->blob.data() + start[i];
  } else if (auto* d64 = dynamic_cast<Decimal64VectorBatch*>(&b)) {
    const orcg_type_info t = r_.getType(id);
    d64->precision = (int32_t)t.precision;
    d64->scale = (int32_t)t.scale;
    r_.copy(d64->values, v.data, n);
  } else if (auto* d128 = dynamic_cast<Decimal128VectorBatch*>(&b)) {
    const orcg_type_info t = r_.getType(id);
    d128->precision = (int32_t)t.precision;
    d128->scale = (int32_t)t.scale;
    r_.copy(d128->values, v.data, n);  // [hi, lo] per value = Int128's layout
  } else if (auto* ts = dynamic_cast<TimestampVectorBatch*>(&b)) {
    r_.copy(ts->data, v.data, n);
    r_.copy(ts->nanoseconds, v.secondary, n);
  } else if (auto* lb = dynamic_cast<ListVectorBatch*>(&b)) {
    r_.copy(lb->offsets, v.offsets, n + 1);
    fill(subs[0], *lb->elements);
  } else if (auto* mb = dynamic_cast<MapVectorBatch*>(&b)) {
    r_.copy(mb->offsets, v.offsets, n + 1);
    fill(subs[0], *mb->keys);
    fill(subs[1], *mb->elements);
  } else if (auto* sb = dynamic_cast<StructVectorBatch*>(&b)) {
    for (size_t i = 0; i < subs.size(); ++i) fill(subs[i], *sb->fields[i]);
  }
}

}  // namespace cxx
}  // namespace orcg
