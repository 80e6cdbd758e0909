// C++ adapter: the reference's Reader / RowReader -> ColumnVectorBatch surface
// over the liborcgpu file reader (include/orcg_reader.h). Header-only; host
// code only.
//
// Reference interfaces mirrored (apache/orc):
//   orc::createReader, Reader::getNumberOfRows / getNumberOfStripes /
//     getType / getContentLength / getSoftwareVersion / getMetadataKeys /
//     getMetadataValue / createRowReader(RowReaderOptions)
//                                          c++/include/orc/Reader.hh:460-633
//   RowReaderOptions::include / range / setEnableLazyDecoding
//                                          c++/include/orc/Reader.hh:150-300
//   RowReader::createRowBatch(capacity) / next(batch) / getRowNumber /
//     seekToRow                            c++/include/orc/Reader.hh:754-776
//   ColumnVectorBatch family (capacity, numElements, notNull, hasNulls;
//   LongVectorBatch data, DoubleVectorBatch data, StringVectorBatch
//   data/length, EncodedStringVectorBatch index + dictionary,
//   Decimal64VectorBatch values/precision/scale, Decimal128VectorBatch values
//   (Int128 = {highbits, lowbits}), TimestampVectorBatch data / nanoseconds,
//   ListVectorBatch / MapVectorBatch offsets + children, StructVectorBatch
//   fields, UnionVectorBatch tags / offsets / children)
//                                          c++/include/orc/Vector.hh:46-352
//
// next() follows RowReaderImpl::next (c++/src/Reader.cc:1392-1442): at most
// capacity rows, never across a stripe. The GPU decodes a whole stripe into
// HBM once (host decompression, one H2D, HIP kernels); each batch copies its
// row range of every selected column into the batch's host buffers. String
// data pointers point into the batch's host copy of the string bytes (the
// dictionary, or the span of direct strings the batch covers). Inside the
// reference build these stand-in batch classes are the orc::*VectorBatch
// classes themselves (same member names).
#pragma once

#include <cstdint>
#include <cstring>
#include <limits>
#include <functional>
#include <list>
#include <map>
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
  ColumnVectorBatch(uint32_t kind_, uint64_t cap) : kind(kind_), capacity(cap) {}
  virtual ~ColumnVectorBatch() = default;
  uint32_t kind;  // orc::TypeKind
  uint64_t capacity;
  uint64_t numElements = 0;
  std::vector<char> notNull;
  bool hasNulls = false;
  bool isEncoded = false;
};
struct LongVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<int64_t> data;
};
// RowReaderOptions::setUseTightNumericVector batches (Vector.hh IntegerVectorBatch<T>,
// FloatingVectorBatch<float>): BOOLEAN / BYTE -> Byte, SHORT -> Short, INT ->
// Int, FLOAT -> Float (ColumnReader.cc:1703-1790)
struct IntVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<int32_t> data;
};
struct ShortVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<int16_t> data;
};
struct ByteVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<int8_t> data;
};
struct DoubleVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<double> data;
};
struct FloatVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<float> data;
};
struct StringVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<char*> data;
  std::vector<int64_t> length;
  std::vector<char> blob;  // host copy of the string bytes the batch points into
};
// orc::StringDictionary (Vector.hh:232-254)
struct StringDictionary {
  std::vector<char> dictionaryBlob;
  std::vector<int64_t> dictionaryOffset;
  void getValueByIndex(int64_t index, char*& valPtr, int64_t& length) {
    if (index < 0 || static_cast<uint64_t>(index) + 1 >= dictionaryOffset.size())
      throw std::out_of_range("index out of range.");
    valPtr = dictionaryBlob.data() + dictionaryOffset[index];
    length = dictionaryOffset[index + 1] - dictionaryOffset[index];
  }
};
// orc::EncodedStringVectorBatch (Vector.hh:256-269): with lazy decoding the
// dictionary columns fill index + dictionary only
struct EncodedStringVectorBatch : StringVectorBatch {
  using StringVectorBatch::StringVectorBatch;
  std::shared_ptr<StringDictionary> dictionary;
  std::vector<int64_t> index;
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
struct UnionVectorBatch : ColumnVectorBatch {
  using ColumnVectorBatch::ColumnVectorBatch;
  std::vector<unsigned char> tags;
  std::vector<uint64_t> offsets;
  std::vector<std::unique_ptr<ColumnVectorBatch>> children;
};

// orc::RowReaderOptions (the options the decode path honours)
class RowReaderOptions {
 public:
  RowReaderOptions& include(const std::list<uint64_t>& typeIds) {
    include_ = typeIds;
    hasInclude_ = true;
    return *this;
  }
  RowReaderOptions& range(uint64_t offset, uint64_t length) {
    offset_ = offset;
    length_ = length;
    return *this;
  }
  RowReaderOptions& setEnableLazyDecoding(bool on) {
    lazy_ = on;
    return *this;
  }
  RowReaderOptions& setUseTightNumericVector(bool on) {
    tight_ = on;
    return *this;
  }
  bool getUseTightNumericVector() const { return tight_; }
  uint64_t getOffset() const { return offset_; }
  uint64_t getLength() const { return length_; }
  bool getEnableLazyDecoding() const { return lazy_; }
  bool hasInclude() const { return hasInclude_; }
  const std::list<uint64_t>& getInclude() const { return include_; }

 private:
  std::list<uint64_t> include_;
  bool hasInclude_ = false;
  uint64_t offset_ = 0, length_ = std::numeric_limits<uint64_t>::max();
  bool lazy_ = false;
  bool tight_ = false;
};

class Reader;

class RowReader {
 public:
  RowReader(Reader& r, const RowReaderOptions& opts);
  ~RowReader() { orcg_row_reader_destroy(rr_); }
  RowReader(const RowReader&) = delete;
  RowReader& operator=(const RowReader&) = delete;
  std::unique_ptr<ColumnVectorBatch> createRowBatch(uint64_t capacity) const;
  bool next(ColumnVectorBatch& batch);
  uint64_t getRowNumber() const { return orcg_row_reader_row_number(rr_); }
  void seekToRow(uint64_t rowNumber);
  // RowReader::getSelectedColumns()[id]
  bool isSelected(uint32_t id) const { return orcg_row_reader_is_selected(rr_, id) != 0; }

 private:
  void fill(uint32_t id, ColumnVectorBatch& b);
  Reader& r_;
  orcg_row_reader* rr_ = nullptr;
  bool lazy_ = false;
  bool tight_ = false;
  // the current stripe's dictionaries, shared by its batches (lazy decoding:
  // StringDictionary; eager: the blob the batches' data pointers point into,
  // as the reference's batches point into the column reader's dictionary)
  uint64_t dict_stripe_ = ~0ull;
  std::map<uint32_t, std::shared_ptr<StringDictionary>> dicts_;
  std::map<uint32_t, std::shared_ptr<std::vector<char>>> blobs_;
  // per type: the children fill() visits (struct: the selected fields)
  std::vector<std::vector<uint32_t>> subs_;
  std::vector<uint8_t> subs_known_;
  const std::vector<uint32_t>& subs(uint32_t id, uint32_t kind);
  void new_stripe();
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
  uint64_t getContentLength() const { return orcg_reader_content_length(r_); }
  uint64_t getRowIndexStride() const { return orcg_reader_row_index_stride(r_); }
  std::string getSoftwareVersion() const { return orcg_reader_software_version(r_); }
  std::list<std::string> getMetadataKeys() const {
    std::list<std::string> keys;
    for (uint32_t i = 0; i < orcg_reader_num_metadata(r_); ++i) keys.push_back(orcg_reader_metadata_key(r_, i));
    return keys;
  }
  bool hasMetadataValue(const std::string& key) const {
    for (const auto& k : getMetadataKeys())
      if (k == key) return true;
    return false;
  }
  std::string getMetadataValue(const std::string& key) const {
    for (uint32_t i = 0; i < orcg_reader_num_metadata(r_); ++i)
      if (key == orcg_reader_metadata_key(r_, i)) {
        uint64_t n = 0;
        const uint8_t* p = orcg_reader_metadata_value(r_, i, &n);
        return std::string((const char*)p, n);
      }
    throw std::range_error("key not found");
  }
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
  // the selected children of a type (RowReader::getSelectedType's shape)
  std::vector<uint32_t> getSelectedSubtypes(uint32_t id) const {
    std::vector<uint32_t> out;
    for (uint32_t s : getSubtypes(id))
      if (orcg_reader_is_selected(r_, s)) out.push_back(s);
    return out;
  }
  std::vector<std::string> getSelectedFieldNames(uint32_t id) const {
    std::vector<std::string> out;
    const auto subs = getSubtypes(id);
    for (uint32_t i = 0; i < subs.size(); ++i)
      if (orcg_reader_is_selected(r_, subs[i])) out.push_back(getFieldName(id, i));
    return out;
  }
  std::unique_ptr<RowReader> createRowReader() { return createRowReader(RowReaderOptions()); }
  std::unique_ptr<RowReader> createRowReader(const RowReaderOptions& opts) {
    return std::make_unique<RowReader>(*this, opts);
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
  void copy(std::vector<T>& dst, const void* src, uint64_t count, uint64_t first = 0) {
    dst.resize(count);
    if (count) check(orcg_reader_copy_to_host(r_, dst.data(), (const T*)src + first, count * sizeof(T)));
  }
  // row reader views point into its pinned host slab: plain copies
  template <typename T>
  static void hcopy(std::vector<T>& dst, const void* src, uint64_t count, uint64_t first = 0) {
    dst.resize(count);
    if (count) memcpy(dst.data(), (const T*)src + first, count * sizeof(T));
  }

 private:
  Context& ctx_;
  orcg_reader* r_ = nullptr;
};

using Selected = std::function<bool(uint32_t)>;

inline std::unique_ptr<ColumnVectorBatch> make_batch(const Reader& r, uint32_t id, uint64_t cap, bool lazy,
                                                     const Selected& sel, bool tight = false) {
  const orcg_type_info t = r.getType(id);
  switch (t.kind) {
    case ORCG_TYPE_BOOLEAN:
    case ORCG_TYPE_BYTE:
      if (tight) return std::make_unique<ByteVectorBatch>(t.kind, cap);
      return std::make_unique<LongVectorBatch>(t.kind, cap);
    case ORCG_TYPE_SHORT:
      if (tight) return std::make_unique<ShortVectorBatch>(t.kind, cap);
      return std::make_unique<LongVectorBatch>(t.kind, cap);
    case ORCG_TYPE_INT:
      if (tight) return std::make_unique<IntVectorBatch>(t.kind, cap);
      return std::make_unique<LongVectorBatch>(t.kind, cap);
    case ORCG_TYPE_FLOAT:
      if (tight) return std::make_unique<FloatVectorBatch>(t.kind, cap);
      return std::make_unique<DoubleVectorBatch>(t.kind, cap);
    case ORCG_TYPE_DOUBLE: return std::make_unique<DoubleVectorBatch>(t.kind, cap);
    case ORCG_TYPE_STRING:
    case ORCG_TYPE_BINARY:
    case ORCG_TYPE_VARCHAR:
    case ORCG_TYPE_CHAR:
      // Type::createRowBatch: an encoded batch when lazy decoding is on
      if (lazy) return std::make_unique<EncodedStringVectorBatch>(t.kind, cap);
      return std::make_unique<StringVectorBatch>(t.kind, cap);
    case ORCG_TYPE_DECIMAL:
      if (t.precision > 18 || t.precision == 0) return std::make_unique<Decimal128VectorBatch>(t.kind, cap);
      return std::make_unique<Decimal64VectorBatch>(t.kind, cap);
    case ORCG_TYPE_TIMESTAMP:
    case ORCG_TYPE_TIMESTAMP_INSTANT: return std::make_unique<TimestampVectorBatch>(t.kind, cap);
    case ORCG_TYPE_LIST: {
      auto b = std::make_unique<ListVectorBatch>(t.kind, cap);
      b->elements = make_batch(r, r.getSubtypes(id)[0], cap, lazy, sel, tight);
      return b;
    }
    case ORCG_TYPE_MAP: {
      auto b = std::make_unique<MapVectorBatch>(t.kind, cap);
      const auto s = r.getSubtypes(id);
      b->keys = make_batch(r, s[0], cap, lazy, sel, tight);
      b->elements = make_batch(r, s[1], cap, lazy, sel, tight);
      return b;
    }
    case ORCG_TYPE_STRUCT: {
      // the selected fields only (Type::createRowBatch of the selected type)
      auto b = std::make_unique<StructVectorBatch>(t.kind, cap);
      for (uint32_t s : r.getSubtypes(id))
        if (sel(s)) b->fields.push_back(make_batch(r, s, cap, lazy, sel, tight));
      return b;
    }
    case ORCG_TYPE_UNION: {
      auto b = std::make_unique<UnionVectorBatch>(t.kind, cap);
      for (uint32_t s : r.getSubtypes(id)) b->children.push_back(make_batch(r, s, cap, lazy, sel, tight));
      return b;
    }
    default: return std::make_unique<LongVectorBatch>(t.kind, cap);
  }
}

inline RowReader::RowReader(Reader& r, const RowReaderOptions& opts)
    : r_(r), lazy_(opts.getEnableLazyDecoding()), tight_(opts.getUseTightNumericVector()) {
  std::vector<uint8_t> inc;
  orcg_row_reader_options o;
  memset(&o, 0, sizeof(o));
  o.offset = opts.getOffset();
  o.length = opts.getLength();
  o.lazy_dictionary = lazy_ ? 1 : 0;
  if (opts.hasInclude()) {
    // RowReaderOptions::include(list<uint64_t>) selects type ids
    const uint32_t nt = orcg_reader_num_types(r.get());
    inc.assign(nt, 0);
    for (uint64_t id : opts.getInclude())
      if (id < nt) inc[id] = 1;
    o.include = inc.data();
    o.include_len = nt;
  }
  r_.check(orcg_row_reader_create(r.get(), &o, &rr_));
}

inline std::unique_ptr<ColumnVectorBatch> RowReader::createRowBatch(uint64_t capacity) const {
  return make_batch(r_, 0, capacity, lazy_, [this](uint32_t id) { return isSelected(id); }, tight_);
}

inline bool RowReader::next(ColumnVectorBatch& batch) {
  uint64_t rows = 0;
  r_.check(orcg_row_reader_next(rr_, batch.capacity, &rows));
  batch.numElements = rows;
  if (rows == 0) return false;
  fill(0, batch);
  return true;
}

inline void RowReader::seekToRow(uint64_t rowNumber) { r_.check(orcg_row_reader_seek_to_row(rr_, rowNumber)); }

template <typename T, typename S>
inline void narrow_copy(std::vector<T>& dst, const void* src, uint64_t n, uint64_t first) {
  // static_cast<T> of the decoded values, as the reference's decoders narrow
  const S* p = (const S*)src + first;
  dst.resize(n);
  for (uint64_t i = 0; i < n; ++i) dst[i] = static_cast<T>(p[i]);
}

inline const std::vector<uint32_t>& RowReader::subs(uint32_t id, uint32_t kind) {
  if (subs_.empty()) {
    // sized once for every type: fill() holds a reference across its
    // recursive calls, so the outer vector never reallocates
    const uint32_t nt = orcg_reader_num_types(r_.get());
    subs_.resize(nt);
    subs_known_.assign(nt, 0);
  }
  if (id >= subs_.size()) throw InvalidArgument("type id " + std::to_string(id) + " out of range");
  if (!subs_known_[id]) {
    for (uint32_t s : r_.getSubtypes(id))
      if (kind != ORCG_TYPE_STRUCT || isSelected(s)) subs_[id].push_back(s);
    subs_known_[id] = 1;
  }
  return subs_[id];
}

inline void RowReader::new_stripe() {
  const uint64_t stripe = orcg_row_reader_stripe(rr_);
  if (stripe != dict_stripe_) {
    dicts_.clear();
    blobs_.clear();
    dict_stripe_ = stripe;
  }
}

inline void RowReader::fill(uint32_t id, ColumnVectorBatch& b) {
  orcg_column_view v;
  uint64_t first = 0, n = 0;
  r_.check(orcg_row_reader_column(rr_, id, &v, &first, &n));
  if (!v.decoded)  // TIMESTAMP of a non-UTC writer zone (include/orcg_reader.h)
    throw InvalidArgument("column " + std::to_string(id) + " is not decoded by the GPU reader");
  // the view points into the row reader's host slab: plain copies
  b.numElements = n;
  if (n > b.capacity) b.capacity = n;  // children grow like the reference's resize()
  b.hasNulls = v.has_nulls != 0;
  if (b.hasNulls) Reader::hcopy(b.notNull, v.not_null, n, first);
  else b.notNull.assign(n, 1);
  const std::vector<uint32_t>& subs = this->subs(id, v.kind);
  if (auto* l = dynamic_cast<LongVectorBatch*>(&b)) {
    Reader::hcopy(l->data, v.data, n, first);
  } else if (auto* i32 = dynamic_cast<IntVectorBatch*>(&b)) {
    narrow_copy<int32_t, int64_t>(i32->data, v.data, n, first);
  } else if (auto* i16 = dynamic_cast<ShortVectorBatch*>(&b)) {
    narrow_copy<int16_t, int64_t>(i16->data, v.data, n, first);
  } else if (auto* i8 = dynamic_cast<ByteVectorBatch*>(&b)) {
    narrow_copy<int8_t, int64_t>(i8->data, v.data, n, first);
  } else if (auto* d = dynamic_cast<DoubleVectorBatch*>(&b)) {
    Reader::hcopy(d->data, v.data, n, first);
  } else if (auto* f = dynamic_cast<FloatVectorBatch*>(&b)) {
    narrow_copy<float, double>(f->data, v.data, n, first);
  } else if (auto* e = dynamic_cast<EncodedStringVectorBatch*>(&b); e && v.index) {
    // nextEncoded: index + the stripe's dictionary (ColumnReader.cc:596-607),
    // one host dictionary per stripe shared by its batches
    e->isEncoded = true;
    Reader::hcopy(e->index, v.index, n, first);
    new_stripe();
    std::shared_ptr<StringDictionary>& dict = dicts_[id];
    if (!dict) {
      dict = std::make_shared<StringDictionary>();
      Reader::hcopy(dict->dictionaryBlob, v.blob, v.blob_len);
      Reader::hcopy(dict->dictionaryOffset, v.dict_offsets, v.dict_size + 1);
    }
    e->dictionary = dict;
    e->data.assign(n, nullptr);
    e->length.assign(n, 0);
    for (uint64_t i = 0; i < n; ++i)
      if (!b.hasNulls || b.notNull[i]) dict->getValueByIndex(e->index[i], e->data[i], e->length[i]);
  } else if (auto* s = dynamic_cast<StringVectorBatch*>(&b)) {
    const int64_t* start = (const int64_t*)v.data + first;  // the slab's (start, length) pairs
    Reader::hcopy(s->length, v.length, n, first);
    s->data.resize(n);
    if (v.index) {
      // dictionary: the stripe's blob, copied once and shared by its batches
      new_stripe();
      std::shared_ptr<std::vector<char>>& blob = blobs_[id];
      if (!blob) {
        blob = std::make_shared<std::vector<char>>();
        Reader::hcopy(*blob, v.blob, v.blob_len);
      }
      s->blob.clear();
      char* base = blob->data();
      for (uint64_t i = 0; i < n; ++i) s->data[i] = base + (s->length[i] > 0 ? start[i] : 0);
    } else {
      // direct: the byte span the batch covers
      uint64_t lo = ~0ull, hi = 0;
      for (uint64_t i = 0; i < n; ++i)
        if (s->length[i] > 0) {
          lo = std::min<uint64_t>(lo, (uint64_t)start[i]);
          hi = std::max<uint64_t>(hi, (uint64_t)(start[i] + s->length[i]));
        }
      if (lo == ~0ull) lo = hi = 0;
      Reader::hcopy(s->blob, v.blob, hi - lo, lo);
      for (uint64_t i = 0; i < n; ++i) s->data[i] = s->blob.data() + (s->length[i] > 0 ? start[i] - (int64_t)lo : 0);
    }
  } else if (auto* d64 = dynamic_cast<Decimal64VectorBatch*>(&b)) {
    const orcg_type_info t = r_.getType(id);
    d64->precision = (int32_t)t.precision;
    d64->scale = (int32_t)t.scale;
    Reader::hcopy(d64->values, v.data, n, first);
  } else if (auto* d128 = dynamic_cast<Decimal128VectorBatch*>(&b)) {
    const orcg_type_info t = r_.getType(id);
    d128->precision = (int32_t)t.precision;
    // Hive 0.11 decimals: the forced scale (DecimalHive11ColumnReader::next)
    d128->scale = t.precision == 0 ? (int32_t)orcg_reader_hive11_scale(r_.get()) : (int32_t)t.scale;
    Reader::hcopy(d128->values, v.data, n, first);  // [hi, lo] per value = Int128's layout
  } else if (auto* ts = dynamic_cast<TimestampVectorBatch*>(&b)) {
    Reader::hcopy(ts->data, v.data, n, first);
    Reader::hcopy(ts->nanoseconds, v.secondary, n, first);
  } else if (auto* lb = dynamic_cast<ListVectorBatch*>(&b)) {
    Reader::hcopy(lb->offsets, v.offsets, n + 1, first);
    const int64_t base = lb->offsets[0];
    for (auto& o : lb->offsets) o -= base;
    fill(subs[0], *lb->elements);
  } else if (auto* mb = dynamic_cast<MapVectorBatch*>(&b)) {
    Reader::hcopy(mb->offsets, v.offsets, n + 1, first);
    const int64_t base = mb->offsets[0];
    for (auto& o : mb->offsets) o -= base;
    fill(subs[0], *mb->keys);
    fill(subs[1], *mb->elements);
  } else if (auto* sb = dynamic_cast<StructVectorBatch*>(&b)) {
    for (size_t i = 0; i < subs.size(); ++i) fill(subs[i], *sb->fields[i]);
  } else if (auto* ub = dynamic_cast<UnionVectorBatch*>(&b)) {
    Reader::hcopy(ub->tags, v.tags, n, first);
    std::vector<int64_t> offs;
    Reader::hcopy(offs, v.offsets, n, first);
    // offsets relative to each child's first row in this batch
    std::vector<int64_t> base(subs.size(), -1);
    for (uint64_t i = 0; i < n; ++i)
      if ((!b.hasNulls || b.notNull[i]) && ub->tags[i] < subs.size() && base[ub->tags[i]] < 0)
        base[ub->tags[i]] = offs[i];
    ub->offsets.resize(n);
    for (uint64_t i = 0; i < n; ++i)
      ub->offsets[i] = (!b.hasNulls || b.notNull[i]) ? (uint64_t)(offs[i] - base[ub->tags[i]]) : 0;
    for (size_t k = 0; k < subs.size(); ++k) fill(subs[k], *ub->children[k]);
  }
}

}  // namespace cxx
}  // namespace orcg
