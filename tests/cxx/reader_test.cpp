// Reference-style host program over the C++ RowReader adapter
// (orc_amd/csrc/GpuRowReader.hh): reads every stripe of an ORC file through
// Reader / RowReader::next(ColumnVectorBatch&) the way orc-contents does
// (tools/src/FileContents.cc) and prints one JSON object per row, so the
// Python test can compare it with pyarrow's rows.
//
//   reader_test <file.orc>
#include <cmath>
#include <cstdio>
#include <string>

#include "../../orc_amd/csrc/GpuRowReader.hh"

using namespace orcg::cxx;

static std::string json_str(const char* p, int64_t n) {
  std::string s = "\"";
  for (int64_t i = 0; i < n; ++i) {
    const unsigned char c = (unsigned char)p[i];
    if (c == '"' || c == '\\') {
      s += '\\';
      s += (char)c;
    } else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      s += b;
    } else {
      s += (char)c;
    }
  }
  return s + "\"";
}

static std::string decimal_str(__int128 v, int32_t scale) {
  const bool neg = v < 0;
  unsigned __int128 m = neg ? (unsigned __int128)(-(v + 1)) + 1 : (unsigned __int128)v;
  std::string digits;
  do {
    digits.insert(digits.begin(), (char)('0' + (int)(m % 10)));
    m /= 10;
  } while (m);
  while ((int32_t)digits.size() <= scale) digits.insert(digits.begin(), '0');
  if (scale > 0) digits.insert(digits.end() - scale, '.');
  return "\"" + std::string(neg ? "-" : "") + digits + "\"";
}

static std::string value(const ColumnVectorBatch& b, uint64_t i) {
  if (b.hasNulls && !b.notNull[i]) return "null";
  if (auto* l = dynamic_cast<const LongVectorBatch*>(&b)) {
    if (b.kind == ORCG_TYPE_BOOLEAN) return l->data[i] ? "true" : "false";
    return std::to_string(l->data[i]);
  }
  if (auto* d = dynamic_cast<const DoubleVectorBatch*>(&b)) {
    if (std::isnan(d->data[i])) return "NaN";
    if (std::isinf(d->data[i])) return d->data[i] > 0 ? "Infinity" : "-Infinity";
    char buf[64];
    snprintf(buf, sizeof buf, "%.17g", d->data[i]);
    return buf;
  }
  if (auto* s = dynamic_cast<const StringVectorBatch*>(&b)) {
    if (b.kind == ORCG_TYPE_BINARY) {
      std::string r = "[";
      for (int64_t k = 0; k < s->length[i]; ++k)
        r += (k ? "," : "") + std::to_string((unsigned char)s->data[i][k]);
      return r + "]";
    }
    return json_str(s->data[i], s->length[i]);
  }
  if (auto* d64 = dynamic_cast<const Decimal64VectorBatch*>(&b)) return decimal_str(d64->values[i], d64->scale);
  if (auto* d128 = dynamic_cast<const Decimal128VectorBatch*>(&b)) {
    const Int128 x = d128->values[i];
    const __int128 v = (__int128)(((unsigned __int128)(uint64_t)x.highbits << 64) | x.lowbits);
    return decimal_str(v, d128->scale);
  }
  if (auto* t = dynamic_cast<const TimestampVectorBatch*>(&b))
    return "[" + std::to_string(t->data[i]) + "," + std::to_string(t->nanoseconds[i]) + "]";
  if (auto* lb = dynamic_cast<const ListVectorBatch*>(&b)) {
    std::string r = "[";
    for (int64_t k = lb->offsets[i]; k < lb->offsets[i + 1]; ++k)
      r += (k > lb->offsets[i] ? "," : "") + value(*lb->elements, (uint64_t)k);
    return r + "]";
  }
  if (auto* sb = dynamic_cast<const StructVectorBatch*>(&b)) {  // nested struct: its field values in order
    std::string r = "[";
    for (size_t f = 0; f < sb->fields.size(); ++f) r += (f ? "," : "") + value(*sb->fields[f], i);
    return r + "]";
  }
  if (auto* mb = dynamic_cast<const MapVectorBatch*>(&b)) {
    std::string r = "[";
    for (int64_t k = mb->offsets[i]; k < mb->offsets[i + 1]; ++k)
      r += std::string(k > mb->offsets[i] ? "," : "") + "[" + value(*mb->keys, (uint64_t)k) + "," +
           value(*mb->elements, (uint64_t)k) + "]";
    return r + "]";
  }
  return "null";
}

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s <file.orc>\n", argv[0]);
    return 2;
  }
  try {
    Context ctx(0);
    Reader reader(ctx, argv[1]);
    std::vector<std::string> names;
    const auto subs = reader.getSubtypes(0);
    for (size_t i = 0; i < subs.size(); ++i) names.push_back(reader.getFieldName(0, (uint32_t)i));
    auto rows = reader.createRowReader();
    auto batch = rows->createRowBatch();
    uint64_t total = 0;
    while (rows->next(*batch)) {
      const auto& root = dynamic_cast<const StructVectorBatch&>(*batch);
      for (uint64_t i = 0; i < batch->numElements; ++i) {
        std::string line = "{";
        for (size_t f = 0; f < names.size(); ++f)
          line += (f ? ", " : "") + json_str(names[f].data(), (int64_t)names[f].size()) + ": " +
                  value(*root.fields[f], i);
        puts((line + "}").c_str());
      }
      total += batch->numElements;
    }
    fprintf(stderr, "rows %llu\n", (unsigned long long)total);
    return total == reader.getNumberOfRows() ? 0 : 1;
  } catch (const std::exception& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
