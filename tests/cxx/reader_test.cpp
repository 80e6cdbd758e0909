// Reference-style host program over the C++ RowReader adapter
// (orc_amd/csrc/GpuRowReader.hh): reads an ORC file through Reader /
// RowReader::next(ColumnVectorBatch&) the way tools/test/TestMatch.cc
// (Contents) and orc-contents (tools/src/FileContents.cc) do, printing one
// row per line in the reference ColumnPrinter's JSON shape
// (c++/src/ColumnPrinter.cc) so the Python test can compare every line with
// examples/expected/*.jsn.gz.
//
//   reader_test <file.orc> [--batch N] [--seek r1,r2,...] [--range OFF LEN] [--lazy] [--tight] [--bench] [--include id,...]
//
// --seek: for each row r, seekToRow(r) then one next(); prints "#seek r <getRowNumber>"
//         before the batch's rows.
// Every batch is checked against the contract: numElements <= capacity and
// getRowNumber() == the batch's first row; the program exits non-zero when
// it is broken or when the rows read differ from the file's row count.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <ctime>
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

// DecimalColumnPrinter: every scale digit, no quotes
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
  return std::string(neg ? "-" : "") + digits;
}

// DateColumnPrinter: days since the epoch -> "YYYY-MM-DD" (proleptic Gregorian)
static std::string date_str(int64_t days) {
  int64_t z = days + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t y = yoe + era * 400;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  const int64_t d = doy - (153 * mp + 2) / 5 + 1;
  const int64_t mo = mp < 10 ? mp + 3 : mp - 9;
  if (mo <= 2) ++y;
  char b[32];
  snprintf(b, sizeof b, "\"%04lld-%02lld-%02lld\"", (long long)y, (long long)mo, (long long)d);
  return b;
}

// TimestampColumnPrinter (ColumnPrinter.cc:668-700)
static std::string timestamp_str(int64_t secs, int64_t nanos) {
  time_t t = (time_t)secs;
  struct tm tmv;
  gmtime_r(&t, &tmv);
  char buf[32];
  strftime(buf, sizeof buf, "%Y-%m-%d %H:%M:%S", &tmv);
  int zero = 0;
  if (nanos == 0) zero = 8;
  else
    while (nanos % 10 == 0) {
      nanos /= 10;
      ++zero;
    }
  const std::string num = std::to_string(nanos);
  std::string r = std::string("\"") + buf + ".";
  for (int i = 0; i < 9 - zero - (int)num.size(); ++i) r += '0';
  return r + num + "\"";
}

static std::string value(const ColumnVectorBatch& b, uint64_t i, const std::vector<std::string>* names = nullptr);

static std::string value(const ColumnVectorBatch& b, uint64_t i, const std::vector<std::string>* names) {
  if (b.hasNulls && !b.notNull[i]) return "null";
  if (auto* l = dynamic_cast<const LongVectorBatch*>(&b)) {
    if (b.kind == ORCG_TYPE_BOOLEAN) return l->data[i] ? "true" : "false";
    if (b.kind == ORCG_TYPE_DATE) return date_str(l->data[i]);
    return std::to_string(l->data[i]);
  }
  // setUseTightNumericVector batches print as their wide counterparts
  if (auto* x = dynamic_cast<const IntVectorBatch*>(&b)) return std::to_string(x->data[i]);
  if (auto* x = dynamic_cast<const ShortVectorBatch*>(&b)) return std::to_string(x->data[i]);
  if (auto* x = dynamic_cast<const ByteVectorBatch*>(&b)) {
    if (b.kind == ORCG_TYPE_BOOLEAN) return x->data[i] ? "true" : "false";
    return std::to_string(x->data[i]);
  }
  const DoubleVectorBatch* dv = dynamic_cast<const DoubleVectorBatch*>(&b);
  const FloatVectorBatch* fv = dynamic_cast<const FloatVectorBatch*>(&b);
  if (dv || fv) {
    const double x = dv ? dv->data[i] : (double)fv->data[i];
    if (std::isnan(x)) return "NaN";
    if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
    // DoubleColumnPrinter (ColumnPrinter.cc:345-353): %.7g for FLOAT, %.14g for DOUBLE
    char buf[64];
    snprintf(buf, sizeof buf, b.kind == ORCG_TYPE_FLOAT ? "%.7g" : "%.14g", x);
    return buf;
  }
  if (auto* s = dynamic_cast<const StringVectorBatch*>(&b)) {
    if (b.kind == ORCG_TYPE_BINARY) {
      std::string r = "[";
      for (int64_t k = 0; k < s->length[i]; ++k)
        r += (k ? ", " : "") + std::to_string((unsigned char)s->data[i][k]);
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
  if (auto* t = dynamic_cast<const TimestampVectorBatch*>(&b)) return timestamp_str(t->data[i], t->nanoseconds[i]);
  if (auto* lb = dynamic_cast<const ListVectorBatch*>(&b)) {
    std::string r = "[";
    for (int64_t k = lb->offsets[i]; k < lb->offsets[i + 1]; ++k)
      r += (k > lb->offsets[i] ? ", " : "") + value(*lb->elements, (uint64_t)k);
    return r + "]";
  }
  if (auto* mb = dynamic_cast<const MapVectorBatch*>(&b)) {
    std::string r = "[";
    for (int64_t k = mb->offsets[i]; k < mb->offsets[i + 1]; ++k)
      r += std::string(k > mb->offsets[i] ? ", " : "") + "{\"key\": " + value(*mb->keys, (uint64_t)k) +
           ", \"value\": " + value(*mb->elements, (uint64_t)k) + "}";
    return r + "]";
  }
  if (auto* ub = dynamic_cast<const UnionVectorBatch*>(&b)) {
    const unsigned tag = ub->tags[i];
    return "{\"tag\": " + std::to_string(tag) + ", \"value\": " + value(*ub->children[tag], ub->offsets[i]) + "}";
  }
  if (auto* sb = dynamic_cast<const StructVectorBatch*>(&b)) {
    std::string r = "{";
    for (size_t f = 0; f < sb->fields.size(); ++f) {
      const std::string nm = names ? (*names)[f] : "f" + std::to_string(f);
      r += (f ? ", " : "") + json_str(nm.data(), (int64_t)nm.size()) + ": " + value(*sb->fields[f], i);
    }
    return r + "}";
  }
  return "null";
}

// Every batch of the tree: notNull covers numElements rows and, when the
// batch has no nulls, holds only 1s (the reference's ColumnReader::next
// leaves the decoded all-ones PRESENT mask there).
static bool not_null_ok(const ColumnVectorBatch& b) {
  if (b.notNull.size() < b.numElements) return false;
  if (!b.hasNulls)
    for (uint64_t i = 0; i < b.numElements; ++i)
      if (b.notNull[i] != 1) return false;
  if (auto* lb = dynamic_cast<const ListVectorBatch*>(&b)) return not_null_ok(*lb->elements);
  if (auto* mb = dynamic_cast<const MapVectorBatch*>(&b)) return not_null_ok(*mb->keys) && not_null_ok(*mb->elements);
  if (auto* sb = dynamic_cast<const StructVectorBatch*>(&b)) {
    for (const auto& f : sb->fields)
      if (!not_null_ok(*f)) return false;
  }
  if (auto* ub = dynamic_cast<const UnionVectorBatch*>(&b)) {
    for (const auto& c : ub->children)
      if (!not_null_ok(*c)) return false;
  }
  return true;
}

static const RowReader* g_rows = nullptr;  // the row reader's selection (RowReader::getSelectedColumns)

// the children a batch holds: a struct's selected fields, every other child
static std::vector<uint32_t> batch_subs(const Reader& r, uint32_t id) {
  std::vector<uint32_t> out;
  for (uint32_t s : r.getSubtypes(id))
    if (r.getType(id).kind != ORCG_TYPE_STRUCT || g_rows->isSelected(s)) out.push_back(s);
  return out;
}

// selected field names of every struct in the type tree, by type id
static void names_of(const Reader& r, uint32_t id, std::vector<std::vector<std::string>>& out) {
  if (r.getType(id).kind == ORCG_TYPE_STRUCT) {
    const auto subs = r.getSubtypes(id);
    for (uint32_t i = 0; i < subs.size(); ++i)
      if (g_rows->isSelected(subs[i])) out[id].push_back(r.getFieldName(id, i));
  }
  for (uint32_t s : r.getSubtypes(id)) names_of(r, s, out);
}

static std::vector<std::vector<std::string>> g_names;

// value() with nested struct field names (walks the batch tree alongside the type tree)
static std::string row(const Reader& r, uint32_t id, const ColumnVectorBatch& b, uint64_t i) {
  if (b.hasNulls && !b.notNull[i]) return "null";
  const auto subs = batch_subs(r, id);
  if (auto* sb = dynamic_cast<const StructVectorBatch*>(&b)) {
    std::string s = "{";
    for (size_t f = 0; f < sb->fields.size(); ++f) {
      const std::string& nm = g_names[id][f];
      s += (f ? ", " : "") + json_str(nm.data(), (int64_t)nm.size()) + ": " + row(r, subs[f], *sb->fields[f], i);
    }
    return s + "}";
  }
  if (auto* lb = dynamic_cast<const ListVectorBatch*>(&b)) {
    std::string s = "[";
    for (int64_t k = lb->offsets[i]; k < lb->offsets[i + 1]; ++k)
      s += (k > lb->offsets[i] ? ", " : "") + row(r, subs[0], *lb->elements, (uint64_t)k);
    return s + "]";
  }
  if (auto* mb = dynamic_cast<const MapVectorBatch*>(&b)) {
    std::string s = "[";
    for (int64_t k = mb->offsets[i]; k < mb->offsets[i + 1]; ++k)
      s += std::string(k > mb->offsets[i] ? ", " : "") + "{\"key\": " + row(r, subs[0], *mb->keys, (uint64_t)k) +
           ", \"value\": " + row(r, subs[1], *mb->elements, (uint64_t)k) + "}";
    return s + "]";
  }
  if (auto* ub = dynamic_cast<const UnionVectorBatch*>(&b)) {
    const unsigned tag = ub->tags[i];
    return "{\"tag\": " + std::to_string(tag) + ", \"value\": " + row(r, subs[tag], *ub->children[tag], ub->offsets[i]) +
           "}";
  }
  return value(b, i);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <file.orc> [--batch N] [--seek r1,r2,...] [--range OFF LEN] [--lazy] [--include ids]\n",
            argv[0]);
    return 2;
  }
  uint64_t cap = 1024;
  std::vector<uint64_t> seeks;
  RowReaderOptions opts;
  bool ranged = false, bench = false, pinned = false;
  for (int a = 2; a < argc; ++a) {
    if (!strcmp(argv[a], "--batch") && a + 1 < argc) cap = strtoull(argv[++a], nullptr, 10);
    else if (!strcmp(argv[a], "--lazy")) opts.setEnableLazyDecoding(true);
    else if (!strcmp(argv[a], "--tight")) opts.setUseTightNumericVector(true);
    else if (!strcmp(argv[a], "--bench")) bench = true;
    else if (!strcmp(argv[a], "--pinned")) pinned = true;
    else if (!strcmp(argv[a], "--include") && a + 1 < argc) {
      std::list<uint64_t> ids;
      char* p = argv[++a];
      while (*p) {
        ids.push_back(strtoull(p, &p, 10));
        if (*p == ',') ++p;
      }
      opts.include(ids);
    }
    else if (!strcmp(argv[a], "--range") && a + 2 < argc) {
      opts.range(strtoull(argv[a + 1], nullptr, 10), strtoull(argv[a + 2], nullptr, 10));
      a += 2;
      ranged = true;
    } else if (!strcmp(argv[a], "--seek") && a + 1 < argc) {
      char* p = argv[++a];
      while (*p) {
        seeks.push_back(strtoull(p, &p, 10));
        if (*p == ',') ++p;
      }
    }
  }
  try {
    Context ctx(0);
    // --pinned: batches in page-locked memory from the caller's pool
    // (ReaderOptions::setMemoryPool, the orc::MemoryPool seam)
    PinnedMemoryPool pinned_pool;
    ReaderOptions ropts;
    if (pinned) ropts.setMemoryPool(pinned_pool);
    const auto tc = std::chrono::steady_clock::now();
    Reader reader(ctx, argv[1], ropts);
    auto rows = reader.createRowReader(opts);
    rows->setProfiling(bench);
    g_rows = rows.get();
    g_names.assign(orcg_reader_num_types(reader.get()), {});
    names_of(reader, 0, g_names);
    auto batch = rows->createRowBatch(cap);
    if (!seeks.empty()) {
      for (uint64_t s : seeks) {
        rows->seekToRow(s);
        const bool more = rows->next(*batch);
        printf("#seek %llu %llu %llu\n", (unsigned long long)s, (unsigned long long)rows->getRowNumber(),
               (unsigned long long)(more ? batch->numElements : 0));
        if (more && (batch->numElements > cap || rows->getRowNumber() != s)) return 3;
        for (uint64_t i = 0; more && i < batch->numElements; ++i) puts(row(reader, 0, *batch, i).c_str());
      }
      return 0;
    }
    if (bench) {
      // the reference caller's scan loop (tools/src/FileScan.cc:22-44):
      // next() until the end, every batch filled into host ColumnVectorBatches
      const auto t0 = std::chrono::steady_clock::now();
      uint64_t n = 0, batches = 0;
      while (rows->next(*batch)) {
        n += batch->numElements;
        ++batches;
      }
      const auto t1 = std::chrono::steady_clock::now();
      const double s = std::chrono::duration<double>(t1 - t0).count();
      const double sc = std::chrono::duration<double>(t1 - tc).count();
      const std::vector<double> p = rows->getProfile();
      printf("{\"rows\": %llu, \"batches\": %llu, \"seconds\": %.6f, \"mrows_per_s\": %.3f, "
             "\"seconds_from_open\": %.6f, \"profile_s\": {\"c_next\": %.4f, \"fill\": %.4f, \"copies\": %.4f, "
             "\"worker_prepare\": %.4f, \"worker_decode\": %.4f, \"worker_d2h\": %.4f, \"worker_slab_alloc\": %.4f, "
             "\"worker_lookahead\": %.4f, \"caller_wait\": %.4f}}\n",
             (unsigned long long)n, (unsigned long long)batches, s, n / s / 1e6, sc, p[0], p[1], p[2],
             p.size() > 3 ? p[3] : 0., p.size() > 4 ? p[4] : 0., p.size() > 5 ? p[5] : 0., p.size() > 6 ? p[6] : 0.,
             p.size() > 7 ? p[7] : 0., p.size() > 8 ? p[8] : 0.);
      return n == reader.getNumberOfRows() || ranged ? 0 : 1;
    }
    uint64_t total = 0;
    bool first = true;
    while (rows->next(*batch)) {
      if (batch->numElements > cap) return 3;
      if (!ranged && rows->getRowNumber() != total) return 4;
      if (!not_null_ok(*batch)) {
        fprintf(stderr, "notNull: a batch without nulls has a 0 flag, or fewer flags than rows\n");
        return 5;
      }
      if (ranged && first) printf("#first %llu\n", (unsigned long long)rows->getRowNumber());
      first = false;
      for (uint64_t i = 0; i < batch->numElements; ++i) puts(row(reader, 0, *batch, i).c_str());
      total += batch->numElements;
    }
    fprintf(stderr, "rows %llu row_number %llu\n", (unsigned long long)total,
            (unsigned long long)rows->getRowNumber());
    if (ranged) return 0;
    return total == reader.getNumberOfRows() && rows->getRowNumber() == total ? 0 : 1;
  } catch (const std::exception& e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
