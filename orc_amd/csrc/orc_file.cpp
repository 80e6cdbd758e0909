// ORC tail / stripe-footer parsing and block decompression (see orc_file.hh).
#include "orc_file.hh"

#include <dlfcn.h>
#include <string.h>
#include <zlib.h>


namespace orcg {
namespace file {
namespace {

// Protocol-buffers wire format: (field << 3 | wire type) keys, base-128
// varints, 64/32-bit little-endian fixed fields, length-delimited bytes.
struct Pb {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  Pb(const uint8_t* b, uint64_t n) : p(b), end(b + n) {}
  bool more() const { return ok && p < end; }
  uint64_t varint() {
    uint64_t r = 0;
    for (int sh = 0; sh < 70; sh += 7) {
      if (p >= end) {
        ok = false;
        return 0;
      }
      const uint8_t b = *p++;
      if (sh < 64) r |= (uint64_t)(b & 0x7f) << sh;
      if (!(b & 0x80)) return r;
    }
    ok = false;
    return 0;
  }
  bool key(uint32_t& field, uint32_t& wire) {
    const uint64_t k = varint();
    field = (uint32_t)(k >> 3);
    wire = (uint32_t)(k & 7);
    return ok;
  }
  Pb bytes() {
    const uint64_t n = varint();
    if (!ok || n > (uint64_t)(end - p)) {
      ok = false;
      return Pb(p, 0);
    }
    Pb sub(p, n);
    p += n;
    return sub;
  }
  void skip(uint32_t wire) {
    switch (wire) {
      case 0: varint(); break;
      case 1: if (end - p < 8) ok = false; else p += 8; break;
      case 2: bytes(); break;
      case 5: if (end - p < 4) ok = false; else p += 4; break;
      default: ok = false;
    }
  }
  std::string str() {
    Pb s = bytes();
    return std::string((const char*)s.p, (size_t)(s.end - s.p));
  }
  // repeated uint32, packed (wire 2) or not (wire 0)
  void u32s(uint32_t wire, std::vector<uint32_t>& out) {
    if (wire == 2) {
      Pb s = bytes();
      while (s.more()) out.push_back((uint32_t)s.varint());
      if (!s.ok) ok = false;
    } else if (wire == 0) {
      out.push_back((uint32_t)varint());
    } else {
      ok = false;
    }
  }
};

bool parse_stripe_info(Pb m, StripeInfo& s) {
  uint32_t f, w;
  while (m.more() && m.key(f, w)) {
    if (w == 0 && f >= 1 && f <= 5) {
      const uint64_t v = m.varint();
      if (f == 1) s.offset = v;
      else if (f == 2) s.index_length = v;
      else if (f == 3) s.data_length = v;
      else if (f == 4) s.footer_length = v;
      else s.num_rows = v;
    } else {
      m.skip(w);
    }
  }
  return m.ok;
}

bool parse_type(Pb m, TypeInfo& t) {
  uint32_t f, w;
  while (m.more() && m.key(f, w)) {
    if (f == 1 && w == 0) t.kind = (uint32_t)m.varint();
    else if (f == 2) m.u32s(w, t.subtypes);
    else if (f == 3 && w == 2) t.field_names.push_back(m.str());
    else if (f == 4 && w == 0) t.maximum_length = (uint32_t)m.varint();
    else if (f == 5 && w == 0) t.precision = (uint32_t)m.varint();
    else if (f == 6 && w == 0) t.scale = (uint32_t)m.varint();
    else m.skip(w);
  }
  return m.ok;
}

}  // namespace

bool parse_row_index(const uint8_t* p, uint64_t n, std::vector<std::vector<uint64_t>>& entries) {
  // message RowIndex { repeated RowIndexEntry entry = 1; }
  // message RowIndexEntry { repeated uint64 positions = 1 [packed = true];
  //                         optional ColumnStatistics statistics = 2; }
  Pb m(p, n);
  uint32_t f, w;
  while (m.more() && m.key(f, w)) {
    if (f == 1 && w == 2) {
      Pb e = m.bytes();
      std::vector<uint64_t> pos;
      uint32_t ef, ew;
      while (e.more() && e.key(ef, ew)) {
        if (ef == 1 && ew == 2) {
          Pb q = e.bytes();
          while (q.more()) pos.push_back(q.varint());
          if (!q.ok) return false;
        } else if (ef == 1 && ew == 0) {
          pos.push_back(e.varint());
        } else {
          e.skip(ew);
        }
      }
      if (!e.ok) return false;
      entries.push_back(std::move(pos));
    } else {
      m.skip(w);
    }
  }
  return m.ok;
}

namespace {

// ---- snappy (raw block format) -------------------------------------------
// The reference links libsnappy (SnappyDecompressionStream, Compression.cc);
// this is the published block format: a varint uncompressed length, then
// literal / copy elements selected by the low two tag bits.
bool snappy_decompress(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t& out_len,
                       std::string& err) {
  const uint8_t* p = in;
  const uint8_t* end = in + n;
  uint64_t ulen = 0;
  for (int sh = 0;; sh += 7) {
    if (p >= end || sh > 35) { err = "snappy: bad length"; return false; }
    const uint8_t b = *p++;
    ulen |= (uint64_t)(b & 0x7f) << sh;
    if (!(b & 0x80)) break;
  }
  if (ulen > cap) { err = "snappy: output exceeds the compression block size"; return false; }
  uint64_t o = 0;
  while (p < end) {
    const uint8_t tag = *p++;
    const uint32_t kind = tag & 3u;
    if (kind == 0) {
      uint64_t len = (tag >> 2) + 1u;
      if (len > 60) {
        const uint32_t nb = (uint32_t)len - 60;
        if ((uint64_t)(end - p) < nb) { err = "snappy: truncated literal"; return false; }
        len = 0;
        for (uint32_t i = 0; i < nb; ++i) len |= (uint64_t)p[i] << (8 * i);
        len += 1;
        p += nb;
      }
      if ((uint64_t)(end - p) < len || o + len > ulen) { err = "snappy: literal out of range"; return false; }
      memcpy(out + o, p, len);
      p += len;
      o += len;
    } else {
      uint64_t len, off;
      if (kind == 1) {
        if (p >= end) { err = "snappy: truncated copy"; return false; }
        len = 4 + ((tag >> 2) & 7u);
        off = ((uint64_t)(tag >> 5) << 8) | *p++;
      } else if (kind == 2) {
        if (end - p < 2) { err = "snappy: truncated copy"; return false; }
        len = 1 + (tag >> 2);
        off = (uint64_t)p[0] | ((uint64_t)p[1] << 8);
        p += 2;
      } else {
        if (end - p < 4) { err = "snappy: truncated copy"; return false; }
        len = 1 + (tag >> 2);
        off = (uint64_t)p[0] | ((uint64_t)p[1] << 8) | ((uint64_t)p[2] << 16) | ((uint64_t)p[3] << 24);
        p += 4;
      }
      if (off == 0 || off > o || o + len > ulen) { err = "snappy: copy out of range"; return false; }
      uint8_t* d = out + o;
      const uint8_t* s = d - off;
      if (off >= len) memcpy(d, s, len);
      else for (uint64_t i = 0; i < len; ++i) d[i] = s[i];  // overlapping copy
      o += len;
    }
  }
  if (o != ulen) { err = "snappy: length mismatch"; return false; }
  out_len = o;
  return true;
}

// ---- LZO1X (the reference implements it itself: c++/src/LzoDecompressor.cc) --
// An LZO1X block is a sequence of instructions. A literal run copies bytes
// from the input; a match copies `len` bytes from `dist` back in the output
// (overlapping copies repeat). Every match carries, in the low two bits of
// its last distance byte, the count (0-3) of literals that follow it.
//   first byte > 17      : literal run of (byte - 17), then state "after literals"
//   0000LLLL             : literal run of L + 3 (L = 0: 15 + 255 per zero byte + next)
//   after a run, 0000DDSS: 3-byte match, dist = 1 + 0x800 + (D | next << 2)
//   after a match, 0000DDSS: 2-byte match, dist = 1 + (D | next << 2)
//   LLLDDDSS (>= 64)     : match of L + 1 bytes, dist = 1 + (D | next << 3)
//   001LLLLL (32..63)    : match of L + 2 (L = 0: 31 + 255 per zero + next), dist = 1 + (u16le >> 2)
//   0001HLLL (16..31)    : match of L + 2 (L = 0: 7 + ...), dist = 0x4000 + (H << 14) + (u16le >> 2);
//                          distance 0x4000 exactly ends the block
namespace {

bool lzo_decompress(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t& out_len,
                    std::string& err) {
  const uint8_t* ip = in;
  const uint8_t* const ie = in + n;
  uint64_t op = 0;
  auto fail = [&](const char* m) {
    err = std::string("LZO: ") + m;
    return false;
  };
  auto literals = [&](uint64_t t) -> bool {
    if ((uint64_t)(ie - ip) < t) return false;
    if (cap - op < t) return false;
    memcpy(out + op, ip, t);
    ip += t;
    op += t;
    return true;
  };
  auto copy_match = [&](uint64_t dist, uint64_t len) -> bool {
    if (dist == 0 || dist > op || cap - op < len) return false;
    const uint64_t from = op - dist;
    for (uint64_t k = 0; k < len; ++k) out[op + k] = out[from + k];  // may overlap forward
    op += len;
    return true;
  };
  auto long_length = [&](uint64_t base, uint64_t& t) -> bool {
    // t == 0: 255 per zero byte, then base + the next byte
    while (true) {
      if (ip >= ie) return false;
      if (*ip != 0) break;
      t += 255;
      ++ip;
    }
    t += base + *ip++;
    return true;
  };
  if (ip >= ie) return fail("empty input");
  // state: 0 = expecting an instruction after a match with no trailing
  // literals, 1 = right after a literal run of >= 4 bytes, 2 = right after
  // a match with 1-3 trailing literals
  int state = 0;
  uint64_t t = 0;
  if (*ip > 17) {
    t = *ip++ - 17u;
    if (!literals(t)) return fail("literal run past the end");
    state = t < 4 ? 2 : 1;
  }
  while (true) {
    if (ip >= ie) return fail("truncated input");
    t = *ip++;
    uint64_t len = 0, dist = 0;
    if (t < 16) {
      if (state == 0) {
        // literal run
        if (t == 0 && !long_length(15, t)) return fail("truncated run length");
        if (!literals(t + 3)) return fail("literal run past the end");
        state = 1;
        continue;
      }
      if (ip >= ie) return fail("truncated match");
      dist = 1 + (t >> 2) + ((uint64_t)*ip++ << 2);
      if (state == 1) {
        dist += 0x800;
        len = 3;
      } else {
        len = 2;
      }
    } else if (t >= 64) {
      if (ip >= ie) return fail("truncated match");
      dist = 1 + ((t >> 2) & 7u) + ((uint64_t)*ip++ << 3);
      len = (t >> 5) + 1;
    } else if (t >= 32) {
      len = t & 31u;
      if (len == 0 && !long_length(31, len)) return fail("truncated match length");
      len += 2;
      if (ie - ip < 2) return fail("truncated match");
      dist = 1 + ((ip[0] >> 2) | ((uint64_t)ip[1] << 6));
      ip += 2;
    } else {
      len = t & 7u;
      if (len == 0 && !long_length(7, len)) return fail("truncated match length");
      len += 2;
      if (ie - ip < 2) return fail("truncated match");
      dist = ((uint64_t)(t & 8u) << 11) + ((ip[0] >> 2) | ((uint64_t)ip[1] << 6));
      ip += 2;
      if (dist == 0) {  // the end-of-stream marker
        if (ip != ie) return fail("data after the end of the block");
        out_len = op;
        return true;
      }
      dist += 0x4000;
    }
    if (!copy_match(dist, len)) return fail("match outside the output");
    // trailing literals: the low two bits of the last distance byte read
    const uint64_t lit = ip[-2] & 3u;
    if (lit) {
      if (!literals(lit)) return fail("literal run past the end");
      state = 2;
    } else {
      state = 0;
    }
  }
}

}  // namespace

// ---- lz4 / zstd through the system libraries (dlopen) ----------------------
// The reference links liblz4 (LZ4_decompress_safe, Compression.cc Lz4
// DecompressionStream) and libzstd (ZSTD_decompressDCtx). Only the runtime
// .so files are in this image; the two entry points are resolved at run time.
typedef int (*lz4_fn)(const char*, char*, int, int);
typedef size_t (*zstd_fn)(void*, size_t, const void*, size_t);
typedef unsigned (*zstd_err_fn)(size_t);

struct DynCodecs {
  lz4_fn lz4 = nullptr;
  zstd_fn zstd = nullptr;
  zstd_err_fn zstd_is_error = nullptr;
  DynCodecs() {
    if (void* h = dlopen("liblz4.so.1", RTLD_NOW | RTLD_LOCAL)) lz4 = (lz4_fn)dlsym(h, "LZ4_decompress_safe");
    if (void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL)) {
      // usable only when both entry points resolve
      const zstd_fn d = (zstd_fn)dlsym(h, "ZSTD_decompress");
      const zstd_err_fn e = (zstd_err_fn)dlsym(h, "ZSTD_isError");
      if (d && e) {
        zstd = d;
        zstd_is_error = e;
      }
    }
  }
};

const DynCodecs& codecs() {
  static DynCodecs c;
  return c;
}

}  // namespace

const char* compression_name(uint32_t c) {
  switch (c) {
    case kNone: return "none";
    case kZlib: return "zlib";
    case kSnappy: return "snappy";
    case kLzo: return "lzo";
    case kLz4: return "lz4";
    case kZstd: return "zstd";
  }
  return "unknown";
}

bool parse_postscript(const uint8_t* p, uint64_t n, PostScript& ps) {
  Pb m(p, n);
  uint32_t f, w;
  while (m.more() && m.key(f, w)) {
    if (f == 1 && w == 0) ps.footer_length = m.varint();
    else if (f == 2 && w == 0) ps.compression = (uint32_t)m.varint();
    else if (f == 3 && w == 0) ps.block_size = m.varint();
    else if (f == 4) m.u32s(w, ps.version);
    else if (f == 5 && w == 0) ps.metadata_length = m.varint();
    else if (f == 6 && w == 0) ps.writer_version = (uint32_t)m.varint();
    else if (f == 8000 && w == 2) ps.magic = m.str();
    else m.skip(w);
  }
  return m.ok;
}

bool parse_footer(const uint8_t* p, uint64_t n, Footer& ft) {
  Pb m(p, n);
  uint32_t f, w;
  while (m.more() && m.key(f, w)) {
    if (f == 1 && w == 0) ft.header_length = m.varint();
    else if (f == 2 && w == 0) ft.content_length = m.varint();
    else if (f == 3 && w == 2) {
      ft.stripes.emplace_back();
      if (!parse_stripe_info(m.bytes(), ft.stripes.back())) return false;
    } else if (f == 4 && w == 2) {
      ft.types.emplace_back();
      if (!parse_type(m.bytes(), ft.types.back())) return false;
    } else if (f == 6 && w == 0) ft.num_rows = m.varint();
    else if (f == 8 && w == 0) ft.row_index_stride = (uint32_t)m.varint();
    else if (f == 9 && w == 0) ft.writer = (uint32_t)m.varint();
    else if (f == 12 && w == 2) {
      ft.has_software_version = true;
      ft.software_version = m.str();
    } else if (f == 5 && w == 2) {
      // UserMetadataItem {name = 1, value = 2}
      Pb u = m.bytes();
      std::string name, value;
      uint32_t g, v;
      while (u.more() && u.key(g, v)) {
        if (g == 1 && v == 2) name = u.str();
        else if (g == 2 && v == 2) value = u.str();
        else u.skip(v);
      }
      if (!u.ok) return false;
      ft.metadata.emplace_back(std::move(name), std::move(value));
    } else m.skip(w);
  }
  return m.ok;
}

bool parse_stripe_footer(const uint8_t* p, uint64_t n, uint64_t stripe_offset, StripeFooter& sf) {
  Pb m(p, n);
  uint32_t f, w;
  uint64_t off = stripe_offset;
  while (m.more() && m.key(f, w)) {
    if (f == 1 && w == 2) {
      Pb s = m.bytes();
      StreamInfo si;
      uint32_t g, v;
      while (s.more() && s.key(g, v)) {
        if (g == 1 && v == 0) si.kind = (uint32_t)s.varint();
        else if (g == 2 && v == 0) si.column = (uint32_t)s.varint();
        else if (g == 3 && v == 0) si.length = s.varint();
        else s.skip(v);
      }
      if (!s.ok) return false;
      si.offset = off;  // streams are laid out back to back in footer order
      if (__builtin_add_overflow(off, si.length, &off)) return false;  // lengths past 2^64: corrupt
      sf.streams.push_back(si);
    } else if (f == 2 && w == 2) {
      Pb s = m.bytes();
      ColumnEncoding ce;
      uint32_t g, v;
      while (s.more() && s.key(g, v)) {
        if (g == 1 && v == 0) ce.kind = (uint32_t)s.varint();
        else if (g == 2 && v == 0) ce.dictionary_size = (uint32_t)s.varint();
        else s.skip(v);
      }
      if (!s.ok) return false;
      sf.encodings.push_back(ce);
    } else if (f == 3 && w == 2) {
      sf.writer_timezone = m.str();
    } else {
      m.skip(w);
    }
  }
  return m.ok;
}

bool split_chunks(const uint8_t* file, uint64_t off, uint64_t len, uint32_t compression, std::vector<Chunk>& out,
                  std::string& err) {
  if (compression == kNone) {
    Chunk c;
    c.src_off = off;
    c.src_len = len;
    c.original = true;
    out.push_back(c);
    return true;
  }
  uint64_t p = off;
  uint64_t end;
  if (__builtin_add_overflow(off, len, &end)) {
    err = "Read past EOF in DecompressionStream::readBuffer";
    return false;
  }
  while (p < end) {
    if (end - p < 3) {
      err = "Read past EOF in DecompressionStream::readBuffer";
      return false;
    }
    const uint32_t h = (uint32_t)file[p] | ((uint32_t)file[p + 1] << 8) | ((uint32_t)file[p + 2] << 16);
    Chunk c;
    c.original = (h & 1u) != 0;
    c.src_len = h >> 1;
    c.src_off = p + 3;
    if (c.src_len > end - c.src_off) {
      err = "Read past EOF in DecompressionStream::readBuffer";
      return false;
    }
    out.push_back(c);
    p = c.src_off + c.src_len;
  }
  return true;
}

bool decompress_chunk(uint32_t compression, const uint8_t* file, Chunk& c, uint8_t* dst, uint64_t cap,
                      std::string& err) {
  const uint8_t* in = file + c.src_off;
  if (c.original) {
    if (c.src_len > cap) { err = "chunk larger than the compression block size"; return false; }
    memcpy(dst, in, c.src_len);
    c.dst_len = c.src_len;
    return true;
  }
  switch (compression) {
    case kZlib: {
      // raw deflate (inflateInit2 with -15 window bits), ZlibDecompressionStream
      z_stream zs;
      memset(&zs, 0, sizeof(zs));
      if (inflateInit2(&zs, -15) != Z_OK) { err = "Failed to initialize inflate"; return false; }
      zs.next_in = const_cast<Bytef*>(in);
      zs.avail_in = (uInt)c.src_len;
      zs.next_out = dst;
      zs.avail_out = (uInt)cap;
      const int r = inflate(&zs, Z_FINISH);
      c.dst_len = cap - zs.avail_out;
      inflateEnd(&zs);
      if (r != Z_STREAM_END) {
        err = r == Z_BUF_ERROR ? "Buffer error in ZlibDecompressionStream::NextDecompress"
                               : "Failed to inflate input data in ZlibDecompressionStream";
        return false;
      }
      return true;
    }
    case kSnappy:
      return snappy_decompress(in, c.src_len, dst, cap, c.dst_len, err);
    case kLz4: {
      const auto& k = codecs();
      if (!k.lz4) { err = "lz4 codec library (liblz4.so.1) not available"; return false; }
      const int r = k.lz4((const char*)in, (char*)dst, (int)c.src_len, (int)cap);
      if (r < 0) { err = "Corrupt lz4 compressed block"; return false; }
      c.dst_len = (uint64_t)r;
      return true;
    }
    case kZstd: {
      const auto& k = codecs();
      if (!k.zstd) { err = "zstd codec library (libzstd.so.1) not available"; return false; }
      const size_t r = k.zstd(dst, cap, in, c.src_len);
      if (k.zstd_is_error(r)) { err = "Corrupt zstd compressed block"; return false; }
      c.dst_len = r;
      return true;
    }
    case kLzo:
      return lzo_decompress(in, c.src_len, dst, cap, c.dst_len, err);
  }
  err = "Unknown compression type";
  return false;
}

bool read_range(const uint8_t* file, uint64_t off, uint64_t len, uint32_t compression, uint64_t block_size,
                std::vector<uint8_t>& out, std::string& err) {
  std::vector<Chunk> chunks;
  if (!split_chunks(file, off, len, compression, chunks, err)) return false;
  out.clear();
  for (auto& c : chunks) {
    const uint64_t at = out.size();
    const uint64_t cap = c.original ? c.src_len : block_size;
    out.resize(at + cap);
    if (!decompress_chunk(compression, file, c, out.data() + at, cap, err)) return false;
    out.resize(at + c.dst_len);
  }
  return true;
}

}  // namespace file
}  // namespace orcg
