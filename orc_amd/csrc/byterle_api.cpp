// liborcgpu C ABI for byte / boolean RLE streams (PRESENT, BOOLEAN, BYTE),
// the null scatter of nullable columns and the string-dictionary gather.
// Reference: ByteRleDecoder (c++/src/ByteRLE.hh:71-126, ByteRLE.cc:359-643),
// IntegerColumnReader::next + ColumnReader::next (c++/src/ColumnReader.cc:
// 81-104, 224-258), StringDictionaryColumnReader (ColumnReader.cc:509-613),
// loadStringDictionary (c++/src/DictionaryLoader.cc:43-97).
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "orcg_internal.hh"

using namespace orcg;

// Host walk of the control bytes (ByteRleDecoderImpl::readHeader,
// ByteRLE.cc:378-388): segments + decodable byte count + first bad group.
orcg_rlev2_plan* make_byte_plan(const uint8_t* src, uint64_t len, uint64_t max_bytes, uint64_t max_values) {
  auto* p = new orcg_rlev2_plan();
  uint64_t pos = 0, vi = 0, seg_b = 0, seg_v = 0;
  bool open = false;
  while (pos < len) {
    const uint32_t h = src[pos];
    const uint64_t L = h < 0x80 ? h + 3 : 256 - h;
    const uint64_t bytes = h < 0x80 ? 2 : 1 + L;
    if (pos + bytes > len) {  // truncated group: the read fails here
      p->err = kErrByteBadRead;
      p->err_at = vi;
      break;
    }
    if (!open || pos - seg_b >= max_bytes || vi - seg_v >= max_values) {
      p->segs.push_back({pos, vi});
      seg_b = pos;
      seg_v = vi;
      open = true;
    }
    pos += bytes;
    vi += L;
  }
  p->values = vi;
  return p;
}

namespace {

// H2D + byte-RLE decode of decoded bytes [0, count) into host `out`.
int decode_bytes_host(Ctx* c, const uint8_t* src, uint64_t len, const orcg_rlev2_plan* plan, uint64_t count,
                      uint8_t* out) {
  if (count == 0) return ORCG_OK;
  (void)hipSetDevice(c->device);
  void *d_src, *d_seg, *d_out;
  int rc = scratch(c, 0, len + 16, &d_src);
  if (!rc) rc = scratch(c, 1, plan->segs.size() * sizeof(orcg_segment), &d_seg);
  if (!rc) rc = scratch(c, 2, count + 16, &d_out);
  if (rc) return rc;
  rc = hip_check(c, hipMemcpyAsync(d_src, src, len, hipMemcpyHostToDevice, c->stream), "H2D stream");
  if (!rc)
    rc = hip_check(c, hipMemcpyAsync(d_seg, plan->segs.data(), plan->segs.size() * sizeof(orcg_segment),
                                     hipMemcpyHostToDevice, c->stream),
                   "H2D segments");
  if (!rc)
    rc = launch_byterle(c, (const uint8_t*)d_src, len, (const uint64_t*)d_seg, plan->segs.size(), false, 0, count,
                        (uint8_t*)d_out);
  if (!rc) rc = hip_check(c, hipMemcpyAsync(out, d_out, count, hipMemcpyDeviceToHost, c->stream), "D2H bytes");
  if (!rc) rc = sync_ctx(c);
  return rc;
}

}  // namespace

struct orcg_byte_rle_decoder {
  Ctx* ctx = nullptr;
  bool boolean = false;
  std::vector<uint8_t> src;
  std::unique_ptr<orcg_rlev2_plan> plan;
  uint64_t origin = 0;          // stream byte offset the decoded bytes start at
  std::vector<uint8_t> values;  // decoded bytes from `origin`
  uint64_t cursor = 0;          // in bytes (byte mode) or bits (boolean mode)
  std::string last_error;

  int fail(int st, const std::string& m) {
    last_error = m;
    return st;
  }
  int load_from(uint64_t from) {
    origin = from;
    cursor = 0;
    const uint8_t* s = src.data() + from;
    const uint64_t len = src.size() - from;
    plan.reset(make_byte_plan(s, len, 16u << 10, 16384));
    values.assign(plan->values, 0);
    int rc = decode_bytes_host(ctx, s, len, plan.get(), plan->values, values.data());
    return rc ? fail(rc, ctx->last_error) : ORCG_OK;
  }
  uint64_t avail_units() const { return boolean ? values.size() * 8 : values.size(); }
  int eof() { return fail(ORCG_PARSE_ERROR, dev_error_message(kErrByteBadRead)); }
  uint8_t unit(uint64_t i) const { return boolean ? (values[i >> 3] >> (7 - (i & 7))) & 1 : values[i]; }

  // ByteRleDecoderImpl::next (ByteRLE.cc:449-505; null slots untouched) and
  // BooleanRleDecoderImpl::next (:578-643; null slots get 0).
  int next(char* data, uint64_t n, const char* nn) {
    uint64_t k = n;
    if (nn) {
      k = 0;
      for (uint64_t i = 0; i < n; ++i) k += nn[i] ? 1 : 0;
    }
    // the boolean decoder reads whole bytes (ByteRLE.cc:618-624)
    uint64_t need = cursor + k;
    if (boolean) need = (need + 7) / 8 * 8;
    if (need > avail_units()) {
      // bytes up to the failure are delivered, then the read fails
      const uint64_t have = avail_units() > cursor ? avail_units() - cursor : 0;
      uint64_t j = 0;
      for (uint64_t i = 0; i < n && j < have; ++i) {
        if (nn && !nn[i]) {
          if (boolean) data[i] = 0;
          continue;
        }
        data[i] = (char)unit(cursor + j++);
      }
      cursor += j;
      return eof();
    }
    for (uint64_t i = 0; i < n; ++i) {
      if (nn && !nn[i]) {
        if (boolean) data[i] = 0;
        continue;
      }
      data[i] = (char)unit(cursor++);
    }
    return ORCG_OK;
  }
  int skip(uint64_t n) {
    uint64_t need = cursor + n;
    if (boolean && need % 8) need = (need + 7) / 8 * 8;
    if (need > avail_units()) return eof();
    cursor += n;
    return ORCG_OK;
  }
  // byte RLE position: (byte offset, bytes to skip); boolean adds the bits
  // consumed of the next byte (BooleanRleDecoderImpl::seek, ByteRLE.cc:549-560)
  int seek(const uint64_t* pos, uint64_t npos) {
    if (npos < (boolean ? 3u : 2u)) return fail(ORCG_INVALID_ARGUMENT, "bad position");
    const uint64_t byte = pos[0], skipb = pos[1], bits = boolean ? pos[2] : 0;
    if (byte > src.size()) return fail(ORCG_INVALID_ARGUMENT, "Seek past end of stream");
    if (bits > 8) return fail(ORCG_PARSE_ERROR, "bad position");
    // is `byte` a group start of the current decoding?
    bool found = false;
    uint64_t vi = 0;
    if (byte >= origin) {
      const uint64_t rel = byte - origin;
      auto it = std::upper_bound(plan->segs.begin(), plan->segs.end(), rel,
                                 [](uint64_t b, const orcg_segment& s) { return b < s.byte_offset; });
      if (it != plan->segs.begin()) {
        --it;
        uint64_t p = it->byte_offset, v = it->value_index;
        const uint8_t* s = src.data() + origin;
        const uint64_t len = src.size() - origin;
        while (p < rel && p < len) {
          const uint32_t h = s[p];
          p += h < 0x80 ? 2 : 1 + (256 - h);
          v += h < 0x80 ? h + 3 : 256 - h;
        }
        if (p == rel) {
          found = true;
          vi = v;
        }
      }
    }
    if (!found) {
      int rc = load_from(byte);
      if (rc) return rc;
    }
    cursor = boolean ? 8 * (vi + skipb) : vi + skipb;
    if (cursor > avail_units()) return eof();
    if (boolean && bits) {
      if (cursor + 8 > avail_units()) return eof();
      cursor += bits;
    }
    return ORCG_OK;
  }
};

extern "C" {

int orcg_byterle_plan_create(const uint8_t* src, uint64_t len, uint64_t max_bytes, uint64_t max_values,
                             orcg_rlev2_plan** out) {
  if (!out || (len && !src)) return ORCG_INVALID_ARGUMENT;
  *out = make_byte_plan(src, len, max_bytes ? max_bytes : (16u << 10), max_values ? max_values : 16384);
  return ORCG_OK;
}

int orcg_byterle_decode_device(orcg_ctx* c, const uint8_t* d_src, uint64_t src_len, const orcg_segment* d_segs,
                               uint64_t nsegs, uint64_t value_begin, uint64_t nvalues, uint8_t* d_dst) {
  if (!c || (nsegs && (!d_src || !d_segs)) || (nvalues && !d_dst)) return ORCG_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  return launch_byterle(c, d_src, src_len, (const uint64_t*)d_segs, nsegs, false, value_begin, nvalues, d_dst, nullptr);
}

int orcg_boolrle_decode_device(orcg_ctx* c, const uint8_t* d_src, uint64_t src_len, const orcg_segment* d_segs,
                               uint64_t nsegs, uint64_t row_begin, uint64_t nrows, uint8_t* d_dst) {
  if (!c || (nsegs && (!d_src || !d_segs)) || (nrows && !d_dst)) return ORCG_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  return launch_byterle(c, d_src, src_len, (const uint64_t*)d_segs, nsegs, true, row_begin, nrows, d_dst, nullptr);
}

int orcg_byte_rle_decoder_create(orcg_ctx* c, const uint8_t* src, uint64_t len, int boolean,
                                 orcg_byte_rle_decoder** out) {
  if (!c || !out || (len && !src)) return ORCG_INVALID_ARGUMENT;
  *out = nullptr;
  auto* d = new orcg_byte_rle_decoder();
  d->ctx = c;
  d->boolean = boolean != 0;
  d->src.assign(src, src + len);
  int rc = d->load_from(0);
  if (rc) {
    c->last_error = d->last_error;
    delete d;
    return rc;
  }
  *out = d;
  return ORCG_OK;
}

void orcg_byte_rle_decoder_destroy(orcg_byte_rle_decoder* d) { delete d; }

int orcg_byte_rle_decoder_next(orcg_byte_rle_decoder* d, char* data, uint64_t n, const char* not_null) {
  if (!d || (n && !data)) return ORCG_INVALID_ARGUMENT;
  return d->next(data, n, not_null);
}

int orcg_byte_rle_decoder_skip(orcg_byte_rle_decoder* d, uint64_t n) {
  return d ? d->skip(n) : ORCG_INVALID_ARGUMENT;
}

int orcg_byte_rle_decoder_seek(orcg_byte_rle_decoder* d, const uint64_t* positions, uint64_t npos) {
  if (!d || !positions) return ORCG_INVALID_ARGUMENT;
  return d->seek(positions, npos);
}

const char* orcg_byte_rle_decoder_last_error(const orcg_byte_rle_decoder* d) {
  return d ? d->last_error.c_str() : "";
}

int orcg_scatter_not_null_device(orcg_ctx* c, const void* d_dense, const uint8_t* d_not_null, uint64_t n,
                                 void* d_out, int width, int fill_nulls, int64_t fill_value) {
  if (!c || (n && (!d_dense || !d_not_null || !d_out))) return ORCG_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  return launch_scatter(c, d_dense, d_not_null, n, d_out, width, fill_nulls, fill_value);
}

int orcg_dict_offsets_device(orcg_ctx* c, const int64_t* d_lengths, uint64_t dict_size, int64_t* d_offsets) {
  if (!c || !d_offsets || (dict_size && !d_lengths)) return ORCG_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  return launch_dict_offsets(c, d_lengths, dict_size, d_offsets);
}

int orcg_dict_gather_device(orcg_ctx* c, const void* d_indices, int index_width, const uint8_t* d_not_null,
                            uint64_t n, const int64_t* d_offsets, uint64_t dict_size, int64_t* d_start,
                            int64_t* d_length) {
  if (!c || (n && (!d_indices || !d_offsets || !d_start || !d_length))) return ORCG_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  return launch_dict_gather(c, d_indices, index_width, d_not_null, n, d_offsets, dict_size, d_start, d_length);
}

// IntegerColumnReader<LongVectorBatch>::next over a whole stripe column
// (ColumnReader.cc:81-104, 224-258): PRESENT (boolean RLE, may be absent)
// and DATA (RLEv2) host streams -> not_null[n] (1 = value present) and
// data[n]; null slots of `data` are left untouched.
int orcg_decode_integer_column(orcg_ctx* c, const uint8_t* present, uint64_t present_len, const uint8_t* data,
                               uint64_t data_len, int is_signed, uint64_t n, int64_t* out, char* not_null) {
  if (!c || (n && !out) || (data_len && !data) || (present_len && !present)) return ORCG_INVALID_ARGUMENT;
  std::vector<char> nn;
  uint64_t k = n;
  if (present && present_len) {
    orcg_byte_rle_decoder* pd = nullptr;
    int rc = orcg_byte_rle_decoder_create(c, present, present_len, 1, &pd);
    if (rc) return rc;
    std::unique_ptr<orcg_byte_rle_decoder> guard(pd);
    nn.assign(n, 0);
    rc = pd->next(nn.data(), n, nullptr);
    if (rc) return set_error(c, rc, pd->last_error);
    k = 0;
    for (uint64_t i = 0; i < n; ++i) k += nn[i] ? 1 : 0;
    if (not_null) memcpy(not_null, nn.data(), n);
  } else if (not_null) {
    memset(not_null, 1, n);
  }
  std::unique_ptr<orcg_rlev2_plan> plan(make_plan(data, data_len, 16u << 10, 8192));
  if (k > plan->values) {
    const uint32_t e = plan->err != kErrNone ? plan->err : (uint32_t)kErrBadRead;
    return set_error(c, dev_error_status(e), dev_error_message(e));
  }
  if (nn.empty()) return decode_host_dense(c, data, data_len, is_signed, plan.get(), k, out, 8);
  std::vector<int64_t> dense(k);
  int rc = decode_host_dense(c, data, data_len, is_signed, plan.get(), k, dense.data(), 8);
  if (rc) return rc;
  uint64_t j = 0;
  for (uint64_t i = 0; i < n; ++i)
    if (nn[i]) out[i] = dense[j++];
  return ORCG_OK;
}

}  // extern "C"
