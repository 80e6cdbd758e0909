// RLEv1 host planning and C ABI (orcg_rlev1_*).
//
// The plan walks the control bytes and varint terminators of a host stream
// (RleDecoderV1::readHeader / readLong, c++/src/RLEv1.cc:154-191) and cuts it
// into header-aligned segments for rlev1_kernel; it decodes no values.
#include <memory>

#include "orcg_internal.hh"

using namespace orcg;

// Ends of the varint starting at `p` (one past its terminator), or len + 1
// when the stream ends first.
static uint64_t varint_end(const uint8_t* s, uint64_t len, uint64_t p) {
  while (p < len && (s[p] & 0x80u)) ++p;
  return p < len ? p + 1 : len + 1;
}

orcg_rlev2_plan* make_v1_plan(const uint8_t* src, uint64_t len, uint64_t max_bytes, uint64_t max_values) {
  auto* p = new orcg_rlev2_plan();
  uint64_t pos = 0, vi = 0, seg_b = 0, seg_v = 0;
  bool open = false;
  while (pos < len) {
    if (!open || pos - seg_b >= max_bytes || vi - seg_v >= max_values) {
      p->segs.push_back(orcg_segment{pos, vi});
      seg_b = pos;
      seg_v = vi;
      open = true;
    }
    const int32_t h = (int32_t)(int8_t)src[pos];
    if (h >= 0) {
      const uint64_t e = pos + 2 <= len ? varint_end(src, len, pos + 2) : len + 1;
      if (e > len) {
        p->err = kErrV1BadRead;
        p->err_at = vi;
        break;
      }
      pos = e;
      vi += (uint64_t)h + 3;
    } else {
      uint64_t q = pos + 1, k = (uint64_t)(-h), done = 0;
      while (done < k) {
        const uint64_t e = varint_end(src, len, q);
        if (e > len) break;
        q = e;
        ++done;
      }
      if (done < k) {
        p->err = kErrV1BadRead;
        p->err_at = vi + done;
        vi += done;
        break;
      }
      pos = q;
      vi += k;
    }
  }
  p->values = vi;
  return p;
}

template <typename T>
static int v1_decode_host(orcg_ctx* c, const uint8_t* src, uint64_t len, int is_signed, const char* not_null,
                          uint64_t n, T* dst) {
  if (!c || (len && !src) || (n && !dst)) return ORCG_INVALID_ARGUMENT;
  uint64_t k = n;
  if (not_null) {
    k = 0;
    for (uint64_t i = 0; i < n; ++i) k += not_null[i] ? 1 : 0;
  }
  std::unique_ptr<orcg_rlev2_plan> plan(make_v1_plan(src, len, 16u << 10, 8192));
  if (k > plan->values) {
    const uint32_t e = plan->err != kErrNone ? plan->err : (uint32_t)kErrV1BadRead;
    return set_error(c, dev_error_status(e), dev_error_message(e));
  }
  if (k == 0) return ORCG_OK;
  hipSetDevice(c->device);
  void *d_src, *d_seg, *d_out;
  int rc = scratch(c, 0, len + 16, &d_src);
  if (!rc) rc = scratch(c, 1, plan->segs.size() * sizeof(orcg_segment), &d_seg);
  if (!rc) rc = scratch(c, 2, k * sizeof(T), &d_out);
  if (rc) return rc;
  rc = hip_check(c, hipMemcpyAsync(d_src, src, len, hipMemcpyHostToDevice, c->stream), "H2D stream");
  if (!rc)
    rc = hip_check(c, hipMemcpyAsync(d_seg, plan->segs.data(), plan->segs.size() * sizeof(orcg_segment),
                                     hipMemcpyHostToDevice, c->stream),
                   "H2D segments");
  if (!rc)
    rc = launch_rlev1(c, (const uint8_t*)d_src, len, is_signed, (const uint64_t*)d_seg, plan->segs.size(), 0, k,
                      d_out, sizeof(T));
  if (not_null) {
    std::vector<T> dense(k);
    if (!rc)
      rc = hip_check(c, hipMemcpyAsync(dense.data(), d_out, k * sizeof(T), hipMemcpyDeviceToHost, c->stream),
                     "D2H values");
    if (!rc) rc = sync_ctx(c);
    if (rc) return rc;
    uint64_t j = 0;
    for (uint64_t i = 0; i < n; ++i)
      if (not_null[i]) dst[i] = dense[j++];
    return ORCG_OK;
  }
  if (!rc)
    rc = hip_check(c, hipMemcpyAsync(dst, d_out, k * sizeof(T), hipMemcpyDeviceToHost, c->stream), "D2H values");
  if (!rc) rc = sync_ctx(c);
  return rc;
}

extern "C" {

int orcg_rlev1_plan_create(const uint8_t* src, uint64_t len, uint64_t max_bytes, uint64_t max_values,
                           orcg_rlev2_plan** out) {
  if (!out || (len && !src)) return ORCG_INVALID_ARGUMENT;
  *out = make_v1_plan(src, len, max_bytes ? max_bytes : (16u << 10), max_values ? max_values : 8192);
  return ORCG_OK;
}

int orcg_rlev1_decode_device(orcg_ctx* c, const uint8_t* d_src, uint64_t src_len, int is_signed,
                             const orcg_segment* d_segs, uint64_t nsegs, uint64_t value_begin, uint64_t nvalues,
                             void* d_dst, int dst_bytes) {
  if (!c || (nsegs && (!d_src || !d_segs)) || (nvalues && !d_dst)) return ORCG_INVALID_ARGUMENT;
  hipSetDevice(c->device);
  return launch_rlev1(c, d_src, src_len, is_signed, (const uint64_t*)d_segs, nsegs, value_begin, nvalues, d_dst,
                      dst_bytes);
}

int orcg_rlev1_decode_i64(orcg_ctx* c, const uint8_t* s, uint64_t l, int sg, const char* nn, uint64_t n,
                          int64_t* d) {
  return v1_decode_host(c, s, l, sg, nn, n, d);
}
int orcg_rlev1_decode_i32(orcg_ctx* c, const uint8_t* s, uint64_t l, int sg, const char* nn, uint64_t n,
                          int32_t* d) {
  return v1_decode_host(c, s, l, sg, nn, n, d);
}

}  // extern "C"
