// C ABI of the decimal and timestamp value decoders (include/orcg.h):
// device-resident streams, the same kernels the file reader uses
// (decimal_kernels.hip).
#include "orcg_internal.hh"

using namespace orcg;

extern "C" {

static int decimal_decode(orcg_ctx* c, const uint8_t* d_src, uint64_t src_len, const int64_t* d_scales,
                          uint64_t nvalues, uint32_t precision, int32_t scale, void* d_out, uint8_t* d_keep) {
  if (!c || (src_len && !d_src) || (nvalues && (!d_scales || !d_out)) || precision > 38)
    return ORCG_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  const uint64_t ntiles_max = src_len / kVarintTile + 2;
  void *d_counts, *d_base;
  int rc = scratch(c, 5, ntiles_max * sizeof(int64_t), &d_counts);
  if (!rc) rc = scratch(c, 6, (ntiles_max + 1) * sizeof(int64_t), &d_base);
  if (rc) return rc;
  uint64_t ntiles = 0;
  if ((rc = launch_varint_tile_counts(c, d_src, src_len, (int64_t*)d_counts, &ntiles))) return rc;
  uint64_t total = 0;
  if (ntiles) {
    if ((rc = launch_exclusive_scan(c, (const int64_t*)d_counts, ntiles, (int64_t*)d_base))) return rc;
    if ((rc = hip_check(c, hipMemcpyAsync(&total, (int64_t*)d_base + ntiles, 8, hipMemcpyDeviceToHost, c->stream),
                        "D2H varint count")))
      return rc;
    if ((rc = sync_ctx(c))) return rc;
  }
  if (total < nvalues) return set_error(c, ORCG_PARSE_ERROR, "Read past end of stream in Decimal64ColumnReader");
  const int mode = precision == 0 ? (d_keep ? 3 : 2) : (precision > 18 ? 1 : 0);
  if ((rc = launch_varint_decimal(c, d_src, src_len, (const int64_t*)d_base, d_scales, nvalues, scale, mode, d_out,
                                  d_keep)))
    return rc;
  return sync_ctx(c);
}

int orcg_decimal_decode_device(orcg_ctx* c, const uint8_t* d_src, uint64_t src_len, const int64_t* d_scales,
                               uint64_t nvalues, uint32_t precision, int32_t scale, void* d_out) {
  return decimal_decode(c, d_src, src_len, d_scales, nvalues, precision, scale, d_out, nullptr);
}

int orcg_hive11_decimal_decode_device(orcg_ctx* c, const uint8_t* d_src, uint64_t src_len, const int64_t* d_scales,
                                      uint64_t nvalues, int32_t scale, int throw_on_overflow, void* d_out,
                                      uint8_t* d_keep) {
  if (!throw_on_overflow && nvalues && !d_keep) return ORCG_INVALID_ARGUMENT;
  return decimal_decode(c, d_src, src_len, d_scales, nvalues, 0, scale, d_out, throw_on_overflow ? nullptr : d_keep);
}

int orcg_timestamp_decode_device(orcg_ctx* c, int64_t* d_seconds, int64_t* d_nanos, uint64_t n, int64_t epoch) {
  if (!c || (n && (!d_seconds || !d_nanos))) return ORCG_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  const int rc = launch_timestamp(c, d_seconds, d_nanos, n, epoch);
  return rc ? rc : sync_ctx(c);
}

}  // extern "C"
