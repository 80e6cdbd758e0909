// Decimal and timestamp column kernels (gfx950).
//
// Decimal64ColumnReader / Decimal128ColumnReader::next (c++/src/ColumnReader.cc
// :1300-1527): the DATA stream is a sequence of zigzag base-128 varints (one
// per non-null value, no run structure), the SECONDARY stream holds each
// value's scale (signed RLE, decoded by the RLE kernels). A value is rescaled
// to the column's scale: Decimal64 multiplies / divides by a power of ten
// (readInt64 :1329-1350, "Decimal scale out of range" past 18 digits),
// Decimal128 loops in steps of 10^18 (scaleInt128 :1439-1456).
//
// Varints have no headers to walk, so the stream is cut anywhere: the grid
// covers it in 4 KB tiles; pass 1 counts terminator bytes (< 0x80) per tile,
// an exclusive scan gives every tile its first value index, pass 2 stages the
// tile (plus 64 bytes of look-back) in LDS, every thread assembles the
// varints that END in its 16 bytes (a varint that starts in a neighbour's
// bytes is assembled from the look-back) into an LDS value stage at their
// rank in the tile, then the workgroup rescales the staged values with
// their scales and stores them, both coalesced (a thread's own values are
// consecutive indices: loading their scales and storing them per thread
// serialised one global load per varint and scattered the stores).
//
// TimestampColumnReader::next (:308-349): seconds (signed RLE) + the writer
// time zone's epoch, nanos (unsigned RLE) with the trailing-zero code in the
// low 3 bits; writer and reader in the same (or a rule-free) zone.
#include "orcg_internal.hh"

namespace orcg {
namespace {

constexpr int kVThreads = 256;
constexpr uint32_t kVTile = (uint32_t)kVarintTile;
constexpr uint32_t kVPer = kVTile / kVThreads;  // 16 bytes per thread
constexpr uint32_t kLook = 64;                 // look-back bytes staged before the tile

__device__ const int64_t kPow10[19] = {1LL,
                                       10LL,
                                       100LL,
                                       1000LL,
                                       10000LL,
                                       100000LL,
                                       1000000LL,
                                       10000000LL,
                                       100000000LL,
                                       1000000000LL,
                                       10000000000LL,
                                       100000000000LL,
                                       1000000000000LL,
                                       10000000000000LL,
                                       100000000000000LL,
                                       1000000000000000LL,
                                       10000000000000000LL,
                                       100000000000000000LL,
                                       1000000000000000000LL};

__device__ __forceinline__ uint32_t term_bits(uint32_t w) {
  // bit i = byte i of w is a varint terminator (< 0x80)
  const uint32_t m = (~w >> 7) & 0x01010101u;
  return (m * 0x10204080u) >> 28;
}

__global__ __launch_bounds__(kVThreads) void varint_count_kernel(const uint8_t* __restrict__ src, uint64_t len,
                                                                 int64_t* __restrict__ counts) {
  const uint64_t t0 = (uint64_t)blockIdx.x * kVTile;
  uint32_t c = 0;
  for (uint32_t o = threadIdx.x * 4u; o < kVTile; o += kVThreads * 4u) {
    const uint64_t p = t0 + o;
    if (p + 4 <= len) {
      uint32_t w;
      __builtin_memcpy(&w, src + p, 4);
      c += __builtin_popcount(term_bits(w));
    } else {
      for (uint64_t q = p; q < len && q < p + 4; ++q) c += src[q] < 0x80u;
    }
  }
  // block reduction
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor((int)c, m);
  __shared__ uint32_t s[kVThreads / 64];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = (int64_t)(s[0] + s[1] + s[2] + s[3]);
}

struct U128 {
  uint64_t lo, hi;
};

__device__ __forceinline__ U128 mul128_u64(U128 a, uint64_t b) {
  // (a * b) mod 2^128
  const uint64_t lo = a.lo * b;
  const uint64_t hi = __umul64hi(a.lo, b) + a.hi * b;
  return U128{lo, hi};
}

// |a| / d for d < 2^32, in 32-bit limbs (Int128 singleDivide, Int128.cc:271-286)
__device__ __forceinline__ U128 div128_u32(U128 a, uint32_t d) {
  uint64_t r = 0;
  uint32_t q[4];
  const uint32_t limb[4] = {(uint32_t)(a.hi >> 32), (uint32_t)a.hi, (uint32_t)(a.lo >> 32), (uint32_t)a.lo};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r = (r << 32) | limb[j];
    q[j] = (uint32_t)(r / d);
    r %= d;
  }
  return U128{((uint64_t)q[2] << 32) | q[3], ((uint64_t)q[0] << 32) | q[1]};
}

__device__ __forceinline__ U128 neg128(U128 a) {
  const uint64_t lo = ~a.lo + 1;
  return U128{lo, ~a.hi + (lo == 0 ? 1 : 0)};
}

// value / 10^k, truncated toward zero (Int128::divide sign rules, :288-...),
// k <= 18, as two divisions by factors below 2^32
__device__ __forceinline__ U128 div128_pow10(U128 v, uint32_t k) {
  const bool neg = (int64_t)v.hi < 0;
  U128 m = neg ? neg128(v) : v;
  const uint32_t k1 = k > 9 ? 9 : k, k2 = k - k1;
  m = div128_u32(m, (uint32_t)kPow10[k1]);
  if (k2) m = div128_u32(m, (uint32_t)kPow10[k2]);
  return neg ? neg128(m) : m;
}

// kMode 0: Decimal64 (int64 out, readInt64); 1: Decimal128 ([hi, lo] int64
// pairs = orc::Int128's layout, readInt128); 2: Hive 0.11 decimals (precision
// 0, DecimalHive11ColumnReader::readInt128, ColumnReader.cc:1586-1617): as 1,
// plus the 128-bit varint limit and the 38-digit range check, both reported
// as "Hive 0.11 decimal was more than 38 digits." (throwOnHive11DecimalOverflow);
// 3: as 2 with throwOnHive11DecimalOverflow(false): such a value becomes NULL
// (keep[k] = 0, value 0; :1646-1677), every other keep[k] = 1.
template <int kMode>
__device__ __forceinline__ void varint_decimal_tile(const uint8_t* __restrict__ src, uint64_t len,
                                                    const int64_t* __restrict__ tile_base,
                                                    const int64_t* __restrict__ scales, uint64_t nvalues,
                                                    int32_t col_scale, void* __restrict__ out, unsigned long long* err,
                                                    uint8_t* __restrict__ keep, uint64_t tile) {
  constexpr bool kHive = kMode >= 2;
  __shared__ uint8_t s_bad[kMode == 3 ? kVTile : 1];  // mode 3: the varint ran past 128 bits
  __shared__ uint32_t s_buf[(kLook + kVTile) / 4 + 1];
  __shared__ uint32_t s_wsum[kVThreads / 64];
  // the tile's varints, by rank: unscaled values (Decimal64: zigzag-decoded
  // int64; Decimal128: the raw 128-bit varint, unzigzagged in pass 2)
  __shared__ uint64_t s_lo[kVTile];
  __shared__ uint64_t s_hi[kMode == 0 ? 1 : kVTile];
  const uint64_t t0 = tile * kVTile;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the tile's first value index and value count (the scan of the tile
  // counts), then every load the tile needs issued up front: its bytes and
  // the scales of its values (pass 2's scale loads, one dependent load a
  // loop trip, made the kernel latency-bound: 60 us a configs[3] stripe)
  const uint64_t kt = (uint64_t)tile_base[tile];  // value index of the tile's first varint
  const uint64_t kn = (uint64_t)tile_base[tile + 1];
  const uint32_t lim = kt >= nvalues ? 0u : (uint32_t)min(min(kn - kt, (uint64_t)kVTile), nvalues - kt);
  constexpr int kStage = (int)((kLook + kVTile + kVThreads * 4u - 1) / (kVThreads * 4u));
  constexpr int kScales = (int)(kVTile / kVThreads);
  uint32_t w[kStage];
  int32_t sc[kScales];
#pragma unroll
  for (int j = 0; j < kStage; ++j) {
    // stage [t0 - kLook, t0 + kVTile) (zero past the stream; bytes before 0
    // are marked as terminators so the first varint starts at 0)
    const uint32_t o = (uint32_t)tid * 4u + (uint32_t)j * kVThreads * 4u;
    const int64_t p = (int64_t)t0 - (int64_t)kLook + o;
    w[j] = 0;
    if (o >= kLook + kVTile) continue;
    if (p >= 0 && (uint64_t)p + 4 <= len) {
      __builtin_memcpy(&w[j], src + p, 4);
    } else {
      for (int i = 0; i < 4; ++i) {
        const int64_t q = p + i;
        const uint32_t b = q < 0 ? 0u : ((uint64_t)q < len ? src[q] : 0x80u);
        w[j] |= b << (8 * i);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kScales; ++j) {
    const uint32_t i = (uint32_t)tid + (uint32_t)j * kVThreads;
    sc[j] = i < lim ? (int32_t)scales[kt + i] : 0;
  }
#pragma unroll
  for (int j = 0; j < kStage; ++j) {
    const uint32_t o = (uint32_t)tid * 4u + (uint32_t)j * kVThreads * 4u;
    if (o < kLook + kVTile) s_buf[o / 4] = w[j];
  }
  __syncthreads();
  const uint32_t r0 = kLook + (uint32_t)tid * kVPer;  // my bytes in s_buf
  uint32_t mine[kVPer / 4];
  uint32_t tmask = 0;
#pragma unroll
  for (int i = 0; i < (int)kVPer / 4; ++i) {
    mine[i] = s_buf[r0 / 4 + i];
    tmask |= term_bits(mine[i]) << (4 * i);
  }
  // bytes past the end of the stream are not terminators
  const uint64_t my0 = t0 + (uint64_t)tid * kVPer;
  if (my0 + kVPer > len) tmask &= my0 >= len ? 0u : ((1u << (len - my0)) - 1u);
  const uint32_t cnt = __builtin_popcount(tmask);
  // rank of my first varint in the tile: exclusive scan of the counts
  uint32_t incl = cnt;
  for (int m = 1; m < 64; m <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, m);
    if (lane >= m) incl += y;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint32_t rk = incl - cnt;
  for (int w = 0; w < wave; ++w) rk += s_wsum[w];

  // pass 1: assemble my varints into the stage
  if (cnt && kt + rk < nvalues) {
    uint64_t acc_lo = 0, acc_hi = 0;
    uint32_t shift = 0;
    bool too_long = false;  // kMode 2: more than 128 bits (:1600)
    auto push = [&](uint32_t b) {
      const uint64_t x = b & 0x7fu;
      if constexpr (kHive) too_long = too_long || shift > 128 || (shift == 126 && x > 3);
      if constexpr (kMode == 0) {
        acc_lo |= x << (shift & 63u);  // x86 shift-count masking of readInt64's UB shift
      } else {
        if (shift < 64) {
          acc_lo |= x << shift;
          if (shift > 57) acc_hi |= x >> (64 - shift);
        } else if (shift < 128) {
          acc_hi |= x << (shift - 64);
        }
      }
      shift += 7;
    };
    {
      // first byte of the varint: scan back over continuation bytes
      int64_t s = (int64_t)my0 - 1;
      for (;;) {
        if (s < 0) break;
        uint32_t b;
        const int64_t rel = s - ((int64_t)t0 - (int64_t)kLook);
        if (rel >= 0) b = (s_buf[rel >> 2] >> ((rel & 3) * 8)) & 0xffu;
        else b = src[s];
        if (b < 0x80u) break;
        --s;
      }
      for (uint64_t q = (uint64_t)(s + 1); q < my0; ++q) {
        const int64_t rel = (int64_t)q - ((int64_t)t0 - (int64_t)kLook);
        const uint32_t b = rel >= 0 ? (s_buf[rel >> 2] >> ((rel & 3) * 8)) & 0xffu : src[q];
        push(b);
      }
    }
    uint32_t r = rk;
#pragma unroll
    for (int i = 0; i < (int)kVPer; ++i) {
      const uint32_t b = (mine[i >> 2] >> ((i & 3) * 8)) & 0xffu;
      push(b);
      if ((tmask >> i) & 1u) {
        if constexpr (kMode == 0) {
          s_lo[r] = (acc_lo >> 1) ^ (0 - (acc_lo & 1));
        } else {
          s_lo[r] = acc_lo;
          s_hi[r] = acc_hi;
          if constexpr (kMode == 2)
            if (too_long && kt + r < nvalues) atomicMin(err, (unsigned long long)(((kt + r) << 8) | kErrHive11Overflow));
          if constexpr (kMode == 3) s_bad[r] = too_long ? 1 : 0;
        }
        ++r;
        acc_lo = acc_hi = 0;
        shift = 0;
        too_long = false;
      }
    }
  }
  __syncthreads();

  // pass 2: rescale the staged values with their scales; stores coalesced
#pragma unroll
  for (int j = 0; j < kScales; ++j) {
    const uint32_t i = (uint32_t)tid + (uint32_t)j * kVThreads;
    if (i >= lim) break;
    const uint64_t k = kt + i;
    const int32_t cur = sc[j];
    if constexpr (kMode == 0) {
      int64_t v = (int64_t)s_lo[i];
      if (col_scale > cur && (uint64_t)(uint32_t)(col_scale - cur) <= 18) {
        v = (int64_t)((uint64_t)v * (uint64_t)kPow10[col_scale - cur]);
      } else if (col_scale < cur && (uint64_t)(uint32_t)(cur - col_scale) <= 18) {
        v /= kPow10[cur - col_scale];
      } else if (col_scale != cur) {
        atomicMin(err, (unsigned long long)((k << 8) | kErrDecimalScale));
      }
      ((int64_t*)out)[k] = v;
    } else {
      const uint64_t acc_lo = s_lo[i], acc_hi = s_hi[i];
      // unZigZagInt128 (:1291-1298): logical >> 1, negate and - 1 if odd
      const bool odd = acc_lo & 1;
      U128 v{(acc_lo >> 1) | (acc_hi << 63), acc_hi >> 1};
      if (odd) {
        v = neg128(v);
        const uint64_t lo = v.lo - 1;
        v.hi -= (v.lo == 0) ? 1 : 0;
        v.lo = lo;
      }
      // scaleInt128 (:1439-1456) with unsigned scales
      uint32_t s = (uint32_t)col_scale, c = (uint32_t)cur;
      if (s > c) {
        while (s > c && (v.lo | v.hi)) {
          const uint32_t a = min(18u, s - c);
          v = mul128_u64(v, (uint64_t)kPow10[a]);
          c += a;
        }
      } else {
        while (c > s && (v.lo | v.hi)) {
          const uint32_t a = min(18u, c - s);
          v = div128_pow10(v, a);
          c -= a;
        }
      }
      if constexpr (kHive) {
        // value >= MIN_VALUE && value <= MAX_VALUE, |v| <= 10^38 - 1 (:1616)
        const U128 m = (int64_t)v.hi < 0 ? neg128(v) : v;
        const uint64_t kHi = 0x4B3B4CA85A86C47Aull, kLo = 0x098A223FFFFFFFFFull;
        const bool over = m.hi > kHi || (m.hi == kHi && m.lo > kLo);
        if constexpr (kMode == 2) {
          if (over) atomicMin(err, (unsigned long long)((k << 8) | kErrHive11Overflow));
        } else {
          const bool null_it = over || s_bad[i];
          keep[k] = null_it ? 0 : 1;
          if (null_it) v = U128{0, 0};
        }
      }
      int64_t* o = (int64_t*)out + 2 * k;
      o[0] = (int64_t)v.hi;
      o[1] = (int64_t)v.lo;
    }
  }
}

template <int kMode>
__global__ __launch_bounds__(kVThreads) void varint_decimal_kernel(
    const uint8_t* __restrict__ src, uint64_t len, const int64_t* __restrict__ tile_base,
    const int64_t* __restrict__ scales, uint64_t nvalues, int32_t col_scale, void* __restrict__ out,
    unsigned long long* err, uint8_t* __restrict__ keep) {
  varint_decimal_tile<kMode>(src, len, tile_base, scales, nvalues, col_scale, out, err, keep, blockIdx.x);
}

// Several columns' decodes in one launch (the reader's batch: the stripe's
// decimal columns without nulls, after their SECONDARY streams): workgroup ->
// job by the jobs' first launch-wide tiles.
template <int kMode>
__global__ __launch_bounds__(kVThreads) void varint_decimal_multi_kernel(const DecJob* __restrict__ jobs,
                                                                         uint32_t njobs) {
  uint32_t lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (jobs[mid].tile0 <= blockIdx.x) lo = mid;
    else hi = mid - 1;
  }
  const DecJob& J = jobs[lo];
  varint_decimal_tile<kMode>(J.src, J.len, J.tile_base, J.scales, J.nvalues, J.scale, J.out, J.err, nullptr,
                             blockIdx.x - J.tile0);
}

// TimestampColumnReader::next (ColumnReader.cc:318-347) for writer == reader
// time zone rules (no adjustment): secs += epoch; nanos decoded from the
// trailing-zero code; one second back for negative times with nanos > 999999.
__global__ __launch_bounds__(256) void timestamp_kernel(int64_t* __restrict__ secs, int64_t* __restrict__ nanos,
                                                         uint64_t n, int64_t epoch) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int64_t nv = nanos[i];
  const uint64_t zeros = (uint64_t)nv & 7u;
  nv >>= 3;
  if (zeros != 0)
    for (uint64_t j = 0; j <= zeros; ++j) nv *= 10;
  int64_t t = secs[i] + epoch;
  if (t < 0 && nv > 999999) t -= 1;
  secs[i] = t;
  nanos[i] = nv;
}

}  // namespace

int launch_varint_tile_counts(Ctx* ctx, const uint8_t* d_src, uint64_t len, int64_t* d_counts, uint64_t* ntiles) {
  *ntiles = (len + kVTile - 1) / kVTile;
  if (*ntiles == 0) return ORCG_OK;
  hipLaunchKernelGGL(varint_count_kernel, dim3((unsigned)*ntiles), dim3(kVThreads), 0, ctx->stream, d_src, len,
                     d_counts);
  return hip_check(ctx, hipGetLastError(), "varint_count_kernel launch");
}

int launch_varint_decimal(Ctx* ctx, const uint8_t* d_src, uint64_t len, const int64_t* d_tile_base,
                          const int64_t* d_scales, uint64_t nvalues, int32_t scale, int mode, void* d_out,
                          uint8_t* d_keep) {
  const uint64_t ntiles = (len + kVTile - 1) / kVTile;
  if (ntiles == 0 || nvalues == 0) return ORCG_OK;
  if (mode == 3 && !d_keep) return set_error(ctx, ORCG_INVALID_ARGUMENT, "mode 3 needs a keep array");
  const dim3 grid((unsigned)ntiles), block(kVThreads);
  if (mode == 3)
    hipLaunchKernelGGL(varint_decimal_kernel<3>, grid, block, 0, ctx->stream, d_src, len, d_tile_base, d_scales,
                       nvalues, scale, d_out, ctx->d_err, d_keep);
  else if (mode == 2)
    hipLaunchKernelGGL(varint_decimal_kernel<2>, grid, block, 0, ctx->stream, d_src, len, d_tile_base, d_scales,
                       nvalues, scale, d_out, ctx->d_err, d_keep);
  else if (mode == 1)
    hipLaunchKernelGGL(varint_decimal_kernel<1>, grid, block, 0, ctx->stream, d_src, len, d_tile_base, d_scales,
                       nvalues, scale, d_out, ctx->d_err, d_keep);
  else
    hipLaunchKernelGGL(varint_decimal_kernel<0>, grid, block, 0, ctx->stream, d_src, len, d_tile_base, d_scales,
                       nvalues, scale, d_out, ctx->d_err, d_keep);
  return hip_check(ctx, hipGetLastError(), "varint_decimal_kernel launch");
}

int launch_decimal_jobs(Ctx* ctx, const DecJob* d_jobs, uint32_t njobs, uint64_t tiles, int mode) {
  if (njobs == 0 || tiles == 0) return ORCG_OK;
  if (tiles > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many decimal tiles");
  const dim3 grid((unsigned)tiles), block(kVThreads);
  if (mode == 1)
    hipLaunchKernelGGL(varint_decimal_multi_kernel<1>, grid, block, 0, ctx->stream, d_jobs, njobs);
  else
    hipLaunchKernelGGL(varint_decimal_multi_kernel<0>, grid, block, 0, ctx->stream, d_jobs, njobs);
  return hip_check(ctx, hipGetLastError(), "varint_decimal_multi_kernel launch");
}

int launch_timestamp(Ctx* ctx, int64_t* d_secs, int64_t* d_nanos, uint64_t n, int64_t epoch) {
  if (n == 0) return ORCG_OK;
  hipLaunchKernelGGL(timestamp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, d_secs, d_nanos,
                     n, epoch);
  return hip_check(ctx, hipGetLastError(), "timestamp_kernel launch");
}

}  // namespace orcg

// A no-op launch that makes HIP load this file's code object (warm_modules).
namespace orcg {
namespace {
__global__ void warm_decimal_kernel() {}
}  // namespace
void warm_decimal(hipStream_t s) { hipLaunchKernelGGL(warm_decimal_kernel, dim3(1), dim3(64), 0, s); }
}  // namespace orcg
