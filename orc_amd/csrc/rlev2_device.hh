// Device helpers shared by the RLEv2 kernels: width tables, the big-endian
// bit-field extract, wavefront scans and the run-header parser.
#pragma once

#include "orcg_internal.hh"

namespace orcg {
namespace dev {

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

constexpr int kWave = 64;
constexpr int kMaxRunUnroll = 8;  // 512 values / 64 lanes

// FBSToBitWidthMap (c++/src/RLEV2Util.cc:24-26)
__device__ __forceinline__ uint32_t fbs_width(uint32_t code) {
  if (code < 24) return code + 1;
  const uint64_t t = 0x40383028201E1C1Aull;  // 26,28,30,32,40,48,56,64
  return (uint32_t)((t >> (8 * (code - 24))) & 0xff);
}

// getClosestFixedBits (c++/src/RLEV2Util.hh:38-44, RLEV2Util.cc:29-32)
__device__ __forceinline__ uint32_t closest_fixed_bits(uint32_t n) {
  if (n == 0) return 1;
  if (n <= 24) return n;
  if (n <= 26) return 26;
  if (n <= 28) return 28;
  if (n <= 30) return 30;
  if (n <= 32) return 32;
  if (n <= 40) return 40;
  if (n <= 48) return 48;
  if (n <= 56) return 56;
  return 64;
}

// unZigZag (c++/src/RLE.hh:32-34)
__device__ __forceinline__ uint64_t unzigzag(uint64_t v) { return (v >> 1) ^ (0 - (v & 1)); }

// Values the wave agrees on but the compiler cannot prove uniform (loaded
// from LDS or computed from such loads): readfirstlane puts them in SGPRs, so
// the code that depends on them stays scalar (a v_readlane with a VGPR lane
// index becomes a waterfall loop).
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// The W-bit big-endian field starting `sh` bits into byte `rel`, given the
// three little-endian dwords at (rel & ~3). W in 1..64, W + sh <= 64 for
// every width the format can produce (non byte-multiple widths are <= 30).
__device__ __forceinline__ uint64_t field(u32x3 w, uint32_t rel, uint32_t sh, uint32_t W) {
  const uint32_t r = rel & 3u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(w.y, w.x, r);
  const uint32_t hi = __builtin_amdgcn_alignbyte(w.z, w.y, r);
  const uint64_t be = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
  return (be << sh) >> (64 - W);
}

// Wavefront inclusive prefix sums on DPP (no LDS round trips): Kogge-Stone
// inside each 16-lane row with row_shr:1,2,4,8, then row_bcast:15 (rows 1,3)
// and row_bcast:31 (rows 2,3) carry the row totals across. Requires all 64
// lanes active. Invalid source lanes read 0 (bound_ctrl).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kCtrl, kRowMask, 0xf, true);
}

__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t x) {
  x += dpp0<0x111, 0xf>(x);  // row_shr:1
  x += dpp0<0x112, 0xf>(x);  // row_shr:2
  x += dpp0<0x114, 0xf>(x);  // row_shr:4
  x += dpp0<0x118, 0xf>(x);  // row_shr:8
  x += dpp0<0x142, 0xa>(x);  // row_bcast:15
  x += dpp0<0x143, 0xc>(x);  // row_bcast:31
  return x;
}

template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint64_t dpp0_64(uint64_t x) {
  const uint32_t lo = dpp0<kCtrl, kRowMask>((uint32_t)x), hi = dpp0<kCtrl, kRowMask>((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_inclusive_scan(uint64_t x, int /*lane*/ = 0) {
  x += dpp0_64<0x111, 0xf>(x);
  x += dpp0_64<0x112, 0xf>(x);
  x += dpp0_64<0x114, 0xf>(x);
  x += dpp0_64<0x118, 0xf>(x);
  x += dpp0_64<0x142, 0xa>(x);
  x += dpp0_64<0x143, 0xc>(x);
  return x;
}

// Value of lane 63 (wave-uniform, scalar register).
__device__ __forceinline__ uint64_t last_lane(uint64_t x) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), 63) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
}

__device__ __forceinline__ void report(unsigned long long* err, uint64_t value_index, uint32_t code) {
  atomicMin(err, (unsigned long long)((value_index << 8) | code));
}

template <typename T>
__device__ __forceinline__ void put(T* dst, uint64_t idx, uint64_t v) {
  dst[idx] = (T)(int64_t)v;
}

// A parsed run header (RleDecoderV2::next* header logic, RleDecoderV2.cc:
// 184-435). Offsets are relative to the run's first byte.
struct Run {
  uint32_t kind;   // 0 SHORT_REPEAT, 1 DIRECT, 2 PATCHED_BASE, 3 DELTA
  uint32_t W;      // bit width of the packed data (0 = fixed delta)
  uint32_t L;      // values in the run
  uint32_t data;   // offset of the packed data
  uint32_t bytes;  // total run length in bytes
  uint32_t pbs, pl, cfb;
  uint64_t a;      // SR value (unzigzagged) / PATCHED base / DELTA first value
  uint64_t b;      // DELTA delta base
  uint32_t err;    // DevErr
};

// Parses the header whose first byte is byte(0); `avail` = stream bytes from
// the run start to the end of the stream (for the truncation errors, checked
// in the order the reference reads its bytes). `lim` bounds how far the
// header may be read (window size); longer varints report a bad read.
template <class ByteFn>
__device__ __forceinline__ Run parse_run(ByteFn byte, uint64_t avail, uint32_t lim, int is_signed) {
  Run r;
  r.pbs = r.pl = r.cfb = 0;
  r.a = r.b = 0;
  r.err = kErrNone;
  const uint32_t fb = byte(0);
  r.kind = fb >> 6;
  if (r.kind == 0) {
    const uint32_t nb = ((fb >> 3) & 7u) + 1u;
    r.W = 8 * nb;
    r.L = (fb & 7u) + 3u;
    r.data = 1;
    r.bytes = 1 + nb;
    if (r.bytes > avail) { r.err = kErrBadRead; return r; }
    uint64_t v = 0;
    for (uint32_t i = 0; i < nb; ++i) v = (v << 8) | byte(1 + i);
    r.a = is_signed ? unzigzag(v) : v;
    return r;
  }
  if (avail < 2) { r.err = kErrBadRead; r.L = 0; r.W = 0; r.bytes = 0; r.data = 0; return r; }
  r.L = ((fb & 1u) << 8 | byte(1)) + 1;
  if (r.kind == 1 || r.kind == 2) {
    r.W = fbs_width((fb >> 1) & 0x1fu);
    r.data = 2;
    if (r.kind == 2) {
      if (avail < 4) { r.err = kErrBadRead; return r; }
      const uint32_t third = byte(2), fourth = byte(3);
      const uint32_t bw = (third >> 5) + 1u;
      r.pbs = fbs_width(third & 0x1fu);
      const uint32_t pgw = (fourth >> 5) + 1u;
      r.pl = fourth & 0x1fu;
      if (r.pl == 0) { r.err = kErrPatchedPl0; return r; }
      if (avail < 4 + bw) { r.err = kErrBadRead; return r; }
      uint64_t base = 0;
      for (uint32_t i = 0; i < bw; ++i) base = (base << 8) | byte(4 + i);
      const uint64_t m = 1ull << (bw * 8 - 1);
      if (base & m) base = 0 - (base & ~m);  // sign-magnitude (:311-317)
      r.a = base;
      r.data = 4 + bw;
      if (r.data + (r.W * r.L + 7) / 8 > avail) { r.err = kErrBadRead; return r; }
      if (r.pbs + pgw > 64) { r.err = kErrPatchedWidth; return r; }
      r.cfb = closest_fixed_bits(r.pbs + pgw);
    }
    r.bytes = r.data + (r.W * r.L + 7) / 8 + (r.cfb * r.pl + 7) / 8;
    if (r.bytes > avail) r.err = kErrBadRead;
    return r;
  }
  // DELTA
  const uint32_t fbo = (fb >> 1) & 0x1fu;
  r.W = fbo ? fbs_width(fbo) : 0u;
  uint32_t q = 2;
  uint64_t vals[2] = {0, 0};
  for (int k = 0; k < 2; ++k) {
    uint64_t acc = 0;
    uint32_t shift = 0, b;
    do {
      if (q >= avail || q >= lim) { r.err = kErrBadRead; return r; }
      b = byte(q);
      ++q;
      if (shift < 64) acc |= (uint64_t)(b & 0x7fu) << shift;
      shift += 7;
    } while (b >= 0x80u);
    vals[k] = acc;
  }
  r.a = is_signed ? unzigzag(vals[0]) : vals[0];
  r.b = unzigzag(vals[1]);
  if (r.W != 0 && r.L < 2) { r.err = kErrDeltaLength; return r; }
  r.data = q;
  r.bytes = q + (r.W ? (r.W * (r.L - 2) + 7) / 8 : 0);
  if (r.bytes > avail) r.err = kErrBadRead;
  return r;
}

}  // namespace dev
}  // namespace orcg
