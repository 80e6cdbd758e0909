// RLEv1 integer decode on CDNA4 (gfx950).
//
// Replaces RleDecoderV1::next<T> (c++/src/RLEv1.cc:234-300) with readHeader
// (:180-191) and readLong (:154-170) — the integer / length / dictionary
// index streams of DIRECT and DICTIONARY column encodings (format 0.11
// files, e.g. examples/demo-11-*.orc). Format (site/specification/ORCv1.md,
// "Integer Run Length Encoding, version 1"): a signed control byte h >= 0 is
// a run of h + 3 values base + i * delta (delta a signed byte, base a varint);
// h < 0 is a literal group of -h base-128 varints. Signed streams zigzag.
//
// One wavefront per segment (header-aligned byte offset + first value index,
// host-planned). Runs (3..130 values) are expanded by all lanes. Literal
// groups are decoded 64 stream bytes at a time: every lane loads one byte,
// a ballot of "terminator" bytes (< 0x80) delimits the varints, each lane
// holding a terminator assembles its varint from its predecessors' bytes
// (cross-lane reads), and stores it at its rank.
#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

struct VWin {  // 256 stream bytes at `base` (descriptor-relative), one dword per lane
  uint32_t word = 0, base = 0xffffffffu;
  __device__ __forceinline__ void cover(__amdgpu_buffer_rsrc_t rs, uint32_t rel, uint32_t n, int lane) {
    if (base == 0xffffffffu || rel < base || rel + n > base + 256) {
      base = rel & ~3u;
      word = __builtin_amdgcn_raw_buffer_load_b32(rs, base + 4u * lane, 0, 0);
    }
  }
  __device__ __forceinline__ uint32_t byte(uint32_t rel) const {
    const uint32_t o = rel - base;
    return (rdlane(word, o >> 2) >> ((o & 3u) * 8)) & 0xffu;
  }
};

template <typename T>
__device__ __forceinline__ void put_v(T* dst, uint64_t o, uint64_t begin, uint64_t end, uint64_t v) {
  if (o >= begin && o < end) dst[o - begin] = (T)(int64_t)v;
}

// Wave-uniform varint at stream offset `pos` (readLong). Returns false when
// the stream ends first. Bits past 64 are dropped.
__device__ __forceinline__ bool uniform_varint(VWin& w, __amdgpu_buffer_rsrc_t rs, uint64_t bias, uint64_t& pos,
                                               uint64_t src_len, int lane, uint64_t& out) {
  uint64_t r = 0;
  uint32_t sh = 0;
  for (;;) {
    if (pos >= src_len) return false;
    const uint32_t rel = (uint32_t)(pos - bias);
    w.cover(rs, rel, 1, lane);
    const uint32_t b = w.byte(rel);
    ++pos;
    if (sh < 64) r |= (uint64_t)(b & 0x7fu) << sh;
    sh += 7;
    if (b < 0x80u) break;
  }
  out = r;
  return true;
}

template <typename T>
__global__ __launch_bounds__(kWave) void rlev1_kernel(const uint8_t* __restrict__ src, uint64_t src_len,
                                                       int is_signed, const uint64_t* __restrict__ segtab,
                                                       uint64_t nsegs, uint64_t value_begin, uint64_t nvalues,
                                                       T* __restrict__ dst, unsigned long long* err) {
  const uint64_t g = blockIdx.x;
  const int lane = (int)threadIdx.x;
  const uint64_t value_end = value_begin + nvalues;
  const uint64_t seg_start = segtab[2 * g];
  uint64_t vi = segtab[2 * g + 1];
  uint64_t seg_end = src_len, v_next = ~0ull;
  if (g + 1 < nsegs) {
    seg_end = segtab[2 * (g + 1)];
    v_next = segtab[2 * (g + 1) + 1];
  }
  if (seg_end > src_len) seg_end = src_len;
  if (vi >= value_end || v_next <= value_begin) return;

  const uintptr_t base_abs = ((uintptr_t)src + seg_start) & ~(uintptr_t)3;
  const uintptr_t end_abs = ((uintptr_t)src + src_len + 3) & ~(uintptr_t)3;
  const uint64_t span = (uint64_t)(end_abs - base_abs);
  const uint32_t nrec = span > 0xfffffff0ull ? 0xfffffff0u : (uint32_t)span;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base_abs, (short)0, (int)nrec, 0x00020000);
  const uint64_t bias = (uint64_t)(base_abs - (uintptr_t)src);
  const uint64_t lt_mask = (1ull << lane) - 1;  // lanes below this one

  VWin w;
  uint64_t pos = seg_start;
  while (pos < seg_end && vi < value_end) {
    const uint32_t rel = (uint32_t)(pos - bias);
    w.cover(rs, rel, 2, lane);
    const int32_t h = (int32_t)(int8_t)w.byte(rel);
    if (h >= 0) {
      // run: h + 3 values, signed-byte delta, varint base
      const uint32_t L = (uint32_t)h + 3;
      if (pos + 2 > src_len) { if (lane == 0) report(err, vi, kErrV1BadRead); return; }
      const int64_t delta = (int64_t)(int8_t)w.byte(rel + 1);
      pos += 2;
      uint64_t u;
      if (!uniform_varint(w, rs, bias, pos, src_len, lane, u)) { if (lane == 0) report(err, vi, kErrV1BadRead); return; }
      const uint64_t base = is_signed ? unzigzag(u) : u;
      for (uint32_t j = lane; j < L; j += kWave) put_v(dst, vi + j, value_begin, value_end, base + (uint64_t)j * (uint64_t)delta);
      vi += L;
    } else {
      uint32_t k = (uint32_t)(-h);  // literal varints left in the group
      uint64_t q = pos + 1;
      while (k > 0) {
        const uint64_t at = q + (uint64_t)lane;
        const bool valid = at < src_len;
        uint32_t b = 0;
        if (valid) {
          const uint32_t br = (uint32_t)(at - bias);
          b = (__builtin_amdgcn_raw_buffer_load_b32(rs, br & ~3u, 0, 0) >> ((br & 3u) * 8)) & 0xffu;
        }
        const uint64_t term = __ballot(valid && b < 0x80u);
        if (term == 0) {
          if (!valid) { if (lane == 0) report(err, vi, kErrV1BadRead); return; }
          // a varint longer than 64 bytes (corrupt but decodable): one at a time
          uint64_t u;
          if (!uniform_varint(w, rs, bias, q, src_len, lane, u)) { if (lane == 0) report(err, vi, kErrV1BadRead); return; }
          if (lane == 0) put_v(dst, vi, value_begin, value_end, is_signed ? unzigzag(u) : u);
          ++vi;
          --k;
          continue;
        }
        const uint32_t m = (uint32_t)__popcll(term);
        const uint32_t t = m < k ? m : k;
        const bool is_term = (term >> lane) & 1ull;
        const uint32_t rank = (uint32_t)__popcll(term & lt_mask);
        const uint64_t prev = term & lt_mask;
        const uint32_t start = prev ? (uint32_t)(64 - __clzll(prev)) : 0u;  // first byte of this lane's varint
        // assemble: byte i of the varint sits in lane start + i
        uint64_t r = 0;
        const uint32_t nb = (uint32_t)lane + 1 - start;
        for (uint32_t i = 0; i < 10; ++i) {
          const uint32_t srcl = start + i < 64 ? start + i : 63u;
          const uint32_t bi = (uint32_t)__shfl((int)b, (int)srcl, kWave);
          if (i < nb) r |= (uint64_t)(bi & 0x7fu) << (7 * i);
          if (!__any(i + 1 < nb && is_term && rank < t)) break;
        }
        if (is_term && rank < t) put_v(dst, vi + rank, value_begin, value_end, is_signed ? unzigzag(r) : r);
        // advance past the t-th varint
        const uint64_t last = __ballot(is_term && rank == t - 1);
        q += (uint64_t)__ffsll((unsigned long long)last);  // lane index + 1
        vi += t;
        k -= t;
      }
      pos = q;
    }
    if (pos > seg_end) { if (lane == 0) report(err, vi, kErrBadSegment); return; }
  }
  if (lane == 0 && v_next != ~0ull && vi < value_end && vi != v_next) report(err, vi, kErrBadSegment);
  // the last segment ran out of stream before the requested values
  if (lane == 0 && v_next == ~0ull && vi < value_end) report(err, vi, kErrV1BadRead);
}

}  // namespace

int launch_rlev1(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed, const uint64_t* d_segtab,
                 uint64_t nsegs, uint64_t value_begin, uint64_t nvalues, void* d_dst, int dst_bytes) {
  if (nsegs == 0 || nvalues == 0) return ORCG_OK;
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  const dim3 grid((unsigned)nsegs), block(kWave);
  const int sg = is_signed ? 1 : 0;
  if (dst_bytes == 8)
    hipLaunchKernelGGL(rlev1_kernel<int64_t>, grid, block, 0, ctx->stream, d_src, src_len, sg, d_segtab, nsegs,
                       value_begin, nvalues, (int64_t*)d_dst, ctx->d_err);
  else if (dst_bytes == 4)
    hipLaunchKernelGGL(rlev1_kernel<int32_t>, grid, block, 0, ctx->stream, d_src, src_len, sg, d_segtab, nsegs,
                       value_begin, nvalues, (int32_t*)d_dst, ctx->d_err);
  else if (dst_bytes == 2)
    hipLaunchKernelGGL(rlev1_kernel<int16_t>, grid, block, 0, ctx->stream, d_src, src_len, sg, d_segtab, nsegs,
                       value_begin, nvalues, (int16_t*)d_dst, ctx->d_err);
  else
    return set_error(ctx, ORCG_INVALID_ARGUMENT, "dst_bytes must be 8, 4 or 2");
  return hip_check(ctx, hipGetLastError(), "rlev1_kernel launch");
}

}  // namespace orcg
