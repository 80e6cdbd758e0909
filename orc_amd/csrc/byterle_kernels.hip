// Byte RLE and Boolean RLE decode on CDNA4 (gfx950).
//
// Replaces ByteRleDecoderImpl::nextInternal (c++/src/ByteRLE.cc:449-505) and
// BooleanRleDecoderImpl::next (:578-643) — the PRESENT (null) streams,
// BOOLEAN / BYTE columns and UNION tags. Format (site/specification/
// ORCv1.md:672-695): a control byte h < 0x80 is a run of h + 3 copies of the
// next byte; h >= 0x80 is a literal group of 256 - h bytes. Booleans are the
// bits of those bytes, most significant first.
//
// One wavefront per segment (run-aligned byte offset + index of its first
// decoded byte). The wave walks the control bytes with wave-uniform scalar
// arithmetic out of a 256-byte slice held one dword per lane, kept covering
// the whole next group (control byte + up to 128 literal bytes): runs (<= 130
// bytes) and literals (<= 128 bytes) are expanded by all 64 lanes, literal
// bytes gathered from the slice with ds_bpermute (no memory round trip per
// group).
// In boolean mode every decoded byte becomes 8 output rows (chars 0/1).
#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

struct GWin {  // 256 stream bytes at `base` (descriptor-relative), one dword per lane
  uint32_t word = 0, base = 0xffffffffu;
  // make [rel, rel + need) resident (need <= 252)
  __device__ __forceinline__ void cover(__amdgpu_buffer_rsrc_t rs, uint32_t rel, int lane, uint32_t need = 4) {
    if (base == 0xffffffffu || rel < base || rel + need > base + 256) {
      base = rel & ~3u;
      word = __builtin_amdgcn_raw_buffer_load_b32(rs, base + 4u * lane, 0, 0);
    }
  }
  __device__ __forceinline__ uint32_t byte(uint32_t rel) const {
    const uint32_t o = rel - base;
    return (rdlane(word, o >> 2) >> ((o & 3u) * 8)) & 0xffu;
  }
};

// Write decoded byte `b` (decoded-byte index `i`) to the output.
template <bool kBool>
__device__ __forceinline__ void emit(uint8_t* dst, uint64_t i, uint32_t b, uint64_t begin, uint64_t end) {
  if constexpr (!kBool) {
    if (i >= begin && i < end) dst[i - begin] = (uint8_t)b;
  } else {
    // rows 8i .. 8i+7, MSB first
    const uint64_t r0 = 8 * i;
    if (r0 >= begin && r0 + 8 <= end && ((uintptr_t)(dst + (r0 - begin)) & 7u) == 0) {
      uint64_t w = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) w |= (uint64_t)((b >> (7 - k)) & 1u) << (8 * k);
      *(uint64_t*)(dst + (r0 - begin)) = w;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t r = r0 + k;
        if (r >= begin && r < end) dst[r - begin] = (uint8_t)((b >> (7 - k)) & 1u);
      }
    }
  }
}

// segtab: (byte offset, first decoded-byte index) pairs. [begin, end) is in
// decoded bytes (kBool = false) or rows (kBool = true).
template <bool kBool>
__global__ __launch_bounds__(kWave) void byterle_kernel(const uint8_t* __restrict__ src, uint64_t src_len,
                                                         const uint64_t* __restrict__ segtab, uint64_t nsegs,
                                                         uint64_t begin, uint64_t nout, uint8_t* __restrict__ dst,
                                                         unsigned long long* err) {
  const uint64_t g = blockIdx.x;
  const int lane = (int)threadIdx.x;
  const uint64_t end = begin + nout;
  const uint64_t scale = kBool ? 8 : 1;  // output units per decoded byte
  const uint64_t seg_start = segtab[2 * g];
  uint64_t vi = segtab[2 * g + 1];
  uint64_t seg_end = src_len, v_next = ~0ull;
  if (g + 1 < nsegs) {
    seg_end = segtab[2 * (g + 1)];
    v_next = segtab[2 * (g + 1) + 1];
  }
  if (seg_end > src_len) seg_end = src_len;
  if (vi * scale >= end || (v_next != ~0ull && v_next * scale <= begin)) return;

  const uintptr_t base_abs = ((uintptr_t)src + seg_start) & ~(uintptr_t)3;
  const uintptr_t end_abs = ((uintptr_t)src + src_len + 3) & ~(uintptr_t)3;
  const uint64_t span = (uint64_t)(end_abs - base_abs);
  const uint32_t nrec = span > 0xfffffff0ull ? 0xfffffff0u : (uint32_t)span;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base_abs, (short)0, (int)nrec, 0x00020000);
  const uint64_t bias = (uint64_t)(base_abs - (uintptr_t)src);

  GWin w;
  uint64_t pos = seg_start;
  while (pos < seg_end && vi * scale < end) {
    const uint32_t rel = (uint32_t)(pos - bias);
    w.cover(rs, rel, lane, 132);
    const uint32_t h = w.byte(rel);
    if (h < 0x80) {  // run of h + 3 copies (readHeader, ByteRLE.cc:378-388)
      const uint32_t L = h + 3;
      if (pos + 2 > src_len) { if (lane == 0) report(err, vi, kErrByteBadRead); return; }
      const uint32_t b = w.byte(rel + 1);
      for (uint32_t j = lane; j < L; j += kWave) emit<kBool>(dst, vi + j, b, begin, end);
      pos += 2;
      vi += L;
    } else {  // literal group of 256 - h bytes
      const uint32_t L = 256 - h;
      if (pos + 1 + L > src_len) { if (lane == 0) report(err, vi, kErrByteBadRead); return; }
      for (uint32_t j0 = 0; j0 < L; j0 += kWave) {
        // every lane takes part in the gather (a wave-uniform loop)
        const uint32_t j = j0 + (uint32_t)lane;
        const uint32_t o = rel + 1 + j - w.base;
        const uint32_t wd = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((o >> 2) & 63u) * 4, (int)w.word);
        if (j < L) emit<kBool>(dst, vi + j, (wd >> ((o & 3u) * 8)) & 0xffu, begin, end);
      }
      pos += 1 + L;
      vi += L;
    }
    if (pos > seg_end) { if (lane == 0) report(err, vi, kErrBadSegment); return; }
  }
  if (lane == 0 && v_next != ~0ull && vi * scale < end && vi != v_next) report(err, vi, kErrBadSegment);
  // the last segment ran out of stream before the requested values
  if (lane == 0 && v_next == ~0ull && vi * scale < end) report(err, vi, kErrByteBadRead);
}

}  // namespace

int launch_byterle(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, const uint64_t* d_segtab, uint64_t nsegs,
                   bool boolean, uint64_t begin, uint64_t nout, uint8_t* d_dst) {
  if (nsegs == 0 || nout == 0) return ORCG_OK;
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  const dim3 grid((unsigned)nsegs), block(kWave);
  if (boolean)
    hipLaunchKernelGGL(byterle_kernel<true>, grid, block, 0, ctx->stream, d_src, src_len, d_segtab, nsegs, begin,
                       nout, d_dst, ctx->d_err);
  else
    hipLaunchKernelGGL(byterle_kernel<false>, grid, block, 0, ctx->stream, d_src, src_len, d_segtab, nsegs, begin,
                       nout, d_dst, ctx->d_err);
  return hip_check(ctx, hipGetLastError(), "byterle_kernel launch");
}

}  // namespace orcg
