// Byte RLE and Boolean RLE decode on CDNA4 (gfx950).
//
// Replaces ByteRleDecoderImpl::nextInternal (c++/src/ByteRLE.cc:449-505) and
// BooleanRleDecoderImpl::next (:578-643) — the PRESENT (null) streams,
// BOOLEAN / BYTE columns and UNION tags. Format (site/specification/
// ORCv1.md:672-695): a control byte h < 0x80 is a run of h + 3 copies of the
// next byte; h >= 0x80 is a literal group of 256 - h bytes. Booleans are the
// bits of those bytes, most significant first.
//
// One 256-thread workgroup per segment (run-aligned byte offset + index of
// its first decoded byte). The segment streams through an LDS window (4 KB of
// group starts + the longest group's tail, one coalesced 16-B load per
// thread); wave 0 walks the control bytes on the scalar unit, reading them
// from a 256-byte slice of the window held one dword per lane (v_readlane, no
// LDS round trip per group), into a group table {window offset, first decoded
// byte}; then the waves expand the groups, one group per wave at a time and
// one decoded byte per lane (runs: the value byte; literals: their byte), so
// every store instruction writes one contiguous span.
// In boolean mode every decoded byte becomes 8 output rows (chars 0/1).
#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

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

constexpr int kBThreads = 256;
constexpr uint32_t kBChunk = 4096;                 // groups starting in a window's first kBChunk bytes
constexpr uint32_t kBWinBytes = kBChunk + 256;     // + the longest group's tail (129 B) + the 16-B alignment
constexpr uint32_t kBMaxGroups = kBChunk / 2 + 16; // every group is >= 2 bytes (+ the alignment slack)

// segtab: (byte offset, first decoded-byte index) pairs. [begin, end) is in
// decoded bytes (kBool = false) or rows (kBool = true).
template <bool kBool>
__global__ __launch_bounds__(kBThreads) void byterle_kernel(const uint8_t* __restrict__ src, uint64_t src_len,
                                                            const uint64_t* __restrict__ segtab, uint64_t nsegs,
                                                            uint64_t begin, uint64_t nout, uint8_t* __restrict__ dst,
                                                            unsigned long long* err) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint32_t s_win[(kBWinBytes + 256) / 4];
  __shared__ uint16_t s_off[kBMaxGroups];
  __shared__ uint32_t s_start[kBMaxGroups + 1];
  __shared__ uint32_t s_ctl[4];
  const uint8_t* s_bytes = (const uint8_t*)s_win;
  const uint64_t g = blockIdx.x;
  const int tid = (int)threadIdx.x;
  const int lane = tid % kWave, wave = tid / kWave;
  const uint64_t end = begin + nout;
  const uint64_t scale = kBool ? 8 : 1;  // output units per decoded byte
  const uint64_t vend = (end + scale - 1) / scale;  // decoded bytes needed: index < vend
  const uint64_t seg_start = segtab[2 * g];
  uint64_t vi = segtab[2 * g + 1];
  uint64_t seg_end = src_len, v_next = ~0ull;
  if (g + 1 < nsegs) {
    seg_end = segtab[2 * (g + 1)];
    v_next = segtab[2 * (g + 1) + 1];
  }
  if (seg_end > src_len) seg_end = src_len;
  if (vi * scale >= end || (v_next != ~0ull && v_next * scale <= begin)) return;

  // range-checked descriptor over [seg_start & ~15, end of stream): loads
  // past the stream return zeros
  const uintptr_t base_abs = ((uintptr_t)src + seg_start) & ~(uintptr_t)15;
  const uintptr_t end_abs = ((uintptr_t)src + src_len + 3) & ~(uintptr_t)3;
  const uint64_t span = (uint64_t)(end_abs - base_abs);
  const uint32_t nrec = span > 0xfffff000ull ? 0xfffff000u : (uint32_t)span;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base_abs, (short)0, (int)nrec, 0x00020000);
  const uint64_t bias = (uint64_t)(base_abs - (uintptr_t)src);

  uint64_t pos = seg_start;
  while (pos < seg_end && vi < vend) {
    const uint32_t wrel = (uint32_t)(pos - bias) & ~15u;
    const uint64_t wpos = bias + wrel;  // stream offset of window byte 0
    for (uint32_t off = (uint32_t)tid * 16u; off < kBWinBytes; off += kBThreads * 16u)
      *(u4*)((char*)s_win + off) = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, wrel + off, 0, 0));
    __syncthreads();
    if (wave == 0) {
      // ByteRleDecoderImpl::readHeader / nextInternal's group loop
      // (ByteRLE.cc:378-388, 449-505) over the groups starting in the chunk
      uint32_t p = (uint32_t)(pos - wpos), v = 0, n = 0, stop = 0;
      const uint64_t seg_left = seg_end - wpos, src_left = src_len - wpos;
      const uint32_t lim = seg_left < kBChunk ? (uint32_t)seg_left : kBChunk;
      uint32_t sbase = 0xffffffffu, sword = 0;
      while (p < lim && vi + v < vend) {
        if (sbase == 0xffffffffu || p >= sbase + 256) {
          sbase = p & ~3u;
          sword = s_win[(sbase >> 2) + (uint32_t)lane];
        }
        const uint32_t o = p - sbase;
        const uint32_t h = (rdlane(sword, o >> 2) >> ((o & 3u) * 8u)) & 0xffu;
        const uint32_t glen = h < 0x80 ? 2u : 257u - h;    // run: h + 3 copies of one byte; literal: 256 - h bytes
        const uint32_t L = h < 0x80 ? h + 3u : 256u - h;
        if ((uint64_t)p + glen > src_left) {
          if (lane == 0) report(err, vi + v, kErrByteBadRead);
          stop = 1;
          break;
        }
        if (lane == 0) {
          s_off[n] = (uint16_t)p;
          s_start[n] = v;
        }
        ++n;
        p += glen;
        v += L;
        if ((uint64_t)p > seg_left) {  // the group runs past the segment
          if (lane == 0) report(err, vi + v, kErrBadSegment);
          stop = 1;
          break;
        }
      }
      if (lane == 0) {
        s_start[n] = v;
        s_ctl[0] = n;
        s_ctl[1] = p;
        s_ctl[2] = v;
        s_ctl[3] = stop;
      }
    }
    __syncthreads();
    const uint32_t n = s_ctl[0], np = s_ctl[1], nv = s_ctl[2], stop = s_ctl[3];
    // group-parallel expansion: wave w takes groups w, w + 4, ...; its lanes
    // take the group's decoded bytes lane, lane + 64, ... (a group is <= 130
    // bytes: at most three rounds); the group's table entries are uniform
    // loads, its literal bytes consecutive ones, and every round stores one
    // contiguous span (8 rows per lane in boolean mode)
    for (uint32_t gi = (uint32_t)wave; gi < n; gi += kBThreads / kWave) {
      const uint32_t o = s_off[gi];
      const uint32_t d0 = s_start[gi], len = s_start[gi + 1] - d0;
      const uint32_t h = s_bytes[o];
      const uint32_t rb = s_bytes[o + 1];
      for (uint32_t j = (uint32_t)lane; j < len; j += kWave) {
        const uint32_t b = h < 0x80 ? rb : s_bytes[o + 1u + j];
        emit<kBool>(dst, vi + d0 + j, b, begin, end);
      }
    }
    __syncthreads();  // the window and the table are rewritten by the next pass
    if (stop) return;
    pos = wpos + np;
    vi += nv;
  }
  if (tid == 0 && v_next != ~0ull && vi < vend && vi != v_next) report(err, vi, kErrBadSegment);
  // the last segment ran out of stream before the requested values
  if (tid == 0 && v_next == ~0ull && vi < vend) report(err, vi, kErrByteBadRead);
}

}  // namespace

int launch_byterle(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, const uint64_t* d_segtab, uint64_t nsegs,
                   bool boolean, uint64_t begin, uint64_t nout, uint8_t* d_dst) {
  if (nsegs == 0 || nout == 0) return ORCG_OK;
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  const dim3 grid((unsigned)nsegs), block(kBThreads);
  if (boolean)
    hipLaunchKernelGGL(byterle_kernel<true>, grid, block, 0, ctx->stream, d_src, src_len, d_segtab, nsegs, begin,
                       nout, d_dst, ctx->d_err);
  else
    hipLaunchKernelGGL(byterle_kernel<false>, grid, block, 0, ctx->stream, d_src, src_len, d_segtab, nsegs, begin,
                       nout, d_dst, ctx->d_err);
  return hip_check(ctx, hipGetLastError(), "byterle_kernel launch");
}

}  // namespace orcg
