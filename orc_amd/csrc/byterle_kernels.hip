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
// thread); the window's group starts are found in parallel (chunk exits,
// block hops, a workgroup scan: byterle_kernel below) and the decoded bytes
// are assembled a dword per lane through an owner map, stored coalesced.
// In boolean mode every decoded byte becomes 8 output rows (chars 0/1).
#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

// Write decoded byte `b` (decoded-byte index `i`) to the output; in boolean
// mode `ones` counts the set rows written (the column's non-null rows when
// the stream is a PRESENT stream).
template <bool kBool>
__device__ __forceinline__ void emit(uint8_t* dst, uint64_t i, uint32_t b, uint64_t begin, uint64_t end,
                                     uint32_t& ones) {
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
      ones += (uint32_t)__builtin_popcount(b & 0xffu);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t r = r0 + k;
        const uint32_t bit = (b >> (7 - k)) & 1u;
        if (r >= begin && r < end) {
          dst[r - begin] = (uint8_t)bit;
          ones += bit;
        }
      }
    }
  }
}

// Phase profiling (build with -DORCG_PHASE_PROF; scripts/ab_streams.py
// --phases): thread 0 of every workgroup adds the wall-clock ticks between
// consecutive marks to g_bphase[k].
#ifdef ORCG_PHASE_PROF
__device__ unsigned long long g_bphase[8];
#define BPROF_MARK(k)                                                        \
  do {                                                                       \
    if (threadIdx.x == 0) {                                                  \
      const uint64_t now_ = wall_clock64();                                  \
      atomicAdd(&g_bphase[k], (unsigned long long)(now_ - prof_last_));      \
      prof_last_ = now_;                                                     \
    }                                                                        \
  } while (0)
#else
#define BPROF_MARK(k) \
  do {                \
  } while (0)
#endif

constexpr int kBThreads = 256;
constexpr uint32_t kBChunk = 4096;                 // groups starting in a window's first kBChunk bytes
constexpr uint32_t kBWinBytes = kBChunk + 256;     // + the longest group's tail (129 B) + the 16-B alignment
constexpr uint32_t kBBlock = 128;                  // hop granularity of the chain walk
constexpr uint32_t kBBlocks = kBChunk / kBBlock;
constexpr uint16_t kBNone = 0xffffu;

typedef uint32_t bu4 __attribute__((ext_vector_type(4)));

// byte `i` (0..15, dynamic) of a 16-byte chunk held in four dwords
__device__ __forceinline__ uint32_t chunk_byte(bu4 c, uint32_t i) {
  const uint32_t w = i < 8 ? (i < 4 ? c.x : c.y) : (i < 12 ? c.z : c.w);
  return (w >> ((i & 3u) * 8u)) & 0xffu;
}

// Group header at byte h: (stream bytes, decoded bytes). A control byte
// below 0x80 is a run of h + 3 copies of the next byte (2 stream bytes), one
// at or above it a literal of 256 - h bytes (ByteRleDecoderImpl::readHeader,
// ByteRLE.cc:378-388).
__device__ __forceinline__ uint32_t group_len(uint32_t h) { return h < 0x80 ? 2u : 257u - h; }
__device__ __forceinline__ uint32_t group_dec(uint32_t h) { return h < 0x80 ? h + 3u : 256u - h; }

// segtab: (byte offset, first decoded-byte index) pairs. [begin, end) is in
// decoded bytes (kBool = false) or rows (kBool = true).
//
// One workgroup per segment; the segment streams through an LDS window of
// kBWinBytes (every group starting in its first kBChunk bytes is whole in
// it). A window's group starts are found in parallel instead of by a serial
// walk of the control bytes (the round-3 kernel spent ~200 ns per group
// there: 10 %-null PRESENT streams average ~4.5 bytes per group):
//   1. thread t owns bytes [16t, 16t + 16): for each of them, the first group
//      start at or past its chunk's end if a group started there (a
//      backward pass over the 16 bytes in registers) -> s_exit;
//   2. the same per 128-byte block, by hopping s_exit (<= 7 hops) -> s_exit2;
//   3. one lane hops the true chain block by block (<= 32 LDS reads) and
//      records each block's first group start;
//   4. each thread hops from its block's first start to its own chunk
//      (<= 7 hops) and walks the groups starting in its chunk (<= 8);
//   5. a workgroup scan of the groups' decoded bytes gives each group its
//      first decoded index;
//   6. the groups go to a table and an owner map (a scatter of group
//      indices at their first whole dword, then a prefix max); each thread
//      assembles dwords of decoded bytes from the groups the map names and
//      stores them straight out, consecutive dwords on consecutive lanes.
// Errors are reported per group with atomicMin on (decoded index, code), so
// the earliest in stream order wins, as the reference's serial loop raises
// it (ByteRleDecoderImpl::nextInternal, :449-505).
template <bool kBool>
__global__ __launch_bounds__(kBThreads) void byterle_kernel(const uint8_t* __restrict__ src, uint64_t src_len,
                                                            const uint64_t* __restrict__ segtab, uint64_t nsegs,
                                                            uint64_t begin, uint64_t nout, uint8_t* __restrict__ dst,
                                                            unsigned long long* err,
                                                            unsigned long long* __restrict__ ones_total,
                                                            const uint64_t* __restrict__ d_nout) {
#ifdef ORCG_PHASE_PROF
  uint64_t prof_last_ = wall_clock64();
#endif
  __shared__ __attribute__((aligned(16))) uint32_t s_win[(kBWinBytes + 256) / 4];
  // s_exit / s_exit2 (steps 1-4), then the stage of decoded bytes (step 6)
  __shared__ __attribute__((aligned(16))) uint16_t s_exit[2 * kBChunk];
  __shared__ uint16_t s_bentry[kBBlocks + 1];
  __shared__ uint32_t s_wsum[2][kBThreads / kWave];
  __shared__ uint32_t s_ctl[4];  // next window position, -, error seen
  // the window's groups: stream position, first decoded byte (step 6)
  __shared__ uint16_t s_gpos[kBChunk / 2 + 1];
  __shared__ uint32_t s_gdec[kBChunk / 2 + 1];
  __shared__ uint32_t s_wmax[kBThreads / kWave];
  uint16_t* s_exit2 = s_exit + kBChunk;
  const uint8_t* s_bytes = (const uint8_t*)s_win;
  const uint64_t g = blockIdx.x;
  const int tid = (int)threadIdx.x;
  const int lane = tid % kWave, wave = tid / kWave;
  const uint64_t end = begin + (d_nout ? *d_nout : nout);
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
  if (vi * scale >= end || (v_next != ~0ull && v_next * scale <= begin)) return;  // nothing to decode

  // range-checked descriptor over [seg_start & ~15, end of stream): loads
  // past the stream return zeros
  const uintptr_t base_abs = ((uintptr_t)src + seg_start) & ~(uintptr_t)15;
  const uintptr_t end_abs = ((uintptr_t)src + src_len + 3) & ~(uintptr_t)3;
  const uint64_t span = (uint64_t)(end_abs - base_abs);
  const uint32_t nrec = span > 0xfffff000ull ? 0xfffff000u : (uint32_t)span;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base_abs, (short)0, (int)nrec, 0x00020000);
  const uint64_t bias = (uint64_t)(base_abs - (uintptr_t)src);

  uint32_t ones = 0;  // set rows this thread wrote (boolean mode)
  bool stopped = false;
  uint64_t pos = seg_start;
  const uint32_t cs = (uint32_t)tid * 16u;  // my chunk
  while (pos < seg_end && vi < vend) {
    const uint32_t wrel = (uint32_t)(pos - bias) & ~15u;
    const uint64_t wpos = bias + wrel;  // stream offset of window byte 0
    for (uint32_t off = (uint32_t)tid * 16u; off < kBWinBytes; off += kBThreads * 16u)
      *(bu4*)((char*)s_win + off) = __builtin_bit_cast(bu4, __builtin_amdgcn_raw_buffer_load_b128(rs, wrel + off, 0, 0));
    if (tid <= (int)kBBlocks) s_bentry[tid] = kBNone;
    if (tid < 4) s_ctl[tid] = 0;
    const uint32_t p0 = (uint32_t)(pos - wpos);  // < 16
    const uint64_t seg_left = seg_end - wpos, src_left = src_len - wpos;
    const uint32_t lim = seg_left < kBChunk ? (uint32_t)seg_left : kBChunk;  // groups starting below lim
    __syncthreads();
    BPROF_MARK(0);

    // 1. chunk exits, backward over my 16 bytes (ex packed as bytes: 16..145)
    const bu4 mine = *(const bu4*)((const char*)s_win + cs);
    uint32_t pk[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 15; e >= 0; --e) {
      const uint32_t nx = (uint32_t)e + group_len(chunk_byte(mine, (uint32_t)e));
      uint32_t ex = nx;
      if (nx < 16) {
        const uint32_t w = nx < 8 ? (nx < 4 ? pk[0] : pk[1]) : (nx < 12 ? pk[2] : pk[3]);
        ex = (w >> ((nx & 3u) * 8u)) & 0xffu;
      }
      pk[e >> 2] |= ex << ((e & 3) * 8);
    }
    uint32_t q[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) q[e] = cs + ((pk[e >> 2] >> ((e & 3) * 8)) & 0xffu);
    {
      uint32_t w[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) w[k] = q[2 * k] | (q[2 * k + 1] << 16);
      *(bu4*)(s_exit + cs) = bu4{w[0], w[1], w[2], w[3]};
      *(bu4*)(s_exit + cs + 8) = bu4{w[4], w[5], w[6], w[7]};
    }
    __syncthreads();
    BPROF_MARK(1);

    // 2. block exits: hop chunk exits to my block's end
    const uint32_t be = (cs | (kBBlock - 1)) + 1;
#pragma unroll
    for (int h = 0; h < (int)(kBBlock / 16) - 1; ++h) {
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (q[e] < be) q[e] = s_exit[q[e]];
    }
    {
      uint32_t w[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) w[k] = q[2 * k] | (q[2 * k + 1] << 16);
      *(bu4*)(s_exit2 + cs) = bu4{w[0], w[1], w[2], w[3]};
      *(bu4*)(s_exit2 + cs + 8) = bu4{w[4], w[5], w[6], w[7]};
    }
    __syncthreads();
    BPROF_MARK(2);

    // 3. the chain, block by block (one lane)
    if (tid == 0) {
      for (uint32_t p = p0; p < lim; p = s_exit2[p]) s_bentry[p / kBBlock] = (uint16_t)p;
    }
    __syncthreads();
    BPROF_MARK(3);

    // 4. my chunk's first group start, then my groups
    uint32_t qs = kBNone;  // my first group start
    uint32_t ng = 0, dec = 0;
    if (cs < lim) {
      uint32_t p = s_bentry[cs / kBBlock];
      if (p != kBNone) {
        while (p < cs) p = s_exit[p];
        if (p < cs + 16 && p < lim) {
          qs = p;
          while (p < cs + 16 && p < lim) {
            const uint32_t h = chunk_byte(mine, p - cs);
            ++ng;
            dec += group_dec(h);
            p += group_len(h);
          }
          if (p >= lim) s_ctl[0] = p;  // the group crossing lim: the next window starts after it
        }
      }
    }
    // 5. workgroup scan of (groups, decoded bytes)
    const uint32_t ng_inc = wave_scan_u32(ng), dec_inc = wave_scan_u32(dec);
    if (lane == kWave - 1) {
      s_wsum[0][wave] = ng_inc;
      s_wsum[1][wave] = dec_inc;
    }
    __syncthreads();
    BPROF_MARK(4);
    uint32_t dec_base = dec_inc - dec, dec_total = 0;
#pragma unroll
    for (int w = 0; w < kBThreads / kWave; ++w) {
      const uint32_t d = s_wsum[1][w];
      dec_base += w < wave ? d : 0u;
      dec_total += d;
    }
    const uint32_t np = s_ctl[0];
    // 5b. my groups in stream order: the errors (the serial loop's checks, at
    // each group's decoded index; atomicMin keeps the earliest), none past
    // the bytes needed
    if (qs != kBNone) {
      uint32_t p = qs, d = dec_base;
      while (p < cs + 16 && p < lim) {
        const uint64_t di = vi + d;  // decoded index of this group's first byte
        if (di >= vend) break;       // the serial loop stops once enough bytes are decoded
        const uint32_t h = chunk_byte(mine, p - cs);
        const uint32_t gl = group_len(h), L = group_dec(h);
        if ((uint64_t)p + gl > src_left) {
          report(err, di, kErrByteBadRead);
          s_ctl[2] = 1;
          break;
        }
        if ((uint64_t)p + gl > seg_left) {  // the group runs past the segment
          report(err, di + L, kErrBadSegment);
          s_ctl[2] = 1;
          break;
        }
        p += gl;
        d += L;
      }
    }
    // 6. the window's decoded bytes straight to the output, one dword of them
    // (4 bytes, 32 rows) per thread per step, consecutive dwords on
    // consecutive lanes. A dword's bytes come from the last group starting at
    // or before its first byte (and the groups after it): the groups go to a
    // table (stream position, first decoded byte), each scatters its index
    // into an owner map at its first whole dword, and a prefix max fills the
    // map, 4096 dwords (16 KB of decoded bytes) per round.
    uint32_t ng_base = ng_inc - ng;
#pragma unroll
    for (int w = 0; w < kBThreads / kWave; ++w) ng_base += w < wave ? s_wsum[0][w] : 0u;
    if (qs != kBNone) {
      uint32_t p = qs, d = dec_base;
      for (uint32_t k = 0; k < ng; ++k) {
        s_gpos[ng_base + k] = (uint16_t)p;
        s_gdec[ng_base + k] = d;
        const uint32_t h = chunk_byte(mine, p - cs);
        p += group_len(h);
        d += group_dec(h);
      }
    }
    uint32_t* s_own = (uint32_t*)s_exit;  // s_exit's 16 KB, dead now
    constexpr uint32_t kRound = 2 * kBChunk * sizeof(uint16_t) / 4;  // dwords per round
    for (uint32_t sb = 0; sb < dec_total; sb += 4 * kRound) {
      for (uint32_t k = (uint32_t)tid; k < kRound; k += kBThreads) s_own[k] = 0;
      __syncthreads();
      if (qs != kBNone) {
        uint32_t d = dec_base;
        for (uint32_t k = 0; k < ng; ++k) {
          const uint32_t slot = d <= sb ? 0u : (d - sb + 3u) >> 2;
          if (slot < kRound) atomicMax(&s_own[slot], ng_base + k);
          d += group_dec(chunk_byte(mine, s_gpos[ng_base + k] - cs));
        }
      }
      __syncthreads();
      {
        // prefix max: thread t holds slots [16t, 16t + 16)
        bu4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *(const bu4*)(s_own + 16 * tid + 4 * k);
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          m = max(m, v[k].x); v[k].x = m;
          m = max(m, v[k].y); v[k].y = m;
          m = max(m, v[k].z); v[k].z = m;
          m = max(m, v[k].w); v[k].w = m;
        }
        uint32_t inc = m;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
          const uint32_t u = (uint32_t)__shfl_up((int)inc, o);
          if (lane >= o) inc = max(inc, u);
        }
        if (lane == kWave - 1) s_wmax[wave] = inc;
        uint32_t before = (uint32_t)__shfl_up((int)inc, 1);
        if (lane == 0) before = 0;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < kBThreads / kWave; ++w)
          if (w < wave) before = max(before, s_wmax[w]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k].x = max(v[k].x, before);
          v[k].y = max(v[k].y, before);
          v[k].z = max(v[k].z, before);
          v[k].w = max(v[k].w, before);
          *(bu4*)(s_own + 16 * tid + 4 * k) = v[k];
        }
      }
      __syncthreads();
      const uint32_t left = dec_total - sb;
      const uint32_t nd = left >= 4 * kRound ? kRound : (left + 3u) >> 2;
      for (uint32_t j = (uint32_t)tid; j < nd; j += kBThreads) {
        const uint32_t x0 = sb + 4u * j;  // decoded offset of the dword in the window
        uint32_t g = s_own[j];
        uint32_t d = s_gdec[g], p = s_gpos[g], h = s_bytes[p];
        uint32_t gend = d + group_dec(h);
        uint32_t w4;
        if (gend >= x0 + 4u) {
          if (h < 0x80) {
            w4 = (uint32_t)s_bytes[p + 1] * 0x01010101u;
          } else {
            const uint32_t so = p + 1u + (x0 - d);
            const uint32_t* w = s_win + (so >> 2);
            w4 = __builtin_amdgcn_alignbyte(w[1], w[0], so & 3u);
          }
        } else {
          w4 = 0;
          for (uint32_t b = 0; b < 4 && x0 + b < dec_total; ++b) {
            while (x0 + b >= gend) {
              ++g;
              d = s_gdec[g];
              p = s_gpos[g];
              h = s_bytes[p];
              gend = d + group_dec(h);
            }
            const uint32_t y = h < 0x80 ? s_bytes[p + 1] : s_bytes[p + 1u + (x0 + b - d)];
            w4 |= y << (8 * b);
          }
        }
        const uint64_t i = vi + x0;
        const uint32_t nb = dec_total - x0 < 4u ? dec_total - x0 : 4u;
        if constexpr (!kBool) {
          if (nb == 4 && i >= begin && i + 4 <= end && ((uintptr_t)(dst + (i - begin)) & 3u) == 0) {
            *(uint32_t*)(dst + (i - begin)) = w4;
            continue;
          }
        }
        for (uint32_t b = 0; b < nb; ++b) emit<kBool>(dst, i + b, (w4 >> (8 * b)) & 0xffu, begin, end, ones);
      }
      __syncthreads();  // the map is rebuilt by the next round
    }
    const bool stop = s_ctl[2] != 0;
    __syncthreads();  // the window and the tables are rewritten by the next pass
    BPROF_MARK(6);
    if (stop) {
      stopped = true;
      break;
    }
    pos = wpos + np;
    vi += dec_total;
  }
  if (kBool && ones_total) {
    for (int m = 32; m >= 1; m >>= 1) ones += (uint32_t)__shfl_xor((int)ones, m);
    if (lane == 0 && ones) atomicAdd(ones_total, (unsigned long long)ones);
  }
  BPROF_MARK(7);
  if (stopped) return;  // at an error (reported)
  if (tid == 0 && v_next != ~0ull && vi < vend && vi != v_next) report(err, vi, kErrBadSegment);
  // the last segment ran out of stream before the requested values
  if (tid == 0 && v_next == ~0ull && vi < vend) report(err, vi, kErrByteBadRead);
}

}  // namespace

int launch_byterle(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, const uint64_t* d_segtab, uint64_t nsegs,
                   bool boolean, uint64_t begin, uint64_t nout, uint8_t* d_dst, uint64_t* d_ones,
                   const uint64_t* d_nout) {
  if (nsegs == 0 || nout == 0) return ORCG_OK;
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  const dim3 grid((unsigned)nsegs), block(kBThreads);
  if (boolean)
    hipLaunchKernelGGL(byterle_kernel<true>, grid, block, 0, ctx->stream, d_src, src_len, d_segtab, nsegs, begin,
                       nout, d_dst, ctx->d_err, (unsigned long long*)d_ones, d_nout);
  else
    hipLaunchKernelGGL(byterle_kernel<false>, grid, block, 0, ctx->stream, d_src, src_len, d_segtab, nsegs, begin,
                       nout, d_dst, ctx->d_err, (unsigned long long*)nullptr, d_nout);
  return hip_check(ctx, hipGetLastError(), "byterle_kernel launch");
}

}  // namespace orcg

#ifdef ORCG_PHASE_PROF
extern "C" int orcg_debug_byterle_phases(unsigned long long* out, int n, int reset) {
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(orcg::g_bphase), sizeof(h)) != hipSuccess) return -1;
  for (int i = 0; i < n && i < 8; ++i) out[i] = h[i];
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(orcg::g_bphase), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// A no-op launch that makes HIP load this file's code object (warm_modules).
namespace orcg {
namespace {
__global__ void warm_byterle_kernel() {}
}  // namespace
void warm_byterle(hipStream_t s) { hipLaunchKernelGGL(warm_byterle_kernel, dim3(1), dim3(64), 0, s); }
}  // namespace orcg
