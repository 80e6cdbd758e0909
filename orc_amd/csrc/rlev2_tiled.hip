// RLEv2 decode, tiled through LDS (the default kernels).
//
// One 256-thread workgroup per segment. The segment's bytes stream through an
// LDS window filled by buffer_load ... lds (LDS-DMA, 1 KB per wave
// instruction, range-checked so reads past the stream return zeros). The run
// headers are walked in LDS (RleDecoderV2::next's run loop,
// c++/src/RleDecoderV2.cc:132-170) into a run table, and waves expand runs
// round-robin straight out of LDS:
//   SHORT_REPEAT  broadcast                                      (:184-222)
//   DIRECT        per-lane big-endian W-bit extract + zigzag     (:224-248)
//   PATCHED_BASE  extract + base, patches applied in registers   (:250-370)
//   DELTA         wavefront int64 inclusive scan                 (:372-435)
// A window holds every run that STARTS in its first (kWin - kMaxRun) bytes;
// runs are at most kMaxRun bytes, so they end inside it. The next window
// starts at the first unprocessed run.
//
// Two structures (template kPipe):
//  * kPipe = false: all 4 waves fill one window, wave 0 walks, 4 waves expand.
//  * kPipe = true : wave 0 is the producer (fill window k+1 by LDS-DMA, wait,
//    walk it) while waves 1-3 expand window k; double-buffered windows and
//    run tables, one raw s_barrier per window. The producer never stores and
//    the consumers never wait on vmcnt, so output stores stay in flight across
//    windows.
#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr uint32_t kMaxRun = 4608;  // >= 4356, the longest legal run
constexpr int kMaxRuns = 512;       // run-table capacity per window

// kOpt bits
constexpr int kOptNTStore = 1;  // non-temporal output stores (streamed, never re-read)
constexpr int kOptNTLoad = 2;   // non-temporal LDS-DMA loads of the stream
constexpr int kOptReuse = 4;    // carry the window tail over in LDS; never load past the segment
constexpr int kOptFast = 8;     // predicate-free path for full DIRECT runs inside the output range

template <int kOpt, typename T>
__device__ __forceinline__ void store1(T* p, uint64_t v) {
  if constexpr ((kOpt & kOptNTStore) != 0) __builtin_nontemporal_store((T)(int64_t)v, p);
  else *p = (T)(int64_t)v;
}

__device__ __forceinline__ uint32_t lds_byte(const uint32_t* w, uint32_t o) {
  return (w[o >> 2] >> ((o & 3u) * 8)) & 0xffu;
}

__device__ __forceinline__ u32x3 lds12(const uint32_t* w, uint32_t o) {
  const uint32_t i = o >> 2;
  u32x3 r;
  r.x = w[i];
  r.y = w[i + 1];
  r.z = w[i + 2];
  return r;
}

// Run headers are parsed from a 256-byte slice of the LDS window held one
// dword per lane and read back with v_readlane: one LDS round trip per slice
// instead of one per header byte. kHdrLim bounds how far a header may reach
// (DELTA's two varints take <= 22 bytes; longer ones are corrupt).
constexpr uint32_t kHdrLim = 64;

struct LaneWin {
  uint32_t word = 0, base = 0xffffffffu;
  __device__ __forceinline__ void load(const uint32_t* win, uint32_t hoff, uint32_t nwords, int lane) {
    base = hoff & ~3u;
    uint32_t idx = (base >> 2) + (uint32_t)lane;
    if (idx >= nwords) idx = nwords - 1;
    word = win[idx];
  }
  // make sure [hoff, hoff + kHdrLim) is inside the slice
  __device__ __forceinline__ void cover(const uint32_t* win, uint32_t hoff, uint32_t nwords, int lane) {
    if (base == 0xffffffffu || hoff < base || hoff + kHdrLim > base + 256) load(win, hoff, nwords, lane);
  }
  __device__ __forceinline__ uint32_t byte(uint32_t o) const {
    o -= base;
    return (rdlane(word, o >> 2) >> ((o & 3u) * 8)) & 0xffu;
  }
};

// Expand one run (already validated by the walk) with one wave.
template <int kOpt, typename T>
__device__ __forceinline__ void expand_run(const uint32_t* win, uint32_t nwords, uint32_t hoff, uint64_t v0,
                                           int is_signed, uint64_t value_begin, uint64_t value_end, T* dst,
                                           int lane) {
  LaneWin hw;
  hw.load(win, hoff, nwords, lane);
  const Run r = parse_run([&](uint32_t i) { return hw.byte(hoff + i); }, ~0ull, kHdrLim, is_signed);
  const uint32_t L = r.L;
  if (v0 + L <= value_begin || v0 >= value_end) return;  // outside the requested rows
  const uint32_t d = hoff + r.data;  // LDS offset of the packed data
  const uint32_t niter = (L + kWave - 1) / kWave;

  if (r.kind == 0) {
    const uint64_t o = v0 + (uint64_t)lane;
    if ((uint32_t)lane < L && o >= value_begin && o < value_end) store1<kOpt>(dst + (o - value_begin), r.a);
    return;
  }
  if (r.kind == 1) {
    const uint32_t W = r.W;
    if ((kOpt & kOptFast) && L == 512 && v0 >= value_begin && v0 + 512 <= value_end) {
      // Full run entirely inside the output range: no per-value predicates.
      T* out = dst + (v0 - value_begin);
      if (W == 64) {
        // 8 bytes per value at d + 8j: one uniform byte alignment per run
        const uint32_t r4 = d & 3u;
#pragma unroll
        for (int it = 0; it < kMaxRunUnroll; ++it) {
          const uint32_t j = it * kWave + lane;
          const u32x3 w = lds12(win, d + 8 * j);
          const uint32_t lo = __builtin_amdgcn_alignbyte(w.y, w.x, r4);
          const uint32_t hi = __builtin_amdgcn_alignbyte(w.z, w.y, r4);
          uint64_t v = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
          if (is_signed) v = unzigzag(v);
          store1<kOpt>(out + j, v);
        }
      } else {
#pragma unroll
        for (int it = 0; it < kMaxRunUnroll; ++it) {
          const uint32_t j = it * kWave + lane;
          const uint32_t bit = j * W;
          const uint32_t br = d + (bit >> 3);
          uint64_t v = field(lds12(win, br), br, bit & 7u, W);
          if (is_signed) v = unzigzag(v);
          store1<kOpt>(out + j, v);
        }
      }
      return;
    }
#pragma unroll
    for (int it = 0; it < kMaxRunUnroll; ++it) {
      if ((uint32_t)it < niter) {
        const uint32_t j = it * kWave + lane;
        const uint32_t bit = j * W;
        const uint32_t br = d + (bit >> 3);
        uint64_t v = field(lds12(win, br), br, bit & 7u, W);
        if (is_signed) v = unzigzag(v);
        const uint64_t o = v0 + j;
        if (j < L && o >= value_begin && o < value_end) store1<kOpt>(dst + (o - value_begin), v);
      }
    }
    return;
  }
  if (r.kind == 2) {
    // PATCHED_BASE. The patch list (<= 31 entries of cfb bits) is held one
    // entry per lane; positions are the inclusive prefix sum of the gap
    // fields (an escape entry, gap 255 / patch 0, contributes its 255), and
    // the entries are applied in order exactly like nextPatched's loop
    // (:340-366) with adjustGapAndPatch (:250-271): escapes only advance, a
    // patch that does not move past the previous one stalls the walk, and
    // positions >= L are never reached. Low register footprint: one 64-value
    // chunk of literals at a time, patches consumed with a scalar cursor.
    const uint32_t W = r.W;
    const uint32_t p0 = d + (W * L + 7) / 8;  // patch list
    uint64_t entry = 0;
    if ((uint32_t)lane < r.pl) {
      const uint32_t bit = lane * r.cfb;
      const uint32_t br = p0 + (bit >> 3);
      entry = field(lds12(win, br), br, bit & 7u, r.cfb);
    }
    const uint64_t pmask = (1ull << r.pbs) - 1;  // pbs <= 63 (checked by the walk)
    const uint32_t gap = (uint32_t)lane < r.pl ? (uint32_t)(entry >> r.pbs) : 0u;  // <= 255
    const uint32_t cum = wave_scan_u32(gap);  // positions (<= 31 * 255)
    const uint64_t patch = entry & pmask;
    const uint32_t p_lo = (uint32_t)patch, p_hi = (uint32_t)(patch >> 32);
    // scalar pass: which entries apply (bitmask over entries)
    uint64_t applied = 0;
    {
      uint32_t prev = 0;
      bool first = true;
      for (uint32_t k = 0; k < r.pl; ++k) {
        const uint32_t c = rdlane(cum, k), g = rdlane(gap, k);
        const bool esc = g == 255 && rdlane(p_lo, k) == 0 && rdlane(p_hi, k) == 0;
        if (esc) continue;
        if ((!first && c == prev) || c >= L) break;
        applied |= 1ull << k;
        prev = c;
        first = false;
      }
    }
    uint64_t todo = applied;
#pragma unroll 1
    for (uint32_t it = 0; it < niter; ++it) {
      const uint32_t j = it * kWave + lane;
      const uint32_t bit = j * W;
      const uint32_t br = d + (bit >> 3);
      uint64_t lit = field(lds12(win, br), br, bit & 7u, W);
      // patches whose position falls in this chunk (positions increase)
      while (todo) {
        const uint32_t k = (uint32_t)__builtin_ctzll(todo);
        const uint32_t c = rdlane(cum, k);
        if (c / kWave != it) break;
        const uint64_t pv = ((uint64_t)rdlane(p_hi, k) << 32) | rdlane(p_lo, k);
        if ((uint32_t)lane == c % kWave) lit |= pv << (W & 63u);
        todo &= todo - 1;
      }
      const uint64_t o = v0 + j;
      if (j < L && o >= value_begin && o < value_end) store1<kOpt>(dst + (o - value_begin), r.a + lit);
    }
    return;
  }
  // DELTA
  if (r.W == 0) {
#pragma unroll
    for (int it = 0; it < kMaxRunUnroll; ++it) {
      const uint32_t j = it * kWave + lane;
      const uint64_t o = v0 + j;
      if ((uint32_t)it < niter && j < L && o >= value_begin && o < value_end)
        store1<kOpt>(dst + (o - value_begin), r.a + (uint64_t)j * r.b);
    }
    return;
  }
  const uint32_t W = r.W;
  const uint64_t v1 = r.a + r.b;
  const bool neg = (int64_t)r.b < 0;
  uint64_t carry = 0;  // wave-uniform running |delta| total
  if (W <= 26) {
    // 64 deltas of <= 26 bits sum below 2^32: scan in 32 bits
#pragma unroll 1
    for (uint32_t it = 0; it < niter; ++it) {
      const uint32_t j = it * kWave + lane;
      const int32_t k = (int32_t)j - 2;
      uint32_t dlt = 0;
      if (k >= 0 && j < L) {
        const uint32_t bit = (uint32_t)k * W;
        const uint32_t br = d + (bit >> 3);
        dlt = (uint32_t)field(lds12(win, br), br, bit & 7u, W);
      }
      const uint32_t s32 = wave_scan_u32(dlt);
      const uint64_t sum = carry + s32;
      carry += (uint32_t)__builtin_amdgcn_readlane((int)s32, 63);
      const uint64_t v = j == 0 ? r.a : (j == 1 ? v1 : (neg ? v1 - sum : v1 + sum));
      const uint64_t o = v0 + j;
      if (j < L && o >= value_begin && o < value_end) store1<kOpt>(dst + (o - value_begin), v);
    }
    return;
  }
#pragma unroll 1
  for (uint32_t it = 0; it < niter; ++it) {
    const uint32_t j = it * kWave + lane;
    const int32_t k = (int32_t)j - 2;
    uint64_t dlt = 0;
    if (k >= 0 && j < L) {
      const uint32_t bit = (uint32_t)k * W;
      const uint32_t br = d + (bit >> 3);
      dlt = field(lds12(win, br), br, bit & 7u, W);
    }
    const uint64_t sum = wave_inclusive_scan(dlt) + carry;
    carry = last_lane(sum);
    const uint64_t v = j == 0 ? r.a : (j == 1 ? v1 : (neg ? v1 - sum : v1 + sum));
    const uint64_t o = v0 + j;
    if (j < L && o >= value_begin && o < value_end) store1<kOpt>(dst + (o - value_begin), v);
  }
}

// Fill `bytes` (multiple of 1 KB) of LDS at `win` from descriptor offset
// `wrel` with `nw` waves (wave index `w`).
template <int kOpt>
__device__ __forceinline__ void fill(uint32_t* win, __amdgpu_buffer_rsrc_t rs, uint32_t wrel,
                                     uint32_t bytes, int w, int nw, int lane) {
  for (uint32_t off = w * 1024u; off < bytes; off += nw * 1024u)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)((char*)win + off),
                                             16, wrel + off + lane * 16, 0, 0,
                                             (kOpt & kOptNTLoad) ? 2 : 0);
}

struct WalkResult {
  uint32_t n, stop, dpos, dval;
};

// Wave-uniform header walk over the window [wpos, wpos + kWin): records runs
// starting at pos.. into (run_off, run_val) until the next run starts past
// kWin - kMaxRun, leaves the segment, or the table is full.
template <uint32_t kWin>
__device__ __forceinline__ WalkResult walk(const uint32_t* win, uint32_t* run_off, uint32_t* run_val,
                                           uint64_t wpos, uint64_t pos, uint64_t vi, uint64_t seg_end,
                                           uint64_t src_len, uint64_t value_end, int is_signed,
                                           unsigned long long* err, int lane, uint32_t lim = kWin) {
  constexpr uint32_t kChunk = kWin - kMaxRun;
  uint64_t p = pos, v = vi;
  uint32_t n = 0, stop = 0;
  LaneWin hw;
  while (p < seg_end && v < value_end && n < (uint32_t)kMaxRuns) {
    const uint32_t lp = (uint32_t)(p - wpos);
    if (lp >= kChunk && n > 0) break;  // starts in the next window
    hw.cover(win, lp, kWin / 4 + 8, lane);
    const Run r = parse_run([&](uint32_t i) { return hw.byte(lp + i); }, src_len - p, kHdrLim, is_signed);
    uint32_t e = r.err;
    if (e == kErrNone && p + r.bytes > seg_end) e = kErrBadSegment;
    if (e == kErrNone && lp + r.bytes > lim) e = kErrBadRead;  // only a corrupt varint gets here
    if (e != kErrNone) {
      if (lane == 0) report(err, v, e);
      stop = 1;
      break;
    }
    if (lane == 0) {
      run_off[n] = lp;
      run_val[n] = (uint32_t)(v - vi);
    }
    ++n;
    p += r.bytes;
    v += r.L;
  }
  return WalkResult{n, stop, (uint32_t)(p - pos), (uint32_t)(v - vi)};
}

__device__ __forceinline__ void lds_barrier() {
  // LDS ordering only: never drains the output stores (vmcnt).
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <typename T, bool kPositions, int kOpt, int kWinKB, bool kPipe, int kMinWaves>
__global__ __launch_bounds__(kThreads, kMinWaves) void rlev2_tiled_kernel(
    const uint8_t* __restrict__ src, uint64_t src_len, int is_signed,
    const uint64_t* __restrict__ segtab, uint64_t nsegs, uint64_t rows_per_group,
    uint64_t value_begin, uint64_t nvalues, T* __restrict__ dst, unsigned long long* err) {
  constexpr uint32_t kWin = kWinKB * 1024u;
  constexpr int kBufs = kPipe ? 2 : 1;
  __shared__ uint32_t s_win[kBufs][kWin / 4 + 8];  // + 32 B: the 12-byte extract may read past a run
  __shared__ uint32_t s_off[kBufs][kMaxRuns];
  __shared__ uint32_t s_val[kBufs][kMaxRuns];
  __shared__ uint32_t s_ctl[kBufs][4];

  const uint64_t g = blockIdx.x;
  const int tid = (int)threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const uint64_t value_end = value_begin + nvalues;

  const uint64_t seg_start = segtab[2 * g];
  uint64_t vi = kPositions ? g * rows_per_group - segtab[2 * g + 1] : segtab[2 * g + 1];
  uint64_t seg_end = src_len;
  uint64_t v_next = ~0ull;
  if (g + 1 < nsegs) {
    seg_end = segtab[2 * (g + 1)];
    v_next = kPositions ? (g + 1) * rows_per_group - segtab[2 * (g + 1) + 1] : segtab[2 * (g + 1) + 1];
  }
  if (seg_end > src_len) seg_end = src_len;
  if (vi >= value_end || v_next <= value_begin) return;
  if (seg_start >= seg_end) {
    if (tid == 0 && v_next != ~0ull && v_next != vi && seg_start < src_len) report(err, vi, kErrBadSegment);
    return;
  }

  // Range-checked descriptor over [seg_start & ~15, end of stream).
  const uintptr_t base_abs = ((uintptr_t)src + seg_start) & ~(uintptr_t)15;
  const uintptr_t end_abs = ((uintptr_t)src + src_len + 3) & ~(uintptr_t)3;
  const uint64_t span = (uint64_t)(end_abs - base_abs);
  const uint32_t nrec = span > 0xfffff000ull ? 0xfffff000u : (uint32_t)span;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base_abs, (short)0, (int)nrec, 0x00020000);
  const uint64_t bias = (uint64_t)(base_abs - (uintptr_t)src);  // stream offset of descriptor byte 0

  uint64_t pos = seg_start;
  if constexpr (!kPipe) {
    uint64_t pwpos = ~0ull;  // previous window (stream offset) and its valid bytes
    uint32_t pneed = 0;
    while (pos < seg_end && vi < value_end) {
      const uint32_t wrel = (uint32_t)(pos - bias) & ~15u;
      const uint64_t wpos = bias + wrel;
      uint32_t need = kWin, keep = 0;
      if constexpr ((kOpt & kOptReuse) != 0) {
        // never load past the segment: its runs end at seg_end
        const uint64_t end_rel = (seg_end - bias + 15) & ~15ull;
        if (end_rel - wrel < need) need = (uint32_t)(end_rel - wrel);
        // the previous window's tail [wpos, pwpos + pneed) is already in LDS:
        // move it to the front instead of re-reading it (source and
        // destination must not overlap: the shift is at least the length)
        // A walk that stopped on a full run table (many tiny runs) may have
        // advanced less than the tail it would keep: then reload instead of
        // an overlapping LDS move.
        if (pwpos != ~0ull && pwpos + pneed > wpos && wpos - pwpos >= pwpos + pneed - wpos) {
          keep = (uint32_t)(pwpos + pneed - wpos);
          if (keep > need) keep = need;
          const uint32_t so = (uint32_t)(wpos - pwpos);
          typedef uint32_t u4 __attribute__((ext_vector_type(4)));
          for (uint32_t o = tid * 16u; o < keep; o += kThreads * 16u)
            *(u4*)((char*)s_win[0] + o) = *(const u4*)((const char*)s_win[0] + so + o);
          __syncthreads();  // reads of the tail finish before the DMA below lands
        }
        for (uint32_t off = keep + wave * 1024u; off < need; off += kWaves * 1024u)
          if (off + lane * 16u < need)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)((char*)s_win[0] + off), 16,
                wrel + off + lane * 16u, 0, 0, (kOpt & kOptNTLoad) ? 2 : 0);
      } else {
        fill<kOpt>(s_win[0], rs, wrel, kWin, wave, kWaves, lane);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (wave == 0) {
        const WalkResult w = walk<kWin>(s_win[0], s_off[0], s_val[0], wpos, pos, vi, seg_end, src_len,
                                        value_end, is_signed, err, lane, need);
        if (lane == 0) {
          s_ctl[0][0] = w.n;
          s_ctl[0][1] = w.stop;
          s_ctl[0][2] = w.dpos;
          s_ctl[0][3] = w.dval;
        }
      }
      __syncthreads();
      const uint32_t n = s_ctl[0][0], stop = s_ctl[0][1];
      const uint64_t next_pos = pos + s_ctl[0][2], next_vi = vi + s_ctl[0][3];
      for (uint32_t k = wave; k < n; k += kWaves)
        expand_run<kOpt>(s_win[0], kWin / 4 + 8, s_off[0][k], vi + s_val[0][k], is_signed, value_begin, value_end, dst, lane);
      __syncthreads();  // the window is refilled next
      if (stop) return;
      pos = next_pos;
      vi = next_vi;
      pwpos = wpos;
      pneed = need;
    }
  } else {
    // prologue: the producer fills and walks window 0
    if (wave == 0) {
      const uint32_t wrel = (uint32_t)(pos - bias) & ~15u;
      fill<kOpt>(s_win[0], rs, wrel, kWin, 0, 1, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const WalkResult w = walk<kWin>(s_win[0], s_off[0], s_val[0], bias + wrel, pos, vi, seg_end, src_len,
                                      value_end, is_signed, err, lane);
      if (lane == 0) {
        s_ctl[0][0] = w.n;
        s_ctl[0][1] = w.stop;
        s_ctl[0][2] = w.dpos;
        s_ctl[0][3] = w.dval;
      }
    }
    lds_barrier();
    for (uint32_t b = 0;; b ^= 1) {
      const uint32_t n = s_ctl[b][0], stop = s_ctl[b][1];
      const uint64_t next_pos = pos + s_ctl[b][2], next_vi = vi + s_ctl[b][3];
      const bool more = !stop && next_pos < seg_end && next_vi < value_end;
      if (wave == 0) {
        if (more) {  // produce window b^1 while the consumers expand window b
          const uint32_t wrel = (uint32_t)(next_pos - bias) & ~15u;
          fill<kOpt>(s_win[b ^ 1], rs, wrel, kWin, 0, 1, lane);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          const WalkResult w = walk<kWin>(s_win[b ^ 1], s_off[b ^ 1], s_val[b ^ 1], bias + wrel, next_pos,
                                          next_vi, seg_end, src_len, value_end, is_signed, err, lane);
          if (lane == 0) {
            s_ctl[b ^ 1][0] = w.n;
            s_ctl[b ^ 1][1] = w.stop;
            s_ctl[b ^ 1][2] = w.dpos;
            s_ctl[b ^ 1][3] = w.dval;
          }
        }
      } else {
        for (uint32_t k = wave - 1; k < n; k += kWaves - 1)
          expand_run<kOpt>(s_win[b], kWin / 4 + 8, s_off[b][k], vi + s_val[b][k], is_signed, value_begin, value_end, dst,
                           lane);
      }
      lds_barrier();
      if (stop) return;
      pos = next_pos;
      vi = next_vi;
      if (!more) break;
    }
  }
  if (tid == 0 && v_next != ~0ull && vi < value_end && vi != v_next) report(err, vi, kErrBadSegment);
}

}  // namespace

// Variants (ctx->rlev2_variant): 0 = default; 2.. = tuning experiments.
int launch_rlev2_tiled(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                       const uint64_t* d_segtab, uint64_t nsegs, bool positions_mode,
                       uint64_t rows_per_group, uint64_t value_begin, uint64_t nvalues, void* d_dst,
                       int dst_bytes) {
  if (nsegs == 0 || nvalues == 0) return ORCG_OK;
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  if (dst_bytes != 8 && dst_bytes != 4 && dst_bytes != 2)
    return set_error(ctx, ORCG_INVALID_ARGUMENT, "dst_bytes must be 8, 4 or 2");
  const dim3 grid((unsigned)nsegs), block(kThreads);
  const int sg = is_signed ? 1 : 0;

#define ORCG_K(T, P, O, WKB, PIPE)                                                                   \
  hipLaunchKernelGGL((rlev2_tiled_kernel<T, P, O, WKB, PIPE, MW>), grid, block, 0, ctx->stream, d_src, \
                     src_len, sg, d_segtab, nsegs, rows_per_group, value_begin, nvalues, (T*)d_dst, \
                     ctx->d_err)
#define ORCG_KT(O, WKB, PIPE, MWV)                                                   \
  do {                                                                              \
    constexpr int MW = MWV;                                                         \
    if (dst_bytes == 8) {                                                           \
      if (positions_mode) ORCG_K(int64_t, true, O, WKB, PIPE);                       \
      else ORCG_K(int64_t, false, O, WKB, PIPE);                                     \
    } else if (dst_bytes == 4) {                                                    \
      if (positions_mode) ORCG_K(int32_t, true, O, WKB, PIPE);                       \
      else ORCG_K(int32_t, false, O, WKB, PIPE);                                     \
    } else {                                                                        \
      if (positions_mode) ORCG_K(int16_t, true, O, WKB, PIPE);                       \
      else ORCG_K(int16_t, false, O, WKB, PIPE);                                     \
    }                                                                               \
  } while (0)

  switch (ctx->rlev2_variant) {
    case 8: ORCG_KT(kOptNTStore | kOptReuse | kOptFast, 21, false, 6); break;  // 21 KB + fast
    case 9: ORCG_KT(kOptNTStore | kOptReuse, 33, false, 1); break;             // 33 KB, 4 WG/CU
    default: {
      // ORCG_RLEV2_TILED picks the window by stream density: wide values
      // (>= 5 stream bytes per value, e.g. W >= 40) stream best through
      // 33 KB windows (4 WG/CU); narrower ones need more workgroups in
      // flight per CU to keep HBM busy: 21 KB windows (6 WG/CU) + the
      // predicate-free full-run path. Measured: scripts/ab_rlev2.py.
      const uint64_t est_values = positions_mode ? nsegs * rows_per_group : nvalues;
      if (src_len >= 5 * est_values) ORCG_KT(kOptNTStore | kOptReuse, 33, false, 1);
      else ORCG_KT(kOptNTStore | kOptReuse | kOptFast, 21, false, 6);
      break;
    }
  }
#undef ORCG_KT
#undef ORCG_K
  return hip_check(ctx, hipGetLastError(), "rlev2_tiled_kernel launch");
}

}  // namespace orcg
