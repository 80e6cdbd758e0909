// RLEv2 decode, tiled through LDS (the default kernels).
//
// One 256-thread workgroup per segment. The segment's bytes stream through an
// LDS window filled by buffer_load ... lds (LDS-DMA, 1 KB per wave
// instruction, range-checked so reads past the stream return zeros), or, in
// the wide-value instance, by 16-byte buffer loads into registers that are
// all in flight before the LDS writes (kOptRegFill). The run
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
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <vector>

#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

// Phase profiling (build with -DORCG_PHASE_PROF, scripts/phase_prof.py):
// thread 0 adds the cycles between consecutive phase marks to g_phase[k].
#ifdef ORCG_PHASE_PROF
__device__ unsigned long long g_phase[16];
// union instances: per workgroup {wall-clock ticks, dense passes | serial passes << 32}
constexpr uint32_t kWgDurMax = 16384;
__device__ unsigned long long g_wgdur[2 * kWgDurMax];
#define PROF_MARK(k)                                                        \
  do {                                                                      \
    if (threadIdx.x == 0) {                                                 \
      const uint64_t now_ = wall_clock64();                                 \
      atomicAdd(&g_phase[k], (unsigned long long)(now_ - prof_last_));      \
      prof_last_ = now_;                                                    \
    }                                                                       \
  } while (0)
#define PROF_DECL uint64_t prof_last_ = wall_clock64()
#else
#define PROF_MARK(k) \
  do {               \
  } while (0)
#define PROF_DECL
#endif

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr uint32_t kMaxRun = 4608;  // >= 4356, the longest legal run

// Dense (short-run) mode. A stream of short runs (SHORT_REPEAT-heavy
// low-cardinality columns: 2-9 bytes per run) makes the one-wave serial header
// walk the bottleneck. Dense mode discovers run starts in parallel over a slab
// of kSlab bytes: thread t owns bytes [t*kBlk, (t+1)*kBlk) and computes, for
// every position of its block, the chain exit "first run start past the block
// if a run started here" and the values in between (a backward scan, since a
// run ending inside the block continues from a later position of the same
// block); one lane then chains the 256 blocks (one LDS read per block instead
// of one header parse per run), and every thread re-walks its own block from
// its true entry to emit the run table. Short runs are then expanded one lane
// per run into a per-wave LDS stage, flushed with coalesced stores.
constexpr uint32_t kSlab = 2048;
constexpr uint32_t kBlk = kSlab / kThreads;  // 8 bytes per thread
constexpr uint32_t kDenseRuns = kSlab / 2;   // every run is >= 2 bytes
constexpr uint32_t kStage = 256;             // values staged per wave
constexpr uint32_t kShortL = 16;             // runs of <= kShortL values go lane-per-run
constexpr uint32_t kVparL = 256;             // dense expansion: runs of kVparMin+1 .. kVparL values go
#ifndef ORCG_VPAR_MIN                         // value-parallel
#define ORCG_VPAR_MIN 16
#endif
constexpr uint32_t kVparMin = ORCG_VPAR_MIN;
#ifndef ORCG_VPAR_FRAG
#define ORCG_VPAR_FRAG 2
#endif
constexpr uint32_t kVparFrag = ORCG_VPAR_FRAG;  // short-run groups per 64 runs before all go value-parallel
constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kDpErr = 0x80000000u;     // DP entry: a corrupt run starts here
constexpr uint16_t kSink = 0xffffu;          // chain successor: none
constexpr uint32_t kWalkDone = 0x80000000u;  // published-runs flag: the walk has finished
// density hysteresis (stream bytes per run of the last pass)
constexpr uint32_t kToDense = 24, kToSerial = 64;
// two-pass (kOptTable) instances: dense discovery no longer pays for the
// expansion, and a serial walk over medium runs (DELTA / DIRECT runs of tens
// of bytes) was the launch's tail (one wave walking a whole row group while
// co-resident workgroups share the CU): dense up to far longer runs
#ifndef ORCG_TAB_TO_DENSE
#define ORCG_TAB_TO_DENSE 128
#endif
#ifndef ORCG_TAB_TO_SERIAL
#define ORCG_TAB_TO_SERIAL 512
#endif
constexpr uint32_t kTabToDense = ORCG_TAB_TO_DENSE, kTabToSerial = ORCG_TAB_TO_SERIAL;

// kOpt bits
constexpr int kOptNTStore = 1;  // non-temporal output stores (streamed, never re-read)
constexpr int kOptNTLoad = 2;   // non-temporal LDS-DMA loads of the stream
constexpr int kOptReuse = 4;    // carry the window tail over in LDS; never load past the segment
constexpr int kOptFast = 8;     // predicate-free paths for full (512-value) runs inside the output range
constexpr int kOptRegFill = 16; // fill windows through registers (16 B buffer loads, then LDS writes), not LDS-DMA
constexpr int kOptT4 = 32;
constexpr int kOptD3 = 64;      // dense discovery: predicated chain marks, wave-reduced control atomics, inline probe
constexpr int kOptDirect = 128; // dense expansion: lanes store their short runs' values straight to the output (no stage)
constexpr int kOptPair = 256;   // full DIRECT runs: two values per lane, one 16-byte store (16-byte aligned int64 output)
constexpr int kOptUnion = 1024; // dense v2 instance whose serial (long-run) windows also cover the dense stage and
                                // marks: one instance routes each window by its runs (dense or serial), no queue
constexpr int kOptScan = 4096;      // dense discovery: block entries by a wave scan of entry-state functions (DPP,
                                    // no LDS gathers), the pointer-doubling chain only when a run jumps too far
constexpr int kOptPrefetch = 2048;  // register-filled serial windows: every wave loads its share of the next window
                                    // into registers as soon as the walk is done, while it expands this one
constexpr int kOptGrpT = 8192;      // serial groups of short runs (one lane per run, scattered 8-byte stores):
                                    // temporal stores, so L2 merges the partial lines before they reach HBM
constexpr int kOptTable = 16384;    // two-pass (RunTab): dense passes write their runs to the run table for
                                    // rlev2_expand_kernel instead of expanding them

// Debug build only (ORCG_AB_FLAGS=-DORCG_DEBUG_COVER): every expansion path
// counts the values of the runs it expands; each pass checks the count
// against the values its discovery consumed.
#ifdef ORCG_DEBUG_COVER
#define ORCG_COVER_ADD(x) atomicAdd(s_cover_ptr(), (uint32_t)(x))
__device__ __forceinline__ uint32_t* s_cover_ptr() {
  __shared__ uint32_t s_cover;
  return &s_cover;
}
#else
#define ORCG_COVER_ADD(x) \
  do {                    \
  } while (0)
#endif

template <int kOpt, typename T>
__device__ __forceinline__ void store1(T* p, uint64_t v) {
  if constexpr ((kOpt & kOptNTStore) != 0) __builtin_nontemporal_store((T)(int64_t)v, p);
  else *p = (T)(int64_t)v;
}

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
// two consecutive int64 values, one 16-byte store (p 16-byte aligned)
template <int kOpt>
__device__ __forceinline__ void store2(int64_t* p, uint64_t a, uint64_t b) {
  u64x2 v;
  v.x = a;
  v.y = b;
  if constexpr ((kOpt & kOptNTStore) != 0) __builtin_nontemporal_store(v, (u64x2*)p);
  else *(u64x2*)p = v;
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

// terminator bits of a dword's bytes (bit i = byte i < 0x80)
__device__ __forceinline__ uint32_t term4(uint32_t w) {
  const uint32_t m = (~w >> 7) & 0x01010101u;
  return (m * 0x10204080u) >> 28;
}

struct LaneWin {
  uint32_t word = 0, base = 0xffffffffu;
  uint32_t t4 = 0;  // term4(word): the walk's varint ends, computed once per slice on the VALU
  __device__ __forceinline__ void load(const uint32_t* win, uint32_t hoff, uint32_t nwords, int lane) {
    base = hoff & ~3u;
    uint32_t idx = (base >> 2) + (uint32_t)lane;
    if (idx >= nwords) idx = nwords - 1;
    word = win[idx];
    t4 = term4(word);
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
  Run r;
  if ((hw.byte(hoff) >> 6) == 3) {
    // DELTA header of a run the walk validated, one header byte per lane: varint
    // ends from a ballot of the terminator bytes, values OR-reduced in the
    // DPP rows, instead of a
    // scalar byte loop (the kernel's scalar unit is its busiest on DELTA
    // streams)
    const uint32_t fb = hw.byte(hoff);
    r.kind = 3;
    r.pbs = r.pl = r.cfb = 0;
    r.err = kErrNone;
    r.L = ((fb & 1u) << 8 | hw.byte(hoff + 1)) + 1u;
    const uint32_t fbo = (fb >> 1) & 0x1fu;
    r.W = fbo ? fbs_width(fbo) : 0u;
    const uint32_t hb = lds_byte(win, hoff + 2u + (uint32_t)lane);
    const uint64_t term = __ballot(hb < 0x80u);
    const uint32_t n1 = (uint32_t)__builtin_ctzll(term) + 1u;
    const uint32_t n2 = (uint32_t)__builtin_ctzll(term >> n1) + 1u;
    const uint32_t b7 = hb & 0x7fu, k2 = (uint32_t)lane - n1;
    uint64_t ca = ((uint32_t)lane < n1 && lane < 10) ? (uint64_t)b7 << (7 * lane) : 0ull;
    uint64_t cb = ((uint32_t)lane >= n1 && k2 < n2 && k2 < 10u) ? (uint64_t)b7 << (7 * k2) : 0ull;
#define ORCG_OR_ROWS(x)                  \
  x |= dpp0_64<0x111, 0xf>(x);           \
  x |= dpp0_64<0x112, 0xf>(x);           \
  x |= dpp0_64<0x114, 0xf>(x);           \
  x |= dpp0_64<0x118, 0xf>(x)
    ORCG_OR_ROWS(ca);
    ORCG_OR_ROWS(cb);
#undef ORCG_OR_ROWS
    // the row totals sit in lanes 15 / 31 / 47 / 63 (a header reaches 64 bytes)
    auto rows_or = [](uint64_t x) -> uint64_t {
      const uint32_t lo = rdlane((uint32_t)x, 15) | rdlane((uint32_t)x, 31) | rdlane((uint32_t)x, 47) |
                          rdlane((uint32_t)x, 63);
      const uint32_t hi = rdlane((uint32_t)(x >> 32), 15) | rdlane((uint32_t)(x >> 32), 31) |
                          rdlane((uint32_t)(x >> 32), 47) | rdlane((uint32_t)(x >> 32), 63);
      return ((uint64_t)hi << 32) | lo;
    };
    const uint64_t a_raw = rows_or(ca), b_raw = rows_or(cb);
    r.a = is_signed ? unzigzag(a_raw) : a_raw;
    r.b = unzigzag(b_raw);
    r.data = 2u + n1 + n2;
    r.bytes = r.data + (r.W ? (r.W * (r.L - 2u) + 7u) / 8u : 0u);
  } else {
    r = parse_run([&](uint32_t i) { return hw.byte(hoff + i); }, ~0ull, kHdrLim, is_signed);
  }
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
      if constexpr ((kOpt & kOptPair) != 0 && sizeof(T) == 8) {
        if ((((uintptr_t)out) & 15u) == 0) {
          // lane pairs of values: a wave stores 1 KB per instruction
          if (W == 64) {
            const uint32_t r4 = d & 3u;
#pragma unroll
            for (int it = 0; it < kMaxRunUnroll / 2; ++it) {
              const uint32_t j = 2u * (uint32_t)(it * kWave + lane);
              const uint32_t i = (d + 8u * j) >> 2;
              const uint32_t w0 = win[i], w1 = win[i + 1], w2 = win[i + 2], w3 = win[i + 3], w4 = win[i + 4];
              uint64_t a = ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, r4)) << 32) |
                           __builtin_bswap32(__builtin_amdgcn_alignbyte(w2, w1, r4));
              uint64_t b = ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(w3, w2, r4)) << 32) |
                           __builtin_bswap32(__builtin_amdgcn_alignbyte(w4, w3, r4));
              if (is_signed) {
                a = unzigzag(a);
                b = unzigzag(b);
              }
              store2<kOpt>((int64_t*)out + j, a, b);
            }
          } else {
#pragma unroll
            for (int it = 0; it < kMaxRunUnroll / 2; ++it) {
              const uint32_t j = 2u * (uint32_t)(it * kWave + lane);
              const uint32_t bit = j * W, bit2 = bit + W;
              const uint32_t br = d + (bit >> 3), br2 = d + (bit2 >> 3);
              uint64_t a = field(lds12(win, br), br, bit & 7u, W);
              uint64_t b = field(lds12(win, br2), br2, bit2 & 7u, W);
              if (is_signed) {
                a = unzigzag(a);
                b = unzigzag(b);
              }
              store2<kOpt>((int64_t*)out + j, a, b);
            }
          }
          return;
        }
      }
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
    if ((kOpt & kOptFast) && L == 512 && v0 >= value_begin && v0 + 512 <= value_end) {
      // full run inside the output range: all 8 chunks' literals in
      // registers, the (few) patches OR-ed into the lane that owns their
      // position, then predicate-free stores
      T* out = dst + (v0 - value_begin);
      uint64_t lit[kMaxRunUnroll];
#pragma unroll
      for (int it = 0; it < kMaxRunUnroll; ++it) {
        const uint32_t bit = (uint32_t)(it * kWave + lane) * W;
        const uint32_t br = d + (bit >> 3);
        lit[it] = field(lds12(win, br), br, bit & 7u, W);
      }
      for (uint64_t t = applied; t; t &= t - 1) {
        const uint32_t k = (uint32_t)__builtin_ctzll(t);
        const uint32_t c = rdlane(cum, k);
        const uint64_t add = (((uint64_t)rdlane(p_hi, k) << 32) | rdlane(p_lo, k)) << (W & 63u);
#pragma unroll
        for (int it = 0; it < kMaxRunUnroll; ++it)
          if (c == (uint32_t)(it * kWave + lane)) lit[it] |= add;
      }
#pragma unroll
      for (int it = 0; it < kMaxRunUnroll; ++it) store1<kOpt>(out + it * kWave + lane, r.a + lit[it]);
      return;
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
  if (W <= 26 && (kOpt & kOptFast) && L == 512 && v0 >= value_begin && v0 + 512 <= value_end) {
    // full run inside the output range: all 8 chunks' deltas loaded up
    // front, no per-value predicates, one 32-bit wave scan per chunk
    T* out = dst + (v0 - value_begin);
    uint32_t dl[kMaxRunUnroll];
#pragma unroll
    for (int it = 0; it < kMaxRunUnroll; ++it) {
      const uint32_t j = it * kWave + lane;
      const uint32_t k = j >= 2 ? j - 2 : 0u;  // j < 2: a dummy in-range read, masked below
      const uint32_t bit = k * W;
      const uint32_t br = d + (bit >> 3);
      dl[it] = (uint32_t)field(lds12(win, br), br, bit & 7u, W);
    }
    if (lane < 2) dl[0] = 0;
#pragma unroll
    for (int it = 0; it < kMaxRunUnroll; ++it) {
      const uint32_t j = it * kWave + lane;
      const uint32_t s32 = wave_scan_u32(dl[it]);
      const uint64_t sum = carry + s32;
      carry += (uint32_t)__builtin_amdgcn_readlane((int)s32, 63);
      const uint64_t v = j == 0 ? r.a : (j == 1 ? v1 : (neg ? v1 - sum : v1 + sum));
      store1<kOpt>(out + j, v);
    }
    return;
  }
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
  uint32_t n, stop, dpos, dval, items, shrt;  // shrt: stopped by the probe (short runs)
};

// Work items of a serial pass (the walk publishes item ends): a group of up
// to 64 consecutive short runs, expanded one lane per run, or one long /
// PATCHED_BASE run (flag kItemLong), expanded by a whole wave.
constexpr uint16_t kItemLong = 0x8000;
#ifndef ORCG_ITEM_MAX
#define ORCG_ITEM_MAX 64
#endif
constexpr uint32_t kItemMax = ORCG_ITEM_MAX;  // short runs per group (<= 64)

// The serial walk's view of a run: bytes, values and the error parse_run
// would report, in its order. SHORT_REPEAT / DIRECT from the first two
// bytes, DELTA from a terminator mask of the 24 bytes after its header
// (two varints of <= 11 bytes: every writer's); PATCHED_BASE and longer
// varints through parse_run.
template <bool kT4>
__device__ __forceinline__ void walk_extent(const LaneWin& hw, uint32_t lp, uint32_t avail, int is_signed,
                                            uint32_t* bytes, uint32_t* L, uint32_t* err, uint32_t* rkind) {
  const uint32_t fb = hw.byte(lp), kind = fb >> 6;
  *err = kErrNone;
  *rkind = kind;
  if (kind < 2) {
    // SHORT_REPEAT / DIRECT, straight-line scalar code (a DIRECT run short
    // of its second header byte has >= 2 bytes > avail: the same bad read)
    const uint32_t L2 = ((fb & 1u) << 8 | hw.byte(lp + 1)) + 1u;
    const uint32_t db = 2u + (fbs_width((fb >> 1) & 0x1fu) * L2 + 7u) / 8u;
    *bytes = kind ? db : 2u + ((fb >> 3) & 7u);
    *L = kind ? L2 : (fb & 7u) + 3u;
    if (*bytes > avail) *err = kErrBadRead;
    return;
  }
  if (kind != 2) {
    if (avail < 2) {
      *err = kErrBadRead;
      *bytes = 0;
      *L = 0;
      return;
    }
    const uint32_t L2 = ((fb & 1u) << 8 | hw.byte(lp + 1)) + 1u;
    const uint32_t code = (fb >> 1) & 0x1fu;
    // DELTA: varint lengths from the terminator mask of bytes lp+2 .. lp+25
    // (the slice's per-dword terminator nibbles, gathered and realigned)
    const uint32_t o = lp + 2u - hw.base, i0 = o >> 2, sh = o & 3u;
    uint32_t t = 0;
    if constexpr (kT4) {
#pragma unroll
      for (uint32_t k = 0; k < 7; ++k) t |= rdlane(hw.t4, i0 + k) << (4 * k);
      t = (t >> sh) & 0xffffffu;
    } else {
      uint32_t prev = rdlane(hw.word, i0);
#pragma unroll
      for (uint32_t k = 0; k < 6; ++k) {
        const uint32_t nx = rdlane(hw.word, i0 + k + 1);
        t |= term4(__builtin_amdgcn_alignbyte(nx, prev, sh)) << (4 * k);
        prev = nx;
      }
    }
    const uint32_t n1 = t ? (uint32_t)__builtin_ctz(t) + 1u : 32u;
    const uint32_t t2 = n1 < 24 ? t >> n1 : 0u;
    const uint32_t n2 = t2 ? (uint32_t)__builtin_ctz(t2) + 1u : 32u;
    if (n1 <= 11 && n2 <= 11) {
      const uint32_t W = code ? fbs_width(code) : 0u;
      *L = L2;
      if (2u + n1 + n2 > avail) {
        *err = kErrBadRead;
        return;
      }
      if (W != 0 && L2 < 2) {
        *err = kErrDeltaLength;
        return;
      }
      *bytes = 2u + n1 + n2 + (W ? (W * (L2 - 2u) + 7u) / 8u : 0u);
      if (*bytes > avail) *err = kErrBadRead;
      return;
    }
  }
  const Run r = parse_run([&](uint32_t i) { return hw.byte(lp + i); }, avail, kHdrLim, is_signed);
  *bytes = r.bytes;
  *L = r.L;
  *err = r.err;
}

// Wave-uniform header walk over the window [wpos, wpos + kWin): records runs
// starting at pos.. into (run_off, run_val) until the next run starts past
// kWin - kMaxRun and does not end inside the loaded bytes (`lim`), leaves the
// segment, or the table is full. With `pub` the
// walk also cuts the runs into work items (`items`, ends by run index) and
// publishes the item count as items close, so expanding waves start early.
template <uint32_t kWin, uint32_t kCap, bool kT4 = false, typename OffT = uint32_t>
__device__ __forceinline__ WalkResult walk(const uint32_t* win, OffT* run_off, uint32_t* run_val,
                                           uint64_t wpos, uint64_t pos, uint64_t vi, uint64_t seg_end,
                                           uint64_t src_len, uint64_t value_end, int is_signed,
                                           unsigned long long* err, int lane, uint32_t lim = kWin,
                                           uint32_t cap = kCap, uint32_t* pub = nullptr,
                                           uint16_t* items = nullptr, uint32_t probe_n = 0,
                                           bool probe_values = false) {
  static_assert(kCap < kItemLong, "run indices must leave the item flag free");
  constexpr uint32_t kChunk = kWin - kMaxRun;
  // everything wave-uniform and 32-bit, relative to the window / the first
  // value: the loop stays on the scalar unit (no 64-bit VALU compares)
  const uint32_t sp = (uint32_t)(pos - wpos);
  const uint32_t a_seg = seg_end - wpos < 0xfffff000ull ? (uint32_t)(seg_end - wpos) : 0xfffff000u;
  const uint32_t a_src = src_len - wpos < 0xfffff000ull ? (uint32_t)(src_len - wpos) : 0xfffff000u;
  const uint32_t v_lim = value_end - vi < 0xffffffffull ? (uint32_t)(value_end - vi) : 0xffffffffu;
  uint32_t lp = sp, vr = 0;
  uint32_t n = 0, stop = 0, shrt = 0;
  LaneWin hw;
  hw.load(win, sp, kWin / 4 + 8, lane);
  // run k waits in lane k % 64 (r_off, r_val) until the table write of its
  // batch: one LDS round trip (and one release store) per item or per 64
  // runs instead of one per run
  uint32_t r_off = 0, r_val = 0, flushed = 0, gstart = 0, nitems = 0;
  auto flush = [&]() {
    const uint32_t r = flushed + (((uint32_t)lane - flushed) & (kWave - 1));
    if (r < n) {
      run_off[r] = (OffT)r_off;
      run_val[r] = r_val;
    }
    flushed = n;
  };
  const uint32_t lim_all = uni(min(min(a_src, a_seg), lim));
  const bool items_on = uni(pub != nullptr ? 1u : 0u) != 0;
  while (lp < a_seg && vr < v_lim && n < cap) {
    // a run starting past the chunk is taken only when all of its bytes are
    // loaded (its extent depends on its own bytes only); otherwise it starts
    // the next window
    const bool past = lp >= kChunk && n > 0;
    if (past && lp + 2u > lim) break;
    if (lp + kHdrLim > hw.base + 256) hw.load(win, lp, kWin / 4 + 8, lane);
    // the two header bytes from two lanes of the slice, realigned on the
    // scalar unit; SHORT_REPEAT / DIRECT sized inline (branch-free selects),
    // DELTA / PATCHED_BASE through walk_extent
    const uint32_t o = lp - hw.base, wi = o >> 2;
    const uint64_t w2 = ((uint64_t)rdlane(hw.word, wi + 1) << 32) | rdlane(hw.word, wi);
    const uint32_t hdr = (uint32_t)(w2 >> ((o & 3u) * 8u));
    const uint32_t fb = hdr & 0xffu, kind = fb >> 6;
    uint32_t rbytes, rL, e = kErrNone;
    if (kind < 2) {
      const uint32_t L2 = ((fb & 1u) << 8 | ((hdr >> 8) & 0xffu)) + 1u;
      const uint32_t code = (fb >> 1) & 0x1fu;
      const uint32_t wt = (uint32_t)(0x40383028201E1C1Aull >> (((code - 24u) & 7u) * 8u)) & 0xffu;
      const uint32_t W = code < 24 ? code + 1u : wt;  // fbs_width
      uint32_t bits;
      asm("s_mul_i32 %0, %1, %2" : "=s"(bits) : "s"(uni(W)), "s"(uni(L2)));
      rbytes = kind ? 2u + ((bits + 7u) >> 3) : 2u + ((fb >> 3) & 7u);
      rL = kind ? L2 : (fb & 7u) + 3u;
    } else {
      uint32_t kd;
      walk_extent<kT4>(hw, lp, a_src - lp, is_signed, &rbytes, &rL, &e, &kd);
      rbytes = uni(rbytes);  // keep the merged values scalar
      rL = uni(rL);
      e = uni(e);
    }
    if (past && (e != kErrNone || lp + rbytes > lim)) break;  // the next window decides
    if (e != kErrNone || lp + rbytes > lim_all) {
      // the first failing check, in the order parse / segment / window
      if (e == kErrNone)
        e = lp + rbytes > a_src ? kErrBadRead : (lp + rbytes > a_seg ? kErrBadSegment : kErrBadRead);
      if (lane == 0) report(err, vi + vr, e);
      stop = 1;
      break;
    }
    // a per-lane select, not v_writelane: the compiler may copy r_off /
    // r_val with a partial EXEC inside a branch it cannot prove uniform, which
    // is only safe when no lane's value is written by another lane
    const bool mine = (uint32_t)lane == (n & (kWave - 1));
    r_off = mine ? lp : r_off;
    r_val = mine ? vr : r_val;
    ++n;
    lp += rbytes;
    vr += rL;
    if (items_on) {
      if (rL > kShortL || kind == 2) {
        // close the open group of short runs, then this run as its own item
        flush();
        const uint32_t grp = n - 1 > gstart ? 1u : 0u;
        if (lane == 0) {
          if (grp) items[nitems] = (uint16_t)(n - 1);
          items[nitems + grp] = (uint16_t)(n | kItemLong);
        }
        nitems += grp + 1;
        gstart = n;
        // expanding waves may claim the items as soon as they are published
        if (lane == 0) __hip_atomic_store(pub, nitems, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (n - gstart == kItemMax) {
        flush();
        if (lane == 0) items[nitems] = (uint16_t)n;
        ++nitems;
        gstart = n;
        if (lane == 0) __hip_atomic_store(pub, nitems, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else if (n - flushed == kWave) {
      flush();
    }
    // the probe: the first probe_n runs of a segment average < kToDense
    // bytes (a short-run segment), the caller switches to dense discovery
    // (probe_values: their values average <= kShortL, whatever their bytes)
    if (n == probe_n && (probe_values ? vr <= probe_n * kShortL : lp - sp < probe_n * kToDense)) {
      shrt = 1;
      break;
    }
  }
  if (n != flushed) flush();
  if (pub && n > gstart) {
    // the last group: published by the caller's final (walk done) store
    if (lane == 0) items[nitems] = (uint16_t)n;
    ++nitems;
  }
  return WalkResult{n, stop, lp - sp, vr, nitems, shrt};
}

// Value j of a short run (kind SHORT_REPEAT / DIRECT / DELTA) parsed at
// window offset `hoff`; `acc` carries a variable-width DELTA run's |delta| sum.
__device__ __forceinline__ uint64_t short_value(const uint32_t* win, const Run& r, uint32_t hoff, uint32_t j,
                                                int is_signed, uint64_t& acc) {
  if (r.kind == 0) return r.a;
  if (r.kind == 1) {
    const uint32_t bit = j * r.W;
    const uint32_t br = hoff + r.data + (bit >> 3);
    uint64_t v = field(lds12(win, br), br, bit & 7u, r.W);
    return is_signed ? unzigzag(v) : v;
  }
  if (r.W == 0) return r.a + (uint64_t)j * r.b;
  if (j == 0) return r.a;
  const uint64_t v1 = r.a + r.b;
  if (j == 1) return v1;
  const uint32_t bit = (j - 2) * r.W;
  const uint32_t br = hoff + r.data + (bit >> 3);
  acc += field(lds12(win, br), br, bit & 7u, r.W);
  return (int64_t)r.b < 0 ? v1 - acc : v1 + acc;
}

// Expand runs [r0, r1) (r1 - r0 <= 64, each SHORT_REPEAT / DIRECT / DELTA of
// <= kShortL values) one lane per run, storing straight to the output.
template <int kOpt, typename T, typename OffT>
__device__ __forceinline__ void group_expand(const uint32_t* win, const OffT* s_off, const uint32_t* s_val,
                                             uint32_t r0, uint32_t r1, uint64_t vi, int is_signed,
                                             uint64_t value_begin, uint64_t value_end, T* dst, int lane) {
  constexpr int kGrpOpt = (kOpt & kOptGrpT) != 0 ? (kOpt & ~kOptNTStore) : kOpt;
  const uint32_t r = r0 + (uint32_t)lane;
  const bool act = r < r1;
  const uint32_t hoff = act ? s_off[r] : s_off[r0];
  const uint64_t o0 = vi + (act ? s_val[r] : 0u);
  const uint32_t w0 = hoff >> 2, sh = hoff & 3u;
  const uint32_t d0 = win[w0], d1 = win[w0 + 1], d2 = win[w0 + 2], d3 = win[w0 + 3];
  const uint32_t b0 = __builtin_amdgcn_alignbyte(d1, d0, sh), b1 = __builtin_amdgcn_alignbyte(d2, d1, sh),
                 b2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
  const uint32_t fb = b0 & 0xffu;
  if (__ballot(act && (fb >> 6) != 0) == 0) {
    // SHORT_REPEAT only: W + 1 value bytes, big endian
    const uint32_t L = act ? (fb & 7u) + 3u : 0u;
    const uint32_t nb = ((fb >> 3) & 7u) + 1u;
    const uint64_t be = ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(b1, b0, 1)) << 32) |
                        __builtin_bswap32(__builtin_amdgcn_alignbyte(b2, b1, 1));
    uint64_t a = be >> (64 - 8 * nb);
    if (is_signed) a = unzigzag(a);
    ORCG_COVER_ADD(L);
    for (uint32_t j = 0; __ballot(j < L) != 0; ++j) {
      const uint64_t o = o0 + j;
      if (j < L && o >= value_begin && o < value_end) store1<kGrpOpt>(dst + (o - value_begin), a);
    }
    return;
  }
  const Run run = parse_run([&](uint32_t i) { return lds_byte(win, hoff + i); }, ~0ull, kHdrLim, is_signed);
  const uint32_t L = act ? run.L : 0u;
  ORCG_COVER_ADD(L);
  uint64_t acc = 0;
  for (uint32_t j = 0; __ballot(j < L) != 0; ++j) {
    const uint64_t o = o0 + j;
    if (j < L) {
      const uint64_t x = short_value(win, run, hoff, j, is_signed, acc);
      if (o >= value_begin && o < value_end) store1<kGrpOpt>(dst + (o - value_begin), x);
    }
  }
}

// ---- dense mode -----------------------------------------------------------

struct DenseResult {
  uint32_t n, stop, dpos, dval;
};

// Header of the run at window offset lq, with every check the serial walk
// applies (same order): truncated stream, run past the segment, run past the
// loaded bytes. Returns the error code (kErrNone when the run is good).
__device__ __forceinline__ uint32_t checked_run(const uint32_t* win, uint32_t lq, uint64_t wpos, uint64_t seg_end,
                                                uint64_t src_len, uint32_t need, int is_signed, Run* out) {
  const uint64_t pabs = wpos + lq;
  const uint64_t avail = pabs < src_len ? src_len - pabs : 0;
  const Run r = parse_run([&](uint32_t i) { return lds_byte(win, lq + i); }, avail, kHdrLim, is_signed);
  uint32_t e = r.err;
  if (e == kErrNone && pabs + r.bytes > seg_end) e = kErrBadSegment;
  if (e == kErrNone && lq + r.bytes > need) e = kErrBadRead;
  *out = r;
  return e;
}

// ---- dense mode v2 -----------------------------------------------------
// The same contract as dense_discover, restructured for the CDNA issue model
// (the v1 code spent ~3.7 SALU instructions per decoded value on exec-mask
// bookkeeping of divergent branches):
//  * the speculative header parse at every position is branch-free (all
//    kinds computed, selected by kind) and the in-block DP lives in
//    registers, indexed at compile time (select chains), not through LDS;
//  * PATCHED_BASE headers and DELTA varints over 10 bytes are "unknown" to
//    the DP: a block whose path meets one re-walks exactly (checked_run), as
//    v1 does for corrupt runs; such a block also ends the pass;
//  * the chain keeps each thread's 8 successors in registers and one u16 LDS
//    slot per position (single-buffered: a barrier on each side of the
//    write); marks propagate only from threads holding a marked position;
//  * a block's runs come from a forward pass over the DP registers (no
//    header re-parse), appended to the run table with predicated writes.
constexpr uint32_t kDpUnknown = 0x80000000u;

// FBSToBitWidthMap without a branch (RLEV2Util.cc:24-26)
__device__ __forceinline__ uint32_t fbs_width_nb(uint32_t code) {
  const uint32_t hi = (uint32_t)((0x40383028201E1C1Aull >> (8 * ((code - 24u) & 7u))) & 0xffu);
  return code < 24 ? code + 1 : hi;
}

template <int kOpt, typename OffT>
__device__ __forceinline__ DenseResult dense2_discover(const uint32_t* win, OffT* s_off, uint32_t* s_val,
                                                       uint16_t* s_nxt, uint32_t* s_mark, uint32_t* s_ctl,
                                                       uint64_t wpos, uint32_t sb, uint32_t lim, uint64_t vi,
                                                       uint64_t seg_end, uint64_t src_len, uint64_t value_end,
                                                       uint32_t need, int is_signed, unsigned long long* err,
                                                       int tid
#ifdef ORCG_PHASE_PROF
                                                       , uint64_t& prof_last_
#endif
) {
  const int wave = tid / kWave, lane = tid % kWave;
  const uint32_t lo = (uint32_t)tid * kBlk, hi = lo + kBlk;
  __builtin_amdgcn_s_setprio(2);
  // runs may not start at or past the segment end
  {
    const uint64_t sa = wpos + sb;
    const uint64_t seg_room = seg_end > sa ? seg_end - sa : 0;
    if (seg_room < lim) lim = (uint32_t)seg_room;
  }
  // (1) per position e of the block: ent[e] = exit (first run start past the
  // block on the path from e) | values on the path << 15, or kDpUnknown;
  // info (two positions per register): in-block successor (e + run bytes,
  // 15 = past the block) | L << 4
  uint32_t ent[kBlk], info2[kBlk / 2];
  {
    const uint32_t a0 = sb + lo, sh = a0 & 3u, w0 = a0 >> 2;
    uint32_t b4[kBlk / 4 + 8];
    {
      uint32_t prev = win[w0];
#pragma unroll
      for (int i = 0; i < (int)kBlk / 4 + 8; ++i) {
        const uint32_t nx = win[w0 + i + 1];
        b4[i] = __builtin_amdgcn_alignbyte(nx, prev, sh);
        prev = nx;
      }
    }
    uint64_t term = 0;  // bit i: byte i < 0x80 (varint terminators)
#pragma unroll
    for (int i = 0; i < (int)kBlk / 4 + 8 && i < 16; ++i) {
      const uint32_t m = (~b4[i] >> 7) & 0x01010101u;
      term |= (uint64_t)((m * 0x10204080u) >> 28) << (4 * i);
    }
    auto B = [&](int i) -> uint32_t { return (b4[i >> 2] >> ((i & 3) * 8)) & 0xffu; };
    // bytes from block byte 0 that a run may use: inside the stream, the
    // segment and the loaded window
    const uint64_t pblk = wpos + sb + lo;
    const uint64_t lim_abs = src_len < seg_end ? src_len : seg_end;
    const uint64_t r1 = lim_abs > pblk ? lim_abs - pblk : 0;
    const uint32_t r2 = need > sb + lo ? need - (sb + lo) : 0u;
    const uint32_t room0 = r1 < (uint64_t)r2 ? (uint32_t)r1 : r2;
#pragma unroll
    for (int e = (int)kBlk - 1; e >= 0; --e) {
      const uint32_t fb = B(e), b1 = B(e + 1);
      const uint32_t kind = fb >> 6, code = (fb >> 1) & 0x1fu;
      const uint32_t W = fbs_width_nb(code);
      const uint32_t L2 = ((fb & 1u) << 8 | b1) + 1u;
      const uint32_t sr_bytes = 2u + ((fb >> 3) & 7u), sr_L = (fb & 7u) + 3u;
      const uint32_t di_bytes = 2u + (W * L2 + 7u) / 8u;
      const uint32_t Wd = code ? W : 0u;
      const uint64_t t1 = term >> (e + 2);
      const uint32_t n1 = t1 ? (uint32_t)__builtin_ctzll(t1) + 1u : 64u;
      const uint64_t t2 = n1 < 32 ? t1 >> n1 : 0ull;
      const uint32_t n2 = t2 ? (uint32_t)__builtin_ctzll(t2) + 1u : 64u;
      const bool de_ok = n1 <= 10 && n2 <= 10 && !(Wd != 0 && L2 < 2);
      const uint32_t de_bytes = 2u + n1 + n2 + (Wd ? (Wd * (L2 - 2u) + 7u) / 8u : 0u);
      const uint32_t bytes = kind == 0 ? sr_bytes : (kind == 1 ? di_bytes : de_bytes);
      const uint32_t L = kind == 0 ? sr_L : L2;
      const uint32_t room = room0 > (uint32_t)e ? room0 - (uint32_t)e : 0u;
      const bool ok = kind != 2 && (kind != 3 || de_ok) && bytes <= room;
      const uint32_t nx = (uint32_t)e + bytes;
      const uint32_t inf = (nx < 15u ? nx : 15u) | (L << 4);
      if (e & 1) info2[e >> 1] = inf << 16;
      else info2[e >> 1] |= inf;
      uint32_t sel = lo + nx;  // the exit when the run leaves the block
      bool past = true;
#pragma unroll
      for (int k = e + 2; k < (int)kBlk; ++k) {
        if (nx == (uint32_t)k) {
          sel = ent[k];
          past = false;
        }
      }
      const bool path_ok = past || !(sel & kDpUnknown);
      ent[e] = (ok && path_ok) ? (past ? sel | (L << 15) : sel + (L << 15)) : kDpUnknown;
    }
  }
  PROF_MARK(3);
  // (2) every block's entry on the chain from slab position 0
  bool has = false;
  uint32_t eb = 0;
  bool chained = false;
  if constexpr ((kOpt & kOptScan) != 0) {
    // f_t: entry state -> entry state of block t + 1, over 16 states (0-7:
    // offset in block t; 8-15: offset in block t + 1, block t skipped), one
    // byte each (0x80 = dead: unknown run, or past the pass's limit); a wave
    // inclusive scan of the compositions (DPP, no LDS) gives each block's
    // entry; a run from an entry that jumps past the next two blocks cannot
    // be expressed, and sends the slab to the pointer-doubling chain below
    // when (and only when) the chain itself takes it
    uint32_t fd[4];
    uint32_t ovf = 0;
#pragma unroll
    for (int x = 0; x < 16; ++x) {
      uint32_t y;
      if (x < (int)kBlk) {
        const uint32_t en = ent[x];
        const uint32_t q = en & 0x7fffu;
        const bool dead = (en & kDpUnknown) || q >= lim;
        const uint32_t rel = q - (lo + kBlk);
        const bool far = !dead && rel >= 16u;
        ovf |= far ? (1u << x) : 0u;
        y = (dead || far) ? 0x80u : rel;
      } else {
        y = (uint32_t)x - kBlk;
      }
      if ((x & 3) == 0) fd[x >> 2] = y;
      else fd[x >> 2] |= y << (8 * (x & 3));
    }
    auto fget = [](const uint32_t* d, uint32_t y) -> uint32_t {
      const uint32_t w = y < 8u ? (y < 4u ? d[0] : d[1]) : (y < 12u ? d[2] : d[3]);
      return (w >> ((y & 3u) * 8u)) & 0xffu;
    };
    // own <- own o fetched (fetched applied first); lanes without a source
    // keep the identity (bound_ctrl off: the old operand)
    auto step = [&](auto ctrl_tag, auto mask_tag) {
      constexpr int kCtrl = decltype(ctrl_tag)::value, kMask = decltype(mask_tag)::value;
      const uint32_t idn[4] = {0x03020100u, 0x07060504u, 0x0B0A0908u, 0x0F0E0D0Cu};
      uint32_t f[4], r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        f[k] = (uint32_t)__builtin_amdgcn_update_dpp((int)idn[k], (int)fd[k], kCtrl, kMask, 0xf, false);
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        const uint32_t y = (f[x >> 2] >> (8 * (x & 3))) & 0xffu;
        const uint32_t z = y < 16u ? fget(fd, y) : 0x80u;
        if ((x & 3) == 0) r[x >> 2] = z;
        else r[x >> 2] |= z << (8 * (x & 3));
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) fd[k] = r[k];
    };
    step(std::integral_constant<int, 0x111>{}, std::integral_constant<int, 0xf>{});  // row_shr:1
    step(std::integral_constant<int, 0x112>{}, std::integral_constant<int, 0xf>{});  // row_shr:2
    step(std::integral_constant<int, 0x114>{}, std::integral_constant<int, 0xf>{});  // row_shr:4
    step(std::integral_constant<int, 0x118>{}, std::integral_constant<int, 0xf>{});  // row_shr:8
    step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xa>{});  // row_bcast:15
    step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xc>{});  // row_bcast:31
    // the wave totals through LDS (the marks' words are free here)
    if (lane == kWave - 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) s_mark[4 * wave + k] = fd[k];
    }
    if (tid == 0) s_mark[16] = 0;
    __syncthreads();
    uint32_t xw = 0;  // the wave's entry state: the slab starts at position 0
    for (int w = 0; w < wave; ++w) {
      const uint32_t t[4] = {s_mark[4 * w], s_mark[4 * w + 1], s_mark[4 * w + 2], s_mark[4 * w + 3]};
      xw = xw < 16u ? fget(t, xw) : 0x80u;
    }
    const uint32_t nxt = xw < 16u ? fget(fd, xw) : 0x80u;  // block t + 1's entry state
    const uint32_t cur = (uint32_t)__builtin_amdgcn_update_dpp((int)xw, (int)nxt, 0x138, 0xf, 0xf, false);  // wave_shr:1
    has = cur < kBlk;
    eb = has ? cur : 0u;
    const bool bad = has && ((ovf >> eb) & 1u);
    if (__ballot(bad) != 0 && lane == 0) s_mark[16] = 1u;
    __syncthreads();
    chained = s_mark[16] != 0;
    if (chained) __syncthreads();  // every wave has read the flag before the chain rewrites the marks
  } else {
    chained = true;
  }
  if (chained) {
    // (2) the chain from slab position 0 by pointer doubling over two
    // successor tables (read one, write the other: one barrier per level)
    uint32_t na[kBlk];
  #pragma unroll
    for (int e = 0; e < (int)kBlk; ++e) {
      const uint32_t x = ent[e] & 0x7fffu;
      na[e] = ((ent[e] & kDpUnknown) || x >= lim) ? (uint32_t)kSink : x;
    }
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    auto put8 = [&](uint16_t* t) {
      u4 w;
      w.x = na[0] | na[1] << 16;
      w.y = na[2] | na[3] << 16;
      w.z = na[4] | na[5] << 16;
      w.w = na[6] | na[7] << 16;
      *(u4*)(t + lo) = w;
    };
    uint16_t* ta = s_nxt;
    uint16_t* tb = s_nxt + kSlab;
    put8(ta);
#ifndef ORCG_DOUBLING_CHAIN
    // (2) the chain by hops, O(slab) work in three barriers: ta = each
    // position's block exit; tb = its 64-byte super-block exit (<= 7 hops
    // over ta, every thread for its 8 positions); one lane hops the <= 32
    // super-blocks from position 0 and records each one's first chain
    // position; every thread hops from its super-block's entry to its own
    // block (<= 7 hops). The pointer doubling below (ORCG_DOUBLING_CHAIN)
    // took 8 levels of marks and gathers over the whole slab.
    constexpr uint32_t kSup = 8u * kBlk;
    __syncthreads();
    {
      const uint32_t send = (lo / kSup + 1u) * kSup;
      uint32_t q[kBlk];
  #pragma unroll
      for (int e = 0; e < (int)kBlk; ++e) q[e] = na[e];
  #pragma unroll
      for (int h = 0; h < 7; ++h) {
  #pragma unroll
        for (int e = 0; e < (int)kBlk; ++e) {
          const bool in = q[e] != kSink && q[e] < send;
          const uint32_t v = ta[in ? q[e] : lo + (uint32_t)e];
          q[e] = in ? v : q[e];
        }
      }
      typedef uint32_t u4h __attribute__((ext_vector_type(4)));
      u4h w;
      w.x = q[0] | q[1] << 16;
      w.y = q[2] | q[3] << 16;
      w.z = q[4] | q[5] << 16;
      w.w = q[6] | q[7] << 16;
      *(u4h*)(tb + lo) = w;
    }
    if (tid < (int)(kSlab / kSup)) s_mark[tid] = kSink;  // the super-blocks' chain entries
    __syncthreads();
    if (tid == 0) {
      uint32_t p = 0;
      while (p != kSink && p < lim) {
        s_mark[p / kSup] = p;
        p = tb[p];
      }
    }
    __syncthreads();
    {
      uint32_t p = s_mark[lo / kSup];
      for (int h = 0; h < 7 && p != kSink && p < lo; ++h) p = ta[p];
      has = p != kSink && p >= lo && p < hi && p < lim;
      eb = has ? p - lo : 0u;
    }
    static_assert(kSlab / kSup <= kSlab / 32, "super-block entries fit the marks");
#else
    if (tid < (int)(kSlab / 32)) s_mark[tid] = tid == 0;  // position 0 starts the chain
    __syncthreads();
  #pragma unroll 1
    for (int lev = 0; lev < 8; ++lev) {
      const uint32_t m8 = (s_mark[lo >> 5] >> (lo & 31u)) & 0xffu;
      if (m8) {
        // marked positions mark their successor (marks only grow, and every
        // marked position is a chain element, so racing with this level's
        // readers is harmless)
  #pragma unroll
        for (int e = 0; e < (int)kBlk; ++e) {
          const bool go = ((m8 >> e) & 1u) && na[e] != kSink;
          if constexpr ((kOpt & kOptD3) != 0) {
            if (go) atomicOr(&s_mark[na[e] >> 5], 1u << (na[e] & 31u));
          } else {
            const uint32_t n = go ? na[e] : 0u;
            atomicOr(&s_mark[n >> 5], go ? 1u << (n & 31u) : 0u);
          }
        }
      }
  #pragma unroll
      for (int e = 0; e < (int)kBlk; ++e) {
        const bool valid = na[e] != kSink;
        const uint32_t v = ta[valid ? na[e] : lo + (uint32_t)e];
        na[e] = valid ? v : (uint32_t)kSink;
      }
      put8(tb);
      uint16_t* t = ta;
      ta = tb;
      tb = t;
      __syncthreads();
    }
    const uint32_t mb = (s_mark[lo >> 5] >> (lo & 31u)) & 0xffu;
    has = mb != 0;
    eb = has ? (uint32_t)__builtin_ctz(mb) : 0u;
#endif
  }
  PROF_MARK(4);
  // (3) the block's entry, its runs (a forward pass over the DP registers),
  // one combined scan of the values and run counts
  uint32_t ee = ent[0];
#pragma unroll
  for (int k = 1; k < (int)kBlk; ++k) ee = eb == (uint32_t)k ? ent[k] : ee;
  const bool exact = has && (ee & kDpUnknown);
  uint32_t cnt = 0, pk_off = 0, cum = 0, p_end = ee & 0x7fffu;
  uint64_t pk_val = 0;
  bool stopped = false;
  if (has && !exact) {
    uint32_t reach = 1u << eb;
#pragma unroll
    for (int e = 0; e < (int)kBlk; ++e) {
      const bool on = ((reach >> e) & 1u) && !stopped;
      const bool st = on && lo + (uint32_t)e >= lim;
      p_end = st ? lo + (uint32_t)e : p_end;
      stopped = stopped || st;
      const bool em = on && !st;
      const uint32_t inf = (info2[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
      const uint32_t nx = inf & 15u, Le = inf >> 4;
      pk_off |= em ? (uint32_t)e << (3 * cnt) : 0u;
      pk_val |= em ? (uint64_t)cum << (16 * cnt) : 0ull;
      cnt += em ? 1u : 0u;
      reach |= (em && nx < kBlk) ? 1u << nx : 0u;
      cum += em ? Le : 0u;
    }
  }
  uint32_t* s_wsum = s_ctl + 4;  // [0..3] value totals, [4..7] run-count totals of the waves
  const uint32_t vincl = wave_scan_u32(cum), cincl = wave_scan_u32(cnt);
  if (lane == kWave - 1) {
    s_wsum[wave] = vincl;
    s_wsum[4 + wave] = cincl;
  }
  if (tid == 0) {
    s_ctl[3] = 0;       // stop (corrupt run)
    s_ctl[12] = kNone;  // first block whose walk stopped inside it
    s_ctl[13] = 0;      // last block with an entry
    s_ctl[14] = 0;      // runs of the exact-walk block
  }
  __syncthreads();
  uint32_t vb = vincl - cum, base = cincl - cnt;
  for (int w = 0; w < wave; ++w) {
    vb += s_wsum[w];
    base += s_wsum[4 + w];
  }
  uint32_t total = s_wsum[4] + s_wsum[5] + s_wsum[6] + s_wsum[7];
  uint32_t v_end = vb + cum;
  if (exact) {
    // the path meets a run the DP cannot vouch for (it is the pass's last
    // block with an entry): walk it exactly
    uint32_t p = lo + eb, v = vb;
    while (p < hi && p < lim && vi + v < value_end) {
      Run r;
      const uint32_t e = checked_run(win, sb + p, wpos, seg_end, src_len, need, is_signed, &r);
      if (e != kErrNone) {
        report(err, vi + v, e);
        s_ctl[3] = 1;
        break;
      }
      pk_off |= (p - lo) << (3 * cnt);
      pk_val |= (uint64_t)(v - vb) << (16 * cnt);
      ++cnt;
      p += r.bytes;
      v += r.L;
    }
    stopped = p < hi;
    p_end = p;
    v_end = v;
    s_ctl[14] = cnt;
  }
  if constexpr ((kOpt & kOptD3) != 0) {
    // one atomic per wave: its first stopped lane, its last lane with an entry
    const uint64_t bs = __ballot(has && stopped), bh = __ballot(has);
    if (bs && lane == __builtin_ctzll(bs)) atomicMin(&s_ctl[12], (uint32_t)tid);
    if (bh && lane == 63 - __builtin_clzll(bh)) atomicMax(&s_ctl[13], (uint32_t)tid);
  } else if (has) {
    if (stopped) atomicMin(&s_ctl[12], (uint32_t)tid);
    atomicMax(&s_ctl[13], (uint32_t)tid);
  }
  // the successor tables are dead: the run table may overwrite them
  __syncthreads();
  {
    const uint32_t fin = s_ctl[12] != kNone ? s_ctl[12] : s_ctl[13];
    if ((uint32_t)tid == fin) {
      s_ctl[1] = p_end;
      s_ctl[2] = v_end;
    }
  }
  total += s_ctl[14];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (k < cnt) {
      s_off[base + k] = (OffT)(sb + lo + ((pk_off >> (3 * k)) & 7u));
      s_val[base + k] = vb + (uint32_t)((pk_val >> (16 * k)) & 0xffffu);
    }
  __syncthreads();
  PROF_MARK(5);
  __builtin_amdgcn_s_setprio(0);
  return DenseResult{uni(total), uni(s_ctl[3]), uni(s_ctl[1]), uni(s_ctl[2])};
}

// Expand runs [r0, r1) of the run table with one wave: maximal groups of
// consecutive short runs (<= kStage values) are decoded one lane per run into
// the wave's LDS stage and flushed with coalesced stores; any other run
// (long, PATCHED_BASE) goes through expand_run.
template <int kOpt, typename T, typename OffT>
__device__ __forceinline__ void dense_expand(const uint32_t* win, uint32_t nwords, const OffT* s_off,
                                             const uint32_t* s_val, uint64_t* stage, uint32_t r0, uint32_t r1,
                                             uint64_t vi, int is_signed, uint64_t value_begin, uint64_t value_end,
                                             T* dst, int lane) {
  uint32_t c = r0;
  while (c < r1) {
    const uint32_t r = c + (uint32_t)lane;
    const bool act = r < r1;
    const uint32_t hoff = act ? s_off[r] : s_off[c];
    const uint32_t val = act ? s_val[r] : 0u;
    // the run's first 12 bytes in registers (one LDS round trip)
    const uint32_t w0 = hoff >> 2, sh = hoff & 3u;
    const uint32_t d0 = win[w0], d1 = win[w0 + 1], d2 = win[w0 + 2], d3 = win[w0 + 3];
    const uint32_t b0 = __builtin_amdgcn_alignbyte(d1, d0, sh), b1 = __builtin_amdgcn_alignbyte(d2, d1, sh),
                   b2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
    const uint32_t fb = b0 & 0xffu;
    Run run;
    if (__ballot(act && (fb >> 6) != 0) == 0) {
      // SHORT_REPEAT only (low-cardinality streams): W + 1 value bytes, big endian
      run.kind = 0;
      run.L = (fb & 7u) + 3u;
      const uint32_t nb = ((fb >> 3) & 7u) + 1u;
      const uint64_t be = ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(b1, b0, 1)) << 32) |
                          __builtin_bswap32(__builtin_amdgcn_alignbyte(b2, b1, 1));
      const uint64_t v = be >> (64 - 8 * nb);
      run.a = is_signed ? unzigzag(v) : v;
      run.W = 8 * nb;
      run.data = 1;
      run.b = 0;
    } else {
      run = parse_run([&](uint32_t i) { return lds_byte(win, hoff + i); }, ~0ull, kHdrLim, is_signed);
    }
    // SHORT_REPEAT, DIRECT and constant-step DELTA runs of kVparMin + 1 ..
    // kVparL values are expanded value-parallel (below); short runs (<=
    // kShortL) one lane per run through the stage; the rest (long runs,
    // PATCHED_BASE) by the whole wave each
    // Short runs stay one lane per run (their stage flush needs them
    // consecutive) unless the longer runs between them cut them into more
    // than kVparFrag groups (low-cardinality dictionary indices: a flush per
    // group of a few runs); then every eligible run goes value-parallel
    const bool elig = act && run.L <= kVparL && (run.kind <= 1 || (run.kind == 3 && run.W == 0));
    const bool sh0 = act && run.kind != 2 && run.L <= kShortL;
    const uint64_t shm = __ballot(sh0);
    const bool frag = (uint32_t)__builtin_popcountll(shm & ~(shm << 1)) > kVparFrag;
    const bool vpr = elig && (run.L > kVparMin || frag);
    const bool shortr = sh0 && !vpr;
    const uint32_t Ls = shortr ? run.L : 0u;
    const uint32_t incl = wave_scan_u32(Ls);
    constexpr bool kStraight = (kOpt & kOptDirect) != 0;
    // every run parsed here is expanded before the next 64 are parsed
    // (a mix of short and long runs, e.g. low-cardinality dictionary
    // indices, used to parse its 64 headers again after every long run):
    // first the runs of consecutive short runs, through the stage (or
    // straight), then each long / PATCHED_BASE run by the whole wave, once
    // the parsed runs are dead (fewer live registers around expand_run)
    const uint32_t nact = r1 - c < (uint32_t)kWave ? r1 - c : (uint32_t)kWave;
    const uint64_t longm = __ballot(act && !vpr && !shortr);
    {
      // value-parallel: lane o of each step takes value o of the runs'
      // concatenation, finds its run by a binary search over the runs' first
      // values (ds_bpermute, 6 steps), and decodes it by random access (a
      // lane per run left most lanes idle behind the longest run of the 64,
      // and runs of 17-256 values went one whole-wave expansion each: the
      // low-cardinality dictionary indices of C4 spent 120 us a workgroup
      // here)
      const uint32_t Lv = vpr ? run.L : 0u;
      const uint32_t inclv = wave_scan_u32(Lv);
      const uint32_t exclv = inclv - Lv;
      const uint32_t Tv = rdlane(inclv, kWave - 1);
      if (Tv) {
        const uint32_t pk = (hoff + run.data) | (run.W << 16) | (run.kind << 24);
        const uint32_t a_lo = (uint32_t)run.a, a_hi = (uint32_t)(run.a >> 32);
        const bool anyd = __ballot(vpr && run.kind == 3) != 0;
        for (uint32_t o = (uint32_t)lane; __ballot(o < Tv) != 0; o += kWave) {
          uint32_t lo = 0, hi = kWave;
#pragma unroll
          for (int st = 0; st < 6; ++st) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint32_t e = (uint32_t)__shfl((int)exclv, (int)mid);
            if (e <= o) lo = mid;
            else hi = mid;
          }
          const uint32_t k = lo;
          const uint32_t p = (uint32_t)__shfl((int)pk, (int)k), e = (uint32_t)__shfl((int)exclv, (int)k);
          const uint32_t vk = (uint32_t)__shfl((int)val, (int)k);
          const uint64_t ak = (uint64_t)(uint32_t)__shfl((int)a_lo, (int)k) |
                              (uint64_t)(uint32_t)__shfl((int)a_hi, (int)k) << 32;
          const uint32_t j = o - e, kind = p >> 24;
          uint64_t x = ak;
          if (kind == 1) {
            const uint32_t W = (p >> 16) & 0xffu, bit = j * W, br = (p & 0xffffu) + (bit >> 3);
            const uint64_t v = field(lds12(win, br), br, bit & 7u, W);
            x = is_signed ? unzigzag(v) : v;
          }
          if (anyd) {
            const uint64_t bk = (uint64_t)(uint32_t)__shfl((int)(uint32_t)run.b, (int)k) |
                                (uint64_t)(uint32_t)__shfl((int)(uint32_t)(run.b >> 32), (int)k) << 32;
            if (kind == 3) x = ak + (uint64_t)j * bk;
          }
          const uint64_t g = vi + vk + j;
          if (o < Tv && g >= value_begin && g < value_end) store1<kOpt>(dst + (g - value_begin), x);
        }
        ORCG_COVER_ADD(vpr ? run.L : 0u);
      }
    }
    for (uint64_t rem = __ballot(shortr); rem;) {
      const uint32_t a = (uint32_t)__builtin_ctzll(rem);
      // short runs [a, b): consecutive in the output; a stage-full at most
      const uint32_t base = a ? rdlane(incl, a - 1) : 0u;
      const uint64_t stop_m = __ballot((uint32_t)lane >= a && (!shortr || (!kStraight && incl - base > kStage)));
      uint32_t b = stop_m ? (uint32_t)__builtin_ctzll(stop_m) : (uint32_t)kWave;
      if (b > nact) b = nact;
      rem &= b >= (uint32_t)kWave ? 0ull : ~((1ull << b) - 1ull);
      const bool mine = (uint32_t)lane >= a && (uint32_t)lane < b;
      const uint32_t myl = mine ? Ls : 0u;
      ORCG_COVER_ADD(myl);
      if constexpr (kStraight) {
        // each lane stores its run's values at their output positions
        const uint64_t g0 = vi + val;
        if (__ballot(mine && run.kind != 0) == 0) {
          for (uint32_t j = 0; __ballot(j < myl) != 0; ++j) {
            const uint64_t g = g0 + j;
            if (j < myl && g >= value_begin && g < value_end) store1<kOpt>(dst + (g - value_begin), run.a);
          }
        } else {
          uint64_t acc = 0;
          for (uint32_t j = 0; __ballot(j < myl) != 0; ++j) {
            const uint64_t g = g0 + j;
            const uint64_t x = j < myl ? short_value(win, run, hoff, j, is_signed, acc) : 0ull;
            if (j < myl && g >= value_begin && g < value_end) store1<kOpt>(dst + (g - value_begin), x);
          }
        }
        continue;
      }
      const uint32_t st0 = incl - Ls - base;
      if (__ballot(mine && run.kind != 0) == 0) {
        for (uint32_t j = 0; __ballot(j < myl) != 0; ++j)
          if (j < myl) stage[st0 + j] = run.a;
      } else {
        uint64_t acc = 0;
        for (uint32_t j = 0; __ballot(j < myl) != 0; ++j)
          if (j < myl) stage[st0 + j] = short_value(win, run, hoff, j, is_signed, acc);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const uint32_t tot = rdlane(incl, b - 1) - base;
      const uint64_t g0 = vi + rdlane(val, a);
      for (uint32_t o = (uint32_t)lane; o < tot; o += kWave) {
        const uint64_t g = g0 + o;
        if (g >= value_begin && g < value_end) store1<kOpt>(dst + (g - value_begin), stage[o]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    for (uint64_t m = longm; m; m &= m - 1) {
      const uint32_t a = (uint32_t)__builtin_ctzll(m);
#ifdef ORCG_DEBUG_COVER
      if (lane == 0) ORCG_COVER_ADD(parse_run([&](uint32_t i) { return lds_byte(win, uni(s_off[c + a]) + i); }, ~0ull,
                                              kHdrLim, is_signed).L);
#endif
      expand_run<kOpt>(win, nwords, uni(s_off[c + a]), vi + uni(s_val[c + a]), is_signed, value_begin, value_end, dst,
                       lane);
    }
    c += nact;
  }
}

__device__ __forceinline__ void lds_barrier() {
  // LDS ordering only: never drains the output stores (vmcnt).
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Dense v2 LDS: the run table (u16 window offsets, u32 value offsets) shares
// its bytes with the chain's single successor table (dead once the runs are
// emitted); per-wave value stages; chain marks.
struct Dense2Lds {
  union {
    struct {
      uint16_t off[kDenseRuns];
      uint32_t val[kDenseRuns];
      uint16_t items[kDenseRuns];  // serial passes: work item ends
    } tab;
    uint16_t nxt[2 * kSlab];
  };
  uint64_t stage[kThreads / kWave][kStage];
  uint32_t mark[kSlab / 32];
};

// Union instances (kOptUnion): the run table / successor tables only; the
// value stages and the marks live past the dense window inside s_win, which a
// serial window covers whole.
struct Dense2TabLds {
  union {
    struct {
      uint16_t off[kDenseRuns];
      uint32_t val[kDenseRuns];
      uint16_t items[kDenseRuns];
    } tab;
    uint16_t nxt[2 * kSlab];
  };
};

// Deferral (kDefer): a serial-walk instance (kDefer = 1) whose probe pass
// finds short runs stops at the end of that pass and records {stamp, byte
// offset, value index} in the segment's own entry of `defer_q` (3 words per
// launch-wide segment; stamp = the launch pair's sequence number
// `defer_par`); the dense instance launched right after it (kDefer = 2)
// decodes the stamped segments with a persistent grid, each workgroup a
// static share, so a short-run segment never runs the one-wave header walk,
// whatever the stream's overall density. Entries of older launches carry
// older stamps: nothing is ever reset.
template <typename T, bool kPositions, int kOpt, int kWinKB, bool kPipe, int kMinWaves, int kDense = 0, int kDefer = 0,
          bool kMulti = false>
__global__ __launch_bounds__(kThreads, kMinWaves) void rlev2_tiled_kernel(
    const uint8_t* __restrict__ p_src, uint64_t p_src_len, int p_is_signed,
    const uint64_t* __restrict__ p_segtab, uint64_t p_nsegs, uint64_t rows_per_group,
    uint64_t p_value_begin, uint64_t p_nvalues, T* __restrict__ p_dst, unsigned long long* p_err,
    unsigned long long* __restrict__ defer_q, uint32_t defer_par, const RleJob* __restrict__ jobs,
    uint32_t njobs, const uint64_t* __restrict__ p_dcount, const RunTab rtab) {
  // dense instances get 512 B more so the window's run-start chunk is a
  // whole number of 2 KB slabs (no partially occupied discovery pass)
  constexpr uint32_t kWin = kWinKB * 1024u + (kDense ? 512u : 0u);
  constexpr uint32_t kChunk = kWin - kMaxRun;
  // union instances: serial windows of kWinS bytes = the dense window, its
  // 32-byte slack, the value stages and the marks
  constexpr bool kUnion = kDense == 2 && (kOpt & kOptUnion) != 0;
  // density hysteresis (stream bytes per run)
  constexpr uint32_t kDenseB = (kOpt & kOptTable) ? kTabToDense : kToDense;
  constexpr uint32_t kSerialB = (kOpt & kOptTable) ? kTabToSerial : kToSerial;
  constexpr uint32_t kWinS = kUnion ? kWin + (uint32_t)(kWaves * kStage * 8 + kSlab / 8) : kWin;
  constexpr uint32_t kChunkS = kWinS - kMaxRun;
  static_assert(!kUnion || (kWin + 32) % 8 == 0, "stage alignment");
  static_assert(!kDense || kChunk % kSlab == 0, "dense window chunk must be whole slabs");
  constexpr int kBufs = kPipe ? 2 : 1;
  static_assert(!(kDense && kPipe), "dense mode is a non-pipelined instance");
  // run table capacity; in dense v1 instances the slab DP table aliases it
  constexpr uint32_t kCap = kDense ? kDenseRuns : 512u;
  static_assert(!kDense || 2 * kCap >= kSlab, "DP table must fit the run table");
  static_assert(!kDense || kChunk >= kSlab, "window too small for a slab");
  using OffT = typename std::conditional<kDense == 2, uint16_t, uint32_t>::type;
  __shared__ __attribute__((aligned(16))) uint32_t s_win[kBufs][kWinS / 4 + 8];  // + 32 B: the 12-byte extract may read past a run
  __shared__ uint32_t s_ctl[kBufs][16];
  __shared__ uint32_t s_sync[2][2];  // serial passes: {published runs, claimed runs}, by pass parity
  OffT* s_off[kBufs];
  uint32_t* s_val[kBufs];
  uint16_t* s_nxt2 = nullptr;   // v2: successor table, marks, stages
  uint32_t* s_mark2 = nullptr;
  uint64_t* s_stage2 = nullptr;
  uint16_t* s_items = nullptr;  // serial passes (non-pipelined): work item ends
  if constexpr (kUnion) {
    __shared__ __attribute__((aligned(16))) Dense2TabLds s_d2;
    s_items = s_d2.tab.items;
    s_off[0] = s_d2.tab.off;
    s_val[0] = s_d2.tab.val;
    s_nxt2 = s_d2.nxt;
    s_stage2 = (uint64_t*)((char*)s_win[0] + kWin + 32);
    s_mark2 = (uint32_t*)((char*)s_win[0] + kWin + 32 + kWaves * kStage * 8);
  } else if constexpr (kDense == 2) {
    __shared__ __attribute__((aligned(16))) Dense2Lds s_d2;
    s_items = s_d2.tab.items;
    s_off[0] = s_d2.tab.off;
    s_val[0] = s_d2.tab.val;
    s_nxt2 = s_d2.nxt;
    s_mark2 = s_d2.mark;
    s_stage2 = &s_d2.stage[0][0];
  } else {
    __shared__ uint32_t s_tab[kBufs][2 * kCap];
    for (int b = 0; b < kBufs; ++b) {
      s_off[b] = s_tab[b];
      s_val[b] = s_tab[b] + kCap;
    }
    if constexpr (!kPipe) {
      __shared__ uint16_t s_itm[kCap];
      s_items = s_itm;
    }
  }

  const int tid = (int)threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
#ifdef ORCG_PHASE_PROF
  const uint64_t wg_t0 = wall_clock64();
  uint32_t wg_dense = 0, wg_serial = 0;
#endif
  // the stream of the segment being decoded: the launch's, or (multi-stream
  // instances, kMulti) the job of `jobs` that owns the launch-wide segment
  // index (single-stream instances never rebind: the arguments stay as they
  // are, scalar and rematerialisable)
  const uint8_t* src = p_src;
  uint64_t src_len = p_src_len;
  int is_signed = p_is_signed;
  const uint64_t* segtab = p_segtab;
  const int64_t* trip = nullptr;  // multi-stream row-index jobs (RleJob::trip)
  const int64_t* rows = nullptr;
  uint64_t nsegs = p_nsegs;
  uint64_t value_begin = p_value_begin;
  // (p_dcount: the value count lives on the device, e.g. a nullable
  // column's non-null rows counted by its PRESENT decode; p_nvalues is then
  // only the output's capacity)
  uint64_t value_end = p_value_begin + (p_dcount ? uni64(*p_dcount) : p_nvalues);
  T* dst = p_dst;
  unsigned long long* err = p_err;
  uint32_t tab_base = 0;  // kOptTable: the stream's first run-table entry
  uint32_t job_idx = 0;   // kMulti: the segment's job
  auto bind = [&](const uint64_t gg) -> uint64_t {
    if constexpr (!kMulti) return gg;
    uint32_t lo = 0, hi = njobs - 1;
    while (lo < hi) {  // last job whose first segment is <= gg
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (uni64(jobs[mid].seg_base) <= gg) lo = mid;
      else hi = mid - 1;
    }
    const RleJob* J = jobs + lo;
    src = (const uint8_t*)uni64((uint64_t)(uintptr_t)J->src);
    src_len = uni64(J->src_len);
    is_signed = (int)uni(J->is_signed);
    segtab = (const uint64_t*)uni64((uint64_t)(uintptr_t)J->segtab);
    trip = (const int64_t*)uni64((uint64_t)(uintptr_t)J->trip);
    rows = (const int64_t*)uni64((uint64_t)(uintptr_t)J->rows);
    nsegs = uni64(J->nsegs);
    value_begin = 0;
    const uint64_t jdc = uni64((uint64_t)(uintptr_t)J->dcount);
    value_end = jdc ? uni64(*(const uint64_t*)(uintptr_t)jdc) : uni64(J->nvalues);
    dst = (T*)uni64((uint64_t)(uintptr_t)J->dst);
    const uint64_t je = uni64((uint64_t)(uintptr_t)J->err);
    err = je ? (unsigned long long*)(uintptr_t)je : p_err;
    tab_base = uni(J->tab_base);
    job_idx = lo;
    return gg - uni64(J->seg_base);
  };

  // one segment, from its start or (queued) from a byte offset / value index
  auto run_segment = [&](const uint64_t gg, const bool queued, const uint64_t q_pos, const uint64_t q_vi) {
  const uint64_t g = bind(gg);
  // segment g: {first byte, index of its first value}
  auto seg_at = [&](const uint64_t s, uint64_t* off) -> uint64_t {
    if (kMulti && trip) {
      const int64_t v = rows[s] - trip[3 * s + 1];
      *off = (uint64_t)trip[3 * s];
      return v < 0 ? 0ull : (uint64_t)v;
    }
    *off = segtab[2 * s];
    return kPositions ? s * rows_per_group - segtab[2 * s + 1] : segtab[2 * s + 1];
  };
  uint64_t seg_first = 0;
  const uint64_t vi0 = queued ? 0ull : seg_at(g, &seg_first);
  const uint64_t seg_start = queued ? q_pos : seg_first;
  uint64_t vi = queued ? q_vi : vi0;
  uint64_t seg_end = src_len;
  uint64_t v_next = ~0ull;
  if (g + 1 < nsegs) v_next = seg_at(g + 1, &seg_end);
  if (seg_end > src_len) seg_end = src_len;
  // kOptTable: the segment's header and run table (RunTab). Its runs lie in
  // [seg_first, next segment's first byte) and are >= 2 bytes each, so
  // seg_first / 2 + g leaves every earlier segment room for its runs.
  constexpr bool kTable = (kOpt & kOptTable) != 0;
  uint32_t* thdr = nullptr;
  uint64_t* ttab = nullptr;
  uint32_t tcnt = 0;                                     // entries written
  const uint64_t tlim = (uint64_t)rtab.spg * rtab.slice;  // values the slices cover
  if constexpr (kTable) {
    thdr = rtab.hdr + gg * (kRtHdr + rtab.spg);
    const uint32_t tb = tab_base + (uint32_t)(seg_first >> 1) + (uint32_t)g;
    ttab = rtab.tab + tb;
    if (tid == 0) {
      thdr[0] = 0;
      thdr[1] = 0;
      thdr[2] = (uint32_t)vi0;
      thdr[3] = (uint32_t)(vi0 >> 32);
      thdr[4] = tb;
      thdr[5] = job_idx;
    }
  }
  if (vi >= value_end || v_next <= value_begin) return;
  if (seg_start >= seg_end) {
    if (tid == 0 && v_next != ~0ull && v_next != vi && seg_start < src_len) report(err, vi, kErrBadSegment);
    if (tid == 0 && v_next == ~0ull) report(err, vi, kErrBadRead);  // no stream left for the requested values
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
  uint32_t sync_par = 0;
  if (tid < 4) s_sync[tid >> 1][tid & 1] = 0;  // ordered before use by the first window's barrier
  PROF_DECL;
  if constexpr (!kPipe) {
    uint64_t pwpos = ~0ull;  // previous window (stream offset) and its valid bytes
    uint32_t pneed = 0;
    // kOptPrefetch: the next window's bytes, loaded into registers during
    // the previous window's expansion (pf_wrel: its descriptor offset)
    constexpr bool kPf = (kOpt & kOptPrefetch) != 0 && (kOpt & kOptRegFill) != 0 && (kOpt & kOptReuse) != 0 &&
                         kDense == 0;
    typedef uint32_t pf_u4 __attribute__((ext_vector_type(4)));
    constexpr int kPfPer = kPf ? (int)((kWinS + kThreads * 16 - 1) / (kThreads * 16)) : 1;
    pf_u4 pf[kPfPer];
    uint32_t pf_wrel = ~0u, pf_need = 0;
    // wave-uniform mode of the next pass (dense instances only): the
    // segment's first pass is a short serial probe (32 runs in v1, 4 in v2)
    // whose bytes per run pick the mode
    bool dense = queued;
    bool probe = !queued;
    if constexpr (kDense == 2 && (kOpt & kOptD3) != 0) {
      // queued segments (short runs by values) are sized by the inline
      // probe too: dense discovery for short runs in bytes, the serial walk
      // with staged group expansion for wide ones
      dense = false;
      probe = true;
    }
    while (pos < seg_end && vi < value_end) {
      const uint32_t wrel = (uint32_t)(pos - bias) & ~15u;
      const uint64_t wpos = bias + wrel;
      // union instances: a window whose runs are known to be long (the probe
      // is done and the mode is serial) is a serial window of kWinS bytes:
      // serial passes only, short-run groups expanded without the stage
      const bool big = kUnion && !dense && !probe;
      uint32_t need = big ? kWinS : kWin, keep = 0;
      if constexpr ((kOpt & kOptReuse) != 0) {
        // never load past the segment: its runs end at seg_end
        const uint64_t end_rel = (seg_end - bias + 15) & ~15ull;
        if (end_rel - wrel < need) need = (uint32_t)(end_rel - wrel);
        // the previous window's tail [wpos, pwpos + pneed) is already in LDS:
        // move it to the front instead of re-reading it (source and
        // destination must not overlap: the shift is at least the length;
        // otherwise reload)
        const bool prefetched = kPf && pf_wrel == wrel && pf_need == need;
        if (!prefetched && pwpos != ~0ull && pwpos + pneed > wpos && wpos - pwpos >= pwpos + pneed - wpos) {
          keep = (uint32_t)(pwpos + pneed - wpos);
          if (keep > need) keep = need;
          const uint32_t so = (uint32_t)(wpos - pwpos);
          typedef uint32_t u4 __attribute__((ext_vector_type(4)));
          for (uint32_t o = tid * 16u; o < keep; o += kThreads * 16u)
            *(u4*)((char*)s_win[0] + o) = *(const u4*)((const char*)s_win[0] + so + o);
          __syncthreads();  // reads of the tail finish before the DMA below lands
        }
        if constexpr ((kOpt & kOptRegFill) != 0) {
          // every lane issues all of its 16-byte loads before the first LDS
          // write (measured: +4 % over LDS-DMA on a pure window copy)
          typedef uint32_t u4 __attribute__((ext_vector_type(4)));
          constexpr int kPer = (kWinS + kThreads * 16 - 1) / (kThreads * 16);
          if (kPf && prefetched) {
            // the whole window arrived in registers during the last expansion
#pragma unroll
            for (int i = 0; i < kPfPer; ++i) {
              const uint32_t off = (uint32_t)(i * kThreads + tid) * 16u;
              if (off < need) *(u4*)((char*)s_win[0] + off) = __builtin_bit_cast(u4, pf[i]);
            }
          } else {
            u4 v[kPer];
#pragma unroll
            for (int i = 0; i < kPer; ++i) {
              const uint32_t off = keep + (uint32_t)(i * kThreads + tid) * 16u;
              if (off < need)
                v[i] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, wrel + off, 0, 2));
            }
#pragma unroll
            for (int i = 0; i < kPer; ++i) {
              const uint32_t off = keep + (uint32_t)(i * kThreads + tid) * 16u;
              if (off < need) *(u4*)((char*)s_win[0] + off) = v[i];
            }
          }
          pf_wrel = ~0u;
        } else {
          for (uint32_t off = keep + wave * 1024u; off < need; off += kWaves * 1024u)
            if (off + lane * 16u < need)
              __builtin_amdgcn_raw_ptr_buffer_load_lds(
                  rs, (__attribute__((address_space(3))) void*)((char*)s_win[0] + off), 16,
                  wrel + off + lane * 16u, 0, 0, (kOpt & kOptNTLoad) ? 2 : 0);
        }
      } else {
        fill<kOpt>(s_win[0], rs, wrel, kWin, wave, kWaves, lane);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      PROF_MARK(0);
      if constexpr (kDense == 2 && (kOpt & kOptD3) != 0) {
        // inline probe (no serial pass): one lane sizes the segment's first
        // runs; short ones (< kToDense stream bytes each) start it dense
        if (probe) {
          if (tid == 0) {
            uint32_t p = (uint32_t)(pos - wpos), nb = 0, nr = 0;
            while (nr < 4 && nb < 4 * kDenseB && p + kHdrLim < need) {
              const Run r = parse_run([&](uint32_t i) { return lds_byte(s_win[0], p + i); }, ~0ull, kHdrLim, is_signed);
              if (r.err != kErrNone || r.kind == 2) break;
              nb += r.bytes;
              p += r.bytes;
              ++nr;
            }
            s_ctl[0][15] = (nr == 4 && nb < 4 * kDenseB) ? 1u : 0u;
          }
          __syncthreads();
          dense = uni(s_ctl[0][15]) != 0;
          probe = false;
        }
      }
      // every run that starts in the window's first kChunk bytes ends inside
      // it: consume them all (several passes) before moving the window
      do {
        uint32_t n, stop, dpos, dval, shrt = 0;
#ifdef ORCG_DEBUG_COVER
        if (tid == 0) *s_cover_ptr() = 0;
        __syncthreads();
#endif
        bool was_dense = false;
        bool tabled = false;  // kOptTable: this pass's runs went to the run table
        if constexpr (kDense) was_dense = dense;
        if (was_dense) {
          const uint32_t sb = (uint32_t)(pos - wpos);
          const uint32_t lim = min(kSlab, kChunk - sb);
          DenseResult d;
          if constexpr (kDense == 2) {
            d = dense2_discover<kOpt>(s_win[0], s_off[0], s_val[0], s_nxt2, s_mark2, s_ctl[0], wpos, sb, lim, vi, seg_end,
                                src_len, value_end, need, is_signed, err, tid
#ifdef ORCG_PHASE_PROF
                                , prof_last_
#endif
            );
          }
          n = d.n;
          stop = d.stop;
          dpos = d.dpos;
          dval = d.dval;
          if constexpr (kTable) {
            // the runs go to the run table (entry: stream byte offset | first
            // value in the segment << 32); a run holding slice boundary k * S
            // is where slice k starts (runs are <= 512 < S values: one each)
            const uint64_t vrel = vi - vi0;
            if (vrel + dval <= tlim) {
              tabled = true;
              const uint32_t vr = (uint32_t)vrel, S = rtab.slice;
              for (uint32_t r = (uint32_t)tid; r < n; r += kThreads) {
                const uint32_t v = vr + s_val[0][r];
                const uint32_t ve = vr + (r + 1 < n ? s_val[0][r + 1] : dval);
                ttab[tcnt + r] = (wpos + s_off[0][r]) | ((uint64_t)v << 32);
                const uint32_t kb = (v + S - 1) / S;
                if (kb >= 1 && kb * S < ve) thdr[kRtHdr + kb] = tcnt + r;
              }
              tcnt += n;
            }
          }
          if constexpr (kDense != 0) {
            if (!tabled) {
              uint64_t* const stage = s_stage2 + wave * kStage;
              const uint32_t r0 = (uint32_t)(((uint64_t)n * wave) / kWaves),
                             r1 = (uint32_t)(((uint64_t)n * (wave + 1)) / kWaves);
              dense_expand<kOpt>(s_win[0], kWin / 4 + 8, s_off[0], s_val[0], stage, r0, r1, vi, is_signed,
                                 value_begin, value_end, dst, lane);
            }
          }
        } else {
          // Wave 0 walks and publishes work items (a group of short runs or
          // one long run) as they close; every wave (wave 0 once its walk is
          // done) claims published items from an LDS counter and expands
          // them, so the walk overlaps the expansion.
          uint32_t* s_pub = &s_sync[sync_par][0];
          uint32_t* s_claim = &s_sync[sync_par][1];
          if (wave == 0) {
            // the walk is the workgroup's critical path: raise its issue
            // priority over co-resident waves that are expanding
            __builtin_amdgcn_s_setprio(3);
            // a segment's first walk probes its first runs (4 in dense v2
            // instances, 8 in queueing serial ones) and stops there when
            // they are short; a long-run segment just walks on (dense v1:
            // a separate 32-run probe pass)
            const uint32_t probe_n = (probe && (kDense == 2 || kDefer == 1)) ? (kDense == 2 ? 4u : 8u) : 0u;
            constexpr bool kProbeValues = kDefer == 1 && (kOpt & kOptD3) != 0;
            const uint32_t cap = (kDense == 1 && probe) ? 32u : kCap;
            const WalkResult w =
                big ? walk<kWinS, kCap, (kOpt & kOptT4) != 0, OffT>(s_win[0], s_off[0], s_val[0], wpos, pos, vi, seg_end,
                                                                    src_len, value_end, is_signed, err, lane, need, cap,
                                                                    s_pub, s_items, probe_n, kProbeValues)
                    : walk<kWin, kCap, (kOpt & kOptT4) != 0, OffT>(s_win[0], s_off[0], s_val[0], wpos, pos, vi, seg_end,
                                                                   src_len, value_end, is_signed, err, lane, need, cap,
                                                                   s_pub, s_items, probe_n, kProbeValues);
            if (lane == 0) {
              s_ctl[0][0] = w.n;
              s_ctl[0][1] = w.stop;
              s_ctl[0][2] = w.dpos;
              s_ctl[0][3] = w.dval;
              s_ctl[0][4] = w.shrt;
              __hip_atomic_store(s_pub, w.items | kWalkDone, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            PROF_MARK(1);  // wave 0's walk of this pass
#ifdef ORCG_PHASE_PROF
            if (tid == 0) {
              atomicAdd(&g_phase[8], (unsigned long long)w.n);  // runs walked
              atomicAdd(&g_phase[9], 1ull);                     // serial passes
            }
#endif
            __builtin_amdgcn_s_setprio(0);
          }
          bool pf_issued = !kPf;
          for (;;) {
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(s_claim, 1u);
            k = uni(k);
            uint32_t pub;
            // waiting waves back off: polling shares the CU's scalar unit with
            // the walk (a short-run walk publishes an item every ~64 runs)
            for (uint32_t spin = 0;; ++spin) {
              pub = uni(__hip_atomic_load(s_pub, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
              if (k < (pub & ~kWalkDone) || (pub & kWalkDone)) break;
              if (spin < 2) __builtin_amdgcn_s_sleep(2);
              else __builtin_amdgcn_s_sleep(24);
            }
            if constexpr (kPf) {
              if (!pf_issued && (pub & kWalkDone)) {
                // the walk is done: if this pass ends the window, load this
                // thread's share of the next one while the items expand
                pf_issued = true;
                const uint64_t npos = pos + uni(s_ctl[0][2]);
                const uint64_t nvi = vi + uni(s_ctl[0][3]);
                const uint32_t chunk = big ? kChunkS : kChunk;
                if (!uni(s_ctl[0][1]) && npos >= wpos + chunk && npos < seg_end && nvi < value_end) {
                  const uint32_t nwrel = (uint32_t)(npos - bias) & ~15u;
                  const uint64_t end_rel = (seg_end - bias + 15) & ~15ull;
                  const uint32_t nneed = end_rel - nwrel < kWinS ? (uint32_t)(end_rel - nwrel) : kWinS;
#pragma unroll
                  for (int i = 0; i < kPfPer; ++i) {
                    const uint32_t off = (uint32_t)(i * kThreads + tid) * 16u;
                    if (off < nneed)
                      pf[i] = __builtin_bit_cast(pf_u4, __builtin_amdgcn_raw_buffer_load_b128(rs, nwrel + off, 0, 2));
                  }
                  pf_wrel = nwrel;
                  pf_need = nneed;
                }
              }
            }
            if (k >= (pub & ~kWalkDone)) break;  // the walk is done and every item is claimed
            const uint32_t e = uni(s_items[k]);
            const uint32_t r0 = k ? (uni(s_items[k - 1]) & ~(uint32_t)kItemLong) : 0u;
            if (e & kItemLong) {
#ifdef ORCG_DEBUG_COVER
              if (lane == 0) {
                const uint32_t h = uni(s_off[0][r0]);
                ORCG_COVER_ADD(parse_run([&](uint32_t i) { return lds_byte(s_win[0], h + i); }, ~0ull, kHdrLim,
                                         is_signed).L);
              }
#endif
              expand_run<kOpt>(s_win[0], kWinS / 4 + 8, uni(s_off[0][r0]), vi + uni(s_val[0][r0]), is_signed,
                               value_begin, value_end, dst, lane);
            }
            else if (kDense == 2 && (kOpt & kOptD3) != 0 && !big)
              // coalesced stores through the wave's value stage
              dense_expand<kOpt>(s_win[0], kWin / 4 + 8, s_off[0], s_val[0], s_stage2 + wave * kStage, r0, e, vi,
                                 is_signed, value_begin, value_end, dst, lane);
            else
              group_expand<kOpt>(s_win[0], s_off[0], s_val[0], r0, e, vi, is_signed, value_begin, value_end, dst,
                                 lane);
          }
          // the other parity's counters are idle: clear them for the next serial pass
          if (tid == 0) {
            s_sync[sync_par ^ 1][0] = 0;
            s_sync[sync_par ^ 1][1] = 0;
          }
          sync_par ^= 1;
          __syncthreads();
          n = uni(s_ctl[0][0]);
          stop = uni(s_ctl[0][1]);
          dpos = uni(s_ctl[0][2]);
          dval = uni(s_ctl[0][3]);
          shrt = uni(s_ctl[0][4]);
        }
        __syncthreads();  // the run table (and the window) are rewritten next
#ifdef ORCG_DEBUG_COVER
        if (tid == 0 && !stop && *s_cover_ptr() != dval) report(err, vi, was_dense ? 0x71u : 0x70u);
        __syncthreads();
#endif
        PROF_MARK(was_dense ? 6 : 2);
#ifdef ORCG_PHASE_PROF
        if (was_dense) ++wg_dense;
        else ++wg_serial;
#endif
        if constexpr (kTable) {
          // a pass expanded here: slices starting inside it start at the next
          // table entry; then the segment header (read by the second pass)
          const uint64_t vrel = vi - vi0, vend = vrel + dval;
          if (!tabled) {
            const uint64_t S = rtab.slice, ve = vend < tlim ? vend : tlim;
            const uint64_t kb0 = vrel == 0 ? 1u : (vrel + S - 1) / S;
            for (uint64_t kb = kb0 + (uint64_t)tid; kb * S < ve; kb += kThreads) thdr[kRtHdr + kb] = tcnt;
          }
          if (tid == 0) {
            thdr[0] = tcnt;
            thdr[1] = vend < 0xffffffffull ? (uint32_t)vend : 0xffffffffu;
          }
        }
        if (stop) return;
        pos += dpos;
        vi += dval;
        const bool was_probe = probe;
        probe = false;
        if constexpr (kDefer == 1) {
          // a short-run segment: queue the rest for the dense instance
          if (shrt && pos < seg_end && vi < value_end) {
            if (tid == 0) {
              // the segment's own entry, stamped with this launch pair's
              // sequence number (no shared counter: one atomic per queued
              // segment on one word serialised whole launches)
              defer_q[3 * gg + 1] = pos;
              defer_q[3 * gg + 2] = vi;
              __hip_atomic_store(&defer_q[3 * gg], (unsigned long long)defer_par, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
              // the launch-wide "something was queued" word (after the
              // launch's last segment entry): written once per launch pair
              // in the common case (a load first, so a stream whose every
              // segment queues does not serialise on one address)
              unsigned long long* any = &defer_q[3 * p_nsegs];
              if (__hip_atomic_load(any, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (unsigned long long)defer_par)
                __hip_atomic_store(any, (unsigned long long)defer_par, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
          }
        }
        if constexpr (kDense) {
          // hysteresis on the stream bytes per run of this pass
          if (n > 0) {
            const uint32_t bpr = dpos / n;
            if (shrt || (!dense && (n >= 8 || (was_probe && n >= 4)) && bpr < kDenseB)) dense = true;
            else if (dense && bpr >= kSerialB) dense = false;
          }
        }
        if (n == 0 && dpos == 0) break;  // nothing consumed (cannot happen for a good window)
        // a union instance leaves a serial window as soon as its runs turn
        // short: the next window is a dense one
        if (big && dense) break;
      } while (pos < wpos + (big ? kChunkS : kChunk) && pos < seg_end && vi < value_end);
      pwpos = wpos;
      pneed = need;
    }
  } else {
    // prologue: the producer fills and walks window 0
    if (wave == 0) {
      const uint32_t wrel = (uint32_t)(pos - bias) & ~15u;
      fill<kOpt>(s_win[0], rs, wrel, kWin, 0, 1, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const WalkResult w = walk<kWin, kCap>(s_win[0], s_off[0], s_val[0], bias + wrel, pos, vi, seg_end, src_len,
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
      const uint32_t n = uni(s_ctl[b][0]), stop = uni(s_ctl[b][1]);
      const uint64_t next_pos = pos + uni(s_ctl[b][2]), next_vi = vi + uni(s_ctl[b][3]);
      const bool more = !stop && next_pos < seg_end && next_vi < value_end;
      if (wave == 0) {
        if (more) {  // produce window b^1 while the consumers expand window b
          const uint32_t wrel = (uint32_t)(next_pos - bias) & ~15u;
          fill<kOpt>(s_win[b ^ 1], rs, wrel, kWin, 0, 1, lane);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          const WalkResult w = walk<kWin, kCap>(s_win[b ^ 1], s_off[b ^ 1], s_val[b ^ 1], bias + wrel, next_pos,
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
          expand_run<kOpt>(s_win[b], kWin / 4 + 8, uni(s_off[b][k]), vi + uni(s_val[b][k]), is_signed, value_begin,
                           value_end, dst, lane);
      }
      lds_barrier();
      if (stop) return;
      pos = next_pos;
      vi = next_vi;
      if (!more) break;
    }
  }
  if (tid == 0 && v_next != ~0ull && vi < value_end && vi != v_next) report(err, vi, kErrBadSegment);
  if (tid == 0 && v_next == ~0ull && vi < value_end) report(err, vi, kErrBadRead);  // stream ended early
  };

  if constexpr (kDefer == 2) {
    // the drain: one workgroup per launch-wide segment; a segment the serial
    // launch stamped with this pair's sequence number is decoded from its
    // queued byte offset / value index, any other exits after one load (the
    // hardware hands out the queued segments as workgroups free up: the
    // earlier persistent grid of 6 workgroups per CU, each a static share,
    // ran 19 % slower on all-short-run streams)
    // nothing queued by the serial launch (long-run streams): one load, exit
    if (uni64(__hip_atomic_load(&defer_q[3 * p_nsegs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) !=
        (unsigned long long)defer_par)
      return;
    const uint64_t q = blockIdx.x;
    if (q >= p_nsegs || uni64(defer_q[3 * q]) != (unsigned long long)defer_par) return;
    run_segment(q, true, uni64(defer_q[3 * q + 1]), uni64(defer_q[3 * q + 2]));
  } else {
    // (one call site per instance: a second one makes the compiler outline
    // run_segment into a call with a ~700-byte stack frame)
    run_segment(blockIdx.x, false, 0, 0);
  }
#ifdef ORCG_PHASE_PROF
  if (kUnion && tid == 0 && blockIdx.x < kWgDurMax) {
    g_wgdur[2 * blockIdx.x] = wall_clock64() - wg_t0;
    g_wgdur[2 * blockIdx.x + 1] = wg_dense | ((uint64_t)wg_serial << 32);
  }
#endif
}

}  // namespace

// Variants (ctx->rlev2_variant, include/orcg.h): 0 = the density-adaptive
// default; 2-8 pin one instance (the parity tests run each: 6 = the union
// instance in two passes, the default's below 1.25 B/value; 8 = the same in
// one pass); 1 = the wave-walk kernel (rlev2_kernels.hip). (The round 1-5
// tuning instances of the A/B sweeps were removed in round 6.)
bool rlev2_variant_valid(int v) { return v >= 0 && v <= 8; }

static int defer_queue(Ctx* ctx, uint64_t nsegs, unsigned long long** out) {
  // {stamp, byte offset, value index} per launch-wide segment, stamps zeroed
  // at allocation (launch sequence numbers start at 1); word 3 * nsegs is
  // the launch's "something was queued" stamp
  if (ctx->defer_cap < nsegs + 1) {
    if (ctx->d_defer) {
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipFree(ctx->d_defer);
      ctx->d_defer = nullptr;
      ctx->defer_cap = 0;
    }
    const uint64_t cap = std::max<uint64_t>(nsegs + nsegs / 4, 4096);
    int rc = hip_check(ctx, hipMalloc(&ctx->d_defer, 3 * cap * 8), "hipMalloc defer queue");
    if (!rc) rc = hip_check(ctx, hipMemsetAsync(ctx->d_defer, 0, 3 * cap * 8, ctx->stream), "defer queue reset");
    if (rc) return rc;
    ctx->defer_cap = cap;
  }
  *out = (unsigned long long*)ctx->d_defer;
  return ORCG_OK;
}

// The default's instance for a stream, by its stream bytes per value
// (profiles/r03/sweep.md):
//  * >= 5 B/value (wide values, W >= 40): 33 KB windows (4 WG/CU) filled
//    through registers, one walking wave, no queue (writers emit wide random
//    values in long DIRECT runs; the empty queue drain cost 4 us of C2's 290);
//  * 1.25 - 5 B/value: 21 KB serial windows (6 WG/CU), queueing segments whose
//    first runs are short by values for the dense drain (long DIRECT / DELTA /
//    PATCHED_BASE runs of 10-40-bit values: 5.3-6.1 TB/s; short runs of wide
//    values 20 % slower than the union instance, the price of the rule);
//  * < 1.25 B/value (low-cardinality columns, SHORT_REPEAT 0.2-1 B/value): the
//    union instance, which routes each window by its own runs (8.5 KB dense
//    windows with parallel run discovery, 16.75 KB serial windows once a
//    segment's runs are long).
// The dense-capable instances walk long runs 15-20 % slower than the serial
// ones (at 6 WG/CU they carry 56 B/lane of scratch, the serial ones none), so long-run
// streams above 1.25 B/value stay on the serial instance.
static int default_variant(uint64_t src_len, uint64_t est_values) {
  return src_len >= 5 * est_values ? 2 : (4 * src_len >= 5 * est_values ? 3 : 6);
}

static int cu_count(Ctx* ctx) {
  if (ctx->num_cus == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0)
      cus = 256;
    ctx->num_cus = cus;
  }
  return ctx->num_cus;
}

// The union instance runs in two passes (kOptTable + rlev2_expand_kernel)
// when its launch has at most this many segments per CU: a launch of a few
// segments per CU lasts as long as its slowest segments' discovery +
// expansion, and balancing the expansion by values pays (configs[3]'s
// multi-stream launch, 1,336 segments: 297 -> 150 + 86 us; configs[4]'s
// child streams, 264: 93 -> 57 + 20 us); with many more segments than the
// chip holds at once, the one-pass instance's expansion already overlaps
// other workgroups' discovery and the second pass only adds its own latency
// and the run table's traffic (the stream sweep's 10,000-segment launches:
// SHORT_REPEAT 12-bit 2,016 GB/s in one pass, 1,267 in two; profiles/r06/
// sweep_*).
constexpr uint64_t kTwoPassSegsPerCu = 12;
static int union_variant(Ctx* ctx, uint64_t nsegs) {
  return nsegs <= kTwoPassSegsPerCu * (uint64_t)cu_count(ctx) ? 6 : 8;
}

// One launch (or serial + drain pair) of instance `variant` over nsegs
// segments of one stream, or (jobs_d) over the launch-wide segments of a
// device job table.
// ORCG_DEBUG_DEFER: after a serial launch, how many of its segments it
// queued for the dense drain (stderr; synchronises the stream)
static void debug_defer(Ctx* ctx, const unsigned long long* dq, uint64_t nsegs, uint32_t dpar) {
  if (!debug_on("defer")) return;
  std::vector<unsigned long long> h(3 * nsegs + 1);
  if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
      hipMemcpy(h.data(), dq, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return;
  uint64_t q = 0;
  for (uint64_t g = 0; g < nsegs; ++g) q += h[3 * g] == dpar ? 1 : 0;
  fprintf(stderr, "defer: %llu of %llu segments queued (any %d)\n", (unsigned long long)q,
          (unsigned long long)nsegs, h[3 * nsegs] == dpar ? 1 : 0);
}

// Two-pass shape for segments of at most `seg_values` values (a bound: a
// segment that turns out longer has its later passes expanded by the first
// kernel): slices of <= kSliceMax values, a multiple of 256, spg per segment.
static void two_pass_shape(uint64_t seg_values, uint32_t* spg, uint32_t* slice) {
  const uint64_t n = std::max<uint64_t>(seg_values, 1);
  const uint64_t smax = kSliceMax;
  const uint64_t k = std::min<uint64_t>((n + smax - 1) / smax, 256);
  uint64_t s = (n + k - 1) / k;
  s = std::min<uint64_t>((s + 255) & ~255ull, smax);
  *spg = (uint32_t)k;
  *slice = (uint32_t)s;
}

// A segment's value bound for the two-pass shape: its share of the values,
// + 1/8 and one run (row-index segments start up to 511 values early).
static uint64_t seg_value_bound(uint64_t values, uint64_t nsegs) {
  const uint64_t avg = (values + nsegs - 1) / std::max<uint64_t>(nsegs, 1);
  return avg + avg / 8 + 512;
}

// The context's run table (entries) and segment headers (nsegs x (kRtHdr +
// spg) words), grow-only; nothing needs clearing (the first kernel writes
// every segment's header before the second reads it).
static int runtab_buffers(Ctx* ctx, uint64_t entries, uint64_t nsegs, uint32_t spg, uint32_t slice, RunTab* rt) {
  const uint64_t tb = std::max<uint64_t>(entries, 1) * 8, hb = nsegs * (kRtHdr + spg) * 4;
  if (ctx->rtab_cap < tb || ctx->rhdr_cap < hb) {
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->rtab_cap < tb) {
      if (ctx->d_rtab) (void)hipFree(ctx->d_rtab);
      ctx->d_rtab = nullptr;
      ctx->rtab_cap = 0;
      const uint64_t cap = std::max<uint64_t>(tb + tb / 4, 1u << 20);
      int rc = hip_check(ctx, hipMalloc(&ctx->d_rtab, cap), "hipMalloc run table");
      if (rc) return rc;
      ctx->rtab_cap = cap;
    }
    if (ctx->rhdr_cap < hb) {
      if (ctx->d_rhdr) (void)hipFree(ctx->d_rhdr);
      ctx->d_rhdr = nullptr;
      ctx->rhdr_cap = 0;
      const uint64_t cap = std::max<uint64_t>(hb + hb / 4, 256u << 10);
      int rc = hip_check(ctx, hipMalloc(&ctx->d_rhdr, cap), "hipMalloc run-table headers");
      if (rc) return rc;
      ctx->rhdr_cap = cap;
    }
  }
  *rt = RunTab{(uint64_t*)ctx->d_rtab, (uint32_t*)ctx->d_rhdr, spg, slice};
  return ORCG_OK;
}

static int launch_tiled(Ctx* ctx, int variant, const uint8_t* d_src, uint64_t src_len, int is_signed,
                        const uint64_t* d_segtab, uint64_t nsegs, bool positions_mode, uint64_t rows_per_group,
                        uint64_t value_begin, uint64_t nvalues, void* d_dst, int dst_bytes, const RleJob* jobs_d,
                        uint32_t njobs_d, const uint64_t* dcount = nullptr, const MultiLaunch* ml = nullptr) {
  if (nsegs == 0 || nvalues == 0) return ORCG_OK;
  RunTab rtab{nullptr, nullptr, 0, 0};
  if (variant == 6) {
    // the union instance in two passes, when the run table can address the
    // stream (u32 entries and offsets)
    uint64_t entries = 0, bound = 0;
    uint32_t spg = 0, slice = 0;
    if (jobs_d) {
      if (ml && ml->spg) {
        entries = ml->tab_entries;
        spg = ml->spg;
        slice = ml->slice;
      }
    } else if (src_len < 0xffff0000ull && nsegs < 0x7fff0000ull) {
      entries = src_len / 2 + nsegs + 1;
      bound = positions_mode ? rows_per_group + 512 : seg_value_bound(nvalues, nsegs);
      two_pass_shape(bound, &spg, &slice);
    }
    if (spg && entries < 0xffff0000ull && nsegs * spg < 0x7fffffffull) {
      const int rc = runtab_buffers(ctx, entries, nsegs, spg, slice, &rtab);
      if (rc) return rc;
    } else {
      variant = 8;  // one pass
    }
  }
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  if (dst_bytes != 8 && dst_bytes != 4 && dst_bytes != 2)
    return set_error(ctx, ORCG_INVALID_ARGUMENT, "dst_bytes must be 8, 4 or 2");
  const dim3 block(kThreads);
  const int sg = is_signed ? 1 : 0;
  unsigned long long* dq = nullptr;
  uint32_t dpar = 0;
  (void)cu_count(ctx);

#define ORCG_K(T, P, O, WKB, PIPE, ML)                                                               \
  hipLaunchKernelGGL((rlev2_tiled_kernel<T, P, O, WKB, PIPE, MW, DN, DF, ML>), grid, block, 0, ctx->stream,   \
                     d_src, src_len, sg, d_segtab, nsegs, rows_per_group, value_begin, nvalues, (T*)d_dst, \
                     ctx->d_err, dq, dpar, jobs_d, njobs_d, dcount, rtab)
// single-stream instances (+ the multi-stream one for the default's
// instances, ORCG_KX; the tuning variants have none, ORCG_KX1)
#define ORCG_KX1(O, WKB, PIPE, MWV, DNV, DFV, GRIDV)                                 \
  do {                                                                              \
    constexpr int MW = MWV;                                                         \
    constexpr int DN = (int)(DNV);                                                  \
    constexpr int DF = DFV;                                                         \
    const dim3 grid(GRIDV);                                                         \
    if (dst_bytes == 8) {                                                           \
      if (positions_mode) ORCG_K(int64_t, true, O, WKB, PIPE, false);                \
      else ORCG_K(int64_t, false, O, WKB, PIPE, false);                              \
    } else if (dst_bytes == 4) {                                                    \
      if (positions_mode) ORCG_K(int32_t, true, O, WKB, PIPE, false);                \
      else ORCG_K(int32_t, false, O, WKB, PIPE, false);                              \
    } else {                                                                        \
      if (positions_mode) ORCG_K(int16_t, true, O, WKB, PIPE, false);                \
      else ORCG_K(int16_t, false, O, WKB, PIPE, false);                              \
    }                                                                               \
  } while (0)
#define ORCG_KX(O, WKB, PIPE, MWV, DNV, DFV, GRIDV)                                  \
  do {                                                                              \
    constexpr int MW = MWV;                                                         \
    constexpr int DN = (int)(DNV);                                                  \
    constexpr int DF = DFV;                                                         \
    const dim3 grid(GRIDV);                                                         \
    if (jobs_d) {                                                                   \
      ORCG_K(int64_t, false, O, WKB, PIPE, true);                                   \
    } else if (dst_bytes == 8) {                                                    \
      if (positions_mode) ORCG_K(int64_t, true, O, WKB, PIPE, false);                \
      else ORCG_K(int64_t, false, O, WKB, PIPE, false);                              \
    } else if (dst_bytes == 4) {                                                    \
      if (positions_mode) ORCG_K(int32_t, true, O, WKB, PIPE, false);                \
      else ORCG_K(int32_t, false, O, WKB, PIPE, false);                              \
    } else {                                                                        \
      if (positions_mode) ORCG_K(int16_t, true, O, WKB, PIPE, false);                \
      else ORCG_K(int16_t, false, O, WKB, PIPE, false);                              \
    }                                                                               \
  } while (0)
#define ORCG_KT(O, WKB, PIPE, MWV, DNV) ORCG_KX1(O, WKB, PIPE, MWV, DNV, 0, grid_s)

  // the default's instances
  constexpr int kSer = kOptNTStore | kOptReuse | kOptFast | kOptT4;  // serial-walk paths
  constexpr int kWide = kSer | kOptRegFill;
  // a serial instance that queues short-run segments, then the dense
  // instance that drains the queue
#define ORCG_DEFERRING(O, WKB, MWV, DO)                                               \
  do {                                                                              \
    int rc_ = defer_queue(ctx, nsegs, &dq);                                          \
    if (rc_) return rc_;                                                            \
    dpar = (uint32_t)(ctx->defer_seq++ % 0xffffffffull) + 1u; /* never 0 */         \
    ORCG_KX(O, WKB, false, MWV, 0, 1, (unsigned)nsegs);                              \
    debug_defer(ctx, dq, nsegs, dpar);                                                \
    ORCG_KX(DO, 8, false, 6, 2, 2, (unsigned)nsegs);                                 \
  } while (0)

  const unsigned grid_s = (unsigned)nsegs;
  switch (variant) {
    case 2: ORCG_KX(kWide | kOptD3, 33, false, 1, 0, 0, grid_s); break;  // 33 KB register-filled serial, no queue
    case 3: ORCG_DEFERRING(kSer | kOptD3, 21, 6, kSer | kOptD3); break;   // 21 KB serial + dense drain
    case 4: ORCG_KX(kSer | kOptD3, 8, false, 6, 2, 0, grid_s); break;   // dense v3, 8.5 KB
    case 5: ORCG_KX(kSer | kOptD3, 12, false, 5, 2, 0, grid_s); break;  // dense v3, 12.5 KB
    case 6: {
      // union, two passes: dense passes table their runs, rlev2_expand_kernel
      // expands them in value slices
      ORCG_KX(kSer | kOptD3 | kOptUnion | kOptTable, 8, false, 6, 2, 0, grid_s);
      const int rc = hip_check(ctx, hipGetLastError(), "rlev2_tiled_kernel launch");
      if (rc) return rc;
      return launch_rlev2_expand(ctx, d_src, src_len, sg, value_begin, nvalues, d_dst, dst_bytes, dcount, jobs_d,
                                 njobs_d, nsegs, rtab);
    }
    case 7: ORCG_DEFERRING(kWide | kOptD3, 33, 1, kSer | kOptD3); break;  // 33 KB serial + dense drain (round-3 default, A/B)
    case 8: ORCG_KX(kSer | kOptD3 | kOptUnion, 8, false, 6, 2, 0, grid_s); break;  // union in one pass (round-5 default)
    default: return set_error(ctx, ORCG_INVALID_ARGUMENT, "unknown RLEv2 kernel variant");
  }
#undef ORCG_DEFERRING
#undef ORCG_KT
#undef ORCG_KX
#undef ORCG_KX1
#undef ORCG_K
  return hip_check(ctx, hipGetLastError(), "rlev2_tiled_kernel launch");
}

int launch_rlev2_tiled(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                       const uint64_t* d_segtab, uint64_t nsegs, bool positions_mode,
                       uint64_t rows_per_group, uint64_t value_begin, uint64_t nvalues, void* d_dst,
                       int dst_bytes, const uint64_t* d_count) {
  int variant = ctx->rlev2_variant;
  if (variant == 0) {
    const uint64_t est = positions_mode ? nsegs * rows_per_group : nvalues;
    variant = default_variant(src_len, est);
    if (variant == 6) variant = union_variant(ctx, nsegs);
    // more than 8.1 stream bytes a value is more than any 64-bit payload:
    // the excess is run headers, i.e. runs of ~20 values or fewer of wide
    // values (short DIRECT / PATCHED_BASE), whose expansion the two-pass
    // union balances by values at any segment count (sweep short DIRECT
    // 64-bit, 10,000 segments: 217 GB/s in the serial walk, 270 in one union
    // pass, 379 in two; profiles/r06/sweep_shortdirect_64_548c478.jsonl).
    // 512-value W=64 runs (configs[1]) are 8.004 B/value: the serial walk.
    else if (variant == 2 && 10 * src_len > 81 * est) variant = 6;
  }
  return launch_tiled(ctx, variant, d_src, src_len, is_signed, d_segtab, nsegs, positions_mode, rows_per_group,
                      value_begin, nvalues, d_dst, dst_bytes, nullptr, 0, d_count);
}

// Job tables go through a pinned ring mirrored on the device (entries are
// reused only after the stream has drained: a wrap synchronises first), or
// into the caller's arena (Ctx::arena_*), which the caller uploads itself.
int stage_table(Ctx* ctx, const void* src, size_t bytes, const void** out) {
  const uint64_t need = (bytes + 255) & ~(uint64_t)255;
  if (ctx->arena_h) {
    if (ctx->arena_used + need > ctx->arena_cap) return set_error(ctx, ORCG_INVALID_ARGUMENT, "job arena full");
    memcpy(ctx->arena_h + ctx->arena_used, src, bytes);
    *out = ctx->arena_d + ctx->arena_used;
    ctx->arena_used += need;
    return ORCG_OK;
  }
  if (ctx->jobs_cap < need) {
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->d_jobs) (void)hipFree(ctx->d_jobs);
    if (ctx->h_jobs) (void)hipHostFree(ctx->h_jobs);
    ctx->d_jobs = ctx->h_jobs = nullptr;
    ctx->jobs_cap = ctx->jobs_used = 0;
    const uint64_t cap = std::max<uint64_t>(4 * need, 256u << 10);
    int rc = hip_check(ctx, hipMalloc(&ctx->d_jobs, cap), "hipMalloc job table");
    if (!rc) rc = hip_check(ctx, hipHostMalloc(&ctx->h_jobs, cap, hipHostMallocDefault), "hipHostMalloc job table");
    if (rc) return rc;
    ctx->jobs_cap = cap;
  }
  if (ctx->jobs_used + need > ctx->jobs_cap) {
    int rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "job ring wrap");
    if (rc) return rc;
    ctx->jobs_used = 0;
  }
  uint8_t* h = (uint8_t*)ctx->h_jobs + ctx->jobs_used;
  uint8_t* d = (uint8_t*)ctx->d_jobs + ctx->jobs_used;
  memcpy(h, src, bytes);
  ctx->jobs_used += need;
  *out = d;
  return hip_check(ctx, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, ctx->stream), "H2D jobs");
}

bool rlev2_multi_capable(int variant) { return variant == 0 || (variant >= 2 && variant <= 8); }

int plan_rlev2_multi(Ctx* ctx, const RleJob* jobs, uint32_t njobs, std::vector<MultiLaunch>& out) {
  const int pinned = ctx->rlev2_variant;
  if (!rlev2_multi_capable(pinned)) {
    // not a multi-stream instance: one launch per stream (the reader queues
    // only segment-table jobs for these variants, rlev2_multi_capable)
    for (uint32_t j = 0; j < njobs; ++j) {
      if (!jobs[j].segtab) return set_error(ctx, ORCG_INVALID_ARGUMENT, "row-index job needs a multi-stream instance");
      out.push_back(MultiLaunch{3, pinned, jobs + j, 1, jobs[j].nsegs, jobs[j].nvalues});
    }
    return ORCG_OK;
  }
  // one launch per instance: group the streams by the instance they get
  std::vector<RleJob> group[9];
  for (uint32_t j = 0; j < njobs; ++j) {
    const RleJob& J = jobs[j];
    if (J.nsegs == 0 || J.nvalues == 0) continue;
    group[pinned ? pinned : default_variant(J.src_len, J.nvalues)].push_back(J);
  }
  if (debug_on("jobs"))
    for (int v = 2; v <= 8; ++v)
      for (const RleJob& J : group[v])
        fprintf(stderr, "rle job: instance %d bytes %llu values %llu segments %llu (%.3f B/value)\n", v,
                (unsigned long long)J.src_len, (unsigned long long)J.nvalues, (unsigned long long)J.nsegs,
                (double)J.src_len / (double)J.nvalues);
  for (int v = 2; v <= 8; ++v) {
    std::vector<RleJob>& g = group[v];
    if (g.empty()) continue;
    // workgroups start in index order: the streams with the most stream
    // bytes per value (the most runs per segment, the slowest segments) first,
    // so the launch does not end on a tail of slow segments
    std::stable_sort(g.begin(), g.end(), [](const RleJob& a, const RleJob& b) {
      return (double)a.src_len * (double)b.nvalues > (double)b.src_len * (double)a.nvalues;
    });
    uint64_t segs = 0, values = 0, entries = 0, bound = 0;
    for (RleJob& J : g) {
      J.seg_base = segs;
      segs += J.nsegs;
      values += J.nvalues;
      // two-pass (the union instance): the job's run-table range
      J.tab_base = (uint32_t)std::min<uint64_t>(entries, 0xffffffffull);
      entries += J.src_len / 2 + J.nsegs + 1;
      bound = std::max(bound, seg_value_bound(J.nvalues, J.nsegs));
    }
    if (segs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
    const RleJob* d = nullptr;
    const int rc = stage_rle_jobs(ctx, g.data(), (uint32_t)g.size(), &d);
    if (rc) return rc;
    const int lv = (v == 6 && !pinned) ? union_variant(ctx, segs) : v;
    MultiLaunch m{0, lv, d, (uint32_t)g.size(), segs, values};
    if (lv == 6 && entries < 0xffff0000ull) {
      m.tab_entries = entries;
      two_pass_shape(bound, &m.spg, &m.slice);
    }
    out.push_back(m);
  }
  return ORCG_OK;
}

// The planned launches, in order. The work before the join runs side by
// side: the critical RLEv2 instance (the two-pass one, else the one with the
// most values) on this stream, every other instance on a side lane of its
// own, and the varint tile counts and RLEv1 segments (kinds 4, 1) on one
// more lane; then this stream waits for the lanes and runs what reads their
// outputs (dictionaries, decimals, length scans: kinds 2, 5, 6) itself. The
// critical path never changes queues: a dependency across HIP queues costs
// 12-30 us a hop on the MI355X (configs[3] timelines), so the lanes, done
// long before the critical instance, are the ones waited on, and the
// post-join kernels follow the critical instance on its own queue.
int run_multi(Ctx* ctx, const std::vector<MultiLaunch>& ls) {
  int ninst = 0, crit = -1;
  bool aux = false;
  for (size_t i = 0; i < ls.size(); ++i) {
    const MultiLaunch& m = ls[i];
    if (m.kind == 1 || m.kind == 4) aux = true;
    if (m.kind != 0) continue;
    ++ninst;
    const bool two = m.spg > 0, ctwo = crit >= 0 && ls[crit].spg > 0;
    if (crit < 0 || (two && !ctwo) || (two == ctwo && m.values > ls[crit].values)) crit = (int)i;
  }
  const int nlanes = (ninst > 0 ? ninst - 1 : 0) + (aux && ninst > 0 ? 1 : 0);
  const bool par = nlanes > 0 && side_lanes() > 1 && (size_t)nlanes <= side_lanes() &&
                   ctx_lane(ctx, (size_t)nlanes - 1) != nullptr;
  Ctx* const base = ctx;
  int used = 0, aux_lane = -1, rc = ORCG_OK;
  if (par) rc = hip_check(ctx, hipEventRecord(ctx->ev_fork, ctx->stream), "fork event");
  auto fork = [&](Ctx** c) -> int {  // the next lane, started after the fork point
    *c = base->lanes[used++];
    return hip_check(base, hipStreamWaitEvent((*c)->stream, base->ev_fork, 0), "fork wait");
  };
  bool joined = false;
  auto join = [&]() -> int {
    int r = ORCG_OK;
    for (int k = 0; k < used; ++k) {
      int jr = hip_check(base, hipEventRecord(base->ev_join[k], base->lanes[k]->stream), "join event");
      if (!jr) jr = hip_check(base, hipStreamWaitEvent(base->stream, base->ev_join[k], 0), "join wait");
      if (jr && !r) r = jr;
    }
    joined = true;
    return r;
  };
  for (size_t i = 0; i < ls.size() && !rc; ++i) {
    const MultiLaunch& m = ls[i];
    if ((m.kind == 2 || m.kind == 5 || m.kind == 6) && !joined && (rc = join())) break;
    debug_stale("run_multi: before a launch");
    if (m.kind == 0) {
      Ctx* c = base;
      if (par && (int)i != crit && (rc = fork(&c))) break;
      // jobs without a record of their own report into the base's (the
      // lane's own record is the lane's: it frees it)
      unsigned long long* const own = c->d_err;
      c->d_err = base->d_err;
      rc = launch_tiled(c, m.variant, nullptr, 0, 0, nullptr, m.grid, false, 0, 0, m.values, nullptr, 8,
                        (const RleJob*)m.d_jobs, m.njobs, nullptr, &m);
      c->d_err = own;
      if (rc) {
        char b[160];
        snprintf(b, sizeof b, " (instance %d, %u streams, %llu segments%s)", m.variant, m.njobs,
                 (unsigned long long)m.grid, c == base ? "" : ", side lane");
        base->last_error = c->last_error + b;
      }
    } else if (m.kind == 1 || m.kind == 4) {
      Ctx* c = base;
      if (par && !joined) {
        if (aux_lane < 0) {
          if ((rc = fork(&c))) break;
          aux_lane = used - 1;
        }
        c = base->lanes[aux_lane];
      }
      unsigned long long* const own = c->d_err;
      c->d_err = base->d_err;
      if (m.kind == 1) {
        rc = launch_rlev1_jobs(c, (const V1SegDesc*)m.d_jobs, m.grid, m.variant);
      } else {
        const VarintJob& J = *(const VarintJob*)m.d_jobs;
        uint64_t ntiles = 0;
        rc = launch_varint_tile_counts(c, J.src, J.len, J.counts, &ntiles);
        if (!rc) rc = launch_exclusive_scan(c, J.counts, ntiles, J.base, nullptr, J.total);
      }
      c->d_err = own;
      if (rc && c != base) base->last_error = c->last_error;
    } else if (m.kind == 2) {
      rc = launch_dict_jobs(base, (const DictJob*)m.d_jobs, m.njobs, m.grid);
    } else if (m.kind == 5) {
      rc = launch_decimal_jobs(base, (const DecJob*)m.d_jobs, m.njobs, m.grid, m.variant);
    } else if (m.kind == 6) {
      const ScanJob& J = *(const ScanJob*)m.d_jobs;
      rc = launch_exclusive_scan(base, J.in, J.n, J.out, J.flags, J.total);
    } else {
      // a pinned single-stream variant: host job (d_jobs is a host pointer)
      const RleJob& J = *(const RleJob*)m.d_jobs;
      unsigned long long* const saved = base->d_err;  // the job's own error record
      if (J.err) base->d_err = J.err;
      rc = launch_rlev2(base, J.src, J.src_len, (int)J.is_signed, J.segtab, J.nsegs, false, 0, 0, J.nvalues, J.dst, 8);
      base->d_err = saved;
    }
  }
  if (!joined) {  // join what was forked (also after a failure)
    const int jr = join();
    if (jr && !rc) rc = jr;
  }
  return rc;
}

int launch_rlev2_multi(Ctx* ctx, const RleJob* jobs, uint32_t njobs) {
  std::vector<MultiLaunch> ls;
  const int rc = plan_rlev2_multi(ctx, jobs, njobs, ls);
  return rc ? rc : run_multi(ctx, ls);
}

}  // namespace orcg

#ifdef ORCG_PHASE_PROF
extern "C" int orcg_debug_wg_durations(unsigned long long* out, int n) {
  if (n > (int)(2 * orcg::kWgDurMax)) n = 2 * orcg::kWgDurMax;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(orcg::g_wgdur), (size_t)n * 8) == hipSuccess ? 0 : -1;
}

extern "C" int orcg_debug_phase_counters(unsigned long long* out, int n, int reset) {
  unsigned long long h[16];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(orcg::g_phase), sizeof(h)) != hipSuccess) return -1;
  for (int i = 0; i < n && i < 16; ++i) out[i] = h[i];
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(orcg::g_phase), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// A no-op launch that makes HIP load this file's code object (warm_modules).
namespace orcg {
namespace {
__global__ void warm_rlev2_tiled_kernel() {}
}  // namespace
void warm_rlev2_tiled(hipStream_t s) { hipLaunchKernelGGL(warm_rlev2_tiled_kernel, dim3(1), dim3(64), 0, s); }
}  // namespace orcg
