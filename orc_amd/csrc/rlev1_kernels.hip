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
// One 256-thread workgroup per segment (header-aligned byte offset + first
// value index: a host plan, or the ROW_INDEX positions). The segment streams
// through an LDS window; nothing about a window is walked serially except one
// lane's hop over at most 32 block entries (rlev1_kernel below). Round 4's
// kernel was one wavefront walking every header and 64-byte literal slice
// through global loads: 52 us per 5,000-value stream of configs[0].
#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

constexpr int kV1Threads = 256;
constexpr uint32_t kV1Tail = 1536;  // >= the longest group of <= 10-byte varints (1 + 128 * 10)
constexpr uint32_t kNone = 0xffffu;
constexpr uint32_t kLaneRun = 32;  // runs up to this many values expand on one lane

typedef uint32_t v1u4 __attribute__((ext_vector_type(4)));

// Phase profiling (build with -DORCG_PHASE_PROF; scripts/ab_rlev1.py
// --phases): thread 0 of every workgroup adds the wall-clock ticks between
// consecutive marks to g_v1phase[k].
#ifdef ORCG_PHASE_PROF
__device__ unsigned long long g_v1phase[10];
#define V1PROF_MARK(k)                                                       \
  do {                                                                       \
    if (threadIdx.x == 0) {                                                  \
      const uint64_t now_ = wall_clock64();                                  \
      atomicAdd(&g_v1phase[k], (unsigned long long)(now_ - prof_last_));     \
      prof_last_ = now_;                                                     \
    }                                                                        \
  } while (0)
#else
#define V1PROF_MARK(k) \
  do {                 \
  } while (0)
#endif

// Window geometry for kCB bytes per thread: groups starting in the first
// kChunk bytes of a window are decoded by it; kBlock = 8 chunks is the hop
// granularity of the chain walk (32 blocks per window either way).
template <int kCB>
struct V1Geo {
  static constexpr uint32_t kChunk = kV1Threads * kCB;
  static constexpr uint32_t kWin = kChunk + kV1Tail;
  static constexpr uint32_t kWords = kWin / 32;  // terminator bitmap dwords
  static constexpr uint32_t kBlock = 8 * kCB;
  static constexpr uint32_t kBlocks = kChunk / kBlock;
  static constexpr uint32_t kMaxGroups = kChunk / 2;  // a group is >= 2 bytes
  static constexpr uint32_t kMaxRuns = kChunk / 3 + 1;  // a run is >= 3 bytes
  static constexpr uint32_t kTailChunks = kV1Tail / kCB;
  static constexpr int kPasses = 1 + (int)((kTailChunks + kV1Threads - 1) / kV1Threads);
  static_assert(kWin % 32 == 0 && kWords <= 2 * kV1Threads, "bitmap words");
};

// byte e (static) of kCB bytes held as kCB / 4 dwords
template <int kCB>
__device__ __forceinline__ uint32_t cbyte(const uint32_t (&w)[kCB / 4], int e) {
  return (w[e >> 2] >> ((e & 3) * 8)) & 0xffu;
}

// A load the compiler must not sink under the branch that uses its value
// (the hops' loads of one round issue together instead of one per branch).
__device__ __forceinline__ uint32_t pinned_u16(const uint16_t* p) {
  uint32_t v = *p;
  asm volatile("" : "+v"(v));
  return v;
}

// Values of a group: h + 3 for a run, -h for a literal (readHeader, :180-191).
__device__ __forceinline__ uint32_t group_values(uint32_t hb) {
  const int32_t h = (int32_t)(int8_t)hb;
  return h >= 0 ? (uint32_t)h + 3u : (uint32_t)(-h);
}

template <typename T>
__device__ __forceinline__ void put_v(T* dst, uint64_t o, uint64_t begin, uint64_t end, uint64_t v) {
  if (o >= begin && o < end) dst[o - begin] = (T)(int64_t)v;
}

// A wave-uniform varint read byte by byte through the descriptor (the rare
// path: a group longer than a whole window, i.e. varints past 10 bytes).
__device__ __forceinline__ bool slow_varint(__amdgpu_buffer_rsrc_t rs, uint64_t bias, uint64_t& pos, uint64_t src_len,
                                            uint64_t& out) {
  uint64_t r = 0;
  uint32_t sh = 0;
  for (;;) {
    if (pos >= src_len) return false;
    const uint32_t rel = (uint32_t)(pos - bias);
    const uint32_t b = (__builtin_amdgcn_raw_buffer_load_b32(rs, rel & ~3u, 0, 0) >> ((rel & 3u) * 8)) & 0xffu;
    ++pos;
    if (sh < 64) r |= (uint64_t)(b & 0x7fu) << sh;
    sh += 7;
    if (b < 0x80u) break;
  }
  out = r;
  return true;
}

// The segment of launch-wide index gg: its stream and segment bounds.
struct V1Seg {
  const uint8_t* src;
  uint64_t src_len;
  int is_signed;
  void* dst;
  unsigned long long* err;
  uint64_t begin, end;  // output value range
  uint64_t seg_start, vi, seg_end, v_next;
};

// segtab: {byte offset, first value index} per segment, or (jobs) the job's
// table / row-index triplets, as rlev2_tiled_kernel's multi-stream instances
// read them (value index = rows[g] - skip, clamped at 0, rg_segtab_kernel).
__device__ __forceinline__ void seg_bounds(const uint64_t* segtab, const int64_t* trip, const int64_t* rows,
                                           uint64_t nsegs, uint64_t g, uint64_t src_len, V1Seg& s) {
  auto at = [&](uint64_t k, uint64_t* off) -> uint64_t {
    if (trip) {
      const int64_t v = rows[k] - trip[3 * k + 1];
      *off = (uint64_t)trip[3 * k];
      return v < 0 ? 0ull : (uint64_t)v;
    }
    *off = segtab[2 * k];
    return segtab[2 * k + 1];
  };
  s.vi = at(g, &s.seg_start);
  s.seg_end = src_len;
  s.v_next = ~0ull;
  if (g + 1 < nsegs) s.v_next = at(g + 1, &s.seg_end);
  if (s.seg_end > src_len) s.seg_end = src_len;
}

// One workgroup per segment; kCB bytes per thread (16: 4 KB windows for
// long segments, e.g. a row group; 4: 1 KB windows for the short segments of
// small streams, whose latency is set by each thread's serial share of the
// window). Per window (kWin bytes of the segment in LDS; every group starting
// in its first kChunk bytes is whole in it unless a varint runs past 10
// bytes):
//   1. a terminator bitmap (bytes < 0x80), its per-dword ranks and the list
//      of terminator positions: the k-th varint end at or after byte x is
//      tpos[rank(x) + k - 1], so every byte knows where a group starting there
//      would end (a run: the end of its base varint at x + 2; a literal of k
//      varints: the k-th terminator after x + 1) in O(1);
//   2. chunk exits (thread t owns bytes [kCB t, kCB t + kCB)): the first group
//      start at or past the chunk's end if a group started at each byte, by a
//      backward pass in registers; block exits (8 chunks) by <= 7 hop rounds;
//   3. one lane hops the true chain block by block (<= 32 LDS reads) and
//      records each block's first group; every thread hops to its own chunk
//      and walks its groups; a workgroup scan gives each group its first
//      value; the owners of run headers decode their bases into a run table;
//   4. literal values: each thread streams the varints ending in its chunk
//      out of registers (a varint begun earlier resumed from the 16 bytes
//      before), consecutive values on consecutive chunks;
//   5. runs: up to kLaneRun values one lane per run (consecutive runs on
//      consecutive lanes: a column of short runs, e.g. 500 runs of 10, costs
//      a few store rounds instead of one wave round per run), longer ones one
//      wave per run, base + j * delta on lane j (their indices listed while
//      the run table is written).
// Errors keep the serial decoder's order: a group truncated by the stream's
// end reports at its first value it cannot produce (the reference throws
// from readByte when that value is requested), with atomicMin on the record.
template <typename T, bool kMulti, int kCB>
__global__ __launch_bounds__(kV1Threads) void rlev1_kernel(const uint8_t* __restrict__ p_src, uint64_t p_src_len,
                                                           int p_is_signed, const uint64_t* __restrict__ p_segtab,
                                                           uint64_t p_nsegs, uint64_t value_begin, uint64_t nvalues,
                                                           T* __restrict__ p_dst, unsigned long long* p_err,
                                                           const V1SegDesc* __restrict__ descs) {
  using G = V1Geo<kCB>;
  constexpr uint32_t kChunk = G::kChunk, kWin = G::kWin, kWords = G::kWords, kBlock = G::kBlock;
  constexpr uint32_t kBlocks = G::kBlocks;
  constexpr int kNW = kCB / 4;  // dwords per chunk
  // 16 bytes of slack before the window (a chunk's prologue reads the 16
  // bytes before it) and after it
  __shared__ __attribute__((aligned(16))) uint32_t s_winbuf[4 + kWin / 4 + 4];
  __shared__ uint32_t s_bits[kWords];
  __shared__ uint32_t s_pre[kWords + 1];
  __shared__ __attribute__((aligned(16))) uint16_t s_tpos[kWin];  // then (step 3b) the runs' metadata
  // chunk exits and block exits (steps 2-3), then (step 3b) the runs' bases
  __shared__ __attribute__((aligned(16))) uint16_t s_exit[2 * kChunk];
  __shared__ uint16_t s_bentry[kBlocks + 1];
  // the window's groups: header position; first value | first varint's rank
  // << 24 | header byte << 40
  __shared__ uint16_t s_gpos[G::kMaxGroups + 1];
  __shared__ uint64_t s_gmeta[G::kMaxGroups + 1];
  __shared__ uint32_t s_wsum[3][kV1Threads / kWave];
  // [0] next window start, [1] incomplete group + 1, [2] stop, [3] long runs
  __shared__ uint32_t s_ctl[4];
  __shared__ uint16_t s_rlong[G::kMaxRuns];  // the window's runs of more than kLaneRun values
  static_assert(G::kMaxRuns * 8 <= kWin * 2 && G::kMaxRuns * 8 <= 4 * kChunk, "run tables");
  uint32_t* const s_win = s_winbuf + 4;
  uint16_t* s_exit2 = s_exit + kChunk;
  const uint8_t* s_bytes = (const uint8_t*)s_win;
  uint64_t* const s_rmeta = (uint64_t*)s_tpos;
  uint64_t* const s_rbase = (uint64_t*)s_exit;

#ifdef ORCG_PHASE_PROF
  uint64_t prof_last_ = wall_clock64();
  const uint64_t prof_t0_ = prof_last_;
#endif
  const int tid = (int)threadIdx.x;
  const int lane = tid % kWave, wave = tid / kWave;

  // the segment and its stream
  V1Seg S;
  {
    const uint64_t gg = blockIdx.x;
    if constexpr (kMulti) {
      const V1SegDesc* J = descs + gg;
      S.src = (const uint8_t*)uni64((uint64_t)(uintptr_t)J->src);
      S.src_len = uni64(J->src_len);
      S.is_signed = (int)uni(J->is_signed);
      S.dst = (void*)uni64((uint64_t)(uintptr_t)J->dst);
      const uint64_t je = uni64((uint64_t)(uintptr_t)J->err);
      S.err = je ? (unsigned long long*)(uintptr_t)je : p_err;
      S.begin = 0;
      S.end = uni64(J->nvalues);
      S.seg_start = uni64(J->seg_start);
      S.vi = uni64(J->vi);
      S.seg_end = uni64(J->seg_end);
      S.v_next = uni64(J->v_next);
      if (S.seg_end > S.src_len) S.seg_end = S.src_len;
    } else {
      S.src = p_src;
      S.src_len = p_src_len;
      S.is_signed = p_is_signed;
      S.dst = p_dst;
      S.err = p_err;
      S.begin = value_begin;
      S.end = value_begin + nvalues;
      seg_bounds(p_segtab, nullptr, nullptr, p_nsegs, gg, p_src_len, S);
    }
  }
  T* const dst = (T*)S.dst;
  const uint64_t vend = S.end;
  uint64_t vi = S.vi;
  if (vi >= vend || S.v_next <= S.begin || S.seg_start >= S.seg_end) {
    // (an empty segment still checks its value index)
    if (tid == 0 && S.seg_start >= S.seg_end && vi < vend && S.v_next != ~0ull && vi != S.v_next && S.v_next > S.begin)
      report(S.err, vi, kErrBadSegment);
    if (tid == 0 && S.seg_start >= S.seg_end && S.v_next == ~0ull && vi < vend) report(S.err, vi, kErrV1BadRead);
    return;
  }

  // range-checked descriptor over [seg_start & ~15, end of stream): loads
  // past the stream return zeros
  const uintptr_t base_abs = ((uintptr_t)S.src + S.seg_start) & ~(uintptr_t)15;
  const uintptr_t end_abs = ((uintptr_t)S.src + S.src_len + 3) & ~(uintptr_t)3;
  const uint64_t span = (uint64_t)(end_abs - base_abs);
  const uint32_t nrec = span > 0xfffff000ull ? 0xfffff000u : (uint32_t)span;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base_abs, (short)0, (int)nrec, 0x00020000);
  const uint64_t bias = (uint64_t)(base_abs - (uintptr_t)S.src);
  const int sg = S.is_signed;

  V1PROF_MARK(0);
  uint64_t pos = S.seg_start;
  bool stopped = false;
  const uint32_t cs = (uint32_t)tid * kCB;  // my chunk
  while (pos < S.seg_end && vi < vend) {
    const uint32_t wrel = (uint32_t)(pos - bias) & ~15u;
    const uint64_t wpos = bias + wrel;  // stream offset of window byte 0
    for (uint32_t off = (uint32_t)tid * 16u; off < kWin; off += kV1Threads * 16u)
      *(v1u4*)((char*)s_win + off) = __builtin_bit_cast(v1u4, __builtin_amdgcn_raw_buffer_load_b128(rs, wrel + off, 0, 0));
    if (tid <= (int)kBlocks) s_bentry[tid] = (uint16_t)kNone;
    if (tid < 4) s_ctl[tid] = tid == 0 ? kNone : 0u;
    const uint32_t p0 = (uint32_t)(pos - wpos);  // < 16
    const uint64_t seg_left = S.seg_end - wpos, src_left = S.src_len - wpos;
    const uint32_t lim = seg_left < kChunk ? (uint32_t)seg_left : kChunk;  // groups starting below lim
    const uint32_t valid = src_left < kWin ? (uint32_t)src_left : kWin;    // stream bytes in the window
    const bool at_end = src_left <= kWin;                                  // the window holds the stream's end
    __syncthreads();
    V1PROF_MARK(1);

    // 1. terminator bitmap (thread t < kWords: bytes [32t, 32t + 32)) and ranks
    uint32_t bits = 0;
    if (tid < (int)kWords) {
      const v1u4 a = *(const v1u4*)(s_win + 8 * tid), b = *(const v1u4*)(s_win + 8 * tid + 4);
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t t = ~w[k] & 0x80808080u;  // bit 7 of each terminator byte
        bits |= (((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u)) << (4 * k);
      }
      const uint32_t b0 = 32u * (uint32_t)tid;
      if (b0 + 32u > valid) bits &= valid > b0 ? ((1u << (valid - b0)) - 1u) : 0u;
      s_bits[tid] = bits;
    }
    const uint32_t cnt = (uint32_t)__builtin_popcount(bits);
    const uint32_t cnt_inc = wave_scan_u32(cnt);
    if (lane == kWave - 1) s_wsum[0][wave] = cnt_inc;
    __syncthreads();
    uint32_t tbase = cnt_inc - cnt, T_total = 0;
#pragma unroll
    for (int w = 0; w < kV1Threads / kWave; ++w) {
      tbase += w < wave ? s_wsum[0][w] : 0u;
      T_total += s_wsum[0][w];
    }
    if (tid < (int)kWords) {
      s_pre[tid] = tbase;
      uint32_t m = bits, r = tbase;
      while (m) {
        s_tpos[r++] = (uint16_t)(32u * (uint32_t)tid + (uint32_t)__builtin_ctz(m));
        m &= m - 1u;
      }
    }
    if (tid == 0) s_pre[kWords] = T_total;
    __syncthreads();
    V1PROF_MARK(2);

    // 2. where a group starting at each of my bytes would end (kNone: not in
    // the window) and its first varint's rank, then chunk exits, backward.
    // Every array index is static (the arrays stay in registers).
    uint32_t mine[kNW];
#pragma unroll
    for (int k = 0; k < kNW; ++k) mine[k] = s_win[cs / 4 + k];
    const uint32_t dc = cs >> 5;  // bytes cs .. cs + kCB + 1 lie in bitmap dwords dc, dc + 1
    const uint32_t pre0 = s_pre[dc], pre1 = s_pre[dc + 1], bits0 = s_bits[dc], bits1 = s_bits[dc + 1];
    auto rank_near = [&](uint32_t x) -> uint32_t {  // x in [cs, cs + 32)
      const bool hi = (x >> 5) != dc;
      const uint32_t m = (1u << (x & 31u)) - 1u;
      return hi ? pre1 + (uint32_t)__builtin_popcount(bits1 & m) : pre0 + (uint32_t)__builtin_popcount(bits0 & m);
    };
    uint32_t endv[kCB], exv[kCB], rk[kCB];
#pragma unroll
    for (int e = 0; e < kCB; ++e) {
      const uint32_t x = cs + (uint32_t)e;
      const uint32_t hb = cbyte<kCB>(mine, e);
      const bool run = hb < 0x80u;
      const uint32_t r = rank_near(run ? x + 2 : x + 1);
      const uint32_t ri = r + (run ? 0u : 256u - hb - 1u);
      const uint32_t t = pinned_u16(s_tpos + (ri < kWin ? ri : 0u));
      rk[e] = r;
      endv[e] = ri < T_total ? t + 1u : kNone;
    }
#pragma unroll
    for (int e = kCB - 1; e >= 0; --e) {
      uint32_t ex = endv[e];
#pragma unroll
      for (int j = e + 1; j < kCB; ++j) ex = endv[e] == cs + (uint32_t)j ? exv[j] : ex;
      exv[e] = ex;
    }
#pragma unroll
    for (int k = 0; k < kCB / 2; ++k) ((uint32_t*)s_exit)[cs / 2 + k] = exv[2 * k] | (exv[2 * k + 1] << 16);
    __syncthreads();

    // 2b. block exits: hop chunk exits to my block's end (every round's loads
    // issue together)
    {
      const uint32_t be = (cs | (kBlock - 1)) + 1;
      uint32_t q[kCB];
#pragma unroll
      for (int e = 0; e < kCB; ++e) q[e] = exv[e];
#pragma unroll
      for (int hh = 0; hh < 7; ++hh) {
#pragma unroll
        for (int e = 0; e < kCB; ++e) {
          const uint32_t nq = pinned_u16(s_exit + (q[e] < be ? q[e] : 0u));
          q[e] = q[e] < be ? nq : q[e];
        }
      }
#pragma unroll
      for (int k = 0; k < kCB / 2; ++k) ((uint32_t*)s_exit2)[cs / 2 + k] = q[2 * k] | (q[2 * k + 1] << 16);
    }
    __syncthreads();
    V1PROF_MARK(3);

    // 3. the chain, block by block (one lane)
    if (tid == 0) {
      for (uint32_t p = p0; p < lim; p = s_exit2[p]) s_bentry[p / kBlock] = (uint16_t)p;
    }
    __syncthreads();
    V1PROF_MARK(4);

    // 3b. my chunk's groups (a static walk over my bytes): count, values,
    // runs; the group crossing lim sets the next window; a group whose end is
    // not in the window stops the chain. Also each of my chunks' rank and the
    // terminator before it (the literal decode's prologue), while s_tpos is
    // alive.
    uint32_t first = kNone;
    if (cs < lim) {
      uint32_t p = s_bentry[cs / kBlock];
      if (p != kNone) {
        while (p < cs) p = s_exit[p];
        if (p < cs + kCB && p < lim) first = p;
      }
    }
    uint32_t rcv[G::kPasses], prv[G::kPasses];
#pragma unroll
    for (int ps = 0; ps < G::kPasses; ++ps) {
      const uint32_t c0 = ps == 0 ? cs : kChunk + (uint32_t)(ps - 1) * kV1Threads * kCB + cs;
      rcv[ps] = 0;
      prv[ps] = kNone;
      if (c0 < kWin) {
        const uint32_t r = s_pre[c0 >> 5] + (uint32_t)__builtin_popcount(s_bits[c0 >> 5] & ((1u << (c0 & 31u)) - 1u));
        rcv[ps] = r;
        prv[ps] = r ? (uint32_t)s_tpos[r - 1] : kNone;
      }
    }
    uint32_t ng = 0, nv = 0, nr = 0, gmask = 0;
    uint32_t inc_at = kNone, inc_v = 0, inc_avail = 0;  // an incomplete group: position, values before it, values it has
    {
      uint32_t q = first;
#pragma unroll
      for (int e = 0; e < kCB; ++e) {
        if (q == cs + (uint32_t)e && q < lim) {
          const uint32_t hb = cbyte<kCB>(mine, e);
          if (endv[e] == kNone) {
            inc_at = q;
            inc_v = nv;
            if (at_end && hb >= 0x80u) {
              // a literal cut by the stream's end: its whole varints decode
              inc_avail = T_total > rk[e] ? T_total - rk[e] : 0u;
              if (inc_avail) {
                ++ng;
                nv += inc_avail;
                gmask |= 1u << e;
              }
            }
            s_ctl[1] = q + 1;
            q = kNone - 1;  // stop (never a chunk byte, below kNone)
          } else {
            ++ng;
            nv += group_values(hb);
            nr += hb < 0x80u ? 1u : 0u;
            gmask |= 1u << e;
            q = endv[e];
          }
        }
      }
      if (first != kNone && inc_at == kNone && q >= lim) s_ctl[0] = q;  // the next window starts here
    }
    // workgroup scan of (groups, values, runs)
    const uint32_t ng_inc = wave_scan_u32(ng), nv_inc = wave_scan_u32(nv), nr_inc = wave_scan_u32(nr);
    if (lane == kWave - 1) {
      s_wsum[0][wave] = ng_inc;
      s_wsum[1][wave] = nv_inc;
      s_wsum[2][wave] = nr_inc;
    }
    __syncthreads();
    uint32_t ng_base = ng_inc - ng, nv_base = nv_inc - nv, nr_base = nr_inc - nr, NG = 0, NV = 0, NR = 0;
#pragma unroll
    for (int w = 0; w < kV1Threads / kWave; ++w) {
      const uint32_t a = s_wsum[0][w], b = s_wsum[1][w], c = s_wsum[2][w];
      ng_base += w < wave ? a : 0u;
      nv_base += w < wave ? b : 0u;
      nr_base += w < wave ? c : 0u;
      NG += a;
      NV += b;
      NR += c;
    }
    const uint32_t inc_pos1 = s_ctl[1];
    const uint32_t np = s_ctl[0];
    // the bytes the window's groups cover: [p0, stop_at)
    const uint32_t stop_at = inc_pos1 ? (at_end ? valid : inc_pos1 - 1) : (np < valid ? np : valid);
    V1PROF_MARK(5);
    // the group table and the run table (first value | length | delta, base),
    // written by the thread that owns the header (s_tpos and s_exit are dead)
    {
      uint32_t k = ng_base, d = nv_base, rr = nr_base;
#pragma unroll
      for (int e = 0; e < kCB; ++e) {
        if ((gmask >> e) & 1u) {
          const uint32_t x = cs + (uint32_t)e;
          const uint32_t hb = cbyte<kCB>(mine, e);
          s_gpos[k] = (uint16_t)x;
          s_gmeta[k] = (uint64_t)d | ((uint64_t)rk[e] << 24) | ((uint64_t)hb << 40);
          const uint32_t gv = x == inc_at ? inc_avail : group_values(hb);
          // a group running past the segment (segment table not group aligned)
          if (endv[e] != kNone && (uint64_t)endv[e] > seg_left && vi + d < vend) {
            report(S.err, vi + d + gv, kErrBadSegment);
            s_ctl[2] = 1;
          }
          if (hb < 0x80u) {
            // the run's delta byte and base varint
            const uint64_t delta = (uint64_t)(int64_t)(int8_t)s_bytes[x + 1];
            uint64_t acc = 0;
            uint32_t sh = 0;
            for (uint32_t bb = x + 2; bb < endv[e]; ++bb, sh += 7)
              if (sh < 64) acc |= (uint64_t)(s_bytes[bb] & 0x7fu) << sh;
            s_rbase[rr] = sg ? unzigzag(acc) : acc;
            s_rmeta[rr] = (uint64_t)d | ((uint64_t)(hb + 3u) << 32) | ((delta & 0xffu) << 48);
            if (hb + 3u > kLaneRun) s_rlong[atomicAdd(&s_ctl[3], 1u)] = (uint16_t)rr;
            ++rr;
          }
          ++k;
          d += gv;
        }
      }
    }
    if (inc_at != kNone && at_end) {
      // the stream ends inside this group: its first value it cannot produce
      const uint64_t ev = vi + nv_base + inc_v + inc_avail;
      if (ev < vend) report(S.err, ev, kErrV1BadRead);
      s_ctl[2] = 1;
    }
    __syncthreads();
    V1PROF_MARK(6);

    // 4. literal values: each thread streams the varints ending in its chunk
    // (then in its tail chunks) out of registers; a varint begun before the
    // chunk is resumed from the 16 bytes before it
#pragma unroll
    for (int ps = 0; ps < G::kPasses; ++ps) {
      const uint32_t c0 = ps == 0 ? cs : kChunk + (uint32_t)(ps - 1) * kV1Threads * kCB + cs;
      if (c0 >= kWin || c0 >= stop_at || c0 + kCB <= p0) continue;
      const uint32_t gm = ps == 0 ? gmask : 0u;
      uint32_t cur[kNW];
#pragma unroll
      for (int k = 0; k < kNW; ++k) cur[k] = ps == 0 ? mine[k] : s_win[c0 / 4 + k];
      // the group covering byte c0 (unless one starts there): the last one before
      const uint32_t eg = ps == 0 ? ng_base : NG;  // groups before this chunk
      bool lit = false;
      uint32_t vnext = 0, kleft = 0, sh = 0;
      uint64_t acc = 0;
      if (eg > 0 && !(gm & 1u)) {
        const uint64_t m = s_gmeta[eg - 1];
        const uint32_t hb = (uint32_t)(m >> 40) & 0xffu;
        if (hb >= 0x80u) {
          const uint32_t gp = s_gpos[eg - 1];
          const uint32_t j0 = rcv[ps] - (uint32_t)((m >> 24) & 0xffffu);  // its varints ended before c0
          lit = true;
          vnext = (uint32_t)(m & 0xffffffu) + j0;
          kleft = j0 < 256u - hb ? 256u - hb - j0 : 0u;  // (0: it ended before c0)
          // resume the varint in progress: bytes (max(prev terminator, gp), c0)
          const uint32_t pv_ = prv[ps];
          const uint32_t from = (pv_ != kNone && pv_ > gp ? pv_ : gp) + 1u;
          if (from + 16u >= c0) {
            uint32_t pw[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) pw[k] = s_win[(int)(c0 / 4) - 4 + k];  // (the slack before the window)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const uint32_t y = (pw[e >> 2] >> ((e & 3) * 8)) & 0xffu;
              if ((int)c0 - 16 + e >= (int)from) {
                if (sh < 64) acc |= (uint64_t)(y & 0x7fu) << sh;
                sh += 7;
              }
            }
          } else {  // a varint longer than 16 bytes (corrupt but decodable)
            for (uint32_t bb = from; bb < c0; ++bb, sh += 7)
              if (sh < 64) acc |= (uint64_t)(s_bytes[bb] & 0x7fu) << sh;
          }
        }
      }
      uint32_t d = nv_base;  // first value of the next group starting in this chunk
#pragma unroll
      for (int e = 0; e < kCB; ++e) {
        const uint32_t x = c0 + (uint32_t)e;
        const uint32_t y = cbyte<kCB>(cur, e);
        if ((gm >> e) & 1u) {
          // a group header: a literal starts its varints after it
          lit = y >= 0x80u;
          vnext = d;
          kleft = lit ? 256u - y : 0u;
          acc = 0;
          sh = 0;
          d += x == inc_at ? inc_avail : group_values(y);
        } else if (lit && kleft && x >= p0 && x < stop_at) {
          if (sh < 64) acc |= (uint64_t)(y & 0x7fu) << sh;
          sh += 7;
          if (y < 0x80u) {
            put_v(dst, vi + vnext, S.begin, vend, sg ? unzigzag(acc) : acc);
            ++vnext;
            --kleft;
            acc = 0;
            sh = 0;
          }
        }
      }
    }
    V1PROF_MARK(7);
    // 5. runs: a short run (<= kLaneRun values) on one lane, a long one on
    // a whole wave (base + j * delta on lane j); the long ones were listed
    // by the table step
    for (uint32_t r = (uint32_t)tid; r < NR; r += kV1Threads) {
      const uint64_t m = s_rmeta[r];
      const uint32_t L = (uint32_t)(m >> 32) & 0xffu;
      if (L > kLaneRun) continue;
      const uint64_t base = s_rbase[r];
      const uint64_t v0 = vi + (uint32_t)m;
      const uint64_t delta = (uint64_t)(int64_t)(int8_t)(uint8_t)(m >> 48);
      for (uint32_t j = 0; j < L; ++j) put_v(dst, v0 + j, S.begin, vend, base + (uint64_t)j * delta);
    }
    const uint32_t nlong = s_ctl[3];
    for (uint32_t q = (uint32_t)wave; q < nlong; q += kV1Threads / kWave) {
      const uint32_t r = uni(s_rlong[q]);
      const uint64_t m = s_rmeta[r];
      const uint64_t base = s_rbase[r];
      const uint64_t v0 = vi + (uint32_t)m;
      if (v0 >= vend) continue;
      const uint32_t L = (uint32_t)(m >> 32) & 0xffu;
      const uint64_t delta = (uint64_t)(int64_t)(int8_t)(uint8_t)(m >> 48);
      for (uint32_t j = (uint32_t)lane; j < L; j += kWave) put_v(dst, v0 + j, S.begin, vend, base + (uint64_t)j * delta);
    }
    const bool stop = s_ctl[2] != 0;
    __syncthreads();  // the window and the tables are rewritten by the next pass
    V1PROF_MARK(8);
#ifdef ORCG_PHASE_PROF
    if (threadIdx.x == 0) atomicMax(&g_v1phase[9], (unsigned long long)(wall_clock64() - prof_t0_));
#endif
    vi += NV;
    if (stop) {
      stopped = true;
      break;
    }
    if (inc_pos1 != 0) {
      const uint32_t p = inc_pos1 - 1;
      if (p != p0) {
        pos = wpos + p;  // the next window starts at the long group
        continue;
      }
      // a group longer than a whole window (varints past 10 bytes, legal for
      // readLong): wave 0 decodes it serially through the descriptor
      if (wave == 0) {
        uint64_t q = pos;
        const uint32_t hb = s_bytes[p];  // (the window is dead, but its first bytes are intact)
        bool bad = false;
        if ((int8_t)hb >= 0) {
          const uint32_t L = hb + 3u;
          uint64_t u = 0;
          q += 1;
          if (q >= S.src_len) bad = true;
          const uint64_t delta = bad ? 0 : (uint64_t)(int64_t)(int8_t)s_bytes[p + 1];
          q += 1;
          if (!bad && !slow_varint(rs, bias, q, S.src_len, u)) bad = true;
          if (!bad) {
            const uint64_t base = sg ? unzigzag(u) : u;
            for (uint32_t j = (uint32_t)lane; j < L; j += kWave) put_v(dst, vi + j, S.begin, vend, base + (uint64_t)j * delta);
          } else if (lane == 0) {
            report(S.err, vi, kErrV1BadRead);
          }
          if (!bad) vi += L;
        } else {
          const uint32_t k = (uint32_t)(-(int32_t)(int8_t)hb);
          q += 1;
          for (uint32_t j = 0; j < k; ++j) {
            uint64_t u;
            if (!slow_varint(rs, bias, q, S.src_len, u)) {
              if (lane == 0) report(S.err, vi, kErrV1BadRead);
              bad = true;
              break;
            }
            if (lane == 0) put_v(dst, vi, S.begin, vend, sg ? unzigzag(u) : u);
            ++vi;
          }
        }
        if (lane == 0) {
          s_ctl[3] = bad ? 1u : 0u;
          s_wsum[1][0] = (uint32_t)(q - wpos);
          s_wsum[1][1] = (uint32_t)(vi >> 32);
          s_wsum[1][2] = (uint32_t)vi;
        }
      }
      __syncthreads();
      const bool bad = s_ctl[3] != 0;
      pos = wpos + s_wsum[1][0];
      vi = ((uint64_t)s_wsum[1][1] << 32) | s_wsum[1][2];
      __syncthreads();
      if (bad) {
        stopped = true;
        break;
      }
      if (pos > S.seg_end) {
        if (tid == 0) report(S.err, vi, kErrBadSegment);
        stopped = true;
        break;
      }
      continue;
    }
    if (np == kNone) {  // (cannot happen: the chain ends past lim or at an incomplete group)
      stopped = true;
      break;
    }
    pos = wpos + np;
  }
  if (stopped) return;  // at an error (reported)
  if (tid == 0 && S.v_next != ~0ull && vi < vend && vi != S.v_next) report(S.err, vi, kErrBadSegment);
  // the last segment ran out of stream before the requested values
  if (tid == 0 && S.v_next == ~0ull && vi < vend) report(S.err, vi, kErrV1BadRead);
}

}  // namespace

// Chunk width for segments averaging `seg_bytes`: 4-byte chunks (1 KB
// windows, twice the workgroups' parallelism per byte) up to 2 KB segments.
static int v1_chunk(uint64_t seg_bytes) { return seg_bytes <= 2048 ? 4 : 16; }

int launch_rlev1(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed, const uint64_t* d_segtab,
                 uint64_t nsegs, uint64_t value_begin, uint64_t nvalues, void* d_dst, int dst_bytes) {
  if (nsegs == 0 || nvalues == 0) return ORCG_OK;
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  const dim3 grid((unsigned)nsegs), block(kV1Threads);
  const int sg = is_signed ? 1 : 0;
  const bool narrow = v1_chunk(src_len / nsegs) == 4;
#define ORCG_V1(T, CB)                                                                                          \
  hipLaunchKernelGGL((rlev1_kernel<T, false, CB>), grid, block, 0, ctx->stream, d_src, src_len, sg, d_segtab, nsegs, \
                     value_begin, nvalues, (T*)d_dst, ctx->d_err, nullptr)
  if (dst_bytes == 8) {
    if (narrow) ORCG_V1(int64_t, 4);
    else ORCG_V1(int64_t, 16);
  } else if (dst_bytes == 4) {
    if (narrow) ORCG_V1(int32_t, 4);
    else ORCG_V1(int32_t, 16);
  } else if (dst_bytes == 2) {
    if (narrow) ORCG_V1(int16_t, 4);
    else ORCG_V1(int16_t, 16);
  } else {
    return set_error(ctx, ORCG_INVALID_ARGUMENT, "dst_bytes must be 8, 4 or 2");
  }
#undef ORCG_V1
  return hip_check(ctx, hipGetLastError(), "rlev1_kernel launch");
}

int plan_rlev1_multi(Ctx* ctx, const V1SegDesc* segs, uint64_t nsegs, std::vector<MultiLaunch>& out) {
  // one launch per chunk width, by segment bytes; the longest segments first
  // in each (their workgroups walk the most windows)
  std::vector<V1SegDesc> g[2];
  for (uint64_t j = 0; j < nsegs; ++j) {
    const V1SegDesc& d = segs[j];
    if (d.vi >= d.nvalues && d.seg_start < d.seg_end) continue;  // nothing requested (and nothing to check)
    const uint64_t end = d.seg_end < d.src_len ? d.seg_end : d.src_len;
    g[v1_chunk(end > d.seg_start ? end - d.seg_start : 0) == 4 ? 0 : 1].push_back(d);
  }
  for (int w = 1; w >= 0; --w) {
    std::vector<V1SegDesc>& v = g[w];
    if (v.empty()) continue;
    std::stable_sort(v.begin(), v.end(), [](const V1SegDesc& a, const V1SegDesc& b) {
      return a.seg_end - a.seg_start > b.seg_end - b.seg_start;
    });
    if (v.size() > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
    const void* d = nullptr;
    const int rc = stage_table(ctx, v.data(), v.size() * sizeof(V1SegDesc), &d);
    if (rc) return rc;
    out.push_back(MultiLaunch{1, w == 0 ? 4 : 16, d, 0, v.size(), 0});
  }
  return ORCG_OK;
}

int launch_rlev1_jobs(Ctx* ctx, const V1SegDesc* d_segs, uint64_t nsegs, int chunk) {
  if (chunk == 4)
    hipLaunchKernelGGL((rlev1_kernel<int64_t, true, 4>), dim3((unsigned)nsegs), dim3(kV1Threads), 0, ctx->stream,
                       nullptr, 0ull, 0, nullptr, 0ull, 0ull, 0ull, nullptr, ctx->d_err, d_segs);
  else
    hipLaunchKernelGGL((rlev1_kernel<int64_t, true, 16>), dim3((unsigned)nsegs), dim3(kV1Threads), 0, ctx->stream,
                       nullptr, 0ull, 0, nullptr, 0ull, 0ull, 0ull, nullptr, ctx->d_err, d_segs);
  return hip_check(ctx, hipGetLastError(), "rlev1_kernel launch");
}

int launch_rlev1_multi(Ctx* ctx, const V1SegDesc* segs, uint64_t nsegs) {
  std::vector<MultiLaunch> ls;
  const int rc = plan_rlev1_multi(ctx, segs, nsegs, ls);
  return rc ? rc : run_multi(ctx, ls);
}

}  // namespace orcg

#ifdef ORCG_PHASE_PROF
extern "C" int orcg_debug_rlev1_phases(unsigned long long* out, int n, int reset) {
  unsigned long long h[10];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(orcg::g_v1phase), sizeof(h)) != hipSuccess) return -1;
  for (int i = 0; i < n && i < 10; ++i) out[i] = h[i];
  if (reset) {
    unsigned long long z[10] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(orcg::g_v1phase), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// A no-op launch that makes HIP load this file's code object (warm_modules).
namespace orcg {
namespace {
__global__ void warm_rlev1_kernel() {}
}  // namespace
void warm_rlev1(hipStream_t s) { hipLaunchKernelGGL(warm_rlev1_kernel, dim3(1), dim3(64), 0, s); }
}  // namespace orcg
