// RLEv2 two-pass decode, second pass (DESIGN.md §3.1 "Two passes").
//
// The union instance's dense (short-run) passes no longer expand their runs:
// they write each run's start to a run table in HBM (RunTab: stream byte
// offset | first value in the segment) and, per segment, where each value
// slice's runs start. Here one 256-thread workgroup takes one slice of a
// segment (<= kSliceMax values), so the expansion is balanced by values
// across the chip instead of lasting as long as the slowest segment's
// discovery + expansion:
//  (1) up to kRound tabled runs of the slice are loaded, their header bytes
//      staged in LDS (one load round trip) and parsed, one thread per run
//      (RleDecoderV2::next's header logic, c++/src/RleDecoderV2.cc:184-435);
//  (2) every value of the slice is produced value-parallel into an LDS stage:
//      a binary search over the runs' first values finds its run, and the
//      value is read by random access — SHORT_REPEAT the value (:184-222),
//      DIRECT the W-bit field at j*W (:224-248), PATCHED_BASE base + field
//      (:250-370), DELTA a + j*b for a fixed step, else the signed delta
//      (:372-435);
//  (3) PATCHED_BASE patches are applied one thread per run (nextPatched's
//      loop, :340-366, with adjustGapAndPatch, :250-271); variable-width
//      DELTA runs are summed by one workgroup segmented scan over the stage
//      (a run's first value starts a segment; so does every other value);
//  (4) the stage is stored coalesced, only the values the tabled runs cover
//      (values of runs the first kernel expanded itself are left alone).
// A slice with more than kRound runs takes several rounds. Runs were checked
// by the first kernel; the packed bytes are read through a range-checked
// buffer descriptor (reads past the stream return zeros).
#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

// Phase profiling (-DORCG_PHASE_PROF): thread 0 adds the wall-clock ticks
// between consecutive marks to g_xphase[k] (orcg_debug_expand_phases).
#ifdef ORCG_PHASE_PROF
__device__ unsigned long long g_xphase[8];
#define XMARK(k)                                                        \
  do {                                                                  \
    if (threadIdx.x == 0) {                                             \
      const uint64_t now_ = wall_clock64();                             \
      atomicAdd(&g_xphase[k], (unsigned long long)(now_ - xlast_));     \
      xlast_ = now_;                                                    \
    }                                                                   \
  } while (0)
#else
#define XMARK(k) \
  do {           \
  } while (0)
#endif

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
// Slices of kSliceMax values (orcg_internal.hh), kRound runs a round: 18 KB
// of LDS and <= 80 VGPRs, so 6 workgroups share a CU (the kernel is latency
// bound: each workgroup waits on a few dependent loads). Measured on
// configs[3] / [4] (profiles/r06/ab_expand_*): 2,048-value slices with
// 512-run rounds at 4 workgroups a CU took 102 / 25 us a launch, these 86 /
// 20 us.
constexpr uint32_t kRound = 256;
constexpr int kWavesMin = 6;
constexpr uint32_t kPer = kSliceMax / kThreads;  // values per thread
constexpr int kRunsPer = kRound / kThreads;      // runs per thread in a round
static_assert(kRunsPer >= 1 && kRunsPer * kThreads == kRound, "whole runs per thread");
static_assert(kRound * 32 <= kSliceMax * 8, "header staging fits the value stage");

struct Desc {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t bias;  // descriptor offset of stream byte 0
};

__device__ __forceinline__ Desc make_desc(const uint8_t* src, uint64_t src_len) {
  const uintptr_t base = (uintptr_t)src & ~(uintptr_t)15;
  const uint64_t span = ((uintptr_t)src + src_len + 3 - base) & ~3ull;
  const uint32_t nrec = span > 0xfffff000ull ? 0xfffff000u : (uint32_t)span;
  Desc d;
  d.rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nrec, 0x00020000);
  d.bias = (uint32_t)((uintptr_t)src - base);
  return d;
}

__device__ __forceinline__ uint32_t ld32(const Desc& d, uint32_t off) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(d.rs, off, 0, 0);
}

// The W-bit big-endian field `bit` bits past descriptor offset `dp`.
__device__ __forceinline__ uint64_t fld(const Desc& d, uint32_t dp, uint32_t bit, uint32_t W) {
  const uint32_t y = dp + (bit >> 3), a = y & ~3u;
  u32x3 w;
  w.x = ld32(d, a);
  w.y = ld32(d, a + 4);
  w.z = ld32(d, a + 8);
  return field(w, y, bit & 7u, W);
}

template <typename T>
__device__ __forceinline__ void store_nt(T* p, uint64_t v) {
  __builtin_nontemporal_store((T)(int64_t)v, p);
}


__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, uint32_t d) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)x, d), hi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}

template <typename T, bool kMulti>
__global__ __launch_bounds__(kThreads, kWavesMin) void rlev2_expand_kernel(const uint8_t* __restrict__ p_src, uint64_t p_src_len,
                                                                int p_is_signed, uint64_t p_value_begin,
                                                                uint64_t p_nvalues, T* __restrict__ p_dst,
                                                                const uint64_t* __restrict__ p_dcount,
                                                                const RleJob* __restrict__ jobs, uint32_t njobs,
                                                                const RunTab rt) {
  // stage slot of value o: one padding slot after every kPer values
  auto stage_at = [](uint32_t o) -> uint32_t { return o + o / kPer; };
  __shared__ int32_t s_v[kRound];      // run's first value - the slice's first
  __shared__ uint32_t s_meta[kRound];  // kind | W << 2 | L << 9
  __shared__ uint32_t s_dp[kRound];    // descriptor offset of the packed data
  __shared__ uint64_t s_a[kRound];     // SR value / PATCHED base / DELTA first value
  __shared__ uint64_t s_b[kRound];     // DELTA step; PATCHED pl | pbs << 8 | cfb << 16
  __shared__ __attribute__((aligned(16))) uint64_t s_stage[kSliceMax + kSliceMax / kPer];
  __shared__ uint8_t s_covb[kSliceMax / kPer];  // bit e: value kPer * i + e is covered by a run of this round
  __shared__ uint32_t s_ctl[4];               // [0] runs, [1] kinds present (1 DELTA W > 0, 2 PATCHED)
  __shared__ uint64_t s_wsum[kWaves];
  __shared__ uint32_t s_wflg[kWaves];
  __shared__ uint64_t s_carry;

  const int tid = (int)threadIdx.x, lane = tid % kWave, wave = tid / kWave;
#ifdef ORCG_PHASE_PROF
  uint64_t xlast_ = wall_clock64();
  if (tid == 0) atomicAdd(&g_xphase[7], 1ull);  // workgroups
#endif
  const uint32_t spg = rt.spg, S = rt.slice;
  const uint64_t gg = blockIdx.x / spg;
  const uint32_t k = blockIdx.x - (uint32_t)(gg * spg);
  const uint32_t* hdr = rt.hdr + gg * (kRtHdr + spg);
  const uint32_t cnt = uni(hdr[0]), vdone = uni(hdr[1]);
  const uint32_t s0 = k * S;
  if (s0 >= vdone || cnt == 0) return;
  uint32_t i = k ? uni(hdr[kRtHdr + k]) : 0u;
  if (i >= cnt) return;
  const uint32_t slen = min(S, vdone - s0);
  const uint64_t vi0 = (uint64_t)uni(hdr[2]) | ((uint64_t)uni(hdr[3]) << 32);
  const uint64_t* tab = rt.tab + uni(hdr[4]);

  // the first round's table entries, requested before the job's fields (the
  // two loads overlap)
  uint64_t pre[kRunsPer] = {};
#pragma unroll
  for (int h = 0; h < kRunsPer; ++h) {
    const uint32_t idx = i + (uint32_t)tid + h * kThreads;
    if (idx < cnt) pre[h] = tab[idx];
  }
  const uint8_t* src = p_src;
  uint64_t src_len = p_src_len;
  int is_signed = p_is_signed;
  T* dst = p_dst;
  uint64_t value_begin = p_value_begin;
  uint64_t value_end = p_value_begin + (p_dcount ? uni64(*p_dcount) : p_nvalues);
  if constexpr (kMulti) {
    const RleJob* J = jobs + min(uni(hdr[5]), njobs - 1);  // the segment's job (the first kernel's lookup)
    src = (const uint8_t*)uni64((uint64_t)(uintptr_t)J->src);
    src_len = uni64(J->src_len);
    is_signed = (int)uni(J->is_signed);
    dst = (T*)uni64((uint64_t)(uintptr_t)J->dst);
    value_begin = 0;
    const uint64_t jdc = uni64((uint64_t)(uintptr_t)J->dcount);
    value_end = jdc ? uni64(*(const uint64_t*)(uintptr_t)jdc) : uni64(J->nvalues);
  }
  const uint64_t a0 = vi0 + s0;  // the slice's first value index
  if (a0 >= value_end || a0 + slen <= value_begin) return;
  const Desc d = make_desc(src, src_len);
  XMARK(0);  // header, job
  uint8_t* s_hb = (uint8_t*)s_stage;  // header staging: 32 bytes per run

  for (bool first = true;; first = false) {
    if (tid == 0) {
      s_ctl[0] = 0;
      s_ctl[1] = 0;
    }
    __syncthreads();
    // (1) the round's runs: table entries i.. that start inside the slice
    //     (sorted by value, so they are a prefix); header bytes to LDS
    uint32_t xoff[kRunsPer] = {}, xv[kRunsPer] = {};
    bool ok[kRunsPer] = {};
#pragma unroll
    for (int h = 0; h < kRunsPer; ++h) {
      const uint32_t r = (uint32_t)tid + h * kThreads, idx = i + r;
      if (idx < cnt) {
        const uint64_t e = first ? pre[h] : tab[idx];
        xoff[h] = (uint32_t)e;
        xv[h] = (uint32_t)(e >> 32);
        ok[h] = xv[h] < s0 + slen;
      }
      if (ok[h]) {
        const uint32_t y = d.bias + xoff[h], a = y & ~3u;
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 w0, w1;
        w0.x = ld32(d, a);
        w0.y = ld32(d, a + 4);
        w0.z = ld32(d, a + 8);
        w0.w = ld32(d, a + 12);
        w1.x = ld32(d, a + 16);
        w1.y = ld32(d, a + 20);
        w1.z = ld32(d, a + 24);
        w1.w = ld32(d, a + 28);
        *(u4*)(s_hb + r * 32u) = w0;
        *(u4*)(s_hb + r * 32u + 16u) = w1;
      }
    }
    uint32_t mine = 0;
#pragma unroll
    for (int h = 0; h < kRunsPer; ++h) mine += ok[h] ? 1u : 0u;
    const uint32_t wtot = wave_scan_u32(mine);
    if (lane == kWave - 1 && wtot) atomicAdd(&s_ctl[0], wtot);
    __syncthreads();
    XMARK(1);  // table entries, header bytes staged
    const uint32_t nr = uni(s_ctl[0]);
    if (nr == 0) return;
    // parse (one thread per run); the staged bytes are dead afterwards
    uint32_t kinds = 0;
#pragma unroll
    for (int h = 0; h < kRunsPer; ++h) {
      const uint32_t r = (uint32_t)tid + h * kThreads;
      if (!ok[h]) continue;
      const uint32_t sh = (d.bias + xoff[h]) & 3u;
      const uint8_t* hb = s_hb + r * 32u + sh;
      Run rn = parse_run([&](uint32_t q) { return (uint32_t)hb[q]; }, ~0ull, 32u - sh, is_signed);
      if (rn.err != kErrNone) {
        // a header past the 32 staged bytes (over-long DELTA varints, which
        // the first kernel accepts up to its 64-byte limit): from the stream
        const uint8_t* g = src + xoff[h];
        const uint64_t avail = src_len - xoff[h];
        rn = parse_run([&](uint32_t q) { return (uint32_t)g[q]; }, avail, 64u, is_signed);
      }
      s_v[r] = (int32_t)(xv[h] - s0);
      s_meta[r] = rn.kind | (rn.W << 2) | (rn.L << 9);
      s_dp[r] = d.bias + xoff[h] + rn.data;
      s_a[r] = rn.a;
      s_b[r] = rn.kind == 2 ? (uint64_t)(rn.pl | (rn.pbs << 8) | (rn.cfb << 16)) : rn.b;
      kinds |= (rn.kind == 3 && rn.W != 0) ? 1u : (rn.kind == 2 ? 2u : 0u);
    }
    {
      uint32_t kw = kinds;
      for (int o = 32; o >= 1; o >>= 1) kw |= (uint32_t)__shfl_xor((int)kw, o);
      if (lane == 0 && kw) atomicOr(&s_ctl[1], kw);
    }
    __syncthreads();
    XMARK(2);  // parsed
    const uint32_t kinds_all = uni(s_ctl[1]);
    const int32_t v_first = (int32_t)uni((uint32_t)s_v[0]);
    const uint32_t m_last = uni(s_meta[nr - 1]);
    const int32_t v_last = (int32_t)uni((uint32_t)s_v[nr - 1]);
    const uint32_t o_lo = v_first > 0 ? (uint32_t)v_first : 0u;
    const int64_t e_last = (int64_t)v_last + (int64_t)((m_last >> 9) & 0x3ffu);
    const uint32_t o_hi = e_last < (int64_t)slen ? (uint32_t)(e_last > 0 ? e_last : 0) : slen;
    // a variable-width DELTA run begun before the slice: its value at the
    // slice's first position, by one wave (the scan starts a segment there)
    const uint32_t m0 = uni(s_meta[0]);
    const bool carry = first && v_first < 0 && (m0 & 3u) == 3u && ((m0 >> 2) & 127u) != 0;
    if (carry && wave == 0) {
      const uint32_t W = (m0 >> 2) & 127u, j0 = (uint32_t)(-v_first);
      const uint64_t a = s_a[0], b = s_b[0];
      const uint32_t dp = s_dp[0];
      uint64_t sum = 0;
      for (uint32_t q = (uint32_t)lane; q + 1 < j0; q += kWave) sum += fld(d, dp, q * W, W);
      sum = last_lane(wave_inclusive_scan(sum));
      if (lane == 0) s_carry = (int64_t)b < 0 ? a + b - sum : a + b + sum;
    }
    if (carry) __syncthreads();
    // (2) the values, kPer consecutive ones per thread in registers: one
    //     binary search for the thread's first, then the run cursor advances;
    //     every value's packed bytes are requested before any is used (one
    //     memory latency per thread instead of one per value)
    const uint32_t q0 = (o_lo & ~(kPer - 1)) + (uint32_t)tid * kPer;
    uint64_t x[kPer];
    uint32_t cov = 0, beg = 0;  // bit e: value q0 + e is covered / starts a scan segment
    if (q0 < o_hi) {
      const uint32_t f0 = q0 > o_lo ? q0 : o_lo;
      uint32_t r = 0, hi = nr;  // the last run starting at or before f0
      while (hi - r > 1) {
        const uint32_t mid = (r + hi) >> 1;
        if (s_v[mid] <= (int32_t)f0) r = mid;
        else hi = mid;
      }
      int32_t vnext = r + 1 < nr ? s_v[r + 1] : 0x7fffffff;
      uint32_t re[kPer], je[kPer];
      u32x3 w[kPer];
#pragma unroll
      for (uint32_t e = 0; e < kPer; ++e) {
        const uint32_t o = q0 + e;
        while ((int32_t)o >= vnext) {  // the next run (between two tabled runs: the first kernel's values)
          ++r;
          vnext = r + 1 < nr ? s_v[r + 1] : 0x7fffffff;
        }
        const uint32_t m = s_meta[r], W = (m >> 2) & 127u, L = (m >> 9) & 0x3ffu;
        const uint32_t j = (uint32_t)((int32_t)o - s_v[r]);
        const bool in = o >= f0 && o < o_hi && j < L;
        cov |= in ? 1u << e : 0u;
        re[e] = r;
        je[e] = j;
        // the W-bit field of value j (DELTA: delta j - 2); SHORT_REPEAT and
        // uncovered values read a harmless in-stream dword
        const uint32_t kind = m & 3u;
        const uint32_t k = kind == 3 ? (j >= 2 ? j - 2 : 0u) : j;
        const uint32_t bit = (in && kind != 0 && W != 0) ? k * W : 0u;
        const uint32_t y = s_dp[r] + (bit >> 3), ya = y & ~3u;
        w[e].x = ld32(d, ya);
        w[e].y = ld32(d, ya + 4);
        w[e].z = ld32(d, ya + 8);
      }
#pragma unroll
      for (uint32_t e = 0; e < kPer; ++e) {
        const uint32_t o = q0 + e;
        x[e] = 0;
        bool bg = true;
        if ((cov >> e) & 1u) {
          const uint32_t rr = re[e], j = je[e];
          const uint32_t m = s_meta[rr], kind = m & 3u, W = (m >> 2) & 127u;
          const uint32_t k = kind == 3 ? (j >= 2 ? j - 2 : 0u) : j;
          const uint32_t bit = k * W, y = s_dp[rr] + (bit >> 3);
          const uint64_t a = s_a[rr];
          if (kind == 0) {
            x[e] = a;
          } else if (kind == 1) {
            const uint64_t f = field(w[e], y, bit & 7u, W);
            x[e] = is_signed ? unzigzag(f) : f;
          } else if (kind == 2) {
            x[e] = a + field(w[e], y, bit & 7u, W);
          } else {
            const uint64_t b = s_b[rr];
            if (W == 0) {
              x[e] = a + (uint64_t)j * b;
            } else if (j == 0) {
              x[e] = a;
            } else if (o == 0 && carry) {
              x[e] = s_carry;
            } else if (j == 1) {
              x[e] = b;
              bg = false;
            } else {
              const uint64_t dl = field(w[e], y, bit & 7u, W);
              x[e] = (int64_t)b < 0 ? 0 - dl : dl;
              bg = false;
            }
          }
        }
        beg |= bg ? 1u << e : 0u;
      }
    } else {
      beg = (1u << kPer) - 1;
#pragma unroll
      for (uint32_t e = 0; e < kPer; ++e) x[e] = 0;
    }
    // (3) variable-width DELTA: segmented inclusive scan across the threads
    //     (a segment starts at a run's first value and at every other kind's)
    if (kinds_all & 1u) {
      uint64_t acc = 0;
      uint32_t f = 0;
#pragma unroll
      for (uint32_t e = 0; e < kPer; ++e) {
        if ((beg >> e) & 1u) {
          acc = x[e];
          f = 1;
        } else {
          acc += x[e];
        }
      }
      uint64_t sv = acc;
      for (uint32_t dd = 1; dd < (uint32_t)kWave; dd <<= 1) {
        const uint64_t so = shfl_up64(sv, dd);
        const uint32_t fo = (uint32_t)__shfl_up((int)f, dd);
        if ((uint32_t)lane >= dd) {
          if (!f) sv += so;
          f |= fo;
        }
      }
      if (lane == kWave - 1) {
        s_wsum[wave] = sv;
        s_wflg[wave] = f;
      }
      uint64_t ex = shfl_up64(sv, 1);
      uint32_t exf = (uint32_t)__shfl_up((int)f, 1);
      if (lane == 0) {
        ex = 0;
        exf = 0;
      }
      __syncthreads();
      uint64_t ws = 0;
      for (int w = 0; w < wave; ++w) ws = s_wflg[w] ? s_wsum[w] : ws + s_wsum[w];
      uint64_t run = exf ? ex : ws + ex;
#pragma unroll
      for (uint32_t e = 0; e < kPer; ++e) {
        run = ((beg >> e) & 1u) ? x[e] : run + x[e];
        x[e] = run;
      }
    }
    // the stage (one padding slot per kPer values: conflict-free-ish rows)
    if (q0 < o_hi) {
#pragma unroll
      for (uint32_t e = 0; e < kPer; ++e) s_stage[stage_at(q0 + e)] = x[e];
      s_covb[q0 / kPer] = (uint8_t)cov;
    }
    __syncthreads();
    XMARK(3);  // values (+ scan) in the stage
    // (4) PATCHED_BASE patches, one thread per run: position = running sum of
    //     the gaps; an escape (gap 255, patch 0) only advances; a patch that
    //     does not move past the previous one, or lands past the run, ends it
    if (kinds_all & 2u) {
      for (uint32_t r = (uint32_t)tid; r < nr; r += kThreads) {
        const uint32_t m = s_meta[r];
        if ((m & 3u) != 2u) continue;
        const uint32_t W = (m >> 2) & 127u, L = (m >> 9) & 0x3ffu;
        const uint64_t pk = s_b[r], a = s_a[r];
        const uint32_t pl = (uint32_t)pk & 0xffu, pbs = (uint32_t)(pk >> 8) & 0xffu, cfb = (uint32_t)(pk >> 16) & 0xffu;
        const uint32_t p0 = s_dp[r] + (W * L + 7u) / 8u;
        const uint64_t pmask = (1ull << pbs) - 1;
        const int32_t v = s_v[r];
        uint32_t c = 0, prev = 0;
        bool any = false;
        for (uint32_t q = 0; q < pl; ++q) {
          const uint64_t e = fld(d, p0, q * cfb, cfb);
          const uint32_t gap = (uint32_t)(e >> pbs);
          const uint64_t patch = e & pmask;
          c += gap;
          if (gap == 255u && patch == 0) continue;
          if ((any && c == prev) || c >= L) break;
          const int32_t o = v + (int32_t)c;
          if (o >= (int32_t)o_lo && o < (int32_t)o_hi) {
            const uint32_t si = stage_at((uint32_t)o);
            const uint64_t lit = s_stage[si] - a;
            s_stage[si] = a + (lit | (patch << (W & 63u)));
          }
          prev = c;
          any = true;
        }
      }
      __syncthreads();
    }
    // (5) coalesced stores of the covered values
    for (uint32_t base = o_lo & ~(uint32_t)(kThreads - 1); base < o_hi; base += kThreads) {
      const uint32_t o = base + (uint32_t)tid;
      if (o >= o_lo && o < o_hi && ((s_covb[o / kPer] >> (o % kPer)) & 1u)) {
        const uint64_t g = a0 + o;
        if (g >= value_begin && g < value_end) store_nt(dst + (g - value_begin), s_stage[stage_at(o)]);
      }
    }
    XMARK(4);  // patches, stores issued
    i += nr;
    if (nr < kRound || i >= cnt) return;
    __syncthreads();  // the stage and run parameters are rewritten by the next round
  }
}

__global__ void warm_rlev2_expand_kernel() {}

}  // namespace

int launch_rlev2_expand(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed, uint64_t value_begin,
                        uint64_t nvalues, void* d_dst, int dst_bytes, const uint64_t* d_count, const RleJob* jobs_d,
                        uint32_t njobs, uint64_t nsegs, const RunTab& rt) {
  if (!rt.tab || !rt.hdr || rt.spg == 0 || rt.slice == 0 || rt.slice > kSliceMax || rt.slice % kThreads)
    return set_error(ctx, ORCG_INVALID_ARGUMENT, "bad run table");
  const uint64_t grid = nsegs * rt.spg;
  if (grid == 0) return ORCG_OK;
  if (grid > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many slices");
  const dim3 g((unsigned)grid), b(kThreads);
if (jobs_d) {
    hipLaunchKernelGGL((rlev2_expand_kernel<int64_t, true>), g, b, 0, ctx->stream, nullptr, 0, 0, 0, 0, nullptr,
                       nullptr, jobs_d, njobs, rt);
  } else if (dst_bytes == 8) {
    hipLaunchKernelGGL((rlev2_expand_kernel<int64_t, false>), g, b, 0, ctx->stream, d_src, src_len, is_signed,
                       value_begin, nvalues, (int64_t*)d_dst, d_count, nullptr, 0, rt);
  } else if (dst_bytes == 4) {
    hipLaunchKernelGGL((rlev2_expand_kernel<int32_t, false>), g, b, 0, ctx->stream, d_src, src_len, is_signed,
                       value_begin, nvalues, (int32_t*)d_dst, d_count, nullptr, 0, rt);
  } else {
    hipLaunchKernelGGL((rlev2_expand_kernel<int16_t, false>), g, b, 0, ctx->stream, d_src, src_len, is_signed,
                       value_begin, nvalues, (int16_t*)d_dst, d_count, nullptr, 0, rt);
  }
  return hip_check(ctx, hipGetLastError(), "rlev2_expand_kernel launch");
}

#ifdef ORCG_PHASE_PROF
extern "C" int orcg_debug_expand_phases(unsigned long long* out, int n, int reset) {
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_xphase), sizeof(h)) != hipSuccess) return -1;
  for (int i = 0; i < n && i < 8; ++i) out[i] = h[i];
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_xphase), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

void warm_rlev2_expand(hipStream_t s) { hipLaunchKernelGGL(warm_rlev2_expand_kernel, dim3(1), dim3(64), 0, s); }

}  // namespace orcg
