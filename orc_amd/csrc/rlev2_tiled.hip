// RLEv2 decode, tiled through LDS (the default kernel).
//
// One 256-thread workgroup per segment. The segment's bytes stream through a
// 33 KB LDS window filled by buffer_load ... lds (LDS-DMA, 1 KB per wave
// instruction, range-checked so reads past the stream return zeros). Wave 0
// walks the run headers in LDS (RleDecoderV2::next's run loop,
// c++/src/RleDecoderV2.cc:132-170) and publishes a run table; all four waves
// then expand runs round-robin straight out of LDS:
//   SHORT_REPEAT  broadcast                                      (:184-222)
//   DIRECT        per-lane big-endian W-bit extract + zigzag     (:224-248)
//   PATCHED_BASE  extract + base, patches applied in registers   (:250-370)
//   DELTA         wavefront int64 inclusive scan                 (:372-435)
// A window holds every run that STARTS in its first kChunk bytes; runs are at
// most kMaxRun bytes, so they end inside it. The next window starts at the
// first unprocessed run.
#include "rlev2_device.hh"

namespace orcg {
namespace {
using namespace dev;

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr uint32_t kWin = 33 * 1024;             // LDS window (multiple of 1 KB)
constexpr uint32_t kMaxRun = 4608;               // >= 4356, the longest legal run
constexpr uint32_t kChunk = kWin - kMaxRun;      // run starts per window
constexpr int kMaxRuns = 512;                    // run-table capacity per window

struct Lds {
  uint32_t win[kWin / 4 + 8];  // + 32 B pad: the 12-byte extract may read past a run
  uint32_t run_off[kMaxRuns];  // LDS byte offset of each run header
  uint32_t run_val[kMaxRuns];  // value offset of each run from the window's first value
  uint32_t ctl[8];
};

__device__ __forceinline__ uint32_t lds_byte(const Lds& s, uint32_t o) {
  return (s.win[o >> 2] >> ((o & 3u) * 8)) & 0xffu;
}

__device__ __forceinline__ u32x3 lds12(const Lds& s, uint32_t o) {
  const uint32_t i = o >> 2;
  u32x3 w;
  w.x = s.win[i];
  w.y = s.win[i + 1];
  w.z = s.win[i + 2];
  return w;
}

// Expand one run (already validated by the walk) with one wave.
template <typename T>
__device__ __forceinline__ void expand_run(const Lds& s, uint32_t hoff, uint64_t v0, int is_signed,
                                           uint64_t value_begin, uint64_t value_end, T* dst,
                                           int lane) {
  const Run r = parse_run([&](uint32_t i) { return lds_byte(s, hoff + i); }, ~0ull, kMaxRun, is_signed);
  const uint32_t L = r.L;
  // clip to the requested output range
  if (v0 + L <= value_begin || v0 >= value_end) return;
  const uint32_t d = hoff + r.data;  // LDS offset of the packed data
  const uint32_t niter = (L + kWave - 1) / kWave;

  if (r.kind == 0) {
    const uint64_t o = v0 + (uint64_t)lane;
    if ((uint32_t)lane < L && o >= value_begin && o < value_end) put(dst, o - value_begin, r.a);
    return;
  }
  if (r.kind == 1) {
    const uint32_t W = r.W;
#pragma unroll
    for (int it = 0; it < kMaxRunUnroll; ++it) {
      if ((uint32_t)it < niter) {
        const uint32_t j = it * kWave + lane;
        const uint32_t bit = j * W;
        const uint32_t br = d + (bit >> 3);
        uint64_t v = field(lds12(s, br), br, bit & 7u, W);
        if (is_signed) v = unzigzag(v);
        const uint64_t o = v0 + j;
        if (j < L && o >= value_begin && o < value_end) put(dst, o - value_begin, v);
      }
    }
    return;
  }
  if (r.kind == 2) {
    // Literals into registers, then the patch list walked in order exactly as
    // nextPatched (:340-366) with adjustGapAndPatch (:250-271): an escape
    // (gap 255, patch 0) only advances; a patch that does not move past the
    // previous one stalls the walk; positions >= L are never reached.
    const uint32_t W = r.W;
    uint64_t lit[kMaxRunUnroll];
#pragma unroll
    for (int it = 0; it < kMaxRunUnroll; ++it) {
      lit[it] = 0;
      if ((uint32_t)it < niter) {
        const uint32_t bit = (it * kWave + lane) * W;
        const uint32_t br = d + (bit >> 3);
        lit[it] = field(lds12(s, br), br, bit & 7u, W);
      }
    }
    const uint32_t p0 = d + (W * L + 7) / 8;  // patch list
    uint64_t entry = 0;
    if ((uint32_t)lane < r.pl) {
      const uint32_t bit = lane * r.cfb;
      const uint32_t br = p0 + (bit >> 3);
      entry = field(lds12(s, br), br, bit & 7u, r.cfb);
    }
    const uint64_t pmask = (1ull << r.pbs) - 1;  // pbs <= 63 (checked by the walk)
    const uint32_t e_lo = (uint32_t)entry, e_hi = (uint32_t)(entry >> 32);
    uint64_t cum = 0, prev = 0;
    bool first = true;
    for (uint32_t k = 0; k < r.pl; ++k) {
      const uint64_t e = ((uint64_t)rdlane(e_hi, k) << 32) | rdlane(e_lo, k);
      const uint64_t gp = e >> r.pbs, pv = e & pmask;
      cum += gp;
      if (gp == 255 && pv == 0) continue;
      if ((!first && cum == prev) || cum >= L) break;
      const uint32_t slot = (uint32_t)cum / kWave, who = (uint32_t)cum % kWave;
      const uint64_t add = pv << (W & 63u);
#pragma unroll
      for (int it = 0; it < kMaxRunUnroll; ++it)
        if ((uint32_t)it == slot && (uint32_t)lane == who) lit[it] |= add;
      prev = cum;
      first = false;
    }
#pragma unroll
    for (int it = 0; it < kMaxRunUnroll; ++it) {
      const uint32_t j = it * kWave + lane;
      const uint64_t o = v0 + j;
      if ((uint32_t)it < niter && j < L && o >= value_begin && o < value_end)
        put(dst, o - value_begin, r.a + lit[it]);
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
        put(dst, o - value_begin, r.a + (uint64_t)j * r.b);
    }
    return;
  }
  const uint32_t W = r.W;
  const uint64_t v1 = r.a + r.b;
  const bool neg = (int64_t)r.b < 0;
  uint64_t carry = 0;
#pragma unroll
  for (int it = 0; it < kMaxRunUnroll; ++it) {
    if ((uint32_t)it < niter) {
      const uint32_t j = it * kWave + lane;
      const int32_t k = (int32_t)j - 2;
      uint64_t dlt = 0;
      if (k >= 0 && j < L) {
        const uint32_t bit = (uint32_t)k * W;
        const uint32_t br = d + (bit >> 3);
        dlt = field(lds12(s, br), br, bit & 7u, W);
      }
      const uint64_t sum = wave_inclusive_scan(dlt, lane) + carry;
      carry = (uint64_t)__shfl(sum, kWave - 1, kWave);
      const uint64_t v = j == 0 ? r.a : (j == 1 ? v1 : (neg ? v1 - sum : v1 + sum));
      const uint64_t o = v0 + j;
      if (j < L && o >= value_begin && o < value_end) put(dst, o - value_begin, v);
    }
  }
}

template <typename T, bool kPositions>
__global__ __launch_bounds__(kThreads) void rlev2_tiled_kernel(
    const uint8_t* __restrict__ src, uint64_t src_len, int is_signed,
    const uint64_t* __restrict__ segtab, uint64_t nsegs, uint64_t rows_per_group,
    uint64_t value_begin, uint64_t nvalues, T* __restrict__ dst, unsigned long long* err) {
  __shared__ Lds s;
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
    if (tid == 0 && v_next != ~0ull && v_next != vi && seg_start < src_len)
      report(err, vi, kErrBadSegment);
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
  while (pos < seg_end && vi < value_end) {
    const uint32_t wrel = (uint32_t)(pos - bias) & ~15u;  // window start (descriptor-relative)
    const uint64_t wpos = bias + wrel;                     // window start (stream offset)
    // ---- fill the window: 1 KB per wave instruction, 4 KB per round
#pragma unroll
    for (uint32_t r = 0; r < (kWin + 4095) / 4096; ++r) {
      const uint32_t off = r * 4096 + wave * 1024;
      if (off < kWin)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)((char*)s.win + off), 16,
            wrel + off + lane * 16, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- walk the run headers (wave 0, wave-uniform)
    if (wave == 0) {
      uint64_t p = pos, v = vi;
      uint32_t n = 0, stop = 0;
      while (p < seg_end && v < value_end && n < (uint32_t)kMaxRuns) {
        const uint32_t lp = (uint32_t)(p - wpos);
        if (lp >= kChunk && n > 0) break;  // starts in the next window
        const Run r = parse_run([&](uint32_t i) { return lds_byte(s, lp + i); }, src_len - p, kMaxRun,
                                is_signed);
        uint32_t e = r.err;
        if (e == kErrNone && p + r.bytes > seg_end) e = kErrBadSegment;
        if (e == kErrNone && lp + r.bytes > kWin) e = kErrBadRead;  // cannot happen for legal headers
        if (e != kErrNone) {
          if (lane == 0) report(err, v, e);
          stop = 1;
          break;
        }
        if (lane == 0) {
          s.run_off[n] = lp;
          s.run_val[n] = (uint32_t)(v - vi);
        }
        ++n;
        p += r.bytes;
        v += r.L;
      }
      if (lane == 0) {
        s.ctl[0] = n;
        s.ctl[1] = stop;
        s.ctl[2] = (uint32_t)(p - pos);
        s.ctl[3] = (uint32_t)(v - vi);
      }
    }
    __syncthreads();
    const uint32_t n = s.ctl[0], stop = s.ctl[1];
    const uint64_t next_pos = pos + s.ctl[2], next_vi = vi + s.ctl[3];

    // ---- expand: run k on wave k % kWaves
    for (uint32_t k = wave; k < n; k += kWaves)
      expand_run(s, s.run_off[k], vi + s.run_val[k], is_signed, value_begin, value_end, dst, lane);
    __syncthreads();  // the window is refilled next
    if (stop) return;
    pos = next_pos;
    vi = next_vi;
  }
  if (tid == 0 && v_next != ~0ull && vi < value_end && vi != v_next) report(err, vi, kErrBadSegment);
}

}  // namespace

int launch_rlev2_tiled(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                       const uint64_t* d_segtab, uint64_t nsegs, bool positions_mode,
                       uint64_t rows_per_group, uint64_t value_begin, uint64_t nvalues, void* d_dst,
                       int dst_bytes) {
  if (nsegs == 0 || nvalues == 0) return ORCG_OK;
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  const dim3 grid((unsigned)nsegs), block(kThreads);
  const int sg = is_signed ? 1 : 0;
#define ORCG_LAUNCH(T, P)                                                                     \
  hipLaunchKernelGGL((rlev2_tiled_kernel<T, P>), grid, block, 0, ctx->stream, d_src, src_len, \
                     sg, d_segtab, nsegs, rows_per_group, value_begin, nvalues, (T*)d_dst,    \
                     ctx->d_err)
  switch (dst_bytes) {
    case 8:
      if (positions_mode) ORCG_LAUNCH(int64_t, true); else ORCG_LAUNCH(int64_t, false);
      break;
    case 4:
      if (positions_mode) ORCG_LAUNCH(int32_t, true); else ORCG_LAUNCH(int32_t, false);
      break;
    case 2:
      if (positions_mode) ORCG_LAUNCH(int16_t, true); else ORCG_LAUNCH(int16_t, false);
      break;
    default:
      return set_error(ctx, ORCG_INVALID_ARGUMENT, "dst_bytes must be 8, 4 or 2");
  }
#undef ORCG_LAUNCH
  return hip_check(ctx, hipGetLastError(), "rlev2_tiled_kernel launch");
}

}  // namespace orcg
