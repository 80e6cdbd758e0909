// RLEv2 integer-stream decode on CDNA4 (gfx950).
//
// Replaces the per-run loop of orc::RleDecoderV2 (c++/src/RleDecoderV2.cc:
// 132-453) and the scalar / AVX-512 bit unpackers it dispatches to
// (c++/src/BpackingDefault.cc:33-366, c++/src/BpackingAvx512.cc:152-2586).
//
// Work decomposition: one wavefront per SEGMENT, a run-aligned
// byte range whose first value index is known up front (a row-index position
// or a host-planned cut). Inside a segment the wave walks the run headers with
// wave-uniform (scalar) arithmetic out of a 256-byte header window held one
// dword per lane, and all 64 lanes expand each run:
//   SHORT_REPEAT  broadcast store                              (:184-222)
//   DIRECT        per-lane W-bit big-endian extract + zigzag   (:224-248)
//   PATCHED_BASE  extract + base, patch list scattered via LDS (:250-370)
//   DELTA         wavefront int64 inclusive scan of |delta|    (:372-435)
// Every global read goes through a range-checked buffer descriptor, so reads
// past the end of the caller's stream return zero instead of faulting; the
// reference's truncation errors are detected from the header arithmetic.
#include "orcg_internal.hh"

namespace orcg {
namespace {

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

constexpr int kWave = 64;
constexpr int kMaxRunUnroll = 8;  // 512 values / 64 lanes

// FBSToBitWidthMap (c++/src/RLEV2Util.cc:24-26)
__device__ __forceinline__ uint32_t fbs_width(uint32_t code) {
  // 1..24 map to themselves (+1); 24..31 -> 26,28,30,32,40,48,56,64
  if (code < 24) return code + 1;
  const uint32_t hi = code - 24;  // 0..7
  // packed table of {26,28,30,32,40,48,56,64}
  const uint64_t t = 0x40383028201E1C1Aull;
  return (uint32_t)((t >> (8 * hi)) & 0xff);
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

__device__ __forceinline__ uint64_t unzigzag(uint64_t v) { return (v >> 1) ^ (0 - (v & 1)); }

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// 12 bytes starting at the dword containing `rel` (relative to the
// descriptor base, which is 4-byte aligned).
__device__ __forceinline__ u32x3 load12(__amdgpu_buffer_rsrc_t r, uint32_t rel) {
  return __builtin_amdgcn_raw_buffer_load_b96(r, rel & ~3u, 0, 0);
}

// The W-bit big-endian field starting `sh` bits into byte `rel` (W in 1..64,
// sh in 0..7, W + sh <= 64 for every width ORC can produce).
__device__ __forceinline__ uint64_t field(u32x3 w, uint32_t rel, uint32_t sh, uint32_t W) {
  const uint32_t r = rel & 3u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(w.y, w.x, r);
  const uint32_t hi = __builtin_amdgcn_alignbyte(w.z, w.y, r);
  const uint64_t be = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
  return (be << sh) >> (64 - W);
}

// Wavefront inclusive prefix sum of a 64-bit value.
__device__ __forceinline__ uint64_t wave_inclusive_scan(uint64_t x, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, kWave);
    if (lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ void report(unsigned long long* err, uint64_t value_index, uint32_t code) {
  atomicMin(err, (unsigned long long)((value_index << 8) | code));
}

template <typename T>
__device__ __forceinline__ void put(T* dst, uint64_t idx, uint64_t v) {
  dst[idx] = (T)(int64_t)v;
}

// Header window: 256 stream bytes starting at the 4-aligned `base`, one dword
// per lane; bytes are fetched with v_readlane (scalar).
struct Window {
  uint32_t word;
  uint32_t base;  // relative to the descriptor base
  __device__ __forceinline__ uint32_t byte(uint32_t rel) const {
    const uint32_t o = rel - base;
    const uint32_t w = rdlane(word, o >> 2);
    return (w >> ((o & 3u) * 8)) & 0xffu;
  }
};

// kJava: 0 = the C++ reader's rules; 1 = Java's RunLengthIntegerReaderV2
// (java/core/src/java/org/apache/orc/impl/RunLengthIntegerReaderV2.java):
// readDeltaValues (:86-147) never rejects a one-value DELTA run with a bit
// width (it emits the first value and first + deltaBase: two values, no
// packed deltas); readPatchedBaseValues (:149-260) reads an empty patch list
// and fails on unpackedPatch[0] (after the run's bytes), and fails on pw +
// pgw > 64 with its IOException; 2 = Java with skipCorrupt, which reads such
// a list at getClosestFixedBits(pw + pgw) bits an entry with Java's shifts
// (by the width mod 64: pw = 64 gives gap = the entry, patch = 0).
template <typename T, bool kPositions, int kJava>
__global__ __launch_bounds__(kWave) void rlev2_decode_kernel(
    const uint8_t* __restrict__ src, uint64_t src_len, int is_signed,
    const uint64_t* __restrict__ segtab, uint64_t nsegs, uint64_t rows_per_group,
    uint64_t value_begin, uint64_t nvalues, T* __restrict__ dst, unsigned long long* err) {
  __shared__ uint64_t patch_lds[512];

  const uint64_t g = blockIdx.x;
  const int lane = (int)threadIdx.x;
  const uint64_t value_end = value_begin + nvalues;

  uint64_t seg_start = segtab[2 * g];
  uint64_t vi = kPositions ? g * rows_per_group - segtab[2 * g + 1] : segtab[2 * g + 1];
  uint64_t seg_end = src_len;
  uint64_t v_next = ~0ull;  // first value of the next segment, when known
  if (g + 1 < nsegs) {
    seg_end = segtab[2 * (g + 1)];
    v_next = kPositions ? (g + 1) * rows_per_group - segtab[2 * (g + 1) + 1] : segtab[2 * (g + 1) + 1];
  }
  if (seg_end > src_len) seg_end = src_len;
  if (vi >= value_end || v_next <= value_begin) return;  // no overlap with the output range
  if (seg_start >= seg_end) {
    if (v_next != ~0ull && v_next != vi && seg_start < src_len) report(err, vi, kErrBadSegment);
    if (v_next == ~0ull) report(err, vi, kErrBadRead);  // no stream left for the requested values
    return;
  }

  // Range-checked descriptor over [seg_start & ~3, src_len rounded up to 4).
  const uintptr_t base_abs = ((uintptr_t)src + seg_start) & ~(uintptr_t)3;
  const uintptr_t end_abs = ((uintptr_t)src + src_len + 3) & ~(uintptr_t)3;
  const uint64_t span = (uint64_t)(end_abs - base_abs);
  const uint32_t nrec = span > 0xfffffff0ull ? 0xfffffff0u : (uint32_t)span;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base_abs, (short)0, (int)nrec, 0x00020000);
  // stream offset p  ->  descriptor-relative offset p - bias
  const uint64_t bias = (uint64_t)(base_abs - (uintptr_t)src);

  Window win;
  win.base = 0xffffffffu;
  win.word = 0;

  bool patch_lds_clean = false;  // zeroed lazily on the first PATCHED_BASE run
  uint64_t pos = seg_start;
  // Values past the output range are never needed: stop there, so corrupt
  // runs beyond it are not reported (the reference throws lazily too).
  while (pos < seg_end && vi < value_end) {
    const uint32_t rel = (uint32_t)(pos - bias);
    if (win.base == 0xffffffffu || rel < win.base || rel + 32 > win.base + 256) {
      win.base = rel & ~3u;
      win.word = __builtin_amdgcn_raw_buffer_load_b32(rs, win.base + 4u * lane, 0, 0);
    }
    const uint32_t fb = win.byte(rel);
    const uint32_t kind = fb >> 6;
    uint64_t L;
    uint64_t run_end;

    if (kind == 0) {  // ---------------------------------------- SHORT_REPEAT
      const uint32_t nb = ((fb >> 3) & 7u) + 1u;
      L = (fb & 7u) + 3u;
      run_end = pos + 1 + nb;
      if (run_end > src_len) { report(err, vi, kErrBadRead); return; }
      if (run_end > seg_end) { report(err, vi, kErrBadSegment); return; }
      uint64_t v = 0;
      for (uint32_t i = 0; i < nb; ++i) v = (v << 8) | win.byte(rel + 1 + i);
      if (is_signed) v = unzigzag(v);
      const uint64_t j = (uint64_t)lane;
      if (j < L && vi + j >= value_begin && vi + j < value_end) put(dst, vi + j - value_begin, v);
    } else if (kind == 1 || kind == 2) {  // ------------- DIRECT / PATCHED_BASE
      const uint32_t W = fbs_width((fb >> 1) & 0x1fu);
      if (pos + 2 > src_len) { report(err, vi, kErrBadRead); return; }
      L = ((uint64_t)(fb & 1u) << 8 | win.byte(rel + 1)) + 1;
      uint64_t data = pos + 2;
      uint64_t base = 0;
      uint32_t pbs = 0, pl = 0, cfb = 0;
      if (kind == 2) {
        if (pos + 4 > src_len) { report(err, vi, kErrBadRead); return; }
        const uint32_t third = win.byte(rel + 2);
        const uint32_t fourth = win.byte(rel + 3);
        const uint32_t bw = (third >> 5) + 1u;
        pbs = fbs_width(third & 0x1fu);
        const uint32_t pgw = (fourth >> 5) + 1u;
        pl = fourth & 0x1fu;
        if (pl == 0 && kJava == 0) { report(err, vi, kErrPatchedPl0); return; }
        if (pos + 4 + bw > src_len) { report(err, vi, kErrBadRead); return; }
        for (uint32_t i = 0; i < bw; ++i) base = (base << 8) | win.byte(rel + 4 + i);
        const uint64_t m = 1ull << (bw * 8 - 1);
        if (base & m) base = 0 - (base & ~m);  // sign-magnitude (:311-317)
        data = pos + 4 + bw;
        if (data + ((uint64_t)W * L + 7) / 8 > src_len) { report(err, vi, kErrBadRead); return; }
        if (pbs + pgw > 64 && kJava != 2) {
          report(err, vi, kJava ? kErrJavaCorrupt : kErrPatchedWidth);
          return;
        }
        cfb = closest_fixed_bits(pbs + pgw);
      }
      const uint64_t data_end = data + ((uint64_t)W * L + 7) / 8;
      run_end = data_end + ((uint64_t)cfb * pl + 7) / 8;
      if (run_end > src_len) { report(err, vi, kErrBadRead); return; }
      if (kJava && kind == 2 && pl == 0) { report(err, vi, kErrJavaPatchIndex); return; }
      if (run_end > seg_end) { report(err, vi, kErrBadSegment); return; }

      if (vi + L > value_begin && vi < value_end) {
        // Issue every load of the run before any use (one latency per run).
        const uint32_t drel = (uint32_t)(data - bias);
        const uint32_t niter = (uint32_t)((L + kWave - 1) / kWave);
        u32x3 raw[kMaxRunUnroll];
#pragma unroll
        for (int it = 0; it < kMaxRunUnroll; ++it) {
          const uint32_t bit = (uint32_t)(it * kWave + lane) * W;
          raw[it] = load12(rs, drel + (bit >> 3));
        }
        if (kind == 2) {
          // Patch list: pl entries of cfb bits, entry = (gap << pbs) | patch,
          // one per lane. Walked in order exactly like nextPatched's loop
          // (:340-366) with adjustGapAndPatch (:250-271): an escape entry
          // (gap 255, patch 0) only advances the position; a patch whose
          // position does not move past the previous one stalls the walk;
          // positions >= L are never reached.
          const uint32_t prel = (uint32_t)(data_end - bias);
          uint64_t entry = 0;
          if ((uint32_t)lane < pl) {
            const uint32_t bit = (uint32_t)lane * cfb;
            entry = field(load12(rs, prel + (bit >> 3)), prel + (bit >> 3), bit & 7u, cfb);
          }
          // pbs <= 63 here, except under skipCorrupt: Java shifts by the
          // width mod 64 (pw = 64: no patch bits, the whole entry is the gap)
          const uint32_t psh = pbs & 63u;
          const uint64_t pmask = (1ull << psh) - 1;
          const uint32_t e_lo = (uint32_t)entry, e_hi = (uint32_t)(entry >> 32);
          if (!patch_lds_clean) {
#pragma unroll
            for (int i = 0; i < 512 / kWave; ++i) patch_lds[i * kWave + lane] = 0;
            __syncthreads();
            patch_lds_clean = true;
          }
          for (int pass = 0; pass < 2; ++pass) {  // pass 0: scatter, pass 1: clear
            uint64_t cum = 0, prev = 0;
            bool first = true;
            for (uint32_t k = 0; k < pl; ++k) {
              const uint64_t e = ((uint64_t)rdlane(e_hi, k) << 32) | rdlane(e_lo, k);
              const uint64_t gp = e >> psh, pv = e & pmask;
              cum += gp;
              if (gp == 255 && pv == 0) continue;
              if ((!first && cum == prev) || cum >= L) break;
              if (lane == 0) patch_lds[cum] = pass == 0 ? (pv << (W & 63u)) : 0;
              prev = cum;
              first = false;
            }
            __syncthreads();
            if (pass == 0) {
#pragma unroll
              for (int it = 0; it < kMaxRunUnroll; ++it) {
                if ((uint32_t)it < niter) {
                  const uint64_t j = (uint64_t)(it * kWave + lane);
                  const uint32_t bit = (uint32_t)j * W;
                  const uint32_t br = drel + (bit >> 3);
                  if (j < L) {
                    const uint64_t lit = field(raw[it], br, bit & 7u, W);
                    const uint64_t v = base + (lit | patch_lds[j]);
                    const uint64_t o = vi + j;
                    if (o >= value_begin && o < value_end) put(dst, o - value_begin, v);
                  }
                }
              }
              __syncthreads();
            }
          }
        } else {
#pragma unroll
          for (int it = 0; it < kMaxRunUnroll; ++it) {
            if ((uint32_t)it < niter) {
              const uint64_t j = (uint64_t)(it * kWave + lane);
              const uint32_t bit = (uint32_t)j * W;
              const uint32_t br = drel + (bit >> 3);
              if (j < L) {
                uint64_t v = field(raw[it], br, bit & 7u, W);
                if (is_signed) v = unzigzag(v);
                const uint64_t o = vi + j;
                if (o >= value_begin && o < value_end) put(dst, o - value_begin, v);
              }
            }
          }
        }
      }
    } else {  // ------------------------------------------------------- DELTA
      const uint32_t fbo = (fb >> 1) & 0x1fu;
      const uint32_t W = fbo ? fbs_width(fbo) : 0u;
      if (pos + 2 > src_len) { report(err, vi, kErrBadRead); return; }
      L = ((uint64_t)(fb & 1u) << 8 | win.byte(rel + 1)) + 1;
      // two varints: base (zigzag if signed) and delta base (always zigzag)
      uint64_t q = pos + 2;
      uint64_t vals[2] = {0, 0};
      for (int k = 0; k < 2; ++k) {
        uint64_t acc = 0;
        uint32_t shift = 0;
        uint32_t b;
        do {
          if (q >= src_len) { report(err, vi, kErrBadRead); return; }
          if ((uint32_t)(q - bias) + 1 > win.base + 256) {  // never for well-formed varints
            report(err, vi, kErrBadRead);
            return;
          }
          b = win.byte((uint32_t)(q - bias));
          ++q;
          if (shift < 64) acc |= (uint64_t)(b & 0x7fu) << shift;
          shift += 7;
        } while (b >= 0x80u);
        vals[k] = acc;
      }
      const uint64_t first = is_signed ? unzigzag(vals[0]) : vals[0];
      const uint64_t dbase = unzigzag(vals[1]);
      if (W != 0 && L < 2) {
        if (kJava == 0) { report(err, vi, kErrDeltaLength); return; }
        L = 2;  // Java: the first value and first + deltaBase (:125-145)
      }
      const uint64_t data = q;
      run_end = data + (W ? ((uint64_t)W * (L - 2) + 7) / 8 : 0);
      if (run_end > src_len) { report(err, vi, kErrBadRead); return; }
      if (run_end > seg_end) { report(err, vi, kErrBadSegment); return; }
      if (vi + L > value_begin && vi < value_end) {
        const uint32_t niter = (uint32_t)((L + kWave - 1) / kWave);
        if (W == 0) {
          // fixed delta: v_j = first + j * deltaBase (:405-409)
#pragma unroll
          for (int it = 0; it < kMaxRunUnroll; ++it) {
            if ((uint32_t)it < niter) {
              const uint64_t j = (uint64_t)(it * kWave + lane);
              const uint64_t o = vi + j;
              if (j < L && o >= value_begin && o < value_end) put(dst, o - value_begin, first + j * dbase);
            }
          }
        } else {
          // v_0 = first, v_1 = first + deltaBase, v_j = v_{j-1} +/- |d_j| (:411-430)
          const uint32_t drel = (uint32_t)(data - bias);
          u32x3 raw[kMaxRunUnroll];
#pragma unroll
          for (int it = 0; it < kMaxRunUnroll; ++it) {
            const int64_t k = (int64_t)(it * kWave + lane) - 2;
            const uint32_t bit = (uint32_t)(k < 0 ? 0 : k) * W;
            raw[it] = load12(rs, drel + (bit >> 3));
          }
          const uint64_t v1 = first + dbase;
          const bool neg = (int64_t)dbase < 0;
          uint64_t carry = 0;
#pragma unroll
          for (int it = 0; it < kMaxRunUnroll; ++it) {
            if ((uint32_t)it < niter) {
              const uint64_t j = (uint64_t)(it * kWave + lane);
              const int64_t k = (int64_t)j - 2;
              const uint32_t bit = (uint32_t)(k < 0 ? 0 : k) * W;
              const uint32_t br = drel + (bit >> 3);
              const uint64_t d = (k >= 0 && j < L) ? field(raw[it], br, bit & 7u, W) : 0;
              const uint64_t s = wave_inclusive_scan(d, lane) + carry;
              carry = (uint64_t)__shfl(s, kWave - 1, kWave);
              uint64_t v;
              if (j == 0) v = first;
              else if (j == 1) v = v1;
              else v = neg ? v1 - s : v1 + s;
              const uint64_t o = vi + j;
              if (j < L && o >= value_begin && o < value_end) put(dst, o - value_begin, v);
            }
          }
        }
      }
    }
    pos = run_end;
    vi += L;
  }
  if (v_next != ~0ull && vi < value_end && vi != v_next) report(err, vi, kErrBadSegment);
  if (v_next == ~0ull && vi < value_end) report(err, vi, kErrBadRead);  // stream ended early
}

}  // namespace

int launch_rlev2_decode(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                        const uint64_t* d_segtab, uint64_t nsegs, bool positions_mode,
                        uint64_t rows_per_group, uint64_t value_begin, uint64_t nvalues,
                        void* d_dst, int dst_bytes, int java) {
  if (nsegs == 0 || nvalues == 0) return ORCG_OK;
  if (nsegs > 0x7fffffffull) return set_error(ctx, ORCG_INVALID_ARGUMENT, "too many segments");
  if (src_len >= (1ull << 56)) return set_error(ctx, ORCG_INVALID_ARGUMENT, "stream too long");
  if (java && positions_mode) return set_error(ctx, ORCG_INVALID_ARGUMENT, "Java rules take segment tables");
  const dim3 grid((unsigned)nsegs), block(kWave);
  const int sg = is_signed ? 1 : 0;
#define ORCG_LAUNCH1(T, P, J)                                                                     \
  hipLaunchKernelGGL((rlev2_decode_kernel<T, P, J>), grid, block, 0, ctx->stream, d_src, src_len, \
                     sg, d_segtab, nsegs, rows_per_group, value_begin, nvalues, (T*)d_dst,        \
                     ctx->d_err)
#define ORCG_LAUNCH(T, P)                                  \
  do {                                                     \
    if (java == 2) ORCG_LAUNCH1(T, false, 2);              \
    else if (java == 1) ORCG_LAUNCH1(T, false, 1);         \
    else ORCG_LAUNCH1(T, P, 0);                            \
  } while (0)
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
#undef ORCG_LAUNCH1
  return hip_check(ctx, hipGetLastError(), "rlev2_decode_kernel launch");
}

}  // namespace orcg

// A no-op launch that makes HIP load this file's code object (warm_modules).
namespace orcg {
namespace {
__global__ void warm_rlev2_walk_kernel() {}
}  // namespace
void warm_rlev2_walk(hipStream_t s) { hipLaunchKernelGGL(warm_rlev2_walk_kernel, dim3(1), dim3(64), 0, s); }
}  // namespace orcg
