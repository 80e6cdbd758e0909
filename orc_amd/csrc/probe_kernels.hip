// Roofline calibration probes: device copies of the same byte counts the
// decoder moves, in the access shapes it can use. bench.py / scripts report
// the decoder's bandwidth next to these (measured on the same box).
#include "orcg_internal.hh"

namespace orcg {
namespace {

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

// mode 0: 16 B/lane loads + 16 B/lane stores
// mode 1: 16 B/lane loads + 16 B/lane non-temporal stores
// mode 2:  8 B/lane loads +  8 B/lane non-temporal stores (the decoder's store shape)
// mode 3:  8 B/lane loads +  8 B/lane stores
template <int kMode>
__global__ __launch_bounds__(256) void copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   uint64_t bytes) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (kMode <= 1) {
    const u4* s = (const u4*)src;
    u4* d = (u4*)dst;
    for (uint64_t i = t0; i < bytes / 16; i += stride) {
      const u4 v = s[i];
      if constexpr (kMode == 0) d[i] = v;
      else __builtin_nontemporal_store(v, d + i);
    }
  } else {
    const u2* s = (const u2*)src;
    u2* d = (u2*)dst;
    for (uint64_t i = t0; i < bytes / 8; i += stride) {
      const u2 v = s[i];
      if constexpr (kMode == 2) __builtin_nontemporal_store(v, d + i);
      else d[i] = v;
    }
  }
}

// mode 4/5: every thread copies 4 consecutive 16-byte chunks (64 B), one
// pass over the buffer (no grid stride); 5 = non-temporal stores.
// mode 6: 8 B/lane, 4 independent loads in flight per thread, NT stores.
template <int kMode>
__global__ __launch_bounds__(256) void copy_wide_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                        uint64_t bytes) {
  if constexpr (kMode == 6) {
    const u2* s = (const u2*)src;
    u2* d = (u2*)dst;
    const uint64_t n = bytes / 8, stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
      const u2 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
      __builtin_nontemporal_store(a, d + i);
      __builtin_nontemporal_store(b, d + i + stride);
      __builtin_nontemporal_store(c, d + i + 2 * stride);
      __builtin_nontemporal_store(e, d + i + 3 * stride);
    }
    for (; i < n; i += stride) __builtin_nontemporal_store(s[i], d + i);
  } else {
    const u4* s = (const u4*)src;
    u4* d = (u4*)dst;
    const uint64_t n = bytes / 16;
    // wave-contiguous: a wave's 64 lanes cover 4 x 1 KB, lane-interleaved
    const uint64_t base = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * 4 + (threadIdx.x & 63u);
    u4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = base + 64 * k < n ? s[base + 64 * k] : u4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (base + 64 * k < n) {
        if constexpr (kMode == 5) __builtin_nontemporal_store(v[k], d + base + 64 * k);
        else d[base + 64 * k] = v[k];
      }
  }
}

// modes 7-9: the decoder's data movement without the decoding. Every
// workgroup owns an 80 KB segment and moves it through LDS windows filled
// by LDS-DMA (buffer_load ... lds, 16 B/lane), then drains each window with
// 8 B/lane non-temporal stores. 7: one 32 KB window, s_waitcnt vmcnt(0)
// (the tiled decoder's shape); 9: one 16 KB window; 8: two 16 KB windows,
// the fill of window k+1 in flight while window k drains, waiting only for
// the loads (vmcnt counts the later stores too, in issue order).
constexpr uint32_t kProbeSeg = 80u * 1024u;
template <int kWinKB, bool kDouble>
__global__ __launch_bounds__(256) void copy_lds_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       uint64_t bytes) {
  constexpr uint32_t kWin = kWinKB * 1024u;
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[kDouble ? 2 : 1][kWin];
  const int tid = (int)threadIdx.x, wave = tid / 64, lane = tid % 64;
  const uint64_t seg0 = (uint64_t)blockIdx.x * kProbeSeg;
  if (seg0 >= bytes) return;
  const uint32_t seg_len = (uint32_t)min((uint64_t)kProbeSeg, bytes - seg0);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(src + seg0), (short)0, (int)seg_len, 0x00020000);
  u2* out = (u2*)(dst + seg0);
  auto fill = [&](uint8_t* buf, uint32_t w, uint32_t len) {
    for (uint32_t off = wave * 1024u; off < len; off += 4 * 1024u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(buf + off), 16,
                                               w + off + lane * 16u, 0, 0, 0);
  };
  auto drain = [&](const uint8_t* buf, uint32_t w, uint32_t len) {
    for (uint32_t o = tid * 8u; o < len; o += 256u * 8u)
      __builtin_nontemporal_store(*(const u2*)(buf + o), out + (w + o) / 8);
  };
  const uint32_t nwin = (seg_len + kWin - 1) / kWin;
  if constexpr (!kDouble) {
    for (uint32_t k = 0; k < nwin; ++k) {
      const uint32_t w = k * kWin, len = min(kWin, seg_len - w);
      fill(s_buf[0], w, len);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      drain(s_buf[0], w, len);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    static_assert(kWin == 16384, "the vmcnt immediates assume 4 loads + 8 stores per lane per window");
    fill(s_buf[0], 0, min(kWin, seg_len));
    for (uint32_t k = 0; k < nwin; ++k) {
      const uint32_t w = k * kWin, len = min(kWin, seg_len - w);
      const bool has_next = k + 1 < nwin;
      const bool next_full = has_next && seg_len - (w + kWin) >= kWin;
      if (has_next) fill(s_buf[(k + 1) & 1], w + kWin, min(kWin, seg_len - w - kWin));
      // outstanding after fill(k): drain(k-1)'s 8 stores (k > 0) and fill(k+1)'s 4 loads
      if (!next_full) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (k == 0) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      __syncthreads();
      drain(s_buf[k & 1], w, len);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();  // buffer k&1 is refilled next iteration
    }
  }
}

// modes 10/11: as 9/7, but the window is filled through registers (every
// lane issues all its 16-byte global loads, then writes them to LDS).
template <int kWinKB>
__global__ __launch_bounds__(256) void copy_reg_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       uint64_t bytes) {
  constexpr uint32_t kWin = kWinKB * 1024u;
  constexpr int kPer = kWin / (256 * 16);
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[kWin];
  const int tid = (int)threadIdx.x;
  const uint64_t seg0 = (uint64_t)blockIdx.x * kProbeSeg;
  if (seg0 >= bytes) return;
  const uint32_t seg_len = (uint32_t)min((uint64_t)kProbeSeg, bytes - seg0);
  const u4* in = (const u4*)(src + seg0);
  u2* out = (u2*)(dst + seg0);
  for (uint32_t w = 0; w < seg_len; w += kWin) {
    const uint32_t len = min(kWin, seg_len - w);
    u4 v[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const uint32_t o = (uint32_t)(i * 256 + tid) * 16u;
      v[i] = o < len ? __builtin_nontemporal_load(in + (w + o) / 16) : u4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) *(u4*)(s_buf + (uint32_t)(i * 256 + tid) * 16u) = v[i];
    __syncthreads();
    for (uint32_t o = tid * 8u; o < len; o += 256u * 8u)
      __builtin_nontemporal_store(*(const u2*)(s_buf + o), out + (w + o) / 8);
    __syncthreads();
  }
}

}  // namespace
}  // namespace orcg

using namespace orcg;

// A/B build only (not declared in include/orcg.h): device copies in the
// decoder's access shapes, the roofline references of scripts/ab_rlev2.py.
extern "C" int orcg_probe_copy(orcg_ctx* c, const void* d_src, void* d_dst, uint64_t bytes, int mode) {
  if (!c || !d_src || !d_dst || (bytes % 1024) != 0 || mode < 0 || mode > 11) return ORCG_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  const unsigned grid = 256 * 16;  // 16 workgroups per CU, grid-stride
  switch (mode) {
    case 0: hipLaunchKernelGGL(copy_kernel<0>, dim3(grid), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes); break;
    case 1: hipLaunchKernelGGL(copy_kernel<1>, dim3(grid), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes); break;
    case 2: hipLaunchKernelGGL(copy_kernel<2>, dim3(grid), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes); break;
    case 3: hipLaunchKernelGGL(copy_kernel<3>, dim3(grid), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes); break;
    case 4:
    case 5: {
      const unsigned wide_grid = (unsigned)((bytes / 16 + 1023) / 1024);  // 256 threads x 4 chunks
      if (mode == 4) hipLaunchKernelGGL(copy_wide_kernel<4>, dim3(wide_grid), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes);
      else hipLaunchKernelGGL(copy_wide_kernel<5>, dim3(wide_grid), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes);
      break;
    }
    case 6: hipLaunchKernelGGL(copy_wide_kernel<6>, dim3(grid), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes); break;
    case 7:
    case 8:
    case 9: {
      const unsigned segs = (unsigned)((bytes + kProbeSeg - 1) / kProbeSeg);
      if (mode == 7) hipLaunchKernelGGL((copy_lds_kernel<32, false>), dim3(segs), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes);
      else if (mode == 8) hipLaunchKernelGGL((copy_lds_kernel<16, true>), dim3(segs), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes);
      else hipLaunchKernelGGL((copy_lds_kernel<16, false>), dim3(segs), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes);
      break;
    }
    case 10:
    case 11: {
      const unsigned segs = (unsigned)((bytes + kProbeSeg - 1) / kProbeSeg);
      if (mode == 10) hipLaunchKernelGGL((copy_reg_kernel<16>), dim3(segs), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes);
      else hipLaunchKernelGGL((copy_reg_kernel<32>), dim3(segs), dim3(256), 0, c->stream, (const uint8_t*)d_src, (uint8_t*)d_dst, bytes);
      break;
    }
  }
  return hip_check(c, hipGetLastError(), "probe copy launch");
}
