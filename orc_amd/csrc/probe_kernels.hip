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

}  // namespace
}  // namespace orcg

using namespace orcg;

extern "C" int orcg_probe_copy(orcg_ctx* c, const void* d_src, void* d_dst, uint64_t bytes, int mode) {
  if (!c || !d_src || !d_dst || (bytes % 1024) != 0 || mode < 0 || mode > 6) return ORCG_INVALID_ARGUMENT;
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
  }
  return hip_check(c, hipGetLastError(), "probe copy launch");
}
