// liborcgpu C ABI: contexts, the host run planner, host/device decode entry
// points and the stateful drop-in decoder for orc::RleDecoder
// (c++/src/RLE.hh:109-163). Kernels live in *_kernels.hip.
#include <stdio.h>
#include <string.h>

#include <linux/mempolicy.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <memory>
#include <string>
#include <vector>

#include "orcg_internal.hh"

namespace orcg {

const char* dev_error_message(uint32_t code) {
  switch (code) {
    case kErrBadRead: return "bad read in RleDecoderV2::readByte";
    case kErrPatchedPl0: return "Corrupt PATCHED_BASE encoded data (pl==0)!";
    case kErrPatchedWidth: return "Corrupt PATCHED_BASE encoded data (patchBitSize + pgw > 64)!";
    case kErrDeltaLength: return "Illegal run length for delta encoding: 1";
    case kErrBadSegment: return "Stream position is not at a run boundary";
    case kErrByteBadRead: return "bad read in nextBuffer";
    case kErrDictIndex: return "Entry index out of range in StringDictionaryColumn";
    case kErrV1BadRead: return "bad read in readByte";
    case kErrDecimalScale: return "Decimal scale out of range";
    case kErrHive11Overflow: return "Hive 0.11 decimal was more than 38 digits.";
    case kErrJavaCorrupt:
      return "Corruption in ORC data encountered. To skip reading corrupted data, set "
             "hive.exec.orc.skip.corrupt.data to true";
    case kErrJavaPatchIndex: return "Index 0 out of bounds for length 0";
  }
  return "unknown device error";
}

int dev_error_status(uint32_t code) {
  return code == kErrBadSegment ? ORCG_INVALID_ARGUMENT : ORCG_PARSE_ERROR;
}

int set_error(Ctx* ctx, int status, const std::string& msg) {
  if (ctx) ctx->last_error = msg;
  return status;
}

int hip_check(Ctx* ctx, hipError_t e, const char* what) {
  if (e == hipSuccess) return ORCG_OK;
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return set_error(ctx, e == hipErrorOutOfMemory ? ORCG_OUT_OF_MEMORY : ORCG_DEVICE_ERROR, m);
}

int scratch(Ctx* ctx, int slot, size_t bytes, void** out) {
  if (bytes == 0) bytes = 16;
  if (ctx->scratch_cap[slot] < bytes) {
    if (ctx->d_scratch[slot]) {
      hipStreamSynchronize(ctx->stream);
      hipFree(ctx->d_scratch[slot]);
      ctx->d_scratch[slot] = nullptr;
      ctx->scratch_cap[slot] = 0;
    }
    size_t cap = std::max(bytes, (size_t)1 << 20);
    int rc = hip_check(ctx, hipMalloc(&ctx->d_scratch[slot], cap), "hipMalloc scratch");
    if (rc) return rc;
    ctx->scratch_cap[slot] = cap;
  }
  *out = ctx->d_scratch[slot];
  return ORCG_OK;
}

// ------------------------------------------------------------------------
// Host run walk. Header arithmetic identical to the device walk (and to
// RleDecoderV2::next*, c++/src/RleDecoderV2.cc:184-435); only header bytes
// are read. Errors are recorded with the first value index of the bad run.
// ------------------------------------------------------------------------
namespace {

const uint8_t kFbs[32] = {1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16,
                          17, 18, 19, 20, 21, 22, 23, 24, 26, 28, 30, 32, 40, 48, 56, 64};

uint32_t closest_fixed_bits(uint32_t n) {
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

// Parses the run at `pos`. Returns kErrNone and sets run_len (values) and
// run_end (bytes), or a DevErr.
uint32_t parse_run(const uint8_t* s, uint64_t len, uint64_t pos, uint64_t* run_len,
                   uint64_t* run_end, int java = 0) {
  const uint32_t fb = s[pos];
  const uint32_t kind = fb >> 6;
  if (kind == 0) {
    const uint32_t nb = ((fb >> 3) & 7) + 1;
    *run_len = (fb & 7) + 3;
    *run_end = pos + 1 + nb;
    return *run_end > len ? kErrBadRead : kErrNone;
  }
  if (pos + 2 > len) return kErrBadRead;
  uint64_t L = ((uint64_t)(fb & 1) << 8 | s[pos + 1]) + 1;
  *run_len = L;
  if (kind == 1 || kind == 2) {
    const uint32_t W = kFbs[(fb >> 1) & 0x1f];
    uint64_t data = pos + 2;
    uint32_t cfb = 0, pl = 0;
    if (kind == 2) {
      if (pos + 4 > len) return kErrBadRead;
      const uint32_t third = s[pos + 2], fourth = s[pos + 3];
      const uint32_t bw = (third >> 5) + 1;
      const uint32_t pbs = kFbs[third & 0x1f];
      const uint32_t pgw = (fourth >> 5) + 1;
      pl = fourth & 0x1f;
      if (pl == 0 && !java) return kErrPatchedPl0;
      if (pos + 4 + bw > len) return kErrBadRead;
      data = pos + 4 + bw;
      if (data + (W * L + 7) / 8 > len) return kErrBadRead;
      // Java (RunLengthIntegerReaderV2.java:196-202): with skipCorrupt the
      // list is read at getClosestFixedBits(pw + pgw) bits an entry
      if (pbs + pgw > 64 && java != 2) return java ? kErrJavaCorrupt : kErrPatchedWidth;
      cfb = closest_fixed_bits(pbs + pgw);
    }
    *run_end = data + (W * L + 7) / 8 + ((uint64_t)cfb * pl + 7) / 8;
    if (*run_end > len) return kErrBadRead;
    return kind == 2 && pl == 0 ? kErrJavaPatchIndex : kErrNone;  // Java: unpackedPatch[0] of an empty list
  }
  const uint32_t fbo = (fb >> 1) & 0x1f;
  const uint32_t W = fbo ? kFbs[fbo] : 0;
  uint64_t q = pos + 2;
  for (int k = 0; k < 2; ++k) {
    uint32_t b;
    do {
      if (q >= len) return kErrBadRead;
      b = s[q++];
    } while (b >= 0x80);
  }
  if (W != 0 && L < 2) {
    if (!java) return kErrDeltaLength;
    *run_len = L = 2;  // Java (:125-145): the first value, first + deltaBase, no deltas
  }
  *run_end = q + (W ? ((uint64_t)W * (L - 2) + 7) / 8 : 0);
  return *run_end > len ? kErrBadRead : kErrNone;
}

}  // namespace
// Page-locked host memory. Large buffers (the reader's staging, the row
// reader's slabs) are anonymous mappings advised to transparent huge pages,
// faulted in by several threads and then registered with HIP: measured on the
// MI355X hosts (scripts/probes/pin_probe.cpp), 256 MB costs ~15 ms to fault +
// 0.5 ms to register this way against ~48 ms for hipHostMalloc (4 KB pages
// pinned one by one), at the same D2H rate (57 GB/s). Small buffers, or a
// failed registration, use hipHostMalloc.
namespace {
std::mutex g_pin_mu;
std::unordered_map<void*, size_t> g_pin_maps;  // registered mappings -> length
constexpr size_t kHuge = size_t(2) << 20;
}  // namespace

int current_numa_node() {
  unsigned cpu = 0, node = 0;
  return getcpu(&cpu, &node) == 0 ? (int)node : -1;
}

void* pinned_alloc(size_t bytes, int node) {
  if (bytes == 0) bytes = 1;
  if (bytes >= (size_t(8) << 20)) {
    const size_t len = (bytes + kHuge - 1) & ~(kHuge - 1);
    void* m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m != MAP_FAILED) {
      (void)madvise(m, len, MADV_HUGEPAGE);
      if (node >= 0 && node < 64) {  // before the faults below place the pages
        const unsigned long mask = 1ul << node;
        (void)syscall(SYS_mbind, m, len, MPOL_PREFERRED, &mask, 64ul, 0u);
      }
      // fault the pages in on a few threads (one write per 4 KB page: a huge
      // page faults whole on its first write, a small one each)
      const size_t pages = len >> 12;
      const unsigned nt = (unsigned)std::min<size_t>(8, std::max<size_t>(1, len / (size_t(32) << 20)));
      std::vector<std::thread> ts;
      for (unsigned t = 0; t < nt; ++t)
        ts.emplace_back([=] {
          volatile char* b = (volatile char*)m;
          for (size_t pg = pages * t / nt; pg < pages * (t + 1) / nt; ++pg) b[pg << 12] = 0;
        });
      for (auto& th : ts) th.join();
      if (hipHostRegister(m, len, hipHostRegisterDefault) == hipSuccess) {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        g_pin_maps[m] = len;
        return m;
      }
      (void)hipGetLastError();
      munmap(m, len);
    }
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void pinned_free(void* p) {
  if (!p) return;
  size_t len = 0;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pin_maps.find(p);
    if (it != g_pin_maps.end()) {
      len = it->second;
      g_pin_maps.erase(it);
    }
  }
  if (len) {
    (void)hipHostUnregister(p);
    munmap(p, len);
  } else {
    (void)hipHostFree(p);
  }
}

// ORCG_DEBUG: comma-separated topics (alloc, stale, rowreader, defer, jobs)
// whose diagnostics go to stderr
bool debug_on(const char* topic) {
  static const std::string topics = [] {
    const char* e = getenv("ORCG_DEBUG");
    return std::string(",") + (e ? e : "") + ",";
  }();
  return topics.find(std::string(",") + topic + ",") != std::string::npos;
}

void debug_stale(const char* where) {
  if (!debug_on("stale")) return;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fprintf(stderr, "orcg: pending HIP error at %s: %s\n", where, hipGetErrorString(e));
}

unsigned side_lanes() {
  static const unsigned n = [] {
    const char* e = getenv("ORCG_LANES");
    const int v = e ? atoi(e) : 4;
    return (unsigned)std::max(1, std::min(v, 16));
  }();
  return n;
}

Ctx* ctx_lane(Ctx* base, size_t k) {
  if (!base->ev_fork && hipEventCreateWithFlags(&base->ev_fork, hipEventDisableTiming) != hipSuccess) {
    base->ev_fork = nullptr;
    return nullptr;
  }
  while (base->lanes.size() <= k) {
    orcg_ctx* l = nullptr;
    hipEvent_t e = nullptr;
    if (orcg_ctx_create(base->device, &l) != ORCG_OK) return nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      orcg_ctx_destroy(l);
      return nullptr;
    }
    base->lanes.push_back(l);
    base->ev_join.push_back(e);
  }
  Ctx* l = base->lanes[k];
  l->rlev2_variant = base->rlev2_variant;
  if (!l->num_cus) l->num_cus = base->num_cus;
  return l;
}
}  // namespace orcg

using namespace orcg;


namespace orcg {
uint32_t host_parse_run(const uint8_t* s, uint64_t len, uint64_t pos, uint64_t* run_len, uint64_t* run_end) {
  return parse_run(s, len, pos, run_len, run_end);
}
}  // namespace orcg

orcg_rlev2_plan* make_plan(const uint8_t* src, uint64_t len, uint64_t max_bytes,
                                  uint64_t max_values, int java) {
  auto* p = new orcg_rlev2_plan();
  uint64_t pos = 0, vi = 0;
  uint64_t seg_b = 0, seg_v = 0;
  bool open = false;
  while (pos < len) {
    uint64_t L = 0, end = 0;
    const uint32_t e = parse_run(src, len, pos, &L, &end, java);
    if (e != kErrNone) {
      p->err = e;
      p->err_at = vi;
      break;
    }
    if (!open || pos - seg_b >= max_bytes || vi - seg_v >= max_values) {
      p->segs.push_back({pos, vi});
      seg_b = pos;
      seg_v = vi;
      open = true;
    }
    pos = end;
    vi += L;
  }
  p->values = vi;
  return p;
}

extern "C" {

const char* orcg_version(void) { return "orcg 0.1.0 (gfx950)"; }

int orcg_host_register(void* p, uint64_t bytes) {
  if (!p || !bytes) return ORCG_INVALID_ARGUMENT;
  return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? ORCG_OK : ORCG_DEVICE_ERROR;
}

int orcg_host_unregister(void* p) {
  if (!p) return ORCG_INVALID_ARGUMENT;
  return hipHostUnregister(p) == hipSuccess ? ORCG_OK : ORCG_DEVICE_ERROR;
}

int orcg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int orcg_ctx_create(int device, orcg_ctx** out) {
  if (!out) return ORCG_INVALID_ARGUMENT;
  *out = nullptr;
  int n = orcg_device_count();
  if (device < 0 || device >= n) return ORCG_DEVICE_ERROR;
  auto* c = new orcg_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_err, sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(c->d_err, 0xff, sizeof(unsigned long long)) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    delete c;
    return ORCG_DEVICE_ERROR;
  }
  c->stream = c->own_stream;
  // the process's first context on a device loads every kernel file's code
  // object now (orcg_internal.hh warm_*)
  static std::mutex warm_mu;
  static std::vector<int> warmed;
  static const bool warm = [] {
    const char* e = getenv("ORCG_WARMUP");
    return !e || atoi(e) != 0;
  }();
  if (warm) {
    std::lock_guard<std::mutex> lk(warm_mu);
    if (std::find(warmed.begin(), warmed.end(), device) == warmed.end()) {
      orcg::warm_rlev2_walk(c->stream);
      orcg::warm_rlev2_tiled(c->stream);
      orcg::warm_rlev2_expand(c->stream);
      orcg::warm_byterle(c->stream);
      orcg::warm_columns(c->stream);
      orcg::warm_rlev1(c->stream);
      orcg::warm_decimal(c->stream);
      // and the copy paths: the process's first host <-> device copies cost
      // ~10-100 ms of runtime setup (scripts/probes/pin_first_dma.py: a
      // fresh pinned buffer copies at full rate afterwards)
      void* h = nullptr;
      void* dv = nullptr;
      if (hipHostMalloc(&h, 4096, hipHostMallocDefault) == hipSuccess && hipMalloc(&dv, 4096) == hipSuccess) {
        (void)hipMemcpyAsync(dv, h, 4096, hipMemcpyHostToDevice, c->stream);
        (void)hipMemcpyAsync(h, dv, 4096, hipMemcpyDeviceToHost, c->stream);
        (void)hipStreamSynchronize(c->stream);
      }
      (void)hipGetLastError();
      if (dv) (void)hipFree(dv);
      if (h) (void)hipHostFree(h);
      // large copies take the DMA engines (small ones a blit kernel): one
      // each way from registered pinned memory (ORCG_WARMUP_MB, default 16)
      static const size_t big = [] {
        const char* e = getenv("ORCG_WARMUP_MB");
        return (size_t)(e ? std::max(0, atoi(e)) : 16) << 20;
      }();
      void* hb = big ? pinned_alloc(big) : nullptr;
      void* db = nullptr;
      if (hb && hipMalloc(&db, big) == hipSuccess) {
        (void)hipMemcpyAsync(db, hb, big, hipMemcpyHostToDevice, c->stream);
        (void)hipMemcpyAsync(hb, db, big, hipMemcpyDeviceToHost, c->stream);
        (void)hipStreamSynchronize(c->stream);
      }
      (void)hipGetLastError();
      if (db) (void)hipFree(db);
      if (hb) pinned_free(hb);
      if (hipStreamSynchronize(c->stream) != hipSuccess) {
        (void)hipGetLastError();
        orcg_ctx_destroy(c);
        return ORCG_DEVICE_ERROR;
      }
      // only a warm-up that completed marks the device (a failed one is
      // retried by the next context)
      warmed.push_back(device);
    }
  }
  *out = c;
  return ORCG_OK;
}

void* orcg_host_alloc(uint64_t bytes) { return orcg::pinned_alloc(bytes); }

void orcg_host_free(void* p) { orcg::pinned_free(p); }

void orcg_ctx_destroy(orcg_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  for (Ctx* l : c->lanes) orcg_ctx_destroy(static_cast<orcg_ctx*>(l));
  if (c->ev_fork) hipEventDestroy(c->ev_fork);
  for (hipEvent_t e : c->ev_join)
    if (e) hipEventDestroy(e);
  if (c->stream) hipStreamSynchronize(c->stream);
  for (int i = 0; i < 8; ++i)
    if (c->d_scratch[i]) hipFree(c->d_scratch[i]);
  if (c->h_pinned) hipHostFree(c->h_pinned);
  if (c->d_err) hipFree(c->d_err);
  if (c->d_defer) hipFree(c->d_defer);
  if (c->d_lb) hipFree(c->d_lb);
  if (c->d_rtab) hipFree(c->d_rtab);
  if (c->d_rhdr) hipFree(c->d_rhdr);
  if (c->d_jobs) hipFree(c->d_jobs);
  if (c->h_jobs) hipHostFree(c->h_jobs);
  if (c->own_stream) hipStreamDestroy(c->own_stream);
  delete c;
}

int orcg_ctx_set_stream(orcg_ctx* c, void* s) {
  if (!c) return ORCG_INVALID_ARGUMENT;
  c->stream = s ? (hipStream_t)s : c->own_stream;
  return ORCG_OK;
}

int orcg_rlev2_variants(int* out, int cap) {
  int n = 0;
  for (int v = 0; v <= kMaxRlev2Variant; ++v)
    if (rlev2_variant_valid(v)) {
      if (out && n < cap) out[n] = v;
      ++n;
    }
  return n;
}

int orcg_ctx_set_rlev2_variant(orcg_ctx* c, int v) {
  // 0 tiled (default), 1 wave-walk; the others pin one tiled instance
  // (rlev2_tiled.hip launch_rlev2_tiled, rlev2_variant_valid)
  if (!c || !rlev2_variant_valid(v)) return ORCG_INVALID_ARGUMENT;
  c->rlev2_variant = v;
  return ORCG_OK;
}

void* orcg_ctx_stream(orcg_ctx* c) { return c ? (void*)c->stream : nullptr; }

const char* orcg_ctx_last_error(const orcg_ctx* c) { return c ? c->last_error.c_str() : ""; }

int orcg_ctx_synchronize(orcg_ctx* c) { return c ? sync_ctx(c) : ORCG_INVALID_ARGUMENT; }

}  // extern "C"

namespace orcg {
int sync_ctx(Ctx* c) {
  (void)hipSetDevice(c->device);
  int rc = hip_check(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  if (rc) return rc;
  unsigned long long rec = kNoError;
  rc = hip_check(c, hipMemcpy(&rec, c->d_err, sizeof rec, hipMemcpyDeviceToHost), "read error record");
  if (rc) return rc;
  if (rec == kNoError) return ORCG_OK;
  const uint32_t code = (uint32_t)(rec & 0xff);
  c->last_error_value = rec >> 8;
  hipMemset(c->d_err, 0xff, sizeof rec);
  return set_error(c, dev_error_status(code), dev_error_message(code));
}
}  // namespace orcg

extern "C" {

// ---- plan ----------------------------------------------------------------
int orcg_rlev2_plan_create(const uint8_t* src, uint64_t len, uint64_t max_bytes, uint64_t max_values,
                           orcg_rlev2_plan** out) {
  if (!out || (len && !src)) return ORCG_INVALID_ARGUMENT;
  *out = make_plan(src, len, max_bytes ? max_bytes : (16u << 10), max_values ? max_values : 8192);
  return ORCG_OK;
}
void orcg_rlev2_plan_destroy(orcg_rlev2_plan* p) { delete p; }
uint64_t orcg_rlev2_plan_values(const orcg_rlev2_plan* p) { return p ? p->values : 0; }
uint64_t orcg_rlev2_plan_segments(const orcg_rlev2_plan* p, const orcg_segment** segs) {
  if (!p) return 0;
  if (segs) *segs = p->segs.data();
  return p->segs.size();
}
int orcg_rlev2_plan_error(const orcg_rlev2_plan* p, uint64_t* at, const char** msg) {
  if (!p || p->err == kErrNone) return ORCG_OK;
  if (at) *at = p->err_at;
  if (msg) *msg = dev_error_message(p->err);
  return dev_error_status(p->err);
}

// ---- device entry points ---------------------------------------------------
int orcg_rlev2_decode_device(orcg_ctx* c, const uint8_t* d_src, uint64_t src_len, int is_signed,
                             const orcg_segment* d_segs, uint64_t nsegs, uint64_t value_begin,
                             uint64_t nvalues, void* d_dst, int dst_bytes) {
  if (!c || (nsegs && (!d_src || !d_segs)) || (nvalues && !d_dst)) return ORCG_INVALID_ARGUMENT;
  hipSetDevice(c->device);
  return launch_rlev2(c, d_src, src_len, is_signed, (const uint64_t*)d_segs, nsegs, false, 0,
                             value_begin, nvalues, d_dst, dst_bytes);
}

int orcg_rlev2_decode_positions_device(orcg_ctx* c, const uint8_t* d_src, uint64_t src_len,
                                       int is_signed, const uint64_t* d_positions, uint64_t ngroups,
                                       uint64_t rows_per_group, uint64_t value_begin,
                                       uint64_t nvalues, void* d_dst, int dst_bytes) {
  if (!c || (ngroups && (!d_src || !d_positions)) || (nvalues && !d_dst) || rows_per_group == 0)
    return ORCG_INVALID_ARGUMENT;
  hipSetDevice(c->device);
  return launch_rlev2(c, d_src, src_len, is_signed, d_positions, ngroups, true,
                             rows_per_group, value_begin, nvalues, d_dst, dst_bytes);
}

}  // extern "C"

// ---- host-buffer decode ----------------------------------------------------
// Decodes the first `count` values of a host stream into host `out` (dense).
int decode_host_dense(Ctx* c, const uint8_t* src, uint64_t len, int is_signed,
                             const orcg_rlev2_plan* plan, uint64_t count, void* out, int width, int java) {
  if (count == 0) return ORCG_OK;
  hipSetDevice(c->device);
  void *d_src, *d_seg, *d_out;
  int rc = scratch(c, 0, len + 16, &d_src);
  if (!rc) rc = scratch(c, 1, plan->segs.size() * sizeof(orcg_segment), &d_seg);
  if (!rc) rc = scratch(c, 2, count * (size_t)width, &d_out);
  if (rc) return rc;
  rc = hip_check(c, hipMemcpyAsync(d_src, src, len, hipMemcpyHostToDevice, c->stream), "H2D stream");
  if (!rc)
    rc = hip_check(c, hipMemcpyAsync(d_seg, plan->segs.data(), plan->segs.size() * sizeof(orcg_segment),
                                     hipMemcpyHostToDevice, c->stream),
                   "H2D segments");
  if (!rc)
    rc = java ? launch_rlev2_decode(c, (const uint8_t*)d_src, len, is_signed, (const uint64_t*)d_seg,
                                    plan->segs.size(), false, 0, 0, count, d_out, width, java)
              : launch_rlev2(c, (const uint8_t*)d_src, len, is_signed, (const uint64_t*)d_seg,
                             plan->segs.size(), false, 0, 0, count, d_out, width);
  if (!rc)
    rc = hip_check(c, hipMemcpyAsync(out, d_out, count * (size_t)width, hipMemcpyDeviceToHost, c->stream),
                   "D2H values");
  if (!rc) rc = sync_ctx(c);
  return rc;
}

template <typename T>
static int decode_host(orcg_ctx* c, const uint8_t* src, uint64_t len, int is_signed,
                       const char* not_null, uint64_t n, T* dst) {
  if (!c || (len && !src) || (n && !dst)) return ORCG_INVALID_ARGUMENT;
  uint64_t k = n;
  if (not_null) {
    k = 0;
    for (uint64_t i = 0; i < n; ++i) k += not_null[i] ? 1 : 0;
  }
  std::unique_ptr<orcg_rlev2_plan> plan(make_plan(src, len, 16u << 10, 8192));
  if (k > plan->values) {
    const uint32_t e = plan->err != kErrNone ? plan->err : (uint32_t)kErrBadRead;
    return set_error(c, dev_error_status(e), dev_error_message(e));
  }
  if (!not_null) return decode_host_dense(c, src, len, is_signed, plan.get(), k, dst, sizeof(T));
  std::vector<T> dense(k);
  int rc = decode_host_dense(c, src, len, is_signed, plan.get(), k, dense.data(), sizeof(T));
  if (rc) return rc;
  uint64_t j = 0;
  for (uint64_t i = 0; i < n; ++i)
    if (not_null[i]) dst[i] = dense[j++];
  return ORCG_OK;
}

extern "C" {
int orcg_rlev2_decode_i64(orcg_ctx* c, const uint8_t* s, uint64_t l, int sg, const char* nn, uint64_t n,
                          int64_t* d) {
  return decode_host(c, s, l, sg, nn, n, d);
}
int orcg_rlev2_decode_i32(orcg_ctx* c, const uint8_t* s, uint64_t l, int sg, const char* nn, uint64_t n,
                          int32_t* d) {
  return decode_host(c, s, l, sg, nn, n, d);
}
int orcg_rlev2_decode_i16(orcg_ctx* c, const uint8_t* s, uint64_t l, int sg, const char* nn, uint64_t n,
                          int16_t* d) {
  return decode_host(c, s, l, sg, nn, n, d);
}
}  // extern "C"

// ---- stateful decoder ----------------------------------------------------------
struct orcg_rle_decoder {
  Ctx* ctx = nullptr;
  int is_signed = 0;
  int java = 0;  // Java's RunLengthIntegerReaderV2 rules (launch_rlev2_decode `java`)
  std::vector<uint8_t> src;
  std::unique_ptr<orcg_rlev2_plan> plan;
  uint64_t origin = 0;          // byte offset the decoded values start at
  std::vector<int64_t> values;  // dense decoded values from `origin`
  uint64_t cursor = 0;
  std::string last_error;

  int fail(int status, const std::string& m) {
    last_error = m;
    return status;
  }
  // (Re)decode the stream suffix starting at byte `from`.
  int load_from(uint64_t from) {
    origin = from;
    cursor = 0;
    const uint8_t* s = src.data() + from;
    const uint64_t len = src.size() - from;
    plan.reset(make_plan(s, len, 16u << 10, 8192, java));
    values.assign(plan->values, 0);
    int rc = decode_host_dense(ctx, s, len, is_signed, plan.get(), plan->values, values.data(), 8, java);
    if (rc) return fail(rc, ctx->last_error);
    return ORCG_OK;
  }
  int need(uint64_t k) {
    if (cursor + k <= values.size()) return ORCG_OK;
    const uint32_t e = plan->err != kErrNone ? plan->err : (uint32_t)kErrBadRead;
    return fail(dev_error_status(e), dev_error_message(e));
  }
  template <typename T>
  int next(T* data, uint64_t n, const char* nn) {
    if (n && !data) return fail(ORCG_INVALID_ARGUMENT, "null data");
    uint64_t k = n;
    if (nn) {
      k = 0;
      for (uint64_t i = 0; i < n; ++i) k += nn[i] ? 1 : 0;
    }
    // values up to the failing run are delivered before the error, like the
    // reference's partially filled batch
    const uint64_t avail = std::min<uint64_t>(k, values.size() - cursor);
    uint64_t j = 0;
    for (uint64_t i = 0; i < n && j < avail; ++i) {
      if (nn && !nn[i]) continue;
      data[i] = (T)values[cursor + j++];
    }
    if (avail < k) {
      cursor += avail;
      return need(k - avail);
    }
    cursor += k;
    return ORCG_OK;
  }
};

extern "C" {

int orcg_rle_decoder_create(orcg_ctx* c, const uint8_t* src, uint64_t len, int is_signed,
                            int version, orcg_rle_decoder** out) {
  if (!c || !out || (len && !src)) return ORCG_INVALID_ARGUMENT;
  *out = nullptr;
  if (version != 2)
    return set_error(c, ORCG_INVALID_ARGUMENT, "only RleVersion_2 streams decode on the GPU");
  auto* d = new orcg_rle_decoder();
  d->ctx = c;
  d->is_signed = is_signed;
  d->src.assign(src, src + len);
  int rc = d->load_from(0);
  if (rc) {
    c->last_error = d->last_error;
    delete d;
    return rc;
  }
  *out = d;
  return ORCG_OK;
}

// new RunLengthIntegerReaderV2(input, signed, skipCorrupt)
// (java/core/src/java/org/apache/orc/impl/RunLengthIntegerReaderV2.java:47-52)
int orcg_rle_decoder_create_java(orcg_ctx* c, const uint8_t* src, uint64_t len, int is_signed, int skip_corrupt,
                                 orcg_rle_decoder** out) {
  if (!c || !out || (len && !src)) return ORCG_INVALID_ARGUMENT;
  *out = nullptr;
  auto* d = new orcg_rle_decoder();
  d->ctx = c;
  d->is_signed = is_signed;
  d->java = skip_corrupt ? 2 : 1;
  d->src.assign(src, src + len);
  int rc = d->load_from(0);
  if (rc) {
    c->last_error = d->last_error;
    delete d;
    return rc;
  }
  *out = d;
  return ORCG_OK;
}

void orcg_rle_decoder_destroy(orcg_rle_decoder* d) { delete d; }

int orcg_rle_decoder_next_i64(orcg_rle_decoder* d, int64_t* data, uint64_t n, const char* nn) {
  return d ? d->next(data, n, nn) : ORCG_INVALID_ARGUMENT;
}
int orcg_rle_decoder_next_i32(orcg_rle_decoder* d, int32_t* data, uint64_t n, const char* nn) {
  return d ? d->next(data, n, nn) : ORCG_INVALID_ARGUMENT;
}
int orcg_rle_decoder_next_i16(orcg_rle_decoder* d, int16_t* data, uint64_t n, const char* nn) {
  return d ? d->next(data, n, nn) : ORCG_INVALID_ARGUMENT;
}

int orcg_rle_decoder_skip(orcg_rle_decoder* d, uint64_t n) {
  if (!d) return ORCG_INVALID_ARGUMENT;
  const uint64_t avail = std::min<uint64_t>(n, d->values.size() - d->cursor);
  d->cursor += avail;
  return avail < n ? d->need(n - avail) : ORCG_OK;
}

int orcg_rle_decoder_seek(orcg_rle_decoder* d, const uint64_t* pos, uint64_t npos) {
  if (!d) return ORCG_INVALID_ARGUMENT;
  if (!pos || npos < 2) return d->fail(ORCG_INVALID_ARGUMENT, "uncompressed RLE position needs 2 values");
  const uint64_t byte = pos[0], skip = pos[1];
  if (byte > d->src.size()) return d->fail(ORCG_INVALID_ARGUMENT, "Seek past end of stream");
  // Is `byte` a run start of the current decoding? Walk run headers from the
  // nearest segment cut (host bytes; cheap).
  bool found = false;
  uint64_t vi = 0;
  if (byte >= d->origin) {
    const uint64_t rel = byte - d->origin;
    const auto& segs = d->plan->segs;
    auto it = std::upper_bound(segs.begin(), segs.end(), rel,
                               [](uint64_t b, const orcg_segment& s) { return b < s.byte_offset; });
    if (it != segs.begin()) {
      --it;
      uint64_t p = it->byte_offset, v = it->value_index;
      const uint8_t* s = d->src.data() + d->origin;
      const uint64_t len = d->src.size() - d->origin;
      while (p < rel && p < len) {
        uint64_t L, end;
        if (parse_run(s, len, p, &L, &end) != kErrNone) break;
        p = end;
        v += L;
      }
      if (p == rel && v <= d->values.size()) {
        found = true;
        vi = v;
      }
    }
  }
  if (found) {
    d->cursor = vi;
  } else {
    int rc = d->load_from(byte);
    if (rc) return rc;
  }
  return orcg_rle_decoder_skip(d, skip);
}

int orcg_rle_decoder_next_vector_java(orcg_rle_decoder* d, int64_t* vector, const uint8_t* is_null,
                                      uint64_t n, int* is_repeating) {
  if (!d || (n && !vector) || !is_repeating) return ORCG_INVALID_ARGUMENT;
  // RunLengthIntegerReaderV2.nextVector (RunLengthIntegerReaderV2.java:371-396)
  if (*is_repeating && is_null && n > 0 && is_null[0]) return ORCG_OK;
  if (is_null) {
    std::vector<char> nn(n);
    for (uint64_t i = 0; i < n; ++i) nn[i] = is_null[i] ? 0 : 1;
    int rc = d->next(vector, n, nn.data());
    if (rc) return rc;
    for (uint64_t i = 0; i < n; ++i)
      if (is_null[i]) vector[i] = 1;
  } else {
    int rc = d->next(vector, n, nullptr);
    if (rc) return rc;
  }
  bool rep = true;
  for (uint64_t i = 0; i < n; ++i) {
    if (rep && i > 0 &&
        (vector[0] != vector[i] || (is_null ? is_null[0] != is_null[i] : false)))
      rep = false;
  }
  *is_repeating = rep ? 1 : 0;
  return ORCG_OK;
}

int orcg_rle_decoder_next_vector_java_int(orcg_rle_decoder* d, int32_t* vector, const uint8_t* is_null, uint64_t n,
                                          int is_repeating) {
  if (!d || (n && !vector)) return ORCG_INVALID_ARGUMENT;
  // RunLengthIntegerReaderV2.nextVector(ColumnVector, int[], int)
  // (RunLengthIntegerReaderV2.java:399-411): (int) narrowing, null slots 1,
  // an all-null repeating vector is left alone, isRepeating is not computed
  if (!is_null) return d->next(vector, n, nullptr);
  if (is_repeating && n > 0 && is_null[0]) return ORCG_OK;
  std::vector<char> nn(n);
  for (uint64_t i = 0; i < n; ++i) nn[i] = is_null[i] ? 0 : 1;
  const int rc = d->next(vector, n, nn.data());
  if (rc) return rc;
  for (uint64_t i = 0; i < n; ++i)
    if (is_null[i]) vector[i] = 1;
  return ORCG_OK;
}

const char* orcg_rle_decoder_last_error(const orcg_rle_decoder* d) {
  return d ? d->last_error.c_str() : "";
}

}  // extern "C"

// Test hook (tests/test_gpu_scan.py): the reader's exclusive scan of int64
// values, d_out[0..n] (n + 1 entries), on the context's stream.
extern "C" int orcg_debug_exclusive_scan(orcg_ctx* c, const int64_t* d_in, uint64_t n, int64_t* d_out) {
  if (!c || (n && !d_in) || !d_out) return ORCG_INVALID_ARGUMENT;
  hipSetDevice(c->device);
  return orcg::launch_exclusive_scan(c, d_in, n, d_out);
}

// Test hook: the next look-back launch on this context uses epoch `e` + 1
// (tests/test_gpu_scan.py runs across the 16-bit epoch wrap in a few launches).
extern "C" int orcg_debug_set_lb_epoch(orcg_ctx* c, uint32_t e) {
  if (!c || e > 0xffffu) return ORCG_INVALID_ARGUMENT;
  c->lb_epoch = e;
  return ORCG_OK;
}
