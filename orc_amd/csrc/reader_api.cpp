// File-level reader (include/orcg_reader.h): ORC tail -> stripe streams ->
// host decompression -> one H2D per stripe -> HIP decode of every selected
// column into device batches.
//
// Column semantics follow the reference's column readers
// (c++/src/ColumnReader.cc): ColumnReader::next's PRESENT handling with the
// parent's incoming mask (:81-104; a child's PRESENT stream has bits only for
// the parent's non-null rows), IntegerColumnReader (:225-258),
// BooleanColumnReader (:131-186), ByteColumnReader (:188-223),
// DoubleColumnReader (:359-450), StringDictionaryColumnReader (:509-607),
// StringDirectColumnReader (:615-793), StructColumnReader (:795-880),
// ListColumnReader / MapColumnReader (:882-1157). Encodings pick RLE v1 or v2
// (createRleDecoder, c++/src/RLE.cc:48-60 via ColumnReader.cc
// convertRleVersion).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>

#include "../../include/orcg_reader.h"
#include "orc_file.hh"
#include "orcg_internal.hh"

using namespace orcg;
using namespace orcg::file;

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

unsigned host_threads() {
  if (const char* e = getenv("ORCG_HOST_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return (unsigned)v;
  }
  const unsigned hc = std::thread::hardware_concurrency();
  return std::max(1u, std::min(16u, hc ? hc : 1u));
}

// work_bytes / bytes_per_thread caps the thread count: a thread costs tens
// of microseconds to start and join, so a small stripe's few KB of streams
// (configs[0]'s 5,000-row stripes: ~1 KB compressed each) run on the calling
// thread instead of paying for 16 threads three times per stripe.
template <typename F>
void parallel_for(size_t n, F&& f, uint64_t work_bytes = ~0ull, uint64_t bytes_per_thread = 1) {
  const uint64_t by_work = std::max<uint64_t>(1, work_bytes / std::max<uint64_t>(1, bytes_per_thread));
  const unsigned nt = (unsigned)std::min<uint64_t>(std::min<size_t>(host_threads(), n), by_work);
  if (nt <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> ts;
  for (unsigned t = 0; t < nt; ++t)
    ts.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& t : ts) t.join();
}

bool is_string_kind(uint32_t k) {
  return k == ORCG_TYPE_STRING || k == ORCG_TYPE_VARCHAR || k == ORCG_TYPE_CHAR || k == ORCG_TYPE_BINARY;
}
bool is_int_kind(uint32_t k) {
  return k == ORCG_TYPE_SHORT || k == ORCG_TYPE_INT || k == ORCG_TYPE_LONG || k == ORCG_TYPE_DATE;
}
// Zones whose rules are UTC: TIMESTAMP columns written in them decode with
// no adjustment against the default reader zone, GMT (ColumnReader.cc:333-345
// is a no-op; epoch 2015-01-01 00:00:00 UTC = 1420070400). Other writer
// zones need the IANA rules (Timezone.cc) and are not decoded.
bool utc_zone(const std::string& z) {
  static const char* kUtc[] = {"GMT", "UTC", "UCT", "Zulu", "Universal", "Greenwich", "GMT0", "GMT+0", "GMT-0",
                               "Etc/GMT", "Etc/UTC", "Etc/UCT", "Etc/Zulu", "Etc/Universal", "Etc/Greenwich",
                               "Etc/GMT0", "Etc/GMT+0", "Etc/GMT-0"};
  for (const char* u : kUtc)
    if (z == u) return true;
  return false;
}
constexpr int64_t kOrcEpochUtc = 1420070400;

// [off, off + len) lies inside [0, end), written so that no sum can wrap
// (offsets and lengths come from the file and are untrusted)
bool range_ok(uint64_t off, uint64_t len, uint64_t end) { return off <= end && len <= end - off; }

// Columns this reader decodes: every primitive, list / map / struct / union,
// decimals (Hive 0.11 precision-0 decimals at the forced scale), timestamps
// of UTC writers.
bool is_supported(const file::TypeInfo& t, const std::string& writer_tz) {
  const uint32_t k = t.kind;
  if (k == ORCG_TYPE_UNION) return true;
  if (k == ORCG_TYPE_DECIMAL) return true;
  if (k == ORCG_TYPE_TIMESTAMP) return utc_zone(writer_tz);
  if (k == ORCG_TYPE_TIMESTAMP_INSTANT) return true;
  return k <= ORCG_TYPE_CHAR || k == ORCG_TYPE_DATE || k == ORCG_TYPE_VARCHAR;
}

// Device arena of a decoded stripe: allocations bump through one hipMalloc'd
// chunk and are all released together when the slot decodes its next stripe,
// so a stripe's buffers are contiguous (the row reader copies them to the
// host in a few large D2H copies). A stripe that outgrows the chunk takes a
// new one; the next stripe then starts from one chunk of the combined size.
struct DevPool {
  int device = 0;
  std::vector<std::pair<uint8_t*, size_t>> chunks;  // the last is the active one
  size_t off = 0;                                   // bump offset in the active chunk
  size_t want = 0;                                  // bytes the last stripe used (all chunks)
  size_t used_now = 0;
  size_t hint = 0;                                  // the caller's estimate for a fresh slot
  ~DevPool() {
    for (auto& c : chunks) (void)hipFree(c.first);
  }
  void release_all() {
    if (chunks.size() > 1 || (!chunks.empty() && chunks.back().second < want)) {
      // consolidate: one chunk for the whole of the last stripe
      for (auto& c : chunks) (void)hipFree(c.first);
      chunks.clear();
    }
    want = std::max(want, used_now);
    off = 0;
    used_now = 0;
  }
  void* get(size_t bytes) {
    bytes = std::max<size_t>(256, (bytes + 255) & ~(size_t)255);
    used_now += bytes;
    if (chunks.empty() || off + bytes > chunks.back().second) {
      const size_t cap = std::max<size_t>({bytes + (bytes >> 2), want + (want >> 3), hint, size_t(1) << 20});
      uint8_t* p = nullptr;
      if (hipMalloc((void**)&p, cap) != hipSuccess) {
        (void)hipGetLastError();  // the failure must not stick to a later launch check
        if (hipMalloc((void**)&p, bytes) != hipSuccess) {
          (void)hipGetLastError();
          if (debug_on("alloc")) fprintf(stderr, "orcg: device allocation of %zu bytes failed\n", bytes);
          return nullptr;
        }
        chunks.push_back({p, bytes});
      } else {
        chunks.push_back({p, cap});
      }
      off = 0;
    }
    void* p = chunks.back().first + off;
    off += bytes;
    return p;
  }
};

struct StreamBuf {
  bool present = false;
  uint64_t host_off = 0;  // offset in staging (== device offset)
  uint64_t len = 0;       // decompressed bytes
  std::unique_ptr<orcg_rlev2_plan> plan;
  uint64_t seg_off = 0;   // offset of the plan's segment table in staging
  // row-index segmentation: per row group {byte offset, values to skip, bits
  // to skip} (int64 x 3) in staging at rg_off; no host plan
  bool pos = false;
  std::vector<int64_t> trip;
  uint64_t rg_off = 0;
};

struct Col {
  bool decoded = false;
  uint32_t kind = 0, encoding = 0;
  uint64_t n = 0;
  bool has_nulls = false;
  uint8_t* nn = nullptr;
  void* data = nullptr;
  int64_t* length = nullptr;
  int64_t* offsets = nullptr;
  uint8_t* blob = nullptr;
  uint64_t blob_len = 0;
  uint64_t dict_size = 0;  // ColumnEncoding.dictionarySize of this stripe
  bool supported = false;  // decoded by this reader (is_supported for this stripe's writer zone)
  int64_t* secondary = nullptr;  // TIMESTAMP nanoseconds
  uint8_t* tags = nullptr;       // UNION: child of each row (UnionVectorBatch::tags)
  int64_t* index = nullptr;      // dictionary strings: entry of each row (EncodedStringVectorBatch::index)
  int64_t* dict_offsets = nullptr;  // dictionary strings: dict_size + 1 entry offsets (StringDictionary)
  StreamBuf s[5];  // PRESENT, DATA, LENGTH, DICTIONARY_DATA, SECONDARY
  // has_nulls is provisional until the stripe's checks run: the non-null
  // count stayed on the device (orcg_reader::device_counts)
  bool nulls_deferred = false;
};

enum { kSlotPresent = 0, kSlotData = 1, kSlotLength = 2, kSlotDict = 3, kSlotSecondary = 4 };

int slot_of(uint32_t stream_kind) {
  switch (stream_kind) {
    case kPresent: return kSlotPresent;
    case kData: return kSlotData;
    case kLength: return kSlotLength;
    case kDictionaryData: return kSlotDict;
    case kSecondary: return kSlotSecondary;
  }
  return -1;
}

}  // namespace

// One stripe prepared on the host: stream bytes decompressed into pinned
// staging, run plans and their segment tables appended (no device work).
struct HostStage {
  uint64_t stripe = ~0ull;
  std::vector<Col> cols;  // streams (and, while decoding, the outputs)
  uint8_t* h = nullptr;   // pinned staging
  size_t cap = 0;
  uint64_t used = 0;
  int rc = ORCG_OK;
  std::string err;
  double t_parse = 0, t_decomp = 0, t_plan = 0;
  uint64_t ngroups = 0;    // row groups with row-index positions (0: host plans only)
  uint64_t n_pos = 0, n_plan = 0;  // RLE streams cut by the row index / by a host plan
  uint64_t n_chunks = 0;            // compression chunks inflated (ReaderMetrics::DecompressionCall)
  uint64_t n_io = 0;                // stream reads (ReaderMetrics::IOCount)
  double t_io = 0;                  // their blocking time: page-ins of the mapped stripe (IOBlockingLatencyUs)
  uint64_t io_sink = 0;
  uint64_t rows_off = 0;   // staging offset of int64 rows[g] = g * stride
  // room kept past the prepared bytes for the upload's tail (read-back block
  // and job arena, upload_tail_bytes): upload_and_decode never reallocates
  uint64_t slack = 0;
  ~HostStage() { pinned_free(h); }
  bool pinned_mapped = false;  // h is hipHostMalloc'd (the device can read it through the same pointer)
  bool ensure(uint64_t bytes, uint64_t keep) {
    if (bytes <= cap) return true;
    const uint64_t ncap = std::max<uint64_t>(bytes + (bytes >> 2), 1 << 20) + slack;
    uint8_t* nh = (uint8_t*)pinned_alloc(ncap);
    if (!nh) return false;
    if (h) {
      if (keep) memcpy(nh, h, keep);
      pinned_free(h);
    }
    h = nh;
    cap = ncap;
    pinned_mapped = ncap < (size_t(8) << 20);  // pinned_alloc's hipHostMalloc range
    return true;
  }
  int fail(int status, const std::string& m) {
    rc = status;
    err = m;
    return status;
  }
};

struct ColOut {
  bool decoded = false;
  uint32_t kind = 0, encoding = 0;
  uint64_t n = 0;
  bool has_nulls = false;
  const uint8_t* nn = nullptr;
  const void* data = nullptr;
  const int64_t* length = nullptr;
  const int64_t* offsets = nullptr;
  const uint8_t* blob = nullptr;
  uint64_t blob_len = 0;
  const int64_t* secondary = nullptr;
  const uint8_t* tags = nullptr;
  const int64_t* index = nullptr;
  const int64_t* dict_offsets = nullptr;
  uint64_t dict_size = 0;
};

// One decoded stripe in HBM: its device allocations and column views.
struct DevSlot {
  uint64_t stripe = ~0ull;
  DevPool pool;
  uint8_t* d_stage = nullptr;
  // the read-back block, uploaded initialised with the stripe and copied
  // back once after the decode: per column its error record, its PRESENT
  // decode's non-null count, then the summary slots (rb_alloc)
  uint64_t* d_rb = nullptr;
  unsigned long long* d_errs = nullptr;  // device error record per column (the kernels' atomicMin word)
  uint64_t* d_ones = nullptr;            // per column: non-null rows its PRESENT decode wrote
  std::vector<ColOut> out;
};

// A timed pair of events around a stripe's integer-RLE (kind 0) or byte-RLE
// (kind 1) launches (ReaderMetrics with metrics timing)
struct EvPair {
  hipEvent_t a, b;
  int kind;
};

struct orcg_reader {
  // serialises decodes: the reader's own reads and the row readers' prefetch
  // workers share its decode state (stages, batch tables, checks)
  std::mutex mu;
  // The reader's own options: its context (fixed at open), its column
  // selection and lazy-dictionary flag (changed under mu). Entry points that
  // run outside a decode (copy_to_host, is_selected, row reader creation)
  // read only these; a row reader's worker never writes them.
  Ctx* own_ctx = nullptr;
  std::vector<uint8_t> own_sel;  // per type id
  bool own_lazy = false;
  // The options of the decode in progress (valid under mu, set by Active):
  // the reader's own for its reads, a row reader's for that row reader's
  // prefetch decodes.
  Ctx* ctx = nullptr;
  std::vector<uint8_t> selected;
  bool lazy_dict = false;
  struct Active {
    orcg_reader* r;
    Active(orcg_reader* r_, Ctx* c, const std::vector<uint8_t>& sel, bool lazy) : r(r_) {
      r->ctx = c;
      r->selected = sel;
      r->lazy_dict = lazy;
    }
    ~Active() { r->ctx = nullptr; }
  };
  const uint8_t* file = nullptr;
  uint64_t file_len = 0;
  void* mapped = nullptr;
  PostScript ps;
  Footer footer;
  std::string last_error;
  HostStage stages[3];  // read_stripes: stripe i in stages[i % 3]
  bool decimal_as_long = false;  // PostScript version 1.9999 (UNSTABLE-PRE-2.0): Decimal64V2 columns (Reader.cc:1693-1699)
  int32_t hive11_scale = 6;  // RowReaderOptions::forcedScaleOnHive11Decimal (Reader.cc RowReaderOptionsPrivate: 6)
  bool hive11_throw = true;  // RowReaderOptions::throwOnHive11DecimalOverflow (default true)
  std::string software_version;  // orcg_reader_software_version's buffer
  std::vector<std::unique_ptr<DevSlot>> slots;  // results of the last read, in stripe order
  size_t nslots = 0;
  // decode() state: the host stage and device slot of the stripe being decoded
  HostStage* H = nullptr;
  DevSlot* D = nullptr;
  double timings[5] = {0, 0, 0, 0, 0};
  uint64_t stream_stats[2] = {0, 0};  // last read: RLE streams cut by the row index, by host plans
  // ReaderMetrics (Reader.hh:59-76) over the reader's life, in orcg_reader_metrics
  // order; atomics, as the reference's (the caller's thread counts next()
  // calls while a row reader's worker decodes)
  enum {
    kMReaderCall, kMReaderLatency, kMDecompressCall, kMDecompressLatency, kMDecodeCall, kMDecodeLatency,
    kMByteCall, kMByteLatency, kMIOCount, kMIOLatency, kMSelectedRG, kMEvaluatedRG, kMCacheHits, kMCacheMisses
  };
  std::atomic<uint64_t> metrics[14] = {};
  void madd(int i, uint64_t v) { metrics[i].fetch_add(v, std::memory_order_relaxed); }
  // DecodingLatencyUs / ByteDecodingLatencyUs from HIP events around the
  // integer-RLE and byte-RLE launches of a stripe (orcg_reader_set_metrics_timing;
  // off: DecodingLatencyUs is the stripe's device phase, ByteDecoding 0)
  bool metrics_timing = false;
  std::vector<hipEvent_t> ev_pool;
  hipEvent_t ev_get() {
    if (ev_pool.empty()) {
      hipEvent_t e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      return e;
    }
    hipEvent_t e = ev_pool.back();
    ev_pool.pop_back();
    return e;
  }
  // brackets the launches `f` enqueues on ctx->stream with a timed event pair
  template <class Fn>
  int timed(int kind, Fn&& f) {
    if (!metrics_timing) return f();
    hipEvent_t a = ev_get(), b = ev_get();
    if (a) (void)hipEventRecord(a, ctx->stream);
    const int rc = f();
    if (b) (void)hipEventRecord(b, ctx->stream);
    if (a && b) F->ev_used.push_back(EvPair{a, b, kind});
    else {
      if (a) ev_pool.push_back(a);
      if (b) ev_pool.push_back(b);
    }
    return rc;
  }
  // after the stripe's synchronisation: the pairs' times into the metrics
  void collect_event_times() {
    double us[2] = {0, 0};
    for (const EvPair& p : F->ev_used) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) us[p.kind] += ms * 1e3;
      ev_pool.push_back(p.a);
      ev_pool.push_back(p.b);
    }
    F->ev_used.clear();
    madd(kMDecodeLatency, (uint64_t)us[0]);
    madd(kMByteLatency, (uint64_t)us[1]);
  }
  uint64_t batched_streams = 0;       // last read: RLEv2 streams decoded by multi-stream launches
  uint64_t stage_bytes = 0;           // last read: bytes uploaded (decompressed streams + plans)

  // A stripe between its launches (issue) and its host checks (finish): its
  // stage and slot, the checks whose operands are device scalars (dictionary
  // blob size, varint counts, string bytes: their D2H copies are queued on
  // the stream and the checks run, in column order, after the stripe's one
  // synchronisation instead of a synchronisation each; the reference makes
  // them inline), the pinned read-back mirror, the inline failure, and the
  // event after the stripe's last copy. read_stripes keeps two in flight:
  // stripe i + 1 is issued before stripe i is finished.
  struct Flight {
    HostStage* hs = nullptr;
    DevSlot* ds = nullptr;
    uint64_t* h_defer = nullptr;
    size_t defer_cap = 0, defer_used = 0;
    // (column, check): run in column order with the columns' device errors
    std::vector<std::pair<uint32_t, std::function<int()>>> checks;
    // the read-back block's pinned mirror (valid after the stripe's copy)
    uint64_t* h_rb = nullptr;
    size_t h_rb_cap = 0, rb_words = 0, rb_used = 0;
    std::vector<EvPair> ev_used;  // metrics timing events
    hipEvent_t done = nullptr;    // recorded after the read-back copy
    // GPU-time split of the flight (timings[3] / [4]): before and after the
    // stripe's upload, and after its last decode launch
    hipEvent_t ev_up0 = nullptr, ev_up1 = nullptr, ev_dec = nullptr;
    bool ev_split = false;
    bool enqueued = false;        // done / the read-back copy belong to this issue
    int rc = ORCG_OK;             // the inline (host-detected) failure of the issue
    uint32_t err_col = 0;
    std::string err_msg;
    double t0 = 0, t1 = 0;
  };
  Flight flights[2];
  Flight* F = &flights[0];
  // the column decode() is working on, and the column of the first inline
  // (host-detected) failure of this stripe
  static constexpr uint32_t kNoCol = 0xffffffffu;
  uint32_t cur_col = kNoCol, err_col = kNoCol;
  int first_error(int inline_rc);
  // `count` words of the read-back block: the device address a kernel writes,
  // and (*host) where the host reads it after the stripe's synchronisation
  uint64_t* rb_alloc(size_t count, const uint64_t** host) {
    if (!D->d_rb || F->rb_used + count > F->rb_words) return nullptr;
    uint64_t* d = D->d_rb + F->rb_used;
    *host = F->h_rb + F->rb_used;
    F->rb_used += count;
    return d;
  }
  const uint64_t* defer(const void* d_src, size_t count) {
    // a value in the read-back block rides its one copy
    if (D && D->d_rb && (const uint64_t*)d_src >= D->d_rb && (const uint64_t*)d_src + count <= D->d_rb + F->rb_words)
      return F->h_rb + ((const uint64_t*)d_src - D->d_rb);
    if (F->defer_used + count > F->defer_cap) return nullptr;
    uint64_t* h = F->h_defer + F->defer_used;
    F->defer_used += count;
    if (hipMemcpyAsync(h, d_src, count * 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) return nullptr;
    return h;
  }

  // Mid-stripe reads the host must wait for (list / map totals, union
  // counts). Up to kPublishMax counts per stream: publish_kernel writes them
  // and a generation flag into coherent pinned memory and the host polls the
  // flag (launch_publish); more: 8-byte D2H copies into pinned memory (one
  // DMA each), then one stream synchronisation.
  uint64_t* h_pub = nullptr;  // kPubSlots slots of kPubStride words: counts, then the flag
  uint64_t* d_pub = nullptr;
  uint64_t pub_gen = 0;
  static constexpr size_t kPubSlots = 32, kPubStride = 32;
  // srcs[i] on stream lanes[i]; 1 = more counts on one stream than a slot
  // holds (the caller copies them instead)
  int poll_counts(const std::vector<Ctx*>& lanes, const std::vector<const void*>& srcs, uint64_t* out) {
    if (!h_pub) {
      void* h = nullptr;
      if (hipHostMalloc(&h, kPubSlots * kPubStride * 8, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        return 1;
      }
      void* d = nullptr;
      if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(h);
        return 1;
      }
      memset(h, 0, kPubSlots * kPubStride * 8);
      h_pub = (uint64_t*)h;
      d_pub = (uint64_t*)d;
    }
    std::vector<Ctx*> order;  // one slot per stream, in first-use order
    std::vector<PublishArgs> args;
    std::vector<std::vector<size_t>> where;
    for (size_t i = 0; i < srcs.size(); ++i) {
      size_t g = 0;
      while (g < order.size() && order[g] != lanes[i]) ++g;
      if (g == order.size()) {
        if (g == kPubSlots) return 1;
        order.push_back(lanes[i]);
        args.push_back(PublishArgs{});
        where.emplace_back();
      }
      if (args[g].n == kPublishMax) return 1;
      args[g].src[args[g].n++] = (const int64_t*)srcs[i];
      where[g].push_back(i);
    }
    const uint64_t gen = ++pub_gen;
    for (size_t g = 0; g < order.size(); ++g) {
      const int rc = launch_publish(order[g], args[g], d_pub + g * kPubStride, d_pub + g * kPubStride + kPublishMax,
                                    gen);
      if (rc) return fail(rc, order[g]->last_error);
    }
    for (size_t g = 0; g < order.size(); ++g) {
      const uint64_t* flag = h_pub + g * kPubStride + kPublishMax;
      const double t0 = now_s();
      for (uint32_t spin = 1; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != gen; ++spin) {
        if ((spin & 1023) != 0) continue;
        // a failed stream never sets the flag; a long wait gives the core back
        const hipError_t q = hipStreamQuery(order[g]->stream);
        if (q != hipSuccess && q != hipErrorNotReady) {
          const int rc = hip_check(order[g], q, "publish wait");
          return fail(rc, order[g]->last_error);
        }
        if (q == hipSuccess || now_s() - t0 > 2e-3) {
          const int rc = hip_check(order[g], hipStreamSynchronize(order[g]->stream), "hipStreamSynchronize");
          if (rc) return fail(rc, order[g]->last_error);
          if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != gen)
            return fail(ORCG_DEVICE_ERROR, "mid-stripe counts were not published");
          break;
        }
      }
      for (size_t k = 0; k < where[g].size(); ++k) out[where[g][k]] = h_pub[g * kPubStride + k];
    }
    return ORCG_OK;
  }
  uint64_t* h_sync = nullptr;
  size_t sync_cap = 0;
  int read_back(const std::vector<const void*>& src, uint64_t* out) {
    {
      const int pr = poll_counts(std::vector<Ctx*>(src.size(), ctx), src, out);
      if (pr != 1) return pr;
    }
    if (src.size() > sync_cap) {
      if (h_sync) (void)hipHostFree(h_sync);
      h_sync = nullptr;
      sync_cap = 0;
      const size_t cap = std::max<size_t>(64, src.size());
      if (hipHostMalloc((void**)&h_sync, cap * 8, hipHostMallocDefault) != hipSuccess)
        return fail(ORCG_OUT_OF_MEMORY, "pinned allocation failed");
      sync_cap = cap;
    }
    for (size_t i = 0; i < src.size(); ++i) {
      const int rc = hip_check(ctx, hipMemcpyAsync(h_sync + i, src[i], 8, hipMemcpyDeviceToHost, ctx->stream), "D2H");
      if (rc) return fail_ctx(rc);
    }
    const int rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    if (rc) return fail_ctx(rc);
    for (size_t i = 0; i < src.size(); ++i) out[i] = h_sync[i];
    return ORCG_OK;
  }

  ~orcg_reader() {
    if (ev_pre) (void)hipEventDestroy(ev_pre);
    if (h_pub) (void)hipHostFree(h_pub);
    slots.clear();
    if (mapped) munmap(mapped, file_len);
    if (h_sync) (void)hipHostFree(h_sync);
    for (Flight& f : flights) {
      if (f.h_defer) (void)hipHostFree(f.h_defer);
      if (f.h_rb) (void)hipHostFree(f.h_rb);
      for (const EvPair& p : f.ev_used) ev_pool.push_back(p.a), ev_pool.push_back(p.b);
      if (f.done) (void)hipEventDestroy(f.done);
      for (hipEvent_t e : {f.ev_up0, f.ev_up1, f.ev_dec})
        if (e) (void)hipEventDestroy(e);
    }
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
  }
  int fail(int status, const std::string& m) {
    if (err_col == kNoCol) err_col = cur_col;
    last_error = m;
    if (ctx) ctx->last_error = m;
    return status;
  }
  int fail_ctx(int rc) { return fail(rc, ctx ? ctx->last_error : std::string("device error")); }
  // a failure outside a decode (argument F->checks of the caller's thread):
  // last_error is shared with the row readers' workers, so under mu
  int fail_user(int status, const std::string& m) {
    std::lock_guard<std::mutex> lk(mu);
    last_error = m;
    if (own_ctx) own_ctx->last_error = m;
    return status;
  }
  int fail_oom(int line) {
    if (debug_on("alloc")) fprintf(stderr, "orcg: reader device allocation failed at reader_api.cpp:%d (column %u)\n", line, cur_col);
    return fail(ORCG_OUT_OF_MEMORY, "device allocation failed");
  }

  int open_tail();
  // (sel: the column selection of the read it prepares for; prepare reads
  // nothing else the decodes change, so it runs without mu)
  int prepare(uint64_t s, HostStage& hs, const std::vector<uint8_t>& sel) const;
  int prepare(uint64_t s, HostStage& hs) const { return prepare(s, hs, selected); }
  int read_stripes(uint64_t first, uint64_t count);
  int upload_and_decode(HostStage& hs, DevSlot& ds);  // issue + finish
  void issue(HostStage& hs, DevSlot& ds, Flight& fl);
  int finish(Flight& fl);
  // d_in_count (may be null): in_count is on the device (the parent's
  // non-null rows), in_count is then an upper bound; in_col: the column whose
  // mask in_nn is
  int decode(uint32_t id, uint64_t n, const uint8_t* in_nn, uint64_t in_count, const int64_t* rg_rows,
             const uint64_t* d_in_count = nullptr, Col* in_col = nullptr);
  // Columns whose value streams take a device-resident value count (RLEv2
  // through the tiled instances): their PRESENT decode's non-null count is
  // not read back mid-stripe (one stream synchronisation per nullable column
  // saved); has_nulls is settled with the stripe's F->checks.
  bool device_counts(const Col& c) const;
  // Whether decode(id) launches device work: false when everything it needs
  // came from the stripe's batched launches (streams, dictionaries)
  bool device_work(uint32_t id) const;
  // Side streams for sibling subtrees (ORCG_LANES, default 4; 1 = one
  // stream). in_lane: decode() runs on a side context (no nested forks).
  bool in_lane = false;
  // A list / map decoded under a fork whose children wait for its element
  // count (offsets[n] on the device), decoded on the same side context.
  struct Pending {
    uint32_t id;
    const int64_t* d_total;
    int64_t* child_rows;
    Ctx* lane;
  };
  std::vector<Pending>* pending = nullptr;
  // read_back over several side contexts: the D2H copies on each one's
  // stream, then one synchronisation per stream used
  int read_back_lanes(const std::vector<Pending>& ps, uint64_t* out) {
    {
      std::vector<Ctx*> lanes(ps.size());
      std::vector<const void*> srcs(ps.size());
      for (size_t i = 0; i < ps.size(); ++i) {
        lanes[i] = ps[i].lane;
        srcs[i] = ps[i].d_total;
      }
      const int pr = poll_counts(lanes, srcs, out);
      if (pr != 1) return pr;
    }
    if (ps.size() > sync_cap) {
      if (h_sync) (void)hipHostFree(h_sync);
      h_sync = nullptr;
      sync_cap = 0;
      const size_t cap = std::max<size_t>(64, ps.size());
      if (hipHostMalloc((void**)&h_sync, cap * 8, hipHostMallocDefault) != hipSuccess)
        return fail(ORCG_OUT_OF_MEMORY, "pinned allocation failed");
      sync_cap = cap;
    }
    std::vector<Ctx*> lanes_used;
    for (size_t i = 0; i < ps.size(); ++i) {
      const int rc = hip_check(ps[i].lane, hipMemcpyAsync(h_sync + i, ps[i].d_total, 8, hipMemcpyDeviceToHost,
                                                          ps[i].lane->stream), "D2H");
      if (rc) return fail(rc, ps[i].lane->last_error);
      if (std::find(lanes_used.begin(), lanes_used.end(), ps[i].lane) == lanes_used.end())
        lanes_used.push_back(ps[i].lane);
    }
    for (Ctx* l : lanes_used) {
      const int rc = hip_check(l, hipStreamSynchronize(l->stream), "hipStreamSynchronize");
      if (rc) return fail(rc, l->last_error);
    }
    for (size_t i = 0; i < ps.size(); ++i) out[i] = h_sync[i];
    return ORCG_OK;
  }
  static unsigned num_lanes() { return side_lanes(); }
  // row-group context of the column being decoded (segments())
  const int64_t* cur_rows = nullptr;  // device: first row of each row group, in the column's rows
  uint64_t cur_n = 0;
  const uint8_t* cur_in_nn = nullptr;
  const uint8_t* cur_row_nn = nullptr;
  int segments(Col& c, int slot, bool boolean, const uint64_t** d_seg, uint64_t* nseg);
  // RLE integer stream: v1 for DIRECT / DICTIONARY encodings (convertRleVersion,
  // DictionaryLoader.hh:42) unless force_v2 (Decimal64ColumnReaderV2 is always RLEv2)
  // (*out: the stream's values, decoded by this stripe's multi-stream batch
  // when collect() queued it, else allocated and decoded now)
  // (dcount: the value count on the device, `count` then only sizes the output)
  int int_stream(Col& c, int slot, bool is_signed, uint64_t count, int64_t** out, bool force_v2 = false,
                 const uint64_t* dcount = nullptr);
  // Multi-stream batch: before decode(), the RLEv2 streams whose value
  // counts and segments are known without device results (columns with no
  // PRESENT stream, under parents with none) are queued and decoded by one
  // launch per kernel instance (launch_rlev2_multi); decode() then finds
  // their outputs here.
  bool batch_on = true;
  std::vector<RleJob> batch;          // RLEv2 streams
  std::vector<V1SegDesc> v1_segs;     // RLEv1 streams' segments
  // dictionary columns of the batch (no nulls, <= kDictLds entries): their
  // offsets and gathers in one launch after the streams (dict_multi_kernel)
  struct DictDone {
    int64_t* offsets;
    const uint64_t* h_summary;
    int64_t* start;
    int64_t* len;
    int64_t* idx;
  };
  std::vector<DictJob> dict_batch;
  std::unordered_map<uint32_t, DictDone> dict_done;
  // dictionaries of columns the batch cannot take whole (nullable, under a
  // list / map): their entry offsets and summary only, from the same launch
  std::unordered_map<uint32_t, DictDone> dict_pre;
  int collect_dicts(uint32_t id);
  // a batch of such dictionaries only runs on side lane 0 (issue()); the
  // gathers reading its offsets and the stripe's read-back wait on ev_pre
  hipEvent_t ev_pre = nullptr;
  bool pre_on_lane = false;
  // varint decimal DATA streams whose tile counts + scan run with the batch
  // (before its join): their tile bases and value-count slots by column
  std::deque<VarintJob> varint_jobs;
  std::unordered_map<uint32_t, std::pair<int64_t*, const uint64_t*>> varint_pre;
  int queue_varint(uint32_t id);
  // varint decimal columns (no nulls, not Hive 0.11) decoded by one launch
  // per mode after the batch's join (varint_decimal_multi_kernel)
  std::vector<DecJob> dec_batch[2];
  std::unordered_map<uint32_t, void*> dec_done;
  int queue_decimal(uint32_t id, uint64_t n);
  // direct string columns (no nulls) whose length scan runs after the
  // batch's join, beside the dictionaries and decimals
  struct ScanDone {
    int64_t* starts;
    const uint64_t* h_flags;
    const uint64_t* h_need;
    uint64_t n;
  };
  std::deque<ScanJob> scan_jobs;
  std::unordered_map<uint32_t, ScanDone> scan_done;
  int queue_scan(uint32_t id, uint64_t n);
  std::vector<MultiLaunch> launches;
  std::unordered_map<uint64_t, std::pair<int64_t*, uint64_t>> batched;  // (column, slot) -> (values, count)
  int queue_stream(uint32_t id, int slot, bool is_signed, uint64_t count, bool force_v2);
  int queue_dict(uint32_t id, uint64_t n);
  int collect(uint32_t id, uint64_t n, const int64_t* rg_rows);
  int byte_stream(Col& c, int slot, bool boolean, uint64_t count, uint8_t* out, uint64_t* d_ones = nullptr,
                  const uint64_t* d_count = nullptr);
  int scatter(const void* dense, const uint8_t* nn, uint64_t n, void* out, int width);
  template <typename T>
  T* alloc(uint64_t count) {
    return (T*)D->pool.get(std::max<uint64_t>(count, 1) * sizeof(T));
  }
};

int orcg_reader::open_tail() {
  // ReaderImpl tail read (c++/src/Reader.cc:1650-1700, readPostscript :1548-1567)
  if (file_len < 4) return fail(ORCG_PARSE_ERROR, "File size too small");
  const uint64_t ps_len = file[file_len - 1];
  if (ps_len < 3) return fail(ORCG_PARSE_ERROR, "Invalid ORC postscript length");
  if (memcmp(file + file_len - 1 - 3, "ORC", 3) != 0 && memcmp(file, "ORC", 3) != 0)
    return fail(ORCG_PARSE_ERROR, "Not an ORC file");
  if (file_len < 1 + ps_len)
    return fail(ORCG_PARSE_ERROR, "Invalid ORC postscript length: " + std::to_string(ps_len) +
                                      ", file length = " + std::to_string(file_len));
  if (!parse_postscript(file + file_len - 1 - ps_len, ps_len, ps))
    return fail(ORCG_PARSE_ERROR, "Failed to parse the postscript");
  if (ps.block_size == 0) ps.block_size = 256 * 1024;
  decimal_as_long = ps.version.size() == 2 && ps.version[0] == 1 && ps.version[1] == 9999;
  // file_len >= 1 + ps_len here, so the subtraction cannot wrap
  if (ps.footer_length >= file_len - 1 - ps_len)
    return fail(ORCG_PARSE_ERROR, "Invalid tail size: footerSize=" + std::to_string(ps.footer_length) +
                                      ", postscriptLength=" + std::to_string(ps_len) +
                                      ", fileLength=" + std::to_string(file_len));
  if (ps.compression > kZstd) return fail(ORCG_PARSE_ERROR, "Unknown compression type");
  std::vector<uint8_t> fbytes;
  std::string err;
  const uint64_t tail = 1 + ps_len + ps.footer_length;
  if (!read_range(file, file_len - tail, ps.footer_length, ps.compression, ps.block_size, fbytes, err))
    return fail(ORCG_PARSE_ERROR, err);
  if (!parse_footer(fbytes.data(), fbytes.size(), footer)) return fail(ORCG_PARSE_ERROR, "Failed to parse the footer");
  // checkProtoTypes (Reader.cc:1575-1605)
  const size_t nt = footer.types.size();
  if (nt == 0) return fail(ORCG_PARSE_ERROR, "Footer is corrupt: no types found");
  for (size_t i = 0; i < nt; ++i) {
    const auto& t = footer.types[i];
    if (t.kind == ORCG_TYPE_STRUCT && t.subtypes.size() != t.field_names.size())
      return fail(ORCG_PARSE_ERROR, "Footer is corrupt: STRUCT type " + std::to_string(i) + " has " +
                                        std::to_string(t.subtypes.size()) + " subTypes, but has " +
                                        std::to_string(t.field_names.size()) + " fieldNames");
    for (size_t j = 0; j < t.subtypes.size(); ++j) {
      const uint32_t st = t.subtypes[j];
      if (st <= i)
        return fail(ORCG_PARSE_ERROR, "Footer is corrupt: malformed link from type " + std::to_string(i) +
                                          " to " + std::to_string(st));
      if (st >= nt) return fail(ORCG_PARSE_ERROR, "Footer is corrupt: types(" + std::to_string(st) + ") not exists");
      if (j > 0 && t.subtypes[j - 1] >= st)
        return fail(ORCG_PARSE_ERROR, "Footer is corrupt: subType(" + std::to_string(j - 1) + ") >= subType(" +
                                          std::to_string(j) + ") in types(" + std::to_string(i) + ")");
    }
  }
  own_sel.assign(nt, 1);
  return ORCG_OK;
}

int orcg_reader::scatter(const void* dense, const uint8_t* nn, uint64_t n, void* out, int width) {
  return launch_scatter(ctx, dense, nn, n, out, width, 1, 0);
}

#define ORCG_ALLOC(T, v, count)                                                   \
  T* v = alloc<T>(count);                                                         \
  if (!v) return fail_oom(__LINE__)
#define ORCG_ALLOC_TO(T, v, count)                                                \
  do {                                                                            \
    v = alloc<T>(count);                                                          \
    if (!v) return fail_oom(__LINE__);                                            \
  } while (0)

// The stream's segment table: the host plan's, or (row-index streams) built
// on the device from the row groups' positions and the present-row prefix
// at each row group's first row (PRESENT streams count the incoming rows).
int orcg_reader::segments(Col& c, int slot, bool boolean, const uint64_t** d_seg, uint64_t* nseg) {
  StreamBuf& sb = c.s[slot];
  if (!sb.pos) {
    *d_seg = (const uint64_t*)(D->d_stage + sb.seg_off);
    *nseg = sb.plan->segs.size();
    return ORCG_OK;
  }
  const uint64_t G = H->ngroups;
  if (!cur_rows) return fail(ORCG_INVALID_ARGUMENT, "row groups without row starts");
  const uint8_t* mask = slot == kSlotPresent ? cur_in_nn : cur_row_nn;
  const int64_t* prefix = cur_rows;
  int rc;
  if (mask) {
    // the row groups' set-row prefix and the segment table in one launch
    ORCG_ALLOC(int64_t, pre, G + 1);
    ORCG_ALLOC(uint64_t, seg, 2 * G);
    if ((rc = launch_rg_prefix_segtab(ctx, mask, cur_n, cur_rows, G, (const int64_t*)(D->d_stage + sb.rg_off), boolean,
                                      pre, seg)))
      return fail_ctx(rc);
    *d_seg = seg;
    *nseg = G;
    return ORCG_OK;
  }
  ORCG_ALLOC(uint64_t, seg, 2 * G);
  if ((rc = launch_rg_segtab(ctx, (const int64_t*)(D->d_stage + sb.rg_off), prefix, G, boolean, seg)))
    return fail_ctx(rc);
  *d_seg = seg;
  *nseg = G;
  return ORCG_OK;
}

bool orcg_reader::device_counts(const Col& c) const {
  if (!rlev2_multi_capable(ctx->rlev2_variant)) return false;
  const uint32_t k = c.kind;
  if (k == ORCG_TYPE_STRUCT) return true;
  if (c.encoding == kDirect || c.encoding == kDictionary) return false;  // RLEv1
  if (is_int_kind(k) || k == ORCG_TYPE_LIST || k == ORCG_TYPE_MAP || k == ORCG_TYPE_TIMESTAMP ||
      k == ORCG_TYPE_TIMESTAMP_INSTANT)
    return true;
  return is_string_kind(k) && c.encoding == kDictionaryV2;
}

bool orcg_reader::device_work(uint32_t id) const {
  const Col& c = H->cols[id];
  if (!selected[id] || !c.supported) return false;
  if (c.s[kSlotPresent].present) return true;
  const uint32_t k = c.kind;
  auto done = [&](int slot) { return !c.s[slot].present || batched.count((uint64_t)id * 8 + (uint64_t)slot) != 0; };
  if (k == ORCG_TYPE_STRUCT) {
    for (uint32_t st : footer.types[id].subtypes)
      if (device_work(st)) return true;
    return false;
  }
  if (is_int_kind(k)) return !done(kSlotData);
  if (k == ORCG_TYPE_DOUBLE) return false;  // the stream bytes are the values
  if (k == ORCG_TYPE_DECIMAL && dec_done.count(id)) return false;  // the batch's decimal launch
  if (is_string_kind(k) && (c.encoding == kDictionary || c.encoding == kDictionaryV2)) return dict_done.count(id) == 0;
  return true;
}

int orcg_reader::int_stream(Col& c, int slot, bool is_signed, uint64_t count, int64_t** pout, bool force_v2,
                            const uint64_t* dcount) {
  const uint64_t key = (uint64_t)(&c - H->cols.data()) * 8 + (uint64_t)slot;
  const auto it = batched.find(key);
  if (it != batched.end() && it->second.second == count) {
    *pout = it->second.first;
    return ORCG_OK;
  }
  int64_t* out = alloc<int64_t>(count);
  if (!out) return fail_oom(__LINE__);
  *pout = out;
  StreamBuf& sb = c.s[slot];
  if (count == 0) return ORCG_OK;
  if (!sb.present) return fail(ORCG_PARSE_ERROR, "stream not found in column");
  const bool v1 = !force_v2 && (c.encoding == kDirect || c.encoding == kDictionary);
  // (with a device count the kernel reports a stream short of values)
  if (!dcount && !sb.pos && count > sb.plan->values) {
    const uint32_t e = sb.plan->err != kErrNone ? sb.plan->err : (uint32_t)(v1 ? kErrV1BadRead : kErrBadRead);
    return fail(dev_error_status(e), dev_error_message(e));
  }
  const uint8_t* d_src = D->d_stage + sb.host_off;
  const uint64_t* d_seg;
  uint64_t nseg;
  int rc = segments(c, slot, false, &d_seg, &nseg);
  if (rc) return rc;
  const int sg = is_signed ? 1 : 0;
  madd(kMDecodeCall, 1);
  rc = timed(0, [&]() -> int {
    if (v1) return launch_rlev1(ctx, d_src, sb.len, sg, d_seg, nseg, 0, count, out, 8);
    return dcount ? launch_rlev2_tiled(ctx, d_src, sb.len, sg, d_seg, nseg, false, 0, 0, count, out, 8, dcount)
                  : launch_rlev2(ctx, d_src, sb.len, sg, d_seg, nseg, false, 0, 0, count, out, 8);
  });
  return rc ? fail_ctx(rc) : ORCG_OK;
}

int orcg_reader::queue_stream(uint32_t id, int slot, bool is_signed, uint64_t count, bool force_v2) {
  Col& c = H->cols[id];
  StreamBuf& sb = c.s[slot];
  // left to decode(): empty or missing streams, RLEv1, a host plan short of
  // values (decode() raises the error in column order)
  if (count == 0 || !sb.present) return ORCG_OK;
  const bool v1 = !force_v2 && (c.encoding == kDirect || c.encoding == kDictionary);
  if (!sb.pos && count > sb.plan->values) return ORCG_OK;
  // (collect() runs before the stripe's upload: no device work here)
  if (sb.pos && !(cur_rows && (v1 || rlev2_multi_capable(ctx->rlev2_variant)))) return ORCG_OK;
  if (v1) {
    // RLEv1: one host-built descriptor per segment (the plan's cuts, or the
    // row index with the stripe's row-group starts g * stride)
    int64_t* out = alloc<int64_t>(count);
    if (!out) return fail_oom(__LINE__);
    const uint8_t* d_src = D->d_stage + sb.host_off;
    const uint64_t stride = footer.row_index_stride;
    const size_t ns = sb.pos ? (size_t)H->ngroups : sb.plan->segs.size();
    auto at = [&](size_t g, uint64_t* off) -> uint64_t {
      if (sb.pos) {
        *off = (uint64_t)sb.trip[3 * g];
        const int64_t v = (int64_t)(g * stride) - sb.trip[3 * g + 1];
        return v < 0 ? 0ull : (uint64_t)v;
      }
      *off = sb.plan->segs[g].byte_offset;
      return sb.plan->segs[g].value_index;
    };
    for (size_t g = 0; g < ns; ++g) {
      V1SegDesc d{};
      d.src = d_src;
      d.src_len = sb.len;
      d.vi = at(g, &d.seg_start);
      d.seg_end = sb.len;
      d.v_next = ~0ull;
      if (g + 1 < ns) d.v_next = at(g + 1, &d.seg_end);
      d.dst = out;
      d.nvalues = count;
      d.err = D->d_errs + id;
      d.is_signed = is_signed ? 1u : 0u;
      v1_segs.push_back(d);
    }
    madd(kMDecodeCall, 1);
    batched[(uint64_t)id * 8 + (uint64_t)slot] = {out, count};
    return ORCG_OK;
  }
  RleJob j{};
  if (sb.pos) {
    // the row index is the segment table (no rg_segtab launch): collect()
    // only queues columns whose rows are all values (no mask)
    j.trip = (const int64_t*)(D->d_stage + sb.rg_off);
    j.rows = cur_rows;
    j.nsegs = H->ngroups;
  } else {
    const uint64_t* d_seg;
    uint64_t nseg;
    int rc = segments(c, slot, false, &d_seg, &nseg);
    if (rc) return rc;
    j.segtab = d_seg;
    j.nsegs = nseg;
  }
  int64_t* out = alloc<int64_t>(count);
  if (!out) return fail_oom(__LINE__);
  j.src = D->d_stage + sb.host_off;
  j.src_len = sb.len;
  j.dst = out;
  j.nvalues = count;
  j.is_signed = is_signed ? 1u : 0u;
  j.err = D->d_errs + id;
  batch.push_back(j);
  madd(kMDecodeCall, 1);
  batched[(uint64_t)id * 8 + (uint64_t)slot] = {out, count};
  return ORCG_OK;
}

// A dictionary column whose streams are both batched: its offsets and row
// gather join the stripe's dictionary launch (decode() then only wires the
// outputs and registers its F->checks).
int orcg_reader::queue_dict(uint32_t id, uint64_t n) {
  Col& c = H->cols[id];
  const uint64_t D_ = c.dict_size;
  if (D_ > kDictLds || !c.s[kSlotData].present) return ORCG_OK;
  if (D_ > 0 && !c.s[kSlotLength].present) return ORCG_OK;  // decode() raises the missing stream
  const auto li = batched.find((uint64_t)id * 8 + kSlotLength);
  const auto di = batched.find((uint64_t)id * 8 + kSlotData);
  if ((D_ > 0 && li == batched.end()) || (n > 0 && di == batched.end())) return ORCG_OK;
  DictJob j{};
  j.lengths = D_ ? li->second.first : nullptr;
  j.dict_size = D_;
  ORCG_ALLOC_TO(int64_t, j.offsets, D_ + 1);
  const uint64_t* h_summary = nullptr;
  j.summary = rb_alloc(2, &h_summary);
  if (!j.summary) return ORCG_OK;
  j.idx = n ? di->second.first : nullptr;
  j.nn = nullptr;
  j.n = lazy_dict ? 0 : n;
  if (!lazy_dict) {
    ORCG_ALLOC_TO(int64_t, j.start, n);
    ORCG_ALLOC_TO(int64_t, j.len, n);
  }
  j.err = D->d_errs + id;
  dict_batch.push_back(j);
  dict_done[id] = DictDone{j.offsets, h_summary, j.start, j.len, const_cast<int64_t*>(j.idx)};
  return ORCG_OK;
}

int orcg_reader::queue_varint(uint32_t id) {
  Col& c = H->cols[id];
  const StreamBuf& sb = c.s[kSlotData];
  if (!sb.present || sb.len == 0) return ORCG_OK;
  VarintJob j{};
  j.src = D->d_stage + sb.host_off;
  j.len = sb.len;
  ORCG_ALLOC_TO(int64_t, j.counts, sb.len / kVarintTile + 2);
  ORCG_ALLOC_TO(int64_t, j.base, sb.len / kVarintTile + 3);
  const uint64_t* h_total = nullptr;
  j.total = rb_alloc(1, &h_total);
  if (!j.total) return ORCG_OK;  // no read-back slot: decode() counts it itself
  varint_jobs.push_back(j);
  varint_pre[id] = {j.base, h_total};
  launches.push_back(MultiLaunch{4, 0, &varint_jobs.back(), 1, 0, 0});
  return ORCG_OK;
}

int orcg_reader::queue_decimal(uint32_t id, uint64_t n) {
  const file::TypeInfo& t = footer.types[id];
  if (t.precision == 0 || n == 0) return ORCG_OK;  // Hive 0.11: the per-column path (its checks, nulling)
  const auto vp = varint_pre.find(id);
  const auto sc = batched.find((uint64_t)id * 8 + (uint64_t)kSlotSecondary);
  if (vp == varint_pre.end() || sc == batched.end() || sc->second.second != n) return ORCG_OK;
  const bool wide = t.precision > 18;
  Col& c = H->cols[id];
  const StreamBuf& sb = c.s[kSlotData];
  DecJob j{};
  j.src = D->d_stage + sb.host_off;
  j.len = sb.len;
  j.tile_base = vp->second.first;
  j.scales = sc->second.first;
  j.nvalues = n;
  j.err = D->d_errs + id;
  j.scale = (int32_t)t.scale;
  int64_t* out = nullptr;
  ORCG_ALLOC_TO(int64_t, out, wide ? 2 * n : n);
  j.out = out;
  dec_batch[wide ? 1 : 0].push_back(j);
  dec_done[id] = out;
  return ORCG_OK;
}

int orcg_reader::queue_scan(uint32_t id, uint64_t n) {
  const auto li = batched.find((uint64_t)id * 8 + kSlotLength);
  if (n == 0 || li == batched.end() || li->second.second != n || !H->cols[id].s[kSlotData].present) return ORCG_OK;
  ScanJob j{};
  j.in = li->second.first;
  j.n = n;
  ORCG_ALLOC_TO(int64_t, j.out, n + 1);
  const uint64_t *h_fl = nullptr, *h_need = nullptr;
  j.flags = rb_alloc(2, &h_fl);
  j.total = j.flags ? rb_alloc(1, &h_need) : nullptr;
  if (!j.total) return ORCG_OK;  // no read-back slots: decode() scans it itself
  scan_jobs.push_back(j);
  scan_done[id] = ScanDone{j.out, h_fl, h_need, n};
  return ORCG_OK;
}

// Dictionaries below a column collect() does not descend into (a nullable
// column's subtree, a list's or map's children): a dictionary's size is in
// the stripe footer, so its LENGTH stream and entry offsets join the batch
// instead of being decoded after the parent's counts come back mid-stripe
// (configs[4]: the map keys' dictionary took three dependent launches on an
// idle GPU after the element counts were published, each blocking the host
// ~60-80 us, profiles/r06/inv/hip_api_c5_548c478.txt). LoadStringDictionary
// reads it whole whatever the rows (DictionaryLoader.cc:43-97).
int orcg_reader::collect_dicts(uint32_t id) {
  Col& c = H->cols[id];
  if (!selected[id] || !c.supported) return ORCG_OK;
  const uint32_t k = c.kind;
  if (is_string_kind(k) && (c.encoding == kDictionary || c.encoding == kDictionaryV2)) {
    const uint64_t D_ = c.dict_size;
    if (D_ == 0 || D_ > kDictLds || !c.s[kSlotLength].present) return ORCG_OK;
    int rc = queue_stream(id, kSlotLength, false, D_, false);
    if (rc) return rc;
    const auto li = batched.find((uint64_t)id * 8 + kSlotLength);
    if (li == batched.end() || li->second.second != D_) return ORCG_OK;
    DictJob j{};
    j.lengths = li->second.first;
    j.dict_size = D_;
    ORCG_ALLOC_TO(int64_t, j.offsets, D_ + 1);
    const uint64_t* h_summary = nullptr;
    j.summary = rb_alloc(2, &h_summary);
    if (!j.summary) return ORCG_OK;
    j.n = 0;  // offsets and summary only: decode() gathers the rows
    j.err = D->d_errs + id;
    dict_batch.push_back(j);
    dict_pre[id] = DictDone{j.offsets, h_summary, nullptr, nullptr, nullptr};
    return ORCG_OK;
  }
  for (uint32_t st : footer.types[id].subtypes) {
    const int rc = collect_dicts(st);
    if (rc) return rc;
  }
  return ORCG_OK;
}

// The streams decode() will read with host-known counts, in its order
// (same slots, signedness and counts as decode()'s int_stream calls).
int orcg_reader::collect(uint32_t id, uint64_t n, const int64_t* rg_rows) {
  Col& c = H->cols[id];
  if (!selected[id] || !c.supported) return ORCG_OK;
  if (c.s[kSlotPresent].present) return collect_dicts(id);  // its counts come from the device
  cur_rows = rg_rows;
  cur_n = n;
  cur_in_nn = nullptr;
  cur_row_nn = nullptr;
  const uint32_t k = c.kind;
  int rc = ORCG_OK;
  if (k == ORCG_TYPE_DECIMAL) {
    if (decimal_as_long && footer.types[id].precision - 1u < 18u) {
      rc = queue_stream(id, kSlotData, true, n, true);
    } else {
      rc = queue_stream(id, kSlotSecondary, true, n, false);
      if (!rc && c.s[kSlotSecondary].present) rc = queue_varint(id);
      if (!rc && c.s[kSlotData].present) rc = queue_decimal(id, n);
    }
  } else if (k == ORCG_TYPE_TIMESTAMP || k == ORCG_TYPE_TIMESTAMP_INSTANT) {
    rc = queue_stream(id, kSlotData, true, n, false);
    if (!rc) rc = queue_stream(id, kSlotSecondary, false, n, false);
  } else if (is_int_kind(k)) {
    rc = queue_stream(id, kSlotData, true, n, false);
  } else if (is_string_kind(k)) {
    if (c.encoding == kDictionary || c.encoding == kDictionaryV2) {
      rc = queue_stream(id, kSlotLength, false, c.dict_size, false);
      if (!rc) rc = queue_stream(id, kSlotData, false, n, false);
      if (!rc) rc = queue_dict(id, n);
    } else {
      rc = queue_stream(id, kSlotLength, false, n, false);
      if (!rc) rc = queue_scan(id, n);
    }
  } else if (k == ORCG_TYPE_LIST || k == ORCG_TYPE_MAP) {
    rc = queue_stream(id, kSlotLength, false, n, false);
    for (uint32_t st : footer.types[id].subtypes)
      if (!rc) rc = collect_dicts(st);
  } else if (k == ORCG_TYPE_STRUCT) {
    for (uint32_t st : footer.types[id].subtypes)
      if ((rc = collect(st, n, rg_rows))) break;
  }
  return rc;
}

int orcg_reader::byte_stream(Col& c, int slot, bool boolean, uint64_t count, uint8_t* out, uint64_t* d_ones,
                             const uint64_t* d_count) {
  StreamBuf& sb = c.s[slot];
  if (count == 0) return ORCG_OK;
  if (!sb.present) return fail(ORCG_PARSE_ERROR, "stream not found in column");
  if (!sb.pos && !d_count) {  // (with a device count the kernel reports a short stream)
    const uint64_t avail = boolean ? sb.plan->values * 8 : sb.plan->values;
    if (count > avail) {
      const uint32_t e = sb.plan->err != kErrNone ? sb.plan->err : (uint32_t)kErrByteBadRead;
      return fail(dev_error_status(e), dev_error_message(e));
    }
  }
  const uint64_t* d_seg;
  uint64_t nseg;
  int rc = segments(c, slot, boolean, &d_seg, &nseg);
  if (rc) return rc;
  madd(kMByteCall, 1);
  rc = timed(1, [&]() -> int {
    return launch_byterle(ctx, D->d_stage + sb.host_off, sb.len, d_seg, nseg, boolean, 0, count, out, d_ones, d_count);
  });
  return rc ? fail_ctx(rc) : ORCG_OK;
}


int orcg_reader::decode(uint32_t id, uint64_t n, const uint8_t* in_nn, uint64_t in_count, const int64_t* rg_rows,
                        const uint64_t* d_in_count, Col* in_col) {
  Col& c = H->cols[id];
  if (!selected[id] || !c.supported) return ORCG_OK;
  // this column's kernels report into its own device error record
  struct Scope {
    orcg_reader* r;
    uint32_t col;
    unsigned long long* err;
    ~Scope() {
      r->cur_col = col;
      r->ctx->d_err = err;
    }
  } scope{this, cur_col, ctx->d_err};
  cur_col = id;
  ctx->d_err = D->d_errs + id;
  c.n = n;
  c.decoded = true;
  int rc;
  cur_rows = rg_rows;
  cur_n = n;
  cur_in_nn = in_nn;
  cur_row_nn = nullptr;
  // ColumnReader::next: PRESENT bits for the incoming non-null rows
  // (d_in: their count is on the device, in_count an upper bound)
  const bool dev = device_counts(c);
  const uint64_t* d_in = in_nn ? d_in_count : nullptr;
  if (d_in && !dev) {  // this column needs the incoming count on the host
    if ((rc = read_back({d_in}, &in_count))) return rc;
    d_in = nullptr;
  }
  uint64_t nonnull = in_nn ? in_count : n;  // exact, or (d_nonnull) an upper bound
  const uint64_t* d_nonnull = d_in;
  uint8_t* nn = nullptr;
  if (c.s[kSlotPresent].present) {
    ORCG_ALLOC(uint8_t, bits, in_count + 8);
    // the decode counts the set rows it writes: the non-null rows, with or
    // without the parent's mask scattered in
    uint64_t* ones = D->d_ones + id;
    if ((rc = byte_stream(c, kSlotPresent, true, in_nn ? in_count : n, bits, ones, d_in))) return rc;
    if (in_nn) {
      ORCG_ALLOC_TO(uint8_t, nn, n);
      if ((rc = scatter(bits, in_nn, n, nn, 1))) return fail_ctx(rc);
    } else {
      nn = bits;
    }
    if (dev) {
      nonnull = n;
      d_nonnull = ones;
    } else {
      if ((rc = read_back({ones}, &nonnull))) return rc;
      d_nonnull = nullptr;
    }
  } else if (in_nn) {
    nn = const_cast<uint8_t*>(in_nn);
  }
  c.has_nulls = nn != nullptr && (d_nonnull != nullptr || nonnull < n);
  if (in_nn && !c.s[kSlotPresent].present) c.has_nulls = true;  // incoming mask copied (:97-101)
  c.nn = c.has_nulls ? nn : nullptr;
  // provisional has_nulls: settled by the stripe's F->checks (column order:
  // a parent's before its children's)
  if (c.s[kSlotPresent].present && d_nonnull) {
    const uint64_t* h = defer(d_nonnull, 1);
    if (!h) return fail(ORCG_DEVICE_ERROR, "D2H of the non-null count failed");
    c.nulls_deferred = true;
    Col* cp = &c;
    F->checks.emplace_back(cur_col, [cp, h, n]() -> int {
      if (*h >= n) {
        cp->has_nulls = false;
        cp->nn = nullptr;
      }
      return ORCG_OK;
    });
  } else if (in_nn && !c.s[kSlotPresent].present && in_col && in_col->nulls_deferred) {
    c.nulls_deferred = true;
    Col* cp = &c;
    F->checks.emplace_back(cur_col, [cp, in_col]() -> int {
      if (!in_col->has_nulls) {  // the parent had no nulls after all: no mask was passed down
        cp->has_nulls = false;
        cp->nn = nullptr;
      }
      return ORCG_OK;
    });
  }
  const uint8_t* row_nn = c.nn;
  cur_row_nn = row_nn;

  auto place_i64 = [&](int64_t* dense) -> int64_t* {
    if (!row_nn) return dense;
    int64_t* out = alloc<int64_t>(n);
    if (!out) return nullptr;
    return scatter(dense, row_nn, n, out, 8) ? nullptr : out;
  };

  const uint32_t k = c.kind;
  const bool has_data = c.s[kSlotData].present, has_len = c.s[kSlotLength].present;
  const bool has_sec = c.s[kSlotSecondary].present;
  if (k == ORCG_TYPE_DECIMAL) {
    const file::TypeInfo& t = footer.types[id];
    const std::string cid = std::to_string(id);
    if (decimal_as_long && t.precision - 1u < 18u) {  // precision 1..18 (0 = Hive 0.11 first)
      // Decimal64ColumnReaderV2 (ColumnReader.cc:1529-1576): RLEv2 unscaled values
      if (!has_data) return fail(ORCG_PARSE_ERROR, "DATA stream not found in Decimal64V2 column. ColumnId=" + cid);
      int64_t* dense;
      if ((rc = int_stream(c, kSlotData, true, nonnull, &dense, true))) return rc;
      if (!(c.data = place_i64(dense))) return fail_ctx(ORCG_DEVICE_ERROR);
    } else {
      // Decimal64ColumnReader / Decimal128ColumnReader (:1384-1527): varint
      // DATA, per-value scales in SECONDARY (signed RLE)
      if (!has_data) return fail(ORCG_PARSE_ERROR, "DATA stream not found in Decimal64Column");
      if (!has_sec) return fail(ORCG_PARSE_ERROR, "SECONDARY stream not found in Decimal64Column");
      // Hive 0.11 (precision 0): Decimal128 at the forced scale (DecimalHive11ColumnReader, :1627-1687)
      const bool hive11 = t.precision == 0;
      const bool wide = hive11 || t.precision > 18;
      int64_t* scales;
      if ((rc = int_stream(c, kSlotSecondary, true, nonnull, &scales))) return rc;
      const StreamBuf& sb = c.s[kSlotData];
      const uint8_t* d_src = D->d_stage + sb.host_off;
      int64_t* base = nullptr;
      const uint64_t* total = nullptr;
      const auto vp = varint_pre.find(id);
      if (vp != varint_pre.end()) {
        // tile counts + scan ran with the batch (queue_varint)
        base = vp->second.first;
        total = vp->second.second;
      } else {
        uint64_t ntiles = 0;
        ORCG_ALLOC(int64_t, counts, sb.len / kVarintTile + 2);
        ORCG_ALLOC_TO(int64_t, base, sb.len / kVarintTile + 3);
        const uint64_t* h_total = nullptr;
        uint64_t* d_total = rb_alloc(1, &h_total);
        if ((rc = launch_varint_tile_counts(ctx, d_src, sb.len, counts, &ntiles))) return fail_ctx(rc);
        if ((rc = launch_exclusive_scan(ctx, counts, ntiles, base, nullptr, d_total))) return fail_ctx(rc);
        total = d_total ? h_total : defer(base + ntiles, 1);
        if (!total) return fail(ORCG_DEVICE_ERROR, "D2H of the varint count failed");
      }
      F->checks.emplace_back(cur_col, [this, total, nonnull, cid]() -> int {
        return *total < nonnull ? fail(ORCG_PARSE_ERROR, "Read past end of stream in Decimal64ColumnReader column " +
                                                             cid + " kind DATA")
                                : ORCG_OK;
      });
      const auto dd = dec_done.find(id);
      if (dd != dec_done.end() && !row_nn) {
        // decoded by the batch's decimal launch (queue_decimal)
        c.data = dd->second;
        return ORCG_OK;
      }
      ORCG_ALLOC(int64_t, dense, wide ? 2 * nonnull : nonnull);
      // throwOnHive11DecimalOverflow(false): overflowing values become NULL
      const bool nullify = hive11 && !hive11_throw;
      uint8_t* keep = nullptr;
      if (nullify) {
        ORCG_ALLOC_TO(uint8_t, keep, nonnull + 8);
      }
      if ((rc = launch_varint_decimal(ctx, d_src, sb.len, base, scales, nonnull,
                                    hive11 ? hive11_scale : (int32_t)t.scale,
                                    hive11 ? (nullify ? 3 : 2) : (wide ? 1 : 0), dense, keep)))
        return fail_ctx(rc);
      if (!row_nn) {
        c.data = dense;
      } else {
        ORCG_ALLOC(int64_t, out, wide ? 2 * n : n);
        if ((rc = scatter(dense, row_nn, n, out, wide ? 16 : 8))) return fail_ctx(rc);
        c.data = out;
      }
      if (nullify && nonnull) {
        // the row mask: rows present in the stream AND kept (the reference
        // clears notNull[i] and sets hasNulls, ColumnReader.cc:1650-1677)
        uint8_t* rnn = keep;
        if (row_nn) {
          ORCG_ALLOC_TO(uint8_t, rnn, n + 8);
          if ((rc = scatter(keep, row_nn, n, rnn, 1))) return fail_ctx(rc);
        }
        // the column's own count word: sibling decimal columns decode on
        // other side lanes concurrently
        const uint64_t* h_kept = nullptr;
        uint64_t* kept_d = rb_alloc(1, &h_kept);
        if (!kept_d) ORCG_ALLOC_TO(uint64_t, kept_d, 1);
        if ((rc = launch_count_nonzero(ctx, rnn, n, kept_d))) return fail_ctx(rc);
        const uint64_t* kept = defer(kept_d, 1);
        if (!kept) return fail(ORCG_DEVICE_ERROR, "D2H of the kept decimal count failed");
        Col* cp = &c;
        F->checks.emplace_back(cur_col, [cp, kept, rnn, n]() -> int {
          if (*kept < n) {
            cp->has_nulls = true;
            cp->nn = rnn;
          }
          return ORCG_OK;
        });
      }
    }
  } else if (k == ORCG_TYPE_TIMESTAMP || k == ORCG_TYPE_TIMESTAMP_INSTANT) {
    // TimestampColumnReader (:259-349): seconds (signed RLE), nanos (unsigned RLE)
    if (!has_data) return fail(ORCG_PARSE_ERROR, "DATA stream not found in Timestamp column");
    if (!has_sec) return fail(ORCG_PARSE_ERROR, "SECONDARY stream not found in Timestamp column");
    int64_t *secs, *nanos;
    if ((rc = int_stream(c, kSlotData, true, nonnull, &secs, false, d_nonnull))) return rc;
    if ((rc = int_stream(c, kSlotSecondary, false, nonnull, &nanos, false, d_nonnull))) return rc;
    if ((rc = launch_timestamp(ctx, secs, nanos, nonnull, kOrcEpochUtc))) return fail_ctx(rc);
    if (!(c.data = place_i64(secs)) || !(c.secondary = place_i64(nanos))) return fail_ctx(ORCG_DEVICE_ERROR);
  } else if (is_int_kind(k)) {
    if (!has_data) return fail(ORCG_PARSE_ERROR, "DATA stream not found in Integer column");
    int64_t* dense;
    if ((rc = int_stream(c, kSlotData, true, nonnull, &dense, false, d_nonnull))) return rc;
    if (!(c.data = place_i64(dense))) return fail_ctx(ORCG_DEVICE_ERROR);
  } else if (k == ORCG_TYPE_BOOLEAN || k == ORCG_TYPE_BYTE) {
    if (!has_data)
      return fail(ORCG_PARSE_ERROR, k == ORCG_TYPE_BOOLEAN ? "DATA stream not found in Boolean column"
                                                           : "DATA stream not found in Byte column");
    ORCG_ALLOC(uint8_t, bytes, nonnull + 8);
    if ((rc = byte_stream(c, kSlotData, k == ORCG_TYPE_BOOLEAN, nonnull, bytes))) return rc;
    ORCG_ALLOC(int64_t, dense, nonnull);
    if ((rc = launch_widen(ctx, bytes, k == ORCG_TYPE_BYTE ? kWidenI8 : kWidenU8, nonnull, dense))) return fail_ctx(rc);
    if (!(c.data = place_i64(dense))) return fail_ctx(ORCG_DEVICE_ERROR);
  } else if (k == ORCG_TYPE_FLOAT || k == ORCG_TYPE_DOUBLE) {
    if (!has_data) return fail(ORCG_PARSE_ERROR, "DATA stream not found in Double column");
    StreamBuf& sb = c.s[kSlotData];
    const uint64_t w = k == ORCG_TYPE_FLOAT ? 4 : 8;
    if (sb.len < w * nonnull) return fail(ORCG_PARSE_ERROR, "bad read in DoubleColumnReader::next()");
    const void* raw = D->d_stage + sb.host_off;
    double* dense;
    if (k == ORCG_TYPE_FLOAT) {
      ORCG_ALLOC_TO(double, dense, nonnull);
      if ((rc = launch_widen(ctx, raw, kWidenF32, nonnull, dense))) return fail_ctx(rc);
    } else {
      dense = (double*)raw;  // zero copy: the stream bytes are the values
    }
    if (row_nn) {
      ORCG_ALLOC(double, out, n);
      if ((rc = scatter(dense, row_nn, n, out, 8))) return fail_ctx(rc);
      c.data = out;
    } else {
      c.data = dense;
    }
  } else if (is_string_kind(k)) {
    const bool dict = c.encoding == kDictionary || c.encoding == kDictionaryV2;
    int64_t* start = nullptr;
    int64_t* len = nullptr;
    if (!(dict && lazy_dict) && !(dict && dict_done.count(id))) {
      ORCG_ALLOC_TO(int64_t, start, n);
      ORCG_ALLOC_TO(int64_t, len, n);
    }
    const auto dd = dict ? dict_done.find(id) : dict_done.end();
    if (dd != dict_done.end()) {
      // batched (queue_dict): offsets, summary and gather come from the
      // stripe's dictionary launch; the reference's F->checks, in its order
      const std::string cid = std::to_string(id);
      const uint64_t* h = dd->second.h_summary;
      StreamBuf& db = c.s[kSlotDict];
      Col* cp = &c;
      const bool db_present = db.present;
      const uint64_t db_len = db.present ? db.len : 0;
      F->checks.emplace_back(cur_col, [this, h, cp, db_present, db_len, cid]() -> int {
        if (h[1]) return fail(ORCG_PARSE_ERROR, "Negative dictionary entry length for column " + cid);
        if (h[0] > 0 && !db_present)
          return fail(ORCG_PARSE_ERROR, "DICTIONARY_DATA stream not found in StringDictionaryColumn for column " + cid);
        if (h[0] > db_len) return fail(ORCG_PARSE_ERROR, "bad read in readFully");
        cp->blob_len = h[0];
        return ORCG_OK;
      });
      c.blob = db.present ? D->d_stage + db.host_off : nullptr;
      c.index = dd->second.idx;
      c.dict_offsets = dd->second.offsets;
      start = dd->second.start;
      len = dd->second.len;
    } else if (dict) {
      // loadStringDictionary (DictionaryLoader.cc:43-97), then
      // StringDictionaryColumnReader::next (ColumnReader.cc:561-594)
      const uint64_t dict_size = c.dict_size;
      const std::string cid = std::to_string(id);
      if (dict_size > 0 && !has_len)
        return fail(ORCG_PARSE_ERROR, "LENGTH stream not found in StringDictionaryColumn for column " + cid);
      int64_t* doff;
      const uint64_t* h;
      const auto pre = dict_pre.find(id);
      if (pre != dict_pre.end()) {
        // offsets and summary from the stripe's dictionary launch (collect_dicts)
        doff = pre->second.offsets;
        h = pre->second.h_summary;
        if (pre_on_lane && (rc = hip_check(ctx, hipStreamWaitEvent(ctx->stream, ev_pre, 0), "dictionary batch wait")))
          return fail_ctx(rc);
      } else {
        int64_t* dlen;
        ORCG_ALLOC_TO(int64_t, doff, dict_size + 1);
        if ((rc = int_stream(c, kSlotLength, false, dict_size, &dlen))) return rc;
        const uint64_t* h_sum = nullptr;
        uint64_t* summary = rb_alloc(2, &h_sum);  // blob bytes, negative-length flag
        if (!summary) ORCG_ALLOC_TO(uint64_t, summary, 2);
        if (dict_size <= 65536) {
          // offsets, blob size and the negative-length check in one launch
          if ((rc = launch_dict_offsets(ctx, dlen, dict_size, doff, summary))) return fail_ctx(rc);
        } else {
          if ((rc = launch_flag_negative(ctx, dlen, dict_size, summary + 1))) return fail_ctx(rc);
          if ((rc = launch_exclusive_scan(ctx, dlen, dict_size, doff))) return fail_ctx(rc);
          if ((rc = hip_check(ctx, hipMemcpyAsync(summary, doff + dict_size, 8, hipMemcpyDeviceToDevice, ctx->stream),
                              "copy")))
            return fail_ctx(rc);
        }
        h = defer(summary, 2);
        if (!h) return fail(ORCG_DEVICE_ERROR, "D2H of the dictionary size failed");
      }
      StreamBuf& db = c.s[kSlotDict];
      Col* cp = &c;
      const bool db_present = db.present;
      const uint64_t db_len = db.present ? db.len : 0;
      F->checks.emplace_back(cur_col, [this, h, cp, db_present, db_len, cid]() -> int {
        if (h[1]) return fail(ORCG_PARSE_ERROR, "Negative dictionary entry length for column " + cid);
        if (h[0] > 0 && !db_present)
          return fail(ORCG_PARSE_ERROR, "DICTIONARY_DATA stream not found in StringDictionaryColumn for column " + cid);
        if (h[0] > db_len) return fail(ORCG_PARSE_ERROR, "bad read in readFully");
        cp->blob_len = h[0];
        return ORCG_OK;
      });
      if (!has_data) return fail(ORCG_PARSE_ERROR, "DATA stream not found in StringDictionaryColumn");
      c.blob = db.present ? D->d_stage + db.host_off : nullptr;
      int64_t* idx;
      if ((rc = int_stream(c, kSlotData, false, nonnull, &idx, false, d_nonnull))) return rc;
      int64_t* ridx = idx;
      if (row_nn) {
        ORCG_ALLOC_TO(int64_t, ridx, n);
        if ((rc = scatter(idx, row_nn, n, ridx, 8))) return fail_ctx(rc);
      }
      c.index = ridx;
      c.dict_offsets = doff;
      if (!lazy_dict) {
        // StringDictionaryColumnReader::next: bounds-checked gather; nextEncoded
        // (lazy) hands out the indices and the dictionary unchecked (:596-607)
        if (row_nn) {
          if ((rc = hip_check(ctx, hipMemsetAsync(start, 0, n * 8, ctx->stream), "memset"))) return fail_ctx(rc);
          if ((rc = hip_check(ctx, hipMemsetAsync(len, 0, n * 8, ctx->stream), "memset"))) return fail_ctx(rc);
        }
        if ((rc = launch_dict_gather(ctx, ridx, 8, row_nn, n, doff, dict_size, start, len))) return fail_ctx(rc);
      }
    } else {
      if (!has_len) return fail(ORCG_PARSE_ERROR, "LENGTH stream not found in StringDirectColumn");
      if (!has_data) return fail(ORCG_PARSE_ERROR, "DATA stream not found in StringDirectColumn");
      int64_t* dlen;
      if ((rc = int_stream(c, kSlotLength, false, nonnull, &dlen, false))) return rc;
      const uint64_t ns = nonnull;
      // computeSize's checks (ColumnReader.cc:694-710) ride the scan: a
      // negative length, the total's overflow (then the blob's size below),
      // in the reference's order; the flags start at 0 (read-back block).
      // The batch's scan (queue_scan) already ran for a column without nulls.
      const auto sd = scan_done.find(id);
      const bool pre = sd != scan_done.end() && !row_nn && sd->second.n == ns;
      int64_t* dstart = nullptr;
      const uint64_t* h_fl = nullptr;
      const uint64_t* need = nullptr;
      uint64_t* flags = nullptr;
      if (pre) {
        dstart = sd->second.starts;
        h_fl = sd->second.h_flags;
        need = sd->second.h_need;
      } else {
        ORCG_ALLOC_TO(int64_t, dstart, ns + 1);
        flags = rb_alloc(2, &h_fl);
        if (!flags) {
          ORCG_ALLOC_TO(uint64_t, flags, 2);
          if ((rc = hip_check(ctx, hipMemsetAsync(flags, 0, 16, ctx->stream), "flags memset"))) return fail_ctx(rc);
        }
        uint64_t* d_need = rb_alloc(1, &need);
        if ((rc = launch_exclusive_scan(ctx, dlen, ns, dstart, flags, d_need))) return fail_ctx(rc);
      }
      StreamBuf& db = c.s[kSlotData];
      c.blob = D->d_stage + db.host_off;
      c.blob_len = db.len;
      if (!h_fl && !(h_fl = defer(flags, 2))) return fail(ORCG_DEVICE_ERROR, "D2H of the string length checks failed");
      if (!need && !(need = defer(dstart + ns, 1))) return fail(ORCG_DEVICE_ERROR, "D2H of the string bytes failed");
      const uint64_t blob_len = c.blob_len;
      const uint32_t col_id = cur_col;
      F->checks.emplace_back(cur_col, [this, need, blob_len, h_fl, col_id]() -> int {
        if (h_fl[0])
          return fail(ORCG_PARSE_ERROR,
                      "Negative string length in StringDirectColumnReader for column " + std::to_string(col_id));
        if (h_fl[1])
          return fail(ORCG_PARSE_ERROR,
                      "String length overflow in StringDirectColumnReader for column " + std::to_string(col_id));
        return *need > blob_len ? fail(ORCG_PARSE_ERROR, "failed to read in StringDirectColumnReader.next") : ORCG_OK;
      });
      if (row_nn) {
        if ((rc = scatter(dstart, row_nn, n, start, 8))) return fail_ctx(rc);
        if ((rc = scatter(dlen, row_nn, n, len, 8))) return fail_ctx(rc);
      } else {
        start = dstart;
        len = dlen;
      }
    }
    c.data = start;
    c.length = len;
  } else if (k == ORCG_TYPE_LIST || k == ORCG_TYPE_MAP) {
    if (!has_len)
      return fail(ORCG_PARSE_ERROR, k == ORCG_TYPE_LIST ? "LENGTH stream not found in List column"
                                                        : "LENGTH stream not found in Map column");
    int64_t* dlen;
    if ((rc = int_stream(c, kSlotLength, false, nonnull, &dlen, false, d_nonnull))) return rc;
    int64_t* rlen = dlen;
    if (row_nn) {
      ORCG_ALLOC_TO(int64_t, rlen, n);
      if ((rc = scatter(dlen, row_nn, n, rlen, 8))) return fail_ctx(rc);
    }
    ORCG_ALLOC(int64_t, off, n + 1);
    if ((rc = launch_exclusive_scan(ctx, rlen, n, off))) return fail_ctx(rc);
    c.offsets = off;
    // the children's row groups start at the list offsets of the parent's
    int64_t* child_rows = nullptr;
    if (rg_rows && H->ngroups) {
      ORCG_ALLOC_TO(int64_t, child_rows, H->ngroups);
      if ((rc = launch_rg_child_rows(ctx, off, rg_rows, H->ngroups, child_rows))) return fail_ctx(rc);
    }
    if (pending) {
      // under a fork: the children wait for the fork's next level, whose
      // element counts are read back together (one synchronisation per level
      // instead of one per list / map, which would stall the other lanes)
      pending->push_back(Pending{id, off + n, child_rows, ctx});
      return ORCG_OK;
    }
    uint64_t total = 0;
    if ((rc = read_back({off + n}, &total))) return rc;
    for (uint32_t st : footer.types[id].subtypes)
      if ((rc = decode(st, total, nullptr, total, child_rows))) return rc;
  } else if (k == ORCG_TYPE_STRUCT) {
    std::vector<uint32_t> kids;
    size_t busy = 0;  // subtrees with launches of their own (the rest only wire batched outputs)
    for (uint32_t st : footer.types[id].subtypes)
      if (selected[st] && H->cols[st].supported) {
        kids.push_back(st);
        busy += device_work(st) ? 1 : 0;
      }
    // side streams only pay when at least two subtrees launch work
    const unsigned nl = in_lane || busy < 2 ? 1u : (unsigned)std::min<size_t>(num_lanes(), kids.size());
    if (nl <= 1) {
      for (uint32_t st : kids)
        if ((rc = decode(st, n, c.nn, nonnull, rg_rows, c.nn ? d_nonnull : nullptr, &c))) return rc;
    } else {
      // sibling subtrees on side streams (their kernels run concurrently:
      // most launches of a stripe are one workgroup per row group, a
      // fraction of the chip), forked after this column's work and joined
      // back before anything reads their outputs
      Ctx* base = ctx;
      if (!ctx_lane(base, 0)) return fail(ORCG_DEVICE_ERROR, "side stream creation failed");
      if ((rc = hip_check(ctx, hipEventRecord(base->ev_fork, base->stream), "fork event"))) return fail_ctx(rc);
      std::vector<uint8_t> used(nl, 0);
      std::vector<Pending> level;  // lists / maps whose children wait for their element counts
      pending = &level;
      for (size_t j = 0; j < kids.size() && !rc; ++j) {
        Ctx* L = ctx_lane(base, j % nl);
        if (!L) {
          rc = fail(ORCG_DEVICE_ERROR, "side stream creation failed");
          break;
        }
        if (!used[j % nl]) {
          used[j % nl] = 1;
          if ((rc = hip_check(base, hipStreamWaitEvent(L->stream, base->ev_fork, 0), "fork wait"))) {
            rc = fail_ctx(rc);
            break;
          }
        }
        ctx = L;
        in_lane = true;
        rc = decode(kids[j], n, c.nn, nonnull, rg_rows, c.nn ? d_nonnull : nullptr, &c);
        in_lane = false;
        ctx = base;
      }
      // the waiting children, level by level. Within a level the subtrees
      // with the most columns are enqueued first: the host's enqueue of a
      // level takes longer than a short chain runs (configs[4]: the map's
      // keys chain, the longest, started ~110 us late behind the list's
      // items). Errors keep column order: after a failure only columns
      // before it go on (their device errors would come first), the earliest
      // column's failure is the one reported, and a level below keeps only
      // the subtrees before it.
      const int fork_rc = rc;
      const uint32_t fork_col = err_col;
      const std::string fork_msg = last_error;
      uint32_t fail_col = fork_rc ? fork_col : kNoCol;
      int fail_rc = fork_rc;
      std::string fail_msg = fork_rc ? fork_msg : std::string();
      int hard = ORCG_OK;  // a failure outside any column's decode: stop
      std::function<uint32_t(uint32_t)> cols_in = [&](uint32_t t) -> uint32_t {
        uint32_t k = selected[t] && H->cols[t].supported ? 1u : 0u;
        for (uint32_t st : footer.types[t].subtypes) k += cols_in(st);
        return k;
      };
      while (!level.empty() && !hard) {
        std::vector<Pending> cur;
        cur.swap(level);
        size_t keep = 0;  // (pre-order: ascending ids)
        while (keep < cur.size() && cur[keep].id < fail_col) ++keep;
        cur.resize(keep);
        if (cur.empty()) break;
        std::vector<uint64_t> totals(cur.size(), 0);
        if ((hard = read_back_lanes(cur, totals.data()))) break;
        std::vector<uint32_t> weight(cur.size());
        std::vector<size_t> ord(cur.size());
        for (size_t q = 0; q < cur.size(); ++q) {
          weight[q] = cols_in(cur[q].id);
          ord[q] = q;
        }
        std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return weight[x] > weight[y]; });
        for (size_t q : ord) {
          if (cur[q].id >= fail_col) continue;  // after an earlier failure
          // a map's keys and values are siblings too: when both launch work
          // the values go to the next lane of this fork, after what that lane
          // already holds (C5: the string keys' dictionary chain and the
          // nullable values' chain, ~190 + ~115 us, ran back to back on the
          // map's lane while the list's lane idled; a lane of its own would
          // share one of the process's 4 hardware queues, HIP's default)
          const std::vector<uint32_t>& subs = footer.types[cur[q].id].subtypes;
          std::vector<Ctx*> on(subs.size(), cur[q].lane);
          size_t li = 0;
          while (li < nl && base->lanes[li] != cur[q].lane) ++li;
          if (subs.size() == 2 && nl >= 2 && li < nl && device_work(subs[0]) && device_work(subs[1])) {
            const size_t alt = (li + 1) % nl;
            Ctx* const L2 = base->lanes[alt];
            hard = hip_check(base, hipEventRecord(base->ev_join[li], cur[q].lane->stream), "fork event");
            if (!hard) hard = hip_check(base, hipStreamWaitEvent(L2->stream, base->ev_join[li], 0), "fork wait");
            if (hard) {
              hard = fail_ctx(hard);
              break;
            }
            used[alt] = 1;
            on[1] = L2;
          }
          in_lane = true;
          err_col = kNoCol;
          int lr = ORCG_OK;
          for (size_t si = 0; si < subs.size() && !lr; ++si) {
            ctx = on[si];
            lr = decode(subs[si], totals[q], nullptr, totals[q], cur[q].child_rows);
          }
          in_lane = false;
          ctx = base;
          if (lr) {
            const uint32_t ec = err_col != kNoCol ? err_col : cur[q].id;
            if (ec < fail_col) {
              fail_col = ec;
              fail_rc = lr;
              fail_msg = last_error;
            }
          }
        }
      }
      pending = nullptr;
      if (hard) {
        rc = hard;
      } else if (fail_rc) {
        rc = fail_rc;
        err_col = fail_col;
        last_error = fail_msg;
        ctx->last_error = fail_msg;
      }
      for (unsigned l = 0; l < nl; ++l) {
        if (!used[l]) continue;
        int jr = hip_check(base, hipEventRecord(base->ev_join[l], base->lanes[l]->stream), "join event");
        if (!jr) jr = hip_check(base, hipStreamWaitEvent(base->stream, base->ev_join[l], 0), "join wait");
        if (jr && !rc) rc = fail_ctx(jr);
      }
      if (rc) return rc;
    }
  } else if (k == ORCG_TYPE_UNION) {
    // UnionColumnReader (ColumnReader.cc:1158-1274): byte-RLE tags for the
    // non-null rows; each row's offset is its rank among the rows of its
    // tag; child k reads as many rows as carry tag k
    if (!has_data) return fail(ORCG_PARSE_ERROR, "LENGTH stream not found in Union column");
    const std::vector<uint32_t> subs = footer.types[id].subtypes;
    const uint32_t nch = (uint32_t)subs.size();
    ORCG_ALLOC(uint8_t, dtags, nonnull + 8);
    if ((rc = byte_stream(c, kSlotData, false, nonnull, dtags))) return rc;
    ORCG_ALLOC(uint64_t, bad, 1);
    if ((rc = launch_union_check(ctx, dtags, nonnull, nch, bad))) return fail_ctx(rc);
    ORCG_ALLOC(int64_t, doffs, nonnull);
    ORCG_ALLOC(int64_t, flags, nonnull);
    // dense index of each row group's first row (children's row groups)
    const int64_t* dense_rows = rg_rows;
    if (rg_rows && H->ngroups && row_nn) {
      ORCG_ALLOC(int64_t, cnt, H->ngroups);
      ORCG_ALLOC(int64_t, pre, H->ngroups + 1);
      if ((rc = launch_rg_prefix(ctx, row_nn, n, rg_rows, H->ngroups, cnt, pre))) return fail_ctx(rc);
      dense_rows = pre;
    }
    std::vector<int64_t*> scans(nch, nullptr);
    std::vector<const void*> rb;  // per child its row count, then the first bad tag
    for (uint32_t kk = 0; kk < nch; ++kk) {
      ORCG_ALLOC_TO(int64_t, scans[kk], nonnull + 1);
      if ((rc = launch_union_flags(ctx, dtags, nonnull, kk, flags)) ||
          (rc = launch_exclusive_scan(ctx, flags, nonnull, scans[kk])) ||
          (rc = launch_union_offsets(ctx, dtags, nonnull, kk, scans[kk], doffs)))
        return fail_ctx(rc);
      rb.push_back(scans[kk] + nonnull);
    }
    rb.push_back(bad);
    std::vector<uint64_t> counts(nch + 1, 0);
    if ((rc = read_back(rb, counts.data()))) return rc;
    const uint64_t first_bad = counts[nch];
    if (first_bad != ~0ull)
      return fail(ORCG_PARSE_ERROR, "Invalid union tag " + std::to_string(first_bad & 0xff) + " for union with " +
                                        std::to_string(nch) + " children");
    if (row_nn) {
      ORCG_ALLOC(uint8_t, rtags, n);
      ORCG_ALLOC(int64_t, roffs, n);
      if ((rc = scatter(dtags, row_nn, n, rtags, 1)) || (rc = scatter(doffs, row_nn, n, roffs, 8))) return fail_ctx(rc);
      c.tags = rtags;
      c.offsets = roffs;
    } else {
      c.tags = dtags;
      c.offsets = doffs;
    }
    for (uint32_t kk = 0; kk < nch; ++kk) {
      int64_t* child_rows = nullptr;
      if (dense_rows && H->ngroups) {
        ORCG_ALLOC_TO(int64_t, child_rows, H->ngroups);
        if ((rc = launch_rg_child_rows(ctx, scans[kk], dense_rows, H->ngroups, child_rows))) return fail_ctx(rc);
      }
      if ((rc = decode(subs[kk], counts[kk], nullptr, counts[kk], child_rows))) return rc;
    }
  }
  return ORCG_OK;
}

// What upload_and_decode appends to a stripe's staging for nc columns: the
// read-back block (error records, non-null counts, summary slots) and the
// job arena of the batched launches, each 256-byte aligned.
static uint64_t rb_words_for(size_t nc) { return 2 * nc + 1 + 4 * nc + 16; }
static uint64_t arena_bytes_for(size_t nc, uint64_t v1_segs, uint64_t dict_tiles) {
  // (dictionary jobs: one copy per 2,048-row tile of a column)
  return 5 * (nc + 1) * sizeof(RleJob) + (nc + 1) * sizeof(DictJob) * dict_tiles + v1_segs * sizeof(V1SegDesc) +
         16 * 256;
}
static uint64_t upload_tail_bytes(size_t nc, uint64_t v1_segs, uint64_t dict_tiles) {
  return 256 + 8 * rb_words_for(nc) + 256 + arena_bytes_for(nc, v1_segs, dict_tiles) + 64;
}
// RLEv1 segments of a prepared stripe (each a descriptor in the arena)
static uint64_t v1_segments(const HostStage& hs) {
  uint64_t n = 0;
  for (const Col& c : hs.cols) {
    if (c.encoding != kDirect && c.encoding != kDictionary) continue;
    for (const StreamBuf& sb : c.s)
      if (sb.present) n += sb.pos ? hs.ngroups : (sb.plan ? sb.plan->segs.size() : 0);
  }
  return n;
}

// Host half of a stripe read (thread-safe w.r.t. the device half of another
// stripe): stripe footer (Reader.cc getStripeFooter :620-640), stream
// location (StripeStream.cc:82-125), decompression of every selected stream
// (Compression.cc) in parallel chunks, run plans + segment tables.
// (Small streams on host plans instead of row-index segment tables were
// measured in round 4, profiles/r04/*small_stream_ab*: no gain, dropped.)

// RLEv1 streams up to this size decode in 1 KB host-plan segments
constexpr uint64_t kV1SmallStream = 64u << 10;

// Whether an RLEv2 stream's first runs (up to 32) average >= 96 bytes: a
// stream of long DIRECT / PATCHED_BASE runs (header bytes only are read).
static bool long_runs(const uint8_t* p, uint64_t len) {
  uint64_t pos = 0, runs = 0;
  while (pos < len && runs < 32) {
    uint64_t L = 0, end = 0;
    if (host_parse_run(p, len, pos, &L, &end) != kErrNone) return false;
    pos = end;
    ++runs;
  }
  return runs > 0 && pos >= 96 * runs;
}

int orcg_reader::prepare(uint64_t s, HostStage& hs, const std::vector<uint8_t>& selected) const {
  hs.stripe = s;
  hs.rc = ORCG_OK;
  hs.err.clear();
  const double t0 = now_s();
  const StripeInfo& si = footer.stripes[s];
  std::string err;
  std::vector<uint8_t> fb;
  // stripe = [offset, + index, + data, + footer), every sum checked
  // (RowReaderImpl::startNextStripe, Reader.cc:1257-1268)
  uint64_t foff = 0, total = 0;
  if (__builtin_add_overflow(si.offset, si.index_length, &foff) ||
      __builtin_add_overflow(foff, si.data_length, &foff) ||
      __builtin_add_overflow(foff, si.footer_length, &total) || total >= file_len)
    return hs.fail(ORCG_PARSE_ERROR, "Malformed StripeInformation at stripe index " + std::to_string(s) +
                                         ": fileLength=" + std::to_string(file_len) + ", StripeInfo=(offset=" +
                                         std::to_string(si.offset) + ", indexLength=" +
                                         std::to_string(si.index_length) + ", dataLength=" +
                                         std::to_string(si.data_length) + ", footerLength=" +
                                         std::to_string(si.footer_length) + ")");
  if (!read_range(file, foff, si.footer_length, ps.compression, ps.block_size, fb, err))
    return hs.fail(ORCG_PARSE_ERROR, err);
  StripeFooter sf;
  if (!parse_stripe_footer(fb.data(), fb.size(), si.offset, sf))
    return hs.fail(ORCG_PARSE_ERROR, std::string("bad StripeFooter from ") + compression_name(ps.compression));
  // Reader.cc:634-640
  const size_t nt = footer.types.size();
  if (sf.encodings.size() != nt)
    return hs.fail(ORCG_PARSE_ERROR, "bad number of ColumnEncodings in StripeFooter: expected=" +
                                         std::to_string(nt) + ", actual=" + std::to_string(sf.encodings.size()));
  hs.cols = std::vector<Col>(nt);
  hs.slack = upload_tail_bytes(nt, 0, (si.num_rows + 2047) / 2048 + 1);
  for (size_t i = 0; i < nt; ++i) {
    hs.cols[i].kind = footer.types[i].kind;
    hs.cols[i].encoding = sf.encodings[i].kind;
    hs.cols[i].dict_size = sf.encodings[i].dictionary_size;
    hs.cols[i].supported = is_supported(footer.types[i], sf.writer_timezone);
  }
  struct Need {
    uint32_t col;
    int slot;
    std::vector<Chunk> chunks;
    uint64_t file_off = 0;  // stream start in the file
  };
  std::vector<int> row_index(nt, -1);  // ROW_INDEX stream of each column (index into sf.streams)
  std::vector<Need> needs;
  const uint64_t data_end = foff;  // <= file_len (checked above)
  for (size_t i = 0; i < sf.streams.size(); ++i) {
    const StreamInfo& st = sf.streams[i];
    const bool in_stripe = st.offset >= si.offset && range_ok(st.offset, st.length, data_end);
    if (st.kind == kRowIndex && st.column < nt && selected[st.column] && hs.cols[st.column].supported && in_stripe)
      row_index[st.column] = (int)i;
    const int slot = slot_of(st.kind);
    if (slot < 0 || st.column >= nt) continue;
    if (!selected[st.column] || !hs.cols[st.column].supported) continue;
    if (!in_stripe)
      return hs.fail(ORCG_PARSE_ERROR, "Malformed stream meta at stream index " + std::to_string(i) + " in stripe " +
                                           std::to_string(s));
    Need nd{st.column, slot, {}, st.offset};
    if (!split_chunks(file, st.offset, st.length, ps.compression, nd.chunks, err)) return hs.fail(ORCG_PARSE_ERROR, err);
    needs.push_back(std::move(nd));
  }
  // I/O (ReaderMetrics::IOCount / IOBlockingLatencyUs): the reference preads
  // each stream (SeekableFileInputStream); this reader maps the file, so its
  // blocking I/O is the page-in of the streams' byte ranges: one touch per
  // page, timed (page-cache hits cost ~nothing, cold pages their read)
  {
    const double ti = now_s();
    uint64_t sink = 0;
    for (const Need& nd : needs)
      for (const Chunk& ch : nd.chunks) {
        const uint8_t* b = file + ch.src_off;
        for (uint64_t o = 0; o < ch.src_len; o += 4096) sink += ((const volatile uint8_t*)b)[o];
      }
    hs.io_sink = sink;
    hs.t_io = now_s() - ti;
    hs.n_io = needs.size() + 1;  // + the stripe footer
  }
  // staging: every chunk gets a slot of its maximum size, compacted after
  uint64_t at = 0;
  std::vector<std::pair<size_t, size_t>> all;
  for (size_t i = 0; i < needs.size(); ++i) {
    at = (at + 255) & ~(uint64_t)255;
    for (size_t j = 0; j < needs[i].chunks.size(); ++j) {
      Chunk& ch = needs[i].chunks[j];
      ch.dst_off = at;
      at += ch.original ? ch.src_len : ps.block_size;
      all.emplace_back(i, j);
    }
  }
  if (!hs.ensure(at + 64, 0)) return hs.fail(ORCG_OUT_OF_MEMORY, "pinned staging allocation failed");
  const double t1 = now_s();
  std::vector<std::string> errs(all.size());
  std::atomic<bool> bad{false};
  uint64_t src_bytes = 0;
  for (auto& nd : needs)
    for (auto& ch : nd.chunks) src_bytes += ch.src_len;
  // ~64 KB of compressed input per thread (stored chunks are copies: more)
  parallel_for(all.size(), [&](size_t q) {
    Chunk& ch = needs[all[q].first].chunks[all[q].second];
    const uint64_t cap = ch.original ? ch.src_len : ps.block_size;
    if (!decompress_chunk(ps.compression, file, ch, hs.h + ch.dst_off, cap, errs[q])) bad = true;
  }, src_bytes, ps.compression == kNone ? (1u << 20) : (64u << 10));
  if (bad)
    for (auto& e : errs)
      if (!e.empty()) return hs.fail(ORCG_PARSE_ERROR, e);
  uint64_t w = 0;  // compact (destinations never pass their sources)
  for (size_t i = 0; i < needs.size(); ++i) {
    w = (w + 255) & ~(uint64_t)255;
    const uint64_t s0 = w;
    for (auto& ch : needs[i].chunks) {
      if (ch.dst_off != w) memmove(hs.h + w, hs.h + ch.dst_off, ch.dst_len);
      w += ch.dst_len;
    }
    StreamBuf& sb = hs.cols[needs[i].col].s[needs[i].slot];
    sb.present = true;
    sb.host_off = s0;
    sb.len = w - s0;
  }
  const double t15 = now_s();
  // Row-index segmentation: the positions every row group records for each of
  // the column's streams (ColumnReader::seekToRowGroup order, ColumnReader.cc;
  // the writers' recordPosition order, ColumnWriter.cc) give run-aligned cut
  // points, so those streams need no host header walk.
  hs.ngroups = 0;
  // ORCG_NO_ROW_INDEX=1 forces the host plans (A/B and tests)
  const char* no_ri = getenv("ORCG_NO_ROW_INDEX");
  if (footer.row_index_stride > 0 && si.num_rows > 0 && !(no_ri && no_ri[0] == '1')) {
    const uint64_t G = (si.num_rows + footer.row_index_stride - 1) / footer.row_index_stride;
    std::vector<int> need_of(nt * 5, -1);
    for (size_t i = 0; i < needs.size(); ++i) need_of[needs[i].col * 5 + needs[i].slot] = (int)i;
    const bool compressed = ps.compression != kNone;
    enum { kRaw = 0, kInt = 1, kByteRle = 2, kBool = 3 };
    // one column per task: decompress + parse its ROW_INDEX, map positions
    std::atomic<bool> any{false};
    uint64_t ri_bytes = 0;
    for (size_t col = 0; col < nt; ++col)
      if (row_index[col] >= 0) ri_bytes += sf.streams[row_index[col]].length;
    parallel_for(nt, [&](size_t col) {
      if (row_index[col] < 0) return;
      Col& c = hs.cols[col];
      const uint32_t k = c.kind;
      std::vector<std::pair<int, int>> order;  // (slot, stream kind)
      if (c.s[kSlotPresent].present) order.push_back({kSlotPresent, kBool});
      const bool dict = c.encoding == kDictionary || c.encoding == kDictionaryV2;
      if (k == ORCG_TYPE_BOOLEAN) order.push_back({kSlotData, kBool});
      else if (k == ORCG_TYPE_BYTE || k == ORCG_TYPE_UNION) order.push_back({kSlotData, kByteRle});
      else if (is_int_kind(k)) order.push_back({kSlotData, kInt});
      else if (k == ORCG_TYPE_FLOAT || k == ORCG_TYPE_DOUBLE) order.push_back({kSlotData, kRaw});
      else if (is_string_kind(k)) {
        if (dict) order.push_back({kSlotData, kInt});
        else {
          order.push_back({kSlotData, kRaw});
          order.push_back({kSlotLength, kInt});
        }
      } else if (k == ORCG_TYPE_DECIMAL) {
        if (decimal_as_long && footer.types[col].precision - 1u < 18u) order.push_back({kSlotData, kInt});
        else {
          order.push_back({kSlotData, kRaw});
          order.push_back({kSlotSecondary, kInt});
        }
      } else if (k == ORCG_TYPE_TIMESTAMP || k == ORCG_TYPE_TIMESTAMP_INSTANT) {
        order.push_back({kSlotData, kInt});
        order.push_back({kSlotSecondary, kInt});
      } else if (k == ORCG_TYPE_LIST || k == ORCG_TYPE_MAP) {
        order.push_back({kSlotLength, kInt});
      }
      bool ok = !order.empty();
      for (auto& o : order) ok = ok && c.s[o.first].present && need_of[col * 5 + o.first] >= 0;
      if (!ok) return;
      const StreamInfo& ri = sf.streams[row_index[col]];
      std::vector<uint8_t> ib;
      std::vector<std::vector<uint64_t>> entries;
      std::string e2;
      if (!read_range(file, ri.offset, ri.length, ps.compression, ps.block_size, ib, e2) ||
          !parse_row_index(ib.data(), ib.size(), entries) || entries.size() != G)
        return;
      // per stream: chunk header offsets (in the stream) -> decompressed starts
      std::vector<std::vector<std::pair<uint64_t, uint64_t>>> cmap(order.size());
      for (size_t o = 0; o < order.size(); ++o) {
        const Need& nd = needs[need_of[col * 5 + order[o].first]];
        uint64_t d = 0;
        for (const Chunk& ch : nd.chunks) {
          const uint64_t hdr = compressed ? ch.src_off - 3 - nd.file_off : ch.src_off - nd.file_off;
          cmap[o].push_back({hdr, d});
          d += ch.dst_len;
        }
        cmap[o].push_back({nd.file_off + 0, d});  // sentinel: the stream's end
        cmap[o].back().first = ~0ull;
      }
      std::vector<std::vector<int64_t>> trips(order.size());
      for (uint64_t g = 0; g < G && ok; ++g) {
        const std::vector<uint64_t>& pv = entries[g];
        size_t at = 0;
        for (size_t o = 0; o < order.size() && ok; ++o) {
          const size_t need_n = (compressed ? 2 : 1) + (order[o].second == kBool ? 2 : order[o].second == kRaw ? 0 : 1);
          if (at + need_n > pv.size()) {
            ok = false;
            break;
          }
          uint64_t off;
          const StreamBuf& sb = c.s[order[o].first];
          if (compressed) {
            const uint64_t chunk = pv[at], in = pv[at + 1];
            auto& m = cmap[o];
            auto it = std::lower_bound(m.begin(), m.end() - 1, std::make_pair(chunk, (uint64_t)0));
            if (it != m.end() - 1 && it->first == chunk) off = it->second + in;
            else if (it == m.end() - 1) off = m.back().second + in;  // position at the stream's end
            else {
              ok = false;
              break;
            }
            at += 2;
          } else {
            off = pv[at++];
          }
          if (off > sb.len) {
            ok = false;
            break;
          }
          if (order[o].second != kRaw) {
            const int64_t skip = (int64_t)pv[at++];
            const int64_t bits = order[o].second == kBool ? (int64_t)pv[at++] : 0;
            auto& t = trips[o];
            if (!t.empty() && (uint64_t)t[t.size() - 3] > off) ok = false;
            t.push_back((int64_t)off);
            t.push_back(skip);
            t.push_back(bits);
          }
        }
      }
      if (!ok) return;
      for (size_t o = 0; o < order.size(); ++o) {
        if (order[o].second == kRaw) continue;
        StreamBuf& sb = c.s[order[o].first];
        sb.pos = true;
        sb.trip = std::move(trips[o]);
      }
      any = true;
    }, ri_bytes, 16u << 10);  // row indexes: ~16 KB of (compressed) entries per thread
    if (any) hs.ngroups = G;
  }
  // columns whose value streams decode in a launch of their own, never in the
  // stripe's multi-stream batch (collect() stops at a PRESENT stream and at a
  // list's or map's children): a column with nulls, or one below a list, a
  // map or a column with nulls (configs[4]'s map keys)
  std::vector<uint8_t> alone(nt, 0);
  for (size_t i = 0; i < nt; ++i) {
    const Col& c = hs.cols[i];
    const bool down = alone[i] || c.s[kSlotPresent].present || c.kind == ORCG_TYPE_LIST || c.kind == ORCG_TYPE_MAP;
    if (c.s[kSlotPresent].present) alone[i] = 1;
    if (down)
      for (uint32_t st : footer.types[i].subtypes)
        if (st < nt && st > i) alone[st] = 1;  // (pre-order ids: children after parents)
  }
  // host run plans (header walks only) for every RLE stream, in parallel
  std::vector<StreamBuf*> rle;
  std::vector<int> rle_kind;  // 0 byte RLE, 1 RLEv1, 2 RLEv2
  for (size_t i = 0; i < nt; ++i) {
    Col& c = hs.cols[i];
    if (!selected[i] || !c.supported) continue;
    const bool v1 = c.encoding == kDirect || c.encoding == kDictionary;
    for (int sl : {kSlotPresent, kSlotData, kSlotLength, kSlotSecondary}) {
      StreamBuf& sb = c.s[sl];
      if (!sb.present) continue;
      int kind;
      if (sl == kSlotPresent) kind = 0;
      else if (sl == kSlotData) {
        if (c.kind == ORCG_TYPE_BOOLEAN || c.kind == ORCG_TYPE_BYTE || c.kind == ORCG_TYPE_UNION) kind = 0;
        else if (is_int_kind(c.kind) || c.kind == ORCG_TYPE_TIMESTAMP || c.kind == ORCG_TYPE_TIMESTAMP_INSTANT ||
                 (is_string_kind(c.kind) && (c.encoding == kDictionary || c.encoding == kDictionaryV2)))
          kind = v1 ? 1 : 2;
        else if (c.kind == ORCG_TYPE_DECIMAL && decimal_as_long && footer.types[i].precision - 1u < 18u)
          kind = 2;  // Decimal64ColumnReaderV2: RLEv2 (ColumnReader.cc:1544-1556)
        else continue;  // raw bytes / varints
      } else {
        kind = v1 ? 1 : 2;
      }
      // cut by the row index, unless a byte-RLE stream's row groups are too
      // coarse to fill the GPU: a child column's row groups hold several
      // rows per parent row (C5's list items: ~40k PRESENT bits, 5 KB per
      // row group), one workgroup each while most of the GPU idles; such a
      // stream gets a host plan with 1 KB segments, as streams without a row
      // index do (its walk hops ~129 bytes at a time, in address order: cheap
      // on the host). Integer streams keep the row index: their host walk
      // chases run headers ~2 KB apart through memory (~45 ns a run, 0.9 ms
      // for a 42 MB stream), which lands on the host-bound critical path
      //
      // An RLEv2 stream of long runs (its first runs average >= 96 bytes:
      // DIRECT / PATCHED_BASE runs of hundreds of values) in a launch of its
      // own (`alone`: a nullable column, or one below a list, a map or a
      // nullable column) gets a host plan with 8 KB segments too: a child
      // column's row group holds ~40,000 values in several serial window
      // passes of one workgroup (C5's list items, map keys and map values:
      // 260 workgroups per stream; the keys' launch took 135 us a stripe),
      // while the host walk costs ~45 ns a run, a few thousand runs a
      // stripe. Batched columns keep the row index: their streams
      // share one multi-stream launch with the short-run streams, whose
      // latency sets its length, and the extra host walk lands on the
      // host-bound wall (C4: device 3.46 -> 3.64 ms, host plans 3.4 -> 7.8 ms
      // with fine plans on every long-run stream).
      bool fine = false;
      if (sb.pos) {
        const uint64_t per_group = hs.ngroups ? sb.len / hs.ngroups : 0;
        if (kind == 1 && sb.len <= kV1SmallStream) {
          // a small RLEv1 stream (configs[0]: 5,000-row stripes, <= 5 KB
          // streams, one row group): 1 KB host-plan segments instead of one
          // row-group segment, so the stream's windows decode side by side
          // (rlev1_kernel's narrow instance) -- the host walk is ~1 ns a byte
        } else if (kind == 0) {
          if (per_group <= (2u << 10)) continue;
        } else if (kind == 2 && alone[i] && per_group > (8u << 10) && long_runs(hs.h + sb.host_off, sb.len)) {
          fine = true;
        } else {
          continue;
        }
        sb.pos = false;
        sb.trip.clear();
      }
      rle.push_back(&sb);
      rle_kind.push_back(fine ? 3 : kind);
    }
  }
  uint64_t plan_bytes = 0;
  for (auto* sb : rle) plan_bytes += sb->len;
  parallel_for(rle.size(), [&](size_t q) {
    StreamBuf& sb = *rle[q];
    const uint8_t* p = hs.h + sb.host_off;
    // byte / boolean RLE without row-index segments: 4 KB segments, one
    // byterle_kernel window each (C5's child PRESENT streams: 45.7 -> 32.8 us
    // a launch against 1 KB segments, whose workgroups each paid the
    // window's fixed phase latencies for a quarter of the bytes)
    constexpr uint32_t byte_seg = 4u << 10;
    if (rle_kind[q] == 0) sb.plan.reset(make_byte_plan(p, sb.len, byte_seg, byte_seg));
    else if (rle_kind[q] == 1)
      sb.plan.reset(make_v1_plan(p, sb.len, sb.len <= kV1SmallStream ? (1u << 10) : (16u << 10), 8192));
    else if (rle_kind[q] == 3) sb.plan.reset(make_plan(p, sb.len, 8u << 10, 4096));
    else sb.plan.reset(make_plan(p, sb.len, 16u << 10, 8192));
  }, plan_bytes, 512u << 10);  // header walks: ~512 KB of stream per thread
  hs.n_plan = rle.size();
  hs.n_chunks = all.size();
  hs.n_pos = 0;
  for (auto& c : hs.cols)
    for (auto& sb : c.s) hs.n_pos += sb.pos ? 1 : 0;
  hs.slack = upload_tail_bytes(nt, v1_segments(hs), (si.num_rows + 2047) / 2048 + 1);
  uint64_t seg_bytes = 0;
  for (auto* sb : rle) seg_bytes += ((sb->plan->segs.size() * sizeof(orcg_segment)) + 255) & ~(uint64_t)255;
  w = (w + 255) & ~(uint64_t)255;
  if (!hs.ensure(w + seg_bytes + 64, w)) return hs.fail(ORCG_OUT_OF_MEMORY, "pinned staging allocation failed");
  for (auto* sb : rle) {
    sb->seg_off = w;
    const size_t nb = sb->plan->segs.size() * sizeof(orcg_segment);
    if (nb) memcpy(hs.h + w, sb->plan->segs.data(), nb);
    w = (w + nb + 255) & ~(uint64_t)255;
  }
  // row-index triplets and the row-group start rows
  uint64_t rg_bytes = hs.ngroups ? ((hs.ngroups * 8 + 255) & ~(uint64_t)255) : 0;
  for (auto& c : hs.cols)
    for (auto& sb : c.s)
      if (sb.pos) rg_bytes += ((sb.trip.size() * 8) + 255) & ~(uint64_t)255;
  if (rg_bytes) {
    if (!hs.ensure(w + rg_bytes + 64, w)) return hs.fail(ORCG_OUT_OF_MEMORY, "pinned staging allocation failed");
    hs.rows_off = w;
    for (uint64_t g = 0; g < hs.ngroups; ++g) ((int64_t*)(hs.h + w))[g] = (int64_t)(g * footer.row_index_stride);
    w = (w + hs.ngroups * 8 + 255) & ~(uint64_t)255;
    for (auto& c : hs.cols)
      for (auto& sb : c.s)
        if (sb.pos) {
          sb.rg_off = w;
          memcpy(hs.h + w, sb.trip.data(), sb.trip.size() * 8);
          w = (w + sb.trip.size() * 8 + 255) & ~(uint64_t)255;
        }
  }
  hs.used = w;
  const double t2 = now_s();
  hs.t_parse = t1 - t0;
  hs.t_decomp = t15 - t1;
  hs.t_plan = t2 - t15;
  return ORCG_OK;
}

// The stripe's first error, in column order (type ids are pre-order, the
// order decode() visits the columns): for each column up to the one that
// failed inline (`inline_rc`, detected on the host while launching), its
// deferred F->checks, then its device error record (the first bad value of its
// kernels), as the reference raises them while reading that column; then the
// inline failure itself; then the context's own record.
int orcg_reader::first_error(int inline_rc) {
  const std::string inline_msg = last_error;
  const uint32_t inline_col = err_col;
  cur_col = kNoCol;
  // the stripe's read-back copy (error records, non-null counts, summary
  // slots) and its deferred copies were queued by issue(): wait for them
  const size_t nc = H->cols.size();
  if (hipEventSynchronize(F->done) != hipSuccess) return fail(ORCG_DEVICE_ERROR, "stream synchronize failed");
  std::vector<unsigned long long> rec(F->h_rb, F->h_rb + nc);
  const uint32_t last = inline_rc ? (inline_col == kNoCol ? 0u : inline_col) : (uint32_t)nc;
  // checks grouped by column once (stable: a column's checks keep their
  // order), then one walk over columns and checks together
  std::stable_sort(F->checks.begin(), F->checks.end(),
                   [](const std::pair<uint32_t, std::function<int()>>& a,
                      const std::pair<uint32_t, std::function<int()>>& b) { return a.first < b.first; });
  size_t ci = 0;
  for (uint32_t col = 0; col < nc && col <= last; ++col) {
    for (; ci < F->checks.size() && F->checks[ci].first <= col; ++ci) {
      const int rc = F->checks[ci].second();
      if (rc) return rc;
    }
    if (rec[col] != kNoError) {
      const uint32_t code = (uint32_t)(rec[col] & 0xff);
      ctx->last_error_value = rec[col] >> 8;
      std::string m = dev_error_message(code);
      if (m == "unknown device error") {
        char b[96];
        snprintf(b, sizeof b, " (column %u, record 0x%llx)", col, (unsigned long long)rec[col]);
        m += b;
      }
      return fail(dev_error_status(code), m);
    }
  }
  if (inline_rc) return fail(inline_rc, inline_msg);
  for (auto& ch : F->checks)
    if (ch.first >= nc) {
      const int rc = ch.second();
      if (rc) return rc;
    }
  // the context's own record (launches outside a column's scope)
  const unsigned long long own = F->h_rb[2 * nc];
  if (own != kNoError) {
    const uint32_t code = (uint32_t)(own & 0xff);
    ctx->last_error_value = own >> 8;
    return fail(dev_error_status(code), dev_error_message(code));
  }
  return ORCG_OK;
}

// Device half, launch side: one H2D of the staging buffer (streams, the
// initialised read-back block, the batched launches' job tables), the
// batched launches, every selected column's launches, the read-back copy and
// the flight's event. Host checks wait for finish().
void orcg_reader::issue(HostStage& hs, DevSlot& ds, Flight& fl) {
  F = &fl;
  fl.hs = &hs;
  fl.ds = &ds;
  fl.t0 = now_s();
  fl.rc = ORCG_OK;
  fl.enqueued = false;
  // Launch checks read hipGetLastError (per host thread): drop a failure a
  // call whose result was already checked or deliberately ignored (frees in
  // destructors, a retried allocation) left behind, so it cannot surface as
  // this stripe's first launch error.
  {
    const hipError_t stale = hipGetLastError();
    if (debug_on("stale") && stale != hipSuccess) fprintf(stderr, "orcg: stale HIP error before upload: %s\n", hipGetErrorString(stale));
  }
  cur_col = err_col = kNoCol;
  auto early = [&](int rc) {  // a failure before anything was enqueued
    fl.rc = rc;
    fl.err_col = err_col;
    fl.err_msg = last_error;
    fl.t1 = now_s();
    H = nullptr;
    D = nullptr;
  };
  ds.stripe = hs.stripe;
  ds.pool.release_all();
  // a fresh slot's first chunk: the staging plus ~16 bytes per row and
  // selected column (outputs and scratch); later stripes use what it took
  {
    size_t nsel = 0;
    for (size_t i = 0; i < hs.cols.size(); ++i) nsel += selected[i] && hs.cols[i].supported ? 1 : 0;
    ds.pool.hint = hs.used + hs.slack + 16 * nsel * footer.stripes[hs.stripe].num_rows + (1u << 20);
  }
  const size_t nc = hs.cols.size();
  const uint64_t nrows_stripe = footer.stripes[hs.stripe].num_rows;
  // after the streams: the read-back block (error records 0xff.., non-null
  // counts and summary slots 0) and the job arena (the batched launches'
  // tables): one upload carries the stripe, its initialised counters and
  // its job tables
  const uint64_t rb_off = (hs.used + 255) & ~(uint64_t)255;
  fl.rb_words = rb_words_for(nc);
  fl.rb_used = 2 * nc + 1;  // word 2 nc: the context's own record during this stripe
  const uint64_t arena_off = (rb_off + 8 * fl.rb_words + 255) & ~(uint64_t)255;
  const uint64_t arena_cap = arena_bytes_for(nc, v1_segments(hs), (nrows_stripe + 2047) / 2048 + 1);
  const uint64_t total = arena_off + arena_cap;
  if (!hs.ensure(total + 64, hs.used)) return early(fail(ORCG_OUT_OF_MEMORY, "pinned staging allocation failed"));
  memset(hs.h + rb_off, 0xff, 8 * nc);
  memset(hs.h + rb_off + 8 * nc, 0, 8 * (fl.rb_words - nc));
  memset(hs.h + rb_off + 8 * (2 * nc), 0xff, 8);
  ds.d_stage = (uint8_t*)ds.pool.get(total + 64);
  if (!ds.d_stage) return early(fail_oom(__LINE__));
  ds.d_rb = (uint64_t*)(ds.d_stage + rb_off);
  ds.d_errs = (unsigned long long*)ds.d_rb;
  ds.d_ones = ds.d_rb + nc;
  if (fl.h_rb_cap < fl.rb_words) {
    if (fl.h_rb) (void)hipHostFree(fl.h_rb);
    fl.h_rb = nullptr;
    fl.h_rb_cap = 0;
    if (hipHostMalloc((void**)&fl.h_rb, fl.rb_words * 8, hipHostMallocDefault) != hipSuccess)
      return early(fail(ORCG_OUT_OF_MEMORY, "pinned allocation failed"));
    fl.h_rb_cap = fl.rb_words;
  }
  if (!fl.done && hipEventCreateWithFlags(&fl.done, hipEventDisableTiming) != hipSuccess) {
    fl.done = nullptr;
    return early(fail(ORCG_DEVICE_ERROR, "event creation failed"));
  }
  for (hipEvent_t* e : {&fl.ev_up0, &fl.ev_up1, &fl.ev_dec})
    if (!*e && hipEventCreate(e) != hipSuccess) *e = nullptr;
  fl.ev_split = fl.ev_up0 && fl.ev_up1 && fl.ev_dec;
  const size_t need_defer = 4 * nc + 16;
  if (fl.defer_cap < need_defer) {
    if (fl.h_defer) (void)hipHostFree(fl.h_defer);
    fl.h_defer = nullptr;
    fl.defer_cap = 0;
    if (hipHostMalloc((void**)&fl.h_defer, need_defer * 8, hipHostMallocDefault) != hipSuccess)
      return early(fail(ORCG_OUT_OF_MEMORY, "pinned allocation failed"));
    fl.defer_cap = need_defer;
  }
  fl.defer_used = 0;
  fl.checks.clear();
  H = &hs;
  D = &ds;
  // the context's own record for this stripe rides the read-back block (the
  // stripe's one copy back replaces sync_ctx's synchronous record read)
  struct OwnRecord {
    Ctx* c;
    unsigned long long* saved;
    ~OwnRecord() { c->d_err = saved; }
  } own_rec{ctx, ctx->d_err};
  ctx->d_err = (unsigned long long*)(ds.d_rb + 2 * nc);
  batch.clear();
  v1_segs.clear();
  batched.clear();
  dict_batch.clear();
  dict_done.clear();
  dict_pre.clear();
  varint_jobs.clear();
  varint_pre.clear();
  dec_batch[0].clear();
  dec_batch[1].clear();
  dec_done.clear();
  scan_jobs.clear();
  scan_done.clear();
  launches.clear();
  const uint64_t nrows = nrows_stripe;
  const int64_t* rg_rows = hs.ngroups ? (const int64_t*)(ds.d_stage + hs.rows_off) : nullptr;
  // the batch: streams (and dictionaries) whose counts the host knows, their
  // job tables staged into the arena before the upload
  int rc = ORCG_OK;
  if (batch_on) {
    ctx->arena_h = hs.h + arena_off;
    ctx->arena_d = ds.d_stage + arena_off;
    ctx->arena_cap = arena_cap;
    ctx->arena_used = 0;
    rc = collect(0, nrows, rg_rows);
    if (!rc && !batch.empty() && (rc = plan_rlev2_multi(ctx, batch.data(), (uint32_t)batch.size(), launches)))
      rc = fail_ctx(rc);
    if (!rc && !v1_segs.empty() && (rc = plan_rlev1_multi(ctx, v1_segs.data(), v1_segs.size(), launches)))
      rc = fail_ctx(rc);
    if (!rc && !dict_batch.empty() &&
        (rc = plan_dict_multi(ctx, dict_batch.data(), (uint32_t)dict_batch.size(), launches)))
      rc = fail_ctx(rc);
    for (int mode = 0; mode < 2 && !rc; ++mode) {
      std::vector<DecJob>& g = dec_batch[mode];
      if (g.empty()) continue;
      uint64_t tiles = 0;
      for (DecJob& j : g) {
        j.tile0 = tiles;
        tiles += (j.len + kVarintTile - 1) / kVarintTile;
      }
      const void* d = nullptr;
      if ((rc = stage_table(ctx, g.data(), g.size() * sizeof(DecJob), &d))) {
        rc = fail_ctx(rc);
        break;
      }
      launches.push_back(MultiLaunch{5, mode, d, (uint32_t)g.size(), tiles, 0});
    }
    for (const ScanJob& j : scan_jobs) launches.push_back(MultiLaunch{6, 0, &j, 1, 0, 0});
    ctx->arena_h = ctx->arena_d = nullptr;
    ctx->arena_cap = 0;
  }
  const uint64_t up = arena_off + ctx->arena_used;
  stage_bytes += up;
  // (uploaded even after a failure above: finish() reads the records back);
  // a small stripe (configs[0]: ~60 KB) is pulled by a kernel from the
  // pinned staging, a large one copied by the DMA engine
  constexpr uint64_t pull_max = 256u << 10;
  if (fl.ev_split && hipEventRecord(fl.ev_up0, ctx->stream) != hipSuccess) fl.ev_split = false;
  const int urc = up <= pull_max && hs.pinned_mapped
                      ? launch_pull(ctx, ds.d_stage, hs.h, up)
                      : hip_check(ctx, hipMemcpyAsync(ds.d_stage, hs.h, up, hipMemcpyHostToDevice, ctx->stream),
                                  "H2D stripe");
  if (urc && !rc) rc = fail_ctx(urc);
  if (fl.ev_split && hipEventRecord(fl.ev_up1, ctx->stream) != hipSuccess) fl.ev_split = false;
  fl.t1 = now_s();
  // A batch of nested or nullable columns' dictionaries only (collect_dicts;
  // configs[4]'s map keys): nothing reads its offsets before the fork's next
  // level, so it runs on side lane 0 beside the stripe's first decodes, not
  // ahead of them on the base stream (4 launches, ~45 us of a C5 stripe)
  pre_on_lane = false;
  Ctx* pre_lane = nullptr;
  if (!rc && !launches.empty() && batched.size() == dict_pre.size() && dict_done.empty() && scan_jobs.empty() &&
      dec_batch[0].empty() && dec_batch[1].empty() && varint_jobs.empty() && side_lanes() > 1 &&
      (ev_pre || hipEventCreateWithFlags(&ev_pre, hipEventDisableTiming) == hipSuccess))
    pre_lane = ctx_lane(ctx, 0);
  if (!rc && pre_lane) {
    rc = hip_check(ctx, hipEventRecord(ctx->ev_fork, ctx->stream), "fork event");
    if (!rc) rc = hip_check(ctx, hipStreamWaitEvent(pre_lane->stream, ctx->ev_fork, 0), "fork wait");
    if (!rc && (rc = run_multi(pre_lane, launches))) ctx->last_error = pre_lane->last_error;
    if (!rc) rc = hip_check(ctx, hipEventRecord(ev_pre, pre_lane->stream), "dictionary batch event");
    if (rc) rc = fail_ctx(rc);
    pre_on_lane = !rc;
  } else if (!rc && !launches.empty() && (rc = timed(0, [&]() -> int { return run_multi(ctx, launches); }))) {
    rc = fail_ctx(rc);
  }
  if (!rc) rc = decode(0, nrows, nullptr, nrows, rg_rows);
  if (pre_on_lane && hipStreamWaitEvent(ctx->stream, ev_pre, 0) != hipSuccess && !rc)
    rc = fail(ORCG_DEVICE_ERROR, "dictionary batch wait failed");
  batched_streams += batched.size();
  fl.rc = rc;
  fl.err_col = err_col;
  fl.err_msg = last_error;
  if (fl.ev_split && hipEventRecord(fl.ev_dec, ctx->stream) != hipSuccess) fl.ev_split = false;
  // the read-back copy, then the flight's event (queued copies land before
  // the buffers are reused)
  if (hipMemcpyAsync(fl.h_rb, ds.d_rb, 8 * fl.rb_used, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipEventRecord(fl.done, ctx->stream) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipStreamSynchronize(ctx->stream);
    if (!fl.rc) {
      fl.rc = ORCG_DEVICE_ERROR;
      fl.err_msg = "read error records";
    }
    // (the records are unreadable: finish() reports fl.rc)
    memset(fl.h_rb, 0xff, 8 * fl.rb_used);
    (void)hipEventRecord(fl.done, ctx->stream);
  }
  fl.enqueued = true;
  H = nullptr;
  D = nullptr;
}

// Device half, host side: the first error in column order, as the reference
// raises them one column at a time, then the stripe's column views.
int orcg_reader::finish(Flight& fl) {
  F = &fl;
  H = fl.hs;
  D = fl.ds;
  HostStage& hs = *fl.hs;
  DevSlot& ds = *fl.ds;
  int rc = fl.rc;
  if (!fl.enqueued) {  // failed before anything was enqueued
    H = nullptr;
    D = nullptr;
    return fail(rc, fl.err_msg);
  }
  err_col = fl.err_col;
  last_error = fl.err_msg;
  rc = first_error(rc);
  fl.checks.clear();
  ds.out.assign(hs.cols.size(), ColOut());
  for (size_t i = 0; i < hs.cols.size(); ++i) {
    const Col& c = hs.cols[i];
    ColOut& o = ds.out[i];
    o.kind = c.kind;
    o.encoding = c.encoding;
    o.decoded = c.decoded && !rc;
    o.n = c.n;
    o.has_nulls = c.has_nulls;
    o.nn = c.nn;
    o.data = c.data;
    o.length = c.length;
    o.offsets = c.offsets;
    o.blob = c.blob;
    o.blob_len = c.blob_len;
    o.secondary = c.secondary;
    o.tags = c.tags;
    o.index = c.index;
    o.dict_offsets = c.dict_offsets;
    o.dict_size = c.dict_offsets ? c.dict_size : 0;
  }
  H = nullptr;
  D = nullptr;
  const double t_end = now_s();
  // the upload's and the decode's GPU time (the flight's events, complete
  // here: first_error waited for `done`); host clocks without them
  float up_ms = 0, dec_ms = 0;
  if (fl.ev_split && hipEventElapsedTime(&up_ms, fl.ev_up0, fl.ev_up1) == hipSuccess &&
      hipEventElapsedTime(&dec_ms, fl.ev_up1, fl.ev_dec) == hipSuccess) {
    timings[3] += up_ms * 1e-3;
    timings[4] += dec_ms * 1e-3;
  } else {
    (void)hipGetLastError();
    timings[3] += fl.t1 - fl.t0;
    timings[4] += t_end - fl.t1;
  }
  // ReaderMetrics (ReaderCall / ReaderInclusiveLatencyUs are counted per
  // caller-facing call: orcg_reader_read_stripe(s), orcg_row_reader_next):
  // the stripe's decompression, I/O and decode work
  madd(kMDecompressCall, hs.n_chunks);
  madd(kMDecompressLatency, (uint64_t)(hs.t_decomp * 1e6));
  madd(kMIOCount, hs.n_io);
  madd(kMIOLatency, (uint64_t)(hs.t_io * 1e6));
  if (metrics_timing) collect_event_times();
  else madd(kMDecodeLatency, (uint64_t)((t_end - fl.t1) * 1e6));
  return rc;
}

int orcg_reader::upload_and_decode(HostStage& hs, DevSlot& ds) {
  issue(hs, ds, flights[0]);
  return finish(flights[0]);
}

// Stripes [first, first + count), pipelined three ways: a host thread
// prepares stripe i + 1 (decompression, plans) while the caller's thread
// issues stripe i (upload, launches) and then finishes stripe i - 1 (its
// synchronisation and host checks) -- so the GPU starts stripe i while the
// host checks stripe i - 1. Stripe i lives in stages[i % 3] and
// flights[i & 1]; the preparer of stripe i waits for stripe i - 3 to be
// finished. One thread for the whole read: a thread per stripe cost more
// than a configs[0] stripe decodes in.
int orcg_reader::read_stripes(uint64_t first, uint64_t count) {
  if (!ctx) return fail(ORCG_INVALID_ARGUMENT, "reader has no device context");
  if (first > footer.stripes.size() || count > footer.stripes.size() - first)
    return fail(ORCG_INVALID_ARGUMENT, "stripe index out of range");
  hipSetDevice(ctx->device);
  for (auto& t : timings) t = 0;
  stream_stats[0] = stream_stats[1] = 0;
  batched_streams = 0;
  stage_bytes = 0;
  while (slots.size() < count) slots.emplace_back(new DevSlot());
  nslots = 0;
  if (count == 0) return ORCG_OK;
  std::mutex pm;
  std::condition_variable pcv;
  uint64_t prepared = 0, released = 0;  // stripes prepared; stripes finished (their stages free)
  bool quit = false;
  std::thread prep([&] {
    for (uint64_t k = 0; k < count; ++k) {
      {
        std::unique_lock<std::mutex> lk(pm);
        pcv.wait(lk, [&] { return quit || k < released + 3; });  // stripe k - 3 released stages[k % 3]
        if (quit) return;
      }
      prepare(first + k, stages[k % 3]);
      {
        std::lock_guard<std::mutex> lk(pm);
        prepared = k + 1;
      }
      pcv.notify_all();
      if (stages[k % 3].rc) return;  // the decode raises it when it reaches stripe k
    }
  });
  auto release = [&](uint64_t n) {
    {
      std::lock_guard<std::mutex> lk(pm);
      released = n;
    }
    pcv.notify_all();
  };
  int rc = ORCG_OK;
  bool pending = false;  // stripe k - 1 issued, not finished
  for (uint64_t k = 0; k <= count; ++k) {
    bool issued = false;
    if (k < count) {
      {
        std::unique_lock<std::mutex> lk(pm);
        pcv.wait(lk, [&] { return prepared > k; });
      }
      HostStage& cur = stages[k % 3];
      timings[0] += cur.t_parse;
      timings[1] += cur.t_decomp;
      timings[2] += cur.t_plan;
      stream_stats[0] += cur.n_pos;
      stream_stats[1] += cur.n_plan;
      if (cur.rc) {
        if (pending) {
          const int prc = finish(flights[(k - 1) & 1]);
          if (!prc) nslots = k;
          rc = prc ? prc : fail(cur.rc, cur.err);
        } else {
          rc = fail(cur.rc, cur.err);
        }
        pending = false;
        break;
      }
      issue(cur, *slots[k], flights[k & 1]);
      issued = true;
    }
    if (pending) {
      const int prc = finish(flights[(k - 1) & 1]);
      release(k);
      if (prc) {
        rc = prc;
        if (issued) {  // let the issued stripe drain before its buffers go
          (void)hipEventSynchronize(flights[k & 1].done);
          issued = false;
        }
        break;
      }
      nslots = k;
    }
    pending = issued;
  }
  {
    std::lock_guard<std::mutex> lk(pm);
    quit = true;
  }
  pcv.notify_all();
  prep.join();
  return rc;
}

// ---- RowReader: batches of at most `capacity` rows over the stripes of a
// byte range (c++/src/Reader.cc RowReaderImpl: ctor :307-363, next
// :1392-1442, seekToRow :428-499, getRowNumber :424-426, markEndOfFile
// :1128-1139, startNextStripe's prefetch :1336-1360).
//
// The GPU decodes a whole stripe into HBM, which is copied once into a pinned
// host slab; each batch is a row range of that slab (per column an element
// range, through list / map offsets and union tags), so next() touches no
// device and waits for nothing but the slab of a new stripe. A worker thread
// per row reader prepares (host decompression), decodes and copies stripe
// s + 1 (and decompresses s + 2) while the caller consumes stripe s. The
// row reader keeps its own RowReaderOptions (include, lazy decoding), its own
// device slot and slabs; decodes take the reader's lock.

// A decoded stripe in pinned host memory.
struct HostSlab {
  uint64_t stripe = ~0ull;
  uint8_t* h = nullptr;
  size_t cap = 0;
  std::vector<ColOut> out;  // host pointers into h
  int rc = ORCG_OK;
  std::string err;
  ~HostSlab() { pinned_free(h); }
};

// The buffers of a decoded column, in the batch layout of
// include/orcg_reader.h: (field, bytes) pairs; col_field reads / rebinds one.
enum ColField { kFNn, kFData, kFLength, kFOffsets, kFBlob, kFSecondary, kFTags, kFIndex, kFDictOffsets };
static void col_buffers(const ColOut& o, const TypeInfo& t, std::vector<std::pair<int, uint64_t>>& b) {
  const uint64_t n = o.n;
  auto add = [&](int f, const void* p, uint64_t bytes) {
    if (p && bytes) b.push_back({f, bytes});
  };
  if (o.has_nulls) add(kFNn, o.nn, n);
  const uint32_t k = o.kind;
  if (k == ORCG_TYPE_DECIMAL) {
    add(kFData, o.data, (t.precision > 18 || t.precision == 0 ? 16 : 8) * n);
  } else if (k == ORCG_TYPE_LIST || k == ORCG_TYPE_MAP) {
    add(kFOffsets, o.offsets, 8 * (n + 1));
  } else if (k == ORCG_TYPE_UNION) {
    add(kFTags, o.tags, n);
    add(kFOffsets, o.offsets, 8 * n);
  } else if (k != ORCG_TYPE_STRUCT) {
    add(kFData, o.data, 8 * n);
  }
  add(kFLength, o.length, 8 * n);
  add(kFSecondary, o.secondary, 8 * n);
  add(kFIndex, o.index, 8 * n);
  add(kFDictOffsets, o.dict_offsets, 8 * (o.dict_size + 1));
  add(kFBlob, o.blob, o.blob_len);
}
static const void* col_get(const ColOut& o, int f) {
  switch (f) {
    case kFNn: return o.nn;
    case kFData: return o.data;
    case kFLength: return o.length;
    case kFOffsets: return o.offsets;
    case kFBlob: return o.blob;
    case kFSecondary: return o.secondary;
    case kFTags: return o.tags;
    case kFIndex: return o.index;
    default: return o.dict_offsets;
  }
}
static void col_set(ColOut& o, int f, const void* p) {
  switch (f) {
    case kFNn: o.nn = (const uint8_t*)p; break;
    case kFData: o.data = p; break;
    case kFLength: o.length = (const int64_t*)p; break;
    case kFOffsets: o.offsets = (const int64_t*)p; break;
    case kFBlob: o.blob = (const uint8_t*)p; break;
    case kFSecondary: o.secondary = (const int64_t*)p; break;
    case kFTags: o.tags = (const uint8_t*)p; break;
    case kFIndex: o.index = (const int64_t*)p; break;
    default: o.dict_offsets = (const int64_t*)p; break;
  }
}

struct orcg_row_reader {
  orcg_reader* r = nullptr;
  // this row reader's RowReaderOptions
  std::vector<uint8_t> selected;
  bool lazy_dict = false;
  uint64_t nstripes = 0, first = 0, last = 0;  // stripes [first, last) are in range
  uint64_t current = 0, row_in_stripe = 0, rows_in_stripe = 0;
  uint64_t previous_row = 0;
  std::vector<uint64_t> first_row;  // firstRowOfStripe_
  uint64_t batch_stripe = ~0ull, batch_row0 = 0, batch_rows = 0;
  std::vector<uint64_t> begin, count;  // per type id: element range of the current batch
  std::vector<uint8_t> in_batch;
  const HostSlab* cur = nullptr;  // the slab of the current batch

  // decode pipeline: host stages, one device slot, two host slabs (stripe
  // s in slab s & 1); slab_state 0 empty, 1 queued / decoding, 2 ready
  HostStage stage[2];
  uint64_t prepared[2] = {~0ull, ~0ull};
  std::unique_ptr<DevSlot> dev{new DevSlot()};
  HostSlab slab[2];
  int slab_state[2] = {0, 0};
  uint64_t slab_want[2] = {~0ull, ~0ull};
  std::thread worker;
  std::mutex m;
  std::condition_variable cv;
  std::string last_error;  // this row reader's last failure (orcg_row_reader_last_error)
  std::deque<uint64_t> jobs;
  bool stop = false;
  // worker seconds: [0] prepare inside a job (host decompression the
  // look-ahead did not do), [1] upload + decode, [2] D2H into the slab,
  // [3] slab (re)allocation, [4] look-ahead prepare; [5] caller waits for a
  // slab (orcg_row_reader_timings)
  std::atomic<uint64_t> prof[6] = {};  // nanoseconds
  uint64_t last_d2h = 0;               // bytes of the last slab copy (debug output)
  // NUMA node of the thread that created the row reader: the caller's
  // batch copies read the slabs, so their pages live there (the copy
  // helpers are placed there too, GpuRowReader.hh CopyPool)
  int node = -1;
  void addp(int i, double sec) { prof[i].fetch_add((uint64_t)(sec * 1e9), std::memory_order_relaxed); }
  // the worker's own context (stream, error record, scratch, queues): the
  // caller's context may be driven by its thread while the worker decodes
  // ahead, e.g. by another reader sharing it
  orcg_ctx* own = nullptr;

  ~orcg_row_reader() {
    {
      std::lock_guard<std::mutex> lk(m);
      stop = true;
      jobs.clear();
    }
    cv.notify_all();
    if (worker.joinable()) worker.join();
    if (own) orcg_ctx_destroy(own);
  }

  void mark_end_of_file() {
    current = last;
    row_in_stripe = 0;
    rows_in_stripe = 0;
    previous_row = last == 0 ? 0 : first_row[last - 1] + r->footer.stripes[last - 1].num_rows;
  }

  // --- worker side -------------------------------------------------------
  // (every decode runs under r->mu with this row reader's options and
  // context as the reader's active ones, orcg_reader::Active; the reader's
  // own options are never touched)
  // D2H of every decoded column of `dev` into the slab: the stripe's
  // buffers sit in one device arena (DevPool), so sorted by address they
  // merge into a few ranges (gaps up to 1 MB copied along), one copy each;
  // then one synchronisation
  int copy_out(HostSlab& sl) {
    sl.out = dev->out;
    struct Buf {
      size_t col;
      int f;
      const uint8_t* d;
      uint64_t bytes;
      size_t range;
    };
    std::vector<Buf> bufs;
    std::vector<std::pair<int, uint64_t>> cb;
    for (size_t i = 0; i < sl.out.size(); ++i) {
      if (!sl.out[i].decoded) continue;
      ColOut& o = sl.out[i];
      if (o.index && o.dict_offsets && o.kind != ORCG_TYPE_DECIMAL) {
        // a dictionary column travels as entry + dictionary (8 B a row
        // instead of 24): the host looks up each row's start and length,
        // as StringDictionaryColumnReader::next does (ColumnReader.cc:561-594)
        o.data = nullptr;
        o.length = nullptr;
      }
      cb.clear();
      col_buffers(o, r->footer.types[i], cb);
      for (auto& x : cb) bufs.push_back(Buf{i, x.first, (const uint8_t*)col_get(sl.out[i], x.first), x.second, 0});
    }
    std::vector<size_t> order(bufs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return bufs[a].d < bufs[b].d; });
    struct Range {
      const uint8_t* d;
      uint64_t bytes, hoff;
    };
    std::vector<Range> rs;
    constexpr uint64_t kGap = 1u << 20;
    for (size_t q : order) {
      Buf& bf = bufs[q];
      if (!rs.empty() && bf.d >= rs.back().d && bf.d <= rs.back().d + rs.back().bytes + kGap) {
        const uint64_t end = (uint64_t)(bf.d - rs.back().d) + bf.bytes;
        rs.back().bytes = std::max(rs.back().bytes, end);
      } else {
        rs.push_back(Range{bf.d, bf.bytes, 0});
      }
      bf.range = rs.size() - 1;
    }
    uint64_t total = 0;
    for (Range& rg : rs) {
      rg.hoff = total;
      total += (rg.bytes + 255) & ~(uint64_t)255;
    }
    if (total > sl.cap) {
      const double ta = now_s();
      pinned_free(sl.h);
      sl.h = nullptr;
      sl.cap = 0;
      const uint64_t ncap = std::max<uint64_t>(total + (total >> 3), 1 << 20);
      if (!(sl.h = (uint8_t*)pinned_alloc(ncap, node)))
        return r->fail(ORCG_OUT_OF_MEMORY, "pinned row batch allocation failed");
      sl.cap = ncap;
      addp(3, now_s() - ta);
    }
    last_d2h = 0;
    for (const Range& rg : rs) last_d2h += rg.bytes;
    for (const Range& rg : rs) {
      const int rc = hip_check(r->ctx, hipMemcpyAsync(sl.h + rg.hoff, rg.d, rg.bytes, hipMemcpyDeviceToHost,
                                                      r->ctx->stream), "D2H row batch");
      if (rc) return r->fail_ctx(rc);
    }
    for (const Buf& bf : bufs) {  // the slab's views point at host memory
      const Range& rg = rs[bf.range];
      col_set(sl.out[bf.col], bf.f, sl.h + rg.hoff + (uint64_t)(bf.d - rg.d));
    }
    const int rc = hip_check(r->ctx, hipStreamSynchronize(r->ctx->stream), "hipStreamSynchronize");
    return rc ? r->fail_ctx(rc) : ORCG_OK;
  }
  void run_job(uint64_t t) {
    HostSlab& sl = slab[t & 1];
    HostStage& hs = stage[t & 1];
    int rc;
    std::string err;
    const double t0 = now_s();
    // host work ahead, concurrently with this stripe's decode and copies:
    // decompress stripe t + 1 into the other stage (stripe t - 1 is done
    // with it); prepare reads only the file and this row reader's selection
    // (when stripe t itself is not prepared yet, as for the first stripe, its
    // decompression goes first: the two would share the host threads and
    // delay the first batch)
    std::thread ahead;
    const uint64_t u = t + 1;
    auto start_ahead = [&] {
      if (u < last && prepared[u & 1] != u) {
        prepared[u & 1] = u;
        ahead = std::thread([this, u] {
          const double tp = now_s();
          (void)r->prepare(u, stage[u & 1], selected);  // a failure is kept in the stage
          addp(4, now_s() - tp);
        });
      }
    };
    if (prepared[t & 1] == t) start_ahead();
    {
      std::lock_guard<std::mutex> lk(r->mu);
      orcg_reader::Active act(r, own, selected, lazy_dict);
      (void)hipSetDevice(r->ctx->device);
      rc = ORCG_OK;
      if (prepared[t & 1] != t) {
        prepared[t & 1] = t;
        rc = r->prepare(t, hs);
        start_ahead();
      } else {
        rc = hs.rc;
      }
      if (rc) err = hs.err;
      const double t1 = now_s();
      if (!rc) {
        const double g3 = r->timings[3], g4 = r->timings[4];
        rc = r->upload_and_decode(hs, *dev);
        const double t2 = now_s();
        if (!rc) rc = copy_out(sl);
        if (rc) err = r->last_error;
        addp(1, t2 - t1);
        addp(2, now_s() - t2);
        if (debug_on("rowreader"))
          fprintf(stderr, "row reader stripe %llu: prepare %.2f ms, upload+decode %.2f ms (GPU upload %.2f, decode %.2f), "
                  "D2H %.2f ms (%.1f MB, %.1f GB/s)\n", (unsigned long long)t, (t1 - t0) * 1e3, (t2 - t1) * 1e3,
                  (r->timings[3] - g3) * 1e3, (r->timings[4] - g4) * 1e3, (now_s() - t2) * 1e3, last_d2h / 1e6,
                  last_d2h / 1e9 / std::max(now_s() - t2, 1e-9));
      }
      addp(0, t1 - t0);
      prepared[t & 1] = ~0ull;  // the stage is reused by stripe t + 2
    }
    {
      std::lock_guard<std::mutex> lk(m);
      sl.stripe = t;
      sl.rc = rc;
      sl.err = err;
      slab_state[t & 1] = 2;
    }
    cv.notify_all();
    if (ahead.joinable()) ahead.join();
  }
  void loop() {
    for (;;) {
      uint64_t t;
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return stop || !jobs.empty(); });
        if (stop) return;
        t = jobs.front();
        jobs.pop_front();
      }
      run_job(t);
    }
  }
  // queue stripe t into slab t & 1 (caller holds m)
  void post(std::unique_lock<std::mutex>& lk, uint64_t t) {
    // a queued / running decode into the same slab finishes first
    cv.wait(lk, [&] { return slab_state[t & 1] != 1; });
    slab_state[t & 1] = 1;
    slab_want[t & 1] = t;
    jobs.push_back(t);
    if (!worker.joinable()) worker = std::thread([this] { loop(); });
    cv.notify_all();
  }

  // --- caller side -------------------------------------------------------
  // make stripe s current (decoding it now if it is not already on its way),
  // then start the decode of s + 1
  int load(uint64_t s) {
    std::unique_lock<std::mutex> lk(m);
    HostSlab& sl = slab[s & 1];
    const bool mine = (slab_state[s & 1] == 2 && sl.stripe == s) || (slab_state[s & 1] == 1 && slab_want[s & 1] == s);
    if (!mine) post(lk, s);
    const double tw = now_s();
    cv.wait(lk, [&] { return slab_state[s & 1] == 2; });
    addp(5, now_s() - tw);
    if (sl.rc) {
      const int rc = sl.rc;
      last_error = sl.err;
      lk.unlock();
      r->fail_user(rc, sl.err);  // also the reader's (its workers write it under r->mu)
      lk.lock();
      slab_state[s & 1] = 0;  // a later seek decodes it again
      cur = nullptr;
      return rc;
    }
    cur = &sl;
    const uint64_t u = s + 1;
    if (u < last && !((slab_state[u & 1] == 2 && slab[u & 1].stripe == u) ||
                      (slab_state[u & 1] == 1 && slab_want[u & 1] == u)))
      post(lk, u);
    return ORCG_OK;
  }
  // element range [b, b + c) of column `id` and, recursively, its children
  void ranges(uint32_t id, uint64_t b, uint64_t c) {
    const ColOut& o = cur->out[id];
    if (!o.decoded) return;
    begin[id] = b;
    count[id] = c;
    in_batch[id] = 1;
    const auto& t = r->footer.types[id];
    if (t.kind == ORCG_TYPE_STRUCT) {
      for (uint32_t st : t.subtypes) ranges(st, b, c);
    } else if (t.kind == ORCG_TYPE_LIST || t.kind == ORCG_TYPE_MAP) {
      const int64_t e0 = o.offsets[b], e1 = o.offsets[b + c];
      for (uint32_t st : t.subtypes) ranges(st, (uint64_t)e0, (uint64_t)(e1 - e0));
    } else if (t.kind == ORCG_TYPE_UNION) {
      // child k's rows are the ranks of this batch's non-null tag-k rows
      for (uint32_t k = 0; k < t.subtypes.size(); ++k) {
        uint64_t cb = ~0ull, cc = 0;
        for (uint64_t i = b; i < b + c; ++i)
          if ((!o.has_nulls || o.nn[i]) && o.tags[i] == k) {
            if (cb == ~0ull) cb = (uint64_t)o.offsets[i];
            ++cc;
          }
        if (cb == ~0ull) cb = 0;  // no row of this batch carries tag k: an empty range
        ranges(t.subtypes[k], cb, cc);
      }
    }
  }
};

static thread_local std::string t_open_error;

extern "C" {

const char* orcg_reader_open_error(void) { return t_open_error.c_str(); }

int orcg_reader_open(orcg_ctx* ctx, const uint8_t* file, uint64_t file_len, orcg_reader** out) {
  if (!out || (file_len && !file)) return ORCG_INVALID_ARGUMENT;
  *out = nullptr;
  std::unique_ptr<orcg_reader> r(new orcg_reader());
  r->own_ctx = ctx;
  r->file = file;
  r->file_len = file_len;
  const int rc = r->open_tail();
  if (rc) {
    t_open_error = r->last_error;
    if (ctx) ctx->last_error = r->last_error;
    return rc;
  }
  *out = r.release();
  return ORCG_OK;
}

int orcg_reader_open_file(orcg_ctx* ctx, const char* path, orcg_reader** out) {
  if (!out || !path) return ORCG_INVALID_ARGUMENT;
  *out = nullptr;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) {
    t_open_error = std::string("Can't open ") + path;
    if (ctx) ctx->last_error = t_open_error;
    return ORCG_INVALID_ARGUMENT;
  }
  struct stat st;
  fstat(fd, &st);
  const uint64_t len = (uint64_t)st.st_size;
  void* m = len ? mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
  close(fd);
  if (len && m == MAP_FAILED) {
    t_open_error = std::string("Can't map ") + path;
    if (ctx) ctx->last_error = t_open_error;
    return ORCG_INVALID_ARGUMENT;
  }
  std::unique_ptr<orcg_reader> r(new orcg_reader());
  r->own_ctx = ctx;
  r->file = (const uint8_t*)m;
  r->file_len = len;
  r->mapped = m;
  const int rc = r->open_tail();
  if (rc) {
    t_open_error = r->last_error;
    if (ctx) ctx->last_error = r->last_error;
    return rc;
  }
  *out = r.release();
  return ORCG_OK;
}

void orcg_reader_destroy(orcg_reader* r) { delete r; }
const char* orcg_reader_last_error(const orcg_reader* r) { return r ? r->last_error.c_str() : "null reader"; }
uint64_t orcg_reader_num_rows(const orcg_reader* r) { return r ? r->footer.num_rows : 0; }
uint64_t orcg_reader_num_stripes(const orcg_reader* r) { return r ? r->footer.stripes.size() : 0; }
uint32_t orcg_reader_row_index_stride(const orcg_reader* r) { return r ? r->footer.row_index_stride : 0; }
uint32_t orcg_reader_compression(const orcg_reader* r) { return r ? r->ps.compression : 0; }
uint64_t orcg_reader_compression_block_size(const orcg_reader* r) { return r ? r->ps.block_size : 0; }
uint32_t orcg_reader_writer_version(const orcg_reader* r) { return r ? r->ps.writer_version : 0; }
uint64_t orcg_reader_content_length(const orcg_reader* r) { return r ? r->footer.content_length : 0; }
const char* orcg_reader_software_version(const orcg_reader* r) {
  if (!r) return "";
  static const char* kNames[] = {"ORC Java", "ORC C++", "Presto", "Scritchley Go", "Trino", "CUDF"};
  auto* rr = const_cast<orcg_reader*>(r);
  const uint32_t id = r->footer.writer;
  rr->software_version = id < 6 ? kNames[id] : "Unknown(" + std::to_string(id) + ")";
  if (r->footer.has_software_version) rr->software_version += " " + r->footer.software_version;
  return rr->software_version.c_str();
}
uint32_t orcg_reader_num_metadata(const orcg_reader* r) { return r ? (uint32_t)r->footer.metadata.size() : 0; }
const char* orcg_reader_metadata_key(const orcg_reader* r, uint32_t i) {
  return r && i < r->footer.metadata.size() ? r->footer.metadata[i].first.c_str() : nullptr;
}
const uint8_t* orcg_reader_metadata_value(const orcg_reader* r, uint32_t i, uint64_t* len) {
  if (!r || i >= r->footer.metadata.size()) return nullptr;
  if (len) *len = r->footer.metadata[i].second.size();
  return (const uint8_t*)r->footer.metadata[i].second.data();
}
int orcg_reader_set_lazy_dictionary(orcg_reader* r, int on) {
  if (!r) return ORCG_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(r->mu);
  r->own_lazy = on != 0;
  return ORCG_OK;
}
int orcg_reader_set_hive11_decimal(orcg_reader* r, int32_t forced_scale, int throw_on_overflow) {
  if (!r || forced_scale < 0 || forced_scale > 38) return ORCG_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(r->mu);
  r->hive11_scale = forced_scale;
  r->hive11_throw = throw_on_overflow != 0;
  return ORCG_OK;
}
int32_t orcg_reader_hive11_scale(const orcg_reader* r) { return r ? r->hive11_scale : 6; }
int orcg_reader_format_version(const orcg_reader* r, uint32_t* major, uint32_t* minor) {
  if (!r || !major || !minor) return ORCG_INVALID_ARGUMENT;
  // the reference reports 0.11 when the version is absent (FileVersion::v_0_11)
  *major = r->ps.version.size() > 0 ? r->ps.version[0] : 0;
  *minor = r->ps.version.size() > 1 ? r->ps.version[1] : 11;
  return ORCG_OK;
}
uint32_t orcg_reader_num_types(const orcg_reader* r) { return r ? (uint32_t)r->footer.types.size() : 0; }
int orcg_reader_type(const orcg_reader* r, uint32_t id, orcg_type_info* out) {
  if (!r || !out || id >= r->footer.types.size()) return ORCG_INVALID_ARGUMENT;
  const TypeInfo& t = r->footer.types[id];
  out->kind = t.kind;
  out->num_subtypes = (uint32_t)t.subtypes.size();
  out->maximum_length = t.maximum_length;
  out->precision = t.precision;
  out->scale = t.scale;
  return ORCG_OK;
}
int orcg_reader_subtypes(const orcg_reader* r, uint32_t id, uint32_t* out, uint32_t cap) {
  if (!r || id >= r->footer.types.size() || (cap && !out)) return ORCG_INVALID_ARGUMENT;
  const auto& st = r->footer.types[id].subtypes;
  for (uint32_t i = 0; i < cap && i < st.size(); ++i) out[i] = st[i];
  return ORCG_OK;
}
const char* orcg_reader_field_name(const orcg_reader* r, uint32_t id, uint32_t i) {
  if (!r || id >= r->footer.types.size() || i >= r->footer.types[id].field_names.size()) return nullptr;
  return r->footer.types[id].field_names[i].c_str();
}
int orcg_reader_stripe(const orcg_reader* r, uint64_t s, orcg_stripe_info* out) {
  if (!r || !out || s >= r->footer.stripes.size()) return ORCG_INVALID_ARGUMENT;
  const StripeInfo& si = r->footer.stripes[s];
  out->offset = si.offset;
  out->index_length = si.index_length;
  out->data_length = si.data_length;
  out->footer_length = si.footer_length;
  out->num_rows = si.num_rows;
  return ORCG_OK;
}

// RowReaderOptions::include by type id: the columns, their subtrees and
// their ancestors (NULL = every column)
static int compute_selection(orcg_reader* r, const uint8_t* include, uint32_t ntypes, std::vector<uint8_t>& sel) {
  const size_t nt = r->footer.types.size();
  sel.assign(nt, 1);
  if (!include) return ORCG_OK;
  if (ntypes > nt) return r->fail_user(ORCG_INVALID_ARGUMENT, "include list longer than the type list");
  std::vector<uint32_t> parent(nt, 0);
  for (size_t i = 0; i < nt; ++i)
    for (uint32_t st : r->footer.types[i].subtypes) parent[st] = (uint32_t)i;
  for (auto& c : sel) c = 0;
  sel[0] = 1;
  for (uint32_t i = 0; i < ntypes; ++i) {
    if (!include[i]) continue;
    for (uint32_t a = i; a != 0; a = parent[a]) sel[a] = 1;
    std::vector<uint32_t> st{i};
    while (!st.empty()) {
      const uint32_t x = st.back();
      st.pop_back();
      sel[x] = 1;
      for (uint32_t y : r->footer.types[x].subtypes) st.push_back(y);
    }
  }
  return ORCG_OK;
}

int orcg_reader_select(orcg_reader* r, const uint8_t* include, uint32_t ntypes) {
  if (!r) return ORCG_INVALID_ARGUMENT;
  std::vector<uint8_t> sel;
  const int rc = compute_selection(r, include, ntypes, sel);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(r->mu);
  r->own_sel.swap(sel);
  return ORCG_OK;
}

int orcg_reader_is_selected(const orcg_reader* r, uint32_t type_id) {
  return r && type_id < r->own_sel.size() && r->own_sel[type_id] ? 1 : 0;
}

// ReaderMetrics::ReaderCall / ReaderInclusiveLatencyUs around a caller-facing
// call (the reference's SCOPED_STOPWATCH in RowReaderImpl::next, Reader.cc:1393)
struct ReaderCallScope {
  orcg_reader* r;
  double t0 = now_s();
  explicit ReaderCallScope(orcg_reader* rr) : r(rr) {}
  ~ReaderCallScope() {
    r->madd(orcg_reader::kMReaderCall, 1);
    r->madd(orcg_reader::kMReaderLatency, (uint64_t)((now_s() - t0) * 1e6));
  }
};

int orcg_reader_read_stripe(orcg_reader* r, uint64_t stripe) {
  if (!r) return ORCG_INVALID_ARGUMENT;
  ReaderCallScope call(r);
  std::lock_guard<std::mutex> lk(r->mu);
  orcg_reader::Active act(r, r->own_ctx, r->own_sel, r->own_lazy);
  return r->read_stripes(stripe, 1);
}

int orcg_reader_bench_stripe_decode(orcg_reader* r, uint64_t stripe, uint32_t iters, double* decode_s, double* h2d_s) {
  if (!r || !decode_s || !h2d_s || iters == 0) return ORCG_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(r->mu);
  orcg_reader::Active act(r, r->own_ctx, r->own_sel, r->own_lazy);
  if (!r->ctx) return r->fail(ORCG_INVALID_ARGUMENT, "reader has no device context");
  if (stripe >= r->footer.stripes.size()) return r->fail(ORCG_INVALID_ARGUMENT, "stripe index out of range");
  hipSetDevice(r->ctx->device);
  int rc = r->prepare(stripe, r->stages[0]);
  if (rc) return rc;
  if (r->slots.empty()) r->slots.emplace_back(new DevSlot());
  // one untimed decode (allocations), then `iters` back-to-back decodes of
  // the prepared stripe: the GPU never waits for host decompression
  rc = r->upload_and_decode(r->stages[0], *r->slots[0]);
  for (auto& t : r->timings) t = 0;
  for (uint32_t i = 0; i < iters && !rc; ++i) rc = r->upload_and_decode(r->stages[0], *r->slots[0]);
  r->nslots = rc ? 0 : 1;
  *decode_s = r->timings[4] / iters;
  *h2d_s = r->timings[3] / iters;
  return rc;
}

int orcg_reader_read_stripes(orcg_reader* r, uint64_t first, uint64_t count) {
  if (!r) return ORCG_INVALID_ARGUMENT;
  ReaderCallScope call(r);
  std::lock_guard<std::mutex> lk(r->mu);
  orcg_reader::Active act(r, r->own_ctx, r->own_sel, r->own_lazy);
  return r->read_stripes(first, count);
}

int orcg_reader_stripe_column(const orcg_reader* r, uint64_t k, uint32_t id, orcg_column_view* out) {
  if (!r || !out || id >= r->footer.types.size() || k >= r->nslots) return ORCG_INVALID_ARGUMENT;
  const ColOut& c = r->slots[k]->out[id];
  memset(out, 0, sizeof(*out));
  out->type_id = id;
  out->kind = r->footer.types[id].kind;
  out->encoding = c.encoding;
  out->decoded = c.decoded ? 1u : 0u;
  if (!c.decoded) return ORCG_OK;  // not selected, or not decodable (view.decoded == 0)
  out->num_elements = c.n;
  out->has_nulls = c.has_nulls ? 1 : 0;
  out->not_null = c.nn;
  out->data = c.data;
  out->length = c.length;
  out->offsets = c.offsets;
  out->blob = c.blob;
  out->blob_len = c.blob_len;
  out->secondary = c.secondary;
  out->tags = c.tags;
  out->index = c.index;
  out->dict_offsets = c.dict_offsets;
  out->dict_size = c.dict_size;
  return ORCG_OK;
}

int orcg_reader_column(const orcg_reader* r, uint32_t id, orcg_column_view* out) {
  return orcg_reader_stripe_column(r, 0, id, out);
}

int orcg_reader_copy_to_host(orcg_reader* r, void* dst, const void* src, uint64_t bytes) {
  if (!r || !r->own_ctx || (bytes && (!dst || !src))) return ORCG_INVALID_ARGUMENT;
  if (!bytes) return ORCG_OK;
  Ctx* c = r->own_ctx;  // never a row reader worker's context
  int rc = hip_check(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream), "D2H");
  if (!rc) rc = sync_ctx(c);
  return rc;
}

int orcg_row_reader_create(orcg_reader* r, const orcg_row_reader_options* o, orcg_row_reader** out) {
  if (!r || !out) return ORCG_INVALID_ARGUMENT;
  *out = nullptr;
  if (!r->own_ctx) return r->fail_user(ORCG_INVALID_ARGUMENT, "reader has no device context");
  const uint64_t off = o ? o->offset : 0;
  const uint64_t len = o ? o->length : ~0ull;
  std::unique_ptr<orcg_row_reader> rr(new orcg_row_reader());
  rr->r = r;
  int rc = compute_selection(r, o ? o->include : nullptr, o && o->include ? o->include_len : 0, rr->selected);
  if (rc) return rc;
  rr->lazy_dict = o && o->lazy_dictionary != 0;
  rr->node = current_numa_node();
  if ((rc = orcg_ctx_create(r->own_ctx->device, &rr->own)) != ORCG_OK)
    return r->fail_user(rc, "row reader context creation failed");
  // the caller's kernel choice, snapshotted once: the worker never reads the
  // caller's context
  rr->own->rlev2_variant = r->own_ctx->rlev2_variant;
  // its side lanes (streams, events, error records) now, not in the first
  // stripe's decode
  if (side_lanes() > 1) (void)ctx_lane(rr->own, side_lanes() - 1);
  const uint64_t ns = r->footer.stripes.size();
  rr->nstripes = ns;
  rr->current = ns;
  rr->last = 0;
  rr->first_row.resize(ns);
  uint64_t total = 0;
  for (uint64_t i = 0; i < ns; ++i) {
    rr->first_row[i] = total;
    const StripeInfo& si = r->footer.stripes[i];
    total += si.num_rows;
    // isStripeInRange: offset in [off, off + len), without wrapping
    if (si.offset >= off && si.offset - off < len) {
      if (i < rr->current) rr->current = i;
      if (i >= rr->last) rr->last = i + 1;
    }
  }
  rr->first = rr->current;
  if (rr->current == 0) rr->previous_row = ~0ull;
  else if (rr->current == ns) rr->previous_row = r->footer.num_rows;
  else rr->previous_row = rr->first_row[rr->first] - 1;
  const size_t nt = r->footer.types.size();
  rr->begin.assign(nt, 0);
  rr->count.assign(nt, 0);
  rr->in_batch.assign(nt, 0);
  // the first stripe's decode starts now, on the worker, so the process's
  // first-use costs (code objects, device and pinned allocations: ~40 ms on
  // configs[4]) overlap the caller's setup instead of its first next()
  if (rr->first < rr->last) {
    std::unique_lock<std::mutex> lk(rr->m);
    rr->post(lk, rr->first);
  }
  *out = rr.release();
  return ORCG_OK;
}

void orcg_row_reader_destroy(orcg_row_reader* rr) { delete rr; }

int orcg_row_reader_is_selected(const orcg_row_reader* rr, uint32_t type_id) {
  return rr && type_id < rr->selected.size() && rr->selected[type_id] ? 1 : 0;
}

int orcg_row_reader_next(orcg_row_reader* rr, uint64_t capacity, uint64_t* rows) {
  if (!rr || !rows) return ORCG_INVALID_ARGUMENT;
  ReaderCallScope call(rr->r);
  *rows = 0;
  std::fill(rr->in_batch.begin(), rr->in_batch.end(), 0);
  rr->batch_rows = 0;
  if (rr->current >= rr->last) {
    rr->mark_end_of_file();
    return ORCG_OK;
  }
  int rc;
  if (rr->row_in_stripe == 0 || !rr->cur || rr->cur->stripe != rr->current) {
    // startNextStripe (its slab was decoded ahead while the last one was read)
    if ((rc = rr->load(rr->current))) return rc;
    rr->rows_in_stripe = rr->r->footer.stripes[rr->current].num_rows;
  }
  const uint64_t n = std::min(capacity, rr->rows_in_stripe - rr->row_in_stripe);
  if (n == 0) {
    rr->mark_end_of_file();
    return ORCG_OK;
  }
  rr->batch_stripe = rr->current;
  rr->batch_row0 = rr->row_in_stripe;
  rr->batch_rows = n;
  rr->ranges(0, rr->row_in_stripe, n);
  rr->previous_row = rr->first_row[rr->current] + rr->row_in_stripe;
  rr->row_in_stripe += n;
  if (rr->row_in_stripe >= rr->rows_in_stripe) {
    rr->current += 1;
    rr->row_in_stripe = 0;
  }
  *rows = n;
  return ORCG_OK;
}

int orcg_row_reader_timings(orcg_row_reader* rr, double* out6) {
  if (!rr || !out6) return ORCG_INVALID_ARGUMENT;
  for (int i = 0; i < 6; ++i) out6[i] = rr->prof[i].load(std::memory_order_relaxed) * 1e-9;
  return ORCG_OK;
}

uint64_t orcg_row_reader_row_number(const orcg_row_reader* rr) { return rr ? rr->previous_row : 0; }

const char* orcg_row_reader_last_error(const orcg_row_reader* rr) { return rr ? rr->last_error.c_str() : "null row reader"; }

uint64_t orcg_row_reader_stripe(const orcg_row_reader* rr) { return rr ? rr->batch_stripe : ~0ull; }

int orcg_row_reader_seek_to_row(orcg_row_reader* rr, uint64_t row) {
  if (!rr) return ORCG_INVALID_ARGUMENT;
  if (rr->last == 0) return ORCG_OK;  // empty file / range
  const uint64_t ns = rr->nstripes;
  const uint64_t nrows = rr->r->footer.num_rows;
  if ((rr->last == ns && row >= nrows) || (rr->last < ns && row >= rr->first_row[rr->last])) {
    rr->current = ns;
    rr->previous_row = nrows;
    return ORCG_OK;
  }
  uint64_t s = 0;
  while (s + 1 < rr->last && rr->first_row[s + 1] <= row) ++s;
  if (s < rr->first) {
    rr->current = ns;
    rr->previous_row = nrows;
    return ORCG_OK;
  }
  rr->previous_row = row;
  rr->current = s;
  rr->row_in_stripe = row - rr->first_row[s];
  int rc = rr->load(s);
  if (rc) return rc;
  rr->rows_in_stripe = rr->r->footer.stripes[s].num_rows;
  return ORCG_OK;
}

int orcg_row_reader_column(const orcg_row_reader* rr, uint32_t id, orcg_column_view* view, uint64_t* begin,
                           uint64_t* count) {
  if (!rr || !view || !begin || !count || id >= rr->in_batch.size()) return ORCG_INVALID_ARGUMENT;
  memset(view, 0, sizeof(*view));
  view->type_id = id;
  view->kind = rr->r->footer.types[id].kind;
  *begin = *count = 0;
  if (!rr->in_batch[id] || !rr->cur) return ORCG_OK;  // no batch, or the column is not decoded
  const ColOut& c = rr->cur->out[id];
  view->encoding = c.encoding;
  view->decoded = c.decoded ? 1u : 0u;
  if (!c.decoded) return ORCG_OK;
  view->num_elements = c.n;
  view->has_nulls = c.has_nulls ? 1 : 0;
  view->not_null = c.nn;
  view->data = c.data;
  view->length = c.length;
  view->offsets = c.offsets;
  view->blob = c.blob;
  view->blob_len = c.blob_len;
  view->secondary = c.secondary;
  view->tags = c.tags;
  view->index = c.index;
  view->dict_offsets = c.dict_offsets;
  view->dict_size = c.dict_size;
  *begin = rr->begin[id];
  *count = rr->count[id];
  return ORCG_OK;
}

int orcg_reader_last_timings(const orcg_reader* r, double* out5) {
  if (!r || !out5) return ORCG_INVALID_ARGUMENT;
  for (int i = 0; i < 5; ++i) out5[i] = r->timings[i];
  return ORCG_OK;
}

int orcg_reader_last_stream_stats(const orcg_reader* r, uint64_t* out2) {
  if (!r || !out2) return ORCG_INVALID_ARGUMENT;
  out2[0] = r->stream_stats[0];
  out2[1] = r->stream_stats[1];
  return ORCG_OK;
}

uint64_t orcg_reader_last_batched_streams(const orcg_reader* r) { return r ? r->batched_streams : 0; }

int orcg_reader_get_metrics(orcg_reader* r, orcg_reader_metrics* out) {
  if (!r || !out) return ORCG_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(r->mu);
  static_assert(sizeof(orcg_reader_metrics) == 14 * sizeof(uint64_t), "orcg_reader_metrics layout");
  uint64_t* o = (uint64_t*)out;
  for (int i = 0; i < 14; ++i) o[i] = r->metrics[i].load(std::memory_order_relaxed);
  return ORCG_OK;
}

int orcg_reader_reset_metrics(orcg_reader* r) {
  if (!r) return ORCG_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(r->mu);
  for (auto& m : r->metrics) m.store(0, std::memory_order_relaxed);
  return ORCG_OK;
}

int orcg_reader_set_metrics_timing(orcg_reader* r, int on) {
  if (!r) return ORCG_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(r->mu);
  r->metrics_timing = on != 0;
  return ORCG_OK;
}
uint64_t orcg_reader_last_stage_bytes(const orcg_reader* r) { return r ? r->stage_bytes : 0; }

int orcg_reader_set_stream_batching(orcg_reader* r, int on) {
  if (!r) return ORCG_INVALID_ARGUMENT;
  r->batch_on = on != 0;
  return ORCG_OK;
}

}  // extern "C"
