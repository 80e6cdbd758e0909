// C++ adapter: the reference's Reader / RowReader -> ColumnVectorBatch surface
// over the liborcgpu file reader (include/orcg_reader.h). Header-only; host
// code only.
//
// Reference interfaces mirrored (apache/orc):
//   orc::createReader, Reader::getNumberOfRows / getNumberOfStripes /
//     getType / getContentLength / getSoftwareVersion / getMetadataKeys /
//     getMetadataValue / createRowReader(RowReaderOptions)
//                                          c++/include/orc/Reader.hh:460-633
//   RowReaderOptions::include / range / setEnableLazyDecoding
//                                          c++/include/orc/Reader.hh:150-300
//   RowReader::createRowBatch(capacity) / next(batch) / getRowNumber /
//     seekToRow                            c++/include/orc/Reader.hh:754-776
//   ColumnVectorBatch family (capacity, numElements, notNull, hasNulls;
//   LongVectorBatch data, DoubleVectorBatch data, StringVectorBatch
//   data/length, EncodedStringVectorBatch index + dictionary,
//   Decimal64VectorBatch values/precision/scale, Decimal128VectorBatch values
//   (Int128 = {highbits, lowbits}), TimestampVectorBatch data / nanoseconds,
//   ListVectorBatch / MapVectorBatch offsets + children, StructVectorBatch
//   fields, UnionVectorBatch tags / offsets / children)
//                                          c++/include/orc/Vector.hh:46-352
//
// next() follows RowReaderImpl::next (c++/src/Reader.cc:1392-1442): at most
// capacity rows, never across a stripe. The GPU decodes a whole stripe into
// HBM once (host decompression, one H2D, HIP kernels) and the row reader's
// worker copies it into a pinned host slab; each batch copies its row range of
// every selected column into the batch's buffers, DataBuffers allocated from
// the caller's MemoryPool (ReaderOptions::setMemoryPool, Reader.hh:123, 163;
// MemoryPool.hh:27-33; PinnedMemoryPool for batches that go to a device
// next). The copies of one batch run on the caller's thread and a few helper
// threads of the row reader (CopyPool). String data pointers point into the
// batch's host copy of the string bytes (the dictionary, or the span of direct
// strings the batch covers). Inside the reference build these stand-in batch
// classes are the orc::*VectorBatch classes themselves (same member names).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <pthread.h>
#include <sched.h>
#include <limits>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/orcg_reader.h"
#include "GpuRleDecoder.hh"

namespace orcg {
namespace cxx {

// orc::MemoryPool (c++/include/orc/MemoryPool.hh:27-33): the caller's
// allocator for batch memory.
class MemoryPool {
 public:
  virtual ~MemoryPool() = default;
  virtual char* malloc(uint64_t size) = 0;
  virtual void free(char* p) = 0;
};
class DefaultMemoryPool : public MemoryPool {
 public:
  char* malloc(uint64_t size) override { return static_cast<char*>(std::malloc(size ? size : 1)); }
  void free(char* p) override { std::free(p); }
};
// orc::getDefaultPool (MemoryPool.cc)
inline MemoryPool* getDefaultPool() {
  static DefaultMemoryPool pool;
  return &pool;
}
// Pinned host memory (orcg_host_alloc): batches a caller DMAs to a device.
class PinnedMemoryPool : public MemoryPool {
 public:
  char* malloc(uint64_t size) override {
    char* p = static_cast<char*>(orcg_host_alloc(size));
    if (!p) throw std::bad_alloc();
    return p;
  }
  void free(char* p) override { orcg_host_free(p); }
};

// orc::DataBuffer<T> (c++/include/orc/MemoryPool.hh:35-80) for trivially
// copyable T: memory from the pool; resize keeps the contents and leaves new
// elements uninitialised, as the reference's does for POD types.
template <typename T>
class DataBuffer {
  static_assert(std::is_trivially_copyable<T>::value, "DataBuffer holds trivially copyable values");

 public:
  explicit DataBuffer(MemoryPool& pool = *getDefaultPool(), uint64_t size = 0) : pool_(&pool) { resize(size); }
  ~DataBuffer() {
    if (buf_) pool_->free(reinterpret_cast<char*>(buf_));
  }
  DataBuffer(const DataBuffer&) = delete;
  DataBuffer& operator=(const DataBuffer&) = delete;
  DataBuffer(DataBuffer&& o) noexcept : pool_(o.pool_), buf_(o.buf_), size_(o.size_), cap_(o.cap_) {
    o.buf_ = nullptr;
    o.size_ = o.cap_ = 0;
  }
  T* data() { return buf_; }
  const T* data() const { return buf_; }
  uint64_t size() const { return size_; }
  uint64_t capacity() const { return cap_; }
  bool empty() const { return size_ == 0; }
  T& operator[](uint64_t i) { return buf_[i]; }
  const T& operator[](uint64_t i) const { return buf_[i]; }
  T* begin() { return buf_; }
  T* end() { return buf_ + size_; }
  const T* begin() const { return buf_; }
  const T* end() const { return buf_ + size_; }
  MemoryPool& getMemoryPool() const { return *pool_; }
  void reserve(uint64_t n) {
    if (n <= cap_) return;
    T* nb = reinterpret_cast<T*>(pool_->malloc(n * sizeof(T)));
    if (size_) memcpy(nb, buf_, size_ * sizeof(T));
    if (buf_) pool_->free(reinterpret_cast<char*>(buf_));
    buf_ = nb;
    cap_ = n;
  }
  void resize(uint64_t n) {
    if (n > cap_) reserve(std::max<uint64_t>(n, cap_ + cap_ / 2));
    size_ = n;
  }
  void assign(uint64_t n, const T& v) {
    resize(n);
    for (uint64_t i = 0; i < n; ++i) buf_[i] = v;
  }
  void zeroOut() {
    if (size_) memset(buf_, 0, size_ * sizeof(T));
  }

 private:
  MemoryPool* pool_;
  T* buf_ = nullptr;
  uint64_t size_ = 0, cap_ = 0;
};

// The copies of one batch, spread over the calling thread and a few helper
// threads. The work is cut into byte-balanced contiguous parts and thread t
// first works through part t: a batch's column layout repeats, so each thread
// writes the same batch buffers every batch and finds them in its own cache
// (claims from one shared counter, which moved the buffers between cores
// batch after batch, measured 63-80 Mrows/s on configs[3] at capacity 1,024
// against 100-107 for fixed parts). A thread done with its part takes what is
// left of the others', so a helper the OS has parked does not hold the batch.
// Helpers spin between batches (a batch of 1,024 rows is ~5-15 us of copying;
// waking sleeping threads per batch would cost more than it saves) and sleep
// after ~50 us without work; after a small batch each helper prefetches the
// slab rows that follow its part, the rows the next batch reads. Besides byte
// copies a task builds a string column's data pointers (and, from a
// dictionary, its lengths): the per-row work of StringVectorBatch.
class CopyPool {
 public:
  struct Task {
    void* dst;
    const void* src;
    uint64_t bytes;              // kind 0: bytes to copy; kinds 1, 2: rows
    int kind = 0;                // 0 memcpy; 1 dst[i] = base + (len[i] > 0 ? src[i] - shift : 0);
                                 // 2 dictionary entries src[i]: dst[i] = base + offs[e],
                                 //   out_len[i] = offs[e + 1] - offs[e] (null rows: base, 0)
    const int64_t* len = nullptr;
    char* base = nullptr;
    int64_t shift = 0;
    int64_t* out_len = nullptr;  // kind 2
    const int64_t* offs = nullptr;
    const char* nn = nullptr;
  };
  static uint64_t weight(const Task& t) { return t.kind == 0 ? t.bytes : t.kind == 1 ? 16 * t.bytes : 24 * t.bytes; }
  static void exec(const Task& t) {
    if (t.kind == 0) {
      if (t.bytes) memcpy(t.dst, t.src, t.bytes);
      return;
    }
    char** d = (char**)t.dst;
    const int64_t* st = (const int64_t*)t.src;
    if (t.kind == 1) {
      for (uint64_t i = 0; i < t.bytes; ++i) d[i] = t.base + (t.len[i] > 0 ? st[i] - t.shift : 0);
      return;
    }
    for (uint64_t i = 0; i < t.bytes; ++i) {
      if (t.nn && !t.nn[i]) {
        d[i] = t.base;
        t.out_len[i] = 0;
      } else {
        const int64_t o = t.offs[st[i]];
        d[i] = t.base + o;
        t.out_len[i] = t.offs[st[i] + 1] - o;
      }
    }
  }
  explicit CopyPool(unsigned helpers) : parts_(helpers + 1) {
    for (unsigned i = 0; i < helpers; ++i) ts_.emplace_back([this, i] { loop(i + 1); });
    // helpers on the caller's NUMA node (the slabs are placed there too):
    // a helper the scheduler put on the other socket copies across it (with
    // threads and slabs left where they fell, configs[4] at capacity 1,024
    // ranged 69-126 Mrows/s from run to run; placed, 104-109)
    cpu_set_t cs;
    if (!ts_.empty() && node_cpus(&cs))
      for (auto& t : ts_) (void)pthread_setaffinity_np(t.native_handle(), sizeof(cs), &cs);
  }
  // the CPUs of the calling thread's NUMA node the process may use
  static bool node_cpus(cpu_set_t* out) {
    unsigned cpu = 0, node = 0;
    cpu_set_t allowed;
    if (getcpu(&cpu, &node) != 0 || sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
    char path[64];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%u/cpulist", node);
    FILE* f = fopen(path, "r");
    if (!f) return false;
    char buf[1024];
    const bool ok = fgets(buf, sizeof buf, f) != nullptr;
    fclose(f);
    if (!ok) return false;
    CPU_ZERO(out);
    for (char* p = buf; *p && *p != '\n';) {  // "0-63,128-191"
      char* e = nullptr;
      const long a = strtol(p, &e, 10);
      if (e == p) return false;
      long b = a;
      if (*e == '-') {
        p = e + 1;
        b = strtol(p, &e, 10);
        if (e == p) return false;
      }
      for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
        if (c >= 0 && CPU_ISSET(c, &allowed)) CPU_SET(c, out);
      p = *e == ',' ? e + 1 : e;
    }
    return CPU_COUNT(out) > 0;
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      stop_flag_.store(true, std::memory_order_relaxed);
    }
    cv_.notify_all();
    for (auto& t : ts_) t.join();
  }
  CopyPool(const CopyPool&) = delete;
  CopyPool& operator=(const CopyPool&) = delete;
  // run every task (cut into <= 64 KB pieces) and return when all are done
  void run(const std::vector<Task>& tasks) {
    uint64_t total = 0;
    for (const Task& t : tasks) total += weight(t);
    if (ts_.empty() || total < (96u << 10)) {
      for (const Task& t : tasks) exec(t);
      return;
    }
    work_.clear();
    constexpr uint64_t piece = 64u << 10;
    for (const Task& t : tasks) {
      if (t.kind == 0) {
        for (uint64_t o = 0; o < t.bytes; o += piece)
          work_.push_back(Task{(char*)t.dst + o, (const char*)t.src + o, std::min(piece, t.bytes - o)});
      } else {
        const uint64_t rows = piece / 16;
        for (uint64_t o = 0; o < t.bytes; o += rows) {
          Task q = t;
          q.dst = (char**)t.dst + o;
          q.src = (const int64_t*)t.src + o;
          q.bytes = std::min(rows, t.bytes - o);
          if (t.len) q.len = t.len + o;
          if (t.out_len) q.out_len = t.out_len + o;
          if (t.nn) q.nn = t.nn + o;
          work_.push_back(q);
        }
      }
    }
    const uint64_t n = work_.size();
    if (n >= kMaxTasks) {
      for (const Task& t : work_) exec(t);
      return;
    }
    // parts: thread t starts on [b_t, b_{t+1}), about total / T bytes each
    const uint64_t T = parts_.size(), g = ++gen_ & kGenMask;
    uint64_t acc = 0, b = 0, p = 0;
    for (uint64_t i = 0; i <= n; ++i) {
      while (p < T && (i == n || acc >= total * (p + 1) / T)) {
        parts_[p].w.store((g << 40) | ((i > b ? i : b) << 20) | b, std::memory_order_relaxed);
        b = std::max(b, i);
        ++p;
      }
      if (i < n) acc += weight(work_[i]);
    }
    prefetch_.store(total <= kPrefetchMax, std::memory_order_relaxed);
    done_.store(0, std::memory_order_relaxed);
    // seq_cst store and load: with release / acquire this store and the
    // sleepers_ load may pass each other (a store-buffer reordering) while a
    // helper going to sleep misses the new generation, and no one wakes it
    go_.store(g, std::memory_order_seq_cst);
    if (sleepers_.load(std::memory_order_seq_cst)) {
      std::lock_guard<std::mutex> lk(m_);
      cv_.notify_all();
    }
    std::vector<std::pair<const char*, uint64_t>> none;
    work(g, 0, none);
    for (uint32_t spin = 1; done_.load(std::memory_order_acquire) < n; ++spin) {
      if ((spin & 0xffff) == 0 && sleepers_.load(std::memory_order_seq_cst)) {
        std::lock_guard<std::mutex> lk(m_);
        cv_.notify_all();
      }
    }
  }

 private:
  static constexpr uint64_t kGenMask = (1u << 24) - 1, kMaxTasks = 1u << 20, kPrefetchMax = 512u << 10;
  // part word: generation (24 bits) | end (20) | next (20); a claim is a
  // compare-and-swap that checks the generation, so a thread still on an
  // older batch never takes a task of the current one
  struct alignas(64) Part {
    std::atomic<uint64_t> w{0};
  };
  void work(uint64_t g, unsigned id, std::vector<std::pair<const char*, uint64_t>>& pf) {
    const bool want_pf = id && prefetch_.load(std::memory_order_relaxed);
    uint64_t mine = 0;
    const unsigned T = (unsigned)parts_.size();
    for (unsigned j = 0; j < T; ++j) {
      std::atomic<uint64_t>& w = parts_[(id + j) % T].w;
      uint64_t c = w.load(std::memory_order_acquire);
      for (;;) {
        const uint64_t next = c & 0xfffff, end = (c >> 20) & 0xfffff;
        if ((c >> 40) != g || next >= end) break;
        if (!w.compare_exchange_weak(c, c + 1, std::memory_order_acq_rel, std::memory_order_acquire)) continue;
        const Task& t = work_[next];
        exec(t);
        ++mine;
        if (want_pf && j == 0) {
          if (t.kind == 0) {
            pf.push_back({(const char*)t.src + t.bytes, t.bytes});
          } else {
            pf.push_back({(const char*)((const int64_t*)t.src + t.bytes), 8 * t.bytes});
            if (t.len) pf.push_back({(const char*)(t.len + t.bytes), 8 * t.bytes});
          }
        }
        ++c;
      }
    }
    if (mine) done_.fetch_add(mine, std::memory_order_acq_rel);
    // (after the batch is released: the caller returns meanwhile; prefetch
    // never faults, a range past the slab's end included)
    for (const auto& r : pf)
      for (uint64_t o = 0; o < r.second; o += 64) __builtin_prefetch(r.first + o, 0, 3);
    pf.clear();
  }
  void loop(unsigned id) {
    uint64_t seen = 0;
    std::vector<std::pair<const char*, uint64_t>> pf;
    for (;;) {
      uint64_t g = 0;
      bool got = false;
      for (int spin = 0; spin < 20000; ++spin) {
        g = go_.load(std::memory_order_acquire);
        if (g != seen) {
          got = true;
          break;
        }
        if (stop_flag_.load(std::memory_order_relaxed)) return;
      }
      if (!got) {
        std::unique_lock<std::mutex> lk(m_);
        sleepers_.fetch_add(1, std::memory_order_seq_cst);
        cv_.wait(lk, [&] { return stop_ || go_.load(std::memory_order_seq_cst) != seen; });
        sleepers_.fetch_sub(1, std::memory_order_acq_rel);
        if (stop_) return;
        g = go_.load(std::memory_order_acquire);
      }
      seen = g;
      work(g, id, pf);
    }
  }
  std::vector<std::thread> ts_;
  std::vector<Task> work_;
  std::vector<Part> parts_;
  uint64_t gen_ = 0;
  std::atomic<uint64_t> go_{0};
  std::atomic<uint64_t> done_{0};
  std::atomic<bool> prefetch_{false};
  std::atomic<int> sleepers_{0};
  std::atomic<bool> stop_flag_{false};
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
};

struct Int128 {  // orc::Int128 member order (c++/include/orc/Int128.hh:325-326)
  int64_t highbits = 0;
  uint64_t lowbits = 0;
};

// which concrete batch a ColumnVectorBatch is (fill() switches on it instead
// of trying dynamic_casts)
enum class BatchClass {
  kLong, kInt, kShort, kByte, kDouble, kFloat, kString, kEncodedString, kDecimal64, kDecimal128, kTimestamp,
  kList, kMap, kStruct, kUnion
};

struct ColumnVectorBatch {
  ColumnVectorBatch(uint32_t kind_, uint64_t cap, MemoryPool& pool, BatchClass cls_)
      : kind(kind_), capacity(cap), notNull(pool, cap), memoryPool(pool), cls(cls_) {}
  virtual ~ColumnVectorBatch() = default;
  uint32_t kind;  // orc::TypeKind
  uint64_t capacity;
  uint64_t numElements = 0;
  DataBuffer<char> notNull;  // the rows' non-null flags (all 1 when !hasNulls)
  bool hasNulls = false;
  bool notNullOnes_ = false;  // (adapter state: notNull holds only 1s)
  bool isEncoded = false;
  MemoryPool& memoryPool;
  const BatchClass cls;
};
#define ORCG_BATCH(Name, Cls)                                              \
  Name(uint32_t k, uint64_t cap, MemoryPool& pool = *getDefaultPool())     \
      : ColumnVectorBatch(k, cap, pool, BatchClass::Cls)
struct LongVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(LongVectorBatch, kLong), data(pool, cap) {}
  DataBuffer<int64_t> data;
};
// RowReaderOptions::setUseTightNumericVector batches (Vector.hh IntegerVectorBatch<T>,
// FloatingVectorBatch<float>): BOOLEAN / BYTE -> Byte, SHORT -> Short, INT ->
// Int, FLOAT -> Float (ColumnReader.cc:1703-1790)
struct IntVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(IntVectorBatch, kInt), data(pool, cap) {}
  DataBuffer<int32_t> data;
};
struct ShortVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(ShortVectorBatch, kShort), data(pool, cap) {}
  DataBuffer<int16_t> data;
};
struct ByteVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(ByteVectorBatch, kByte), data(pool, cap) {}
  DataBuffer<int8_t> data;
};
struct DoubleVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(DoubleVectorBatch, kDouble), data(pool, cap) {}
  DataBuffer<double> data;
};
struct FloatVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(FloatVectorBatch, kFloat), data(pool, cap) {}
  DataBuffer<float> data;
};
struct StringVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(StringVectorBatch, kString), data(pool, cap), length(pool, cap), blob(pool) {}
  DataBuffer<char*> data;
  DataBuffer<int64_t> length;
  DataBuffer<char> blob;  // host copy of the string bytes the batch points into

 protected:
  StringVectorBatch(uint32_t k, uint64_t cap, MemoryPool& pool, BatchClass c)
      : ColumnVectorBatch(k, cap, pool, c), data(pool, cap), length(pool, cap), blob(pool) {}
};
// orc::StringDictionary (Vector.hh:232-254)
struct StringDictionary {
  explicit StringDictionary(MemoryPool& pool = *getDefaultPool()) : dictionaryBlob(pool), dictionaryOffset(pool) {}
  DataBuffer<char> dictionaryBlob;
  DataBuffer<int64_t> dictionaryOffset;
  void getValueByIndex(int64_t index, char*& valPtr, int64_t& length) {
    if (index < 0 || static_cast<uint64_t>(index) + 1 >= dictionaryOffset.size())
      throw std::out_of_range("index out of range.");
    valPtr = dictionaryBlob.data() + dictionaryOffset[index];
    length = dictionaryOffset[index + 1] - dictionaryOffset[index];
  }
};
// orc::EncodedStringVectorBatch (Vector.hh:256-269): with lazy decoding the
// dictionary columns fill index + dictionary only
struct EncodedStringVectorBatch : StringVectorBatch {
  EncodedStringVectorBatch(uint32_t k, uint64_t cap, MemoryPool& pool = *getDefaultPool())
      : StringVectorBatch(k, cap, pool, BatchClass::kEncodedString), index(pool, cap) {}
  std::shared_ptr<StringDictionary> dictionary;
  DataBuffer<int64_t> index;
};
struct Decimal64VectorBatch : ColumnVectorBatch {
  ORCG_BATCH(Decimal64VectorBatch, kDecimal64), values(pool, cap) {}
  int32_t precision = 0, scale = 0;
  DataBuffer<int64_t> values;
};
struct Decimal128VectorBatch : ColumnVectorBatch {
  ORCG_BATCH(Decimal128VectorBatch, kDecimal128), values(pool, cap) {}
  int32_t precision = 0, scale = 0;
  DataBuffer<Int128> values;
};
struct TimestampVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(TimestampVectorBatch, kTimestamp), data(pool, cap), nanoseconds(pool, cap) {}
  DataBuffer<int64_t> data, nanoseconds;
};
struct ListVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(ListVectorBatch, kList), offsets(pool, cap + 1) {}
  DataBuffer<int64_t> offsets;
  std::unique_ptr<ColumnVectorBatch> elements;
};
struct MapVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(MapVectorBatch, kMap), offsets(pool, cap + 1) {}
  DataBuffer<int64_t> offsets;
  std::unique_ptr<ColumnVectorBatch> keys, elements;
};
struct StructVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(StructVectorBatch, kStruct) {}
  std::vector<std::unique_ptr<ColumnVectorBatch>> fields;
};
struct UnionVectorBatch : ColumnVectorBatch {
  ORCG_BATCH(UnionVectorBatch, kUnion), tags(pool, cap), offsets(pool, cap) {}
  DataBuffer<unsigned char> tags;
  DataBuffer<uint64_t> offsets;
  std::vector<std::unique_ptr<ColumnVectorBatch>> children;
};
#undef ORCG_BATCH

// orc::RowReaderOptions (the options the decode path honours)
class RowReaderOptions {
 public:
  RowReaderOptions& include(const std::list<uint64_t>& typeIds) {
    include_ = typeIds;
    hasInclude_ = true;
    return *this;
  }
  RowReaderOptions& range(uint64_t offset, uint64_t length) {
    offset_ = offset;
    length_ = length;
    return *this;
  }
  RowReaderOptions& setEnableLazyDecoding(bool on) {
    lazy_ = on;
    return *this;
  }
  RowReaderOptions& setUseTightNumericVector(bool on) {
    tight_ = on;
    return *this;
  }
  bool getUseTightNumericVector() const { return tight_; }
  uint64_t getOffset() const { return offset_; }
  uint64_t getLength() const { return length_; }
  bool getEnableLazyDecoding() const { return lazy_; }
  bool hasInclude() const { return hasInclude_; }
  const std::list<uint64_t>& getInclude() const { return include_; }

 private:
  std::list<uint64_t> include_;
  bool hasInclude_ = false;
  uint64_t offset_ = 0, length_ = std::numeric_limits<uint64_t>::max();
  bool lazy_ = false;
  bool tight_ = false;
};

// orc::ReaderOptions (c++/include/orc/Reader.hh:112-200): the memory pool
// batches and dictionaries are allocated from.
class ReaderOptions {
 public:
  ReaderOptions& setMemoryPool(MemoryPool& pool) {
    pool_ = &pool;
    return *this;
  }
  MemoryPool* getMemoryPool() const { return pool_; }

 private:
  MemoryPool* pool_ = getDefaultPool();
};

class Reader;

class RowReader {
 public:
  RowReader(Reader& r, const RowReaderOptions& opts);
  ~RowReader() { orcg_row_reader_destroy(rr_); }
  RowReader(const RowReader&) = delete;
  RowReader& operator=(const RowReader&) = delete;
  std::unique_ptr<ColumnVectorBatch> createRowBatch(uint64_t capacity) const;
  bool next(ColumnVectorBatch& batch);
  uint64_t getRowNumber() const { return orcg_row_reader_row_number(rr_); }
  void seekToRow(uint64_t rowNumber);
  // RowReader::getSelectedColumns()[id]
  bool isSelected(uint32_t id) const { return orcg_row_reader_is_selected(rr_, id) != 0; }
  // diagnostics (no reference counterpart): with profiling on, seconds spent
  // in next() on [0] the row reader's C call (waits for a stripe's slab
  // included), [1] fill (views, per-row work), [2] the bulk copies; [3..8]
  // the row reader's own counters (orcg_row_reader_timings)
  void setProfiling(bool on) { prof_on_ = on; }
  std::vector<double> getProfile() const {
    std::vector<double> p(prof_, prof_ + 3);
    double w[6];
    if (orcg_row_reader_timings(rr_, w) == ORCG_OK) p.insert(p.end(), w, w + 6);
    return p;
  }

 private:
  void fill(uint32_t id, ColumnVectorBatch& b);
  bool prof_on_ = false;
  double prof_[3] = {0, 0, 0};
  Reader& r_;
  orcg_row_reader* rr_ = nullptr;
  bool lazy_ = false;
  bool tight_ = false;
  // the current stripe's dictionaries, shared by its batches (lazy decoding:
  // StringDictionary; eager: the blob the batches' data pointers point into,
  // as the reference's batches point into the column reader's dictionary)
  uint64_t dict_stripe_ = ~0ull;
  std::map<uint32_t, std::shared_ptr<StringDictionary>> dicts_;
  // eager blobs: two per column, by stripe parity, reused from stripe to
  // stripe (a caller pool of pinned memory paid one page-locked allocation
  // per column and stripe: configs[0]'s 385 small stripes ran at 6 Mrows/s);
  // the previous stripe's blob stays intact while this stripe's batches fill
  struct Blob {
    DataBuffer<char> buf[2];
    uint64_t stripe[2] = {~0ull, ~0ull};
    explicit Blob(MemoryPool& pool) : buf{DataBuffer<char>(pool), DataBuffer<char>(pool)} {}
  };
  std::map<uint32_t, std::unique_ptr<Blob>> blobs_;
  char* stripe_blob(uint32_t id, const orcg_column_view& v);
  // per type: the children fill() visits (struct: the selected fields) and
  // the type's scale / precision (decimals)
  std::vector<std::vector<uint32_t>> subs_;
  std::vector<uint8_t> subs_known_;
  std::vector<orcg_type_info> types_;
  const std::vector<uint32_t>& subs(uint32_t id, uint32_t kind);
  void new_stripe();
  // the batch's bulk copies (slab -> batch buffers), run together at the end
  // of next() on this thread and the copy pool's helpers
  std::vector<CopyPool::Task> copies_;
  std::unique_ptr<CopyPool> pool_;
  template <typename T>
  void copy(DataBuffer<T>& dst, const void* src, uint64_t count, uint64_t first = 0) {
    dst.resize(count);
    if (count) copies_.push_back(CopyPool::Task{dst.data(), (const T*)src + first, count * sizeof(T)});
  }
};

class Reader {
 public:
  Reader(Context& ctx, const std::string& path, const ReaderOptions& opts = ReaderOptions())
      : ctx_(ctx), pool_(opts.getMemoryPool()) {
    if (orcg_reader_open_file(ctx.get(), path.c_str(), &r_) != ORCG_OK) {
      const std::string m = orcg_reader_open_error();
      throw ParseError(m);
    }
  }
  ~Reader() { orcg_reader_destroy(r_); }
  Reader(const Reader&) = delete;
  Reader& operator=(const Reader&) = delete;
  uint64_t getNumberOfRows() const { return orcg_reader_num_rows(r_); }
  uint64_t getNumberOfStripes() const { return orcg_reader_num_stripes(r_); }
  uint64_t getContentLength() const { return orcg_reader_content_length(r_); }
  uint64_t getRowIndexStride() const { return orcg_reader_row_index_stride(r_); }
  std::string getSoftwareVersion() const { return orcg_reader_software_version(r_); }
  std::list<std::string> getMetadataKeys() const {
    std::list<std::string> keys;
    for (uint32_t i = 0; i < orcg_reader_num_metadata(r_); ++i) keys.push_back(orcg_reader_metadata_key(r_, i));
    return keys;
  }
  bool hasMetadataValue(const std::string& key) const {
    for (const auto& k : getMetadataKeys())
      if (k == key) return true;
    return false;
  }
  std::string getMetadataValue(const std::string& key) const {
    for (uint32_t i = 0; i < orcg_reader_num_metadata(r_); ++i)
      if (key == orcg_reader_metadata_key(r_, i)) {
        uint64_t n = 0;
        const uint8_t* p = orcg_reader_metadata_value(r_, i, &n);
        return std::string((const char*)p, n);
      }
    throw std::range_error("key not found");
  }
  orcg_type_info getType(uint32_t id) const {
    orcg_type_info t;
    check(orcg_reader_type(r_, id, &t));
    return t;
  }
  std::vector<uint32_t> getSubtypes(uint32_t id) const {
    std::vector<uint32_t> s(getType(id).num_subtypes);
    if (!s.empty()) check(orcg_reader_subtypes(r_, id, s.data(), (uint32_t)s.size()));
    return s;
  }
  std::string getFieldName(uint32_t id, uint32_t i) const { return orcg_reader_field_name(r_, id, i); }
  // the selected children of a type (RowReader::getSelectedType's shape)
  std::vector<uint32_t> getSelectedSubtypes(uint32_t id) const {
    std::vector<uint32_t> out;
    for (uint32_t s : getSubtypes(id))
      if (orcg_reader_is_selected(r_, s)) out.push_back(s);
    return out;
  }
  std::vector<std::string> getSelectedFieldNames(uint32_t id) const {
    std::vector<std::string> out;
    const auto subs = getSubtypes(id);
    for (uint32_t i = 0; i < subs.size(); ++i)
      if (orcg_reader_is_selected(r_, subs[i])) out.push_back(getFieldName(id, i));
    return out;
  }
  std::unique_ptr<RowReader> createRowReader() { return createRowReader(RowReaderOptions()); }
  std::unique_ptr<RowReader> createRowReader(const RowReaderOptions& opts) {
    return std::make_unique<RowReader>(*this, opts);
  }
  MemoryPool& getMemoryPool() const { return *pool_; }

  // internals for RowReader
  void check(int rc) const {
    if (rc != ORCG_OK) {
      const char* m = orcg_reader_last_error(r_);
      throwOnError(rc, m ? m : "orcg reader error");
    }
  }
  orcg_reader* get() const { return r_; }

 private:
  Context& ctx_;
  MemoryPool* pool_;
  orcg_reader* r_ = nullptr;
};

using Selected = std::function<bool(uint32_t)>;

inline std::unique_ptr<ColumnVectorBatch> make_batch(const Reader& r, uint32_t id, uint64_t cap, bool lazy,
                                                     const Selected& sel, bool tight = false) {
  const orcg_type_info t = r.getType(id);
  MemoryPool& pool = r.getMemoryPool();
  switch (t.kind) {
    case ORCG_TYPE_BOOLEAN:
    case ORCG_TYPE_BYTE:
      if (tight) return std::make_unique<ByteVectorBatch>(t.kind, cap, pool);
      return std::make_unique<LongVectorBatch>(t.kind, cap, pool);
    case ORCG_TYPE_SHORT:
      if (tight) return std::make_unique<ShortVectorBatch>(t.kind, cap, pool);
      return std::make_unique<LongVectorBatch>(t.kind, cap, pool);
    case ORCG_TYPE_INT:
      if (tight) return std::make_unique<IntVectorBatch>(t.kind, cap, pool);
      return std::make_unique<LongVectorBatch>(t.kind, cap, pool);
    case ORCG_TYPE_FLOAT:
      if (tight) return std::make_unique<FloatVectorBatch>(t.kind, cap, pool);
      return std::make_unique<DoubleVectorBatch>(t.kind, cap, pool);
    case ORCG_TYPE_DOUBLE: return std::make_unique<DoubleVectorBatch>(t.kind, cap, pool);
    case ORCG_TYPE_STRING:
    case ORCG_TYPE_BINARY:
    case ORCG_TYPE_VARCHAR:
    case ORCG_TYPE_CHAR:
      // Type::createRowBatch: an encoded batch when lazy decoding is on
      if (lazy) return std::make_unique<EncodedStringVectorBatch>(t.kind, cap, pool);
      return std::make_unique<StringVectorBatch>(t.kind, cap, pool);
    case ORCG_TYPE_DECIMAL:
      if (t.precision > 18 || t.precision == 0) return std::make_unique<Decimal128VectorBatch>(t.kind, cap, pool);
      return std::make_unique<Decimal64VectorBatch>(t.kind, cap, pool);
    case ORCG_TYPE_TIMESTAMP:
    case ORCG_TYPE_TIMESTAMP_INSTANT: return std::make_unique<TimestampVectorBatch>(t.kind, cap, pool);
    case ORCG_TYPE_LIST: {
      auto b = std::make_unique<ListVectorBatch>(t.kind, cap, pool);
      b->elements = make_batch(r, r.getSubtypes(id)[0], cap, lazy, sel, tight);
      return b;
    }
    case ORCG_TYPE_MAP: {
      auto b = std::make_unique<MapVectorBatch>(t.kind, cap, pool);
      const auto s = r.getSubtypes(id);
      b->keys = make_batch(r, s[0], cap, lazy, sel, tight);
      b->elements = make_batch(r, s[1], cap, lazy, sel, tight);
      return b;
    }
    case ORCG_TYPE_STRUCT: {
      // the selected fields only (Type::createRowBatch of the selected type)
      auto b = std::make_unique<StructVectorBatch>(t.kind, cap, pool);
      for (uint32_t s : r.getSubtypes(id))
        if (sel(s)) b->fields.push_back(make_batch(r, s, cap, lazy, sel, tight));
      return b;
    }
    case ORCG_TYPE_UNION: {
      auto b = std::make_unique<UnionVectorBatch>(t.kind, cap, pool);
      for (uint32_t s : r.getSubtypes(id)) b->children.push_back(make_batch(r, s, cap, lazy, sel, tight));
      return b;
    }
    default: return std::make_unique<LongVectorBatch>(t.kind, cap, pool);
  }
}

inline RowReader::RowReader(Reader& r, const RowReaderOptions& opts)
    : r_(r), lazy_(opts.getEnableLazyDecoding()), tight_(opts.getUseTightNumericVector()) {
  std::vector<uint8_t> inc;
  orcg_row_reader_options o;
  memset(&o, 0, sizeof(o));
  o.offset = opts.getOffset();
  o.length = opts.getLength();
  o.lazy_dictionary = lazy_ ? 1 : 0;
  if (opts.hasInclude()) {
    // RowReaderOptions::include(list<uint64_t>) selects type ids
    const uint32_t nt = orcg_reader_num_types(r.get());
    inc.assign(nt, 0);
    for (uint64_t id : opts.getInclude())
      if (id < nt) inc[id] = 1;
    o.include = inc.data();
    o.include_len = nt;
  }
  r_.check(orcg_row_reader_create(r.get(), &o, &rr_));
  // helper threads for the batch copies: ORCG_COPY_THREADS, else up to 3
  // beside the caller's (a quarter of the host's threads)
  unsigned helpers = 0;
  if (const char* e = getenv("ORCG_COPY_THREADS")) {
    helpers = (unsigned)std::max(0, atoi(e));
  } else {
    const unsigned hc = std::thread::hardware_concurrency();
    helpers = std::min(3u, hc >= 8 ? hc / 4 : 0u);
  }
  pool_.reset(new CopyPool(helpers));
}

inline std::unique_ptr<ColumnVectorBatch> RowReader::createRowBatch(uint64_t capacity) const {
  return make_batch(r_, 0, capacity, lazy_, [this](uint32_t id) { return isSelected(id); }, tight_);
}

inline bool RowReader::next(ColumnVectorBatch& batch) {
  uint64_t rows = 0;
  using clk = std::chrono::steady_clock;
  clk::time_point t0, t1, t2;
  if (prof_on_) t0 = clk::now();
  r_.check(orcg_row_reader_next(rr_, batch.capacity, &rows));
  batch.numElements = rows;
  if (rows == 0) return false;
  if (prof_on_) t1 = clk::now();
  copies_.clear();
  fill(0, batch);
  if (prof_on_) t2 = clk::now();
  pool_->run(copies_);
  if (prof_on_) {
    const clk::time_point t3 = clk::now();
    prof_[0] += std::chrono::duration<double>(t1 - t0).count();
    prof_[1] += std::chrono::duration<double>(t2 - t1).count();
    prof_[2] += std::chrono::duration<double>(t3 - t2).count();
  }
  return true;
}

inline void RowReader::seekToRow(uint64_t rowNumber) { r_.check(orcg_row_reader_seek_to_row(rr_, rowNumber)); }

template <typename T, typename S>
inline void narrow_copy(DataBuffer<T>& dst, const void* src, uint64_t n, uint64_t first) {
  // static_cast<T> of the decoded values, as the reference's decoders narrow
  const S* p = (const S*)src + first;
  dst.resize(n);
  T* d = dst.data();
  for (uint64_t i = 0; i < n; ++i) d[i] = static_cast<T>(p[i]);
}

inline const std::vector<uint32_t>& RowReader::subs(uint32_t id, uint32_t kind) {
  if (subs_.empty()) {
    // sized once for every type: fill() holds a reference across its
    // recursive calls, so the outer vector never reallocates
    const uint32_t nt = orcg_reader_num_types(r_.get());
    subs_.resize(nt);
    subs_known_.assign(nt, 0);
    types_.resize(nt);
  }
  if (id >= subs_.size()) throw InvalidArgument("type id " + std::to_string(id) + " out of range");
  if (!subs_known_[id]) {
    for (uint32_t s : r_.getSubtypes(id))
      if (kind != ORCG_TYPE_STRUCT || isSelected(s)) subs_[id].push_back(s);
    types_[id] = r_.getType(id);
    subs_known_[id] = 1;
  }
  return subs_[id];
}

inline char* RowReader::stripe_blob(uint32_t id, const orcg_column_view& v) {
  new_stripe();
  std::unique_ptr<Blob>& b = blobs_[id];
  if (!b) b.reset(new Blob(r_.getMemoryPool()));
  const int k = (int)(dict_stripe_ & 1);
  if (b->stripe[k] != dict_stripe_) {
    b->buf[k].resize(0);  // (no copy of the old bytes when it grows)
    b->buf[k].resize(v.blob_len);
    if (v.blob_len) memcpy(b->buf[k].data(), v.blob, v.blob_len);
    b->stripe[k] = dict_stripe_;
  }
  return b->buf[k].data();
}

inline void RowReader::new_stripe() {
  const uint64_t stripe = orcg_row_reader_stripe(rr_);
  if (stripe != dict_stripe_) {
    dicts_.clear();
    dict_stripe_ = stripe;
  }
}

// One column of the batch (and its children): views point into the row
// reader's host slab; bulk copies are queued (copies_, run by next()), the
// per-row work (string pointers, offset rebasing, narrowing) done here.
inline void RowReader::fill(uint32_t id, ColumnVectorBatch& b) {
  orcg_column_view v;
  uint64_t first = 0, n = 0;
  r_.check(orcg_row_reader_column(rr_, id, &v, &first, &n));
  if (!v.decoded)  // TIMESTAMP of a non-UTC writer zone (include/orcg_reader.h)
    throw InvalidArgument("column " + std::to_string(id) + " is not decoded by the GPU reader");
  b.numElements = n;
  if (n > b.capacity) b.capacity = n;  // children grow like the reference's resize()
  b.hasNulls = v.has_nulls != 0;
  // notNull: the decoded flags, or all 1s as the reference's PRESENT decode
  // leaves them for a batch without nulls (ColumnReader::next,
  // ColumnReader.cc:81-104), sized with a child's grown capacity; the 1s are
  // rewritten only after a batch with nulls or a growth
  if (b.hasNulls) {
    copy(b.notNull, v.not_null, n, first);
    b.notNullOnes_ = false;
  } else if (!b.notNullOnes_ || b.notNull.size() < n) {
    b.notNull.resize(std::max<uint64_t>(n, b.notNull.size()));
    if (b.notNull.size()) memset(b.notNull.data(), 1, b.notNull.size());
    b.notNullOnes_ = true;
  }
  const std::vector<uint32_t>& subs = this->subs(id, v.kind);
  const char* nn = b.hasNulls ? (const char*)v.not_null + first : nullptr;
  switch (b.cls) {
    case BatchClass::kLong: copy(static_cast<LongVectorBatch&>(b).data, v.data, n, first); break;
    case BatchClass::kInt: narrow_copy<int32_t, int64_t>(static_cast<IntVectorBatch&>(b).data, v.data, n, first); break;
    case BatchClass::kShort:
      narrow_copy<int16_t, int64_t>(static_cast<ShortVectorBatch&>(b).data, v.data, n, first);
      break;
    case BatchClass::kByte: narrow_copy<int8_t, int64_t>(static_cast<ByteVectorBatch&>(b).data, v.data, n, first); break;
    case BatchClass::kDouble: copy(static_cast<DoubleVectorBatch&>(b).data, v.data, n, first); break;
    case BatchClass::kFloat: narrow_copy<float, double>(static_cast<FloatVectorBatch&>(b).data, v.data, n, first); break;
    case BatchClass::kEncodedString:
      if (v.index) {
        // nextEncoded: index + the stripe's dictionary (ColumnReader.cc:596-607),
        // one host dictionary per stripe shared by its batches
        auto& e = static_cast<EncodedStringVectorBatch&>(b);
        e.isEncoded = true;
        copy(e.index, v.index, n, first);
        new_stripe();
        std::shared_ptr<StringDictionary>& dict = dicts_[id];
        if (!dict) {
          dict = std::make_shared<StringDictionary>(r_.getMemoryPool());
          dict->dictionaryBlob.resize(v.blob_len);
          if (v.blob_len) memcpy(dict->dictionaryBlob.data(), v.blob, v.blob_len);
          dict->dictionaryOffset.resize(v.dict_size + 1);
          memcpy(dict->dictionaryOffset.data(), v.dict_offsets, 8 * (v.dict_size + 1));
        }
        e.dictionary = dict;
        e.data.resize(n);
        e.length.resize(n);
        const int64_t* idx = (const int64_t*)v.index + first;
        char** d = e.data.data();
        int64_t* l = e.length.data();
        for (uint64_t i = 0; i < n; ++i) {
          if (nn && !nn[i]) {
            d[i] = nullptr;
            l[i] = 0;
          } else {
            dict->getValueByIndex(idx[i], d[i], l[i]);
          }
        }
        break;
      }
      // an eager (non-dictionary) column in a lazy row reader
      [[fallthrough]];
    case BatchClass::kString: {
      auto& s = static_cast<StringVectorBatch&>(b);
      s.data.resize(n);
      char** d = s.data.data();
      if (v.index && !v.data) {
        // dictionary: the slab holds each row's entry; starts and lengths
        // are looked up in the stripe's dictionary (StringDictionaryColumnReader
        // ::next, ColumnReader.cc:561-594), whose blob is copied once and
        // shared by the stripe's batches
        char* const blob = stripe_blob(id, v);
        s.length.resize(n);
        if (n) {
          CopyPool::Task t{d, (const int64_t*)v.index + first, n, 2};
          t.base = blob;
          t.out_len = s.length.data();
          t.offs = (const int64_t*)v.dict_offsets;
          t.nn = nn;
          copies_.push_back(t);
        }
        break;
      }
      const int64_t* start = (const int64_t*)v.data + first;  // the slab's (start, length) pairs
      const int64_t* len = (const int64_t*)v.length + first;
      copy(s.length, v.length, n, first);
      if (v.index) {
        // dictionary: the stripe's blob, copied once and shared by its batches
        char* const blob = stripe_blob(id, v);
        if (n) copies_.push_back(CopyPool::Task{d, start, n, 1, len, blob, 0});
      } else {
        // direct: the byte span the batch covers (non-empty values' starts
        // ascend with the row: their first and last bound it)
        uint64_t lo = 0, hi = 0, i0 = 0, i1 = n;
        while (i0 < n && len[i0] <= 0) ++i0;
        while (i1 > i0 && len[i1 - 1] <= 0) --i1;
        if (i0 < i1) {
          lo = (uint64_t)start[i0];
          hi = (uint64_t)(start[i1 - 1] + len[i1 - 1]);
          // the decode rejects negative lengths and short blobs; never build
          // pointers outside the stripe's bytes whatever the views say
          if (start[i0] < 0 || hi < lo || hi > v.blob_len)
            throw ParseError("failed to read in StringDirectColumnReader.next");
        }
        copy(s.blob, v.blob, hi - lo, lo);
        if (n) copies_.push_back(CopyPool::Task{d, start, n, 1, len, s.blob.data(), (int64_t)lo});
      }
      break;
    }
    case BatchClass::kDecimal64: {
      auto& d64 = static_cast<Decimal64VectorBatch&>(b);
      d64.precision = (int32_t)types_[id].precision;
      d64.scale = (int32_t)types_[id].scale;
      copy(d64.values, v.data, n, first);
      break;
    }
    case BatchClass::kDecimal128: {
      auto& d128 = static_cast<Decimal128VectorBatch&>(b);
      d128.precision = (int32_t)types_[id].precision;
      // Hive 0.11 decimals: the forced scale (DecimalHive11ColumnReader::next)
      d128.scale = types_[id].precision == 0 ? (int32_t)orcg_reader_hive11_scale(r_.get()) : (int32_t)types_[id].scale;
      copy(d128.values, v.data, n, first);  // [hi, lo] per value = Int128's layout
      break;
    }
    case BatchClass::kTimestamp: {
      auto& ts = static_cast<TimestampVectorBatch&>(b);
      copy(ts.data, v.data, n, first);
      copy(ts.nanoseconds, v.secondary, n, first);
      break;
    }
    case BatchClass::kList:
    case BatchClass::kMap: {
      DataBuffer<int64_t>& offs =
          b.cls == BatchClass::kList ? static_cast<ListVectorBatch&>(b).offsets : static_cast<MapVectorBatch&>(b).offsets;
      const int64_t* src = (const int64_t*)v.offsets + first;
      offs.resize(n + 1);
      const int64_t base = src[0];
      for (uint64_t i = 0; i <= n; ++i) offs[i] = src[i] - base;
      if (b.cls == BatchClass::kList) {
        fill(subs[0], *static_cast<ListVectorBatch&>(b).elements);
      } else {
        auto& mb = static_cast<MapVectorBatch&>(b);
        fill(subs[0], *mb.keys);
        fill(subs[1], *mb.elements);
      }
      break;
    }
    case BatchClass::kStruct: {
      auto& sb = static_cast<StructVectorBatch&>(b);
      for (size_t i = 0; i < subs.size(); ++i) fill(subs[i], *sb.fields[i]);
      break;
    }
    case BatchClass::kUnion: {
      auto& ub = static_cast<UnionVectorBatch&>(b);
      const uint8_t* tags = (const uint8_t*)v.tags + first;
      const int64_t* offs = (const int64_t*)v.offsets + first;
      ub.tags.resize(n);
      if (n) memcpy(ub.tags.data(), tags, n);
      // offsets relative to each child's first row in this batch
      std::vector<int64_t> base(subs.size(), -1);
      for (uint64_t i = 0; i < n; ++i)
        if ((!nn || nn[i]) && tags[i] < subs.size() && base[tags[i]] < 0) base[tags[i]] = offs[i];
      ub.offsets.resize(n);
      for (uint64_t i = 0; i < n; ++i) ub.offsets[i] = (!nn || nn[i]) ? (uint64_t)(offs[i] - base[tags[i]]) : 0;
      for (size_t k = 0; k < subs.size(); ++k) fill(subs[k], *ub.children[k]);
      break;
    }
  }
}

}  // namespace cxx
}  // namespace orcg
