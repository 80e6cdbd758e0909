// Internal declarations shared by the liborcgpu translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/orcg.h"

namespace orcg {

// Device-side error codes (the low byte of the packed device error record).
// Messages are the reference's ParseError texts (c++/src/RleDecoderV2.cc).
enum DevErr : uint32_t {
  kErrNone = 0,
  kErrBadRead = 1,         // "bad read in RleDecoderV2::readByte"            :38
  kErrPatchedPl0 = 2,      // "Corrupt PATCHED_BASE encoded data (pl==0)!"     :307
  kErrPatchedWidth = 3,    // "... (patchBitSize + pgw > 64)!"                 :328-330
  kErrDeltaLength = 4,     // "Illegal run length for delta encoding: 1"       :412-415
  kErrBadSegment = 5,      // positions / segment table not run aligned (InvalidArgument)
  kErrByteBadRead = 6,     // "bad read in nextBuffer" (ByteRLE.cc:364)
  kErrDictIndex = 7,       // "Entry index out of range in StringDictionaryColumn" (ColumnReader.cc:578)
  kErrV1BadRead = 8,       // "bad read in readByte" (RLEv1.cc:141-146)
  kErrDecimalScale = 9,    // "Decimal scale out of range" (ColumnReader.cc:1348)
  kErrHive11Overflow = 10, // "Hive 0.11 decimal was more than 38 digits." (ColumnReader.cc:1654)
  // Java face (RunLengthIntegerReaderV2.java, readPatchedBaseValues :149-260)
  kErrJavaCorrupt = 11,    // IOException "Corruption in ORC data encountered. ..." (pw + pgw > 64, :196-200)
  kErrJavaPatchIndex = 12, // ArrayIndexOutOfBoundsException: pl == 0 reads unpackedPatch[0] (:207)
};

const char* dev_error_message(uint32_t code);
int dev_error_status(uint32_t code);

// The device error record: min over (value_index << 8 | code). ~0 = none.
constexpr unsigned long long kNoError = ~0ull;

struct Ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  unsigned long long* d_err = nullptr;  // device error record
  std::string last_error;
  uint64_t last_error_value = 0;
  // grow-only device scratch
  // scratch slots: 0 stream, 1 segments, 2 dense values, 3 not-null,
  // 4 column output, 5 tile counts, 6 tile offsets, 7 misc
  void* d_scratch[8] = {};
  size_t scratch_cap[8] = {};
  void* h_pinned = nullptr;
  size_t pinned_cap = 0;
  int rlev2_variant = ORCG_RLEV2_TILED;  // which RLEv2 kernel to launch
  void* d_defer = nullptr;  // RLEv2 short-run segment queue (rlev2_tiled.hip defer_queue)
  uint64_t defer_cap = 0;
  uint64_t defer_seq = 0;  // serial + drain launch pairs so far (their entries' stamps)
  int num_cus = 0;         // compute units of `device` (0 = not queried yet)
  // decoupled look-back status words (column_kernels.hip lb_status): one
  // buffer per context (its launches are ordered), a 16-bit epoch per launch
  void* d_lb = nullptr;
  uint64_t lb_cap = 0;
  uint32_t lb_epoch = 0;
  // two-pass RLEv2 run table and segment headers (RunTab), grow-only
  void* d_rtab = nullptr;
  uint64_t rtab_cap = 0;
  void* d_rhdr = nullptr;
  uint64_t rhdr_cap = 0;
  // job tables of multi-stream launches: a pinned host ring and its device
  // mirror, in bytes (stage_table)
  void* h_jobs = nullptr;
  void* d_jobs = nullptr;
  uint64_t jobs_cap = 0, jobs_used = 0;
  // or an arena the caller uploads itself (the file reader's stripe staging):
  // stage_table writes a table to arena_h and hands out arena_d; the caller
  // orders the arena's upload before the launches (plan_* / run_multi)
  uint8_t* arena_h = nullptr;
  uint8_t* arena_d = nullptr;
  uint64_t arena_cap = 0, arena_used = 0;
  // side contexts (own stream, scratch, queues) the file reader decodes
  // sibling column subtrees on concurrently, forked from and joined back into
  // this context's stream with events; created on first use (ctx_lane)
  std::vector<Ctx*> lanes;
  hipEvent_t ev_fork = nullptr;
  std::vector<hipEvent_t> ev_join;
};

// Side context k of `base` (created on first use, settings copied from base);
// nullptr if it cannot be created.
Ctx* ctx_lane(Ctx* base, size_t k);
// One no-op launch per kernel file on `s`: HIP loads a file's code object at
// its first launch (tens of ms for all of them), so the first context of a
// process pays it at creation instead of inside its first decode
// (ORCG_WARMUP=0: lazily).
void warm_rlev2_walk(hipStream_t s);
void warm_rlev2_tiled(hipStream_t s);
void warm_byterle(hipStream_t s);
void warm_columns(hipStream_t s);
void warm_rlev1(hipStream_t s);
void warm_decimal(hipStream_t s);

// Side streams the file reader may use (ORCG_LANES, default 4; 1 = none).
unsigned side_lanes();

// One RLEv2 stream of a multi-stream launch: its bytes, segments, output
// (int64) and value count; seg_base = the launch-wide index of its first
// segment (set by the launcher). Segments are either a table ({byte offset,
// value index} per segment) or, for row-index streams of a column without
// nulls, the row index itself: {byte offset, values to skip, bits} triplets
// (trip) and the first row of each row group (rows): value index = rows[g] -
// skip, clamped at 0, as rg_segtab_kernel computes it.
struct RleJob {
  const uint8_t* src;
  uint64_t src_len;
  const uint64_t* segtab;
  const int64_t* trip;
  const int64_t* rows;
  uint64_t nsegs;
  void* dst;
  uint64_t nvalues;
  uint64_t seg_base;
  uint32_t is_signed;
  uint32_t tab_base;  // two-pass launches: the job's first run-table entry (set by the launcher)
  unsigned long long* err;  // the job's device error record (the reader's per-column word), or null = the launch's
  const uint64_t* dcount;   // non-null: the value count on the device (nvalues is then the output's capacity)
};

// One RLEv1 segment of a multi-stream launch, built on the host from the
// stream's plan or row index: a workgroup reads its whole description in one
// load (no job search through the table on the device).
struct V1SegDesc {
  const uint8_t* src;
  uint64_t src_len;
  uint64_t seg_start, vi;  // first byte (a group header) and its first value
  uint64_t seg_end, v_next;  // the next segment's, or (src_len, ~0) for the last
  void* dst;               // int64 values [0, nvalues)
  uint64_t nvalues;
  unsigned long long* err;
  uint32_t is_signed, pad;
};

int set_error(Ctx* ctx, int status, const std::string& msg);
// ORCG_DEBUG=topic[,topic...]: stderr diagnostics of that topic (alloc,
// stale, rowreader, defer, jobs)
bool debug_on(const char* topic);
// ORCG_DEBUG_STALE=1: report (and clear) a HIP error left pending on this
// host thread at `where` (launch checks read hipGetLastError).
void debug_stale(const char* where);
// page-locked host memory (transparent huge pages + hipHostRegister for large
// buffers, hipHostMalloc otherwise); pinned_free takes either kind
// node >= 0: large buffers prefer that NUMA node's memory (the node of the
// thread that will read them)
void* pinned_alloc(size_t bytes, int node = -1);
// the NUMA node the calling thread runs on (-1 if unknown)
int current_numa_node();
void pinned_free(void* p);
int hip_check(Ctx* ctx, hipError_t e, const char* what);
int scratch(Ctx* ctx, int slot, size_t bytes, void** out);
// Wait for the context stream and fold the device error record into a status.
int sync_ctx(Ctx* ctx);

// Kernel launchers (rlev2_kernels.hip). segtab is either orcg_segment[] or the
// row-index positions array (positions_mode, with rows_per_group).
// java: 0 = the C++ reader's rules; 1 = Java's RunLengthIntegerReaderV2
// (DELTA runs of one value with a bit width decode two values, PATCHED_BASE
// with pl == 0 fails as Java's array index, pw + pgw > 64 fails with Java's
// IOException); 2 = Java with skipCorrupt (pw + pgw > 64 decodes, :196-202).
int launch_rlev2_decode(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                        const uint64_t* d_segtab, uint64_t nsegs, bool positions_mode,
                        uint64_t rows_per_group, uint64_t value_begin, uint64_t nvalues,
                        void* d_dst, int dst_bytes, int java = 0);


// Two-pass short-run RLEv2 decode (DESIGN.md §3.1 "Two passes"): the union
// instance's dense (short-run) passes write their run starts to `tab` instead
// of expanding them, and rlev2_expand_kernel then expands every segment's
// tabled runs in value slices of `slice` values (spg slices per segment), a
// workgroup per slice. Per launch-wide segment g, hdr[g * (kRtHdr + spg) + i]:
// [0] table entries, [1] values the passes reached (segment-relative), [2..3]
// the segment's first value index, [4] its first table entry, [kRtHdr + k]
// the entry to start slice k from (k >= 1), [5] the segment's job (multi-
// stream launches). An entry is the run's stream byte
// offset | its first value (segment-relative) << 32. Runs of passes the first
// kernel expands itself (long runs, values past spg * slice) are not tabled.
constexpr uint32_t kRtHdr = 6;
constexpr uint32_t kSliceMax = 1024;
struct RunTab {
  uint64_t* tab;
  uint32_t* hdr;
  uint32_t spg;
  uint32_t slice;
};
// The second pass over `nsegs` launch-wide segments (single stream: d_src ..
// d_count as launch_rlev2_tiled; multi-stream: jobs_d, int64 output).
int launch_rlev2_expand(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed, uint64_t value_begin,
                        uint64_t nvalues, void* d_dst, int dst_bytes, const uint64_t* d_count, const RleJob* jobs_d,
                        uint32_t njobs, uint64_t nsegs, const RunTab& rt);
void warm_rlev2_expand(hipStream_t s);

// RLEv2 kernel variants a context accepts (orcg_rlev2_variants): 0 default,
// 1 wave-walk, and pins of single tiled instances (launch_rlev2_tiled).
constexpr int kMaxRlev2Variant = 8;
bool rlev2_variant_valid(int v);
// d_count (may be null): the value count on the device, nvalues then
// bounds the output only.
int launch_rlev2_tiled(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                       const uint64_t* d_segtab, uint64_t nsegs, bool positions_mode,
                       uint64_t rows_per_group, uint64_t value_begin, uint64_t nvalues,
                       void* d_dst, int dst_bytes, const uint64_t* d_count = nullptr);

// Every stream of `jobs` (segment-table mode, int64 output) in one launch per
// instance the default's density rule picks (or the pinned variant);
// variant 1 falls back to one launch per stream.
int launch_rlev2_multi(Ctx* ctx, const RleJob* jobs, uint32_t njobs);
// Variants whose instances take job tables with row-index segments (RleJob::trip).
bool rlev2_multi_capable(int variant);
// Copies a job table into the context's arena (no copy enqueued) or its
// pinned ring and device mirror (an H2D ordered on ctx->stream); *out = the
// device copy.
int stage_table(Ctx* ctx, const void* src, size_t bytes, const void** out);
inline int stage_rle_jobs(Ctx* ctx, const RleJob* jobs, uint32_t n, const RleJob** out) {
  return stage_table(ctx, jobs, (size_t)n * sizeof(RleJob), (const void**)out);
}

// A multi-stream launch planned ahead of the upload that carries its job
// table (stage_table in arena mode): plan_* group, order and stage the
// jobs; run_multi enqueues the kernels (RLEv2 instances on side lanes).
struct MultiLaunch {
  int kind;           // 0 RLEv2 instance `variant`, 1 RLEv1, 2 dictionaries, 3 pinned single-stream RLEv2
                      // (host job), 4 varint tile counts + scan (host VarintJob), 5 decimal columns (DecJob
                      // table, `variant` = the decimal mode), 6 a direct string column's length scan (host
                      // ScanJob)
  int variant;
  const void* d_jobs;
  uint32_t njobs;
  uint64_t grid;      // segments / tiles
  uint64_t values;
  // two-pass RLEv2 launch (kind 0, spg > 0): run-table entries, slices per
  // segment and values per slice (RunTab)
  uint64_t tab_entries = 0;
  uint32_t spg = 0, slice = 0;
};
int plan_rlev2_multi(Ctx* ctx, const RleJob* jobs, uint32_t njobs, std::vector<MultiLaunch>& out);
// A varint DATA stream's tile counts and their scan (the first value of each
// kVarintTile-byte tile) ahead of its decode: the decimal columns' first two
// launches, run before the batch's join (they need only the stream bytes).
struct VarintJob {
  const uint8_t* src;
  uint64_t len;
  int64_t* counts;
  int64_t* base;    // ntiles + 1
  uint64_t* total;  // the values in the stream (read-back slot)
};
// A direct string column's starts: the exclusive scan of its batched LENGTH
// stream with computeSize's checks (launch_exclusive_scan's flags / total),
// run after the join beside the dictionaries and decimals.
struct ScanJob {
  const int64_t* in;
  uint64_t n;
  int64_t* out;     // n + 1
  uint64_t* flags;  // 2 (read-back slots)
  uint64_t* total;  // read-back slot
};
int plan_rlev1_multi(Ctx* ctx, const V1SegDesc* segs, uint64_t nsegs, std::vector<MultiLaunch>& out);
int run_multi(Ctx* ctx, const std::vector<MultiLaunch>& launches);

// d_ones (boolean mode, may be null): += the set rows written (a PRESENT
// stream's non-null rows), one atomic per wave. d_nout (may be null): the
// output count on the device (nout then bounds the output only).
int launch_byterle(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, const uint64_t* d_segtab, uint64_t nsegs,
                   bool boolean, uint64_t begin, uint64_t nout, uint8_t* d_dst, uint64_t* d_ones = nullptr,
                   const uint64_t* d_nout = nullptr);
int launch_rlev1(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed, const uint64_t* d_segtab,
                 uint64_t nsegs, uint64_t value_begin, uint64_t nvalues, void* d_dst, int dst_bytes);
// The segments of several RLEv1 streams (int64 output) in one launch per
// chunk width (rlev1_kernel's narrow instance for short segments).
int launch_rlev1_multi(Ctx* ctx, const V1SegDesc* segs, uint64_t nsegs);
int launch_rlev1_jobs(Ctx* ctx, const V1SegDesc* d_segs, uint64_t nsegs, int chunk);
int launch_scatter(Ctx* ctx, const void* d_dense, const uint8_t* d_nn, uint64_t n, void* d_out, int width,
                   int fill_mode, int64_t fill);
// (d_summary, may be null: [0] blob bytes, [1] any negative length)
int launch_dict_offsets(Ctx* ctx, const int64_t* d_lengths, uint64_t dict_size, int64_t* d_offsets,
                        uint64_t* d_summary = nullptr);
int launch_dict_gather(Ctx* ctx, const void* d_idx, int idx_width, const uint8_t* d_nn, uint64_t n,
                       const int64_t* d_offsets, uint64_t dict_size, int64_t* d_start, int64_t* d_len);
// One dictionary column of a batched launch (dict_multi_kernel): entry
// lengths -> offsets + {blob bytes, negative-length flag} summary, and the
// bounds-checked gather of n rows (n = 0: offsets only, lazy decoding).
constexpr uint32_t kDictLds = 4096;  // largest dictionary a batch takes
struct DictJob {
  const int64_t* lengths;
  uint64_t dict_size;
  int64_t* offsets;   // dict_size + 1
  uint64_t* summary;  // [0] blob bytes, [1] any negative length
  const int64_t* idx;
  const uint8_t* nn;  // row not-null mask, or null
  uint64_t n;
  int64_t* start;
  int64_t* len;
  unsigned long long* err;
  uint64_t tile_base;  // set by the launcher
};
int launch_dict_multi(Ctx* ctx, const DictJob* jobs, uint32_t njobs);
int plan_dict_multi(Ctx* ctx, const DictJob* jobs, uint32_t njobs, std::vector<MultiLaunch>& out);
int launch_dict_jobs(Ctx* ctx, const DictJob* d_jobs, uint32_t njobs, uint64_t tiles);

// Varint decimals (decimal_kernels.hip): per-tile (kVarintTile bytes) terminator counts,
// then (after an exclusive scan of the counts) the decode + rescale into
// int64 (Decimal64) or [hi, lo] int64 pairs (Decimal128, orc::Int128 layout).
int launch_varint_tile_counts(Ctx* ctx, const uint8_t* d_src, uint64_t len, int64_t* d_counts, uint64_t* ntiles);
constexpr uint64_t kVarintTile = 4096;
// mode: 0 Decimal64, 1 Decimal128, 2 Hive 0.11 (overflow raises), 3 Hive 0.11
// with overflowing values nulled (d_keep[k] = 0; 1 otherwise)
int launch_varint_decimal(Ctx* ctx, const uint8_t* d_src, uint64_t len, const int64_t* d_tile_base,
                          const int64_t* d_scales, uint64_t nvalues, int32_t scale, int mode, void* d_out,
                          uint8_t* d_keep = nullptr);
// One decimal column of a batched launch (mode 0 Decimal64 / 1 Decimal128,
// no nulls): varint DATA, its tile bases, the decoded SECONDARY scales;
// tile0 = its first launch-wide tile (set by the planner).
struct DecJob {
  const uint8_t* src;
  uint64_t len;
  const int64_t* tile_base;
  const int64_t* scales;
  uint64_t nvalues;
  void* out;
  unsigned long long* err;
  uint64_t tile0;
  int32_t scale;
  int32_t pad;
};
int launch_decimal_jobs(Ctx* ctx, const DecJob* d_jobs, uint32_t njobs, uint64_t tiles, int mode);
// TimestampColumnReader value construction, in place.
int launch_timestamp(Ctx* ctx, int64_t* d_secs, int64_t* d_nanos, uint64_t n, int64_t epoch);

// Row-index segmentation (column_kernels.hip): prefix[g] = non-zero bytes of
// mask before row rows[g] (counts: scratch of G entries; prefix: G + 1);
// segment table from {offset, skip, bit skip} triplets; list / map child row
// group starts.
int launch_rg_prefix(Ctx* ctx, const uint8_t* d_mask, uint64_t n, const int64_t* d_rows, uint64_t G,
                     int64_t* d_counts, int64_t* d_prefix);
int launch_rg_segtab(Ctx* ctx, const int64_t* d_trip, const int64_t* d_prefix, uint64_t G, bool boolean,
                     uint64_t* d_seg);
int launch_rg_child_rows(Ctx* ctx, const int64_t* d_offsets, const int64_t* d_rows, uint64_t G, int64_t* d_out);
// rg_prefix + rg_segtab in one launch (decoupled look-back over the row
// groups' counts): d_prefix (G + 1 entries) and the segment table.
int launch_rg_prefix_segtab(Ctx* ctx, const uint8_t* d_mask, uint64_t n, const int64_t* d_rows, uint64_t G,
                            const int64_t* d_trip, bool boolean, int64_t* d_prefix, uint64_t* d_seg);

// UNION tags (UnionColumnReader): flags[j] = tags[j] == k; the first tag >=
// nchildren as (index << 8 | tag), ~0 when none; offsets[j] = scan_k[j] for
// the rows with tag k.
int launch_union_flags(Ctx* ctx, const uint8_t* d_tags, uint64_t n, uint32_t k, int64_t* d_flags);
int launch_union_check(Ctx* ctx, const uint8_t* d_tags, uint64_t n, uint32_t nchildren, uint64_t* d_first_bad);
int launch_union_offsets(Ctx* ctx, const uint8_t* d_tags, uint64_t n, uint32_t k, const int64_t* d_scan_k,
                         int64_t* d_offsets);

// Multi-workgroup exclusive scan: d_out[0..n] (n + 1 entries). Scratch 7.
// d_flags (may be null; zero on entry): StringDirect length checks fused into
// the scan, [0] |= 1 for a negative input, [1] |= 1 when the total wraps.
// d_total (may be null): the total (d_out[n]) also written there (e.g. a
// slot of the reader's read-back block: no separate copy).
int launch_exclusive_scan(Ctx* ctx, const int64_t* d_in, uint64_t n, int64_t* d_out, uint64_t* d_flags = nullptr,
                          uint64_t* d_total = nullptr);
// Number of non-zero bytes of d_nn[0..n) into *d_total (device). Scratch 5, 6.
int launch_count_nonzero(Ctx* ctx, const uint8_t* d_nn, uint64_t n, uint64_t* d_total);
// *d_flag = 1 if any d_v[i] < 0, else 0.
int launch_flag_negative(Ctx* ctx, const int64_t* d_v, uint64_t n, uint64_t* d_flag);
enum WidenKind { kWidenI8 = 0, kWidenU8 = 1, kWidenF32 = 2 };
int launch_widen(Ctx* ctx, const void* d_in, int kind, uint64_t n, void* d_out);
// Host (pinned, device-mapped) -> device copy by a kernel on ctx->stream;
// both buffers 16-byte aligned, rounded up to whole 16-byte words.
int launch_pull(Ctx* ctx, void* d_dst, const void* h_src, uint64_t bytes);
// up to kPublishMax device int64 counts -> d_dst (coherent pinned memory),
// then *d_flag = gen (system-scope release): the host polls the flag
constexpr uint32_t kPublishMax = 16;
struct PublishArgs {
  const int64_t* src[kPublishMax];
  uint32_t n;
};
int launch_publish(Ctx* ctx, const PublishArgs& a, uint64_t* d_dst, uint64_t* d_flag, uint64_t gen);

// Dispatch on ctx->rlev2_variant.
inline int launch_rlev2(Ctx* ctx, const uint8_t* d_src, uint64_t src_len, int is_signed,
                        const uint64_t* d_segtab, uint64_t nsegs, bool positions_mode,
                        uint64_t rows_per_group, uint64_t value_begin, uint64_t nvalues,
                        void* d_dst, int dst_bytes) {
  if (ctx->rlev2_variant == ORCG_RLEV2_WAVE_WALK)
    return launch_rlev2_decode(ctx, d_src, src_len, is_signed, d_segtab, nsegs, positions_mode,
                               rows_per_group, value_begin, nvalues, d_dst, dst_bytes);
  return launch_rlev2_tiled(ctx, d_src, src_len, is_signed, d_segtab, nsegs, positions_mode,
                            rows_per_group, value_begin, nvalues, d_dst, dst_bytes);
}

}  // namespace orcg

struct orcg_ctx : orcg::Ctx {};

// Host run walk result (RLEv2 or byte RLE): segment cuts, decodable values,
// first corrupt run.
struct orcg_rlev2_plan {
  std::vector<orcg_segment> segs;
  uint64_t values = 0;
  uint32_t err = orcg::kErrNone;
  uint64_t err_at = 0;
};

orcg_rlev2_plan* make_plan(const uint8_t* src, uint64_t len, uint64_t max_bytes, uint64_t max_values, int java = 0);
namespace orcg {
// The RLEv2 run at `pos` (host): kErrNone with its value count and end, or a DevErr.
uint32_t host_parse_run(const uint8_t* s, uint64_t len, uint64_t pos, uint64_t* run_len, uint64_t* run_end);
}  // namespace orcg
orcg_rlev2_plan* make_v1_plan(const uint8_t* src, uint64_t len, uint64_t max_bytes, uint64_t max_values);
orcg_rlev2_plan* make_byte_plan(const uint8_t* src, uint64_t len, uint64_t max_bytes, uint64_t max_values);
// H2D + RLEv2 decode of the first `count` values + D2H into host `out`.
int decode_host_dense(orcg::Ctx* c, const uint8_t* src, uint64_t len, int is_signed,
                      const orcg_rlev2_plan* plan, uint64_t count, void* out, int width, int java = 0);
