// Java tree-reader face of the C ABI (include/orcg.h "Java TreeReader face"):
// what java/core's TreeReader.nextVector and StringDictionaryTreeReader build
// from the decoded streams, so a JNI shim can fill ColumnVector fields
// directly. The streams themselves are decoded on the GPU by the stateful
// decoders (orcg_byte_rle_decoder: PRESENT through the boolean RLE kernel;
// orcg_rle_decoder: the dictionary DATA indices through the RLEv2 kernels);
// this file only applies the Java rules to their output on the host.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/orcg.h"
#include "orcg_internal.hh"

namespace {

thread_local std::string t_java_error;

int java_fail(int status, const std::string& m) {
  t_java_error = m;
  return status;
}

}  // namespace

extern "C" {

const char* orcg_java_last_error(void) { return t_java_error.c_str(); }

// TreeReader.nextVector (java/core/src/java/org/apache/orc/impl/
// TreeReaderFactory.java:405-441): with a PRESENT stream or a parent mask,
// noNulls starts true; for each row a null parent makes it null, otherwise
// BitFieldReader.next() (BitFieldReader.java:51-57, the MSB-first bits of the
// boolean RLE stream) != 1 makes it null; isRepeating = !noNulls && allNull.
// Without either, every row is present and isRepeating is left as it was.
int orcg_java_tree_present_next(orcg_byte_rle_decoder* present, const uint8_t* parent_is_null, uint64_t batch,
                                uint8_t* is_null, int* no_nulls, int* is_repeating) {
  if ((batch && !is_null) || !no_nulls || !is_repeating) return java_fail(ORCG_INVALID_ARGUMENT, "null argument");
  if (!present && !parent_is_null) {
    *no_nulls = 1;
    if (batch) memset(is_null, 0, batch);
    return ORCG_OK;
  }
  // the bits of the rows whose parent is present, in row order (the boolean
  // decoder consumes one bit per non-null slot of its notNull argument)
  std::vector<char> bits(batch, 1);
  if (present) {
    std::vector<char> live;
    if (parent_is_null) {
      live.resize(batch);
      for (uint64_t i = 0; i < batch; ++i) live[i] = parent_is_null[i] ? 0 : 1;
    }
    const int rc = orcg_byte_rle_decoder_next(present, bits.data(), batch, parent_is_null ? live.data() : nullptr);
    if (rc) return java_fail(rc, orcg_byte_rle_decoder_last_error(present));
  }
  bool nonulls = true, all_null = true;
  for (uint64_t i = 0; i < batch; ++i) {
    if (!parent_is_null || !parent_is_null[i]) {
      if (present && bits[i] != 1) {
        nonulls = false;
        is_null[i] = 1;
      } else {
        is_null[i] = 0;
        all_null = false;
      }
    } else {
      nonulls = false;
      is_null[i] = 1;
    }
  }
  *no_nulls = nonulls ? 1 : 0;
  *is_repeating = (!nonulls && all_null) ? 1 : 0;
  return ORCG_OK;
}

// StringDictionaryTreeReader.readDictionaryByteArray (TreeReaderFactory.java:
// 2396-2466), no filter: the DATA reader's nextVector into the scratch vector
// (RunLengthIntegerReaderV2.java:371-396: null slots 1, isRepeating computed,
// an all-null repeating batch left untouched), then per row
// BytesColumnVector.setRef(i, dictionaryBuffer, offset, length) with
// getDictionaryEntryLength (:2468-2478), (0, 0) for null rows; a repeating
// index vector sets row 0 only. dictionaryBuffer == null (has_buffer 0):
// non-null rows are empty strings, or, without dictionary offsets either, the
// batch is one repeating null.
int orcg_java_dictionary_next(orcg_rle_decoder* data, const int32_t* dict_offsets, uint64_t dict_offsets_len,
                              int has_buffer, int64_t buffer_len, uint8_t* is_null, int* no_nulls, int* is_repeating,
                              uint64_t batch, int64_t* scratch, int32_t* start, int32_t* length) {
  if (!no_nulls || !is_repeating || (batch && (!is_null || !start || !length)))
    return java_fail(ORCG_INVALID_ARGUMENT, "null argument");
  if (!has_buffer) {
    if (!dict_offsets) {
      // "Entire stripe contains null strings."
      *is_repeating = 1;
      *no_nulls = 0;
      if (batch) {
        is_null[0] = 1;
        start[0] = 0;
        length[0] = 0;
      }
      return ORCG_OK;
    }
    for (uint64_t i = 0; i < batch; ++i)
      if (!is_null[i]) start[i] = length[i] = 0;  // EMPTY_BYTE_ARRAY
    return ORCG_OK;
  }
  if (!data || !dict_offsets || (batch && !scratch)) return java_fail(ORCG_INVALID_ARGUMENT, "null argument");
  // scratchlcv shares isNull / noNulls / isRepeating with the result
  int rep = *is_repeating;
  int rc = orcg_rle_decoder_next_vector_java(data, scratch, *no_nulls ? nullptr : is_null, batch, &rep);
  if (rc) return java_fail(rc, orcg_rle_decoder_last_error(data));
  auto entry = [&](int64_t idx, int32_t* off, int32_t* len) -> int {
    // dictionaryOffsets[(int) idx] (an int cast, then Java's bounds check)
    const int32_t e = (int32_t)idx;
    if (e < 0 || (uint64_t)e >= dict_offsets_len) {
      char m[96];
      snprintf(m, sizeof m, "Index %d out of bounds for length %llu", e, (unsigned long long)dict_offsets_len);
      return java_fail(ORCG_PARSE_ERROR, m);
    }
    *off = dict_offsets[e];
    *len = (uint64_t)e < dict_offsets_len - 1 ? dict_offsets[e + 1] - *off : (int32_t)(buffer_len - *off);
    return ORCG_OK;
  };
  if (!rep) {
    for (uint64_t i = 0; i < batch; ++i) {
      if (!is_null[i]) {
        if ((rc = entry(scratch[i], &start[i], &length[i]))) return rc;
      } else {
        start[i] = length[i] = 0;
      }
    }
  } else if (batch) {
    if ((rc = entry(scratch[0], &start[0], &length[0]))) return rc;
  }
  *is_repeating = rep;
  return ORCG_OK;
}

}  // extern "C"
