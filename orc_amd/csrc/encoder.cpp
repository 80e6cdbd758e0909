// Minimal RLEv2 writer used to build synthetic device-resident streams for the
// benchmark and the parity tests. It emits the four sub-encodings exactly as
// the format defines them (site/specification/ORCv1.md:723-886) and records
// row-index positions the way RleEncoderV2::recordPosition does
// (c++/src/RleEncoderV2.cc). It is writer-side tooling, not on the decode path.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/orcg.h"

namespace {

// BitWidthToFBSMap (c++/src/RLEV2Util.cc:40-61) restated: width -> 5-bit code.
int width_code(uint32_t w) {
  if (w <= 1) return 0;
  if (w <= 24) return (int)w - 1;
  switch (w) {
    case 26: return 24;
    case 28: return 25;
    case 30: return 26;
    case 32: return 27;
    case 40: return 28;
    case 48: return 29;
    case 56: return 30;
    case 64: return 31;
  }
  return -1;
}

// ClosestFixedBitsMap / ClosestAlignedFixedBitsMap (c++/src/RLEV2Util.cc:29-38).
uint32_t closest_fixed(uint32_t n) {
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
uint32_t closest_aligned(uint32_t n) {
  if (n <= 1) return 1;
  if (n <= 2) return 2;
  if (n <= 4) return 4;
  if (n <= 8) return 8;
  if (n <= 16) return 16;
  if (n <= 24) return 24;
  if (n <= 32) return 32;
  if (n <= 40) return 40;
  if (n <= 48) return 48;
  if (n <= 56) return 56;
  return 64;
}

uint32_t bits_of(uint64_t v) { return v ? 64u - (uint32_t)__builtin_clzll(v) : 0u; }
uint64_t zigzag(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }

struct Out {
  uint8_t* dst;
  uint64_t cap;
  uint64_t len = 0;
  bool overflow = false;
  void byte(uint32_t b) {
    if (len < cap) dst[len] = (uint8_t)b;
    else overflow = true;
    ++len;
  }
  void varint(uint64_t v) {
    while (v >= 0x80) {
      byte((uint32_t)(v & 0x7f) | 0x80);
      v >>= 7;
    }
    byte((uint32_t)v);
  }
  void be(uint64_t v, uint32_t nbytes) {
    for (int i = (int)nbytes - 1; i >= 0; --i) byte((uint32_t)(v >> (8 * i)) & 0xff);
  }
  // MSB-first bit packing of n fields of w bits, padded to a byte.
  void pack(const uint64_t* v, uint64_t n, uint32_t w) {
    if (w % 8 == 0) {
      for (uint64_t i = 0; i < n; ++i) be(v[i], w / 8);
      return;
    }
    uint64_t acc = 0;  // pending bits, right aligned
    uint32_t nacc = 0;
    const uint64_t mask = (1ull << w) - 1;  // w < 64 here
    for (uint64_t i = 0; i < n; ++i) {
      acc = (acc << w) | (v[i] & mask);
      nacc += w;
      while (nacc >= 8) {
        nacc -= 8;
        byte((uint32_t)(acc >> nacc) & 0xff);
      }
      acc &= (1ull << nacc) - 1;
    }
    if (nacc) byte((uint32_t)(acc << (8 - nacc)) & 0xff);
  }
};

void emit_direct(Out& o, const uint64_t* u, uint32_t L, uint32_t w) {
  const int code = width_code(w);
  o.byte(0x40u | ((uint32_t)code << 1) | ((L - 1) >> 8));
  o.byte((L - 1) & 0xff);
  o.pack(u, L, w);
}

int encode_short_repeat(Out& o, const int64_t* v, uint32_t L, bool sgn) {
  if (L < 3 || L > 10) return ORCG_INVALID_ARGUMENT;
  for (uint32_t i = 1; i < L; ++i)
    if (v[i] != v[0]) return ORCG_INVALID_ARGUMENT;
  const uint64_t u = sgn ? zigzag(v[0]) : (uint64_t)v[0];
  uint32_t nb = (bits_of(u) + 7) / 8;
  if (nb == 0) nb = 1;
  o.byte(((nb - 1) << 3) | (L - 3));
  o.be(u, nb);
  return ORCG_OK;
}

int encode_direct(Out& o, const int64_t* v, uint32_t L, bool sgn, bool aligned) {
  if (L < 1 || L > 512) return ORCG_INVALID_ARGUMENT;
  uint64_t u[512];
  uint32_t maxb = 0;
  for (uint32_t i = 0; i < L; ++i) {
    u[i] = sgn ? zigzag(v[i]) : (uint64_t)v[i];
    maxb = std::max(maxb, bits_of(u[i]));
  }
  emit_direct(o, u, L, aligned ? closest_aligned(maxb) : closest_fixed(maxb));
  return ORCG_OK;
}

// PATCHED_BASE (ORCv1.md:802-863): base = min, W covers the 95th percentile
// of the adjusted widths, the rest is patched through a gap list.
int encode_patched(Out& o, const int64_t* v, uint32_t L) {
  if (L < 1 || L > 512) return ORCG_INVALID_ARGUMENT;
  int64_t mn = v[0];
  for (uint32_t i = 1; i < L; ++i) mn = std::min(mn, v[i]);
  uint64_t adj[512];
  uint32_t widths[512];
  uint32_t maxb = 0;
  for (uint32_t i = 0; i < L; ++i) {
    adj[i] = (uint64_t)v[i] - (uint64_t)mn;
    widths[i] = bits_of(adj[i]);
    maxb = std::max(maxb, widths[i]);
  }
  std::vector<uint32_t> sorted(widths, widths + L);
  std::sort(sorted.begin(), sorted.end());
  uint32_t w = closest_fixed(sorted[(size_t)((L - 1) * 95 / 100)]);
  if (w >= maxb) {  // nothing to patch: use the widest table width below maxb
    if (maxb <= 1) return ORCG_INVALID_ARGUMENT;
    w = maxb - 1;
    while (w > 0 && width_code(w) < 0) --w;
    if (w == 0) return ORCG_INVALID_ARGUMENT;
  }
  const uint32_t pw = closest_fixed(maxb - w);
  if (width_code(pw) < 0) return ORCG_INVALID_ARGUMENT;
  // gap list with escapes (gap 255, patch 0) for gaps > 255
  std::vector<uint64_t> gaps, patches;
  uint32_t prev = 0;
  bool first = true;
  uint32_t maxgap = 0;
  for (uint32_t i = 0; i < L; ++i) {
    if (widths[i] <= w) continue;
    uint32_t gap = first ? i : i - prev;
    while (gap > 255) {
      gaps.push_back(255);
      patches.push_back(0);
      gap -= 255;
      maxgap = 255;
    }
    gaps.push_back(gap);
    patches.push_back(adj[i] >> w);
    maxgap = std::max(maxgap, gap);
    prev = i;
    first = false;
  }
  const uint32_t pl = (uint32_t)gaps.size();
  if (pl == 0 || pl > 31) return ORCG_INVALID_ARGUMENT;
  uint32_t pgw = std::max(1u, bits_of(maxgap));
  if (pgw > 8) return ORCG_INVALID_ARGUMENT;
  if (pw + pgw > 64) return ORCG_INVALID_ARGUMENT;
  const uint32_t cfb = closest_fixed(pw + pgw);
  // base: sign-magnitude in the fewest bytes with room for the sign bit
  const uint64_t mag = mn < 0 ? (uint64_t)0 - (uint64_t)mn : (uint64_t)mn;
  uint32_t bw = (bits_of(mag) + 1 + 7) / 8;
  if (bw == 0) bw = 1;
  if (bw > 8) return ORCG_INVALID_ARGUMENT;
  uint64_t base_enc = mag;
  if (mn < 0) base_enc |= 1ull << (bw * 8 - 1);
  o.byte(0x80u | ((uint32_t)width_code(w) << 1) | ((L - 1) >> 8));
  o.byte((L - 1) & 0xff);
  o.byte(((bw - 1) << 5) | (uint32_t)width_code(pw));
  o.byte(((pgw - 1) << 5) | pl);
  o.be(base_enc, bw);
  uint64_t lits[512];
  const uint64_t wmask = w >= 64 ? ~0ull : ((1ull << w) - 1);
  for (uint32_t i = 0; i < L; ++i) lits[i] = adj[i] & wmask;
  o.pack(lits, L, w);
  std::vector<uint64_t> entries(pl);
  for (uint32_t k = 0; k < pl; ++k) entries[k] = (gaps[k] << pw) | patches[k];
  o.pack(entries.data(), pl, cfb);
  return ORCG_OK;
}

// DELTA (ORCv1.md:865-886): fixed delta when every step equals the first.
int encode_delta(Out& o, const int64_t* v, uint32_t L, bool sgn) {
  if (L < 1 || L > 512) return ORCG_INVALID_ARGUMENT;
  const uint64_t base = sgn ? zigzag(v[0]) : (uint64_t)v[0];
  const int64_t db = L > 1 ? (int64_t)((uint64_t)v[1] - (uint64_t)v[0]) : 0;
  bool fixed = true;
  for (uint32_t i = 2; i < L; ++i)
    if ((int64_t)((uint64_t)v[i] - (uint64_t)v[i - 1]) != db) fixed = false;
  if (fixed) {
    o.byte(0xC0u | ((L - 1) >> 8));
    o.byte((L - 1) & 0xff);
    o.varint(base);
    o.varint(zigzag(db));
    return ORCG_OK;
  }
  uint64_t d[512];
  uint32_t maxb = 0;
  for (uint32_t i = 2; i < L; ++i) {
    const int64_t step = (int64_t)((uint64_t)v[i] - (uint64_t)v[i - 1]);
    if ((db < 0 && step > 0) || (db >= 0 && step < 0)) return ORCG_INVALID_ARGUMENT;
    d[i - 2] = db < 0 ? (uint64_t)0 - (uint64_t)step : (uint64_t)step;
    maxb = std::max(maxb, bits_of(d[i - 2]));
  }
  uint32_t w = closest_fixed(maxb);
  if (w < 2) w = 2;  // code 0 means "fixed delta", so a 1-bit delta uses width 2
  o.byte(0xC0u | ((uint32_t)width_code(w) << 1) | ((L - 1) >> 8));
  o.byte((L - 1) & 0xff);
  o.varint(base);
  o.varint(zigzag(db));
  o.pack(d, L - 2, w);
  return ORCG_OK;
}

}  // namespace

extern "C" int orcg_rlev2_encode_direct(const int64_t* values, uint64_t n, int is_signed,
                                        int aligned, uint8_t* dst, uint64_t dst_cap,
                                        uint64_t* out_len, uint64_t rows_per_group,
                                        uint64_t* positions) {
  if (!out_len || (n && !values)) return ORCG_INVALID_ARGUMENT;
  Out o{dst, dst_cap};
  uint64_t group = 0;
  for (uint64_t i = 0; i < n; i += 512) {
    const uint32_t L = (uint32_t)std::min<uint64_t>(512, n - i);
    // row-index positions of every row group that starts inside this run:
    // (byte offset of the run, values of the run before the row)
    if (positions && rows_per_group) {
      while (group * rows_per_group < i + L && group * rows_per_group < n) {
        positions[2 * group] = o.len;
        positions[2 * group + 1] = group * rows_per_group - i;
        ++group;
      }
    }
    encode_direct(o, values + i, L, is_signed != 0, aligned != 0);
  }
  *out_len = o.len;
  return o.overflow ? ORCG_OUT_OF_MEMORY : ORCG_OK;
}

extern "C" int orcg_rlev2_encode_runs(const int64_t* values, uint64_t n, int is_signed,
                                      const uint8_t* kinds, const uint32_t* lengths,
                                      uint64_t nruns, uint8_t* dst, uint64_t dst_cap,
                                      uint64_t* out_len, uint64_t* run_offsets) {
  if (!out_len || !kinds || !lengths) return ORCG_INVALID_ARGUMENT;
  Out o{dst, dst_cap};
  uint64_t at = 0;
  for (uint64_t r = 0; r < nruns; ++r) {
    const uint32_t L = lengths[r];
    if (at + L > n) return ORCG_INVALID_ARGUMENT;
    if (run_offsets) run_offsets[r] = o.len;
    int rc;
    switch (kinds[r]) {
      case 0: rc = encode_short_repeat(o, values + at, L, is_signed != 0); break;
      case 1: rc = encode_direct(o, values + at, L, is_signed != 0, false); break;
      case 2: rc = encode_patched(o, values + at, L); break;
      case 3: rc = encode_delta(o, values + at, L, is_signed != 0); break;
      default: rc = ORCG_INVALID_ARGUMENT;
    }
    if (rc != ORCG_OK) return rc;
    at += L;
  }
  *out_len = o.len;
  return o.overflow ? ORCG_OUT_OF_MEMORY : ORCG_OK;
}
