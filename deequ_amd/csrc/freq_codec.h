// freq_codec.h -- group-key codec of the hash group-by (freq.hip), host + device.
//
// Everything here is DQ_HD so that the exact code the kernels run can be exercised on the CPU
// (tests/test_freq_codec.py builds tools/freq_codec_check.cpp against this header under ASan).
//
// Two key modes (FrequencyBasedAnalyzer.computeFrequencies, GroupingAnalyzers.scala:53-80):
//   * exact  -- one fixed-width key column: the group is the value widened to 64 bits and its
//               64-bit hash h = fmix_bij(value) is a BIJECTION (murmur3's fmix64), so h alone is
//               the group and the value is recovered with fmix_inv;
//   * hashed -- strings and multi-column keys: h = a 64-bit hash of the composite key, and the
//               group is the encoded key (below), which is compared byte for byte whenever two
//               rows or records meet on the same h (a hash collision never merges groups).
// Encoded key: per key column a u32 tag (0 = NULL, 1 = value) and then either 8 little-endian
// bytes (the value widened to 64 bits) or, for utf8, a u32 byte length and the bytes zero-padded
// to a multiple of 4.  Histogram (null_as_group, one utf8 key) reads a NULL as the string
// "NullValue", exactly as the reference's na.fill (Histogram.scala:59-66), so a real "NullValue"
// string and NULL are one group there as well.
#pragma once

#include <stdint.h>

#include "engine.h"

namespace dq {

constexpr int kMaxKeys = 8;

struct KeyCol {
  int32_t type;
  int32_t pad;
  const uint8_t* valid;
  const void* values;
  const uint8_t* data;
};

struct KeySet {
  KeyCol cols[kMaxKeys];
  int32_t n_keys;
  int32_t null_as_group;
};

DQ_HD uint32_t kbit(const uint8_t* bm, int64_t r) {
  return bm ? ((bm[r >> 3] >> (r & 7)) & 1u) : 1u;
}

DQ_HD uint64_t kwiden(int type, const void* v, int64_t r) {
  switch (type) {
    case DQ_INT8: return (uint64_t)(int64_t) reinterpret_cast<const int8_t*>(v)[r];
    case DQ_INT16: return (uint64_t)(int64_t) reinterpret_cast<const int16_t*>(v)[r];
    case DQ_INT32: return (uint64_t)(int64_t) reinterpret_cast<const int32_t*>(v)[r];
    case DQ_INT64: return (uint64_t) reinterpret_cast<const int64_t*>(v)[r];
    case DQ_FLOAT32: {
      uint32_t b;
      __builtin_memcpy(&b, reinterpret_cast<const float*>(v) + r, 4);
      return b;
    }
    case DQ_FLOAT64: {
      uint64_t b;
      __builtin_memcpy(&b, reinterpret_cast<const double*>(v) + r, 8);
      return b;
    }
    case DQ_BOOL: return kbit(reinterpret_cast<const uint8_t*>(v), r);
    default: return 0;
  }
}

// murmur3 fmix64: xor-shifts by >= 32 and odd multiplies, each invertible, so the map is a
// bijection of uint64; fmix_inv undoes it (the multipliers' inverses mod 2^64).
constexpr uint64_t kFmixC1 = 0xff51afd7ed558ccdULL, kFmixC1Inv = 0x4f74430c22a54005ULL;
constexpr uint64_t kFmixC2 = 0xc4ceb9fe1a85ec53ULL, kFmixC2Inv = 0x9cb4b2f8129337dbULL;
DQ_HD uint64_t fmix_bij(uint64_t k) {
  k ^= k >> 33;
  k *= kFmixC1;
  k ^= k >> 33;
  k *= kFmixC2;
  k ^= k >> 33;
  return k;
}
DQ_HD uint64_t fmix_inv(uint64_t k) {
  k ^= k >> 33;
  k *= kFmixC2Inv;
  k ^= k >> 33;
  k *= kFmixC1Inv;
  k ^= k >> 33;
  return k;
}

// Byte reader for xxh_bytes valid on host and device (unaligned loads within the string).
struct MemBytes {
  const uint8_t* p;
  DQ_HD uint64_t u64(int64_t o) const {
    uint64_t v;
    __builtin_memcpy(&v, p + o, 8);
    return v;
  }
  DQ_HD uint32_t u32(int64_t o) const {
    uint32_t v;
    __builtin_memcpy(&v, p + o, 4);
    return v;
  }
  DQ_HD uint32_t u8(int64_t o) const { return p[o]; }
};

// "NullValue" (Histogram.NullFieldReplacement, Histogram.scala:108) as constants: a string view
// with p == nullptr IS this literal, so no code path needs memory for it.
constexpr int32_t kNullValueLen = 9;
constexpr uint64_t kNullValueLo = 0x756c61566c6c754eULL;  // "NullValu", little-endian
constexpr uint32_t kNullValueHi = 0x65u;                   // "e"

struct SView {
  const uint8_t* p;  // nullptr: the "NullValue" literal
  int32_t len;
};
DQ_HD uint32_t sv_byte(const SView& v, int32_t q) {
  if (v.p) return v.p[q];
  return q < 8 ? (uint32_t)(kNullValueLo >> (8 * q)) & 0xffu : (q == 8 ? kNullValueHi : 0u);
}

enum RowKind : int32_t { ROW_SKIP = 0, ROW_KEY = 1, ROW_NULL_GROUP = 2 };

// utf8 key column k at row r; a NULL in Histogram mode is the "NullValue" literal.
DQ_HD bool key_str(const KeySet& ks, int k, int64_t r, SView& v) {
  const KeyCol& c = ks.cols[k];
  if (!kbit(c.valid, r)) {
    if (!ks.null_as_group) return false;
    v.p = nullptr;
    v.len = kNullValueLen;
    return true;
  }
  const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
  const int32_t s = off[r];
  v.p = c.data + s;
  v.len = off[r + 1] - s;
  return true;
}

// What row r contributes: a keyed row, a row of the exact-mode NULL group (Histogram on a
// fixed-width column), or nothing (a NULL key in a grouping: GroupingAnalyzers.scala:62-65).
DQ_HD int row_kind(const KeySet& ks, int64_t r, bool exact) {
  if (exact) {
    if (kbit(ks.cols[0].valid, r)) return ROW_KEY;
    return ks.null_as_group ? ROW_NULL_GROUP : ROW_SKIP;
  }
  for (int k = 0; k < ks.n_keys; ++k) {
    const KeyCol& c = ks.cols[k];
    if (!kbit(c.valid, r)) {
      if (!(ks.null_as_group && c.type == DQ_UTF8)) return ROW_SKIP;
    }
  }
  return ROW_KEY;
}

// Histogram groups cast(col as string) (Histogram.scala:63): every NaN prints as "NaN", so in
// Histogram mode NaN payloads fold into the canonical NaN (a grouping keeps Spark 2.2's binary
// key equality).
DQ_HD uint64_t exact_canon(const KeySet& ks, uint64_t v) {
  const int t = ks.cols[0].type;
  if (ks.null_as_group) {
    if (t == DQ_FLOAT64 && (v & 0x7fffffffffffffffULL) > 0x7ff0000000000000ULL)
      v = 0x7ff8000000000000ULL;
    if (t == DQ_FLOAT32 && (v & 0x7fffffffULL) > 0x7f800000ULL) v = 0x7fc00000ULL;
  }
  return v;
}
DQ_HD uint64_t exact_key(const KeySet& ks, int64_t r) {
  const KeyCol& c = ks.cols[0];
  return exact_canon(ks, kwiden(c.type, c.values, r));
}
DQ_HD uint64_t row_hash_exact(const KeySet& ks, int64_t r) { return fmix_bij(exact_key(ks, r)); }

// Composite 64-bit hash of a keyed row (hashed mode): per column XXH64 with a per-column seed,
// folded with an XXH64 merge step, then fmix.
constexpr uint64_t kRowHashSeed = 0x243F6A8885A308D3ULL;
DQ_HD uint64_t fold_col_hash(uint64_t h, uint64_t ch) { return rotl64(h ^ ch, 27) * P1 + P4; }
// Column hash of a string of at most 16 bytes held in (w0, w1) (little-endian, zero past its
// end): two odd multiplies, no loop and no data-dependent branch, so the lanes of a wave hashing
// strings of different lengths never diverge.  For a fixed (w1, len) the map w0 -> hash is a
// bijection; the row hash (fold_col_hash, fmix_bij) adds the avalanche.  (Only the group-by uses
// it: the value is internal to the frequency table, never a reference-visible hash.)
constexpr int32_t kHash16Max = 16;
DQ_HD uint64_t str_hash16(uint64_t w0, uint64_t w1, int32_t len, uint64_t seed) {
  const uint64_t a = rotl64(w0 * P1 + seed, 31);
  const uint64_t b = (w1 + (uint64_t)len * P5) * P2;
  return a ^ b;
}
// (w0, w1) of a string of at most 16 bytes in memory, bytewise (a host build reads no byte past
// the string)
DQ_HD void mem_str16(const uint8_t* p, int32_t len, uint64_t& w0, uint64_t& w1) {
  w0 = w1 = 0;
  for (int32_t q = 0; q < len; ++q) {
    if (q < 8) w0 |= (uint64_t)p[q] << (8 * q);
    else w1 |= (uint64_t)p[q] << (8 * (q - 8));
  }
}
// A string longer than 16 bytes: its 16-byte chunks (little-endian words, the last one zero-padded)
// mixed in order, then an avalanche -- three multiplies per chunk, and chunks a device thread
// builds from aligned dwords in registers (str_hash_long_dev).  Internal to the frequency table
// like every group-by hash (XXH64 over the bytes took a dependent chain of loads per 8 bytes).
DQ_HD uint64_t str_long_chunk(uint64_t acc, uint64_t w0, uint64_t w1) {
  return rotl64(acc ^ rotl64(w0 * P1, 31) ^ (w1 * P2), 27) * P1 + P4;
}
DQ_HD uint64_t str_long_final(uint64_t acc) {
  acc ^= acc >> 33;
  acc *= P2;
  acc ^= acc >> 29;
  return acc;
}
DQ_HD uint64_t str_long_seed(int32_t len, uint64_t seed) { return seed ^ ((uint64_t)len * P5); }
DQ_HD uint64_t str_bytes_hash(const uint8_t* p, int32_t len, int k) {
  if (len <= kHash16Max) {
    uint64_t w0, w1;
    mem_str16(p, len, w0, w1);
    return str_hash16(w0, w1, len, 17 + k);
  }
  uint64_t acc = str_long_seed(len, 17 + k);
  for (int32_t o = 0; o < len; o += 16) {
    uint64_t w0, w1;
    mem_str16(p + o, len - o < 16 ? len - o : 16, w0, w1);
    acc = str_long_chunk(acc, w0, w1);
  }
  return str_long_final(acc);
}
DQ_HD uint64_t str_col_hash(const SView& v, int k) {
  return v.p ? str_bytes_hash(v.p, v.len, k)
             : str_hash16(kNullValueLo, kNullValueHi, kNullValueLen, 17 + k);
}

DQ_HD uint64_t row_hash_hashed(const KeySet& ks, int64_t r) {
  uint64_t h = kRowHashSeed;
  for (int k = 0; k < ks.n_keys; ++k) {
    const KeyCol& c = ks.cols[k];
    uint64_t ch;
    if (c.type == DQ_UTF8) {
      SView v;
      key_str(ks, k, r, v);
      ch = str_col_hash(v, k);
    } else {
      ch = xxh_long(kwiden(c.type, c.values, r), 17 + k);
    }
    h = fold_col_hash(h, ch);
  }
  return fmix_bij(h);
}

// The row hash of a one-column utf8 key (row_hash_hashed with n_keys == 1).
DQ_HD uint64_t str_row_hash(const SView& v) { return fmix_bij(fold_col_hash(kRowHashSeed, str_col_hash(v, 0))); }
// The same, out of line, for phase A's strings longer than 16 bytes (rare in a wave; one copy of
// the XXH64 loop instead of one per unrolled round)
__host__ __device__ __attribute__((noinline)) uint64_t str_row_hash_long(const uint8_t* p,
                                                                         int32_t len) {
  return str_row_hash(SView{p, len});
}
// The same for a non-NULL string of len <= 16 bytes already in registers.
DQ_HD uint64_t str_row_hash_reg(uint64_t w0, uint64_t w1, int32_t len) {
  return fmix_bij(fold_col_hash(kRowHashSeed, str_hash16(w0, w1, len, 17)));
}

// Short form of a one-column utf8 key of at most 15 bytes: (k0, k1) = its bytes 0..7 and
// 8..14 with the length in k1's top byte (zero for such a string), so two short keys are equal
// iff both words are.  Every other key has k1 = kNoShort (top byte 0xFF), never equal to a short
// key.  A NULL in Histogram mode is the 9-byte "NullValue" literal and gets that string's short
// form, so it meets a real "NullValue" string in LDS (Histogram.scala:59-66).
constexpr uint64_t kNoShort = ~0ULL;
constexpr uint64_t kShortNotReady = 0xFEULL << 56;  // top byte 0xFE: never a short form
constexpr int32_t kShortMax = 15;
DQ_HD void str_short_key_reg(uint64_t w0, uint64_t w1, int32_t len, uint64_t& k0, uint64_t& k1) {
  if (len > kShortMax) {
    k0 = 0;
    k1 = kNoShort;
    return;
  }
  k0 = w0;
  k1 = w1 | ((uint64_t)len << 56);
}
DQ_HD void str_short_key(const SView& v, uint64_t& k0, uint64_t& k1) {
  if (!v.p) {
    str_short_key_reg(kNullValueLo, kNullValueHi, kNullValueLen, k0, k1);
    return;
  }
  if (v.len > kShortMax) {
    k0 = 0;
    k1 = kNoShort;
    return;
  }
  uint64_t w0 = 0, w1 = 0;
  for (int32_t q = 0; q < v.len; ++q) {
    if (q < 8) w0 |= (uint64_t)v.p[q] << (8 * q);
    else w1 |= (uint64_t)v.p[q] << (8 * (q - 8));
  }
  str_short_key_reg(w0, w1, v.len, k0, k1);
}

// A string of len <= 16 bytes from the aligned dwords d[0..4] that hold it, starting sh (0..3)
// bytes into d[0]: (w0, w1) little-endian, zero past its end.
DQ_HD void str16_from_dwords(const uint32_t* d, int sh, int32_t len, uint64_t& w0, uint64_t& w1) {
  uint64_t lo = (uint64_t)d[0] | ((uint64_t)d[1] << 32);
  uint64_t mid = (uint64_t)d[2] | ((uint64_t)d[3] << 32);
  if (sh) {
    lo = (lo >> (8 * sh)) | (mid << (64 - 8 * sh));
    mid = (mid >> (8 * sh)) | ((uint64_t)d[4] << (64 - 8 * sh));
  }
  if (len <= 0) {
    lo = mid = 0;
  } else if (len < 8) {
    lo &= (1ULL << (8 * len)) - 1;
    mid = 0;
  } else if (len < 16) {
    mid &= (1ULL << (8 * (len - 8))) - 1;
  }
  w0 = lo;
  w1 = mid;
}

// Bytes [p, p + len) of a string, len <= 16: reads the aligned dwords that overlap it (each holds
// a byte of the string, so no read reaches a page the string does not lie on).
DQ_HD void load_str16(const uint8_t* p, int32_t len, uint64_t& w0, uint64_t& w1) {
  w0 = w1 = 0;
  if (len <= 0) return;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
  const int sh = (int)(reinterpret_cast<uintptr_t>(p) & 3u);
  const int last = ((sh + len + 3) >> 2) - 1;  // 0..4
  uint32_t d[5];
  for (int k = 0; k < 5; ++k) d[k] = q[k < last ? k : last];
  str16_from_dwords(d, sh, len, w0, w1);
}


#ifdef __HIPCC__
// str_bytes_hash(p, len, k) for 16 < len, the string read as aligned dwords: up to 48 bytes with
// every load in flight together (each dword holds a byte of the string), then 16 bytes per round.
__device__ inline uint64_t str_hash_long_dev(const uint8_t* p, int32_t len, int k) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
  const int sh = (int)(reinterpret_cast<uintptr_t>(p) & 3u);
  uint64_t acc = str_long_seed(len, 17 + k);
  int32_t o = 0;
  if (len <= 48) {
    const int last = ((sh + len + 3) >> 2) - 1;  // <= 12
    uint32_t d[13];
#pragma unroll
    for (int j = 0; j < 13; ++j) d[j] = q[j < last ? j : last];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (16 * c >= len) break;
      uint64_t w0, w1;
      str16_from_dwords(d + 4 * c, sh, len - 16 * c < 16 ? len - 16 * c : 16, w0, w1);
      acc = str_long_chunk(acc, w0, w1);
    }
    return str_long_final(acc);
  }
  for (; o < len; o += 16) {
    uint64_t w0, w1;
    load_str16(p + o, len - o < 16 ? len - o : 16, w0, w1);
    acc = str_long_chunk(acc, w0, w1);
  }
  return str_long_final(acc);
}
#endif

DQ_HD uint32_t pad4(uint32_t n) { return (n + 3u) & ~3u; }

DQ_HD uint32_t row_enc_size(const KeySet& ks, int64_t r) {
  uint32_t n = 0;
  for (int k = 0; k < ks.n_keys; ++k) {
    const KeyCol& c = ks.cols[k];
    n += 4;
    if (c.type == DQ_UTF8) {
      SView v;
      if (key_str(ks, k, r, v)) n += 4 + pad4((uint32_t)v.len);
    } else if (kbit(c.valid, r)) {
      n += 8;
    }
  }
  return n;
}

// Writes the encoded key of row r at dst (4-byte aligned, row_enc_size(ks, r) bytes).
DQ_HD void row_encode(const KeySet& ks, int64_t r, uint32_t* dst) {
  for (int k = 0; k < ks.n_keys; ++k) {
    const KeyCol& c = ks.cols[k];
    if (c.type == DQ_UTF8) {
      SView v;
      if (!key_str(ks, k, r, v)) {
        *dst++ = 0;
        continue;
      }
      *dst++ = 1;
      *dst++ = (uint32_t)v.len;
      for (int32_t q = 0; q < v.len; q += 4) {
        uint32_t w = 0;
        for (int b = 0; b < 4 && q + b < v.len; ++b) w |= sv_byte(v, q + b) << (8 * b);
        *dst++ = w;
      }
    } else if (!kbit(c.valid, r)) {
      *dst++ = 0;
    } else {
      const uint64_t v = kwiden(c.type, c.values, r);
      *dst++ = 1;
      *dst++ = (uint32_t)v;
      *dst++ = (uint32_t)(v >> 32);
    }
  }
}

// n bytes at a and b equal?  8-, 4-, 2-, 1-byte unaligned loads, never past either string.
DQ_HD bool bytes_equal(const uint8_t* a, const uint8_t* b, int32_t n) {
  int32_t q = 0;
  for (; q + 8 <= n; q += 8) {
    uint64_t x, y;
    __builtin_memcpy(&x, a + q, 8);
    __builtin_memcpy(&y, b + q, 8);
    if (x != y) return false;
  }
  if (q + 4 <= n) {
    uint32_t x, y;
    __builtin_memcpy(&x, a + q, 4);
    __builtin_memcpy(&y, b + q, 4);
    if (x != y) return false;
    q += 4;
  }
  if (q + 2 <= n) {
    uint16_t x, y;
    __builtin_memcpy(&x, a + q, 2);
    __builtin_memcpy(&y, b + q, 2);
    if (x != y) return false;
    q += 2;
  }
  return q == n || a[q] == b[q];
}

// Are two keyed rows (of the same batch) the same group?
DQ_HD bool rows_equal(const KeySet& ks, int64_t r1, int64_t r2) {
  for (int k = 0; k < ks.n_keys; ++k) {
    const KeyCol& c = ks.cols[k];
    if (c.type == DQ_UTF8) {
      SView a, b;
      const bool v1 = key_str(ks, k, r1, a), v2 = key_str(ks, k, r2, b);
      if (v1 != v2) return false;
      if (!v1) continue;
      if (a.len != b.len) return false;
      if (a.p && b.p) {
        if (!bytes_equal(a.p, b.p, a.len)) return false;
      } else {
        for (int32_t q = 0; q < a.len; ++q)
          if (sv_byte(a, q) != sv_byte(b, q)) return false;
      }
    } else {
      const uint32_t v1 = kbit(c.valid, r1), v2 = kbit(c.valid, r2);
      if (v1 != v2) return false;
      if (v1 && kwiden(c.type, c.values, r1) != kwiden(c.type, c.values, r2)) return false;
    }
  }
  return true;
}

// The same three for a key of one utf8 column at a non-NULL row (phase A's one-string-column
// path): what the generic forms compute for such a row, without their per-type code.
DQ_HD SView str1_view(const KeySet& ks, int64_t r) {
  const int32_t* off = reinterpret_cast<const int32_t*>(ks.cols[0].values);
  const int32_t s = off[r];
  return SView{ks.cols[0].data + s, off[r + 1] - s};
}
DQ_HD uint32_t str1_enc_size(const KeySet& ks, int64_t r) {
  return 8 + pad4((uint32_t)str1_view(ks, r).len);
}
DQ_HD void str1_encode(const KeySet& ks, int64_t r, uint32_t* dst) {
  const SView v = str1_view(ks, r);
  dst[0] = 1;
  dst[1] = (uint32_t)v.len;
  for (int32_t q = 0; q < v.len; q += 4) {
    uint32_t w = 0;
    for (int b = 0; b < 4 && q + b < v.len; ++b) w |= (uint32_t)v.p[q + b] << (8 * b);
    dst[2 + q / 4] = w;
  }
}
// str1_encode of a key whose short form (str_short_key_reg: bytes 0..7 in k0, bytes 8..14 and the
// length in k1, zero past the end) is at hand: no reads.
DQ_HD uint32_t str1_short_len(uint64_t k1) { return (uint32_t)(k1 >> 56); }
DQ_HD void str1_encode_short(uint64_t k0, uint64_t k1, uint32_t* dst) {
  const uint32_t len = str1_short_len(k1);
  const uint32_t w[4] = {(uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1,
                         (uint32_t)(k1 >> 32) & 0xFFFFFFu};
  dst[0] = 1;
  dst[1] = len;
  for (uint32_t q = 0; 4 * q < len; ++q) dst[2 + q] = w[q];
}
// str1_encode of the string p[0, len) from aligned dword loads, up to 9 in flight (every dword read
// holds a byte of the string), instead of one dependent load per byte.
__device__ inline void str1_encode_copy(const uint8_t* p, int32_t len, uint32_t* dst) {
  dst[0] = 1;
  dst[1] = (uint32_t)len;
  const uintptr_t ad = reinterpret_cast<uintptr_t>(p);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(ad & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(ad & 3u) * 8u;
  const int32_t nsrc = ((int32_t)(ad & 3u) + len + 3) >> 2;  // source dwords with string bytes
  const int32_t nw = (len + 3) >> 2;
  for (int32_t q0 = 0; q0 < nw; q0 += 8) {
    uint32_t d[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) d[k] = q0 + k < nsrc ? src[q0 + k] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int32_t q = q0 + k;
      if (q >= nw) break;
      uint32_t w = sh ? (d[k] >> sh) | (d[k + 1] << (32u - sh)) : d[k];
      const int32_t nb = len - 4 * q;  // bytes of the string in this word
      if (nb < 4) w &= (1u << (8 * nb)) - 1u;
      dst[2 + q] = w;
    }
  }
}
// The same two encodings with 16-byte stores, at a 16-byte aligned dst with room for the encoding
// rounded up to 16 bytes (str1_enc_size16): one store instruction per 16 bytes instead of one per
// word (scattered 4-byte stores made the string path's arena writes the slowest part of a tile).
DQ_HD uint32_t str1_enc_size16(int32_t len) { return (8u + pad4((uint32_t)len) + 15u) & ~15u; }
#ifdef __HIPCC__
__device__ inline void str1_encode_short16(uint64_t k0, uint64_t k1, uint32_t* dst) {
  const uint32_t len = str1_short_len(k1);
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4(1u, len, (uint32_t)k0, (uint32_t)(k0 >> 32));
  if (len > 8) d[1] = make_uint4((uint32_t)k1, (uint32_t)(k1 >> 32) & 0xFFFFFFu, 0u, 0u);
}
__device__ inline void str1_encode_copy16(const uint8_t* p, int32_t len, uint32_t* dst) {
  const uintptr_t ad = reinterpret_cast<uintptr_t>(p);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(ad & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(ad & 3u) * 8u;
  const int32_t nsrc = ((int32_t)(ad & 3u) + len + 3) >> 2;  // source dwords with string bytes
  const int32_t nw = (len + 3) >> 2;                           // string words of the encoding
  uint4* d = reinterpret_cast<uint4*>(dst);
  // word i of the encoding: 0 -> 1, 1 -> len, 2 + q -> string word q
  auto sword = [&](int32_t q, const uint32_t* dd) -> uint32_t {  // dd: source dwords from q's
    uint32_t w = sh ? (dd[0] >> sh) | (dd[1] << (32u - sh)) : dd[0];
    const int32_t nb = len - 4 * q;
    if (nb < 4) w &= (1u << (8 * nb)) - 1u;
    return w;
  };
  for (int32_t c = 0; 4 * c < 2 + nw; c += 4) {  // 4 stores (16 words) per round of loads
    uint32_t sd[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) {
      const int32_t j = 4 * c - 2 + k;  // source dword index (string word j needs dwords j, j+1)
      sd[k] = j >= 0 && j < nsrc ? src[j] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int32_t i0 = 4 * (c + u);  // first encoding word of this store
      if (i0 >= 2 + nw) break;
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int32_t i = i0 + e;
        w[e] = i == 0 ? 1u : i == 1 ? (uint32_t)len : (i - 2 < nw ? sword(i - 2, sd + (i - 2 - (4 * c - 2))) : 0u);
      }
      d[c + u] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}
#endif

// (out of line: only long strings get here, so one copy instead of one per call site)
__host__ __device__ __attribute__((noinline)) bool str1_rows_equal(const KeySet& ks, int64_t r1,
                                                                   int64_t r2) {
  const SView a = str1_view(ks, r1), b = str1_view(ks, r2);
  return a.len == b.len && bytes_equal(a.p, b.p, a.len);
}

// Size in bytes of an encoded key.
DQ_HD uint32_t enc_size(const uint32_t* enc, const int32_t* types, int n_keys) {
  uint32_t w = 0;
  for (int k = 0; k < n_keys; ++k) {
    const uint32_t tag = enc[w++];
    if (!tag) continue;
    if (types[k] == DQ_UTF8) w += 1 + pad4(enc[w]) / 4;
    else w += 2;
  }
  return 4 * w;
}

DQ_HD bool enc_equal(const uint32_t* a, const uint32_t* b, const int32_t* types, int n_keys) {
  const uint32_t n = enc_size(a, types, n_keys);
  if (enc_size(b, types, n_keys) != n) return false;
  for (uint32_t q = 0; q < n / 4; ++q)
    if (a[q] != b[q]) return false;
  return true;
}

// enc_equal for the device's arena (phase C's hash hits, MutualInformation's lookups): the same
// answer with few dependent round trips.  The encoding is self-delimiting, so two keys are equal
// iff the first enc_size(a) bytes of both are; the words of a 4-word chunk are loaded together
// (one round trip per chunk, where enc_equal's early-exit loop took one per word).  The first
// chunk is read unconditionally: every arena keeps >= 64 bytes past its last entry (grow_keep's
// callers, and a borrowed arena is another table's), so 64 bytes from any entry's start are
// mapped.
__device__ inline bool enc_equal_arena(const uint32_t* a, const uint32_t* b, const int32_t* types,
                                       int n_keys) {
  // the first 16 words of both keys in one round trip (a one-column utf8 key of <= 56 bytes
  // is decided by it), then 8 words per round
  uint32_t wa[16], wb[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    wa[k] = a[k];
    wb[k] = b[k];
  }
  uint32_t n;  // words of a's encoding
  if (n_keys == 1 && types[0] == DQ_UTF8) n = wa[0] ? 2 + pad4(wa[1]) / 4 : 1;
  else n = enc_size(a, types, n_keys) / 4;
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) x |= (uint32_t)k < n ? wa[k] ^ wb[k] : 0u;
  if (x) return false;
  for (uint32_t q = 16; q < n; q += 8) {
    x = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) x |= q + k < n ? a[q + k] ^ b[q + k] : 0u;
    if (x) return false;
  }
  return true;
}

// Hash of an encoded key: the same value row_hash_hashed gives for the row it encodes.
DQ_HD uint64_t enc_hash(const uint32_t* enc, const int32_t* types, int n_keys) {
  uint64_t h = 0x243F6A8885A308D3ULL;
  uint32_t w = 0;
  for (int k = 0; k < n_keys; ++k) {
    const uint32_t tag = enc[w++];
    uint64_t ch;
    if (types[k] == DQ_UTF8) {
      const uint32_t len = tag ? enc[w++] : 0;
      ch = str_bytes_hash(reinterpret_cast<const uint8_t*>(enc + w), (int32_t)len, k);
      w += pad4(len) / 4;
    } else {
      uint64_t v = 0;
      if (tag) {
        v = (uint64_t)enc[w] | ((uint64_t)enc[w + 1] << 32);
        w += 2;
      }
      ch = xxh_long(v, 17 + k);
    }
    h = rotl64(h ^ ch, 27) * P1 + P4;
  }
  return fmix_bij(h);
}

// ------------------------------------------------------------------------------------------------
// Records: how the group-by carries (group, count) pairs between its passes.
//   exact  record (8 B):  (h << 8) | code        -- the top 8 bits of h are implied by the bucket
//   hashed record (16 B): {h, (rep << 8) | code} -- rep = arena offset of the encoded key
// `code` carries a count as one base-4 digit: count = (code & 3) << 2 * (code >> 2); a count c
// travels as one record per non-zero base-4 digit of c (at most 32), and every pass SUMS counts.
// ------------------------------------------------------------------------------------------------
DQ_HD uint64_t code_count(uint32_t code) {
  return (uint64_t)(code & 3u) << (2u * (code >> 2));
}
DQ_HD int count_digits(uint64_t c) {
  int n = 0;
  for (; c; c >>= 2) n += (c & 3) != 0;
  return n;
}

}  // namespace dq
