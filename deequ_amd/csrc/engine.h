// engine.h -- records and arithmetic shared by the host runtime (api.cpp) and the HIP kernels
// (scan.hip, freq.hip).  Everything here is __host__ __device__ so that the merge rules applied
// across workgroups, across batches, and across GPUs (rank-ordered merge after the all-gather)
// are literally the same code.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/deequ_amd.h"

#define DQ_HD __host__ __device__ __forceinline__

namespace dq {

// ------------------------------------------------------------------------------------------------
// Fused-scan task kinds.  The planner (api.cpp) maps every dq_agg of a suite onto a small set of
// column tasks; each task reads its column buffers once per batch and produces one Acc.
// ------------------------------------------------------------------------------------------------
enum TaskKind : int32_t {
  TK_NUMERIC = 1,    // one numeric column: n, Sum, Min, Max, (n, avg, m2), <= 3 fused predicates
  TK_VALIDITY = 2,   // popcount(validity & where): Completeness numerator
  TK_STR_IN = 3,     // [col IS NULL OR] col [NOT] IN ('a','b',...) on a utf8 column
  TK_BOOLMAP = 4,    // counts over a materialised predicate bitmap (generic predicates / where)
  TK_COMOMENTS = 5,  // two numeric columns: (n, xAvg, yAvg, ck, xMk, yMk)
  TK_HLL = 6,        // HLL++ registers (P = 9, 512 registers) of one column
  TK_DTYPE = 7,      // DataType: counts of NULL / Fractional / Integral / Boolean / String values
  TK_DECIMAL = 8     // one decimal(p, s) column: n, exact Sum, 128-bit Min / Max, (n, avg, m2)
};

constexpr int kMaxPreds = 3;          // fused predicates per TK_NUMERIC task
constexpr int kHllP = 9;              // HyperLogLogPlusPlusUtils.P for RELATIVE_SD 0.05 (:155-159)
constexpr int kHllM = 1 << kHllP;     // 512 registers
constexpr int kHllWords = 52;         // NUM_WORDS (:152)
constexpr int kHllRegsPerWord = 10;   // REGISTERS_PER_WORD
constexpr int kHllRegBits = 6;        // REGISTER_SIZE
constexpr int kBlock = 256;           // threads per scan workgroup (4 waves)
constexpr int kWaveRows = 1024;       // rows per wave iteration of a streaming body (16 per lane)
// Work-item size target in buffer bytes: big enough that the one dequeue word (~88 dequeues/us)
// is never the bound, small enough that the persistent grid's tail stays short.
#ifndef DQ_ITEM_BYTES
#define DQ_ITEM_BYTES 262144
#endif
constexpr double kItemBytes = DQ_ITEM_BYTES;
constexpr int kItemAlign = 1024;      // work items are whole wave iterations (rows % 1024 == 0)
constexpr int kFinParts = 32;         // first-stage finalize workgroups per logical task
constexpr int kListLenSlots = 65;     // STR_IN lists bucketed by length 0..64, then "longer"

// Fused numeric predicate:  [col IS NULL OR] (col op1 lo [AND col op2 hi])
struct NumPred {
  int32_t op1, op2;       // dq_xop comparison, op2 == 0 when absent
  int32_t as_double;      // compare in double (Spark NaN-safe order) instead of int64
  int32_t null_is_true;   // "col IS NULL OR ..." form
  int64_t lo_i, hi_i;
  double lo_d, hi_d;
};

// One (task, batch) descriptor as the scan kernel sees it: it carries the batch's pointers and the
// range of global work items [item_begin, item_begin + n_items) that cover the batch's rows.
struct TaskDesc {
  int32_t kind, type, type2, n_preds;
  int32_t out;            // logical task = accumulator index
  int32_t hll_out;        // HLL register-file index of the logical task (TK_HLL) or of the HLL
                          // task a BC_CORR_HLL descriptor also fills, else -1
  int32_t batch;          // batch index of this descriptor
  int32_t negate;         // TK_STR_IN: NOT IN
  int32_t null_is_true;   // TK_STR_IN: IS NULL OR ...
  int32_t n_list;         // TK_STR_IN list length
  int32_t vec_ok;         // buffers aligned for the vector path
  int32_t list_small;     // TK_STR_IN: <= 8 entries, each <= 7 bytes (packed-key compare path)
  int32_t body;           // scan body class (kernels.h BodyClass)
  int32_t hll_side;       // BC_CORR_HLL: the column the fused HLL task hashes (0 = x, 1 = y)
  uint64_t list_lenmask;  // TK_STR_IN small lists: bit L set when an entry has length L
  // TK_STR_IN small lists: entry k as (bytes, zero-padded) | length << 56; unused = 0xFE << 56
  // (a row of 8+ bytes keys to ~0, so it matches neither an entry nor an unused slot)
  uint64_t list_key[8];
  int64_t rows;
  int64_t item_rows;      // rows per work item (multiple of kItemAlign)
  int64_t item_begin;     // first global item index of this descriptor
  int64_t n_items;
  // guided tail: items [0, n_big) take item_rows rows each, the rest small_rows each (the queue
  // hands the small ones out last, so waves finish within a small item of each other)
  int64_t n_big;
  int64_t small_rows;
  const uint8_t* valid;   // column 1
  const void* values;
  const uint8_t* data;
  const uint8_t* valid2;  // column 2 (TK_COMOMENTS)
  const void* values2;
  const uint8_t* w_val;   // where bitmap (value bits), NULL = no where
  const uint8_t* w_vld;   // where bitmap (validity bits), NULL = never NULL
  const uint8_t* b_val;   // TK_BOOLMAP: counted expression bitmap (value bits)
  const uint8_t* b_vld;   //            (validity bits)
  // TK_STR_IN list (device), entries sorted by byte length: entries of length L <= 64 are
  // [list_start[L], list_start[L + 1]), longer ones [list_start[65], list_start[66]).
  const int32_t* list_start;
  const int32_t* list_len;
  const int32_t* list_boff;   // byte offset of each entry in list_bytes (padded by 8 bytes)
  const uint64_t* list_pre;   // first min(len, 8) bytes of each entry, little-endian
  const uint8_t* list_bytes;
  NumPred preds[kMaxPreds];
};

// Accumulator record: the aggregation buffer of one task.  128 bytes.
//   TK_NUMERIC  : i0 n, i1 Long sum (wrapping), i2 min key, i3 max key, i4..6 pred TRUE,
//                 i7..9 pred non-NULL; d0 double sum, d1 avg, d2 m2
//   TK_VALIDITY : i0 count
//   TK_STR_IN / TK_BOOLMAP : i0 TRUE count, i1 non-NULL count
//   TK_COMOMENTS: i0 n; d0 xAvg, d1 yAvg, d2 ck, d3 xMk, d4 yMk
//   TK_DTYPE    : i0 NULL, i1 Fractional, i2 Integral, i3 Boolean, i4 String
//   TK_DECIMAL  : i0 n, i1..i3 the sum of the unscaled values (192-bit two's complement, little-
//                 endian limbs: exact for any row count), i4/i5 min (lo, hi), i6/i7 max (lo, hi);
//                 d1 avg, d2 m2 of the values cast to double (as TK_NUMERIC)
struct alignas(16) Acc {
  int64_t i[10];
  double d[6];
};

DQ_HD void acc_init(int kind, Acc& a) {
  for (int k = 0; k < 10; ++k) a.i[k] = 0;
  for (int k = 0; k < 6; ++k) a.d[k] = 0.0;
  if (kind == TK_NUMERIC) {
    a.i[2] = INT64_MAX;  // min key
    a.i[3] = INT64_MIN;  // max key
  }
  if (kind == TK_DECIMAL) {  // min = INT128_MAX, max = INT128_MIN
    a.i[4] = -1;
    a.i[5] = INT64_MAX;
    a.i[6] = 0;
    a.i[7] = INT64_MIN;
  }
}

// 128-bit signed order of (lo, hi) pairs held in int64 words
DQ_HD bool i128_lt(int64_t alo, int64_t ahi, int64_t blo, int64_t bhi) {
  return ahi < bhi || (ahi == bhi && (uint64_t)alo < (uint64_t)blo);
}
// s[0..2] += sign-extended (lo, hi)
DQ_HD void add192(int64_t* s, uint64_t lo, int64_t hi) {
  const uint64_t x[3] = {lo, (uint64_t)hi, hi < 0 ? ~0ULL : 0ULL};
  uint64_t c = 0;
  for (int k = 0; k < 3; ++k) {
    const uint64_t a = (uint64_t)s[k];
    const uint64_t t = a + x[k];
    const uint64_t c1 = t < a ? 1 : 0;
    const uint64_t u = t + c;
    const uint64_t c2 = u < t ? 1 : 0;
    s[k] = (int64_t)u;
    c = c1 + c2;
  }
}
DQ_HD void add192_3(int64_t* s, const int64_t* b) {
  uint64_t c = 0;
  for (int k = 0; k < 3; ++k) {
    const uint64_t a = (uint64_t)s[k];
    const uint64_t t = a + (uint64_t)b[k];
    const uint64_t c1 = t < a ? 1 : 0;
    const uint64_t u = t + c;
    const uint64_t c2 = u < t ? 1 : 0;
    s[k] = (int64_t)u;
    c = c1 + c2;
  }
}

DQ_HD int64_t wrap_add(int64_t a, int64_t b) {
  return (int64_t)((uint64_t)a + (uint64_t)b);
}

// Total-order key of a double that sorts like Spark's NaN-safe comparison (NaN largest).  Both
// zeros keep their own keys (-0.0 < 0.0), so the extreme is deterministic.
DQ_HD int64_t f64_key(double x) {
  if (x != x) return INT64_MAX;
  int64_t b = __builtin_bit_cast(int64_t, x);
  return b >= 0 ? b : (b ^ INT64_MAX);
}
DQ_HD double f64_from_key(int64_t k) {
  if (k == INT64_MAX) return __builtin_bit_cast(double, (int64_t)0x7ff8000000000000LL);
  int64_t b = k >= 0 ? k : (k ^ INT64_MAX);
  return __builtin_bit_cast(double, b);
}

// Chan et al. pairwise merge of (n, avg, m2), written as Spark's CentralMomentAgg merge /
// StandardDeviationState.sum (StandardDeviation.scala:37-44).
DQ_HD void moments_merge(double na, double& avg, double& m2, double nb, double avg_b, double m2_b) {
  double n = na + nb;
  double delta = avg_b - avg;
  double delta_n = (n == 0.0) ? 0.0 : delta / n;
  avg = avg + delta_n * nb;
  m2 = m2 + m2_b + delta * delta_n * na * nb;
}

// Spark Corr merge / CorrelationState.sum (Correlation.scala:37-52).
DQ_HD void comoments_merge(double n1, double* a, double n2, const double* b) {
  double n = n1 + n2;
  double dx = b[0] - a[0];
  double dxn = (n == 0.0) ? 0.0 : dx / n;
  double dy = b[1] - a[1];
  double dyn = (n == 0.0) ? 0.0 : dy / n;
  a[0] = a[0] + dxn * n2;
  a[1] = a[1] + dyn * n2;
  a[2] = a[2] + b[2] + dx * dyn * n1 * n2;
  a[3] = a[3] + b[3] + dx * dxn * n1 * n2;
  a[4] = a[4] + b[4] + dy * dyn * n1 * n2;
}

// Merge of two aggregation buffers of the same task (Spark's partial-aggregate merge).
DQ_HD void acc_merge(int kind, Acc& a, const Acc& b) {
  switch (kind) {
    case TK_NUMERIC: {
      if (b.i[0] == 0 && b.i[7] == 0 && b.i[8] == 0 && b.i[9] == 0) return;
      double na = (double)a.i[0], nb = (double)b.i[0];
      if (b.i[0] > 0) {
        if (a.i[0] == 0) {
          a.d[1] = b.d[1];
          a.d[2] = b.d[2];
        } else {
          moments_merge(na, a.d[1], a.d[2], nb, b.d[1], b.d[2]);
        }
      }
      a.i[0] += b.i[0];
      a.i[1] = wrap_add(a.i[1], b.i[1]);
      a.i[2] = a.i[2] < b.i[2] ? a.i[2] : b.i[2];
      a.i[3] = a.i[3] > b.i[3] ? a.i[3] : b.i[3];
      for (int k = 4; k < 10; ++k) a.i[k] += b.i[k];
      a.d[0] += b.d[0];
      break;
    }
    case TK_COMOMENTS: {
      if (b.i[0] == 0) return;
      if (a.i[0] == 0) {
        a = b;
        return;
      }
      comoments_merge((double)a.i[0], a.d, (double)b.i[0], b.d);
      a.i[0] += b.i[0];
      break;
    }
    case TK_DTYPE:
      for (int k = 0; k < 5; ++k) a.i[k] += b.i[k];
      break;
    case TK_DECIMAL: {
      if (b.i[0] == 0) return;
      if (a.i[0] == 0) {
        a = b;
        return;
      }
      moments_merge((double)a.i[0], a.d[1], a.d[2], (double)b.i[0], b.d[1], b.d[2]);
      a.i[0] += b.i[0];
      add192_3(&a.i[1], &b.i[1]);
      if (i128_lt(b.i[4], b.i[5], a.i[4], a.i[5])) {
        a.i[4] = b.i[4];
        a.i[5] = b.i[5];
      }
      if (i128_lt(a.i[6], a.i[7], b.i[6], b.i[7])) {
        a.i[6] = b.i[6];
        a.i[7] = b.i[7];
      }
      break;
    }
    default:
      a.i[0] += b.i[0];
      a.i[1] += b.i[1];
      break;
  }
}

// ------------------------------------------------------------------------------------------------
// XXH64 (Spark XXH64 == the standard algorithm over the value's little-endian bytes).
// ------------------------------------------------------------------------------------------------
constexpr uint64_t P1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t P2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t P3 = 0x165667B19E3779F9ULL;
constexpr uint64_t P4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t P5 = 0x27D4EB2F165667C5ULL;

DQ_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
DQ_HD uint64_t xxh_fmix(uint64_t h) {
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}
// XXH64.hashLong(input, seed)
DQ_HD uint64_t xxh_long(uint64_t v, uint64_t seed) {
  uint64_t h = seed + P5 + 8;
  uint64_t k = rotl64(v * P2, 31) * P1;
  h ^= k;
  h = rotl64(h, 27) * P1 + P4;
  return xxh_fmix(h);
}
// XXH64.hashInt(input, seed)
DQ_HD uint64_t xxh_int(uint32_t v, uint64_t seed) {
  uint64_t h = seed + P5 + 4;
  h ^= (uint64_t)v * P1;
  h = rotl64(h, 23) * P2 + P3;
  return xxh_fmix(h);
}
DQ_HD uint64_t xxh_round(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl64(acc, 31);
  return acc * P1;
}
DQ_HD uint64_t xxh_merge_round(uint64_t acc, uint64_t v) {
  acc ^= xxh_round(0, v);
  return acc * P1 + P4;
}

// XXH64.hashUnsafeBytes over `len` bytes read through `Reader` (reader.u64(off), .u32(off),
// .u8(off) return little-endian values at byte offset off).
template <typename Reader>
DQ_HD uint64_t xxh_bytes(const Reader& rd, int64_t len, uint64_t seed) {
  int64_t off = 0;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    int64_t limit = len - 32;
    do {
      v1 = xxh_round(v1, rd.u64(off));
      v2 = xxh_round(v2, rd.u64(off + 8));
      v3 = xxh_round(v3, rd.u64(off + 16));
      v4 = xxh_round(v4, rd.u64(off + 24));
      off += 32;
    } while (off <= limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh_merge_round(h, v1);
    h = xxh_merge_round(h, v2);
    h = xxh_merge_round(h, v3);
    h = xxh_merge_round(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  while (off + 8 <= len) {
    h ^= xxh_round(0, rd.u64(off));
    h = rotl64(h, 27) * P1 + P4;
    off += 8;
  }
  if (off + 4 <= len) {
    h ^= (uint64_t)rd.u32(off) * P1;
    h = rotl64(h, 23) * P2 + P3;
    off += 4;
  }
  while (off < len) {
    h ^= (uint64_t)rd.u8(off) * P5;
    h = rotl64(h, 11) * P1;
    off += 1;
  }
  return xxh_fmix(h);
}

// XXH64.hashUnsafeBytes (xxh_bytes above) of a string of len <= 64 bytes held in registers:
// w[j] = its bytes [4j, 4j + 4).  Every step of xxh_bytes is unrolled with compile-time register
// indices, taken under its own condition on len, so no register array is indexed at run time.
DQ_HD uint64_t xxh_bytes_regs64(const uint32_t (&w)[16], int32_t len, uint64_t seed) {
  auto w64 = [&](int j) { return (uint64_t)w[2 * j] | ((uint64_t)w[2 * j + 1] << 32); };
  uint64_t h;
  const int ns = len >> 5;  // 32-byte stripes: 0, 1 or 2
  if (ns) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    v1 = xxh_round(v1, w64(0));
    v2 = xxh_round(v2, w64(1));
    v3 = xxh_round(v3, w64(2));
    v4 = xxh_round(v4, w64(3));
    if (ns > 1) {
      v1 = xxh_round(v1, w64(4));
      v2 = xxh_round(v2, w64(5));
      v3 = xxh_round(v3, w64(6));
      v4 = xxh_round(v4, w64(7));
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh_merge_round(h, v1);
    h = xxh_merge_round(h, v2);
    h = xxh_merge_round(h, v3);
    h = xxh_merge_round(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
#pragma unroll
  for (int j = 0; j < 8; ++j) {  // the 8-byte words after the stripes
    if (j >= 4 * ns && 8 * j + 8 <= len) {
      h ^= xxh_round(0, w64(j));
      h = rotl64(h, 27) * P1 + P4;
    }
  }
  const int nw = len >> 3;
  if ((len & 7) >= 4) {  // one 4-byte word at 8 * nw
    uint32_t d = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) d = j == nw ? w[2 * j] : d;
    h ^= (uint64_t)d * P1;
    h = rotl64(h, 23) * P2 + P3;
  }
  const int nb = len & 3;
  if (nb) {  // the last len % 4 bytes, from the dword at 4 * (len / 4)
    uint32_t d = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) d = j == (len >> 2) ? w[j] : d;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      if (b < nb) {
        h ^= (uint64_t)((d >> (8 * b)) & 0xffu) * P5;
        h = rotl64(h, 11) * P1;
      }
    }
  }
  return xxh_fmix(h);
}

struct HostBytes {
  const uint8_t* p;
  DQ_HD uint64_t u64(int64_t o) const {
    uint64_t v = 0;
    for (int k = 7; k >= 0; --k) v = (v << 8) | p[o + k];
    return v;
  }
  DQ_HD uint32_t u32(int64_t o) const {
    uint32_t v = 0;
    for (int k = 3; k >= 0; --k) v = (v << 8) | p[o + k];
    return v;
  }
  DQ_HD uint32_t u8(int64_t o) const { return p[o]; }
};

// HLL++ register update for one hash (StatefulHyperloglogPlus.update :87-113): index from the top
// P bits, rank = number of leading zeros of the remaining bits (padded) + 1.
DQ_HD void hll_index_rank(uint64_t x, uint32_t& idx, uint32_t& pw) {
  idx = (uint32_t)(x >> (64 - kHllP));
  uint64_t w = (x << kHllP) | (1ULL << (kHllP - 1));
  pw = (uint32_t)__builtin_clzll(w) + 1;
}

}  // namespace dq
