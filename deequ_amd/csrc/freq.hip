// freq.hip -- the hash group-by of the frequency analyzers (FrequencyBasedAnalyzer.
// computeFrequencies, GroupingAnalyzers.scala:53-80; Histogram.scala:54-69) and the one
// aggregation over the frequency table that every ScanShareableFrequencyBasedAnalyzer shares
// (AnalysisRunner.scala:490-500): Σ[count == 1], count(*), Σ −(c/n)·ln(c/n); plus Histogram's
// top-N (Histogram.scala:78-79).
//
// A radix-partitioned group-by, so that every pass streams HBM and every count happens in LDS
// (random HBM atomics into a billion-slot table ran at 1.4 % of HBM peak in round 1):
//
//   phase A (per added batch; freq_phaseA): one 1024-thread workgroup per chunk of 8192 rows
//     (4096 in hashed mode).  Each row's key is hashed (freq_codec.h); the first 1024 rows of the
//     chunk go through a 2048-slot LDS table that collapses repeated keys (bypassed for the rest
//     of the chunk when fewer than 1/16 of them repeated, i.e. high-cardinality keys), and every
//     resulting record is counting-sorted in LDS by the top 9 bits of its hash (512 buckets) and
//     written out as ONE contiguous chunk region plus a 513-entry u16 bucket histogram.
//   phase B (finalize; freq_phaseB): the chunk histograms are transposed and scanned per bucket;
//     a bucket's records are cut into units of ~kTile/2 records (whole chunk segments), and each
//     unit is counting-sorted by the next s hash bits (s chosen so that a final partition holds a
//     few thousand groups) into a contiguous output plus its sub-bucket histogram.
//   phase C (finalize; freq_phaseC): one workgroup per partition (bucket, sub-bucket) gathers its
//     pieces of every unit of the bucket and counts them in an LDS hash table (8192 slots exact,
//     4608 hashed), then emits the partition's Σ[c==1], #groups and entropy partial, optionally
//     its top-4 groups (Histogram) or every group (export, merge, repartition).  A partition whose
//     groups do not fit is recounted in 2, 4, ... passes over disjoint hash subsets.
//
// Exact mode (one fixed-width key) carries 8-byte records (h << 8 | count digit) whose hash is a
// bijection of the value; hashed mode (strings, several keys, Histogram on strings) carries
// 16-byte records {h, rep << 8 | count digit} where rep points at the group's encoded key in a
// device arena, and groups that meet on one hash are compared byte for byte (freq_codec.h), so a
// 64-bit collision never merges groups.  Counts of equal keys are SUMMED in every pass, which is
// also what FrequenciesAndNumRows.sum (GroupingAnalyzers.scala:128-148) needs: merging two tables
// appends one's chunks to the other's.
#include <hip/hip_runtime.h>

#include <type_traits>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <array>
#include <map>
#include <mutex>
#include <vector>

#include "engine.h"
#include "freq_codec.h"
#include "kernels.h"
#include "stream_load.h"

// freq_phaseC_x's probe rounds: branch-light (1) or round 5's per-record branches (0, a build
// for A/B runs through DQ_LIB_PATH)
#ifndef DQ_LEAN_PROBE
#define DQ_LEAN_PROBE 1
#endif
#ifndef DQ_C_EXPERIMENT  // timing builds only (wrong results): 1 no statistics, 2 no inserts
#define DQ_C_EXPERIMENT 0
#endif
#ifndef DQ_AX_EXPERIMENT  // timing builds only (wrong results): freq_phaseA_xp 1 no record stores,
#define DQ_AX_EXPERIMENT 0  // 2 no counting sort (records in row order), 3 neither
#endif
#ifndef DQ_A_NOCOPY  // timing builds only (wrong results): phase A writes no arena key bytes
#define DQ_A_NOCOPY 0
#endif

namespace dq {

#define DQ_DEV __device__ __forceinline__

constexpr int kBucketBits = 9;
constexpr int kBuckets = 1 << kBucketBits;
constexpr int kHistRow = kBuckets + 1;  // u16 exclusive bucket prefix of a chunk + its total
constexpr int kThreads = 1024;
constexpr int kMaxSubBits = 10;
constexpr int kMinPkSubBits = 7;  // packed phase-C slots need a partition of >= 9 + 7 fixed bits
constexpr int kFilterShift = 32;        // hash bits that split an overflowing partition
constexpr int kCand = 4;                // top groups kept per partition for Histogram
constexpr int kSmallCounts = 64;        // phase C histograms group counts below this
constexpr int kMaxParts = 64;
constexpr uint64_t kEmptyKey = ~0ULL;
constexpr uint64_t kNotReady = ~0ULL;

// C_MAXCNT: an upper bound of the count any phase-A record carries (packed phase-C slots at
// fewer than kMaxSubBits sub-bits need every record count below 2^(s-3); merges add the bounds)
// C_NAN_FOLDED: keyed rows of a Histogram-mode floating-point table whose NaN payload was folded
// into the canonical NaN (zero: the table's groups are also the grouping's, dq_freq_folded_nan_rows)
enum Counter { C_NULL_ROWS = 0, C_NULL_GROUP, C_COLLISIONS, C_DBG_NOTREADY, C_DBG_DIFF, C_DBG_FULL, C_DBG_BYPASS,
               C_MAXCNT, C_NAN_FOLDED, C_N };

template <bool HASHED>
struct FM;
template <>
struct FM<false> {
  static constexpr int kTile = 8192;    // rows (and at most records) per phase-A chunk
  static constexpr int kRB = 8;         // bytes per record
  static constexpr int kDedupe = 2048;  // phase-A LDS table slots
  static constexpr int kTableC = 4096;  // phase-C LDS table slots (two workgroups per CU)
  static constexpr int kTarget = 2000;  // records per final partition the sizing aims at
};
template <>
struct FM<true> {
  static constexpr int kTile = 2048;
  static constexpr int kRB = 16;
  static constexpr int kDedupe = 1024;
  static constexpr int kTableC = 2560;
  // (freq_phaseC_h takes up to 4096 records and 3584 groups per partition: ~1900-record partitions
  // halve its per-item costs against ~950, configs[4] 176.3 -> 171.5 ms, A/B
  // DQ_FREQ_PARTITION_TARGET_H)
  static constexpr int kTarget = 2400;
};
// records per phase-B unit (whole chunk segments of one bucket): hashed two tiles (~32 records per
// partition run); exact one (8192 records: the whole-unit scatter then stages 64 KB and two
// workgroups share a CU, configs[2] 26.3 -> 25.0 ms)
constexpr int kUnitTilesH = 2, kUnitTilesX = 1;

struct RecIn {  // == dq_freq_record
  uint64_t key;
  uint64_t count;
  uint64_t enc_off;
};

struct Group {  // one materialised group
  uint64_t h;
  uint64_t count;
  uint64_t rep;  // hashed: arena offset of the encoded key
};

struct FEntry {  // phase-C work item of a recount: partition p, hash subset v of 2^f
  uint32_t p, f, v, pad;
};

struct SrcSegs {
  int64_t rec_start[kMaxParts + 1];
  int64_t var_base[kMaxParts];
  int32_t n_src;
};

// ------------------------------------------------------------------------------------------------
// Device helpers
// ------------------------------------------------------------------------------------------------
DQ_DEV uint64_t lds_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
DQ_DEV void lds_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ockl wavefront reductions / scans: DPP row and broadcast steps, no LDS round trips (the
// __shfl_* forms are ds_bpermute, a few hundred cycles for a 6-step 64-bit chain)
extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);
extern "C" __device__ uint64_t __ockl_wfred_add_u64(uint64_t);
extern "C" __device__ double __ockl_wfred_add_f64(double);
extern "C" __device__ uint64_t __ockl_wfred_max_u64(uint64_t);
extern "C" __device__ uint32_t __ockl_wfscan_add_u32(uint32_t, bool);

// Exclusive scan of one u32 per thread over the workgroup; returns the thread's prefix and sets
// `total`.  Every thread of the block must call it.
DQ_DEV uint32_t block_excl_scan(uint32_t v, uint32_t* s_wave, uint32_t& total) {
  const int lane = __lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t x = __ockl_wfscan_add_u32(v, true);
  if (lane == 63) s_wave[wave] = x;
  __syncthreads();
  if (wave == 0) {
    const uint32_t w = __ockl_wfscan_add_u32(lane < nw ? s_wave[lane] : 0u, true);
    if (lane < nw) s_wave[lane] = w;
  }
  __syncthreads();
  const uint32_t base = wave ? s_wave[wave - 1] : 0u;
  total = s_wave[nw - 1];
  __syncthreads();
  return base + x - v;
}

template <typename T>
DQ_DEV T wave_sum(T v) {
  if constexpr (std::is_same_v<T, double>) return __ockl_wfred_add_f64(v);
  else if constexpr (sizeof(T) == 8) return (T)__ockl_wfred_add_u64((uint64_t)v);
  else return (T)__ockl_wfred_add_u32((uint32_t)v);
}

// Fixed-order block sums (every thread calls; the result is valid in every thread).
DQ_DEV uint64_t block_sum_u64(uint64_t v, uint64_t* s) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (__lane_id() == 0) s[wave] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int w = 0; w < nw; ++w) t += s[w];
  __syncthreads();
  return t;
}
DQ_DEV double block_sum_f64(double v, double* s) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (__lane_id() == 0) s[wave] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < nw; ++w) t += s[w];
  __syncthreads();
  return t;
}

// Sum over the wave, added to a table counter by lane 0 (counters are single addresses).
DQ_DEV void wave_count(unsigned long long* counter, unsigned long long v) {
  v = wave_sum(v);
  if (__lane_id() == 0 && v) atomicAdd(counter, v);
}
extern "C" __device__ uint64_t __ockl_wfred_max_u64(uint64_t);
// A workgroup's largest record count into an LDS word, only when it could bar packed slots
// (>= 16 = 2^(7-3)); the workgroup then makes one global atomic (one per wave on one address
// serialised phase A over records: 9.4 -> 50 ms per configs[4] run)
DQ_DEV void wave_max_lds(unsigned long long* s_slot, uint64_t v) {
  v = __ockl_wfred_max_u64(v);
  if (__lane_id() == 0 && v >= 16) atomicMax(s_slot, (unsigned long long)v);
}

// last index j in [0, n) with pos[j] <= x (pos non-decreasing, pos[0] = 0 <= x)
DQ_DEV uint32_t seg_of(const uint32_t* pos, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;  // answer in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pos[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

DQ_DEV int64_t seg_var_base(const SrcSegs& s, int64_t i) {
  int j = 0;
  while (j + 1 < s.n_src && i >= s.rec_start[j + 1]) ++j;
  return s.var_base[j];
}

template <typename F>
DQ_DEV void for_digits(uint64_t c, F&& f) {
  for (uint32_t e = 0; c; c >>= 2, ++e)
    if (c & 3) f((e << 2) | (uint32_t)(c & 3));
}

DQ_DEV uint32_t bucket_of(uint64_t h) { return (uint32_t)(h >> (64 - kBucketBits)); }
// sub-bucket (the s hash bits below the bucket bits); x = h or the exact record >> 8 (both hold
// hash bits 54..0 in place)
DQ_DEV uint32_t sub_of(uint64_t x, int s) {
  return s ? (uint32_t)((x >> (64 - kBucketBits - s)) & ((1u << s) - 1u)) : 0u;
}
DQ_DEV uint64_t xrec_h(uint64_t rec, uint32_t b) {
  return ((uint64_t)b << 55) | ((rec >> 8) & ((1ULL << 55) - 1));
}

// ------------------------------------------------------------------------------------------------
// Phase A: rows (or received records) -> bucket-sorted chunk regions
//
// Each workgroup takes `tiles_per_wg` consecutive tiles.  Its LDS dedupe table persists across
// those tiles, so a low-cardinality key (priority: 3 groups) leaves the workgroup as a handful of
// records for its whole range, written at the end into the workgroup's own extra chunk
// (n_tiles + blockIdx.x).  Round 0 of every 8th tile measures the table's hit rate; below 1/16
// the table is bypassed (high cardinality: it would only cost probes).  Every tile's other rows
// are counting-sorted by bucket into the tile's chunk region.
// ------------------------------------------------------------------------------------------------
struct AArgs {
  KeySet ks;
  int32_t types[kMaxKeys];
  int32_t n_keys;
  int32_t tiles_per_wg;
  int64_t n_items;
  int64_t tile_items;
  const RecIn* rin;
  uint64_t var_arena_base;
  SrcSegs segs;
  uint8_t* recs;
  uint16_t* hist;
  uint8_t* arena;
  unsigned long long* arena_cursor;
  unsigned long long* counters;
  unsigned long long* dbg_clock;  // DQ_FREQ_DEBUG=2: workgroup 0's phase timestamps (wall clock)
  // the small-key path (freq_phaseA_small) tried this batch first when fast_epoch != 0:
  // fast_words = {epoch of the last batch it could not take, its NULL rows, its NULL-group rows}
  unsigned long long* fast_words;
  uint64_t fast_epoch;
  int32_t vec_ok;  // offsets / validity aligned for the 16-byte / dword streaming loads
  int32_t fast_poll;  // steps between polls of the give-up word (0: never)
  // the batch's groups merged across workgroups (freq_phaseA_small): kBatchSlots keys (+1, 0 =
  // free), their counts, then the workgroups' arrival counter; zeroed before the launch
  unsigned long long* batch_tab;
  // freq_phaseA_small: general-kernel workgroups (tile ranges + chunk) per small-kernel workgroup
  int32_t small_merge;
  // exact rows, bucket pieces (pstart != nullptr): the batch's records go to one region of
  // n_items records at `recs`, bucket-major; workgroup w's records of bucket b fill the piece that
  // starts at tot-prefix(b) + ph[w][b] (freq_prepass_x / freq_prepass_scan), and the workgroup
  // writes its pieces' starts and lengths (rows of the table's piece arrays)
  const uint32_t* ph;    // [n_wg][kBuckets]: exclusive prefix over workgroups, per bucket
  const uint32_t* ptot;  // [kBuckets]: the batch's rows per bucket
  uint32_t* pstart;      // [n_wg][kBuckets]
  uint32_t* plen;        // [n_wg][kBuckets]
  // one-utf8-column rows into bucket pieces of fixed capacity (pstart != nullptr in
  // freq_phaseA<STR1>): piece (workgroup w, bucket b) holds up to piece_cap records at
  // piece_base + (w * kBuckets + b) * piece_cap; a tile's records past a full piece go to its chunk
  uint32_t piece_cap;
  uint64_t piece_base;
  // dense integer keys (freq_dense_count / freq_dense_emit; nullptr: not tried for this batch):
  // {max, ~min} of the keyed values (sign-flipped, so unsigned order is signed order; 0 = none),
  // the epoch of the last batch the dense path took, the epoch of the last one it declined
  unsigned long long* dense_words;
  uint64_t dense_epoch;
  // freq_phaseA_xp: hist rows [zero_off, zero_off + zero_rows) (the batch's piece chunks, which
  // hold no records) zeroed by the kernel's workgroups instead of a memset launch per batch
  int64_t zero_off, zero_rows;
};

// Dedupe slots: every entry's count digits must fit the flush chunk (D x digits <= kTile), and
// the LDS must allow two workgroups per CU (<= 80 KB).
// Device forms of row_hash_hashed / row_encode (freq_codec.h) for phase A's multi-column keys: a
// utf8 value of at most 16 bytes is read once, as the aligned dwords that hold it (load_str16:
// every read holds a byte of the string), instead of byte by byte.  Same results: load_str16 and
// the byte path give the same words (tools/freq_codec_check.cpp).
DQ_DEV uint64_t row_hash_hashed_dw(const KeySet& ks, int64_t r) {
  uint64_t h = kRowHashSeed;
  for (int k = 0; k < ks.n_keys; ++k) {
    const KeyCol& c = ks.cols[k];
    uint64_t ch;
    if (c.type == DQ_UTF8) {
      SView v;
      key_str(ks, k, r, v);
      if (v.p && v.len <= kHash16Max) {
        uint64_t w0, w1;
        load_str16(v.p, v.len, w0, w1);
        ch = str_hash16(w0, w1, v.len, 17 + k);
      } else {
        ch = str_col_hash(v, k);
      }
    } else {
      ch = xxh_long(kwiden(c.type, c.values, r), 17 + k);
    }
    h = fold_col_hash(h, ch);
  }
  return fmix_bij(h);
}

DQ_DEV void row_encode_dw(const KeySet& ks, int64_t r, uint32_t* dst) {
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
      if (v.p && v.len <= kHash16Max) {
        uint64_t w0, w1;
        load_str16(v.p, v.len, w0, w1);
        const uint32_t d[4] = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (4 * q < v.len) *dst++ = d[q];
      } else {
        for (int32_t q = 0; q < v.len; q += 4) {
          uint32_t w = 0;
          for (int b = 0; b < 4 && q + b < v.len; ++b) w |= sv_byte(v, q + b) << (8 * b);
          *dst++ = w;
        }
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

// Short form of a two-utf8-column key whose values are both at most 7 bytes (the MutualInformation
// joints of low-cardinality string columns): k0, k1 = each value's bytes | its length << 56, an
// exact key, so phase A's dedupe decides a hit in LDS (dsk0 / dsk1) instead of re-reading both
// rows' strings; any other key has k1 = kNoShort.  (Keyed rows of a multi-column key have no NULL.)
DQ_DEV void multi_short_key(const KeySet& ks, int64_t r, uint64_t& k0, uint64_t& k1) {
  k0 = 0;
  k1 = kNoShort;
  if (ks.n_keys != 2 || ks.cols[0].type != DQ_UTF8 || ks.cols[1].type != DQ_UTF8) return;
  uint64_t w[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    SView v;
    if (!key_str(ks, k, r, v) || !v.p || v.len > 7) return;
    uint64_t w0, w1;
    load_str16(v.p, v.len, w0, w1);
    w[k] = w0 | ((uint64_t)v.len << 56);
  }
  k0 = w[0];
  k1 = w[1];
}

// Two-utf8-column keys (the MutualInformation joints of string columns) in phase A: each row's
// offsets, then <= 16 bytes per value as the aligned dwords that hold them (STR1's row loads), so
// a thread issues every round's loads before it uses any; the row hash, short key and encoding
// are row_hash_hashed_dw's, multi_short_key's and row_encode_dw's, computed from registers.
struct Str2Row {
  int32_t s0[2], len[2];
  int sh[2];
  uint32_t d[2][5];
};
DQ_DEV bool str2_key(const KeySet& ks) {
  return ks.n_keys == 2 && ks.cols[0].type == DQ_UTF8 && ks.cols[1].type == DQ_UTF8 && !ks.null_as_group;
}
DQ_DEV void str2_offsets(const KeySet& ks, int64_t r, Str2Row& x) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int32_t* off = reinterpret_cast<const int32_t*>(ks.cols[c].values);
    x.s0[c] = off[r];
    x.len[c] = off[r + 1];
  }
}
// (after str2_offsets' loads: len becomes the length; a value that is empty, NULL or longer
// than 16 bytes reads its column's first offset instead, always mapped)
DQ_DEV void str2_bytes(const KeySet& ks, Str2Row& x) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    x.len[c] -= x.s0[c];
    const bool reg = x.len[c] > 0 && x.len[c] <= 16;
    const uint8_t* p = reg ? ks.cols[c].data + x.s0[c] : reinterpret_cast<const uint8_t*>(ks.cols[c].values);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    x.sh[c] = (int)(reinterpret_cast<uintptr_t>(p) & 3u);
    const int last = reg ? ((x.sh[c] + x.len[c] + 3) >> 2) - 1 : 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) x.d[c][k] = q[k < last ? k : last];
  }
}
DQ_DEV void str2_words(const Str2Row& x, int c, uint64_t& w0, uint64_t& w1) {
  w0 = w1 = 0;
  if (x.len[c] > 0 && x.len[c] <= kHash16Max) str16_from_dwords(x.d[c], x.sh[c], x.len[c], w0, w1);
}
DQ_DEV uint64_t str2_hash(const KeySet& ks, const Str2Row& x, uint64_t& k0, uint64_t& k1) {
  uint64_t h = kRowHashSeed, sw[2];
  bool shrt = true;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    uint64_t w0, w1;
    str2_words(x, c, w0, w1);
    const uint64_t ch = x.len[c] <= kHash16Max ? str_hash16(w0, w1, x.len[c], 17 + c)
                                               : str_hash_long_dev(ks.cols[c].data + x.s0[c], x.len[c], c);
    h = fold_col_hash(h, ch);
    shrt = shrt && x.len[c] <= 7;
    sw[c] = w0 | ((uint64_t)(uint32_t)x.len[c] << 56);
  }
  k0 = shrt ? sw[0] : 0;
  k1 = shrt ? sw[1] : kNoShort;
  return fmix_bij(h);
}
DQ_DEV uint32_t str2_enc_size(const Str2Row& x) {
  return 16 + pad4((uint32_t)x.len[0]) + pad4((uint32_t)x.len[1]);
}
DQ_DEV void str2_encode(const KeySet& ks, const Str2Row& x, uint32_t* dst) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    *dst++ = 1;
    *dst++ = (uint32_t)x.len[c];
    if (x.len[c] <= kHash16Max) {
      uint64_t w0, w1;
      str2_words(x, c, w0, w1);
      const uint32_t d[4] = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (4 * q < x.len[c]) *dst++ = d[q];
    } else {
      const uint8_t* b = ks.cols[c].data + x.s0[c];
      for (int32_t q = 0; q < x.len[c]; q += 4) {
        uint32_t w = 0;
        for (int k = 0; k < 4 && q + k < x.len[c]; ++k) w |= (uint32_t)b[q + k] << (8 * k);
        *dst++ = w;
      }
    }
  }
}

template <bool HASHED, bool FROM_REC>
struct AKeys {
  static constexpr int kDedupe = FROM_REC ? (HASHED ? 128 : 256) : (HASHED ? 256 : 512);
  // a workgroup's rows: counts < 4^(kTile / kDedupe), so the digits of every entry fit
  // (records: tiles of tile / max-digits records, so many per workgroup -- one per workgroup made a
  // 1.2e8-record marginal 234 K workgroups and as many workgroup chunks)
  static constexpr int kTilesPerWg = FROM_REC ? 16 : (HASHED ? 15 : 16);
  // the string rows: 512-thread workgroups, two per CU (LDS <= 80 KB, <= 128 VGPRs), so one
  // workgroup's load latency overlaps the other's hashing and dedupe between their barriers
  static constexpr int kThreads = HASHED && !FROM_REC ? 512 : 1024;
  static constexpr int kMinWaves = HASHED && !FROM_REC ? 4 : 1;  // per SIMD: two workgroups
};

// STR1: the key is one utf8 column (its own instantiation: the generic multi-column path would
// otherwise hold registers the string path needs, and spill)
template <bool HASHED, bool FROM_REC, bool STR1 = false>
__global__ void __launch_bounds__((AKeys<HASHED, FROM_REC>::kThreads),
                                  (AKeys<HASHED, FROM_REC>::kMinWaves)) freq_phaseA(AArgs a) {
  constexpr int kThreads = AKeys<HASHED, FROM_REC>::kThreads;
  using M = FM<HASHED>;
  constexpr int T = M::kTile, D = AKeys<HASHED, FROM_REC>::kDedupe, W = M::kRB / 8;
  constexpr int ROUNDS = FROM_REC ? 1 : T / kThreads;
  __shared__ uint32_t bh[kBuckets], bcur[kBuckets];
  __shared__ uint64_t dkey[D], dcnt[D];
  __shared__ uint64_t drep[HASHED ? D : 1];
  // one-column utf8 keys: the short forms (str_short_key) of the slots' keys and the tile's rows,
  // so most hits are decided in LDS instead of re-reading both strings
  constexpr bool SK = HASHED && !FROM_REC;
  __shared__ uint64_t dsk0[SK ? D : 1], dsk1[SK ? D : 1];
  __shared__ uint64_t ssk0[SK ? T : 1], ssk1[SK ? T : 1];
  __shared__ uint32_t s_wave[kThreads / 64];
  __shared__ uint64_t s_red[kThreads / 64];
  __shared__ uint32_t s_hits, s_bypass;
  __shared__ unsigned long long s_arena_base, s_arena_cur;
  // the tile's rows, hashed: exact h per row; hashed (h, row index or arena offset) per row.  The
  // round loops read it back with dynamic indices (no unrolling: the kernel stays small enough for
  // the instruction cache).
  __shared__ uint64_t stash[T * W];
  __shared__ uint64_t scnt[FROM_REC ? kThreads : 1];
  // exact rows into bucket pieces (a.pstart): each bucket's next record slot in the batch region
  constexpr bool XP = !HASHED && !FROM_REC;
  __shared__ uint32_t wcur[XP ? kBuckets : 1];
  // STR1 rows into fixed-capacity bucket pieces: each piece's fill (u16: the LDS of two
  // workgroups per CU has 1.7 KB left)
  __shared__ uint16_t wfill[STR1 ? kBuckets : 1];
  const bool hpieces = STR1 && a.pstart != nullptr;
  const bool str2 = HASHED && !FROM_REC && !STR1 && str2_key(a.ks);  // (block-uniform)

  const int tid = threadIdx.x;
  if constexpr (STR1) {
    if (a.fast_epoch) {  // freq_phaseA_small ran first: it either took the batch or gave it up
      const bool taken = a.fast_words[0] != a.fast_epoch;
      if (blockIdx.x == 0 && tid == 0) {  // its NULL counts count only if its output stands
        if (taken) {
          a.counters[C_NULL_ROWS] += a.fast_words[1];
          a.counters[C_NULL_GROUP] += a.fast_words[2];
        }
        a.fast_words[1] = a.fast_words[2] = 0;
      }
      if (taken) return;
    }
  }
  const int64_t n_tiles = (a.n_items + a.tile_items - 1) / a.tile_items;
  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t t1 = min(t0 + (int64_t)a.tiles_per_wg, n_tiles);
  for (int i = tid; i < D; i += kThreads) {
    dkey[i] = kEmptyKey;
    dcnt[i] = 0;
    if (HASHED) drep[i] = kNotReady;
    if (SK) dsk1[i] = kShortNotReady;
  }
  for (int i = tid; i < kBuckets; i += kThreads) bh[i] = 0;
  if constexpr (STR1)
    if (hpieces)
      for (int i = tid; i < kBuckets; i += kThreads) wfill[i] = 0;
  if (tid == 0) s_bypass = 0;
  if constexpr (STR1) {
    // the arena bytes of every key this workgroup may encode, reserved once: at most 8 + len + 3
    // per row (a per-chunk reservation made every workgroup's tiles queue on the one cursor word)
    if (tid == 0) {
      const int32_t* off = reinterpret_cast<const int32_t*>(a.ks.cols[0].values);
      const int64_t r0 = min(t0 * a.tile_items, a.n_items), r1 = min(t1 * a.tile_items, a.n_items);
      // (16-byte aligned keys, str1_enc_size16: at most 8 + len + 3 + 12 bytes each)
      const uint64_t need = r1 > r0 ? (uint64_t)(r1 - r0) * 23 + (uint64_t)(off[r1] - off[r0]) + 16 : 0;
      const unsigned long long base = need ? atomicAdd(a.arena_cursor, (unsigned long long)need) : 0ULL;
      s_arena_base = (base + 15ULL) & ~15ULL;
      s_arena_cur = 0;
    }
  }
  const bool pieces = XP && a.pstart != nullptr;
  if constexpr (XP) {
    if (pieces) {
      // bucket b of the batch starts at the prefix of the batch's bucket totals; this workgroup's
      // piece of it at the prefix of the earlier workgroups' rows of b (freq_prepass_scan)
      uint32_t all;
      const uint32_t tot = tid < kBuckets ? a.ptot[tid] : 0u;
      const uint32_t bb = block_excl_scan(tot, s_wave, all);
      if (tid < kBuckets) {
        const uint32_t st = bb + a.ph[(int64_t)blockIdx.x * kBuckets + tid];
        wcur[tid] = st;
        a.pstart[(int64_t)blockIdx.x * kBuckets + tid] = st;
      }
      // the batch's chunk rows (tiles and workgroup chunks) hold no records: empty histograms
      const int64_t nt = (a.n_items + a.tile_items - 1) / a.tile_items;
      const int64_t r1 = min((int64_t)(blockIdx.x + 1) * a.tiles_per_wg, nt);
      for (int64_t r = (int64_t)blockIdx.x * a.tiles_per_wg; r < r1; ++r)
        for (int i = tid; i < kHistRow; i += kThreads) a.hist[r * kHistRow + i] = 0;
      for (int i = tid; i < kHistRow; i += kThreads) a.hist[(nt + blockIdx.x) * kHistRow + i] = 0;
    }
  }
  unsigned long long nulls = 0, nullg = 0;
  uint64_t maxcnt = 1;  // the largest count a record of this workgroup carries (row records: 1)
  // debug event counts (rare events) in LDS: dedupe is an out-of-line lambda, and locals it
  // updated through its captures lived in scratch
  __shared__ uint32_t s_dbg[3];  // not-ready retries, hash collisions, table full
  __shared__ unsigned long long s_maxcnt;
  if (tid < 3) s_dbg[tid] = 0;
  if (tid == 0) s_maxcnt = 0;
  unsigned long long dbg_bypass = 0;

  // Counting sort of a chunk's records: bucket counts are in bh; begin_chunk scans them, writes
  // the chunk's histogram row and reserves the chunk's arena bytes; records then go straight to
  // their place in the chunk region (a 64 KB region: the runs meet in L2).
  auto begin_chunk = [&](int64_t chunk, uint64_t arena_need) -> uint32_t {
    __syncthreads();
    uint32_t total;
    const uint32_t mine = tid < kBuckets ? bh[tid] : 0u;
    const uint32_t ex = block_excl_scan(mine, s_wave, total);
    uint16_t* hrow = a.hist + chunk * kHistRow;
    if (tid < kBuckets) {
      bcur[tid] = ex;
      hrow[tid] = (uint16_t)ex;
    }
    if (tid == 0) hrow[kBuckets] = (uint16_t)total;
    if constexpr (HASHED && !FROM_REC && !STR1) {
      const uint64_t all = block_sum_u64(arena_need, s_red);
      if (tid == 0) {
        s_arena_base = all ? atomicAdd(a.arena_cursor, (unsigned long long)all) : 0ULL;
        s_arena_cur = 0;
      }
    }
    __syncthreads();
    return total;
  };
  auto end_chunk = [&]() {
    __syncthreads();
    if constexpr (STR1)
      if (hpieces)  // the tile's records taken by each piece
        for (int i = tid; i < kBuckets; i += kThreads)
          wfill[i] = (uint16_t)(wfill[i] + min(bh[i], a.piece_cap - (uint32_t)wfill[i]));
    for (int i = tid; i < kBuckets; i += kThreads) bh[i] = 0;
    __syncthreads();
  };
  // STR1 pieces: the tile's chunk holds only what its pieces cannot take; bcur[b] = the bucket's
  // overflow offset in the chunk << 16 | the rank counter of its records in this tile
  auto begin_tile_pieces = [&](int64_t chunk) {
    __syncthreads();
    uint32_t ovf = 0, total;
    if (tid < kBuckets) ovf = bh[tid] - min(bh[tid], a.piece_cap - (uint32_t)wfill[tid]);
    const uint32_t ex = block_excl_scan(ovf, s_wave, total);
    uint16_t* hrow = a.hist + chunk * kHistRow;
    if (tid < kBuckets) {
      bcur[tid] = ex << 16;
      hrow[tid] = (uint16_t)ex;
    }
    if (tid == 0) hrow[kBuckets] = (uint16_t)total;
    __syncthreads();
  };
  auto put_pieces = [&](int64_t chunk, uint64_t h, uint32_t code, uint64_t rep) {
    const uint32_t b = bucket_of(h);
    const uint32_t o = atomicAdd(&bcur[b], 1u), k = o & 0xffffu;
    const uint32_t fill = wfill[b], take = min(bh[b], a.piece_cap - fill);
    const uint64_t slot = k < take
        ? a.piece_base + ((uint64_t)blockIdx.x * kBuckets + b) * a.piece_cap + fill + k
        : (uint64_t)chunk * T + (o >> 16) + (k - take);
    *reinterpret_cast<ulonglong2*>(reinterpret_cast<uint64_t*>(a.recs) + slot * W) =
        make_ulonglong2(h, (rep << 8) | code);
  };
  auto put = [&](int64_t chunk, uint64_t h, uint32_t code, uint64_t rep) {
    const uint32_t pos = atomicAdd(&bcur[bucket_of(h)], 1u);
    uint64_t* out = reinterpret_cast<uint64_t*>(a.recs) + (chunk * (int64_t)T + pos) * W;
    if constexpr (HASHED) {  // one 16-byte store (records are 16-byte aligned)
      *reinterpret_cast<ulonglong2*>(out) = make_ulonglong2(h, (rep << 8) | code);
    } else {
      out[0] = (h << 8) | code;
    }
  };
  auto arena_rep = [&](int64_t row) -> uint64_t {  // hashed rows: copy the key into the arena
    const uint32_t sz = STR1 ? str1_enc_size(a.ks, row) : row_enc_size(a.ks, row);
    const uint64_t off = s_arena_base + atomicAdd(&s_arena_cur, (unsigned long long)sz);
    if constexpr (STR1) {
      const SView v = str1_view(a.ks, row);
      if (!DQ_A_NOCOPY) str1_encode_copy(v.p, v.len, reinterpret_cast<uint32_t*>(a.arena + off));
    } else {
      if (!DQ_A_NOCOPY) row_encode_dw(a.ks, row, reinterpret_cast<uint32_t*>(a.arena + off));
    }
    return off;
  };
  // one-column utf8: a key of at most 15 bytes is encoded from its short form in LDS (k1 !=
  // kNoShort), with no global reads; a longer one through arena_rep
  auto enc_size_sk = [&](int64_t row, uint64_t k1) -> uint32_t {
    if constexpr (STR1)
      if (k1 != kNoShort) return 8 + pad4(str1_short_len(k1));
    return STR1 ? str1_enc_size(a.ks, row) : row_enc_size(a.ks, row);
  };
  auto arena_rep_sk = [&](int64_t row, uint64_t k0, uint64_t k1) -> uint64_t {
    if constexpr (STR1) {
      if (k1 != kNoShort) {
        const uint64_t off = s_arena_base +
            atomicAdd(&s_arena_cur, (unsigned long long)(8 + pad4(str1_short_len(k1))));
        if (!DQ_A_NOCOPY) str1_encode_short(k0, k1, reinterpret_cast<uint32_t*>(a.arena + off));
        return off;
      }
    }
    return arena_rep(row);
  };
  // LDS dedupe: 0 = not counted (table full), 1 = claimed a new slot, 2 = added to an existing
  // slot, 3 = the key's slot is being claimed: retry after the next barrier
  static_assert(!STR1 || (HASHED && !FROM_REC), "STR1 is the row path of a utf8 key");
  auto dedupe = [&](uint64_t h, uint64_t c, uint64_t rep, uint64_t k0, uint64_t k1) -> int {
    if (h == kEmptyKey) return 0;
    uint32_t slot = (uint32_t)(h >> 20) & (D - 1);
    for (int pr = 0; pr < 4; ++pr) {
      uint64_t k = lds_load(&dkey[slot]);
      // short utf8 keys: the slot's short form is read beside its key, so a hit costs two LDS
      // round trips (key + dsk1, then dsk0) instead of four.  A claimer writes the key, dsk0,
      // then (released) dsk1, and every field is written once: a dsk1 other than
      // kShortNotReady is final, and dsk0 read after it (acquire) is too.
      const uint64_t b1 = SK ? __hip_atomic_load(&dsk1[slot], __ATOMIC_ACQUIRE,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
      const uint64_t b0 = SK ? lds_load(&dsk0[slot]) : 0;
      bool claimed = false;
      if (k == kEmptyKey) {
        const uint64_t prev = atomicCAS((unsigned long long*)&dkey[slot], kEmptyKey, h);
        if (prev == kEmptyKey) claimed = true;
        else k = prev;
      }
      if (claimed) {
        if constexpr (SK) {
          lds_store(&dsk0[slot], k0);
          __hip_atomic_store(&dsk1[slot], k1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the short key before drep
        }
        if (HASHED) lds_store(&drep[slot], rep);
        atomicAdd((unsigned long long*)&dcnt[slot], c);
        return 1;
      }
      if (k == h) {
        bool same = true;
        if constexpr (HASHED) {
          if (SK && b1 == kShortNotReady) {  // being claimed right now (another lane / wave)
            atomicAdd(&s_dbg[0], 1u);
            return 3;
          }
          if (SK && (k1 != kNoShort || b1 != kNoShort)) {
            same = k1 == b1 && k0 == b0;
          } else {
            const uint64_t r2 = lds_load(&drep[slot]);
            if (r2 == kNotReady) {  // being claimed right now (another lane / wave)
              atomicAdd(&s_dbg[0], 1u);
              return 3;
            }
            if (r2 != rep) {
              if constexpr (FROM_REC)
                same = enc_equal_arena(reinterpret_cast<const uint32_t*>(a.arena + r2),
                                       reinterpret_cast<const uint32_t*>(a.arena + rep), a.types,
                                       a.n_keys);
              else if constexpr (STR1)
                same = str1_rows_equal(a.ks, (int64_t)r2, (int64_t)rep);
              else
                same = rows_equal(a.ks, (int64_t)r2, (int64_t)rep);
            }
          }
          if (!same) atomicAdd(&s_dbg[1], 1u);
        }
        if (same) {
          atomicAdd((unsigned long long*)&dcnt[slot], c);
          return 2;
        }
      }
      slot = (slot + 1) & (D - 1);
    }
    atomicAdd(&s_dbg[2], 1u);
    return 0;
  };

  // DQ_FREQ_DEBUG=2: workgroup 0 stamps each tile's phases (wall clock, after the barriers)
  auto mark = [&](int64_t t, int k) {
    if (a.dbg_clock && blockIdx.x == 0 && tid == 0 && t - t0 < 16)
      a.dbg_clock[(t - t0) * 8 + k] = wall_clock64();
  };
  __syncthreads();
  for (int64_t t = t0; t < t1; ++t) {
    mark(t, 0);
    const int64_t i0 = t * a.tile_items;
    const int64_t i1 = min(i0 + a.tile_items, a.n_items);
    const bool probe = ((t - t0) & 7) == 0;
    if (tid == 0) s_hits = 0;
    uint32_t keyed = 0, raw = 0;  // bit j: round j
    // 1. load + hash.  The row paths issue every round's loads before any value is used (one
    // memory latency per tile instead of one per round); records and multi-column keys loop.
    if constexpr (FROM_REC) {
#pragma unroll 1
      for (int j = 0; j < ROUNDS; ++j) {
        const int64_t i = i0 + (int64_t)j * kThreads + tid;
        const int q = j * kThreads + tid;
        if (i >= i1) continue;
        const RecIn r = a.rin[i];
        scnt[tid] = r.count;
        stash[q * W] = HASHED ? r.key : fmix_bij(r.key);
        if (HASHED) stash[q * W + 1] = a.var_arena_base + (uint64_t)seg_var_base(a.segs, i) + r.enc_off;
        if (r.count) keyed |= 1u << j;
      }
    } else if constexpr (!HASHED) {  // one fixed-width column
      // branch-free loads (an out-of-tile lane re-reads the tile's last row): a divergent branch
      // around a load makes the compiler wait for it before the join
      const KeyCol& c = a.ks.cols[0];
      int64_t ic[ROUNDS];
      uint32_t ok = 0;
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j) {
        const int64_t i = i0 + (int64_t)j * kThreads + tid;
        ok |= (i < i1 ? 1u : 0u) << j;
        ic[j] = i < i1 ? i : i1 - 1;
      }
      uint32_t vb = ~0u;
      if (c.valid) {
        uint32_t byte[ROUNDS];
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) byte[j] = c.valid[ic[j] >> 3];
        vb = 0;
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) vb |= ((byte[j] >> (ic[j] & 7)) & 1u) << j;
      }
      uint64_t v[ROUNDS];
      auto load_all = [&](auto type_tag) {
        constexpr int TY = decltype(type_tag)::value;
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) v[j] = kwiden(TY, c.values, ic[j]);
      };
      switch (c.type) {  // block-uniform: one unrolled load loop per width
        case DQ_INT8: load_all(std::integral_constant<int, DQ_INT8>{}); break;
        case DQ_INT16: load_all(std::integral_constant<int, DQ_INT16>{}); break;
        case DQ_INT32: load_all(std::integral_constant<int, DQ_INT32>{}); break;
        case DQ_FLOAT32: load_all(std::integral_constant<int, DQ_FLOAT32>{}); break;
        case DQ_FLOAT64: load_all(std::integral_constant<int, DQ_FLOAT64>{}); break;
        case DQ_BOOL: load_all(std::integral_constant<int, DQ_BOOL>{}); break;
        default: load_all(std::integral_constant<int, DQ_INT64>{}); break;
      }
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j) {
        if (!((ok >> j) & 1u)) continue;
        if ((vb >> j) & 1u) {
          keyed |= 1u << j;
          stash[(j * kThreads + tid) * W] = fmix_bij(exact_canon(a.ks, v[j]));
        } else {
          const unsigned long long ng = a.ks.null_as_group ? 1ULL : 0ULL;
          nullg += ng;
          nulls += 1ULL - ng;
        }
      }
    } else if constexpr (STR1) {  // one utf8 column: offsets, then <= 16 bytes per row, then hash
      const KeyCol& c = a.ks.cols[0];
      const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
      int64_t ic[ROUNDS];
      uint32_t ok = 0;
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j) {
        const int64_t i = i0 + (int64_t)j * kThreads + tid;
        ok |= (i < i1 ? 1u : 0u) << j;
        ic[j] = i < i1 ? i : i1 - 1;
      }
      int32_t s0[ROUNDS], len[ROUNDS];
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j) {
        s0[j] = off[ic[j]];
        len[j] = off[ic[j] + 1];
      }
      uint32_t byte[ROUNDS];  // validity bytes, in flight with the offsets
      if (c.valid) {
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) byte[j] = c.valid[ic[j] >> 3];
      }
      // <= 16 bytes per row as aligned dwords: dword k is read at min(k, last) so every read
      // holds a byte of the string (no read reaches a page the string does not lie on); rows
      // that are NULL, empty or longer read the first offset instead (always mapped)
      uint32_t d[ROUNDS][5];
      int sh[ROUNDS];
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j) {
        len[j] -= s0[j];
        // (Arrow keeps a NULL slot's offsets monotonic, so its range is inside the buffer too)
        const bool reg = len[j] > 0 && len[j] <= 16;
        const uint8_t* p = reg ? c.data + s0[j] : reinterpret_cast<const uint8_t*>(off);
        const uint32_t* q =
            reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
        sh[j] = (int)(reinterpret_cast<uintptr_t>(p) & 3u);
        const int last = reg ? ((sh[j] + len[j] + 3) >> 2) - 1 : 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) d[j][k] = q[k < last ? k : last];
      }
      uint32_t vb = ~0u;
      if (c.valid) {
        vb = 0;
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) vb |= ((byte[j] >> (ic[j] & 7)) & 1u) << j;
      }
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j) {
        if (!((ok >> j) & 1u)) continue;
        const int64_t i = ic[j];
        const int q = j * kThreads + tid;
        uint64_t h, k0 = 0, k1 = kNoShort;
        if ((vb >> j) & 1u) {
          if (len[j] <= 16) {
            uint64_t w0, w1;
            str16_from_dwords(d[j], sh[j], len[j], w0, w1);
            h = str_row_hash_reg(w0, w1, len[j]);
            str_short_key_reg(w0, w1, len[j], k0, k1);
          } else {
            h = fmix_bij(fold_col_hash(kRowHashSeed, str_hash_long_dev(c.data + s0[j], len[j], 0)));
          }
          // a key without a short form carries its offset and length instead (k0 is only read
          // beside a short k1), so its arena copy needs no second read of the offsets
          if (k1 == kNoShort) k0 = ((uint64_t)(uint32_t)len[j] << 32) | (uint32_t)s0[j];
        } else {
          // a NULL row.  Histogram: the NULL rows are one group kept apart (C_NULL_GROUP), so
          // this table also serves the column's grouping; the caller folds it into the
          // "NullValue" string group (Histogram.scala:59-66) with the literal's count from phase
          // C (dq_freq_null_literal).  (Counted without a branch: selecting between the two
          // counters made the compiler address them in scratch.)
          const unsigned long long ng = a.ks.null_as_group ? 1ULL : 0ULL;
          nullg += ng;
          nulls += 1ULL - ng;
          continue;
        }
        keyed |= 1u << j;
        stash[q * W] = h;
        stash[q * W + 1] = (uint64_t)i;
        if constexpr (SK) {
          ssk0[q] = k0;
          ssk1[q] = k1;
        }
      }
    } else if (str2) {  // two utf8 columns: two rounds' loads in flight at a time, then hash
      constexpr int G = 2;  // (rounds per group: four held 64 more VGPRs and spilled)
#pragma unroll 1
      for (int j0 = 0; j0 < ROUNDS; j0 += G) {
        Str2Row x[G];
        uint32_t byte[2][G];
        int64_t ic[G];
        uint32_t ok = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int64_t i = i0 + (int64_t)(j0 + g) * kThreads + tid;
          ok |= (i < i1 ? 1u : 0u) << g;
          ic[g] = i < i1 ? i : i1 - 1;
          str2_offsets(a.ks, ic[g], x[g]);
#pragma unroll
          for (int c = 0; c < 2; ++c) byte[c][g] = a.ks.cols[c].valid ? a.ks.cols[c].valid[ic[g] >> 3] : 0xffu;
        }
#pragma unroll
        for (int g = 0; g < G; ++g) str2_bytes(a.ks, x[g]);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if (!((ok >> g) & 1u)) continue;
          const bool valid = ((byte[0][g] & byte[1][g]) >> (ic[g] & 7)) & 1u;
          if (!valid) {  // a NULL key: the row is skipped (row_kind)
            ++nulls;
            continue;
          }
          const int j = j0 + g, q = j * kThreads + tid;
          uint64_t k0, k1;
          keyed |= 1u << j;
          stash[q * W] = str2_hash(a.ks, x[g], k0, k1);
          stash[q * W + 1] = (uint64_t)ic[g];
          if constexpr (SK) {
            ssk0[q] = k0;
            ssk1[q] = k1;
          }
        }
      }
    } else {  // several key columns
#pragma unroll 1
      for (int j = 0; j < ROUNDS; ++j) {
        const int64_t i = i0 + (int64_t)j * kThreads + tid;
        const int q = j * kThreads + tid;
        if (i >= i1) continue;
        const int kind = row_kind(a.ks, i, false);
        if (kind == ROW_SKIP) {
          ++nulls;
        } else {
          keyed |= 1u << j;
          stash[q * W] = row_hash_hashed_dw(a.ks, i);
          stash[q * W + 1] = (uint64_t)i;  // the row until it is encoded
          if constexpr (SK) multi_short_key(a.ks, i, ssk0[q], ssk1[q]);
        }
      }
    }
    __syncthreads();
    mark(t, 1);
    // 2. dedupe (round 0 of a probing tile measures the hit rate).  A hashed key whose slot is
    // claimed but not yet published by its claimer (another lane or wave) is retried after a
    // block barrier -- never a spin, lanes of one wave would wait on each other -- once per tile
    // (and right after round 0 when probing), so the rounds themselves run barrier-free.
    uint32_t wait = 0;  // bit j: round j must retry
    auto count_raw = [&](int j, uint64_t h, uint64_t c) {
      raw |= 1u << j;
      const uint32_t b = bucket_of(h);
      for_digits(c, [&](uint32_t) { atomicAdd(&bh[b], 1u); });
    };
    auto retry = [&](uint32_t rounds_mask, uint32_t& hits) {
      if constexpr (HASHED) {
        uint32_t w = wait & rounds_mask;
        while (__syncthreads_or(w ? 1 : 0)) {
#pragma unroll 1
          for (int j = 0; j < ROUNDS; ++j) {
            if (!((w >> j) & 1u)) continue;
            const int q = j * kThreads + tid;
            const uint64_t h = stash[q * W], rep = stash[q * W + 1];
            const uint64_t c = FROM_REC ? scnt[tid] : 1;
            const int res = dedupe(h, c, rep, SK ? ssk0[q] : 0, SK ? ssk1[q] : kNoShort);
            if (res == 3) continue;
            w &= ~(1u << j);
            if (res == 2) ++hits;
            if (!res) count_raw(j, h, c);
          }
        }
        wait &= ~rounds_mask;
      }
    };
    // One-string-column keys: a batched first probe of every round's home slot, with all rounds'
    // LDS reads in flight together (two LDS round trips for the thread's rows instead of two per
    // row in sequence), counts the rows whose short key already sits in its home slot -- nearly
    // every row of a low-cardinality column; the rest take the full dedupe below.  (Not on
    // probing tiles, whose round 0 decides the bypass for the rest.)
    uint32_t fast = 0;  // bit j: round j was counted here
    if constexpr (STR1) {
      if (!probe && !s_bypass) {
        uint64_t hk[ROUNDS], kk[ROUNDS], b1[ROUNDS], b0[ROUNDS], k0v[ROUNDS], k1v[ROUNDS];
        uint32_t sl[ROUNDS];
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) {
          const int q = j * kThreads + tid;
          hk[j] = stash[q * W];
          sl[j] = (uint32_t)(hk[j] >> 20) & (D - 1);
          kk[j] = lds_load(&dkey[sl[j]]);
          b1[j] = lds_load(&dsk1[sl[j]]);
          k0v[j] = ssk0[q];
          k1v[j] = ssk1[q];
        }
        // dsk1 is written (released) after dsk0: a final dsk1 read before this fence makes the
        // dsk0 read after it final too
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) b0[j] = lds_load(&dsk0[sl[j]]);
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) {
          const bool hit = ((keyed >> j) & 1u) && hk[j] != kEmptyKey && kk[j] == hk[j] &&
                           k1v[j] != kNoShort && b1[j] == k1v[j] && b0[j] == k0v[j];
          if (hit) {
            atomicAdd((unsigned long long*)&dcnt[sl[j]], 1ULL);
            fast |= 1u << j;
          }
        }
      }
    }
#pragma unroll 1
    for (int j = 0; j < ROUNDS; ++j) {
      const int q = j * kThreads + tid;
      const bool on = probe && j == 0 ? true : !s_bypass;
      uint32_t hits = 0;
      int res = -1;
      if (((keyed & ~fast) >> j) & 1u) {
        const uint64_t h = stash[q * W];
        const uint64_t rep = HASHED ? stash[q * W + 1] : 0;
        const uint64_t c = FROM_REC ? scnt[tid] : 1;
        res = on ? dedupe(h, c, rep, SK ? ssk0[q] : 0, SK ? ssk1[q] : kNoShort) : 0;
        if (res == 3) wait |= 1u << j;
        else if (res == 2) ++hits;
        else if (!res) count_raw(j, h, c);
      }

      if (probe && j == 0) {
        retry(1u, hits);
        const uint32_t wh = wave_sum(hits);  // every lane: the shuffles need the whole wave
        if (__lane_id() == 0 && wh) atomicAdd(&s_hits, wh);
        __syncthreads();
        if (tid == 0) s_bypass = s_hits * 16u < (uint32_t)kThreads ? 1u : 0u;
        __syncthreads();
        if (tid == 0) dbg_bypass += s_bypass;
      }
    }
    {
      uint32_t hits = 0;
      retry(~0u, hits);
    }
    const bool any_raw = __syncthreads_or(raw ? 1 : 0);
    mark(t, 2);
    if (!any_raw) {  // every row collapsed into the dedupe table: an empty chunk, no sort
      uint16_t* hrow = a.hist + t * kHistRow;
      if (!pieces)
        for (int i = tid; i < kHistRow; i += kThreads) hrow[i] = 0;
      mark(t, 3);
      mark(t, 4);
      continue;
    }
    uint64_t need = 0;
    // two utf8 columns: every raw round's offsets loaded together, then the bytes needed
    auto str2_raw_offsets = [&](Str2Row (&x)[ROUNDS]) {
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j)
        str2_offsets(a.ks, (raw >> j) & 1u ? (int64_t)stash[(j * kThreads + tid) * W + 1] : i0, x[j]);
    };
    if (HASHED && !FROM_REC && !STR1 && str2) {
      Str2Row x[ROUNDS];
      str2_raw_offsets(x);
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j)
        need += (raw >> j) & 1u ? 16u + pad4((uint32_t)(x[j].len[0] - x[j].s0[0])) +
                                      pad4((uint32_t)(x[j].len[1] - x[j].s0[1]))
                                : 0u;
    } else if constexpr (HASHED && !FROM_REC && !STR1) {  // (STR1 reserved its arena up front)
#pragma unroll 1
      for (int j = 0; j < ROUNDS; ++j)
        if ((raw >> j) & 1u) {
          const int q = j * kThreads + tid;
          const int64_t row = (int64_t)stash[q * W + 1];
          need += enc_size_sk(row, SK ? ssk1[q] : kNoShort);
        }
    }
    // 3. counting sort of the raw rows into the tile's chunk
    if constexpr (XP) {
      if (pieces) {
        // ... or, bucket pieces: sorted in LDS by bucket, then written to each bucket's next
        // slots in the batch region (runs of ~16 records per bucket and tile, each continuing
        // the workgroup's piece of that bucket)
        __syncthreads();
        uint32_t ctotal;
        const uint32_t cnt = tid < kBuckets ? bh[tid] : 0u;
        const uint32_t ex = block_excl_scan(cnt, s_wave, ctotal);
        if (tid < kBuckets) bcur[tid] = ex;
        __syncthreads();
        mark(t, 3);
        uint32_t pv[ROUNDS];
        uint64_t hv[ROUNDS];
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) {
          if (!((raw >> j) & 1u)) continue;
          hv[j] = stash[j * kThreads + tid];
          pv[j] = atomicAdd(&bcur[bucket_of(hv[j])], 1u);
        }
        __syncthreads();
        if (tid < kBuckets) {  // bcur: the bucket's region slot minus its first sorted position
          const uint32_t c = bh[tid], st = bcur[tid] - c;
          bcur[tid] = wcur[tid] - st;
          wcur[tid] += c;
        }
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j)
          if ((raw >> j) & 1u) stash[pv[j]] = hv[j];
        __syncthreads();
        uint64_t* out = reinterpret_cast<uint64_t*>(a.recs);
        for (uint32_t i = tid; i < ctotal; i += kThreads) {
          const uint64_t hh = stash[i];
          out[(uint32_t)(bcur[bucket_of(hh)] + i)] = (hh << 8) | 1u;  // the count-1 digit code
        }
        end_chunk();
        mark(t, 4);
        continue;
      }
    }
    uint32_t ctotal = 0;
    if (STR1 && hpieces) begin_tile_pieces(t);
    else ctotal = begin_chunk(t, need);
    mark(t, 3);
    if constexpr (!HASHED && !FROM_REC) {
      // exact rows (count 1: one record each): sorted in LDS over the stash, then written out as
      // one contiguous 16-byte-store stream (scattered 8-byte global stores were ~half the tile)
      uint64_t rv[ROUNDS];
      uint32_t pv[ROUNDS];
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j) {
        if (!((raw >> j) & 1u)) continue;
        const uint64_t h = stash[j * kThreads + tid];
        pv[j] = atomicAdd(&bcur[bucket_of(h)], 1u);
        rv[j] = (h << 8) | 1u;  // the count-1 digit code (for_digits(1))
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j)
        if ((raw >> j) & 1u) stash[pv[j]] = rv[j];
      __syncthreads();
      uint64_t* out = reinterpret_cast<uint64_t*>(a.recs) + t * (int64_t)T;
      const uint32_t pairs = ctotal >> 1;
      for (uint32_t i = tid; i < pairs; i += kThreads) {
        const ulonglong2 v = make_ulonglong2(stash[2 * i], stash[2 * i + 1]);
        reinterpret_cast<ulonglong2*>(out)[i] = v;
      }
      if ((ctotal & 1u) && tid == 0) out[ctotal - 1] = stash[ctotal - 1];
    } else if (HASHED && !FROM_REC && !STR1 && str2) {
      // two utf8 columns: each round's arena bytes (one LDS atomic per wave and round) and
      // encodings
      constexpr int G = 2;  // rounds whose values are in flight together (again: L2 hits)
#pragma unroll 1
      for (int j0 = 0; j0 < ROUNDS; j0 += G) {
        Str2Row x[G];
#pragma unroll
        for (int g = 0; g < G; ++g)
          str2_offsets(a.ks, (raw >> (j0 + g)) & 1u ? (int64_t)stash[((j0 + g) * kThreads + tid) * W + 1] : i0,
                       x[g]);
#pragma unroll
        for (int g = 0; g < G; ++g) str2_bytes(a.ks, x[g]);
#pragma unroll
        for (int g = 0; g < G; ++g) {  // (wave-uniform trip count)
          const int j = j0 + g;
          const bool on = (raw >> j) & 1u;
          const int q = j * kThreads + tid;
          const uint32_t sz = on ? str2_enc_size(x[g]) : 0u;
          const uint32_t incl = __ockl_wfscan_add_u32(sz, true);
          const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
          unsigned long long wbase = 0;
          if (__lane_id() == 63 && wtot) wbase = atomicAdd(&s_arena_cur, (unsigned long long)wtot);
          wbase = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(wbase >> 32), 63) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)wbase, 63);
          if (!on) continue;
          const uint64_t off = s_arena_base + wbase + (incl - sz);
          if (!DQ_A_NOCOPY) str2_encode(a.ks, x[g], reinterpret_cast<uint32_t*>(a.arena + off));
          put(t, stash[q * W], 1u, off);
        }
      }
    } else if constexpr (HASHED && !FROM_REC) {
      // row keys into the arena: each wave reserves its round's bytes with one LDS atomic (a
      // per-row atomic on the one cursor word serialised every row of the tile)
#pragma unroll 1
      for (int j = 0; j < ROUNDS; ++j) {  // (wave-uniform trip count)
        const bool on = (raw >> j) & 1u;
        const int q = j * kThreads + tid;
        const int64_t row = on ? (int64_t)stash[q * W + 1] : 0;
        const uint64_t k0 = SK && on ? ssk0[q] : 0, k1 = SK && on ? ssk1[q] : kNoShort;
        // (STR1: a long key's offset and length from k0)
        uint32_t sz = !on ? 0u : STR1 && k1 == kNoShort ? 8u + pad4((uint32_t)(k0 >> 32)) : enc_size_sk(row, k1);
        if constexpr (STR1) sz = (sz + 15u) & ~15u;  // 16-byte aligned keys: vector stores
        const uint32_t incl = __ockl_wfscan_add_u32(sz, true);
        const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        unsigned long long wbase = 0;
        if (__lane_id() == 63 && wtot) wbase = atomicAdd(&s_arena_cur, (unsigned long long)wtot);
        wbase = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(wbase >> 32), 63) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)wbase, 63);
        if (!on) continue;
        const uint64_t off = s_arena_base + wbase + (incl - sz);
        if constexpr (STR1) {
          if (k1 != kNoShort) {
            if (!DQ_A_NOCOPY) str1_encode_short16(k0, k1, reinterpret_cast<uint32_t*>(a.arena + off));
          } else {
            if (!DQ_A_NOCOPY) str1_encode_copy16(a.ks.cols[0].data + (uint32_t)k0, (int32_t)(k0 >> 32),
                               reinterpret_cast<uint32_t*>(a.arena + off));
          }
        } else {
          if (!DQ_A_NOCOPY) row_encode_dw(a.ks, row, reinterpret_cast<uint32_t*>(a.arena + off));
        }
        if (STR1 && hpieces) put_pieces(t, stash[q * W], 1u, off);
        else put(t, stash[q * W], 1u, off);  // (row keys: one record, the count-1 digit code)
      }
    } else {
#pragma unroll 1
      for (int j = 0; j < ROUNDS; ++j) {
        if (!((raw >> j) & 1u)) continue;
        const int q = j * kThreads + tid;
        const uint64_t h = stash[q * W];
        uint64_t rep = HASHED ? stash[q * W + 1] : 0;
        if constexpr (FROM_REC) maxcnt = scnt[tid] > maxcnt ? scnt[tid] : maxcnt;
        for_digits(FROM_REC ? scnt[tid] : 1, [&](uint32_t code) { put(t, h, code, rep); });
      }
    }
    end_chunk();
    mark(t, 4);
  }
  if constexpr (XP) {
    if (pieces) {  // the collapsed groups into their buckets' pieces, then the pieces' lengths
      uint64_t* out = reinterpret_cast<uint64_t*>(a.recs);
      __syncthreads();
      for (int sl = tid; sl < D; sl += kThreads) {
        const uint64_t k = dkey[sl];
        if (k == kEmptyKey) continue;
        const uint32_t b = bucket_of(k);
        maxcnt = dcnt[sl] > maxcnt ? dcnt[sl] : maxcnt;
        for_digits(dcnt[sl], [&](uint32_t code) { out[atomicAdd(&wcur[b], 1u)] = (k << 8) | code; });
      }
      wave_max_lds(&s_maxcnt, maxcnt);
      __syncthreads();
      if (tid == 0 && s_maxcnt) atomicMax(&a.counters[C_MAXCNT], s_maxcnt);
      if (tid < kBuckets)
        a.plen[(int64_t)blockIdx.x * kBuckets + tid] =
            wcur[tid] - a.pstart[(int64_t)blockIdx.x * kBuckets + tid];
      wave_count(&a.counters[C_NULL_ROWS], nulls);
      wave_count(&a.counters[C_NULL_GROUP], nullg);
      __syncthreads();
      if (tid < 3 && s_dbg[tid]) atomicAdd(&a.counters[C_DBG_NOTREADY + tid], (unsigned long long)s_dbg[tid]);
      wave_count(&a.counters[C_DBG_BYPASS], dbg_bypass);
      return;
    }
  }
  // the collapsed groups of the whole range -> this workgroup's own chunk
  uint64_t need = 0;
  for (int sl = tid; sl < D; sl += kThreads) {
    const uint64_t k = dkey[sl];
    if (k == kEmptyKey) continue;
    const uint32_t b = bucket_of(k);
    for_digits(dcnt[sl], [&](uint32_t) { atomicAdd(&bh[b], 1u); });
    if constexpr (HASHED && !FROM_REC) need += enc_size_sk((int64_t)drep[sl], SK ? dsk1[sl] : kNoShort);
  }
  const int64_t fchunk = n_tiles + blockIdx.x;
  begin_chunk(fchunk, need);
  for (int sl = tid; sl < D; sl += kThreads) {
    const uint64_t k = dkey[sl];
    if (k == kEmptyKey) continue;
    uint64_t rep = HASHED ? drep[sl] : 0;
    if constexpr (HASHED && !FROM_REC)
      rep = arena_rep_sk((int64_t)rep, SK ? dsk0[sl] : 0, SK ? dsk1[sl] : kNoShort);
    maxcnt = dcnt[sl] > maxcnt ? dcnt[sl] : maxcnt;
    for_digits(dcnt[sl], [&](uint32_t code) { put(fchunk, k, code, rep); });
  }
  wave_max_lds(&s_maxcnt, maxcnt);
  if (!FROM_REC) {
    wave_count(&a.counters[C_NULL_ROWS], nulls);
    wave_count(&a.counters[C_NULL_GROUP], nullg);
  }
  if constexpr (STR1)
    if (hpieces && tid < kBuckets) {  // this workgroup's pieces: their starts and fills
      const int64_t r = (int64_t)blockIdx.x * kBuckets + tid;
      a.pstart[r] = (uint32_t)(a.piece_base + (uint64_t)r * a.piece_cap);
      a.plen[r] = wfill[tid];
    }
  __syncthreads();
  if (tid == 0 && s_maxcnt) atomicMax(&a.counters[C_MAXCNT], s_maxcnt);
  if (tid < 3 && s_dbg[tid]) atomicAdd(&a.counters[C_DBG_NOTREADY + tid], (unsigned long long)s_dbg[tid]);
  wave_count(&a.counters[C_DBG_BYPASS], dbg_bypass);
}

// ------------------------------------------------------------------------------------------------
// Phase A0, exact rows: the rows of each phase-A workgroup per bucket, so that phase A can write
// the batch bucket-major (bucket b of the batch is one contiguous region when no rows collapse in
// the dedupe table, and phase B then reads whole buckets as streams instead of gathering 128-byte
// chunk segments).  Same tile ranges and the same hash as freq_phaseA<false, false>; only
// non-NULL rows are keyed.
// ------------------------------------------------------------------------------------------------
// row base + r of a fixed-width column, the base (wave-uniform) applied to the pointer
template <int TY>
DQ_DEV uint64_t kload_at(const void* v, int64_t base, int r) {
  if constexpr (TY == DQ_BOOL) {
    return kwiden(TY, v, base + r);
  } else {
    constexpr int W = TY == DQ_INT8 ? 1 : TY == DQ_INT16 ? 2 : (TY == DQ_INT32 || TY == DQ_FLOAT32) ? 4 : 8;
    return kwiden(TY, reinterpret_cast<const char*>(v) + base * W, r);
  }
}
constexpr int kPreThreads = 1024;
constexpr uint64_t kDenseSign = 1ULL << 63;
// DENSE: also the batch's key range for the dense path (a second instantiation: the range's
// registers cost the plain pre-pass a wave per SIMD)
template <bool DENSE>
__global__ void __launch_bounds__(kPreThreads) freq_prepass_x(AArgs a, uint32_t* ph) {
  constexpr int ROUNDS = FM<false>::kTile / kPreThreads;
  __shared__ uint32_t bh[kBuckets];
  const int tid = threadIdx.x;
  for (int i = tid; i < kBuckets; i += kPreThreads) bh[i] = 0;
  __syncthreads();
  const KeyCol& c = a.ks.cols[0];
  const int64_t n_tiles = (a.n_items + a.tile_items - 1) / a.tile_items;
  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t t1 = min(t0 + (int64_t)a.tiles_per_wg, n_tiles);
  const bool full_ok = (reinterpret_cast<uintptr_t>(c.valid) & 7u) == 0 && (a.tile_items & 63) == 0;
  uint64_t umax = 0, umin = ~0ULL;  // the keyed values' range, sign-flipped (dense path)
  auto tile_loop = [&](auto type_tag) {
    constexpr int TY = decltype(type_tag)::value;
    for (int64_t t = t0; t < t1; ++t) {
      const int64_t i0 = t * a.tile_items, i1 = min(i0 + a.tile_items, a.n_items);
      uint32_t ok = 0, vb = ~0u;
      uint64_t v[ROUNDS];
      if (i1 - i0 == FM<false>::kTile && full_ok) {  // as freq_phaseA_xp's full tiles
        ok = (1u << ROUNDS) - 1u;
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) v[j] = kload_at<TY>(c.values, i0 + (int64_t)j * kPreThreads, tid);
        if (c.valid) {
          const int64_t wrow = i0 + 64 * (int64_t)__builtin_amdgcn_readfirstlane(tid >> 6);
          vb = 0;
#pragma unroll
          for (int j = 0; j < ROUNDS; ++j) {
            const uint64_t w =
                *reinterpret_cast<const uint64_t*>(c.valid + ((wrow + (int64_t)j * kPreThreads) >> 3));
            vb |= (uint32_t)((w >> __lane_id()) & 1u) << j;
          }
        }
      } else {
        int64_t ic[ROUNDS];
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) {
          const int64_t i = i0 + (int64_t)j * kPreThreads + tid;
          ok |= (i < i1 ? 1u : 0u) << j;
          ic[j] = i < i1 ? i : i1 - 1;
        }
        if (c.valid) {
          uint32_t byte[ROUNDS];
#pragma unroll
          for (int j = 0; j < ROUNDS; ++j) byte[j] = c.valid[ic[j] >> 3];
          vb = 0;
#pragma unroll
          for (int j = 0; j < ROUNDS; ++j) vb |= ((byte[j] >> (ic[j] & 7)) & 1u) << j;
        }
#pragma unroll
        for (int j = 0; j < ROUNDS; ++j) v[j] = kwiden(TY, c.values, ic[j]);
      }
#pragma unroll
      for (int j = 0; j < ROUNDS; ++j)
        if ((ok & vb) >> j & 1u) {
          atomicAdd(&bh[bucket_of(fmix_bij(exact_canon(a.ks, v[j])))], 1u);
          if constexpr (DENSE) {
            const uint64_t u = v[j] ^ kDenseSign;  // (integer keys: the widened value)
            umax = u > umax ? u : umax;
            umin = u < umin ? u : umin;
          }
        }
    }
  };
  switch (c.type) {  // block-uniform: one unrolled load loop per width
    case DQ_INT8: tile_loop(std::integral_constant<int, DQ_INT8>{}); break;
    case DQ_INT16: tile_loop(std::integral_constant<int, DQ_INT16>{}); break;
    case DQ_INT32: tile_loop(std::integral_constant<int, DQ_INT32>{}); break;
    case DQ_FLOAT32: tile_loop(std::integral_constant<int, DQ_FLOAT32>{}); break;
    case DQ_FLOAT64: tile_loop(std::integral_constant<int, DQ_FLOAT64>{}); break;
    case DQ_BOOL: tile_loop(std::integral_constant<int, DQ_BOOL>{}); break;
    default: tile_loop(std::integral_constant<int, DQ_INT64>{}); break;
  }
  // the batch's key range for the dense path: waves -> LDS -> one global atomic per workgroup
  // (per wave, ~15 K same-address atomics per batch serialised in L2: +40 % on this kernel)
  __shared__ unsigned long long s_mm[2];
  if (DENSE) {
    if (tid < 2) s_mm[tid] = 0;
    __syncthreads();
    umax = __ockl_wfred_max_u64(umax);
    umin = ~__ockl_wfred_max_u64(~umin);
    if (__lane_id() == 0 && umin <= umax) {  // (a wave without keyed rows: umin > umax)
      atomicMax(&s_mm[0], (unsigned long long)umax);
      atomicMax(&s_mm[1], (unsigned long long)~umin);
    }
  }
  __syncthreads();
  if (DENSE && tid == 0 && s_mm[0] | s_mm[1]) {
    atomicMax(&a.dense_words[0], s_mm[0]);
    atomicMax(&a.dense_words[1], s_mm[1]);
  }
  for (int i = tid; i < kBuckets; i += kPreThreads) ph[(int64_t)blockIdx.x * kBuckets + i] = bh[i];
}

// ------------------------------------------------------------------------------------------------
// Phase A, exact rows into bucket pieces (the pieces layout of freq_phaseA<false, false> with
// a.pstart set; same tile ranges, dedupe table and bypass probing, same records).  A lean kernel
// of its own: 512 threads x 16 rounds per 8192-row tile and ~80 KB of LDS, so TWO workgroups
// share a CU and one's loads overlap the other's sort and stores (the generic kernel, 1024 threads
// at 128 VGPRs with spills, ran one workgroup per CU with every phase behind a barrier).  The
// bucket-counting atomic returns the row's rank in its bucket, so the counting sort takes one LDS
// atomic per row instead of two.
// ------------------------------------------------------------------------------------------------
// p[lo, hi) = 0 by the block's threads: 16-byte stores over the aligned middle (the tile rows of
// a small-key workgroup are ~46 KB of u16, zeroed 2 bytes a store before)
DQ_DEV void zero_u16(uint16_t* p, int64_t lo, int64_t hi, int tid, int nt) {
  if (lo >= hi) return;
  const int64_t a0 = min(hi, (lo + 7) & ~(int64_t)7), a1 = max(a0, hi & ~(int64_t)7);
  for (int64_t i = lo + tid; i < a0; i += nt) p[i] = 0;
  for (int64_t i = a0 / 8 + tid; i < a1 / 8; i += nt) reinterpret_cast<uint4*>(p)[i] = make_uint4(0, 0, 0, 0);
  for (int64_t i = a1 + tid; i < hi; i += nt) p[i] = 0;
}

constexpr int kAXThreads = 512;

template <int TY>
__global__ void __launch_bounds__(kAXThreads, 4) freq_phaseA_xp(AArgs a) {  // 4 waves per SIMD: two workgroups per CU
  constexpr int T = FM<false>::kTile, R = T / kAXThreads, D = AKeys<false, false>::kDedupe;
  static_assert(R <= 32, "round bits");
  __shared__ uint32_t bh[kBuckets];     // counts of the tile's raw rows, then their sorted starts
  __shared__ uint32_t gdel[kBuckets];   // region slot of a sorted position, minus that position
  __shared__ uint32_t wcur[kBuckets];   // each bucket's next region slot (the workgroup's piece)
  // fixed-capacity pieces (a.piece_cap > 0): the chunk slot of a sorted position past the piece's
  // room, minus that position
  __shared__ uint32_t odel[kBuckets];
  __shared__ unsigned long long dkey[D];
  __shared__ uint32_t dcnt[D];          // (a workgroup's rows: < 2^32)
  __shared__ uint64_t stash[T];
  __shared__ uint32_t s_wave[kAXThreads / 64];
  __shared__ uint32_t s_hits, s_bypass, s_full;
  __shared__ unsigned long long s_maxcnt;
  const int tid = threadIdx.x;
  if (a.zero_rows) {  // this workgroup's share of the piece chunks' hist rows
    const int64_t tot = a.zero_rows * kHistRow, per = (tot + gridDim.x - 1) / gridDim.x;
    const int64_t lo = a.zero_off * kHistRow + (int64_t)blockIdx.x * per;
    zero_u16(a.hist, lo, min(lo + per, (a.zero_off + a.zero_rows) * kHistRow), tid, kAXThreads);
  }
  if (a.dense_words && __hip_atomic_load(&a.dense_words[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                           a.dense_epoch) {  // the dense path took the batch: empty pieces
    a.pstart[(int64_t)blockIdx.x * kBuckets + tid] = 0;
    a.plen[(int64_t)blockIdx.x * kBuckets + tid] = 0;
    return;
  }
  const KeyCol& c = a.ks.cols[0];
  const int64_t n_tiles = (a.n_items + a.tile_items - 1) / a.tile_items;
  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t t1 = min(t0 + (int64_t)a.tiles_per_wg, n_tiles);
  for (int i = tid; i < D; i += kAXThreads) {
    dkey[i] = kEmptyKey;
    dcnt[i] = 0;
  }
  const uint32_t cap = a.piece_cap;  // 0: pieces laid out by the pre-pass's counts
  {
    uint32_t st;
    if (cap) {  // piece (w, b) at piece_base + (w kBuckets + b) cap; wcur = its fill
      st = (uint32_t)(a.piece_base + ((uint64_t)blockIdx.x * kBuckets + tid) * cap);
      wcur[tid] = 0;
    } else {
      uint32_t all;
      const uint32_t bb = block_excl_scan(a.ptot[tid], s_wave, all);  // (kAXThreads == kBuckets)
      st = bb + a.ph[(int64_t)blockIdx.x * kBuckets + tid];
      wcur[tid] = st;
    }
    a.pstart[(int64_t)blockIdx.x * kBuckets + tid] = st;
    bh[tid] = 0;
    // the batch's chunk rows hold no records: empty histograms
    for (int64_t r = t0; r < t1; ++r)
      for (int i = tid; i < kHistRow; i += kAXThreads) a.hist[r * kHistRow + i] = 0;
    for (int i = tid; i < kHistRow; i += kAXThreads) a.hist[(n_tiles + blockIdx.x) * kHistRow + i] = 0;
  }
  if (tid == 0) {
    s_bypass = 0;
    s_full = 0;
    s_maxcnt = 0;
  }
  unsigned long long nulls = 0, nullg = 0, dbg_bypass = 0, nanf = 0;
  uint64_t* out = reinterpret_cast<uint64_t*>(a.recs);
  // the full-tile loads: 8-byte-aligned bitmap words, tiles on 64-row boundaries
  const bool full_ok = (reinterpret_cast<uintptr_t>(c.valid) & 7u) == 0 && (a.tile_items & 63) == 0;
  // 1 claimed, 2 added, 0 table full (the row stays raw)
  auto dedupe = [&](uint64_t h) -> int {
    uint32_t slot = (uint32_t)(h >> 20) & (D - 1);
    for (int pr = 0; pr < 4; ++pr) {
      unsigned long long k = lds_load(reinterpret_cast<const uint64_t*>(&dkey[slot]));
      if (k == kEmptyKey) {
        const unsigned long long prev = atomicCAS(&dkey[slot], kEmptyKey, (unsigned long long)h);
        if (prev == kEmptyKey) {
          atomicAdd(&dcnt[slot], 1u);
          return 1;
        }
        k = prev;
      }
      if (k == h) {
        atomicAdd(&dcnt[slot], 1u);
        return 2;
      }
      slot = (slot + 1) & (D - 1);
    }
    return 0;
  };
  __syncthreads();
  {
#pragma unroll 1
    for (int64_t t = t0; t < t1; ++t) {
      const int64_t i0 = t * a.tile_items, i1 = min(i0 + a.tile_items, a.n_items);
      const bool probe = ((t - t0) & 7) == 0;
      // 1. loads, then hash.  A full tile: each round's rows from a uniform base (one offset
      // register) and each wave's 64 validity bits as one scalar load of a bitmap word.  The last
      // tile: branch-free clamped loads (an out-of-tile lane re-reads the tile's last row).
      uint64_t h[R];
      uint32_t ok = 0, vb = ~0u;
      if (i1 - i0 == T && full_ok) {
        ok = (1u << R) - 1u;
#pragma unroll
        for (int j = 0; j < R; ++j) h[j] = kload_at<TY>(c.values, i0 + (int64_t)j * kAXThreads, tid);
        if (c.valid) {
          const int64_t wrow = i0 + 64 * (int64_t)__builtin_amdgcn_readfirstlane(tid >> 6);
          vb = 0;
#pragma unroll
          for (int j = 0; j < R; ++j) {
            const uint64_t w =
                *reinterpret_cast<const uint64_t*>(c.valid + ((wrow + (int64_t)j * kAXThreads) >> 3));
            vb |= (uint32_t)((w >> __lane_id()) & 1u) << j;
          }
        }
      } else {
        int64_t ic[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const int64_t i = i0 + (int64_t)j * kAXThreads + tid;
          ok |= (i < i1 ? 1u : 0u) << j;
          ic[j] = i < i1 ? i : i1 - 1;
        }
#pragma unroll
        for (int j = 0; j < R; ++j) h[j] = kwiden(TY, c.values, ic[j]);
        if (c.valid) {
          uint32_t byte[R];
#pragma unroll
          for (int j = 0; j < R; ++j) byte[j] = c.valid[ic[j] >> 3];
          vb = 0;
#pragma unroll
          for (int j = 0; j < R; ++j) vb |= ((byte[j] >> (ic[j] & 7)) & 1u) << j;
        }
      }
      const uint32_t keyed = ok & vb;
      {
        const unsigned long long nn = (unsigned long long)__builtin_popcount(ok & ~vb);
        const unsigned long long ng = a.ks.null_as_group ? nn : 0ULL;
        nullg += ng;
        nulls += nn - ng;
      }
      if constexpr (TY == DQ_FLOAT64 || TY == DQ_FLOAT32) {  // (Histogram mode folds NaN payloads)
#pragma unroll
        for (int j = 0; j < R; ++j)
          nanf += ((keyed >> j) & 1u) && exact_canon(a.ks, h[j]) != h[j] ? 1u : 0u;
      }
#pragma unroll
      for (int j = 0; j < R; ++j) h[j] = fmix_bij(exact_canon(a.ks, h[j]));
      // 2. dedupe: round 0 of a probing tile measures the hit rate, which decides the bypass
      uint32_t raw = keyed;
      if (probe) {
        if (tid == 0) s_hits = 0;
        __syncthreads();
        int res = -1;
        if (keyed & 1u) {
          res = dedupe(h[0]);
          if (res) raw &= ~1u;
          if (!res) atomicAdd(&s_full, 1u);
        }
        const uint32_t wh = (uint32_t)__builtin_popcountll(__ballot(res == 2));  // whole wave
        if (__lane_id() == 0 && wh) atomicAdd(&s_hits, wh);
        __syncthreads();
        if (tid == 0) s_bypass = s_hits * 16u < (uint32_t)kAXThreads ? 1u : 0u;
        __syncthreads();
        dbg_bypass += tid == 0 ? s_bypass : 0u;
      }
      if (!s_bypass) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          if (!((keyed >> j) & 1u) || (probe && j == 0)) continue;
          const int res = dedupe(h[j]);
          if (res) raw &= ~(1u << j);
          else atomicAdd(&s_full, 1u);
        }
      }
      if (!__syncthreads_or(raw ? 1 : 0)) continue;  // every row collapsed: nothing to write
#if DQ_AX_EXPERIMENT & 2  // (timing only: no counting sort -- the tile's records in row order)
      {
#pragma unroll
        for (int j = 0; j < R; ++j)
          if (!(DQ_AX_EXPERIMENT & 1) && ((raw >> j) & 1u))
            out[a.piece_base + (uint64_t)t * T + (uint64_t)(j * kAXThreads + tid)] = (h[j] << 8) | 1u;
        continue;
      }
#endif
      // 3. counting sort by bucket: the counting atomic gives each raw row its rank
      uint32_t rk[R];
#pragma unroll
      for (int j = 0; j < R; ++j)
        if ((raw >> j) & 1u) rk[j] = atomicAdd(&bh[bucket_of(h[j])], 1u);
      __syncthreads();
      uint32_t ctotal;
      const uint32_t cnt = bh[tid];
      const uint32_t ex = block_excl_scan(cnt, s_wave, ctotal);
      uint32_t lim = 0;  // (cap: sorted positions below ex + take go to the piece)
      if (cap) {  // the piece takes what fits; the rest goes to this tile's chunk, bucket-sorted
        const uint32_t take = min(cnt, cap - wcur[tid]), ovf = cnt - take;
        uint32_t otot;
        const uint32_t oex = block_excl_scan(ovf, s_wave, otot);
        gdel[tid] = (uint32_t)(a.piece_base + ((uint64_t)blockIdx.x * kBuckets + tid) * cap) + wcur[tid] - ex;
        odel[tid] = (uint32_t)(t * T) + oex - ex - take;
        if (otot) {  // (the tile's chunk row was emptied at the start)
          uint16_t* hrow = a.hist + t * kHistRow;
          hrow[tid] = (uint16_t)oex;
          if (tid == 0) hrow[kBuckets] = (uint16_t)otot;
        }
        wcur[tid] += take;
        lim = ex + take;
      } else {
        gdel[tid] = wcur[tid] - ex;
        wcur[tid] += cnt;
      }
      bh[tid] = ex;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < R; ++j)
        if ((raw >> j) & 1u) stash[bh[bucket_of(h[j])] + rk[j]] = h[j];
      __syncthreads();
      // 4. the sorted tile to each bucket's next slots: runs of ~16 records per bucket
      if (cap) {
        bh[tid] = lim;
        __syncthreads();
        auto put = [&](uint32_t i) {
          const uint64_t hh = stash[i];
          const uint32_t b = bucket_of(hh);
          if (!(DQ_AX_EXPERIMENT & 1))  // (timing builds: 1 = no record stores)
            out[(uint32_t)((i < bh[b] ? gdel[b] : odel[b]) + i)] = (hh << 8) | 1u;
        };
        // int64 keys: four records' LDS reads in flight per step (422 -> 414-419 us per configs[2]
        // batch, profiles/r6ak/); the other widths spill with it.  (Fully unrolled -- every
        // round's stash words, then destinations, then stores -- spilled at every batch size.)
        if constexpr (TY == DQ_INT64) {
#pragma unroll 4
          for (uint32_t i = tid; i < ctotal; i += kAXThreads) put(i);
        } else {
          for (uint32_t i = tid; i < ctotal; i += kAXThreads) put(i);
        }
      } else {
        for (uint32_t i = tid; i < ctotal; i += kAXThreads) {
          const uint64_t hh = stash[i];
          out[(uint32_t)(gdel[bucket_of(hh)] + i)] = (hh << 8) | 1u;  // the count-1 digit code
        }
      }
      __syncthreads();
      bh[tid] = 0;  // (visible after the next tile's barriers)
    }
  }
  // the collapsed groups into their buckets' pieces, then the pieces' lengths
  __syncthreads();
  uint64_t maxcnt = 1;
  if (cap) {  // (one dedupe slot per thread) the digits that fit the piece, the rest bucket-sorted
              // into this workgroup's chunk
    static_assert(D == kAXThreads, "one dedupe slot per thread");
    odel[tid] = 0;
    __syncthreads();
    const uint64_t k = dkey[tid];
    const uint32_t c = k == kEmptyKey ? 0u : dcnt[tid], b = k == kEmptyKey ? 0u : bucket_of(k);
    uint32_t nd = 0;
    for (uint32_t x = c; x; x >>= 2) nd += (x & 3) ? 1u : 0u;
    const uint32_t s0 = nd ? atomicAdd(&wcur[b], nd) : 0u;
    const uint32_t np = s0 < cap ? min(nd, cap - s0) : 0u;
    const uint32_t o = nd > np ? atomicAdd(&odel[b], nd - np) : 0u;
    maxcnt = c > maxcnt ? c : maxcnt;
    __syncthreads();
    uint32_t otot;
    const uint32_t oex = block_excl_scan(odel[tid], s_wave, otot);
    const int64_t wchunk = n_tiles + blockIdx.x;
    if (otot) {
      uint16_t* hrow = a.hist + wchunk * kHistRow;
      hrow[tid] = (uint16_t)oex;
      if (tid == 0) hrow[kBuckets] = (uint16_t)otot;
    }
    gdel[tid] = oex;
    __syncthreads();
    const uint64_t pb = a.piece_base + ((uint64_t)blockIdx.x * kBuckets + b) * cap;
    uint32_t d = 0;
    for_digits(c, [&](uint32_t code) {
      const uint64_t slot = d < np ? pb + s0 + d : (uint64_t)wchunk * T + gdel[b] + o + (d - np);
      out[slot] = (k << 8) | code;
      ++d;
    });
  } else {
    for (int sl = tid; sl < D; sl += kAXThreads) {
      const uint64_t k = dkey[sl];
      if (k == kEmptyKey) continue;
      const uint32_t b = bucket_of(k);
      maxcnt = dcnt[sl] > maxcnt ? dcnt[sl] : maxcnt;
      for_digits(dcnt[sl], [&](uint32_t code) { out[atomicAdd(&wcur[b], 1u)] = (k << 8) | code; });
    }
  }
  wave_max_lds(&s_maxcnt, maxcnt);
  __syncthreads();
  if (tid == 0 && s_maxcnt) atomicMax(&a.counters[C_MAXCNT], s_maxcnt);
  a.plen[(int64_t)blockIdx.x * kBuckets + tid] =
      cap ? min(wcur[tid], cap) : wcur[tid] - a.pstart[(int64_t)blockIdx.x * kBuckets + tid];
  wave_count(&a.counters[C_NULL_ROWS], nulls);
  wave_count(&a.counters[C_NULL_GROUP], nullg);
  wave_count(&a.counters[C_DBG_BYPASS], dbg_bypass);
  wave_count(&a.counters[C_NAN_FOLDED], nanf);
  if (tid == 0 && s_full) atomicAdd(&a.counters[C_DBG_FULL], (unsigned long long)s_full);
}

// ------------------------------------------------------------------------------------------------
// Phase A, dense integer keys: a batch of an integer (or boolean) key whose keyed values span
// fewer than kDenseW consecutive values (the pre-pass measured the range: numViews, status codes,
// years -- low-cardinality columns the bucket pieces would write a record per row for) is counted
// by value in LDS instead: freq_dense_count adds each row to its value's counter (one LDS add,
// no hash, no sort) and writes each workgroup's counters; freq_dense_emit sums them per value and
// writes one record per nonzero count digit, bucket-sorted in the batch's first chunks -- the
// chunk layout phase A leaves for collapsed keys, so phases B and C see a few records per value
// instead of one per row.  A wider batch is declined (both kernels return at once) and
// freq_phaseA_xp does it; when the dense path takes it, freq_phaseA_xp leaves empty pieces.
// ------------------------------------------------------------------------------------------------
constexpr int kDenseW = 79 * 512;  // values counted per batch (158 KiB of LDS counters)
constexpr int kDenseV = 512;       // values per emitted chunk (<= 16 digits each: <= kTile records)
constexpr int kDenseSumV = 128;    // values per summing workgroup (four threads each)
constexpr int kDenseThreads = 1024;
constexpr int kDenseBlocks = 256;  // counting workgroups (one per CU): their counter rows

// The batch's window, or false (declined): the keyed values' range fits kDenseW and the
// emitting chunks fit the batch's chunk slots (tiles + workgroup chunks).
DQ_DEV bool dense_window(const AArgs& a, uint64_t& lo, uint32_t& nvals) {
  const uint64_t mxe = __hip_atomic_load(&a.dense_words[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t mne = ~__hip_atomic_load(&a.dense_words[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (mxe < mne || mxe - mne >= (uint64_t)kDenseW) return false;  // (no keyed row / too wide)
  nvals = (uint32_t)(mxe - mne) + 1u;
  const int64_t n_tiles = (a.n_items + a.tile_items - 1) / a.tile_items;
  const int64_t chunks = n_tiles + (n_tiles + a.tiles_per_wg - 1) / a.tiles_per_wg;
  if ((int64_t)((nvals + kDenseV - 1) / kDenseV) > chunks) return false;
  lo = mne ^ kDenseSign;  // the smallest keyed value (widened)
  return true;
}

template <int TY>
__global__ void __launch_bounds__(kDenseThreads) freq_dense_count(AArgs a, uint32_t* part) {
  __shared__ uint32_t cnt[kDenseW];
  uint64_t lo;
  uint32_t nvals;
  if (!dense_window(a, lo, nvals)) return;  // (block-uniform)
  const int tid = threadIdx.x;
  for (uint32_t i = tid; i < nvals; i += kDenseThreads) cnt[i] = 0;
  __syncthreads();
  const KeyCol& c = a.ks.cols[0];
  unsigned long long nn = 0;
  const int64_t stride = (int64_t)gridDim.x * kDenseThreads * 4;
  for (int64_t r0 = (int64_t)blockIdx.x * kDenseThreads * 4; r0 < a.n_items; r0 += stride) {
    uint64_t v[4];
    uint32_t ok = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // rows r0 + 1024 j + tid: each wave-instruction contiguous
      const int64_t r = r0 + (int64_t)j * kDenseThreads + tid;
      const bool in = r < a.n_items;
      v[j] = kwiden(TY, c.values, in ? r : 0);
      ok |= (in && kbit(c.valid, r) ? 1u : 0u) << j;
      nn += in && !((ok >> j) & 1u) ? 1u : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((ok >> j) & 1u) atomicAdd(&cnt[(uint32_t)(v[j] - lo)], 1u);
  }
  __shared__ unsigned long long s_nn;  // the workgroup's NULL rows: one global atomic
  if (tid == 0) s_nn = 0;
  __syncthreads();
  nn = wave_sum(nn);
  if (__lane_id() == 0 && nn) atomicAdd(&s_nn, nn);
  __syncthreads();
  if (tid == 0 && s_nn) atomicAdd(&a.counters[a.ks.null_as_group ? C_NULL_GROUP : C_NULL_ROWS], s_nn);
  for (uint32_t i = tid; i < nvals; i += kDenseThreads) part[(size_t)blockIdx.x * kDenseW + i] = cnt[i];
}

// The counting workgroups' rows summed per value (kDenseSumV values per workgroup, a quarter of
// the rows per thread): sums[v].
__global__ void __launch_bounds__(kBuckets) freq_dense_sum(AArgs a, const uint32_t* part, int n_part,
                                                           unsigned long long* sums) {
  constexpr int kSlices = kBuckets / kDenseSumV;
  __shared__ unsigned long long s_sum[kSlices][kDenseSumV];
  uint64_t lo;
  uint32_t nvals;
  if (!dense_window(a, lo, nvals)) return;
  const int tid = threadIdx.x, q = tid / kDenseSumV, i = tid % kDenseSumV;
  const uint32_t v = blockIdx.x * kDenseSumV + (uint32_t)i;
  if (blockIdx.x * kDenseSumV >= nvals) return;  // (block-uniform)
  uint64_t acc = 0;
  if (v < nvals) {
#pragma unroll 16
    for (int g = q; g < n_part; g += kSlices) acc += part[(size_t)g * kDenseW + v];
  }
  s_sum[q][i] = acc;
  __syncthreads();
  if (tid < kDenseSumV && v < nvals) {
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < kSlices; ++k) t += s_sum[k][tid];
    sums[v] = t;
  }
}

// One block per kDenseV values: one record per nonzero base-4 digit of each value's count,
// counting-sorted by bucket into chunk blockIdx.x of the batch; the batch's other chunk rows are
// emptied.
__global__ void __launch_bounds__(kDenseV) freq_dense_emit(AArgs a, const unsigned long long* sums) {
  __shared__ uint32_t bh[kBuckets];
  __shared__ uint32_t s_wave[kDenseV / 64];
  __shared__ unsigned long long s_maxcnt;
  uint64_t lo;
  uint32_t nvals;
  const int tid = threadIdx.x;
  if (!dense_window(a, lo, nvals)) {
    if (blockIdx.x == 0 && tid == 0)
      __hip_atomic_store(&a.dense_words[3], (unsigned long long)a.dense_epoch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  static_assert(kDenseV == kBuckets, "one bucket per thread");
  const int64_t n_tiles = (a.n_items + a.tile_items - 1) / a.tile_items;
  const int64_t chunks = n_tiles + (n_tiles + a.tiles_per_wg - 1) / a.tiles_per_wg;
  if ((int64_t)blockIdx.x >= chunks) return;  // (a batch of fewer chunks than blocks)
  // the rows of the chunks past the grid: empty
  for (int64_t r = (int64_t)gridDim.x + blockIdx.x; r < chunks; r += gridDim.x)
    for (int i = tid; i < kHistRow; i += kDenseV) a.hist[r * kHistRow + i] = 0;
  bh[tid] = 0;
  if (tid == 0) s_maxcnt = 0;
  __syncthreads();
  const uint32_t v = blockIdx.x * kDenseV + tid;
  const uint64_t cn = v < nvals ? sums[v] : 0ULL;
  const uint64_t h = fmix_bij(lo + v);  // the exact key hash of value lo + v
  uint32_t nd = 0;
  for (uint64_t x = cn; x; x >>= 2) nd += (x & 3) ? 1u : 0u;
  const uint32_t b = bucket_of(h);
  const uint32_t rank = nd ? atomicAdd(&bh[b], nd) : 0u;
  __syncthreads();
  uint32_t total;
  const uint32_t cb = bh[tid];
  const uint32_t ex = block_excl_scan(cb, s_wave, total);
  uint16_t* hrow = a.hist + (int64_t)blockIdx.x * kHistRow;
  hrow[tid] = (uint16_t)ex;
  if (tid == 0) hrow[kBuckets] = (uint16_t)total;
  __syncthreads();
  bh[tid] = ex;
  __syncthreads();
  if (nd) {
    uint64_t* out = reinterpret_cast<uint64_t*>(a.recs) + (int64_t)blockIdx.x * FM<false>::kTile;
    uint32_t pos = bh[b] + rank;
    for_digits(cn, [&](uint32_t code) { out[pos++] = (h << 8) | code; });
  }
  wave_max_lds(&s_maxcnt, cn);
  __syncthreads();
  if (tid == 0) {
    if (s_maxcnt) atomicMax(&a.counters[C_MAXCNT], s_maxcnt);
    if (blockIdx.x == 0)
      __hip_atomic_store(&a.dense_words[2], (unsigned long long)a.dense_epoch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Per bucket (one block each): ph[*][b] -> its exclusive prefix over the workgroups, tot[b] = sum.
__global__ void __launch_bounds__(256) freq_prepass_scan(uint32_t* ph, int64_t n_wg, uint32_t* tot) {
  __shared__ uint32_t s_wave[4];
  const int b = blockIdx.x;
  uint32_t carry = 0;
  for (int64_t w0 = 0; w0 < n_wg; w0 += 256) {
    const int64_t w = w0 + threadIdx.x;
    const uint32_t v = w < n_wg ? ph[w * kBuckets + b] : 0u;
    uint32_t t;
    const uint32_t ex = block_excl_scan(v, s_wave, t);
    if (w < n_wg) ph[w * kBuckets + b] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) tot[b] = carry;
}

// ------------------------------------------------------------------------------------------------
// Phase A, small keys: a one-utf8-column key whose strings are at most 7 bytes long and that takes
// few distinct values (priority: 3) -- the common low-cardinality case -- counted at streaming
// speed, without hashing, LDS tables or barriers per tile.
//
// A string of at most 7 bytes is its own exact 64-bit key: bytes | length << 56.  Each wave walks
// 1024-row steps like the scan's TK_STR_IN body (16-byte offset loads, one unaligned 8-byte load
// per string, the validity slice redistributed across the wave) and keeps up to kSmallCand
// candidate keys, wave-uniform, with one u32 counter per candidate per lane: a row costs a few
// compares and adds in registers.  A key not among the candidates joins them (a wave-uniform loop,
// once per new key per wave).  A string longer than 7 bytes, or a (kSmallCand + 1)-th key in a
// wave, gives the batch up: the wave stores the batch's epoch in fast_words[0] and every wave
// stops at its next step, and the general phase A (launched right behind, freq_phaseA<STR1>)
// sees the epoch and does the batch itself.  Otherwise the general kernel returns at once and this
// kernel's output stands: every tile chunk of the workgroup empty, and the workgroup's groups in
// its own chunk (n_tiles + blockIdx.x), exactly the layout phase A leaves for collapsed keys --
// records {h, arena offset << 8 | count digit} with the row hash of freq_codec.h and the key
// encoded in the arena as str1_encode would.
// ------------------------------------------------------------------------------------------------
constexpr int kSmallCand = 8;
constexpr int kSmallThreads = 256;
constexpr int kBatchSlots = 64;
constexpr int kBatchTabWords = 2 * kBatchSlots + 1;
// one table per XCD class of workgroups (blockIdx % 8): 8x less contention on its slots and its
// arrival counter (2000+ workgroups adding into one table serialised the kernel's tail), 8 records
// per group per batch instead of one
constexpr int kBatchTabs = 8;
constexpr uint64_t kLongKey = ~0ULL;
// an unused candidate: length byte 0xFE, which neither a short key (<= 7) nor kLongKey (0xFF) has,
// so a long string never matches a free slot and is always seen as a miss
constexpr uint64_t kFreeCand = 0xFEULL << 56;

DQ_DEV uint64_t small_key(uint64_t v, int32_t len) {  // branch-free: selects, no exec masking
  const uint32_t sh = 8u * ((uint32_t)len & 7u);
  const uint64_t m = sh ? (~0ULL >> (64u - sh)) : 0ULL;
  const uint64_t k = (v & m) | ((uint64_t)(uint32_t)len << 56);
  return len > 7 ? kLongKey : k;
}

// The loads of one 1024-row step that do not depend on the character data: four 16-byte offset
// loads per lane (+ each 256-row group's closing offset) and the step's validity bitmap slice.
struct StrOffsets {
  int4 q[4];
  int32_t last[4];
  ChunkBits c;
  DQ_DEV void load(const int32_t* off, const uint8_t* valid, int64_t r0, int l) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint4 u = ld16(off + r0 + 256 * g + 4 * l);
      q[g] = make_int4((int)u.x, (int)u.y, (int)u.z, (int)u.w);
      last[g] = ldg_i32(off + r0 + 256 * g + 256);
    }
    c.load(valid, r0);  // (never null here)
  }
  // o[g][0..4]: the offsets of lane l's rows 256 g + 4 l .. + 3 and the one after them
  DQ_DEV void offsets(int32_t (&o)[4][5], int l) const {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int32_t nxt = __shfl_down(q[g].x, 1);
      o[g][0] = q[g].x;
      o[g][1] = q[g].y;
      o[g][2] = q[g].z;
      o[g][3] = q[g].w;
      o[g][4] = l == 63 ? last[g] : nxt;
    }
  }
};


__global__ void __launch_bounds__(kSmallThreads) freq_phaseA_small(AArgs a) {
  constexpr int NW = kSmallThreads / 64;
  __shared__ uint64_t s_key[NW * kSmallCand], s_cnt[NW * kSmallCand];
  __shared__ uint32_t s_nc[NW];
  // the workgroup's groups (+ the batch table's, for the last workgroup)
  __shared__ uint64_t g_key[NW * kSmallCand + kBatchSlots], g_cnt[NW * kSmallCand + kBatchSlots],
      g_off[NW * kSmallCand + kBatchSlots];
  __shared__ uint32_t g_rec[NW * kSmallCand + kBatchSlots];  // records (count digits) per group
  __shared__ uint32_t s_ng;
  const int tid = threadIdx.x, lane = (int)__lane_id(), wave = tid >> 6;
  const KeyCol& c = a.ks.cols[0];
  const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
  const int64_t n_tiles = (a.n_items + a.tile_items - 1) / a.tile_items;
  // this workgroup stands for the general kernel's workgroups [v0, v1): their tiles, and their
  // chunks n_tiles + v -- the first holds this workgroup's records, the others stay empty (fewer,
  // longer workgroups: the per-workgroup tail -- merge, table adds, records -- amortised)
  const int64_t n_vwg = (n_tiles + a.tiles_per_wg - 1) / a.tiles_per_wg;
  const int64_t v0 = (int64_t)blockIdx.x * a.small_merge;
  const int64_t v1 = min(v0 + (int64_t)a.small_merge, n_vwg);
  const int64_t t0 = v0 * a.tiles_per_wg;
  const int64_t t1 = min(v1 * (int64_t)a.tiles_per_wg, n_tiles);
  zero_u16(a.hist, t0 * kHistRow, t1 * kHistRow, tid, kSmallThreads);
  zero_u16(a.hist, (n_tiles + v0 + 1) * kHistRow, (n_tiles + v1) * kHistRow, tid, kSmallThreads);
  const int64_t r_begin = t0 * a.tile_items, r_end = min(t1 * a.tile_items, a.n_items);
  const int32_t dlen = off[a.n_items];

  uint64_t cand[kSmallCand];
  uint32_t cnt[kSmallCand];
#pragma unroll
  for (int k = 0; k < kSmallCand; ++k) {
    cand[k] = kFreeCand;
    cnt[k] = 0;
  }
  int nc = 0;
  bool gave_up = false;
  unsigned long long nulls = 0;
  // count the rows of `pend` (bit i: key[i]) that match a candidate; returns the rest.  Each row
  // finds its candidate index (unused candidates hold kFreeCand, which no row's key equals) and adds
  // one to that index's byte of a packed per-lane counter word (<= 16 per byte per call).
  // NC: the candidates compared (a wave with at most 4 -- 3-value columns like priority -- skips
  // the other half of the compares; the slots past nc hold kFreeCand)
  auto count_nc = [&](const uint64_t* key, uint32_t pend, auto nc_const) -> uint32_t {
    constexpr int NC = decltype(nc_const)::value;
    uint64_t packed = 0;
    uint32_t miss = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int idx = kSmallCand;
#pragma unroll
      for (int k = 0; k < NC; ++k) idx = key[i] == cand[k] ? k : idx;
      const bool p = (pend >> i) & 1u;
      packed += (p && idx < kSmallCand) ? (1ULL << (8 * idx)) : 0ULL;
      miss |= (p && idx == kSmallCand ? 1u : 0u) << i;
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) cnt[k] += (uint32_t)(packed >> (8 * k)) & 0xffu;
    return miss;
  };
  auto count = [&](const uint64_t* key, uint32_t pend) -> uint32_t {
    return count_nc(key, pend, std::integral_constant<int, kSmallCand>{});
  };
  // rows whose key is not yet a candidate: add their keys (wave-uniform), then count them
  auto admit = [&](const uint64_t* key, uint32_t pend) {
    while (true) {
      const uint64_t any = __ballot(pend != 0);
      if (!any) break;
      const int src = __builtin_ctzll(any);
      uint64_t fk = 0;
#pragma unroll
      for (int i = 15; i >= 0; --i)
        if ((pend >> i) & 1u) fk = key[i];
      const uint64_t nk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(fk >> 32), src) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fk, src);
      if (nc == kSmallCand || nk == kLongKey) {
        gave_up = true;
        break;
      }
#pragma unroll
      for (int k = 0; k < kSmallCand; ++k)
        if (k == nc) cand[k] = nk;
      ++nc;
      pend = count(key, pend);
    }
  };

  const bool vec = a.vec_ok != 0;
  const int64_t stride = (int64_t)NW * kWaveRows;
  int64_t r0 = r_begin + (int64_t)wave * kWaveRows;
  if (vec) {
    // software pipeline (as the scan's str_in_item): the next step's offsets and validity are in
    // flight while this step's strings load and count.  Lane l owns rows r0 + 256 g + 4 l + j.
    // Every load of a step is unconditional (the last step re-reads itself, a missing validity
    // bitmap reads the offsets and is ignored), so the compiler counts the loads in flight exactly
    // and waits for each string load alone -- a conditional prefetch made it wait for the next
    // step's offsets before the last string of this one.
    const uint8_t* vsrc = c.valid ? c.valid : reinterpret_cast<const uint8_t*>(off);
    StrOffsets cur;
    if (r0 + kWaveRows <= r_end) cur.load(off, vsrc, r0, lane);
    while (r0 + kWaveRows <= r_end && !gave_up) {
      // another wave may have given the batch up (read with the step's loads, checked at its end;
      // a.fast_poll: every that many steps, 0 never -- a wave that gives up stops alone)
      unsigned long long flag = 0;
      if (a.fast_poll && (r0 / stride) % a.fast_poll == 0)
        flag = __hip_atomic_load(&a.fast_words[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t rn = r0 + stride + kWaveRows <= r_end ? r0 + stride : r0;
      int32_t o[4][5];
      cur.offsets(o, lane);
      uint32_t vb = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) vb |= cur.c.get(256 * g + 4 * lane, 4) << (4 * g);
      if (!c.valid) vb = 0xffffu;
      const int32_t step_end = cur.last[3];
      uint64_t key[16];
      if ((int64_t)step_end + 8 <= (int64_t)dlen) {  // every string has 8 readable bytes
        uint64_t v[16];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) v[4 * g + j] = ldg64_unaligned(c.data + o[g][j]);
        __builtin_amdgcn_sched_barrier(0);
        cur.load(off, vsrc, rn, lane);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) key[4 * g + j] = small_key(v[4 * g + j], o[g][j + 1] - o[g][j]);
      } else {  // the batch's last strings: loads that stay inside the data buffer
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int32_t len = o[g][j + 1] - o[g][j];
            uint64_t w0 = 0, w1 = 0;
            if (len > 0 && len <= 7) load_str16(c.data + o[g][j], len, w0, w1);
            key[4 * g + j] = small_key(w0, len);
          }
        cur.load(off, vsrc, rn, lane);
      }
      nulls += 16 - __popc(vb);
      const uint32_t pend = __builtin_amdgcn_readfirstlane(nc) <= 4
                                ? count_nc(key, vb, std::integral_constant<int, 4>{})
                                : count(key, vb);
      if (__ballot(pend != 0)) admit(key, pend);
      if (flag == a.fast_epoch) gave_up = true;
      r0 += stride;
    }
  }
  // batch tail or unaligned buffers: lane l owns rows r0 + 64 i + l, bounds-checked
  for (; r0 < r_end && !gave_up; r0 += stride) {
    if (__hip_atomic_load(&a.fast_words[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        a.fast_epoch) {
      gave_up = true;  // another wave gave the batch up
      break;
    }
    uint64_t key[16];
    uint32_t vb = 0, in = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t r = r0 + 64 * i + lane;
      key[i] = kLongKey;
      in |= (r < r_end ? 1u : 0u) << i;
      if (r < r_end && kbit(c.valid, r)) {
        vb |= 1u << i;
        const int32_t s0 = off[r], len = off[r + 1] - s0;
        uint64_t w0 = 0, w1 = 0;
        if (len > 0 && len <= 7) load_str16(c.data + s0, len, w0, w1);
        key[i] = small_key(w0, len);
      }
    }
    nulls += __popc(in & ~vb);
    const uint32_t pend = count(key, vb);
    if (__ballot(pend != 0)) admit(key, pend);
  }
  if (gave_up && lane == 0)
    __hip_atomic_store(&a.fast_words[0], (unsigned long long)a.fast_epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (__syncthreads_or(gave_up ? 1 : 0)) return;  // every wave of the workgroup returns here
  // the wave's candidates and counts -> LDS; thread 0 merges the waves' lists
  if (lane == 0) s_nc[wave] = (uint32_t)nc;
#pragma unroll
  for (int k = 0; k < kSmallCand; ++k) {
    const uint64_t tot = wave_sum((uint64_t)cnt[k]);
    if (lane == 0 && k < nc) {
      s_key[wave * kSmallCand + k] = cand[k];
      s_cnt[wave * kSmallCand + k] = tot;
    }
  }
  nulls = wave_sum(nulls);
  if (lane == 0 && nulls)
    atomicAdd(&a.fast_words[a.ks.null_as_group ? 2 : 1], nulls);
  __syncthreads();
  // The waves' lists merged (<= NW * kSmallCand groups, thread 0, LDS only), then added into the
  // batch's device table, one thread per group (a batch of a 3-value column then leaves 3 records,
  // not 3 per workgroup: phase C would otherwise count ~2000 records of one key per partition, a
  // serial chain of LDS atomics on one slot); a group the full table cannot take stays in this
  // workgroup's own records.  The last workgroup to arrive writes the table's groups as its
  // records too.
  __shared__ uint32_t s_ng0, s_last;
  __shared__ uint32_t s_placed[NW * kSmallCand];
  __shared__ uint64_t s_tkey[kBatchSlots], s_tcnt[kBatchSlots];
  if (tid == 0) {
    uint32_t ng = 0;
    for (int w = 0; w < NW; ++w)
      for (uint32_t k = 0; k < s_nc[w]; ++k) {
        const uint64_t key = s_key[w * kSmallCand + k], ct = s_cnt[w * kSmallCand + k];
        if (!ct) continue;
        uint32_t g = 0;
        while (g < ng && g_key[g] != key) ++g;
        if (g == ng) {
          g_key[ng] = key;
          g_cnt[ng++] = 0;
        }
        g_cnt[g] += ct;
      }
    s_ng0 = ng;
  }
  __syncthreads();
  const int tab = (int)(blockIdx.x % kBatchTabs);
  unsigned long long* tkeys = a.batch_tab + (size_t)tab * kBatchTabWords;
  unsigned long long* tcnts = tkeys + kBatchSlots;
  if (tid < (int)s_ng0) {  // group tid into the table (CAS on its key, then add its count)
    const unsigned long long tag = (unsigned long long)g_key[tid] + 1ULL;  // never 0
    uint32_t slot = (uint32_t)(fmix_bij(g_key[tid]) & (kBatchSlots - 1));
    uint32_t placed = 0;
    for (int probe = 0; probe < kBatchSlots && !placed; ++probe, slot = (slot + 1) & (kBatchSlots - 1)) {
      const unsigned long long prev = atomicCAS(&tkeys[slot], 0ULL, tag);
      if (prev == 0ULL || prev == tag) {
        atomicAdd(&tcnts[slot], (unsigned long long)g_cnt[tid]);
        placed = 1;
      }
    }
    s_placed[tid] = placed;
    __threadfence();  // this thread's adds complete before the workgroup arrives
  }
  __syncthreads();
  if (tid == 0) {
    const unsigned long long arrived = atomicAdd(&tkeys[2 * kBatchSlots], 1ULL);
    const unsigned int members = (gridDim.x - (unsigned)tab + kBatchTabs - 1) / kBatchTabs;
    s_last = arrived == (unsigned long long)members - 1 ? 1u : 0u;
  }
  __syncthreads();
  const bool last = s_last != 0;
  if (last && tid < kBatchSlots) {  // every workgroup's adds are in: read the table
    __threadfence();
    s_tkey[tid] = __hip_atomic_load(&tkeys[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tcnt[tid] = __hip_atomic_load(&tcnts[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (tid == 0) {
    const uint32_t ng0 = s_ng0;
    uint32_t kept = 0;  // groups the table did not take, compacted to the front
    for (uint32_t g = 0; g < ng0; ++g)
      if (!s_placed[g]) {
        g_key[kept] = g_key[g];
        g_cnt[kept++] = g_cnt[g];
      }
    if (last)  // the table's groups join this workgroup's records
      for (int slot = 0; slot < kBatchSlots; ++slot) {
        if (!s_tkey[slot]) continue;
        g_key[kept] = s_tkey[slot] - 1ULL;
        g_cnt[kept++] = s_tcnt[slot];
      }
    uint32_t ng = kept;
    uint64_t bytes = 0;
    for (uint32_t g = 0; g < ng; ++g) bytes += 8 + pad4((uint32_t)(g_key[g] >> 56));
    uint64_t at = bytes ? atomicAdd(a.arena_cursor, (unsigned long long)bytes) : 0ULL;
    for (uint32_t g = 0; g < ng; ++g) {  // str1_encode of the key: {1, len, bytes as LE words}
      const uint32_t len = (uint32_t)(g_key[g] >> 56);
      const uint64_t w0 = g_key[g] & ((1ULL << 56) - 1);
      uint32_t* dst = reinterpret_cast<uint32_t*>(a.arena + at);
      dst[0] = 1;
      dst[1] = len;
      if (len > 0) dst[2] = (uint32_t)w0;
      if (len > 4) dst[3] = (uint32_t)(w0 >> 32);
      g_off[g] = at;
      at += 8 + pad4(len);
      g_key[g] = str_row_hash_reg(w0, 0, (int32_t)len);  // from here on: the group's row hash
      uint32_t nd = 0;
      for (uint64_t x = g_cnt[g]; x; x >>= 2) nd += (x & 3) ? 1u : 0u;
      g_rec[g] = nd;
    }
    s_ng = ng;
  }
  __syncthreads();
  // the workgroup's chunk: records bucket-sorted (groups of one bucket in group order), its
  // histogram row the exclusive prefix of the records per bucket
  const uint32_t ng = s_ng;
  const int64_t fchunk = n_tiles + v0;
  uint16_t* hrow = a.hist + fchunk * kHistRow;
  for (int b = tid; b <= kBuckets; b += kSmallThreads) {
    uint32_t before = 0;
    for (uint32_t g = 0; g < ng; ++g)
      if (b == kBuckets || bucket_of(g_key[g]) < (uint32_t)b) before += g_rec[g];
    hrow[b] = (uint16_t)before;
  }
  if (tid < (int)ng) {
    const uint32_t g = (uint32_t)tid, bg = bucket_of(g_key[g]);
    uint32_t pos = 0;
    for (uint32_t q = 0; q < ng; ++q) {
      const uint32_t bq = bucket_of(g_key[q]);
      if (bq < bg || (bq == bg && q < g)) pos += g_rec[q];
    }
    uint64_t* out = reinterpret_cast<uint64_t*>(a.recs) + (fchunk * (int64_t)FM<true>::kTile + pos) * 2;
    const uint64_t h = g_key[g], rep = g_off[g];
    uint32_t d = 0;
    for_digits(g_cnt[g], [&](uint32_t code) {
      out[2 * d] = h;
      out[2 * d + 1] = (rep << 8) | code;
      ++d;
    });
  }
}

// ------------------------------------------------------------------------------------------------
// Finalize: transpose the chunk histograms, scan them per bucket
// ------------------------------------------------------------------------------------------------
// Non-empty chunks, in order: a low-cardinality key leaves almost every tile's chunk empty (its
// rows collapse in phase A's LDS table), and finalize then runs over the non-empty ones only.
// C1 counts per 1024 chunks, freq_part_scan turns the counts into offsets, C2 writes the ids.
__global__ void __launch_bounds__(kThreads) freq_chunk_count(const uint16_t* hist, int64_t n,
                                                             unsigned long long* bcount) {
  __shared__ uint32_t s_wave[kThreads / 64];
  const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint32_t f = c < n && hist[c * kHistRow + kBuckets] != 0 ? 1u : 0u;
  uint32_t tot;
  block_excl_scan(f, s_wave, tot);
  if (threadIdx.x == 0) bcount[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(kThreads) freq_chunk_ids(const uint16_t* hist, int64_t n,
                                                           const unsigned long long* boff,
                                                           uint32_t* ids) {
  __shared__ uint32_t s_wave[kThreads / 64];
  const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint32_t f = c < n && hist[c * kHistRow + kBuckets] != 0 ? 1u : 0u;
  uint32_t tot;
  const uint32_t pos = block_excl_scan(f, s_wave, tot);
  if (f) ids[boff[blockIdx.x] + pos] = (uint32_t)c;
}

// ------------------------------------------------------------------------------------------------
// Segments.  Phase B reads each bucket as a list of segments (record ranges of `recs`): the
// bucket's part of every non-empty chunk (hashed mode, records path: runs of a few records) and
// every bucket piece of the exact batches (runs of ~250 records, adjacent ones contiguous).  One
// array pair per bucket, J columns: segS = first record, segP = length, then (freq_seg_scan) the
// list compacted -- empty segments dropped, contiguous neighbours merged (an exact batch's bucket
// is then ONE segment) -- with segP the exclusive record prefix and nseg the count.
// ------------------------------------------------------------------------------------------------
// cmap (optional): the chunk each of the n rows stands for (the non-empty chunks, in order)
__global__ void __launch_bounds__(256) freq_hist_transpose(const uint16_t* hist, int64_t n,
                                                           const uint32_t* cmap, int tile, int64_t J,
                                                           unsigned long long* segS, uint32_t* segP) {
  __shared__ uint16_t tl[64][kHistRow + 1];
  __shared__ uint32_t tc[64];
  const int64_t c0 = (int64_t)blockIdx.x * 64;
  for (int idx = threadIdx.x; idx < 64 * kHistRow; idx += 256) {
    const int cc = idx / kHistRow, b = idx % kHistRow;
    const int64_t c = c0 + cc;
    tl[cc][b] = c < n ? hist[(cmap ? (int64_t)cmap[c] : c) * kHistRow + b] : 0;
  }
  if (threadIdx.x < 64) {
    const int64_t c = c0 + threadIdx.x;
    tc[threadIdx.x] = c < n ? (cmap ? cmap[c] : (uint32_t)c) : 0u;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < kBuckets * 64; idx += 256) {
    const int b = idx / 64, cc = idx % 64;
    if (c0 + cc < n) {
      segS[(int64_t)b * J + c0 + cc] = (unsigned long long)tc[cc] * (unsigned)tile + tl[cc][b];
      segP[(int64_t)b * (J + 1) + c0 + cc] = (uint32_t)(tl[cc][b + 1] - tl[cc][b]);
    }
  }
}

// The bucket pieces of n_prow piece rows -> columns [col0, col0 + n_prow).
__global__ void __launch_bounds__(256) freq_piece_transpose(const uint32_t* pstart, const uint32_t* plen,
                                                            const unsigned long long* pbase, int64_t n_prow,
                                                            int64_t col0, int64_t J,
                                                            unsigned long long* segS, uint32_t* segP) {
  const int64_t total = n_prow * kBuckets;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i % n_prow, b = i / n_prow;  // consecutive threads: consecutive columns
    const int64_t src = r * kBuckets + b;
    segS[b * J + col0 + r] = pbase[r] + pstart[src];
    segP[b * (J + 1) + col0 + r] = plen[src];
  }
}

// Per bucket (one block each): compacts the bucket's J segments in place -- drops the empty ones,
// merges a segment into its predecessor entry when it starts where that one ends -- and turns the
// lengths into the exclusive record prefix (segP[nseg] = the bucket's records).
__global__ void __launch_bounds__(kThreads) freq_seg_scan(unsigned long long* segS, uint32_t* segP,
                                                          int64_t J, uint32_t* nseg,
                                                          unsigned long long* totals) {
  __shared__ uint32_t s_wave[kThreads / 64];
  __shared__ unsigned long long s_end[kThreads];  // each entry's end (start + length), or ~0
  __shared__ unsigned long long s_carry_end;
  const int b = blockIdx.x;
  unsigned long long* S = segS + (int64_t)b * J;
  uint32_t* P = segP + (int64_t)b * (J + 1);
  uint32_t carry_m = 0, carry_r = 0;
  if (threadIdx.x == 0) s_carry_end = ~0ULL;
  for (int64_t base = 0; base < J; base += kThreads) {
    const int64_t j = base + threadIdx.x;
    const bool in = j < J;
    const uint32_t len = in ? P[j] : 0u;
    const unsigned long long st = in ? S[j] : 0ULL;
    s_end[threadIdx.x] = len ? st + len : ~0ULL;
    __syncthreads();
    const unsigned long long prev_end = threadIdx.x ? s_end[threadIdx.x - 1] : s_carry_end;
    const uint32_t fresh = len && prev_end != st ? 1u : 0u;  // starts a compacted segment
    uint32_t tm, tr;
    const uint32_t m = block_excl_scan(fresh, s_wave, tm) + carry_m;
    const uint32_t r = block_excl_scan(len, s_wave, tr) + carry_r;
    // (every read of this round is done: the barriers of the scans)
    if (fresh) {
      S[m] = st;
      P[m] = r;
    }
    if (threadIdx.x == kThreads - 1) s_carry_end = s_end[kThreads - 1];
    carry_m += tm;
    carry_r += tr;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    P[carry_m] = carry_r;
    nseg[b] = carry_m;
    totals[b] = carry_r;
  }
}

// unit_c0[unit_start[b] + u] = the compacted segment holding the bucket's record u*H (units are
// record ranges [u*H, (u+1)*H) of the bucket), unit_b[unit] = b.
__global__ void __launch_bounds__(256) freq_unit_map(const uint32_t* segP, int64_t J, const uint32_t* nseg,
                                                     const uint32_t* unit_start, uint32_t H,
                                                     uint32_t* unit_c0, uint16_t* unit_b) {
  const int b = blockIdx.y;
  const uint32_t ub = unit_start[b], U = unit_start[b + 1] - ub;
  const uint32_t* P = segP + (int64_t)b * (J + 1);
  const int64_t n = nseg[b];
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t lo = P[c], hi = P[c + 1];
    for (uint64_t u = (lo + H - 1) / H; u * H < hi && u < U; ++u) unit_c0[ub + u] = (uint32_t)c;
  }
  if (blockIdx.x == 0)
    for (uint32_t u = threadIdx.x; u < U; u += blockDim.x) unit_b[ub + u] = (uint16_t)b;
}

// ------------------------------------------------------------------------------------------------
// Phase B: a bucket's records -> partition-contiguous records (radix scatter by the next s bits)
//
// A bucket's records are cut into units of H records (ranges of its segment list).  B1 counts
// each unit's records per sub-bucket, B2 turns the counts into each unit's offsets inside every
// partition (a scan over the bucket's units per sub-bucket) and the partitions' sizes, and B3
// re-reads the unit and writes every record to its final place: a partition's records end up in
// one contiguous range, written as runs of (records per unit / 2^s) per (unit, partition) whose
// neighbours come from the neighbouring units of the same XCD (units are handed out
// XCD-contiguously, so a partition's runs meet in one L2).
// ------------------------------------------------------------------------------------------------
struct BArgs {
  const uint8_t* recs;
  const unsigned long long* segS;  // [kBuckets][J] compacted segment starts
  const uint32_t* segP;            // [kBuckets][J + 1] their exclusive record prefix
  const uint32_t* nseg;            // [kBuckets]
  int64_t J;
  uint32_t H;                      // records per unit
  const uint32_t* unit_start;
  const uint32_t* unit_c0;
  const uint16_t* unit_b;
  int32_t s;
  uint32_t n_units;
  uint32_t* uhist;                        // [unit][S]: counts (B1) -> offsets in the partition (B2)
  unsigned long long* part_base;          // [P + 1]
  uint8_t* recsB;
  // capacity layout (cap_mode): each unit's run of partition p at atomicAdd(part_end[p], run),
  // within part_base[p] + bcap[bucket]; a run past it sets *bovf and is not written
  int32_t cap_mode;
  unsigned long long* part_end;
  const unsigned long long* bcap;
  unsigned int* bovf;
};

struct UnitLds {
  uint32_t sw_pos[kThreads];             // window-local prefix of the segments' records in the unit
  unsigned long long sw_s[kThreads];     // record index of each window segment's first such record
  uint32_t s_wave[kThreads / 64];
  uint32_t s_b, s_lo, s_hi;
  int64_t s_c0, s_c1;
};

DQ_DEV void unit_range(const BArgs& a, uint32_t w, UnitLds& L) {
  if (threadIdx.x == 0) {
    const uint32_t b = a.unit_b[w];
    const int64_t n = a.nseg[b];
    const uint32_t* P = a.segP + (int64_t)b * (a.J + 1);
    const uint32_t lo = (w - a.unit_start[b]) * a.H;
    L.s_b = b;
    L.s_lo = lo;
    L.s_hi = (uint32_t)min((uint64_t)lo + a.H, (uint64_t)P[n]);
    L.s_c0 = min((int64_t)a.unit_c0[w], n);
    L.s_c1 = w + 1 < a.unit_start[b + 1] ? min((int64_t)a.unit_c0[w + 1] + 1, n) : n;
  }
  __syncthreads();
}

// Loads the window of segments [cw, cw + kThreads) of the unit: each one's records inside the
// unit's range, as an exclusive prefix (sw_pos) and a first record (sw_s).  Returns the window's
// records; every thread of the block must call it.
DQ_DEV uint32_t unit_window(const BArgs& a, UnitLds& L, int64_t cw, uint32_t& nwin) {
  const int tid = threadIdx.x;
  const int64_t c = cw + tid, c1 = L.s_c1;
  uint32_t len = 0;
  unsigned long long st = 0;
  if (c < c1) {
    const uint32_t* P = a.segP + (int64_t)L.s_b * (a.J + 1);
    const uint32_t ps = P[c], pe = P[c + 1];
    const uint32_t a0 = max(ps, L.s_lo), a1 = min(pe, L.s_hi);
    len = a1 > a0 ? a1 - a0 : 0u;
    st = a.segS[(int64_t)L.s_b * a.J + c] + (a0 - ps);
  }
  uint32_t wtot;
  const uint32_t pos = block_excl_scan(len, L.s_wave, wtot);
  L.sw_pos[tid] = pos;
  L.sw_s[tid] = st;
  nwin = (uint32_t)min((int64_t)kThreads, c1 - cw);
  __syncthreads();
  return wtot;
}

DQ_DEV int64_t window_rec(const UnitLds& L, uint32_t nwin, uint32_t li) {
  const uint32_t j = seg_of(L.sw_pos, nwin, li);
  return (int64_t)L.sw_s[j] + (li - L.sw_pos[j]);
}

// Calls f(record words) for every record of the unit.  Every thread of the block must call it.
// Each thread loads PB records before it uses any (one HBM round trip per PB records; an
// out-of-range lane re-reads the window's last record and drops it).
template <bool HASHED, typename F>
DQ_DEV void for_unit_records(const BArgs& a, UnitLds& L, F&& f) {
  constexpr int W = FM<HASHED>::kRB / 8, PB = 8;
  const int tid = threadIdx.x;
  for (int64_t cw = L.s_c0; cw < L.s_c1; cw += kThreads) {
    uint32_t nwin;
    const uint32_t wtot = unit_window(a, L, cw, nwin);
    for (uint32_t base = 0; base < wtot; base += (uint32_t)PB * kThreads) {
      uint64_t rv[PB][W];
#pragma unroll
      for (int k = 0; k < PB; ++k) {
        uint32_t li = base + (uint32_t)k * kThreads + tid;
        li = li < wtot ? li : wtot - 1;
        const uint64_t* src = reinterpret_cast<const uint64_t*>(a.recs) + window_rec(L, nwin, li) * W;
#pragma unroll
        for (int x = 0; x < W; ++x) rv[k][x] = src[x];
      }
#pragma unroll
      for (int k = 0; k < PB; ++k)
        if (base + (uint32_t)k * kThreads + tid < wtot) f(rv[k]);
    }
    __syncthreads();
  }
}

DQ_DEV uint32_t rec_sub(const uint64_t* r, int s, bool hashed) {
  return sub_of(hashed ? r[0] : (r[0] >> 8), s);
}

// B1: per unit, records per sub-bucket
template <bool HASHED>
__global__ void __launch_bounds__(kThreads) freq_phaseB_count(BArgs a) {
  __shared__ UnitLds L;
  __shared__ uint32_t sh[1 << kMaxSubBits];
  const int S = 1 << a.s;
  for (int i = threadIdx.x; i < S; i += kThreads) sh[i] = 0;
  unit_range(a, blockIdx.x, L);
  for_unit_records<HASHED>(a, L, [&](const uint64_t* r) { atomicAdd(&sh[rec_sub(r, a.s, HASHED)], 1u); });
  uint32_t* row = a.uhist + (int64_t)blockIdx.x * S;
  for (int i = threadIdx.x; i < S; i += kThreads) row[i] = sh[i];
}

// B1, one wave per unit: the sixteen waves of a workgroup count sixteen units each on its own, in
// a histogram of its own in LDS, with no block barrier -- a unit's chain of dependent loads
// (unit -> bucket -> segments -> records) overlaps fifteen others' instead of stalling its
// workgroup (one unit per 1024-thread workgroup left ~two chains in flight per CU).  Same counts.
constexpr int kBcWaves = 16;
template <bool HASHED>
__global__ void __launch_bounds__(kBcWaves * 64) freq_phaseB_count_w(BArgs a) {
  constexpr int W = FM<HASHED>::kRB / 8, PB = 8;
  __shared__ uint32_t sh[kBcWaves][1 << kMaxSubBits];
  __shared__ uint32_t s_pos[kBcWaves][64];
  __shared__ unsigned long long s_st[kBcWaves][64];
  const int lane = (int)__lane_id(), wv = threadIdx.x >> 6;
  const uint32_t w = blockIdx.x * kBcWaves + (uint32_t)wv;
  if (w >= a.n_units) return;  // (wave-uniform: nothing below waits for the other waves)
  const int S = 1 << a.s;
  uint32_t* h = sh[wv];
  for (int i = lane; i < S; i += 64) h[i] = 0;
  const uint32_t b = a.unit_b[w];
  const int64_t n = a.nseg[b];
  const uint32_t* P = a.segP + (int64_t)b * (a.J + 1);
  const uint32_t lo = (w - a.unit_start[b]) * a.H;
  const uint32_t hi = (uint32_t)min((uint64_t)lo + a.H, (uint64_t)P[n]);
  const int64_t c0 = min((int64_t)a.unit_c0[w], n);
  const int64_t c1 = w + 1 < a.unit_start[b + 1] ? min((int64_t)a.unit_c0[w + 1] + 1, n) : n;
  for (int64_t cw = c0; cw < c1; cw += 64) {  // windows of 64 segments, a lane each
    const int64_t c = cw + lane;
    uint32_t len = 0;
    unsigned long long st = 0;
    if (c < c1) {
      const uint32_t ps = P[c], pe = P[c + 1];
      const uint32_t a0 = max(ps, lo), a1 = min(pe, hi);
      len = a1 > a0 ? a1 - a0 : 0u;
      st = a.segS[(int64_t)b * a.J + c] + (a0 - ps);
    }
    const uint32_t incl = __ockl_wfscan_add_u32(len, true);
    const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    s_pos[wv][lane] = incl - len;
    s_st[wv][lane] = st;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the window, before any lane reads it
    const uint32_t nwin = (uint32_t)min((int64_t)64, c1 - cw);
    for (uint32_t base = 0; base < wtot; base += (uint32_t)PB * 64) {
      uint64_t rv[PB];
#pragma unroll
      for (int k = 0; k < PB; ++k) {
        uint32_t li = base + (uint32_t)k * 64 + (uint32_t)lane;
        li = li < wtot ? li : wtot - 1;
        const uint32_t j = seg_of(s_pos[wv], nwin, li);
        rv[k] = reinterpret_cast<const uint64_t*>(a.recs)[(s_st[wv][j] + (li - s_pos[wv][j])) * W];
      }
#pragma unroll
      for (int k = 0; k < PB; ++k)
        if (base + (uint32_t)k * 64 + (uint32_t)lane < wtot)
          atomicAdd(&h[sub_of(HASHED ? rv[k] : rv[k] >> 8, a.s)], 1u);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // every lane's reads of the window done
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // every count in
  uint32_t* row = a.uhist + (int64_t)w * S;
  for (int i = lane; i < S; i += 64) row[i] = h[i];
}

// B2: per bucket, each unit's offset inside every partition, and the partitions' sizes
__global__ void __launch_bounds__(kThreads) freq_phaseB_scan(BArgs a) {
  const uint32_t b = blockIdx.x, S = 1u << a.s;
  const uint32_t u0 = a.unit_start[b], u1 = a.unit_start[b + 1];
  for (uint32_t sb = threadIdx.x; sb < S; sb += kThreads) {
    uint64_t run = 0;
    for (uint32_t u = u0; u < u1; ++u) {
      uint32_t* cell = a.uhist + (int64_t)u * S + sb;
      const uint32_t v = *cell;
      *cell = (uint32_t)run;
      run += v;
    }
    a.part_base[(uint64_t)b * S + sb] = run;  // sizes; freq_part_scan makes them offsets
  }
}

// exclusive scan of the P partition sizes in place; part_base[P] = total
__global__ void __launch_bounds__(kThreads) freq_part_scan(unsigned long long* v, int64_t P) {
  __shared__ uint32_t s_wave[kThreads / 64];
  __shared__ uint64_t s_red[kThreads / 64];
  const int64_t per = (P + kThreads - 1) / kThreads;
  const int64_t lo = threadIdx.x * per, hi = min(lo + per, P);
  uint64_t sum = 0;
  for (int64_t i = lo; i < hi; ++i) sum += v[i];
  // exclusive scan of the per-thread sums (64-bit: two 32-bit halves are not enough in general)
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  uint64_t x = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_red[wave] = x;
  __syncthreads();
  uint64_t base = 0;
  for (int w = 0; w < wave; ++w) base += s_red[w];
  uint64_t run = base + x - sum;
  for (int64_t i = lo; i < hi; ++i) {
    const uint64_t t = v[i];
    v[i] = run;
    run += t;
  }
  if (threadIdx.x == kThreads - 1) v[P] = run;
  (void)s_wave;
}

// B3: scatter every record of the unit to its partition, staged in LDS: each round of up to SUB
// records is counting-sorted by sub-bucket in LDS, then written out in staged order, so the lanes
// of a wave write runs of neighbouring addresses (a sub-bucket's records of the round) instead of
// 64 scattered 8-byte stores to 64 partitions.
// SUBB: staged bytes' worth of 8-byte words per round (8192: 64 KB staged, one workgroup per
// CU; 4096: 32 KB, two per CU so one's loads overlap the other's sort and stores)
template <bool HASHED, int SUBB = 8192>
__global__ void __launch_bounds__(kThreads) freq_phaseB_scatter(BArgs a) {
  constexpr int W = FM<HASHED>::kRB / 8;
  constexpr int SUB = SUBB / W;  // records per round
  constexpr int PER = SUB / kThreads;
  constexpr int SMAX = 1 << kMaxSubBits;
  __shared__ UnitLds L;
  __shared__ unsigned long long cur[SMAX];  // the unit's next output position per sub-bucket
  __shared__ unsigned long long gbs[SMAX];  // this round's output base per sub-bucket
  __shared__ uint32_t hcnt[SMAX];           // this round's count, then local base, per sub-bucket
  __shared__ uint64_t staged[SUB * W];
  __shared__ uint16_t ssb[SUB];
  // XCD-contiguous units: workgroup g runs on XCD g % 8; XCD x takes units [x*q, (x+1)*q)
  const uint32_t g = blockIdx.x, q = (a.n_units + 7) / 8;
  const uint32_t w = (g & 7u) * q + (g >> 3);
  if (w >= a.n_units) return;
  const int S = 1 << a.s;
  const int tid = threadIdx.x;
  unit_range(a, w, L);
  const uint32_t* row = a.uhist + (int64_t)w * S;
  for (int i = tid; i < S; i += kThreads) cur[i] = a.part_base[(uint64_t)L.s_b * S + i] + row[i];
  uint64_t* out = reinterpret_cast<uint64_t*>(a.recsB);
  for (int64_t cw = L.s_c0; cw < L.s_c1; cw += kThreads) {  // windows of segments
    uint32_t nwin;
    const uint32_t wtot = unit_window(a, L, cw, nwin);
    for (uint32_t base = 0; base < wtot; base += SUB) {
      const uint32_t nr = min((uint32_t)SUB, wtot - base);
      for (int i = tid; i < S; i += kThreads) hcnt[i] = 0;
      __syncthreads();
      uint64_t rv[PER][W];
      uint32_t sbv[PER], lpos[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const uint32_t r = (uint32_t)k * kThreads + tid;
        sbv[k] = 0;
        if (r >= nr) continue;
        const uint64_t* src = reinterpret_cast<const uint64_t*>(a.recs) + window_rec(L, nwin, base + r) * W;
#pragma unroll
        for (int x = 0; x < W; ++x) rv[k][x] = src[x];
        sbv[k] = rec_sub(rv[k], a.s, HASHED);
        lpos[k] = atomicAdd(&hcnt[sbv[k]], 1u);
      }
      __syncthreads();
      const uint32_t cnt = tid < S ? hcnt[tid] : 0u;
      uint32_t tot;
      const uint32_t ex = block_excl_scan(cnt, L.s_wave, tot);  // (barriers: every count is read)
      if (tid < S) {
        hcnt[tid] = ex;
        gbs[tid] = cur[tid];
        cur[tid] += cnt;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const uint32_t r = (uint32_t)k * kThreads + tid;
        if (r >= nr) continue;
        const uint32_t slot = hcnt[sbv[k]] + lpos[k];
#pragma unroll
        for (int x = 0; x < W; ++x) staged[slot * W + x] = rv[k][x];
        ssb[slot] = (uint16_t)sbv[k];
      }
      __syncthreads();
      for (uint32_t i = tid; i < nr; i += kThreads) {
        const uint32_t sb = ssb[i];
        const unsigned long long d = gbs[sb] + (i - hcnt[sb]);
#pragma unroll
        for (int x = 0; x < W; ++x) out[d * W + x] = staged[i * W + x];
      }
      __syncthreads();
    }
    __syncthreads();
  }
}

// B3, whole units: a unit of at most PER * kThreads records is loaded into registers, counted,
// placed in LDS in sub-bucket order and written out once, so each (unit, partition) run leaves as
// one stream of ~H / 2^s records (the round-based kernel above wrote it in ~H / SUB pieces, each
// a partial line the L2 had to merge).
template <bool HASHED, int PER>
__global__ void __launch_bounds__(kThreads) freq_phaseB_scatter_u(BArgs a) {
  constexpr int W = FM<HASHED>::kRB / 8;
  constexpr int SMAX = 1 << kMaxSubBits;
  constexpr uint32_t NR = (uint32_t)PER * kThreads;
  // the segment window is dead once the unit's records are in registers, before anything is
  // staged: one LDS region for both (PER = 8: 76 KB, two workgroups per CU)
  __shared__ union {
    UnitLds L;
    uint64_t staged[NR * W];
  } su;
  UnitLds& L = su.L;
  uint64_t* staged = su.staged;
  __shared__ unsigned long long gbs[SMAX];  // the unit's output base per sub-bucket
  __shared__ uint32_t hcnt[SMAX];           // the unit's count, then its local base, per sub-bucket
  // XCD-contiguous units: workgroup g runs on XCD g % 8; XCD x takes units [x*q, (x+1)*q)
  const uint32_t g = blockIdx.x, q = (a.n_units + 7) / 8;
  const uint32_t w = (g & 7u) * q + (g >> 3);
  if (w >= a.n_units) return;
  const int S = 1 << a.s;
  const int tid = threadIdx.x;
  for (int i = tid; i < S; i += kThreads) hcnt[i] = 0;
  unit_range(a, w, L);
  const uint32_t nrec = L.s_hi - L.s_lo;  // <= NR (the host sizes units so)
  uint64_t rv[PER][W];
  uint32_t done = 0;
  for (int64_t cw = L.s_c0; cw < L.s_c1; cw += kThreads) {  // windows of segments (usually one)
    uint32_t nwin;
    const uint32_t wtot = unit_window(a, L, cw, nwin);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t r = (uint32_t)j * kThreads + tid;
      if (r >= done && r < done + wtot) {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(a.recs) + window_rec(L, nwin, r - done) * W;
#pragma unroll
        for (int x = 0; x < W; ++x) rv[j][x] = src[x];
      }
    }
    done += wtot;
    __syncthreads();
  }
  uint32_t lpos[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if ((uint32_t)j * kThreads + tid < nrec) lpos[j] = atomicAdd(&hcnt[rec_sub(rv[j], a.s, HASHED)], 1u);
  __syncthreads();
  const uint32_t cnt = tid < S ? hcnt[tid] : 0u;
  uint32_t tot;
  const uint32_t ex = block_excl_scan(cnt, L.s_wave, tot);  // (barriers: every count is read)
  if (tid < S) {
    hcnt[tid] = ex;
    if (a.cap_mode) {  // (the unit's run of each partition: one device-scope cursor add per run)
      const uint64_t p = (uint64_t)L.s_b * S + tid;
      unsigned long long g = 0;
      if (cnt) {
        g = atomicAdd(&a.part_end[p], (unsigned long long)cnt);
        if (g + cnt > a.part_base[p] + a.bcap[L.s_b]) {  // past the capacity: not written
          atomicOr(a.bovf, 1u);
          g = ~0ULL;
        }
      }
      gbs[tid] = g;
    } else {
      gbs[tid] = a.part_base[(uint64_t)L.s_b * S + tid] + a.uhist[(int64_t)w * S + tid];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if ((uint32_t)j * kThreads + tid >= nrec) continue;
    const uint32_t slot = hcnt[rec_sub(rv[j], a.s, HASHED)] + lpos[j];
#pragma unroll
    for (int x = 0; x < W; ++x) staged[slot * W + x] = rv[j][x];
  }
  __syncthreads();
  uint64_t* out = reinterpret_cast<uint64_t*>(a.recsB);
  for (uint32_t i = tid; i < nrec; i += kThreads) {
    uint64_t r[W];
#pragma unroll
    for (int x = 0; x < W; ++x) r[x] = staged[i * W + x];
    const uint32_t sb = rec_sub(r, a.s, HASHED);
    if (gbs[sb] == ~0ULL) continue;  // (an overflowing run: the table falls back to the count)
    const unsigned long long d = gbs[sb] + (i - hcnt[sb]);
#pragma unroll
    for (int x = 0; x < W; ++x) out[d * W + x] = r[x];
  }
}

// The capacity layout's partition starts (bucket base + sub-bucket x the bucket's capacity), and
// its cursors, which the scatter's adds advance to the partitions' ends.
__global__ void __launch_bounds__(256) freq_cap_layout(const unsigned long long* __restrict__ words,
                                                       int s, int64_t P,
                                                       unsigned long long* __restrict__ part_base,
                                                       unsigned long long* __restrict__ part_end) {
  const unsigned long long* bbase = words;              // [kBuckets + 1]
  const unsigned long long* bcap = words + kBuckets + 1;  // [kBuckets]
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < P; p += (int64_t)gridDim.x * 256) {
    const int64_t b = p >> s, sb = p & ((1LL << s) - 1);
    const unsigned long long v = bbase[b] + (unsigned long long)sb * bcap[b];
    part_base[p] = v;
    part_end[p] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) part_base[P] = bbase[kBuckets];
}

// B3, whole units, persistent: workgroup g of an XCD takes that XCD's units g, g + G/8, ... and
// issues the loads of its next unit right after placing the current one in LDS, so they are in
// flight while the current unit's runs are written (freq_phaseB_scatter_u, one workgroup per CU by
// LDS and one unit per workgroup, left every load latency exposed).  Same output.
template <bool HASHED, int PER>
__global__ void __launch_bounds__(kThreads) freq_phaseB_scatter_p(BArgs a) {
  constexpr int W = FM<HASHED>::kRB / 8;
  constexpr int SMAX = 1 << kMaxSubBits;
  constexpr uint32_t NR = (uint32_t)PER * kThreads;
  __shared__ UnitLds L;
  __shared__ unsigned long long gbs[SMAX];
  __shared__ uint32_t hcnt[SMAX];
  __shared__ uint64_t staged[NR * W];
  const uint32_t g = blockIdx.x, per_xcd = gridDim.x / 8u, q = (a.n_units + 7) / 8;
  const uint32_t x = g & 7u, gl = g >> 3;
  const uint32_t uend = min((x + 1) * q, a.n_units);
  uint32_t w = x * q + gl;
  if (w >= uend) return;  // (workgroup-uniform)
  const int S = 1 << a.s;
  const int tid = threadIdx.x;
  for (int i = tid; i < S; i += kThreads) hcnt[i] = 0;
  uint64_t rv[PER][W];
  // the unit's records into rv (the loads are left in flight); returns its record count
  auto load_unit = [&](uint32_t u) -> uint32_t {
    unit_range(a, u, L);
    const uint32_t nrec = L.s_hi - L.s_lo;  // <= NR (the host sizes units so)
    uint32_t done = 0;
    for (int64_t cw = L.s_c0; cw < L.s_c1; cw += kThreads) {  // windows of segments (usually one)
      uint32_t nwin;
      const uint32_t wtot = unit_window(a, L, cw, nwin);
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const uint32_t r = (uint32_t)j * kThreads + tid;
        if (r >= done && r < done + wtot) {
          const uint64_t* src = reinterpret_cast<const uint64_t*>(a.recs) + window_rec(L, nwin, r - done) * W;
#pragma unroll
          for (int y = 0; y < W; ++y) rv[j][y] = src[y];
        }
      }
      done += wtot;
      __syncthreads();
    }
    return nrec;
  };
  uint32_t nrec = load_unit(w), b = L.s_b;
  uint64_t* out = reinterpret_cast<uint64_t*>(a.recsB);
  while (true) {
    uint32_t lpos[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if ((uint32_t)j * kThreads + tid < nrec) lpos[j] = atomicAdd(&hcnt[rec_sub(rv[j], a.s, HASHED)], 1u);
    __syncthreads();
    const uint32_t cnt = tid < S ? hcnt[tid] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(cnt, L.s_wave, tot);  // (barriers: every count is read)
    if (tid < S) {
      hcnt[tid] = ex;
      gbs[tid] = a.part_base[(uint64_t)b * S + tid] + a.uhist[(int64_t)w * S + tid];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if ((uint32_t)j * kThreads + tid >= nrec) continue;
      const uint32_t slot = hcnt[rec_sub(rv[j], a.s, HASHED)] + lpos[j];
#pragma unroll
      for (int y = 0; y < W; ++y) staged[slot * W + y] = rv[j][y];
    }
    __syncthreads();
    // the next unit's loads go out before this unit's stores
    const uint32_t wn = w + per_xcd;
    const bool more = wn < uend;
    uint32_t nrec_n = 0, b_n = 0;
    if (more) {
      nrec_n = load_unit(wn);
      b_n = L.s_b;
    }
    for (uint32_t i = tid; i < nrec; i += kThreads) {
      uint64_t r[W];
#pragma unroll
      for (int y = 0; y < W; ++y) r[y] = staged[i * W + y];
      const uint32_t sb = rec_sub(r, a.s, HASHED);
      const unsigned long long d = gbs[sb] + (i - hcnt[sb]);
#pragma unroll
      for (int y = 0; y < W; ++y) out[d * W + y] = r[y];
    }
    if (!more) break;
    __syncthreads();
    for (int i = tid; i < S; i += kThreads) hcnt[i] = 0;
    __syncthreads();
    w = wn;
    nrec = nrec_n;
    b = b_n;
  }
}

// ------------------------------------------------------------------------------------------------
// Phase C: count partitions in LDS
//
// Persistent: workgroup w takes work items w, w + grid, ...  (a work item is a partition, or on a
// recount one hash subset of one), and the loads of the next item's first records are in flight
// while the current item's statistics are reduced, so the chain of dependent HBM round trips that
// bounded one-partition-per-workgroup launches is hidden.
// ------------------------------------------------------------------------------------------------
struct CArgs {
  const uint8_t* recsB;
  const unsigned long long* part_base;  // partition p's records: [part_base[p], part_end[p])
  const unsigned long long* part_end;   // (the counted layout: part_base + 1)
  int32_t s;
  int32_t n_work;                       // partitions (first pass) or entries (recount)
  const uint8_t* arena;
  int32_t types[kMaxKeys];
  int32_t n_keys;
  int32_t want_cand;
  double num_rows;
  const FEntry* entries;  // nullptr: the first pass over every partition
  unsigned long long* part_groups;
  unsigned long long* part_unique;
  unsigned long long* part_entropy;  // per partition: the fixed-point sum (lo, hi)
  unsigned long long* part_off;  // materialised groups of partition p start here
  FEntry* ovf_out;
  unsigned int* ovf_n;
  Group* cand;
  Group* groups;  // materialise every group (nullptr: statistics only)
  unsigned long long* counters;
  // Histogram on a string column: the count of the "NullValue" string group is added to
  // *lit_count (nullptr: no probe); lit_h is that key's row hash
  uint64_t lit_h;
  unsigned long long* lit_count;
  unsigned long long* dbg_clock;  // DQ_FREQ_DEBUG=2: workgroup 0's per-item stamps (wall clock)
  // 0: groups materialise at their partition's record offset; else work item wi's groups go to
  // groups[wi * group_stride ..] (dq_freq_topk's recount of a few partitions)
  uint32_t group_stride;
  // freq_phaseC_x, first pass: the work items' record ranges come from a per-lane cache of 64
  // items' bounds (vector loads issued 64 items ahead) instead of scalar loads per item (< 2^32
  // records; 0: the scalar loads)
  uint32_t bcache;
  // freq_phaseC_x: workgroup g takes the contiguous items [g * ipw, (g + 1) * ipw) instead of
  // g, g + grid, ... (0: strided)
  uint32_t contig;
};

// Is the encoded one-column utf8 key at p the 9-byte string "NullValue"?
DQ_DEV bool enc_is_null_literal(const uint8_t* p) {
  const uint32_t* e = reinterpret_cast<const uint32_t*>(p);
  return e[0] == 1u && e[1] == (uint32_t)kNullValueLen && e[2] == (uint32_t)kNullValueLo &&
         e[3] == (uint32_t)(kNullValueLo >> 32) && e[4] == kNullValueHi;
}

constexpr int kCThreads = 512;  // phase-C workgroup: two per CU by LDS, 128 VGPRs per lane
// freq_phaseC_x's workgroup: packed tables run one 1024-thread workgroup per CU (a 128 KB table)
template <bool PK>
constexpr int kCThreadsX = PK ? 1024 : kCThreads;
// records per thread loaded ahead: exact partitions (~kTarget records) arrive whole
template <bool HASHED>
constexpr int kPF = HASHED ? 2 : 4;

// A work item and the raw words of its first kPF * kCThreads records (decoded at insert time,
// so the prefetch holds one word per exact record).
template <bool HASHED>
struct CItem {
  uint32_t p, f, fv;
  uint64_t r0, r1;
  uint64_t w[kPF<HASHED>][FM<HASHED>::kRB / 8];
  uint32_t valid;
};

template <bool HASHED>
DQ_DEV void c_decode(const uint64_t* w, uint32_t b, uint64_t& h, uint64_t& c, uint64_t& rep) {
  if constexpr (HASHED) {
    h = w[0];
    c = code_count((uint32_t)(w[1] & 0xff));
    rep = w[1] >> 8;
  } else {
    h = xrec_h(w[0], b);
    c = code_count((uint32_t)(w[0] & 0xff));
    rep = 0;
  }
}

// A work item's partition / hash subset and its record range, loaded one item ahead of its
// records (so fetching the records of the next item is one HBM round trip, not two).
struct CBounds {
  uint32_t p, f, fv;
  uint64_t r0, r1;
};
// (wave-uniform reads of words phase C never writes, through the constant address space: scalar
// loads, counted by lgkmcnt -- as vector loads, a wait for them in the next item was also a wait
// for every vector store issued before it)
DQ_DEV void c_bounds(const CArgs& a, int wi, CBounds& bd) {
  if (wi >= a.n_work) return;
  using cu64 = const __attribute__((address_space(4))) uint64_t;
  using cu32 = const __attribute__((address_space(4))) uint32_t;
  bd.f = bd.fv = 0;
  if (a.entries) {
    cu32* e = (cu32*)(size_t)(a.entries + wi);
    bd.p = e[0];
    bd.f = e[1];
    bd.fv = e[2];
  } else {
    bd.p = (uint32_t)wi;
  }
  cu64* pb = (cu64*)(size_t)a.part_base;
  cu64* pe = (cu64*)(size_t)a.part_end;
  bd.r0 = pb[bd.p];
  bd.r1 = pe[bd.p];
}

// Work item wi (bounds bd): the raw words of its first kPF * kCThreads records.
template <bool HASHED, int CTH = kCThreads>
DQ_DEV void c_fetch(const CArgs& a, int wi, const CBounds& bd, CItem<HASHED>& it) {
  constexpr int W = FM<HASHED>::kRB / 8;
  it.valid = 0;
  if (wi >= a.n_work) return;
  it.p = bd.p;
  it.f = bd.f;
  it.fv = bd.fv;
  it.r0 = bd.r0;
  it.r1 = bd.r1;
  // (32-bit lane offsets: a partition's prefetch window is kPF * CTH records)
  const uint64_t n64 = it.r1 - it.r0;
  const uint32_t n = n64 < (uint64_t)kPF<HASHED> * CTH ? (uint32_t)n64 : (uint32_t)kPF<HASHED> * CTH;
  const uint64_t* src = reinterpret_cast<const uint64_t*>(a.recsB) + it.r0 * W;
#pragma unroll
  for (int q = 0; q < kPF<HASHED>; ++q) {
    const uint32_t li = (uint32_t)q * CTH + threadIdx.x;
#pragma unroll
    for (int k = 0; k < W; ++k) it.w[q][k] = 0;
    if (li < n) {
#pragma unroll
      for (int k = 0; k < W; ++k) it.w[q][k] = src[li * W + k];
      it.valid |= 1u << q;
    }
  }
}

// -(c/n) ln(c/n), out of line: the statistics pass calls it from every unrolled slot, and inlined
// copies of log() there made phase C several times larger than the instruction cache holds
__device__ __attribute__((noinline)) double entropy_term(uint64_t c, double n) {
  const double pr = (double)c / n;
  return -pr * log(pr);
}

// ---- Exact sums of fp64 terms (Entropy's -p ln p, MutualInformation's p ln(p / (px py))) ----
// A term enters as a signed 128-bit fixed-point integer at 2^-112 (exact for every term of
// magnitude >= 2^-60, cut below 2^-112), so a sum is the same integer in ANY order: the table's
// entropy is the sum of its groups' terms whatever the phase-C insert order, the partition depth,
// the recount subsets or the order partial sums meet in -- bit-stable from run to run.  Terms are
// bounded (|term| <= ln(rows) < 2^6), sums stay far inside 2^15.
using fix128 = __int128;
constexpr double kFixUlp = 0x1p-112;
DQ_HD fix128 fix_of(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const int ex = (int)((b >> 52) & 0x7ff);
  if (ex == 0) return 0;  // zero (and subnormals, < 2^-1022: cut)
  const uint64_t m = (b & ((1ULL << 52) - 1)) | (1ULL << 52);
  const int sh = ex - 1075 + 112;  // x = m 2^(ex - 1075); fixed = m 2^(ex - 1075 + 112)
  const fix128 v = sh >= 0 ? ((fix128)m << sh) : (sh > -64 ? (fix128)(m >> -sh) : (fix128)0);
  return (b >> 63) ? -v : v;
}
// (a fixed sequence of roundings: deterministic, within 2 ulp)
DQ_HD double fix_to_f64(fix128 v) {
  const int64_t hi = (int64_t)(v >> 64);
  const uint64_t lo = (uint64_t)v;
  return ((double)hi * 18446744073709551616.0 + (double)lo) * kFixUlp;
}
DQ_DEV fix128 wave_sum_fix(fix128 v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const uint64_t lo = __shfl_xor((unsigned long long)(uint64_t)v, o);
    const uint64_t hi = __shfl_xor((unsigned long long)(uint64_t)(v >> 64), o);
    v += (fix128)(((unsigned __int128)hi << 64) | lo);
  }
  return v;
}
// p[0..1] += v (lo, hi words): the carry of each lo add goes with that add's hi, so the total is
// exact whatever order the adds land in
DQ_DEV void atomic_add_fix(unsigned long long* p, fix128 v) {
  const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
  const uint64_t old = atomicAdd(p, (unsigned long long)lo);
  const uint64_t up = hi + (old + lo < old ? 1u : 0u);
  if (up) atomicAdd(p + 1, (unsigned long long)up);
}
DQ_DEV void store_fix(unsigned long long* p, fix128 v) {
  p[0] = (uint64_t)v;
  p[1] = (uint64_t)(v >> 64);
}

// Per work item: the inserts, then ONE pass over the LDS table that reads every slot once for
// the statistics, the Histogram candidates (kept in registers) and the lit probe, and clears it
// for the next item (when the groups are materialised, the output pass clears instead).  The
// flags and the special cell the inserts update are double-buffered by item parity, so they are
// reset for item i + 1 while item i runs, between two of its barriers: three barriers per item.
template <bool HASHED>
__global__ void __launch_bounds__(kCThreads, 4) freq_phaseC(CArgs a) {
  using M = FM<HASHED>;
  constexpr int KT = M::kTableC, W = M::kRB / 8, NW = kCThreads / 64;
  __shared__ uint64_t tkey[KT], tcnt[KT];
  __shared__ uint64_t trep[HASHED ? KT : 1];
  __shared__ uint32_t s_wg[NW], s_wc[NW];
  __shared__ uint64_t s_red[NW];
  __shared__ uint32_t s_ovf[2];
  __shared__ unsigned long long s_spec_cnt[2], s_gbase;
  __shared__ uint64_t s_spec_rep[2];
  __shared__ uint32_t s_chist[2][kSmallCounts];
  __shared__ unsigned long long s_efix[2][2];  // per item parity: the entropy, fixed point (lo, hi)
  // Histogram candidates: packed (count << 16 | tid << 2 | q) maxima, top-1 .. top-kCand
  __shared__ unsigned long long s_top[2][kCand];

  const int tid = threadIdx.x, lane = __lane_id(), wave = tid >> 6;
  unsigned long long collisions = 0;
  for (int i = tid; i < KT; i += kCThreads) {
    tkey[i] = kEmptyKey;
    tcnt[i] = 0;
    if (HASHED) trep[i] = kNotReady;
  }
  if (tid < 2) {
    s_ovf[tid] = 0;
    s_spec_cnt[tid] = 0;
    s_spec_rep[tid] = kNotReady;
#pragma unroll
    for (int r = 0; r < kCand; ++r) s_top[tid][r] = 0;
  }
  if (tid < 2 * kSmallCounts) (&s_chist[0][0])[tid] = 0;
  if (tid < 4) (&s_efix[0][0])[tid] = 0;
  // exact mode fetches records two items ahead: item i + 2's loads are in flight through all of
  // item i + 1 (one item's inserts and reduction are shorter than an HBM round trip under load).
  // Hashed mode has no registers for it and fetches one item ahead.
  constexpr int kAhead = HASHED ? 1 : 2;
  CBounds nb;
  CItem<HASHED> cur, nxt;
  c_bounds(a, blockIdx.x, nb);
  c_fetch<HASHED>(a, blockIdx.x, nb, cur);
  c_bounds(a, blockIdx.x + gridDim.x, nb);
  if constexpr (kAhead == 2) {
    c_fetch<HASHED>(a, blockIdx.x + gridDim.x, nb, nxt);
    c_bounds(a, blockIdx.x + 2 * gridDim.x, nb);
  }
  __syncthreads();

  uint32_t par = 0;
  int item = 0;
  auto mark = [&](int k) {
    if (a.dbg_clock && blockIdx.x == 0 && tid == 0 && item < 16)
      a.dbg_clock[item * 4 + k] = wall_clock64();
  };
  for (int wi = blockIdx.x; wi < a.n_work; wi += gridDim.x, par ^= 1u, ++item) {
    mark(0);
    const uint32_t p = cur.p, b = p >> a.s, f = cur.f, fv = cur.fv;
    const uint32_t fmask = (1u << f) - 1u;
    const uint64_t r0 = cur.r0, nrec = cur.r1 - cur.r0;
    uint32_t claims = 0;  // slots this thread claimed (load check after the inserts)
    uint32_t* ovf = &s_ovf[par];
    unsigned long long* spec_cnt = &s_spec_cnt[par];
    uint64_t* spec_rep = &s_spec_rep[par];

    // Returns false when the record must wait: its group's slot is claimed but the claimer has
    // not published the representative yet (hashed mode).  Waiting is a retry after the next
    // block barrier, never a spin, so lanes of one wave can never wait on each other.
    auto insert = [&](uint64_t h, uint64_t c, uint64_t rep) -> bool {
      if (h == kEmptyKey) {  // the table's empty marker: its own cell
        if constexpr (HASHED) {
          const uint64_t prev = atomicCAS((unsigned long long*)spec_rep, kNotReady, rep);
          if (prev != kNotReady && prev != rep &&
              !enc_equal_arena(reinterpret_cast<const uint32_t*>(a.arena + prev),
                         reinterpret_cast<const uint32_t*>(a.arena + rep), a.types, a.n_keys))
            ++collisions;
        }
        atomicAdd(spec_cnt, (unsigned long long)c);
        return true;
      }
      uint32_t slot = HASHED ? (uint32_t)(((uint64_t)(uint32_t)h * KT) >> 32) : ((uint32_t)h & (KT - 1));
      for (int probe = 0; probe < KT; ++probe) {
        // compare-and-swap first: it returns the slot's key, so a claim (most records of a
        // mostly-unique key) costs one LDS round trip instead of a load and then the swap
        const uint64_t k = atomicCAS((unsigned long long*)&tkey[slot], kEmptyKey, h);
        const bool claimed = k == kEmptyKey;
        if (claimed) {
          if (HASHED) lds_store(&trep[slot], rep);
          atomicAdd((unsigned long long*)&tcnt[slot], (unsigned long long)c);
          ++claims;
          return true;
        }
        if (k == h) {
          bool same = true;
          if constexpr (HASHED) {
            const uint64_t r2 = lds_load(&trep[slot]);
            if (r2 == kNotReady) return false;
            if (r2 != rep)
              same = enc_equal_arena(reinterpret_cast<const uint32_t*>(a.arena + r2),
                               reinterpret_cast<const uint32_t*>(a.arena + rep), a.types, a.n_keys);
            if (!same) ++collisions;  // two keys on one 64-bit hash: kept as two groups
          }
          if (same) {
            atomicAdd((unsigned long long*)&tcnt[slot], (unsigned long long)c);
            return true;
          }
        }
        if constexpr ((KT & (KT - 1)) == 0) slot = (slot + 1) & (KT - 1);
        else slot = slot + 1 == (uint32_t)KT ? 0u : slot + 1;
      }
      *ovf = 1;  // table full
      return true;
    };
    constexpr int PF = kPF<HASHED>;
    // decodes the valid records of w[PF][W] (raw words) and inserts those of this item's hash
    // subset; ends with a block barrier
    auto insert_all = [&](uint64_t (*w)[W], uint32_t valid) {
      uint32_t pending = 0;
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        if (!((valid >> q) & 1u)) continue;
        uint64_t h, c, rep;
        c_decode<HASHED>(w[q], b, h, c, rep);
        if (f == 0 || ((uint32_t)(h >> kFilterShift) & fmask) == fv) pending |= 1u << q;
      }
      if constexpr (HASHED) {
        while (__syncthreads_or(pending ? 1 : 0)) {
#pragma unroll
          for (int q = 0; q < PF; ++q) {
            if (!((pending >> q) & 1u)) continue;
            uint64_t h, c, rep;
            c_decode<HASHED>(w[q], b, h, c, rep);
            if (insert(h, c, rep)) pending &= ~(1u << q);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < PF; ++q) {
          if (!((pending >> q) & 1u)) continue;
          uint64_t h, c, rep;
          c_decode<HASHED>(w[q], b, h, c, rep);
          insert(h, c, rep);
        }
        __syncthreads();
      }
    };
    // the prefetched first records, then the rest of a long partition            [barrier 1]
    insert_all(cur.w, cur.valid);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(a.recsB) + r0 * W;
    for (uint64_t base = (uint64_t)PF * kCThreads; base < nrec; base += (uint64_t)PF * kCThreads) {
      uint64_t w[PF][W];
      uint32_t valid = 0;
      const bool go = !*ovf;
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const uint64_t li = base + (uint64_t)q * kCThreads + tid;
#pragma unroll
        for (int k = 0; k < W; ++k) w[q][k] = 0;
        if (li < nrec && go) {
#pragma unroll
          for (int k = 0; k < W; ++k) w[q][k] = src[li * W + k];
          valid |= 1u << q;
        }
      }
      insert_all(w, valid);
    }
    mark(1);
    // the table is final.  Next item's records (bounds already here) and the bounds after it are
    // in flight while this one is reduced; the other parity's flags are reset for it.
    if constexpr (kAhead == 2) {
      cur = nxt;
      c_fetch<HASHED>(a, wi + 2 * gridDim.x, nb, nxt);
      c_bounds(a, wi + 3 * gridDim.x, nb);
    } else {
      c_fetch<HASHED>(a, wi + gridDim.x, nb, cur);
      c_bounds(a, wi + 2 * gridDim.x, nb);
    }
    if (tid == 0) {
      s_ovf[par ^ 1u] = 0;
      s_spec_cnt[par ^ 1u] = 0;
      s_spec_rep[par ^ 1u] = kNotReady;
#pragma unroll
      for (int r = 0; r < kCand; ++r) s_top[par ^ 1u][r] = 0;
    }
    if (tid < kSmallCounts) s_chist[par ^ 1u][tid] = 0;
    if (tid < 2) s_efix[par ^ 1u][tid] = 0;
    const bool overflow = *ovf != 0;
    const uint64_t sc = *spec_cnt, sr = HASHED ? *spec_rep : 0;

    // statistics: -p ln p depends on the count alone, so small counts are histogrammed and each
    // distinct one takes ONE log (unique keys: one per partition)
    const bool keep = a.groups != nullptr;  // the output pass reads the table, then clears it
    const bool cand = a.want_cand && f == 0;
    uint32_t g = 0;
    uint64_t un = 0;
    uint64_t tc[kCand], tk[kCand], tr[kCand];
#pragma unroll
    for (int q = 0; q < kCand; ++q) tc[q] = tk[q] = tr[q] = 0;
    auto term = [&](uint64_t c) { return fix_of(entropy_term(c, a.num_rows)); };
    auto count_group = [&](uint64_t c) {
      ++g;
      if (c == 1) ++un;  // the common count: a register, not an LDS atomic on one address
      else if (c < kSmallCounts) atomicAdd(&s_chist[par][c], 1u);
      else atomic_add_fix(&s_efix[par][0], term(c));  // (rare: fixed point, any order)
    };
    auto offer = [&](uint64_t c, uint64_t k, uint64_t r) {  // insertion, static indices
#pragma unroll
      for (int q = 0; q < kCand; ++q) {
        if (c > tc[q]) {
          const uint64_t c2 = tc[q], k2 = tk[q], r2 = tr[q];
          tc[q] = c;
          tk[q] = k;
          tr[q] = r;
          c = c2;
          k = k2;
          r = r2;
        }
      }
    };
#pragma unroll
    for (int sl = tid; sl < KT; sl += kCThreads) {
      const uint64_t k = tkey[sl];
      if (k == kEmptyKey) continue;
      const uint64_t c = tcnt[sl];
      const uint64_t r = HASHED ? trep[sl] : 0;
      if (!keep) {
        tkey[sl] = kEmptyKey;
        tcnt[sl] = 0;
        if (HASHED) trep[sl] = kNotReady;
      }
      if (overflow) continue;
      if constexpr (HASHED)
        if (a.lit_count && k == a.lit_h && enc_is_null_literal(a.arena + r))
          atomicAdd(a.lit_count, (unsigned long long)c);
      count_group(c);
      // (a branch, not selects: with mostly-unique keys nearly every slot fails the first test)
      if (cand && c > tc[kCand - 1]) offer(c, k, r);
    }
    if (tid == 0 && sc && !overflow) {
      count_group(sc);
      if (cand) offer(sc, kEmptyKey, sr);
    }
    const uint32_t gin = __ockl_wfscan_add_u32(g, true);  // inclusive prefix over the wave
    const uint32_t wclaims = __ockl_wfred_add_u32(claims);
    const uint64_t wun = __ockl_wfred_add_u64(un);
    if (lane == 63) {
      s_wg[wave] = gin;
      s_wc[wave] = wclaims;
      s_red[wave] = wun;
    }
    // Histogram candidates, round 1: the block's largest (count, tid, q)
    static_assert(kCThreads <= 1024 && kCand <= 4, "candidate packing: tid in 10 bits, q in 2");
    auto pack = [&](int q) -> uint64_t {
      uint64_t c = 0;
#pragma unroll
      for (int i = 0; i < kCand; ++i) c = i == q ? tc[i] : c;
      return c ? (c << 16) | ((uint64_t)tid << 2) | (uint64_t)q : 0ULL;
    };
    int taken = 0;  // this thread's candidates already placed (they leave in count order)
    if (cand) {
      const uint64_t w1 = __ockl_wfred_max_u64(pack(0));
      if (lane == 0 && w1) atomicMax(&s_top[par][0], (unsigned long long)w1);
    }
    __syncthreads();  //                                                            [barrier 2]
    mark(2);
    uint32_t gtot = 0, gex = gin - g, all_claims = 0;
    uint64_t utot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      gtot += s_wg[w];
      if (w < wave) gex += s_wg[w];
      all_claims += s_wc[w];
      utot += s_red[w];
    }
    if (overflow || all_claims > (uint32_t)(KT * 7 / 8)) {  // too full: recount (block-uniform)
      if (tid == 0) {
        const unsigned int q = atomicAdd(a.ovf_n, 2u);
        a.ovf_out[q] = FEntry{p, f + 1, fv, 0};
        a.ovf_out[q + 1] = FEntry{p, f + 1, fv | (1u << f), 0};
      }
      if (keep) {  // the output pass would have cleared the table
        for (int sl = tid; sl < KT; sl += kCThreads) {
          tkey[sl] = kEmptyKey;
          tcnt[sl] = 0;
          if (HASHED) trep[sl] = kNotReady;
        }
        __syncthreads();
      }
      continue;
    }
    if (tid > 1 && tid < kSmallCounts && s_chist[par][tid])
      atomic_add_fix(&s_efix[par][0], term(tid) * (fix128)s_chist[par][tid]);
    if (tid == 0 && utot) atomic_add_fix(&s_efix[par][0], term(1) * (fix128)utot);
    if (cand) {  // round 2: the largest of the rest (the top-1 owner offers its second)
      const uint64_t top1 = s_top[par][0];
      taken = top1 && top1 == pack(0) ? 1 : 0;
      const uint64_t w2 = __ockl_wfred_max_u64(pack(taken));
      if (lane == 0 && w2) atomicMax(&s_top[par][1], (unsigned long long)w2);
    }
    const bool sub = f != 0;  // a recount subset: several work items add to one partition
    if (tid == 0 && keep) {
      a.part_off[p] = r0;
      s_gbase = sub ? atomicAdd(&a.part_groups[p], (unsigned long long)gtot) : 0ULL;
    }
    __syncthreads();  //                                                            [barrier 3]
    mark(3);
    if (tid == 0) {
      const fix128 etot = (fix128)(((unsigned __int128)s_efix[par][1] << 64) | s_efix[par][0]);
      if (!keep || !sub) {
        if (sub) atomicAdd(&a.part_groups[p], (unsigned long long)gtot);
        else a.part_groups[p] = gtot;
      }
      if (sub) {
        if (utot) atomicAdd(&a.part_unique[p], (unsigned long long)utot);
        if (etot) atomic_add_fix(&a.part_entropy[2 * (uint64_t)p], etot);
      } else {
        a.part_unique[p] = utot;
        store_fix(&a.part_entropy[2 * (uint64_t)p], etot);
      }
    }
    if (cand) {
      // rounds 3 .. kCand (their own barriers; cand is block-uniform): the winner of each round
      // advances past the candidate it placed.  Skipped when the second candidate's count is at
      // most 1 (every later one is too: mostly-unique keys pay no extra barriers); the check
      // (freq_cand_check) then sees two filled places.
      const bool more_rounds = (s_top[par][1] >> 16) > 1;
#pragma unroll
      for (int r = 2; r < kCand && more_rounds; ++r) {
        const uint64_t prev = s_top[par][r - 1];
        if (prev && prev == pack(taken)) ++taken;
        const uint64_t w = __ockl_wfred_max_u64(pack(taken));
        if (lane == 0 && w) atomicMax(&s_top[par][r], (unsigned long long)w);
        __syncthreads();
      }
      // each winner's owner writes it; an empty place is written by thread 0
#pragma unroll
      for (int r = 0; r < kCand; ++r) {
        const uint64_t t = s_top[par][r];
        Group* cslot = a.cand + (uint64_t)p * kCand + r;
        if (!t) {
          if (tid == 0) *cslot = Group{0, 0, 0};
        } else if ((int)((t >> 2) & 1023u) == tid) {
          const int q = (int)(t & 3u);
          uint64_t gk = 0, gc = 0, gr = 0;
#pragma unroll
          for (int i = 0; i < kCand; ++i) {
            gk = i == q ? tk[i] : gk;
            gc = i == q ? tc[i] : gc;
            gr = i == q ? tr[i] : gr;
          }
          *cslot = Group{gk, gc, HASHED ? gr : 0};
        }
      }
    }
    if (keep) {  // materialise the groups, clearing the table
      Group* out = a.groups + r0 + s_gbase + gex;
      uint32_t q = 0;
      for (int sl = tid; sl < KT; sl += kCThreads) {
        const uint64_t k = tkey[sl];
        if (k == kEmptyKey) continue;
        out[q++] = Group{k, tcnt[sl], HASHED ? trep[sl] : 0};
        tkey[sl] = kEmptyKey;
        tcnt[sl] = 0;
        if (HASHED) trep[sl] = kNotReady;
      }
      if (tid == 0 && sc) out[q++] = Group{kEmptyKey, sc, HASHED ? sr : 0};
      __syncthreads();
    }
  }
  if (collisions) atomicAdd(&a.counters[C_COLLISIONS], collisions);
}

// ------------------------------------------------------------------------------------------------
// Phase C, exact mode (one fixed-width key: the hash is the key, no arena, no representative).
//
// The generic kernel above spends most of its issue slots on per-partition work that does not
// depend on the records: a pass over all kTableC slots (empty ones included), a 4-deep candidate
// insertion per occupied slot, three barriers.  Here every claim appends its slot to an LDS list
// (one LDS atomic per wave and insert round), so the statistics pass visits the partition's groups
// only, and the work per partition is:
//   inserts: the first probe of all of a thread's records in flight together (linear probing
//            after that);                                                        [barrier 1]
//   stats:   over the list -- Σ[c==1] in a register, counts 2..63 into an LDS histogram (one log
//            per distinct count), larger counts' terms summed; each slot is cleared as it is read;
//            Histogram candidates: the first kCand groups of the list, plus a per-lane top-kCand of
//            the groups with count > 1;                                          [barrier 2]
// and the partition's statistics and candidates are written by wave 0 during the NEXT item, right
// after that item's loads are issued.  (Global stores count in vmcnt like loads, so a store issued
// at the end of an item made the next item's wait for its prefetched records a wait for the store
// too: a full store round trip per item.  Every vector-memory operation of an item is now issued
// at its start, one item before anything waits for it.)
// Only when a partition's largest count exceeds 1 AND Histogram wants candidates do kCand more
// rounds (with barriers) pick its exact top kCand; a mostly-unique key never takes them.
// Entropy stays deterministic: count-1 groups are counted, counts < kSmallCounts histogrammed, and
// the partials are added in a fixed order.  Same outputs as freq_phaseC<false>.
// DBG: DQ_FREQ_DEBUG=2's instantiation, workgroup 0 stamps each item's phases (wall clock).
// ------------------------------------------------------------------------------------------------
// PK: packed slots, for tables partitioned at least kMinPkSubBits deep (a partition then fixes the
// top kBucketBits + s >= 16 hash bits): one u64 per slot = count << KB | the key's low KB = 55 - s
// hash bits, so a claim installs key AND count in one CAS, a duplicate adds count << KB, and the
// table holds 8192 slots in the LDS of 4096 two-word slots (load ~0.22 instead of ~0.44: fewer
// probe rounds, the wave's longest probe sequence bounding every round).  A count field of 9 + s
// bits can only overflow when some record carries a count >= 2^(s-3) (128 at s = 10) or the
// partition has more than 4096 records; such an item is handed on (an ovf entry of the whole
// partition, f = 0) to the two-word kernel.  (s = 7..9: the configs[4]-sized tables.)
template <bool DBG, bool PK, bool BIG = false>
__global__ void __launch_bounds__(kCThreadsX<PK && BIG>, 4) freq_phaseC_x(CArgs a) {
  // PK && BIG (partitions of more than 2048 records on average: configs[2]'s 1e9-row keys): one
  // 1024-thread workgroup per CU over a 16384-slot table (128 KB of LDS), so an item of up to 4096
  // records is inserted in ONE round at a load factor <= 1/4.  The probe rounds are a chain of LDS
  // atomic round trips (~600 cycles each under load: tools/micro/lds_insert_bench), and a round
  // takes as many as its wave's longest probe sequence -- two rounds at up to 44 % load took ~11
  // of them per item, one round at <= 25 % takes ~4.  Smaller partitions (configs[4]'s 1.25e8
  // rows: ~1,800 records) keep two 512-thread workgroups per CU over 8192 slots, one round each:
  // there the 1024-thread form ran 1.73 against 1.05 ms per table (profiles/r6p vs r5zi), its
  // per-item costs spread over half the records.
  constexpr int CT = kCThreadsX<PK && BIG>;
  constexpr int KT = PK ? (BIG ? 16384 : 8192) : FM<false>::kTableC, NW = CT / 64, PF = kPF<false>;
  // list capacity = most records of a packed item: two insert rounds of PF * CT, the table then
  // at most half full.  (Items of ~7,300 records -- kTargetPk 7400, one level shallower -- ran
  // phase C in the same time as ~3,600 in one round, 6.46 ms both, profiles/r6n: half the items'
  // fixed costs against longer probe chains at twice the load; ~1,800 took 9.2 ms, r6l.)
  constexpr int KL = PK ? 2 * PF * CT : KT;
  // PK: the partition fixes the hash's top 9 + s bits, the slot keeps the other KB = 55 - s
  // (45..48 for s = 10..7) under a count field of 9 + s bits
  const int KB = 55 - (int)a.s;
  const uint64_t MK = (1ULL << KB) - 1;
  const uint64_t cmax = 1ULL << (a.s > 3 ? a.s - 3 : 0);  // record counts below this: no overflow
  __shared__ uint64_t tkey[KT], tcnt[PK ? 1 : KT];
  __shared__ uint16_t list[KL];
  __shared__ uint32_t s_n[2], s_ovf[2];
  __shared__ unsigned long long s_spec[2];
  __shared__ uint32_t s_chist[2][kSmallCounts];
  __shared__ unsigned long long s_efix[2][2];  // per item parity: the entropy, fixed point (lo, hi)
  __shared__ unsigned long long s_wun[2][NW], s_wmax[2][NW];
  __shared__ double s_term[kSmallCounts];
  // each wave's top kCand groups of the item (count 0: none), merged by the next item's tail
  __shared__ uint64_t s_wk[2][NW][kCand], s_wc[2][NW][kCand];
  __shared__ unsigned long long s_gbase;
  // an item's outputs, written during the next item: partition, first group slot, #groups, flags
  __shared__ uint32_t s_tp[2], s_tg[2], s_tfl[2];
  __shared__ uint64_t s_tr0[2];
  enum { TF_VALID = 1, TF_SUB = 2, TF_CANDFAST = 4, TF_CANDONE = 8 };

  const int tid = threadIdx.x, lane = __lane_id(), wave = tid >> 6;
  for (int i = tid; i < KT; i += CT) {
    tkey[i] = kEmptyKey;
    if (!PK) tcnt[i] = 0;
  }
  if (tid < 2) {
    s_n[tid] = 0;
    s_ovf[tid] = 0;
    s_spec[tid] = 0;
    s_tfl[tid] = 0;
  }
  if (tid < 2 * kSmallCounts) (&s_chist[0][0])[tid] = 0;
  if (tid < 4) (&s_efix[0][0])[tid] = 0;
  if (tid < kSmallCounts) s_term[tid] = tid ? entropy_term((uint64_t)tid, a.num_rows) : 0.0;
  const bool keep = a.groups != nullptr;
  // (a scan of the whole table instead of the list of claimed slots -- 16 slots per thread,
  // conflict-free 16-byte reads, no list appends -- measured slower: statistics 3.5 against
  // 2.0 us per item, profiles/r6j; kept off)
  constexpr bool scan_stats = false;
  __shared__ uint32_t s_wgn[2][NW];  // scan_stats: each wave's groups of the item

  // Wave 0: the statistics and candidates of the item of parity q (its words stay untouched until
  // the item after next resets them, behind that item's barrier 1).
  // (wv 1 merges the candidates while wv 0 writes the statistics: neither holds up the inserts
  // that wait at barrier 1 for the slowest wave)
  auto tail = [&](uint32_t q, int wv) {
    // (wave-uniform words: scalars, so the candidates' addresses take no VGPRs)
    const uint32_t fl = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tfl[q]);
    if (!(fl & TF_VALID)) return;
    const uint32_t p = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tp[q]);
    uint32_t gtot = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tg[q]);
    if (scan_stats) {
#pragma unroll
      for (int w = 0; w < NW; ++w) gtot += s_wgn[q][w];
    }
    const bool sub = (fl & TF_SUB) != 0;
    if ((fl & TF_CANDFAST) && wv == 1) {  // the item's top kCand: rounds of wave maxima over the waves' lists
      static_assert(NW * kCand <= 64, "one wave merges the lists");
      const bool in = lane < NW * kCand;
      const int w = in ? lane / kCand : 0, r = lane % kCand;
      const uint64_t c = in ? s_wc[q][w][r] : 0;
      if (fl & TF_CANDONE) {  // every count is 1: the first kCand candidates
        const uint64_t bal = __ballot(c != 0);
        const uint32_t rank = (uint32_t)__builtin_popcountll(bal & ((1ULL << lane) - 1ULL));
        if (c && rank < (uint32_t)kCand)
          a.cand[(uint64_t)p * kCand + rank] = Group{s_wk[q][w][r], c, 0};
        if (lane < kCand && (uint32_t)lane >= (uint32_t)__builtin_popcountll(bal))
          a.cand[(uint64_t)p * kCand + lane] = Group{0, 0, 0};
      } else {
        uint64_t mine = c ? (c << 8) | (uint64_t)(63 - lane) : 0ULL;  // ties: the lower lane
#pragma unroll
        for (int k = 0; k < kCand; ++k) {
          const uint64_t wm = __ockl_wfred_max_u64(mine);
          if (wm && wm == mine) {
            a.cand[(uint64_t)p * kCand + k] = Group{s_wk[q][w][r], c, 0};
            mine = 0;
          } else if (!wm && lane == 0) {
            a.cand[(uint64_t)p * kCand + k] = Group{0, 0, 0};
          }
        }
      }
    }
    if (wv != 0) return;
    const uint32_t hc = lane > 1 ? s_chist[q][lane] : 0u;
    // counts 2..63 join the item's LDS sum (this wave's LDS operations complete in order, so
    // lane 0 reads it after every lane's add)
    if (hc) atomic_add_fix(&s_efix[q][0], fix_of(s_term[lane]) * (fix128)hc);
    if (lane == 0) {
      uint64_t utot = 0;
      fix128 etot = (fix128)(((unsigned __int128)s_efix[q][1] << 64) | s_efix[q][0]);
#pragma unroll
      for (int w = 0; w < NW; ++w) utot += s_wun[q][w];
      if (utot) etot += fix_of(s_term[1]) * (fix128)utot;
      if (sub) {
        if (!keep) atomicAdd(&a.part_groups[p], (unsigned long long)gtot);
        if (utot) atomicAdd(&a.part_unique[p], (unsigned long long)utot);
        if (etot) atomic_add_fix(&a.part_entropy[2 * (uint64_t)p], etot);
      } else {
        a.part_groups[p] = gtot;
        a.part_unique[p] = utot;
        store_fix(&a.part_entropy[2 * (uint64_t)p], etot);
      }
      if (keep) a.part_off[p] = s_tr0[q];
    }
  };

  // Bounds ring (a.bcache, the first pass): this workgroup's items t's record ranges (32-bit start,
  // count) at ring[t % 512], filled 256 items at a time, 256 items ahead (one load per thread and
  // one exposed round trip per 256 items).  A scalar load of the bounds of item i + 2 per item was
  // waited for by the item's first LDS wait (s_waitcnt lgkmcnt(0) covers SMEM loads too): one HBM
  // round trip per item exposed in its CAS rounds.
  // this workgroup's item t -> work item (a.n_work: none).  Contiguous items (a.contig) walk the
  // records region in order (one page run per workgroup), strided ones jump P / grid partitions.
  const int ipw = a.contig ? (a.n_work + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  auto wmap = [&](int t) -> int {
    if (ipw) {
      const int w = (int)blockIdx.x * ipw + t;
      return t < ipw && w < a.n_work ? w : a.n_work;
    }
    return (int)blockIdx.x + t * (int)gridDim.x;
  };
  constexpr int kRing = 512;
  __shared__ uint32_t ring_r0[kRing], ring_n[kRing];
  const bool bcache = a.bcache != 0 && a.entries == nullptr;  // (block-uniform)
  auto bfill = [&](int t0, int cnt) {  // items [t0, t0 + cnt), one per thread (cnt <= CT)
    if (tid < cnt) {
      const int64_t w = wmap(t0 + tid);
      uint32_t r0v = 0, nv = 0;
      if (w < a.n_work) {
        const uint64_t x0 = a.part_base[w], x1 = a.part_end[w];
        r0v = (uint32_t)x0;
        nv = (uint32_t)(x1 - x0);
      }
      ring_r0[(t0 + tid) & (kRing - 1)] = r0v;
      ring_n[(t0 + tid) & (kRing - 1)] = nv;
    }
  };
  auto bget = [&](int t, CBounds& bd) {  // this workgroup's item t (in the ring)
    const int64_t w = wmap(t);
    if (w >= a.n_work) return;
    bd.p = (uint32_t)w;
    bd.f = bd.fv = 0;
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ring_r0[t & (kRing - 1)]);
    const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)ring_n[t & (kRing - 1)]);
    bd.r0 = r0;
    bd.r1 = (uint64_t)r0 + n;
  };

  // One item ahead, issued at the top of an item and taken over at its end: the records of item
  // i + 1 and the bounds of item i + 2 are in flight through all of item i.
  CBounds nb;
  CItem<false> cur;
  if (bcache) {
    bfill(0, CT < kRing ? CT : kRing);
    __syncthreads();
    bget(0, nb);
  } else {
    c_bounds(a, wmap(0), nb);
  }
  c_fetch<false, CT>(a, wmap(0), nb, cur);
  if (bcache) bget(1, nb);
  else c_bounds(a, wmap(1), nb);
  __syncthreads();

  uint32_t par = 0;
  int item = 0;
  auto mark = [&](int kk) {
    if constexpr (DBG)
      if (blockIdx.x == 0 && tid == 0 && item < 16) a.dbg_clock[item * 8 + kk] = wall_clock64();
  };
  for (int wi = wmap(0); wi < a.n_work; par ^= 1u, ++item, wi = wmap(item)) {
    mark(0);
    const uint32_t p = cur.p, b = p >> a.s, f = cur.f, fv = cur.fv;
    const uint32_t fmask = (1u << f) - 1u;
    const uint64_t r0 = cur.r0, nrec = cur.r1 - cur.r0;
    CItem<false> pf;
    CBounds nb2;

    // Decodes one round of (at most PF) raw records per thread, then inserts them and appends the
    // claimed slots to the list.  Every thread calls it (the list append is wave-aggregated).
    // `issue` runs between the two, behind scheduling barriers: the first round issues the next
    // item's loads and the last item's stores there, after the only wait for this item's words.
    auto insert_round = [&](const uint64_t (*w)[1], uint32_t valid, auto&& issue) {
      uint64_t h[PF], c[PF], old[PF];
      uint32_t slot[PF], todo = 0;
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        h[q] = xrec_h(w[q][0], b);
        c[q] = code_count((uint32_t)(w[q][0] & 0xff));
        slot[q] = (uint32_t)h[q] & (KT - 1);
        const bool in = ((valid >> q) & 1u) && (f == 0 || ((uint32_t)(h[q] >> kFilterShift) & fmask) == fv);
        if constexpr (PK) {
          if (in && c[q] >= cmax) s_ovf[par] = 1;  // a count field could overflow: hand it on
          if (in) todo |= 1u << q;
          h[q] = (c[q] << KB) | (h[q] & MK);  // the packed word
        } else {
          if (in && h[q] == kEmptyKey) atomicAdd(&s_spec[par], (unsigned long long)c[q]);
          else if (in) todo |= 1u << q;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      mark(4);
      issue();
      mark(5);
      __builtin_amdgcn_sched_barrier(0);
      // Probe rounds with every pending record's CAS in flight together (a wave takes as many
      // rounds as its longest probe sequence, not the sum over its records); double hashing (an
      // odd step from high hash bits) keeps those sequences short.
      // (PK: the step comes from key bits 30..43 of the packed word -- bits 45 and up may be the
      // count (KB = 55 - s >= 45), and records of one key with different counts must walk the
      // same sequence; the slot is bits 0..13)
      uint32_t step[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) step[q] = ((uint32_t)(h[q] >> (PK ? 30 : 40)) | 1u) & (KT - 1);
      uint32_t mine = 0;
#if DQ_C_EXPERIMENT & 2  // (timing experiment only: no inserts)
      todo = 0;
#endif
      if constexpr (PK && DQ_LEAN_PROBE) {
        // One CAS instruction per probe round: each lane works on its next pending record, so a
        // round is a full-width LDS atomic while the wave's records last, instead of PF
        // instructions whose lanes thin out to the longest probe sequence.  The CAS instructions,
        // not the lanes in them, set an LDS atomic round trip (16 waves queue theirs), and a
        // wave's chain of round trips sets the insert phase (tools/micro/lds_insert_bench).
        // The lane's records move through a shift register (a PK first pass has no hash filter,
        // so its pending records are a prefix of the PF); the slots it claims go to cl[0..ncl)
        // (then to the list below, as `mine` bits 0..ncl-1 over slot[]).
        // (a record's slot, step and count add all come from its packed word: slot = bits 0..13,
        // step = bits 30..43 | 1, add = the count field -- only the words ride the shift register)
        uint64_t ch = h[0];
        uint32_t cs = (uint32_t)ch & (KT - 1), cst = ((uint32_t)(ch >> 30) | 1u) & (KT - 1);
        uint32_t rest = todo >> 1, ncl = 0, cl[PF];
#pragma unroll
        for (int x = 0; x < PF; ++x) cl[x] = 0;
        bool act = (todo & 1u) != 0;
        for (int pr = 0; act && pr < 4 * KT; ++pr) {
          const uint64_t o = atomicCAS((unsigned long long*)&tkey[cs], kEmptyKey, ch);
          const bool e = o == kEmptyKey;
          const bool m = !e && ((o ^ ch) & MK) == 0;
          if (m) atomicAdd((unsigned long long*)&tkey[cs], (unsigned long long)(ch & ~MK));
          if (e || m) {
            if (e) {
#pragma unroll
              for (int x = 0; x < PF; ++x) cl[x] = (uint32_t)x == ncl ? cs : cl[x];
              ++ncl;
            }
            act = (rest & 1u) != 0;
            rest >>= 1;
            ch = h[1];
            cs = (uint32_t)ch & (KT - 1);
            cst = ((uint32_t)(ch >> 30) | 1u) & (KT - 1);
#pragma unroll
            for (int x = 1; x + 1 < PF; ++x) h[x] = h[x + 1];
          } else {
            cs = (cs + cst) & (KT - 1);
          }
        }
        todo = act ? 1u : 0u;  // (a record still pending: the table is full)
        mine = (1u << ncl) - 1u;
#pragma unroll
        for (int x = 0; x < PF; ++x) slot[x] = cl[x];
      } else {  // (PF records per lane in flight together; -DDQ_LEAN_PROBE=0: also for PK)
        // (a branch-light form of these rounds -- outcomes as bit masks, slots advanced with
        // selects -- measured no faster, profiles/r6g, and spilled the two-word kernel)
        for (int pr = 0; todo && pr < KT; ++pr) {
#pragma unroll
          for (int q = 0; q < PF; ++q)
            old[q] = (todo >> q) & 1u ? atomicCAS((unsigned long long*)&tkey[slot[q]], kEmptyKey, h[q]) : 0ULL;
#pragma unroll
          for (int q = 0; q < PF; ++q) {
            if (!((todo >> q) & 1u)) continue;
            const bool claimed = old[q] == kEmptyKey;
            const bool match = PK ? ((old[q] ^ h[q]) & MK) == 0 : old[q] == h[q];
            if (claimed || match) {
              if constexpr (PK) {
                if (!claimed) atomicAdd((unsigned long long*)&tkey[slot[q]], (unsigned long long)(c[q] << KB));
              } else {
                atomicAdd((unsigned long long*)&tcnt[slot[q]], (unsigned long long)c[q]);
              }
              if (claimed) mine |= 1u << q;
              todo &= ~(1u << q);
            } else {
              slot[q] = (slot[q] + step[q]) & (KT - 1);
            }
          }
        }
      }
      if (todo) s_ovf[par] = 1;  // the table is full
      if (scan_stats) mine = 0;  // (no list: the statistics scan the table)
      const uint32_t nm = (uint32_t)__builtin_popcount(mine);
      const uint32_t incl = __ockl_wfscan_add_u32(nm, true);
      const uint32_t wtot = __builtin_amdgcn_readlane(incl, 63);
      if (wtot) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&s_n[par], wtot);
        uint32_t pos = __builtin_amdgcn_readlane(base, 0) + incl - nm;
#pragma unroll
        for (int q = 0; q < PF; ++q)
          if ((mine >> q) & 1u) list[pos++] = (uint16_t)slot[q];
      }
      mark(6);
    };
    // the ring's other half: items [item + 256, item + 512), read from item + 254 on (barriers
    // between); the half it replaces held items before this one
    if (bcache && item > 0 && (item & (kRing / 2 - 1)) == 0) bfill(item + kRing / 2, kRing / 2);
    const bool too_long = PK && nrec > (uint64_t)KL;  // (handed on whole, see `overflow`)
    // The rest of a long partition (packed items hold up to 2 * PF * CT records; a column
    // of heavy values puts every workgroup's records of a heavy key in one partition): the first
    // round's issue slot loads this item's second round of words, and the LAST round's issue slot
    // prefetches the next item -- so neither is an exposed HBM round trip, and at most one round of
    // words is in flight beside the round being inserted (VGPRs: the kernel sits at 128).
    constexpr uint64_t STEP = (uint64_t)PF * CT;
    const bool rest = nrec > STEP && !too_long;
    // (the rounds' words travel in pf's registers: the next item's prefetch goes out last, and a
    // second buffer, live where the two paths join, spilled the kernel)
    auto load = [&](uint64_t base) {  // (32-bit offsets inside the round)
      const uint64_t* src = reinterpret_cast<const uint64_t*>(a.recsB) + r0 + base;
      const uint64_t left = nrec - base;
      const uint32_t m = left < STEP ? (uint32_t)left : (uint32_t)STEP;
      pf.valid = 0;
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const uint32_t li = (uint32_t)q * CT + tid;
        pf.w[q][0] = li < m ? src[li] : 0ULL;
        pf.valid |= (li < m ? 1u : 0u) << q;
      }
    };
    auto issue_next = [&]() {
      if (bcache) bget(item + 2, nb2);
      c_fetch<false, CT>(a, wmap(item + 1), nb, pf);
      if (!bcache) c_bounds(a, wmap(item + 2), nb2);
    };
    // One insert round per STEP records, all through ONE inlined insert_round (two copies, the
    // first round and the rest, spilled the kernel): each round's issue slot loads the next round's
    // words into pf, or -- in the last round -- prefetches the next item there.
    {
      uint32_t valid = too_long ? 0u : cur.valid;
      for (uint64_t base = 0;; base += STEP) {
        const bool last = !rest || base + STEP >= nrec;
        insert_round(cur.w, valid, [&]() {
          if (last) issue_next();
          else load(base + STEP);
        });
        if (last) break;
#pragma unroll
        for (int q = 0; q < PF; ++q) cur.w[q][0] = pf.w[q][0];  // (cur's words are dead after decode)
        valid = pf.valid;
      }
    }
    // the last item's outputs, after this wave's inserts (its records are no longer live; the
    // stores come after the prefetch, so the next item's wait for its records leaves them be)
    if (wave < 2) tail(par ^ 1u, wave);
    __syncthreads();  //                                                            [barrier 1]
    mark(1);
    const uint32_t n = s_n[par];
    const uint64_t sc = s_spec[par];
    // PK: any count field at risk, or a partition longer than the list: the two-word kernel
    const bool overflow = s_ovf[par] != 0 || (!scan_stats && n > (uint32_t)(KT * 7 / 8)) ||
                          (PK && nrec > (uint64_t)KL);
    const bool sub = f != 0;  // a recount subset: several work items add to one partition
    const bool cand = a.want_cand && f == 0 && !overflow;
    // the other parity's words, for item + 1 (the last item's tail has read them)
    if (tid == 0) {
      s_n[par ^ 1u] = 0;
      s_ovf[par ^ 1u] = 0;
      s_spec[par ^ 1u] = 0;
      s_tfl[par ^ 1u] = 0;
    }
    if (tid < kSmallCounts) s_chist[par ^ 1u][tid] = 0;
    if (tid < 2) s_efix[par ^ 1u][tid] = 0;
    const uint32_t gtot = n + (sc ? 1u : 0u);
    uint64_t gbase = 0;
    if (keep && sub && !overflow) {  // block-uniform
      if (tid == 0) s_gbase = atomicAdd(&a.part_groups[p], (unsigned long long)gtot);
      __syncthreads();
      gbase = s_gbase;
    }
    const uint64_t obase = a.group_stride ? (uint64_t)wi * a.group_stride : r0 + gbase;

    // statistics over the list, clearing the table.  Per group: a count-1 test and a 32-bit
    // count; counts above 1 (rare in a high-cardinality key) take the branch with the histogram,
    // the entropy term and the candidate insertion; a PK key is rebuilt from its packed word only
    // where it is kept (materialised groups, candidates)
    uint32_t un = 0;
    bool gt1 = false;  // some count of this lane's groups exceeds 1
    uint64_t tc[kCand], tk[kCand];  // this lane's top groups with count > 1
#pragma unroll
    for (int q = 0; q < kCand; ++q) tc[q] = tk[q] = 0;
    uint64_t k1 = 0;  // a count-1 group of this lane (k1c: present; PK: its packed word)
    bool k1c = false;
    // k: the key, or (PK) the packed slot word, rebuilt by key_of
    auto key_of = [&](uint64_t k) -> uint64_t { return PK ? (((uint64_t)p << KB) | (k & MK)) : k; };
    auto stat = [&](uint32_t i, uint64_t k, uint64_t c) {
#if DQ_C_EXPERIMENT & 1  // (timing experiment only: no statistics)
      return;
#endif
      if (keep) a.groups[obase + i] = Group{key_of(k), c, 0};
      if (c == 1) {
        ++un;
        if (cand && !k1c) k1 = k;
        k1c = true;
      } else {
        gt1 = true;
        if (c < kSmallCounts) atomicAdd(&s_chist[par][c], 1u);
        else atomic_add_fix(&s_efix[par][0], fix_of(entropy_term(c, a.num_rows)));  // (rare)
        if (cand && c > tc[kCand - 1]) {
          k = key_of(k);
#pragma unroll
          for (int q = 0; q < kCand; ++q) {
            if (c > tc[q]) {
              const uint64_t c2 = tc[q], k2 = tk[q];
              tc[q] = c;
              tk[q] = k;
              c = c2;
              k = k2;
            }
          }
        }
      }
    };
    uint32_t gn = 0;  // scan_stats: this lane's groups
    if (scan_stats) {
      static_assert(!PK || KT % (2 * CT) == 0, "whole 16-byte pairs per thread");
      constexpr int J = PK ? KT / (2 * CT) : 2, JH = J / 2;  // (two halves: registers)
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        ulonglong2 v[JH];
#pragma unroll
        for (int j = 0; j < JH; ++j) v[j] = reinterpret_cast<const ulonglong2*>(tkey)[(half * JH + j) * CT + tid];
#pragma unroll
        for (int j = 0; j < JH; ++j)
          reinterpret_cast<ulonglong2*>(tkey)[(half * JH + j) * CT + tid] = make_ulonglong2(kEmptyKey, kEmptyKey);
        if (!overflow) {
#pragma unroll
          for (int j = 0; j < JH; ++j) {
            if (v[j].x != kEmptyKey) {
              ++gn;
              stat(0, v[j].x, v[j].x >> KB);
            }
            if (v[j].y != kEmptyKey) {
              ++gn;
              stat(0, v[j].y, v[j].y >> KB);
            }
          }
        }
      }
    } else {  // the first 4 entries per thread with all their LDS reads in flight, then the rest
      constexpr int U = 4;
      uint32_t sl[U];
      uint64_t kv[U], cv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = tid + (uint32_t)u * CT;
        sl[u] = i < n ? list[i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kv[u] = tkey[sl[u]];
        cv[u] = PK ? 0 : tcnt[sl[u]];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = tid + (uint32_t)u * CT;
        if (i < n) {
          tkey[sl[u]] = kEmptyKey;
          if (!PK) tcnt[sl[u]] = 0;
        }
        if (PK) cv[u] = kv[u] >> KB;  // (the key stays packed: key_of)
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = tid + (uint32_t)u * CT;
        if (i < n && !overflow) stat(i, kv[u], cv[u]);
      }
      for (uint32_t i = tid + (uint32_t)U * CT; i < n; i += CT) {
        const uint32_t s = list[i];
        uint64_t kk = tkey[s], c = PK ? 0 : tcnt[s];
        tkey[s] = kEmptyKey;
        if (!PK) tcnt[s] = 0;
        if (PK) c = kk >> KB;
        if (!overflow) stat(i, kk, c);
      }
    }
    if (tid == 0 && sc && !overflow) stat(n, kEmptyKey, sc);  // (!PK only: PK never counts sc)
    const bool wgt1 = __ballot(gt1) != 0;
    if (cand && !wgt1) {  // every count of the wave is 1: its first four count-1 groups
      const uint64_t bal = __ballot(k1c);
      const uint32_t rank = (uint32_t)__builtin_popcountll(bal & ((1ULL << lane) - 1ULL));
      if (k1c && rank < (uint32_t)kCand) {
        s_wk[par][wave][rank] = key_of(k1);
        s_wc[par][wave][rank] = 1;
      }
      if (lane < kCand && (uint32_t)lane >= (uint32_t)__builtin_popcountll(bal)) s_wc[par][wave][lane] = 0;
    } else if (cand) {  // the wave's top kCand: each lane offers its groups with count > 1 in count
      // order, then its count-1 group; rounds of packed wave maxima, no block barrier
      int taken = 0;
#pragma unroll
      for (int r = 0; r < kCand; ++r) {
        uint64_t c = 0;
#pragma unroll
        for (int i2 = 0; i2 < kCand; ++i2) c = i2 == taken ? tc[i2] : c;
        const bool one = !c && k1c;
        const uint64_t mine = c ? (c << 8) | ((uint64_t)lane << 2) | (uint64_t)taken
                                : (one ? (1ULL << 8) | ((uint64_t)lane << 2) | 3ULL : 0ULL);
        const uint64_t wm = __ockl_wfred_max_u64(mine);
        if (wm && wm == mine) {
          uint64_t kk = key_of(k1), cc = 1;
          if (!one) {
#pragma unroll
            for (int i2 = 0; i2 < kCand; ++i2) {
              kk = i2 == taken ? tk[i2] : kk;
              cc = i2 == taken ? tc[i2] : cc;
            }
            ++taken;
          } else {
            k1c = false;
          }
          s_wk[par][wave][r] = kk;
          s_wc[par][wave][r] = cc;
        } else if (!wm && lane == 0) {
          s_wc[par][wave][r] = 0;
        }
      }
    }
    {
      const uint32_t wun = __ockl_wfred_add_u32(un);
      const uint32_t wgn = scan_stats ? __ockl_wfred_add_u32(gn) : 0u;
      if (lane == 0) {
        s_wgn[par][wave] = wgn;
        s_wun[par][wave] = wun;
        s_wmax[par][wave] = wgt1 ? 2u : 0u;  // (> 1: some count above 1)
      }
    }
    __syncthreads();  //                                                            [barrier 2]
    mark(2);
    if (overflow) {  // recount over two hash subsets (the table is clear already)
      if (tid == 0 && PK) {  // the whole partition, again, by the two-word kernel
        const unsigned int q = atomicAdd(a.ovf_n, 1u);
        a.ovf_out[q] = FEntry{p, 0, 0, 0};
      } else if (tid == 0) {
        const unsigned int q = atomicAdd(a.ovf_n, 2u);
        a.ovf_out[q] = FEntry{p, f + 1, fv, 0};
        a.ovf_out[q + 1] = FEntry{p, f + 1, fv | (1u << f), 0};
      }
    } else {
      if (tid == 0) {  // this item's outputs, for the next item's wave 0
        s_tp[par] = p;
        s_tg[par] = gtot;
        s_tr0[par] = r0;
        uint64_t M = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) M = s_wmax[par][w] > M ? s_wmax[par][w] : M;
        s_tfl[par] = TF_VALID | (sub ? TF_SUB : 0u) | (cand ? TF_CANDFAST : 0u) |
                     (cand && M <= 1 ? TF_CANDONE : 0u);
      }
    }
    mark(3);
    cur = pf;
    nb = nb2;
  }
  // the last item's outputs (its words were set before its barrier 2... and s_tfl after it)
  __syncthreads();
  if (wave < 2) tail(par ^ 1u, wave);
}

// ------------------------------------------------------------------------------------------------
// Phase C, hashed mode, first pass (freq_phaseC_x's design for 16-byte records): two-word slots,
// the key's 64-bit row hash and rep << 24 | count, so a claim is one CAS and one store and a
// duplicate one atomic add; the inserts of all a thread's records are in flight together (double
// hashing); claimed slots go to an LDS list, so the statistics visit the partition's groups only;
// the item's outputs are written by wave 0 during the next item.  A record that meets its key's
// slot claimed but not yet published (value 0) re-probes the same slot next round -- the claimer
// stores right after its CAS, so no barrier and no spin.  Equal hashes are decided on the arena
// bytes (enc_equal_arena): a 64-bit collision stays two groups.  A partition this kernel cannot
// take exactly (a record count >= 2^12, more than kCL records, the key kEmptyKey, a full table)
// is handed on whole (an ovf entry, f = 0) to freq_phaseC<true>.
// ------------------------------------------------------------------------------------------------
// enc_equal_arena with a rolled loop of 4-word rounds (few registers: it sits inside every probe
// round of freq_phaseC_h); 4 words past a key's end stay inside the arena's 64-byte tail.
DQ_DEV bool enc_equal_lean(const uint8_t* arena, uint64_t x, uint64_t y, const int32_t* types,
                           int n_keys) {
  const uint32_t* a = reinterpret_cast<const uint32_t*>(arena + x);
  const uint32_t* b = reinterpret_cast<const uint32_t*>(arena + y);
  const uint32_t n = n_keys == 1 && types[0] == DQ_UTF8 ? (a[0] ? 2 + pad4(a[1]) / 4 : 1u)
                                                        : enc_size(a, types, n_keys) / 4;
#pragma unroll 1
  for (uint32_t q = 0; q < n; q += 4) {
    uint32_t d = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) d |= q + k < n ? a[q + k] ^ b[q + k] : 0u;
    if (d) return false;
  }
  return true;
}
constexpr int kCHT = 4096;   // slots
constexpr int64_t kTopkRecountMax = 4096;  // dq_freq_topk recounts at most this many partitions
constexpr int kCL = 4096;    // list capacity = most records per partition
template <bool DBG>
__global__ void __launch_bounds__(kCThreads, 4) freq_phaseC_h(CArgs a) {
  constexpr int KT = kCHT, KL = kCL, NW = kCThreads / 64, PF = kPF<true>;
  constexpr uint64_t M24 = (1ULL << 24) - 1;
  __shared__ uint64_t tkey[KT], tval[KT];
  __shared__ uint16_t list[KL];
  __shared__ uint32_t s_n[2], s_ovf[2];
  __shared__ uint32_t s_chist[2][kSmallCounts];
  __shared__ unsigned long long s_efix[2][2];  // per item parity: the entropy, fixed point (lo, hi)
  __shared__ unsigned long long s_wun[2][NW], s_wmax[2][NW];
  __shared__ double s_term[kSmallCounts];
  // each wave's top kCand groups of the item (count 0: none), merged by the next item's tail
  __shared__ uint64_t s_wk[2][NW][kCand], s_wc[2][NW][kCand], s_wr[2][NW][kCand];
  __shared__ uint32_t s_tp[2], s_tg[2], s_tfl[2];
  __shared__ uint64_t s_tr0[2];
  enum { TF_VALID = 1, TF_CANDFAST = 4, TF_CANDONE = 8 };

  const int tid = threadIdx.x, lane = __lane_id(), wave = tid >> 6;
  unsigned long long collisions = 0;
  for (int i = tid; i < KT; i += kCThreads) {
    tkey[i] = kEmptyKey;
    tval[i] = 0;
  }
  if (tid < 2) {
    s_n[tid] = 0;
    s_ovf[tid] = 0;
    s_tfl[tid] = 0;
  }
  if (tid < 2 * kSmallCounts) (&s_chist[0][0])[tid] = 0;
  if (tid < 4) (&s_efix[0][0])[tid] = 0;
  if (tid < kSmallCounts) s_term[tid] = tid ? entropy_term((uint64_t)tid, a.num_rows) : 0.0;
  const bool keep = a.groups != nullptr;

  // waves 0 and 1: the outputs of the item of parity q (wv 1 the candidates, wv 0 the statistics)
  auto tail = [&](uint32_t q, int wv) {
    const uint32_t fl = s_tfl[q];
    if (!(fl & TF_VALID)) return;
    const uint32_t p = s_tp[q], gtot = s_tg[q];
    if ((fl & TF_CANDFAST) && wv == 1) {  // the item's top kCand: rounds of wave maxima over the waves' lists
      static_assert(NW * kCand <= 64, "one wave merges the lists");
      const bool in = lane < NW * kCand;
      const int w = in ? lane / kCand : 0, r = lane % kCand;
      const uint64_t c = in ? s_wc[q][w][r] : 0;
      if (fl & TF_CANDONE) {  // every count is 1: the first kCand candidates
        const uint64_t bal = __ballot(c != 0);
        const uint32_t rank = (uint32_t)__builtin_popcountll(bal & ((1ULL << lane) - 1ULL));
        if (c && rank < (uint32_t)kCand)
          a.cand[(uint64_t)p * kCand + rank] = Group{s_wk[q][w][r], c, s_wr[q][w][r]};
        if (lane < kCand && (uint32_t)lane >= (uint32_t)__builtin_popcountll(bal))
          a.cand[(uint64_t)p * kCand + lane] = Group{0, 0, 0};
      } else {
        uint64_t mine = c ? (c << 8) | (uint64_t)(63 - lane) : 0ULL;  // ties: the lower lane
#pragma unroll
        for (int k = 0; k < kCand; ++k) {
          const uint64_t wm = __ockl_wfred_max_u64(mine);
          if (wm && wm == mine) {
            a.cand[(uint64_t)p * kCand + k] = Group{s_wk[q][w][r], c, s_wr[q][w][r]};
            mine = 0;
          } else if (!wm && lane == 0) {
            a.cand[(uint64_t)p * kCand + k] = Group{0, 0, 0};
          }
        }
      }
    }
    if (wv != 0) return;
    const uint32_t hc = lane > 1 ? s_chist[q][lane] : 0u;
    // counts 2..63 join the item's LDS sum (this wave's LDS operations complete in order, so
    // lane 0 reads it after every lane's add)
    if (hc) atomic_add_fix(&s_efix[q][0], fix_of(s_term[lane]) * (fix128)hc);
    if (lane == 0) {
      uint64_t utot = 0;
      fix128 etot = (fix128)(((unsigned __int128)s_efix[q][1] << 64) | s_efix[q][0]);
#pragma unroll
      for (int w = 0; w < NW; ++w) utot += s_wun[q][w];
      if (utot) etot += fix_of(s_term[1]) * (fix128)utot;
      a.part_groups[p] = gtot;
      a.part_unique[p] = utot;
      store_fix(&a.part_entropy[2 * (uint64_t)p], etot);
      if (keep) a.part_off[p] = s_tr0[q];
    }
  };

  CBounds nb;
  CItem<true> cur;
  c_bounds(a, blockIdx.x, nb);
  c_fetch<true>(a, blockIdx.x, nb, cur);
  c_bounds(a, blockIdx.x + gridDim.x, nb);
  __syncthreads();

  uint32_t par = 0;
  int item = 0;
  auto mark = [&](int kk) {
    if constexpr (DBG)
      if (blockIdx.x == 0 && tid == 0 && item < 16) a.dbg_clock[item * 8 + kk] = wall_clock64();
  };
  for (int wi = blockIdx.x; wi < a.n_work; wi += gridDim.x, par ^= 1u, ++item) {
    mark(0);
    const uint32_t p = cur.p;
    const uint64_t r0 = cur.r0, nrec = cur.r1 - cur.r0;
    CItem<true> pf;
    CBounds nb2;

    auto insert_round = [&](const uint64_t (*w)[2], uint32_t valid, auto&& issue) {
      uint64_t h[PF], v[PF], old[PF];
      uint32_t slot[PF], step[PF], todo = 0;
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        h[q] = w[q][0];
        const uint64_t c = code_count((uint32_t)(w[q][1] & 0xff));
        v[q] = ((w[q][1] >> 8) << 24) | c;  // rep << 24 | count
        slot[q] = (uint32_t)h[q] & (KT - 1);
        step[q] = ((uint32_t)(h[q] >> 40) | 1u) & (KT - 1);
        const bool in = (valid >> q) & 1u;
        if (in && (c >= (1u << 12) || h[q] == kEmptyKey)) s_ovf[par] = 1;  // hand it on
        if (in) todo |= 1u << q;
      }
      __builtin_amdgcn_sched_barrier(0);
      mark(4);
      issue();
      mark(5);
      __builtin_amdgcn_sched_barrier(0);
      uint32_t mine = 0, cmp = 0;  // cmp bit q: the hash matched another record's key; compare
      uint64_t crs[PF];
      auto probe_rounds = [&]() {
        for (int pr = 0; todo && pr < 4 * KT; ++pr) {
#pragma unroll
          for (int q = 0; q < PF; ++q)
            old[q] = (todo >> q) & 1u ? atomicCAS((unsigned long long*)&tkey[slot[q]], kEmptyKey, h[q]) : 0ULL;
#pragma unroll
          for (int q = 0; q < PF; ++q) {
            if (!((todo >> q) & 1u)) continue;
            if (old[q] == kEmptyKey) {  // claimed: publish rep and count (non-zero)
              __hip_atomic_store(&tval[slot[q]], v[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              mine |= 1u << q;
              todo &= ~(1u << q);
            } else if (old[q] == h[q]) {
              const uint64_t sv = __hip_atomic_load(&tval[slot[q]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (!sv) continue;  // claimed, not yet published: the same slot next round
              crs[q] = sv >> 24;
              if (crs[q] == (v[q] >> 24)) {  // (the same arena key: another digit of one group)
                atomicAdd((unsigned long long*)&tval[slot[q]], (unsigned long long)(v[q] & M24));
              } else {
                cmp |= 1u << q;  // decided on the bytes below, every record's loads together
              }
              todo &= ~(1u << q);
            } else {
              slot[q] = (slot[q] + step[q]) & (KT - 1);
            }
          }
        }
      };
      probe_rounds();
      // Equal hashes on different arena keys (duplicates of a key, which phase A wrote once per
      // row): both keys' first 6 words for every such record in flight at once -- one round trip
      // per round of inserts instead of a chain per record -- which decide a one-utf8-column key
      // of <= 16 bytes; a longer key whose first words agree is compared to the end.
      while (__ballot(cmp != 0)) {
        // windows of 8 words, every undecided record's loads of a window in flight together
        uint32_t undecided = cmp, neq = 0, nw[PF];
        for (uint32_t w0 = 0; __ballot(undecided != 0); w0 += 8) {
          uint32_t ka[PF][8], kb[PF][8];
#pragma unroll
          for (int q = 0; q < PF; ++q) {
            const bool on = (undecided >> q) & 1u;
            const uint32_t* x = reinterpret_cast<const uint32_t*>(a.arena + (on ? crs[q] : 0)) + (on ? w0 : 0);
            const uint32_t* y = reinterpret_cast<const uint32_t*>(a.arena + (on ? (v[q] >> 24) : 0)) + (on ? w0 : 0);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              ka[q][k] = x[k];
              kb[q][k] = y[k];
            }
          }
#pragma unroll
          for (int q = 0; q < PF; ++q) {
            if (!((undecided >> q) & 1u)) continue;
            if (w0 == 0)  // words of the slot's key (self-delimiting encoding)
              nw[q] = a.n_keys == 1 && a.types[0] == DQ_UTF8
                          ? (ka[q][0] ? 2 + pad4(ka[q][1]) / 4 : 1u)
                          : enc_size(reinterpret_cast<const uint32_t*>(a.arena + crs[q]), a.types,
                                     a.n_keys) / 4;
            uint32_t d = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) d |= w0 + (uint32_t)k < nw[q] ? ka[q][k] ^ kb[q][k] : 0u;
            if (d) {
              neq |= 1u << q;
              undecided &= ~(1u << q);
            } else if (w0 + 8 >= nw[q]) {
              undecided &= ~(1u << q);  // equal to the end
            }
          }
        }
        uint32_t retry = 0;
#pragma unroll
        for (int q = 0; q < PF; ++q) {
          if (!((cmp >> q) & 1u)) continue;
          if (!((neq >> q) & 1u)) {
            atomicAdd((unsigned long long*)&tval[slot[q]], (unsigned long long)(v[q] & M24));
          } else {  // two keys on one 64-bit hash: two groups; probe on from the next slot
            ++collisions;
            slot[q] = (slot[q] + step[q]) & (KT - 1);
            retry |= 1u << q;
          }
        }
        cmp = 0;
        todo = retry;
        if (__ballot(todo != 0)) probe_rounds();
      }
      if (todo) s_ovf[par] = 1;  // the table is full
      const uint32_t nm = (uint32_t)__builtin_popcount(mine);
      const uint32_t incl = __ockl_wfscan_add_u32(nm, true);
      const uint32_t wtot = __builtin_amdgcn_readlane(incl, 63);
      if (wtot) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&s_n[par], wtot);
        uint32_t pos = __builtin_amdgcn_readlane(base, 0) + incl - nm;
#pragma unroll
        for (int q = 0; q < PF; ++q)
          if ((mine >> q) & 1u) list[pos++] = (uint16_t)slot[q];
      }
      mark(6);
    };
    const bool too_long = nrec > (uint64_t)KL;
    insert_round(cur.w, too_long ? 0u : cur.valid, [&]() {
      c_fetch<true>(a, wi + gridDim.x, nb, pf);
      c_bounds(a, wi + 2 * gridDim.x, nb2);
    });
    // the last item's outputs, after this wave's inserts (its records are no longer live; the
    // stores come after the prefetch, so the next item's wait for its records leaves them be)
    if (wave < 2) tail(par ^ 1u, wave);
    if (nrec > (uint64_t)PF * kCThreads && !too_long) {  // the rest of a long partition
      const uint64_t* src = reinterpret_cast<const uint64_t*>(a.recsB) + r0 * 2;
      for (uint64_t base = (uint64_t)PF * kCThreads; base < nrec; base += (uint64_t)PF * kCThreads) {
        uint64_t w[PF][2];
        uint32_t valid = 0;
#pragma unroll
        for (int q = 0; q < PF; ++q) {
          const uint64_t li = base + (uint64_t)q * kCThreads + tid;
          w[q][0] = li < nrec ? src[li * 2] : 0ULL;
          w[q][1] = li < nrec ? src[li * 2 + 1] : 0ULL;
          valid |= (li < nrec ? 1u : 0u) << q;
        }
        insert_round(w, valid, []() {});
      }
    }
    __syncthreads();  //                                                            [barrier 1]
    mark(1);
    const uint32_t n = s_n[par];
    const bool overflow = s_ovf[par] != 0 || n > (uint32_t)(KT * 7 / 8) || too_long;
    const bool cand = a.want_cand && !overflow;
    if (tid == 0) {
      s_n[par ^ 1u] = 0;
      s_ovf[par ^ 1u] = 0;
      s_tfl[par ^ 1u] = 0;
    }
    if (tid < kSmallCounts) s_chist[par ^ 1u][tid] = 0;
    if (tid < 2) s_efix[par ^ 1u][tid] = 0;
    const uint32_t gtot = n;
    const uint64_t obase = a.group_stride ? (uint64_t)wi * a.group_stride : r0;

    uint64_t un = 0, mx = 0;
    uint64_t tc[kCand], tk[kCand], tr[kCand];
#pragma unroll
    for (int q = 0; q < kCand; ++q) tc[q] = tk[q] = tr[q] = 0;
    uint64_t k1 = 0, r1 = 0;
    bool k1c = false;
    auto stat = [&](uint32_t i, uint64_t k, uint64_t c, uint64_t r) {
      if (a.lit_count && k == a.lit_h && enc_is_null_literal(a.arena + r))
        atomicAdd(a.lit_count, (unsigned long long)c);
      if (keep) a.groups[obase + i] = Group{k, c, r};
      if (c == 1) ++un;
      else if (c < kSmallCounts) atomicAdd(&s_chist[par][c], 1u);
      else atomic_add_fix(&s_efix[par][0], fix_of(entropy_term(c, a.num_rows)));  // (rare)
      mx = c > mx ? c : mx;
      if (cand) {
        if (c == 1) {
          if (!k1c) {
            k1 = k;
            r1 = r;
          }
          k1c = true;
        } else if (c > tc[kCand - 1]) {
#pragma unroll
          for (int q = 0; q < kCand; ++q) {
            if (c > tc[q]) {
              const uint64_t c2 = tc[q], k2 = tk[q], r2 = tr[q];
              tc[q] = c;
              tk[q] = k;
              tr[q] = r;
              c = c2;
              k = k2;
              r = r2;
            }
          }
        }
      }
    };
    {
      constexpr int U = 2;
      uint32_t sl[U];
      uint64_t kv[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = tid + (uint32_t)u * kCThreads;
        sl[u] = i < n ? list[i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kv[u] = tkey[sl[u]];
        vv[u] = tval[sl[u]];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = tid + (uint32_t)u * kCThreads;
        if (i < n) {
          tkey[sl[u]] = kEmptyKey;
          tval[sl[u]] = 0;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = tid + (uint32_t)u * kCThreads;
        if (i < n && !overflow) stat(i, kv[u], vv[u] & M24, vv[u] >> 24);
      }
      for (uint32_t i = tid + (uint32_t)U * kCThreads; i < n; i += kCThreads) {
        const uint32_t s = list[i];
        const uint64_t kk = tkey[s], vx = tval[s];
        tkey[s] = kEmptyKey;
        tval[s] = 0;
        if (!overflow) stat(i, kk, vx & M24, vx >> 24);
      }
    }
    const uint64_t wmx1 = __ockl_wfred_max_u64(mx);
    if (cand && wmx1 <= 1) {  // every count of the wave is 1: its first four count-1 groups
      const uint64_t bal = __ballot(k1c);
      const uint32_t rank = (uint32_t)__builtin_popcountll(bal & ((1ULL << lane) - 1ULL));
      if (k1c && rank < (uint32_t)kCand) {
        s_wk[par][wave][rank] = k1;
        s_wc[par][wave][rank] = 1;
        s_wr[par][wave][rank] = r1;
      }
      if (lane < kCand && (uint32_t)lane >= (uint32_t)__builtin_popcountll(bal)) s_wc[par][wave][lane] = 0;
    } else if (cand) {  // the wave's top kCand: each lane offers its groups with count > 1 in count
      // order, then its count-1 group; rounds of packed wave maxima, no block barrier
      int taken = 0;
#pragma unroll
      for (int r = 0; r < kCand; ++r) {
        uint64_t c = 0;
#pragma unroll
        for (int i2 = 0; i2 < kCand; ++i2) c = i2 == taken ? tc[i2] : c;
        const bool one = !c && k1c;
        const uint64_t mine = c ? (c << 8) | ((uint64_t)lane << 2) | (uint64_t)taken
                                : (one ? (1ULL << 8) | ((uint64_t)lane << 2) | 3ULL : 0ULL);
        const uint64_t wm = __ockl_wfred_max_u64(mine);
        if (wm && wm == mine) {
          uint64_t kk = k1, cc = 1, rr = r1;
          if (!one) {
#pragma unroll
            for (int i2 = 0; i2 < kCand; ++i2) {
              kk = i2 == taken ? tk[i2] : kk;
              cc = i2 == taken ? tc[i2] : cc;
              rr = i2 == taken ? tr[i2] : rr;
            }
            ++taken;
          } else {
            k1c = false;
          }
          s_wk[par][wave][r] = kk;
          s_wc[par][wave][r] = cc;
          s_wr[par][wave][r] = rr;
        } else if (!wm && lane == 0) {
          s_wc[par][wave][r] = 0;
        }
      }
    }
    {
      const uint64_t wun = __ockl_wfred_add_u64(un);
      const uint64_t wmx = wmx1;
      if (lane == 0) {
        s_wun[par][wave] = wun;
        s_wmax[par][wave] = wmx;
      }
    }
    __syncthreads();  //                                                            [barrier 2]
    mark(2);
    if (overflow) {
      if (tid == 0) {  // the whole partition, again, by the generic kernel
        const unsigned int q = atomicAdd(a.ovf_n, 1u);
        a.ovf_out[q] = FEntry{p, 0, 0, 0};
      }
    } else {
      if (tid == 0) {
        s_tp[par] = p;
        s_tg[par] = gtot;
        s_tr0[par] = r0;
        uint64_t M = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) M = s_wmax[par][w] > M ? s_wmax[par][w] : M;
        s_tfl[par] = TF_VALID | (cand ? TF_CANDFAST : 0u) | (cand && M <= 1 ? TF_CANDONE : 0u);
      }
    }
    mark(3);
    cur = pf;
    nb = nb2;
  }
  __syncthreads();
  if (wave < 2) tail(par ^ 1u, wave);
  if (collisions) atomicAdd(&a.counters[C_COLLISIONS], collisions);
}

// Multi-block fixed-order reduction of the per-partition statistics: block b sums its contiguous
// range (coalesced: consecutive threads read consecutive partitions), freq_reduce_final adds the
// blocks' partials in block order.  out = {groups, unique, entropy bits}.
constexpr int kRedBlocks = 256;
__global__ void __launch_bounds__(kThreads) freq_reduce_part(const unsigned long long* pg,
                                                             const unsigned long long* pu,
                                                             const unsigned long long* pe, int64_t n,
                                                             unsigned long long* part) {
  __shared__ uint64_t s_red[kThreads / 64];
  __shared__ fix128 s_rede[kThreads / 64];
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = min(lo + per, n);
  uint64_t g = 0, u = 0;
  fix128 e = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
    g += pg[i];
    u += pu[i];
    e += (fix128)(((unsigned __int128)pe[2 * i + 1] << 64) | pe[2 * i]);
  }
  g = block_sum_u64(g, s_red);
  u = block_sum_u64(u, s_red);
  e = wave_sum_fix(e);
  if (__lane_id() == 0) s_rede[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) {
    fix128 t = 0;
    for (int w = 0; w < kThreads / 64; ++w) t += s_rede[w];
    part[blockIdx.x * 4] = g;
    part[blockIdx.x * 4 + 1] = u;
    store_fix(part + blockIdx.x * 4 + 2, t);
  }
}
__global__ void freq_reduce_final(const unsigned long long* part, int nb, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  uint64_t g = 0, u = 0;
  fix128 e = 0;
  for (int b = 0; b < nb; ++b) {
    g += part[b * 4];
    u += part[b * 4 + 1];
    e += (fix128)(((unsigned __int128)part[b * 4 + 3] << 64) | part[b * 4 + 2]);
  }
  out[0] = g;
  out[1] = u;
  out[2] = __builtin_bit_cast(unsigned long long, fix_to_f64(e));
  out[4] = (uint64_t)e;  // (out[3]: the "NullValue" literal's count, written by phase C)
  out[5] = (uint64_t)(e >> 64);
}

// Multi-block exclusive scan of u64 values in place, v[n] = total (large n; freq_part_scan is the
// one-block form): S1 block sums of kScanTile values, freq_part_scan over the sums, S2 scans each
// tile from its offset.
constexpr int kScanPer = 4;
constexpr int64_t kScanTile = (int64_t)kThreads * kScanPer;
__global__ void __launch_bounds__(kThreads) scan_u64_sums(const unsigned long long* v, int64_t n,
                                                          unsigned long long* bsum) {
  __shared__ uint64_t s_red[kThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
  uint64_t t = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k)
    if (base + k < n) t += v[base + k];
  t = block_sum_u64(t, s_red);
  if (threadIdx.x == 0) bsum[blockIdx.x] = t;
}
__global__ void __launch_bounds__(kThreads) scan_u64_apply(unsigned long long* v, int64_t n,
                                                           const unsigned long long* boff) {
  __shared__ uint64_t s_red[kThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
  uint64_t x[kScanPer], t = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    x[k] = base + k < n ? v[base + k] : 0;
    t += x[k];
  }
  // exclusive prefix of t over the block: wave prefix (64-bit) + the waves before
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  uint64_t inc = t;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_red[wave] = inc;
  __syncthreads();
  uint64_t run = boff[blockIdx.x] + inc - t;
  for (int w = 0; w < wave; ++w) run += s_red[w];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (base + k < n) v[base + k] = run;
    run += x[k];
  }
  if (base <= n - 1 && n - 1 < base + kScanPer) v[n] = run;  // the thread holding the last value
}


// ------------------------------------------------------------------------------------------------
// Selection over Group arrays (Histogram top-N), export and repartition helpers
// ------------------------------------------------------------------------------------------------
// hist[k] += #groups with lo <= count < hi falling in bin (count - lo) / width; width == 0
// selects power-of-two bins (bin = floor(log2(count)))
__global__ void __launch_bounds__(256) freq_group_hist(const Group* g, int64_t n, uint64_t lo,
                                                       uint64_t hi, uint64_t width,
                                                       unsigned long long* hist) {
  __shared__ unsigned int lh[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t c = g[i].count;
    const bool act = !(c == 0 || c < lo || c >= hi);
    const uint32_t bin = act ? (uint32_t)(width ? (c - lo) / width : (uint64_t)(63 - __builtin_clzll(c))) : 0u;
    // a wave whose counted groups share one bin (a high-cardinality key: every count 1) adds
    // once -- 64 same-address LDS atomics per wave instruction serialised the kernel
    const uint64_t am = __ballot(act);
    if (!am) continue;
    const int first = __builtin_ctzll(am);
    const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bin, first);
    if (__ballot(act && bin == b0) == am) {
      if ((int)__lane_id() == first) atomicAdd(&lh[b0], (unsigned)__builtin_popcountll(am));
    } else if (act) {
      atomicAdd(&lh[bin], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += blockDim.x)
    if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
}
// every group with count >= hi_take, and groups with lo_tie <= count < hi_take up to `cap`
__global__ void freq_group_select(const Group* g, int64_t n, uint64_t hi_take, uint64_t lo_tie,
                                  unsigned long long cap, Group* out, unsigned long long* n_take,
                                  unsigned long long* n_tie, Group* out_tie) {
  // (wave-aggregated cursors: one device atomic per wave and list, not per group)
  const uint64_t below = (1ULL << __lane_id()) - 1ULL;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const Group x = g[i];
    const bool take = x.count != 0 && x.count >= hi_take;
    const bool tie = x.count != 0 && !take && x.count >= lo_tie;
    const uint64_t bt = __ballot(take), bi = __ballot(tie);
    if (bt) {
      const int first = __builtin_ctzll(bt);
      unsigned long long base = 0;
      if ((int)__lane_id() == first) base = atomicAdd(n_take, (unsigned long long)__builtin_popcountll(bt));
      base = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(base >> 32), first) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, first);
      if (take) out[base + (unsigned long long)__builtin_popcountll(bt & below)] = x;
    }
    // (once the tie list is full, later waves only read its cursor: a high-cardinality key's
    // top-k ties ~1e6 candidates at count 1, and their adds on one address serialised in L2)
    if (bi && __hip_atomic_load(n_tie, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cap) {
      const int first = __builtin_ctzll(bi);
      unsigned long long base = 0;
      if ((int)__lane_id() == first) base = atomicAdd(n_tie, (unsigned long long)__builtin_popcountll(bi));
      base = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(base >> 32), first) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, first);
      const unsigned long long q = base + (unsigned long long)__builtin_popcountll(bi & below);
      if (tie && q < cap) out_tie[q] = x;
    }
  }
}
// partitions with groups beyond their listed candidates whose last candidate beats `tau`: their
// unlisted groups could outrank the selection
__global__ void freq_cand_check(const Group* cand, const unsigned long long* part_groups, int64_t P,
                                uint64_t tau, unsigned long long* bad, FEntry* bad_list, int64_t cap) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    int filled = 0;  // places hold the partition's top groups in count order, empty ones last
    for (int r = 0; r < kCand; ++r) filled += cand[p * kCand + r].count ? 1 : 0;
    if (part_groups[p] > (unsigned long long)filled &&
        (!filled || cand[p * kCand + filled - 1].count > tau)) {
      const unsigned long long q = atomicAdd(bad, 1ULL);
      if ((int64_t)q < cap) bad_list[q] = FEntry{(uint32_t)p, 0, 0, 0};
    }
  }
}

// The candidate places of the listed partitions emptied (their every group is selected instead)
__global__ void freq_cand_clear(Group* cand, const FEntry* list, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * kCand) cand[(uint64_t)list[i / kCand].p * kCand + i % kCand] = Group{0, 0, 0};
}

struct PartTypes {
  int32_t types[kMaxKeys];
  int32_t n_keys;
  int32_t exact;
  uint32_t parts;
  uint32_t pad;
};

// Owner rank of a group for the multi-GPU repartition: the high hash bits, so every owner gets a
// contiguous hash range (and the owner's own partitions stay uniformly loaded).
DQ_DEV uint32_t owner_of(uint64_t h, uint32_t parts) {
  return (uint32_t)(((h >> 40) * (uint64_t)parts) >> 24);
}

__global__ void __launch_bounds__(256) freq_owner_count(const Group* g, int64_t n,
                                                        const uint8_t* arena, PartTypes t,
                                                        unsigned long long* n_rec,
                                                        unsigned long long* n_var) {
  __shared__ unsigned long long lr[kMaxParts], lv[kMaxParts];
  for (int i = threadIdx.x; i < kMaxParts; i += blockDim.x) lr[i] = lv[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const Group x = g[i];
    const uint32_t o = owner_of(x.h, t.parts);
    atomicAdd(&lr[o], 1ULL);
    if (!t.exact)
      atomicAdd(&lv[o],
                (unsigned long long)((enc_size(reinterpret_cast<const uint32_t*>(arena + x.rep),
                                               t.types, t.n_keys) + 7u) & ~7u));
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < t.parts; i += blockDim.x) {
    if (lr[i]) atomicAdd(&n_rec[i], lr[i]);
    if (lv[i]) atomicAdd(&n_var[i], lv[i]);
  }
}

// dq_freq_record per group (exact: the value, fmix_inv(h); hashed: h and the encoded key copied
// into the owner's var segment)
__global__ void __launch_bounds__(256) freq_owner_scatter(
    const Group* g, int64_t n, const uint8_t* arena, PartTypes t,
    const unsigned long long* rec_base, const unsigned long long* var_base,
    unsigned long long* rec_cur, unsigned long long* var_cur, RecIn* out_rec, uint8_t* out_var) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const Group x = g[i];
    const uint32_t o = owner_of(x.h, t.parts);
    const unsigned long long q = atomicAdd(&rec_cur[o], 1ULL);
    RecIn r{t.exact ? fmix_inv(x.h) : x.h, x.count, 0};
    if (!t.exact) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(arena + x.rep);
      const uint32_t size = enc_size(src, t.types, t.n_keys);
      const unsigned long long off = atomicAdd(&var_cur[o], (unsigned long long)((size + 7u) & ~7u));
      uint32_t* dst = reinterpret_cast<uint32_t*>(out_var + var_base[o] + off);
      for (uint32_t w = 0; w < size / 4; ++w) dst[w] = src[w];
      if (size & 4u) dst[size / 4] = 0;  // 8-byte padding
      r.enc_off = off;
    }
    out_rec[rec_base[o] + q] = r;
  }
}

// the largest count_digits of n received records (sizes the records path's tiles)
__global__ void __launch_bounds__(256) freq_max_digits(const RecIn* __restrict__ r, int64_t n,
                                                       unsigned int* out) {
  int m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, count_digits(r[i].count));
  m = (int)__ockl_wfred_max_u64((uint64_t)m);
  if (__lane_id() == 0 && m) atomicMax(out, (unsigned int)m);
}

// hashed merge: the appended chunks' records point into the appended arena bytes
__global__ void freq_rebase(uint64_t* recs, const uint16_t* hist, int64_t chunk0, int tile,
                            uint64_t delta) {
  const int64_t c = chunk0 + blockIdx.x;
  const uint32_t n = hist[c * kHistRow + kBuckets];
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) recs[(c * tile + i) * 2 + 1] += delta << 8;
}

// the same for the records of bucket pieces (hashed: one-utf8-column tables): piece row r's
// bucket b holds plen[r][b] records from pbase[r] + pstart[r][b]
__global__ void freq_rebase_pieces(uint64_t* recs, const uint32_t* pstart, const uint32_t* plen,
                                   const unsigned long long* pbase, uint64_t delta) {
  const int64_t r = blockIdx.x;
  for (int b = threadIdx.x; b < kBuckets; b += blockDim.x) {
    const uint64_t s0 = pbase[r] + pstart[r * kBuckets + b];
    const uint32_t n = plen[r * kBuckets + b];
    for (uint32_t i = 0; i < n; ++i) recs[(s0 + i) * 2 + 1] += delta << 8;
  }
}

// compact the materialised groups: partition p's g_p groups start at src_off[p], go to dst_off[p]
__global__ void freq_compact(const Group* src, const unsigned long long* src_off,
                             const unsigned long long* cnt, const unsigned long long* dst_off,
                             int64_t P, Group* dst) {
  for (int64_t p = blockIdx.x; p < P; p += gridDim.x) {
    const uint64_t n = cnt[p];
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) dst[dst_off[p] + i] = src[src_off[p] + i];
  }
}


}  // namespace dq

using namespace dq;

// ------------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------------

// 8-byte page-locked words (the small-key phase A's give-up flag) carved from shared 4 KB blocks
// kept to process exit: a hipHostMalloc + hipHostFree per table cost ~0.1-0.2 ms each at every
// string Histogram job's boundary.
struct PinnedWords {
  std::mutex m;
  std::vector<unsigned long long*> free_words;
};
static PinnedWords& pinned_words() {
  static PinnedWords* w = new PinnedWords;
  return *w;
}
static hipError_t pinned_word_get(unsigned long long** out) {
  PinnedWords& w = pinned_words();
  std::lock_guard<std::mutex> lock(w.m);
  if (w.free_words.empty()) {
    void* blk = nullptr;
    hipError_t e = hipHostMalloc(&blk, 4096, hipHostMallocDefault);
    if (e != hipSuccess) return e;
    for (int i = 0; i < 512; ++i) w.free_words.push_back(static_cast<unsigned long long*>(blk) + i);
  }
  *out = w.free_words.back();
  w.free_words.pop_back();
  return hipSuccess;
}
// The caller has synchronized the stream of the last copy into the word (dq_freq_destroy), so
// no copy can still land in it; no device-wide barrier (it would wait for other tables' streams).
static void pinned_word_put(unsigned long long* p) {
  PinnedWords& w = pinned_words();
  std::lock_guard<std::mutex> lock(w.m);
  w.free_words.push_back(p);
}

struct dq_freq {
  int device = 0;
  int n_keys = 0;
  // key types as the caller declared them, and the physical layout the group-by runs on
  // (freq_phys_type: dates / timestamps as their integers, decimals as their unscaled long or
  // 16-byte string); every kernel below sees only `types`
  std::vector<int32_t> logical;
  std::vector<int32_t> types;
  bool relabel = false;  // some logical type differs from its physical one
  DevBuf<int64_t> dec_long[kMaxKeys];  // decimal(p <= 18) keys narrowed to their unscaled long
  DevBuf<int32_t> dec_off;             // decimal(p > 18) keys: offsets 0, 16, 32, ... (shared)
  bool exact = false;
  int mode_null_as_group = -1;  // fixed by the first add
  int tile = 0, rb = 0;
  // the table: bucket-sorted chunk regions (phase A output) + their histograms
  DevBuf<uint8_t> recs;
  DevBuf<uint16_t> hist;
  int64_t n_chunks = 0;
  // exact rows: batch regions written bucket-major (freq_prepass_x), one piece row per phase-A
  // workgroup: piece (r, b) = records [pbase[r] + pstart[r][b], + plen[r][b]) of `recs`
  DevBuf<uint32_t> pstart, plen;
  std::vector<unsigned long long> h_pbase;
  int64_t n_prow = 0;
  int64_t n_empty_chunks = 0;  // chunk rows known empty (bucket-piece batches): finalize skips them
  DevBuf<uint32_t> ph, ptot;  // the pre-pass's per-workgroup bucket counts (scratch)
  DevBuf<unsigned long long> pbase;
  DevBuf<uint8_t> arena;                 // hashed: encoded keys
  DevBuf<unsigned long long> dev_words;  // counters[C_N], then the arena cursor
  DevBuf<unsigned long long> batch_tab;  // freq_phaseA_small's cross-workgroup group table
  uint64_t h_counters[C_N] = {0};
  uint64_t arena_used = 0;
  uint64_t rec_var_base = 0;  // arena offset of the last dq_freq_add_records_device's var bytes
  // a table built from another table's records may read that table's arena in place instead of
  // a copy (MutualInformation's marginals, which die before their joint table): then the keys live
  // here and the table takes no further adds
  const uint8_t* arena_view = nullptr;
  // phase A launches leave the device counters and arena cursor ahead of the host copies: they
  // are read back only when needed (finalize, merge, arena growth), so batches queue back to back
  bool counters_stale = false;
  uint64_t arena_hi = 0;  // upper bound of the arena bytes in use (arena_used at the last read-back
                          // + the worst case of every batch added since)
  int64_t num_rows = 0;
  hipStream_t stream = nullptr;
  // the small-key phase A (freq_phaseA_small): the epoch of its last attempt, and a pinned copy of
  // the epoch it last gave up (copied back asynchronously: a table it gave up on stops trying)
  uint64_t fast_epoch = 0;
  bool fast_off = false;
  // every batch went through freq_phaseA_xp, which counts C_NAN_FOLDED (records, merges and the
  // other phase-A kernels do not)
  bool nan_counted = true;
  struct PinnedWord {
    unsigned long long* p = nullptr;
    hipStream_t last_copy = nullptr;  // the stream of the last copy into *p
    // Before a copy into *p is queued on `st`: a copy still queued on another stream could land
    // after it (and after dq_freq_destroy synced only `st`, recycling the word to another table),
    // so that stream is waited for first.  Same stream: stream order already holds.
    hipError_t before_copy(hipStream_t st) {
      hipError_t e = hipSuccess;
      if (last_copy && last_copy != st) e = hipStreamSynchronize(last_copy);
      last_copy = st;
      return e;
    }
    ~PinnedWord() {
      if (p) pinned_word_put(p);
    }
  } fast_seen;
  // the dense integer path (freq_dense_count / _emit): its device words (AArgs::dense_words), the
  // epoch of its last attempt, the counting workgroups' counters, and a pinned copy of the epoch
  // it last declined (a table it declined stops trying)
  DevBuf<unsigned long long> dense_words;
  DevBuf<uint32_t> dense_part;
  uint64_t dense_epoch = 0;
  bool dense_off = false;
  PinnedWord dense_seen;
  // recorded behind the first tried batch's decline-word copy (ahead of its phase A): the second
  // batch waits for that answer instead of trying again (a fresh table per run -- the runner's
  // Histogram tables -- ran the range pre-pass on three or four batches of a wide column)
  hipEvent_t dense_ev = nullptr;
  bool dense_waited = false;
  // finalize cache (phase B)
  bool b_valid = false;
  int s_bits = 0;
  uint64_t R = 0;
  uint32_t n_units = 0;
  std::vector<unsigned long long> h_bucket_base = std::vector<unsigned long long>(kBuckets + 1, 0);
  std::vector<uint32_t> h_unit_start = std::vector<uint32_t>(kBuckets + 1, 0);
  DevBuf<unsigned long long> segS;         // phase B's segments per bucket (freq_seg_scan)
  DevBuf<uint32_t> segP, nseg;
  DevBuf<uint32_t> chunk_id;               // the non-empty chunks (finalize over those only)
  DevBuf<unsigned long long> chunk_boff, scan_tmp;
  DevBuf<uint32_t> unit_start, unit_c0, uhist;
  DevBuf<uint16_t> unit_b;
  DevBuf<unsigned long long> totals, part_base;
  // Capacity layout (exact tables, finalize_b): partition p's records are [part_base[p],
  // part_end[p]) inside a fixed capacity, filled through atomic cursors (no count pass).  The
  // counted layout's ends are part_base + 1.  Rcap: the records region's size in records.
  DevBuf<unsigned long long> part_end, cap_words;  // cap_words: bucket bases [kBuckets + 1], caps
  DevBuf<unsigned int> b_ovf;
  std::vector<unsigned long long> h_cap_words;
  const unsigned long long* part_end_ptr = nullptr;
  uint64_t Rcap = 0;
  bool cap_failed = false;  // a capacity layout overflowed: this table counts from now on
  DevBuf<uint8_t> recsB;
  // (phase C)
  bool c_valid = false, c_groups = false, c_cand = false;
  double c_num_rows = -1.0;
  DevBuf<unsigned long long> part_groups, part_unique, part_off;
  DevBuf<unsigned long long> part_entropy;  // (lo, hi) fixed-point sum per partition
  DevBuf<Group> cand, groups, compact;
  int64_t n_compact = -1;
  DevBuf<FEntry> ovf_a, ovf_b;
  DevBuf<unsigned int> ovf_n;
  DevBuf<unsigned long long> red;
  uint64_t st_groups = 0, st_unique = 0;
  double st_entropy = 0.0;
  fix128 st_entropy_fix = 0;  // the same sum, before its rounding to fp64
  uint64_t st_literal = 0;  // Histogram on a string: count of the "NullValue" string group
  bool recounted = false;
  // last top-k (dq_freq_topk is called twice: sizes, then data)
  int topk_k = -1;
  std::vector<int64_t> topk_counts, topk_offs;
  std::vector<uint8_t> topk_bytes;
};

static unsigned grid_for(uint64_t n, unsigned cap = 4096) {
  uint64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// A Histogram table over one string column: its NULL rows are kept apart from a "NullValue"
// string group that phase C probes for.
static bool has_null_literal(const dq_freq* f) {
  return !f->exact && f->n_keys == 1 && f->types[0] == DQ_UTF8 && f->mode_null_as_group > 0;
}

static void invalidate(dq_freq* f) {
  f->b_valid = false;
  f->c_valid = f->c_groups = f->c_cand = false;
  f->n_compact = -1;
  f->topk_k = -1;
}

// Grows `b` to at least `need` elements keeping the first `used` (stream-ordered copy).
template <typename T>
static hipError_t grow_keep(DevBuf<T>& b, size_t used, size_t need, hipStream_t st) {
  if (need <= b.n && b.p) return hipSuccess;
  DevBuf<T> nb;
  hipError_t e = nb.ensure(std::max(need, b.n * 2));
  if (e != hipSuccess) return e;
#if DQ_A_NOCOPY  // (timing build: the never-written arena reads as zero words, so every key is 4 bytes)
  e = hipMemsetAsync(nb.p, 0, nb.n * sizeof(T), st);
  if (e != hipSuccess) return e;
#endif
  if (used) {
    e = hipMemcpyAsync(nb.p, b.p, used * sizeof(T), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
  }
  b.swap(nb);
  return hipSuccess;
}

static dq_status ensure_chunks(dq_freq* f, int64_t add) {
  const int64_t need = f->n_chunks + add;
  HIP_TRY(grow_keep(f->recs, (size_t)f->n_chunks * f->tile * f->rb, (size_t)need * f->tile * f->rb,
                    f->stream));
  HIP_TRY(grow_keep(f->hist, (size_t)f->n_chunks * kHistRow, (size_t)need * kHistRow, f->stream));
  return DQ_OK;
}

// the counters and the arena cursor as read back (dev_words: C_N counters + the cursor)
static void apply_counters(dq_freq* f, const unsigned long long* w) {
  for (int k = 0; k < C_N; ++k) f->h_counters[k] = w[k];
  f->arena_used = w[C_N];
  f->arena_hi = f->arena_used;
  f->counters_stale = false;
}
static dq_status pull_counters(dq_freq* f) {  // (d2h is ordered after the stream's work)
  unsigned long long w[C_N + 1];
  HIP_TRY(d2h(w, f->dev_words.p, sizeof(w), f->stream));
  apply_counters(f, w);
  return DQ_OK;
}
static dq_status sync_counters(dq_freq* f) { return f->counters_stale ? pull_counters(f) : DQ_OK; }

static dq_status push_counters(dq_freq* f) {
  HIP_TRY(hipStreamSynchronize(f->stream));
  unsigned long long w[C_N + 1];
  for (int k = 0; k < C_N; ++k) w[k] = f->h_counters[k];
  w[C_N] = f->arena_used;
  HIP_TRY(hipMemcpy(f->dev_words.p, w, sizeof(w), hipMemcpyHostToDevice));
  f->arena_hi = f->arena_used;
  f->counters_stale = false;
  return DQ_OK;
}

// Chunks one phase-A launch over n items writes: one per tile + one per workgroup.
static int64_t phaseA_chunks(bool hashed, bool from_rec, int64_t n_items, int64_t tile_items,
                             int64_t* n_wg_out) {
  const int tpw = from_rec ? (hashed ? AKeys<true, true>::kTilesPerWg : AKeys<false, true>::kTilesPerWg)
                           : (hashed ? AKeys<true, false>::kTilesPerWg : AKeys<false, false>::kTilesPerWg);
  const int64_t tiles = (n_items + tile_items - 1) / tile_items;
  const int64_t n_wg = (tiles + tpw - 1) / tpw;
  if (n_wg_out) *n_wg_out = n_wg;
  return tiles + n_wg;
}

template <bool HASHED>
static void launch_phaseA(dq_freq* f, AArgs a, bool from_rec) {
  int64_t n_wg = 0;
  phaseA_chunks(HASHED, from_rec, a.n_items, a.tile_items, &n_wg);
  a.tiles_per_wg = from_rec ? AKeys<HASHED, true>::kTilesPerWg : AKeys<HASHED, false>::kTilesPerWg;
  static int dbg = [] {
    const char* e = getenv("DQ_FREQ_DEBUG");
    return e ? atoi(e) : 0;
  }();
  unsigned long long* clk = nullptr;
  if (dbg >= 2 && hipMalloc(&clk, 16 * 8 * sizeof(unsigned long long)) == hipSuccess)
    (void)hipMemset(clk, 0, 16 * 8 * sizeof(unsigned long long));
  else
    clk = nullptr;
  a.dbg_clock = clk;
  if (from_rec)
    hipLaunchKernelGGL((freq_phaseA<HASHED, true>), dim3((unsigned)n_wg),
                       dim3(AKeys<HASHED, true>::kThreads), 0,
                       f->stream, a);
  else if (HASHED && a.ks.n_keys == 1 && a.ks.cols[0].type == DQ_UTF8)
    hipLaunchKernelGGL((freq_phaseA<HASHED, false, HASHED>), dim3((unsigned)n_wg),
                       dim3(AKeys<HASHED, false>::kThreads), 0,
                       f->stream, a);
  else
    hipLaunchKernelGGL((freq_phaseA<HASHED, false>), dim3((unsigned)n_wg),
                       dim3(AKeys<HASHED, false>::kThreads), 0,
                       f->stream, a);
  if (clk) {  // per-tile phase times of workgroup 0, us (the wall clock ticks at 100 MHz)
    unsigned long long h[16 * 8];
    (void)hipStreamSynchronize(f->stream);
    (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(clk);
    double acc[4] = {0, 0, 0, 0};
    int nt = 0;
    for (int t = 0; t < 16; ++t) {
      if (!h[t * 8 + 4]) break;
      for (int k = 0; k < 4; ++k) acc[k] += (double)(h[t * 8 + k + 1] - h[t * 8 + k]) / 100.0;
      ++nt;
    }
    if (nt)
      fprintf(stderr, "dq_freq phase A%s%s wg0 per tile (us): load+hash %.2f dedupe %.2f begin %.2f "
              "put+end %.2f (%d tiles)\n", HASHED ? " hashed" : " exact",
              a.ks.null_as_group ? " (histogram)" : "", acc[0] / nt, acc[1] / nt, acc[2] / nt,
              acc[3] / nt, nt);
  }
}

// The small-key phase A over one batch of a one-utf8-column key, before the general one (which
// returns at once when this one took the batch).  Tried while the batch's strings average at most
// 8 bytes (its data_bytes hint) and until the table sees it give a batch up.
static bool small_keys_worth_trying(dq_freq* f, const dq_column& k, int64_t rows) {
  static const bool enabled = [] {
    const char* e = getenv("DQ_FREQ_SMALL");
    return !e || atoi(e) != 0;
  }();
  if (!enabled || f->exact || f->n_keys != 1 || f->types[0] != DQ_UTF8 || rows < 4096) return false;
  if (f->fast_off) return false;
  if (f->fast_seen.p && f->fast_epoch && *(volatile unsigned long long*)f->fast_seen.p == f->fast_epoch) {
    f->fast_off = true;  // the last attempt gave its batch up: long strings or many keys
    return false;
  }
  return k.data_bytes > 0 && (int64_t)k.data_bytes <= 8 * rows;
}

static dq_status launch_phaseA_small(dq_freq* f, AArgs& a) {
  if (!f->fast_seen.p) {
    HIP_TRY(pinned_word_get(&f->fast_seen.p));
    *f->fast_seen.p = 0;
  }
  int64_t n_wg = 0;
  phaseA_chunks(true, false, a.n_items, a.tile_items, &n_wg);
  a.tiles_per_wg = AKeys<true, false>::kTilesPerWg;
  a.fast_words = f->dev_words.p + C_N + 1;
  HIP_TRY(f->batch_tab.ensure(kBatchTabs * kBatchTabWords));
  HIP_TRY(hipMemsetAsync(f->batch_tab.p, 0, kBatchTabs * kBatchTabWords * 8, f->stream));
  a.batch_tab = f->batch_tab.p;
  a.fast_epoch = ++f->fast_epoch;
  const KeyCol& c = a.ks.cols[0];
  static const int poll = [] {  // DQ_FREQ_POLL: A/B hook for the give-up poll interval
    const char* e = getenv("DQ_FREQ_POLL");
    return e ? atoi(e) : 0;
  }();
  a.fast_poll = poll;
  a.vec_ok = (reinterpret_cast<uintptr_t>(c.values) & 15u) == 0 &&
             (reinterpret_cast<uintptr_t>(c.valid) & 3u) == 0;
  static const int cus = [] {
    int n = 0, d = 0;
    (void)hipGetDevice(&d);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && n > 0 ? n : 256;
  }();
  // about three workgroups per CU (the kernel's occupancy), each standing for several of the
  // general kernel's
  const int64_t slots = 3LL * cus;
  a.small_merge = (int32_t)std::max<int64_t>(1, (n_wg + slots - 1) / slots);
  const int64_t grid = (n_wg + a.small_merge - 1) / a.small_merge;
  hipLaunchKernelGGL(freq_phaseA_small, dim3((unsigned)grid), dim3(kSmallThreads), 0, f->stream, a);
  HIP_TRY(hipGetLastError());
  return DQ_OK;
}

static const uint8_t* arena_of(const dq_freq* f) { return f->arena_view ? f->arena_view : f->arena.p; }

static AArgs base_args(dq_freq* f) {
  AArgs a;
  memset(&a, 0, sizeof(a));
  for (int k = 0; k < f->n_keys; ++k) {
    a.types[k] = f->types[k];
    a.ks.cols[k].type = f->types[k];
  }
  a.n_keys = f->n_keys;
  a.ks.n_keys = f->n_keys;
  a.ks.null_as_group = f->mode_null_as_group > 0 ? 1 : 0;
  a.recs = f->recs.p + (size_t)f->n_chunks * f->tile * f->rb;
  a.hist = f->hist.p + (size_t)f->n_chunks * kHistRow;
  a.arena = const_cast<uint8_t*>(arena_of(f));
  a.arena_cursor = f->dev_words.p + C_N;
  a.counters = f->dev_words.p;
  return a;
}

// Exact rows into fixed-capacity bucket pieces without the pre-pass (DQ_FREQ_XFIXED=0: pieces
// laid out by the pre-pass's counts)
static bool xfixed_enabled() {
  const char* e = getenv("DQ_FREQ_XFIXED");  // (read per batch: A/B in one process)
  return !e || atoi(e) != 0;
}

// One-utf8-column rows into fixed-capacity bucket pieces (DQ_FREQ_HPIECES=0: chunks only)
static bool hpieces_enabled() {
  const char* e = getenv("DQ_FREQ_HPIECES");  // (read per batch: A/B in one process)
  return !e || atoi(e) != 0;
}

// Exact rows written bucket-major per batch (DQ_FREQ_PIECES=0: the per-tile chunk layout).
static bool pieces_enabled() {
  static const bool on = [] {
    const char* e = getenv("DQ_FREQ_PIECES");
    return !e || atoi(e) != 0;
  }();
  return on;
}

// Pre-pass (rows per workgroup and bucket), its scan, and phase A into bucket pieces; the batch's
// region is the `chunks` chunk slots at f->n_chunks (tiles + workgroup chunks >= rows records).
static dq_status launch_pieces(dq_freq* f, AArgs a, int64_t chunks) {
  int64_t n_wg = 0;
  phaseA_chunks(false, false, a.n_items, a.tile_items, &n_wg);
  a.tiles_per_wg = AKeys<false, false>::kTilesPerWg;
  HIP_TRY(f->ph.ensure((size_t)n_wg * kBuckets));
  HIP_TRY(f->ptot.ensure(kBuckets));
  const size_t rows_need = (size_t)(f->n_prow + n_wg) * kBuckets;
  HIP_TRY(grow_keep(f->pstart, (size_t)f->n_prow * kBuckets, rows_need, f->stream));
  HIP_TRY(grow_keep(f->plen, (size_t)f->n_prow * kBuckets, rows_need, f->stream));
  if (a.dense_words)
    hipLaunchKernelGGL(freq_prepass_x<true>, dim3((unsigned)n_wg), dim3(kPreThreads), 0, f->stream, a, f->ph.p);
  else if (!a.piece_cap)  // (fixed-capacity pieces need no pre-pass)
    hipLaunchKernelGGL(freq_prepass_x<false>, dim3((unsigned)n_wg), dim3(kPreThreads), 0, f->stream, a, f->ph.p);
  if (!a.piece_cap)
    hipLaunchKernelGGL(freq_prepass_scan, dim3(kBuckets), dim3(256), 0, f->stream, f->ph.p, n_wg, f->ptot.p);
  HIP_TRY(hipGetLastError());
  if (a.dense_words) {  // the dense path first (it declines at once when the range is too wide)
    const int g = (int)std::min<int64_t>(kDenseBlocks, (a.n_items + 4 * kDenseThreads - 1) / (4 * kDenseThreads));
    HIP_TRY(f->dense_part.ensure((size_t)kDenseBlocks * kDenseW + 2 * kDenseW));  // + the u64 sums
    auto go = [&](auto kernel) {
      hipLaunchKernelGGL(kernel, dim3((unsigned)g), dim3(kDenseThreads), 0, f->stream, a, f->dense_part.p);
    };
    switch (a.ks.cols[0].type) {
      case DQ_INT8: go(freq_dense_count<DQ_INT8>); break;
      case DQ_INT16: go(freq_dense_count<DQ_INT16>); break;
      case DQ_INT32: go(freq_dense_count<DQ_INT32>); break;
      case DQ_BOOL: go(freq_dense_count<DQ_BOOL>); break;
      default: go(freq_dense_count<DQ_INT64>); break;
    }
    unsigned long long* sums = reinterpret_cast<unsigned long long*>(f->dense_part.p + (size_t)kDenseBlocks * kDenseW);
    hipLaunchKernelGGL(freq_dense_sum, dim3(kDenseW / kDenseSumV), dim3(kBuckets), 0, f->stream, a,
                       f->dense_part.p, g, sums);
    hipLaunchKernelGGL(freq_dense_emit, dim3(kDenseW / kDenseV), dim3(kDenseV), 0, f->stream, a, sums);
    HIP_TRY(hipGetLastError());
    // the host learns (late, without a wait) whether the batch was declined -- copied ahead of
    // the batch's phase A, so the first answer is back while that still runs
    HIP_TRY(f->dense_seen.before_copy(f->stream));
    HIP_TRY(hipMemcpyAsync(f->dense_seen.p, f->dense_words.p + 3, 8, hipMemcpyDeviceToHost, f->stream));
    if (f->dense_epoch == 1) {
      if (!f->dense_ev) HIP_TRY(hipEventCreateWithFlags(&f->dense_ev, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(f->dense_ev, f->stream));
    }
  }
  a.ph = f->ph.p;
  a.ptot = f->ptot.p;
  a.pstart = f->pstart.p + (size_t)f->n_prow * kBuckets;
  a.plen = f->plen.p + (size_t)f->n_prow * kBuckets;
  static const bool generic = [] {  // DQ_FREQ_GENERIC_A=1: A/B hook, the generic kernel
    const char* e = getenv("DQ_FREQ_GENERIC_A");
    return e && atoi(e) != 0;
  }();
  if (generic) {
    if (a.zero_rows)  // (the generic kernel does not zero them)
      HIP_TRY(hipMemsetAsync(a.hist + (size_t)a.zero_off * kHistRow, 0,
                             (size_t)a.zero_rows * kHistRow * sizeof(uint16_t), f->stream));
    a.zero_rows = 0;
    f->nan_counted = false;
    a.piece_cap = 0;  // (the generic kernel lays pieces out by the pre-pass)
    launch_phaseA<false>(f, a, false);
  } else {
    static_assert(kAXThreads == kBuckets, "one bucket per thread");
    a.dbg_clock = nullptr;
    auto go = [&](auto kernel) {
      hipLaunchKernelGGL(kernel, dim3((unsigned)n_wg), dim3(kAXThreads), 0, f->stream, a);
    };
    switch (a.ks.cols[0].type) {  // one kernel per width (one kernel for all spilled heavily)
      case DQ_INT8: go(freq_phaseA_xp<DQ_INT8>); break;
      case DQ_INT16: go(freq_phaseA_xp<DQ_INT16>); break;
      case DQ_INT32: go(freq_phaseA_xp<DQ_INT32>); break;
      case DQ_FLOAT32: go(freq_phaseA_xp<DQ_FLOAT32>); break;
      case DQ_FLOAT64: go(freq_phaseA_xp<DQ_FLOAT64>); break;
      case DQ_BOOL: go(freq_phaseA_xp<DQ_BOOL>); break;
      default: go(freq_phaseA_xp<DQ_INT64>); break;
    }
  }
  HIP_TRY(hipGetLastError());
  const unsigned long long base = (unsigned long long)f->n_chunks * f->tile;
  for (int64_t w = 0; w < n_wg; ++w) f->h_pbase.push_back(base);
  f->n_prow += n_wg;
  // (a dense batch's records are in chunk rows, and so are fixed-capacity pieces' overflows)
  if (!a.dense_words && !a.piece_cap) f->n_empty_chunks += chunks;
  return DQ_OK;
}

// Whether this batch tries the dense path: one integer / boolean key of an exact table that has
// not declined it before (DQ_FREQ_DENSE=0: never).  The declines come back late, through a pinned
// word the stream copies into, so a wide column stops trying after a batch or two.
static bool dense_worth_trying(dq_freq* f, const dq_column& k, int64_t rows) {
  const char* e = getenv("DQ_FREQ_DENSE");  // (read per batch: tests switch it)
  if ((e && atoi(e) == 0) || f->dense_off || !f->exact || f->n_keys != 1 || rows < 4 * kDenseThreads) return false;
  if (k.type != DQ_INT8 && k.type != DQ_INT16 && k.type != DQ_INT32 && k.type != DQ_INT64 &&
      k.type != DQ_BOOL)
    return false;
  if (f->dense_ev && !f->dense_waited && f->dense_epoch == 1) {  // (its phase A keeps the device busy)
    f->dense_waited = true;
    (void)hipEventSynchronize(f->dense_ev);
  }
  if (f->dense_seen.p && *(volatile unsigned long long*)f->dense_seen.p != 0) {
    f->dense_off = true;  // a batch was declined
    return false;
  }
  return true;
}

// ---- finalize: phase B ------------------------------------------------------------------------
static dq_status finalize_b(dq_freq* f) {
  if (f->b_valid) return sync_counters(f);
  const int64_t n_all = f->n_chunks;
  // the non-empty chunks (only when that saves a good part of the finalize)
  int64_t n = n_all;
  const uint32_t* cmap = nullptr;
  if (f->n_empty_chunks == n_all) {  // every chunk row empty (bucket pieces): no read-back
    n = 0;
  } else if (n_all >= 4 * kThreads) {
    const int64_t nb = (n_all + kThreads - 1) / kThreads;
    HIP_TRY(f->chunk_id.ensure(n_all));
    HIP_TRY(f->chunk_boff.ensure(nb + 1));
    hipLaunchKernelGGL(freq_chunk_count, dim3((unsigned)nb), dim3(kThreads), 0, f->stream,
                       f->hist.p, n_all, f->chunk_boff.p);
    hipLaunchKernelGGL(freq_part_scan, dim3(1), dim3(kThreads), 0, f->stream, f->chunk_boff.p, nb);
    HIP_TRY(hipGetLastError());
    unsigned long long m = 0;
    HIP_TRY(d2h(&m, f->chunk_boff.p + nb, 8, f->stream));
    if ((int64_t)m * 4 < n_all * 3) {
      hipLaunchKernelGGL(freq_chunk_ids, dim3((unsigned)nb), dim3(kThreads), 0, f->stream, f->hist.p,
                         n_all, f->chunk_boff.p, f->chunk_id.p);
      HIP_TRY(hipGetLastError());
      n = (int64_t)m;
      cmap = f->chunk_id.p;
    }
  }
  std::fill(f->h_bucket_base.begin(), f->h_bucket_base.end(), 0ULL);
  std::fill(f->h_unit_start.begin(), f->h_unit_start.end(), 0u);
  f->R = 0;
  f->s_bits = 0;
  f->n_units = 0;
  HIP_TRY(f->part_base.ensure(kBuckets + 1));
  const int64_t J = n + f->n_prow;  // segment columns: chunks, then bucket pieces
  f->part_end_ptr = f->part_base.p + 1;  // (the counted layout's ends)
  f->Rcap = 0;
  if (J == 0) {
    HIP_TRY(hipMemsetAsync(f->part_base.p, 0, (kBuckets + 1) * 8, f->stream));
    f->b_valid = true;
    return sync_counters(f);
  }
  HIP_TRY(f->segS.ensure((size_t)kBuckets * J));
  HIP_TRY(f->segP.ensure((size_t)kBuckets * (J + 1)));
  HIP_TRY(f->nseg.ensure(kBuckets));
  HIP_TRY(f->totals.ensure(kBuckets));
  if (n) {
    hipLaunchKernelGGL(freq_hist_transpose, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, f->stream,
                       f->hist.p, n, cmap, f->tile, J, f->segS.p, f->segP.p);
    HIP_TRY(hipGetLastError());
  }
  if (f->n_prow) {
    HIP_TRY(f->pbase.ensure(f->n_prow));
    HIP_TRY(hipMemcpyAsync(f->pbase.p, f->h_pbase.data(), f->n_prow * 8, hipMemcpyHostToDevice,
                           f->stream));
    const int64_t tot = f->n_prow * kBuckets;
    hipLaunchKernelGGL(freq_piece_transpose, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 8192)),
                       dim3(256), 0, f->stream, f->pstart.p, f->plen.p, f->pbase.p, f->n_prow, n, J,
                       f->segS.p, f->segP.p);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(freq_seg_scan, dim3(kBuckets), dim3(kThreads), 0, f->stream, f->segS.p, f->segP.p,
                     J, f->nseg.p, f->totals.p);
  HIP_TRY(hipGetLastError());
  std::vector<unsigned long long> tot(kBuckets);
  if (f->counters_stale) {  // one stream wait for the counters and the bucket totals
    unsigned long long w[C_N + 1];
    const D2HPart parts[2] = {{w, f->dev_words.p, sizeof(w)}, {tot.data(), f->totals.p, kBuckets * 8}};
    HIP_TRY(d2h_n(parts, 2, f->stream));
    apply_counters(f, w);
  } else {
    HIP_TRY(d2h(tot.data(), f->totals.p, kBuckets * 8, f->stream));
  }
  uint64_t R = 0;
  for (auto t : tot) R += t;
  int target = f->exact ? FM<false>::kTarget : FM<true>::kTarget;
  // test hook: a small target forces deep partitioning (all s) on small inputs, a huge one the
  // recount path of overflowing partitions
  if (const char* e = getenv("DQ_FREQ_PARTITION_TARGET")) target = std::max(1, atoi(e));
  if (const char* e = getenv("DQ_FREQ_PARTITION_TARGET_H"))  // (A/B: hashed tables only)
    if (!f->exact) target = std::max(1, atoi(e));
  int s = 0;
  while (s < kMaxSubBits && ((uint64_t)kBuckets << s) * (uint64_t)target < R) ++s;
  // exact tables: one level shallower when the partitions stay packed (pk_ok: s >= kMinPkSubBits,
  // record counts within the count field) and hold <= kTargetPk records on average -- packed
  // slots take up to 4096 -- so phase C's per-item costs cover twice the records (configs[2]
  // 24.75 -> 24.2 ms); a shallower table would fall to the two-word slots (configs[4] +29 ms)
  static const uint64_t kTargetPk = [] {  // DQ_FREQ_TARGET_PK: A/B hook (0: no shallower step)
    const char* e = getenv("DQ_FREQ_TARGET_PK");
    return e ? (uint64_t)std::max(0, atoi(e)) : (uint64_t)3700;
  }();
  if (f->exact && !getenv("DQ_FREQ_PARTITION_TARGET") && kTargetPk)
    while (s - 1 >= kMinPkSubBits && ((uint64_t)kBuckets << (s - 1)) * kTargetPk >= R &&
           f->h_counters[C_MAXCNT] < (1ULL << (s - 1 - 3)))
      --s;
  static const int unit_tiles = [] {  // DQ_FREQ_UNIT_TILES: A/B hook for the phase-B unit size
    const char* e = getenv("DQ_FREQ_UNIT_TILES");
    return e ? std::max(1, atoi(e)) : 0;
  }();
  const uint64_t H = (uint64_t)f->tile * (unit_tiles ? unit_tiles : f->exact ? kUnitTilesX : kUnitTilesH);
  uint32_t u = 0;
  for (int b = 0; b < kBuckets; ++b) {
    f->h_unit_start[b] = u;
    f->h_bucket_base[b + 1] = f->h_bucket_base[b] + tot[b];
    u += (uint32_t)((tot[b] + H - 1) / H);
  }
  f->h_unit_start[kBuckets] = u;
  f->R = R;
  f->s_bits = s;
  f->n_units = u;
  if (getenv("DQ_FREQ_DEBUG")) {
    fprintf(stderr, "dq_freq phase A: notready=%llu diff=%llu full=%llu bypass_tiles=%llu\n",
            (unsigned long long)f->h_counters[C_DBG_NOTREADY],
            (unsigned long long)f->h_counters[C_DBG_DIFF], (unsigned long long)f->h_counters[C_DBG_FULL],
            (unsigned long long)f->h_counters[C_DBG_BYPASS]);
    uint32_t nonempty = 0;
    for (auto t : tot) nonempty += t != 0;
    std::vector<uint32_t> ns(kBuckets);
    (void)d2h(ns.data(), f->nseg.p, kBuckets * 4, f->stream);
    uint64_t segs = 0;
    for (auto v : ns) segs += v;
    fprintf(stderr, "dq_freq finalize: %s chunks=%lld piece_rows=%lld segments=%llu records=%llu s=%d "
            "units=%u buckets=%u\n", f->exact ? "exact" : "hashed", (long long)n, (long long)f->n_prow,
            (unsigned long long)segs, (unsigned long long)R, s, u, nonempty);
  }
  const int64_t P = (int64_t)kBuckets << s;
  HIP_TRY(f->part_base.ensure(P + 1));
  f->part_end_ptr = f->part_base.p + 1;
  f->Rcap = R;
  HIP_TRY(f->unit_start.ensure(kBuckets + 1));
  // (stream-ordered: the host copy is a member, unchanged until the next finalize)
  HIP_TRY(hipMemcpyAsync(f->unit_start.p, f->h_unit_start.data(), (kBuckets + 1) * 4,
                         hipMemcpyHostToDevice, f->stream));
  if (u == 0) {
    HIP_TRY(hipMemsetAsync(f->part_base.p, 0, (P + 1) * 8, f->stream));
    f->b_valid = true;
    return DQ_OK;
  }
  const int S = 1 << s;
  HIP_TRY(f->recsB.ensure(std::max<uint64_t>(R, 1) * f->rb));
  HIP_TRY(f->unit_c0.ensure(u));
  HIP_TRY(f->unit_b.ensure(u));
  HIP_TRY(f->uhist.ensure((size_t)u * S));
  HIP_TRY(hipMemsetAsync(f->unit_c0.p, 0, (size_t)u * 4, f->stream));
  hipLaunchKernelGGL(freq_unit_map, dim3((unsigned)std::min<int64_t>((J + 255) / 256, 64), kBuckets),
                     dim3(256), 0, f->stream, f->segP.p, J, f->nseg.p, f->unit_start.p, (uint32_t)H,
                     f->unit_c0.p, f->unit_b.p);
  HIP_TRY(hipGetLastError());
  BArgs a;
  memset(&a, 0, sizeof(a));
  a.recs = f->recs.p;
  a.segS = f->segS.p;
  a.segP = f->segP.p;
  a.nseg = f->nseg.p;
  a.J = J;
  a.H = (uint32_t)H;
  a.unit_start = f->unit_start.p;
  a.unit_c0 = f->unit_c0.p;
  a.unit_b = f->unit_b.p;
  a.s = s;
  a.n_units = u;
  a.uhist = f->uhist.p;
  a.part_base = f->part_base.p;
  a.recsB = f->recsB.p;
  const unsigned grid = (u + 7) / 8 * 8;
  constexpr uint64_t kUnitX = 16 * kThreads, kUnitH = 4 * kThreads;  // whole-unit capacities
  static const int bsub = [] {  // DQ_FREQ_BSUB: A/B hook for the phase-B3 round size (0: whole units)
    const char* e = getenv("DQ_FREQ_BSUB");
    return e ? atoi(e) : 0;
  }();
  // one unit per workgroup (measured faster than the persistent form: exact, configs[2] 5.08 vs
  // 5.61 ms; hashed, configs[4] 678 vs 826 us per launch once the segment window shares the
  // staging LDS and two workgroups fit a CU).  DQ_FREQ_B3U=1 / DQ_FREQ_B3P=1: A/B hooks
  static const int b3_env = [] {
    const char* e = getenv("DQ_FREQ_B3U");
    const char* p = getenv("DQ_FREQ_B3P");
    return e && atoi(e) ? 1 : (p && atoi(p) ? 2 : 0);
  }();
  const bool b3u = b3_env != 2;
  // Exact tables: the capacity layout, no count pass.  Every partition of bucket b gets room for
  // mean + 8 sqrt(mean) + 32 records (a bijective hash spreads distinct keys uniformly: the
  // overflow odds per partition are ~1e-15), the units' runs are placed by device-scope cursor
  // adds, and a table whose runs overflow anyway (heavy keys whose records all land in one
  // partition) is scattered again by the counted path below, and counts from then on.
  static const bool no_capb = [] {  // DQ_FREQ_CAPB=0: A/B hook, always the counted layout
    const char* e = getenv("DQ_FREQ_CAPB");
    return e && atoi(e) == 0;
  }();
  if (f->exact && !no_capb && !f->cap_failed && bsub == 0 && b3u && H <= kUnitX / 2) {
    std::vector<unsigned long long>& w = f->h_cap_words;
    w.assign(2 * kBuckets + 1, 0ULL);
    // test hook (read per finalize): DQ_FREQ_CAP_SCALE < 1 shrinks the room so runs overflow
    const char* cse = getenv("DQ_FREQ_CAP_SCALE");
    const double cscale = cse ? atof(cse) : 1.0;
    for (int b = 0; b < kBuckets; ++b) {
      const double mean = (double)tot[b] / (double)S;
      const unsigned long long cap =
          tot[b] ? (unsigned long long)std::ceil(cscale * (mean + 8.0 * std::sqrt(mean) + 32.0)) : 0ULL;
      w[kBuckets + 1 + b] = cap;
      w[b + 1] = w[b] + cap * (unsigned long long)S;
    }
    const uint64_t Rcap = w[kBuckets];
    HIP_TRY(f->recsB.ensure(std::max<uint64_t>(Rcap, 1) * f->rb));
    HIP_TRY(f->part_end.ensure(P));
    HIP_TRY(f->cap_words.ensure(2 * kBuckets + 1));
    HIP_TRY(f->b_ovf.ensure(1));
    HIP_TRY(hipMemcpyAsync(f->cap_words.p, w.data(), w.size() * 8, hipMemcpyHostToDevice, f->stream));
    HIP_TRY(hipMemsetAsync(f->b_ovf.p, 0, 4, f->stream));
    hipLaunchKernelGGL(freq_cap_layout, dim3((unsigned)std::min<int64_t>((P + 255) / 256, 4096)), dim3(256),
                       0, f->stream, f->cap_words.p, s, P, f->part_base.p, f->part_end.p);
    a.cap_mode = 1;
    a.recsB = f->recsB.p;
    a.part_end = f->part_end.p;
    a.bcap = f->cap_words.p + kBuckets + 1;
    a.bovf = f->b_ovf.p;
    hipLaunchKernelGGL((freq_phaseB_scatter_u<false, 8>), dim3(grid), dim3(kThreads), 0, f->stream, a);
    HIP_TRY(hipGetLastError());
    unsigned int ovf = 0;
    HIP_TRY(d2h(&ovf, f->b_ovf.p, 4, f->stream));  // (one wait; C would wait for the scatter anyway)
    if (!ovf) {
      f->Rcap = Rcap;
      f->part_end_ptr = f->part_end.p;
      f->b_valid = true;
      return DQ_OK;
    }
    f->cap_failed = true;  // the counted layout, now and for this table's next finalizes
    a.cap_mode = 0;
  }
  static const bool count_w = [] {  // DQ_FREQ_BCOUNT_WAVE=0: A/B hook, a workgroup per unit
    const char* e = getenv("DQ_FREQ_BCOUNT_WAVE");
    return !(e && atoi(e) == 0);
  }();
  const unsigned ugrid = (unsigned)((u + kBcWaves - 1) / kBcWaves);
  if (count_w && f->exact)
    hipLaunchKernelGGL(freq_phaseB_count_w<false>, dim3(ugrid), dim3(kBcWaves * 64), 0, f->stream, a);
  else if (count_w)
    hipLaunchKernelGGL(freq_phaseB_count_w<true>, dim3(ugrid), dim3(kBcWaves * 64), 0, f->stream, a);
  else if (f->exact)
    hipLaunchKernelGGL(freq_phaseB_count<false>, dim3(u), dim3(kThreads), 0, f->stream, a);
  else
    hipLaunchKernelGGL(freq_phaseB_count<true>, dim3(u), dim3(kThreads), 0, f->stream, a);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(freq_phaseB_scan, dim3(kBuckets), dim3(kThreads), 0, f->stream, a);
  HIP_TRY(hipGetLastError());
  if (P <= 4 * kScanTile) {
    hipLaunchKernelGGL(freq_part_scan, dim3(1), dim3(kThreads), 0, f->stream, f->part_base.p, P);
  } else {
    const int64_t nb = (P + kScanTile - 1) / kScanTile;
    HIP_TRY(f->scan_tmp.ensure(nb + 1));
    hipLaunchKernelGGL(scan_u64_sums, dim3((unsigned)nb), dim3(kThreads), 0, f->stream,
                       f->part_base.p, P, f->scan_tmp.p);
    hipLaunchKernelGGL(freq_part_scan, dim3(1), dim3(kThreads), 0, f->stream, f->scan_tmp.p, nb);
    hipLaunchKernelGGL(scan_u64_apply, dim3((unsigned)nb), dim3(kThreads), 0, f->stream,
                       f->part_base.p, P, f->scan_tmp.p);
  }
  HIP_TRY(hipGetLastError());
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, f->device);
  const unsigned pgrid = (unsigned)std::max(8, cus / 8 * 8);  // one per CU (LDS), XCD multiple
  if (bsub == 0 && f->exact && H <= kUnitX && !b3u) {
    hipLaunchKernelGGL((freq_phaseB_scatter_p<false, 16>), dim3(pgrid), dim3(kThreads), 0, f->stream, a);
  } else if (bsub == 0 && !f->exact && H <= kUnitH && !b3u) {
    hipLaunchKernelGGL((freq_phaseB_scatter_p<true, 4>), dim3(pgrid), dim3(kThreads), 0, f->stream, a);
  } else if (bsub == 0 && f->exact && H <= kUnitX / 2) {  // (64 KB staged: two workgroups per CU)
    hipLaunchKernelGGL((freq_phaseB_scatter_u<false, 8>), dim3(grid), dim3(kThreads), 0, f->stream, a);
  } else if (bsub == 0 && f->exact && H <= kUnitX) {
    hipLaunchKernelGGL((freq_phaseB_scatter_u<false, 16>), dim3(grid), dim3(kThreads), 0, f->stream, a);
  } else if (bsub == 0 && !f->exact && H <= kUnitH) {
    hipLaunchKernelGGL((freq_phaseB_scatter_u<true, 4>), dim3(grid), dim3(kThreads), 0, f->stream, a);
  } else if (f->exact) {
    if (bsub == 8192)
      hipLaunchKernelGGL((freq_phaseB_scatter<false, 8192>), dim3(grid), dim3(kThreads), 0, f->stream, a);
    else
      hipLaunchKernelGGL((freq_phaseB_scatter<false, 4096>), dim3(grid), dim3(kThreads), 0, f->stream, a);
  } else {
    if (bsub == 8192)
      hipLaunchKernelGGL((freq_phaseB_scatter<true, 8192>), dim3(grid), dim3(kThreads), 0, f->stream, a);
    else
      hipLaunchKernelGGL((freq_phaseB_scatter<true, 4096>), dim3(grid), dim3(kThreads), 0, f->stream, a);
  }
  HIP_TRY(hipGetLastError());
  f->b_valid = true;
  return DQ_OK;
}

// The partitions' statistics summed in a fixed order into f->red.
static dq_status launch_reduce(dq_freq* f, int64_t P) {
  HIP_TRY(f->scan_tmp.ensure(kRedBlocks * 4));
  const unsigned nbr = (unsigned)std::max<int64_t>(1, std::min<int64_t>(kRedBlocks, (P + kThreads - 1) / kThreads));
  hipLaunchKernelGGL(freq_reduce_part, dim3(nbr), dim3(kThreads), 0, f->stream, f->part_groups.p,
                     f->part_unique.p, f->part_entropy.p, P, f->scan_tmp.p);
  hipLaunchKernelGGL(freq_reduce_final, dim3(1), dim3(64), 0, f->stream, f->scan_tmp.p, (int)nbr,
                     f->red.p);
  HIP_TRY(hipGetLastError());
  return DQ_OK;
}

// ---- finalize: phase C ------------------------------------------------------------------------
// Packed phase-C slots for this table's first pass: at the full depth always (a partition whose
// count field could overflow is handed on); at 7..9 sub-bits only when no record count reaches
// 2^(s-3) (a column of heavy values would hand on nearly every partition: two passes)
static bool pk_ok(const dq_freq* f) {
  if (f->s_bits == kMaxSubBits) return true;
  return f->s_bits >= kMinPkSubBits && f->h_counters[C_MAXCNT] < (1ULL << (f->s_bits - 3));
}

static dq_status finalize_c(dq_freq* f, bool want_groups, bool want_cand) {
  bool reduced = false;  // f->red already holds this pass's sums
  bool read_back = false;  // red_h / cw_h hold the reduction and the counters (one wait for both)
  unsigned long long red_h[6], cw_h[C_N + 1];
  dq_status st = finalize_b(f);
  if (st != DQ_OK) return st;
  const double nr = (double)f->num_rows;
  if (f->c_valid && f->c_num_rows == nr && (!want_groups || f->c_groups) && (!want_cand || f->c_cand))
    return DQ_OK;
  want_groups = want_groups || (f->c_valid && f->c_groups);
  want_cand = want_cand || (f->c_valid && f->c_cand);
  const int64_t P = (int64_t)kBuckets << f->s_bits;
  HIP_TRY(f->part_groups.ensure(P));
  HIP_TRY(f->part_unique.ensure(P));
  HIP_TRY(f->part_off.ensure(P));
  HIP_TRY(f->part_entropy.ensure(2 * P));
  HIP_TRY(f->red.ensure(6));
  HIP_TRY(hipMemsetAsync(f->red.p + 3, 0, 8, f->stream));
  HIP_TRY(f->ovf_n.ensure(1));
  HIP_TRY(hipMemsetAsync(f->part_groups.p, 0, P * 8, f->stream));
  HIP_TRY(hipMemsetAsync(f->part_unique.p, 0, P * 8, f->stream));
  HIP_TRY(hipMemsetAsync(f->part_off.p, 0, P * 8, f->stream));
  HIP_TRY(hipMemsetAsync(f->part_entropy.p, 0, P * 16, f->stream));
  // (groups materialise at their partition's record offsets: the records region's size)
  if (want_groups) HIP_TRY(f->groups.ensure(std::max<uint64_t>(f->Rcap, 1)));
  if (want_cand) {
    HIP_TRY(f->cand.ensure((size_t)P * kCand));
    HIP_TRY(hipMemsetAsync(f->cand.p, 0, (size_t)P * kCand * sizeof(Group), f->stream));
  }
  f->recounted = false;
  if (f->R) {
    CArgs a;
    memset(&a, 0, sizeof(a));
    a.recsB = f->recsB.p;
    a.part_base = f->part_base.p;
    a.part_end = f->part_end_ptr;
    a.s = f->s_bits;
    a.arena = arena_of(f);
    for (int k = 0; k < f->n_keys; ++k) a.types[k] = f->types[k];
    a.n_keys = f->n_keys;
    a.want_cand = want_cand ? 1 : 0;
    a.num_rows = nr;
    a.part_groups = f->part_groups.p;
    a.part_unique = f->part_unique.p;
    a.part_entropy = f->part_entropy.p;
    a.part_off = f->part_off.p;
    a.cand = want_cand ? f->cand.p : nullptr;
    a.groups = want_groups ? f->groups.p : nullptr;
    a.counters = f->dev_words.p;
    if (has_null_literal(f)) {
      a.lit_h = str_row_hash(SView{nullptr, kNullValueLen});
      a.lit_count = f->red.p + 3;
    }
    HIP_TRY(f->ovf_a.ensure(2 * P));
    HIP_TRY(hipMemsetAsync(f->ovf_n.p, 0, 4, f->stream));
    static const bool no_bcache = [] {  // DQ_FREQ_CBCACHE=0: A/B hook, scalar bounds per item
      const char* e = getenv("DQ_FREQ_CBCACHE");
      return e && atoi(e) == 0;
    }();
    a.bcache = !no_bcache && f->Rcap < (1ULL << 32) ? 1u : 0u;
    static const bool no_contig = [] {  // DQ_FREQ_CCONTIG=0: A/B hook, strided phase-C items
      const char* e = getenv("DQ_FREQ_CCONTIG");
      return e && atoi(e) == 0;
    }();
    a.contig = no_contig ? 0u : 1u;
    a.entries = nullptr;
    a.ovf_out = f->ovf_a.p;
    a.ovf_n = f->ovf_n.p;
    a.n_work = (int32_t)P;
    static int dbg = [] {
      const char* e = getenv("DQ_FREQ_DEBUG");
      return e ? atoi(e) : 0;
    }();
    unsigned long long* clk = nullptr;
    if (dbg >= 2 && hipMalloc(&clk, 16 * 8 * sizeof(unsigned long long)) == hipSuccess)
      (void)hipMemset(clk, 0, 16 * 8 * sizeof(unsigned long long));
    else
      clk = nullptr;
    a.dbg_clock = clk;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, f->device);
    const unsigned persistent = (unsigned)std::max(1, cus * 2);
    unsigned grid = (unsigned)std::min<int64_t>(P, persistent);
    static const bool old_c = [] {  // DQ_FREQ_OLDC=1: A/B hook, the generic exact kernel
      const char* e = getenv("DQ_FREQ_OLDC");
      return e && atoi(e) != 0;
    }();
    static const bool old_hc = [] {  // DQ_FREQ_OLDHC=1: A/B hook, the generic hashed kernel
      const char* e = getenv("DQ_FREQ_OLDHC");
      return e && atoi(e) != 0;
    }();
    static const bool no_pk = [] {  // DQ_FREQ_NOPK=1: A/B hook, no packed-slot first pass
      const char* e = getenv("DQ_FREQ_NOPK");
      return e && atoi(e) != 0;
    }();
    for (int round = 0; round < 24; ++round) {
      // packed slots: the first pass of a table partitioned to the full depth (19 fixed bits)
      const bool pk = round == 0 && pk_ok(f) && !no_pk;
      // (packed, partitions of > 2048 records on average: one 1024-thread workgroup per CU)
      const bool big = pk && f->R > (uint64_t)P * 2048;
      const unsigned grid_pk = (unsigned)std::min<int64_t>(P, std::max(1, cus));
      if (f->exact && !old_c && clk && pk && big)
        hipLaunchKernelGGL((freq_phaseC_x<true, true, true>), dim3(grid_pk), dim3(kCThreadsX<true>), 0, f->stream, a);
      else if (f->exact && !old_c && clk && pk)
        hipLaunchKernelGGL((freq_phaseC_x<true, true>), dim3(grid), dim3(kCThreads), 0, f->stream, a);
      else if (f->exact && !old_c && clk)
        hipLaunchKernelGGL((freq_phaseC_x<true, false>), dim3(grid), dim3(kCThreads), 0, f->stream, a);
      else if (f->exact && !old_c && pk && big)
        hipLaunchKernelGGL((freq_phaseC_x<false, true, true>), dim3(grid_pk), dim3(kCThreadsX<true>), 0, f->stream, a);
      else if (f->exact && !old_c && pk)
        hipLaunchKernelGGL((freq_phaseC_x<false, true>), dim3(grid), dim3(kCThreads), 0, f->stream, a);
      else if (f->exact && !old_c)
        hipLaunchKernelGGL((freq_phaseC_x<false, false>), dim3(grid), dim3(kCThreads), 0, f->stream, a);
      else if (f->exact)
        hipLaunchKernelGGL(freq_phaseC<false>, dim3(grid), dim3(kCThreads), 0, f->stream, a);
      else if (round == 0 && !old_hc && clk)
        hipLaunchKernelGGL(freq_phaseC_h<true>, dim3(grid), dim3(kCThreads), 0, f->stream, a);
      else if (round == 0 && !old_hc)
        hipLaunchKernelGGL(freq_phaseC_h<false>, dim3(grid), dim3(kCThreads), 0, f->stream, a);
      else
        hipLaunchKernelGGL(freq_phaseC<true>, dim3(grid), dim3(kCThreads), 0, f->stream, a);
      HIP_TRY(hipGetLastError());
      if (round == 0) {  // the reduction, queued before the wait: read with ovf_n if none overflow
        dq_status rs = launch_reduce(f, P);
        if (rs != DQ_OK) return rs;
        reduced = true;
      }
      unsigned int m = 0;
      if (reduced) {  // the overflow count, the reduction and the counters behind one wait
        const D2HPart parts[3] = {{&m, f->ovf_n.p, 4}, {red_h, f->red.p, sizeof(red_h)},
                                  {cw_h, f->dev_words.p, sizeof(cw_h)}};
        HIP_TRY(d2h_n(parts, 3, f->stream));
        read_back = m == 0;
      } else {
        HIP_TRY(d2h(&m, f->ovf_n.p, 4, f->stream));
      }
      if (m) reduced = false;
      if (clk && ((f->exact && !old_c) || (!f->exact && round == 0 && !old_hc))) {  // C_x / C_h: 8 stamps per item
        unsigned long long h[16 * 8];
        (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
        double acc[7] = {0, 0, 0, 0, 0, 0, 0};
        int ni = 0;
        // 0 top, 4 decoded (top wait), 5 issued (+ tail), 6 inserted, 1 barrier 1, 2 barrier 2, 3 end
        const int order[8] = {0, 4, 5, 6, 1, 2, 3, 8};
        for (int i = 0; i + 1 < 16; ++i) {
          if (!h[(i + 1) * 8]) break;
          for (int q = 0; q < 7; ++q) {
            const unsigned long long t1 = order[q + 1] == 8 ? h[(i + 1) * 8] : h[i * 8 + order[q + 1]];
            acc[q] += (double)(t1 - h[i * 8 + order[q]]) / 100.0;
          }
          ++ni;
        }
        if (ni)
          fprintf(stderr, "dq_freq phase C_x wg0 per item (us): wait+decode %.2f issue+tail %.2f "
                  "cas+append %.2f barrier1 %.2f stats %.2f cand %.2f gap %.2f (%d items)\n",
                  acc[0] / ni, acc[1] / ni, acc[2] / ni, acc[3] / ni, acc[4] / ni, acc[5] / ni,
                  acc[6] / ni, ni);
        (void)hipMemset(clk, 0, sizeof(h));
      } else if (clk) {  // per-item phase times of workgroup 0, us (the wall clock ticks at 100 MHz)
        unsigned long long h[16 * 4];
        (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
        double acc[4] = {0, 0, 0, 0};
        int ni = 0;
        for (int i = 0; i + 1 < 16; ++i) {
          if (!h[(i + 1) * 4]) break;
          acc[0] += (double)(h[i * 4 + 1] - h[i * 4]) / 100.0;
          acc[1] += (double)(h[i * 4 + 2] - h[i * 4 + 1]) / 100.0;
          acc[2] += (double)(h[i * 4 + 3] - h[i * 4 + 2]) / 100.0;
          acc[3] += (double)(h[(i + 1) * 4] - h[i * 4 + 3]) / 100.0;
          ++ni;
        }
        if (ni)
          fprintf(stderr, "dq_freq phase C%s wg0 per item (us): inserts %.2f stats %.2f "
                  "entropy+cand %.2f tail %.2f (%d items, grid %u, round %d)\n",
                  f->exact ? " exact" : " hashed", acc[0] / ni, acc[1] / ni, acc[2] / ni,
                  acc[3] / ni, ni, grid, round);
        (void)hipMemset(clk, 0, sizeof(h));
      }
      if (m == 0) break;
      if (round == 23) {
        if (clk) (void)hipFree(clk);
        return fail(DQ_ERR_OUT_OF_MEMORY, "frequency partition does not fit");
      }
      // recount the overflowing partitions over disjoint hash subsets
      // (a packed-slot first pass hands whole partitions on: no hash subsets yet)
      // (so does the hashed first pass)
      if (!(round == 0 && pk_ok(f) && !no_pk && f->exact && !old_c) &&
          !(round == 0 && !f->exact && !old_hc))
        f->recounted = true;
      f->ovf_a.swap(f->ovf_b);  // ovf_b = this round's entries
      HIP_TRY(f->ovf_a.ensure(2 * (size_t)m));
      HIP_TRY(hipMemsetAsync(f->ovf_n.p, 0, 4, f->stream));
      a.entries = f->ovf_b.p;
      a.ovf_out = f->ovf_a.p;
      a.n_work = (int32_t)m;
      grid = std::min<unsigned>(m, persistent);
    }
    if (clk) (void)hipFree(clk);
  }
  if (!reduced) {
    dq_status rs = launch_reduce(f, P);
    if (rs != DQ_OK) return rs;
  }
  unsigned long long r[6];
  if (read_back) {
    memcpy(r, red_h, sizeof(r));
  } else {
    HIP_TRY(d2h(r, f->red.p, sizeof(r), f->stream));
  }
  f->st_groups = r[0];
  f->st_unique = r[1];
  f->st_entropy = __builtin_bit_cast(double, r[2]);
  f->st_literal = r[3];
  f->st_entropy_fix = (fix128)(((unsigned __int128)r[5] << 64) | r[4]);
  f->c_valid = true;
  f->c_num_rows = nr;
  f->c_groups = want_groups;
  f->c_cand = want_cand;
  f->n_compact = -1;
  if (read_back) {
    apply_counters(f, cw_h);
    return DQ_OK;
  }
  return pull_counters(f);
}

// The materialised groups, compacted: f->compact[0 .. f->n_compact).
static dq_status compact_groups(dq_freq* f) {
  dq_status st = finalize_c(f, true, false);
  if (st != DQ_OK) return st;
  if (f->n_compact >= 0) return DQ_OK;
  const int64_t P = (int64_t)kBuckets << f->s_bits;
  std::vector<unsigned long long> cnt(P), dst(P);
  HIP_TRY(d2h(cnt.data(), f->part_groups.p, P * 8, f->stream));
  unsigned long long tot = 0;
  for (int64_t p = 0; p < P; ++p) {
    dst[p] = tot;
    tot += cnt[p];
  }
  HIP_TRY(f->compact.ensure(std::max<unsigned long long>(tot, 1)));
  if (tot) {
    DevBuf<unsigned long long> d;
    HIP_TRY(d.ensure(P));
    HIP_TRY(hipMemcpy(d.p, dst.data(), P * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(freq_compact, dim3((unsigned)std::min<int64_t>(P, 65536)), dim3(256), 0,
                       f->stream, f->groups.p, f->part_off.p, f->part_groups.p, d.p, P,
                       f->compact.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(f->stream));
  }
  f->n_compact = (int64_t)tot;
  return DQ_OK;
}

// str_row_hash of an arena-encoded utf8 part (tag, length, bytes zero-padded to 4): the bytes
// start dword-aligned, so a key of <= 16 bytes is read as its dwords (no byte loop), masked to its
// length, and hashed from registers (str_row_hash_reg == str_row_hash for such keys).
DQ_DEV uint64_t enc_str_hash(const uint32_t* part) {
  const int32_t len = (int32_t)part[1];
  if (len > 16) return str_row_hash(SView{reinterpret_cast<const uint8_t*>(part + 2), len});
  const int nd = (len + 3) >> 2;
  uint32_t d[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = k < nd ? part[2 + k] : 0u;
  const uint32_t tail = (uint32_t)len & 3u;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (tail && k == nd - 1) d[k] &= (1u << (8 * tail)) - 1u;
  const uint64_t w0 = (uint64_t)d[0] | ((uint64_t)d[1] << 32);
  const uint64_t w1 = (uint64_t)d[2] | ((uint64_t)d[3] << 32);
  return str_row_hash_reg(w0, w1, len);
}

// The marginal of key column k over a hashed table's groups, as records for a one-key table:
// column k's part of a group's encoded key IS the one-column encoding of that value, so a
// record points into the same arena (enc_off), and carries the group's count.  Exact output
// (fixed-width column): key = the value.  Hashed output (utf8): key = the one-column row hash.
__global__ void freq_project(const Group* __restrict__ g, int64_t n, const uint8_t* __restrict__ arena,
                             PartTypes t, int k, RecIn* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* enc = reinterpret_cast<const uint32_t*>(arena + g[i].rep);
  uint32_t w = 0;
  for (int c = 0; c < k; ++c) {  // skip the columns before k
    const uint32_t tag = enc[w++];
    if (!tag) continue;
    if (t.types[c] == DQ_UTF8) w += 1 + pad4(enc[w]) / 4;
    else w += 2;
  }
  RecIn r;
  r.count = g[i].count;
  r.enc_off = g[i].rep + 4ull * w;
  if (t.types[k] == DQ_UTF8) {
    r.key = enc_str_hash(enc + w);
  } else {
    r.key = (uint64_t)enc[w + 1] | ((uint64_t)enc[w + 2] << 32);
  }
  out[i] = r;
}

// Both marginals' records of a two-key table's groups in one pass over the groups and the arena
// (freq_project for key 0 and key 1).
__global__ void freq_project2(const Group* __restrict__ g, int64_t n, const uint8_t* __restrict__ arena,
                              PartTypes t, RecIn* __restrict__ out0, RecIn* __restrict__ out1) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Group gi = g[i];
  const uint32_t* enc = reinterpret_cast<const uint32_t*>(arena + gi.rep);
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    RecIn r;
    r.count = gi.count;
    r.enc_off = gi.rep + 4ull * w;
    const uint32_t tag = enc[w];
    if (t.types[k] == DQ_UTF8) {
      r.key = enc_str_hash(enc + w);
      w += tag ? 2 + pad4(enc[w + 1]) / 4 : 1;
    } else {
      r.key = (uint64_t)enc[w + 1] | ((uint64_t)enc[w + 2] << 32);
      w += tag ? 3 : 1;
    }
    RecIn* o = k ? out1 : out0;  // (nullptr: that side's marginal is built another way)
    if (o) o[i] = r;
  }
}

// ---- small marginals (MutualInformation over a low-cardinality column) ----------------------------
// One pass over the joint groups aggregates each side's marginal in registers and LDS when the
// side has at most kSmallMarg distinct values per wave and keys of at most 8 encoded words: a wave
// keeps its values (row hash + encoded words), matches every group's part against them (hash and
// words), and sums the joint counts per value with one wave reduction per value.  The host merges
// the waves' lists by (hash, words).  A side with more values, a longer key or two values on one
// hash is marked failed and takes the general path (a one-key table of the projected records).
// Also writes every group's row hash of each side (hk[k][i], the hash its marginal is indexed by).
constexpr int kSmallMarg = 16;
struct SmallEntry {
  unsigned long long h, count;
  uint32_t w[8];
};
// freq_small_marginal's per-wave lists of the small sides merged on the device (one workgroup per
// side): values claimed by hash in an LDS table, counts added, then every entry's words checked
// against the first entry of its hash -- the host reads a few KB instead of every wave's list (12.6
// MB for a 1.2e8-group joint, ~4 ms of copies and map inserts).  out_n[k]: the merged values, or
// kSmallMergeHost (more values than the table takes: the host merges the lists as before), or
// kSmallMergeClash (two values on one hash, or the side failed: not small).
constexpr int kSmallMergeSlots = 1024, kSmallMerged = 512;
constexpr uint32_t kSmallMergeHost = 0xFFFFFFFFu, kSmallMergeClash = 0xFFFFFFFEu;
__global__ void __launch_bounds__(1024) freq_small_merge(const SmallEntry* __restrict__ ent,
                                                         const uint32_t* __restrict__ nout, int64_t nw,
                                                         const unsigned int* __restrict__ fail,
                                                         SmallEntry* __restrict__ out, uint32_t* __restrict__ out_n) {
  constexpr int S = kSmallMergeSlots;
  constexpr unsigned long long kFree = ~0ULL;
  __shared__ unsigned long long s_h[S], s_c[S], s_first[S];
  __shared__ uint32_t s_w[S][8];
  __shared__ uint32_t s_full, s_clash;
  const int k = blockIdx.x, tid = threadIdx.x;
  if (fail[k]) {
    if (tid == 0) out_n[k] = kSmallMergeClash;
    return;
  }
  for (int i = tid; i < S; i += blockDim.x) {
    s_h[i] = kFree;
    s_c[i] = 0;
    s_first[i] = kFree;
  }
  if (tid == 0) s_full = s_clash = 0;
  __syncthreads();
  // the slot of entry x's hash (claimed when `claim`), or S: none / the table is full
  auto slot_of = [&](const SmallEntry& e, bool claim) -> uint32_t {
    uint32_t sl = (uint32_t)e.h & (S - 1);
    for (int pr = 0; pr < S; ++pr, sl = (sl + 1) & (S - 1)) {
      const unsigned long long old = claim ? atomicCAS(&s_h[sl], kFree, e.h) : s_h[sl];
      if (old == e.h || (claim && old == kFree)) return sl;
      if (!claim && old == kFree) return S;
    }
    return S;
  };
  // a thread per wave list (its count read once); f(e, x) for each entry x of side k
  auto for_entries = [&](auto&& f) {
    for (int64_t gwv = tid; gwv < nw; gwv += blockDim.x) {
      const uint32_t nl = nout[gwv * 2 + k];
      for (uint32_t c = 0; c < nl; ++c) f(ent[(gwv * 2 + k) * kSmallMarg + c], gwv * kSmallMarg + c);
    }
  };
  for_entries([&](const SmallEntry& e, int64_t x) {  // claims, counts, the first entry per value
    const uint32_t sl = e.h == kFree ? (uint32_t)S : slot_of(e, true);
    if (sl == (uint32_t)S) {
      s_full = 1;
      return;
    }
    atomicAdd(&s_c[sl], e.count);
    atomicMin(&s_first[sl], (unsigned long long)x);
  });
  __syncthreads();
  if (s_full) {
    if (tid == 0) out_n[k] = kSmallMergeHost;
    return;
  }
  for_entries([&](const SmallEntry& e, int64_t x) {  // the first entry of each value: its words
    const uint32_t sl = slot_of(e, false);
    if (sl < (uint32_t)S && s_first[sl] == (unsigned long long)x)
      for (int q = 0; q < 8; ++q) s_w[sl][q] = e.w[q];
  });
  __syncthreads();
  for_entries([&](const SmallEntry& e, int64_t) {  // every entry's words against its value's
    const uint32_t sl = slot_of(e, false);
    bool eq = sl < (uint32_t)S;
    for (int q = 0; q < 8 && eq; ++q) eq = s_w[sl][q] == e.w[q];
    if (!eq) s_clash = 1;
  });
  __syncthreads();
  if (tid == 0) {
    uint32_t m = 0;
    for (int sl = 0; sl < S && m <= (uint32_t)kSmallMerged; ++sl) {
      if (s_h[sl] == kFree) continue;
      if (m < (uint32_t)kSmallMerged) {
        SmallEntry o;
        o.h = s_h[sl];
        o.count = s_c[sl];
        for (int j = 0; j < 8; ++j) o.w[j] = s_w[sl][j];
        out[(int64_t)k * kSmallMerged + m] = o;
      }
      ++m;
    }
    out_n[k] = s_clash ? kSmallMergeClash : (m > (uint32_t)kSmallMerged ? kSmallMergeHost : m);
  }
}

// A side's part of an encoded key from the 16 words loaded at the key's start: its word count,
// its row hash (utf8 <= 16 bytes and fixed-width from the words; longer utf8 from memory) and
// its first 8 words (a side with a longer key is not aggregated here)
DQ_DEV void small_part(const uint32_t (&e)[16], uint32_t w, bool utf8, const uint32_t* enc, uint32_t& nw,
                       uint64_t& h, uint32_t (&pw)[8]) {
  uint32_t ww[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) {  // e[w + j] (w <= 6 for a first side of <= 8 words... else memory)
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) v = (uint32_t)q == w + (uint32_t)j ? e[q] : v;
    ww[j] = w + (uint32_t)j < 16u ? v : enc[w + j];
  }
  const uint32_t tag = ww[0];
  if (utf8) {
    const uint32_t len = ww[1];
    nw = tag ? 2u + pad4(len) / 4 : 1u;
    if (!tag) {
      h = 0;
    } else if (len <= 16) {
      const int nd = (int)((len + 3) >> 2);
      uint32_t d[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) d[k] = k < nd ? ww[2 + k] : 0u;
      const uint32_t tail = len & 3u;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (tail && k == nd - 1) d[k] &= (1u << (8 * tail)) - 1u;
      h = str_row_hash_reg((uint64_t)d[0] | ((uint64_t)d[1] << 32), (uint64_t)d[2] | ((uint64_t)d[3] << 32),
                           (int32_t)len);
    } else {
      h = enc_str_hash(enc + w);
    }
  } else {
    nw = tag ? 3u : 1u;
    h = tag ? fmix_bij((uint64_t)ww[1] | ((uint64_t)ww[2] << 32)) : 0;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) pw[j] = (uint32_t)j < nw ? ww[j] : 0u;
}

__global__ void __launch_bounds__(256)
freq_small_marginal(const Group* __restrict__ g, int64_t n, const uint8_t* __restrict__ arena, PartTypes t,
                    uint32_t try_sides, unsigned long long* __restrict__ hk0, unsigned long long* __restrict__ hk1,
                    SmallEntry* __restrict__ out, uint32_t* __restrict__ nout, unsigned int* __restrict__ fail,
                    RecIn* __restrict__ rec0, RecIn* __restrict__ rec1) {
  __shared__ unsigned long long s_h[4][2][kSmallMarg], s_c[4][2][kSmallMarg];
  __shared__ uint32_t s_w[4][2][kSmallMarg][8];
  constexpr int U = 2;  // groups per lane per step, every load of the step in flight together
  const int lane = (int)__lane_id(), wave = threadIdx.x >> 6;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  int nc[2] = {0, 0};
  bool dead[2] = {!(try_sides & 1u), !(try_sides & 2u)};
  for (int64_t base = gw * 64 * U; base < n; base += (int64_t)gridDim.x * 256 * U) {
    Group gi[U];
    bool on[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 64 + lane;
      on[u] = i < n;
      gi[u] = g[on[u] ? i : n - 1];
    }
    uint32_t e[U][16];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t* enc = reinterpret_cast<const uint32_t*>(arena + gi[u].rep);
#pragma unroll
      for (int q = 0; q < 16; ++q) e[u][q] = enc[q];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 64 + lane;
      const uint32_t* enc = reinterpret_cast<const uint32_t*>(arena + gi[u].rep);
      uint32_t w = 0;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        uint32_t nw, pw[8];
        uint64_t h;
        small_part(e[u], w, t.types[k] == DQ_UTF8, enc, nw, h, pw);
        if (on[u]) (k ? hk1 : hk0)[i] = h;
        RecIn* ro = k ? rec1 : rec0;  // freq_project2's record of this side, for a general marginal
        if (ro && on[u]) {            // (a utf8 part's key hash is its row hash)
          RecIn r;
          r.key = t.types[k] == DQ_UTF8 ? h : ((uint64_t)pw[1] | ((uint64_t)pw[2] << 32));
          r.count = gi[u].count;
          r.enc_off = gi[u].rep + 4ull * w;
          ro[i] = r;
        }
        if (!dead[k] && __ballot(on[u] && (!pw[0] || nw > 8u))) dead[k] = true;  // NULL part, long key
        if (!dead[k]) {
          int m = -1;
          for (int c = 0; c < nc[k]; ++c) {
            bool eq = on[u] && m < 0 && s_h[wave][k][c] == h;
#pragma unroll
            for (int j = 0; j < 8; ++j) eq = eq && s_w[wave][k][c][j] == pw[j];
            if (eq) m = c;
          }
          while (true) {
            const uint64_t need = __ballot(on[u] && m < 0);
            if (!need) break;
            if (nc[k] == kSmallMarg) {
              dead[k] = true;
              break;
            }
            const int leader = __builtin_ctzll(need);
            const uint64_t lh = ((uint64_t)__builtin_amdgcn_readlane((int)(h >> 32), leader) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)h, leader);
            uint32_t lw[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) lw[j] = (uint32_t)__builtin_amdgcn_readlane((int)pw[j], leader);
            bool clash = false;  // another value on this hash: not decidable by hash
            for (int c = 0; c < nc[k]; ++c) clash = clash || s_h[wave][k][c] == lh;
            if (clash) {
              dead[k] = true;
              break;
            }
            const int c = nc[k]++;
            if (lane == 0) {
              s_h[wave][k][c] = lh;
              s_c[wave][k][c] = 0;
#pragma unroll
              for (int j = 0; j < 8; ++j) s_w[wave][k][c][j] = lw[j];
            }
            bool eq = on[u] && m < 0 && h == lh;
#pragma unroll
            for (int j = 0; j < 8; ++j) eq = eq && pw[j] == lw[j];
            if (eq) m = c;
          }
          if (!dead[k]) {
            for (int c = 0; c < nc[k]; ++c) {
              const uint64_t sum = __ockl_wfred_add_u64(m == c ? gi[u].count : 0ULL);
              if (lane == 0) s_c[wave][k][c] += sum;
            }
          }
        }
        w += nw;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t slot = gw * 2 + k;
    if (dead[k]) {
      if (lane == 0) {
        nout[slot] = 0u;
        if (try_sides & (1u << k)) atomicOr(&fail[k], 1u);
      }
      continue;
    }
    if (lane < nc[k]) {
      SmallEntry en;
      en.h = s_h[wave][k][lane];
      en.count = s_c[wave][k][lane];
#pragma unroll
      for (int j = 0; j < 8; ++j) en.w[j] = s_w[wave][k][lane][j];
      out[slot * kSmallMarg + lane] = en;
    }
    if (lane == 0) nout[slot] = (uint32_t)nc[k];
  }
}

// ---- MutualInformation (MutualInformation.scala:41-84) -----------------------------------------
// Column k's part of an encoded multi-key group key.
DQ_DEV const uint32_t* enc_part(const uint32_t* enc, const PartTypes& t, int k) {
  uint32_t w = 0;
  for (int c = 0; c < k; ++c) {
    const uint32_t tag = enc[w++];
    if (!tag) continue;
    if (t.types[c] == DQ_UTF8) w += 1 + pad4(enc[w]) / 4;
    else w += 2;
  }
  return enc + w;
}

// Open-addressing index over a one-key table's groups: slot -> group index + 1 (0 = empty).
struct Lookup {
  const Group* g;
  const uint32_t* slots;
  uint64_t mask;
  const uint8_t* arena;
  int32_t type;
  int32_t exact;
  // a marginal group's rep = rep_base + the joint-arena offset of the key part it was made
  // from (dq_freq_marginal copies the joint arena): a part at that offset IS the group's key
  uint64_t rep_base;
};

__global__ void freq_lookup_build(const Group* __restrict__ g, int64_t n, uint64_t mask,
                                  uint32_t* __restrict__ slots) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s = g[i].h & mask;
  while (atomicCAS(&slots[s], 0u, (uint32_t)(i + 1)) != 0u) s = (s + 1) & mask;
}

// The count of the marginal group whose key is the one-column encoding `part`, at offset
// part_off of the joint arena.
DQ_DEV uint64_t lookup_count(const Lookup& L, const uint32_t* part, uint64_t part_off) {
  uint64_t h;
  if (L.exact) {
    h = fmix_bij((uint64_t)part[1] | ((uint64_t)part[2] << 32));
  } else {
    h = enc_str_hash(part);
  }
  for (uint64_t s = h & L.mask;; s = (s + 1) & L.mask) {
    const uint32_t idx = L.slots[s];
    if (!idx) return 0;  // not reachable: every joint value has its marginal group
    const Group& m = L.g[idx - 1];
    if (m.h != h) continue;
    if (L.exact || m.rep == L.rep_base + part_off) return m.count;  // (its own record: no compare)
    const int32_t ty = DQ_UTF8;
    if (enc_equal_arena(reinterpret_cast<const uint32_t*>(L.arena + m.rep), part, &ty, 1)) return m.count;
  }
}

// terms[i] = (pxy/n) ln((pxy/n) / ((px/n)(py/n))), the reference's UDF (MutualInformation.scala:
// 61-64) with its operation order, per joint group
__global__ void freq_mi_terms(const Group* __restrict__ gj, int64_t n, const uint8_t* __restrict__ arena,
                              PartTypes t, Lookup X, Lookup Y, double total, double* __restrict__ terms) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* enc = reinterpret_cast<const uint32_t*>(arena + gj[i].rep);
  const uint32_t* ex = enc_part(enc, t, 0);
  const uint32_t* ey = enc_part(enc, t, 1);
  const double px = (double)lookup_count(X, ex, gj[i].rep + 4ull * (uint64_t)(ex - enc));
  const double py = (double)lookup_count(Y, ey, gj[i].rep + 4ull * (uint64_t)(ey - enc));
  const double pxy = (double)gj[i].count;
  terms[i] = (pxy / total) * log((pxy / total) / ((px / total) * (py / total)));
}

// A marginal's groups by row hash, for a table with no two keys on one 64-bit hash (its phase C
// counted no collision): slot = {row hash, count}, count 0 = empty, so a lookup is one probe
// sequence with no key bytes compared.
struct CountSlot {
  unsigned long long h, count;
};
// -sum (c/n) ln(c/n) over a small marginal's value counts (count 0: an empty slot), as the
// fixed-point sum phase C keeps (same device entropy_term, so the same bits as a table's)
__global__ void __launch_bounds__(256) freq_slots_entropy(const CountSlot* __restrict__ t, uint64_t n_slots,
                                                          double num_rows, unsigned long long* out) {
  fix128 e = 0;
  for (uint64_t i = threadIdx.x; i < n_slots; i += 256)
    if (t[i].count) e += fix_of(entropy_term(t[i].count, num_rows));
  e = wave_sum_fix(e);
  if (__lane_id() == 0 && e) atomic_add_fix(out, e);
}
__global__ void freq_count_index(const Group* __restrict__ g, int64_t n, uint64_t mask,
                                 CountSlot* __restrict__ slots) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Group gi = g[i];
  uint64_t s = gi.h & mask;
  while (atomicCAS(&slots[s].count, 0ULL, (unsigned long long)gi.count) != 0ULL) s = (s + 1) & mask;
  slots[s].h = gi.h;
}
// Per-partition form (the marginal's phase C partitions, built in LDS, no global atomics):
// partition p = h >> part_shift owns slots [pbase[p], pbase[p] + 2^plog[p]), probed from h's low
// bits.  pbase == nullptr: one table of mask + 1 slots.
struct CountIndex {
  const CountSlot* slots;
  uint64_t mask;
  const unsigned long long* pbase;
  const uint8_t* plog;
  int part_shift;
};
constexpr int kIdxMaxLog = 12;  // the largest per-partition table built in LDS (64 KB)
__global__ void __launch_bounds__(256)
freq_count_index_parts(const Group* __restrict__ groups, const unsigned long long* __restrict__ part_off,
                       const unsigned long long* __restrict__ part_groups, int64_t P,
                       const unsigned long long* __restrict__ pbase, const uint8_t* __restrict__ plog,
                       CountSlot* __restrict__ slots) {
  __shared__ unsigned long long s_h[1 << kIdxMaxLog], s_c[1 << kIdxMaxLog];
  for (int64_t p = blockIdx.x; p < P; p += gridDim.x) {
    const uint32_t R = 1u << plog[p];
    const uint64_t off = part_off[p], n = part_groups[p];
    for (uint32_t j = threadIdx.x; j < R; j += 256) s_c[j] = 0;
    __syncthreads();
    for (uint64_t i = threadIdx.x; i < n; i += 256) {
      const Group gi = groups[off + i];
      uint32_t sl = (uint32_t)gi.h & (R - 1);
      while (atomicCAS(&s_c[sl], 0ULL, (unsigned long long)gi.count) != 0ULL) sl = (sl + 1) & (R - 1);
      s_h[sl] = gi.h;
    }
    __syncthreads();
    CountSlot* out = slots + pbase[p];
    for (uint32_t j = threadIdx.x; j < R; j += 256) out[j] = CountSlot{s_c[j] ? s_h[j] : 0ULL, s_c[j]};
    __syncthreads();
  }
}
DQ_DEV uint64_t count_of(const CountIndex& x, uint64_t h) {
  const CountSlot* sl = x.slots;
  uint64_t mask = x.mask;
  if (x.pbase) {
    const uint64_t p = h >> x.part_shift;
    sl += x.pbase[p];
    mask = (1ULL << x.plog[p]) - 1;
  }
  for (uint64_t s = h & mask;; s = (s + 1) & mask) {
    const CountSlot c = sl[s];
    if (c.h == h || c.count == 0) return c.count;  // (count 0: not reachable, every joint value has its group)
  }
}
// freq_mi_terms with both marginals looked up by the row hashes the projection computed (exact
// keys: the bijective hash of the value), same arithmetic and order
// (k0 / k1: each side's key of group i at k[i * stride]: a RecIn's key (stride 3; exact: the
// value, hashed here) or freq_small_marginal's row hash (stride 1))
__global__ void freq_mi_terms_h(const Group* __restrict__ gj, int64_t n, const uint64_t* __restrict__ k0,
                                int st0, const uint64_t* __restrict__ k1, int st1, int exact0, int exact1,
                                CountIndex x0, CountIndex x1, double total, double* __restrict__ terms) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h0 = exact0 ? fmix_bij(k0[i * st0]) : k0[i * st0];
  const uint64_t h1 = exact1 ? fmix_bij(k1[i * st1]) : k1[i * st1];
  const double px = (double)count_of(x0, h0);
  const double py = (double)count_of(x1, h1);
  const double pxy = (double)gj[i].count;
  terms[i] = (pxy / total) * log((pxy / total) / ((px / total) * (py / total)));
}

// Order-independent sum of the MutualInformation terms (the joint groups' order is phase C's
// output order, which varies from run to run): each term in fixed point (fix_of), summed as
// integers; a non-finite term (a marginal count that is not there) is added as a double beside
// (NaN / inf sums do not depend on order either).  partial[b] = {lo, hi, non-finite sum bits}.
__global__ void __launch_bounds__(256) freq_sum_fix(const double* __restrict__ x, int64_t n,
                                                    unsigned long long* __restrict__ partial) {
  __shared__ fix128 s_red[256 / 64];
  __shared__ double s_nf[256 / 64];
  fix128 acc = 0;
  double nf = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double t = x[i];
    if (fabs(t) < 16384.0) acc += fix_of(t);
    else nf += t;  // (NaN fails the test too)
  }
  acc = wave_sum_fix(acc);
  nf = block_sum_f64(nf, s_nf);
  if (__lane_id() == 0) s_red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    fix128 t = 0;
    for (int w = 0; w < 256 / 64; ++w) t += s_red[w];
    store_fix(partial + 3 * blockIdx.x, t);
    partial[3 * blockIdx.x + 2] = __builtin_bit_cast(unsigned long long, nf);
  }
}

static PartTypes part_types(const dq_freq* f, int parts) {
  PartTypes t;
  memset(&t, 0, sizeof(t));
  for (int k = 0; k < f->n_keys; ++k) t.types[k] = f->types[k];
  t.n_keys = f->n_keys;
  t.exact = f->exact ? 1 : 0;
  t.parts = (uint32_t)parts;
  return t;
}

// Records (+ var bytes) of `n` device groups cut into `parts` owner segments.
static dq_status owner_sizes(dq_freq* f, const Group* g, int64_t n, int parts,
                             std::vector<unsigned long long>& rec, std::vector<unsigned long long>& var) {
  if (f->exact && parts == 1) {  // one segment of n fixed-size records: nothing to count
    rec.assign(1, (unsigned long long)n);
    var.assign(1, 0ULL);
    return DQ_OK;
  }
  DevBuf<unsigned long long> cnt;
  HIP_TRY(cnt.ensure(2 * kMaxParts));
  HIP_TRY(hipMemsetAsync(cnt.p, 0, 2 * kMaxParts * 8, f->stream));
  if (n)
    hipLaunchKernelGGL(freq_owner_count, dim3(grid_for(n)), dim3(256), 0, f->stream, g, n,
                       arena_of(f), part_types(f, parts), cnt.p, cnt.p + kMaxParts);
  HIP_TRY(hipGetLastError());
  std::vector<unsigned long long> h(2 * kMaxParts);
  HIP_TRY(d2h(h.data(), cnt.p, h.size() * 8, f->stream));
  rec.assign(h.begin(), h.begin() + parts);
  var.assign(h.begin() + kMaxParts, h.begin() + kMaxParts + parts);
  return DQ_OK;
}

static dq_status owner_scatter(dq_freq* f, const Group* g, int64_t n, int parts, RecIn* out_rec,
                               uint8_t* out_var, const std::vector<unsigned long long>& rec,
                               const std::vector<unsigned long long>& var) {
  std::vector<unsigned long long> base(4 * kMaxParts, 0);
  unsigned long long tr = 0, tv = 0;
  for (int i = 0; i < parts; ++i) {
    base[i] = tr;
    base[kMaxParts + i] = tv;
    tr += rec[i];
    tv += var[i];
  }
  if (!tr) return DQ_OK;
  DevBuf<unsigned long long> d;
  HIP_TRY(d.ensure(base.size()));
  HIP_TRY(hipMemcpyAsync(d.p, base.data(), base.size() * 8, hipMemcpyHostToDevice, f->stream));
  hipLaunchKernelGGL(freq_owner_scatter, dim3(grid_for(n)), dim3(256), 0, f->stream, g, n,
                     arena_of(f), part_types(f, parts), d.p, d.p + kMaxParts, d.p + 2 * kMaxParts,
                     d.p + 3 * kMaxParts, out_rec, out_var);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(f->stream));
  return DQ_OK;
}

// Encoded keys (export format) of device groups, assembled on the host.
static dq_status encode_groups(dq_freq* f, const Group* g, int64_t n, std::vector<int64_t>& counts,
                               std::vector<int64_t>& offs, std::vector<uint8_t>& bytes) {
  auto put32 = [&](uint32_t v) {
    for (int b = 0; b < 4; ++b) bytes.push_back((uint8_t)(v >> (8 * b)));
  };
  if (n == 0) return DQ_OK;
  std::vector<unsigned long long> rec, var;
  dq_status st = owner_sizes(f, g, n, 1, rec, var);
  if (st != DQ_OK) return st;
  DevBuf<RecIn> dr;
  DevBuf<uint8_t> dv;
  HIP_TRY(dr.ensure(rec[0]));
  HIP_TRY(dv.ensure(std::max<unsigned long long>(var[0], 1)));
  st = owner_scatter(f, g, n, 1, dr.p, dv.p, rec, var);
  if (st != DQ_OK) return st;
  std::vector<RecIn> hr(rec[0]);
  std::vector<uint8_t> hv(var[0]);
  const D2HPart parts[2] = {{hr.data(), dr.p, rec[0] * sizeof(RecIn)}, {hv.data(), dv.p, var[0]}};
  HIP_TRY(d2h_n(parts, var[0] ? 2 : 1, f->stream));
  for (const RecIn& r : hr) {
    offs.push_back((int64_t)bytes.size());
    counts.push_back((int64_t)r.count);
    if (f->exact) {
      put32(1);
      put32((uint32_t)r.key);
      put32((uint32_t)(r.key >> 32));
    } else {
      const uint8_t* e = hv.data() + r.enc_off;
      const uint32_t sz = enc_size(reinterpret_cast<const uint32_t*>(e), f->types.data(), f->n_keys);
      bytes.insert(bytes.end(), e, e + sz);
    }
  }
  return DQ_OK;
}

static void put_null_group(dq_freq* f, std::vector<int64_t>& counts, std::vector<int64_t>& offs,
                           std::vector<uint8_t>& bytes) {
  offs.push_back((int64_t)bytes.size());
  counts.push_back((int64_t)f->h_counters[C_NULL_GROUP]);
  for (int b = 0; b < 4; ++b) bytes.push_back(0);  // tag 0 = NULL
}

// Top `k` groups by count of a device Group array (count 0 entries are holes): the count range
// holding the k-th largest is narrowed with histograms until it is one value (ties are
// arbitrary, like rdd.top) or small enough to bring to the host.
static dq_status select_top(dq_freq* f, const Group* arr, int64_t n, int k, std::vector<Group>& out) {
  out.clear();
  if (n == 0 || k <= 0) return DQ_OK;
  constexpr int kBins = 1024;
  constexpr uint64_t kSmall = 4096;
  DevBuf<unsigned long long> hist;
  HIP_TRY(hist.ensure(kBins + 2));
  std::vector<unsigned long long> hb(kBins);
  auto run_hist = [&](uint64_t lo, uint64_t hi, uint64_t width, int nb) -> dq_status {
    HIP_TRY(hipMemsetAsync(hist.p, 0, kBins * 8, f->stream));
    // (512 workgroups, a few groups per thread: one global add per workgroup and bin -- 4096
    // workgroups' adds on one bin serialised in L2, 53 us per 1e6 candidates)
    hipLaunchKernelGGL(freq_group_hist, dim3(grid_for(n, 512)), dim3(256), 0, f->stream, arr, n, lo, hi,
                       width, hist.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(d2h(hb.data(), hist.p, nb * 8, f->stream));
    return DQ_OK;
  };
  // round 0: powers of two (width 0 selects log2 bins)
  dq_status st = run_hist(1, ~0ULL, 0, 64);
  if (st != DQ_OK) return st;
  uint64_t total = 0;
  for (int j = 0; j < 64; ++j) total += hb[j];
  uint64_t lo, hi, above = 0, inbin;
  if (total <= (uint64_t)k) {
    lo = 1;
    hi = 1;  // take everything
    inbin = 0;
  } else {
    int j = 63;
    while (above + hb[j] < (uint64_t)k) above += hb[j--];
    lo = 1ULL << j;
    hi = j == 63 ? ~0ULL : (1ULL << (j + 1));
    inbin = hb[j];
    while (inbin > kSmall && hi - lo > 1) {
      const uint64_t width = (hi - lo + kBins - 1) / kBins;
      const int nb = (int)((hi - lo + width - 1) / width);
      st = run_hist(lo, hi, width, nb);
      if (st != DQ_OK) return st;
      int i = nb - 1;
      while (above + hb[i] < (uint64_t)k) above += hb[i--];
      const uint64_t lo2 = lo + (uint64_t)i * width;
      hi = std::min(lo2 + width, hi);
      lo = lo2;
      inbin = hb[i];
    }
  }
  const uint64_t cap = hi - lo == 1 ? (uint64_t)k - above : inbin;
  const uint64_t take_cap = std::max<uint64_t>(total <= (uint64_t)k ? total : above, 1);
  DevBuf<Group> take, tie;
  DevBuf<unsigned long long> nt;
  HIP_TRY(take.ensure(take_cap));
  HIP_TRY(tie.ensure(std::max<uint64_t>(cap, 1)));
  HIP_TRY(nt.ensure(2));
  HIP_TRY(hipMemsetAsync(nt.p, 0, 16, f->stream));
  // (512 workgroups: the tie cursor passes `cap` within the first round of waves, later rounds
  // only read it)
  hipLaunchKernelGGL(freq_group_select, dim3(grid_for(n, 512)), dim3(256), 0, f->stream, arr, n, hi, lo,
                     (unsigned long long)cap, take.p, nt.p, nt.p + 1, tie.p);
  HIP_TRY(hipGetLastError());
  // the counts and both buffers at their capacities behind one wait (<= k + 4096 groups: a few
  // tens of KB, against a host round trip per read-back)
  unsigned long long cnts[2];
  std::vector<Group> ht(take_cap), hc(std::max<uint64_t>(cap, 1));
  const D2HPart parts[3] = {{cnts, nt.p, 16}, {ht.data(), take.p, take_cap * sizeof(Group)},
                            {hc.data(), tie.p, cap * sizeof(Group)}};
  HIP_TRY(d2h_n(parts, 3, f->stream));
  const uint64_t nt_take = std::min<uint64_t>(cnts[0], take_cap), nt_tie = std::min<uint64_t>(cnts[1], cap);
  out.assign(ht.begin(), ht.begin() + nt_take);
  out.insert(out.end(), hc.begin(), hc.begin() + nt_tie);
  std::stable_sort(out.begin(), out.end(),
                   [](const Group& x, const Group& y) { return x.count > y.count; });
  if (out.size() > (size_t)k) out.resize(k);
  return DQ_OK;
}

// ------------------------------------------------------------------------------------------------
// Date / timestamp / decimal keys.  Grouping on cast(col as string) (Histogram.scala:63) or on the
// value (GroupingAnalyzers.scala:62-72) puts the same rows together for these types (the casts to
// string are injective at a fixed scale and in UTC), so a table groups the values themselves: a
// date as its int32 and a timestamp as its int64 (the same bytes, relabelled), a decimal(p <= 18)
// as its unscaled long (narrowed: the 16-byte value's low word), a decimal(p > 18) as a 16-byte
// string of its little-endian unscaled value (offsets 0, 16, ...; the value buffer is the
// character data, no copy).  Keys export in those physical forms (deequ_amd.h dq_freq_export).
// ------------------------------------------------------------------------------------------------
static int freq_phys_type(int t) {
  if (t == DQ_DATE32) return DQ_INT32;
  if (t == DQ_TIMESTAMP_US) return DQ_INT64;
  if (DQ_TYPE_ID(t) == DQ_DECIMAL128) return DQ_DECIMAL_PRECISION(t) <= 18 ? DQ_INT64 : DQ_UTF8;
  return t;
}

namespace dq {
__global__ void dec_narrow_kernel(const uint64_t* __restrict__ in, int64_t* __restrict__ out,
                                  int64_t rows) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int64_t)in[2 * i];
}
__global__ void iota16_kernel(int32_t* __restrict__ out, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)(16 * i);
}
}  // namespace dq

static dq_status physical_keys(dq_freq* f, const dq_column* keys, int n_keys, hipStream_t st,
                               dq_column* out) {
  for (int k = 0; k < n_keys; ++k) {
    if (keys[k].type != f->logical[k]) return fail(DQ_ERR_WRONG_TYPE, "key %d has the wrong type", k);
    dq_column c = keys[k];
    c.type = f->types[k];
    const int64_t rows = c.length;
    if (DQ_TYPE_ID(f->logical[k]) == DQ_DECIMAL128 && rows > 0) {
      if (!keys[k].values) return fail(DQ_ERR_INVALID_ARGUMENT, "key %d has no values", k);
      const unsigned grid = (unsigned)std::min<int64_t>((rows + 255) / 256, 4096);
      if (c.type == DQ_INT64) {
        if (f->dec_long[k].n < (size_t)rows) {
          HIP_TRY(hipStreamSynchronize(st));  // (the previous batch may still read the buffer)
          HIP_TRY(f->dec_long[k].ensure((size_t)rows));
        }
        hipLaunchKernelGGL(dec_narrow_kernel, dim3(grid), dim3(256), 0, st,
                           static_cast<const uint64_t*>(keys[k].values), f->dec_long[k].p, rows);
        HIP_TRY(hipGetLastError());
        c.values = f->dec_long[k].p;
      } else {  // 16-byte strings over the value buffer itself
        if (rows >= ((int64_t)1 << 27))
          return fail(DQ_ERR_UNSUPPORTED, "decimal(p > 18) key batch of %lld rows (at most 2^27: "
                                          "int32 string offsets)", (long long)rows);
        if (f->dec_off.n < (size_t)rows + 1) {
          HIP_TRY(hipStreamSynchronize(st));
          HIP_TRY(f->dec_off.ensure((size_t)rows + 1));
          hipLaunchKernelGGL(iota16_kernel, dim3((unsigned)std::min<int64_t>((f->dec_off.n + 255) / 256, 4096)),
                             dim3(256), 0, st, f->dec_off.p, (int64_t)f->dec_off.n);
          HIP_TRY(hipGetLastError());
        }
        c.values = f->dec_off.p;
        c.data = static_cast<const uint8_t*>(keys[k].values);
        c.data_bytes = (int32_t)(16 * rows);
      }
    }
    out[k] = c;
  }
  return DQ_OK;
}

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" dq_status dq_freq_create(int device, int n_keys, const int32_t* key_types,
                                    int64_t capacity_hint, dq_freq** out) {
  if (!out || !key_types || n_keys <= 0) return fail(DQ_ERR_INVALID_ARGUMENT, "bad arguments");
  if (n_keys > kMaxKeys) return fail(DQ_ERR_UNSUPPORTED, "at most %d grouping columns", kMaxKeys);
  *out = nullptr;
  auto f = std::make_unique<dq_freq>();
  f->device = device;
  f->n_keys = n_keys;
  f->logical.assign(key_types, key_types + n_keys);
  for (int t : f->logical) {
    const int p = DQ_DECIMAL_PRECISION(t), sc = DQ_DECIMAL_SCALE(t);
    const bool ok = DQ_TYPE_ID(t) == DQ_DECIMAL128 ? ((t >> 24) == 0 && p >= 1 && p <= 38 && sc <= p)
                                                   : (t >= DQ_BOOL && t <= DQ_TIMESTAMP_US);
    if (!ok) return fail(DQ_ERR_INVALID_ARGUMENT, "bad key type %d", t);
    f->types.push_back(freq_phys_type(t));
    f->relabel = f->relabel || f->types.back() != t;
  }
  f->exact = n_keys == 1 && f->types[0] != DQ_UTF8;
  f->tile = f->exact ? FM<false>::kTile : FM<true>::kTile;
  f->rb = f->exact ? FM<false>::kRB : FM<true>::kRB;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(f->dev_words.ensure(C_N + 4));  // counters, arena cursor, small-key words (3)
  // stream-ordered and waited for: the table's later work may run on a non-blocking stream
  HIP_TRY(hipMemsetAsync(f->dev_words.p, 0, (C_N + 4) * 8, nullptr));
  HIP_TRY(hipStreamSynchronize(nullptr));
  if (capacity_hint > 0) {  // the chunks phase A writes for that many rows (+ per-batch rounding)
    int64_t chunks = phaseA_chunks(!f->exact, false, capacity_hint, f->tile, nullptr) +
                     2 * (capacity_hint >> 24) + 16;
    // one utf8 key: + the fixed-capacity bucket pieces (1.5x the rows; dq_freq_add_device), and
    // their piece rows (growing any of them copies the table and waits for the stream)
    const bool hp = !f->exact && n_keys == 1 && f->types[0] == DQ_UTF8 && hpieces_enabled();
    if (f->exact && pieces_enabled() && xfixed_enabled()) {  // + exact fixed-capacity pieces
      int64_t n_wg = 0;
      phaseA_chunks(false, false, capacity_hint, f->tile, &n_wg);
      n_wg += 2 * (capacity_hint >> 24) + 16;
      const int64_t cap = (5 * (int64_t)f->tile * AKeys<false, false>::kTilesPerWg / kBuckets + 3) / 4;
      chunks += (n_wg * kBuckets * cap + f->tile - 1) / f->tile;
    }
    if (hp) {
      int64_t n_wg = 0;
      phaseA_chunks(true, false, capacity_hint, f->tile, &n_wg);
      n_wg += 2 * (capacity_hint >> 24) + 16;
      const int64_t cap = (3 * (int64_t)f->tile * AKeys<true, false>::kTilesPerWg / kBuckets + 1) / 2;
      chunks += (n_wg * kBuckets * cap + f->tile - 1) / f->tile;
      HIP_TRY(f->pstart.ensure((size_t)n_wg * kBuckets));
      HIP_TRY(f->plen.ensure((size_t)n_wg * kBuckets));
    }
    dq_status st = ensure_chunks(f.get(), chunks);
    if (st != DQ_OK) return st;
    if (f->exact && pieces_enabled()) {  // the pre-pass rows too: growing them waits for the stream
      int64_t n_wg = 0;
      phaseA_chunks(false, false, capacity_hint, f->tile, &n_wg);
      n_wg += 2 * (capacity_hint >> 24) + 16;
      HIP_TRY(f->pstart.ensure((size_t)n_wg * kBuckets));
      HIP_TRY(f->plen.ensure((size_t)n_wg * kBuckets));
    }
  }
  *out = f.release();
  return DQ_OK;
}

extern "C" dq_status dq_freq_reset(dq_freq* f, void* hip_stream) {
  if (!f) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  f->stream = reinterpret_cast<hipStream_t>(hip_stream);
  HIP_TRY(hipMemsetAsync(f->dev_words.p, 0, (C_N + 4) * 8, f->stream));
  for (int k = 0; k < C_N; ++k) f->h_counters[k] = 0;
  f->nan_counted = true;
  f->arena_used = 0;
  f->arena_view = nullptr;  // (a reset table owns its keys again)
  f->rec_var_base = 0;
  f->arena_hi = 0;
  f->counters_stale = false;
  f->num_rows = 0;
  f->n_chunks = 0;
  f->n_prow = 0;
  f->n_empty_chunks = 0;
  f->h_pbase.clear();
  f->fast_off = false;  // (a reset table may see keys the small-key path takes again)
  f->mode_null_as_group = -1;
  invalidate(f);
  return DQ_OK;
}

extern "C" void dq_freq_destroy(dq_freq* f) {
  if (!f) return;
  (void)hipSetDevice(f->device);
  (void)hipStreamSynchronize(f->stream);
  if (f->fast_seen.last_copy && f->fast_seen.last_copy != f->stream)
    (void)hipStreamSynchronize(f->fast_seen.last_copy);  // (the word's copies, pinned_word_put)
  if (f->dense_seen.last_copy && f->dense_seen.last_copy != f->stream)
    (void)hipStreamSynchronize(f->dense_seen.last_copy);
  if (f->dense_ev) (void)hipEventDestroy(f->dense_ev);
  delete f;
}

extern "C" dq_status dq_freq_add_device(dq_freq* f, const dq_column* keys, int n_keys,
                                        int null_as_group, void* hip_stream) {
  if (!f || !keys) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (n_keys != f->n_keys) return fail(DQ_ERR_INVALID_ARGUMENT, "expected %d key columns", f->n_keys);
  dq_column phys[kMaxKeys];
  if (f->relabel) {  // the caller's date / timestamp / decimal keys in the table's physical layout
    HIP_TRY(hipSetDevice(f->device));
    const dq_status ps = physical_keys(f, keys, n_keys, reinterpret_cast<hipStream_t>(hip_stream), phys);
    if (ps != DQ_OK) return ps;
    keys = phys;
  }
  if (f->arena_view) return fail(DQ_ERR_STATE, "a table reading another table's keys takes no adds");
  const int mode = null_as_group ? 1 : 0;
  if (f->mode_null_as_group >= 0 && f->mode_null_as_group != mode)
    return fail(DQ_ERR_STATE, "null_as_group must be the same for every batch");
  if (mode && f->n_keys != 1) return fail(DQ_ERR_UNSUPPORTED, "NULL-as-group needs one key column");
  const int64_t rows = keys[0].length;
  for (int k = 0; k < n_keys; ++k) {
    if (keys[k].type != f->types[k]) return fail(DQ_ERR_WRONG_TYPE, "key %d has the wrong type", k);
    if (keys[k].length != rows) return fail(DQ_ERR_INVALID_ARGUMENT, "key columns differ in length");
    if (rows > 0 && !keys[k].values) return fail(DQ_ERR_INVALID_ARGUMENT, "key %d has no values", k);
    if (rows > 0 && keys[k].type == DQ_UTF8 && !keys[k].data)
      return fail(DQ_ERR_INVALID_ARGUMENT, "utf8 key %d has no character data", k);
  }
  f->mode_null_as_group = mode;
  HIP_TRY(hipSetDevice(f->device));
  f->stream = reinterpret_cast<hipStream_t>(hip_stream);
  f->num_rows += rows;
  invalidate(f);
  if (rows == 0) return DQ_OK;
  const int64_t chunks = phaseA_chunks(!f->exact, false, rows, f->tile, nullptr);
  // one utf8 key not tried by the small-key kernel: bucket pieces of fixed capacity after the
  // batch's chunks (1.5x a workgroup's mean rows per bucket; a tile's records past a full piece
  // stay in its chunk), so phase B reads runs of ~60 records instead of ~4 per chunk
  const bool small = small_keys_worth_trying(f, keys[0], rows);
  const bool xpieces = f->exact && pieces_enabled();
  const bool dense = xpieces && dense_worth_trying(f, keys[0], rows);
  int64_t hp_wg = 0, piece_chunks = 0;
  uint32_t hp_cap = 0;
  if (xpieces && !dense && xfixed_enabled()) {
    // exact rows into fixed-capacity pieces (1.25x a workgroup's mean rows per bucket; a tile's
    // records past a full piece stay in its chunk): no pre-pass over the keys
    phaseA_chunks(false, false, rows, f->tile, &hp_wg);
    hp_cap = (uint32_t)((5 * (int64_t)f->tile * AKeys<false, false>::kTilesPerWg / kBuckets + 3) / 4);
    if (const char* e = getenv("DQ_FREQ_XPIECE_CAP"))  // (tests: small pieces, overflowing tiles)
      hp_cap = (uint32_t)std::max(1, std::min(atoi(e), (int)hp_cap));
    const int64_t recs = hp_wg * kBuckets * (int64_t)hp_cap;
    piece_chunks = (recs + f->tile - 1) / f->tile;
    if ((chunks + piece_chunks) * f->tile >= (int64_t)UINT32_MAX) piece_chunks = 0;  // (u32 starts)
    if (!piece_chunks) hp_cap = 0;
  } else if (!f->exact && n_keys == 1 && keys[0].type == DQ_UTF8 && !small && hpieces_enabled()) {
    phaseA_chunks(true, false, rows, f->tile, &hp_wg);
    hp_cap = (uint32_t)((3 * (int64_t)f->tile * AKeys<true, false>::kTilesPerWg / kBuckets + 1) / 2);
    if (const char* e = getenv("DQ_FREQ_HPIECE_CAP"))  // (tests: small pieces, overflowing tiles)
      hp_cap = (uint32_t)std::max(1, std::min(atoi(e), (int)hp_cap));
    const int64_t recs = hp_wg * kBuckets * (int64_t)hp_cap;
    piece_chunks = (recs + f->tile - 1) / f->tile;
    if ((chunks + piece_chunks) * f->tile >= (int64_t)UINT32_MAX) piece_chunks = 0;  // (u32 starts)
  }
  dq_status st = ensure_chunks(f, chunks + piece_chunks);
  if (st != DQ_OK) return st;
  if (!f->exact) {
    // arena room for the worst case (every row its own record), see row_enc_size; a utf8 key's
    // character bytes come from its data_bytes hint, else from its offsets (a device read)
    uint64_t bound = 0;
    for (int k = 0; k < n_keys; ++k) {
      if (keys[k].type == DQ_UTF8) {
        int64_t bytes = keys[k].data_bytes;
        if (bytes <= 0) {
          int32_t first = 0, last = 0;
          HIP_TRY(hipMemcpy(&first, keys[k].values, 4, hipMemcpyDeviceToHost));
          HIP_TRY(hipMemcpy(&last, reinterpret_cast<const int32_t*>(keys[k].values) + rows, 4,
                            hipMemcpyDeviceToHost));
          if (last < first) return fail(DQ_ERR_INVALID_ARGUMENT, "utf8 key %d has bad offsets", k);
          bytes = last - first;
        }
        bound += (uint64_t)rows * (8 + 3 + kNullValueLen + 3) + (uint64_t)bytes;
      } else {
        bound += (uint64_t)rows * 12;
      }
    }
    // + what a small-key attempt that gives the batch up may have reserved
    int64_t n_wg_a = 0;
    phaseA_chunks(true, false, rows, f->tile, &n_wg_a);
    bound += (uint64_t)n_wg_a * (kSmallThreads / 64) * kSmallCand * 16 + kBatchTabs * kBatchSlots * 16;
    bound += (uint64_t)n_wg_a * 32;  // (the string phase A's per-workgroup 16-byte alignment)
    if (f->arena.n < f->arena_hi + bound + 64) {  // may not fit: learn the true use, then grow
      dq_status cs = pull_counters(f);
      if (cs != DQ_OK) return cs;
      if (f->arena.n < f->arena_used + bound + 64)  // room for a few batches per read-back
        HIP_TRY(grow_keep(f->arena, f->arena_used, f->arena_used + 4 * bound + 64, f->stream));
    }
    f->arena_hi += bound;
  }
  AArgs a = base_args(f);
  for (int k = 0; k < n_keys; ++k)
    a.ks.cols[k] = KeyCol{keys[k].type, 0, keys[k].validity, keys[k].values, keys[k].data};
  a.n_items = rows;
  a.tile_items = f->tile;
  if (piece_chunks && f->exact) {  // the piece chunks' rows hold no records (zeroed by phase A)
    a.zero_off = chunks;
    a.zero_rows = piece_chunks;
    a.piece_cap = hp_cap;
    a.piece_base = (uint64_t)chunks * f->tile;
  } else if (piece_chunks) {  // the piece chunks' rows hold no records; the pieces' rows of this batch
    HIP_TRY(hipMemsetAsync(f->hist.p + (size_t)(f->n_chunks + chunks) * kHistRow, 0,
                           (size_t)piece_chunks * kHistRow * sizeof(uint16_t), f->stream));
    const size_t rows_need = (size_t)(f->n_prow + hp_wg) * kBuckets;
    HIP_TRY(grow_keep(f->pstart, (size_t)f->n_prow * kBuckets, rows_need, f->stream));
    HIP_TRY(grow_keep(f->plen, (size_t)f->n_prow * kBuckets, rows_need, f->stream));
    a.pstart = f->pstart.p + (size_t)f->n_prow * kBuckets;
    a.plen = f->plen.p + (size_t)f->n_prow * kBuckets;
    a.piece_cap = hp_cap;
    a.piece_base = (uint64_t)chunks * f->tile;
    const unsigned long long base = (unsigned long long)f->n_chunks * f->tile;
    for (int64_t w = 0; w < hp_wg; ++w) f->h_pbase.push_back(base);
    f->n_prow += hp_wg;
  }
  if (small) {
    dq_status ss = launch_phaseA_small(f, a);
    if (ss != DQ_OK) return ss;
  }
  if (xpieces) {
    if (dense) {
      if (!f->dense_seen.p) {
        HIP_TRY(pinned_word_get(&f->dense_seen.p));
        *f->dense_seen.p = 0;
      }
      if (!f->dense_words.p) {
        HIP_TRY(f->dense_words.ensure(4));
        HIP_TRY(hipMemsetAsync(f->dense_words.p, 0, 4 * 8, f->stream));
      }
      HIP_TRY(hipMemsetAsync(f->dense_words.p, 0, 2 * 8, f->stream));  // the batch's range
      a.dense_words = f->dense_words.p;
      a.dense_epoch = ++f->dense_epoch;
    }
    dq_status ps = launch_pieces(f, a, chunks);  // (and the decline word's copy, when dense)
    if (ps != DQ_OK) return ps;
  } else if (f->exact) {
    f->nan_counted = false;
    launch_phaseA<false>(f, a, false);
  } else {
    launch_phaseA<true>(f, a, false);
  }
  HIP_TRY(hipGetLastError());
  if (small) {  // the host learns (late, without a wait) whether the attempt gave the batch up
    HIP_TRY(f->fast_seen.before_copy(f->stream));
    HIP_TRY(hipMemcpyAsync(f->fast_seen.p, a.fast_words, 8, hipMemcpyDeviceToHost, f->stream));
  }
  f->n_chunks += chunks + piece_chunks;
  f->counters_stale = true;  // read back at finalize / merge / arena growth
  return DQ_OK;
}

extern "C" dq_status dq_freq_summarize(dq_freq* f, dq_freq_summary* out) {
  if (!f || !out) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = finalize_c(f, false, false);
  if (st != DQ_OK) return st;
  int64_t g = (int64_t)f->st_groups, u = (int64_t)f->st_unique;
  double e = f->st_entropy;
  const uint64_t c = f->h_counters[C_NULL_GROUP];
  if (c) {  // exact-mode NULL group (Histogram on a fixed-width column)
    ++g;
    u += c == 1;
    const double p = (double)c / (double)f->num_rows;
    e += -p * std::log(p);
  }
  out->num_rows = f->num_rows;
  out->n_groups = g;
  out->n_unique = u;
  out->n_null_key_rows = (int64_t)f->h_counters[C_NULL_ROWS];
  out->entropy = e;
  return DQ_OK;
}

extern "C" dq_status dq_freq_summarize_keys(dq_freq* f, dq_freq_summary* out) {
  if (!f || !out) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = finalize_c(f, false, false);
  if (st != DQ_OK) return st;
  out->num_rows = f->num_rows;
  out->n_groups = (int64_t)f->st_groups;
  out->n_unique = (int64_t)f->st_unique;
  out->n_null_key_rows = (int64_t)(f->h_counters[C_NULL_ROWS] + f->h_counters[C_NULL_GROUP]);
  out->entropy = f->st_entropy;
  return DQ_OK;
}

static dq_status marginal_of(dq_freq* joint, int key_index, dq_freq* out, void* hip_stream,
                             bool borrow);
static dq_status add_records(dq_freq* f, const dq_freq_record* records, const uint8_t* var,
                             int n_src, const int64_t* src_records, const int64_t* src_var_bytes,
                             int64_t num_rows, const int64_t* special, int null_as_group,
                             void* hip_stream, bool borrow);

extern "C" dq_status dq_freq_marginal(dq_freq* joint, int key_index, dq_freq* out,
                                     void* hip_stream) {
  return marginal_of(joint, key_index, out, hip_stream, false);
}

// borrow: the marginal reads the joint table's arena in place (it must die first)
static dq_status marginal_of(dq_freq* joint, int key_index, dq_freq* out, void* hip_stream,
                             bool borrow) {
  if (!joint || !out) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (joint->exact || joint->n_keys < 2) return fail(DQ_ERR_INVALID_ARGUMENT, "not a multi-key table");
  if (key_index < 0 || key_index >= joint->n_keys) return fail(DQ_ERR_INVALID_ARGUMENT, "bad key index");
  if (out->n_keys != 1 || out->logical[0] != joint->logical[key_index])
    return fail(DQ_ERR_WRONG_TYPE, "the marginal table must have one key of the column's type");
  if (joint->mode_null_as_group > 0) return fail(DQ_ERR_UNSUPPORTED, "marginal of a Histogram table");
  HIP_TRY(hipSetDevice(joint->device));
  dq_status st = compact_groups(joint);
  if (st != DQ_OK) return st;
  const int64_t n = joint->n_compact;
  DevBuf<RecIn> rec;
  HIP_TRY(rec.ensure(std::max<int64_t>(n, 1)));
  if (n) {
    hipLaunchKernelGGL(freq_project, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, joint->stream,
                       joint->compact.p, n, arena_of(joint), part_types(joint, 1), key_index, rec.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(joint->stream));
  }
  static const int dbg = [] {
    const char* e = getenv("DQ_FREQ_DEBUG");
    return e ? atoi(e) : 0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  const int64_t rc[1] = {n};
  const int64_t vb[1] = {(int64_t)((joint->arena_used + 7) & ~7ULL)};
  const int64_t special[3] = {0, 0, (int64_t)joint->h_counters[C_NULL_ROWS]};
  st = add_records(out, reinterpret_cast<const dq_freq_record*>(rec.p), arena_of(joint), 1, rc, vb,
                   joint->num_rows, special, 0, hip_stream, borrow && !out->exact);
  if (st != DQ_OK) return st;
  HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(hip_stream)));
  if (dbg)
    fprintf(stderr, "dq_freq marginal %d: records added in %.2f ms\n", key_index,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return DQ_OK;
}

extern "C" dq_status dq_freq_mutual_information(dq_freq* joint, double* mi, int* is_null,
                                               void* hip_stream) {
  if (!joint || !mi || !is_null) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (joint->exact || joint->n_keys != 2)
    return fail(DQ_ERR_INVALID_ARGUMENT, "MutualInformation needs a two-key grouping table");
  HIP_TRY(hipSetDevice(joint->device));
  dq_status st = compact_groups(joint);
  if (st != DQ_OK) return st;
  const int64_t n = joint->n_compact;
  *mi = 0.0;
  *is_null = n == 0 ? 1 : 0;  // sum over no joint groups is NULL
  if (!n) return DQ_OK;
  hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
  static const int dbg = [] {  // DQ_FREQ_DEBUG: the MI pass's steps, timed (synchronising)
    const char* e = getenv("DQ_FREQ_DEBUG");
    return e ? atoi(e) : 0;
  }();
  auto t_last = std::chrono::steady_clock::now();
  auto stamp = [&](const char* what) {
    if (!dbg) return;
    (void)hipStreamSynchronize(stream);
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "dq_freq MI %s: %.2f ms\n", what,
            std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  dq_freq* marg[2] = {nullptr, nullptr};
  DevBuf<uint32_t> slots[2];
  DevBuf<CountSlot> cslots[2];
  uint64_t cmask[2] = {0, 0};
  Lookup L[2];
  dq_status res = DQ_OK;
  const char* fl = getenv("DQ_FREQ_MI_LOOKUP");  // =1: the byte-compare lookups (A/B, tests)
  const bool force_lookup = fl && atoi(fl) != 0;
  const char* fsm = getenv("DQ_FREQ_MI_NOSMALL");  // =1: no small-marginal pass (A/B, tests)
  bool small[2] = {false, false};  // side k's marginal aggregated by freq_small_marginal
  DevBuf<unsigned long long> hk[2];
  // each side's records of the joint groups (kept: the lookups read their keys), written by the
  // small-marginal pass for both sides (a side that is not small needs them; otherwise
  // freq_project2 makes them in a pass of its own)
  DevBuf<RecIn> rec[2];
  bool rec_done = false;
  if (!force_lookup && !(fsm && atoi(fsm))) {
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>((n + 511) / 512, 1), 2048);
    const int64_t nw = (int64_t)grid * 4;
    DevBuf<SmallEntry> ent;
    DevBuf<uint32_t> nout;
    DevBuf<unsigned int> sfail;
    HIP_TRY(hk[0].ensure(n));
    HIP_TRY(hk[1].ensure(n));
    HIP_TRY(ent.ensure((size_t)nw * 2 * kSmallMarg));
    HIP_TRY(nout.ensure((size_t)nw * 2));
    HIP_TRY(sfail.ensure(2));
    HIP_TRY(rec[0].ensure(n));
    HIP_TRY(rec[1].ensure(n));
    HIP_TRY(hipMemsetAsync(sfail.p, 0, 8, stream));
    hipLaunchKernelGGL(freq_small_marginal, dim3(grid), dim3(256), 0, stream, joint->compact.p, n,
                       arena_of(joint), part_types(joint, 1), 3u, hk[0].p, hk[1].p, ent.p, nout.p, sfail.p,
                       rec[0].p, rec[1].p);
    HIP_TRY(hipGetLastError());
    rec_done = true;
    unsigned int hf[2];
    HIP_TRY(d2h(hf, sfail.p, 8, stream));
    if (!hf[0] || !hf[1]) {  // merge the waves' lists of each small side by (hash, words)
      DevBuf<SmallEntry> mo;
      DevBuf<uint32_t> mn;
      HIP_TRY(mo.ensure(2 * (size_t)kSmallMerged));
      HIP_TRY(mn.ensure(2));
      hipLaunchKernelGGL(freq_small_merge, dim3(2), dim3(1024), 0, stream, ent.p, nout.p, nw, sfail.p, mo.p, mn.p);
      HIP_TRY(hipGetLastError());
      uint32_t hm[2];
      HIP_TRY(d2h(hm, mn.p, 8, stream));
      const char* hmg = getenv("DQ_FREQ_MI_HOSTMERGE");  // =1: the host merge (A/B, tests)
      if (hmg && atoi(hmg))
        for (int k = 0; k < 2; ++k)
          if (hm[k] != kSmallMergeClash) hm[k] = kSmallMergeHost;
      std::vector<SmallEntry> hme(2 * (size_t)kSmallMerged);
      HIP_TRY(d2h(hme.data(), mo.p, hme.size() * sizeof(SmallEntry), stream));
      // (the host merge of every wave's list, for a side the device table could not take)
      std::vector<uint32_t> hn;
      std::vector<SmallEntry> he;
      if ((!hf[0] && hm[0] == kSmallMergeHost) || (!hf[1] && hm[1] == kSmallMergeHost)) {
        hn.resize((size_t)nw * 2);
        he.resize((size_t)nw * 2 * kSmallMarg);
        HIP_TRY(d2h(hn.data(), nout.p, hn.size() * 4, stream));
        HIP_TRY(d2h(he.data(), ent.p, he.size() * sizeof(SmallEntry), stream));
      }
      for (int k = 0; k < 2; ++k) {
        if (hf[k] || hm[k] == kSmallMergeClash) continue;
        const bool host = hm[k] == kSmallMergeHost;
        // (merged on the device: one list of hm[k] entries, as if from one wave)
        const int64_t lists = host ? nw : 1;
        std::map<uint64_t, std::pair<std::array<uint32_t, 8>, uint64_t>> vals;
        bool ok = true;
        for (int64_t gwv = 0; gwv < lists && ok; ++gwv)
          for (uint32_t c = 0; c < (host ? hn[gwv * 2 + k] : hm[k]) && ok; ++c) {
            const SmallEntry& e = host ? he[((size_t)gwv * 2 + k) * kSmallMarg + c]
                                       : hme[(size_t)k * kSmallMerged + c];
            std::array<uint32_t, 8> wv;
            for (int q = 0; q < 8; ++q) wv[q] = e.w[q];
            auto it = vals.find(e.h);
            if (it == vals.end()) vals.emplace(e.h, std::make_pair(wv, (uint64_t)e.count));
            else if (it->second.first != wv) ok = false;  // two values on one hash
            else it->second.second += e.count;
          }
        if (!ok) continue;
        uint64_t cap = 2;
        while (cap < 2 * (uint64_t)vals.size()) cap <<= 1;
        std::vector<CountSlot> tab(cap, CountSlot{0, 0});
        for (const auto& kv : vals) {
          uint64_t sl = kv.first & (cap - 1);
          while (tab[sl].count) sl = (sl + 1) & (cap - 1);
          tab[sl] = CountSlot{kv.first, kv.second.second};
        }
        HIP_TRY(cslots[k].ensure(cap));
        HIP_TRY(hipMemcpy(cslots[k].p, tab.data(), cap * sizeof(CountSlot), hipMemcpyHostToDevice));
        cmask[k] = cap - 1;
        small[k] = true;
      }
    }
    stamp("small marginals");
  }
  for (int k = 0; k < 2; ++k)
    if (!small[k]) HIP_TRY(rec[k].ensure(n));
  if (!rec_done && (!small[0] || !small[1])) {
    hipLaunchKernelGGL(freq_project2, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, joint->stream,
                       joint->compact.p, n, arena_of(joint), part_types(joint, 1),
                       small[0] ? nullptr : rec[0].p, small[1] ? nullptr : rec[1].p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(joint->stream));
  }
  stamp("project");
  bool by_hash = !force_lookup;  // no marginal has two keys on one 64-bit hash
  for (int k = 0; k < 2 && res == DQ_OK; ++k) {
    if (small[k]) continue;
    const int32_t ty = joint->types[k];
    res = dq_freq_create(joint->device, 1, &ty, 0, &marg[k]);
    stamp(k ? "marginal 1 create" : "marginal 0 create");
    if (res == DQ_OK) {
      const int64_t rc[1] = {n};
      const int64_t vb[1] = {(int64_t)((joint->arena_used + 7) & ~7ULL)};
      const int64_t special[3] = {0, 0, (int64_t)joint->h_counters[C_NULL_ROWS]};
      res = add_records(marg[k], reinterpret_cast<const dq_freq_record*>(rec[k].p), arena_of(joint), 1, rc,
                        vb, joint->num_rows, special, 0, hip_stream, !marg[k]->exact);
    }
    stamp(k ? "marginal 1 records" : "marginal 0 records");
    // statistics first: the entropy identity below may make the groups unnecessary
    if (res == DQ_OK) res = finalize_c(marg[k], false, false);
    stamp(k ? "marginal 1 statistics" : "marginal 0 statistics");
    if (res != DQ_OK) break;
    if (marg[k]->h_counters[C_COLLISIONS]) by_hash = false;
  }
  // MI = E(X) + E(Y) - E(X, Y), every entropy normalised by the same numRows as the reference's
  // terms ((pxy/n) ln((pxy/n) / ((px/n)(py/n))) summed over the joint groups, the marginals
  // summed over them too: MutualInformation.scala:41-75) -- exact algebra over the fixed-point
  // sums of the tables' own -p ln p terms (the joint's and a general side's from phase C, a small
  // side's from its value counts with the same device term).  Taken when MI >= 1/100 of
  // E(X) + E(Y) + E(X, Y): each entropy's rounding is then below 1e-13 of MI (two columns close
  // to independent keep the per-group terms, whose sum does not cancel).
  if (res == DQ_OK) {
    fix128 ex[2];
    for (int k = 0; k < 2 && res == DQ_OK; ++k) {
      if (!small[k]) {
        ex[k] = marg[k]->st_entropy_fix;
        continue;
      }
      DevBuf<unsigned long long> acc;
      unsigned long long w[2];
      if (acc.ensure(2) != hipSuccess || hipMemsetAsync(acc.p, 0, 16, stream) != hipSuccess) {
        res = fail(DQ_ERR_OUT_OF_MEMORY, "MutualInformation entropy");
        break;
      }
      hipLaunchKernelGGL(freq_slots_entropy, dim3(1), dim3(256), 0, stream, cslots[k].p, cmask[k] + 1,
                         (double)joint->num_rows, acc.p);
      if (hipGetLastError() != hipSuccess || d2h(w, acc.p, 16, stream) != hipSuccess) {
        res = fail(DQ_ERR_DEVICE, "MutualInformation entropy");
        break;
      }
      ex[k] = (fix128)(((unsigned __int128)w[1] << 64) | w[0]);
    }
    if (res == DQ_OK) {
      const fix128 exy = joint->st_entropy_fix, v = ex[0] + ex[1] - exy;
      if (v > 0 && v * 100 >= ex[0] + ex[1] + exy) {
        *mi = fix_to_f64(v);
        for (int k = 0; k < 2; ++k)
          if (marg[k]) dq_freq_destroy(marg[k]);
        stamp("entropy identity");
        return DQ_OK;
      }
    }
  }
  for (int k = 0; k < 2 && res == DQ_OK; ++k) {  // the per-group terms: each general side's groups
    if (small[k]) continue;
    // (the groups stay where phase C put them, per partition; compacted only for the
    // byte-compare lookups)
    res = finalize_c(marg[k], true, false);
    stamp(k ? "marginal 1 groups" : "marginal 0 groups");
  }
  if (res == DQ_OK && !by_hash && (small[0] || small[1])) {
    // a general side counted a hash collision: the byte-compare lookups need both sides as
    // tables, so the small sides are built the general way too
    for (int k = 0; k < 2 && res == DQ_OK; ++k) {
      if (!small[k]) continue;
      small[k] = false;
      if (rec[k].ensure(n) != hipSuccess) {
        res = fail(DQ_ERR_OUT_OF_MEMORY, "MutualInformation records");
        break;
      }
      hipLaunchKernelGGL(freq_project, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, joint->stream,
                         joint->compact.p, n, arena_of(joint), part_types(joint, 1), k, rec[k].p);
      const int32_t ty = joint->types[k];
      res = dq_freq_create(joint->device, 1, &ty, 0, &marg[k]);
      if (res == DQ_OK) {
        const int64_t rc[1] = {n};
        const int64_t vb[1] = {(int64_t)((joint->arena_used + 7) & ~7ULL)};
        const int64_t special[3] = {0, 0, (int64_t)joint->h_counters[C_NULL_ROWS]};
        res = add_records(marg[k], reinterpret_cast<const dq_freq_record*>(rec[k].p), arena_of(joint), 1,
                          rc, vb, joint->num_rows, special, 0, hip_stream, !marg[k]->exact);
      }
      if (res == DQ_OK) res = compact_groups(marg[k]);
    }
  }
  CountIndex X[2];
  DevBuf<unsigned long long> pbase[2];
  DevBuf<uint8_t> plog[2];
  for (int k = 0; k < 2; ++k) X[k] = CountIndex{cslots[k].p, cmask[k], nullptr, nullptr, 0};
  for (int k = 0; k < 2 && res == DQ_OK; ++k) {
    if (small[k]) continue;
    const int32_t ty = joint->types[k];
    if (by_hash) {  // per partition, in LDS, when every partition's table fits
      dq_freq* mg = marg[k];
      const int64_t P = (int64_t)kBuckets << mg->s_bits;
      std::vector<unsigned long long> cnt(P), base(P);
      std::vector<uint8_t> lg(P);
      if (d2h(cnt.data(), mg->part_groups.p, P * 8, mg->stream) != hipSuccess) {
        res = fail(DQ_ERR_DEVICE, "marginal index");
        break;
      }
      unsigned long long tot = 0;
      bool fits = true;
      for (int64_t q = 0; q < P; ++q) {
        int l = 4;
        while ((1ULL << l) < 2 * cnt[q]) ++l;
        fits = fits && l <= kIdxMaxLog;
        lg[q] = (uint8_t)l;
        base[q] = tot;
        tot += 1ULL << l;
      }
      if (fits) {
        if (cslots[k].ensure(tot) != hipSuccess || pbase[k].ensure(P) != hipSuccess ||
            plog[k].ensure(P) != hipSuccess ||
            hipMemcpy(pbase[k].p, base.data(), P * 8, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(plog[k].p, lg.data(), P, hipMemcpyHostToDevice) != hipSuccess) {
          res = fail(DQ_ERR_OUT_OF_MEMORY, "marginal index");
          break;
        }
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, joint->device);
        hipLaunchKernelGGL(freq_count_index_parts, dim3((unsigned)std::min<int64_t>(P, 2 * cus)), dim3(256), 0,
                           mg->stream, mg->groups.p, mg->part_off.p, mg->part_groups.p, P, pbase[k].p,
                           plog[k].p, cslots[k].p);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(mg->stream) != hipSuccess) {
          res = fail(DQ_ERR_DEVICE, "marginal index");
          break;
        }
        X[k] = CountIndex{cslots[k].p, 0, pbase[k].p, plog[k].p, 64 - kBucketBits - mg->s_bits};
      } else {  // one table over the compacted groups
        res = compact_groups(mg);
        if (res != DQ_OK) break;
        const int64_t m = mg->n_compact;
        uint64_t cap = 2;
        while (cap < (uint64_t)(2 * m)) cap <<= 1;
        if (cslots[k].ensure(cap) != hipSuccess ||
            hipMemsetAsync(cslots[k].p, 0, cap * sizeof(CountSlot), stream) != hipSuccess) {
          res = fail(DQ_ERR_OUT_OF_MEMORY, "marginal index");
          break;
        }
        if (m)
          hipLaunchKernelGGL(freq_count_index, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream,
                             mg->compact.p, m, cap - 1, cslots[k].p);
        X[k] = CountIndex{cslots[k].p, cap - 1, nullptr, nullptr, 0};
      }
    } else {
      res = compact_groups(marg[k]);
      if (res != DQ_OK) break;
      const int64_t m = marg[k]->n_compact;
      uint64_t cap = 2;
      while (cap < (uint64_t)(2 * m)) cap <<= 1;
      if (slots[k].ensure(cap) != hipSuccess || hipMemsetAsync(slots[k].p, 0, cap * 4, stream) != hipSuccess) {
        res = fail(DQ_ERR_OUT_OF_MEMORY, "marginal index");
        break;
      }
      if (m)
        hipLaunchKernelGGL(freq_lookup_build, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream,
                           marg[k]->compact.p, m, cap - 1, slots[k].p);
      L[k] = Lookup{marg[k]->compact.p, slots[k].p, cap - 1, arena_of(marg[k]), ty, marg[k]->exact ? 1 : 0,
                    marg[k]->rec_var_base};
    }
    stamp(k ? "marginal 1 index" : "marginal 0 index");
  }
  if (res == DQ_OK) {
    DevBuf<double> terms;
    DevBuf<unsigned long long> partial;
    constexpr int kSumBlocks = 1024;
    if (terms.ensure(n) != hipSuccess || partial.ensure(3 * kSumBlocks) != hipSuccess) {
      res = fail(DQ_ERR_OUT_OF_MEMORY, "MutualInformation terms");
    } else {
      if (by_hash) {
        const uint64_t* kp[2];
        int kst[2], kex[2];
        for (int k = 0; k < 2; ++k) {
          kp[k] = small[k] ? reinterpret_cast<const uint64_t*>(hk[k].p) : reinterpret_cast<const uint64_t*>(rec[k].p);
          kst[k] = small[k] ? 1 : (int)(sizeof(RecIn) / 8);
          kex[k] = small[k] ? 0 : (marg[k]->exact ? 1 : 0);
        }
        hipLaunchKernelGGL(freq_mi_terms_h, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                           joint->compact.p, n, kp[0], kst[0], kp[1], kst[1], kex[0], kex[1], X[0], X[1],
                           (double)joint->num_rows, terms.p);
      } else {
        hipLaunchKernelGGL(freq_mi_terms, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                           joint->compact.p, n, arena_of(joint), part_types(joint, 1), L[0], L[1],
                           (double)joint->num_rows, terms.p);
      }
      stamp("terms");
      hipLaunchKernelGGL(freq_sum_fix, dim3(kSumBlocks), dim3(256), 0, stream, terms.p, n, partial.p);
      std::vector<unsigned long long> h(3 * kSumBlocks);
      if (hipGetLastError() != hipSuccess ||
          d2h(h.data(), partial.p, 3 * kSumBlocks * 8, stream) != hipSuccess) {
        res = fail(DQ_ERR_DEVICE, "MutualInformation launch failed");
      } else {
        fix128 sum = 0;
        double nf = 0.0;
        for (int b = 0; b < kSumBlocks; ++b) {
          sum += (fix128)(((unsigned __int128)h[3 * b + 1] << 64) | h[3 * b]);
          nf += __builtin_bit_cast(double, h[3 * b + 2]);
        }
        *mi = fix_to_f64(sum) + nf;
      }
    }
  }
  stamp("sum");
  for (dq_freq* m : marg) dq_freq_destroy(m);
  stamp("destroy");
  return res;
}

// ---- HLL++ registers from a table's records (ApproxCountDistinct beside a grouping) ------------
// The registers depend only on the set of distinct non-NULL values (StatefulHyperloglogPlus.scala:
// 87-113: each value's XXH64, seed 42, raises one register; merges take the max), and raising a
// register twice changes nothing, so the table's partitioned records -- every distinct value at
// least once, fewer records than rows once phase A has collapsed repeated keys -- yield them
// without a pass over the rows and without counting the groups: each record's value (exact mode:
// the bijective hash, its bucket bits from the record's partition, inverted; one utf8 key: its
// arena bytes) is hashed as Spark hashes its type -- floating-point NaN canonical
// (doubleToLongBits / floatToIntBits), integers narrower than long as Int -- and raises its
// register.  One wave per partition.
DQ_DEV uint64_t hll_value_hash(uint64_t v, int type) {  // v: the widened value (kwiden)
  switch (type) {
    case DQ_INT64: return xxh_long(v, 42);
    case DQ_FLOAT64: {
      const bool nan = (v & 0x7fffffffffffffffULL) > 0x7ff0000000000000ULL;
      return xxh_long(nan ? 0x7ff8000000000000ULL : v, 42);
    }
    case DQ_FLOAT32: {
      const uint32_t b = (uint32_t)v;
      return xxh_int((b & 0x7fffffffu) > 0x7f800000u ? 0x7fc00000u : b, 42);
    }
    default: return xxh_int((uint32_t)v, 42);  // int8 / int16 / int32 / boolean (0 / 1)
  }
}

__global__ void __launch_bounds__(256) freq_hll_records(const uint64_t* __restrict__ recs,
                                                        const unsigned long long* __restrict__ part_base,
                                                        const unsigned long long* __restrict__ part_end,
                                                        int64_t P, int s, int exact, int type,
                                                        const uint8_t* __restrict__ arena,
                                                        uint32_t* __restrict__ regs) {
  __shared__ uint32_t s_reg[kHllM];
  for (int i = threadIdx.x; i < kHllM; i += 256) s_reg[i] = 0;
  __syncthreads();
  const int lane = (int)__lane_id(), wave = threadIdx.x >> 6;
  for (int64_t p = (int64_t)blockIdx.x * 4 + wave; p < P; p += (int64_t)gridDim.x * 4) {
    const uint64_t r0 = part_base[p], r1 = part_end[p];
    const uint32_t b = (uint32_t)(p >> s);
    for (uint64_t i = r0 + lane; i < r1; i += 64) {
      uint64_t x;
      if (exact) {
        x = hll_value_hash(fmix_inv(xrec_h(recs[i], b)), type);
      } else {  // one utf8 key: the encoded {1, len, bytes}
        const uint32_t* e = reinterpret_cast<const uint32_t*>(arena + (recs[2 * i + 1] >> 8));
        x = xxh_bytes(MemBytes{reinterpret_cast<const uint8_t*>(e + 2)}, (int64_t)e[1], 42);
      }
      uint32_t idx, pw;
      hll_index_rank(x, idx, pw);
      if (pw > __hip_atomic_load(&s_reg[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
        atomicMax(&s_reg[idx], pw);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHllM; i += 256)
    if (s_reg[i]) atomicMax(&regs[i], s_reg[i]);
}

extern "C" dq_status dq_freq_hll(dq_freq* f, int64_t max_records, uint64_t* words, int* done,
                                 void* hip_stream) {
  if (!f || !words || !done) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  *done = 0;
  if (f->n_keys != 1 || (!f->exact && f->types[0] != DQ_UTF8)) return DQ_OK;  // (not one value)
  // a decimal(p > 18) table holds 16-byte strings, which Spark hashes as BigInteger.toByteArray,
  // not these bytes: the caller scans (decimal(p <= 18) keys are the unscaled longs, hashLong --
  // Spark's; dates / timestamps are their int32 / int64, hashInt / hashLong -- Spark's)
  if (DQ_TYPE_ID(f->logical[0]) == DQ_DECIMAL128 && f->types[0] == DQ_UTF8) return DQ_OK;
  HIP_TRY(hipSetDevice(f->device));
  if (hip_stream) f->stream = reinterpret_cast<hipStream_t>(hip_stream);
  dq_status st = finalize_b(f);
  if (st != DQ_OK) return st;
  if ((int64_t)f->R > max_records) return DQ_OK;  // (the caller scans the rows instead)
  DevBuf<uint32_t> regs;
  HIP_TRY(regs.ensure(kHllM));
  HIP_TRY(hipMemsetAsync(regs.p, 0, kHllM * 4, f->stream));
  if (f->R > 0) {
    const int64_t P = (int64_t)kBuckets << f->s_bits;
    const unsigned grid = (unsigned)std::min<int64_t>((P + 3) / 4, 2048);
    hipLaunchKernelGGL(freq_hll_records, dim3(grid), dim3(256), 0, f->stream,
                       reinterpret_cast<const uint64_t*>(f->recsB.p), f->part_base.p, f->part_end_ptr, P, f->s_bits,
                       f->exact ? 1 : 0, f->types[0], arena_of(f), regs.p);
    HIP_TRY(hipGetLastError());
  }
  uint32_t r[kHllM];
  HIP_TRY(d2h(r, regs.p, sizeof(r), f->stream));  // (regs dies here)
  for (int w = 0; w < kHllWords; ++w) {  // StatefulHyperloglogPlus's 52-word layout
    uint64_t v = 0;
    for (int i = 0; i < kHllRegsPerWord; ++i) {
      const int idx = w * kHllRegsPerWord + i;
      if (idx >= kHllM) break;
      v |= (uint64_t)(r[idx] & 0x3f) << (kHllRegBits * i);
    }
    words[w] = v;
  }
  *done = 1;
  return DQ_OK;
}

extern "C" dq_status dq_freq_folded_nan_rows(dq_freq* f, int64_t* n) {
  if (!f || !n) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = sync_counters(f);
  if (st != DQ_OK) return st;
  *n = f->nan_counted ? (int64_t)f->h_counters[C_NAN_FOLDED] : -1;
  return DQ_OK;
}

extern "C" dq_status dq_freq_num_groups(dq_freq* f, int64_t* n) {
  if (!f || !n) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = finalize_c(f, false, false);
  if (st != DQ_OK) return st;
  *n = (int64_t)(f->st_groups + (f->h_counters[C_NULL_GROUP] ? 1 : 0));
  return DQ_OK;
}

extern "C" dq_status dq_freq_null_literal(dq_freq* f, int64_t* null_group_rows,
                                          int64_t* literal_count) {
  if (!f || !null_group_rows || !literal_count) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = finalize_c(f, false, false);
  if (st != DQ_OK) return st;
  *null_group_rows = (int64_t)f->h_counters[C_NULL_GROUP];
  *literal_count = has_null_literal(f) ? (int64_t)f->st_literal : 0;
  return DQ_OK;
}

extern "C" int64_t dq_freq_num_rows(const dq_freq* f) { return f ? f->num_rows : -1; }

static dq_status copy_out(const std::vector<int64_t>& counts, const std::vector<int64_t>& offs,
                          const std::vector<uint8_t>& bytes, int64_t* counts_out,
                          int64_t* key_offsets_out, uint8_t* key_bytes_out, int64_t capacity,
                          int64_t key_bytes_capacity, int64_t* key_bytes_needed) {
  if (key_bytes_needed) *key_bytes_needed = (int64_t)bytes.size();
  if (!key_bytes_out) return DQ_OK;
  if (capacity < (int64_t)counts.size() || key_bytes_capacity < (int64_t)bytes.size())
    return fail(DQ_ERR_INVALID_ARGUMENT, "export buffers too small");
  if (counts_out && !counts.empty()) memcpy(counts_out, counts.data(), counts.size() * 8);
  if (key_offsets_out) memcpy(key_offsets_out, offs.data(), offs.size() * 8);
  if (!bytes.empty()) memcpy(key_bytes_out, bytes.data(), bytes.size());
  return DQ_OK;
}

extern "C" dq_status dq_freq_export(dq_freq* f, int64_t* counts_out, int64_t* key_offsets_out,
                                    uint8_t* key_bytes_out, int64_t capacity,
                                    int64_t key_bytes_capacity, int64_t* key_bytes_needed) {
  if (!f) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = compact_groups(f);
  if (st != DQ_OK) return st;
  std::vector<int64_t> counts, offs;
  std::vector<uint8_t> bytes;
  st = encode_groups(f, f->compact.p, f->n_compact, counts, offs, bytes);
  if (st != DQ_OK) return st;
  if (f->h_counters[C_NULL_GROUP]) put_null_group(f, counts, offs, bytes);
  offs.push_back((int64_t)bytes.size());
  return copy_out(counts, offs, bytes, counts_out, key_offsets_out, key_bytes_out, capacity,
                  key_bytes_capacity, key_bytes_needed);
}

// The inverse of dq_freq_export (a persisted frequency state loaded back, StateProvider.scala:
// 231-237, 270-278): each group becomes one record -- exact mode: the widened value; hashed mode:
// the encoded key's row hash (enc_hash, the value the row path computes) with the key in the
// var bytes -- and goes through the records path of the repartition.  A one-key group with tag
// 0 is the NULL group of a Histogram table.
extern "C" dq_status dq_freq_import(dq_freq* f, const int64_t* counts, const int64_t* key_offsets,
                                    const uint8_t* key_bytes, int64_t n_groups, int64_t num_rows,
                                    int64_t null_key_rows, int null_as_group, void* hip_stream) {
  if (!f || n_groups < 0 || num_rows < 0 || null_key_rows < 0)
    return fail(DQ_ERR_INVALID_ARGUMENT, "bad arguments");
  if (n_groups && (!counts || !key_offsets || !key_bytes))
    return fail(DQ_ERR_INVALID_ARGUMENT, "null group buffers");
  std::vector<RecIn> rec;
  std::vector<uint8_t> var;
  rec.reserve((size_t)n_groups);
  int64_t special[3] = {0, 0, null_key_rows};
  const int64_t total = n_groups ? key_offsets[n_groups] : 0;
  for (int64_t g = 0; g < n_groups; ++g) {
    const int64_t o0 = key_offsets[g], o1 = key_offsets[g + 1];
    if (o0 < 0 || o1 < o0 || o1 > total || (o0 & 3) || (o1 - o0) < 4)
      return fail(DQ_ERR_INVALID_ARGUMENT, "bad key offsets at group %lld", (long long)g);
    if (counts[g] <= 0) return fail(DQ_ERR_INVALID_ARGUMENT, "group %lld has count <= 0", (long long)g);
    const uint32_t* enc = reinterpret_cast<const uint32_t*>(key_bytes + o0);
    const int64_t sz = (int64_t)enc_size(enc, f->types.data(), f->n_keys);
    if (sz != o1 - o0) return fail(DQ_ERR_INVALID_ARGUMENT, "group %lld: malformed key", (long long)g);
    if (f->n_keys == 1 && enc[0] == 0) {  // the NULL group (Histogram tables only)
      if (!null_as_group) return fail(DQ_ERR_INVALID_ARGUMENT, "NULL key outside a Histogram table");
      special[1] += counts[g];
      continue;
    }
    RecIn r;
    r.count = (uint64_t)counts[g];
    if (f->exact) {
      r.key = (uint64_t)enc[1] | ((uint64_t)enc[2] << 32);
      r.enc_off = 0;
    } else {
      r.key = enc_hash(enc, f->types.data(), f->n_keys);
      r.enc_off = var.size();
      var.insert(var.end(), key_bytes + o0, key_bytes + o1);
      var.resize((var.size() + 7) & ~(size_t)7, 0);
    }
    rec.push_back(r);
  }
  HIP_TRY(hipSetDevice(f->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
  DevBuf<RecIn> drec;
  DevBuf<uint8_t> dvar;
  HIP_TRY(drec.ensure(std::max<size_t>(rec.size(), 1)));
  HIP_TRY(dvar.ensure(std::max<size_t>(var.size(), 8)));
  if (!rec.empty())
    HIP_TRY(hipMemcpyAsync(drec.p, rec.data(), rec.size() * sizeof(RecIn), hipMemcpyHostToDevice, st));
  if (!var.empty()) HIP_TRY(hipMemcpyAsync(dvar.p, var.data(), var.size(), hipMemcpyHostToDevice, st));
  const int64_t rc[1] = {(int64_t)rec.size()};
  const int64_t vb[1] = {(int64_t)var.size()};
  dq_status s = dq_freq_add_records_device(f, reinterpret_cast<const dq_freq_record*>(drec.p),
                                           dvar.p, 1, rc, vb, num_rows, special, null_as_group,
                                           hip_stream);
  if (s != DQ_OK) return s;
  HIP_TRY(hipStreamSynchronize(st));  // the staging buffers die here
  return DQ_OK;
}

// Histogram's details: rdd.top(maxDetailBins)(OrderByAbsoluteCount) (Histogram.scala:78).
// dq_freq_topk when a few partitions may hold unlisted groups that outrank the selection: those
// partitions are counted again with every group materialised (work items of a phase-C launch,
// group_stride slots each), and the top k are selected over the other partitions' candidates
// plus those groups.  done = false: a partition overflowed the first-pass table, so the caller
// takes the exact path over every group.
static dq_status topk_recount(dq_freq* f, int k, FEntry* list, int64_t nb, std::vector<Group>& top,
                              bool& done) {
  done = false;
  const int64_t P = (int64_t)kBuckets << f->s_bits;
  const uint32_t stride = (uint32_t)(f->exact ? FM<false>::kTableC : kCHT) + 1;  // (+ the special group)
  DevBuf<Group> all;  // [the candidates of every partition | the recounted partitions' groups]
  const int64_t nc = P * kCand;
  HIP_TRY(all.ensure((size_t)(nc + nb * (int64_t)stride)));
  HIP_TRY(hipMemsetAsync(all.p + nc, 0, (size_t)nb * stride * sizeof(Group), f->stream));
  HIP_TRY(hipMemcpyAsync(all.p, f->cand.p, (size_t)nc * sizeof(Group), hipMemcpyDeviceToDevice, f->stream));
  hipLaunchKernelGGL(freq_cand_clear, dim3((unsigned)((nb * kCand + 255) / 256)), dim3(256), 0, f->stream,
                     all.p, list, nb);
  HIP_TRY(hipGetLastError());
  CArgs a;
  memset(&a, 0, sizeof(a));
  a.recsB = f->recsB.p;
  a.part_base = f->part_base.p;
  a.part_end = f->part_end_ptr;
  a.s = f->s_bits;
  a.arena = arena_of(f);
  for (int q = 0; q < f->n_keys; ++q) a.types[q] = f->types[q];
  a.n_keys = f->n_keys;
  a.want_cand = 0;
  a.num_rows = (double)f->num_rows;
  a.entries = list;
  a.n_work = (int32_t)nb;
  // the statistics of these partitions are stored again with the same values; the rest of
  // the table's state stays as the full pass left it
  a.part_groups = f->part_groups.p;
  a.part_unique = f->part_unique.p;
  a.part_entropy = f->part_entropy.p;
  a.part_off = f->part_off.p;
  DevBuf<FEntry> ovf;
  DevBuf<unsigned int> novf;
  HIP_TRY(ovf.ensure(2 * (size_t)nb));
  HIP_TRY(novf.ensure(1));
  HIP_TRY(hipMemsetAsync(novf.p, 0, 4, f->stream));
  a.ovf_out = ovf.p;
  a.ovf_n = novf.p;
  a.groups = all.p + nc;
  a.group_stride = stride;
  DevBuf<unsigned long long> scratch_counters;  // (collision counts of a recount: not the table's)
  HIP_TRY(scratch_counters.ensure(C_N));
  HIP_TRY(hipMemsetAsync(scratch_counters.p, 0, C_N * 8, f->stream));
  a.counters = scratch_counters.p;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, f->device);
  const unsigned grid = (unsigned)std::min<int64_t>(nb, 2 * cus);
  if (f->exact)
    hipLaunchKernelGGL((freq_phaseC_x<false, false>), dim3(grid), dim3(kCThreads), 0, f->stream, a);
  else
    hipLaunchKernelGGL(freq_phaseC_h<false>, dim3(grid), dim3(kCThreads), 0, f->stream, a);
  HIP_TRY(hipGetLastError());
  unsigned int m = 0;
  HIP_TRY(d2h(&m, novf.p, 4, f->stream));
  if (m) return DQ_OK;  // (not done)
  dq_status st = select_top(f, all.p, nc + nb * (int64_t)stride, k, top);
  if (st != DQ_OK) return st;
  done = true;
  return DQ_OK;
}

extern "C" dq_status dq_freq_topk(dq_freq* f, int k, int64_t* counts_out, int64_t* key_offsets_out,
                                  uint8_t* key_bytes_out, int64_t key_bytes_capacity, int64_t* n_out,
                                  int64_t* key_bytes_needed) {
  if (!f || !n_out || k < 0) return fail(DQ_ERR_INVALID_ARGUMENT, "bad arguments");
  HIP_TRY(hipSetDevice(f->device));
  if (f->topk_k != k || !f->c_valid) {
    dq_status st = finalize_c(f, false, true);
    if (st != DQ_OK) return st;
    const int64_t P = (int64_t)kBuckets << f->s_bits;
    std::vector<Group> top;
    bool exact_path = f->recounted;
    if (!exact_path) {
      st = select_top(f, f->cand.p, P * kCand, k, top);
      if (st != DQ_OK) return st;
      const uint64_t tau = top.size() == (size_t)k && k > 0 ? top.back().count : 0;
      DevBuf<unsigned long long> bad;
      DevBuf<FEntry> bad_list;
      const int64_t cap = kTopkRecountMax;
      HIP_TRY(bad.ensure(1));
      HIP_TRY(bad_list.ensure(cap));
      HIP_TRY(hipMemsetAsync(bad.p, 0, 8, f->stream));
      hipLaunchKernelGGL(freq_cand_check, dim3(grid_for(P)), dim3(256), 0, f->stream, f->cand.p,
                         f->part_groups.p, P, tau, bad.p, bad_list.p, cap);
      HIP_TRY(hipGetLastError());
      unsigned long long nb = 0;
      HIP_TRY(d2h(&nb, bad.p, 8, f->stream));
      exact_path = nb != 0;
      const char* fe = getenv("DQ_FREQ_TOPK_EXACT");  // =1: every group (A/B, tests)
      if (nb && (int64_t)nb <= cap && !(fe && atoi(fe))) {  // a few partitions: recount just those
        bool done = false;
        st = topk_recount(f, k, bad_list.p, (int64_t)nb, top, done);
        if (st != DQ_OK) return st;
        exact_path = !done;
      }
    }
    if (exact_path) {  // select over every group
      st = compact_groups(f);
      if (st != DQ_OK) return st;
      st = select_top(f, f->compact.p, f->n_compact, k, top);
      if (st != DQ_OK) return st;
    }
    // the exact-mode NULL group competes like any other
    const uint64_t nullg = f->h_counters[C_NULL_GROUP];
    f->topk_counts.clear();
    f->topk_offs.clear();
    f->topk_bytes.clear();
    DevBuf<Group> dg;
    HIP_TRY(dg.ensure(std::max<size_t>(top.size(), 1)));
    if (!top.empty())
      HIP_TRY(hipMemcpyAsync(dg.p, top.data(), top.size() * sizeof(Group), hipMemcpyHostToDevice,
                             f->stream));  // (encode_groups waits for the stream)
    std::vector<int64_t> c1, o1;
    std::vector<uint8_t> b1;
    st = encode_groups(f, dg.p, (int64_t)top.size(), c1, o1, b1);
    if (st != DQ_OK) return st;
    // owner_scatter keeps no order: restore count order, placing the NULL group
    std::vector<size_t> idx(c1.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return c1[x] > c1[y]; });
    o1.push_back((int64_t)b1.size());
    bool null_done = nullg == 0;
    auto emit_null = [&]() {
      put_null_group(f, f->topk_counts, f->topk_offs, f->topk_bytes);
      null_done = true;
    };
    for (size_t i : idx) {
      if ((int)f->topk_counts.size() >= k) break;
      if (!null_done && (int64_t)nullg > c1[i]) emit_null();
      if ((int)f->topk_counts.size() >= k) break;
      f->topk_offs.push_back((int64_t)f->topk_bytes.size());
      f->topk_counts.push_back(c1[i]);
      f->topk_bytes.insert(f->topk_bytes.end(), b1.begin() + o1[i], b1.begin() + o1[i + 1]);
    }
    if (!null_done && (int)f->topk_counts.size() < k) emit_null();
    f->topk_offs.push_back((int64_t)f->topk_bytes.size());
    f->topk_k = k;
  }
  *n_out = (int64_t)f->topk_counts.size();
  return copy_out(f->topk_counts, f->topk_offs, f->topk_bytes, counts_out, key_offsets_out,
                  key_bytes_out, *n_out, key_bytes_capacity, key_bytes_needed);
}

// dst += src (FrequenciesAndNumRows.sum, GroupingAnalyzers.scala:128-148): the source's chunks
// are appended, so equal keys meet in the next finalize and their counts add; numRows add.
extern "C" dq_status dq_freq_merge(dq_freq* dst, const dq_freq* src_c) {
  if (!dst || !src_c) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  dq_freq* src = const_cast<dq_freq*>(src_c);
  if (dst == src) return fail(DQ_ERR_INVALID_ARGUMENT, "cannot merge a table into itself");
  if (dst->arena_view) return fail(DQ_ERR_STATE, "a table reading another table's keys takes no adds");
  if (dst->n_keys != src->n_keys || dst->logical != src->logical)
    return fail(DQ_ERR_STATE, "frequency tables group on different key types");
  if (dst->device != src->device) return fail(DQ_ERR_UNSUPPORTED, "tables on different devices");
  dst->nan_counted = dst->nan_counted && src->nan_counted;
  if (dst->mode_null_as_group >= 0 && src->mode_null_as_group >= 0 &&
      dst->mode_null_as_group != src->mode_null_as_group)
    return fail(DQ_ERR_STATE, "frequency tables differ in NULL handling");
  HIP_TRY(hipSetDevice(dst->device));
  HIP_TRY(hipStreamSynchronize(src->stream));
  dq_status st = pull_counters(src);
  if (st != DQ_OK) return st;
  st = pull_counters(dst);
  if (st != DQ_OK) return st;
  if (dst->mode_null_as_group < 0) dst->mode_null_as_group = src->mode_null_as_group;
  const int64_t nc = src->n_chunks;
  if (nc) {
    st = ensure_chunks(dst, nc);
    if (st != DQ_OK) return st;
    const size_t region = (size_t)dst->tile * dst->rb;
    HIP_TRY(hipMemcpyAsync(dst->recs.p + (size_t)dst->n_chunks * region, src->recs.p, nc * region,
                           hipMemcpyDeviceToDevice, dst->stream));
    HIP_TRY(hipMemcpyAsync(dst->hist.p + (size_t)dst->n_chunks * kHistRow, src->hist.p,
                           (size_t)nc * kHistRow * 2, hipMemcpyDeviceToDevice, dst->stream));
    if (!dst->exact) {
      HIP_TRY(grow_keep(dst->arena, dst->arena_used, dst->arena_used + src->arena_used + 64,
                        dst->stream));
      if (src->arena_used)
        HIP_TRY(hipMemcpyAsync(dst->arena.p + dst->arena_used, arena_of(src), src->arena_used,
                               hipMemcpyDeviceToDevice, dst->stream));
      hipLaunchKernelGGL(freq_rebase, dim3((unsigned)nc), dim3(256), 0, dst->stream,
                         reinterpret_cast<uint64_t*>(dst->recs.p), dst->hist.p, dst->n_chunks,
                         dst->tile, (uint64_t)dst->arena_used);
      HIP_TRY(hipGetLastError());
      if (src->n_prow) {  // (the pieces' records are outside the chunk rows' counts)
        DevBuf<unsigned long long> pb;
        std::vector<unsigned long long> hb(src->h_pbase);
        for (auto& b : hb) b += (unsigned long long)dst->n_chunks * dst->tile;
        HIP_TRY(pb.ensure(hb.size()));
        HIP_TRY(hipMemcpyAsync(pb.p, hb.data(), hb.size() * 8, hipMemcpyHostToDevice, dst->stream));
        hipLaunchKernelGGL(freq_rebase_pieces, dim3((unsigned)src->n_prow), dim3(256), 0, dst->stream,
                           reinterpret_cast<uint64_t*>(dst->recs.p), src->pstart.p, src->plen.p, pb.p,
                           (uint64_t)dst->arena_used);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(dst->stream));  // (hb and pb die here)
      }
      dst->arena_used += src->arena_used;
    }
    if (src->n_prow) {  // the source's bucket pieces, their regions moved with its chunks
      const size_t need = (size_t)(dst->n_prow + src->n_prow) * kBuckets;
      HIP_TRY(grow_keep(dst->pstart, (size_t)dst->n_prow * kBuckets, need, dst->stream));
      HIP_TRY(grow_keep(dst->plen, (size_t)dst->n_prow * kBuckets, need, dst->stream));
      HIP_TRY(hipMemcpyAsync(dst->pstart.p + (size_t)dst->n_prow * kBuckets, src->pstart.p,
                             (size_t)src->n_prow * kBuckets * 4, hipMemcpyDeviceToDevice, dst->stream));
      HIP_TRY(hipMemcpyAsync(dst->plen.p + (size_t)dst->n_prow * kBuckets, src->plen.p,
                             (size_t)src->n_prow * kBuckets * 4, hipMemcpyDeviceToDevice, dst->stream));
      const unsigned long long shift = (unsigned long long)dst->n_chunks * dst->tile;
      for (unsigned long long b : src->h_pbase) dst->h_pbase.push_back(b + shift);
      dst->n_prow += src->n_prow;
      dst->n_empty_chunks += src->n_empty_chunks;
    }
    dst->n_chunks += nc;
  }
  for (int k = 0; k < C_N; ++k) dst->h_counters[k] += src->h_counters[k];
  dst->num_rows += src->num_rows;
  invalidate(dst);
  return push_counters(dst);
}

// ------------------------------------------------------------------------------------------------
// Multi-GPU repartition (records of materialised groups; see the header)
// ------------------------------------------------------------------------------------------------
extern "C" dq_status dq_freq_partition_sizes(dq_freq* f, int n_parts, int64_t* rec_counts,
                                             int64_t* var_bytes, int64_t* special) {
  if (!f || !rec_counts || !var_bytes || !special)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (n_parts < 1 || n_parts > kMaxParts)
    return fail(DQ_ERR_UNSUPPORTED, "n_parts must be in [1, %d]", kMaxParts);
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = compact_groups(f);
  if (st != DQ_OK) return st;
  std::vector<unsigned long long> rec, var;
  st = owner_sizes(f, f->compact.p, f->n_compact, n_parts, rec, var);
  if (st != DQ_OK) return st;
  for (int i = 0; i < n_parts; ++i) {
    rec_counts[i] = (int64_t)rec[i];
    var_bytes[i] = (int64_t)var[i];
  }
  special[0] = 0;
  special[1] = (int64_t)f->h_counters[C_NULL_GROUP];
  special[2] = (int64_t)f->h_counters[C_NULL_ROWS];
  return DQ_OK;
}

extern "C" dq_status dq_freq_partition(dq_freq* f, int n_parts, dq_freq_record* records,
                                       uint8_t* var, void* hip_stream) {
  if (!f) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (n_parts < 1 || n_parts > kMaxParts)
    return fail(DQ_ERR_UNSUPPORTED, "n_parts must be in [1, %d]", kMaxParts);
  HIP_TRY(hipSetDevice(f->device));
  HIP_TRY(hipStreamSynchronize(f->stream));
  f->stream = reinterpret_cast<hipStream_t>(hip_stream);
  dq_status st = compact_groups(f);
  if (st != DQ_OK) return st;
  std::vector<unsigned long long> rec, var_n;
  st = owner_sizes(f, f->compact.p, f->n_compact, n_parts, rec, var_n);
  if (st != DQ_OK) return st;
  unsigned long long tr = 0, tv = 0;
  for (int i = 0; i < n_parts; ++i) {
    tr += rec[i];
    tv += var_n[i];
  }
  if (tr && (!records || (tv && !var))) return fail(DQ_ERR_INVALID_ARGUMENT, "null output buffer");
  return owner_scatter(f, f->compact.p, f->n_compact, n_parts, reinterpret_cast<RecIn*>(records),
                       var, rec, var_n);
}

static dq_status add_records(dq_freq* f, const dq_freq_record* records, const uint8_t* var,
                             int n_src, const int64_t* src_records, const int64_t* src_var_bytes,
                             int64_t num_rows, const int64_t* special, int null_as_group,
                             void* hip_stream, bool borrow);

extern "C" dq_status dq_freq_add_records_device(dq_freq* f, const dq_freq_record* records,
                                                const uint8_t* var, int n_src,
                                                const int64_t* src_records,
                                                const int64_t* src_var_bytes, int64_t num_rows,
                                                const int64_t* special, int null_as_group,
                                                void* hip_stream) {
  return add_records(f, records, var, n_src, src_records, src_var_bytes, num_rows, special,
                     null_as_group, hip_stream, false);
}

// borrow: read the var bytes in place (arena_view) instead of copying them into the table's
// arena -- only for a fresh hashed table that dies before the var bytes do
static dq_status add_records(dq_freq* f, const dq_freq_record* records, const uint8_t* var,
                             int n_src, const int64_t* src_records, const int64_t* src_var_bytes,
                             int64_t num_rows, const int64_t* special, int null_as_group,
                             void* hip_stream, bool borrow) {
  if (!f || !src_records || !src_var_bytes || !special)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (f->arena_view) return fail(DQ_ERR_STATE, "a table reading another table's keys takes no adds");
  f->nan_counted = false;
  if (borrow && (f->exact || f->arena_used || f->n_chunks))
    return fail(DQ_ERR_STATE, "only a fresh hashed table can borrow var bytes");
  if (n_src < 1 || n_src > kMaxParts)
    return fail(DQ_ERR_UNSUPPORTED, "n_src must be in [1, %d]", kMaxParts);
  const int mode = null_as_group ? 1 : 0;
  if (f->mode_null_as_group >= 0 && f->mode_null_as_group != mode)
    return fail(DQ_ERR_STATE, "null_as_group must be the same for every batch");
  f->mode_null_as_group = mode;
  HIP_TRY(hipSetDevice(f->device));
  HIP_TRY(hipStreamSynchronize(f->stream));
  f->stream = reinterpret_cast<hipStream_t>(hip_stream);
  AArgs a = base_args(f);
  int64_t total_rec = 0, total_var = 0;
  a.segs.n_src = n_src;
  for (int j = 0; j < n_src; ++j) {
    if (src_records[j] < 0 || src_var_bytes[j] < 0 || (src_var_bytes[j] & 7))
      return fail(DQ_ERR_INVALID_ARGUMENT, "bad segment sizes for source %d", j);
    a.segs.rec_start[j] = total_rec;
    a.segs.var_base[j] = total_var;
    total_rec += src_records[j];
    total_var += src_var_bytes[j];
  }
  a.segs.rec_start[n_src] = total_rec;
  if (total_rec && !records) return fail(DQ_ERR_INVALID_ARGUMENT, "null records");
  if (!f->exact && total_var && !var) return fail(DQ_ERR_INVALID_ARGUMENT, "null var bytes");
  static const int dbg = [] {  // DQ_FREQ_DEBUG: the steps below, timed (synchronising)
    const char* e = getenv("DQ_FREQ_DEBUG");
    return e ? atoi(e) : 0;
  }();
  auto t_last = std::chrono::steady_clock::now();
  auto stamp = [&](const char* what) {
    if (!dbg) return;
    (void)hipStreamSynchronize(f->stream);
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "dq_freq add_records %s: %.2f ms\n", what,
            std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  dq_status st = pull_counters(f);
  if (st != DQ_OK) return st;
  invalidate(f);
  stamp("counters");
  if (total_rec) {
    // a record's count becomes count_digits(count) <= 32 records: tiles of tile / max digits
    // records never overflow a chunk (a 32x bound sized a marginal of 1e8 groups at 60+ GB)
    int maxd = 32;
    {
      DevBuf<unsigned int> md;
      HIP_TRY(md.ensure(1));
      HIP_TRY(hipMemsetAsync(md.p, 0, 4, f->stream));
      hipLaunchKernelGGL(freq_max_digits, dim3(grid_for(total_rec)), dim3(256), 0, f->stream,
                         reinterpret_cast<const RecIn*>(records), total_rec, md.p);
      HIP_TRY(hipGetLastError());
      unsigned int h = 32;
      HIP_TRY(d2h(&h, md.p, 4, f->stream));
      maxd = std::max(1, (int)std::min(h, 32u));
    }
    // (and at most one record per thread: the records path runs one round per tile)
    const int64_t per = std::min<int64_t>(f->tile / maxd, AKeys<false, true>::kThreads);
    static_assert(AKeys<false, true>::kThreads == AKeys<true, true>::kThreads, "one round");
    const int64_t chunks = phaseA_chunks(!f->exact, true, total_rec, per, nullptr);
    stamp("max digits");
    st = ensure_chunks(f, chunks);
    if (st != DQ_OK) return st;
    stamp("chunks");
    a = [&] {
      AArgs b = base_args(f);
      b.segs = a.segs;
      return b;
    }();
    if (!f->exact && borrow) {  // (the var bytes' owner keeps >= 64 bytes past its last key)
      f->arena_view = var;
      a.arena = const_cast<uint8_t*>(var);
      a.var_arena_base = 0;
      f->rec_var_base = 0;
      f->arena_used = total_var;
    } else if (!f->exact) {
      const uint64_t base = (f->arena_used + 7) & ~7ULL;
      HIP_TRY(grow_keep(f->arena, f->arena_used, base + total_var + 64, f->stream));
      if (total_var)
        HIP_TRY(hipMemcpyAsync(f->arena.p + base, var, total_var, hipMemcpyDeviceToDevice, f->stream));
      a.arena = f->arena.p;
      a.var_arena_base = base;
      f->rec_var_base = base;
      f->arena_used = base + total_var;
    }
    stamp("arena");
    a.rin = reinterpret_cast<const RecIn*>(records);
    a.n_items = total_rec;
    a.tile_items = per;
    if (f->exact) launch_phaseA<false>(f, a, true);
    else launch_phaseA<true>(f, a, true);
    HIP_TRY(hipGetLastError());
    stamp("phase A");
    f->n_chunks += chunks;
  }
  f->h_counters[C_NULL_GROUP] += (uint64_t)special[1];
  f->h_counters[C_NULL_ROWS] += (uint64_t)special[2];
  if (special[0]) return fail(DQ_ERR_INVALID_ARGUMENT, "special[0] is no longer used (must be 0)");
  f->num_rows += num_rows;
  return push_counters(f);
}

// ------------------------------------------------------------------------------------------------
// Multi-GPU raw-key repartition: a one-column fixed-width key of high
// cardinality (a unique id) is exchanged as its raw values, before any local count -- one
// group-by per row on its owner rank and 1-8 bytes per row over xGMI, instead of a local group-by,
// 24-byte records and a second group-by.  The owner is a function of the key the table counts
// (fmix of the canonical widened value, freq_codec.h), so every rank sends equal keys to one owner;
// NULL rows stay home as a count.
// ------------------------------------------------------------------------------------------------
namespace dq {

constexpr int kKeyPartThreads = 256;
constexpr int kKeyPartRows = 16 * kKeyPartThreads;  // rows per block step

DQ_DEV uint32_t raw_owner(int type, const void* values, int64_t r, int null_as_group, int parts) {
  KeySet ks;
  ks.n_keys = 1;
  ks.null_as_group = null_as_group;
  ks.cols[0].type = type;
  const uint64_t h = fmix_bij(exact_canon(ks, kwiden(type, values, r)));
  return (uint32_t)(((h & 0xFFFFFFULL) * (uint64_t)parts) >> 24);  // low bits: the owner's keys
                                                                   // still fill every bucket
}

__global__ void __launch_bounds__(kKeyPartThreads)
key_owner_count(int type, const uint8_t* __restrict__ valid, const void* __restrict__ values,
                int64_t rows, int null_as_group, int parts, unsigned long long* __restrict__ counts,
                unsigned long long* __restrict__ nulls) {
  __shared__ uint32_t s_cnt[kMaxParts];
  for (int i = threadIdx.x; i < parts; i += kKeyPartThreads) s_cnt[i] = 0;
  __syncthreads();
  unsigned long long nn = 0;
  for (int64_t r = (int64_t)blockIdx.x * kKeyPartThreads + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * kKeyPartThreads) {
    if (!kbit(valid, r)) {
      ++nn;
      continue;
    }
    atomicAdd(&s_cnt[raw_owner(type, values, r, null_as_group, parts)], 1u);
  }
  nn = wave_sum(nn);
  if (__lane_id() == 0 && nn) atomicAdd(nulls, nn);
  __syncthreads();
  for (int i = threadIdx.x; i < parts; i += kKeyPartThreads)
    if (s_cnt[i]) atomicAdd(&counts[i], (unsigned long long)s_cnt[i]);
}

// Each block step of kKeyPartRows rows counts its rows per owner in LDS, reserves its run in every
// owner segment with one atomic per owner, then writes every row's value into its run (the runs of
// a step are contiguous per owner, so the stores of a wave land in a few neighbouring lines).
__global__ void __launch_bounds__(kKeyPartThreads)
key_owner_scatter(int type, int elem, const uint8_t* __restrict__ valid,
                  const void* __restrict__ values, int64_t rows, int null_as_group, int parts,
                  unsigned long long* __restrict__ cursor, uint8_t* __restrict__ out) {
  __shared__ uint32_t s_cnt[kMaxParts], s_pos[kMaxParts];
  __shared__ unsigned long long s_base[kMaxParts];
  for (int64_t r0 = (int64_t)blockIdx.x * kKeyPartRows; r0 < rows;
       r0 += (int64_t)gridDim.x * kKeyPartRows) {
    for (int i = threadIdx.x; i < parts; i += kKeyPartThreads) s_cnt[i] = s_pos[i] = 0;
    __syncthreads();
    uint32_t own[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int64_t r = r0 + (int64_t)k * kKeyPartThreads + threadIdx.x;
      own[k] = ~0u;
      if (r < rows && kbit(valid, r)) {
        own[k] = raw_owner(type, values, r, null_as_group, parts);
        atomicAdd(&s_cnt[own[k]], 1u);
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < parts; i += kKeyPartThreads)
      s_base[i] = s_cnt[i] ? atomicAdd(&cursor[i], (unsigned long long)s_cnt[i]) : 0ULL;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (own[k] == ~0u) continue;
      const int64_t r = r0 + (int64_t)k * kKeyPartThreads + threadIdx.x;
      const uint64_t at = s_base[own[k]] + atomicAdd(&s_pos[own[k]], 1u);
      const uint8_t* src = reinterpret_cast<const uint8_t*>(values) + r * elem;
      uint8_t* dst = out + at * elem;
      switch (elem) {
        case 1: *dst = *src; break;
        case 2: *reinterpret_cast<uint16_t*>(dst) = *reinterpret_cast<const uint16_t*>(src); break;
        case 4: *reinterpret_cast<uint32_t*>(dst) = *reinterpret_cast<const uint32_t*>(src); break;
        default: *reinterpret_cast<uint64_t*>(dst) = *reinterpret_cast<const uint64_t*>(src); break;
      }
    }
    __syncthreads();  // s_cnt / s_pos / s_base are reset by the next step
  }
}

}  // namespace dq

static int raw_key_elem(int type) {
  switch (type) {
    case DQ_INT8: return 1;
    case DQ_INT16: return 2;
    case DQ_INT32: case DQ_FLOAT32: return 4;
    case DQ_INT64: case DQ_FLOAT64: return 8;
    default: return 0;  // bool (bit-packed) and strings: the records path
  }
}

extern "C" dq_status dq_key_partition(const dq_column* batches, int n_batches, int n_parts,
                                      int null_as_group, uint8_t* out, int64_t* counts_out,
                                      int64_t* null_rows_out, void* hip_stream) {
  using namespace dq;
  if ((n_batches > 0 && !batches) || n_batches < 0 || !counts_out || !null_rows_out)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (n_parts < 1 || n_parts > kMaxParts)
    return fail(DQ_ERR_UNSUPPORTED, "n_parts must be in [1, %d]", kMaxParts);
  int64_t rows = 0;
  const int ltype = n_batches ? batches[0].type : DQ_INT64;
  // a date / timestamp key is its int32 / int64 (equal keys, equal owner, as a table counts them)
  const int type = ltype == DQ_DATE32 ? DQ_INT32 : ltype == DQ_TIMESTAMP_US ? DQ_INT64 : ltype;
  const int elem = raw_key_elem(type);
  if (!elem) return fail(DQ_ERR_WRONG_TYPE, "raw-key repartition needs a fixed-width key");
  for (int b = 0; b < n_batches; ++b) {
    if (batches[b].type != ltype) return fail(DQ_ERR_WRONG_TYPE, "batches differ in type");
    if (batches[b].length < 0 || (batches[b].length && !batches[b].values))
      return fail(DQ_ERR_INVALID_ARGUMENT, "batch %d has no values", b);
    rows += batches[b].length;
  }
  if (rows && !out) return fail(DQ_ERR_INVALID_ARGUMENT, "null output buffer");
  hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
  DevBuf<unsigned long long> cnt;
  HIP_TRY(cnt.ensure(2 * kMaxParts + 1));
  HIP_TRY(hipMemsetAsync(cnt.p, 0, (2 * kMaxParts + 1) * 8, stream));
  for (int b = 0; b < n_batches; ++b) {
    const dq_column& c = batches[b];
    if (!c.length) continue;
    const unsigned grid = (unsigned)std::min<int64_t>((c.length + kKeyPartRows - 1) / kKeyPartRows * 4, 4096);
    hipLaunchKernelGGL(key_owner_count, dim3(grid), dim3(kKeyPartThreads), 0, stream, type,
                       c.validity, c.values, c.length, null_as_group, n_parts, cnt.p,
                       cnt.p + 2 * kMaxParts);
    HIP_TRY(hipGetLastError());
  }
  unsigned long long h[2 * kMaxParts + 1];
  HIP_TRY(d2h(h, cnt.p, sizeof(h), stream));
  unsigned long long base = 0;
  for (int j = 0; j < n_parts; ++j) {  // segment cursors: the exclusive prefix of the counts
    counts_out[j] = (int64_t)h[j];
    h[kMaxParts + j] = base;
    base += h[j];
  }
  *null_rows_out = (int64_t)h[2 * kMaxParts];
  HIP_TRY(hipMemcpyAsync(cnt.p + kMaxParts, h + kMaxParts, kMaxParts * 8, hipMemcpyHostToDevice, stream));
  for (int b = 0; b < n_batches; ++b) {
    const dq_column& c = batches[b];
    if (!c.length) continue;
    const unsigned grid = (unsigned)std::min<int64_t>((c.length + kKeyPartRows - 1) / kKeyPartRows, 4096);
    hipLaunchKernelGGL(key_owner_scatter, dim3(grid), dim3(kKeyPartThreads), 0, stream, type, elem,
                       c.validity, c.values, c.length, null_as_group, n_parts, cnt.p + kMaxParts, out);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(stream));  // the cursors' buffer dies here
  return DQ_OK;
}
