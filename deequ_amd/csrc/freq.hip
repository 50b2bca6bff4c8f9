// freq.hip -- hash group-by for the frequency analyzers (FrequencyBasedAnalyzer.computeFrequencies,
// GroupingAnalyzers.scala:53-80, and Histogram.scala:54-69) plus the one aggregation over the
// frequency table that every ScanShareableFrequencyBasedAnalyzer shares (AnalysisRunner.scala:
// 490-500): Σ[count == 1], count(*), Σ −(c/n)·ln(c/n).
//
// Table: open addressing (linear probing) in HBM, structure of arrays keys[] / counts[] (/ reps[]).
//   * exact mode  -- one fixed-width key column: the key is the value itself widened to 64 bits;
//   * hashed mode -- string keys, several key columns, or NULL-as-a-group (Histogram): the key is a
//     64-bit hash of the composite key; the first row of every group writes its encoded key into a
//     device arena (reps[] = arena offset) and a verification pass compares every row against its
//     group's encoded key, so a hash collision is detected instead of silently merging groups.
// Each workgroup first aggregates into a 2048-entry LDS table, so low-cardinality keys (priority:
// 3 groups) cost LDS atomics, not HBM atomics; keys that do not fit go straight to the HBM table.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "engine.h"
#include "kernels.h"

namespace dq {

#define DQ_DEV __device__ __forceinline__

constexpr uint64_t kEmpty = 0x8000000000000000ULL;
constexpr int kLdsSlots = 2048;
constexpr int kLdsProbes = 8;
constexpr int kMaxKeys = 8;

enum Counter { C_OCCUPIED = 0, C_NULL_ROWS, C_NULL_GROUP, C_SENTINEL, C_COLLISIONS, C_ARENA_OVF, C_N };

struct KeyCol {
  int32_t type;
  int32_t pad;
  const uint8_t* valid;
  const void* values;
  const uint8_t* data;
};

struct FreqDev {
  uint64_t* keys;
  uint64_t* counts;
  uint64_t* reps;
  uint64_t mask;
  uint8_t* arena;
  uint64_t* arena_cursor;
  uint64_t arena_cap;
  unsigned long long* counters;
  int32_t n_keys;
  int32_t exact;
  int32_t null_as_group;
  int32_t pad;
  KeyCol cols[kMaxKeys];
};

DQ_DEV uint32_t fbit(const uint8_t* bm, int64_t r) { return bm ? ((bm[r >> 3] >> (r & 7)) & 1u) : 1u; }

DQ_HD uint64_t mix64(uint64_t z) {
  z ^= z >> 33;
  z *= 0xff51afd7ed558ccdULL;
  z ^= z >> 33;
  z *= 0xc4ceb9fe1a85ec53ULL;
  z ^= z >> 33;
  return z;
}

DQ_DEV uint64_t widen(int type, const void* v, int64_t r) {
  switch (type) {
    case DQ_INT8: return (uint64_t)(int64_t) reinterpret_cast<const int8_t*>(v)[r];
    case DQ_INT16: return (uint64_t)(int64_t) reinterpret_cast<const int16_t*>(v)[r];
    case DQ_INT32: return (uint64_t)(int64_t) reinterpret_cast<const int32_t*>(v)[r];
    case DQ_INT64: return (uint64_t) reinterpret_cast<const int64_t*>(v)[r];
    case DQ_FLOAT32: return (uint64_t)__builtin_bit_cast(uint32_t, reinterpret_cast<const float*>(v)[r]);
    case DQ_FLOAT64: return __builtin_bit_cast(uint64_t, reinterpret_cast<const double*>(v)[r]);
    case DQ_BOOL: return fbit(reinterpret_cast<const uint8_t*>(v), r);
    default: return 0;
  }
}

struct FBytes {  // aligned-dword reader (see DevBytes in scan.hip)
  const uint8_t* p;
  DQ_DEV uint32_t u32(int64_t o) const {
    uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    uint32_t sh = (uint32_t)(a & 3) * 8;
    uint32_t w0 = w[0];
    if (sh == 0) return w0;
    return (w0 >> sh) | (w[1] << (32 - sh));
  }
  DQ_DEV uint64_t u64(int64_t o) const { return (uint64_t)u32(o) | ((uint64_t)u32(o + 4) << 32); }
  DQ_DEV uint32_t u8(int64_t o) const {
    uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    return (w[0] >> ((a & 3) * 8)) & 0xffu;
  }
};

// Row key: hash (hashed mode) or widened value (exact mode).  Returns false when the row is
// skipped (a NULL key outside histogram mode); sets is_null for an exact-mode NULL group row.
DQ_DEV bool row_key(const FreqDev& f, int64_t r, uint64_t& key, bool& is_null) {
  is_null = false;
  if (f.exact) {
    const KeyCol& c = f.cols[0];
    if (!fbit(c.valid, r)) {
      is_null = true;
      return f.null_as_group != 0;
    }
    key = widen(c.type, c.values, r);
    return true;
  }
  uint64_t h = 0x243F6A8885A308D3ULL;
  for (int k = 0; k < f.n_keys; ++k) {
    const KeyCol& c = f.cols[k];
    uint64_t ch;
    if (!fbit(c.valid, r)) {
      if (!f.null_as_group) return false;
      ch = 0x6e756c6c6e756c6cULL + k;
    } else if (c.type == DQ_UTF8) {
      const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
      int32_t s = off[r], e = off[r + 1];
      FBytes rd{c.data + s};
      ch = xxh_bytes(rd, (int64_t)(e - s), 17 + k);
    } else {
      ch = xxh_long(widen(c.type, c.values, r), 17 + k);
    }
    h = rotl64(h ^ ch, 27) * P1 + P4;
  }
  h = mix64(h);
  if (h == kEmpty) h ^= 1;
  key = h;
  return true;
}

// encoded key: per column u32 tag (0 NULL, 1 value) then 8 value bytes, or u32 length + bytes
// padded to 4
DQ_DEV uint64_t encoded_size(const FreqDev& f, int64_t r) {
  uint64_t n = 0;
  for (int k = 0; k < f.n_keys; ++k) {
    const KeyCol& c = f.cols[k];
    n += 4;
    if (!fbit(c.valid, r)) continue;
    if (c.type == DQ_UTF8) {
      const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
      n += 4 + (((uint64_t)(off[r + 1] - off[r]) + 3) & ~3ULL);
    } else {
      n += 8;
    }
  }
  return n;
}

DQ_DEV void encode_row(const FreqDev& f, int64_t r, uint8_t* dst) {
  uint32_t* w = reinterpret_cast<uint32_t*>(dst);
  for (int k = 0; k < f.n_keys; ++k) {
    const KeyCol& c = f.cols[k];
    if (!fbit(c.valid, r)) {
      *w++ = 0;
      continue;
    }
    *w++ = 1;
    if (c.type == DQ_UTF8) {
      const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
      int32_t s = off[r], e = off[r + 1], len = e - s;
      *w++ = (uint32_t)len;
      FBytes rd{c.data + s};
      for (int32_t q = 0; q < len; q += 4) {
        uint32_t v = 0;
        for (int b = 0; b < 4 && q + b < len; ++b) v |= rd.u8(q + b) << (8 * b);
        *w++ = v;
      }
    } else {
      uint64_t v = widen(c.type, c.values, r);
      *w++ = (uint32_t)v;
      *w++ = (uint32_t)(v >> 32);
    }
  }
}

DQ_DEV bool row_matches(const FreqDev& f, int64_t r, const uint8_t* enc) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(enc);
  for (int k = 0; k < f.n_keys; ++k) {
    const KeyCol& c = f.cols[k];
    uint32_t tag = *w++;
    bool valid = fbit(c.valid, r) != 0;
    if (!valid) {
      if (tag != 0) return false;
      continue;
    }
    if (tag != 1) return false;
    if (c.type == DQ_UTF8) {
      const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
      int32_t s = off[r], e = off[r + 1], len = e - s;
      if (*w++ != (uint32_t)len) return false;
      FBytes rd{c.data + s};
      for (int32_t q = 0; q < len; q += 4) {
        uint32_t v = 0;
        for (int b = 0; b < 4 && q + b < len; ++b) v |= rd.u8(q + b) << (8 * b);
        uint32_t mask = len - q >= 4 ? 0xffffffffu : ((1u << (8 * (len - q))) - 1u);
        if ((*w++ & mask) != v) return false;
      }
    } else {
      uint64_t v = widen(c.type, c.values, r);
      uint64_t s = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
      w += 2;
      if (s != v) return false;
    }
  }
  return true;
}

// Source of a group's encoded key when a new group is created in the HBM table.
struct RowSrc {
  int64_t row;
};
struct ArenaSrc {
  const uint8_t* enc;
  uint64_t size;
};

DQ_DEV void write_arena(const FreqDev& f, uint64_t slot, const RowSrc& s) {
  uint64_t size = encoded_size(f, s.row);
  unsigned long long off = atomicAdd(reinterpret_cast<unsigned long long*>(f.arena_cursor),
                                     (unsigned long long)size);
  if (off + size > f.arena_cap) {
    atomicAdd(&f.counters[C_ARENA_OVF], 1ULL);
    f.reps[slot] = ~0ULL;
    return;
  }
  encode_row(f, s.row, f.arena + off);
  f.reps[slot] = off;
}
DQ_DEV void write_arena(const FreqDev& f, uint64_t slot, const ArenaSrc& s) {
  unsigned long long off = atomicAdd(reinterpret_cast<unsigned long long*>(f.arena_cursor),
                                     (unsigned long long)s.size);
  if (off + s.size > f.arena_cap) {
    atomicAdd(&f.counters[C_ARENA_OVF], 1ULL);
    f.reps[slot] = ~0ULL;
    return;
  }
  const uint32_t* src = reinterpret_cast<const uint32_t*>(s.enc);
  uint32_t* dst = reinterpret_cast<uint32_t*>(f.arena + off);
  for (uint64_t q = 0; q < s.size / 4; ++q) dst[q] = src[q];
  f.reps[slot] = off;
}

// Sum over the wave, added to a table counter by lane 0: the counters are single addresses, so
// one atomic per row (every new group, every NULL row) would serialize the whole launch on them.
// Every lane of the wave must call it (the kernels call it after their row loops).
DQ_DEV void wave_count(unsigned long long* counter, unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (__lane_id() == 0 && v) atomicAdd(counter, v);
}

// Returns 1 when the call created the group (the caller counts C_OCCUPIED with wave_count).
template <typename Src>
DQ_DEV uint32_t insert_global(const FreqDev& f, uint64_t key, uint64_t cnt, const Src& src) {
  if (f.exact && key == kEmpty) {
    atomicAdd(&f.counters[C_SENTINEL], (unsigned long long)cnt);
    return 0;
  }
  uint64_t slot = (f.exact ? mix64(key) : key) & f.mask;
  for (uint64_t probe = 0; probe <= f.mask; ++probe) {
    uint64_t k = __hip_atomic_load(&f.keys[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&f.counts[slot]), (unsigned long long)cnt);
      return 0;
    }
    if (k == kEmpty) {
      unsigned long long prev =
          atomicCAS(reinterpret_cast<unsigned long long*>(&f.keys[slot]), (unsigned long long)kEmpty,
                    (unsigned long long)key);
      if (prev == kEmpty) {
        atomicAdd(reinterpret_cast<unsigned long long*>(&f.counts[slot]), (unsigned long long)cnt);
        if (!f.exact) write_arena(f, slot, src);
        return 1;
      }
      if (prev == key) {
        atomicAdd(reinterpret_cast<unsigned long long*>(&f.counts[slot]), (unsigned long long)cnt);
        return 0;
      }
    }
    slot = (slot + 1) & f.mask;
  }
  atomicAdd(&f.counters[C_ARENA_OVF], 1ULL);  // table full: the host sized it, cannot happen
  return 0;
}

__global__ void __launch_bounds__(256) freq_insert_kernel(FreqDev f, int64_t rows, int64_t chunk) {
  __shared__ unsigned long long lkeys[kLdsSlots];
  __shared__ unsigned int lcnt[kLdsSlots];
  __shared__ long long lrep[kLdsSlots];
  for (int i = threadIdx.x; i < kLdsSlots; i += blockDim.x) {
    lkeys[i] = kEmpty;
    lcnt[i] = 0;
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * chunk;
  const int64_t r1 = min(r0 + chunk, rows);
  unsigned long long nulls = 0, null_group = 0, sentinel = 0, created = 0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    uint64_t key;
    bool is_null;
    if (!row_key(f, r, key, is_null)) {
      ++nulls;
      continue;
    }
    if (is_null) {  // exact mode NULL group (histogram)
      ++null_group;
      continue;
    }
    if (f.exact && key == kEmpty) {  // the key equal to the empty marker lives outside the tables
      ++sentinel;
      continue;
    }
    bool done = false;
    uint32_t ls = (uint32_t)mix64(key) & (kLdsSlots - 1);
    for (int p = 0; p < kLdsProbes && !done; ++p) {
      unsigned long long k = lkeys[ls];
      if (k == key) {
        atomicAdd(&lcnt[ls], 1u);
        done = true;
      } else if (k == kEmpty) {
        unsigned long long prev = atomicCAS(&lkeys[ls], (unsigned long long)kEmpty,
                                            (unsigned long long)key);
        if (prev == kEmpty) {
          lrep[ls] = r;
          atomicAdd(&lcnt[ls], 1u);
          done = true;
        } else if (prev == key) {
          atomicAdd(&lcnt[ls], 1u);
          done = true;
        }
      }
      ls = (ls + 1) & (kLdsSlots - 1);
    }
    if (!done) created += insert_global(f, key, 1, RowSrc{r});
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLdsSlots; i += blockDim.x) {
    if (lkeys[i] != kEmpty) created += insert_global(f, lkeys[i], lcnt[i], RowSrc{lrep[i]});
  }
  wave_count(&f.counters[C_OCCUPIED], created);
  wave_count(&f.counters[C_NULL_ROWS], nulls);
  wave_count(&f.counters[C_NULL_GROUP], null_group);
  wave_count(&f.counters[C_SENTINEL], sentinel);
}

DQ_DEV int64_t find_slot(const FreqDev& f, uint64_t key) {
  uint64_t slot = key & f.mask;
  for (uint64_t probe = 0; probe <= f.mask; ++probe) {
    uint64_t k = f.keys[slot];
    if (k == key) return (int64_t)slot;
    if (k == kEmpty) return -1;
    slot = (slot + 1) & f.mask;
  }
  return -1;
}

__global__ void __launch_bounds__(256) freq_verify_kernel(FreqDev f, int64_t rows) {
  unsigned long long bad = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    uint64_t key;
    bool is_null;
    if (!row_key(f, r, key, is_null)) continue;
    int64_t slot = find_slot(f, key);
    if (slot < 0 || f.reps[slot] == ~0ULL || !row_matches(f, r, f.arena + f.reps[slot])) ++bad;
  }
  if (bad) atomicAdd(&f.counters[C_COLLISIONS], bad);
}

// Re-inserts the groups of another table (merge / rehash).
__global__ void __launch_bounds__(256) freq_merge_kernel(FreqDev dst, const uint64_t* keys,
                                                         const uint64_t* counts, const uint64_t* reps,
                                                         const uint8_t* arena, uint64_t cap,
                                                         int n_keys) {
  unsigned long long created = 0;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = keys[s];
    if (k == kEmpty) continue;
    uint64_t c = counts[s];
    if (dst.exact) {
      created += insert_global(dst, k, c, RowSrc{0});
    } else {
      const uint8_t* enc = arena + reps[s];
      // size of the encoded record
      const uint32_t* w = reinterpret_cast<const uint32_t*>(enc);
      uint64_t size = 0;
      for (int q = 0; q < n_keys; ++q) {
        uint32_t tag = w[size / 4];
        size += 4;
        if (!tag) continue;
        const KeyCol& col = dst.cols[q];
        if (col.type == DQ_UTF8) {
          uint32_t len = w[size / 4];
          size += 4 + ((len + 3) & ~3u);
        } else {
          size += 8;
        }
      }
      created += insert_global(dst, k, c, ArenaSrc{enc, size});
    }
  }
  wave_count(&dst.counters[C_OCCUPIED], created);
}

// Σ[count == 1], count(*), Σ −(c/n)·ln(c/n): per-block partials in a fixed slot order.
__global__ void __launch_bounds__(256) freq_summary_kernel(const uint64_t* keys,
                                                           const uint64_t* counts, uint64_t cap,
                                                           double num_rows, int64_t* out_i,
                                                           double* out_d) {
  __shared__ int64_t sg[256], su[256];
  __shared__ double se[256];
  const uint64_t per = (cap + gridDim.x - 1) / gridDim.x;
  const uint64_t s0 = (uint64_t)blockIdx.x * per, s1 = min(s0 + per, cap);
  int64_t g = 0, u = 0;
  double e = 0.0;
  for (uint64_t s = s0 + threadIdx.x; s < s1; s += blockDim.x) {
    if (keys[s] == kEmpty) continue;
    uint64_t c = counts[s];
    ++g;
    u += c == 1;
    double p = (double)c / num_rows;
    e += -p * log(p);
  }
  sg[threadIdx.x] = g;
  su[threadIdx.x] = u;
  se[threadIdx.x] = e;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) {
      sg[threadIdx.x] += sg[threadIdx.x + st];
      su[threadIdx.x] += su[threadIdx.x + st];
      se[threadIdx.x] += se[threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out_i[2 * blockIdx.x] = sg[0];
    out_i[2 * blockIdx.x + 1] = su[0];
    out_d[blockIdx.x] = se[0];
  }
}

__global__ void __launch_bounds__(256) freq_compact_kernel(const uint64_t* keys,
                                                           const uint64_t* counts,
                                                           const uint64_t* reps, uint64_t cap,
                                                           unsigned long long* cursor,
                                                           uint64_t* out_keys, uint64_t* out_counts,
                                                           uint64_t* out_reps) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * blockDim.x) {
    if (keys[s] == kEmpty) continue;
    unsigned long long i = atomicAdd(cursor, 1ULL);
    out_keys[i] = keys[s];
    out_counts[i] = counts[s];
    if (reps) out_reps[i] = reps[s];
  }
}

// ------------------------------------------------------------------------------------------------
// Hash repartition (multi-GPU frequency path): the reference's groupBy runs a
// partial HashAggregate per partition, a hash-partitioned Exchange and a final aggregate
// (GroupingAnalyzers.scala:70).  Here each rank's table IS the partial aggregate; its groups are cut
// into one segment per owner rank (owner from the HIGH bits of the slot hash, so the owner's own
// table, which indexes by the low bits, stays uniformly loaded), exchanged by RCCL all-to-all, and
// re-inserted with their counts on the owner.
// Wire format per segment: fixed records {key, count, enc_off} (enc_off = byte offset of the group's
// encoded key inside the segment's var bytes; unused in exact mode) + var bytes (8-aligned).
// ------------------------------------------------------------------------------------------------
struct FreqRecord {
  uint64_t key;
  uint64_t count;
  uint64_t enc_off;
};

constexpr int kMaxParts = 64;

DQ_DEV uint32_t owner_of(uint64_t key, int exact, uint32_t parts) {
  uint64_t h = exact ? mix64(key) : key;
  return (uint32_t)(((h >> 40) * (uint64_t)parts) >> 24);
}

DQ_DEV uint64_t enc_record_size(const uint8_t* enc, const int32_t* types, int n_keys) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(enc);
  uint64_t size = 0;
  for (int q = 0; q < n_keys; ++q) {
    uint32_t tag = w[size / 4];
    size += 4;
    if (!tag) continue;
    if (types[q] == DQ_UTF8) size += 4 + ((w[size / 4] + 3) & ~3u);
    else size += 8;
  }
  return size;
}

struct PartArgs {
  int32_t types[kMaxKeys];
  int32_t n_keys;
  int32_t exact;
  uint32_t parts;
  uint32_t pad;
};

// pass 1: records and var bytes per owner
__global__ void __launch_bounds__(256) freq_part_count_kernel(const uint64_t* keys, const uint64_t* reps,
                                                              const uint8_t* arena, uint64_t cap,
                                                              PartArgs a,
                                                              unsigned long long* n_rec,
                                                              unsigned long long* n_var) {
  __shared__ unsigned long long lr[kMaxParts], lv[kMaxParts];
  for (int i = threadIdx.x; i < kMaxParts; i += blockDim.x) lr[i] = lv[i] = 0;
  __syncthreads();
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = keys[s];
    if (k == kEmpty) continue;
    uint32_t o = owner_of(k, a.exact, a.parts);
    atomicAdd(&lr[o], 1ULL);
    if (!a.exact) atomicAdd(&lv[o], (enc_record_size(arena + reps[s], a.types, a.n_keys) + 7) & ~7ULL);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < a.parts; i += blockDim.x) {
    if (lr[i]) atomicAdd(&n_rec[i], lr[i]);
    if (lv[i]) atomicAdd(&n_var[i], lv[i]);
  }
}

// pass 2: scatter into the owner segments (rec_base / var_base = exclusive prefix sums of pass 1)
__global__ void __launch_bounds__(256) freq_part_scatter_kernel(
    const uint64_t* keys, const uint64_t* counts, const uint64_t* reps, const uint8_t* arena,
    uint64_t cap, PartArgs a, const unsigned long long* rec_base, const unsigned long long* var_base,
    unsigned long long* rec_cur, unsigned long long* var_cur, FreqRecord* out_rec, uint8_t* out_var) {
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = keys[s];
    if (k == kEmpty) continue;
    uint32_t o = owner_of(k, a.exact, a.parts);
    unsigned long long i = atomicAdd(&rec_cur[o], 1ULL);
    FreqRecord r{k, counts[s], 0};
    if (!a.exact) {
      const uint8_t* enc = arena + reps[s];
      uint64_t size = enc_record_size(enc, a.types, a.n_keys);
      unsigned long long off = atomicAdd(&var_cur[o], (size + 7) & ~7ULL);
      const uint32_t* src = reinterpret_cast<const uint32_t*>(enc);
      uint32_t* dst = reinterpret_cast<uint32_t*>(out_var + var_base[o] + off);
      for (uint64_t q = 0; q < size / 4; ++q) dst[q] = src[q];
      r.enc_off = off;
    }
    out_rec[rec_base[o] + i] = r;
  }
}

struct SrcSegs {
  int64_t rec_start[kMaxParts + 1];  // records of source j: [rec_start[j], rec_start[j+1])
  int64_t var_base[kMaxParts];       // byte offset of source j's var segment
  int32_t n_src;
};

DQ_DEV const uint8_t* record_enc(const FreqRecord& r, int64_t i, const uint8_t* var,
                                 const SrcSegs& segs) {
  int j = 0;
  while (j + 1 < segs.n_src && i >= segs.rec_start[j + 1]) ++j;
  return var + segs.var_base[j] + r.enc_off;
}

// Re-inserts received groups with their counts (the final aggregate after the Exchange).
__global__ void __launch_bounds__(256) freq_insert_records_kernel(FreqDev f, const FreqRecord* rec,
                                                                  const uint8_t* var, SrcSegs segs,
                                                                  PartArgs a) {
  const int64_t n = segs.rec_start[segs.n_src];
  unsigned long long created = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    FreqRecord r = rec[i];
    if (f.exact) {
      created += insert_global(f, r.key, r.count, RowSrc{0});
    } else {
      const uint8_t* enc = record_enc(r, i, var, segs);
      created += insert_global(f, r.key, r.count,
                               ArenaSrc{enc, enc_record_size(enc, a.types, a.n_keys)});
    }
  }
  wave_count(&f.counters[C_OCCUPIED], created);
}

// Hashed mode: every received group must carry the same encoded key as the group it landed in, so
// a 64-bit hash collision between groups of different ranks is detected, never merged.
__global__ void __launch_bounds__(256) freq_verify_records_kernel(FreqDev f, const FreqRecord* rec,
                                                                  const uint8_t* var, SrcSegs segs,
                                                                  PartArgs a) {
  const int64_t n = segs.rec_start[segs.n_src];
  unsigned long long bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    FreqRecord r = rec[i];
    const uint32_t* enc = reinterpret_cast<const uint32_t*>(record_enc(r, i, var, segs));
    int64_t slot = find_slot(f, r.key);
    if (slot < 0 || f.reps[slot] == ~0ULL) {
      ++bad;
      continue;
    }
    const uint32_t* have = reinterpret_cast<const uint32_t*>(f.arena + f.reps[slot]);
    uint64_t size = enc_record_size(reinterpret_cast<const uint8_t*>(enc), a.types, a.n_keys);
    for (uint64_t q = 0; q < size / 4; ++q)
      if (have[q] != enc[q]) {
        ++bad;
        break;
      }
  }
  if (bad) atomicAdd(&f.counters[C_COLLISIONS], bad);
}

__global__ void fill_u64(uint64_t* p, uint64_t n, uint64_t v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

}  // namespace dq

using namespace dq;

// ------------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------------
struct dq_freq {
  int device = 0;
  int n_keys = 0;
  std::vector<int32_t> types;
  bool exact = false;
  int mode_null_as_group = -1;  // fixed by the first add
  uint64_t cap = 0;             // slots (power of two)
  DevBuf<uint64_t> keys, counts, reps;
  DevBuf<uint8_t> arena;
  DevBuf<uint64_t> arena_cursor;
  DevBuf<unsigned long long> counters;
  uint64_t h_counters[C_N] = {0, 0, 0, 0, 0, 0};
  uint64_t arena_used = 0;
  int64_t num_rows = 0;
  hipStream_t stream = nullptr;
};

static unsigned grid_for(uint64_t n, unsigned cap = 4096) {
  uint64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

static FreqDev dev_view(dq_freq* f) {
  FreqDev d;
  memset(&d, 0, sizeof(d));
  d.keys = f->keys.p;
  d.counts = f->counts.p;
  d.reps = f->exact ? nullptr : f->reps.p;
  d.mask = f->cap - 1;
  d.arena = f->arena.p;
  d.arena_cursor = f->arena_cursor.p;
  d.arena_cap = f->arena.p ? f->arena.n : 0;
  d.counters = f->counters.p;
  d.n_keys = f->n_keys;
  d.exact = f->exact ? 1 : 0;
  d.null_as_group = f->mode_null_as_group > 0 ? 1 : 0;
  // key types are needed by every kernel that sizes an encoded key (rehash / merge re-inserts)
  for (int k = 0; k < f->n_keys; ++k) d.cols[k].type = f->types[k];
  return d;
}

static dq_status pull_counters(dq_freq* f) {
  HIP_TRY(hipStreamSynchronize(f->stream));
  unsigned long long c[C_N];
  HIP_TRY(hipMemcpy(c, f->counters.p, sizeof(c), hipMemcpyDeviceToHost));
  for (int k = 0; k < C_N; ++k) f->h_counters[k] = c[k];
  uint64_t cur = 0;
  if (!f->exact) HIP_TRY(hipMemcpy(&cur, f->arena_cursor.p, 8, hipMemcpyDeviceToHost));
  f->arena_used = cur;
  return DQ_OK;
}

// Grows the slot arrays to `new_cap` and re-inserts every group.
static dq_status rehash(dq_freq* f, uint64_t new_cap) {
  DevBuf<uint64_t> ok, oc, orp;
  ok.swap(f->keys);
  oc.swap(f->counts);
  orp.swap(f->reps);
  uint64_t old_cap = f->cap;
  DevBuf<uint8_t> oarena;
  oarena.swap(f->arena);
  HIP_TRY(f->keys.ensure(new_cap));
  HIP_TRY(f->counts.ensure(new_cap));
  if (!f->exact) HIP_TRY(f->reps.ensure(new_cap));
  hipLaunchKernelGGL(fill_u64, dim3(grid_for(new_cap)), dim3(256), 0, f->stream, f->keys.p, new_cap,
                     kEmpty);
  HIP_TRY(hipMemsetAsync(f->counts.p, 0, new_cap * 8, f->stream));
  f->cap = new_cap;
  if (!f->exact) {
    HIP_TRY(f->arena.ensure(std::max<uint64_t>(oarena.n, 64)));
    HIP_TRY(hipMemsetAsync(f->arena_cursor.p, 0, 8, f->stream));
  }
  // occupied is recounted by the re-insert
  HIP_TRY(hipMemsetAsync(f->counters.p + C_OCCUPIED, 0, 8, f->stream));
  if (old_cap) {
    FreqDev d = dev_view(f);
    hipLaunchKernelGGL(freq_merge_kernel, dim3(grid_for(old_cap)), dim3(256), 0, f->stream, d, ok.p,
                       oc.p, f->exact ? nullptr : orp.p, oarena.p, old_cap, f->n_keys);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(f->stream));
  return pull_counters(f);
}

extern "C" dq_status dq_freq_create(int device, int n_keys, const int32_t* key_types,
                                    int64_t capacity_hint, dq_freq** out) {
  if (!out || !key_types || n_keys <= 0) return fail(DQ_ERR_INVALID_ARGUMENT, "bad arguments");
  if (n_keys > kMaxKeys) return fail(DQ_ERR_UNSUPPORTED, "at most %d grouping columns", kMaxKeys);
  *out = nullptr;
  auto f = std::make_unique<dq_freq>();
  f->device = device;
  f->n_keys = n_keys;
  f->types.assign(key_types, key_types + n_keys);
  for (int t : f->types)
    if (t < DQ_BOOL || t > DQ_UTF8) return fail(DQ_ERR_INVALID_ARGUMENT, "bad key type %d", t);
  f->exact = n_keys == 1 && f->types[0] != DQ_UTF8;
  if (n_keys > 1)
    for (int t : f->types)
      if (t != DQ_UTF8)
        return fail(DQ_ERR_UNSUPPORTED,
                    "grouping on several columns is implemented for string columns only");
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(f->counters.ensure(C_N));
  HIP_TRY(hipMemset(f->counters.p, 0, C_N * 8));
  HIP_TRY(f->arena_cursor.ensure(1));
  HIP_TRY(hipMemset(f->arena_cursor.p, 0, 8));
  uint64_t cap = 1024;
  while (cap < (uint64_t)std::max<int64_t>(0, capacity_hint) * 2) cap <<= 1;
  dq_status st = rehash(f.get(), cap);
  if (st != DQ_OK) return st;
  *out = f.release();
  return DQ_OK;
}

// Empties the table but keeps its capacity (slot arrays and arena), like a Spark task reusing its
// aggregation buffer: repeated group-bys of the same shape pay no device allocation.
extern "C" dq_status dq_freq_reset(dq_freq* f, void* hip_stream) {
  if (!f) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  f->stream = reinterpret_cast<hipStream_t>(hip_stream);
  hipLaunchKernelGGL(fill_u64, dim3(grid_for(f->cap)), dim3(256), 0, f->stream, f->keys.p, f->cap,
                     kEmpty);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemsetAsync(f->counts.p, 0, f->cap * 8, f->stream));
  HIP_TRY(hipMemsetAsync(f->counters.p, 0, C_N * 8, f->stream));
  HIP_TRY(hipMemsetAsync(f->arena_cursor.p, 0, 8, f->stream));
  for (int k = 0; k < C_N; ++k) f->h_counters[k] = 0;
  f->arena_used = 0;
  f->num_rows = 0;
  f->mode_null_as_group = -1;
  return DQ_OK;
}

extern "C" void dq_freq_destroy(dq_freq* f) {
  if (!f) return;
  (void)hipSetDevice(f->device);
  (void)hipStreamSynchronize(f->stream);
  delete f;
}

extern "C" dq_status dq_freq_add_device(dq_freq* f, const dq_column* keys, int n_keys,
                                        int null_as_group, void* hip_stream) {
  if (!f || !keys) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (n_keys != f->n_keys) return fail(DQ_ERR_INVALID_ARGUMENT, "expected %d key columns", f->n_keys);
  int mode = null_as_group ? 1 : 0;
  if (f->mode_null_as_group >= 0 && f->mode_null_as_group != mode)
    return fail(DQ_ERR_STATE, "null_as_group must be the same for every batch");
  f->mode_null_as_group = mode;
  if (mode && f->n_keys != 1) return fail(DQ_ERR_UNSUPPORTED, "NULL-as-group needs one key column");
  int64_t rows = keys[0].length;
  for (int k = 0; k < n_keys; ++k) {
    if (keys[k].type != f->types[k]) return fail(DQ_ERR_WRONG_TYPE, "key %d has the wrong type", k);
    if (keys[k].length != rows) return fail(DQ_ERR_INVALID_ARGUMENT, "key columns differ in length");
    if (rows > 0 && !keys[k].values) return fail(DQ_ERR_INVALID_ARGUMENT, "key %d has no values", k);
  }
  HIP_TRY(hipSetDevice(f->device));
  f->stream = reinterpret_cast<hipStream_t>(hip_stream);
  f->num_rows += rows;
  if (rows == 0) return DQ_OK;
  // capacity: keep the load factor <= 1/2 even if every row is a new group
  uint64_t need = 2 * (f->h_counters[C_OCCUPIED] + (uint64_t)rows);
  if (need > f->cap) {
    uint64_t cap = f->cap;
    while (cap < need) cap <<= 1;
    dq_status st = rehash(f, cap);
    if (st != DQ_OK) return st;
  }
  if (!f->exact) {
    // arena: worst case every row a new group
    uint64_t extra = 0;
    for (int k = 0; k < n_keys; ++k) {
      extra += (uint64_t)rows * 12;
      if (keys[k].type == DQ_UTF8) {
        int32_t last = 0;
        HIP_TRY(hipMemcpy(&last, reinterpret_cast<const int32_t*>(keys[k].values) + rows, 4,
                          hipMemcpyDeviceToHost));
        int32_t first = 0;
        HIP_TRY(hipMemcpy(&first, keys[k].values, 4, hipMemcpyDeviceToHost));
        extra += (uint64_t)(last - first) + (uint64_t)rows * 3;
      }
    }
    uint64_t want = f->arena_used + extra + 64;
    if (want > f->arena.n) {
      // grow, keeping the existing bytes
      DevBuf<uint8_t> bigger;
      HIP_TRY(bigger.ensure(std::max<uint64_t>(want, f->arena.n * 2)));
      if (f->arena_used)
        HIP_TRY(hipMemcpyAsync(bigger.p, f->arena.p, f->arena_used, hipMemcpyDeviceToDevice, f->stream));
      HIP_TRY(hipStreamSynchronize(f->stream));
      f->arena.swap(bigger);
    }
  }
  FreqDev d = dev_view(f);
  for (int k = 0; k < n_keys; ++k)
    d.cols[k] = KeyCol{keys[k].type, 0, keys[k].validity, keys[k].values, keys[k].data};
  unsigned grid = grid_for((uint64_t)rows, 2048);
  int64_t chunk = (rows + grid - 1) / grid;
  hipLaunchKernelGGL(freq_insert_kernel, dim3(grid), dim3(256), 0, f->stream, d, rows, chunk);
  HIP_TRY(hipGetLastError());
  if (!f->exact) {
    hipLaunchKernelGGL(freq_verify_kernel, dim3(grid_for((uint64_t)rows, 4096)), dim3(256), 0,
                       f->stream, d, rows);
    HIP_TRY(hipGetLastError());
  }
  dq_status st = pull_counters(f);
  if (st != DQ_OK) return st;
  if (f->h_counters[C_ARENA_OVF])
    return fail(DQ_ERR_OUT_OF_MEMORY, "frequency table arena overflow");
  if (f->h_counters[C_COLLISIONS])
    return fail(DQ_ERR_UNSUPPORTED,
                "64-bit key-hash collision between distinct groups detected (%llu rows)",
                (unsigned long long)f->h_counters[C_COLLISIONS]);
  return DQ_OK;
}

extern "C" dq_status dq_freq_summarize(dq_freq* f, dq_freq_summary* out) {
  if (!f || !out) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  const unsigned G = grid_for(f->cap, 8192);  // >= 32 blocks per CU: enough loads in flight
  DevBuf<int64_t> pi;
  DevBuf<double> pd;
  HIP_TRY(pi.ensure(2 * G));
  HIP_TRY(pd.ensure(G));
  const double n = (double)f->num_rows;
  hipLaunchKernelGGL(freq_summary_kernel, dim3(G), dim3(256), 0, f->stream, f->keys.p, f->counts.p,
                     f->cap, n, pi.p, pd.p);
  HIP_TRY(hipGetLastError());
  std::vector<int64_t> hi(2 * G);
  std::vector<double> hd(G);
  HIP_TRY(hipStreamSynchronize(f->stream));
  HIP_TRY(hipMemcpy(hi.data(), pi.p, hi.size() * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(hd.data(), pd.p, hd.size() * 8, hipMemcpyDeviceToHost));
  dq_status st = pull_counters(f);
  if (st != DQ_OK) return st;
  int64_t g = 0, u = 0;
  double e = 0.0;
  for (unsigned b = 0; b < G; ++b) {
    g += hi[2 * b];
    u += hi[2 * b + 1];
    e += hd[b];
  }
  auto extra_group = [&](uint64_t c) {
    if (!c) return;
    ++g;
    u += c == 1;
    double p = (double)c / n;
    e += -p * std::log(p);
  };
  extra_group(f->h_counters[C_SENTINEL]);
  extra_group(f->h_counters[C_NULL_GROUP]);
  out->num_rows = f->num_rows;
  out->n_groups = g;
  out->n_unique = u;
  out->n_null_key_rows = (int64_t)f->h_counters[C_NULL_ROWS];
  out->entropy = e;
  return DQ_OK;
}

extern "C" dq_status dq_freq_num_groups(dq_freq* f, int64_t* n) {
  if (!f || !n) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = pull_counters(f);
  if (st != DQ_OK) return st;
  *n = (int64_t)(f->h_counters[C_OCCUPIED] + (f->h_counters[C_SENTINEL] ? 1 : 0) +
                 (f->h_counters[C_NULL_GROUP] ? 1 : 0));
  return DQ_OK;
}

// Exports every group: counts, and the encoded key of each group (see encode_row: per key column a
// u32 tag 0 = NULL / 1 = value, then 8 little-endian value bytes or a u32 length + bytes padded to
// 4).  key_offsets has n + 1 entries.  Pass key_bytes_out = NULL to query the byte size only.
extern "C" dq_status dq_freq_export(dq_freq* f, int64_t* counts_out, int64_t* key_offsets_out,
                                    uint8_t* key_bytes_out, int64_t capacity,
                                    int64_t key_bytes_capacity, int64_t* key_bytes_needed) {
  if (!f) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  int64_t n = 0;
  dq_status st = dq_freq_num_groups(f, &n);
  if (st != DQ_OK) return st;
  const uint64_t occ = f->h_counters[C_OCCUPIED];
  std::vector<uint64_t> hk(occ), hc(occ), hr(f->exact ? 0 : occ);
  if (occ) {
    DevBuf<uint64_t> ok, oc, orp;
    DevBuf<unsigned long long> cur;
    HIP_TRY(ok.ensure(occ));
    HIP_TRY(oc.ensure(occ));
    if (!f->exact) HIP_TRY(orp.ensure(occ));
    HIP_TRY(cur.ensure(1));
    HIP_TRY(hipMemsetAsync(cur.p, 0, 8, f->stream));
    hipLaunchKernelGGL(freq_compact_kernel, dim3(grid_for(f->cap)), dim3(256), 0, f->stream,
                       f->keys.p, f->counts.p, f->exact ? nullptr : f->reps.p, f->cap, cur.p, ok.p,
                       oc.p, f->exact ? nullptr : orp.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(f->stream));
    HIP_TRY(hipMemcpy(hk.data(), ok.p, occ * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(hc.data(), oc.p, occ * 8, hipMemcpyDeviceToHost));
    if (!f->exact) HIP_TRY(hipMemcpy(hr.data(), orp.p, occ * 8, hipMemcpyDeviceToHost));
  }
  std::vector<uint8_t> arena;
  if (!f->exact && f->arena_used) {
    arena.resize(f->arena_used);
    HIP_TRY(hipMemcpy(arena.data(), f->arena.p, f->arena_used, hipMemcpyDeviceToHost));
  }
  // assemble encoded keys
  std::vector<int64_t> counts;
  std::vector<uint8_t> bytes;
  std::vector<int64_t> offs;
  auto put32 = [&](uint32_t v) {
    for (int b = 0; b < 4; ++b) bytes.push_back((uint8_t)(v >> (8 * b)));
  };
  auto put_exact = [&](bool null, uint64_t v, uint64_t c) {
    offs.push_back((int64_t)bytes.size());
    counts.push_back((int64_t)c);
    put32(null ? 0 : 1);
    if (!null) {
      put32((uint32_t)v);
      put32((uint32_t)(v >> 32));
    }
  };
  for (uint64_t i = 0; i < occ; ++i) {
    if (f->exact) {
      put_exact(false, hk[i], hc[i]);
    } else {
      offs.push_back((int64_t)bytes.size());
      counts.push_back((int64_t)hc[i]);
      const uint8_t* enc = arena.data() + hr[i];
      const uint32_t* w = reinterpret_cast<const uint32_t*>(enc);
      uint64_t size = 0;
      for (int q = 0; q < f->n_keys; ++q) {
        uint32_t tag = w[size / 4];
        size += 4;
        if (!tag) continue;
        if (f->types[q] == DQ_UTF8) size += 4 + ((w[size / 4] + 3) & ~3u);
        else size += 8;
      }
      bytes.insert(bytes.end(), enc, enc + size);
    }
  }
  if (f->h_counters[C_SENTINEL]) put_exact(false, kEmpty, f->h_counters[C_SENTINEL]);
  if (f->h_counters[C_NULL_GROUP]) put_exact(true, 0, f->h_counters[C_NULL_GROUP]);
  offs.push_back((int64_t)bytes.size());
  if (key_bytes_needed) *key_bytes_needed = (int64_t)bytes.size();
  if (!key_bytes_out) return DQ_OK;
  if (capacity < (int64_t)counts.size() || key_bytes_capacity < (int64_t)bytes.size())
    return fail(DQ_ERR_INVALID_ARGUMENT, "export buffers too small");
  if (counts_out) memcpy(counts_out, counts.data(), counts.size() * 8);
  if (key_offsets_out) memcpy(key_offsets_out, offs.data(), offs.size() * 8);
  memcpy(key_bytes_out, bytes.data(), bytes.size());
  return DQ_OK;
}

// dst += src (FrequenciesAndNumRows.sum, GroupingAnalyzers.scala:128-148): counts of equal keys
// add, numRows add.
extern "C" dq_status dq_freq_merge(dq_freq* dst, const dq_freq* src) {
  if (!dst || !src) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (dst->n_keys != src->n_keys || dst->types != src->types)
    return fail(DQ_ERR_STATE, "frequency tables group on different key types");
  if (dst->device != src->device) return fail(DQ_ERR_UNSUPPORTED, "tables on different devices");
  if (dst->mode_null_as_group >= 0 && src->mode_null_as_group >= 0 &&
      dst->mode_null_as_group != src->mode_null_as_group)
    return fail(DQ_ERR_STATE, "frequency tables differ in NULL handling");
  HIP_TRY(hipSetDevice(dst->device));
  dq_freq* s = const_cast<dq_freq*>(src);
  HIP_TRY(hipStreamSynchronize(s->stream));
  dq_status st = pull_counters(s);
  if (st != DQ_OK) return st;
  if (dst->mode_null_as_group < 0) dst->mode_null_as_group = s->mode_null_as_group;
  uint64_t need = 2 * (dst->h_counters[C_OCCUPIED] + s->h_counters[C_OCCUPIED]) + 2;
  if (need > dst->cap) {
    uint64_t cap = dst->cap;
    while (cap < need) cap <<= 1;
    st = rehash(dst, cap);
    if (st != DQ_OK) return st;
  }
  if (!dst->exact) {
    uint64_t want = dst->arena_used + s->arena_used + 64;
    if (want > dst->arena.n) {
      DevBuf<uint8_t> bigger;
      HIP_TRY(bigger.ensure(want));
      if (dst->arena_used)
        HIP_TRY(hipMemcpy(bigger.p, dst->arena.p, dst->arena_used, hipMemcpyDeviceToDevice));
      dst->arena.swap(bigger);
    }
  }
  FreqDev d = dev_view(dst);
  for (int k = 0; k < dst->n_keys; ++k) d.cols[k].type = dst->types[k];
  hipLaunchKernelGGL(freq_merge_kernel, dim3(grid_for(s->cap)), dim3(256), 0, dst->stream, d,
                     s->keys.p, s->counts.p, s->exact ? nullptr : s->reps.p, s->arena.p, s->cap,
                     dst->n_keys);
  HIP_TRY(hipGetLastError());
  // special cells
  unsigned long long add[C_N] = {0, 0, 0, 0, 0, 0};
  HIP_TRY(hipStreamSynchronize(dst->stream));
  st = pull_counters(dst);
  if (st != DQ_OK) return st;
  add[C_NULL_ROWS] = dst->h_counters[C_NULL_ROWS] + s->h_counters[C_NULL_ROWS];
  add[C_NULL_GROUP] = dst->h_counters[C_NULL_GROUP] + s->h_counters[C_NULL_GROUP];
  add[C_SENTINEL] = dst->h_counters[C_SENTINEL] + s->h_counters[C_SENTINEL];
  add[C_OCCUPIED] = dst->h_counters[C_OCCUPIED];
  add[C_COLLISIONS] = dst->h_counters[C_COLLISIONS];
  add[C_ARENA_OVF] = dst->h_counters[C_ARENA_OVF];
  HIP_TRY(hipMemcpy(dst->counters.p, add, sizeof(add), hipMemcpyHostToDevice));
  dst->num_rows += s->num_rows;
  return pull_counters(dst);
}

extern "C" int64_t dq_freq_num_rows(const dq_freq* f) { return f ? f->num_rows : -1; }

// ------------------------------------------------------------------------------------------------
// Hash repartition for the multi-GPU frequency path (see the kernels above)
// ------------------------------------------------------------------------------------------------
static PartArgs part_args(const dq_freq* f, int n_parts) {
  PartArgs a;
  memset(&a, 0, sizeof(a));
  for (int k = 0; k < f->n_keys; ++k) a.types[k] = f->types[k];
  a.n_keys = f->n_keys;
  a.exact = f->exact ? 1 : 0;
  a.parts = (uint32_t)n_parts;
  return a;
}

// Per-owner record counts and var bytes (device counting pass).
static dq_status part_sizes(dq_freq* f, int n_parts, std::vector<unsigned long long>& rec,
                            std::vector<unsigned long long>& var) {
  DevBuf<unsigned long long> cnt;
  HIP_TRY(cnt.ensure(2 * kMaxParts));
  HIP_TRY(hipMemsetAsync(cnt.p, 0, 2 * kMaxParts * 8, f->stream));
  hipLaunchKernelGGL(freq_part_count_kernel, dim3(grid_for(f->cap)), dim3(256), 0, f->stream,
                     f->keys.p, f->exact ? nullptr : f->reps.p, f->arena.p, f->cap,
                     part_args(f, n_parts), cnt.p, cnt.p + kMaxParts);
  HIP_TRY(hipGetLastError());
  std::vector<unsigned long long> h(2 * kMaxParts);
  HIP_TRY(hipStreamSynchronize(f->stream));
  HIP_TRY(hipMemcpy(h.data(), cnt.p, h.size() * 8, hipMemcpyDeviceToHost));
  rec.assign(h.begin(), h.begin() + n_parts);
  var.assign(h.begin() + kMaxParts, h.begin() + kMaxParts + n_parts);
  return DQ_OK;
}

extern "C" dq_status dq_freq_partition_sizes(dq_freq* f, int n_parts, int64_t* rec_counts,
                                             int64_t* var_bytes, int64_t* special) {
  if (!f || !rec_counts || !var_bytes || !special)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (n_parts < 1 || n_parts > kMaxParts)
    return fail(DQ_ERR_UNSUPPORTED, "n_parts must be in [1, %d]", kMaxParts);
  HIP_TRY(hipSetDevice(f->device));
  dq_status st = pull_counters(f);
  if (st != DQ_OK) return st;
  std::vector<unsigned long long> rec, var;
  st = part_sizes(f, n_parts, rec, var);
  if (st != DQ_OK) return st;
  for (int i = 0; i < n_parts; ++i) {
    rec_counts[i] = (int64_t)rec[i];
    var_bytes[i] = (int64_t)var[i];
  }
  special[0] = (int64_t)f->h_counters[C_SENTINEL];
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
  std::vector<unsigned long long> rec, var_n;
  dq_status st = part_sizes(f, n_parts, rec, var_n);
  if (st != DQ_OK) return st;
  unsigned long long total_rec = 0, total_var = 0;
  std::vector<unsigned long long> base(4 * kMaxParts, 0);  // rec_base, var_base, rec_cur, var_cur
  for (int i = 0; i < n_parts; ++i) {
    base[i] = total_rec;
    base[kMaxParts + i] = total_var;
    total_rec += rec[i];
    total_var += var_n[i];
  }
  if (total_rec == 0) return DQ_OK;
  if (!records || (total_var && !var)) return fail(DQ_ERR_INVALID_ARGUMENT, "null output buffer");
  DevBuf<unsigned long long> dbase;
  HIP_TRY(dbase.ensure(base.size()));
  HIP_TRY(hipMemcpyAsync(dbase.p, base.data(), base.size() * 8, hipMemcpyHostToDevice, f->stream));
  hipLaunchKernelGGL(freq_part_scatter_kernel, dim3(grid_for(f->cap)), dim3(256), 0, f->stream,
                     f->keys.p, f->counts.p, f->exact ? nullptr : f->reps.p, f->arena.p, f->cap,
                     part_args(f, n_parts), dbase.p, dbase.p + kMaxParts, dbase.p + 2 * kMaxParts,
                     dbase.p + 3 * kMaxParts, reinterpret_cast<FreqRecord*>(records), var);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(f->stream));  // dbase is freed on return
  return DQ_OK;
}

extern "C" dq_status dq_freq_add_records_device(dq_freq* f, const dq_freq_record* records,
                                                const uint8_t* var, int n_src,
                                                const int64_t* src_records,
                                                const int64_t* src_var_bytes, int64_t num_rows,
                                                const int64_t* special, int null_as_group,
                                                void* hip_stream) {
  if (!f || !src_records || !src_var_bytes || !special)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (n_src < 1 || n_src > kMaxParts)
    return fail(DQ_ERR_UNSUPPORTED, "n_src must be in [1, %d]", kMaxParts);
  int mode = null_as_group ? 1 : 0;
  if (f->mode_null_as_group >= 0 && f->mode_null_as_group != mode)
    return fail(DQ_ERR_STATE, "null_as_group must be the same for every batch");
  f->mode_null_as_group = mode;
  HIP_TRY(hipSetDevice(f->device));
  HIP_TRY(hipStreamSynchronize(f->stream));
  f->stream = reinterpret_cast<hipStream_t>(hip_stream);
  SrcSegs segs;
  memset(&segs, 0, sizeof(segs));
  segs.n_src = n_src;
  int64_t total_rec = 0, total_var = 0;
  for (int j = 0; j < n_src; ++j) {
    if (src_records[j] < 0 || src_var_bytes[j] < 0 || (src_var_bytes[j] & 7))
      return fail(DQ_ERR_INVALID_ARGUMENT, "bad segment sizes for source %d", j);
    segs.rec_start[j] = total_rec;
    segs.var_base[j] = total_var;
    total_rec += src_records[j];
    total_var += src_var_bytes[j];
  }
  segs.rec_start[n_src] = total_rec;
  if (total_rec && !records) return fail(DQ_ERR_INVALID_ARGUMENT, "null records");
  if (!f->exact && total_var && !var) return fail(DQ_ERR_INVALID_ARGUMENT, "null var bytes");
  dq_status st = pull_counters(f);
  if (st != DQ_OK) return st;
  uint64_t need = 2 * (f->h_counters[C_OCCUPIED] + (uint64_t)total_rec) + 2;
  if (need > f->cap) {
    uint64_t cap = f->cap;
    while (cap < need) cap <<= 1;
    st = rehash(f, cap);
    if (st != DQ_OK) return st;
  }
  if (!f->exact) {
    uint64_t want = f->arena_used + (uint64_t)total_var + 64;
    if (want > f->arena.n) {
      DevBuf<uint8_t> bigger;
      HIP_TRY(bigger.ensure(std::max<uint64_t>(want, f->arena.n * 2)));
      if (f->arena_used)
        HIP_TRY(hipMemcpyAsync(bigger.p, f->arena.p, f->arena_used, hipMemcpyDeviceToDevice, f->stream));
      HIP_TRY(hipStreamSynchronize(f->stream));
      f->arena.swap(bigger);
    }
  }
  FreqDev d = dev_view(f);
  for (int k = 0; k < f->n_keys; ++k) d.cols[k].type = f->types[k];
  const PartArgs a = part_args(f, n_src);
  const auto* rec = reinterpret_cast<const FreqRecord*>(records);
  if (total_rec) {
    unsigned grid = grid_for((uint64_t)total_rec);
    hipLaunchKernelGGL(freq_insert_records_kernel, dim3(grid), dim3(256), 0, f->stream, d, rec, var,
                       segs, a);
    HIP_TRY(hipGetLastError());
    if (!f->exact) {
      hipLaunchKernelGGL(freq_verify_records_kernel, dim3(grid), dim3(256), 0, f->stream, d, rec,
                         var, segs, a);
      HIP_TRY(hipGetLastError());
    }
  }
  st = pull_counters(f);
  if (st != DQ_OK) return st;
  unsigned long long c[C_N];
  for (int k = 0; k < C_N; ++k) c[k] = f->h_counters[k];
  c[C_SENTINEL] += (unsigned long long)special[0];
  c[C_NULL_GROUP] += (unsigned long long)special[1];
  c[C_NULL_ROWS] += (unsigned long long)special[2];
  HIP_TRY(hipMemcpy(f->counters.p, c, sizeof(c), hipMemcpyHostToDevice));
  f->num_rows += num_rows;
  st = pull_counters(f);
  if (st != DQ_OK) return st;
  if (f->h_counters[C_ARENA_OVF]) return fail(DQ_ERR_OUT_OF_MEMORY, "frequency table arena overflow");
  if (f->h_counters[C_COLLISIONS])
    return fail(DQ_ERR_UNSUPPORTED,
                "64-bit key-hash collision between distinct groups detected (%llu groups)",
                (unsigned long long)f->h_counters[C_COLLISIONS]);
  return DQ_OK;
}
