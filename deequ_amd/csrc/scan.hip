// scan.hip -- the fused scan: one launch evaluates every ScanShareableAnalyzer aggregation of a
// suite over one column batch (the reference's single `data.agg(...)` Spark job,
// AnalysisRunner.scala:296-303), plus the tiny finalize launch that merges workgroup partials in a
// fixed order and folds them into the running state (Spark's final-mode merge).
//
// Work decomposition: every task (one per (column, where) group, see api.cpp) is cut into work
// items of ~128 KiB of buffers; items of all tasks are concatenated and block b owns the
// contiguous item range [b*T/G, (b+1)*T/G).  A block keeps per-lane accumulators in registers
// while it stays on one task and reduces them (wave shuffles -> LDS) once per task it touches.
//
// Memory access: see lane_row0 -- every wave-level load of the values is one contiguous 1 KiB
// (int64/double, 16 B per lane) segment and the 8 loads of a lane are in flight before the first
// is consumed.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "kernels.h"

namespace dq {

#define DQ_DEV __device__ __forceinline__

// ------------------------------------------------------------------------------------------------
// Bit and value loads
// ------------------------------------------------------------------------------------------------
DQ_DEV uint32_t bit1(const uint8_t* bm, int64_t r) {
  return bm ? ((bm[r >> 3] >> (r & 7)) & 1u) : 1u;
}
// two bits (rows r, r+1; r even) from a 4-byte aligned bitmap
DQ_DEV uint32_t bits2_vec(const uint8_t* bm, int64_t r) {
  if (!bm) return 3u;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(bm);
  return (w[r >> 5] >> (r & 31)) & 3u;
}

// Row mapping of a 4096-row block iteration: wave w owns the contiguous 1024 rows
// [r0 + 1024w, r0 + 1024(w+1)); in step k (k < 8) lane l owns rows r0 + 1024w + 128k + 2l + {0,1}.
// Each wave-level load is one contiguous 1 KiB (8-byte values) and the 8 steps of a wave sit
// within 8 KiB of one base address, so the loads need only immediate offsets.
constexpr int64_t kStep = 128;
DQ_DEV int64_t lane_row0(int64_t r0) {
  return r0 + (int64_t)(threadIdx.x >> 6) * (kStep * kUnroll) + 2 * (threadIdx.x & 63);
}

template <typename T>
struct alignas(2 * sizeof(T)) Pair {
  T a, b;
};

template <typename T>
DQ_DEV double to_f64(T v) {
  return (double)v;
}

// Three-way compare in Spark's order: doubles NaN-safe (NaN == NaN, NaN largest, -0.0 == 0.0).
DQ_DEV int cmp3_f64(double a, double b) {
  bool an = a != a, bn = b != b;
  if ((an && bn) || a == b) return 0;
  if (an) return 1;
  if (bn) return -1;
  return a > b ? 1 : -1;
}
DQ_DEV int cmp3_i64(int64_t a, int64_t b) { return a == b ? 0 : (a > b ? 1 : -1); }

// truth table of a comparison op over the three-way result c in {-1,0,1}: bit (c+1)
DQ_HD uint32_t op_mask(int op) {
  switch (op) {
    case DQ_X_EQ: return 0b010;
    case DQ_X_NE: return 0b101;
    case DQ_X_LT: return 0b001;
    case DQ_X_LE: return 0b011;
    case DQ_X_GT: return 0b100;
    case DQ_X_GE: return 0b110;
    default: return 0b111;
  }
}

// Byte reader over a device utf8 buffer using only aligned dword loads that contain at least one
// byte of the string (never faults past the end of the allocation).
struct DevBytes {
  const uint8_t* p;
  DQ_DEV uint32_t u32(int64_t o) const {
    uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    uint32_t sh = (uint32_t)(a & 3) * 8;
    uint32_t w0 = w[0];
    if (sh == 0) return w0;
    uint32_t w1 = w[1];
    return (w0 >> sh) | (w1 << (32 - sh));
  }
  DQ_DEV uint64_t u64(int64_t o) const { return (uint64_t)u32(o) | ((uint64_t)u32(o + 4) << 32); }
  DQ_DEV uint32_t u8(int64_t o) const {
    uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    return (w[0] >> ((a & 3) * 8)) & 0xffu;
  }
  // first min(len, 8) bytes, little-endian, zero padded
  DQ_DEV uint64_t prefix8(int64_t len) const {
    if (len <= 0) return 0;
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    uint32_t sh = (uint32_t)(a & 3) * 8;
    int64_t take = len < 8 ? len : 8;
    int64_t last = (int64_t)((a & 3) + take - 1) >> 2;  // index of last dword needed
    uint64_t w0 = w[0];
    uint64_t w1 = last >= 1 ? (uint64_t)w[1] : 0;
    uint64_t w2 = last >= 2 ? (uint64_t)w[2] : 0;
    uint64_t lo = w0 | (w1 << 32);
    uint64_t v = sh ? ((lo >> sh) | (w2 << (64 - sh))) : lo;
    if (take < 8) v &= (1ULL << (take * 8)) - 1;
    return v;
  }
};

// Loads one value of a runtime-typed numeric column as double / as int64.
DQ_DEV double load_f64(int type, const void* v, int64_t r) {
  switch (type) {
    case DQ_INT8: return (double)reinterpret_cast<const int8_t*>(v)[r];
    case DQ_INT16: return (double)reinterpret_cast<const int16_t*>(v)[r];
    case DQ_INT32: return (double)reinterpret_cast<const int32_t*>(v)[r];
    case DQ_INT64: return (double)reinterpret_cast<const int64_t*>(v)[r];
    case DQ_FLOAT32: return (double)reinterpret_cast<const float*>(v)[r];
    case DQ_FLOAT64: return reinterpret_cast<const double*>(v)[r];
    case DQ_BOOL: return (double)bit1(reinterpret_cast<const uint8_t*>(v), r);
    default: return 0.0;
  }
}
DQ_DEV int64_t load_i64(int type, const void* v, int64_t r) {
  switch (type) {
    case DQ_INT8: return reinterpret_cast<const int8_t*>(v)[r];
    case DQ_INT16: return reinterpret_cast<const int16_t*>(v)[r];
    case DQ_INT32: return reinterpret_cast<const int32_t*>(v)[r];
    case DQ_INT64: return reinterpret_cast<const int64_t*>(v)[r];
    case DQ_BOOL: return bit1(reinterpret_cast<const uint8_t*>(v), r);
    default: return 0;
  }
}
DQ_HD bool is_float_type(int type) { return type == DQ_FLOAT32 || type == DQ_FLOAT64; }

// Spark XxHash64Function.hash(value, type, 42) for one non-null row.
DQ_DEV uint64_t hash_row(int type, const void* values, const uint8_t* data, int64_t r) {
  const uint64_t seed = 42;
  switch (type) {
    case DQ_INT8: return xxh_int((uint32_t)(int32_t)reinterpret_cast<const int8_t*>(values)[r], seed);
    case DQ_INT16:
      return xxh_int((uint32_t)(int32_t)reinterpret_cast<const int16_t*>(values)[r], seed);
    case DQ_INT32: return xxh_int((uint32_t)reinterpret_cast<const int32_t*>(values)[r], seed);
    case DQ_INT64: return xxh_long((uint64_t)reinterpret_cast<const int64_t*>(values)[r], seed);
    case DQ_BOOL: return xxh_int(bit1(reinterpret_cast<const uint8_t*>(values), r), seed);
    case DQ_FLOAT32: {
      float f = reinterpret_cast<const float*>(values)[r];
      uint32_t b = (f != f) ? 0x7fc00000u : __builtin_bit_cast(uint32_t, f);  // floatToIntBits
      return xxh_int(b, seed);
    }
    case DQ_FLOAT64: {
      double d = reinterpret_cast<const double*>(values)[r];
      uint64_t b = (d != d) ? 0x7ff8000000000000ULL : __builtin_bit_cast(uint64_t, d);
      return xxh_long(b, seed);
    }
    case DQ_UTF8: {
      const int32_t* off = reinterpret_cast<const int32_t*>(values);
      int32_t s = off[r], e = off[r + 1];
      DevBytes rd{data + s};
      return xxh_bytes(rd, (int64_t)(e - s), seed);
    }
    default: return 0;
  }
}

// ------------------------------------------------------------------------------------------------
// Reductions
// ------------------------------------------------------------------------------------------------
DQ_DEV void wave_reduce(int kind, Acc& a) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    Acc o;
#pragma unroll
    for (int f = 0; f < 10; ++f) o.i[f] = __shfl_xor(a.i[f], off);
#pragma unroll
    for (int f = 0; f < 6; ++f) o.d[f] = __shfl_xor(a.d[f], off);
    acc_merge(kind, a, o);
  }
}

// Reduces the block's lane accumulators and stores the block partial (fixed merge order).
DQ_DEV void block_store(int kind, Acc& a, Acc* out, Acc* sh) {
  wave_reduce(kind, a);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) sh[wave] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc r = sh[0];
    for (int w = 1; w < kBlock / 64; ++w) acc_merge(kind, r, sh[w]);
    *out = r;
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// TK_NUMERIC
// ------------------------------------------------------------------------------------------------
struct NumLane {
  int64_t n = 0, si = 0, kmin = INT64_MAX, kmax = INT64_MIN;
  double sd = 0.0, mean = 0.0, m2 = 0.0;
  int64_t pt[kMaxPreds] = {0, 0, 0}, pn[kMaxPreds] = {0, 0, 0};
};

template <typename T>
DQ_DEV int64_t num_key(T v) {
  if constexpr (std::is_floating_point<T>::value) {
    return f64_key((double)v);
  } else {
    return (int64_t)v;
  }
}

// Truth bits of a fused predicate over the lane's 16 values (NULL handling is done by the caller).
template <typename T>
DQ_DEV uint32_t pred_bits(const NumPred& P, const T (&x)[16]) {
  const uint32_t m1 = op_mask(P.op1), m2 = op_mask(P.op2);
  uint32_t r = 0;
  if (P.as_double) {
    const double lo = P.lo_d, hi = P.hi_d;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const double xd = (double)x[i];
      uint32_t ok = (m1 >> (cmp3_f64(xd, lo) + 1)) & 1u;
      if (P.op2) ok &= (m2 >> (cmp3_f64(xd, hi) + 1)) & 1u;
      r |= ok << i;
    }
  } else {
    const int64_t lo = P.lo_i, hi = P.hi_i;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t xi = (int64_t)x[i];
      uint32_t ok = (m1 >> (cmp3_i64(xi, lo) + 1)) & 1u;
      if (P.op2) ok &= (m2 >> (cmp3_i64(xi, hi) + 1)) & 1u;
      r |= ok << i;
    }
  }
  return r;
}

// Processes the lane's 16 rows of one block iteration.  vb = validity bits, wt = where-TRUE bits
// (bit i <-> value x[i]); rows past the end have vb = wt = 0.
template <typename T>
DQ_DEV void num_rows(NumLane& L, const T (&x)[16], uint32_t vb, uint32_t wt, const TaskDesc& t) {
  const uint32_t sel = vb & wt;
  const int nb = __popc(sel);
  if (nb) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if ((sel >> i) & 1u) {
        if constexpr (!std::is_floating_point<T>::value) L.si = wrap_add(L.si, (int64_t)x[i]);
        s += (double)x[i];
        int64_t k = num_key(x[i]);
        L.kmin = k < L.kmin ? k : L.kmin;
        L.kmax = k > L.kmax ? k : L.kmax;
      }
    }
    L.sd += s;
    // two-pass moments of this 16-row batch in registers, then a Chan merge (one division each)
    const double mb = s / (double)nb;
    double m2b = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      double d = (double)x[i] - mb;
      m2b += ((sel >> i) & 1u) ? d * d : 0.0;
    }
    if (L.n == 0) {
      L.mean = mb;
      L.m2 = m2b;
    } else {
      moments_merge((double)L.n, L.mean, L.m2, (double)nb, mb, m2b);
    }
    L.n += nb;
  }
  if (t.n_preds == 0) return;
  const uint32_t nulls_all = wt & ~vb & 0xffffu;
#pragma unroll
  for (int p = 0; p < kMaxPreds; ++p) {
    if (p >= t.n_preds) break;
    const NumPred& P = t.preds[p];
    const uint32_t r = pred_bits<T>(P, x);
    const uint32_t nulls = P.null_is_true ? nulls_all : 0u;
    L.pt[p] += __popc(r & sel) + __popc(nulls);
    L.pn[p] += __popc(sel) + __popc(nulls);
  }
}

template <typename T, bool FAST>
DQ_DEV void num_iter(NumLane& L, const TaskDesc& t, int64_t r0, int64_t r_end) {
  const T* v = reinterpret_cast<const T*>(t.values);
  T x[16];
  uint32_t vb = 0, wt = 0;
  const int64_t rb = lane_row0(r0);
  if constexpr (FAST) {
    Pair<T> p[kUnroll];
    uint32_t vv[kUnroll], ww[kUnroll], wv[kUnroll];
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      p[k] = *reinterpret_cast<const Pair<T>*>(v + rb + kStep * k);
      vv[k] = bits2_vec(t.valid, rb + kStep * k);
      ww[k] = t.w_val ? bits2_vec(t.w_val, rb + kStep * k) : 3u;
      wv[k] = bits2_vec(t.w_vld, rb + kStep * k);
    }
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      x[2 * k] = p[k].a;
      x[2 * k + 1] = p[k].b;
      vb |= vv[k] << (2 * k);
      wt |= (ww[k] & wv[k]) << (2 * k);
    }
  } else {
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t r = rb + kStep * k + j;
        const int i = 2 * k + j;
        if (r < r_end) {
          x[i] = v[r];
          vb |= bit1(t.valid, r) << i;
          uint32_t w = t.w_val ? (bit1(t.w_val, r) & bit1(t.w_vld, r)) : 1u;
          wt |= w << i;
        } else {
          x[i] = T(0);
        }
      }
    }
  }
  num_rows<T>(L, x, vb, wt, t);
}

template <typename T>
DQ_DEV void run_numeric(const TaskDesc& t, int64_t lo, int64_t hi, Acc* out, Acc* sh) {
  NumLane L;
  const int64_t r_begin = lo * t.item_rows;
  const int64_t r_end = min(hi * t.item_rows, t.rows);
  int64_t r = r_begin;
  if (t.vec_ok) {
    for (; r + kRowsPerIter <= r_end; r += kRowsPerIter) num_iter<T, true>(L, t, r, r_end);
  }
  for (; r < r_end; r += kRowsPerIter) num_iter<T, false>(L, t, r, r_end);
  Acc a;
  acc_init(TK_NUMERIC, a);
  a.i[0] = L.n;
  a.i[1] = L.si;
  a.i[2] = L.kmin;
  a.i[3] = L.kmax;
  for (int p = 0; p < kMaxPreds; ++p) {
    a.i[4 + p] = L.pt[p];
    a.i[7 + p] = L.pn[p];
  }
  a.d[0] = L.sd;
  a.d[1] = L.mean;
  a.d[2] = L.m2;
  block_store(TK_NUMERIC, a, out, sh);
}

// ------------------------------------------------------------------------------------------------
// TK_VALIDITY / TK_BOOLMAP: popcounts over bitmaps.  count0 = |A & B & W|, count1 = |B & W|
// where A = value bits (validity of a column, or an expression's value bits), B = validity bits of
// the expression (absent for TK_VALIDITY), W = where-TRUE bits.  Absent bitmaps are all ones.
// ------------------------------------------------------------------------------------------------
DQ_DEV uint32_t ld32(const uint8_t* bm, int64_t word) {
  return bm ? reinterpret_cast<const uint32_t*>(bm)[word] : 0xffffffffu;
}
DQ_DEV uint32_t ld32_slow(const uint8_t* bm, int64_t word, int64_t rows) {
  if (!bm) return 0xffffffffu;
  uint32_t v = 0;
  for (int b = 0; b < 4; ++b) {
    int64_t byte = word * 4 + b;
    if (byte * 8 < rows) v |= (uint32_t)bm[byte] << (8 * b);
  }
  return v;
}

DQ_DEV void run_bits(const TaskDesc& t, int64_t lo, int64_t hi, Acc* out, Acc* sh) {
  const uint8_t* A = t.kind == TK_VALIDITY ? t.valid : t.b_val;
  const uint8_t* B = t.kind == TK_VALIDITY ? nullptr : t.b_vld;
  const uint8_t* WV = t.w_val;
  const uint8_t* WD = t.w_val ? t.w_vld : nullptr;
  const int64_t r_begin = lo * t.item_rows;
  const int64_t r_end = min(hi * t.item_rows, t.rows);
  // rows [r_begin, r_end) -> 32-bit words; r_begin is a multiple of 32
  const int64_t w_begin = r_begin >> 5;
  const int64_t w_full = r_end >> 5;          // words entirely inside
  const int64_t w_end = (r_end + 31) >> 5;
  int64_t c0 = 0, c1 = 0;
  int64_t w_slow = w_begin;  // first word left for the scalar loop
  if (t.vec_ok) {
    // 16-byte groups of 4 words; w_begin is a multiple of 128 words (item rows % 4096 == 0)
    const int64_t n_groups = (w_full - w_begin) >> 2;
    const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
    for (int64_t g = threadIdx.x; g < n_groups; g += kBlock) {
      const int64_t byte = 4 * (w_begin + 4 * g);
      uint4 a = A ? *reinterpret_cast<const uint4*>(A + byte) : ones;
      uint4 b = B ? *reinterpret_cast<const uint4*>(B + byte) : ones;
      uint4 x = WV ? *reinterpret_cast<const uint4*>(WV + byte) : ones;
      uint4 y = WD ? *reinterpret_cast<const uint4*>(WD + byte) : ones;
      uint32_t m0 = b.x & x.x & y.x, m1 = b.y & x.y & y.y, m2 = b.z & x.z & y.z, m3 = b.w & x.w & y.w;
      c0 += __popc(a.x & m0) + __popc(a.y & m1) + __popc(a.z & m2) + __popc(a.w & m3);
      c1 += __popc(m0) + __popc(m1) + __popc(m2) + __popc(m3);
    }
    w_slow = w_begin + 4 * n_groups;
  }
  {
    for (int64_t w = w_slow + threadIdx.x; w < w_end; w += kBlock) {
      uint32_t mask = 0xffffffffu;
      if (w == w_end - 1 && (r_end & 31)) mask = (1u << (r_end & 31)) - 1u;
      uint32_t a = ld32_slow(A, w, t.rows), b = ld32_slow(B, w, t.rows);
      uint32_t x = ld32_slow(WV, w, t.rows), y = ld32_slow(WD, w, t.rows);
      uint32_t m = b & x & y & mask;
      c0 += __popc(a & m);
      c1 += __popc(m);
    }
  }
  Acc acc;
  acc_init(t.kind, acc);
  acc.i[0] = c0;
  acc.i[1] = c1;
  block_store(t.kind, acc, out, sh);
}

// ------------------------------------------------------------------------------------------------
// TK_STR_IN:  when(where, [c IS NULL OR] c [NOT] IN (list))  -> TRUE count, non-NULL count
// ------------------------------------------------------------------------------------------------
DQ_DEV uint32_t str_match(const TaskDesc& t, const uint8_t* s, int32_t len) {
  DevBytes rd{s};
  const uint64_t pre = rd.prefix8(len);
  for (int j = 0; j < t.n_list; ++j) {
    const int32_t ls = t.list_off[j], le = t.list_off[j + 1];
    if (le - ls != len) continue;
    if (t.list_pre[j] != pre) continue;
    bool eq = true;
    for (int32_t k = 8; k < len; ++k) {
      if (rd.u8(k) != t.list_bytes[ls + k]) {
        eq = false;
        break;
      }
    }
    if (eq) return 1u;
  }
  return 0u;
}

DQ_DEV void run_str_in(const TaskDesc& t, int64_t lo, int64_t hi, Acc* out, Acc* sh) {
  const int64_t r_begin = lo * t.item_rows;
  const int64_t r_end = min(hi * t.item_rows, t.rows);
  const int32_t* off = reinterpret_cast<const int32_t*>(t.values);
  int64_t ct = 0, cn = 0;
  for (int64_t r0 = r_begin; r0 < r_end; r0 += kRowsPerIter) {
    const int64_t rb = lane_row0(r0);
    const bool fast = t.vec_ok && (r0 + kRowsPerIter <= r_end);
    int2 o01[kUnroll];
    int32_t o2[kUnroll];
    uint32_t vv[kUnroll], ww[kUnroll];
    if (fast) {
#pragma unroll
      for (int k = 0; k < kUnroll; ++k) {
        const int64_t r = rb + kStep * k;
        o01[k] = *reinterpret_cast<const int2*>(off + r);
        o2[k] = off[r + 2];
        vv[k] = bits2_vec(t.valid, r);
        ww[k] = t.w_val ? (bits2_vec(t.w_val, r) & bits2_vec(t.w_vld, r)) : 3u;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kUnroll; ++k) {
        const int64_t r = rb + kStep * k;
        vv[k] = 0;
        ww[k] = 0;
        o01[k] = make_int2(0, 0);
        o2[k] = 0;
        if (r < r_end) {
          o01[k].x = off[r];
          o01[k].y = off[r + 1];
          vv[k] |= bit1(t.valid, r);
          ww[k] |= t.w_val ? (bit1(t.w_val, r) & bit1(t.w_vld, r)) : 1u;
        }
        if (r + 1 < r_end) {
          o2[k] = off[r + 2];
          vv[k] |= bit1(t.valid, r + 1) << 1;
          ww[k] |= (t.w_val ? (bit1(t.w_val, r + 1) & bit1(t.w_vld, r + 1)) : 1u) << 1;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (!((ww[k] >> j) & 1u)) continue;
        if ((vv[k] >> j) & 1u) {
          const int32_t s = j ? o01[k].y : o01[k].x;
          const int32_t e = j ? o2[k] : o01[k].y;
          ct += str_match(t, t.data + s, e - s) ^ (uint32_t)t.negate;
          cn += 1;
        } else if (t.null_is_true) {
          ct += 1;
          cn += 1;
        }
      }
    }
  }
  Acc a;
  acc_init(TK_STR_IN, a);
  a.i[0] = ct;
  a.i[1] = cn;
  block_store(TK_STR_IN, a, out, sh);
}

// ------------------------------------------------------------------------------------------------
// TK_COMOMENTS (Correlation): rows where x and y are both non-NULL (and where is TRUE).
// ------------------------------------------------------------------------------------------------
DQ_DEV void run_comoments(const TaskDesc& t, int64_t lo, int64_t hi, Acc* out, Acc* sh) {
  const int64_t r_begin = lo * t.item_rows;
  const int64_t r_end = min(hi * t.item_rows, t.rows);
  int64_t n = 0;
  double c[5] = {0, 0, 0, 0, 0};  // xAvg, yAvg, ck, xMk, yMk
  for (int64_t r0 = r_begin; r0 < r_end; r0 += kRowsPerIter) {
    const int64_t rb = lane_row0(r0);
    double xs[16], ys[16];
    uint32_t sel = 0;
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t r = rb + kStep * k + j;
        const int i = 2 * k + j;
        xs[i] = 0.0;
        ys[i] = 0.0;
        if (r < r_end) {
          uint32_t s = bit1(t.valid, r) & bit1(t.valid2, r);
          if (t.w_val) s &= bit1(t.w_val, r) & bit1(t.w_vld, r);
          if (s) {
            xs[i] = load_f64(t.type, t.values, r);
            ys[i] = load_f64(t.type2, t.values2, r);
          }
          sel |= s << i;
        }
      }
    }
    const int nb = __popc(sel);
    if (!nb) continue;
    double sx = 0, sy = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      sx += xs[i];
      sy += ys[i];
    }
    double b[5];
    b[0] = sx / nb;
    b[1] = sy / nb;
    b[2] = b[3] = b[4] = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if ((sel >> i) & 1u) {
        double dx = xs[i] - b[0], dy = ys[i] - b[1];
        b[2] += dx * dy;
        b[3] += dx * dx;
        b[4] += dy * dy;
      }
    }
    if (n == 0) {
      for (int f = 0; f < 5; ++f) c[f] = b[f];
    } else {
      comoments_merge((double)n, c, (double)nb, b);
    }
    n += nb;
  }
  Acc a;
  acc_init(TK_COMOMENTS, a);
  a.i[0] = n;
  for (int f = 0; f < 5; ++f) a.d[f] = c[f];
  block_store(TK_COMOMENTS, a, out, sh);
}

// ------------------------------------------------------------------------------------------------
// TK_HLL: 512 registers in LDS, atomicMax only when the rank can raise the register.
// ------------------------------------------------------------------------------------------------
DQ_DEV void run_hll(const TaskDesc& t, int64_t lo, int64_t hi, uint8_t* out_regs, uint32_t* regs) {
  for (int i = threadIdx.x; i < kHllM; i += kBlock) regs[i] = 0;
  __syncthreads();
  const int64_t r_begin = lo * t.item_rows;
  const int64_t r_end = min(hi * t.item_rows, t.rows);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += kRowsPerIter) {
    const int64_t rb = lane_row0(r0);
#pragma unroll 2
    for (int k = 0; k < kUnroll; ++k) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t r = rb + kStep * k + j;
        if (r >= r_end) continue;
        uint32_t s = bit1(t.valid, r);
        if (t.w_val) s &= bit1(t.w_val, r) & bit1(t.w_vld, r);
        if (!s) continue;
        uint64_t x = hash_row(t.type, t.values, t.data, r);
        uint32_t idx, pw;
        hll_index_rank(x, idx, pw);
        if (pw > regs[idx]) atomicMax(&regs[idx], pw);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHllM; i += kBlock) out_regs[i] = (uint8_t)regs[i];
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// The fused scan kernel
// ------------------------------------------------------------------------------------------------
// FULL = false is the streaming family (numeric int32/int64/float/double, bitmap counts, string
// IN-lists): the S10 suite.  Compiling it without the hashing / co-moment bodies keeps its register
// allocation (and so its occupancy) at what those bodies need.
template <bool FULL>
__global__ void __launch_bounds__(kBlock) scan_kernel(const TaskDesc* __restrict__ tasks, int n_tasks,
                                                      int64_t total_items, Acc* __restrict__ partial,
                                                      uint8_t* __restrict__ hll_partial) {
  __shared__ Acc sh[kBlock / 64];
  __shared__ uint32_t regs[FULL ? kHllM : 1];
  const int64_t G = gridDim.x;
  const int64_t ib = (int64_t)blockIdx.x * total_items / G;
  const int64_t ie = ((int64_t)blockIdx.x + 1) * total_items / G;
  for (int ti = 0; ti < n_tasks; ++ti) {
    const TaskDesc& t = tasks[ti];
    const int64_t tb = t.item_begin, te = t.item_begin + t.n_items;
    if (te <= ib || tb >= ie) continue;
    const int64_t lo = max(ib, tb) - tb, hi = min(ie, te) - tb;
    Acc* out = partial + (int64_t)ti * G + blockIdx.x;
    switch (t.kind) {
      case TK_NUMERIC:
        switch (t.type) {
          case DQ_INT32: run_numeric<int32_t>(t, lo, hi, out, sh); break;
          case DQ_INT64: run_numeric<int64_t>(t, lo, hi, out, sh); break;
          case DQ_FLOAT32: run_numeric<float>(t, lo, hi, out, sh); break;
          case DQ_FLOAT64: run_numeric<double>(t, lo, hi, out, sh); break;
          case DQ_INT8:
            if constexpr (FULL) run_numeric<int8_t>(t, lo, hi, out, sh);
            break;
          case DQ_INT16:
            if constexpr (FULL) run_numeric<int16_t>(t, lo, hi, out, sh);
            break;
          default: break;
        }
        break;
      case TK_VALIDITY:
      case TK_BOOLMAP: run_bits(t, lo, hi, out, sh); break;
      case TK_STR_IN: run_str_in(t, lo, hi, out, sh); break;
      case TK_COMOMENTS:
        if constexpr (FULL) run_comoments(t, lo, hi, out, sh);
        break;
      case TK_HLL:
        if constexpr (FULL)
          run_hll(t, lo, hi, hll_partial + ((int64_t)t.hll_slot * G + blockIdx.x) * kHllM, regs);
        break;
      default: break;
    }
  }
}

// Merges, in a fixed order, the partials of every (descriptor, block) pair that belongs to logical
// task blockIdx.x -- all batches of one task -- into the running accumulator.  One workgroup per
// logical task; the per-thread order is (block, descriptor) ascending, then a fixed tree.
__global__ void __launch_bounds__(kBlock) finalize_kernel(const TaskDesc* __restrict__ tasks,
                                                          int n_desc, int64_t total_items, int G,
                                                          const Acc* __restrict__ partial,
                                                          const uint8_t* __restrict__ hll_partial,
                                                          Acc* __restrict__ acc,
                                                          uint8_t* __restrict__ hll_acc) {
  __shared__ Acc sh[kBlock];
  const int task = blockIdx.x;
  int kind = 0, hll_out = -1;
  for (int d = 0; d < n_desc; ++d)
    if (tasks[d].out == task) {
      kind = tasks[d].kind;
      hll_out = tasks[d].hll_out;
      break;
    }
  if (kind == 0) return;
  if (kind == TK_HLL) {
    for (int reg = threadIdx.x; reg < kHllM; reg += kBlock) {
      uint32_t m = hll_acc[(int64_t)hll_out * kHllM + reg];
      for (int d = 0; d < n_desc; ++d) {
        const TaskDesc& t = tasks[d];
        if (t.out != task) continue;
        const int64_t tb = t.item_begin, te = t.item_begin + t.n_items;
        for (int b = 0; b < G; ++b) {
          const int64_t ib = (int64_t)b * total_items / G, ie = ((int64_t)b + 1) * total_items / G;
          if (te <= ib || tb >= ie) continue;
          uint32_t v = hll_partial[((int64_t)t.hll_slot * G + b) * kHllM + reg];
          m = v > m ? v : m;
        }
      }
      hll_acc[(int64_t)hll_out * kHllM + reg] = (uint8_t)m;
    }
    return;
  }
  Acc a;
  acc_init(kind, a);
  for (int b = threadIdx.x; b < G; b += kBlock) {
    const int64_t ib = (int64_t)b * total_items / G, ie = ((int64_t)b + 1) * total_items / G;
    for (int d = 0; d < n_desc; ++d) {
      const TaskDesc& t = tasks[d];
      if (t.out != task) continue;
      const int64_t tb = t.item_begin, te = t.item_begin + t.n_items;
      if (te <= ib || tb >= ie) continue;
      acc_merge(kind, a, partial[(int64_t)d * G + b]);
    }
  }
  sh[threadIdx.x] = a;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) acc_merge(kind, sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    Acc r = acc[task];
    acc_merge(kind, r, sh[0]);
    acc[task] = r;
  }
}

// ------------------------------------------------------------------------------------------------
// Generic predicate evaluation (the slow path for expressions that the planner cannot fuse):
// a postfix program over typed values with Kleene logic; one lane per row, results ballot-packed
// into Arrow boolean bitmaps (value bits, validity bits).
// ------------------------------------------------------------------------------------------------
struct V {
  int32_t tag;  // 0 NULL, 1 BOOL, 2 I64, 3 F64, 4 STR
  int32_t len;
  int64_t i;
  double d;
  const uint8_t* p;
};

DQ_DEV int cmp_str(const uint8_t* a, int32_t la, const uint8_t* b, int32_t lb) {
  DevBytes ra{a}, rb{b};
  int32_t n = la < lb ? la : lb;
  for (int32_t k = 0; k < n; ++k) {
    int32_t d = (int32_t)ra.u8(k) - (int32_t)rb.u8(k);
    if (d) return d < 0 ? -1 : 1;
  }
  return la == lb ? 0 : (la < lb ? -1 : 1);
}

// three-way compare of two non-NULL values; returns 2 when incomparable
DQ_DEV int cmp_vals(const V& a, const V& b) {
  if (a.tag == 4 && b.tag == 4) return cmp_str(a.p, a.len, b.p, b.len);
  if (a.tag == 4 || b.tag == 4) return 2;
  if (a.tag == 3 || b.tag == 3) {
    double x = a.tag == 3 ? a.d : (double)a.i, y = b.tag == 3 ? b.d : (double)b.i;
    return cmp3_f64(x, y);
  }
  return cmp3_i64(a.i, b.i);
}

// Java Double.parseDouble subset (what Spark 2.2's Cast(StringType -> DoubleType) calls): trims
// ASCII whitespace/control chars, sign, digits, '.', exponent, optional [dDfF] suffix, NaN,
// Infinity.  Correctly rounded when the decimal significand < 2^53 and |exp10| <= 22; otherwise the
// nearest of two roundings (documented).  Returns false when the string is not a number -> NULL.
DQ_DEV bool parse_f64(const uint8_t* s, int32_t len, double& out) {
  DevBytes rd{s};
  int32_t b = 0, e = len;
  while (b < e && rd.u8(b) <= 32) ++b;
  while (e > b && rd.u8(e - 1) <= 32) --e;
  if (b >= e) return false;
  bool neg = false;
  uint32_t c = rd.u8(b);
  if (c == '+' || c == '-') {
    neg = c == '-';
    ++b;
  }
  if (e - b == 3 && rd.u8(b) == 'N' && rd.u8(b + 1) == 'a' && rd.u8(b + 2) == 'N') {
    out = __builtin_nan("");
    return true;
  }
  if (e - b == 8) {
    const char* inf = "Infinity";
    bool ok = true;
    for (int k = 0; k < 8; ++k) ok &= rd.u8(b + k) == (uint32_t)inf[k];
    if (ok) {
      out = neg ? -__builtin_inf() : __builtin_inf();
      return true;
    }
  }
  if (e > b) {
    uint32_t last = rd.u8(e - 1);
    if (last == 'd' || last == 'D' || last == 'f' || last == 'F') --e;
  }
  uint64_t mant = 0;
  int digits = 0, exp10 = 0;
  bool any = false, dot = false, overflow_digits = false;
  int32_t k = b;
  for (; k < e; ++k) {
    c = rd.u8(k);
    if (c >= '0' && c <= '9') {
      any = true;
      if (mant < 100000000000000000ULL) {
        mant = mant * 10 + (c - '0');
        if (mant) ++digits;
        if (dot) --exp10;
      } else {
        overflow_digits = true;
        if (!dot) ++exp10;
      }
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (!any) return false;
  if (k < e) {
    c = rd.u8(k);
    if (c != 'e' && c != 'E') return false;
    ++k;
    bool eneg = false;
    if (k < e && (rd.u8(k) == '+' || rd.u8(k) == '-')) {
      eneg = rd.u8(k) == '-';
      ++k;
    }
    if (k >= e) return false;
    int ev = 0;
    for (; k < e; ++k) {
      c = rd.u8(k);
      if (c < '0' || c > '9') return false;
      if (ev < 100000) ev = ev * 10 + (c - '0');
    }
    exp10 += eneg ? -ev : ev;
  }
  (void)overflow_digits;
  (void)digits;
  double v = (double)mant;
  const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                          1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  if (exp10 >= 0) {
    while (exp10 > 22) {
      v *= 1e22;
      exp10 -= 22;
    }
    v *= p10[exp10];
  } else {
    while (exp10 < -22) {
      v /= 1e22;
      exp10 += 22;
    }
    v /= p10[-exp10];
  }
  out = neg ? -v : v;
  return true;
}

__global__ void __launch_bounds__(kBlock) expr_kernel(const XInstr* __restrict__ prog, int n_instr,
                                                      const DevCol* __restrict__ cols,
                                                      const uint8_t* __restrict__ pool, int64_t rows,
                                                      uint64_t* __restrict__ out_val,
                                                      uint64_t* __restrict__ out_vld) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
  const int64_t n_words = (rows + 63) >> 6;
  for (int64_t w = wave; w < n_words; w += n_waves) {
    const int64_t r = w * 64 + lane;
    V st[kMaxStack];
    int sp = 0;
    bool in_range = r < rows;
    if (in_range) {
      for (int pc = 0; pc < n_instr; ++pc) {
        const XInstr ins = prog[pc];
        switch (ins.op) {
          case XI_COL: {
            const DevCol& c = cols[ins.a];
            V v{};
            if (!bit1(c.valid, r)) {
              v.tag = 0;
            } else if (c.type == DQ_UTF8) {
              const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
              v.tag = 4;
              v.p = c.data + off[r];
              v.len = off[r + 1] - off[r];
            } else if (c.type == DQ_BOOL) {
              v.tag = 1;
              v.i = bit1(reinterpret_cast<const uint8_t*>(c.values), r);
            } else if (is_float_type(c.type)) {
              v.tag = 3;
              v.d = load_f64(c.type, c.values, r);
            } else {
              v.tag = 2;
              v.i = load_i64(c.type, c.values, r);
            }
            st[sp++] = v;
            break;
          }
          case XI_NULL: st[sp++] = V{0, 0, 0, 0.0, nullptr}; break;
          case XI_BOOL: st[sp++] = V{1, 0, ins.imm, 0.0, nullptr}; break;
          case XI_I64: st[sp++] = V{2, 0, ins.imm, 0.0, nullptr}; break;
          case XI_F64: st[sp++] = V{3, 0, 0, __builtin_bit_cast(double, ins.imm), nullptr}; break;
          case XI_STR: st[sp++] = V{4, ins.a, 0, 0.0, pool + ins.imm}; break;
          case XI_IS_NULL: st[sp - 1] = V{1, 0, st[sp - 1].tag == 0 ? 1 : 0, 0.0, nullptr}; break;
          case XI_IS_NOT_NULL: st[sp - 1] = V{1, 0, st[sp - 1].tag != 0 ? 1 : 0, 0.0, nullptr}; break;
          case XI_NOT:
            if (st[sp - 1].tag != 0) st[sp - 1].i = st[sp - 1].i ? 0 : 1;
            break;
          case XI_AND: {
            V b = st[--sp];
            V a = st[sp - 1];
            // Kleene: FALSE dominates, then NULL
            bool af = a.tag != 0 && !a.i, bf = b.tag != 0 && !b.i;
            if (af || bf) st[sp - 1] = V{1, 0, 0, 0.0, nullptr};
            else if (a.tag == 0 || b.tag == 0) st[sp - 1] = V{0, 0, 0, 0.0, nullptr};
            else st[sp - 1] = V{1, 0, 1, 0.0, nullptr};
            break;
          }
          case XI_OR: {
            V b = st[--sp];
            V a = st[sp - 1];
            bool at = a.tag != 0 && a.i, bt = b.tag != 0 && b.i;
            if (at || bt) st[sp - 1] = V{1, 0, 1, 0.0, nullptr};
            else if (a.tag == 0 || b.tag == 0) st[sp - 1] = V{0, 0, 0, 0.0, nullptr};
            else st[sp - 1] = V{1, 0, 0, 0.0, nullptr};
            break;
          }
          case XI_CMP: {
            V b = st[--sp];
            V a = st[sp - 1];
            if (ins.a == DQ_X_EQ_NULL_SAFE) {
              int eq;
              if (a.tag == 0 || b.tag == 0) eq = (a.tag == 0 && b.tag == 0);
              else eq = cmp_vals(a, b) == 0;
              st[sp - 1] = V{1, 0, eq, 0.0, nullptr};
            } else if (a.tag == 0 || b.tag == 0) {
              st[sp - 1] = V{0, 0, 0, 0.0, nullptr};
            } else {
              int c = cmp_vals(a, b);
              if (c == 2) st[sp - 1] = V{0, 0, 0, 0.0, nullptr};
              else st[sp - 1] = V{1, 0, (op_mask(ins.a) >> (c + 1)) & 1, 0.0, nullptr};
            }
            break;
          }
          case XI_IN: {
            const int n = ins.a;
            const int base = sp - n - 1;
            V x = st[base];
            V res{0, 0, 0, 0.0, nullptr};
            if (x.tag != 0) {
              bool found = false, saw_null = false;
              for (int q = 0; q < n; ++q) {
                const V& it = st[base + 1 + q];
                if (it.tag == 0) {
                  saw_null = true;
                } else if (cmp_vals(x, it) == 0) {
                  found = true;
                }
              }
              if (found) res = V{1, 0, 1, 0.0, nullptr};
              else if (!saw_null) res = V{1, 0, 0, 0.0, nullptr};
            }
            sp = base;
            st[sp++] = res;
            break;
          }
          case XI_CAST_F64: {
            V& a = st[sp - 1];
            if (a.tag == 2 || a.tag == 1) {
              a.d = (double)a.i;
              a.tag = 3;
            } else if (a.tag == 4) {
              double d;
              if (parse_f64(a.p, a.len, d)) a = V{3, 0, 0, d, nullptr};
              else a = V{0, 0, 0, 0.0, nullptr};
            }
            break;
          }
          default: break;
        }
      }
    }
    const V& res = st[0];
    const bool valid = in_range && sp == 1 && res.tag != 0;
    const bool truth = valid && res.i != 0;
    const uint64_t bv = __ballot(truth);
    const uint64_t bn = __ballot(valid);
    if (lane == 0) {
      out_val[w] = bv;
      out_vld[w] = bn;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Host-side launchers
// ------------------------------------------------------------------------------------------------
hipError_t launch_expr(const XInstr* prog, int n_instr, const DevCol* cols, const uint8_t* pool,
                       int64_t rows, uint64_t* out_val, uint64_t* out_vld, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  int64_t words = (rows + 63) / 64;
  int64_t blocks = (words + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(expr_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, prog, n_instr,
                     cols, pool, rows, out_val, out_vld);
  return hipGetLastError();
}

hipError_t launch_scan(const TaskDesc* tasks, int n_tasks, int n_logical, int64_t total_items,
                       int grid, bool full, Acc* partial, uint8_t* hll_partial, Acc* acc,
                       uint8_t* hll_acc, hipStream_t stream) {
  if (total_items <= 0 || n_tasks == 0) return hipSuccess;
  if (full)
    hipLaunchKernelGGL(scan_kernel<true>, dim3(grid), dim3(kBlock), 0, stream, tasks, n_tasks,
                       total_items, partial, hll_partial);
  else
    hipLaunchKernelGGL(scan_kernel<false>, dim3(grid), dim3(kBlock), 0, stream, tasks, n_tasks,
                       total_items, partial, hll_partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(finalize_kernel, dim3(n_logical), dim3(kBlock), 0, stream, tasks, n_tasks,
                     total_items, grid, partial, hll_partial, acc, hll_acc);
  return hipGetLastError();
}

int scan_max_blocks_per_cu(bool full) {
  int n = 0;
  hipError_t e = full ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scan_kernel<true>, kBlock, 0)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scan_kernel<false>, kBlock, 0);
  if (e != hipSuccess) n = 2;
  return n > 0 ? n : 1;
}

}  // namespace dq
