// scan.hip -- the fused scan: one launch evaluates every ScanShareableAnalyzer aggregation of a
// suite over every record batch (the reference's single `data.agg(...)` Spark job,
// AnalysisRunner.scala:296-303), followed by two tiny finalize launches that merge the per-item
// partials in a fixed order and fold them into the running state (Spark's final-mode merge).
//
// Work decomposition.  The host cuts every (task, batch) descriptor into work items of
// `item_rows` rows (~256 KiB of the task's buffers, a multiple of 1024 rows) and numbers the items
// task-major, so each logical task owns one contiguous range of global item indices.  The grid is
// persistent (a few workgroups per CU); every WAVE pulls items from one global counter (one
// returning atomic per ~256 KiB), streams the item's rows and writes the item's partial
// aggregation buffer (Acc) to partial[item].  Because a partial depends only on its item, never
// on which wave ran it, the result is bit-identical from run to run although the schedule is
// dynamic, and HBM-bound bodies of different cost (bitmap popcounts, Welford moments, string
// IN-lists, hashing) balance across the chip without a static cost model.
//
// Memory access.  A streaming body moves 16 values per lane per iteration with 16-byte loads:
// in step k lane l reads the contiguous 16 bytes at element (64 k + l) * VPL, so every
// wave-instruction is one contiguous 1 KiB segment and all loads of an iteration are in flight
// before the first is consumed.  The 1024-row chunk's 128-byte validity slice is fetched with one
// dword load per lane and redistributed with ds_bpermute (no LDS traffic, no barrier).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device_util.h"
#include "kernels.h"
#include "stream_load.h"

namespace dq {

// ------------------------------------------------------------------------------------------------
// Reductions
// ------------------------------------------------------------------------------------------------
// Butterfly over the wave: every lane ends with the merge of all 64 (fixed order per lane set).
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

DQ_DEV uint32_t ld32_slow(const uint8_t* bm, int64_t word, int64_t rows) {
  if (!bm) return 0xffffffffu;
  uint32_t v = 0;
  for (int b = 0; b < 4; ++b) {
    int64_t byte = word * 4 + b;
    if (byte * 8 < rows) v |= (uint32_t)bm[byte] << (8 * b);
  }
  return v;
}

// ------------------------------------------------------------------------------------------------
// TK_NUMERIC: n, wrapping Long sum, min/max in the column type, (n, avg, m2), fused predicates
// ------------------------------------------------------------------------------------------------
struct NumLane {
  int64_t n = 0, si = 0, kmin = INT64_MAX, kmax = INT64_MIN;
  double sd = 0.0, mean = 0.0, m2 = 0.0;
  uint32_t pt[kMaxPreds] = {0, 0, 0}, pn[kMaxPreds] = {0, 0, 0};  // <= item_rows / 64 per lane
};

template <typename T>
DQ_DEV int64_t num_key(T v) {
  if constexpr (std::is_floating_point<T>::value) {
    return f64_key((double)v);
  } else {
    return (int64_t)v;
  }
}

// Truth bits of a fused predicate over NV values (NULL handling is done by the caller).
template <typename T, int NV>
DQ_DEV uint32_t pred_bits(const NumPred& P, const T* x) {
  const uint32_t m1 = op_mask(P.op1), m2 = op_mask(P.op2);
  uint32_t r = 0;
  if (P.as_double) {
    const double lo = P.lo_d, hi = P.hi_d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const double xd = (double)x[i];
      uint32_t ok = (m1 >> (cmp3_f64(xd, lo) + 1)) & 1u;
      if (P.op2) ok &= (m2 >> (cmp3_f64(xd, hi) + 1)) & 1u;
      r |= ok << i;
    }
  } else {
    const int64_t lo = P.lo_i, hi = P.hi_i;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int64_t xi = (int64_t)x[i];
      uint32_t ok = (m1 >> (cmp3_i64(xi, lo) + 1)) & 1u;
      if (P.op2) ok &= (m2 >> (cmp3_i64(xi, hi) + 1)) & 1u;
      r |= ok << i;
    }
  }
  return r;
}

// NV values of the lane.  vb = validity bits, wt = where-TRUE bits (bit i <-> x[i]); values past
// the end have vb = wt = 0.  Moments: a two-pass (mean, m2) of the NV values in registers, then
// one Chan merge -- two divisions per NV rows instead of one per row.
template <typename T, int NV>
DQ_DEV void num_vals(NumLane& L, const T* x, uint32_t vb, uint32_t wt, const TaskDesc& t) {
  const uint32_t sel = vb & wt;
  const int nb = __popc(sel);
  if (nb) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const bool on = (sel >> i) & 1u;
      if constexpr (!std::is_floating_point<T>::value) L.si = wrap_add(L.si, on ? (int64_t)x[i] : 0);
      s += on ? (double)x[i] : 0.0;
      const int64_t k = num_key(x[i]);
      L.kmin = (on && k < L.kmin) ? k : L.kmin;
      L.kmax = (on && k > L.kmax) ? k : L.kmax;
    }
    if constexpr (std::is_floating_point<T>::value) L.sd += s;
    const double mb = s / (double)nb;
    double m2b = 0.0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const double d = (double)x[i] - mb;
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
  const uint32_t nulls_all = wt & ~vb & ((1u << NV) - 1u);
#pragma unroll
  for (int p = 0; p < kMaxPreds; ++p) {
    if (p >= t.n_preds) break;
    const NumPred& P = t.preds[p];
    const uint32_t r = pred_bits<T, NV>(P, x);
    const uint32_t nulls = P.null_is_true ? nulls_all : 0u;
    L.pt[p] += __popc(r & sel) + __popc(nulls);
    L.pn[p] += __popc(sel) + __popc(nulls);
  }
}

// The lane's 16 values of one iteration, in two halves (bounds the live converted values).
template <typename T>
DQ_DEV void num_rows(NumLane& L, const T (&x)[16], uint32_t vb, uint32_t wt, const TaskDesc& t) {
  num_vals<T, 8>(L, x, vb & 0xffu, wt & 0xffu, t);
  num_vals<T, 8>(L, x + 8, vb >> 8, wt >> 8, t);
}

// One 1024-row chunk, vector path: VPL values per 16-byte load, U loads per lane.  (A variant
// that prefetches chunk k+1 before chunk k's arithmetic measured 10 % slower at 168 VGPRs.)
template <typename T>
DQ_DEV void num_chunk_fast(NumLane& L, const TaskDesc& t, int64_t r0) {
  constexpr int VPL = 16 / (int)sizeof(T);
  constexpr int U = 16 / VPL;
  const int l = lane_id();
  const T* v = reinterpret_cast<const T*>(t.values) + r0;
  uint4 raw[U];
#pragma unroll
  for (int k = 0; k < U; ++k) raw[k] = ld16(v + (k * 64 + l) * VPL);
  uint32_t vb = 0xffffu, wt = 0xffffu;
  if (t.valid) {
    ChunkBits c;
    c.load(t.valid, r0);
    vb = 0;
#pragma unroll
    for (int k = 0; k < U; ++k) vb |= c.get((k * 64 + l) * VPL, VPL) << (k * VPL);
  }
  if (t.w_val) {
    ChunkBits a, b;
    a.load(t.w_val, r0);
    b.load(t.w_vld, r0);
    wt = 0;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int o = (k * 64 + l) * VPL;
      wt |= (a.get(o, VPL) & b.get(o, VPL)) << (k * VPL);
    }
  }
  T x[16];
  __builtin_memcpy(x, raw, sizeof(x));
  num_rows<T>(L, x, vb, wt, t);
}

// Same row mapping with per-element bounds checks (batch tails, unaligned buffers), one 16-byte
// group at a time so that this rarely used path does not set the kernel's register budget.
template <typename T>
DQ_DEV void num_chunk_slow(NumLane& L, const TaskDesc& t, int64_t r0, int64_t r_end) {
  constexpr int VPL = 16 / (int)sizeof(T);
  constexpr int U = 16 / VPL;
  const int l = lane_id();
  const T* v = reinterpret_cast<const T*>(t.values);
#pragma unroll 1
  for (int k = 0; k < U; ++k) {
    T x[VPL];
    uint32_t vb = 0, wt = 0;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int64_t r = r0 + (int64_t)(k * 64 + l) * VPL + j;
      x[j] = T(0);
      if (r < r_end) {
        x[j] = v[r];
        vb |= bit1(t.valid, r) << j;
        const uint32_t w = t.w_val ? (bit1(t.w_val, r) & bit1(t.w_vld, r)) : 1u;
        wt |= w << j;
      }
    }
    num_vals<T, VPL>(L, x, vb, wt, t);
  }
}

template <typename T>
DQ_DEV void num_item(const TaskDesc& t, int64_t r_begin, int64_t r_end, Acc& a) {
  NumLane L;
  int64_t r0 = r_begin;
  if (t.vec_ok)
    for (; r0 + kWaveRows <= r_end; r0 += kWaveRows) num_chunk_fast<T>(L, t, r0);
  for (; r0 < r_end; r0 += kWaveRows) num_chunk_slow<T>(L, t, r0, r_end);
  a.i[0] = L.n;
  a.i[1] = L.si;
  a.i[2] = L.kmin;
  a.i[3] = L.kmax;
#pragma unroll
  for (int p = 0; p < kMaxPreds; ++p) {
    a.i[4 + p] = L.pt[p];
    a.i[7 + p] = L.pn[p];
  }
  a.d[0] = L.sd;
  a.d[1] = L.mean;
  a.d[2] = L.m2;
}

// ------------------------------------------------------------------------------------------------
// TK_VALIDITY / TK_BOOLMAP: popcounts over bitmaps.  count0 = |A & B & W|, count1 = |B & W|
// where A = value bits (validity of a column, or an expression's value bits), B = validity bits of
// the expression (absent for TK_VALIDITY), W = where-TRUE bits.  Absent bitmaps are all ones.
// ------------------------------------------------------------------------------------------------
DQ_DEV void bits_item(const TaskDesc& t, int64_t r_begin, int64_t r_end, Acc& acc) {
  const uint8_t* A = t.kind == TK_VALIDITY ? t.valid : t.b_val;
  const uint8_t* B = t.kind == TK_VALIDITY ? nullptr : t.b_vld;
  const uint8_t* WV = t.w_val;
  const uint8_t* WD = t.w_val ? t.w_vld : nullptr;
  const int l = lane_id();
  int64_t c0 = 0, c1 = 0;
  int64_t r0 = r_begin;
  if (t.vec_ok) {
    const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
    // 4 KiB of each bitmap per wave and step: four 1 KiB wave-instructions in flight per bitmap
    for (; r0 + 32768 <= r_end; r0 += 32768) {
      uint4 a[4], b[4], x[4], y[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t byte = (r0 >> 3) + 1024 * k + 16 * l;
        a[k] = A ? ld16(A + byte) : ones;
        b[k] = B ? ld16(B + byte) : ones;
        x[k] = WV ? ld16(WV + byte) : ones;
        y[k] = WD ? ld16(WD + byte) : ones;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t m0 = b[k].x & x[k].x & y[k].x, m1 = b[k].y & x[k].y & y[k].y,
                       m2 = b[k].z & x[k].z & y[k].z, m3 = b[k].w & x[k].w & y[k].w;
        c0 += __popc(a[k].x & m0) + __popc(a[k].y & m1) + __popc(a[k].z & m2) +
              __popc(a[k].w & m3);
        c1 += __popc(m0) + __popc(m1) + __popc(m2) + __popc(m3);
      }
    }
    for (; r0 + 8192 <= r_end; r0 += 8192) {  // 1 KiB of each bitmap per wave-instruction
      const int64_t byte = (r0 >> 3) + 16 * l;
      const uint4 a = A ? ld16(A + byte) : ones;
      const uint4 b = B ? ld16(B + byte) : ones;
      const uint4 x = WV ? ld16(WV + byte) : ones;
      const uint4 y = WD ? ld16(WD + byte) : ones;
      const uint32_t m0 = b.x & x.x & y.x, m1 = b.y & x.y & y.y, m2 = b.z & x.z & y.z,
                     m3 = b.w & x.w & y.w;
      c0 += __popc(a.x & m0) + __popc(a.y & m1) + __popc(a.z & m2) + __popc(a.w & m3);
      c1 += __popc(m0) + __popc(m1) + __popc(m2) + __popc(m3);
    }
  }
  const int64_t w_end = (r_end + 31) >> 5;  // r0 is a multiple of 32
  for (int64_t w = (r0 >> 5) + l; w < w_end; w += 64) {
    uint32_t mask = 0xffffffffu;
    if (w == w_end - 1 && (r_end & 31)) mask = (1u << (r_end & 31)) - 1u;
    const uint32_t a = ld32_slow(A, w, t.rows), b = ld32_slow(B, w, t.rows);
    const uint32_t x = ld32_slow(WV, w, t.rows), y = ld32_slow(WD, w, t.rows);
    const uint32_t m = b & x & y & mask;
    c0 += __popc(a & m);
    c1 += __popc(m);
  }
  acc.i[0] = c0;
  acc.i[1] = c1;
}

// ------------------------------------------------------------------------------------------------
// TK_STR_IN:  when(where, [c IS NULL OR] c [NOT] IN (list))  -> TRUE count, non-NULL count
// ------------------------------------------------------------------------------------------------
// Membership of the string data[s, s + len) in the list; only entries of equal length are
// compared (the list is bucketed by length), first on their 8-byte prefix.  `dlen` = bytes of the
// batch's data buffer, so no read leaves it.
DQ_DEV uint32_t str_in_match(const TaskDesc& t, const uint8_t* data, int32_t s, int32_t len,
                             int32_t dlen) {
  const int b = len <= 64 ? len : kListLenSlots;
  const int lo = t.list_start[b], hi = t.list_start[b + 1];
  if (lo >= hi) return 0u;
  const uint64_t pre = load_prefix8(data + s, len, (int64_t)dlen - s);
  for (int k = lo; k < hi; ++k) {
    if (t.list_len[k] != len || t.list_pre[k] != pre) continue;
    const uint8_t* lb = t.list_bytes + t.list_boff[k];
    bool eq = true;
    for (int32_t o = 8; o < len && eq; o += 8) {
      const int32_t take = len - o < 8 ? len - o : 8;
      eq = load_prefix8(data + s + o, take, (int64_t)dlen - s - o) == load_prefix8(lb + o, take, 8);
    }
    if (eq) return 1u;
  }
  return 0u;
}

// Small lists (<= 8 entries of <= 7 bytes, the isContainedIn form): a row's 8-byte load and its
// length pack into one key -- (bytes below the length) | length << 56, ~0 for 8+ bytes, which no
// entry has -- compared against the entries' keys held in scalar registers.
struct SmallList {
  uint64_t key[8];
  DQ_DEV void load(const TaskDesc& t) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t v = t.list_key[k];
      key[k] = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
               __builtin_amdgcn_readfirstlane((uint32_t)v);
    }
  }
  // v = 8 bytes starting at the string (bytes past its end are masked off), l = its length
  DQ_DEV uint32_t match(uint64_t v, int32_t l) const {
    const uint64_t m = (1ULL << (8 * (l & 7))) - 1ULL;
    const uint64_t k = l < 8 ? ((v & m) | ((uint64_t)l << 56)) : ~0ULL;
    uint32_t hit = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) hit |= k == key[e] ? 1u : 0u;
    return hit;
  }
};

// Rows of one lane: o[0..4] offsets of 4 consecutive rows, vb / wt their validity / where bits.
DQ_DEV void str_in_rows(const TaskDesc& t, const int32_t (&o)[5], uint32_t vb, uint32_t wt,
                        int32_t dlen, int64_t& ct, int64_t& cn) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!((wt >> j) & 1u)) continue;
    if ((vb >> j) & 1u) {
      ct += str_in_match(t, t.data, o[j], o[j + 1] - o[j], dlen) ^ (uint32_t)t.negate;
      cn += 1;
    } else if (t.null_is_true) {
      ct += 1;
      cn += 1;
    }
  }
}

// Lane l owns rows r0 + 256g + 4l .. + 3 (g < 4) of a 1024-row step: one 16-byte offsets load per
// lane and group (the fifth offset comes from the next lane), then -- small lists -- one unaligned
// 8-byte load per candidate string, all 16 in flight together; the wave's string loads of a
// group fall into the same ~1 KiB of character data, so the bytes leave HBM once.
// The loads of one 1024-row step that do not depend on the character data: 4 x 16-byte offset
// loads (+ the group-closing offsets) and the validity bitmap slice.
struct StrStep {
  int4 q[4];
  int32_t last[4];
  ChunkBits c;
  DQ_DEV void load(const TaskDesc& t, const int32_t* off, int64_t r0, int l) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      {
        const uint4 u = ld16(off + r0 + 256 * g + 4 * l);
        q[g] = make_int4((int)u.x, (int)u.y, (int)u.z, (int)u.w);
      }
      last[g] = ldg_i32(off + r0 + 256 * g + 256);
    }
    // (unconditional: without a validity bitmap it reads the offsets and is ignored, so the loads
    // of a step are a fixed count the compiler can wait on one by one)
    c.load(t.valid ? t.valid : reinterpret_cast<const uint8_t*>(off), r0);
  }
};

DQ_DEV void str_in_item(const TaskDesc& t, int64_t r_begin, int64_t r_end, Acc& acc) {
  const int l = lane_id();
  const int32_t* off = reinterpret_cast<const int32_t*>(t.values);
  const int32_t dlen = off[t.rows];
  int64_t ct = 0, cn = 0;
  int64_t r0 = r_begin;
  if (t.vec_ok && r0 + kWaveRows <= r_end) {
    // software pipeline: step k+1's offsets and bitmaps are in flight while step k's strings
    // load.  The prefetch is unconditional (the last step re-reads itself): with a conditional one
    // the compiler could not count the loads in flight and waited for the prefetch before the
    // step's last strings.
    StrStep cur;
    cur.load(t, off, r0, l);
    for (; r0 + kWaveRows <= r_end; r0 += kWaveRows) {
      const int64_t rn = r0 + 2 * kWaveRows <= r_end ? r0 + kWaveRows : r0;
      uint32_t vb = 0xffffu, wt = 0xffffu;
      if (t.valid) {
        vb = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) vb |= cur.c.get(256 * g + 4 * l, 4) << (4 * g);
      }
      if (t.w_val) {  // where bitmaps: not prefetched (keeps the step's registers <= 168)
        ChunkBits wa, wb;
        wa.load(t.w_val, r0);
        wb.load(t.w_vld, r0);
        wt = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int o = 256 * g + 4 * l;
          wt |= (wa.get(o, 4) & wb.get(o, 4)) << (4 * g);
        }
      }
      int32_t o[4][5];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int32_t nxt = __shfl_down(cur.q[g].x, 1);
        o[g][0] = cur.q[g].x;
        o[g][1] = cur.q[g].y;
        o[g][2] = cur.q[g].z;
        o[g][3] = cur.q[g].w;
        o[g][4] = l == 63 ? cur.last[g] : nxt;
      }
      const int32_t step_end = cur.last[3];
      // small list and every string of the step has 8 readable bytes: one unconditional
      // unaligned 8-byte load per row, all 16 in flight, and no per-row branches
      if (t.list_small && (int64_t)step_end + 8 <= (int64_t)dlen) {
        SmallList sl;
        sl.load(t);
        uint64_t v[16];
#if DQ_STRIN_CONTIG  // diagnostic build only (wrong matches): the same bytes as compact loads
        {
          const uint8_t* base = t.data + __shfl(o[0][0], 0);  // the step's first byte
#pragma unroll
          for (int i = 0; i < 16; ++i) v[i] = ldg64_unaligned(base + 4 * (64 * i + l));
        }
#else
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) v[4 * g + j] = ldg64_unaligned(t.data + o[g][j]);
#endif
        __builtin_amdgcn_sched_barrier(0);
        cur.load(t, off, rn, l);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t hits = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            hits |= sl.match(v[4 * g + j], o[g][j + 1] - o[g][j]) << (4 * g + j);
        const uint32_t sel = vb & wt, nulls = t.null_is_true ? (wt & ~vb & 0xffffu) : 0u;
        ct += __popc((t.negate ? ~hits : hits) & sel) + __popc(nulls);
        cn += __popc(sel) + __popc(nulls);
      } else {
        cur.load(t, off, rn, l);
#pragma unroll
        for (int g = 0; g < 4; ++g) str_in_rows(t, o[g], vb >> (4 * g), wt >> (4 * g), dlen, ct, cn);
      }
    }
  }
  for (; r0 < r_end; r0 += 256) {  // tail (and unaligned buffers): 4 rows per lane, bounds-checked
    const int64_t rb = r0 + 4 * l;
    int32_t o[5];
    uint32_t vb = 0, wt = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) o[j] = (rb + j <= r_end) ? off[rb + j] : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t r = rb + j;
      if (r < r_end) {
        vb |= bit1(t.valid, r) << j;
        wt |= (t.w_val ? (bit1(t.w_val, r) & bit1(t.w_vld, r)) : 1u) << j;
      }
    }
    str_in_rows(t, o, vb, wt, dlen, ct, cn);
  }
  acc.i[0] = ct;
  acc.i[1] = cn;
}

// ------------------------------------------------------------------------------------------------
// TK_DTYPE (DataType, StatefulDataType.scala:36-69): each value of when(where, col) as a string is
// NULL, else the first of FRACTIONAL ^(-|\+)? ?\d*\.\d*$, INTEGRAL ^(-|\+)? ?\d*$ (which matches
// ""), BOOLEAN ^(true|false)$ it fully matches, else STRING.  Non-string columns are classified
// as their cast to string: integers are Integral, booleans Boolean, and a double / float prints
// with a '.' (Fractional) exactly when it is finite and 0 or 1e-3 <= |x| < 1e7 (Java's
// Double/Float.toString switch to E-notation, or NaN / Infinity, are String).
// ------------------------------------------------------------------------------------------------
enum DtypeClass { DT_NULL = 0, DT_FRACTIONAL, DT_INTEGRAL, DT_BOOLEAN, DT_STRING };

DQ_DEV int dtype_of_string(const uint8_t* p, int32_t n) {
  DevBytes b{p};
  int32_t i = 0;
  if (i < n && (b.u8(i) == '-' || b.u8(i) == '+')) ++i;
  if (i < n && b.u8(i) == ' ') ++i;
  while (i < n && b.u8(i) - '0' < 10u) ++i;
  if (i == n) return DT_INTEGRAL;  // no '.': FRACTIONAL fails, INTEGRAL matches
  if (b.u8(i) == '.') {
    ++i;
    while (i < n && b.u8(i) - '0' < 10u) ++i;
    if (i == n) return DT_FRACTIONAL;
  }
  if (n == 4 && b.u8(0) == 't' && b.u8(1) == 'r' && b.u8(2) == 'u' && b.u8(3) == 'e') return DT_BOOLEAN;
  if (n == 5 && b.u8(0) == 'f' && b.u8(1) == 'a' && b.u8(2) == 'l' && b.u8(3) == 's' && b.u8(4) == 'e')
    return DT_BOOLEAN;
  return DT_STRING;
}

// A string whose first byte is none of - + space digit . t f is STRING (no pattern above can
// match it); only the others take dtype_of_string's walk.
DQ_DEV bool dtype_needs_walk(uint32_t c0) {
  return c0 - '0' < 10u || c0 == '-' || c0 == '+' || c0 == ' ' || c0 == '.' || c0 == 't' ||
         c0 == 'f';
}

// utf8 columns: lane l classifies rows r0 + 64j + l (j < 4) of each 256-row step, with the four
// rows' offsets and then their first data dwords loaded together (one round trip each for the
// step, not per row); most strings are decided by their first byte.
DQ_DEV void dtype_str_rows(const TaskDesc& t, int64_t r_begin, int64_t r_end, int64_t (&c)[5]) {
  const int l = lane_id();
  const int32_t* off = reinterpret_cast<const int32_t*>(t.values);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 256) {
    int32_t s[4], n[4];
    uint32_t ok = 0, in = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t r = r0 + 64 * j + l;
      s[j] = n[j] = 0;
      if (r < r_end) {
        in |= 1u << j;
        uint32_t v = bit1(t.valid, r);
        if (t.w_val) v &= bit1(t.w_val, r) & bit1(t.w_vld, r);
        ok |= v << j;
        s[j] = off[r];
        n[j] = off[r + 1] - s[j];
      }
    }
    uint32_t d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // the dword holding each string's first byte
      const uintptr_t a = reinterpret_cast<uintptr_t>(t.data + s[j]);
      d[j] = ((ok >> j) & 1u) && n[j] > 0 ? *reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3)) >> (8 * (a & 3))
                                          : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!((in >> j) & 1u)) continue;
      int k;
      if (!((ok >> j) & 1u)) k = DT_NULL;
      else if (n[j] == 0) k = DT_INTEGRAL;  // "" matches INTEGRAL's pattern
      else if (dtype_needs_walk(d[j] & 0xffu)) k = dtype_of_string(t.data + s[j], n[j]);
      else k = DT_STRING;
#pragma unroll
      for (int q = 0; q < 5; ++q) c[q] += k == q;
    }
  }
}

DQ_DEV void dtype_item(const TaskDesc& t, int64_t r_begin, int64_t r_end, Acc& acc) {
  int64_t c[5] = {0, 0, 0, 0, 0};
  const int32_t* off = reinterpret_cast<const int32_t*>(t.values);
  if (t.type == DQ_UTF8) {
    dtype_str_rows(t, r_begin, r_end, c);
#pragma unroll
    for (int q = 0; q < 5; ++q) acc.i[q] = c[q];
    return;
  }
  const int tid = DQ_TYPE_ID(t.type);
  for (int64_t r = r_begin + lane_id(); r < r_end; r += 64) {
    const uint32_t w = t.w_val ? bit1(t.w_val, r) & bit1(t.w_vld, r) : 1u;
    int k;
    if (!w || !bit1(t.valid, r)) {
      k = DT_NULL;
    } else if (tid == DQ_DATE32 || tid == DQ_TIMESTAMP_US) {
      k = DT_STRING;  // "yyyy-MM-dd[ HH:mm:ss...]" matches none of the three patterns
    } else if (tid == DQ_DECIMAL128) {
      // BigDecimal.toString: an integer at scale 0, plain "d.ddd" while the adjusted exponent is
      // >= -6, else "d.dddE-n" (which no pattern matches)
      const uint64_t* v = reinterpret_cast<const uint64_t*>(t.values) + 2 * r;
      const int sc = DQ_DECIMAL_SCALE(t.type);
      k = sc == 0 ? DT_INTEGRAL
                  : (dec_adjusted(v[0], (int64_t)v[1], sc) >= -6 ? DT_FRACTIONAL : DT_STRING);
    } else if (t.type == DQ_UTF8) {
      const int32_t s = off[r];
      k = dtype_of_string(t.data + s, off[r + 1] - s);
    } else if (t.type == DQ_BOOL) {
      k = DT_BOOLEAN;
    } else if (t.type == DQ_FLOAT64 || t.type == DQ_FLOAT32) {
      const double x = load_f64(t.type, t.values, r);
      const double ax = x < 0 ? -x : x;
      k = (x == x && (ax == 0.0 || (ax >= 1e-3 && ax < 1e7))) ? DT_FRACTIONAL : DT_STRING;
    } else {
      k = DT_INTEGRAL;
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) c[q] += k == q;
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) acc.i[q] = c[q];
}

// ------------------------------------------------------------------------------------------------
// TK_DECIMAL: one decimal(p, s) column, 16 bytes per row.  Lane l takes row r0 + 64 k + l of each
// 256-row step (every wave-instruction reads one contiguous 1 KiB of values): n, the exact 192-bit
// sum of the unscaled values (Spark's decimal Sum before its result-type check), the 128-bit Min /
// Max in the column's own order, and the moments of the values cast to double
// (CentralMomentAgg's DoubleType input: Decimal.toDouble, correctly rounded, dec_to_double) --
// a lane's 4 rows two-pass, then one Chan merge.
// ------------------------------------------------------------------------------------------------
DQ_DEV void dec_item(const TaskDesc& t, int64_t r_begin, int64_t r_end, Acc& acc) {
  const int scale = DQ_DECIMAL_SCALE(t.type);
  const uint4* v = reinterpret_cast<const uint4*>(t.values);
  const int l = lane_id();
  int64_t n = 0;
  int64_t s[3] = {0, 0, 0};
  int64_t mnlo = -1, mnhi = INT64_MAX, mxlo = 0, mxhi = INT64_MIN;
  double mean = 0.0, m2 = 0.0;
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 256) {
    double x[4];
    uint32_t sel = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t r = r0 + 64 * k + l;
      x[k] = 0.0;
      if (r >= r_end) continue;
      uint32_t ok = bit1(t.valid, r);
      if (t.w_val) ok &= bit1(t.w_val, r) & bit1(t.w_vld, r);
      if (!ok) continue;
      const uint4 q = v[r];
      const uint64_t lo = (uint64_t)q.x | ((uint64_t)q.y << 32);
      const int64_t hi = (int64_t)((uint64_t)q.z | ((uint64_t)q.w << 32));
      add192(s, lo, hi);
      if (i128_lt((int64_t)lo, hi, mnlo, mnhi)) {
        mnlo = (int64_t)lo;
        mnhi = hi;
      }
      if (i128_lt(mxlo, mxhi, (int64_t)lo, hi)) {
        mxlo = (int64_t)lo;
        mxhi = hi;
      }
      x[k] = dec_to_double(lo, hi, scale);
      sel |= 1u << k;
    }
    const int nb = __popc(sel);
    if (!nb) continue;
    double sum = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) sum += x[k];
    const double mb = sum / (double)nb;
    double m2b = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double d = x[k] - mb;
      m2b += ((sel >> k) & 1u) ? d * d : 0.0;
    }
    if (n == 0) {
      mean = mb;
      m2 = m2b;
    } else {
      moments_merge((double)n, mean, m2, (double)nb, mb, m2b);
    }
    n += nb;
  }
  acc.i[0] = n;
  acc.i[1] = s[0];
  acc.i[2] = s[1];
  acc.i[3] = s[2];
  acc.i[4] = mnlo;
  acc.i[5] = mnhi;
  acc.i[6] = mxlo;
  acc.i[7] = mxhi;
  acc.d[1] = mean;
  acc.d[2] = m2;
}

// ------------------------------------------------------------------------------------------------
// TK_COMOMENTS (Correlation): rows where x and y are both non-NULL (and where is TRUE).
// Lane l owns rows r0 + 128k + 2l + {0, 1} (k < 4) of a 512-row step.
// ------------------------------------------------------------------------------------------------
// Vector path for two 8-byte columns (Long / Double), 1024 rows per wave: sixteen 16-byte loads
// per lane in flight (each wave-instruction one contiguous 1 KiB); lane l owns rows
// r0 + 128k + 2l + {0, 1} (k < 8).  The lane's 16 selected rows form one block: two-pass
// (mean, co-moments), then one Chan merge -- 2 divisions per 16 rows instead of per 8.
DQ_DEV double as_f64(uint64_t bits, bool is_long) {
  return is_long ? (double)(int64_t)bits : __builtin_bit_cast(double, bits);
}

// The co-moments of a lane's 16 rows (bit i of sel: row i selected) merged into (n, c).
template <int K = 8>
DQ_DEV void corr_fold16(const uint4* qx, const uint4* qy, uint32_t sel, bool xl, bool yl, int64_t& n,
                        double* c) {
  const int nb = __popc(sel);
  if (!nb) return;
  double xs[2 * K], ys[2 * K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    xs[2 * k] = as_f64((uint64_t)qx[k].x | ((uint64_t)qx[k].y << 32), xl);
    xs[2 * k + 1] = as_f64((uint64_t)qx[k].z | ((uint64_t)qx[k].w << 32), xl);
    ys[2 * k] = as_f64((uint64_t)qy[k].x | ((uint64_t)qy[k].y << 32), yl);
    ys[2 * k + 1] = as_f64((uint64_t)qy[k].z | ((uint64_t)qy[k].w << 32), yl);
  }
  double sx = 0, sy = 0;
#pragma unroll
  for (int i = 0; i < 2 * K; ++i) {
    if ((sel >> i) & 1u) {
      sx += xs[i];
      sy += ys[i];
    }
  }
  double b[5];
  b[0] = sx / nb;
  b[1] = sy / nb;
  b[2] = b[3] = b[4] = 0.0;
#pragma unroll
  for (int i = 0; i < 2 * K; ++i) {
    if ((sel >> i) & 1u) {
      const double dx = xs[i] - b[0], dy = ys[i] - b[1];
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

DQ_DEV void corr_chunk8(const TaskDesc& t, int64_t r0, bool xl, bool yl, int64_t& n, double* c) {
  const int l = lane_id();
  const uint64_t* X = reinterpret_cast<const uint64_t*>(t.values) + r0 + 2 * l;
  const uint64_t* Y = reinterpret_cast<const uint64_t*>(t.values2) + r0 + 2 * l;
  uint4 qx[8], qy[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    qx[k] = ld16(X + 128 * k);
    qy[k] = ld16(Y + 128 * k);
  }
  const int64_t w0 = (r0 >> 5) + (l >> 4);
  const uint32_t sh = (uint32_t)(2 * l) & 31u;
  uint32_t sel = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t w = w0 + 4 * k;
    uint32_t s = bits32(t.valid, w) & bits32(t.valid2, w);
    if (t.w_val) s &= bits32(t.w_val, w) & bits32(t.w_vld, w);
    sel |= ((s >> sh) & 3u) << (2 * k);
  }
  corr_fold16(qx, qy, sel, xl, yl, n, c);
}

DQ_DEV void hll_update(uint32_t* regs, uint64_t h);
template <int K>
DQ_DEV void corr_hll_chunk8(const TaskDesc& t, int64_t r0, bool xl, bool yl, int64_t& n, double* c,
                            uint32_t* regs);

// HLL = true (BC_CORR_HLL): the same pass also feeds the rows of column t.hll_side into the HLL
// registers `regs` of the fused ApproxCountDistinct task.
// K: 16-byte loads per lane and column per chunk (K = 8: 1024 rows per wave; K = 4: 512 rows, half
// the registers, so more waves per SIMD hide the loads behind the hashing)
template <bool HLL, int K = 8>
DQ_DEV void corr_rows(const TaskDesc& t, int64_t r_begin, int64_t r_end, Acc& acc, uint32_t* regs) {
  const int l = lane_id();
  int64_t n = 0;
  double c[5] = {0, 0, 0, 0, 0};  // xAvg, yAvg, ck, xMk, yMk
  int64_t r_fast = r_begin;
  const bool x8 = t.type == DQ_INT64 || t.type == DQ_FLOAT64;
  const bool y8 = t.type2 == DQ_INT64 || t.type2 == DQ_FLOAT64;
  if (t.vec_ok && x8 && y8) {
    const bool xl = t.type == DQ_INT64, yl = t.type2 == DQ_INT64;
    if constexpr (HLL) {
      for (; r_fast + 128 * K <= r_end; r_fast += 128 * K) corr_hll_chunk8<K>(t, r_fast, xl, yl, n, c, regs);
    } else {
      for (; r_fast + 1024 <= r_end; r_fast += 1024) corr_chunk8(t, r_fast, xl, yl, n, c);
    }
  }
  for (int64_t r0 = r_fast; r0 < r_end; r0 += 512) {
    double xs[8], ys[8];
    uint32_t sel = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t r = r0 + 128 * k + 2 * l + j;
        const int i = 2 * k + j;
        xs[i] = 0.0;
        ys[i] = 0.0;
        if (r < r_end) {
          const uint32_t wm = t.w_val ? bit1(t.w_val, r) & bit1(t.w_vld, r) : 1u;
          const uint32_t s = bit1(t.valid, r) & bit1(t.valid2, r) & wm;
          if (s) {
            xs[i] = load_f64(t.type, t.values, r);
            ys[i] = load_f64(t.type2, t.values2, r);
          }
          sel |= s << i;
          if constexpr (HLL) {
            const bool hy = t.hll_side != 0;
            if (bit1(hy ? t.valid2 : t.valid, r) & wm)
              hll_update(regs, hash_wide(hy ? t.type2 : t.type, hy ? t.values2 : t.values, r));
          }
        }
      }
    }
    const int nb = __popc(sel);
    if (!nb) continue;
    double sx = 0, sy = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sx += xs[i];
      sy += ys[i];
    }
    double b[5];
    b[0] = sx / nb;
    b[1] = sy / nb;
    b[2] = b[3] = b[4] = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if ((sel >> i) & 1u) {
        const double dx = xs[i] - b[0], dy = ys[i] - b[1];
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
  acc.i[0] = n;
  for (int f = 0; f < 5; ++f) acc.d[f] = c[f];
}
DQ_DEV void corr_item(const TaskDesc& t, int64_t r_begin, int64_t r_end, Acc& acc) {
  corr_rows<false>(t, r_begin, r_end, acc, nullptr);
}

// ------------------------------------------------------------------------------------------------
// TK_HLL: the workgroup's 512 registers of each HLL task live in LDS (one u32 per register);
// atomicMax only when the rank can raise the register.  Flushed once per workgroup at the end.
// ------------------------------------------------------------------------------------------------
DQ_DEV void hll_update(uint32_t* regs, uint64_t h) {
  uint32_t idx, pw;
  hll_index_rank(h, idx, pw);
  if (pw > regs[idx]) atomicMax(&regs[idx], pw);
}

// 8-byte keys (Long, Double), 1024 rows per wave: eight 16-byte loads per lane in flight (each
// wave-instruction one contiguous 1 KiB), lane l owns rows r0 + 128k + 2l and +1; their validity /
// where bits come from one dword per bitmap and k (L1-resident, the wave's 128-byte slice).
DQ_DEV void hll_chunk8(const TaskDesc& t, int64_t r0, bool dbl, uint32_t* regs) {
  const int l = lane_id();
  const uint64_t* v = reinterpret_cast<const uint64_t*>(t.values);
  uint4 q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) q[k] = ld16(v + r0 + 128 * k + 2 * l);
  const int64_t w0 = (r0 >> 5) + (l >> 4);
  const uint32_t sh = (uint32_t)(2 * l) & 31u;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t w = w0 + 4 * k;
    uint32_t s = bits32(t.valid, w);
    if (t.w_val) s &= bits32(t.w_val, w) & bits32(t.w_vld, w);
    s = (s >> sh) & 3u;
    uint64_t x0 = (uint64_t)q[k].x | ((uint64_t)q[k].y << 32);
    uint64_t x1 = (uint64_t)q[k].z | ((uint64_t)q[k].w << 32);
    if (dbl) {  // doubleToLongBits: every NaN hashes as the canonical one
      if (__builtin_bit_cast(double, x0) != __builtin_bit_cast(double, x0)) x0 = 0x7ff8000000000000ULL;
      if (__builtin_bit_cast(double, x1) != __builtin_bit_cast(double, x1)) x1 = 0x7ff8000000000000ULL;
    }
    const uint64_t h0 = xxh_long(x0, 42), h1 = xxh_long(x1, 42);
    if (s & 1u) hll_update(regs, h0);
    if (s & 2u) hll_update(regs, h1);
  }
}

// TK_HLL over a utf8 column: lane l takes row r0 + l of each 64-row step.  A string of at most 64
// bytes is read as the aligned dwords that hold it -- all issued before any is used, as many as
// the wave's longest such string needs (each dword holds a byte of the string, so none leaves
// its buffer) -- and hashed from registers; longer strings take xxh_bytes' loop.
DQ_DEV void hll_str_rows(const TaskDesc& t, int64_t r_begin, int64_t r_end, uint32_t* regs) {
  const int l = lane_id();
  const int32_t* off = reinterpret_cast<const int32_t*>(t.values);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 64) {
    const int64_t r = r0 + l;
    uint32_t ok = 0;
    int32_t s = 0, e = 0;
    if (r < r_end) {
      ok = bit1(t.valid, r);
      if (t.w_val) ok &= bit1(t.w_val, r) & bit1(t.w_vld, r);
      s = off[r];
      e = off[r + 1];
    }
    const int32_t len = e - s;
    const bool reg = ok && len <= 64;
    const uintptr_t a = reinterpret_cast<uintptr_t>(t.data + s);
    const uint32_t* base = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t sh = (uint32_t)(a & 3);
    const int nd = reg && len > 0 ? (int)((sh + (uint32_t)len + 3) >> 2) : 0;  // dwords: <= 17
    int ndw = nd;
#pragma unroll
    for (int o = 32; o; o >>= 1) ndw = max(ndw, __shfl_xor(ndw, o));
    ndw = __builtin_amdgcn_readfirstlane(ndw);
    uint32_t dw[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) {
      dw[k] = 0;
      if (k < ndw) dw[k] = nd ? base[min(k, nd - 1)] : 0u;
    }
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_alignbyte(dw[j + 1], dw[j], sh);
    if (reg) hll_update(regs, xxh_bytes_regs64(w, len, 42));
    if (ok && !reg) hll_update(regs, xxh_bytes(UBytes{t.data + s}, (int64_t)len, 42));
  }
}

DQ_DEV void hll_item(const TaskDesc& t, int64_t r_begin, int64_t r_end, uint32_t* regs) {
  if (t.type == DQ_UTF8) {
    hll_str_rows(t, r_begin, r_end, regs);
    return;
  }
  const int l = lane_id();
  int64_t r_fast = r_begin;
  if (t.vec_ok && (t.type == DQ_INT64 || t.type == DQ_FLOAT64)) {
    const bool dbl = t.type == DQ_FLOAT64;
    for (; r_fast + 1024 <= r_end; r_fast += 1024) hll_chunk8(t, r_fast, dbl, regs);
  }
  for (int64_t r0 = r_fast; r0 < r_end; r0 += 256) {
#pragma unroll 2
    for (int k = 0; k < 4; ++k) {
      const int64_t r = r0 + 64 * k + l;
      if (r >= r_end) continue;
      uint32_t s = bit1(t.valid, r);
      if (t.w_val) s &= bit1(t.w_val, r) & bit1(t.w_vld, r);
      if (!s) continue;
      hll_update(regs, hash_row(t.type, t.values, t.data, r));
    }
  }
}

// BC_CORR_HLL vector path: ApproxCountDistinct(x) + Correlation(x, y) (BASELINE.json configs[3])
// read x and y once.  Loads and co-moments as corr_chunk8; the HLL rows are the non-NULL rows of
// column t.hll_side (and where), hashed as hll_chunk8 does.
template <int K>
DQ_DEV void corr_hll_chunk8(const TaskDesc& t, int64_t r0, bool xl, bool yl, int64_t& n, double* c,
                            uint32_t* regs) {
  const int l = lane_id();
  const uint64_t* X = reinterpret_cast<const uint64_t*>(t.values) + r0 + 2 * l;
  const uint64_t* Y = reinterpret_cast<const uint64_t*>(t.values2) + r0 + 2 * l;
  uint4 qx[K], qy[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    qx[k] = ld16(X + 128 * k);
    qy[k] = ld16(Y + 128 * k);
  }
  const bool hy = t.hll_side != 0;
  const bool hdbl = (hy ? t.type2 : t.type) == DQ_FLOAT64;
  const int64_t w0 = (r0 >> 5) + (l >> 4);
  const uint32_t sh = (uint32_t)(2 * l) & 31u;
  uint32_t sel = 0, hsel = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t w = w0 + 4 * k;
    const uint32_t vx = bits32(t.valid, w), vy = bits32(t.valid2, w);
    const uint32_t wm = t.w_val ? bits32(t.w_val, w) & bits32(t.w_vld, w) : ~0u;
    sel |= (((vx & vy & wm) >> sh) & 3u) << (2 * k);
    hsel |= ((((hy ? vy : vx) & wm) >> sh) & 3u) << (2 * k);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint4 q = hy ? qy[k] : qx[k];
    uint64_t x0 = (uint64_t)q.x | ((uint64_t)q.y << 32);
    uint64_t x1 = (uint64_t)q.z | ((uint64_t)q.w << 32);
    if (hdbl) {  // doubleToLongBits: every NaN hashes as the canonical one
      if (__builtin_bit_cast(double, x0) != __builtin_bit_cast(double, x0)) x0 = 0x7ff8000000000000ULL;
      if (__builtin_bit_cast(double, x1) != __builtin_bit_cast(double, x1)) x1 = 0x7ff8000000000000ULL;
    }
    const uint64_t h0 = xxh_long(x0, 42), h1 = xxh_long(x1, 42);
    if ((hsel >> (2 * k)) & 1u) hll_update(regs, h0);
    if ((hsel >> (2 * k + 1)) & 1u) hll_update(regs, h1);
  }
  corr_fold16<K>(qx, qy, sel, xl, yl, n, c);
}

// ------------------------------------------------------------------------------------------------
// Work queue: kQueueHeads head words per launch kind (kernels.h).  Items [lo, hi) are cut into
// kQueueHeads contiguous slices; a wave pulls from its home slice (the workgroup's XCD under the
// round-robin dispatch -- for speed only, any placement is correct), then from the others in
// turn.  Every call either returns an item or moves to the next slice, so a wave ends after at
// most kQueueHeads empty pulls, and a queue that was not re-armed just ends every wave.
// ------------------------------------------------------------------------------------------------
// The rows of global work item `item` of descriptor t: big items first, then the small tail items.
DQ_DEV void item_range(const TaskDesc& t, uint32_t item, int64_t& r_begin, int64_t& r_end) {
  const int64_t li = (int64_t)item - t.item_begin;
  if (li < t.n_big) {
    r_begin = li * t.item_rows;
    r_end = min(r_begin + t.item_rows, t.rows);
  } else {
    r_begin = t.n_big * t.item_rows + (li - t.n_big) * t.small_rows;
    r_end = min(r_begin + t.small_rows, t.rows);
  }
}

DQ_DEV bool queue_next(uint32_t* heads, uint32_t lo, uint32_t hi, int home, int& step,
                       uint32_t& item) {
  const uint32_t n = hi - lo;
  while (step < kQueueHeads) {
    const int x = (home + step) % kQueueHeads;
    const uint32_t b = lo + (uint32_t)((uint64_t)n * x / kQueueHeads);
    const uint32_t e = lo + (uint32_t)((uint64_t)n * (x + 1) / kQueueHeads);
    uint32_t v = 0;
    if (b < e) {
      if (lane_id() == 0) v = atomicAdd(&heads[x * kQueueStride], 1u);
      v = __builtin_amdgcn_readfirstlane(v);
      if (v < e - b) {
        item = b + v;
        return true;
      }
    }
    ++step;
  }
  return false;
}

// ------------------------------------------------------------------------------------------------
// The scan kernels (persistent; waves pull items from a queue)
// ------------------------------------------------------------------------------------------------
// One instantiation per body class (kernels.h): a launch runs the items of every task of its class,
// so each body is compiled alone and its register allocation -- hence its occupancy -- is what that
// body needs, not the maximum over all bodies.  A suite is one launch per class it uses (S10: the
// validity, numeric-int64 and string-IN classes) plus the two finalize launches; items of all
// batches of a class run in the same launch.
// The fused HLL + co-moment body (BC_CORR_HLL) is bound by its 64-bit multiplies as much as by
// HBM: it is held to 128 VGPRs so four waves per SIMD hide the loads behind the hashing.
template <int BC, int K = 8>
__global__ void __launch_bounds__(kBlock, (BC == BC_CORR_HLL ? (K == 8 ? 4 : 5) : 1)) scan_kernel(const TaskDesc* __restrict__ tasks, int n_desc,
                                                      uint32_t item_lo, uint32_t item_hi,
                                                      const uint32_t* __restrict__ order,
                                                      uint32_t* __restrict__ queue,
                                                      Acc* __restrict__ partial,
                                                      uint32_t* __restrict__ hll_stage, int n_hll) {
  extern __shared__ uint32_t hll_lds[];
  constexpr bool kRegs = BC == BC_HLL || BC == BC_CORR_HLL;  // HLL registers in LDS
  if constexpr (kRegs) {
    for (int i = threadIdx.x; i < n_hll * kHllM; i += kBlock) hll_lds[i] = 0;
    __syncthreads();
  }
  const int l = lane_id();
  int step = 0;
  uint32_t item = 0;
  // with an order list the queue runs over its entries (item_lo = 0, item_hi = entries)
  while (queue_next(queue, item_lo, item_hi, (int)(blockIdx.x % kQueueHeads), step, item)) {
    if (order) item = order[item];
    // descriptor = the last one whose first item is <= item (empty descriptors share their
    // first item with the next non-empty one, so they are never selected)
    int lo = 0, hi = n_desc - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((uint64_t)tasks[mid].item_begin <= item) lo = mid;
      else hi = mid - 1;
    }
    const TaskDesc& t = tasks[lo];
    int64_t r_begin, r_end;
    item_range(t, item, r_begin, r_end);
    Acc a;
    acc_init(t.kind, a);
    if constexpr (BC == BC_NUM_I8) num_item<int8_t>(t, r_begin, r_end, a);
    if constexpr (BC == BC_NUM_I16) num_item<int16_t>(t, r_begin, r_end, a);
    if constexpr (BC == BC_NUM_I32) num_item<int32_t>(t, r_begin, r_end, a);
    if constexpr (BC == BC_NUM_I64) num_item<int64_t>(t, r_begin, r_end, a);
    if constexpr (BC == BC_NUM_F32) num_item<float>(t, r_begin, r_end, a);
    if constexpr (BC == BC_NUM_F64) num_item<double>(t, r_begin, r_end, a);
    if constexpr (BC == BC_BITS) bits_item(t, r_begin, r_end, a);
    if constexpr (BC == BC_STR_IN) str_in_item(t, r_begin, r_end, a);
    if constexpr (BC == BC_DTYPE) dtype_item(t, r_begin, r_end, a);
    if constexpr (BC == BC_CORR) corr_item(t, r_begin, r_end, a);
    if constexpr (BC == BC_DECIMAL) dec_item(t, r_begin, r_end, a);
    if constexpr (BC == BC_CORR_HLL) corr_rows<true, K>(t, r_begin, r_end, a, hll_lds + t.hll_out * kHllM);
    if constexpr (BC == BC_HLL) {
      hll_item(t, r_begin, r_end, hll_lds + t.hll_out * kHllM);
    } else {
      constexpr int kind = BC <= BC_NUM_F64 ? TK_NUMERIC
                           : BC == BC_BITS  ? TK_VALIDITY
                           : BC == BC_DTYPE ? TK_DTYPE
                           : BC == BC_CORR || BC == BC_CORR_HLL ? TK_COMOMENTS
                           : BC == BC_DECIMAL ? TK_DECIMAL
                                            : TK_STR_IN;
      wave_reduce(kind, a);
      if (l == 0) partial[item] = a;
    }
  }
  if constexpr (kRegs) {
    __syncthreads();
    for (int i = threadIdx.x; i < n_hll * kHllM; i += kBlock) {
      const uint32_t v = hll_lds[i];
      if (v) atomicMax(&hll_stage[i], v);
    }
  }
}

// HLL never rides in the mixed launch (kernels.h kMixedHllMax): its XXH64 body compiled in here
// cost 48 bytes of spilled constants per lane.
static_assert(kMixedHllMax == 0, "scan_mixed_kernel has no HLL body");

// Mixed launch: the items of every non-HLL body class in one grid.  Queue position q runs item
// order[q]; the host interleaves the classes' items in proportion to their counts, so at any time
// the chip holds a blend of string-gather waves (latency-bound) and streaming waves (bandwidth-
// bound) instead of one class at a time.  The body is chosen per item (a wave-uniform branch on
// the descriptor).  Inlined side by side the bodies would need ~173 VGPRs (2 waves/SIMD); the
// kernel is pinned to 3 waves/SIMD (168 VGPRs) like the string body alone.
// MASK: the body classes compiled in (bit per BodyClass).  kMixedS10 (validity bits, Long
// columns, string IN: BASELINE configs[1]) leaves out the bodies that spilled 28 bytes per lane
// into the all-class kernel.
template <uint32_t MASK>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 3)))
scan_mixed_kernel(const TaskDesc* __restrict__ tasks, int n_desc, uint32_t n_order,
                  const uint32_t* __restrict__ order, uint32_t* __restrict__ queue,
                  Acc* __restrict__ partial, uint32_t* __restrict__ hll_stage, int n_hll) {
  // HLL items (compute-bound XXH64) interleave with the streaming bodies; their registers live in
  // this workgroup's LDS as in scan_kernel<BC_HLL> and are flushed once at the end
  extern __shared__ uint32_t mix_lds[];
  if (n_hll) {
    for (int i = threadIdx.x; i < n_hll * kHllM; i += kBlock) mix_lds[i] = 0;
    __syncthreads();
  }
  const int l = lane_id();
  int step = 0;
  uint32_t q = 0;
  while (queue_next(queue, 0, n_order, (int)(blockIdx.x % kQueueHeads), step, q)) {
    const uint32_t item = order[q];
    int lo = 0, hi = n_desc - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((uint64_t)tasks[mid].item_begin <= item) lo = mid;
      else hi = mid - 1;
    }
    const TaskDesc& t = tasks[lo];
    int64_t r_begin, r_end;
    item_range(t, item, r_begin, r_end);
    Acc a;
    acc_init(t.kind, a);
#define DQ_BODY(BCV, CALL) \
  case BCV:                \
    if constexpr ((MASK >> BCV) & 1u) CALL; \
    break;
    switch (t.body) {
      DQ_BODY(BC_NUM_I8, (num_item<int8_t>(t, r_begin, r_end, a)))
      DQ_BODY(BC_NUM_I16, (num_item<int16_t>(t, r_begin, r_end, a)))
      DQ_BODY(BC_NUM_I32, (num_item<int32_t>(t, r_begin, r_end, a)))
      DQ_BODY(BC_NUM_I64, (num_item<int64_t>(t, r_begin, r_end, a)))
      DQ_BODY(BC_NUM_F32, (num_item<float>(t, r_begin, r_end, a)))
      DQ_BODY(BC_NUM_F64, (num_item<double>(t, r_begin, r_end, a)))
      DQ_BODY(BC_BITS, (bits_item(t, r_begin, r_end, a)))
      DQ_BODY(BC_STR_IN, (str_in_item(t, r_begin, r_end, a)))
      DQ_BODY(BC_DTYPE, (dtype_item(t, r_begin, r_end, a)))
      DQ_BODY(BC_CORR, (corr_item(t, r_begin, r_end, a)))
      default: break;
    }
#undef DQ_BODY
    wave_reduce(t.kind, a);
    if (l == 0) partial[item] = a;
  }
  if (n_hll) {
    __syncthreads();
    for (int i = threadIdx.x; i < n_hll * kHllM; i += kBlock) {
      const uint32_t v = mix_lds[i];
      if (v) atomicMax(&hll_stage[i], v);
    }
  }
}

// Item range [lo, hi) of logical task `task` (descriptors are numbered task-major), kind and HLL
// register file, with the block's threads reading the descriptors in parallel (every thread of the
// block must call it): a one-thread walk is a chain of dependent scalar loads, tens of
// microseconds per finalize launch at S10's 60 descriptors.
DQ_DEV void task_range_block(const TaskDesc* tasks, int n_desc, int task, int64_t& lo, int64_t& hi,
                             int& kind, int& hll_out) {
  __shared__ unsigned long long s_lo, s_hi;
  __shared__ int s_kind, s_hll;
  if (threadIdx.x == 0) {
    s_lo = ~0ULL;
    s_hi = 0;
    s_kind = 0;
    s_hll = -1;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < n_desc; d += blockDim.x) {
    const TaskDesc& t = tasks[d];
    if (t.out != task) continue;
    atomicMin(&s_lo, (unsigned long long)t.item_begin);
    atomicMax(&s_hi, (unsigned long long)(t.item_begin + t.n_items));
    s_kind = t.kind;  // (one value per task: every descriptor of the task carries it)
    s_hll = t.hll_out;
  }
  __syncthreads();
  lo = s_lo == ~0ULL ? 0 : (int64_t)s_lo;
  hi = s_lo == ~0ULL ? 0 : (int64_t)s_hi;
  kind = s_kind;
  hll_out = s_hll;
  __syncthreads();  // (the shared cells may be reused by a later call)
}

// acc_merge over the wave, lane i with lane i + s for s = 32, 16, ..., 1 (a fixed tree); the
// wave's result in lane 0.  Shuffles, no LDS and no barriers.
DQ_DEV void wave_merge_tree(int kind, Acc& a) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    Acc b;
#pragma unroll
    for (int k = 0; k < 10; ++k) b.i[k] = __shfl_down(a.i[k], s);
#pragma unroll
    for (int k = 0; k < 6; ++k) b.d[k] = __shfl_down(a.d[k], s);
    if (lane_id() < s) acc_merge(kind, a, b);
  }
}

// The finalize: workgroup (task, f) merges slice f of the task's item partials -- thread i takes
// items i, i + kBlock, ... of the slice in order, then a fixed tree (each wave by shuffles, then
// the waves in order) -- into partial2[task][f]; the LAST workgroup of a task to finish (an arrival
// counter, left at zero for the next launch) folds the kFinParts slices in a fixed tree into the
// running accumulator (reset: from the initial values, dq_state_reset queues no device work).
// HLL tasks: slice 0 merges the staging registers into the running registers and clears them.
// Workgroup (0, 0) re-arms the scan queues.  One launch (the two-launch form spent ~26 us per
// S10 step, most of it in an 8-level LDS tree with a barrier per level).
__global__ void __launch_bounds__(kBlock) finalize_kernel(const TaskDesc* __restrict__ tasks,
                                                          int n_desc,
                                                          const Acc* __restrict__ partial,
                                                          Acc* __restrict__ partial2,
                                                          Acc* __restrict__ acc,
                                                          uint32_t* __restrict__ hll_stage,
                                                          uint8_t* __restrict__ hll_acc,
                                                          uint32_t* __restrict__ queue,
                                                          uint32_t* __restrict__ arrivals, int reset) {
  __shared__ Acc sh[kBlock / 64];
  __shared__ Acc sh2[kFinParts];
  __shared__ uint32_t s_last;
  const int task = blockIdx.x, f = blockIdx.y;
  int64_t lo, hi;
  int kind, hll_out;
  task_range_block(tasks, n_desc, task, lo, hi, kind, hll_out);
  if (task == 0 && f == 0)
    for (int i = threadIdx.x; i < kQueues * kQueueHeads; i += blockDim.x) queue[i * kQueueStride] = 0u;
  if (kind == TK_HLL) {
    if (f != 0) return;
    for (int reg = threadIdx.x; reg < kHllM; reg += blockDim.x) {
      const int64_t i = (int64_t)hll_out * kHllM + reg;
      const uint32_t m = reset ? 0u : hll_acc[i], v = hll_stage[i];
      hll_acc[i] = (uint8_t)(v > m ? v : m);
      hll_stage[i] = 0;
    }
    return;
  }
  if (kind == 0) return;  // (block-uniform: a task without descriptors)
  Acc a;
  acc_init(kind, a);
  const int64_t m = hi - lo;
  const int64_t b = lo + m * f / kFinParts, e = lo + m * (f + 1) / kFinParts;
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) acc_merge(kind, a, partial[i]);
  wave_merge_tree(kind, a);
  const int wave = threadIdx.x >> 6;
  if (lane_id() == 0) sh[wave] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc r = sh[0];
    for (int w = 1; w < kBlock / 64; ++w) acc_merge(kind, r, sh[w]);
    partial2[(int64_t)task * kFinParts + f] = r;
    __threadfence();  // the slice is visible before the arrival
    s_last = atomicAdd(&arrivals[task], 1u) == (uint32_t)(kFinParts - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last) return;
  // the task's last workgroup: the kFinParts slices in a fixed tree, into the accumulator
  __threadfence();
  static_assert(kFinParts <= kBlock && (kFinParts & (kFinParts - 1)) == 0, "power of 2");
  if (threadIdx.x < kFinParts) sh2[threadIdx.x] = partial2[(int64_t)task * kFinParts + threadIdx.x];
  __syncthreads();
  for (int s2 = kFinParts / 2; s2 > 0; s2 >>= 1) {
    if (threadIdx.x < s2) acc_merge(kind, sh2[threadIdx.x], sh2[threadIdx.x + s2]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    Acc r;
    if (reset) acc_init(kind, r);
    else r = acc[task];
    acc_merge(kind, r, sh2[0]);
    acc[task] = r;
    arrivals[task] = 0u;  // (for the next launch)
  }
}

// ------------------------------------------------------------------------------------------------
// Host-side launchers
// ------------------------------------------------------------------------------------------------
size_t scan_lds_bytes(int body, int n_hll) {
  return body == BC_HLL || body == BC_CORR_HLL ? (size_t)n_hll * kHllM * 4 : 0;
}

// DQ_CORR_K=4: A/B hook, the fused co-moment + HLL body on 4-deep chunks at 6 waves per SIMD
static int corr_k() {
  static const int k = [] {
    const char* e = getenv("DQ_CORR_K");
    return e && atoi(e) == 4 ? 4 : 8;
  }();
  return k;
}

template <int BC>
static void launch_body(const ScanLaunch& L, const TaskDesc* tasks, int n_desc, int n_hll,
                        uint32_t* queues, Acc* partial, uint32_t* hll_stage, hipStream_t stream) {
  auto go = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, dim3(L.grid), dim3(kBlock), scan_lds_bytes(BC, n_hll), stream,
                       tasks, n_desc, L.item_lo, L.item_hi, L.order,
                       queues + BC * kQueueHeads * kQueueStride, partial, hll_stage, n_hll);
  };
  if constexpr (BC == BC_CORR_HLL) {
    if (corr_k() == 4) {
      go(scan_kernel<BC, 4>);
      return;
    }
  }
  go(scan_kernel<BC>);
}

template <int BC>
static int occupancy_of(int n_hll) {
  int n = 0;
  hipError_t e;
  if constexpr (BC == BC_CORR_HLL) {
    e = corr_k() == 4
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scan_kernel<BC, 4>, kBlock, scan_lds_bytes(BC, n_hll))
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scan_kernel<BC>, kBlock, scan_lds_bytes(BC, n_hll));
  } else {
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scan_kernel<BC>, kBlock, scan_lds_bytes(BC, n_hll));
  }
  if (e != hipSuccess) n = 2;
  return n > 0 ? n : 1;
}

hipError_t launch_scan(const TaskDesc* tasks, int n_desc, int n_tasks, const ScanLaunch* launches,
                       int n_launches, int n_hll, uint32_t* queues, Acc* partial, Acc* partial2,
                       uint32_t* hll_stage, Acc* acc, uint8_t* hll_acc, uint32_t* arrivals,
                       hipStream_t stream, int reset) {
  if (n_desc == 0 || n_launches == 0) return hipSuccess;
  for (int k = 0; k < n_launches; ++k) {
    const ScanLaunch& L = launches[k];
    if (L.item_hi <= L.item_lo) continue;
    if (L.body == kBodyMixed) {
      const int mix_hll = L.lds_hll;
      auto go = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, dim3(L.grid), dim3(kBlock), (size_t)mix_hll * kHllM * 4, stream,
                           tasks, n_desc, L.item_hi, L.order,
                           queues + kBodyMixed * kQueueHeads * kQueueStride, partial, hll_stage,
                           mix_hll);
      };
      static const bool all = getenv("DQ_MIXED_ALL") != nullptr;  // A/B hook
      if ((L.classes & ~kMixedS10) == 0 && !all) go(scan_mixed_kernel<kMixedS10>);
      else go(scan_mixed_kernel<kMixedAll>);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      continue;
    }
    switch (L.body) {
      case BC_NUM_I8: launch_body<BC_NUM_I8>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_NUM_I16: launch_body<BC_NUM_I16>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_NUM_I32: launch_body<BC_NUM_I32>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_NUM_I64: launch_body<BC_NUM_I64>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_NUM_F32: launch_body<BC_NUM_F32>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_NUM_F64: launch_body<BC_NUM_F64>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_BITS: launch_body<BC_BITS>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_STR_IN: launch_body<BC_STR_IN>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_DTYPE: launch_body<BC_DTYPE>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_CORR: launch_body<BC_CORR>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_HLL: launch_body<BC_HLL>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_CORR_HLL: launch_body<BC_CORR_HLL>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      case BC_DECIMAL: launch_body<BC_DECIMAL>(L, tasks, n_desc, n_hll, queues, partial, hll_stage, stream); break;
      default: return hipErrorInvalidValue;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(finalize_kernel, dim3(n_tasks, kFinParts), dim3(kBlock), 0, stream, tasks,
                     n_desc, partial, partial2, acc, hll_stage, hll_acc, queues, arrivals, reset);
  return hipGetLastError();
}

int scan_max_blocks_per_cu(int body, int n_hll) {
  switch (body) {
    case BC_NUM_I8: return occupancy_of<BC_NUM_I8>(n_hll);
    case BC_NUM_I16: return occupancy_of<BC_NUM_I16>(n_hll);
    case BC_NUM_I32: return occupancy_of<BC_NUM_I32>(n_hll);
    case BC_NUM_I64: return occupancy_of<BC_NUM_I64>(n_hll);
    case BC_NUM_F32: return occupancy_of<BC_NUM_F32>(n_hll);
    case BC_NUM_F64: return occupancy_of<BC_NUM_F64>(n_hll);
    case BC_BITS: return occupancy_of<BC_BITS>(n_hll);
    case BC_STR_IN: return occupancy_of<BC_STR_IN>(n_hll);
    case BC_DTYPE: return occupancy_of<BC_DTYPE>(n_hll);
    case BC_CORR: return occupancy_of<BC_CORR>(n_hll);
    case BC_HLL: return occupancy_of<BC_HLL>(n_hll);
    case BC_CORR_HLL: return occupancy_of<BC_CORR_HLL>(n_hll);
    case BC_DECIMAL: return occupancy_of<BC_DECIMAL>(n_hll);
    case kBodyMixed: {
      int n = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scan_mixed_kernel<kMixedAll>, kBlock,
                                                       (size_t)n_hll * kHllM * 4) != hipSuccess)
        n = 2;
      return n > 0 ? n : 1;
    }
    default: return 1;
  }
}

}  // namespace dq
