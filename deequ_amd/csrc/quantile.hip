// quantile.hip -- the device half of ApproxQuantile (ApproxQuantile.scala:41-104).
//
// The reference feeds every non-NULL value, as a double, into Spark's ApproximatePercentile
// (QuantileSummaries, Greenwald-Khanna with relativeError).  Here the values are order-preserving
// 64-bit keys (Java's Double.compare order as unsigned order: NaNs canonical and largest, -0.0
// before 0.0) and the host gets either
//   * every value, sorted (rocPRIM radix sort) -- few enough that the host replays Spark's own
//     insert + compress exactly, or relativeError 0 (the exact summary); or
//   * the values at m evenly spaced exact ranks floor(j (n - 1) / (m - 1)) (a GK summary whose
//     error is far inside relativeError), found by a radix SELECT straight over the columns:
//     histogram passes narrow every rank to a bin of the keys' top bits, and only once the bins
//     that hold a rank are small are their keys compacted (and, when few, sorted).
// Every pass runs over a fixed row -> block map: a block's histogram lands in a row of per-block
// partials, so a compaction knows each block's output offset from the pass before it (no
// cursor atomic: one global atomic per step on one address bound the old gather at ~1.3 TB/s).
// A pass also takes each active prefix's smallest and largest key, so a rank whose bin holds one
// distinct value (integers of a narrow range: every further pass would only spend bits) is
// decided at once.
// The summary arithmetic -- insert, compress, merge, query -- is host code
// (deequ_amd/analyzers/quantile.py).
#include <hip/hip_runtime.h>

#include <memory>

#include <cstring>  // rocprim headers use memset without including it

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <vector>

#include "device_util.h"
#include "decimal.h"
#include "kernels.h"

using namespace dq;

extern "C" __device__ uint64_t __ockl_wfred_add_u64(uint64_t);
extern "C" __device__ uint64_t __ockl_wfred_min_u64(uint64_t);
extern "C" __device__ uint64_t __ockl_wfred_max_u64(uint64_t);

namespace {

constexpr int kRsThreads = 256;
constexpr int kRsK = 16;  // keys per thread per step, all loads in flight before the first is used
constexpr int64_t kRsStep = (int64_t)kRsThreads * kRsK;
constexpr int kSelBins = 8192;         // a pass's bins: A active prefixes << D digit bits
constexpr int kSelMaxTargets = 2048;   // ranks selected (more: one sort of every key)
constexpr int kMapBits = 13;           // prefixes this short find their index in an LDS map
constexpr int kKeys = 0;               // source type: an array of keys (every one present)
constexpr int kTargetBlocks = 1024;    // blocks of a pass over all the sources

// Double.compare order as unsigned order (the canonical NaN is the largest key)
DQ_HD uint64_t ordered_key(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  return (b >> 63) ? ~b : (b | (1ULL << 63));
}
DQ_HD double from_ordered(uint64_t k) {
  return __builtin_bit_cast(double, (k >> 63) ? (k & ~(1ULL << 63)) : ~k);
}

// One batch of a numeric column, or an array of keys, and its first block in the pass.
struct Src {
  const uint8_t* valid;
  const void* values;
  int64_t rows;
  int64_t blk0;
};

// The sources of one launch: up to kMaxSrc batches, their blocks back to back from blk0 of the first
constexpr int kMaxSrc = 8;
struct Srcs {
  Src s[kMaxSrc];
  int n;
};
// this block's source and its block index within it
DQ_DEV const Src& block_src(const Srcs& ss, int64_t& local) {
  const int64_t blk = ss.s[0].blk0 + blockIdx.x;
  int j = 0;
  while (j + 1 < ss.n && ss.s[j + 1].blk0 <= blk) ++j;
  local = blk - ss.s[j].blk0;
  return ss.s[j];
}

// What a pass bins by: the keys whose top `bits` bits are one of the A (sorted) prefixes, by
// their next D bits (bin a << D | digit); R rows per block.
struct Pass {
  const uint64_t* act;
  int A, bits, D;
  int64_t R;
  int minmax;  // also each prefix's min / max key (every pass with bits > 0; pass 0 of integers)
};

template <int TY> struct Ty { using T = double; };
template <> struct Ty<kKeys> { using T = uint64_t; };
template <> struct Ty<DQ_INT8> { using T = int8_t; };
template <> struct Ty<DQ_INT16> { using T = int16_t; };
template <> struct Ty<DQ_INT32> { using T = int32_t; };
template <> struct Ty<DQ_INT64> { using T = int64_t; };
template <> struct Ty<DQ_FLOAT32> { using T = float; };
// rows per 16-byte load (VEC: the values are 16-byte aligned)
template <int TY, bool VEC>
constexpr int vec_of() {
  return !VEC ? 1 : sizeof(typename Ty<TY>::T) == 8 ? 2 : sizeof(typename Ty<TY>::T) == 4 ? 4 : 1;
}

template <int TY>
DQ_DEV uint64_t to_key(typename Ty<TY>::T v) {
  if constexpr (TY == kKeys) {
    return v;
  } else {
    double d = (double)v;
    if (d != d) d = __builtin_nan("");  // Double.compare: every NaN is the canonical one
    return ordered_key(d);
  }
}

// The keys of one step of a block (rows i0 + (u * kRsThreads + tid) * V + j, j < V): each lane's V
// consecutive rows come with one 16-byte load and one validity byte (V <= 4 rows from an aligned
// row: their bits share the byte).  ok: present and in range.
template <int TY, bool VEC>
DQ_DEV void step_keys(const Src& s, int64_t i0, int64_t r_end, uint64_t (&k)[kRsK], bool (&ok)[kRsK]) {
  using T = typename Ty<TY>::T;
  constexpr int V = vec_of<TY, VEC>(), U = kRsK / V;
  const T* vals = reinterpret_cast<const T*>(s.values);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t r = i0 + ((int64_t)u * kRsThreads + threadIdx.x) * V;
    const int64_t rc = r < r_end ? r : r_end - 1;  // (in bounds; discarded below)
    T v[V];
    if constexpr (V > 1) {
      if (r + V <= r_end) {
        const uint4 x = *reinterpret_cast<const uint4*>(vals + r);
        __builtin_memcpy(v, &x, 16);
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] = vals[r + j < r_end ? r + j : r_end - 1];
      }
    } else {
      v[0] = vals[rc];
    }
    uint32_t vb = 0xffu;
    if constexpr (TY != kKeys)
      if (s.valid) vb = (uint32_t)s.valid[rc >> 3] >> (r & 7);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      ok[u * V + j] = ((vb >> j) & 1u) && r + j < r_end;
      k[u * V + j] = to_key<TY>(v[j]);
    }
  }
}

DQ_DEV int find_prefix(const uint64_t* act, int A, uint64_t p) {
  int lo = 0, hi = A;  // first index with act[i] >= p
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (act[mid] < p) lo = mid + 1;
    else hi = mid;
  }
  return lo < A && act[lo] == p ? lo : -1;
}

// LDS of a pass: the prefixes, (bits > 0) their min / max keys, (bits <= kMapBits) the prefix map
struct PassLds {
  uint64_t* act;
  unsigned long long *mn, *mx;
  int16_t* map;
  bool mapped;
  DQ_DEV void load(const Pass& p, uint64_t* base, bool minmax) {
    act = base;
    mn = reinterpret_cast<unsigned long long*>(base + p.A);
    mx = mn + p.A;
    map = reinterpret_cast<int16_t*>(base + p.A + (minmax ? 2 * p.A : 0));
    mapped = p.bits > 0 && p.bits <= kMapBits;
    for (int i = threadIdx.x; i < p.A; i += kRsThreads) {
      act[i] = p.act[i];
      if (minmax) {
        mn[i] = ~0ULL;
        mx[i] = 0ULL;
      }
    }
    if (mapped) {
      __syncthreads();
      for (int i = threadIdx.x; i < (1 << p.bits); i += kRsThreads) map[i] = -1;
      __syncthreads();
      for (int i = threadIdx.x; i < p.A; i += kRsThreads) map[act[i]] = (int16_t)i;
    }
  }
  DQ_DEV int index(const Pass& p, uint64_t k) const {
    if (p.bits == 0) return 0;
    const uint64_t pre = k >> (64 - p.bits);
    return mapped ? (int)map[pre] : find_prefix(act, p.A, pre);
  }
};
DQ_HD size_t pass_lds_words(const Pass& p, bool minmax) {  // in u64 words, before the bins
  return (size_t)p.A * (minmax ? 3 : 1) +
         (p.bits > 0 && p.bits <= kMapBits ? ((2u << p.bits) + 7) / 8 : 0);
}
DQ_DEV uint32_t digit_of(const Pass& p, uint64_t k) {
  return p.D ? (uint32_t)((k << p.bits) >> (64 - p.D)) : 0u;
}

// A pass's histogram: block g's counts -> partial[g][A << D]; with bits > 0 also each prefix's
// min / max key -> pmm[g][2A].
template <int TY, bool VEC>
__global__ void __launch_bounds__(kRsThreads)
rs_hist(Srcs ss, Pass p, uint32_t* __restrict__ partial, unsigned long long* __restrict__ pmm) {
  extern __shared__ uint64_t rs_lds[];
  int64_t lb;
  const Src& s = block_src(ss, lb);
  const bool minmax = p.minmax != 0;
  PassLds L;
  L.load(p, rs_lds, minmax);
  const int nb = p.A << p.D;
  uint32_t* s_hist = reinterpret_cast<uint32_t*>(rs_lds + pass_lds_words(p, minmax));
  for (int i = threadIdx.x; i < nb; i += kRsThreads) s_hist[i] = 0;
  __syncthreads();
  const int64_t r_begin = lb * p.R;
  const int64_t r_end = r_begin + p.R < s.rows ? r_begin + p.R : s.rows;
  // pass 0 (one prefix, the whole column): each thread's running min / max, reduced once
  const bool mm0 = minmax && p.bits == 0;
  uint64_t tlo = ~0ULL, thi = 0ULL;
  for (int64_t i0 = r_begin; i0 < r_end; i0 += kRsStep) {
    uint64_t k[kRsK];
    bool ok[kRsK];
    step_keys<TY, VEC>(s, i0, r_end, k, ok);
#pragma unroll
    for (int u = 0; u < kRsK; ++u) {
      const int a = ok[u] ? L.index(p, k[u]) : -1;
      if (a >= 0) atomicAdd(&s_hist[(a << p.D) | (int)digit_of(p, k[u])], 1u);
      if (mm0) {
        if (ok[u]) {
          tlo = k[u] < tlo ? k[u] : tlo;
          thi = k[u] > thi ? k[u] : thi;
        }
      } else if (minmax) {  // a wave whose keys share one prefix (narrow data) reduces before its atomic
        const int a0 = __builtin_amdgcn_readfirstlane(a);
        if (__ballot(a == a0) == ~0ULL) {
          if (a0 >= 0) {
            const uint64_t lo = __ockl_wfred_min_u64(k[u]), hi = __ockl_wfred_max_u64(k[u]);
            if (__lane_id() == 0) {
              atomicMin(&L.mn[a0], (unsigned long long)lo);
              atomicMax(&L.mx[a0], (unsigned long long)hi);
            }
          }
        } else if (a >= 0) {
          atomicMin(&L.mn[a], (unsigned long long)k[u]);
          atomicMax(&L.mx[a], (unsigned long long)k[u]);
        }
      }
    }
  }
  if (mm0) {
    tlo = __ockl_wfred_min_u64(tlo);
    thi = __ockl_wfred_max_u64(thi);
    if (__lane_id() == 0) {
      atomicMin(&L.mn[0], (unsigned long long)tlo);
      atomicMax(&L.mx[0], (unsigned long long)thi);
    }
  }
  __syncthreads();
  const int64_t g = s.blk0 + lb;
  uint32_t* row = partial + (size_t)g * nb;
  for (int i = threadIdx.x; i < nb; i += kRsThreads) row[i] = s_hist[i];
  if (minmax) {
    unsigned long long* mrow = pmm + (size_t)g * 2 * p.A;
    for (int i = threadIdx.x; i < p.A; i += kRsThreads) {
      mrow[2 * i] = L.mn[i];
      mrow[2 * i + 1] = L.mx[i];
    }
  }
}

// hist[bin] = sum over the blocks of partial[g][bin]; blockIdx.y takes 32 blocks' rows
__global__ void __launch_bounds__(256)
rs_sum(const uint32_t* __restrict__ partial, int64_t G, int nb, unsigned long long* __restrict__ hist) {
  const int bin = blockIdx.x * 256 + threadIdx.x;
  if (bin >= nb) return;
  const int64_t g0 = (int64_t)blockIdx.y * 32, g1 = g0 + 32 < G ? g0 + 32 : G;
  unsigned long long t = 0;
  for (int64_t g = g0; g < g1; ++g) t += partial[(size_t)g * nb + bin];
  if (t) atomicAdd(&hist[bin], t);
}

// mm[2a] = min, mm[2a + 1] = max over the blocks of prefix a's keys (mm preset to ~0 / 0)
__global__ void __launch_bounds__(256)
rs_minmax(const unsigned long long* __restrict__ pmm, int64_t G, int A, unsigned long long* __restrict__ mm) {
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (a >= A) return;
  const int64_t g0 = (int64_t)blockIdx.y * 32, g1 = g0 + 32 < G ? g0 + 32 : G;
  unsigned long long lo = ~0ULL, hi = 0ULL;
  for (int64_t g = g0; g < g1; ++g) {
    const unsigned long long x = pmm[(size_t)g * 2 * A + 2 * a], y = pmm[(size_t)g * 2 * A + 2 * a + 1];
    lo = x < lo ? x : lo;
    hi = y > hi ? y : hi;
  }
  if (lo != ~0ULL) atomicMin(&mm[2 * a], lo);
  if (hi) atomicMax(&mm[2 * a + 1], hi);
}

// kept[g] = block g's keys in the selected bins (sel: an nb-bit mask)
__global__ void __launch_bounds__(256)
rs_kept(const uint32_t* __restrict__ partial, int nb, const uint32_t* __restrict__ sel,
        unsigned long long* __restrict__ kept) {
  __shared__ unsigned long long s_red[4];
  const uint32_t* row = partial + (size_t)blockIdx.x * nb;
  unsigned long long t = 0;
  for (int i = threadIdx.x; i < nb; i += 256)
    if ((sel[i >> 5] >> (i & 31)) & 1u) t += row[i];
  t = (unsigned long long)__ockl_wfred_add_u64((uint64_t)t);
  if (__lane_id() == 0) s_red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) kept[blockIdx.x] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

// base = exclusive scan of kept[0..G) (one block)
__global__ void __launch_bounds__(1024) rs_scan(const unsigned long long* __restrict__ kept, int64_t G,
                                                unsigned long long* __restrict__ base) {
  __shared__ unsigned long long s_w[16];
  __shared__ unsigned long long s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 < G; c0 += 1024) {
    const int64_t g = c0 + threadIdx.x;
    const unsigned long long v = g < G ? kept[g] : 0ULL;
    unsigned long long x = v;  // inclusive scan in the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(x, d);
      if ((int)__lane_id() >= d) x += y;
    }
    const int w = threadIdx.x >> 6;
    if (__lane_id() == 63) s_w[w] = x;
    __syncthreads();
    unsigned long long before = s_carry;
    for (int j = 0; j < w; ++j) before += s_w[j];
    if (g < G) base[g] = before + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) s_carry = before + x;
    __syncthreads();
  }
}

// The keys in the selected bins of a pass (same blocks and rows as its rs_hist) -> out[base[g] ..]
template <int TY, bool VEC>
__global__ void __launch_bounds__(kRsThreads)
rs_compact(Srcs ss, Pass p, const uint32_t* __restrict__ sel, const unsigned long long* __restrict__ base,
           uint64_t* __restrict__ out) {
  extern __shared__ uint64_t rs_lds[];
  int64_t lb;
  const Src& s = block_src(ss, lb);
  __shared__ uint32_t s_cur;
  PassLds L;
  L.load(p, rs_lds, false);
  const int nb = p.A << p.D;
  uint32_t* s_sel = reinterpret_cast<uint32_t*>(rs_lds + pass_lds_words(p, false));
  for (int i = threadIdx.x; i < (nb + 31) / 32; i += kRsThreads) s_sel[i] = sel[i];
  if (threadIdx.x == 0) s_cur = 0;
  __syncthreads();
  const unsigned long long ob = base[s.blk0 + lb];
  const int lane = (int)__lane_id();
  const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;
  const int64_t r_begin = lb * p.R;
  const int64_t r_end = r_begin + p.R < s.rows ? r_begin + p.R : s.rows;
  for (int64_t i0 = r_begin; i0 < r_end; i0 += kRsStep) {
    uint64_t k[kRsK];
    bool ok[kRsK];
    step_keys<TY, VEC>(s, i0, r_end, k, ok);
#pragma unroll
    for (int u = 0; u < kRsK; ++u) {
      bool keep = false;
      if (ok[u]) {
        const int a = L.index(p, k[u]);
        if (a >= 0) {
          const uint32_t bin = ((uint32_t)a << p.D) | digit_of(p, k[u]);
          keep = (s_sel[bin >> 5] >> (bin & 31)) & 1u;
        }
      }
      const uint64_t bal = __ballot(keep);
      if (!bal) continue;
      uint32_t off = 0;
      if (lane == 0) off = atomicAdd(&s_cur, (uint32_t)__builtin_popcountll(bal));
      off = __shfl(off, 0);
      if (keep) out[ob + off + (uint32_t)__builtin_popcountll(bal & lt)] = k[u];
    }
  }
}

// out[j] = from_ordered(keys[idx[j]])
__global__ void select_pick(const uint64_t* __restrict__ keys, const int64_t* __restrict__ idx,
                            int64_t m, double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < m) out[j] = from_ordered(keys[idx[j]]);
}

// Dense counting select for integer columns of a narrow range (every keyed value in
// [lo, lo + n_vals), n_vals <= kDenseQ and its counters fit the device's LDS): each workgroup adds its rows to per-value LDS counters
// (one LDS add per row) and writes them to its row of `partial`; rs_sum then totals them per value
// and the host reads the ranks off the running counts -- one pass over the column instead of the
// radix select's histogram passes and compaction.  The value is the one the select would return:
// the row's double (Spark feeds ApproxQuantile doubles), as an integer.
constexpr int kDenseQ = 40960;  // 160 KiB of u32 counters: one workgroup per CU
constexpr int kDenseQThreads = 1024;
template <int TY>
__global__ void __launch_bounds__(kDenseQThreads)
rs_dense(Srcs ss, int64_t lo, int n_vals, uint32_t* __restrict__ partial) {
  extern __shared__ uint32_t dq_cnt[];
  for (int i = threadIdx.x; i < n_vals; i += kDenseQThreads) dq_cnt[i] = 0;
  __syncthreads();
  using T = typename Ty<TY>::T;
  for (int j = 0; j < ss.n; ++j) {  // every source, grid-strided (a few rows per thread in flight)
    const Src& s = ss.s[j];
    const T* vals = reinterpret_cast<const T*>(s.values);
    const int64_t stride = (int64_t)gridDim.x * kDenseQThreads * 4;
    for (int64_t r0 = (int64_t)blockIdx.x * kDenseQThreads * 4; r0 < s.rows; r0 += stride) {
      T v[4];
      uint32_t ok = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t r = r0 + (int64_t)u * kDenseQThreads + threadIdx.x;
        const bool in = r < s.rows;
        v[u] = vals[in ? r : 0];
        ok |= (in && (!s.valid || ((s.valid[r >> 3] >> (r & 7)) & 1u)) ? 1u : 0u) << u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if ((ok >> u) & 1u) atomicAdd(&dq_cnt[(uint32_t)((int64_t)(double)v[u] - lo)], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n_vals; i += kDenseQThreads) partial[(size_t)blockIdx.x * n_vals + i] = dq_cnt[i];
}

// out[j] = from_ordered(sorted[j])
__global__ void keys_to_doubles(const uint64_t* __restrict__ sorted, int64_t n, double* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
    out[j] = from_ordered(sorted[j]);
}

hipError_t sort_keys(const uint64_t* in, uint64_t* out, size_t n, DevBuf<uint8_t>& tmp,
                     hipStream_t stream) {
  size_t tmp_bytes = 0;
  hipError_t e = rocprim::radix_sort_keys(nullptr, tmp_bytes, in, out, n, 0, 64, stream);
  if (e != hipSuccess) return e;
  e = tmp.ensure(std::max<size_t>(tmp_bytes, 16));
  if (e != hipSuccess) return e;
  return rocprim::radix_sort_keys(tmp.p, tmp_bytes, in, out, n, 0, 64, stream);
}

// The keys a pass runs over: the batches of a column (type TY) or one array of keys, cut into
// blocks of R rows.
struct Source {
  int type;
  std::vector<Src> parts;
  int64_t R = kRsStep, G = 0, M = 0;  // rows per block, blocks, keys (non-NULL rows: after pass 0)
  bool aligned16() const {
    for (const Src& s : parts)
      if (reinterpret_cast<uintptr_t>(s.values) & 15) return false;
    return true;
  }
  void cut(int64_t total_rows) {
    R = std::max<int64_t>(4 * kRsStep, (total_rows / kTargetBlocks + kRsStep - 1) / kRsStep * kRsStep);
    G = 0;
    for (Src& s : parts) {
      s.blk0 = G;
      G += (s.rows + R - 1) / R;
    }
  }
};

// The sources in launches of at most kMaxSrc batches each (blocks back to back)
template <class F>
void for_launches(const Source& src, F&& f) {
  for (size_t i = 0; i < src.parts.size(); i += kMaxSrc) {
    Srcs ss;
    ss.n = (int)std::min<size_t>(kMaxSrc, src.parts.size() - i);
    int64_t blocks = 0;
    for (int j = 0; j < ss.n; ++j) {
      ss.s[j] = src.parts[i + j];
      blocks += (ss.s[j].rows + src.R - 1) / src.R;
    }
    f(ss, (unsigned)blocks);
  }
}

template <int TY, bool VEC>
void launch_hist_t(const Source& src, Pass p, uint32_t* partial, unsigned long long* pmm, hipStream_t st) {
  p.R = src.R;
  const size_t lds = pass_lds_words(p, p.minmax != 0) * 8 + (size_t)(p.A << p.D) * 4;
  for_launches(src, [&](const Srcs& ss, unsigned blocks) {
    hipLaunchKernelGGL(HIP_KERNEL_NAME(rs_hist<TY, VEC>), dim3(blocks), dim3(kRsThreads), lds, st, ss, p, partial, pmm);
  });
}
template <int TY, bool VEC>
void launch_compact_t(const Source& src, Pass p, const uint32_t* sel, const unsigned long long* base,
                      uint64_t* out, hipStream_t st) {
  p.R = src.R;
  const size_t lds = pass_lds_words(p, false) * 8 + (size_t)(((p.A << p.D) + 31) / 32) * 4;
  for_launches(src, [&](const Srcs& ss, unsigned blocks) {
    hipLaunchKernelGGL(HIP_KERNEL_NAME(rs_compact<TY, VEC>), dim3(blocks), dim3(kRsThreads), lds, st, ss, p, sel, base, out);
  });
}
#define RS_DISPATCH_V(fn, V, ...)                              \
  switch (src.type) {                                          \
    case kKeys: fn<kKeys, V>(__VA_ARGS__); break;              \
    case DQ_INT8: fn<DQ_INT8, V>(__VA_ARGS__); break;          \
    case DQ_INT16: fn<DQ_INT16, V>(__VA_ARGS__); break;        \
    case DQ_INT32: fn<DQ_INT32, V>(__VA_ARGS__); break;        \
    case DQ_INT64: fn<DQ_INT64, V>(__VA_ARGS__); break;        \
    case DQ_FLOAT32: fn<DQ_FLOAT32, V>(__VA_ARGS__); break;    \
    default: fn<DQ_FLOAT64, V>(__VA_ARGS__); break;            \
  }
#define RS_DISPATCH(fn, ...)                    \
  if (src.aligned16()) {                        \
    RS_DISPATCH_V(fn, true, __VA_ARGS__)        \
  } else {                                      \
    RS_DISPATCH_V(fn, false, __VA_ARGS__)       \
  }

// One pass over `src`: its bins' counts (host `h`, A << D of them) and, with bits > 0, each
// prefix's min / max key (host `mm`); the per-block partials stay on the device for a compaction.
struct Passer {
  hipStream_t st;
  DevBuf<uint32_t> partial;
  DevBuf<unsigned long long> pmm, hist, mm, kept, base;
  DevBuf<uint64_t> act;
  DevBuf<uint32_t> sel;
  std::vector<unsigned long long> h, mmh;
  dq_status run(const Source& src, const std::vector<uint64_t>& prefixes, int bits, int D, Pass& p,
                bool with_minmax = false) {
    const int A = (int)prefixes.size(), nb = A << D;
    const bool minmax = bits > 0 || with_minmax;
    // LDS of rs_hist: A prefixes + their min / max (24 B each), the prefix map (16 KB at 13 bits)
    // and the bins (A << D <= kSelBins counters): at most 2048 ranks -> 96 KB, inside gfx950's
    // 160 KB per workgroup; checked against the device so a smaller part fails loudly
    {
      const Pass q{nullptr, A, bits, D, src.R, minmax ? 1 : 0};
      const size_t need = pass_lds_words(q, minmax) * 8 + (size_t)nb * 4;
      int dev = 0, cap = 0;
      HIP_TRY(hipGetDevice(&dev));
      HIP_TRY(hipDeviceGetAttribute(&cap, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
      if (need > (size_t)cap)
        return fail(DQ_ERR_UNSUPPORTED, "radix select pass needs %zu B of LDS (device: %d)", need, cap);
    }
    HIP_TRY(act.ensure(A));
    HIP_TRY(hipMemcpyAsync(act.p, prefixes.data(), (size_t)A * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(partial.ensure((size_t)src.G * nb));
    HIP_TRY(hist.ensure(nb));
    HIP_TRY(hipMemsetAsync(hist.p, 0, (size_t)nb * 8, st));
    p = Pass{act.p, A, bits, D, src.R, minmax ? 1 : 0};
    if (minmax) {
      HIP_TRY(pmm.ensure((size_t)src.G * 2 * A));
      HIP_TRY(mm.ensure((size_t)2 * A));
      std::vector<unsigned long long> init(2 * (size_t)A);
      for (int a = 0; a < A; ++a) init[2 * a] = ~0ULL, init[2 * a + 1] = 0ULL;
      mmh.swap(init);
      HIP_TRY(hipMemcpyAsync(mm.p, mmh.data(), (size_t)A * 16, hipMemcpyHostToDevice, st));
    }
    RS_DISPATCH(launch_hist_t, src, p, partial.p, pmm.p, st);
    HIP_TRY(hipGetLastError());
    const unsigned gy = (unsigned)((src.G + 31) / 32);
    hipLaunchKernelGGL(rs_sum, dim3((unsigned)((nb + 255) / 256), gy), dim3(256), 0, st, partial.p, src.G,
                       nb, hist.p);
    HIP_TRY(hipGetLastError());
    if (minmax) {
      hipLaunchKernelGGL(rs_minmax, dim3((unsigned)((A + 255) / 256), gy), dim3(256), 0, st, pmm.p, src.G,
                         A, mm.p);
      HIP_TRY(hipGetLastError());
    }
    h.resize(nb);
    HIP_TRY(d2h(h.data(), hist.p, (size_t)nb * 8, st));
    if (minmax) HIP_TRY(d2h(mmh.data(), mm.p, (size_t)A * 16, st));
    return DQ_OK;
  }
  // the keys of the last pass's selected bins (mask: nb bits) -> dst (T of them)
  dq_status compact(const Source& src, const Pass& p, const std::vector<uint32_t>& mask, uint64_t* dst) {
    HIP_TRY(sel.ensure(mask.size()));
    HIP_TRY(hipMemcpyAsync(sel.p, mask.data(), mask.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(kept.ensure((size_t)src.G));
    HIP_TRY(base.ensure((size_t)src.G));
    hipLaunchKernelGGL(rs_kept, dim3((unsigned)src.G), dim3(256), 0, st, partial.p, p.A << p.D, sel.p, kept.p);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(rs_scan, dim3(1), dim3(1024), 0, st, kept.p, src.G, base.p);
    HIP_TRY(hipGetLastError());
    RS_DISPATCH(launch_compact_t, src, p, sel.p, base.p, dst, st);
    HIP_TRY(hipGetLastError());
    return DQ_OK;
  }
};

struct Target {
  uint64_t prefix;  // the top `bits` bits of the target's key
  int64_t q;        // rank among the keys with this prefix
  int j;            // output index
};

// The values at the exact ranks of `tg`, into res[j].  Pass 0 (one prefix, D0 bits) has run: `h`
// holds its bins.  Histogram passes narrow every rank to a bin; a rank whose prefix holds one
// distinct key is decided by the prefix's min = max; once the selected bins are small (or hold
// at most half of the keys a pass reads) their keys are compacted, and when few enough sorted.
dq_status radix_select(Source src, Passer& ps, Pass p, std::vector<Target> tg, std::vector<double>& res) {
  constexpr int64_t kSortBudget = 1 << 20;
  hipStream_t st = ps.st;
  DevBuf<uint64_t> buf[2];
  DevBuf<uint8_t> tmp;
  DevBuf<int64_t> didx;
  DevBuf<double> dpick;
  int which = 0;
  std::vector<uint64_t> cur{0};  // the prefixes of this pass (sorted; pass 0: the empty prefix)
  while (true) {
    // each prefix's running bin counts (one pass over the bins; a bin-by-bin walk per rank cost
    // ~0.3 ms of host time for 201 ranks over 8,192 bins), then a binary search per rank
    const size_t nd = (size_t)1 << p.D;
    std::vector<int64_t> cum(ps.h.size());
    for (size_t a = 0; a < cur.size(); ++a) {
      int64_t run = 0;
      for (size_t d = 0; d < nd; ++d) cum[a * nd + d] = run += (int64_t)ps.h[a * nd + d];
    }
    // decided by min = max: the prefix holds one distinct key
    std::vector<Target> left;
    for (Target& t : tg) {
      const int a = (int)(std::lower_bound(cur.begin(), cur.end(), t.prefix) - cur.begin());
      if (p.minmax && ps.mmh[2 * a] == ps.mmh[2 * a + 1]) {
        res[t.j] = from_ordered(ps.mmh[2 * a]);
        continue;
      }
      const int64_t* c = cum.data() + (size_t)a * nd;
      const size_t d = (size_t)(std::upper_bound(c, c + nd, t.q) - c);  // first bin past rank q
      if (d == nd) return fail(DQ_ERR_STATE, "radix select lost a rank (counts changed under it)");
      const int64_t below = d ? c[d - 1] : 0;
      left.push_back(Target{(t.prefix << p.D) | (uint64_t)d, t.q - below, t.j});
    }
    tg.swap(left);
    const int bits = p.bits + p.D;
    if (tg.empty()) return DQ_OK;
    if (bits == 64) {  // every bit decided: the prefix IS the key
      for (const Target& t : tg) res[t.j] = from_ordered(t.prefix);
      return DQ_OK;
    }
    // the bins that now hold a rank, and their keys
    std::vector<std::pair<uint64_t, int64_t>> sel;  // (prefix, keys), ascending
    for (const Target& t : tg) sel.push_back({t.prefix, 0});
    std::sort(sel.begin(), sel.end());
    sel.erase(std::unique(sel.begin(), sel.end()), sel.end());
    int64_t T = 0;
    std::vector<uint32_t> mask(((size_t)(p.A << p.D) + 31) / 32, 0u);
    for (auto& s : sel) {
      const int a = (int)(std::lower_bound(cur.begin(), cur.end(), s.first >> p.D) - cur.begin());
      const uint32_t bin = ((uint32_t)a << p.D) | (uint32_t)(s.first & ((1ULL << p.D) - 1));
      s.second = (int64_t)ps.h[bin];
      mask[bin >> 5] |= 1u << (bin & 31);
      T += s.second;
    }
    const bool finish = T <= kSortBudget;
    if (finish || 2 * T <= src.M) {  // compact the selected bins' keys (into the buffer src is not)
      DevBuf<uint64_t>& dst = buf[which];
      HIP_TRY(dst.ensure((size_t)std::max<int64_t>(T, 1)));
      dq_status cs = ps.compact(src, p, mask, dst.p);
      if (cs != DQ_OK) return cs;
      Source next;
      next.type = kKeys;
      next.parts.push_back(Src{nullptr, dst.p, T, 0});
      next.cut(T);
      next.M = T;
      src = next;
      which ^= 1;
    }
    if (finish) {  // sort them; a target's key sits at (keys of the bins before its own) + q
      DevBuf<uint64_t>& sorted = buf[which];
      HIP_TRY(sorted.ensure((size_t)std::max<int64_t>(T, 1)));
      HIP_TRY(sort_keys(reinterpret_cast<const uint64_t*>(src.parts[0].values), sorted.p, (size_t)T, tmp, st));
      const int u = (int)tg.size();
      std::vector<int64_t> idx(u);
      for (int i = 0; i < u; ++i) {
        int64_t before = 0;
        for (const auto& s : sel) {
          if (s.first == tg[i].prefix) break;
          before += s.second;
        }
        idx[i] = before + tg[i].q;
      }
      HIP_TRY(didx.ensure(u));
      HIP_TRY(dpick.ensure(u));
      HIP_TRY(hipMemcpyAsync(didx.p, idx.data(), (size_t)u * 8, hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(select_pick, dim3((unsigned)((u + 255) / 256)), dim3(256), 0, st, sorted.p, didx.p,
                         (int64_t)u, dpick.p);
      HIP_TRY(hipGetLastError());
      std::vector<double> v(u);
      HIP_TRY(d2h(v.data(), dpick.p, (size_t)u * 8, st));  // idx and v die here
      for (int i = 0; i < u; ++i) res[tg[i].j] = v[i];
      return DQ_OK;
    }
    // the next pass: the selected bins' prefixes, as many digit bits as the bins allow
    cur.clear();
    for (const auto& s : sel) cur.push_back(s.first);
    const int A = (int)cur.size();
    int D = 1;
    while (D < 64 - bits && ((int64_t)A << (D + 1)) <= kSelBins) ++D;
    dq_status rs = ps.run(src, cur, bits, D, p);
    if (rs != DQ_OK) return rs;
  }
}

}  // namespace

namespace dq {
__global__ void dec_to_f64_kernel(const uint64_t* __restrict__ in, double* __restrict__ out,
                                  int64_t rows, int scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = dec_to_double(in[2 * i], (int64_t)in[2 * i + 1], scale);
}
}  // namespace dq

extern "C" dq_status dq_sorted_sample(int device, const dq_column* batches, int n_batches,
                                      int64_t head_values, int64_t max_values, double* out,
                                      int64_t* n_out, int64_t* count_out, void* hip_stream) {
  if (!n_out || !count_out || (n_batches > 0 && !batches) || n_batches < 0 || max_values < 2 ||
      head_values < 0)
    return fail(DQ_ERR_INVALID_ARGUMENT, "bad argument to dq_sorted_sample");
  hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
  HIP_TRY(hipSetDevice(device));
  int64_t rows = 0;
  const bool dec = n_batches > 0 && DQ_TYPE_ID(batches[0].type) == DQ_DECIMAL128;
  for (int b = 0; b < n_batches; ++b) {
    const dq_column& c = batches[b];
    if (!dec && (c.type == DQ_UTF8 || c.type == DQ_BOOL || c.type < DQ_BOOL || c.type > DQ_UTF8))
      return fail(DQ_ERR_WRONG_TYPE, "ApproxQuantile needs a numeric column");
    if (b && c.type != batches[0].type) return fail(DQ_ERR_WRONG_TYPE, "batches differ in type");
    if (c.length < 0 || (c.length > 0 && !c.values))
      return fail(DQ_ERR_INVALID_ARGUMENT, "batch %d has no values", b);
    rows += c.length;
  }
  *n_out = 0;
  *count_out = 0;
  if (rows == 0) return DQ_OK;
  // a decimal column enters as its values cast to double (StatefulApproxQuantile's DoubleType
  // input: Decimal.toDouble, correctly rounded, decimal.h), one device buffer per batch
  std::vector<dq_column> as_f64;
  std::vector<std::unique_ptr<DevBuf<double>>> f64_bufs;
  if (dec) {
    for (int b = 0; b < n_batches; ++b) {
      dq_column c = batches[b];
      f64_bufs.emplace_back(new DevBuf<double>());
      HIP_TRY(f64_bufs.back()->ensure((size_t)std::max<int64_t>(1, c.length)));
      if (c.length) {
        hipLaunchKernelGGL(dec_to_f64_kernel, dim3((unsigned)std::min<int64_t>((c.length + 255) / 256, 4096)),
                           dim3(256), 0, stream, static_cast<const uint64_t*>(c.values),
                           f64_bufs.back()->p, c.length, DQ_DECIMAL_SCALE(c.type));
        HIP_TRY(hipGetLastError());
      }
      c.type = DQ_FLOAT64;
      c.values = f64_bufs.back()->p;
      as_f64.push_back(c);
    }
    batches = as_f64.data();
  }
  // pass 0 over the columns: the count and the keys' top bits (through the engine's device cache:
  // buffers reused across columns, released on OOM)
  Source col;
  col.type = batches[0].type;
  for (int b = 0; b < n_batches; ++b)
    if (batches[b].length) col.parts.push_back(Src{batches[b].validity, batches[b].values, batches[b].length, 0});
  col.cut(rows);
  Passer ps;
  ps.st = stream;
  Pass p;
  constexpr int kD0 = 13;
  const int ty = batches[0].type;
  const bool integral = ty == DQ_INT8 || ty == DQ_INT16 || ty == DQ_INT32 || ty == DQ_INT64;
  dq_status st = ps.run(col, std::vector<uint64_t>{0}, 0, kD0, p, integral);
  if (st != DQ_OK) return st;
  unsigned long long count = 0;
  for (unsigned long long x : ps.h) count += x;
  col.M = (int64_t)count;
  *count_out = (int64_t)count;
  if (!count) return DQ_OK;
  const int64_t n = (int64_t)count <= std::max(head_values, max_values) ? (int64_t)count : max_values;
  *n_out = n;
  if (!out) return DQ_OK;  // size query only
  if (n == (int64_t)count || n > kSelMaxTargets) {  // every key, compacted and sorted
    DevBuf<uint64_t> keys, sorted;
    DevBuf<uint8_t> tmp;
    DevBuf<double> picks;
    HIP_TRY(keys.ensure((size_t)count));
    HIP_TRY(sorted.ensure((size_t)count));
    HIP_TRY(picks.ensure((size_t)n));
    const std::vector<uint32_t> all((1 << kD0) / 32, ~0u);  // (alive until the stream syncs below)
    st = ps.compact(col, p, all, keys.p);
    if (st != DQ_OK) return st;
    HIP_TRY(sort_keys(keys.p, sorted.p, (size_t)count, tmp, stream));
    if (n == (int64_t)count) {  // every value, sorted
      hipLaunchKernelGGL(keys_to_doubles, dim3((unsigned)std::min<int64_t>((n + 4095) / 4096, 4096)), dim3(256),
                         0, stream, sorted.p, n, picks.p);
      HIP_TRY(hipGetLastError());
      HIP_TRY(d2h(out, picks.p, (size_t)n * 8, stream));
    } else {  // many ranks: the picks of the sorted keys
      std::vector<int64_t> rank(n);
      for (int64_t j = 0; j < n; ++j) rank[j] = (int64_t)(((__int128)j * ((int64_t)count - 1)) / (n - 1));
      DevBuf<int64_t> didx;
      HIP_TRY(didx.ensure((size_t)n));
      HIP_TRY(hipMemcpyAsync(didx.p, rank.data(), (size_t)n * 8, hipMemcpyHostToDevice, stream));
      hipLaunchKernelGGL(select_pick, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                         sorted.p, didx.p, n, picks.p);
      HIP_TRY(hipGetLastError());
      HIP_TRY(d2h(out, picks.p, (size_t)n * 8, stream));  // rank dies here
    }
    return DQ_OK;
  }
  // a narrow integer column: the values at the ranks by dense counting (DQ_QUANTILE_DENSE=0: never)
  const char* dense_env = getenv("DQ_QUANTILE_DENSE");
  if (integral && !(dense_env && atoi(dense_env) == 0)) {
    const double dlo = from_ordered(ps.mmh[0]), dhi = from_ordered(ps.mmh[1]);
    const int64_t lo = dlo > -0x1p62 ? (int64_t)dlo : 0, hi = dhi < 0x1p62 ? (int64_t)dhi : 0;
    if (dlo > -0x1p62 && dhi < 0x1p62 && hi >= lo && (uint64_t)(hi - lo) < (uint64_t)kDenseQ) {
      const int nv = (int)(hi - lo) + 1;
      int dev = 0, cus = 0, lds_cap = 0;
      HIP_TRY(hipGetDevice(&dev));
      HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      HIP_TRY(hipDeviceGetAttribute(&lds_cap, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
      if ((int64_t)nv * 4 > lds_cap) goto radix;  // (a part with less LDS: the radix select)
      const int64_t G = std::max<int64_t>(1, std::min<int64_t>(cus, (rows + 4 * kDenseQThreads - 1) / (4 * kDenseQThreads)));
      HIP_TRY(ps.partial.ensure((size_t)G * nv));
      HIP_TRY(ps.hist.ensure(nv));
      HIP_TRY(hipMemsetAsync(ps.hist.p, 0, (size_t)nv * 8, stream));
      for (size_t i = 0; i < col.parts.size(); i += kMaxSrc) {  // (the launches add into one row set)
        Srcs ss;
        ss.n = (int)std::min<size_t>(kMaxSrc, col.parts.size() - i);
        for (int j = 0; j < ss.n; ++j) ss.s[j] = col.parts[i + j];
        auto go = [&](auto kernel) {
          hipLaunchKernelGGL(kernel, dim3((unsigned)G), dim3(kDenseQThreads), (size_t)nv * 4, stream, ss, lo, nv,
                             ps.partial.p);
        };
        switch (ty) {
          case DQ_INT8: go(rs_dense<DQ_INT8>); break;
          case DQ_INT16: go(rs_dense<DQ_INT16>); break;
          case DQ_INT32: go(rs_dense<DQ_INT32>); break;
          default: go(rs_dense<DQ_INT64>); break;
        }
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(rs_sum, dim3((unsigned)((nv + 255) / 256), (unsigned)((G + 31) / 32)), dim3(256), 0, stream,
                           ps.partial.p, G, nv, ps.hist.p);
        HIP_TRY(hipGetLastError());
      }
      std::vector<unsigned long long> cnt(nv);
      HIP_TRY(d2h(cnt.data(), ps.hist.p, (size_t)nv * 8, stream));
      std::vector<int64_t> cum(nv);
      int64_t run = 0;
      for (int i = 0; i < nv; ++i) cum[i] = run += (int64_t)cnt[i];
      if (run != (int64_t)count) return fail(DQ_ERR_STATE, "dense quantile counts %lld of %llu rows",
                                             (long long)run, (unsigned long long)count);
      for (int64_t j = 0; j < n; ++j) {
        const int64_t q = (int64_t)(((__int128)j * ((int64_t)count - 1)) / (n - 1));
        const int64_t i = std::upper_bound(cum.begin(), cum.end(), q) - cum.begin();
        out[j] = (double)(lo + i);
      }
      return DQ_OK;
    }
  }
radix:
  // the values at the ranks floor(j (count - 1) / (n - 1)), by radix select from pass 0
  std::vector<Target> tg(n);
  for (int64_t j = 0; j < n; ++j)
    tg[j] = Target{0, (int64_t)(((__int128)j * ((int64_t)count - 1)) / (n - 1)), (int)j};
  std::vector<double> res(n);
  st = radix_select(col, ps, p, std::move(tg), res);
  if (st != DQ_OK) return st;
  memcpy(out, res.data(), (size_t)n * 8);
  return DQ_OK;
}
