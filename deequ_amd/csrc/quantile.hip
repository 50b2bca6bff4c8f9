// quantile.hip -- the device half of ApproxQuantile (ApproxQuantile.scala:41-104).
//
// The reference feeds every non-NULL value, as a double, into Spark's ApproximatePercentile
// (QuantileSummaries, Greenwald-Khanna with relativeError).  Here the values of all batches are
// gathered as order-preserving 64-bit keys (Java's Double.compare order as unsigned order: NaNs
// canonical and largest, -0.0 before 0.0) and handed to the host as either
//   * every value, sorted (rocPRIM radix sort) -- few enough that the host replays Spark's own
//     insert + compress exactly, or relativeError 0 (the exact summary); or
//   * the values at m evenly spaced exact ranks floor(j (n - 1) / (m - 1)) (a GK summary whose
//     error is far inside relativeError), found by a radix SELECT: a few histogram passes over the
//     keys narrow every rank to one bin, and only the bins that hold a rank are compacted and
//     sorted -- instead of sorting every value.
// The summary arithmetic -- insert, compress, merge, query -- is host code
// (deequ_amd/analyzers/quantile.py).
#include <hip/hip_runtime.h>

#include <cstring>  // rocprim headers use memset without including it

#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <vector>

#include "device_util.h"
#include "kernels.h"

using namespace dq;

namespace {

constexpr int kGatherThreads = 256;
constexpr int kGatherWaves = kGatherThreads / 64;
constexpr int kGatherRounds = 16;  // rows per thread per block step: 4096 rows a step
constexpr int64_t kGatherStep = (int64_t)kGatherRounds * kGatherThreads;

static_assert(kGatherRounds * kGatherWaves == 64, "one wave scans the step's counts");

// Double.compare order as unsigned order (the canonical NaN is the largest key)
DQ_HD uint64_t ordered_key(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  return (b >> 63) ? ~b : (b | (1ULL << 63));
}
DQ_HD double from_ordered(uint64_t k) {
  return __builtin_bit_cast(double, (k >> 63) ? (k & ~(1ULL << 63)) : ~k);
}

// A block step of 4096 items (round i: item base + 256 i + tid) keeps the items whose bit is set
// in keep[i]; their values land at out[*cursor ...] in (round, wave, lane) order of the step,
// placed by one exclusive scan over the step's 64 (round, wave) ballot counts and ONE cursor
// atomic per step (one atomic per wave on one address serialised the kernel).
struct StepPlacer {
  uint32_t* s_cnt;  // kGatherRounds * kGatherWaves
  unsigned long long* s_base;
  DQ_DEV void place(const bool (&keep)[kGatherRounds], const uint64_t (&v)[kGatherRounds],
                    uint64_t* __restrict__ out, unsigned long long* __restrict__ cursor) {
    const int tid = threadIdx.x, lane = (int)__lane_id(), wave = tid >> 6;
    const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;  // lanes below this one
    uint64_t m[kGatherRounds];
#pragma unroll
    for (int i = 0; i < kGatherRounds; ++i) {
      m[i] = __ballot(keep[i]);
      if (lane == 0) s_cnt[i * kGatherWaves + wave] = (uint32_t)__popcll(m[i]);
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the 64 (round, wave) counts, round-major
      const uint32_t c = s_cnt[tid];
      uint32_t x = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
      }
      const uint32_t total = __shfl(x, 63);
      unsigned long long base = 0;
      if (lane == 63 && total) base = atomicAdd(cursor, (unsigned long long)total);
      base = __shfl(base, 63);
      s_cnt[tid] = x - c;
      if (lane == 0) *s_base = base;
    }
    __syncthreads();
    const unsigned long long base = *s_base;
#pragma unroll
    for (int i = 0; i < kGatherRounds; ++i)
      if ((m[i] >> lane) & 1u) out[base + s_cnt[i * kGatherWaves + wave] + __popcll(m[i] & lt)] = v[i];
    __syncthreads();  // s_cnt / s_base are rewritten by the next step
  }
};

// Non-NULL values of one batch -> ordered keys at out[*cursor ...] (order irrelevant).
__global__ void __launch_bounds__(kGatherThreads)
quantile_gather(int type, const uint8_t* __restrict__ valid, const void* __restrict__ values,
                int64_t rows, uint64_t* __restrict__ out, unsigned long long* __restrict__ cursor) {
  __shared__ uint32_t s_cnt[kGatherRounds * kGatherWaves];
  __shared__ unsigned long long s_base;
  StepPlacer pl{s_cnt, &s_base};
  for (int64_t r0 = (int64_t)blockIdx.x * kGatherStep; r0 < rows; r0 += (int64_t)gridDim.x * kGatherStep) {
    bool keep[kGatherRounds];
    uint64_t v[kGatherRounds];
#pragma unroll
    for (int i = 0; i < kGatherRounds; ++i) {
      const int64_t r = r0 + (int64_t)i * kGatherThreads + threadIdx.x;
      keep[i] = r < rows && bit1(valid, r);
      double d = keep[i] ? load_f64(type, values, r) : 0.0;
      if (d != d) d = __builtin_nan("");  // Double.compare: every NaN is the canonical one
      v[i] = ordered_key(d);
    }
    pl.place(keep, v, out, cursor);
  }
}

// The first radix pass, fused into the read of the columns: a histogram of the ordered keys' top
// kQ0Bits bits (no key is written; the keys of the bins that hold a rank are gathered afterwards by
// quantile_compact0, so the column is read twice and only those keys are written).
constexpr int kQ0Bits = 13;
constexpr int kQ0Bins = 1 << kQ0Bits;

__global__ void __launch_bounds__(256)
quantile_hist0(int type, const uint8_t* __restrict__ valid, const void* __restrict__ values,
               int64_t rows, uint32_t* __restrict__ partial) {
  __shared__ uint32_t s_hist[kQ0Bins];
  for (int i = threadIdx.x; i < kQ0Bins; i += 256) s_hist[i] = 0;
  __syncthreads();
  constexpr int kU = 8;  // rows per thread per step, all loads in flight before the first count
  for (int64_t i0 = (int64_t)blockIdx.x * 256 * kU; i0 < rows; i0 += (int64_t)gridDim.x * 256 * kU) {
    uint64_t k[kU];
    bool ok[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t r = i0 + (int64_t)u * 256 + threadIdx.x;
      ok[u] = r < rows && bit1(valid, r);
      double d = ok[u] ? load_f64(type, values, r) : 0.0;
      if (d != d) d = __builtin_nan("");
      k[u] = ordered_key(d);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (ok[u]) atomicAdd(&s_hist[k[u] >> (64 - kQ0Bits)], 1u);
  }
  __syncthreads();
  // the block's counts as one coalesced row of partials (a global atomic per bin and block was
  // millions of atomics on 8192 addresses)
  uint32_t* row = partial + (size_t)blockIdx.x * kQ0Bins;
  for (int i = threadIdx.x; i < kQ0Bins; i += 256) row[i] = s_hist[i];
}

// hist[bin] += the blocks' partial counts of the bin (one thread per bin, rows read coalesced)
__global__ void __launch_bounds__(256)
quantile_hist0_sum(const uint32_t* __restrict__ partial, int blocks, unsigned long long* __restrict__ hist) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= kQ0Bins) return;
  unsigned long long t = 0;
  for (int b = 0; b < blocks; ++b) t += partial[(size_t)b * kQ0Bins + i];
  hist[i] += t;
}

// The non-NULL values of one batch whose key's top kQ0Bits bits are a bin set in `bins` (a
// kQ0Bins-bit mask) -> ordered keys at out[*cursor ...] (order irrelevant).
__global__ void __launch_bounds__(kGatherThreads)
quantile_compact0(int type, const uint8_t* __restrict__ valid, const void* __restrict__ values,
                  int64_t rows, const uint32_t* __restrict__ bins, uint64_t* __restrict__ out,
                  unsigned long long* __restrict__ cursor) {
  __shared__ uint32_t s_bins[kQ0Bins / 32];
  __shared__ uint32_t s_cnt[kGatherRounds * kGatherWaves];
  __shared__ unsigned long long s_base;
  for (int i = threadIdx.x; i < kQ0Bins / 32; i += kGatherThreads) s_bins[i] = bins[i];
  __syncthreads();
  StepPlacer pl{s_cnt, &s_base};
  for (int64_t r0 = (int64_t)blockIdx.x * kGatherStep; r0 < rows; r0 += (int64_t)gridDim.x * kGatherStep) {
    bool keep[kGatherRounds];
    uint64_t v[kGatherRounds];
#pragma unroll
    for (int i = 0; i < kGatherRounds; ++i) {
      const int64_t r = r0 + (int64_t)i * kGatherThreads + threadIdx.x;
      const bool ok = r < rows && bit1(valid, r);
      double d = ok ? load_f64(type, values, r) : 0.0;
      if (d != d) d = __builtin_nan("");
      v[i] = ordered_key(d);
      const uint32_t b = (uint32_t)(v[i] >> (64 - kQ0Bits));
      keep[i] = ok && ((s_bins[b >> 5] >> (b & 31)) & 1u);
    }
    pl.place(keep, v, out, cursor);
  }
}

// ---- radix select -----------------------------------------------------------------------------
// A pass counts the keys whose top `bits` bits equal one of the A active prefixes (sorted, unique)
// by their next D bits: hist[a << D | digit], A << D <= kSelBins, privatised in LDS per block.
constexpr int kSelBins = 8192;  // 32 KB of LDS counters (+ 16 KB of prefixes at most)
constexpr int kSelMaxTargets = 2048;
// passes whose prefixes are at most kMapBits long find a key's prefix through a direct LDS map
// (prefix -> active index, 16 KB) instead of a binary search over the prefixes
constexpr int kMapBits = 13;

DQ_DEV int find_prefix(const uint64_t* act, int A, uint64_t p) {
  int lo = 0, hi = A;  // first index with act[i] >= p
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (act[mid] < p) lo = mid + 1;
    else hi = mid;
  }
  return lo < A && act[lo] == p ? lo : -1;
}

// The active index of every prefix of `bits` <= kMapBits bits (-1: not active), in LDS.
DQ_DEV void build_prefix_map(const uint64_t* act, int A, int bits, int16_t* map) {
  for (int i = threadIdx.x; i < (1 << bits); i += blockDim.x) map[i] = -1;
  __syncthreads();
  for (int i = threadIdx.x; i < A; i += blockDim.x) map[act[i]] = (int16_t)i;
  __syncthreads();
}

__global__ void __launch_bounds__(256)
select_hist(const uint64_t* __restrict__ keys, int64_t n, const uint64_t* __restrict__ active, int A,
            int bits, int D, unsigned long long* __restrict__ hist) {
  extern __shared__ uint64_t sel_lds[];
  uint64_t* s_act = sel_lds;                                            // A
  unsigned int* s_hist = reinterpret_cast<unsigned int*>(sel_lds + A);  // A << D
  const int nb = A << D;
  int16_t* s_map = reinterpret_cast<int16_t*>(s_hist + nb);  // 1 << bits, when bits <= kMapBits
  const bool mapped = bits > 0 && bits <= kMapBits;
  for (int i = threadIdx.x; i < A; i += 256) s_act[i] = active[i];
  for (int i = threadIdx.x; i < nb; i += 256) s_hist[i] = 0;
  __syncthreads();
  if (mapped) build_prefix_map(s_act, A, bits, s_map);
  // 8 keys per thread per step, all loads in flight before the first is counted
  constexpr int kU = 8;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 * kU; i0 < n; i0 += (int64_t)gridDim.x * 256 * kU) {
    uint64_t kk[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + (int64_t)u * 256 + threadIdx.x;
      kk[u] = i < n ? keys[i] : 0ULL;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (i0 + (int64_t)u * 256 + threadIdx.x >= n) continue;
      const uint64_t k = kk[u];
      int a = 0;
      if (bits) {
        a = mapped ? (int)s_map[k >> (64 - bits)] : find_prefix(s_act, A, k >> (64 - bits));
        if (a < 0) continue;
      }
      const uint32_t d = (uint32_t)((k << bits) >> (64 - D));
      atomicAdd(&s_hist[(a << D) | (int)d], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += 256)
    if (s_hist[i]) atomicAdd(&hist[i], (unsigned long long)s_hist[i]);  // (u64: a bin may pass 2^32 keys)
}

// The keys whose top `bits` bits are one of the A prefixes -> out[*cursor ...].
__global__ void __launch_bounds__(kGatherThreads)
select_compact(const uint64_t* __restrict__ keys, int64_t n, const uint64_t* __restrict__ active,
               int A, int bits, uint64_t* __restrict__ out, unsigned long long* __restrict__ cursor) {
  extern __shared__ uint64_t sel_lds[];
  __shared__ uint32_t s_cnt[kGatherRounds * kGatherWaves];
  __shared__ unsigned long long s_base;
  int16_t* s_map = reinterpret_cast<int16_t*>(sel_lds + A);  // 1 << bits, when bits <= kMapBits
  const bool mapped = bits <= kMapBits;
  for (int i = threadIdx.x; i < A; i += kGatherThreads) sel_lds[i] = active[i];
  __syncthreads();
  if (mapped) build_prefix_map(sel_lds, A, bits, s_map);
  StepPlacer pl{s_cnt, &s_base};
  for (int64_t i0 = (int64_t)blockIdx.x * kGatherStep; i0 < n; i0 += (int64_t)gridDim.x * kGatherStep) {
    bool keep[kGatherRounds];
    uint64_t v[kGatherRounds];
#pragma unroll
    for (int r = 0; r < kGatherRounds; ++r) {
      const int64_t i = i0 + (int64_t)r * kGatherThreads + threadIdx.x;
      v[r] = i < n ? keys[i] : 0ULL;
      keep[r] = i < n && (mapped ? s_map[v[r] >> (64 - bits)] >= 0
                                 : find_prefix(sel_lds, A, v[r] >> (64 - bits)) >= 0);
    }
    pl.place(keep, v, out, cursor);
  }
}

// out[j] = from_ordered(keys[idx[j]])
__global__ void select_pick(const uint64_t* __restrict__ keys, const int64_t* __restrict__ idx,
                            int64_t m, double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < m) out[j] = from_ordered(keys[idx[j]]);
}

// out[j] = from_ordered(sorted[j])
__global__ void keys_to_doubles(const uint64_t* __restrict__ sorted, int64_t n, double* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
    out[j] = from_ordered(sorted[j]);
}

unsigned grid_of(int64_t n, int64_t per_block, int64_t cap) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + per_block - 1) / per_block, cap));
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

// The values at the exact ranks rank[0..m) (ascending) of the n keys at `keys`, into out_dev[m]
// (doubles).  Histogram passes narrow every rank to a bin of the keys' top bits; once the bins
// that hold a rank hold few keys (or every bit is decided) those keys are compacted and sorted.
struct Target {
  uint64_t prefix;  // the top `bits` bits of the target's key
  int64_t q;        // rank among the keys with this prefix
};

// `keys` (n of them) are exactly the keys whose top `bits0` bits are one of the targets' prefixes
// (every key when bits0 = 0).
dq_status radix_select(const uint64_t* keys, int64_t n, std::vector<Target> tg, int bits0,
                       double* out_dev, hipStream_t stream) {
  const int m = (int)tg.size();
  // keys sorted at the end: always when this few; and up to kStallBudget when a pass stopped
  // narrowing (a bin of one repeated value -- integers of a narrow range -- never shrinks: more
  // passes over it only spend bits)
  constexpr int64_t kSortBudget = 1 << 24, kStallBudget = 1 << 26;
  int64_t T_prev = n;
  DevBuf<uint64_t> buf[2], act;
  DevBuf<unsigned long long> hist;
  DevBuf<unsigned long long> cur;
  DevBuf<uint8_t> tmp;
  DevBuf<int64_t> didx;
  HIP_TRY(cur.ensure(1));
  const uint64_t* src = keys;
  int64_t M = n;
  int which = 0;
  int bits = bits0;
  std::vector<uint64_t> prefixes, sp;  // (alive until the copies from them have run)
  std::vector<unsigned long long> h;
  while (true) {
    prefixes.clear();
    for (const Target& t : tg) prefixes.push_back(t.prefix);
    std::sort(prefixes.begin(), prefixes.end());
    prefixes.erase(std::unique(prefixes.begin(), prefixes.end()), prefixes.end());
    const int A = (int)prefixes.size();
    int D = 1;
    while (D < 64 - bits && ((int64_t)A << (D + 1)) <= kSelBins) ++D;
    const int nb = A << D;
    HIP_TRY(act.ensure(A));
    HIP_TRY(hipMemcpyAsync(act.p, prefixes.data(), A * 8, hipMemcpyHostToDevice, stream));
    HIP_TRY(hist.ensure(nb));
    HIP_TRY(hipMemsetAsync(hist.p, 0, (size_t)nb * 8, stream));
    const size_t lds = (size_t)A * 8 + (size_t)nb * 4 + (bits && bits <= kMapBits ? 2u << bits : 0u);
    // (a few blocks per CU: each flushes up to kSelBins counters)
    hipLaunchKernelGGL(select_hist, dim3(grid_of(M, 256 * 64, 1024)), dim3(256), lds, stream, src,
                       M, act.p, A, bits, D, hist.p);
    HIP_TRY(hipGetLastError());
    h.resize(nb);
    HIP_TRY(hipMemcpyAsync(h.data(), hist.p, (size_t)nb * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    // every target: the bin of its prefix that holds its rank
    for (Target& t : tg) {
      const int a = (int)(std::lower_bound(prefixes.begin(), prefixes.end(), t.prefix) - prefixes.begin());
      int64_t below = 0;
      int d = 0;
      for (; d < (1 << D); ++d) {
        const int64_t c = h[((size_t)a << D) | d];
        if (t.q < below + c) break;
        below += c;
      }
      if (d == (1 << D)) return fail(DQ_ERR_STATE, "radix select lost a rank (counts changed under it)");
      t.prefix = (t.prefix << D) | (uint64_t)d;
      t.q -= below;
    }
    const int nbits = bits + D;
    // the bins that now hold a rank, and the keys in them
    std::vector<std::pair<uint64_t, int64_t>> sel;  // (prefix, keys), ascending
    for (const Target& t : tg) sel.push_back({t.prefix, 0});
    std::sort(sel.begin(), sel.end());
    sel.erase(std::unique(sel.begin(), sel.end()), sel.end());
    int64_t T = 0;
    for (auto& s : sel) {
      const uint64_t parent = s.first >> D;  // (0, the only prefix, on the first pass)
      const int a = (int)(std::lower_bound(prefixes.begin(), prefixes.end(), parent) - prefixes.begin());
      s.second = h[((size_t)a << D) | (s.first & ((1ULL << D) - 1))];
      T += s.second;
    }
    bits = nbits;
    if (bits == 64) {  // every bit decided: the prefix IS the key
      std::vector<double> v(m);
      for (int j = 0; j < m; ++j) v[j] = from_ordered(tg[j].prefix);
      HIP_TRY(hipMemcpyAsync(out_dev, v.data(), (size_t)m * 8, hipMemcpyHostToDevice, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      return DQ_OK;
    }
    const bool finish = T <= kSortBudget || (T <= kStallBudget && 2 * T > T_prev);
    T_prev = T;
    if (!finish && T > M / 2) continue;  // narrowing did not pay for a copy yet
    // compact the selected bins' keys (into the buffer src is not)
    sp.resize(sel.size());
    for (size_t i = 0; i < sel.size(); ++i) sp[i] = sel[i].first;
    const int S = (int)sp.size();
    HIP_TRY(act.ensure(S));
    HIP_TRY(hipMemcpyAsync(act.p, sp.data(), (size_t)S * 8, hipMemcpyHostToDevice, stream));
    DevBuf<uint64_t>& dst = buf[which];
    HIP_TRY(dst.ensure((size_t)std::max<int64_t>(T, 1)));
    HIP_TRY(hipMemsetAsync(cur.p, 0, 8, stream));
    hipLaunchKernelGGL(select_compact, dim3(grid_of(M, kGatherStep, 2048)), dim3(kGatherThreads),
                       (size_t)S * 8 + (bits <= kMapBits ? 2u << bits : 0u), stream, src, M, act.p, S,
                       bits, dst.p, cur.p);
    HIP_TRY(hipGetLastError());
    src = dst.p;
    M = T;
    which ^= 1;
    if (!finish) continue;
    // sort the compacted keys; a target's key sits at (keys of the bins before its own) + q
    DevBuf<uint64_t>& sorted = buf[which];
    HIP_TRY(sorted.ensure((size_t)std::max<int64_t>(T, 1)));
    HIP_TRY(sort_keys(src, sorted.p, (size_t)T, tmp, stream));
    std::vector<int64_t> idx(m);
    for (int j = 0; j < m; ++j) {
      int64_t before = 0;
      for (const auto& s : sel) {
        if (s.first == tg[j].prefix) break;
        before += s.second;
      }
      idx[j] = before + tg[j].q;
    }
    HIP_TRY(didx.ensure(m));
    HIP_TRY(hipMemcpyAsync(didx.p, idx.data(), (size_t)m * 8, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(select_pick, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream,
                       sorted.p, didx.p, (int64_t)m, out_dev);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(stream));  // the host vectors above die here
    return DQ_OK;
  }
}

}  // namespace

extern "C" dq_status dq_sorted_sample(int device, const dq_column* batches, int n_batches,
                                      int64_t head_values, int64_t max_values, double* out,
                                      int64_t* n_out, int64_t* count_out, void* hip_stream) {
  if (!n_out || !count_out || (n_batches > 0 && !batches) || n_batches < 0 || max_values < 2 ||
      head_values < 0)
    return fail(DQ_ERR_INVALID_ARGUMENT, "bad argument to dq_sorted_sample");
  hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
  HIP_TRY(hipSetDevice(device));
  int64_t rows = 0;
  for (int b = 0; b < n_batches; ++b) {
    const dq_column& c = batches[b];
    if (c.type == DQ_UTF8 || c.type == DQ_BOOL || c.type < DQ_BOOL || c.type > DQ_UTF8)
      return fail(DQ_ERR_WRONG_TYPE, "ApproxQuantile needs a numeric column");
    if (b && c.type != batches[0].type) return fail(DQ_ERR_WRONG_TYPE, "batches differ in type");
    if (c.length < 0 || (c.length > 0 && !c.values))
      return fail(DQ_ERR_INVALID_ARGUMENT, "batch %d has no values", b);
    rows += c.length;
  }
  *n_out = 0;
  *count_out = 0;
  if (rows == 0) return DQ_OK;
  // through the engine's device cache (dev_alloc): reused across columns, released on OOM
  DevBuf<uint64_t> keys, sorted;
  DevBuf<double> picks;
  DevBuf<unsigned long long> cur, hist;
  DevBuf<uint32_t> partial, mask;
  DevBuf<uint8_t> tmp;
  // pass 1: the count and the keys' top-kQ0Bits histogram, straight from the columns
  constexpr int kHistBlocks = 512;
  HIP_TRY(hist.ensure(kQ0Bins));
  HIP_TRY(partial.ensure((size_t)kHistBlocks * kQ0Bins));
  HIP_TRY(hipMemsetAsync(hist.p, 0, (size_t)kQ0Bins * 8, stream));
  for (int b = 0; b < n_batches; ++b) {
    const dq_column& c = batches[b];
    if (!c.length) continue;
    const unsigned g = grid_of(c.length, 256 * 8 * 4, kHistBlocks);
    hipLaunchKernelGGL(quantile_hist0, dim3(g), dim3(256), 0, stream, c.type, c.validity, c.values,
                       c.length, partial.p);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(quantile_hist0_sum, dim3(kQ0Bins / 256), dim3(256), 0, stream, partial.p, (int)g,
                       hist.p);
    HIP_TRY(hipGetLastError());
  }
  std::vector<unsigned long long> h0(kQ0Bins);
  HIP_TRY(hipMemcpyAsync(h0.data(), hist.p, (size_t)kQ0Bins * 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  unsigned long long count = 0;
  for (unsigned long long x : h0) count += x;
  *count_out = (int64_t)count;
  if (!count) return DQ_OK;
  const int64_t n = (int64_t)count <= std::max(head_values, max_values) ? (int64_t)count : max_values;
  *n_out = n;
  if (!out) return DQ_OK;  // size query only
  HIP_TRY(picks.ensure((size_t)n));
  HIP_TRY(cur.ensure(1));
  HIP_TRY(hipMemsetAsync(cur.p, 0, 8, stream));
  if (n == (int64_t)count || n > kSelMaxTargets) {  // every key, gathered and sorted
    HIP_TRY(keys.ensure((size_t)count));
    for (int b = 0; b < n_batches; ++b) {
      const dq_column& c = batches[b];
      if (!c.length) continue;
      hipLaunchKernelGGL(quantile_gather, dim3(grid_of(c.length, kGatherStep, 2048)),
                         dim3(kGatherThreads), 0, stream, c.type, c.validity, c.values, c.length,
                         keys.p, cur.p);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(sorted.ensure((size_t)count));
    HIP_TRY(sort_keys(keys.p, sorted.p, (size_t)count, tmp, stream));
    if (n == (int64_t)count) {  // every value, sorted
      hipLaunchKernelGGL(keys_to_doubles, dim3(grid_of(n, 256 * 16, 4096)), dim3(256), 0, stream,
                         sorted.p, n, picks.p);
      HIP_TRY(hipGetLastError());
    } else {  // many ranks: the picks of the sorted keys
      std::vector<int64_t> rank(n);
      for (int64_t j = 0; j < n; ++j) rank[j] = (int64_t)(((__int128)j * ((int64_t)count - 1)) / (n - 1));
      DevBuf<int64_t> didx;
      HIP_TRY(didx.ensure((size_t)n));
      HIP_TRY(hipMemcpyAsync(didx.p, rank.data(), (size_t)n * 8, hipMemcpyHostToDevice, stream));
      hipLaunchKernelGGL(select_pick, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                         sorted.p, didx.p, n, picks.p);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipStreamSynchronize(stream));  // rank dies here
    }
  } else {  // the values at the ranks floor(j (count - 1) / (n - 1)), by radix select
    // every rank's bin of pass 1 (ranks ascend, so one sweep), and the bins' keys gathered
    std::vector<Target> tg(n);
    std::vector<uint32_t> bm(kQ0Bins / 32, 0u);
    int64_t below = 0, T = 0;
    int d = 0;
    for (int64_t j = 0; j < n; ++j) {
      const int64_t r = (int64_t)(((__int128)j * ((int64_t)count - 1)) / (n - 1));
      while (r >= below + (int64_t)h0[d]) below += (int64_t)h0[d++];
      tg[j] = Target{(uint64_t)d, r - below};
      if (!((bm[d >> 5] >> (d & 31)) & 1u)) {
        bm[d >> 5] |= 1u << (d & 31);
        T += (int64_t)h0[d];
      }
    }
    HIP_TRY(keys.ensure((size_t)T));
    HIP_TRY(mask.ensure(kQ0Bins / 32));
    HIP_TRY(hipMemcpyAsync(mask.p, bm.data(), (kQ0Bins / 32) * 4, hipMemcpyHostToDevice, stream));
    for (int b = 0; b < n_batches; ++b) {
      const dq_column& c = batches[b];
      if (!c.length) continue;
      hipLaunchKernelGGL(quantile_compact0, dim3(grid_of(c.length, kGatherStep, 2048)),
                         dim3(kGatherThreads), 0, stream, c.type, c.validity, c.values, c.length,
                         mask.p, keys.p, cur.p);
      HIP_TRY(hipGetLastError());
    }
    const dq_status st = radix_select(keys.p, T, std::move(tg), kQ0Bits, picks.p, stream);
    if (st != DQ_OK) return st;
  }
  HIP_TRY(hipMemcpyAsync(out, picks.p, (size_t)n * 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  return DQ_OK;
}
