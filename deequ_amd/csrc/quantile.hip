// quantile.hip -- the device half of ApproxQuantile (ApproxQuantile.scala:41-104).
//
// The reference feeds every non-NULL value, as a double, into Spark's ApproximatePercentile
// (QuantileSummaries, Greenwald-Khanna with relativeError).  Here the values of all batches are
// gathered as doubles, sorted on the device (rocPRIM radix sort: the order is Java's
// Double.compare once NaNs are canonical, -0.0 before 0.0), and handed to the host as either every
// value (few enough that the host replays Spark's own insert + compress exactly) or values at
// evenly spaced exact ranks (a GK summary whose error is far inside relativeError).  The summary
// arithmetic -- insert, compress, merge, query -- is host code (deequ_amd/analyzers/quantile.py).
#include <hip/hip_runtime.h>

#include <cstring>  // rocprim headers use memset without including it

#include <rocprim/rocprim.hpp>

#include <vector>

#include "device_util.h"
#include "kernels.h"

using namespace dq;

namespace {

constexpr int kGatherThreads = 256;
constexpr int kGatherWaves = kGatherThreads / 64;
constexpr int kGatherRounds = 16;  // rows per thread per block step: 4096 rows a step

static_assert(kGatherRounds * kGatherWaves == 64, "one wave scans the step's counts");

// Non-NULL values of one batch -> doubles at out[*cursor ...] (order irrelevant: sorted next).
// A block step covers 4096 rows (round i: rows r0 + 256 i + tid, coalesced); the kept rows of a
// step are placed by one exclusive scan over its (round, wave) ballot counts and ONE cursor
// atomic per step -- one per wave (a same-address atomic every 64 rows) serialised the kernel.
__global__ void __launch_bounds__(kGatherThreads)
quantile_gather(int type, const uint8_t* __restrict__ valid, const void* __restrict__ values,
                int64_t rows, double* __restrict__ out, unsigned long long* __restrict__ cursor) {
  __shared__ uint32_t s_cnt[kGatherRounds * kGatherWaves];
  __shared__ unsigned long long s_base;
  const int tid = threadIdx.x, lane = (int)__lane_id(), wave = tid >> 6;
  const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;  // lanes below this one
  constexpr int64_t kStep = (int64_t)kGatherRounds * kGatherThreads;
  for (int64_t r0 = (int64_t)blockIdx.x * kStep; r0 < rows; r0 += (int64_t)gridDim.x * kStep) {
    double v[kGatherRounds];
    uint64_t m[kGatherRounds];
#pragma unroll
    for (int i = 0; i < kGatherRounds; ++i) {
      const int64_t r = r0 + (int64_t)i * kGatherThreads + tid;
      const bool keep = r < rows && bit1(valid, r);
      v[i] = keep ? load_f64(type, values, r) : 0.0;
      if (v[i] != v[i]) v[i] = __builtin_nan("");  // Double.compare: every NaN is the canonical one
      m[i] = __ballot(keep);
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
      if (lane == 0) s_base = base;
    }
    __syncthreads();
    const unsigned long long base = s_base;
#pragma unroll
    for (int i = 0; i < kGatherRounds; ++i)
      if ((m[i] >> lane) & 1u)
        out[base + s_cnt[i * kGatherWaves + wave] + __popcll(m[i] & lt)] = v[i];
    __syncthreads();  // s_cnt / s_base are rewritten by the next step
  }
}

// out[j] = sorted[floor(j * (count - 1) / (n - 1))], j < n: the min, the max and evenly spaced
// exact ranks between
__global__ void quantile_pick(const double* __restrict__ sorted, int64_t count, int64_t n,
                              double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t r = n > 1 ? (int64_t)(((__int128)j * (count - 1)) / (n - 1)) : 0;
  out[j] = sorted[r];
}

}  // namespace

extern "C" dq_status dq_sorted_sample(int device, const dq_column* batches, int n_batches,
                                      int64_t head_values, int64_t max_values, double* out,
                                      int64_t* n_out,
                                      int64_t* count_out, void* hip_stream) {
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
  DevBuf<double> keys, sorted, picks;
  DevBuf<unsigned long long> cur;
  DevBuf<uint8_t> tmp;
  HIP_TRY(keys.ensure((size_t)rows));
  HIP_TRY(sorted.ensure((size_t)rows));
  HIP_TRY(cur.ensure(1));
  HIP_TRY(hipMemsetAsync(cur.p, 0, 8, stream));
  double* kp = keys.p;
  unsigned long long* cp = cur.p;
  for (int b = 0; b < n_batches; ++b) {
    const dq_column& c = batches[b];
    if (!c.length) continue;
    const int64_t step = (int64_t)kGatherRounds * kGatherThreads;
    const int64_t blocks = std::min<int64_t>((c.length + step - 1) / step, 2048);
    hipLaunchKernelGGL(quantile_gather, dim3((unsigned)blocks), dim3(kGatherThreads), 0, stream,
                       c.type, c.validity, c.values, c.length, kp, cp);
    HIP_TRY(hipGetLastError());
  }
  unsigned long long count = 0;
  HIP_TRY(hipMemcpyAsync(&count, cp, 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  *count_out = (int64_t)count;
  if (!count) return DQ_OK;
  size_t tmp_bytes = 0;
  HIP_TRY(rocprim::radix_sort_keys(nullptr, tmp_bytes, kp, sorted.p, (size_t)count, 0, 64, stream));
  HIP_TRY(tmp.ensure(std::max<size_t>(tmp_bytes, 16)));
  HIP_TRY(rocprim::radix_sort_keys(tmp.p, tmp_bytes, kp, sorted.p, (size_t)count, 0, 64, stream));
  const int64_t n = (int64_t)count <= std::max(head_values, max_values) ? (int64_t)count : max_values;
  *n_out = n;
  if (!out) return DQ_OK;  // size query only
  if (n == (int64_t)count) {
    HIP_TRY(hipMemcpyAsync(out, sorted.p, (size_t)n * 8, hipMemcpyDeviceToHost, stream));
  } else {
    HIP_TRY(picks.ensure((size_t)n));
    hipLaunchKernelGGL(quantile_pick, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                       sorted.p, (int64_t)count, n, picks.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, picks.p, (size_t)n * 8, hipMemcpyDeviceToHost, stream));
  }
  HIP_TRY(hipStreamSynchronize(stream));
  return DQ_OK;
}
