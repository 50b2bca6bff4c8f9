// cast.hip -- Spark 2.2 Cast(StringType -> LongType | DoubleType) of a utf8 column on the device:
// the ColumnProfiler's second pass casts the string columns its first pass inferred Integral or
// Fractional (ColumnProfiler.scala:311-320 castColumn, 389-405 castNumericStringColumns) before
// Minimum / Maximum / Mean / StandardDeviation / Sum / ApproxQuantiles run over them.
//
// One thread per 8 rows, so every thread writes one whole validity byte (LSB-first).
//   LongType:   UTF8String.toLong (Spark 2.2): optional sign, digits, optionally '.' and digits
//               (truncated); no whitespace; overflow or any other byte -> NULL.
//   DoubleType: java.lang.Double.parseDouble (Cast: `s.toString.toDouble`, NumberFormatException ->
//               NULL) over decimal strings: bytes <= ' ' trimmed at both ends, optional sign,
//               digits with at most one '.', at least one digit.  Converted exactly (one correctly
//               rounded multiply or divide by an exact power of ten: <= 19 significant digits,
//               value digits <= 2^53, |exponent| <= 22).  A string parseDouble would read but this
//               path cannot convert exactly -- exponents, "NaN", "Infinity", hex, a 'd'/'f'
//               suffix, more digits -- is counted in *n_unsupported and left NULL; the caller fails
//               loudly on a non-zero count rather than guess.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "kernels.h"

namespace dq {
namespace {

constexpr int kCastThreads = 256;

__device__ bool spark_to_long(const uint8_t* s, int32_t n, int64_t& out) {
  if (n == 0) return false;
  int32_t i = 0;
  const bool neg = s[0] == '-';
  if (neg || s[0] == '+') {
    if (n == 1) return false;
    i = 1;
  }
  const int64_t stop = INT64_MIN / 10;
  int64_t r = 0;  // accumulated negatively (INT64_MIN has no positive counterpart)
  for (; i < n; ++i) {
    const uint8_t b = s[i];
    if (b == '.') {
      ++i;
      break;
    }
    if (b < '0' || b > '9') return false;
    if (r < stop) return false;
    r = r * 10 - (int64_t)(b - '0');
    if (r > 0) return false;
  }
  for (; i < n; ++i)
    if (s[i] < '0' || s[i] > '9') return false;
  if (!neg) {
    if (r == INT64_MIN) return false;
    r = -r;
  }
  out = r;
  return true;
}

__device__ double pow10_exact(int e) {  // 10^e, exact in fp64 for 0 <= e <= 22
  double p = 1.0;
  for (int k = 0; k < e; ++k) p *= 10.0;
  return p;
}

// 0 = NULL (NumberFormatException), 1 = value, 2 = readable by parseDouble but not converted here
__device__ int java_parse_double(const uint8_t* s, int32_t n, double& out) {
  int32_t a = 0, b = n;
  while (a < b && s[a] <= ' ') ++a;
  while (b > a && s[b - 1] <= ' ') --b;
  if (a == b) return 0;
  bool neg = false;
  if (s[a] == '-' || s[a] == '+') {
    neg = s[a] == '-';
    ++a;
  }
  uint64_t w = 0;
  int sig = 0, e10 = 0, digits = 0;
  bool dot = false, lost = false;
  for (int32_t i = a; i < b; ++i) {
    const uint8_t c = s[i];
    if (c == '.') {
      if (dot) return 0;
      dot = true;
      continue;
    }
    if (c >= '0' && c <= '9') {
      ++digits;
      if (w == 0 && c == '0') {  // leading zeros: only the exponent moves
        if (dot) --e10;
        continue;
      }
      if (sig < 19) {
        w = w * 10 + (uint64_t)(c - '0');
        ++sig;
        if (dot) --e10;
      } else {
        if (c != '0') lost = true;  // a digit beyond 19 significant ones
        if (!dot) ++e10;
      }
      continue;
    }
    // letters parseDouble may accept (exponent, NaN, Infinity, hex, type suffix)
    if (c == 'e' || c == 'E' || c == 'N' || c == 'I' || c == 'x' || c == 'X' || c == 'p' ||
        c == 'P' || c == 'd' || c == 'D' || c == 'f' || c == 'F')
      return 2;
    return 0;
  }
  if (digits == 0) return 0;
  if (lost) return 2;
  if (w == 0) {
    out = neg ? -0.0 : 0.0;
    return 1;
  }
  // trailing zeros of w move into the exponent (keeps w small for the exact path)
  while (e10 < 0 && w % 10 == 0) {
    w /= 10;
    ++e10;
  }
  while (e10 > 22 && w <= (1ULL << 53) / 10) {
    w *= 10;
    --e10;
  }
  if (w > (1ULL << 53) || e10 > 22 || e10 < -22) return 2;
  const double x = (double)w;  // exact
  double v = e10 >= 0 ? x * pow10_exact(e10) : x / pow10_exact(-e10);
  out = neg ? -v : v;
  return 1;
}

__global__ void __launch_bounds__(kCastThreads) cast_utf8_kernel(
    const int32_t* __restrict__ off, const uint8_t* __restrict__ data,
    const uint8_t* __restrict__ valid, int64_t n, int to_type, void* __restrict__ values,
    uint8_t* __restrict__ validity_out, unsigned long long* __restrict__ n_unsupported) {
  const int64_t byte = (int64_t)blockIdx.x * kCastThreads + threadIdx.x;
  const int64_t r0 = byte * 8;
  if (r0 >= n) return;
  uint32_t vbits = 0, bad = 0;
  for (int k = 0; k < 8 && r0 + k < n; ++k) {
    const int64_t r = r0 + k;
    bool ok = false;
    if (!valid || ((valid[r >> 3] >> (r & 7)) & 1u)) {
      const int32_t s = off[r], len = off[r + 1] - s;
      if (to_type == DQ_INT64) {
        int64_t v = 0;
        ok = spark_to_long(data + s, len, v);
        static_cast<int64_t*>(values)[r] = ok ? v : 0;
      } else {
        double v = 0.0;
        const int res = java_parse_double(data + s, len, v);
        ok = res == 1;
        bad += res == 2;
        static_cast<double*>(values)[r] = ok ? v : 0.0;
      }
    } else if (to_type == DQ_INT64) {
      static_cast<int64_t*>(values)[r] = 0;
    } else {
      static_cast<double*>(values)[r] = 0.0;
    }
    vbits |= (ok ? 1u : 0u) << k;
  }
  validity_out[byte] = (uint8_t)vbits;
  if (bad) atomicAdd(n_unsupported, (unsigned long long)bad);
}

// Arrow bitmap at bit offset `bit` -> LSB-first bitmap at bit 0 (one thread per output byte).
// Reads only bytes that hold bits of rows [bit, bit + rows).
__global__ void __launch_bounds__(kCastThreads)
bitmap_rebase_kernel(const uint8_t* __restrict__ src, int64_t bit, int64_t rows,
                     uint8_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * kCastThreads + threadIdx.x;
  const int64_t n_out = (rows + 7) / 8;
  if (i >= n_out) return;
  const int64_t last_src = (bit + rows - 1) / 8;  // last source byte holding a row's bit
  const int64_t j = bit / 8 + i;
  const uint32_t sh = (uint32_t)(bit & 7);
  uint32_t v = src[j] >> sh;
  if (sh && j + 1 <= last_src) v |= (uint32_t)src[j + 1] << (8 - sh);
  dst[i] = (uint8_t)v;
}

}  // namespace

hipError_t launch_bitmap_rebase(const uint8_t* src, int64_t bit, int64_t rows, uint8_t* dst,
                                hipStream_t stream) {
  const int64_t n_out = (rows + 7) / 8;
  if (n_out <= 0) return hipSuccess;
  hipLaunchKernelGGL(bitmap_rebase_kernel, dim3((unsigned)((n_out + kCastThreads - 1) / kCastThreads)),
                     dim3(kCastThreads), 0, stream, src, bit, rows, dst);
  return hipGetLastError();
}

}  // namespace dq

using namespace dq;

extern "C" dq_status dq_cast_utf8(const dq_column* in, int to_type, void* values_out,
                                  uint8_t* validity_out, int64_t* n_unsupported, void* hip_stream) {
  if (!in || !n_unsupported) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (in->type != DQ_UTF8) return fail(DQ_ERR_WRONG_TYPE, "dq_cast_utf8 casts a utf8 column");
  if (to_type != DQ_INT64 && to_type != DQ_FLOAT64)
    return fail(DQ_ERR_UNSUPPORTED, "dq_cast_utf8 casts to int64 or float64 only");
  *n_unsupported = 0;
  if (in->length == 0) return DQ_OK;
  if (!in->values || !in->data || !values_out || !validity_out)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null column buffers");
  hipStream_t st = reinterpret_cast<hipStream_t>(hip_stream);
  unsigned long long* cnt = nullptr;
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&cnt), sizeof(*cnt), st));
  HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(*cnt), st));
  const int64_t bytes = (in->length + 7) / 8;
  const unsigned grid = (unsigned)((bytes + kCastThreads - 1) / kCastThreads);
  hipLaunchKernelGGL(cast_utf8_kernel, dim3(grid), dim3(kCastThreads), 0, st,
                     static_cast<const int32_t*>(in->values), in->data, in->validity, in->length,
                     to_type, values_out, validity_out, cnt);
  HIP_TRY(hipGetLastError());
  unsigned long long h = 0;
  HIP_TRY(hipMemcpyAsync(&h, cnt, sizeof(h), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipFreeAsync(cnt, st));
  HIP_TRY(hipStreamSynchronize(st));
  *n_unsupported = (int64_t)h;
  return DQ_OK;
}
