// synth.hip -- device generator of the synthetic "Item" table (SURVEY.md §8(d);
// examples/entities.scala:19-25) used by bench.py and the full-size GPU tests.  Built into
// libdq_synth.so, separate from the engine.  The recipe is integer-only and is restated bit for
// bit by deequ_amd/synth.py (numpy), so any row range can be regenerated on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rnd(uint64_t s, uint64_t row) {
  return mix(s ^ (row * 0xD1B54A32D192ED03ULL));
}

struct Streams {
  uint64_t s[8][4];  // [column][draw]
};

enum Col { ID = 0, NAME = 1, DESC = 2, PRIORITY = 3, NUMVIEWS = 4, SCORE = 5 };

__device__ __forceinline__ bool is_null(const Streams& st, int col, uint64_t row) {
  return rnd(st.s[col][0], row) % 100 < 5;
}

__device__ __forceinline__ int64_t num_views(const Streams& st, uint64_t row) {
  uint64_t h1 = rnd(st.s[NUMVIEWS][1], row) | (1ULL << 40);
  uint64_t h2 = rnd(st.s[NUMVIEWS][2], row);
  int64_t g = __builtin_ctzll(h1);
  int64_t v = ((g << 10) + (int64_t)(h2 & 1023)) * 2 / 3;
  if (rnd(st.s[NUMVIEWS][3], row) % 100 == 0) v = -v;
  return v;
}

__device__ __forceinline__ int name_len(const Streams& st, uint64_t row) {
  return 7 + 4 + (int)(rnd(st.s[NAME][1], row) % 5);
}
__device__ __forceinline__ int priority_code(const Streams& st, uint64_t row) {
  return (int)(rnd(st.s[PRIORITY][1], row) % 3);
}
__device__ __forceinline__ int priority_len(int code) { return code == 0 ? 4 : (code == 1 ? 3 : 6); }

// fixed-width columns + validity bitmaps + string lengths for rows [row0, row0 + n)
__global__ void gen_fixed(Streams st, uint64_t row0, int64_t n, int64_t* id, uint64_t* id_valid,
                          int64_t* views, uint64_t* views_valid, double* score,
                          uint64_t* score_valid, int32_t* name_len_out, uint64_t* name_valid,
                          int32_t* prio_len_out, uint64_t* prio_valid) {
  const int lane = threadIdx.x & 63;
  for (int64_t base = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~63LL; base < n;
       base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + lane;
    const bool in = i < n;
    const uint64_t row = row0 + (uint64_t)i;
    bool v_id = false, v_vw = false, v_sc = false, v_nm = false, v_pr = false;
    if (in) {
      v_id = !is_null(st, ID, row);
      id[i] = v_id ? (int64_t)mix(row ^ 0x5DEECE66DULL) : 0;
      v_vw = !is_null(st, NUMVIEWS, row);
      int64_t vw = num_views(st, row);
      views[i] = v_vw ? vw : 0;
      if (score) {
        v_sc = !is_null(st, SCORE, row);
        uint64_t h = rnd(st.s[SCORE][1], row);
        score[i] = v_sc ? (double)vw * 0.5 + (double)(h & 0xFFFF) / 65536.0 : 0.0;
      }
      v_nm = !is_null(st, NAME, row);
      name_len_out[i] = v_nm ? name_len(st, row) : 0;
      v_pr = !is_null(st, PRIORITY, row);
      prio_len_out[i] = v_pr ? priority_len(priority_code(st, row)) : 0;
    }
    uint64_t b_id = __ballot(v_id), b_vw = __ballot(v_vw), b_sc = __ballot(v_sc);
    uint64_t b_nm = __ballot(v_nm), b_pr = __ballot(v_pr);
    if (lane == 0) {
      const int64_t w = base >> 6;
      id_valid[w] = b_id;
      views_valid[w] = b_vw;
      if (score_valid) score_valid[w] = b_sc;
      name_valid[w] = b_nm;
      prio_valid[w] = b_pr;
    }
  }
}

__global__ void gen_strings(Streams st, uint64_t row0, int64_t n, const int32_t* name_off,
                            uint8_t* name_data, const int32_t* prio_off, uint8_t* prio_data) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t row = row0 + (uint64_t)i;
    int32_t s = name_off[i], e = name_off[i + 1];
    if (e > s) {
      const char* pre = "Thingy ";
      for (int k = 0; k < 7; ++k) name_data[s + k] = (uint8_t)pre[k];
      uint64_t h = rnd(st.s[NAME][2], row);
      for (int k = 7; k < e - s; ++k) name_data[s + k] = (uint8_t)('a' + ((h >> (8 * (k - 7))) & 0xFF) % 26);
    }
    s = prio_off[i];
    e = prio_off[i + 1];
    if (e > s) {
      int code = priority_code(st, row);
      const char* v = code == 0 ? "high" : (code == 1 ? "low" : "medium");
      for (int k = 0; k < e - s; ++k) prio_data[s + k] = (uint8_t)v[k];
    }
  }
}

Streams make_streams(uint64_t seed) {
  Streams st;
  for (int c = 0; c < 8; ++c)
    for (int k = 0; k < 4; ++k) {
      uint64_t z = seed * 0x1000193ULL + (uint64_t)c * 64 + (uint64_t)k;
      // host copy of mix()
      z += 0x9E3779B97F4A7C15ULL;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
      st.s[c][k] = z ^ (z >> 31);
    }
  return st;
}

unsigned grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace

extern "C" int dq_synth_fixed(uint64_t seed, uint64_t row0, int64_t n, int64_t* id,
                              uint64_t* id_valid, int64_t* views, uint64_t* views_valid,
                              double* score, uint64_t* score_valid, int32_t* name_len,
                              uint64_t* name_valid, int32_t* prio_len, uint64_t* prio_valid,
                              void* stream) {
  Streams st = make_streams(seed);
  hipLaunchKernelGGL(gen_fixed, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, st, row0, n, id,
                     id_valid, views, views_valid, score, score_valid, name_len, name_valid,
                     prio_len, prio_valid);
  return (int)hipGetLastError();
}

extern "C" int dq_synth_strings(uint64_t seed, uint64_t row0, int64_t n, const int32_t* name_off,
                                uint8_t* name_data, const int32_t* prio_off, uint8_t* prio_data,
                                void* stream) {
  Streams st = make_streams(seed);
  hipLaunchKernelGGL(gen_strings, dim3(grid(n)), dim3(256), 0, (hipStream_t)stream, st, row0, n,
                     name_off, name_data, prio_off, prio_data);
  return (int)hipGetLastError();
}

// configs[4]'s URL-bearing text: row r of `out` = a prefix + row r of `src`; the prefix carries an
// https URL when bit 62 of r * 0x9E3779B97F4A7C15 is set (about half the rows), else none.
// out_off holds the caller's offsets (it knows both lengths).
namespace {
__constant__ const char kUrlPrefix[] = "see https://www.example.com/item/";  // 33 bytes
__constant__ const char kPlainPrefix[] = "no link: ";                        // 9 bytes
__global__ void gen_describe(uint64_t row0, int64_t n, const int32_t* src_off, const uint8_t* src,
                             const int32_t* out_off, uint8_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool url = (((row0 + (uint64_t)i) * 0x9E3779B97F4A7C15ULL) >> 62) & 1ULL;
  const char* pre = url ? kUrlPrefix : kPlainPrefix;
  const int plen = url ? 33 : 9;
  uint8_t* o = out + out_off[i];
  for (int k = 0; k < plen; ++k) o[k] = (uint8_t)pre[k];
  const int32_t s = src_off[i], len = src_off[i + 1] - s;
  for (int k = 0; k < len; ++k) o[plen + k] = src[s + k];
}
}  // namespace

extern "C" int dq_synth_describe(uint64_t row0, int64_t n, const int32_t* src_off,
                                 const uint8_t* src, const int32_t* out_off, uint8_t* out,
                                 void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gen_describe, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, row0, n, src_off, src, out_off, out);
  return (int)hipGetLastError();
}
