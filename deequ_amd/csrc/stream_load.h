// stream_load.h -- streaming global loads shared by the scan (scan.hip) and the group-by
// (freq.hip): 16-byte non-temporal vector loads, scalar loads through the global address space,
// unaligned 8-byte loads, and a 1024-row chunk's validity bits redistributed across the wave.
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

namespace dq {

// Once-read streaming loads: 16 bytes per lane, non-temporal by default (DQ_NT_LOADS=0 builds the
// default-policy variant for A/B measurement).  Every buffer these paths stream is read once.
#ifndef DQ_NT_LOADS
#define DQ_NT_LOADS 1
#endif
__device__ __forceinline__ uint4 ld16(const void* p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) v4u* gptr;  // global: global_load, not flat_load
#if DQ_NT_LOADS
  const v4u v = __builtin_nontemporal_load((gptr)p);
#else
  const v4u v = *(gptr)p;
#endif
  return make_uint4(v.x, v.y, v.z, v.w);
}
// Scalar loads through the global address space (global_load_*, not flat_load_*: flat loads also
// count against lgkmcnt, so every LDS / scalar wait would wait for them too).
__device__ __forceinline__ uint32_t ldg32(const void* p) {
  return *(const __attribute__((address_space(1))) uint32_t*)p;
}
__device__ __forceinline__ int32_t ldg_i32(const int32_t* p) {
  return *(const __attribute__((address_space(1))) int32_t*)p;
}
__device__ __forceinline__ uint64_t ldg64_unaligned(const void* p) {
  typedef uint64_t __attribute__((aligned(1))) u64u;
  return *(const __attribute__((address_space(1))) u64u*)p;
}
// 32 rows of a validity / where bitmap (all ones when the bitmap is absent)
__device__ __forceinline__ uint32_t bits32(const uint8_t* bm, int64_t word) {
  return bm ? ldg32(reinterpret_cast<const uint32_t*>(bm) + word) : ~0u;
}

// Validity (or where) bits of a 1024-row chunk: lane l < 32 holds dword l of the chunk's 128-byte
// bitmap slice (lanes 32..63 mirror them); get(o, n) returns n (<= 16, o % n == 0) bits at bit o.
struct ChunkBits {
  uint32_t w;
  __device__ __forceinline__ void load(const uint8_t* bm, int64_t r0) {
    w = ldg32(reinterpret_cast<const uint32_t*>(bm) + (r0 >> 5) + ((int)__lane_id() & 31));
  }
  __device__ __forceinline__ uint32_t get(int o, int n) const {
    const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((o >> 5) << 2, (int)w);
    return (v >> (o & 31)) & ((1u << n) - 1u);
  }
};

}  // namespace dq
