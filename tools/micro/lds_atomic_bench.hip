// Microbenchmark: LDS atomic costs on gfx950, in the shape of phase C's inserts (512-thread
// workgroups, two per CU, a 4096-slot u64 table, 4 random slots per thread per round).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#ifndef KTS
#define KTS 8192
#endif
constexpr int KT = KTS, T = 512, ROUNDS = 256;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

template <int MODE>
__global__ void __launch_bounds__(T, 4) k(unsigned long long* out, int reps) {
  // one 64 KB region (two workgroups per CU, as phase C): the arrays alias (a rate benchmark)
  __shared__ unsigned long long buf[KT];
  unsigned long long* tab = buf;
  unsigned long long* cnt = buf;
  uint32_t* tab32 = reinterpret_cast<uint32_t*>(buf);
  for (int i = threadIdx.x; i < KT; i += T) { tab[i] = ~0ULL; cnt[i] = 0; tab32[i] = ~0u; }
  __syncthreads();
  unsigned long long acc = 0;
  uint64_t seed = mix(blockIdx.x * 7919ULL + threadIdx.x);
  for (int r = 0; r < reps; ++r) {
    uint64_t h[4];
    uint32_t sl[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) { h[q] = mix(seed + r * 4 + q); sl[q] = (uint32_t)h[q] & (KT - 1); }
    if (MODE == 0) {  // CAS64 with return
      unsigned long long o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = atomicCAS(&tab[sl[q]], ~0ULL, h[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += o[q];
    } else if (MODE == 1) {  // CAS64 + add64 (no return)
      unsigned long long o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = atomicCAS(&tab[sl[q]], ~0ULL, h[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q) { atomicAdd(&cnt[sl[q]], 1ULL); acc += o[q]; }
    } else if (MODE == 2) {  // CAS32 with return
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = atomicCAS(&tab32[sl[q]], ~0u, (uint32_t)h[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += o[q];
    } else if (MODE == 3) {  // plain 64-bit read + write
      unsigned long long o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = tab[sl[q]];
#pragma unroll
      for (int q = 0; q < 4; ++q) { tab[sl[q]] = h[q]; acc += o[q]; }
    } else if (MODE == 4) {  // add64 no return only
#pragma unroll
      for (int q = 0; q < 4; ++q) atomicAdd(&cnt[sl[q]], 1ULL);
    } else if (MODE == 5) {  // add32 no return only
#pragma unroll
      for (int q = 0; q < 4; ++q) atomicAdd(&tab32[sl[q]], 1u);
    } else if (MODE == 6) {  // the hashing alone
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += h[q] ^ sl[q];
    }
    if ((r & 15) == 15) {  // keep the table from filling (reset every 16 rounds)
      __syncthreads();
      for (int i = threadIdx.x; i < KT; i += T) { tab[i] = ~0ULL; tab32[i] = ~0u; }
      __syncthreads();
    }
  }
  if (acc == 12345) out[0] = acc + cnt[threadIdx.x];
}

int main() {
  unsigned long long* out;
  hipMalloc(&out, 8);
  const char* names[] = {"cas64", "cas64+add64", "cas32", "rw64", "add64", "add32", "hash-only"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 7; ++mode) {
    for (int it = 0; it < 2; ++it) {
      hipEventRecord(e0);
      switch (mode) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(512), dim3(T), 0, 0, out, ROUNDS); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(512), dim3(T), 0, 0, out, ROUNDS); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(512), dim3(T), 0, 0, out, ROUNDS); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(512), dim3(T), 0, 0, out, ROUNDS); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(512), dim3(T), 0, 0, out, ROUNDS); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(512), dim3(T), 0, 0, out, ROUNDS); break;
        case 6: hipLaunchKernelGGL(k<6>, dim3(512), dim3(T), 0, 0, out, ROUNDS); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (it) {
        const double rounds_per_wg = ROUNDS;
        // per workgroup-round: 2048 ops (512 threads x 4)
        printf("%-12s %.3f ms  %.1f ns per workgroup-round (2048 ops)\n", names[mode], ms,
               ms * 1e6 / rounds_per_wg);
      }
    }
  }
  return 0;
}
