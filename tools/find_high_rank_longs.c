/* Finds int64 values whose Spark XXH64 hash (hashLong, seed 42) gives an HLL++ rank
 * pw = nlz((h << 9) | 1 << 8) + 1 >= MIN_PW (StatefulHyperloglogPlus.scala:87-113).  Used once to
 * make the register >= 31 fixture of tests/golden/make_golden.py (a 1e9-row column reaches such
 * ranks; the golden tables do not).  Prints "value pw idx" lines.
 *   gcc -O3 -fopenmp tools/find_high_rank_longs.c -o /tmp/find_high_rank && /tmp/find_high_rank 31 40 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define P1 0x9E3779B185EBCA87ULL
#define P2 0xC2B2AE3D27D4EB4FULL
#define P3 0x165667B19E3779F9ULL
#define P4 0x85EBCA77C2B2AE63ULL
#define P5 0x27D4EB2F165667C5ULL
static inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t hash_long(uint64_t v, uint64_t seed) {
  uint64_t h = seed + P5 + 8;
  h ^= rotl(v * P2, 31) * P1;
  h = rotl(h, 27) * P1 + P4;
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

int main(int argc, char** argv) {
  int min_pw = argc > 1 ? atoi(argv[1]) : 31, max_pw = argc > 2 ? atoi(argv[2]) : 40;
  int found[64] = {0};
  int remaining = max_pw - min_pw + 1;
  uint64_t chunk = 1ULL << 24;
  for (uint64_t base = 0; remaining > 0 && base < (1ULL << 44); base += 64 * chunk) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int c = 0; c < 64; ++c) {
      for (uint64_t v = base + c * chunk; v < base + (c + 1) * chunk; ++v) {
        uint64_t h = hash_long(v, 42);
        uint64_t w = (h << 9) | (1ULL << 8);
        int pw = __builtin_clzll(w) + 1;
        if (pw >= min_pw && pw <= max_pw) {
#pragma omp critical
          if (!found[pw]) {
            found[pw] = 1;
            --remaining;
            printf("%llu %d %llu\n", (unsigned long long)v, pw, (unsigned long long)(h >> 55));
            fflush(stdout);
          }
        }
      }
    }
  }
  return 0;
}
