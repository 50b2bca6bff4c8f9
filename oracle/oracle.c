/*
 * ORACLE -- test infrastructure only (never linked into or called by the product).
 *
 * C restatement of the Spark 2.2 / deequ per-row aggregation semantics for the benchmark
 * workloads, used (a) by the GPU parity tests at 1e6..1e8 rows, where the pure-Python oracle
 * (oracle/deequ_oracle.py) is too slow, and (b) as bench.py's `cpu_baseline` ("port": a CPU
 * restatement of Spark 2.2 deequ semantics -- not Spark; no JVM exists in this image).
 *
 * Execution model = Spark local[N]: the rows are split into `nthreads` contiguous partitions, each
 * partition runs the aggregate's sequential per-row update (Spark's partial aggregation), and the
 * partition buffers are merged in partition order with the aggregate's merge rule.
 *
 * Cited semantics (M/ = /root/reference/src/main/scala/com/amazon/deequ/):
 *   count / completeness   M/analyzers/Size.scala:36-40, M/analyzers/Completeness.scala:42-45
 *   compliance             M/analyzers/Compliance.scala:47-49 (NULL predicate: not counted)
 *   Sum (Long, wrapping)   M/analyzers/Sum.scala:35 + Spark Sum over LongType
 *   Min / Max              M/analyzers/Minimum.scala:36, Maximum.scala:36
 *   StdDev (Welford)       M/analyzers/catalyst/StatefulStdDevPop.scala:24-34 (CentralMomentAgg
 *                          update), merge M/analyzers/StandardDeviation.scala:37-44
 *   Correlation            M/analyzers/catalyst/StatefulCorrelation.scala:24-49 (Corr update),
 *                          merge M/analyzers/Correlation.scala:37-52
 *   HLL++ registers        M/analyzers/catalyst/StatefulHyperloglogPlus.scala:87-137
 *   frequencies            M/analyzers/GroupingAnalyzers.scala:53-80, Entropy.scala:33-40
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline int bit(const uint8_t* bm, int64_t r) { return bm ? (bm[r >> 3] >> (r & 7)) & 1 : 1; }

/* ---------------------------------------------------------------- numeric column (S10) ---- */
typedef struct {
  int64_t count;      /* non-null values                     */
  int64_t sum_long;   /* wrapping Long sum                   */
  int64_t min, max;
  double n, avg, m2;  /* CentralMomentAgg buffer             */
  int64_t pred_true;  /* numViews >= lit (NULL not counted)  */
  int64_t pred_nonnull;
} or_numeric;

static void numeric_merge(or_numeric* a, const or_numeric* b) {
  if (b->count == 0) return;
  if (a->count == 0) {
    *a = *b;
    return;
  }
  double n = a->n + b->n, delta = b->avg - a->avg, delta_n = n == 0.0 ? 0.0 : delta / n;
  a->avg = a->avg + delta_n * b->n;
  a->m2 = a->m2 + b->m2 + delta * delta_n * a->n * b->n;
  a->n = n;
  a->count += b->count;
  a->sum_long = (int64_t)((uint64_t)a->sum_long + (uint64_t)b->sum_long);
  if (b->min < a->min) a->min = b->min;
  if (b->max > a->max) a->max = b->max;
  a->pred_true += b->pred_true;
  a->pred_nonnull += b->pred_nonnull;
}

/* op: 0 none, 12 '=', 13 '<>', 14 '<', 15 '<=', 16 '>', 17 '>=' (dq_xop numbering) */
static inline int cmp_op(int op, int64_t x, int64_t lit) {
  switch (op) {
    case 12: return x == lit;
    case 13: return x != lit;
    case 14: return x < lit;
    case 15: return x <= lit;
    case 16: return x > lit;
    case 17: return x >= lit;
    default: return 0;
  }
}

void or_numeric_i64(const int64_t* v, const uint8_t* valid, int64_t n, int op, int64_t lit,
                    int nthreads, or_numeric* out) {
  if (nthreads < 1) nthreads = 1;
  or_numeric* parts = (or_numeric*)calloc((size_t)nthreads, sizeof(or_numeric));
#pragma omp parallel for num_threads(nthreads) schedule(static, 1)
  for (int p = 0; p < nthreads; ++p) {
    int64_t r0 = n * p / nthreads, r1 = n * (p + 1) / nthreads;
    or_numeric s;
    memset(&s, 0, sizeof(s));
    s.min = INT64_MAX;
    s.max = INT64_MIN;
    for (int64_t r = r0; r < r1; ++r) {
      if (!bit(valid, r)) continue;
      int64_t x = v[r];
      s.count += 1;
      s.sum_long = (int64_t)((uint64_t)s.sum_long + (uint64_t)x);
      if (x < s.min) s.min = x;
      if (x > s.max) s.max = x;
      double xd = (double)x;
      double n2 = s.n + 1.0, delta = xd - s.avg, delta_n = delta / n2;
      s.avg += delta_n;
      s.m2 += delta * (delta - delta_n);
      s.n = n2;
      if (op) {
        s.pred_nonnull += 1;
        s.pred_true += cmp_op(op, x, lit);
      }
    }
    parts[p] = s;
  }
  or_numeric acc;
  memset(&acc, 0, sizeof(acc));
  acc.min = INT64_MAX;
  acc.max = INT64_MIN;
  for (int p = 0; p < nthreads; ++p) numeric_merge(&acc, &parts[p]);
  *out = acc;
  free(parts);
}

int64_t or_validity_count(const uint8_t* valid, int64_t n, int nthreads) {
  if (!valid) return n;
  int64_t total = 0;
#pragma omp parallel for num_threads(nthreads) reduction(+ : total) schedule(static)
  for (int64_t r = 0; r < n; ++r) total += bit(valid, r);
  return total;
}

/* [col IS NULL OR] col IN (list): TRUE count and non-NULL count */
void or_str_in(const int32_t* off, const uint8_t* data, const uint8_t* valid, int64_t n,
               const uint8_t* list_bytes, const int32_t* list_off, int n_list, int null_is_true,
               int nthreads, int64_t* t_out, int64_t* nn_out) {
  int64_t t = 0, nn = 0;
#pragma omp parallel for num_threads(nthreads) reduction(+ : t, nn) schedule(static)
  for (int64_t r = 0; r < n; ++r) {
    if (!bit(valid, r)) {
      if (null_is_true) {
        t += 1;
        nn += 1;
      }
      continue;
    }
    int32_t s = off[r], len = off[r + 1] - off[r];
    int match = 0;
    for (int j = 0; j < n_list && !match; ++j) {
      int32_t ls = list_off[j], ll = list_off[j + 1] - ls;
      if (ll == len && memcmp(data + s, list_bytes + ls, (size_t)len) == 0) match = 1;
    }
    t += match;
    nn += 1;
  }
  *t_out = t;
  *nn_out = nn;
}

/* ------------------------------------------------------- S10 as ONE pass (bench baseline) --- */
/* The reference runs a suite as one Spark job (AnalysisRunner.scala:279-326): each task walks its
 * partition once and updates every aggregate of the suite per row.  Same here for S10: Size,
 * Completeness(id), Completeness(name), Compliance(numViews >= 0), Compliance(priority IS NULL OR
 * priority IN (list)), Sum / Mean / StdDev / Min / Max(numViews); partitions merged in order. */
typedef struct {
  int64_t rows, id_nonnull, name_nonnull, prio_true;
  or_numeric views;
} or_s10;

void or_s10_fused(const uint8_t* id_valid, const uint8_t* name_valid, const int64_t* views,
                  const uint8_t* views_valid, const int32_t* prio_off, const uint8_t* prio_data,
                  const uint8_t* prio_valid, int64_t n, const uint8_t* list_bytes,
                  const int32_t* list_off, int n_list, int nthreads, or_s10* out) {
  if (nthreads < 1) nthreads = 1;
  or_s10* parts = (or_s10*)calloc((size_t)nthreads, sizeof(or_s10));
#pragma omp parallel for num_threads(nthreads) schedule(static, 1)
  for (int p = 0; p < nthreads; ++p) {
    int64_t r0 = n * p / nthreads, r1 = n * (p + 1) / nthreads;
    or_s10 s;
    memset(&s, 0, sizeof(s));
    s.views.min = INT64_MAX;
    s.views.max = INT64_MIN;
    for (int64_t r = r0; r < r1; ++r) {
      s.rows += 1;
      s.id_nonnull += bit(id_valid, r);
      s.name_nonnull += bit(name_valid, r);
      if (bit(views_valid, r)) {
        int64_t x = views[r];
        s.views.count += 1;
        s.views.sum_long = (int64_t)((uint64_t)s.views.sum_long + (uint64_t)x);
        if (x < s.views.min) s.views.min = x;
        if (x > s.views.max) s.views.max = x;
        double xd = (double)x;
        double n2 = s.views.n + 1.0, delta = xd - s.views.avg, delta_n = delta / n2;
        s.views.avg += delta_n;
        s.views.m2 += delta * (delta - delta_n);
        s.views.n = n2;
        s.views.pred_nonnull += 1;
        s.views.pred_true += x >= 0;
      }
      if (!bit(prio_valid, r)) {
        s.prio_true += 1;
      } else {
        int32_t st = prio_off[r], len = prio_off[r + 1] - st;
        for (int j = 0; j < n_list; ++j) {
          int32_t ls = list_off[j], ll = list_off[j + 1] - ls;
          if (ll == len && memcmp(prio_data + st, list_bytes + ls, (size_t)len) == 0) {
            s.prio_true += 1;
            break;
          }
        }
      }
    }
    parts[p] = s;
  }
  or_s10 acc;
  memset(&acc, 0, sizeof(acc));
  acc.views.min = INT64_MAX;
  acc.views.max = INT64_MIN;
  for (int p = 0; p < nthreads; ++p) {
    acc.rows += parts[p].rows;
    acc.id_nonnull += parts[p].id_nonnull;
    acc.name_nonnull += parts[p].name_nonnull;
    acc.prio_true += parts[p].prio_true;
    numeric_merge(&acc.views, &parts[p].views);
  }
  *out = acc;
  free(parts);
}

/* ---------------------------------------------------------------- XXH64 ------------------- */
#define XP1 0x9E3779B185EBCA87ULL
#define XP2 0xC2B2AE3D27D4EB4FULL
#define XP3 0x165667B19E3779F9ULL
#define XP4 0x85EBCA77C2B2AE63ULL
#define XP5 0x27D4EB2F165667C5ULL

static inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
static inline uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static inline uint64_t xround(uint64_t acc, uint64_t in) { return rotl(acc + in * XP2, 31) * XP1; }
static inline uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * XP1 + XP4; }

uint64_t or_xxh64(const uint8_t* p, int64_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    const uint8_t* limit = end - 32;
    do {
      v1 = xround(v1, rd64(p));
      v2 = xround(v2, rd64(p + 8));
      v3 = xround(v3, rd64(p + 16));
      v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = xmerge(h, v1);
    h = xmerge(h, v2);
    h = xmerge(h, v3);
    h = xmerge(h, v4);
  } else {
    h = seed + XP5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= xround(0, rd64(p));
    h = rotl(h, 27) * XP1 + XP4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32(p) * XP1;
    h = rotl(h, 23) * XP2 + XP3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * XP5;
    h = rotl(h, 11) * XP1;
    ++p;
  }
  h ^= h >> 33;
  h *= XP2;
  h ^= h >> 29;
  h *= XP3;
  h ^= h >> 32;
  return h;
}

static inline void hll_update(uint8_t* regs, uint64_t x) {
  uint32_t idx = (uint32_t)(x >> 55);
  uint64_t w = (x << 9) | (1ULL << 8);
  uint8_t pw = (uint8_t)(__builtin_clzll(w) + 1);
  if (pw > regs[idx]) regs[idx] = pw;
}

/* type: 5 = long (hashLong), 7 = double (doubleToLongBits), 8 = utf8 */
void or_hll(int type, const void* values, const uint8_t* data, const uint8_t* valid, int64_t n,
            int nthreads, uint8_t* regs_out) {
  uint8_t* parts = (uint8_t*)calloc((size_t)nthreads * 512, 1);
#pragma omp parallel for num_threads(nthreads) schedule(static, 1)
  for (int p = 0; p < nthreads; ++p) {
    uint8_t* regs = parts + (size_t)p * 512;
    int64_t r0 = n * p / nthreads, r1 = n * (p + 1) / nthreads;
    for (int64_t r = r0; r < r1; ++r) {
      if (!bit(valid, r)) continue;
      uint64_t x;
      if (type == 8) {
        const int32_t* off = (const int32_t*)values;
        x = or_xxh64(data + off[r], off[r + 1] - off[r], 42);
      } else if (type == 7) {
        double d = ((const double*)values)[r];
        uint64_t b;
        if (d != d) b = 0x7ff8000000000000ULL;
        else memcpy(&b, &d, 8);
        x = or_xxh64((const uint8_t*)&b, 8, 42);
      } else {
        x = or_xxh64((const uint8_t*)&((const int64_t*)values)[r], 8, 42);
      }
      hll_update(regs, x);
    }
  }
  memset(regs_out, 0, 512);
  for (int p = 0; p < nthreads; ++p)
    for (int i = 0; i < 512; ++i)
      if (parts[(size_t)p * 512 + i] > regs_out[i]) regs_out[i] = parts[(size_t)p * 512 + i];
  free(parts);
}

/* Corr over (long x, double y) */
void or_corr(const int64_t* x, const uint8_t* vx, const double* y, const uint8_t* vy, int64_t n,
             int nthreads, double* out6) {
  double* parts = (double*)calloc((size_t)nthreads * 6, sizeof(double));
#pragma omp parallel for num_threads(nthreads) schedule(static, 1)
  for (int p = 0; p < nthreads; ++p) {
    double s[6] = {0, 0, 0, 0, 0, 0};
    int64_t r0 = n * p / nthreads, r1 = n * (p + 1) / nthreads;
    for (int64_t r = r0; r < r1; ++r) {
      if (!bit(vx, r) || !bit(vy, r)) continue;
      double xv = (double)x[r], yv = y[r];
      double n2 = s[0] + 1.0, dx = xv - s[1], dxn = dx / n2, dy = yv - s[2], dyn = dy / n2;
      double xa = s[1] + dxn, ya = s[2] + dyn;
      s[3] += dx * (yv - ya);
      s[4] += dx * (xv - xa);
      s[5] += dy * (yv - ya);
      s[0] = n2;
      s[1] = xa;
      s[2] = ya;
    }
    memcpy(parts + 6 * p, s, sizeof(s));
  }
  double a[6] = {0, 0, 0, 0, 0, 0};
  for (int p = 0; p < nthreads; ++p) {
    const double* b = parts + 6 * p;
    if (b[0] == 0.0) continue;
    double n1 = a[0], n2 = b[0], nn = n1 + n2;
    double dx = b[1] - a[1], dxn = nn == 0.0 ? 0.0 : dx / nn;
    double dy = b[2] - a[2], dyn = nn == 0.0 ? 0.0 : dy / nn;
    a[1] += dxn * n2;
    a[2] += dyn * n2;
    a[3] += b[3] + dx * dyn * n1 * n2;
    a[4] += b[4] + dx * dxn * n1 * n2;
    a[5] += b[5] + dy * dyn * n1 * n2;
    a[0] = nn;
  }
  memcpy(out6, a, sizeof(a));
  free(parts);
}

/* frequencies of a long column (NULLs skipped): groups, count==1 groups, entropy */
static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}
void or_freq_i64(const int64_t* v, const uint8_t* valid, int64_t n, int64_t num_rows,
                 int64_t* groups, int64_t* unique, double* ent) {
  int64_t m = 0;
  int64_t* buf = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
  for (int64_t r = 0; r < n; ++r)
    if (bit(valid, r)) buf[m++] = v[r];
  qsort(buf, (size_t)m, 8, cmp_i64);
  int64_t g = 0, u = 0;
  double e = 0.0;
  for (int64_t i = 0; i < m;) {
    int64_t j = i;
    while (j < m && buf[j] == buf[i]) ++j;
    int64_t c = j - i;
    ++g;
    u += c == 1;
    double p = (double)c / (double)num_rows;
    e += -p * log(p);
    i = j;
  }
  *groups = g;
  *unique = u;
  *ent = e;
  free(buf);
}

/* ------------------------------------------------- frequency family, hash-partitioned (CPU) ----
 * computeFrequencies (M/analyzers/GroupingAnalyzers.scala:53-80: where all keys are not null,
 * groupBy(keys).agg(count)) and the one aggregation over the frequency table that Uniqueness /
 * Distinctness / UniqueValueRatio / CountDistinct / Entropy share (AnalysisRunner.scala:490-500;
 * Σ[c==1], count(*), Σ -(c/numRows) ln(c/numRows), Entropy.scala:33-40), plus Histogram's
 * top-k (Histogram.scala:54-79: NULL is a group of its own when null_as_group, its key
 * "NullValue"; rdd.top(k) by count, ties in any order).
 * Execution = Spark local[N]'s hash Exchange + HashAggregate: every thread hash-partitions its
 * contiguous row range into P shuffle partitions (count, then scatter of row ids), then each
 * partition is aggregated in an open-addressing table; partition partials are combined in
 * partition order.  type 0: int64 keys; type 1: utf8 (int32 offsets + bytes), equal keys compared
 * byte for byte.  topk_rows: a row of each top group (-1: the NULL group).
 */
typedef struct {
  int64_t groups, unique, null_rows;
  double entropy;
} or_freq_out;

static inline uint64_t or_mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

typedef struct {
  int64_t c, row;
} or_top;

/* min-heap of the k largest counts */
static void top_push(or_top* h, int* nh, int k, int64_t c, int64_t row) {
  if (k <= 0) return;
  if (*nh < k) {
    int i = (*nh)++;
    h[i].c = c;
    h[i].row = row;
    while (i > 0 && h[(i - 1) / 2].c > h[i].c) {
      or_top t = h[i];
      h[i] = h[(i - 1) / 2];
      h[(i - 1) / 2] = t;
      i = (i - 1) / 2;
    }
    return;
  }
  if (c <= h[0].c) return;
  h[0].c = c;
  h[0].row = row;
  for (int i = 0;;) {
    int l = 2 * i + 1, r = l + 1, m = i;
    if (l < *nh && h[l].c < h[m].c) m = l;
    if (r < *nh && h[r].c < h[m].c) m = r;
    if (m == i) break;
    or_top t = h[i];
    h[i] = h[m];
    h[m] = t;
    i = m;
  }
}

static int top_cmp_desc(const void* a, const void* b) {
  int64_t x = ((const or_top*)a)->c, y = ((const or_top*)b)->c;
  return (x < y) - (x > y);
}

static inline uint64_t key_hash(int type, const void* values, const uint8_t* data, int64_t r) {
  if (type == 0) return or_mix64((uint64_t)((const int64_t*)values)[r]);
  const int32_t* off = (const int32_t*)values;
  return or_xxh64(data + off[r], off[r + 1] - off[r], 0);
}

static inline int key_eq(int type, const void* values, const uint8_t* data, int64_t a, int64_t b) {
  if (type == 0) return ((const int64_t*)values)[a] == ((const int64_t*)values)[b];
  const int32_t* off = (const int32_t*)values;
  const int32_t la = off[a + 1] - off[a], lb = off[b + 1] - off[b];
  return la == lb && memcmp(data + off[a], data + off[b], (size_t)la) == 0;
}

void or_freq(int type, const void* values, const uint8_t* data, const uint8_t* valid, int64_t n,
             int null_as_group, int64_t num_rows, int k, int nthreads, or_freq_out* out,
             int64_t* topk_counts, int64_t* topk_rows, int* n_top) {
  const int P = 256;  /* shuffle partitions */
  const double nr = (double)num_rows;
  int64_t* cnt = (int64_t*)calloc((size_t)nthreads * P + 1, sizeof(int64_t));
  uint64_t* hs = (uint64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
  int64_t* rows = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
  int64_t nulls = 0;
  /* the shuffle write: hash every keyed row, count per (thread, partition), scatter row ids */
#pragma omp parallel num_threads(nthreads) reduction(+ : nulls)
  {
    const int t = omp_get_thread_num();
    const int64_t r0 = n * t / nthreads, r1 = n * (t + 1) / nthreads;
    int64_t* c = cnt + (size_t)t * P;
    for (int64_t r = r0; r < r1; ++r) {
      if (!bit(valid, r)) {
        ++nulls;
        hs[r] = 0;
        continue;
      }
      hs[r] = key_hash(type, values, data, r);
      ++c[hs[r] >> 56];
    }
  }
  /* offsets: partition-major, thread order inside a partition */
  int64_t* base = (int64_t*)malloc(((size_t)nthreads * P + 1) * sizeof(int64_t));
  int64_t acc = 0;
  for (int p = 0; p < P; ++p)
    for (int t = 0; t < nthreads; ++t) {
      base[(size_t)t * P + p] = acc;
      acc += cnt[(size_t)t * P + p];
    }
  int64_t* pbeg = (int64_t*)malloc((size_t)(P + 1) * sizeof(int64_t));
  for (int p = 0; p < P; ++p) pbeg[p] = base[p];
  pbeg[P] = acc;
#pragma omp parallel num_threads(nthreads)
  {
    const int t = omp_get_thread_num();
    const int64_t r0 = n * t / nthreads, r1 = n * (t + 1) / nthreads;
    int64_t* b = base + (size_t)t * P;
    for (int64_t r = r0; r < r1; ++r)
      if (bit(valid, r)) rows[b[hs[r] >> 56]++] = r;
  }
  /* the shuffle read + final aggregation, one partition at a time per thread */
  int64_t* pg = (int64_t*)calloc(P, sizeof(int64_t));
  int64_t* pu = (int64_t*)calloc(P, sizeof(int64_t));
  double* pe = (double*)calloc(P, sizeof(double));
  or_top* ptop = (or_top*)malloc((size_t)P * (k > 0 ? k : 1) * sizeof(or_top));
  int* pnt = (int*)calloc(P, sizeof(int));
  int64_t lit_count = 0, lit_row = -1;  /* (one partition holds it: no race) */
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
  for (int p = 0; p < P; ++p) {
    const int64_t m = pbeg[p + 1] - pbeg[p];
    size_t cap = 16;
    while (cap < (size_t)m * 2) cap <<= 1;
    int64_t* trow = (int64_t*)malloc(cap * sizeof(int64_t));
    int64_t* tcnt = (int64_t*)malloc(cap * sizeof(int64_t));
    for (size_t i = 0; i < cap; ++i) trow[i] = -1;
    for (int64_t i = pbeg[p]; i < pbeg[p + 1]; ++i) {
      const int64_t r = rows[i];
      size_t s = (size_t)(hs[r] & (cap - 1));
      for (;;) {
        if (trow[s] < 0) {
          trow[s] = r;
          tcnt[s] = 1;
          break;
        }
        if (hs[trow[s]] == hs[r] && key_eq(type, values, data, trow[s], r)) {
          ++tcnt[s];
          break;
        }
        s = (s + 1) & (cap - 1);
      }
    }
    int64_t g = 0, u = 0;
    double e = 0.0;
    for (size_t s = 0; s < cap; ++s) {
      if (trow[s] < 0) continue;
      const int64_t c = tcnt[s];
      if (type == 1 && null_as_group) {  /* a real "NullValue": merged with the NULL group */
        const int32_t* off = (const int32_t*)values;
        const int64_t r = trow[s];
        if (off[r + 1] - off[r] == 9 && memcmp(data + off[r], "NullValue", 9) == 0) {
          lit_count = c;
          lit_row = r;
          continue;
        }
      }
      ++g;
      u += c == 1;
      const double pr = (double)c / nr;
      e += -pr * log(pr);
      top_push(ptop + (size_t)p * k, &pnt[p], k, c, trow[s]);
    }
    pg[p] = g;
    pu[p] = u;
    pe[p] = e;
    free(trow);
    free(tcnt);
  }
  or_freq_out o = {0, 0, nulls, 0.0};
  or_top* heap = (or_top*)malloc((size_t)(k > 0 ? k : 1) * sizeof(or_top));
  int nh = 0;
  for (int p = 0; p < P; ++p) {
    o.groups += pg[p];
    o.unique += pu[p];
    o.entropy += pe[p];
    for (int i = 0; i < pnt[p]; ++i) top_push(heap, &nh, k, ptop[(size_t)p * k + i].c, ptop[(size_t)p * k + i].row);
  }
  if (null_as_group && nulls + lit_count) {  /* Histogram: the NULL group ("NullValue") */
    const int64_t c = nulls + lit_count;
    ++o.groups;
    o.unique += c == 1;
    const double pr = (double)c / nr;
    o.entropy += -pr * log(pr);
    top_push(heap, &nh, k, c, nulls ? -1 : lit_row);
  }
  qsort(heap, (size_t)nh, sizeof(or_top), top_cmp_desc);
  for (int i = 0; i < nh; ++i) {
    topk_counts[i] = heap[i].c;
    topk_rows[i] = heap[i].row;
  }
  *n_top = nh;
  *out = o;
  free(heap);
  free(pg);
  free(pu);
  free(pe);
  free(ptop);
  free(pnt);
  free(pbeg);
  free(base);
  free(rows);
  free(hs);
  free(cnt);
}

/* ------------------------------------------- configs[4] baseline helpers (cpu_baseline) ---- */
/* Double column: count, Sum (double), Min, Max, CentralMomentAgg (n, avg, m2) and `x >= lit`
 * (M/analyzers/Sum.scala:35, Minimum.scala:36, Maximum.scala:36, StandardDeviation.scala:37-44,
 * Compliance.scala:47-49), partition partials merged in partition order. */
typedef struct {
  int64_t count;
  double sum, min, max, n, avg, m2;
  int64_t pred_true;
} or_numeric_d;

void or_numeric_f64(const double* v, const uint8_t* valid, int64_t n, double lit, int nthreads,
                    or_numeric_d* out) {
  if (nthreads < 1) nthreads = 1;
  or_numeric_d* parts = (or_numeric_d*)calloc((size_t)nthreads, sizeof(or_numeric_d));
#pragma omp parallel for num_threads(nthreads) schedule(static, 1)
  for (int p = 0; p < nthreads; ++p) {
    int64_t r0 = n * p / nthreads, r1 = n * (p + 1) / nthreads;
    or_numeric_d s;
    memset(&s, 0, sizeof(s));
    s.min = INFINITY;
    s.max = -INFINITY;
    for (int64_t r = r0; r < r1; ++r) {
      if (!bit(valid, r)) continue;
      const double x = v[r];
      s.count += 1;
      s.sum += x;
      s.min = x < s.min ? x : s.min;
      s.max = x > s.max ? x : s.max;
      double n2 = s.n + 1.0, delta = x - s.avg, delta_n = delta / n2;
      s.avg += delta_n;
      s.m2 += delta * (delta - delta_n);
      s.n = n2;
      s.pred_true += x >= lit;
    }
    parts[p] = s;
  }
  or_numeric_d a;
  memset(&a, 0, sizeof(a));
  a.min = INFINITY;
  a.max = -INFINITY;
  for (int p = 0; p < nthreads; ++p) {
    const or_numeric_d* b = &parts[p];
    if (!b->count) continue;
    double nn = a.n + b->n, delta = b->avg - a.avg, delta_n = nn == 0.0 ? 0.0 : delta / nn;
    a.avg += delta_n * b->n;
    a.m2 += b->m2 + delta * delta_n * a.n * b->n;
    a.n = nn;
    a.count += b->count;
    a.sum += b->sum;
    a.min = b->min < a.min ? b->min : a.min;
    a.max = b->max > a.max ? b->max : a.max;
    a.pred_true += b->pred_true;
  }
  *out = a;
  free(parts);
}

/* PatternMatch's per-row test as a walk of a byte DFA (the table layout of CompiledRegex.blob:
 * byte_class[256], status per state 0 undecided / 1 accepted / 2 rejected, u16 next[state][class],
 * the last class = end of text): the count of matching non-NULL rows.  A timing baseline for the
 * regex scan (a DFA walk is the fastest CPU form of it; Spark runs java.util.regex per row). */
int64_t or_dfa_count(const int32_t* off, const uint8_t* data, const uint8_t* valid, int64_t n,
                     const uint8_t* byte_class, const uint8_t* status, const uint16_t* next,
                     int n_classes, int start, int nthreads) {
  int64_t hits = 0;
#pragma omp parallel for num_threads(nthreads) reduction(+ : hits) schedule(static)
  for (int64_t r = 0; r < n; ++r) {
    if (!bit(valid, r)) continue;
    int st = start;
    for (int32_t i = off[r]; i < off[r + 1] && !status[st]; ++i)
      st = next[st * n_classes + byte_class[data[i]]];
    if (!status[st]) st = next[st * n_classes + n_classes - 1];
    hits += status[st] == 1;
  }
  return hits;
}

/* DataType over a utf8 column (M/analyzers/catalyst/StatefulDataType.scala:36-69): each non-NULL
 * value is classified by the first of three full matches, FRACTIONAL ^(-|\+)? ?\d*\.\d*$, then
 * INTEGRAL ^(-|\+)? ?\d*$, then BOOLEAN ^(true|false)$ (\d = [0-9], Java's default), else String;
 * NULL rows count apart.  out5 = (NULL, Fractional, Integral, Boolean, String). */
static int dtype_class(const uint8_t* s, int32_t len) {
  int32_t i = 0;
  if (i < len && (s[i] == '-' || s[i] == '+')) ++i;
  if (i < len && s[i] == ' ') ++i;
  while (i < len && s[i] >= '0' && s[i] <= '9') ++i;
  if (i == len) return 2;  /* INTEGRAL (the empty string too) */
  if (s[i] == '.') {
    ++i;
    while (i < len && s[i] >= '0' && s[i] <= '9') ++i;
    if (i == len) return 1;  /* FRACTIONAL */
  }
  if ((len == 4 && memcmp(s, "true", 4) == 0) || (len == 5 && memcmp(s, "false", 5) == 0)) return 3;
  return 4;
}

void or_dtype_utf8(const int32_t* off, const uint8_t* data, const uint8_t* valid, int64_t n,
                   int nthreads, int64_t* out5) {
  int64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0;
#pragma omp parallel for num_threads(nthreads) reduction(+ : c0, c1, c2, c3, c4) schedule(static)
  for (int64_t r = 0; r < n; ++r) {
    if (!bit(valid, r)) {
      ++c0;
      continue;
    }
    switch (dtype_class(data + off[r], off[r + 1] - off[r])) {
      case 1: ++c1; break;
      case 2: ++c2; break;
      case 3: ++c3; break;
      default: ++c4; break;
    }
  }
  out5[0] = c0;
  out5[1] = c1;
  out5[2] = c2;
  out5[3] = c3;
  out5[4] = c4;
}

/* MutualInformation of two utf8 columns (M/analyzers/MutualInformation.scala:41-84): the joint
 * frequencies of the rows where both are non-NULL (a hash-partitioned aggregation, as or_freq), the
 * two marginals re-aggregated from the joint groups, and the sum over the joint groups of
 * (c/n) ln((c/n) / ((cx/n)(cy/n))) with n = num_rows, partition partials added in partition order. */
typedef struct {
  int64_t row, c;
} or_group;

static inline uint64_t utf8_hash(const int32_t* off, const uint8_t* data, int64_t r, uint64_t seed) {
  return or_xxh64(data + off[r], off[r + 1] - off[r], seed);
}
static inline int utf8_eq(const int32_t* off, const uint8_t* data, int64_t a, int64_t b) {
  const int32_t la = off[a + 1] - off[a], lb = off[b + 1] - off[b];
  return la == lb && memcmp(data + off[a], data + off[b], (size_t)la) == 0;
}

/* counts per distinct value of column (off, data) over the rows `rows[0..m)` weighted by w[]:
 * a hash table of representative rows; returns the number of groups, fills grow/gcnt */
static int64_t agg_rows(const int32_t* off, const uint8_t* data, const int64_t* rows,
                        const int64_t* w, int64_t m, int64_t* grow, int64_t* gcnt, int64_t* slot_of) {
  size_t cap = 16;
  while (cap < (size_t)m * 2) cap <<= 1;
  int64_t* trow = (int64_t*)malloc(cap * sizeof(int64_t));
  int64_t* tidx = (int64_t*)malloc(cap * sizeof(int64_t));
  uint64_t* th = (uint64_t*)malloc(cap * sizeof(uint64_t));
  for (size_t i = 0; i < cap; ++i) trow[i] = -1;
  int64_t g = 0;
  for (int64_t i = 0; i < m; ++i) {
    const int64_t r = rows[i];
    const uint64_t h = utf8_hash(off, data, r, 0);
    size_t s = (size_t)(h & (cap - 1));
    for (;;) {
      if (trow[s] < 0) {
        trow[s] = r;
        th[s] = h;
        tidx[s] = g;
        grow[g] = r;
        gcnt[g] = w ? w[i] : 1;
        slot_of[i] = g++;
        break;
      }
      if (th[s] == h && utf8_eq(off, data, trow[s], r)) {
        gcnt[tidx[s]] += w ? w[i] : 1;
        slot_of[i] = tidx[s];
        break;
      }
      s = (s + 1) & (cap - 1);
    }
  }
  free(trow);
  free(tidx);
  free(th);
  return g;
}

double or_mi_utf8(const int32_t* off1, const uint8_t* d1, const uint8_t* v1, const int32_t* off2,
                  const uint8_t* d2, const uint8_t* v2, int64_t n, int64_t num_rows, int nthreads) {
  /* joint rows by the hash of (x, y): P partitions, then per partition the joint groups */
  const int P = 256;
  int64_t* rows = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
  uint64_t* hs = (uint64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
  int64_t* cnt = (int64_t*)calloc((size_t)nthreads * P, sizeof(int64_t));
#pragma omp parallel num_threads(nthreads)
  {
    const int t = omp_get_thread_num();
    const int64_t r0 = n * t / nthreads, r1 = n * (t + 1) / nthreads;
    for (int64_t r = r0; r < r1; ++r) {
      if (!bit(v1, r) || !bit(v2, r)) {
        hs[r] = 0;
        continue;
      }
      hs[r] = utf8_hash(off1, d1, r, 0) * 31 + utf8_hash(off2, d2, r, 1);
      ++cnt[(size_t)t * P + (hs[r] >> 56)];
    }
  }
  int64_t* base = (int64_t*)malloc((size_t)nthreads * P * sizeof(int64_t));
  int64_t* pbeg = (int64_t*)malloc((size_t)(P + 1) * sizeof(int64_t));
  int64_t acc = 0;
  for (int p = 0; p < P; ++p) {
    pbeg[p] = acc;
    for (int t = 0; t < nthreads; ++t) {
      base[(size_t)t * P + p] = acc;
      acc += cnt[(size_t)t * P + p];
    }
  }
  pbeg[P] = acc;
#pragma omp parallel num_threads(nthreads)
  {
    const int t = omp_get_thread_num();
    const int64_t r0 = n * t / nthreads, r1 = n * (t + 1) / nthreads;
    int64_t* b = base + (size_t)t * P;
    for (int64_t r = r0; r < r1; ++r)
      if (bit(v1, r) && bit(v2, r)) rows[b[hs[r] >> 56]++] = r;
  }
  /* joint groups (representative row, count), partition by partition */
  or_group* jg = (or_group*)malloc((size_t)(acc > 0 ? acc : 1) * sizeof(or_group));
  int64_t* jn = (int64_t*)calloc(P, sizeof(int64_t));
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
  for (int p = 0; p < P; ++p) {
    const int64_t m = pbeg[p + 1] - pbeg[p];
    size_t cap = 16;
    while (cap < (size_t)m * 2) cap <<= 1;
    int64_t* trow = (int64_t*)malloc(cap * sizeof(int64_t));
    int64_t* tix = (int64_t*)malloc(cap * sizeof(int64_t));
    for (size_t i = 0; i < cap; ++i) trow[i] = -1;
    or_group* out = jg + pbeg[p];
    int64_t g = 0;
    for (int64_t i = pbeg[p]; i < pbeg[p + 1]; ++i) {
      const int64_t r = rows[i];
      size_t s = (size_t)(hs[r] & (cap - 1));
      for (;;) {
        if (trow[s] < 0) {
          trow[s] = r;
          tix[s] = g;
          out[g].row = r;
          out[g].c = 1;
          ++g;
          break;
        }
        const int64_t q = trow[s];
        if (hs[q] == hs[r] && utf8_eq(off1, d1, q, r) && utf8_eq(off2, d2, q, r)) {
          ++out[tix[s]].c;
          break;
        }
        s = (s + 1) & (cap - 1);
      }
    }
    jn[p] = g;
    free(trow);
    free(tix);
  }
  /* compact the joint groups; the marginals from them (weighted by the joint counts) */
  int64_t G = 0;
  for (int p = 0; p < P; ++p) {
    memmove(jg + G, jg + pbeg[p], (size_t)jn[p] * sizeof(or_group));
    G += jn[p];
  }
  int64_t* grows = (int64_t*)malloc((size_t)(G > 0 ? G : 1) * 8);
  int64_t* gw = (int64_t*)malloc((size_t)(G > 0 ? G : 1) * 8);
  for (int64_t i = 0; i < G; ++i) {
    grows[i] = jg[i].row;
    gw[i] = jg[i].c;
  }
  int64_t* mrow = (int64_t*)malloc((size_t)(G > 0 ? G : 1) * 8);
  int64_t* mx = (int64_t*)malloc((size_t)(G > 0 ? G : 1) * 8);
  int64_t* my = (int64_t*)malloc((size_t)(G > 0 ? G : 1) * 8);
  int64_t* sx = (int64_t*)malloc((size_t)(G > 0 ? G : 1) * 8);
  int64_t* sy = (int64_t*)malloc((size_t)(G > 0 ? G : 1) * 8);
  agg_rows(off1, d1, grows, gw, G, mrow, mx, sx);
  agg_rows(off2, d2, grows, gw, G, mrow, my, sy);
  const double tot = (double)num_rows;
  double* pe = (double*)calloc((size_t)nthreads, sizeof(double));
#pragma omp parallel num_threads(nthreads)
  {
    const int t = omp_get_thread_num();
    const int64_t i0 = G * t / nthreads, i1 = G * (t + 1) / nthreads;
    double e = 0.0;
    for (int64_t i = i0; i < i1; ++i) {
      const double pxy = (double)gw[i] / tot, px = (double)mx[sx[i]] / tot, py = (double)my[sy[i]] / tot;
      e += pxy * log(pxy / (px * py));
    }
    pe[t] = e;
  }
  double mi = 0.0;
  for (int t = 0; t < nthreads; ++t) mi += pe[t];
  free(pe);
  free(sy);
  free(sx);
  free(my);
  free(mx);
  free(mrow);
  free(gw);
  free(grows);
  free(jn);
  free(jg);
  free(pbeg);
  free(base);
  free(cnt);
  free(hs);
  free(rows);
  return mi;
}
