// CPU check of the group-key codec (deequ_amd/csrc/freq_codec.h) -- the same DQ_HD functions the
// group-by kernels run, built for the host with g++ (under ASan by tests/test_freq_codec.py).
//
// Inputs mirror the GPU tests' tables: a 1-row (int64 = INT64_MIN, string) key -- the row the
// round-1 mixed-key grouping faulted on -- and seeded 5000-row (int64, string) / (string, string)
// / (int32, double, string) tables with NULLs, empty strings and long strings, in grouping and in
// Histogram ("NullValue") mode.  For every pair of rows, rows_equal must agree with equality of
// the encoded keys; the encoded size, the hash of the encoding and the row hash must agree; and
// fmix_inv must invert fmix_bij.  Prints "OK <checks>" and exits 0, or the first failure.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "../deequ_amd/csrc/freq_codec.h"

using namespace dq;

struct HostCol {
  int32_t type;
  std::vector<uint8_t> valid;  // empty = no NULLs
  std::vector<uint8_t> values;
  std::vector<uint8_t> data;
  KeyCol view() const {
    return KeyCol{type, 0, valid.empty() ? nullptr : valid.data(), values.data(),
                  data.empty() ? nullptr : data.data()};
  }
};

static long checks = 0;
#define CHECK(c, ...)                          \
  do {                                         \
    ++checks;                                  \
    if (!(c)) {                                \
      printf("FAIL %s:%d: ", __FILE__, __LINE__); \
      printf(__VA_ARGS__);                     \
      printf("\n");                            \
      exit(1);                                 \
    }                                          \
  } while (0)

static void set_valid(HostCol& c, int64_t n, const std::vector<bool>& nulls) {
  bool any = false;
  for (bool b : nulls) any |= b;
  if (!any) return;
  c.valid.assign((n + 7) / 8 + 16, 0);
  for (int64_t r = 0; r < n; ++r)
    if (!nulls[r]) c.valid[r >> 3] |= (uint8_t)(1u << (r & 7));
}

static HostCol int64_col(const std::vector<int64_t>& v, const std::vector<bool>& nulls) {
  HostCol c;
  c.type = DQ_INT64;
  c.values.resize(v.size() * 8 + 16);  // exact size + padding, like the device tables
  memcpy(c.values.data(), v.data(), v.size() * 8);
  set_valid(c, (int64_t)v.size(), nulls);
  return c;
}
static HostCol int32_col(const std::vector<int32_t>& v, const std::vector<bool>& nulls) {
  HostCol c;
  c.type = DQ_INT32;
  c.values.resize(v.size() * 4 + 16);
  memcpy(c.values.data(), v.data(), v.size() * 4);
  set_valid(c, (int64_t)v.size(), nulls);
  return c;
}
static HostCol f64_col(const std::vector<double>& v, const std::vector<bool>& nulls) {
  HostCol c;
  c.type = DQ_FLOAT64;
  c.values.resize(v.size() * 8 + 16);
  memcpy(c.values.data(), v.data(), v.size() * 8);
  set_valid(c, (int64_t)v.size(), nulls);
  return c;
}
static HostCol str_col(const std::vector<std::string>& v, const std::vector<bool>& nulls) {
  HostCol c;
  c.type = DQ_UTF8;
  std::vector<int32_t> off(v.size() + 1, 0);
  for (size_t i = 0; i < v.size(); ++i) {
    off[i + 1] = off[i] + (int32_t)(nulls[i] ? 0 : v[i].size());
    if (!nulls[i]) c.data.insert(c.data.end(), v[i].begin(), v[i].end());
  }
  c.values.resize(off.size() * 4);
  memcpy(c.values.data(), off.data(), off.size() * 4);
  // no padding after the character bytes: reads past a string's end would trip ASan
  if (c.data.empty()) c.data.push_back(0);
  set_valid(c, (int64_t)v.size(), nulls);
  return c;
}

static void check_table(const std::vector<HostCol>& cols, int64_t n, int null_as_group,
                        bool all_pairs) {
  KeySet ks;
  memset(&ks, 0, sizeof(ks));
  ks.n_keys = (int32_t)cols.size();
  ks.null_as_group = null_as_group;
  int32_t types[kMaxKeys] = {0};
  for (size_t k = 0; k < cols.size(); ++k) {
    ks.cols[k] = cols[k].view();
    types[k] = cols[k].type;
  }
  const bool exact = cols.size() == 1 && cols[0].type != DQ_UTF8;
  std::vector<std::vector<uint32_t>> enc(n);
  std::vector<int> kind(n);
  std::vector<uint64_t> h(n);
  for (int64_t r = 0; r < n; ++r) {
    kind[r] = row_kind(ks, r, exact);
    if (kind[r] != ROW_KEY) continue;
    if (exact) {
      h[r] = row_hash_exact(ks, r);
      const uint64_t v = exact_key(ks, r);
      CHECK(fmix_inv(h[r]) == v, "fmix_inv row %lld", (long long)r);
      continue;
    }
    const uint32_t sz = row_enc_size(ks, r);
    CHECK(sz % 4 == 0, "size %u not a multiple of 4", sz);
    enc[r].assign(sz / 4 + 1, 0xDEADBEEFu);  // one guard word
    row_encode(ks, r, enc[r].data());
    CHECK(enc[r][sz / 4] == 0xDEADBEEFu, "row_encode wrote past row_enc_size (row %lld)",
          (long long)r);
    enc[r].pop_back();
    CHECK(enc_size(enc[r].data(), types, ks.n_keys) == sz, "enc_size row %lld", (long long)r);
    h[r] = row_hash_hashed(ks, r);
    if (ks.n_keys == 1 && types[0] == DQ_UTF8) {  // phase A's one-column fast path
      SView v;
      CHECK(key_str(ks, 0, r, v), "key_str on a keyed row");
      CHECK(str_row_hash(v) == h[r], "str_row_hash != row_hash_hashed, row %lld", (long long)r);
      if (v.p && v.len <= 16) {  // phase A's register path: aligned-dword loads, then hash
        for (int shift = 0; shift < 4; ++shift) {
          // the device reads whole aligned dwords: give the copy the room a page would
          alignas(8) uint8_t room[40] = {0};
          memset(room, 0xEE, sizeof(room));
          memcpy(room + 4 + shift, v.p, v.len);
          uint64_t w0 = 0, w1 = 0;
          load_str16(room + 4 + shift, v.len, w0, w1);
          CHECK(str_row_hash_reg(w0, w1, v.len) == h[r], "str_row_hash_reg row %lld shift %d",
                (long long)r, shift);
          uint64_t a0, a1, b0, b1;
          str_short_key_reg(w0, w1, v.len, a0, a1);
          str_short_key(v, b0, b1);
          CHECK(a0 == b0 && a1 == b1, "str_short_key_reg row %lld", (long long)r);
          if (a1 != kNoShort) {  // phase A encodes a short key from its short form
            std::vector<uint32_t> e(enc[r].size() + 1, 0xDEADBEEFu);
            str1_encode_short(a0, a1, e.data());
            CHECK(e.back() == 0xDEADBEEFu, "str1_encode_short wrote past the key (row %lld)",
                  (long long)r);
            e.pop_back();
            CHECK(e == enc[r], "str1_encode_short != row_encode, row %lld", (long long)r);
          }
        }
      }
    }
    CHECK(enc_hash(enc[r].data(), types, ks.n_keys) == h[r], "enc_hash != row hash, row %lld",
          (long long)r);
  }
  std::mt19937_64 rng(n * 31 + cols.size());
  const int64_t pairs = all_pairs ? n * n : 200000;
  for (int64_t q = 0; q < pairs; ++q) {
    const int64_t a = all_pairs ? q / n : (int64_t)(rng() % n);
    const int64_t b = all_pairs ? q % n : (int64_t)(rng() % n);
    if (kind[a] != ROW_KEY || kind[b] != ROW_KEY || exact) continue;
    const bool eq = rows_equal(ks, a, b);
    const bool enc_eq = enc[a] == enc[b];
    CHECK(eq == enc_eq, "rows_equal(%lld,%lld)=%d but encodings equal=%d", (long long)a,
          (long long)b, (int)eq, (int)enc_eq);
    CHECK(eq == enc_equal(enc[a].data(), enc[b].data(), types, ks.n_keys), "enc_equal");
    if (eq) CHECK(h[a] == h[b], "equal rows, different hashes");
    if (ks.n_keys == 1 && types[0] == DQ_UTF8) {  // short forms decide equality when either is short
      SView va, vb;
      key_str(ks, 0, a, va);
      key_str(ks, 0, b, vb);
      uint64_t a0, a1, b0, b1;
      str_short_key(va, a0, a1);
      str_short_key(vb, b0, b1);
      if (a1 != kNoShort || b1 != kNoShort)
        CHECK((a0 == b0 && a1 == b1) == eq, "short keys of rows %lld, %lld disagree with rows_equal",
              (long long)a, (long long)b);
    }
  }
}

// TK_HLL's register path for utf8 (scan.hip hll_str_rows): the aligned dwords that hold a string
// of <= 64 bytes (the last one repeated up to 17), realigned by alignbyte, hashed by
// xxh_bytes_regs64 -- equal to xxh_bytes (Spark's hashUnsafeBytes) at every length and alignment.
static void check_hll_regs() {
  std::mt19937_64 g(5);
  for (int len = 0; len <= 64; ++len) {
    for (int shift = 0; shift < 4; ++shift) {
      for (int rep = 0; rep < 20; ++rep) {
        alignas(8) uint8_t room[96];
        memset(room, 0xEE, sizeof(room));
        uint8_t* p = room + 4 + shift;
        for (int k = 0; k < len; ++k) p[k] = (uint8_t)g();
        const uint64_t want = xxh_bytes(HostBytes{p}, len, 42);
        const uint32_t* base = reinterpret_cast<const uint32_t*>(room + 4);
        const int nd = len > 0 ? (shift + len + 3) >> 2 : 0;
        uint32_t dw[17];
        for (int k = 0; k < 17; ++k) {
          dw[k] = 0;
          if (nd) memcpy(&dw[k], base + (k < nd - 1 ? k : nd - 1), 4);
        }
        uint32_t w[16];
        for (int j = 0; j < 16; ++j) {  // __builtin_amdgcn_alignbyte(dw[j + 1], dw[j], shift)
          const uint64_t both = ((uint64_t)dw[j + 1] << 32) | dw[j];
          w[j] = (uint32_t)(both >> (8 * shift));
        }
        CHECK(xxh_bytes_regs64(w, len, 42) == want, "xxh_bytes_regs64 len %d shift %d", len, shift);
      }
    }
  }
}

int main() {
  // fmix is a bijection with the stated inverse
  std::mt19937_64 rng(7);
  for (int i = 0; i < 100000; ++i) {
    const uint64_t x = rng();
    CHECK(fmix_inv(fmix_bij(x)) == x, "fmix_inv");
  }
  CHECK(code_count((2u << 2) | 3u) == 48, "code_count");
  check_hll_regs();
  // the round-1 fault input: one row, (int64 INT64_MIN, "high")
  for (int nag = 0; nag < 1; ++nag) {
    std::vector<HostCol> c = {int64_col({INT64_MIN}, {false}), str_col({"high"}, {false})};
    check_table(c, 1, nag, true);
  }
  // seeded 5000-row tables
  const int64_t n = 5000;
  std::mt19937_64 g(11);
  const char* words[] = {"high", "low", "medium", "", "NullValue", "Thingy qqqqqqqqqqqqqqqqqqqqqqqqqqqqqq",
                         "1234567", "12345678", "abc\0", "abc", "0123456789abcdef", "0123456789abcde",
                         "0123456789abcdefg"};
  std::vector<int64_t> ids(n);
  std::vector<int32_t> i32(n);
  std::vector<double> dbl(n);
  std::vector<std::string> s(n), u(n);
  std::vector<bool> n1(n), n2(n), n3(n), none(n, false);
  for (int64_t r = 0; r < n; ++r) {
    ids[r] = r < 3 ? INT64_MIN : (int64_t)(g() % (n / 2));
    i32[r] = (int32_t)(g() % 7) - 3;
    const double dv[] = {0.0, -0.0, 1.5, -2.25, 1e300};
    dbl[r] = dv[g() % 5];
    {
      const int w = (int)(g() % 13);  // word 8 holds an embedded NUL byte
      s[r] = w == 8 ? std::string("abc\0", 4) : std::string(words[w]);
    }
    u[r] = "u" + std::to_string(g() % n);
    n1[r] = g() % 20 == 0;
    n2[r] = g() % 20 == 0;
    n3[r] = g() % 20 == 0;
  }
  check_table({int64_col(ids, n1)}, n, 0, false);
  check_table({int64_col(ids, n1)}, n, 1, false);
  check_table({int64_col(ids, n1), str_col(s, n2)}, n, 0, false);
  check_table({str_col(s, n2), str_col(u, n3)}, n, 0, false);
  check_table({int32_col(i32, n1), f64_col(dbl, n2), str_col(s, n3)}, n, 0, false);
  check_table({str_col(s, n2)}, n, 1, false);  // Histogram: NULL == "NullValue"
  check_table({str_col(s, none)}, n, 0, false);
  {  // NULL and "NullValue" are one Histogram group
    std::vector<HostCol> c = {str_col({"NullValue", "x"}, {false, true})};
    KeySet ks;
    memset(&ks, 0, sizeof(ks));
    ks.n_keys = 1;
    ks.null_as_group = 1;
    ks.cols[0] = c[0].view();
    CHECK(rows_equal(ks, 0, 1), "NULL must equal \"NullValue\" in Histogram mode");
    CHECK(row_hash_hashed(ks, 0) == row_hash_hashed(ks, 1), "NullValue hash");
  }
  printf("OK %ld\n", checks);
  return 0;
}
