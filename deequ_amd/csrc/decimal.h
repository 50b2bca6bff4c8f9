// decimal.h -- Spark 2.2 DecimalType / DateType / TimestampType arithmetic shared by the host
// runtime (api.cpp) and the kernels (scan.hip, expr.hip, freq.hip, quantile.hip).  Everything is
// __host__ __device__ so the value a kernel aggregates and the value the host finalises (a merged
// state, a Histogram key's text) come from the same code.
//
//   * A decimal value is its unscaled 128-bit two's-complement integer (Arrow decimal128, the
//     column's scale implied), as Spark's Decimal holds it at the column's DecimalType.
//   * dec_to_double is Spark's Cast(Decimal AS DOUBLE) = Decimal.toDouble =
//     java.math.BigDecimal.doubleValue: the double nearest to unscaled / 10^scale, ties to even.
//   * dec_format / date_format / ts_format are Spark's Cast(... AS STRING): BigDecimal.toString,
//     DateTimeUtils.dateToString ("yyyy-MM-dd") and timestampToString ("yyyy-MM-dd HH:mm:ss" and
//     the nanoseconds without trailing zeros) with UTC as the session time zone.
//   * dec_hash is XxHash64Function.hash of a Decimal (Spark's InterpretedHashFunction): hashLong of
//     the unscaled long for precision <= 18, else hashUnsafeBytes of
//     BigInteger.toByteArray (minimal big-endian two's complement).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine.h"

namespace dq {

struct Dec128 {
  uint64_t lo;
  int64_t hi;
};

DQ_HD bool dec_lt(Dec128 a, Dec128 b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
DQ_HD bool dec_is_neg(Dec128 a) { return a.hi < 0; }
// |a| as an unsigned 128-bit (lo, hi) pair (|INT128_MIN| = 2^127 fits unsigned)
DQ_HD void dec_abs(Dec128 a, uint64_t& lo, uint64_t& hi) {
  lo = a.lo;
  hi = (uint64_t)a.hi;
  if (a.hi < 0) {
    lo = ~lo + 1;
    hi = ~hi + (lo == 0 ? 1 : 0);
  }
}

// ------------------------------------------------------------------------------------------------
// 192-bit unsigned helpers (three little-endian limbs) for the exact quotient of dec_to_double
// ------------------------------------------------------------------------------------------------
struct U192 {
  uint64_t w[3];
};
DQ_HD int u192_bitlen(const U192& a) {
  for (int k = 2; k >= 0; --k)
    if (a.w[k]) return 64 * k + 64 - __builtin_clzll(a.w[k]);
  return 0;
}
DQ_HD bool u192_ge(const U192& a, const U192& b) {
  for (int k = 2; k >= 0; --k)
    if (a.w[k] != b.w[k]) return a.w[k] > b.w[k];
  return true;
}
DQ_HD void u192_sub(U192& a, const U192& b) {
  uint64_t borrow = 0;
  for (int k = 0; k < 3; ++k) {
    const uint64_t x = a.w[k], y = b.w[k];
    const uint64_t d = x - y - borrow;
    borrow = (x < y || (x == y && borrow)) ? 1 : 0;
    a.w[k] = d;
  }
}
DQ_HD U192 u192_shl(const U192& a, int s) {  // 0 <= s < 192
  U192 r{{0, 0, 0}};
  const int q = s >> 6, b = s & 63;
  for (int k = 2; k >= 0; --k) {
    if (k - q < 0) continue;
    uint64_t v = a.w[k - q] << b;
    if (b && k - q - 1 >= 0) v |= a.w[k - q - 1] >> (64 - b);
    r.w[k] = v;
  }
  return r;
}
DQ_HD U192 u192_shr1(const U192& a) {
  return U192{{(a.w[0] >> 1) | (a.w[1] << 63), (a.w[1] >> 1) | (a.w[2] << 63), a.w[2] >> 1}};
}
// 10^e as 192 bits (e <= 57 fits)
DQ_HD U192 pow10_192(int e) {
  U192 p{{1, 0, 0}};
  for (int k = 0; k < e; ++k) {
    // p *= 10 = (p << 3) + (p << 1)
    const U192 a = u192_shl(p, 3), b = u192_shl(p, 1);
    uint64_t c = 0;
    for (int j = 0; j < 3; ++j) {
      const uint64_t s = a.w[j] + b.w[j];
      const uint64_t c1 = s < a.w[j] ? 1 : 0;
      const uint64_t t = s + c;
      const uint64_t c2 = t < s ? 1 : 0;
      p.w[j] = t;
      c = c1 + c2;
    }
  }
  return p;
}

// Cast(Decimal AS DOUBLE): nearest double to (lo, hi) / 10^scale, ties to even (0 <= scale <= 38).
DQ_HD double dec_to_double(uint64_t lo_in, int64_t hi_in, int scale) {
  uint64_t lo, hi;
  const bool neg = hi_in < 0;
  dec_abs(Dec128{lo_in, hi_in}, lo, hi);
  if (lo == 0 && hi == 0) return 0.0;  // BigDecimal has no negative zero
  const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                          1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  if (hi == 0 && lo < (1ULL << 53) && scale <= 22) {
    // both operands exact: one IEEE division is correctly rounded (BigDecimal's fast path)
    const double v = (double)lo / p10[scale];
    return neg ? -v : v;
  }
  // exact: q = floor(N 2^sh / D) with 55..56 significant bits, plus a sticky remainder bit
  const U192 N{{lo, hi, 0}};
  const U192 D = pow10_192(scale);
  const int nb = u192_bitlen(N), db = u192_bitlen(D);
  const int sh = 55 + db - nb;
  U192 A = sh >= 0 ? u192_shl(N, sh) : N;
  U192 B = sh >= 0 ? D : u192_shl(D, -sh);
  uint64_t q = 0;
  U192 Bs = u192_shl(B, 56);
  for (int i = 56; i >= 0; --i) {
    q <<= 1;
    if (u192_ge(A, Bs)) {
      u192_sub(A, Bs);
      q |= 1;
    }
    Bs = u192_shr1(Bs);
  }
  const bool sticky = (A.w[0] | A.w[1] | A.w[2]) != 0;
  const int qb = 64 - __builtin_clzll(q);  // 55 or 56
  const int drop = qb - 53;
  const uint64_t half = 1ULL << (drop - 1);
  const uint64_t rem = q & ((1ULL << drop) - 1);
  uint64_t m = q >> drop;
  if (rem > half || (rem == half && (sticky || (m & 1)))) ++m;
  // value = m 2^(drop - sh) (m may have become 2^53: still exact in a double)
  const double v = ldexp((double)m, drop - sh);
  return neg ? -v : v;
}

// Number of decimal digits of an unsigned 128-bit value (1 for zero).
DQ_HD int u128_digits(uint64_t lo, uint64_t hi) {
  int d = 1;
  U192 p{{10, 0, 0}};
  const U192 v{{lo, hi, 0}};
  while (d < 39 && u192_ge(v, p)) {
    ++d;
    const U192 a = u192_shl(p, 3), b = u192_shl(p, 1);
    uint64_t c = 0;
    for (int j = 0; j < 3; ++j) {
      const uint64_t s = a.w[j] + b.w[j];
      const uint64_t c1 = s < a.w[j] ? 1 : 0;
      const uint64_t t = s + c;
      p.w[j] = t;
      c = c1 + (t < s ? 1 : 0);
    }
  }
  return d;
}

// (hi:lo) / d for hi < d (bit-serial: no 128-bit division on either side)
DQ_HD uint64_t udiv128_64(uint64_t hi, uint64_t lo, uint64_t d, uint64_t& rem) {
  uint64_t q = 0;
  for (int i = 63; i >= 0; --i) {
    const bool top = (hi >> 63) != 0;
    hi = (hi << 1) | (lo >> 63);
    lo <<= 1;
    q <<= 1;
    if (top || hi >= d) {
      hi -= d;
      q |= 1;
    }
  }
  rem = hi;
  return q;
}

// The decimal digits of an unsigned 128-bit value, most significant first; returns the count.
DQ_HD int u128_to_digits(uint64_t lo, uint64_t hi, char* out /* >= 40 */) {
  char tmp[40];
  int n = 0;
  const uint64_t kChunk = 10000000000000000000ULL;  // 10^19
  uint64_t chunks[3];
  int nc = 0;
  while (hi != 0) {
    uint64_t r;
    const uint64_t qh = hi / kChunk;
    const uint64_t ql = udiv128_64(hi % kChunk, lo, kChunk, r);
    chunks[nc++] = r;
    hi = qh;
    lo = ql;
  }
  chunks[nc++] = lo;
  // the top chunk without leading zeros, the others zero-padded to 19 digits
  for (int c = 0; c < nc; ++c) {
    uint64_t v = chunks[c];
    const bool top = c == nc - 1;
    int k = 0;
    do {
      tmp[n++] = (char)('0' + v % 10);
      v /= 10;
      ++k;
    } while (top ? v != 0 : k < 19);
  }
  for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
  return n;
}

constexpr int kFmtMax = 64;  // bytes of the longest text below (decimal: 49)

// java.math.BigDecimal.toString of unscaled / 10^scale (scale >= 0): plain when the adjusted
// exponent (digits - 1 - scale) is >= -6, else one digit, '.', the rest and "E-n".
DQ_HD int dec_format(uint64_t lo_in, int64_t hi_in, int scale, char* out) {
  uint64_t lo, hi;
  dec_abs(Dec128{lo_in, hi_in}, lo, hi);
  char dg[40];
  const int nd = u128_to_digits(lo, hi, dg);
  int n = 0;
  if (hi_in < 0) out[n++] = '-';
  const int adjusted = nd - 1 - scale;
  if (scale == 0) {
    for (int i = 0; i < nd; ++i) out[n++] = dg[i];
  } else if (adjusted >= -6) {
    if (nd > scale) {
      for (int i = 0; i < nd - scale; ++i) out[n++] = dg[i];
      out[n++] = '.';
      for (int i = nd - scale; i < nd; ++i) out[n++] = dg[i];
    } else {
      out[n++] = '0';
      out[n++] = '.';
      for (int i = 0; i < scale - nd; ++i) out[n++] = '0';
      for (int i = 0; i < nd; ++i) out[n++] = dg[i];
    }
  } else {
    out[n++] = dg[0];
    if (nd > 1) {
      out[n++] = '.';
      for (int i = 1; i < nd; ++i) out[n++] = dg[i];
    }
    out[n++] = 'E';
    out[n++] = '-';
    int e = -adjusted;
    char t[4];
    int k = 0;
    do {
      t[k++] = (char)('0' + e % 10);
      e /= 10;
    } while (e);
    while (k) out[n++] = t[--k];
  }
  return n;
}

// The adjusted exponent of BigDecimal.toString's layout (digits - 1 - scale), for DataType.
DQ_HD int dec_adjusted(uint64_t lo_in, int64_t hi_in, int scale) {
  uint64_t lo, hi;
  dec_abs(Dec128{lo_in, hi_in}, lo, hi);
  return u128_digits(lo, hi) - 1 - scale;
}

// Proleptic Gregorian civil date of a day count since 1970-01-01 (days_from_civil's inverse).
DQ_HD void civil_from_days(int64_t z, int64_t& y, int& m, int& d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  d = (int)(doy - (153 * mp + 2) / 5 + 1);
  m = (int)(mp < 10 ? mp + 3 : mp - 9);
  y = yoe + era * 400 + (m <= 2 ? 1 : 0);
}

DQ_HD int put_uint(char* out, int64_t v, int width) {  // zero-padded to `width`, v >= 0
  char t[24];
  int k = 0;
  do {
    t[k++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (k < width) t[k++] = '0';
  int n = 0;
  while (k) out[n++] = t[--k];
  return n;
}

// "yyyy-MM-dd" (SimpleDateFormat: the year of era, at least 4 digits)
DQ_HD int date_format(int64_t days, char* out) {
  int64_t y;
  int m, d;
  civil_from_days(days, y, m, d);
  int n = put_uint(out, y > 0 ? y : 1 - y, 4);
  out[n++] = '-';
  n += put_uint(out + n, m, 2);
  out[n++] = '-';
  n += put_uint(out + n, d, 2);
  return n;
}

// "yyyy-MM-dd HH:mm:ss" + ".<nanoseconds without trailing zeros>" unless they are zero
// (DateTimeUtils.timestampToString over toJavaTimestamp's floored seconds)
DQ_HD int ts_format(int64_t micros, char* out) {
  int64_t sec = micros / 1000000, us = micros % 1000000;
  if (us < 0) {
    us += 1000000;
    sec -= 1;
  }
  int64_t day = sec / 86400, sod = sec % 86400;
  if (sod < 0) {
    sod += 86400;
    day -= 1;
  }
  int n = date_format(day, out);
  out[n++] = ' ';
  n += put_uint(out + n, sod / 3600, 2);
  out[n++] = ':';
  n += put_uint(out + n, (sod / 60) % 60, 2);
  out[n++] = ':';
  n += put_uint(out + n, sod % 60, 2);
  if (us) {
    char t[9];
    put_uint(t, us * 1000, 9);
    int len = 9;
    while (len > 0 && t[len - 1] == '0') --len;
    out[n++] = '.';
    for (int i = 0; i < len; ++i) out[n++] = t[i];
  }
  return n;
}

// XxHash64Function.hash of a Decimal of precision p (StatefulHyperloglogPlus.scala:91)
DQ_HD uint64_t dec_hash(uint64_t lo, int64_t hi, int precision, uint64_t seed) {
  if (precision <= 18) return xxh_long(lo, seed);
  // BigInteger.toByteArray: the minimal big-endian two's complement (bitLength / 8 + 1 bytes)
  const uint64_t mlo = hi < 0 ? ~lo : lo, mhi = hi < 0 ? ~(uint64_t)hi : (uint64_t)hi;
  const int bitlen = mhi ? 128 - __builtin_clzll(mhi) : (mlo ? 64 - __builtin_clzll(mlo) : 0);
  const int len = bitlen / 8 + 1;
  uint8_t be[16];
  for (int i = 0; i < len; ++i) {
    const int byte = len - 1 - i;  // little-endian byte index of big-endian position i
    be[i] = byte < 8 ? (uint8_t)(lo >> (8 * byte)) : (uint8_t)((uint64_t)hi >> (8 * (byte - 8)));
  }
  struct Rd {
    const uint8_t* p;
    DQ_HD uint64_t u64(int64_t o) const {
      uint64_t v = 0;
      for (int k = 7; k >= 0; --k) v = (v << 8) | p[o + k];
      return v;
    }
    DQ_HD uint32_t u32(int64_t o) const {
      uint32_t v = 0;
      for (int k = 3; k >= 0; --k) v = (v << 8) | p[o + k];
      return v;
    }
    DQ_HD uint32_t u8(int64_t o) const { return p[o]; }
  };
  return xxh_bytes(Rd{be}, len, seed);
}

// Does the 192-bit two's-complement sum (s0, s1, s2) fit decimal(min(p + 10, 38), s), i.e.
// |sum| < 10^min(p + 10, 38)?  (Spark 2.2's Sum result type, Sum.scala:35 over Spark's Sum)
DQ_HD bool dec_sum_fits(uint64_t s0, uint64_t s1, uint64_t s2, int precision) {
  const int rp = precision + 10 < 38 ? precision + 10 : 38;
  U192 m{{s0, s1, s2}};
  if ((int64_t)s2 < 0) {  // negate
    m.w[0] = ~m.w[0];
    m.w[1] = ~m.w[1];
    m.w[2] = ~m.w[2];
    uint64_t c = 1;
    for (int k = 0; k < 3; ++k) {
      m.w[k] += c;
      c = (c && m.w[k] == 0) ? 1 : 0;
    }
  }
  return !u192_ge(m, pow10_192(rp));
}

// Correctly rounded double of a 192-bit two's-complement sum over 10^scale (a Sum's cast; the
// sum fits decimal(38) when it is used, so the top limb is only sign extension or small).
DQ_HD double dec192_to_double(uint64_t s0, uint64_t s1, uint64_t s2, int scale) {
  // a sum that passed dec_sum_fits is < 10^38 < 2^127: the 128-bit path is exact
  (void)s2;
  return dec_to_double(s0, (int64_t)s1, scale);
}

}  // namespace dq
