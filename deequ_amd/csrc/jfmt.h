// jfmt.h -- Java's Double.toString / Float.toString (what Spark 2.2's Cast(DoubleType|FloatType ->
// StringType) calls, Cast.scala castToString -> UTF8String.fromString(d.toString)) for host and
// device code.  Used where deequ matches or classifies a floating-point column as text:
// PatternMatch / RLIKE (PatternMatch.scala:44-48, regexp_extract over the implicit cast).
//
// Digits: the shortest decimal that rounds back to the value, nearest of those to the exact value
// (Adams' Ryu, PLDI 2018 -- the d2d step, restated for both IEEE formats over one 125-bit table,
// ryu_tables.h).  Layout, from java.lang.Double.toString's javadoc: NaN, Infinity, -Infinity,
// 0.0 / -0.0; plain "ddd.ddd" (at least one fraction digit) when the leading digit's exponent E
// is in [-3, 6], i.e. 1e-3 <= |x| < 1e7; otherwise "d.dddE<E>" (at least one fraction digit).
//
// Parity: JDK 8's FloatingDecimal is not always shortest (JDK-4511638, fixed in JDK 19): for a
// small set of values it prints a longer digit string that still reads back to the same double.
// Those values, and subnormals whose shortest form is one digit (FloatingDecimal's estimator prints
// Double.MIN_VALUE as 4.9E-324 -- restated below -- and the others are not documented), are
// parity unpinned.
#pragma once

#include <stdint.h>

#include "ryu_tables.h"

#ifndef DQ_HD
#define DQ_HD __host__ __device__ __forceinline__
#endif

namespace dq {
namespace jfmt {

constexpr int kMaxChars = 26;  // "-1.2345678901234567E-308" is 24

DQ_HD int32_t pow5bits(int32_t e) { return ((e * 1217359) >> 19) + 1; }    // ceil(log2 5^e)
DQ_HD int32_t log10pow2(int32_t e) { return (e * 78913) >> 18; }           // floor(e log10 2)
DQ_HD int32_t log10pow5(int32_t e) { return (e * 732923) >> 20; }          // floor(e log10 5)

DQ_HD uint32_t pow5_factor(uint64_t v) {
  uint32_t c = 0;
  while (v && v % 5 == 0) {
    v /= 5;
    ++c;
  }
  return c;
}

// floor(m * mul / 2^j) for the 126-bit table entry mul = {lo, hi}, j >= 64.
DQ_HD uint64_t mul_shift(uint64_t m, const uint64_t* mul, int32_t j) {
  const unsigned __int128 b0 = (unsigned __int128)m * mul[0];
  const unsigned __int128 b2 = (unsigned __int128)m * mul[1];
  return (uint64_t)(((b0 >> 64) + b2) >> (j - 64));
}

struct Decimal {
  uint64_t digits;  // significand, no trailing zeros beyond what the shortest form needs
  int32_t exp10;    // value = digits * 10^exp10
};

// Shortest round-trip decimal of a finite, non-zero IEEE value with MBITS fraction bits and
// exponent bias BIAS, given its raw fraction and biased exponent fields.
template <int MBITS, int BIAS>
DQ_HD Decimal shortest(uint64_t ieee_m, uint32_t ieee_e) {
  int32_t e2;
  uint64_t m2;
  if (ieee_e == 0) {
    e2 = 1 - BIAS - MBITS - 2;
    m2 = ieee_m;
  } else {
    e2 = (int32_t)ieee_e - BIAS - MBITS - 2;
    m2 = (1ULL << MBITS) | ieee_m;
  }
  const bool accept_bounds = (m2 & 1) == 0;  // round-half-even reading of the interval ends
  const uint64_t mv = 4 * m2;                // the value, in quarter units of 2^e2
  const uint32_t mm_shift = ieee_m != 0 || ieee_e <= 1;  // lower gap halves at a binade edge
  uint64_t vr, vp, vm;
  int32_t e10;
  bool vm_tz = false, vr_tz = false;  // the lower end / the value are exact at this e10
  if (e2 >= 0) {
    const int32_t q = log10pow2(e2) - (e2 > 3);
    e10 = q;
    const int32_t i = -e2 + q + kPow5InvBits + pow5bits(q) - 1;
    vr = mul_shift(mv, kPow5Inv[q], i);
    vp = mul_shift(mv + 2, kPow5Inv[q], i);
    vm = mul_shift(mv - 1 - mm_shift, kPow5Inv[q], i);
    if (q <= 21) {  // beyond, 5^q cannot divide a 55-bit number
      if (mv % 5 == 0) vr_tz = pow5_factor(mv) >= (uint32_t)q;
      else if (accept_bounds) vm_tz = pow5_factor(mv - 1 - mm_shift) >= (uint32_t)q;
      else vp -= pow5_factor(mv + 2) >= (uint32_t)q;
    }
  } else {
    const int32_t q = log10pow5(-e2) - (-e2 > 1);
    e10 = q + e2;
    const int32_t i = -e2 - q;
    const int32_t j = q - (pow5bits(i) - kPow5Bits);
    vr = mul_shift(mv, kPow5[i], j);
    vp = mul_shift(mv + 2, kPow5[i], j);
    vm = mul_shift(mv - 1 - mm_shift, kPow5[i], j);
    if (q <= 1) {
      vr_tz = true;
      if (accept_bounds) vm_tz = mm_shift == 1;
      else --vp;
    } else if (q < 63) {
      vr_tz = (mv & ((1ULL << q) - 1)) == 0;  // mv * 5^i / 2^q is an integer
    }
  }
  // Drop digits while the interval (vm, vp) still holds a shorter decimal.
  int32_t removed = 0;
  uint32_t last = 0;
  uint64_t out;
  if (vm_tz || vr_tz) {
    while (vp / 10 > vm / 10) {
      vm_tz &= vm % 10 == 0;
      vr_tz &= last == 0;
      last = (uint32_t)(vr % 10);
      vr /= 10;
      vp /= 10;
      vm /= 10;
      ++removed;
    }
    if (vm_tz) {
      while (vm % 10 == 0) {
        vr_tz &= last == 0;
        last = (uint32_t)(vr % 10);
        vr /= 10;
        vp /= 10;
        vm /= 10;
        ++removed;
      }
    }
    if (vr_tz && last == 5 && vr % 2 == 0) last = 4;  // exact tie: round half even
    out = vr + ((vr == vm && (!accept_bounds || !vm_tz)) || last >= 5);
  } else {
    bool round_up = false;
    while (vp / 10 > vm / 10) {
      round_up = vr % 10 >= 5;
      vr /= 10;
      vp /= 10;
      vm /= 10;
      ++removed;
    }
    out = vr + (vr == vm || round_up);
  }
  return Decimal{out, e10 + removed};
}

DQ_HD int decimal_length(uint64_t v) {
  int n = 1;
  while (v >= 10) {
    v /= 10;
    ++n;
  }
  return n;
}

// Java's layout of a shortest decimal; returns the character count.
DQ_HD int java_layout(bool neg, Decimal d, char* buf) {
  char dig[20];
  const int nd = decimal_length(d.digits);
  uint64_t v = d.digits;
  for (int k = nd - 1; k >= 0; --k) {
    dig[k] = (char)('0' + v % 10);
    v /= 10;
  }
  const int32_t e = d.exp10 + nd - 1;  // exponent of the leading digit
  int n = 0;
  if (neg) buf[n++] = '-';
  if (e >= 0 && e < 7) {
    for (int k = 0; k <= e; ++k) buf[n++] = k < nd ? dig[k] : '0';
    buf[n++] = '.';
    if (nd > e + 1) {
      for (int k = e + 1; k < nd; ++k) buf[n++] = dig[k];
    } else {
      buf[n++] = '0';
    }
  } else if (e < 0 && e >= -3) {
    buf[n++] = '0';
    buf[n++] = '.';
    for (int k = -1; k > e; --k) buf[n++] = '0';
    for (int k = 0; k < nd; ++k) buf[n++] = dig[k];
  } else {
    buf[n++] = dig[0];
    buf[n++] = '.';
    if (nd > 1) {
      for (int k = 1; k < nd; ++k) buf[n++] = dig[k];
    } else {
      buf[n++] = '0';
    }
    buf[n++] = 'E';
    int32_t ae = e;
    if (e < 0) {
      buf[n++] = '-';
      ae = -e;
    }
    char t[4];
    int nt = 0;
    do {
      t[nt++] = (char)('0' + ae % 10);
      ae /= 10;
    } while (ae);
    while (nt) buf[n++] = t[--nt];
  }
  return n;
}

DQ_HD int copy_lit(const char* s, char* buf) {
  int n = 0;
  for (; s[n]; ++n) buf[n] = s[n];
  return n;
}

// Double.toString(x) into buf (kMaxChars); returns the length.
DQ_HD int double_to_java(double x, char* buf) {
  const uint64_t bits = __builtin_bit_cast(uint64_t, x);
  const bool neg = bits >> 63;
  const uint64_t m = bits & ((1ULL << 52) - 1);
  const uint32_t e = (uint32_t)(bits >> 52) & 0x7ffu;
  if (e == 0x7ffu) return copy_lit(m ? "NaN" : (neg ? "-Infinity" : "Infinity"), buf);
  if (e == 0 && m == 0) return copy_lit(neg ? "-0.0" : "0.0", buf);
  if (e == 0 && m == 1) return copy_lit(neg ? "-4.9E-324" : "4.9E-324", buf);  // Double.MIN_VALUE
  return java_layout(neg, shortest<52, 1023>(m, e), buf);
}

// Float.toString(x) into buf (kMaxChars); returns the length.
DQ_HD int float_to_java(float x, char* buf) {
  const uint32_t bits = __builtin_bit_cast(uint32_t, x);
  const bool neg = bits >> 31;
  const uint32_t m = bits & ((1u << 23) - 1);
  const uint32_t e = (bits >> 23) & 0xffu;
  if (e == 0xffu) return copy_lit(m ? "NaN" : (neg ? "-Infinity" : "Infinity"), buf);
  if (e == 0 && m == 0) return copy_lit(neg ? "-0.0" : "0.0", buf);
  if (e == 0 && m == 1) return copy_lit(neg ? "-1.4E-45" : "1.4E-45", buf);  // Float.MIN_VALUE
  return java_layout(neg, shortest<23, 127>(m, e), buf);
}

}  // namespace jfmt
}  // namespace dq
