// expr.hip -- the generic predicate interpreter: materialises a `where` filter or a Compliance
// predicate that the planner could not fuse into a column task as two Arrow boolean bitmaps (value
// bits, validity bits), with Spark SQL three-valued logic (Analyzers.conditionalSelection,
// Analyzer.scala:385-408; Compliance.scala:37-53).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device_util.h"
#include "kernels.h"
#include "jfmt.h"

namespace dq {

// ------------------------------------------------------------------------------------------------
// Generic predicate evaluation (the slow path for expressions that the planner cannot fuse):
// a postfix program over typed values with Kleene logic; one lane per row, results ballot-packed
// into Arrow boolean bitmaps (value bits, validity bits).
// ------------------------------------------------------------------------------------------------
struct V {
  int32_t tag;  // 0 NULL, 1 BOOL, 2 I64, 3 F64, 4 STR, 5 DECIMAL (i = low word, d = high word's
                // bits, len = scale), 6 DATE (i = days), 7 TIMESTAMP (i = microseconds)
  int32_t len;
  int64_t i;
  double d;
  const uint8_t* p;
};

DQ_DEV int cmp_str(const uint8_t* a, int32_t la, const uint8_t* b, int32_t lb) {
  DevBytes ra{a}, rb{b};
  int32_t n = la < lb ? la : lb;
  for (int32_t k = 0; k < n; ++k) {
    int32_t d = (int32_t)ra.u8(k) - (int32_t)rb.u8(k);
    if (d) return d < 0 ? -1 : 1;
  }
  return la == lb ? 0 : (la < lb ? -1 : 1);
}

// three-way compare of two non-NULL values; returns 2 when incomparable
DQ_DEV int cmp_vals(const V& a, const V& b) {
  if (a.tag == 5 && b.tag == 5) {  // unscaled at one scale (the plan aligns a literal's scale)
    const int64_t ah = __builtin_bit_cast(int64_t, a.d), bh = __builtin_bit_cast(int64_t, b.d);
    if (ah != bh) return ah < bh ? -1 : 1;
    if (a.i == b.i) return 0;
    return (uint64_t)a.i < (uint64_t)b.i ? -1 : 1;
  }
  if (a.tag >= 5 || b.tag >= 5) return 2;  // (dq_plan_create admits no other pairing)
  if (a.tag == 4 && b.tag == 4) return cmp_str(a.p, a.len, b.p, b.len);
  if (a.tag == 4 || b.tag == 4) return 2;
  if (a.tag == 3 || b.tag == 3) {
    double x = a.tag == 3 ? a.d : (double)a.i, y = b.tag == 3 ? b.d : (double)b.i;
    return cmp3_f64(x, y);
  }
  return cmp3_i64(a.i, b.i);
}

// Java Double.parseDouble subset (what Spark 2.2's Cast(StringType -> DoubleType) calls): trims
// ASCII whitespace/control chars, sign, digits, '.', exponent, optional [dDfF] suffix, NaN,
// Infinity.  Correctly rounded when the decimal significand < 2^53 and |exp10| <= 22; otherwise the
// nearest of two roundings (documented).  Returns false when the string is not a number -> NULL.
DQ_DEV bool parse_f64(const uint8_t* s, int32_t len, double& out) {
  DevBytes rd{s};
  int32_t b = 0, e = len;
  while (b < e && rd.u8(b) <= 32) ++b;
  while (e > b && rd.u8(e - 1) <= 32) --e;
  if (b >= e) return false;
  bool neg = false;
  uint32_t c = rd.u8(b);
  if (c == '+' || c == '-') {
    neg = c == '-';
    ++b;
  }
  if (e - b == 3 && rd.u8(b) == 'N' && rd.u8(b + 1) == 'a' && rd.u8(b + 2) == 'N') {
    out = __builtin_nan("");
    return true;
  }
  if (e - b == 8) {
    const char* inf = "Infinity";
    bool ok = true;
    for (int k = 0; k < 8; ++k) ok &= rd.u8(b + k) == (uint32_t)inf[k];
    if (ok) {
      out = neg ? -__builtin_inf() : __builtin_inf();
      return true;
    }
  }
  if (e > b) {
    uint32_t last = rd.u8(e - 1);
    if (last == 'd' || last == 'D' || last == 'f' || last == 'F') --e;
  }
  uint64_t mant = 0;
  int digits = 0, exp10 = 0;
  bool any = false, dot = false, overflow_digits = false;
  int32_t k = b;
  for (; k < e; ++k) {
    c = rd.u8(k);
    if (c >= '0' && c <= '9') {
      any = true;
      if (mant < 100000000000000000ULL) {
        mant = mant * 10 + (c - '0');
        if (mant) ++digits;
        if (dot) --exp10;
      } else {
        overflow_digits = true;
        if (!dot) ++exp10;
      }
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (!any) return false;
  if (k < e) {
    c = rd.u8(k);
    if (c != 'e' && c != 'E') return false;
    ++k;
    bool eneg = false;
    if (k < e && (rd.u8(k) == '+' || rd.u8(k) == '-')) {
      eneg = rd.u8(k) == '-';
      ++k;
    }
    if (k >= e) return false;
    int ev = 0;
    for (; k < e; ++k) {
      c = rd.u8(k);
      if (c < '0' || c > '9') return false;
      if (ev < 100000) ev = ev * 10 + (c - '0');
    }
    exp10 += eneg ? -ev : ev;
  }
  (void)overflow_digits;
  (void)digits;
  double v = (double)mant;
  const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                          1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  if (exp10 >= 0) {
    while (exp10 > 22) {
      v *= 1e22;
      exp10 -= 22;
    }
    v *= p10[exp10];
  } else {
    while (exp10 < -22) {
      v /= 1e22;
      exp10 += 22;
    }
    v /= p10[-exp10];
  }
  out = neg ? -v : v;
  return true;
}

__global__ void __launch_bounds__(kBlock) expr_kernel(const XInstr* __restrict__ prog, int n_instr,
                                                      const DevCol* __restrict__ cols,
                                                      const uint8_t* __restrict__ pool, int64_t rows,
                                                      uint64_t* __restrict__ out_val,
                                                      uint64_t* __restrict__ out_vld) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
  const int64_t n_words = (rows + 63) >> 6;
  for (int64_t w = wave; w < n_words; w += n_waves) {
    const int64_t r = w * 64 + lane;
    V st[kMaxStack];
    int sp = 0;
    bool in_range = r < rows;
    if (in_range) {
      for (int pc = 0; pc < n_instr; ++pc) {
        const XInstr ins = prog[pc];
        switch (ins.op) {
          case XI_COL: {
            const DevCol& c = cols[ins.a];
            V v{};
            const int tid = DQ_TYPE_ID(c.type);
            if (!bit1(c.valid, r)) {
              v.tag = 0;
            } else if (tid == DQ_DECIMAL128) {
              const uint64_t* dv = reinterpret_cast<const uint64_t*>(c.values) + 2 * r;
              v.tag = 5;
              v.i = (int64_t)dv[0];
              v.d = __builtin_bit_cast(double, dv[1]);
              v.len = DQ_DECIMAL_SCALE(c.type);
            } else if (tid == DQ_DATE32) {
              v.tag = 6;
              v.i = reinterpret_cast<const int32_t*>(c.values)[r];
            } else if (tid == DQ_TIMESTAMP_US) {
              v.tag = 7;
              v.i = reinterpret_cast<const int64_t*>(c.values)[r];
            } else if (c.type == DQ_UTF8) {
              const int32_t* off = reinterpret_cast<const int32_t*>(c.values);
              v.tag = 4;
              v.p = c.data + off[r];
              v.len = off[r + 1] - off[r];
            } else if (c.type == DQ_BOOL) {
              v.tag = 1;
              v.i = bit1(reinterpret_cast<const uint8_t*>(c.values), r);
            } else if (is_float_type(c.type)) {
              v.tag = 3;
              v.len = c.type == DQ_FLOAT32;  // the cast to string prints a float as Float.toString
              v.d = load_f64(c.type, c.values, r);
            } else {
              v.tag = 2;
              v.i = load_i64(c.type, c.values, r);
            }
            st[sp++] = v;
            break;
          }
          case XI_NULL: st[sp++] = V{0, 0, 0, 0.0, nullptr}; break;
          case XI_BOOL: st[sp++] = V{1, 0, ins.imm, 0.0, nullptr}; break;
          case XI_I64: st[sp++] = V{2, 0, ins.imm, 0.0, nullptr}; break;
          case XI_F64: st[sp++] = V{3, 0, 0, __builtin_bit_cast(double, ins.imm), nullptr}; break;
          case XI_DEC128: st[sp++] = V{5, 0, ins.imm, 0.0, nullptr}; break;
          case XI_DEC128_HI: st[sp - 1].d = __builtin_bit_cast(double, ins.imm); break;
          case XI_STR: st[sp++] = V{4, ins.a, 0, 0.0, pool + ins.imm}; break;
          case XI_IS_NULL: st[sp - 1] = V{1, 0, st[sp - 1].tag == 0 ? 1 : 0, 0.0, nullptr}; break;
          case XI_IS_NOT_NULL: st[sp - 1] = V{1, 0, st[sp - 1].tag != 0 ? 1 : 0, 0.0, nullptr}; break;
          case XI_NOT:
            if (st[sp - 1].tag != 0) st[sp - 1].i = st[sp - 1].i ? 0 : 1;
            break;
          case XI_AND: {
            V b = st[--sp];
            V a = st[sp - 1];
            // Kleene: FALSE dominates, then NULL
            bool af = a.tag != 0 && !a.i, bf = b.tag != 0 && !b.i;
            if (af || bf) st[sp - 1] = V{1, 0, 0, 0.0, nullptr};
            else if (a.tag == 0 || b.tag == 0) st[sp - 1] = V{0, 0, 0, 0.0, nullptr};
            else st[sp - 1] = V{1, 0, 1, 0.0, nullptr};
            break;
          }
          case XI_OR: {
            V b = st[--sp];
            V a = st[sp - 1];
            bool at = a.tag != 0 && a.i, bt = b.tag != 0 && b.i;
            if (at || bt) st[sp - 1] = V{1, 0, 1, 0.0, nullptr};
            else if (a.tag == 0 || b.tag == 0) st[sp - 1] = V{0, 0, 0, 0.0, nullptr};
            else st[sp - 1] = V{1, 0, 0, 0.0, nullptr};
            break;
          }
          case XI_CMP: {
            V b = st[--sp];
            V a = st[sp - 1];
            if (ins.a == DQ_X_EQ_NULL_SAFE) {
              int eq;
              if (a.tag == 0 || b.tag == 0) eq = (a.tag == 0 && b.tag == 0);
              else eq = cmp_vals(a, b) == 0;
              st[sp - 1] = V{1, 0, eq, 0.0, nullptr};
            } else if (a.tag == 0 || b.tag == 0) {
              st[sp - 1] = V{0, 0, 0, 0.0, nullptr};
            } else {
              int c = cmp_vals(a, b);
              if (c == 2) st[sp - 1] = V{0, 0, 0, 0.0, nullptr};
              else st[sp - 1] = V{1, 0, (op_mask(ins.a) >> (c + 1)) & 1, 0.0, nullptr};
            }
            break;
          }
          case XI_IN: {
            const int n = ins.a;
            const int base = sp - n - 1;
            V x = st[base];
            V res{0, 0, 0, 0.0, nullptr};
            if (x.tag != 0) {
              bool found = false, saw_null = false;
              for (int q = 0; q < n; ++q) {
                const V& it = st[base + 1 + q];
                if (it.tag == 0) {
                  saw_null = true;
                } else if (cmp_vals(x, it) == 0) {
                  found = true;
                }
              }
              if (found) res = V{1, 0, 1, 0.0, nullptr};
              else if (!saw_null) res = V{1, 0, 0, 0.0, nullptr};
            }
            sp = base;
            st[sp++] = res;
            break;
          }
          case XI_CAST_F64: {  // ins.a = 1: CAST AS FLOAT (rounded to float, prints as Float.toString)
            V& a = st[sp - 1];
            const bool to_f32 = ins.a != 0;
            if (a.tag == 2 || a.tag == 1) {
              a.d = to_f32 ? (double)(float)a.i : (double)a.i;  // (float)long: one rounding
              a.tag = 3;
            } else if (a.tag == 5) {  // Decimal.toDouble: correctly rounded
              a.d = dec_to_double((uint64_t)a.i, __builtin_bit_cast(int64_t, a.d), a.len);
              a.tag = 3;
            } else if (a.tag == 4) {
              double d;
              if (parse_f64(a.p, a.len, d)) a = V{3, 0, 0, d, nullptr};
              else a = V{0, 0, 0, 0.0, nullptr};
            } else if (a.tag == 3 && to_f32) {
              a.d = (double)(float)a.d;
            }
            // the type of the result decides how a regex prints it (Double / Float.toString)
            if (a.tag == 3) a.len = to_f32 ? 1 : 0;
            break;
          }
          case XI_REGEX: {  // find() over x's text with a compiled automaton (regex.py)
            V& a = st[sp - 1];
            if (a.tag == 0) {  // NULL: null_mode 1 (PatternMatch's otherwise(0)) -> FALSE
              if (ins.a) a = V{1, 0, 0, 0.0, nullptr};
              else a = V{0, 0, 0, 0.0, nullptr};
              break;
            }
            const uint8_t* blob = pool + ins.imm;
            const int32_t ns = reinterpret_cast<const int32_t*>(blob)[0];
            const int32_t nc = reinterpret_cast<const int32_t*>(blob)[1];
            uint32_t q = (uint32_t)reinterpret_cast<const int32_t*>(blob)[2];
            const uint8_t* cls = blob + 16;
            const uint8_t* status = blob + 16 + 256;
            const uint16_t* nx = reinterpret_cast<const uint16_t*>(blob + 16 + 256 + ((ns + 3) & ~3));
            if (a.tag == 4) {
              DevBytes rd{a.p};
              for (int32_t k = 0; k < a.len && !status[q]; ++k) q = nx[q * nc + cls[rd.u8(k)]];
            } else {  // Spark's cast to string: decimal integer, true / false, Double.toString,
                      // BigDecimal.toString, yyyy-MM-dd [HH:mm:ss[.f]] (decimal.h)
              char buf[kFmtMax > jfmt::kMaxChars ? kFmtMax : jfmt::kMaxChars];
              int nb = 0;
              if (a.tag == 5) {
                nb = dec_format((uint64_t)a.i, __builtin_bit_cast(int64_t, a.d), a.len, buf);
              } else if (a.tag == 6) {
                nb = date_format(a.i, buf);
              } else if (a.tag == 7) {
                nb = ts_format(a.i, buf);
              } else if (a.tag == 3) {
                nb = a.len ? jfmt::float_to_java((float)a.d, buf) : jfmt::double_to_java(a.d, buf);
              } else if (a.tag == 1) {
                const char* t = a.i ? "true" : "false";
                for (; t[nb]; ++nb) buf[nb] = t[nb];
              } else {
                uint64_t m = a.i < 0 ? 0ULL - (uint64_t)a.i : (uint64_t)a.i;
                char tmp[20];
                int nd = 0;
                do {
                  tmp[nd++] = (char)('0' + m % 10);
                  m /= 10;
                } while (m);
                if (a.i < 0) buf[nb++] = '-';
                while (nd) buf[nb++] = tmp[--nd];
              }
              for (int k = 0; k < nb && !status[q]; ++k) q = nx[q * nc + cls[(uint8_t)buf[k]]];
            }
            if (!status[q]) q = nx[q * nc + nc - 1];  // end of text
            a = V{1, 0, status[q] == 1 ? 1 : 0, 0.0, nullptr};
            break;
          }
          default: break;
        }
      }
    }
    const V& res = st[0];
    const bool valid = in_range && sp == 1 && res.tag != 0;
    const bool truth = valid && res.i != 0;
    const uint64_t bv = __ballot(truth);
    const uint64_t bn = __ballot(valid);
    if (lane == 0) {
      out_val[w] = bv;
      out_vld[w] = bn;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// PatternMatch over a utf8 column (the program [XI_COL c, XI_REGEX]): its own kernel instead of the
// interpreter walk.  The automaton arrives fused (RegexTable, built on the host by
// build_regex_table): one u8 successor per (state, byte) -- the byte classes folded in, terminal
// states (sticky accept / dead) made self-loops -- then per state bit 0 = accepted after the
// end-of-text symbol, bit 1 = terminal.  The block stages it in LDS with 16-byte copies, so a byte
// costs one dependent LDS read.  A lane walks two rows (rows r and r + 64 of a 128-row pair of
// bitmap words: two independent chains in flight), loading each string 16 bytes at a time with one
// unaligned load; a row stops at its end or in a terminal state, the wave when every row has.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 ldg128_unaligned(const uint8_t* p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4), aligned(1)));
  const v4u v = *(const __attribute__((address_space(1))) v4u*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}

struct RxRow {
  int32_t pos, end;  // byte range left to walk in the data buffer (Arrow utf8: int32 offsets)
  uint32_t q;
  DQ_DEV bool active(const uint8_t* fin) const { return pos < end && !(fin[q] & 2u); }
  // the next (at most) 16 bytes of the row
  DQ_DEV void chunk(const uint8_t* data, int32_t data_len, uint32_t (&w)[4]) const {
    if ((int64_t)pos + 16 <= (int64_t)data_len) {
      const uint4 u = ldg128_unaligned(data + pos);
      w[0] = u.x;
      w[1] = u.y;
      w[2] = u.z;
      w[3] = u.w;
    } else {  // the buffer's last bytes: no read past its end
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = 0;
      for (int j = 0; j < 16 && j < end - pos; ++j) w[j >> 2] |= (uint32_t)data[pos + j] << (8 * (j & 3));
    }
  }
};

// HR: rows per lane (independent chains of dependent LDS reads in flight)
template <int HR>
__global__ void __launch_bounds__(kBlock, HR == 4 ? 4 : 1)
regex_find_kernel(const uint8_t* __restrict__ valid, const int32_t* __restrict__ off,
                  const uint8_t* __restrict__ data, int64_t rows, const uint8_t* __restrict__ table,
                  int32_t ns, int32_t start, int32_t null_mode, uint64_t* __restrict__ out_val,
                  uint64_t* __restrict__ out_vld) {
  extern __shared__ uint4 rx_lds[];
  uint8_t* T = reinterpret_cast<uint8_t*>(rx_lds);
  const uint8_t* fin = T + (size_t)ns * 256;
  const int n16 = (ns * 257 + 15) / 16;
  for (int i = threadIdx.x; i < n16; i += kBlock) rx_lds[i] = reinterpret_cast<const uint4*>(table)[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * kBlock) >> 6;
  const int64_t n_words = (rows + 63) >> 6;
  const int32_t data_len = rows ? off[rows] : 0;
  for (int64_t w = HR * wave; w < n_words; w += HR * n_waves) {
    RxRow rr[HR];
    bool vld[HR];
#pragma unroll
    for (int h = 0; h < HR; ++h) {
      const int64_t r = (w + h) * 64 + lane;
      vld[h] = r < rows && bit1(valid, r);
      rr[h].q = (uint32_t)start;
      rr[h].pos = vld[h] ? off[r] : 0;
      rr[h].end = vld[h] ? off[r + 1] : 0;
    }
    auto any_active = [&]() {
      bool x = false;
#pragma unroll
      for (int h = 0; h < HR; ++h) x = x || rr[h].active(fin);
      return x;
    };
    while (__ballot(any_active())) {
      uint32_t c[HR][4];
#pragma unroll
      for (int h = 0; h < HR; ++h) {
        if (rr[h].active(fin)) rr[h].chunk(data, data_len, c[h]);
        else c[h][0] = c[h][1] = c[h][2] = c[h][3] = 0;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) {
#pragma unroll
        for (int h = 0; h < HR; ++h) {
          const uint32_t b = (c[h][j >> 2] >> (8 * (j & 3))) & 0xffu;
          const uint32_t nq = T[rr[h].q * 256u + b];
          rr[h].q = j < rr[h].end - rr[h].pos ? nq : rr[h].q;
        }
      }
#pragma unroll
      for (int h = 0; h < HR; ++h) rr[h].pos = rr[h].end - rr[h].pos > 16 ? rr[h].pos + 16 : rr[h].end;
    }
#pragma unroll
    for (int h = 0; h < HR; ++h) {
      // NULL: null_mode 1 (PatternMatch's otherwise(0)) -> FALSE, else NULL
      const bool res_valid = (w + h) * 64 + lane < rows && (vld[h] || null_mode);
      const bool truth = vld[h] && (fin[rr[h].q] & 1u);
      const uint64_t bv = __ballot(truth), bn = __ballot(res_valid);
      if (lane == 0 && w + h < n_words) {
        out_val[w + h] = bv;
        out_vld[w + h] = bn;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Host-side launchers
// ------------------------------------------------------------------------------------------------
hipError_t launch_expr(const XInstr* prog, int n_instr, const DevCol* cols, const uint8_t* pool,
                       int64_t rows, uint64_t* out_val, uint64_t* out_vld, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  int64_t words = (rows + 63) / 64;
  int64_t blocks = (words + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(expr_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, prog, n_instr,
                     cols, pool, rows, out_val, out_vld);
  return hipGetLastError();
}

hipError_t launch_regex(const uint8_t* valid, const int32_t* offsets, const uint8_t* data,
                        int64_t rows, const uint8_t* table, int ns, int start, int null_mode,
                        uint64_t* out_val, uint64_t* out_vld, hipStream_t stream) {
  if (rows <= 0) return hipSuccess;
  if (ns < 1 || ns > kRegexMaxStates) return hipErrorInvalidValue;
  static const int hr = [] {  // DQ_RX_ROWS=2: A/B hook, two rows per lane
    const char* e = getenv("DQ_RX_ROWS");
    return e && atoi(e) == 2 ? 2 : 4;
  }();
  const int64_t groups = ((rows + 63) / 64 + hr - 1) / hr;
  int64_t blocks = (groups + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  const size_t lds = ((size_t)ns * 257 + 15) / 16 * 16;
  if (hr == 2)
    hipLaunchKernelGGL(regex_find_kernel<2>, dim3((unsigned)blocks), dim3(kBlock), lds, stream, valid,
                       offsets, data, rows, table, ns, start, null_mode, out_val, out_vld);
  else
    hipLaunchKernelGGL(regex_find_kernel<4>, dim3((unsigned)blocks), dim3(kBlock), lds, stream, valid,
                       offsets, data, rows, table, ns, start, null_mode, out_val, out_vld);
  return hipGetLastError();
}

}  // namespace dq
