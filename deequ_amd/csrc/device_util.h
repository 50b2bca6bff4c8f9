// device_util.h -- device helpers shared by the HIP kernels (scan.hip, expr.hip): bitmap and
// value loads, Spark's NaN-safe three-way compares, byte readers over utf8 buffers, and
// Spark's XxHash64Function.hash per column type.
#pragma once

#include <hip/hip_runtime.h>

#include "decimal.h"
#include "engine.h"

namespace dq {

#define DQ_DEV __device__ __forceinline__

// ------------------------------------------------------------------------------------------------
// Bit and value loads
// ------------------------------------------------------------------------------------------------
DQ_DEV uint32_t bit1(const uint8_t* bm, int64_t r) {
  return bm ? ((bm[r >> 3] >> (r & 7)) & 1u) : 1u;
}
// Lane index within the wave64 and a cross-lane read (ds_bpermute: no LDS memory traffic).
DQ_DEV int lane_id() { return (int)__lane_id(); }
DQ_DEV uint32_t lane_read(uint32_t v, int src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}
DQ_DEV int64_t wave_uniform(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Three-way compare in Spark's order: doubles NaN-safe (NaN == NaN, NaN largest, -0.0 == 0.0).
DQ_DEV int cmp3_f64(double a, double b) {
  bool an = a != a, bn = b != b;
  if ((an && bn) || a == b) return 0;
  if (an) return 1;
  if (bn) return -1;
  return a > b ? 1 : -1;
}
DQ_DEV int cmp3_i64(int64_t a, int64_t b) { return a == b ? 0 : (a > b ? 1 : -1); }

// truth table of a comparison op over the three-way result c in {-1,0,1}: bit (c+1)
DQ_HD uint32_t op_mask(int op) {
  switch (op) {
    case DQ_X_EQ: return 0b010;
    case DQ_X_NE: return 0b101;
    case DQ_X_LT: return 0b001;
    case DQ_X_LE: return 0b011;
    case DQ_X_GT: return 0b100;
    case DQ_X_GE: return 0b110;
    default: return 0b111;
  }
}

// Byte reader over a device utf8 buffer using only aligned dword loads that contain at least one
// byte of the string (never faults past the end of the allocation).
struct DevBytes {
  const uint8_t* p;
  DQ_DEV uint32_t u32(int64_t o) const {
    uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    uint32_t sh = (uint32_t)(a & 3) * 8;
    uint32_t w0 = w[0];
    if (sh == 0) return w0;
    uint32_t w1 = w[1];
    return (w0 >> sh) | (w1 << (32 - sh));
  }
  DQ_DEV uint64_t u64(int64_t o) const { return (uint64_t)u32(o) | ((uint64_t)u32(o + 4) << 32); }
  DQ_DEV uint32_t u8(int64_t o) const {
    uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    return (w[0] >> ((a & 3) * 8)) & 0xffu;
  }
  // first min(len, 8) bytes, little-endian, zero padded
  DQ_DEV uint64_t prefix8(int64_t len) const {
    if (len <= 0) return 0;
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    uint32_t sh = (uint32_t)(a & 3) * 8;
    int64_t take = len < 8 ? len : 8;
    int64_t last = (int64_t)((a & 3) + take - 1) >> 2;  // index of last dword needed
    uint64_t w0 = w[0];
    uint64_t w1 = last >= 1 ? (uint64_t)w[1] : 0;
    uint64_t w2 = last >= 2 ? (uint64_t)w[2] : 0;
    uint64_t lo = w0 | (w1 << 32);
    uint64_t v = sh ? ((lo >> sh) | (w2 << (64 - sh))) : lo;
    if (take < 8) v &= (1ULL << (take * 8)) - 1;
    return v;
  }
};

// Unaligned little-endian reads through global_load_dword{,x2} at any byte address (gfx950 HSA
// runs in unaligned-access mode).  Only for reads that stay inside the buffer: xxh_bytes reads
// u64 at o + 8 <= len, u32 at o + 4 <= len and single bytes, so a string's own bytes suffice.
struct UBytes {
  const uint8_t* p;
  DQ_DEV uint64_t u64(int64_t o) const {
    uint64_t v;
    __builtin_memcpy(&v, p + o, 8);
    return v;
  }
  DQ_DEV uint32_t u32(int64_t o) const {
    uint32_t v;
    __builtin_memcpy(&v, p + o, 4);
    return v;
  }
  DQ_DEV uint32_t u8(int64_t o) const { return p[o]; }
};

// First min(len, 8) bytes at p, little-endian, zero padded; `room` = bytes readable from p.
DQ_DEV uint64_t load_prefix8(const uint8_t* p, int32_t len, int64_t room) {
  if (len <= 0) return 0;
  uint64_t v;
  if (room >= 8) {
    __builtin_memcpy(&v, p, 8);
  } else {
    v = 0;
    for (int k = 0; k < (int)room; ++k) v |= (uint64_t)p[k] << (8 * k);
  }
  return len >= 8 ? v : (v & ((1ULL << (8 * len)) - 1));
}

// Loads one value of a runtime-typed numeric column as double / as int64.
DQ_DEV double load_f64(int type, const void* v, int64_t r) {
  switch (type) {
    case DQ_INT8: return (double)reinterpret_cast<const int8_t*>(v)[r];
    case DQ_INT16: return (double)reinterpret_cast<const int16_t*>(v)[r];
    case DQ_INT32: return (double)reinterpret_cast<const int32_t*>(v)[r];
    case DQ_INT64: return (double)reinterpret_cast<const int64_t*>(v)[r];
    case DQ_FLOAT32: return (double)reinterpret_cast<const float*>(v)[r];
    case DQ_FLOAT64: return reinterpret_cast<const double*>(v)[r];
    case DQ_BOOL: return (double)bit1(reinterpret_cast<const uint8_t*>(v), r);
    default: return 0.0;
  }
}
DQ_DEV int64_t load_i64(int type, const void* v, int64_t r) {
  switch (type) {
    case DQ_INT8: return reinterpret_cast<const int8_t*>(v)[r];
    case DQ_INT16: return reinterpret_cast<const int16_t*>(v)[r];
    case DQ_INT32: return reinterpret_cast<const int32_t*>(v)[r];
    case DQ_INT64: return reinterpret_cast<const int64_t*>(v)[r];
    case DQ_BOOL: return bit1(reinterpret_cast<const uint8_t*>(v), r);
    default: return 0;
  }
}
DQ_HD bool is_float_type(int type) { return type == DQ_FLOAT32 || type == DQ_FLOAT64; }

// Spark XxHash64Function.hash(value, type, 42) for one non-null row.
// A decimal row, out of line: inlined into the unrolled HLL loops (8 copies in the fused
// Correlation + HLL body) its BigInteger byte hashing spilled 272 bytes per lane and took
// configs[3] from 4.0 to 7.2 ms per step (round 6); a call on this rare path costs them nothing.
static __device__ __attribute__((noinline)) uint64_t hash_row_decimal(int type, const void* values,
                                                                      int64_t r) {
  const uint64_t* v = reinterpret_cast<const uint64_t*>(values) + 2 * r;
  return dec_hash(v[0], (int64_t)v[1], DQ_DECIMAL_PRECISION(type), 42);
}

// hash_row for the only columns the fused Correlation + HLL body takes (api.cpp: 8-byte int64 /
// float64 columns): the general switch's other cases cost that unrolled body registers
DQ_DEV uint64_t hash_wide(int type, const void* values, int64_t r) {
  const uint64_t v = reinterpret_cast<const uint64_t*>(values)[r];
  if (type == DQ_FLOAT64) {
    const double d = __builtin_bit_cast(double, v);
    return xxh_long(d != d ? 0x7ff8000000000000ULL : v, 42);  // doubleToLongBits
  }
  return xxh_long(v, 42);
}

DQ_DEV uint64_t hash_row(int type, const void* values, const uint8_t* data, int64_t r) {
  const uint64_t seed = 42;
  int tid = DQ_TYPE_ID(type);
  // dates hash as Spark's IntegerType, timestamps as LongType (their physical values)
  tid = tid == DQ_DATE32 ? DQ_INT32 : tid == DQ_TIMESTAMP_US ? DQ_INT64 : tid;
  switch (tid) {
    case DQ_DECIMAL128: return hash_row_decimal(type, values, r);
    case DQ_INT8: return xxh_int((uint32_t)(int32_t)reinterpret_cast<const int8_t*>(values)[r], seed);
    case DQ_INT16:
      return xxh_int((uint32_t)(int32_t)reinterpret_cast<const int16_t*>(values)[r], seed);
    case DQ_INT32: return xxh_int((uint32_t)reinterpret_cast<const int32_t*>(values)[r], seed);
    case DQ_INT64: return xxh_long((uint64_t)reinterpret_cast<const int64_t*>(values)[r], seed);
    case DQ_BOOL: return xxh_int(bit1(reinterpret_cast<const uint8_t*>(values), r), seed);
    case DQ_FLOAT32: {
      float f = reinterpret_cast<const float*>(values)[r];
      uint32_t b = (f != f) ? 0x7fc00000u : __builtin_bit_cast(uint32_t, f);  // floatToIntBits
      return xxh_int(b, seed);
    }
    case DQ_FLOAT64: {
      double d = reinterpret_cast<const double*>(values)[r];
      uint64_t b = (d != d) ? 0x7ff8000000000000ULL : __builtin_bit_cast(uint64_t, d);
      return xxh_long(b, seed);
    }
    case DQ_UTF8: {
      const int32_t* off = reinterpret_cast<const int32_t*>(values);
      int32_t s = off[r], e = off[r + 1];
      UBytes rd{data + s};
      return xxh_bytes(rd, (int64_t)(e - s), seed);
    }
    default: return 0;
  }
}

}  // namespace dq
