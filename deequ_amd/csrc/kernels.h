// kernels.h -- host-visible launch interface of the HIP kernels (scan.hip, freq.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "engine.h"

namespace dq {

// Sets the thread-local dq_last_error() message and returns `code`.
dq_status fail(dq_status code, const char* fmt, ...);

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      return ::dq::fail(_e == hipErrorOutOfMemory ? DQ_ERR_OUT_OF_MEMORY : DQ_ERR_DEVICE,    \
                        "HIP error %s (%d) at %s:%d", hipGetErrorString(_e), (int)_e,        \
                        __FILE__, __LINE__);                                                 \
    }                                                                                        \
  } while (0)

// Device buffer that grows on demand (contents are not preserved across growth).
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) {
      (void)hipFree(p);
      p = nullptr;
      n = 0;
    }
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(&p, count * sizeof(T));
    if (e == hipSuccess) n = count;
    return e;
  }
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
  }
};

// Column as the generic predicate interpreter sees it.
struct DevCol {
  int32_t type;
  int32_t pad;
  const uint8_t* valid;
  const void* values;
  const uint8_t* data;
};

// Postfix instruction of the generic predicate interpreter.
enum XiOp : int32_t {
  XI_COL = 1,
  XI_NULL,
  XI_BOOL,
  XI_I64,
  XI_F64,
  XI_STR,        // a = length, imm = offset into the string pool
  XI_IS_NULL,
  XI_IS_NOT_NULL,
  XI_NOT,
  XI_AND,
  XI_OR,
  XI_CMP,        // a = dq_xop comparison
  XI_IN,         // a = number of list items
  XI_CAST_F64
};

struct XInstr {
  int32_t op;
  int32_t a;
  int64_t imm;
};

constexpr int kMaxStack = 16;

hipError_t launch_expr(const XInstr* prog, int n_instr, const DevCol* cols, const uint8_t* pool,
                       int64_t rows, uint64_t* out_val, uint64_t* out_vld, hipStream_t stream);
// tasks: n_tasks descriptors (one per logical task and batch); n_logical accumulators.
hipError_t launch_scan(const TaskDesc* tasks, int n_tasks, int n_logical, int64_t total_items,
                       int grid, bool full, Acc* partial, uint8_t* hll_partial, Acc* acc,
                       uint8_t* hll_acc, hipStream_t stream);
int scan_max_blocks_per_cu(bool full);

}  // namespace dq
