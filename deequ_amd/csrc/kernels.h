// kernels.h -- host-visible launch interface of the HIP kernels (scan.hip, freq.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>
#include <vector>

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

// Device memory cache (api.cpp).  A group-by allocates gigabytes per table; hipMalloc/hipFree of
// such blocks, once per table and per growth step, cost more than the table's kernels when a run
// builds twenty tables (configs[4]).  Freed blocks are kept per device and handed out again to
// requests they cover within 2x; the device is synchronised on free, as hipFree does, so a block
// is never reused while a kernel still reads it.  On hipMalloc failure the cache is released and
// the allocation retried.
hipError_t dev_alloc(void** p, size_t bytes, size_t* got, int* device);
void dev_free(void* p, size_t bytes, int device);

// Device -> host copy of a small result (counts, bounds, a histogram, the top-k records) after
// the work queued on `st`: stream-ordered into page-locked staging (api.cpp keeps a few blocks),
// then memcpy'd to `dst`.  A plain hipMemcpy into pageable memory goes through the runtime's own
// staging: measured ~20 us for 16 bytes and ~100 us for 64 KB, against ~10 us from pinned.
hipError_t d2h(void* dst, const void* src, size_t bytes, hipStream_t st);
// Several such copies behind ONE wait: each part stream-ordered into its slice of one staging
// block, then the block waited for once (a finalize's counters, totals and reductions: one host
// round trip instead of one per read-back).
struct D2HPart {
  void* dst;
  const void* src;
  size_t bytes;
};
hipError_t d2h_n(const D2HPart* parts, int n, hipStream_t st);

// Device buffer that grows on demand (contents are not preserved across growth).
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  size_t bytes = 0;
  int dev = -1;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) dev_free(p, bytes, dev);
  }
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) {
      dev_free(p, bytes, dev);
      p = nullptr;
      n = bytes = 0;
    }
    if (count == 0) count = 1;
    void* q = nullptr;
    size_t got = 0;
    hipError_t e = dev_alloc(&q, count * sizeof(T), &got, &dev);
    if (e == hipSuccess) {
      p = static_cast<T*>(q);
      bytes = got;
      n = got / sizeof(T);
    }
    return e;
  }
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(bytes, o.bytes);
    std::swap(dev, o.dev);
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
  XI_CAST_F64,
  XI_REGEX,      // a = null_mode, imm = offset of the automaton in the pool
  XI_DEC128,     // imm = low word of a decimal literal (unscaled at its column's scale) ...
  XI_DEC128_HI   // ... imm = its high word (always right after XI_DEC128)
};

struct XInstr {
  int32_t op;
  int32_t a;
  int64_t imm;
};

constexpr int kMaxStack = 16;

// Arrow bitmap at a bit offset -> bitmap at bit 0 (cast.hip; sliced Arrow arrays at the ABI).
hipError_t launch_bitmap_rebase(const uint8_t* src, int64_t bit, int64_t rows, uint8_t* dst,
                                hipStream_t stream);
hipError_t launch_expr(const XInstr* prog, int n_instr, const DevCol* cols, const uint8_t* pool,
                       int64_t rows, uint64_t* out_val, uint64_t* out_vld, hipStream_t stream);
// PatternMatch over a utf8 column with a fused automaton table (expr.hip): ns * 256 u8 successors
// then ns flag bytes (bit 0 accepted after end of text, bit 1 terminal), 16-byte aligned.
constexpr int kRegexMaxStates = 255;
hipError_t launch_regex(const uint8_t* valid, const int32_t* offsets, const uint8_t* data,
                        int64_t rows, const uint8_t* table, int ns, int start, int null_mode,
                        uint64_t* out_val, uint64_t* out_vld, hipStream_t stream);
// Body classes of the scan: one kernel instantiation each (scan.hip).
enum BodyClass : int32_t {
  BC_NUM_I8 = 0,
  BC_NUM_I16,
  BC_NUM_I32,
  BC_NUM_I64,
  BC_NUM_F32,
  BC_NUM_F64,
  BC_BITS,     // TK_VALIDITY, TK_BOOLMAP
  BC_STR_IN,
  BC_DTYPE,     // TK_DTYPE
  BC_CORR,
  BC_HLL,
  BC_CORR_HLL,  // TK_COMOMENTS task that also fills an HLL task's registers from one of its columns
  BC_DECIMAL,   // TK_DECIMAL (always its own launch: the mixed kernel has no decimal body)
  kBodyClasses
};
// A launch of the mixed kernel: every non-HLL body class in one grid, items taken in an
// interleaved order so latency-bound bodies (string gathers) overlap bandwidth-bound ones.
constexpr int kBodyMixed = kBodyClasses;
constexpr int kQueues = kBodyClasses + 1;  // one work queue per launch kind
// A queue is kQueueHeads head words, one per XCD, each on its own 128-byte line: the items of a
// launch are cut into kQueueHeads contiguous slices and a wave dequeues from the slice of its
// workgroup's XCD first (one device-scope head saturates at ~88 dequeues/us with 256 CUs pulling;
// MI355X_MICROARCH.md "dequeue"), then drains the other slices in turn.
constexpr int kQueueHeads = 8;
constexpr int kQueueStride = 32;  // u32 words between heads
constexpr int kQueueWords = kQueues * kQueueHeads * kQueueStride;

// One scan launch: the items [item_lo, item_hi) of every task of body class `body`.
struct ScanLaunch {
  int32_t body;            // BodyClass, or kBodyMixed
  int32_t grid;
  uint32_t item_lo, item_hi;  // with `order`: item_lo = 0, item_hi = entries of `order`
  const uint32_t* order;   // queue position -> global item index (kBodyMixed always; a one-class
                           // launch when its descriptors have small tail items), else nullptr
  int32_t lds_hll = 0;     // kBodyMixed: HLL tasks whose registers the launch keeps in LDS
  uint32_t classes = 0;    // kBodyMixed: the body classes of its items (bit per BodyClass)
};
// Mixed-kernel instantiations: every class it has a body for, and BASELINE configs[1]'s three
constexpr uint32_t kMixedAll = ((1u << kBodyClasses) - 1u) & ~(1u << BC_DECIMAL);
constexpr uint32_t kMixedS10 = (1u << BC_BITS) | (1u << BC_NUM_I64) | (1u << BC_STR_IN);

// Most HLL tasks whose LDS registers (2 KiB each) ride in the mixed launch.  0 = HLL always keeps
// its own launch: measured on MI355X at configs[3] (1.25e9 rows), HLL inside the mixed grid took
// 6.18 ms per step vs 5.74 ms as its own launch (and 11.19 vs 10.45 ms with the earlier 128 KiB
// work-sized items) -- the XXH64 body is bound by quarter-rate 64-bit multiplies and needs the
// occupancy the mixed kernel's 3 waves/SIMD denies.
constexpr int kMixedHllMax = 0;

// Fused scan over n_desc (task, batch) descriptors numbered class-major then task-major (each
// logical task owns one contiguous range of work items), one launch per entry of `launches`, then
// the two finalize launches that fold the item partials into acc[n_tasks] / hll_acc.
// queues[kQueueWords] must be 0 on entry (finalize re-arms them), `partial` holds one record per
// item, `partial2` n_tasks * kFinParts, `hll_stage` n_hll * kHllM zeroed u32 registers (finalize
// clears them again).
hipError_t launch_scan(const TaskDesc* tasks, int n_desc, int n_tasks, const ScanLaunch* launches,
                       int n_launches, int n_hll, uint32_t* queues, Acc* partial, Acc* partial2,
                       uint32_t* hll_stage, Acc* acc, uint8_t* hll_acc, uint32_t* arrivals,
                       hipStream_t stream, int reset = 0);
size_t scan_lds_bytes(int body, int n_hll);
int scan_max_blocks_per_cu(int body, int n_hll);
// Per column of a plan: 0 not read, 1 validity bitmap only, 2 every buffer (api.cpp).
void plan_column_needs(const dq_plan* plan, std::vector<int>& need);

}  // namespace dq
