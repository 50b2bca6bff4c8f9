// loader.cpp -- columnar handoff: host-resident Arrow batches (what a Spark partition exports
// through the Arrow C Data Interface) staged into HBM for the device entry points.
//
// Two staging slots alternate, each a pinned host buffer plus a device buffer.  dq_loader_stage
// copies the caller's (pageable) buffers into the slot's pinned buffer on the host -- several
// threads for large batches -- and queues one DMA per column buffer from there on the loader's own
// copy stream; the scan of the slot waits for its DMA on the caller's stream.  So batch k's DMA
// overlaps batch k-1's HBM-bound scan, and a DMA from pinned memory runs at the link rate instead
// of the driver's pageable bounce path.  A slot is refilled only after its previous DMA has drained
// (host wait, before the pinned buffer is overwritten) and the work that read its device buffer
// (recorded by dq_loader_release) has finished.
//
// Buffer lifetime: the caller's host buffers are read only inside dq_loader_stage (and
// dq_scan_host / dq_freq_add_host): they may be freed or reused as soon as the call returns.  The
// reference's equivalent is Spark feeding UnsafeRows of a partition into the aggregation iterator
// (AnalysisRunner.scala:303); ownership stays with the caller exactly as there.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "engine.h"
#include "kernels.h"

using namespace dq;

namespace {

struct Slot {
  DevBuf<uint8_t> buf;
  uint8_t* pinned = nullptr;  // hipHostMalloc'd staging copy of the batch
  size_t pinned_n = 0;
  hipEvent_t copied = nullptr;
  hipEvent_t consumed = nullptr;
  bool used = false;
  bool dma = false;  // a DMA from `pinned` was queued
};

// memcpy of large buffers split over a few host threads (one thread streams ~10 GB/s, below the
// host link's rate)
void host_copy(uint8_t* dst, const void* src, size_t bytes) {
  constexpr size_t kPerThread = (size_t)16 << 20;
  const size_t nt = std::min<size_t>(8, bytes / kPerThread);
  if (nt <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (bytes + nt - 1) / nt;
  for (size_t t = 0; t < nt; ++t) {
    const size_t lo = t * per, hi = std::min(bytes, lo + per);
    if (lo < hi)
      th.emplace_back([=] { memcpy(dst + lo, static_cast<const uint8_t*>(src) + lo, hi - lo); });
  }
  for (auto& x : th) x.join();
}

size_t fixed_width(int t) {
  if (DQ_TYPE_ID(t) == DQ_DECIMAL128) return 16;
  switch (t) {
    case DQ_INT8: return 1;
    case DQ_INT16: return 2;
    case DQ_INT32: case DQ_FLOAT32: case DQ_DATE32: return 4;
    case DQ_INT64: case DQ_FLOAT64: case DQ_TIMESTAMP_US: return 8;
    default: return 0;
  }
}

size_t round_up(size_t v) { return (v + 255) & ~(size_t)255; }

}  // namespace

struct dq_loader {
  int device = 0;
  hipStream_t copy = nullptr;
  Slot slot[2];
  int next = 0;
  int staged = -1;
  ~dq_loader() {
    for (Slot& s : slot) {
      if (s.pinned) (void)hipHostFree(s.pinned);
      if (s.copied) (void)hipEventDestroy(s.copied);
      if (s.consumed) (void)hipEventDestroy(s.consumed);
    }
    if (copy) (void)hipStreamDestroy(copy);
  }
};

extern "C" dq_status dq_loader_create(int device, dq_loader** out) {
  if (!out) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  if (device < 0) return fail(DQ_ERR_INVALID_ARGUMENT, "loader needs a device");
  auto l = new dq_loader();
  l->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&l->copy, hipStreamNonBlocking);
  for (int k = 0; k < 2 && e == hipSuccess; ++k) {
    e = hipEventCreateWithFlags(&l->slot[k].copied, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&l->slot[k].consumed, hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    delete l;
    return fail(DQ_ERR_DEVICE, "HIP error %s creating the loader", hipGetErrorString(e));
  }
  *out = l;
  return DQ_OK;
}

extern "C" void dq_loader_destroy(dq_loader* l) {
  if (!l) return;
  (void)hipSetDevice(l->device);
  for (Slot& s : l->slot)
    if (s.used) (void)hipEventSynchronize(s.consumed);
  (void)hipStreamSynchronize(l->copy);
  delete l;
}

// need (optional, per column): 0 stage nothing, 1 the validity bitmap only, 2 every buffer; an
// unstaged values / data buffer is given a non-null device address that nothing reads.
static dq_status stage(dq_loader* l, const dq_column* host_cols, int n_cols, dq_column* dev_cols,
                       void* hip_stream, const int* need) {
  if (!l || (n_cols > 0 && (!host_cols || !dev_cols)) || n_cols < 0)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (l->staged >= 0) return fail(DQ_ERR_STATE, "previous staged batch was not released");
  hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
  HIP_TRY(hipSetDevice(l->device));
  // layout of the slot: per column validity | values | data, each 256-byte aligned
  std::vector<size_t> nv(n_cols), nval(n_cols), ndat(n_cols), dlo(n_cols, 0);
  size_t total = 0;
  for (int c = 0; c < n_cols; ++c) {
    const dq_column& h = host_cols[c];
    if (h.length < 0) return fail(DQ_ERR_INVALID_ARGUMENT, "column %d: negative length", c);
    const size_t n = (size_t)h.length;
    const int nd = need ? need[c] : 2;
    nv[c] = h.validity && nd >= 1 ? (n + 7) / 8 : 0;
    if (nd < 2) {  // unread values / data are never touched (not even the offsets)
      nval[c] = ndat[c] = 0;
    } else if (h.type == DQ_UTF8) {
      nval[c] = h.values ? 4 * (n + 1) : 0;
      const int32_t* off = static_cast<const int32_t*>(h.values);
      const int32_t end = off ? off[n] : 0;
      if (end < 0 || (off && off[0] < 0) || (off && off[0] > end))
        return fail(DQ_ERR_INVALID_ARGUMENT, "column %d: bad string offsets", c);
      // a sliced array (off[0] > 0): only the bytes from off[0] (rounded down to 256, keeping the
      // staged pointer's alignment) cross the link; the device data pointer is moved back by as
      // much, so the offsets stay absolute and every string still starts inside the staged bytes
      dlo[c] = off ? (size_t)off[0] & ~(size_t)255 : 0;
      ndat[c] = h.data ? (size_t)end - dlo[c] : 0;
    } else if (h.type == DQ_BOOL) {
      nval[c] = h.values ? (n + 7) / 8 : 0;
      ndat[c] = 0;
    } else {
      const size_t w = fixed_width(h.type);
      if (!w) return fail(DQ_ERR_WRONG_TYPE, "column %d: unknown type %d", c, h.type);
      nval[c] = h.values ? w * n : 0;
      ndat[c] = 0;
    }
    total += round_up(nv[c]) + round_up(nval[c]) + round_up(ndat[c]);
  }
  total = std::max<size_t>(total, 256);  // the stand-in address of unstaged buffers
  const int k = l->next;
  l->next ^= 1;
  Slot& s = l->slot[k];
  if (s.dma) HIP_TRY(hipEventSynchronize(s.copied));  // the pinned buffer is about to be rewritten
  if (s.used) {
    if (s.buf.n < total) HIP_TRY(hipEventSynchronize(s.consumed));  // about to free it
    else HIP_TRY(hipStreamWaitEvent(l->copy, s.consumed, 0));
  }
  if (s.buf.n < total) HIP_TRY(s.buf.ensure(total + total / 8));
  if (s.pinned_n < total) {
    if (s.pinned) HIP_TRY(hipHostFree(s.pinned));
    s.pinned = nullptr;
    s.pinned_n = 0;
    HIP_TRY(hipHostMalloc((void**)&s.pinned, total + total / 8, hipHostMallocDefault));
    s.pinned_n = total + total / 8;
  }
  uint8_t* p = s.buf.p;
  uint8_t* hp = s.pinned;
  for (int c = 0; c < n_cols; ++c) {
    const dq_column& h = host_cols[c];
    dq_column d = h;
    auto put = [&](const void* src, size_t bytes, const void** dst_field) -> hipError_t {
      if (!bytes) return hipSuccess;
      host_copy(hp, src, bytes);
      hipError_t e = hipMemcpyAsync(p, hp, bytes, hipMemcpyHostToDevice, l->copy);
      *dst_field = p;
      p += round_up(bytes);
      hp += round_up(bytes);
      return e;
    };
    const void* vp = nullptr;
    const void* dp = nullptr;
    const void* valp = nullptr;
    HIP_TRY(put(h.validity, nv[c], &vp));
    HIP_TRY(put(h.values, nval[c], &valp));
    HIP_TRY(put(h.data ? static_cast<const uint8_t*>(h.data) + dlo[c] : nullptr, ndat[c], &dp));
    if (dp) dp = static_cast<const uint8_t*>(dp) - dlo[c];
    const int nd = need ? need[c] : 2;
    d.validity = static_cast<const uint8_t*>(h.validity && nd >= 1 ? vp : nullptr);
    if (nd == 2) {
      d.values = h.values ? valp : nullptr;
      d.data = static_cast<const uint8_t*>(h.data ? dp : nullptr);
    } else {  // a stand-in address: the plan reads neither
      d.values = s.buf.p;
      d.data = h.type == DQ_UTF8 ? s.buf.p : nullptr;
    }
    if (nd == 2 && h.type == DQ_UTF8 && h.data && ndat[c] == 0) d.data = s.buf.p;  // empty strings
    if (nd == 2 && h.values && nval[c] == 0) d.values = s.buf.p;                   // zero-row column
    dev_cols[c] = d;
  }
  HIP_TRY(hipEventRecord(s.copied, l->copy));
  s.dma = true;
  HIP_TRY(hipStreamWaitEvent(stream, s.copied, 0));
  l->staged = k;
  return DQ_OK;
}

extern "C" dq_status dq_loader_stage(dq_loader* l, const dq_column* host_cols, int n_cols,
                                     dq_column* dev_cols, void* hip_stream) {
  return stage(l, host_cols, n_cols, dev_cols, hip_stream, nullptr);
}

extern "C" dq_status dq_loader_release(dq_loader* l, void* hip_stream) {
  if (!l) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (l->staged < 0) return fail(DQ_ERR_STATE, "no staged batch");
  HIP_TRY(hipSetDevice(l->device));
  Slot& s = l->slot[l->staged];
  HIP_TRY(hipEventRecord(s.consumed, reinterpret_cast<hipStream_t>(hip_stream)));
  s.used = true;
  l->staged = -1;
  return DQ_OK;
}

extern "C" dq_status dq_scan_host(dq_loader* l, const dq_plan* plan, const dq_column* host_cols,
                                  int n_cols, dq_state* state, void* hip_stream) {
  std::vector<dq_column> dev(std::max(0, n_cols));
  if (!plan) return fail(DQ_ERR_INVALID_ARGUMENT, "null plan");
  std::vector<int> need;  // only what the plan reads crosses the host link
  plan_column_needs(plan, need);
  if ((int)need.size() != n_cols) return fail(DQ_ERR_INVALID_ARGUMENT, "plan has %d columns", (int)need.size());
  dq_status st = stage(l, host_cols, n_cols, dev.data(), hip_stream, need.data());
  if (st != DQ_OK) return st;
  st = dq_scan_device(plan, dev.data(), n_cols, state, hip_stream);
  dq_status rs = dq_loader_release(l, hip_stream);
  return st != DQ_OK ? st : rs;
}

extern "C" dq_status dq_freq_add_host(dq_loader* l, dq_freq* freq, const dq_column* host_keys,
                                      int n_keys, int null_as_group, void* hip_stream) {
  std::vector<dq_column> dev(std::max(0, n_keys));
  dq_status st = dq_loader_stage(l, host_keys, n_keys, dev.data(), hip_stream);
  if (st != DQ_OK) return st;
  st = dq_freq_add_device(freq, dev.data(), n_keys, null_as_group, hip_stream);
  dq_status rs = dq_loader_release(l, hip_stream);
  return st != DQ_OK ? st : rs;
}
