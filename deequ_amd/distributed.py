"""Multi-GPU sharding: one process per GPU, rows sharded contiguously across
ranks, each rank runs the fused scan on its shard, and the per-rank aggregation buffers meet on
the device (exchange_states): counters and wrapping sums in one all-reduce SUM, extremes and HLL
registers in one all-reduce MAX, the fp64 moments in one all-gather merged in rank order by a
kernel -- the Spark merge rules, no host merge.  The previous exchange (an all-gather of the
serialized states + the rank-ordered host merge, merge_states_across_ranks) is kept as the check.
Over RCCL (`nccl` backend) the collectives run on the device; with `gloo` on host tensors.
"""
from __future__ import annotations

import ctypes
from typing import List

import numpy as np

from . import _native as N

# Bytes this rank moved through collectives since the last reset_comm_bytes(): sent to and
# received from OTHER ranks (over RCCL: the xGMI traffic; a rank's own segment never leaves it).
# All-to-all: the off-rank splits; all-gather / all-reduce: the payload to / from each peer.
COMM_BYTES = {"sent": 0, "recv": 0}


def reset_comm_bytes() -> None:
    COMM_BYTES["sent"] = COMM_BYTES["recv"] = 0


def _count_a2a(in_splits, out_splits, rank: int) -> None:
    COMM_BYTES["sent"] += int(sum(int(v) for j, v in enumerate(in_splits) if j != rank))
    COMM_BYTES["recv"] += int(sum(int(v) for j, v in enumerate(out_splits) if j != rank))


def _count_reduce(t) -> None:
    """A ring all-reduce of tensor t: 2 (world - 1) / world of its bytes each way."""
    import torch.distributed as dist
    w = dist.get_world_size()
    b = 2 * (w - 1) * t.numel() * t.element_size() // w
    COMM_BYTES["sent"] += b
    COMM_BYTES["recv"] += b


def _count_gather(nbytes: int, world: int, others_bytes: int = None) -> None:
    COMM_BYTES["sent"] += int(nbytes) * (world - 1)
    COMM_BYTES["recv"] += int(nbytes) * (world - 1) if others_bytes is None else int(others_bytes)


def serialize_state(plan, state) -> bytes:
    size = int(N.lib.dq_state_serialized_size(plan.handle))
    buf = ctypes.create_string_buffer(size)
    N.check(N.lib.dq_state_serialize(state, buf, size))
    return buf.raw


def merge_serialized(plan, images: List[bytes]):
    """Rank-ordered merge of serialized states into a host-only state; returns the result row."""
    from .runners.engine import read_row
    acc = ctypes.c_void_p()
    tmp = ctypes.c_void_p()
    N.check(N.lib.dq_state_create(plan.handle, -1, ctypes.byref(acc)))
    N.check(N.lib.dq_state_create(plan.handle, -1, ctypes.byref(tmp)))
    try:
        for img in images:
            buf = ctypes.create_string_buffer(img, len(img))
            N.check(N.lib.dq_state_deserialize(tmp, buf, len(img)))
            N.check(N.lib.dq_state_merge(acc, tmp))
        return read_row(plan, acc)
    finally:
        N.lib.dq_state_destroy(tmp)
        N.lib.dq_state_destroy(acc)


def all_gather_bytes(payload: bytes, device=None) -> List[bytes]:
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    backend = dist.get_backend()
    t = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
    if backend == "nccl":
        t = t.to(device)
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=t.device)
    dist.all_gather_into_tensor(out, t)
    _count_gather(t.numel(), world)
    host = out.cpu().numpy()
    n = len(payload)
    return [host[r * n:(r + 1) * n].tobytes() for r in range(world)]


def merge_states_across_ranks(plan, state, device=None):
    """All ranks: gather every rank's synced state and merge in rank order; returns the row."""
    N.check(N.lib.dq_state_sync(state))
    images = all_gather_bytes(serialize_state(plan, state), device)
    return merge_serialized(plan, images)


_XCHG_BUFS: dict = {}


def _exchange_buffers(plan, home, cdev, world: int):
    """The exchange's buffers for (plan, device, world), allocated once and reused every step:
    isum / imax (int64), mom (fp64), hll (uint8) on the state's side, their collective-side
    copies (the same tensors when the collectives run on the state's device) and the gathered
    moments."""
    import torch
    key = (id(plan), str(home), str(cdev), world)
    hit = _XCHG_BUFS.get(key)
    if hit is not None and hit["plan"] is plan:
        return hit
    ns, nm, nd, nh = (ctypes.c_int64() for _ in range(4))
    N.check(N.lib.dq_state_exchange_sizes(plan.handle, ctypes.byref(ns), ctypes.byref(nm),
                                          ctypes.byref(nd), ctypes.byref(nh)))
    b = {"plan": plan, "nd": nd.value, "nh": nh.value,
         "isum": torch.empty(ns.value, dtype=torch.int64, device=home),
         "imax": torch.empty(max(1, nm.value), dtype=torch.int64, device=home),
         "mom": torch.empty(max(1, nd.value), dtype=torch.float64, device=home),
         "hll": torch.empty(max(1, nh.value), dtype=torch.uint8, device=home)}
    same = str(home) == str(cdev)
    for k in ("isum", "imax", "mom", "hll"):
        b[k + "_c"] = b[k] if same else torch.empty_like(b[k], device=cdev)
    b["gathered_c"] = torch.empty(max(1, world * nd.value), dtype=torch.float64, device=cdev)
    b["gathered"] = b["gathered_c"] if same else torch.empty_like(b["gathered_c"], device=home)
    b["nm"] = nm.value
    _XCHG_BUFS[key] = b
    return b


def exchange_states(plan, state, device=None):
    """All ranks: the scan states merged on the device, as north_star states them -- counters and
    wrapping Long sums by ONE all-reduce SUM, extremes by ONE all-reduce MAX (min keys travel
    bitwise-NOT), the HLL registers as uint8 by ONE all-reduce MAX, the fp64 moments (and a decimal
    task's exact words) by ONE all-gather merged in rank order by a kernel
    (dq_state_exchange_pack / _unpack).  No host merge and no host wait but the merged state's
    read-back (dq_state_sync); the buffers are reused across steps (_exchange_buffers).  Equal,
    byte for byte, to merge_states_across_ranks (the rank-ordered dq_state_merge of the serialized
    states, kept as the check).  `device` None: a host-only state (device -1; the CPU tests),
    collectives over gloo on host tensors.  Returns the result row."""
    import torch
    import torch.distributed as dist
    from .runners.engine import read_row
    world = dist.get_world_size()
    home = torch.device(device) if device is not None else torch.device("cpu")
    cdev = _comm_device(home) if device is not None else torch.device("cpu")
    b = _exchange_buffers(plan, home, cdev, world)
    nd, nh, nm = b["nd"], b["nh"], b["nm"]
    stream = (ctypes.c_void_p(torch.cuda.current_stream(home).cuda_stream)
              if home.type == "cuda" else None)
    N.check(N.lib.dq_state_exchange_pack(state, b["isum"].data_ptr(), b["imax"].data_ptr(),
                                         b["mom"].data_ptr(), b["hll"].data_ptr(), stream))
    if b["isum_c"] is not b["isum"]:
        for k in ("isum", "imax", "mom", "hll"):
            b[k + "_c"].copy_(b[k])
    dist.all_reduce(b["isum_c"], op=dist.ReduceOp.SUM)
    if nm:
        dist.all_reduce(b["imax_c"], op=dist.ReduceOp.MAX)
    if nh:
        dist.all_reduce(b["hll_c"], op=dist.ReduceOp.MAX)
    if nd:
        dist.all_gather_into_tensor(b["gathered_c"][: world * nd], b["mom_c"][:nd])
    _count_reduce(b["isum_c"])
    if nm:
        _count_reduce(b["imax_c"])
    if nh:
        _count_reduce(b["hll_c"])
    _count_gather(nd * 8, world)
    if b["isum_c"] is not b["isum"]:
        for k in ("isum", "imax", "hll"):
            b[k].copy_(b[k + "_c"])
        b["gathered"].copy_(b["gathered_c"])
    N.check(N.lib.dq_state_exchange_unpack(state, b["isum"].data_ptr(), b["imax"].data_ptr(),
                                           b["gathered"].data_ptr(), b["hll"].data_ptr(), world,
                                           stream))
    N.check(N.lib.dq_state_sync(state))
    return read_row(plan, state)


def shard_bounds(n_rows: int, rank: int, world: int, align: int = 4096):
    """Contiguous row range of `rank`, boundaries aligned so every shard keeps the vector path."""
    per = -(-n_rows // world)
    per = -(-per // align) * align
    lo = min(n_rows, rank * per)
    return lo, min(n_rows, lo + per)


def run_scan_distributed(table_shard, specs):
    """The distributed counterpart of runners.engine.run_scan: scan the local shard, then the
    device-side state exchange (exchange_states)."""
    from .runners.engine import get_plan, scan_into
    plan = get_plan(table_shard.schema, specs)
    state = plan.state(table_shard.device_index())
    N.check(N.lib.dq_state_reset(state))
    scan_into(table_shard, plan, state)
    return exchange_states(plan, state, table_shard.device)


# ------------------------------------------------------------------------------------------------
# Frequency path: hash repartition by owner rank, then a local count
# ------------------------------------------------------------------------------------------------
def freq_partition(table, n_parts: int, stream=None):
    """Cuts a rank's partial frequency table into `n_parts` owner segments on the device.

    Returns (records, var, rec_counts, var_bytes, special): `records` / `var` are uint8 device
    tensors holding the segments back to back (24-byte dq_freq_record each; 8-aligned encoded keys),
    `rec_counts` / `var_bytes` the per-owner sizes, `special` the groups kept outside the slot table
    (dq_freq_partition_sizes)."""
    import torch
    rc = np.zeros(n_parts, np.int64)
    vb = np.zeros(n_parts, np.int64)
    sp = np.zeros(3, np.int64)
    N.check(N.lib.dq_freq_partition_sizes(table.handle, n_parts, rc.ctypes.data, vb.ctypes.data,
                                          sp.ctypes.data))
    dev = f"cuda:{table.device}"
    rec = torch.empty(int(rc.sum()) * N.FREQ_RECORD_BYTES, dtype=torch.uint8, device=dev)
    var = torch.empty(int(vb.sum()), dtype=torch.uint8, device=dev)
    if stream is None:
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    N.check(N.lib.dq_freq_partition(table.handle, n_parts, rec.data_ptr() if rec.numel() else None,
                                    var.data_ptr() if var.numel() else None, stream))
    return rec, var, rc, vb, sp


def all_gather_varbytes(payload: bytes, device=None) -> List[bytes]:
    """Every rank's byte string (sizes may differ): one all-gather of the sizes, then one of the
    payloads padded to the largest -- tensors, on the device over RCCL, never pickled objects."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    dev = device if dist.get_backend() == "nccl" else "cpu"
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    sizes = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(sizes, n)
    _count_gather(n.numel() * n.element_size(), dist.get_world_size())
    sizes = sizes.cpu().tolist()
    width = max(1, max(sizes))
    t = torch.zeros(width, dtype=torch.uint8)
    if payload:
        t[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
    t = t.to(dev)
    out = torch.empty(world * width, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, t)
    _count_gather(width, world)
    host = out.cpu().numpy()
    return [host[r * width: r * width + sizes[r]].tobytes() for r in range(world)]


def _pack_groups(counts, offs, raw) -> bytes:
    """(counts, key offsets, encoded keys) of dq_freq_topk / dq_freq_export as one byte string."""
    head = np.array([len(counts), len(raw)], np.int64)
    return (head.tobytes() + np.asarray(counts, np.int64).tobytes()
            + np.asarray(offs, np.int64).tobytes() + np.asarray(raw, np.uint8).tobytes())


def _unpack_groups(b: bytes):
    n, nraw = (int(v) for v in np.frombuffer(b, np.int64, 2))
    counts = np.frombuffer(b, np.int64, n, 16)
    offs = np.frombuffer(b, np.int64, n + 1, 16 + 8 * n)
    raw = np.frombuffer(b, np.uint8, nraw, 16 + 8 * n + 8 * (n + 1))
    return counts, offs, raw


def _comm_device(dev):
    """Where a collective's tensors live: the GPU over RCCL, the host over gloo (CPU tests and the
    two-ranks-on-one-GPU test)."""
    import torch.distributed as dist
    return dev if dist.get_backend() == "nccl" else "cpu"


def exchange_segments(rec, var, rec_counts, var_bytes):
    """All-to-all of owner segments (segment j of every rank goes to rank j): one all-to-all of the
    sizes, then one of the fixed records and one of the encoded keys.  Over RCCL each peer pair has
    its own xGMI link, so the exchange runs on all 7 links at once.  Returns the received
    (records, var, src_rec_counts, src_var_bytes) on the device, sources in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    home = rec.device
    dev = _comm_device(home)
    rec, var = rec.to(dev), var.to(dev)
    sizes = torch.from_numpy(np.stack([rec_counts, var_bytes], 1).reshape(-1).copy()).to(dev)
    got = torch.empty_like(sizes)
    dist.all_to_all_single(got, sizes)
    got = got.cpu().numpy().reshape(world, 2)
    src_rc, src_vb = got[:, 0].copy(), got[:, 1].copy()
    rb = N.FREQ_RECORD_BYTES
    recv_rec = torch.empty(int(src_rc.sum()) * rb, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv_rec, rec, output_split_sizes=(src_rc * rb).tolist(),
                           input_split_sizes=(np.asarray(rec_counts) * rb).tolist())
    me = dist.get_rank()
    _count_a2a(np.asarray(rec_counts) * rb, src_rc * rb, me)
    _count_a2a([16] * world, [16] * world, me)  # the sizes
    recv_var = torch.empty(int(src_vb.sum()), dtype=torch.uint8, device=dev)
    if int(np.sum(var_bytes)) or int(src_vb.sum()):
        dist.all_to_all_single(recv_var, var, output_split_sizes=src_vb.tolist(),
                               input_split_sizes=np.asarray(var_bytes).tolist())
        _count_a2a(np.asarray(var_bytes), src_vb, me)
    return recv_rec.to(home), recv_var.to(home), src_rc, src_vb


def freq_add_records(table, rec, var, src_rc, src_vb, num_rows: int, special,
                     null_as_group: bool = False, stream=None) -> None:
    import torch
    n_src = len(src_rc)
    rc = np.ascontiguousarray(src_rc, np.int64)
    vb = np.ascontiguousarray(src_vb, np.int64)
    sp = np.ascontiguousarray(special, np.int64)
    if stream is None:
        stream = ctypes.c_void_p(torch.cuda.current_stream(f"cuda:{table.device}").cuda_stream)
    N.check(N.lib.dq_freq_add_records_device(
        table.handle, rec.data_ptr() if rec.numel() else None,
        var.data_ptr() if var.numel() else None, n_src, rc.ctypes.data, vb.ctypes.data,
        int(num_rows), sp.ctypes.data, 1 if null_as_group else 0, stream))


def freq_repartition(local, null_as_group: bool = False):
    """The Exchange + final aggregate of the distributed groupBy: every rank partitions its partial
    table by owner, the segments meet in one all-to-all, and each rank counts the groups it owns.
    Afterwards every group lives on exactly one rank; every rank's numRows is the global row count
    (data.count(), GroupingAnalyzers.scala:74-77); the outside-table groups live on rank 0."""
    import torch
    import torch.distributed as dist
    from .analyzers.grouping import FrequencyTable
    world, rank = dist.get_world_size(), dist.get_rank()
    rec, var, rc, vb, sp = freq_partition(local, world)
    recv_rec, recv_var, src_rc, src_vb = exchange_segments(rec, var, rc, vb)
    tot = torch.tensor([local.num_rows, *sp.tolist()], dtype=torch.int64,
                       device=_comm_device(rec.device))
    dist.all_reduce(tot)
    _count_reduce(tot)
    tot = tot.cpu().numpy()
    owned = FrequencyTable(local.key_columns, local.key_types, local.device,
                           capacity_hint=int(src_rc.sum()))
    special = tot[1:] if rank == 0 else np.zeros(3, np.int64)
    freq_add_records(owned, recv_rec, recv_var, src_rc, src_vb, int(tot[0]), special, null_as_group)
    return owned


class DistributedFrequencies:
    """The frequency table of a distributed groupBy: each rank holds the groups it owns.  The one
    aggregation over the table (AnalysisRunner.scala:490-500) is a local summary plus an int64 sum
    all-reduce and a rank-ordered fp64 sum of the entropy partials (deterministic)."""

    def __init__(self, owned):
        self.owned = owned
        self.key_columns = owned.key_columns
        self.key_types = owned.key_types

    @property
    def num_rows(self) -> int:
        return self.owned.num_rows

    def summarize(self):
        import torch
        import torch.distributed as dist
        s = self.owned.summarize()
        dev = "cpu" if dist.get_backend() == "gloo" else f"cuda:{self.owned.device}"
        ints = torch.tensor([s.n_groups, s.n_unique, s.n_null_key_rows], dtype=torch.int64,
                            device=dev)
        dist.all_reduce(ints)
        _count_reduce(ints)
        ent = torch.tensor([s.entropy], dtype=torch.float64, device=dev)
        parts = torch.empty(dist.get_world_size(), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(parts, ent)
        _count_gather(ent.numel() * ent.element_size(), dist.get_world_size())
        out = N.dq_freq_summary()
        out.num_rows = s.num_rows
        out.n_groups, out.n_unique, out.n_null_key_rows = (int(v) for v in ints.cpu().tolist())
        total = 0.0
        for v in parts.cpu().tolist():  # rank order
            total += v
        out.entropy = total
        return out

    def count(self) -> int:
        return int(self.summarize().n_groups)

    def null_literal(self):
        """(NULL-group rows, "NullValue" string count) summed over the ranks: each lives on one."""
        import torch
        import torch.distributed as dist
        nullg, lit = self.owned.null_literal()
        dev = "cpu" if dist.get_backend() == "gloo" else f"cuda:{self.owned.device}"
        t = torch.tensor([nullg, lit], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        _count_reduce(t)
        a, b = (int(v) for v in t.cpu().tolist())
        return a, b

    def export(self):
        """Every group of every rank (each group lives on exactly one), rank order."""
        parts = all_gather_varbytes(_pack_groups(*self.owned.export_raw()),
                                    f"cuda:{self.owned.device}")
        return [g for p in parts for g in self.owned.decode_groups(*_unpack_groups(p))]

    def topk(self, k: int):
        """Global top-k by count: each group lives on one rank, so the k largest are among the
        union of the ranks' local top-k (Histogram.scala:78, ties in any order).  Each rank's k
        groups travel as dq_freq_topk's arrays in one device all-gather."""
        parts = all_gather_varbytes(_pack_groups(*self.owned.topk_raw(k)),
                                    f"cuda:{self.owned.device}")
        merged = [g for p in parts for g in self.owned.decode_groups(*_unpack_groups(p))]
        merged.sort(key=lambda g: -g[1])  # stable: ties keep rank order
        return merged[:k]


def is_distributed(data=None) -> bool:
    """A row-sharded run: a process group of more than one rank is initialised (and the table was
    not marked rank-local with ``data.rank_local = True``).  The runners then compute every metric
    over the union of the ranks' shards."""
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return False
    if getattr(data, "rank_local", False):
        return False
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


RAW_KEY_ELEM = {N.INT8: 1, N.INT16: 2, N.INT32: 4, N.INT64: 8, N.FLOAT32: 4, N.FLOAT64: 8,
                N.DATE32: 4, N.TIMESTAMP_US: 8}  # (a date / timestamp key: its int32 / int64)
RAW_SAMPLE_ROWS = 1 << 20
RAW_MIN_DISTINCT = 0.5  # sampled groups per non-NULL row at or above which raw keys travel


def _raw_keys_pay(data_shard, column, dtype) -> bool:
    """Whether the raw-key exchange beats partial aggregation: the groups per non-NULL row of the
    first RAW_SAMPLE_ROWS rows of every rank's first batch, summed over the ranks (one all-reduce,
    so every rank takes the same path).  A unique id samples ~1.0, a low-cardinality key ~0."""
    import torch
    import torch.distributed as dist
    from .analyzers.grouping import FrequencyTable
    from .table import ColumnBatch
    groups = rows = 0
    if data_shard.batches and data_shard.batches[0][column].length:
        c = data_shard.batches[0][column]
        m = min(c.length, RAW_SAMPLE_ROWS)
        t = FrequencyTable([column], [dtype], data_shard.device_index(), capacity_hint=m)
        t.add([ColumnBatch(dtype, m, c.validity, c.values)])
        s = t.summarize()
        groups, rows = int(s.n_groups), int(s.num_rows - s.n_null_key_rows)
    v = torch.tensor([groups, rows], dtype=torch.int64,
                     device=_comm_device(f"cuda:{data_shard.device_index()}"))
    dist.all_reduce(v)
    _count_reduce(v)
    g, r = (int(x) for x in v.cpu().tolist())
    return r > 0 and g >= RAW_MIN_DISTINCT * r


def raw_key_repartition(data_shard, column, dtype, null_as_group: bool = False):
    """The Exchange of a high-cardinality one-column fixed-width key as raw values: every rank cuts
    its rows into owner segments on the device (dq_key_partition), the segments meet in one
    all-to-all (1-8 bytes per row over xGMI), and each owner counts what it received in ONE
    group-by.  NULL rows stay home as counts; numRows and the NULL counts are summed in one
    all-reduce and the NULL group lives on rank 0, as in freq_repartition."""
    import torch
    import torch.distributed as dist
    from .analyzers.grouping import FrequencyTable
    from .table import ColumnBatch
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = f"cuda:{data_shard.device_index()}"
    elem = RAW_KEY_ELEM[dtype]
    cols = [b[column] for b in data_shard.batches]
    rows = sum(c.length for c in cols)
    arr = (N.dq_column * max(1, len(cols)))(*[c.to_c() for c in cols])
    out = torch.empty(max(1, rows * elem), dtype=torch.uint8, device=dev)
    counts = np.zeros(world, np.int64)
    nulls = ctypes.c_int64()
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    N.check(N.lib.dq_key_partition(arr, len(cols), world, 1 if null_as_group else 0,
                                   out.data_ptr(), counts.ctypes.data, ctypes.byref(nulls), stream))
    cdev = _comm_device(dev)
    sizes = torch.from_numpy(counts.copy()).to(cdev)
    got = torch.empty_like(sizes)
    dist.all_to_all_single(got, sizes)
    src = got.cpu().numpy()
    sent = out[: int(counts.sum()) * elem].to(cdev)
    recv = torch.empty(max(1, int(src.sum()) * elem), dtype=torch.uint8, device=cdev)
    dist.all_to_all_single(recv[: int(src.sum()) * elem], sent,
                           output_split_sizes=(src * elem).tolist(),
                           input_split_sizes=(counts * elem).tolist())
    _count_a2a(counts * elem, src * elem, rank)
    _count_a2a([8] * world, [8] * world, rank)  # the sizes
    recv = recv.to(dev)
    del out, sent
    n_recv = int(src.sum())
    owned = FrequencyTable([column], [dtype], data_shard.device_index(), capacity_hint=n_recv)
    step = 1 << 26
    for lo in range(0, n_recv, step):
        m = min(step, n_recv - lo)
        owned.add([ColumnBatch(dtype, m, None, recv[lo * elem: (lo + m) * elem])],
                  null_as_group=null_as_group)
    tot = torch.tensor([rows, nulls.value], dtype=torch.int64, device=cdev)
    dist.all_reduce(tot)
    _count_reduce(tot)
    tot_rows, tot_nulls = (int(v) for v in tot.cpu().tolist())
    special = np.zeros(3, np.int64)
    if rank == 0:
        special[1 if null_as_group else 2] = tot_nulls
    zero = np.zeros(1, np.int64)
    N.check(N.lib.dq_freq_add_records_device(
        owned.handle, None, None, 1, zero.ctypes.data, zero.ctypes.data, tot_rows - n_recv,
        special.ctypes.data, 1 if null_as_group else 0, stream))
    return owned


def compute_frequencies_distributed(data_shard, grouping_columns, null_as_group: bool = False):
    """FrequencyBasedAnalyzer.computeFrequencies (GroupingAnalyzers.scala:53-80) over a row-sharded
    table: a one-column fixed-width key of high cardinality travels as raw values
    (raw_key_repartition); every other key is aggregated locally first (the partial aggregate of
    each rank's shard), then freq_repartition exchanges the groups."""
    from .analyzers.grouping import FrequenciesAndNumRows, FrequencyTable
    types = [data_shard.schema[c].dtype for c in grouping_columns]
    if len(grouping_columns) == 1 and types[0] in RAW_KEY_ELEM and \
            _raw_keys_pay(data_shard, grouping_columns[0], types[0]):
        owned = raw_key_repartition(data_shard, grouping_columns[0], types[0], null_as_group)
        return FrequenciesAndNumRows(DistributedFrequencies(owned), owned.num_rows)
    local = FrequencyTable(grouping_columns, types, data_shard.device_index())
    for batch in data_shard.batches:
        local.add([batch[c] for c in grouping_columns], null_as_group=null_as_group)
    owned = freq_repartition(local, null_as_group)
    return FrequenciesAndNumRows(DistributedFrequencies(owned), owned.num_rows)
