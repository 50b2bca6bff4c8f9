"""Multi-GPU sharding: one process per GPU, rows sharded contiguously across
ranks, each rank runs the fused scan on its shard, and the per-rank aggregation buffers meet in
ONE collective -- an all-gather of the serialized states (a few hundred bytes; latency-bound, so
one gather beats separate sum / min / max / register-max all-reduces) -- followed by a
deterministic rank-ordered merge with the engine's own Spark-merge rules (dq_state_merge).  Over
RCCL (`nccl` backend) the gather runs on the device; with `gloo` (CPU tests) on host tensors.
"""
from __future__ import annotations

import ctypes
from typing import List

import numpy as np

from . import _native as N


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
    host = out.cpu().numpy()
    n = len(payload)
    return [host[r * n:(r + 1) * n].tobytes() for r in range(world)]


def merge_states_across_ranks(plan, state, device=None):
    """All ranks: gather every rank's synced state and merge in rank order; returns the row."""
    N.check(N.lib.dq_state_sync(state))
    images = all_gather_bytes(serialize_state(plan, state), device)
    return merge_serialized(plan, images)


def shard_bounds(n_rows: int, rank: int, world: int, align: int = 4096):
    """Contiguous row range of `rank`, boundaries aligned so every shard keeps the vector path."""
    per = -(-n_rows // world)
    per = -(-per // align) * align
    lo = min(n_rows, rank * per)
    return lo, min(n_rows, lo + per)


def run_scan_distributed(table_shard, specs):
    """The distributed counterpart of runners.engine.run_scan: scan the local shard, then the
    all-gather + rank-ordered merge."""
    from .runners.engine import get_plan, scan_into
    plan = get_plan(table_shard.schema, specs)
    state = plan.state(table_shard.device_index())
    N.check(N.lib.dq_state_reset(state))
    scan_into(table_shard, plan, state)
    return merge_states_across_ranks(plan, state, table_shard.device)
