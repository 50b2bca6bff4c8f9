"""The device-side state exchange (distributed.exchange_states: all-reduce SUM of the counters and
wrapping sums, all-reduce MAX of the extremes and HLL registers, all-gather + rank-ordered merge of
the fp64 moments) against the rank-ordered dq_state_merge of the serialized states, on gloo ranks
of world size 2 and 3 on the CPU (host-only states: the same merge code the exchange kernels run,
DQ_HD functions in api.cpp).  Bar: the merged states are equal byte for byte.

Every rank crafts every rank's aggregation buffers from a seed (the scan's layout per task kind,
api.cpp / engine.h Acc: a task's unused fields zero), so the reference merge needs no collective.
Cases the merge rules single out are planted: empty ranks (n = 0: skipped, or copied into an empty
accumulator), -0.0 double sums, Long sums that wrap, extremes at INT64_MIN / INT64_MAX, and a
decimal(38, 4) column's task (192-bit sums with carries across words, 128-bit extremes: the words
travel in the gathered block and merge in rank order, not through the word-wise collectives).
"""
import os
import socket
import struct

import numpy as np
import pytest

MAGIC = 0x3130514445455144  # "DQEEDQ01"
I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _plan():
    from deequ_amd import _native as N
    from deequ_amd.analyzers import (ApproxCountDistinct, Completeness, Compliance, Correlation,
                                     DataType, Maximum, Mean, Minimum, Size, StandardDeviation, Sum)
    from deequ_amd.runners.engine import get_plan
    from deequ_amd.table import StructField, StructType
    sch = StructType([StructField("x", N.INT64), StructField("d", N.FLOAT64),
                      StructField("s", N.UTF8), StructField("m", N.decimal_type(38, 4))])
    suite = [Size(), Completeness("s"), Compliance("c", "x >= 0"), Sum("x"), Mean("x"),
             StandardDeviation("x"), Minimum("x"), Maximum("x"), Minimum("d"), Maximum("d"),
             Sum("d"), Correlation("x", "d"), ApproxCountDistinct("x"), ApproxCountDistinct("s"),
             DataType("s"), Compliance("c2", "s = 'a' OR x > 3"), Sum("m"), Minimum("m"),
             Maximum("m"), StandardDeviation("m"), Completeness("m")]
    return get_plan(sch, [s for a in suite for s in a.aggregation_functions()])


def _s64(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def _kinds(plan):
    kinds = []
    for line in plan.explain().splitlines():
        if line.startswith("task["):
            kinds.append(line.split()[1])
    return kinds


def _image(plan, seed, rank):
    """Rank `rank`'s serialized state: per task kind, values as a scan would leave them."""
    kinds = _kinds(plan)
    n_hll = kinds.count("hll")
    rng = np.random.default_rng(seed * 1000 + rank)
    empty = rng.random() < 0.3 and rank != 1  # an empty rank (rank 1 never, so n > 0 somewhere)
    body = b""
    for k in kinds:
        i, d = [0] * 10, [0.0] * 6
        n = 0 if empty else int(rng.integers(1, 1 << 40))
        if k == "validity":
            i[0] = n
        elif k == "numeric":
            i[0] = n
            i[2], i[3] = I64_MAX, I64_MIN
            if n:
                i[1] = int(rng.integers(I64_MIN, I64_MAX, dtype=np.int64))
                lo, hi = sorted(int(v) for v in rng.integers(I64_MIN, I64_MAX, 2, dtype=np.int64))
                i[2], i[3] = (I64_MIN if rng.random() < 0.2 else lo), (I64_MAX if rng.random() < 0.2 else hi)
                i[7] = int(rng.integers(0, n + 1))
                i[4] = int(rng.integers(0, i[7] + 1))
                d[0] = -0.0 if rng.random() < 0.3 else float(rng.normal(0, 1e12))
                d[1] = float(rng.normal(0, 1e6))
                d[2] = float(abs(rng.normal(0, 1e15)))
        elif k == "comoments":
            i[0] = n
            if n:
                d[:5] = [float(v) for v in rng.normal(0, 1e6, 5)]
                d[3], d[4] = abs(d[3]), abs(d[4])
        elif k == "decimal":
            i[0] = n
            i[4], i[5], i[6], i[7] = -1, I64_MAX, 0, I64_MIN  # the empty extremes
            if n:
                w = int(rng.integers(0, 1 << 62)) << 100 | int(rng.integers(0, 1 << 62))
                w = -w if rng.random() < 0.5 else w  # a 192-bit sum: carries cross the words
                w &= (1 << 192) - 1
                i[1:4] = [_s64(w >> (64 * q) & 0xFFFFFFFFFFFFFFFF) for q in range(3)]
                lo, hi = sorted(int(rng.integers(-(1 << 62), 1 << 62)) << 60 | int(rng.integers(0, 1 << 60))
                                for _ in range(2))
                for at, v in ((4, lo), (6, hi)):
                    v &= (1 << 128) - 1
                    i[at], i[at + 1] = _s64(v & 0xFFFFFFFFFFFFFFFF), _s64(v >> 64)
                d[1] = float(rng.normal(0, 1e6))
                d[2] = float(abs(rng.normal(0, 1e15)))
        elif k == "dtype":
            i[:5] = [0 if empty else int(v) for v in rng.integers(0, 1 << 30, 5)]
        elif k in ("boolmap", "str_in"):
            i[1] = n
            i[0] = int(rng.integers(0, n + 1)) if n else 0
        body += struct.pack("<10q6d", *i, *d)
    regs = bytes(0 if empty else int(v) for v in rng.integers(0, 40, 512 * n_hll))
    rows = 0 if empty else int(rng.integers(1, 1 << 41))
    return struct.pack("<4Q", MAGIC, len(kinds), n_hll, rows) + body + regs


def _host_state(plan, img=None):
    import ctypes
    from deequ_amd import _native as N
    st = ctypes.c_void_p()
    N.check(N.lib.dq_state_create(plan.handle, -1, ctypes.byref(st)))
    if img is not None:
        buf = ctypes.create_string_buffer(img, len(img))
        N.check(N.lib.dq_state_deserialize(st, buf, len(img)))
    return st


def _serialized(st):
    from deequ_amd.distributed import serialize_state
    return serialize_state(_plan(), st)


def _worker(rank, world, port, seed, out_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from deequ_amd import _native as N
        from deequ_amd.distributed import exchange_states, merge_serialized
        plan = _plan()
        imgs = [_image(plan, seed, r) for r in range(world)]
        # the reference: dq_state_merge of every rank's state in rank order
        ref = _host_state(plan)
        tmp = _host_state(plan)
        import ctypes
        for img in imgs:
            buf = ctypes.create_string_buffer(img, len(img))
            N.check(N.lib.dq_state_deserialize(tmp, buf, len(img)))
            N.check(N.lib.dq_state_merge(ref, tmp))
        ref_bytes = _serialized(ref)
        ref_row = merge_serialized(plan, imgs)
        # the exchange
        st = _host_state(plan, imgs[rank])
        row = exchange_states(plan, st)
        got_bytes = _serialized(st)
        for h in (ref, tmp, st):
            N.lib.dq_state_destroy(h)
        out_q.put((rank, got_bytes == ref_bytes, repr(row) == repr(ref_row), got_bytes.hex()))  # (NaN-safe)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,seed", [(2, 1), (2, 2), (3, 3), (3, 4)])
def test_exchange_equals_rank_ordered_merge_byte_for_byte(world, seed):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r][0], f"rank {r}: exchanged state differs from the rank-ordered merge"
        assert res[r][1], f"rank {r}: result row differs"
    assert len({res[r][2] for r in range(world)}) == 1  # every rank holds the same state


def test_exchange_sizes_follow_the_plan():
    import ctypes
    from deequ_amd import _native as N
    plan = _plan()
    kinds = _kinds(plan)
    ns, nm, nd, nh = (ctypes.c_int64() for _ in range(4))
    N.check(N.lib.dq_state_exchange_sizes(plan.handle, ctypes.byref(ns), ctypes.byref(nm),
                                          ctypes.byref(nd), ctypes.byref(nh)))
    T, H = len(kinds), kinds.count("hll")
    assert "decimal" in kinds
    assert (ns.value, nm.value, nd.value, nh.value) == (10 * T + 1, 2 * T, 16 * T, 512 * H)
