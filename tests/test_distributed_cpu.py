"""world_size-2 `gloo` test of the multi-GPU exchange step on the CPU.

Each rank holds the aggregation buffer of its contiguous row shard -- built here from the shard's
values exactly as the scan kernels would leave it (n, wrapping Long sum, min/max keys, Welford
(avg, m2), the predicate counters) -- and then runs the product's exchange step
(`merge_states_across_ranks`: all-gather of the serialized states + rank-ordered merge through
dq_state_merge).  The merged row must equal the single-pass oracle over the whole column: counts,
wrapping sums and extremes bit-exact, (avg, m2) within the 1e-12 relative tolerance of
StandardDeviation (Spark's Chan merge, StandardDeviation.scala:37-44).  No GPU is touched: the
states are host-only (dq_state_create(device = -1)).
"""
import os
import socket
import struct

import numpy as np
import pytest

MAGIC = 0x3130514445455144  # "DQEEDQ01", the engine's serialized-state header (api.cpp)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _suite():
    from deequ_amd.analyzers import (Compliance, Maximum, Mean, Minimum, Size, StandardDeviation,
                                     Sum)
    return [Size(), Sum("x"), Mean("x"), StandardDeviation("x"), Minimum("x"), Maximum("x"),
            Compliance("x non-negative", "x >= 0")]


def _schema():
    from deequ_amd import _native as N
    from deequ_amd.table import StructField, StructType
    return StructType([StructField("x", N.INT64)])


def _column(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.integers(-(2 ** 40), 2 ** 40, size=n, dtype=np.int64)
    x[:5] = np.iinfo(np.int64).max  # forces the Long sum to wrap
    valid = rng.random(n) > 0.05
    return x, valid


def _wrapping_sum(xs):
    return int(np.sum(xs.astype(np.uint64), dtype=np.uint64).astype(np.int64))


def _shard_image(plan, x, valid):
    """The serialized state a rank's scan would produce for its shard (one TK_NUMERIC task)."""
    text = plan.explain()
    assert text.count("task[") == 1 and "numeric" in text, text
    xs = x[valid]
    n = int(xs.size)
    i = [0] * 10
    d = [0.0] * 6
    i[0] = n
    i[1] = _wrapping_sum(xs) if n else 0
    i[2] = int(xs.min()) if n else int(np.iinfo(np.int64).max)
    i[3] = int(xs.max()) if n else int(np.iinfo(np.int64).min)
    i[4] = int(np.sum(xs >= 0))  # predicate TRUE
    i[7] = n                     # predicate non-NULL
    avg = m2 = 0.0
    for k, v in enumerate(xs.astype(np.float64).tolist(), 1):  # CentralMomentAgg update per row
        delta = v - avg
        avg += delta / k
        m2 += delta * (v - avg)
    d[0] = float(np.sum(xs.astype(np.float64)))
    d[1], d[2] = avg, m2
    hdr = struct.pack("<4Q", MAGIC, 1, 0, int(x.size))
    return hdr + struct.pack("<10q6d", *i, *d)


def _worker(rank, world, port, n, seed, out_q):
    import ctypes

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from deequ_amd import _native as N
        from deequ_amd.distributed import merge_states_across_ranks, shard_bounds
        from deequ_amd.runners.engine import get_plan
        suite = _suite()
        plan = get_plan(_schema(), [s for a in suite for s in a.aggregation_functions()])
        x, valid = _column(n, seed)
        lo, hi = shard_bounds(n, rank, world, align=64)
        img = _shard_image(plan, x[lo:hi], valid[lo:hi])
        st = ctypes.c_void_p()
        N.check(N.lib.dq_state_create(plan.handle, -1, ctypes.byref(st)))
        buf = ctypes.create_string_buffer(img, len(img))
        N.check(N.lib.dq_state_deserialize(st, buf, len(img)))
        row = merge_states_across_ranks(plan, st)
        N.lib.dq_state_destroy(st)
        out_q.put((rank, row))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [1000, 4099])
def test_gloo_world2_merge_matches_single_pass(n):
    import torch.multiprocessing as mp
    world, seed = 2, 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    rows = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert rows[0] == rows[1]  # every rank merges in rank order: identical rows

    x, valid = _column(n, seed)
    xs = x[valid]
    size, s, mean_sum, mean_cnt, sd, mn, mx, c_true, c_cnt = rows[0]
    assert size == n and mean_cnt == n
    wrapped = _wrapping_sum(xs)
    assert s == float(wrapped) and mean_sum == float(wrapped)
    assert mn == float(xs.min()) and mx == float(xs.max())
    assert c_true == int(np.sum(xs >= 0)) and c_cnt == n
    f = xs.astype(np.float64)
    m2 = float(np.sum((f - f.mean()) ** 2))
    assert sd[0] == xs.size
    assert sd[1] == pytest.approx(f.mean(), rel=1e-12)
    assert sd[2] == pytest.approx(m2, rel=1e-12)


def _exchange_worker(rank, world, port, out_q):
    """Each rank sends owner segment j (records tagged (src, dst, i), var bytes tagged too) to rank
    j through the product's exchange step (deequ_amd.distributed.exchange_segments)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from deequ_amd.distributed import exchange_segments
        rc = np.array([(rank + 2 * j) % 4 for j in range(world)], np.int64)   # ragged, some empty
        vb = np.array([8 * ((rank * 3 + j) % 3) for j in range(world)], np.int64)
        recs, var = [], []
        for j in range(world):
            for i in range(int(rc[j])):
                recs.append(np.array([rank, j, i], np.uint64))
            var.append(np.full(int(vb[j]), 16 * rank + j, np.uint8))
        rec_t = torch.from_numpy(np.concatenate(recs).view(np.uint8).copy() if recs
                                 else np.zeros(0, np.uint8))
        var_t = torch.from_numpy(np.concatenate(var))
        got_rec, got_var, src_rc, src_vb = exchange_segments(rec_t, var_t, rc, vb)
        out_q.put((rank, got_rec.numpy().view(np.uint64).reshape(-1, 3).tolist(),
                   got_var.numpy().tolist(), src_rc.tolist(), src_vb.tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_world3_frequency_segment_exchange():
    """The all-to-all of the multi-GPU frequency path routes owner segment j of
    every rank to rank j, sources in rank order, with ragged and empty segments."""
    import torch.multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (rec, var, rc, vb) for r, rec, var, rc, vb in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for dst in range(world):
        rec, var, rc, vb = res[dst]
        exp_rec, exp_var = [], []
        for src in range(world):
            n = (src + 2 * dst) % 4
            exp_rec += [[src, dst, i] for i in range(n)]
            exp_var += [16 * src + dst] * (8 * ((src * 3 + dst) % 3))
            assert rc[src] == n
        assert rec == exp_rec
        assert var == exp_var


def _varbytes_worker(rank, world, port, out_q):
    """Each rank gathers a ragged byte string (empty on rank 1) and a packed group list through the
    product's device-gather helpers (deequ_amd.distributed.all_gather_varbytes, _pack_groups)."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from deequ_amd.distributed import _pack_groups, _unpack_groups, all_gather_varbytes
        payload = b"" if rank == 1 else bytes(range(rank * 7 % 251)) * (rank + 1)
        got = all_gather_varbytes(payload)
        counts = np.arange(rank + 2, dtype=np.int64) * 10 + rank
        offs = np.arange(rank + 3, dtype=np.int64) * 12
        raw = np.full(12 * (rank + 2), rank, np.uint8)
        groups = [tuple(a.tolist() for a in _unpack_groups(b))
                  for b in all_gather_varbytes(_pack_groups(counts, offs, raw))]
        out_q.put((rank, got, groups))
    finally:
        dist.destroy_process_group()


def test_gloo_world3_varbytes_gather():
    """The tensor all-gather that carries Histogram's per-rank top-k, frequency exports and
    quantile summaries (instead of pickled objects): ragged and empty payloads arrive intact, in
    rank order, on every rank."""
    import torch.multiprocessing as mp
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_varbytes_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (got, groups) for r, got, groups in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = [b"" if r == 1 else bytes(range(r * 7 % 251)) * (r + 1) for r in range(world)]
    for r in range(world):
        got, groups = res[r]
        assert got == exp
        for src, (counts, offs, raw) in enumerate(groups):
            assert counts == (np.arange(src + 2) * 10 + src).tolist()
            assert offs == (np.arange(src + 3) * 12).tolist()
            assert raw == [src] * (12 * (src + 2))
