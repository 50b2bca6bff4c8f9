"""world-size-2 / 3 `gloo` test of the multi-GPU workload harness (tools/bench_workloads.py
--gpus N, run_distributed) on the CPU: the per-rank statistics gather, the report (whole-job
rows/s over the SLOWEST rank, weak scaling), and the collective byte accounting of the product's
exchange step (deequ_amd.distributed.COMM_BYTES: only bytes to / from other ranks count)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bench_workloads import dist_report, gather_rank_stats
        from deequ_amd import distributed as D
        D.reset_comm_bytes()
        # an exchange with known splits: rank r sends (r + 1) * (j + 1) records to rank j
        rc = np.array([(rank + 1) * (j + 1) for j in range(world)], np.int64)
        vb = np.zeros(world, np.int64)
        rb = 24
        rec = torch.zeros(int(rc.sum()) * rb, dtype=torch.uint8)
        D.exchange_segments(rec, torch.zeros(0, dtype=torch.uint8), rc, vb)
        sent, recv = D.COMM_BYTES["sent"], D.COMM_BYTES["recv"]
        secs, s_all, r_all = gather_rank_stats(1.0 + rank, sent, recv, "cpu")
        rep = dist_report("c3", secs, 4, 1000, s_all, r_all, dist.get_backend())
        q.put((rank, sent, recv, secs, s_all, r_all, rep))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_harness_gather_and_report(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rb = 24
    for r in range(world):
        sent, recv, secs, s_all, r_all, rep = res[r]
        # off-rank record bytes + the sizes' all-to-all (16 B per peer each way)
        exp_sent = sum((r + 1) * (j + 1) * rb for j in range(world) if j != r) + 16 * (world - 1)
        exp_recv = sum((j + 1) * (r + 1) * rb for j in range(world) if j != r) + 16 * (world - 1)
        assert (sent, recv) == (exp_sent, exp_recv)
        assert secs == [1.0 + k for k in range(world)]          # every rank sees every rank
        assert s_all == [res[k][0] for k in range(world)] and r_all == [res[k][1] for k in range(world)]
        assert rep["n_gpus"] == world and rep["scaling"] == "weak" and rep["rows"] == 1000 * world
        assert rep["ms_per_step"] == pytest.approx(world / 4 * 1e3)   # the slowest rank: world s
        assert rep["value"] == pytest.approx(1000 * world * 4 / world)
        assert rep["collective_bytes_per_step"]["sent"] == [b / 4 for b in s_all]
        assert rep["collective_bytes_per_step"]["backend"] == "gloo"
