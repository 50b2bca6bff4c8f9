"""One rank of the two-rank run of tests/test_gpu_distributed.py: both ranks share cuda:0 and
meet over gloo (127.0.0.1).  Rank r takes its contiguous row shard of the seeded table, runs
AnalysisRunner over it (scan -> all-gather + rank-ordered merge; groupings and Histogram -> local
partial group-by + owner repartition), and rank 0 writes the metrics as JSON.

usage: python tests/workers/dist_ranks.py RANK WORLD PORT OUT_JSON"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def exchange_check(df):
    """The scan states of the suite exchanged on the device (exchange_states: SUM / MAX
    all-reduces + the gathered moments merged by a kernel) and by the serialized all-gather +
    rank-ordered host merge (merge_states_across_ranks): the merged states' bytes must agree.
    Also returns the engine's host waits during the device exchange (dq_host_wait_count): one,
    the merged state's read-back (dq_state_sync)."""
    import ctypes

    from deequ_amd import _native as N
    from deequ_amd.analyzers.base import ScanShareableAnalyzer
    from deequ_amd.distributed import exchange_states, merge_states_across_ranks, serialize_state
    from deequ_amd.runners.engine import get_plan, scan_into
    from dist_suite import suite
    specs = [s for a in suite() if isinstance(a, ScanShareableAnalyzer)
             for s in a.aggregation_functions()]
    plan = get_plan(df.schema, specs)
    out = []
    for how in ("device", "host"):
        st = ctypes.c_void_p()
        N.check(N.lib.dq_state_create(plan.handle, 0, ctypes.byref(st)))
        scan_into(df, plan, st)
        if how == "device":
            w0 = N.lib.dq_host_wait_count()
            row = exchange_states(plan, st, df.device)
            waits = N.lib.dq_host_wait_count() - w0  # the engine's host waits in the exchange
            img = serialize_state(plan, st)
        else:
            row = merge_states_across_ranks(plan, st, df.device)
            from deequ_amd.distributed import all_gather_bytes
            imgs = all_gather_bytes(serialize_state(plan, st), df.device)
            acc, tmp = ctypes.c_void_p(), ctypes.c_void_p()
            N.check(N.lib.dq_state_create(plan.handle, -1, ctypes.byref(acc)))
            N.check(N.lib.dq_state_create(plan.handle, -1, ctypes.byref(tmp)))
            for b in imgs:
                buf = ctypes.create_string_buffer(b, len(b))
                N.check(N.lib.dq_state_deserialize(tmp, buf, len(b)))
                N.check(N.lib.dq_state_merge(acc, tmp))
            img = serialize_state(plan, acc)
            N.lib.dq_state_destroy(acc)
            N.lib.dq_state_destroy(tmp)
        N.lib.dq_state_destroy(st)
        out.append((img, repr(row)))
    return [out[0][0] == out[1][0], out[0][1] == out[1][1], waits]


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    from dist_suite import metrics_of, suite, table
    from deequ_amd.distributed import shard_bounds
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    t = table()
    lo, hi = shard_bounds(t.num_rows, rank, world, align=1024)
    df = Table.from_arrow(t.slice(lo, hi - lo), device="cuda:0", max_batch_rows=6000)
    ctx = AnalysisRunner.do_analysis_run(df, suite())
    res = metrics_of(ctx)
    res["__exchange__"] = exchange_check(df)
    dist.barrier()
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
