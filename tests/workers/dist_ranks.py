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
    dist.barrier()
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
