"""One rank over RCCL (backend "nccl", world size 1, 127.0.0.1) on cuda:0: the device-side
collective branches of deequ_amd/distributed.py -- the scan-state exchange (all-reduce SUM / MAX,
all-gather of the moments on GPU tensors), the raw-key all-to-all and the partial-aggregate
repartition, and DistributedFrequencies' reductions -- run on the GPU's own collectives, and
their results must equal the local (non-distributed) computation.  A world of one exchanges
nothing between ranks, but every collective call, buffer placement and device copy of the
`nccl` branches executes (the 2- and 8-rank runs need more GPUs than a test box has).

usage: python tests/workers/nccl_world1.py PORT OUT_JSON"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "workers"))


def main():
    port, out = int(sys.argv[1]), sys.argv[2]
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    from dist_ranks import exchange_check
    from dist_suite import table
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.distributed import compute_frequencies_distributed
    from deequ_amd.table import Table
    res = {"backend": dist.get_backend()}
    df = Table.from_arrow(table(), device="cuda:0", max_batch_rows=6000)
    res["exchange"] = exchange_check(df)
    fr = {}
    for col in ("uid", "uid32", "id", "s"):
        dist_f = compute_frequencies_distributed(df, [col], null_as_group=False)
        s = dist_f.frequencies.summarize()
        local = FrequencyTable([col], [df.schema[col].dtype], 0)
        for b in df.batches:
            local.add([b[col]])
        ls = local.summarize()
        fr[col] = [[int(s.n_groups), int(s.n_unique), float(s.entropy)],
                   [int(ls.n_groups), int(ls.n_unique), float(ls.entropy)],
                   [c for _, c in dist_f.frequencies.topk(5)], [c for _, c in local.topk(5)]]
    res["frequencies"] = fr
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
