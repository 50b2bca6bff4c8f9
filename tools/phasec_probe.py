"""Diagnostic: one group-by of a high-cardinality string column (the configs[4] `name` column,
1.25e8 rows) with DQ_FREQ_DEBUG=2 phase timings (phase A tiles, phase C items of workgroup 0)
and the device time of its finalize.

Usage: DQ_FREQ_DEBUG=2 python tools/phasec_probe.py [rows] [column]  (configs[4] columns too)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
    col = sys.argv[2] if len(sys.argv) > 2 else "name"
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.synth import item_table_device, profiling_table_device
    if col in ("name", "priority", "id", "numViews"):
        t = item_table_device(rows, seed=101, device="cuda:0")
    else:  # a configs[4] column (description_0, name_0, ...)
        t = profiling_table_device(rows, batch_rows=1 << 25, device="cuda:0")
    torch.cuda.synchronize()
    for rep in range(2):
        ft = FrequencyTable([col], [t.schema[col].dtype], 0, capacity_hint=rows)
        t0 = time.perf_counter()
        for b in t.batches:
            ft.add([b[col]], null_as_group=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        s = ft.summarize()
        top = ft.topk(1000)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"rep {rep}: add {1e3 * (t1 - t0):.2f} ms, finalize+topk {1e3 * (t2 - t1):.2f} ms, "
              f"groups {s.n_groups}, unique {s.n_unique}, top1 {top[0][1]}", flush=True)


if __name__ == "__main__":
    main()
