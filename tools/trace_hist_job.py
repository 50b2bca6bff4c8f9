"""Host time of each stage of one Histogram job of configs[4] (create, each batch's add, the
top-k / NULL-group / count calls, destroy), to find the host gaps between the step's kernels.

Usage: python tools/trace_hist_job.py [--rows N] [--columns a,b]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=125_000_000)
    ap.add_argument("--columns", default="numViews_0,name_0")
    args = ap.parse_args()
    import torch
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.synth import profiling_table_device
    table = profiling_table_device(args.rows, batch_rows=1 << 25, device="cuda:0")
    torch.cuda.empty_cache()
    us = lambda a, b: f"{1e6 * (b - a):8.1f}"  # noqa: E731
    for col in args.columns.split(","):
        dtype = table.schema[col].dtype
        for rep in range(4):
            torch.cuda.synchronize()
            t = [time.perf_counter()]
            ft = FrequencyTable([col], [dtype], 0, capacity_hint=table.num_rows)
            t.append(time.perf_counter())
            for b in table.batches:
                ft.add([b[col]], null_as_group=True)
                t.append(time.perf_counter())
            torch.cuda.synchronize()
            t.append(time.perf_counter())
            ft.topk_raw(1002)
            t.append(time.perf_counter())
            ft.null_literal()
            ft.count()
            t.append(time.perf_counter())
            del ft
            t.append(time.perf_counter())
            print(f"{col} rep {rep}: create {us(t[0], t[1])} adds "
                  + " ".join(us(t[i], t[i + 1]) for i in range(1, len(t) - 5))
                  + f" | device {us(t[-5], t[-4])} topk {us(t[-4], t[-3])} null+count "
                  f"{us(t[-3], t[-2])} destroy {us(t[-2], t[-1])} (us)", flush=True)


if __name__ == "__main__":
    main()
