"""Experiment: configs[2]'s two group-bys (int64 `id`, string `priority`) with `priority`'s table
driven on a side HIP stream, so its kernels can fill CUs `id`'s phases leave idle.  Prints the
per-step time of the plain order (both on the current stream) and of the overlapped one, and
checks that both orders give the same results.  Not product code: a measurement for DESIGN.md.

Usage: python tools/exp_c3_overlap.py [--rows N] [--steps K]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from deequ_amd import _native as N
    from deequ_amd.analyzers.grouping import FrequencyTable, KeyedFrequencies, _fold_null_group
    from deequ_amd.synth import item_table_device
    table = item_table_device(args.rows, seed=9, batch_rows=1 << 26, device="cuda:0")
    torch.cuda.synchronize()
    fid = FrequencyTable(["id"], [N.INT64], 0, capacity_hint=args.rows)
    fpr = FrequencyTable(["priority"], [N.UTF8], 0)
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def finish(ft, dtype):
        top, bins = _fold_null_group(ft, dtype, 1000)
        s = KeyedFrequencies(ft).summarize()
        return (bins, len(top), s.n_groups, s.n_unique, s.entropy)

    def plain():
        out = []
        for col, ft, dt in (("id", fid, N.INT64), ("priority", fpr, N.UTF8)):
            ft.reset()
            for b in table.batches:
                ft.add([b[col]], null_as_group=True)
            out.append(finish(ft, dt))
        return out

    def overlapped():
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            fpr.reset()
            for b in table.batches:
                fpr.add([b["priority"]], null_as_group=True)
        fid.reset()
        for b in table.batches:
            fid.add([b["id"]], null_as_group=True)
        r_id = finish(fid, N.INT64)
        with torch.cuda.stream(side):
            r_pr = finish(fpr, N.UTF8)
        main_s.wait_stream(side)
        return [r_id, r_pr]

    res = {}
    for name, fn in (("plain", plain), ("overlapped", overlapped), ("plain2", plain),
                     ("overlapped2", overlapped)):
        for _ in range(2):
            ref = fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            got = fn()
        torch.cuda.synchronize()
        res[name] = 1e3 * (time.perf_counter() - t0) / args.steps
        res[name + "_result"] = repr(got)
        assert repr(got) == repr(ref)
    assert res["plain_result"] == res["overlapped_result"], (res["plain_result"],
                                                           res["overlapped_result"])
    print(json.dumps({k: v for k, v in res.items() if not k.endswith("_result")}), flush=True)


if __name__ == "__main__":
    main()
