"""Times sub-suites of S10 separately on the device-resident synthetic Item table (diagnostic).

Usage: python tools/scan_ablation.py [rows] [reps]
Prints one line per sub-suite: ms per scan launch (HIP events), algorithmic bytes, GB/s.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    from deequ_amd import _native as N
    from deequ_amd.analyzers import (Completeness, Compliance, Maximum, Mean, Minimum, Size,
                                     StandardDeviation, Sum)
    from deequ_amd.runners.engine import get_plan, scan_into
    from deequ_amd.synth import item_table_device
    table = item_table_device(rows, seed=7, device="cuda:0")
    nv = Compliance("numViews is non-negative", "numViews >= 0")
    pr = Compliance("priority contained in high,low", "priority IS NULL OR priority IN ('high','low')")
    moments = [Sum("numViews"), Mean("numViews"), StandardDeviation("numViews"),
               Minimum("numViews"), Maximum("numViews")]
    n = rows
    vb = (n + 7) // 8
    pbytes = sum(int(b["priority"].values[b["priority"].length].item()) for b in table.batches)
    suites = {
        "size": ([Size()], 0),
        "completeness(id)": ([Completeness("id")], vb),
        "completeness(id,name)": ([Completeness("id"), Completeness("name")], 2 * vb),
        "numeric pred only": ([nv], 8 * n + vb),
        "numeric moments": (moments, 8 * n + vb),
        "numeric all": (moments + [nv], 8 * n + vb),
        "str_in priority": ([pr], 4 * n + pbytes + vb),
        "S10": ([Size(), Completeness("id"), Completeness("name"), nv, pr] + moments,
                4 * vb + 8 * n + 4 * n + pbytes),
    }
    stream = torch.cuda.current_stream()
    sh = ctypes.c_void_p(stream.cuda_stream)
    for name, (suite, nbytes) in suites.items():
        specs = [s for a in suite for s in a.aggregation_functions()]
        plan = get_plan(table.schema, specs)
        st = plan.state(0)
        for _ in range(2):
            N.check(N.lib.dq_state_reset(st))
            scan_into(table, plan, st, sh)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            N.check(N.lib.dq_state_reset(st))
            scan_into(table, plan, st, sh)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"{name:28s} {ms:9.3f} ms  {nbytes / 1e9:7.3f} GB  {nbytes / ms / 1e6:8.1f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
