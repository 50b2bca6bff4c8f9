"""Host-side profile of one configs[4] step (AnalysisRunner over the c5 suite): cProfile of the
Python runner with the native calls' time attributed to their Python callers (ctypes calls are not
separate entries).  Used to find the host gaps between the step's kernels.

Usage: python tools/trace_c5_host.py [--rows N] [--top K]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=125_000_000)
    ap.add_argument("--top", type=int, default=45)
    args = ap.parse_args()
    import torch
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.synth import profiling_table_device
    from tools.bench_workloads import c5_suite
    table = profiling_table_device(args.rows, batch_rows=1 << 25, device="cuda:0")
    torch.cuda.empty_cache()
    suite = c5_suite()
    AnalysisRunner.do_analysis_run(table, suite)  # warm-up: pools, kernels, caches
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    AnalysisRunner.do_analysis_run(table, suite)
    torch.cuda.synchronize()
    print(f"step without profiler: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    AnalysisRunner.do_analysis_run(table, suite)
    torch.cuda.synchronize()
    pr.disable()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(args.top)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
