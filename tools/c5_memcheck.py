"""Device-memory check of the configs[4] suite across steps: after each AnalysisRunner step, the
free device memory, the FrequencyTable objects still alive (and what holds the first of them),
and what gc.collect() finds.  Usage: python tools/c5_memcheck.py [rows] [steps]"""
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    import torch
    from deequ_amd import analyzers as A
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.synth import profiling_table_device
    table = profiling_table_device(rows, batch_rows=1 << 25, device="cuda:0")
    torch.cuda.empty_cache()
    num = ["id"] + [f"numViews_{k}" for k in range(5)] + [f"score_{k}" for k in range(4)]
    strs = ([f"name_{k}" for k in range(3)] + [f"priority_{k}" for k in range(3)]
            + [f"description_{k}" for k in range(4)])
    suite = [A.Size()]
    for c in num + strs:
        suite += [A.Completeness(c), A.ApproxCountDistinct(c), A.Uniqueness([c]),
                  A.Distinctness([c]), A.UniqueValueRatio([c]), A.CountDistinct([c]),
                  A.Entropy(c), A.Histogram(c)]
    for c in num:
        suite += [A.Sum(c), A.Mean(c), A.StandardDeviation(c), A.Minimum(c), A.Maximum(c),
                  A.Compliance(f"{c} non-negative", f"{c} >= 0"), A.ApproxQuantile(c, 0.5)]
    for c in strs:
        suite += [A.DataType(c), A.PatternMatch(c, A.Patterns.URL)]
    suite += [A.Correlation("numViews_0", "score_0"), A.MutualInformation("name_0", "priority_2")]
    gc.disable()
    for s in range(steps):
        t0 = time.perf_counter()
        ctx = AnalysisRunner.do_analysis_run(table, suite)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        del ctx
        free, total = torch.cuda.mem_get_info()
        alive = [o for o in gc.get_objects() if isinstance(o, FrequencyTable)]
        print(f"step {s}: {dt * 1e3:.1f} ms, free {free / 2**30:.1f} GiB of {total / 2**30:.1f}, "
              f"FrequencyTables alive {len(alive)}", flush=True)
        if alive:
            o = alive[0]
            chain = []
            for _ in range(6):
                refs = [r for r in gc.get_referrers(o) if r is not alive and not isinstance(r, list)]
                if not refs:
                    break
                r = refs[0]
                chain.append(type(r).__name__ + (":" + ",".join(list(r.keys())[:6]) if isinstance(r, dict) else ""))
                o = r
            print("   held by: " + " <- ".join(chain), flush=True)
        del alive
        n = gc.collect()
        free2, _ = torch.cuda.mem_get_info()
        print(f"   gc.collect(): {n} objects, free after {free2 / 2**30:.1f} GiB", flush=True)


if __name__ == "__main__":
    main()
