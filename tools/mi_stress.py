"""Repeats MutualInformation(name_0, priority_2) on the configs[4] table and times its parts (the
joint group-by, its finalize, the device MI pass), to catch the intermittent multi-second runs
seen in the configs[4] suite.  Usage: python tools/mi_stress.py [rows] [reps]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    import torch
    from deequ_amd import _native as N
    from deequ_amd.analyzers.grouping import compute_frequencies
    from deequ_amd.synth import profiling_table_device
    table = profiling_table_device(rows, batch_rows=1 << 25, device="cuda:0")
    torch.cuda.empty_cache()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for i in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = compute_frequencies(table, ["name_0", "priority_2"])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        n = st.frequencies.count()  # finalize (phases B, C, compaction)
        t2 = time.perf_counter()
        mi, null = ctypes.c_double(), ctypes.c_int()
        N.check(N.lib.dq_freq_mutual_information(st.frequencies.handle, ctypes.byref(mi),
                                                 ctypes.byref(null), stream))
        t3 = time.perf_counter()
        print(f"rep {i}: add {1e3 * (t1 - t0):.1f} ms, finalize {1e3 * (t2 - t1):.1f} ms, "
              f"MI {1e3 * (t3 - t2):.1f} ms ({n} groups, mi {mi.value:.12f})", flush=True)
        del st


if __name__ == "__main__":
    main()
