"""Host-side cost of one S10 bench step, part by part (GPU box): dq_state_reset, scan_into's
host work (until the launch call returns), dq_state_sync (waits for the GPU), read_row."""
import ctypes
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402
from deequ_amd import _native as N  # noqa: E402
from deequ_amd.runners.engine import get_plan, read_row, scan_into  # noqa: E402
from deequ_amd.synth import item_table_device  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
table = item_table_device(rows, seed=7, batch_rows=1 << 26, device="cuda:0")
suite = bench.s10_suite()
specs = [s for a in suite for s in a.aggregation_functions()]
plan = get_plan(table.schema, specs)
state = plan.state(0)
sh = ctypes.c_void_p(torch.cuda.current_stream("cuda:0").cuda_stream)
acc = {"reset": 0.0, "scan_into": 0.0, "sync": 0.0, "read_row": 0.0}
K = 20
for it in range(K + 3):
    t0 = time.perf_counter()
    N.check(N.lib.dq_state_reset(state))
    t1 = time.perf_counter()
    scan_into(table, plan, state, sh)
    t2 = time.perf_counter()
    N.check(N.lib.dq_state_sync(state))
    t3 = time.perf_counter()
    read_row(plan, state)
    t4 = time.perf_counter()
    if it >= 3:
        for k, v in zip(acc, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            acc[k] += v / K
print({k: round(v * 1e6, 1) for k, v in acc.items()}, "us per step")
