"""Diagnostic (not a test): host-side pointer-range report for a mixed fixed-width + string
grouping on the 1-row table that faulted (DQ_CHECK_PTRS in a diagnostic build: the insert kernel is
NOT launched; dq_freq_add_device returns the report as its error)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
os.environ["DQ_CHECK_PTRS"] = "1"
from deequ_amd.analyzers.grouping import FrequencyTable  # noqa: E402
from deequ_amd.table import Table  # noqa: E402
from test_gpu_freq import _table  # noqa: E402

for n in (1, 5000):
    t = _table(n, seed=n + 1)
    df = Table.from_arrow(t, device="cuda:0")
    cols = ["id", "s"]
    ft = FrequencyTable(cols, [df.schema[c].dtype for c in cols], 0)
    try:
        for b in df.batches:
            ft.add([b[c] for c in cols])
    except Exception as e:  # noqa: BLE001
        print(n, e, flush=True)
