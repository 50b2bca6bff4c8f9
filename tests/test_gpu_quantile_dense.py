"""ApproxQuantile's dense counting select (quantile.hip rs_dense): an integer column whose values
span few enough consecutive integers has its ranks read off per-value counts instead of the
radix select's passes (up to 40,960 values: 160 KiB of LDS counters).  Both pick the values at the same exact ranks floor(j (n - 1) / (m - 1))
of the summary, so the metrics must be identical to the radix select's (DQ_QUANTILE_DENSE=0) and
within relativeError * n of the exact rank (ApproxQuantile.scala:41-104, Spark's
ApproximatePercentile)."""
import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

CASES = [  # (arrow type, low, high, rows, batch rows)
    (pa.int32(), -5000, 20000, 300_000, 30_000),     # 10 batches: two launches of 8 sources
    (pa.int8(), -128, 127, 100_000, 100_000),
    (pa.int16(), -300, 300, 80_000, 20_000),
    (pa.int64(), 10 ** 12, 10 ** 12 + 40959, 200_000, 50_000),  # the window's full width
    (pa.int64(), 0, 40960, 200_000, 50_000),         # one value too wide: the radix select
    (pa.int64(), 7, 7, 50_000, 50_000),              # one distinct value
]
QS = [0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_dense_select_equals_radix_select(case, gpu_device, monkeypatch):
    from deequ_amd.analyzers import ApproxQuantile
    from deequ_amd.table import Table
    from oracle.deequ_oracle import quantile_rank_error
    at, lo, hi, n, batch = CASES[case]
    rng = np.random.default_rng(case)
    v = rng.integers(lo, hi, n, endpoint=True, dtype=np.int64)
    if hi > lo:
        v[:2] = [lo, hi]
    mask = rng.random(n) < 0.05
    mask[:2] = False
    df = Table.from_arrow(pa.table({"x": pa.array(v, mask=mask, type=at)}), device=gpu_device,
                          max_batch_rows=batch)
    got = [ApproxQuantile("x", q).calculate(df).value.get() for q in QS]
    monkeypatch.setenv("DQ_QUANTILE_DENSE", "0")
    ref = [ApproxQuantile("x", q).calculate(df).value.get() for q in QS]
    assert got == ref, (got, ref)
    vals = v[~mask].astype(np.float64)
    for q, g in zip(QS, got):
        assert quantile_rank_error(vals, q, g) <= 0.01 * len(vals), (q, g)
