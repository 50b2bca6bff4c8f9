"""The determinism contract of the group-by's fp64 outputs.

Entropy (-p ln p per group) and MutualInformation (p ln(p / (px py)) per joint group) are sums of
per-group fp64 terms.  The engine adds the terms as 128-bit fixed-point integers at 2^-112
(freq.hip fix_of: exact for every term >= 2^-60), so the sum does not depend on the order the
groups are met in.  Contract, asserted here:
  * bit-identical across runs on freshly built tables, across batchings of the same rows, across
    partition depths (DQ_FREQ_PARTITION_TARGET: the sub-bucket bits) and the recount path of
    overflowing partitions, and across the two marginal-lookup paths of MutualInformation;
  * within 1e-12 relative of the exactly rounded sum of the same terms (math.fsum; Spark's own
    sequential sum depends on its partitioning in the last bits and drifts with many groups).
Reference: GroupingAnalyzers.scala (Entropy :170-189), MutualInformation.scala:35-97.
"""
import math

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


def _table(n, seed):
    """Counts of every kind the statistics treat apart: 1, 2..63 (histogrammed), >= 64 (summed
    term by term), in an int64 column (exact mode) and a string column (hashed mode)."""
    rng = np.random.default_rng(seed)
    heavy = rng.integers(0, 40, n // 4)                       # ~40 groups of ~n/160 rows
    mid = rng.integers(1000, 1000 + n // 20, n // 4)          # counts ~5
    uniq = np.arange(10 ** 6, 10 ** 6 + n - 2 * (n // 4))     # count 1
    x = np.concatenate([heavy, mid, uniq]).astype(np.int64)
    rng.shuffle(x)
    mask = rng.random(n) < 0.03
    y = rng.integers(0, 300, n)
    return pa.table({"x": pa.array(x, mask=mask),
                     "s": pa.array([None if m else f"k{v:07d}" for v, m in zip(x, mask)]),
                     "y": pa.array([f"y{v}" for v in y])})


def _run(t, device, batch, analyzers):
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    df = Table.from_arrow(t, device=device, max_batch_rows=batch)
    ctx = AnalysisRunner.do_analysis_run(df, analyzers)
    return [ctx.metric(a).value.get() for a in analyzers]


def test_entropy_is_bit_stable_across_runs_batchings_and_partitionings(gpu_device, monkeypatch):
    from deequ_amd.analyzers import Entropy
    from oracle.deequ_oracle import OTable, frequencies
    t = _table(300_007, 5)
    suite = [Entropy("x"), Entropy("s")]
    ref = _run(t, gpu_device, 1 << 20, suite)
    runs = {"fresh table": _run(t, gpu_device, 1 << 20, suite),
            "batches of 7000": _run(t, gpu_device, 7000, suite),
            "batches of 65537": _run(t, gpu_device, 65537, suite)}
    for target in ("20", "300", "1000000000"):  # deep partitions .. s = 0 with recounts
        monkeypatch.setenv("DQ_FREQ_PARTITION_TARGET", target)
        runs["partition target " + target] = _run(t, gpu_device, 1 << 20, suite)
    monkeypatch.delenv("DQ_FREQ_PARTITION_TARGET")
    for what, got in runs.items():
        assert got == ref, (what, got, ref)  # bit for bit
    ot = OTable({c: t.column(c).to_pylist() for c in ("x", "s")}, {"x": "long", "s": "string"})
    n = t.num_rows
    for a, got in zip(suite, ref):
        # the exactly rounded sum of the terms (math.fsum): a sequential sum of ~1e5 equal small
        # terms drifts by ~1e-11 relative on its own (each add rounds the same way)
        exp = math.fsum(-(c / n) * math.log(c / n) for c in frequencies(ot, [a.column]).values())
        assert abs(got - exp) <= 1e-12 * exp, (str(a), got, exp)


def test_mutual_information_is_bit_stable(gpu_device, monkeypatch):
    from deequ_amd.analyzers import MutualInformation
    from oracle.deequ_oracle import OTable, mutual_information
    t = _table(200_003, 9)
    suite = [MutualInformation("x", "y"), MutualInformation("s", "y")]
    ref = _run(t, gpu_device, 1 << 20, suite)
    runs = {"fresh table": _run(t, gpu_device, 1 << 20, suite),
            "batches of 9000": _run(t, gpu_device, 9000, suite)}
    monkeypatch.setenv("DQ_FREQ_MI_LOOKUP", "1")  # marginals by key bytes instead of by hash
    runs["byte lookups"] = _run(t, gpu_device, 1 << 20, suite)
    monkeypatch.delenv("DQ_FREQ_MI_LOOKUP")
    monkeypatch.setenv("DQ_FREQ_PARTITION_TARGET", "50")
    runs["partition target 50"] = _run(t, gpu_device, 1 << 20, suite)
    monkeypatch.delenv("DQ_FREQ_PARTITION_TARGET")
    for what, got in runs.items():
        assert got == ref, (what, got, ref)
    ot = OTable({c: t.column(c).to_pylist() for c in ("x", "s", "y")},
                {"x": "long", "s": "string", "y": "string"})
    for a, got in zip(suite, ref):
        exp = mutual_information(ot, a.columns[0], a.columns[1])
        assert abs(got - exp) <= 1e-12 * abs(exp), (str(a), got, exp)
