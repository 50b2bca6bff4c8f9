"""The dense integer path of the group-by (freq.hip freq_dense_count / freq_dense_emit): a batch of
an integer or boolean key whose values span at most kDenseW consecutive values is counted by value
in LDS instead of written as a record per row.  Parity bar: every group's count bit-exact against
a host count of the same column (the reference's groupBy(col).count(),
GroupingAnalyzers.scala:53-80), NULL rows kept apart (or as the NULL group in Histogram mode), for
every integer width, negative and extreme values, the window's edges (kDenseW and kDenseW + 1
values), and
tables whose batches alternate between the dense path and the bucket pieces."""
from collections import Counter

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

W = 79 * 512  # freq.hip kDenseW: values a dense batch may span


def _groups(ft):
    return {k[0]: c for k, c in ft.export()}


def _expected(values, mask):
    return Counter(int(v) for v, m in zip(values, mask) if not m)


def _run(arr, dtype, device, batch, null_as_group=False):
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    df = Table.from_arrow(pa.table({"k": arr}), device=device, max_batch_rows=batch)
    ft = FrequencyTable(["k"], [dtype], 0)
    for b in df.batches:
        ft.add([b["k"]], null_as_group=null_as_group)
    return ft


CASES = [  # (arrow type, native type name, low, high)
    (pa.int8(), "INT8", -128, 127),
    (pa.int16(), "INT16", -20000, 12000),
    (pa.int32(), "INT32", -5, 30000),
    (pa.int64(), "INT64", -(1 << 62), -(1 << 62) + 25000),
    (pa.int64(), "INT64", (1 << 63) - 1 - 4000, (1 << 63) - 1),
    (pa.int64(), "INT64", -(1 << 63), -(1 << 63) + 100),
]


@pytest.mark.parametrize("null_as_group", [False, True])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_dense_counts_equal_host_counts(case, null_as_group, gpu_device):
    from deequ_amd import _native as N
    at, tn, lo, hi = CASES[case]
    rng = np.random.default_rng(case)
    n = 150_001
    v = rng.integers(lo, hi, n, endpoint=True, dtype=np.int64)
    v[:2] = [lo, hi]  # both ends of the range
    mask = rng.random(n) < 0.05
    mask[:2] = False
    ft = _run(pa.array(v, mask=mask, type=at), getattr(N, tn), gpu_device, 40_000, null_as_group)
    nulls = int(mask.sum())
    exp = _expected(v, mask)
    if null_as_group:  # (Histogram mode: the NULL rows are a group of their own)
        exp[None] = nulls
    assert _groups(ft) == exp
    s = ft.summarize()
    exp_groups = len(exp)
    assert s.n_groups == exp_groups
    assert s.n_null_key_rows == (0 if null_as_group else nulls)


def test_dense_boolean(gpu_device):
    from deequ_amd import _native as N
    rng = np.random.default_rng(7)
    n = 70_000
    v = rng.random(n) < 0.3
    mask = rng.random(n) < 0.1
    ft = _run(pa.array(v, mask=mask, type=pa.bool_()), N.BOOL, gpu_device, 30_000)
    exp = _expected(v.astype(np.int64), mask)
    assert _groups(ft) == {bool(k): c for k, c in exp.items()} or _groups(ft) == exp


@pytest.mark.parametrize("width", [W - 1, W])
def test_window_edges(width, gpu_device, monkeypatch):
    """Values spanning W - 1 (W values: the dense path) and W (W + 1 values: declined)."""
    from deequ_amd import _native as N
    rng = np.random.default_rng(width)
    n = 1_000_000
    v = rng.integers(0, width, n, endpoint=True, dtype=np.int64) - 1000
    v[:2] = [-1000, width - 1000]
    mask = np.zeros(n, bool)
    ft = _run(pa.array(v, type=pa.int64()), N.INT64, gpu_device, 1 << 20)
    assert _groups(ft) == _expected(v, mask)
    # records: the dense path leaves about one per value and digit, the pieces about one per row
    dense = ft.hll_words(n // 4) is not None
    assert dense == (width < W), (width, dense)
    monkeypatch.setenv("DQ_FREQ_DENSE", "0")
    ft0 = _run(pa.array(v, type=pa.int64()), N.INT64, gpu_device, 1 << 20)
    assert _groups(ft0) == _groups(ft)
    assert ft0.hll_words(n // 4) is None


def test_batches_alternate_between_paths(gpu_device):
    """A narrow batch (dense), a wide one (pieces; the table stops trying), narrow ones again:
    one table, every count exact, summary and top-k as with the pieces alone."""
    from deequ_amd import _native as N
    rng = np.random.default_rng(11)
    parts = [rng.integers(0, 3000, 50_000), rng.integers(-10 ** 12, 10 ** 12, 50_000),
             rng.integers(0, 3000, 50_000), rng.integers(100, 200, 50_000)]
    v = np.concatenate(parts).astype(np.int64)
    mask = rng.random(len(v)) < 0.02
    ft = _run(pa.array(v, mask=mask, type=pa.int64()), N.INT64, gpu_device, 50_000)
    exp = _expected(v, mask)
    assert _groups(ft) == exp
    top = ft.topk(5)
    want = sorted(exp.values(), reverse=True)[:5]
    assert sorted((c for _, c in top), reverse=True) == want


def test_runner_metrics_with_and_without_dense(gpu_device, monkeypatch):
    """The frequency family and Histogram over a dense column: the same metrics either way."""
    from deequ_amd.analyzers import (CountDistinct, Distinctness, Entropy, Histogram,
                                     UniqueValueRatio, Uniqueness)
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    rng = np.random.default_rng(5)
    n = 120_000
    g = np.minimum(rng.geometric(0.5, n) - 1, 40)
    v = ((1024 * g + rng.integers(0, 1024, n)) * 2) // 3  # numViews' shape
    mask = rng.random(n) < 0.05
    df = Table.from_arrow(pa.table({"v": pa.array(v, mask=mask, type=pa.int64())}),
                          device=gpu_device, max_batch_rows=50_000)
    suite = [Uniqueness(["v"]), Distinctness(["v"]), UniqueValueRatio(["v"]), CountDistinct(["v"]),
             Entropy("v"), Histogram("v")]
    got = AnalysisRunner.do_analysis_run(df, suite)
    monkeypatch.setenv("DQ_FREQ_DENSE", "0")
    ref = AnalysisRunner.do_analysis_run(df, suite)
    for a in suite[:-1]:
        assert got.metric(a).value.get() == ref.metric(a).value.get(), str(a)
    h1, h2 = got.metric(suite[-1]).value.get(), ref.metric(suite[-1]).value.get()
    assert h1.number_of_bins == h2.number_of_bins
    assert sorted(x.absolute for x in h1.values.values()) == \
        sorted(x.absolute for x in h2.values.values())


@pytest.mark.parametrize("cap", [None, "1", "9"])
@pytest.mark.parametrize("null_as_group", [False, True])
def test_fixed_capacity_pieces(cap, null_as_group, gpu_device, monkeypatch):
    """Exact keys the dense path declines (wide integers, doubles) go to fixed-capacity bucket
    pieces without the pre-pass (freq_phaseA_xp with AArgs::piece_cap): the same groups as the
    pre-pass layout (DQ_FREQ_XFIXED=0), with the default capacity and with tiny ones that send most
    records to the tiles' chunks, heavy keys collapsing in the dedupe table included."""
    from deequ_amd import _native as N
    rng = np.random.default_rng(21)
    n = 300_001
    v = np.concatenate([rng.integers(-10 ** 15, 10 ** 15, n - n // 3),
                        rng.integers(0, 40, n // 3) * 10 ** 13]).astype(np.int64)
    rng.shuffle(v)
    mask = rng.random(n) < 0.05
    d = (v % 1000).astype(np.float64) / 8
    if cap:
        monkeypatch.setenv("DQ_FREQ_XPIECE_CAP", cap)
    monkeypatch.setenv("DQ_FREQ_DENSE", "0")
    for arr, t in ((pa.array(v, mask=mask, type=pa.int64()), N.INT64),
                   (pa.array(d, mask=mask, type=pa.float64()), N.FLOAT64)):
        ft = _run(arr, t, gpu_device, 70_000, null_as_group)
        got, s = _groups(ft), ft.summarize()
        monkeypatch.setenv("DQ_FREQ_XFIXED", "0")
        ft0 = _run(arr, t, gpu_device, 70_000, null_as_group)
        monkeypatch.delenv("DQ_FREQ_XFIXED")
        assert got == _groups(ft0)
        s0 = ft0.summarize()
        assert (s.n_groups, s.n_unique, s.entropy) == (s0.n_groups, s0.n_unique, s0.entropy)
    exp = _expected(v, mask)
    if null_as_group:
        exp[None] = int(mask.sum())
    assert _groups(_run(pa.array(v, mask=mask, type=pa.int64()), N.INT64, gpu_device, 70_000,
                        null_as_group)) == exp
