"""One-utf8-column group-bys into fixed-capacity bucket pieces (freq.hip freq_phaseA<STR1> with
AArgs::pstart): each workgroup's records of a bucket fill a piece of 1.5x the mean, and a tile's
records past a full piece stay in the tile's chunk.  Bar: the same groups and counts as the
chunk-only layout (DQ_FREQ_HPIECES=0) and as the oracle (GroupingAnalyzers.scala:53-80), with
the default capacity and with tiny ones that send most records to the chunks, for the grouping,
Histogram mode (NULL group kept apart) and a multi-batch table; the frequency-family metrics and
Histogram top-k through the runner."""
from collections import Counter

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


def _strings(n, seed):
    rng = np.random.default_rng(seed)
    # long keys (no small-key attempt): a heavy head, a mid tail and near-unique rows
    ids = np.concatenate([rng.integers(0, 20, n // 4), rng.integers(0, n // 10, n // 4),
                          rng.integers(0, 10 ** 9, n - 2 * (n // 4))])
    rng.shuffle(ids)
    mask = rng.random(n) < 0.04
    vals = [None if m else f"key-{v:012d}" + ("x" * int(v % 7)) for v, m in zip(ids, mask)]
    return pa.array(vals, pa.string()), vals


def _table(arr, device, batch, null_as_group):
    from deequ_amd import _native as N
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    df = Table.from_arrow(pa.table({"k": arr}), device=device, max_batch_rows=batch)
    ft = FrequencyTable(["k"], [N.UTF8], 0)
    for b in df.batches:
        ft.add([b["k"]], null_as_group=null_as_group)
    return {k[0]: c for k, c in ft.export()}, ft.summarize()


@pytest.mark.parametrize("null_as_group", [False, True])
@pytest.mark.parametrize("cap", [None, "1", "7"])
def test_pieces_equal_chunks_and_oracle(cap, null_as_group, gpu_device, monkeypatch):
    arr, vals = _strings(120_001, 4)
    exp = Counter(v for v in vals if v is not None)
    if null_as_group:
        exp[None] = sum(v is None for v in vals)
    if cap:
        monkeypatch.setenv("DQ_FREQ_HPIECE_CAP", cap)
    got, s = _table(arr, gpu_device, 50_000, null_as_group)
    assert got == exp
    monkeypatch.setenv("DQ_FREQ_HPIECES", "0")
    ref, s0 = _table(arr, gpu_device, 50_000, null_as_group)
    assert ref == exp
    assert (s.n_groups, s.n_unique, s.entropy) == (s0.n_groups, s0.n_unique, s0.entropy)


def test_runner_metrics_with_pieces(gpu_device, monkeypatch):
    from deequ_amd.analyzers import (CountDistinct, Distinctness, Entropy, Histogram,
                                     UniqueValueRatio, Uniqueness)
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    arr, _ = _strings(90_001, 6)
    df = Table.from_arrow(pa.table({"k": arr}), device=gpu_device, max_batch_rows=40_000)
    suite = [Uniqueness(["k"]), Distinctness(["k"]), UniqueValueRatio(["k"]),
             CountDistinct(["k"]), Entropy("k"), Histogram("k")]
    monkeypatch.setenv("DQ_FREQ_HPIECE_CAP", "5")
    got = AnalysisRunner.do_analysis_run(df, suite)
    monkeypatch.delenv("DQ_FREQ_HPIECE_CAP")
    monkeypatch.setenv("DQ_FREQ_HPIECES", "0")
    ref = AnalysisRunner.do_analysis_run(df, suite)
    for a in suite[:-1]:
        assert got.metric(a).value.get() == ref.metric(a).value.get(), str(a)
    h1, h2 = got.metric(suite[-1]).value.get(), ref.metric(suite[-1]).value.get()
    assert h1.number_of_bins == h2.number_of_bins
    assert sorted(x.absolute for x in h1.values.values()) == \
        sorted(x.absolute for x in h2.values.values())
