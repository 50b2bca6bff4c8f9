"""Partition-state parity (the reference's StateAggregationTests.scala:30-48 and
IncrementalAnalyzerTest patterns) on the GPU: random row partitions of a seeded table -- null
masks and split points drawn by hypothesis -- each scanned / grouped into its own state, merged
with State.sum (dq_state_merge semantics for scans, dq_freq_merge for FrequenciesAndNumRows.sum),
must give the metric of the whole table.  Bar: counts, HLL, groupings exact; fp64 1e-12 relative.
Also: save_states_with per partition + AnalysisRunner.run_on_aggregated_states == one run."""
import math

import numpy as np
import pyarrow as pa
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu

REL = 1e-12
N_ROWS = 3000


def _close(a, b):
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b or abs(a - b) <= REL * max(abs(a), abs(b))


def _table(seed, null_rates):
    rng = np.random.default_rng(seed)
    n = N_ROWS
    att = np.array(["extended", "Intimate Organics", "consumer_electronics", "pc", "toy", ""])

    def mask(r):
        return rng.random(n) < r
    return pa.table({
        "item": pa.array([f"B00{v:07d}" for v in rng.integers(0, 800, n)], mask=mask(null_rates[0]),
                         type=pa.string()),
        "value": pa.array(att[rng.integers(0, len(att), n)], mask=mask(null_rates[1]),
                          type=pa.string()),
        "numbersA": pa.array(rng.random(n), mask=mask(null_rates[2]), type=pa.float64()),
        "numbersB": pa.array(rng.random(n), mask=mask(null_rates[3]), type=pa.float64()),
        "count": pa.array(rng.integers(-5, 40, n), mask=mask(null_rates[4]), type=pa.int64()),
    })


def _analyzers():
    from deequ_amd.analyzers import (ApproxCountDistinct, Completeness, Compliance, CountDistinct,
                                     Correlation, Distinctness, Entropy, Histogram, Maximum, Mean,
                                     Minimum, Size, StandardDeviation, Sum, Uniqueness,
                                     UniqueValueRatio)
    return [Size(), Size("count > 3"), Completeness("item"), Completeness("value", "count > 0"),
            Compliance("a", "numbersA > 0.5"), Compliance("v", "value IN ('pc','toy')", "count < 30"),
            Sum("count"), Sum("numbersA"), Mean("numbersB"), Minimum("count"), Maximum("numbersA"),
            StandardDeviation("numbersA"), StandardDeviation("count", "count > 0"),
            Correlation("numbersA", "numbersB"), ApproxCountDistinct("item"),
            ApproxCountDistinct("count"), Uniqueness(["item"]), Distinctness(["value"]),
            Entropy("value"), UniqueValueRatio(["item", "value"]), CountDistinct(["count"]),
            Uniqueness(["count", "value"]), Histogram("value"), Histogram("count")]


def _value(m):
    v = m.value
    if not v.is_success:
        return ("failure", type(v.exception).__name__)
    x = v.get()
    if hasattr(x, "number_of_bins"):
        return (x.number_of_bins, {k: d.absolute for k, d in x.values.items()})
    return x


def _same(a, b):
    if isinstance(a, tuple) and isinstance(b, tuple):
        if a and a[0] == "failure":
            return a == b
        return a[0] == b[0] and a[1] == b[1]
    return _close(a, b)


@settings(max_examples=6, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(seed=st.integers(0, 2 ** 16),
       null_rates=st.tuples(*[st.sampled_from([0.0, 0.1, 0.5, 1.0])] * 5),
       cuts=st.lists(st.integers(0, N_ROWS), min_size=1, max_size=3))
def test_partition_states_merge_to_the_whole_table(seed, null_rates, cuts, gpu_device):
    from deequ_amd.analyzers.base import merge_states
    from deequ_amd.table import Table
    t = _table(seed, null_rates)
    bounds = sorted(set([0, N_ROWS] + cuts))
    parts = [Table.from_arrow(t.slice(lo, hi - lo), device=gpu_device, max_batch_rows=1000)
             for lo, hi in zip(bounds[:-1], bounds[1:])]
    whole = Table.from_arrow(t, device=gpu_device, max_batch_rows=1000)
    for a in _analyzers():
        states, error = [], None
        for p in parts:
            try:
                states.append(a.compute_state_from(p))
            except Exception as e:  # noqa: BLE001 -- the reference fails the analyzer
                error = e
                break
        if error is not None:  # a throwing partition is a failure metric, never a dropped state
            merged = a.to_failure_metric(error)
            assert not a.calculate(whole).value.is_success, (str(a), bounds, repr(error))
            assert not merged.value.is_success
            continue
        try:  # Analyzer.calculate's try (Analyzer.scala:88-103) around computeMetricFrom
            merged = a.compute_metric_from(merge_states(*states))
        except Exception as e:  # noqa: BLE001
            merged = a.to_failure_metric(e)
        if any(x is None for x in states) and any(x is not None for x in states):
            # the reference drops a partition whose state is None -- its aggregation came back
            # NULL: every value NULL or filtered (ifNoNullsIn: Mean.scala:45-50, Compliance's
            # sum of a NULL predicate, Sum, Min/Max, ...) -- together with its count(*) rows
            # (Analyzers.merge, Analyzer.scala:343-362), so the merged metric is NOT the whole
            # table's: it is the metric of the partitions that kept a state, run as one table.
            keep = [(lo, hi) for (lo, hi), x in zip(zip(bounds[:-1], bounds[1:]), states)
                    if x is not None]
            kept = pa.concat_tables([t.slice(lo, hi - lo) for lo, hi in keep])
            direct = a.calculate(Table.from_arrow(kept, device=gpu_device, max_batch_rows=1000))
        else:
            direct = a.calculate(whole)
        assert _same(_value(merged), _value(direct)), (str(a), bounds, _value(merged),
                                                       _value(direct))


def test_saved_partition_states_run_on_aggregated_states(gpu_device):
    """IncrementalAnalyzerTest / AnalysisRunner.runOnAggregatedStates (AnalysisRunner.scala:375-446):
    each partition's run persists its states; the metrics computed from the aggregated states alone
    equal one run over the whole table."""
    from deequ_amd.analyzers import InMemoryStateProvider
    from deequ_amd.runners import Analysis, AnalysisRunner
    from deequ_amd.table import Table
    t = _table(17, (0.1, 0.1, 0.0, 0.1, 0.05))
    analysis = Analysis(_analyzers())
    providers = []
    for lo, hi in [(0, 1000), (1000, 2500), (2500, N_ROWS)]:
        prov = InMemoryStateProvider()
        AnalysisRunner.run(Table.from_arrow(t.slice(lo, hi - lo), device=gpu_device), analysis,
                           save_states_with=prov)
        providers.append(prov)
    whole = Table.from_arrow(t, device=gpu_device)
    agg = AnalysisRunner.run_on_aggregated_states(whole.schema, analysis, providers)
    direct = AnalysisRunner.run(whole, analysis)
    for a in analysis.analyzers:
        assert _same(_value(agg.metric(a)), _value(direct.metric(a))), str(a)


def test_states_persisted_to_disk_run_on_aggregated_states(gpu_device, tmp_path):
    """The same with HdfsStateProvider (StateProvider.scala:71-294, StateProviderTest.scala
    "restore their state from the filesystem"): every partition's states go through the
    reference's on-disk layouts -- big-endian .bin files, frequency tables as Parquet (Histogram's
    cast to string) -- and load back into metrics equal to one run over the whole table."""
    from deequ_amd.analyzers import HdfsStateProvider
    from deequ_amd.runners import Analysis, AnalysisRunner
    from deequ_amd.table import Table
    from deequ_amd.analyzers import Histogram
    t = _table(23, (0.1, 0.2, 0.0, 0.1, 0.05))
    # Histogram("count") is left out: its frequency DataFrame would hold two "count" columns,
    # which Spark's Parquet writer refuses (asserted below)
    analysis = Analysis([a for a in _analyzers() if a != Histogram("count")])
    providers = []
    for i, (lo, hi) in enumerate([(0, 1200), (1200, N_ROWS)]):
        prov = HdfsStateProvider(str(tmp_path / f"part{i}"))
        AnalysisRunner.run(Table.from_arrow(t.slice(lo, hi - lo), device=gpu_device), analysis,
                           save_states_with=prov)
        providers.append(prov)
    whole = Table.from_arrow(t, device=gpu_device)
    agg = AnalysisRunner.run_on_aggregated_states(whole.schema, analysis, providers)
    direct = AnalysisRunner.run(whole, analysis)
    for a in analysis.analyzers:
        assert _same(_value(agg.metric(a)), _value(direct.metric(a))), str(a)
    h = Histogram("count")
    with pytest.raises(ValueError):
        HdfsStateProvider(str(tmp_path / "dup")).persist(h, h.compute_state_from(whole))


def test_frequency_states_round_trip_through_parquet(gpu_device, tmp_path):
    """persist -> load of FrequenciesAndNumRows / Histogram states: the loaded table holds the same
    groups and numRows (assertCorrectlyRestoresFrequencyBasedState, StateProviderTest.scala)."""
    from deequ_amd.analyzers import Entropy, HdfsStateProvider, Histogram, Uniqueness
    from deequ_amd.table import Table
    t = _table(29, (0.1, 0.2, 0.0, 0.0, 0.1))
    data = Table.from_arrow(t, device=gpu_device)
    prov = HdfsStateProvider(str(tmp_path / "st"))
    for a in [Uniqueness(["item"]), Uniqueness(["item", "count"]), Entropy("value"),
              Histogram("value"), Histogram("item")]:
        st = a.compute_state_from(data)
        prov.persist(a, st)
        back = prov.load(a)
        assert back.num_rows == st.num_rows, str(a)
        if isinstance(a, Histogram):
            assert back.string_groups() == st.string_groups(), str(a)
            assert _same(_value(a.compute_metric_from(back)), _value(a.compute_metric_from(st)))
        else:
            assert dict(back.frequencies.export()) == dict(st.frequencies.export()), str(a)
            assert _same(_value(a.compute_metric_from(back)), _value(a.compute_metric_from(st)))
