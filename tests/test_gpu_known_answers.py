"""The reference's known-answer tests, run through the HIP engine (deequ_amd -> C ABI -> GPU)."""
import json
import math
import os

import pytest

from tests.fixtures import arrow_table
from tests.oracle_runner import matches

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                     "reference_known_answers.json")))


def table(name):
    from deequ_amd import Table
    return Table.from_arrow(arrow_table(name), device="cuda:0")


def build(cls, args, kwargs):
    import deequ_amd.analyzers as A
    return getattr(A, cls)(*args, **kwargs)


def value_of(metric):
    from deequ_amd.exceptions import EmptyStateException
    if metric.value.is_success:
        return metric.value.get()
    return "EMPTY" if isinstance(metric.value.failed, EmptyStateException) else "FAILURE"


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=lambda c: c["cite"])
def test_known_answer_on_gpu(case, gpu_device):
    cls, args, kwargs = case["analyzer"]
    metric = build(cls, args, kwargs).calculate(table(case["fixture"]))
    got = value_of(metric)
    exp = case["expected"]
    if exp == "FAILURE":
        assert got in ("FAILURE", "EMPTY") and metric.value.is_failure
    else:
        assert matches(got, exp, rel=1e-12), (got, exp)


@pytest.mark.parametrize("case", GOLDEN["histograms"], ids=lambda c: c["cite"])
def test_histogram_on_gpu(case, gpu_device):
    from deequ_amd.analyzers import Histogram
    m = Histogram(case["column"], max_detail_bins=case["max_detail_bins"]).calculate(
        table(case["fixture"]))
    d = m.value.get()
    assert d.number_of_bins == case["bins"]
    assert set(d.values) == set(case["keys"])


@pytest.mark.parametrize("case", GOLDEN["states"], ids=lambda c: c["cite"])
def test_states_on_gpu(case, gpu_device):
    import deequ_amd.analyzers as A
    cls, args, kwargs = case["analyzer"]
    state = build(cls, args, kwargs).compute_state_from(table(case["fixture"]))
    if case["state"] is None:
        assert state is None
    else:
        name, fields = case["state"]
        assert state == getattr(A, name)(*fields)


def test_empty_state_message(gpu_device):
    # NullHandlingTests.scala:107-118
    from deequ_amd.analyzers import Mean
    m = Mean("numericCol").calculate(table("dataWithNullColumns"))
    assert str(m.value.failed) == ("Empty state for analyzer Mean(numericCol,None), all input "
                                   "values were NULL.")


def test_analysis_runs_each_analyzer_once_and_shares_the_scan(gpu_device):
    # AnalysisTest.scala:41-52 and the scan-sharing contract of AnalysisRunnerTests.scala:34-58
    from deequ_amd import Analysis
    from deequ_amd.analyzers import (Completeness, Compliance, Maximum, Mean, Minimum, Size,
                                     StandardDeviation)
    from deequ_amd.runners import engine
    df = table("dfWithNumericValues")
    res = Analysis().add_analyzer(Size()).add_analyzer(Size()).add_analyzer(Size()).run(df)
    assert len(res.all_metrics()) == 1 and res.metric(Size()).value.get() == 6
    calls = []
    real = engine.run_scan
    engine_mod_run = lambda data, specs: calls.append(len(specs)) or real(data, specs)  # noqa
    import deequ_amd.runners as R
    R.run_scan = engine_mod_run
    try:
        ctx = Analysis([Size(), Completeness("att1"), Compliance("r", "att1 > 3"), Mean("att1"),
                        StandardDeviation("att1"), Minimum("att1"), Maximum("att1")]).run(df)
    finally:
        R.run_scan = real
    assert calls == [10]  # ONE fused scan for all seven analyzers (1+2+2+2+1+1+1 slots)
    assert ctx.metric(Mean("att1")).value.get() == 3.5


def test_failing_expression_fails_every_shareable_analyzer(gpu_device):
    # AnalysisRunner.scala:310-313
    from deequ_amd import Analysis
    from deequ_amd.analyzers import Compliance, Size
    ctx = Analysis([Size(), Compliance("r", "nosuch > 3")]).run(table("dfWithNumericValues"))
    assert ctx.metric(Size()).value.is_failure
    assert ctx.metric(Compliance("r", "nosuch > 3")).value.is_failure
