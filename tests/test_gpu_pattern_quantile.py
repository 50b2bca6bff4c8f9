"""GPU parity of PatternMatch (the device automaton, expr.hip XI_REGEX) and ApproxQuantile (device
sort + Spark's summary) against the ORACLE and the reference's known answers
(AnalyzerTests.scala:595-688, AnalysisTest.scala:79-80)."""
import math
import random

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


def _df(cols, device, batch=None):
    from deequ_amd.table import Table
    return Table.from_arrow(pa.table(cols), device=device, max_batch_rows=batch)


def test_pattern_match_known_answers(gpu_device):
    from deequ_amd.analyzers import PatternMatch, Patterns
    from test_regex import KNOWN
    for pattern, rows, expected in KNOWN:
        df = _df({"some": pa.array(rows, pa.string())}, gpu_device)
        m = PatternMatch("some", pattern).calculate(df)
        assert m.value.get() == expected / len(rows), pattern


def test_pattern_match_integral_and_null_rows(gpu_device):
    """An integral column is matched as Spark's cast to string; NULL rows count in the
    denominator only (AnalyzerTests.scala:597-601 uses a double column: Java's Double.toString is
    not on the device, so such a column is a failure metric, never a different number)."""
    from deequ_amd.analyzers import PatternMatch
    df = _df({"i": pa.array([11, None, -32, 4], pa.int64()),
              "d": pa.array([1.1, None, 3.2, 4.4], pa.float64())}, gpu_device)
    assert PatternMatch("i", r"\d\d").calculate(df).value.get() == 0.5
    assert PatternMatch("i", r"^-").calculate(df).value.get() == 0.25
    assert PatternMatch("d", r"\d\.\d").calculate(df).value.is_failure


@pytest.mark.parametrize("pattern", [r"(https?|ftp)://[^\s/$.?#].[^\s]*", r"\d{3}-\d{2}",
                                     r"[aeiou]{2}(?!x)", r"\bab", r"z+$"])
def test_pattern_match_matches_oracle_on_random_rows(pattern, gpu_device):
    from deequ_amd.analyzers import PatternMatch
    from oracle.deequ_oracle import OTable, agg_pattern_match
    rng = random.Random(len(pattern))
    alphabet = "aeioxbz0123456789-: /.htpsfé例"
    if r"\b" in pattern:  # non-ASCII next to \b: regex.py's documented approximation
        alphabet = "aeioxbz0123456789-: /.htpsf"
    n = 30_011
    vals = [None if rng.random() < 0.05 else
            "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 24))) for _ in range(n)]
    k = [rng.randint(0, 9) for _ in range(n)]
    df = _df({"s": pa.array(vals, pa.string()), "k": pa.array(k, pa.int64())}, gpu_device, 7000)
    ot = OTable({"s": vals, "k": k}, {"s": "string", "k": "long"})
    for where in (None, "k > 3"):
        st = PatternMatch("s", pattern, where).compute_state_from(df)
        hits, cnt = agg_pattern_match(ot, "s", pattern, where)
        assert (st.num_matches, st.count) == (hits, cnt), (pattern, where)


def test_approx_quantile_known_answers(gpu_device):
    from deequ_amd.analyzers import ApproxQuantile
    df = _df({"att1": pa.array([1, 2, 3, 4, 5, 6], pa.int64()),
              "numViews": pa.array([0, 0, 5, 10, 12, None], pa.int64())}, gpu_device)
    assert ApproxQuantile("att1", 0.5).calculate(df).value.get() == 3.0
    assert ApproxQuantile("numViews", 0.5).calculate(df).value.get() == 5.0


@pytest.mark.parametrize("n,batch", [(7, None), (4999, 1000), (50000, 16384)])
@pytest.mark.parametrize("dtype", ["int32", "float64"])
def test_approx_quantile_matches_spark_replay(n, batch, dtype, gpu_device):
    from deequ_amd.analyzers import ApproxQuantile
    from oracle.deequ_oracle import spark_approx_quantile
    rng = np.random.default_rng(n)
    if dtype == "int32":
        vals = rng.integers(-1000, 1000, n).astype(np.int32)
    else:
        vals = rng.normal(0, 10, n)
        vals[::53] = -0.0
        vals[1::97] = np.nan
    mask = rng.random(n) < 0.1
    df = _df({"x": pa.array(vals, mask=mask)}, gpu_device, batch)
    py = [None if m else float(v) for v, m in zip(vals, mask)]
    for q in (0.0, 0.1, 0.5, 0.9, 1.0):
        got = ApproxQuantile("x", q).calculate(df).value.get()
        exp = spark_approx_quantile(py, q)
        assert (math.isnan(got) and math.isnan(exp)) or got == exp, (n, dtype, q, got, exp)


def test_approx_quantile_large_is_within_eps(gpu_device):
    from deequ_amd.analyzers import ApproxQuantile
    from oracle.deequ_oracle import quantile_rank_error
    n = 1_000_003
    vals = np.random.default_rng(3).lognormal(0, 1, n)
    df = _df({"x": pa.array(vals)}, gpu_device, 1 << 18)
    for q in (0.05, 0.5, 0.95):
        got = ApproxQuantile("x", q).calculate(df).value.get()
        assert quantile_rank_error(vals, q, got) <= 0.01 * n


def test_approx_quantile_of_all_null_column_is_empty(gpu_device):
    from deequ_amd.analyzers import ApproxQuantile
    df = _df({"x": pa.array([None, None], pa.float64())}, gpu_device)
    assert ApproxQuantile("x", 0.5).calculate(df).value.is_failure


def test_approx_quantiles_keyed_metric(gpu_device):
    """ApproxQuantiles.scala:76-88: one summary, one entry per quantile keyed by its toString;
    an all-NULL column gives an empty map (not a failure)."""
    from deequ_amd.analyzers import ApproxQuantiles
    df = _df({"att1": pa.array([1, 2, 3, 4, 5, 6], pa.int64()),
              "n": pa.array([None] * 6, pa.float64())}, gpu_device)
    m = ApproxQuantiles("att1", [0.5, 0.25, 1.0]).calculate(df)
    assert m.value.get() == {"0.5": 3.0, "0.25": 2.0, "1.0": 6.0}
    assert [x.name for x in m.flatten()] == ["ApproxQuantiles-0.5", "ApproxQuantiles-0.25",
                                             "ApproxQuantiles-1.0"]
    assert ApproxQuantiles("n", [0.5]).calculate(df).value.get() == {}
