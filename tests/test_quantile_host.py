"""ApproxQuantile's summary arithmetic (deequ_amd/analyzers/quantile.py: Spark 2.2 QuantileSummaries
insert / compress / merge / query) against the ORACLE's restatement and the reference's known
answers (AnalysisTest.scala:79-80: ApproxQuantile(att1, 0.5) of 1..6 = 3.0; BasicExample.scala:
56: the median of numViews 0,0,5,10,12 = 5.0).  Host only."""
import random

import numpy as np
import pytest

from deequ_amd.analyzers.quantile import QuantileSummaries
from oracle.deequ_oracle import quantile_rank_error, spark_approx_quantile


def _summary(values, eps=0.01):
    return QuantileSummaries.from_sorted(np.sort(np.asarray(values, np.float64)), eps)


def test_reference_known_answers():
    assert _summary([1, 2, 3, 4, 5, 6]).query(0.5) == 3.0
    assert _summary([0, 0, 5, 10, 12]).query(0.5) == 5.0


@pytest.mark.parametrize("n", [1, 2, 7, 49, 50, 51, 333, 4000, 50000])
@pytest.mark.parametrize("eps", [0.01, 0.05, 0.25])
def test_replay_matches_oracle(n, eps):
    rng = random.Random(n * 7 + int(eps * 100))
    vals = [rng.randint(-50, 50) * 0.5 for _ in range(n)]
    s = _summary(vals, eps)
    for q in (0.0, 0.001, 0.1, 0.25, 0.5, 0.77, 0.99, 1.0):
        assert s.query(q) == spark_approx_quantile(vals, q, eps), (n, eps, q)


@pytest.mark.parametrize("parts", [2, 3, 7])
def test_merged_partitions_stay_within_eps(parts):
    rng = np.random.default_rng(parts)
    vals = rng.normal(0, 1, 30000)
    eps = 0.01
    cuts = np.sort(rng.choice(np.arange(1, len(vals)), parts - 1, replace=False))
    merged = QuantileSummaries(eps, [], 0)
    for chunk in np.split(vals, cuts):
        merged = merged.merge(_summary(chunk, eps))
    assert merged.count == len(vals)
    for q in (0.05, 0.25, 0.5, 0.9):
        assert quantile_rank_error(vals, q, merged.query(q)) <= eps * len(vals) + 1


def test_rank_summary_stays_within_eps():
    rng = np.random.default_rng(5)
    vals = np.sort(rng.exponential(3.0, 200001))
    eps = 0.01
    m = 201
    picks = vals[[(j * (len(vals) - 1)) // (m - 1) for j in range(m)]]
    s = QuantileSummaries.from_ranks(picks, len(vals), eps)
    for q in (0.02, 0.3, 0.5, 0.75, 0.97):
        assert quantile_rank_error(vals, q, s.query(q)) <= eps * len(vals)
