"""Metrics repositories and their JSON (repository/AnalysisResultSerde.scala, fs/, memory/):
round trips of every analyzer / metric kind, the repository queries
(MetricsRepositoryMultipleResultsLoaderTest pattern) and the success-metrics JSON rows."""
import json

from deequ_amd.analyzers import (ApproxCountDistinct, ApproxQuantile, ApproxQuantiles,
                                 Completeness, Compliance, Correlation, CountDistinct, DataType,
                                 Distinctness, Entropy, Histogram, Maximum, Mean, Minimum,
                                 MutualInformation, PatternMatch, Size, StandardDeviation, Sum,
                                 UniqueValueRatio, Uniqueness)
from deequ_amd.metrics import (Distribution, DistributionValue, DoubleMetric, Entity, Failure,
                               HistogramMetric, KeyedDoubleMetric, Success)
from deequ_amd.repository import (AnalysisResult, AnalysisResultSerde, FileSystemMetricsRepository,
                                  InMemoryMetricsRepository, ResultKey, analyzer_from_json,
                                  analyzer_to_json, success_metrics_as_json)
from deequ_amd.runners import AnalyzerContext

ANALYZERS = [Size(), Size("a > 1"), Completeness("c"), Completeness("c", "x = 'y'"),
             Compliance("rule", "att1 > 0"), PatternMatch("c", r"\d+"), Sum("n"), Mean("n"),
             Minimum("n"), Maximum("n"), CountDistinct(["a", "b"]), Distinctness(["a"]),
             Entropy("a"), MutualInformation(["a", "b"]), UniqueValueRatio(["a"]),
             Uniqueness(["a", "b"]), Histogram("a"), Histogram("a", None, 10), DataType("s"),
             ApproxCountDistinct("a"), Correlation("x", "y"), StandardDeviation("n"),
             ApproxQuantile("n", 0.5), ApproxQuantile("n", 0.25, 0.1),
             ApproxQuantiles("n", [0.1, 0.5, 1.0])]


def _ctx():
    m = {}
    for i, a in enumerate(ANALYZERS):
        if isinstance(a, Histogram):
            m[a] = HistogramMetric(a.column, Success(Distribution(
                {"x": DistributionValue(3, 0.75), "NullValue": DistributionValue(1, 0.25)}, 2)))
        elif isinstance(a, ApproxQuantiles):
            m[a] = KeyedDoubleMetric(Entity.Column, "ApproxQuantiles", "n",
                                     Success({"0.1": 1.0, "0.5": 2.5, "1.0": 9.0}))
        else:
            m[a] = DoubleMetric(Entity.Column, type(a).__name__, "c", Success(0.5 + i))
    return AnalyzerContext(m)


def test_every_analyzer_round_trips_through_json():
    for a in ANALYZERS:
        j = analyzer_to_json(a)
        assert analyzer_from_json(json.loads(json.dumps(j))) == a, str(a)
    assert "where" not in analyzer_to_json(Size())  # Gson drops null properties


def test_analysis_results_round_trip():
    results = [AnalysisResult(ResultKey(1507975810, {"Region": "EU"}), _ctx()),
               AnalysisResult(ResultKey(1, {}), AnalyzerContext.empty())]
    back = AnalysisResultSerde.deserialize(AnalysisResultSerde.serialize(results))
    assert [r.result_key for r in back] == [r.result_key for r in results]
    assert back[0].analyzer_context.metric_map == results[0].analyzer_context.metric_map


def test_repositories_keep_successes_and_answer_queries(tmp_path):
    ctx = _ctx()
    failing = AnalyzerContext({Sum("z"): DoubleMetric(Entity.Column, "Sum", "z",
                                                      Failure(ValueError("x")))})
    for repo in (InMemoryMetricsRepository(), FileSystemMetricsRepository(str(tmp_path / "m.json"))):
        k1, k2, k3 = ResultKey(10, {"r": "EU"}), ResultKey(20, {"r": "NA"}), ResultKey(30, {})
        repo.save(k1, ctx + failing)
        repo.save(k2, ctx)
        repo.save(k3, ctx)
        assert Sum("z") not in repo.load_by_key(k1).metric_map  # failures are not kept
        assert repo.load_by_key(k1).metric_map == ctx.metric_map
        assert repo.load_by_key(ResultKey(99, {})) is None
        assert [r.result_key for r in repo.load().with_tag_values({"r": "EU"}).get()] == [k1]
        assert {r.result_key for r in repo.load().after(15).get()} == {k2, k3}
        assert {r.result_key for r in repo.load().before(20).get()} == {k1, k2}
        got = repo.load().for_analyzers([Size(), Entropy("a")]).get()
        assert all(set(r.analyzer_context.metric_map) == {Size(), Entropy("a")} for r in got)
        repo.save(k1, AnalyzerContext.empty())  # same key: replaced
        assert repo.load_by_key(k1).metric_map == {}


def test_success_metrics_json_rows_carry_date_and_tags():
    ctx = AnalyzerContext({Size(): DoubleMetric(Entity.Dataset, "Size", "*", Success(4.0))})
    rows = json.loads(success_metrics_as_json(AnalysisResult(ResultKey(1507975810, {"Region": "EU"}),
                                                             ctx)))
    assert rows == [{"entity": "Dataset", "instance": "*", "name": "Size", "value": 4.0,
                     "dataset_date": 1507975810, "region": "EU"}]
