"""Metrics repositories (reference: repository/MetricsRepository.scala, AnalysisResult.scala,
memory/InMemoryMetricsRepository.scala): where AnalysisRunner / VerificationSuite /
ColumnProfiler save successful metrics under a ResultKey and reuse them on later runs
(AnalysisRunner.scala:123-138, ColumnProfiler.scala:215-290)."""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Optional, Sequence


@dataclass(frozen=True)
class ResultKey:
    """ResultKey(dataSetDate: Long, tags: Map[String, String]) -- a value type (case class)."""
    data_set_date: int
    tags: Mapping[str, str] = field(default_factory=dict)

    def __hash__(self):
        return hash((self.data_set_date, tuple(sorted(self.tags.items()))))

    def __eq__(self, other):
        return (isinstance(other, ResultKey) and self.data_set_date == other.data_set_date
                and dict(self.tags) == dict(other.tags))


@dataclass
class AnalysisResult:
    result_key: ResultKey
    analyzer_context: object  # runners.AnalyzerContext


class MetricsRepository:
    def save(self, result_key: ResultKey, analyzer_context) -> None:
        raise NotImplementedError

    def load_by_key(self, result_key: ResultKey):
        raise NotImplementedError

    def load(self) -> "MetricsRepositoryMultipleResultsLoader":
        raise NotImplementedError


class MetricsRepositoryMultipleResultsLoader:
    """MetricsRepositoryMultipleResultsLoader.scala: a query over the saved results."""

    def __init__(self, results: Sequence[AnalysisResult]):
        self._results = list(results)
        self._tags: Optional[Dict[str, str]] = None
        self._analyzers: Optional[List] = None
        self._before: Optional[int] = None
        self._after: Optional[int] = None

    def with_tag_values(self, tag_values: Mapping[str, str]):
        self._tags = dict(tag_values)
        return self

    def for_analyzers(self, analyzers: Sequence):
        self._analyzers = list(analyzers)
        return self

    def before(self, date_time: int):
        self._before = date_time
        return self

    def after(self, date_time: int):
        self._after = date_time
        return self

    def get(self) -> List[AnalysisResult]:
        from .runners import AnalyzerContext
        out = []
        for r in self._results:
            k = r.result_key
            if self._after is not None and k.data_set_date < self._after:
                continue
            if self._before is not None and k.data_set_date > self._before:
                continue
            if self._tags is not None and any(k.tags.get(t) != v for t, v in self._tags.items()):
                continue
            ctx = r.analyzer_context
            if self._analyzers is not None:
                ctx = AnalyzerContext({a: m for a, m in ctx.metric_map.items()
                                       if a in self._analyzers})
            out.append(AnalysisResult(k, ctx))
        return out


class InMemoryMetricsRepository(MetricsRepository):
    """Keeps the successful metrics only (InMemoryMetricsRepository.scala:37-50)."""

    def __init__(self):
        self._results: Dict[ResultKey, AnalysisResult] = {}
        self._lock = threading.Lock()

    def save(self, result_key: ResultKey, analyzer_context) -> None:
        from .runners import AnalyzerContext
        ok = {a: m for a, m in analyzer_context.metric_map.items() if m.value.is_success}
        with self._lock:
            self._results[result_key] = AnalysisResult(result_key, AnalyzerContext(ok))

    def load_by_key(self, result_key: ResultKey):
        with self._lock:
            r = self._results.get(result_key)
        return r.analyzer_context if r is not None else None

    def load(self) -> MetricsRepositoryMultipleResultsLoader:
        with self._lock:
            return MetricsRepositoryMultipleResultsLoader(list(self._results.values()))


__all__ = ["ResultKey", "AnalysisResult", "MetricsRepository", "InMemoryMetricsRepository",
           "MetricsRepositoryMultipleResultsLoader"]


# ------------------------------------------------------------------------------------------------
# JSON (repository/AnalysisResultSerde.scala:56-614): the format FileSystemMetricsRepository
# writes, so a repository file is shared with JVM deequ.
# ------------------------------------------------------------------------------------------------
def _scala_num(x: float) -> str:
    """Scala Double.toString of a quantile list entry ("0.5", "1.0", "1.0E-4")."""
    from .analyzers.grouping import java_double_to_string
    return java_double_to_string(float(x))


def analyzer_to_json(a) -> dict:
    from . import analyzers as A
    # Gson drops null properties: no "where" key without a filter
    where = lambda: {"where": a.where} if getattr(a, "where", None) is not None else {}  # noqa: E731
    simple = {A.Completeness: "Completeness", A.Sum: "Sum", A.Mean: "Mean", A.Minimum: "Minimum",
              A.Maximum: "Maximum", A.DataType: "DataType",
              A.ApproxCountDistinct: "ApproxCountDistinct",
              A.StandardDeviation: "StandardDeviation"}
    multi = {A.CountDistinct: "CountDistinct", A.Distinctness: "Distinctness",
             A.MutualInformation: "MutualInformation", A.UniqueValueRatio: "UniqueValueRatio",
             A.Uniqueness: "Uniqueness"}
    t = type(a)
    if t is A.Size:
        return {"analyzerName": "Size", **where()}
    if t in simple:
        return {"analyzerName": simple[t], "column": a.column, **where()}
    if t is A.Compliance:
        return {"analyzerName": "Compliance", **where(), "instance": a.instance,
                "predicate": a.predicate}
    if t is A.PatternMatch:
        return {"analyzerName": "PatternMatch", "column": a.column, **where(),
                "pattern": a.pattern}
    if t in multi:
        return {"analyzerName": multi[t], "columns": list(a.columns)}
    if t is A.Entropy:
        return {"analyzerName": "Entropy", "column": a.column}
    if t is A.Histogram and a.binning_udf is None:
        return {"analyzerName": "Histogram", "column": a.column, "maxDetailBins": a.max_detail_bins}
    if t is A.Correlation:
        return {"analyzerName": "Correlation", "firstColumn": a.first_column,
                "secondColumn": a.second_column, **where()}
    if t is A.ApproxQuantile:
        return {"analyzerName": "ApproxQuantile", "column": a.column, "quantile": a.quantile,
                "relativeError": a.relative_error}
    if t is A.ApproxQuantiles:
        return {"analyzerName": "ApproxQuantiles", "column": a.column,
                "quantiles": ",".join(_scala_num(q) for q in a.quantiles),
                "relativeError": a.relative_error}
    raise ValueError(f"Unable to serialize analyzer {a}.")


def analyzer_from_json(j: dict):
    from . import analyzers as A
    n = j["analyzerName"]
    w = j.get("where")
    ctor = {"Completeness": A.Completeness, "Sum": A.Sum, "Mean": A.Mean, "Minimum": A.Minimum,
            "Maximum": A.Maximum, "DataType": A.DataType,
            "ApproxCountDistinct": A.ApproxCountDistinct,
            "StandardDeviation": A.StandardDeviation}
    multi = {"CountDistinct": A.CountDistinct, "Distinctness": A.Distinctness,
             "MutualInformation": A.MutualInformation, "UniqueValueRatio": A.UniqueValueRatio,
             "Uniqueness": A.Uniqueness}
    if n == "Size":
        return A.Size(w)
    if n in ctor:
        return ctor[n](j["column"], w)
    if n == "Compliance":
        return A.Compliance(j["instance"], j["predicate"], w)
    if n == "PatternMatch":
        return A.PatternMatch(j["column"], j["pattern"], w)
    if n in multi:
        return multi[n](list(j["columns"]))
    if n == "Entropy":
        return A.Entropy(j["column"])
    if n == "Histogram":
        return A.Histogram(j["column"], None, int(j["maxDetailBins"]))
    if n == "Correlation":
        return A.Correlation(j["firstColumn"], j["secondColumn"], w)
    if n == "ApproxQuantile":
        return A.ApproxQuantile(j["column"], float(j["quantile"]), float(j["relativeError"]))
    if n == "ApproxQuantiles":
        return A.ApproxQuantiles(j["column"], [float(q) for q in j["quantiles"].split(",")],
                                 float(j["relativeError"]))
    raise ValueError(f"Unable to deserialize analyzer {n}.")


def metric_to_json(m) -> dict:
    from .metrics import DoubleMetric, HistogramMetric, KeyedDoubleMetric
    if not m.value.is_success:
        raise ValueError("Unable to serialize failed metrics.")
    if isinstance(m, DoubleMetric):
        return {"metricName": "DoubleMetric", "entity": str(m.entity), "instance": m.instance,
                "name": m.name, "value": m.value.get()}
    if isinstance(m, HistogramMetric):
        d = m.value.get()
        return {"metricName": "HistogramMetric", "column": m.column,
                "numberOfBins": d.number_of_bins,
                "value": {"numberOfBins": d.number_of_bins,
                          "values": {k: {"absolute": v.absolute, "ratio": v.ratio}
                                     for k, v in d.values.items()}}}
    if isinstance(m, KeyedDoubleMetric):
        return {"metricName": "KeyedDoubleMetric", "entity": str(m.entity),
                "instance": m.instance, "name": m.name, "value": dict(m.value.get())}
    raise ValueError(f"Unable to serialize metrics {m}.")


def metric_from_json(j: dict):
    from .metrics import (DoubleMetric, Distribution, DistributionValue, Entity, Failure,
                          HistogramMetric, KeyedDoubleMetric, Success)
    n = j["metricName"]
    if n == "DoubleMetric":
        return DoubleMetric(Entity(j["entity"]), j["name"], j["instance"], Success(float(j["value"])))
    if n == "HistogramMetric":
        v = j["value"]
        d = Distribution({k: DistributionValue(int(x["absolute"]), float(x["ratio"]))
                          for k, x in v["values"].items()}, int(v["numberOfBins"]))
        return HistogramMetric(j["column"], Success(d))
    if n == "KeyedDoubleMetric":
        val = Success({k: float(x) for k, x in j["value"].items()}) if "value" in j \
            else Failure(ValueError("no value"))
        return KeyedDoubleMetric(Entity(j["entity"]), j["name"], j["instance"], val)
    raise ValueError(f"Unable to deserialize analyzer {n}.")


class AnalysisResultSerde:
    @staticmethod
    def serialize(results: Sequence[AnalysisResult]) -> str:
        out = []
        for r in results:
            out.append({
                "resultKey": {"dataSetDate": r.result_key.data_set_date,
                              "tags": dict(r.result_key.tags)},
                "analyzerContext": {"metricMap": [
                    {"analyzer": analyzer_to_json(a), "metric": metric_to_json(m)}
                    for a, m in r.analyzer_context.metric_map.items()]}})
        import json
        return json.dumps(out)

    @staticmethod
    def deserialize(text: str) -> List[AnalysisResult]:
        import json
        from .runners import AnalyzerContext
        out = []
        for r in json.loads(text):
            k = r["resultKey"]
            ctx = AnalyzerContext({analyzer_from_json(e["analyzer"]): metric_from_json(e["metric"])
                                   for e in r["analyzerContext"]["metricMap"]})
            out.append(AnalysisResult(ResultKey(int(k["dataSetDate"]), dict(k.get("tags") or {})),
                                      ctx))
        return out


def success_metrics_as_json(result: AnalysisResult, for_analyzers: Sequence = (),
                            with_tags: Sequence[str] = ()) -> str:
    """AnalysisResult.getSuccessMetricsAsJson (AnalysisResult.scala:70-92): the success rows of
    the context plus dataset_date and one lower-cased column per tag."""
    import json
    from .runners import AnalyzerContext
    rows = AnalyzerContext.success_metrics_as_rows(result.analyzer_context, for_analyzers)
    for r in rows:
        r["dataset_date"] = result.result_key.data_set_date
    for tag, value in result.result_key.tags.items():
        if with_tags and tag not in with_tags:
            continue
        name = tag.lower().replace(" ", "_")  # formatTagColumnNameInJson
        if rows and name in rows[0]:
            name = f"tag_{name}"
        for r in rows:
            r[name] = value
    return json.dumps(rows)


class FileSystemMetricsRepository(MetricsRepository):
    """fs/FileSystemMetricsRepository.scala: every result in one JSON file (a local path), read
    and rewritten whole on each save."""

    def __init__(self, path: str):
        self.path = path
        self._lock = threading.Lock()

    def _all(self) -> List[AnalysisResult]:
        import os
        if not os.path.exists(self.path):
            return []
        with open(self.path, encoding="utf-8") as fh:
            text = fh.read()
        return AnalysisResultSerde.deserialize(text) if text.strip() else []

    def save(self, result_key: ResultKey, analyzer_context) -> None:
        from .runners import AnalyzerContext
        ok = AnalyzerContext({a: m for a, m in analyzer_context.metric_map.items()
                              if m.value.is_success})
        with self._lock:
            prev = [r for r in self._all() if r.result_key != result_key]
            text = AnalysisResultSerde.serialize(prev + [AnalysisResult(result_key, ok)])
            with open(self.path, "w", encoding="utf-8") as fh:
                fh.write(text)

    def load_by_key(self, result_key: ResultKey):
        with self._lock:
            for r in self._all():
                if r.result_key == result_key:
                    return r.analyzer_context
        return None

    def load(self) -> MetricsRepositoryMultipleResultsLoader:
        with self._lock:
            return MetricsRepositoryMultipleResultsLoader(self._all())


__all__ += ["AnalysisResultSerde", "FileSystemMetricsRepository", "success_metrics_as_json",
            "analyzer_to_json", "analyzer_from_json", "metric_to_json", "metric_from_json"]
