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
