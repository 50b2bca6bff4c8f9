"""ApproxQuantile (ApproxQuantile.scala:41-104) over the engine's device sort.

The reference aggregates with Spark's ApproximatePercentile, whose state is a Greenwald-Khanna
QuantileSummaries (relativeError, default 0.01).  Its arithmetic is restated here as host code
over SMALL arrays -- insert of one sorted head buffer, compress, merge, query (Spark 2.2
QuantileSummaries) -- while the values come from the device (dq_sorted_sample, quantile.hip):

  * a partition with at most HEAD_SIZE non-NULL values (Spark's head buffer, so one insert before
    the compress at query time) hands over every sorted value and the summary is the one Spark
    builds, so the quantile is Spark's to the bit;
  * a larger one hands over values at 2/eps + 1 evenly spaced exact ranks: a GK summary with
    g <= eps*n, delta = 0, so its answers are within eps*n ranks as the contract requires (Spark's
    own samples there depend on the row order of its 50000-row head buffers).

States merge with Spark's QuantileSummaries.merge (FrequenciesAndNumRows-like partition merges,
StateAggregationTests).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from .. import _native as N
from ..exceptions import IllegalAnalyzerParameterException
from .base import Analyzer, Preconditions, State, empty_state_exception
from ..metrics import DoubleMetric
from .base import entity_from, metric_from_empty, metric_from_failure, metric_from_value

HEAD_SIZE = 50000  # QuantileSummaries.defaultHeadSize

Sample = Tuple[float, int, int]  # (value, g, delta)


def _compress_immut(samples: List[Sample], merge_threshold: float) -> List[Sample]:
    """QuantileSummaries.compressImmut: merge from the right, keep the last and the minimum."""
    if not samples:
        return []
    res: List[Sample] = []
    head = samples[-1]
    i = len(samples) - 2
    while i >= 1:
        s1 = samples[i]
        if s1[1] + head[1] + head[2] < merge_threshold:
            head = (head[0], head[1] + s1[1], head[2])
        else:
            res.append(head)
            head = s1
        i -= 1
    res.append(head)
    res.reverse()
    first = samples[0]
    if first[0] <= head[0] and len(samples) > 1:
        res.insert(0, first)
    return res


@dataclass
class QuantileSummaries:
    relative_error: float
    sampled: List[Sample] = field(default_factory=list)
    count: int = 0

    @staticmethod
    def from_sorted(values: np.ndarray, relative_error: float) -> "QuantileSummaries":
        """An empty summary after inserting one sorted head buffer (withHeadBufferInserted), then
        compressed (what getPercentiles / serialize do first)."""
        n = len(values)
        out: List[Sample] = []
        for k in range(n):
            cur = k + 1
            delta = 0 if (k == 0 or k == n - 1) else int(math.floor(2 * relative_error * cur))
            out.append((float(values[k]), 1, delta))
        s = QuantileSummaries(relative_error, out, n)
        return s.compress()

    @staticmethod
    def from_ranks(values: np.ndarray, count: int, relative_error: float) -> "QuantileSummaries":
        """values[j] = the sorted value at rank floor(j (count-1) / (m-1)): a GK summary with
        g = the rank gap, delta = 0."""
        m = len(values)
        ranks = [(j * (count - 1)) // (m - 1) for j in range(m)]  # (exact: Python integers)
        gaps = [1] + [ranks[j] - ranks[j - 1] for j in range(1, m)]
        out: List[Sample] = list(zip(np.asarray(values, np.float64)[:m].tolist(), gaps, [0] * m))
        return QuantileSummaries(relative_error, out, count).compress()

    def compress(self) -> "QuantileSummaries":
        return QuantileSummaries(self.relative_error,
                                 _compress_immut(self.sampled, 2 * self.relative_error * self.count),
                                 self.count)

    def merge(self, other: "QuantileSummaries") -> "QuantileSummaries":
        if other.count == 0:
            return QuantileSummaries(self.relative_error, list(self.sampled), self.count)
        if self.count == 0:
            return QuantileSummaries(other.relative_error, list(other.sampled), other.count)
        res = sorted(self.sampled + other.sampled, key=lambda s: s[0])
        comp = _compress_immut(res, 2 * self.relative_error * self.count)
        return QuantileSummaries(other.relative_error, comp, other.count + self.count)

    def query(self, quantile: float) -> float:
        s = self.sampled
        if quantile <= self.relative_error:
            return s[0][0]
        if quantile >= 1 - self.relative_error:
            return s[-1][0]
        rank = math.ceil(quantile * self.count)
        target_error = math.ceil(self.relative_error * self.count)
        min_rank = 0
        i = 1
        while i < len(s) - 1:
            v, g, delta = s[i]
            min_rank += g
            max_rank = min_rank + delta
            if max_rank - target_error <= rank <= min_rank + target_error:
                return v
            i += 1
        return s[-1][0]


@dataclass
class ApproxQuantileState(State):
    summaries: QuantileSummaries

    def sum(self, other: "ApproxQuantileState") -> "ApproxQuantileState":
        return ApproxQuantileState(self.summaries.merge(other.summaries))


def quantile_summaries(data, column: str, relative_error: float) -> QuantileSummaries:
    """The summary of `column`'s non-NULL values over every batch of a device table.

    The device returns every sorted value when they fit Spark's head buffer, when relativeError is
    0 (accuracy 1/0.0 = Infinity: Spark keeps every sample and answers the exact order statistic,
    ApproxQuantile.scala:39-41) or when 2/eps + 1 ranks would cover every value; otherwise only the
    2/eps + 1 evenly spaced exact order statistics the summary keeps (so no more than those cross
    the link or pass through host code)."""
    import torch
    batches = [b[column] for b in data.batches]
    arr = (N.dq_column * max(1, len(batches)))(*[c.to_c() for c in batches])
    total = sum(int(arr[i].length) for i in range(len(batches)))
    device = data.device_index()
    ranks = int(math.ceil(2.0 / relative_error)) + 1 if relative_error > 0 else None
    head = total if ranks is None else max(HEAD_SIZE, ranks)
    picks = 2 if ranks is None else ranks
    out = np.empty(max(2, min(max(head, picks), total)), np.float64)
    n_out, count = ctypes.c_int64(), ctypes.c_int64()
    stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    N.retry_on_oom(lambda: N.check(N.lib.dq_sorted_sample(
        device, arr, len(batches), head, picks, out.ctypes.data, ctypes.byref(n_out),
        ctypes.byref(count), stream)))
    n, cnt = int(n_out.value), int(count.value)
    if cnt == 0:
        return QuantileSummaries(relative_error, [], 0)
    if n == cnt:
        if cnt <= HEAD_SIZE:  # one head buffer: Spark's own insert + compress, replayed
            return QuantileSummaries.from_sorted(out[:n], relative_error)
        # every value as a sample of g = 1, delta = 0: the exact summary (Spark's at eps = 0)
        s = QuantileSummaries(relative_error, list(zip(out[:n].tolist(), [1] * n, [0] * n)), cnt)
        return s.compress() if relative_error > 0 else s
    # 2/eps + 1 order statistics at the exact ranks floor(j (cnt - 1) / (n - 1)): rank gaps
    # <= eps * cnt / 2
    return QuantileSummaries.from_ranks(out[:n], cnt, relative_error)


@dataclass(frozen=True)
class ApproxQuantile(Analyzer):
    """ApproxQuantile.scala:41-104 -- its own device pass (a sort), not part of the fused scan."""
    column: str
    quantile: float
    relative_error: float = 0.01

    def __str__(self):
        return f"ApproxQuantile({self.column},{_scala_double(self.quantile)},{_scala_double(self.relative_error)})"

    def _param_check(self, _schema):
        if self.quantile < 0.0 or self.quantile > 1.0:
            raise IllegalAnalyzerParameterException(
                "Quantile parameter must be in the closed interval [0, 1]. "
                f"Currently, the value is: {_scala_double(self.quantile)}!")
        if self.relative_error < 0.0 or self.relative_error > 1.0:
            raise IllegalAnalyzerParameterException(
                "Relative error parameter must be in the closed interval [0, 1]. "
                f"Currently, the value is: {_scala_double(self.relative_error)}!")

    def preconditions(self):
        return [self._param_check, Preconditions.has_column(self.column),
                Preconditions.is_numeric(self.column)]

    def compute_state_from(self, data):
        from ..distributed import is_distributed
        s = quantile_summaries(data, self.column, self.relative_error)
        if is_distributed(data):  # every rank's summary (arrays, one device gather), rank order
            from ..distributed import all_gather_varbytes
            m = len(s.sampled)
            v = np.array([x[0] for x in s.sampled], np.float64)
            gd = np.array([[x[1], x[2]] for x in s.sampled], np.int64).reshape(m, 2)
            blob = np.array([s.count, m], np.int64).tobytes() + v.tobytes() + gd.tobytes()
            parts = all_gather_varbytes(blob, f"cuda:{data.device_index()}")
            s = QuantileSummaries(self.relative_error, [], 0)
            for b in parts:
                cnt, m = (int(x) for x in np.frombuffer(b, np.int64, 2))
                v = np.frombuffer(b, np.float64, m, 16)
                gd = np.frombuffer(b, np.int64, 2 * m, 16 + 8 * m).reshape(m, 2)
                sampled = [(float(v[i]), int(gd[i, 0]), int(gd[i, 1])) for i in range(m)]
                s = s.merge(QuantileSummaries(self.relative_error, sampled, cnt))
        return ApproxQuantileState(s) if s.count else None

    def compute_metric_from(self, state):
        if state is None:
            return metric_from_empty(self, "ApproxQuantile", self.column, entity_from([self.column]))
        return metric_from_value(state.summaries.query(self.quantile), "ApproxQuantile",
                                 self.column, entity_from([self.column]))

    def to_failure_metric(self, exception):
        return metric_from_failure(exception, "ApproxQuantile", self.column,
                                   entity_from([self.column]))


@dataclass(frozen=True)
class ApproxQuantiles(Analyzer):
    """ApproxQuantiles.scala:39-101: several quantiles of one column from one summary, as a
    KeyedDoubleMetric keyed by the quantile's Scala toString.  Unlike ApproxQuantile an all-NULL
    column is not an empty state: getPercentiles of an empty digest is empty, so the metric is
    a Success of an empty map."""
    column: str
    quantiles: Tuple[float, ...]
    relative_error: float = 0.01

    def __init__(self, column, quantiles, relative_error: float = 0.01):
        object.__setattr__(self, "column", column)
        object.__setattr__(self, "quantiles", tuple(float(q) for q in quantiles))
        object.__setattr__(self, "relative_error", relative_error)

    def __str__(self):
        qs = ", ".join(_scala_double(q) for q in self.quantiles)
        return f"ApproxQuantiles({self.column},List({qs}),{_scala_double(self.relative_error)})"

    def _param_check(self, _schema):
        for q in self.quantiles:
            ApproxQuantile(self.column, q, self.relative_error)._param_check(_schema)
        ApproxQuantile(self.column, 0.5, self.relative_error)._param_check(_schema)

    def preconditions(self):
        return [self._param_check, Preconditions.has_column(self.column),
                Preconditions.is_numeric(self.column)]

    def compute_state_from(self, data):
        s = ApproxQuantile(self.column, 0.5, self.relative_error).compute_state_from(data)
        return s if s is not None else ApproxQuantileState(
            QuantileSummaries(self.relative_error, [], 0))

    def compute_metric_from(self, state):
        from ..metrics import Entity, KeyedDoubleMetric, Success
        if state is None:
            return self.to_failure_metric(empty_state_exception(self))
        s = state.summaries
        vals = {} if s.count == 0 else {_scala_double(q): s.query(q) for q in self.quantiles}
        return KeyedDoubleMetric(Entity.Column, "ApproxQuantiles", self.column, Success(vals))

    def to_failure_metric(self, exception):
        from ..exceptions import wrap_if_necessary
        from ..metrics import Entity, Failure, KeyedDoubleMetric
        return KeyedDoubleMetric(Entity.Column, "ApproxQuantiles", self.column,
                                 Failure(wrap_if_necessary(exception)))


def _scala_double(x: float) -> str:
    from .grouping import java_double_to_string
    return java_double_to_string(float(x))


__all__ = ["ApproxQuantile", "ApproxQuantiles", "ApproxQuantileState", "QuantileSummaries", "quantile_summaries"]
