"""DataType (DataType.scala:25-183, StatefulDataType.scala:26-83): a histogram of the value
classes of a column -- NULL (reported as "Unknown"), Fractional, Integral, Boolean, String -- from
the fused scan (TK_DTYPE body, scan.hip), plus the type decision the profiler uses."""
from __future__ import annotations

from dataclasses import dataclass
from enum import Enum
from typing import Optional

from .. import _native as N
from ..exceptions import wrap_if_necessary
from ..metrics import Distribution, DistributionValue, Failure, HistogramMetric, Success
from .base import AggSpec, Preconditions, State, StandardScanShareableAnalyzer, empty_state_exception


class DataTypeInstances(Enum):
    """DataType.scala:27-33"""
    Unknown = 0
    Fractional = 1
    Integral = 2
    Boolean = 3
    String = 4


@dataclass(frozen=True)
class DataTypeHistogram(State):
    num_null: int
    num_fractional: int
    num_integral: int
    num_boolean: int
    num_string: int

    def sum(self, other: "DataTypeHistogram") -> "DataTypeHistogram":
        return DataTypeHistogram(self.num_null + other.num_null,
                                 self.num_fractional + other.num_fractional,
                                 self.num_integral + other.num_integral,
                                 self.num_boolean + other.num_boolean,
                                 self.num_string + other.num_string)

    def to_distribution(self) -> Distribution:
        """DataTypeHistogram.toDistribution (DataType.scala:103-122): ratio = count / total
        (NaN on an empty table, as the JVM's 0.0 / 0)."""
        total = self.num_null + self.num_string + self.num_boolean + self.num_integral + \
            self.num_fractional

        def ratio(c):
            return c / total if total else float("nan")
        pairs = [(DataTypeInstances.Unknown, self.num_null),
                 (DataTypeInstances.Fractional, self.num_fractional),
                 (DataTypeInstances.Integral, self.num_integral),
                 (DataTypeInstances.Boolean, self.num_boolean),
                 (DataTypeInstances.String, self.num_string)]
        return Distribution({k.name: DistributionValue(c, ratio(c)) for k, c in pairs}, 5)


def determine_type(dist: Distribution) -> DataTypeInstances:
    """DataTypeHistogram.determineType (DataType.scala:124-150)."""
    def r(k: DataTypeInstances) -> float:
        v = dist.values.get(k.name)
        return v.ratio if v is not None else 0.0
    if r(DataTypeInstances.Unknown) == 1.0:
        return DataTypeInstances.Unknown
    if r(DataTypeInstances.String) > 0.0 or (
            r(DataTypeInstances.Boolean) > 0.0 and
            (r(DataTypeInstances.Integral) > 0.0 or r(DataTypeInstances.Fractional) > 0.0)):
        return DataTypeInstances.String
    if r(DataTypeInstances.Boolean) > 0.0:
        return DataTypeInstances.Boolean
    if r(DataTypeInstances.Fractional) > 0.0:
        return DataTypeInstances.Fractional
    return DataTypeInstances.Integral


@dataclass(frozen=True)
class DataType(StandardScanShareableAnalyzer):
    """DataType.scala:162-183"""
    column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "DataType"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        return [AggSpec(N.AGG_DTYPE, col=self.column, where=self.where)]

    def from_aggregation_result(self, result, offset):
        v = result[offset]
        return None if v is None else DataTypeHistogram(*v)

    def compute_metric_from(self, state):
        if state is None:
            return self.to_failure_metric(empty_state_exception(self))
        return HistogramMetric(self.column, Success(state.to_distribution()))

    def to_failure_metric(self, exception):
        return HistogramMetric(self.column, Failure(wrap_if_necessary(exception)))

    def preconditions(self):
        return [Preconditions.has_column(self.column)]


__all__ = ["DataType", "DataTypeHistogram", "DataTypeInstances", "determine_type"]
