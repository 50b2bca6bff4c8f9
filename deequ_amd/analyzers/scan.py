"""Scan-shareable analyzers: every one of them runs inside the single fused scan.

Each class cites the reference file it mirrors; ``aggregation_functions`` returns the same
aggregations (as AggSpecs) in the same order, so the offsets the runner computes are the
reference's offsets, and ``from_aggregation_result`` applies the same null rules.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple

from .. import _native as N
from ..exceptions import HllBiasTablesUnavailableException
from ..metrics import Entity
from .base import (AggSpec, DoubleValuedState, NumMatchesAndCount, Preconditions,
                   StandardScanShareableAnalyzer, conditional_count, count_all, if_no_nulls_in)


# ------------------------------------------------------------------------------------------------
# Size (Size.scala:23-48)
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class NumMatches(DoubleValuedState):
    num_matches: int

    def sum(self, other: "NumMatches") -> "NumMatches":
        return NumMatches(self.num_matches + other.num_matches)

    def metric_value(self) -> float:
        return float(self.num_matches)


@dataclass(frozen=True)
class Size(StandardScanShareableAnalyzer):
    where: Optional[str] = None
    _options = ("where",)
    _name = "Size"
    _entity = Entity.Dataset

    def _instance(self):
        return "*"

    def aggregation_functions(self):
        return [conditional_count(self.where)]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 1, lambda: NumMatches(int(result[offset])))


# ------------------------------------------------------------------------------------------------
# Completeness (Completeness.scala:26-46)
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Completeness(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "Completeness"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        return [AggSpec(N.AGG_COUNT_NOTNULL, col=self.column, where=self.where),
                conditional_count(self.where)]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 2, lambda: NumMatchesAndCount(
            int(result[offset]), int(result[offset + 1])))

    def additional_preconditions(self):
        return [Preconditions.has_column(self.column)]


# ------------------------------------------------------------------------------------------------
# Compliance (Compliance.scala:37-53)
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Compliance(StandardScanShareableAnalyzer):
    instance: str
    predicate: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "Compliance"

    def _instance(self):
        return self.instance

    def aggregation_functions(self):
        return [AggSpec(N.AGG_COUNT_TRUE, expr=self.predicate, where=self.where),
                conditional_count(self.where)]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 2, lambda: NumMatchesAndCount(
            int(result[offset]), int(result[offset + 1])))


# ------------------------------------------------------------------------------------------------
# PatternMatch (PatternMatch.scala:41-53)
# ------------------------------------------------------------------------------------------------
class Patterns:
    """PatternMatch.scala:56-72 (Java regex syntax, compiled by deequ_amd/regex.py)."""
    EMAIL = (r"""(?:[a-z0-9!#$%&'*+/=?^_`{|}~-]+(?:\.[a-z0-9!#$%&'*+/=?^_`{|}~-]+)*|"(?:[\x01-\x08\x0b"""
             r"""\x0c\x0e-\x1f\x21\x23-\x5b\x5d-\x7f]|\\[\x01-\x09\x0b\x0c\x0e-\x7f])*")@(?:(?:[a-z0-9]"""
             r"""(?:[a-z0-9-]*[a-z0-9])?\.)+[a-z0-9](?:[a-z0-9-]*[a-z0-9])?|\[(?:(?:25[0-5]|2[0-4][0-9]|"""
             r"""[01]?[0-9][0-9]?)\.){3}(?:25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?|[a-z0-9-]*[a-z0-9]:(?:"""
             r"""[\x01-\x08\x0b\x0c\x0e-\x1f\x21-\x5a\x53-\x7f]|\\[\x01-\x09\x0b\x0c\x0e-\x7f])+)\])""")
    URL = r"(https?|ftp)://[^\s/$.?#].[^\s]*"
    SOCIAL_SECURITY_NUMBER_US = (
        r"((?!219-09-9999|078-05-1120)(?!666|000|9\d{2})\d{3}-(?!00)\d{2}-(?!0{4})\d{4})|"
        r"((?!219 09 9999|078 05 1120)(?!666|000|9\d{2})\d{3} (?!00)\d{2} (?!0{4})\d{4})|"
        r"((?!219099999|078051120)(?!666|000|9\d{2})\d{3}(?!00)\d{2}(?!0{4})\d{4})")
    CREDITCARD = (r"\b(?:3[47]\d{2}([\ \-]?)\d{6}\1\d|(?:(?:4\d|5[1-5]|65)\d{2}|6011)([\ \-]?)"
                  r"\d{4}\2\d{4}\2)\d{4}\b")


def _sql_string(s: str) -> str:
    return "'" + s.replace("\\", "\\\\").replace("'", "''") + "'"


@dataclass(frozen=True)
class PatternMatch(StandardScanShareableAnalyzer):
    """Fraction of rows (where `where` holds) whose first regex find() match in `column` is
    non-empty: sum(when(regexp_extract(col, p, 0) != "", 1).otherwise(0)) / count(*).  The
    pattern compiles to a byte automaton the device runs per row (XI_REGEX); an unsupported
    pattern is a failure metric, never a different answer."""
    column: str
    pattern: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "PatternMatch"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        from ..sqlexpr import FIND_NONEMPTY
        col = "`" + self.column.replace("`", "``") + "`"
        return [AggSpec(N.AGG_COUNT_TRUE, expr=f"{FIND_NONEMPTY}({col}, {_sql_string(self.pattern)})",
                        where=self.where),
                conditional_count(self.where)]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 2, lambda: NumMatchesAndCount(
            int(result[offset]), int(result[offset + 1])))

    def preconditions(self):
        return [Preconditions.has_column(self.column)] + super().preconditions()


# ------------------------------------------------------------------------------------------------
# Sum (Sum.scala:25-52)
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class SumState(DoubleValuedState):
    sum_value: float

    def sum(self, other: "SumState") -> "SumState":
        return SumState(self.sum_value + other.sum_value)

    def metric_value(self) -> float:
        return self.sum_value


@dataclass(frozen=True)
class Sum(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "Sum"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        return [AggSpec(N.AGG_SUM, col=self.column, where=self.where)]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 1, lambda: SumState(float(result[offset])))

    def additional_preconditions(self):
        return [Preconditions.has_column(self.column), Preconditions.is_numeric(self.column)]


# ------------------------------------------------------------------------------------------------
# Mean (Mean.scala:25-53) -- the denominator is count(*) over ALL rows
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class MeanState(DoubleValuedState):
    sum_value: float
    count: int

    def sum(self, other: "MeanState") -> "MeanState":
        return MeanState(self.sum_value + other.sum_value, self.count + other.count)

    def metric_value(self) -> float:
        if self.count == 0:
            return float("nan")
        return self.sum_value / self.count


@dataclass(frozen=True)
class Mean(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "Mean"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        return [AggSpec(N.AGG_SUM, col=self.column, where=self.where), count_all()]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 2, lambda: MeanState(
            float(result[offset]), int(result[offset + 1])))

    def additional_preconditions(self):
        return [Preconditions.has_column(self.column), Preconditions.is_numeric(self.column)]


# ------------------------------------------------------------------------------------------------
# Minimum / Maximum (Minimum.scala:25-53, Maximum.scala:25-53)
# ------------------------------------------------------------------------------------------------
def _scala_min(a: float, b: float) -> float:
    """scala.math.min on doubles: NaN if either is NaN."""
    if math.isnan(a) or math.isnan(b):
        return float("nan")
    return min(a, b)


def _scala_max(a: float, b: float) -> float:
    if math.isnan(a) or math.isnan(b):
        return float("nan")
    return max(a, b)


@dataclass(frozen=True)
class MinState(DoubleValuedState):
    min_value: float

    def sum(self, other: "MinState") -> "MinState":
        return MinState(_scala_min(self.min_value, other.min_value))

    def metric_value(self) -> float:
        return self.min_value


@dataclass(frozen=True)
class MaxState(DoubleValuedState):
    max_value: float

    def sum(self, other: "MaxState") -> "MaxState":
        return MaxState(_scala_max(self.max_value, other.max_value))

    def metric_value(self) -> float:
        return self.max_value


@dataclass(frozen=True)
class Minimum(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "Minimum"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        return [AggSpec(N.AGG_MIN, col=self.column, where=self.where)]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 1, lambda: MinState(float(result[offset])))

    def additional_preconditions(self):
        return [Preconditions.has_column(self.column), Preconditions.is_numeric(self.column)]


@dataclass(frozen=True)
class Maximum(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "Maximum"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        return [AggSpec(N.AGG_MAX, col=self.column, where=self.where)]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 1, lambda: MaxState(float(result[offset])))

    def additional_preconditions(self):
        return [Preconditions.has_column(self.column), Preconditions.is_numeric(self.column)]


# ------------------------------------------------------------------------------------------------
# StandardDeviation (StandardDeviation.scala:25-73)
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class StandardDeviationState(DoubleValuedState):
    n: float
    avg: float
    m2: float

    def __post_init__(self):
        if not self.n > 0.0:
            raise ValueError("requirement failed: Standard deviation is undefined for n = 0.")

    def metric_value(self) -> float:
        return math.sqrt(self.m2 / self.n)

    def sum(self, other: "StandardDeviationState") -> "StandardDeviationState":
        new_n = self.n + other.n
        delta = other.avg - self.avg
        delta_n = 0.0 if new_n == 0.0 else delta / new_n
        return StandardDeviationState(new_n, self.avg + delta_n * other.n,
                                      self.m2 + other.m2 + delta * delta_n * self.n * other.n)


@dataclass(frozen=True)
class StandardDeviation(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "StandardDeviation"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        return [AggSpec(N.AGG_STDDEV_POP, col=self.column, where=self.where)]

    def from_aggregation_result(self, result, offset):
        row = result[offset]
        if row is None:
            return None
        n, avg, m2 = row
        if n == 0.0:
            return None
        return StandardDeviationState(n, avg, m2)

    def additional_preconditions(self):
        return [Preconditions.has_column(self.column), Preconditions.is_numeric(self.column)]


# ------------------------------------------------------------------------------------------------
# Correlation (Correlation.scala:26-105)
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class CorrelationState(DoubleValuedState):
    n: float
    x_avg: float
    y_avg: float
    ck: float
    x_mk: float
    y_mk: float

    def __post_init__(self):
        if not self.n > 0.0:
            raise ValueError("requirement failed: Correlation undefined for n = 0.")

    def sum(self, other: "CorrelationState") -> "CorrelationState":
        n1, n2 = self.n, other.n
        new_n = n1 + n2
        dx = other.x_avg - self.x_avg
        dx_n = 0.0 if new_n == 0.0 else dx / new_n
        dy = other.y_avg - self.y_avg
        dy_n = 0.0 if new_n == 0.0 else dy / new_n
        return CorrelationState(new_n, self.x_avg + dx_n * n2, self.y_avg + dy_n * n2,
                                self.ck + other.ck + dx * dy_n * n1 * n2,
                                self.x_mk + other.x_mk + dx * dx_n * n1 * n2,
                                self.y_mk + other.y_mk + dy * dy_n * n1 * n2)

    def metric_value(self) -> float:
        denom = math.sqrt(self.x_mk * self.y_mk) if self.x_mk * self.y_mk >= 0 else float("nan")
        if denom == 0.0:
            return float("nan") if self.ck == 0.0 else math.copysign(float("inf"), self.ck)
        return self.ck / denom


@dataclass(frozen=True)
class Correlation(StandardScanShareableAnalyzer):
    first_column: str
    second_column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "Correlation"
    _entity = Entity.Mutlicolumn

    def _instance(self):
        return f"{self.first_column},{self.second_column}"

    def aggregation_functions(self):
        return [AggSpec(N.AGG_CORR, col=self.first_column, col2=self.second_column,
                        where=self.where)]

    def from_aggregation_result(self, result, offset):
        row = result[offset]
        if row is None:
            return None
        if row[0] > 0.0:
            return CorrelationState(*row)
        return None

    def additional_preconditions(self):
        return [Preconditions.has_column(self.first_column),
                Preconditions.is_numeric(self.first_column),
                Preconditions.has_column(self.second_column),
                Preconditions.is_numeric(self.second_column)]


# ------------------------------------------------------------------------------------------------
# ApproxCountDistinct (ApproxCountDistinct.scala:26-64 + StatefulHyperloglogPlus.scala)
# ------------------------------------------------------------------------------------------------
_M = 512
_REG_BITS = 6
_REGS_PER_WORD = 10
_MASK = 0x3F


def _signed64(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= (1 << 63) else v


def hll_merge_words(w1: Tuple[int, ...], w2: Tuple[int, ...]) -> Tuple[int, ...]:
    """HyperLogLogPlusPlusUtils.merge (StatefulHyperloglogPlus.scala:186-206)."""
    out = []
    idx = 0
    for a, b in zip(w1, w2):
        a &= 0xFFFFFFFFFFFFFFFF
        b &= 0xFFFFFFFFFFFFFFFF
        word, mask, i = 0, _MASK, 0
        while idx < _M and i < _REGS_PER_WORD:
            word |= max(a & mask, b & mask)
            mask <<= _REG_BITS
            i += 1
            idx += 1
        out.append(_signed64(word))
    return tuple(out)


def hll_words_to_bytes(words) -> bytes:
    """wordsToBytes: 52 longs, big-endian (StatefulHyperloglogPlus.scala:168-176)."""
    return b"".join((w & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "big") for w in words)


def hll_words_from_bytes(data: bytes) -> Tuple[int, ...]:
    if len(data) != 52 * 8:
        raise ValueError("requirement failed")
    return tuple(_signed64(int.from_bytes(data[8 * i: 8 * i + 8], "big")) for i in range(52))


@dataclass(frozen=True)
class ApproxCountDistinctState(DoubleValuedState):
    words: Tuple[int, ...]

    def sum(self, other: "ApproxCountDistinctState") -> "ApproxCountDistinctState":
        return ApproxCountDistinctState(hll_merge_words(self.words, other.words))

    def metric_value(self) -> float:
        """HyperLogLogPlusPlusUtils.count (StatefulHyperloglogPlus.scala:208-255).  Where the
        reference would subtract its empirical bias (E < 5M, no linear counting) the tables are
        missing here, so the metric is a Failure rather than a silently different number."""
        est, needs_bias = N.hll_count(self.words)
        if needs_bias:
            raise HllBiasTablesUnavailableException(
                f"ApproxCountDistinct raw estimate {est:.0f} lies in the HLL++ bias-correction range "
                f"(< {5 * _M}); Spark's BIAS_DATA tables are not available to this engine")
        return est

    def raw_estimate(self) -> float:
        """The estimate without the bias correction (equal to deequ's outside that range)."""
        return N.hll_count(self.words)[0]


@dataclass(frozen=True)
class ApproxCountDistinct(StandardScanShareableAnalyzer):
    column: str
    where: Optional[str] = None
    _options = ("where",)
    _name = "ApproxCountDistinct"

    def _instance(self):
        return self.column

    def aggregation_functions(self):
        return [AggSpec(N.AGG_HLL, col=self.column, where=self.where)]

    def from_aggregation_result(self, result, offset):
        return if_no_nulls_in(result, offset, 1,
                              lambda: ApproxCountDistinctState(tuple(result[offset])))

    def additional_preconditions(self):
        return [Preconditions.has_column(self.column)]


__all__ = [
    "NumMatches", "Size", "Completeness", "Compliance", "SumState", "Sum", "MeanState", "Mean",
    "MinState", "MaxState", "Minimum", "Maximum", "StandardDeviationState", "StandardDeviation",
    "CorrelationState", "Correlation", "ApproxCountDistinctState", "ApproxCountDistinct",
    "hll_merge_words", "hll_words_to_bytes", "hll_words_from_bytes",
]
