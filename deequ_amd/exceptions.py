"""Exception hierarchy of runners/MetricCalculationException.scala:19-78."""
from __future__ import annotations


class MetricCalculationException(Exception):
    pass


class MetricCalculationRuntimeException(MetricCalculationException):
    def __init__(self, message=None, cause: BaseException = None):
        if cause is not None and message is None:
            message = f"{type(cause).__name__}: {cause}"
        super().__init__(message)
        self.__cause__ = cause


class MetricCalculationPreconditionException(MetricCalculationException):
    pass


class NoSuchColumnException(MetricCalculationPreconditionException):
    pass


class WrongColumnTypeException(MetricCalculationPreconditionException):
    pass


class NoColumnsSpecifiedException(MetricCalculationPreconditionException):
    pass


class NumberOfSpecifiedColumnsException(MetricCalculationPreconditionException):
    pass


class IllegalAnalyzerParameterException(MetricCalculationPreconditionException):
    pass


class EmptyStateException(MetricCalculationRuntimeException):
    def __init__(self, message: str):
        super().__init__(message)


class HllBiasTablesUnavailableException(MetricCalculationRuntimeException):
    """ApproxCountDistinct's estimate fell in HLL++'s empirical-bias range (raw estimate E < 5M and
    no linear counting): the reference subtracts estimateBias(E) from Spark's RAW_ESTIMATE_DATA /
    BIAS_DATA tables (StatefulHyperloglogPlus.scala:235-237, 257-295), which are not available to
    this engine.  Raised instead of returning a value that would differ from deequ's.

    In that range the sketch's linear counting already estimates more than LINEAR_COUNTING_FLOOR
    distinct values (HyperLogLogPlusPlus.THRESHOLDS(P - 4) for P = 9): consumers that only compare
    the count with a smaller bound (the ColumnProfiler's histogram threshold) can still decide."""
    LINEAR_COUNTING_FLOOR = 400


class AnalysisException(Exception):
    """Stand-in for Spark's AnalysisException (unresolvable column / unparseable expression)."""


class ReusingNotPossibleResultsMissingException(RuntimeError):
    pass


def wrap_if_necessary(exception: BaseException) -> MetricCalculationException:
    """MetricCalculationException.wrapIfNecessary (MetricCalculationException.scala:69-76)."""
    if isinstance(exception, MetricCalculationException):
        return exception
    return MetricCalculationRuntimeException(cause=exception)
