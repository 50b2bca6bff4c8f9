"""Analyzer / State algebra (reference: analyzers/Analyzer.scala).

Every analyzer is a frozen dataclass, so -- like the reference's case classes -- analyzers are
compared and hashed by value (AnalyzerContext maps are keyed by them, duplicates run once).
Scan-shareable analyzers describe their aggregation functions as :class:`AggSpec` values; the
runner concatenates them, and the HIP engine evaluates all of them in one fused pass, returning a
result row that ``from_aggregation_result(row, offset)`` reads exactly like the Scala code reads
the Spark ``Row``.
"""
from __future__ import annotations

from dataclasses import dataclass, fields
from typing import Callable, List, Optional, Sequence

from .. import _native as N
from ..exceptions import (EmptyStateException, MetricCalculationException,
                          NoColumnsSpecifiedException,
                          NoSuchColumnException, NumberOfSpecifiedColumnsException,
                          WrongColumnTypeException, wrap_if_necessary)
from ..metrics import DoubleMetric, Entity, Failure, Success

COL_PREFIX = "com_amazon_deequ_dq_metrics_"
COUNT_COL = COL_PREFIX + "count"


# ------------------------------------------------------------------------------------------------
# States
# ------------------------------------------------------------------------------------------------
class State:
    """A state (sufficient statistic) computed from data; a commutative semigroup under ``sum``
    (Analyzer.scala:34-48)."""

    def sum(self, other: "State") -> "State":
        raise NotImplementedError

    def __add__(self, other):
        return self.sum(other)


class DoubleValuedState(State):
    def metric_value(self) -> float:
        raise NotImplementedError


@dataclass(frozen=True)
class NumMatchesAndCount(DoubleValuedState):
    """Analyzer.scala:220-234"""
    num_matches: int
    count: int

    def sum(self, other: "NumMatchesAndCount") -> "NumMatchesAndCount":
        return NumMatchesAndCount(self.num_matches + other.num_matches, self.count + other.count)

    def metric_value(self) -> float:
        if self.count == 0:
            return float("nan")
        return self.num_matches / self.count


# ------------------------------------------------------------------------------------------------
# Aggregation specs (the Spark Columns of aggregationFunctions())
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class AggSpec:
    kind: int                       # _native.AGG_*
    col: Optional[str] = None
    col2: Optional[str] = None
    expr: Optional[str] = None      # SQL of the counted predicate (AGG_COUNT_TRUE)
    where: Optional[str] = None     # SQL of the where filter


def count_all() -> AggSpec:
    return AggSpec(N.AGG_COUNT_ALL)


def conditional_count(where: Optional[str]) -> AggSpec:
    """Analyzers.conditionalCount (Analyzer.scala:404-408): sum(expr(where).cast(Long)) or
    count(*)."""
    if where is None:
        return count_all()
    return AggSpec(N.AGG_COUNT_TRUE, expr=where)


# ------------------------------------------------------------------------------------------------
# Preconditions (Analyzer.scala:275-335)
# ------------------------------------------------------------------------------------------------
_NUMERIC_NAMES = "ByteType,ShortType,IntegerType,LongType,FloatType,DoubleType,DecimalType"


class Preconditions:
    @staticmethod
    def find_first_failing(schema, conditions: Sequence[Callable]) -> Optional[Exception]:
        for condition in conditions:
            try:
                condition(schema)
            except Exception as e:  # noqa: BLE001 -- mirrors `case e: Exception`
                return e
        return None

    @staticmethod
    def at_least_one(columns: Sequence[str]):
        def check(_schema):
            if len(columns) == 0:
                raise NoColumnsSpecifiedException("At least one column needs to be specified!")
        return check

    @staticmethod
    def exactly_n_columns(columns: Sequence[str], n: int):
        def check(_schema):
            if len(columns) != n:
                raise NumberOfSpecifiedColumnsException(
                    f"{n} columns have to be specified! Currently, columns contains only "
                    f"{len(columns)} column(s): {','.join(columns)}!")
        return check

    @staticmethod
    def has_column(column: str):
        def check(schema):
            if column not in schema.field_names:
                raise NoSuchColumnException(f"Input data does not include column {column}!")
        return check

    @staticmethod
    def is_numeric(column: str):
        def check(schema):
            dtype = schema[column].dtype
            if not N.is_numeric(dtype):
                raise WrongColumnTypeException(
                    f"Expected type of column {column} to be one of ({_NUMERIC_NAMES}), but found "
                    f"{schema[column].type_name} instead!")
        return check


# ------------------------------------------------------------------------------------------------
# Analyzers
# ------------------------------------------------------------------------------------------------
def _scala_str(value, is_option: bool) -> str:
    if is_option:
        return "None" if value is None else f"Some({_scala_str(value, False)})"
    if isinstance(value, (list, tuple)):
        return "List(" + ", ".join(_scala_str(v, False) for v in value) + ")"
    if isinstance(value, bool):
        return "true" if value else "false"
    return str(value)


class Analyzer:
    """Common trait of all analyzers (Analyzer.scala:56-155)."""

    _options: tuple = ()

    # -- Scala case-class toString, used in EmptyStateException messages
    def __str__(self) -> str:
        parts = [_scala_str(getattr(self, f.name), f.name in self._options) for f in fields(self)]
        return f"{type(self).__name__}({','.join(parts)})"

    def compute_state_from(self, data):
        raise NotImplementedError

    def compute_metric_from(self, state):
        raise NotImplementedError

    def preconditions(self) -> List[Callable]:
        return []

    def to_failure_metric(self, exception: Exception):
        raise NotImplementedError

    def calculate(self, data, aggregate_with=None, save_states_with=None):
        """Analyzer.calculate (Analyzer.scala:88-103)."""
        try:
            for condition in self.preconditions():
                condition(data.schema)
            state = self.compute_state_from(data)
            return self.calculate_metric(state, aggregate_with, save_states_with)
        except Exception as e:  # noqa: BLE001
            return self.to_failure_metric(e)

    def calculate_metric(self, state, aggregate_with=None, save_states_with=None):
        """Analyzer.scala:107-128"""
        loaded = aggregate_with.load(self) if aggregate_with is not None else None
        to_compute = merge_states(state, loaded)
        if to_compute is not None and save_states_with is not None:
            save_states_with.persist(self, to_compute)
        return self.compute_metric_from(to_compute)

    def aggregate_state_to(self, source_a, source_b, target) -> None:
        """Analyzer.scala:130-147"""
        a, b = source_a.load(self), source_b.load(self)
        agg = merge_states(a, b)
        if agg is not None:
            target.persist(self, agg)

    def load_state_and_compute_metric(self, source):
        state = source.load(self)
        return None if state is None else self.compute_metric_from(state)


def merge_states(*states):
    """Analyzers.merge (Analyzer.scala:343-362): Option-wise State.sum."""
    result = None
    for s in states:
        if s is None:
            continue
        result = s if result is None else result.sum(s)
    return result


class ScanShareableAnalyzer(Analyzer):
    """Analyzer.scala:159-187"""

    def aggregation_functions(self) -> List[AggSpec]:
        raise NotImplementedError

    def from_aggregation_result(self, result, offset: int):
        raise NotImplementedError

    def compute_state_from(self, data):
        """Runs this analyzer's aggregation functions alone (Analyzer.scala:168-172)."""
        from ..runners.engine import run_scan
        row = run_scan(data, self.aggregation_functions())
        return self.from_aggregation_result(row, 0)

    def metric_from_aggregation_result(self, result, offset, aggregate_with=None,
                                       save_states_with=None):
        state = self.from_aggregation_result(result, offset)
        return self.calculate_metric(state, aggregate_with, save_states_with)


def metric_from_value(value: float, name: str, instance: str,
                      entity: Entity = Entity.Column) -> DoubleMetric:
    return DoubleMetric(entity, name, instance, Success(value))


def empty_state_exception(analyzer: Analyzer) -> EmptyStateException:
    return EmptyStateException(f"Empty state for analyzer {analyzer}, all input values were NULL.")


def metric_from_failure(exception: BaseException, name: str, instance: str,
                        entity: Entity = Entity.Column) -> DoubleMetric:
    return DoubleMetric(entity, name, instance, Failure(wrap_if_necessary(exception)))


def metric_from_empty(analyzer, name, instance, entity=Entity.Column) -> DoubleMetric:
    return metric_from_failure(empty_state_exception(analyzer), name, instance, entity)


def entity_from(columns: Sequence[str]) -> Entity:
    return Entity.Column if len(columns) == 1 else Entity.Mutlicolumn


def if_no_nulls_in(result, offset: int, how_many: int = 1, func=None):
    """Analyzers.ifNoNullsIn (Analyzer.scala:365-379)"""
    if any(result[i] is None for i in range(offset, offset + how_many)):
        return None
    return func()


class StandardScanShareableAnalyzer(ScanShareableAnalyzer):
    """Analyzer.scala:190-216: a scan-shareable analyzer producing a DoubleMetric.  Subclasses
    provide ``_name``, ``_instance()`` and ``_entity``."""

    _name: str = ""
    _entity: Entity = Entity.Column

    def _instance(self) -> str:
        raise NotImplementedError

    def compute_metric_from(self, state) -> DoubleMetric:
        if state is not None:
            try:
                value = state.metric_value()
            except MetricCalculationException as e:
                return self.to_failure_metric(e)
            return metric_from_value(value, self._name, self._instance(), self._entity)
        return metric_from_empty(self, self._name, self._instance(), self._entity)

    def to_failure_metric(self, exception) -> DoubleMetric:
        return metric_from_failure(exception, self._name, self._instance(), self._entity)

    def additional_preconditions(self) -> List[Callable]:
        return []

    def preconditions(self) -> List[Callable]:
        return self.additional_preconditions()


class GroupingAnalyzer(Analyzer):
    """Analyzer.scala:263-272"""

    def grouping_columns(self) -> List[str]:
        raise NotImplementedError

    def preconditions(self) -> List[Callable]:
        return [Preconditions.has_column(c) for c in self.grouping_columns()]
