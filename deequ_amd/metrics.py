"""Metric results (reference: metrics/Metric.scala:21-68, metrics/HistogramMetric.scala:21-61)
and a minimal Scala ``Try`` (``Success`` / ``Failure``) so that results compare like the
reference's case classes do."""
from __future__ import annotations

import math
from dataclasses import dataclass
from enum import Enum
from typing import Any, Dict, List


class Entity(Enum):
    # the misspelling "Mutlicolumn" is the reference's (Metric.scala:22)
    Dataset = "Dataset"
    Column = "Column"
    Mutlicolumn = "Mutlicolumn"

    def __str__(self) -> str:
        return self.value


class Try:
    is_success: bool = False

    @property
    def is_failure(self) -> bool:
        return not self.is_success


class Success(Try):
    is_success = True

    def __init__(self, value: Any):
        self.value = value

    def get(self):
        return self.value

    def __eq__(self, other):
        if not isinstance(other, Success):
            return NotImplemented
        a, b = self.value, other.value
        if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
            return True  # Scala Double boxed equality treats NaN == NaN
        return a == b

    def __hash__(self):
        return hash(("Success", self.value))

    def __repr__(self):
        return f"Success({self.value!r})"


class Failure(Try):
    is_success = False

    def __init__(self, exception: BaseException):
        self.exception = exception

    def get(self):
        raise self.exception

    @property
    def failed(self) -> BaseException:
        return self.exception

    def __eq__(self, other):
        if not isinstance(other, Failure):
            return NotImplemented
        return self.exception is other.exception

    def __hash__(self):
        return hash(("Failure", id(self.exception)))

    def __repr__(self):
        return f"Failure({type(self.exception).__name__}: {self.exception})"


class Metric:
    entity: Entity
    name: str
    instance: str
    value: Try

    def flatten(self) -> List["DoubleMetric"]:
        raise NotImplementedError


@dataclass(frozen=True, eq=True)
class DoubleMetric(Metric):
    entity: Entity
    name: str
    instance: str
    value: Try

    def flatten(self) -> List["DoubleMetric"]:
        return [self]


@dataclass(frozen=True, eq=True)
class KeyedDoubleMetric(Metric):
    entity: Entity
    name: str
    instance: str
    value: Try  # Try[Dict[str, float]]

    def flatten(self) -> List[DoubleMetric]:
        if self.value.is_success:
            return [DoubleMetric(self.entity, f"{self.name}-{k}", self.instance, Success(v))
                    for k, v in self.value.get().items()]
        return [DoubleMetric(self.entity, self.name, self.instance, Failure(self.value.failed))]


@dataclass(frozen=True, eq=True)
class DistributionValue:
    absolute: int
    ratio: float


@dataclass(frozen=True)
class Distribution:
    values: Dict[str, DistributionValue]
    number_of_bins: int

    def __getitem__(self, key: str) -> DistributionValue:
        return self.values[key]

    def __eq__(self, other):
        return isinstance(other, Distribution) and self.values == other.values and \
            self.number_of_bins == other.number_of_bins

    def __hash__(self):
        return hash((tuple(sorted(self.values.items())), self.number_of_bins))

    def argmax(self) -> str:
        return max(self.values.items(), key=lambda kv: kv[1].absolute)[0]


@dataclass(frozen=True, eq=True)
class HistogramMetric(Metric):
    column: str
    value: Try  # Try[Distribution]

    @property
    def entity(self) -> Entity:
        return Entity.Column

    @property
    def instance(self) -> str:
        return self.column

    @property
    def name(self) -> str:
        return "Histogram"

    def flatten(self) -> List[DoubleMetric]:
        if self.value.is_failure:
            return [DoubleMetric(self.entity, f"{self.name}.bins", self.instance,
                                 Failure(self.value.failed))]
        d: Distribution = self.value.get()
        out = [DoubleMetric(self.entity, f"{self.name}.bins", self.instance,
                            Success(float(d.number_of_bins)))]
        for k, v in d.values.items():
            out.append(DoubleMetric(self.entity, f"{self.name}.abs.{k}", self.instance,
                                    Success(float(v.absolute))))
            out.append(DoubleMetric(self.entity, f"{self.name}.ratio.{k}", self.instance,
                                    Success(v.ratio)))
        return out
