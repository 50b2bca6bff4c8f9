"""Thin callers over the engine: deequ's Check / Constraint DSL.

A Check is a list of constraints; each analysis-based constraint names one analyzer, a value
picker and an assertion.  VerificationSuite (verification.py) collects every check's
required analyzers, runs them in ONE AnalysisRunner pass (the fused HIP scan + the grouping
passes) and evaluates the constraints on the metrics.

Reference: M/checks/Check.scala:34-899, M/constraints/Constraint.scala:60-560,
M/constraints/AnalysisBasedConstraint.scala:38-128.  Method names are the Scala ones in
snake_case; optional Scala arguments are keyword arguments.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Callable, List, Optional, Sequence

from .analyzers import (ApproxCountDistinct, ApproxQuantile, Completeness, DataType,
                        MutualInformation, Compliance, Correlation, Distinctness,
                        Entropy, Histogram, Maximum, Mean, Minimum, PatternMatch, Patterns, Size,
                        StandardDeviation, Sum, UniqueValueRatio, Uniqueness)
from .analyzers.grouping import java_double_to_string


class ConstrainableDataTypes(Enum):
    """Constraint.scala ConstrainableDataTypes"""
    Null = 0
    Fractional = 1
    Integral = 2
    Boolean = 3
    String = 4
    Numeric = 5


class CheckLevel(Enum):
    """Check.scala:29-31"""
    Error = "Error"
    Warning = "Warning"


class CheckStatus(Enum):
    """Check.scala:34-36 (ordered Success < Warning < Error)."""
    Success = 0
    Warning = 1
    Error = 2


class ConstraintStatus(Enum):
    """Constraint.scala:24-26"""
    Success = "Success"
    Failure = "Failure"


MISSING_ANALYSIS = "Missing Analysis, can't run the constraint!"   # AnalysisBasedConstraint:123
PROBLEMATIC_METRIC_PICKER = "Can't retrieve the value to assert on"
ASSERTION_EXCEPTION = "Can't execute the assertion"


def _scala_str(v: Any) -> str:
    """`s"$v"` for the values constraints assert on (Double -> Java Double.toString)."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return java_double_to_string(v)
    return str(v)


@dataclass
class ConstraintResult:
    constraint: "Constraint"
    status: ConstraintStatus
    message: Optional[str] = None
    metric: Any = None


class Constraint:
    def evaluate(self, metric_map) -> ConstraintResult:
        raise NotImplementedError


class AnalysisBasedConstraint(Constraint):
    """AnalysisBasedConstraint.scala:38-115: pick the value from the analyzer's metric, run the
    assertion; a failed metric fails the constraint with the exception's message."""

    def __init__(self, analyzer, assertion: Callable, value_picker: Optional[Callable] = None,
                 hint: Optional[str] = None):
        self.analyzer = analyzer
        self.assertion = assertion
        self.value_picker = value_picker
        self.hint = hint

    def __str__(self):  # the Scala case class's toString
        picker = "Some(<function1>)" if self.value_picker else "None"
        hint = f"Some({self.hint})" if self.hint is not None else "None"
        return f"AnalysisBasedConstraint({self.analyzer},<function1>,{picker},{hint})"

    __repr__ = __str__

    def evaluate(self, metric_map) -> ConstraintResult:
        metric = metric_map.get(self.analyzer)
        if metric is None:
            return ConstraintResult(self, ConstraintStatus.Failure, MISSING_ANALYSIS)
        if metric.value.is_failure:
            return ConstraintResult(self, ConstraintStatus.Failure, str(metric.value.failed),
                                    metric)
        value = metric.value.get()
        try:
            assert_on = self.value_picker(value) if self.value_picker else value
        except Exception as e:  # noqa: BLE001
            return ConstraintResult(self, ConstraintStatus.Failure,
                                    f"{PROBLEMATIC_METRIC_PICKER}: {e}!", metric)
        try:
            ok = bool(self.assertion(assert_on))
        except Exception as e:  # noqa: BLE001
            return ConstraintResult(self, ConstraintStatus.Failure,
                                    f"{ASSERTION_EXCEPTION}: {e}!", metric)
        if ok:
            return ConstraintResult(self, ConstraintStatus.Success, None, metric)
        msg = f"Value: {_scala_str(assert_on)} does not meet the constraint requirement!"
        if self.hint:
            msg += f" {self.hint}"
        return ConstraintResult(self, ConstraintStatus.Failure, msg, metric)


class NamedConstraint(Constraint):
    """Constraint.scala:60-77: a decorator that gives the inner constraint its toString."""

    def __init__(self, inner: Constraint, name: str):
        self.inner = inner
        self.name = name

    def evaluate(self, metric_map) -> ConstraintResult:
        r = self.inner.evaluate(metric_map)
        return ConstraintResult(self, r.status, r.message, r.metric)

    def __str__(self):
        return self.name

    __repr__ = __str__


def _named(analyzer, assertion, kind: str, picker=None, hint=None, label=None):
    return NamedConstraint(AnalysisBasedConstraint(analyzer, assertion, picker, hint),
                           f"{kind}({label if label is not None else analyzer})")


def IS_ONE(v) -> bool:  # noqa: N802 -- Check.IsOne (Check.scala:49)
    return v == 1.0


@dataclass
class CheckResult:
    check: "Check"
    status: CheckStatus
    constraint_results: List[ConstraintResult]


@dataclass
class Check:
    """Check.scala:58-899.  Immutable: every builder returns a new Check."""
    level: CheckLevel
    description: str
    constraints: List[Constraint] = field(default_factory=list)
    _last_filterable: Optional[Callable] = field(default=None, repr=False, compare=False)

    # -- plumbing ---------------------------------------------------------------------------
    def add_constraint(self, constraint: Constraint) -> "Check":
        return Check(self.level, self.description, self.constraints + [constraint])

    def _add_filterable(self, creation: Callable[[Optional[str]], Constraint]) -> "Check":
        """addFilterableConstraint (Check.scala:76-84): `.where(filter)` replaces the last one."""
        return Check(self.level, self.description, self.constraints + [creation(None)], creation)

    def where(self, filter_: str) -> "Check":
        """CheckWithLastConstraintFilterable.where (CheckWithLastConstraintFilterable.scala:27)."""
        if self._last_filterable is None:
            raise AttributeError("where() applies to a filterable constraint only")
        return Check(self.level, self.description,
                     self.constraints[:-1] + [self._last_filterable(filter_)])

    # -- constraints (Check.scala / Constraint.scala) ----------------------------------------
    def has_size(self, assertion: Callable[[int], bool], hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(Size(w), assertion, "SizeConstraint",
                                                     picker=lambda v: int(v), hint=hint))

    def is_complete(self, column: str, hint=None) -> "Check":
        return self.has_completeness(column, IS_ONE, hint)

    def has_completeness(self, column: str, assertion, hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(Completeness(column, w), assertion,
                                                     "CompletenessConstraint", hint=hint))

    def is_unique(self, column: str, hint=None) -> "Check":
        return self.has_uniqueness([column], IS_ONE, hint)

    def is_primary_key(self, column: str, *columns: str, hint=None) -> "Check":
        return self.has_uniqueness([column, *columns], IS_ONE, hint)

    def has_uniqueness(self, columns, assertion, hint=None) -> "Check":
        cols = [columns] if isinstance(columns, str) else list(columns)
        return self.add_constraint(_named(Uniqueness(cols), assertion, "UniquenessConstraint",
                                          hint=hint))

    def has_distinctness(self, columns, assertion, hint=None) -> "Check":
        cols = [columns] if isinstance(columns, str) else list(columns)
        return self.add_constraint(_named(Distinctness(cols), assertion,
                                          "DistinctnessConstraint", hint=hint))

    def has_unique_value_ratio(self, columns, assertion, hint=None) -> "Check":
        cols = [columns] if isinstance(columns, str) else list(columns)
        a = UniqueValueRatio(cols)
        # Constraint.scala:255 (the closing parenthesis is missing in the reference)
        return self.add_constraint(NamedConstraint(AnalysisBasedConstraint(a, assertion, None, hint),
                                                   f"UniqueValueRatioConstraint({a}"))

    def has_number_of_distinct_values(self, column: str, assertion, binning_udf=None,
                                      max_bins: int = 1000, hint=None) -> "Check":
        """Check.scala:269-285: a histogram-bin constraint on numberOfBins."""
        h = Histogram(column, binning_udf, max_bins)
        return self.add_constraint(_named(h, assertion, "HistogramBinConstraint",
                                          picker=lambda d: d.number_of_bins, hint=hint))

    def has_histogram_values(self, column: str, assertion, binning_udf=None,
                             max_bins: int = 1000, hint=None) -> "Check":
        h = Histogram(column, binning_udf, max_bins)
        return self.add_constraint(_named(h, assertion, "HistogramConstraint", hint=hint))

    def has_entropy(self, column: str, assertion, hint=None) -> "Check":
        return self.add_constraint(_named(Entropy(column), assertion, "EntropyConstraint",
                                          hint=hint))

    def has_min(self, column: str, assertion, hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(Minimum(column, w), assertion,
                                                     "MinimumConstraint", hint=hint))

    def has_max(self, column: str, assertion, hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(Maximum(column, w), assertion,
                                                     "MaximumConstraint", hint=hint))

    def has_mean(self, column: str, assertion, hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(Mean(column, w), assertion,
                                                     "MeanConstraint", hint=hint))

    def has_sum(self, column: str, assertion, hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(Sum(column, w), assertion,
                                                     "SumConstraint", hint=hint))

    def has_standard_deviation(self, column: str, assertion, hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(StandardDeviation(column, w), assertion,
                                                     "StandardDeviationConstraint", hint=hint))

    def has_approx_count_distinct(self, column: str, assertion, hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(ApproxCountDistinct(column, w), assertion,
                                                     "ApproxCountDistinctConstraint", hint=hint))

    def has_correlation(self, column_a: str, column_b: str, assertion, hint=None) -> "Check":
        return self._add_filterable(lambda w: _named(Correlation(column_a, column_b, w),
                                                     assertion, "CorrelationConstraint",
                                                     hint=hint))

    def satisfies(self, column_condition: str, constraint_name: str, assertion=None,
                  hint=None) -> "Check":
        """Check.scala:538-548 -> complianceConstraint (Constraint.scala:266-280)."""
        assertion = assertion or IS_ONE
        return self._add_filterable(lambda w: _named(
            Compliance(constraint_name, column_condition, w), assertion, "ComplianceConstraint",
            hint=hint))

    def is_non_negative(self, column: str, hint=None) -> "Check":
        # Check.scala:676: the constraint name carries the reference's "Fnon-negative" typo
        return self.satisfies(f"{column} >= 0", f"{column} is Fnon-negative", hint=hint)

    def is_positive(self, column: str) -> "Check":
        return self.satisfies(f"{column} > 0", f"{column} is positive")

    def is_less_than(self, a: str, b: str, hint=None) -> "Check":
        return self.satisfies(f"{a} < {b}", f"{a} is less than {b}", hint=hint)

    def is_less_than_or_equal_to(self, a: str, b: str, hint=None) -> "Check":
        return self.satisfies(f"{a} <= {b}", f"{a} is less than or equal to {b}", hint=hint)

    def is_greater_than(self, a: str, b: str, hint=None) -> "Check":
        return self.satisfies(f"{a} > {b}", f"{a} is greater than {b}", hint=hint)

    def is_greater_than_or_equal_to(self, a: str, b: str, hint=None) -> "Check":
        return self.satisfies(f"{a} >= {b}", f"{a} is greater than or equal to {b}", hint=hint)

    def is_contained_in(self, column: str, allowed_values: Sequence[str] = None,
                        assertion=None, hint=None, *, lower_bound: float = None,
                        upper_bound: float = None, include_lower_bound: bool = True,
                        include_upper_bound: bool = True) -> "Check":
        """Check.scala:770-869: the value-list form, or (lower_bound / upper_bound) the range
        form.  The range form reproduces the reference's use of include_lower_bound for BOTH
        operators (Check.scala:863); include_upper_bound is accepted and ignored, as there."""
        if allowed_values is not None:
            values = ",".join("'" + v.replace("'", "''") + "'" for v in allowed_values)
            pred = f"{column} IS NULL OR {column} IN ({values})"
            return self.satisfies(pred, f"{column} contained in {','.join(allowed_values)}",
                                  assertion, hint)
        left = ">=" if include_lower_bound else ">"
        right = "<=" if include_lower_bound else "<"
        lo, hi = _scala_str(float(lower_bound)), _scala_str(float(upper_bound))
        pred = f"{column} IS NULL OR ({column} {left} {lo} AND {column} {right} {hi})"
        return self.satisfies(pred, f"{column} between {lo} and {hi}", hint=hint)

    def has_pattern(self, column: str, pattern: str, assertion=None, name=None,
                    hint=None) -> "Check":
        """Check.scala:560-571 -> patternMatchConstraint (Constraint.scala:291-311)."""
        assertion = assertion or IS_ONE

        def make(w):
            c = AnalysisBasedConstraint(PatternMatch(column, pattern, w), assertion, hint=hint)
            return NamedConstraint(c, name or f"PatternMatchConstraint({column}, {pattern})")
        return self._add_filterable(make)

    def contains_credit_card_number(self, column: str, assertion=None, hint=None) -> "Check":
        return self.has_pattern(column, Patterns.CREDITCARD, assertion,
                                f"containsCreditCardNumber({column})", hint)

    def contains_email(self, column: str, assertion=None, hint=None) -> "Check":
        return self.has_pattern(column, Patterns.EMAIL, assertion, f"containsEmail({column})", hint)

    def contains_url(self, column: str, assertion=None, hint=None) -> "Check":
        return self.has_pattern(column, Patterns.URL, assertion, f"containsURL({column})", hint)

    def contains_social_security_number(self, column: str, assertion=None,
                                        hint=None) -> "Check":
        return self.has_pattern(column, Patterns.SOCIAL_SECURITY_NUMBER_US, assertion,
                                f"containsSocialSecurityNumber({column})", hint)

    def has_approx_quantile(self, column: str, quantile: float, assertion,
                            hint=None) -> "Check":
        """Check.scala:391-398 -> approxQuantileConstraint (Constraint.scala:368-381)."""
        a = ApproxQuantile(column, quantile)
        return self.add_constraint(NamedConstraint(AnalysisBasedConstraint(a, assertion, hint=hint),
                                                   f"ApproxQuantileConstraint({a})"))

    def has_data_type(self, column: str, data_type: "ConstrainableDataTypes", assertion=None,
                      hint=None) -> "Check":
        """Check.scala:653-661 -> dataTypeConstraint (Constraint.scala:549-579): the ratio of
        `data_type` in DataType(column)'s distribution (0.0 when absent); Numeric = Fractional +
        Integral.  The reference leaves this constraint unnamed."""
        assertion = assertion or IS_ONE

        def pick(dist):
            def ratio(k):
                v = dist.values.get(k)
                return v.ratio if v is not None else 0.0
            if data_type == ConstrainableDataTypes.Numeric:
                return ratio("Fractional") + ratio("Integral")
            return ratio({ConstrainableDataTypes.Null: "Unknown"}.get(data_type, data_type.name))
        return self.add_constraint(AnalysisBasedConstraint(DataType(column), assertion, pick, hint))

    def has_mutual_information(self, column_a: str, column_b: str, assertion,
                               hint=None) -> "Check":
        """Check.scala:371-379 -> mutualInformationConstraint (Constraint.scala:344-357)."""
        mi = MutualInformation([column_a, column_b])
        return self.add_constraint(NamedConstraint(AnalysisBasedConstraint(mi, assertion, hint=hint),
                                                   f"MutualInformationConstraint({mi})"))

    # -- evaluation --------------------------------------------------------------------------
    def evaluate(self, context) -> CheckResult:
        """Check.scala:876-888"""
        results = [c.evaluate(context.metric_map) for c in self.constraints]
        failed = any(r.status == ConstraintStatus.Failure for r in results)
        if failed:
            status = CheckStatus.Error if self.level == CheckLevel.Error else CheckStatus.Warning
        else:
            status = CheckStatus.Success
        return CheckResult(self, status, results)

    def required_analyzers(self) -> list:
        """Check.scala:890-899 (a set; order of first appearance kept)."""
        out = []
        for c in self.constraints:
            inner = c.inner if isinstance(c, NamedConstraint) else c
            if isinstance(inner, AnalysisBasedConstraint) and inner.analyzer not in out:
                out.append(inner.analyzer)
        return out

    def __hash__(self):
        return id(self)

    def __eq__(self, other):
        return self is other
