"""Check / Constraint DSL and VerificationSuite (M/checks/Check.scala,
M/constraints/AnalysisBasedConstraint.scala, M/VerificationSuite.scala:264-282).

CPU: constraint evaluation over hand-built metrics -- statuses, the reference's message format
(`Value: $v does not meet the constraint requirement!`, AnalysisBasedConstraint.scala:83),
constraint names, where-replacement, predicate text of isContainedIn / isNonNegative.
GPU: the README BasicExample (configs[0]) end to end through the fused HIP scan and group-by.
"""
import pytest

from deequ_amd.analyzers import Completeness, Compliance, Size, Uniqueness
from deequ_amd.checks import Check, CheckLevel, CheckStatus, ConstraintStatus
from deequ_amd.metrics import DoubleMetric, Entity, Failure, Success
from deequ_amd.runners import AnalyzerContext
from deequ_amd.verification import VerificationSuite


def _ctx(pairs):
    return AnalyzerContext({a: DoubleMetric(Entity.Column, type(a).__name__, "x", v)
                            for a, v in pairs})


def test_completeness_failure_message_and_status():
    check = Check(CheckLevel.Error, "integrity").is_complete("name").has_size(lambda n: n == 5)
    ctx = _ctx([(Completeness("name"), Success(0.8)), (Size(), Success(5.0))])
    r = check.evaluate(ctx)
    assert r.status == CheckStatus.Error
    c0, c1 = r.constraint_results
    assert str(c0.constraint) == "CompletenessConstraint(Completeness(name,None))"
    assert c0.status == ConstraintStatus.Failure
    assert c0.message == "Value: 0.8 does not meet the constraint requirement!"
    assert c1.status == ConstraintStatus.Success
    assert str(c1.constraint) == "SizeConstraint(Size(None))"


def test_warning_level_and_hint_and_missing_and_failed_metric():
    check = (Check(CheckLevel.Warning, "w").has_completeness("a", lambda v: v > 0.9, hint="why")
             .is_complete("b").is_complete("c"))
    ctx = _ctx([(Completeness("a"), Success(0.5)),
                (Completeness("b"), Failure(RuntimeError("boom")))])
    r = check.evaluate(ctx)
    assert r.status == CheckStatus.Warning
    a, b, c = r.constraint_results
    assert a.message == "Value: 0.5 does not meet the constraint requirement! why"
    assert b.message == "boom"
    assert c.message == "Missing Analysis, can't run the constraint!"


def test_where_replaces_last_constraint_and_predicates():
    check = Check(CheckLevel.Error, "c").is_complete("a").where("b > 0")
    assert check.required_analyzers() == [Completeness("a", "b > 0")]
    check = Check(CheckLevel.Error, "c").is_contained_in("priority", ["high", "lo'w"])
    (a,) = check.required_analyzers()
    assert a == Compliance("priority contained in high,lo'w",
                           "priority IS NULL OR priority IN ('high','lo''w')")
    check = Check(CheckLevel.Error, "c").is_non_negative("numViews")
    assert check.required_analyzers() == [Compliance("numViews is Fnon-negative", "numViews >= 0")]
    # the range form tests include_lower_bound for both operators (Check.scala:863)
    check = Check(CheckLevel.Error, "c").is_contained_in("x", lower_bound=1, upper_bound=2,
                                                          include_lower_bound=False)
    (a,) = check.required_analyzers()
    assert a.predicate == "x IS NULL OR (x > 1.0 AND x < 2.0)"


def test_data_type_and_mutual_information_checks():
    """Check.scala:653-661 (unnamed: the AnalysisBasedConstraint's own toString) and :371-379."""
    from deequ_amd.analyzers import DataType, MutualInformation
    from deequ_amd.checks import ConstrainableDataTypes
    from deequ_amd.metrics import Distribution, DistributionValue, HistogramMetric
    check = (Check(CheckLevel.Error, "t").has_data_type("c", ConstrainableDataTypes.Numeric,
                                                       lambda v: v >= 0.5)
             .has_mutual_information("a", "b", lambda v: v > 0.1))
    assert check.required_analyzers() == [DataType("c"), MutualInformation(["a", "b"])]
    assert str(check.constraints[0]) == \
        "AnalysisBasedConstraint(DataType(c,None),<function1>,Some(<function1>),None)"
    assert str(check.constraints[1]) == "MutualInformationConstraint(MutualInformation(List(a, b)))"
    dist = Distribution({"Unknown": DistributionValue(1, 0.25), "Fractional": DistributionValue(1, 0.25),
                         "Integral": DistributionValue(1, 0.25), "Boolean": DistributionValue(0, 0.0),
                         "String": DistributionValue(1, 0.25)}, 5)
    ctx = AnalyzerContext({DataType("c"): HistogramMetric("c", Success(dist)),
                           MutualInformation(["a", "b"]): DoubleMetric(Entity.Mutlicolumn,
                                                                      "MutualInformation", "a,b",
                                                                      Success(0.05))})
    r = check.evaluate(ctx)
    assert [c.status for c in r.constraint_results] == [ConstraintStatus.Success,
                                                        ConstraintStatus.Failure]


def test_pattern_and_quantile_checks_require_their_analyzers():
    """Check.scala:560-642 / 391-398: containsURL & co. are hasPattern with the Patterns regexes
    and their own names; hasApproxQuantile names ApproxQuantileConstraint(ApproxQuantile(...))."""
    from deequ_amd.analyzers import ApproxQuantile, PatternMatch, Patterns
    check = (Check(CheckLevel.Warning, "d").contains_url("description", lambda v: v >= 0.5)
             .contains_email("e").contains_credit_card_number("c")
             .contains_social_security_number("s").has_pattern("p", r"\d+")
             .has_approx_quantile("n", 0.5, lambda v: v <= 10))
    assert check.required_analyzers() == [
        PatternMatch("description", Patterns.URL), PatternMatch("e", Patterns.EMAIL),
        PatternMatch("c", Patterns.CREDITCARD), PatternMatch("s", Patterns.SOCIAL_SECURITY_NUMBER_US),
        PatternMatch("p", r"\d+"), ApproxQuantile("n", 0.5)]
    names = [str(c) for c in check.constraints]
    assert names == ["containsURL(description)", "containsEmail(e)", "containsCreditCardNumber(c)",
                     "containsSocialSecurityNumber(s)", "PatternMatchConstraint(p, \\d+)",
                     "ApproxQuantileConstraint(ApproxQuantile(n,0.5,0.01))"]


def test_suite_status_is_the_worst_check():
    ok = Check(CheckLevel.Error, "ok").has_size(lambda n: n == 5)
    warn = Check(CheckLevel.Warning, "w").is_complete("a")
    ctx = _ctx([(Size(), Success(5.0)), (Completeness("a"), Success(0.5))])
    res = VerificationSuite.evaluate([ok, warn], ctx)
    assert res.status == CheckStatus.Warning
    rows = res.check_results_as_rows(res)
    assert [r["constraint_status"] for r in rows] == ["Success", "Failure"]


@pytest.mark.gpu
def test_basic_example_end_to_end(gpu_device):
    """M/examples/BasicExample.scala:25-76 on the GPU, both checks: isComplete(name) = 0.8 fails
    (Error), containsURL(description) = 0.4 fails (Warning), the median of numViews is 5.0 and every
    other constraint passes; the suite status is Error."""
    import pyarrow as pa

    from deequ_amd import Table
    data = pa.table({
        "id": pa.array([1, 2, 3, 4, 5], pa.int64()),
        "name": pa.array(["Thingy A", "Thingy B", None, "Thingy D", "Thingy E"]),
        "description": pa.array(["awesome thing.", "available at http://thingb.com", None,
                                 "checkout https://thingd.ca", None]),
        "priority": pa.array(["high", None, "low", "low", "high"]),
        "numViews": pa.array([0, 0, 5, 10, 12], pa.int64()),
    })
    df = Table.from_arrow(data, device=gpu_device)
    integrity = (Check(CheckLevel.Error, "integrity checks").has_size(lambda n: n == 5)
                 .is_complete("id").is_unique("id").is_complete("name")
                 .is_contained_in("priority", ["high", "low"]).is_non_negative("numViews"))
    distribution = (Check(CheckLevel.Warning, "distribution checks")
                    .contains_url("description", lambda v: v >= 0.5)
                    .has_approx_quantile("numViews", 0.5, lambda v: v <= 10))
    res = VerificationSuite().on_data(df).add_check(integrity).add_check(distribution).run()
    assert res.status == CheckStatus.Error
    assert res.check_results[integrity].status == CheckStatus.Error
    assert res.check_results[distribution].status == CheckStatus.Warning
    statuses = [(str(c.constraint), c.status, c.message)
                for c in res.check_results[integrity].constraint_results]
    failed = [s for s in statuses if s[1] != ConstraintStatus.Success]
    assert failed == [("CompletenessConstraint(Completeness(name,None))",
                       ConstraintStatus.Failure,
                       "Value: 0.8 does not meet the constraint requirement!")]
    url, median = res.check_results[distribution].constraint_results
    assert str(url.constraint) == "containsURL(description)"
    assert url.status == ConstraintStatus.Failure
    assert url.message == "Value: 0.4 does not meet the constraint requirement!"
    assert str(median.constraint) == "ApproxQuantileConstraint(ApproxQuantile(numViews,0.5,0.01))"
    assert median.status == ConstraintStatus.Success
    assert res.metrics[Uniqueness(["id"])].value.get() == 1.0
    from deequ_amd.analyzers import ApproxQuantile
    assert res.metrics[ApproxQuantile("numViews", 0.5)].value.get() == 5.0
