"""VerificationSuite (M/VerificationSuite.scala:35-145, 264-282) and VerificationResult
(M/VerificationResult.scala:32-119): the config-1 entry point.

    VerificationSuite().on_data(table).add_check(check).run()

All checks' required analyzers run in ONE AnalysisRunner pass (the fused HIP scan plus the
grouping passes), exactly as `doVerificationRun` builds `requiredAnalyzers ++ checks.flatMap(
_.requiredAnalyzers())`; the checks are then evaluated on the metrics.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence

from .checks import Check, CheckResult, CheckStatus, ConstraintStatus
from .runners import AnalysisRunner, AnalyzerContext


@dataclass
class VerificationResult:
    status: CheckStatus
    check_results: Dict[Check, CheckResult]
    metrics: Dict[object, object]

    @staticmethod
    def check_results_as_rows(result: "VerificationResult") -> List[dict]:
        """VerificationResult.checkResultsAsDataFrame columns: check, check_level,
        check_status, constraint, constraint_status, constraint_message."""
        rows = []
        for check, cr in result.check_results.items():
            for c in cr.constraint_results:
                rows.append({"check": check.description, "check_level": check.level.value,
                             "check_status": cr.status.name, "constraint": str(c.constraint),
                             "constraint_status": c.status.value,
                             "constraint_message": c.message or ""})
        return rows

    @staticmethod
    def success_metrics_as_rows(result: "VerificationResult", for_analyzers: Sequence = ()):
        return AnalyzerContext.success_metrics_as_rows(AnalyzerContext(result.metrics),
                                                       for_analyzers)


class VerificationSuite:
    def on_data(self, data) -> "VerificationRunBuilder":
        return VerificationRunBuilder(data)

    @staticmethod
    def do_verification_run(data, checks: Sequence[Check], required_analyzers: Sequence = (),
                            aggregate_with=None, save_states_with=None) -> VerificationResult:
        """VerificationSuite.doVerificationRun (VerificationSuite.scala:108-145)."""
        analyzers = list(required_analyzers)
        for c in checks:
            for a in c.required_analyzers():
                if a not in analyzers:
                    analyzers.append(a)
        ctx = AnalysisRunner.do_analysis_run(data, analyzers, aggregate_with, save_states_with)
        return VerificationSuite.evaluate(checks, ctx)

    @staticmethod
    def evaluate(checks: Sequence[Check], ctx: AnalyzerContext) -> VerificationResult:
        """VerificationSuite.evaluate (VerificationSuite.scala:264-282): overall status = the
        worst check status."""
        results = {c: c.evaluate(ctx) for c in checks}
        status = CheckStatus.Success
        for r in results.values():
            if r.status.value > status.value:
                status = r.status
        return VerificationResult(status, results, dict(ctx.metric_map))


@dataclass
class VerificationRunBuilder:
    """VerificationRunBuilder.scala:29-120 (checks, required analyzers, state loader/persister)."""
    data: object
    checks: List[Check] = field(default_factory=list)
    required_analyzers: List[object] = field(default_factory=list)
    _aggregate_with: object = None
    _save_states_with: object = None

    def add_check(self, check: Check) -> "VerificationRunBuilder":
        self.checks.append(check)
        return self

    def add_checks(self, checks: Sequence[Check]) -> "VerificationRunBuilder":
        self.checks.extend(checks)
        return self

    def add_required_analyzer(self, analyzer) -> "VerificationRunBuilder":
        self.required_analyzers.append(analyzer)
        return self

    def add_required_analyzers(self, analyzers) -> "VerificationRunBuilder":
        self.required_analyzers.extend(analyzers)
        return self

    def aggregate_with(self, loader) -> "VerificationRunBuilder":
        self._aggregate_with = loader
        return self

    def save_states_with(self, persister) -> "VerificationRunBuilder":
        self._save_states_with = persister
        return self

    def run(self) -> VerificationResult:
        return VerificationSuite.do_verification_run(self.data, self.checks,
                                                     self.required_analyzers,
                                                     self._aggregate_with, self._save_states_with)


__all__ = ["VerificationSuite", "VerificationResult", "VerificationRunBuilder",
           "ConstraintStatus"]
