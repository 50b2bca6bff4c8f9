"""deequ_amd -- an MI355X-native engine for deequ's metric-computation hot path.

The public surface mirrors deequ's (analyzers, states, AnalysisRunner, metrics); the computation
runs in hand-written HIP kernels behind a C ABI (include/deequ_amd.h, libdeequ_amd.so).
"""
from . import _native  # noqa: F401  -- fails loudly if the HIP engine is not built
from .analyzers import *  # noqa: F401,F403
from .metrics import (Distribution, DistributionValue, DoubleMetric, Entity, Failure,  # noqa: F401
                      HistogramMetric, KeyedDoubleMetric, Success)
from .runners import Analysis, AnalysisRunner, AnalyzerContext  # noqa: F401
from .table import Table  # noqa: F401
from .checks import Check, CheckLevel, CheckResult, CheckStatus, ConstraintStatus  # noqa: F401
from .verification import VerificationResult, VerificationSuite  # noqa: F401

__version__ = "0.1.0"
