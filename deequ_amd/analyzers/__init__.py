"""Analyzers mirroring com.amazon.deequ.analyzers (the hot-path subset)."""
from .base import (AggSpec, Analyzer, DoubleValuedState, GroupingAnalyzer, NumMatchesAndCount,
                   Preconditions, ScanShareableAnalyzer, StandardScanShareableAnalyzer, State,
                   merge_states)
from .grouping import (CountDistinct, Distinctness, Entropy, FrequenciesAndNumRows,
                       FrequencyBasedAnalyzer, FrequencyTable, Histogram, HistogramState,
                       MutualInformation,
                       ScanShareableFrequencyBasedAnalyzer, UniqueValueRatio, Uniqueness,
                       compute_frequencies)
from .scan import (ApproxCountDistinct, ApproxCountDistinctState, Completeness, Compliance,
                   Correlation, CorrelationState, MaxState, Maximum, Mean, MeanState, MinState,
                   Minimum, NumMatches, PatternMatch, Patterns, Size, StandardDeviation,
                   StandardDeviationState, Sum, SumState)
from .datatype import DataType, DataTypeHistogram, DataTypeInstances, determine_type
from .quantile import ApproxQuantile, ApproxQuantiles, ApproxQuantileState, QuantileSummaries
from .state_provider import HdfsStateProvider, InMemoryStateProvider, StateLoader, StatePersister
