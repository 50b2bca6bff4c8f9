"""Single-column profiling (reference: profiles/ColumnProfiler.scala:80-230, 510-600,
ColumnProfile.scala, ColumnProfilerRunner.scala, ColumnProfilerRunBuilder.scala) in three device
passes, each one fused scan or group-by of the engine:

  pass 1  Size + per column Completeness + ApproxCountDistinct (+ DataType for strings): one fused
          scan; the inferred type of a string column is DataTypeHistogram.determineType.
  pass 2  Minimum / Maximum / Mean / StandardDeviation / Sum / ApproxQuantiles(0.01 .. 1.00) of the
          numeric columns -- string columns inferred Integral / Fractional are first cast on the
          device (dq_cast_utf8, Spark 2.2 Cast semantics): one fused scan + the quantile sorts.
  pass 3  exact histograms (every value, NULL -> "NullValue") of the string columns inferred String
          with at most `low_cardinality_histogram_threshold` approximate distinct values: one
          device group-by per column.

As in the reference, `columns` empty means pass 1 over every column and NO profiles (passes 2 and
3 and the profiles themselves are taken over `columns`; ColumnProfiler.scala:175-195, 562).
"""
from __future__ import annotations

import ctypes
import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from . import _native as N
from .analyzers import (ApproxCountDistinct, ApproxQuantiles, Completeness, DataType, Histogram,
                        Maximum, Mean, Minimum, Size, StandardDeviation, Sum)
from .analyzers.datatype import DataTypeInstances, determine_type
from .exceptions import HllBiasTablesUnavailableException, ReusingNotPossibleResultsMissingException
from .metrics import Distribution, DistributionValue, HistogramMetric, Success
from .runners import AnalysisRunBuilder, AnalyzerContext

DEFAULT_CARDINALITY_THRESHOLD = 120


@dataclass
class StandardColumnProfile:
    column: str
    completeness: float
    approximate_num_distinct_values: Optional[int]  # None: HLL++ bias range, no tables
    data_type: DataTypeInstances
    is_data_type_inferred: bool
    type_counts: Dict[str, int]
    histogram: Optional[Distribution]


@dataclass
class NumericColumnProfile(StandardColumnProfile):
    mean: Optional[float] = None
    maximum: Optional[float] = None
    minimum: Optional[float] = None
    sum: Optional[float] = None
    std_dev: Optional[float] = None
    approx_percentiles: Optional[List[float]] = None


@dataclass
class ColumnProfiles:
    profiles: Dict[str, StandardColumnProfile]
    num_records: int

    @staticmethod
    def to_json(column_profiles: Sequence[StandardColumnProfile]) -> str:
        """ColumnProfiles.toJson (ColumnProfile.scala:66-150), Gson pretty printing."""
        cols = []
        for p in column_profiles:
            j = {"column": p.column, "dataType": p.data_type.name,
                 "isDataTypeInferred": str(p.is_data_type_inferred).lower(),
                 "completeness": p.completeness,
                 "approximateNumDistinctValues": p.approximate_num_distinct_values}
            if p.histogram is not None:
                j["histogram"] = [{"value": k, "count": v.absolute, "ratio": v.ratio}
                                  for k, v in p.histogram.values.items()]
            if isinstance(p, NumericColumnProfile):
                for key, v in (("mean", p.mean), ("maximum", p.maximum), ("minimum", p.minimum),
                               ("sum", p.sum), ("stdDev", p.std_dev)):
                    if v is not None:
                        j[key] = v
                j["approxPercentiles"] = list(p.approx_percentiles or [])
            cols.append(j)
        return json.dumps({"columns": cols}, indent=2)


@dataclass
class _GenericStatistics:
    num_records: int
    inferred_types: Dict[str, DataTypeInstances]
    known_types: Dict[str, DataTypeInstances]
    type_detection_histograms: Dict[str, Dict[str, int]]
    approximate_num_distincts: Dict[str, Optional[int]]
    completenesses: Dict[str, float]

    def type_of(self, column: str) -> DataTypeInstances:
        merged = dict(self.inferred_types)
        merged.update(self.known_types)
        return merged[column]


def _known_type(dtype: int, spark_name: str = "") -> DataTypeInstances:
    # ColumnProfiler.scala:374-381: ShortType | LongType | IntegerType -> Integral;
    # DecimalType() | FloatType | DoubleType -> Fractional; BooleanType -> Boolean;
    # TimestampType -> String; anything else (ByteType, DateType, BinaryType ...) is
    # "Unable to map" -> Unknown
    if spark_name == "BinaryType":
        return DataTypeInstances.Unknown
    if dtype in (N.INT16, N.INT32, N.INT64):
        return DataTypeInstances.Integral
    if dtype in (N.FLOAT32, N.FLOAT64) or N.is_decimal(dtype):
        return DataTypeInstances.Fractional
    if dtype == N.BOOL:
        return DataTypeInstances.Boolean
    if dtype == N.TIMESTAMP_US:
        return DataTypeInstances.String
    return DataTypeInstances.Unknown


class ColumnProfiler:
    DEFAULT_CARDINALITY_THRESHOLD = DEFAULT_CARDINALITY_THRESHOLD

    @staticmethod
    def profile(data, columns: Sequence[str] = (), print_status_updates: bool = False,
                low_cardinality_histogram_threshold: int = DEFAULT_CARDINALITY_THRESHOLD,
                metrics_repository=None, reuse_existing_results_using_key=None,
                fail_if_results_for_reusing_missing: bool = False,
                save_in_metrics_repository_using_key=None) -> ColumnProfiles:
        columns = list(columns)
        names = data.schema.field_names
        for c in columns:
            if c not in names:
                raise ValueError(f"requirement failed: Unable to find column {c}")
        repo = (metrics_repository, reuse_existing_results_using_key,
                fail_if_results_for_reusing_missing, save_in_metrics_repository_using_key)

        # pass 1
        if print_status_updates:
            print("### PROFILING: Computing generic column statistics in pass (1/3)...")
        first = []
        for f in data.schema.fields:
            if columns and f.name not in columns:
                continue
            first += [Completeness(f.name), ApproxCountDistinct(f.name)]
            if f.type_name == "StringType":
                first.append(DataType(f.name))
        builder = AnalysisRunBuilder(data).add_analyzers(first).add_analyzer(Size())
        first_results = _with_repository(builder, *repo).run()
        generic = _extract_generic_statistics(columns, data.schema, first_results)

        # pass 2
        if print_status_updates:
            print("### PROFILING: Computing numeric column statistics in pass (2/3)...")
        casted = _cast_numeric_string_columns(columns, data, generic)
        percentiles = [k / 100 for k in range(1, 101)]
        second = []
        for name in columns:
            if generic.type_of(name) in (DataTypeInstances.Integral, DataTypeInstances.Fractional):
                second += [Minimum(name), Maximum(name), Mean(name), StandardDeviation(name),
                           Sum(name), ApproxQuantiles(name, percentiles)]
        builder = AnalysisRunBuilder(casted).add_analyzers(second)
        second_results = _with_repository(builder, *repo).run()
        numeric = _extract_numeric_statistics(second_results)

        # pass 3
        if print_status_updates:
            print("### PROFILING: Computing histograms of low-cardinality columns in pass (3/3)...")
        targets = _target_columns_for_histograms(data.schema, generic,
                                                 low_cardinality_histogram_threshold)
        existing = AnalyzerContext.empty()
        if metrics_repository is not None and reuse_existing_results_using_key is not None:
            prev = metrics_repository.load_by_key(reuse_existing_results_using_key)
            if prev is not None:
                existing = AnalyzerContext({
                    a: m for a, m in prev.metric_map.items()
                    if isinstance(a, Histogram) and a.column in targets and Histogram(a.column) == a})
        missing = [c for c in targets if existing.metric(Histogram(c)) is None]
        if missing:
            if fail_if_results_for_reusing_missing:
                raise ReusingNotPossibleResultsMissingException(
                    "Could not find all necessary results in the MetricsRepository, the calculation "
                    f"of the histograms for these columns would be required: {', '.join(missing)}")
            dists = _compute_histograms(data, missing)
            ctx = AnalyzerContext({Histogram(c): HistogramMetric(c, Success(d))
                                   for c, d in dists.items()}) + existing
            if metrics_repository is not None and save_in_metrics_repository_using_key is not None:
                cur = (metrics_repository.load_by_key(save_in_metrics_repository_using_key)
                       or AnalyzerContext.empty())
                metrics_repository.save(save_in_metrics_repository_using_key, cur + ctx)
        else:
            if print_status_updates:
                print("### PROFILING: Skipping pass (3/3), no new histograms need to be calculated.")
            ctx = existing
        histograms = {a.column: m.value.get() for a, m in ctx.metric_map.items()
                      if isinstance(a, Histogram) and m.value.is_success}
        return _create_profiles(columns, generic, numeric, histograms)


def _with_repository(builder, repository, reuse_key, fail_if_missing, save_key):
    if repository is not None:
        builder = builder.use_repository(repository)
        if reuse_key is not None:
            builder = builder.reuse_existing_results_for_key(reuse_key, fail_if_missing)
        if save_key is not None:
            builder = builder.save_or_append_result(save_key)
    return builder


def _extract_generic_statistics(columns, schema, results) -> _GenericStatistics:
    num_records = None
    inferred, hists, distincts, compl = {}, {}, {}, {}
    for a, m in results.metric_map.items():
        if isinstance(a, Size):
            num_records = int(m.value.get())
        elif isinstance(a, DataType):
            dist = m.value.get()
            inferred[a.column] = determine_type(dist)
            hists[a.column] = {k: v.absolute for k, v in dist.values.items()}
        elif isinstance(a, ApproxCountDistinct):
            if not m.value.is_success and isinstance(m.value.failed,
                                                     HllBiasTablesUnavailableException):
                distincts[a.column] = None  # unavailable: HLL++ bias range (see below)
            else:
                distincts[a.column] = int(m.value.get())  # Double.toLong truncates
        elif isinstance(a, Completeness):
            compl[a.column] = m.value.get()
    known = {f.name: _known_type(f.dtype, f.type_name) for f in schema.fields
             if f.name in columns and f.type_name != "StringType"}
    return _GenericStatistics(num_records, inferred, known, hists, distincts, compl)


def _cast_column(data, name: str, to_type: int):
    """castColumn (ColumnProfiler.scala:311-320): the column replaced by its device cast."""
    import torch
    from .table import ColumnBatch, StructField, StructType, Table
    batches = []
    for b in data.batches:
        c = b[name]
        values = N.retry_on_oom(torch.empty, max(c.length, 1), device=data.device,
                                dtype=torch.int64 if to_type == N.INT64 else torch.float64)
        validity = N.retry_on_oom(torch.empty, max((c.length + 7) // 8, 1), dtype=torch.uint8,
                                  device=data.device)
        bad = ctypes.c_int64()
        stream = ctypes.c_void_p(torch.cuda.current_stream(data.device).cuda_stream)
        col = c.to_c()
        N.check(N.lib.dq_cast_utf8(ctypes.byref(col), to_type, values.data_ptr(),
                                   validity.data_ptr(), ctypes.byref(bad), stream))
        if bad.value:
            raise NotImplementedError(
                f"cast of column {name} to double: {bad.value} value(s) need parseDouble forms "
                "(exponent / NaN / Infinity / > 19 significant digits) this build does not convert")
        nb = dict(b)
        nb[name] = ColumnBatch(to_type, c.length, validity, values, None, 0)
        batches.append(nb)
    fields = [StructField(f.name, to_type if f.name == name else f.dtype)
              for f in data.schema.fields]
    return Table(StructType(fields), batches, data.device)


def _cast_numeric_string_columns(columns, data, generic):
    out = data
    for name in columns:
        if data.schema[name].type_name != "StringType":
            continue  # a cast of a numeric column to long / double leaves every metric unchanged
        t = generic.type_of(name)
        if t == DataTypeInstances.Integral:
            out = _cast_column(out, name, N.INT64)
        elif t == DataTypeInstances.Fractional:
            out = _cast_column(out, name, N.FLOAT64)
    return out


@dataclass
class _NumericStatistics:
    means: Dict[str, float] = field(default_factory=dict)
    std_devs: Dict[str, float] = field(default_factory=dict)
    minima: Dict[str, float] = field(default_factory=dict)
    maxima: Dict[str, float] = field(default_factory=dict)
    sums: Dict[str, float] = field(default_factory=dict)
    approx_percentiles: Dict[str, List[float]] = field(default_factory=dict)


def _extract_numeric_statistics(results) -> _NumericStatistics:
    s = _NumericStatistics()
    slots = {Mean: s.means, StandardDeviation: s.std_devs, Maximum: s.maxima, Minimum: s.minima,
             Sum: s.sums}
    for a, m in results.metric_map.items():
        if not m.value.is_success:
            continue
        if isinstance(a, ApproxQuantiles):
            s.approx_percentiles[a.column] = sorted(m.value.get().values())
        elif type(a) in slots:
            slots[type(a)][a.column] = m.value.get()
    return s


def _target_columns_for_histograms(schema, generic, threshold) -> List[str]:
    """getHistogramsOfLowCardinalityColumns' selection (ColumnProfiler.scala:416-433).  A column
    whose ApproxCountDistinct fell in the HLL++ bias range has no number here (Spark's bias tables
    are missing, HllBiasTablesUnavailableException), but there linear counting already puts it
    above LINEAR_COUNTING_FLOOR distinct values: it is not a target for any threshold below that,
    and a larger threshold cannot be decided without the tables (raised, never guessed)."""
    strings = {f.name for f in schema.fields if f.type_name == "StringType"}
    out = []
    for c, n in generic.approximate_num_distincts.items():
        if c not in strings or generic.type_of(c) != DataTypeInstances.String:
            continue
        if n is None:
            if threshold >= HllBiasTablesUnavailableException.LINEAR_COUNTING_FLOOR:
                raise HllBiasTablesUnavailableException(
                    f"column {c}: its approximate distinct count lies in the HLL++ bias-correction "
                    f"range, so it cannot be compared with a histogram threshold of {threshold}")
            continue
        if n <= threshold:
            out.append(c)
    return out


def _compute_histograms(data, targets) -> Dict[str, Distribution]:
    """computeHistograms (ColumnProfiler.scala:505-545): every value of each target column,
    NULL -> "NullValue", ratio = count / rows; numberOfBins = #values."""
    out = {}
    for col in targets:
        state = Histogram(col).compute_state_from(data)
        groups = state.string_groups()
        total = sum(groups.values())
        values = {k: DistributionValue(c, c / total) for k, c in groups.items()}
        out[col] = Distribution(values, len(values))
    return out


def _create_profiles(columns, generic, numeric, histograms) -> ColumnProfiles:
    profiles = {}
    for name in columns:
        t = generic.type_of(name)
        base = dict(column=name, completeness=generic.completenesses[name],
                    approximate_num_distinct_values=generic.approximate_num_distincts[name],
                    data_type=t, is_data_type_inferred=name in generic.inferred_types,
                    type_counts=generic.type_detection_histograms.get(name, {}),
                    histogram=histograms.get(name))
        if t in (DataTypeInstances.Integral, DataTypeInstances.Fractional):
            profiles[name] = NumericColumnProfile(
                **base, mean=numeric.means.get(name), maximum=numeric.maxima.get(name),
                minimum=numeric.minima.get(name), sum=numeric.sums.get(name),
                std_dev=numeric.std_devs.get(name),
                approx_percentiles=numeric.approx_percentiles.get(name))
        else:
            profiles[name] = StandardColumnProfile(**base)
    return ColumnProfiles(profiles, generic.num_records)


class ColumnProfilerRunBuilder:
    """ColumnProfilerRunBuilder.scala (file outputs: to a local path)."""

    def __init__(self, data):
        self.data = data
        self._columns: Optional[List[str]] = None
        self._threshold = DEFAULT_CARDINALITY_THRESHOLD
        self._print = False
        self._repository = None
        self._reuse_key = None
        self._fail_if_missing = False
        self._save_key = None
        self._json_path: Optional[str] = None
        self._overwrite = False

    def print_status_updates(self, flag: bool):
        self._print = flag
        return self

    def cache_inputs(self, _flag: bool):  # the table is already resident in HBM
        return self

    def with_low_cardinality_histogram_threshold(self, threshold: int):
        self._threshold = threshold
        return self

    def only_consider_column_subset(self, columns: Sequence[str]):
        self._columns = list(columns)
        return self

    def use_repository(self, repository):
        self._repository = repository
        return self

    def reuse_existing_results_for_key(self, key, fail_if_results_missing: bool = False):
        self._reuse_key = key
        self._fail_if_missing = fail_if_results_missing
        return self

    def save_or_append_result(self, key):
        self._save_key = key
        return self

    def save_column_profiles_json_to_path(self, path: str):
        self._json_path = path
        return self

    def overwrite_previous_files(self, flag: bool):
        self._overwrite = flag
        return self

    def run(self) -> ColumnProfiles:
        profiles = ColumnProfiler.profile(
            self.data, self._columns or [], self._print, self._threshold, self._repository,
            self._reuse_key, self._fail_if_missing, self._save_key)
        if self._json_path is not None:
            import os
            if os.path.exists(self._json_path) and not self._overwrite:
                raise FileExistsError(f"{self._json_path} already exists")
            with open(self._json_path, "w") as fh:
                fh.write(ColumnProfiles.to_json(list(profiles.profiles.values())) + "\n")
        return profiles


class ColumnProfilerRunner:
    def on_data(self, data) -> ColumnProfilerRunBuilder:
        return ColumnProfilerRunBuilder(data)


__all__ = ["ColumnProfiler", "ColumnProfilerRunner", "ColumnProfilerRunBuilder", "ColumnProfiles",
           "StandardColumnProfile", "NumericColumnProfile", "DEFAULT_CARDINALITY_THRESHOLD"]
