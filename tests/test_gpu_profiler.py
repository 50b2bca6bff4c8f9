"""ColumnProfiler (profiles/ColumnProfiler.scala) on the GPU against the reference's own tests
(T/profiles/ColumnProfilerTest.scala:14-131, ColumnProfilerRunnerTest.scala:35-66) and the device
string cast (dq_cast_utf8, Spark 2.2 Cast semantics) against a host restatement."""
import math

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

PERCENTILES = [1.0] + [2.0] * 32 + [3.0] * 17 + [4.0] * 16 + [5.0] * 17 + [6.0] * 17


def _df_complete_and_incomplete(device):
    from deequ_amd.table import Table
    return Table.from_pydict({"item": ["1", "2", "3", "4", "5", "6"],
                              "att1": ["a", "b", "a", "a", "b", "a"],
                              "att2": ["f", "d", None, "f", None, "f"]},
                             {"item": "string", "att1": "string", "att2": "string"}, device=device)


def test_standard_column_profile(gpu_device):
    """ColumnProfilerTest.scala:14-36"""
    from deequ_amd.analyzers.datatype import DataTypeInstances
    from deequ_amd.profiles import ColumnProfiler, StandardColumnProfile
    p = ColumnProfiler.profile(_df_complete_and_incomplete(gpu_device), ["att2"], False, 1)
    assert p.profiles["att2"] == StandardColumnProfile(
        "att2", 2.0 / 3.0, 2, DataTypeInstances.String, True,
        {"Boolean": 0, "Fractional": 0, "Integral": 0, "Unknown": 2, "String": 4}, None)
    assert p.num_records == 6


def test_numeric_profile_of_a_numeric_string_column(gpu_device):
    """ColumnProfilerTest.scala:38-73: "item" holds "1".."6", inferred Integral, cast on the device."""
    from deequ_amd.analyzers.datatype import DataTypeInstances
    from deequ_amd.profiles import ColumnProfiler, NumericColumnProfile
    p = ColumnProfiler.profile(_df_complete_and_incomplete(gpu_device), ["item"], False, 1)
    assert p.profiles["item"] == NumericColumnProfile(
        "item", 1.0, 6, DataTypeInstances.Integral, True,
        {"Boolean": 0, "Fractional": 0, "Integral": 6, "Unknown": 0, "String": 0}, None,
        3.5, 6.0, 1.0, 21.0, 1.707825127659933, PERCENTILES)


def test_numeric_profile_of_a_double_column(gpu_device):
    """ColumnProfilerTest.scala:75-104 (getDfWithNumericFractionalValues)."""
    from deequ_amd.analyzers.datatype import DataTypeInstances
    from deequ_amd.profiles import ColumnProfiler, NumericColumnProfile
    from deequ_amd.table import Table
    data = Table.from_pydict({"item": ["1", "2", "3", "4", "5", "6"],
                              "att1": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0],
                              "att2": [0.0, 0.0, 0.0, 5.0, 6.0, 7.0]},
                             {"item": "string", "att1": "float64", "att2": "float64"},
                             device=gpu_device)
    p = ColumnProfiler.profile(data, ["att1"], False, 1)
    assert p.profiles["att1"] == NumericColumnProfile(
        "att1", 1.0, 6, DataTypeInstances.Fractional, False, {}, None,
        3.5, 6.0, 1.0, 21.0, 1.707825127659933, PERCENTILES)


def test_histograms_of_low_cardinality_columns(gpu_device):
    """ColumnProfilerTest.scala:106-132"""
    from deequ_amd.analyzers.datatype import DataTypeInstances
    from deequ_amd.metrics import Distribution, DistributionValue
    from deequ_amd.profiles import ColumnProfiler, StandardColumnProfile
    p = ColumnProfiler.profile(_df_complete_and_incomplete(gpu_device), ["att2"], False, 10)
    assert p.profiles["att2"] == StandardColumnProfile(
        "att2", 2.0 / 3.0, 2, DataTypeInstances.String, True,
        {"Boolean": 0, "Fractional": 0, "Integral": 0, "Unknown": 2, "String": 4},
        Distribution({"d": DistributionValue(1, 0.16666666666666666),
                      "f": DistributionValue(3, 0.5),
                      "NullValue": DistributionValue(2, 0.3333333333333333)}, 3))


def test_runner_saves_and_reuses_results(gpu_device, tmp_path):
    """ColumnProfilerRunnerTest.scala:35-66: a second run reusing the saved key computes nothing
    (fail_if_results_missing would raise otherwise) and returns the same profiles; the JSON file is
    written (ColumnProfilerRunner.scala:95-113)."""
    from deequ_amd.profiles import ColumnProfilerRunner
    from deequ_amd.repository import InMemoryMetricsRepository, ResultKey
    data = _df_complete_and_incomplete(gpu_device)
    repo, key = InMemoryMetricsRepository(), ResultKey(0, {})
    cols = ["item", "att1", "att2"]
    first = (ColumnProfilerRunner().on_data(data).only_consider_column_subset(cols)
             .use_repository(repo).save_or_append_result(key).run())
    again = (ColumnProfilerRunner().on_data(data).only_consider_column_subset(cols)
             .use_repository(repo).reuse_existing_results_for_key(key, True)
             .save_column_profiles_json_to_path(str(tmp_path / "p.json")).run())
    assert first == again
    assert (tmp_path / "p.json").read_text().count('"column"') == 3
    assert ColumnProfilerRunner().on_data(data).run().profiles == {}  # no subset: no profiles


def _spark_to_long(s):
    """UTF8String.toLong (Spark 2.2), restated for the test."""
    b = s.encode()
    if not b:
        return None
    neg = b[:1] == b"-"
    i = 1 if b[:1] in (b"-", b"+") else 0
    if i and len(b) == 1:
        return None
    ip, _, fp = b[i:].partition(b".")
    if not all(48 <= c <= 57 for c in ip) or not all(48 <= c <= 57 for c in fp):
        return None
    v = int(ip) if ip else 0
    v = -v if neg else v
    return v if -(1 << 63) <= v < (1 << 63) else None


def _java_parse_double(s):
    t = s.strip("".join(chr(c) for c in range(33)))
    body = t[1:] if t[:1] in "+-" else t
    if not body or body.count(".") > 1 or not all(c.isdigit() or c == "." for c in body) \
            or not any(c.isdigit() for c in body):
        return None
    return float(t)


def test_device_string_cast_matches_spark_semantics(gpu_device):
    from deequ_amd import _native as N
    from deequ_amd.profiles import _cast_column
    from deequ_amd.table import Table
    rng = np.random.default_rng(5)
    vals = ["1", "-2", "+3", "", "-", "+", "4.5", "4.", ".5", "-.25", "1.2.3", " 7", "7 ", "- 8",
            "9223372036854775807", "9223372036854775808", "-9223372036854775808", "12a", "0.000",
            "-0", "00012.3400", "123456789012345678", "0.1", "3.14159", None, "1e5", "NaN"]
    vals += [str(int(x)) for x in rng.integers(-10**12, 10**12, 300)]
    vals += [f"{x:.{int(d)}f}" for x, d in zip(rng.normal(0, 1e4, 300), rng.integers(0, 9, 300))]
    t = pa.table({"s": pa.array(vals, type=pa.string())})
    data = Table.from_arrow(t, device=gpu_device, max_batch_rows=128)
    as_long = _cast_column(data, "s", N.INT64)
    got = [v for b in as_long.batches for v in _to_list(b["s"], np.int64)]
    assert got == [None if v is None else _spark_to_long(v) for v in vals]
    # (> 15 digits or an exponent: parseDouble forms the device path reports, tested below)
    ok = [v for v in vals if v is None or ("e" not in v and "N" not in v
                                           and sum(c.isdigit() for c in v) <= 15)]
    data2 = Table.from_arrow(pa.table({"s": pa.array(ok, type=pa.string())}), device=gpu_device)
    as_dbl = _cast_column(data2, "s", N.FLOAT64)
    got = [v for b in as_dbl.batches for v in _to_list(b["s"], np.float64)]
    exp = [None if v is None else _java_parse_double(v) for v in ok]
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        assert (g is None and e is None) or (g == e and math.copysign(1, g) == math.copysign(1, e))
    with pytest.raises(NotImplementedError):  # exponent forms: loud, never a guess
        _cast_column(data, "s", N.FLOAT64)


def _to_list(col, dt):
    v = col.values.cpu().numpy().view(dt)[: col.length]
    bits = np.unpackbits(col.validity.cpu().numpy(), bitorder="little")[: col.length]
    return [x.item() if b else None for x, b in zip(v, bits)]


def test_success_metrics_json_known_answer(gpu_device):
    """SimpleResultSerdeTest (T/repository/AnalysisResultSerdeTest.scala:176-222): the success
    metrics of an analysis over getDfFull as JSON rows with the dataset date and the tag."""
    import json
    from deequ_amd.analyzers import Completeness, Distinctness, MutualInformation, Size, Uniqueness
    from deequ_amd.repository import AnalysisResult, ResultKey, success_metrics_as_json
    from deequ_amd.runners import Analysis
    from deequ_amd.table import Table
    df = Table.from_pydict({"item": ["1", "2", "3", "4"], "att1": ["a", "a", "a", "b"],
                            "att2": ["c", "c", "c", "d"]},
                           {"item": "string", "att1": "string", "att2": "string"}, device=gpu_device)
    ctx = Analysis([Size(), Distinctness("item"), Completeness("att1"), Uniqueness("att1"),
                    Distinctness("att1"), Completeness("att2"), Uniqueness("att2"),
                    MutualInformation("att1", "att2")]).run(df)
    got = json.loads(success_metrics_as_json(AnalysisResult(ResultKey(1507975810, {"Region": "EU"}),
                                                             ctx)))
    exp = [("Column", "att2", "Completeness", 1.0), ("Column", "att1", "Completeness", 1.0),
           ("Column", "att2", "Uniqueness", 0.25), ("Column", "item", "Distinctness", 1.0),
           ("Dataset", "*", "Size", 4.0), ("Column", "att1", "Uniqueness", 0.25),
           ("Column", "att1", "Distinctness", 0.5),
           ("Mutlicolumn", "att1,att2", "MutualInformation", 0.5623351446188083)]
    want = sorted({"dataset_date": 1507975810, "entity": e, "region": "EU", "instance": i,
                   "name": n, "value": v}.items() for e, i, n, v in exp)
    assert sorted(sorted(r.items()) for r in got) == sorted(sorted(w) for w in want)


def test_profile_of_a_column_in_the_hll_bias_range(gpu_device):
    """About 1000 distinct values put ApproxCountDistinct in HLL++'s bias-correction range (Spark's
    BIAS_DATA tables are absent): the profile still completes, the column's distinct count is
    reported as unavailable (None) instead of a different number, it is not a histogram target
    at the default threshold (linear counting already exceeds 400), and a low-cardinality column
    next to it is profiled as usual."""
    from deequ_amd.profiles import ColumnProfiler
    from deequ_amd.table import Table
    n = 5000
    df = Table.from_pydict({"ids": [f"k{i % 1000}" for i in range(n)],
                            "low": ["ab"[i % 2] for i in range(n)]},
                           {"ids": "string", "low": "string"}, device=gpu_device)
    p = ColumnProfiler.profile(df, ["ids", "low"])
    assert p.num_records == n
    assert p.profiles["ids"].approximate_num_distinct_values is None
    assert p.profiles["ids"].histogram is None
    assert p.profiles["low"].approximate_num_distinct_values == 2
    assert set(p.profiles["low"].histogram.values) == {"a", "b"}
    from deequ_amd.exceptions import HllBiasTablesUnavailableException
    with pytest.raises(HllBiasTablesUnavailableException):
        ColumnProfiler.profile(df, ["ids", "low"], low_cardinality_histogram_threshold=500)
