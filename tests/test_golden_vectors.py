"""Committed golden vectors (tests/golden/vectors.json, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every vector (it is the checker, so it must be stable), and the
XXH64 seed-42 vectors agree with the independent `xxhash` package.
GPU: the HIP path, called through the C ABI, reproduces every vector -- counts, Long sums,
min/max, HLL register words and frequency counts bit-exact; Welford / co-moment states and
Entropy within 1e-12 relative (north_star).
"""
import json
import math
import os
import struct

import pytest

from golden_inputs import CASES, FREQ_COLS, SCAN_AGGS, golden_table

HERE = os.path.dirname(os.path.abspath(__file__))
REL = 1e-12
GOLD = json.load(open(os.path.join(HERE, "golden", "vectors.json")))
CASE_NAMES = [c[0] for c in CASES]
CASE_BY_NAME = {c[0]: c for c in CASES}


def _close(a, b, rel=REL):
    if a is None or b is None:
        return a is b
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b or abs(a - b) <= rel * max(abs(a), abs(b))


def _same(a, b):
    """Exact equality that treats NaN == NaN."""
    if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
        return True
    return a == b


# ------------------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", CASE_NAMES)
def test_oracle_reproduces_golden_vectors(name):
    import make_golden_shim as mg
    _, n, seed, null_rate, _ = CASE_BY_NAME[name]
    ot = mg.oracle_table(golden_table(n, seed, null_rate))
    case = GOLD["cases"][name]
    for key, kind, arg, where in SCAN_AGGS:
        got = mg.scan_expected(ot, kind, arg, where)
        exp = case["scan"][key]
        if isinstance(exp, list):
            assert all(_same(float(x), float(y)) for x, y in zip(got, exp)), key
        else:
            assert _same(got, exp), (key, got, exp)
    for cols in FREQ_COLS:
        assert mg.freq_expected(ot, cols) == case["freq"][",".join(cols)]


def test_oracle_reproduces_high_register_hll_vectors():
    """Registers 29..56: count() shifts a Scala Int by the register (StatefulHyperloglogPlus.
    scala:220), so registers >= 31 do not contribute 2^-m (the fixture pins that restatement)."""
    import make_golden_shim as mg
    from oracle import deequ_oracle as O
    for regs, exp in zip(mg.hll_high_register_sets(), GOLD["hll_high_registers"]):
        words = O.hll_words(regs)
        assert [int(w) for w in words] == exp["words"]
        assert O.hll_count(words) == (exp["estimate"], exp["bias_corrected"])
    col = GOLD["hll_high_rank_column"]
    assert mg.high_rank_column_expected() == col


def test_engine_hll_count_matches_high_register_vectors():
    from deequ_amd import _native as N
    for exp in GOLD["hll_high_registers"] + [GOLD["hll_high_rank_column"]]:
        assert N.hll_count(exp["words"]) == (exp["estimate"], exp["bias_corrected"])


def test_high_rank_longs_hash_to_their_ranks():
    xxhash = pytest.importorskip("xxhash")
    for v, pw, idx in GOLD["hll_high_rank_column"]["high_rank_longs"]:
        h = xxhash.xxh64_intdigest(struct.pack("<q", v), seed=42)
        w = ((h << 9) & (2 ** 64 - 1)) | (1 << 8)
        assert (64 - w.bit_length() + 1, h >> 55) == (pw, idx)


@pytest.mark.parametrize("ty", ["int", "long", "double", "string"])
def test_golden_xxh64_matches_xxhash_package(ty):
    xxhash = pytest.importorskip("xxhash")
    for v, h in GOLD["xxh64_seed42"][ty]:
        if ty == "int":
            b = struct.pack("<i", v)
        elif ty == "long":
            b = struct.pack("<q", v)
        elif ty == "double":
            v = float(v)
            b = struct.pack("<d", float("nan") if math.isnan(v) else v)
            if math.isnan(v):   # Spark canonicalises NaN (doubleToLongBits)
                b = struct.pack("<Q", 0x7FF8000000000000)
        else:
            b = v.encode("utf-8")
        d = xxhash.xxh64_intdigest(b, seed=42)
        assert d == h, (ty, v)


# ------------------------------------------------------------------------------------------- GPU
def _scan_analyzer(kind, arg, where):
    from deequ_amd.analyzers import (ApproxCountDistinct, Completeness, Compliance, Correlation,
                                     Maximum, Minimum, Size, StandardDeviation, Sum)
    return {
        "count": lambda: Size(where),
        "notnull": lambda: Completeness(arg, where),
        "compliance": lambda: Compliance("golden", arg, where),
        "sum": lambda: Sum(arg, where),
        "min": lambda: Minimum(arg, where),
        "max": lambda: Maximum(arg, where),
        "stddev": lambda: StandardDeviation(arg, where),
        "corr": lambda: Correlation(arg[0], arg[1], where),
        "hll": lambda: ApproxCountDistinct(arg, where),
    }[kind]()


def _state_value(kind, st):
    if st is None:
        return None
    if kind in ("count", "notnull", "compliance"):
        return st.num_matches
    if kind == "sum":
        return st.sum_value
    if kind == "min":
        return st.min_value
    if kind == "max":
        return st.max_value
    if kind == "stddev":
        return [st.n, st.avg, st.m2]
    if kind == "corr":
        return [st.n, st.x_avg, st.y_avg, st.ck, st.x_mk, st.y_mk]
    if kind == "hll":
        return list(st.words)
    raise ValueError(kind)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASE_NAMES)
def test_hip_scan_reproduces_golden_vectors(name, gpu_device):
    from deequ_amd import Analysis, Table
    from deequ_amd.runners.engine import run_scan
    _, n, seed, null_rate, batch = CASE_BY_NAME[name]
    df = Table.from_arrow(golden_table(n, seed, null_rate), device=gpu_device,
                          max_batch_rows=batch)
    case = GOLD["cases"][name]
    analyzers = [_scan_analyzer(kind, arg, where) for _, kind, arg, where in SCAN_AGGS]
    Analysis(analyzers).run(df)     # the fused suite runs as one plan
    for (key, kind, arg, where), a in zip(SCAN_AGGS, analyzers):
        st = a.from_aggregation_result(run_scan(df, a.aggregation_functions()), 0)
        got, exp = _state_value(kind, st), case["scan"][key]
        if kind in ("notnull", "compliance") and where is not None and case["scan"]["size_w"] is None:
            # conditionalCount(where) is NULL when every `where` is NULL -> ifNoNullsIn gives None
            # (Analyzer.scala:365-379, 404-408); the fixture holds the numerator alone
            assert st is None, key
            continue
        if kind == "hll":
            assert got == exp["words"], key
            m = a.compute_metric_from(st)
            if exp["bias_corrected"]:   # needs Spark's BIAS_DATA tables: a loud failure
                assert m.value.is_failure, key
            else:
                assert m.value.get() == exp["estimate"], (key, m.value.get(), exp["estimate"])
        elif kind == "count" and where is None:
            assert got == exp
        elif kind in ("stddev", "corr"):
            if exp[0] == 0:
                assert got is None, key
            else:
                assert got[0] == exp[0], key
                assert all(_close(float(g), float(e)) for g, e in zip(got[1:], exp[1:])), \
                    (key, got, exp)
        else:
            assert _same(got, exp), (key, got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASE_NAMES)
def test_hip_frequency_reproduces_golden_vectors(name, gpu_device):
    from deequ_amd import Table
    from deequ_amd.analyzers import (CountDistinct, Distinctness, Entropy, Histogram,
                                     UniqueValueRatio, Uniqueness)
    from deequ_amd.runners import AnalysisRunner
    _, n, seed, null_rate, batch = CASE_BY_NAME[name]
    df = Table.from_arrow(golden_table(n, seed, null_rate), device=gpu_device,
                          max_batch_rows=batch)
    case = GOLD["cases"][name]
    analyzers = []
    for cols in FREQ_COLS:
        c = tuple(cols)
        analyzers += [Uniqueness(c), Distinctness(c), UniqueValueRatio(c), CountDistinct(c)]
        if len(c) == 1:     # Entropy(column: String), Entropy.scala:28
            analyzers.append(Entropy(c[0]))
    analyzers += [Histogram("c"), Histogram("s")]
    ctx = AnalysisRunner.do_analysis_run(df, analyzers)
    for cols in FREQ_COLS:
        c = tuple(cols)
        exp = case["freq"][",".join(cols)]
        pairs = [(Uniqueness(c), exp["uniqueness"]), (Distinctness(c), exp["distinctness"]),
                 (UniqueValueRatio(c), exp["unique_value_ratio"]),
                 (CountDistinct(c), exp["count_distinct"])]
        for a, v in pairs:
            m = ctx.metric(a)
            if v is None:
                assert m.value.is_failure, str(a)
            else:
                assert m.value.get() == v, (str(a), m.value.get(), v)
        if len(c) > 1:
            continue
        m = ctx.metric(Entropy(c[0]))
        if exp["entropy"] is None:
            assert m.value.is_failure
        else:
            assert _close(m.value.get(), exp["entropy"]), (cols, m.value.get(), exp["entropy"])
    for col in ("c", "s"):
        exp = case["histogram"][col]
        dist = ctx.metric(Histogram(col)).value.get()
        assert dist.number_of_bins == exp["bins"]
        got = {k: v.absolute for k, v in dist.values.items()}
        if exp["bins"] <= 1000:
            assert got == exp["counts"], col
        for k, v in dist.values.items():
            assert v.ratio == v.absolute / exp["num_rows"]



@pytest.mark.gpu
@pytest.mark.parametrize("batch", [None, 1000])
def test_hip_hll_registers_at_rank_31_and_above(batch, gpu_device):
    """Rows whose hash has rank 31..39 -- what a 1e9-row column produces: the HIP registers and the
    estimate (with count()'s Int-shift, StatefulHyperloglogPlus.scala:220) equal the fixture."""
    import pyarrow as pa
    from deequ_amd import Table
    from deequ_amd.analyzers import ApproxCountDistinct
    col = GOLD["hll_high_rank_column"]
    values = list(range(4090)) + [v for v, _, _ in col["high_rank_longs"]]
    df = Table.from_arrow(pa.table({"id": pa.array(values, pa.int64())}), device=gpu_device,
                          max_batch_rows=batch)
    a = ApproxCountDistinct("id")
    st = a.compute_state_from(df)
    assert list(st.words) == col["words"]
    regs = [(w >> (6 * i)) & 0x3F for w in (x & (2 ** 64 - 1) for x in st.words) for i in range(10)]
    assert max(regs) == 39
    assert a.calculate(df).value.get() == col["estimate"]
