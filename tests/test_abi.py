"""CPU tests of the C ABI (no compute calls): the library loads, exports every symbol the header
declares, plans compile (planning is host code), and host helpers agree with independent
implementations."""
import ctypes
import os
import re
import struct
import subprocess

import pytest
import xxhash

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "deequ_amd.h")).read()
    return sorted(set(re.findall(r"\b(dq_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from deequ_amd import _native as N
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (dq_[a-z0-9_]+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    assert set(N.EXPORTED) <= exported


def test_version_and_device_count_callable_without_gpu():
    from deequ_amd import _native as N
    assert N.lib.dq_version() == 100
    assert N.device_count() >= 0


@pytest.mark.parametrize("data", [b"", b"a", b"high", b"0123456789abcdef" * 5, "ünï".encode()])
def test_engine_xxhash_matches_package(data):
    from deequ_amd import _native as N
    assert N.xxhash64(data, 42) == xxhash.xxh64_intdigest(data, seed=42)


def _table(cols, types):
    from deequ_amd import _native as N
    from deequ_amd.table import StructField, StructType
    return StructType([StructField(c, t) for c, t in zip(cols, types)])


def test_s10_plan_fuses_into_four_tasks_and_two_launches():
    from deequ_amd import _native as N
    from deequ_amd.analyzers import (Completeness, Compliance, Maximum, Mean, Minimum, Size,
                                     StandardDeviation, Sum)
    from deequ_amd.runners.engine import Plan
    schema = _table(["id", "name", "priority", "numViews"], [N.INT64, N.UTF8, N.UTF8, N.INT64])
    suite = [Size(), Completeness("id"), Completeness("name"),
             Compliance("numViews is non-negative", "numViews >= 0"),
             Compliance("priority contained in high,low",
                        "priority IS NULL OR priority IN ('high','low')"),
             Sum("numViews"), Mean("numViews"), StandardDeviation("numViews"),
             Minimum("numViews"), Maximum("numViews")]
    specs = [s for a in suite for s in a.aggregation_functions()]
    plan = Plan(schema, specs)
    text = plan.explain()
    assert text.count("task[") == 4, text
    assert "numeric col=3" in text and "str_in col=2" in text
    # ONE mixed scan launch for the three body classes (validity, numeric int64, string IN) + the
    # finalize launch
    assert plan.launches_per_batch == 2


def test_where_filters_materialise_once_per_distinct_expression():
    from deequ_amd import _native as N
    from deequ_amd.analyzers import Completeness, Maximum, Minimum
    from deequ_amd.runners.engine import Plan
    schema = _table(["item", "att1"], [N.UTF8, N.INT32])
    suite = [Completeness("att1", "item IN ('1','2')"), Minimum("att1", "item IN ('1','2')"),
             Maximum("att1", "item != '6'")]
    plan = Plan(schema, [s for a in suite for s in a.aggregation_functions()])
    text = plan.explain()
    assert text.count("expr[") == 2, text


def test_bad_expression_is_an_analysis_error():
    from deequ_amd import _native as N
    from deequ_amd.analyzers import Compliance
    from deequ_amd.exceptions import AnalysisException
    from deequ_amd.runners.engine import Plan
    schema = _table(["att1"], [N.INT32])
    with pytest.raises(AnalysisException):
        Plan(schema, Compliance("r", "attNoSuchColumn > 3").aggregation_functions())


@pytest.mark.parametrize("operand", ["column", "literal"])
def test_plan_refuses_cast_of_a_string_to_float(operand):
    """DQ_X_CAST_F32 over a utf8 column or a string literal: Spark's Float.parseFloat is not
    restated, so dq_plan_create refuses it (a C-ABI caller cannot bypass sqlexpr's check)."""
    import ctypes
    import struct
    from deequ_amd import _native as N
    x = [N.X_COL, 0] if operand == "column" else [N.X_STR, 3, int.from_bytes(b"1.5", "little")]
    one = struct.unpack("<q", struct.pack("<d", 1.0))[0]
    words = [N.X_GT, N.X_CAST_F32] + x + [N.X_F64, one]
    buf = (ctypes.c_int64 * len(words))(*words)
    expr = (N.dq_expr * 1)()
    expr[0].words = ctypes.cast(buf, ctypes.POINTER(ctypes.c_int64))
    expr[0].n_words = len(words)
    agg = N.dq_agg()
    agg.kind, agg.col, agg.col2, agg.expr, agg.where = N.AGG_COUNT_TRUE, -1, -1, 0, -1
    aggs = (N.dq_agg * 1)(agg)
    types = (ctypes.c_int32 * 1)(N.UTF8)
    desc = N.dq_plan_desc()
    desc.n_columns, desc.column_types, desc.n_exprs, desc.exprs = 1, types, 1, expr
    desc.n_aggs, desc.aggs = 1, aggs
    handle = ctypes.c_void_p()
    assert N.lib.dq_plan_create(ctypes.byref(desc), ctypes.byref(handle)) == N.ERR_UNSUPPORTED
    assert b"FLOAT" in N.lib.dq_last_error()
    # the same cast of an integral column plans
    types[0] = N.INT64
    words[2:2 + len(x)] = [N.X_COL, 0]
    buf = (ctypes.c_int64 * len(words))(*words)
    expr[0].words = ctypes.cast(buf, ctypes.POINTER(ctypes.c_int64))
    expr[0].n_words = len(words)
    assert N.lib.dq_plan_create(ctypes.byref(desc), ctypes.byref(handle)) == 0
    N.lib.dq_plan_destroy(handle)


def test_hll_count_matches_oracle_on_random_registers():
    import random
    from deequ_amd import _native as N
    from oracle import deequ_oracle as O
    rng = random.Random(5)
    for trial in range(50):
        regs = [rng.choice([0] * trial + list(range(1, 12))) for _ in range(512)]
        words = O.hll_words(regs)
        assert N.hll_count(words) == O.hll_count(words)


def test_approx_count_distinct_in_bias_range_is_a_failure_not_a_wrong_number():
    """~1000 distinct values: E < 5M and no linear counting, where the reference subtracts Spark's
    empirical bias (StatefulHyperloglogPlus.scala:235-237); those tables are absent, so the metric
    must fail loudly (HllBiasTablesUnavailableException) instead of returning the raw estimate."""
    from deequ_amd.analyzers import ApproxCountDistinct
    from deequ_amd.analyzers.scan import ApproxCountDistinctState
    from deequ_amd.exceptions import HllBiasTablesUnavailableException
    from oracle import deequ_oracle as O
    words = tuple(O.hll_words(O.hll_registers(list(range(1000)), "long")))
    assert O.hll_count(words)[1]
    m = ApproxCountDistinct("c").compute_metric_from(ApproxCountDistinctState(words))
    assert m.value.is_failure
    assert isinstance(m.value.exception, HllBiasTablesUnavailableException)
    small = tuple(O.hll_words(O.hll_registers(list(range(50)), "long")))
    assert ApproxCountDistinct("c").compute_metric_from(ApproxCountDistinctState(small)).value.get() \
        == O.hll_count(small)[0]


@pytest.mark.parametrize("offset", [0, 8, 3, 13])
def test_sliced_arrow_arrays_import_at_their_offset(offset):
    """dq_column_from_arrow honours ArrowArray.offset (a sliced Spark partition export): values
    and utf8 offsets aliased at the first row, bitmaps at a bit offset re-based to bit 0 (host
    buffers here; the device path is in test_gpu_loader.py)."""
    import ctypes

    import numpy as np
    import pyarrow as pa

    from deequ_amd.loader import ArrowColumn
    rng = np.random.default_rng(offset)
    n = 200
    mask = rng.random(n) < 0.3
    cases = [pa.array(rng.integers(-99, 99, n), mask=mask, type=pa.int64()),
             pa.array(rng.normal(size=n).astype(np.float32), mask=mask, type=pa.float32()),
             pa.array(rng.integers(-9, 9, n).astype(np.int16), mask=mask, type=pa.int16()),
             pa.array(rng.random(n) < 0.5, mask=mask, type=pa.bool_()),
             pa.array([None if m else "x" * (k % 5) for k, m in enumerate(mask)], pa.string())]
    length = n - offset - 7
    for arr in cases:
        sl = arr.slice(offset, length)
        col = ArrowColumn(sl)
        c = col.to_c()
        assert c.length == length
        bits = lambda ptr, k: np.unpackbits(  # noqa: E731
            np.frombuffer(ctypes.string_at(ptr, (k + 7) // 8), np.uint8), bitorder="little")[:k]
        valid = np.array([x is not None for x in sl.to_pylist()])
        assert (bits(c.validity, length).astype(bool) == valid).all(), str(arr.type)
        if pa.types.is_boolean(arr.type):
            got = bits(c.values, length).astype(bool)
            exp = np.array([bool(x) for x in sl.fill_null(False).to_pylist()])
            assert (got[valid] == exp[valid]).all()
        elif pa.types.is_string(arr.type):
            offs = np.frombuffer(ctypes.string_at(c.values, 4 * (length + 1)), np.int32)
            data = ctypes.string_at(c.data, int(offs[-1]))
            got = [data[offs[k]:offs[k + 1]].decode() for k in range(length)]
            assert [g for g, v in zip(got, valid) if v] == [x for x in sl.to_pylist() if x is not None]
        else:
            npt = arr.type.to_pandas_dtype()
            w = np.dtype(npt).itemsize
            got = np.frombuffer(ctypes.string_at(c.values, w * length), npt)
            exp = np.asarray(arr.to_numpy(zero_copy_only=False))[offset:offset + length]
            assert (got[valid] == exp[valid]).all()
        del col
