"""DecimalType / DateType / TimestampType on the host side (no GPU): the boundary's type words and
Arrow import, the shared conversions the device also runs (dq_decimal_to_double, dq_format_values:
decimal.h compiled for the host) against the oracle's independent restatements, the SQL typing of
decimal comparisons, and the plan's handling of the three types.

Reference: Analyzer.scala:277-278, 322-327 (DecimalType is numeric), AnalyzerTests.scala:454-470
(Minimum on a decimal(38,18) column = 99.0, in tests/golden/reference_known_answers.json), Spark
2.2's Decimal.toDouble / BigDecimal.toString / DateTimeUtils.dateToString / timestampToString
(restated in oracle/deequ_oracle.py; parity pinned by that known answer and by Python's exact
decimal arithmetic, not by further reference tests)."""
import datetime
import random
from decimal import Decimal

import pyarrow as pa
import pytest

from oracle import deequ_oracle as O

C = O._DEC_CTX


def test_decimal_type_word():
    from deequ_amd import _native as N
    t = N.decimal_type(38, 18)
    assert N.type_id(t) == N.DECIMAL128 and N.decimal_precision(t) == 38 and N.decimal_scale(t) == 18
    assert N.type_name(t) == "DecimalType(38,18)" and N.is_numeric(t)
    assert not N.is_numeric(N.DATE32) and N.type_name(N.TIMESTAMP_US) == "TimestampType"
    for p, s in ((0, 0), (39, 0), (10, 11)):
        with pytest.raises(ValueError):
            N.decimal_type(p, s)


def test_decimal_to_double_is_correctly_rounded():
    """The device's Cast(decimal AS DOUBLE) (decimal.h dec_to_double), run on the host, against
    Python's correctly rounded float(Decimal): random unscaled values of 8..126 bits at every
    scale, and exact halfway cases (ties to even)."""
    from deequ_amd import _native as N
    rng = random.Random(7)
    for _ in range(20000):
        sc = rng.randint(0, 38)
        u = rng.getrandbits(rng.choice([8, 30, 53, 54, 60, 64, 90, 100, 126]))
        u = -u if rng.random() < 0.5 else u
        if abs(u) >= 10 ** 38:
            continue
        assert N.decimal_to_double(u, sc) == float(Decimal(u).scaleb(-sc, context=C)), (u, sc)
    for _ in range(2000):  # halfway between two doubles: (2m + 1) 2^e with m of 53 bits
        m = rng.getrandbits(52) | (1 << 52)
        u = (2 * m + 1) << rng.randint(0, 70)
        if u < 10 ** 38:
            assert N.decimal_to_double(u, 0) == float(u)
    assert N.decimal_to_double(0, 18) == 0.0
    assert N.decimal_to_double(-(10 ** 38 - 1), 0) == -1e38


@pytest.mark.parametrize("sc", [0, 1, 2, 6, 7, 18, 38])
def test_decimal_text_is_bigdecimal_to_string(sc):
    from deequ_amd import _native as N
    vals = [0, 1, -1, 7, 12345, -12345, 10 ** 6, 99 * 10 ** 18, 10 ** 37, -(10 ** 38 - 1)]
    got = N.format_values(N.decimal_type(38, sc), vals)
    exp = [O.java_bigdecimal_to_string(Decimal(v).scaleb(-sc, context=C), sc) for v in vals]
    assert got == exp


def test_date_and_timestamp_text():
    from deequ_amd import _native as N
    days = [0, -1, 18000, 2932896, -719162, 11016, -25567]
    got = N.format_values(N.DATE32, days)
    exp = [O.java_date_to_string(datetime.date(1970, 1, 1) + datetime.timedelta(days=d)) for d in days]
    assert got == exp
    micros = [0, -1, 1500000, 1700000000123456, -62135596800000000, 951782400000010, -123456789]
    got = N.format_values(N.TIMESTAMP_US, micros)
    exp = [O.java_timestamp_to_string(datetime.datetime(1970, 1, 1) + datetime.timedelta(microseconds=m))
           for m in micros]
    assert got == exp
    assert got[2] == "1970-01-01 00:00:01.5" and got[0] == "1970-01-01 00:00:00"


def test_oracle_decimal_hash_is_biginteger_bytes():
    """XxHash64Function on a Decimal: hashLong(unscaled) for p <= 18, else hashUnsafeBytes of
    BigInteger.toByteArray -- the minimal big-endian two's complement (0 -> one 0x00 byte, 255 ->
    00 ff, -1 -> ff)."""
    import xxhash
    assert O.spark_xxhash64(Decimal("1.5"), "decimal(10,1)") == \
        xxhash.xxh64_intdigest((15).to_bytes(8, "little"), seed=42)
    for v, b in ((0, b"\x00"), (255, b"\x00\xff"), (-1, b"\xff"), (128, b"\x00\x80"), (-129, b"\xff\x7f")):
        assert O.spark_xxhash64(Decimal(v), "decimal(38,0)") == xxhash.xxh64_intdigest(b, seed=42)


def test_arrow_import_maps_spark_types_and_keeps_unsupported_columns():
    """Table.from_arrow reads decimal128 / date32 / date64 / timestamp (any unit) / binary, and a
    column of any other type no longer refuses the table: it imports validity-only (Completeness
    and Size still work, anything else is a WrongColumnTypeException)."""
    from deequ_amd import Table
    from deequ_amd import _native as N
    t = pa.table({
        "d": pa.array([Decimal("1.25"), None, Decimal("-3.50")], type=pa.decimal128(10, 2)),
        "day": pa.array([datetime.date(2020, 1, 2), None, datetime.date(1969, 12, 31)]),
        "ms": pa.array([0, 1500, None], type=pa.timestamp("ms", tz="UTC")),
        "b": pa.array([b"x", None, b"\xff"], type=pa.binary()),
        "l": pa.array([[1], None, []], type=pa.list_(pa.int64())),
    })
    tab = Table.from_arrow(t, device="cpu")
    f = {x.name: x for x in tab.schema.fields}
    assert f["d"].dtype == N.decimal_type(10, 2) and f["d"].type_name == "DecimalType(10,2)"
    assert f["day"].dtype == N.DATE32 and f["ms"].dtype == N.TIMESTAMP_US
    assert f["b"].dtype == N.UTF8 and f["b"].type_name == "BinaryType"
    assert f["l"].dtype == N.UNSUPPORTED and "list" in f["l"].type_name
    b = tab.batches[0]
    words = b["d"].values.numpy()
    assert words[:6].tolist() == [125, 0, 0, 0, (-350) & 0xFFFFFFFFFFFFFFFF, 0xFFFFFFFFFFFFFFFF]
    assert b["day"].values.numpy()[:3].tolist()[0] == 18263
    assert b["ms"].values.numpy()[:2].tolist() == [0, 1500000]  # milliseconds -> microseconds
    assert b["l"].stand_in and b["l"].validity is not None


def _plan(schema, analyzers):
    from deequ_amd.runners.engine import Plan
    return Plan(schema, [s for a in analyzers for s in a.aggregation_functions()])


def test_plan_puts_decimal_aggregations_in_one_decimal_task():
    from deequ_amd import _native as N
    from deequ_amd.analyzers import (ApproxCountDistinct, Completeness, Maximum, Mean, Minimum,
                                     StandardDeviation, Sum)
    from deequ_amd.table import StructField, StructType
    sch = StructType([StructField("m", N.decimal_type(38, 18)), StructField("day", N.DATE32)])
    p = _plan(sch, [Sum("m"), Mean("m"), Minimum("m"), Maximum("m"), StandardDeviation("m"),
                    Completeness("m"), ApproxCountDistinct("m"), ApproxCountDistinct("day"),
                    Completeness("day")])
    tasks = [ln.split()[1] for ln in p.explain().splitlines() if ln.startswith("task[")]
    assert tasks.count("decimal") == 1 and tasks.count("hll") == 2 and "numeric" not in tasks


def test_plan_refuses_what_the_engine_cannot_evaluate_exactly():
    from deequ_amd import _native as N
    from deequ_amd.analyzers import Compliance, Correlation, Sum
    from deequ_amd.exceptions import AnalysisException, WrongColumnTypeException
    from deequ_amd.table import StructField, StructType
    sch = StructType([StructField("m", N.decimal_type(12, 2)), StructField("x", N.INT64),
                      StructField("day", N.DATE32), StructField("l", N.UNSUPPORTED, None, "list")])
    with pytest.raises(N.EngineError):  # co-moments read Long / Double only
        _plan(sch, [Correlation("m", "x")])
    with pytest.raises(AnalysisException):  # Spark 2.2 compares a date with a string as text
        _plan(sch, [Compliance("c", "day >= '2020-01-01'")])
    with pytest.raises(WrongColumnTypeException):
        _plan(sch, [Sum("l")])
    _plan(sch, [Compliance("c", "day IS NULL OR m >= 0")])  # admitted


def test_decimal_comparisons_are_exact_at_the_column_scale():
    """Spark 2.2 DecimalPrecision: a decimal column against an integral / decimal literal compares
    exactly; the host rescales the literal to the column's scale (x_unscaled OP t 10^s, a
    non-integral bound replaced by its floor / ceiling) and emits DQ_X_DEC128 words."""
    from deequ_amd import _native as N
    from deequ_amd.sqlexpr import compile_expr
    from deequ_amd.table import StructField, StructType
    sch = StructType([StructField("p", N.decimal_type(10, 2)), StructField("f", N.FLOAT64)])
    idx = {"p": 0, "f": 1}.__getitem__

    def words(sql):
        return compile_expr(sql, sch, idx).words

    assert words("p >= 0") == [N.X_GE, N.X_COL, 0, N.X_DEC128, 0, 0]
    assert words("p < 1.005") == [N.X_LE, N.X_COL, 0, N.X_DEC128, 100, 0]
    assert words("p > 1.005") == [N.X_GE, N.X_COL, 0, N.X_DEC128, 101, 0]
    assert words("-2.5 < p") == [N.X_GT, N.X_COL, 0, N.X_DEC128, -250, -1]
    lim = 10 ** 38
    assert words("p = 1.005") == [N.X_EQ, N.X_COL, 0, N.X_DEC128, lim & (2 ** 64 - 1) - (1 << 64)
                                  if (lim & (2 ** 64 - 1)) >= 1 << 63 else lim & (2 ** 64 - 1),
                                  lim >> 64]
    # against a double (D suffix) or a double column: Cast(decimal AS DOUBLE)
    assert words("p > 1.5D")[:3] == [N.X_GT, N.X_CAST_F64, N.X_COL]
    assert words("p IN (1.5, 2, NULL)") == [N.X_IN, 3, N.X_COL, 0, N.X_DEC128, 150, 0,
                                           N.X_DEC128, 200, 0, N.X_NULL]


def test_oracle_decimal_sum_overflow_is_null():
    """Spark 2.2 Sum over decimal(p, s) returns decimal(min(p + 10, 38), s): NULL when it does not
    fit (Cast's changePrecision)."""
    t = O.OTable({"v": [Decimal(10 ** 37)] * 20}, {"v": "decimal(38,0)"})
    assert O.agg_sum_decimal(t, "v", None) is None
    t = O.OTable({"v": [Decimal("99999999.99")] * 3}, {"v": "decimal(10,2)"})
    assert O.agg_sum_decimal(t, "v", None) == Decimal("299999999.97")
