"""GPU parity of DecimalType / DateType / TimestampType columns against the ORACLE
(oracle/deequ_oracle.py: Python's exact Decimal arithmetic, datetime values, the restated Spark 2.2
hash / cast-to-string) on seeded tables of several record batches.

  * the fused scan's decimal task (TK_DECIMAL): exact Sum (192-bit, checked word for word against
    the oracle's Decimal sum), Mean, Minimum / Maximum in the decimal order (AnalyzerTests.scala:
    454-470 is in the known-answer suite), StandardDeviation over the values' correctly rounded
    casts (1e-12), Completeness, with and without a where filter;
  * ApproxCountDistinct registers bit-exact (hashLong of the unscaled long for p <= 18,
    BigInteger.toByteArray bytes above; hashInt / hashLong of days / microseconds);
  * the grouping family and Histogram (keys = Spark's cast to string), DataType, PatternMatch and
    Compliance predicates (exact decimal comparisons), ApproxQuantile over the values as doubles.
Parity beyond the known answer rests on the oracle's restatement of Spark 2.2 (documented in
DESIGN.md; dates before 1582-10-15 and decimal sums that overflow inside one Spark partition are
unpinned)."""
import datetime
import math
import random
from decimal import Decimal

import pyarrow as pa
import pytest

from oracle import deequ_oracle as O

pytestmark = pytest.mark.gpu

C = O._DEC_CTX
EPOCH = datetime.datetime(1970, 1, 1)


def _dec(u, s):
    return Decimal(u).scaleb(-s, context=C)


def _data(n=9000, seed=5):
    rng = random.Random(seed)

    def nul(p):
        return rng.random() < p

    price = [None if nul(0.1) else _dec(rng.randint(-10 ** 9, 10 ** 9), 2) for _ in range(n)]
    # a low-cardinality decimal(38, 18) (groups repeat) with huge and tiny members
    # (|unscaled| < 10^33: the sum of 9000 stays inside decimal(38, 18); overflow has its own test)
    pool = [_dec(rng.randint(-10 ** 33, 10 ** 33), 18) for _ in range(40)] + \
           [_dec(v, 18) for v in (0, 1, -1, 5 * 10 ** 17, 99 * 10 ** 18)]
    big = [None if nul(0.05) else rng.choice(pool) for _ in range(n)]
    whole = [None if nul(0.05) else Decimal(rng.randint(-10 ** 30, 10 ** 30)) for _ in range(n)]
    day = [None if nul(0.05) else datetime.date(1970, 1, 1) + datetime.timedelta(days=rng.randint(-30000, 30000))
           for _ in range(n)]
    ts = [None if nul(0.05) else EPOCH + datetime.timedelta(
        microseconds=rng.randint(-2 * 10 ** 15, 2 * 10 ** 15) // rng.choice([1, 1000, 10 ** 6]))
        for _ in range(n)]
    x = [rng.randint(-5, 5) for _ in range(n)]
    cols = {"price": (price, pa.decimal128(10, 2), "decimal(10,2)"),
            "big": (big, pa.decimal128(38, 18), "decimal(38,18)"),
            "whole": (whole, pa.decimal128(31, 0), "decimal(31,0)"),
            "day": (day, pa.date32(), "date"),
            "ts": (ts, pa.timestamp("us"), "timestamp"),
            "x": (x, pa.int64(), "long")}
    at = pa.table({k: pa.array(v, type=t) for k, (v, t, _) in cols.items()})
    ot = O.OTable({k: v for k, (v, _, _) in cols.items()}, {k: o for k, (_, _, o) in cols.items()})
    return at, ot


@pytest.fixture(scope="module")
def tables(gpu_device):
    from deequ_amd import Table
    at, ot = _data()
    return Table.from_arrow(at, device=gpu_device, max_batch_rows=4096), ot


def _close(a, b, rel=1e-12):
    if a is None or b is None:
        return a is None and b is None
    return a == b or abs(a - b) <= rel * max(abs(a), abs(b))


def _metric(table, analyzer):
    m = analyzer.calculate(table)
    return m.value.get() if m.value.is_success else None


def _exact_sum_words(table, col, where=None):
    """The engine's exact decimal sum (dq_value.words[0..3], 256-bit two's complement)."""
    import ctypes
    from deequ_amd import _native as N
    from deequ_amd.analyzers.base import AggSpec
    from deequ_amd.runners.engine import get_plan, scan_into
    plan = get_plan(table.schema, [AggSpec(N.AGG_SUM, col=col, where=where)])
    st = plan.state(table.device_index())
    N.check(N.lib.dq_state_reset(st))
    scan_into(table, plan, st)
    N.check(N.lib.dq_state_sync(st))
    v = N.dq_value()
    N.check(N.lib.dq_state_get(st, 0, ctypes.byref(v)))
    w = sum(int(v.words[q]) << (64 * q) for q in range(4))
    return (w - (1 << 256) if w >> 255 else w), bool(v.is_null), float(v.f64[0])


@pytest.mark.parametrize("col", ["price", "big", "whole"])
@pytest.mark.parametrize("where", [None, "x > 0"])
def test_decimal_scan_aggregations(tables, col, where):
    from deequ_amd.analyzers import (Completeness, Maximum, Mean, Minimum, StandardDeviation, Sum)
    t, ot = tables
    sc = O.decimal_ps(ot.types[col])[1]
    # exact sum, word for word
    words, is_null, f = _exact_sum_words(t, col, where)
    exp = O.agg_sum_decimal(ot, col, where)
    assert is_null == (exp is None) and exp is not None
    assert words == O.unscaled(exp, sc)
    assert f == float(exp)
    assert _metric(t, Sum(col, where)) == O.agg_sum(ot, col, where)
    n_all = ot.n
    assert _metric(t, Mean(col, where)) == O.agg_sum(ot, col, where) / n_all
    assert _metric(t, Minimum(col, where)) == O.agg_min(ot, col, where)
    assert _metric(t, Maximum(col, where)) == O.agg_max(ot, col, where)
    n, avg, m2 = O.agg_stddev(ot, col, where)
    assert _close(_metric(t, StandardDeviation(col, where)), math.sqrt(m2 / n))
    num = O.agg_sum_notnull(ot, col, where)
    den = O.agg_conditional_count(ot, where)
    assert _metric(t, Completeness(col, where)) == num / den


def test_decimal_sum_overflow_is_an_empty_state(gpu_device):
    """A sum outside decimal(min(p + 10, 38), s) is NULL in Spark 2.2 (Cast's changePrecision): the
    Sum metric is then the empty-state failure, and Mean too."""
    from deequ_amd import Table
    from deequ_amd.analyzers import Mean, Sum
    from deequ_amd.exceptions import EmptyStateException
    vals = [Decimal(10 ** 37 + k) for k in range(20)]
    t = Table.from_arrow(pa.table({"v": pa.array(vals, type=pa.decimal128(38, 0))}), device=gpu_device)
    ot = O.OTable({"v": vals}, {"v": "decimal(38,0)"})
    assert O.agg_sum_decimal(ot, "v", None) is None
    for a in (Sum("v"), Mean("v")):
        m = a.calculate(t)
        assert m.value.is_failure and isinstance(m.value.failed, EmptyStateException)
    vals = [Decimal("99999999.99")] * 1000  # decimal(10, 2): the result type decimal(20, 2) holds it
    t = Table.from_arrow(pa.table({"v": pa.array(vals, type=pa.decimal128(10, 2))}), device=gpu_device)
    assert Sum("v").calculate(t).value.get() == 99999999990.0


@pytest.mark.parametrize("col", ["price", "big", "whole", "day", "ts"])
def test_hll_registers_bit_exact(tables, col):
    from deequ_amd.analyzers import ApproxCountDistinct
    t, ot = tables
    st = ApproxCountDistinct(col).compute_state_from(t)
    assert list(st.words) == O.agg_hll(ot, col, None)
    st = ApproxCountDistinct(col, "x >= 2").compute_state_from(t)
    assert list(st.words) == O.agg_hll(ot, col, "x >= 2")


@pytest.mark.parametrize("col", ["price", "big", "whole", "day", "ts"])
def test_grouping_family_and_histogram(tables, col):
    from deequ_amd.analyzers import (CountDistinct, Distinctness, Entropy, Histogram, Uniqueness,
                                     UniqueValueRatio)
    from deequ_amd.runners import AnalysisRunner
    t, ot = tables
    suite = [Uniqueness([col]), Distinctness([col]), UniqueValueRatio([col]), CountDistinct([col]),
             Entropy(col), Histogram(col)]
    ctx = AnalysisRunner.do_analysis_run(t, suite)
    freq = O.frequencies(ot, [col])
    assert ctx.metric(Uniqueness([col])).value.get() == O.uniqueness(freq, ot.n)
    assert ctx.metric(Distinctness([col])).value.get() == O.distinctness(freq, ot.n)
    assert ctx.metric(UniqueValueRatio([col])).value.get() == O.unique_value_ratio(freq)
    assert ctx.metric(CountDistinct([col])).value.get() == O.count_distinct(freq)
    assert _close(ctx.metric(Entropy(col)).value.get(), O.entropy(freq, ot.n))
    groups, _ = O.histogram(ot, col)
    d = ctx.metric(Histogram(col)).value.get()
    assert d.number_of_bins == len(groups)
    # the details: the top counts, every key Spark's cast to string with its exact count
    for key, dv in d.values.items():
        assert groups[key] == dv.absolute, key
    assert sorted((dv.absolute for dv in d.values.values()), reverse=True) == \
        sorted(groups.values(), reverse=True)[: len(d.values)]


@pytest.mark.parametrize("col", ["price", "big", "whole", "day", "ts"])
def test_datatype_over_the_cast_to_string(tables, col):
    from deequ_amd.analyzers import DataType
    t, ot = tables
    d = DataType(col).calculate(t).value.get()
    got = tuple(d.values[k].absolute for k in ("Unknown", "Fractional", "Integral", "Boolean", "String"))
    assert got == O.datatype_counts(ot, col, None)


@pytest.mark.parametrize("col,pattern", [("price", r"\.5"), ("big", r"E-"), ("big", r"^-?\d{3}\."),
                                         ("whole", r"7$"), ("day", r"^19[0-6]"), ("ts", r"\.\d{6}$"),
                                         ("ts", r" 00:00:00$")])
def test_pattern_match_over_the_cast_to_string(tables, col, pattern):
    from deequ_amd.analyzers import PatternMatch
    t, ot = tables
    hits, n = O.agg_pattern_match(ot, col, pattern, None)
    assert PatternMatch(col, pattern).calculate(t).value.get() == hits / n


@pytest.mark.parametrize("pred", ["price >= 10.5", "price < -1000000", "price = 0.01",
                                  "price IS NULL OR price IN (1.5, 2, -3.25)",
                                  "big > 0.5", "big <= -123.000000000000000001",
                                  "whole >= 1000000000000000000000000", "price > 1.5D",
                                  "day IS NULL", "ts IS NOT NULL AND big IS NULL"])
def test_compliance_predicates(tables, pred):
    from deequ_amd.analyzers import Compliance
    t, ot = tables
    num = O.agg_compliance(ot, pred, None)
    den = O.agg_conditional_count(ot, None)
    assert Compliance("c", pred).calculate(t).value.get() == num / den


def test_approx_quantile_over_decimal(tables):
    from deequ_amd.analyzers import ApproxQuantile
    t, ot = tables
    vals = [float(v) for v in ot.columns["price"] if v is not None]
    for q in (0.1, 0.5, 0.9):
        got = ApproxQuantile("price", q).calculate(t).value.get()
        assert got == O.spark_approx_quantile(vals, q)


def test_distributed_exchange_merges_decimal_states(gpu_device):
    """Rank-sharded decimal scans merged through the exchange's rank-ordered pass equal one scan of
    the whole table (exact sums / extremes; moments within 1e-12): host-only states stand for the
    ranks (the gloo world-2/3 byte-equality test is test_distributed_exchange_cpu.py)."""
    import ctypes
    from deequ_amd import Table
    from deequ_amd import _native as N
    from deequ_amd.analyzers import Maximum, Minimum, StandardDeviation, Sum
    from deequ_amd.distributed import merge_serialized, serialize_state
    from deequ_amd.runners.engine import get_plan, read_row, scan_into
    at, _ = _data(n=6000, seed=9)
    whole = Table.from_arrow(at, device=gpu_device, max_batch_rows=2048)
    specs = [s for a in (Sum("big"), Minimum("big"), Maximum("big"), StandardDeviation("big"))
             for s in a.aggregation_functions()]
    plan = get_plan(whole.schema, specs)
    images = []
    for lo in (0, 2048, 4096):
        part = whole.select_rows(lo, lo + 2048)
        st = plan.state(whole.device_index())
        N.check(N.lib.dq_state_reset(st))
        scan_into(part, plan, st)
        N.check(N.lib.dq_state_sync(st))
        images.append(serialize_state(plan, st))
    merged = merge_serialized(plan, images)
    st = plan.state(whole.device_index())
    N.check(N.lib.dq_state_reset(st))
    scan_into(whole, plan, st)
    one = read_row(plan, st)
    assert merged[:3] == one[:3]
    assert all(_close(a, b) for a, b in zip(merged[3], one[3]))
    del ctypes
