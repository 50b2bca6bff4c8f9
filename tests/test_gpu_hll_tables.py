"""ApproxCountDistinct's HLL++ registers from a frequency table's records (dq_freq_hll; the runner
takes them from a column's Histogram table instead of scanning it).  The
registers depend only on the set of distinct non-NULL values (StatefulHyperloglogPlus.scala:87-113),
so the table's records (each distinct value at least once) must give the scan's register words bit for bit, for every key type: the
exact-mode values recovered from the bijective hash (int8..int64, boolean, float32 / float64 with
NaN payloads, -0.0 and infinities -- Spark hashes doubleToLongBits / floatToIntBits), and utf8
keys from the arena (empty strings, a real "NullValue", multibyte characters)."""
import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


def _columns(n, seed):
    rng = np.random.default_rng(seed)
    mask = rng.random(n) < 0.06
    small = rng.integers(-300, 300, n)
    f64 = np.where(rng.random(n) < 0.5, small * 0.25, rng.choice(
        np.array([np.inf, -np.inf, 0.0, -0.0, 1.5]), n))
    bits = f64.view(np.uint64).copy()
    bits[::101] = 0x7ff8000000000123  # NaN payloads: one canonical NaN for HLL
    bits[1::101] = 0xfff0000000000001
    f64 = bits.view(np.float64)
    f32 = f64.astype(np.float32)
    words = ["", "NullValue", "é", "a", "b", "ccc", "twelve bytes", "a" * 40, "漢字"]
    return {
        "i64": pa.array(small * 1_000_003, mask=mask, type=pa.int64()),
        "i32": pa.array(small, mask=mask, type=pa.int32()),
        "i16": pa.array(small, mask=mask, type=pa.int16()),
        "i8": pa.array(small % 100, mask=mask, type=pa.int8()),
        "b": pa.array(small > 0, mask=mask, type=pa.bool_()),
        "f64": pa.array(f64, mask=mask, type=pa.float64()),
        "f32": pa.array(f32, mask=mask, type=pa.float32()),
        "s": pa.array([None if m else words[v % len(words)] for v, m in zip(small, mask)],
                      pa.string()),
    }


@pytest.mark.parametrize("null_as_group", [False, True])
def test_table_registers_equal_the_scan(null_as_group, gpu_device):
    from deequ_amd.analyzers import ApproxCountDistinct
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.table import Table
    from oracle import deequ_oracle as O
    cols = _columns(40_003, 3)
    t = pa.table(cols)
    df = Table.from_arrow(t, device=gpu_device, max_batch_rows=9000)
    ot = O.OTable({c: t.column(c).to_pylist() for c in cols},
                  {"i64": "long", "i32": "int", "i16": "short", "i8": "byte", "b": "boolean",
                   "f64": "double", "f32": "float", "s": "string"})
    for c in cols:
        ft = FrequencyTable([c], [df.schema[c].dtype], 0)
        for b in df.batches:
            ft.add([b[c]], null_as_group=null_as_group)
        words = ft.hll_words(1 << 20)
        assert words is not None, c
        scan = ApproxCountDistinct(c).compute_state_from(df)
        assert words == tuple(scan.words), c
        assert [w & ((1 << 64) - 1) for w in words] == \
            [w & ((1 << 64) - 1) for w in O.agg_hll(ot, c, None)], c
        assert ft.hll_words(1) is None  # more records than allowed: the caller scans


def test_runner_takes_registers_from_histogram_tables(gpu_device, monkeypatch):
    """AnalysisRunner over ApproxCountDistinct + Histogram of low-cardinality columns: the same
    metrics with the registers from the Histogram tables as with the scan (DQ_HLL_FROM_TABLE=0),
    and high-cardinality columns keep their scan (a record per row: hashing the records would
    cost as much as the scan)."""
    from deequ_amd.analyzers import ApproxCountDistinct, Histogram, Uniqueness
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    cols = _columns(70_001, 8)
    cols["hi"] = pa.array(np.arange(70_001, dtype=np.int64))
    cols["hs"] = pa.array([f"key {i}" for i in range(70_001)])
    df = Table.from_arrow(pa.table(cols), device=gpu_device, max_batch_rows=30_000)
    names = ["i64", "i32", "b", "s", "hi", "hs"]
    suite = [a for c in names for a in (ApproxCountDistinct(c), Histogram(c), Uniqueness([c]))]
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.metrics import Distribution
    taken = {}
    orig = FrequencyTable.hll_words

    def spy(self, max_records):  # which tables gave their registers
        w = orig(self, max_records)
        taken[self.key_columns[0]] = w is not None
        return w
    monkeypatch.setattr(FrequencyTable, "hll_words", spy)
    got = AnalysisRunner.do_analysis_run(df, suite)
    # low-cardinality tables collapse to a few records (the small-key path: one per group);
    # a record per row keeps the scan
    assert taken["b"] and taken["s"] and not taken["hi"] and not taken["hs"], taken
    monkeypatch.setenv("DQ_HLL_FROM_TABLE", "0")
    ref = AnalysisRunner.do_analysis_run(df, suite)

    def same(m1, m2):  # (a Failure holds an exception object: compare its message)
        v1, v2 = m1.value, m2.value
        if v1.is_success and v2.is_success:
            if isinstance(m1.value.get(), Distribution):  # top-k ties come in any order
                d1, d2 = m1.value.get(), m2.value.get()
                return (d1.number_of_bins == d2.number_of_bins and
                        sorted(v.absolute for v in d1.values.values()) ==
                        sorted(v.absolute for v in d2.values.values()))
            return m1 == m2
        return (not v1.is_success and not v2.is_success
                and type(v1.failed) is type(v2.failed) and str(v1.failed) == str(v2.failed))
    for a in suite:
        assert same(got.metric(a), ref.metric(a)), str(a)
