"""Deterministic inputs for the committed golden vectors (tests/golden/vectors.json).

numpy's PCG64 stream is stable across numpy releases, so a (n, seed, null_rate) triple fully
determines a table; the fixture stores only the triple plus the expected outputs.  Columns:
a int64, b float64, c int32, s utf8 (incl. "" and "NullValue"), each with i.i.d. NULLs.
"""
import numpy as np
import pyarrow as pa

TYPES = {"a": "long", "b": "double", "c": "int", "s": "string"}
CATS = ["high", "low", "medium", "", "NullValue", "x" * 20, "Thingy A", "Thingy B"]

# (name, n, seed, null_rate, batch_rows)
CASES = [
    ("n1e3_p0", 1000, 101, 0.0, None),
    ("n1e4_p5", 10_000, 102, 0.05, 4096),
    ("n1e4_p100", 10_000, 103, 1.0, None),
    ("n3e4_p30", 30_011, 104, 0.3, 8192),
]

WHERE = "c > -20"

# scan aggregations the fixture pins: (key, kind, column(s) / predicate, where)
SCAN_AGGS = [
    ("size", "count", None, None),
    ("size_w", "count", None, WHERE),
    ("compl_a", "notnull", "a", None),
    ("compl_s_w", "notnull", "s", WHERE),
    ("nonneg_a", "compliance", "a >= 0", None),
    ("in_s", "compliance", "s IS NULL OR s IN ('high','low')", None),
    ("range_b", "compliance", "b IS NULL OR (b >= 900.0 AND b <= 1100.0)", None),
    ("lt_c_w", "compliance", "c < 10", WHERE),
    ("gt_ac", "compliance", "a > c", None),
    ("sum_a", "sum", "a", None),
    ("sum_c_w", "sum", "c", WHERE),
    ("min_a", "min", "a", None),
    ("max_a", "max", "a", None),
    ("min_b", "min", "b", None),
    ("max_c_w", "max", "c", WHERE),
    ("sd_a", "stddev", "a", None),
    ("sd_b", "stddev", "b", None),
    ("corr_ab", "corr", ("a", "b"), None),
    ("hll_a", "hll", "a", None),
    ("hll_s", "hll", "s", None),
    ("hll_b_w", "hll", "b", WHERE),
]

FREQ_COLS = [["a"], ["c"], ["s"]]


def golden_table(n: int, seed: int, null_rate: float) -> pa.Table:
    rng = np.random.default_rng(seed)

    def mask():
        return rng.random(n) < null_rate

    a = rng.integers(-10 ** 6, 10 ** 6, n)
    a[:: 7] = a[:: 7] % 500          # repeated keys for the frequency family
    b = rng.normal(1000.0, 250.0, n)
    c = rng.integers(-50, 50, n).astype(np.int32)
    s = np.array(CATS)[rng.integers(0, len(CATS), n)]
    ms = mask()
    return pa.table({
        "a": pa.array(a, mask=mask(), type=pa.int64()),
        "b": pa.array(b, mask=mask(), type=pa.float64()),
        "c": pa.array(c, mask=mask(), type=pa.int32()),
        "s": pa.array([None if m else v for v, m in zip(s.tolist(), ms)], type=pa.string()),
    })


# XXH64 (seed 42) vector inputs per Spark type; the fixture stores the digests.
XXH_INPUTS = {
    "int": [0, 1, -1, 42, 2 ** 31 - 1, -2 ** 31, 123456789],
    "long": [0, 1, -1, 42, 2 ** 63 - 1, -2 ** 63, 1 << 40, -987654321012],
    "double": [0.0, -0.0, 1.0, -1.5, 3.141592653589793, 1e300, float("inf"), float("-inf"),
               float("nan")],
    "string": ["", "a", "high", "low", "medium", "NullValue", "Thingy 1234",
               "http://example.com/x", "héllo wörld", "x" * 100],
}
