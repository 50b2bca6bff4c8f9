"""The C/OpenMP frequency restatement (oracle/oracle.c or_freq, the configs[2] / configs[4] CPU
baseline) against the pure-Python oracle: groups, Σ[c==1], entropy and Histogram's top-k, over
int64 and utf8 keys, NULLs skipped (grouping) or a group of their own merged with a real
"NullValue" string (Histogram.scala:59-66).  CPU only."""
import math

import numpy as np
import pyarrow as pa
import pytest

from oracle import c_oracle as C
from oracle import deequ_oracle as O


def _buffers(arr):
    arr = arr.combine_chunks() if isinstance(arr, pa.ChunkedArray) else arr
    bufs = arr.buffers()
    n = len(arr)
    valid = (np.frombuffer(bufs[0], np.uint8).copy() if bufs[0] is not None
             else np.full((n + 7) // 8, 0xFF, np.uint8))
    if pa.types.is_string(arr.type):
        off = np.frombuffer(bufs[1], np.int32)[: n + 1].copy()
        data = np.frombuffer(bufs[2], np.uint8).copy() if bufs[2] is not None else np.zeros(1, np.uint8)
        return off, data, valid
    return np.frombuffer(bufs[1], np.int64)[:n].copy(), None, valid


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("kind", ["long", "string"])
def test_c_frequency_family_matches_python_oracle(kind, threads):
    rng = np.random.default_rng(7 + threads)
    n = 30_000
    ids = rng.integers(0, n // 3, n)
    mask = rng.random(n) < 0.05
    if kind == "long":
        arr = pa.array(ids, mask=mask, type=pa.int64())
    else:
        words = np.array([f"w{v}" for v in ids], dtype=object)
        words[::97] = "NullValue"
        arr = pa.array([None if m else str(w) for w, m in zip(words, mask)], type=pa.string())
    t = O.OTable({"k": arr.to_pylist()}, {"k": kind})
    values, data, valid = _buffers(arr)
    out, _, _ = C.freq(kind, values, data, valid, n, n, threads=threads)
    freq = O.frequencies(t, ["k"])
    assert out.groups == len(freq)
    assert out.unique == sum(1 for c in freq.values() if c == 1)
    assert out.null_rows == int(mask.sum())
    ent = -math.fsum((c / n) * math.log(c / n) for c in freq.values())
    assert abs(out.entropy - ent) <= 1e-12 * ent
    # Histogram: NULL -> "NullValue" (merged with a real one), top-k by count
    hout, tc, tr = C.freq(kind, values, data, valid, n, n, null_as_group=True, k=50, threads=threads)
    hist, _ = O.histogram(t, "k")
    assert hout.groups == len(hist)
    assert list(tc) == sorted(hist.values(), reverse=True)[:50]
    vals = arr.to_pylist()
    for c, r in zip(tc, tr):
        key = "NullValue" if r < 0 or vals[r] is None else O.java_to_string(vals[r], kind)
        assert hist[key] == c


@pytest.mark.parametrize("threads", [1, 5])
def test_c_double_column_aggregates_match_python_oracle(threads):
    """or_numeric_f64 (the configs[4] CPU baseline's double columns) against the Python oracle."""
    rng = np.random.default_rng(threads)
    n = 20_000
    vals = rng.normal(3.0, 7.0, n)
    mask = rng.random(n) < 0.05
    arr = pa.array(vals, mask=mask, type=pa.float64())
    v = np.frombuffer(arr.buffers()[1], np.float64)[:n].copy()
    valid = np.frombuffer(arr.buffers()[0], np.uint8).copy()
    got = C.numeric_f64(v, valid, 0.0, threads)
    py = [None if m else float(x) for x, m in zip(vals, mask)]
    t = O.OTable({"x": py}, {"x": "double"})
    nn, avg, m2 = O.agg_stddev(t, "x", None)
    assert got.count == sum(x is not None for x in py)
    assert got.min == O.agg_min(t, "x", None) and got.max == O.agg_max(t, "x", None)
    assert abs(got.sum - math.fsum(x for x in py if x is not None)) <= 1e-9 * abs(got.sum)
    assert got.n == nn and abs(got.avg - avg) <= 1e-12 * abs(avg) and abs(got.m2 - m2) <= 1e-12 * m2
    assert got.pred_true == sum(1 for x in py if x is not None and x >= 0.0)


@pytest.mark.parametrize("pattern", [r"(https?|ftp)://[^\s/$.?#].[^\s]*", r"\d*", r"(?i)ab+"])
def test_c_dfa_walk_counts_like_the_python_oracle(pattern):
    """or_dfa_count (the PatternMatch timing baseline) walks the compiled table: the same hits as
    the oracle's Java find() restatement."""
    import random
    from deequ_amd.regex import compile_java_regex
    rng = random.Random(3)
    alpha = list("abAB09 :/.htpsé") + ["http://", "ftp://"]
    rows = [None if rng.random() < 0.05 else
            "".join(rng.choice(alpha) for _ in range(rng.randint(0, 12))) for _ in range(5000)]
    off, data, valid = _buffers(pa.array(rows, pa.string()))
    got = C.dfa_count(off, data, valid, len(rows), compile_java_regex(pattern), threads=3)
    assert got == sum(O.regex_find_nonempty(r, pattern) for r in rows if r is not None)


@pytest.mark.parametrize("threads", [1, 5])
def test_c_datatype_matches_python_oracle(threads):
    """or_dtype_utf8 (the configs[4] CPU baseline's DataType) against deequ_oracle.datatype_counts
    (the three regexes of StatefulDataType.scala:36-38 through Python `re`)."""
    rng = np.random.default_rng(threads)
    pool = ["1.5", "-3", " 4", "+ 7", "- .5", "true", "false", "", ".", "abc", "1e5", "12a",
            "+-1", "  1", "TRUE", "007", "3.", "-", "+", " ", "1.2.3", "falsey", "٣"]
    vals = [None if rng.random() < 0.07 else str(rng.choice(pool)) for _ in range(20_011)]
    arr = pa.array(vals, type=pa.string())
    off, data, valid = _buffers(arr)
    got = C.dtype_utf8(off, data, valid, len(vals), threads)
    exp = O.datatype_counts(O.OTable({"s": vals}, {"s": "string"}), "s", None)
    assert got == exp


@pytest.mark.parametrize("threads", [1, 4])
def test_c_mutual_information_matches_python_oracle(threads):
    rng = np.random.default_rng(40 + threads)
    n = 30_000
    a = [None if rng.random() < 0.05 else f"a{v}" for v in rng.integers(0, 300, n)]
    b = [None if rng.random() < 0.05 else f"b{v}" for v in rng.integers(0, 7, n)]
    A, B = _buffers(pa.array(a, pa.string())), _buffers(pa.array(b, pa.string()))
    got = C.mi_utf8(A, B, n, n, threads)
    exp = O.mutual_information(O.OTable({"a": a, "b": b}, {"a": "string", "b": "string"}), "a", "b")
    assert math.isclose(got, exp, rel_tol=1e-12), (got, exp)
