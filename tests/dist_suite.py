"""The table and suite shared by tests/test_gpu_distributed.py and its rank workers."""
import math

import numpy as np
import pyarrow as pa


def table(n=30_000, seed=5):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, n // 3, n)
    b = rng.normal(10.0, 3.0, n)
    words = np.array(["high", "low", "medium", "", "NullValue", "long string " * 3])
    s = words[rng.integers(0, len(words), n)]
    u = np.array([f"u{v}" for v in rng.integers(0, n, n)])
    uid = rng.permutation(n).astype(np.int64) * 7919 - n  # unique: the raw-key exchange
    uid32 = rng.permutation(n).astype(np.int32)

    def mask():
        return rng.random(n) < 0.05
    return pa.table({
        "id": pa.array(ids, mask=mask(), type=pa.int64()),
        "b": pa.array(b, mask=mask(), type=pa.float64()),
        "s": pa.array([None if m else v for v, m in zip(s, mask())], type=pa.string()),
        "u": pa.array([None if m else v for v, m in zip(u, mask())], type=pa.string()),
        "uid": pa.array(uid, mask=mask(), type=pa.int64()),
        "uid32": pa.array(uid32, mask=mask(), type=pa.int32()),
    })


TYPES = {"id": "long", "b": "double", "s": "string", "u": "string", "uid": "long", "uid32": "int"}


def suite():
    from deequ_amd.analyzers import (ApproxCountDistinct, Completeness, CountDistinct, Correlation,
                                     Distinctness, Entropy, Histogram, Maximum, Mean, Size,
                                     StandardDeviation, Uniqueness, UniqueValueRatio)
    return [Size(), Completeness("s"), Mean("id"), StandardDeviation("b"), Maximum("b"),
            ApproxCountDistinct("id"), ApproxCountDistinct("u"), Correlation("id", "b"),
            Uniqueness(["id"]), Distinctness(["id"]), Entropy("id"), UniqueValueRatio(["s"]),
            CountDistinct(["s", "u"]), Uniqueness(["id", "s"]), Histogram("s"), Histogram("id"),
            Uniqueness(["uid"]), Distinctness(["uid"]), Entropy("uid"), CountDistinct(["uid"]),
            Histogram("uid"), Uniqueness(["uid32"]), Entropy("uid32"), Histogram("uid32")]


def oracle_metrics(t):
    """The oracle's value of every grouping / Histogram / scan metric of suite() on table t:
    {str(analyzer): value}, Histograms as (bins, sorted counts)."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import deequ_oracle as O
    from deequ_amd.analyzers import (Completeness, CountDistinct, Distinctness, Entropy, Histogram,
                                     Maximum, Mean, Size, Uniqueness, UniqueValueRatio)
    ot = O.OTable({c: t.column(c).to_pylist() for c in t.column_names}, TYPES)
    n = t.num_rows
    out = {}
    for a in suite():
        if isinstance(a, (Uniqueness, Distinctness, CountDistinct, UniqueValueRatio, Entropy)):
            cols = list(a.columns) if hasattr(a, "columns") else [a.column]
            f = O.frequencies(ot, cols)
            fn = {Uniqueness: lambda: O.uniqueness(f, n), Distinctness: lambda: O.distinctness(f, n),
                  CountDistinct: lambda: O.count_distinct(f),
                  UniqueValueRatio: lambda: O.unique_value_ratio(f),
                  Entropy: lambda: O.entropy(f, n)}[type(a)]
            out[str(a)] = fn()
        elif isinstance(a, Histogram):
            h, _rows = O.histogram(ot, a.column)
            out[str(a)] = [len(h), sorted(h.values(), reverse=True)]
        elif isinstance(a, Size):
            out[str(a)] = float(n)
        elif isinstance(a, Completeness):
            out[str(a)] = O.agg_sum_notnull(ot, a.column, None) / n
        elif isinstance(a, Mean):
            out[str(a)] = O.agg_sum(ot, a.column, None) / n  # count("*"): Mean.scala:40
        elif isinstance(a, Maximum):
            out[str(a)] = O.agg_max(ot, a.column, None)
    return out


def metrics_of(ctx):
    """{str(analyzer): value} -- Histograms as (bins, sorted top counts, {key: count})."""
    out = {}
    for a in suite():
        v = ctx.metric(a).value
        if not v.is_success:
            out[str(a)] = ["failure", str(v)]
            continue
        x = v.get()
        if hasattr(x, "number_of_bins"):
            out[str(a)] = [x.number_of_bins,
                           sorted((d.absolute for d in x.values.values()), reverse=True),
                           {k: d.absolute for k, d in x.values.items()}]
        else:
            out[str(a)] = x
    return out


def close(a, b, rel=1e-12):
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b or abs(a - b) <= rel * max(abs(a), abs(b))
