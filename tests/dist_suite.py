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

    def mask():
        return rng.random(n) < 0.05
    return pa.table({
        "id": pa.array(ids, mask=mask(), type=pa.int64()),
        "b": pa.array(b, mask=mask(), type=pa.float64()),
        "s": pa.array([None if m else v for v, m in zip(s, mask())], type=pa.string()),
        "u": pa.array([None if m else v for v, m in zip(u, mask())], type=pa.string()),
    })


def suite():
    from deequ_amd.analyzers import (ApproxCountDistinct, Completeness, CountDistinct, Correlation,
                                     Distinctness, Entropy, Histogram, Maximum, Mean, Size,
                                     StandardDeviation, Uniqueness, UniqueValueRatio)
    return [Size(), Completeness("s"), Mean("id"), StandardDeviation("b"), Maximum("b"),
            ApproxCountDistinct("id"), ApproxCountDistinct("u"), Correlation("id", "b"),
            Uniqueness(["id"]), Distinctness(["id"]), Entropy("id"), UniqueValueRatio(["s"]),
            CountDistinct(["s", "u"]), Uniqueness(["id", "s"]), Histogram("s"), Histogram("id")]


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
