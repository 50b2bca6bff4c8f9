"""GPU parity of DataType (the TK_DTYPE scan body) and MutualInformation (dq_freq_marginal +
dq_freq_mutual_information) against the ORACLE and the reference's known answers
(AnalyzerTests.scala:132-153 and :266-330, NullHandlingTests.scala:96-101)."""
import math
import random
import zlib

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


def _df(cols, device, batch=None):
    from deequ_amd.table import Table
    return Table.from_arrow(pa.table(cols), device=device, max_batch_rows=batch)


def _counts(metric):
    d = metric.value.get()
    assert d.number_of_bins == 5
    return tuple(d.values[k].absolute for k in ("Unknown", "Fractional", "Integral", "Boolean",
                                                  "String"))


def test_datatype_known_answers(gpu_device):
    from deequ_amd.analyzers import DataType
    df = _df({"s": pa.array(["1", "2", "3", "4", "5", "6"]),
              "i": pa.array([1, 2, 3, 4, 5, 6], pa.int64()),
              "f": pa.array([1.0, 2.0, 3.0, 4.0, 5.0, 6.0], pa.float32()),
              "neg": pa.array(["-1.0", "-2.0", "-3.0", "-4.0", "-1.5", "-2.5"]),
              "mixed": pa.array(["1.0", "1", "a", None, "true", "false"])}, gpu_device)
    assert _counts(DataType("s").calculate(df)) == (0, 0, 6, 0, 0)
    assert _counts(DataType("i").calculate(df)) == (0, 0, 6, 0, 0)
    assert _counts(DataType("f").calculate(df)) == (0, 6, 0, 0, 0)
    assert _counts(DataType("neg").calculate(df)) == (0, 6, 0, 0, 0)
    assert _counts(DataType("mixed").calculate(df)) == (1, 1, 1, 2, 1)
    m = DataType("mixed").calculate(df).value.get()
    assert m.values["Boolean"].ratio == 2 / 6


def test_datatype_all_null_column(gpu_device):
    """NullHandlingTests.scala:96-101: DataType over 8 NULLs = (8, 0, 0, 0, 0)."""
    from deequ_amd.analyzers import DataType
    df = _df({"x": pa.array([None] * 8, pa.string())}, gpu_device)
    assert _counts(DataType("x").calculate(df)) == (8, 0, 0, 0, 0)


@pytest.mark.parametrize("dtype", ["string", "int32", "float64", "bool"])
def test_datatype_matches_oracle(dtype, gpu_device):
    from deequ_amd.analyzers import DataType
    from oracle.deequ_oracle import OTable, datatype_counts
    rng = random.Random(zlib.crc32(dtype.encode()))
    n = 20_011
    if dtype == "string":
        pieces = ["", "-", "+", " ", "1", "23", ".", "5", "true", "false", "x", "e", "\n"]
        vals = ["".join(rng.choice(pieces) for _ in range(rng.randint(0, 4))) for _ in range(n)]
        arr = pa.array([None if rng.random() < 0.05 else v for v in vals], pa.string())
        otype = "string"
    elif dtype == "int32":
        arr = pa.array([None if rng.random() < 0.05 else rng.randint(-10**6, 10**6)
                        for _ in range(n)], pa.int32())
        otype = "int"
    elif dtype == "float64":
        pool = [0.0, -0.0, 1e-3, 9.99e-4, 1e7, 9999999.0, -123.5, float("nan"), float("inf"),
                -float("inf"), 1e300, 5e-324]
        arr = pa.array([None if rng.random() < 0.05 else rng.choice(pool) * (1 if rng.random() < .5
                                                                               else -1)
                        for _ in range(n)], pa.float64())
        otype = "double"
    else:
        arr = pa.array([None if rng.random() < 0.05 else rng.random() < 0.5 for _ in range(n)],
                       pa.bool_())
        otype = "boolean"
    k = [rng.randint(0, 9) for _ in range(n)]
    df = _df({"x": arr, "k": pa.array(k, pa.int64())}, gpu_device, 7000)
    ot = OTable({"x": arr.to_pylist(), "k": k}, {"x": otype, "k": "long"})
    for where in (None, "k > 4"):
        got = _counts(DataType("x", where).calculate(df))
        assert got == datatype_counts(ot, "x", where), (dtype, where)


def test_mutual_information_known_answers(gpu_device):
    from deequ_amd.analyzers import Entropy, MutualInformation
    full = _df({"item": pa.array(["1", "2", "3", "4"]), "att1": pa.array(["a", "a", "a", "b"]),
                "att2": pa.array(["c", "c", "c", "d"])}, gpu_device)
    mi = MutualInformation("att1", "att2").calculate(full).value.get()
    assert math.isclose(mi, -(0.75 * math.log(0.75) + 0.25 * math.log(0.25)), rel_tol=1e-12)
    uninformative = _df({"att1": pa.array([1, 2, 3], pa.int64()),
                         "att2": pa.array([0, 0, 0], pa.int64())}, gpu_device)
    assert MutualInformation("att1", "att2").calculate(uninformative).value.get() == 0.0
    same = MutualInformation("att1", "att1").calculate(full).value.get()
    assert math.isclose(same, Entropy("att1").calculate(full).value.get(), rel_tol=1e-12)


def test_mutual_information_of_null_columns_is_empty(gpu_device):
    """NullHandlingTests.scala:100-101."""
    from deequ_amd.analyzers import MutualInformation
    df = _df({"a": pa.array([None] * 4, pa.float64()), "b": pa.array([1.0] * 4)}, gpu_device)
    assert MutualInformation("a", "b").calculate(df).value.is_failure


@pytest.mark.parametrize("kinds", [("long", "string"), ("string", "string"), ("long", "long"),
                                   ("double", "string")])
def test_mutual_information_matches_oracle(kinds, gpu_device):
    from deequ_amd.analyzers import MutualInformation
    from oracle.deequ_oracle import OTable, mutual_information
    rng = np.random.default_rng(len("".join(kinds)))
    n = 40_000

    def col(kind, card):
        v = rng.integers(0, card, n)
        mask = rng.random(n) < 0.05
        if kind == "string":
            return pa.array([None if m else f"v{x}" for x, m in zip(v, mask)], pa.string())
        if kind == "double":
            return pa.array(v * 0.5, mask=mask, type=pa.float64())
        return pa.array(v, mask=mask, type=pa.int64())
    a, b = col(kinds[0], 50), col(kinds[1], 700)
    df = _df({"a": a, "b": b}, gpu_device, 9000)
    ot = OTable({"a": a.to_pylist(), "b": b.to_pylist()}, {"a": kinds[0], "b": kinds[1]})
    got = MutualInformation("a", "b").calculate(df).value.get()
    exp = mutual_information(ot, "a", "b")
    assert abs(got - exp) <= 1e-12 * max(1.0, abs(exp)), (got, exp)


@pytest.mark.parametrize("kinds", [("string", "string"), ("long", "string"), ("double", "long")])
def test_mutual_information_hash_lookups_equal_byte_lookups(kinds, gpu_device, monkeypatch):
    """The marginal counts looked up by row hash (no two marginal keys on one 64-bit hash) give
    the same MI as the lookups that compare key bytes (DQ_FREQ_MI_LOOKUP=1) and the oracle;
    high-cardinality strings on both sides, ragged batches."""
    from deequ_amd.analyzers import MutualInformation
    rng = np.random.default_rng(77)
    n = 150_001

    def col(kind, card):
        v = rng.integers(0, card, n)
        mask = rng.random(n) < 0.05
        if kind == "string":
            return pa.array([None if m else f"key-{x}-{x * 7919 % 1000}" for x, m in zip(v, mask)],
                            pa.string())
        if kind == "double":
            return pa.array(v * 0.25, mask=mask, type=pa.float64())
        return pa.array(v, mask=mask, type=pa.int64())
    from oracle.deequ_oracle import OTable, mutual_information
    a, b = col(kinds[0], 60_000), col(kinds[1], 40)
    df = _df({"a": a, "b": b}, gpu_device, 50_000)
    fast = MutualInformation("a", "b").calculate(df).value.get()
    monkeypatch.setenv("DQ_FREQ_MI_LOOKUP", "1")
    slow = MutualInformation("a", "b").calculate(df).value.get()
    # each run builds its own joint table (the groups come in another order), but the terms are
    # the same function of the counts and their sum is order-free (fixed point): bit-identical
    assert fast == slow, (fast, slow)
    exp = mutual_information(OTable({"a": a.to_pylist(), "b": b.to_pylist()},
                                    {"a": kinds[0], "b": kinds[1]}), "a", "b")
    assert abs(fast - exp) <= 1e-12 * max(1.0, abs(exp)), (fast, exp)


@pytest.mark.parametrize("kinds,cards", [(("string", "string"), (50_000, 3)),
                                         (("string", "string"), (4, 3)),
                                         (("long", "string"), (7, 60_000)),
                                         (("double", "long"), (12, 5)),
                                         (("string", "long"), (20, 9)),
                                         # a general side of each record kind next to a small
                                         # one: fixed-width, and utf8 over 16 bytes (hashed
                                         # from memory)
                                         (("long", "string"), (80_000, 3)),
                                         (("double", "string"), (70_000, 4)),
                                         (("lstring", "string"), (40_000, 5))])
def test_mutual_information_small_marginals(kinds, cards, gpu_device, monkeypatch):
    """A side with few values has its marginal aggregated in one pass over the joint groups
    (freq_small_marginal: per-wave value lists merged by hash and key words); a side with more
    values than a wave can list takes the general path.  Bar: the oracle within 1e-12, and the
    same as with the small pass off (DQ_FREQ_MI_NOSMALL=1)."""
    from deequ_amd.analyzers import MutualInformation
    from oracle.deequ_oracle import OTable, mutual_information
    rng = np.random.default_rng(sum(cards))
    n = 120_001

    def col(kind, card):
        v = rng.integers(0, card, n)
        mask = rng.random(n) < 0.05
        if kind == "string":
            return pa.array([None if m else f"val-{x}" for x, m in zip(v, mask)], pa.string())
        if kind == "lstring":
            return pa.array([None if m else f"a-value-longer-than-sixteen-bytes-{x}"
                             for x, m in zip(v, mask)], pa.string())
        if kind == "double":
            return pa.array(v * 0.5 - 1.0, mask=mask, type=pa.float64())
        return pa.array(v, mask=mask, type=pa.int64())
    a, b = col(kinds[0], cards[0]), col(kinds[1], cards[1])
    df = _df({"a": a, "b": b}, gpu_device, 40_000)
    got = MutualInformation("a", "b").calculate(df).value.get()
    okind = {"lstring": "string"}
    exp = mutual_information(OTable({"a": a.to_pylist(), "b": b.to_pylist()},
                                    {"a": okind.get(kinds[0], kinds[0]),
                                     "b": okind.get(kinds[1], kinds[1])}), "a", "b")
    assert abs(got - exp) <= 1e-12 * max(1.0, abs(exp)), (got, exp)
    # the waves' lists merged on the host instead of by freq_small_merge: the same value counts,
    # so the same bits
    monkeypatch.setenv("DQ_FREQ_MI_HOSTMERGE", "1")
    host = MutualInformation("a", "b").calculate(df).value.get()
    assert host == got, (host, got)
    monkeypatch.delenv("DQ_FREQ_MI_HOSTMERGE")
    monkeypatch.setenv("DQ_FREQ_MI_NOSMALL", "1")
    ref = MutualInformation("a", "b").calculate(df).value.get()
    assert abs(got - ref) <= 1e-12 * max(1.0, abs(ref)), (got, ref)


def test_mutual_information_of_merged_states(gpu_device):
    """FrequenciesAndNumRows.sum (GroupingAnalyzers.scala:128-148) then MutualInformation."""
    from deequ_amd.analyzers import MutualInformation
    from deequ_amd.analyzers.base import merge_states
    from oracle.deequ_oracle import OTable, mutual_information
    rng = np.random.default_rng(9)
    n = 12_000
    a = pa.array([f"s{x}" for x in rng.integers(0, 30, n)])
    b = pa.array(rng.integers(0, 9, n), pa.int64())
    t = pa.table({"a": a, "b": b})
    from deequ_amd.table import Table
    parts = [Table.from_arrow(t.slice(lo, 4000), device=gpu_device) for lo in (0, 4000, 8000)]
    an = MutualInformation("a", "b")
    merged = merge_states(*[an.compute_state_from(p) for p in parts])
    got = an.compute_metric_from(merged).value.get()
    exp = mutual_information(OTable({"a": a.to_pylist(), "b": b.to_pylist()},
                                    {"a": "string", "b": "long"}), "a", "b")
    assert abs(got - exp) <= 1e-12 * max(1.0, abs(exp))
