"""configs[2]'s frequency family at its STATED size (1e9 rows) on a high-cardinality int64 key WITH
duplicates: `test_gpu_fullsize.py` checks `id`, a bijection of the
row number, where every group has count 1.  Here the key comes from a generator whose count
distribution is known exactly:

  * row r belongs to group q = r // 3 (three rows per group), except that when q % 7 == 0 the
    third row r = 3q + 2 is planted as a singleton group of its own (group id N + q);
  * rows with r % 20 == 19 are NULL;
  * the value is (g * K) ^ X (mod 2^64) for group id g: a bijection, so groups and values
    correspond one to one, and the values span the whole 64-bit range (the hashed exact path, not
    the dense one).

So the groups have counts 1, 2 and 3 in proportions the host computes exactly from the formula
(no pass over the device data), and Uniqueness, Distinctness, Entropy, and Histogram's bins and
top-1000 follow.  One batch (the first 2^26 rows) is also run alone through the engine and checked
against oracle/oracle.c's or_freq over the same buffers copied to the host.

Reference: GroupingAnalyzers.scala:53-80 (the group-by and numRows), Uniqueness.scala:26-32,
Distinctness.scala:29-35, Entropy.scala:27-39, Histogram.scala:41-116.  The oracle is the checker
only.
"""
import math

import numpy as np
import pytest

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

ROWS = 1_000_000_000
BATCH = 1 << 26
THREADS = 16
K = 0x9E3779B97F4A7C15          # odd: g -> g * K is a bijection mod 2^64
X = 0x5DEECE66D
M64 = (1 << 64) - 1


def _signed(v: int) -> int:
    return v - (1 << 64) if v >> 63 else v


def _dup_table(n: int, device):
    """The generator above, as an int64 column `k` in HBM (torch ops on the device)."""
    import torch
    from deequ_amd import _native as N
    from deequ_amd.table import ColumnBatch, StructField, StructType, Table
    dev = torch.device(device)
    weights = torch.tensor([1 << i for i in range(8)], dtype=torch.int32, device=dev)
    batches, pos = [], 0
    while pos < n:
        m = min(BATCH, n - pos)
        assert m % 8 == 0
        r = torch.arange(pos, pos + m, dtype=torch.int64, device=dev)
        q = torch.div(r, 3, rounding_mode="floor")
        split = (q % 7 == 0) & (r % 3 == 2)
        g = torch.where(split, q + n, q)
        vals = torch.empty(m + 2, dtype=torch.int64, device=dev)
        vals[:m] = (g * _signed(K)) ^ X
        vals[m:] = 0
        valid = (r % 20 != 19).view(-1, 8).to(torch.int32)
        bits = (valid * weights).sum(dim=1).to(torch.uint8)
        vbuf = torch.zeros(m // 8 + 16, dtype=torch.uint8, device=dev)
        vbuf[: m // 8] = bits
        del r, q, split, g, valid
        batches.append({"k": ColumnBatch(N.INT64, m, vbuf, vals)})
        pos += m
    torch.cuda.synchronize(dev)
    return Table(StructType([StructField("k", N.INT64)]), batches, device)


def _expected_counts(n: int):
    """Exact count-of-counts {c: #groups with count c} of the generator over n rows, and the
    non-NULL row count."""
    hist = np.zeros(4, np.int64)
    nq = (n + 2) // 3
    step = 1 << 24
    for q0 in range(0, nq, step):
        q = np.arange(q0, min(nq, q0 + step), dtype=np.int64)
        split = q % 7 == 0
        main = np.zeros(len(q), np.int64)
        for r in range(3):
            row = 3 * q + r
            present = (row < n) & (row % 20 != 19)
            if r == 2:
                hist += np.bincount(present & split, minlength=2)[1] * np.array([0, 1, 0, 0])
                present &= ~split
            main += present
        hist += np.bincount(main, minlength=4)[:4]
    hist[0] = 0
    nn = int(sum(c * hist[c] for c in range(4)))
    return {c: int(hist[c]) for c in (1, 2, 3)}, nn


def _count_of_key(v: int, n: int) -> int:
    """The generator's count for the group whose value is v (0: no such group)."""
    g = ((v ^ X) * pow(K, -1, 1 << 64)) & M64
    if g >= n:                                   # a planted singleton: row 3q + 2
        q = g - n
        row = 3 * q + 2
        return int(q % 7 == 0 and row < n and row % 20 != 19)
    rows = [3 * g + r for r in range(3 if g % 7 else 2)]
    return sum(1 for row in rows if row < n and row % 20 != 19)


def _suite():
    from deequ_amd.analyzers import Distinctness, Entropy, Histogram, Uniqueness
    return [Uniqueness(["k"]), Distinctness(["k"]), Entropy("k"), Histogram("k")]


def test_duplicate_bearing_key_at_1e9_rows_follows_the_generator(gpu_device):
    import torch
    from deequ_amd.analyzers import Distinctness, Entropy, Histogram, Uniqueness
    from deequ_amd.runners import AnalysisRunner
    counts, nn = _expected_counts(ROWS)
    t = _dup_table(ROWS, gpu_device)
    try:
        ctx = AnalysisRunner.do_analysis_run(t, _suite())
    finally:
        del t
        torch.cuda.empty_cache()
    n = ROWS
    groups = sum(counts.values())
    assert counts[1] > 0 and counts[2] > 0 and counts[3] > 0
    assert ctx.metric(Uniqueness(["k"])).value.get() == counts[1] / n
    assert ctx.metric(Distinctness(["k"])).value.get() == groups / n
    ent = -math.fsum(nc * (c / n) * math.log(c / n) for c, nc in counts.items())
    got = ctx.metric(Entropy("k")).value.get()
    assert got == ent or abs(got - ent) <= 1e-12 * ent, (got, ent)
    hist = ctx.metric(Histogram("k")).value.get()
    assert hist.number_of_bins == groups + 1
    assert len(hist.values) == 1000
    assert hist.values["NullValue"].absolute == n - nn       # the largest bin
    seen = set()
    for key, dv in hist.values.items():
        if key == "NullValue":
            continue
        v = int(key) & M64
        assert v not in seen
        seen.add(v)
        assert dv.absolute == 3, key                         # the top 999 are count-3 groups
        assert _count_of_key(v, n) == 3, key


def test_one_batch_of_the_duplicate_key_matches_or_freq(gpu_device):
    import torch
    from deequ_amd.analyzers import Distinctness, Entropy, Histogram, Uniqueness
    from deequ_amd.runners import AnalysisRunner
    t = _dup_table(BATCH, gpu_device)
    try:
        ctx = AnalysisRunner.do_analysis_run(t, _suite())
        col = t.batches[0]["k"]
        vals = col.values[:BATCH].cpu().numpy()
        vb = col.validity[: BATCH // 8].cpu().numpy()
    finally:
        del t
        torch.cuda.empty_cache()
    out, tc, tr = C.freq("long", vals, None, vb, BATCH, BATCH, null_as_group=True, k=8,
                         threads=THREADS)
    counts, nn = _expected_counts(BATCH)
    assert out.null_rows == BATCH - nn
    assert out.groups == sum(counts.values()) + 1          # (+ the NULL group)
    assert out.unique == counts[1]
    n = BATCH
    assert ctx.metric(Uniqueness(["k"])).value.get() == out.unique / n
    assert ctx.metric(Distinctness(["k"])).value.get() == (out.groups - 1) / n
    ent = ctx.metric(Entropy("k")).value.get()
    exp = -math.fsum(nc * (c / n) * math.log(c / n) for c, nc in counts.items())
    assert ent == exp or abs(ent - exp) <= 1e-12 * exp
    hist = ctx.metric(Histogram("k")).value.get()
    assert hist.number_of_bins == out.groups
    assert hist.values["NullValue"].absolute == out.null_rows
    assert int(tc[0]) == out.null_rows and int(tr[0]) == -1
    for key, dv in hist.values.items():
        if key != "NullValue":
            assert dv.absolute == _count_of_key(int(key) & M64, n) == 3
