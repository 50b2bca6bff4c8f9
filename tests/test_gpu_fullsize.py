"""The headline configurations at their STATED sizes (BASELINE.json configs[1]-[3]), checked after
the engine ran them on the device:

  * configs[1] S10 over 1e9 synthetic Item rows: counts, the wrapping Long sum and min / max
    bit-exact, StandardDeviation within 1e-12, against oracle/oracle.c run batch by batch over the
    same device buffers copied to the host (Spark's partitions, merged as Spark merges them);
  * configs[2] the frequency family + Histogram on `id` and `priority` over 1e9 rows through
    AnalysisRunner.  `id` is a bijection of the row number (synth.hip: splitmix64 of row ^ c), so
    every non-NULL id is its own group: #groups = #unique = non-NULL rows, Histogram has
    non-NULL + 1 bins, Entropy = (nn / n) ln n, and every listed id inverts to a non-NULL row of
    the table.  `priority`'s group counts must equal oracle/oracle.c's or_freq exactly;
  * configs[3] ApproxCountDistinct(id) + Correlation(id, score) over 1.25e9 rows (the per-GPU
    shard of 1e10 over 8): the HLL registers bit-exact against or_hll, the co-moments against
    or_corr within 1e-12 of their scale.

Reference: AnalysisRunner.scala:296-303 (one aggregation per suite over all partitions),
StatefulHyperloglogPlus.scala:87-137, Correlation.scala:37-52, GroupingAnalyzers.scala:53-80,
Histogram.scala:41-116.  The oracle is the checker only: it never produces what is measured.
"""
import math

import numpy as np
import pytest

from oracle import c_oracle as C
from oracle.deequ_oracle import corr_merge, hll_words, moments_merge

pytestmark = pytest.mark.gpu

ROWS = 1_000_000_000          # configs[1] / configs[2]
ROWS_C3 = 1_250_000_000       # configs[3]: 1e10 rows over 8 GPUs
THREADS = 16                  # the GPU box's CPU share


def rel_close(a, b, tol=1e-12):
    return a == b or abs(a - b) <= tol * max(abs(a), abs(b))


@pytest.fixture(scope="module")
def item_1e9(gpu_device):
    import torch
    from deequ_amd.synth import item_table_device
    t = item_table_device(ROWS, seed=7, batch_rows=1 << 26, device=gpu_device)
    yield t
    del t
    torch.cuda.empty_cache()


def _host(col, m):
    """A device column's first m rows as host numpy buffers: (values or offsets, bytes, validity)."""
    valid = col.validity[: (m + 7) // 8].cpu().numpy()
    if col.data is not None:
        off = col.values[: m + 1].cpu().numpy()
        return off, col.data[: int(off[-1]) + 1].cpu().numpy(), valid
    return col.values[:m].cpu().numpy(), None, valid


def test_s10_at_1e9_rows_matches_c_oracle(item_1e9):
    from deequ_amd import Analysis
    from deequ_amd.analyzers import (Completeness, Compliance, Maximum, Mean, Minimum, Size,
                                     StandardDeviation, Sum)
    suite = [Size(), Completeness("id"), Completeness("name"),
             Compliance("numViews is non-negative", "numViews >= 0"),
             Compliance("priority contained in high,low",
                        "priority IS NULL OR priority IN ('high','low')"),
             Sum("numViews"), Mean("numViews"), StandardDeviation("numViews"),
             Minimum("numViews"), Maximum("numViews")]
    ctx = Analysis(suite).run(item_1e9)
    n = item_1e9.num_rows
    assert n == ROWS
    parts, comp_id, comp_name, pt = [], 0, 0, 0
    for b in item_1e9.batches:
        m = b["id"].length
        v, _, vb = _host(b["numViews"], m)
        parts.append(C.numeric_i64(v, vb, op=17, lit=0, threads=THREADS))
        comp_id += C.validity_count(_host(b["id"], m)[2], m, THREADS)
        comp_name += C.validity_count(b["name"].validity.cpu().numpy(), m, THREADS)
        off, data, pv = _host(b["priority"], m)
        pt += C.str_in(off, data, pv, m, ["high", "low"], True, THREADS)[0]
    s = sum(p.sum_long for p in parts)
    s = (s + (1 << 63)) % (1 << 64) - (1 << 63)          # Spark's Long sum wraps
    assert ctx.metric(Size()).value.get() == n
    assert ctx.metric(Completeness("id")).value.get() == comp_id / n
    assert ctx.metric(Completeness("name")).value.get() == comp_name / n
    assert ctx.metric(suite[3]).value.get() == sum(p.pred_true for p in parts) / n
    assert ctx.metric(suite[4]).value.get() == pt / n
    assert ctx.metric(Sum("numViews")).value.get() == float(s)
    assert ctx.metric(Mean("numViews")).value.get() == float(s) / n
    assert ctx.metric(Minimum("numViews")).value.get() == float(min(p.min for p in parts))
    assert ctx.metric(Maximum("numViews")).value.get() == float(max(p.max for p in parts))
    st = (0.0, 0.0, 0.0)
    for p in parts:                                       # Spark's partition merge, batch order
        st = moments_merge(st, (p.n, p.avg, p.m2))
    assert rel_close(ctx.metric(StandardDeviation("numViews")).value.get(),
                     math.sqrt(st[2] / st[0]))


def _splitmix_inverse(z: int) -> int:
    """Inverse of synth.hip's mix() (splitmix64's finaliser after adding the golden gamma)."""
    m64 = (1 << 64) - 1
    z ^= (z >> 31) ^ (z >> 62)
    z = (z * pow(0x94D049BB133111EB, -1, 1 << 64)) & m64
    z ^= (z >> 27) ^ (z >> 54)
    z = (z * pow(0xBF58476D1CE4E5B9, -1, 1 << 64)) & m64
    z ^= (z >> 30) ^ (z >> 60)
    return (z - 0x9E3779B97F4A7C15) & m64


def test_frequency_family_at_1e9_rows_on_its_invariants(item_1e9):
    from deequ_amd.analyzers import Distinctness, Entropy, Histogram, Uniqueness
    from deequ_amd.runners import AnalysisRunner
    suite = [a for c in ("id", "priority")
             for a in (Uniqueness([c]), Distinctness([c]), Entropy(c), Histogram(c))]
    ctx = AnalysisRunner.do_analysis_run(item_1e9, suite)
    n = item_1e9.num_rows
    valid_bits = []
    nn = 0
    for b in item_1e9.batches:
        m = b["id"].length
        vb = b["id"].validity[: (m + 7) // 8].cpu().numpy()
        valid_bits.append((m, vb))
        nn += C.validity_count(vb, m, THREADS)
    # id: one group per non-NULL row
    assert ctx.metric(Uniqueness(["id"])).value.get() == nn / n
    assert ctx.metric(Distinctness(["id"])).value.get() == nn / n
    assert rel_close(ctx.metric(Entropy("id")).value.get(), nn / n * math.log(n))
    hist = ctx.metric(Histogram("id")).value.get()
    assert hist.number_of_bins == nn + 1
    assert len(hist.values) == 1000
    assert hist.values["NullValue"].absolute == n - nn     # the largest bin
    starts = np.cumsum([0] + [m for m, _ in valid_bits])
    for key, dv in hist.values.items():
        if key == "NullValue":
            continue
        assert dv.absolute == 1, key
        row = _splitmix_inverse(int(key) & ((1 << 64) - 1)) ^ 0x5DEECE66D
        assert row < n, key
        bi = int(np.searchsorted(starts, row, side="right")) - 1
        r = row - starts[bi]
        assert valid_bits[bi][1][r >> 3] >> (r & 7) & 1, key   # the id of a non-NULL row
    # priority: the group counts against or_freq over every batch (top 4 of 3 values + NULL)
    counts = {}
    for b in item_1e9.batches:
        m = b["priority"].length
        off, data, pv = _host(b["priority"], m)
        out, tc, tr = C.freq("string", off, data, pv, m, m, null_as_group=True, k=4,
                             threads=THREADS)
        for c, r in zip(tc.tolist(), tr.tolist()):
            key = "NullValue" if r < 0 else bytes(data[off[r]:off[r + 1]]).decode()
            counts[key] = counts.get(key, 0) + c
    assert sum(counts.values()) == n
    ph = ctx.metric(Histogram("priority")).value.get()
    assert ph.number_of_bins == len(counts) == 4
    assert {k: v.absolute for k, v in ph.values.items()} == counts
    groups = [c for k, c in counts.items() if k != "NullValue"]
    assert ctx.metric(Uniqueness(["priority"])).value.get() == 0.0
    assert ctx.metric(Distinctness(["priority"])).value.get() == 3 / n
    ent = -math.fsum(c / n * math.log(c / n) for c in groups)
    assert rel_close(ctx.metric(Entropy("priority")).value.get(), ent)


def test_hll_and_correlation_at_1_25e9_rows_match_c_oracle(gpu_device):
    import torch
    from deequ_amd.analyzers import ApproxCountDistinct, Correlation
    from deequ_amd.runners.engine import get_plan, run_scan
    from deequ_amd.synth import item_table_device
    t = item_table_device(ROWS_C3, seed=9, batch_rows=1 << 26, device=gpu_device, extra=True)
    try:
        hll, corr = ApproxCountDistinct("id"), Correlation("id", "score")
        aggs = hll.aggregation_functions() + corr.aggregation_functions()
        assert "+hll[" in get_plan(t.schema, aggs).explain()  # the fused configs[3] pass
        row = run_scan(t, aggs)
        st = hll.from_aggregation_result(row, 0)
        cst = corr.from_aggregation_result(row, len(hll.aggregation_functions()))
        regs = np.zeros(512, np.uint8)
        mom = (0.0,) * 6
        for b in t.batches:
            m = b["id"].length
            x, _, vx = _host(b["id"], m)
            y, _, vy = _host(b["score"], m)
            regs = np.maximum(regs, C.hll(5, x, None, vx, m, THREADS))
            mom = corr_merge(mom, C.corr(x, vx, y.view(np.float64), vy, THREADS))
    finally:
        del t
        torch.cuda.empty_cache()
    assert list(st.words) == hll_words(regs.tolist())
    assert cst.n == mom[0]
    got = (cst.n, cst.x_avg, cst.y_avg, cst.ck, cst.x_mk, cst.y_mk)
    for g, e in zip(got[1:], mom[1:]):
        assert rel_close(g, e), (got, mom)
    ref = mom[3] / math.sqrt(mom[4] * mom[5])
    assert rel_close(cst.metric_value(), ref)
