"""The columnar loader (loader.cpp: dq_scan_host, dq_freq_add_host) against the ORACLE on
multi-batch host Arrow tables, and its buffer-lifetime contract: a host batch is overwritten the
moment each call returns, and the results must not change (include/deequ_amd.h, loader section)."""
import math

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-12


def _close(a, b):
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b or abs(a - b) <= REL * max(abs(a), abs(b))


def _table(n, seed):
    rng = np.random.default_rng(seed)
    words = np.array(["high", "low", "medium", "", "NullValue", "y" * 19])

    def mask():
        return rng.random(n) < 0.07
    return pa.table({
        "a": pa.array(rng.integers(-1000, 1000, n), mask=mask(), type=pa.int64()),
        "b": pa.array(rng.normal(5.0, 2.0, n), mask=mask(), type=pa.float64()),
        "s": pa.array([None if m else v for v, m in
                       zip(words[rng.integers(0, len(words), n)], mask())], type=pa.string()),
        # read by Completeness only: the loader stages its validity bitmap alone
        "c": pa.array([None if m else f"v{k}" for k, m in enumerate(mask())], type=pa.string()),
    })


def _otable(t):
    from oracle.deequ_oracle import OTable
    return OTable({k: t.column(k).to_pylist() for k in t.column_names},
                  {"a": "long", "b": "double", "s": "string", "c": "string"})


def _clobbered(batch):
    """A copy of a host batch whose buffers are overwritten right after the call that reads it."""
    from deequ_amd.loader import HostColumn
    return {k: HostColumn(c.dtype, c.length, None if c.validity is None else c.validity.copy(),
                          c.values.copy(), None if c.data is None else c.data.copy())
            for k, c in batch.items()}


def _clobber(batch):
    for c in batch.values():
        for buf in (c.validity, c.values, c.data):
            if buf is not None:
                buf.view(np.uint8)[:] = 0xA5


@pytest.mark.parametrize("n,batch", [(30_000, 7_000), (100_003, 16_384)])
def test_scan_host_matches_oracle_and_outlives_host_buffers(n, batch, gpu_device):
    from deequ_amd.analyzers import (ApproxCountDistinct, Completeness, Compliance, Maximum, Mean,
                                     Size, StandardDeviation, Sum)
    from deequ_amd.loader import HostLoader, HostTable
    from deequ_amd.runners.engine import get_plan, read_row
    from deequ_amd import _native as N
    from oracle import deequ_oracle as O
    t = _table(n, n)
    ht = HostTable.from_arrow(t, max_batch_rows=batch)
    assert len(ht.batches) > 2
    suite = [Size(), Sum("a"), Mean("b"), Maximum("b"), StandardDeviation("a"),
             Compliance("in", "s IN ('high','low')"), ApproxCountDistinct("s"), Completeness("c")]
    specs = [s for a in suite for s in a.aggregation_functions()]
    plan = get_plan(ht.schema, specs)
    state = plan.state(0)
    N.check(N.lib.dq_state_reset(state))
    loader = HostLoader(0)
    for b in ht.batches:
        tmp = _clobbered(b)
        loader.scan(plan, state, tmp)
        _clobber(tmp)                       # the caller drops its buffers right away
    row = read_row(plan, state)
    ot = _otable(t)
    off = 0
    got = {}
    for a in suite:
        got[a] = a.from_aggregation_result(row, off)
        off += len(a.aggregation_functions())
    assert got[suite[0]].num_matches == n
    assert got[suite[1]].sum_value == O.agg_sum(ot, "a", None)
    n_, avg, m2 = O.agg_stddev(ot, "a", None)
    st = got[suite[4]]
    assert st.n == n_ and _close(st.avg, avg) and abs(st.m2 - m2) <= 1e-11 * abs(m2)
    assert got[suite[5]].num_matches == O.agg_compliance(ot, "s IN ('high','low')", None)
    assert list(got[suite[6]].words) == O.agg_hll(ot, "s", None)
    assert _close(got[suite[3]].max_value, O.agg_max(ot, "b", None))
    assert got[suite[7]].num_matches == O.agg_sum_notnull(ot, "c", None)


@pytest.mark.parametrize("cols,null_as_group", [(("a",), False), (("s",), False), (("a", "s"), False),
                                                (("s",), True)])
def test_freq_add_host_matches_oracle(cols, null_as_group, gpu_device):
    from deequ_amd.analyzers.grouping import FrequencyTable
    from deequ_amd.loader import HostLoader, HostTable
    from oracle import deequ_oracle as O
    t = _table(40_000, 3)
    ht = HostTable.from_arrow(t, max_batch_rows=9_000)
    ft = FrequencyTable(list(cols), [ht.schema[c].dtype for c in cols], 0)
    loader = HostLoader(0)
    for b in ht.batches:
        tmp = _clobbered(b)
        loader.freq_add(ft, tmp, cols, null_as_group)
        _clobber(tmp)
    if null_as_group:
        exp = {}
        for v in t.column(cols[0]).to_pylist():
            exp[(v,)] = exp.get((v,), 0) + 1  # the NULL group kept apart (tag 0)
    else:
        exp = O.frequencies(_otable(t), list(cols))
    assert dict(ft.export()) == exp
    assert ft.num_rows == t.num_rows
