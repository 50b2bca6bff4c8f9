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
    assert st.n == n_ and _close(st.avg, avg) and abs(st.m2 - m2) <= 1e-12 * abs(m2)
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


@pytest.mark.parametrize("offset", [0, 8, 5, 3000])
def test_sliced_arrow_export_scans_like_the_unsliced_copy(offset, gpu_device):
    """A Spark partition exported through the Arrow C Data Interface may be a slice (non-zero
    ArrowArray.offset): imported by dq_column_from_arrow (HostTable.from_arrow_c) and scanned by
    dq_scan_host it must give the state of the same rows exported unsliced, and the oracle's."""
    from deequ_amd.analyzers import (ApproxCountDistinct, Completeness, Compliance, Maximum, Mean,
                                     Size, StandardDeviation, Sum)
    from deequ_amd.loader import HostTable, run_scan_host
    from oracle import deequ_oracle as O
    n = 40_000
    t = _table(n + 64, offset + 1)
    f = pa.array(np.arange(n + 64) % 3 == 0, mask=np.arange(n + 64) % 7 == 0)
    t = t.append_column("f", f)
    # (offset 3000: the strings start ~30 KB into the data buffer; the loader stages only the
    # bytes from the slice's first offset, rounded down to 256)
    sliced = [rb.slice(offset, min(n // 2, rb.num_rows - offset))
              for rb in t.to_batches(max_chunksize=(n + 64) // 2)]
    copies = [pa.Table.from_batches([rb]).combine_chunks().to_batches()[0] for rb in sliced]
    copies = [pa.RecordBatch.from_arrays([pa.array(c.to_pylist(), c.type) for c in rb.columns],
                                         schema=rb.schema) for rb in copies]
    assert all(c.offset == 0 for rb in copies for c in rb.columns)
    assert offset == 0 or all(c.offset == offset for c in sliced[0].columns)
    suite = [Size(), Completeness("a"), Completeness("s"), Completeness("f"),
             Compliance("pos", "a > 0"), Compliance("f", "f"), Sum("a"), Mean("b"),
             StandardDeviation("b"), Maximum("b"), ApproxCountDistinct("s"),
             Compliance("in", "s IN ('high','low')")]
    specs = [sp for an in suite for sp in an.aggregation_functions()]
    row_sliced = run_scan_host(HostTable.from_arrow_c(sliced), specs)
    row_copy = run_scan_host(HostTable.from_arrow_c(copies), specs)
    assert row_sliced == row_copy
    whole = pa.Table.from_batches(sliced)
    ot = O.OTable({k: whole.column(k).to_pylist() for k in whole.column_names},
                  {"a": "long", "b": "double", "s": "string", "c": "string", "f": "boolean"})
    got, off = {}, 0
    for an in suite:
        got[an] = an.from_aggregation_result(row_sliced, off)
        off += len(an.aggregation_functions())
    assert got[suite[0]].num_matches == whole.num_rows
    assert got[suite[1]].num_matches == O.agg_sum_notnull(ot, "a", None)
    assert got[suite[2]].num_matches == O.agg_sum_notnull(ot, "s", None)
    assert got[suite[3]].num_matches == O.agg_sum_notnull(ot, "f", None)
    assert got[suite[4]].num_matches == O.agg_compliance(ot, "a > 0", None)
    assert got[suite[6]].sum_value == O.agg_sum(ot, "a", None)
    assert _close(got[suite[9]].max_value, O.agg_max(ot, "b", None))
    assert list(got[suite[10]].words) == O.agg_hll(ot, "s", None)
    assert got[suite[11]].num_matches == O.agg_compliance(ot, "s IN ('high','low')", None)


def test_device_bitmap_at_a_bit_offset_is_rebased_on_the_device(gpu_device):
    """dq_column_from_arrow over DEVICE buffers at a bit offset: the validity bitmap is re-based
    on the device (cast.hip bitmap_rebase_kernel) into a library-owned buffer."""
    import ctypes

    import torch

    from deequ_amd import _native as N
    from deequ_amd.loader import ArrowArrayC, ArrowSchemaC
    rng = np.random.default_rng(9)
    n, off = 10_000, 13
    mask = rng.random(n + off) < 0.3
    arr = pa.array(rng.integers(0, 9, n + off), mask=mask, type=pa.int64())
    bufs = arr.buffers()
    dev = [torch.from_numpy(np.frombuffer(b, np.uint8).copy()).to(gpu_device) for b in bufs]
    ptrs = (ctypes.c_void_p * 2)(dev[0].data_ptr(), dev[1].data_ptr())
    a = ArrowArrayC(length=n, null_count=int(mask[off:].sum()), offset=off, n_buffers=2,
                    n_children=0, buffers=ptrs)
    s = ArrowSchemaC(format=b"l", name=b"x", flags=2)
    col = N.dq_column()
    N.check(N.lib.dq_column_from_arrow(ctypes.addressof(a), ctypes.addressof(s), ctypes.byref(col)))
    assert col.values == dev[1].data_ptr() + 8 * off
    assert col.validity != dev[0].data_ptr()
    out = np.zeros((n + 7) // 8, np.uint8)
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.synchronize()
    assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(col.validity),
                         ctypes.c_size_t(len(out)), 2) == 0
    got = np.unpackbits(out, bitorder="little")[:n].astype(bool)
    assert (got == ~mask[off:]).all()
    N.lib.dq_column_release(ctypes.byref(col))
