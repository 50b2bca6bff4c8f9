"""Bridge from the analyzers' aggregation functions to the HIP engine (the C ABI).

``run_scan(table, specs)`` is the counterpart of ``data.agg(aggregations...).collect().head``
(AnalysisRunner.scala:303, Analyzer.scala:170): it compiles the AggSpecs into one engine plan,
runs the fused scan over every record batch of the table in one launch, and returns the result
row -- one Python value per aggregation, ``None`` where Spark's aggregate would be NULL.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Dict, List, Sequence, Tuple

from .. import _native as N
from ..analyzers.base import AggSpec
from ..exceptions import AnalysisException, WrongColumnTypeException
from ..sqlexpr import SqlError, compile_expr


class Plan:
    """An engine plan (dq_plan*) plus the per-device states created for it."""

    def __init__(self, schema, specs: Sequence[AggSpec]):
        self.schema = schema
        self.specs = list(specs)
        self.types = [f.engine_type for f in schema.fields]
        names = schema.field_names

        def col_index(name: str) -> int:
            resolved = schema.resolve(name)
            if resolved is None:
                raise AnalysisException(
                    f"cannot resolve '`{name}`' given input columns: [{', '.join(names)}]")
            return names.index(resolved)

        expr_sql: List[str] = []
        expr_words: List[List[int]] = []

        def expr_index(sql: str) -> int:
            if sql in expr_sql:
                return expr_sql.index(sql)
            try:
                compiled = compile_expr(sql, schema, col_index)
            except SqlError as e:
                raise AnalysisException(str(e)) from e
            expr_sql.append(sql)
            expr_words.append(compiled.words)
            return len(expr_sql) - 1

        def readable(name: str, kind: int) -> None:
            """An UNSUPPORTED column reaches the device as its validity bitmap only: a
            Completeness numerator reads nothing else; anything more is refused here."""
            f = schema[schema.resolve(name) or name] if schema.resolve(name) else None
            if f is not None and f.dtype == N.UNSUPPORTED and kind != N.AGG_COUNT_NOTNULL:
                raise WrongColumnTypeException(
                    f"Column {f.name} has type {f.type_name}, which the engine does not read")

        aggs = []
        for s in self.specs:
            for c in (s.col, s.col2):
                if c is not None:
                    readable(c, s.kind)
            a = N.dq_agg()
            a.kind = s.kind
            a.col = col_index(s.col) if s.col is not None else -1
            a.col2 = col_index(s.col2) if s.col2 is not None else -1
            a.expr = expr_index(s.expr) if s.expr is not None else -1
            a.where = expr_index(s.where) if s.where is not None else -1
            aggs.append(a)
        self.expr_sql = expr_sql
        # keep the buffers alive for the duration of dq_plan_create
        self._word_bufs = [(ctypes.c_int64 * max(1, len(w)))(*w) for w in expr_words]
        exprs = (N.dq_expr * max(1, len(expr_words)))()
        for i, w in enumerate(expr_words):
            exprs[i].words = ctypes.cast(self._word_bufs[i], ctypes.POINTER(ctypes.c_int64))
            exprs[i].n_words = len(w)
        types = (ctypes.c_int32 * max(1, len(self.types)))(*self.types)
        agg_arr = (N.dq_agg * max(1, len(aggs)))(*aggs)
        desc = N.dq_plan_desc()
        desc.n_columns = len(self.types)
        desc.column_types = types
        desc.n_exprs = len(expr_words)
        desc.exprs = exprs
        desc.n_aggs = len(aggs)
        desc.aggs = agg_arr
        handle = ctypes.c_void_p()
        N.check(N.lib.dq_plan_create(ctypes.byref(desc), ctypes.byref(handle)))
        self.handle = handle
        self._states: Dict[int, ctypes.c_void_p] = {}
        self.lock = threading.Lock()  # one run_scan at a time per cached state

    def __del__(self):
        try:
            for st in self._states.values():
                N.lib.dq_state_destroy(st)
            if getattr(self, "handle", None):
                N.lib.dq_plan_destroy(self.handle)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    def explain(self) -> str:
        buf = ctypes.create_string_buffer(8192)
        N.check(N.lib.dq_plan_explain(self.handle, buf, len(buf)))
        return buf.value.decode()

    @property
    def launches_per_batch(self) -> int:
        return int(N.lib.dq_plan_launches_per_batch(self.handle))

    def state(self, device: int) -> ctypes.c_void_p:
        st = self._states.get(device)
        if st is None:
            st = ctypes.c_void_p()
            N.check(N.lib.dq_state_create(self.handle, device, ctypes.byref(st)))
            self._states[device] = st
        return st


_PLAN_CACHE: Dict[Tuple, Plan] = {}
_LOCK = threading.Lock()


def get_plan(schema, specs: Sequence[AggSpec]) -> Plan:
    key = (tuple((f.name, f.dtype) for f in schema.fields), tuple(specs))
    with _LOCK:
        p = _PLAN_CACHE.get(key)
        if p is None:
            p = Plan(schema, specs)
            _PLAN_CACHE[key] = p
        return p


def column_array(table, plan: Plan):
    """dq_column[n_batches][n_cols] for every batch of the table.  Built once per (table, plan)
    and kept on the table, keyed by the batch objects (a batch's buffers do not change once
    built): rebuilding the ctypes descriptors of every column of every batch cost tens of
    microseconds per scan."""
    n_cols = len(plan.types)
    n_b = len(table.batches)
    cache = table.__dict__.setdefault("_column_arrays", {})
    key = (id(plan), n_cols)
    hit = cache.get(key)
    # (the entry holds the plan and the batches themselves, so their ids cannot be reused)
    if (hit is not None and hit[0] is plan and len(hit[2]) == n_b
            and all(x is y for x, y in zip(hit[2], table.batches))):
        return hit[1], n_cols, n_b
    arr = (N.dq_column * max(1, n_b * n_cols))()
    names = table.schema.field_names
    for b, batch in enumerate(table.batches):
        for c, name in enumerate(names):
            arr[b * n_cols + c] = batch[name].to_c()
    cache[key] = (plan, arr, tuple(table.batches))
    return arr, n_cols, n_b


def current_stream_handle(table):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(table.device).cuda_stream)


def scan_into(table, plan: Plan, state, stream=None) -> None:
    """Enqueues the fused scan of every batch of ``table`` into ``state`` (no sync)."""
    arr, n_cols, n_b = column_array(table, plan)
    if stream is None:
        stream = current_stream_handle(table)
    N.check(N.lib.dq_scan_device_batches(plan.handle, arr, n_cols, n_b, state, stream))


def read_row(plan: Plan, state) -> List[object]:
    N.check(N.lib.dq_state_sync(state))
    n = len(plan.specs)
    vals = plan.__dict__.get("_values")
    if vals is None or len(vals) != max(1, n):
        vals = plan.__dict__["_values"] = (N.dq_value * max(1, n))()
    N.check(N.lib.dq_state_get_all(state, n, vals))
    return [decode_value(spec.kind, vals[i]) for i, spec in enumerate(plan.specs)]


def decode_value(kind: int, v: "N.dq_value"):
    if kind in (N.AGG_COUNT_ALL, N.AGG_COUNT_NOTNULL, N.AGG_COUNT_TRUE):
        return None if v.is_null else int(v.i64)
    if kind in (N.AGG_SUM, N.AGG_MIN, N.AGG_MAX):
        return None if v.is_null else float(v.f64[0])
    if kind == N.AGG_STDDEV_POP:
        return (float(v.f64[0]), float(v.f64[1]), float(v.f64[2]))
    if kind == N.AGG_CORR:
        return tuple(float(v.f64[k]) for k in range(6))
    if kind == N.AGG_DTYPE:
        return tuple(int(v.words[q]) for q in range(5))
    if kind == N.AGG_HLL:
        return tuple(int(w) - (1 << 64) if w >= (1 << 63) else int(w) for w in v.words)
    raise ValueError(kind)


def run_scan(table, specs: Sequence[AggSpec]) -> List[object]:
    """One fused pass over ``table`` computing every aggregation in ``specs``."""
    if not specs:
        return []
    plan = get_plan(table.schema, specs)
    with plan.lock:
        state = plan.state(table.device_index())
        N.check(N.lib.dq_state_reset(state))
        scan_into(table, plan, state)
        return read_row(plan, state)
