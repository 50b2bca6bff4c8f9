"""Frequency-based analyzers (reference: analyzers/GroupingAnalyzers.scala, Uniqueness.scala,
Distinctness.scala, UniqueValueRatio.scala, CountDistinct.scala, Entropy.scala, Histogram.scala).

The frequency table (``SELECT keys, COUNT(*) ... WHERE keys NOT NULL GROUP BY keys``) is built by
the engine's hash group-by (dq_freq_*), and lives in device memory.  The one aggregation over it
that all ScanShareableFrequencyBasedAnalyzers of a grouping share (AnalysisRunner.scala:490-500)
is the engine's dq_freq_summarize: Σ[count == 1], count(*), Σ −(c/n)·ln(c/n).
"""
from __future__ import annotations

import ctypes
import math
import struct
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .. import _native as N
from ..exceptions import IllegalAnalyzerParameterException, wrap_if_necessary
from ..metrics import Distribution, DistributionValue, Failure, HistogramMetric, Success
from .base import (Analyzer, GroupingAnalyzer, Preconditions, State, empty_state_exception, entity_from,
                   metric_from_empty, metric_from_failure, metric_from_value)


# ------------------------------------------------------------------------------------------------
# Device frequency table
# ------------------------------------------------------------------------------------------------
class FrequencyTable:
    """A dq_freq handle: (key..., count) groups in HBM."""

    def __init__(self, key_columns: Sequence[str], key_types: Sequence[int], device: int,
                 capacity_hint: int = 0):
        self.key_columns = list(key_columns)
        self.key_types = list(key_types)
        self.device = device
        types = (ctypes.c_int32 * len(key_types))(*key_types)
        h = ctypes.c_void_p()
        N.check(N.lib.dq_freq_create(device, len(key_types), types, capacity_hint, ctypes.byref(h)))
        self.handle = h

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                N.lib.dq_freq_destroy(self.handle)
                self.handle = None
        except Exception:  # noqa: BLE001
            pass

    def add(self, columns: Sequence, null_as_group: bool = False, stream=None) -> None:
        arr = (N.dq_column * len(columns))(*[c.to_c() for c in columns])
        if stream is None:
            import torch
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        N.check(N.lib.dq_freq_add_device(self.handle, arr, len(columns), 1 if null_as_group else 0,
                                         stream))

    def reset(self, stream=None) -> None:
        """Empties the table, keeping its device capacity (dq_freq_reset)."""
        if stream is None:
            import torch
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        N.check(N.lib.dq_freq_reset(self.handle, stream))

    @property
    def num_rows(self) -> int:
        return int(N.lib.dq_freq_num_rows(self.handle))

    def summarize(self) -> N.dq_freq_summary:
        s = N.dq_freq_summary()
        N.check(N.lib.dq_freq_summarize(self.handle, ctypes.byref(s)))
        return s

    def count(self) -> int:
        n = ctypes.c_int64()
        N.check(N.lib.dq_freq_num_groups(self.handle, ctypes.byref(n)))
        return int(n.value)

    def hll_words(self, max_records: int):
        """ApproxCountDistinct's 52 register words (signed, as the scan's state holds them) from
        this one-column table's partitioned records (dq_freq_hll), or None when it holds more
        than max_records or is not a one-column table: the caller scans the rows instead."""
        words = (ctypes.c_uint64 * 52)()
        done = ctypes.c_int()
        N.check(N.lib.dq_freq_hll(self.handle, int(max_records), words, ctypes.byref(done), None))
        if not done.value:
            return None
        return tuple(int(w) - (1 << 64) if w >= (1 << 63) else int(w) for w in words)

    def folded_nan_rows(self) -> int:
        """Keyed rows of this Histogram-mode floating-point table whose NaN payload was folded into
        the canonical NaN (dq_freq_folded_nan_rows); 0: its keyed groups are the grouping's;
        -1: not counted."""
        n = ctypes.c_int64()
        N.check(N.lib.dq_freq_folded_nan_rows(self.handle, ctypes.byref(n)))
        return int(n.value)

    def null_literal(self) -> Tuple[int, int]:
        """(rows of the NULL group, count of the "NullValue" string group) of a Histogram table
        (dq_freq_null_literal); the second is 0 unless the key is one string column."""
        nullg, lit = ctypes.c_int64(), ctypes.c_int64()
        N.check(N.lib.dq_freq_null_literal(self.handle, ctypes.byref(nullg), ctypes.byref(lit)))
        return int(nullg.value), int(lit.value)

    def export(self) -> List[Tuple[tuple, int]]:
        """All groups as (key tuple, count); a NULL key component is None."""
        return self.decode_groups(*self.export_raw())

    def export_raw(self):
        """dq_freq_export's arrays: (counts[n], key offsets[n + 1], encoded key bytes)."""
        n = self.count()
        need = ctypes.c_int64()
        N.check(N.lib.dq_freq_export(self.handle, None, None, None, 0, 0, ctypes.byref(need)))
        counts = np.zeros(max(1, n), np.int64)
        offs = np.zeros(n + 1, np.int64)
        raw = np.zeros(max(1, need.value), np.uint8)
        N.check(N.lib.dq_freq_export(self.handle, counts.ctypes.data, offs.ctypes.data,
                                     raw.ctypes.data, n, need.value, ctypes.byref(need)))
        return counts[:n], offs[:n + 1], raw[:need.value]

    def topk(self, k: int) -> List[Tuple[tuple, int]]:
        """The k largest groups by count, descending (dq_freq_topk: only these keys leave the
        device; rdd.top(maxDetailBins) in Histogram.scala:78, ties in any order)."""
        return self.decode_groups(*self.topk_raw(k))

    def topk_raw(self, k: int):
        """dq_freq_topk's arrays: (counts[n], key offsets[n + 1], encoded key bytes)."""
        n, need = ctypes.c_int64(), ctypes.c_int64()
        N.check(N.lib.dq_freq_topk(self.handle, k, None, None, None, 0, ctypes.byref(n),
                                   ctypes.byref(need)))
        counts = np.zeros(max(1, n.value), np.int64)
        offs = np.zeros(n.value + 1, np.int64)
        raw = np.zeros(max(1, need.value), np.uint8)
        N.check(N.lib.dq_freq_topk(self.handle, k, counts.ctypes.data, offs.ctypes.data,
                                   raw.ctypes.data, need.value, ctypes.byref(n),
                                   ctypes.byref(need)))
        return counts[:n.value], offs[:n.value + 1], raw[:need.value]

    def decode_groups(self, counts, offs, raw) -> List[Tuple[tuple, int]]:
        n = len(counts)
        if n and len(self.key_types) == 1:
            return list(zip(self._decode_one_key(n, offs, raw), counts[:n].tolist()))
        data = bytes(raw)
        return [(self._decode(data, int(offs[g])), int(counts[g])) for g in range(n)]

    def _decode_one_key(self, n: int, offs, raw) -> list:
        """The keys of a one-column table's encoded groups, decoded with array operations (the
        per-key struct unpacking of _decode held Histogram's host side for ~1 ms per 1000 keys).
        Same values as _decode."""
        t = self.key_types[0]
        data = bytes(raw)
        words = np.frombuffer(data[: len(data) // 4 * 4], np.uint32)
        at = np.asarray(offs[:n], np.int64) // 4  # encodings start 4-byte aligned
        last = len(words) - 1
        tags = words[at]
        w1 = words[np.minimum(at + 1, last)]
        if _wide_decimal(t):  # 16-byte strings of the unscaled value (dq_freq_export)
            starts = (4 * at + 8).tolist()
            return [(int.from_bytes(data[b: b + 16], "little", signed=True),) if tg else (None,)
                    for b, tg in zip(starts, tags.tolist())]
        if t == N.UTF8:
            starts = (4 * at + 8).tolist()
            return [(data[b: b + ln].decode("utf-8", "replace"),) if tg else (None,)
                    for b, ln, tg in zip(starts, w1.tolist(), tags.tolist())]
        w2 = words[np.minimum(at + 2, last)]
        bits = w1.astype(np.uint64) | (w2.astype(np.uint64) << np.uint64(32))
        if t == N.FLOAT64:
            vals = bits.view(np.float64).tolist()
        elif t == N.FLOAT32:
            vals = w1.view(np.float32).astype(np.float64).tolist()
        elif t == N.BOOL:
            vals = (bits != 0).tolist()
        else:
            vals = bits.view(np.int64).tolist()
        return [(v,) if tg else (None,) for v, tg in zip(vals, tags.tolist())]

    def _decode(self, data: bytes, pos: int) -> tuple:
        key = []
        for t in self.key_types:
            tag = struct.unpack_from("<I", data, pos)[0]
            pos += 4
            if tag == 0:
                key.append(None)
                continue
            if _wide_decimal(t):
                pos += 4  # (the length word: 16)
                key.append(int.from_bytes(data[pos: pos + 16], "little", signed=True))
                pos += 16
            elif t == N.UTF8:
                ln = struct.unpack_from("<I", data, pos)[0]
                pos += 4
                key.append(data[pos: pos + ln].decode("utf-8", "replace"))
                pos += (ln + 3) & ~3
            else:
                v = struct.unpack_from("<Q", data, pos)[0]
                pos += 8
                key.append(_decode_fixed(t, v))
        return tuple(key)

    def marginal(self, key_index: int, stream=None) -> "FrequencyTable":
        """The one-key table of key column `key_index`'s marginal counts over this multi-key
        table's groups (dq_freq_marginal); numRows is this table's."""
        out = FrequencyTable([self.key_columns[key_index]], [self.key_types[key_index]], self.device)
        if stream is None:
            import torch
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        N.check(N.lib.dq_freq_marginal(self.handle, key_index, out.handle, stream))
        return out

    @staticmethod
    def encode_key(key: tuple, key_types: Sequence[int]) -> bytes:
        """A group key in the dq_freq_export format (per column: u32 tag, then 8 value bytes or a
        u32 length + the UTF-8 bytes padded to 4; a decimal(p > 18) key: length 16 + the
        little-endian unscaled value)."""
        out = []
        for v, t in zip(key, key_types):
            if v is None:
                out.append(struct.pack("<I", 0))
            elif _wide_decimal(t):
                out.append(struct.pack("<II", 1, 16) + int(v).to_bytes(16, "little", signed=True))
            elif t == N.UTF8:
                b = v.encode("utf-8")
                out.append(struct.pack("<II", 1, len(b)) + b + b"\0" * ((-len(b)) % 4))
            else:
                out.append(struct.pack("<I", 1) + struct.pack("<Q", _encode_fixed(t, v)))
        return b"".join(out)

    @staticmethod
    def from_groups(key_columns, key_types, device: int, groups, num_rows: int,
                    null_key_rows: int = 0, null_as_group: bool = False,
                    stream=None) -> "FrequencyTable":
        """A table holding the given (key tuple, count) groups (dq_freq_import, the inverse of
        export): how a persisted frequency state is loaded back (StateProvider.scala:270-278)."""
        ft = FrequencyTable(list(key_columns), list(key_types), device)
        keys = [FrequencyTable.encode_key(k, key_types) for k, _ in groups]
        offs = np.zeros(len(keys) + 1, np.int64)
        offs[1:] = np.cumsum([len(k) for k in keys]) if keys else []
        raw = np.frombuffer(b"".join(keys) or b"\0", np.uint8).copy()
        counts = np.ascontiguousarray([c for _, c in groups] or [0], np.int64)
        if stream is None:
            import torch
            stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
        N.check(N.lib.dq_freq_import(ft.handle, counts.ctypes.data, offs.ctypes.data,
                                     raw.ctypes.data, len(keys), int(num_rows), int(null_key_rows),
                                     1 if null_as_group else 0, stream))
        return ft

    def merged(self, other: "FrequencyTable") -> "FrequencyTable":
        out = FrequencyTable(self.key_columns, self.key_types, self.device)
        N.check(N.lib.dq_freq_merge(out.handle, self.handle))
        N.check(N.lib.dq_freq_merge(out.handle, other.handle))
        return out


class KeyedFrequencies:
    """The grouping of one column read off its Histogram-mode table (NULL as a group): the keyed
    groups only, as ``SELECT col, COUNT(*) ... WHERE col IS NOT NULL GROUP BY col`` would give
    (GroupingAnalyzers.scala:62-65).  Valid when the two group-bys put the same non-NULL rows in
    the same groups -- see Histogram.table_serves_grouping."""

    def __init__(self, table: FrequencyTable):
        self.table = table
        self.key_columns = table.key_columns
        self.key_types = table.key_types

    @property
    def num_rows(self) -> int:
        return self.table.num_rows

    def summarize(self) -> N.dq_freq_summary:
        s = N.dq_freq_summary()
        N.check(N.lib.dq_freq_summarize_keys(self.table.handle, ctypes.byref(s)))
        return s

    def export(self) -> List[Tuple[tuple, int]]:
        return [(k, c) for k, c in self.table.export() if k != (None,)]

    def count(self) -> int:
        return int(self.summarize().n_groups)


def _wide_decimal(t: int) -> bool:
    """A decimal(p > 18) key: the table groups it as a 16-byte string of its unscaled value (a
    decimal(p <= 18) key is its unscaled long, a date / timestamp key its int32 / int64)."""
    return N.is_decimal(t) and N.decimal_precision(t) > 18


def _encode_fixed(t: int, v) -> int:
    """The widened 64-bit pattern of a fixed-width key (the inverse of _decode_fixed)."""
    if t == N.FLOAT64:
        return struct.unpack("<Q", struct.pack("<d", v))[0]
    if t == N.FLOAT32:
        return struct.unpack("<I", struct.pack("<f", v))[0]
    if t == N.BOOL:
        return 1 if v else 0
    return int(v) & 0xFFFFFFFFFFFFFFFF


def _decode_fixed(t: int, v: int):
    if t == N.FLOAT64:
        return struct.unpack("<d", struct.pack("<Q", v))[0]
    if t == N.FLOAT32:
        return float(np.frombuffer(struct.pack("<I", v & 0xFFFFFFFF), np.float32)[0])
    if t == N.BOOL:
        return bool(v)
    return v - (1 << 64) if v >= (1 << 63) else v


# ------------------------------------------------------------------------------------------------
# State
# ------------------------------------------------------------------------------------------------
@dataclass
class FrequenciesAndNumRows(State):
    """GroupingAnalyzers.scala:124-157"""
    frequencies: FrequencyTable
    num_rows: int

    def sum(self, other: "FrequenciesAndNumRows") -> "FrequenciesAndNumRows":
        return FrequenciesAndNumRows(self.frequencies.merged(other.frequencies),
                                     self.num_rows + other.num_rows)


def compute_frequencies(data, grouping_columns: Sequence[str],
                        num_rows: Optional[int] = None) -> FrequenciesAndNumRows:
    """FrequencyBasedAnalyzer.computeFrequencies (GroupingAnalyzers.scala:53-80)."""
    types = [data.schema[c].dtype for c in grouping_columns]
    table = FrequencyTable(grouping_columns, types, data.device_index(),
                           capacity_hint=data.num_rows)  # sized once: no growth copies
    for batch in data.batches:
        table.add([batch[c] for c in grouping_columns])
    n = num_rows if num_rows is not None else data.count()
    return FrequenciesAndNumRows(table, n)


# ------------------------------------------------------------------------------------------------
# Analyzers
# ------------------------------------------------------------------------------------------------
class FrequencyBasedAnalyzer(GroupingAnalyzer):
    """GroupingAnalyzers.scala:29-45"""

    def _columns(self) -> List[str]:
        raise NotImplementedError

    def grouping_columns(self) -> List[str]:
        return list(self._columns())

    def compute_state_from(self, data):
        return compute_frequencies(data, self.grouping_columns())

    def preconditions(self) -> List[Callable]:
        cols = self._columns()
        return [Preconditions.at_least_one(cols)] + [Preconditions.has_column(c) for c in cols] + \
            super().preconditions()


@dataclass(frozen=True)
class FreqAgg:
    """One aggregation over the frequency table."""
    kind: str  # "unique", "distinct", "count", "entropy"


def frequency_row(summary: "N.dq_freq_summary", aggs: Sequence[FreqAgg], num_rows: int) -> list:
    """Evaluates the shared aggregation over the frequency table (Spark semantics: a sum over an
    empty table is NULL, count(*) is 0)."""
    empty = summary.n_groups == 0
    row = []
    for a in aggs:
        if a.kind == "unique":
            row.append(None if empty else float(summary.n_unique))
        elif a.kind == "distinct":
            row.append(None if empty else float(summary.n_groups))
        elif a.kind == "count":
            row.append(int(summary.n_groups))
        elif a.kind == "entropy":
            row.append(None if empty else float(summary.entropy))
        elif a.kind == "unique_ratio_of_rows":
            row.append(None if empty else float(summary.n_unique) / num_rows)
        elif a.kind == "distinct_ratio_of_rows":
            row.append(None if empty else float(summary.n_groups) / num_rows)
        else:
            raise ValueError(a.kind)
    return row


class ScanShareableFrequencyBasedAnalyzer(FrequencyBasedAnalyzer):
    """GroupingAnalyzers.scala:84-121"""

    _name = ""

    def aggregation_functions(self, num_rows: int) -> List[FreqAgg]:
        raise NotImplementedError

    def _instance(self) -> str:
        return ",".join(self._columns())

    def compute_metric_from(self, state):
        if state is None:
            return metric_from_empty(self, self._name, self._instance(), entity_from(self._columns()))
        aggs = self.aggregation_functions(state.num_rows)
        row = frequency_row(state.frequencies.summarize(), aggs, state.num_rows)
        return self.from_aggregation_result(row, 0)

    def to_failure_metric(self, exception):
        return metric_from_failure(exception, self._name, self._instance(),
                                   entity_from(self._columns()))

    def to_success_metric(self, value: float):
        return metric_from_value(value, self._name, self._instance(), entity_from(self._columns()))

    def from_aggregation_result(self, result, offset):
        if result[offset] is None:
            return metric_from_empty(self, self._name, self._instance(), entity_from(self._columns()))
        return self.to_success_metric(float(result[offset]))


def _cols(columns) -> Tuple[str, ...]:
    return (columns,) if isinstance(columns, str) else tuple(columns)


@dataclass(frozen=True)
class Uniqueness(ScanShareableFrequencyBasedAnalyzer):
    """Uniqueness.scala:26-32: Σ[count == 1] / numRows"""
    columns: Tuple[str, ...]
    _name = "Uniqueness"

    def __init__(self, columns):
        object.__setattr__(self, "columns", _cols(columns))

    def _columns(self):
        return list(self.columns)

    def aggregation_functions(self, num_rows):
        return [FreqAgg("unique_ratio_of_rows")]


@dataclass(frozen=True)
class Distinctness(ScanShareableFrequencyBasedAnalyzer):
    """Distinctness.scala:29-35: Σ[count >= 1] / numRows"""
    columns: Tuple[str, ...]
    _name = "Distinctness"

    def __init__(self, columns):
        object.__setattr__(self, "columns", _cols(columns))

    def _columns(self):
        return list(self.columns)

    def aggregation_functions(self, num_rows):
        return [FreqAgg("distinct_ratio_of_rows")]


@dataclass(frozen=True)
class UniqueValueRatio(ScanShareableFrequencyBasedAnalyzer):
    """UniqueValueRatio.scala:25-38: Σ[count == 1] / count(*)"""
    columns: Tuple[str, ...]
    _name = "UniqueValueRatio"

    def __init__(self, columns):
        object.__setattr__(self, "columns", _cols(columns))

    def _columns(self):
        return list(self.columns)

    def aggregation_functions(self, num_rows):
        return [FreqAgg("unique"), FreqAgg("count")]

    def from_aggregation_result(self, result, offset):
        if result[offset] is None:
            # Row.getDouble on a NULL slot throws in the reference -> failure metric
            raise TypeError(f"Value at index {offset} is null")
        unique, distinct = float(result[offset]), float(result[offset + 1])
        return self.to_success_metric(unique / distinct if distinct else float("nan"))


@dataclass(frozen=True)
class CountDistinct(ScanShareableFrequencyBasedAnalyzer):
    """CountDistinct.scala:24-34: count(*) over the groups"""
    columns: Tuple[str, ...]
    _name = "CountDistinct"

    def __init__(self, columns):
        object.__setattr__(self, "columns", _cols(columns))

    def _columns(self):
        return list(self.columns)

    def aggregation_functions(self, num_rows):
        return [FreqAgg("count")]

    def from_aggregation_result(self, result, offset):
        return self.to_success_metric(float(result[offset]))


@dataclass(frozen=True)
class Entropy(ScanShareableFrequencyBasedAnalyzer):
    """Entropy.scala:28-42: Σ −(c/numRows)·ln(c/numRows)"""
    column: str
    _name = "Entropy"

    def _columns(self):
        return [self.column]

    def __str__(self):
        return f"Entropy({self.column})"

    def aggregation_functions(self, num_rows):
        return [FreqAgg("entropy")]


@dataclass(frozen=True)
class MutualInformation(FrequencyBasedAnalyzer):
    """MutualInformation.scala:35-97: sum over the joint groups of
    (pxy/n) ln((pxy/n) / ((px/n)(py/n))), the marginals re-aggregated from the joint table
    (dq_freq_mutual_information: marginals and the join on the device, the reference's per-group
    arithmetic, a fixed-order sum)."""
    columns: Tuple[str, ...]
    _name = "MutualInformation"

    def __init__(self, columns, column_b: Optional[str] = None):
        cols = (columns, column_b) if column_b is not None else _cols(columns)
        object.__setattr__(self, "columns", tuple(cols))

    def _columns(self):
        return list(self.columns)

    def preconditions(self):
        return [Preconditions.exactly_n_columns(list(self.columns), 2)] + super().preconditions()

    def _instance(self):
        return ",".join(self.columns)

    def compute_metric_from(self, state):
        if state is None:
            return metric_from_empty(self, self._name, self._instance(), entity_from(self.columns))
        joint = state.frequencies
        if isinstance(joint, FrequencyTable):  # the reference's per-group terms, on the device
            mi, null = ctypes.c_double(), ctypes.c_int()
            import torch
            stream = ctypes.c_void_p(torch.cuda.current_stream(joint.device).cuda_stream)
            N.check(N.lib.dq_freq_mutual_information(joint.handle, ctypes.byref(mi),
                                                     ctypes.byref(null), stream))
            if null.value:  # sum over no joint groups is NULL
                return metric_from_empty(self, self._name, self._instance(),
                                         entity_from(self.columns))
            return metric_from_value(mi.value, self._name, self._instance(),
                                     entity_from(self.columns))
        # a repartitioned (multi-GPU) joint table: H(X) + H(Y) - H(X,Y), the same sum regrouped,
        # from the three distributed entropies (a value's groups may sit on several ranks)
        s = joint.summarize()
        if s.n_groups == 0:
            return metric_from_empty(self, self._name, self._instance(), entity_from(self.columns))
        hx = _marginal_entropy(joint, 0)
        hy = _marginal_entropy(joint, 1)
        return metric_from_value(hx + hy - s.entropy, self._name, self._instance(),
                                 entity_from(self.columns))

    def to_failure_metric(self, exception):
        return metric_from_failure(exception, self._name, self._instance(),
                                   entity_from(self.columns))


def _marginal_entropy(joint, k: int) -> float:
    from ..distributed import DistributedFrequencies, freq_repartition
    if isinstance(joint, DistributedFrequencies):  # a value's groups may sit on several ranks
        return DistributedFrequencies(freq_repartition(joint.owned.marginal(k))).summarize().entropy
    return joint.marginal(k).summarize().entropy


# ------------------------------------------------------------------------------------------------
# Histogram (Histogram.scala:41-116)
# ------------------------------------------------------------------------------------------------
NULL_FIELD_REPLACEMENT = "NullValue"
MAXIMUM_ALLOWED_DETAIL_BINS = 1000


def java_double_to_string(d: float) -> str:
    """Java Double.toString (Spark 2.2 Cast(DoubleType -> StringType)): the formatter the device
    runs for PatternMatch over a double column (csrc/jfmt.h: shortest round-trip digits, Java's
    plain / E-notation layout).  JDK 8's few non-shortest outputs are parity unpinned (jfmt.h)."""
    return N.java_double_to_string(float(d))


def java_float_to_string(f: float) -> str:
    """Java Float.toString (Cast(FloatType -> StringType)), the device formatter on the host."""
    return N.java_float_to_string(float(f))


def cast_to_string(value, dtype: int) -> str:
    """Spark 2.2's Cast(x AS STRING) of a key (Histogram.scala:63).  Date / timestamp / decimal
    keys are held as their days / microseconds / unscaled value and formatted by the engine's
    formatter (dq_format_values: BigDecimal.toString, yyyy-MM-dd, yyyy-MM-dd HH:mm:ss[.f] UTC)."""
    if value is None:
        return NULL_FIELD_REPLACEMENT
    if dtype == N.UTF8:
        return value
    if dtype in (N.DATE32, N.TIMESTAMP_US) or N.is_decimal(dtype):
        return N.format_values(dtype, [int(value)])[0]
    if dtype == N.BOOL:
        return "true" if value else "false"
    if dtype == N.FLOAT64:
        return java_double_to_string(value)
    if dtype == N.FLOAT32:
        return java_float_to_string(value)
    return str(int(value))


def _python_dtype(value, column_dtype: int) -> int:
    """Type of a binning UDF's result, for its cast to string."""
    if value is None or isinstance(value, str):
        return N.UTF8
    if isinstance(value, bool):
        return N.BOOL
    if isinstance(value, float):
        return N.FLOAT64
    if isinstance(value, int):
        return N.INT64
    return column_dtype


_INT_KEY_TYPES = (N.INT8, N.INT16, N.INT32, N.INT64)


def _int_key_strings(counts, offs, raw) -> List[Tuple[str, int]]:
    """(Cast(key AS STRING), count) of a one-integer-column table's encoded groups (tag word, then
    the value as 8 little-endian bytes: dq_freq_export), NULL keys dropped; the values
    _decode_one_key gives, formatted as cast_to_string does."""
    n = len(counts)
    if not n:
        return []
    data = bytes(raw)
    words = np.frombuffer(data[: len(data) // 4 * 4], np.uint32)
    at = np.asarray(offs[:n], np.int64) // 4
    last = len(words) - 1
    tags = words[at]
    bits = (words[np.minimum(at + 1, last)].astype(np.uint64) |
            (words[np.minimum(at + 2, last)].astype(np.uint64) << np.uint64(32))).view(np.int64)
    keep = tags != 0
    return list(zip(map(str, bits[keep].tolist()), np.asarray(counts[:n])[keep].tolist()))


def _fold_null_group(frequencies, dtype: int, k: int):
    """Histogram's details and numberOfBins from a table whose NULL rows form a group kept apart:
    na.fill("NullValue") (Histogram.scala:59-66) makes them one group with any real "NullValue"
    string, so that group's count is the sum of both (dq_freq_null_literal) and it is placed by
    that count among the device top-N (ties in any order, like rdd.top)."""
    if dtype in _INT_KEY_TYPES and hasattr(frequencies, "topk_raw"):
        # integer keys: decoded and cast to their digits with array operations, no per-key
        # tuples (configs[2]'s id Histogram: ~0.4 -> 0.15 ms of host time per step)
        top = _int_key_strings(*frequencies.topk_raw(k + 2))
        nullg, lit = frequencies.null_literal()  # (after topk: the same finalize serves both)
        kept = None
    else:
        raw = frequencies.topk(k + 2)  # up to two raw entries fold into one
        nullg, lit = frequencies.null_literal()  # (after topk: the same finalize serves both)
        kept = [(key, c) for (key,), c in raw
                if not (key is None or (dtype == N.UTF8 and key == NULL_FIELD_REPLACEMENT))]
    if kept is None:
        pass
    elif dtype in (N.FLOAT64, N.FLOAT32):  # Double/Float.toString of every key in one call
        texts = N.java_doubles_to_strings([k for k, _ in kept], dtype == N.FLOAT32)
        top = [(s, c) for s, (_, c) in zip(texts, kept)]
    elif dtype in (N.DATE32, N.TIMESTAMP_US) or N.is_decimal(dtype):  # one formatter call
        texts = N.format_values(dtype, [k for k, _ in kept])
        top = [(s, c) for s, (_, c) in zip(texts, kept)]
    elif dtype == N.UTF8:
        top = kept
    elif dtype == N.BOOL:
        top = [("true" if k else "false", c) for k, c in kept]
    else:  # integers: the decimal digits (cast_to_string per key held Histogram's host side for
        # ~0.6 ms per 1000 keys, inside configs[2]'s step)
        top = [(str(k), c) for k, c in kept]
    folded = nullg + lit
    if folded:
        at = next((i for i, (_, c) in enumerate(top) if c < folded), len(top))
        top.insert(at, (NULL_FIELD_REPLACEMENT, folded))
    bins = frequencies.count() - (1 if nullg and lit else 0)
    return top[:k], bins


@dataclass
class HistogramState(FrequenciesAndNumRows):
    dtype: int = N.UTF8
    binning_udf: Optional[Callable] = None

    def string_groups(self) -> dict:
        """Every group keyed by Spark's cast-to-string of the (binned) value, NULL -> "NullValue"
        (Histogram.scala:59-66).  The binning function is host code (a Spark UDF in the
        reference), so it runs on the distinct values after the device group-by."""
        out: dict = {}
        for (key,), cnt in self.frequencies.export():
            if self.binning_udf is not None:
                key = self.binning_udf(key)
                s = cast_to_string(key, _python_dtype(key, self.dtype))
            else:
                s = cast_to_string(key, self.dtype)
            out[s] = out.get(s, 0) + cnt
        return out

    def as_string_table(self) -> "HistogramState":
        """The same state keyed by the cast-to-string values, NULL -> "NullValue" (the reference's
        own state: a persisted Histogram state loads back like this)."""
        if self.dtype == N.UTF8 and self.binning_udf is None:
            return self
        groups = [((k,), c) for k, c in self.string_groups().items()]
        col = self.frequencies.key_columns[0]
        ft = FrequencyTable.from_groups([col], [N.UTF8], self.frequencies.device, groups,
                                        self.frequencies.num_rows, null_as_group=True)
        return HistogramState(ft, self.num_rows, N.UTF8, None)

    def sum(self, other):
        a, b = self, other
        if a.dtype != b.dtype or (a.binning_udf is None) != (b.binning_udf is None):
            a, b = a.as_string_table(), b.as_string_table()  # e.g. one side loaded from disk
        return HistogramState(a.frequencies.merged(b.frequencies),
                              a.num_rows + b.num_rows, a.dtype, a.binning_udf)


@dataclass(frozen=True)
class Histogram(Analyzer):
    """Not a GroupingAnalyzer in the reference: it runs as its own jobs (AnalysisRunner.scala:
    321-323)."""
    column: str
    binning_udf: Optional[Callable] = None
    max_detail_bins: int = MAXIMUM_ALLOWED_DETAIL_BINS

    def __str__(self):
        udf = "None" if self.binning_udf is None else f"Some({self.binning_udf})"
        return f"Histogram({self.column},{udf},{self.max_detail_bins})"

    def grouping_columns(self):
        return [self.column]

    def _param_check(self, _schema):
        if self.max_detail_bins > MAXIMUM_ALLOWED_DETAIL_BINS:
            raise IllegalAnalyzerParameterException(
                f"Cannot return histogram values for more than {MAXIMUM_ALLOWED_DETAIL_BINS} values")

    def preconditions(self):
        return [self._param_check, Preconditions.has_column(self.column)]

    @staticmethod
    def table_serves_grouping(data, column: str) -> bool:
        """Can this column's Histogram table also serve its grouping (Uniqueness, Distinctness,
        Entropy, ... on [column])?  Integral, boolean and string columns: their NULL rows form a
        separate group that the keyed view drops (a string column's NULL group is folded into the
        "NullValue" string only when Histogram reads the table, _fold_null_group).
        Floating-point columns too, provisionally: Histogram folds NaN payloads (cast to string)
        and the grouping does not, so the table serves the grouping only when it folded no row
        (FrequencyTable.folded_nan_rows() == 0, checked by the runner after the table is built;
        otherwise the grouping runs its own group-by)."""
        dtype = data.schema[column].dtype
        # (date / timestamp / decimal: their casts to string are injective, so the string groups
        # and the value groups are the same groups)
        return (dtype in (N.BOOL, N.INT8, N.INT16, N.INT32, N.INT64, N.UTF8, N.FLOAT32, N.FLOAT64,
                          N.DATE32, N.TIMESTAMP_US) or N.is_decimal(dtype))

    def compute_state_from(self, data):
        from ..distributed import compute_frequencies_distributed, is_distributed
        dtype = data.schema[self.column].dtype
        if is_distributed(data):  # each rank's partial groupBy, repartitioned by owner rank
            st = compute_frequencies_distributed(data, [self.column], null_as_group=True)
            return HistogramState(st.frequencies, st.num_rows, dtype, self.binning_udf)
        total = data.count()
        table = FrequencyTable([self.column], [dtype], data.device_index(), capacity_hint=total)
        for batch in data.batches:
            table.add([batch[self.column]], null_as_group=True)
        return HistogramState(table, total, dtype, self.binning_udf)

    def compute_metric_from(self, state):
        if state is None:
            return HistogramMetric(self.column, Failure(empty_state_exception(self)))
        try:
            if state.binning_udf is None:
                # device top-N: only max_detail_bins groups reach the host (Histogram.scala:78-79)
                top, bins = _fold_null_group(state.frequencies, state.dtype, self.max_detail_bins)
            else:
                groups = state.string_groups()
                # rdd.top(maxDetailBins)(OrderByAbsoluteCount): ties are arbitrary in the reference
                top = sorted(groups.items(), key=lambda kv: (-kv[1], kv[0]))[: self.max_detail_bins]
                bins = len(groups)
            details = {k: DistributionValue(c, c / state.num_rows) for k, c in top}
            return HistogramMetric(self.column, Success(Distribution(details, bins)))
        except Exception as e:  # noqa: BLE001
            return HistogramMetric(self.column, Failure(wrap_if_necessary(e)))

    def to_failure_metric(self, exception):
        return HistogramMetric(self.column, Failure(wrap_if_necessary(exception)))


__all__ = ["FrequencyTable", "KeyedFrequencies", "FrequenciesAndNumRows", "MutualInformation", "compute_frequencies",
           "FrequencyBasedAnalyzer", "ScanShareableFrequencyBasedAnalyzer", "Uniqueness",
           "Distinctness", "UniqueValueRatio", "CountDistinct", "Entropy", "Histogram",
           "HistogramState", "java_double_to_string", "java_float_to_string", "cast_to_string"]
