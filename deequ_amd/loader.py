"""Host-resident Arrow batches through the engine's columnar loader (dq_loader_*, dq_scan_host,
dq_freq_add_host; loader.cpp): the path a Spark partition's Arrow export takes through the JNI
shim.  Each batch is copied into a pinned staging slot, DMA'd to HBM on the
loader's copy stream and scanned on the caller's stream, so batch k+1's transfer overlaps batch
k's scan.  Host buffers may be dropped as soon as each call returns (include/deequ_amd.h).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _native as N
from .table import _ARROW_TO_DQ, StructField, StructType, array_to_host


@dataclass
class HostColumn:
    """One column of one batch in host memory (numpy buffers, engine layout)."""
    dtype: int
    length: int
    validity: Optional[np.ndarray]
    values: np.ndarray
    data: Optional[np.ndarray] = None

    def to_c(self) -> N.dq_column:
        c = N.dq_column()
        c.type = self.dtype
        c.length = self.length
        c.validity = self.validity.ctypes.data if self.validity is not None else None
        c.values = self.values.ctypes.data
        c.data = self.data.ctypes.data if self.data is not None else None
        if self.data is not None and self.data.nbytes < (1 << 31):
            c.data_bytes = self.data.nbytes
        return c

    def nbytes(self) -> int:
        return sum(b.nbytes for b in (self.validity, self.values, self.data) if b is not None)


class ArrowSchemaC(ctypes.Structure):
    pass


class ArrowArrayC(ctypes.Structure):
    pass


ArrowSchemaC._fields_ = [("format", ctypes.c_char_p), ("name", ctypes.c_char_p),
                         ("metadata", ctypes.c_char_p), ("flags", ctypes.c_int64),
                         ("n_children", ctypes.c_int64),
                         ("children", ctypes.POINTER(ctypes.POINTER(ArrowSchemaC))),
                         ("dictionary", ctypes.POINTER(ArrowSchemaC)),
                         ("release", ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowSchemaC))),
                         ("private_data", ctypes.c_void_p)]
ArrowArrayC._fields_ = [("length", ctypes.c_int64), ("null_count", ctypes.c_int64),
                        ("offset", ctypes.c_int64), ("n_buffers", ctypes.c_int64),
                        ("n_children", ctypes.c_int64),
                        ("buffers", ctypes.POINTER(ctypes.c_void_p)),
                        ("children", ctypes.POINTER(ctypes.POINTER(ArrowArrayC))),
                        ("dictionary", ctypes.POINTER(ArrowArrayC)),
                        ("release", ctypes.CFUNCTYPE(None, ctypes.POINTER(ArrowArrayC))),
                        ("private_data", ctypes.c_void_p)]


class ArrowColumn:
    """One host pyarrow array handed to the engine through the Arrow C Data Interface, as the JNI
    shim hands a Spark partition's export: exported with _export_to_c and
    imported by dq_column_from_arrow, which honours ArrowArray.offset (sliced arrays).  Keeps the
    export alive until the engine column is released."""

    def __init__(self, arr):
        self.array = ArrowArrayC()
        self.schema = ArrowSchemaC()
        arr._export_to_c(ctypes.addressof(self.array), ctypes.addressof(self.schema))
        self.column = N.dq_column()
        try:
            N.check(N.lib.dq_column_from_arrow(ctypes.addressof(self.array),
                                               ctypes.addressof(self.schema),
                                               ctypes.byref(self.column)))
        except Exception:
            self._release_export()
            raise
        self.dtype = int(self.column.type)
        self.length = int(self.column.length)

    def to_c(self) -> N.dq_column:
        return self.column

    def _release_export(self):
        for s in (self.array, self.schema):
            if s.release:
                s.release(ctypes.byref(s))

    def __del__(self):
        try:
            N.lib.dq_column_release(ctypes.byref(self.column))
            self._release_export()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class HostTable:
    """Record batches of host columns (the host counterpart of table.Table)."""

    def __init__(self, schema: StructType, batches: List[Dict[str, HostColumn]]):
        self.schema = schema
        self.batches = batches

    @property
    def num_rows(self) -> int:
        if not self.schema.fields or not self.batches:
            return 0
        first = self.schema.fields[0].name
        return sum(b[first].length for b in self.batches)

    def nbytes(self) -> int:
        return sum(c.nbytes() for b in self.batches for c in b.values())

    @staticmethod
    def from_arrow(data, max_batch_rows: Optional[int] = None) -> "HostTable":
        import pyarrow as pa
        if isinstance(data, pa.RecordBatch):
            data = pa.Table.from_batches([data])
        if max_batch_rows:
            batches = data.to_batches(max_chunksize=max_batch_rows)
        else:
            batches = data.combine_chunks().to_batches() if data.num_rows else []
        fields = []
        for f in data.schema:
            key = str(f.type)
            if key not in _ARROW_TO_DQ:
                raise TypeError(f"unsupported Arrow type {f.type} for column {f.name}")
            fields.append(StructField(f.name, _ARROW_TO_DQ[key]))
        out = []
        for rb in batches:
            cols = {}
            for f, arr in zip(fields, rb.columns):
                v, vals, d = array_to_host(arr, f.dtype)
                cols[f.name] = HostColumn(f.dtype, len(arr), v, vals, d)
            out.append(cols)
        return HostTable(StructType(fields), out)

    @staticmethod
    def from_arrow_c(batches, schema=None) -> "HostTable":
        """Record batches (or sliced ones) imported through the Arrow C Data Interface, buffers
        aliased where the engine can (ArrowColumn): the JNI shim's path."""
        import pyarrow as pa
        batches = list(batches)
        schema = schema or batches[0].schema
        fields = []
        for f in schema:
            if f.type == pa.large_string():
                raise TypeError(f"column {f.name}: large_string has 64-bit offsets")
            fields.append(StructField(f.name, _ARROW_TO_DQ[str(f.type)]))
        out = [{f.name: ArrowColumn(rb.column(i)) for i, f in enumerate(fields)} for rb in batches]
        return HostTable(StructType(fields), out)


class HostLoader:
    """A dq_loader: two pinned + device staging slots on one device (one per thread / stream)."""

    def __init__(self, device: int = 0):
        self.device = device
        h = ctypes.c_void_p()
        N.check(N.lib.dq_loader_create(device, ctypes.byref(h)))
        self.handle = h

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                N.lib.dq_loader_destroy(self.handle)
                self.handle = None
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    def _stream(self, stream):
        if stream is not None:
            return stream
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def scan(self, plan, state, batch: Dict[str, HostColumn], stream=None) -> None:
        """dq_scan_host: stage one host batch and enqueue its fused scan into ``state``."""
        names = plan.schema.field_names
        arr = (N.dq_column * max(1, len(names)))(*[batch[n].to_c() for n in names])
        N.check(N.lib.dq_scan_host(self.handle, plan.handle, arr, len(names), state,
                                   self._stream(stream)))

    def freq_add(self, table, batch: Dict[str, HostColumn], columns: Sequence[str],
                 null_as_group: bool = False, stream=None) -> None:
        """dq_freq_add_host: stage one host batch's key columns and group them into ``table``."""
        arr = (N.dq_column * len(columns))(*[batch[c].to_c() for c in columns])
        N.check(N.lib.dq_freq_add_host(self.handle, table.handle, arr, len(columns),
                                       1 if null_as_group else 0, self._stream(stream)))


def run_scan_host(host_table: HostTable, specs, device: int = 0,
                  loader: Optional[HostLoader] = None) -> list:
    """runners.engine.run_scan over host batches: one fused scan per batch through the loader,
    all into one state (the per-batch partials merge in the state, in batch order)."""
    from .runners.engine import get_plan, read_row
    if not specs:
        return []
    plan = get_plan(host_table.schema, specs)
    state = plan.state(device)
    N.check(N.lib.dq_state_reset(state))
    loader = loader or HostLoader(device)
    for b in host_table.batches:
        loader.scan(plan, state, b)
    return read_row(plan, state)


def compute_frequencies_host(host_table: HostTable, columns: Sequence[str], device: int = 0,
                             null_as_group: bool = False, loader: Optional[HostLoader] = None):
    """The frequency table of ``columns`` over host batches (dq_freq_add_host per batch)."""
    from .analyzers.grouping import FrequencyTable
    types = [host_table.schema[c].dtype for c in columns]
    table = FrequencyTable(list(columns), types, device)
    loader = loader or HostLoader(device)
    for b in host_table.batches:
        loader.freq_add(table, b, columns, null_as_group)
    return table


__all__ = ["ArrowColumn", "HostColumn", "HostTable", "HostLoader", "run_scan_host", "compute_frequencies_host"]
