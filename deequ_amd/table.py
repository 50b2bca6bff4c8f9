"""Columnar handoff: a DataFrame as Arrow-style value / validity / offset buffers in HBM.

The reference analyses a Spark ``DataFrame``; here the unit of data is a :class:`Table`: a schema
plus one or more record batches whose column buffers live in device memory (HBM).  Each column
batch is exactly the Arrow columnar layout (validity bitmap LSB-first, fixed-width values, or
int32 offsets + UTF-8 bytes), so a Spark partition exported through the Arrow C Data Interface
maps onto it without conversion.  Device memory is allocated through torch
(allocation/streams only -- every computation runs in the HIP engine).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _native as N

_ARROW_TO_DQ = {
    "bool": N.BOOL, "int8": N.INT8, "int16": N.INT16, "int32": N.INT32, "int64": N.INT64,
    "float": N.FLOAT32, "double": N.FLOAT64, "string": N.UTF8, "large_string": N.UTF8,
    "binary": N.UTF8, "large_binary": N.UTF8, "date32[day]": N.DATE32,
}
_NP_OF = {N.INT8: np.int8, N.INT16: np.int16, N.INT32: np.int32, N.INT64: np.int64,
          N.FLOAT32: np.float32, N.FLOAT64: np.float64, N.DATE32: np.int32,
          N.TIMESTAMP_US: np.int64}


def arrow_field_type(t):
    """(dq type word, Spark type name override or None, the Arrow type the column is imported as)
    of an Arrow type.  Spark's types map onto the engine's: binary is read as its bytes (hashed,
    grouped and matched exactly like a string, Spark's BinaryType), date64 as date32 days, a
    timestamp of any unit / zone as UTC microseconds (Spark's TimestampType), decimal128(p, s) as
    itself.  Anything else (lists, structs, maps, decimal256, ...) is UNSUPPORTED: only its validity
    bitmap reaches the device."""
    import pyarrow as pa
    key = str(t)
    if key in ("binary", "large_binary"):
        return N.UTF8, "BinaryType", pa.binary()
    if key in _ARROW_TO_DQ:
        return _ARROW_TO_DQ[key], None, t
    if pa.types.is_date64(t):
        return N.DATE32, None, pa.date32()
    if pa.types.is_timestamp(t):
        return N.TIMESTAMP_US, None, pa.timestamp("us", tz=t.tz)
    if pa.types.is_decimal128(t) and 1 <= t.precision <= 38 and 0 <= t.scale <= t.precision:
        return N.decimal_type(t.precision, t.scale), None, t
    return N.UNSUPPORTED, None, t


@dataclass
class StructField:
    name: str
    dtype: int  # dq type word (N.UNSUPPORTED: an Arrow type the engine does not read)
    spark_name: Optional[str] = None  # Spark's type name when the type word does not say it
    arrow_type: Optional[str] = None  # the Arrow type of an UNSUPPORTED column

    @property
    def type_name(self) -> str:
        if self.spark_name:
            return self.spark_name
        if self.dtype == N.UNSUPPORTED:
            return f"UnsupportedType({self.arrow_type})"
        return N.type_name(self.dtype)

    @property
    def engine_type(self) -> int:
        """The type word the engine's plan sees (an UNSUPPORTED column: a validity-only stand-in)."""
        return N.INT8 if self.dtype == N.UNSUPPORTED else self.dtype


@dataclass
class StructType:
    fields: List[StructField]

    @property
    def field_names(self) -> List[str]:
        return [f.name for f in self.fields]

    def __getitem__(self, name: str) -> StructField:
        for f in self.fields:
            if f.name == name:
                return f
        raise KeyError(name)

    def index(self, name: str) -> int:
        return self.field_names.index(name)

    def resolve(self, name: str) -> Optional[str]:
        """Spark resolves column names case-insensitively by default."""
        if name in self.field_names:
            return name
        low = name.lower()
        hits = [f for f in self.field_names if f.lower() == low]
        return hits[0] if len(hits) == 1 else None


@dataclass
class ColumnBatch:
    """One column of one record batch, as device buffers."""
    dtype: int
    length: int
    validity: Optional[object]  # torch.uint8 tensor or None
    values: object              # torch tensor (values / bit-packed bools / int32 offsets)
    data: Optional[object] = None  # torch.uint8 tensor (utf8 bytes)
    null_count: int = 0
    stand_in: bool = False  # an UNSUPPORTED column: validity only, `values` a 16-byte stand-in

    def to_c(self) -> N.dq_column:
        c = N.dq_column()
        c.type = self.dtype
        c.length = self.length
        c.validity = self.validity.data_ptr() if self.validity is not None else None
        c.values = self.values.data_ptr() if self.values is not None else None
        c.data = self.data.data_ptr() if self.data is not None else None
        if self.data is not None and self.data.numel() < (1 << 31):
            c.data_bytes = self.data.numel()  # an upper bound of the string bytes (padding incl.)
        return c

    def nbytes(self) -> int:
        n = 0
        for b in (self.validity, self.values, self.data):
            if b is not None:
                n += b.numel() * b.element_size()
        return n


@dataclass
class Table:
    schema: StructType
    batches: List[Dict[str, ColumnBatch]] = field(default_factory=list)
    device: str = "cuda:0"

    @property
    def columns(self) -> List[str]:
        return self.schema.field_names

    @property
    def num_rows(self) -> int:
        if not self.schema.fields:
            return 0
        first = self.schema.fields[0].name
        return sum(b[first].length for b in self.batches)

    def count(self) -> int:
        return self.num_rows

    def device_index(self) -> int:
        d = str(self.device)
        return int(d.split(":")[1]) if ":" in d else 0

    def select_rows(self, start: int, stop: int) -> "Table":
        """Rows [start, stop) as views of this table's device buffers (used to shard a table across
        ranks).  A batch that straddles a bound is cut; a cut must fall on a multiple of 8 rows
        (bitmaps are byte-addressed views) or ValueError is raised -- rows are never dropped."""
        start, stop = max(0, start), min(self.num_rows, stop)
        out, pos = [], 0
        for b in self.batches:
            n = next(iter(b.values())).length if b else 0
            lo, hi = max(start, pos), min(stop, pos + n)
            if lo < hi:
                if lo == pos and hi == pos + n:
                    out.append(b)
                else:
                    out.append({k: _slice_column(c, lo - pos, hi - pos) for k, c in b.items()})
            pos += n
        if not out:
            out.append({f.name: _empty_column(f.dtype, self.device) for f in self.schema.fields})
        return Table(self.schema, out, self.device)

    # -------------------------------------------------------------------------------------------
    # construction
    # -------------------------------------------------------------------------------------------
    @staticmethod
    def from_arrow(data, device: str = "cuda:0", max_batch_rows: Optional[int] = None) -> "Table":
        """Copies a pyarrow Table / RecordBatch into device buffers (one batch per chunk)."""
        import pyarrow as pa
        if isinstance(data, pa.RecordBatch):
            data = pa.Table.from_batches([data])
        if max_batch_rows:
            batches = data.to_batches(max_chunksize=max_batch_rows)
        else:
            batches = data.combine_chunks().to_batches() if data.num_rows else []
        fields, casts = [], []
        for f in data.schema:
            dtype, spark_name, as_type = arrow_field_type(f.type)
            fields.append(StructField(f.name, dtype, spark_name,
                                      str(f.type) if dtype == N.UNSUPPORTED else None))
            casts.append(as_type if dtype != N.UNSUPPORTED and as_type != f.type else None)
        schema = StructType(fields)
        out = []
        for rb in batches:
            cols = {}
            for f, arr, cast in zip(fields, rb.columns, casts):
                if cast is not None:  # (exact: a cast that would drop digits raises)
                    arr = arr.cast(cast)
                cols[f.name] = _array_to_device(arr, f.dtype, device)
            out.append(cols)
        if not out:
            out.append({f.name: _empty_column(f.dtype, device) for f in fields})
        return Table(schema, out, device)

    @staticmethod
    def from_pydict(columns: Dict[str, Sequence], types: Optional[Dict[str, str]] = None,
                    device: str = "cuda:0") -> "Table":
        """Test helper: python lists (None = NULL) -> device table.  ``types`` maps a column to an
        Arrow type name ("int64", "double", "string", ...) or a pyarrow DataType
        (pa.decimal128(38, 18), pa.timestamp("us"), ...)."""
        import pyarrow as pa
        arrays, names = [], []
        for name, vals in columns.items():
            t = (types or {}).get(name)
            if isinstance(t, str):
                t = getattr(pa, t)()
            arrays.append(pa.array(list(vals), type=t))
            names.append(name)
        return Table.from_arrow(pa.Table.from_arrays(arrays, names=names), device=device)


def _slice_column(c: ColumnBatch, lo: int, hi: int) -> ColumnBatch:
    """Rows [lo, hi) of a device column as views (no copy)."""
    if lo % 8 and lo != hi:
        raise ValueError(f"row slice starts at row {lo} of a batch: cuts must fall on a multiple "
                         f"of 8 rows (bitmap views are byte-addressed)")
    m = hi - lo
    validity = c.validity[lo // 8:] if c.validity is not None else None
    if c.stand_in:
        values = c.values
    elif N.is_decimal(c.dtype):
        values = c.values[2 * lo:]  # two uint64 words per row
    elif c.dtype == N.BOOL:
        values = c.values[lo // 8:]
    elif c.dtype == N.UTF8:
        values = c.values[lo:]  # absolute offsets into the same character buffer
    else:
        values = c.values[lo:]
    # null_count of a view is not recounted (it stays informational: the bitmap is the truth)
    return ColumnBatch(c.dtype, m, validity, values, c.data, 0, c.stand_in)


def _to_device(np_buf: np.ndarray, device: str):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(np_buf))
    return N.retry_on_oom(t.to, device)


def _empty_column(dtype: int, device: str) -> ColumnBatch:
    if dtype == N.UNSUPPORTED:
        return ColumnBatch(N.INT8, 0, None, _to_device(np.zeros(16, np.uint8), device),
                           stand_in=True)
    if dtype == N.UTF8:
        return ColumnBatch(dtype, 0, None, _to_device(np.zeros(1, np.int32), device),
                           _to_device(np.zeros(16, np.uint8), device))
    return ColumnBatch(dtype, 0, None, _to_device(np.zeros(16, np.uint8), device))


def _bits(buf, offset: int, length: int) -> Optional[np.ndarray]:
    """Arrow bitmap (possibly at a bit offset) -> LSB-first packed bitmap starting at bit 0."""
    if buf is None:
        return None
    raw = np.frombuffer(buf, dtype=np.uint8)
    if offset % 8 == 0:
        out = raw[offset // 8: offset // 8 + (length + 7) // 8].copy()
    else:
        bits = np.unpackbits(raw, bitorder="little")[offset: offset + length]
        out = np.packbits(bits, bitorder="little")
    pad = (-len(out)) % 16
    return np.concatenate([out, np.zeros(pad + 16, np.uint8)])


def array_to_host(arr, dtype: int):
    """Arrow array -> (validity, values, data) numpy buffers in the engine's column layout: bitmaps
    re-based to bit 0, string offsets re-based to 0, every buffer zero-padded to a multiple of 16
    bytes (+16) so the vector loads of a batch tail stay inside it.  validity is None without
    NULLs, data None for fixed-width columns."""
    n = len(arr)
    bufs = arr.buffers()
    validity = _bits(bufs[0], arr.offset, n) if arr.null_count else None
    if dtype == N.UNSUPPORTED:  # the validity bitmap alone; a stand-in values buffer
        return validity, np.zeros(16, np.uint8), None
    if N.is_decimal(dtype):  # 16-byte little-endian unscaled values, as two uint64 words each
        vals = np.frombuffer(bufs[1], dtype="<u8")[2 * arr.offset: 2 * (arr.offset + n)]
        return validity, np.concatenate([vals, np.zeros(2, np.uint64)]), None
    if dtype == N.BOOL:
        values = _bits(bufs[1], arr.offset, n)
        if values is None:
            values = np.zeros(16, np.uint8)
        return validity, values, None
    if dtype == N.UTF8:
        import pyarrow as pa
        if str(arr.type) in ("large_string", "large_binary"):
            arr = arr.cast(pa.binary() if "binary" in str(arr.type) else pa.string())
            bufs = arr.buffers()
        offs = np.frombuffer(bufs[1], dtype=np.int32)[arr.offset: arr.offset + n + 1].astype(np.int64)
        base = int(offs[0]) if n else 0
        data = np.frombuffer(bufs[2], dtype=np.uint8)[base: int(offs[-1]) if n else base] \
            if bufs[2] is not None else np.zeros(0, np.uint8)
        offs = (offs - base).astype(np.int32)
        data = np.concatenate([data, np.zeros(16 + (-len(data)) % 16, np.uint8)])
        offs = np.concatenate([offs, np.zeros((-len(offs)) % 4 + 4, np.int32)])
        return validity, offs, data
    npt = _NP_OF[dtype]
    vals = np.frombuffer(bufs[1], dtype=npt)[arr.offset: arr.offset + n]
    pad = (-len(vals)) % (16 // np.dtype(npt).itemsize) + 16 // np.dtype(npt).itemsize
    vals = np.concatenate([vals, np.zeros(pad, npt)])
    return validity, vals, None


def _array_to_device(arr, dtype: int, device: str) -> ColumnBatch:
    validity, values, data = array_to_host(arr, dtype)
    stand_in = dtype == N.UNSUPPORTED
    return ColumnBatch(N.INT8 if stand_in else dtype, len(arr),  # (StructField.engine_type)
                       _to_device(validity, device) if validity is not None else None,
                       _to_device(values, device),
                       _to_device(data, device) if data is not None else None, arr.null_count,
                       stand_in)
