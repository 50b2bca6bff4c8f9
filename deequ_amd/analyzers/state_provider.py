"""StateLoader / StatePersister / InMemoryStateProvider / HdfsStateProvider (reference:
analyzers/StateProvider.scala:36-294).  In-memory states are the analyzers' own state objects (device
frequency tables included); HdfsStateProvider writes the reference's on-disk layouts, so a state
persisted here loads in JVM deequ and vice versa:

  {prefix}-{id}.bin          java.io.DataOutputStream, big-endian: Long / Double fields in the
                             reference's order, or Int length + bytes (HLL words, DataType counts,
                             the ApproxQuantile digest)
  {prefix}-{id}-frequencies.pqt   a Parquet directory of the frequency table (the grouping columns
                             + `count`), and {prefix}-{id}-num_rows.bin (Long)

with id = MurmurHash3.stringHash(analyzer.toString, 42) (StateProvider.scala:81-83).  Only local
paths are supported (no HDFS / S3 client in this build).
"""
from __future__ import annotations

import os
import struct
import threading


class StateLoader:
    def load(self, analyzer):
        raise NotImplementedError


class StatePersister:
    def persist(self, analyzer, state) -> None:
        raise NotImplementedError


class InMemoryStateProvider(StateLoader, StatePersister):
    def __init__(self):
        self._states = {}
        self._lock = threading.Lock()

    def load(self, analyzer):
        with self._lock:
            return self._states.get(analyzer)

    def persist(self, analyzer, state) -> None:
        with self._lock:
            self._states[analyzer] = state

    def __str__(self):
        return "".join(f"{a} => {s}\n" for a, s in self._states.items())


# ------------------------------------------------------------------------------------------------
# scala.util.hashing.MurmurHash3.stringHash (Scala 2.11 standard library; not vendored in the
# reference).  The string is hashed as UTF-16 code units, two per 32-bit block (hi << 16) + lo.
# ------------------------------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def _rotl32(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & _M32


def _mix_last(h: int, k: int) -> int:
    k = (k * 0xCC9E2D51) & _M32
    k = _rotl32(k, 15)
    k = (k * 0x1B873593) & _M32
    return h ^ k


def _mix(h: int, k: int) -> int:
    h = _mix_last(h, k)
    h = _rotl32(h, 13)
    return (h * 5 + 0xE6546B64) & _M32


def _avalanche(h: int) -> int:
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    h ^= h >> 16
    return h


def murmur3_string_hash(s: str, seed: int) -> int:
    """MurmurHash3.stringHash(str, seed) as a signed 32-bit Int."""
    units = s.encode("utf-16-be")
    cu = [int.from_bytes(units[i:i + 2], "big") for i in range(0, len(units), 2)]
    h = seed & _M32
    i = 0
    while i + 1 < len(cu):
        h = _mix(h, ((cu[i] << 16) + cu[i + 1]) & _M32)
        i += 2
    if i < len(cu):
        h = _mix_last(h, cu[i])
    h = _avalanche(h ^ len(cu))
    return h - (1 << 32) if h & 0x80000000 else h


# ------------------------------------------------------------------------------------------------
# Spark 2.2 ApproximatePercentile.PercentileDigestSerializer (not vendored): Int compressThreshold,
# Double relativeError, Long count, Int #samples, then (Double value, Long g, Long delta) per
# sample, big-endian (java.nio.ByteBuffer), of the compressed summary.
# ------------------------------------------------------------------------------------------------
COMPRESS_THRESHOLD = 10000  # QuantileSummaries.defaultCompressThreshold
COUNT_COL = "com_amazon_deequ_dq_metrics_count"  # Analyzers.COUNT_COL (Analyzer.scala:338-339)


def digest_to_bytes(summaries) -> bytes:
    s = summaries.compress() if summaries.count else summaries
    out = [struct.pack(">idqi", COMPRESS_THRESHOLD, s.relative_error, s.count, len(s.sampled))]
    out += [struct.pack(">dqq", v, g, d) for v, g, d in s.sampled]
    return b"".join(out)


def digest_from_bytes(b: bytes):
    from .quantile import QuantileSummaries
    _thr, rel, count, n = struct.unpack_from(">idqi", b, 0)
    pos = struct.calcsize(">idqi")
    sampled = []
    for _ in range(n):
        v, g, d = struct.unpack_from(">dqq", b, pos)
        pos += 24
        sampled.append((v, g, d))
    return QuantileSummaries(rel, sampled, count)


class HdfsStateProvider(StateLoader, StatePersister):
    """StateProvider.scala:71-294 on the local filesystem."""

    def __init__(self, location_prefix: str, num_partitions_for_histogram: int = 10,
                 allow_overwrite: bool = False, device: int = 0):
        self.location_prefix = location_prefix
        self.num_partitions_for_histogram = num_partitions_for_histogram
        self.allow_overwrite = allow_overwrite
        self.device = device

    # -- files ------------------------------------------------------------------------------------
    def _identifier(self, analyzer) -> str:
        return str(murmur3_string_hash(str(analyzer), 42))

    def _path(self, ident: str, suffix: str = ".bin") -> str:
        return f"{self.location_prefix}-{ident}{suffix}"

    def _write(self, path: str, data: bytes) -> None:
        # FileSystem.create(path, overwrite): an existing file is an error unless overwriting
        if os.path.exists(path) and not self.allow_overwrite:
            raise FileExistsError(f"{path} already exists")
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "wb") as f:
            f.write(data)

    @staticmethod
    def _read(path: str) -> bytes:
        with open(path, "rb") as f:
            return f.read()

    def _write_bytes(self, ident: str, payload: bytes) -> None:
        self._write(self._path(ident), struct.pack(">i", len(payload)) + payload)

    def _read_bytes(self, ident: str) -> bytes:
        b = self._read(self._path(ident))
        (n,) = struct.unpack_from(">i", b, 0)
        return b[4: 4 + n]

    # -- persist ----------------------------------------------------------------------------------
    def persist(self, analyzer, state) -> None:
        from . import datatype as DT
        from . import grouping as G
        from . import quantile as Q
        from . import scan as S
        ident = self._identifier(analyzer)
        if isinstance(analyzer, S.Size):
            self._write(self._path(ident), struct.pack(">q", state.num_matches))
        elif isinstance(analyzer, (S.Completeness, S.Compliance, S.PatternMatch)):
            self._write(self._path(ident), struct.pack(">qq", state.num_matches, state.count))
        elif isinstance(analyzer, S.Sum):
            self._write(self._path(ident), struct.pack(">d", state.sum_value))
        elif isinstance(analyzer, S.Mean):
            self._write(self._path(ident), struct.pack(">dq", state.sum_value, state.count))
        elif isinstance(analyzer, S.Minimum):
            self._write(self._path(ident), struct.pack(">d", state.min_value))
        elif isinstance(analyzer, S.Maximum):
            self._write(self._path(ident), struct.pack(">d", state.max_value))
        elif isinstance(analyzer, (G.FrequencyBasedAnalyzer, G.Histogram)):
            self._persist_frequencies(analyzer, state, ident)
        elif isinstance(analyzer, DT.DataType):
            self._write_bytes(ident, struct.pack(">5q", state.num_null, state.num_fractional,
                                                 state.num_integral, state.num_boolean,
                                                 state.num_string))
        elif isinstance(analyzer, S.ApproxCountDistinct):
            # HyperLogLogPlusPlusUtils.wordsToBytes: 52 longs, big-endian
            self._write_bytes(ident, struct.pack(">52q", *[_s64(w) for w in state.words]))
        elif isinstance(analyzer, S.Correlation):
            self._write(self._path(ident), struct.pack(">6d", state.n, state.x_avg, state.y_avg,
                                                       state.ck, state.x_mk, state.y_mk))
        elif isinstance(analyzer, S.StandardDeviation):
            self._write(self._path(ident), struct.pack(">3d", state.n, state.avg, state.m2))
        elif isinstance(analyzer, Q.ApproxQuantile):
            self._write_bytes(ident, digest_to_bytes(state.summaries))
        else:
            raise ValueError(f"Unable to persist state for analyzer {analyzer}.")

    def _persist_frequencies(self, analyzer, state, ident: str) -> None:
        import pyarrow as pa
        import pyarrow.parquet as pq
        from . import grouping as G
        path = self._path(ident, "-frequencies.pqt")
        if os.path.exists(path):  # DataFrameWriter's default SaveMode.ErrorIfExists
            raise FileExistsError(f"{path} already exists")
        if isinstance(state, G.HistogramState):
            # the reference's table is already cast to string with NULL -> "NullValue"
            groups = state.string_groups()
            cols = [analyzer.column]
            arrays = [pa.array(list(groups.keys()), type=pa.string())]
            counts = list(groups.values())
        else:
            groups = state.frequencies.export()
            cols = list(state.frequencies.key_columns)
            arrays = [_key_array([k[i] for k, _ in groups], t)
                      for i, t in enumerate(state.frequencies.key_types)]
            counts = [c for _, c in groups]
        # the frequency DataFrame's count column: Analyzers.COUNT_COL for a grouping
        # (GroupingAnalyzers.scala:71), Spark's `.count()` for Histogram (Histogram.scala:66)
        count_col = "count" if isinstance(state, G.HistogramState) else COUNT_COL
        if count_col in cols:  # Spark's Parquet writer refuses duplicate column names
            raise ValueError(f"Found duplicate column(s) in the data schema: `{count_col}`")
        table = pa.table(arrays + [pa.array(counts, type=pa.int64())], names=cols + [count_col])
        os.makedirs(path)
        pq.write_table(table, os.path.join(path, "part-00000.snappy.parquet"), compression="snappy")
        open(os.path.join(path, "_SUCCESS"), "wb").close()
        self._write(self._path(ident, "-num_rows.bin"), struct.pack(">q", state.num_rows))

    # -- load -------------------------------------------------------------------------------------
    def load(self, analyzer):
        from . import base as B
        from . import datatype as DT
        from . import grouping as G
        from . import quantile as Q
        from . import scan as S
        ident = self._identifier(analyzer)
        # a state never persisted loads as None, like InMemoryStateProvider (the reference's
        # Hadoop read would throw; AnalysisRunner persists a grouping's state under its first
        # analyzer only, so runOnAggregatedStates asks for the others too)
        if isinstance(analyzer, (G.FrequencyBasedAnalyzer, G.Histogram)):
            if not os.path.exists(self._path(ident, "-num_rows.bin")):
                return None
            return self._load_frequencies(analyzer, ident)
        if not os.path.exists(self._path(ident)):
            return None
        if isinstance(analyzer, (DT.DataType, S.ApproxCountDistinct, Q.ApproxQuantile)):
            b = self._read_bytes(ident)
            if isinstance(analyzer, DT.DataType):
                return DT.DataTypeHistogram(*struct.unpack(">5q", b))
            if isinstance(analyzer, S.ApproxCountDistinct):
                return S.ApproxCountDistinctState(tuple(w & 0xFFFFFFFFFFFFFFFF
                                                        for w in struct.unpack(">52q", b)))
            return Q.ApproxQuantileState(digest_from_bytes(b))
        b = self._read(self._path(ident))
        if isinstance(analyzer, S.Size):
            return S.NumMatches(*struct.unpack(">q", b[:8]))
        if isinstance(analyzer, (S.Completeness, S.Compliance, S.PatternMatch)):
            return B.NumMatchesAndCount(*struct.unpack(">qq", b[:16]))
        if isinstance(analyzer, S.Sum):
            return S.SumState(*struct.unpack(">d", b[:8]))
        if isinstance(analyzer, S.Mean):
            return S.MeanState(*struct.unpack(">dq", b[:16]))
        if isinstance(analyzer, S.Minimum):
            return S.MinState(*struct.unpack(">d", b[:8]))
        if isinstance(analyzer, S.Maximum):
            return S.MaxState(*struct.unpack(">d", b[:8]))
        if isinstance(analyzer, S.Correlation):
            return S.CorrelationState(*struct.unpack(">6d", b[:48]))
        if isinstance(analyzer, S.StandardDeviation):
            return S.StandardDeviationState(*struct.unpack(">3d", b[:24]))
        raise ValueError(f"Unable to load state for analyzer {analyzer}.")

    def _load_frequencies(self, analyzer, ident: str):
        import pyarrow.parquet as pq
        from . import grouping as G
        from .. import _native as N
        (num_rows,) = struct.unpack(">q", self._read(self._path(ident, "-num_rows.bin"))[:8])
        table = pq.read_table(self._path(ident, "-frequencies.pqt"))
        hist = isinstance(analyzer, G.Histogram)
        count_col = "count" if hist else COUNT_COL
        names = [n for n in table.column_names if n != count_col]
        types = [_from_arrow(table.schema.field(n).type) for n in names]
        keys = list(zip(*[_key_values(table.column(n), t) for n, t in zip(names, types)])) \
            if names else []
        counts = table.column(count_col).to_pylist()
        ft = G.FrequencyTable.from_groups(names, types, self.device, list(zip(keys, counts)),
                                          num_rows=num_rows, null_as_group=hist)
        if hist:
            return G.HistogramState(ft, num_rows, N.UTF8, analyzer.binning_udf)
        return G.FrequenciesAndNumRows(ft, num_rows)


def _s64(w: int) -> int:
    w &= 0xFFFFFFFFFFFFFFFF
    return w - (1 << 64) if w >> 63 else w


def _arrow_types():
    import pyarrow as pa
    from .. import _native as N
    return {N.BOOL: pa.bool_(), N.INT8: pa.int8(), N.INT16: pa.int16(), N.INT32: pa.int32(),
            N.INT64: pa.int64(), N.FLOAT32: pa.float32(), N.FLOAT64: pa.float64(),
            N.UTF8: pa.string()}


class _LazyArrow(dict):
    def __missing__(self, key):
        self.update(_arrow_types())
        return dict.__getitem__(self, key)


_ARROW = _LazyArrow()


def _from_arrow(t) -> int:
    for k, v in _arrow_types().items():
        if v == t:
            return k
    import pyarrow as pa
    from .. import _native as N
    if t == pa.large_string():
        return N.UTF8
    if t == pa.date32():
        return N.DATE32
    if pa.types.is_timestamp(t):
        return N.TIMESTAMP_US
    if pa.types.is_decimal128(t):
        return N.decimal_type(t.precision, t.scale)
    raise ValueError(f"unsupported frequency key type {t}")


def _key_array(values, t: int):
    """A frequency table's key column as the Spark type it holds: dates / timestamps (held as
    days / microseconds) as date32 / timestamp[us], decimals (held unscaled) as decimal128(p, s)."""
    import pyarrow as pa
    from decimal import Decimal
    from .. import _native as N
    if t == N.DATE32:
        return pa.array(values, type=pa.int32()).cast(pa.date32())
    if t == N.TIMESTAMP_US:
        return pa.array(values, type=pa.int64()).cast(pa.timestamp("us"))
    if N.is_decimal(t):
        sc = N.decimal_scale(t)
        return pa.array([None if v is None else Decimal(int(v)).scaleb(-sc) for v in values],
                        type=pa.decimal128(N.decimal_precision(t), sc))
    return pa.array(values, type=_ARROW[t])


def _key_values(column, t: int) -> list:
    """The inverse of _key_array: days / microseconds / unscaled ints."""
    import pyarrow as pa
    from .. import _native as N
    if t == N.DATE32:
        return column.cast(pa.int32()).to_pylist()
    if t == N.TIMESTAMP_US:
        return column.cast(pa.int64()).to_pylist()
    if N.is_decimal(t):
        sc = N.decimal_scale(t)
        return [None if v is None else int(v.scaleb(sc)) for v in column.to_pylist()]
    return column.to_pylist()


__all__ = ["StateLoader", "StatePersister", "InMemoryStateProvider", "HdfsStateProvider",
           "murmur3_string_hash", "digest_to_bytes", "digest_from_bytes"]
