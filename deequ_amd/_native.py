"""ctypes binding of the C ABI in include/deequ_amd.h (libdeequ_amd.so, built in-tree).

The library is the product: there is no CPU fallback.  If it is missing, importing the engine
raises immediately (``build()`` in ``__graft_entry__`` or ``make -C deequ_amd/csrc`` builds it).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char, c_char_p, c_double, c_int, c_int32, c_int64,
                    c_float, c_size_t, c_uint8, c_uint64, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
# DQ_LIB_PATH: diagnostic A/B builds only (tools/); the product loads the in-tree library
LIB_PATH = os.environ.get("DQ_LIB_PATH") or os.path.join(_HERE, "libdeequ_amd.so")

# dq_type (a type word: the dq_type in bits 0-7; a decimal's precision / scale in bits 8-15 / 16-23)
BOOL, INT8, INT16, INT32, INT64, FLOAT32, FLOAT64, UTF8, DECIMAL128, DATE32, TIMESTAMP_US = range(1, 12)
# a column of an Arrow type the engine does not read (list, struct, ...): only its validity bitmap
# reaches the device (Completeness / Size work, anything else is a WrongColumnTypeException)
UNSUPPORTED = 0
TYPE_NAMES = {BOOL: "BooleanType", INT8: "ByteType", INT16: "ShortType", INT32: "IntegerType",
              INT64: "LongType", FLOAT32: "FloatType", FLOAT64: "DoubleType", UTF8: "StringType",
              DATE32: "DateType", TIMESTAMP_US: "TimestampType"}
NUMERIC_TYPES = {INT8, INT16, INT32, INT64, FLOAT32, FLOAT64}
INTEGRAL_TYPES = {INT8, INT16, INT32, INT64}


def type_id(t: int) -> int:
    return t & 0xFF


def decimal_type(precision: int, scale: int) -> int:
    """DQ_DECIMAL_TYPE(p, s): Spark DecimalType(p, s) (1 <= p <= 38, 0 <= s <= p)."""
    if not (1 <= precision <= 38 and 0 <= scale <= precision):
        raise ValueError(f"decimal({precision},{scale}): the engine reads 1 <= p <= 38, 0 <= s <= p")
    return DECIMAL128 | (precision << 8) | (scale << 16)


def is_decimal(t: int) -> bool:
    return t & 0xFF == DECIMAL128


def decimal_precision(t: int) -> int:
    return (t >> 8) & 0xFF


def decimal_scale(t: int) -> int:
    return (t >> 16) & 0xFF


def is_numeric(t: int) -> bool:
    """Preconditions.isNumeric (Analyzer.scala:322-333): Byte .. Double and every DecimalType."""
    return t in NUMERIC_TYPES or is_decimal(t)


def type_name(t: int) -> str:
    """Spark's name of a type word (DecimalType(p,s) with its precision and scale)."""
    if is_decimal(t):
        return f"DecimalType({decimal_precision(t)},{decimal_scale(t)})"
    return TYPE_NAMES.get(t, "UnsupportedType")

# dq_xop
(X_COL, X_NULL, X_BOOL, X_I64, X_F64, X_STR, X_IS_NULL, X_IS_NOT_NULL, X_NOT, X_AND, X_OR, X_EQ,
 X_NE, X_LT, X_LE, X_GT, X_GE, X_EQ_NULL_SAFE, X_IN, X_CAST_F64, X_REGEX, X_CAST_F32,
 X_DEC128) = range(1, 24)

# dq_agg_kind
(AGG_COUNT_ALL, AGG_COUNT_NOTNULL, AGG_COUNT_TRUE, AGG_SUM, AGG_MIN, AGG_MAX, AGG_STDDEV_POP,
 AGG_CORR, AGG_HLL, AGG_DTYPE) = range(1, 11)

# dq_status
DQ_OK = 0
ERR_INVALID_ARGUMENT, ERR_NO_SUCH_COLUMN, ERR_WRONG_TYPE, ERR_OUT_OF_MEMORY, ERR_DEVICE, \
    ERR_UNSUPPORTED, ERR_STATE = range(1, 8)


class dq_column(Structure):
    _fields_ = [("type", c_int32), ("data_bytes", c_int32), ("length", c_int64),
                ("validity", c_void_p), ("values", c_void_p), ("data", c_void_p)]


class dq_expr(Structure):
    _fields_ = [("words", POINTER(c_int64)), ("n_words", c_int32), ("reserved", c_int32)]


class dq_agg(Structure):
    _fields_ = [("kind", c_int32), ("col", c_int32), ("col2", c_int32), ("expr", c_int32),
                ("where", c_int32), ("reserved", c_int32)]


class dq_plan_desc(Structure):
    _fields_ = [("n_columns", c_int32), ("column_types", POINTER(c_int32)), ("n_exprs", c_int32),
                ("exprs", POINTER(dq_expr)), ("n_aggs", c_int32), ("aggs", POINTER(dq_agg))]


class dq_value(Structure):
    _fields_ = [("kind", c_int32), ("is_null", c_int32), ("i64", c_int64), ("f64", c_double * 6),
                ("words", c_uint64 * 52)]


class dq_freq_summary(Structure):
    _fields_ = [("num_rows", c_int64), ("n_groups", c_int64), ("n_unique", c_int64),
                ("n_null_key_rows", c_int64), ("entropy", c_double)]


class EngineError(RuntimeError):
    """A non-OK dq_status, carrying the library's dq_last_error() message."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP engine first (python -c "
            "'import __graft_entry__ as g; g.build()' or make -C deequ_amd/csrc)")
    # One HIP runtime per process: torch's wheel bundles libamdhip64 (soname libamdhip64.so.7).
    # Loading torch first lets our DT_NEEDED libamdhip64.so.7 bind to that same copy; loading
    # /opt/rocm's first would leave two HSA runtimes in the process and the second finds no device.
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "dq_last_error": (c_char_p, []),
        "dq_version": (c_int, []),
        "dq_device_count": (c_int, []),
        "dq_column_from_arrow": (c_int, [c_void_p, c_void_p, POINTER(dq_column)]),
        "dq_plan_create": (c_int, [POINTER(dq_plan_desc), POINTER(c_void_p)]),
        "dq_plan_destroy": (None, [c_void_p]),
        "dq_plan_explain": (c_int, [c_void_p, c_char_p, c_size_t]),
        "dq_plan_launches_per_batch": (c_int, [c_void_p]),
        "dq_state_create": (c_int, [c_void_p, c_int, POINTER(c_void_p)]),
        "dq_state_destroy": (None, [c_void_p]),
        "dq_state_reset": (c_int, [c_void_p]),
        "dq_scan_device": (c_int, [c_void_p, POINTER(dq_column), c_int, c_void_p, c_void_p]),
        "dq_scan_device_batches": (c_int, [c_void_p, POINTER(dq_column), c_int, c_int, c_void_p,
                                           c_void_p]),
        "dq_state_sync": (c_int, [c_void_p]),
        "dq_state_get": (c_int, [c_void_p, c_int, POINTER(dq_value)]),
        "dq_state_get_all": (c_int, [c_void_p, c_int, POINTER(dq_value)]),
        "dq_state_merge": (c_int, [c_void_p, c_void_p]),
        "dq_state_serialized_size": (c_int64, [c_void_p]),
        "dq_state_serialize": (c_int, [c_void_p, c_void_p, c_int64]),
        "dq_state_deserialize": (c_int, [c_void_p, c_void_p, c_int64]),
        "dq_hll_count": (c_double, [POINTER(c_uint64), POINTER(c_int)]),
        "dq_xxhash64": (c_uint64, [c_void_p, c_int64, c_uint64]),
        "dq_column_release": (None, [POINTER(dq_column)]),
        "dq_java_double_to_string": (c_int, [c_double, c_char_p]),
        "dq_java_float_to_string": (c_int, [c_float, c_char_p]),
        "dq_java_doubles_to_strings": (None, [c_void_p, c_int64, c_int, c_void_p, c_void_p]),
        "dq_freq_create": (c_int, [c_int, c_int, POINTER(c_int32), c_int64, POINTER(c_void_p)]),
        "dq_freq_destroy": (None, [c_void_p]),
        "dq_freq_reset": (c_int, [c_void_p, c_void_p]),
        "dq_freq_add_device": (c_int, [c_void_p, POINTER(dq_column), c_int, c_int, c_void_p]),
        "dq_freq_summarize": (c_int, [c_void_p, POINTER(dq_freq_summary)]),
        "dq_freq_summarize_keys": (c_int, [c_void_p, POINTER(dq_freq_summary)]),
        "dq_freq_marginal": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
        "dq_freq_mutual_information": (c_int, [c_void_p, POINTER(c_double), POINTER(c_int),
                                               c_void_p]),
        "dq_sorted_sample": (c_int, [c_int, POINTER(dq_column), c_int, c_int64, c_int64, c_void_p,
                                     POINTER(c_int64), POINTER(c_int64), c_void_p]),
        "dq_freq_num_groups": (c_int, [c_void_p, POINTER(c_int64)]),
        "dq_freq_null_literal": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64)]),
        "dq_release_cached_memory": (None, []),
        "dq_cached_device_bytes": (c_int64, [c_int]),
        "dq_freq_hll": (c_int, [c_void_p, c_int64, c_void_p, POINTER(c_int), c_void_p]),
        "dq_freq_folded_nan_rows": (c_int, [c_void_p, POINTER(c_int64)]),
        "dq_state_exchange_sizes": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64),
                                            POINTER(c_int64), POINTER(c_int64)]),
        "dq_state_exchange_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p]),
        "dq_state_exchange_unpack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_int, c_void_p]),
        "dq_host_wait_count": (c_int64, []),
        "dq_decimal_to_double": (c_double, [c_uint64, c_int64, c_int32]),
        "dq_format_values": (c_int, [c_int32, c_void_p, c_int64, c_void_p, c_void_p]),
        "dq_cast_utf8": (c_int, [POINTER(dq_column), c_int, c_void_p, c_void_p, POINTER(c_int64), c_void_p]),
        "dq_freq_import": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                   c_int64, c_int, c_void_p]),
        "dq_freq_num_rows": (c_int64, [c_void_p]),
        "dq_freq_export": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                   POINTER(c_int64)]),
        "dq_freq_merge": (c_int, [c_void_p, c_void_p]),
        "dq_freq_topk": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int64,
                                 POINTER(c_int64), POINTER(c_int64)]),
        "dq_loader_create": (c_int, [c_int, POINTER(c_void_p)]),
        "dq_loader_destroy": (None, [c_void_p]),
        "dq_loader_stage": (c_int, [c_void_p, POINTER(dq_column), c_int, POINTER(dq_column),
                                    c_void_p]),
        "dq_loader_release": (c_int, [c_void_p, c_void_p]),
        "dq_scan_host": (c_int, [c_void_p, c_void_p, POINTER(dq_column), c_int, c_void_p,
                                 c_void_p]),
        "dq_freq_add_host": (c_int, [c_void_p, c_void_p, POINTER(dq_column), c_int, c_int,
                                     c_void_p]),
        "dq_freq_partition_sizes": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
        "dq_freq_partition": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
        "dq_key_partition": (c_int, [POINTER(dq_column), c_int, c_int, c_int, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
        "dq_freq_add_records_device": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                               c_void_p, c_int64, c_void_p, c_int, c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()

# every symbol the header declares (checked by tests/test_abi.py)
EXPORTED = [
    "dq_last_error", "dq_version", "dq_device_count", "dq_column_from_arrow", "dq_plan_create",
    "dq_plan_destroy", "dq_plan_explain", "dq_plan_launches_per_batch", "dq_state_create",
    "dq_state_destroy", "dq_state_reset", "dq_scan_device", "dq_scan_device_batches",
    "dq_state_sync", "dq_state_get", "dq_state_get_all", "dq_state_merge", "dq_state_serialized_size",
    "dq_state_serialize", "dq_state_deserialize", "dq_hll_count", "dq_xxhash64", "dq_column_release", "dq_java_double_to_string", "dq_java_float_to_string", "dq_java_doubles_to_strings", "dq_freq_create",
    "dq_freq_destroy", "dq_freq_reset", "dq_freq_add_device", "dq_freq_summarize", "dq_freq_summarize_keys", "dq_sorted_sample", "dq_freq_marginal", "dq_freq_mutual_information", "dq_freq_num_groups", "dq_freq_null_literal", "dq_freq_import", "dq_cast_utf8", "dq_release_cached_memory", "dq_cached_device_bytes", "dq_freq_hll", "dq_freq_folded_nan_rows",
    "dq_state_exchange_sizes", "dq_state_exchange_pack", "dq_state_exchange_unpack",
    "dq_host_wait_count", "dq_decimal_to_double", "dq_format_values",
    "dq_freq_num_rows", "dq_freq_export", "dq_freq_merge", "dq_freq_topk", "dq_loader_create",
    "dq_loader_destroy", "dq_loader_stage", "dq_loader_release", "dq_scan_host",
    "dq_freq_add_host", "dq_freq_partition_sizes", "dq_freq_partition",
    "dq_freq_add_records_device", "dq_key_partition",
]
FREQ_RECORD_BYTES = 24  # sizeof(dq_freq_record)


def check(status: int) -> None:
    if status != DQ_OK:
        msg = lib.dq_last_error()
        raise EngineError(status, msg.decode("utf-8", "replace") if msg else f"status {status}")


def device_count() -> int:
    return int(lib.dq_device_count())


def hll_count(words) -> tuple:
    arr = (c_uint64 * 52)(*[w & 0xFFFFFFFFFFFFFFFF for w in words])
    flag = c_int(0)
    est = lib.dq_hll_count(arr, ctypes.byref(flag))
    return est, bool(flag.value)


def xxhash64(data: bytes, seed: int = 42) -> int:
    buf = ctypes.create_string_buffer(data, len(data))
    return int(lib.dq_xxhash64(buf, len(data), seed))


def java_double_to_string(d: float) -> str:
    """Double.toString(d) -- the formatter the device uses (jfmt.h), run on the host."""
    buf = ctypes.create_string_buffer(32)
    n = lib.dq_java_double_to_string(d, buf)
    return buf.raw[:n].decode("ascii")


def java_doubles_to_strings(values, is_float: bool = False) -> list:
    """java_double_to_string (java_float_to_string) of many values in one call."""
    import numpy as np
    v = np.ascontiguousarray(values, np.float64)
    n = len(v)
    out = np.zeros(max(1, n) * 32, np.uint8)
    lens = np.zeros(max(1, n), np.int32)
    lib.dq_java_doubles_to_strings(v.ctypes.data, n, 1 if is_float else 0, out.ctypes.data,
                                   lens.ctypes.data)
    data = out.tobytes()
    return [data[32 * i: 32 * i + ln].decode("ascii") for i, ln in enumerate(lens[:n].tolist())]


def java_float_to_string(f: float) -> str:
    """Float.toString(f) -- the formatter the device uses (jfmt.h), run on the host."""
    buf = ctypes.create_string_buffer(32)
    n = lib.dq_java_float_to_string(f, buf)
    return buf.raw[:n].decode("ascii")


def release_cached_memory() -> None:
    """Frees the engine's cached device blocks (dev_alloc's pool) and torch's cached blocks, so
    either allocator can reclaim memory the other one holds idle."""
    lib.dq_release_cached_memory()
    import torch
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


def retry_on_oom(fn, *args, **kwargs):
    """Runs an idempotent device allocation / call; when torch or the engine runs out of device
    memory, releases both caches and runs it once more (the second failure propagates)."""
    import torch
    try:
        return fn(*args, **kwargs)
    except torch.OutOfMemoryError:
        pass
    except EngineError as e:
        if e.code != ERR_OUT_OF_MEMORY:
            raise
    release_cached_memory()
    return fn(*args, **kwargs)


def decimal_to_double(unscaled: int, scale: int) -> float:
    """Cast(Decimal AS DOUBLE) of one unscaled value (the device's dec_to_double, on the host)."""
    u = unscaled & ((1 << 128) - 1)
    hi = u >> 64
    return float(lib.dq_decimal_to_double(u & 0xFFFFFFFFFFFFFFFF, hi - (1 << 64) if hi >= (1 << 63) else hi,
                                          scale))


def format_values(dtype: int, values) -> list:
    """Spark 2.2's cast to string of date / timestamp / decimal values (dq_format_values): ints of
    days / microseconds, or unscaled ints for a decimal type word."""
    import numpy as np
    n = len(values)
    if is_decimal(dtype):
        raw = np.zeros(2 * max(1, n), np.uint64)
        for i, v in enumerate(values):
            u = int(v) & ((1 << 128) - 1)
            raw[2 * i] = u & 0xFFFFFFFFFFFFFFFF
            raw[2 * i + 1] = u >> 64
    elif dtype == DATE32:
        raw = np.ascontiguousarray(list(values) or [0], np.int32)
    elif dtype == TIMESTAMP_US:
        raw = np.ascontiguousarray(list(values) or [0], np.int64)
    else:
        raise ValueError(f"format_values: type {dtype}")
    out = np.zeros(max(1, n) * 64, np.uint8)
    lens = np.zeros(max(1, n), np.int32)
    check(lib.dq_format_values(dtype, raw.ctypes.data, n, out.ctypes.data, lens.ctypes.data))
    data = out.tobytes()
    return [data[64 * i: 64 * i + ln].decode("ascii") for i, ln in enumerate(lens[:n].tolist())]
