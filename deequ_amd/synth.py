"""Synthetic "Item" tables (examples/entities.scala:19-25).

Counter-based, integer-only recipe, identical on the GPU (csrc/synth.hip, libdq_synth.so) and in
numpy here, so any row range of a 1e9-row device table can be regenerated on the host:

    mix(z)        = splitmix64 finaliser
    S(c, k)       = mix(seed * 0x1000193 + 64 c + k)               (per column / draw stream)
    rnd(c, k, r)  = mix(S(c, k) ^ (r * 0xD1B54A32D192ED03))
    NULL          : rnd(c, 0, r) % 100 < 5                         (i.i.d. 5 % per column)
    id            : (int64) mix(r ^ 0x5DEECE66D)                   (a bijection: all unique)
    name          : "Thingy " + 4..8 letters
    priority      : ["high", "low", "medium"][rnd(3, 1, r) % 3]
    numViews      : g = ctz(rnd(4,1,r) | 2^40); v = (1024 g + (rnd(4,2,r) & 1023)) * 2 // 3,
                    negated when rnd(4, 3, r) % 100 == 0           (≈ Exponential, mean ≈ 1000)
    score (extra) : numViews * 0.5 + (rnd(5, 1, r) & 0xFFFF) / 65536   (fp64, for Correlation)
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import numpy as np

from . import _native as N
from .table import ColumnBatch, StructField, StructType, Table

ID, NAME, DESC, PRIORITY, NUMVIEWS, SCORE = range(6)
_M64 = (1 << 64) - 1
PRIORITIES = ["high", "low", "medium"]


def _mix_int(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def streams(seed: int) -> List[List[int]]:
    return [[_mix_int((seed * 0x1000193 + c * 64 + k) & _M64) for k in range(4)] for c in range(8)]


def _rnd(s: int, rows: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        return _mix(np.uint64(s) ^ (rows * np.uint64(0xD1B54A32D192ED03)))


def _ctz(x: np.ndarray) -> np.ndarray:
    low = x & (~x + np.uint64(1))  # lowest set bit
    return np.log2(low.astype(np.float64)).astype(np.int64)


def item_columns_numpy(n: int, seed: int = 7, start: int = 0, extra: bool = False) -> dict:
    """Host restatement of the device generator for rows [start, start + n): dict of numpy
    arrays (values, validity masks, string lists)."""
    st = streams(seed)
    rows = np.arange(start, start + n, dtype=np.uint64)
    out = {}
    valid = lambda c: (_rnd(st[c][0], rows) % np.uint64(100)) >= np.uint64(5)  # noqa: E731
    out["id_valid"] = valid(ID)
    out["id"] = np.where(out["id_valid"], _mix(rows ^ np.uint64(0x5DEECE66D)).view(np.int64), 0)
    h1 = _rnd(st[NUMVIEWS][1], rows) | np.uint64(1 << 40)
    h2 = _rnd(st[NUMVIEWS][2], rows)
    g = _ctz(h1)
    v = ((g << 10) + (h2 & np.uint64(1023)).astype(np.int64)) * 2 // 3
    neg = (_rnd(st[NUMVIEWS][3], rows) % np.uint64(100)) == np.uint64(0)
    v = np.where(neg, -v, v)
    out["numViews_valid"] = valid(NUMVIEWS)
    out["numViews"] = np.where(out["numViews_valid"], v, 0).astype(np.int64)
    if extra:
        out["score_valid"] = valid(SCORE)
        h = _rnd(st[SCORE][1], rows)
        sc = v.astype(np.float64) * 0.5 + (h & np.uint64(0xFFFF)).astype(np.float64) / 65536.0
        out["score"] = np.where(out["score_valid"], sc, 0.0)
    out["name_valid"] = valid(NAME)
    lens = (_rnd(st[NAME][1], rows) % np.uint64(5)).astype(np.int64) + 4
    hn = _rnd(st[NAME][2], rows)
    letters = np.stack([((hn >> np.uint64(8 * k)) & np.uint64(0xFF)) % np.uint64(26) for k in range(8)],
                       axis=1).astype(np.uint8) + ord("a")
    names = [None] * n
    nv = out["name_valid"]
    for i in range(n):
        if nv[i]:
            names[i] = "Thingy " + letters[i, : lens[i]].tobytes().decode()
    out["name"] = names
    out["priority_valid"] = valid(PRIORITY)
    code = (_rnd(st[PRIORITY][1], rows) % np.uint64(3)).astype(np.int64)
    out["priority_code"] = code
    pv = out["priority_valid"]
    out["priority"] = [PRIORITIES[code[i]] if pv[i] else None for i in range(n)]
    return out


def item_table_arrow(n: int, seed: int = 7, start: int = 0, extra: bool = False):
    import pyarrow as pa
    c = item_columns_numpy(n, seed, start, extra)
    arrays = [
        pa.array(c["id"], mask=~c["id_valid"], type=pa.int64()),
        pa.array(c["name"], type=pa.string()),
        pa.array(c["priority"], type=pa.string()),
        pa.array(c["numViews"], mask=~c["numViews_valid"], type=pa.int64()),
    ]
    names = ["id", "name", "priority", "numViews"]
    if extra:
        arrays.append(pa.array(c["score"], mask=~c["score_valid"], type=pa.float64()))
        names.append("score")
    return pa.Table.from_arrays(arrays, names=names)


# ------------------------------------------------------------------------------------------------
# device generator
# ------------------------------------------------------------------------------------------------
_SYNTH = None


def _synth_lib():
    global _SYNTH
    if _SYNTH is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdq_synth.so")
        lib = ctypes.CDLL(path)
        vp, i64, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64
        lib.dq_synth_fixed.argtypes = [u64, u64, i64] + [vp] * 11
        lib.dq_synth_fixed.restype = ctypes.c_int
        lib.dq_synth_strings.argtypes = [u64, u64, i64, vp, vp, vp, vp, vp]
        lib.dq_synth_strings.restype = ctypes.c_int
        _SYNTH = lib
    return _SYNTH


def item_table_device(n: int, seed: int = 7, batch_rows: int = 1 << 26, device: str = "cuda:0",
                      extra: bool = False, start: int = 0) -> Table:
    """Generates rows [start, start + n) of the Item table directly in HBM, in batches of
    ``batch_rows`` rows (int32 string offsets per batch)."""
    import torch
    lib = _synth_lib()
    dev = torch.device(device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    fields = [StructField("id", N.INT64), StructField("name", N.UTF8),
              StructField("priority", N.UTF8), StructField("numViews", N.INT64)]
    if extra:
        fields.append(StructField("score", N.FLOAT64))
    batches = []
    pos = 0
    while pos < n:
        m = min(batch_rows, n - pos)
        words = (m + 63) // 64 + 2
        u64 = lambda: torch.zeros(words, dtype=torch.int64, device=dev)  # noqa: E731
        idv, id_valid = torch.empty(m + 2, dtype=torch.int64, device=dev), u64()
        views, views_valid = torch.empty(m + 2, dtype=torch.int64, device=dev), u64()
        score = torch.empty(m + 2, dtype=torch.float64, device=dev) if extra else None
        score_valid = u64() if extra else None
        name_len = torch.empty(m, dtype=torch.int32, device=dev)
        prio_len = torch.empty(m, dtype=torch.int32, device=dev)
        name_valid, prio_valid = u64(), u64()
        rc = lib.dq_synth_fixed(seed, start + pos, m, idv.data_ptr(), id_valid.data_ptr(),
                                views.data_ptr(), views_valid.data_ptr(),
                                score.data_ptr() if extra else None,
                                score_valid.data_ptr() if extra else None, name_len.data_ptr(),
                                name_valid.data_ptr(), prio_len.data_ptr(), prio_valid.data_ptr(),
                                stream)
        if rc:
            raise RuntimeError(f"dq_synth_fixed failed ({rc})")
        name_off = torch.zeros(m + 4, dtype=torch.int32, device=dev)
        prio_off = torch.zeros(m + 4, dtype=torch.int32, device=dev)
        name_off[1: m + 1] = torch.cumsum(name_len, 0, dtype=torch.int64).to(torch.int32)
        prio_off[1: m + 1] = torch.cumsum(prio_len, 0, dtype=torch.int64).to(torch.int32)
        name_bytes = int(name_off[m].item())
        prio_bytes = int(prio_off[m].item())
        name_data = torch.zeros(name_bytes + 16, dtype=torch.uint8, device=dev)
        prio_data = torch.zeros(prio_bytes + 16, dtype=torch.uint8, device=dev)
        rc = lib.dq_synth_strings(seed, start + pos, m, name_off.data_ptr(), name_data.data_ptr(),
                                  prio_off.data_ptr(), prio_data.data_ptr(), stream)
        if rc:
            raise RuntimeError(f"dq_synth_strings failed ({rc})")
        u8 = lambda t: t.view(torch.uint8)  # noqa: E731
        b = {
            "id": ColumnBatch(N.INT64, m, u8(id_valid), idv),
            "name": ColumnBatch(N.UTF8, m, u8(name_valid), name_off, name_data),
            "priority": ColumnBatch(N.UTF8, m, u8(prio_valid), prio_off, prio_data),
            "numViews": ColumnBatch(N.INT64, m, u8(views_valid), views),
        }
        if extra:
            b["score"] = ColumnBatch(N.FLOAT64, m, u8(score_valid), score)
        batches.append(b)
        pos += m
    torch.cuda.synchronize(dev)
    return Table(StructType(fields), batches, device)


def item_buffers_numpy(n: int, seed: int = 7, start: int = 0) -> dict:
    """Arrow-style host buffers of the S10 columns for rows [start, start + n) without building
    Python strings (for the CPU baseline): packed validity bitmaps, numViews values, priority
    offsets + bytes."""
    st = streams(seed)
    rows = np.arange(start, start + n, dtype=np.uint64)
    valid = lambda c: (_rnd(st[c][0], rows) % np.uint64(100)) >= np.uint64(5)  # noqa: E731
    pack = lambda m: np.concatenate([np.packbits(m, bitorder="little"), np.zeros(16, np.uint8)])  # noqa
    out = {"n": n}
    out["id_valid"] = pack(valid(ID))
    out["name_valid"] = pack(valid(NAME))
    vv = valid(NUMVIEWS)
    out["numViews_valid"] = pack(vv)
    h1 = _rnd(st[NUMVIEWS][1], rows) | np.uint64(1 << 40)
    h2 = _rnd(st[NUMVIEWS][2], rows)
    v = ((_ctz(h1) << 10) + (h2 & np.uint64(1023)).astype(np.int64)) * 2 // 3
    neg = (_rnd(st[NUMVIEWS][3], rows) % np.uint64(100)) == np.uint64(0)
    out["numViews"] = np.where(vv, np.where(neg, -v, v), 0).astype(np.int64)
    pv = valid(PRIORITY)
    code = (_rnd(st[PRIORITY][1], rows) % np.uint64(3)).astype(np.int64)
    lens = np.where(pv, np.array([4, 3, 6])[code], 0).astype(np.int64)
    off = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    out["priority_valid"] = pack(pv)
    out["priority_offsets"] = off.astype(np.int32)
    table = np.frombuffer(b"high\0\0low\0\0\0medium", np.uint8).reshape(3, 6)
    starts = np.repeat(off[:-1], lens)
    within = np.arange(int(off[-1]), dtype=np.int64) - starts
    codes = np.repeat(code, lens)
    out["priority_data"] = np.concatenate([table[codes, within], np.zeros(16, np.uint8)])
    return out


def profiling_table_device(n: int, batch_rows: int = 1 << 26, device: str = "cuda:0",
                           start: int = 0) -> Table:
    """BASELINE configs[4]'s table: 20 mixed columns generated in HBM -- 10 numeric (id; numViews
    of five Item tables with different seeds; score of four) and 10 strings (name and priority of
    three Item tables; four `description` columns = name + a prefix that carries an https URL in
    about half the rows, the containsURL workload).  Every column has ~5 % NULLs."""
    import torch
    lib = _synth_lib()
    if not hasattr(lib, "_describe_ready"):
        vp = ctypes.c_void_p
        lib.dq_synth_describe.argtypes = [ctypes.c_uint64, ctypes.c_int64, vp, vp, vp, vp, vp]
        lib.dq_synth_describe.restype = ctypes.c_int
        lib._describe_ready = True
    parts = [item_table_device(n, seed=100 + k, batch_rows=batch_rows, device=device, extra=True,
                               start=start) for k in range(5)]
    dev = torch.device(device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    fields = [StructField("id", N.INT64)]
    fields += [StructField(f"numViews_{k}", N.INT64) for k in range(5)]
    fields += [StructField(f"score_{k}", N.FLOAT64) for k in range(4)]
    fields += [StructField(f"name_{k}", N.UTF8) for k in range(3)]
    fields += [StructField(f"priority_{k}", N.UTF8) for k in range(3)]
    fields += [StructField(f"description_{k}", N.UTF8) for k in range(4)]
    batches = []
    pos = start  # (rows [start, start + n): a rank's shard of the same table)
    for bi in range(len(parts[0].batches)):
        b = {"id": parts[0].batches[bi]["id"]}
        for k in range(5):
            b[f"numViews_{k}"] = parts[k].batches[bi]["numViews"]
        for k in range(4):
            b[f"score_{k}"] = parts[k].batches[bi]["score"]
        for k in range(3):
            b[f"name_{k}"] = parts[k].batches[bi]["name"]
            b[f"priority_{k}"] = parts[k].batches[bi]["priority"]
        for k in range(4):
            src = parts[k + 1].batches[bi]["name"]
            m = src.length
            rows = torch.arange(pos, pos + m, dtype=torch.int64, device=dev)
            url = ((rows * -7046029254386353131) >> 62) & 1  # bit 62 of r * 0x9E3779B97F4A7C15
            lens = (src.values[1: m + 1] - src.values[:m]).to(torch.int64) + torch.where(
                url.bool(), torch.tensor(33, device=dev), torch.tensor(9, device=dev))
            off = torch.zeros(m + 4, dtype=torch.int32, device=dev)
            off[1: m + 1] = torch.cumsum(lens, 0).to(torch.int32)
            data = torch.zeros(int(off[m].item()) + 16, dtype=torch.uint8, device=dev)
            rc = lib.dq_synth_describe(pos, m, src.values.data_ptr(), src.data.data_ptr(),
                                       off.data_ptr(), data.data_ptr(), stream)
            if rc:
                raise RuntimeError(f"dq_synth_describe failed ({rc})")
            b[f"description_{k}"] = ColumnBatch(N.UTF8, m, src.validity, off, data)
        batches.append(b)
        pos += parts[0].batches[bi]["id"].length
    torch.cuda.synchronize(dev)
    return Table(StructType(fields), batches, device)
