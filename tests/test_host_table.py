"""Host-side layout of the loader's input (deequ_amd.loader.HostTable, table.array_to_host): no
GPU.  Bitmaps re-based to bit 0 for sliced arrays, string offsets re-based to 0, buffers padded to
16 bytes, and the dq_column pointers/lengths the C ABI receives."""
import numpy as np
import pyarrow as pa

from deequ_amd import _native as N
from deequ_amd.loader import HostTable


def test_sliced_arrays_are_rebased():
    t = pa.table({"x": pa.array([1, None, 3, 4, None, 6, 7, 8, 9, 10], type=pa.int64()),
                  "s": pa.array(["a", "bb", None, "ddd", "", "f", "g", "h", "i", "j"])})
    ht = HostTable.from_arrow(t.slice(3, 6))
    b = ht.batches[0]
    x, s = b["x"], b["s"]
    assert x.length == 6 and s.length == 6
    bits = np.unpackbits(x.validity, bitorder="little")[:6]
    assert bits.tolist() == [1, 0, 1, 1, 1, 1]          # rows 3..8: 4, None, 6, 7, 8, 9
    assert x.values[0] == 4 and x.values[2] == 6 and x.values[5] == 9
    assert s.values[0] == 0                              # offsets re-based
    strs = [bytes(s.data[s.values[i]:s.values[i + 1]]).decode() for i in range(6)]
    assert strs == ["ddd", "", "f", "g", "h", "i"]
    assert s.validity is None                            # no NULL in the slice
    for c in (x, s):
        for buf in (c.validity, c.values, c.data):
            if buf is not None:
                assert buf.nbytes % 16 == 0


def test_dq_column_points_at_the_host_buffers():
    t = pa.table({"b": pa.array([True, False, None]), "f": pa.array([1.5, None, 2.5])})
    ht = HostTable.from_arrow(t, max_batch_rows=2)
    assert [b["b"].length for b in ht.batches] == [2, 1]
    c = ht.batches[0]["f"].to_c()
    assert c.type == N.FLOAT64 and c.length == 2
    assert c.values == ht.batches[0]["f"].values.ctypes.data
    assert ht.num_rows == 3
