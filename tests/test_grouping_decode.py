"""FrequencyTable's array decode of one-key group encodings (dq_freq_export / dq_freq_topk
layout: a u32 tag, then a u32 length + bytes padded to 4 for utf8, or the 8-byte widened value)
agrees with the per-key struct decoder.  Host only."""
import struct

import numpy as np
import pytest

from deequ_amd import _native as N
from deequ_amd.analyzers.grouping import FrequencyTable, _encode_fixed


def _encode(t, keys):
    raw, offs = bytearray(), []
    for k in keys:
        offs.append(len(raw))
        if k is None:
            raw += struct.pack("<I", 0)
        elif t == N.UTF8:
            b = k.encode("utf-8")
            raw += struct.pack("<II", 1, len(b)) + b + b"\0" * ((-len(b)) % 4)
        else:
            raw += struct.pack("<IQ", 1, _encode_fixed(t, k))
    offs.append(len(raw))
    return np.array(offs, np.int64), np.frombuffer(bytes(raw), np.uint8)


@pytest.mark.parametrize("t,keys", [
    (N.UTF8, ["a", "", "Thingy abcdefgh", None, "é€x", "NullValue"]),
    (N.INT64, [0, -1, 2**63 - 1, -2**63, None, 42]),
    (N.INT32, [7, -7, None]),
    (N.FLOAT64, [0.0, -0.0, 1.5, float("inf"), float("-inf"), None, 1e-310]),
    (N.FLOAT32, [0.5, -3.25, None, 1e38]),
    (N.BOOL, [True, False, None]),
])
def test_one_key_decode_matches_per_key_decoder(t, keys):
    ft = object.__new__(FrequencyTable)
    ft.key_types = [t]
    offs, raw = _encode(t, keys)
    counts = np.arange(1, len(keys) + 1, dtype=np.int64)
    fast = ft.decode_groups(counts, offs, raw)
    data = bytes(raw)
    slow = [(ft._decode(data, int(offs[g])), int(counts[g])) for g in range(len(keys))]
    assert [(k, c) for k, c in fast] == slow
    for (k,), _ in fast:  # the same Python types as the per-key decoder
        assert k is None or type(k) in (str, int, float, bool)
