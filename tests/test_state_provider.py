"""HdfsStateProvider (StateProvider.scala:71-294): the reference's on-disk layouts, on CPU -- every
scalar state persists as java.io.DataOutputStream big-endian fields and loads back equal (the
StateProviderTest.scala "restore their state from the filesystem" pattern); the frequency-table
states (Parquet + num_rows.bin) need the device and are in tests/test_gpu_state_provider.py."""
import os
import struct

import pytest

from deequ_amd.analyzers import (ApproxCountDistinct, ApproxQuantile, Completeness, Compliance,
                                 Correlation, DataType, Maximum, Mean, Minimum, PatternMatch, Size,
                                 StandardDeviation, Sum)
from deequ_amd.analyzers.base import NumMatchesAndCount
from deequ_amd.analyzers.datatype import DataTypeHistogram
from deequ_amd.analyzers.quantile import ApproxQuantileState, QuantileSummaries
from deequ_amd.analyzers.scan import (ApproxCountDistinctState, CorrelationState, MaxState,
                                      MeanState, MinState, NumMatches, StandardDeviationState,
                                      SumState)
from deequ_amd.analyzers.state_provider import (HdfsStateProvider, digest_from_bytes,
                                                digest_to_bytes, murmur3_string_hash)

CASES = [
    (Size(), NumMatches(5), ">q"),
    (Completeness("att1"), NumMatchesAndCount(3, 6), ">qq"),
    (Compliance("rule", "att1 = 'b'"), NumMatchesAndCount(2, 6), ">qq"),
    (PatternMatch("att1", r"\d"), NumMatchesAndCount(0, 6), ">qq"),
    (Sum("price"), SumState(-12.5), ">d"),
    (Mean("price"), MeanState(7.25, 4), ">dq"),
    (Minimum("price"), MinState(float("-inf")), ">d"),
    (Maximum("price"), MaxState(1e300), ">d"),
    (StandardDeviation("price"), StandardDeviationState(4.0, 2.5, 1.25), ">3d"),
    (Correlation("count", "price"), CorrelationState(3.0, 1.0, 2.0, 0.5, 0.25, 0.125), ">6d"),
]


@pytest.mark.parametrize("analyzer,state,fmt", CASES, ids=[str(c[0]) for c in CASES])
def test_scalar_states_round_trip_in_reference_layout(analyzer, state, fmt, tmp_path):
    p = HdfsStateProvider(str(tmp_path / "states"))
    p.persist(analyzer, state)
    path = f"{tmp_path}/states-{murmur3_string_hash(str(analyzer), 42)}.bin"
    raw = open(path, "rb").read()
    assert len(raw) == struct.calcsize(fmt)
    assert p.load(analyzer) == state
    with pytest.raises(FileExistsError):  # FileSystem.create(path, overwrite = false)
        p.persist(analyzer, state)
    HdfsStateProvider(str(tmp_path / "states"), allow_overwrite=True).persist(analyzer, state)


def test_byte_states_carry_an_int_length(tmp_path):
    p = HdfsStateProvider(str(tmp_path / "s"))
    words = tuple((i * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF for i in range(52))
    p.persist(ApproxCountDistinct("att1"), ApproxCountDistinctState(words))
    raw = open(f"{tmp_path}/s-{murmur3_string_hash(str(ApproxCountDistinct('att1')), 42)}.bin",
               "rb").read()
    assert struct.unpack(">i", raw[:4])[0] == 416  # HyperLogLogPlusPlusUtils.wordsToBytes
    assert p.load(ApproxCountDistinct("att1")).words == words
    dt = DataTypeHistogram(1, 2, 3, 4, 5)
    p.persist(DataType("item"), dt)
    assert p.load(DataType("item")) == dt


def test_quantile_digest_round_trip(tmp_path):
    import numpy as np
    s = QuantileSummaries.from_sorted(np.arange(1000, dtype=np.float64), 0.01)
    b = digest_to_bytes(s)
    assert struct.unpack(">i", b[:4])[0] == 10000  # compressThreshold
    back = digest_from_bytes(b)
    assert back.count == s.count and back.sampled == s.sampled
    assert back.query(0.5) == s.query(0.5)
    p = HdfsStateProvider(str(tmp_path / "q"))
    p.persist(ApproxQuantile("price", 0.5), ApproxQuantileState(s))
    assert p.load(ApproxQuantile("price", 0.5)).summaries.sampled == s.sampled


def test_murmur3_string_hash_structure():
    """scala.util.hashing.MurmurHash3.stringHash (Scala stdlib, parity unpinned: no reference test
    holds a value): a signed Int, seed-dependent, and sensitive to UTF-16 code-unit order."""
    a = murmur3_string_hash("Size(None)", 42)
    assert -(1 << 31) <= a < (1 << 31)
    assert a != murmur3_string_hash("Size(None)", 43)
    assert murmur3_string_hash("ab", 42) != murmur3_string_hash("ba", 42)
    assert murmur3_string_hash("é€", 42) == murmur3_string_hash("é€", 42)
    assert os.sep  # file names use the decimal Int


def test_missing_state_loads_as_none(tmp_path):
    assert HdfsStateProvider(str(tmp_path / "none")).load(Size()) is None
