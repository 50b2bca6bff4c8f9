"""Pins the ORACLE against the reference's own known answers (tests/golden/
reference_known_answers.json, every case citing its reference test file:line) and against the
independent `xxhash` package."""
import json
import os
import struct

import pytest
import xxhash

from oracle import deequ_oracle as O
from oracle import c_oracle as C
from tests.fixtures import oracle_table
from tests.oracle_runner import matches, oracle_metric

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                     "reference_known_answers.json")))


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=lambda c: c["cite"])
def test_oracle_reproduces_reference_known_answer(case):
    cls, args, kwargs = case["analyzer"]
    got = oracle_metric(oracle_table(case["fixture"]), cls, args, kwargs)
    assert matches(got, case["expected"], rel=0.0), (got, case["expected"])


@pytest.mark.parametrize("case", GOLDEN["histograms"], ids=lambda c: c["cite"])
def test_oracle_histogram(case):
    groups, n = O.histogram(oracle_table(case["fixture"]), case["column"])
    assert len(groups) == case["bins"]
    top = sorted(groups.items(), key=lambda kv: (-kv[1], kv[0]))[: case["max_detail_bins"]]
    assert {k for k, _ in top} == set(case["keys"])


def test_oracle_stddev_two_partitions_matches_single():
    # Spark merges partition buffers (StandardDeviation.scala:37-44); any partitioning must agree
    t = oracle_table("dfWithNumericValues")
    one = O.agg_stddev(t, "att1", None, partitions=1)
    two = O.agg_stddev(t, "att1", None, partitions=2)
    assert abs((two[2] / two[0]) ** 0.5 - 1.707825127659933) < 1e-15
    assert one[0] == two[0]


@pytest.mark.parametrize("v", [0, 1, -1, 42, 2 ** 62, -(2 ** 63), 123456789012345])
def test_xxhash_long_matches_package(v):
    assert O.spark_xxhash64(v, "long") == xxhash.xxh64_intdigest(struct.pack("<q", v), seed=42)
    assert C.xxh64(struct.pack("<q", v)) == xxhash.xxh64_intdigest(struct.pack("<q", v), seed=42)


@pytest.mark.parametrize("s", ["", "a", "high", "medium", "Thingy abcd", "x" * 31, "y" * 32,
                               "z" * 77, "héllo wörld"])
def test_xxhash_string_matches_package(s):
    b = s.encode()
    assert O.spark_xxhash64(s, "string") == xxhash.xxh64_intdigest(b, seed=42)
    assert C.xxh64(b) == xxhash.xxh64_intdigest(b, seed=42)


def test_hll_small_cardinalities_are_exact_linear_counting():
    # linear counting branch (H <= THRESHOLDS(P-4) = 400) gives the exact count for tiny sets,
    # which is what the reference's tests pin (AnalyzerTests.scala:476-498, AnalysisTest.scala:76)
    for n in (0, 1, 5, 6):
        est, biased = O.hll_count(O.hll_words(O.hll_registers(list(range(n)), "long")))
        assert est == n and not biased
