"""Java Double.toString / Float.toString (Spark 2.2's cast of a floating-point column to string,
what PatternMatch.scala:44-48 matches and Histogram.scala:59-66 groups): the engine's formatter
(csrc/jfmt.h, run on the host through dq_java_*_to_string) against the oracle's independent
restatement (Python repr / numpy Dragon4 digits + Java's layout).  CPU only: the same header is
compiled into the device kernels, whose output the GPU tests check through PatternMatch."""
import math
import random
import struct

import numpy as np
import pytest

from deequ_amd import _native as N
from oracle.deequ_oracle import java_double_to_string, java_float_to_string

# Java's own outputs for values whose text the javadoc / JDK fix the layout of (JDK 8 and 19 agree).
KNOWN_DOUBLES = [(0.0, "0.0"), (-0.0, "-0.0")] + list({
    1.0: "1.0", -1.5: "-1.5", 100.0: "100.0", 0.001: "0.001",
    1e7: "1.0E7", 9999999.0: "9999999.0", 1e-4: "1.0E-4", 123456.789: "123456.789",
    1.7976931348623157e308: "1.7976931348623157E308", 5e-324: "4.9E-324",
    2.2250738585072014e-308: "2.2250738585072014E-308", 0.1: "0.1", 1.1: "1.1",
    float("nan"): "NaN", float("inf"): "Infinity", float("-inf"): "-Infinity",
    3.2: "3.2", 4.4: "4.4", 1e21: "1.0E21", 12345678.9: "1.23456789E7",
}.items())


@pytest.mark.parametrize("value,text", KNOWN_DOUBLES)
def test_known_double_strings(value, text):
    assert N.java_double_to_string(value) == text
    assert java_double_to_string(value) == text


def test_known_float_strings():
    for v, t in [(1.1, "1.1"), (0.1, "0.1"), (1e7, "1.0E7"), (16777216.0, "1.6777216E7"),
                 (3.4028235e38, "3.4028235E38"), (1e-45, "1.4E-45"), (0.001, "0.001"),
                 (-2.5, "-2.5"), (float("nan"), "NaN")]:
        f = float(np.float32(v))
        assert N.java_float_to_string(f) == t, v
        assert java_float_to_string(f) == t, v


def _doubles(rng, n):
    out = [struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0] for _ in range(n)]
    out += [rng.uniform(-1e8, 1e8) for _ in range(n // 4)]
    out += [round(rng.uniform(-1e4, 1e4), rng.randint(0, 6)) for _ in range(n // 4)]
    out += [math.ldexp(1.0, e) for e in range(-1074, 1024)]          # every binade edge
    out += [math.ldexp(k, -1074) for k in range(1, 2048)]            # small subnormals
    out += [float(10.0 ** k) for k in range(-30, 30)] + [float(f"{d}e{k}") for d in range(1, 10)
                                                          for k in (-4, -3, 6, 7, 22, 23)]
    return out


def test_random_doubles_match_the_oracle():
    rng = random.Random(7)
    for v in _doubles(rng, 60000):
        assert N.java_double_to_string(v) == java_double_to_string(v), repr(v)


def test_random_floats_match_the_oracle():
    rng = random.Random(11)
    bits = [rng.getrandbits(32) for _ in range(60000)] + list(range(1, 2048))
    bits += [e << 23 for e in range(1, 255)]
    for b in bits:
        f = float(np.frombuffer(struct.pack("<I", b), dtype=np.float32)[0])
        assert N.java_float_to_string(f) == java_float_to_string(f), (hex(b), f)


def test_formatted_strings_read_back():
    rng = random.Random(3)
    for v in _doubles(rng, 20000):
        if math.isfinite(v):
            assert float(N.java_double_to_string(v)) == v


def test_batch_formatter_matches_one_value_calls():
    """dq_java_doubles_to_strings (Histogram's keys of a floating-point column in one call) gives
    each value's dq_java_double_to_string / dq_java_float_to_string text."""
    rng = random.Random(5)
    vals = [0.0, -0.0, 1.0, 1e7, 1e-3, 123456789.125, float("inf"), float("-inf"), float("nan"),
            5e-324, 1.7976931348623157e308] + [rng.uniform(-1e9, 1e9) for _ in range(300)]
    assert N.java_doubles_to_strings(vals) == [N.java_double_to_string(v) for v in vals]
    with np.errstate(over="ignore"):
        fl = np.array(vals, np.float64).astype(np.float32).astype(np.float64).tolist()
    assert N.java_doubles_to_strings(fl, True) == [N.java_float_to_string(v) for v in fl]
    assert N.java_doubles_to_strings([]) == []
