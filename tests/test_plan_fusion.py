"""Host-side planning of the configs[3] fusion (api.cpp dq_plan_create): ApproxCountDistinct(x)
beside Correlation(x, y) or (y, x) under the same where runs as one pass (BC_CORR_HLL) that
hashes x; other combinations keep their own passes.  Plans are built on the host (no GPU)."""
import pytest

from deequ_amd import _native as N
from deequ_amd.analyzers import ApproxCountDistinct, Correlation
from deequ_amd.runners.engine import Plan
from deequ_amd.table import StructField, StructType


def _schema():
    return StructType([StructField("x", N.INT64), StructField("y", N.FLOAT64),
                       StructField("i", N.INT32), StructField("s", N.UTF8)])


def _explain(*analyzers):
    return Plan(_schema(), [s for a in analyzers for s in a.aggregation_functions()]).explain()


@pytest.mark.parametrize("hll,corr,side", [
    (ApproxCountDistinct("x"), Correlation("x", "y"), ""),
    (ApproxCountDistinct("y"), Correlation("x", "y"), "2"),
    (ApproxCountDistinct("x", "i > 0"), Correlation("y", "x", "i > 0"), "2"),
])
def test_hll_rides_in_the_comoment_pass(hll, corr, side):
    e = _explain(hll, corr)
    assert f"+hll[0] of col{side}\n" in e, e
    assert "rows hashed by a fused co-moment pass" in e, e


@pytest.mark.parametrize("hll,corr", [
    (ApproxCountDistinct("x", "i > 0"), Correlation("x", "y")),   # different where
    (ApproxCountDistinct("s"), Correlation("x", "y")),            # column not in the pair
    (ApproxCountDistinct("i"), Correlation("i", "y")),            # 4-byte column: no vector path
])
def test_no_fusion_otherwise(hll, corr):
    assert "+hll[" not in _explain(hll, corr)


def test_no_fuse_env_keeps_two_passes(monkeypatch):
    monkeypatch.setenv("DQ_NO_FUSE", "1")
    assert "+hll[" not in _explain(ApproxCountDistinct("x"), Correlation("x", "y"))
