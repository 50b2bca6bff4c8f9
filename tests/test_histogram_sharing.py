"""Host logic of the runner's one-group-by-for-two plan (runners/__init__.py
_histogram_columns_for_groupings): which columns' Histogram tables may serve their grouping."""
from types import SimpleNamespace

from deequ_amd import _native as N
from deequ_amd.analyzers import Entropy, Histogram, Uniqueness
from deequ_amd.runners import _histogram_columns_for_groupings


def _data(dtype, bitmaps):
    schema = {"c": SimpleNamespace(dtype=dtype)}
    batches = [{"c": SimpleNamespace(validity=object() if b else None)} for b in bitmaps]
    return SimpleNamespace(schema=schema, batches=batches)


def test_integral_and_boolean_columns_always_share():
    for t in (N.BOOL, N.INT8, N.INT16, N.INT32, N.INT64):
        assert Histogram.table_serves_grouping(_data(t, [True, False]), "c")


def test_strings_share_with_or_without_nulls():
    # the NULL rows are a group kept apart in the table; Histogram folds it into "NullValue"
    assert Histogram.table_serves_grouping(_data(N.UTF8, [False, False]), "c")
    assert Histogram.table_serves_grouping(_data(N.UTF8, [False, True]), "c")


def test_floating_point_shares_provisionally():
    # Histogram folds NaN payloads (cast to string), the grouping keeps them apart: the table
    # serves the grouping only when it folded no row, which the runner checks after building it
    # (FrequencyTable.folded_nan_rows; tests/test_gpu_float_sharing.py)
    for t in (N.FLOAT32, N.FLOAT64):
        assert Histogram.table_serves_grouping(_data(t, [False]), "c")


def test_no_sharing_when_states_are_aggregated_or_saved():
    data = _data(N.INT64, [False])
    grouping, scanning = [Uniqueness(["c"]), Entropy("c")], [Histogram("c")]
    assert _histogram_columns_for_groupings(data, grouping, scanning, object(), None) == []
    assert _histogram_columns_for_groupings(data, grouping, scanning, None, object()) == []


def test_no_sharing_without_a_grouping_of_that_column():
    data = _data(N.INT64, [False])
    assert _histogram_columns_for_groupings(data, [Uniqueness(["c", "d"])], [Histogram("c")],
                                            None, None) == []
    assert _histogram_columns_for_groupings(data, [Uniqueness(["c"])], [Histogram("c")],
                                            None, None) == ["c"]
