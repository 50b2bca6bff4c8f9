"""Imports tests/golden/make_golden.py (a script, not a package module) for the tests."""
import importlib.util
import os

_p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "make_golden.py")
_spec = importlib.util.spec_from_file_location("make_golden", _p)
_m = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_m)
oracle_table = _m.oracle_table
scan_expected = _m.scan_expected
freq_expected = _m.freq_expected
histogram_expected = _m.histogram_expected
hll_high_register_sets = _m.hll_high_register_sets
high_rank_column_expected = _m.high_rank_column_expected
