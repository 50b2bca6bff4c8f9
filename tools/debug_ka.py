"""Debug helper: run every known-answer case through the GPU engine and print failures."""
import json, os, sys, traceback
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_known_answers import GOLDEN, table, build, value_of
from tests.oracle_runner import matches
bad = 0
for case in GOLDEN["cases"]:
    cls, args, kwargs = case["analyzer"]
    try:
        m = build(cls, args, kwargs).calculate(table(case["fixture"]))
        got = value_of(m)
        exp = case["expected"]
        ok = (got in ("FAILURE", "EMPTY")) if exp == "FAILURE" else matches(got, exp, rel=1e-12)
        if not ok:
            bad += 1
            print("MISMATCH", case["cite"], cls, args, got, exp)
            if m.value.is_failure:
                e = m.value.failed
                traceback.print_exception(type(e), e, e.__traceback__)
    except Exception:
        bad += 1
        print("EXC", case["cite"]); traceback.print_exc()
print("bad", bad, "of", len(GOLDEN["cases"]))
