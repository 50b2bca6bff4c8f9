"""Debug helper: one tiny Completeness scan with DQ_DEBUG launch tracing."""
import os, sys, time
os.environ["DQ_DEBUG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.fixtures import arrow_table
from deequ_amd import Table
from deequ_amd.analyzers import Completeness, Mean, Compliance
t = Table.from_arrow(arrow_table("dfMissing"), device="cuda:0")
for a in [Completeness("att1"), Compliance("x", "att1 IN ('a')")]:
    t0 = time.time()
    m = a.calculate(t)
    print(a, m.value, time.time() - t0, flush=True)
t = Table.from_arrow(arrow_table("dfWithNumericValues"), device="cuda:0")
print(Mean("att1").calculate(t).value, flush=True)
