"""Two ranks on one GPU (gloo, 127.0.0.1): AnalysisRunner over row shards must reproduce the
one-rank run of the whole table -- counts, HLL estimates, groupings bit-exact, fp64 within 1e-12
relative.  The ranks run as child processes of the test (no
exec from a GPU-initialised process)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_reproduce_one_rank(gpu_device, tmp_path):
    sys.path.insert(0, HERE)
    from dist_suite import close, metrics_of, suite, table
    from deequ_amd.runners import AnalysisRunner
    from deequ_amd.table import Table
    whole = metrics_of(AnalysisRunner.do_analysis_run(
        Table.from_arrow(table(), device=gpu_device, max_batch_rows=6000), suite()))
    out = tmp_path / "ranks.json"
    port = _port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "workers", "dist_ranks.py"),
                               str(r), "2", str(port), str(out)], env=env)
             for r in range(2)]
    codes = [p.wait(timeout=240) for p in procs]
    assert codes == [0, 0], codes
    got = json.loads(out.read_text())
    # the device-side exchange equals the serialized all-gather + rank-ordered merge, byte for
    # byte, and waits on the host once (the merged state's read-back) -- pack / unpack queue
    # without a wait
    assert got.pop("__exchange__") == [True, True, 1]
    assert set(got) == set(whole)
    for k, v in whole.items():
        g = got[k]
        if isinstance(v, list) and v and v[0] == "failure":
            assert g[0] == "failure", k
        elif isinstance(v, list):  # Histogram: bins and the top counts exactly
            assert g[0] == v[0] and g[1] == v[1], k
            for key, c in g[2].items():
                if key in v[2]:
                    assert v[2][key] == c, (k, key)
        else:
            assert close(g, v), (k, g, v)


def test_two_ranks_match_the_oracle(gpu_device, tmp_path):
    """The same two-rank run against the oracle (not only against the engine's one-rank run):
    every grouping metric -- including the unique int64 / int32 ids that take the raw-key exchange
    (dq_key_partition) and the low-cardinality keys that take the partial-aggregate exchange --
    Histogram bins and counts, and the scan metrics.  Bar: counts and bins exact, fp64 1e-12."""
    sys.path.insert(0, HERE)
    from dist_suite import close, oracle_metrics, table
    exp = oracle_metrics(table())
    out = tmp_path / "ranks.json"
    port = _port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "workers", "dist_ranks.py"),
                               str(r), "2", str(port), str(out)], env=env)
             for r in range(2)]
    codes = [p.wait(timeout=240) for p in procs]
    assert codes == [0, 0], codes
    got = json.loads(out.read_text())
    for k, v in exp.items():
        g = got[k]
        if isinstance(v, list):  # Histogram: bins, and the top counts (ties in any order)
            assert g[0] == v[0], k
            assert g[1] == v[1][:len(g[1])], k
        else:
            assert close(g, v), (k, g, v)
