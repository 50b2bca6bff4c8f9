"""The RCCL (torch.distributed "nccl") branches of deequ_amd/distributed.py on the GPU, with one
rank: the device-side scan-state exchange against the serialized host merge (byte for byte, one
host wait), and the distributed frequency paths (raw-key all-to-all, partial-aggregate
repartition, DistributedFrequencies' reductions) against the local group-by.  The rank runs as a
child process of the test (no exec from a GPU-initialised process).  SURVEY.md §8(e)."""
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


def test_rccl_branches_with_one_rank(gpu_device, tmp_path):
    out = tmp_path / "nccl.json"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.Popen([sys.executable, os.path.join(HERE, "workers", "nccl_world1.py"),
                          str(_port()), str(out)], env=env)
    assert p.wait(timeout=240) == 0
    got = json.loads(out.read_text())
    assert got["backend"] == "nccl"
    assert got["exchange"] == [True, True, 1]
    for col, (dist_s, local_s, dist_top, local_top) in got["frequencies"].items():
        assert dist_s[:2] == local_s[:2], col
        assert dist_s[2] == local_s[2] or abs(dist_s[2] - local_s[2]) <= 1e-12 * abs(local_s[2]), col
        assert dist_top == local_top, col
