"""CPU build of the group-by key codec (deequ_amd/csrc/freq_codec.h, the DQ_HD functions the HIP
group-by kernels run) under AddressSanitizer + UBSan: the 1-row (INT64_MIN, string) key the
round-1 mixed-key grouping faulted on, and seeded 5000-row tables with NULLs, in grouping and
Histogram ("NullValue") mode (tools/freq_codec_check.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_codec_under_asan(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "freq_codec_check")
    subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    os.path.join(ROOT, "tools", "freq_codec_check.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK"), out.stdout
