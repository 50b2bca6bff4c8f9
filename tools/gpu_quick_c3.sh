#!/bin/bash
# Quick configs[2] check: the frequency GPU tests, one timed run, one DQ_FREQ_DEBUG=2 run.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_freq.py tests/test_gpu_configs4.py -x -q --timeout 120 --timeout-method thread > $O/freq_tests_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1 &&
DQ_FREQ_DEBUG=2 timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 1 --warmup 0 > $O/dbg_c3_$T.log 2>&1
