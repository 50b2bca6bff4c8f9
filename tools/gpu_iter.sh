#!/bin/bash
# Iteration session: the frequency-family GPU tests, then configs[2] A/B (DQ_FREQ_OLDC=1 = the
# generic exact phase C) and a rocprofv3 kernel-stats run.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-it}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_freq.py tests/test_gpu_configs4.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/freq_tests_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1 &&
DQ_FREQ_OLDC=1 timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_old_$T.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$T -o run -- python3 tools/bench_workloads.py c3 --steps 2 > $O/prof_c3_$T.log 2>&1
