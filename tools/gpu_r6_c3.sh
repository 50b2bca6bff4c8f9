#!/bin/bash
# Round 6: the configs[2] tests (incl. the duplicate-bearing key at 1e9 rows), then configs[2]
# timed and its rocprofv3 kernel stats.  TAG names the outputs; TESTS overrides the test list.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r6}
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_fullsize_dups.py tests/test_gpu_freq.py} -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 10 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$T -o run -- python3 tools/bench_workloads.py c3 --steps 3 > $O/prof_c3_$T.log 2>&1
