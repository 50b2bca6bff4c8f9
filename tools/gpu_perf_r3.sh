#!/bin/bash
# Round-3 measurement session: configs[4] parity tests, configs[2] with and without the small-key
# phase A (DQ_FREQ_SMALL), its kernel stats, then configs[4] throughput and kernel stats.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs4.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests_c4par_$T.log 2>&1 &&
DQ_FREQ_SMALL=0 timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_nosmall_$T.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$T -o run -- python3 tools/bench_workloads.py c3 --steps 2 > $O/prof_c3_$T.log 2>&1 &&
timeout -k 10 500 python -u tools/bench_workloads.py c5 --steps 2 > $O/wl_c5_$T.json 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 1 --warmup 1 > $O/prof_c5_$T.log 2>&1
