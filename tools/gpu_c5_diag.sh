#!/bin/bash
# c5 diagnosis: kernel summary and a cProfile of one step, DQ_RUN_WORKERS=${W:-1}
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r3y}
mkdir -p $O
export DQ_RUN_WORKERS=${W:-1}
timeout -k 10 300 python -u tools/bench_workloads.py c5 --steps 1 --pyprof > $O/c5_pyprof_$T.txt 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 1 --warmup 1 > $O/prof_c5_$T.log 2>&1
