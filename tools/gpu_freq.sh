#!/bin/bash
# Frequency-path session: the -m gpu frequency tests, then the configs[2] measurement + rocprofv3
# kernel stats.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_freq_tests_$T.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$T -o run -- python3 tools/bench_workloads.py c3 --steps 2 > $O/prof_c3_$T.log 2>&1 &&
# workgroup-0 phase-A tile timings (DQ_FREQ_DEBUG=2), 1e8 rows
DQ_FREQ_DEBUG=2 timeout -k 10 200 python -u tools/bench_workloads.py c3 --rows 100000000 --steps 1 --warmup 0 > $O/dbg_c3_$T.json 2> $O/dbg_c3_$T.err
