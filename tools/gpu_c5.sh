#!/bin/bash
# configs[4] (c5): small validation run, the 2.5e8-row measurement, and its kernel stats. TAG names outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r2}
mkdir -p $O
timeout -k 10 200 python -u tools/bench_workloads.py c5 --rows 10000000 --steps 1 > $O/wl_c5_small_$T.json 2>&1 &&
timeout -k 10 500 python -u tools/bench_workloads.py c5 --steps 2 > $O/wl_c5_$T.json 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 1 --warmup 0 > $O/prof_c5_$T.log 2>&1
