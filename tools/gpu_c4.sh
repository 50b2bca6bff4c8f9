#!/bin/bash
# configs[3] measurement + its rocprofv3 kernel stats (and the unfused A/B); TAG names the outputs
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r2}
mkdir -p $O
timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 5 > $O/wl_c4_$T.json 2>&1 &&
DQ_NO_FUSE=1 timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 5 > $O/wl_c4_nofuse_$T.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_$T -o run -- python3 tools/bench_workloads.py c4 --steps 3 > $O/prof_c4_$T.log 2>&1
