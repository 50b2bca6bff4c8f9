#!/bin/bash
# Round-3 combined session (one box): the whole -m gpu suite, smoke(), the S10 bench with its
# rocprofv3 kernel stats and PMC traffic passes, the S10 sub-suite ablation (also against the
# diagnostic compact-load build DQ_LIB_PATH=deequ_amd/libdq_exp.so when present), then configs[3],
# configs[2] (+ kernel stats) and configs[4] (+ kernel stats) lines.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke_$T.log 2>&1 &&
TAG=$T bash tools/gpu_s10_prof.sh &&
timeout -k 10 300 python -u tools/scan_ablation.py 1000000000 5 > $O/ablation_$T.log 2>&1 &&
{ [ ! -f deequ_amd/libdq_exp.so ] || DQ_LIB_PATH=deequ_amd/libdq_exp.so timeout -k 10 300 python -u tools/scan_ablation.py 1000000000 5 > $O/ablation_exp_$T.log 2>&1; } &&
timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 5 > $O/wl_c4_$T.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c3 --steps 3 > $O/wl_c3_$T.json 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$T -o run -- python3 tools/bench_workloads.py c3 --steps 2 > $O/prof_c3_$T.log 2>&1 &&
timeout -k 10 500 python -u tools/bench_workloads.py c5 --steps 3 > $O/wl_c5_$T.json 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$T -o run -- python3 tools/bench_workloads.py c5 --steps 1 --warmup 1 > $O/prof_c5_$T.log 2>&1
