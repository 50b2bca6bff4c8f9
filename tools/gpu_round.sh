#!/bin/bash
# End-of-round session: the whole -m gpu suite, smoke(), the bench line (S10, configs[1]) with its
# rocprofv3 kernel stats, then configs[3] and configs[4] lines.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke_$T.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s10_$T -o run -- python3 bench.py --steps 10 --warmup 2 --no-h2d --no-cpu-baseline > $O/prof_s10_$T.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_workloads.py c4 --steps 5 > $O/wl_c4_$T.json 2>&1 &&
timeout -k 10 600 python -u tools/bench_workloads.py c5 --steps 2 > $O/wl_c5_$T.json 2>&1
