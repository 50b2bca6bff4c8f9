#!/bin/bash
# One GPU session: the -m gpu suite, smoke(), and a 1-GPU bench line.  TAG names the outputs.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke_$T.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $O/bench_$T.json 2> $O/bench_$T.err
