#!/bin/bash
# Round-1 GPU session: parity tests, ablation (mixed vs per-class launches), bench, rocprofv3.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-r1}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python -u tools/scan_ablation.py 1000000000 5 > $O/abl_mixed_$T.log 2>&1 &&
DQ_NO_MIXED=1 timeout -k 10 200 python -u tools/scan_ablation.py 1000000000 5 > $O/abl_nomixed_$T.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$T -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$T -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write_$T.log 2>&1
